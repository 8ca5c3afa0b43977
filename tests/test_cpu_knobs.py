"""The product library's environment knobs (csrc/knobs.h): measurement knobs exist only in the
-DSKY_MEASURE build (build_measure/, tools only), and every knob the product library reads is
exercised by a test."""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROD = os.path.join(ROOT, "flink-skyline-qos_amd", "build", "libskyline_hip.so")

# measurement-only: each can skip or truncate work (results invalid) or only reshapes a launch
MEASURE_ONLY = {"SKY_FILTER_DBG", "SKY_MBR_DBG", "SKY_CSV_STOP", "SKY_CSV_CHUNK_BYTES", "SKY_DEBUG",
                "SKY_TRACE_ALLOC", "SKY_PLANES", "SKY_HIST_COUNT", "SKY_BRUTE_MAX", "SKY_MBR_ORDER",
                "SKY_STAGE_THREADS", "SKY_PART_HOSTPROF", "SKY_DOM_PPT", "SKY_DOM_TX", "SKY_DOM_R",
                "SKY_RADIX_ITEMS", "SKY_RADIX_COMPRESS", "SKY_SAMPLE_WG", "SKY_FILTER_TPB", "SKY_DEFER_WG",
                "SKY_OUT_TPB", "SKY_PREFILTER_M2", "SKY_MBR_QCAP", "SKY_FILTER_COUNT"}
NOT_KNOBS = {"SKY_DIST_STATS_WORDS"}   # a header macro named in an error message


def _names(path):
    with open(path, "rb") as f:
        return {m.decode() for m in re.findall(rb"SKY_[A-Z0-9_]+", f.read())}


@pytest.mark.skipif(not os.path.exists(PROD), reason="product library not built")
def test_product_library_has_no_measurement_knobs():
    names = _names(PROD)
    assert not (names & MEASURE_ONLY), sorted(names & MEASURE_ONLY)


@pytest.mark.skipif(not os.path.exists(PROD), reason="product library not built")
def test_every_product_knob_is_named_by_a_test():
    text = ""
    for p in glob.glob(os.path.join(ROOT, "tests", "*.py")):
        if os.path.basename(p) != os.path.basename(__file__):
            with open(p) as f:
                text += f.read()
    knobs = _names(PROD) - NOT_KNOBS
    assert knobs, "no knob strings found"
    missing = sorted(k for k in knobs if not re.search(r"\b%s\b" % k, text))
    assert not missing, missing
