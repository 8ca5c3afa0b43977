"""Hash of the sources a kernel is compiled from, so that a committed counter measurement
(profiles/traffic_filter.json) is only reported for the build it was measured on."""
import hashlib
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL_SOURCES = {
    "k_filter": ["flink-skyline-qos_amd/csrc/k_partition.hip", "flink-skyline-qos_amd/csrc/sky_device.h",
                 "flink-skyline-qos_amd/csrc/sky_common.h", "flink-skyline-qos_amd/csrc/sky_internal.h",
                 "flink-skyline-qos_amd/Makefile"],
}


def kernel_src_sha(kernel="k_filter"):
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES[kernel]:
        with open(os.path.join(REPO, rel), "rb") as f:
            h.update(rel.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]
