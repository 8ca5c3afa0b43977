"""skyline — Python host side of the MI355X-native skyline engine.

    from skyline import SkylineEngine          # one context per GPU (C ABI handle)
    from skyline.operators import ...          # mirror of the reference Flink operators

All skyline computation runs in libskyline_hip.so (gfx950 HIP kernels).
"""
from ._abi import SkylineError, lib, LIB_PATH  # noqa: F401
from .engine import SkylineEngine, SkylineStream, synth_host  # noqa: F401
