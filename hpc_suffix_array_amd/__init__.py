"""hpc_suffix_array_amd -- MI355X-native (gfx950 HIP) Manber-Myers suffix-array
construction behind the C ABI of a-rtemis99/hpc_suffix_array
(src/common/suffix_array.h) plus a 64-bit extended ABI (include/sa_hip.h).
"""
from ._native import SAError, build_library, device_count, lib  # noqa: F401
from .builder import DeviceBuilder, SuffixArray, build_suffix_array, check_suffix_array, lcp_array  # noqa: F401

__all__ = ["SAError", "DeviceBuilder", "SuffixArray", "build_suffix_array", "check_suffix_array",
           "lcp_array", "build_library", "device_count", "lib"]
