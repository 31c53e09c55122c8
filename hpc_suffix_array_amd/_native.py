"""ctypes binding of libsa_hip.so (include/sa_hip.h, include/suffix_array.h).

The library is built in-tree by ``hpc_suffix_array_amd/csrc/Makefile`` into
``hpc_suffix_array_amd/lib/libsa_hip.so``.  Loading it never touches the GPU;
every compute entry point fails loudly (SAError) when no HIP device is
present -- there is no CPU fallback anywhere in this package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "lib", "libsa_hip.so")
# A/B runs of build variants point SA_LIB_PATH at another in-tree build
LIB_PATH = os.environ.get("SA_LIB_PATH", LIB_PATH)
CSRC = os.path.join(PKG_DIR, "csrc")

SA_MAX_ROUNDS = 64
KERNEL_KINDS = ["init", "hist_first", "hist_keys", "scan", "scatter_first", "scatter_keys",
                "heads", "heads_scan", "rerank", "seg_count", "seg_scan", "seg_write", "alphabet", "pack",
                "sort_u", "windows", "local_sort", "pivot_keys", "pivot_count", "pivot_write"]
SCHEDULE_PACKED = 0
SCHEDULE_REFERENCE = 1
ROUND1_AUTO = 0
ROUND1_LSD = 1
ROUND1_BUCKETED = 2
SA_K_COUNT = len(KERNEL_KINDS)

# every symbol include/*.h declares
DROPIN_SYMBOLS = ["create_suffix_array", "destroy_suffix_array", "build_suffix_array",
                  "build_lcp_array", "find_longest_repeated_substring", "is_valid_suffix_array"]
EXT_SYMBOLS = ["sa_context_create", "sa_context_destroy", "sa_context_set_debug", "sa_workspace_bytes", "sa_build_device",
               "sa_build_ex", "sa_check_device", "sa_check", "sa_lcp_device", "sa_lcp", "sa_generate_text_device",
               "sa_alphabet_device", "sa_pack_keys_device", "sa_sort_pairs_device", "sa_scatter_u64_device",
               "sa_gather_u64_device", "sa_running_max_i64_device", "sa_inclusive_sum_i64_device",
               "sa_count_below_u64_device", "sa_select_u8_device",
               "sa_dist_begin", "sa_dist_cuts", "sa_dist_plan_cuts", "sa_dist_reserve", "sa_dist_release", "sa_dist_round1", "sa_dist_req_count", "sa_dist_req_fill",
               "sa_dist_answer", "sa_dist_refine",
               "sa_last_error", "sa_host_syncs", "sa_device_count", "sa_version", "sa_struct_size"]


class SAError(RuntimeError):
    """A libsa_hip entry point returned an error code."""


# sa_opts.debug flags (include/sa_hip.h SA_DEBUG_*): alternative paths the
# tests force; every combination gives the same suffix array
DEBUG_FLAGS = {"no_cmp": 0x1, "no_pk8": 0x2, "no_pad": 0x4, "pad_overflow": 0x8, "no_fast32": 0x10,
               "no_pivot": 0x20, "perm_always": 0x40, "no_xq": 0x80, "xq_overflow": 0x100,
               "no_tied": 0x200, "no_key1_round": 0x400, "no_eonly": 0x800,
               "eonly": 0x1000}


def debug_bits(names) -> int:
    bits = 0
    for x in names or ():
        if x not in DEBUG_FLAGS:
            raise ValueError(f"unknown debug flag {x!r} (one of {sorted(DEBUG_FLAGS)})")
        bits |= DEBUG_FLAGS[x]
    return bits


class SaOpts(ctypes.Structure):
    _fields_ = [("profile", ctypes.c_int32), ("schedule", ctypes.c_int32), ("init_chars", ctypes.c_int32),
                ("radix", ctypes.c_int32), ("round1", ctypes.c_int32), ("debug", ctypes.c_uint32),
                ("span_extra", ctypes.c_int32), ("tune", ctypes.c_int32)]


class SaStats(ctypes.Structure):
    _fields_ = [
        ("rounds", ctypes.c_int32),
        ("n_kinds", ctypes.c_int32),
        ("total_ms", ctypes.c_double),
        ("h2d_ms", ctypes.c_double),
        ("d2h_ms", ctypes.c_double),
        ("round_ms", ctypes.c_double * SA_MAX_ROUNDS),
        ("distinct", ctypes.c_uint64 * SA_MAX_ROUNDS),
        ("passes", ctypes.c_int32 * SA_MAX_ROUNDS),
        ("sorted_n", ctypes.c_uint64 * SA_MAX_ROUNDS),
        ("prefix_len", ctypes.c_uint64 * SA_MAX_ROUNDS),
        ("schedule", ctypes.c_int32),
        ("init_chars", ctypes.c_int32),
        ("sigma", ctypes.c_int32),
        ("sparse_ranks", ctypes.c_int32),
        ("round1", ctypes.c_int32),
        ("largest_window", ctypes.c_int32),
        ("model_bytes", ctypes.c_uint64),
        ("kern_ms", ctypes.c_double * SA_K_COUNT),
        ("kern_launches", ctypes.c_uint64 * SA_K_COUNT),
        ("kern_bytes", ctypes.c_uint64 * SA_K_COUNT),
        ("round1_segments", ctypes.c_int32),
        ("round1_layout", ctypes.c_int32),
        ("round_bytes", ctypes.c_uint64 * SA_MAX_ROUNDS),
    ]

    def to_dict(self) -> dict:
        r = self.rounds
        return {
            "rounds": r,
            "total_ms": self.total_ms,
            "h2d_ms": self.h2d_ms,
            "d2h_ms": self.d2h_ms,
            "round_ms": list(self.round_ms[:r]),
            "distinct": [int(x) for x in self.distinct[:r]],
            "passes": list(self.passes[:r]),
            "sorted_n": [int(x) for x in self.sorted_n[:r]],
            "prefix_len": [int(x) for x in self.prefix_len[:r]],
            "schedule": "reference" if self.schedule == SCHEDULE_REFERENCE else "packed",
            "init_chars": self.init_chars,
            "sigma": self.sigma,
            "sparse_ranks": bool(self.sparse_ranks),
            "round1": {ROUND1_LSD: "lsd", ROUND1_BUCKETED: "bucketed", 3: "pivot"}.get(self.round1, "lsd"),
            "largest_window": self.largest_window,
            "round1_segments": {0: "exact", 1: "padded", 2: "padded-overflow", 3: "striped-records",
                                4: "striped-records-overflow"}.get(self.round1_segments, "exact"),
            "round1_layout": {"compact": bool(self.round1_layout & 1), "pk8": bool(self.round1_layout & 2),
                              "xq": bool(self.round1_layout & 4), "eonly": bool(self.round1_layout & 8)},
            "reference_model_bytes": int(self.model_bytes),
            "round_bytes": [int(x) for x in self.round_bytes[:r]],
            "kernels": {k: {"ms": self.kern_ms[i], "launches": int(self.kern_launches[i]),
                            "bytes": int(self.kern_bytes[i])} for i, k in enumerate(KERNEL_KINDS)},
        }


DIST_OK = 0
DIST_UNSUPPORTED = 1
DIST_UNBALANCED = 2


class SaDistInfo(ctypes.Structure):
    """sa_dist_info of include/sa_hip.h (range-partitioned build, per rank)."""
    _fields_ = [("status", ctypes.c_int32), ("sigma", ctypes.c_int32), ("K", ctypes.c_int32),
                ("bucket_bits", ctypes.c_int32), ("m", ctypes.c_uint64), ("sa_off", ctypes.c_uint64),
                ("m_max", ctypes.c_uint64), ("bucket_lo", ctypes.c_uint32), ("bucket_hi", ctypes.c_uint32),
                ("round1_ok", ctypes.c_int32), ("reserved", ctypes.c_int32), ("heads", ctypes.c_uint64),
                ("unsorted", ctypes.c_uint64), ("groups", ctypes.c_uint64)]


class SuffixArrayStruct(ctypes.Structure):
    """SuffixArray of suffix_array.h:16-21 (32 bytes: str@0 n@8 sa@16 lcp@24)."""
    _fields_ = [("str", ctypes.c_void_p), ("n", ctypes.c_int),
                ("sa", ctypes.POINTER(ctypes.c_int)), ("lcp", ctypes.POINTER(ctypes.c_int))]


_lib = None


def source_hash() -> str:
    """SHA-256 (first 16 hex digits) of the sources libsa_hip.so is built
    from: bench.py stamps it on its line and profiles/summarize.py on each
    rocprof summary, so a summary is matched to the code it measured."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(CSRC, "sa_*")) + [os.path.join(CSRC, "Makefile")]
                   + glob.glob(os.path.join(PKG_DIR, "..", "include", "*.h")))
    for p in files:
        with open(p, "rb") as f:
            h.update(os.path.basename(p).encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def build_library(force: bool = False) -> str:
    """Compile libsa_hip.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", CSRC], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SAError(f"{LIB_PATH} is missing: run `make -C {CSRC}` (or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
    L.sa_context_create.argtypes = [i32, u64, ctypes.POINTER(vp)]
    L.sa_context_create.restype = i32
    L.sa_context_destroy.argtypes = [vp]
    L.sa_context_destroy.restype = None
    L.sa_context_set_debug.argtypes = [vp, ctypes.POINTER(SaOpts)]
    L.sa_context_set_debug.restype = i32
    L.sa_workspace_bytes.argtypes = [u64]
    L.sa_workspace_bytes.restype = u64
    L.sa_build_device.argtypes = [vp, vp, u64, vp, vp, ctypes.POINTER(SaOpts), ctypes.POINTER(SaStats)]
    L.sa_build_device.restype = i32
    L.sa_build_ex.argtypes = [vp, u64, vp, i32, ctypes.POINTER(SaOpts), ctypes.POINTER(SaStats)]
    L.sa_build_ex.restype = i32
    L.sa_check_device.argtypes = [vp, vp, u64, vp, vp]
    L.sa_check_device.restype = i32
    L.sa_check.argtypes = [vp, u64, vp, i32]
    L.sa_check.restype = i32
    L.sa_lcp_device.argtypes = [vp, vp, u64, vp, vp, ctypes.POINTER(u64), ctypes.POINTER(u64), vp]
    L.sa_lcp_device.restype = i32
    L.sa_lcp.argtypes = [vp, u64, vp, i32, vp, ctypes.POINTER(u64), ctypes.POINTER(u64)]
    L.sa_lcp.restype = i32
    L.sa_alphabet_device.argtypes = [vp, u64, ctypes.POINTER(ctypes.c_uint32), vp]
    L.sa_alphabet_device.restype = i32
    L.sa_pack_keys_device.argtypes = [vp, vp, u64, u64, u64, ctypes.POINTER(ctypes.c_uint16), u64,
                                      ctypes.c_uint32, vp, vp]
    L.sa_pack_keys_device.restype = i32
    L.sa_sort_pairs_device.argtypes = [vp, vp, vp, u64, ctypes.c_uint32, vp, vp, vp]
    L.sa_sort_pairs_device.restype = i32
    L.sa_scatter_u64_device.argtypes = [vp, u64, vp, ctypes.c_int64, vp, u64, vp]
    L.sa_scatter_u64_device.restype = i32
    L.sa_gather_u64_device.argtypes = [vp, vp, u64, vp, ctypes.c_int64, u64, vp]
    L.sa_gather_u64_device.restype = i32
    L.sa_running_max_i64_device.argtypes = [vp, u64, vp]
    L.sa_running_max_i64_device.restype = i32
    L.sa_inclusive_sum_i64_device.argtypes = [vp, u64, vp]
    L.sa_inclusive_sum_i64_device.restype = i32
    L.sa_count_below_u64_device.argtypes = [vp, u64, vp, u64, i32, vp, vp]
    L.sa_count_below_u64_device.restype = i32
    L.sa_select_u8_device.argtypes = [vp, u64, vp, ctypes.POINTER(u64), vp]
    L.sa_select_u8_device.restype = i32
    DI = ctypes.POINTER(SaDistInfo)
    L.sa_dist_begin.argtypes = [vp, vp, u64, i32, i32, ctypes.POINTER(ctypes.c_uint32), vp, vp, DI]
    L.sa_dist_cuts.argtypes = [vp, ctypes.POINTER(u64), DI]
    L.sa_dist_plan_cuts.argtypes = [i32, u64, i32, ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_uint32),
                                    ctypes.POINTER(u64)]
    L.sa_dist_release.argtypes = [vp]
    L.sa_dist_reserve.argtypes = [vp, u64, i32]
    L.sa_dist_round1.argtypes = [vp, vp, vp, DI, ctypes.POINTER(SaStats)]
    L.sa_dist_req_count.argtypes = [vp, u64, ctypes.POINTER(u64), vp, DI]
    L.sa_dist_req_fill.argtypes = [vp, u64, vp, vp]
    L.sa_dist_answer.argtypes = [vp, vp, u64, vp, vp]
    L.sa_dist_refine.argtypes = [vp, u64, vp, vp, vp, DI]
    for f in (L.sa_dist_begin, L.sa_dist_cuts, L.sa_dist_plan_cuts, L.sa_dist_reserve, L.sa_dist_release,
              L.sa_dist_round1, L.sa_dist_req_count, L.sa_dist_req_fill,
              L.sa_dist_answer, L.sa_dist_refine):
        f.restype = i32
    L.sa_generate_text_device.argtypes = [vp, u64, u64, ctypes.c_char_p, ctypes.c_uint32, vp]
    L.sa_generate_text_device.restype = i32
    L.sa_last_error.argtypes = []
    L.sa_last_error.restype = ctypes.c_char_p
    L.sa_host_syncs.argtypes = []
    L.sa_host_syncs.restype = ctypes.c_uint64
    L.sa_device_count.argtypes = []
    L.sa_device_count.restype = i32
    L.sa_version.argtypes = []
    L.sa_version.restype = ctypes.c_char_p
    P = ctypes.POINTER(SuffixArrayStruct)
    L.create_suffix_array.argtypes = [ctypes.c_char_p, i32]
    L.create_suffix_array.restype = P
    L.destroy_suffix_array.argtypes = [P]
    L.destroy_suffix_array.restype = None
    L.build_suffix_array.argtypes = [P]
    L.build_suffix_array.restype = None
    L.build_lcp_array.argtypes = [P]
    L.build_lcp_array.restype = None
    L.find_longest_repeated_substring.argtypes = [P]
    L.find_longest_repeated_substring.restype = vp
    L.is_valid_suffix_array.argtypes = [P]
    L.is_valid_suffix_array.restype = i32
    _lib = L
    return L


def check(rc: int, what: str) -> int:
    if rc < 0:
        raise SAError(f"{what}: {lib().sa_last_error().decode(errors='replace')} (code {rc})")
    return rc


def device_count() -> int:
    return lib().sa_device_count()


def require_device() -> None:
    """Fail loudly when the HIP path cannot run (no silent fallback)."""
    if device_count() <= 0:
        raise SAError("no HIP device visible: libsa_hip builds suffix arrays on an MI355X only")
