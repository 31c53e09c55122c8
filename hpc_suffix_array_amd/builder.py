"""Host-side mirror of the reference's suffix-array interface over libsa_hip.

Reference interface (src/common/suffix_array.h:24-29, manber_myers.c):
    create_suffix_array / build_suffix_array / build_lcp_array /
    find_longest_repeated_substring / is_valid_suffix_array / destroy
``SuffixArray`` below drives exactly those six C symbols of libsa_hip.so
through ctypes (the drop-in boundary), with the same argument meaning and
the same results.  ``build_suffix_array`` / ``check_suffix_array`` use the
64-bit extended ABI (sa_build_ex / sa_check) and ``DeviceBuilder`` the
device-resident one (sa_build_device) that bench.py times.

Nothing here computes a suffix array on the CPU: every path runs the HIP
kernels, and raises SAError when no GPU is visible.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _native as N


def _as_bytes_array(text) -> np.ndarray:
    if isinstance(text, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(text), dtype=np.uint8)
    if isinstance(text, str):
        return np.frombuffer(text.encode("latin-1"), dtype=np.uint8)
    return np.ascontiguousarray(text, dtype=np.uint8)


SCHEDULES = {"packed": N.SCHEDULE_PACKED, "reference": N.SCHEDULE_REFERENCE}
RADIX = {"onesweep": 0, "reduce_scan": 1}
ROUND1 = {"auto": N.ROUND1_AUTO, "lsd": N.ROUND1_LSD, "bucketed": N.ROUND1_BUCKETED}


def _opts(profile: bool = False, schedule: str = "packed", init_chars: int = 0,
          radix: str = "onesweep", round1: str = "auto", debug=(), span_extra: int = 0,
          tune: int = 0) -> N.SaOpts:
    """sa_opts; ``debug``: names of N.DEBUG_FLAGS (alternative paths the
    tests force), ``span_extra`` / ``tune``: the debug / A/B fields of
    include/sa_hip.h."""
    o = N.SaOpts()
    o.profile = 1 if profile else 0
    o.schedule = SCHEDULES[schedule]
    o.init_chars = int(init_chars)
    o.radix = RADIX[radix]
    o.round1 = ROUND1[round1]
    o.debug = N.debug_bits(debug)
    o.span_extra = int(span_extra)
    o.tune = int(tune)
    return o


def build_suffix_array(text, width: int = 4, profile: bool = False, return_stats: bool = False,
                       schedule: str = "packed", init_chars: int = 0, radix: str = "onesweep",
                       round1: str = "auto", debug=(), span_extra: int = 0, tune: int = 0):
    """Suffix array of ``text`` (bytes / uint8 array), built on the GPU.

    Unsigned-byte order, end of string smallest (== the reference's order on
    its valid domain, manber_myers.c:81-133).  Returns uint32 (width 4) or
    int64 (width 8); with ``return_stats`` also the per-round statistics.
    ``schedule``: "packed" (default; packed K-symbol first round, later rounds
    re-sort unsorted groups only) or "reference" (h = 1, 2, 4, ... over all
    n suffixes, round for round as manber_myers.c:94-125).  ``round1``
    (packed): "auto", "lsd" (full radix sort of the packed first key) or
    "bucketed" (two bucket passes + per-window LDS sort).  ``debug`` /
    ``span_extra`` / ``tune``: forced alternative paths (tests, A/B runs)."""
    t = _as_bytes_array(text)
    n = int(t.size)
    N.require_device()
    out = np.empty(max(n, 1), dtype=np.uint32 if width == 4 else np.int64)
    st = N.SaStats()
    L = N.lib()
    N.check(L.sa_build_ex(t.ctypes.data if n else None, n, out.ctypes.data, width,
                          ctypes.byref(_opts(profile, schedule, init_chars, radix, round1, debug, span_extra, tune)),
                          ctypes.byref(st)),
            "sa_build_ex")
    out = out[:n]
    return (out, st.to_dict()) if return_stats else out


def check_suffix_array(text, sa) -> bool:
    """O(n) GPU validity check (replaces is_valid_suffix_array, :184-202)."""
    t = _as_bytes_array(text)
    s = np.ascontiguousarray(sa)
    if s.dtype not in (np.uint32, np.int32, np.int64):
        s = s.astype(np.int64)
    if s.size != t.size:
        return False
    N.require_device()
    width = 8 if s.dtype == np.int64 else 4
    r = N.check(N.lib().sa_check(t.ctypes.data if t.size else None, t.size,
                                 s.ctypes.data if s.size else None, width), "sa_check")
    return bool(r)


def lcp_array(text, sa, width: int = 4):
    """LCP array of a valid suffix array on the GPU plus the longest repeated
    substring (replaces build_lcp_array, manber_myers.c:135-157, and
    find_longest_repeated_substring, :159-182).

    Returns (lcp, lrs) with lcp[0] = 0, lcp[r] = lcp(SA[r-1], SA[r]) as uint32
    (width 4) or int64 (width 8), and lrs = (length, SA position) of the first
    r with the strictly largest lcp ((0, 0) when nothing repeats)."""
    t = _as_bytes_array(text)
    s = np.ascontiguousarray(sa)
    if s.dtype not in (np.uint32, np.int32, np.int64):
        s = s.astype(np.int64)
    n = int(t.size)
    if s.size != n:
        raise ValueError(f"SA has {s.size} entries for a text of {n} bytes")
    N.require_device()
    out = np.empty(max(n, 1), dtype=np.uint32 if width == 4 else np.int64)
    ln, pos = ctypes.c_uint64(), ctypes.c_uint64()
    N.check(N.lib().sa_lcp(t.ctypes.data if n else None, n, s.ctypes.data if n else None,
                           8 if s.dtype == np.int64 else 4, out.ctypes.data, ctypes.byref(ln), ctypes.byref(pos)),
            "sa_lcp")
    return out[:n], (int(ln.value), int(pos.value))


class SuffixArray:
    """The reference's SuffixArray object (suffix_array.h:16-21) driven
    through the drop-in C symbols of libsa_hip.so.

    >>> s = SuffixArray(b"banana"); s.build(); s.sa   -> [5, 3, 1, 0, 4, 2]
    """

    def __init__(self, text, n: Optional[int] = None):
        raw = bytes(_as_bytes_array(text))
        self.L = N.lib()
        self.n = len(raw) if n is None else int(n)
        self._buf = ctypes.create_string_buffer(raw, max(len(raw), self.n) + 1)
        self.p = self.L.create_suffix_array(self._buf, self.n)     # manber_myers.c:51-69
        if not self.p:
            raise MemoryError("create_suffix_array returned NULL")

    def build(self) -> None:
        if self.n > 0:
            N.require_device()
        self.L.build_suffix_array(self.p)                           # :81-133

    def build_lcp(self) -> None:
        self.L.build_lcp_array(self.p)                              # :135-157

    def longest_repeated_substring(self) -> Optional[bytes]:
        r = self.L.find_longest_repeated_substring(self.p)          # :159-182
        if not r:
            return None
        s = ctypes.string_at(r)
        ctypes.CDLL(None).free(ctypes.c_void_p(r))
        return s

    def is_valid(self) -> bool:
        if self.n > 0:
            N.require_device()
        return bool(self.L.is_valid_suffix_array(self.p))           # :184-202

    @property
    def text(self) -> bytes:
        return ctypes.string_at(self.p.contents.str, self.n)

    @property
    def sa(self) -> np.ndarray:
        if self.n == 0:
            return np.zeros(0, dtype=np.int32)
        return np.ctypeslib.as_array(self.p.contents.sa, shape=(self.n,)).copy()

    @property
    def lcp(self) -> np.ndarray:
        if self.n == 0:
            return np.zeros(0, dtype=np.int32)
        return np.ctypeslib.as_array(self.p.contents.lcp, shape=(self.n,)).copy()

    def close(self) -> None:
        if getattr(self, "p", None):
            self.L.destroy_suffix_array(self.p)                     # :71-78
            self.p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class DeviceBuilder:
    """Device-resident builder: text and SA live in HBM (torch tensors or raw
    device pointers).  Holds one sa_context (workspace sized for max_n)."""

    def __init__(self, max_n: int, device: int = 0):
        N.require_device()
        self.L = N.lib()
        self.ctx = ctypes.c_void_p()
        N.check(self.L.sa_context_create(device, max_n, ctypes.byref(self.ctx)), "sa_context_create")
        self.device = device

    @staticmethod
    def _ptr(x) -> int:
        return x if isinstance(x, int) else int(x.data_ptr())

    def build(self, d_text, n: int, d_sa, stream=None, profile: bool = False, schedule: str = "packed",
              init_chars: int = 0, radix: str = "onesweep", round1: str = "auto", debug=(), span_extra: int = 0,
              tune: int = 0) -> dict:
        """Build the SA of the n bytes at d_text into the n uint32 at d_sa."""
        st = N.SaStats()
        s = None if stream is None else ctypes.c_void_p(int(stream))
        N.check(self.L.sa_build_device(self.ctx, self._ptr(d_text), n, self._ptr(d_sa), s,
                                       ctypes.byref(_opts(profile, schedule, init_chars, radix, round1, debug,
                                                          span_extra, tune)),
                                       ctypes.byref(st)),
                "sa_build_device")
        return st.to_dict()

    def set_debug(self, debug=(), span_extra: int = 0, tune: int = 0) -> None:
        """Debug / tune fields for the context's sa_dist_* phases (they take
        no sa_opts; sa_build_device applies its own)."""
        N.check(self.L.sa_context_set_debug(self.ctx, ctypes.byref(_opts(debug=debug, span_extra=span_extra,
                                                                          tune=tune))), "sa_context_set_debug")

    def generate_text(self, d_out, n: int, alphabet: bytes, seed: int = 1, stream=None) -> None:
        """Fill n device bytes with the seeded splitmix64 text."""
        s = None if stream is None else ctypes.c_void_p(int(stream))
        N.check(self.L.sa_generate_text_device(self._ptr(d_out), n, seed, alphabet, len(alphabet), s),
                "sa_generate_text_device")

    def check(self, d_text, n: int, d_sa, stream=None) -> bool:
        s = None if stream is None else ctypes.c_void_p(int(stream))
        return bool(N.check(self.L.sa_check_device(self.ctx, self._ptr(d_text), n, self._ptr(d_sa), s),
                            "sa_check_device"))

    def lcp(self, d_text, n: int, d_sa, d_lcp, stream=None) -> tuple:
        """LCP of the SA at d_sa into the n uint32 at d_lcp; returns the longest
        repeated substring as (length, SA position)."""
        s = None if stream is None else ctypes.c_void_p(int(stream))
        ln, pos = ctypes.c_uint64(), ctypes.c_uint64()
        N.check(self.L.sa_lcp_device(self.ctx, self._ptr(d_text), n, self._ptr(d_sa), self._ptr(d_lcp),
                                     ctypes.byref(ln), ctypes.byref(pos), s), "sa_lcp_device")
        return int(ln.value), int(pos.value)

    def close(self) -> None:
        if self.ctx:
            self.L.sa_context_destroy(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
