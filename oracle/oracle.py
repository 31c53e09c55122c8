"""oracle/oracle.py -- Python side of the CPU oracle.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker; the product path
(hpc_suffix_array_amd) never does.

Contents
  * gen_text        -- the seeded splitmix64 input generator of SURVEY.md 8(d)
                       (numpy, bit-identical to oracle_gen_text in mm_oracle.c)
  * sa_c / lcp_c / lrs_c / check_c / is_valid_ref_c
                    -- ctypes wrappers over oracle/build/liboracle.so, the C
                       restatement of src/sequential/manber_myers.c:15-202
  * sa_numpy        -- an independent prefix-doubling restatement with
                       numpy.lexsort (small n), used to cross-check the C one
  * RefLib          -- ctypes driver for oracle/_ref/libmm.so, the reference's
                       own manber_myers.c compiled from /root/reference (only
                       present in the survey container; used to pin fixtures)
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import string
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
REF_LIB_PATH = os.path.join(HERE, "_ref", "libmm.so")

# alphabets of SURVEY.md 8(d); "alnum" is the reference's "random" data,
# scripts/generate_large_datasets.py:14 (ascii_letters + digits, in that order)
ALPHABETS = {
    "dna": b"ACGT",
    "alnum": (string.ascii_letters + string.digits).encode(),
    "ascii127": bytes(range(1, 128)),
    "byte256": bytes(range(256)),
    "binary": b"ab",
}

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def gen_text(kind: str, n: int, seed: int = 1, chunk: int = 1 << 24) -> np.ndarray:
    """splitmix64 text generator; returns a uint8 array.

    z = seed + (i+1)*0x9E3779B97F4A7C15; z = (z^z>>30)*0xBF58476D1CE4E5B9;
    z = (z^z>>27)*0x94D049BB133111EB; z ^= z>>31;
    sym = alphabet[((z>>32)*sigma)>>32].
    ``kind`` "degenerate" gives n copies of 'a' (config 5).
    """
    if kind == "degenerate":
        return np.full(n, ord("a"), dtype=np.uint8)
    alpha = np.frombuffer(ALPHABETS[kind], dtype=np.uint8)
    sigma = np.uint64(len(alpha))
    out = np.empty(n, dtype=np.uint8)
    with np.errstate(over="ignore"):
        for lo in range(0, n, chunk):
            hi = min(n, lo + chunk)
            i = np.arange(lo + 1, hi + 1, dtype=np.uint64)
            z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            z = z ^ (z >> np.uint64(31))
            out[lo:hi] = alpha[((z >> np.uint64(32)) * sigma) >> np.uint64(32)]
    return out


def sha256(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# ----------------------------------------------------------------------------
# C restatement (liboracle.so)
# ----------------------------------------------------------------------------
_lib = None


def build_oracle() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "oracle"], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build_oracle()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        u64 = ctypes.c_uint64
        L.oracle_gen_text.argtypes = [u8p, u64, u64, u8p, ctypes.c_uint32]
        L.oracle_build_sa.argtypes = [u8p, u64, u32p, ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
        L.oracle_build_sa.restype = ctypes.c_int
        L.oracle_lcp.argtypes = [u8p, u64, u32p, u32p]
        L.oracle_lcp.restype = ctypes.c_int
        L.oracle_lrs.argtypes = [u64, u32p, u32p, ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_lrs.restype = ctypes.c_uint64
        L.oracle_is_valid_ref.argtypes = [u8p, u64, u32p]
        L.oracle_is_valid_ref.restype = ctypes.c_int
        L.oracle_check_sa.argtypes = [u8p, u64, u32p]
        L.oracle_check_sa.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def _text(text) -> np.ndarray:
    if isinstance(text, (bytes, bytearray)):
        return np.frombuffer(bytes(text), dtype=np.uint8)
    t = np.ascontiguousarray(text, dtype=np.uint8)
    return t if t.size else np.zeros(1, np.uint8)[:0]


def gen_text_c(kind: str, n: int, seed: int = 1) -> np.ndarray:
    alpha = np.frombuffer(ALPHABETS[kind], dtype=np.uint8).copy()
    out = np.empty(max(n, 1), dtype=np.uint8)
    lib().oracle_gen_text(_p(out, ctypes.c_uint8), n, seed, _p(alpha, ctypes.c_uint8), len(alpha))
    return out[:n]


def sa_c(text, stats: bool = False):
    """Reference-identical rank doubling (manber_myers.c:81-133), unsigned bytes.

    Returns the SA as uint32; with ``stats`` also (rounds, round_ms, D_j)."""
    t = _text(text)
    n = t.size
    sa = np.empty(max(n, 1), dtype=np.uint32)
    ms = np.zeros(64, dtype=np.float64)
    dj = np.zeros(64, dtype=np.uint64)
    tt = t if n else np.zeros(1, np.uint8)
    r = lib().oracle_build_sa(_p(tt, ctypes.c_uint8), n, _p(sa, ctypes.c_uint32),
                              _p(ms, ctypes.c_double), _p(dj, ctypes.c_uint64), 64)
    if r < 0:
        raise MemoryError("oracle_build_sa: allocation failed")
    sa = sa[:n]
    if stats:
        return sa, r, ms[:r].tolist(), [int(x) for x in dj[:r]]
    return sa


def lcp_c(text, sa) -> np.ndarray:
    t = _text(text)
    n = t.size
    sa = np.ascontiguousarray(sa, dtype=np.uint32)
    lcp = np.zeros(max(n, 1), dtype=np.uint32)
    if n:
        lib().oracle_lcp(_p(t, ctypes.c_uint8), n, _p(sa, ctypes.c_uint32), _p(lcp, ctypes.c_uint32))
    return lcp[:n]


def lrs_c(text, sa, lcp) -> bytes:
    """Longest repeated substring as find_longest_repeated_substring
    (manber_myers.c:159-182) returns it; b"" when there is none."""
    t = _text(text)
    n = t.size
    if n == 0:
        return b""
    sa = np.ascontiguousarray(sa, dtype=np.uint32)
    lcp = np.ascontiguousarray(lcp, dtype=np.uint32)
    pos = ctypes.c_uint64(0)
    ln = lib().oracle_lrs(n, _p(sa, ctypes.c_uint32), _p(lcp, ctypes.c_uint32), ctypes.byref(pos))
    return bytes(t[pos.value:pos.value + ln])


def check_c(text, sa) -> bool:
    """O(n) suffix-array checker (permutation + adjacent-pair ISA test)."""
    t = _text(text)
    sa = np.ascontiguousarray(sa, dtype=np.uint32)
    if t.size != sa.size:
        return False
    if t.size == 0:
        return True
    return bool(lib().oracle_check_sa(_p(t, ctypes.c_uint8), t.size, _p(sa, ctypes.c_uint32)))


def is_valid_ref_c(text, sa) -> bool:
    """Reference validator semantics (manber_myers.c:184-202)."""
    t = _text(text)
    sa = np.ascontiguousarray(sa, dtype=np.uint32)
    if t.size == 0:
        return True
    return bool(lib().oracle_is_valid_ref(_p(t, ctypes.c_uint8), t.size, _p(sa, ctypes.c_uint32)))


# ----------------------------------------------------------------------------
# independent numpy restatement (prefix doubling with lexsort), small n
# ----------------------------------------------------------------------------
def sa_numpy(text) -> np.ndarray:
    """Prefix doubling with numpy.lexsort: rank_2h from (rank_h[i], rank_h[i+h]).
    Unsigned bytes, end-of-string smallest.  Independent of the C code."""
    t = _text(text).astype(np.int64)
    n = t.size
    if n == 0:
        return np.zeros(0, dtype=np.uint32)
    rank = t + 1
    h = 1
    while True:
        nxt = np.zeros(n, dtype=np.int64)
        if h < n:
            nxt[:n - h] = rank[h:]
        order = np.lexsort((nxt, rank))
        a, b = rank[order], nxt[order]
        flag = np.ones(n, dtype=np.int64)
        flag[1:] = (a[1:] != a[:-1]) | (b[1:] != b[:-1])
        new = np.empty(n, dtype=np.int64)
        new[order] = np.cumsum(flag)
        rank = new
        if rank.max() == n or h >= n:
            return order.astype(np.uint32)
        h *= 2


# ----------------------------------------------------------------------------
# the reference itself, compiled from /root/reference (survey container only)
# ----------------------------------------------------------------------------
class _SuffixArray(ctypes.Structure):
    # layout of SuffixArray, src/common/suffix_array.h:16-21
    _fields_ = [("str", ctypes.c_void_p), ("n", ctypes.c_int),
                ("sa", ctypes.POINTER(ctypes.c_int)), ("lcp", ctypes.POINTER(ctypes.c_int))]


class RefLib:
    """Drives oracle/_ref/libmm.so (reference manber_myers.c, unmodified)."""

    def __init__(self, path: str = REF_LIB_PATH):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        L = ctypes.CDLL(path)
        L.create_suffix_array.argtypes = [ctypes.c_char_p, ctypes.c_int]
        L.create_suffix_array.restype = ctypes.POINTER(_SuffixArray)
        L.destroy_suffix_array.argtypes = [ctypes.POINTER(_SuffixArray)]
        L.build_suffix_array.argtypes = [ctypes.POINTER(_SuffixArray)]
        L.build_lcp_array.argtypes = [ctypes.POINTER(_SuffixArray)]
        L.find_longest_repeated_substring.argtypes = [ctypes.POINTER(_SuffixArray)]
        L.find_longest_repeated_substring.restype = ctypes.c_void_p
        L.is_valid_suffix_array.argtypes = [ctypes.POINTER(_SuffixArray)]
        L.is_valid_suffix_array.restype = ctypes.c_int
        self.L = L
        self.libc = ctypes.CDLL(None)
        self.libc.free.argtypes = [ctypes.c_void_p]

    def run(self, text: bytes, lcp: bool = False):
        """Returns (sa int32 array, lcp or None, lrs bytes or None, valid)."""
        n = len(text)
        p = self.L.create_suffix_array(text, n)
        if not p:
            raise MemoryError("create_suffix_array returned NULL")
        try:
            self.L.build_suffix_array(p)
            sa = np.ctypeslib.as_array(p.contents.sa, shape=(n,)).copy() if n else np.zeros(0, np.int32)
            lc, lrs, valid = None, None, None
            if lcp:
                self.L.build_lcp_array(p)
                lc = np.ctypeslib.as_array(p.contents.lcp, shape=(n,)).copy()
                r = self.L.find_longest_repeated_substring(p)
                if r:
                    lrs = ctypes.string_at(r)
                    self.libc.free(r)
                valid = bool(self.L.is_valid_suffix_array(p))
            return sa, lc, lrs, valid
        finally:
            self.L.destroy_suffix_array(p)
