"""The 2-bit packed digit layout of the DNA paths, restated on the host.

k_split_text<.., DNA> (sa_split.h) packs each staged word of four dense
digits (one per byte, the first in the low byte) into one byte with the first
digit on top, and keys position l0 + j of a lane from the 64-bit window
bswap(alignbyte(...)) of the packed bytes at l0 / 4: D = window << 2j >> (64 -
2s), r = (window << 2j >> (64 - 2K)) & (4^R - 1).  k_bucket_hist<.., 3, .., DNA>
(sa_bucket.h) packs a lane's 16 digits into one word the same way and takes
a position's bucket as the top bb bits of its shifted window.  This checks
both against D / r / bucket computed digit by digit (manber_myers.c's ranks
in the packed schedule's key1 layout), for random DNA tiles and
every lane offset the kernels use."""
import numpy as np

DNA = np.frombuffer(b"ACGT", np.uint8)


def swar_digits(word: int) -> int:
    # ((b >> 1) ^ (b >> 2)) & 3 per byte: A C G T -> 0 1 2 3
    return ((word >> 1) ^ (word >> 2)) & 0x03030303


def pack_byte(o: int) -> int:
    # the kernels' expression: four digits, the first (low byte) on top
    return ((o & 3) << 6) | ((o >> 4) & 0x30) | ((o >> 14) & 0xC) | (o >> 24)


def alignbyte(hi: int, lo: int, sh: int) -> int:
    return (((hi << 32) | lo) >> (8 * sh)) & 0xFFFFFFFF


def bswap32(x: int) -> int:
    return int.from_bytes(x.to_bytes(4, "little"), "big")


def test_swar_digit_map():
    for b, d in zip(b"ACGT", range(4)):
        assert swar_digits(b) & 3 == d
    w = int.from_bytes(b"GATC", "little")
    assert swar_digits(w) == int.from_bytes(bytes([2, 0, 3, 1]), "little")


def test_first_pass_windows():
    rng = np.random.default_rng(7)
    items, s, R = 12, 9, 11
    K = s + R
    bb = 17
    for trial in range(20):
        text = DNA[rng.integers(0, 4, 6144 + 64)]
        digits = ((text >> 1) ^ (text >> 2)) & 3
        words = [int.from_bytes(text[4 * w: 4 * w + 4].tobytes(), "little") for w in range(len(text) // 4)]
        packed = bytes(pack_byte(swar_digits(w)) for w in words) + bytes(16)
        p32 = [int.from_bytes(packed[4 * i: 4 * i + 4], "little") for i in range(len(packed) // 4)]
        for dg in list(range(0, 512, 37)) + [511]:
            l0 = items * dg
            bo = l0 // 4
            sh = bo & 3
            w0, w1, w2 = p32[bo >> 2], p32[(bo >> 2) + 1], p32[(bo >> 2) + 2]
            win = (bswap32(alignbyte(w1, w0, sh)) << 32) | bswap32(alignbyte(w2, w1, sh))
            for j in range(items):
                x = (win << (2 * j)) & (2**64 - 1)
                D = x >> (64 - 2 * s)
                r = (x >> (64 - 2 * K)) & ((1 << (2 * R)) - 1)
                p = l0 + j
                wantD = 0
                for q in range(s):
                    wantD = wantD * 4 + int(digits[p + q])
                wantr = 0
                for q in range(R):
                    wantr = wantr * 4 + int(digits[p + s + q])
                assert (D, r) == (wantD, wantr), (trial, dg, j)
                assert D >> (2 * s - bb) == x >> (64 - bb)   # the bucket as a bit field of the window


def test_record_scan_words():
    rng = np.random.default_rng(11)
    run, bb, s = 16, 17, 9
    text = DNA[rng.integers(0, 4, 4096 + 64)]
    digits = ((text >> 1) ^ (text >> 2)) & 3
    lane_words = []
    for lane in range(256 + 4):
        pk = 0
        for q in range(4):
            o = swar_digits(int.from_bytes(text[16 * lane + 4 * q: 16 * lane + 4 * q + 4].tobytes(), "little"))
            pk |= pack_byte(o) << (24 - 8 * q)
        lane_words.append(pk)
    # the halo words as wave 0 builds them: 16 lanes' digits OR-ed
    for i in range(4):
        v = 0
        for y in range(16):
            v |= int(digits[4096 + 16 * i + y]) << (30 - 2 * y)
        assert v == lane_words[256 + i]
    for lane in range(256):
        wpk = (lane_words[lane] << 32) | lane_words[lane + 1]
        for j in range(run):
            p = 16 * lane + j
            D = 0
            for q in range(s):
                D = D * 4 + int(digits[p + q])
            assert ((wpk << (2 * j)) & (2**64 - 1)) >> (64 - bb) == D >> (2 * s - bb)
