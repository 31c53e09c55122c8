"""Generate tests/golden/ fixtures from the reference itself.

Run in the survey container only (needs /root/reference):
    make -C oracle ref && python tests/golden/make_golden.py

Inputs come from the seeded splitmix64 generator or are the
reference's own smoke strings (Makefile:119-138, generate_large_datasets.py:
90-96).  Expected outputs (SA, LCP, LRS, validator verdict) are produced by
oracle/_ref/libmm.so, i.e. the reference's src/sequential/manber_myers.c
compiled unmodified from where it lies.  Inputs outside the reference's valid
domain (bytes >= 0x80 or NUL) cannot come from it: those
fixtures are produced by this repo's C restatement AND the independent numpy
restatement, which must agree, and are tagged source="restatement".

Output: golden.npz (arrays) + golden.json (index, hashes, provenance).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def cases():
    # reference smoke strings (Makefile:119-138; generate_large_datasets.py:90-96)
    yield "banana", b"banana"
    yield "mississippi", b"mississippi"
    yield "abcabcabc", b"abcabcabc"
    yield "a_x1000", b"a" * 1000
    yield "ab_x500", b"ab" * 500
    yield "single", b"x"
    yield "pair_desc", b"ba"
    yield "pair_eq", b"zz"
    # seeded random, ragged and power-of-two-adjacent sizes
    for kind in ("dna", "alnum", "ascii127", "binary"):
        for n in (2, 3, 7, 63, 64, 65, 1000, 4095, 4097, 65536):
            yield f"{kind}_{n}", O.gen_text(kind, n, seed=1).tobytes()
    # periodic text (many long repeats)
    period = O.gen_text("alnum", 97, seed=7).tobytes()
    yield "periodic97_20000", (period * (20000 // 97 + 1))[:20000]
    # outside the reference domain: unsigned bytes incl. NUL and 0xFF
    for n in (1, 2, 255, 4096, 65536):
        yield f"byte256_{n}", O.gen_text("byte256", n, seed=1).tobytes()
    yield "ff_ff", b"\xff\xff"


def main():
    ref = O.RefLib()
    arrays, index = {}, {}
    for name, text in cases():
        t = np.frombuffer(text, dtype=np.uint8)
        in_domain = len(text) > 0 and t.min() >= 1 and t.max() <= 0x7F
        sa_c = O.sa_c(t)
        sa_np = O.sa_numpy(t)
        assert (sa_c == sa_np).all(), name
        lcp = O.lcp_c(t, sa_c)
        lrs = O.lrs_c(t, sa_c, lcp)
        if in_domain:
            sa_r, lcp_r, lrs_r, valid_r = ref.run(text, lcp=True)
            assert (sa_r.astype(np.uint32) == sa_c).all(), f"restatement != reference on {name}"
            assert (lcp_r.astype(np.uint32) == lcp).all(), f"lcp mismatch on {name}"
            assert (lrs_r or b"") == lrs, f"lrs mismatch on {name}"
            assert valid_r, name
            source = "reference"
        else:
            source = "restatement"
        arrays[f"{name}__text"] = t
        arrays[f"{name}__sa"] = sa_c.astype(np.uint32)
        arrays[f"{name}__lcp"] = lcp
        index[name] = {
            "n": len(text), "source": source,
            "lrs": lrs.hex(), "sa_sha256_i32": O.sha256(sa_c.astype(np.int32)),
        }
    np.savez_compressed(os.path.join(OUT, "golden.npz"), **arrays)

    # large known answers (SHA-256 of int32 little-endian SA): regenerated
    # here from the reference at 1 MiB; the 64 MiB and 2^30-1 rows are the
    # reference runs recorded in SURVEY.md 8(c) (the 64 MiB row is re-derived
    # by tests/test_oracle.py::test_known_answer_64mib with the restatement).
    known = {}
    for kind in ("alnum", "ascii127", "dna"):
        t = O.gen_text(kind, 1 << 20, seed=1)
        sa_r, _, lrs_r, _ = ref.run(t.tobytes(), lcp=True)
        known[f"{kind}_1MiB"] = {"kind": kind, "n": 1 << 20, "seed": 1, "text_sha256": O.sha256(t),
                                 "sa_sha256_i32": O.sha256(sa_r.astype(np.int32)),
                                 "lrs": (lrs_r or b"").decode(), "source": "reference"}
    t = O.gen_text("byte256", 1 << 20, seed=1)
    known["byte256_1MiB"] = {"kind": "byte256", "n": 1 << 20, "seed": 1, "text_sha256": O.sha256(t),
                             "sa_sha256_i32": O.sha256(O.sa_c(t).astype(np.int32)),
                             "source": "restatement+numpy (reference crashes on bytes >= 0x80)"}
    known["dna_64MiB"] = {"kind": "dna", "n": 1 << 26, "seed": 1,
                          "text_sha256": "a6613097b9f345c7a28348b29b68bbdd947df369d245b62a861109781434590c",
                          "sa_sha256_i32": "f08a0541d457003c33744e8d7107aa1c645d3d21241dc340376dd6a62344b3dc",
                          "rounds": 5, "source": "reference (SURVEY.md 8(c))"}
    known["dna_1GiB_minus_1"] = {"kind": "dna", "n": (1 << 30) - 1, "seed": 1,
                                 "text_sha256": "0257ad9a94d5893f8c4e473c02eecbb1de66e27edec8826919c5f2c1096753ee",
                                 "sa_sha256_i32": "1f5e7640ba5c615c149a57c0dcad960e0733957a0e2a0c6e3350e4f7553aac14",
                                 "rounds": 5, "lrs": "CGAGGGGGTAACTCTTCTACTGACCACT",
                                 "source": "reference (SURVEY.md 8(c))"}
    with open(os.path.join(OUT, "golden.json"), "w") as f:
        json.dump({"cases": index, "known_answers": known}, f, indent=1, sort_keys=True)
    print(f"wrote {len(index)} cases")


if __name__ == "__main__":
    main()
