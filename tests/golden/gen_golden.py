"""Generate tests/golden/rs_golden.json from the CPU oracle (run in the build container only).

    python tests/golden/gen_golden.py

Inputs are regenerated in the tests from the recorded pattern (splitmix64 seed / constant /
ramp), so only expected outputs are stored: full parity bytes for shards <= 64 B, otherwise the
SHA-256 of every parity shard. Reconstruct cases record the erasure pattern; the expected output
of a reconstruct is the original codeword, so its digests are the data/parity digests.
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import rs_oracle as o  # noqa: E402

CODES = [(2, 1), (1, 1), (4, 2), (5, 5), (10, 4), (17, 3), (32, 32)]
LENS = [1, 15, 16, 64, 1000, 4096]
PATTERNS = ["splitmix", "zeros", "ones", "ramp"]
SEED = 0xCE550000


def make_data(k, length, pattern, code_id):
    if pattern == "zeros":
        return [np.zeros(length, np.uint8) for _ in range(k)]
    if pattern == "ones":
        return [np.full(length, 0xFF, np.uint8) for _ in range(k)]
    if pattern == "ramp":
        return [((np.arange(length) + 7 * j) & 0xFF).astype(np.uint8) for j in range(k)]
    seg_bytes = ((k * length + 7) // 8) * 8
    seg = o.synthetic_segment(SEED + code_id, length, seg_bytes)
    return [seg[j * length:(j + 1) * length].copy() for j in range(k)]


def digest(a):
    return hashlib.sha256(a.tobytes()).hexdigest()


def main():
    rng = np.random.default_rng(1234)
    cases = []
    for ci, (k, m) in enumerate(CODES):
        rs = o.ReedSolomon(k, m)
        for length in LENS:
            for pat in PATTERNS:
                if pat != "splitmix" and length not in (16, 1000):
                    continue
                data = make_data(k, length, pat, ci)
                par = rs.encode(data)
                c = {"k": k, "m": m, "len": length, "pattern": pat, "code_id": ci,
                     "data_sha256": [digest(d) for d in data],
                     "parity_sha256": [digest(p) for p in par]}
                if length <= 64:
                    c["parity_hex"] = [p.tobytes().hex() for p in par]
                # erasure patterns
                n = k + m
                pats = []
                if (k, m) == (2, 1):
                    pats = [[i] for i in range(3)]
                else:
                    for _ in range(3):
                        e = int(rng.integers(1, m + 1))
                        pats.append(sorted(rng.choice(n, size=e, replace=False).tolist()))
                rec = []
                for erased in pats:
                    shards = list(data) + list(par)
                    for i in erased:
                        shards[i] = None
                    for data_only in (False, True):
                        out = rs.reconstruct(list(shards), data_only=data_only)
                        full = list(data) + list(par)
                        for i in range(n):
                            if out[i] is None:
                                assert data_only and i >= k
                                continue
                            assert np.array_equal(out[i], full[i]), (k, m, erased, i)
                        rec.append({"erased": erased, "data_only": data_only})
                c["reconstruct"] = rec
                cases.append(c)
    e21 = o.build_matrix(2, 3)
    e3232 = o.build_matrix(32, 64)
    kat = {
        "source": "public known answers (Backblaze JavaReedSolomon / klauspost reedsolomon unit "
                  "tests; not present in /root/reference) + oracle-derived CESS matrices",
        "one_encode_5_5": {"data": [[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]],
                           "parity": [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]]},
        "gal_mul": [[3, 4, 12], [7, 7, 21], [23, 45, 41]],
        "gal_exp": [[2, 2, 4], [5, 20, 235], [13, 7, 43]],
        "inverse_3x3": {"in": [[56, 23, 98], [3, 100, 200], [45, 201, 123]],
                        "out": [[175, 133, 33], [130, 13, 245], [112, 35, 126]]},
        "inverse_5x5": {"in": [[1, 0, 0, 0, 0], [0, 1, 0, 0, 0], [0, 0, 0, 1, 0],
                               [0, 0, 0, 0, 1], [7, 7, 6, 6, 1]],
                        "out": [[1, 0, 0, 0, 0], [0, 1, 0, 0, 0], [123, 123, 1, 122, 122],
                                [0, 0, 1, 0, 0], [0, 0, 0, 1, 0]]},
        "mat_mul_2x2": {"a": [[1, 2], [3, 4]], "b": [[5, 6], [7, 8]], "out": [[11, 22], [19, 42]]},
        "matrix_2_1": e21,
        "matrix_32_32_parity_hex": bytes(sum(e3232[32:], [])).hex(),
    }
    # the splitmix64 input generator, pinned by its first words
    gen = o.synthetic_segment(SEED + 1, 3, 32)
    out = {"seed": SEED, "kat": kat, "splitmix_seed1_seg3_32B": gen.tobytes().hex(),
           "cases": cases}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rs_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0, separators=(",", ":"))
    print(f"wrote {len(cases)} cases to {path} ({os.path.getsize(path)} bytes)")


if __name__ == "__main__":
    main()
