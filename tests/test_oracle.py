"""Pin the CPU oracle (Python and C restatements) before trusting it as the checker.

Sources: public known answers (Backblaze / klauspost unit-test values, recorded in
tests/golden/rs_golden.json "kat"), NIST SHAVS vectors shipped in the reference
(utils/ring/third_party/NIST/SHAVS/SHA256{Short,Long}Msg.rsp, SHA256Monte.rsp) and the
reference's digest test inputs (utils/ring/tests/digest_tests.txt:25-33).
"""
import hashlib
import itertools

import numpy as np
import pytest

from tests.conftest import case_data, parse_shavs
from oracle.c_oracle import c_encode, c_sha256_hex, ptrs


def test_galois_kats(orc, golden):
    kat = golden["kat"]
    for a, b, want in kat["gal_mul"]:
        assert orc.gal_mul(a, b) == want
    for a, n, want in kat["gal_exp"]:
        assert orc.gal_exp(a, n) == want
    assert orc.mat_invert(kat["inverse_3x3"]["in"]) == kat["inverse_3x3"]["out"]
    assert orc.mat_invert(kat["inverse_5x5"]["in"]) == kat["inverse_5x5"]["out"]
    mm = kat["mat_mul_2x2"]
    assert orc.mat_mul(mm["a"], mm["b"]) == mm["out"]


def test_one_encode_5_5(orc, corc, golden):
    """Backblaze/klauspost TestOneEncode: RS(5,5) over 2-byte shards."""
    kat = golden["kat"]["one_encode_5_5"]
    data = [np.array(d, np.uint8) for d in kat["data"]]
    assert [p.tolist() for p in orc.ReedSolomon(5, 5).encode(data)] == kat["parity"]
    assert [p.tolist() for p in c_encode(corc, 5, 5, data)] == kat["parity"]


def test_cess_matrices(orc, corc, golden):
    kat = golden["kat"]
    assert orc.build_matrix(2, 3) == kat["matrix_2_1"]
    assert kat["matrix_2_1"][2] == [3, 2]  # p = 3*d0 ^ 2*d1
    m = np.zeros(64 * 32, np.uint8)
    corc.orc_matrix(32, 32, m.ctypes.data_as(__import__("ctypes").POINTER(
        __import__("ctypes").c_uint8)))
    assert m[32 * 32:].tobytes().hex() == kat["matrix_32_32_parity_hex"]


def test_shavs_short_long(corc):
    vecs = parse_shavs("SHA256ShortMsg.rsp") + parse_shavs("SHA256LongMsg.rsp")
    assert len(vecs) == 65 + 64
    for msg, md in vecs:
        assert hashlib.sha256(msg).hexdigest() == md
        assert c_sha256_hex(corc, msg).decode() == md


def test_shavs_monte(corc):
    """SHAVS Monte Carlo: MD_i = SHA256(MD_{i-3} || MD_{i-2} || MD_{i-1}), 1000 per checkpoint."""
    import os
    from tests.conftest import GOLDEN
    seed, mds = None, []
    with open(os.path.join(GOLDEN, "SHA256Monte.rsp")) as f:
        for line in f:
            line = line.strip()
            if line.startswith("Seed ="):
                seed = bytes.fromhex(line.split("=")[1].strip())
            elif line.startswith("MD ="):
                mds.append(line.split("=")[1].strip())
    md = seed
    for want in mds[:3]:  # 3 checkpoints = 3000 hashes keeps the CPU suite fast
        a = b = c = md
        for _ in range(1000):
            m = a + b + c
            a, b, c = b, c, bytes.fromhex(c_sha256_hex(corc, m).decode())
        md = c
        assert md.hex() == want


def test_digest_tests_txt(corc):
    """utils/ring/tests/digest_tests.txt:25-33 (SHA256 "abc" and the 448-bit message)."""
    assert c_sha256_hex(corc, b"abc").decode() == \
        "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"
    msg = b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq"
    assert c_sha256_hex(corc, msg).decode() == \
        "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"


def test_golden_cases_python_and_c(orc, corc, golden):
    """Both restatements reproduce every golden parity digest."""
    for case in golden["cases"]:
        k, m = case["k"], case["m"]
        data = case_data(case)
        assert [hashlib.sha256(d.tobytes()).hexdigest() for d in data] == case["data_sha256"]
        py = orc.ReedSolomon(k, m).encode(data)
        c = c_encode(corc, k, m, data)
        for p, q, want in zip(py, c, case["parity_sha256"]):
            assert hashlib.sha256(p.tobytes()).hexdigest() == want
            assert np.array_equal(p, q)
        if "parity_hex" in case:
            assert [p.tobytes().hex() for p in py] == case["parity_hex"]


def test_c_reconstruct_golden(orc, corc, golden):
    for case in golden["cases"]:
        if case["len"] > 1000:
            continue
        k, m = case["k"], case["m"]
        data = case_data(case)
        full = data + c_encode(corc, k, m, data)
        for rec in case["reconstruct"]:
            shards = [s.copy() for s in full]
            present = np.ones(k + m, np.uint8)
            for i in rec["erased"]:
                shards[i][:] = 0
                present[i] = 0
            rc = corc.orc_reconstruct(k, m, ptrs(shards),
                                      present.ctypes.data_as(__import__("ctypes").POINTER(
                                          __import__("ctypes").c_uint8)),
                                      case["len"], int(rec["data_only"]))
            assert rc == 0
            for i in range(k + m):
                if rec["data_only"] and i >= k and i in rec["erased"]:
                    continue
                assert np.array_equal(shards[i], full[i]), (k, m, rec, i)


@pytest.mark.parametrize("k,m", [(2, 1), (3, 2), (4, 3)])
def test_any_k_of_n_exhaustive(orc, k, m):
    rs = orc.ReedSolomon(k, m)
    rng = np.random.default_rng(k * 10 + m)
    data = [rng.integers(0, 256, 37, dtype=np.uint8) for _ in range(k)]
    full = data + rs.encode(data)
    n = k + m
    for e in range(1, m + 1):
        for erased in itertools.combinations(range(n), e):
            shards = [None if i in erased else full[i] for i in range(n)]
            out = rs.reconstruct(shards)
            assert all(np.array_equal(a, b) for a, b in zip(out, full))
    with pytest.raises(ValueError):
        rs.reconstruct([None] * (m + 1) + full[m + 1:])


def test_split_and_segment_list(orc):
    rs = orc.ReedSolomon(2, 1)
    sh = rs.split(b"abcde")
    assert [s.tobytes() for s in sh] == [b"abc", b"de\x00", b"\x00\x00\x00"]
    with pytest.raises(ValueError):
        rs.split(b"")
    segs = orc.segment_list(b"x" * 100, segment_size=64)
    assert len(segs) == 2 and all(len(f) == 3 and len(h) == 64 for h, f in segs)


def test_synthetic_generator_pinned(orc, corc, golden):
    want = bytes.fromhex(golden["splitmix_seed1_seg3_32B"])
    assert orc.synthetic_segment(golden["seed"] + 1, 3, 32).tobytes() == want
    buf = np.zeros(32, np.uint8)
    corc.orc_fill_synthetic(buf.ctypes.data, 32, 1, 3, golden["seed"] + 1)
    assert buf.tobytes() == want


@pytest.mark.parametrize("k,m", [(4, 3), (2, 1), (32, 32)])
def test_c_simd_matches_scalar(corc, k, m):
    """Scalar table, AVX2 split-nibble and AVX-512 GFNI affine forms of the C oracle agree
    (each form the host lacks falls back, so the comparison is against what runs)."""
    rng = np.random.default_rng(5 + k)
    data = [rng.integers(0, 256, 4099, dtype=np.uint8) for _ in range(k)]
    corc.orc_set_simd(0)
    a = c_encode(corc, k, m, data)
    for mode in (1, 2, -1):
        got = corc.orc_set_simd(mode)
        b = c_encode(corc, k, m, data)
        assert all(np.array_equal(x, y) for x, y in zip(a, b)), (mode, got)
    corc.orc_set_simd(-1)


def test_c_segment_ops_threaded(corc):
    """orc_segment_ops (config 1's CPU leg): encode + every single-erasure rebuild of one segment
    split over threads leaves the shards a consistent codeword."""
    from oracle.c_oracle import ptrs
    k, m, F = 2, 1, (1 << 16) + 40
    rng = np.random.default_rng(11)
    data = [rng.integers(0, 256, F, dtype=np.uint8) for _ in range(k)]
    want = data + c_encode(corc, k, m, data)
    sh = [d.copy() for d in data] + [np.zeros(F, np.uint8)]
    corc.orc_segment_ops(k, m, ptrs(sh), F, 5, 2)
    assert all(np.array_equal(x, y) for x, y in zip(sh, want))
