"""Host SHA-256 of libcessec (cec_sha256_host, cess_amd/csrc/sha256_host.cpp), CPU only: every
form the CPU has (portable, SHA-NI x1 / x2 / x4, AVX-512 x16) against the reference's NIST SHAVS
vectors (tests/golden/SHA256{Short,Long}Msg.rsp, from utils/ring/third_party/NIST/SHAVS/) and
against hashlib at the padding edges, with prefix digests (a segment chain's fragment-0 digest)
and groups that do not fill a form's width, on one and several threads."""
import ctypes
import hashlib

import numpy as np
import pytest

from tests.conftest import parse_shavs

FORMS = {"scalar": 0, "ni1": 1, "ni2": 2, "ni4": 3, "x16": 4}


@pytest.fixture(scope="module")
def lib():
    from cess_amd import _lib
    return _lib.load()


def host_hex(lib, bufs, length, prefix=0, threads=1):
    n = len(bufs)
    keep = [np.frombuffer(b, np.uint8) if len(b) else np.zeros(1, np.uint8) for b in bufs]
    ptrs = (ctypes.c_void_p * max(1, n))(*[k.ctypes.data for k in keep])
    hexo = np.zeros(64 * max(1, n), np.uint8)
    phex = np.zeros(64 * max(1, n), np.uint8)
    rc = lib.cec_sha256_host(ptrs, n, length, hexo.ctypes.data, prefix,
                             phex.ctypes.data if prefix else None, threads)
    assert rc == 0
    out = [bytes(hexo[64 * i:64 * i + 64]).decode() for i in range(n)]
    pre = [bytes(phex[64 * i:64 * i + 64]).decode() for i in range(n)] if prefix else None
    return out, pre


def forms(lib):
    out = []
    for name, f in FORMS.items():
        if lib.cec_host_sha_set_form(f) == 0:
            out.append(name)
    lib.cec_host_sha_set_form(-1)
    return out


def test_shavs_every_form(lib):
    vecs = parse_shavs("SHA256ShortMsg.rsp") + parse_shavs("SHA256LongMsg.rsp")
    assert len(vecs) == 129
    have = forms(lib)
    assert "scalar" in have
    try:
        for name in have:
            assert lib.cec_host_sha_set_form(FORMS[name]) == 0
            for msg, md in vecs:
                # the message as a group of 16 equal chains: every lane / interleave slot
                got, _ = host_hex(lib, [msg] * 16, len(msg))
                assert got == [md] * 16, (name, len(msg))
    finally:
        lib.cec_host_sha_set_form(-1)


@pytest.mark.parametrize("length", [0, 1, 55, 56, 63, 64, 65, 119, 120, 127, 128, 4096 + 13])
@pytest.mark.parametrize("n", [1, 2, 3, 5, 16, 17, 35])
def test_lengths_and_groups_vs_hashlib(lib, length, n):
    rng = np.random.default_rng(length * 131 + n)
    bufs = [rng.integers(0, 256, length, dtype=np.uint8).tobytes() for _ in range(n)]
    want = [hashlib.sha256(b).hexdigest() for b in bufs]
    prefix = 64 if length >= 64 else 0
    for name in forms(lib):
        lib.cec_host_sha_set_form(FORMS[name])
        try:
            for threads in (1, 3):
                got, pre = host_hex(lib, bufs, length, prefix, threads)
                assert got == want, (name, threads)
                if prefix:
                    assert pre == [hashlib.sha256(b[:prefix]).hexdigest() for b in bufs]
        finally:
            lib.cec_host_sha_set_form(-1)


def test_segment_chain_prefix_is_fragment_zero(lib):
    """The record convention: a segment's chain yields data fragment 0's digest as its prefix
    (the split is contiguous), as the GPU hash queue's cec_hashq_add_prefix does."""
    F = 4096 * 3
    segs = [np.random.default_rng(s).integers(0, 256, 2 * F, dtype=np.uint8).tobytes()
            for s in range(20)]
    got, pre = host_hex(lib, segs, 2 * F, F, threads=4)
    assert got == [hashlib.sha256(s).hexdigest() for s in segs]
    assert pre == [hashlib.sha256(s[:F]).hexdigest() for s in segs]


def test_arguments(lib):
    buf = np.zeros(128, np.uint8)
    ptrs = (ctypes.c_void_p * 1)(buf.ctypes.data)
    hexo = np.zeros(64, np.uint8)
    assert lib.cec_sha256_host(ptrs, 1, 128, hexo.ctypes.data, 32, hexo.ctypes.data, 1) == -1
    assert lib.cec_sha256_host(ptrs, 1, 128, hexo.ctypes.data, 192, hexo.ctypes.data, 1) == -1
    assert lib.cec_sha256_host(ptrs, 1, 128, hexo.ctypes.data, 64, None, 1) == -1
    assert lib.cec_sha256_host(None, 1, 128, hexo.ctypes.data, 0, None, 1) == -1
    assert lib.cec_sha256_host(None, 0, 128, None, 0, None, 1) == 0
    assert lib.cec_host_sha_set_form(99) == -1
    assert lib.cec_host_sha_probe(99, 1 << 16, 1) < 0
    assert lib.cec_host_sha_probe(0, 1 << 12, 1) > 0


def test_concurrent_jobs_share_the_lanes(lib):
    """Jobs of different lengths (with and without prefix digests) submitted at once from several
    threads: the pool's workers mix their chains in one register's lanes and refill a lane as its
    chain ends; every digest still equals hashlib's."""
    import concurrent.futures as cf
    rng = np.random.default_rng(11)
    jobs = []
    for j, (n, length, prefix) in enumerate([(37, 64 * 300, 64 * 100), (5, 64 * 1000 + 7, 0),
                                             (23, 64 * 50, 64 * 50), (64, 119, 0),
                                             (16, 64 * 777, 64), (3, 0, 0)]):
        bufs = [rng.integers(0, 256, length, dtype=np.uint8).tobytes() for _ in range(n)]
        jobs.append((bufs, length, prefix))

    def run(job):
        bufs, length, prefix = job
        got, pre = host_hex(lib, bufs, length, prefix, threads=8)
        ok = got == [hashlib.sha256(b).hexdigest() for b in bufs]
        if prefix:
            ok = ok and pre == [hashlib.sha256(b[:prefix]).hexdigest() for b in bufs]
        return ok

    for name in forms(lib):
        lib.cec_host_sha_set_form(FORMS[name])
        try:
            with cf.ThreadPoolExecutor(len(jobs)) as ex:
                for _ in range(3):
                    assert all(ex.map(run, jobs)), name
        finally:
            lib.cec_host_sha_set_form(-1)


def test_greedy_lanes_then_tail_spill(lib):
    """More chains than 11 per worker: workers fill all 16 lanes; the job's last chains, taken
    by a few workers, are given back to the idle ones mid-chain (the spill) and finish there.
    Every digest (and every prefix digest) still equals hashlib's."""
    rng = np.random.default_rng(3)
    n, length, prefix = 200, 64 * 2000 + 5, 64 * 700
    base = rng.integers(0, 256, length + n, dtype=np.uint8).tobytes()
    bufs = [base[i:i + length] for i in range(n)]
    if "x16" in forms(lib):
        lib.cec_host_sha_set_form(FORMS["x16"])
    try:
        for _ in range(2):
            got, pre = host_hex(lib, bufs, length, prefix, threads=16)
            assert got == [hashlib.sha256(b).hexdigest() for b in bufs]
            assert pre == [hashlib.sha256(b[:prefix]).hexdigest() for b in bufs]
    finally:
        lib.cec_host_sha_set_form(-1)


def test_python_wrapper_prefix():
    """cess_amd.sha256_hex_host with prefix_len: (hexes, prefix hexes), as SegmentEncoder uses it
    for the segment chains (data fragment 0's digest on the way)."""
    from cess_amd.reedsolomon import sha256_hex_host
    rng = np.random.default_rng(4)
    F = 64 * 50
    segs = [rng.integers(0, 256, 2 * F, dtype=np.uint8) for _ in range(9)]
    hexes, pre = sha256_hex_host(segs, 2 * F, 4, F)
    assert hexes == [hashlib.sha256(s).hexdigest().encode() for s in segs]
    assert pre == [hashlib.sha256(s[:F]).hexdigest().encode() for s in segs]
    assert sha256_hex_host([], 10, 1, 64) == ([], [])
    assert sha256_hex_host(segs[:2], 2 * F, 1) == hexes[:2]


_K = [int(x, 16) for x in (
    "428a2f98 71374491 b5c0fbcf e9b5dba5 3956c25b 59f111f1 923f82a4 ab1c5ed5 d807aa98 12835b01 "
    "243185be 550c7dc3 72be5d74 80deb1fe 9bdc06a7 c19bf174 e49b69c1 efbe4786 0fc19dc6 240ca1cc "
    "2de92c6f 4a7484aa 5cb0a9dc 76f988da 983e5152 a831c66d b00327c8 bf597fc7 c6e00bf3 d5a79147 "
    "06ca6351 14292967 27b70a85 2e1b2138 4d2c6dfc 53380d13 650a7354 766a0abb 81c2c92e 92722c85 "
    "a2bfe8a1 a81a664b c24b8b70 c76c51a3 d192e819 d6990624 f40e3585 106aa070 19a4c116 1e376c08 "
    "2748774c 34b0bcb5 391c0cb3 4ed8aa4a 5b9cca4f 682e6ff3 748f82ee 78a5636f 84c87814 8cc70208 "
    "90befffa a4506ceb bef9a3f7 c67178f2").split()]


def _compress(h, block):
    """One FIPS 180-4 compression (test checker for the states the host hasher hands out)."""
    ror = lambda x, n: ((x >> n) | (x << (32 - n))) & 0xFFFFFFFF  # noqa: E731
    w = [int.from_bytes(block[4 * t:4 * t + 4], "big") for t in range(16)]
    for t in range(16, 64):
        s0 = ror(w[t - 15], 7) ^ ror(w[t - 15], 18) ^ (w[t - 15] >> 3)
        s1 = ror(w[t - 2], 17) ^ ror(w[t - 2], 19) ^ (w[t - 2] >> 10)
        w.append((w[t - 16] + s0 + w[t - 7] + s1) & 0xFFFFFFFF)
    a, b, c, d, e, f, g, hh = h
    for t in range(64):
        t1 = (hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + _K[t] + w[t])
        t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c))
        hh, g, f, e, d, c, b, a = g, f, e, (d + t1) & 0xFFFFFFFF, c, b, a, (t1 + t2) & 0xFFFFFFFF
    return [(x + y) & 0xFFFFFFFF for x, y in zip(h, [a, b, c, d, e, f, g, hh])]


def test_state_after_full_blocks(lib):
    """cec_sha256_host_state: each chain's hex and its state after len bytes (len a multiple of
    64), in every form and lane position: the state equals a restatement's compression chain, and
    its hex equals hashlib's."""
    iv = [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab,
          0x5be0cd19]
    rng = np.random.default_rng(12)
    length = 64 * 5
    bufs = [rng.integers(0, 256, length, dtype=np.uint8) for _ in range(19)]
    want_state = []
    for b in bufs:
        h = list(iv)
        for o in range(0, length, 64):
            h = _compress(h, b[o:o + 64].tobytes())
        want_state.append(h)
    ptrs = (ctypes.c_void_p * len(bufs))(*[b.ctypes.data for b in bufs])
    for name in forms(lib):
        lib.cec_host_sha_set_form(FORMS[name])
        try:
            for threads in (1, 4):
                hexo = np.zeros(64 * len(bufs), np.uint8)
                st = np.zeros(8 * len(bufs), np.uint32)
                assert lib.cec_sha256_host_state(ptrs, len(bufs), length, hexo.ctypes.data,
                                                 st.ctypes.data, threads) == 0
                assert [list(st[8 * i:8 * i + 8]) for i in range(len(bufs))] == want_state, name
                assert [bytes(hexo[64 * i:64 * i + 64]).decode() for i in range(len(bufs))] == \
                    [hashlib.sha256(b).hexdigest() for b in bufs]
        finally:
            lib.cec_host_sha_set_form(-1)
    assert lib.cec_sha256_host_state(ptrs, 1, 65, hexo.ctypes.data, st.ctypes.data, 1) == -1
