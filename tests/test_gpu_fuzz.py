"""Seeded randomized sweep of the batch codec against the C oracle (oracle/rs_oracle.c): random
codes RS(k, m) (k + m <= 256), random shard lengths (odd, unaligned, tiny and large), random
per-segment erasure patterns of 0..m shards with and without data_only. Encode must equal the
oracle's parity byte for byte; every rebuild must restore the erased shards of the oracle's
codeword exactly, and leave every other shard untouched (data_only: parity erasures stay as they
were). The convention is SURVEY.md §8a a11 (GF(2^8) 0x11D, E = V inv(V_top)); klauspost's
Encode / Reconstruct / ReconstructData shape."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a GPU"
    t.cuda.init()
    return t


@pytest.fixture(scope="module")
def cess(torch):
    import cess_amd
    return cess_amd


def _cases(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        k = int(rng.choice([1, 2, 3, 4, 5, 6, 8, 10, 12, 16, 17, 20, 28, 32, 40, 64]))
        m = int(rng.choice([1, 2, 3, 4, 5, 8, 12, 16, 32]))
        if k + m > 256:
            m = 256 - k
        ln = int(rng.choice([1, 3, 15, 16, 63, 64, 100, 1000, 1024, 4095, 4096, 4099, 8192,
                             65536 + 48, 70001]))
        nseg = int(rng.integers(1, 6))
        out.append((k, m, ln, nseg, int(rng.integers(1 << 30))))
    return out


@pytest.mark.parametrize("k,m,ln,nseg,seed", _cases(96, 2026))
def test_random_codes_against_oracle(torch, cess, corc, k, m, ln, nseg, seed):
    from oracle.c_oracle import c_encode
    rng = np.random.default_rng(seed)
    n = k + m
    data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
    want_par = np.stack([np.stack(c_encode(corc, k, m, [data[s, i] for i in range(k)]))
                         for s in range(nseg)])
    enc = cess.New(k, m)
    d_data = torch.from_numpy(data).cuda()
    d_par = torch.zeros((nseg, m, ln), dtype=torch.uint8, device="cuda")
    enc.EncodeBatch(d_data, d_par, nseg, ln)
    torch.cuda.synchronize()
    assert np.array_equal(d_par.cpu().numpy(), want_par)
    for data_only in (False, True):
        present = np.ones((nseg, n), np.uint8)
        for s in range(nseg):
            present[s, rng.choice(n, size=int(rng.integers(0, m + 1)), replace=False)] = 0
        dd, dp = d_data.clone(), d_par.clone()
        junk = torch.from_numpy(rng.integers(0, 256, (nseg, n, ln), dtype=np.uint8)).cuda()
        for s in range(nseg):  # erased shards hold junk, not zeros
            for f in range(n):
                if not present[s, f]:
                    (dd[s, f] if f < k else dp[s, f - k]).copy_(junk[s, f])
        enc.ReconstructBatch(dd, dp, nseg, ln, present, data_only=data_only)
        torch.cuda.synchronize()
        got_d, got_p = dd.cpu().numpy(), dp.cpu().numpy()
        junk_h = junk.cpu().numpy()
        for s in range(nseg):
            assert np.array_equal(got_d[s], data[s]), (s, data_only)
            for j in range(m):
                if present[s, k + j] or not data_only:
                    assert np.array_equal(got_p[s, j], want_par[s, j]), (s, j, data_only)
                else:  # data_only leaves an erased parity shard as it was
                    assert np.array_equal(got_p[s, j], junk_h[s, k + j]), (s, j)
    enc.close()


def test_graph_capture_of_compile_time_calls(torch, cess, corc):
    """The capturable calls (include/cess_ec.h: RS(2,1) and RS(32,32) encodes, RS(2,1) rebuilds
    of one pattern) replayed from one HIP graph read the buffers at replay time: new data written
    between replays comes out with the C oracle's parity, and every erased fragment rebuilt."""
    from oracle.c_oracle import c_encode
    for k, m, ln, nseg in ((2, 1, (1 << 16) + 48, 3), (32, 32, 4096, 2)):
        enc = cess.New(k, m)
        d_data = torch.empty((nseg, k, ln), dtype=torch.uint8, device="cuda")
        d_par = torch.empty((nseg, m, ln), dtype=torch.uint8, device="cuda")
        side = torch.cuda.Stream()
        pats = ([np.array([int(i != e) for i in range(k + m)], np.uint8) for e in range(k + m)]
                if k == 2 else [])

        def step(st):
            enc.EncodeBatch(d_data, d_par, nseg, ln, stream=st)
            for p in pats:
                enc.ReconstructBatch(d_data, d_par, nseg, ln, p, stream=st)
        cess.fill_synthetic(d_data, k * ln, nseg, 0, 77)
        torch.cuda.synchronize()
        with torch.cuda.stream(side):
            step(side)  # the uncaptured call of the same shape
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            step(torch.cuda.current_stream())
        for seed in (5, 6):
            cess.fill_synthetic(d_data, k * ln, nseg, 0, seed)
            d_par.zero_()
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            data, par = d_data.cpu().numpy(), d_par.cpu().numpy()
            for s in range(nseg):
                want = np.stack(c_encode(corc, k, m, [data[s, i] for i in range(k)]))
                assert np.array_equal(par[s], want), (k, m, seed, s)
        enc.close()
