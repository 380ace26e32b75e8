"""Partial rebuilds (cec_reconstruct_partial_batch) and the GF(2^8) combine (cec_xor_batch): the
partial-product exchange of a multi-GPU degraded read (each GPU multiplies the
survivors it holds by their decode coefficients, the partials travel to the decoder and are
XOR-ed there). The XOR of the partials over a partition of every segment's survivors must equal
the C oracle's codeword, bit-exact; survivors a part does not hold are filled with garbage to show
they are never read."""
import numpy as np
import pytest

from oracle.c_oracle import c_encode

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a GPU"
    return t


@pytest.fixture(scope="module")
def cess(torch):
    import cess_amd
    return cess_amd


def _codewords(corc, k, m, ln, nseg, rng):
    data = rng.integers(0, 256, (nseg, k, ln), dtype=np.uint8)
    par = np.stack([np.stack(c_encode(corc, k, m, list(data[s]))) for s in range(nseg)])
    return np.concatenate([data, par], axis=1)  # [nseg][n][ln]


def _erasures(k, m, nseg, rng):
    n = k + m
    present = np.ones((nseg, n), np.uint8)
    for s in range(nseg):
        present[s, rng.choice(n, size=int(rng.integers(1, m + 1)), replace=False)] = 0
    return present


def _partials(torch, cess, enc, full, present, held, rng, data_only=False):
    """Run one partial rebuild per part on its own batch; returns the parts' batches
    [P][nseg][n][ln] on the device (one contiguous buffer, data then parity per part)."""
    nseg, n, ln = full.shape
    k = enc.DataShards
    P = held.shape[0]
    bufs = torch.empty((P, nseg * n * ln), dtype=torch.uint8, device="cuda")
    for r in range(P):
        # held survivors hold their bytes; every other slot holds garbage
        b = rng.integers(0, 256, full.shape, dtype=np.uint8)
        b[held[r].astype(bool)] = full[held[r].astype(bool)]
        host = np.concatenate([b[:, :k].reshape(-1), b[:, k:].reshape(-1)])
        bufs[r].copy_(torch.from_numpy(host))
        enc.ReconstructPartialBatch(bufs[r, :nseg * k * ln], bufs[r, nseg * k * ln:], nseg, ln,
                                    present, held[r], data_only=data_only)
    return bufs


def _as_batch(buf, nseg, k, m, ln):
    h = buf.cpu().numpy()
    return np.concatenate([h[:nseg * k * ln].reshape(nseg, k, ln),
                           h[nseg * k * ln:].reshape(nseg, m, ln)], axis=1)


@pytest.mark.parametrize("k,m,ln,nseg,P", [(2, 1, 4096, 9, 2), (4, 2, 1000, 7, 3),
                                           (10, 4, 4099, 6, 4), (32, 32, 4096, 5, 8),
                                           (32, 32, (1 << 16) + 16, 4, 8), (2, 1, 1, 3, 3)])
@pytest.mark.parametrize("rt_mode", [0, 1, 3])
def test_partials_xor_to_codeword(torch, cess, corc, k, m, ln, nseg, P, rt_mode):
    """Fragment f of segment s held by part (s + f) mod P (the multi-GPU placement); XOR of the
    P partials = every lost fragment; data_only rebuilds the lost data fragments only."""
    rng = np.random.default_rng(k * 7919 + ln * 31 + P)
    n = k + m
    full = _codewords(corc, k, m, ln, nseg, rng)
    present = _erasures(k, m, nseg, rng)
    held = np.zeros((P, nseg, n), np.uint8)
    for s in range(nseg):
        for f in range(n):
            held[(s + f) % P, s, f] = present[s, f]
    enc = cess.New(k, m)
    enc.set_option(4, rt_mode)
    for data_only in (False, True):
        bufs = _partials(torch, cess, enc, full, present, held, rng, data_only)
        cess.xor_batch(bufs[0], bufs[1], P - 1, bufs.shape[1], bufs.shape[1])
        torch.cuda.synchronize()
        got = _as_batch(bufs[0], nseg, k, m, ln)
        for s in range(nseg):
            for f in range(n):
                if not present[s, f] and (f < k or not data_only):
                    assert np.array_equal(got[s, f], full[s, f]), (s, f, data_only)


def test_partial_edges(torch, cess, corc):
    """A part holding every survivor = the full rebuild; a part holding none = zeros; a repeated
    call reuses the cached plan; nothing lost = nothing written."""
    k, m, ln, nseg = 4, 2, 2048, 5
    rng = np.random.default_rng(3)
    n = k + m
    full = _codewords(corc, k, m, ln, nseg, rng)
    present = _erasures(k, m, nseg, rng)
    enc = cess.New(k, m)
    for _ in range(2):
        b = _as_batch(_partials(torch, cess, enc, full, present, present[None], rng)[0],
                      nseg, k, m, ln)
        assert np.array_equal(b, full)  # present slots were copied, lost ones rebuilt
    none = np.zeros((1, nseg, n), np.uint8)
    b = _as_batch(_partials(torch, cess, enc, full, present, none, rng)[0], nseg, k, m, ln)
    for s in range(nseg):
        for f in range(n):
            if not present[s, f]:
                assert not b[s, f].any()
    allp = np.ones((nseg, n), np.uint8)
    bufs = _partials(torch, cess, enc, full, allp, allp[None], rng)
    assert np.array_equal(_as_batch(bufs[0], nseg, k, m, ln), full)
    with pytest.raises(ValueError):
        enc.ReconstructPartialBatch(bufs[0], bufs[0], nseg, ln, present, present[:1])
    with pytest.raises(cess.ErrTooFewShards):
        few = present.copy()
        few[0, :m + 1] = 0
        enc.ReconstructPartialBatch(bufs[0, :nseg * k * ln], bufs[0, nseg * k * ln:], nseg, ln,
                                    few, few)


@pytest.mark.parametrize("ln", [0, 1, 15, 4096, (1 << 20) + 3])
@pytest.mark.parametrize("nsrc", [0, 1, 2, 7])
def test_xor_batch(torch, cess, ln, nsrc):
    rng = np.random.default_rng(ln + nsrc)
    stride = ln + (16 if ln % 16 == 0 else 5)
    dst = rng.integers(0, 256, max(ln, 1), dtype=np.uint8)
    src = rng.integers(0, 256, max(nsrc * stride, 1), dtype=np.uint8)
    want = dst.copy()
    for j in range(nsrc):
        want[:ln] ^= src[j * stride:j * stride + ln]
    d_dst, d_src = torch.from_numpy(dst).cuda(), torch.from_numpy(src).cuda()
    cess.xor_batch(d_dst, d_src, nsrc, stride, ln)
    torch.cuda.synchronize()
    assert np.array_equal(d_dst.cpu().numpy(), want)
    if nsrc > 1 and ln > 1:
        with pytest.raises(cess.CecError):
            cess.xor_batch(d_dst, d_src, nsrc, ln - 1, ln)  # overlapping sources
