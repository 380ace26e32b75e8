"""GPU hash queue (cec_hashq_*): streaming SHA-256 with chain state in HBM, against hashlib and
the reference's own NIST SHAVS vectors (utils/ring/third_party/NIST/SHAVS, copied as data into
tests/golden/), through ticks of every size, interleaved adds, unaligned buffers and the
segment/fragment layouts of SegmentList (c-pallets/file-bank/src/types.rs:13-16)."""
import hashlib

import numpy as np
import pytest

from tests.conftest import parse_shavs

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


@pytest.fixture(params=[1, 2, 3, 4], ids=["tick2w", "tick2w_pf2", "tick1w", "tick_lanepair"])
def tick_variant(cess, request):
    """Every test below runs on each tick kernel (CEC_HQOPT_TICK, set per queue by mkq)."""
    return request.param


def mkq(cess, tick, **kw):
    q = cess.HashQueue(**kw)
    q.set_option(1, tick)
    return q


def hexes(t):
    return [bytes(r).decode() for r in t.cpu().numpy().reshape(-1, 64)]


def test_shavs_through_queue(torch, cess, tick_variant):
    """Every NIST short/long message as its own chain at an odd device offset, ticked a few
    blocks at a time while more messages are added."""
    vecs = parse_shavs("SHA256ShortMsg.rsp") + parse_shavs("SHA256LongMsg.rsp")
    offs, pos = [], 0
    for msg, _ in vecs:
        offs.append(pos + 3)  # 3: every buffer start unaligned
        pos += len(msg) + 3
    buf = np.zeros(pos + 64, np.uint8)
    for (msg, _), o in zip(vecs, offs):
        buf[o:o + len(msg)] = np.frombuffer(msg, np.uint8)
    d = torch.from_numpy(buf).cuda()
    d_hex = torch.zeros((len(vecs), 64), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    with mkq(cess, tick_variant, capacity=1024, stream=st) as q:
        tickets = []
        for i, ((msg, _), o) in enumerate(zip(vecs, offs)):
            tickets.append(q.add(d.data_ptr() + o, 1, 1, 0, 0, len(msg), d_hex, 1, i * 64))
            if i % 7 == 0:
                q.tick(2)
        q.finish()
        assert all(q.done(t) for t in tickets) and q.live_chains == 0
        torch.cuda.synchronize()
    got = hexes(d_hex)
    for (msg, md), g in zip(vecs, got):
        assert g == md, (len(msg), g, md)


@pytest.mark.parametrize("k,m,F", [(2, 1, 65536), (4, 2, 4160), (32, 32, 1000), (2, 1, 56)])
@pytest.mark.parametrize("max_blocks", [1, 37, 0])
@pytest.mark.parametrize("combined", [False, True], ids=["separate", "prefix"])
def test_batch_window(torch, cess, k, m, F, max_blocks, combined, tick_variant):
    """Fragments + segment hashes of several batches added one per step, one tick per step
    (a window of batches in flight), then drained: every hex matches hashlib. "prefix": one
    add_segment_lists per batch, fragment 0's hash from the segment chain's prefix digest
    (F % 64 == 0; F = 1000 and 56 take the separate-chain fallback)."""
    nseg, nbatch = 5, 4
    rng = np.random.default_rng(k * 1000 + F + max_blocks)
    data = rng.integers(0, 256, (nbatch, nseg, k, F), dtype=np.uint8)
    par = rng.integers(0, 256, (nbatch, nseg, m, F), dtype=np.uint8)
    d_data, d_par = torch.from_numpy(data).cuda(), torch.from_numpy(par).cuda()
    d_fhex = torch.zeros((nbatch, nseg, k + m, 64), dtype=torch.uint8, device="cuda")
    d_shex = torch.zeros((nbatch, nseg, 64), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    q = mkq(cess, tick_variant, capacity=2048, stream=st)
    tickets = []
    for b in range(nbatch):
        if combined:
            t1 = t2 = q.add_segment_lists(d_data[b], d_par[b], nseg, k, m, F, d_shex[b],
                                          d_fhex[b])
        else:
            t1 = q.add_fragments(d_data[b], d_par[b], nseg, k, m, F, d_fhex[b])
            t2 = q.add_segments(d_data[b], nseg, k * F, d_shex[b])
        tickets.append((t1, t2))
        q.tick(max_blocks)
        if max_blocks == 0:
            assert q.done(t1) and q.done(t2)
    need = cess.sha256_blocks(k * F)
    if max_blocks and need > max_blocks * nbatch:
        assert not q.done(tickets[0][1])
    q.finish()
    torch.cuda.synchronize()
    assert q.live_chains == 0 and all(q.done(t) for tt in tickets for t in tt)
    q.close()
    fh = np.array(hexes(d_fhex)).reshape(nbatch, nseg, k + m)
    sh = np.array(hexes(d_shex)).reshape(nbatch, nseg)
    for b in range(nbatch):
        for s in range(nseg):
            assert sh[b, s] == hashlib.sha256(data[b, s].tobytes()).hexdigest()
            for i in range(k + m):
                frag = data[b, s, i] if i < k else par[b, s, i - k]
                assert fh[b, s, i] == hashlib.sha256(frag.tobytes()).hexdigest(), (b, s, i)


@pytest.mark.parametrize("max_blocks", [1, 5, 0])
def test_prefix_digest(torch, cess, max_blocks, tick_variant):
    """cec_hashq_add_prefix: chains of different lengths whose prefix ends at the first
    block, mid-chain, at the last whole block and at the full (64-multiple) length; ticks of
    1, 5 and all blocks put the prefix boundary inside, at the start and at the end of a tick."""
    cases = [(64 * 9, 64), (64 * 9, 64 * 5), (64 * 9 + 57, 64 * 9), (64 * 12, 64 * 12),
             (64 * 20 + 3, 64 * 10)]
    rng = np.random.default_rng(77 + max_blocks)
    st = torch.cuda.current_stream()
    q = mkq(cess, tick_variant, capacity=64, stream=st)
    bufs, outs = [], []
    for n, (length, plen) in enumerate(cases):
        data = rng.integers(0, 256, (3, length), dtype=np.uint8)
        d = torch.from_numpy(data).cuda()
        hx = torch.zeros((3, 64), dtype=torch.uint8, device="cuda")
        px = torch.zeros((3, 64), dtype=torch.uint8, device="cuda")
        q.add(d, 3, 1, length, length, length, hx, 1, 0, plen, px, 1, 0)
        q.tick(max_blocks)
        bufs.append((data, plen))
        outs.append((hx, px, d))  # d stays alive until the chains are done
    q.finish()
    torch.cuda.synchronize()
    q.close()
    for (data, plen), (hx, px, _) in zip(bufs, outs):
        for i in range(3):
            assert hexes(hx)[i] == hashlib.sha256(data[i].tobytes()).hexdigest()
            assert hexes(px)[i] == hashlib.sha256(data[i, :plen].tobytes()).hexdigest(), plen


def test_prefix_rejects_bad_length(torch, cess):
    d = torch.zeros(1024, dtype=torch.uint8, device="cuda")
    hx = torch.zeros((1, 64), dtype=torch.uint8, device="cuda")
    with cess.HashQueue(capacity=16) as q:
        for plen in (63, 2048):
            with pytest.raises(Exception):
                q.add(d, 1, 1, 0, 0, 1024, hx, 1, 0, plen, hx, 1, 0)


def test_matches_batch_kernel_full_geometry(torch, cess, tick_variant):
    """Config-5 geometry (64 segments of 32 x 512 KiB data + 32 parity): the queue's hexes equal
    the one-shot batch kernel's (k_sha256_2w) and hashlib's for all 4096 fragments."""
    k, m, F, nseg = 32, 32, 512 * 1024, 64
    d_data = torch.empty((nseg, k, F), dtype=torch.uint8, device="cuda")
    d_par = torch.empty((nseg, m, F), dtype=torch.uint8, device="cuda")
    cess.fill_synthetic(d_data, k * F, nseg, 0, 0xCE550005)
    enc = cess.New(k, m)
    enc.EncodeBatch(d_data, d_par, nseg, F)
    a = torch.zeros((nseg, k + m, 64), dtype=torch.uint8, device="cuda")
    b = torch.zeros_like(a)
    enc.Sha256Batch(d_data, d_par, nseg, F, a)
    q = mkq(cess, tick_variant, capacity=1 << 13, stream=torch.cuda.current_stream())
    q.add_fragments(d_data, d_par, nseg, k, m, F, b)
    while q.live_chains:
        q.tick(1000)
    torch.cuda.synchronize()
    q.close()
    assert torch.equal(a, b)
    got = hexes(b)
    frags = np.concatenate([d_data.cpu().numpy(), d_par.cpu().numpy()], axis=1)  # [nseg][64][F]
    import concurrent.futures as cf
    with cf.ThreadPoolExecutor(8) as ex:  # hashlib releases the GIL on large buffers
        want = list(ex.map(lambda j: hashlib.sha256(frags[j // (k + m), j % (k + m)]).hexdigest(),
                           range(nseg * (k + m))))
    assert got == want


def test_edge_cases(torch, cess, tick_variant):
    """Empty chains, lengths around the 55/56/64-byte padding boundaries, a full ring."""
    lens = [0, 1, 55, 56, 57, 63, 64, 65, 119, 120, 128]
    buf = np.arange(256, dtype=np.uint8)
    d = torch.from_numpy(buf).cuda()
    d_hex = torch.zeros((len(lens), 64), dtype=torch.uint8, device="cuda")
    q = mkq(cess, tick_variant, capacity=16, stream=torch.cuda.current_stream())
    for i, ln in enumerate(lens):
        q.add(d, 1, 1, 0, 0, ln, d_hex, 1, i * 64)
    with pytest.raises(cess.CecError):
        q.add(d, 6, 1, 0, 0, 10, None)  # 11 live + 6 > 16
    q.tick(1)
    q.add(d, 5, 1, 1, 1, 10, None)  # 1-block chains completed: room again
    q.finish()
    torch.cuda.synchronize()
    q.close()
    got = hexes(d_hex)
    for ln, g in zip(lens, got):
        assert g == hashlib.sha256(buf[:ln].tobytes()).hexdigest(), ln
