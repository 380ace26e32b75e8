"""Multi-process (gloo, world_size 2 and 3) tests of the sharding and the degraded-read gather.

The gather moves survivors between ranks exactly as on GPUs (RCCL on MI355X); on CPU the decode
step is checked with the oracle (the product decode needs a GPU and is covered by
tests/test_gpu_parity.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cess_amd import distributed as D


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_partitions():
    for nseg in (0, 1, 7, 64, 4096):
        for world in (1, 2, 3, 8):
            rs = [D.shard_range(nseg, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == nseg
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            sizes = [b - a for a, b in rs]
            assert max(sizes) - min(sizes) <= 1


def test_plan_gather_counts():
    k, m, G, F = 2, 1, 8, 1 << 20
    lost = {s: [s % 3] for s in range(64)}
    plan = D.plan_gather(lost, k, m, G, F)
    assert sum(len(v) for v in plan.segments.values()) == 64
    # every segment reads exactly k survivors, all from other GPUs when G >= n
    assert len(plan.moves) == 64 * k
    assert plan.bytes_moved == 64 * k * F
    with pytest.raises(ValueError):
        D.plan_gather({0: [0, 1]}, k, m, G, F)
    with pytest.raises(ValueError):
        D.plan_gather({0: [3]}, k, m, G, F)  # index outside 0..k+m-1
    # a segment with nothing lost is skipped (no decoder, no moves)
    p2 = D.plan_gather({0: [], 1: [2]}, k, m, G, F)
    assert list(p2.lost) == [1] and len(p2.moves) == k


def _worker(rank, world, port, k, m, nseg, F, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import rs_oracle as o
    rs = o.ReedSolomon(k, m)
    n = k + m
    rng = np.random.default_rng(42)  # same on every rank: full codewords known to all
    full = []
    for s in range(nseg):
        data = [rng.integers(0, 256, F, dtype=np.uint8) for _ in range(k)]
        full.append(data + rs.encode(data))
    mine = D.local_fragments(nseg, n, world, rank)
    store = D.FragmentStore({sf: i for i, sf in enumerate(mine)},
                            torch.from_numpy(np.stack([full[s][f] for s, f in mine])))
    lost = {s: sorted(rng.choice(n, size=1 + (s % m), replace=False).tolist())
            for s in range(nseg)}
    plan = D.plan_gather(lost, k, m, world, F, exchange="survivors")
    sd, sp, present, segs = D.gather_survivors(plan, store, k, m, rank)
    ok = True
    for i, s in enumerate(segs):
        shards = []
        for f in range(n):
            got = (sd[i, f] if f < k else sp[i, f - k]).numpy()
            if f in plan.survivors[s]:
                ok &= np.array_equal(got, full[s][f])
                shards.append(got.copy())
            else:
                ok &= bool(present[i][f]) == (f not in lost[s])  # decoder flags: all but lost
                shards.append(None)  # lost, or an unused survivor (uninitialised staging)
        rec = rs.reconstruct(shards)
        ok &= all(np.array_equal(rec[f], full[s][f]) for f in lost[s])
    q.put((rank, ok, len(segs)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,k,m", [(2, 2, 1), (3, 2, 1), (2, 4, 2)])
def test_degraded_gather_gloo(world, k, m):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    nseg, F = 9, 4096
    procs = [ctx.Process(target=_worker, args=(r, world, port, k, m, nseg, F, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res), res
    assert sum(n for _, _, n in res) == nseg


def test_plan_exchange_choice():
    """Partial-product exchange: 'auto' takes partials only where they move fewer
    bytes; RS(32,32) on 8 GPUs with one lost fragment: 7 partials instead of 27-28 survivors."""
    k, m, G, F = 32, 32, 8, 512 * 1024
    lost = {s: [s % 64] for s in range(16)}
    surv = D.plan_gather(lost, k, m, G, F, exchange="survivors")
    auto = D.plan_gather(lost, k, m, G, F)  # the default
    assert not surv.partial and set(auto.partial) == set(lost) and not auto.moves
    assert all(len(h) == G - 1 for h in auto.partial.values())
    assert auto.bytes_moved == 16 * (G - 1) * F
    # 27-28 of the 32 survivors (the codec's choice, cec_survivors) live off the decoder
    want = sum(sum((s + f) % G != (2 * s) % G  # decoder: the lost fragment's home
                   for f in D.survivors_of(k, m, [f != s % 64 for f in range(64)]))
               for s in range(16))
    assert surv.bytes_moved == want * F and want >= 16 * 27
    # RS(2,1) spread over >= 3 GPUs: 2 survivors vs 2 partials, a tie -> survivors
    l21 = {s: [s % 3] for s in range(30)}
    assert not D.plan_gather(l21, 2, 1, 8, F, exchange="auto").partial
    # many erasures: partials cost e * holders and lose
    many = {s: list(range(32)) for s in range(4)}
    assert not D.plan_gather(many, k, m, G, F, exchange="auto").partial
    forced = D.plan_gather(many, k, m, G, F, exchange="partials")
    assert forced.bytes_moved == sum(32 * len(h) for h in forced.partial.values()) * F
    with pytest.raises(ValueError):
        D.plan_gather(lost, k, m, G, F, exchange="bogus")


class _OracleEnc:
    """CPU stand-in for the libcessec Encoder in the gloo tests: the oracle does the arithmetic
    (the HIP kernels behind ReconstructBatch / ReconstructPartialBatch / xor_batch are checked
    against the oracle in tests/test_gpu_partial.py); this exercises the exchange itself."""

    def __init__(self, k, m):
        from oracle import rs_oracle as o
        self.o, self.rs = o, o.ReedSolomon(k, m)
        self.DataShards, self.ParityShards = k, m

    def _views(self, sd, sp, i):
        k = self.DataShards
        return [sd[i, f] if f < k else sp[i, f - k] for f in range(k + self.ParityShards)]

    def _survivors(self, present):
        # the codec's survivor choice (cec_survivors): the only shards the product reads
        k, m = self.DataShards, self.ParityShards
        return set(D.survivors_of(k, m, [bool(p) for p in present]))

    def ReconstructBatch(self, sd, sp, nseg, F, present, stream=None):
        for i in range(nseg):
            v = self._views(sd, sp, i)
            surv = self._survivors(present[i])
            rec = self.rs.reconstruct([v[f].numpy().copy() if f in surv else None
                                       for f in range(len(v))])
            for f in range(len(v)):
                if not present[i][f]:
                    v[f].copy_(torch.from_numpy(rec[f]))

    def ReconstructPartialBatch(self, sd, sp, nseg, F, present, held, stream=None):
        for i in range(nseg):
            v = self._views(sd, sp, i)
            sv = self._survivors(present[i])
            surv, outs, rows = self.rs.decode_plan([f in sv for f in range(len(v))])
            cols = [j for j, f in enumerate(surv) if held[i][f]]
            vals = (self.o.code_rows([[r[j] for j in cols] for r in rows],
                                     [v[surv[j]].numpy() for j in cols])
                    if cols else [np.zeros(F, np.uint8) for _ in outs])
            for o_, val in zip(outs, vals):
                if not present[i][o_]:
                    v[o_].copy_(torch.from_numpy(np.asarray(val, np.uint8)))


def _xor_cpu(dst, src, nsrc, stride, length):
    rows = torch.as_strided(src, (nsrc, length), (stride, 1), src.storage_offset())
    d = dst.view(-1)[:length]
    for j in range(nsrc):
        d ^= rows[j]


def _exchange_worker(rank, world, port, k, m, nseg, F, exchange, q, group_transfers=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if group_transfers:
        D.GROUP_TRANSFERS = group_transfers
    from oracle import rs_oracle as o
    rs = o.ReedSolomon(k, m)
    n = k + m
    rng = np.random.default_rng(11)
    full = []
    for s in range(nseg):
        data = [rng.integers(0, 256, F, dtype=np.uint8) for _ in range(k)]
        full.append(data + rs.encode(data))
    mine = D.local_fragments(nseg, n, world, rank)
    store = D.FragmentStore({sf: i for i, sf in enumerate(mine)},
                            torch.from_numpy(np.stack([full[s][f] for s, f in mine])))
    lost = {s: sorted(rng.choice(n, size=1 + (s % m), replace=False).tolist())
            for s in range(nseg)}
    plan = D.plan_gather(lost, k, m, world, F, exchange=exchange)
    out = D.degraded_read(plan, store, _OracleEnc(k, m), rank, xor=_xor_cpu)
    ok = all(np.array_equal(t.numpy(), full[s][f]) for (s, f), t in out.items())
    q.put((rank, ok, len(out), len(plan.partial)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,k,m,exchange", [(2, 2, 1, "partials"), (3, 4, 2, "auto"),
                                                (3, 4, 2, "partials"), (2, 4, 2, "partials"),
                                                (3, 10, 4, "auto")])
def test_degraded_read_partials_gloo(world, k, m, exchange):
    """degraded_read with the partial-product exchange at world 2/3 (gloo): every lost fragment
    comes back equal to the oracle's codeword; 'auto' mixes both exchanges in one call."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    nseg, F = 9, 2048
    procs = [ctx.Process(target=_exchange_worker,
                         args=(r, world, port, k, m, nseg, F, exchange, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _, _ in res), res
    assert sum(n for _, _, n, _ in res) == sum(1 + (s % m) for s in range(nseg))
    assert all(npart > 0 for _, _, _, npart in res)


@pytest.mark.parametrize("world,k,m,exchange,gt", [(2, 2, 1, "survivors", 1),
                                                   (3, 4, 2, "auto", 2),
                                                   (3, 10, 4, "partials", 3),
                                                   (3, 4, 2, "survivors", 5)])
def test_degraded_read_small_batches_gloo(world, k, m, exchange, gt):
    """The torch path with its transfers cut into many grouped batches (GROUP_TRANSFERS, the
    same cuts on every rank): every lost fragment still comes back equal to the oracle's."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    nseg, F = 11, 1024
    procs = [ctx.Process(target=_exchange_worker,
                         args=(r, world, port, k, m, nseg, F, exchange, q, gt))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _, _ in res), res
    assert sum(n for _, _, n, _ in res) == sum(1 + (s % m) for s in range(nseg))


@pytest.mark.parametrize("k,m", [(2, 1), (4, 2), (10, 4), (32, 32)])
def test_c_plan_matches_python_plan(k, m):
    """cec_dist_plan (the plan libcessec's RCCL degraded read runs, cec_dist_degraded_read) equals
    plan_gather's for random lost maps (duplicates, up to m erasures, unsorted) at worlds 1..8."""
    from cess_amd.reedsolomon import CecError, ErrTooFewShards
    rng = np.random.default_rng(k * 100 + m)
    n = k + m
    for world in range(1, 9):
        lost = {}
        for s in rng.choice(1000, size=40, replace=False).tolist():
            e = rng.choice(n, size=int(rng.integers(1, m + 1)), replace=False).tolist()
            lost[s] = e + e[:1]  # a duplicate entry
        moves, dec = D.c_plan(lost, k, m, world, "survivors")
        plan = D.plan_gather(lost, k, m, world, 1, exchange="survivors")
        assert {(s, f): (src, dst) for s, f, src, dst, _ in moves} == plan.moves
        assert [(s, f) for s, f, _, _, _ in moves] == sorted(plan.moves)  # the issue order
        assert all(kind == 0 for *_, kind in moves)
        for (s, f), r in dec.items():
            assert s in plan.segments[r]
        for ex in ("partials", "auto"):  # the partial-product exchange
            moves, dec = D.c_plan(lost, k, m, world, ex)
            plan = D.plan_gather(lost, k, m, world, 1, exchange=ex)
            assert {(s, f): (src, dst) for s, f, src, dst, kind in moves if kind == 0} \
                == plan.moves
            want = {(s, f, h, plan.decoder[s]) for s, hs in plan.partial.items()
                    for h in hs for f in plan.lost[s]}
            assert {(s, f, src, dst) for s, f, src, dst, kind in moves if kind == 1} == want
            assert all(plan.decoder[s] == r for (s, _), r in dec.items())
    with pytest.raises(CecError):
        D.c_plan({3: [n]}, k, m, 2)  # index outside 0..n-1
    with pytest.raises(ErrTooFewShards):
        D.c_plan({3: list(range(m + 1))}, k, m, 2)


def test_survivor_choice():
    """cec_survivors: k present shards; klauspost's first k present for every code but
    RS(32,32), whose rebuilds read every present shard of the coset with fewer losses plus as
    many of the other coset as that lost, packed into whole lane-pair slots (2j, 2j + 1) where
    the pattern allows (the syndrome-row decoder's rows then fill the fewest slots)."""
    rng = np.random.default_rng(3)
    for k, m in ((2, 1), (4, 2), (10, 4), (17, 3)):
        for _ in range(20):
            pres = np.ones(k + m, bool)
            pres[rng.choice(k + m, size=int(rng.integers(0, m + 1)), replace=False)] = False
            assert D.survivors_of(k, m, pres) == [f for f in range(k + m) if pres[f]][:k]
    for e in range(0, 33):
        for _ in range(10):
            pres = np.ones(64, bool)
            pres[rng.choice(64, size=e, replace=False)] = False
            sv = D.survivors_of(32, 32, pres)
            assert len(sv) == 32 == len(set(sv)) and all(pres[f] for f in sv)
            nd, np_ = (~pres[:32]).sum(), (~pres[32:]).sum()
            a, b = (range(32, 64), range(32)) if np_ < nd else (range(32), range(32, 64))
            assert all(f in sv for f in a if pres[f])  # all of coset A that survived
            rb = [f - b[0] for f in sv if f in b]
            assert len(rb) == 32 - sum(pres[f] for f in a)
            # whole present slots are used before split ones
            whole = sum(1 for j in range(16) if pres[b[0] + 2 * j] and pres[b[0] + 2 * j + 1])
            used_whole = sum(1 for j in range(16) if 2 * j in rb and 2 * j + 1 in rb)
            assert used_whole == min(whole, len(rb) // 2)
    import cess_amd
    with pytest.raises(cess_amd.CecError):
        D.survivors_of(4, 2, [True, True, True, False, False, False])


@pytest.mark.parametrize("k,m,world,exchange,bound", [(2, 1, 8, "survivors", 64),
                                                      (32, 32, 8, "survivors", 1024),
                                                      (32, 32, 3, "partials", 200),
                                                      (10, 4, 2, "auto", 7),
                                                      (4, 2, 4, "auto", 1),
                                                      (32, 32, 8, "auto", 0)])
def test_c_plan_groups(k, m, world, exchange, bound):
    """cec_dist_plan_groups (the group cuts libcessec's degraded read issues, CEC_DIST_OPT_GROUP_OPS)
    equals a restatement from the plan's moves: per round of 256 segments, a new group before a
    segment whose transfers would take any rank past the bound; rounds always start a group; no
    group holds more than the bound on any rank unless one segment alone does."""
    rng = np.random.default_rng(k * 7 + world)
    n = k + m
    lost = {}
    for s in sorted(rng.choice(5000, size=700, replace=False).tolist()):
        lost[s] = rng.choice(n, size=int(rng.integers(1, m + 1)), replace=False).tolist()
    moves, _ = D.c_plan(lost, k, m, world, exchange)
    order = sorted(lost)
    pos = {s: i for i, s in enumerate(order)}
    per_seg = [[0] * world for _ in order]
    for s, f, src, dst, kind in moves:
        if src != dst:
            per_seg[pos[s]][src] += 1
            per_seg[pos[s]][dst] += 1
    want = []
    for r0 in range(0, len(order), 256):
        want.append(r0)
        cnt = [0] * world
        for i in range(r0, min(len(order), r0 + 256)):
            if bound and i > want[-1] and any(c + o > bound for c, o in zip(cnt, per_seg[i])):
                want.append(i)
                cnt = [0] * world
            cnt = [c + o for c, o in zip(cnt, per_seg[i])]
    got = D.c_plan_groups(lost, k, m, world, exchange, bound)
    assert got == want
    ends = got[1:] + [len(order)]
    for a, b in zip(got, ends):
        tot = [sum(per_seg[i][w] for i in range(a, b)) for w in range(world)]
        assert not bound or b - a == 1 or max(tot) <= bound
    if bound == 0:
        assert got == list(range(0, len(order), 256))
