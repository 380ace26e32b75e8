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
    plan = D.plan_gather(lost, k, m, world, F)
    sd, sp, present, segs = D.gather_survivors(plan, store, k, m, rank)
    ok = True
    for i, s in enumerate(segs):
        shards = []
        for f in range(n):
            got = (sd[i, f] if f < k else sp[i, f - k]).numpy()
            if present[i][f]:
                ok &= np.array_equal(got, full[s][f])
                shards.append(got.copy())
            else:
                shards.append(None)  # unused slot (uninitialised staging)
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
        moves, dec = D.c_plan(lost, k, m, world)
        plan = D.plan_gather(lost, k, m, world, 1)
        assert {(s, f): (src, dst) for s, f, src, dst in moves} == plan.moves
        assert [(s, f) for s, f, _, _ in moves] == sorted(plan.moves)  # the issue order
        for (s, f), r in dec.items():
            assert s in plan.segments[r]
    with pytest.raises(CecError):
        D.c_plan({3: [n]}, k, m, 2)  # index outside 0..n-1
    with pytest.raises(ErrTooFewShards):
        D.c_plan({3: list(range(m + 1))}, k, m, 2)
