"""Multi-GPU degraded read over RCCL (BASELINE config 4's exchange step): two or more ranks, one
process per GPU, backend "nccl" (= RCCL over xGMI). Survivors of each segment are gathered on the
lost fragment's home GPU (fragment f of segment s on GPU (s + f) mod G,
c-pallets/file-bank/src/functions.rs:187-283) and rebuilt by libcessec; every rebuilt fragment is
compared with the C oracle's. Skips cleanly when fewer than two GPUs are visible (the same path
is covered on CPU by tests/test_distributed.py with gloo)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, k, m, nseg, F, q, exchange="survivors"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch
    import torch.distributed as dist
    import cess_amd
    from cess_amd import distributed as D
    from oracle.c_oracle import c_encode, load_c_oracle
    torch.cuda.set_device(rank)
    dev = torch.device("cuda", rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    dist.barrier()  # a collective over every rank before the grouped point-to-point ops
    corc = load_c_oracle()
    n = k + m
    rng = np.random.default_rng(7)  # same on every rank: every codeword known to all
    full = []
    for s in range(nseg):
        data = [rng.integers(0, 256, F, dtype=np.uint8) for _ in range(k)]
        full.append(data + c_encode(corc, k, m, data))
    mine = D.local_fragments(nseg, n, world, rank)
    store = D.FragmentStore({sf: i for i, sf in enumerate(mine)},
                            torch.from_numpy(np.stack([full[s][f] for s, f in mine])).to(dev))
    lost = {s: sorted(rng.choice(n, size=1 + s % m, replace=False).tolist()) for s in range(nseg)}
    plan = D.plan_gather(lost, k, m, world, F, exchange=exchange)
    out = D.degraded_read(plan, store, cess_amd.New(k, m, device=rank), rank)
    torch.cuda.synchronize(dev)
    ok = all(np.array_equal(t.cpu().numpy(), full[s][f]) for (s, f), t in out.items())
    q.put((rank, ok, len(out), plan.bytes_moved))
    dist.barrier()
    dist.destroy_process_group()


# RS(32,32) at 1 MiB fragments loses 1..12 fragments per segment: from four on, the FFT-domain
# decoders rebuild them from the gathered survivors only (the first k present)
WIDE = [(32, 32, "survivors"), (32, 32, "partials")]


@pytest.mark.parametrize("k,m,exchange", [(2, 1, "survivors"), (4, 2, "survivors"),
                                          (4, 2, "partials"), (10, 4, "auto")] + WIDE)
def test_degraded_read_rccl(k, m, exchange):
    import torch
    import torch.multiprocessing as mp
    world = min(torch.cuda.device_count(), 8)
    if world < 2:
        pytest.skip("RCCL degraded read needs >= 2 visible GPUs")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    nseg, F = 12, 1 << 20
    procs = [ctx.Process(target=_rank, args=(r, world, port, k, m, nseg, F, q, exchange))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _, _ in res), res
    assert sum(n for _, _, n, _ in res) == sum(1 + s % m for s in range(nseg))
    assert res[0][3] > 0  # survivors crossed GPUs


def _gloo_rank(rank, world, port, k, m, nseg, F, exchange, q):
    """One rank of a multi-process degraded read whose ranks share GPU 0 and talk over gloo
    (fragments staged through host memory): the product path of partial_exchange and
    gather_survivors (libcessec partial rebuilds, XOR combine, survivor rebuilds) end to end on
    the one-GPU box; only the transport differs from RCCL."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import cess_amd
    from cess_amd import distributed as D
    dist.init_process_group("gloo", rank=rank, world_size=world)
    full, lost = _codewords(k, m, nseg, F, seed=5)
    n = k + m
    mine = D.local_fragments(nseg, n, world, rank)
    store = D.FragmentStore({sf: i for i, sf in enumerate(mine)},
                            torch.from_numpy(np.stack([full[s][f] for s, f in mine])).cuda())
    plan = D.plan_gather(lost, k, m, world, F, exchange=exchange)
    out = D.degraded_read(plan, store, cess_amd.New(k, m), rank)
    torch.cuda.synchronize()
    ok = all(np.array_equal(t.cpu().numpy(), full[s][f]) for (s, f), t in out.items())
    q.put((rank, ok, len(out), len(plan.partial)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,k,m,exchange,F", [(3, 4, 2, "partials", (1 << 16) + 32),
                                                  (3, 10, 4, "auto", (1 << 16) + 32),
                                                  (2, 32, 32, "auto", (1 << 16) + 32),
                                                  (2, 32, 32, "survivors", 1 << 16),
                                                  (3, 32, 32, "auto", 1 << 16)])
def test_degraded_read_partials_shared_gpu(world, k, m, exchange, F):
    """F a multiple of 1024 with RS(32,32): segments losing 4..10 fragments rebuild through the
    FFT-domain decoders from the k gathered survivors (the staging holds nothing else)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    nseg = 10
    procs = [ctx.Process(target=_gloo_rank, args=(r, world, port, k, m, nseg, F, exchange, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _, _ in res), res
    assert sum(nr for _, _, nr, _ in res) == sum(1 + s % m for s in range(nseg))
    if exchange != "survivors":
        assert all(npart > 0 for *_, npart in res)


def _codewords(k, m, nseg, F, seed=7):
    from oracle.c_oracle import c_encode, load_c_oracle
    corc = load_c_oracle()
    rng = np.random.default_rng(seed)
    full = []
    for s in range(nseg):
        data = [rng.integers(0, 256, F, dtype=np.uint8) for _ in range(k)]
        full.append(data + c_encode(corc, k, m, data))
    lost = {s: sorted(rng.choice(k + m, size=1 + s % m, replace=False).tolist())
            for s in range(nseg)}
    return full, lost


@pytest.mark.parametrize("k,m,nseg,F,exchange", [(2, 1, 12, (1 << 20) + 64, "survivors"),
                                                  (4, 2, 12, (1 << 20) + 64, "survivors"),
                                                  (10, 4, 12, (1 << 20) + 64, "survivors"),
                                                  (2, 1, 600, 65536, "survivors"),
                                                  (10, 4, 12, (1 << 20) + 64, "partials"),
                                                  (4, 2, 600, 4096, "partials"),
                                                  (32, 32, 12, 1 << 16, "survivors"),
                                                  (32, 32, 12, 1 << 16, "partials")])
def test_c_dist_degraded_read_world1(k, m, nseg, F, exchange):
    """cec_dist_degraded_read (libcessec's own RCCL group, the C form of degraded_read) at world
    1: plan, agreement all-reduce, local survivor copies, per-segment rebuild and copy-out, every
    rebuilt fragment equal to the C oracle's codeword; a store missing a survivor fails with
    CEC_EINVAL before any byte moves. 600 segments take three rounds of the bounded staging."""
    import torch
    import cess_amd
    from cess_amd import distributed as D
    from cess_amd.reedsolomon import CecError
    full, lost = _codewords(k, m, nseg, F)
    n = k + m
    mine = D.local_fragments(nseg, n, 1, 0)
    store = D.FragmentStore({sf: i for i, sf in enumerate(mine)},
                            torch.from_numpy(np.stack([full[s][f] for s, f in mine])).cuda())
    enc = cess_amd.New(k, m)
    g = D.RcclGroup(enc, D.RcclGroup.unique_id(), 1, 0, exchange)
    try:
        out = g.degraded_read(lost, store)
        assert len(out) == sum(len(v) for v in lost.values())
        for (s, f), t in out.items():
            assert np.array_equal(t.cpu().numpy(), full[s][f]), (s, f)
        out2 = g.degraded_read({3: [0]}, store)  # a second call reuses the staging
        assert np.array_equal(out2[(3, 0)].cpu().numpy(), full[3][0])
        gone = D.FragmentStore({sf: i for sf, i in store.slots.items() if sf != (5, k)},
                               store.data)
        with pytest.raises(CecError) as ei:
            g.degraded_read({5: [0]}, gone)
        assert ei.value.code == -1
    finally:
        g.close()


def test_c_dist_abort_in_group_world1():
    """The in-group failure path of cec_dist_degraded_read (CEC_DIST_OPT_TEST_ABORT): the round's
    group is ended and the communicator aborted, the call returns CEC_ENCCL, later calls on the
    handle too, destroying it is clean, and a new group on the same thread and codec then
    rebuilds bit-exact (the thread's RCCL group state was left consistent)."""
    import torch
    import cess_amd
    from cess_amd import distributed as D
    from cess_amd.reedsolomon import CecError
    k, m, nseg, F = 4, 2, 6, 65536
    full, lost = _codewords(k, m, nseg, F)
    mine = D.local_fragments(nseg, k + m, 1, 0)
    store = D.FragmentStore({sf: i for i, sf in enumerate(mine)},
                            torch.from_numpy(np.stack([full[s][f] for s, f in mine])).cuda())
    enc = cess_amd.New(k, m)
    g = D.RcclGroup(enc, D.RcclGroup.unique_id(), 1, 0, "survivors")
    g.set_test_abort(0)
    with pytest.raises(CecError) as ei:
        g.degraded_read(lost, store)
    assert ei.value.code == -6
    with pytest.raises(CecError) as ei:
        g.degraded_read(lost, store)
    assert ei.value.code == -6
    g.close()
    g2 = D.RcclGroup(enc, D.RcclGroup.unique_id(), 1, 0, "survivors")
    try:
        out = g2.degraded_read(lost, store)
        for (s, f), t in out.items():
            assert np.array_equal(t.cpu().numpy(), full[s][f]), (s, f)
    finally:
        g2.close()


def _c_rank(rank, world, uid_path, k, m, nseg, F, q, exchange="survivors"):
    os.environ.update(HSA_ENABLE_IPC_MODE_LEGACY="0")
    import time
    import torch
    import cess_amd
    from cess_amd import distributed as D
    torch.cuda.set_device(rank)
    full, lost = _codewords(k, m, nseg, F)
    n = k + m
    if rank == 0:
        with open(uid_path + ".tmp", "wb") as f:
            f.write(D.RcclGroup.unique_id())
        os.rename(uid_path + ".tmp", uid_path)
    while not os.path.exists(uid_path):
        time.sleep(0.05)
    uid = open(uid_path, "rb").read()
    mine = D.local_fragments(nseg, n, world, rank)
    store = D.FragmentStore({sf: i for i, sf in enumerate(mine)},
                            torch.from_numpy(np.stack([full[s][f] for s, f in mine])).cuda())
    g = D.RcclGroup(cess_amd.New(k, m, device=rank), uid, world, rank, exchange)
    out = g.degraded_read(lost, store)
    ok = all(np.array_equal(t.cpu().numpy(), full[s][f]) for (s, f), t in out.items())
    g.close()
    q.put((rank, ok, len(out)))


@pytest.mark.parametrize("k,m,exchange", [(2, 1, "survivors"), (4, 2, "survivors"),
                                          (4, 2, "partials"), (10, 4, "auto")] + WIDE)
def test_c_dist_degraded_read_rccl(k, m, exchange, tmp_path):
    """The C-ABI degraded read across every visible GPU up to 8 (one process each, the group id
    handed over through a file as a non-Python host would through its control plane)."""
    import torch
    import torch.multiprocessing as mp
    world = min(torch.cuda.device_count(), 8)
    if world < 2:
        pytest.skip("RCCL degraded read needs >= 2 visible GPUs")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    nseg, F = 12, 1 << 20
    uid = str(tmp_path / "uid")
    procs = [ctx.Process(target=_c_rank, args=(r, world, uid, k, m, nseg, F, q, exchange))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res), res
    assert sum(n for _, _, n in res) == sum(1 + s % m for s in range(nseg))


def test_c_dist_from_c(tmp_path):
    """The same world-1 degraded read driven from C (tests/native/dist_world1.c): the path a cgo /
    FFI host takes, with HBM buffers from the HIP runtime and a locate callback."""
    import subprocess
    from tests.conftest import ROOT
    exe = tmp_path / "dist_world1"
    subprocess.run(["gcc", "-O2", "-D__HIP_PLATFORM_AMD__", f"{ROOT}/tests/native/dist_world1.c",
                    f"-I{ROOT}/include", "-I/opt/rocm/include", f"-L{ROOT}/cess_amd", "-lcessec",
                    "-L/opt/rocm/lib", "-lamdhip64", "-lrccl",
                    f"-Wl,-rpath,{ROOT}/cess_amd:/opt/rocm/lib", "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    assert "dist world1 ok" in r.stdout
    # destroy_under_load: a codec, then a dist handle and its codec, destroyed while another
    # codec's ~25 ms batch ran on a side stream (that batch then checked bit-exact); whether the
    # side stream was still running right after each destroy is reported (1 = the destroy did not
    # drain the device), with a bare ncclCommDestroy as the control for the dist handle's
    busy = [ln for ln in r.stdout.splitlines() if ln.startswith("side stream busy")]
    assert busy, r.stdout
    print(busy[0])
    # a codec's teardown waits for its own stream only (r04: stream-ordered frees, pinned blocks
    # cached instead of hipHostFree)
    assert busy[0].startswith("side stream busy after codec destroy: 1"), busy[0]
