#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: "RS encode/decode GB/s per GPU and whole node; % of HBM
roofline", on the CESS segment -> fragment codec (libcessec, HIP kernels for gfx950).

Default workload = BASELINE.json configs[1]: batched encode of 1 GiB of synthetic 16 MiB
segments per GPU, RS(k=2, m=1), 8 MiB fragments, device-resident (inputs already in HBM when
the timed region starts). A "step" is one batched encode launch over the rank's 64 segments.
Bytes counted per segment = (k+m) * F (k fragments read, m written).

    python bench.py [--gpus N --steps K --warmup W] [--config 1|2|3|4|5]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one rank per GPU, weak scaling)

`--gpus N` alone (no WORLD_SIZE in the environment) starts the N ranks itself: the process counts
the visible GPUs without initialising HIP and runs torch.distributed.run as a child. Fewer GPUs
than N, or WORLD_SIZE != N under an external launcher, exits with status 2 instead of measuring
fewer GPUs than asked. Rehearsal on one GPU: CESS_DIST_BACKEND=gloo CESS_DEVICE=0 lets the ranks
share device 0.

Rank 0 prints one JSON line. `roofline` is the dominant kernel's algorithmic bytes per launch /
its average launch time (HIP events on the launch stream); `cpu_baseline` times the C oracle
(oracle/rs_oracle.c, kind "port": the reference ships no codec) on a bounded sample on rank 0.
The default line also carries, at every N: `extra.config4` (BASELINE config 4's 64 GiB file
sharded over the N GPUs, T1 on one GPU, efficiency T1 / (N T_N), sampled segments checked against
the C oracle) and `extra.host_e2e` (an in-memory file per GPU through the C pipeline,
PCIe-inclusive, with and without SegmentList hashing, the hashes on the GPU, on host threads or
hybrid, plus records_stream: SegmentCount-size files back to back through one session); at N = 1
the one-GPU legs (reconstruct,
`extra.wide_code`: RS(32,32) encode / restoral / rebuilds / verify, `extra.config5`: BASELINE
config 5's encode + SHA-256 step); at N > 1 `extra.degraded_gather` and its wide-code and C-ABI
forms: the RCCL survivor / partial-product exchange of BASELINE config 4 (fragment f of segment s
on GPU (s + f) mod N) and the rebuild after it.
Config 1 is the CPU codec alone (one 16 MiB segment: encode + the 3 single-erasure rebuilds at
1 thread and at the host's CPU share); config 4 is 64 GiB sharded over the ranks with the
degraded-read gather inside every step.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

T_START = time.perf_counter()  # the process's start (extra.resources wall times)
MiB = 1 << 20
GB = 1e9
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
# VALU issue peak, full-rate lane-ops/s: 256 CUs x 4 SIMDs x 32 lanes x 2.4 GHz (SURVEY.md §8d:
# the roofline of the SHA-256 stage; half-rate instructions take two of these slots)
VALU_PEAK_TLANE = 256 * 4 * 32 * 2.4e9 / 1e12
METRIC = "RS encode/decode GB/s per GPU and whole node; % of HBM roofline"
SEED0 = 0xCE550000

CONFIGS = {
    # id: (k, m, fragment bytes, segments per GPU, description)
    1: (2, 1, 8 * MiB, 1, "single 16 MiB segment RS(2,1): encode + the 3 single-erasure "
                          "reconstructs, CPU codec (no GPU)"),
    2: (2, 1, 8 * MiB, 64, "batched RS(2,1) encode of 1 GiB of 16 MiB segments per GPU"),
    3: (2, 1, 8 * MiB, 64, "degraded reconstruct RS(2,1), erased fragment = seg mod 3, 1 GiB"),
    4: (2, 1, 8 * MiB, 4096, "64 GiB file (4096 x 16 MiB segments) encoded, sharded over GPUs, "
                             "+ cross-GPU degraded-read gather (RCCL) of 64 segments per GPU "
                             "and their rebuild, every step"),
    5: (32, 32, 512 * 1024, 64, "RS(32,32) encode of 1 GiB + SHA-256 of all 64 fragments "
                                "(encode + GPU hash queue, a window of batches hashing at once)"),
    # stress variant of config 3 for the wide code (not a BASELINE config): every segment loses
    # m random fragments; decode matrices are run-time (host-inverted per pattern)
    6: (32, 32, 512 * 1024, 64, "RS(32,32) degraded reconstruct, 32 random erasures/segment"),
    # single-fragment repair of the wide code (the restoral case: one lost fragment per segment)
    7: (32, 32, 512 * 1024, 64, "RS(32,32) repair of one random fragment per segment, 1 GiB"),
    # a common general-purpose code with no compile-time kernel: run-time coefficients
    8: (10, 4, 2 * MiB, 64, "RS(10,4) encode (run-time coefficients), 1.25 GiB of 20 MiB segments"),
}


# exit status of a run whose C-ABI exchange legs stalled (cabi_legs' watchdog): the line is
# printed, but the process does not report success
WATCHDOG_EXIT = 3

GPU_BOX_CPU_SHARE = 16  # CPUs the harness gives one GPU's job on the box (its pools obey this)


def cpu_threads(gpus: int = 1) -> int:
    """Threads for the CPU baseline: the host's CPU share for the GPUs in use. The GPU box shows
    the whole machine's CPUs to nproc / os.cpu_count() but gives each GPU's job a 16-CPU share,
    and worker pools must stay within it; the CPU rate is therefore quoted at that share (16 per
    GPU the job holds: the whole node's share on an 8-GPU run), with the per-thread rate
    beside it."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(GPU_BOX_CPU_SHARE * max(1, gpus), n))


SIMD_NAMES = {0: "scalar table", 1: "AVX2 split-nibble", 2: "AVX-512BW + GFNI affine"}


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(k: int, m: int, F: int, target_s: float, gpus: int = 1) -> dict:
    """Time the C oracle (oracle/rs_oracle.c) on a bounded sample of the same workload, on the
    CPU share of the `gpus` GPUs the job holds (the whole node's share for a multi-GPU line)."""
    from oracle.c_oracle import load_c_oracle
    orc = load_c_oracle()
    simd = orc.orc_set_simd(-1)  # the best form the host has
    # same workload shape as the GPU step (1 GiB of segments), larger than the host's LLC
    nseg = max(1, (1 << 30) // (k * F))
    data = np.empty(nseg * k * F, np.uint8)
    par = np.empty(nseg * m * F, np.uint8)
    orc.orc_fill_synthetic(data.ctypes.data, k * F, nseg, 0, SEED0 + 2)
    threads = cpu_threads(gpus)
    orc.orc_encode_batch(k, m, data.ctypes.data, par.ctypes.data, nseg, F, threads, 1)  # touch
    t1 = orc.orc_encode_batch(k, m, data.ctypes.data, par.ctypes.data, nseg, F, threads, 1)
    reps = max(1, int(target_s / max(t1, 1e-6)))
    t = orc.orc_encode_batch(k, m, data.ctypes.data, par.ctypes.data, nseg, F, threads, reps)
    n1 = min(nseg, 8)
    st = orc.orc_encode_batch(k, m, data.ctypes.data, par.ctypes.data, n1, F, 1, 1)
    per_seg = (k + m) * F
    return {
        "value": round(reps * nseg * per_seg / t / GB, 3),
        "unit": "GB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{reps} x {nseg} segments of {k * F // MiB} MiB, RS({k},{m}), "
                  f"{SIMD_NAMES[simd]} C oracle, {threads} threads (the CPU share of the "
                  f"{gpus} GPU(s) in use: {GPU_BOX_CPU_SHARE} per GPU), {t:.1f} s",
        "value_1thread": round(n1 * per_seg / st / GB, 3),
        "cpu_model": cpu_model(),
        "host_cpus_visible": os.cpu_count(),
        "gpus_in_use": gpus,
    }


def cpu_sha256(k: int, m: int, F: int, target_s: float) -> dict:
    """CPU leg of config 5's hashing: OpenSSL SHA-256 (hashlib; SHA-NI where the host has it)
    over the fragments of one batch, on the CPU share (hashlib releases the GIL)."""
    import concurrent.futures as cf
    import hashlib
    nfrag = (1 << 30) // F  # 1 GiB of fragments
    buf = np.frombuffer(np.random.default_rng(5).bytes(nfrag * F), np.uint8).reshape(nfrag, F)
    threads = cpu_threads()
    t0 = time.perf_counter()
    reps = 0
    with cf.ThreadPoolExecutor(threads) as ex:
        while True:
            list(ex.map(lambda i: hashlib.sha256(buf[i]).digest(), range(nfrag)))
            reps += 1
            if time.perf_counter() - t0 > target_s:
                break
    t = time.perf_counter() - t0
    t1 = time.perf_counter()
    for i in range(min(nfrag, 64)):
        hashlib.sha256(buf[i]).digest()
    t1 = time.perf_counter() - t1
    return {"value": round(reps * nfrag * F / t / GB, 3), "unit": "GB/s hashed",
            "cores": threads, "kind": "library (OpenSSL via hashlib)",
            "sample": f"{reps} x {nfrag} fragments of {F // 1024} KiB, {threads} threads",
            "value_1thread": round(min(nfrag, 64) * F / t1 / GB, 3)}


def config1_cpu(args) -> dict:
    """BASELINE config 1: one 16 MiB segment, RS(2,1): encode + the 3 single-erasure rebuilds,
    on the CPU codec (oracle/rs_oracle.c, kind "port": the reference has no codec), at 1 thread
    and at this GPU's CPU share; the same ops on the GPU (device resident) beside it."""
    from oracle.c_oracle import load_c_oracle, ptrs
    k, m, F = 2, 1, 8 * MiB
    orc = load_c_oracle()
    simd = orc.orc_set_simd(-1)
    seg = np.empty(k * F, np.uint8)
    orc.orc_fill_synthetic(seg.ctypes.data, k * F, 1, 0, SEED0 + 1)
    shards = [seg[:F].copy(), seg[F:].copy(), np.zeros(F, np.uint8)]
    per_op = (k + m) * F  # read k, write 1 (RS(2,1)): 24 MiB per op
    ops = 1 + (k + m)
    out = {}
    for th in (1, cpu_threads()):
        orc.orc_segment_ops(k, m, ptrs(shards), F, th, 1)
        t1 = orc.orc_segment_ops(k, m, ptrs(shards), F, th, 1)
        reps = max(1, int(args.cpu_seconds / 2 / max(t1, 1e-6)))
        t = orc.orc_segment_ops(k, m, ptrs(shards), F, th, reps)
        out[th] = (reps * ops * per_op / t / GB, reps, t)
    threads = cpu_threads()
    res = {
        "metric": METRIC, "value": round(out[threads][0], 3), "unit": "GB/s", "n_gpus": 0,
        "steps": out[threads][1], "warmup": 1,
        "ms_per_step": round(out[threads][2] / out[threads][1] * 1e3, 4),
        "higher_is_better": True, "scaling": "none", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (splitmix64 counter generator)",
        "config": {"workload": CONFIGS[1][4], "baseline_config": 1, "k": k, "m": m,
                   "fragment_bytes": F, "ops_per_step": "encode + rebuild of shard 0, 1, 2",
                   "bytes_per_op": per_op},
        "roofline": None,
        "cpu_baseline": {"value": round(out[threads][0], 3), "unit": "GB/s", "cores": threads,
                         "kind": "port",
                         "sample": f"{out[threads][1]} x (encode + 3 rebuilds) of one 16 MiB "
                                   f"segment, {SIMD_NAMES[simd]}, columns split over {threads} "
                                   f"threads (this GPU's CPU share)",
                         "value_1thread": round(out[1][0], 3), "cpu_model": cpu_model(),
                         "host_cpus_visible": os.cpu_count()},
        "note": "the reference ships no codec (SURVEY.md §0.1); the CPU codec is this repo's C "
                "restatement of klauspost/reedsolomon",
    }
    try:
        import torch
        if torch.cuda.is_available():
            import cess_amd
            dev = torch.device("cuda", 0)
            d_data = torch.from_numpy(seg.reshape(1, k, F)).to(dev)
            d_par = torch.empty((1, m, F), dtype=torch.uint8, device=dev)
            enc = cess_amd.New(k, m)
            st = torch.cuda.current_stream(dev)
            pats = [np.array([int(i != e) for i in range(k + m)], np.uint8) for e in range(k + m)]

            def step():
                enc.EncodeBatch(d_data, d_par, 1, F, stream=st)
                for p in pats:
                    enc.ReconstructBatch(d_data, d_par, 1, F, p, stream=st)
            for _ in range(5):
                step()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(50):
                step()
            b.record(st)
            torch.cuda.synchronize(dev)
            ms = a.elapsed_time(b) / 50
            res["gpu_same_workload"] = {"GBps": round(ops * per_op / (ms * 1e-3) / GB, 2),
                                        "ms_per_step": round(ms, 4),
                                        "note": "one segment per launch: launch-latency bound"}
            # the same step replayed as one HIP graph (the compile-time RS(2,1) kernels read no
            # codec-owned memory, so their launches capture safely once warm)
            side = torch.cuda.Stream(dev)
            side.wait_stream(st)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=side):
                cur = torch.cuda.current_stream(dev)
                enc.EncodeBatch(d_data, d_par, 1, F, stream=cur)
                for p in pats:
                    enc.ReconstructBatch(d_data, d_par, 1, F, p, stream=cur)
            torch.cuda.synchronize(dev)
            with torch.cuda.stream(side):
                for _ in range(5):
                    g.replay()
                a.record(side)
                for _ in range(200):
                    g.replay()
                b.record(side)
            torch.cuda.synchronize(dev)
            gms = a.elapsed_time(b) / 200
            res["gpu_same_workload"].update(
                {"graph_ms_per_step": round(gms, 4),
                 "graph_GBps": round(ops * per_op / (gms * 1e-3) / GB, 2)})
    except Exception as e:  # noqa: BLE001 - the CPU leg stands on its own
        res["gpu_same_workload"] = {"error": str(e)[:200]}
    return res


def degraded_gather(enc, k: int, m: int, F: int, world: int, rank: int, dev, nseg: int,
                    exchange: str = "survivors", transport: str = "torch"):
    """BASELINE config 4's exchange step, set up once: segments 0..nseg*world-1 stored under the
    miner-spread placement (fragment f of segment s on GPU (s + f) mod world,
    c-pallets/file-bank/src/functions.rs:187-283), every segment losing fragment s mod (k+m).
    Returns (run, verify, plan, close): run() moves survivors (or, exchange "partials"/"auto",
    partial rebuilds: SURVEY.md §8e) between the ranks (RCCL point to point; RCCL has no XOR
    reduction) and rebuilds the lost fragments with libcessec. transport "torch": the
    torch.distributed process group (distributed.degraded_read); "cabi": libcessec's own RCCL
    communicator behind the C ABI (cec_dist_degraded_read, what a Go / Rust host calls), its
    group id handed to the other ranks over the process group."""
    import torch
    import cess_amd
    from cess_amd import distributed as D
    n = k + m
    total = nseg * world
    mine = D.local_fragments(total, n, world, rank)
    store = D.FragmentStore({sf: i for i, sf in enumerate(mine)},
                            torch.empty((max(1, len(mine)), F), dtype=torch.uint8, device=dev))
    seg_d = torch.empty((1, k, F), dtype=torch.uint8, device=dev)
    seg_p = torch.empty((1, m, F), dtype=torch.uint8, device=dev)
    for s in range(total):
        if not any((s, f) in store.slots for f in range(n)):
            continue
        cess_amd.fill_synthetic(seg_d, k * F, 1, s, SEED0 + 4)
        enc.EncodeBatch(seg_d, seg_p, 1, F)
        for f in range(n):
            if (s, f) in store.slots:
                store.data[store.slots[(s, f)]].copy_(seg_d[0, f] if f < k else seg_p[0, f - k])
    torch.cuda.synchronize(dev)
    lost = {s: [s % n] for s in range(total)}
    plan = D.plan_gather(lost, k, m, world, F, exchange=exchange)
    group = None
    if transport == "cabi":
        import torch.distributed as dist
        uid = [D.RcclGroup.unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        group = D.RcclGroup(enc, uid[0], world, rank, exchange)

        def run():
            return group.degraded_read(lost, store)
    else:
        def run():
            return D.degraded_read(plan, store, enc, rank)

    def verify(out) -> bool:
        ok = True
        for (s, f), got in out.items():
            cess_amd.fill_synthetic(seg_d, k * F, 1, s, SEED0 + 4)
            enc.EncodeBatch(seg_d, seg_p, 1, F)
            ok &= bool(torch.equal(got, seg_d[0, f] if f < k else seg_p[0, f - k]))
        return ok

    def close():
        if group is not None:
            group.close()
    return run, verify, plan, close


def cu_split_streams(c: int, dev):
    """Two HIP streams on disjoint CU sets (hipExtStreamCreateWithCUMask): c CUs for the first,
    the rest for the second. The c CUs are spread so that each group of 32 consecutive CU indices
    and each residue class mod 8 gets an equal share (either XCD numbering)."""
    import ctypes
    import torch
    hip = ctypes.CDLL("libamdhip64.so")
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    groups = ncu // 32
    q = c // groups
    sel = set()
    for x in range(groups):
        for r in range(q):
            sel.add(32 * x + (x + 8 * r + r // 4) % 32)
    words = (ncu + 31) // 32
    m1 = (ctypes.c_uint32 * words)()
    m2 = (ctypes.c_uint32 * words)()
    for i in range(ncu):
        (m1 if i in sel else m2)[i // 32] |= 1 << (i % 32)
    out = []
    for m in (m1, m2):
        h = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(words), m)
        if rc != 0:
            raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
        out.append(torch.cuda.ExternalStream(h.value, device=dev))
    return out


def load_valu_slots(tag: str):
    """Static VALU issue slots per 64-byte block of the hash-queue tick (profiles/valu_<tag>.json,
    written by tools/sha_slots.py from the built code object), or None."""
    try:
        with open(os.path.join(ROOT, "profiles", f"valu_{tag}.json")) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


# per-rank resource marks the legs record (extra.resources: the N = 8 line's footprint)
RES = {}


def hbm_used_gib(dev) -> float:
    import torch
    free, total = torch.cuda.mem_get_info(dev)
    return round((total - free) / 2**30, 2)


def resources(dev, world: int, rank: int, t_start: float) -> dict:
    """Every rank's peak host RSS, peak torch HBM, the HBM marks the legs recorded and its wall
    time so far, gathered to rank 0 (None elsewhere)."""
    import resource
    import torch
    import torch.distributed as dist
    mine = dict(RES, rank=rank, wall_s=round(time.perf_counter() - t_start, 1),
                peak_rss_GiB=round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20, 2),
                torch_peak_reserved_GiB=round(torch.cuda.max_memory_reserved(dev) / 2**30, 2),
                hbm_used_now_GiB=hbm_used_gib(dev))
    if world == 1:
        return {"ranks": [mine]}
    got = [None] * world
    dist.all_gather_object(got, mine)
    if rank != 0:
        return None
    return {"ranks": got, "note": "hbm_used_* = the whole device's used HBM (mem_get_info) at "
                                  "that point; ranks sharing one GPU (CESS_DEVICE rehearsal) all "
                                  "see the same device"}


def load_clock(tag: str, kernel: str):
    """Shader clock (GHz) under `kernel` from profiles/r06/pmc_<tag>_clock.json (written by
    tools/pmc_clock.py from a GRBM_GUI_ACTIVE pass), or None."""
    try:
        with open(os.path.join(ROOT, "profiles", "r06", f"pmc_{tag}_clock.json")) as f:
            ks = json.load(f)["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    for name, v in ks.items():
        if kernel in name:
            return v.get("clock_GHz")
    return None


def load_traffic(tag: str, algo_bytes: int, kernel: str):
    """Per-launch HBM bytes from the PMC passes (profiles/traffic_<tag>.json), if they were
    collected for this kernel at this launch size; None otherwise."""
    path = os.path.join(ROOT, "profiles", f"traffic_{tag}.json")
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    if t.get("algorithmic_bytes_per_launch") != algo_bytes or t.get("kernel") not in kernel:
        return None
    return t.get("bytes_per_launch")


def traffic_source(tag: str) -> str:
    return (f"profiles/traffic_{tag}.json (PMC FETCH_SIZE + WRITE_SIZE of the same launch, "
            f"recorded by a rocprofv3 --pmc run of this bench; not measured in this run)")


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def world_check(gpus: int, env=os.environ, visible=None) -> tuple:
    """What `--gpus N` means in this process: ("run", world) when the ranks already exist (under
    torchrun WORLD_SIZE must equal N), ("launch", N) when this process must start N ranks itself,
    ("error", message) otherwise. `visible` = GPUs this process could use (counted without
    initialising HIP); ranks may share one GPU only in the rehearsal mode (CESS_DEVICE set)."""
    if gpus < 1:
        return "error", f"--gpus {gpus}: need at least one GPU"
    if "WORLD_SIZE" in env:
        ws = int(env["WORLD_SIZE"])
        if ws != gpus:
            return "error", (f"WORLD_SIZE={ws} but --gpus {gpus}: launch exactly --gpus ranks "
                             f"(one per GPU)")
        return "run", ws
    if gpus == 1:
        return "run", 1
    if "CESS_DEVICE" not in env and (visible or 0) < gpus:
        return "error", f"--gpus {gpus} but {visible or 0} GPU(s) visible"
    return "launch", gpus


def launch_ranks(n: int, argv) -> int:
    """Start n rank processes (torch.distributed.run, one per GPU, rendezvous on 127.0.0.1) as a
    child and wait for it. This process never initialises HIP: it only counted the devices."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
           str(n), "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def cabi_legs(ex_out, gather_leg, degraded_gather, enc, code, world, rank, dev, deadline,
              emit, torch_legs=False, cabi=True):
    """The cross-GPU exchange legs of the N > 1 line, run last, after every other measurement,
    under one watchdog: with `torch_legs` the degraded read over the torch.distributed group
    (RS(2,1) survivors, RS(32,32) both exchanges), then (`cabi`) the same through libcessec's
    own RCCL communicator (cec_dist_*, the C ABI a Go / Rust host uses), on the same placement.
    A leg that raises is recorded as an error and the next one runs. A rank that fails or stalls
    inside a collective exchange would otherwise hold every rank in it, so past `deadline`
    seconds each rank records the unfinished legs as such, rank 0 prints the line it has (`emit`),
    and the process ends with status WATCHDOG_EXIT (os._exit: the peers are stuck in RCCL), so the
    driver's rc records that a rank hung while the line stays parseable."""
    import threading
    import torch
    import torch.distributed as dist
    import cess_amd
    k, m, F = code
    done = threading.Event()
    legs = ((("degraded_gather", "wide_degraded_gather") if torch_legs else ()) +
            (("degraded_gather_cabi", "wide_degraded_gather_cabi") if cabi else ()))

    def watchdog():
        if done.wait(deadline):
            return
        try:
            for name in legs:
                if name not in ex_out:
                    ex_out[name] = {"error": f"not finished after {deadline:.0f} s (a rank failed "
                                             "or stalled inside the cec_dist exchange)"}
            emit()
        finally:
            if rank != 0:
                # a failing rank makes torchrun stop the others: give rank 0 time to print first
                time.sleep(10)
            os._exit(WATCHDOG_EXIT)

    threading.Thread(target=watchdog, daemon=True).start()
    ok = 1
    for via, suffix, transport in (("torch", "", "torch.distributed group"),
                                   ("cabi", "_cabi",
                                    "libcessec cec_dist_degraded_read (own RCCL communicator)")):
        if "degraded_gather" + suffix not in legs:
            continue
        try:
            leg = gather_leg(degraded_gather(enc, k, m, F, world, rank, dev, 64, "survivors",
                                             via))
            leg["transport"] = transport
            ex_out["degraded_gather" + suffix] = leg
            # the wide code's single-fragment degraded read, both exchanges:
            # RS(32,32) with 16 MiB segments (F = 512 KiB), 8 fragments per GPU at world 8; 32
            # segments per GPU keep the survivor leg's grouped point-to-point batch under ~900
            # transfers per rank
            wk, wm, wF = CONFIGS[5][:3]
            wenc = cess_amd.New(wk, wm, device=dev.index)
            try:
                wide = {}
                for ex in ("survivors", "partials"):
                    wide[ex] = gather_leg(degraded_gather(wenc, wk, wm, wF, world, rank, dev, 32,
                                                          ex, via), code=(wk, wF))
                    wide[ex]["transport"] = transport
                ex_out["wide_degraded_gather" + suffix] = wide
            finally:
                wenc.close()
        except Exception as e:  # noqa: BLE001 - reported in the line
            ok = 0
            for name in ("degraded_gather" + suffix, "wide_degraded_gather" + suffix):
                ex_out.setdefault(name, {"error": f"{type(e).__name__}: {e}"[:400]})
    # every rank that got here agrees (cec_dist fails a caller error on all ranks alike); a rank
    # stuck in the exchange never arrives, and the watchdog then ends the ones waiting here
    if world > 1:
        flag = torch.tensor([ok], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    done.set()


def erasure_patterns(k: int, m: int, nseg: int, ne: int, seed: int,
                     lose_parity: bool = False, run: bool = False) -> np.ndarray:
    """Configs 6 / 7: [nseg][k + m] present flags, ne random erasures per segment (or every
    parity shard lost; or, `run`, ne consecutive shard indices from a random start, wrapping: a
    correlated loss such as neighbouring miners of the placement going down together);
    tests/test_host.py replays the chooser on the same patterns."""
    rng = np.random.default_rng(seed)
    present = np.ones((nseg, k + m), np.uint8)
    for s_ in range(nseg):
        if lose_parity:
            present[s_, k:] = 0
        elif run:
            present[s_, (int(rng.integers(0, k + m)) + np.arange(ne)) % (k + m)] = 0
        else:
            present[s_, rng.choice(k + m, size=ne, replace=False)] = 0
    return present


def kernel_label(config: int, fd_frac, erasures: int, generic: bool, rt_mode: int, k: int,
                 fdd_frac=0) -> str:
    """The dominant kernel of a bench line. Config 6: fd_frac = share of the timed rebuilds the
    library sent to the FFT-domain decoders (CEC_STAT_FFTDEC_SEGMENTS), fdd_frac the share of them
    on the formal-derivative one (CEC_STAT_FFTDEC_D_SEGMENTS)."""
    if config == 6:
        fdm = (fd_frac or 0) - (fdd_frac or 0)
        name = ("k_fftdec_d" if fdd_frac == 1 else
                "k_fftdec_m" if fd_frac == 1 and not fdd_frac else
                "k_rthx<8>" if fd_frac == 0 and erasures > 4 else
                "k_rtb" if fd_frac == 0 else
                f"k_fftdec_m ({fdm:.0%} of segments) + k_fftdec_d ({fdd_frac or 0:.0%}) + "
                f"k_rthx<8> (by pattern cost)")
    else:
        name = {2: "k_ct<EncCT<2, 1>>",
                3: "k_ct_dec1_mixed21 (Dec1CT<2, 1, e> / EncCT<2, 1> per segment)",
                4: "k_ct<EncCT<2, 1>>", 5: "k_fft3232<true, true>", 7: "k_rtb<1>",
                8: "k_rtb<4>"}[config]
    if generic:
        name = "k_rthx" if k <= 32 else "k_rt"
    if rt_mode and (generic or config in (6, 7, 8)):
        name = {1: "k_rt", 2: "k_rth", 3: "k_rtb"}[rt_mode]
    return name


def wide_code_legs(dev, local, stream, nseg=64, reps=10) -> dict:
    """RS(32,32) legs timed with HIP events on `stream` (64 segments of 16 MiB, 2 GiB per batch):
    encode, restoral of one random lost fragment per segment, rebuilds of 8 and 32 random
    erasures per segment (per-segment patterns; the library picks k_fftdec_m or k_rthx by its
    cost model), verify. Algorithmic bytes as the bench line's: (k + outputs) x F per segment
    (encode and verify: (k + m) x F). The batch is checked with the fused verify afterwards."""
    import torch

    import cess_amd
    k, m, F = 32, 32, 512 * 1024
    enc = cess_amd.New(k, m, device=local)
    d_data = torch.empty((nseg, k, F), dtype=torch.uint8, device=dev)
    d_par = torch.empty((nseg, m, F), dtype=torch.uint8, device=dev)
    cess_amd.fill_synthetic(d_data, k * F, nseg, 0, 0xCE550005, stream=stream)
    rng = np.random.default_rng(0xCE55)

    # A VALU-heavy kernel's first ~30 launches ride a clock transient (k_fftdec_d under rocprof:
    # 0.82 -> 1.12 -> 0.82 ms over launches 1..30, profiles/r03/fdd_clock_transient.txt): each leg
    # reports the mean of its first `warm` launches (cold: what a short restoral burst sees; one
    # untimed call before them builds the decode plans) beside the mean of the `reps` after them
    warm = 3 * reps

    def timed_ms(fn):
        fn()  # plans built / cached
        torch.cuda.synchronize(dev)
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0.record(stream)
        for _ in range(warm):
            fn()
        c1.record(stream)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(reps):
            fn()
        b.record(stream)
        torch.cuda.synchronize(dev)
        return a.elapsed_time(b) / reps, c0.elapsed_time(c1) / warm

    legs = {}

    def leg(name, fn, outs):
        ms, cold = timed_ms(fn)
        byt = nseg * (k + outs) * F
        legs[name] = {"ms": round(ms, 4), "GBps": round(byt / (ms * 1e-3) / GB, 1),
                      f"cold_ms_first{warm}": round(cold, 4),
                      "cold_GBps": round(byt / (cold * 1e-3) / GB, 1)}

    leg("encode", lambda: enc.EncodeBatch(d_data, d_par, nseg, F, stream=stream), m)
    for ne, name in ((1, "restoral_1_lost"), (8, "rebuild_8_lost"), (32, "rebuild_32_lost")):
        pres = np.ones((nseg, k + m), np.uint8)
        for s_ in range(nseg):
            pres[s_, rng.choice(k + m, size=ne, replace=False)] = 0
        fd0, fdd0 = enc.stat(4), enc.stat(5)
        leg(name, lambda: enc.ReconstructBatch(d_data, d_par, nseg, F, pres, stream=stream), ne)
        legs[name]["fftdec_segment_share"] = round(
            (enc.stat(4) - fd0) / (nseg * (reps + warm + 1)), 3)
        legs[name]["fftdec_d_segment_share"] = round(
            (enc.stat(5) - fdd0) / (nseg * (reps + warm + 1)), 3)
    d_ok = torch.empty(nseg, dtype=torch.uint8, device=dev)
    leg("verify", lambda: enc.VerifyBatch(d_data, d_par, nseg, F, d_ok=d_ok, stream=stream), m)
    torch.cuda.synchronize(dev)
    legs["codeword_consistent_after_rebuilds"] = bool(d_ok.cpu().numpy().all())
    legs["workload"] = f"RS(32,32), {nseg} segments of 16 MiB (F = 512 KiB) per launch"
    enc.close()
    del d_data, d_par
    return legs


class HashPipeline:
    """BASELINE config 5's step, windowed over steps: step i encodes into parity buffer i % (W+1)
    on the launch stream, then (on the hash stream, after the encode) adds the batch's
    nseg * (k+m) fragment chains to the GPU hash queue and ticks it once: each tick advances every
    live chain by ceil(blocks per fragment / W) blocks, so a batch's hashes complete W ticks
    after its encode and W batches hash together (W x nseg x (k+m) chains in flight). The data
    batch is read-only and shared; parity and hex are (W+1)-buffered: the batch a step overwrites
    completed one tick earlier, so the encode of step i + 1 waits for tick i - 1 and overlaps
    tick i."""

    def __init__(self, enc, d_data, d_par, nseg, F, dev, local, stream, sha_stream, W,
                 tick_pf=0):
        import torch
        import cess_amd
        k, m = enc.DataShards, enc.ParityShards
        self.enc, self.d_data, self.nseg, self.F = enc, d_data, nseg, F
        self.k, self.m, self.W, self.NB = k, m, W, W + 1
        self.stream, self.sha_stream = stream, sha_stream
        d_hex = torch.empty((nseg, k + m, 64), dtype=torch.uint8, device=dev)
        self.pipe_par = [d_par] + [torch.empty_like(d_par) for _ in range(self.NB - 1)]
        self.pipe_hex = [d_hex] + [torch.empty_like(d_hex) for _ in range(self.NB - 1)]
        chains = W * nseg * (k + m)
        self.hq = cess_amd.HashQueue(capacity=1 << max(10, (chains - 1).bit_length()),
                                     device=local, stream=sha_stream)
        if tick_pf:
            self.hq.set_option(1, tick_pf)
        self.tick_blocks = -(-cess_amd.sha256_blocks(F) // W)
        self.ev_enc = [torch.cuda.Event() for _ in range(self.NB)]
        self.ev_free = [torch.cuda.Event() for _ in range(self.NB)]
        self.i = 0

    def step(self):
        i, NB, W = self.i, self.NB, self.W
        self.i += 1
        b = i % NB
        if i >= NB:
            self.stream.wait_event(self.ev_free[b])  # batch i - NB's hashes done: b reusable
        self.enc.EncodeBatch(self.d_data, self.pipe_par[b], self.nseg, self.F, stream=self.stream)
        self.ev_enc[b].record(self.stream)
        self.sha_stream.wait_event(self.ev_enc[b])
        self.hq.add_fragments(self.d_data, self.pipe_par[b], self.nseg, self.k, self.m, self.F,
                              self.pipe_hex[b])
        self.hq.tick(self.tick_blocks)
        # this tick completed batch i - W + 1, whose buffer step i + 2 takes
        self.ev_free[(i - W + 1) % NB].record(self.sha_stream)

    def drain(self):
        self.hq.finish()
        if self.sha_stream is not self.stream:
            self.stream.wait_stream(self.sha_stream)


def config5_leg(dev, local, W: int = 96, warmup: int = 10, sample: int = 48) -> dict:
    """BASELINE config 5 inside the default line: RS(32,32) encode of 64 x 16 MiB segments plus
    SHA-256 of all 4,096 fragments per step through the hash-queue pipeline (window W on a second
    stream), timed over 4 W steps with the window drained at the end, so every timed batch is
    fully hashed inside the region. Reports the whole step's rate in fragment bytes (encode and
    hash of (k+m) x F per segment), the hash ticks against the VALU issue roofline, and a hashlib
    check of `sample` fragment digests from several pipeline buffers."""
    import hashlib
    import torch
    import cess_amd
    k, m, F, nseg = CONFIGS[5][0], CONFIGS[5][1], CONFIGS[5][2], CONFIGS[5][3]
    # The encode runs on the current stream, the ticks on a fresh one. A fresh encode stream too
    # (round 4's leg) can land on the ticks' hardware queue (HIP hands its 4 queues to streams
    # round robin; this process has made many by now): the two then serialise and the step takes
    # 1.70-1.71 ms instead of 1.53-1.54 on the same box (profiles/r05/c5_gap2/; CESS_C5_STREAM=new
    # reproduces it)
    stream = (torch.cuda.Stream(dev) if os.environ.get("CESS_C5_STREAM") == "new"
              else torch.cuda.current_stream(dev))
    sha_stream = torch.cuda.Stream(dev)
    enc = cess_amd.New(k, m, device=local)
    d_data = torch.empty((nseg, k, F), dtype=torch.uint8, device=dev)
    d_par = torch.empty((nseg, m, F), dtype=torch.uint8, device=dev)
    cess_amd.fill_synthetic(d_data, k * F, nseg, 0, SEED0 + 5, stream=stream)
    pipe = HashPipeline(enc, d_data, d_par, nseg, F, dev, local, stream, sha_stream, W)
    for _ in range(warmup):
        pipe.step()
    pipe.drain()
    torch.cuda.synchronize(dev)
    # 4 W steps (>= W + 20): the final drain, where fewer chains are left in flight, is a small
    # part of the region (W + 20 steps: 1.86 ms per step; the standalone config 5 over 200-400
    # steps: 1.55-1.63)
    steps = 4 * W
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record(stream)
    for _ in range(steps):
        pipe.step()
    pipe.drain()
    b.record(stream)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    gpu_ms = a.elapsed_time(b)
    step_bytes = nseg * (k + m) * F
    out = {"workload": CONFIGS[5][4], "k": k, "m": m, "fragment_bytes": F, "segments": nseg,
           "window": W, "steps": steps, "warmup": warmup,
           "chains_in_flight": W * nseg * (k + m), "tick_blocks": pipe.tick_blocks,
           "ms_per_step": round(gpu_ms / steps, 4),
           "step_GBps": round(steps * step_bytes / (gpu_ms * 1e-3) / GB, 1),
           "step_GBps_host_clock": round(steps * step_bytes / elapsed / GB, 1),
           "bytes_per_step": step_bytes,
           "basis": "fragment bytes per step ((k+m) x F per segment: encoded and hashed) / "
                    "GPU time of the timed steps incl. the final drain (HIP events on the "
                    "encode stream, which waits for the hash stream at the end)"}
    slots = load_valu_slots("c5")
    if slots:
        blocks = nseg * (k + m) * cess_amd.sha256_blocks(F) * steps
        ach = blocks * slots["issue_slots_per_block"] / (gpu_ms * 1e-3) / 1e12
        out["sha_roofline"] = {
            "bound": "valu", "kernel": "k_sha256_tick1", "achieved": round(ach, 2),
            "peak": round(VALU_PEAK_TLANE, 2), "unit": "T lane-slots/s",
            "frac": round(ach / VALU_PEAK_TLANE, 4),
            "issue_slots_per_block": slots["issue_slots_per_block"],
            "basis": "whole step (hash ticks share the chip with the encode); peak at 2.4 GHz"}
        clk = load_clock("c5", "k_sha256_tick1")
        if clk:
            out["sha_roofline"].update({
                "clock_GHz": clk, "frac_at_clock": round(ach / (VALU_PEAK_TLANE * clk / 2.4), 4),
                "clock_source": "profiles/r06/pmc_c5_clock.json (GRBM_GUI_ACTIVE / 8 XCDs / "
                                "duration of the tick dispatches in a rocprofv3 --pmc pass of "
                                "bench.py --config 5; not measured in this run)"})
    # digests: every batch encodes the same data, so each buffer's hex must be the hashlib digest
    # of the data fragments and of the parity fragments in that buffer
    rng = np.random.default_rng(0xC5)
    ok = True
    checked = 0
    for bi in rng.choice(pipe.NB, size=min(pipe.NB, 6), replace=False):
        hexb = pipe.pipe_hex[int(bi)].cpu().numpy()
        for s_, f_ in zip(rng.integers(0, nseg, sample // 6), rng.integers(0, k + m, sample // 6)):
            frag = (d_data[s_, f_] if f_ < k else pipe.pipe_par[int(bi)][s_, f_ - k]).cpu().numpy()
            ok &= hashlib.sha256(frag.tobytes()).hexdigest().encode() == hexb[s_, f_].tobytes()
            checked += 1
    out["digests_checked"] = checked
    out["digests_match_hashlib"] = bool(ok)
    enc.close()
    del pipe, d_data, d_par
    torch.cuda.empty_cache()
    return out


def oracle_sample_check(d_data, d_par, rows, seg0: int, k: int, m: int, F: int, seed: int) -> bool:
    """The checker (test infrastructure, after the timed region): the sampled segments' data equal
    the counter generator's bytes and their parity equals the C oracle's encode
    (oracle/rs_oracle.c), byte for byte. rows = batch rows; seg0 + row = the file's segment."""
    from oracle.c_oracle import load_c_oracle
    orc = load_c_oracle()
    got_d = d_data[rows].cpu().numpy()
    got_p = d_par[rows].cpu().numpy()
    want_d = np.empty((len(rows), k, F), np.uint8)
    want_p = np.empty((len(rows), m, F), np.uint8)
    for i, r in enumerate(rows):
        orc.orc_fill_synthetic(want_d[i].ctypes.data, k * F, 1, seg0 + int(r), seed)
    orc.orc_encode_batch(k, m, want_d.ctypes.data, want_p.ctypes.data, len(rows), F,
                         cpu_threads(), 1)
    return bool(np.array_equal(got_d, want_d) and np.array_equal(got_p, want_p))


def config4_leg(dev, local: int, world: int, rank: int, backend: str, reps: int = 10) -> dict:
    """BASELINE config 4's encode at every N, inside the default line: the 64 GiB file (4096 x
    16 MiB segments, RS(2,1)) sharded contiguously over the ranks, 4096 / N segments per GPU, one
    batched encode launch per GPU per pass. T1 = the whole file encoded by one GPU (rank 0, in
    this process, every other rank waiting), T_N = the max over ranks of the per-pass time of the
    sharded encode, efficiency = T1 / (N T_N). Both are HIP-event means over
    `reps` back-to-back passes on the launch stream (host clock, barrier to barrier, beside
    them). Sampled segments of every pass buffer are checked against the C oracle afterwards.
    Buffers are freed before the later legs. Segment placement: contiguous shards, the encode
    half of c-pallets/file-bank/src/functions.rs:187-283 (segments are independent: no collective
    on the data path)."""
    import torch
    import torch.distributed as dist
    import cess_amd
    k, m, F = CONFIGS[4][:3]
    total = CONFIGS[4][3]
    seed = SEED0 + 4
    per_seg = (k + m) * F
    stream = torch.cuda.current_stream(dev)
    enc = cess_amd.New(k, m, device=local)
    shared = "CESS_DEVICE" in os.environ  # ranks share one GPU (rehearsal)

    def reduce_max(vals):
        if world == 1:
            return vals
        t = torch.tensor(vals, dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return [float(x) for x in t]

    def barrier():
        if world > 1:
            dist.barrier()

    def encode_pass(seg0: int, nseg: int, timed_alone: bool):
        """Allocate + fill nseg segments from seg0, encode reps times; (event ms, host ms, ok)."""
        free, _ = torch.cuda.mem_get_info(dev)
        if free < nseg * per_seg + (1 << 30):
            return None
        d_data = torch.empty((nseg, k, F), dtype=torch.uint8, device=dev)
        d_par = torch.empty((nseg, m, F), dtype=torch.uint8, device=dev)
        cess_amd.fill_synthetic(d_data, k * F, nseg, seg0, seed, stream=stream)
        for _ in range(2):
            enc.EncodeBatch(d_data, d_par, nseg, F, stream=stream)
        torch.cuda.synchronize(dev)
        if not timed_alone:
            barrier()
        torch.cuda.synchronize(dev)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record(stream)
        for _ in range(reps):
            enc.EncodeBatch(d_data, d_par, nseg, F, stream=stream)
        b.record(stream)
        torch.cuda.synchronize(dev)
        if not timed_alone:
            barrier()
        host_ms = (time.perf_counter() - t0) * 1e3 / reps
        ev_ms = a.elapsed_time(b) / reps
        RES["hbm_used_after_t1_GiB" if timed_alone else "hbm_used_after_shards_GiB"] = \
            hbm_used_gib(dev)
        rows = sorted({0, 1, nseg // 3, nseg // 2, (2 * nseg) // 3, nseg - 2, nseg - 1} &
                      set(range(nseg)))
        ok = oracle_sample_check(d_data, d_par, rows, seg0, k, m, F, seed)
        del d_data, d_par
        torch.cuda.empty_cache()
        return ev_ms, host_ms, ok, len(rows)

    out = {"workload": f"64 GiB file = {total} x 16 MiB segments, RS({k},{m}), F = 8 MiB, "
                       f"contiguous shard of {total // world} segments per GPU (one batched "
                       f"encode launch per GPU per pass)",
           "segments_total": total, "file_bytes": total * k * F,
           "algorithmic_bytes_per_pass": total * per_seg, "n_gpus": world, "reps": reps,
           "scaling": "strong (fixed 64 GiB file)"}
    # T1: the whole file on one GPU (rank 0), the other ranks waiting
    t1 = encode_pass(0, total, True) if rank == 0 else None
    barrier()
    # T_N: every rank its contiguous shard (the general split also covers N not dividing 4096)
    s0, s1 = total * rank // world, total * (rank + 1) // world
    if world == 1:
        tn = t1
    else:
        tn = encode_pass(s0, s1 - s0, False)
    mine_ok = tn is not None and tn[2]
    vals = reduce_max([tn[0] if tn else float("inf"), tn[1] if tn else float("inf"),
                       0.0 if mine_ok else 1.0])
    enc.close()
    if t1 is not None:
        out.update({"t1_ms": round(t1[0], 4), "t1_host_ms": round(t1[1], 4),
                    "t1_GBps": round(total * per_seg / (t1[0] * 1e-3) / GB, 1),
                    "t1_segments_checked": t1[3], "t1_bit_exact_sampled": t1[2]})
    elif rank == 0:
        out["t1_skipped"] = "not enough free HBM for the whole file on one GPU"
    if vals[0] == float("inf"):
        out["error"] = "a rank could not hold its shard"
        return out
    tn_ms, tn_host_ms, bad = vals
    out.update({"tN_ms": round(tn_ms, 4), "tN_host_ms": round(tn_host_ms, 4),
                "whole_file_GBps": round(total * per_seg / (tn_ms * 1e-3) / GB, 1),
                "per_gpu_GBps": round(total * per_seg / (tn_ms * 1e-3) / GB / world, 1),
                "bit_exact_sampled": not bad and (t1 is None or t1[2]),
                "segments_checked_per_rank": tn[3],
                "checker": "C oracle (oracle/rs_oracle.c) on sampled segments of every shard, "
                           "after the timed passes"})
    # HBM bytes of the whole-file launch from the PMC passes (tools/r05_pmc_c4.sh)
    tr = load_traffic("c4", total * per_seg, "k_ct<EncCT<2, 1>>")
    if tr is not None:
        out["t1_traffic"] = {"bytes_per_launch": tr,
                             "over_algorithmic": round(tr / (total * per_seg), 6),
                             "source": traffic_source("c4")}
    if t1 is not None:
        out["efficiency"] = round(t1[0] / (world * tn_ms), 4)
        out["efficiency_basis"] = "T1 / (N x T_N), HIP-event times per pass, T_N max over ranks"
    if shared and world > 1:
        out["note"] = ("ranks share one GPU (CESS_DEVICE rehearsal): T_N and the efficiency "
                       "measure contention on one device, not scaling")
    return out


def host_e2e_leg(dev, local: int, world: int, rank: int, backend: str,
                 gib_per_rank: int = 8, stream_files: int = 4,
                 stream_segments: int = 1000, reps: int = 5) -> dict:
    """The host-resident path at every N (PCIe-inclusive; never `value`): every rank streams its
    own synthetic in-memory file (`gib_per_rank` GiB of 16 MiB segments, RS(2,1)) through
    libcessec's C pipeline (cec_pipeline_*: pinned host ring, H2D / encode / D2H on three HIP
    streams, the north_star's pinned hipMemcpyAsync multi-buffering): without hashing, then
    emitting every SegmentList record (c-pallets/file-bank/src/types.rs:13-16) with the hashes on
    the GPU hash queue, on 16 host SHA-256 threads (cec_sha256_host: AVX-512 16-lane / SHA-NI
    multi-chain), and hybrid (segment chains on the host, the other fragments on the GPU queue,
    the last batches on the host: the placement encode_file_records and the CLI use). Each
    placement's pipeline is created once and warmed up outside the timed run (a long-lived
    uploader pins its ring once). records_stream: `stream_files` files of `stream_segments`
    segments (SegmentCount = 1000, runtime/src/lib.rs:1026: the largest declarable file) back to
    back through one hybrid session in one run, records per file (each file is the rank's buffer
    read as pieces, so no second copy is held); three such runs, the median reported. Segments are sharded per GPU with no collective.
    Whole-node rate = all ranks' file bytes / the max over ranks of the run time (barrier to
    barrier). Sampled records are checked afterwards with hashlib and the C oracle, and every
    placement's records against the GPU-hashed ones."""
    import hashlib
    import torch
    import torch.distributed as dist
    import cess_amd
    from cess_amd.pipeline import Pipeline, RecordsSession
    k, m, F = 2, 1, 8 * MiB
    seg_bytes = k * F
    nseg = gib_per_rank * (1 << 30) // seg_bytes
    seed = SEED0 + 9
    seg0 = rank * nseg
    # the rank's file: the counter generator on the GPU, copied out 1 GiB at a time
    buf = np.empty(nseg * seg_bytes, np.uint8)
    piece = 64
    d = torch.empty((piece, seg_bytes), dtype=torch.uint8, device=dev)
    hb = torch.from_numpy(buf)
    for s in range(0, nseg, piece):
        n = min(piece, nseg - s)
        cess_amd.fill_synthetic(d, seg_bytes, n, seg0 + s, seed)
        hb[s * seg_bytes:(s + n) * seg_bytes].copy_(d[:n].reshape(-1))
    del d
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()

    def barrier():
        if world > 1:
            dist.barrier()

    def reduce_max(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0])

    def rate(t, n_bytes=nseg * seg_bytes):
        return {"node_GBps": round(world * n_bytes / t / GB, 2),
                "per_gpu_GBps": round(n_bytes / t / GB, 2)}

    out = {"workload": f"{gib_per_rank} GiB in-memory file per GPU ({nseg} x 16 MiB segments, "
                       f"RS(2,1)) through the C pipeline (cec_pipeline: 3 pinned 1 GiB host "
                       f"batches, H2D / encode / D2H streams)",
           "file_bytes_per_gpu": nseg * seg_bytes, "n_gpus": world,
           "basis": "file bytes of all ranks / max over ranks of the run (barrier to barrier); "
                    "PCIe Gen5 x16 = 63 GB/s per direction per GPU; pipelines created and warmed "
                    "up before the timed runs; seconds = the median of `runs_s`; cpu_s_runs / "
                    "cpu_s = rank 0's process CPU seconds per run (every thread: readers, host "
                    "SHA-256 pool)"}
    import resource

    def cpu_s() -> float:  # this process's CPU time, every thread (readers, host SHA pool)
        r = resource.getrusage(resource.RUSAGE_SELF)
        return r.ru_utime + r.ru_stime

    cpu_runs = {}

    def timed_runs(run, key=None):
        """`reps` timed runs, each barrier to barrier and max over ranks; (median s, all s,
        last result). With `key`, rank 0's CPU seconds per run go to cpu_runs[key]."""
        ts, cs, res = [], [], None
        for _ in range(reps):
            barrier()
            c0 = cpu_s()
            t0 = time.perf_counter()
            res = run()
            dt = time.perf_counter() - t0
            cs.append(round(cpu_s() - c0, 3))
            ts.append(reduce_max(dt))
        if key:
            cpu_runs[key] = cs
        return sorted(ts)[len(ts) // 2], [round(t, 4) for t in ts], res

    # ranks sharing one GPU (the CESS_DEVICE rehearsal) split its HBM: the hash windows shrink
    # with the world (every pipeline also fits its window to free HBM when it is created)
    shared = "CESS_DEVICE" in os.environ and world > 1
    gpu_window = max(2, 32 // world) if shared else 32
    hybrid_window = max(2, 32 // world) if shared else 0
    if shared:
        out["shared_gpu_windows"] = {"gpu": gpu_window, "hybrid": hybrid_window}
    recs = {}
    enc = cess_amd.New(k, m, device=local)
    for name, hashing in (("no_hash", False), ("segment_lists", True)):
        with Pipeline(enc, F, batch_segments=64, depth=3, hash=hashing, window=gpu_window) as p:
            p.run(buf[:64 * seg_bytes])  # warm-up: pinned ring, device slots, hash queue
            on_rec = (lambda s, sh, fl: recs.__setitem__(s, (sh, fl))) if hashing else None
            t, runs, st = timed_runs(lambda: p.run(buf, on_record=on_rec), name)
        out[name] = {"seconds": round(t, 4), "runs_s": runs, "segments": int(st.segments),
                     "cpu_s_runs": cpu_runs[name], **rate(t)}
        if hashing:
            out[name]["hash_on"] = "gpu"
    enc.close()

    def same(rec) -> bool:
        return len(rec.segments) == nseg and all(
            (rec.segments[s].hash, list(rec.segments[s].fragment_list)) ==
            (recs[s][0], list(recs[s][1])) for s in range(nseg) if s in recs)

    # the same records hashed on host threads and hybrid (long-lived sessions)
    lib = cess_amd._lib.load()
    for name, mode in (("segment_lists_host_sha", "host"), ("segment_lists_hybrid", "hybrid")):
        with RecordsSession(k, m, seg_bytes, local, mode, batch_segments=64,
                            host_threads=16, window=hybrid_window) as ses:
            ses.encode(buf[:64 * seg_bytes])  # warm-up
            t, runs, (rec, st) = timed_runs(lambda: ses.encode(buf), name)
            info = ses.pipe.info()
            leg = {"seconds": round(t, 4), "runs_s": runs, "segments": len(rec.segments),
                   "cpu_s_runs": cpu_runs[name],
                   "hash_threads": 16,
                   "host_sha_form": {0: "scalar", 1: "sha-ni x1", 2: "sha-ni x2",
                                     3: "sha-ni x4", 4: "avx-512 x16"}.get(
                                         lib.cec_host_sha_form(), "?"),
                   "window": info["window"], "depth": info["depth"]}
            leg["records_equal_gpu_hashed"] = bool(not reduce_max(0.0 if same(rec) else 1.0))
            if mode == "hybrid" and stream_files:
                # records_stream: SegmentCount-size files back to back in one run
                per = stream_segments * seg_bytes
                pieces, left = [], per
                while left:
                    take = min(left, buf.size)
                    pieces.append(buf[:take])
                    left -= take
                # three runs (the rate varies a few per cent from run to run); the median's
                # seconds, file completion times and CPU seconds are reported
                sruns, sok = [], True
                for _ in range(3):
                    done_t = []
                    barrier()
                    c1 = cpu_s()
                    t1 = time.perf_counter()
                    srecs, sst = ses.encode_many(
                        [pieces] * stream_files,
                        on_file=lambda f, r, fs: done_t.append(time.perf_counter() - t1))
                    ts = time.perf_counter() - t1
                    cs = round(cpu_s() - c1, 3)
                    barrier()
                    sok &= all(len(r.segments) == stream_segments for r in srecs)
                    for r in srecs:  # segment s of a stream file is buffer segment s % nseg
                        for s in sorted({0, nseg - 1, nseg, stream_segments - 1}):
                            want = recs.get(s % nseg)
                            sok &= want is not None and (r.segments[s].hash, list(
                                r.segments[s].fragment_list)) == (want[0], list(want[1]))
                    sruns.append((reduce_max(ts), cs, [round(x, 3) for x in done_t]))
                tsm, cs, done_med = sorted(sruns)[1]
                out["records_stream"] = {
                    "files": stream_files, "segments_per_file": stream_segments,
                    "file_bytes": per, "seconds": round(tsm, 4),
                    "runs_s": [round(r[0], 4) for r in sruns],
                    "file_done_s": done_med, "cpu_s": cs,
                    "cpu_s_runs": [r[1] for r in sruns],
                    **rate(tsm, stream_files * per),
                    "records_per_file": True, "hash_on": "hybrid",
                    "records_equal_gpu_hashed_sampled": bool(not reduce_max(0.0 if sok else 1.0))}
        leg.update(rate(t))
        out[name] = leg
    # checker: sampled records against hashlib over the file bytes and the C oracle's parity
    from oracle.c_oracle import load_c_oracle
    orc = load_c_oracle()
    ok = len(recs) == nseg
    for s in sorted({0, nseg // 2, nseg - 1}):
        seg = buf[s * seg_bytes:(s + 1) * seg_bytes]
        par = np.empty(F, np.uint8)
        orc.orc_encode_batch(k, m, seg.ctypes.data, par.ctypes.data, 1, F, 1, 1)
        want_seg = hashlib.sha256(seg).hexdigest().encode()
        want = [hashlib.sha256(seg[:F]).hexdigest().encode(),
                hashlib.sha256(seg[F:]).hexdigest().encode(),
                hashlib.sha256(par).hexdigest().encode()]
        got = recs.get(s)
        ok &= got is not None and got[0] == want_seg and list(got[1]) == want
    bad = reduce_max(0.0 if ok else 1.0)
    out["records_match_hashlib_and_oracle"] = not bad
    out["records_checked_per_gpu"] = 3
    RES["hbm_used_in_host_e2e_GiB"] = hbm_used_gib(dev)
    del buf
    return out


def guarded(leg, *a) -> dict:
    """Run one `extra` leg; an exception becomes {"error": ...} in the line instead of costing
    the whole line (line_problems still flags the leg)."""
    try:
        return leg(*a)
    except Exception as e:  # noqa: BLE001 - reported in the line
        import torch
        torch.cuda.empty_cache()
        return {"error": f"{type(e).__name__}: {e}"[:400]}


def line_problems(out: dict) -> list:
    """What a bench line lacks against the driver's contract and VERDICT's asks (empty = none):
    the contract keys, `roofline` and `cpu_baseline` at every N (at N > 1 on the CPU share of the
    GPUs held), and for the default config: config 4's 64 GiB strong-scaling encode (T_N, T1,
    efficiency, sampled segments bit-exact) at every N; at N = 1 the config-5 step with checked digests and
    the wide-code legs with their cold means; at N > 1 both degraded-read transports (the torch
    group and libcessec's own RCCL communicator, or the reason it could not form) bit-exact."""
    bad = []
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                "roofline", "cpu_baseline"):
        if key not in out:
            bad.append(f"missing {key}")
    rl = out.get("roofline") or {}
    for key in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        if key not in rl:
            bad.append(f"roofline lacks {key}")
    cb = out.get("cpu_baseline") or {}
    for key in ("value", "unit", "cores", "kind", "sample"):
        if key not in cb:
            bad.append(f"cpu_baseline lacks {key}")
    n = out.get("n_gpus", 1)
    if cb and cb.get("cores", 0) < min(GPU_BOX_CPU_SHARE * cb.get("gpus_in_use", n),
                                       cb.get("host_cpus_visible") or 1 << 30):
        bad.append("cpu_baseline below the CPU share of the GPUs in use")
    if (out.get("config") or {}).get("baseline_config") != 2 or "extra" not in out:
        return bad
    ex = out["extra"]
    c4 = ex.get("config4") or {}
    if not c4.get("bit_exact_sampled") or not c4.get("tN_ms"):
        bad.append("extra.config4 missing, unmeasured or not bit-exact")
    elif "efficiency" not in c4:
        bad.append("extra.config4 lacks T1 / efficiency")
    e2e = ex.get("host_e2e")
    if e2e is not None and not e2e.get("records_match_hashlib_and_oracle"):
        bad.append("extra.host_e2e records unchecked or wrong")
    for leg in ("segment_lists_host_sha", "segment_lists_hybrid"):
        if e2e is not None and leg in e2e and not e2e[leg].get("records_equal_gpu_hashed"):
            bad.append(f"extra.host_e2e.{leg} records differ from the GPU-hashed ones")
    if e2e is not None and "error" not in e2e and not (e2e.get("records_stream") or {}).get(
            "records_equal_gpu_hashed_sampled"):
        bad.append("extra.host_e2e.records_stream missing or its records wrong")
    if n == 1:
        c5 = ex.get("config5") or {}
        if not c5.get("digests_match_hashlib") or not c5.get("step_GBps"):
            bad.append("extra.config5 missing or its digests unchecked")
        if "error" in (ex.get("wide_code") or {}):
            bad.append(f"extra.wide_code: {ex['wide_code']['error']}")
        for name, leg in (ex.get("wide_code") or {}).items():
            if isinstance(leg, dict) and "ms" in leg and not any(
                    key.startswith("cold_ms") for key in leg):
                bad.append(f"wide_code.{name} lacks its cold mean")
    else:
        legs = {"degraded_gather": ex.get("degraded_gather"),
                "degraded_gather_cabi": ex.get("degraded_gather_cabi")}
        for ename in ("wide_degraded_gather", "wide_degraded_gather_cabi"):
            w = ex.get(ename) or {}
            if "skipped" in w:
                legs[ename] = w
            for xname in ("survivors", "partials"):
                if "skipped" not in w:
                    legs[f"{ename}.{xname}"] = w.get(xname)
        for name, leg in legs.items():
            if not leg:
                bad.append(f"extra.{name} missing")
            elif "skipped" in leg:
                if "cabi" not in name:
                    bad.append(f"extra.{name} skipped")
            elif "error" in leg:
                bad.append(f"extra.{name}: {leg['error']}")
            elif leg.get("bit_exact") is not True:
                bad.append(f"extra.{name} not bit-exact")
    return bad


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed steps (default 10; config 6: 30, past the clock transient a "
                         "VALU-heavy decoder rides over its first ~30 launches, "
                         "profiles/r03/fdd_clock_transient.txt)")
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--variant", type=int, default=-1, help="CT kernel variant (tuning)")
    ap.add_argument("--generic", action="store_true", help="force run-time-coefficient kernel")
    ap.add_argument("--segments", type=int, default=0,
                    help="segments per GPU (default: the config's; config 5 at 1024 = 16 GiB in "
                         "flight, enough fragments to give every SIMD a SHA-256 wave)")
    ap.add_argument("--sha-mode", type=int, default=0, help="0 auto, 1 one wave, 2 two waves")
    ap.add_argument("--window", type=int, default=96,
                    help="config 5: batches hashing at once in the GPU hash queue (96 x 4096 "
                         "fragment chains: 6 one-wave tick workgroups per SIMD; 64 -> 1.74 ms "
                         "per step, 96..192 -> 1.61-1.63)")
    ap.add_argument("--hash-stream", type=int, default=1,
                    help="config 5: 1 = hash queue on a second stream, 0 = after the encode")
    ap.add_argument("--cu-split", type=int, default=0,
                    help="config 5: run the encode on a stream masked to this many CUs (a multiple "
                         "of 8, spread over the XCDs) and the hash ticks on the other CUs")
    ap.add_argument("--prio", type=int, default=0,
                    help="config 5: 1 = encode on a high-priority stream, hashing on a low one")
    ap.add_argument("--tick-pf", type=int, default=0,
                    help="hash-queue tick prefetch depth (1 or 2; 0 = library default)")
    ap.add_argument("--rt-mode", type=int, default=0,
                    help="run-time kernel: 0 Horner over input groups, index-mode XORs (k <= 32), "
                         "1 per-bit masks, 2 Horner with v_mov table reads, 3 bit-plane "
                         "accumulators (<= 4 outputs)")
    ap.add_argument("--fftdec-min", type=int, default=-1,
                    help="RS(32,32) rebuilds of at least this many shards run the FFT-domain "
                         "decoder (CEC_OPT_FFTDEC_MIN; 0 = never; -1 = library default)")
    ap.add_argument("--fftdec-mode", type=int, default=0, choices=[0, 1, 2],
                    help="RS(32,32) rebuilds: 0 = the cost model's pick of the FFT-domain decoders "
                         "and k_rthx (library default), 1 = always the syndrome-row decoder, "
                         "2 = always the formal-derivative decoder (CEC_OPT_FFTDEC_MODE)")
    ap.add_argument("--erasure-run", action="store_true",
                    help="config 6: the erasures of a segment are consecutive shard indices "
                         "(random start, wrapping) instead of random ones")
    ap.add_argument("--cabi-deadline", type=float, default=240.0,
                    help="world > 1: seconds the exchange legs (torch group, then the C-ABI "
                         "cec_dist) may take before the line is printed without the unfinished")
    ap.add_argument("--erasures", type=int, default=0,
                    help="config 6: random erasures per segment (default m)")
    ap.add_argument("--lose-parity", action="store_true",
                    help="config 6: every segment loses exactly its m parity shards (the rebuild "
                         "is the encode)")
    ap.add_argument("--erase", type=int, default=-1,
                    help="config 3: erased fragment index of every segment (-1: seg mod (k+m), "
                         "the BASELINE pattern)")
    ap.add_argument("--events", choices=["step", "region"], default="region",
                    help="HIP events around the timed region (default: the mean time per launch "
                         "over the region, rocprof's average within 0.2%%) or around every step "
                         "(each event pair costs ~7 us of GPU time per step)")
    ap.add_argument("--exchange", choices=["survivors", "partials", "auto"], default="survivors",
                    help="config 4: degraded-read exchange (survivors to the decoder, or partial "
                         "rebuilds from every GPU holding survivors, SURVEY.md §8e)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--sweep", type=str, default="",
                    help="comma list of CT variants: interleaved A/B in one process, prints "
                         "median launch ms per variant and exits")
    args = ap.parse_args()
    if args.warmup is None:
        args.warmup = 30 if args.config == 6 else 10

    if args.config == 1:  # CPU codec alone (the GPU on the same workload beside it)
        print(json.dumps(config1_cpu(args)), flush=True)
        return

    import torch
    # --gpus N without an external launcher: start the N ranks here, before any HIP call
    # (device_count does not initialise the GPU on this image)
    what, val = world_check(args.gpus, os.environ,
                            None if "WORLD_SIZE" in os.environ or args.gpus == 1
                            else torch.cuda.device_count())
    if what == "error":
        print(f"bench.py: {val}", file=sys.stderr, flush=True)
        sys.exit(2)
    if what == "launch":
        sys.exit(launch_ranks(val, sys.argv[1:]))

    import torch.distributed as dist
    import cess_amd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal knobs for a one-GPU box: CESS_DIST_BACKEND=gloo CESS_DEVICE=0 runs several ranks
    # on one GPU. The driver's multi-GPU run uses the defaults (RCCL, one rank per GPU).
    backend = os.environ.get("CESS_DIST_BACKEND", "nccl")
    if "CESS_DEVICE" in os.environ:
        local = int(os.environ["CESS_DEVICE"])
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    k, m, F, nseg_cfg, desc = CONFIGS[args.config]
    if args.config == 6 and args.erasures:
        desc = desc.replace("32 random erasures", f"{args.erasures} random erasures")
    if args.config == 6 and args.erasure_run:
        desc = desc.replace("random erasures", "consecutive erasures")
    if args.segments:
        nseg_cfg = args.segments
        desc = f"{desc} [{args.segments} segments per GPU = {args.segments * k * F / 2**30:g} GiB]"
    nseg = nseg_cfg // world if args.config == 4 else nseg_cfg
    seg0 = rank * nseg
    stream = torch.cuda.current_stream(dev)

    d_data = torch.empty((nseg, k, F), dtype=torch.uint8, device=dev)
    d_par = torch.empty((nseg, m, F), dtype=torch.uint8, device=dev)
    cess_amd.fill_synthetic(d_data, k * F, nseg, seg0, SEED0 + args.config, stream=stream)
    # kernel variants (--variant / --sweep) live in the tuning build of the library only
    tuning = bool(args.sweep) or args.variant != -1
    enc = cess_amd.New(k, m, device=local, tuning=tuning)
    if args.generic:
        enc.set_option(1, 1)
    if tuning:
        enc.set_option(2, args.variant)
    enc.set_option(3, args.sha_mode)
    enc.set_option(4, args.rt_mode)
    if args.fftdec_min >= 0:
        enc.set_option(7, args.fftdec_min)
    enc.set_option(8, args.fftdec_mode)
    enc.EncodeBatch(d_data, d_par, nseg, F, stream=stream)  # valid parity for config 3

    present = None
    if args.config == 3:
        present = np.ones((nseg, k + m), np.uint8)
        lost = ((seg0 + np.arange(nseg)) % (k + m) if args.erase < 0
                else np.full(nseg, args.erase))
        present[np.arange(nseg), lost] = 0
    elif args.config in (6, 7):
        ne = (args.erasures or m) if args.config == 6 else 1
        present = erasure_patterns(k, m, nseg, ne, seed=seg0 + args.config,
                                   lose_parity=args.lose_parity and args.config == 6,
                                   run=args.erasure_run and args.config == 6)
    d_hex = None
    gather = None
    if args.config == 4:
        # the degraded-read gather of 64 segments per rank runs inside every step
        gather = degraded_gather(enc, k, m, F, world, rank, dev, 64, args.exchange)
    if args.config == 5:
        W = max(1, args.window)
        # --hash-stream 1: hash queue on its own stream (ticks overlap the next encode);
        # 0: one stream, encode then tick (the tick keeps the whole chip)
        if args.cu_split:
            # disjoint CU sets: the HBM-bound encode and the VALU-bound ticks side by side
            torch.cuda.synchronize(dev)
            stream, sha_stream = cu_split_streams(args.cu_split, dev)
        elif args.prio:
            # the encode's waves are dispatched ahead of the tick's as CUs free up: the HBM-bound
            # encode and the VALU-bound ticks share the chip instead of taking turns
            torch.cuda.synchronize(dev)  # inputs were produced on the default stream
            stream = torch.cuda.Stream(dev, priority=-1)
            sha_stream = torch.cuda.Stream(dev, priority=0)
        else:
            if os.environ.get("CESS_C5_STREAM") == "new":  # (the queue-collision A/B knob, see
                # config5_leg; the standalone process has too few streams to collide)
                torch.cuda.synchronize(dev)
                stream = torch.cuda.Stream(dev)
            sha_stream = torch.cuda.Stream(dev) if args.hash_stream else stream
        pipe = HashPipeline(enc, d_data, d_par, nseg, F, dev, local, stream, sha_stream, W,
                            args.tick_pf)
        d_hex, tick_blocks = pipe.pipe_hex[0], pipe.tick_blocks

    def step():
        if args.config in (3, 6, 7):
            enc.ReconstructBatch(d_data, d_par, nseg, F, present, stream=stream)
        elif args.config == 5:
            pipe.step()
        elif args.config == 4:
            enc.EncodeBatch(d_data, d_par, nseg, F, stream=stream)
            gather[0]()
        else:
            enc.EncodeBatch(d_data, d_par, nseg, F, stream=stream)

    def drain():
        if args.config == 5:
            pipe.drain()

    def step_codec():  # the codec kernel alone (config 5's step also hashes)
        if args.config in (3, 6, 7):
            enc.ReconstructBatch(d_data, d_par, nseg, F, present, stream=stream)
        else:
            enc.EncodeBatch(d_data, d_par, nseg, F, stream=stream)

    if args.sweep:
        # forms alternate launch by launch in one process: a screen, not a verdict — forms whose
        # power or LDS use differ can come out a few per cent apart here and equal one per process
        # (profiles/r04/swz_standalone_runs.jsonl); confirm with --variant, one form per process
        step = step_codec  # noqa: F811
        variants = [int(v) for v in args.sweep.split(",")]
        times = {v: [] for v in variants}
        for _ in range(args.warmup):
            step()
        for rnd in range(args.steps):
            for v in variants:
                enc.set_option(2, v)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                step()
                a.record(stream)
                step()
                step()
                b.record(stream)
                torch.cuda.synchronize(dev)
                times[v].append(a.elapsed_time(b) / 2)
        per_seg = (k + (1 if args.config == 7 else m)) * F
        for v in variants:
            med = float(np.median(times[v]))
            print(json.dumps({"config": args.config, "variant": v, "median_ms": round(med, 4),
                              "min_ms": round(float(np.min(times[v])), 4),
                              "GBps": round(nseg * per_seg / med / 1e6, 1)}), flush=True)
        return

    fd_seg0 = enc.stat(4)  # segments the FFT-domain decoders rebuilt before this run
    fdd_seg0 = enc.stat(5)  # of those, the formal-derivative decoder
    for _ in range(args.warmup):
        step()
    drain()  # the timed region starts with an empty hash window and ends with it drained
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)

    # --events step: an event pair around every step (mean of the per-launch durations);
    # region: one pair around the whole timed region (mean time per launch, gaps included)
    per_step = args.events == "step"
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps if per_step else 1)]
    t0 = time.perf_counter()
    if not per_step:
        ev[0][0].record(stream)
    for i in range(args.steps):
        if per_step:
            ev[i][0].record(stream)
        step()
        if per_step:
            ev[i][1].record(stream)
    if not per_step:
        ev[0][1].record(stream)
    drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    fd_seg1 = enc.stat(4)
    fdd_seg1 = enc.stat(5)

    launch_ms = (float(np.mean([a.elapsed_time(b) for a, b in ev])) if per_step
                 else ev[0][0].elapsed_time(ev[0][1]) / args.steps)
    if world > 1:
        t = torch.tensor([elapsed, launch_ms], dtype=torch.float64,
                         device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, launch_ms = float(t[0]), float(t[1])

    # algorithmic bytes per segment: read k*F, write m*F (encode) or one erased fragment each
    # (config 7 repairs one fragment: (k+1)*F)
    per_seg = (k + (1 if args.config == 7 else
                    (args.erasures or m) if args.config == 6 else m)) * F
    bytes_step_gpu = nseg * per_seg
    value = world * bytes_step_gpu * args.steps / elapsed / GB
    achieved = bytes_step_gpu / (launch_ms * 1e-3) / GB

    def timed(fn, reps=5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(reps):
            fn()
        b.record(stream)
        torch.cuda.synchronize(dev)
        return a.elapsed_time(b) / reps

    sha_note = None
    if args.config == 4:
        # the step holds encode + the degraded-read gather; the roofline is the encode kernel's
        launch_ms = timed(lambda: enc.EncodeBatch(d_data, d_par, nseg, F, stream=stream), 10)
        achieved = bytes_step_gpu / (launch_ms * 1e-3) / GB
    if args.config == 5:
        # the step holds encode + SHA-256; time each kernel alone for the roofline
        enc_ms = timed(lambda: enc.EncodeBatch(d_data, d_par, nseg, F, stream=stream), 20)
        sha_ms = timed(lambda: enc.Sha256Batch(d_data, d_par, nseg, F, d_hex, stream=stream), 3)
        achieved = bytes_step_gpu / (enc_ms * 1e-3) / GB
        launch_ms = enc_ms  # the step's events also hold the pipeline's wait on the hash stream
        sha_note = {"one_batch_sha256_ms": round(sha_ms, 3), "encode_ms": round(enc_ms, 4),
                    "one_batch_sha256_GBps": round(bytes_step_gpu / (sha_ms * 1e-3) / GB, 2),
                    "streams": nseg * (k + m), "sha_mode": args.sha_mode,
                    "window": W, "chains_in_flight": W * nseg * (k + m),
                    "tick_blocks": tick_blocks,
                    "pipeline": f"GPU hash queue: batch i's {nseg * (k + m)} fragment chains "
                                f"hash over ticks i..i+{W - 1} (one tick per step, "
                                + ("on a second stream" if args.hash_stream else
                                   "after the step's encode") +
                                "); the timed region ends with the window drained",
                    "note": "SHA-256 is one sequential chain per fragment: bounded by streams x "
                            "per-wave issue rate, reported apart from the HBM roofline"}
        try:  # measured HBM bytes of a whole step (both kernels), profiles/traffic_c5_step.json
            with open(os.path.join(ROOT, "profiles", "traffic_c5_step.json")) as f:
                st = json.load(f)
            sha_note["step_traffic"] = {"bytes": st["step_bytes"],
                                        "over_algorithmic": round(st["step_over_algorithmic"], 3),
                                        "note": "encode 1x + the ticks' re-read of every fragment"}
        except (OSError, ValueError, KeyError):
            pass
        slots = load_valu_slots("c5")
        if slots:
            # the step's hashing against the VALU issue roofline: every block of every fragment
            # chain costs the tick loop's issue slots on one lane
            blocks = nseg * (k + m) * cess_amd.sha256_blocks(F) * args.steps
            ach = blocks * slots["issue_slots_per_block"] / elapsed / 1e12
            sha_note["roofline"] = {
                "bound": "valu", "kernel": "k_sha256_tick1", "achieved": round(ach, 2),
                "peak": round(VALU_PEAK_TLANE, 2), "unit": "T lane-slots/s",
                "frac": round(ach / VALU_PEAK_TLANE, 4),
                "issue_slots_per_block": slots["issue_slots_per_block"],
                "valu_instr_per_block": slots["valu_instr_per_block"],
                "basis": "whole step (hash ticks share the chip with the encode); peak at 2.4 GHz"}

    # share of the timed rebuilds the library sent to the FFT-domain decoder (CEC_STAT 4)
    fd_frac = fdd_frac = None
    if args.config == 6:
        fd_frac = (fd_seg1 - fd_seg0) / max(1, nseg * (args.steps + args.warmup))
        fd_frac = round(min(1.0, fd_frac), 4)
        fdd_frac = round(min(1.0, (fdd_seg1 - fdd_seg0) / max(1, nseg * (args.steps + args.warmup))), 4)
    tag = f"c{args.config}"
    kernel_name = kernel_label(args.config, fd_frac, args.erasures or m, args.generic,
                               args.rt_mode, k, fdd_frac)
    traffic = load_traffic(tag, bytes_step_gpu, kernel_name)
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak" if args.config != 4 else "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 counter generator, generated in HBM)",
        "config": {"workload": desc, "baseline_config": args.config, "k": k, "m": m,
                   "fragment_bytes": F, "segments_per_gpu": nseg,
                   "bytes_per_step_per_gpu": bytes_step_gpu, "parallelism": f"shard{world}",
                   "kernel": kernel_name},
        "per_gpu_GBps": round(value / world, 2),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": traffic,
                     "traffic_source": traffic_source(tag) if traffic is not None else None,
                     "launch_ms": round(launch_ms, 4),
                     "algorithmic_bytes_per_launch": bytes_step_gpu},
    }
    if sha_note:
        out["sha256"] = sha_note

    def gather_leg(run_verify_plan, reps=5, code=(k, F)) -> dict:
        """Time the degraded read (exchange over the process group + rebuild) alone,
        synchronised per rep, max over ranks; verify the rebuilt fragments."""
        run, verify, plan, close = run_verify_plan
        fb = code[1]
        times = []
        res = None
        for _ in range(reps + 1):
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            res = run()
            torch.cuda.synchronize(dev)
            if world > 1:
                dist.barrier()
            times.append(time.perf_counter() - t0)
        t = float(np.median(times[1:]))
        ok = verify(res)
        v = torch.tensor([t, 0.0 if ok else 1.0], dtype=torch.float64,
                         device=dev if (world == 1 or backend == "nccl") else "cpu")
        if world > 1:
            dist.all_reduce(v, op=dist.ReduceOp.MAX)
        t, bad = float(v[0]), bool(v[1])
        close()
        nrebuilt = len(plan.lost)
        kk = code[0]
        return {"segments": nrebuilt, "lost_per_segment": 1,
                "exchange": ("partials" if plan.partial and not plan.moves else
                             "mixed" if plan.partial else "survivors"),
                "placement": "fragment f of segment s on GPU (s + f) mod N "
                             "(c-pallets/file-bank/src/functions.rs:187-283)",
                "gather_bytes": plan.bytes_moved, "seconds": round(t, 5),
                "gather_GBps": round(plan.bytes_moved / t / GB, 2) if plan.bytes_moved else None,
                "rebuilt_GBps": round(nrebuilt * (kk + 1) * fb / t / GB, 2),
                "xgmi_GBps_per_link": 153,
                "backend": (backend if world > 1 else "local (one GPU: no bytes move)"),
                "bit_exact": not bad}

    if not args.no_extra and args.config == 2:
        # BASELINE config 4's strong-scaling encode (64 GiB over the N GPUs, T1 on one GPU beside
        # it) at every N: the driver only ever runs the default command
        out.setdefault("extra", {})["config4"] = guarded(config4_leg, dev, local, world, rank,
                                                         backend)
        # the host-resident path at every N: a file per GPU through the C pipeline
        # (PCIe-inclusive; the north_star's pinned double-buffering, sharded per GPU)
        out["extra"]["host_e2e"] = guarded(host_e2e_leg, dev, local, world, rank, backend)

    exchange_pending = cabi_pending = False
    if args.config == 4:
        out["degraded_gather"] = gather_leg(gather)
    elif world > 1 and not args.no_extra and args.config == 2:
        # config 4's exchange step measured in the default (scaling) run as well, through both
        # transports: the torch.distributed group and libcessec's own RCCL communicator (the C
        # ABI a Go / Rust host uses), on the same placement and lost list. Both run last, under
        # one watchdog (cabi_legs below): they are the line's only cross-GPU collectives
        ex_out = out.setdefault("extra", {})
        exchange_pending = True
        if "CESS_DEVICE" in os.environ:
            # ranks sharing one GPU (the one-GPU rehearsal): RCCL refuses a communicator with
            # two ranks on one device ("Duplicate GPU detected"), so the C-ABI group cannot form
            why = ("skipped: the ranks share one GPU (CESS_DEVICE rehearsal) and RCCL refuses "
                   "two ranks on one device; runs on a multi-GPU node")
            ex_out["degraded_gather_cabi"] = {"skipped": why}
            ex_out["wide_degraded_gather_cabi"] = {"skipped": why}
        else:
            cabi_pending = True  # run last, under a deadline (cabi_legs below)

    if not args.no_extra and args.config == 2:
        # decode rate in the same process (BASELINE config 3 workload, same bytes)
        pres = np.ones((nseg, k + m), np.uint8)
        pres[np.arange(nseg), (seg0 + np.arange(nseg)) % (k + m)] = 0
        for _ in range(3):
            enc.ReconstructBatch(d_data, d_par, nseg, F, pres, stream=stream)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(20):
            enc.ReconstructBatch(d_data, d_par, nseg, F, pres, stream=stream)
        b.record(stream)
        torch.cuda.synchronize(dev)
        dms = a.elapsed_time(b) / 20
        out.setdefault("extra", {}).update(
            {"reconstruct_GBps_per_gpu": round(bytes_step_gpu / (dms * 1e-3) / GB, 2),
             "reconstruct_ms": round(dms, 4)})
        if world == 1:
            # one-GPU legs (at N > 1 every rank would repeat them, and config 5's hash window
            # holds ~100 GiB of parity per rank: ranks sharing a GPU in the rehearsal do not fit).
            # The wide code (BASELINE config 5's RS(32,32), 16 MiB segments: F = 512 KiB), so the
            # driver's own line carries its encode, restoral and multi-erasure rebuild rates
            out["extra"]["wide_code"] = guarded(wide_code_legs, dev, local, stream)
            # BASELINE config 5 (RS(32,32) encode + SHA-256 of every fragment) as the driver runs
            out["extra"]["config5"] = guarded(config5_leg, dev, local)
        # the measured-copy ceiling beside the spec peak: a device-to-device copy
        # of the same 1 GiB data batch (HIP's blit kernel), read + write bytes per copy
        src = d_data.view(-1)
        dst = torch.empty_like(src)
        for _ in range(3):
            dst.copy_(src)
        a.record(stream)
        for _ in range(20):
            dst.copy_(src)
        b.record(stream)
        torch.cuda.synchronize(dev)
        cms = a.elapsed_time(b) / 20
        out["roofline"]["copy_ceiling"] = {
            "guide_float4_copy_GBps": 6290.0,
            "hipmemcpy_d2d_GBps": round(2 * src.numel() / (cms * 1e-3) / GB, 1),
            "what": "measured-copy ceilings beside the 8 TB/s spec: the guide's float4 copy "
                    "kernel (MI355X_MICROARCH.md) and, measured here, a D2D copy of the 1 GiB data "
                    "batch through the HIP runtime (torch copy_), read + write bytes / time"}
        del dst

    if rank == 0 and not args.no_cpu_baseline:
        # after the GPU region; at N > 1 on rank 0 alone, on the CPU share of the GPUs the job
        # holds (16 per GPU: the whole node's at N = 8; ranks sharing one GPU hold one)
        gpus_held = 1 if "CESS_DEVICE" in os.environ else world
        out["cpu_baseline"] = cpu_baseline(k, m, F, args.cpu_seconds, gpus_held)
        out["cpu_baseline"]["node_GBps_gpu"] = out["value"]
        if args.config == 5:
            out["cpu_baseline"]["sha256"] = cpu_sha256(k, m, F, args.cpu_seconds / 2)
        elif args.config == 2 and world == 1 and not args.no_extra:
            # the default line carries config 5's step (extra.config5): its hashing's CPU
            # baseline beside it (OpenSSL SHA-256, SHA-NI where the host has it)
            wk, wm, wF = CONFIGS[5][:3]
            out["cpu_baseline"]["sha256"] = cpu_sha256(wk, wm, wF, args.cpu_seconds / 2)

    if not args.no_extra and args.config == 2:
        res = resources(dev, world, rank, T_START)
        if rank == 0:
            out.setdefault("extra", {})["resources"] = res

    if exchange_pending:
        cabi_legs(out["extra"], gather_leg, degraded_gather, enc, (k, m, F), world, rank, dev,
                  args.cabi_deadline, lambda: print(json.dumps(out), flush=True) if rank == 0
                  else None, torch_legs=True, cabi=cabi_pending)

    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
