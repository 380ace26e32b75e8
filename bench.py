#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: "RS encode/decode GB/s per GPU and whole node; % of HBM
roofline", on the CESS segment -> fragment codec (libcessec, HIP kernels for gfx950).

Default workload = BASELINE.json configs[1]: batched encode of 1 GiB of synthetic 16 MiB
segments per GPU, RS(k=2, m=1), 8 MiB fragments, device-resident (inputs already in HBM when
the timed region starts). A "step" is one batched encode launch over the rank's 64 segments.
Bytes counted per segment = (k+m) * F (k fragments read, m written).

    python bench.py [--gpus N --steps K --warmup W] [--config 2|3|4|5]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one rank per GPU, weak scaling)

Rank 0 prints one JSON line. `roofline` is the dominant kernel's algorithmic bytes per launch /
its average launch time (HIP events on the launch stream); `cpu_baseline` times the C oracle
(oracle/rs_oracle.c, kind "port": the reference ships no codec) on a bounded sample on rank 0.
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

MiB = 1 << 20
GB = 1e9
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
METRIC = "RS encode/decode GB/s per GPU and whole node; % of HBM roofline"
SEED0 = 0xCE550000

CONFIGS = {
    # id: (k, m, fragment bytes, segments per GPU, description)
    2: (2, 1, 8 * MiB, 64, "batched RS(2,1) encode of 1 GiB of 16 MiB segments per GPU"),
    3: (2, 1, 8 * MiB, 64, "degraded reconstruct RS(2,1), erased fragment = seg mod 3, 1 GiB"),
    4: (2, 1, 8 * MiB, 4096, "64 GiB file (4096 x 16 MiB segments) encoded, sharded over GPUs"),
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


def cpu_threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))  # a GPU box gives one GPU a 16-CPU share


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(k: int, m: int, F: int, target_s: float) -> dict:
    """Time the C oracle (oracle/rs_oracle.c) on a bounded sample of the same workload."""
    from oracle.c_oracle import load_c_oracle
    orc = load_c_oracle()
    simd = orc.orc_set_simd(-1)
    # same workload shape as the GPU step (1 GiB of segments), larger than the host's LLC
    nseg = max(1, (1 << 30) // (k * F))
    data = np.empty(nseg * k * F, np.uint8)
    par = np.empty(nseg * m * F, np.uint8)
    orc.orc_fill_synthetic(data.ctypes.data, k * F, nseg, 0, SEED0 + 2)
    threads = cpu_threads()
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
                  f"{'AVX2 split-nibble' if simd == 1 else 'scalar table'} C oracle, "
                  f"{threads} threads, {t:.1f} s",
        "value_1thread": round(n1 * per_seg / st / GB, 3),
        "cpu_model": cpu_model(),
    }


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


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--variant", type=int, default=-1, help="CT kernel variant (tuning)")
    ap.add_argument("--generic", action="store_true", help="force run-time-coefficient kernel")
    ap.add_argument("--segments", type=int, default=0,
                    help="segments per GPU (default: the config's; config 5 at 1024 = 16 GiB in "
                         "flight, enough fragments to give every SIMD a SHA-256 wave)")
    ap.add_argument("--sha-mode", type=int, default=0, help="0 auto, 1 one wave, 2 two waves")
    ap.add_argument("--window", type=int, default=64,
                    help="config 5: batches hashing at once in the GPU hash queue")
    ap.add_argument("--hash-stream", type=int, default=1,
                    help="config 5: 1 = hash queue on a second stream, 0 = after the encode")
    ap.add_argument("--tick-pf", type=int, default=0,
                    help="hash-queue tick prefetch depth (1 or 2; 0 = library default)")
    ap.add_argument("--rt-mode", type=int, default=0,
                    help="run-time kernel: 0 Horner over input groups, index-mode XORs (k <= 32), "
                         "1 per-bit masks, 2 Horner with v_mov table reads")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--sweep", type=str, default="",
                    help="comma list of CT variants: interleaved A/B in one process, prints "
                         "median launch ms per variant and exits")
    args = ap.parse_args()

    import torch
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
    enc.EncodeBatch(d_data, d_par, nseg, F, stream=stream)  # valid parity for config 3

    present = None
    if args.config == 3:
        present = np.ones((nseg, k + m), np.uint8)
        present[np.arange(nseg), (seg0 + np.arange(nseg)) % (k + m)] = 0
    elif args.config in (6, 7):
        rng = np.random.default_rng(seg0 + args.config)
        present = np.ones((nseg, k + m), np.uint8)
        ne = m if args.config == 6 else 1
        for s_ in range(nseg):
            present[s_, rng.choice(k + m, size=ne, replace=False)] = 0
    d_hex = None
    if args.config == 5:
        # Windowed pipeline over steps: step i encodes into parity buffer i % W on the launch
        # stream, then (on the hash stream, after the encode) adds the batch's 64 * nseg
        # fragment chains to the GPU hash queue and ticks it once: each tick advances every
        # live chain by ceil(blocks per fragment / W) blocks, so a batch's hashes complete W
        # ticks after its encode and W batches hash together (W x nseg x (k+m) chains in
        # flight). The data batch is read-only and shared; parity and hex are (W+1)-buffered.
        W = max(1, args.window)
        d_hex = torch.empty((nseg, k + m, 64), dtype=torch.uint8, device=dev)
        # W + 1 buffers: the batch a step overwrites completed one tick earlier, so the encode
        # of step i + 1 waits for tick i - 1 and overlaps tick i
        NB = W + 1
        pipe_par = [d_par] + [torch.empty_like(d_par) for _ in range(NB - 1)]
        pipe_hex = [d_hex] + [torch.empty_like(d_hex) for _ in range(NB - 1)]
        # --hash-stream 1: hash queue on its own stream (ticks overlap the next encode);
        # 0: one stream, encode then tick (the tick keeps the whole chip)
        sha_stream = torch.cuda.Stream(dev) if args.hash_stream else stream
        chains = W * nseg * (k + m)
        hq = cess_amd.HashQueue(capacity=1 << max(10, (chains - 1).bit_length()), device=local,
                                stream=sha_stream)
        if args.tick_pf:
            hq.set_option(1, args.tick_pf)
        tick_blocks = -(-cess_amd.sha256_blocks(F) // W)
        ev_enc = [torch.cuda.Event() for _ in range(NB)]
        ev_free = [torch.cuda.Event() for _ in range(NB)]
        pipe_i = [0]

    def step():
        if args.config in (3, 6, 7):
            enc.ReconstructBatch(d_data, d_par, nseg, F, present, stream=stream)
        elif args.config == 5:
            i = pipe_i[0]
            pipe_i[0] += 1
            b = i % NB
            if i >= NB:
                stream.wait_event(ev_free[b])  # batch i - NB's hashes done: buffer b reusable
            enc.EncodeBatch(d_data, pipe_par[b], nseg, F, stream=stream)
            ev_enc[b].record(stream)
            sha_stream.wait_event(ev_enc[b])
            hq.add_fragments(d_data, pipe_par[b], nseg, k, m, F, pipe_hex[b])
            hq.tick(tick_blocks)
            # this tick completed batch i - W + 1, whose buffer step i + 2 takes
            ev_free[(i - W + 1) % NB].record(sha_stream)
        else:
            enc.EncodeBatch(d_data, d_par, nseg, F, stream=stream)

    def drain():
        if args.config == 5:
            hq.finish()
            if sha_stream is not stream:
                stream.wait_stream(sha_stream)

    def step_codec():  # the codec kernel alone (config 5's step also hashes)
        if args.config in (3, 6, 7):
            enc.ReconstructBatch(d_data, d_par, nseg, F, present, stream=stream)
        else:
            enc.EncodeBatch(d_data, d_par, nseg, F, stream=stream)

    if args.sweep:
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

    for _ in range(args.warmup):
        step()
    drain()  # the timed region starts with an empty hash window and ends with it drained
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0

    launch_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if world > 1:
        t = torch.tensor([elapsed, launch_ms], dtype=torch.float64,
                         device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, launch_ms = float(t[0]), float(t[1])

    # algorithmic bytes per segment: read k*F, write m*F (encode) or one erased fragment each
    # (config 7 repairs one fragment: (k+1)*F)
    per_seg = (k + (1 if args.config == 7 else m)) * F
    bytes_step_gpu = nseg * per_seg
    value = world * bytes_step_gpu * args.steps / elapsed / GB
    achieved = bytes_step_gpu / (launch_ms * 1e-3) / GB

    sha_note = None
    if args.config == 5:
        # the step holds encode + SHA-256; time each kernel alone for the roofline
        def timed(fn, reps=5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for _ in range(reps):
                fn()
            b.record(stream)
            torch.cuda.synchronize(dev)
            return a.elapsed_time(b) / reps
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

    tag = f"c{args.config}"
    kernel_name = {2: "k_ct<EncCT<2, 1>>", 3: "k_ct_dec1_mixed21 (Dec1CT<2, 1, e> / EncCT<2, 1> per segment)",
                   4: "k_ct<EncCT<2, 1>>", 5: "k_hg<EncCT<32, 32>, 4>", 6: "k_rthx<8>",
                   7: "k_rthx<8>", 8: "k_rthx<3>"}[args.config]
    if args.generic:
        kernel_name = "k_rthx" if k <= 32 else "k_rt"
    if args.rt_mode and (args.generic or args.config in (6, 7, 8)):
        kernel_name = {1: "k_rt", 2: "k_rth"}[args.rt_mode]
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
                     "traffic": traffic, "launch_ms": round(launch_ms, 4),
                     "algorithmic_bytes_per_launch": bytes_step_gpu},
    }
    if sha_note:
        out["sha256"] = sha_note

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
        out["extra"] = {"reconstruct_GBps_per_gpu": round(bytes_step_gpu / (dms * 1e-3) / GB, 2),
                        "reconstruct_ms": round(dms, 4)}

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(k, m, F, args.cpu_seconds)

    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
