#!/usr/bin/env python3
"""Cross-GPU degraded read (BASELINE config 4's exchange step), one process per GPU.

Fragment f of segment s lives on GPU (s + f) mod G (the miner spread of
c-pallets/file-bank/src/functions.rs:187-283). Every segment loses fragment (s mod n); the k
survivors are gathered on the lost fragment's home GPU with grouped point-to-point send/recv
(RCCL over xGMI; RCCL has no XOR reduction) and the fragment is rebuilt there by libcessec.
With --exchange partials (or auto) the GPUs holding survivors send partial rebuilds instead
(SURVEY.md §8e). Reports exchanged bytes / time, decode time, and checks every rebuilt fragment.

    torchrun --nproc-per-node G tools/degraded_bench.py [--nseg 64] [--frag-mib 8]
        [--data-shards 32 --parity-shards 32 --frag-kib 512] [--exchange survivors|partials|auto]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nseg", type=int, default=64)
    ap.add_argument("--frag-mib", type=int, default=8)
    ap.add_argument("--frag-kib", type=int, default=0, help="fragment size in KiB (overrides MiB)")
    ap.add_argument("--exchange", choices=["survivors", "partials", "auto"], default="auto")
    ap.add_argument("--data-shards", type=int, default=2)
    ap.add_argument("--parity-shards", type=int, default=1)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    import cess_amd
    from cess_amd import distributed as D

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("CESS_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    backend = os.environ.get("CESS_DIST_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    k, m, nseg = args.data_shards, args.parity_shards, args.nseg
    F = args.frag_kib << 10 if args.frag_kib else args.frag_mib << 20
    n = k + m
    enc = cess_amd.New(k, m, device=local)
    # every rank regenerates the codewords deterministically and keeps the fragments it owns
    mine = D.local_fragments(nseg, n, world, rank)
    store = D.FragmentStore({sf: i for i, sf in enumerate(mine)},
                            torch.empty((len(mine), F), dtype=torch.uint8, device=dev))
    seg_d = torch.empty((1, k, F), dtype=torch.uint8, device=dev)
    seg_p = torch.empty((1, m, F), dtype=torch.uint8, device=dev)
    for s in range(nseg):
        cess_amd.fill_synthetic(seg_d, k * F, 1, s, 0xCE550004)
        enc.EncodeBatch(seg_d, seg_p, 1, F)
        for f in range(n):
            if (s, f) in store.slots:
                store.data[store.slots[(s, f)]].copy_(seg_d[0, f] if f < k else seg_p[0, f - k])
    torch.cuda.synchronize()
    lost = {s: [s % n] for s in range(nseg)}
    plan = D.plan_gather(lost, k, m, world, F, exchange=args.exchange)
    times = []
    for _ in range(args.reps + 1):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = D.degraded_read(plan, store, enc, rank)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        times.append(time.perf_counter() - t0)
    t = float(np.median(times[1:]))
    # verify rebuilt fragments against the owner's stored copy regenerated locally
    ok = True
    for (s, f), got in out.items():
        cess_amd.fill_synthetic(seg_d, k * F, 1, s, 0xCE550004)
        enc.EncodeBatch(seg_d, seg_p, 1, F)
        want = seg_d[0, f] if f < k else seg_p[0, f - k]
        ok &= bool(torch.equal(got, want))
    res = torch.tensor([t, 1.0 if ok else 0.0, len(out)], dtype=torch.float64,
                       device=dev if backend == "nccl" else "cpu")
    if world > 1:
        r_max = res.clone()
        dist.all_reduce(r_max, op=dist.ReduceOp.MAX)
        r_min = res.clone()
        dist.all_reduce(r_min, op=dist.ReduceOp.MIN)
        r_sum = res.clone()
        dist.all_reduce(r_sum, op=dist.ReduceOp.SUM)
        t, ok, rebuilt = float(r_max[0]), bool(r_min[1]), int(r_sum[2])
    else:
        rebuilt = len(out)
    if rank == 0:
        print(json.dumps({"degraded_read": True, "gpus": world, "segments": nseg, "k": k, "m": m,
                          "fragment_bytes": F, "rebuilt": rebuilt, "bit_exact": ok,
                          "exchange": args.exchange, "partial_segments": len(plan.partial),
                          "gather_bytes": plan.bytes_moved, "seconds": round(t, 5),
                          "gather_plus_decode_GBps": round(plan.bytes_moved / t / 1e9, 2)
                          if plan.bytes_moved else None,
                          "decoded_GBps": round(nseg * (k + 1) * F / t / 1e9, 2),
                          "backend": backend if world > 1 else "none"}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
