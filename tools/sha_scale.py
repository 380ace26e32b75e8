#!/usr/bin/env python3
"""Hash-queue tick throughput vs chains in flight (one MI355X): N chains of `blocks` 64-byte
blocks at `stride` bytes apart, one tick of `blocks` blocks each (the padding block is left for
a second, untimed tick). Prints per-N JSON lines: tick ms, us per block, GB/s hashed.

usage: python tools/sha_scale.py [--blocks 256] [--stride 524288] [--pf 1] [--chains 4096,...]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=256)
    ap.add_argument("--stride", type=int, default=512 * 1024)
    ap.add_argument("--pf", type=int, default=0, help="tick kernel (0 auto, 1/2 two-wave, 3 one-wave)")
    ap.add_argument("--chains", default="4096,16384,32768,65536,98304,131072")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    import cess_amd
    ln = args.blocks * 64
    stride = max(args.stride, ln)
    nmax = max(int(c) for c in args.chains.split(","))
    buf = torch.empty(nmax * stride, dtype=torch.uint8, device="cuda")
    cess_amd.fill_synthetic(buf, stride, nmax, 0, 7)
    st = torch.cuda.Stream()
    with cess_amd.HashQueue(capacity=1 << 10, stream=st) as q:  # warm-up (code load, clocks)
        q.set_option(1, args.pf)
        q.add(buf, 1024, 1, stride, stride, ln, None)
        q.finish()
        st.synchronize()
    for n in [int(c) for c in args.chains.split(",")]:
        q = cess_amd.HashQueue(capacity=1 << max(10, (n - 1).bit_length()), stream=st)
        q.set_option(1, args.pf)  # CEC_HQOPT_TICK
        times = []
        for _ in range(args.reps):
            q.add(buf, n, 1, stride, stride, ln, None)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            q.tick(args.blocks)
            b.record(st)
            q.finish()
            st.synchronize()
            times.append(a.elapsed_time(b))
        q.close()
        ms = min(times)
        print(json.dumps({"chains": n, "blocks": args.blocks, "pf": args.pf, "stride": stride,
                          "tick_ms": round(ms, 4),
                          "us_per_block": round(ms * 1e3 / args.blocks, 3),
                          "GBps": round(n * ln / (ms * 1e-3) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
