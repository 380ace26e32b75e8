#!/usr/bin/env python3
"""Host-resident end-to-end rate of the file -> SegmentList pipeline (PCIe-inclusive; never the
bench `value`): a synthetic in-memory file is read through pinned buffers, copied to HBM,
encoded, parity copied back and every segment/fragment hashed (host SHA-NI or GPU SHA-256).

usage: python tools/e2e_bench.py [--gib 2] [--k 2 --m 1] [--hash auto|host|gpu] [--window W]"""
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
    ap.add_argument("--gib", type=float, default=2.0)
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--m", type=int, default=1)
    ap.add_argument("--hash", default="auto")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--window", type=int, default=32, help="GPU hash queue window (batches)")
    args = ap.parse_args()
    from cess_amd.segments import SegmentEncoder
    seg = 16 << 20
    nseg = int(args.gib * (1 << 30)) // seg
    # synthetic file bytes: the codec's own splitmix64 generator on the GPU, copied out in 1 GiB
    # pieces into host memory (the in-memory "file" the pipeline then reads)
    import torch
    import cess_amd
    buf = np.empty(nseg * seg, np.uint8)
    piece = 64
    d = torch.empty(piece * seg, dtype=torch.uint8, device="cuda")
    hb = torch.from_numpy(buf)
    for s0 in range(0, nseg, piece):
        n = min(piece, nseg - s0)
        cess_amd.fill_synthetic(d, seg, n, s0, 0xCE550009)
        hb[s0 * seg:(s0 + n) * seg].copy_(d[:n * seg])
    del d
    se = SegmentEncoder(args.k, args.m, seg, batch_segments=64, hash_on=args.hash,
                        hash_threads=args.threads, window=args.window)
    se.encode_file(buf[: 64 * seg])  # warm-up (allocations, pools)
    t0 = time.perf_counter()
    rec = se.encode_file(buf)  # in-memory file, copied into pinned buffers by 8 threads
    dt = time.perf_counter() - t0
    se.close()
    print(json.dumps({"e2e_GBps_file_bytes": round(nseg * seg / dt / 1e9, 2), "seconds": round(dt, 3),
                      "segments": len(rec.segments), "k": args.k, "m": args.m,
                      "hash_on": se.hash_on, "threads": args.threads,
                      "window": args.window if se.hash_on == "gpu" else None}))


if __name__ == "__main__":
    main()
