#!/usr/bin/env python3
"""Host-resident pipeline sweep (PCIe-inclusive): an in-memory file through cec_pipeline with
different batch sizes, ring depths and hash windows; one JSON line per setting.

usage: python tools/e2e_sweep.py [--gib 8] [--batches 8,16,32,64] [--depths 3,4]
                                 [--windows 16,32,64]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cess_amd  # noqa: E402
from cess_amd.pipeline import Pipeline  # noqa: E402

MiB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=8)
    ap.add_argument("--batches", default="8,16,32,64")
    ap.add_argument("--depths", default="3,4")
    ap.add_argument("--windows", default="16,32,64")
    args = ap.parse_args()
    k, m, F = 2, 1, 8 * MiB
    seg = k * F
    nseg = args.gib * 1024 // 16
    buf = np.empty(nseg * seg, np.uint8)
    d = torch.empty((64, seg), dtype=torch.uint8, device="cuda")
    hb = torch.from_numpy(buf)
    for s in range(0, nseg, 64):
        n = min(64, nseg - s)
        cess_amd.fill_synthetic(d, seg, n, s, 0xCE550009)
        hb[s * seg:(s + n) * seg].copy_(d[:n].reshape(-1))
    del d
    enc = cess_amd.New(k, m)
    for hashing in (False, True):
        for batch in [int(x) for x in args.batches.split(",")]:
            for depth in [int(x) for x in args.depths.split(",")]:
                for window in ([int(x) for x in args.windows.split(",")] if hashing else (16,)):
                    with Pipeline(enc, F, batch_segments=batch, depth=depth, hash=hashing,
                                  window=window) as p:
                        p.run(buf[:batch * seg])
                        best = None
                        for _ in range(2):
                            t0 = time.perf_counter()
                            p.run(buf, read_threads=8)
                            t = time.perf_counter() - t0
                            best = t if best is None else min(best, t)
                    print(json.dumps({"hash": hashing, "batch_segments": batch, "depth": depth,
                                      "window": window if hashing else None,
                                      "GBps": round(nseg * seg / best / 1e9, 2),
                                      "seconds": round(best, 4), "gib": args.gib}), flush=True)
    enc.close()


if __name__ == "__main__":
    main()
