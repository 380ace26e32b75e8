#!/usr/bin/env python3
"""Repeat the RS(32,32) full-geometry per-segment decode (config 6 shape) and count wrong dwords
per run for the run-time kernels (catches timing-dependent faults that one run can miss).
usage: CESS_EC_LIB=... python tools/stress_rthx.py [--runs 10] [--mode 0]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=10)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--nseg", type=int, default=64)
    args = ap.parse_args()
    import torch
    import cess_amd
    k, m, F, nseg = 32, 32, 512 * 1024, args.nseg
    d_data = torch.empty((nseg, k, F), dtype=torch.uint8, device="cuda")
    d_par = torch.empty((nseg, m, F), dtype=torch.uint8, device="cuda")
    cess_amd.fill_synthetic(d_data, k * F, nseg, 0, 0xCE550005)
    enc = cess_amd.New(k, m)
    enc.EncodeBatch(d_data, d_par, nseg, F)
    ref_d, ref_p = d_data.clone(), d_par.clone()
    rng = np.random.default_rng(3)
    present = np.ones((nseg, k + m), np.uint8)
    for s in range(nseg):
        present[s, rng.choice(k + m, size=m, replace=False)] = 0
    pres_t = torch.from_numpy(present).cuda().bool()
    enc.set_option(4, args.mode)
    bad = []
    for _ in range(args.runs):
        dd, dp = ref_d.clone(), ref_p.clone()
        dd.mul_(pres_t[:, :k, None])
        dp.mul_(pres_t[:, k:, None])
        enc.ReconstructBatch(dd, dp, nseg, F, present)
        torch.cuda.synchronize()
        bad.append(int((dd != ref_d).sum() + (dp != ref_p).sum()))
    print(os.environ.get("CESS_EC_LIB", "default"), "mode", args.mode, "bad bytes per run", bad,
          flush=True)


if __name__ == "__main__":
    main()
