#!/usr/bin/env python3
"""Repeat the RS(32,32) full-geometry per-segment decode (config 6 shape: 32 random erasures per
segment, run-time coefficients) and count wrong bytes per run against the C oracle (data =
the synthetic generator, parity = oracle/rs_oracle.c), for the run-time kernels. A repeat-run
check for timing-dependent faults; the static wait-state rule of k_rthx is pinned on the code
object by tests/test_host.py::test_rthx_index_mode_wait_states.
usage: python tools/stress_rthx.py [--runs 10] [--mode 0] [--nseg 64]"""
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
    from oracle.c_oracle import load_c_oracle
    orc = load_c_oracle()
    k, m, F, nseg = 32, 32, 512 * 1024, args.nseg
    seed = 0xCE550005
    data = np.empty((nseg, k, F), np.uint8)
    par = np.empty((nseg, m, F), np.uint8)
    orc.orc_fill_synthetic(data.ctypes.data, k * F, nseg, 0, seed)
    orc.orc_encode_batch(k, m, data.ctypes.data, par.ctypes.data, nseg, F,
                         min(16, os.cpu_count() or 1), 1)
    ref_d = torch.from_numpy(data).cuda()
    ref_p = torch.from_numpy(par).cuda()
    rng = np.random.default_rng(3)
    present = np.ones((nseg, k + m), np.uint8)
    for s in range(nseg):
        present[s, rng.choice(k + m, size=m, replace=False)] = 0
    pres_t = torch.from_numpy(present).cuda().bool()
    enc = cess_amd.New(k, m)
    enc.set_option(4, args.mode)
    bad = []
    for _ in range(args.runs):
        dd, dp = ref_d.clone(), ref_p.clone()
        dd.mul_(pres_t[:, :k, None])
        dp.mul_(pres_t[:, k:, None])
        enc.ReconstructBatch(dd, dp, nseg, F, present)
        torch.cuda.synchronize()
        bad.append(int((dd != ref_d).sum() + (dp != ref_p).sum()))
    print("mode", args.mode, "wrong bytes per run vs the C oracle", bad, flush=True)
    return 1 if any(bad) else 0


if __name__ == "__main__":
    sys.exit(main())
