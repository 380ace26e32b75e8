#!/usr/bin/env python3
"""Probe: are libcessec's batch calls capturable into a HIP graph once their plans are cached?
BASELINE config 1's GPU leg (one 16 MiB RS(2,1) segment: encode + the 3 single-erasure rebuilds
per step) is launch-latency bound eagerly; replaying the step as one graph removes the per-call
host work. Prints eager and graph ms per step and whether the graph's outputs are bit-exact."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cess_amd  # noqa: E402

MiB = 1 << 20


def main():
    k, m, F, nseg = 2, 1, 8 * MiB, int(sys.argv[1]) if len(sys.argv) > 1 else 1
    dev = torch.device("cuda", 0)
    d_data = torch.empty((nseg, k, F), dtype=torch.uint8, device=dev)
    d_par = torch.empty((nseg, m, F), dtype=torch.uint8, device=dev)
    cess_amd.fill_synthetic(d_data, k * F, nseg, 0, 0xCE550001)
    enc = cess_amd.New(k, m)
    side = torch.cuda.Stream(dev)
    pats = [np.array([int(i != e) for i in range(k + m)], np.uint8) for e in range(k + m)]

    def step(st):
        enc.EncodeBatch(d_data, d_par, nseg, F, stream=st)
        for p in pats:
            enc.ReconstructBatch(d_data, d_par, nseg, F, p, stream=st)

    torch.cuda.synchronize()
    for _ in range(5):
        step(side)
    torch.cuda.synchronize()
    ref_d, ref_p = d_data.clone(), d_par.clone()

    def timed(fn, reps=200):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(side):
            a.record()
            for _ in range(reps):
                fn()
            b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    eager = timed(lambda: step(side))
    out = {"nseg": nseg, "eager_ms": round(eager, 4)}
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            step(torch.cuda.current_stream(dev))
        torch.cuda.synchronize()
        d_par.zero_()
        g.replay()
        torch.cuda.synchronize()
        out["graph_bit_exact"] = bool(torch.equal(d_par, ref_p) and torch.equal(d_data, ref_d))
        out["graph_ms"] = round(timed(g.replay), 4)
        per_step = 4 * nseg * (k + m) * F
        out["eager_GBps"] = round(per_step / (eager * 1e-3) / 1e9, 1)
        out["graph_GBps"] = round(per_step / (out["graph_ms"] * 1e-3) / 1e9, 1)
    except Exception as e:  # noqa: BLE001 - the probe reports what failed
        out["graph_error"] = f"{type(e).__name__}: {e}"[:400]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
