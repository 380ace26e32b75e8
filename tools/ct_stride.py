#!/usr/bin/env python3
"""RS(2,1) encode (k_ct) throughput against the shard length (= the distance between the two data
fragments a lane reads and the parity it writes), power-of-two vs padded.
usage: python tools/ct_stride.py [F_KiB,...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import cess_amd
    fs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else
                           "8192,8193,8196,8200,8256,8704,4096,4097,16384,16385").split(",")]
    enc = cess_amd.New(2, 1)
    for fk in fs:
        F = fk * 1024
        nseg = max(1, (1 << 30) // (2 * F))
        d = torch.empty((nseg, 2, F), dtype=torch.uint8, device="cuda")
        p = torch.empty((nseg, 1, F), dtype=torch.uint8, device="cuda")
        cess_amd.fill_synthetic(d, 2 * F, nseg, 0, 5)
        for _ in range(5):
            enc.EncodeBatch(d, p, nseg, F)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(50):
            enc.EncodeBatch(d, p, nseg, F)
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 50
        print(json.dumps({"F_KiB": fk, "nseg": nseg, "ms": round(ms, 4),
                          "GBps": round(nseg * 3 * F / ms / 1e6, 1)}), flush=True)
        del d, p


if __name__ == "__main__":
    main()
