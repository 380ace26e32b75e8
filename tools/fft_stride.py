#!/usr/bin/env python3
"""RS(32,32) encode (k_fft3232) throughput against the shard length, i.e. the distance between
the 64 shards a wave reads and writes at one column offset (power-of-two strides vs padded ones).
usage: python tools/fft_stride.py [F_KiB,...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import cess_amd
    fs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else
                           "512,513,516,520,544,640,256,257,1024,1025").split(",")]
    enc = cess_amd.New(32, 32)
    for fk in fs:
        F = fk * 1024
        nseg = max(1, (1 << 30) // (32 * F))
        d = torch.empty((nseg, 32, F), dtype=torch.uint8, device="cuda")
        p = torch.empty((nseg, 32, F), dtype=torch.uint8, device="cuda")
        cess_amd.fill_synthetic(d, 32 * F, nseg, 0, 5)
        for _ in range(3):
            enc.EncodeBatch(d, p, nseg, F)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            enc.EncodeBatch(d, p, nseg, F)
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 20
        print(json.dumps({"F_KiB": fk, "nseg": nseg, "ms": round(ms, 4),
                          "GBps": round(nseg * 64 * F / ms / 1e6, 1)}), flush=True)
        del d, p


if __name__ == "__main__":
    main()
