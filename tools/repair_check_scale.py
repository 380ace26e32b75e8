"""Recorded-hash check of rebuilt fragments (repair_batch, §8f rank 2) on the GPU against host
threads, by the number of fragments checked: RS(2,1), 8 MiB fragments, every segment losing one
fragment. One JSON line per count. Sets repair.AUTO_GPU_CHECK_FRAGMENTS from the crossover.
usage: python tools/repair_check_scale.py [--counts 64,256,512,1024] [--reps 3]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--counts", default="64,256,512,1024")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch
    import cess_amd
    from cess_amd import repair
    k, m, F = 2, 1, 8 << 20
    n = k + m
    enc = cess_amd.New(k, m)
    for nseg in [int(c) for c in a.counts.split(",")]:
        d = torch.empty((nseg, k, F), dtype=torch.uint8, device="cuda")
        p = torch.empty((nseg, m, F), dtype=torch.uint8, device="cuda")
        cess_amd.fill_synthetic(d, k * F, nseg, 0, 0xCE550002)
        enc.EncodeBatch(d, p, nseg, F)
        torch.cuda.synchronize()
        present = np.ones((nseg, n), np.uint8)
        present[np.arange(nseg), np.arange(nseg) % n] = 0
        frag = lambda s, i: d[s, i] if i < k else p[s, i - k]  # noqa: E731
        rec = cess_amd.sha256_hex_device([frag(s, s % n).data_ptr() for s in range(nseg)], F)
        expected = [{s % n: rec[s]} for s in range(nseg)]
        out = {"fragments": nseg, "fragment_bytes": F}
        for on in ("gpu", "host"):
            ts = []
            for _ in range(a.reps + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ok = repair.repair_batch(enc, d, p, nseg, F, present, expected, hash_on=on)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
                assert all(ok)
            out[f"{on}_s"] = round(float(np.median(ts[1:])), 4)
        print(json.dumps(out), flush=True)
        del d, p
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
