#!/usr/bin/env python3
"""Where GPU SegmentList hashing starts to beat the host: an in-memory file of each size encoded
with every record through encode_file_records, (a) hash_on="gpu": the C pipeline hashing on the
GPU (hash queue; a file ends one 16 MiB segment chain, ~0.47 s, after its last batch lands),
(b) hash_on="host": SegmentEncoder hashing on the host (OpenSSL SHA-256, 16 threads, one pass
over segment + fragment 0). One JSON line per size.

usage: python tools/records_crossover.py [--sizes-mib 16,64,256,1024,2048,4096,8192,12288]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cess_amd  # noqa: E402
from cess_amd.pipeline import encode_file_records  # noqa: E402

MiB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mib", default="16,64,256,1024,2048,4096,8192,12288")
    args = ap.parse_args()
    sizes = [int(x) * MiB for x in args.sizes_mib.split(",")]
    seg = 16 * MiB
    big = max(sizes)
    buf = np.empty(big, np.uint8)
    d = torch.empty((64, seg), dtype=torch.uint8, device="cuda")
    hb = torch.from_numpy(buf)
    nseg = big // seg
    for s in range(0, nseg, 64):
        n = min(64, nseg - s)
        cess_amd.fill_synthetic(d, seg, n, s, 0xCE55000A)
        hb[s * seg:(s + n) * seg].copy_(d[:n].reshape(-1))
    del d
    encode_file_records(buf[:seg])  # warm-up (library, pinned blocks)
    encode_file_records(buf[:seg], hash_on="host")
    # the GPU path's fixed cost, phase by phase, for a one-segment and a 64-segment file
    from cess_amd.pipeline import Pipeline
    from cess_amd.reedsolomon import Encoder
    for n in (1, 64):
        t = [time.perf_counter()]
        enc = Encoder(2, 1, 0)
        t.append(time.perf_counter())
        p = Pipeline(enc, seg // 2, batch_segments=n)
        t.append(time.perf_counter())
        p.run(buf[:n * seg], on_record=lambda *a: None)
        t.append(time.perf_counter())
        p.close()
        t.append(time.perf_counter())
        enc.close()
        t.append(time.perf_counter())
        print(json.dumps({"phases_segments": n, **{k: round(t[i + 1] - t[i], 4) for i, k in
                          enumerate(("codec", "pipeline_create", "run", "pipeline_destroy",
                                     "codec_close"))}}), flush=True)
    for size in sizes:
        src = buf[:size]
        # both legs as encode_file_records runs them: codec, pinned and device buffers sized to
        # the file, set up and torn down inside the timed call
        t0 = time.perf_counter()
        rec_g, _ = encode_file_records(src, hash_on="gpu")
        tg = time.perf_counter() - t0
        t0 = time.perf_counter()
        rec_h, _ = encode_file_records(src, hash_on="host")
        th = time.perf_counter() - t0
        same = [(s.hash, s.fragment_list) for s in rec_g.segments] == \
            [(s.hash, s.fragment_list) for s in rec_h.segments]
        print(json.dumps({"MiB": size // MiB, "gpu_hash_s": round(tg, 4),
                          "host_hash_s": round(th, 4),
                          "gpu_GBps": round(size / tg / 1e9, 2),
                          "host_GBps": round(size / th / 1e9, 2), "records_equal": same}),
              flush=True)


if __name__ == "__main__":
    main()
