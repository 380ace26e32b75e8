#!/usr/bin/env python3
"""File retrieval throughput (cess_amd.retrieve, the download side of the path): a synthetic
in-memory file is encoded into records + fragments held in host memory, one fragment of every
segment is dropped (rotating index, so data and parity losses alternate), and the file is
retrieved: fetch, fragment hashes checked on host threads, lost data fragments rebuilt on the
GPU (one ReconstructBatch launch per batch), segment hashes checked, joined. The untimed warm-up
run's output is compared byte for byte with the source, the timed run's at both ends of every
write. One JSON line.

usage: python tools/retrieve_bench.py [--gib 4] [--threads 16] [--intact]"""
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
from cess_amd.retrieve import Retriever  # noqa: E402

MiB = 1 << 20


class CompareSink:
    """Checks writes against the source bytes at their offset: every byte (`full`, the untimed
    warm-up run) or the first and last 4 KiB of every write (the timed run, so the sink's
    single-threaded compare is not what is measured)."""

    def __init__(self, src, full: bool):
        self.src = src
        self.full = full
        self.n = 0
        self.same = True

    def write(self, b):
        a = np.frombuffer(b, np.uint8)
        ref = self.src[self.n:self.n + a.size]
        if self.full or a.size <= 8192:
            self.same &= bool(np.array_equal(a, ref))
        else:
            self.same &= bool(np.array_equal(a[:4096], ref[:4096]) and
                              np.array_equal(a[-4096:], ref[-4096:]))
        self.n += a.size
        return a.size


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=4)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--intact", action="store_true", help="lose no fragment")
    ap.add_argument("--separate-segment-pass", action="store_true",
                    help="A/B: drop the streamed segment digest, hash every segment again")
    args = ap.parse_args()
    seg = 16 * MiB
    nseg = args.gib * 1024 // 16
    size = nseg * seg - 12345  # ragged tail
    buf = np.empty(nseg * seg, np.uint8)
    d = torch.empty((64, seg), dtype=torch.uint8, device="cuda")
    hb = torch.from_numpy(buf)
    for s in range(0, nseg, 64):
        n = min(64, nseg - s)
        cess_amd.fill_synthetic(d, seg, n, s, 0xCE55000B)
        hb[s * seg:(s + n) * seg].copy_(d[:n].reshape(-1))
    del d
    src = buf[:size]
    store = {}
    t0 = time.perf_counter()
    rec, _ = encode_file_records(
        src, hash_on="host",
        on_fragment=lambda s, i, v: store.__setitem__((s, i), np.array(v, copy=True)))
    t_enc = time.perf_counter() - t0
    lost = set() if args.intact else {(s, s % 3) for s in range(nseg)}

    def fetch(s, f, _h):
        return None if (s, f) in lost else store[(s, f)]

    if args.separate_segment_pass:
        gather = Retriever._gather
        import hashlib
        Retriever._gather = lambda self, *a: gather(self, *a)[:3] + ((hashlib.sha256(), 0),)
    with Retriever(threads=args.threads) as r:
        full = CompareSink(src, True)
        r.retrieve(rec, fetch, full)  # warm-up (codec, device batch), every byte compared
        sink = CompareSink(src, False)
        t0 = time.perf_counter()
        st = r.retrieve(rec, fetch, sink)
        t = time.perf_counter() - t0
    print(json.dumps({"file_bytes": size, "segments": nseg, "lost_fragments": len(lost),
                      "rebuilt_segments": st["rebuilt_segments"],
                      "rebuilt_fragments": st["rebuilt_fragments"], "seconds": round(t, 4),
                      "GBps": round(size / t / 1e9, 2), "threads": args.threads,
                      "output_equal_source": full.same and full.n == size and sink.same and sink.n == size, "intact": args.intact,
                      "separate_segment_pass": args.separate_segment_pass,
                      "encode_records_seconds": round(t_enc, 4)}), flush=True)


if __name__ == "__main__":
    main()
