"""SegmentList emission (file -> records) through one long-lived
RecordsSession per hash placement: an in-memory file (splitmix-free random bytes, generated once)
streamed through the C pipeline, records hashed on the GPU queue, on host threads, or hybrid.
Each placement's session is created once and timed over `--reps` runs (no pinning in the timed
region); a records_stream leg runs `--stream` files back to back in one run (the same buffer
each time: the rate does not depend on the bytes). Records of sampled segments are checked
against hashlib. One JSON line per measurement.
Usage: python tools/records_bench.py [--gib 8] [--modes none,gpu,host,hybrid] [--tails -1,0,2]
"""
import argparse
import hashlib
import json
import os
import resource
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def cpu_seconds():
    r = resource.getrusage(resource.RUSAGE_SELF)
    return r.ru_utime + r.ru_stime


def check(rec, buf, seg, k, picks):
    for s in picks:
        a = buf[s * seg:(s + 1) * seg]
        if len(a) < seg:
            a = np.concatenate([a, np.zeros(seg - len(a), np.uint8)])
        sl = rec.segments[s]
        if sl.hash != hashlib.sha256(a).hexdigest().encode():
            return False
        F = seg // k
        for j in range(k):
            if sl.fragment_list[j] != hashlib.sha256(a[j * F:(j + 1) * F]).hexdigest().encode():
                return False
    return True


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=8)
    ap.add_argument("--modes", default="none,gpu,host,hybrid")
    ap.add_argument("--tails", default="-1")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--depth", type=int, default=0, help="0: the pipeline's default")
    ap.add_argument("--window", type=int, default=0)
    ap.add_argument("--batch", type=int, default=64, help="segments per batch")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--stream", type=int, default=0, help="files in the records_stream leg")
    ap.add_argument("--stream-segments", type=int, default=1000)
    ap.add_argument("--form", type=int, default=-1, help="cec_host_sha_set_form")
    ap.add_argument("--pieces", action="store_true",
                    help="stream files as in bench.py: the file buffer read as pieces")
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime: torch first)
    from cess_amd import _lib
    from cess_amd.pipeline import Pipeline, RecordsSession
    from cess_amd.reedsolomon import Encoder
    lib = _lib.load()
    if a.form >= 0:
        assert lib.cec_host_sha_set_form(a.form) == 0
    k, m, seg = 2, 1, 16 << 20
    size = int(a.gib * (1 << 30))
    nstream = a.stream_segments * seg if a.stream else 0
    buf = np.empty(max(size, nstream), np.uint8)
    rng = np.random.default_rng(5)
    step = 1 << 28
    for o in range(0, buf.size, step):
        buf[o:o + step] = rng.integers(0, 256, min(step, buf.size - o), dtype=np.uint8)
    src = buf[:size]
    nseg = -(-size // seg)
    picks = [0, nseg // 2, nseg - 1]
    print(json.dumps({"file_bytes": size, "segments": nseg, "host_sha_form":
                      lib.cec_host_sha_form()}), flush=True)
    for mode in a.modes.split(","):
        for tail in ([int(t) for t in a.tails.split(",")] if mode == "hybrid" else [-1]):
            t0 = time.perf_counter()
            if mode == "none":
                enc = Encoder(k, m, 0)
                pipe = Pipeline(enc, seg // k, hash=False, depth=a.depth,
                                batch_segments=a.batch)
                ses = None
            else:
                ses = RecordsSession(k, m, seg, 0, mode, depth=a.depth, window=a.window,
                                     host_threads=a.threads, tail_batches=tail,
                                     batch_segments=a.batch)
            t_create = time.perf_counter() - t0
            times, cpus, ok = [], [], True
            for _ in range(a.reps):
                c0 = cpu_seconds()
                t0 = time.perf_counter()
                if ses is None:
                    st = pipe.run(src)
                else:
                    rec, st = ses.encode(src)
                times.append(time.perf_counter() - t0)
                cpus.append(cpu_seconds() - c0)
                if ses is not None:
                    ok = ok and check(rec, src, seg, k, picks) and len(rec.segments) == nseg
            info = (ses.pipe if ses else pipe).info()
            out = {"mode": mode, "tail_batches": tail, "batch_segments": a.batch, "create_s": round(t_create, 3),
                   "seconds": [round(t, 4) for t in times],
                   "cpu_seconds": [round(c, 3) for c in cpus], "best_GBps":
                   round(size / min(times) / 1e9, 2), "records_ok": ok, **info}
            print(json.dumps(out), flush=True)
            if a.stream and ses is not None:
                if a.pieces:  # bench.py's host_e2e: the --gib buffer repeated up to the size
                    pieces, left = [], nstream
                    while left:
                        take = min(left, size)
                        pieces.append(buf[:take])
                        left -= take
                    files = [pieces] * a.stream
                else:
                    files = [buf[:nstream]] * a.stream
                done_t = []
                c0 = cpu_seconds()
                t0 = time.perf_counter()
                recs, st = ses.encode_many(files, on_file=lambda f, r, s: done_t.append(
                    time.perf_counter() - t0))
                dt = time.perf_counter() - t0
                dc = cpu_seconds() - c0
                ok2 = all(check(r, buf, seg, k, [0, a.stream_segments - 1]) for r in recs)
                print(json.dumps({"mode": mode, "tail_batches": tail, "records_stream": a.stream,
                                  "file_bytes": nstream, "seconds": round(dt, 4),
                                  "cpu_seconds": round(dc, 3),
                                  "GBps": round(a.stream * nstream / dt / 1e9, 2),
                                  "file_done_s": [round(x, 3) for x in done_t],
                                  "records_ok": ok2}), flush=True)
            t0 = time.perf_counter()
            if ses is None:
                pipe.close()
                enc.close()
            else:
                ses.close()
            print(json.dumps({"mode": mode, "destroy_s": round(time.perf_counter() - t0, 3)}),
                  flush=True)


if __name__ == "__main__":
    main()
