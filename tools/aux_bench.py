#!/usr/bin/env python3
"""Measurements of the §8f rows beside the codec (one MI355X), one JSON line each:
  repair   (f2) 64 RS(2,1) segments of 8 MiB fragments, each losing fragment s mod 3: the batched
           rebuild (HBM roofline, (k+1)*F bytes per segment) and the recorded-hash check of the
           64 rebuilt fragments on the GPU (one SHA-256 chain per fragment: latency bound);
  audit    (f3) the 47 challenged 8 KiB chunks of all 192 fragments of a 1 GiB batch: the gather
           (2 x chunk bytes moved) and gather + SHA-256 of every chunk;
  fillers  (f4) 64 idle fillers of 8 MiB: generation in HBM and their SHA-256 hashes;
  partial  (§8e) the two GPU steps of the partial-product exchange for RS(32,32) (64 segments of
           512 KiB fragments, one lost each, placement (s + f) mod 8): one holder GPU's partial
           rebuild from the survivors it holds, the decoder's XOR of 7 received partials, and the
           full rebuild of the same segments beside them.
usage: python tools/aux_bench.py [--reps 5] [--only partial]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GB = 1e9


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    import numpy as np
    import torch
    import cess_amd
    from cess_amd import audit, repair
    k, m, F, nseg = 2, 1, 8 << 20, 64
    n = k + m
    dev = torch.device("cuda", 0)
    enc = cess_amd.New(k, m)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))

    if args.only == "partial":
        return partial_row(args, torch, np, cess_amd, dev)
    if args.only == "plan":
        return plan_row(args, torch, np, cess_amd, dev)
    if args.only == "verify":
        return verify_row(args, torch, np, cess_amd, dev)
    d = torch.empty((nseg, k, F), dtype=torch.uint8, device=dev)
    p = torch.empty((nseg, m, F), dtype=torch.uint8, device=dev)
    cess_amd.fill_synthetic(d, k * F, nseg, 0, 0xCE550002)
    enc.EncodeBatch(d, p, nseg, F)
    torch.cuda.synchronize()
    present = np.ones((nseg, n), np.uint8)
    present[np.arange(nseg), np.arange(nseg) % n] = 0
    frag = lambda s, i: d[s, i] if i < k else p[s, i - k]  # noqa: E731
    recorded = cess_amd.sha256_hex_device([frag(s, s % n).data_ptr() for s in range(nseg)], F)
    expected = [{s % n: recorded[s]} for s in range(nseg)]
    t_rebuild = timed(lambda: enc.ReconstructBatch(d, p, nseg, F, present))
    ok = []
    t_all = timed(lambda: ok.append(repair.repair_batch(enc, d, p, nseg, F, present, expected,
                                                        hash_on="gpu")))
    t_host = timed(lambda: ok.append(repair.repair_batch(enc, d, p, nseg, F, present, expected,
                                                         hash_on="host")))
    assert all(all(x) for x in ok)
    print(json.dumps({"row": "f2 repair", "segments": nseg, "fragment_bytes": F,
                      "rebuild_s": round(t_rebuild, 6),
                      "rebuild_GBps": round(nseg * (k + 1) * F / t_rebuild / GB, 1),
                      "rebuild_roofline_frac": round(nseg * (k + 1) * F / t_rebuild / GB / 8000, 3),
                      "rebuild_and_hash_check_s": round(t_all, 4),
                      "rebuild_and_host_hash_check_s": round(t_host, 4),
                      "host_hash_threads": 16,
                      "hash_check_note": "SHA-256 of each 8 MiB rebuilt fragment is one serial "
                                         "131,073-block chain: latency bound"}), flush=True)

    idx, _ = audit.challenge_indices(list(range(1, 4096)))
    nfrag, chunk = nseg * n, F // audit.CHUNK_COUNT
    d_chunks = torch.empty((nfrag, len(idx), chunk), dtype=torch.uint8, device=dev)
    d_hex = torch.empty((nfrag, len(idx), 64), dtype=torch.uint8, device=dev)
    t_g = timed(lambda: audit.audit_chunks(enc, d, p, nseg, F, idx, d_chunks=d_chunks))
    t_h = timed(lambda: audit.audit_chunks(enc, d, p, nseg, F, idx, d_chunks=d_chunks,
                                           d_hex=d_hex))
    cb = nfrag * len(idx) * chunk
    print(json.dumps({"row": "f3 audit", "fragments": nfrag, "chunks_per_fragment": len(idx),
                      "chunk_bytes": chunk, "gather_s": round(t_g, 6),
                      "gather_GBps_moved": round(2 * cb / t_g / GB, 1),
                      "gather_and_sha256_s": round(t_h, 5),
                      "chunks_per_s": round(nfrag * len(idx) / t_h, 1)}), flush=True)

    out = {}
    for on in ("gpu", "host"):
        t_f = timed(lambda: out.update(r=repair.generate_fillers(nseg, hash_on=on)))
        print(json.dumps({"row": "f4 fillers", "fillers": nseg, "filler_bytes": F,
                          "hash_on": on, "generate_and_hash_s": round(t_f, 4),
                          "GBps": round(nseg * F / t_f / GB, 2)}), flush=True)
    partial_row(args, torch, np, cess_amd, dev)


def verify_row(args, torch, np, cess_amd, dev):
    """cec_verify_batch over a 1 GiB batch: parity recomputed into scratch, compared."""
    for k, m, F in ((2, 1, 8 << 20), (32, 32, 512 << 10)):
        nseg = 64
        enc = cess_amd.New(k, m)
        d = torch.empty((nseg, k, F), dtype=torch.uint8, device=dev)
        p = torch.empty((nseg, m, F), dtype=torch.uint8, device=dev)
        ok = torch.empty(nseg, dtype=torch.uint8, device=dev)
        cess_amd.fill_synthetic(d, k * F, nseg, 0, 0xCE550007)
        enc.EncodeBatch(d, p, nseg, F)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        enc.VerifyBatch(d, p, nseg, F, ok)
        a.record()
        for _ in range(20):
            enc.VerifyBatch(d, p, nseg, F, ok)
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 20
        assert bool(ok.all())
        fused = (k, m) in ((2, 1), (32, 32))  # one read-only pass (else scratch + compare)
        moved = nseg * ((k + m) if fused else (k + 3 * m)) * F
        print(json.dumps({"row": "verify batch", "code": f"RS({k},{m})", "segments": nseg,
                          "fragment_bytes": F, "ms": round(ms, 4),
                          "path": ("fused k_verify21" if k == 2 else "fused k_fft3232_verify")
                          if fused else "encode to scratch + compare",
                          "GBps_of_k_plus_m": round(nseg * (k + m) * F / (ms * 1e-3) / GB, 1),
                          "GBps_moved": round(moved / (ms * 1e-3) / GB, 1)}), flush=True)


def plan_row(args, torch, np, cess_amd, dev):
    """Host cost of a per-segment rebuild whose erasure patterns are new to the decode cache
    (matrix inversions + program uploads) against the same call with a cached plan."""
    k, m, F, nseg = 32, 32, 512 << 10, 64
    n = k + m
    enc = cess_amd.New(k, m)
    d = torch.empty((nseg, k, F), dtype=torch.uint8, device=dev)
    p = torch.empty((nseg, m, F), dtype=torch.uint8, device=dev)
    cess_amd.fill_synthetic(d, k * F, nseg, 0, 0xCE550006)
    enc.EncodeBatch(d, p, nseg, F)
    rng = np.random.default_rng(1)

    def fresh(e):
        pres = np.ones((nseg, n), np.uint8)
        for s in range(nseg):
            pres[s, rng.choice(n, size=e, replace=False)] = 0
        return pres

    out = {"row": "plan build", "code": "RS(32,32)", "segments": nseg, "fragment_bytes": F}
    for e in (1, 4, 16):
        ts_new, ts_cached = [], []
        for _ in range(max(3, args.reps)):
            pres = fresh(e)
            for ts in (ts_new, ts_cached):  # first call builds the plan, second reuses it
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                enc.ReconstructBatch(d, p, nseg, F, pres)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
        out[f"e{e}_new_patterns_ms"] = round(float(np.median(ts_new)) * 1e3, 3)
        out[f"e{e}_cached_plan_ms"] = round(float(np.median(ts_cached)) * 1e3, 3)
    print(json.dumps(out), flush=True)


def partial_row(args, torch, np, cess_amd, dev):
    k, m, F, nseg, G = 32, 32, 512 << 10, 64, 8
    n = k + m
    enc = cess_amd.New(k, m)
    d = torch.empty((nseg, k, F), dtype=torch.uint8, device=dev)
    p = torch.empty((nseg, m, F), dtype=torch.uint8, device=dev)
    cess_amd.fill_synthetic(d, k * F, nseg, 0, 0xCE550005)
    enc.EncodeBatch(d, p, nseg, F)
    present = np.ones((nseg, n), np.uint8)
    present[np.arange(nseg), np.arange(nseg) % n] = 0
    # survivors (first k present) held by rank 1 under (s + f) mod G
    held = np.zeros_like(present)
    for s in range(nseg):
        surv = np.flatnonzero(present[s])[:k]
        held[s, [f for f in surv if (s + f) % G == 1]] = 1
    nheld = int(held.sum())

    def ev_time(fn, reps):
        fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps * 1e-3

    reps = max(10, args.reps * 4)
    t_part = ev_time(lambda: enc.ReconstructPartialBatch(d, p, nseg, F, present, held), reps)
    t_full = ev_time(lambda: enc.ReconstructBatch(d, p, nseg, F, present), reps)
    H = G - 1
    acc = torch.empty((H + 1, nseg, F), dtype=torch.uint8, device=dev)
    t_xor = ev_time(lambda: cess_amd.xor_batch(acc[0], acc[1], H, nseg * F, nseg * F), reps)
    part_bytes = (nheld + nseg) * F  # held survivors read, one partial written per segment
    print(json.dumps({
        "row": "e partial exchange", "code": "RS(32,32)", "segments": nseg, "fragment_bytes": F,
        "lost_per_segment": 1, "world_modelled": G,
        "holder_partial_s": round(t_part, 7), "holder_inputs": nheld,
        "holder_partial_GBps": round(part_bytes / t_part / GB, 1),
        "decoder_xor_s": round(t_xor, 7),
        "decoder_xor_GBps": round((H + 2) * nseg * F / t_xor / GB, 1),
        "full_rebuild_s": round(t_full, 7),
        "full_rebuild_GBps": round((k + 1) * nseg * F / t_full / GB, 1),
        "xgmi_fragments_per_segment": {"survivors": "27-28", "partials": H}}), flush=True)


if __name__ == "__main__":
    main()
