"""File retrieval: the download side of the segment -> fragment path.

A file uploaded through `FileBank::upload_declaration` (c-pallets/file-bank/src/lib.rs:423-428)
is recorded as one `SegmentList { hash, fragment_list }` per segment
(c-pallets/file-bank/src/types.rs:13-16): the segment's hash and, in index order, the hashes of
its k data and m parity fragments, which miners store (`FragmentInfo { hash, avail, miner }`,
types.rs:64-76; `avail = false` is an erasure the restoral flow repairs, lib.rs:943-1122). Getting
the file back is a degraded read per segment:

  * fetch the data fragments; a fragment whose SHA-256 differs from its recorded hash counts as
    lost (a miner serving wrong bytes is an erasure, not an error in the file);
  * while fewer than k fragments check out, fetch parity fragments;
  * rebuild the lost data fragments of every such segment on the GPU, one
    `cec_reconstruct_batch` launch per batch (data_only: the parity is not needed);
  * check each segment against its recorded hash, join the k data fragments of every segment
    (the contiguous klauspost Split), drop the last segment's zero padding.

The hashes are SHA-256 hex (the ecosystem convention, see segments.py). The GPU is used only for
the rebuild; a batch whose segments all arrived intact never touches it.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import json
import os
import re
import stat
import time
from typing import BinaryIO, Callable, Dict, Optional, Union

import numpy as np

from . import geometry
from .reedsolomon import ErrTooFewShards
from .segments import FileRecord, SegmentList, file_hash

# fetch(segment index, fragment index, recorded fragment hash hex) -> the fragment's bytes, or None
# when no miner serves it
FetchFn = Callable[[int, int, bytes], Optional[Union[bytes, bytearray, memoryview, np.ndarray]]]


class ErrSegmentHashMismatch(ValueError):
    """A rebuilt or joined segment does not hash to its recorded SegmentList hash."""


class ErrRecordsInconsistent(ValueError):
    """The records' file hash is not the hash of their segment hashes."""


def record_from_json(obj: Union[str, dict]) -> FileRecord:
    """FileRecord from FileRecord.to_json() (the `cess_amd.cli encode` output)."""
    if isinstance(obj, str):
        obj = json.loads(obj)
    segs = [SegmentList(s["hash"].encode(), [f.encode() for f in s["fragment_list"]])
            for s in obj["segments"]]
    return FileRecord(obj["file_hash"].encode(), int(obj["size"]), segs)


_HEX64 = re.compile(rb"[0-9a-f]{64}")


def dir_fetch(directory: str) -> FetchFn:
    """Fragments stored as files named by their hash (what `cli encode --out DIR` writes). A
    recorded hash is used as a file name only when it is exactly 64 lowercase hex chars (a crafted
    record must not name "../x", an absolute path or a device), and only regular files are read;
    anything else is a missing fragment."""
    def fetch(_seg: int, _frag: int, h: bytes):
        if not _HEX64.fullmatch(h):
            return None
        path = os.path.join(directory, h.decode())
        try:
            fd = os.open(path, os.O_RDONLY | getattr(os, "O_NONBLOCK", 0))
        except (FileNotFoundError, NotADirectoryError):
            return None
        try:
            if not stat.S_ISREG(os.fstat(fd).st_mode):
                return None
            with os.fdopen(fd, "rb", closefd=False) as f:
                return f.read()
        finally:
            os.close(fd)
    return fetch


class Retriever:
    """Rebuilds files from their records and whatever fragments `fetch` returns. The codec and
    the device batch are created on the first segment that needs a rebuild."""

    def __init__(self, k: int = geometry.DATA_SHARDS, m: int = geometry.PARITY_SHARDS,
                 segment_size: int = geometry.SEGMENT_SIZE, device: int = 0,
                 batch_segments: int = 64, threads: int = 16):
        if segment_size % k:
            raise ValueError("segment_size must be a multiple of k")
        self.k, self.m, self.n = k, m, k + m
        self.seg = segment_size
        self.F = segment_size // k
        self.device = device
        self.B = max(1, batch_segments)
        # two executors: `pool` runs the fetches + fragment checks of the next batch while
        # `work` stages this batch's valid fragments, rebuilds and checks its segments (on one
        # FIFO executor the staging and checks queued behind the next batch's gathers, so the
        # rebuild did not overlap them). The default 16 threads is the GPU's CPU share.
        self.pool = cf.ThreadPoolExecutor(max_workers=max(1, threads))
        self.work = cf.ThreadPoolExecutor(max_workers=max(1, threads))
        self.enc = None
        self.d_data = self.d_par = self.h_data = self.h_par = None

    def close(self) -> None:
        self.pool.shutdown(wait=True)
        self.work.shutdown(wait=True)
        if self.enc is not None:
            self.enc.close()
            self.enc = None
        self.d_data = self.d_par = self.h_data = self.h_par = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _gather(self, s: int, sl: SegmentList, fetch: FetchFn):
        """The fragments of segment s that check out: ({index: uint8 array}, fetched, rejected,
        (segment hasher, p): the hasher has streamed the first p data fragments), data first,
        parity only while fewer than k are valid (runs on a pool thread)."""
        if len(sl.fragment_list) != self.n:
            raise ValueError(f"segment {s}: {len(sl.fragment_list)} fragment hashes, "
                             f"expected k + m = {self.n} (check_file_spec)")
        good: Dict[int, np.ndarray] = {}
        fetched = rejected = 0
        # the segment's hash streams over the leading valid data fragments in order: fragment 0's
        # digest is that stream's prefix digest (one pass serves both, as on upload); the segment
        # check later streams only the data fragments after the valid prefix (all rebuilt or
        # after a gap), so a segment whose data fragments all check out is hashed once
        seg_h = hashlib.sha256()
        prefix = 0
        for f in range(self.n):
            if f >= self.k and len(good) >= self.k:
                break
            raw = fetch(s, f, sl.fragment_list[f])
            if raw is None:
                continue
            fetched += 1
            a = np.frombuffer(raw, np.uint8) if not isinstance(raw, np.ndarray) else \
                raw.reshape(-1).view(np.uint8)
            if a.size != self.F:
                valid = False
            elif f == 0:
                seg_h.update(a)
                valid = seg_h.copy().hexdigest().encode() == sl.fragment_list[0]
                if valid:
                    prefix = 1
                else:
                    seg_h = hashlib.sha256()  # the wrong bytes leave the stream
            else:
                valid = hashlib.sha256(a).hexdigest().encode() == sl.fragment_list[f]
                if valid and f == prefix and f < self.k:
                    seg_h.update(a)
                    prefix += 1
            if not valid:
                rejected += 1  # wrong bytes: an erasure like a missing fragment
                continue
            good[f] = a
        if len(good) < self.k:
            raise ErrTooFewShards(f"segment {s}: {len(good)} of {self.n} fragments valid, "
                                  f"need {self.k}")
        return good, fetched, rejected, (seg_h, prefix)

    def _rebuild(self, todo, stats: dict) -> None:
        """Rebuild the lost data fragments of [(s, good)] (one launch). The valid fragments go
        through a pinned staging batch (copied in on the pool's threads); only the rebuilt
        fragments come back, into the same staging rows, which `good` then refers to (valid until
        the next batch's rebuild)."""
        import torch
        import cess_amd
        k, m, F = self.k, self.m, self.F
        if self.enc is None:
            self.enc = cess_amd.New(k, m, device=self.device)
            dev = torch.device("cuda", self.device)
            self.d_data = torch.empty((self.B, k, F), dtype=torch.uint8, device=dev)
            self.d_par = torch.empty((self.B, m, F), dtype=torch.uint8, device=dev)
            self.h_data = torch.empty((self.B, k, F), dtype=torch.uint8, pin_memory=True)
            self.h_par = torch.empty((self.B, m, F), dtype=torch.uint8, pin_memory=True)
        nb = len(todo)
        hd, hp = self.h_data.numpy(), self.h_par.numpy()
        present = np.zeros((nb, self.n), np.uint8)
        copies = []
        for i, (_s, good) in enumerate(todo):
            for f, a in good.items():
                present[i, f] = 1
                copies.append((i, f, a))

        def stage(c):
            i, f, a = c
            np.copyto(hd[i, f] if f < k else hp[i, f - k], a)
        list(self.work.map(stage, copies))
        # only the valid fragments cross PCIe: the gather stops at k of them, so they are exactly
        # the survivors the rebuild reads (the slots of lost fragments are never read)
        for i, f, _a in copies:
            if f < k:
                self.d_data[i, f].copy_(self.h_data[i, f], non_blocking=True)
            else:
                self.d_par[i, f - k].copy_(self.h_par[i, f - k], non_blocking=True)
        st = torch.cuda.current_stream(self.d_data.device)  # the copies' stream
        self.enc.ReconstructBatch(self.d_data[:nb], self.d_par[:nb], nb, F, present,
                                  data_only=True, stream=st)
        lost = [(i, f) for i in range(nb) for f in range(k) if not present[i, f]]
        for i, f in lost:
            self.h_data[i, f].copy_(self.d_data[i, f], non_blocking=True)
        st.synchronize()
        for i, f in lost:
            todo[i][1][f] = hd[i, f]
        stats["rebuilt_segments"] += nb
        stats["rebuilt_fragments"] += len(lost)

    def retrieve(self, rec: FileRecord, fetch: FetchFn, out: Union[str, BinaryIO],
                 check_segments: bool = True) -> dict:
        """Write the file `rec` describes to `out` (a path or a binary file object) from the
        fragments `fetch` returns. Raises ErrTooFewShards when a segment has fewer than k valid
        fragments, ErrSegmentHashMismatch when a segment does not hash to its record (checked
        unless check_segments=False), ErrRecordsInconsistent when the file hash does not match
        the segment hashes. Returns counters (fragments fetched / rejected, segments and
        fragments rebuilt on the GPU, seconds)."""
        t0 = time.perf_counter()
        if file_hash(rec.segments) != rec.file_hash:
            raise ErrRecordsInconsistent("file hash is not SHA-256 over the segment hashes")
        nseg = len(rec.segments)
        if rec.size > nseg * self.seg or rec.size <= (nseg - 1) * self.seg:
            raise ValueError(f"size {rec.size} does not fit {nseg} segments of {self.seg} bytes")
        stats = {"segments": nseg, "fetched": 0, "rejected": 0, "rebuilt_segments": 0,
                 "rebuilt_fragments": 0}
        own = isinstance(out, str)
        # a path is written under a temporary name and renamed once every segment checked out:
        # a failed retrieval leaves no partial file behind
        tmp = out + ".part" if own else None
        fo = open(tmp, "wb") if own else out
        ok = False

        def gather(b0):  # the batch's fetch + fragment checks, queued on the pool
            return [self.pool.submit(self._gather, s, rec.segments[s], fetch)
                    for s in range(b0, min(nseg, b0 + self.B))]
        pending = gather(0) if nseg else []
        try:
            written = 0
            for b0 in range(0, nseg, self.B):
                idx = list(range(b0, min(nseg, b0 + self.B)))
                got = [f.result() for f in pending]
                # the next batch's fetches and fragment checks run on `pool` while this one is
                # staged, rebuilt on the GPU and checked on `work`
                pending = gather(b0 + self.B) if b0 + self.B < nseg else []
                goods = [g for g, _, _, _ in got]
                streams = [h for _, _, _, h in got]  # (hasher, data fragments streamed)
                stats["fetched"] += sum(n for _, n, _, _ in got)
                stats["rejected"] += sum(r for _, _, r, _ in got)
                todo = [(s, g) for s, g in zip(idx, goods) if any(f not in g
                                                                   for f in range(self.k))]
                if todo:
                    self._rebuild(todo, stats)

                def check(i):  # the segment's hash over its k data fragments, no joined copy
                    if check_segments:
                        h, p = streams[i]
                        for f in range(p, self.k):  # the rebuilt ones and any after them
                            h.update(goods[i][f])
                        if h.hexdigest().encode() != rec.segments[idx[i]].hash:
                            raise ErrSegmentHashMismatch(f"segment {idx[i]} does not match "
                                                         f"its recorded hash")
                    return goods[i]
                for g in self.work.map(check, range(len(idx))):
                    for f in range(self.k):  # the data fragments in order, the padding dropped
                        take = min(self.F, rec.size - written)
                        if take <= 0:
                            break
                        fo.write(memoryview(g[f][:take]))
                        written += take
            ok = True
        finally:
            for f in pending:  # after a failure: drop the next batch's queued work
                f.cancel()
            if own:
                fo.close()
                if ok:
                    os.replace(tmp, out)
                else:
                    os.unlink(tmp)
        stats["bytes"] = rec.size
        stats["seconds"] = round(time.perf_counter() - t0, 4)
        return stats


def retrieve_file(rec: FileRecord, fetch: FetchFn, out: Union[str, BinaryIO],
                  k: int = geometry.DATA_SHARDS, m: int = geometry.PARITY_SHARDS,
                  segment_size: int = geometry.SEGMENT_SIZE, device: int = 0, **kw) -> dict:
    """One-shot Retriever(...).retrieve(rec, fetch, out)."""
    with Retriever(k, m, segment_size, device, **kw) as r:
        return r.retrieve(rec, fetch, out)
