"""File -> segments -> fragments -> `SegmentList` records.

What the chain consumes (reference):
  * `SegmentList { hash, fragment_list: BoundedVec<Hash, FragmentCount> }`
    (c-pallets/file-bank/src/types.rs:13-16), one per 16 MiB segment, submitted with
    `upload_declaration(file_hash, deal_info, user_brief)` (c-pallets/file-bank/src/lib.rs:423);
  * `check_file_spec`: every fragment_list has FragmentCount entries (functions.rs:4-14);
  * space locked = segments x SEGMENT_SIZE x 15 / 10 (lib.rs:440);
  * `Hash([u8; 64])` (primitives/common/src/lib.rs:16).
Hash convention [ecosystem, unpinned by the reference]: 64 lowercase hex chars of SHA-256; the
last segment is zero padded to SEGMENT_SIZE. File hash [build convention]: SHA-256 (hex) of the
concatenated hex segment hashes — a two-level hash, so no serial pass over the whole file
(one serial SHA-256 stream caps a file at ~2 GB/s).

Pipeline (one GPU): batches of up to 64 segments (1 GiB) go through pinned host buffers and two
device slots. Batch i+1's H2D copy and encode overlap the hashing of batch i. Hashes are
computed where they are cheapest: on the host (OpenSSL SHA-NI via hashlib, threaded) for the
few long fragments of the CESS geometry (3 x 8 MiB per segment), on the GPU (k_sha256) for wide
codes with thousands of short fragments per batch.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import io
from dataclasses import dataclass, field
from typing import BinaryIO, Callable, List, Optional, Union

import numpy as np

from . import geometry
from .reedsolomon import New

HashFn = Callable[[memoryview], bytes]


def sha256_hex(buf) -> bytes:
    return hashlib.sha256(buf).hexdigest().encode()


@dataclass
class SegmentList:
    """types.rs:13-16 — segment hash + fragment hashes in fragment index order."""

    hash: bytes
    fragment_list: List[bytes]

    def to_json(self) -> dict:
        return {"hash": self.hash.decode(), "fragment_list": [f.decode() for f in
                                                              self.fragment_list]}


@dataclass
class FileRecord:
    file_hash: bytes
    size: int
    segments: List[SegmentList] = field(default_factory=list)

    def to_json(self) -> dict:
        return {"file_hash": self.file_hash.decode(), "size": self.size,
                "segments": [s.to_json() for s in self.segments]}


def file_hash(seg_list: List[SegmentList]) -> bytes:
    """SHA-256 hex over the concatenated segment hashes (two-level file hash)."""
    h = hashlib.sha256()
    for sgl in seg_list:
        h.update(sgl.hash)
    return h.hexdigest().encode()


def check_file_spec(seg_list: List[SegmentList],
                    fragment_count: int = geometry.FRAGMENT_COUNT) -> bool:
    """c-pallets/file-bank/src/functions.rs:4-14."""
    return all(len(s.fragment_list) == fragment_count for s in seg_list)


def needed_space(seg_list: List[SegmentList],
                 segment_size: int = geometry.SEGMENT_SIZE) -> int:
    """c-pallets/file-bank/src/lib.rs:440: segments x SEGMENT_SIZE x 15 / 10."""
    return len(seg_list) * (segment_size * 15 // 10)


class _Limited(io.RawIOBase):
    """Read at most `n` bytes from a file object."""

    def __init__(self, f, n: int):
        self.f, self.left = f, n

    def readable(self):
        return True

    def readinto(self, b):
        if self.left <= 0:
            return 0
        mv = memoryview(b)[: self.left]
        n = self.f.readinto(mv)
        self.left -= n or 0
        return n


def encode_file_sharded(path: str, rank: int, world: int, group=None, **kw) -> Optional[FileRecord]:
    """Encode a file across `world` GPU ranks (one process per GPU): rank r encodes a
    contiguous range of segments (distributed.shard_range) with no data exchange, then the
    SegmentLists are gathered on rank 0 (object gather over the process group), which returns
    the whole-file record. Other ranks return None."""
    import os as _os

    from .distributed import shard_range
    seg_size = kw.get("segment_size", geometry.SEGMENT_SIZE)
    size = _os.path.getsize(path)
    nseg = (size + seg_size - 1) // seg_size
    a, b = shard_range(nseg, world, rank)
    part = []
    if b > a:
        se = SegmentEncoder(**kw)
        part = se.encode_range(path, a, b).segments
        se.close()
    if world > 1:
        import torch.distributed as dist
        parts = [None] * world if rank == 0 else None
        dist.gather_object(part, parts, dst=0, group=group)
        if rank != 0:
            return None
    else:
        parts = [part]
    rec = FileRecord(b"", size)
    for p in parts:
        rec.segments.extend(p)
    rec.file_hash = file_hash(rec.segments)
    return rec


class SegmentEncoder:
    """Encode whole files into CESS fragments on one GPU."""

    def __init__(self, k: int = geometry.DATA_SHARDS, m: int = geometry.PARITY_SHARDS,
                 segment_size: int = geometry.SEGMENT_SIZE, batch_segments: int = 64,
                 device: int = 0, hash_on: str = "auto", hash_threads: int = 8):
        import torch
        if segment_size % k:
            raise ValueError("segment_size must be a multiple of k")
        self.k, self.m, self.seg = k, m, segment_size
        self.F = segment_size // k
        self.batch = batch_segments
        self.dev = torch.device("cuda", device)
        self.enc = New(k, m, device=device)
        frags_per_batch = batch_segments * (k + m)
        self.hash_on = ("gpu" if frags_per_batch >= 2048 else "host") if hash_on == "auto" \
            else hash_on
        self.pool = cf.ThreadPoolExecutor(max_workers=hash_threads)
        self.streams = [torch.cuda.Stream(self.dev) for _ in range(2)]
        self.h_data = [torch.empty((batch_segments, k, self.F), dtype=torch.uint8,
                                   pin_memory=True) for _ in range(2)]
        self.h_par = [torch.empty((batch_segments, m, self.F), dtype=torch.uint8,
                                  pin_memory=True) for _ in range(2)]
        self.d_data = [torch.empty((batch_segments, k, self.F), dtype=torch.uint8,
                                   device=self.dev) for _ in range(2)]
        self.d_par = [torch.empty((batch_segments, m, self.F), dtype=torch.uint8,
                                  device=self.dev) for _ in range(2)]
        self.d_hex = [torch.empty((batch_segments, k + m, 64), dtype=torch.uint8,
                                  device=self.dev) for _ in range(2)]
        self.events = [None, None]

    def _read_batch(self, f: BinaryIO, slot: int) -> int:
        """Fill slot's pinned buffer with up to `batch` segments; returns segments read."""
        buf = self.h_data[slot].numpy().reshape(-1)
        got = 0
        cap = self.batch * self.seg
        mv = memoryview(buf)
        while got < cap:
            n = f.readinto(mv[got:cap])
            if not n:
                break
            got += n
        if got == 0:
            return 0
        self._bytes += got
        nseg = (got + self.seg - 1) // self.seg
        if got < nseg * self.seg:  # zero-pad the last segment
            buf[got:nseg * self.seg] = 0
        return nseg

    def _launch(self, slot: int, nseg: int):
        import torch
        st = self.streams[slot]
        with torch.cuda.stream(st):
            self.d_data[slot][:nseg].copy_(self.h_data[slot][:nseg], non_blocking=True)
            self.enc.EncodeBatch(self.d_data[slot], self.d_par[slot], nseg, self.F, stream=st)
            if self.hash_on == "gpu":
                self.enc.Sha256Batch(self.d_data[slot], self.d_par[slot], nseg, self.F,
                                     self.d_hex[slot], stream=st)
            self.h_par[slot][:nseg].copy_(self.d_par[slot][:nseg], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(st)
        self.events[slot] = ev

    def _submit_host_hashes(self, slot: int, nseg: int):
        """Segment hashes (and data-fragment hashes on the host path) need only the host copy:
        start them as soon as the batch is read, beside the GPU work."""
        data = self.h_data[slot].numpy()
        seg_futs = [self.pool.submit(sha256_hex, memoryview(data[s].reshape(-1)))
                    for s in range(nseg)]
        dfuts = None
        if self.hash_on == "host":
            dfuts = [[self.pool.submit(sha256_hex, memoryview(data[s, i]))
                      for i in range(self.k)] for s in range(nseg)]
        return seg_futs, dfuts

    def _finish(self, slot: int, nseg: int, seg_base: int, futs, out: FileRecord,
                on_fragment: Optional[Callable]) -> None:
        data = self.h_data[slot].numpy()
        k, m = self.k, self.m
        seg_futs, dfuts = futs
        self.events[slot].synchronize()
        par = self.h_par[slot].numpy()
        if self.hash_on == "host":
            pfuts = [[self.pool.submit(sha256_hex, memoryview(par[s, o])) for o in range(m)]
                     for s in range(nseg)]
            frag = [[f.result() for f in dfuts[s]] + [f.result() for f in pfuts[s]]
                    for s in range(nseg)]
        else:
            hexes = self.d_hex[slot][:nseg].cpu().numpy()
            frag = [[hexes[s, i].tobytes() for i in range(k + m)] for s in range(nseg)]
        for s in range(nseg):
            out.segments.append(SegmentList(seg_futs[s].result(), frag[s]))
            if on_fragment is not None:
                for i in range(k + m):
                    on_fragment(seg_base + s, i, data[s, i] if i < k else par[s, i - k])

    def encode_range(self, path: str, seg_start: int, seg_stop: int,
                     on_fragment: Optional[Callable[[int, int, np.ndarray], None]] = None
                     ) -> FileRecord:
        """Encode segments [seg_start, seg_stop) of a file (one rank's shard of a file encoded
        across GPUs). `file_hash` of the result covers only this range's segments."""
        with open(path, "rb") as f:
            f.seek(seg_start * self.seg)
            limited = io.BufferedReader(_Limited(f, (seg_stop - seg_start) * self.seg))
            rec = self.encode_file(limited, on_fragment=on_fragment)
        return rec

    def encode_file(self, src: Union[str, bytes, BinaryIO],
                    on_fragment: Optional[Callable[[int, int, np.ndarray], None]] = None
                    ) -> FileRecord:
        """Encode a file (path, bytes or binary stream). `on_fragment(seg, idx, bytes)` sees
        every fragment (e.g. to write it out) before its buffer is reused."""
        if isinstance(src, bytes):
            f, close = io.BytesIO(src), True
        elif isinstance(src, str):
            f, close = open(src, "rb"), True
        else:
            f, close = src, False
        out = FileRecord(b"", 0)
        self._bytes = 0
        try:
            pending = None  # (slot, nseg, seg_base)
            seg_base, slot = 0, 0
            while True:
                nseg = self._read_batch(f, slot)
                futs = None
                if nseg:
                    self._launch(slot, nseg)
                    futs = self._submit_host_hashes(slot, nseg)
                if pending is not None:
                    self._finish(*pending, out, on_fragment)
                if not nseg:
                    break
                pending = (slot, nseg, seg_base, futs)
                seg_base += nseg
                slot ^= 1
        finally:
            if close:
                f.close()
        if not out.segments:
            from .reedsolomon import ErrShortData
            raise ErrShortData(ErrShortData.__doc__)
        out.size = self._bytes
        out.file_hash = file_hash(out.segments)
        return out

    def close(self):
        self.pool.shutdown(wait=True)
        self.enc.close()

