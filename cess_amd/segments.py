"""File -> segments -> fragments -> `SegmentList` records.

What the chain consumes (reference):
  * `SegmentList { hash, fragment_list: BoundedVec<Hash, FragmentCount> }`
    (c-pallets/file-bank/src/types.rs:13-16), one per 16 MiB segment, submitted with
    `upload_declaration(file_hash, deal_info, user_brief)` (c-pallets/file-bank/src/lib.rs:423);
  * `check_file_spec`: every fragment_list has FragmentCount entries (functions.rs:4-14);
  * space locked = segments x SEGMENT_SIZE x 15 / 10 (lib.rs:440);
  * `Hash([u8; 64])` (primitives/common/src/lib.rs:16).
Hash convention [ecosystem, unpinned by the reference]: 64 lowercase hex chars of SHA-256; the
last segment is zero padded to SEGMENT_SIZE; the file hash is SHA-256 of the file bytes.

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


def check_file_spec(seg_list: List[SegmentList],
                    fragment_count: int = geometry.FRAGMENT_COUNT) -> bool:
    """c-pallets/file-bank/src/functions.rs:4-14."""
    return all(len(s.fragment_list) == fragment_count for s in seg_list)


def needed_space(seg_list: List[SegmentList],
                 segment_size: int = geometry.SEGMENT_SIZE) -> int:
    """c-pallets/file-bank/src/lib.rs:440: segments x SEGMENT_SIZE x 15 / 10."""
    return len(seg_list) * (segment_size * 15 // 10)


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

    def _read_batch(self, f: BinaryIO, slot: int, file_hash) -> int:
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
        file_hash.update(mv[:got])
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

    def _finish(self, slot: int, nseg: int, seg_base: int, out: FileRecord,
                on_fragment: Optional[Callable]) -> None:
        data = self.h_data[slot].numpy()
        k, m = self.k, self.m
        # segment hashes (and data-fragment hashes on the host path) need only host data,
        # so they start before the GPU batch completes
        seg_futs = [self.pool.submit(sha256_hex, memoryview(data[s].reshape(-1)))
                    for s in range(nseg)]
        dfuts = None
        if self.hash_on == "host":
            dfuts = [[self.pool.submit(sha256_hex, memoryview(data[s, i])) for i in range(k)]
                     for s in range(nseg)]
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
        fh = hashlib.sha256()
        out = FileRecord(b"", 0)
        self._bytes = 0
        try:
            pending = None  # (slot, nseg, seg_base)
            seg_base, slot = 0, 0
            while True:
                nseg = self._read_batch(f, slot, fh)
                if nseg:
                    self._launch(slot, nseg)
                if pending is not None:
                    self._finish(*pending, out, on_fragment)
                if not nseg:
                    break
                pending = (slot, nseg, seg_base)
                seg_base += nseg
                slot ^= 1
        finally:
            if close:
                f.close()
        if not out.segments:
            from .reedsolomon import ErrShortData
            raise ErrShortData(ErrShortData.__doc__)
        out.size = self._bytes
        out.file_hash = fh.hexdigest().encode()
        return out

    def close(self):
        self.pool.shutdown(wait=True)
        self.enc.close()

