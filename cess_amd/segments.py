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

Pipeline (one GPU): batches of up to 64 segments (1 GiB) go through pinned host buffers into
device slots. Batch i+1's H2D copy and encode overlap the hashing of batch i. Hashes are
computed on the host (OpenSSL SHA-NI via hashlib, threaded) or on the GPU through the hash
queue (cess_amd.hashq), which keeps a window of batches resident in HBM and hashes all their
segment and fragment chains together (see SegmentEncoder).
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


def segment_and_first_fragment_hex(seg2d) -> tuple:
    """(SHA-256 hex of the whole segment, SHA-256 hex of data fragment 0) from ONE pass over
    fragment 0. The split is contiguous (fragment i = segment bytes [i*F, (i+1)*F)), so the
    segment's SHA-256 stream is fragment 0's unpadded stream continued with fragments 1..k-1:
    the fragment-0 digest is taken from a copy of the running state. For the CESS geometry
    (k = 2, F = 8 MiB) this hashes 32 MiB per segment instead of 40 MiB."""
    h = hashlib.sha256(seg2d[0])
    d0 = h.copy().hexdigest().encode()
    for i in range(1, len(seg2d)):
        h.update(seg2d[i])
    return h.hexdigest().encode(), d0


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

    def deal_info_scale(self) -> bytes:
        """SCALE bytes of upload_declaration's deal_info (records.deal_info); raises
        records.ErrTooManySegments past SegmentCount = 1000 segments."""
        from .records import deal_info
        return deal_info(self.segments)

    def upload_declaration(self, account: bytes, file_name: bytes, bucket_name: bytes) -> bytes:
        """Call data of FileBank::upload_declaration for this file (records.upload_declaration)."""
        from .records import upload_declaration
        return upload_declaration(self.file_hash, self.segments, account, file_name,
                                  bucket_name)


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


class _ParallelReader:
    """File-like source whose readinto() fills a large (pinned) buffer with several threads:
    numpy copies and os.preadv release the GIL, so one Python thread's memcpy (~5-10 GB/s) does
    not cap a pipeline that PCIe feeds at ~50 GB/s. Source: a uint8 array or an open fd."""

    def __init__(self, pool: cf.ThreadPoolExecutor, nthreads: int, arr: Optional[np.ndarray]
                 = None, fd: Optional[int] = None, start: int = 0, stop: int = 0):
        self.pool, self.nthreads = pool, max(1, nthreads)
        self.arr, self.fd = arr, fd
        self.pos, self.stop = start, stop

    def _pread(self, mv: memoryview, off: int) -> None:
        import os
        got = 0
        while got < len(mv):
            n = os.preadv(self.fd, [mv[got:]], off + got)
            if n <= 0:
                raise IOError("short read")
            got += n

    def readinto(self, b) -> int:
        mv = memoryview(b).cast("B")
        n = min(len(mv), self.stop - self.pos)
        if n <= 0:
            return 0
        step = max(4 << 20, -(-n // self.nthreads))
        futs = []
        for a in range(0, n, step):
            e = min(n, a + step)
            if self.arr is not None:
                dst = np.frombuffer(mv[a:e], dtype=np.uint8)
                futs.append(self.pool.submit(np.copyto, dst, self.arr[self.pos + a:self.pos + e]))
            else:
                futs.append(self.pool.submit(self._pread, mv[a:e], self.pos + a))
        for fu in futs:
            fu.result()
        self.pos += n
        return n


def encode_file_sharded(path: str, rank: int, world: int, group=None, **kw) -> Optional[FileRecord]:
    """Encode a file across `world` GPU ranks (one process per GPU): rank r encodes a
    contiguous range of segments (distributed.shard_range) with no data exchange through the C
    pipeline (pipeline.RecordsSession: hybrid record hashes by default; keyword arguments as
    RecordsSession's, `device` defaulting to 0), then the SegmentLists are gathered on rank 0
    (object gather over the process group), which returns the whole-file record. Other ranks
    return None."""
    import os as _os

    from .distributed import shard_range
    from .pipeline import RecordsSession
    seg_size = kw.get("segment_size", geometry.SEGMENT_SIZE)
    size = _os.path.getsize(path)
    nseg = (size + seg_size - 1) // seg_size
    a, b = shard_range(nseg, world, rank)
    part = []
    if b > a:
        kw.setdefault("batch_segments", max(1, min(64, b - a)))
        with RecordsSession(**kw) as ses:
            part = ses.encode_range(path, a, b)[0].segments
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
    """Encode whole files into CESS fragments on one GPU.

    hash_on = "host": SHA-256 on the host (libcessec's multi-chain host hasher, `hash_threads`
    threads) beside the GPU encode. hash_on = "gpu": every segment and fragment hash on the GPU through
    the hash queue (cess_amd.hashq): each batch's chains are added after its encode and the
    queue is ticked once per batch, so `window` batches (window x batch_segments x (k+m+1)
    chains) hash together and a batch's records land `window` batches after its encode; the
    window's segments stay resident in HBM until then (288 GB of HBM holds a window of tens of
    GiB). "auto" picks the GPU when a batch alone has >= 2048 fragments (wide codes) or the
    source is known to hold >= AUTO_GPU_BYTES, and the host otherwise (small files of the CESS
    geometry finish sooner on SHA-NI than through the GPU's ~0.5 s per-chain latency for a
    16 MiB segment).
    """

    def __init__(self, k: int = geometry.DATA_SHARDS, m: int = geometry.PARITY_SHARDS,
                 segment_size: int = geometry.SEGMENT_SIZE, batch_segments: int = 64,
                 device: int = 0, hash_on: str = "auto", hash_threads: int = 8,
                 window: int = 32):
        import torch
        if segment_size % k:
            raise ValueError("segment_size must be a multiple of k")
        self.k, self.m, self.seg = k, m, segment_size
        self.F = segment_size // k
        self.batch = batch_segments
        self.dev = torch.device("cuda", device)
        self.enc = New(k, m, device=device)
        frags_per_batch = batch_segments * (k + m)
        if hash_on not in ("gpu", "host", "auto"):
            raise ValueError("hash_on must be 'gpu', 'host' or 'auto'")
        self.hash_mode = hash_on
        self.wide = frags_per_batch >= 2048
        self.window = max(1, window)
        self.hash_threads = hash_threads
        self.pool = cf.ThreadPoolExecutor(max_workers=4)  # host SHA-256 jobs (their threads: C)
        self.io_threads = 8
        self.io_pool = cf.ThreadPoolExecutor(max_workers=self.io_threads)
        self.streams = [torch.cuda.Stream(self.dev) for _ in range(2)]
        self.h_data = [torch.empty((batch_segments, k, self.F), dtype=torch.uint8,
                                   pin_memory=True) for _ in range(2)]
        self.h_par = [torch.empty((batch_segments, m, self.F), dtype=torch.uint8,
                                  pin_memory=True) for _ in range(2)]
        self.events = [None, None]
        self.hash_on = None
        self.hq = None
        self._configure("gpu" if hash_on == "gpu" or (hash_on == "auto" and self.wide)
                        else "host")

    # "auto" hashes on the GPU for wide codes, and for the CESS geometry once the source is known
    # to be at least this large: a 16 MiB segment chain has ~0.5 s of latency on the GPU, so small
    # files finish sooner on SHA-NI (measured e2e with the shared segment/fragment-0 stream on the
    # host: host 16.1 vs GPU 12.8 GB/s at 8 GiB, host 15.1 vs GPU 17.2 at 12 GiB, GPU 34.7 at
    # 64 GiB; DESIGN.md §5, profiles/r01/e2e_host_shared_stream.txt)
    AUTO_GPU_BYTES = 10 << 30

    def _configure(self, mode: str) -> None:
        """(Re)allocate the device slots (and the hash queue) for a hash placement."""
        import torch
        if mode == self.hash_on:
            return
        if self.hq is not None:
            self.hq.close()
            self.hq = None
        self.d_data = self.d_par = None
        torch.cuda.synchronize(self.dev)
        k, m, F, nb = self.k, self.m, self.F, self.batch
        self.hash_on = mode
        self.W = self.window if mode == "gpu" else 2
        # GPU hashing: W + 1 device slots, so the slot a batch reuses was freed one tick
        # before, and its H2D + encode overlap the current tick
        nd = self.W + 1 if mode == "gpu" else 2
        self.d_data = [torch.empty((nb, k, F), dtype=torch.uint8, device=self.dev)
                       for _ in range(nd)]
        self.d_par = [torch.empty((nb, m, F), dtype=torch.uint8, device=self.dev)
                      for _ in range(nd)]
        if mode == "gpu":
            from .hashq import HashQueue, sha256_blocks
            self.hash_stream = torch.cuda.Stream(self.dev)
            chains = self.W * nb * (k + m + 1)
            self.hq = HashQueue(capacity=1 << max(10, (chains - 1).bit_length()),
                                device=self.dev.index, stream=self.hash_stream)
            # a segment chain completes `window` ticks after its add
            self.tick_blocks = -(-sha256_blocks(self.seg) // self.W)
            self.d_fhex = [torch.empty((nb, k + m, 64), dtype=torch.uint8, device=self.dev)
                           for _ in range(nd)]
            self.d_shex = [torch.empty((nb, 64), dtype=torch.uint8, device=self.dev)
                           for _ in range(nd)]
            self.h_fhex = [torch.empty((nb, k + m, 64), dtype=torch.uint8, pin_memory=True)
                           for _ in range(nd)]
            self.h_shex = [torch.empty((nb, 64), dtype=torch.uint8, pin_memory=True)
                           for _ in range(nd)]
            self.slot_free = [None] * nd  # event: slot's hashes copied out (slot reusable)

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

    def _launch(self, slot: int, dslot: int, nseg: int):
        import torch
        st = self.streams[slot]
        with torch.cuda.stream(st):
            if self.hash_on == "gpu" and self.slot_free[dslot] is not None:
                st.wait_event(self.slot_free[dslot])  # batch dslot - W fully hashed
            self.d_data[dslot][:nseg].copy_(self.h_data[slot][:nseg], non_blocking=True)
            self.enc.EncodeBatch(self.d_data[dslot], self.d_par[dslot], nseg, self.F, stream=st)
            if self.hash_on == "gpu":
                ready = torch.cuda.Event()
                ready.record(st)
            self.h_par[slot][:nseg].copy_(self.d_par[dslot][:nseg], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(st)
        self.events[slot] = ev
        if self.hash_on == "gpu":
            k, m, F = self.k, self.m, self.F
            self.hash_stream.wait_event(ready)
            # segment chains also give data fragment 0's hash (prefix digest, cec_hashq_add_prefix)
            return self.hq.add_segment_lists(self.d_data[dslot], self.d_par[dslot], nseg, k, m, F,
                                             self.d_shex[dslot], self.d_fhex[dslot])
        return None

    def _copy_hashes(self, dslot: int, nseg: int):
        """Enqueue the D2H of a completed batch's hex (on the hash stream, after its tick)."""
        import torch
        with torch.cuda.stream(self.hash_stream):
            self.h_fhex[dslot][:nseg].copy_(self.d_fhex[dslot][:nseg], non_blocking=True)
            self.h_shex[dslot][:nseg].copy_(self.d_shex[dslot][:nseg], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.hash_stream)
        self.slot_free[dslot] = ev
        return ev

    def _submit_host_hashes(self, slot: int, nseg: int):
        """Host path: segment and data-fragment hashes need only the host copy, so they start
        as soon as the batch is read, beside the GPU work: one libcessec host SHA-256 job each
        (cec_sha256_host, multi-chain) for the segment chains, which give data fragment 0's hash
        as their prefix digest, and for the other data fragments."""
        if self.hash_on != "host":
            return None
        from .reedsolomon import sha256_hex_host
        data = self.h_data[slot].numpy()
        k, F, th = self.k, self.F, self.hash_threads
        prefix = F if F % 64 == 0 else 0
        seg_fut = self.pool.submit(sha256_hex_host, [data[s].reshape(-1) for s in range(nseg)],
                                   self.seg, th, prefix)
        d0 = 0 if prefix else 1  # without the prefix trick fragment 0 is hashed on its own
        dfut = self.pool.submit(sha256_hex_host, [data[s, i] for s in range(nseg)
                                                  for i in range(1 - d0, k)], F, th)
        return seg_fut, dfut, prefix

    def _finish_encode(self, slot: int, nseg: int, seg_base: int, futs,
                       on_fragment: Optional[Callable]):
        """Wait for a batch's encode + parity D2H; run the fragment callback; on the host path
        also collect its hashes (returns the batch's SegmentLists then, else None)."""
        data = self.h_data[slot].numpy()
        k, m = self.k, self.m
        self.events[slot].synchronize()
        par = self.h_par[slot].numpy()
        recs = None
        if self.hash_on == "host":
            from .reedsolomon import sha256_hex_host
            seg_fut, dfut, prefix = futs
            phex = sha256_hex_host([par[s, o] for s in range(nseg) for o in range(m)], self.F,
                                   self.hash_threads)
            seg_res, dhex = seg_fut.result(), dfut.result()
            shex, d0hex = seg_res if prefix else (seg_res, None)
            nd = k - 1 if prefix else k  # data fragments hashed on their own, per segment
            recs = []
            for s in range(nseg):
                frags = ([d0hex[s]] if prefix else []) + dhex[s * nd:(s + 1) * nd]
                recs.append(SegmentList(shex[s], frags + phex[s * m:(s + 1) * m]))
        if on_fragment is not None:
            for s in range(nseg):
                for i in range(k + m):
                    on_fragment(seg_base + s, i, data[s, i] if i < k else par[s, i - k])
        return recs

    def _gpu_records(self, dslot: int, nseg: int, ev) -> List[SegmentList]:
        ev.synchronize()
        fh = self.h_fhex[dslot][:nseg].numpy()
        sh = self.h_shex[dslot][:nseg].numpy()
        return [SegmentList(sh[s].tobytes(), [fh[s, i].tobytes() for i in range(self.k + self.m)])
                for s in range(nseg)]

    def encode_range(self, path: str, seg_start: int, seg_stop: int,
                     on_fragment: Optional[Callable[[int, int, np.ndarray], None]] = None
                     ) -> FileRecord:
        """Encode segments [seg_start, seg_stop) of a file (one rank's shard of a file encoded
        across GPUs). `file_hash` of the result covers only this range's segments."""
        import os
        fd = os.open(path, os.O_RDONLY)
        try:
            size = os.fstat(fd).st_size
            src = _ParallelReader(self.io_pool, self.io_threads, fd=fd, start=seg_start * self.seg,
                                  stop=min(size, seg_stop * self.seg))
            rec = self.encode_file(src, on_fragment=on_fragment)
        finally:
            os.close(fd)
        return rec

    def encode_file(self, src: Union[str, bytes, BinaryIO],
                    on_fragment: Optional[Callable[[int, int, np.ndarray], None]] = None
                    ) -> FileRecord:
        """Encode a file (path, bytes / uint8 array, or binary stream). `on_fragment(seg, idx, bytes)` sees
        every fragment (e.g. to write it out) before its buffer is reused; on the GPU hash path
        it runs before the fragment's hash is known."""
        close_fd = None
        if isinstance(src, (bytes, bytearray, memoryview, np.ndarray)):
            arr = np.frombuffer(src, dtype=np.uint8) if not isinstance(src, np.ndarray) \
                else src.reshape(-1).view(np.uint8)
            f, close = _ParallelReader(self.io_pool, self.io_threads, arr=arr, stop=arr.size), False
        elif isinstance(src, str):
            import os
            close_fd = os.open(src, os.O_RDONLY)
            f = _ParallelReader(self.io_pool, self.io_threads, fd=close_fd,
                                stop=os.fstat(close_fd).st_size)
            close = False
        else:
            f, close = src, False
        if self.hash_mode == "auto" and not self.wide:
            size = f.stop - f.pos if isinstance(f, _ParallelReader) else None
            self._configure("gpu" if size is not None and size >= self.AUTO_GPU_BYTES
                            else "host")
        out = FileRecord(b"", 0)
        self._bytes = 0
        gpu = self.hash_on == "gpu"
        inflight = []  # GPU path: [batch no, dslot, nseg, ticket, copy event or None]
        try:
            pending = None  # (slot, nseg, seg_base, futs)
            seg_base, i = 0, 0
            while True:
                slot = i & 1
                nseg = self._read_batch(f, slot)
                futs = None
                if nseg:
                    dslot = i % len(self.d_data)
                    if gpu:  # the slot's previous batch must be hashed and copied out first
                        for b in inflight:
                            if b[1] == dslot and b[4] is None:
                                while not self.hq.done(b[3]):
                                    self.hq.tick(self.tick_blocks)
                                b[4] = self._copy_hashes(b[1], b[2])
                    ticket = self._launch(slot, dslot, nseg)
                    futs = self._submit_host_hashes(slot, nseg)
                    if gpu:
                        inflight.append([i, dslot, nseg, ticket, None])
                        self.hq.tick(self.tick_blocks)
                if gpu and not nseg:
                    self.hq.finish()
                if gpu:
                    for b in inflight:
                        if b[4] is None and self.hq.done(b[3]):
                            b[4] = self._copy_hashes(b[1], b[2])
                if pending is not None:
                    recs = self._finish_encode(*pending, on_fragment)
                    if recs is not None:
                        out.segments.extend(recs)
                # GPU records in batch order, once their hex copies are enqueued; the slot is
                # reused W batches later, so wait for the oldest before it is overwritten
                while gpu and inflight and inflight[0][4] is not None and (
                        not nseg or len(inflight) >= len(self.d_data) or inflight[0][4].query()):
                    _, dslot_, nseg_, _, ev = inflight.pop(0)
                    out.segments.extend(self._gpu_records(dslot_, nseg_, ev))
                if not nseg:
                    break
                pending = (slot, nseg, seg_base, futs)
                seg_base += nseg
                i += 1
        finally:
            if close:
                f.close()
            if close_fd is not None:
                import os
                os.close(close_fd)
        if not out.segments:
            from .reedsolomon import ErrShortData
            raise ErrShortData(ErrShortData.__doc__)
        out.size = self._bytes
        out.file_hash = file_hash(out.segments)
        return out

    def close(self):
        self.pool.shutdown(wait=True)
        self.io_pool.shutdown(wait=True)
        if self.hq is not None:
            self.hq.close()
            self.hq = None
        self.enc.close()
