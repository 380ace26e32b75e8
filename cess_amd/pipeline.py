"""Python mirror of libcessec's host pipeline (include/cess_ec.h `cec_pipeline_*`): a file in host
memory -> segments -> fragments + SegmentList hashes through one GPU, with the pinned
hipMemcpyAsync multi-buffering done in C++ (cess_amd/csrc/pipeline.cpp).

The records it produces are `SegmentList { hash, fragment_list }`
(c-pallets/file-bank/src/types.rs:13-16) for FileBank::upload_declaration
(c-pallets/file-bank/src/lib.rs:419-428). Callbacks run on the calling thread; a Python exception
raised in one aborts the run and is re-raised here.
"""
from __future__ import annotations

import concurrent.futures as cf
import ctypes
import os
from ctypes import byref, c_void_p
from typing import BinaryIO, Callable, Optional, Union

import numpy as np

from . import _lib, geometry
from .reedsolomon import CecError, Encoder, check

Source = Union[str, bytes, bytearray, memoryview, np.ndarray, BinaryIO]


class _Reader:
    """read() callback over a path (parallel os.preadv, GIL released), an in-memory buffer
    (parallel numpy copies) or a binary stream (readinto)."""

    def __init__(self, src: Source, threads: int = 8, start: int = 0,
                 stop: Optional[int] = None):
        self.pool = cf.ThreadPoolExecutor(max_workers=threads)
        self.threads = threads
        self.fd = self.arr = self.stream = None
        self.pos = 0
        if isinstance(src, str):
            self.fd = os.open(src, os.O_RDONLY)
            self.size = os.fstat(self.fd).st_size
            self.pos = start  # absolute offsets in the file: bytes [start, stop)
            if stop is not None:
                self.size = min(self.size, stop)
        elif isinstance(src, (bytes, bytearray, memoryview, np.ndarray)):
            arr = (src.reshape(-1).view(np.uint8) if isinstance(src, np.ndarray)
                   else np.frombuffer(src, np.uint8))
            self.arr = arr[start:stop]
            self.size = self.arr.size
        else:
            if start or stop is not None:
                raise ValueError("a byte range needs a path or an in-memory source")
            self.stream = src
            self.size = None

    def _pread(self, mv: memoryview, off: int) -> None:
        got = 0
        while got < len(mv):
            n = os.preadv(self.fd, [mv[got:]], off + got)
            if n <= 0:
                raise IOError("short read")
            got += n

    def __call__(self, dst: int, cap: int) -> int:
        mv = memoryview((ctypes.c_uint8 * cap).from_address(dst)).cast("B")
        if self.stream is not None:
            n = self.stream.readinto(mv)
            return n or 0
        n = min(cap, self.size - self.pos)
        if n <= 0:
            return 0
        step = max(4 << 20, -(-n // self.threads))
        futs = []
        for a in range(0, n, step):
            e = min(n, a + step)
            if self.arr is not None:
                futs.append(self.pool.submit(np.copyto, np.frombuffer(mv[a:e], np.uint8),
                                             self.arr[self.pos + a:self.pos + e]))
            else:
                futs.append(self.pool.submit(self._pread, mv[a:e], self.pos + a))
        for f in futs:
            f.result()
        self.pos += n
        return n

    def close(self) -> None:
        self.pool.shutdown(wait=True)
        if self.fd is not None:
            os.close(self.fd)
            self.fd = None


class Pipeline:
    """cec_pipeline bound to one codec: `depth` pinned host batches of `batch_segments`
    segments, GPU SegmentList hashing over a window of `window` batches when hash=True."""

    def __init__(self, enc: Encoder, shard_len: int = geometry.FRAGMENT_SIZE,
                 batch_segments: int = 64, depth: int = 3, hash: bool = True, window: int = 32,
                 max_segments: int = 0):
        self.enc = enc
        self.k, self.m = enc.DataShards, enc.ParityShards
        self.F = shard_len
        self.opts = _lib.PipelineOpts(shard_len, batch_segments, depth, 1 if hash else 0, window,
                                      max_segments)
        self._lib = enc._lib
        self._h = c_void_p()
        check(self._lib.cec_pipeline_create(enc._h, byref(self.opts), byref(self._h)),
              "Pipeline")

    def close(self) -> None:
        if self._h:
            self._lib.cec_pipeline_destroy(self._h)
            self._h = c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def run(self, src: Source,
            on_fragments: Optional[Callable[[int, list], None]] = None,
            on_record: Optional[Callable[[int, bytes, list], None]] = None,
            read_threads: int = 8, start: int = 0,
            stop: Optional[int] = None) -> _lib.PipelineStats:
        """Stream `src` (bytes [start, stop) of a path or an in-memory buffer) through the GPU.
        on_fragments(seg, [k+m uint8 views]) sees every segment's shards (views valid during the
        call only; seg counts from the range's first segment); on_record(seg, seg_hex,
        [k+m fragment hex]) its hashes (hash=True). Returns the run's PipelineStats."""
        n = self.k + self.m
        F = self.F
        reader = _Reader(src, read_threads, start, stop)
        err = []

        def rd(_u, dst, cap):
            try:
                return reader(dst, cap)
            except BaseException as e:  # noqa: BLE001 - re-raised after the C call returns
                err.append(e)
                return -1

        def fr(_u, seg, shards, _len):
            try:
                views = [np.ctypeslib.as_array((ctypes.c_uint8 * F).from_address(shards[i]))
                         for i in range(n)]
                on_fragments(seg, views)
                return 0
            except BaseException as e:  # noqa: BLE001
                err.append(e)
                return -1

        def rc_(_u, seg, seg_hex, frag_hex):
            try:
                fh = ctypes.string_at(frag_hex, 64 * n)
                on_record(seg, ctypes.string_at(seg_hex, 64),
                          [fh[64 * i:64 * (i + 1)] for i in range(n)])
                return 0
            except BaseException as e:  # noqa: BLE001
                err.append(e)
                return -1

        cb_read = _lib.READ_FN(rd)
        cb_frag = _lib.FRAGMENTS_FN(fr) if on_fragments else _lib.FRAGMENTS_FN()
        cb_rec = _lib.RECORD_FN(rc_) if on_record else _lib.RECORD_FN()
        stats = _lib.PipelineStats()
        try:
            rc = self._lib.cec_pipeline_run(self._h, cb_read, cb_frag, cb_rec, None, byref(stats))
        finally:
            reader.close()
        if err:
            raise err[0]
        if rc == _lib.CEC_ESEGCOUNT:
            from .records import ErrTooManySegments
            raise ErrTooManySegments(ErrTooManySegments.__doc__)
        check(rc, "Pipeline.run")
        return stats


def _source_size(src: Source) -> Optional[int]:
    if isinstance(src, str):
        return os.path.getsize(src)
    if isinstance(src, (np.ndarray, memoryview)):
        return src.nbytes
    if isinstance(src, (bytes, bytearray)):
        return len(src)
    return None  # a stream


# encode_file_records(hash_on="auto") hashes on the GPU from this size up. Measured fresh per
# call, RS(2,1), 16 host threads (profiles/r05/records_crossover.jsonl): the GPU path pays
# ~0.3 s pinning + ~0.3 s unpinning its 4.5 GiB ring and the last segment chain (0.5 s when the
# chip is busy, 1.15 s for a lone one-segment file), so the host wins up to 16 GiB (1.26 s
# against 1.43) and the GPU from 32 GiB (1.75 s against 2.28; 30 GB/s against 15.6 at 64 GiB).
# CESS's SegmentCount = 1000 segments (15.6 GiB) keeps every declarable file on the host.
AUTO_GPU_RECORD_BYTES = 20 << 30


def record_hash_placement(hash_on: str, size: Optional[int], k: int, m: int) -> str:
    """"gpu" or "host" for encode_file_records' hash_on ("auto" resolved by source size and
    code width: a batch of >= 2048 fragments keeps the GPU's hash lanes busy)."""
    if hash_on != "auto":
        return hash_on
    return "host" if (size is not None and size < AUTO_GPU_RECORD_BYTES
                      and 64 * (k + m) < 2048) else "gpu"


def encode_file_records(path_or_buf: Source, k: int = geometry.DATA_SHARDS,
                        m: int = geometry.PARITY_SHARDS,
                        segment_size: int = geometry.SEGMENT_SIZE, device: int = 0,
                        on_fragment: Optional[Callable[[int, int, np.ndarray], None]] = None,
                        max_segments: int = 0, hash_on: str = "gpu", hash_threads: int = 16,
                        **kw):
    """File -> FileRecord (SegmentLists + two-level file hash), encoded on the GPU.
    on_fragment(seg, idx, view) sees each fragment (before its hash is known on the GPU path).

    hash_on "gpu": the C pipeline (pinned multi-buffered copies, SegmentList hashes through the
    GPU hash queue); a file's records land one 16 MiB segment chain (~0.47 s) after its last
    batch. "host": SegmentEncoder with SHA-256 (OpenSSL SHA-NI) on `hash_threads` host threads
    beside the GPU encode. "auto": the host below AUTO_GPU_RECORD_BYTES for codes whose batch
    holds < 2048 fragments, the GPU otherwise and for streams of unknown size. The records are
    the same either way."""
    from .segments import FileRecord, SegmentList, file_hash
    if segment_size % k:
        raise ValueError("segment_size must be a multiple of k")
    if hash_on not in ("gpu", "host", "auto"):
        raise ValueError("hash_on must be 'gpu', 'host' or 'auto'")
    size = _source_size(path_or_buf)
    hash_on = record_hash_placement(hash_on, size, k, m)
    if hash_on == "host":
        return _encode_file_records_host(path_or_buf, size, k, m, segment_size, device,
                                         on_fragment, max_segments, hash_threads,
                                         kw.get("batch_segments"))
    recs = {}
    if size is not None:  # a small file does not need 1 GiB pinned batches
        # (the window stays: a chain finishes after `window` ticks of blocks/window each, so a
        # narrower window only makes each tick coarser; measured 1.52 s against 1.11 at 8 GiB)
        kw.setdefault("batch_segments", max(1, min(64, -(-size // segment_size))))
    enc = Encoder(k, m, device)
    try:
        with Pipeline(enc, segment_size // k, max_segments=max_segments, **kw) as p:
            def frags(seg, views):
                for i, v in enumerate(views):
                    on_fragment(seg, i, v)

            st = p.run(path_or_buf, frags if on_fragment else None,
                       lambda seg, sh, fl: recs.__setitem__(seg, SegmentList(sh, fl)))
    finally:
        enc.close()
    if not recs:
        from .reedsolomon import ErrShortData
        raise ErrShortData(ErrShortData.__doc__)
    out = FileRecord(b"", int(st.bytes_in), [recs[s] for s in range(len(recs))])
    out.file_hash = file_hash(out.segments)
    return out, st


def _encode_file_records_host(src, size, k, m, segment_size, device, on_fragment, max_segments,
                              hash_threads, batch_segments=None):
    """encode_file_records' host-hash path: SegmentEncoder (GPU encode, pinned double-buffered
    batches sized to the file unless batch_segments is given, SHA-256 on host threads; the C
    pipeline's other options do not apply). Returns (FileRecord, PipelineStats)."""
    import time

    from .segments import SegmentEncoder
    if size is None:
        raise ValueError("hash_on='host' needs a path or an in-memory source (known size)")
    nseg = -(-size // segment_size)
    if size == 0:
        from .reedsolomon import ErrShortData
        raise ErrShortData(ErrShortData.__doc__)
    if max_segments and nseg > max_segments:
        from .records import ErrTooManySegments
        raise ErrTooManySegments(ErrTooManySegments.__doc__)
    t0 = time.perf_counter()
    se = SegmentEncoder(k, m, segment_size, batch_segments=batch_segments or min(64, nseg),
                        device=device, hash_on="host", hash_threads=hash_threads)
    try:
        rec = se.encode_file(src, on_fragment=on_fragment)
    finally:
        se.close()
    st = _lib.PipelineStats(len(rec.segments), rec.size, time.perf_counter() - t0, 0.0, 0.0)
    return rec, st


def encode_file_records_multi(src: Union[str, bytes, bytearray, memoryview, np.ndarray],
                              devices, k: int = geometry.DATA_SHARDS,
                              m: int = geometry.PARITY_SHARDS,
                              segment_size: int = geometry.SEGMENT_SIZE,
                              max_segments: int = 0, read_threads: int = 8, **kw):
    """File -> FileRecord with the segments sharded over several GPUs from ONE host process (an
    uploader on a multi-GPU node): contiguous segment ranges per device
    (distributed.shard_range; segments are independent, no data exchange), one C pipeline per
    device on its own host thread (pinned multi-buffered copies per GPU), records merged in
    segment order. `devices` may repeat a device (several pipelines sharing one GPU).
    Returns (FileRecord, [PipelineStats per device])."""
    from .distributed import shard_range
    from .segments import FileRecord, SegmentList, file_hash
    size = os.path.getsize(src) if isinstance(src, str) else (
        src.nbytes if isinstance(src, np.ndarray) else len(src))
    if size == 0:
        from .reedsolomon import ErrShortData
        raise ErrShortData(ErrShortData.__doc__)
    nseg = -(-size // segment_size)
    if max_segments and nseg > max_segments:
        from .records import ErrTooManySegments
        raise ErrTooManySegments(ErrTooManySegments.__doc__)
    devices = list(devices)
    kw.setdefault("batch_segments", max(1, min(64, -(-nseg // len(devices)))))

    def work(i):
        a, b = shard_range(nseg, len(devices), i)
        if b <= a:
            return {}, None
        recs = {}
        enc = Encoder(k, m, devices[i])
        try:
            with Pipeline(enc, segment_size // k, **kw) as p:
                st = p.run(src, on_record=lambda s, sh, fl: recs.__setitem__(
                    a + s, SegmentList(sh, fl)), read_threads=read_threads,
                    start=a * segment_size, stop=min(size, b * segment_size))
        finally:
            enc.close()
        return recs, st

    with cf.ThreadPoolExecutor(max_workers=len(devices)) as ex:
        parts = list(ex.map(work, range(len(devices))))
    recs = {}
    for r, _ in parts:
        recs.update(r)
    out = FileRecord(b"", size, [recs[s] for s in range(nseg)])
    out.file_hash = file_hash(out.segments)
    return out, [st for _, st in parts if st is not None]


__all__ = ["Pipeline", "encode_file_records", "encode_file_records_multi", "CecError",
           "AUTO_GPU_RECORD_BYTES", "record_hash_placement"]
