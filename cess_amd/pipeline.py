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


def _as_u8(x) -> np.ndarray:
    return x.reshape(-1).view(np.uint8) if isinstance(x, np.ndarray) else np.frombuffer(x,
                                                                                      np.uint8)


class _Reader:
    """read() callback over a path (parallel os.preadv, GIL released), an in-memory buffer
    (parallel numpy copies), a list of in-memory buffers read back to back as one file (pieces
    gathered from elsewhere, no joined copy) or a binary stream (readinto)."""

    def __init__(self, src: Source, threads: int = 8, start: int = 0,
                 stop: Optional[int] = None, pool: Optional[cf.ThreadPoolExecutor] = None):
        self.own_pool = pool is None
        self.pool = pool or cf.ThreadPoolExecutor(max_workers=threads)
        self.threads = threads
        self.fd = self.arr = self.stream = self.parts = None
        self.pos = 0
        if isinstance(src, str):
            self.fd = os.open(src, os.O_RDONLY)
            self.size = os.fstat(self.fd).st_size
            self.pos = start  # absolute offsets in the file: bytes [start, stop)
            if stop is not None:
                self.size = min(self.size, stop)
        elif isinstance(src, (bytes, bytearray, memoryview, np.ndarray)):
            self.arr = _as_u8(src)[start:stop]
            self.size = self.arr.size
        elif isinstance(src, (list, tuple)):
            if start or stop is not None:
                raise ValueError("a byte range needs a path or a single in-memory buffer")
            self.parts = [_as_u8(x) for x in src]
            self.size = sum(x.size for x in self.parts)
        else:
            if start or stop is not None:
                raise ValueError("a byte range needs a path or an in-memory source")
            self.stream = src
            self.size = None
        # bytes this reader yields in all (None for a stream)
        self.nbytes = None if self.size is None else max(0, self.size - self.pos)

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
        if self.parts is not None:  # copy runs of the pieces that cover [pos, pos + n)
            off, done = self.pos, 0
            for x in self.parts:
                if off >= x.size:
                    off -= x.size
                    continue
                take = min(x.size - off, n - done)
                for a in range(0, take, step):
                    e = min(take, a + step)
                    futs.append(self.pool.submit(np.copyto, np.frombuffer(
                        mv[done + a:done + e], np.uint8), x[off + a:off + e]))
                done += take
                off = 0
                if done == n:
                    break
        for a in range(0, n if self.parts is None else 0, step):
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
        if self.own_pool:
            self.pool.shutdown(wait=True)
        if self.fd is not None:
            os.close(self.fd)
            self.fd = None


HASH_MODES = {False: _lib.CEC_PIPE_HASH_NONE, True: _lib.CEC_PIPE_HASH_GPU,
              "none": _lib.CEC_PIPE_HASH_NONE, "gpu": _lib.CEC_PIPE_HASH_GPU,
              "host": _lib.CEC_PIPE_HASH_HOST, "hybrid": _lib.CEC_PIPE_HASH_HYBRID}


class Pipeline:
    """cec_pipeline bound to one codec: `depth` pinned host batches of `batch_segments`
    segments; SegmentList hashes where `hash` says: "gpu" (True; the GPU hash queue over a window
    of `window` batches), "host" (`host_threads` host threads, cec_sha256_host), "hybrid" (the
    segment chains on the host, the other fragments on the GPU queue, the last `tail_batches`
    batches of a run's last source wholly on the host; -1 = auto) or "none" (False)."""

    def __init__(self, enc: Encoder, shard_len: int = geometry.FRAGMENT_SIZE,
                 batch_segments: int = 64, depth: int = 3, hash=True, window: int = 0,
                 max_segments: int = 0, host_threads: int = 16, tail_batches: int = -1):
        self.enc = enc
        self.k, self.m = enc.DataShards, enc.ParityShards
        self.F = shard_len
        if hash not in HASH_MODES:
            raise ValueError("hash must be one of " + ", ".join(map(repr, HASH_MODES)))
        self.mode = HASH_MODES[hash]
        self.opts = _lib.PipelineOpts(shard_len, batch_segments, depth, self.mode, window,
                                      max_segments, host_threads, tail_batches)
        self._lib = enc._lib
        self._h = c_void_p()
        check(self._lib.cec_pipeline_create(enc._h, byref(self.opts), byref(self._h)),
              "Pipeline")

    def info(self) -> dict:
        """The window the pipeline settled on (fitted to free HBM), device slots, host batches."""
        w, nd, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(self._lib.cec_pipeline_info(self._h, byref(w), byref(nd), byref(d)),
              "Pipeline.info")
        return {"window": w.value, "device_slots": nd.value, "depth": d.value}

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
        [k+m fragment hex]) its hashes. Returns the run's PipelineStats."""
        fr = (lambda _f, seg, views: on_fragments(seg, views)) if on_fragments else None
        rc_ = (lambda _f, seg, sh, fl: on_record(seg, sh, fl)) if on_record else None
        return self.run_files([src], fr, rc_, None, read_threads, [(start, stop)])

    def run_files(self, srcs, on_fragments: Optional[Callable[[int, int, list], None]] = None,
                  on_record: Optional[Callable[[int, int, bytes, list], None]] = None,
                  on_done: Optional[Callable[[int, _lib.PipelineStats], None]] = None,
                  read_threads: int = 8, ranges=None) -> _lib.PipelineStats:
        """Several sources in one run (cec_pipeline_run_files): the pipeline stays full across
        files, each file's records come in segment order and on_done(file, stats) once its last
        record is out (in file order) while later files already stream. Callbacks take the file's
        index first: on_fragments(file, seg, views), on_record(file, seg, seg_hex, [hex]).
        `ranges`: optional (start, stop) byte range per source. Returns the run's stats."""
        n = self.k + self.m
        F = self.F
        readers = []
        err = []
        pool = cf.ThreadPoolExecutor(max_workers=read_threads)  # shared by the sources' readers
        try:
            for i, src in enumerate(srcs):
                a, b = ranges[i] if ranges else (0, None)
                readers.append(_Reader(src, read_threads, a, b, pool))
        except BaseException:
            for r in readers:
                r.close()
            pool.shutdown(wait=True)
            raise

        def make_read(reader):
            def rd(_u, dst, cap):
                try:
                    return reader(dst, cap)
                except BaseException as e:  # noqa: BLE001 - re-raised after the C call returns
                    err.append(e)
                    return -1
            return _lib.READ_FN(rd)

        def fr(_u, f, seg, shards, _len):
            try:
                views = [np.ctypeslib.as_array((ctypes.c_uint8 * F).from_address(shards[i]))
                         for i in range(n)]
                on_fragments(f, seg, views)
                return 0
            except BaseException as e:  # noqa: BLE001
                err.append(e)
                return -1

        def rc_(_u, f, seg, seg_hex, frag_hex):
            try:
                fh = ctypes.string_at(frag_hex, 64 * n)
                on_record(f, seg, ctypes.string_at(seg_hex, 64),
                          [fh[64 * i:64 * (i + 1)] for i in range(n)])
                return 0
            except BaseException as e:  # noqa: BLE001
                err.append(e)
                return -1

        def dn(_u, f, st):
            try:
                on_done(f, st.contents)
                return 0
            except BaseException as e:  # noqa: BLE001
                err.append(e)
                return -1

        cbs = [make_read(r) for r in readers]
        arr = (_lib.Source * max(1, len(readers)))()
        for i, r in enumerate(readers):
            arr[i].read = cbs[i]
            arr[i].user = None
            arr[i].size = r.nbytes or 0
        cb_frag = _lib.FILE_FRAGMENTS_FN(fr) if on_fragments else _lib.FILE_FRAGMENTS_FN()
        cb_rec = _lib.FILE_RECORD_FN(rc_) if on_record else _lib.FILE_RECORD_FN()
        cb_done = _lib.FILE_DONE_FN(dn) if on_done else _lib.FILE_DONE_FN()
        stats = _lib.PipelineStats()
        try:
            rc = self._lib.cec_pipeline_run_files(self._h, arr, len(readers), cb_frag, cb_rec,
                                                  cb_done, None, byref(stats))
        finally:
            for r in readers:
                r.close()
            pool.shutdown(wait=True)
        if err:
            raise err[0]
        if rc == _lib.CEC_ESEGCOUNT:
            from .records import ErrTooManySegments
            raise ErrTooManySegments(ErrTooManySegments.__doc__)
        check(rc, "Pipeline.run_files")
        return stats


class RecordsSession:
    """A long-lived uploader: one codec and one pipeline (pinned ring pinned once, device slots
    allocated once) for many files, each turned into its FileRecord (SegmentLists + file hash).
    `hash_on`: "hybrid" (default: host SHA-256 on the segment chains, the GPU queue on the other
    fragments, the run's last batches wholly on the host), "host", "gpu". encode_many() streams
    several files back to back in one pipeline run, so one file's last hashes overlap the next
    file's copies."""

    def __init__(self, k: int = geometry.DATA_SHARDS, m: int = geometry.PARITY_SHARDS,
                 segment_size: int = geometry.SEGMENT_SIZE, device: int = 0,
                 hash_on: str = "hybrid", batch_segments: int = 64, depth: int = 0,
                 window: int = 0, host_threads: int = 16, tail_batches: int = -1,
                 max_segments: int = 0, read_threads: int = 8):
        if segment_size % k:
            raise ValueError("segment_size must be a multiple of k")
        if hash_on not in ("gpu", "host", "hybrid"):
            raise ValueError("hash_on must be 'gpu', 'host' or 'hybrid'")
        self.k, self.m, self.segment_size = k, m, segment_size
        self.hash_on = hash_on
        self.read_threads = read_threads
        self.enc = Encoder(k, m, device)
        try:
            self.pipe = Pipeline(self.enc, segment_size // k, batch_segments=batch_segments,
                                 depth=depth, hash=hash_on, window=window,
                                 max_segments=max_segments, host_threads=host_threads,
                                 tail_batches=tail_batches)
        except BaseException:
            self.enc.close()
            raise

    def encode_many(self, srcs, on_fragment=None, on_file=None):
        """[FileRecord] of every source, in one pipeline run. on_fragment(file, seg, idx, view)
        sees each fragment; on_file(file, FileRecord, stats) each file as soon as its records are
        complete (later files still streaming). Returns ([FileRecord], run PipelineStats)."""
        from .segments import FileRecord, SegmentList, file_hash
        srcs = list(srcs)
        recs = [dict() for _ in srcs]
        out = [None] * len(srcs)

        def on_rec(f, seg, sh, fl):
            recs[f][seg] = SegmentList(sh, fl)

        def on_done(f, st):
            if not recs[f]:
                from .reedsolomon import ErrShortData
                raise ErrShortData(ErrShortData.__doc__)
            r = FileRecord(b"", int(st.bytes_in), [recs[f][s] for s in range(len(recs[f]))])
            r.file_hash = file_hash(r.segments)
            recs[f] = None
            out[f] = r
            if on_file is not None:
                on_file(f, r, _lib.PipelineStats(st.segments, st.bytes_in, st.seconds,
                                                 st.read_seconds, st.wait_seconds))

        def frags(f, seg, views):
            for i, v in enumerate(views):
                on_fragment(f, seg, i, v)

        st = self.pipe.run_files(srcs, frags if on_fragment else None, on_rec, on_done,
                                 self.read_threads)
        return out, st

    def encode_range(self, src: Source, seg_start: int, seg_stop: int):
        """(FileRecord, PipelineStats) of segments [seg_start, seg_stop) of a file or buffer (one
        rank's or one device's contiguous shard of a file encoded across GPUs); segment numbers
        count from the range's first segment, `file_hash` covers the range only."""
        from .segments import FileRecord, SegmentList, file_hash
        size = _source_size(src)
        if size is None:
            raise ValueError("encode_range needs a path or an in-memory buffer")
        a, b = seg_start * self.segment_size, min(size, seg_stop * self.segment_size)
        if seg_start < 0 or b <= a:
            from .reedsolomon import ErrShortData
            raise ErrShortData(ErrShortData.__doc__)
        recs = {}
        st = self.pipe.run_files([src], None, lambda _f, s, sh, fl: recs.__setitem__(
            s, SegmentList(sh, fl)), None, self.read_threads, [(a, b)])
        out = FileRecord(b"", b - a, [recs[s] for s in range(len(recs))])
        out.file_hash = file_hash(out.segments)
        return out, st

    def encode(self, src: Source, on_fragment=None):
        """(FileRecord, PipelineStats) of one file."""
        cb = (lambda _f, seg, idx, v: on_fragment(seg, idx, v)) if on_fragment else None
        recs, st = self.encode_many([src], cb)
        return recs[0], st

    def close(self) -> None:
        self.pipe.close()
        self.enc.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def _source_size(src: Source) -> Optional[int]:
    if isinstance(src, str):
        return os.path.getsize(src)
    if isinstance(src, (np.ndarray, memoryview)):
        return src.nbytes
    if isinstance(src, (bytes, bytearray)):
        return len(src)
    if isinstance(src, (list, tuple)):  # in-memory pieces read back to back
        return sum(_source_size(x) for x in src)
    return None  # a stream


def record_hash_placement(hash_on: str, size: Optional[int] = None, k: int = 2,
                          m: int = 1) -> str:
    """Where encode_file_records' record hashes run: "gpu", "host" or "hybrid". "auto" is the
    hybrid placement (segment chains on host SHA-256 threads, the other fragments on the GPU hash
    queue, the last batches wholly on the host); with it the pipeline itself moves every batch of
    a file too small to outlast one GPU chain to the host (cec_pipeline_opts.tail_batches = -1),
    so no size threshold is needed here. Measured on one MI355X + its 16-CPU share, 8 GiB
    in-memory file, RS(2,1): see `extra.host_e2e` of the bench line."""
    if hash_on not in ("gpu", "host", "hybrid", "auto"):
        raise ValueError("hash_on must be 'gpu', 'host', 'hybrid' or 'auto'")
    return "hybrid" if hash_on == "auto" else hash_on


def encode_file_records(path_or_buf: Source, k: int = geometry.DATA_SHARDS,
                        m: int = geometry.PARITY_SHARDS,
                        segment_size: int = geometry.SEGMENT_SIZE, device: int = 0,
                        on_fragment: Optional[Callable[[int, int, np.ndarray], None]] = None,
                        max_segments: int = 0, hash_on: str = "auto", hash_threads: int = 16,
                        session: Optional["RecordsSession"] = None, **kw):
    """File -> (FileRecord, PipelineStats): SegmentLists + two-level file hash, encoded on the GPU
    through the C pipeline. on_fragment(seg, idx, view) sees each fragment as soon as its
    batch's parity is back (before its hash is known).

    hash_on: "hybrid" / "auto" (segment chains on `hash_threads` host threads, the other
    fragments on the GPU hash queue, the last batches on the host), "host" (every chain on the
    host threads), "gpu" (every chain on the GPU hash queue). The records are the same either
    way. `session`: a RecordsSession to reuse (its pinned ring and device slots stay allocated
    between files); without one, a session sized to the file is created and closed here."""
    if segment_size % k:
        raise ValueError("segment_size must be a multiple of k")
    hash_on = record_hash_placement(hash_on, None, k, m)
    if session is not None:
        return session.encode(path_or_buf, on_fragment)
    size = _source_size(path_or_buf)
    if size is not None:  # a small file does not need 1 GiB pinned batches
        kw.setdefault("batch_segments", max(1, min(64, -(-size // segment_size))))
    with RecordsSession(k, m, segment_size, device, hash_on, max_segments=max_segments,
                        host_threads=hash_threads, **kw) as ses:
        return ses.encode(path_or_buf, on_fragment)


def encode_file_records_multi(src: Union[str, bytes, bytearray, memoryview, np.ndarray],
                              devices, k: int = geometry.DATA_SHARDS,
                              m: int = geometry.PARITY_SHARDS,
                              segment_size: int = geometry.SEGMENT_SIZE,
                              max_segments: int = 0, read_threads: int = 8,
                              hash_on: str = "auto", hash_threads: int = 16, **kw):
    """File -> FileRecord with the segments sharded over several GPUs from ONE host process (an
    uploader on a multi-GPU node): contiguous segment ranges per device
    (distributed.shard_range; segments are independent, no data exchange), one RecordsSession
    (C pipeline) per device on its own host thread, records merged in segment order. `devices`
    may repeat a device (several pipelines sharing one GPU). hash_on as in encode_file_records;
    each pipeline hashes on its own `hash_threads` host threads (the GPU's CPU share) and takes
    its own HBM: window + 3 device batch slots of up to 1.5 GiB (a CESS batch of 64 segments;
    batch_segments shrinks for small shards), fitted to the free HBM when it is created, so
    pipelines sharing a GPU split what is left. Returns (FileRecord, [PipelineStats per device])."""
    from .distributed import shard_range
    from .segments import FileRecord, file_hash
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
    mode = record_hash_placement(hash_on)
    kw.setdefault("batch_segments", max(1, min(64, -(-nseg // len(devices)))))

    def work(i):
        a, b = shard_range(nseg, len(devices), i)
        if b <= a:
            return [], None
        with RecordsSession(k, m, segment_size, devices[i], mode, host_threads=hash_threads,
                            read_threads=read_threads, **kw) as ses:
            rec, st = ses.encode_range(src, a, b)
        return rec.segments, st

    with cf.ThreadPoolExecutor(max_workers=len(devices)) as ex:
        parts = list(ex.map(work, range(len(devices))))
    segs = [sl for p, _ in parts for sl in p]
    out = FileRecord(b"", size, segs)
    out.file_hash = file_hash(out.segments)
    return out, [st for _, st in parts if st is not None]


__all__ = ["Pipeline", "RecordsSession", "encode_file_records", "encode_file_records_multi",
           "CecError", "record_hash_placement"]
