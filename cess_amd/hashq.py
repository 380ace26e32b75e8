"""Streaming SHA-256 of fragments and segments on the GPU (libcessec hash queue,
include/cess_ec.h `cec_hashq_*`).

The records it produces are the `Hash` values of `SegmentList { hash, fragment_list }`
(c-pallets/file-bank/src/types.rs:13-16; `Hash([u8; 64])`, primitives/common/src/lib.rs:16):
64 lowercase hex chars of SHA-256 [ecosystem convention, SURVEY.md §8a a4].

Why a queue: a buffer's SHA-256 is one serial chain, and one GPU lane runs a chain at about one
wave's instruction issue rate, so hashing throughput is (chains in flight) x (per-chain rate).
One 1 GiB batch has 4096 fragment chains (RS(32,32)) or 192 (RS(2,1)): a few percent of the
chip. The queue keeps chain state in HBM, so each `tick` advances the chains of every batch
added so far; adding one batch per step and ticking once per step keeps a window of batches
hashing together. Completion is known on the host from lengths alone: `done(ticket)` turns true
once the ticks enqueued so far cover that add (the hex is in HBM when the stream gets there).
"""
from __future__ import annotations

from ctypes import byref, c_int, c_size_t, c_uint64, c_void_p
from typing import Optional

from . import _lib
from .reedsolomon import _dev_ptr, _stream_handle, check


def sha256_blocks(length: int) -> int:
    """64-byte compressions of one SHA-256 chain over `length` bytes, padding included."""
    return (length >> 6) + (2 if (length & 63) >= 56 else 1)


class HashQueue:
    """GPU hash queue bound to one device and one stream (all its work is ordered there)."""

    def __init__(self, capacity: int = 1 << 18, device: int = 0, stream=None):
        lib = _lib.load()
        h = c_void_p()
        self.stream = stream
        check(lib.cec_hashq_create(device, capacity, _stream_handle(stream), byref(h)),
              "HashQueue")
        self._h = h
        self.capacity = capacity

    def close(self) -> None:
        if getattr(self, "_h", None):
            _lib.load().cec_hashq_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def add(self, d_base, n: int, per: int, outer_stride: int, inner_stride: int, length: int,
            d_hex=None, hex_outer: int = 0, hex_offset: int = 0, prefix_len: int = 0,
            d_prefix_hex=None, prefix_hex_outer: int = 0, prefix_hex_offset: int = 0) -> int:
        """Append n chains (buffer i at base + (i // per) * outer + (i % per) * inner, `length`
        bytes; hex at d_hex + hex_offset + ((i // per) * hex_outer + i % per) * 64). With
        d_prefix_hex, chain i also writes the hex of its first prefix_len bytes (a multiple of 64)
        at d_prefix_hex + prefix_hex_offset + ((i // per) * prefix_hex_outer + i % per) * 64
        (cec_hashq_add_prefix). Returns the add's ticket."""
        t = c_uint64()
        hexp = None if d_hex is None else _dev_ptr(d_hex) + hex_offset
        prep = None if d_prefix_hex is None else _dev_ptr(d_prefix_hex) + prefix_hex_offset
        check(_lib.load().cec_hashq_add_prefix(self._h, _dev_ptr(d_base), n, per, outer_stride,
                                               inner_stride, length, hexp, hex_outer,
                                               prefix_len if prep else 0, prep,
                                               prefix_hex_outer, byref(t)),
              "HashQueue.add")
        return t.value

    def add_fragments(self, d_data, d_parity, nseg: int, k: int, m: int, shard_len: int,
                      d_hex, with_parity: bool = True) -> int:
        """Hash every fragment of a batch ([nseg][k][len] data, [nseg][m][len] parity) into
        d_hex[nseg][k+m][64] (fragment index order of SegmentList.fragment_list). Returns the
        ticket of the last add."""
        n_sh = k + m
        t = self.add(d_data, nseg * k, k, k * shard_len, shard_len, shard_len, d_hex,
                     n_sh, 0)
        if with_parity and m:
            t = self.add(d_parity, nseg * m, m, m * shard_len, shard_len, shard_len, d_hex,
                         n_sh, k * 64)
        return t

    def add_segments(self, d_data, nseg: int, seg_len: int, d_hex, seg_stride: Optional[int]
                     = None) -> int:
        """Hash nseg contiguous segments (SegmentList.hash) into d_hex[nseg][64]."""
        stride = seg_len if seg_stride is None else seg_stride
        return self.add(d_data, nseg, 1, stride, stride, seg_len, d_hex, 1, 0)

    def add_segment_lists(self, d_data, d_parity, nseg: int, k: int, m: int, shard_len: int,
                          d_seg_hex, d_frag_hex) -> int:
        """Every hash of a batch's SegmentLists ([nseg][k][len] data, [nseg][m][len] parity):
        segment hashes into d_seg_hex[nseg][64], fragment hashes into d_frag_hex[nseg][k+m][64].
        Data fragment 0's hash is the prefix digest of its segment's chain, so fragment 0 is
        hashed once (k*len + (k-1)*len + m*len bytes per segment instead of (2k+m)*len).
        Needs shard_len % 64 == 0 (else fragment 0 gets its own chain). Returns the ticket of
        the segment chains, the longest of the batch (the batch is done when they are)."""
        n_sh = k + m
        seg = k * shard_len
        if shard_len % 64 == 0:
            t = self.add(d_data, nseg, 1, seg, seg, seg, d_seg_hex, 1, 0, shard_len,
                         d_frag_hex, n_sh, 0)
            if k > 1:
                # data fragments 1..k-1: base shifted by one fragment, per = k - 1
                self.add(_dev_ptr(d_data) + shard_len, nseg * (k - 1), k - 1, seg, shard_len,
                         shard_len, d_frag_hex, n_sh, 64)
        else:
            t = self.add(d_data, nseg, 1, seg, seg, seg, d_seg_hex, 1, 0)
            self.add(d_data, nseg * k, k, seg, shard_len, shard_len, d_frag_hex, n_sh, 0)
        if m:
            self.add(d_parity, nseg * m, m, m * shard_len, shard_len, shard_len, d_frag_hex,
                     n_sh, k * 64)
        return t

    def set_option(self, option: int, value: int) -> None:
        """cec_hashq_set_option (CEC_HQOPT_TICK: 0 auto, 1/2 two-wave prefetch depth, 3 one
        wave, 4 lane pairs: the shortest chain latency)."""
        check(_lib.load().cec_hashq_set_option(self._h, option, value), "HashQueue.set_option")

    def tick(self, max_blocks: int = 0) -> None:
        """Advance every live chain by at most max_blocks blocks (0: to completion)."""
        check(_lib.load().cec_hashq_tick(self._h, max_blocks), "HashQueue.tick")

    def finish(self) -> None:
        """Enqueue ticks until every chain added so far is complete."""
        check(_lib.load().cec_hashq_finish(self._h), "HashQueue.finish")

    def status(self, ticket: int = 0):
        done, live, left = c_int(), c_size_t(), c_uint64()
        check(_lib.load().cec_hashq_status(self._h, ticket, byref(done), byref(live),
                                           byref(left)), "HashQueue.status")
        return bool(done.value), live.value, left.value

    def done(self, ticket: int) -> bool:
        return self.status(ticket)[0]

    @property
    def live_chains(self) -> int:
        return self.status()[1]

    @property
    def blocks_left(self) -> int:
        return self.status()[2]
