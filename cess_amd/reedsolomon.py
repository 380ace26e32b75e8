"""klauspost/reedsolomon-shaped encoder over libcessec (MI355X).

This mirrors the off-chain codec API whose outputs the CESS chain records:
`New(k, m)` returns an Encoder with Encode / Verify / Reconstruct / ReconstructData / Split /
Join, the same argument meaning and the same error names (ErrTooFewShards, ErrShardNoData,
ErrShardSize, ErrShortData, ErrInvShardNum, ErrMaxShardNum, ErrReconstructRequired). Shards are
host buffers (numpy uint8 arrays / bytearrays) of equal length; a missing shard is None or empty.

For HBM-resident segment batches use the *Batch methods with device tensors laid out
[nseg][k][shard_len] (data) and [nseg][m][shard_len] (parity).

The reference chain fixes k = 2, m = 1 (primitives/common/src/lib.rs:60-61,
runtime/src/lib.rs:1027) and consumes the fragment hashes in
FileBank::upload_declaration (c-pallets/file-bank/src/lib.rs:423).
"""
from __future__ import annotations

import ctypes
from ctypes import POINTER, byref, c_int, c_uint8, c_void_p
from typing import BinaryIO, List, Optional, Sequence

import numpy as np

from . import _lib


class CecError(Exception):
    """Base error; `code` is the C ABI return code."""

    code = _lib.CEC_EINVAL


class ErrInvShardNum(CecError, ValueError):
    """cannot create Encoder with less than one data shard or less than zero parity shards"""


class ErrMaxShardNum(CecError, ValueError):
    """cannot create Encoder with more than 256 data+parity shards"""


class ErrTooFewShards(CecError, ValueError):
    """too few shards given"""

    code = _lib.CEC_ETOOFEW


class ErrShardNoData(CecError, ValueError):
    """no shard data"""

    code = _lib.CEC_ESHARDLEN


class ErrShardSize(CecError, ValueError):
    """shard sizes do not match"""

    code = _lib.CEC_ESHARDLEN


class ErrShortData(CecError, ValueError):
    """not enough data to fill the number of requested shards"""

    code = _lib.CEC_ESHORTDATA


class ErrReconstructRequired(CecError, ValueError):
    """reconstruction required as one or more required data shards are nil"""


class HipError(CecError, RuntimeError):
    code = _lib.CEC_EHIP


_CODE_TO_EXC = {
    _lib.CEC_ETOOFEW: ErrTooFewShards,
    _lib.CEC_ESHARDLEN: ErrShardSize,
    _lib.CEC_ESHORTDATA: ErrShortData,
    _lib.CEC_EHIP: HipError,
    _lib.CEC_ENOMEM: HipError,
    _lib.CEC_ENODEV: HipError,
    _lib.CEC_ENCCL: HipError,
}


def check(rc: int, what: str = "") -> None:
    if rc == _lib.CEC_OK:
        return
    lib = _lib.load()
    msg = lib.cec_strerror(rc).decode()
    detail = lib.cec_last_error().decode()
    exc = _CODE_TO_EXC.get(rc, CecError)
    e = exc(f"{what}: {msg}" + (f" ({detail})" if detail else ""))
    e.code = rc
    raise e


def _as_u8(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        if buf.dtype != np.uint8 or not buf.flags.c_contiguous:
            raise TypeError("shards must be contiguous uint8 arrays")
        return buf
    if isinstance(buf, (bytearray, memoryview)):
        return np.frombuffer(buf, dtype=np.uint8)
    raise TypeError(f"unsupported shard type {type(buf)!r}")


def _present(s) -> bool:
    return s is not None and len(s) > 0


def _ptr_array(arrs: Sequence[np.ndarray]):
    return (c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


def _dev_ptr(t) -> int:
    """Device address of a torch tensor (or an int address)."""
    if isinstance(t, int):
        return t
    if not t.is_cuda or not t.is_contiguous():
        raise TypeError("batch buffers must be contiguous device tensors")
    return t.data_ptr()


def _stream_handle(stream) -> Optional[int]:
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream  # torch.cuda.Stream


class Encoder:
    """One codec bound to one GPU (klauspost Encoder). `tuning=True` binds the tuning build of
    the library (kernel variants for sweeps; never the product path)."""

    def __init__(self, data_shards: int, parity_shards: int, device: int = 0,
                 tuning: bool = False):
        if data_shards <= 0 or parity_shards < 0:
            raise ErrInvShardNum(ErrInvShardNum.__doc__)
        if data_shards + parity_shards > 256:
            raise ErrMaxShardNum(ErrMaxShardNum.__doc__)
        self.DataShards = data_shards
        self.ParityShards = parity_shards
        self.Shards = data_shards + parity_shards
        self.device = device
        self._h = c_void_p()
        self._lib = None
        if parity_shards > 0:
            self._lib = _lib.load(tuning)
            check(self._lib.cec_create(data_shards, parity_shards, device, byref(self._h)), "New")

    # -- lifetime ----------------------------------------------------------------------------
    def close(self) -> None:
        if self._h:
            self._lib.cec_destroy(self._h)
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

    # -- helpers -----------------------------------------------------------------------------
    def matrix(self) -> np.ndarray:
        """(k+m) x k encode matrix."""
        out = np.zeros((self.Shards, self.DataShards), dtype=np.uint8)
        if self.ParityShards == 0:
            return np.eye(self.DataShards, dtype=np.uint8)
        check(self._lib.cec_matrix(self._h, out.ctypes.data_as(POINTER(c_uint8))), "matrix")
        return out

    def set_option(self, option: int, value: int) -> None:
        """cec_set_option on this codec only (CEC_OPT_*)."""
        check(self._lib.cec_set_option(self._h, option, value), "set_option")

    def stat(self, which: int) -> int:
        v = ctypes.c_uint64()
        check(self._lib.cec_get_stat(self._h, which, byref(v)), "stat")
        return v.value

    def _check_shards(self, shards, nil_ok: bool) -> int:
        size = next((len(s) for s in shards if _present(s)), 0)
        if size == 0:
            raise ErrShardNoData(ErrShardNoData.__doc__)
        for s in shards:
            n = len(s) if s is not None else 0
            if n != size and (n != 0 or not nil_ok):
                raise ErrShardSize(ErrShardSize.__doc__)
        return size

    # -- klauspost API -----------------------------------------------------------------------
    def Encode(self, shards: List) -> None:
        """Compute parity shards[k:] from data shards[:k] in place."""
        if len(shards) != self.Shards:
            raise ErrTooFewShards(ErrTooFewShards.__doc__)
        size = self._check_shards(shards, nil_ok=False)
        if self.ParityShards == 0:
            return
        arrs = [_as_u8(s) for s in shards]
        check(self._lib.cec_encode(self._h, _ptr_array(arrs), size), "Encode")

    def Verify(self, shards: Sequence) -> bool:
        if len(shards) != self.Shards:
            raise ErrTooFewShards(ErrTooFewShards.__doc__)
        size = self._check_shards(shards, nil_ok=False)
        if self.ParityShards == 0:
            return True
        arrs = [_as_u8(s) for s in shards]
        ok = c_int(0)
        check(self._lib.cec_verify(self._h, _ptr_array(arrs), size, byref(ok)), "Verify")
        return bool(ok.value)

    def _reconstruct(self, shards: List, data_only: bool) -> None:
        if len(shards) != self.Shards:
            raise ErrTooFewShards(ErrTooFewShards.__doc__)
        size = self._check_shards(shards, nil_ok=True)
        present = [_present(s) for s in shards]
        if all(present) or (data_only and all(present[: self.DataShards])):
            return
        if sum(present) < self.DataShards:
            raise ErrTooFewShards(ErrTooFewShards.__doc__)
        for i in range(self.Shards):
            if not present[i] and (i < self.DataShards or not data_only):
                shards[i] = np.zeros(size, dtype=np.uint8)
        arrs = [_as_u8(s) if _present(s) else np.zeros(size, dtype=np.uint8) for s in shards]
        flags = (c_uint8 * self.Shards)(*[1 if p else 0 for p in present])
        check(self._lib.cec_reconstruct(self._h, _ptr_array(arrs), flags, size,
                                          1 if data_only else 0), "Reconstruct")
        for i in range(self.Shards):
            if not present[i] and (i < self.DataShards or not data_only):
                shards[i] = arrs[i]

    def Reconstruct(self, shards: List) -> None:
        """Recreate every missing (None / empty) shard in place."""
        self._reconstruct(shards, data_only=False)

    def ReconstructData(self, shards: List) -> None:
        """Recreate only missing data shards."""
        self._reconstruct(shards, data_only=True)

    def Split(self, data) -> List[np.ndarray]:
        """Split data into k equal shards (last zero padded) plus m zeroed parity shards."""
        src = _as_u8(data) if not isinstance(data, bytes) else np.frombuffer(data, np.uint8)
        if len(src) == 0:
            raise ErrShortData(ErrShortData.__doc__)
        per = (len(src) + self.DataShards - 1) // self.DataShards
        shards = [np.empty(per, dtype=np.uint8) for _ in range(self.DataShards)]
        check(_lib.load().cec_split_segment(src.ctypes.data, len(src), self.DataShards,
                                            _ptr_array(shards), per), "Split")
        return shards + [np.zeros(per, dtype=np.uint8) for _ in range(self.ParityShards)]

    def Join(self, dst: BinaryIO, shards: Sequence, out_size: int) -> None:
        """Write the first out_size bytes of the concatenated data shards to dst."""
        if len(shards) < self.DataShards:
            raise ErrTooFewShards(ErrTooFewShards.__doc__)
        shards = shards[: self.DataShards]
        if any(not _present(s) for s in shards):
            raise ErrReconstructRequired(ErrReconstructRequired.__doc__)
        if sum(len(s) for s in shards) < out_size:
            raise ErrShortData(ErrShortData.__doc__)
        left = out_size
        for s in shards:
            b = bytes(_as_u8(s)[: left])
            dst.write(b)
            left -= len(b)
            if left == 0:
                break

    # -- HBM-resident batches ----------------------------------------------------------------
    def EncodeBatch(self, d_data, d_parity, nseg: int, shard_len: int, stream=None) -> None:
        """Enqueue encode of nseg segments ([nseg][k][len] -> [nseg][m][len]) on `stream`."""
        check(self._lib.cec_encode_batch(self._h, _dev_ptr(d_data), _dev_ptr(d_parity), nseg,
                                           shard_len, _stream_handle(stream)), "EncodeBatch")

    def ReconstructBatch(self, d_data, d_parity, nseg: int, shard_len: int, present,
                         data_only: bool = False, stream=None) -> None:
        """Rebuild missing shards in place. `present`: n flags (one pattern) or nseg x n."""
        p = np.ascontiguousarray(np.asarray(present, dtype=np.uint8))
        per_segment = 1 if p.ndim == 2 else 0
        if per_segment and p.shape != (nseg, self.Shards):
            raise ValueError("present must be (nseg, k+m)")
        if not per_segment and p.shape != (self.Shards,):
            raise ValueError("present must have k+m flags")
        check(self._lib.cec_reconstruct_batch(
            self._h, _dev_ptr(d_data), _dev_ptr(d_parity), nseg, shard_len,
            p.ctypes.data_as(POINTER(c_uint8)), per_segment, 1 if data_only else 0,
            _stream_handle(stream)), "ReconstructBatch")

    def ReconstructPartialBatch(self, d_data, d_parity, nseg: int, shard_len: int, present,
                                held, data_only: bool = False, stream=None) -> None:
        """Partial rebuild (cec_reconstruct_partial_batch): every missing shard of segment s gets
        the contribution of the survivors of `present[s]` flagged in `held[s]` (both nseg x n).
        XOR of the partials over a partition of the survivors = ReconstructBatch's result."""
        p = np.ascontiguousarray(np.asarray(present, dtype=np.uint8))
        h = np.ascontiguousarray(np.asarray(held, dtype=np.uint8))
        if p.shape != (nseg, self.Shards) or h.shape != (nseg, self.Shards):
            raise ValueError("present and held must be (nseg, k+m)")
        check(self._lib.cec_reconstruct_partial_batch(
            self._h, _dev_ptr(d_data), _dev_ptr(d_parity), nseg, shard_len,
            p.ctypes.data_as(POINTER(c_uint8)), h.ctypes.data_as(POINTER(c_uint8)),
            1 if data_only else 0, _stream_handle(stream)), "ReconstructPartialBatch")

    def VerifyBatch(self, d_data, d_parity, nseg: int, shard_len: int, d_ok=None,
                    stream=None):
        """klauspost Verify over an HBM batch (cec_verify_batch): with `d_ok` (device uint8
        [nseg]) the per-segment flags are enqueued there; without, they are returned as a numpy
        bool array (synchronous)."""
        import torch
        out = d_ok
        if out is None:
            out = torch.empty(max(1, nseg), dtype=torch.uint8,
                              device=torch.device("cuda", self.device))
            if stream is None:  # read back below on torch's current stream: launch there too
                stream = torch.cuda.current_stream(out.device)
        check(self._lib.cec_verify_batch(self._h, _dev_ptr(d_data), _dev_ptr(d_parity), nseg,
                                         shard_len, _dev_ptr(out), _stream_handle(stream)),
              "VerifyBatch")
        if d_ok is not None:
            return None
        if stream is not None:
            stream.synchronize()
        return out[:nseg].cpu().numpy().astype(bool)

    def Sha256Batch(self, d_data, d_parity, nseg: int, shard_len: int, d_hex,
                    stream=None) -> None:
        """Hex SHA-256 of every shard into d_hex ([nseg][k+m][64] bytes, device)."""
        check(self._lib.cec_sha256_batch(
            self._h, _dev_ptr(d_data), 0 if d_parity is None else _dev_ptr(d_parity), nseg,
            shard_len, _dev_ptr(d_hex), _stream_handle(stream)), "Sha256Batch")


def New(data_shards: int, parity_shards: int, device: int = 0, tuning: bool = False) -> Encoder:
    """klauspost reedsolomon.New(dataShards, parityShards) on a GPU."""
    return Encoder(data_shards, parity_shards, device, tuning)


def fill_synthetic(d_out, seg_bytes: int, nseg: int, seg0: int, seed: int, stream=None) -> None:
    """Counter-based synthetic segments in HBM (SURVEY.md §8d input generator)."""
    check(_lib.load().cec_fill_synthetic(_dev_ptr(d_out), seg_bytes, nseg, seg0, seed,
                                         _stream_handle(stream)), "fill_synthetic")


def xor_batch(d_dst, d_src, nsrc: int, src_stride: int, length: int, stream=None) -> None:
    """d_dst[:length] ^= XOR of nsrc buffers at d_src + j * src_stride (cec_xor_batch: GF(2^8)
    addition of the partial rebuilds other GPUs sent)."""
    check(_lib.load().cec_xor_batch(_dev_ptr(d_dst), _dev_ptr(d_src), nsrc, src_stride, length,
                                    _stream_handle(stream)), "xor_batch")


def sha256_hex_host(bufs, length: int, threads: int = 16, prefix_len: int = 0):
    """SHA-256 hex of equal-length HOST buffers (numpy arrays / bytes-likes, or addresses) with
    libcessec's multi-chain host hasher (cec_sha256_host: 16 chains per core in AVX-512 lanes or
    SHA-NI interleaved, on `threads` threads; the GIL is released during the call). With
    `prefix_len` (a multiple of 64, <= length) returns (hexes, hexes of each buffer's first
    prefix_len bytes): a segment chain yields data fragment 0's hash on the way."""
    n = len(bufs)
    if n == 0:
        return ([], []) if prefix_len else []
    keep = []
    ptrs = []
    for b in bufs:
        if isinstance(b, int):
            ptrs.append(b)
            continue
        a = b if isinstance(b, np.ndarray) else np.frombuffer(b, np.uint8)
        if a.nbytes < length:
            raise ValueError("buffer shorter than length")
        if length and not a.flags.c_contiguous:
            a = np.ascontiguousarray(a)
        keep.append(a)
        ptrs.append(a.ctypes.data)
    out = np.zeros(n * 64, dtype=np.uint8)
    pre = np.zeros(n * 64, dtype=np.uint8) if prefix_len else None
    arr = (c_void_p * n)(*ptrs)
    check(_lib.load().cec_sha256_host(arr, n, length, out.ctypes.data, prefix_len,
                                      pre.ctypes.data if prefix_len else None, threads),
          "sha256_hex_host")
    hexes = [out[i * 64:(i + 1) * 64].tobytes() for i in range(n)]
    if prefix_len:
        return hexes, [pre[i * 64:(i + 1) * 64].tobytes() for i in range(n)]
    return hexes


def sha256_hex_device(d_ptrs: Sequence[int], length: int) -> List[bytes]:
    """SHA-256 hex of device buffers (addresses) of equal length, computed on the GPU."""
    n = len(d_ptrs)
    out = np.zeros(n * 64, dtype=np.uint8)
    arr = (c_void_p * n)(*d_ptrs)
    check(_lib.load().cec_sha256_hex(arr, n, length, out.ctypes.data_as(POINTER(c_uint8)),
                                     None), "sha256_hex")
    return [out[i * 64:(i + 1) * 64].tobytes() for i in range(n)]
