"""On-chain records of the codec's outputs, SCALE-encoded by libcessec (host only, no GPU).

    FileBank::upload_declaration(file_hash: Hash,
        deal_info: BoundedVec<SegmentList<T>, T::SegmentCount>, user_brief: UserBrief<T>)
                                              c-pallets/file-bank/src/lib.rs:419-428
    SegmentList { hash: Hash, fragment_list: BoundedVec<Hash, FragmentCount> }  types.rs:13-16
    UserBrief { user: AccountId32, file_name, bucket_name: BoundedVec<u8, NameStrLimit> }
                                              types.rs:105-109
    Hash([u8; 64])                            primitives/common/src/lib.rs:16
    SEGMENT_COUNT = 1000, FRAGMENT_COUNT = 3  runtime/src/lib.rs:1026-1027
    Hash::from_shard_id (64 of 68 bytes)      primitives/common/src/lib.rs:45-49
    upload_filler(tee_worker, Vec<FillerInfo>) call_index(8), lib.rs:795-833; FillerInfo
        { block_num: u32, miner_address: AccountId32, filler_hash: Hash } types.rs:82-86;
        UploadFillerLimit = 10 runtime/src/lib.rs:1033
    restoral calls 13-16                      lib.rs:940-1122
    audit random_number's subject             c-pallets/audit/src/lib.rs:1067-1076

A file of more than SegmentCount segments (16,000 MiB) cannot be declared in one extrinsic:
encoding its deal_info raises ErrTooManySegments (the chain would reject it as BoundedVecError).
"""
from __future__ import annotations

from ctypes import byref, c_size_t, c_uint64
from dataclasses import dataclass
from typing import List, Sequence

import numpy as np

from . import _lib
from .reedsolomon import CecError, check

SEGMENT_COUNT = _lib.CEC_SEGMENT_COUNT
FRAGMENT_COUNT = _lib.CEC_FRAGMENT_COUNT
UPLOAD_FILLER_LIMIT = _lib.CEC_UPLOAD_FILLER_LIMIT
FILLER_SIZE = _lib.CEC_FILLER_SIZE
AUDIT_PALLET_ID = _lib.CEC_AUDIT_PALLET_ID


@dataclass
class FillerInfo:
    """c-pallets/file-bank/src/types.rs:82-86."""
    block_num: int
    miner_address: bytes  # AccountId32
    filler_hash: bytes    # 64 hex chars


class ErrTooManySegments(CecError, ValueError):
    """file exceeds SegmentCount segments: one upload_declaration carries at most 1000"""

    code = _lib.CEC_ESEGCOUNT


def _call(fn_name: str, *args) -> bytes:
    lib = _lib.load()
    fn = getattr(lib, fn_name)
    n = c_size_t()
    check(fn(*args, None, 0, byref(n)), fn_name)
    out = np.zeros(max(1, n.value), np.uint8)
    check(fn(*args, out.ctypes.data, n.value, byref(n)), fn_name)
    return out[: n.value].tobytes()


def _hex_block(hashes: Sequence[bytes], width: int = 64) -> np.ndarray:
    a = np.frombuffer(b"".join(hashes), np.uint8) if hashes else np.zeros(0, np.uint8)
    if a.size != len(hashes) * width:
        raise ValueError("every hash must be 64 hex characters")
    return np.ascontiguousarray(a)


def scale_compact(n: int) -> bytes:
    return _call("cec_scale_compact", n)


def _flat(segments) -> tuple:
    nseg = len(segments)
    if nseg > SEGMENT_COUNT:
        raise ErrTooManySegments(f"{nseg} segments > SegmentCount = {SEGMENT_COUNT}")
    nfrag = len(segments[0].fragment_list) if nseg else FRAGMENT_COUNT
    if any(len(s.fragment_list) != nfrag for s in segments):
        raise ValueError("every segment needs the same fragment count (check_file_spec)")
    seg = _hex_block([s.hash for s in segments])
    frag = _hex_block([f for s in segments for f in s.fragment_list])
    return seg, frag, nseg, nfrag


def deal_info(segments) -> bytes:
    """SCALE of deal_info: compact(n) ++ per SegmentList: hash ++ compact(3) ++ 3 hashes."""
    seg, frag, nseg, nfrag = _flat(segments)
    try:
        return _call("cec_scale_deal_info", seg.ctypes.data, frag.ctypes.data, nseg, nfrag)
    except CecError as e:
        if e.code == _lib.CEC_ESEGCOUNT:
            raise ErrTooManySegments(str(e)) from None
        raise


def upload_declaration(file_hash: bytes, segments, account: bytes, file_name: bytes,
                       bucket_name: bytes) -> bytes:
    """Call data of FileBank::upload_declaration (pallet 60, call 0) for a file record."""
    if len(account) != 32:
        raise ValueError("account must be a 32-byte AccountId32")
    seg, frag, nseg, nfrag = _flat(segments)
    fh = _hex_block([file_hash])
    acc = np.frombuffer(account, np.uint8).copy()
    fn = np.frombuffer(file_name, np.uint8).copy() if file_name else np.zeros(1, np.uint8)
    bn = np.frombuffer(bucket_name, np.uint8).copy() if bucket_name else np.zeros(1, np.uint8)
    return _call("cec_scale_upload_declaration", fh.ctypes.data, seg.ctypes.data,
                 frag.ctypes.data, nseg, nfrag, acc.ctypes.data, fn.ctypes.data, len(file_name),
                 bn.ctypes.data, len(bucket_name))


def shard_id(hash_hex: bytes, index: int) -> bytes:
    """68-byte shard id: 64 hex chars ++ "-NNN" (c-pallets/audit/src/tests.rs:267-269)."""
    h = _hex_block([hash_hex])
    out = np.zeros(68, np.uint8)
    check(_lib.load().cec_shard_id(h.ctypes.data, index, out.ctypes.data), "shard_id")
    return out.tobytes()


def hash_from_shard_id(sid: bytes) -> bytes:
    """Hash::from_shard_id: the first 64 of the 68 bytes."""
    if len(sid) != 68:
        raise ValueError("a shard id is 68 bytes")
    src = np.frombuffer(sid, np.uint8).copy()
    out = np.zeros(64, np.uint8)
    check(_lib.load().cec_hash_from_shard_id(src.ctypes.data, out.ctypes.data),
          "hash_from_shard_id")
    return out.tobytes()


def split_declarations(segments) -> List[list]:
    """Consecutive runs of at most SegmentCount segments (one upload_declaration each), for a
    caller that declares a large file as several files."""
    return [list(segments[i:i + SEGMENT_COUNT]) for i in range(0, len(segments), SEGMENT_COUNT)]


def _account(a: bytes, what: str) -> np.ndarray:
    if len(a) != 32:
        raise ValueError(f"{what} must be a 32-byte AccountId32")
    return np.frombuffer(bytes(a), np.uint8).copy()


def upload_filler(tee_worker: bytes, fillers: Sequence[FillerInfo]) -> bytes:
    """Call data of FileBank::upload_filler (pallet 60, call 8): tee_worker ++ Vec<FillerInfo>.
    More than UploadFillerLimit = 10 fillers raise CecError (the chain's LengthExceedsLimit)."""
    tw = _account(tee_worker, "tee_worker")
    n = len(fillers)
    blk = np.array([f.block_num for f in fillers] or [0], np.uint32)
    miners = np.frombuffer(b"".join(bytes(f.miner_address) for f in fillers) or bytes(32),
                           np.uint8).copy()
    if miners.size != max(1, n) * 32:
        raise ValueError("miner_address must be a 32-byte AccountId32")
    hx = _hex_block([f.filler_hash for f in fillers]) if n else np.zeros(64, np.uint8)
    from ctypes import POINTER, c_uint32
    return _call("cec_scale_upload_filler", tw.ctypes.data,
                 blk.ctypes.data_as(POINTER(c_uint32)), miners.ctypes.data, hx.ctypes.data, n)


def upload_filler_calls(tee_worker: bytes, fillers: Sequence[FillerInfo]) -> List[bytes]:
    """upload_filler call data for any number of fillers, UploadFillerLimit per call."""
    return [upload_filler(tee_worker, fillers[i:i + UPLOAD_FILLER_LIMIT])
            for i in range(0, len(fillers), UPLOAD_FILLER_LIMIT)]


def generate_restoral_order(file_hash: bytes, fragment_hash: bytes) -> bytes:
    """Call 13 (lib.rs:940-984): the holder of a lost fragment opens a restoral order."""
    return _call("cec_scale_generate_restoral_order", _hex_block([file_hash]).ctypes.data,
                 _hex_block([fragment_hash]).ctypes.data)


def claim_restoral_order(fragment_hash: bytes) -> bytes:
    """Call 14 (lib.rs:986-1014): a miner claims an open order."""
    return _call("cec_scale_claim_restoral_order", _hex_block([fragment_hash]).ctypes.data)


def claim_restoral_exist_order(miner: bytes, file_hash: bytes, fragment_hash: bytes) -> bytes:
    """Call 15 (lib.rs:1016-1070): claim a fragment of an exiting miner (RestoralTarget)."""
    return _call("cec_scale_claim_restoral_exist_order", _account(miner, "miner").ctypes.data,
                 _hex_block([file_hash]).ctypes.data, _hex_block([fragment_hash]).ctypes.data)


def restoral_order_complete(fragment_hash: bytes) -> bytes:
    """Call 16 (lib.rs:1072-1122): the rebuilt fragment is stored; emit only after its SHA-256
    matched the recorded fragment hash."""
    return _call("cec_scale_restoral_order_complete", _hex_block([fragment_hash]).ctypes.data)


def audit_random_subject(seed: int, pallet_id: bytes = AUDIT_PALLET_ID) -> bytes:
    """The 12 bytes Audit::random_number(seed) hands the chain's randomness:
    (MyPalletId, seed).encode() (c-pallets/audit/src/lib.rs:1067-1076)."""
    if len(pallet_id) != 8:
        raise ValueError("a PalletId is 8 bytes")
    pid = np.frombuffer(pallet_id, np.uint8).copy()
    out = np.zeros(12, np.uint8)
    check(_lib.load().cec_audit_random_subject(pid.ctypes.data, seed, out.ctypes.data),
          "audit_random_subject")
    return out.tobytes()


def audit_random_u64(randomness: bytes) -> int:
    """random_number's result from the randomness output: its first 8 bytes as u64 LE."""
    r = np.frombuffer(bytes(randomness), np.uint8).copy() if randomness else np.zeros(1, np.uint8)
    v = c_uint64()
    check(_lib.load().cec_audit_random_u64(r.ctypes.data, len(randomness), byref(v)),
          "audit_random_u64")
    return v.value
