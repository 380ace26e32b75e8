"""Storage-audit chunks on HBM-resident fragment batches.

Reference: a fragment is CHUNK_COUNT = 1024 chunks (primitives/common/src/lib.rs:62), so an 8 MiB
fragment is 1024 chunks of 8 KiB. A challenge (`generation_challenge`,
c-pallets/audit/src/lib.rs:901-988) names need = CHUNK_COUNT * 46 / 1000 = 47 distinct chunk
indices (`NetSnapShot.random_index_list`, types.rs:21): for seed = 1, 2, ..., index =
random_number(seed) % CHUNK_COUNT, repeats skipped (lib.rs:955-964), where random_number is the
chain's randomness decoded as u64 (lib.rs:1067-1076). Given that random stream, the selection
and the chunk bytes are byte-exact; the PoDR2 tags computed over the chunks live in the TEE and
are not in the reference (unpinned, not provided here).
"""
from __future__ import annotations

from ctypes import POINTER, byref, c_size_t, c_uint32, c_uint64
from typing import Optional, Sequence

import numpy as np

from . import _lib
from .reedsolomon import Encoder, _dev_ptr, _stream_handle, check

CHUNK_COUNT = _lib.CEC_CHUNK_COUNT
CHALLENGE_NEED = CHUNK_COUNT * 46 // 1000  # 47


def challenge_indices(randoms: Sequence[int], chunk_count: int = CHUNK_COUNT,
                      need: int = CHALLENGE_NEED):
    """The reference's selection loop over random_number(1), random_number(2), ...:
    returns (indices, randoms consumed)."""
    r = np.ascontiguousarray(np.asarray(randoms, dtype=np.uint64))
    out = np.zeros(max(1, need), np.uint32)
    used = c_size_t()
    check(_lib.load().cec_challenge_indices(r.ctypes.data_as(POINTER(c_uint64)), r.size,
                                            chunk_count, need,
                                            out.ctypes.data_as(POINTER(c_uint32)), byref(used)),
          "challenge_indices")
    return out[:need].tolist(), used.value


RANDOM_BYTES = _lib.CEC_CHALLENGE_RANDOM_BYTES


def challenge_random_list(randomness: Sequence[bytes], need: int = CHALLENGE_NEED):
    """NetSnapShot.random_list (c-pallets/audit/src/lib.rs:966-974, generate_challenge_random
    :1079-1096): randomness[i] = the chain's 32-byte randomness output for the subject
    (MyPalletId, now + 2 + i) (records.audit_random_subject(now + 2 + i); None as 32 zero bytes).
    Returns (the `need` distinct 20-byte values in order, outputs consumed)."""
    buf = b"".join(bytes(r) if r is not None else bytes(32) for r in randomness)
    if any(r is not None and len(r) != 32 for r in randomness):
        raise ValueError("each randomness output is 32 bytes (an H256)")
    src = np.frombuffer(buf, np.uint8).copy() if buf else np.zeros(1, np.uint8)
    out = np.zeros(max(1, need) * RANDOM_BYTES, np.uint8)
    used = c_size_t()
    check(_lib.load().cec_challenge_random_list(src.ctypes.data, len(randomness), need,
                                                out.ctypes.data, byref(used)),
          "challenge_random_list")
    return [out[i * RANDOM_BYTES:(i + 1) * RANDOM_BYTES].tobytes() for i in range(need)], \
        used.value


def audit_chunks(enc: Encoder, d_data, d_parity, nseg: int, shard_len: int,
                 indices: Sequence[int], d_chunks=None, d_hex=None,
                 chunk_count: int = CHUNK_COUNT, stream=None) -> None:
    """Gather the challenged chunks of every fragment of a batch ([nseg][k][len] data and, if
    given, [nseg][m][len] parity) into d_chunks [nfrag][nidx][len / chunk_count] and/or their
    SHA-256 hex into d_hex [nfrag][nidx][64] (fragments in batch order)."""
    idx = np.ascontiguousarray(np.asarray(indices, dtype=np.uint32))
    check(enc._lib.cec_audit_chunks(
        enc._h, _dev_ptr(d_data), None if d_parity is None else _dev_ptr(d_parity), nseg,
        shard_len, chunk_count, idx.ctypes.data_as(POINTER(c_uint32)), idx.size,
        None if d_chunks is None else _dev_ptr(d_chunks),
        None if d_hex is None else _dev_ptr(d_hex), _stream_handle(stream)), "audit_chunks")
