"""cess_amd: MI355X-native Reed-Solomon codec for CESS's segment -> fragment path.

The compute path is libcessec (HIP kernels for gfx950 behind the C ABI in include/cess_ec.h);
this package is the host-side mirror of the off-chain codec API (klauspost/reedsolomon shape)
plus the CESS segment / fragment records.
"""
from . import audit, geometry, records
from .hashq import HashQueue, sha256_blocks
from .records import ErrTooManySegments
from .reedsolomon import (
    CecError,
    Encoder,
    ErrInvShardNum,
    ErrMaxShardNum,
    ErrReconstructRequired,
    ErrShardNoData,
    ErrShardSize,
    ErrShortData,
    ErrTooFewShards,
    HipError,
    New,
    fill_synthetic,
    sha256_hex_device,
    sha256_hex_host,
    xor_batch,
)

__all__ = [
    "geometry", "CecError", "Encoder", "New", "ErrInvShardNum", "ErrMaxShardNum",
    "ErrReconstructRequired", "ErrShardNoData", "ErrShardSize", "ErrShortData",
    "ErrTooFewShards", "HipError", "fill_synthetic", "sha256_hex_device", "sha256_hex_host",
    "HashQueue", "sha256_blocks", "records", "ErrTooManySegments", "audit", "xor_batch",
]
