"""Repair (restoral) service and idle fillers.

Restoral flow on chain (reference c-pallets/file-bank/src/lib.rs):
  * `generate_restoral_order(file_hash, restoral_fragment)` (:943-984) marks a fragment
    unavailable (`avail = false`, :971);
  * a miner claims it (`claim_restoral_order`, :989-1014), rebuilds the fragment off chain from
    k surviving fragments of the same segment, and
  * `restoral_order_complete(fragment_hash)` (:1075-1122) marks it available again.
The off-chain step is what this module does: rebuild one fragment and check that its SHA-256
hex equals the `FragmentInfo.hash` recorded for it (types.rs:70-76) before reporting.

Idle fillers (`upload_filler`, lib.rs:798-833) are 8 MiB blocks whose content generator is not
in the reference; here they are the splitmix64 counter stream of libcessec (parity unpinned).
"""
from __future__ import annotations

import hashlib
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import geometry
from .reedsolomon import CecError, Encoder, ErrTooFewShards, sha256_hex_device


class ErrFragmentHashMismatch(CecError, ValueError):
    """rebuilt fragment does not match the recorded fragment hash"""


def repair_fragment(enc: Encoder, survivors: Dict[int, np.ndarray], index: int,
                    expected_hash: Optional[bytes] = None) -> np.ndarray:
    """Rebuild fragment `index` of one segment from `survivors` ({fragment index: bytes}, at
    least k of them) on the GPU. With `expected_hash` (64 hex chars), raise
    ErrFragmentHashMismatch unless SHA-256(rebuilt) equals it."""
    n = enc.Shards
    if not 0 <= index < n:
        raise ValueError("fragment index out of range")
    if len([i for i in survivors if i != index]) < enc.DataShards:
        raise ErrTooFewShards(ErrTooFewShards.__doc__)
    shards: List[Optional[np.ndarray]] = [None] * n
    for i, b in survivors.items():
        if i != index:
            shards[i] = np.ascontiguousarray(b, dtype=np.uint8)
    if index < enc.DataShards:
        enc.ReconstructData(shards)
    else:
        enc.Reconstruct(shards)
    out = shards[index]
    if expected_hash is not None:
        got = hashlib.sha256(out).hexdigest().encode()
        if got != bytes(expected_hash):
            raise ErrFragmentHashMismatch(f"fragment {index}: {got.decode()} != "
                                          f"{bytes(expected_hash).decode()}")
    return out


# Fragments to check at once from which the GPU's hash beats the host's: one SHA-256 chain per
# fragment runs ~35 MB/s on a GPU lane (1.8 us per 64-byte block), so the GPU's time is flat up to
# thousands of fragments (64 rebuilt 8 MiB fragments: 0.233 s), while the host's grows with the
# count (8 threads: 0.140 s for the same 64, ~2.2 ms per fragment; the f2 row of
# profiles/r02/aux_bench.jsonl, tools/aux_bench.py).
AUTO_GPU_CHECK_FRAGMENTS = 128


def repair_batch(enc: Encoder, d_data, d_parity, nseg: int, shard_len: int, present,
                 expected: Optional[Sequence[Dict[int, bytes]]] = None, stream=None,
                 hash_on: str = "auto", hash_threads: int = 16):
    """Rebuild every missing fragment of an HBM-resident batch in place (one launch for all
    erasure patterns) and, with `expected` ([{fragment index: recorded hash}] per segment),
    return per-segment booleans: rebuilt fragments hash to the recorded values. hash_on "gpu":
    all of them hashed in one GPU launch, one chain per fragment, where they were rebuilt;
    "host": copied out once and hashed by `hash_threads` host threads (OpenSSL via hashlib);
    "auto": the host below AUTO_GPU_CHECK_FRAGMENTS fragments (a chain is serial, so a few
    chains run faster on host cores), the GPU from there."""
    import torch
    if hash_on not in ("gpu", "host", "auto"):
        raise ValueError("hash_on must be 'gpu', 'host' or 'auto'")
    enc.ReconstructBatch(d_data, d_parity, nseg, shard_len, present, stream=stream)
    if expected is None:
        return None
    if stream is None:
        torch.cuda.current_stream(d_data.device).synchronize()
    else:
        stream.synchronize()
    k = enc.DataShards
    which = [(s, i, bytes(h)) for s in range(nseg) for i, h in expected[s].items()]
    frags = [d_data[s, i] if i < k else d_parity[s, i - k] for s, i, _ in which]
    if hash_on == "auto":
        hash_on = "gpu" if len(which) >= AUTO_GPU_CHECK_FRAGMENTS else "host"
    if not which:
        got = []
    elif hash_on == "gpu":
        got = sha256_hex_device([t.data_ptr() for t in frags], shard_len)
    else:
        import concurrent.futures as cf
        host = torch.stack(frags).cpu().numpy()
        with cf.ThreadPoolExecutor(max(1, hash_threads)) as ex:  # hashlib drops the GIL
            got = list(ex.map(lambda a: hashlib.sha256(a).hexdigest().encode(), host))
    ok = [True] * nseg
    for (s, _, h), g in zip(which, got):
        ok[s] &= g == h
    return ok


def generate_fillers(n: int, seed: int = 0xF111E5, filler_size: int = geometry.FRAGMENT_SIZE,
                     first: int = 0, device: int = 0):
    """n idle fillers of `filler_size` bytes generated in HBM (splitmix64 counter stream,
    filler i = segment first+i of the generator) with their SHA-256 hex hashes (as
    `upload_filler` records them), hashed on the GPU. Returns (device tensor [n][filler_size],
    [hash])."""
    import torch
    from .reedsolomon import fill_synthetic
    d = torch.empty((n, filler_size), dtype=torch.uint8, device=torch.device("cuda", device))
    fill_synthetic(d, filler_size, n, first, seed)
    torch.cuda.synchronize(device)
    hashes = sha256_hex_device([d[i].data_ptr() for i in range(n)], filler_size) if n else []
    return d, hashes
