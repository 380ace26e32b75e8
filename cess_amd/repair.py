"""Repair (restoral) service and idle fillers.

Restoral flow on chain (reference c-pallets/file-bank/src/lib.rs):
  * `generate_restoral_order(file_hash, restoral_fragment)` (:943-984) marks a fragment
    unavailable (`avail = false`, :971);
  * a miner claims it (`claim_restoral_order`, :989-1014), rebuilds the fragment off chain from
    k surviving fragments of the same segment, and
  * `restoral_order_complete(fragment_hash)` (:1075-1122) marks it available again.
The off-chain step is what this module does: rebuild one fragment and check that its SHA-256
hex equals the `FragmentInfo.hash` recorded for it (types.rs:70-76) before reporting. The report
itself is the call data of `restoral_order_complete` (records.restoral_order_complete), emitted
only for a fragment whose rebuilt hash matched.

Idle fillers (`upload_filler`, lib.rs:795-833) are 8 MiB blocks whose content generator is not
in the reference; here they are the splitmix64 counter stream of libcessec (content unpinned).
Their on-chain record is pinned: `FillerInfo { block_num, miner_address, filler_hash }`
(types.rs:82-86), at most UploadFillerLimit = 10 per `upload_filler` call (runtime/src/lib.rs:1033).
"""
from __future__ import annotations

import hashlib
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import geometry, records
from .reedsolomon import (CecError, Encoder, ErrTooFewShards, sha256_hex_device,
                          sha256_hex_host)


class ErrFragmentHashMismatch(CecError, ValueError):
    """rebuilt fragment does not match the recorded fragment hash"""


def repair_fragment(enc: Encoder, survivors: Dict[int, np.ndarray], index: int,
                    expected_hash: Optional[bytes] = None, complete_call: bool = False):
    """Rebuild fragment `index` of one segment from `survivors` ({fragment index: bytes}, at
    least k of them) on the GPU. With `expected_hash` (64 hex chars), raise
    ErrFragmentHashMismatch unless SHA-256(rebuilt) equals it. With `complete_call` (needs
    `expected_hash`) return (fragment, restoral_order_complete call data): the call exists only
    for a fragment that passed the check."""
    if complete_call and expected_hash is None:
        raise ValueError("complete_call needs the recorded fragment hash")
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
    if complete_call:
        return out, records.restoral_order_complete(bytes(expected_hash))
    return out


# Fragments to check at once from which the GPU's hash beats the host's: one SHA-256 chain per
# fragment runs ~38 MB/s on a GPU lane (1.7 us per 64-byte block), so the GPU's time is flat up to
# thousands of fragments (0.223-0.229 s for 64..1024 rebuilt 8 MiB fragments), while the host's
# grows with the count: copied out in pinned chunks and hashed on 16 threads (cec_sha256_host)
# as the chunks land, 0.020 / 0.059 / 0.105 / 0.208 s for 64 / 256 / 512 / 1024
# (profiles/r06/repair_check_scale.jsonl, tools/repair_check_scale.py). Round 5's threshold of
# 128 came from hashlib on 8 threads after one pageable copy-out (0.140 s for 64).
AUTO_GPU_CHECK_FRAGMENTS = 1024


# Host-side check staging: a ring of pinned chunk buffers kept between calls (pinning costs ~0.1 s
# per GiB; a repair service checks batch after batch), CHECK_RING chunks of CHECK_CHUNK fragments.
_STAGE = {}
CHECK_CHUNK = 16
CHECK_RING = 6


def _host_check_hashes(frags, shard_len: int, threads: int, device) -> List[bytes]:
    """SHA-256 hex of device fragments on host threads: copied out chunk by chunk into a ring of
    pinned buffers on a side stream, each chunk hashed (cec_sha256_host) as soon as its copy lands
    while the next chunks copy; the chunks' jobs share the host SHA pool's lanes. A ring buffer
    is refilled once its previous chunk is hashed, so the pinned memory stays at CHECK_RING x
    CHECK_CHUNK fragments whatever the batch."""
    import concurrent.futures as cf
    import torch
    n = len(frags)
    nchunks = -(-n // CHECK_CHUNK)
    ring = min(CHECK_RING, nchunks)
    need = ring * CHECK_CHUNK * shard_len
    stage = _STAGE.get(device)
    if stage is None or stage.numel() < need:
        stage = torch.empty(need, dtype=torch.uint8, pin_memory=True)
        _STAGE[device] = stage
    bufs = stage[:need].view(ring, CHECK_CHUNK, shard_len)
    st = torch.cuda.Stream(device)
    st.wait_stream(torch.cuda.current_stream(device))

    def check(c, ev):
        ev.synchronize()
        hv = bufs[c % ring].numpy()
        return sha256_hex_host([hv[j] for j in range(min(CHECK_CHUNK, n - c * CHECK_CHUNK))],
                               shard_len, threads)

    futs = []
    with cf.ThreadPoolExecutor(max_workers=ring) as ex:
        for c in range(nchunks):
            if c >= ring:
                futs[c - ring].result()  # that ring buffer's chunk is hashed: reuse it
            with torch.cuda.stream(st):
                for j in range(c * CHECK_CHUNK, min(n, (c + 1) * CHECK_CHUNK)):
                    bufs[c % ring][j - c * CHECK_CHUNK].copy_(frags[j], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(st)
            futs.append(ex.submit(check, c, ev))
        return [h for f in futs for h in f.result()]


def repair_batch(enc: Encoder, d_data, d_parity, nseg: int, shard_len: int, present,
                 expected: Optional[Sequence[Dict[int, bytes]]] = None, stream=None,
                 hash_on: str = "auto", hash_threads: int = 16, complete_calls: bool = False):
    """Rebuild every missing fragment of an HBM-resident batch in place (one launch for all
    erasure patterns) and, with `expected` ([{fragment index: recorded hash}] per segment),
    return per-segment booleans: rebuilt fragments hash to the recorded values. hash_on "gpu":
    all of them hashed in one GPU launch, one chain per fragment, where they were rebuilt;
    "host": copied out once and hashed by `hash_threads` host threads (cec_sha256_host);
    "auto": the host below AUTO_GPU_CHECK_FRAGMENTS fragments (a chain is serial, so a few
    chains run faster on host cores), the GPU from there. With `complete_calls`, return
    (ok, calls): calls = {(segment, fragment index): restoral_order_complete call data} for
    exactly the fragments whose rebuilt hash equals the recorded one."""
    import torch
    if hash_on not in ("gpu", "host", "auto"):
        raise ValueError("hash_on must be 'gpu', 'host' or 'auto'")
    enc.ReconstructBatch(d_data, d_parity, nseg, shard_len, present, stream=stream)
    if expected is None:
        if complete_calls:
            raise ValueError("complete_calls needs the recorded hashes (expected)")
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
        got = _host_check_hashes(frags, shard_len, hash_threads, d_data.device)
    ok = [True] * nseg
    calls = {}
    for (s, i, h), g in zip(which, got):
        ok[s] &= g == h
        if complete_calls and g == h:
            calls[(s, i)] = records.restoral_order_complete(h)
    return (ok, calls) if complete_calls else ok


def generate_fillers(n: int, seed: int = 0xF111E5, filler_size: int = geometry.FRAGMENT_SIZE,
                     first: int = 0, device: int = 0, hash_on: str = "auto",
                     hash_threads: int = 16):
    """n idle fillers of `filler_size` bytes generated in HBM (splitmix64 counter stream,
    filler i = segment first+i of the generator) with their SHA-256 hex hashes (as
    `upload_filler` records them). Returns (device tensor [n][filler_size], [hash]). hash_on
    "gpu": one chain per filler on the GPU (flat ~0.22 s for 8 MiB fillers up to thousands);
    "host": copied out in pinned chunks and hashed on `hash_threads` host threads as they land
    (the copy a miner uploading them makes anyway); "auto": the host below
    AUTO_GPU_CHECK_FRAGMENTS fillers, as the repair check."""
    import torch
    from .reedsolomon import fill_synthetic
    if hash_on not in ("gpu", "host", "auto"):
        raise ValueError("hash_on must be 'gpu', 'host' or 'auto'")
    dev = torch.device("cuda", device)
    d = torch.empty((n, filler_size), dtype=torch.uint8, device=dev)
    fill_synthetic(d, filler_size, n, first, seed)
    torch.cuda.synchronize(device)
    if hash_on == "auto":
        hash_on = "gpu" if n >= AUTO_GPU_CHECK_FRAGMENTS else "host"
    if not n:
        hashes = []
    elif hash_on == "gpu":
        hashes = sha256_hex_device([d[i].data_ptr() for i in range(n)], filler_size)
    else:
        hashes = _host_check_hashes([d[i] for i in range(n)], filler_size, hash_threads, dev)
    return d, hashes


def filler_records(hashes: Sequence[bytes], miner: bytes, block_num: int):
    """FillerInfo records (types.rs:82-86) of fillers with these SHA-256 hex hashes."""
    return [records.FillerInfo(block_num, bytes(miner), bytes(h)) for h in hashes]


def generate_filler_upload(n: int, miner: bytes, tee_worker: bytes, block_num: int,
                           seed: int = 0xF111E5, first: int = 0, device: int = 0):
    """n 8 MiB idle fillers generated and hashed on the GPU, with their on-chain records: returns
    (device tensor [n][8 MiB], hashes, [FillerInfo], [upload_filler call data]) — one call per
    UploadFillerLimit = 10 fillers (c-pallets/file-bank/src/lib.rs:795-833)."""
    d, hashes = generate_fillers(n, seed=seed, filler_size=records.FILLER_SIZE, first=first,
                                 device=device)
    fillers = filler_records(hashes, miner, block_num)
    return d, hashes, fillers, records.upload_filler_calls(tee_worker, fillers)
