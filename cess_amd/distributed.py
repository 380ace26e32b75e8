"""Multi-GPU placement and the degraded-read gather.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on MI355X, "gloo" on
CPU for tests). Encode needs no collective: segments are independent, each rank encodes a
contiguous range (`shard_range`). The one real exchange is a degraded read / repair: the k
surviving fragments of a segment live on different GPUs and must meet on the GPU that rebuilds
the lost one. RCCL has no XOR reduction (rccl.h ncclRedOp_t: sum/prod/max/min/avg), so
survivors are moved with grouped point-to-point send/recv (`batch_isend_irecv`) and decoded
locally by libcessec.

Two exchanges, chosen per segment by `plan_gather(exchange=...)`:
  * survivors: the k survivors travel to the decoder, which rebuilds the lost fragments;
  * partials: every other GPU holding survivors multiplies them by their decode coefficients
    (cec_reconstruct_partial_batch) and sends one partial per lost fragment; the decoder XORs
    the partials into its own (cec_xor_batch: addition in GF(2^8)). The rebuild is linear, so
    the sum is the lost fragment. It moves e * (holders) fragments instead of (k - local): for a
    wide code on 8 GPUs (RS(32,32), 8 fragments per GPU) a single lost fragment costs 7
    partials instead of 28 survivors. For RS(2,1) the counts tie and survivors are used.

Placement mirrors the chain's miner assignment, which spreads a segment's fragments over
distinct miners (c-pallets/file-bank/src/functions.rs:187-283, `random_assign_miner`, and
`:256-276`): fragment f of segment s is stored on GPU (s + f) mod G.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Dict, List, Sequence, Tuple

import numpy as np


def shard_range(nseg: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [start, stop) segment range of `rank` (encode sharding, no collective)."""
    base, extra = divmod(nseg, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def fragment_owner(seg: int, frag: int, world: int) -> int:
    return (seg + frag) % world


@dataclass
class FragmentStore:
    """Fragments a rank holds under the (s + f) mod G placement: `slots[(s, f)]` indexes the
    rows of `data`, a [nslots, F] uint8 tensor (HBM on GPU ranks)."""

    slots: Dict[Tuple[int, int], int]
    data: "object"  # torch.Tensor [nslots, F]


def local_fragments(nseg: int, n: int, world: int, rank: int) -> List[Tuple[int, int]]:
    return [(s, f) for s in range(nseg) for f in range(n) if fragment_owner(s, f, world) == rank]


@dataclass
class GatherPlan:
    """Who sends which survivor to whom for a set of lost fragments."""

    # per decoding rank: ordered list of segments it rebuilds
    segments: Dict[int, List[int]]
    # (segment, survivor fragment) -> (source rank, destination rank)
    moves: Dict[Tuple[int, int], Tuple[int, int]]
    # segment -> present flags (k+m) the decoder passes: every fragment not erased. The codec
    # reads only its k survivors of them (`survivors`), so only those are moved; flagging the unused
    # ones present keeps the rebuild to the lost fragments alone (e outputs, not n - k)
    present: Dict[int, np.ndarray]
    # segment -> erased fragment indices
    lost: Dict[int, List[int]]
    bytes_moved: int
    # partial-product segments: segment -> ranks other than the decoder that hold some of its
    # survivors and send one partial per lost fragment (no survivor moves for these segments)
    partial: Dict[int, List[int]] = field(default_factory=dict)
    # segment -> decoding rank
    decoder: Dict[int, int] = field(default_factory=dict)
    world: int = 1
    # segment -> the survivors the rebuild reads (cec_survivors: index order)
    survivors: Dict[int, List[int]] = field(default_factory=dict)


EXCHANGES = ("survivors", "partials", "auto")


def survivors_of(k: int, m: int, present) -> List[int]:
    """The k survivors a rebuild of pattern `present` reads (cec_survivors, host only): the
    first k present fragments, or for RS(32,32) the set the FFT-domain decoders prefer. The
    gather moves exactly these."""
    from . import _lib
    from .reedsolomon import check
    flags = (ctypes.c_uint8 * (k + m))(*[1 if p else 0 for p in present])
    out = (ctypes.c_uint8 * k)()
    check(_lib.load().cec_survivors(k, m, flags, out), "cec_survivors")
    return list(out)


def plan_gather(lost: Dict[int, Sequence[int]], k: int, m: int, world: int,
                frag_bytes: int, exchange: str = "auto") -> GatherPlan:
    """Plan the degraded read of `lost` = {segment: erased fragment indices}.

    The decoder of a segment is the home GPU of its first lost fragment (repair restores the
    fragment where it lives). Survivors = the k fragments the codec reads (`survivors`: the
    first k present, or for RS(32,32) the FFT-domain decoders' choice; cec_survivors) (the
    codec's survivor choice), so exactly k fragments per segment are read. `exchange`:
    "survivors" moves the survivors the decoder lacks; "partials" moves one partial rebuild per
    lost fragment from every other GPU holding survivors; "auto" takes, per segment, whichever
    moves fewer bytes (survivors on a tie; the default: RS(2,1) over >= 3 GPUs always ties)."""
    if exchange not in EXCHANGES:
        raise ValueError(f"exchange must be one of {EXCHANGES}")
    n = k + m
    segs: Dict[int, List[int]] = {}
    moves = {}
    present = {}
    partial = {}
    decoder = {}
    survivors = {}
    moved = 0
    for s in sorted(lost):
        erased = set(lost[s])
        if not erased:
            continue  # nothing lost: no decoder, no moves
        bad = [f for f in erased if not 0 <= f < n]
        if bad:
            raise ValueError(f"segment {s}: fragment indices {bad} outside 0..{n - 1}")
        if len(erased) > m:
            raise ValueError(f"segment {s}: {len(erased)} erasures > m = {m}")
        dec = fragment_owner(s, min(erased), world)
        segs.setdefault(dec, []).append(s)
        decoder[s] = dec
        surv = survivors_of(k, m, [f not in erased for f in range(n)])
        survivors[s] = surv
        flags = np.ones(n, np.uint8)
        flags[sorted(erased)] = 0
        present[s] = flags
        holders = sorted({fragment_owner(s, f, world) for f in surv} - {dec})
        n_surv = sum(fragment_owner(s, f, world) != dec for f in surv)
        n_part = len(erased) * len(holders)
        if exchange == "partials" or (exchange == "auto" and n_part < n_surv):
            partial[s] = holders
            moved += n_part * frag_bytes
            continue
        for f in surv:
            src = fragment_owner(s, f, world)
            moves[(s, f)] = (src, dec)
            if src != dec:
                moved += frag_bytes
    return GatherPlan(segs, moves, present, {s: sorted(set(v)) for s, v in lost.items() if v},
                      moved, partial, decoder, world, survivors)


# Transfers per grouped point-to-point batch (one RCCL group each), counted over the whole plan:
# a batch holds the transfers of a run of the plan, the same run on every rank, so each rank's
# batch holds both ends of its transfers (the C path's CEC_DIST_OPT_GROUP_OPS, dist.cpp)
GROUP_TRANSFERS = 1024


def _p2p(ops_spec, group, stage: bool):
    """Issue [(batch, is_send, tensor, peer)] as grouped point-to-point batches, one per `batch`
    index in increasing order (all enqueued before any wait), and wait. gloo (CPU tests,
    rehearsals) needs host buffers: device tensors are staged through host memory."""
    import torch
    import torch.distributed as dist
    batches, copies = {}, []
    for b, is_send, t, peer in ops_spec:
        ops = batches.setdefault(b, [])
        if is_send:
            ops.append(dist.P2POp(dist.isend, t.cpu() if stage else t, peer, group))
        elif stage:
            h = torch.empty(t.shape, dtype=t.dtype)
            copies.append((t, h))
            ops.append(dist.P2POp(dist.irecv, h, peer, group))
        else:
            ops.append(dist.P2POp(dist.irecv, t, peer, group))
    reqs = []
    for b in sorted(batches):
        reqs += dist.batch_isend_irecv(batches[b])
    for req in reqs:
        req.wait()
    for t, h in copies:
        t.copy_(h)


def _staged(dev, group) -> bool:
    import torch.distributed as dist
    return dev.type == "cuda" and dist.is_initialized() and dist.get_backend(group) == "gloo"


def gather_survivors(plan: GatherPlan, store: FragmentStore, k: int, m: int, rank: int,
                     group=None):
    """Run the gather for this rank. Returns (staging_data [nseg_d][k][F],
    staging_parity [nseg_d][m][F], present [nseg_d][k+m], segment list) on the decoding rank;
    the staging tensors hold every used survivor at its shard index; the other slots are left
    uninitialised (the lost ones are written by the rebuild, the unused survivors are flagged
    present but never read: the codec reads exactly its survivors).
    Non-decoding ranks only send and return None for the staging tensors."""
    import torch
    import torch.distributed as dist

    F = store.data.shape[1]
    dev = store.data.device
    # partial-product segments are served by partial_exchange
    mysegs = [s for s in plan.segments.get(rank, []) if s not in plan.partial]
    row = {s: i for i, s in enumerate(mysegs)}
    sd = torch.empty((len(mysegs), k, F), dtype=torch.uint8, device=dev)
    sp = torch.empty((len(mysegs), m, F), dtype=torch.uint8, device=dev)

    def dst_view(s, f):
        return sd[row[s], f] if f < k else sp[row[s], f - k]

    # RCCL/NCCL moves HBM buffers directly (xGMI); the plan's cross-rank moves in batches of
    # GROUP_TRANSFERS, numbered the same on every rank
    ops = []
    moved = 0
    for (s, f), (src, dst) in sorted(plan.moves.items()):
        if src == dst == rank:
            dst_view(s, f).copy_(store.data[store.slots[(s, f)]])
        if src == dst:
            continue
        b = moved // GROUP_TRANSFERS
        moved += 1
        if src == rank:
            ops.append((b, True, store.data[store.slots[(s, f)]], dst))
        elif dst == rank:
            ops.append((b, False, dst_view(s, f), src))
    _p2p(ops, group, _staged(dev, group))
    if not mysegs:
        return None, None, None, []
    present = np.stack([plan.present[s] for s in mysegs])
    return sd, sp, present, mysegs


def partial_exchange(plan: GatherPlan, store: FragmentStore, enc, rank: int, group=None,
                     xor=None):
    """The partial-product segments of `plan` on this rank: rebuild, from the survivors this rank
    holds, the partial of every lost fragment of every partial segment it holds survivors of or
    decodes (one cec_reconstruct_partial_batch launch); send the partials to their decoders;
    on the decoder, XOR the received partials into its own (one cec_xor_batch launch).
    Returns {(segment, fragment): tensor[F]} of the fragments this rank rebuilt."""
    import torch
    if xor is None:
        from .reedsolomon import xor_batch as xor
    k, m = enc.DataShards, enc.ParityShards
    n = k + m
    F = store.data.shape[1]
    dev = store.data.device
    mine = [s for s in sorted(plan.partial)
            if plan.decoder[s] == rank or rank in plan.partial[s]]
    if not mine:
        return {}
    row = {s: i for i, s in enumerate(mine)}
    sd = torch.empty((len(mine), k, F), dtype=torch.uint8, device=dev)
    sp = torch.empty((len(mine), m, F), dtype=torch.uint8, device=dev)

    def slot(s, f):
        return sd[row[s], f] if f < k else sp[row[s], f - k]

    pres = np.stack([plan.present[s] for s in mine])
    held = np.zeros_like(pres)
    for s in mine:
        for f in plan.survivors[s]:
            if fragment_owner(s, f, plan.world) == rank:
                held[row[s], f] = 1
                slot(s, f).copy_(store.data[store.slots[(s, f)]])
    enc.ReconstructPartialBatch(sd, sp, len(mine), F, pres, held,
                                stream=torch.cuda.current_stream(dev) if dev.type == "cuda"
                                else None)
    dsegs = [s for s in mine if plan.decoder[s] == rank]
    pairs = [(s, f) for s in dsegs for f in plan.lost[s]]
    pidx = {p: i for i, p in enumerate(pairs)}
    H = max([len(plan.partial[s]) for s in dsegs], default=0)
    # row 0: this rank's partials; rows 1..H: the holders' (zero where a segment has fewer)
    acc = torch.empty((H + 1, max(1, len(pairs)), F), dtype=torch.uint8, device=dev)
    for (s, f), i in pidx.items():
        acc[0, i].copy_(slot(s, f))
    if any(len(plan.partial[s]) < H for s in dsegs):
        acc[1:].zero_()
    # batch of each partial segment: its first transfer's position in the whole plan's partial
    # transfers (every rank numbers them alike) // GROUP_TRANSFERS
    batch, moved = {}, 0
    for s in sorted(plan.partial):
        batch[s] = moved // GROUP_TRANSFERS
        moved += len(plan.lost[s]) * len(plan.partial[s])
    ops = []
    for s in mine:  # the same (segment, fragment) order on both sides of every pair
        if plan.decoder[s] == rank:
            for h, src in enumerate(plan.partial[s]):
                for f in plan.lost[s]:
                    ops.append((batch[s], False, acc[1 + h, pidx[(s, f)]], src))
        else:
            for f in plan.lost[s]:
                ops.append((batch[s], True, slot(s, f), plan.decoder[s]))
    _p2p(ops, group, _staged(dev, group))
    if H and pairs:
        # on the current stream, after the received partials and before whoever reads acc[0]
        # (torch side streams do not order against the null stream)
        if dev.type == "cuda":
            with torch.cuda.device(dev):
                xor(acc[0], acc[1], H, acc.stride(0), len(pairs) * F,
                    stream=torch.cuda.current_stream(dev))
        else:
            xor(acc[0], acc[1], H, acc.stride(0), len(pairs) * F)
    return {p: acc[0, i] for p, i in pidx.items()}


def degraded_read(plan: GatherPlan, store: FragmentStore, enc, rank: int, group=None,
                  xor=None):
    """Rebuild the lost fragments of `plan` over the process group (RCCL on GPUs): survivor
    segments by gathering survivors and one libcessec rebuild, partial-product segments by
    partial_exchange. Returns {(segment, fragment): tensor[F]} of rebuilt fragments for this
    rank."""
    k, m = enc.DataShards, enc.ParityShards
    sd, sp, present, segs = gather_survivors(plan, store, k, m, rank, group)
    out = {}
    if segs:
        import torch
        enc.ReconstructBatch(sd, sp, len(segs), sd.shape[2], present,
                             stream=torch.cuda.current_stream(sd.device) if sd.is_cuda else None)
        for i, s in enumerate(segs):
            for f in plan.lost[s]:
                out[(s, f)] = sd[i, f] if f < k else sp[i, f - k]
    if plan.partial:
        out.update(partial_exchange(plan, store, enc, rank, group, xor))
    return out


# -- the same exchange through the C ABI (cec_dist_*, for hosts without torch.distributed) -------

def c_plan(lost: Dict[int, Sequence[int]], k: int, m: int, world: int,
           exchange: str = "auto"):
    """cec_dist_plan_ex: (moves [(seg, frag, src, dst, kind)] in issue order, {(seg, frag):
    decoder rank}) of the plan libcessec's degraded read runs for `lost` (host only); kind 0 = a
    survivor fragment, 1 = a partial rebuild of lost fragment `frag`."""
    from ctypes import byref, c_int32, c_size_t, c_uint8, c_uint64
    from . import _lib
    from .reedsolomon import check
    pairs = [(s, f) for s in sorted(lost) for f in lost[s]]
    segs = (c_uint64 * max(1, len(pairs)))(*[s for s, _ in pairs])
    frags = (c_uint8 * max(1, len(pairs)))(*[f for _, f in pairs])
    lib = _lib.load()
    n = c_size_t()
    ex = EXCHANGES.index(exchange)
    check(lib.cec_dist_plan_ex(k, m, world, ex, segs, frags, len(pairs), None, 0, byref(n),
                               None), "cec_dist_plan_ex")
    moves = (_lib.DistMove * max(1, n.value))()
    dec = (c_int32 * max(1, len(pairs)))()
    check(lib.cec_dist_plan_ex(k, m, world, ex, segs, frags, len(pairs), moves, n.value,
                               byref(n), dec), "cec_dist_plan_ex")
    return ([(mv.seg, mv.frag, mv.src, mv.dst, mv.kind) for mv in moves[:n.value]],
            {p: dec[i] for i, p in enumerate(pairs)})


def c_plan_groups(lost: Dict[int, Sequence[int]], k: int, m: int, world: int,
                  exchange: str = "auto", group_ops: int = 1024) -> List[int]:
    """cec_dist_plan_groups: the plan positions (index of the segment among the lost segments in
    ascending order) where the RCCL transfer groups of libcessec's degraded read start, with at
    most `group_ops` transfers on any rank per group (host only)."""
    from ctypes import byref, c_size_t, c_uint8, c_uint64
    from . import _lib
    from .reedsolomon import check
    pairs = [(s, f) for s in sorted(lost) for f in lost[s]]
    segs = (c_uint64 * max(1, len(pairs)))(*[s for s, _ in pairs])
    frags = (c_uint8 * max(1, len(pairs)))(*[f for _, f in pairs])
    lib = _lib.load()
    n = c_size_t()
    ex = EXCHANGES.index(exchange)
    check(lib.cec_dist_plan_groups(k, m, world, ex, group_ops, segs, frags, len(pairs), None, 0,
                                   byref(n)), "cec_dist_plan_groups")
    out = (c_uint64 * max(1, n.value))()
    check(lib.cec_dist_plan_groups(k, m, world, ex, group_ops, segs, frags, len(pairs), out,
                                   n.value, byref(n)), "cec_dist_plan_groups")
    return list(out[:n.value])


class RcclGroup:
    """cec_dist_*: libcessec's own RCCL group for the degraded read (one per rank; every rank
    creates it with the same `uid`, made by `RcclGroup.unique_id()` on one rank)."""

    @staticmethod
    def unique_id() -> bytes:
        from . import _lib
        from .reedsolomon import check
        buf = (ctypes.c_uint8 * _lib.CEC_DIST_ID_BYTES)()
        check(_lib.load().cec_dist_unique_id(buf), "cec_dist_unique_id")
        return bytes(buf)

    def __init__(self, enc, uid: bytes, world: int, rank: int, exchange: str = "auto"):
        from ctypes import byref, c_void_p
        from . import _lib
        from .reedsolomon import check
        self._lib = _lib.load()
        self._h = c_void_p()
        self.enc, self.world, self.rank = enc, world, rank
        idb = (ctypes.c_uint8 * _lib.CEC_DIST_ID_BYTES).from_buffer_copy(uid)
        check(self._lib.cec_dist_create(enc._h, idb, world, rank, byref(self._h)),
              "cec_dist_create")
        self.exchange = exchange
        check(self._lib.cec_dist_set_option(self._h, _lib.CEC_DIST_OPT_EXCHANGE,
                                            EXCHANGES.index(exchange)), "cec_dist_set_option")

    def set_test_abort(self, round_index: int) -> None:
        """Test hook (CEC_DIST_OPT_TEST_ABORT): fail inside round `round_index`'s transfer group
        as an RCCL error there would (the group is aborted); -1 turns it off."""
        from . import _lib
        from .reedsolomon import check
        check(self._lib.cec_dist_set_option(self._h, _lib.CEC_DIST_OPT_TEST_ABORT, round_index),
              "cec_dist_set_option")

    def set_group_ops(self, n: int) -> None:
        """CEC_DIST_OPT_GROUP_OPS: at most n point-to-point transfers on any rank per RCCL group
        (default 1024; 0 = one group per round of 256 segments). Same value on every rank."""
        from . import _lib
        from .reedsolomon import check
        check(self._lib.cec_dist_set_option(self._h, _lib.CEC_DIST_OPT_GROUP_OPS, n),
              "cec_dist_set_option")

    def groups(self) -> int:
        """Transfer groups this handle has issued (cec_dist_groups)."""
        from ctypes import byref, c_uint64
        from .reedsolomon import check
        g = c_uint64()
        check(self._lib.cec_dist_groups(self._h, byref(g)), "cec_dist_groups")
        return g.value

    def close(self) -> None:
        if self._h:
            self._lib.cec_dist_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def degraded_read(self, lost: Dict[int, Sequence[int]], store: FragmentStore, stream=None):
        """Rebuild `lost` = {segment: erased fragments} (the same on every rank) from the ranks'
        stores; returns {(segment, fragment): tensor[F]} of the fragments this rank rebuilt."""
        import torch
        from ctypes import byref, c_size_t, c_uint8, c_uint64, c_void_p
        from . import _lib
        from .reedsolomon import check, _stream_handle
        F = store.data.shape[1]
        lost = {s: sorted(set(v)) for s, v in lost.items() if len(v)}
        pairs = [(s, f) for s in sorted(lost) for f in lost[s]]
        _, dec = c_plan(lost, self.enc.DataShards, self.enc.ParityShards, self.world,
                        self.exchange)
        out = {p: torch.empty(F, dtype=torch.uint8, device=store.data.device)
               for p in pairs if dec[p] == self.rank}
        segs = (c_uint64 * max(1, len(pairs)))(*[s for s, _ in pairs])
        frags = (c_uint8 * max(1, len(pairs)))(*[f for _, f in pairs])
        d_out = (c_void_p * max(1, len(pairs)))(*[out[p].data_ptr() if p in out else None
                                                   for p in pairs])
        base, row = store.data.data_ptr(), store.data.stride(0)

        def locate(_user, seg, frag):
            i = store.slots.get((seg, frag))
            return None if i is None else base + i * row

        cb = _lib.LOCATE_FN(locate)
        n = c_size_t()
        st = _stream_handle(stream if stream is not None
                            else torch.cuda.current_stream(store.data.device))
        check(self._lib.cec_dist_degraded_read(self._h, segs, frags, len(pairs), F, cb, None,
                                               d_out, st, byref(n)), "cec_dist_degraded_read")
        assert n.value == len(out)
        return out

