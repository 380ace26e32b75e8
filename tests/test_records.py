"""On-chain records (CPU, no GPU): the SCALE bytes libcessec emits for upload_declaration's
deal_info and call data, checked against a hand-built encoding written from the reference's
types (c-pallets/file-bank/src/lib.rs:419-428, types.rs:13-16 and 105-109,
primitives/common/src/lib.rs:16 and 45-49, runtime/src/lib.rs:1026-1027, 1532)."""
import hashlib
import struct

import numpy as np
import pytest

from cess_amd import records
from cess_amd.segments import SegmentList


def compact(n):
    """parity-scale-codec Compact<u32>, restated here independently of the product."""
    if n < 1 << 6:
        return bytes([n << 2])
    if n < 1 << 14:
        return struct.pack("<H", (n << 2) | 1)
    if n < 1 << 30:
        return struct.pack("<I", (n << 2) | 2)
    return b"\x03" + struct.pack("<I", n)


def hx(tag, i):
    return hashlib.sha256(f"{tag}-{i}".encode()).hexdigest().encode()


def seglists(nseg, nfrag=3):
    return [SegmentList(hx("seg", s), [hx(f"frag{s}", f) for f in range(nfrag)])
            for s in range(nseg)]


def hand_deal_info(segs):
    out = compact(len(segs))
    for s in segs:
        out += s.hash + compact(len(s.fragment_list)) + b"".join(s.fragment_list)
    return out


@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 16383, 16384, (1 << 30) - 1, 1 << 30,
                               0xFFFFFFFF])
def test_compact_boundaries(n):
    assert records.scale_compact(n) == compact(n)


@pytest.mark.parametrize("nseg", [1, 2, 63, 64, 1000])
def test_deal_info_matches_hand_built(nseg):
    segs = seglists(nseg)
    got = records.deal_info(segs)
    assert got == hand_deal_info(segs)
    # layout: compact(nseg) then (64 + 1 + 3 * 64) bytes per SegmentList
    assert len(got) == len(compact(nseg)) + nseg * (64 + 1 + 192)


def test_deal_info_rejects_more_than_segment_count():
    with pytest.raises(records.ErrTooManySegments):
        records.deal_info(seglists(1001))
    parts = records.split_declarations(seglists(2500))
    assert [len(p) for p in parts] == [1000, 1000, 500]
    assert records.deal_info(parts[0]) == hand_deal_info(parts[0])


def test_deal_info_rejects_bad_specs():
    import cess_amd
    with pytest.raises(cess_amd.CecError):  # FragmentCount = 3 bounds fragment_list
        records.deal_info(seglists(2, nfrag=4))
    bad = seglists(1)
    bad[0].hash = b"X" * 64  # not lowercase hex
    with pytest.raises(cess_amd.CecError):
        records.deal_info(bad)


def test_upload_declaration_call_data():
    segs = seglists(5)
    fh = hx("file", 0)
    acct = bytes(range(32))
    got = records.upload_declaration(fh, segs, acct, b"report.pdf", b"bucket1")
    want = (bytes([60, 0]) + fh + hand_deal_info(segs) + acct + compact(10) + b"report.pdf"
            + compact(7) + b"bucket1")
    assert got == want
    import cess_amd
    for fn, bn in [(b"ab", b"bucket"), (b"name", b"x" * 64)]:  # NameMinLength 3, NameStrLimit 63
        with pytest.raises(cess_amd.CecError):
            records.upload_declaration(fh, segs, acct, fn, bn)


def test_shard_id_round_trip():
    """c-pallets/audit/src/tests.rs:267-269 builds file_hash ++ "-001"; Hash::from_shard_id
    (primitives/common/src/lib.rs:45-49) reads the first 64 bytes back."""
    fh = hx("file", 1)
    sid = records.shard_id(fh, 1)
    assert sid == fh + b"-001" and len(sid) == 68
    assert records.hash_from_shard_id(sid) == fh
    assert records.shard_id(fh, 999)[-4:] == b"-999"
    import cess_amd
    with pytest.raises(cess_amd.CecError):
        records.shard_id(fh, 1000)


def test_deal_info_requires_exactly_fragment_count():
    """check_file_spec (c-pallets/file-bank/src/functions.rs:4-11) rejects any fragment_list whose
    length is not FragmentCount = 3: such call data would always fail with SpecError."""
    import cess_amd
    for nfrag in (1, 2, 4):
        with pytest.raises(cess_amd.CecError):
            records.deal_info(seglists(2, nfrag=nfrag))
    assert records.deal_info(seglists(2, nfrag=3)) == hand_deal_info(seglists(2, nfrag=3))


def acct(i):
    return bytes((i * 7 + j) & 0xFF for j in range(32))


def test_upload_filler_call_data():
    """FileBank::upload_filler(tee_worker: AccountId, filler_list: Vec<FillerInfo>), call_index(8)
    (c-pallets/file-bank/src/lib.rs:795-833); FillerInfo { block_num: u32, miner_address:
    AccountId, filler_hash: Hash } (types.rs:82-86), SCALE: u32 LE ++ 32 bytes ++ 64 bytes."""
    tee = acct(9)
    fl = [records.FillerInfo(1000 + i, acct(i), hx("filler", i)) for i in range(10)]
    got = records.upload_filler(tee, fl)
    want = bytes([60, 8]) + tee + compact(10) + b"".join(
        struct.pack("<I", f.block_num) + f.miner_address + f.filler_hash for f in fl)
    assert got == want
    assert len(got) == 2 + 32 + 1 + 10 * (4 + 32 + 64)
    assert records.upload_filler(tee, []) == bytes([60, 8]) + tee + compact(0)
    import cess_amd
    with pytest.raises(cess_amd.CecError):  # UploadFillerLimit = 10 (runtime/src/lib.rs:1033)
        records.upload_filler(tee, fl + fl[:1])
    calls = records.upload_filler_calls(tee, fl * 2 + fl[:3])
    assert [c[34] for c in calls] == [compact(10)[0], compact(10)[0], compact(3)[0]]
    assert calls[0] == got
    bad = [records.FillerInfo(1, acct(1), b"Z" * 64)]
    with pytest.raises(cess_amd.CecError):
        records.upload_filler(tee, bad)


def test_restoral_call_data():
    """The restoral calls of c-pallets/file-bank/src/lib.rs:940-1122 (pallet 60): Hash arguments
    are 64 bytes, AccountId 32, in declaration order."""
    fh, fr, miner = hx("file", 3), hx("frag", 7), acct(5)
    assert records.generate_restoral_order(fh, fr) == bytes([60, 13]) + fh + fr
    assert records.claim_restoral_order(fr) == bytes([60, 14]) + fr
    assert records.claim_restoral_exist_order(miner, fh, fr) == bytes([60, 15]) + miner + fh + fr
    assert records.restoral_order_complete(fr) == bytes([60, 16]) + fr
    import cess_amd
    with pytest.raises(cess_amd.CecError):
        records.restoral_order_complete(b"A" * 64)


def test_audit_random_subject():
    """Audit::random_number(seed) (c-pallets/audit/src/lib.rs:1067-1076) hands the chain's
    randomness (T::MyPalletId::get(), seed).encode(): PalletId([u8; 8]) then u32 LE; the audit
    pallet's MyPalletId is SegbkPalletId = PalletId(*b"rewardpt") (runtime/src/lib.rs:984,1004).
    The output's first 8 bytes decode as u64 LE."""
    assert records.AUDIT_PALLET_ID == b"rewardpt"
    for seed in (0, 1, 47, 20220509, 0xFFFFFFFF):
        assert records.audit_random_subject(seed) == b"rewardpt" + struct.pack("<I", seed)
    assert records.audit_random_subject(5, b"py/trsry") == b"py/trsry" + struct.pack("<I", 5)
    r = bytes(range(32))
    assert records.audit_random_u64(r) == struct.unpack("<Q", r[:8])[0]
    import cess_amd
    with pytest.raises(cess_amd.CecError):
        records.audit_random_u64(b"1234567")
    # the challenge chain: randomness per seed -> u64 -> cec_challenge_indices (blake2b stands
    # in for the chain randomness, which is chain state and not reproducible offline)
    from cess_amd import audit
    rnd = [hashlib.blake2b(records.audit_random_subject(s), digest_size=32).digest()
           for s in range(1, 200)]
    idx, used = audit.challenge_indices([records.audit_random_u64(x) for x in rnd])
    want = []
    for x in rnd:
        i = struct.unpack("<Q", x[:8])[0] % 1024
        if i not in want:
            want.append(i)
        if len(want) == 47:
            break
    assert list(idx) == want and used == 48


def _random_list_restated(now, randomness_of, need=47):
    """c-pallets/audit/src/lib.rs:966-974 with generate_challenge_random (:1079-1096) inlined,
    line for line: seed from `now`, seed += 1, increase = seed + 1, randomness of
    (MyPalletId, increase).encode(), H256 decode, first 20 bytes, pushed unless already listed.
    `randomness_of(subject)` stands in for T::MyRandomness (None -> Default::default())."""
    random_list = []
    seed = now
    while len(random_list) < need:
        seed = seed + 1
        increase = seed
        while True:
            increase += 1
            r_seed = randomness_of(records.AUDIT_PALLET_ID + struct.pack("<I", increase))
            random_seed = r_seed if r_seed is not None else bytes(32)
            if len(random_seed) >= 20:
                random_number = random_seed[0:20]
                break
        if random_number not in random_list:
            random_list.append(random_number)
    return random_list


@pytest.mark.parametrize("now", [0, 1, 20220509])
def test_challenge_random_list(now):
    """NetSnapShot.random_list: cec_challenge_random_list over the randomness outputs for
    subjects (MyPalletId, now + 2 + i) equals the pallet's loop, duplicates and None outputs
    included (blake2b stands in for the chain's randomness, which is chain state)."""
    from cess_amd import audit

    def rnd(subject):
        seed = struct.unpack("<I", subject[8:])[0]
        if seed % 11 == 3:
            return None  # the randomness source had no output: Default (zeros)
        # every 5th subject repeats an earlier output: the loop must skip the duplicate
        key = seed - (seed % 5 == 0) * 2
        return hashlib.blake2b(records.AUDIT_PALLET_ID + struct.pack("<I", key),
                               digest_size=32).digest()

    want = _random_list_restated(now, rnd)
    outputs = [rnd(records.audit_random_subject(now + 2 + i)) for i in range(80)]
    got, used = audit.challenge_random_list(outputs)
    assert got == want and len(got) == audit.CHALLENGE_NEED
    assert len(set(got)) == len(got)
    # consumed exactly up to the 47th distinct value
    assert audit.challenge_random_list(outputs[:used])[0] == want
    import cess_amd
    with pytest.raises(cess_amd.CecError):
        audit.challenge_random_list(outputs[:used - 1])
    with pytest.raises(ValueError):
        audit.challenge_random_list([b"short"])
