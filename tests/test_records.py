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
