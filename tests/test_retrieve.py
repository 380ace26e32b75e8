"""File retrieval (cess_amd.retrieve): SegmentList records + the fragments miners still serve ->
the original file. Fragments and records come from the oracle (oracle/rs_oracle.py, the checker)
on CPU; the GPU cases rebuild lost and corrupted fragments with libcessec and compare the file
byte for byte. Records: c-pallets/file-bank/src/types.rs:13-16; erasures = FragmentInfo.avail
(types.rs:64-76), the restoral flow's premise (c-pallets/file-bank/src/lib.rs:943-1122)."""
import io
import json

import numpy as np
import pytest

from cess_amd import ErrTooFewShards
from cess_amd.retrieve import (ErrRecordsInconsistent, ErrSegmentHashMismatch, Retriever,
                               record_from_json, retrieve_file)
from cess_amd.segments import FileRecord, SegmentList, file_hash


def _file(size, k, m, seg, seed=3):
    """(blob, FileRecord, {(segment, fragment): bytes}) from the oracle."""
    from oracle import rs_oracle as o
    blob = np.random.default_rng(seed).integers(0, 256, size, dtype=np.uint8).tobytes()
    rs = o.ReedSolomon(k, m)
    frags = {}
    for s in range(-(-size // seg)):
        padded = np.zeros(seg, np.uint8)
        chunk = np.frombuffer(blob[s * seg:(s + 1) * seg], np.uint8)
        padded[:len(chunk)] = chunk
        shards = rs.split(padded.tobytes())
        shards[k:] = rs.encode(shards[:k])
        for f, x in enumerate(shards):
            frags[(s, f)] = bytes(np.asarray(x, np.uint8))
    segs = [SegmentList(h, list(fl)) for h, fl in o.segment_list(blob, k, m, seg)]
    return blob, FileRecord(file_hash(segs), size, segs), frags


def _fetch(frags):
    return lambda s, f, _h: frags.get((s, f))


def test_intact_file_needs_no_gpu():
    """Every data fragment present and valid: the file comes back without a codec (no GPU)."""
    k, m, seg = 2, 1, 1 << 16
    blob, rec, frags = _file(5 * seg + 123, k, m, seg)
    out = io.BytesIO()
    with Retriever(k, m, seg) as r:
        st = r.retrieve(rec, _fetch(frags), out)
        assert r.enc is None
    assert out.getvalue() == blob
    assert st["rebuilt_segments"] == 0 and st["rejected"] == 0 and st["fetched"] == 6 * k


def test_records_json_roundtrip_and_checks():
    k, m, seg = 4, 2, 4096 * 4
    blob, rec, frags = _file(3 * seg, k, m, seg)
    again = record_from_json(json.dumps(rec.to_json()))
    assert again == rec
    out = io.BytesIO()
    retrieve_file(again, _fetch(frags), out, k, m, seg)
    assert out.getvalue() == blob
    # a record whose file hash does not cover its segments
    bad = FileRecord(b"0" * 64, rec.size, rec.segments)
    with pytest.raises(ErrRecordsInconsistent):
        retrieve_file(bad, _fetch(frags), io.BytesIO(), k, m, seg)
    # a size the segment count cannot hold
    with pytest.raises(ValueError):
        retrieve_file(FileRecord(rec.file_hash, 10 * seg, rec.segments), _fetch(frags),
                      io.BytesIO(), k, m, seg)


def test_too_few_valid_fragments_fail_before_any_rebuild():
    """More than m fragments of a segment lost or wrong: ErrTooFewShards, no codec created."""
    k, m, seg = 2, 1, 1 << 14
    blob, rec, frags = _file(4 * seg, k, m, seg)
    frags = dict(frags)
    del frags[(2, 0)]
    frags[(2, 2)] = b"\0" * (seg // k)  # wrong bytes count as lost
    r = Retriever(k, m, seg)
    with pytest.raises(ErrTooFewShards):
        r.retrieve(rec, _fetch(frags), io.BytesIO())
    assert r.enc is None
    r.close()


def test_failed_retrieval_leaves_no_file(tmp_path):
    """Retrieving to a path: written under a temporary name, renamed only when every segment
    checked out; a failure removes it."""
    k, m, seg = 2, 1, 1 << 14
    blob, rec, frags = _file(3 * seg + 5, k, m, seg)
    out = tmp_path / "f.bin"
    retrieve_file(rec, _fetch(frags), str(out), k, m, seg)
    assert out.read_bytes() == blob and not (tmp_path / "f.bin.part").exists()
    bad = dict(frags)
    del bad[(2, 0)], bad[(2, 1)]
    out2 = tmp_path / "g.bin"
    with pytest.raises(ErrTooFewShards):
        retrieve_file(rec, _fetch(bad), str(out2), k, m, seg)
    assert not out2.exists() and not (tmp_path / "g.bin.part").exists()


def test_segment_hash_checked():
    """Fragments that hash right but a segment record that does not match: refused."""
    k, m, seg = 2, 1, 1 << 14
    blob, rec, frags = _file(2 * seg, k, m, seg)
    segs = [SegmentList(b"f" * 64, rec.segments[0].fragment_list), rec.segments[1]]
    wrong = FileRecord(file_hash(segs), rec.size, segs)
    with pytest.raises(ErrSegmentHashMismatch):
        retrieve_file(wrong, _fetch(frags), io.BytesIO(), k, m, seg)


@pytest.mark.gpu
@pytest.mark.parametrize("k,m,seg,size", [(2, 1, 1 << 20, 7 * (1 << 20) - 5),
                                          (4, 2, 1 << 18, 300 * (1 << 18) + 77),
                                          (32, 32, 1 << 21, 5 * (1 << 21))])
def test_rebuilds_lost_and_corrupted(k, m, seg, size):
    """Up to m fragments per segment missing or corrupted (data and parity, every pattern
    position): the lost data fragments are rebuilt on the GPU in batches and the file is
    byte-identical; the counters say what happened."""
    blob, rec, frags = _file(size, k, m, seg, seed=k)
    rng = np.random.default_rng(size)
    frags = dict(frags)
    nseg = len(rec.segments)
    lost_data = 0
    for s in range(nseg):
        gone = rng.choice(k + m, size=int(rng.integers(0, m + 1)), replace=False)
        for j, f in enumerate(gone):
            if j % 2:
                b = bytearray(frags[(s, int(f))])
                b[len(b) // 2] ^= 0x40  # a miner serving wrong bytes
                frags[(s, int(f))] = bytes(b)
            else:
                del frags[(s, int(f))]
        lost_data += sum(int(f) < k for f in gone)
    out = io.BytesIO()
    with Retriever(k, m, seg, batch_segments=64) as r:
        st = r.retrieve(rec, _fetch(frags), out)
    assert out.getvalue() == blob
    assert st["rebuilt_fragments"] == lost_data
    assert st["rebuilt_segments"] > 0


@pytest.mark.gpu
def test_cli_encode_then_decode(tmp_path):
    """`cli encode --out DIR` then `cli decode` with a fragment deleted from every segment and one
    corrupted: the file comes back byte for byte; one more loss in a segment fails cleanly."""
    from cess_amd import cli
    seg = 1 << 20
    blob = np.random.default_rng(9).integers(0, 256, 5 * seg + 999, dtype=np.uint8).tobytes()
    src = tmp_path / "f.bin"
    src.write_bytes(blob)
    frag_dir = tmp_path / "frags"
    import contextlib
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        assert cli.main(["encode", str(src), "--out", str(frag_dir),
                         "--segment-size", str(seg)]) == 0
    recs = json.loads(buf.getvalue().strip().splitlines()[-1])
    (tmp_path / "rec.json").write_text(json.dumps(recs))
    for s, sl in enumerate(recs["segments"]):
        if s == 2:  # a data fragment with wrong bytes (fetched, rejected, rebuilt from parity)
            victim = frag_dir / sl["fragment_list"][1]
            victim.write_bytes(b"\1" * victim.stat().st_size)
        else:
            (frag_dir / sl["fragment_list"][s % 3]).unlink()
    out = tmp_path / "back.bin"
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        assert cli.main(["decode", str(tmp_path / "rec.json"), str(frag_dir), str(out),
                         "--segment-size", str(seg)]) == 0
    assert out.read_bytes() == blob
    st = json.loads(buf.getvalue().strip().splitlines()[-1])
    assert st["rejected"] == 1 and st["rebuilt_segments"] >= 1
    (frag_dir / recs["segments"][0]["fragment_list"][1]).unlink()  # segment 0: two lost
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        assert cli.main(["decode", str(tmp_path / "rec.json"), str(frag_dir), str(out),
                         "--segment-size", str(seg)]) == 2
    assert "segment 0" in json.loads(buf.getvalue().strip().splitlines()[-1])["error"]


def test_cli_decode_tampered_records_and_fragment_names(tmp_path):
    """`cli decode` answers every records problem with a JSON error and rc 2 (no traceback): a
    file hash that does not cover the segments, a size the segments cannot hold, a fragment list
    of the wrong length, unparsable JSON. dir_fetch opens only 64-hex names of regular files, so a
    crafted record cannot make decode read "../x", an absolute path or a FIFO."""
    import contextlib
    import os
    from cess_amd import cli
    from cess_amd.retrieve import dir_fetch
    k, m, seg = 2, 1, 1 << 14
    blob, rec, frags = _file(3 * seg + 5, k, m, seg)
    d = tmp_path / "frags"
    d.mkdir()
    for (s, f), b in frags.items():
        (d / rec.segments[s].fragment_list[f].decode()).write_bytes(b)
    good = rec.to_json()

    def run(obj_or_text):
        p = tmp_path / "rec.json"
        p.write_text(obj_or_text if isinstance(obj_or_text, str) else json.dumps(obj_or_text))
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            rc = cli.main(["decode", str(p), str(d), str(tmp_path / "out.bin"), "--segment-size",
                           str(seg)])
        return rc, json.loads(buf.getvalue().strip().splitlines()[-1])

    rc, st = run(good)
    assert rc == 0 and (tmp_path / "out.bin").read_bytes() == blob
    bad_hash = dict(good, file_hash="0" * 64)
    bad_size = dict(good, size=100 * seg)
    short = json.loads(json.dumps(good))
    short["segments"][1]["fragment_list"] = short["segments"][1]["fragment_list"][:2]
    for obj, what in [(bad_hash, "ErrRecordsInconsistent"), (bad_size, "ValueError"),
                      (short, ""), ("{not json", "records")]:
        rc, st = run(obj)
        assert rc == 2 and what in st["error"], (what, st)
    # fragment names from the records
    fetch = dir_fetch(str(d))
    h = rec.segments[0].fragment_list[0]
    assert fetch(0, 0, h) == frags[(0, 0)]
    (tmp_path / "secret").write_bytes(b"x")
    for name in (b"../secret", str(tmp_path / "secret").encode(), h.upper(), h[:63], h + b"0"):
        assert fetch(0, 0, name) is None
    fifo = d / ("f" * 64)
    os.mkfifo(fifo)
    assert fetch(0, 0, b"f" * 64) is None  # not a regular file: no blocking open / read
    (d / ("e" * 64)).mkdir()
    assert fetch(0, 0, b"e" * 64) is None
