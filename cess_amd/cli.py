"""cess-ec command line.

  python -m cess_amd.cli encode <file> [<file> ...] [--out DIR] [--scale FILE] [--k 2 --m 1]
                                   [--devices 0,1,..] [--hash-on auto|hybrid|host|gpu]
      streams the files through one GPU pipeline (RS encode; SegmentList hashes by --hash-on:
      "hybrid" / "auto" = segment chains on host SHA-256 threads, the other fragments on the GPU
      hash queue, the last batches on the host; "host" = every hash on host threads; "gpu" =
      every hash on the GPU hash queue) and prints each file's SegmentList records (the
      deal_info of FileBank::upload_declaration, c-pallets/file-bank/src/lib.rs:419-428) as JSON:
      one object for one file, one line per file for several, which share one pipeline (pinned
      once) and stream back to back. --out writes every fragment as DIR/<fragment hash> while the
      files stream (host memory holds the pipeline's pinned batches, not the files). --scale
      writes the SCALE bytes of deal_info; --call also writes the whole upload_declaration call
      data (needs --account, --name, --bucket); both for a single file. A file over
      SegmentCount = 1000 segments (runtime/src/lib.rs:1026) is rejected unless
      --no-segment-limit.
  python -m cess_amd.cli verify <file> <json>
      re-encodes and compares the records.
  python -m cess_amd.cli decode <json> <fragment dir> <out file> [--k 2 --m 1]
      retrieves the file from its records and the fragments in DIR (named by hash, as encode
      --out writes them): every fragment checked against its recorded hash (a wrong one counts
      as lost), up to m lost fragments per segment rebuilt on the GPU, every segment checked
      against its recorded hash (cess_amd.retrieve).
"""
import argparse
import json
import os
import sys

from . import geometry


def _placement(args) -> str:
    """Where the record hashes ran: "gpu", "host" or "hybrid"."""
    from .pipeline import record_hash_placement
    return record_hash_placement(args.hash_on)


def _report(args, rec, st) -> dict:
    from .segments import check_file_spec, needed_space
    out = rec.to_json()
    out["check_file_spec"] = check_file_spec(rec.segments, args.k + args.m)
    out["needed_space"] = needed_space(rec.segments, args.segment_size)
    out["pipeline"] = {"seconds": round(st.seconds, 4), "read_seconds": round(st.read_seconds, 4),
                       "GBps": round(st.bytes_in / max(st.seconds, 1e-9) / 1e9, 3),
                       "hash_on": _placement(args)}
    return out


def _encode(args) -> int:
    from .records import ErrTooManySegments
    from .reedsolomon import ErrShortData
    limit = 0 if args.no_segment_limit else geometry.SEGMENT_COUNT
    if args.devices and args.out:
        print("--devices (several GPUs) does not write fragments; drop --out", file=sys.stderr)
        return 2
    if len(args.file) > 1 and (args.devices or args.scale or args.call):
        print("--devices, --scale and --call take a single file", file=sys.stderr)
        return 2
    tmp = {}
    writer = None
    if args.out:
        os.makedirs(args.out, exist_ok=True)

        def writer(f, seg, idx, view):  # hash not known yet: temporary name, renamed on its record
            path = os.path.join(args.out, f".part-{f}-{seg}-{idx}")
            with open(path, "wb") as fh:
                fh.write(memoryview(view))
            tmp[(f, seg, idx)] = path
    try:
        if args.devices:
            from .pipeline import encode_file_records_multi
            devs = [int(x) for x in args.devices.split(",")]
            rec, sts = encode_file_records_multi(args.file[0], devs, args.k, args.m,
                                                 args.segment_size, max_segments=limit,
                                                 hash_on=args.hash_on, window=args.window)
            st = sts[0]
            st.seconds = max(x.seconds for x in sts)
            st.read_seconds = max(x.read_seconds for x in sts)
            st.bytes_in = sum(x.bytes_in for x in sts)
            results = [(rec, st)]
        else:
            from .pipeline import RecordsSession, _source_size, record_hash_placement
            nseg = max(-(-_source_size(p) // args.segment_size) for p in args.file)
            results = []
            with RecordsSession(args.k, args.m, args.segment_size, args.device,
                                record_hash_placement(args.hash_on),
                                batch_segments=max(1, min(64, nseg)), window=args.window,
                                max_segments=limit) as ses:
                recs, _ = ses.encode_many(args.file, on_fragment=writer,
                                          on_file=lambda f, r, fst: results.append((r, fst)))
    except (ErrTooManySegments, ErrShortData) as e:
        for p in tmp.values():
            os.unlink(p)
        msg = (f"file exceeds SegmentCount = {geometry.SEGMENT_COUNT} segments of "
               f"{args.segment_size} bytes") if isinstance(e, ErrTooManySegments) else \
            "empty file"
        print(json.dumps({"error": msg}))
        return 2
    if args.out:
        for (f, s, i), p in tmp.items():
            os.replace(p, os.path.join(args.out,
                                       results[f][0].segments[s].fragment_list[i].decode()))
    rec, st = results[0]
    if args.scale:
        with open(args.scale, "wb") as f:
            f.write(rec.deal_info_scale())
    if args.call:
        if not (args.account and args.name and args.bucket):
            print("--call needs --account, --name and --bucket", file=sys.stderr)
            return 2
        with open(args.call, "wb") as f:
            f.write(rec.upload_declaration(bytes.fromhex(args.account), args.name.encode(),
                                           args.bucket.encode()))
    if len(results) == 1:
        json.dump(_report(args, rec, st), sys.stdout)
        print()
    else:
        for path, (r, s) in zip(args.file, results):
            out = _report(args, r, s)
            out["file"] = path
            print(json.dumps(out))
    return 0


def _decode(args) -> int:
    from .reedsolomon import ErrTooFewShards
    from .retrieve import (ErrRecordsInconsistent, ErrSegmentHashMismatch, dir_fetch,
                           record_from_json, retrieve_file)
    try:
        with open(args.records) as f:
            rec = record_from_json(f.read())
    except (ValueError, KeyError, TypeError) as e:
        print(json.dumps({"error": f"records: {type(e).__name__}: {e}"}))
        return 2
    try:
        st = retrieve_file(rec, dir_fetch(args.fragments), args.out, args.k, args.m,
                           args.segment_size, args.device)
    except (ErrTooFewShards, ErrSegmentHashMismatch, ErrRecordsInconsistent, ValueError) as e:
        # ValueError: a size / segment count the records cannot hold, a fragment count other
        # than k + m (ErrSegmentHashMismatch and ErrRecordsInconsistent are ValueErrors too)
        print(json.dumps({"error": f"{type(e).__name__}: {e}"}))
        return 2
    print(json.dumps(st))
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="cess-ec")
    sub = ap.add_subparsers(dest="cmd", required=True)
    e = sub.add_parser("encode")
    e.add_argument("file", nargs="+")
    e.add_argument("--out", default=None)
    e.add_argument("--scale", default=None, help="write deal_info's SCALE bytes here")
    e.add_argument("--call", default=None, help="write upload_declaration call data here")
    e.add_argument("--account", default=None, help="AccountId32 as 64 hex chars")
    e.add_argument("--name", default=None)
    e.add_argument("--bucket", default=None)
    e.add_argument("--k", type=int, default=geometry.DATA_SHARDS)
    e.add_argument("--m", type=int, default=geometry.PARITY_SHARDS)
    e.add_argument("--segment-size", type=int, default=geometry.SEGMENT_SIZE)
    e.add_argument("--window", type=int, default=0, help="GPU hash-queue window in batches "
                   "(0: the pipeline's default, 32 GPU / 16 hybrid)")
    e.add_argument("--hash-on", choices=("auto", "hybrid", "gpu", "host"), default="auto",
                   help="where the SegmentList hashes run (default auto = hybrid). gpu: the same "
                        "rate as hybrid on long multi-file streams at about a quarter of the "
                        "host CPU time, slower for a lone file (its 16 MiB chains drain last)")
    e.add_argument("--device", type=int, default=0)
    e.add_argument("--devices", default="",
                   help="comma list of GPUs: the file's segments sharded over them from this "
                        "process (contiguous ranges, one pipeline per GPU)")
    e.add_argument("--no-segment-limit", action="store_true")
    v = sub.add_parser("verify")
    v.add_argument("file")
    v.add_argument("records")
    d = sub.add_parser("decode")
    d.add_argument("records")
    d.add_argument("fragments")
    d.add_argument("out")
    d.add_argument("--k", type=int, default=geometry.DATA_SHARDS)
    d.add_argument("--m", type=int, default=geometry.PARITY_SHARDS)
    d.add_argument("--segment-size", type=int, default=geometry.SEGMENT_SIZE)
    d.add_argument("--device", type=int, default=0)
    args = ap.parse_args(argv)

    if args.cmd == "encode":
        return _encode(args)
    if args.cmd == "decode":
        return _decode(args)
    from .pipeline import encode_file_records
    with open(args.records) as f:
        want = json.load(f)
    got = encode_file_records(args.file, hash_on="auto")[0].to_json()
    ok = got["segments"] == want["segments"] and got["file_hash"] == want["file_hash"]
    print(json.dumps({"ok": ok}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
