"""cess-ec command line: `python -m cess_amd.cli encode <file> [--out DIR] [--k 2 --m 1]`
prints the file's SegmentList records (the `deal_info` of FileBank::upload_declaration,
c-pallets/file-bank/src/lib.rs:423) as JSON; with --out every fragment is written as
DIR/<fragment hash>. `verify <file> <json>` re-encodes and compares the records."""
import argparse
import json
import os
import sys

from . import geometry


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="cess-ec")
    sub = ap.add_subparsers(dest="cmd", required=True)
    e = sub.add_parser("encode")
    e.add_argument("file")
    e.add_argument("--out", default=None)
    e.add_argument("--k", type=int, default=geometry.DATA_SHARDS)
    e.add_argument("--m", type=int, default=geometry.PARITY_SHARDS)
    e.add_argument("--segment-size", type=int, default=geometry.SEGMENT_SIZE)
    e.add_argument("--device", type=int, default=0)
    v = sub.add_parser("verify")
    v.add_argument("file")
    v.add_argument("records")
    args = ap.parse_args(argv)

    from .segments import SegmentEncoder, check_file_spec, needed_space
    if args.cmd == "encode":
        se = SegmentEncoder(args.k, args.m, args.segment_size, device=args.device)
        writer = None
        if args.out:
            os.makedirs(args.out, exist_ok=True)
            pending = {}

            def writer(s, i, buf):  # hash is known only after the batch: stash, write below
                pending[(s, i)] = bytes(buf)
        rec = se.encode_file(args.file, on_fragment=writer)
        if args.out:
            for (s, i), buf in pending.items():
                with open(os.path.join(args.out, rec.segments[s].fragment_list[i].decode()),
                          "wb") as f:
                    f.write(buf)
        se.close()
        out = rec.to_json()
        out["check_file_spec"] = check_file_spec(rec.segments, args.k + args.m)
        out["needed_space"] = needed_space(rec.segments, args.segment_size)
        json.dump(out, sys.stdout)
        print()
        return 0
    with open(args.records) as f:
        want = json.load(f)
    se = SegmentEncoder()
    got = se.encode_file(args.file).to_json()
    se.close()
    ok = got["segments"] == want["segments"] and got["file_hash"] == want["file_hash"]
    print(json.dumps({"ok": ok}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
