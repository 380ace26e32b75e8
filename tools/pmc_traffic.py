#!/usr/bin/env python3
"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) into per-launch HBM bytes.

usage: pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> <kernel substr>
       <out json> [algorithmic bytes per launch]

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced streaming read, so it is
doubled; WRITE_SIZE is exact for 16 B/lane streaming stores.
"""
import csv
import json
import statistics
import sys


def per_dispatch(path, counter, kern):
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if kern not in row.get("Kernel_Name", ""):
                continue
            if row.get("Counter_Name") != counter:
                continue
            d = row.get("Dispatch_Id")
            vals[d] = vals.get(d, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    fpath, wpath, kern, out = sys.argv[1:5]
    algo = int(sys.argv[5]) if len(sys.argv) > 5 else None
    fetch = per_dispatch(fpath, "FETCH_SIZE", kern)
    write = per_dispatch(wpath, "WRITE_SIZE", kern)
    if not fetch or not write:
        sys.exit(f"no rows for {kern!r}")
    fb = statistics.median(fetch) * 1024 * 2
    wb = statistics.median(write) * 1024
    res = {"kernel": kern, "dispatches": [len(fetch), len(write)],
           "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
           "bytes_per_launch": fb + wb,
           "raw_FETCH_SIZE_KiB": statistics.median(fetch),
           "raw_WRITE_SIZE_KiB": statistics.median(write),
           "correction": "FETCH_SIZE x 2 (gfx950 wide-read undercount), KiB -> bytes"}
    if algo:
        res["algorithmic_bytes_per_launch"] = algo
        res["traffic_over_algorithmic"] = (fb + wb) / algo
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
