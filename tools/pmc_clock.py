"""Shader clock under each kernel of a rocprofv3 --pmc run that collected GRBM_GUI_ACTIVE
(+ SQ_INSTS_VALU, SQ_WAVES): clock = GRBM_GUI_ACTIVE / XCDs / kernel duration (the counter sums
the busy cycles of the 8 XCDs, MI355X_MICROARCH.md), duration-weighted over the dispatches of
each kernel. Writes a JSON summary.
usage: python tools/pmc_clock.py <counter_collection.csv> <out.json> [xcds=8]"""
import csv
import json
import sys
from collections import defaultdict


def main():
    path, out = sys.argv[1], sys.argv[2]
    xcds = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    disp = defaultdict(dict)  # dispatch -> {counter: value, name, dur}
    with open(path) as f:
        for r in csv.DictReader(f):
            d = disp[r["Dispatch_Id"]]
            d["name"] = r["Kernel_Name"]
            d["dur"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            d["grid"] = int(r["Grid_Size"])
            d[r["Counter_Name"]] = float(r["Counter_Value"])
    per = defaultdict(lambda: {"dispatches": 0, "ns": 0, "grbm": 0.0, "valu": 0.0, "waves": 0.0})
    for d in disp.values():
        key = d["name"].split("(")[0]
        p = per[key]
        p["dispatches"] += 1
        p["ns"] += d["dur"]
        p["grbm"] += d.get("GRBM_GUI_ACTIVE", 0.0)
        p["valu"] += d.get("SQ_INSTS_VALU", 0.0)
        p["waves"] += d.get("SQ_WAVES", 0.0)
    res = {}
    for key, p in per.items():
        if not p["ns"]:
            continue
        res[key] = {"dispatches": p["dispatches"], "mean_us": round(p["ns"] / p["dispatches"] / 1e3, 3),
                    "clock_GHz": round(p["grbm"] / xcds / p["ns"], 4),
                    "valu_per_wave": round(p["valu"] / p["waves"], 1) if p["waves"] else None}
    json.dump({"source": path, "xcds": xcds, "basis": "GRBM_GUI_ACTIVE / xcds / duration, "
               "duration-weighted over the dispatches of each kernel", "kernels": res},
              open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
