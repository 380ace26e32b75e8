#!/usr/bin/env python3
"""Per-kernel SQ counter summary from rocprofv3 counter_collection CSVs (mean per dispatch of the
kernels whose name contains a pattern). usage: pmc_summary.py <pattern> <csv>..."""
import csv
import sys
from collections import defaultdict


def main():
    pat, files = sys.argv[1], sys.argv[2:]
    v = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                v[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(x) / len(x) for k, x in v.items()}
    w = m.get("SQ_WAVES", 0)
    out = {k: round(x) for k, x in sorted(m.items())}
    if w:
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD",
                  "SQ_INSTS_VMEM_WR"):
            if k in m:
                out[k + "_per_wave"] = round(m[k] / w, 1)
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in m:
                out[k + "_frac_of_wave_cycles"] = round(m[k] / wc, 3)
        if "SQ_INSTS_VALU" in m:  # SQ_WAVE_CYCLES counts quad-cycles (MI355X_MICROARCH.md)
            out["valu_per_wave_cycle"] = round(m["SQ_INSTS_VALU"] / (4 * wc), 3)
    print(out)


if __name__ == "__main__":
    main()
