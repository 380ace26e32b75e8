#!/usr/bin/env python3
"""Fit the RS(32,32) decoder cost model (cess_amd/csrc/fftdec_cost.h) to a warm config-6 sweep
(tools/gpu_r4_refit.sh: every decoder forced, then the default chooser, at 4..32 random erasures;
tools/fftdec_sweep_golden.py condenses it). Per-batch features come from the chooser tool
(tests/native/fftdec_chooser.cpp) over bench.py's own patterns: the per-segment means of
outputs x syndrome slots for each size class of the syndrome-row decoder. Least squares:
  k_fftdec_m ~ a + b_small * rows_small + b_big * rows_big + c * frac_big  (per 64 x 512 KiB)
  k_fftdec_d ~ a + b * erasures, on 12..32 erasures (where the choice between them is made)
  matrix decoders ~ a + b * erasures past four outputs
Prints the constants and each leg's relative error; the header is edited by hand from them.

usage: python tools/fit_fftdec_cost.py tests/golden/fftdec_sweep_r04.json"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def features(gold):
    import bench
    es = sorted(map(int, gold["ms"]))
    with tempfile.TemporaryDirectory() as t:
        exe = os.path.join(t, "chooser")
        subprocess.run(["g++", "-std=c++20", "-O1", "-fconstexpr-ops-limit=2000000000",
                        os.path.join(ROOT, "tests", "native", "fftdec_chooser.cpp"), "-o", exe],
                       check=True)
        text = []
        for e in es:
            present = bench.erasure_patterns(32, 32, gold["segments"], e, seed=6)
            text.append(f"{len(present)} {gold['fragment_bytes']}")
            text += ["".join("1" if f else "0" for f in row) for row in present]
        r = subprocess.run([exe], input="\n".join(text) + "\n", capture_output=True, text=True,
                           check=True)
    out = []
    for line in r.stdout.splitlines():
        tok = line.split()
        out.append(dict(zip(tok[::2], map(float, tok[1::2]))))
    return es, out


def main(path: str) -> None:
    gold = json.load(open(path))
    es, feat = features(gold)
    us = {leg: np.array([gold["ms"][str(e)][leg] * 1e3 for e in es]) for leg in ("m", "d", "rt")}
    X = np.array([[1, f["rows_small"], f["rows_big"], f["frac_big"]] for f in feat])
    cm, *_ = np.linalg.lstsq(X, us["m"], rcond=None)
    print("fdm: small %.1f + %.3f * nout * nrs; big %.1f + %.3f * nout * nrs"
          % (cm[0], cm[1], cm[0] + cm[3], cm[2]))
    print("  rel err", np.round((X @ cm - us["m"]) / us["m"], 3).tolist())
    sel = [i for i, e in enumerate(es) if e >= 12]
    Xd = np.array([[1, es[i]] for i in sel])
    cd, *_ = np.linalg.lstsq(Xd, us["d"][sel], rcond=None)
    print("fdd: %.1f + %.2f * nout" % (cd[0], cd[1]))
    print("  rel err (12..32)", np.round((Xd @ cd - us["d"][sel]) / us["d"][sel], 3).tolist())
    sel = [i for i, e in enumerate(es) if e > 4]
    Xr = np.array([[1, es[i]] for i in sel])
    cr, *_ = np.linalg.lstsq(Xr, us["rt"][sel], rcond=None)
    print("rt (> 4 outputs): %.1f + %.2f * nout" % (cr[0], cr[1]))


if __name__ == "__main__":
    main(sys.argv[1])
