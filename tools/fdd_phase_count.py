#!/usr/bin/env python3
"""Per-phase VALU instruction count of k_fftdec_d (the RS(32,32) formal-derivative decoder) on the
gfx950 code object: builds tools/fdd_phases.hip (probe kernels that run one phase each on a lane's
16 x 8 register slots) and counts each probe's VALU instructions against the empty probe, then
scales to one 512-column block at 32 erasures (every slot holds an output: 16 input and 16 output
transposes and multiplies). CPU only (hipcc cross-compiles).

usage: python tools/fdd_phase_count.py [> profiles/r04/fdd_phase_counts.txt]"""
import collections
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import sha_slots  # noqa: E402  (disassembler of the offload bundle)


def counts(obj: str):
    d = sha_slots.disassemble(obj)
    out = {}
    for name in ("p_none", "p_tr8", "p_mul", "p_ifft64", "p_derivative", "p_fft64_upper",
                 "p_fft64_tail"):
        m = re.search(r"<_ZN3cec\d+" + name + r"\w*>:\n(.*?)\n\n", d, re.S)
        c = collections.Counter()
        for line in m.group(1).splitlines():
            tok = line.strip().split()
            if tok and tok[0].startswith("v_"):
                c["dpp" if "quad_perm" in line else "valu"] += 1
                if tok[0].startswith("v_lshlrev"):
                    c["half_shift"] += 1
            elif tok and tok[0].startswith("ds_swizzle"):
                c["swizzle"] += 1
        out[name] = c
    return out


def main() -> None:
    with tempfile.TemporaryDirectory() as t:
        obj = os.path.join(t, "p.o")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20",
                        "-c", os.path.join(HERE, "fdd_phases.hip"), "-o", obj], check=True)
        c = counts(obj)
    base = c["p_none"]
    per = {k: {x: c[k][x] - base[x] for x in ("valu", "dpp", "half_shift", "swizzle")}
           for k in c}
    rows = [("transposes in + out (2 x 16 tr8)", 2, "p_tr8"),
            ("run-time multiplies in + out (2 x 16)", 2, "p_mul"),
            ("IFFT_64 (layers 0, 1 cross-lane; 2..5 in-lane)", 1, "p_ifft64"),
            ("formal derivative", 1, "p_derivative"),
            ("FFT_64 layers 5..2 (in-lane)", 1, "p_fft64_upper"),
            ("FFT_64 layers 1, 0 (cross-lane, 16 slots)", 1, "p_fft64_tail")]
    tot = collections.Counter()
    print("k_fftdec_d per 512-column block and wave at 32 erasures (VALU incl. DPP; DPP; "
          "half-rate left shifts; ds_swizzle, no VALU slot)")
    for what, times, k in rows:
        v = {x: times * per[k][x] for x in per[k]}
        tot.update(v)
        print(f"{what:52s} {v['valu'] + v['dpp']:6d} {v['dpp']:5d} {v['half_shift']:5d} "
              f"{v['swizzle']:5d}")
    print(f"{'sum':52s} {tot['valu'] + tot['dpp']:6d} {tot['dpp']:5d} {tot['half_shift']:5d} "
          f"{tot['swizzle']:5d}")


if __name__ == "__main__":
    main()
