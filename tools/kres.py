#!/usr/bin/env python3
"""Per-kernel register / LDS / spill usage of a built HIP object (gfx950 code object notes).
usage: python tools/kres.py build/obj/sha256.o [name-regex]"""
import re
import subprocess
import sys
import tempfile

B = "/opt/rocm/lib/llvm/bin"
KEYS = ["vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
        "group_segment_fixed_size", "private_segment_fixed_size"]


def main():
    obj, pat = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""
    with tempfile.TemporaryDirectory() as t:
        subprocess.run([f"{B}/llvm-objcopy", f"--dump-section=.hip_fatbin={t}/fb.bin", obj],
                       check=True)
        subprocess.run([f"{B}/clang-offload-bundler", "--unbundle", "--type=o",
                        f"--input={t}/fb.bin", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--output={t}/k.co"], check=True)
        notes = subprocess.run([f"{B}/llvm-readelf", "--notes", f"{t}/k.co"], check=True,
                               capture_output=True, text=True).stdout
    # each kernel's metadata map: keys appear in alphabetical order, .name before .vgpr_*
    cur, rows = {}, []
    for line in notes.splitlines():
        m = re.match(r"\s+\.([a-z_]+):\s+(\S+)", line)
        if not m:
            continue
        cur[m.group(1)] = m.group(2)
        if m.group(1) == "vgpr_spill_count":
            rows.append(dict(cur))
    for r in rows:
        if re.search(pat, r.get("name", "")):
            vals = " ".join(f"{k.replace('_count', '').replace('_fixed_size', '')}={r.get(k)}"
                            for k in KEYS)
            print(f"{r.get('name', '?')[:72]:72s} {vals}")


if __name__ == "__main__":
    main()
