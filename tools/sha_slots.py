#!/usr/bin/env python3
"""VALU instructions and issue slots per 64-byte block of the one-wave hash-queue tick
(k_sha256_tick1), counted on the built gfx950 code object: the instructions of its block loop
(the backward branch whose range holds the most v_alignbit), weighted by the issue costs
measured with tools/valu_bench.hip (profiles/r01/valu_bench_*.jsonl: left shifts, v_alignbit,
v_add3, v_perm, v_bfe and v_lshl_or issue at half rate; right shifts, v_add, v_bitop3 and the
logic ops at full rate).
The loop range includes the general-path branch (unaligned / padding blocks), a few dozen
instructions the fast path skips, so the figures are a slight upper bound.

usage: python tools/sha_slots.py [cess_amd/libcessec.so] [> profiles/valu_c5.json]"""
import collections
import json
import re
import subprocess
import sys
import tempfile

B = "/opt/rocm/lib/llvm/bin"
HALF = ("v_alignbit_b32", "v_add3_u32", "v_lshlrev_b32", "v_lshl_or_b32", "v_perm_b32",
        "v_lshl_add_u32", "v_bfe_u32", "v_alignbyte_b32", "v_xad_u32", "v_mul_u32_u24")
KERNEL = r"k_sha256_tick1"


def disassemble(obj: str) -> str:
    """gfx950 disassembly of every offload bundle in `obj` (an object file holds one; the
    shared library one per linked object)."""
    out = []
    with tempfile.TemporaryDirectory() as t:
        subprocess.run([f"{B}/llvm-objcopy", f"--dump-section=.hip_fatbin={t}/fb.bin", obj,
                        f"{t}/copy"], check=True)
        fb = open(f"{t}/fb.bin", "rb").read()
        starts = [m.start() for m in re.finditer(b"__CLANG_OFFLOAD_BUNDLE__", fb)] + [len(fb)]
        for n, (a, b) in enumerate(zip(starts, starts[1:])):
            with open(f"{t}/b{n}.bin", "wb") as f:
                f.write(fb[a:b])
            subprocess.run([f"{B}/clang-offload-bundler", "--unbundle", "--type=o",
                            f"--input={t}/b{n}.bin", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                            f"--output={t}/k{n}.co"], check=True)
            out.append(subprocess.run([f"{B}/llvm-objdump", "-d", f"{t}/k{n}.co"], check=True,
                                      capture_output=True, text=True).stdout)
    return "\n".join(out)


def kernel_resources(obj: str) -> dict:
    """{kernel symbol: {vgpr_count, sgpr_count, private_segment_fixed_size, ...}} from the code
    object notes of every offload bundle in `obj`."""
    rows = {}
    with tempfile.TemporaryDirectory() as t:
        subprocess.run([f"{B}/llvm-objcopy", f"--dump-section=.hip_fatbin={t}/fb.bin", obj,
                        f"{t}/copy"], check=True)
        fb = open(f"{t}/fb.bin", "rb").read()
        starts = [m.start() for m in re.finditer(b"__CLANG_OFFLOAD_BUNDLE__", fb)] + [len(fb)]
        for n, (a, b) in enumerate(zip(starts, starts[1:])):
            with open(f"{t}/b{n}.bin", "wb") as f:
                f.write(fb[a:b])
            subprocess.run([f"{B}/clang-offload-bundler", "--unbundle", "--type=o",
                            f"--input={t}/b{n}.bin", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                            f"--output={t}/k{n}.co"], check=True)
            notes = subprocess.run([f"{B}/llvm-readelf", "--notes", f"{t}/k{n}.co"], check=True,
                                   capture_output=True, text=True).stdout
            cur = {}
            for line in notes.splitlines():
                m = re.match(r"\s+\.([a-z_]+):\s+(\S+)", line)
                if m:
                    cur[m.group(1)] = m.group(2)
                    if m.group(1) == "vgpr_spill_count":
                        rows[cur.get("name", "?")] = dict(cur)
    return rows


def loop_counts(dis: str, kernel: str = KERNEL):
    """(symbol, Counter of VALU opcodes) of the kernel's block loop."""
    lines, sym = [], None
    for ln in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", ln)
        if m:
            if sym:
                break
            if re.search(kernel, m.group(1)):
                sym = m.group(1)
            continue
        if sym and ln.startswith("\t"):
            m = re.search(r"// ([0-9A-F]+):", ln)
            tgt = re.search(r"<" + re.escape(sym) + r"\+0x([0-9a-f]+)>", ln)
            ins = ln.strip().split("//")[0].strip()
            if m and ins:
                lines.append((int(m.group(1), 16), ins, int(tgt.group(1), 16) if tgt else None))
    base = lines[0][0]
    best = None
    for i, (addr, ins, tgt) in enumerate(lines):
        if tgt is not None and ins.startswith(("s_cbranch", "s_branch")) and base + tgt < addr:
            body = [x for a, x, _ in lines if base + tgt <= a <= addr]
            n_align = sum(x.startswith("v_alignbit") for x in body)
            if best is None or n_align > best[0]:
                best = (n_align, body)
    ops = collections.Counter(x.split()[0].removesuffix("_e32").removesuffix("_e64")
                              for x in best[1] if x.startswith("v_"))
    return sym, ops


def main():
    obj = sys.argv[1] if len(sys.argv) > 1 else "cess_amd/libcessec.so"
    sym, ops = loop_counts(disassemble(obj))
    instr = sum(ops.values())
    slots = sum(n * (2 if op in HALF else 1) for op, n in ops.items())
    print(json.dumps({
        "kernel": sym, "valu_instr_per_block": instr, "issue_slots_per_block": slots,
        "half_rate_ops": {op: n for op, n in ops.items() if op in HALF},
        "full_rate_ops": {op: n for op, n in sorted(ops.items()) if op not in HALF},
        "source": "tools/sha_slots.py on cess_amd/libcessec.so (static count of the block loop; "
                  "issue costs from profiles/r01/valu_bench_*.jsonl)"}, indent=1))


if __name__ == "__main__":
    main()
