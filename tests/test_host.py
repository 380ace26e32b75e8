"""CPU-side checks of the product: the C ABI library loads and exports what include/cess_ec.h
declares, host-only entry points behave, the Python mirror raises klauspost's errors, and the
product's host matrix / decode-plan builder (gf256.h) agrees with the oracle."""
import os
import re
import subprocess

import numpy as np
import pytest

from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "cess_ec.h")


def header_symbols():
    with open(HEADER) as f:
        txt = f.read()
    return sorted(set(re.findall(r"\b(cec_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from cess_amd import _lib
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 17
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib.SIGNATURES), "ctypes table and header disagree"
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                        text=True, check=True).stdout
    for s in syms:
        assert re.search(rf"\bT {s}$", nm, re.M), s


def test_library_is_gfx950_code_object():
    """The embedded offload bundle targets gfx950 only (no other GPU arch, no CUDA)."""
    from cess_amd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100", b"sm_"):
        assert other not in blob


def test_host_only_entry_points():
    from cess_amd import _lib
    lib = _lib.load()
    assert lib.cec_version().startswith(b"cessec")
    assert lib.cec_strerror(_lib.CEC_ETOOFEW) == b"too few shards given"
    assert lib.cec_strerror(_lib.CEC_ESHARDLEN) == b"shard sizes do not match"


def test_split_segment_matches_oracle(orc):
    import cess_amd
    from cess_amd import reedsolomon as rs
    enc = object.__new__(rs.Encoder)  # Split is host-only; skip device codec creation
    enc.DataShards, enc.ParityShards, enc.Shards = 2, 1, 3
    for data in (b"a", b"abcde", bytes(range(256)) * 3):
        got = rs.Encoder.Split(enc, data)
        want = orc.ReedSolomon(2, 1).split(data)
        assert [g.tobytes() for g in got] == [w.tobytes() for w in want]
    with pytest.raises(cess_amd.ErrShortData):
        rs.Encoder.Split(enc, b"")


def test_python_api_errors_without_gpu():
    import cess_amd
    with pytest.raises(cess_amd.ErrInvShardNum):
        cess_amd.New(0, 1)
    with pytest.raises(cess_amd.ErrInvShardNum):
        cess_amd.New(2, -1)
    with pytest.raises(cess_amd.ErrMaxShardNum):
        cess_amd.New(200, 57)
    enc = cess_amd.New(3, 0)  # no parity: no device codec needed
    sh = [np.ones(4, np.uint8)] * 3
    enc.Encode(sh)
    assert enc.Verify(sh)
    with pytest.raises(cess_amd.ErrTooFewShards):
        enc.Encode(sh[:2])
    with pytest.raises(cess_amd.ErrShardNoData):
        enc.Encode([np.zeros(0, np.uint8)] * 3)
    with pytest.raises(cess_amd.ErrShardSize):
        enc.Encode([np.ones(4, np.uint8), np.ones(5, np.uint8), np.ones(4, np.uint8)])


def test_records_hash_placement_arguments():
    """encode_file_records' hash_on is checked before any device work; "auto" is the hybrid
    placement, which the C pipeline refines per batch (cec_pipeline_opts.tail_batches)."""
    import io
    from cess_amd import pipeline
    with pytest.raises(ValueError, match="hash_on"):
        pipeline.encode_file_records(b"x", hash_on="cpu")
    assert pipeline._source_size(np.zeros((3, 5), np.uint16)) == 30
    assert pipeline._source_size(memoryview(bytes(7))) == 7
    assert pipeline._source_size(io.BytesIO(b"x")) is None
    place = pipeline.record_hash_placement
    assert place("auto", 1 << 30, 2, 1) == "hybrid" and place("auto", None, 32, 32) == "hybrid"
    assert place("host", 64 << 30, 2, 1) == "host" and place("gpu", 1, 2, 1) == "gpu"
    with pytest.raises(ValueError):
        place("tpu")


def test_reader_byte_counts(tmp_path):
    """The pipeline's reader reports each source's size (the hybrid tail placement needs it)."""
    import io
    from cess_amd.pipeline import _Reader
    p = tmp_path / "f"
    p.write_bytes(bytes(1000))
    for src, a, b, want in [(str(p), 0, None, 1000), (str(p), 100, 700, 600),
                            (str(p), 900, 5000, 100), (bytes(50), 10, None, 40),
                            (np.zeros(8, np.uint16), 0, None, 16), (io.BytesIO(b"x"), 0, None,
                                                                    None)]:
        r = _Reader(src, 2, a, b)
        try:
            assert r.nbytes == want
        finally:
            r.close()


def test_join(tmp_path):
    import io
    import cess_amd
    from cess_amd import reedsolomon as rs
    enc = object.__new__(rs.Encoder)
    enc.DataShards, enc.ParityShards, enc.Shards = 2, 1, 3
    shards = rs.Encoder.Split(enc, b"hello world")
    buf = io.BytesIO()
    rs.Encoder.Join(enc, buf, shards, 11)
    assert buf.getvalue() == b"hello world"
    with pytest.raises(cess_amd.ErrReconstructRequired):
        rs.Encoder.Join(enc, io.BytesIO(), [None, shards[1]], 11)
    with pytest.raises(cess_amd.ErrShortData):
        rs.Encoder.Join(enc, io.BytesIO(), shards, 100)


def test_no_gpu_fails_loudly():
    import torch
    import cess_amd
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(cess_amd.HipError):
        cess_amd.New(2, 1)


@pytest.fixture(scope="module")
def plan_dump(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("native") / "gf_plan_dump")
    subprocess.run(["g++", "-std=c++20", "-O1", "-fconstexpr-ops-limit=2000000000",
                    os.path.join(ROOT, "tests", "native", "gf_plan_dump.cpp"), "-o", exe],
                   check=True)
    return exe


@pytest.mark.parametrize("k,m", [(2, 1), (4, 2), (10, 4), (32, 32), (100, 30)])
def test_product_matrix_and_plans_match_oracle(plan_dump, orc, k, m):
    n = k + m
    rng = np.random.default_rng(n)
    pats = []
    for _ in range(4):
        e = int(rng.integers(1, m + 1))
        erased = set(rng.choice(n, size=e, replace=False).tolist())
        pats.append(("".join("0" if i in erased else "1" for i in range(n)),
                     int(rng.integers(0, 2))))
    pats.append(("0" * (m + 1) + "1" * (k - 1), 0))  # too few -> error
    args = [plan_dump, str(k), str(m)]
    for p, d in pats:
        args += [p, str(d)]
    lines = subprocess.run(args, capture_output=True, text=True, check=True).stdout.splitlines()
    e = list(map(int, lines[0].split()[1:]))
    assert e == sum(orc.build_matrix(k, n), [])
    rs = orc.ReedSolomon(k, m)
    for (p, d), line in zip(pats, lines[1:]):
        tok = line.split()
        rc = int(tok[1])
        present = [c == "1" for c in p]
        if sum(present) < k:
            assert rc == -1
            continue
        assert rc == 0
        i_in, i_out, i_coef = tok.index("in"), tok.index("out"), tok.index("coef")
        surv, outs, rows = rs.decode_plan(present, data_only=bool(d))
        assert list(map(int, tok[i_in + 1:i_out])) == surv
        assert list(map(int, tok[i_out + 1:i_coef])) == outs
        assert list(map(int, tok[i_coef + 1:])) == sum(rows, [])


def test_fftdec_plans_model(tmp_path):
    """The RS(32,32) FFT-domain decoder's plans (cess_amd/csrc/fftdec_plan.h) run through a CPU
    model of the kernel (T1 transform, syndromes, the bit-plane masks exactly as the kernel
    applies them) rebuild every erased shard of random patterns of 1..32 erasures, both sides,
    with and without data_only, equal to the product's encode matrix; the formal-derivative
    decoder's plans (fftdec_plan_d) through the byte-level 64-point IFFT / derivative / FFT on the
    same patterns (tests/native/fftdec_model.cpp)."""
    exe = str(tmp_path / "fftdec_model")
    subprocess.run(["g++", "-std=c++20", "-O1", "-fconstexpr-ops-limit=2000000000",
                    os.path.join(ROOT, "tests", "native", "fftdec_model.cpp"), "-o", exe],
                   check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "0 failures; mode D:" in r.stdout and r.stdout.strip().endswith(" 0 failures")


def _chooser_lines(exe, batches):
    """Run tests/native/fftdec_chooser.cpp over [(present [nseg][64], shard_len)]."""
    text = []
    for present, shard_len in batches:
        text.append(f"{len(present)} {shard_len}")
        text += ["".join("1" if f else "0" for f in row) for row in present]
    r = subprocess.run([exe], input="\n".join(text) + "\n", capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    out = []
    for line in r.stdout.splitlines():
        tok = line.split()
        out.append(dict(zip(tok[::2], map(float, tok[1::2]))))
    assert len(out) == len(batches)
    return out


@pytest.mark.parametrize("golden,run,model", [("fftdec_sweep_r04.json", False, True),
                                               ("fftdec_sweep_run_r04.json", True, False)])
def test_fftdec_chooser_on_recorded_costs(tmp_path, golden, run, model):
    """The RS(32,32) decoder chooser (cess_amd/csrc/fftdec_cost.h, the rule cess_ec.cpp applies
    per pattern and per batch) replayed on CPU over bench.py's config-6 patterns against the warm
    sweep recorded on the MI355X (tests/golden/fftdec_sweep_r04.json, from
    profiles/r04/c6_sweep_warm30.jsonl by tools/fftdec_sweep_golden.py): its split matches the one
    the library ran, the batch it picks never loses to the best single decoder by more than the
    run-to-run noise, and its cost model predicts every all-on-one-decoder leg. The same on
    consecutive-erasure patterns (bench.py --erasure-run, tests/golden/fftdec_sweep_run_r04.json
    from profiles/r04/c6_sweep_run_warm30.jsonl), where the chooser's split beats both decoders
    at 20..32 erasures; the model is fitted to random patterns and is not checked there (the
    decoders skip slots with nothing to read or write, which it does not count)."""
    import json
    import bench
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", golden)))
    exe = str(tmp_path / "fftdec_chooser")
    subprocess.run(["g++", "-std=c++20", "-O1", "-fconstexpr-ops-limit=2000000000",
                    os.path.join(ROOT, "tests", "native", "fftdec_chooser.cpp"), "-o", exe],
                   check=True)
    nseg, flen = gold["segments"], gold["fragment_bytes"]
    es = sorted(map(int, gold["ms"]))
    got = _chooser_lines(exe, [(bench.erasure_patterns(32, 32, nseg, e, seed=6, run=run), flen)
                               for e in es])
    for e, g in zip(es, got):
        rec = gold["ms"][str(e)]
        us = {leg: rec[leg] * 1e3 for leg in ("m", "d", "rt", "auto")}
        # the choice is the one the library made in the recorded run (its kernel label)
        label = rec["auto_kernel"]
        if label == "k_fftdec_m":
            assert g["m"] == nseg, (e, g)
        elif label == "k_fftdec_d":
            assert g["d"] == nseg, (e, g)
        else:
            pm, pd = map(int, re.findall(r"\((\d+)%", label)[:2])
            assert (round(100 * g["m"] / nseg), round(100 * g["d"] / nseg)) == (pm, pd), (e, g)
        # ... and never loses to the best single decoder (1.5 % = the sweep's run-to-run spread:
        # the auto and all-derivative legs of one assignment differ by up to 0.9 %)
        best = min(us["m"], us["d"], us["rt"])
        assert us["auto"] <= 1.015 * best, (e, us)
        if not model:
            continue
        # the model behind it: every single-decoder leg within 3 % in the band where the choice
        # is close (16..32 erasures), within 10 % below it; the chosen split within 5 %
        tol = 0.03 if e >= 16 else 0.10
        for leg, key in (("m", "cost_m"), ("d", "cost_d"), ("rt", "cost_rt")):
            assert abs(g[key] - us[leg]) <= tol * us[leg], (e, leg, g[key], us[leg])
        assert abs(g["cost_chosen"] - us["auto"]) <= 0.05 * us["auto"], (e, g, us)


@pytest.mark.parametrize("k,flen", [(2, 4096), (2, 1000), (3, 64), (1, 77)])
def test_segment_hash_shares_fragment0_stream(k, flen):
    """The host path hashes fragment 0 once for both its own hash and the segment's
    (segments.segment_and_first_fragment_hex): both digests equal independent SHA-256s."""
    import hashlib
    from cess_amd.segments import segment_and_first_fragment_hex
    rng = np.random.default_rng(k * 1000 + flen)
    seg = rng.integers(0, 256, size=(k, flen), dtype=np.uint8)
    seg_hex, d0_hex = segment_and_first_fragment_hex([memoryview(seg[i]) for i in range(k)])
    assert seg_hex == hashlib.sha256(seg.tobytes()).hexdigest().encode()
    assert d0_hex == hashlib.sha256(seg[0].tobytes()).hexdigest().encode()


LLVM = "/opt/rocm/lib/llvm/bin"


@pytest.fixture(scope="module")
def gfx950_code_object(tmp_path_factory):
    """The gfx950 code object embedded in the shipped libcessec.so: (disassembly, notes)."""
    from cess_amd import _lib
    t = tmp_path_factory.mktemp("co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={t}/fb.bin",
                    _lib.LIB_PATH, f"{t}/lib.copy"], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                    f"--input={t}/fb.bin", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                    f"--output={t}/k.co"], check=True)
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", f"{t}/k.co"], check=True,
                         capture_output=True, text=True).stdout
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", f"{t}/k.co"], check=True,
                           capture_output=True, text=True).stdout
    return dis, notes


def kernel_bodies(dis, pat):
    """{symbol: [instruction text]} for kernels whose symbol matches `pat`."""
    out, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1) if re.search(pat, m.group(1)) else None
            if cur:
                out[cur] = []
            continue
        if cur and line.startswith("\t"):
            ins = line.strip().split("//")[0].strip()
            if ins:
                out[cur].append(ins)
    return out


def test_rthx_index_mode_wait_states(gfx950_code_object):
    """k_rthx (run-time Horner with M0-indexed table XORs, kernels.hip) is correct only if every
    SALU write of M0 (s_set_gpr_idx_on / _idx / _off) is followed by one wait state before the next
    VALU, only table XORs (SRC0 in the reserved v24..v151 range) run in index mode, and nothing
    else in the kernel touches M0 (the asm blocks clobber it). Checked on the shipped code object,
    so a compiler change that moves or drops a wait state fails here, without a GPU."""
    dis, _ = gfx950_code_object
    bodies = kernel_bodies(dis, r"k_rthx")
    assert len(bodies) == 6, sorted(bodies)  # NG = 1, 2, 3, 4, 6, 8
    for name, ins in bodies.items():
        n_idx, on = 0, False
        for i, t in enumerate(ins):
            op = t.split()[0]
            if op.startswith("s_set_gpr_idx_"):
                n_idx += 1
                assert ins[i + 1].split()[0] == "s_nop", (name, i, t, ins[i + 1])
                on = op != "s_set_gpr_idx_off"
                continue
            if on and op.startswith("v_"):
                m = re.match(r"v_xor_b32_e32 v\d+, v(\d+), v\d+$", t)
                assert m and 24 <= int(m.group(1)) < 152, (name, i, t)
            assert "m0" not in t, (name, i, t)
        assert not on, name
        assert n_idx > 0, name


def test_rthx_resources(gfx950_code_object):
    """k_rthx<NG> reserves v[24, 24 + 16 NG) for its tables above a 24-register compiler budget:
    the descriptor must count them, with no scratch and no AGPRs."""
    _, notes = gfx950_code_object
    rows, cur = [], {}
    for line in notes.splitlines():
        m = re.match(r"\s+\.([a-z_]+):\s+(\S+)", line)
        if m:
            cur[m.group(1)] = m.group(2)
            if m.group(1) == "vgpr_spill_count":
                rows.append(dict(cur))
    rthx = {r["name"]: r for r in rows if "k_rthx" in r.get("name", "")}
    assert len(rthx) == 6
    for name, r in rthx.items():
        ng = int(re.search(r"k_rthxILi(\d+)E", name).group(1))
        assert int(r["private_segment_fixed_size"]) == 0, name
        assert int(r["vgpr_spill_count"]) == 0 and int(r["sgpr_spill_count"]) == 0, name
        assert int(r.get("agpr_count", 0)) == 0, name
        assert int(r["vgpr_count"]) >= 24 + 16 * ng, (name, r["vgpr_count"])


def test_sha_tick_slot_count_matches_library():
    """bench.py prices config 5's hashing against the VALU roofline with the issue slots per block
    in profiles/valu_c5.json; they must be those of the shipped k_sha256_tick1 block loop."""
    import json
    import os
    import sys
    from cess_amd import _lib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tools"))
    import sha_slots
    sym, ops = sha_slots.loop_counts(sha_slots.disassemble(_lib.LIB_PATH))
    with open(os.path.join(root, "profiles", "valu_c5.json")) as f:
        rec = json.load(f)
    assert rec["kernel"] == sym
    assert rec["valu_instr_per_block"] == sum(ops.values())
    assert ops["v_alignbit_b32"] >= 64 * 6 + 48 * 4  # every rotate of the rounds and schedule


def test_rust_crate_declares_every_header_symbol():
    """utils/ec-hip (not compiled here: no rustc) declares every C-ABI entry point of the header."""
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "utils", "ec-hip", "src", "lib.rs")) as f:
        rs = set(re.findall(r"pub fn (cec_[a-z0-9_]+)\s*\(", f.read()))
    assert rs == set(header_symbols())


def test_product_kernel_occupancy():
    """Register budgets the measured rates depend on: the RS(32,32) FFT encode at
    3 waves per SIMD (<= 168 VGPRs), the one-wave hash tick at 4 (<= 128), the bit-plane restoral
    kernel k_rtb<1..2> at 6 or more (<= 80), the fused RS(32,32) verify and the FFT-domain
    erasure decoder for more than four syndrome slots at 2 (<= 224, <= 256), the decoder for up to
    four at 3 (<= 168), the formal-derivative decoder at 3 (<= 168), none with scratch."""
    import os
    import sys
    from cess_amd import _lib
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "tools"))
    import sha_slots
    res = sha_slots.kernel_resources(_lib.LIB_PATH)
    budget = {"k_fft3232I": 168, "k_sha256_tick1": 128, "k_ct_dec1_mixed21": 64,
              "k_rtbILi1E": 80, "k_rtbILi2E": 80, "k_fft3232_verify": 224,
              "k_fftdec_m": 256, "k_fftdec_mILj0ELb0E": 168, "k_fftdec_mILj1ELb0E": 168,
              "k_fftdec_d": 168}
    scratch_cap = {}
    for pat, cap in budget.items():
        ks = {n: r for n, r in res.items() if pat in n}
        assert ks, pat
        for n, r in ks.items():
            assert int(r["vgpr_count"]) <= cap, (n, r["vgpr_count"])
            cap_s = next((v for p, v in scratch_cap.items() if p in n), 0)
            assert int(r["private_segment_fixed_size"]) <= cap_s, n


def test_host_code_under_sanitizers(tmp_path):
    """host ASan + UBSan (GPU sanitizers are unavailable on the pool). libcessec's
    host-only code (SCALE records, the degraded-read plan of every exchange, the GF(2^8) matrix
    builder and decode plans for every erasure pattern of small codes) and the CPU codec (scalar,
    AVX2, GFNI forms) run clean, leak checking on (tests/native/sanitize_host.cpp)."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
           "-O1", "-g"]
    obj = tmp_path / "oracle.o"
    subprocess.run(["gcc", "-c", *san, "-pthread", f"{root}/oracle/rs_oracle.c", "-o", str(obj)],
                   check=True)
    exe = tmp_path / "sanitize_host"
    subprocess.run(["g++", "-std=c++20", *san, "-fconstexpr-ops-limit=4000000000",
                    "-fconstexpr-loop-limit=100000000", "-D__HIP_PLATFORM_AMD__",
                    "-I/opt/rocm/include", f"{root}/tests/native/sanitize_host.cpp",
                    f"{root}/cess_amd/csrc/records.cpp", f"{root}/cess_amd/csrc/dist.cpp", str(obj),
                    "-L/opt/rocm/lib", "-lamdhip64", "-ldl", "-pthread",
                    "-Wl,-rpath,/opt/rocm/lib", "-o", str(exe)], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "sanitize host ok" in r.stdout


def test_reader_pieces():
    """A file given as several in-memory pieces is read back to back (no joined copy), across
    piece boundaries at any read size."""
    from cess_amd.pipeline import _Reader, _source_size
    rng = np.random.default_rng(4)
    parts = [rng.integers(0, 256, n, dtype=np.uint8) for n in (5 << 20, 1, 3 << 20, 777)]
    want = np.concatenate(parts)
    assert _source_size(parts) == want.size
    for cap in (1 << 20, 5 << 20, (5 << 20) + 1, 123457):
        r = _Reader(parts, 3)
        assert r.nbytes == want.size
        out, tmp = [], np.zeros(cap, np.uint8)
        try:
            while True:
                n = r(tmp.ctypes.data, cap)
                if not n:
                    break
                out.append(tmp[:n].copy())
        finally:
            r.close()
        assert np.array_equal(np.concatenate(out), want)
