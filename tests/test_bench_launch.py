"""bench.py's `--gpus N` contract (CPU): N ranks or a non-zero exit, never a silent one-GPU line.
The driver's multi-GPU scaling run is `bench.py --gpus N` (under torchrun or alone)."""
import json
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_world_check_decisions():
    wc = bench.world_check
    assert wc(1, {}, None) == ("run", 1)
    assert wc(8, {"WORLD_SIZE": "8"}, None) == ("run", 8)
    assert wc(4, {}, 8) == ("launch", 4)
    assert wc(8, {}, 8) == ("launch", 8)
    # fewer GPUs than asked: an error, not a one-GPU line
    what, msg = wc(8, {}, 1)
    assert what == "error" and "1 GPU" in msg
    what, msg = wc(2, {}, 0)
    assert what == "error"
    # an external launcher with a different world size
    what, msg = wc(8, {"WORLD_SIZE": "2"}, None)
    assert what == "error" and "WORLD_SIZE=2" in msg
    what, _ = wc(1, {"WORLD_SIZE": "4"}, None)
    assert what == "error"
    # rehearsal: ranks share device 0 on a one-GPU box
    assert wc(2, {"CESS_DEVICE": "0"}, 1) == ("launch", 2)
    assert wc(0, {}, 8)[0] == "error"


def _run(args, env_extra):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                          capture_output=True, text=True, timeout=240, env=env)


def test_world_size_mismatch_exits_nonzero():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"], {"WORLD_SIZE": "3"})
    assert r.returncode == 2, (r.stdout, r.stderr)
    assert "WORLD_SIZE=3" in r.stderr
    assert r.stdout.strip() == ""  # no bench line


def test_too_few_gpus_exits_nonzero():
    import torch
    if torch.cuda.device_count() >= 64:
        pytest.skip("this host has 64 GPUs")
    r = _run(["--gpus", "64", "--steps", "1", "--warmup", "0"], {})
    assert r.returncode == 2, (r.stdout, r.stderr)
    assert "--gpus 64" in r.stderr
    assert r.stdout.strip() == ""


def test_kernel_label_every_config():
    """bench.py's line names its dominant kernel for every config (config 6 from the share of
    segments each FFT-domain decoder took), with no GPU."""
    import bench
    for cfg in (2, 3, 4, 5, 7, 8):
        assert bench.kernel_label(cfg, None, 1, False, 0, 2).startswith("k_")
    assert bench.kernel_label(6, 1.0, 8, False, 0, 32) == "k_fftdec_m"
    assert bench.kernel_label(6, 0.0, 32, False, 0, 32) == "k_rthx<8>"
    assert bench.kernel_label(6, 0.0, 3, False, 0, 32) == "k_rtb"
    assert "50%" in bench.kernel_label(6, 0.5, 16, False, 0, 32)
    # the formal-derivative decoder's share (CEC_STAT_FFTDEC_D_SEGMENTS)
    assert bench.kernel_label(6, 1.0, 32, False, 0, 32, 1.0) == "k_fftdec_d"
    mixed = bench.kernel_label(6, 1.0, 24, False, 0, 32, 0.66)
    assert "k_fftdec_m (34%" in mixed and "k_fftdec_d (66%)" in mixed
    assert bench.kernel_label(2, None, 1, True, 0, 2) == "k_rthx"


def _line(n, **extra):
    line = {"metric": bench.METRIC, "value": 1.0, "unit": "GB/s", "n_gpus": n, "steps": 1,
            "warmup": 1, "ms_per_step": 1.0, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"baseline_config": 2},
            "roofline": {"bound": "hbm", "achieved": 1, "peak": 8000, "unit": "GB/s",
                         "frac": 0.1, "traffic": None},
            "cpu_baseline": {"value": 1, "unit": "GB/s", "cores": 16 * n, "kind": "port",
                             "sample": "s", "gpus_in_use": n, "host_cpus_visible": 256}}
    line.update(extra)
    return line


C4 = {"tN_ms": 2.1, "t1_ms": 16.4, "efficiency": 0.97, "bit_exact_sampled": True}


def test_line_keys_config4():
    """Config 4's 64 GiB strong-scaling encode is in the default line at every N, bit-exact on
    its sampled segments, with T1 and the efficiency."""
    for n in (1, 8):
        assert not any("config4" in p for p in bench.line_problems(_line(n, extra={"config4": C4})))
        gone = bench.line_problems(_line(n, extra={}))
        assert "extra.config4 missing, unmeasured or not bit-exact" in gone
        wrong = bench.line_problems(_line(n, extra={"config4": dict(C4, bit_exact_sampled=False)}))
        assert "extra.config4 missing, unmeasured or not bit-exact" in wrong
        no_t1 = {k: v for k, v in C4.items() if k != "efficiency"}
        assert "extra.config4 lacks T1 / efficiency" in bench.line_problems(
            _line(n, extra={"config4": no_t1}))


def test_line_keys_host_e2e():
    """The host-resident leg's records: the GPU-hashed ones checked against hashlib and the C
    oracle, the host-hashed and hybrid ones equal to the GPU-hashed ones, and the records_stream
    leg (SegmentCount-size files back to back) present with its sampled records right."""
    ok = {"records_match_hashlib_and_oracle": True,
          "segment_lists_host_sha": {"records_equal_gpu_hashed": True},
          "segment_lists_hybrid": {"records_equal_gpu_hashed": True},
          "records_stream": {"records_equal_gpu_hashed_sampled": True}}
    assert not any("host_e2e" in p for p in bench.line_problems(
        _line(1, extra={"config4": C4, "host_e2e": ok})))
    for leg in ("segment_lists_host_sha", "segment_lists_hybrid"):
        differ = dict(ok, **{leg: {"records_equal_gpu_hashed": False}})
        assert f"extra.host_e2e.{leg} records differ from the GPU-hashed ones" in \
            bench.line_problems(_line(1, extra={"config4": C4, "host_e2e": differ}))
    unchecked = dict(ok, records_match_hashlib_and_oracle=False)
    assert "extra.host_e2e records unchecked or wrong" in bench.line_problems(
        _line(1, extra={"config4": C4, "host_e2e": unchecked}))
    no_stream = {k: v for k, v in ok.items() if k != "records_stream"}
    assert "extra.host_e2e.records_stream missing or its records wrong" in bench.line_problems(
        _line(1, extra={"config4": C4, "host_e2e": no_stream}))


def test_line_keys_multi_gpu():
    """The N > 1 default line must carry cpu_baseline at the node's CPU share and both
    degraded-read transports (torch group, libcessec's own RCCL communicator) bit-exact."""
    ok_leg = {"bit_exact": True, "gather_GBps": 1.0}
    extra = {"config4": C4, "degraded_gather": ok_leg, "degraded_gather_cabi": ok_leg,
             "wide_degraded_gather": {"survivors": ok_leg, "partials": ok_leg},
             "wide_degraded_gather_cabi": {"survivors": ok_leg, "partials": ok_leg}}
    assert bench.line_problems(_line(8, extra=extra)) == []
    # the C-ABI group may be skipped only with its reason (ranks sharing one GPU)
    rehearsal = dict(extra, degraded_gather_cabi={"skipped": "ranks share one GPU"},
                     wide_degraded_gather_cabi={"skipped": "ranks share one GPU"})
    line = _line(2, extra=rehearsal)
    line["cpu_baseline"].update(cores=16, gpus_in_use=1)
    assert bench.line_problems(line) == []
    # a dropped cpu_baseline, a non-bit-exact exchange or a missing transport are problems
    no_cpu = _line(8, extra=extra)
    del no_cpu["cpu_baseline"]
    assert "missing cpu_baseline" in bench.line_problems(no_cpu)
    few = _line(8, extra=extra)
    few["cpu_baseline"]["cores"] = 16
    assert any("CPU share" in p for p in bench.line_problems(few))
    wrong = dict(extra, degraded_gather_cabi={"bit_exact": False})
    assert "extra.degraded_gather_cabi not bit-exact" in bench.line_problems(_line(8, extra=wrong))
    gone = dict(extra)
    del gone["wide_degraded_gather_cabi"]
    assert any("wide_degraded_gather_cabi" in p for p in bench.line_problems(_line(8, extra=gone)))


def test_line_keys_one_gpu():
    """The N = 1 default line carries config 5's step with checked digests and the wide-code
    legs with their cold means."""
    extra = {"config4": C4, "config5": {"step_GBps": 1300.0, "digests_match_hashlib": True},
             "wide_code": {"encode": {"ms": 0.37, "cold_ms_first30": 0.38}}}
    assert bench.line_problems(_line(1, extra=extra)) == []
    assert bench.line_problems(_line(1, extra=dict(extra, config5={"step_GBps": 1.0})))
    cold_less = dict(extra, wide_code={"encode": {"ms": 0.37}})
    assert bench.line_problems(_line(1, extra=cold_less)) == ["wide_code.encode lacks its cold mean"]


# problems line_problems() reports for lines recorded before round 6 added the leg
R06_NEW = {"extra.host_e2e.records_stream missing or its records wrong"}


@pytest.mark.parametrize("name", ["bench_default_b.json", "bench_default_c.json",
                                  "bench_default_e.json", "bench_default_g.json",
                                  "bench_default_h.json", "bench_default_i.json", "bench_default_j.json",
                                  "bench_default_k.json", "bench_default_l.json",
                                  "bench_gpus2_gloo_one_gpu_c.json", "bench_gpus4_gloo_one_gpu_c.json",
                                  "bench_gpus2_gloo_one_gpu_b.json",
                                  "bench_gpus4_gloo_one_gpu_b.json"])
def test_recorded_lines_have_every_key(name):
    """The lines round 5's GPU runs printed (profiles/r05/): the N = 1 default line and the
    one-GPU rehearsals of the N = 2 and N = 4 lines (gloo ranks sharing GPU 0) carry everything
    line_problems() asks for, except the legs round 6 added (R06_NEW)."""
    import json
    path = os.path.join(ROOT, "profiles", "r05", name)
    with open(path) as f:
        line = json.load(f)
    assert [p for p in bench.line_problems(line) if p not in R06_NEW] == []
    if line["n_gpus"] > 1:
        ex = line["extra"]
        assert ex["degraded_gather"]["bit_exact"] and ex["degraded_gather"]["backend"] == "gloo"
        assert all(ex["wide_degraded_gather"][x]["bit_exact"] for x in ("survivors", "partials"))
        assert "RCCL refuses" in ex["degraded_gather_cabi"]["skipped"]


@pytest.mark.parametrize("name", ["bench_gpus8_gloo_one_gpu.json"])
def test_recorded_round6_lines(name):
    """Round 6's recorded lines (profiles/r06/): the one-GPU rehearsal of the N = 8 default line
    (8 gloo ranks sharing GPU 0) carries every key line_problems() asks for,
    the host_e2e records_stream leg included, and its per-rank footprint (extra.resources: peak
    host RSS, HBM after config 4's T1 and shards) for all 8 ranks; its wall time (bench start to
    exit, beside it) is well inside the driver's 600 s."""
    import json
    with open(os.path.join(ROOT, "profiles", "r06", name)) as f:
        line = json.load(f)
    assert line["n_gpus"] == 8 and bench.line_problems(line) == []
    res = line["extra"]["resources"]["ranks"]
    assert sorted(r["rank"] for r in res) == list(range(8))
    assert all(r["peak_rss_GiB"] > 0 and "hbm_used_after_shards_GiB" in r for r in res)
    assert "hbm_used_after_t1_GiB" in res[0]
    with open(os.path.join(ROOT, "profiles", "r06", name.replace(".json", "_wall.json"))) as f:
        wall = json.load(f)
    assert wall["rc"] == 0 and wall["wall_s"] < 300


def test_cabi_legs_watchdog_ends_a_stalled_exchange(tmp_path):
    """bench.cabi_legs (the C-ABI exchange legs of the N > 1 line, run last): an exchange that
    never returns (a peer stuck in RCCL) does not cost the line. Past the deadline the legs are
    recorded as not finished, the line is printed, and the process exits with
    bench.WATCHDOG_EXIT (3: a rank hung in RCCL; the driver's rc records it)."""
    import subprocess
    import sys
    script = tmp_path / "stall.py"
    script.write_text(
        "import json, sys, time\n"
        f"sys.path.insert(0, {str(ROOT)!r})\n"
        "import torch\n"
        "import bench\n"
        "out = {'extra': {}}\n"
        "def stall(*a, **k):\n"
        "    time.sleep(3600)\n"
        "bench.cabi_legs(out['extra'], lambda g, **k: g, stall, None, (2, 1, 4096), 1, 0,\n"
        "                torch.device('cpu'), 2.0, lambda: print(json.dumps(out), flush=True))\n"
        "print('not reached')\n")
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=120)
    assert r.returncode == bench.WATCHDOG_EXIT == 3, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and "not reached" not in r.stdout, r.stdout
    ex = json.loads(lines[0])["extra"]
    for name in ("degraded_gather_cabi", "wide_degraded_gather_cabi"):
        assert "not finished after 2 s" in ex[name]["error"], ex


def test_cabi_legs_error_is_reported():
    """An exchange leg that raises is recorded as an error in the line (and flagged by
    line_problems), not a crash."""
    import torch
    ex = {}

    def boom(*a, **k):
        raise RuntimeError("cec_dist_create: no RCCL")

    bench.cabi_legs(ex, lambda g, **k: g, boom, None, (2, 1, 4096), 1, 0, torch.device("cpu"),
                    30.0, lambda: None)
    assert ex["degraded_gather_cabi"]["error"] == "RuntimeError: cec_dist_create: no RCCL"
    line = {"config": {"baseline_config": 2}, "n_gpus": 2, "extra": ex}
    assert any("cec_dist_create: no RCCL" in p for p in bench.line_problems(line))


def test_exchange_legs_torch_error_then_cabi():
    """The N > 1 line's exchange legs (torch group first, then the C ABI) under one watchdog: a
    torch-group leg that raises is recorded as an error and the C-ABI legs still run."""
    import torch
    ex = {}

    def gather(*a, **k):
        via = a[9] if len(a) > 9 else k.get("transport", "torch")
        if via == "torch":
            raise RuntimeError("NCCL error: unhandled system error")
        return {"bit_exact": True, "via": via}

    bench.cabi_legs(ex, lambda g, **k: dict(g), gather, None, (2, 1, 4096), 1, 0,
                    torch.device("cpu"), 30.0, lambda: None, torch_legs=True)
    assert "NCCL error" in ex["degraded_gather"]["error"]
    assert "NCCL error" in ex["wide_degraded_gather"]["error"]
    assert ex["degraded_gather_cabi"]["via"] == "cabi"
    assert ex["degraded_gather_cabi"]["transport"].startswith("libcessec")
    # (the wide legs build an RS(32,32) codec, which needs a GPU: on CPU they record that error)
    assert "NCCL error" not in json.dumps(ex["wide_degraded_gather_cabi"])
