"""bench.py's `--gpus N` contract (CPU): N ranks or a non-zero exit, never a silent one-GPU line.
The driver's multi-GPU scaling run is `bench.py --gpus N` (under torchrun or alone)."""
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
