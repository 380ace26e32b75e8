"""Condense a config-6 warm sweep (bench.py --config 6 --erasures e, one line per decoder leg:
--fftdec-mode 1 = k_fftdec_m, 2 = k_fftdec_d, --fftdec-min 0 = the matrix decoders, then the
default chooser; see tools/gpu_r4_refit.sh) into tests/golden/fftdec_sweep_r04.json, the recorded
costs the chooser test (tests/test_host.py::test_fftdec_chooser_on_recorded_costs) replays.

usage: python tools/fftdec_sweep_golden.py profiles/r04/c6_sweep_warm30.jsonl \
           tests/golden/fftdec_sweep_r04.json
"""
import json
import re
import sys


def main(src: str, dst: str) -> None:
    rows = [json.loads(l) for l in open(src) if l.startswith("{")]
    legs = ("m", "d", "rt", "auto")
    assert len(rows) % len(legs) == 0, "one line per leg per erasure count"
    out = {"source": src, "fragment_bytes": None, "segments": None, "warmup": None,
           "steps": None, "ms": {}}
    for i in range(0, len(rows), len(legs)):
        group = rows[i:i + len(legs)]
        e = int(re.search(r"(\d+) (?:random|consecutive) erasures",
                          group[0]["config"]["workload"]).group(1))
        cfg = group[0]["config"]
        out["fragment_bytes"] = cfg["fragment_bytes"]
        out["segments"] = cfg["segments_per_gpu"]
        out["warmup"], out["steps"] = group[0]["warmup"], group[0]["steps"]
        rec = {}
        for leg, r in zip(legs, group):
            assert str(e) in r["config"]["workload"]
            rec[leg] = r["roofline"]["launch_ms"]
        rec["auto_kernel"] = group[3]["config"]["kernel"]
        out["ms"][str(e)] = rec
    with open(dst, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
