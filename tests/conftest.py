import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "rs_golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def orc():
    """Python oracle module (test infrastructure)."""
    from oracle import rs_oracle
    return rs_oracle


@pytest.fixture(scope="session")
def corc():
    """C oracle (test infrastructure), built on demand."""
    from oracle.c_oracle import load_c_oracle
    return load_c_oracle()


def parse_shavs(name):
    """[(msg bytes, md hex)] from a NIST SHAVS .rsp file (reference fixture)."""
    out, ln, msg = [], None, None
    with open(os.path.join(GOLDEN, name)) as f:
        for line in f:
            line = line.strip()
            if line.startswith("Len ="):
                ln = int(line.split("=")[1])
            elif line.startswith("Msg ="):
                msg = bytes.fromhex(line.split("=")[1].strip())
            elif line.startswith("MD =") and ln is not None:
                out.append((msg[: ln // 8], line.split("=")[1].strip()))
                ln = msg = None
    return out


def case_data(case):
    """Regenerate a golden case's data shards (tests/golden/gen_golden.py:make_data)."""
    from tests.golden.gen_golden import make_data
    return make_data(case["k"], case["len"], case["pattern"], case["code_id"])
