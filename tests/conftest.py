import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def _ensure_oracle():
    so = os.path.join(ROOT, "oracle", "libyref.so")
    src = os.path.join(ROOT, "oracle", "yref.c")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


_ensure_oracle()


@pytest.fixture(scope="session")
def golden():
    import json

    out = {}
    for name in ("kat", "map", "array", "nested"):
        with open(os.path.join(ROOT, "tests", "golden", f"{name}.json")) as f:
            out[name] = json.load(f)["cases"]
    return out
