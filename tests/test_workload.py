"""The synthetic workload generator (crdt_amd/workload) is pinned byte-for-byte against real Yjs
(tests/golden/workload.json, made by tests/golden/gen/make_workload_pins.py), and the oracle
reproduces Yjs's merged state of those batches."""
import json
import os

import pytest

from crdt_amd.workload import gen_map
from oracle.yref import Doc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def pins():
    with open(os.path.join(ROOT, "tests", "golden", "workload.json")) as f:
        return json.load(f)["cases"]


def test_generator_matches_yjs(pins):
    for c in pins:
        ups, _ = gen_map(**c["cfg"])
        assert [u.hex() for u in ups] == c["updates"], c["name"]


def test_oracle_merges_pinned_workloads(pins):
    for c in pins:
        d = Doc(0x7FFFFFF0)
        for u in c["updates"]:
            d.apply_update(bytes.fromhex(u))
        assert d.encode_state_as_update().hex() == c["state"], c["name"]
        assert json.loads(d.root_json("users", "map")) == c["json"], c["name"]


def test_generator_deterministic():
    a, _ = gen_map(n_keys=100, n_replicas=5, ops_per_replica=50, seed=9)
    b, _ = gen_map(n_keys=100, n_replicas=5, ops_per_replica=50, seed=9)
    c, _ = gen_map(n_keys=100, n_replicas=5, ops_per_replica=50, seed=10)
    assert a == b and a != c
