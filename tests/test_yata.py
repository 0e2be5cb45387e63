"""Many-replica YArray integration (config C3's op mix, 64-256 replicas), no GPU.

* tests/golden/yata.json (gen_yata_fixtures.js, Yjs 13.5.16): the CPU oracle (oracle/yref.c)
  reproduces Yjs's merged state for 64-256 replicas' wire deltas.
* The origin-tree formulation the GPU kernels implement (yc_yata.hip; restated in
  scripts/yata_tree_proto.py) orders every list exactly like the sequential B.1 loop, on the same
  fixtures and on seeded oracle histories.
"""
import json
import os
import sys

import pytest

from oracle.yref import Doc as ODoc
from tests.v1util import canonical_update

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import yata_tree_proto as proto  # noqa: E402


def _cases():
    with open(os.path.join(ROOT, "tests", "golden", "yata.json")) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("i", range(6))
def test_oracle_matches_yjs_many_replicas(i):
    c = _cases()[i]
    d = ODoc(0x7FFFFFF0)
    for u in c["updates"]:
        d.apply_update(bytes.fromhex(u))
    assert canonical_update(d.encode_state_as_update()).hex() == c["state"], c["name"]
    assert json.loads(d.root_json("messages", "array")) == c["json"]["messages"]


@pytest.mark.parametrize("i", range(6))
def test_tree_order_equals_sequential_loop(i):
    c = _cases()[i]
    tot = [0, 0, 0, 0]
    proto.check([bytes.fromhex(u) for u in c["updates"]], c["name"], tot)
    assert tot[2] < tot[0]  # the sibling loops scan less than the whole-list loop


def test_tree_order_on_seeded_histories():
    from tests.histories import array_history

    tot = [0, 0, 0, 0]
    for seed in range(25):
        states, wire = array_history(7100 + seed, n_replicas=2 + seed % 9, rounds=2 + seed % 4, ops=3 + seed % 9)
        proto.check(states + wire, f"seed {seed}", tot)
