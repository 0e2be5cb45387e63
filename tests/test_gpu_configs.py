"""GPU parity on reduced-scale versions of BASELINE.json configs C3 / C4 / C5, expected outputs
from Yjs 13.5.16 itself (tests/golden/configs.json, gen_config_fixtures.js):

* C3: one YArray edited by 8-16 replicas (push / unshift / insert / cut, gossip rounds) — YATA;
* C4: YMap keys holding nested YArrays, 10 % of keys overwritten (nested GC), 6-12 replicas;
* C5: 60 small docs of 2-4 clients with lagging peer state vectors — the delta the sync responder
  sends (crdt.js:286-291) and the fleet state-vector exchange (libycrdt's
  ycrdt_comm_fleet_sv_allreduce_max over RCCL).
"""
import json
import os

import pytest

crdt_amd = pytest.importorskip("crdt_amd")

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _cases(prefix):
    with open(os.path.join(HERE, "golden", "configs.json")) as f:
        return [c for c in json.load(f)["cases"] if c["name"].startswith(prefix)]


def _check(d, c):
    assert d.encode_state_as_update().hex() == c["state"], c["name"]
    assert d.encode_state_vector().hex() == c["sv"], c["name"]
    for df in c["diffs"]:
        assert d.encode_state_as_update(bytes.fromhex(df["sv"])).hex() == df["update"], c["name"]
    for root, val in c["json"].items():
        kind = "array" if isinstance(val, list) else "map"
        assert json.loads(d.root_json(root, kind)) == val, (c["name"], root)


@pytest.mark.parametrize("prefix", ["c3_", "c4_", "c5_"])
def test_gpu_config_batch(prefix):
    for c in _cases(prefix):
        d = crdt_amd.Doc(client_id=0x7FFFFFF0)
        d.apply_updates([bytes.fromhex(u) for u in c["updates"]])
        _check(d, c)


@pytest.mark.parametrize("prefix", ["c3_", "c4_", "c5_"])
def test_gpu_config_one_at_a_time(prefix):
    for c in _cases(prefix)[:20]:
        d = crdt_amd.Doc(client_id=0x7FFFFFF0)
        for u in c["updates"]:
            d.apply_update(bytes.fromhex(u))
        _check(d, c)


def test_gpu_config_merge_updates_then_apply():
    """Y.mergeUpdates of the replicas' states, applied to a fresh doc, gives Yjs's merged state."""
    for c in _cases("c3_") + _cases("c4_"):
        m = crdt_amd.merge_updates([bytes.fromhex(u) for u in c["updates"]])
        d = crdt_amd.Doc(client_id=0x7FFFFFF0)
        d.apply_update(m)
        _check(d, c)


def _fleet_worker(q):
    """A fresh process: libycrdt's own RCCL communicator (world 1), the native fleet exchange."""
    cases = _cases("c5_")
    eng = crdt_amd.Engine()
    svs = {}
    for i, c in enumerate(cases):
        d = crdt_amd.Doc(client_id=0x7FFFFFF0, engine=eng)
        d.apply_updates([bytes.fromhex(u) for u in c["updates"]])
        svs[3 * i + 1] = d.encode_state_vector()
    comm = crdt_amd.Comm(eng, 1, 0, crdt_amd.Comm.unique_id())
    try:
        got = comm.fleet_sv_allreduce_max(svs)
    finally:
        comm.close()
    q.put([(got.get(3 * i + 1, b"").hex(), c["sv"], c["name"]) for i, c in enumerate(cases)] + [(sorted(got), sorted(svs), "ids")])


def test_gpu_config_fleet_state_vectors():
    """C5 fleet: each doc merged on the GPU, its state vector through libycrdt's native fleet
    all-reduce (ycrdt_comm_fleet_sv_allreduce_max, world 1 over RCCL, in a fresh process) equals
    Yjs's."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    p = ctx.Process(target=_fleet_worker, args=(q,))
    p.start()
    p.join(180)
    assert p.exitcode == 0, p.exitcode
    for got, want, name in q.get():
        assert got == want, name
