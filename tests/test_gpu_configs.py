"""GPU parity on reduced-scale versions of BASELINE.json configs C3 / C4 / C5, expected outputs
from Yjs 13.5.16 itself (tests/golden/configs.json, gen_config_fixtures.js):

* C3: one YArray edited by 8-16 replicas (push / unshift / insert / cut, gossip rounds) — YATA;
* C4: YMap keys holding nested YArrays, 10 % of keys overwritten (nested GC), 6-12 replicas;
* C5: 60 small docs of 2-4 clients with lagging peer state vectors — the delta the sync responder
  sends (crdt.js:286-291) and the fleet state-vector exchange (crdt_amd/fleet.py).
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


def _fleet_worker(port, q):
    """torch / RCCL first, then the engine — the order bench.py's ranks use."""
    import torch
    import torch.distributed as dist

    from crdt_amd import fleet

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{port}")
    try:
        cases = _cases("c5_")
        svs = {}
        for i, c in enumerate(cases):
            d = crdt_amd.Doc(client_id=0x7FFFFFF0)
            d.apply_updates([bytes.fromhex(u) for u in c["updates"]])
            svs[i] = d.encode_state_vector()
        got = fleet.sv_allreduce_max(svs)
        q.put([(got[i].hex(), c["sv"], c["name"]) for i, c in enumerate(cases)])
    finally:
        dist.destroy_process_group()


def test_gpu_config_fleet_state_vectors():
    """C5 fleet: each doc merged on the GPU, its state vector through the fleet all-reduce (world 1
    over RCCL, in a fresh process) equals Yjs's."""
    import multiprocessing as mp
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    p = ctx.Process(target=_fleet_worker, args=(port, q))
    p.start()
    p.join(180)
    assert p.exitcode == 0, p.exitcode
    for got, want, name in q.get():
        assert got == want, name
