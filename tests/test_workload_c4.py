"""The C4 workload generator (crdt_amd/workload/ycw_nested.cpp) produces updates the Yjs restatement
accepts, with the nested-array shape C4 names: every key of 'docs' holds a YArray, some replaced by
a replica's own array (nested-type GC), concurrent appends and deletes. (The generator itself is not
pinned to Yjs — parity unpinned — the GPU tests compare the engine with the oracle on its output.)"""
import json

from crdt_amd.workload import gen_nested
from oracle.yref import Doc


def test_c4_generator_shape_and_oracle_accepts():
    ups, st = gen_nested(12, 40, 150, seed=5)
    assert len(ups) == 13 and st["items"] > 1000 and st["deletes"] > 0
    d = Doc(0x7FFFFFF0)
    for u in ups:
        d.apply_update(u)
    j = json.loads(d.root_json("docs", "map"))
    assert len(j) == 40 and all(isinstance(v, list) for v in j.values())
    # order independence on the oracle: the base, then the replicas in reverse order
    r = Doc(0x7FFFFFF0)
    for u in [ups[0]] + ups[:0:-1]:
        r.apply_update(u)
    assert r.encode_state_as_update() == d.encode_state_as_update()


def test_c4_generator_deterministic():
    assert gen_nested(5, 10, 40, seed=3) == gen_nested(5, 10, 40, seed=3)
