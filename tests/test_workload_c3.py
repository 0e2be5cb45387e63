"""The C3-shaped YArray generator (crdt_amd/workload/ycw_array.cpp; bench and GPU property input),
no GPU: its updates decode, and the list order it keeps for the replica views (an independent
re-implementation of the origin-tree YATA) is the order the CPU oracle (oracle/yref.c, sequential
Yjs restatement) integrates the same updates into."""
import json

import pytest

from crdt_amd.workload import gen_array
from oracle.yref import Doc as ODoc
from oracle.ymerge import ITEM, Dec, lazy_structs


def _any_json(b, p):
    t = b[p]
    if t == 119:
        n = b[p + 1]
        return b[p + 2:p + 2 + n].decode(), p + 2 + n
    assert t == 125
    r = b[p + 1]
    v, shift, q = r & 63, 6, p + 2
    while r & 0x80:
        r = b[q]
        v |= (r & 0x7F) << shift
        shift += 7
        q += 1
    return v, q


@pytest.mark.parametrize("reps,rounds,items,seed", [(8, 4, 4000, 1), (32, 6, 20000, 2), (64, 3, 12000, 3)])
def test_generator_order_is_the_oracle_order(reps, rounds, items, seed):
    ups, st = gen_array(reps, rounds, items, seed, order=True)
    assert len(ups) == reps * rounds
    vals = {}
    for u in ups:
        for s in lazy_structs(Dec(u)):
            if s.kind != ITEM:
                continue
            for i, raw in enumerate(s.content):
                vals[(s.client, s.clock + i)] = _any_json(raw, 0)[0]
    d = ODoc(0x7FFFFFF0)
    for u in ups:
        d.apply_update(u)
    got = json.loads(d.root_json("messages", "array"))
    assert got == [vals[k] for k in st["order"]]
