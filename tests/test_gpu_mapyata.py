"""YMap entries whose items carry right origins, against Yjs 13.5.16 itself
(tests/golden/mapyata.json, tests/golden/gen/gen_mapyata_fixtures.js): real YATA histories of a
YArray rewritten so that the list is the YMap entry 'users'.'k'. typeMapSet never writes a right
origin, but Yjs's Item.integrate (Y@77594) orders such an entry like a YArray, keeps the last item
as the value and deletes the others; the engine takes these entries through the YATA kernels
(yc_merge.hip k_mapx_flip / k_mapx_fix) instead of the max-client descent. Only the histories whose
Yjs state is the same in both application orders are checked (one of 60 is not: Yjs deletes map
entry items at integration time, relative to what is already integrated)."""
import json
import os

import pytest

crdt_amd = pytest.importorskip("crdt_amd")

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _cases():
    with open(os.path.join(HERE, "golden", "mapyata.json")) as f:
        return [c for c in json.load(f)["cases"] if c["pending_free"]]


def test_mapyata_batch_and_sequential():
    cases = _cases()
    assert len(cases) >= 50
    for c in cases:
        ups = [bytes.fromhex(u) for u in c["updates"]]
        b = crdt_amd.Batch(ups)
        b.merge()
        out, sv = b.result()
        assert out.hex() == c["fwd"]["state"], c["name"]
        assert sv.hex() == c["fwd"]["sv"], c["name"]
        d = crdt_amd.Doc(client_id=5)
        for u in ups:  # one Y.applyUpdate at a time (the pending path where deltas arrive early)
            d.apply_update(u)
        assert d.encode_state_as_update().hex() == c["fwd"]["state"], c["name"]
        assert json.loads(d.root_json("users", "map")) == c["fwd"]["json"], c["name"]
        d2 = crdt_amd.Doc(client_id=5)
        d2.apply_updates(list(reversed(ups)))
        assert d2.encode_state_as_update().hex() == c["rev"]["state"], c["name"]
