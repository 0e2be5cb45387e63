"""`any` encodings lib0's writeAny never produces but readAny accepts, against Yjs 13.5.16
(tests/golden/anyform.json, tests/golden/gen/gen_anyform_fixtures.js). Yjs holds `any` content as
JS values and writes them back with writeAny, so its output is in writeAny's form: integer floats
as varints, float32-exact float64s as float32, NaN as 0x7FF8000000000000, overlong varuints /
varints shortened. The engine flags such content at decode (yc_parse.h ANY_REENCODE) and its
encoders write it canonically (yc_work.h any_canon): Y.applyUpdate + encodeStateAsUpdate,
Y.mergeUpdates and Y.diffUpdate give Yjs's bytes. Object keys that JS reorders (array indices
after other keys) or drops ("__proto__") are refused (YCRDT_E_UNSUPPORTED), as listed.
"""
import json
import os

import pytest

crdt_amd = pytest.importorskip("crdt_amd")

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _cases():
    with open(os.path.join(HERE, "golden", "anyform.json")) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("mode", ["direct", "wave", "chunks"])
def test_anyform_apply(mode, monkeypatch):
    monkeypatch.setenv("YCRDT_DECODE", "direct" if mode == "wave" else mode)
    monkeypatch.setenv("YCRDT_DIRECT_WAVE", "1" if mode == "wave" else "0")
    for c in _cases():
        u = bytes.fromhex(c["update"])
        d = crdt_amd.Doc(client_id=5)
        if c["refused"]:
            with pytest.raises(crdt_amd.YcrdtError):
                d.apply_update(u)
            continue
        d.apply_update(u)
        assert d.encode_state_as_update().hex() == c["state"], c["name"]
        assert d.encode_state_vector().hex() == c["sv"], c["name"]
        if c["json"] is not None:
            assert json.loads(d.root_json("users", "map")) == c["json"], c["name"]
        # beside another update (general encode path: two clients)
        b = crdt_amd.Batch([u, bytes.fromhex(c["other"])])
        b.merge()
        d2 = crdt_amd.Doc(client_id=5)
        d2.apply_updates([u, bytes.fromhex(c["other"])])
        assert b.result()[0] == d2.encode_state_as_update(), c["name"]


def test_anyform_doc_remerge():
    """The doc's state holds what Yjs holds (writeAny of the values readAny built), and a later merge
    into the doc keeps it: a doc state is never rewritten again (an own "__proto__" member that
    writeAny wrote after a `"__proto__": null` would be read back as the prototype setter)."""
    for c in _cases():
        if c["refused"]:
            continue
        d = crdt_amd.Doc(client_id=5)
        d.apply_update(bytes.fromhex(c["update"]))
        assert d.encode_state_as_update().hex() == c["state"], c["name"]
        d.apply_update(bytes.fromhex(c["other"]))
        assert d.encode_state_as_update().hex() == c["state_with_other"], c["name"]


def test_anyform_merge_and_diff():
    for c in _cases():
        if c["refused"]:
            continue
        u, o = bytes.fromhex(c["update"]), bytes.fromhex(c["other"])
        assert crdt_amd.merge_updates([u, o]).hex() == c["merged"], c["name"]
        assert crdt_amd.diff_update(u, b"\x00").hex() == c["diff"], c["name"]
