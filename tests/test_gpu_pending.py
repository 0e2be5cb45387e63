"""Yjs pending-struct semantics on the GPU path, byte for byte against Yjs 13.5.16.

tests/golden/pending.json (tests/golden/gen/gen_pending_fixtures.js) applies seeded replica deltas
to a fresh Yjs doc in non-causal orders (shuffled, reversed, one delta lost) and records what a
reader sees after every Y.applyUpdate: encodeStateAsUpdate (13.6 canonical client order; it carries
the parked structs and delete ranges merged in, Y@22155), encodeStateVector (integrated structs
only), a delta against a replica state vector, toJSON, and whether structs / delete ranges are
pending. The engine defers the merge to the read and replays Yjs's readUpdateV2 on struct headers
(yc_ingest.cpp) only when something is missing.
"""
import json
import os

import pytest

crdt_amd = pytest.importorskip("crdt_amd")
from tests.v1util import canonical_update  # noqa: E402

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cases():
    with open(os.path.join(ROOT, "tests", "golden", "pending.json")) as f:
        return json.load(f)["cases"]


def _canon_sv(b: bytes) -> bytes:
    from oracle.ymerge import decode_sv

    e = sorted(decode_sv(b).items(), key=lambda t: -t[0])
    out = bytearray()

    def vu(v):
        while v > 0x7F:
            out.append(0x80 | (v & 0x7F))
            v >>= 7
        out.append(v)

    vu(len(e))
    for c, k in e:
        vu(c)
        vu(k)
    return bytes(out)


def _check_step(d, c, k, st):
    tag = (c["name"], k)
    assert d.pending() == (st["pending"], st["pending_ds"]), tag
    assert d.encode_state_as_update().hex() == st["state"], tag
    assert _canon_sv(d.encode_state_vector()).hex() == st["sv"], tag
    if "delta" in st:
        got = d.encode_state_as_update(bytes.fromhex(st["delta"]["sv"]))
        assert got.hex() == st["delta"]["update"], tag
    for name, kind in c["roots"].items():
        assert json.loads(d.root_json(name, kind)) == st["json"][name], tag


@pytest.mark.parametrize("part", range(3))
def test_pending_every_step(part):
    """A read after every apply: the doc equals Yjs's after each out-of-order delta."""
    for c in _cases()[part::3]:
        d = crdt_amd.Doc(client_id=0x7FFFFFF0)
        for k, (u, st) in enumerate(zip(c["updates"], c["steps"])):
            d.apply_update(bytes.fromhex(u))
            _check_step(d, c, k, st)


def test_pending_deferred_bursts():
    """Reads only every few applies: the deferred queue replays Yjs's sequence exactly."""
    for i, c in enumerate(_cases()):
        d = crdt_amd.Doc(client_id=0x7FFFFFF0)
        every = 2 + i % 4
        for k, (u, st) in enumerate(zip(c["updates"], c["steps"])):
            d.apply_update(bytes.fromhex(u))
            if k % every == every - 1 or k == len(c["steps"]) - 1:
                _check_step(d, c, k, st)


def test_pending_batch_apply_equals_sequential():
    for c in _cases():
        d = crdt_amd.Doc(client_id=0x7FFFFFF0)
        d.apply_updates([bytes.fromhex(u) for u in c["updates"]])
        _check_step(d, c, len(c["steps"]) - 1, c["steps"][-1])
