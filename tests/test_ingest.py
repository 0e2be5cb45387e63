"""Host side of Y.applyUpdate (no GPU): the update validator and the pending-struct emulation.

* ycrdt_validate_update is what ycrdt_apply_update runs before queueing an update. It must refuse
  exactly what the CPU oracle (oracle/yref.c, restating lib0 0.2.42 / Yjs 13.5.16 decoding) refuses.
* ycrdt_debug_replay drives yc_ingest.cpp's restatement of readUpdateV2 / integrateStructs /
  readAndApplyDeleteSet (Y@21330, Y@19963, Y@11619) on struct headers, with Y.mergeUpdates supplied
  by the oracle (oracle/ymerge.py). After every apply of tests/golden/pending.json (Yjs 13.5.16
  applying replica deltas out of causal order) the emulated store state vector and the presence
  of pending structs / pending delete ranges must be Yjs's.
"""
import json
import os

import pytest

crdt_amd = pytest.importorskip("crdt_amd")
from oracle.yref import Doc as ODoc  # noqa: E402
from oracle.yref import OracleError  # noqa: E402
from oracle.ymerge import merge_updates  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _pending_cases():
    with open(os.path.join(ROOT, "tests", "golden", "pending.json")) as f:
        return json.load(f)["cases"]


def _sv_dict(b: bytes) -> dict:
    from oracle.ymerge import decode_sv

    return dict(decode_sv(b))


def test_validator_accepts_every_golden_update(golden):
    n = 0
    for setname in ("kat", "map", "array", "nested"):
        for c in golden[setname]:
            for u in c["updates"]:
                ok, structs_ok = crdt_amd.validate_update(bytes.fromhex(u))
                assert ok and structs_ok, c["name"]
                n += 1
    assert n > 1000


def _oracle_decodes(u: bytes):
    """True / False = the oracle decoded / refused the bytes; None = no verdict on the bytes: the
    oracle stops at missing dependencies before it reads the delete set, and "Unexpected case" is
    a semantic error raised while integrating (a byte flip that still parses), not a decode one."""
    try:
        ODoc(0x7FFFFFF0).apply_update(u)
        return True
    except OracleError as e:
        if e.code == -2 or "Unexpected case" in str(e):
            return None
        return e.code != -1  # YO_E_DECODE


def test_validator_matches_oracle_on_truncations_and_garbage(golden):
    """Every prefix of a few golden updates, plus byte flips: validator == oracle decode verdict."""
    import random

    rng = random.Random(3)
    cases = [c for s in ("kat", "map", "array", "nested") for c in golden[s]]
    checked = 0
    for c in cases[::9]:
        u = bytes.fromhex(c["updates"][0])
        if len(u) > 700:
            continue
        probes = [u[:k] for k in range(len(u))]
        for _ in range(20):
            b = bytearray(u)
            b[rng.randrange(len(b))] = rng.randrange(256)
            probes.append(bytes(b))
        for p in probes:
            want = _oracle_decodes(p)
            if want is None:
                continue
            ok, _ = crdt_amd.validate_update(p)
            assert ok == want, (c["name"], p.hex())
            checked += 1
    assert checked > 2000


def test_malformed_delete_set_keeps_structs_flag():
    a = ODoc(7)
    a.map_set("users", "k", bytes([125, 5]))
    good = a.encode_state_as_update()
    assert crdt_amd.validate_update(good) == (True, True)
    assert crdt_amd.validate_update(good[:-1]) == (False, True)  # no delete set at all
    assert crdt_amd.validate_update(good[:5]) == (False, False)
    assert crdt_amd.validate_update(b"") == (False, False)


@pytest.mark.parametrize("chunk", range(4))
def test_pending_emulation_matches_yjs(chunk):
    cases = _pending_cases()
    cases = cases[chunk::4]
    steps = 0
    for c in cases:
        ups = [bytes.fromhex(u) for u in c["updates"]]
        for k, st in enumerate(c["steps"]):
            sv, pend, pend_ds = crdt_amd.debug_replay(ups[: k + 1], merge_updates)
            assert _sv_dict(sv) == _sv_dict(bytes.fromhex(st["sv"])), (c["name"], k)
            assert bool(pend) == st["pending"], (c["name"], k)
            assert bool(pend_ds) == st["pending_ds"], (c["name"], k)
            steps += 1
    assert steps > 150
