"""GPU parity: the HIP engine (through the C ABI) against the Yjs golden fixtures and the oracle.

Every supported case must be byte-identical to Yjs 13.6-canonical encodeStateAsUpdate /
encodeStateVector (DS/SV client order normalised); inputs outside the
engine's coverage must fail loudly with YCRDT_E_UNSUPPORTED, never return wrong bytes.
"""
import pytest

crdt_amd = pytest.importorskip("crdt_amd")

pytestmark = pytest.mark.gpu


def _run(case):
    d = crdt_amd.Doc(client_id=0x7FFFFFF0)
    d.apply_updates([bytes.fromhex(u) for u in case["updates"]])
    return d


@pytest.mark.parametrize("setname", ["kat", "map"])
def test_gpu_golden_maps(golden, setname):
    ok = unsupported = 0
    for c in golden[setname]:
        try:
            d = _run(c)
        except crdt_amd.YcrdtError as e:
            assert e.kind == "UNSUPPORTED", (c["name"], str(e))
            unsupported += 1
            continue
        assert d.encode_state_as_update().hex() == c["state"], c["name"]
        assert d.encode_state_vector().hex() == c["sv"], c["name"]
        for df in c["diffs"]:
            assert d.encode_state_as_update(bytes.fromhex(df["sv"])).hex() == df["update"], (c["name"], df["sv"])
        ok += 1
    assert ok > 0
    if setname == "map":
        assert unsupported == 0


@pytest.mark.parametrize("setname", ["array", "nested"])
def test_gpu_unsupported_fails_loudly(golden, setname):
    for c in golden[setname][:6]:
        try:
            d = _run(c)
        except crdt_amd.YcrdtError as e:
            assert e.kind == "UNSUPPORTED", (c["name"], str(e))
            continue
        # a case without arrays/nested types in its inputs must still be exact
        assert d.encode_state_as_update().hex() == c["state"], c["name"]
