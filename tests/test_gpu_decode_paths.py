"""Every decode path for small updates gives the same bytes.

Small updates (<= 16 KiB) are parsed one lane per update (k_direct) when there are many, one
workgroup per update when there are few (k_wlen steps every position, k_wrank ranks each section's
chain by pointer doubling; or, YCRDT_WDECODE=settle, k_wdecode: chunk chains per lane settled
inside a wavefront); large ones take the chunk path (k_spec / k_sync / k_walk). The modes force
one: "direct" = k_direct, "wave" = k_wlen + k_wrank, "settle" = k_wdecode, "chunks" = the chunk path.
All must match the Yjs fixtures and the oracle byte for byte, and report the same malformed input.
"""
import pytest

crdt_amd = pytest.importorskip("crdt_amd")

pytestmark = pytest.mark.gpu
MODES = ("chunks", "direct", "wave", "settle")


def _mode(monkeypatch, mode):
    # wave: few small updates ranked (k_wlen + k_wrank); settle: k_wdecode's settled chains
    wave = mode in ("wave", "settle")
    monkeypatch.setenv("YCRDT_DECODE", "chunks" if mode == "chunks" else "direct")
    if mode != "chunks":
        monkeypatch.setenv("YCRDT_DIRECT_WAVE", "1" if wave else "0")
    monkeypatch.setenv("YCRDT_WDECODE", "settle" if mode == "settle" else "rank")


@pytest.mark.parametrize("mode", MODES)
def test_paths_golden(golden, mode, monkeypatch):
    _mode(monkeypatch, mode)
    for setname in ("kat", "map", "array", "nested"):
        for c in golden[setname]:
            d = crdt_amd.Doc(client_id=0x7FFFFFF0)
            d.apply_updates([bytes.fromhex(u) for u in c["updates"]])
            assert d.encode_state_as_update().hex() == c["state"], (mode, c["name"])
            assert d.encode_state_vector().hex() == c["sv"], (mode, c["name"])
            ups = [bytes.fromhex(u) for u in c["updates"]]
            want = c["merged"] if len(ups) > 1 else c["merged_raw"]
            assert crdt_amd.merge_updates(ups).hex() == want, (mode, c["name"])


@pytest.mark.parametrize("mode", MODES)
def test_paths_generated_vs_oracle(mode, monkeypatch):
    from crdt_amd.workload import C2, gen_map
    from oracle.yref import Doc as ODoc

    _mode(monkeypatch, mode)
    cfg = dict(C2)
    cfg.update(n_keys=2000, n_replicas=300, ops_per_replica=200)
    ups, _ = gen_map(**cfg)
    o = ODoc(0x7FFFFFF0)
    for u in ups:
        o.apply_update(u)
    b = crdt_amd.Batch(ups)
    b.merge()
    assert b.result() == (o.encode_state_as_update(), o.encode_state_vector())


@pytest.mark.parametrize("mode", MODES)
def test_paths_array_vs_oracle(mode, monkeypatch):
    from tests.histories import array_history
    from oracle.yref import Doc as ODoc

    _mode(monkeypatch, mode)
    states, wire = array_history(77, n_replicas=6, rounds=4, ops=10, with_map=True)
    ups = states + wire
    o = ODoc(0x7FFFFFF0)
    for u in ups:
        o.apply_update(u)
    b = crdt_amd.Batch(ups)
    b.merge()
    assert b.result() == (o.encode_state_as_update(), o.encode_state_vector())


@pytest.mark.parametrize("mode", MODES)
def test_paths_malformed(golden, mode, monkeypatch):
    """A truncated update in a batch fails the merge on both paths (Yjs throws on it)."""
    _mode(monkeypatch, mode)
    good = [bytes.fromhex(u) for u in golden["map"][0]["updates"]]
    bad = good[0][: max(3, len(good[0]) // 2)]
    b = crdt_amd.Batch(good + [bad])
    with pytest.raises(crdt_amd.YcrdtError):
        b.merge()
