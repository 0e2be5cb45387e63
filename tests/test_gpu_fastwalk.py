"""The fast walks of large updates (yc_decode.hip k_fastwalk / k_fastwalk_multi) against k_walk.

A large update (> 16 KiB) is decoded by per-chunk struct chains; once the synced chains form one
chain up to the chunk holding a section's last struct (k_chunk_counts records the first chunk whose
entry may be off it), the fast walks take the struct positions from the chains and skip the serial
walk. Every case here is decoded twice — fast walks on (the default) and off (YCRDT_NO_FASTWALK=1:
k_walk alone) — and the merged state and state vector must be byte-identical to each other and to
the CPU oracle. The shapes aim at the place the fast walks trust: where the last struct ends
relative to the chunk grid (a delete set starting just before, at or just after a chunk boundary;
its garbage chain jumping or moving the exit of the last struct's chunk), several sections, and a
snapshot of many clients (the multi-section walk, which must then really take the update:
YCRDT_DEBUG_DECODE=1 reports it).
"""
import random
import re

import pytest

crdt_amd = pytest.importorskip("crdt_amd")
from oracle.yref import Doc as ODoc  # noqa: E402
from tests.histories import any_int, any_str  # noqa: E402

pytestmark = pytest.mark.gpu
CHUNK = 1024


def _merge(batch, monkeypatch, capfd, fast, fwc="1"):
    monkeypatch.setenv("YCRDT_DECODE", "chunks")
    monkeypatch.setenv("YCRDT_DEBUG_DECODE", "1")
    monkeypatch.setenv("YCRDT_FWC", fwc)  # record mode: "force" takes every multi-section large update
    if fast:
        monkeypatch.delenv("YCRDT_NO_FASTWALK", raising=False)
    else:
        monkeypatch.setenv("YCRDT_NO_FASTWALK", "1")
    capfd.readouterr()
    d = crdt_amd.Doc(client_id=0x7FFFFFF0)
    d.apply_updates(batch)
    out = (d.encode_state_as_update(), d.encode_state_vector())
    err = capfd.readouterr().err
    done = sum(int(m.group(1)) for m in re.finditer(r"fastwalk: done (\d+)", err))
    print(err)
    return out, done


def _check(batch, monkeypatch, capfd):
    ref = ODoc(0x7FFFFFF0)
    for u in batch:
        ref.apply_update(u)
    want = (ref.encode_state_as_update(), ref.encode_state_vector())
    fast, n_fast = _merge(batch, monkeypatch, capfd, True)
    rec, n_rec = _merge(batch, monkeypatch, capfd, True, fwc="force")
    slow, n_slow = _merge(batch, monkeypatch, capfd, False)
    assert slow == want
    assert fast == want
    assert rec == want
    assert n_slow == 0
    return n_fast + n_rec


def _replica(client, n_sets, n_keys, seed, value_len=3):
    """One client's update: n_sets map sets over n_keys keys (overwrites delete its own earlier
    entries: the update's delete set grows with n_sets - n_keys)."""
    rng = random.Random(seed)
    d = ODoc(client)
    for i in range(n_sets):
        k = rng.randrange(n_keys)
        d.map_set("users", f"k{k}", any_str("v" * value_len) if i % 3 else any_int(i))
    return d.encode_state_as_update()


def test_single_section_last_struct_around_chunk_edges(monkeypatch, capfd):
    """Single-section updates whose struct section ends at every offset class around a chunk
    boundary, followed by delete sets of different lengths (garbage chains past the structs)."""
    took = 0
    for n_sets in (2400, 2440, 2480, 2520, 2560, 2600, 2640, 2680):
        for n_keys in (n_sets, n_sets // 2, n_sets // 8):
            u = _replica(77 + n_sets, n_sets, n_keys, n_sets * 7 + n_keys)
            assert len(u) > 16384
            took += _check([u], monkeypatch, capfd)
    assert took > 0


def test_value_length_sweep_moves_the_struct_end(monkeypatch, capfd):
    """The same op script with value lengths 1..24: the struct section's end walks through every
    byte offset of a chunk."""
    for vl in range(1, 25):
        u = _replica(1000 + vl, 2400, 300, 99, value_len=vl)
        _check([u], monkeypatch, capfd)


def _snapshot(n_clients, per_client, seed, arrays=True):
    rng = random.Random(seed)
    full = ODoc(1)
    for c in range(n_clients):
        d = ODoc(100 + 13 * c)
        if c % 7 == 3:
            d.apply_update(full.encode_state_as_update())
        for _ in range(per_client):
            k = rng.randrange(2 * per_client)
            if not arrays or rng.random() < 0.7:
                d.map_set("users", f"k{k}", any_int(rng.randrange(1 << 20)))
            else:
                d.array_insert("messages", 0, [any_int(rng.randrange(1000))])
        full.apply_update(d.encode_state_as_update())
    return full.encode_state_as_update()


@pytest.mark.parametrize("n_clients,per_client", [(64, 60), (256, 12), (20, 300), (600, 4)])
def test_multi_section_snapshots(n_clients, per_client, monkeypatch, capfd):
    """Snapshots of many clients (the wire shape of crdt.js's full-state messages): the
    multi-section fast walk must give k_walk's answer — and take some of them."""
    snap = _snapshot(n_clients, per_client, n_clients * 31 + per_client)
    assert len(snap) > 16384
    _check([snap], monkeypatch, capfd)
    extra = ODoc(9)
    extra.map_set("users", "k1", any_int(5))
    _check([snap, extra.encode_state_as_update()], monkeypatch, capfd)


def test_multi_section_walk_is_taken(monkeypatch, capfd):
    """A map-only snapshot of 40 clients (no array values: no long garbage chains through
    contents): the multi-section fast walk takes it (round 4 shadowed its chunk bound, so it never
    did)."""
    snap = _snapshot(40, 200, 5, arrays=False)
    assert len(snap) > 16384
    assert _check([snap], monkeypatch, capfd) >= 1


@pytest.mark.parametrize("fwm_max", [1, 2, 7])
@pytest.mark.parametrize("n_clients,per_client,arrays", [(40, 200, False), (64, 60, True), (600, 4, True)])
def test_multi_section_walk_resumes(fwm_max, n_clients, per_client, arrays, monkeypatch, capfd):
    """k_fastwalk_multi vouches for a prefix of the sections and k_walk resumes at the next header
    (YCRDT_FWM_MAX caps the prefix: the resume path on every snapshot here); the state must be
    k_walk's alone and the oracle's."""
    snap = _snapshot(n_clients, per_client, n_clients * 17 + per_client + fwm_max, arrays=arrays)
    assert len(snap) > 16384
    monkeypatch.setenv("YCRDT_FWM_MAX", str(fwm_max))
    _check([snap], monkeypatch, capfd)
    extra = ODoc(9)
    extra.map_set("users", "k2", any_int(6))
    _check([extra.encode_state_as_update(), snap], monkeypatch, capfd)


def test_document_state_as_one_update_record_mode(monkeypatch, capfd):
    """A C2-shaped document's merged state (hundreds of client sections, > 64 KiB) applied as ONE
    update — crdt.js's full-state message — takes the record mode by default (k_fwc evaluates the
    section step at every chain position; the walker follows the records): equal to the oracle,
    to record mode off and to k_walk alone, and really taken."""
    from crdt_amd.workload import C2, gen_map

    cfg = dict(C2)
    cfg.update(n_keys=2000, n_replicas=300, ops_per_replica=200)
    ups, _ = gen_map(**cfg)
    o = ODoc(0x7FFFFFF0)
    for u in ups:
        o.apply_update(u)
    state = o.encode_state_as_update()
    assert len(state) > 64 * 1024
    want = (state, o.encode_state_vector())
    outs = {}
    for fwc in ("1", "0"):
        outs[fwc] = _merge([state], monkeypatch, capfd, True, fwc=fwc)
    slow, n_slow = _merge([state], monkeypatch, capfd, False)
    assert outs["1"][0] == want and outs["0"][0] == want and slow == want
    assert outs["1"][1] >= 0 and n_slow == 0  # (the base section may be left to the table walk)
    # into a doc holding part of it (a device-resident state beside the update)
    half = ODoc(0x7FFFFFF0)
    for u in ups[: len(ups) // 2]:
        half.apply_update(u)
    for fwc in ("1", "0"):
        monkeypatch.setenv("YCRDT_FWC", fwc)
        d = crdt_amd.Doc(client_id=0x7FFFFFF0)
        d.apply_update(half.encode_state_as_update())
        d.encode_state_vector()
        d.apply_update(state)
        assert (d.encode_state_as_update(), d.encode_state_vector()) == want


@pytest.mark.parametrize("rank", ("1", "0"))
def test_last_section_ranked(rank, monkeypatch, capfd):
    """Record mode stops before the last section (YCRDT_FWM_MAX = sections - 1, the place a
    phase-locked snapshot section stops it); the last section is then ranked by pointer doubling over
    the step table (YCRDT_RANK_LAST=0: k_walk resumes instead). Equal to the oracle either way, and
    the ranked path really taken."""
    from crdt_amd.workload import C2, gen_map

    cfg = dict(C2)
    cfg.update(n_keys=4000, n_replicas=120, ops_per_replica=150)
    ups, _ = gen_map(**cfg)
    o = ODoc(0x7FFFFFF0)
    for u in ups:
        o.apply_update(u)
    state = o.encode_state_as_update()
    nsec, k = 0, 0
    while True:  # the section count (first varuint)
        nsec |= (state[k] & 0x7F) << (7 * k)
        if state[k] < 0x80:
            break
        k += 1
    monkeypatch.setenv("YCRDT_FWM_MAX", str(nsec - 1))
    monkeypatch.setenv("YCRDT_RANK_LAST", rank)
    got, done = _merge([state], monkeypatch, capfd, True, fwc="force")
    assert got == (state, o.encode_state_vector())
    assert done >= (1 if rank == "1" else 0)
    other = ODoc(9)
    other.map_set("users", "k7", any_int(70))
    batch = [other.encode_state_as_update(), state]
    ref = ODoc(0x7FFFFFF0)
    for u in batch:
        ref.apply_update(u)
    got, _ = _merge(batch, monkeypatch, capfd, True, fwc="force")
    assert got == (ref.encode_state_as_update(), ref.encode_state_vector())
