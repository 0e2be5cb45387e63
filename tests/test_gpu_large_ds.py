"""Large delete sets (yc_decode.hip k_dsp_*: decoded grid-wide; yc_merge.hip: applied over the
extra workgroups of k_units past DSA_WAVE ranges) against the CPU oracle and the wavefront decoder.

A delete set is a flat varuint stream (readDeleteSet, Y@11105); one of at least DSP_MIN bytes in a
large update — a full state sent as one update, crdt.js:288,443 — is decoded by terminal-byte
counts, a scan, a per-value decode and a walk over the client blocks. Every case is merged with
the grid path on (the default; its client headers found by parallel 32-header jumps, and with
YCRDT_DS_JUMP=0 by the lane-serial walk) and off (YCRDT_DS_GRID=0: the wavefront per update) and must give
the oracle's bytes; corrupted and truncated delete sets must be refused (or accepted) exactly as
the wavefront does, which tests/test_gpu_corrupt.py pins against Yjs.
"""
import random

import pytest

crdt_amd = pytest.importorskip("crdt_amd")
from oracle.yref import Doc as ODoc  # noqa: E402
from tests.histories import any_int  # noqa: E402

pytestmark = pytest.mark.gpu


def _holes(client, n, step, seed, root="messages"):
    """One client's array of n items with every step-th item deleted: n / step ranges, one block."""
    d = ODoc(client)
    d.array_insert(root, 0, [any_int(i % 1000) for i in range(n)])
    rng = random.Random(seed)
    i = n - 1 - rng.randrange(step)
    while i >= 0:
        d.array_delete(root, i, 1)
        i -= step
    return d


def _state_many(n_clients, n, step, seed):
    """A doc with many clients' arrays, each with holes: one client block per client."""
    full = ODoc(1)
    for c in range(n_clients):
        full.apply_update(_holes(1000 + 7 * c, n, step, seed + c, root=f"m{c % 3}").encode_state_as_update())
    return full.encode_state_as_update()


def _run(batch, monkeypatch, grid):
    # grid True: the grid path with its parallel header jumps (k_dsh_*), "hop": the grid path with
    # the lane-serial header walk (YCRDT_DS_JUMP=0), False: the wavefront per update
    monkeypatch.setenv("YCRDT_DS_GRID", "1" if grid else "0")
    monkeypatch.setenv("YCRDT_DS_JUMP", "0" if grid == "hop" else "1")
    d = crdt_amd.Doc(client_id=0x7FFFFFF0)
    try:
        d.apply_updates(batch)
        err = None
    except crdt_amd.YcrdtError as e:
        err = type(e).__name__
    return err, d.encode_state_as_update(), d.encode_state_vector()


def _check(batch, monkeypatch):
    ref = ODoc(0x7FFFFFF0)
    for u in batch:
        ref.apply_update(u)
    want = (None, ref.encode_state_as_update(), ref.encode_state_vector())
    assert _run(batch, monkeypatch, True) == want
    assert _run(batch, monkeypatch, "hop") == want
    assert _run(batch, monkeypatch, False) == want


@pytest.mark.parametrize("n,step", [(30_000, 2), (20_000, 3), (9000, 2)])
def test_one_client_many_ranges(n, step, monkeypatch):
    """One client block of 4 500 - 15 000 ranges (past DSA_WAVE: the spread apply)."""
    u = _holes(77, n, step, n).encode_state_as_update()
    _check([u], monkeypatch)
    other = ODoc(5)
    other.map_set("users", "a", any_int(1))
    _check([other.encode_state_as_update(), u], monkeypatch)


@pytest.mark.parametrize("n_clients,n,step", [(300, 60, 2), (40, 2000, 3), (1200, 12, 4)])
def test_many_client_blocks(n_clients, n, step, monkeypatch):
    snap = _state_many(n_clients, n, step, n_clients)
    _check([snap], monkeypatch)


def test_state_with_half_applied(monkeypatch):
    """A full state applied to a doc that already holds part of it (the sync step-2 shape)."""
    full = _state_many(200, 100, 2, 9)
    part = _state_many(100, 100, 2, 9)
    _check([part, full], monkeypatch)
    _check([full, part], monkeypatch)




def test_corrupted_and_truncated_delete_sets_like_the_wavefront(monkeypatch):
    """Overlong varuints, huge range counts and cuts inside a large delete set: the grid path must
    answer exactly as the wavefront (which test_gpu_corrupt.py pins against Yjs)."""
    u = bytearray(_holes(77, 12_000, 2, 3).encode_state_as_update())
    rng = random.Random(4)
    cases = []
    n = len(u)
    for cut in (n - 1, n - 2, n - 5, n - 400, n - 3000):
        cases.append(bytes(u[:cut]))
    for _ in range(24):
        v = bytearray(u)
        at = n - 1 - rng.randrange(4000)
        v[at] = rng.choice([0x80, 0xFF, 0x00, 0x7F, v[at] ^ 0x80])
        cases.append(bytes(v))
    v = bytearray(u)
    v[n - 200:n - 192] = b"\x80" * 8  # a varuint of more than 6 bytes
    cases.append(bytes(v))
    for c in cases:
        w = _run([c], monkeypatch, False)
        assert _run([c], monkeypatch, True) == w
        assert _run([c], monkeypatch, "hop") == w


def test_million_item_full_state_as_one_update(monkeypatch):
    """A >= 1 M-item C3 state (256 clients) applied as ONE update — crdt.js's full-state wire shape —
    against the oracle applying the same bytes: the multi-section fast walk, the grid delete set and
    the spread range apply at scale."""
    from crdt_amd.workload import gen_array

    ups, _ = gen_array(256, 16, 1_010_000, 7)
    b = crdt_amd.Batch(ups)
    st = b.merge()
    full = b.result()[0]
    del b
    assert st.items >= 1_000_000
    ref = ODoc(0x7FFFFFF0)
    ref.apply_update(full)
    want = ref.encode_state_as_update()
    assert want == full  # (the merged state is canonical)
    for grid in (True, False):
        err, got, sv = _run([full], monkeypatch, grid)
        assert err is None and got == want and sv == ref.encode_state_vector()
