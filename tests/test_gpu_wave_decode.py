"""Adversarial inputs for the wave decoder (yc_decode.hip k_wdecode), against the CPU oracle.

A few small updates (<= 16 KiB) are parsed one wavefront each: lane 0 walks the first 1/64 of the
update exactly, every other lane follows the all-struct chain of its 1/64 from a hinted start, and
the lanes settle inside the wavefront (lowest-lane overwrite; lanes past the n-th chain position
leave the settling; a lane whose entry changed since its walk blocks that exclusion for the lanes
after it — the race fixed in eb51886). These cases aim at the settling rules: string values that
are themselves valid struct encodings (chains beside the true one), periodic struct streams (chains
locked in a wrong phase), delete sets that parse as long struct chains, truncated and corrupted
updates (test_gpu_corrupt.py, against Yjs's own results in every decode mode), and a seeded fuzz of mixed shapes. YCRDT_DEBUG_DECODE=1 makes the engine report the wave decoder's
work, so every case checks that k_wdecode really took the update.
"""
import random
import re

import pytest

crdt_amd = pytest.importorskip("crdt_amd")
from oracle.yref import Doc as ODoc  # noqa: E402
from tests.histories import any_int  # noqa: E402
from tests.test_gpu_edges import _merge_both, _same, any_str  # noqa: E402

pytestmark = pytest.mark.gpu
WAVE_MAX = 16384  # DIRECT_MAX_BYTES: larger updates take the chunk path


@pytest.fixture(params=["rank", "settle"])
def wave(monkeypatch, request):
    """Few small updates: ranked (k_wlen + k_wrank, the default) or k_wdecode's settled chains."""
    monkeypatch.setenv("YCRDT_DECODE", "direct")
    monkeypatch.setenv("YCRDT_DIRECT_WAVE", "1")
    monkeypatch.setenv("YCRDT_WDECODE", request.param)
    monkeypatch.setenv("YCRDT_DEBUG_DECODE", "1")
    yield


def _wave_count(err_text):
    """Updates the wave decoder handled, from the engine's debug lines."""
    n = 0
    for m in re.finditer(r"wave: done (\d+) unsettled (\d+) other (\d+)", err_text):
        n += sum(int(x) for x in m.groups())
    return n


def _snapshot(n_clients, per_client, seed, value=None, arrays=True):
    rng = random.Random(seed)
    full = ODoc(1)
    for c in range(n_clients):
        d = ODoc(100 + 13 * c)
        if c % 3 == 1:
            d.apply_update(full.encode_state_as_update())
        for _ in range(per_client):
            k = rng.randrange(3 * per_client)
            v = value(rng) if value else any_int(rng.randrange(1000))
            if not arrays or rng.random() < 0.7:
                d.map_set("users", f"k{k}", v)
            else:
                d.array_insert("messages", 0, [v])
        full.apply_update(d.encode_state_as_update())
    return full.encode_state_as_update()


def _check(batch, capfd):
    assert all(len(u) <= WAVE_MAX for u in batch)
    capfd.readouterr()
    d, ref = _merge_both(batch)
    _same(d, ref)
    assert _wave_count(capfd.readouterr().err) > 0


def test_wave_struct_encodings_inside_strings(wave, capfd):
    inner = _snapshot(3, 6, 5)[4:]  # struct bytes of a small update, repeated inside the values
    vals = [inner * k for k in (1, 2, 4)]
    for seed in range(12):
        snap = _snapshot(4, 3, 100 + seed, value=lambda rng: any_str(vals[rng.randrange(3)].decode("latin-1")))
        if len(snap) > WAVE_MAX:
            snap = _snapshot(2, 3, 100 + seed, value=lambda rng: any_str(vals[rng.randrange(2)].decode("latin-1")))
        _check([snap], capfd)
        # beside another update of the same doc (two wavefronts, one merge)
        extra = ODoc(9)
        extra.map_set("users", "k1", any_int(seed))
        _check([snap, extra.encode_state_as_update()], capfd)


def _periodic(n, seed, width=6):
    d = ODoc(7)
    for k in range(n):
        d.map_set("users", f"k{k:0{width}d}", any_int(1000 + (k * 7919 + seed) % 9000))
    return d.encode_state_as_update()


@pytest.mark.parametrize("n", [60, 200, 500, 780])
def test_wave_periodic_streams(wave, capfd, n):
    """Identical struct shapes back to back: every lane's chain can lock into a wrong phase."""
    for seed in range(3):
        u = _periodic(n, seed)
        assert len(u) <= WAVE_MAX
        _check([u], capfd)


def test_wave_lds_sized_to_longest(wave, capfd):
    """k_wrank's LDS is sized to the batch's longest small update (Work::small_max): an update at
    the 16 KiB limit (100 KB of LDS) beside tiny ones, tiny ones alone, and a mid-size one."""
    n = 812
    while len(_periodic(n, 1)) > WAVE_MAX:
        n -= 1
    big = _periodic(n, 1)
    assert len(big) > WAVE_MAX - 64
    tiny = [_periodic(k, 2 + k) for k in (1, 3, 9)]
    _check(tiny + [big], capfd)
    _check([big] + tiny, capfd)
    _check(tiny, capfd)
    _check([_periodic(300, 5)] + tiny, capfd)


def test_wave_long_delete_sets(wave, capfd):
    """An update whose delete set is most of its bytes: many (clock, len) ranges of many clients,
    byte patterns the lanes' chains parse as struct runs."""
    rng = random.Random(3)
    base = ODoc(1)
    for k in range(400):
        base.array_insert("messages", k, [any_int(k % 60)])
    for c in range(30):
        d = ODoc(50 + c)
        for k in range(8):
            d.map_set("users", f"k{c}_{k}", any_int(k))
        base.apply_update(d.encode_state_as_update())
    b = base.encode_state_as_update()
    dels = ODoc(2)
    dels.apply_update(b)
    for _ in range(150):  # scattered single deletes: one range each
        dels.array_delete("messages", rng.randrange(200), 1)
    for c in range(30):
        for k in range(0, 8, 2):
            dels.map_delete("users", f"k{c}_{k}")
    sv = base.encode_state_vector()
    delta = dels.encode_state_as_update(sv)
    assert len(delta) <= WAVE_MAX
    _check([b, delta], capfd)
    # applied one at a time (the delta merges behind the doc's state)
    d = crdt_amd.Doc(client_id=0x7FFFFFF0)
    d.apply_update(b)
    capfd.readouterr()
    d.apply_update(delta)
    ref = ODoc(0x7FFFFFF0)
    ref.apply_update(b)
    ref.apply_update(delta)
    _same(d, ref)
    assert _wave_count(capfd.readouterr().err) > 0


# truncated and corrupted updates in wave mode: tests/test_gpu_corrupt.py (Yjs's own results)


def test_wave_fuzz_mixed_shapes(wave, capfd):
    """Seeded histories of mixed shapes (map sets with short / long / struct-like string values,
    array pushes and inserts, deletes) cut into one small update per replica, merged a few at a
    time: the lanes' settling sees a new layout in every update. Regression net for the settling
    races (eb51886)."""
    inner = _snapshot(2, 4, 9, arrays=False)[4:]
    total = 0
    for seed in range(40):
        rng = random.Random(seed)

        def val(r):
            x = r.random()
            if x < 0.4:
                return any_int(r.randrange(5000))
            if x < 0.7:
                return any_str("v" * r.randrange(1, 300))
            return any_str((inner * r.randrange(1, 3)).decode("latin-1"))

        base = ODoc(1)
        for k in range(rng.randrange(5, 60)):
            base.map_set("users", f"k{k}", val(rng))
        b = base.encode_state_as_update()
        ups = [b]
        for r in range(rng.randrange(2, 6)):
            d = ODoc(1000 + 17 * r + seed)
            d.apply_update(b)
            for _ in range(rng.randrange(1, 40)):
                x = rng.random()
                if x < 0.5:
                    d.map_set("users", f"k{rng.randrange(80)}", val(rng))
                elif x < 0.8:
                    d.array_insert("messages", 0, [val(rng)])
                else:
                    d.map_delete("users", f"k{rng.randrange(80)}")
            ups.append(d.encode_state_as_update(base.encode_state_vector()))
        ups = [u for u in ups if len(u) <= WAVE_MAX]
        _check(ups, capfd)
        total += len(ups)
    assert total > 100


def _vs(s):
    b = s.encode()
    return bytes([len(b)]) + b


def _rare_kinds_update(reps):
    """One section of client 5: runs of Format / String / Embed / JSON / Binary items (the content
    kinds k_wlen leaves unsized until a chain reaches one) behind a common Any item, reps times."""
    out, clock, prev = [], 0, None

    def item(ref, content, length):
        nonlocal clock, prev
        if prev is None:
            s = bytes([ref]) + b"\x01" + _vs("t") + content  # under the root type "t"
        else:
            s = bytes([0x80 | ref, 5, prev]) + content         # origin: (5, prev)
        out.append(s)
        clock += length
        prev = clock - 1

    for r in range(reps):
        item(8, b"\x01\x7d" + bytes([r % 60]), 1)            # Any: one varInt
        item(6, _vs("bold") + _vs("true"), 1)                # Format
        item(4, _vs("hello"), 5)                             # String
        item(5, _vs('{"x":1}'), 1)                           # Embed
        item(2, b"\x01" + _vs('"j"'), 1)                     # JSON, one value
        item(3, b"\x03abc", 1)                               # Binary
    assert clock < 128  # (one-byte clocks above)
    return bytes([1, len(out), 5, 0]) + b"".join(out) + b"\x00"


def test_wave_rare_content_kinds(wave, capfd):
    """Rare content kinds on the chain: the ranked path sizes the positions it skipped, ranks again."""
    for reps in (1, 3, 8):
        _check([_rare_kinds_update(reps)], capfd)
        extra = ODoc(9)
        extra.map_set("users", "k1", any_int(reps))
        _check([_rare_kinds_update(reps), extra.encode_state_as_update()], capfd)
