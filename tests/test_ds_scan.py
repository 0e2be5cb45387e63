"""Y.applyUpdate's host check of a delete set (yc_ingest.cpp scan_update: check_ds skips varuints
eight bytes a load) against a byte-at-a-time restatement of lib0 readVarUint as the engine reads it
(yc_parse.h rd_vu: up to six bytes, a sixth continuation byte is an error) — random delete sets,
cut short, with overlong and six-byte varuints at every offset. No GPU."""
import random

import pytest

crdt_amd = pytest.importorskip("crdt_amd")


def _vu(n: int) -> bytes:
    out = bytearray()
    while n > 127:
        out.append(0x80 | (n & 0x7F))
        n >>= 7
    out.append(n)
    return bytes(out)


def _rd_vu(b: bytes, p: int):
    shift = 0
    while True:
        if p >= len(b):
            return None
        r = b[p]
        p += 1
        shift += 7
        if r < 0x80:
            return p
        if shift > 35:
            return None


def _ds_valid(b: bytes, p: int) -> bool:
    """readDeleteSet over b[p:] (the counts' values matter; the ranges' only their bytes)."""
    def val(q):
        v, shift = 0, 0
        while True:
            r = b[q]
            if shift < 32:
                v |= (r & 0x7F) << shift
            v &= 0xFFFFFFFF
            shift += 7
            q += 1
            if r < 0x80:
                return v
    q = _rd_vu(b, p)
    if q is None:
        return False
    nd = val(p)
    for _ in range(nd):
        q2 = _rd_vu(b, q)
        if q2 is None:
            return False
        q3 = _rd_vu(b, q2)
        if q3 is None:
            return False
        nr = val(q2)
        q = q3
        for _ in range(2 * nr):
            q = _rd_vu(b, q)
            if q is None:
                return False
    return True


def _odd_vu(rng, n: int) -> bytes:
    """n in a form lib0 still reads: overlong (continuation bytes of zeros) up to six bytes."""
    b = bytearray(_vu(n))
    extra = rng.choice([0, 0, 0, 1, 2, 3, 4])
    while extra and len(b) < 6:
        b[-1] |= 0x80
        b.append(0)
        extra -= 1
    return bytes(b)


def _ds(rng) -> bytes:
    nd = rng.randint(0, 6)
    out = bytearray(_vu(nd))
    for _ in range(nd):
        out += _vu(rng.randint(0, 1 << 32 - 1))
        nr = rng.randint(0, 40)
        out += _vu(nr)
        for _ in range(2 * nr):
            out += _odd_vu(rng, rng.choice([rng.randint(0, 127), rng.randint(0, 1 << 20), rng.randint(0, (1 << 32) - 1)]))
    return bytes(out)


def test_delete_set_check_matches_byte_reader():
    rng = random.Random(20261018)
    seen = {True: 0, False: 0}
    for it in range(3000):
        ds = bytearray(_ds(rng))
        mode = it % 5
        if mode == 1 and ds:  # cut short
            ds = ds[: rng.randint(0, len(ds) - 1)]
        elif mode == 2 and ds:  # a run of continuation bytes somewhere
            at = rng.randint(0, len(ds) - 1)
            k = rng.randint(1, 9)
            ds[at:at] = bytes([0x80 | rng.randint(0, 127) for _ in range(k)])
        elif mode == 3 and ds:  # random byte flips
            for _ in range(rng.randint(1, 4)):
                ds[rng.randint(0, len(ds) - 1)] ^= 1 << rng.randint(0, 7)
        elif mode == 4:  # trailing garbage is ignored by readDeleteSet
            ds += bytes(rng.randint(0, 255) for _ in range(rng.randint(1, 12)))
        u = b"\x00" + bytes(ds)
        want = _ds_valid(u, 1)
        got, structs_ok = crdt_amd.validate_update(u)
        assert structs_ok and got == want, (it, mode, bytes(ds).hex())
        seen[want] += 1
    assert seen[True] > 500 and seen[False] > 500, seen


def test_delete_set_check_six_byte_boundaries():
    """A six-byte varuint ends valid; a seventh byte is an error — at every alignment of an 8-byte
    word, after runs of continuation bytes carried across word boundaries."""
    for pad in range(0, 17):
        for body_len in (5, 6, 7):
            lead = b"\x01" * pad  # pad one-byte ranges (pad even: whole ranges)
            nr = (pad + 2) // 2 + 2
            vals = lead + b"\x80" * (body_len - 1) + b"\x00"
            vals += b"\x01" * (2 * nr - pad - 1)
            u = b"\x00" + _vu(1) + _vu(7) + _vu(nr) + vals
            want = _ds_valid(u, 1)
            assert want == (body_len <= 6)
            assert crdt_amd.validate_update(u) == (want, True), (pad, body_len)
