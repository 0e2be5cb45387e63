"""Yjs v1 helpers for tests: canonical (13.6) client order of delete sets / state vectors.
Mirrors tests/golden/gen/v1.js canonicalUpdate / canonicalSv."""
from oracle.ymerge import Dec, lazy_structs, wvu


def _skip_structs(d):
    lazy_structs(d)


def canonical_update(u):
    d = Dec(bytes(u))
    _skip_structs(d)
    end = d.p
    ds = []
    for _ in range(d.vu()):
        client = d.vu()
        ranges = [(d.vu(), d.vu()) for _ in range(d.vu())]
        ds.append((client, ranges))
    if d.p != len(u):
        raise ValueError("trailing bytes")
    ds.sort(key=lambda e: -e[0])
    out = bytearray(u[:end])
    wvu(out, len(ds))
    for client, ranges in ds:
        wvu(out, client)
        wvu(out, len(ranges))
        for c, n in ranges:
            wvu(out, c)
            wvu(out, n)
    return bytes(out)


def delete_set_of(u):
    """The delete set of a v1 update as {client: [(clock, len), ...]}: sorted and merged (Yjs
    sortAndMergeDeleteSet, Y@10246), so byte layouts that mean the same deletions compare equal."""
    d = Dec(bytes(u))
    _skip_structs(d)
    ds = {}
    for _ in range(d.vu()):
        client = d.vu()
        for _ in range(d.vu()):
            c, n = d.vu(), d.vu()
            if n:
                ds.setdefault(client, []).append((c, n))
    out = {}
    for client, rs in ds.items():
        rs.sort()
        m = []
        for c, n in rs:
            if m and m[-1][0] + m[-1][1] >= c:
                m[-1] = (m[-1][0], max(m[-1][0] + m[-1][1], c + n) - m[-1][0])
            else:
                m.append((c, n))
        out[client] = m
    return out
