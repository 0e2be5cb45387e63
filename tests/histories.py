"""Seeded random replica histories built with the CPU oracle (test infrastructure).

Replicas edit a YArray (push / unshift / insert / delete ranges) and optionally a YMap, exchange
state-vector deltas in partial gossip rounds, and every replica's final state (plus the deltas on
the wire) becomes the batch the GPU engine must merge exactly like sequential Y.applyUpdate."""
import random

from oracle.yref import Doc


def any_int(v):
    """lib0 writeAny of a small integer: tag 125 + varInt (L0@8251)."""
    out = [125]
    neg = v < 0
    v = abs(v)
    out.append((0x40 if neg else 0) | (v & 0x3F) | (0x80 if v > 0x3F else 0))
    v >>= 6
    while v:
        out.append((v & 0x7F) | (0x80 if v > 0x7F else 0))
        v >>= 7
    return bytes(out)


def any_str(s):
    b = s.encode()
    assert len(b) < 128
    return bytes([119, len(b)]) + b


def array_history(seed, n_replicas=4, rounds=4, ops=6, with_map=False, clients=None):
    rng = random.Random(seed)
    ids = clients or [rng.randrange(1, 2**31) for _ in range(n_replicas)]
    docs = [Doc(c) for c in ids]
    lens = [0] * n_replicas
    wire = []
    for _ in range(rounds):
        for r, d in enumerate(docs):
            for _ in range(ops):
                x = rng.random()
                n = lens[r]
                vals = [any_int(rng.randrange(-100, 100000)) if rng.random() < 0.6 else any_str("s%d" % rng.randrange(1000))
                        for _ in range(rng.randint(1, 3))]
                if x < 0.35 or n == 0:
                    d.array_insert("messages", n, vals)
                elif x < 0.5:
                    d.array_insert("messages", 0, vals)
                elif x < 0.75:
                    d.array_insert("messages", rng.randrange(n + 1), vals)
                elif with_map and x < 0.85:
                    d.map_set("users", "k%d" % rng.randrange(5), vals[0])
                else:
                    i = rng.randrange(n)
                    d.array_delete("messages", i, min(n - i, rng.randint(1, 3)))
                lens[r] = _len(d)
        # gossip: every replica pulls a delta from one random peer
        for r, d in enumerate(docs):
            p = rng.randrange(n_replicas)
            if p == r:
                continue
            delta = docs[p].encode_state_as_update(d.encode_state_vector())
            wire.append(delta)
            d.apply_update(delta)
            lens[r] = _len(d)
    states = [d.encode_state_as_update() for d in docs]
    return states, wire


def _len(d):
    import json

    return len(json.loads(d.root_json("messages", "array")))
