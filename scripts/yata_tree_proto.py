"""Design check (CPU, test infrastructure): YATA as an origin-tree pre-order.

Claim (parallel YATA): in the final Yjs list, the origin-descendants of every item
form a contiguous block right after it, so the list is a pre-order walk of the origin tree in which
every node's children (items with the same origin, each carrying its block) are ordered by the
B.1 loop run over the children alone: scan siblings from the first until the
child's right origin (when that is a sibling, else to the end); left := o when o.client <
c.client, else stop when o.rightOrigin == c.rightOrigin.

This script restates both on per-clock items (SURVEY §7 hard part 1) decoded from seeded oracle
histories (tests/histories.py) and checks they agree, and counts the sequential loop's scan steps
for two causal integration orders (ascending vs descending client).

    python scripts/yata_tree_proto.py [n_histories]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle.ymerge import ITEM, Dec, lazy_structs  # noqa: E402


def units_of(updates):
    """Per-clock items grouped by list: {list key: {id: (origin id | None, right origin id | None)}}.
    A list key is the explicit (parent, parentSub) of an origin-less item, inherited along origins /
    right origins (Item.getMissing, Y@76507)."""
    units, key = {}, {}
    for u in updates:
        for s in lazy_structs(Dec(u)):
            if s.kind != ITEM:
                continue
            for i in range(s.length):
                uid = (s.client, s.clock + i)
                if uid in units:
                    continue
                o = s.origin if i == 0 else (s.client, s.clock + i - 1)
                units[uid] = (o, s.right_origin)
                if o is None and s.right_origin is None:
                    key[uid] = (bytes(s.parent) if isinstance(s.parent, bytes) else s.parent, s.parent_sub)
    pending = [u for u in units if u not in key]
    while pending:
        nxt = []
        for u in pending:
            o, r = units[u]
            src = o if o is not None else r
            if src in key:
                key[u] = key[src]
            elif src in units:
                nxt.append(u)
        if len(nxt) == len(pending):
            break
        pending = nxt
    lists = {}
    for u, v in units.items():
        lists.setdefault(key.get(u), {})[u] = v
    return lists


def seq_yata(units, descending=False):
    """The B.1 loop (Item.integrate, Y@77594) over units in a causal order (dives on O / R)."""
    right, head = {}, None
    state = {}
    steps = 0
    order = sorted(units, key=lambda x: (-x[0], x[1]) if descending else x)
    for u0 in order:
        if state.get(u0) == 2:
            continue
        stack = [u0]
        state[u0] = 1
        while stack:
            t = stack[-1]
            o_id, r_id = units[t]
            dep = None
            if o_id is not None and state.get(o_id) != 2:
                dep = o_id
            elif r_id is not None and state.get(r_id) != 2:
                dep = r_id
            if dep is not None:
                assert state.get(dep) != 1 and dep in units, "cycle / outside"
                state[dep] = 1
                stack.append(dep)
                continue
            left = o_id
            o = right.get(left) if left is not None else head
            before, confl = set(), set()
            while o is not None and o != r_id:
                steps += 1
                before.add(o)
                confl.add(o)
                oo, orr = units[o]
                if oo == o_id:
                    if o[0] < t[0]:
                        left = o
                        confl = set()
                    elif orr == r_id:
                        break
                elif oo is not None and oo in before:
                    if oo not in confl:
                        left = o
                        confl = set()
                else:
                    break
                o = right.get(o)
            if left is not None:
                r2 = right.get(left)
                right[left] = t
            else:
                r2 = head
                head = t
            right[t] = r2
            state[t] = 2
            stack.pop()
    out = []
    x = head
    while x is not None:
        out.append(x)
        x = right.get(x)
    return out, steps


def tree_yata(units):
    """Origin-tree pre-order with per-node sibling loops (children integrated in descending client
    order, diving on a sibling right origin)."""
    children = {}
    for u, (o, _) in units.items():
        children.setdefault(o, []).append(u)
    steps = 0
    ordered = {}
    for p, kids in children.items():
        kidset = set(kids)
        lst = []
        done = set()
        for c0 in sorted(kids, key=lambda x: (-x[0], x[1])):
            if c0 in done:
                continue
            stack = [c0]
            while stack:
                c = stack[-1]
                r = units[c][1]
                if r in kidset and r not in done:
                    stack.append(r)
                    continue
                left = -1
                for i, o in enumerate(lst):
                    if o == r:
                        break
                    steps += 1
                    if o[0] < c[0]:
                        left = i
                    elif units[o][1] == r:
                        break
                lst.insert(left + 1, c)
                done.add(c)
                stack.pop()
        ordered[p] = lst
    out = []
    stack = [iter(ordered.get(None, []))]
    while stack:
        x = next(stack[-1], None)
        if x is None:
            stack.pop()
            continue
        out.append(x)
        if x in ordered:
            stack.append(iter(ordered[x]))
    return out, steps


def tree_yata_chains(units):
    """tree_yata with every sibling group collapsed into chains first (yc_yata.hip k_tsib_big):
    kids at consecutive ascending (client, clock) positions c_1..c_m of one client with
    rightOrigin(c_k) = c_{k-1}, no other kid naming c_1..c_{m-1} as right origin, run through the
    sibling loop as one member (client, right origin of c_1) and expand to c_m .. c_1."""
    children = {}
    for u, (o, _) in units.items():
        children.setdefault(o, []).append(u)
    ordered = {}
    nchains = 0
    for p, kids in children.items():
        kids = sorted(kids)
        pos = {k: i for i, k in enumerate(kids)}
        ext = set()
        for i, k in enumerate(kids):
            r = units[k][1]
            if r in pos and not (pos[r] + 1 == i and r[0] == k[0]):
                ext.add(pos[r])
        node_of, firsts = [], []
        for i, k in enumerate(kids):
            r = units[k][1]
            link = i > 0 and units[k][1] == kids[i - 1] and r[0] == k[0] and (i - 1) not in ext
            if not link:
                firsts.append(i)
            node_of.append(len(firsts) - 1)
        nn = len(firsts)
        nchains += nn
        client = [kids[firsts[x]][0] for x in range(nn)]
        rn = []
        for x in range(nn):
            r = units[kids[firsts[x]]][1]
            rn.append(("in", node_of[pos[r]]) if r in pos else ("out", r))
        lst = []
        done = set()
        for x0 in range(nn):
            if x0 in done:
                continue
            stack = [x0]
            while stack:
                x = stack[-1]
                kind, r = rn[x]
                if kind == "in" and r not in done:
                    stack.append(r)
                    continue
                left = -1
                for i, o in enumerate(lst):
                    if kind == "in" and o == r:
                        break
                    if client[o] < client[x]:
                        left = i
                    elif rn[o] == rn[x]:
                        break
                lst.insert(left + 1, x)
                done.add(x)
                stack.pop()
        out = []
        for x in lst:
            end = firsts[x + 1] if x + 1 < nn else len(kids)
            out.extend(kids[i] for i in range(end - 1, firsts[x] - 1, -1))
        ordered[p] = out
    out = []
    stack = [iter(ordered.get(None, []))]
    while stack:
        x = next(stack[-1], None)
        if x is None:
            stack.pop()
            continue
        out.append(x)
        if x in ordered:
            stack.append(iter(ordered[x]))
    return out, nchains


def main():
    from tests.histories import array_history

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    tot = [0, 0, 0, 0]
    for seed in range(n):
        reps = 2 + seed % 7
        states, wire = array_history(7000 + seed, n_replicas=reps, rounds=2 + seed % 4, ops=3 + seed % 9)
        check(states + wire, f"seed {seed}", tot)
    print(f"{n} histories agree; scan steps: B.1 ascending {tot[0]}, descending {tot[1]}, tree sibling loops {tot[2]}; units absorbed into chains {tot[3]}")
    import json
    ncase = 0
    for name in ("array", "nested", "configs"):
        with open(os.path.join(ROOT, "tests", "golden", f"{name}.json")) as f:
            for c in json.load(f)["cases"]:
                check([bytes.fromhex(u) for u in c["updates"]], c["name"], tot)
                ncase += 1
    print(f"+ {ncase} golden cases agree; scan steps: B.1 ascending {tot[0]}, descending {tot[1]}, tree sibling loops {tot[2]}; units absorbed into chains {tot[3]}")


def check(updates, name, tot):
    for lk, units in units_of(updates).items():
        if lk is not None and lk[1] is not None:
            continue  # a YMap entry list (parentSub): winner descent, not YATA order
        a, sa = seq_yata(units)
        b, sb = seq_yata(units, descending=True)
        c, sc = tree_yata(units)
        d, nchain = tree_yata_chains(units)
        assert a == b, f"{name}: the loop depends on the causal order"
        assert a == c, f"{name}: tree order differs ({len(units)} units)"
        assert a == d, f"{name}: chain-collapsed order differs ({len(units)} units, {nchain} chains)"
        tot[3] += len(units) - nchain
        tot[0] += sa
        tot[1] += sb
        tot[2] += sc


if __name__ == "__main__":
    main()
