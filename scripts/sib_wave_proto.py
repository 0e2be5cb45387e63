#!/usr/bin/env python3
"""Prototype: the B.1 sibling loop (yc_yata.hip sib_loop) restated over list POSITIONS, the form
k_tsib_wave evaluates with one lane per member (ballots and wave reductions instead of lane 0
walking linked lists). Checked here against the linked-list loop on random groups, including the
inputs valid Yjs never produces (same-client ties, right-origin cycles).

Placement of member c (members sorted by client; rp = in-group right-origin sibling, else an
outside right-origin group keyed by its anchor):
  succ = the placed member of c's right-origin group with the smallest client > c's (ties: the
         one placed first); stop = succ, else rp, else the end
  left = the placed member with the largest position before stop whose client is < c's
  c goes right after left (position 0 without one); every position at or past it moves up by 1
"""
import random
import sys

NONE = None


def sib_loop(cid, rp, anc):
    """Linked-list form (yc_yata.hip sib_loop). anc[i]: ('in', rp) or ('out', anchor index)."""
    n = len(cid)
    done = [0] * n
    nxt, prv, mprv = [NONE] * n, [NONE] * n, [NONE] * n
    mtail, otail = [NONE] * n, [NONE] * n
    head = tail = NONE
    for i0 in range(n):
        if done[i0] == 2:
            continue
        stack = [i0]
        done[i0] = 1
        c = i0
        while stack:
            r = rp[c]
            if r is not NONE and done[r] != 2:
                if done[r] == 1 or len(stack) >= n:
                    return "error"
                done[r] = 1
                stack.append(r)
                c = r
                continue
            cc = cid[c]
            kind, ta = anc[c]
            m = otail[ta] if kind == "out" else mtail[ta]
            succ = NONE
            while m is not NONE and cid[m] > cc:
                succ = m
                m = mprv[m]
            mprv[c] = m
            if succ is not NONE:
                mprv[succ] = c
            elif kind == "out":
                otail[ta] = c
            else:
                mtail[ta] = c
            stop = succ if succ is not NONE else r
            left = prv[stop] if stop is not NONE else tail
            while left is not NONE and cid[left] >= cc:
                left = prv[left]
            nx = nxt[left] if left is not NONE else head
            prv[c], nxt[c] = left, nx
            if left is not NONE:
                nxt[left] = c
            else:
                head = c
            if nx is not NONE:
                prv[nx] = c
            else:
                tail = c
            done[c] = 2
            stack.pop()
            if stack:
                c = stack[-1]
    out = []
    x = head
    while x is not NONE:
        out.append(x)
        x = nxt[x]
    return out


def sib_positions(cid, rp, anc):
    """Position form: every member keeps pos (its index in the list built so far) and seq (when it
    was placed); each step is a handful of wave-wide min / max reductions."""
    n = len(cid)
    done = [0] * n
    pos = [None] * n
    seq = [None] * n
    gkey = [anc[i] for i in range(n)]  # the right-origin group a member belongs to
    placed = 0
    for i0 in range(n):
        if done[i0] == 2:
            continue
        stack = [i0]
        done[i0] = 1
        c = i0
        while stack:
            r = rp[c]
            if r is not NONE and done[r] != 2:
                if done[r] == 1 or len(stack) >= n:
                    return "error"
                done[r] = 1
                stack.append(r)
                c = r
                continue
            cc = cid[c]
            # succ: min (client, seq) over placed members of c's group with client > cc
            best = None
            for j in range(n):
                if done[j] == 2 and gkey[j] == gkey[c] and cid[j] > cc:
                    k = (cid[j], seq[j])
                    if best is None or k < best[0]:
                        best = (k, j)
            succ = best[1] if best else NONE
            stop = succ if succ is not NONE else r
            pstop = pos[stop] if stop is not NONE else placed
            # left: max position < pstop over placed members with client < cc
            lp = -1
            for j in range(n):
                if done[j] == 2 and pos[j] < pstop and cid[j] < cc:
                    lp = max(lp, pos[j])
            p = lp + 1
            for j in range(n):
                if done[j] == 2 and pos[j] >= p:
                    pos[j] += 1
            pos[c] = p
            seq[c] = placed
            placed += 1
            done[c] = 2
            stack.pop()
            if stack:
                c = stack[-1]
    order = [None] * n
    for j in range(n):
        order[pos[j]] = j
    return order


def sib_positions_space(cid, rp, anc):
    """The same loop with the list held in POSITION space (what k_tsib_wave keeps in its lanes):
    P_cid / P_gk / P_mem at list position x. succ = the first position of c's group whose client is
    above c's (a group's members stand in ascending client order, equal clients in placement
    order); left = the last position before stop whose client is below c's; inserting shifts the
    positions at or past it up by one."""
    n = len(cid)
    done = [0] * n
    pos = [None] * n
    P_cid, P_gk, P_mem = [], [], []
    for i0 in range(n):
        if done[i0] == 2:
            continue
        stack = [i0]
        done[i0] = 1
        c = i0
        while stack:
            r = rp[c]
            if r is not NONE and done[r] != 2:
                if done[r] == 1 or len(stack) >= n:
                    return "error"
                done[r] = 1
                stack.append(r)
                c = r
                continue
            cc = cid[c]
            succ = NONE
            for x in range(len(P_cid)):
                if P_gk[x] == anc[c] and P_cid[x] > cc:
                    succ = P_mem[x]
                    break
            stop = succ if succ is not NONE else r
            pstop = pos[stop] if stop is not NONE else len(P_cid)
            p = 0
            for x in range(pstop - 1, -1, -1):
                if P_cid[x] < cc:
                    p = x + 1
                    break
            for j in range(n):
                if done[j] == 2 and pos[j] >= p:
                    pos[j] += 1
            P_cid.insert(p, cc)
            P_gk.insert(p, anc[c])
            P_mem.insert(p, c)
            pos[c] = p
            done[c] = 2
            stack.pop()
            if stack:
                c = stack[-1]
    return P_mem


def random_group(rng, n):
    nclients = rng.randint(1, n)
    cid = sorted(rng.randrange(nclients) for _ in range(n))
    rp = [NONE] * n
    outs = []
    for i in range(n):
        if rng.random() < 0.4 and n > 1:
            j = rng.randrange(n)
            if j != i:
                rp[i] = j
        if rp[i] is NONE:
            outs.append(i)
    # outside right origins: a few distinct units; anchor = first member with the same one
    unit = {i: rng.randrange(max(1, n // 4)) for i in outs}
    anc = [None] * n
    first = {}
    for i in range(n):
        if rp[i] is not NONE:
            anc[i] = ("in", rp[i])
        else:
            u = unit[i]
            first.setdefault(u, i)
            anc[i] = ("out", first[u])
    return cid, rp, anc


def main():
    rng = random.Random(int(sys.argv[1]) if len(sys.argv) > 1 else 1)
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    errs = 0
    for t in range(trials):
        n = rng.randint(1, 64)
        cid, rp, anc = random_group(rng, n)
        a = sib_loop(cid, rp, anc)
        b = sib_positions(cid, rp, anc)
        c = sib_positions_space(cid, rp, anc)
        if a != b or a != c:
            print("MISMATCH", t, n, cid, rp, anc, a, b, c)
            return 1
        errs += a == "error"
    # the kernels' shortcut: one outside right origin for every member and strictly ascending
    # clients give the ascending order (no newcomer ever finds a higher client placed, or a stop)
    for t in range(trials // 4):
        n = rng.randint(1, 64)
        cid = sorted(rng.sample(range(4 * n + 4), n))
        assert sib_loop(cid, [NONE] * n, [("out", 0)] * n) == list(range(n))
    print(f"ok: {trials} groups, {errs} with right-origin cycles (both report them); plain groups ascending")
    return 0


if __name__ == "__main__":
    sys.exit(main())
