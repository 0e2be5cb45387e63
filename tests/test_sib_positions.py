"""The position form of the B.1 sibling loop that k_tsib_wave runs (yc_yata.hip sib_wave) against
the linked-list loop the other sibling kernels run (sib_loop), on random groups of up to 64
members — including inputs valid Yjs never produces (one client twice in a group, right-origin
cycles) — and the shortcut both small-group kernels take (one outside right origin, strictly
ascending clients: ascending order). CPU only: scripts/sib_wave_proto.py holds both forms."""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
import sib_wave_proto as P  # noqa: E402


def test_position_forms_equal_linked_list_loop():
    rng = random.Random(2024)
    cycles = 0
    for _ in range(3000):
        n = rng.randint(1, 64)
        cid, rp, anc = P.random_group(rng, n)
        ref = P.sib_loop(cid, rp, anc)
        assert P.sib_positions(cid, rp, anc) == ref
        assert P.sib_positions_space(cid, rp, anc) == ref
        cycles += ref == "error"
    assert cycles > 0  # the cycle report is exercised too


def test_plain_groups_are_ascending():
    rng = random.Random(7)
    for _ in range(1000):
        n = rng.randint(1, 64)
        cid = sorted(rng.sample(range(4 * n + 4), n))
        assert P.sib_loop(cid, [P.NONE] * n, [("out", 0)] * n) == list(range(n))
