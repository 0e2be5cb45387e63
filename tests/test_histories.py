"""CPU: the order-independence property that licenses a batched merge, checked
on the oracle over seeded random YArray/YMap histories."""
import random

import pytest

from oracle.yref import Doc
from tests.histories import array_history


@pytest.mark.parametrize("seed", range(8))
def test_oracle_merge_order_independent(seed):
    states, wire = array_history(seed, n_replicas=3 + seed % 4, rounds=3, ops=5, with_map=seed % 2 == 0)
    outs = set()
    for k in range(3):
        # any order of the (self-contained) replica states, then the wire deltas in arrival order
        order = list(states)
        random.Random(seed * 10 + k).shuffle(order)
        order += wire if k % 2 == 0 else []
        d = Doc(0x7FFFFFF0)
        for u in order:
            d.apply_update(u)
        outs.add(d.encode_state_as_update())
    assert len(outs) == 1
