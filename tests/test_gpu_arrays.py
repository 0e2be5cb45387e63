"""GPU YArray / YATA parity on seeded random histories (oracle = CPU restatement of Yjs)."""
import json
import random

import pytest

crdt_amd = pytest.importorskip("crdt_amd")
from oracle.yref import Doc as ODoc  # noqa: E402
from tests.histories import array_history  # noqa: E402

pytestmark = pytest.mark.gpu


def _oracle(updates):
    d = ODoc(0x7FFFFFF0)
    for u in updates:
        d.apply_update(u)
    return d


@pytest.mark.parametrize("seed", range(12))
def test_gpu_array_histories(seed):
    states, wire = array_history(seed, n_replicas=2 + seed % 5, rounds=3 + seed % 3, ops=5, with_map=seed % 2 == 1)
    batch = states + wire
    random.Random(seed).shuffle(batch)
    ref = _oracle(states + wire)  # a causal order for the sequential oracle
    want = ref.encode_state_as_update()
    d = crdt_amd.Doc(client_id=0x7FFFFFF0)
    d.apply_updates(batch)
    assert d.encode_state_as_update() == want
    assert d.encode_state_vector() == ref.encode_state_vector()


def test_gpu_array_many_replicas():
    states, wire = array_history(99, n_replicas=16, rounds=4, ops=8)
    ref = _oracle(states)
    d = crdt_amd.Doc(client_id=0x7FFFFFF0)
    d.apply_updates(states)
    assert d.encode_state_as_update() == ref.encode_state_as_update()
