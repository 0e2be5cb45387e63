"""Parallel YATA on the GPU (yc_yata.hip: origin-tree pre-order with per-node sibling loops)
against Yjs 13.5.16 with 64-256 replicas (tests/golden/yata.json, config C3's op mix): the
batched merge, a shuffled one-at-a-time apply, toJSON, and the sequential kernel (YCRDT_YATA=seq)
cross-checked in a child process."""
import json
import os
import random
import subprocess
import sys

import pytest

crdt_amd = pytest.importorskip("crdt_amd")

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cases():
    with open(os.path.join(ROOT, "tests", "golden", "yata.json")) as f:
        return json.load(f)["cases"]


def test_gpu_yata_many_replicas_batch():
    for c in _cases():
        ups = [bytes.fromhex(u) for u in c["updates"]]
        b = crdt_amd.Batch(ups)
        b.merge()
        out, sv = b.result()
        assert out.hex() == c["state"], c["name"]
        d = crdt_amd.Doc(client_id=0x7FFFFFF0)
        d.apply_updates(ups)
        assert json.loads(d.root_json("messages", "array")) == c["json"]["messages"], c["name"]


def test_gpu_yata_many_replicas_shuffled_applies():
    for i, c in enumerate(_cases()):
        ups = [bytes.fromhex(u) for u in c["updates"]]
        random.Random(i).shuffle(ups)  # non-causal order: parked as pending, then integrated
        d = crdt_amd.Doc(client_id=0x7FFFFFF0)
        for u in ups:
            d.apply_update(u)
        assert d.encode_state_as_update().hex() == c["state"], c["name"]
        assert d.pending() == (False, False)


def test_gpu_yata_tree_equals_sequential_kernel():
    code = ("import json,sys; sys.path.insert(0, %r); import crdt_amd\n"
            "cs = json.load(open(%r))['cases']\n"
            "for c in cs:\n"
            "    b = crdt_amd.Batch([bytes.fromhex(u) for u in c['updates']]); b.merge()\n"
            "    assert b.result()[0].hex() == c['state'], c['name']\n"
            "print('ok')\n") % (ROOT, os.path.join(ROOT, "tests", "golden", "yata.json"))
    env = dict(os.environ, YCRDT_YATA="seq")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


@pytest.mark.parametrize("reps,rounds,items,seed", [(64, 4, 200_000, 11), (4096, 2, 60_000, 5)])
def test_gpu_yata_large_sibling_group(reps, rounds, items, seed):
    """C3-generator histories whose list head carries a sibling group larger than one workgroup's
    LDS (every unshift has the list root as origin): (64, 4) collapses it into per-(replica, round)
    chains (k_tsib_big); (4096, 2) leaves too many chains for LDS and runs in place. Byte-exact
    against the oracle, and the list order is the generator's independent origin-tree order."""
    from crdt_amd.workload import gen_array
    from oracle.yref import Doc as ODoc
    from tests.test_workload_c3 import _any_json
    from oracle.ymerge import ITEM, Dec, lazy_structs

    ups, st = gen_array(reps, rounds, items, seed, order=True)
    heads = sum(1 for u in ups for s in lazy_structs(Dec(u)) if s.kind == ITEM and s.origin is None)
    assert heads > 6144  # the root sibling group exceeds k_tsib_big's LDS staging
    ref = ODoc(0x7FFFFFF0)
    for u in ups:
        ref.apply_update(u)
    b = crdt_amd.Batch(ups)
    b.merge()
    assert b.result()[0] == ref.encode_state_as_update()
    vals = {}
    for u in ups:
        for s in lazy_structs(Dec(u)):
            if s.kind == ITEM:
                for i, raw in enumerate(s.content):
                    vals[(s.client, s.clock + i)] = _any_json(raw, 0)[0]
    d = crdt_amd.Doc(client_id=0x7FFFFFF0)
    d.apply_updates(ups)
    assert json.loads(d.root_json("messages", "array")) == [vals[k] for k in st["order"]]
