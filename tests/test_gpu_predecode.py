"""A doc state decoded by the encode that produced it (yc_encode.hip k_state_marks, yc_decode.hip
k_predecoded): the next merge of the doc takes its state's struct starts, section records and
delete-set start from the marks instead of parsing the state again (crdt.js's steady state:
Y.applyUpdate into a resident doc, crdt.js:294, the sync reply crdt.js:288, every local op
crdt.js:433-445).

The marks must be exactly the decode of the state. YCRDT_PREDECODE=check decodes every doc state the
usual way as well and compares it with its marks word for word (a difference fails the merge with a
decode error); YCRDT_PREDECODE=0 turns the marks off. The doc-path suites — every golden case applied
one update at a time, Yjs's pending checkpoints in both client orders, the recorded local-op scripts,
YArray histories, a large many-client state with deltas — run under "check", and their bytes must
equal the marks-off run and the oracle. Reference: Y.applyUpdate / encodeStateAsUpdate.
"""
import pytest

crdt_amd = pytest.importorskip("crdt_amd")
from oracle.yref import Doc as ODoc  # noqa: E402
from tests import test_gpu_compat135 as c135  # noqa: E402
from tests import test_gpu_parity as parity  # noqa: E402
from tests import test_gpu_pending as pending  # noqa: E402
from tests import test_gpu_view as view  # noqa: E402
from tests.histories import any_int  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["check", "0"])
def mode(request, monkeypatch):
    monkeypatch.setenv("YCRDT_PREDECODE", request.param)
    return request.param


@pytest.mark.parametrize("setname", ["kat", "map", "array", "nested"])
def test_predecode_golden_incremental(golden, setname, mode):
    parity.test_gpu_golden_incremental(golden, setname)


def test_predecode_pending(mode):
    for part in range(3):
        pending.test_pending_every_step(part)
    pending.test_pending_batch_apply_equals_sequential()


def test_predecode_pending_135(mode, e135):
    c135.test_135_pending_every_step_raw(0, e135)


@pytest.fixture(scope="module")
def e135():
    import os

    e = crdt_amd.Engine(int(os.environ.get("YCRDT_DEVICE", "0")), compat=135)
    yield e
    e.close()


@pytest.mark.parametrize("chunk", range(2))
def test_predecode_local_ops(chunk, mode):
    view.test_gpu_local_ops_yjs(chunk)


def test_predecode_arrays_and_deltas(mode):
    from tests.histories import array_history

    states, wire = array_history(31, n_replicas=5, rounds=4, ops=12, with_map=True)
    ref = ODoc(0x7FFFFFF0)
    d = crdt_amd.Doc(client_id=0x7FFFFFF0)
    for u in states + wire:
        ref.apply_update(u)
        d.apply_update(u)
        assert d.encode_state_as_update() == ref.encode_state_as_update()
        # the sync reply (a delta against a peer's state vector) re-merges the resident state
        sv = ref.encode_state_vector()
        assert d.encode_state_as_update(sv) == ref.encode_state_as_update(sv)


def test_predecode_large_state_small_deltas(mode):
    """A many-client doc state (a full state of > 64 KiB: record mode on its first decode) and one
    small peer delta at a time, each merged behind the resident state."""
    from crdt_amd.workload import C2, gen_map

    cfg = dict(C2)
    cfg.update(n_keys=3000, n_replicas=200, ops_per_replica=150)
    ups, _ = gen_map(**cfg)
    peer = ODoc(0x5EED0002)
    for u in ups:
        peer.apply_update(u)
    full = peer.encode_state_as_update()
    d = crdt_amd.Doc(client_id=0x7FFFFFF0)
    d.apply_update(full)
    assert d.encode_state_as_update() == full
    for i in range(12):
        sv = peer.encode_state_vector()
        if i % 4 == 3:
            peer.map_delete("users", "k%d" % (i * 37 % 3000))
        else:
            peer.map_set("users", "k%d" % (i * 37 % 3000), any_int(i))
        d.apply_update(peer.encode_state_as_update(sv))
        assert d.encode_state_vector() == peer.encode_state_vector()
    assert d.encode_state_as_update() == peer.encode_state_as_update()
