"""The single-workgroup small-merge kernels under both phase-boundary settings.

k_merge_small, k_view_small, k_decode_tail_small, k_sections_small and k_encode_small separate
their phases with plain barriers; their correctness rests on reading every atomically written
column through ld_fresh (yc_common.h, the invariant above phase_sync). YCRDT_PHASE_FENCE=1 puts
agent-scope fences around every phase boundary of k_merge_small (the one kernel with a fenced build). The suites that take these kernels on every
merge — the golden cases applied whole and one update at a time, Yjs's pending-struct checkpoints
and the per-key reads of crdt.js's per-op loop — run here under the fenced setting too, so the two
builds of the boundary stay equivalent (the default setting runs in their own files).
Reference: Y.applyUpdate / encodeStateAsUpdate / toJSON (crdt.js:294,297-305,347).
"""
import pytest

pytest.importorskip("crdt_amd")
from tests import test_gpu_parity as parity  # noqa: E402
from tests import test_gpu_pending as pending  # noqa: E402
from tests import test_gpu_view_reads as reads  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fenced(monkeypatch):
    monkeypatch.setenv("YCRDT_PHASE_FENCE", "1")


@pytest.mark.parametrize("setname", ["kat", "map", "array", "nested"])
def test_fenced_golden(golden, setname):
    parity.test_gpu_golden(golden, setname)
    parity.test_gpu_golden_incremental(golden, setname)


def test_fenced_pending():
    pending.test_pending_every_step(0)
    pending.test_pending_deferred_bursts()


@pytest.mark.parametrize("setname", ["kat", "map"])
def test_fenced_reads(golden, setname):
    reads.test_reads_match_tojson_golden(golden, setname)
    reads.test_reads_after_local_ops()
    reads.test_two_docs_one_engine_per_op_loop()
