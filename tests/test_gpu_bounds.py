"""The unit passes and the single-workgroup kernels under YCRDT_DEBUG_BOUNDS=1.

Round 5's one GPU fault (an illegal memory access in the pending path while the single-workgroup
small-batch kernels were being written) and the stale client hash of the quick small decode
(k_sections_small skipped its fill when a batch had no section: find_client could return a stale
client index, whose unit base sent k_units' flag stores past the unit table) both end in a table
index past its table. With the flag every unit flag store, key slot, segment count, client count and
output struct of these kernels is checked against the size its table was allocated with, and a
violation is reported (device printf) and stops the merge with a capacity error instead of writing
past the table. The suites that run these kernels on every merge — pending checkpoints, the golden
cases one update at a time, local-op scripts, the delete-set edge shapes — run here with it.
Reference: Y.applyUpdate / encodeStateAsUpdate (crdt.js:294,347).
"""
import pytest

pytest.importorskip("crdt_amd")
from tests import test_gpu_ds_edges as dse  # noqa: E402
from tests import test_gpu_edges as edges  # noqa: E402
from tests import test_gpu_parity as parity  # noqa: E402
from tests import test_gpu_pending as pending  # noqa: E402
from tests import test_gpu_view as view  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _bounds(monkeypatch):
    monkeypatch.setenv("YCRDT_DEBUG_BOUNDS", "1")


def test_bounds_pending():
    for part in range(3):
        pending.test_pending_every_step(part)
    edges.test_missing_dependencies_are_pending_not_refused()


@pytest.mark.parametrize("setname", ["kat", "map", "array", "nested"])
def test_bounds_golden_incremental(golden, setname):
    parity.test_gpu_golden_incremental(golden, setname)


def test_bounds_local_ops():
    view.test_gpu_local_ops_yjs(0)


@pytest.mark.parametrize("mode", ("direct", "wave"))
def test_bounds_delete_only_into_empty_doc(mode, monkeypatch):
    dse.test_delete_only_into_empty_doc_after_other_merges(mode, monkeypatch)


def test_bounds_small_update_past_dsa_wave(monkeypatch):
    dse.test_small_update_past_dsa_wave("direct", True, monkeypatch)
