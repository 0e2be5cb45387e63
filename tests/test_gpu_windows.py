"""Batches laid out in several byte windows (merges past 4 GiB of input, yc_work.h WIN_SHIFT).

A batch larger than 4 GiB keeps every byte position a kernel handles as a u32 within a 2^32-byte
window; the windows are shrunk here to 1-8 MiB (YCRDT_WIN_SHIFT) so that every multi-window path —
the layout and staging of updates across windows, the per-window rebasing of the decoders'
byte / bitmap pointers, struct windows (s_win) in the integrate and encode kernels, 64-bit output
positions — runs on a few megabytes and is compared byte for byte with the one-window merge (which
the rest of the suite pins to Yjs 13.5.16). The full-size run (1 120 C2 documents, > 1 B items,
~15 GB of input) is bench.py --billion.
"""
import os

import pytest

import crdt_amd
from crdt_amd.workload import C2, gen_map

pytestmark = pytest.mark.gpu


def _c2(seed, n_keys=5000, n_replicas=120, ops=200):
    return gen_map(**dict(C2, n_keys=n_keys, n_replicas=n_replicas, ops_per_replica=ops, seed=seed))[0]


def _with_windows(shift, fn):
    old = os.environ.get("YCRDT_WIN_SHIFT")
    os.environ["YCRDT_WIN_SHIFT"] = str(shift)
    try:
        return fn()
    finally:
        if old is None:
            del os.environ["YCRDT_WIN_SHIFT"]
        else:
            os.environ["YCRDT_WIN_SHIFT"] = old


@pytest.mark.parametrize("shift,replicas", [(20, 500), (22, 2000)])
def test_windows_single_document(shift, replicas):
    ups = _c2(7, n_replicas=replicas)
    eng = crdt_amd.Engine()
    b = crdt_amd.Batch(ups, eng)
    st0 = b.merge()
    want = b.result()
    del b

    def run():
        bw = crdt_amd.Batch(ups, eng)
        st = bw.merge()
        return st, bw.result()

    st, got = _with_windows(shift, run)
    assert sum(map(len, ups)) > (1 << shift), "the batch must span several windows"
    assert got == want
    assert st.items == st0.items and st.structs == st0.structs


def test_windows_multi_document():
    docs = [_c2(100 + i, n_keys=2000, n_replicas=40, ops=150) for i in range(12)]
    eng = crdt_amd.Engine()
    b = crdt_amd.Batch(docs=docs, engine=eng)
    b.merge()
    want = b.result_docs()
    del b

    def run():
        bw = crdt_amd.Batch(docs=docs, engine=eng)
        bw.merge()
        return bw.result_docs()

    got = _with_windows(20, run)
    assert got == want


def test_windows_doc_state_prefix():
    """Doc API: the doc state (a device source) staged in front of host updates across windows."""
    ups = _c2(9, n_replicas=600)
    eng = crdt_amd.Engine()
    ref = crdt_amd.Doc(client_id=0x7FFFFFF0, engine=eng)
    ref.apply_updates(ups)
    want = ref.encode_state_as_update()

    def run():
        d = crdt_amd.Doc(client_id=0x7FFFFFF0, engine=eng)
        d.apply_updates(ups[: len(ups) // 2])
        d.flush()
        d.apply_updates(ups[len(ups) // 2:])
        return d.encode_state_as_update(), d.encode_state_vector()

    got, sv = _with_windows(20, run)
    assert got == want
    assert sv == ref.encode_state_vector()
