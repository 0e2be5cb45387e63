"""The reference-language boundary: the Node-API addon + `Y` facade (crdt_amd/js) that
@ypear/crdt receives as router.options.Y (reference crdt.js:175-180)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


def _run(mode, timeout, env=None):
    r = subprocess.run([NODE, os.path.join(ROOT, "tests", "js", "napi_check.js"), mode], capture_output=True, text=True,
                       timeout=timeout, env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_napi_addon_loads_and_fails_loudly_without_gpu():
    import crdt_amd

    try:
        crdt_amd.Engine()
        pytest.skip("a GPU is present: the no-device behaviour is not observable")
    except crdt_amd.YcrdtError:
        pass
    out = _run("cpu", 120)
    assert "napi cpu ok" in out and "any codec ok" in out


@pytest.mark.gpu
def test_napi_golden_on_gpu():
    assert "napi golden ok" in _run("golden", 300)


@pytest.mark.gpu
def test_napi_facade_ops_on_gpu():
    """The crdt.js-facing YMap / YArray facade replays every recorded Yjs op script byte-exactly."""
    assert "napi ops ok" in _run("ops", 300)


@pytest.mark.gpu
def test_napi_crdtjs_traces_on_gpu():
    """crdt.js's own Y call sequence (recorded from crdt.js on a fake router, 2-4 peers, set / del /
    push / insert / unshift / cut / execBatch): every wire update and state vector is Yjs 13.5.16's
    raw bytes (compat 135) and every toJSON / get / has the same value (crdt.c, D1 / D7)."""
    out = _run("trace", 600, {"YCRDT_COMPAT": "135"})
    assert "napi trace ok" in out


@pytest.mark.gpu
def test_napi_observer_events_on_gpu():
    """YMap / YArray observers (crdt.js:620-657) deliver the events Yjs 13.5.16 delivered on the same
    scripts (tests/golden/observe.json): keysChanged and changes.keys from the entries' winning
    items, YArray changes.delta, nested arrays observed on their own list. Both observer modes:
    'sync' (Yjs's timing: every event inside the call that caused it, before any read) and
    'deferred' (events at the next read, one merge per burst of Y.applyUpdate)."""
    assert "napi observe ok" in _run("observe", 300)
