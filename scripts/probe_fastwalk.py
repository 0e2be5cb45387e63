"""Which fast walk takes a large snapshot (YCRDT_DEBUG_DECODE=1 lines on stderr)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["YCRDT_DEBUG_DECODE"] = "1"
import crdt_amd  # noqa: E402
from tests.test_gpu_fastwalk import _snapshot, _replica  # noqa: E402

for name, u in (("snap40x200 maps", _snapshot(40, 200, 5, arrays=False)), ("snap64x60", _snapshot(64, 60, 64 * 31 + 60)),
                ("replica2400", _replica(77, 2400, 300, 1))):
    print(name, len(u), u[:4].hex(), flush=True)
    b = crdt_amd.Batch([u])
    b.merge()
    print(" batch merged", flush=True)
    d = crdt_amd.Doc(client_id=5)
    d.apply_updates([u])
    d.encode_state_as_update()
    print(" doc merged", flush=True)
