"""Regenerates tests/golden/workload.json: small C1/C2-shaped configs exported by the C++
generator as op scripts, replayed through real Yjs by pin_workload.js (test infrastructure)."""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, ROOT)
from crdt_amd.workload import gen_map  # noqa: E402

CONFIGS = {
    "c1_small": dict(n_keys=50, n_replicas=2, ops_per_replica=400, zipf_s=0.0, p_set=0.8, base_snapshot=False,
                     base_client=1, client_mode=1, value_mode=1, seed=42),
    "c2_small": dict(n_keys=200, n_replicas=12, ops_per_replica=60, zipf_s=1.1, p_set=0.8, base_snapshot=True,
                     base_client=1, client_mode=0, value_mode=0, seed=2),
    "c2_hot": dict(n_keys=8, n_replicas=20, ops_per_replica=40, zipf_s=1.1, p_set=0.8, base_snapshot=True,
                   base_client=1, client_mode=0, value_mode=0, seed=7),
    "c1_delheavy": dict(n_keys=10, n_replicas=3, ops_per_replica=200, zipf_s=0.0, p_set=0.4, base_snapshot=False,
                        base_client=1, client_mode=1, value_mode=1, seed=43),
}


def main():
    out = os.path.join(ROOT, "tests", "golden", "workload.json")
    if os.path.exists(out):
        os.remove(out)
    for name, cfg in CONFIGS.items():
        _, script = gen_map(**cfg, script=True)
        with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
            json.dump(script, f)
            sp = f.name
        subprocess.check_call(["node", os.path.join(HERE, "pin_workload.js"), sp, out, name, json.dumps(cfg)])
        os.unlink(sp)


if __name__ == "__main__":
    main()
