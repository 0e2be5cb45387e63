"""The headline and side legs of one bench.py JSON line, in a few lines (GPU-run logs)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"], "roofline", d["roofline"]["kernel"], d["roofline"]["frac"],
      "pipeline", (d.get("pipeline_roofline") or {}).get("frac"))
print("phases", {k: v for k, v in (d.get("phases_ms") or {}).items() if v > 0.3})
if d.get("single_doc"):
    print("single", d["single_doc"])
if d.get("per_op"):
    print("per_op", {k: v["ops_per_s"] for k, v in d["per_op"].items()})
if d.get("c3"):
    print("c3", d["c3"]["ms_per_merge"], "yata", d["c3"]["phases_ms"].get("merge.yata"),
          "full state", {k: (v or {}).get("ms_per_merge") for k, v in d["c3"].get("full_state_ingest", {}).items() if k.startswith("into")})
if d.get("c4"):
    print("c4", d["c4"].get("ms_per_merge"), "chunk_wait", d["c4"].get("phases_ms", {}).get("decode.chunk_wait"),
          "sharded_8_logical", d["c4"].get("sharded_8_logical"))
if d.get("full_state_ingest"):
    print("c2 full state", {k: (v or {}).get("ms_per_merge") for k, v in d["full_state_ingest"].items() if k.startswith("into")})
for k in ("fleet_ingest", "fleet_sync", "apply_loop", "end_to_end"):
    if d.get(k):
        print(k, json.dumps(d[k])[:300])
