"""ContentJSON / ContentEmbed / ContentFormat values (yc_parse.h json_check) against Node's own
JSON: tests/golden/json_forms.json (tests/golden/gen/gen_json_fixtures.js) records, for 2 566
seeded strings, whether JSON.parse throws (the engine must refuse the update: Yjs throws
SyntaxError in readContentJSON / readJSON, Y@72137 / Y@14715) and whether JSON.stringify gives the
text back (Yjs writes the parsed value with JSON.stringify, Y@71991; the engine copies the bytes,
so it refuses — YCRDT_E_UNSUPPORTED — what it would write differently). The host build of the
function the decoder runs: no case may be accepted that Node refuses or writes differently; some
canonical texts are refused conservatively (more than 15 significant digits, subnormal numbers),
counted here."""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def test_json_check_matches_node(tmp_path):
    exe = tmp_path / "json_check"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "crdt_amd", "csrc"),
                           os.path.join(HERE, "csrc", "json_check_main.cpp"), "-o", str(exe)])
    with open(os.path.join(HERE, "golden", "json_forms.json")) as f:
        cases = json.load(f)["cases"]
    inp = "".join(f"{w} {h}\n" for w, h in cases)
    r = subprocess.run([str(exe)], input=inp, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:]
    last = r.stdout.strip().splitlines()[-1].split()
    assert int(last[1]) == len(cases) and int(last[3]) == 0
    assert int(last[5]) < len(cases) // 8  # conservative refusals stay a small minority
    assert {w for w, _ in cases} == {0, 1, 2}
