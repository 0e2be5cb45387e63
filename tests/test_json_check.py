"""ContentJSON / ContentEmbed / ContentFormat values (yc_parse.h json_check, json_canon) against Node's
own JSON: tests/golden/json_forms.json (tests/golden/gen/gen_json_fixtures.js) records, for 5 399
seeded strings, whether JSON.parse throws (the engine must refuse the update: Yjs throws SyntaxError
in readContentJSON / readJSON, Y@72137 / Y@14715), whether JSON.stringify gives the text back, and
JSON.stringify(JSON.parse(s)). Yjs keeps the parsed value and writes it with JSON.stringify
(Y@71991), so the engine rewrites every value not in that form (yc_decode.hip k_json_canon) instead
of refusing it. The host build of the functions the decoder runs: json_check's verdict must match
Node's (a canonical text nested past its level mask may be left unjudged: it is rewritten to
itself), and json_canon's text must equal Node's for every valid case and refuse every malformed
one — long numbers (0.30000000000000004, 800-digit and halfway forms, subnormals, overflow to
null), deep nesting, duplicate / array-index / escaped keys, escapes of every kind."""
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
    inp = "".join(f"{w} {h} {c}\n" for w, h, c in cases)
    r = subprocess.run([str(exe)], input=inp, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:]
    last = r.stdout.strip().splitlines()[-1].split()
    assert int(last[1]) == len(cases) and int(last[3]) == 0 and int(last[9]) == 0
    assert int(last[5]) <= 8  # canonical texts json_check leaves to json_canon (nesting past 64 levels)
    assert int(last[7]) == sum(1 for w, _, _ in cases if w != 1)
    assert {w for w, _, _ in cases} == {0, 1, 2}
    assert any(bytes.fromhex(h) == b"0.30000000000000004" and w == 0 for w, h, _ in cases)


def test_any_canon_matches_yjs(tmp_path):
    """writeAny(readAny(.)) of hand-written `any` values (tests/golden/anyform.json, Yjs 13.5.16):
    the host build of yc_parse.h any_content_canon — what the device rewrite runs for object keys
    JS treats specially (ANY_KEYS: repeated keys, array-index key order, "__proto__") and every
    scalar's writeAny form — gives the content Yjs's state holds; the refused cases are refused."""
    exe = tmp_path / "any_canon"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "crdt_amd", "csrc"),
                           os.path.join(HERE, "csrc", "any_canon_main.cpp"), "-o", str(exe)])
    with open(os.path.join(HERE, "golden", "anyform.json")) as f:
        cases = json.load(f)["cases"]

    def content(u: bytes, key: str) -> bytes:
        # [1 section][1 struct][client 77][clock 0][info 0x28][parent info 1]'users' key, then the
        # content (count + values) and an empty delete set
        head = bytes([1, 1, 77, 0, 0x28, 1, 5]) + b"users" + bytes([len(key)]) + key.encode()
        assert u.startswith(head) and u.endswith(b"\x00")
        return u[len(head):-1]

    inp, want = [], []
    for c in cases:
        if c["name"] == "obj_overlong_key":
            continue  # (the key's overlong length prefix is part of the content here, not the header)
        inp.append(content(bytes.fromhex(c["update"]), "k_" + c["name"]).hex())
        want.append(None if c["refused"] else content(bytes.fromhex(c["state"]), "k_" + c["name"]).hex())
    r = subprocess.run([str(exe)], input="\n".join(inp) + "\n", capture_output=True, text=True, check=True)
    outs = r.stdout.splitlines()
    assert len(outs) == len(want)
    for c, w, g in zip([c for c in cases if c["name"] != "obj_overlong_key"], want, outs):
        if w is None:
            assert g.startswith("ERR"), c["name"]
        else:
            assert g == w, (c["name"], g, w)
