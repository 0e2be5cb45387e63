#!/usr/bin/env node
// Drives the N-API `Y` facade (crdt_amd/js). Modes:
//   cpu     — the addon loads, exports the Y surface, and fails loudly without a GPU
//   golden  — every golden case through Y.applyUpdate / Y.encodeStateAsUpdate / encodeStateVector
'use strict';
const fs = require('fs');
const path = require('path');
const assert = require('assert');

const ROOT = path.join(__dirname, '..', '..');
const Y = require(path.join(ROOT, 'crdt_amd', 'js'));
const hex = (u) => Buffer.from(u).toString('hex');
const unhex = (h) => new Uint8Array(Buffer.from(h, 'hex'));

const mode = process.argv[2] || 'cpu';
for (const f of ['Doc', 'applyUpdate', 'applyUpdates', 'encodeStateAsUpdate', 'encodeStateVector', 'mergeUpdates', 'diffUpdate']) {
  assert.strictEqual(typeof Y[f], 'function', f);
}
assert.ok(/gfx950/.test(Y.version()));
if (mode === 'cpu') {
  let threw = null;
  try { new Y.Doc(); } catch (e) { threw = e; }
  assert.ok(threw instanceof Error, 'no device: new Y.Doc() must throw');
  assert.ok(/device/i.test(threw.message), threw.message);
  console.log('napi cpu ok:', threw.message);
} else {
  let n = 0;
  for (const set of ['kat', 'map', 'array', 'nested']) {
    const cases = JSON.parse(fs.readFileSync(path.join(ROOT, 'tests', 'golden', set + '.json'))).cases;
    for (const c of cases) {
      const d = new Y.Doc({ clientID: 0x7ffffff0 });
      if (n % 2) Y.applyUpdates(d, c.updates.map(unhex));
      else for (const u of c.updates) Y.applyUpdate(d, unhex(u));
      assert.strictEqual(hex(Y.encodeStateAsUpdate(d)), c.state, c.name);
      assert.strictEqual(hex(Y.encodeStateVector(d)), c.sv, c.name);
      for (const df of c.diffs) assert.strictEqual(hex(Y.encodeStateAsUpdate(d, unhex(df.sv))), df.update, c.name);
      assert.strictEqual(hex(Y.mergeUpdates(c.updates.map(unhex))), c.updates.length > 1 ? c.merged : c.merged_raw, c.name);
      n++;
    }
  }
  let threw = null;
  try { Y.applyUpdate(new Y.Doc(), new Uint8Array([0xff, 0xff])); } catch (e) { threw = e; }
  assert.ok(threw && /Integer out of range/.test(threw.message), 'malformed update must throw like Yjs');
  console.log('napi golden ok:', n, 'cases');
}
