#!/usr/bin/env node
// Pins crdt_amd/workload (the C++ synthetic generator) against real Yjs 13.5.16: replays the op
// script the generator exported through Y.Doc / YMap.set / YMap.delete and records the bytes Yjs
// produces for the base snapshot and for every replica's encodeStateAsUpdate(replica, baseSV).
// TEST INFRASTRUCTURE ONLY. Usage: node pin_workload.js <script.json> <out.json> <name> <cfg-json>
'use strict';
const fs = require('fs');
const { loadYjs } = require('./load_yjs.js');
const { canonicalUpdate, hex } = require('./v1.js');

const Y = loadYjs();
const [,, scriptPath, outPath, name, cfgJson] = process.argv;
const script = JSON.parse(fs.readFileSync(scriptPath, 'utf8'));
const root = script.root;
const updates = [];
let baseUpdate = null;
if (script.base.length) {
  const b = new Y.Doc();
  b.clientID = script.base_client;
  const m = b.getMap(root);
  script.base.forEach((v, k) => m.set('user' + k, v));
  baseUpdate = Y.encodeStateAsUpdate(b);
  updates.push(canonicalUpdate(baseUpdate));
}
for (const rep of script.replicas) {
  const d = new Y.Doc();
  d.clientID = rep.client;
  if (baseUpdate) Y.applyUpdate(d, baseUpdate);
  const sv = Y.encodeStateVector(d);
  const m = d.getMap(root);
  for (const op of rep.ops) {
    if (op[0] === 's') m.set('user' + op[1], op[2]);
    else m.delete('user' + op[1]);
  }
  updates.push(canonicalUpdate(Y.encodeStateAsUpdate(d, sv)));
}
// reference merge of the whole batch
const merger = new Y.Doc();
merger.clientID = 0x7ffffff0;
for (const u of updates) Y.applyUpdate(merger, u);
const out = fs.existsSync(outPath) ? JSON.parse(fs.readFileSync(outPath, 'utf8')) : { generator: 'tests/golden/gen/pin_workload.js', yjs: '13.5.16', cases: [] };
out.cases = out.cases.filter((c) => c.name !== name);
out.cases.push({
  name,
  cfg: JSON.parse(cfgJson),
  updates: updates.map(hex),
  state: hex(canonicalUpdate(Y.encodeStateAsUpdate(merger))),
  json: merger.getMap(root).toJSON(),
});
fs.writeFileSync(outPath, JSON.stringify(out));
console.log(name, updates.length, 'updates');
