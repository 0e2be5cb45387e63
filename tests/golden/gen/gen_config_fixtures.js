#!/usr/bin/env node
// Config-shaped golden fixtures (TEST INFRASTRUCTURE ONLY; runs in the build container, never on
// the GPU box). Reduced-scale versions of BASELINE.json configs C3 / C4 / C5 (SURVEY.md §8(d))
// played through the in-image Yjs 13.5.16, with Yjs's own merged result as the expected output:
//   c3: YArray 'messages', replicas doing push / unshift / insert / cut with gossip rounds;
//   c4: YMap 'docs' whose keys hold nested YArrays, pushes into them, 10 % of keys overwritten by
//       a fresh Y.Array (the old one and its items are garbage-collected);
//   c5: a fleet of small docs ('ix' + 'users' maps, 2-4 clients), each with a lagging peer state
//       vector and the delta Yjs encodes for it (crdt.js sync responder, crdt.js:286-291).
// Every case records the input updates, the canonical (13.6 order) encodeStateAsUpdate and
// encodeStateVector of a Yjs doc that applied them all, and toJSON of the roots.
//
// Usage: node gen_config_fixtures.js <out_dir>  ->  <out_dir>/configs.json
'use strict';
const fs = require('fs');
const path = require('path');
const { loadYjs } = require('./load_yjs.js');
const { canonicalUpdate, canonicalSv, hex } = require('./v1.js');

const Y = loadYjs();

function mulberry32(a) {
  return function () {
    a |= 0; a = (a + 0x6D2B79F5) | 0;
    let t = Math.imul(a ^ (a >>> 15), 1 | a);
    t = (t + Math.imul(t ^ (t >>> 7), 61 | t)) ^ t;
    return ((t ^ (t >>> 14)) >>> 0) / 4294967296;
  };
}
function rng(seed) {
  const r = mulberry32(seed);
  return { r, int: (n) => Math.floor(r() * n), pick: (a) => a[Math.floor(r() * a.length)] };
}
const clientOf = (i) => (((i + 1) * 2654435761) >>> 0) || 1;

function gossip(g, docs) {  // every replica pulls a delta from one random peer
  for (let i = 0; i < docs.length; i++) {
    const p = g.int(docs.length);
    if (p === i) continue;
    Y.applyUpdate(docs[i], Y.encodeStateAsUpdate(docs[p], Y.encodeStateVector(docs[i])));
  }
}

function expected(updates, roots) {
  const d = new Y.Doc(); d.clientID = 0x7ffffff0;
  for (const u of updates) Y.applyUpdate(d, u);
  const json = {};
  for (const [name, kind] of Object.entries(roots)) json[name] = (kind === 'map' ? d.getMap(name) : d.getArray(name)).toJSON();
  return { d, state: hex(canonicalUpdate(Y.encodeStateAsUpdate(d))), sv: hex(canonicalSv(Y.encodeStateVector(d))), json: JSON.parse(JSON.stringify(json)) };
}

function arrayOp(g, arr, r, seq) {
  const L = arr.length; const x = g.r();
  const vals = () => { const n = 1 + g.int(4); const v = []; for (let i = 0; i < n; i++) v.push(g.r() < 0.6 ? `m${r}_${seq}_${i}` : g.int(1 << 20)); return v; };
  if (x < 0.4 || L === 0) arr.push(vals());
  else if (x < 0.55) arr.unshift(vals());
  else if (x < 0.85) arr.insert(g.int(L + 1), vals());
  else { const i = g.int(L); arr.delete(i, Math.min(L - i, 1 + g.int(3))); }
}

function c3(seed, nrep, rounds, ops) {
  const g = rng(seed);
  const docs = []; for (let i = 0; i < nrep; i++) { const d = new Y.Doc(); d.clientID = clientOf(i); docs.push(d); }
  let seq = 0;
  for (let k = 0; k < rounds; k++) {
    docs.forEach((d, r) => { for (let j = 0; j < ops; j++) arrayOp(g, d.getArray('messages'), r, seq++); });
    gossip(g, docs);
  }
  const updates = docs.map((d) => Y.encodeStateAsUpdate(d));
  const e = expected(updates, { messages: 'array' });
  return { name: `c3_s${seed}_r${nrep}`, updates: updates.map(hex), state: e.state, sv: e.sv, json: e.json, diffs: [] };
}

function c4(seed, nrep, nkeys, rounds, ops) {
  const g = rng(seed);
  const docs = []; for (let i = 0; i < nrep; i++) { const d = new Y.Doc(); d.clientID = clientOf(100 + i); docs.push(d); }
  let seq = 0;
  for (let k = 0; k < rounds; k++) {
    docs.forEach((d, r) => {
      const m = d.getMap('docs');
      for (let j = 0; j < ops; j++) {
        const key = 'd' + g.int(nkeys);
        let arr = m.get(key);
        if (!(arr instanceof Y.Array) || g.r() < 0.1) { arr = new Y.Array(); m.set(key, arr); }  // overwrite: nested GC
        arrayOp(g, arr, r, seq++);
      }
    });
    gossip(g, docs);
  }
  const updates = docs.map((d) => Y.encodeStateAsUpdate(d));
  const e = expected(updates, { docs: 'map' });
  return { name: `c4_s${seed}_r${nrep}_k${nkeys}`, updates: updates.map(hex), state: e.state, sv: e.sv, json: e.json, diffs: [] };
}

function c5(seed, ndocs) {
  const g = rng(seed);
  const cases = [];
  for (let di = 0; di < ndocs; di++) {
    const nc = 2 + g.int(3);
    const docs = []; for (let i = 0; i < nc; i++) { const d = new Y.Doc(); d.clientID = clientOf(1000 + di * 8 + i); docs.push(d); }
    const snaps = [];
    for (let k = 0; k < 3; k++) {
      docs.forEach((d) => {
        for (let j = 0; j < 1 + g.int(5); j++) {
          if (g.r() < 0.2) d.getMap('ix').set('u' + g.int(10), 'map');
          else if (g.r() < 0.8) d.getMap('users').set('u' + g.int(10), { name: 'n' + g.int(1000), v: g.int(100) });
          else d.getMap('users').delete('u' + g.int(10));
        }
      });
      snaps.push(Y.encodeStateVector(docs[g.int(nc)]));  // a peer's state vector lagging behind
      gossip(g, docs);
    }
    const updates = docs.map((d) => Y.encodeStateAsUpdate(d));
    const e = expected(updates, { ix: 'map', users: 'map' });
    const diffs = snaps.map((sv) => ({ sv: hex(sv), update: hex(canonicalUpdate(Y.encodeStateAsUpdate(e.d, sv))) }));
    cases.push({ name: `c5_s${seed}_doc${di}`, updates: updates.map(hex), state: e.state, sv: e.sv, json: e.json, diffs });
  }
  return cases;
}

function main() {
  const outDir = process.argv[2] || path.join(__dirname, '..');
  const cases = [c3(31, 8, 4, 12), c3(32, 16, 5, 16), c4(41, 6, 20, 4, 15), c4(42, 12, 48, 3, 25), ...c5(51, 60)];
  const f = path.join(outDir, 'configs.json');
  fs.writeFileSync(f, JSON.stringify({ generator: 'tests/golden/gen/gen_config_fixtures.js', yjs: '13.5.16', lib0: '0.2.42', cases }));
  const bytes = cases.reduce((a, c) => a + c.updates.reduce((b, u) => b + u.length / 2, 0), 0);
  console.log(f, cases.length, 'cases', bytes, 'input bytes', fs.statSync(f).size, 'file bytes');
}

main();
