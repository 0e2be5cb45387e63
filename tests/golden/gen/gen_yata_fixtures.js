#!/usr/bin/env node
// Many-replica YArray fixtures (TEST INFRASTRUCTURE ONLY; runs in the build container, never on
// the GPU box): 64-256 replicas of BASELINE.json config C3's op mix (push / unshift / insert /
// cut on YArray 'messages') with gossip rounds, played through the in-image Yjs 13.5.16. The
// inputs are every replica's local-transaction updates (doc.on('update'), the wire deltas crdt.js
// broadcasts); the expected output is a Yjs doc that applied them all (canonical 13.6 order).
// This pins the parallel YATA (origin-tree pre-order, yc_yata.hip) where sibling groups are large.
//
// Usage: node gen_yata_fixtures.js <out_dir>  ->  <out_dir>/yata.json
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
  return { r, int: (n) => Math.floor(r() * n) };
}
const clientOf = (i) => (((i + 1) * 2654435761) >>> 0) || 1;

function run(seed, nrep, rounds, ops, pUnshift) {
  const g = rng(seed);
  const docs = [];
  const wire = [];
  for (let i = 0; i < nrep; i++) {
    const d = new Y.Doc(); d.clientID = clientOf(i);
    d.on('update', (u, origin, doc, tr) => { if (tr.local) wire.push(u); });
    docs.push(d);
  }
  let seq = 0;
  for (let k = 0; k < rounds; k++) {
    docs.forEach((d, r) => {
      const arr = d.getArray('messages');
      for (let j = 0; j < ops; j++) {
        const L = arr.length; const x = g.r();
        const vals = []; const n = 1 + g.int(4);
        for (let i = 0; i < n; i++) vals.push(g.r() < 0.6 ? `m${r}_${seq}_${i}` : g.int(1 << 20));
        seq++;
        if (x < 0.4 - pUnshift / 2 || L === 0) arr.push(vals);
        else if (x < 0.4 + pUnshift / 2) arr.unshift([vals[0]]);
        else if (x < 0.85) arr.insert(g.int(L + 1), vals);
        else { const i = g.int(L); arr.delete(i, Math.min(L - i, 1 + g.int(3))); }
      }
    });
    for (let i = 0; i < docs.length; i++) {  // gossip: every replica pulls a delta from a random peer
      const p = g.int(docs.length);
      if (p !== i) Y.applyUpdate(docs[i], Y.encodeStateAsUpdate(docs[p], Y.encodeStateVector(docs[i])));
    }
  }
  const m = new Y.Doc(); m.clientID = 0x7ffffff0;
  for (const u of wire) Y.applyUpdate(m, u);
  return {
    name: `yata_s${seed}_r${nrep}`, replicas: nrep, updates: wire.map(hex),
    state: hex(canonicalUpdate(Y.encodeStateAsUpdate(m))), sv: hex(canonicalSv(Y.encodeStateVector(m))),
    json: { messages: m.getArray('messages').toJSON() },
  };
}

function main() {
  const outDir = process.argv[2] || path.join(__dirname, '..');
  const cases = [];
  const t0 = Date.now();
  cases.push(run(64001, 64, 4, 6, 0.15));
  cases.push(run(64002, 64, 3, 8, 0.4));    // unshift-heavy: large root sibling groups
  cases.push(run(96001, 96, 3, 5, 0.15));
  cases.push(run(128001, 128, 3, 4, 0.15));
  cases.push(run(128002, 128, 2, 6, 0.5));
  cases.push(run(256001, 256, 2, 3, 0.15));
  const f = path.join(outDir, 'yata.json');
  fs.writeFileSync(f, JSON.stringify({ generator: 'tests/golden/gen/gen_yata_fixtures.js', yjs: '13.5.16', cases }));
  console.log(f, cases.map((c) => `${c.name}: ${c.updates.length} updates, ${c.json.messages.length} items`).join('; '), `${(Date.now() - t0) / 1e3}s`);
}

main();
