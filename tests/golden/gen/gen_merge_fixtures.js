#!/usr/bin/env node
// Golden vectors for Y.mergeUpdates / Y.diffUpdate (TEST INFRASTRUCTURE ONLY; runs in the build
// container with the in-image Yjs 13.5.16, see load_yjs.js). Inputs are the update lists already
// held by tests/golden/{kat,map,array,nested}.json; for each case it records
//   rev     = mergeUpdates(reversed inputs)          (exercises the reader tie order)
//   pair    = mergeUpdates(first two inputs)
//   diffs[] = diffUpdate(u, sv) for u in {merged, first input} and a few state vectors
// Usage: node gen_merge_fixtures.js <golden_dir>   → <golden_dir>/merge.json
'use strict';
const fs = require('fs');
const path = require('path');
const { loadYjs } = require('./load_yjs.js');

const Y = loadYjs();
const hex = (u) => Buffer.from(u).toString('hex');
const unhex = (h) => new Uint8Array(Buffer.from(h, 'hex'));

function main() {
  const dir = process.argv[2] || path.join(__dirname, '..');
  const out = [];
  for (const set of ['kat', 'map', 'array', 'nested']) {
    const cases = JSON.parse(fs.readFileSync(path.join(dir, set + '.json'))).cases;
    cases.forEach((c, idx) => {
      if (set !== 'kat' && idx % 3 !== 0) return; // keep the fixture small
      const ups = c.updates.map(unhex);
      const merged = Y.mergeUpdates(ups);
      const rec = { name: c.name, set, rev: hex(Y.mergeUpdates(ups.slice().reverse())), diffs: [] };
      if (ups.length >= 2) rec.pair = hex(Y.mergeUpdates(ups.slice(0, 2)));
      const svs = [new Uint8Array([0]), Y.encodeStateVectorFromUpdate(ups[0])];
      if (ups.length >= 2) svs.push(Y.encodeStateVectorFromUpdate(ups[ups.length - 1]));
      for (const sv of svs) {
        rec.diffs.push({ src: 'merged', sv: hex(sv), out: hex(Y.diffUpdate(merged, sv)) });
        rec.diffs.push({ src: 'first', sv: hex(sv), out: hex(Y.diffUpdate(ups[0], sv)) });
      }
      out.push(rec);
    });
  }
  const f = path.join(dir, 'merge.json');
  fs.writeFileSync(f, JSON.stringify({ generator: 'tests/golden/gen/gen_merge_fixtures.js', yjs: '13.5.16', cases: out }));
  console.log(f, out.length, 'cases');
}

main();
