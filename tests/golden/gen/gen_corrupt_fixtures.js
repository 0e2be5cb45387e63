#!/usr/bin/env node
// Corrupted-update fixtures (TEST INFRASTRUCTURE ONLY; runs in the build container against the
// in-image Yjs 13.5.16, never on the GPU box). Valid updates (small ones for the wave decoder,
// larger ones for the chunk path) with one byte overwritten, and truncated; each applied by Yjs to
// a doc that already holds a base update. Recorded: whether Y.applyUpdate threw (and the error
// class), and the doc's canonical state and state vector afterwards (Yjs integrates the struct
// section before it reads the delete set, so a throw there leaves the structs applied).
//
// Usage: node gen_corrupt_fixtures.js <out_dir>  ->  <out_dir>/corrupt.json
'use strict';
const fs = require('fs');
const path = require('path');
const { loadYjs } = require('./load_yjs.js');
const { canonicalUpdate, canonicalSv, hex } = require('./v1.js');

const Y = loadYjs();
const sha = (u) => require('crypto').createHash('sha256').update(Buffer.from(u)).digest('hex');

function mulberry32(a) {
  return function () {
    a |= 0; a = (a + 0x6D2B79F5) | 0;
    let t = Math.imul(a ^ (a >>> 15), 1 | a);
    t = (t + Math.imul(t ^ (t >>> 7), 61 | t)) ^ t;
    return ((t ^ (t >>> 14)) >>> 0) / 4294967296;
  };
}

function snapshot(nClients, perClient, seed) {
  const r = mulberry32(seed);
  const full = new Y.Doc(); full.clientID = 1;
  for (let c = 0; c < nClients; c++) {
    const d = new Y.Doc(); d.clientID = 100 + 13 * c;
    if (c % 3 === 1) Y.applyUpdate(d, Y.encodeStateAsUpdate(full));
    const m = d.getMap('users'); const a = d.getArray('messages');
    for (let i = 0; i < perClient; i++) {
      const k = Math.floor(r() * 3 * perClient);
      const x = r();
      const v = x < 0.4 ? Math.floor(r() * 100000) : x < 0.6 ? 'v' + 'é'.repeat(Math.floor(r() * 4)) + i
        : x < 0.8 ? { n: i, s: 'x' + k, l: [1, 2.5, true, null] } : r() * 1000;
      if (r() < 0.7) m.set('k' + k, v); else a.insert(Math.min(a.length, Math.floor(r() * 3)), [v]);
      if (r() < 0.1 && a.length) a.delete(0, 1);
      if (r() < 0.1) m.delete('k' + Math.floor(r() * 3 * perClient));
    }
    Y.applyUpdate(full, Y.encodeStateAsUpdate(d));
  }
  return Y.encodeStateAsUpdate(full);
}

function apply(base, bad) {
  const d = new Y.Doc(); d.clientID = 5;
  Y.applyUpdate(d, base);
  let threw = null;
  try { Y.applyUpdate(d, bad); } catch (e) { threw = (e && e.constructor && e.constructor.name) + ': ' + String(e.message || e); }
  const raw = Y.encodeStateAsUpdate(d);
  let state = null;
  try { state = sha(canonicalUpdate(raw)); } catch (e) { state = null; }  // Yjs wrote bytes its own reader refuses
  return { threw, state_sha256: state, sv: hex(canonicalSv(Y.encodeStateVector(d))) };
}

const base = (() => { const d = new Y.Doc(); d.clientID = 3; d.getMap('users').set('a', 1); return Y.encodeStateAsUpdate(d); })();
const cases = [];
const sources = [['small', snapshot(12, 6, 8)], ['small2', snapshot(6, 14, 9)], ['large', snapshot(120, 12, 10)]];
const r = mulberry32(77);
const VALS = [0x00, 0x1f, 0x7f, 0x80, 0x84, 0xff, 0xc3, 0xed];
for (const [name, u] of sources) {
  const nByte = name === 'large' ? 90 : 70;
  for (let i = 0; i < nByte; i++) {
    const at = 2 + Math.floor(r() * (u.length - 2));
    const val = VALS[Math.floor(r() * VALS.length)];
    if (u[at] === val) continue;
    const bad = Uint8Array.from(u); bad[at] = val;
    cases.push(Object.assign({ name: `${name}_b${at}_${val}`, src: name, at, val }, apply(base, bad)));
  }
  for (const cut of [7, 40, Math.floor(u.length / 3), Math.floor(u.length / 2), u.length - 3, u.length - 1]) {
    const bad = u.subarray(0, cut);
    cases.push(Object.assign({ name: `${name}_cut${cut}`, src: name, cut }, apply(base, bad)));
  }
}
const outDir = process.argv[2] || path.join(__dirname, '..');
const srcs = {};
for (const [n, u] of sources) srcs[n] = hex(u);
fs.writeFileSync(path.join(outDir, 'corrupt.json'), JSON.stringify({ yjs: '13.5.16', base: hex(base), sources: srcs, cases }));
const kinds = {};
for (const c of cases) { const k = c.threw ? c.threw.split(':')[0] + ':' + c.threw.split(':')[1].slice(0, 24) : 'ok'; kinds[k] = (kinds[k] || 0) + 1; }
console.log(`corrupt.json: ${cases.length} cases`, JSON.stringify(kinds));
console.log('sizes', sources.map(([n, u]) => n + ':' + u.length).join(' '));
