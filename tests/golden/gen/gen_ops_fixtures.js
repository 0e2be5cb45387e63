#!/usr/bin/env node
// Local-op golden fixtures (TEST INFRASTRUCTURE ONLY; runs in the build container, never on the
// GPU box). Drives the in-image Yjs 13.5.16 through seeded scripts of the ops @ypear/crdt performs
// on its doc (crdt.js:369-611): YMap.set / delete on root maps, set(key, new Y.Array()) and
// push / unshift / insert / delete on the nested arrays, the same on a root YArray, interleaved
// with remote updates from a concurrent replica. After every step it records the doc's canonical
// encodeStateAsUpdate, and at the end toJSON of every root.
//
// Values are recorded as lib0 `any` encodings produced by writeAny below, which restates lib0
// 0.2.42 writeAny (L0@8251); every value is cross-checked against the bytes Yjs itself writes.
//
// -(2 ** 40) is not drawn: lib0 0.2.42 writeVarInt shifts with `>>>=` (32 bits) and writes a
// continuation byte with nothing after it, an update Yjs itself cannot read back.
//
// Usage: node gen_ops_fixtures.js <out_dir>   ->  <out_dir>/ops.json
'use strict';
const fs = require('fs');
const path = require('path');
const { loadYjs } = require('./load_yjs.js');
const { canonicalUpdate, writeVu, hex } = require('./v1.js');

const Y = loadYjs();

function mulberry32(a) {
  return function () {
    a |= 0; a = (a + 0x6D2B79F5) | 0;
    let t = Math.imul(a ^ (a >>> 15), 1 | a);
    t = (t + Math.imul(t ^ (t >>> 7), 61 | t)) ^ t;
    return ((t ^ (t >>> 14)) >>> 0) / 4294967296;
  };
}
function makeRng(seed) {
  const r = mulberry32(seed);
  const int = (n) => Math.floor(r() * n);
  const pick = (a) => a[int(a.length)];
  return { r, int, pick };
}

// ---- lib0 writeAny restated (tag 127..116)
function pushVu(o, n) { writeVu(o, n); }
function pushStr(o, s) { const b = Buffer.from(s, 'utf8'); pushVu(o, b.length); for (const x of b) o.push(x); }
function pushVi(o, num) {
  let neg = num < 0 || Object.is(num, -0);
  if (neg) num = -num;
  o.push((num > 63 ? 0x80 : 0) | (neg ? 0x40 : 0) | (num & 63));
  num >>>= 6;
  while (num > 0) { o.push((num > 127 ? 0x80 : 0) | (num & 127)); num >>>= 7; }
}
const f32 = new DataView(new ArrayBuffer(4));
function writeAny(o, v) {
  switch (typeof v) {
    case 'string': o.push(119); pushStr(o, v); return;
    case 'number':
      if (Number.isInteger(v) && v <= 0x7fffffff) { o.push(125); pushVi(o, v); return; }
      f32.setFloat32(0, v);
      if (f32.getFloat32(0) === v) { o.push(124); for (let i = 0; i < 4; i++) o.push(f32.getUint8(i)); return; }
      { const d = new DataView(new ArrayBuffer(8)); d.setFloat64(0, v); o.push(123); for (let i = 0; i < 8; i++) o.push(d.getUint8(i)); }
      return;
    case 'boolean': o.push(v ? 120 : 121); return;
    case 'object':
      if (v === null) { o.push(126); return; }
      if (Array.isArray(v)) { o.push(117); pushVu(o, v.length); for (const e of v) writeAny(o, e); return; }
      if (v instanceof Uint8Array) { o.push(116); pushVu(o, v.length); for (const x of v) o.push(x); return; }
      { const ks = Object.keys(v); o.push(118); pushVu(o, ks.length); for (const k of ks) { pushStr(o, k); writeAny(o, v[k]); } }
      return;
    default: o.push(127);
  }
}
function anyHex(v) { const o = []; writeAny(o, v); return Buffer.from(o).toString('hex'); }

// cross-check against Yjs: a fresh doc pushing [v] into root array 'x' writes exactly this update
function checkAny(v) {
  const d = new Y.Doc(); d.clientID = 1;
  d.getArray('x').push([v]);
  const o = [1, 1, 1, 0, 8, 1]; pushStr(o, 'x'); o.push(1); writeAny(o, v); o.push(0);
  const want = Buffer.from(o).toString('hex');
  const got = hex(Y.encodeStateAsUpdate(d));
  if (got !== want) throw new Error('writeAny mismatch for ' + JSON.stringify(v) + ': ' + got + ' vs ' + want);
}

const STRS = ['', 'a', 'hello', 'Ünïcødé', '日本語', 'emoji 😀', 'tab\tnl\n"q"\\'];
function randValue(g, depth = 0) {
  switch (g.int(depth > 1 ? 8 : 10)) {
    case 0: return g.int(100);
    case 1: return -g.int(100000);
    case 2: return g.pick([0, 63, 64, 8191, 8192, 2147483647, -2147483647, 2147483648, 2 ** 40, -(2 ** 31)]);
    case 3: return g.pick([1.5, -0.25, 3.14159, 1e300, 0.1]);
    case 4: return g.pick(STRS) + g.int(1000);
    case 5: return g.r() < 0.5;
    case 6: return null;
    case 7: return 'v' + g.int(100000);
    case 8: { const o = {}; const n = g.int(4); for (let i = 0; i < n; i++) o[g.pick(['name', 'v', 'k' + g.int(5)])] = randValue(g, depth + 1); return o; }
    default: { const a = []; const n = g.int(4); for (let i = 0; i < n; i++) a.push(randValue(g, depth + 1)); return a; }
  }
}

function randClient(g) { return g.pick([() => 1 + g.int(50), () => 20000 + g.int(1 << 20), () => (g.int(2 ** 31) + 1) >>> 0])(); }

function script(seed, nested) {
  const g = makeRng(seed);
  const a = new Y.Doc(); a.clientID = randClient(g);
  const b = new Y.Doc(); do { b.clientID = randClient(g); } while (b.clientID === a.clientID);
  const steps = [];
  const state = () => hex(canonicalUpdate(Y.encodeStateAsUpdate(a)));
  const nOps = 12 + g.int(24);
  // one random op on doc d; returns the op record (only recorded for `a`)
  const randomOp = (d) => {
    const x = g.r();
    const users = d.getMap('users'); const msgs = d.getArray('messages');
    if (x < 0.25) {
      const key = 'k' + g.int(6); const v = randValue(g); checkAny(v === undefined ? null : v);
      users.set(key, v); return { op: 'map_set', root: 'users', key, any: anyHex(v) };
    } else if (x < 0.33) {
      const key = 'k' + g.int(6); users.delete(key); return { op: 'map_delete', root: 'users', key };
    } else if (nested && x < 0.4) {
      const key = 'list' + g.int(3); users.set(key, new Y.Array()); return { op: 'map_set_type', root: 'users', key, type: 0 };
    } else if (nested && x < 0.6) {
      const key = 'list' + g.int(3); const arr = users.get(key);
      if (!(arr instanceof Y.Array)) { users.set(key, new Y.Array()); return { op: 'map_set_type', root: 'users', key, type: 0 }; }
      return arrayOp(arr, 'users', key);
    }
    return arrayOp(msgs, 'messages', null);
  };
  const arrayOp = (arr, root, pkey) => {
    const L = arr.length; const y = g.r();
    if (y < 0.7 || L === 0) {
      const n = 1 + g.int(3); const vs = []; for (let i = 0; i < n; i++) { const v = randValue(g); checkAny(v); vs.push(v); }
      const z = g.r(); let index;
      if (z < 0.4) { index = L; arr.push(vs); } else if (z < 0.6) { index = 0; arr.unshift(vs); } else { index = g.int(L + 1); arr.insert(index, vs); }
      return { op: 'array_insert', root, parent_key: pkey, index, anys: vs.map(anyHex) };
    }
    const index = g.int(L); const length = 1 + g.int(Math.min(3, L - index));
    arr.delete(index, length);
    return { op: 'array_delete', root, parent_key: pkey, index, length };
  };
  for (let i = 0; i < nOps; i++) {
    if (g.r() < 0.2) {  // a concurrent replica edits, then its delta arrives
      const sv = Y.encodeStateVector(a);
      const k = 1 + g.int(3);
      for (let j = 0; j < k; j++) randomOp(b);
      const u = Y.encodeStateAsUpdate(b, sv);
      try { Y.applyUpdate(a, u); } catch (e) { console.error('apply failed', seed, hex(u)); throw e; }
      steps.push({ op: 'apply', update: hex(u), state: state() });
      if (g.r() < 0.5) Y.applyUpdate(b, Y.encodeStateAsUpdate(a, Y.encodeStateVector(b)));
      continue;
    }
    const rec = randomOp(a);
    rec.state = state();
    steps.push(rec);
  }
  return {
    name: (nested ? 'ops_' : 'ops_root_') + seed,
    client: a.clientID,
    steps,
    json: JSON.parse(JSON.stringify({ users: a.getMap('users').toJSON(), messages: a.getArray('messages').toJSON() })),
  };
}

function main() {
  const outDir = process.argv[2] || path.join(__dirname, '..');
  const cases = [];
  for (let s = 1; s <= 40; s++) cases.push(script(5000 + s, true));
  for (let s = 1; s <= 20; s++) cases.push(script(6000 + s, false));  // root types only (oracle-replayable)
  const f = path.join(outDir, 'ops.json');
  fs.writeFileSync(f, JSON.stringify({ generator: 'tests/golden/gen/gen_ops_fixtures.js', yjs: '13.5.16', lib0: '0.2.42', cases }));
  console.log(f, cases.length, 'cases', cases.reduce((a, c) => a + c.steps.length, 0), 'steps');
}

main();
