#!/usr/bin/env node
// Golden-fixture generator (TEST INFRASTRUCTURE ONLY; runs in the build container, never on the
// GPU box). Drives the in-image Yjs 13.5.16 (see load_yjs.js) through seeded random histories and
// records, per case: the input updates, the merged doc's encodeStateAsUpdate / encodeStateVector,
// Y.mergeUpdates of the inputs, state-vector deltas and toJSON of every root type.
//
// Usage: node gen_fixtures.js <out_dir>
// Output: <out_dir>/{kat,map,array,nested}.json  (hex-encoded bytes, see tests/golden/README.md)
'use strict';
const fs = require('fs');
const path = require('path');
const { loadYjs } = require('./load_yjs.js');
const { canonicalUpdate, canonicalSv, updateStats, hex } = require('./v1.js');

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

const STRS = ['', 'a', 'hello', 'Ünïcødé', '日本語テキスト', 'emoji 😀🎉', 'x'.repeat(200), 'tab\tnl\n"q"'];

function randValue(g, depth = 0) {
  const k = g.int(depth > 1 ? 9 : 11);
  switch (k) {
    case 0: return g.int(100);
    case 1: return -g.int(100000);
    case 2: return g.pick([0, 1, 63, 64, 127, 128, 8191, 8192, 2147483647, -2147483647, 2147483648, 2 ** 40, 2 ** 53 - 1]);
    case 3: return g.pick([1.5, -0.25, 3.14159, 1e300, -1e-300, 0.1]);
    case 4: return g.pick(STRS) + (g.r() < 0.5 ? String(g.int(1000)) : '');
    case 5: return g.pick([true, false]);
    case 6: return null;
    case 7: return g.r() < 0.3 ? undefined : 'u' + g.int(50);
    case 8: return 'v' + g.int(100000);
    case 9: { const o = {}; const n = g.int(4); for (let i = 0; i < n; i++) o[g.pick(['name', 'v', 'k' + g.int(5), '1', '0b'])] = randValue(g, depth + 1); return o; }
    default: { const a = []; const n = g.int(4); for (let i = 0; i < n; i++) a.push(randValue(g, depth + 1)); return a; }
  }
}

const av = (v) => (v === undefined ? null : v); // YArray.insert rejects undefined (Y@47498)

function randClient(g, i) {
  // exercise 1..5-byte varuints; clientIDs are uint32
  const styles = [() => i + 1, () => 100 + i * 37, () => 20000 + g.int(1 << 20), () => ((i + 1) * 2654435761) >>> 0, () => (g.int(2 ** 31) + 1) >>> 0];
  return g.pick(styles)();
}

function newDoc(client) {
  const d = new Y.Doc();
  d.clientID = client;
  return d;
}

function finishCase(name, updates, roots, extra = {}) {
  // reference merge: a fresh doc applying every input update in order
  const m = newDoc(0x7ffffff0);
  for (const u of updates) Y.applyUpdate(m, u);
  const state = Y.encodeStateAsUpdate(m);
  // order-independence check (SURVEY.md §4.7): reverse order must give identical canonical bytes
  if (!extra.noReverse) {
    const m2 = newDoc(0x7ffffff1);
    for (let i = updates.length - 1; i >= 0; i--) Y.applyUpdate(m2, updates[i]);
    const s2 = Y.encodeStateAsUpdate(m2);
    if (hex(canonicalUpdate(s2)) !== hex(canonicalUpdate(state))) throw new Error(name + ': order dependence');
    const m3 = newDoc(0x7ffffff2);
    Y.applyUpdate(m3, Y.mergeUpdates(updates));
    if (hex(canonicalUpdate(Y.encodeStateAsUpdate(m3))) !== hex(canonicalUpdate(state))) throw new Error(name + ': mergeUpdates apply mismatch');
  }
  const sv = Y.encodeStateVector(m);
  const merged = Y.mergeUpdates(updates);
  const json = {};
  for (const [rname, kind] of Object.entries(roots)) {
    json[rname] = kind === 'map' ? m.getMap(rname).toJSON() : m.getArray(rname).toJSON();
  }
  const diffs = [];
  for (const d of extra.svDocs || []) {
    const s = Y.encodeStateVector(d);
    diffs.push({ sv: hex(s), update: hex(canonicalUpdate(Y.encodeStateAsUpdate(m, s))) });
  }
  // an empty / partial target SV as well
  diffs.push({ sv: '00', update: hex(canonicalUpdate(Y.encodeStateAsUpdate(m, new Uint8Array([0])))) });
  let items = 0;
  for (const u of updates) items += updateStats(u).items;
  return {
    name,
    roots,
    updates: updates.map(hex),
    items,
    state: hex(canonicalUpdate(state)),
    state_raw: hex(state),
    sv: hex(canonicalSv(sv)),
    sv_raw: hex(sv),
    merged: hex(canonicalUpdate(merged)),
    merged_raw: hex(merged),
    diffs,
    json: JSON.parse(JSON.stringify(json)),
  };
}

// ---------------------------------------------------------------- KATs (SURVEY.md App. A.6)
function katCases() {
  const out = [];
  { const d = newDoc(1); out.push(finishCase('kat_empty', [Y.encodeStateAsUpdate(d)], {})); }
  { const d = newDoc(1); d.getMap('users').set('user1', { name: 'Alice' }); out.push(finishCase('kat_alice', [Y.encodeStateAsUpdate(d)], { users: 'map' })); }
  {
    const a = newDoc(5); const b = newDoc(9);
    a.getMap('m').set('k', 'A'); b.getMap('m').set('k', 'B');
    out.push(finishCase('kat_concurrent', [Y.encodeStateAsUpdate(a), Y.encodeStateAsUpdate(b)], { m: 'map' }, { svDocs: [a, b] }));
  }
  { const d = newDoc(3); const m = d.getMap('u'); for (let i = 0; i < 5; i++) m.set('x', i); out.push(finishCase('kat_overwrite', [Y.encodeStateAsUpdate(d)], { u: 'map' })); }
  { const d = newDoc(3); const m = d.getMap('u'); for (let i = 0; i < 5; i++) m.set('x', i); m.delete('x'); out.push(finishCase('kat_overwrite_delete', [Y.encodeStateAsUpdate(d)], { u: 'map' })); }
  {
    const d = newDoc(7); const a = d.getArray('messages');
    a.push(['Hello']); a.push(['W']); a.unshift(['first']); a.insert(1, ['x', 'y']); a.delete(0, 1);
    out.push(finishCase('kat_array', [Y.encodeStateAsUpdate(d)], { messages: 'array' }));
  }
  {
    const d = newDoc(7); const m = d.getMap('users'); const l = new Y.Array();
    m.set('list', l); l.push(['a', 'b']); l.insert(1, ['c']);
    out.push(finishCase('kat_nested', [Y.encodeStateAsUpdate(d)], { users: 'map' }));
    m.set('list', 'gone');
    out.push(finishCase('kat_nested_gc', [Y.encodeStateAsUpdate(d)], { users: 'map' }));
  }
  {
    const a = newDoc(1); const m = a.getMap('m'); m.set('y', 1);
    const sv = Y.encodeStateVector(a); m.set('x', 2);
    const c = finishCase('kat_delta', [Y.encodeStateAsUpdate(a)], { m: 'map' });
    c.diffs.push({ sv: hex(sv), update: hex(canonicalUpdate(Y.encodeStateAsUpdate(a, sv))) });
    out.push(c);
  }
  { const d = newDoc(1); d.getArray('a').push([1, 'x', true, null, 1.5, -3, { k: [2] }]); out.push(finishCase('kat_any', [Y.encodeStateAsUpdate(d)], { a: 'array' })); }
  { const d = newDoc(300); const m = d.getMap('m'); m.set('k', 2 ** 31); m.set('j', 2 ** 40); m.set('n', -(2 ** 31) + 1); out.push(finishCase('kat_ints', [Y.encodeStateAsUpdate(d)], { m: 'map' })); }
  { const d = newDoc(12); const m = d.getMap('m'); m.set('bin', new Uint8Array([1, 2, 3, 250])); m.set('u', undefined); out.push(finishCase('kat_binary', [Y.encodeStateAsUpdate(d)], { m: 'map' })); }
  return out;
}

// ---------------------------------------------------------------- random histories
function randomHistory(seed, kind) {
  const g = makeRng(seed);
  const nRep = 2 + g.int(kind === 'map' ? 7 : 5);
  const rounds = 1 + g.int(6);
  const opsPerRound = 1 + g.int(kind === 'map' ? 12 : 8);
  const nKeys = 1 + g.int(12);
  const gossip = g.r();
  const used = new Set();
  const docs = [];
  for (let i = 0; i < nRep; i++) {
    let c; do { c = randClient(g, i); } while (used.has(c) || c === 0);
    used.add(c); docs.push(newDoc(c));
  }
  const roots = kind === 'array' ? { messages: 'array', ix: 'map' } : { users: 'map', ix: 'map' };
  if (kind === 'nested') roots.docs = 'map';
  const log = []; // per-round deltas in causal order
  for (let rd = 0; rd < rounds; rd++) {
    for (const d of docs) {
      const before = Y.encodeStateVector(d);
      for (let o = 0; o < opsPerRound; o++) {
        if (kind === 'map') {
          const m = d.getMap('users'); const key = 'user' + g.int(nKeys);
          const x = g.r();
          if (x < 0.7) m.set(key, randValue(g));
          else if (x < 0.9) m.delete(key);
          else if (x < 0.95) m.set(key, new Uint8Array([g.int(256), g.int(256)]));
          else d.getMap('ix').set('users', 'map');
        } else if (kind === 'array') {
          const a = d.getArray('messages'); const x = g.r(); const len = a.length;
          if (x < 0.35) { const n = 1 + g.int(3); const v = []; for (let i = 0; i < n; i++) v.push(av(randValue(g))); a.push(v); } else if (x < 0.5) { a.unshift([av(randValue(g))]); } else if (x < 0.75) { const v = []; const n = 1 + g.int(4); for (let i = 0; i < n; i++) v.push(av(randValue(g))); a.insert(g.int(len + 1), v); } else if (x < 0.8) { a.insert(g.int(len + 1), [new Uint8Array([g.int(256)])]); } else if (len > 0) { const p = g.int(len); a.delete(p, Math.min(len - p, 1 + g.int(3))); }
          if (g.r() < 0.05) d.getMap('ix').set('messages', 'array');
        } else { // nested: arrays and maps inside map entries, overwritten / deleted later
          const m = d.getMap('docs'); const key = 'doc' + g.int(nKeys); const x = g.r();
          if (x < 0.2) { const arr = new Y.Array(); m.set(key, arr); arr.push([av(randValue(g))]); } else if (x < 0.5) {
            const cur = m.get(key);
            if (cur instanceof Y.Array) { const L = cur.length; const y = g.r(); if (y < 0.6 || L === 0) cur.insert(g.int(L + 1), [av(randValue(g)), av(randValue(g))].slice(0, 1 + g.int(2))); else cur.delete(g.int(L), 1); } else if (cur instanceof Y.Map) { cur.set('f' + g.int(4), randValue(g)); } else { m.set(key, randValue(g)); }
          } else if (x < 0.6) { const mm = new Y.Map(); m.set(key, mm); mm.set('f0', randValue(g)); } else if (x < 0.8) { m.set(key, randValue(g)); } else if (x < 0.9) { m.delete(key); } else { d.getMap('users').set('u' + g.int(3), randValue(g)); }
        }
      }
      const delta = Y.encodeStateAsUpdate(d, before);
      log.push(delta);
    }
    // partial gossip: some replicas pull a delta from a random peer
    for (const d of docs) {
      if (g.r() < gossip) {
        const p = g.pick(docs);
        if (p !== d) {
          const u = Y.encodeStateAsUpdate(p, Y.encodeStateVector(d));
          Y.applyUpdate(d, u);
        }
      }
    }
  }
  const full = docs.map((d) => Y.encodeStateAsUpdate(d));
  const cFull = finishCase(`${kind}_full_${seed}`, full, roots, { svDocs: docs.slice(0, 3) });
  const cLog = finishCase(`${kind}_log_${seed}`, log, roots, { noReverse: true });
  return [cFull, cLog];
}

function main() {
  const outDir = process.argv[2] || path.join(__dirname, '..');
  const sets = { kat: katCases(), map: [], array: [], nested: [] };
  for (let s = 1; s <= 40; s++) sets.map.push(...randomHistory(1000 + s, 'map'));
  for (let s = 1; s <= 30; s++) sets.array.push(...randomHistory(2000 + s, 'array'));
  for (let s = 1; s <= 25; s++) sets.nested.push(...randomHistory(3000 + s, 'nested'));
  for (const [k, v] of Object.entries(sets)) {
    const f = path.join(outDir, `${k}.json`);
    fs.writeFileSync(f, JSON.stringify({ generator: 'tests/golden/gen/gen_fixtures.js', yjs: '13.5.16', lib0: '0.2.42', cases: v }));
    console.log(f, v.length, 'cases');
  }
}

main();
