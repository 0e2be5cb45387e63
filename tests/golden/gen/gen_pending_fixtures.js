#!/usr/bin/env node
// Pending-struct fixture generator (TEST INFRASTRUCTURE ONLY; runs in the build container, never
// on the GPU box). Yjs's Y.applyUpdate never throws on missing dependencies: it parks the structs
// (store.pendingStructs + a `missing` state vector) and the delete-set ranges it cannot apply
// (store.pendingDs), retries them when a later update advances a missing client, and
// encodeStateAsUpdate emits them merged in (Y@21330 readUpdateV2, Y@22155 encodeStateAsUpdateV2).
// This script applies seeded replica deltas to a fresh Yjs 13.5.16 doc in NON-causal orders and
// records, after every apply (a "checkpoint"), what a reader of the doc observes:
//   state_raw / sv_raw  (13.5.16 insertion-order bytes), state / sv (13.6 canonical order),
//   a delta against a replica state vector, whether structs / delete ranges are pending, toJSON.
//
// Usage: node gen_pending_fixtures.js <out_dir>   → <out_dir>/pending.json
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
function makeRng(seed) {
  const r = mulberry32(seed);
  const int = (n) => Math.floor(r() * n);
  const pick = (a) => a[int(a.length)];
  return { r, int, pick };
}
function newDoc(client) { const d = new Y.Doc(); d.clientID = client; return d; }
const av = (v) => (v === undefined ? null : v);
function randValue(g) {
  const k = g.int(6);
  if (k === 0) return g.int(1000);
  if (k === 1) return 's' + g.int(100000);
  if (k === 2) return { name: 'n' + g.int(50) };
  if (k === 3) return g.pick([true, false, null]);
  if (k === 4) return 'Ünï 😀' + g.int(9);
  return [g.int(10), 'x'];
}

// one reader-visible snapshot of doc m
function snapshot(m, roots, svDocs, g) {
  const st = Y.encodeStateAsUpdate(m);
  const sv = Y.encodeStateVector(m);
  const snap = {
    state_raw: hex(st), state: hex(canonicalUpdate(st)),
    sv_raw: hex(sv), sv: hex(canonicalSv(sv)),
    pending: m.store.pendingStructs !== null, pending_ds: m.store.pendingDs !== null,
  };
  if (svDocs.length) {
    const tsv = svDocs[g.int(svDocs.length)];
    const d = Y.encodeStateAsUpdate(m, tsv);
    snap.delta = { sv: hex(tsv), update_raw: hex(d), update: hex(canonicalUpdate(d)) };
  }
  const json = {};
  for (const [rname, kind] of Object.entries(roots)) json[rname] = kind === 'map' ? m.getMap(rname).toJSON() : m.getArray(rname).toJSON();
  snap.json = JSON.parse(JSON.stringify(json));
  return snap;
}

// seeded replicas exchanging deltas; returns the per-(round, replica) deltas in causal order plus
// a few replica state vectors taken along the way
function history(seed, kind) {
  const g = makeRng(seed);
  const nRep = 2 + g.int(4);
  const rounds = 2 + g.int(4);
  const ops = 1 + g.int(5);
  const nKeys = 1 + g.int(6);
  const docs = [];
  const used = new Set();
  for (let i = 0; i < nRep; i++) {
    let c; do { c = g.pick([i + 1, 100 + 37 * i, (g.int(2 ** 31) + 1) >>> 0, 20000 + g.int(1 << 20)]); } while (used.has(c) || c === 0);
    used.add(c); docs.push(newDoc(c));
  }
  const roots = kind === 'array' ? { messages: 'array' } : kind === 'nested' ? { docs: 'map' } : { users: 'map' };
  const log = [];
  const svs = [];
  for (let rd = 0; rd < rounds; rd++) {
    for (const d of docs) {
      const before = Y.encodeStateVector(d);
      for (let o = 0; o < ops; o++) {
        if (kind === 'map') {
          const m = d.getMap('users'); const key = 'user' + g.int(nKeys);
          if (g.r() < 0.75) m.set(key, randValue(g)); else m.delete(key);
        } else if (kind === 'array') {
          const a = d.getArray('messages'); const x = g.r(); const len = a.length;
          if (x < 0.35) a.push([av(randValue(g)), av(randValue(g))].slice(0, 1 + g.int(2)));
          else if (x < 0.5) a.unshift([av(randValue(g))]);
          else if (x < 0.8) a.insert(g.int(len + 1), [av(randValue(g))]);
          else if (len > 0) { const p = g.int(len); a.delete(p, Math.min(len - p, 1 + g.int(2))); }
        } else {
          const m = d.getMap('docs'); const key = 'doc' + g.int(nKeys); const x = g.r();
          const cur = m.get(key);
          if (x < 0.25 || !(cur instanceof Y.Array)) { if (g.r() < 0.6) { const arr = new Y.Array(); m.set(key, arr); arr.push([av(randValue(g))]); } else m.set(key, randValue(g)); } else if (x < 0.8) { const L = cur.length; if (L === 0 || g.r() < 0.7) cur.insert(g.int(L + 1), [av(randValue(g))]); else cur.delete(g.int(L), 1); } else m.delete(key);
        }
      }
      log.push(Y.encodeStateAsUpdate(d, before));
    }
    for (const d of docs) {
      if (g.r() < 0.6) {
        const p = g.pick(docs);
        if (p !== d) Y.applyUpdate(d, Y.encodeStateAsUpdate(p, Y.encodeStateVector(d)));
      }
      if (g.r() < 0.3) svs.push(Y.encodeStateVector(d));
    }
  }
  svs.push(new Uint8Array([0]));
  return { g, log, roots, svs, full: docs.map((d) => Y.encodeStateAsUpdate(d)) };
}

function shuffle(g, a) {
  const b = a.slice();
  for (let i = b.length - 1; i > 0; i--) { const j = g.int(i + 1); [b[i], b[j]] = [b[j], b[i]]; }
  return b;
}

// applies `updates` one at a time to a fresh doc; a snapshot after every apply
function runCase(name, updates, roots, svs, g) {
  const m = newDoc(0x7ffffff0);
  const steps = [];
  for (const u of updates) {
    Y.applyUpdate(m, u);
    steps.push(snapshot(m, roots, svs, g));
  }
  return { name, roots, updates: updates.map(hex), steps };
}

function kats() {
  const out = [];
  const none = [];
  const g = makeRng(7);
  { // client 3 edits twice; the second delta arrives first (a clock gap)
    const a = newDoc(3); const m = a.getMap('m');
    m.set('x', 1); const u1 = Y.encodeStateAsUpdate(a);
    const sv = Y.encodeStateVector(a); m.set('y', 2); m.set('x', 3); const u2 = Y.encodeStateAsUpdate(a, sv);
    out.push(runCase('kat_gap', [u2, u1], { m: 'map' }, none, g));
    out.push(runCase('kat_gap_dup', [u2, u2, u1, u2], { m: 'map' }, none, g));
  }
  { // client 9's entry has client 5's entry as origin; 9 arrives first (a missing origin)
    const a = newDoc(5); const b = newDoc(9);
    a.getMap('m').set('k', 'A'); const ua = Y.encodeStateAsUpdate(a);
    Y.applyUpdate(b, ua); b.getMap('m').set('k', 'B'); const ub = Y.encodeStateAsUpdate(b, Y.encodeStateVector(a));
    out.push(runCase('kat_missing_origin', [ub, ua], { m: 'map' }, none, g));
  }
  { // a delete of items the receiver has not seen yet (pendingDs), then the items
    const a = newDoc(4); const arr = a.getArray('l');
    arr.push(['a', 'b', 'c']); const u1 = Y.encodeStateAsUpdate(a);
    const sv = Y.encodeStateVector(a); arr.delete(1, 1); const u2 = Y.encodeStateAsUpdate(a, sv);
    out.push(runCase('kat_pending_ds', [u2, u1], { l: 'array' }, none, g));
    // a delete of another client's items, applied before them
    const b = newDoc(8); Y.applyUpdate(b, u1); b.getArray('l').delete(0, 2);
    const ub = Y.encodeStateAsUpdate(b, Y.encodeStateVector(a));
    out.push(runCase('kat_pending_ds_other', [ub, u1], { l: 'array' }, none, g));
  }
  { // three generations; the last arrives first, then the first, then the middle one
    const a = newDoc(11); const arr = a.getArray('l');
    const ups = [];
    for (let i = 0; i < 3; i++) { const sv = Y.encodeStateVector(a); arr.insert(i === 1 ? 0 : arr.length, ['v' + i]); ups.push(Y.encodeStateAsUpdate(a, sv)); }
    out.push(runCase('kat_chain', [ups[2], ups[0], ups[1]], { l: 'array' }, none, g));
    out.push(runCase('kat_chain_never', [ups[2], ups[1]], { l: 'array' }, [Y.encodeStateVector(a)], g));
  }
  return out;
}

function main() {
  const outDir = process.argv[2] || path.join(__dirname, '..');
  const cases = kats();
  let seed = 5000;
  for (const kind of ['map', 'array', 'nested']) {
    for (let k = 0; k < 14; k++) {
      const h = history(++seed, kind);
      // non-causal permutations of the per-round deltas
      cases.push(runCase(`${kind}_shuffled_${seed}`, shuffle(h.g, h.log), h.roots, h.svs, h.g));
      // reversed deltas: everything pends until the first round arrives last
      if (k % 3 === 0) cases.push(runCase(`${kind}_reversed_${seed}`, h.log.slice().reverse(), h.roots, h.svs, h.g));
      // a lost delta: the rest stays pending for good
      if (k % 3 === 1 && h.log.length > 2) {
        const drop = 1 + h.g.int(h.log.length - 1);
        cases.push(runCase(`${kind}_lost_${seed}`, shuffle(h.g, h.log.filter((_, i) => i !== drop)), h.roots, h.svs, h.g));
      }
    }
  }
  const f = path.join(outDir, 'pending.json');
  fs.writeFileSync(f, JSON.stringify({ generator: 'tests/golden/gen/gen_pending_fixtures.js', yjs: '13.5.16', lib0: '0.2.42', cases }));
  let steps = 0; let pend = 0;
  for (const c of cases) for (const s of c.steps) { steps++; if (s.pending || s.pending_ds) pend++; }
  console.log(f, cases.length, 'cases', steps, 'checkpoints', pend, 'with pending');
}

main();
