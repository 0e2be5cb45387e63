#!/usr/bin/env node
// YMap entries whose items carry right origins (TEST INFRASTRUCTURE ONLY; runs in the build
// container against the in-image Yjs 13.5.16). typeMapSet never writes a right origin, but Yjs's
// reader and Item.integrate (Y@77594) take them: a map entry's items form a YATA list like a YArray
// (the list starts at the entry's leftmost item), the last one is the value, every other is deleted.
// The histories are real YATA histories: replicas insert into a YArray 'm' at random positions
// (single values: a map entry item of several values splits into pieces Yjs leaves undeleted, an
// order-dependent state), sync partially, delete
// now and then; then every update is REWRITTEN so that the list's root items name the YMap 'users'
// with parentSub key 'k' instead of the root array 'm' (items with an origin or right origin carry no
// parent: unchanged). Yjs applies the rewritten updates (in order and reversed); recorded: its
// state, state vector and the map's toJSON.
//
// Usage: node gen_mapyata_fixtures.js <out_dir>  ->  <out_dir>/mapyata.json
'use strict';
const fs = require('fs');
const path = require('path');
const { loadYjs } = require('./load_yjs.js');
const { Reader, writeVu, canonicalUpdate, canonicalSv, hex } = require('./v1.js');

const Y = loadYjs();

function mulberry32(a) {
  return function () {
    a |= 0; a = (a + 0x6D2B79F5) | 0;
    let t = Math.imul(a ^ (a >>> 15), 1 | a);
    t = (t + Math.imul(t ^ (t >>> 7), 61 | t)) ^ t;
    return ((t ^ (t >>> 14)) >>> 0) / 4294967296;
  };
}

const vstr = (s) => { const b = Buffer.from(s, 'utf8'); const o = []; writeVu(o, b.length); return [...o, ...b]; };

// one update with root items of array 'm' moved to map 'users', key 'k'
function rewrite(u) {
  const r = new Reader(Buffer.from(u));
  const out = [];
  const nsec = r.vu(); writeVu(out, nsec);
  for (let s = 0; s < nsec; s++) {
    const n = r.vu(), client = r.vu(), clock = r.vu();
    writeVu(out, n); writeVu(out, client); writeVu(out, clock);
    for (let k = 0; k < n; k++) {
      const p0 = r.p;
      const info = r.u8();
      const ref = info & 31;
      if (ref === 0 || ref === 10) { r.vu(); out.push(...r.b.subarray(p0, r.p)); continue; }
      let hdrEnd;
      if (info & 0x80) { r.vu(); r.vu(); }
      if (info & 0x40) { r.vu(); r.vu(); }
      if ((info & 0xC0) === 0) {
        const pinfo = r.vu();
        if (pinfo !== 1) throw new Error('nested parent');
        const name = r.vstr();
        if (name !== 'm' || (info & 0x20)) throw new Error('unexpected root ' + name);
        out.push(info | 0x20, 1, ...vstr('users'), ...vstr('k'));
        hdrEnd = r.p;
      } else {
        out.push(...r.b.subarray(p0, r.p));
        hdrEnd = r.p;
      }
      // content
      const c0 = r.p;
      switch (ref) {
        case 1: r.vu(); break;
        case 8: { const m = r.vu(); for (let i = 0; i < m; i++) r.any(); break; }
        default: throw new Error('content ' + ref);
      }
      out.push(...r.b.subarray(c0, r.p));
    }
  }
  out.push(...r.b.subarray(r.p));  // the delete set, unchanged
  return Uint8Array.from(out);
}

function history(seed, nrep, rounds, ops) {
  const rnd = mulberry32(seed);
  const docs = [];
  for (let i = 0; i < nrep; i++) { const d = new Y.Doc(); d.clientID = 11 + 7 * i + (seed % 5); docs.push(d); }
  const wire = [];
  let v = 0;
  for (let rd = 0; rd < rounds; rd++) {
    for (const d of docs) {
      const a = d.getArray('m');
      for (let k = 0; k < ops; k++) {
        const x = rnd();
        if (x < 0.15 && a.length > 0) { const i = Math.floor(rnd() * a.length); a.delete(i, Math.min(a.length - i, 1 + Math.floor(rnd() * 2))); }
        else {
          const i = Math.floor(rnd() * (a.length + 1));
          const n = 1;  // (a run of several values in a map entry splits into pieces Yjs keeps alive: order-dependent)
          const vals = [];
          for (let j = 0; j < n; j++) vals.push(v++);
          a.insert(i, vals);
        }
      }
    }
    // partial gossip: each replica pulls a delta from one random peer
    for (const d of docs) {
      const peer = docs[Math.floor(rnd() * docs.length)];
      if (peer === d) continue;
      const delta = Y.encodeStateAsUpdate(peer, Y.encodeStateVector(d));
      wire.push(delta);
      Y.applyUpdate(d, delta);
    }
  }
  for (const d of docs) wire.push(Y.encodeStateAsUpdate(d));
  return wire;
}

const cases = [];
for (let seed = 1; seed <= 60; seed++) {
  const nrep = 2 + (seed % 4), rounds = 1 + (seed % 3), ops = 2 + (seed % 5);
  const wire = history(seed, nrep, rounds, ops).map(rewrite);
  const res = {};
  for (const [key, ups] of [['fwd', wire], ['rev', wire.slice().reverse()]]) {
    const d = new Y.Doc(); d.clientID = 5;
    for (const u of ups) Y.applyUpdate(d, u);
    res[key] = { state: hex(canonicalUpdate(Y.encodeStateAsUpdate(d))), sv: hex(canonicalSv(Y.encodeStateVector(d))),
                 json: JSON.parse(JSON.stringify(d.getMap('users').toJSON())) };
  }
  cases.push({ name: `mapyata_${seed}`, updates: wire.map(hex), fwd: res.fwd, rev: res.rev,
               pending_free: res.fwd.state === res.rev.state });
}
const outDir = process.argv[2] || path.join(__dirname, '..');
fs.writeFileSync(path.join(outDir, 'mapyata.json'), JSON.stringify({ yjs: '13.5.16', cases }));
console.log(`mapyata.json: ${cases.length} cases, ${cases.filter((c) => c.pending_free).length} order-independent`);
