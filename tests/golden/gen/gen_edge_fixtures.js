#!/usr/bin/env node
// Edge-case golden fixtures (TEST INFRASTRUCTURE ONLY; runs in the build container against the
// in-image Yjs 13.5.16, never on the GPU box):
//   deep:     YMap values that are lib0 `any` containers nested 8 .. 2 000 levels deep, along last
//             members ([[[..]]], {a: {a: ..}}) and with members after the nested one (non-tail
//             nesting up to 30 levels); lib0's readAny (L0@1937) recurses without a limit;
//   sections: updates whose struct section holds TWO sections of one client, or sections out of
//             the descending client order Yjs writes — valid input for Yjs's readers: applyUpdate
//             (readClientsStructRefs keeps the last section of a client, Y@19286), mergeUpdates
//             (the lazy readers' sort loop, Y@39011) and diffUpdate (Y@40711).
// Every case records the inputs and what Yjs computes from them.
//
// Usage: node gen_edge_fixtures.js <out_dir>  ->  <out_dir>/edges.json
'use strict';
const fs = require('fs');
const path = require('path');
const { loadYjs } = require('./load_yjs.js');
const { Reader, writeVu, canonicalUpdate, canonicalSv, hex } = require('./v1.js');

const Y = loadYjs();
const hexc = (u) => hex(canonicalUpdate(u));

function nestTail(depth, obj, leaf) {
  let v = leaf;
  for (let i = 0; i < depth; i++) v = obj ? { a: v } : [v];
  return v;
}
function nestNonTail(depth, leaf) {  // every level has a member after the nested container
  let v = leaf;
  for (let i = 0; i < depth; i++) v = i % 2 ? [v, i] : { x: v, y: 'm' + i };
  return v;
}

function result(updates, roots) {
  const d = new Y.Doc(); d.clientID = 0x7ffffff0;
  for (const u of updates) Y.applyUpdate(d, u);
  const json = {};
  for (const [name, kind] of Object.entries(roots)) json[name] = (kind === 'map' ? d.getMap(name) : d.getArray(name)).toJSON();
  return { state: hex(canonicalUpdate(Y.encodeStateAsUpdate(d))), sv: hex(canonicalSv(Y.encodeStateVector(d))),
           json: JSON.parse(JSON.stringify(json)) };
}

const cases = [];

// ---- deep `any` values
{
  const shapes = [];
  for (const depth of [8, 31, 33, 40, 100, 400, 2000]) {
    shapes.push([`arr${depth}`, nestTail(depth, false, 7)]);
    shapes.push([`obj${depth}`, nestTail(depth, true, 'leaf')]);
  }
  for (const depth of [10, 20, 30]) shapes.push([`nontail${depth}`, nestNonTail(depth, [1, 2, 3])]);
  shapes.push(['tail_after_nontail', nestTail(200, false, nestNonTail(20, { deep: nestTail(50, true, null) }))]);
  const a = new Y.Doc(); a.clientID = 101;
  const b = new Y.Doc(); b.clientID = 202;
  const ma = a.getMap('users'); const mb = b.getMap('users');
  const arr = a.getArray('messages');
  shapes.forEach(([name, v], i) => {
    (i % 2 ? ma : mb).set(name, v);
    if (i % 3 === 0) arr.push([v]);
  });
  ma.set('arr40', 'overwritten by a');  // a concurrent overwrite of a deep value
  const ua = Y.encodeStateAsUpdate(a); const ub = Y.encodeStateAsUpdate(b);
  const roots = { users: 'map', messages: 'array' };
  const ups = [ua, ub];
  cases.push(Object.assign({ name: 'deep_any', kind: 'deep', updates: ups.map(hex), roots,
                             merged: hexc(Y.mergeUpdates(ups)), merged_raw: hex(Y.mergeUpdates(ups)) }, result(ups, roots)));
}

// ---- sections of one client twice / out of order
function sections(u) {  // [{n, client, clock, body}] + the delete-set bytes
  const r = new Reader(u);
  const nsec = r.vu(); const out = [];
  for (let s = 0; s < nsec; s++) {
    const n = r.vu(); const client = r.vu(); const clock = r.vu();
    const start = r.p;
    for (let i = 0; i < n; i++) skipStruct(r);
    out.push({ n, client, clock, body: u.subarray(start, r.p) });
  }
  return { secs: out, ds: u.subarray(r.p) };
}
function skipStruct(r) {
  const info = r.u8(); const ref = info & 31;
  if (ref === 0 || ref === 10) { r.vu(); return; }
  if (info & 0x80) { r.vu(); r.vu(); }
  if (info & 0x40) { r.vu(); r.vu(); }
  if ((info & 0xc0) === 0) { if (r.vu() === 1) r.vstr(); else { r.vu(); r.vu(); } if (info & 0x20) r.vstr(); }
  switch (ref) {
    case 1: r.vu(); break;
    case 2: { const len = r.vu(); for (let k = 0; k < len; k++) r.vstr(); break; }
    case 3: { const n2 = r.vu(); r.bytes(n2); break; }
    case 4: case 5: r.vstr(); break;
    case 6: r.vstr(); r.vstr(); break;
    case 7: { const tr = r.vu(); if (tr === 3 || tr === 5) r.vstr(); break; }
    case 8: { const len = r.vu(); for (let k = 0; k < len; k++) r.any(); break; }
    case 9: r.vstr(); r.any(); break;
    default: throw new Error('bad content ref ' + ref);
  }
}
function assemble(secs, ds) {
  const out = []; writeVu(out, secs.length);
  for (const s of secs) { writeVu(out, s.n); writeVu(out, s.client); writeVu(out, s.clock); for (const x of s.body) out.push(x); }
  for (const x of ds) out.push(x);
  return Uint8Array.from(out);
}
{
  const mk = (id) => { const d = new Y.Doc(); d.clientID = id; return d; };
  for (let seed = 0; seed < 6; seed++) {
    const hi = mk(900 + seed); const lo = mk(100 + seed); const mid = mk(500 + seed);
    const mh = hi.getMap('users'); const ml = lo.getMap('users'); const mm = mid.getMap('users');
    const ah = hi.getArray('messages'); const al = lo.getArray('messages');
    for (let i = 0; i < 3 + seed; i++) { mh.set('k' + (i % 4), 'h' + i); ah.push(['x' + i]); }
    const svHi1 = Y.encodeStateVector(hi);
    const u1 = Y.encodeStateAsUpdate(hi);  // hi 0..n1
    for (let i = 0; i < 2 + seed; i++) { mh.set('k' + ((i + 1) % 5), 'H' + i); ah.insert(0, ['y' + i]); }
    mh.delete('k0');
    const u2 = Y.encodeStateAsUpdate(hi, svHi1);  // hi n1..n2 (+ delete set)
    for (let i = 0; i < 4; i++) { ml.set('k' + i, 'l' + i); al.push([i]); }
    const u3 = Y.encodeStateAsUpdate(lo);
    Y.applyUpdate(mid, u1);
    for (let i = 0; i < 3; i++) mm.set('m' + i, i);
    const u4 = Y.encodeStateAsUpdate(mid, svHi1);  // mid's own structs
    const s1 = sections(u1).secs; const s2 = sections(u2); const s3 = sections(u3).secs; const s4 = sections(u4).secs;
    // layouts Yjs itself never writes, each a valid update for its readers
    const layouts = {
      hi_late_first: assemble([s2.secs[0], ...s3, s1[0]], s2.ds),        // hi n1..n2, lo, hi 0..n1
      hi_twice_desc: assemble([s1[0], s2.secs[0], ...s3], s2.ds),        // hi 0..n1, hi n1..n2, lo
      ascending: assemble([...s3, ...s4, s1[0]], new Uint8Array([0])),  // lo, mid, hi: ascending clients
    };
    for (const [lname, x] of Object.entries(layouts)) {
      const others = [u3, u4];
      const roots = { users: 'map', messages: 'array' };
      const sv = Y.encodeStateVector(lo);
      const rec = { name: `sections_${lname}_${seed}`, kind: 'sections', update: hex(x),
                    others: others.map(hex), roots,
                    diff_sv_of: hex(sv), diff_hi1_of: hex(svHi1) };
      // Yjs's bytes (13.5.16 delete-set order: *_raw) and their canonical form (13.6 order)
      const outs = { merged_with_others: Y.mergeUpdates([x, ...others]), merged_others_first: Y.mergeUpdates([...others, x]),
                     merged_pair: Y.mergeUpdates([x, x]), diff_empty: Y.diffUpdate(x, new Uint8Array([0])),
                     diff_sv: Y.diffUpdate(x, sv), diff_hi1: Y.diffUpdate(x, svHi1) };
      for (const [k, v] of Object.entries(outs)) { rec[k] = hexc(v); rec[k + '_raw'] = hex(v); }
      Object.assign(rec, result([x], roots));  // applyUpdate of the update alone
      const both = result([x, ...others], roots);
      rec.state_with_others = both.state; rec.sv_with_others = both.sv; rec.json_with_others = both.json;
      cases.push(rec);
    }
  }
}

// ---- ContentJSON / ContentEmbed / ContentFormat values outside JSON.stringify's form (round 6:
// rewritten, no longer refused). Yjs 13.5 itself writes ContentAny for JS values; these updates are
// hand-assembled the way an older Yjs peer (ContentJSON) or a rich-text peer (Embed / Format) sends
// them, with texts JSON.parse takes but JSON.stringify writes differently. Yjs keeps the parsed
// values (Y@72137) and writes them with JSON.stringify (Y@71991).
{
  const vs = (out, str) => { const b = Buffer.from(str, 'utf8'); writeVu(out, b.length); for (const x of b) out.push(x); };
  // one section of `client` from clock 0: items [{root, sub?, ref, vals | key+val}], chained by origin
  function handUpdate(client, items, overlong, after) {  // after: [client, clock] the first item's origin
    const out = [];
    writeVu(out, 1); writeVu(out, items.length); writeVu(out, client); writeVu(out, 0);
    let clock = 0; let prev = null;
    for (const it of items) {
      const chain = prev && prev.root === it.root && !it.sub && !prev.sub;
      const ext = !prev && after;
      out.push(it.ref | (chain || ext ? 0x80 : 0) | (!chain && !ext && it.sub ? 0x20 : 0));
      if (chain) { writeVu(out, client); writeVu(out, clock - 1); }
      else if (ext) { writeVu(out, after[0]); writeVu(out, after[1]); }
      else { writeVu(out, 1); vs(out, it.root); if (it.sub) vs(out, it.sub); }
      let len = 1;
      if (it.ref === 2) {
        writeVu(out, it.vals.length);
        for (const v of it.vals) {
          if (overlong) { const b = Buffer.from(v, 'utf8'); out.push(0x80 | (b.length & 0x7f), b.length >> 7); for (const x of b) out.push(x); }
          else vs(out, v);
        }
        len = it.vals.length;
      } else if (it.ref === 5) {
        vs(out, it.val);
      } else {
        vs(out, it.key); vs(out, it.val);
      }
      clock += len; prev = it;
    }
    out.push(0);  // no delete set
    return new Uint8Array(out);
  }
  const deep = '['.repeat(90) + ' 1.0 ' + ']'.repeat(90);
  const sets = {
    array_values: [{ root: 'messages', ref: 2, vals: ['0.30000000000000004', ' 1 ', '1.50', '{"b":1,"a":2,"b":3}', '"\\u0041\\/"', '1e400', 'undefined',
      '{"2":1,"1":2,"a":3,"0":[]}', '[1.0, 2.50, -0.0]', '"\\ud83d\\ude00\\ud800"', '123456789012345678901234567890', deep, '1e-7', '{"__proto__":{"x" :1}}'] }],
    map_values: [{ root: 'users', sub: 'k1', ref: 2, vals: [' {"x" : 1e2} '] }, { root: 'users', sub: 'k2', ref: 2, vals: ['-0'] },
      { root: 'users', sub: 'k3', ref: 2, vals: ['{"a":1,"\\u0061":2}'] }, { root: 'users', sub: 'k4', ref: 2, vals: ['0.1', ' "x" '] }],
    embed_format: [{ root: 'messages', ref: 5, val: ' {"insert" : "x", "n": 1.0} ' }, { root: 'messages', ref: 2, vals: ['[ ]'] },
      { root: 'users', sub: 'f', ref: 6, key: 'bold', val: ' true ' }],
    canonical_long: [{ root: 'messages', ref: 2, vals: ['0.30000000000000004', '1.7976931348623157e+308', '5e-324', '123456789012345680000', '"\\u001f"'] }],
  };
  const base = new Y.Doc(); base.clientID = 303;
  base.getMap('users').set('k1', 'base'); base.getArray('messages').push(['m0', 1]);
  const baseU = Y.encodeStateAsUpdate(base);
  Object.entries(sets).forEach(([name, items], i) => {
    for (const overlong of [false, true]) {
      if (overlong && name !== 'array_values' && name !== 'map_values') continue;
      const u = handUpdate(1000 + i, items, overlong);
      const roots = { users: 'map', messages: 'array' };
      const rec = { name: `json_${name}${overlong ? '_overlong' : ''}`, kind: 'json', update: hex(u), base: hex(baseU), roots };
      Object.assign(rec, result([u], roots));
      const both = result([baseU, u], roots);
      rec.state_with_base = both.state; rec.sv_with_base = both.sv; rec.json_with_base = both.json;
      const outs = { merged_with_base: Y.mergeUpdates([baseU, u]), merged_pair: Y.mergeUpdates([u, u]), diff_empty: Y.diffUpdate(u, new Uint8Array([0])) };
      for (const [k, v] of Object.entries(outs)) { rec[k] = hexc(v); rec[k + '_raw'] = hex(v); }
      cases.push(rec);
    }
  });
  // pending: the texts arrive in an update whose first item follows another client's item not yet
  // seen (Yjs parks it: pendingStructs, written back by encodeStateAsUpdate), then the dependency
  {
    const dep = new Y.Doc(); dep.clientID = 1999;
    dep.getArray('messages').push(['d0', 'd1']);
    const depU = Y.encodeStateAsUpdate(dep);
    const u = handUpdate(2000, [{ root: 'messages', ref: 2, vals: [' 1.50 ', '{"b":1,"a":[ 1e2 ],"b":2}', '"\\u00e9"'] }], false, [1999, 1]);
    const roots = { users: 'map', messages: 'array' };
    const rec = { name: 'json_pending', kind: 'json_pending', update: hex(u), dep: hex(depU), roots };
    const d = new Y.Doc(); d.clientID = 0x7ffffff0;
    Y.applyUpdate(d, u);
    rec.state_pending = hex(canonicalUpdate(Y.encodeStateAsUpdate(d)));
    rec.sv_pending = hex(canonicalSv(Y.encodeStateVector(d)));
    Y.applyUpdate(d, depU);
    rec.state = hex(canonicalUpdate(Y.encodeStateAsUpdate(d)));
    rec.sv = hex(canonicalSv(Y.encodeStateVector(d)));
    rec.json = JSON.parse(JSON.stringify({ users: d.getMap('users').toJSON(), messages: d.getArray('messages').toJSON() }));
    cases.push(rec);
  }
}

const outDir = process.argv[2] || path.join(__dirname, '..');
fs.writeFileSync(path.join(outDir, 'edges.json'), JSON.stringify({ yjs: '13.5.16', cases }, null, 0));
console.log(`edges.json: ${cases.length} cases`);
