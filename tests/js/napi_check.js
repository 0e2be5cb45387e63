#!/usr/bin/env node
// Drives the N-API `Y` facade (crdt_amd/js). Modes:
//   cpu     — the addon loads, exports the Y surface, and fails loudly without a GPU
//   golden  — every golden case through Y.applyUpdate / Y.encodeStateAsUpdate / encodeStateVector
//   ops     — every Yjs 13.5.16 local-op script (tests/golden/ops.json) through the YMap / YArray
//             facade crdt.js uses (getMap/getArray, set/delete, set(key, new Y.Array()), push /
//             unshift / insert / delete, toJSON / toArray, observe), byte-identical after every step
//   trace   — the crdt.js-driven Y call traces (tests/golden/crdtjs_traces.json), YCRDT_COMPAT=135
'use strict';
const fs = require('fs');
const path = require('path');
const assert = require('assert');

const ROOT = path.join(__dirname, '..', '..');
const Y = require(path.join(ROOT, 'crdt_amd', 'js'));
const hex = (u) => Buffer.from(u).toString('hex');
const unhex = (h) => new Uint8Array(Buffer.from(h, 'hex'));

const mode = process.argv[2] || 'cpu';
const { encodeAny, decodeAny } = require(path.join(ROOT, 'crdt_amd', 'js', 'any.js'));
const opsCases = () => JSON.parse(fs.readFileSync(path.join(ROOT, 'tests', 'golden', 'ops.json'))).cases;
for (const f of ['Doc', 'applyUpdate', 'applyUpdates', 'applyUpdatesMulti', 'encodeStateAsUpdate', 'encodeStateVector', 'mergeUpdates', 'diffUpdate', 'diffUpdates']) {
  assert.strictEqual(typeof Y[f], 'function', f);
}
assert.ok(/gfx950/.test(Y.version()));
for (const f of ['getMap', 'getArray', 'transact']) assert.strictEqual(typeof Y.Doc.prototype[f], 'function', f);
for (const f of ['set', 'get', 'has', 'delete', 'toJSON', 'observe', 'unobserve']) assert.strictEqual(typeof Y.Map.prototype[f], 'function', f);
for (const f of ['insert', 'push', 'unshift', 'delete', 'toJSON', 'toArray', 'observe', 'unobserve']) assert.strictEqual(typeof Y.Array.prototype[f], 'function', f);
if (mode === 'cpu') {
  // the lib0 any codec against every value Yjs 13.5.16 wrote in the op scripts
  let nv = 0;
  for (const c of opsCases()) {
    for (const s of c.steps) {
      for (const a of s.any ? [s.any] : s.anys || []) {
        const vals = decodeAny(unhex(a));
        assert.strictEqual(vals.length, 1);
        assert.strictEqual(hex(encodeAny(vals)), a, 'any codec ' + a);
        nv++;
      }
    }
  }
  console.log('any codec ok:', nv, 'values');
  let threw = null;
  try { new Y.Doc(); } catch (e) { threw = e; }
  assert.ok(threw instanceof Error, 'no device: new Y.Doc() must throw');
  assert.ok(/device/i.test(threw.message), threw.message);
  console.log('napi cpu ok:', threw.message);
} else if (mode === 'ops') {
  let n = 0, events = 0;
  for (const c of opsCases()) {
    const d = new Y.Doc({ clientID: c.client });
    const users = d.getMap('users');
    const msgs = d.getArray('messages');
    users.observe((ev) => { events++; assert.ok(ev.keysChanged.size > 0 && ev.target === users); });
    c.steps.forEach((s, i) => {
      const tgt = () => (s.parent_key ? users.get(s.parent_key) : d.getArray(s.root));
      if (s.op === 'apply') Y.applyUpdate(d, unhex(s.update));
      else if (s.op === 'map_set') d.getMap(s.root).set(s.key, decodeAny(unhex(s.any))[0]);
      else if (s.op === 'map_set_type') {
        const a = new Y.Array();
        assert.strictEqual(d.getMap(s.root).set(s.key, a), a);
        assert.ok(users.get(s.key) instanceof Y.Array);
      } else if (s.op === 'map_delete') d.getMap(s.root).delete(s.key);
      else if (s.op === 'array_insert') {
        const arr = tgt();
        assert.ok(arr instanceof Y.Array, c.name + ' step ' + i);
        const vals = s.anys.map((a) => decodeAny(unhex(a))[0]);
        const L = arr.length;
        if (s.index === L && i % 2) arr.push(vals);
        else if (s.index === 0 && i % 2) arr.unshift(vals);
        else d.transact(() => arr.insert(s.index, vals));
      } else if (s.op === 'array_delete') tgt().delete(s.index, s.length);
      else throw new Error(s.op);
      assert.strictEqual(hex(Y.encodeStateAsUpdate(d)), s.state, c.name + ' step ' + i + ' ' + s.op);
    });
    assert.deepStrictEqual(JSON.parse(JSON.stringify(users.toJSON())), c.json.users, c.name);
    assert.deepStrictEqual(JSON.parse(JSON.stringify(msgs.toArray())), c.json.messages, c.name);
    n++;
  }
  assert.ok(events > 0, 'YMap observers fired');
  console.log('napi ops ok:', n, 'scripts,', events, 'map events');
} else if (mode === 'observe') {
  // observer events (tests/golden/observe.json, gen_observe_fixtures.js): the Yjs 13.5.16 events of
  // every step, replayed through the facade in both observer modes: 'sync' (the default: every
  // event inside the call that caused it, checked before anything reads the docs) and 'deferred'
  // (events at the next read)
  const cases = JSON.parse(fs.readFileSync(path.join(ROOT, 'tests', 'golden', 'observe.json'))).cases;
  const norm = (v) => (v === undefined ? null : JSON.parse(JSON.stringify(v)));
  let nev = 0;
  for (const om of ['sync', 'deferred']) {
  Y.setObserverMode(om);
  for (const c of cases) {
    const log = [];
    const rec = (peer, target) => (ev) => {
      const r = { peer, target, keysChanged: [], keys: {}, delta: [] };
      if (ev.keysChanged) r.keysChanged = Array.from(ev.keysChanged).sort();
      for (const [k, ch] of ev.changes.keys) r.keys[k] = [ch.action, norm(ch.oldValue)];
      if (!ev.keysChanged) r.delta = norm(ev.changes.delta);
      assert.ok(ev.target && ev.transaction, 'event shape');
      log.push(r);
    };
    const A = new Y.Doc({ clientID: c.clients.A }), B = new Y.Doc({ clientID: c.clients.B });
    for (const [peer, d] of [['A', A], ['B', B]]) {
      d.getMap('users').observe(rec(peer, 'users'));
      d.getArray('messages').observe(rec(peer, 'messages'));
    }
    c.steps.forEach((st, i) => {
      const tag = c.name + ' step ' + i;
      for (const o of st.ops) {
        if (o.op === 'map.set') A.getMap('users').set(o.key, o.value);
        else if (o.op === 'map.delete') A.getMap('users').delete(o.key);
        else if (o.op === 'map.setArray') A.getMap('users').set(o.key, new Y.Array());
        else if (o.op === 'nested.insert') A.getMap('users').get(o.key).insert(o.index, o.values);
        else if (o.op === 'array.insert') A.getArray('messages').insert(o.index, o.values);
        else if (o.op === 'array.delete') A.getArray('messages').delete(o.index, o.length);
        else if (o.op === 'c.set') Y.applyUpdate(B, unhex(o.update));
        else throw new Error(o.op);
      }
      Y.applyUpdate(B, unhex(st.sync));
      const early = om === 'sync' ? log.splice(0) : [];  // delivered before anything read the docs
      const json = { A: norm(A.getMap('users').toJSON()), B: norm(B.getMap('users').toJSON()), Bm: norm(B.getArray('messages').toJSON()) };
      assert.deepStrictEqual(json, st.json, tag + ' toJSON');
      if (st.observeNested) {
        A.getMap('users').get(st.observeNested).observe(rec('A', 'users.' + st.observeNested));
        B.getMap('users').get(st.observeNested).observe(rec('B', 'users.' + st.observeNested));
      }
      const key = (e) => e.peer + ' ' + e.target;
      if (om === 'sync') assert.strictEqual(log.length, 0, tag + ' sync events after a read');
      const got = early.concat(log.splice(0)).sort((x, y) => (key(x) < key(y) ? -1 : key(x) > key(y) ? 1 : 0));
      const want = st.events.slice().sort((x, y) => (key(x) < key(y) ? -1 : key(x) > key(y) ? 1 : 0));
      assert.deepStrictEqual(got, want, tag + ' events');
      nev += want.length;
    });
  }
  }
  console.log('napi observe ok:', cases.length, 'scripts x 2 modes,', nev, 'events');
} else if (mode === 'trace') {
  // crdt.js-driven traces (tests/golden/crdtjs_traces.json, gen_crdtjs_traces.js): every Y call
  // crdt.js made on every peer, replayed in order; every wire update / state vector byte-equal
  // (run with YCRDT_COMPAT=135: Yjs 13.5.16's own bytes) and every toJSON / get / has deep-equal —
  // the values crdt.c is built from (crdt.js:297-305, 372, 494, ...)
  const cases = JSON.parse(fs.readFileSync(path.join(ROOT, 'tests', 'golden', 'crdtjs_traces.json'))).cases;
  const norm = (v) => (v === undefined ? undefined : JSON.parse(JSON.stringify(v)));
  const val = (r) => (r.undef ? undefined : r.v);
  let nwire = 0, njson = 0, ncalls = 0;
  for (const c of cases) {
    const docs = {};
    const typeOf = (ref) => {
      const d = docs[ref.doc];
      if (ref.key === undefined) return ref.kind === 'map' ? d.getMap(ref.root) : d.getArray(ref.root);
      return d.getMap(ref.root).get(ref.key);
    };
    c.calls.forEach((x, i) => {
      const tag = c.name + ' #' + i + ' ' + x.op;
      const m = x.op.split('.')[1];
      switch (x.op) {
        case 'doc': docs[x.doc] = new Y.Doc({ clientID: x.client }); break;
        case 'getMap': docs[x.doc].getMap(x.name); break;
        case 'getArray': docs[x.doc].getArray(x.name); break;
        case 'transact': case 'api': case 'crdt.c': break;  // execBatch's async callback: its ops follow on their own
        case 'applyUpdate': Y.applyUpdate(docs[x.doc], unhex(x.update)); break;
        case 'encodeStateAsUpdate':
          assert.strictEqual(hex(Y.encodeStateAsUpdate(docs[x.doc], x.sv ? unhex(x.sv) : undefined)), x.result, tag);
          nwire++;
          break;
        case 'encodeStateVector': assert.strictEqual(hex(Y.encodeStateVector(docs[x.doc])), x.result, tag); break;
        case 'map.set': typeOf(x.ref).set(x.key, x.type ? new Y.Array() : val(x.value)); break;
        case 'map.get': {
          const r = typeOf(x.ref).get(x.key);
          if (x.result.type) assert.ok(r instanceof Y.Array || r instanceof Y.Map, tag);
          else assert.deepStrictEqual(norm(r), norm(val(x.result)), tag);
          break;
        }
        case 'map.has': assert.strictEqual(typeOf(x.ref).has(...x.args), val(x.result), tag); break;
        case 'map.toJSON': case 'array.toJSON': case 'array.toArray':
          assert.deepStrictEqual(norm(typeOf(x.ref)[m]()), norm(val(x.result)), tag);
          njson++;
          break;
        case 'map.delete': case 'array.push': case 'array.unshift': case 'array.insert': case 'array.delete':
          typeOf(x.ref)[m](...x.args);
          break;
        case 'array.length': assert.strictEqual(typeOf(x.ref).length, x.result, tag); break;
        default: throw new Error('unknown recorded call ' + x.op);
      }
      ncalls++;
    });
  }
  console.log('napi trace ok:', cases.length, 'crdt.js scenarios,', ncalls, 'calls,', nwire, 'wire updates,', njson, 'toJSON');
} else {
  let n = 0;
  const dsrc = [], dsv = [];
  for (const set of ['kat', 'map', 'array', 'nested']) {
    const cases = JSON.parse(fs.readFileSync(path.join(ROOT, 'tests', 'golden', set + '.json'))).cases;
    for (const c of cases) {
      const d = new Y.Doc({ clientID: 0x7ffffff0 });
      if (n % 2) Y.applyUpdates(d, c.updates.map(unhex));
      else for (const u of c.updates) Y.applyUpdate(d, unhex(u));
      assert.strictEqual(hex(Y.encodeStateAsUpdate(d)), c.state, c.name);
      assert.strictEqual(hex(Y.encodeStateVector(d)), c.sv, c.name);
      for (const df of c.diffs) assert.strictEqual(hex(Y.encodeStateAsUpdate(d, unhex(df.sv))), df.update, c.name);
      assert.strictEqual(hex(Y.mergeUpdates(c.updates.map(unhex))), c.updates.length > 1 ? c.merged : c.merged_raw, c.name);
      const st = Y.encodeStateAsUpdate(d);
      for (const df of c.diffs) { dsrc.push(st); dsv.push(unhex(df.sv)); }
      dsrc.push(st); dsv.push(new Uint8Array([0]));
      n++;
    }
  }
  // fleet ingest: every golden case is a document, all their updates in ONE Y.applyUpdatesMulti
  const fleet = [], fdocs = [], fups = [];
  for (const set of ['kat', 'map', 'array', 'nested']) {
    for (const c of JSON.parse(fs.readFileSync(path.join(ROOT, 'tests', 'golden', set + '.json'))).cases) {
      const d = new Y.Doc({ clientID: 0x7ffffff0 });
      fleet.push([d, c]);
      for (const u of c.updates) { fdocs.push(d); fups.push(unhex(u)); }
    }
  }
  Y.applyUpdatesMulti(fdocs, fups);
  for (const [d, c] of fleet) assert.strictEqual(hex(Y.encodeStateAsUpdate(d)), c.state, 'applyUpdatesMulti ' + c.name);
  // a non-Uint8Array update is a TypeError (the addon's error path frees its arrays only after reading them)
  let bad = null;
  try { Y.applyUpdatesMulti([fdocs[0], fdocs[1]], [fups[0], 'not bytes']); } catch (e) { bad = e; }
  assert.ok(bad instanceof TypeError && /Uint8Array/.test(bad.message), 'applyUpdatesMulti type error: ' + bad);
  // the batched sync responder: every (doc state, peer state vector) pair in one call
  const batch = Y.diffUpdates(dsrc, dsv);
  assert.strictEqual(batch.length, dsrc.length);
  for (let i = 0; i < dsrc.length; i++) assert.strictEqual(hex(batch[i]), hex(Y.diffUpdate(dsrc[i], dsv[i])), 'diffUpdates ' + i);
  let threw = null;
  try { Y.applyUpdate(new Y.Doc(), new Uint8Array([0xff, 0xff])); } catch (e) { threw = e; }
  assert.ok(threw && /Integer out of range/.test(threw.message), 'malformed update must throw like Yjs');
  console.log('napi golden ok:', n, 'cases,', dsrc.length, 'batched diffs');
}
