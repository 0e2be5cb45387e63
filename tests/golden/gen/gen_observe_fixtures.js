#!/usr/bin/env node
// Observer-event fixtures (TEST INFRASTRUCTURE ONLY; runs in the build container, never on the GPU
// box): the events YMap.observe / YArray.observe deliver (crdt.js:620-657 forwards them to user
// code), recorded from the in-image Yjs 13.5.16 on seeded scripts. Peer A performs local ops
// (root map 'users', root array 'messages', a YArray nested under users[k] — crdt.js:423-430) with
// unique values; after every op peer B applies A's delta (Y.encodeStateAsUpdate(A, svB)); a third
// peer C makes concurrent sets that reach B as their own step. After each step every event each
// observed type fired is recorded as
//   {peer, target, keysChanged (sorted), keys: {k: [action, oldValue]}, delta}
// (target "users", "messages" or "users.<k>"). tests/js/napi_check.js `observe` replays the steps
// through the Node facade, reads both docs (its events fire at the next read) and compares.
//
// Usage: node gen_observe_fixtures.js <out_dir>  ->  <out_dir>/observe.json
'use strict';
const fs = require('fs');
const path = require('path');
const { loadYjs } = require('./load_yjs.js');
const { hex } = require('./v1.js');

const Y = loadYjs();

function mulberry32(a) {
  return function () {
    a |= 0; a = (a + 0x6D2B79F5) | 0;
    let t = Math.imul(a ^ (a >>> 15), 1 | a);
    t = (t + Math.imul(t ^ (t >>> 7), 61 | t)) ^ t;
    return ((t ^ (t >>> 14)) >>> 0) / 4294967296;
  };
}

const norm = (v) => (v === undefined ? null : JSON.parse(JSON.stringify(v)));

function recorder(log, peer, target) {
  return (ev) => {
    const rec = { peer, target, keysChanged: [], keys: {}, delta: [] };
    if (ev.keysChanged) rec.keysChanged = Array.from(ev.keysChanged).sort();
    if (ev.changes && ev.changes.keys) {
      for (const [k, c] of ev.changes.keys) {
        const ov = c.oldValue;
        rec.keys[k] = [c.action, ov instanceof Y.AbstractType ? { type: ov.toJSON() } : norm(ov)];
      }
    }
    if (!ev.keysChanged) rec.delta = JSON.parse(JSON.stringify(ev.changes.delta));
    log.push(rec);
  };
}

function script(seed, nsteps) {
  const g = mulberry32(seed);
  const int = (n) => Math.floor(g() * n);
  const A = new Y.Doc(); A.clientID = 11 + seed;
  const B = new Y.Doc(); B.clientID = 1000 + seed;
  const C = new Y.Doc(); C.clientID = 5 + seed;  // lower client than A: loses concurrent sets
  const log = [];
  const steps = [];
  for (const [peer, d] of [['A', A], ['B', B]]) {
    d.getMap('users').observe(recorder(log, peer, 'users'));
    d.getArray('messages').observe(recorder(log, peer, 'messages'));
  }
  const nested = new Set();
  let uid = 0;
  const val = () => (g() < 0.5 ? `v${seed}_${uid++}` : { n: uid++, s: `x${seed}` });
  const svB = () => Y.encodeStateVector(B);
  for (let i = 0; i < nsteps; i++) {
    const step = { ops: [], events: [] };
    const x = g();
    const users = A.getMap('users'), msgs = A.getArray('messages');
    if (x < 0.3) {
      const k = 'k' + int(6);
      if (!nested.has(k)) {
        const v = g() < 0.1 && users.has(k) ? users.get(k) : val();  // now and then the same value again
        const vv = v instanceof Y.AbstractType ? val() : v;
        users.set(k, vv);
        step.ops.push({ peer: 'A', op: 'map.set', key: k, value: norm(vv) });
      }
    } else if (x < 0.38) {
      const k = 'k' + int(6);
      if (users.has(k) && !nested.has(k)) { users.delete(k); step.ops.push({ peer: 'A', op: 'map.delete', key: k }); }
    } else if (x < 0.45 && nested.size < 2) {
      const k = 'n' + nested.size;
      users.set(k, new Y.Array());
      nested.add(k);
      step.ops.push({ peer: 'A', op: 'map.setArray', key: k });
      // B observes the nested array once it exists there (after this step's sync)
      step.observeNested = k;
    } else if (x < 0.6 && nested.size) {
      const k = Array.from(nested)[int(nested.size)];
      const arr = users.get(k);
      const vals = [val(), val()].slice(0, 1 + int(2));
      const idx = int(arr.length + 1);
      arr.insert(idx, vals);
      step.ops.push({ peer: 'A', op: 'nested.insert', key: k, index: idx, values: vals.map(norm) });
    } else if (x < 0.85) {
      const vals = [val(), val(), val()].slice(0, 1 + int(3));
      const L = msgs.length, y = g();
      const idx = y < 0.4 ? L : y < 0.6 ? 0 : int(L + 1);
      msgs.insert(idx, vals);
      step.ops.push({ peer: 'A', op: 'array.insert', index: idx, values: vals.map(norm) });
    } else if (x < 0.93) {
      const L = msgs.length;
      if (L) {
        const idx = int(L), n = Math.min(L - idx, 1 + int(2));
        msgs.delete(idx, n);
        step.ops.push({ peer: 'A', op: 'array.delete', index: idx, length: n });
      }
    } else {
      // a concurrent set on C (it knows everything B knows), sent to B as its own update
      Y.applyUpdate(C, Y.encodeStateAsUpdate(B, Y.encodeStateVector(C)));
      const k = 'k' + int(6);
      if (!nested.has(k)) {
        const v = val();
        C.getMap('users').set(k, v);
        step.ops.push({ peer: 'C', op: 'c.set', key: k, value: norm(v), update: hex(Y.encodeStateAsUpdate(C, svB())) });
        Y.applyUpdate(B, Y.encodeStateAsUpdate(C, svB()));
      }
    }
    // B catches up with A
    const u = Y.encodeStateAsUpdate(A, svB());
    step.sync = hex(u);
    Y.applyUpdate(B, u);
    if (step.observeNested) {
      const k = step.observeNested;
      A.getMap('users').get(k).observe(recorder(log, 'A', 'users.' + k));
      B.getMap('users').get(k).observe(recorder(log, 'B', 'users.' + k));
    }
    step.events = log.splice(0);
    step.json = { A: norm(A.getMap('users').toJSON()), B: norm(B.getMap('users').toJSON()), Bm: norm(B.getArray('messages').toJSON()) };
    steps.push(step);
  }
  return { name: `observe_s${seed}`, clients: { A: A.clientID, B: B.clientID, C: C.clientID }, steps };
}

function main() {
  const outDir = process.argv[2] || path.join(__dirname, '..');
  const cases = [];
  for (let s = 1; s <= 6; s++) cases.push(script(s, 60));
  const f = path.join(outDir, 'observe.json');
  fs.writeFileSync(f, JSON.stringify({ generator: 'gen_observe_fixtures.js', yjs: '13.5.16', cases }));
  const nev = cases.reduce((n, c) => n + c.steps.reduce((m, s) => m + s.events.length, 0), 0);
  console.log(`wrote ${f}: ${cases.length} scripts, ${nev} events`);
}

main();
