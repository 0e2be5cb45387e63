#!/usr/bin/env node
// CPU baseline leg of bench.py: the reference path — Yjs itself — timed in Node on this machine's
// host cores (SURVEY.md §8(d)). Never part of the product; only bench.py runs it.
//
// The Yjs that @ypear/crdt would call is the machine's installed copy: this image ships Yjs
// 13.5.16 + lib0 0.2.42 inside JupyterLab's static bundle (SURVEY.md §4.1), loaded in place by
// tests/golden/gen/load_yjs.js. If it is absent the script prints {"available": false}.
//
// Usage: node yjs_baseline.js <batch file> [workers]
//        node yjs_baseline.js <pairs file> diff [W]   (update, state vector) alternating: Y.diffUpdate each,
//                                                   on W worker_threads
//        node yjs_baseline.js <n ops> perop       crdt.js per-op path (bench.py per_op_leg)
//        node yjs_baseline.js <fleet file> fleet W nDocs   C5 fleet ingest on W worker_threads
//   batch file = u32le count, then per update u32le length + bytes (bench.py writes it)
// Single-doc workloads run on ONE core (Yjs integrates a doc on one thread; SURVEY.md §8(d)):
// `for u of batch: Y.applyUpdate(doc, u)` then `Y.encodeStateAsUpdate(doc)`, timed with
// process.hrtime.bigint() around that loop only. With workers > 1 (doc fleets), each
// worker_thread merges its own copy of the batch as an independent doc and the rate is the sum.
'use strict';
const fs = require('fs');
const path = require('path');
const crypto = require('crypto');
const { Worker, isMainThread, parentPort, workerData } = require('worker_threads');

function readBatch(file) {
  const b = fs.readFileSync(file);
  const n = b.readUInt32LE(0);
  const ups = [];
  let p = 4;
  for (let i = 0; i < n; i++) {
    const len = b.readUInt32LE(p);
    p += 4;
    ups.push(new Uint8Array(b.buffer, b.byteOffset + p, len));
    p += len;
  }
  return ups;
}

function runOnce(Y, ups) {
  const doc = new Y.Doc();
  doc.clientID = 0x7ffffff0;
  const t0 = process.hrtime.bigint();
  for (const u of ups) Y.applyUpdate(doc, u);
  const out = Y.encodeStateAsUpdate(doc);
  const t1 = process.hrtime.bigint();
  return { ms: Number(t1 - t0) / 1e6, out };
}

function load() {
  try {
    const { loadYjs } = require(path.join(__dirname, '..', 'tests', 'golden', 'gen', 'load_yjs.js'));
    return loadYjs();
  } catch (e) {
    return null;
  }
}

if (isMainThread) {
  const file = process.argv[2];
  const workers = Math.max(1, parseInt(process.argv[3] || '1', 10));
  const Y = load();
  if (!Y) {
    console.log(JSON.stringify({ available: false, reason: 'Yjs bundle not found on this machine' }));
    process.exit(0);
  }
  if (process.argv[3] === 'fleet') {  // C5 fleet ingest: (doc, update) pairs, W worker_threads
    const W = Math.max(1, parseInt(process.argv[4] || '1', 10));
    const nDocs = parseInt(process.argv[5], 10);
    let done = 0, maxMs = 0;
    const hashes = new Array(W);
    for (let w = 0; w < W; w++) {
      const wk = new Worker(__filename, { workerData: { fleet: file, w, W, nDocs } });
      wk.on('message', (m) => {
        hashes[w] = m.states;
        maxMs = Math.max(maxMs, m.ms);
        if (++done === W) {
          const h = crypto.createHash('sha256');
          for (let d = 0; d < nDocs; d++) h.update(Buffer.from(hashes[d % W][Math.floor(d / W)], 'hex'));
          console.log(JSON.stringify({ available: true, yjs: '13.5.16', lib0: '0.2.42', node: process.version,
            workers: W, cpus: require('os').cpus().length, ms: maxMs, state_sha256: h.digest('hex') }));
        }
      });
    }
    return;
  }
  if (process.argv[3] === 'perop') {  // crdt.js per-op path: A set/delete + full encode, B apply + toJSON
    const { canonicalUpdate } = require(path.join(__dirname, '..', 'tests', 'golden', 'gen', 'v1.js'));
    const n = parseInt(file, 10);
    const a = new Y.Doc(); a.clientID = 1;
    const b = new Y.Doc(); b.clientID = 2;
    const ma = a.getMap('users'), mb = b.getMap('users');
    const t0 = process.hrtime.bigint();
    for (let i = 0; i < n; i++) {
      const key = 'user' + (i % 100);
      if (i % 5 === 4) ma.delete(key); else ma.set(key, 'v' + i);
      const u = Y.encodeStateAsUpdate(a);
      Y.applyUpdate(b, u);
      mb.toJSON();
    }
    const t1 = process.hrtime.bigint();
    const st = canonicalUpdate(Y.encodeStateAsUpdate(b));
    console.log(JSON.stringify({
      available: true, yjs: '13.5.16', lib0: '0.2.42', node: process.version, workers: 1, ops: n,
      ms: Number(t1 - t0) / 1e6, state_sha256: crypto.createHash('sha256').update(st).digest('hex'),
    }));
    process.exit(0);
  }
  const ups = readBatch(file);
  const dw = process.argv[3] === 'diff' ? Math.max(1, parseInt(process.argv[4] || '1', 10)) : 1;
  if (dw > 1) {  // sync responder on W worker_threads: pair i answered by worker i % W
    const { canonicalUpdate } = require(path.join(__dirname, '..', 'tests', 'golden', 'gen', 'v1.js'));
    const npairs = Math.floor(ups.length / 2);
    const outs = new Array(npairs);
    let done = 0, maxMs = 0;
    for (let w = 0; w < dw; w++) {
      const wk = new Worker(__filename, { workerData: { diff: file, w, W: dw } });
      wk.on('message', (m) => {
        maxMs = Math.max(maxMs, m.ms);
        m.outs.forEach((o, k) => { outs[w + k * dw] = Buffer.from(o); });
        if (++done === dw) {
          const h = crypto.createHash('sha256');
          let bytes = 0;
          for (const o of outs) { h.update(canonicalUpdate(o)); bytes += o.length; }
          console.log(JSON.stringify({
            available: true, yjs: '13.5.16', lib0: '0.2.42', node: process.version, workers: dw,
            cpus: require('os').cpus().length, ms: maxMs, pairs: npairs, out_bytes: bytes, out_sha256: h.digest('hex'),
          }));
        }
      });
    }
    return;
  }
  if (process.argv[3] === 'diff') {  // sync responder: (update, sv) pairs, Y.diffUpdate each, one core
    const { canonicalUpdate } = require(path.join(__dirname, '..', 'tests', 'golden', 'gen', 'v1.js'));
    const outs = [];
    const t0 = process.hrtime.bigint();
    for (let i = 0; i + 1 < ups.length; i += 2) outs.push(Y.diffUpdate(ups[i], ups[i + 1]));
    const t1 = process.hrtime.bigint();
    const h = crypto.createHash('sha256');
    let bytes = 0;
    for (const o of outs) { h.update(canonicalUpdate(o)); bytes += o.length; }
    console.log(JSON.stringify({
      available: true, yjs: '13.5.16', lib0: '0.2.42', node: process.version, workers: 1,
      ms: Number(t1 - t0) / 1e6, pairs: outs.length, out_bytes: bytes, out_sha256: h.digest('hex'),
    }));
    process.exit(0);
  }
  if (workers === 1) {
    const r = runOnce(Y, ups);
    const { canonicalUpdate } = require(path.join(__dirname, '..', 'tests', 'golden', 'gen', 'v1.js'));
    const canon = canonicalUpdate(r.out);
    console.log(JSON.stringify({
      available: true, yjs: '13.5.16', lib0: '0.2.42', node: process.version, workers: 1,
      ms: r.ms, out_bytes: r.out.length, out_sha256: crypto.createHash('sha256').update(canon).digest('hex'),
    }));
  } else {
    let done = 0, maxMs = 0;
    for (let w = 0; w < workers; w++) {
      const wk = new Worker(__filename, { workerData: { file } });
      wk.on('message', (m) => {
        maxMs = Math.max(maxMs, m.ms);
        if (++done === workers) {
          console.log(JSON.stringify({ available: true, yjs: '13.5.16', lib0: '0.2.42', node: process.version, workers, ms: maxMs }));
        }
      });
    }
  }
} else if (workerData.diff) {  // sync-responder worker: pairs i with i % W == w
  const Y = load();
  const ups = readBatch(workerData.diff);
  const { w, W } = workerData;
  const outs = [];
  const t0 = process.hrtime.bigint();  // the worker's own Y.diffUpdate calls (load / parse excluded)
  for (let i = w; 2 * i + 1 < ups.length; i += W) outs.push(Y.diffUpdate(ups[2 * i], ups[2 * i + 1]));
  const ms = Number(process.hrtime.bigint() - t0) / 1e6;
  parentPort.postMessage({ ms, outs });
} else if (workerData.fleet) {  // fleet worker: documents d with d % W == w
  const Y = load();
  const { canonicalUpdate } = require(path.join(__dirname, '..', 'tests', 'golden', 'gen', 'v1.js'));
  const b = fs.readFileSync(workerData.fleet);
  const n = b.readUInt32LE(0);
  const { w, W, nDocs } = workerData;
  const docs = new Map();
  let p = 4;
  const mine = [];
  for (let i = 0; i < n; i++) {
    const d = b.readUInt32LE(p), len = b.readUInt32LE(p + 4);
    if (d % W === w) mine.push([d, new Uint8Array(b.buffer, b.byteOffset + p + 8, len)]);
    p += 8 + len;
  }
  const t0 = process.hrtime.bigint();  // the worker's own work: applies + encodes (load / parse excluded)
  for (const [d, u] of mine) {
    let doc = docs.get(d);
    if (!doc) { doc = new Y.Doc(); doc.clientID = 0x7ffffff0; docs.set(d, doc); }
    Y.applyUpdate(doc, u);
  }
  const states = [];
  for (let d = w; d < nDocs; d += W) {
    const doc = docs.get(d) || new Y.Doc();
    states.push(Y.encodeStateAsUpdate(doc));
  }
  const ms = Number(process.hrtime.bigint() - t0) / 1e6;
  parentPort.postMessage({ ms, states: states.map((st) => crypto.createHash('sha256').update(canonicalUpdate(st)).digest('hex')) });
} else {
  const Y = load();
  const r = runOnce(Y, readBatch(workerData.file));
  parentPort.postMessage({ ms: r.ms });
}
