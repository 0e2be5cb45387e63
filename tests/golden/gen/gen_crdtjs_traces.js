#!/usr/bin/env node
// crdt.js-driven trace fixtures (TEST INFRASTRUCTURE ONLY; runs in the build container, never on
// the GPU box, and nothing of crdt.js is committed or shipped).
//
// crdt.js itself (/root/reference/crdt.js) is run by peers on an in-process fake router (SURVEY.md
// §4: `alow` delivering through setImmediate) against the in-image Yjs 13.5.16, with a RECORDING
// `Y` handed in through router.options.Y (crdt.js:175-180, the seam the engine plugs into). Every
// Y.* call crdt.js makes — new Y.Doc, getMap / getArray, YMap set / get / has / delete / toJSON,
// new Y.Array, YArray insert / push / unshift / delete / toArray / toJSON, doc.transact,
// Y.applyUpdate, Y.encodeStateAsUpdate, Y.encodeStateVector — is logged with its arguments and
// its result (the wire updates, the state vectors, every toJSON crdt.c is built from). The crdt.c
// snapshots of every peer after every API call are logged too. tests/js/napi_check.js `trace`
// replays the call log through crdt_amd/js on the GPU and compares every result.
//
// crdt.js needs Node >= 14 (optional chaining, SURVEY D11); a lowered copy is written to a temp
// directory with the five `?.` sites rewritten (exact text matches, or the script fails), next to an
// in-memory `level` module; two scenarios persist one peer in it and restart it (LevelDB replay).
//
// Usage: node gen_crdtjs_traces.js <out_dir>   → <out_dir>/crdtjs_traces.json
'use strict';
const fs = require('fs');
const os = require('os');
const path = require('path');
const { loadYjs } = require('./load_yjs.js');

const Yjs = loadYjs();
const REF = '/root/reference/crdt.js';
const hex = (u) => Buffer.from(u).toString('hex');

// ---------------------------------------------------------------- lowered crdt.js in a temp dir
function loweredCrdt() {
  let src = fs.readFileSync(REF, 'utf8');
  const sites = [
    ['if (!router?.isYpearRouter)', 'if (!(router && router.isYpearRouter))'],
    ['if (router.options.cache?.[options.topic])', 'if (router.options.cache && router.options.cache[options.topic])'],
    ['if (!router.options.cache?.[topic].peerStateVectors)', 'if (!(router.options.cache && router.options.cache[topic].peerStateVectors))'],
    ['target = h[name]?.[key];', 'target = h[name] == null ? undefined : h[name][key];'],
  ];
  for (const [a, b] of sites) {
    const n = src.split(a).length - 1;
    if (n < 1) throw new Error('lowering site not found: ' + a);
    src = src.split(a).join(b);
  }
  if (src.includes('?.')) throw new Error('an optional chain is left');
  const dir = fs.mkdtempSync(path.join(os.tmpdir(), 'crdtjs-'));
  fs.mkdirSync(path.join(dir, 'node_modules', 'level'), { recursive: true });
  // in-memory LevelDB (SURVEY.md §4: get / batch / createReadStream({gt, lt}) / close, notFound
  // errors flagged), shared across crdt.js restarts through a process-global map
  fs.writeFileSync(path.join(dir, 'node_modules', 'level', 'index.js'), `
const { EventEmitter } = require('events');
const stores = global.__fakeLevel || (global.__fakeLevel = new Map());
module.exports = function level(p) {
  let m = stores.get(p);
  if (!m) stores.set(p, (m = new Map()));
  return {
    async get(k) { if (!m.has(k)) { const e = new Error('NotFound: ' + k); e.notFound = true; throw e; } return m.get(k); },
    async put(k, v) { m.set(k, Buffer.from(v)); },
    async batch(ops) { for (const o of ops) { if (o.type === 'put') m.set(o.key, Buffer.from(o.value)); else m.delete(o.key); } },
    createReadStream({ gt, lt }) {
      const e = new EventEmitter();
      setImmediate(() => { for (const k of [...m.keys()].sort()) if (k > gt && k < lt) e.emit('data', { key: k, value: m.get(k) }); e.emit('end'); });
      return e;
    },
    async close() {},
  };
};
`);
  fs.writeFileSync(path.join(dir, 'crdt.js'), src);
  return { dir, crdt: require(path.join(dir, 'crdt.js')) };
}

// ---------------------------------------------------------------- the recording Y
const log = [];
let nDocs = 0;
let nextClient = 2001;
const jsonOf = (v) => (v === undefined ? { undef: true } : { v: JSON.parse(JSON.stringify(v)) });

function wrapType(t, ref) {
  const isMap = t instanceof Yjs.Map;
  return new Proxy(t, {
    get(target, prop) {
      if (prop === '__ref') return ref;
      if (prop === '__raw') return target;
      if (prop === 'length' && !isMap) {
        const r = target.length;
        log.push({ op: 'array.length', ref, result: r });
        return r;
      }
      const f = target[prop];
      if (typeof f !== 'function') return f;
      const name = (isMap ? 'map.' : 'array.') + String(prop);
      return (...args) => {
        const rec = { op: name, ref };
        if (prop === 'set') {
          rec.key = args[0];
          if (args[1] instanceof Yjs.AbstractType) rec.type = args[1] instanceof Yjs.Array ? 'array' : 'map';
          else rec.value = jsonOf(args[1]);
          const raw = args[1] && args[1].__raw ? args[1].__raw : args[1];
          const r = target.set(args[0], raw);
          log.push(rec);
          return rec.type ? wrapType(r, { ...ref, key: args[0], kind: rec.type }) : r;
        }
        if (prop === 'get') {
          rec.key = args[0];
          const r = target.get(args[0]);
          if (r instanceof Yjs.AbstractType) {
            rec.result = { type: r instanceof Yjs.Array ? 'array' : 'map' };
            log.push(rec);
            return wrapType(r, { ...ref, key: args[0], kind: rec.result.type });
          }
          rec.result = jsonOf(r);
          log.push(rec);
          return r;
        }
        if (prop === 'observe' || prop === 'unobserve') { log.push(rec); return f.apply(target, args); }
        rec.args = JSON.parse(JSON.stringify(args));
        const r = f.apply(target, args);
        if (['toJSON', 'toArray', 'has'].includes(prop)) rec.result = jsonOf(r);
        log.push(rec);
        return r;
      };
    },
  });
}

class RDoc extends Yjs.Doc {
  constructor(opts) {
    super(opts);
    this.clientID = nextClient;
    nextClient += 7;
    this.__id = 'd' + nDocs++;
    log.push({ op: 'doc', doc: this.__id, client: this.clientID });
  }
  getMap(name = '') { log.push({ op: 'getMap', doc: this.__id, name }); return wrapType(super.getMap(name), { doc: this.__id, root: name, kind: 'map' }); }
  getArray(name = '') { log.push({ op: 'getArray', doc: this.__id, name }); return wrapType(super.getArray(name), { doc: this.__id, root: name, kind: 'array' }); }
  transact(f, origin) { log.push({ op: 'transact', doc: this.__id }); return super.transact(f, origin); }
}

const Yrec = {
  Doc: RDoc,
  Array: class extends Yjs.Array {},
  Map: Yjs.Map,
  AbstractType: Yjs.AbstractType,
  applyUpdate(doc, u) { log.push({ op: 'applyUpdate', doc: doc.__id, update: hex(u) }); return Yjs.applyUpdate(doc, u); },
  encodeStateAsUpdate(doc, sv) {
    const r = Yjs.encodeStateAsUpdate(doc, sv);
    log.push({ op: 'encodeStateAsUpdate', doc: doc.__id, sv: sv ? hex(sv) : null, result: hex(r) });
    return r;
  },
  encodeStateVector(doc) {
    const r = Yjs.encodeStateVector(doc);
    log.push({ op: 'encodeStateVector', doc: doc.__id, result: hex(r) });
    return r;
  },
};

// ---------------------------------------------------------------- fake router (SURVEY.md §4)
function makeRouter(bus, name, publicKey) {
  const r = {
    isYpearRouter: true,
    options: { username: name, publicKey, networkName: 'trace', cache: {}, Y: Yrec },
    started: false,
    peers: {},
    updateOptions(o) { Object.assign(r.options, o); },
    updateOptionsCache(o) { Object.assign(r.options.cache, o); },
    async start() { r.started = true; },
    async alow(topic, handler) {
      let t = bus.get(topic);
      if (!t) bus.set(topic, (t = new Map()));
      t.set(publicKey, handler);
      const deliver = (h, d) => new Promise((res) => setImmediate(async () => { await h(d); res(); }));
      const others = () => [...t.entries()].filter(([k]) => k !== publicKey).map(([, h]) => h);
      const propagate = async (d) => { for (const h of others()) await deliver(h, d); };
      const toPeer = async (pk, d) => { const h = t.get(pk); if (h) await deliver(h, d); };
      return [propagate, propagate, propagate, toPeer];
    },
  };
  return r;
}

function rng(seed) {
  let a = seed >>> 0;
  const r = () => { a = (a + 0x6d2b79f5) | 0; let t = Math.imul(a ^ (a >>> 15), 1 | a); t = (t + Math.imul(t ^ (t >>> 7), 61 | t)) ^ t; return ((t ^ (t >>> 14)) >>> 0) / 4294967296; };
  return { r, int: (n) => Math.floor(r() * n) };
}

const snap = (peer, api) => log.push({ op: 'crdt.c', peer, c: JSON.parse(JSON.stringify(api.c)) });

// one scenario: `npeers` crdt.js instances on one topic, `nops` seeded API calls. With `persist`,
// peer 0 stores every update in (fake) LevelDB (CRDTPersistence.storeUpdate validates it through two
// scratch docs, crdt.js:30-75) and, after 2/3 of the ops, restarts from it: getYDoc replays every
// stored update into a fresh doc (crdt.js:79-98) and the cache is rebuilt from the 'ix' map.
async function scenario(crdt, seed, npeers, nops, persist = false) {
  const start = log.length;
  const bus = new Map();
  const g = rng(seed);
  const peers = [];
  const opts = (i) => (persist && i === 0 ? { topic: 'trace' + seed, leveldb: 'lvl' + seed } : { topic: 'trace' + seed });
  for (let i = 0; i < npeers; i++) peers.push(await crdt(makeRouter(bus, 'u' + i, 'pk' + i), opts(i)));
  const val = () => { const k = g.int(5); return k === 0 ? g.int(1000) : k === 1 ? 'v' + g.int(100) : k === 2 ? { n: g.int(9), s: 'x' } : k === 3 ? [g.int(5), 'y'] : g.r() < 0.5; };
  for (let i = 0; i < nops; i++) {
    if (persist && i === Math.floor((2 * nops) / 3)) {  // restart peer 0 from its LevelDB
      log.push({ op: 'api', peer: 0, n: i, restart: true });
      peers[0] = await crdt(makeRouter(bus, 'u0', 'pk0'), opts(0));
      snap(0, peers[0]);
    }
    const p = g.int(npeers), api = peers[p];
    const x = g.r();
    log.push({ op: 'api', peer: p, n: i });
    if (x < 0.06) await api.map(['users', 'cfg'][g.int(2)]);
    else if (x < 0.10) await api.array(['messages', 'log'][g.int(2)]);
    else if (x < 0.45) await api.set(['users', 'cfg'][g.int(2)], 'k' + g.int(12), val());
    else if (x < 0.55) await api.del('users', 'k' + g.int(12));
    else if (x < 0.72) await api.push('messages', [val()]);
    else if (x < 0.80) {
      const n = (api.c.messages || []).length;
      await api.insert('messages', [val(), val()].slice(0, 1 + g.int(2)), g.int(n + 1));
    } else if (x < 0.84) await api.unshift('messages', [val()]);  // non-batch: re-encodes only (D2)
    else if (x < 0.88) await api.cut('log', 0, 1);                 // non-batch: re-encodes only (D2)
    else {  // a batch: queued ops, one transaction, one propagate (crdt.js:329-355)
      const n = (api.c.log || []).length;
      api.set('cfg', 'b' + g.int(4), val(), true);
      api.push('log', [val()], true);
      api.unshift('log', [val()], true);
      if (n > 1) api.cut('log', g.int(n - 1), 1, true);
      await api.execBatch();
      await new Promise((res) => setTimeout(res, 5));
    }
    await new Promise((res) => setImmediate(res));
    for (let q = 0; q < npeers; q++) snap(q, peers[q]);
  }
  return { name: `crdtjs_s${seed}_p${npeers}_n${nops}` + (persist ? '_leveldb' : ''), peers: npeers, calls: log.slice(start) };
}

async function main() {
  const out = process.argv[2] || path.join(__dirname, '..');
  const { dir, crdt } = loweredCrdt();
  process.chdir(dir);  // CRDTPersistence mkdirs its storage path
  let t = 1700000000000;
  Date.now = () => t++;  // LevelDB keys carry Date.now(): distinct, ordered, reproducible
  const origLog = console.log;
  console.log = () => {};  // crdt.js logs every update
  const cases = [];
  try {
    for (const [seed, np, n, persist] of [[1, 2, 60], [2, 3, 80], [3, 2, 150], [4, 4, 60], [5, 2, 90, true], [6, 3, 60, true]]) {
      log.length = 0;
      cases.push(await scenario(crdt, seed, np, n, persist));
    }
  } finally {
    console.log = origLog;
  }
  const f = path.join(out, 'crdtjs_traces.json');
  fs.writeFileSync(f, JSON.stringify({ generator: 'tests/golden/gen/gen_crdtjs_traces.js', yjs: '13.5.16', cases }));
  let calls = 0;
  for (const c of cases) calls += c.calls.length;
  console.log(f, cases.length, 'scenarios', calls, 'recorded calls');
  process.exit(0);
}

main().catch((e) => { console.error(e); process.exit(1); });
