// crdt_amd/js/index.js — the `Y` object @ypear/crdt receives through `router.options.Y`
// (reference crdt.js:175-180), backed by the MI355X engine through the Node-API addon.
//
//   const Y = require('crdt_amd/js');  router.updateOptions({ Y });
//
// Exposes the Yjs surface the reference uses (SURVEY.md §8(b)):
//   new Y.Doc(), doc.getMap / getArray / transact, new Y.Array() (prelim, crdt.js:423),
//   YMap set / get / has / delete / toJSON / observe / unobserve,
//   YArray insert / push / unshift / delete / toJSON / toArray / length / observe / unobserve,
//   Y.applyUpdate, Y.encodeStateAsUpdate(doc[, sv]), Y.encodeStateVector, Y.mergeUpdates,
//   Y.diffUpdate, plus the batch entries Y.applyUpdates (one doc) and Y.applyUpdatesMulti (a fleet).
// Every local op is written by the engine as the Yjs v1 struct a Yjs doc would create, so the
// doc's bytes stay identical to Yjs's (tests/js/napi_check.js `ops`). Values go through the
// lib0 `any` codec (any.js). toJSON reads the device-materialised view (map winners, list order).
// Errors are thrown as Error objects whose `message` carries the engine's text (crdt.js:38-39
// only reads e.message). There is no CPU fallback: without an MI355X every call throws.
'use strict';
const path = require('path');
const { encodeAny } = require('./any.js');

const binding = require(path.join(__dirname, 'ycrdt.node'));

let nextClient = null; // deterministic clientIDs for tests (Yjs draws a random uint32, Y@12285)

function randomClientId() {
  if (nextClient !== null) return nextClient++ >>> 0;
  return require('crypto').randomBytes(4).readUInt32LE(0);
}

const TYPE_ARRAY = 0;
const TYPE_MAP = 1;

// Observers (YMap/YArray.observe, crdt.js:620-656). Yjs calls them once per transaction that
// changed the type, synchronously at its end (cleanupTransactions Y@31804). Two modes:
//  - 'sync' (the default, Yjs's timing): a doc with observers settles at the end of every mutation
//    (Y.applyUpdate, set, insert, delete; a transaction at its end), so each event fires inside the
//    call that caused it — the applied update is merged right away instead of at the next read;
//  - 'deferred' (opt-in: Y.setObserverMode('deferred') or new Y.Doc({observers: 'deferred'})): a
//    mutation only marks the doc; the events fire at the next read of the doc (toJSON, get, has,
//    size, length, encode*) or, if nothing reads it, from setImmediate — whichever comes first — so
//    one batched merge serves a burst of applies, which then yields one event per type with the
//    union of their changes (Yjs: one per transaction).
// Either way an event is computed from one read of each observed type, compared with what its
// previous event delivered (taken when observe() was called). Maps compare the winning item id of every entry
// (ycrdt_map_entries): keysChanged = keys whose winning item changed — a set of the same value is a
// new item, and changes inside a nested type are not the map's (YMap.observe, not observeDeep);
// changes.keys carries {action, oldValue}. Arrays carry changes.delta ([{retain}, {delete},
// {insert}] from the common prefix / suffix of the two arrays, exact for one insert or delete).
function jsonOf(t) {
  if (t instanceof YMap) return JSON.parse(binding.mapEntries(t._bound(), t._root, t._pkey));
  return t.toJSONRaw();
}
function arrayDelta(a, b) {
  let p = 0;
  while (p < a.length && p < b.length && JSON.stringify(a[p]) === JSON.stringify(b[p])) ++p;
  let q = 0;
  while (q < a.length - p && q < b.length - p && JSON.stringify(a[a.length - 1 - q]) === JSON.stringify(b[b.length - 1 - q])) ++q;
  const delta = [];
  if (p) delta.push({ retain: p });
  if (a.length - p - q) delta.push({ delete: a.length - p - q });
  if (b.length - p - q) delta.push({ insert: b.slice(p, b.length - q) });
  return delta;
}
let observerMode = 'sync';
function setObserverMode(mode) {
  if (mode !== 'sync' && mode !== 'deferred') throw new Error("observer mode is 'sync' or 'deferred'");
  observerMode = mode;
}
const syncObservers = (doc) => (doc._obsMode || observerMode) === 'sync';
function markChanged(doc, local) {
  if (!doc._observed.size) return;
  doc._local = doc._dirty ? doc._local && local : local;
  doc._dirty = true;
  if (syncObservers(doc)) { if (!doc._firing) fireObservers(doc); return; }  // (inside a callback: after it)
  if (!doc._timer) doc._timer = setImmediate(() => { doc._timer = null; fireObservers(doc); });
}
function fireObservers(doc) {
  if (!doc._dirty || doc._firing) return;
  doc._firing = true;
  try {
    // sync mode: a callback's own mutations are a transaction of their own, delivered after it
    // (bounded: callbacks that keep mutating end after 100 rounds, the rest at the next read)
    for (let round = 0; doc._dirty && round < 100; ++round) {
      doc._dirty = false;
      fireRound(doc);
      if (!syncObservers(doc)) break;
    }
  } finally {
    doc._firing = false;
  }
}
function fireRound(doc) {
  const transaction = { doc, local: doc._local, origin: null };
  for (const t of Array.from(doc._observed)) {
    if (!t._observers.length) continue;
    const nowJson = jsonOf(t);
    const now = JSON.stringify(nowJson);
    const old = t._seen;
    t._seen = now;
    if (old === undefined || now === old) continue;
    const event = { target: t, currentTarget: t, transaction, changes: { added: new Set(), deleted: new Set(), delta: [], keys: new Map() } };
    const a = JSON.parse(old), b = nowJson;
    if (t instanceof YMap) {  // a, b: {key: [winning item id, value]}
      const keys = new Set([...Object.keys(a), ...Object.keys(b)]);
      event.keysChanged = new Set();
      for (const k of keys) {
        const ina = Object.prototype.hasOwnProperty.call(a, k), inb = Object.prototype.hasOwnProperty.call(b, k);
        if (ina && inb && a[k][0] === b[k][0]) continue;
        event.keysChanged.add(k);
        event.changes.keys.set(k, { action: !ina ? 'add' : !inb ? 'delete' : 'update', oldValue: ina ? a[k][1] : undefined });
      }
      if (!event.keysChanged.size) continue;  // only nested contents changed: not this map's event
    } else {
      event.changes.delta = arrayDelta(a, b);
    }
    event.delta = event.changes.delta;
    for (const f of t._observers.slice()) f(event, transaction);
  }
}
// runs one mutation of `doc`; its observers fire at its end (sync) or at the next read / tick
// (deferred), unless a transaction is open
function mutate(doc, fn, local = true) {
  const r = fn();
  if (!doc._txn) markChanged(doc, local);
  return r;
}
// every read of a doc delivers the pending events first (the state it returns is the one they describe)
function settle(doc) { if (doc && doc._dirty) fireObservers(doc); }

class AbstractType {
  constructor() {
    this.doc = null;
    this._root = null;      // root type name
    this._pkey = null;      // nested: key of root map `_root` that holds this type
    this._observers = [];
  }
  _bound() {
    if (!this.doc) throw new Error('Invalid access: Add Yjs type to a document before reading data.');
    return this.doc._h;
  }
  observe(f) {
    this._observers.push(f);
    if (this.doc) {
      settle(this.doc);
      if (this._seen === undefined) this._seen = JSON.stringify(jsonOf(this));
      this.doc._observed.add(this);
    }
  }
  unobserve(f) {
    this._observers = this._observers.filter((g) => g !== f);
    if (this.doc && !this._observers.length) { this.doc._observed.delete(this); this._seen = undefined; }
  }
}

class YMap extends AbstractType {
  // the type's own list only (a nested map does not read its root map's JSON)
  toJSONRaw() { return JSON.parse(binding.typeJson(this._bound(), this._root, this._pkey, 0)); }
  toJSON() { settle(this.doc); return this.toJSONRaw(); }
  // per-key reads go to the view's hash index (no toJSON of the whole map per call)
  has(key) { settle(this.doc); return binding.mapHas(this._bound(), this._root, this._pkey, key); }
  get(key) {
    settle(this.doc);
    const h = this._bound();
    if (this._pkey === null) {
      const tr = binding.mapTypeAt(h, this._root, key);
      if (tr === TYPE_ARRAY || tr === TYPE_MAP) return this.doc._nested(this._root, key, tr);
    }
    const j = binding.mapGet(h, this._root, this._pkey, key);
    return j === undefined ? undefined : JSON.parse(j);
  }
  set(key, value) {
    const h = this._bound();
    const d = this.doc;
    if (value instanceof AbstractType) {
      if (value.doc) throw new Error('This type was already integrated');
      if (value._prelim && value._prelim.length) throw new Error('ycrdt: prelim content in new Y.Array() is not supported');
      const tr = value instanceof YArray ? TYPE_ARRAY : TYPE_MAP;
      mutate(d, () => binding.mapSetType(h, this._root, this._pkey, key, tr));
      if (this._pkey !== null) return value;
      // the prelim becomes the integrated type (Yjs returns the same object, now bound)
      value.doc = d; value._root = this._root; value._pkey = key;
      d._types.set(this._root + '\u0000' + key, value);
      if (value._observers.length) d._observed.add(value);
      return value;
    }
    mutate(d, () => binding.mapSet(h, this._root, this._pkey, key, encodeAny([value])));
    return value;
  }
  delete(key) { const h = this._bound(); mutate(this.doc, () => binding.mapDelete(h, this._root, this._pkey, key)); }
  forEach(f) { const j = this.toJSON(); for (const k of Object.keys(j)) f(j[k], k, this); }
  keys() { return Object.keys(this.toJSON())[Symbol.iterator](); }
  get size() { settle(this.doc); return binding.mapSize(this._bound(), this._root, this._pkey); }
}

class YArray extends AbstractType {
  constructor() { super(); this._prelim = []; }
  // the type's own list only (a nested array does not read its root map's JSON)
  toJSONRaw() { return JSON.parse(binding.typeJson(this._bound(), this._root, this._pkey, 1)); }
  toJSON() { settle(this.doc); return this.toJSONRaw(); }
  toArray() { return this.toJSON(); }
  get length() {
    if (!this.doc) return this._prelim.length;
    settle(this.doc);
    return binding.arrayLength(this._bound(), this._root, this._pkey);
  }
  get(index) {
    if (!this.doc) return this._prelim[index];
    settle(this.doc);
    const j = binding.arrayGet(this._bound(), this._root, this._pkey, index);
    return j === undefined ? undefined : JSON.parse(j);
  }
  insert(index, content) {
    if (!this.doc) { this._prelim.splice(index, 0, ...content); return; }
    const h = this._bound();
    mutate(this.doc, () => binding.arrayInsert(h, this._root, this._pkey, index, encodeAny(content), content.length));
  }
  push(content) {
    if (!this.doc) { this._prelim.push(...content); return; }
    this.insert(this.length, content);
  }
  unshift(content) { this.insert(0, content); }
  delete(index, length = 1) {
    const h = this._bound();
    mutate(this.doc, () => binding.arrayDelete(h, this._root, this._pkey, index, length));
  }
  forEach(f) { this.toJSON().forEach((v, i) => f(v, i, this)); }
  map(f) { return this.toJSON().map((v, i) => f(v, i, this)); }
}

class Doc {
  constructor(opts = {}) {
    this.clientID = opts.clientID !== undefined ? opts.clientID >>> 0 : randomClientId();
    this._h = binding.docCreate(this.clientID);
    this._types = new Map();     // root name / root\0key → the type object handed out
    this._observed = new Set();  // types with observers
    this._txn = 0;
    this._dirty = false;         // mutated since the observers last saw it
    this._local = true;
    this._timer = null;
    this._obsMode = opts.observers;  // 'sync' | 'deferred' | undefined (the module's mode)
    if (this._obsMode !== undefined && this._obsMode !== 'sync' && this._obsMode !== 'deferred') throw new Error("observers: 'sync' or 'deferred'");
  }
  _root(name, Cls) {
    let t = this._types.get(name);
    if (!t) {
      t = new Cls(); t.doc = this; t._root = name;
      this._types.set(name, t);
    } else if (!(t instanceof Cls)) {
      throw new Error(`Type with the name ${name} has already been defined with a different constructor`);
    }
    return t;
  }
  _nested(root, key, typeRef) {
    const id = root + '\u0000' + key;
    let t = this._types.get(id);
    const Cls = typeRef === TYPE_ARRAY ? YArray : YMap;
    if (!t || !(t instanceof Cls)) {
      t = new Cls(); t.doc = this; t._root = root; t._pkey = key;
      this._types.set(id, t);
    }
    return t;
  }
  getMap(name = '') { return this._root(name, YMap); }
  getArray(name = '') { return this._root(name, YArray); }
  // doc.transact(fn) (crdt.js:333): the ops inside are applied as they run; observers fire once at
  // the end, as after a Yjs transaction
  transact(f, origin = null) {
    if (this._txn) return f({ doc: this, origin, local: true });
    settle(this);
    this._txn = 1;
    try {
      return f({ doc: this, origin, local: true });
    } finally {
      this._txn = 0;
      markChanged(this, true);
      settle(this);  // one event per transaction, at its end (Yjs cleanupTransactions)
    }
  }
  destroy() {}
}

// Y.applyUpdate: validated now, merged at the next read (observers: see above)
function applyUpdate(doc, update) {
  mutate(doc, () => binding.applyUpdates(doc._h, update), false);
}

// fleet ingest: Y.applyUpdate(docs[i], updates[i]) for every i, one device pass (not in Yjs)
function applyUpdatesMulti(docs, updates) {
  binding.applyUpdatesMulti(docs.map((d) => d._h), updates);
  for (const d of new Set(docs)) markChanged(d, false);
}
function applyUpdates(doc, updates) {
  mutate(doc, () => binding.applyUpdates(doc._h, updates), false);
}

function encodeStateAsUpdate(doc, encodedTargetStateVector) {
  settle(doc);
  return binding.encodeStateAsUpdate(doc._h, encodedTargetStateVector);
}

function encodeStateVector(doc) {
  settle(doc);
  return binding.encodeStateVector(doc._h);
}

module.exports = {
  Doc,
  Map: YMap,
  Array: YArray,
  AbstractType,
  applyUpdate,
  applyUpdates,
  applyUpdatesMulti,
  encodeStateAsUpdate,
  encodeStateVector,
  mergeUpdates: (updates) => binding.mergeUpdates(updates),
  diffUpdate: (update, sv) => binding.diffUpdate(update, sv),
  // batch entry (not in Yjs): [Y.diffUpdate(u, sv) for each pair] in one device pass — the sync
  // responder (crdt.js:286-291) answering many joining peers / topics at once
  diffUpdates: (updates, svs) => binding.diffUpdates(updates, svs),
  // opt-in incremental local-op encode (not in Yjs): the doc's local ops since the previous call as
  // one update, instead of re-encoding the whole doc after every op (crdt.js:347,383,443,...)
  takeLocalUpdate: (doc) => binding.takeLocalUpdate(doc._h),
  trackLocalUpdates: (doc, on = true) => binding.trackLocalUpdates(doc._h, on),
  lastStats: (doc) => binding.lastStats(doc._h),
  setObserverMode,
  version: binding.version,
  setDevice: binding.setDevice,
  _setNextClientId: (c) => { nextClient = c; },
};
