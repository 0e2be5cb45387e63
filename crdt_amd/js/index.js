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
// changed the type, after the transaction (cleanupTransactions Y@31804). The facade compares
// the observed type's toJSON before and after each transaction and, when it differs, calls the
// observer with (event, transaction); event carries target/currentTarget and, for maps,
// keysChanged + changes.keys ({action, oldValue}) as YMapEvent does. Array deltas are not
// computed (`changes.delta` is empty): the reference forwards the event untouched.
function snapshotObserved(doc) {
  if (!doc._observed.size) return null;
  const snap = new Map();
  for (const t of doc._observed) snap.set(t, JSON.stringify(t.toJSON()));
  return snap;
}
function fireObservers(doc, before, local) {
  if (!before) return;
  const transaction = { doc, local, origin: null };
  for (const [t, old] of before) {
    if (!t._observers.length) continue;
    const nowJson = t.toJSON();
    const now = JSON.stringify(nowJson);
    if (now === old) continue;
    const event = { target: t, currentTarget: t, transaction, changes: { added: new Set(), deleted: new Set(), delta: [], keys: new Map() } };
    if (t instanceof YMap) {
      const a = JSON.parse(old), b = nowJson;
      const keys = new Set([...Object.keys(a), ...Object.keys(b)]);
      event.keysChanged = new Set();
      for (const k of keys) {
        const ina = Object.prototype.hasOwnProperty.call(a, k), inb = Object.prototype.hasOwnProperty.call(b, k);
        if (ina && inb && JSON.stringify(a[k]) === JSON.stringify(b[k])) continue;
        event.keysChanged.add(k);
        event.changes.keys.set(k, { action: !ina ? 'add' : !inb ? 'delete' : 'update', oldValue: ina ? a[k] : undefined });
      }
    }
    for (const f of t._observers.slice()) f(event, transaction);
  }
}
// runs one mutation of `doc`; observers fire after it unless a transaction is open
function mutate(doc, fn) {
  if (doc._txn) return fn();
  const before = snapshotObserved(doc);
  const r = fn();
  fireObservers(doc, before, true);
  return r;
}

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
  observe(f) { this._observers.push(f); if (this.doc) this.doc._observed.add(this); }
  unobserve(f) {
    this._observers = this._observers.filter((g) => g !== f);
    if (this.doc && !this._observers.length) this.doc._observed.delete(this);
  }
}

class YMap extends AbstractType {
  toJSON() {
    const h = this._bound();
    if (this._pkey === null) return JSON.parse(binding.docJson(h, this._root, 0));
    const v = JSON.parse(binding.docJson(h, this._root, 0))[this._pkey];
    return v && typeof v === 'object' && !Array.isArray(v) ? v : {};
  }
  // per-key reads go to the view's hash index (no toJSON of the whole map per call)
  has(key) { return binding.mapHas(this._bound(), this._root, this._pkey, key); }
  get(key) {
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
  get size() { return binding.mapSize(this._bound(), this._root, this._pkey); }
}

class YArray extends AbstractType {
  constructor() { super(); this._prelim = []; }
  toJSON() {
    const h = this._bound();
    if (this._pkey === null) return JSON.parse(binding.docJson(h, this._root, 1));
    const v = JSON.parse(binding.docJson(h, this._root, 0))[this._pkey];
    return Array.isArray(v) ? v : [];
  }
  toArray() { return this.toJSON(); }
  get length() { return this.doc ? binding.arrayLength(this._bound(), this._root, this._pkey) : this._prelim.length; }
  get(index) {
    if (!this.doc) return this._prelim[index];
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
    const before = snapshotObserved(this);
    this._txn = 1;
    try {
      return f({ doc: this, origin, local: true });
    } finally {
      this._txn = 0;
      fireObservers(this, before, true);
    }
  }
  destroy() {}
}

function applyUpdate(doc, update) {
  mutate(doc, () => binding.applyUpdates(doc._h, update));
}

// fleet ingest: Y.applyUpdate(docs[i], updates[i]) for every i, one device pass (not in Yjs)
function applyUpdatesMulti(docs, updates) {
  const before = docs.map((d) => snapshotObserved(d));
  binding.applyUpdatesMulti(docs.map((d) => d._h), updates);
  docs.forEach((d, i) => fireObservers(d, before[i], false));
}
function applyUpdates(doc, updates) {
  mutate(doc, () => binding.applyUpdates(doc._h, updates));
}

function encodeStateAsUpdate(doc, encodedTargetStateVector) {
  return binding.encodeStateAsUpdate(doc._h, encodedTargetStateVector);
}

function encodeStateVector(doc) {
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
  version: binding.version,
  setDevice: binding.setDevice,
  _setNextClientId: (c) => { nextClient = c; },
};
