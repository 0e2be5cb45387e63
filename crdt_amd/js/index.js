// crdt_amd/js/index.js — the `Y` object @ypear/crdt receives through `router.options.Y`
// (reference crdt.js:175-180), backed by the MI355X engine through the Node-API addon.
//
//   const Y = require('crdt_amd/js');  router.updateOptions({ Y });
//
// Exposes the Yjs functions the reference calls (SURVEY.md §8(b)): new Y.Doc(), Y.applyUpdate,
// Y.encodeStateAsUpdate(doc[, sv]), Y.encodeStateVector, Y.mergeUpdates, Y.diffUpdate, plus the
// batch entry Y.applyUpdates.
// Errors are thrown as Error objects whose `message` carries the engine's text (crdt.js:38-39
// only reads e.message). There is no CPU fallback: without an MI355X every call throws.
'use strict';
const path = require('path');

const binding = require(path.join(__dirname, 'ycrdt.node'));

let nextClient = null; // deterministic clientIDs for tests (Yjs draws a random uint32, Y@12285)

function randomClientId() {
  if (nextClient !== null) return nextClient++ >>> 0;
  return require('crypto').randomBytes(4).readUInt32LE(0);
}

class Doc {
  constructor(opts = {}) {
    this.clientID = opts.clientID !== undefined ? opts.clientID >>> 0 : randomClientId();
    this._h = binding.docCreate(this.clientID);
  }
}

function applyUpdate(doc, update) {
  binding.applyUpdates(doc._h, update);
}

function applyUpdates(doc, updates) {
  binding.applyUpdates(doc._h, updates);
}

function encodeStateAsUpdate(doc, encodedTargetStateVector) {
  return binding.encodeStateAsUpdate(doc._h, encodedTargetStateVector);
}

function encodeStateVector(doc) {
  return binding.encodeStateVector(doc._h);
}

module.exports = {
  Doc,
  applyUpdate,
  applyUpdates,
  encodeStateAsUpdate,
  encodeStateVector,
  mergeUpdates: (updates) => binding.mergeUpdates(updates),
  diffUpdate: (update, sv) => binding.diffUpdate(update, sv),
  lastStats: (doc) => binding.lastStats(doc._h),
  version: binding.version,
  setDevice: binding.setDevice,
  _setNextClientId: (c) => { nextClient = c; },
};
