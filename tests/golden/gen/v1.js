// Minimal Yjs v1 update parser used by the fixture generator (test infrastructure only).
// Follows the wire format restated in SURVEY.md Appendix A (lib0 varuint/varint/varString/any,
// Yjs readClientsStructRefs Y@19286 / readDeleteSet Y@11105).
'use strict';

class Reader {
  constructor(buf) { this.b = buf; this.p = 0; }
  u8() { if (this.p >= this.b.length) throw new Error('eof'); return this.b[this.p++]; }
  vu() { // lib0 0.2.42 readVarUint: 7-bit groups, little endian, max 35 bits
    let num = 0; let mult = 1;
    for (;;) {
      const r = this.u8();
      num += (r & 0x7f) * mult;
      mult *= 128;
      if (r < 0x80) return num;
      if (mult > 2 ** 35) throw new Error('varuint overflow');
    }
  }
  vi() {
    let r = this.u8();
    let num = r & 0x3f; let mult = 64;
    const neg = (r & 0x40) > 0 ? -1 : 1;
    if ((r & 0x80) === 0) return neg * num;
    for (;;) {
      r = this.u8();
      num += (r & 0x7f) * mult;
      mult *= 128;
      if (r < 0x80) return neg * num;
    }
  }
  bytes(n) { if (this.p + n > this.b.length) throw new Error('eof'); const s = this.b.subarray(this.p, this.p + n); this.p += n; return s; }
  vstr() { const n = this.vu(); return Buffer.from(this.bytes(n)).toString('utf8'); }
  any() {
    const t = this.u8();
    switch (t) {
      case 127: case 126: case 121: case 120: return;
      case 125: this.vi(); return;
      case 124: this.bytes(4); return;
      case 123: case 122: this.bytes(8); return;
      case 119: this.vstr(); return;
      case 118: { const n = this.vu(); for (let i = 0; i < n; i++) { this.vstr(); this.any(); } return; }
      case 117: { const n = this.vu(); for (let i = 0; i < n; i++) this.any(); return; }
      case 116: { const n = this.vu(); this.bytes(n); return; }
      default: throw new Error('bad any tag ' + t);
    }
  }
}

function writeVu(out, n) {
  while (n > 0x7f) { out.push(0x80 | (n & 0x7f)); n = Math.floor(n / 128); }
  out.push(n & 0x7f);
}

// Skips the struct section; returns {end, items, structs, clients}
function skipStructs(r) {
  let items = 0; let structs = 0;
  const nClients = r.vu();
  const clients = [];
  for (let c = 0; c < nClients; c++) {
    const n = r.vu(); const client = r.vu(); let clock = r.vu();
    clients.push(client);
    for (let i = 0; i < n; i++) {
      const info = r.u8();
      const ref = info & 31;
      structs++;
      if (ref === 0 || ref === 10) { const len = r.vu(); if (ref === 0) items += len; clock += len; continue; }
      if (info & 0x80) { r.vu(); r.vu(); }
      if (info & 0x40) { r.vu(); r.vu(); }
      if ((info & 0xc0) === 0) {
        if (r.vu() === 1) r.vstr(); else { r.vu(); r.vu(); }
        if (info & 0x20) r.vstr();
      }
      let len = 1;
      switch (ref) {
        case 1: len = r.vu(); break;
        case 2: { len = r.vu(); for (let k = 0; k < len; k++) r.vstr(); break; }
        case 3: { const n2 = r.vu(); r.bytes(n2); break; }
        case 4: { const s = r.vstr(); len = s.length; break; }
        case 5: r.vstr(); break;
        case 6: r.vstr(); r.vstr(); break;
        case 7: { const tr = r.vu(); if (tr === 3 || tr === 5) r.vstr(); break; }
        case 8: { len = r.vu(); for (let k = 0; k < len; k++) r.any(); break; }
        case 9: r.vstr(); r.any(); break;
        default: throw new Error('bad content ref ' + ref);
      }
      items += len; clock += len;
    }
  }
  return { items, structs, clients };
}

function readDs(r) {
  const n = r.vu();
  const ds = [];
  for (let i = 0; i < n; i++) {
    const client = r.vu(); const k = r.vu(); const ranges = [];
    for (let j = 0; j < k; j++) ranges.push([r.vu(), r.vu()]);
    ds.push([client, ranges]);
  }
  return ds;
}

function writeDs(out, ds) {
  writeVu(out, ds.length);
  for (const [client, ranges] of ds) {
    writeVu(out, client); writeVu(out, ranges.length);
    for (const [c, l] of ranges) { writeVu(out, c); writeVu(out, l); }
  }
}

// 13.5.16 writes DS and SV clients in Map insertion order; 13.6 sorts them descending
// (SURVEY.md App. C items 1-2). Canonical form = descending client order.
function canonicalUpdate(u) {
  const r = new Reader(u);
  skipStructs(r);
  const structEnd = r.p;
  const ds = readDs(r);
  if (r.p !== u.length) throw new Error('trailing bytes in update');
  ds.sort((a, b) => b[0] - a[0]);
  const out = Array.from(u.subarray(0, structEnd));
  writeDs(out, ds);
  return Uint8Array.from(out);
}

function canonicalSv(sv) {
  const r = new Reader(sv);
  const n = r.vu(); const e = [];
  for (let i = 0; i < n; i++) e.push([r.vu(), r.vu()]);
  e.sort((a, b) => b[0] - a[0]);
  const out = []; writeVu(out, e.length);
  for (const [c, k] of e) { writeVu(out, c); writeVu(out, k); }
  return Uint8Array.from(out);
}

function updateStats(u) {
  const r = new Reader(u);
  const s = skipStructs(r);
  readDs(r);
  return s;
}

const hex = (u) => Buffer.from(u).toString('hex');

module.exports = { Reader, writeVu, canonicalUpdate, canonicalSv, updateStats, hex };
