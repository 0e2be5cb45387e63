// crdt_amd/js/any.js — lib0 0.2.42 `any` value codec (writeAny L0@8251 / readAny L0@1937), the
// encoding Yjs uses for ContentAny (YMap.set / YArray.insert values). The facade writes every
// JS value the reference hands to YMap.set / YArray.insert with encodeAny and passes the bytes
// through the C ABI; decodeAny is the inverse (used by the facade tests).
'use strict';

function pushVu(o, n) {
  while (n > 127) { o.push(0x80 | (n & 127)); n = Math.floor(n / 128); }
  o.push(n & 127);
}
function pushStr(o, s) {
  const b = Buffer.from(s, 'utf8');
  pushVu(o, b.length);
  for (const x of b) o.push(x);
}
// lib0 0.2.42 writeVarInt: sign bit 0x40 in the first byte, six value bits, then 7-bit groups
// shifted with `>>>=` (32-bit), as the bundle does
function pushVi(o, num) {
  const neg = num < 0 || Object.is(num, -0);
  if (neg) num = -num;
  o.push((num > 63 ? 0x80 : 0) | (neg ? 0x40 : 0) | (num & 63));
  num >>>= 6;
  while (num > 0) { o.push((num > 127 ? 0x80 : 0) | (num & 127)); num >>>= 7; }
}
const f32 = new DataView(new ArrayBuffer(4));
const f64 = new DataView(new ArrayBuffer(8));

function writeAny(o, v) {
  switch (typeof v) {
    case 'string': o.push(119); pushStr(o, v); return;
    case 'number':
      if (Number.isInteger(v) && v <= 0x7fffffff) { o.push(125); pushVi(o, v); return; }
      f32.setFloat32(0, v);
      if (f32.getFloat32(0) === v) { o.push(124); for (let i = 0; i < 4; i++) o.push(f32.getUint8(i)); return; }
      f64.setFloat64(0, v); o.push(123); for (let i = 0; i < 8; i++) o.push(f64.getUint8(i));
      return;
    case 'bigint':
      f64.setBigInt64(0, v); o.push(122); for (let i = 0; i < 8; i++) o.push(f64.getUint8(i));
      return;
    case 'boolean': o.push(v ? 120 : 121); return;
    case 'object':
      if (v === null) { o.push(126); return; }
      if (Array.isArray(v)) { o.push(117); pushVu(o, v.length); for (const e of v) writeAny(o, e); return; }
      if (v instanceof Uint8Array) { o.push(116); pushVu(o, v.length); for (const x of v) o.push(x); return; }
      { const ks = Object.keys(v); o.push(118); pushVu(o, ks.length); for (const k of ks) { pushStr(o, k); writeAny(o, v[k]); } }
      return;
    default: o.push(127); // undefined (and functions / symbols, as lib0 does)
  }
}

// values → concatenated encodings (one ContentAny of `values.length` elements)
function encodeAny(values) {
  const o = [];
  for (const v of values) writeAny(o, v);
  return Uint8Array.from(o);
}

function decodeAny(bytes) {
  const b = bytes;
  let p = 0;
  const vu = () => { let n = 0, m = 1, r; do { r = b[p++]; n += (r & 127) * m; m *= 128; } while (r >= 128); return n; };
  const str = () => { const n = vu(); const s = Buffer.from(b.buffer, b.byteOffset + p, n).toString('utf8'); p += n; return s; };
  const dv = new DataView(b.buffer, b.byteOffset, b.byteLength);
  const one = () => {
    const tag = b[p++];
    switch (tag) {
      case 127: return undefined;
      case 126: return null;
      case 125: {
        let r = b[p++]; let num = r & 63; const sign = r & 64 ? -1 : 1; let m = 64;
        while (r & 128) { r = b[p++]; num += (r & 127) * m; m *= 128; }
        return sign * num;
      }
      case 124: { const x = dv.getFloat32(p); p += 4; return x; }
      case 123: { const x = dv.getFloat64(p); p += 8; return x; }
      case 122: { const x = dv.getBigInt64(p); p += 8; return x; }
      case 121: return false;
      case 120: return true;
      case 119: return str();
      case 118: { const n = vu(); const o = {}; for (let i = 0; i < n; i++) { const k = str(); o[k] = one(); } return o; }
      case 117: { const n = vu(); const a = []; for (let i = 0; i < n; i++) a.push(one()); return a; }
      case 116: { const n = vu(); const x = Uint8Array.from(b.subarray(p, p + n)); p += n; return x; }
      default: throw new Error('Integer out of range!');
    }
  };
  const out = [];
  while (p < b.length) out.push(one());
  return out;
}

module.exports = { writeAny, encodeAny, decodeAny };
