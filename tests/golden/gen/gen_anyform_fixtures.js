#!/usr/bin/env node
// `any` encodings lib0's writeAny never produces, but readAny accepts (TEST INFRASTRUCTURE ONLY;
// runs in the build container against the in-image Yjs 13.5.16 + lib0 0.2.42). Yjs keeps `any`
// content as JS values and writes them back with writeAny, so its bytes come out in writeAny's
// form: integer-valued floats become varints, float64s that float32 holds become float32, NaN
// becomes 0x7FF8000000000000, overlong varuints / varints shrink, positive varints past
// 0x7FFFFFFF become floats. Object keys follow Object.keys order (array indices first), a repeated
// key keeps its first place with its last value, "__proto__" sets the prototype — the engine
// rewrites such values (round 6); what it still refuses is listed with `refused: true`.
//
// Every update is one YMap set on root 'users' by client 77, hand-written:
//   [1 section][1 struct][client 77][clock 0] info=0x28 (Any, parentSub) parentInfo=1 'users'
//   key count=1 <value bytes> [empty delete set]
// Usage: node gen_anyform_fixtures.js <out_dir>  ->  <out_dir>/anyform.json
'use strict';
const fs = require('fs');
const path = require('path');
const { loadYjs } = require('./load_yjs.js');
const { canonicalUpdate, canonicalSv, hex } = require('./v1.js');

const Y = loadYjs();

const vs = (s) => { const b = Buffer.from(s, 'utf8'); return [b.length, ...b]; };
const f64 = (x) => { const b = Buffer.alloc(8); b.writeDoubleBE(x); return [...b]; };
const f32 = (x) => { const b = Buffer.alloc(4); b.writeFloatBE(x); return [...b]; };
const update = (key, value, client = 77) => Uint8Array.from([1, 1, client, 0, 0x28, 1, ...vs('users'), ...vs(key), 1, ...value, 0]);

const values = {
  f64_int: [123, ...f64(7)],
  f64_neg_int: [123, ...f64(-5)],
  f64_int_max: [123, ...f64(2147483647)],
  f64_2p31: [123, ...f64(2147483648)],
  f64_1e10: [123, ...f64(1e10)],
  // negative integers between -2^32 and -2^31: writeAny checks `data <= BITS31` (not |data|), so
  // they go out as varints; below -2^32 the engine refuses (writeVarInt's 32-bit shifts)
  f64_neg_2p31: [123, ...f64(-2147483648)],
  f64_neg_2p31m1: [123, ...f64(-2147483649)],
  f64_neg_3e9: [123, ...f64(-3e9)],
  f64_neg_2p32p1: [123, ...f64(-4294967295)],
  f64_1e300: [123, ...f64(1e300)],
  f64_half: [123, ...f64(0.5)],
  f64_inf: [123, ...f64(Infinity)],
  f64_ninf: [123, ...f64(-Infinity)],
  f64_tenth: [123, ...f64(0.1)],
  f64_nan_payload: [123, 0x7f, 0xf8, 0, 0, 0, 0, 0, 1],
  f64_neg_zero: [123, ...f64(-0)],
  f32_int: [124, ...f32(3)],
  f32_nan: [124, 0x7f, 0xc0, 0, 0],
  f32_frac: [124, ...f32(1.25)],
  vi_overlong: [125, 0x87, 0x00],
  vi_overlong_neg: [125, 0xc7, 0x80, 0x00],
  vi_neg_zero: [125, 0x40],
  vi_big_pos: [125, 0x80, 0x80, 0x80, 0x80, 0x0b],          // magnitude past 0x7FFFFFFF
  vi_wrap: [125, 0x81, 0x80, 0x80, 0x80, 0x80, 0x01],       // a group shifted past bit 31 (lib0 wraps)
  str_overlong_len: [119, 0x83, 0x00, 0x61, 0x62, 0x63],
  bytes_overlong_len: [116, 0x82, 0x00, 1, 2],
  arr_overlong_count: [117, 0x82, 0x00, 125, 1, 123, ...f64(2)],
  obj_overlong_key: [118, 1, 0x81, 0x00, 0x6b, 123, ...f64(4)],
  obj_nested_floats: [118, 2, ...vs('a'), 117, 2, 123, ...f64(1), 124, ...f32(0.5), ...vs('b'), 118, 1, ...vs('c'), 123, ...f64(0.1)],
  bigint: [122, 0, 0, 0, 0, 0, 0, 0, 9],
  obj_index_keys_out_of_order: [118, 2, ...vs('b'), 125, 1, ...vs('2'), 125, 2],
  obj_proto_key: [118, 1, ...vs('__proto__'), 125, 1],
  // round 6: object key semantics rewritten on the device (yc_parse.h any_content_canon), not refused
  obj_dup_keys: [118, 3, ...vs('a'), 125, 1, ...vs('b'), 125, 2, ...vs('a'), 125, 3],
  obj_dup_keys_nested: [118, 2, ...vs('x'), 117, 2, 118, 2, ...vs('k'), 125, 1, ...vs('k'), 119, ...vs('v'), 125, 9, ...vs('x'), 118, 2, ...vs('q'), 126, ...vs('q'), 127],
  obj_index_keys_nested: [117, 2, 118, 3, ...vs('z'), 125, 1, ...vs('10'), 125, 2, ...vs('2'), 117, 1, 118, 2, ...vs('b'), 120, ...vs('0'), 121, 125, 4],
  obj_proto_object: [118, 3, ...vs('a'), 125, 1, ...vs('__proto__'), 118, 1, ...vs('p'), 125, 7, ...vs('b'), 125, 2],
  obj_proto_null: [118, 2, ...vs('__proto__'), 126, ...vs('c'), 119, ...vs('s')],
  obj_proto_then_index: [118, 3, ...vs('k'), 120, ...vs('__proto__'), 119, ...vs('x'), ...vs('7'), 125, 7],
  obj_many_keys_dup: [118, 10, ...[...Array(9).keys()].flatMap((i) => [...vs('m' + i), 125, i]), ...vs('m4'), 125, 44],
  obj_deep_dup: [118, 2, ...vs('d'), ...[...Array(24).keys()].flatMap(() => [117, 2]), 118, 2, ...vs('a'), 125, 1, ...vs('a'), 125, 2,
    ...[...Array(24).keys()].flatMap(() => [125, 0]), ...vs('d'), 125, 5],
  obj_dup_keys_canon: [118, 2, ...vs('a'), 125, 1, ...vs('ab'), 125, 2],
  // keys whose repeat-mask bits collide ('ab', 'b_') without repeating: tested exactly, left as is
  obj_mask_collision: [118, 2, ...vs('ab'), 125, 1, ...vs('b_'), 125, 2],
  obj_mask_collision_nested: [118, 3, ...vs('ab'), 125, 1, ...vs('b_'), 117, 1, 125, 2, ...vs('z'), 118, 2, ...vs('ab'), 120, ...vs('b_'), 121],
  // still refused: writeVarInt garbles a negative integer past 2^32; a "__proto__" array makes the
  // object pass `instanceof Array` in writeAny
  f64_neg_5e9: [123, ...f64(-5e9)],
  obj_proto_array: [118, 1, ...vs('__proto__'), 117, 1, 125, 1],
};
const refused = new Set(['f64_neg_5e9', 'obj_proto_array']);
// seeded random values in encodings writeAny never produces: objects with repeated keys, array-index
// keys in any order and "__proto__" members (scalar / object / null values), nested up to 5 levels,
// numbers as varint / float32 / float64 whether or not that is writeAny's form, overlong prefixes
{
  let a = 20240611;
  const r = () => { a |= 0; a = (a + 0x6D2B79F5) | 0; let t = Math.imul(a ^ (a >>> 15), 1 | a); t = (t + Math.imul(t ^ (t >>> 7), 61 | t)) ^ t; return ((t ^ (t >>> 14)) >>> 0) / 4294967296; };
  const pick = (xs) => xs[Math.floor(r() * xs.length)];
  const vu = (n, over) => { const o = []; while (n > 127) { o.push(0x80 | (n & 127)); n = Math.floor(n / 128); } o.push(n); if (over) { o[o.length - 1] |= 0x80; o.push(0); } return o; };
  const key = (k) => { const b = Buffer.from(k, 'utf8'); return [...vu(b.length, r() < 0.05), ...b]; };
  const scalar = () => {
    const x = r();
    if (x < 0.15) return [125, ...vu(Math.floor(r() * 200))];
    if (x < 0.3) return [123, ...f64(pick([0.5, 3, -7, 1e10, 0.1, 2147483648, -2147483649, 1.25, NaN, -0]))];
    if (x < 0.4) return [124, ...f32(pick([1.5, 3, -0.25, 7]))];
    if (x < 0.55) { const b = Buffer.from(pick(['', 'x', 'é', 'long string value', '0']), 'utf8'); return [119, ...vu(b.length, r() < 0.05), ...b]; }
    if (x < 0.65) return [pick([126, 127, 120, 121])];
    if (x < 0.7) return [116, 2, 9, 8];
    return [125, ...vu(Math.floor(r() * 5))];
  };
  const value = (d) => {
    const x = r();
    if (d >= 5 || x < 0.4) return scalar();
    const n = Math.floor(r() * 5);
    if (x < 0.6) { const o = [117, ...vu(n)]; for (let i = 0; i < n; i++) o.push(...value(d + 1)); return o; }
    const o = [118, ...vu(n)];
    const used = [];
    for (let i = 0; i < n; i++) {
      let k;
      const y = r();
      if (used.length && y < 0.2) k = pick(used);                                // a repeated key
      else if (y < 0.45) k = String(Math.floor(r() * 12));                        // an array index
      else if (y < 0.5) k = '__proto__';
      else k = pick(['a', 'b', 'name', 'v', 'é', '01', '4294967295', 'ab', 'b_', '']);
      used.push(k);
      let v = value(d + 1);
      if (k === '__proto__' && (v[0] === 116 || v[0] === 117)) v = [126];         // (refused forms: see above)
      o.push(...key(k), ...v);
    }
    return o;
  };
  for (let i = 0; i < 120; i++) values['fuzz_' + i] = value(0);
}

const cases = [];
for (const [name, v] of Object.entries(values)) {
  const u = update('k_' + name, v);
  const d = new Y.Doc(); d.clientID = 5;
  Y.applyUpdate(d, u);
  const other = new Y.Doc(); other.clientID = 33; other.getMap('users').set('x', 1.5);
  const o = Y.encodeStateAsUpdate(other);
  const merged = Y.mergeUpdates([u, o]);
  let st2 = null;
  try { const d2 = new Y.Doc(); d2.clientID = 5; Y.applyUpdate(d2, u); Y.applyUpdate(d2, o); st2 = hex(canonicalUpdate(Y.encodeStateAsUpdate(d2))); } catch (e) { st2 = 'throws: ' + e.message; }
  const diff = Y.diffUpdate(u, new Uint8Array([0]));
  let st = null; let sv = null; let json = null;
  try { st = hex(canonicalUpdate(Y.encodeStateAsUpdate(d))); sv = hex(canonicalSv(Y.encodeStateVector(d)));
        json = name === 'bigint' ? null : JSON.parse(JSON.stringify(d.getMap('users').toJSON())); } catch (e) { st = 'throws: ' + e.message; }
  cases.push({ name, update: hex(u), other: hex(o), refused: refused.has(name),
               state: st, sv, json, merged: hex(canonicalUpdate(merged)), diff: hex(canonicalUpdate(diff)), state_with_other: st2 });
}
const outDir = process.argv[2] || path.join(__dirname, '..');
fs.writeFileSync(path.join(outDir, 'anyform.json'), JSON.stringify({ yjs: '13.5.16', cases }, null, 0));
console.log(`anyform.json: ${cases.length} cases`);
for (const c of cases) console.log(c.name, c.state.length / 2, JSON.stringify(c.json).slice(0, 60));
