// yc_parse.h — the Yjs v1 / lib0 byte grammar, shared by the gfx950 decoder and the host-side
// update scanner (yc_ingest.cpp), so that both refuse exactly the same inputs.
//
// Compiled by hipcc (as part of yc_common.h, __host__ __device__) and by g++ (plain inline).
#pragma once
#include <cstdint>

#if defined(__HIP__) || defined(__HIPCC__)
#define YC_HD __host__ __device__
#define YC_HDI __host__ __device__ __forceinline__
#else
#define YC_HD
#define YC_HDI inline __attribute__((always_inline))
#endif

#include "yc_num.h"

namespace yc {

// content refs (low 5 bits of the info byte)
enum : uint8_t {
  REF_GC = 0, REF_DELETED = 1, REF_JSON = 2, REF_BINARY = 3, REF_STRING = 4, REF_EMBED = 5,
  REF_FORMAT = 6, REF_TYPE = 7, REF_ANY = 8, REF_DOC = 9, REF_SKIP = 10
};

// ---------------------------------------------------------------- lib0 readers (L0@1937)
// readVarUint: 7-bit groups with 32-bit shift-or accumulation (lib0 0.2.42). A 6th
// continuation byte or running past `end` is "Integer out of range!".
YC_HDI uint32_t rd_vu(const uint8_t* __restrict__ b, uint32_t& p, uint32_t end, bool& ok) {
  uint32_t v = 0;
  uint32_t shift = 0;
#pragma unroll 1
  for (;;) {
    if (p >= end) { ok = false; return 0; }
    uint32_t r = b[p++];
    if (shift < 32) v |= (r & 0x7fu) << shift;
    shift += 7;
    if (r < 0x80u) return v;
    if (shift > 35) { ok = false; return 0; }
  }
}

// readVarInt: sign bit 0x40 in the first byte, 6+7k bits, error past 41 bits.
YC_HDI void skip_vi(const uint8_t* __restrict__ b, uint32_t& p, uint32_t end, bool& ok) {
  if (p >= end) { ok = false; return; }
  uint32_t r = b[p++];
  if (!(r & 0x80u)) return;
  uint32_t shift = 6;
#pragma unroll 1
  for (;;) {
    if (p >= end) { ok = false; return; }
    r = b[p++];
    shift += 7;
    if (r < 0x80u) return;
    if (shift > 41) { ok = false; return; }
  }
}

// A ContentJSON / ContentEmbed / ContentFormat value is JSON.stringify output, decoded by Yjs
// with JSON.parse (Y@71000..): text that cannot start a JSON value (or is empty) makes Yjs throw,
// so the decoder rejects it too. This also lets speculative parses of non-struct bytes fail fast.
YC_HDI bool json_start_ok(uint32_t c) {
  return c == '{' || c == '[' || c == '"' || c == 't' || c == 'f' || c == 'n' || c == 'u' || c == '-' ||
         (c >= '0' && c <= '9') || c == ' ' || c == '\t' || c == '\n' || c == '\r';
}

YC_HDI void skip_bytes(uint32_t& p, uint32_t n, uint32_t end, bool& ok) {
  if (end - p < n) { ok = false; p = end; return; }
  p += n;
}

// lib0 readVarString decodes with decodeURIComponent(escape(bytes)) (L0@1937): anything but
// shortest-form UTF-8 of a scalar value — a stray continuation byte, a truncated sequence, an
// overlong form, a surrogate, a value past U+10FFFF — throws URIError, and Y.applyUpdate with it.
// Every string field of an exactly parsed struct is checked (names, keys, contents, `any` strings
// and object keys); the bytes are in range (the caller skipped them already).
template <class Src>
YC_HDI uint32_t utf8_units(const Src& b, uint32_t p, uint32_t n, bool& ok) {  // UTF-16 code units of valid UTF-8
  const uint32_t e = p + n;
  uint32_t u = 0;
#pragma unroll 1
  while (p < e) {
    if (e - p >= 4 && !(b.w4(p) & 0x80808080u)) { p += 4; u += 4; continue; }  // four ASCII bytes
    const uint32_t c = b.u8(p);
    if (c < 0x80u) { ++p; ++u; continue; }
    uint32_t need, v, lo;
    if ((c & 0xE0u) == 0xC0u) { need = 1; v = c & 0x1Fu; lo = 0x80u; }
    else if ((c & 0xF0u) == 0xE0u) { need = 2; v = c & 0x0Fu; lo = 0x800u; }
    else if ((c & 0xF8u) == 0xF0u) { need = 3; v = c & 0x07u; lo = 0x10000u; }
    else { ok = false; return u; }
    if (e - p - 1 < need) { ok = false; return u; }
    for (uint32_t k = 1; k <= need; ++k) {
      const uint32_t d = b.u8(p + k);
      if ((d & 0xC0u) != 0x80u) { ok = false; return u; }
      v = (v << 6) | (d & 0x3Fu);
    }
    if (v < lo || v > 0x10FFFFu || (v >= 0xD800u && v <= 0xDFFFu)) { ok = false; return u; }
    p += need + 1;
    u += need == 3 ? 2u : 1u;  // a 4-byte sequence is a surrogate pair
  }
  return u;
}
template <class Src>
YC_HDI bool utf8_valid(const Src& b, uint32_t p, uint32_t n) {
  bool ok = true;
  utf8_units(b, p, n, ok);
  return ok;
}
YC_HDI uint32_t le32(const uint8_t* __restrict__ b, uint32_t p) {
  return (uint32_t)b[p] | ((uint32_t)b[p + 1] << 8) | ((uint32_t)b[p + 2] << 16) | ((uint32_t)b[p + 3] << 24);
}
struct PtrSrc {  // utf8_valid over a plain pointer
  const uint8_t* __restrict__ b;
  YC_HDI uint32_t u8(uint32_t p) const { return b[p]; }
  YC_HDI uint32_t w4(uint32_t p) const { return le32(b, p); }
};
// a varString at p: its length, then (UTF8) its text checked; p moves past it
template <bool UTF8, class Src>
YC_HDI uint32_t skip_str(const Src& b, uint32_t& p, uint32_t end, bool& ok) {  // returns the byte length
  const uint32_t n = b.vu(p, end, ok);
  if (!ok) return 0;
  const uint32_t st = p;
  skip_bytes(p, n, end, ok);
  if (UTF8 && ok && !utf8_valid(b, st, n)) ok = false;
  return n;
}

// ---- lib0 writeAny canonical forms (L0@1937: readAny -> JS value -> writeAny). Yjs stores
// `any` content as JS values and writes them back, so an input encoding that is not what writeAny
// produces comes out different: an overlong varuint / varint, an integer-valued float (-> varint
// when <= 0x7FFFFFFF), a float64 that float32 holds exactly (-> float32), a float32 NaN (-> the
// float64 it widens to), a positive varint past 0x7FFFFFFF (-> float32 / float64). Such values are
// flagged ANY_REENCODE and the encoders write them canonically (any_canon below). What needs JS
// object semantics — array-index keys after others or out of order (Object.keys order), the key
// "__proto__" (readAny's obj[key] = v: the prototype setter, no own member), a key that may repeat
// (the last value at the first key's place) — is ANY_KEYS: the struct is rewritten on the device
// before the merge (any_content_canon, yc_decode.hip k_json_canon), as Yjs's decode + writeAny would.
// A repeat is judged by a 64-bit mask of key hashes per object: a false alarm costs a rewrite pass
// that changes nothing. ANY_UNSUP — refused — is left for a negative integer past 2^32 (writeVarInt's
// 32-bit shifts write bytes no reader gets the number back from) and a "__proto__" member holding an
// array or bytes (the object then passes `instanceof Array / Uint8Array` in writeAny).
enum : uint32_t { ANY_REENCODE = 1u, ANY_UNSUP = 2u, ANY_KEYS = 4u };
// the bit of a key in an object's repeat mask (its length and first and last bytes)
YC_HDI uint64_t key_bit(uint32_t n, uint32_t c0, uint32_t c1) { return 1ull << ((n * 7u + c0 * 3u + c1) & 63u); }
YC_HDI uint32_t vu_overlong(const uint8_t* __restrict__ b, uint32_t p0, uint32_t p1) {  // [p0, p1) one varuint
  return (p1 - p0 > 1 && b[p1 - 1] == 0u) ? ANY_REENCODE : 0u;
}
// readVarInt (lib0 0.2.42: 32-bit shifts, so group k lands at bit (6 + 7k) & 31): sign, magnitude
YC_HDI uint32_t vi_decode(const uint8_t* __restrict__ b, uint32_t p0, uint32_t p1, bool& neg) {
  uint32_t r = b[p0], n = r & 0x3Fu, e = 6;
  neg = (r & 0x40u) != 0;
  for (uint32_t q = p0 + 1; q < p1; ++q) { n |= (uint32_t)(b[q] & 0x7Fu) << (e & 31u); e += 7; }
  return n;
}
YC_HDI uint32_t vi_size(uint32_t m) { uint32_t s = 1; m >>= 6; while (m) { ++s; m >>= 7; } return s; }
YC_HDI uint32_t vi_flag(const uint8_t* __restrict__ b, uint32_t p0, uint32_t p1) {
  bool neg;
  const uint32_t m = vi_decode(b, p0, p1, neg);
  if (!neg && m > 0x7FFFFFFFu) return ANY_REENCODE;  // writeAny: a float
  return vi_size(m) == p1 - p0 ? 0u : ANY_REENCODE;  // (a wrapped overlong form is longer too)
}
// the same checks through parse_struct's byte source (the device decoder's LDS window)
template <class S>
YC_HDI uint32_t vu_overlong_at(const S& b, uint32_t p0, uint32_t p1) {
  return (p1 - p0 > 1 && b.u8(p1 - 1) == 0u) ? ANY_REENCODE : 0u;
}
template <class S>
YC_HDI uint32_t vi_flag_at(const S& b, uint32_t p0, uint32_t p1) {
  const uint32_t r = b.u8(p0);
  uint32_t m = r & 0x3Fu, e = 6;
  for (uint32_t q = p0 + 1; q < p1; ++q) { m |= (b.u8(q) & 0x7Fu) << (e & 31u); e += 7; }
  if (!(r & 0x40u) && m > 0x7FFFFFFFu) return ANY_REENCODE;
  return vi_size(m) == p1 - p0 ? 0u : ANY_REENCODE;
}
template <class S>
YC_HDI uint64_t be_at(const S& b, uint32_t p, uint32_t n) {
  uint64_t x = 0;
  for (uint32_t i = 0; i < n; ++i) x = (x << 8) | b.u8(p + i);
  return x;
}
YC_HDI uint32_t be32(const uint8_t* __restrict__ b, uint32_t p) {
  return ((uint32_t)b[p] << 24) | ((uint32_t)b[p + 1] << 16) | ((uint32_t)b[p + 2] << 8) | b[p + 3];
}
YC_HDI uint64_t be64(const uint8_t* __restrict__ b, uint32_t p) { return ((uint64_t)be32(b, p) << 32) | be32(b, p + 4); }
// writeAny(number) of a double: 0 varint, 1 float32, 2 float64, 3 refused (a negative integer
// past 2^32, which writeVarInt's 32-bit arithmetic garbles)
YC_HDI uint32_t num_form(double x) {
  // an integer (finite); the range test comes first: the cast of a NaN, an infinity or a magnitude
  // past 2^63 is undefined (writeAny checks `data <= BITS31`, not |data|: tests/golden/anyform.json
  // pins -2^31 - 1, -3e9 and -2^32 + 1 as varints)
  if (x >= -9.2e18 && x <= 9.2e18 && x == (double)(long long)x) {
    if (x <= 2147483647.0) return x > -4294967296.0 ? 0u : 3u;
  }
  if (x != x) return 2u;  // NaN: float32 does not compare equal
  const float f = (float)x;
  return (double)f == x ? 1u : 2u;
}
YC_HDI double f32_of(uint32_t bits) { union { uint32_t u; float f; } c; c.u = bits; return (double)c.f; }
YC_HDI double f64_of(uint64_t bits) { union { uint64_t u; double d; } c; c.u = bits; return c.d; }
YC_HDI uint32_t f32_flag(uint32_t bits) {
  const double x = f32_of(bits);
  const uint32_t k = num_form(x);
  return k == 3 ? ANY_UNSUP : k == 1 ? 0u : ANY_REENCODE;
}
YC_HDI uint32_t f64_flag(uint64_t bits) {
  const double x = f64_of(bits);
  const uint32_t k = num_form(x);
  if (k == 3) return ANY_UNSUP;
  return k != 2 ? ANY_REENCODE : 0u;  // (a NaN keeps its bits: V8 writes the double it read)
}
// an object key that JS orders first (an array index: "0" or [1-9][0-9]* below 2^32 - 1), or "__proto__"
YC_HDI int64_t key_index(const uint8_t* __restrict__ b, uint32_t p, uint32_t n) {
  if (n == 0 || n > 10 || (n > 1 && b[p] == '0')) return -1;
  uint64_t v = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t c = b[p + i];
    if (c < '0' || c > '9') return -1;
    v = v * 10 + (c - '0');
  }
  return v < 0xFFFFFFFFull ? (int64_t)v : -1;
}
YC_HDI uint32_t fnv_key(const uint8_t* __restrict__ b, uint32_t p, uint32_t n) {
  uint32_t h = 2166136261u;
  for (uint32_t i = 0; i < n; ++i) h = (h ^ b[p + i]) * 16777619u;
  return h;
}
YC_HDI bool key_proto(const uint8_t* __restrict__ b, uint32_t p, uint32_t n) {
  const char* k = "__proto__";
  if (n != 9) return false;
  for (uint32_t i = 0; i < 9; ++i)
    if (b[p + i] != (uint8_t)k[i]) return false;
  return true;
}

// readAny (L0@1937 B): iterative skip with an explicit container stack of depth DEPTH (deeper
// nesting fails the parse: speculative callers use a shallow stack, exact callers a deep one).
template <int DEPTH, bool UTF8 = false>
YC_HD inline bool skip_any(const uint8_t* __restrict__ b, uint32_t& p, uint32_t end, uint32_t& steps, uint32_t* cflags = nullptr) {
  const PtrSrc src{b};
  uint32_t cf = 0;                  // ANY_* flags (UTF8 mode: the exact parse checks the encoding)
  int64_t lastkey[UTF8 ? DEPTH + 1 : 1];  // per object level: the last array-index key, or -2 after a string key
  uint64_t keym[UTF8 ? DEPTH + 1 : 1];    // per object level: the repeat mask of its keys (key_bit)
  // per object level: the FNV-32 hashes of its first KH keys (a repeat is a hash match: exact up to
  // a 2^-32 false alarm, which costs a rewrite pass that changes nothing); past KH keys the mask
  constexpr uint32_t KH = 8;
  uint32_t keyh[UTF8 ? DEPTH + 1 : 1][UTF8 ? KH : 1];
  uint32_t keyn[UTF8 ? DEPTH + 1 : 1];
  // A level is kept only while members FOLLOW the one being read (rem[d] >= 1): the last member of
  // a container is read in the container's place (a tail position), so nesting along last members
  // — [[[..]]], {a: {b: ..}}, however deep — takes no stack, and DEPTH bounds only containers
  // nested inside members that are not their container's last.
  uint32_t rem[DEPTH];
  uint32_t objmask = 0;  // bit d set: level d is an object (key before each member)
  int d = 0;
  bool ok = true;
#pragma unroll 1
  for (;;) {
    if (steps == 0) return false;
    --steps;
    if (p >= end) return false;
    uint32_t tag = b[p++];
    switch (tag) {
      case 127: case 126: case 121: case 120: break;
      case 125: { const uint32_t q0 = p; skip_vi(b, p, end, ok); if (UTF8 && ok) cf |= vi_flag(b, q0, p); break; }
      case 124: { const uint32_t q0 = p; skip_bytes(p, 4, end, ok); if (UTF8 && ok) cf |= f32_flag(be32(b, q0)); break; }
      case 123: { const uint32_t q0 = p; skip_bytes(p, 8, end, ok); if (UTF8 && ok) cf |= f64_flag(be64(b, q0)); break; }
      case 122: skip_bytes(p, 8, end, ok); break;
      case 119: {
        const uint32_t q0 = p;
        uint32_t n = rd_vu(b, p, end, ok);
        const uint32_t st = p;
        if (ok) skip_bytes(p, n, end, ok);
        if (UTF8 && ok && !utf8_valid(src, st, n)) return false;
        if (UTF8 && ok) cf |= vu_overlong(b, q0, st);
        break;
      }
      case 116: {
        const uint32_t q0 = p;
        uint32_t n = rd_vu(b, p, end, ok);
        if (UTF8 && ok) cf |= vu_overlong(b, q0, p);
        if (ok) skip_bytes(p, n, end, ok);
        break;
      }
      case 118: case 117: {
        const uint32_t q0 = p;
        uint32_t n = rd_vu(b, p, end, ok);
        if (!ok) return false;
        if (UTF8) cf |= vu_overlong(b, q0, p);
        if (n > 0) {
          if (n > 1) {  // members follow this one: keep the level
            if (d == DEPTH) { steps = 0; return false; }  // too deep: "unknown" (-1), never "malformed"
            rem[d] = n - 1;
            if (tag == 118) objmask |= 1u << d; else objmask &= ~(1u << d);
            if (UTF8) lastkey[d] = -1;
            ++d;
          }
          if (tag == 118) {  // the first member's key
            const uint32_t q0 = p;
            uint32_t k = rd_vu(b, p, end, ok);
            const uint32_t st = p;
            if (ok) skip_bytes(p, k, end, ok);
            if (UTF8 && ok && !utf8_valid(src, st, k)) return false;
            if (UTF8 && ok) {
              cf |= vu_overlong(b, q0, st);
              if (key_proto(b, st, k)) cf |= (p < end && (b[p] == 116 || b[p] == 117)) ? ANY_UNSUP : ANY_KEYS;
              const int64_t ki = key_index(b, st, k);
              if (n > 1) {
                lastkey[d - 1] = ki >= 0 ? ki : -2;
                keym[d - 1] = key_bit(k, k ? b[st] : 0u, k ? b[st + k - 1] : 0u);
                keyh[d - 1][0] = fnv_key(b, st, k);
                keyn[d - 1] = 1;
              }
            }
          }
          if (!ok) return false;
          continue;  // read the first member value
        }
        break;
      }
      default: return false;
    }
    if (!ok) return false;
    // a value completed: the innermost kept level moves to its next member (the last one is read
    // in the level's place)
    if (d == 0) {
      if (UTF8 && cflags) *cflags |= cf;
      return true;
    }
    const uint32_t lvl = (uint32_t)d - 1;
    if ((objmask >> lvl) & 1u) {  // the next member's key
      const uint32_t q0 = p;
      uint32_t k = rd_vu(b, p, end, ok);
      const uint32_t st = p;
      if (ok) skip_bytes(p, k, end, ok);
      if (!ok || (UTF8 && !utf8_valid(src, st, k))) return false;
      if (UTF8) {
        cf |= vu_overlong(b, q0, st);
        if (key_proto(b, st, k)) cf |= (p < end && (b[p] == 116 || b[p] == 117)) ? ANY_UNSUP : ANY_KEYS;
        // Object.keys order: array-index keys first, ascending; then the others in insertion order
        // (a repeated key keeps its first place: a possible repeat is flagged by the key mask)
        const int64_t ki = key_index(b, st, k), prev = lastkey[lvl];
        if (ki >= 0 && (prev == -2 || (prev >= 0 && ki <= prev))) cf |= ANY_KEYS;
        lastkey[lvl] = ki >= 0 ? ki : -2;
        const uint64_t kb = key_bit(k, k ? b[st] : 0u, k ? b[st + k - 1] : 0u);
        const uint32_t kn = keyn[lvl];
        if (kn <= KH) {  // the hashes of every key so far: exact
          const uint32_t h = fnv_key(b, st, k);
          for (uint32_t j = 0; j < kn; ++j)
            if (keyh[lvl][j] == h) cf |= ANY_KEYS;
          if (kn < KH) keyh[lvl][kn] = h;
          keyn[lvl] = kn + 1;
        } else if (keym[lvl] & kb) {
          cf |= ANY_KEYS;
        }
        keym[lvl] |= kb;
      }
    }
    if (--rem[lvl] == 0) --d;
  }
}

// An object key's flags through a byte source: ANY_KEYS for "__proto__" (ANY_UNSUP when its value,
// the byte after the key, is bytes or an array); ki = its array index (key_index), else -1
template <class S>
YC_HDI uint32_t key_flags_at(const S& b, uint32_t p, uint32_t n, uint32_t end, int64_t& ki) {
  ki = -1;
  const uint32_t c0 = n ? b.u8(p) : 0u;
  if (n == 9 && c0 == '_') {
    const char* k = "__proto__";
    uint32_t i = 0;
    while (i < 9 && b.u8(p + i) == (uint8_t)k[i]) ++i;
    if (i != 9) return 0u;
    const uint32_t t = p + 9 < end ? b.u8(p + 9) : 0u;
    return (t == 116u || t == 117u) ? ANY_UNSUP : ANY_KEYS;
  }
  if (n == 0 || n > 10 || c0 < '0' || c0 > '9' || (n > 1 && c0 == '0')) return 0u;
  uint64_t v = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t c = b.u8(p + i);
    if (c < '0' || c > '9') return 0u;
    v = v * 10 + (c - '0');
  }
  if (v < 0xFFFFFFFFull) ki = (int64_t)v;
  return 0u;
}
// One scalar `any` value after its tag (at p), flags in cf (FULL): 127 undefined, 126 null,
// 121 / 120 false / true, 125 varint, 124 float32, 123 float64, 122 bigint, 119 string, 116 bytes.
template <bool FULL, class S>
YC_HDI void any_scalar(const S& b, uint32_t tag, uint32_t& p, uint32_t end, bool& ok, uint32_t& cf) {
  const uint32_t s0 = p;
  switch (tag) {
    case 125: b.svi(p, end, ok); if (FULL && ok) cf |= vi_flag_at(b, s0, p); break;
    case 124: skip_bytes(p, 4, end, ok); if (FULL && ok) cf |= f32_flag((uint32_t)be_at(b, s0, 4)); break;
    case 123: skip_bytes(p, 8, end, ok); if (FULL && ok) cf |= f64_flag(be_at(b, s0, 8)); break;
    case 122: skip_bytes(p, 8, end, ok); break;
    case 119: {
      const uint32_t n = b.vu(p, end, ok);
      if (FULL && ok) cf |= vu_overlong_at(b, s0, p);
      const uint32_t st = p;
      if (ok) skip_bytes(p, n, end, ok);
      if (FULL && ok && !utf8_valid(b, st, n)) ok = false;
      break;
    }
    case 116: { const uint32_t k = b.vu(p, end, ok); if (FULL && ok) cf |= vu_overlong_at(b, s0, p); if (ok) skip_bytes(p, k, end, ok); break; }
    default: break;  // 127, 126, 121, 120
  }
}
YC_HDI bool any_scalar_tag(uint32_t tag) { return tag >= 116u && tag <= 127u && tag != 117u && tag != 118u; }
// A one-level array / object of at most 8 scalar members (C1's {name, v}, C2's {name}), inline:
// true when it was one (p past it; ok false if malformed), false otherwise (p unchanged: the
// container goes to skip_any_nl).
template <bool FULL, class S>
YC_HDI bool any_flat(const S& b, uint32_t& p, uint32_t end, uint32_t& steps, bool& ok, uint32_t& cf) {
  const uint32_t p0 = p, tag = b.u8(p);
  uint32_t q = p + 1, c = 0, st = steps;
  bool o = true;
  const uint32_t m = b.vu(q, end, o);
  if (!o || m > 8 || st < m + 1) return false;
  if (FULL) c |= vu_overlong_at(b, p0 + 1, q);
  int64_t prev = -1;
  uint64_t km = 0;  // the keys' repeat mask
  for (uint32_t i = 0; i < m; ++i) {
    if (tag == 118) {  // the member's key
      const uint32_t k0 = q, k = b.vu(q, end, o);
      if (!o) { ok = false; p = q; return true; }
      const uint32_t ks = q;
      skip_bytes(q, k, end, o);
      if (FULL && o) {
        if (!utf8_valid(b, ks, k)) o = false;
        c |= vu_overlong_at(b, k0, ks);
        int64_t ki;
        c |= key_flags_at(b, ks, k, end, ki);
        // Object.keys order: array-index keys first, ascending, then the others (skip_any)
        if (ki >= 0 && (prev == -2 || (prev >= 0 && ki <= prev))) c |= ANY_KEYS;
        prev = ki >= 0 ? ki : -2;
        if (m > 1) {  // (one member cannot repeat: C2's {name} values skip the mask)
          // a mask hit is a possible repeat: flagged here, tested exactly by k_json_structs (the test
          // inline cost the struct decode a spilled register: +0.5 ms on the C2 headline)
          const uint64_t kb = key_bit(k, k ? b.u8(ks) : 0u, k ? b.u8(ks + k - 1) : 0u);
          if (km & kb) c |= ANY_KEYS;
          km |= kb;
        }
      }
      if (!o) { ok = false; p = q; return true; }
    }
    if (q >= end) { ok = false; p = q; return true; }
    const uint32_t t = b.u8(q);
    if (!any_scalar_tag(t)) return false;  // a nested container: the general reader
    ++q;
    any_scalar<FULL>(b, t, q, end, o, c);
    if (!o) { ok = false; p = q; return true; }
  }
  p = q;
  steps = st - (m + 1);
  cf |= c;
  return true;
}

// Out of line: the container stack costs DEPTH registers wherever skip_any is inlined, so struct
// parsers take scalar values (and one-level containers of scalars) inline and hand the other
// containers to this call.
// (State goes in and out by value: taking the caller's cursor by address would put it in scratch.)
struct AnySkip { uint32_t p, steps, ok, cf; };
template <int DEPTH, bool UTF8 = false>
YC_HD __attribute__((noinline)) AnySkip skip_any_nl(const uint8_t* __restrict__ b, uint32_t p, uint32_t end, uint32_t steps) {
  uint32_t cf = 0;
  const bool ok = skip_any<DEPTH, UTF8>(b, p, end, steps, &cf);
  return AnySkip{p, steps, ok ? 1u : 0u, cf};
}

// JSON.parse of a ContentJSON / ContentEmbed / ContentFormat value (Y@72137 readContentJSON,
// Y@14715 readJSON), and whether JSON.stringify gives the same text back: Yjs keeps the parsed
// value and writes it with JSON.stringify (Y@71991), while the engine copies the bytes.
//   JSON_OK        valid, in JSON.stringify's form: copied as is;
//   JSON_BAD       JSON.parse throws (SyntaxError): the update is refused, as Yjs refuses it;
//   JSON_NONCANON  valid, but not what JSON.stringify writes (whitespace, an escape it does not
//                  write, a number not in Number::toString's form, a duplicate or array-index
//                  object key, more than 64 levels, more than 15 significant digits, which the
//                  engine does not verify): valid Yjs input refused (YCRDT_E_UNSUPPORTED) instead
//                  of written back differently.
// The text is valid UTF-8 already (lib0's readVarString, checked by the caller). Out of line:
// called only for these rare contents (Yjs itself writes ContentAny for JS values).
enum : uint32_t { JSON_OK = 0, JSON_BAD = 1, JSON_NONCANON = 2 };
YC_HDI bool json_ws(uint32_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
YC_HDI int json_hex(uint32_t c) {
  return c >= '0' && c <= '9' ? (int)(c - '0') : c >= 'a' && c <= 'f' ? (int)(c - 'a' + 10) : c >= 'A' && c <= 'F' ? (int)(c - 'A' + 10) : -1;
}
// a string at p (b[p] == '"'): p past its closing quote; res |= NONCANON for escapes stringify
// does not write; h = FNV-1a of its raw bytes, idx = its array-index value (key_index) or -1
YC_HD inline uint32_t json_string(const uint8_t* __restrict__ b, uint32_t& p, uint32_t e, uint32_t& res, uint64_t& h, int64_t& idx) {
  ++p;
  const uint32_t s0 = p;
  h = 1469598103934665603ull;
  for (;;) {
    if (p >= e) return JSON_BAD;
    const uint32_t c = b[p];
    if (c == '"') break;
    if (c < 0x20u) return JSON_BAD;
    h = (h ^ c) * 1099511628211ull;
    ++p;
    if (c != '\\') continue;
    if (p >= e) return JSON_BAD;
    const uint32_t x = b[p++];
    h = (h ^ x) * 1099511628211ull;
    if (x == '"' || x == '\\' || x == 'b' || x == 'f' || x == 'n' || x == 'r' || x == 't') continue;
    if (x == '/') { res = JSON_NONCANON; continue; }
    if (x != 'u') return JSON_BAD;
    uint32_t v = 0;
    bool lower = true;
    for (int k = 0; k < 4; ++k) {
      if (p >= e) return JSON_BAD;
      const uint32_t d = b[p++];
      const int hv = json_hex(d);
      if (hv < 0) return JSON_BAD;
      if (d >= 'A' && d <= 'F') lower = false;
      h = (h ^ d) * 1099511628211ull;
      v = (v << 4) | (uint32_t)hv;
    }
    // stringify writes \u only for controls without a short escape and for lone surrogates (lowercase)
    const bool ctl = v < 0x20u && v != 8 && v != 9 && v != 10 && v != 12 && v != 13;
    bool lone = false;
    if (v >= 0xD800u && v <= 0xDBFFu) {  // a high surrogate: lone unless a \uDC00-\uDFFF follows
      lone = true;
      if (p + 6 <= e && b[p] == '\\' && b[p + 1] == 'u') {
        uint32_t w2 = 0;
        bool hexok = true;
        for (int k = 0; k < 4; ++k) { const int hv = json_hex(b[p + 2 + k]); if (hv < 0) hexok = false; else w2 = (w2 << 4) | (uint32_t)hv; }
        if (hexok && w2 >= 0xDC00u && w2 <= 0xDFFFu) lone = false;  // a pair: stringify writes the character
      }
    } else if (v >= 0xDC00u && v <= 0xDFFFu) {
      lone = true;  // (a low surrogate after a high one was judged with it: the pair is non-canonical already)
    }
    if (!(ctl || lone) || !lower) res = JSON_NONCANON;
  }
  // array-index keys (JSON.parse keeps them, Object.keys moves them first): key_index's rule
  const uint32_t n = p - s0;
  idx = key_index(b, s0, n);
  ++p;
  return JSON_OK;
}
// a number at p: p past it; res |= NONCANON unless it is Number::toString's form of its value
YC_HD inline uint32_t json_number(const uint8_t* __restrict__ b, uint32_t& p, uint32_t e, uint32_t& res) {
  const uint32_t s0 = p;
  const bool neg = b[p] == '-';
  if (neg) ++p;
  if (p >= e) return JSON_BAD;
  // digits: the integer part, then the fraction
  const uint32_t i0 = p;
  if (b[p] == '0') ++p;
  else if (b[p] >= '1' && b[p] <= '9') { while (p < e && b[p] >= '0' && b[p] <= '9') ++p; }
  else return JSON_BAD;
  const uint32_t i1 = p;
  uint32_t f0 = p, f1 = p;
  if (p < e && b[p] == '.') {
    ++p;
    f0 = p;
    while (p < e && b[p] >= '0' && b[p] <= '9') ++p;
    f1 = p;
    if (f1 == f0) return JSON_BAD;
  }
  int32_t ex = 0;
  if (p < e && (b[p] == 'e' || b[p] == 'E')) {
    ++p;
    bool eneg = false;
    if (p < e && (b[p] == '+' || b[p] == '-')) { eneg = b[p] == '-'; ++p; }
    const uint32_t x0 = p;
    while (p < e && b[p] >= '0' && b[p] <= '9') { if (ex < 100000) ex = ex * 10 + (int32_t)(b[p] - '0'); ++p; }
    if (p == x0) return JSON_BAD;
    if (eneg) ex = -ex;
  }
  if (res == JSON_NONCANON) return JSON_OK;  // (already refused: the form needs no check)
  // significant digits d[0..k) and the decimal exponent n: value = 0.d1..dk x 10^n
  char d[24];
  uint32_t k = 0;
  int32_t n = (int32_t)(i1 - i0) + ex;  // position of the decimal point in int ++ frac, shifted by the exponent
  bool lead = true;
  uint32_t zeros = 0;  // zeros after the last nonzero digit (trailing ones are not significant)
  for (uint32_t q = i0; q < f1; ++q) {
    if (q == i1) { q = f0; if (q >= f1) break; }
    const char c = (char)b[q];
    if (lead && c == '0') { --n; continue; }
    lead = false;
    if (c == '0') { ++zeros; continue; }
    if (k + zeros >= 15) { k = 99; break; }  // more than 15 significant digits: the exact test below
    for (; zeros; --zeros) d[k++] = '0';
    d[k++] = c;
  }
  // the text Number::toString writes for it (ECMA-262 Number::toString, radix 10)
  char t[40];
  uint32_t m = 0;
  if (k == 99 || (k != 0 && (n > 308 || n < -306))) {
    // past what a double holds exactly as 15 digits, or at the ends of its range: JSON.parse's
    // double and its shortest form, in big-integer arithmetic (yc_num.h)
    m = json_number_canon(b, s0, p, t);
    if (m == 0) { res = JSON_NONCANON; return JSON_OK; }
  } else {
    m = num_text(neg, d, k, n, t);
  }
  if (p - s0 != m) { res = JSON_NONCANON; return JSON_OK; }
  for (uint32_t i = 0; i < m; ++i)
    if (b[s0 + i] != (uint8_t)t[i]) { res = JSON_NONCANON; return JSON_OK; }
  return JSON_OK;
}
YC_HD inline __attribute__((noinline)) uint32_t json_check(const uint8_t* __restrict__ b, uint32_t p, uint32_t n) {
  const uint32_t e = p + n;
  uint32_t res = JSON_OK;
  uint64_t objbits = 0;  // bit d: level d is an object
  int d = 0;
  uint32_t kh[32];       // the keys of the open objects (hash, level, array index or NONE): a repeated
  uint8_t kl[32];        // key (or a hash collision: refused either way), or an array-index key after
  uint32_t ki[32];       // another key that is not a smaller index, is not what JSON.stringify writes
  uint32_t nk = 0;
  auto skip_ws = [&]() { while (p < e && json_ws(b[p])) { ++p; res = JSON_NONCANON; } };
  // an object member's key and colon (p at the key)
  auto key = [&]() -> uint32_t {
    if (p >= e || b[p] != '"') return JSON_BAD;
    uint64_t h;
    int64_t idx;
    if (json_string(b, p, e, res, h, idx) != JSON_OK) return JSON_BAD;
    const bool first = nk == 0 || kl[nk - 1] != (uint8_t)(d - 1);
    const uint32_t ix = idx >= 0 ? (uint32_t)idx : 0xFFFFFFFFu, h32 = (uint32_t)(h ^ (h >> 32));
    if (idx >= 0 && !first && (ki[nk - 1] == 0xFFFFFFFFu || ki[nk - 1] >= ix)) res = JSON_NONCANON;  // (JSON.parse moves index keys first)
    for (uint32_t i = nk; i > 0 && kl[i - 1] == (uint8_t)(d - 1); --i)
      if (kh[i - 1] == h32) res = JSON_NONCANON;
    if (nk == 32) res = JSON_NONCANON;
    else { kh[nk] = h32; kl[nk] = (uint8_t)(d - 1); ki[nk] = ix; ++nk; }
    skip_ws();
    if (p >= e || b[p] != ':') return JSON_BAD;
    ++p;
    skip_ws();
    return JSON_OK;
  };
  skip_ws();
  for (;;) {
    // a value at p
    if (p >= e) return JSON_BAD;
    const uint32_t c = b[p];
    if (c == '{' || c == '[') {
      ++p;
      skip_ws();
      if (p >= e) return JSON_BAD;
      if (b[p] == (c == '{' ? '}' : ']')) {
        ++p;
      } else {
        if (d == 64) return JSON_NONCANON;  // deeper than the level mask (valid or not: refused)
        if (c == '{') objbits |= 1ull << d; else objbits &= ~(1ull << d);
        ++d;
        if (c == '{' && key() != JSON_OK) return JSON_BAD;
        continue;
      }
    } else if (c == '"') {
      uint64_t h;
      int64_t idx;
      if (json_string(b, p, e, res, h, idx) != JSON_OK) return JSON_BAD;
    } else if (c == '-' || (c >= '0' && c <= '9')) {
      if (json_number(b, p, e, res) != JSON_OK) return JSON_BAD;
    } else if (c == 't' || c == 'f' || c == 'n') {
      const char* lit = c == 't' ? "true" : c == 'f' ? "false" : "null";
      uint32_t i = 0;
      while (lit[i] && p + i < e && b[p + i] == (uint8_t)lit[i]) ++i;
      if (lit[i]) return JSON_BAD;
      p += i;
    } else {
      return JSON_BAD;
    }
    // a value completed: close containers, or the next member
    for (;;) {
      skip_ws();
      if (d == 0) return p == e ? res : JSON_BAD;
      if (p >= e) return JSON_BAD;
      const bool obj = (objbits >> (d - 1)) & 1ull;
      const uint32_t x = b[p];
      if (x == (obj ? '}' : ']')) {
        ++p;
        --d;
        while (nk > 0 && kl[nk - 1] >= (uint8_t)d) --nk;  // the closed object's keys
        continue;
      }
      if (x != ',') return JSON_BAD;
      ++p;
      skip_ws();
      if (obj && key() != JSON_OK) return JSON_BAD;
      break;
    }
  }
}
// The JSON values of one ContentJSON / ContentEmbed / ContentFormat content [p, end) (Y@72137
// readContentJSON: n varStrings, "undefined" allowed; readContentEmbed: one; readContentFormat: a
// key, then one): 0 ok, 0x100 malformed (JSON.parse throws), -1 not (or not surely) in the form Yjs
// writes back (json_content_canon rewrites it; a value json_check could not judge — nesting past
// its level mask — is validated there).
// Called by the exact decoders once a struct's columns are out (k_struct_decode, the host scanner
// scan_update): inside parse_struct the call kept the whole struct view live across it (+24 VGPRs,
// one wave per SIMD less for every struct).
YC_HD inline __attribute__((noinline)) int json_content(const uint8_t* __restrict__ b, uint32_t p, uint32_t end, uint32_t ref) {
  bool ok = true;
  uint32_t n = 1;
  bool over = false;  // an overlong length prefix: valid, but not writeVarUint's form
  uint32_t q0 = p;
  if (ref == REF_JSON) { n = rd_vu(b, p, end, ok); over |= vu_overlong(b, q0, p) != 0; }
  else if (ref == REF_FORMAT) { const uint32_t k = rd_vu(b, p, end, ok); over |= vu_overlong(b, q0, p) != 0; p += k; }
  int res = 0;
  for (uint32_t i = 0; i < n && ok; ++i) {
    q0 = p;
    const uint32_t k = rd_vu(b, p, end, ok);
    if (!ok) break;
    over |= vu_overlong(b, q0, p) != 0;
    const uint8_t* u = b + p;
    const bool undef = ref == REF_JSON && k == 9 && u[0] == 'u' && u[1] == 'n' && u[2] == 'd' && u[3] == 'e' && u[4] == 'f' &&
                       u[5] == 'i' && u[6] == 'n' && u[7] == 'e' && u[8] == 'd';
    if (!undef) {
      const uint32_t r = json_check(b, p, k);
      if (r == JSON_BAD) return 0x100;
      if (r == JSON_NONCANON) res = -1;  // (the later values may still be malformed)
    }
    p += k;
  }
  if (!ok) return 0x100;
  return over ? -1 : res;
}

// ---- JSON.stringify(JSON.parse(text)): the canonical form of a ContentJSON / Embed / Format value
// that json_check found not in it (whitespace, escapes stringify does not write, numbers not in
// Number::toString's form, duplicate or array-index keys, nesting past its level mask). Yjs keeps
// the parsed value (Y@72137) and writes it with JSON.stringify (Y@71991), so the engine rewrites
// such a value once, on the device (yc_decode.hip k_json_canon), before the update is merged:
//   - strings: the UTF-16 code units JSON.parse makes of the text, written back with
//     stringify's escapes (\" \\ \b \f \n \r \t, \u00xx for other controls, \udxxx for lone
//     surrogates, everything else as UTF-8; a surrogate pair as its 4-byte character);
//   - numbers: yc_num.h json_number_canon (an infinity comes out "null");
//   - objects: one member per distinct key (the last value, at the first key's place), array-index
//     keys first in ascending order (Object.keys order), keys compared by their code units;
//   - no whitespace; any depth (explicit stacks in a caller-provided word arena).
constexpr uint32_t JSON_ARENA = 3;  // the arena is too small for the value's nesting / object sizes
constexpr uint32_t JSON_ARENA_WORDS = 1u << 16;  // the arena the engine gives a value (device lane and host scanner alike)
// the code units of a JSON string's text, escapes decoded (the text is valid: json_valid)
struct JStr {
  uint32_t p;    // next byte
  uint32_t low;  // pending low surrogate of a 4-byte UTF-8 character (0: none)
};
YC_HDI int32_t jstr_next(const uint8_t* __restrict__ b, JStr& s) {
  if (s.low) { const uint32_t u = s.low; s.low = 0; return (int32_t)u; }
  const uint32_t c = b[s.p];
  if (c == '"') return -1;
  if (c == '\\') {
    const uint32_t x = b[s.p + 1];
    s.p += 2;
    switch (x) {
      case 'b': return 8;
      case 'f': return 12;
      case 'n': return 10;
      case 'r': return 13;
      case 't': return 9;
      case 'u': {
        uint32_t v = 0;
        for (int k = 0; k < 4; ++k) v = (v << 4) | (uint32_t)json_hex(b[s.p + k]);
        s.p += 4;
        return (int32_t)v;
      }
      default: return (int32_t)x;  // " \ /
    }
  }
  if (c < 0x80u) { ++s.p; return (int32_t)c; }
  if ((c & 0xE0u) == 0xC0u) { const uint32_t v = ((c & 0x1Fu) << 6) | (b[s.p + 1] & 0x3Fu); s.p += 2; return (int32_t)v; }
  if ((c & 0xF0u) == 0xE0u) {
    const uint32_t v = ((c & 0x0Fu) << 12) | ((b[s.p + 1] & 0x3Fu) << 6) | (b[s.p + 2] & 0x3Fu);
    s.p += 3;
    return (int32_t)v;
  }
  const uint32_t v = ((c & 0x07u) << 18) | ((b[s.p + 1] & 0x3Fu) << 12) | ((b[s.p + 2] & 0x3Fu) << 6) | (b[s.p + 3] & 0x3Fu);
  s.p += 4;
  s.low = 0xDC00u + ((v - 0x10000u) & 0x3FFu);
  return (int32_t)(0xD800u + ((v - 0x10000u) >> 10));
}
struct JOut {
  uint8_t* o;  // null: size only
  uint32_t n;
  YC_HDI void put(uint32_t c) { if (o) o[n] = (uint8_t)c; ++n; }
};
// the string at p (b[p] == '"') in stringify's form; p moves past it. h: FNV-1a of its code units,
// idx: its array-index value (key_index's rule on the code units) or -1
YC_HD inline void jstr_emit(const uint8_t* __restrict__ b, uint32_t& p, JOut* out, uint64_t& h, int64_t& idx) {
  JStr s{p + 1, 0};
  h = 1469598103934665603ull;
  uint64_t v = 0;
  uint32_t nu = 0;
  bool digits = true;
  const char* hex = "0123456789abcdef";
  if (out) out->put('"');
  for (;;) {
    int32_t u = jstr_next(b, s);
    if (u < 0) break;
    h = (h ^ (uint32_t)u) * 1099511628211ull;
    if (u < '0' || u > '9' || (nu == 1 && v == 0) || nu >= 10) digits = false;
    else v = v * 10 + (uint32_t)(u - '0');
    ++nu;
    if (!out) continue;
    if (u >= 0xD800 && u <= 0xDBFF) {  // a pair with the next unit, or a lone surrogate
      JStr t = s;
      const int32_t w = jstr_next(b, t);
      if (w >= 0xDC00 && w <= 0xDFFF) {
        s = t;
        h = (h ^ (uint32_t)w) * 1099511628211ull;
        ++nu;
        const uint32_t cp = 0x10000u + (((uint32_t)u - 0xD800u) << 10) + ((uint32_t)w - 0xDC00u);
        out->put(0xF0u | (cp >> 18));
        out->put(0x80u | ((cp >> 12) & 0x3Fu));
        out->put(0x80u | ((cp >> 6) & 0x3Fu));
        out->put(0x80u | (cp & 0x3Fu));
        continue;
      }
    }
    if (u >= 0xD800 && u <= 0xDFFF) {
      out->put('\\'); out->put('u');
      for (int k = 3; k >= 0; --k) out->put((uint8_t)hex[(u >> (4 * k)) & 15]);
    } else if (u == '"' || u == '\\') {
      out->put('\\'); out->put((uint32_t)u);
    } else if (u < 0x20) {
      out->put('\\');
      if (u == 8) out->put('b');
      else if (u == 9) out->put('t');
      else if (u == 10) out->put('n');
      else if (u == 12) out->put('f');
      else if (u == 13) out->put('r');
      else { out->put('u'); out->put('0'); out->put('0'); out->put(hex[u >> 4]); out->put(hex[u & 15]); }
    } else if (u < 0x80) {
      out->put((uint32_t)u);
    } else if (u < 0x800) {
      out->put(0xC0u | ((uint32_t)u >> 6)); out->put(0x80u | ((uint32_t)u & 0x3Fu));
    } else {
      out->put(0xE0u | ((uint32_t)u >> 12)); out->put(0x80u | (((uint32_t)u >> 6) & 0x3Fu)); out->put(0x80u | ((uint32_t)u & 0x3Fu));
    }
  }
  if (out) out->put('"');
  p = s.p + 1;
  idx = (digits && nu > 0 && v < 0xFFFFFFFFull) ? (int64_t)v : -1;
}
// two strings' code units equal (keys whose hashes matched)
YC_HD inline bool jstr_eq(const uint8_t* __restrict__ b, uint32_t p, uint32_t q) {
  JStr s{p + 1, 0}, t{q + 1, 0};
  for (;;) {
    const int32_t x = jstr_next(b, s), y = jstr_next(b, t);
    if (x != y) return false;
    if (x < 0) return true;
  }
}
// past one (valid) value at p: strings and brackets only
YC_HD inline uint32_t json_skip_value(const uint8_t* __restrict__ b, uint32_t p, uint32_t e) {
  uint32_t depth = 0;
  do {
    const uint32_t c = b[p];
    if (c == '"') {
      ++p;
      while (b[p] != '"') p += b[p] == '\\' ? 2u : 1u;
      ++p;
    } else if (c == '[' || c == '{') {
      ++depth; ++p;
    } else if (c == ']' || c == '}') {
      --depth; ++p;
    } else if (depth == 0) {  // a number or a literal
      while (p < e && b[p] != ',' && b[p] != ']' && b[p] != '}' && !json_ws(b[p])) ++p;
    } else {
      ++p;
    }
  } while (depth > 0);
  return p;
}
// JSON.parse's grammar at any depth (the container kinds of the open levels as bits in the arena):
// JSON_OK, JSON_BAD, or JSON_ARENA
YC_HD inline uint32_t json_valid(const uint8_t* __restrict__ b, uint32_t p, uint32_t n, uint32_t* arena, uint32_t acap) {
  const uint32_t e = p + n;
  uint32_t d = 0, res = 0;
  auto ws = [&]() { while (p < e && json_ws(b[p])) ++p; };
  auto key = [&]() -> bool {
    if (p >= e || b[p] != '"') return false;
    uint64_t h;
    int64_t idx;
    if (json_string(b, p, e, res, h, idx) != JSON_OK) return false;
    ws();
    if (p >= e || b[p] != ':') return false;
    ++p;
    ws();
    return true;
  };
  ws();
  for (;;) {
    if (p >= e) return JSON_BAD;
    const uint32_t c = b[p];
    if (c == '{' || c == '[') {
      ++p;
      ws();
      if (p >= e) return JSON_BAD;
      if (b[p] == (c == '{' ? '}' : ']')) {
        ++p;
      } else {
        if ((d >> 5) >= acap) return JSON_ARENA;
        if (c == '{') arena[d >> 5] |= 1u << (d & 31); else arena[d >> 5] &= ~(1u << (d & 31));
        ++d;
        if (c == '{' && !key()) return JSON_BAD;
        continue;
      }
    } else if (c == '"') {
      uint64_t h;
      int64_t idx;
      if (json_string(b, p, e, res, h, idx) != JSON_OK) return JSON_BAD;
    } else if (c == '-' || (c >= '0' && c <= '9')) {
      res = JSON_NONCANON;  // (the grammar only: no form test)
      if (json_number(b, p, e, res) != JSON_OK) return JSON_BAD;
    } else if (c == 't' || c == 'f' || c == 'n') {
      const char* lit = c == 't' ? "true" : c == 'f' ? "false" : "null";
      uint32_t i = 0;
      while (lit[i] && p + i < e && b[p + i] == (uint8_t)lit[i]) ++i;
      if (lit[i]) return JSON_BAD;
      p += i;
    } else {
      return JSON_BAD;
    }
    for (;;) {
      ws();
      if (d == 0) return p == e ? JSON_OK : JSON_BAD;
      if (p >= e) return JSON_BAD;
      const bool obj = (arena[(d - 1) >> 5] >> ((d - 1) & 31)) & 1u;
      const uint32_t x = b[p];
      if (x == (obj ? '}' : ']')) { ++p; --d; continue; }
      if (x != ',') return JSON_BAD;
      ++p;
      ws();
      if (obj && !key()) return JSON_BAD;
      break;
    }
  }
}
// The canonical text of the JSON value [p, p + n) into out (null: size only), its length in olen.
// The arena holds per open container a frame of 5 words (previous frame, kind 0 array / 1 object,
// member count, next member, position past the object) and per open object its members, 5 words
// each (key position, value position, key hash lo / hi, array index or ~0).
YC_HD inline __attribute__((noinline)) uint32_t json_canon(const uint8_t* __restrict__ b, uint32_t p, uint32_t n, uint8_t* out,
                                                          uint32_t* arena, uint32_t acap, uint32_t& olen) {
  olen = 0;
  const uint32_t vr = json_valid(b, p, n, arena, acap);
  if (vr != JSON_OK) return vr;
  const uint32_t e = p + n;
  JOut o{out, 0};
  constexpr uint32_t NOF = 0xFFFFFFFFu;
  uint32_t top = NOF, used = 0;
  auto ws = [&]() { while (p < e && json_ws(b[p])) ++p; };
  auto mem = [&](uint32_t f, uint32_t i) -> uint32_t* { return arena + f + 5 + 5 * i; };
  auto emit_key = [&](uint32_t f, uint32_t i) {
    uint32_t kp = mem(f, i)[0];
    uint64_t h;
    int64_t idx;
    jstr_emit(b, kp, &o, h, idx);
    o.put(':');
  };
  ws();
  for (;;) {
    // a value at p
    const uint32_t c = b[p];
    bool done = true;
    if (c == '[') {
      ++p;
      ws();
      o.put('[');
      if (b[p] == ']') { ++p; o.put(']'); }
      else {
        if (used + 5 > acap) return JSON_ARENA;
        arena[used] = top; arena[used + 1] = 0; arena[used + 2] = 0; arena[used + 3] = 0; arena[used + 4] = 0;
        top = used;
        used += 5;
        done = false;
      }
    } else if (c == '{') {
      // the members: key, value position, key hash and index, in text order
      const uint32_t f = used;
      if (f + 5 > acap) return JSON_ARENA;
      uint32_t m = 0;
      ++p;
      ws();
      if (b[p] == '}') {
        ++p;
      } else {
        for (;;) {
          ws();
          if (f + 5 + 5 * (m + 1) > acap) return JSON_ARENA;
          uint32_t* r = mem(f, m);
          r[0] = p;
          uint64_t h;
          int64_t idx;
          jstr_emit(b, p, nullptr, h, idx);
          ws();
          ++p;  // ':'
          ws();
          r[1] = p;
          r[2] = (uint32_t)h;
          r[3] = (uint32_t)(h >> 32);
          r[4] = idx >= 0 ? (uint32_t)idx : NOF;
          p = json_skip_value(b, p, e);
          ++m;
          ws();
          if (b[p++] == '}') break;  // else ','
        }
      }
      // one member per key: the last value at the first key's place
      uint32_t k = 0;
      for (uint32_t j = 0; j < m; ++j) {
        uint32_t* rj = mem(f, j);
        bool dup = false;
        for (uint32_t i = 0; i < k; ++i) {
          uint32_t* ri = mem(f, i);
          if (ri[2] == rj[2] && ri[3] == rj[3] && jstr_eq(b, ri[0], rj[0])) { ri[1] = rj[1]; dup = true; break; }
        }
        if (dup) continue;
        if (k != j) { uint32_t* rk = mem(f, k); for (int w = 0; w < 5; ++w) rk[w] = rj[w]; }
        ++k;
      }
      // array-index keys first, ascending (stable: the others keep their order)
      uint32_t ni = 0;
      for (uint32_t j = 0; j < k; ++j) {
        uint32_t* rj = mem(f, j);
        if (rj[4] == NOF) continue;
        uint32_t t[5];
        for (int w = 0; w < 5; ++w) t[w] = rj[w];
        uint32_t i = j;
        // shift the non-index members and larger index members right
        while (i > 0) {
          uint32_t* rp = mem(f, i - 1);
          if (i - 1 < ni && rp[4] <= t[4]) break;
          uint32_t* rc = mem(f, i);
          for (int w = 0; w < 5; ++w) rc[w] = rp[w];
          --i;
        }
        uint32_t* ri = mem(f, i);
        for (int w = 0; w < 5; ++w) ri[w] = t[w];
        ++ni;
      }
      o.put('{');
      if (k == 0) {
        o.put('}');
      } else {
        arena[f] = top; arena[f + 1] = 1; arena[f + 2] = k; arena[f + 3] = 0; arena[f + 4] = p;
        top = f;
        used = f + 5 + 5 * k;
        emit_key(f, 0);
        p = mem(f, 0)[1];
        done = false;
      }
    } else if (c == '"') {
      uint64_t h;
      int64_t idx;
      jstr_emit(b, p, &o, h, idx);
    } else if (c == '-' || (c >= '0' && c <= '9')) {
      uint32_t q = p, res = JSON_OK;
      json_number(b, q, e, res);
      if (res == JSON_OK) {
        for (uint32_t i = p; i < q; ++i) o.put(b[i]);
      } else {
        char t[40];
        const uint32_t m = json_number_canon(b, p, q, t);
        if (m == 0) return JSON_ARENA;
        for (uint32_t i = 0; i < m; ++i) o.put((uint8_t)t[i]);
      }
      p = q;
    } else {  // true / false / null
      const uint32_t len = c == 'f' ? 5u : 4u;
      for (uint32_t i = 0; i < len; ++i) o.put(b[p + i]);
      p += len;
    }
    if (!done) { if (arena[top + 1] == 0) ws(); continue; }
    // a value completed: the enclosing containers move on
    for (;;) {
      if (top == NOF) { olen = o.n; return JSON_OK; }
      if (arena[top + 1] == 0) {  // array: the next element, or its end
        ws();
        if (b[p] == ',') { ++p; ws(); o.put(','); break; }
        ++p;  // ']'
        o.put(']');
        used = top;
        top = arena[top];
        continue;
      }
      const uint32_t k = arena[top + 2], next = arena[top + 3] + 1;  // object: the next member
      if (next < k) {
        arena[top + 3] = next;
        o.put(',');
        emit_key(top, next);
        p = mem(top, next)[1];
        break;
      }
      o.put('}');
      p = arena[top + 4];
      used = top;
      top = arena[top];
    }
  }
}

// The canonical bytes of a whole ContentJSON / Embed / Format content [p, end) — what Yjs writes
// for it (Y@71991 ContentJSON.write: the count, then each value's JSON.stringify, "undefined" as
// is; ContentEmbed / ContentFormat: writeJSON, after Format's key) — into out (null: size only),
// every length prefix in writeVarUint's shortest form. JSON_OK, JSON_BAD or JSON_ARENA.
YC_HD inline __attribute__((noinline)) uint32_t any_content_canon(const uint8_t* __restrict__ b, uint32_t p, uint32_t end, uint8_t* out,
                                                                 uint32_t* arena, uint32_t acap, uint32_t& olen);
YC_HD inline uint32_t json_content_canon(const uint8_t* __restrict__ b, uint32_t p, uint32_t end, uint32_t ref, uint8_t* out,
                                         uint32_t* arena, uint32_t acap, uint32_t& olen) {
  if (ref == REF_ANY) return any_content_canon(b, p, end, out, arena, acap, olen);  // (object key semantics, ANY_KEYS)
  bool ok = true;
  uint32_t o = 0;
  auto put_vu = [&](uint32_t v) {
    while (v > 127u) { if (out) out[o] = (uint8_t)(0x80u | (v & 0x7Fu)); ++o; v >>= 7; }
    if (out) out[o] = (uint8_t)v;
    ++o;
  };
  uint32_t n = 1;
  if (ref == REF_JSON) { n = rd_vu(b, p, end, ok); put_vu(n); }
  else if (ref == REF_FORMAT) {
    const uint32_t k = rd_vu(b, p, end, ok);
    if (!ok || end - p < k) return JSON_BAD;
    put_vu(k);
    for (uint32_t i = 0; i < k; ++i) { if (out) out[o] = b[p + i]; ++o; }
    p += k;
  }
  for (uint32_t i = 0; i < n && ok; ++i) {
    const uint32_t k = rd_vu(b, p, end, ok);
    if (!ok || end - p < k) return JSON_BAD;
    const uint8_t* u = b + p;
    const bool undef = ref == REF_JSON && k == 9 && u[0] == 'u' && u[1] == 'n' && u[2] == 'd' && u[3] == 'e' && u[4] == 'f' &&
                       u[5] == 'i' && u[6] == 'n' && u[7] == 'e' && u[8] == 'd';
    if (undef) {
      put_vu(9);
      for (uint32_t j = 0; j < 9; ++j) { if (out) out[o] = u[j]; ++o; }
    } else {
      uint32_t len = 0;
      const uint32_t r = json_canon(b, p, k, nullptr, arena, acap, len);
      if (r != JSON_OK) return r;
      put_vu(len);
      if (out) {
        uint32_t len2 = 0;
        json_canon(b, p, k, out + o, arena, acap, len2);
      }
      o += len;
    }
    p += k;
  }
  if (!ok || p != end) return JSON_BAD;
  olen = o;
  return JSON_OK;
}

// ---- writeAny(readAny(bytes)) for the `any` values whose object keys JS treats specially (ANY_KEYS):
// readAny builds each object with obj[key] = value (L0@1937), so a "__proto__" member sets the
// prototype instead of a member, a repeated key keeps its first place with its last value, and
// Object.keys — the order writeAny writes (L0 writeAny) — lists array-index keys first, ascending.
// Every scalar comes out in writeAny's form too (any_canon's rules). Iterative over arena frames
// like json_canon: per open container 5 words (previous frame, kind 0 array / 1 object, count,
// next member, position past the object) and per open object 5 words a member (key bytes, key
// length, value position, array index or ~0, key hash).
// past one `any` value at p (any depth; the level counts in arena[base, acap)): false if malformed
// or past the arena
YC_HD inline bool any_skip_deep(const uint8_t* __restrict__ b, uint32_t& p, uint32_t end, uint32_t* arena, uint32_t base, uint32_t acap) {
  bool ok = true;
  uint32_t d = 0;
  for (;;) {
    if (p >= end) return false;
    const uint32_t tag = b[p++];
    switch (tag) {
      case 127: case 126: case 121: case 120: break;
      case 125: skip_vi(b, p, end, ok); break;
      case 124: skip_bytes(p, 4, end, ok); break;
      case 123: case 122: skip_bytes(p, 8, end, ok); break;
      case 119: case 116: { const uint32_t n = rd_vu(b, p, end, ok); if (ok) skip_bytes(p, n, end, ok); break; }
      case 117: case 118: {
        const uint32_t n = rd_vu(b, p, end, ok);
        if (!ok) return false;
        if (n > 0) {
          if (base + d >= acap || n > 0x7FFFFFFFu) return false;
          arena[base + d++] = n | (tag == 118 ? 0x80000000u : 0u);
          if (tag == 118) { const uint32_t k = rd_vu(b, p, end, ok); if (ok) skip_bytes(p, k, end, ok); }
          if (!ok) return false;
          continue;
        }
        break;
      }
      default: return false;
    }
    if (!ok) return false;
    for (;;) {
      if (d == 0) return true;
      uint32_t& top = arena[base + d - 1];
      if (((top & 0x7FFFFFFFu) - 1) == 0) { --d; continue; }
      --top;
      if (top & 0x80000000u) { const uint32_t k = rd_vu(b, p, end, ok); if (ok) skip_bytes(p, k, end, ok); if (!ok) return false; }
      break;
    }
  }
}
// Whether the object at p (tag 118) still reaches Object.prototype's __proto__ accessor once readAny
// has built it: its "__proto__" members assign its prototype in order while it does — null cuts the
// chain (later "__proto__" keys are then own members), an object passes on ITS state. Explicit
// stack of resume positions in arena[base, acap): 0 no, 1 yes, 2 past the arena / malformed.
YC_HD inline uint32_t any_proto_state(const uint8_t* __restrict__ b, uint32_t p, uint32_t end, uint32_t* arena, uint32_t base, uint32_t acap) {
  bool ok = true;
  uint32_t d = 0;  // open objects: (resume position, members left) pairs at arena[base + 2 * i]
  ++p;             // (the tag)
  uint32_t left = rd_vu(b, p, end, ok);
  for (;;) {
    if (!ok) return 2;
    if (left == 0) {  // the object keeps the accessor: its parent goes on after it
      if (d == 0) return 1;
      --d;
      p = arena[base + 2 * d];
      left = arena[base + 2 * d + 1];
      continue;
    }
    --left;
    const uint32_t kl = rd_vu(b, p, end, ok);
    if (!ok || end - p < kl) return 2;
    const bool proto = key_proto(b, p, kl);
    p += kl;
    if (proto && p < end && b[p] == 126) return 0;  // null: no accessor from here on (for every open level)
    if (proto && p < end && b[p] == 118) {          // an object: its own state decides
      uint32_t q = p;
      if (!any_skip_deep(b, q, end, arena, base + 2 * d + 2, acap)) return 2;
      if (base + 2 * d + 2 > acap) return 2;
      arena[base + 2 * d] = q;
      arena[base + 2 * d + 1] = left;
      ++d;
      ++p;
      left = rd_vu(b, p, end, ok);
      continue;
    }
    if (!any_skip_deep(b, p, end, arena, base + 2 * d, acap)) return 2;
  }
}
YC_HD inline __attribute__((noinline)) uint32_t any_content_canon(const uint8_t* __restrict__ b, uint32_t p, uint32_t end, uint8_t* out,
                                                                 uint32_t* arena, uint32_t acap, uint32_t& olen) {
  olen = 0;
  bool ok = true;
  JOut o{out, 0};
  auto put_vu = [&](uint32_t v) { while (v > 0x7Fu) { o.put(0x80u | (v & 0x7Fu)); v >>= 7; } o.put(v); };
  auto put_vi = [&](bool neg, uint32_t m) {
    o.put((m > 63u ? 0x80u : 0u) | (neg ? 0x40u : 0u) | (m & 63u));
    m >>= 6;
    while (m) { o.put((m > 127u ? 0x80u : 0u) | (m & 127u)); m >>= 7; }
  };
  auto put_num = [&](double x) -> bool {  // writeAny(number)
    const uint32_t k = num_form(x);
    if (k == 3) return false;
    if (k == 0) {
      const bool neg = x < 0 || (x == 0 && (f64_bits(x) >> 63));
      put_vi(neg, (uint32_t)(x < 0 ? -x : x));
      return true;
    }
    if (k == 1) {
      union { float f; uint32_t u; } c;
      c.f = (float)x;
      for (int sh = 24; sh >= 0; sh -= 8) o.put((c.u >> sh) & 0xFFu);
      return true;
    }
    const uint64_t u = f64_bits(x);
    for (int sh = 56; sh >= 0; sh -= 8) o.put((uint32_t)(u >> sh) & 0xFFu);
    return true;
  };
  auto num_tag = [&](double x) -> uint32_t { const uint32_t k = num_form(x); return k == 0 ? 125u : k == 1 ? 124u : 123u; };
  constexpr uint32_t NOF = 0xFFFFFFFFu;
  auto mem = [&](uint32_t f, uint32_t i) -> uint32_t* { return arena + f + 5 + 5 * i; };
  const uint32_t n = rd_vu(b, p, end, ok);
  if (!ok) return JSON_BAD;
  put_vu(n);
  for (uint32_t e = 0; e < n; ++e) {
    uint32_t top = NOF, used = 0;
    for (;;) {
      // one value at p
      if (p >= end) return JSON_BAD;
      const uint32_t tag = b[p++], s0 = p;
      bool done = true;
      switch (tag) {
        case 127: case 126: case 121: case 120: o.put(tag); break;
        case 125: {
          skip_vi(b, p, end, ok);
          if (!ok) return JSON_BAD;
          bool neg;
          const uint32_t m = vi_decode(b, s0, p, neg);
          if (!neg && m > 0x7FFFFFFFu) { o.put(num_tag((double)m)); put_num((double)m); }
          else { o.put(125); put_vi(neg, m); }
          break;
        }
        case 124: case 123: {
          skip_bytes(p, tag == 124 ? 4u : 8u, end, ok);
          if (!ok) return JSON_BAD;
          const double x = tag == 124 ? f32_of(be32(b, s0)) : f64_of(be64(b, s0));
          o.put(num_tag(x));
          if (!put_num(x)) return JSON_ARENA;  // (a negative integer past 2^32: refused)
          break;
        }
        case 122: skip_bytes(p, 8, end, ok); if (!ok) return JSON_BAD; o.put(122); for (uint32_t i = s0; i < p; ++i) o.put(b[i]); break;
        case 119: case 116: {
          const uint32_t k = rd_vu(b, p, end, ok);
          if (!ok || end - p < k) return JSON_BAD;
          o.put(tag);
          put_vu(k);
          for (uint32_t i = 0; i < k; ++i) o.put(b[p + i]);
          p += k;
          break;
        }
        case 117: {
          const uint32_t m = rd_vu(b, p, end, ok);
          if (!ok) return JSON_BAD;
          o.put(117);
          put_vu(m);
          if (m > 0) {
            if (used + 5 > acap) return JSON_ARENA;
            arena[used] = top; arena[used + 1] = 0; arena[used + 2] = m; arena[used + 3] = 0; arena[used + 4] = 0;
            top = used;
            used += 5;
            done = false;
          }
          break;
        }
        case 118: {
          const uint32_t m = rd_vu(b, p, end, ok);
          if (!ok) return JSON_BAD;
          const uint32_t f = used;
          if ((uint64_t)f + 5 + 5ull * m > acap) return JSON_ARENA;
          uint32_t k = 0;
          bool acc = true;  // the object still reaches the __proto__ accessor (any_proto_state)
          for (uint32_t j = 0; j < m; ++j) {
            const uint32_t kl = rd_vu(b, p, end, ok);
            if (!ok || end - p < kl) return JSON_BAD;
            const uint32_t ks = p;
            p += kl;
            const uint32_t vp = p;
            if (!any_skip_deep(b, p, end, arena, f + 5 + 5 * m, acap)) return JSON_ARENA;
            if (acc && key_proto(b, ks, kl)) {  // the prototype setter: no own member
              if (b[vp] == 116 || b[vp] == 117) return JSON_ARENA;  // (instanceof Uint8Array / Array: refused)
              if (b[vp] == 126) acc = false;                        // null: later "__proto__" keys are members
              else if (b[vp] == 118) {
                const uint32_t st = any_proto_state(b, vp, end, arena, f + 5 + 5 * m, acap);
                if (st == 2) return JSON_ARENA;
                acc = st == 1;
              }
              continue;
            }
            uint32_t h = 2166136261u;
            for (uint32_t i = 0; i < kl; ++i) h = (h ^ b[ks + i]) * 16777619u;
            bool dup = false;
            for (uint32_t i = 0; i < k && !dup; ++i) {
              uint32_t* r = mem(f, i);
              if (r[4] != h || r[1] != kl) continue;
              uint32_t q = 0;
              while (q < kl && b[r[0] + q] == b[ks + q]) ++q;
              if (q == kl) { r[2] = vp; dup = true; }  // the last value, at the first key's place
            }
            if (dup) continue;
            uint32_t* r = mem(f, k++);
            const int64_t ki = key_index(b, ks, kl);
            r[0] = ks; r[1] = kl; r[2] = vp; r[3] = ki >= 0 ? (uint32_t)ki : NOF; r[4] = h;
          }
          // array-index keys first, ascending (the others keep their order)
          uint32_t ni = 0;
          for (uint32_t j = 0; j < k; ++j) {
            uint32_t* rj = mem(f, j);
            if (rj[3] == NOF) continue;
            uint32_t t[5];
            for (int w = 0; w < 5; ++w) t[w] = rj[w];
            uint32_t i = j;
            while (i > 0) {
              uint32_t* rp = mem(f, i - 1);
              if (i - 1 < ni && rp[3] <= t[3]) break;
              uint32_t* rc = mem(f, i);
              for (int w = 0; w < 5; ++w) rc[w] = rp[w];
              --i;
            }
            uint32_t* ri = mem(f, i);
            for (int w = 0; w < 5; ++w) ri[w] = t[w];
            ++ni;
          }
          o.put(118);
          put_vu(k);
          if (k > 0) {
            arena[f] = top; arena[f + 1] = 1; arena[f + 2] = k; arena[f + 3] = 0; arena[f + 4] = p;
            top = f;
            used = f + 5 + 5 * k;
            const uint32_t* r = mem(f, 0);
            put_vu(r[1]);
            for (uint32_t i = 0; i < r[1]; ++i) o.put(b[r[0] + i]);
            p = r[2];
            done = false;
          }
          break;
        }
        default: return JSON_BAD;
      }
      if (!done) continue;
      // a value completed: the open containers move on
      bool fin = false;
      for (;;) {
        if (top == NOF) { fin = true; break; }
        if (arena[top + 1] == 0) {  // array: its next element follows in the text
          if (--arena[top + 2] > 0) break;
          used = top;
          top = arena[top];
          continue;
        }
        const uint32_t k = arena[top + 2], next = arena[top + 3] + 1;
        if (next < k) {
          arena[top + 3] = next;
          const uint32_t* r = mem(top, next);
          put_vu(r[1]);
          for (uint32_t i = 0; i < r[1]; ++i) o.put(b[r[0] + i]);
          p = r[2];
          break;
        }
        p = arena[top + 4];
        used = top;
        top = arena[top];
      }
      if (fin) break;
    }
  }
  if (p != end) return JSON_BAD;
  olen = o.n;
  return JSON_OK;
}

// Whether a ContentAny content [p, end) holds an object whose keys JS treats specially, exactly
// (skip_any's per-level key hashes; the struct decoder only flags a possible repeat by a mask):
// k_json_structs lists the struct for the rewrite when it does.
YC_HD inline __attribute__((noinline)) bool any_keys_exact(const uint8_t* __restrict__ b, uint32_t p, uint32_t end) {
  bool ok = true;
  const uint32_t n = rd_vu(b, p, end, ok);
  for (uint32_t i = 0; i < n && ok; ++i) {
    uint32_t steps = 0xFFFFFFFFu, cf = 0;
    if (!skip_any<32, true>(b, p, end, steps, &cf)) return true;  // (deeper than the reader: let the rewrite judge)
    if (cf & ANY_KEYS) return true;
  }
  return false;
}

// Decoded view of one struct (Y@19286 readClientsStructRefs + readItemContent).
struct StructView {
  uint8_t info;
  uint8_t ref;
  uint8_t pkind;       // 0 none, 1 root name, 2 parent id
  uint8_t has_psub;
  uint32_t len;        // clock length
  uint32_t oc, ok_;    // origin (client, clock) valid if info&0x80
  uint32_t rc, rk;     // right origin valid if info&0x40
  uint32_t pa, pb;     // root name: (pos of varString, byte length incl. prefix) | parent id (client, clock)
  uint32_t psub_pos, psub_len;  // varString (incl. length prefix)
  uint32_t pn, psn;    // byte lengths of the root name / parentSub strings (FULL parses)
  uint32_t cpos, cend; // content bytes [cpos, cend)
  uint32_t nel;        // Any/JSON element count
  uint32_t anyf;       // ANY_* flags of the content's `any` values (FULL parses)
};

// Byte sources for parse_struct: the lib0 readers over a plain pointer (host and device); the
// device decoder passes a source with word-wide varuint reads (yc_decode.hip FastSrc).
struct RawSrc {
  const uint8_t* __restrict__ b;
  YC_HDI uint32_t u8(uint32_t p) const { return b[p]; }
  YC_HDI uint32_t w4(uint32_t p) const { return le32(b, p); }
  YC_HDI uint32_t vu(uint32_t& p, uint32_t end, bool& ok) const { return rd_vu(b, p, end, ok); }
  YC_HDI void svi(uint32_t& p, uint32_t end, bool& ok) const { skip_vi(b, p, end, ok); }
};

// Parses one struct starting at p. FULL fills `v`. Speculative callers pass a finite
// step budget; exact callers pass 0xFFFFFFFF. Returns 1 = ok, 0 = malformed, -1 = budget hit,
// -2 = ran past `end` (only distinguishable from 0 when `end` is not the update end).
// DEFER: a content that needs the out-of-line `any` reader (containers nested past one level, a
// ContentDoc's options) returns PARSE_DEFER instead of calling it — the caller hands the struct to
// a kernel of its own (a call site in a kernel sizes its registers for the callee's: k_struct_decode
// ran one wave per SIMD short for every struct).
constexpr int PARSE_DEFER = -3;
template <bool FULL, int DEPTH = 32, class Src = RawSrc, bool DEFER = false>
YC_HD inline int parse_struct(const Src& b, uint32_t& p, uint32_t end, uint32_t steps, StructView* v) {
  bool ok = true;
  if (p >= end) return -2;
  uint32_t info = b.u8(p++);
  uint32_t ref = info & 31u;
  if (FULL) { v->info = (uint8_t)info; v->ref = (uint8_t)ref; v->pkind = 0; v->has_psub = 0; v->nel = 0; v->anyf = 0; }
  if (ref == REF_GC || ref == REF_SKIP) {
    uint32_t len = b.vu(p, end, ok);
    if (FULL) { v->len = len; v->cpos = v->cend = p; }
    return ok ? 1 : (p >= end ? -2 : 0);
  }
  if (ref > REF_DOC) return 0;
  if (info & 0x80u) {
    uint32_t c = b.vu(p, end, ok), k = b.vu(p, end, ok);
    if (FULL) { v->oc = c; v->ok_ = k; }
  }
  if (info & 0x40u) {
    uint32_t c = b.vu(p, end, ok), k = b.vu(p, end, ok);
    if (FULL) { v->rc = c; v->rk = k; }
  }
  if (!ok) return p >= end ? -2 : 0;
  if ((info & 0xC0u) == 0) {
    uint32_t pinfo = b.vu(p, end, ok);
    if (!ok) return p >= end ? -2 : 0;
    if (pinfo == 1) {
      uint32_t st = p;
      const uint32_t n = skip_str<FULL>(b, p, end, ok);
      if (FULL) { v->pkind = 1; v->pa = st; v->pb = p - st; v->pn = n; }
    } else {
      uint32_t c = b.vu(p, end, ok), k = b.vu(p, end, ok);
      if (FULL) { v->pkind = 2; v->pa = c; v->pb = k; }
    }
    if (info & 0x20u) {
      uint32_t st = p;
      const uint32_t n = skip_str<FULL>(b, p, end, ok);
      if (FULL) { v->has_psub = 1; v->psub_pos = st; v->psub_len = p - st; v->psn = n; }
    }
    if (!ok) return p >= end ? -2 : 0;
  }
  uint32_t cpos = p;
  uint32_t len = 1;
  switch (ref) {
    case REF_DELETED: len = b.vu(p, end, ok); break;
    case REF_JSON: {
      uint32_t n = b.vu(p, end, ok);
      len = n;
      for (uint32_t i = 0; i < n && ok; ++i) {
        if (steps == 0) return -1;
        --steps;
        uint32_t k = b.vu(p, end, ok);
        if (ok && (k == 0 || (p < end && !json_start_ok(b.u8(p))))) return 0;
        const uint32_t st = p;
        if (ok) skip_bytes(p, k, end, ok);
        if (FULL && ok && !utf8_valid(b, st, k)) ok = false;
      }
      if (FULL) v->nel = n;
      if (ok && steps == 0) return -1;
      break;
    }
    case REF_BINARY: { uint32_t k = b.vu(p, end, ok); if (ok) skip_bytes(p, k, end, ok); break; }
    case REF_EMBED: {
      uint32_t k = b.vu(p, end, ok);
      if (ok && (k == 0 || (p < end && !json_start_ok(b.u8(p))))) return 0;
      const uint32_t st = p;
      if (ok) skip_bytes(p, k, end, ok);
      if (FULL && ok && !utf8_valid(b, st, k)) ok = false;
      break;
    }
    case REF_STRING: {
      uint32_t k = b.vu(p, end, ok);
      uint32_t st = p;
      if (ok) skip_bytes(p, k, end, ok);
      if (FULL && ok) len = utf8_units(b, st, k, ok);  // ContentString length counts UTF-16 code units
      break;
    }
    case REF_FORMAT: {
      skip_str<FULL>(b, p, end, ok);
      uint32_t k = b.vu(p, end, ok);
      if (ok && (k == 0 || (p < end && !json_start_ok(b.u8(p))))) return 0;
      const uint32_t st = p;
      if (ok) skip_bytes(p, k, end, ok);
      if (FULL && ok && !utf8_valid(b, st, k)) ok = false;
      break;
    }
    case REF_TYPE: {
      uint32_t tr = b.vu(p, end, ok);
      if (ok && (tr == 3 || tr == 5)) skip_str<FULL>(b, p, end, ok);
      if (tr > 6) ok = false;
      break;
    }
    case REF_ANY: {
      const uint32_t q0 = p;
      uint32_t n = b.vu(p, end, ok);
      uint32_t cf = FULL && ok ? vu_overlong_at(b, q0, p) : 0u;
      len = n;
      for (uint32_t i = 0; i < n && ok; ++i) {
        const uint32_t tag = p < end ? b.u8(p) : 0u;
        if (p < end && steps > 0 && any_scalar_tag(tag)) {  // a scalar: skip_any's one step
          --steps;
          ++p;
          any_scalar<FULL>(b, tag, p, end, ok, cf);
        } else if (p < end && steps > 0 && (tag == 117u || tag == 118u) && any_flat<FULL>(b, p, end, steps, ok, cf)) {
          // (a one-level container of scalars, inline)
        } else {
          if (DEFER) return PARSE_DEFER;
          const AnySkip r = skip_any_nl<DEPTH, FULL>(b.b, p, end, steps);
          p = r.p;
          steps = r.steps;
          ok = r.ok != 0;
          cf |= r.cf;
        }
      }
      if (!ok && steps == 0) return -1;
      if (FULL) { v->nel = n; v->anyf = cf; }
      if (FULL && ok && (cf & ANY_UNSUP)) return -1;  // valid Yjs input the engine refuses (YCRDT_E_UNSUPPORTED)
      break;
    }
    case REF_DOC: {
      skip_str<FULL>(b, p, end, ok);
      if (ok) {
        if (DEFER) return PARSE_DEFER;
        const AnySkip r = skip_any_nl<DEPTH, FULL>(b.b, p, end, steps);
        p = r.p;
        steps = r.steps;
        ok = r.ok != 0;
        if (FULL && ok && r.cf) return -1;  // a ContentDoc's options not in writeAny's form: refused
      }
      if (!ok && steps == 0) return -1;
      break;
    }
    default: return 0;
  }
  if (FULL) { v->len = len; v->cpos = cpos; v->cend = p; }
  if (!ok && p >= end) return -2;  // ran out of input (the struct may continue past `end`)
  return ok ? 1 : 0;
}

template <bool FULL, int DEPTH = 32>
YC_HD inline int parse_struct(const uint8_t* __restrict__ b, uint32_t& p, uint32_t end, uint32_t steps, StructView* v) {
  return parse_struct<FULL, DEPTH, RawSrc>(RawSrc{b}, p, end, steps, v);
}

YC_HDI uint32_t vu_size_host(uint32_t v) {
  return v < (1u << 7) ? 1 : v < (1u << 14) ? 2 : v < (1u << 21) ? 3 : v < (1u << 28) ? 4 : 5;
}

}  // namespace yc
