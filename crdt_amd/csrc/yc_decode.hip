// yc_decode.hip — K1: decode of Yjs v1 updates on gfx950.
//
// Replaces lib0's sequential readers + readClientsStructRefs (Y@19286) / readDeleteSet
// (Y@11105) with a parallel decode. Small updates (most of a fleet / gossip batch) take the direct
// path; large ones (snapshots) the chunk path:
//   1. k_direct        one lane per small update parses it exactly through a private LDS window
//                      and writes its words of the struct-start bitmap.
//   1'. k_spec         one lane per 1 KiB chunk of a large update follows the all-struct chain
//                      (next(p) = p + struct length, p + 1 where no struct parses) from the chunk's
//                      first byte and marks every position it visits (spec_bits) and its exit.
//                      Such a chain synchronises with the true struct sequence within a few structs
//                      of any start, and from a true struct start on it IS the true sequence.
//                      It also tabulates, for the first XK entry offsets, where the chain from
//                      that entry leaves the chunk (periodic streams hold chains of several
//                      phases that never meet).
//   2'. k_walk         one wavefront per large update follows the true sequence through the
//                      section headers 64 chunks per step: lane j's entry comes from composing the
//                      exit tables of the chunks before it; it parses exactly until it meets its
//                      chunk's chain and counts the rest by popcount; the first lane whose true
//                      exit differs from the predicted one ends the step.
//   3. k_struct_pos    popcount prefix (scan) -> dense struct index for every struct start.
//   4. k_ds_decode     one wavefront per update decodes the delete set, a pure varuint stream, with a
//                      ballot of terminal bytes + in-register gathers (wavefront prefix scan).
//   5. k_struct_decode one lane per struct: full field decode into the SoA struct table.
#include <algorithm>
#include <cstdlib>

#include "yc_work.h"

namespace yc {

// --------------------------------------------------------------------------- 1. struct sizer
// The speculative struct sizer. Exact on every valid struct; on other bytes it only has to be
// deterministic: chains are trusted only from true struct starts on, and every struct on the true
// sequence is re-parsed exactly by k_struct_decode, which reports a malformed one. Varuints are
// read branch-free from an 8-byte register window.
__device__ __forceinline__ uint64_t win8(const uint8_t* __restrict__ b, uint32_t p) {
  const uint32_t* d = (const uint32_t*)(b + (p & ~3u));  // the batch buffer is padded past its end
  return ((uint64_t)d[0] | ((uint64_t)d[1] << 32)) >> ((p & 3u) * 8);
}
__device__ __forceinline__ uint32_t win4(const uint8_t* __restrict__ b, uint32_t p) {
  const uint32_t* d = (const uint32_t*)(b + (p & ~3u));  // the batch buffer is padded past its end
  return __builtin_amdgcn_alignbyte(d[1], d[0], p & 3u);  // v_alignbyte_b32: the shift counts bytes
}
// ---- the register-window sizer (fast path of every struct walk)
// The 24 bytes from the word holding a struct's start sit in six registers, loaded in one round
// (from the lane's LDS window, or from the batch buffer); T marks the bytes that end a varuint
// (high bit clear). A varuint's length is then a count of trailing zeros of T, and the few bytes
// whose values matter (info byte, element counts, tags, short lengths) come out of the registers
// through a three-level select: one round of loads per struct instead of one dependent LDS /
// memory round trip per field. 24 bytes hold the common structs whole (a map set with a 5-byte
// client id and a short value; a root-map item with its parent name and key).
struct RegWin {
  // named words, not an array: an array indexed through the select tree is turned back into a
  // dynamically indexed (LDS-promoted) alloca by the compiler
  uint32_t r0, r1, r2, r3, r4, r5;
  uint32_t T;
  __device__ __forceinline__ static uint32_t sel(uint32_t m, uint32_t a1, uint32_t a0) { return (a1 & m) | (a0 & ~m); }
  __device__ __forceinline__ uint32_t word(uint32_t k) const {  // k < 6
    const uint32_t m0 = 0u - (k & 1u), m1 = 0u - ((k >> 1) & 1u), m2 = 0u - ((k >> 2) & 1u);
    const uint32_t a0 = sel(m0, r1, r0), a1 = sel(m0, r3, r2), a2 = sel(m0, r5, r4);
    return sel(m2, a2, sel(m1, a1, a0));
  }
  __device__ __forceinline__ uint32_t byte(uint32_t i) const { return (word(i >> 2) >> ((i & 3u) * 8)) & 0xFFu; }
  // length (1..5) of the varuint at byte i < 24; 0: it does not end inside the window within 5 bytes
  __device__ __forceinline__ uint32_t vlen(uint32_t i) const {
    const uint32_t t = T >> i;
    const uint32_t e = t ? (uint32_t)__builtin_ctz(t) + 1u : 0u;
    return e <= 5 ? e : 0u;
  }
  __device__ __forceinline__ static uint32_t nib(uint32_t x) {  // bit j = byte j of x < 0x80
    return ((~x & 0x80808080u) * 0x204081u) >> 28;
  }
  __device__ __forceinline__ void mask() {
    T = nib(r0) | nib(r1) << 4 | nib(r2) << 8 | nib(r3) << 12 | nib(r4) << 16 | nib(r5) << 20;
  }
  __device__ __forceinline__ void load(const uint32_t* g) {
    r0 = g[0]; r1 = g[1]; r2 = g[2]; r3 = g[3]; r4 = g[4]; r5 = g[5];
    mask();
  }
};
constexpr uint32_t WIN_SPAN = 24;
// one lib0 `any` value with a scalar tag at window byte q (tag already read): q moves past it;
// false: another tag, or a length byte outside the window
__device__ __forceinline__ bool win_scalar(const RegWin& x, uint32_t& q, uint32_t tag) {
  switch (tag) {
    case 127: case 126: case 121: case 120: return true;
    case 125: {  // varInt: up to 7 bytes (as the general sizer)
      if (q >= WIN_SPAN) return false;
      const uint64_t t = x.T >> q;
      if (!t) return false;
      const uint32_t l = (uint32_t)__builtin_ctzll(t) + 1u;
      q += l;
      return l <= 7;
    }
    case 124: q += 4; return true;
    case 123: case 122: q += 8; return true;
    case 119: case 116: {  // string / bytes with a one-byte length
      if (q >= WIN_SPAN) return false;
      const uint32_t n = x.byte(q);
      q += 1 + n;
      return n < 128;
    }
    default: return false;
  }
}
// Exact length of the struct whose info byte is window byte o, for the shapes Yjs documents are
// made of: an item placed by origin / right origin or under a named parent / parent id (with a
// key), holding Deleted, String, Binary, Type, or Any with up to 4 scalar values or one-level
// containers of up to 4 scalar members; GC / Skip. NONE: another shape, a field outside the
// window, or a struct past `end` — the general sizer decides. A pure function of the bytes at p
// (the chunk chains, the walker and the direct path all size through it).
__device__ __forceinline__ uint32_t win_len(const RegWin& x, uint32_t o, uint32_t p, uint32_t end) {
  const uint32_t info = x.byte(o), ref = info & 31u;
  uint32_t q = o + 1;
  if (ref == REF_GC || ref == REF_SKIP) {
    const uint32_t l = x.vlen(q);
    if (!l) return NONE;
    q += l;
  } else {
    if (info & 0xC0u) {
      const uint32_t nid = ((info >> 7) & 1u) * 2u + ((info >> 6) & 1u) * 2u;
      for (uint32_t k = 0; k < nid; ++k) {
        const uint32_t l = q < WIN_SPAN ? x.vlen(q) : 0u;
        if (!l) return NONE;
        q += l;
      }
    } else {
      const uint32_t l = q < WIN_SPAN ? x.vlen(q) : 0u;
      if (!l) return NONE;
      if (l == 1 && x.byte(q) == 1u) {  // parent by name: a string
        ++q;
        if (q >= WIN_SPAN) return NONE;
        const uint32_t n = x.byte(q);
        if (n >= 128) return NONE;
        q += 1 + n;
      } else {  // parent by id: two varuints
        q += l;
        for (uint32_t k = 0; k < 2; ++k) {
          const uint32_t m = q < WIN_SPAN ? x.vlen(q) : 0u;
          if (!m) return NONE;
          q += m;
        }
      }
      if (info & 0x20u) {  // parentSub: a string
        if (q >= WIN_SPAN) return NONE;
        const uint32_t n = x.byte(q);
        if (n >= 128) return NONE;
        q += 1 + n;
      }
    }
    if (q >= WIN_SPAN) return NONE;
    switch (ref) {
      case REF_DELETED: {
        const uint32_t l = x.vlen(q);
        if (!l) return NONE;
        q += l;
        break;
      }
      case REF_STRING: case REF_BINARY: {
        const uint32_t n = x.byte(q);
        if (n >= 128) return NONE;
        q += 1 + n;
        break;
      }
      case REF_TYPE: {
        const uint32_t tr = x.byte(q);
        if (tr > 6) return NONE;
        ++q;
        if (tr == 3 || tr == 5) {
          if (q >= WIN_SPAN) return NONE;
          const uint32_t n = x.byte(q);
          if (n >= 128) return NONE;
          q += 1 + n;
        }
        break;
      }
      case REF_ANY: {
        const uint32_t c = x.byte(q);
        if (c == 0 || c > 4) return NONE;
        ++q;
        for (uint32_t e = 0; e < c; ++e) {
          if (q >= WIN_SPAN) return NONE;
          const uint32_t tag = x.byte(q);
          ++q;
          if (tag == 118 || tag == 117) {  // object / array of scalars
            if (q >= WIN_SPAN) return NONE;
            const uint32_t m = x.byte(q);
            if (m > 4) return NONE;
            ++q;
            for (uint32_t j = 0; j < m; ++j) {
              if (tag == 118) {
                if (q >= WIN_SPAN) return NONE;
                const uint32_t kl = x.byte(q);
                if (kl >= 128) return NONE;
                q += 1 + kl;
              }
              if (q >= WIN_SPAN) return NONE;
              const uint32_t t2 = x.byte(q);
              ++q;
              if (!win_scalar(x, q, t2)) return NONE;
            }
          } else if (!win_scalar(x, q, tag)) {
            return NONE;
          }
        }
        break;
      }
      default: return NONE;
    }
  }
  const uint32_t len = q - o;
  return p <= end && len <= end - p ? len : NONE;
}

// Byte sources for the sizer: the slice's bytes staged in LDS (plus a halo past its end), with
// a fallback to the batch buffer (through the caches) for reads beyond the staged window.
struct LdsSrc {
  const uint8_t* __restrict__ b;
  const uint32_t* lw;  // staged words of [s0, wend)
  uint32_t s0, wlen;   // wlen = wend - s0
  // the register window of p: 24 bytes from p & ~3 (staged if the window holds them)
  __device__ __forceinline__ void load_win(uint32_t p, RegWin& x) const {
    const uint32_t a = p & ~3u, o = a - s0;
    x.load((wlen >= WIN_SPAN && o <= wlen - WIN_SPAN) ? lw + (o >> 2) : (const uint32_t*)(b + a));
  }
  __device__ __forceinline__ uint32_t u8(uint32_t p) const {
    const uint32_t o = p - s0;
    return o < wlen ? (lw[o >> 2] >> ((o & 3u) * 8)) & 0xFFu : (uint32_t)b[p];
  }
  __device__ __forceinline__ uint64_t w8(uint32_t p) const {
    const uint32_t o = p - s0;
    if (o + 8 <= wlen) return ((uint64_t)lw[o >> 2] | ((uint64_t)lw[(o >> 2) + 1] << 32)) >> ((o & 3u) * 8);
    return win8(b, p);
  }
  __device__ __forceinline__ uint32_t w4(uint32_t p) const {
    const uint32_t o = p - s0;
    if (o + 4 <= wlen) return __builtin_amdgcn_alignbyte(lw[(o >> 2) + 1], lw[o >> 2], o & 3u);
    return win4(b, p);
  }
};
// varuint from a 4-byte window (+ the fifth byte when the first four all continue): one funnel
// shift and a 7-bit-group compaction in 32-bit arithmetic; lib0 0.2.42 accumulates in 32 bits,
// so the fifth byte contributes its low four bits
template <class S>
__device__ __forceinline__ uint32_t vu_fast(const S& b, uint32_t& p, uint32_t end, bool& ok) {
  const uint32_t w = b.w4(p);
  const uint32_t t = ~w & 0x80808080u;  // terminal bytes among the first four
  uint32_t v = (w & 0x7fu) | ((w >> 1) & 0x3f80u) | ((w >> 2) & 0x1fc000u) | ((w >> 3) & 0xfe00000u);
  uint32_t len;
  if (t) {
    len = ((uint32_t)__builtin_ctz(t) >> 3) + 1;
    v &= len >= 4 ? 0x0FFFFFFFu : ((1u << (7 * len)) - 1u);
  } else {
    const uint32_t b4 = b.u8(p + 4);
    len = b4 < 0x80u ? 5u : 6u;
    v |= b4 << 28;
  }
  ok = ok && len <= 5 && end - p >= len && p < end;
  p += len;
  return v;
}
__device__ __forceinline__ void skip_n(uint32_t& p, uint32_t n, uint32_t end, bool& ok) {
  const bool f = p <= end && n <= end - p;
  ok = ok && f;
  p = f ? p + n : end;
}
// one `any` value (L0@1937) that is not a container; false: a container, or more than this sizer does
template <class S>
__device__ __forceinline__ bool any_simple(const S& b, uint32_t& p, uint32_t end, bool& ok) {
  if (p >= end) { ok = false; return true; }
  const uint32_t tag = b.u8(p++);
  switch (tag) {
    case 127: case 126: case 121: case 120: return true;
    case 125: {  // varInt
      const uint64_t t = ~b.w8(p) & 0x8080808080ull;
      const uint32_t len = t ? ((uint32_t)__builtin_ctzll(t) >> 3) + 1
                             : (p + 5 < end && b.u8(p + 5) < 0x80u ? 6u : (p + 6 < end && b.u8(p + 6) < 0x80u ? 7u : 8u));
      ok = ok && len <= 7 && end - p >= len;  // skip_vi: a first byte and up to six more
      p += len;
      return true;
    }
    case 124: skip_n(p, 4, end, ok); return true;
    case 123: case 122: skip_n(p, 8, end, ok); return true;
    case 119: case 116: { const uint32_t n = vu_fast(b, p, end, ok); skip_n(p, n, end, ok); return true; }
    case 118: case 117: return false;
    default: ok = false; return true;
  }
}
constexpr uint32_t SIZER_MAX_ELEMS = 16;
// Length of the varuint at p (1..5 bytes), 0 when its fifth byte still continues.
template <class S>
__device__ __forceinline__ uint32_t vu_len(const S& b, uint32_t p) {
  const uint32_t t = ~b.w4(p) & 0x80808080u;
  return t ? ((uint32_t)__builtin_ctz(t) >> 3) + 1 : (b.u8(p + 4) < 0x80u ? 5u : 0u);
}
// The sizer's fast path for the commonest struct shapes — an item placed by origin and / or right
// origin (no parent info) whose content is Deleted, String, or Any with one scalar value (a map
// set, a list insert): the ids are only skipped (terminal bytes, no value), so a struct step issues
// a fraction of the general path's instructions. Exact lengths on valid structs, as spec_len;
// NONE: another shape or anything spec_len must judge (running past `end`, long varInts).
template <class S>
__device__ __forceinline__ uint32_t spec_len_common(const S& b, uint32_t pos, uint32_t end, uint32_t ref, uint32_t bits) {
  uint32_t p = pos + 1;
  const uint32_t nid = ((bits >> 7) & 1u) * 2u + ((bits >> 6) & 1u) * 2u;  // origin / right origin: 2 varuints each
  for (uint32_t k = 0; k < nid; ++k) {
    const uint32_t l = vu_len(b, p);
    if (!l) return NONE;
    p += l;
  }
  if (ref == REF_ANY) {
    const uint32_t w = b.w4(p);
    if ((w & 0xFFu) != 1u) return NONE;  // one element
    const uint32_t tag = (w >> 8) & 0xFFu;
    p += 2;
    if (tag == 125) {  // varInt: a first byte and up to three more here
      const uint32_t t = ~b.w4(p) & 0x80808080u;
      if (!t) return NONE;
      p += ((uint32_t)__builtin_ctz(t) >> 3) + 1;
    } else if (tag == 119) {  // string
      const uint32_t l = vu_len(b, p);
      if (!l || l > 4) return NONE;
      const uint32_t n = b.w4(p) & 0x7Fu;
      if (l > 1) return NONE;  // short strings only (one length byte)
      p += 1 + n;
    } else if (tag == 120 || tag == 121 || tag == 126 || tag == 127) {
    } else if (tag == 124) {
      p += 4;
    } else if (tag == 123 || tag == 122) {
      p += 8;
    } else {
      return NONE;
    }
  } else {  // Deleted: a length; String: a byte length and the bytes
    const uint32_t w = b.w4(p);
    const uint32_t t = ~w & 0x80808080u;
    if (!t) return NONE;
    const uint32_t l = ((uint32_t)__builtin_ctz(t) >> 3) + 1;
    if (ref == REF_STRING) {
      const uint32_t n = (w & 0x7fu) | ((w >> 1) & 0x3f80u) | ((w >> 2) & 0x1fc000u) | ((w >> 3) & 0xfe00000u);
      p += l + (n & (l >= 4 ? 0x0FFFFFFFu : ((1u << (7 * l)) - 1u)));
    } else {
      p += l;
    }
  }
  return p <= end && p - pos < 0x10000u ? p - pos : NONE;
}
// struct length, 0 = not a struct, 1 = hand over to parse_struct (many elements, deep nesting, Doc)
template <class S>
__device__ __forceinline__ uint32_t spec_len(const S& b, uint32_t pos, uint32_t end, uint32_t cls) {
  const uint32_t ref = cls / 8 + 1, bits = (cls % 8) << 5;
  if ((bits & 0xC0u) && (ref == REF_ANY || ref == REF_STRING || ref == REF_DELETED)) {
    const uint32_t d = spec_len_common(b, pos, end, ref, bits);
    if (d != NONE) return d;
  }
  bool ok = true;
  uint32_t p = pos + 1;
  if (bits & 0x80u) { vu_fast(b, p, end, ok); vu_fast(b, p, end, ok); }
  if (bits & 0x40u) { vu_fast(b, p, end, ok); vu_fast(b, p, end, ok); }
  if (!(bits & 0xC0u)) {
    const uint32_t pinfo = vu_fast(b, p, end, ok);
    if (pinfo == 1) { const uint32_t n = vu_fast(b, p, end, ok); skip_n(p, n, end, ok); }
    else { vu_fast(b, p, end, ok); vu_fast(b, p, end, ok); }
    if (bits & 0x20u) { const uint32_t n = vu_fast(b, p, end, ok); skip_n(p, n, end, ok); }
  }
  switch (ref) {
    case REF_DELETED: vu_fast(b, p, end, ok); break;
    case REF_BINARY: case REF_STRING: { const uint32_t n = vu_fast(b, p, end, ok); skip_n(p, n, end, ok); break; }
    case REF_EMBED: {
      const uint32_t n = vu_fast(b, p, end, ok);
      ok = ok && n > 0 && p < end && json_start_ok(b.u8(p));
      skip_n(p, n, end, ok);
      break;
    }
    case REF_FORMAT: {
      uint32_t n = vu_fast(b, p, end, ok);
      skip_n(p, n, end, ok);
      n = vu_fast(b, p, end, ok);
      ok = ok && n > 0 && p < end && json_start_ok(b.u8(p));
      skip_n(p, n, end, ok);
      break;
    }
    case REF_TYPE: {
      const uint32_t tr = vu_fast(b, p, end, ok);
      if (tr == 3 || tr == 5) { const uint32_t n = vu_fast(b, p, end, ok); skip_n(p, n, end, ok); }
      ok = ok && tr <= 6;
      break;
    }
    // more than SIZER_MAX_ELEMS elements / members: handed over to parse_struct once the first
    // SIZER_MAX_ELEMS parse (a valid struct always passes; garbage on a chunk chain rarely does,
    // and the exact parser would crawl through it byte by byte from memory)
    case REF_JSON: {
      const uint32_t n = vu_fast(b, p, end, ok);
      for (uint32_t i = 0; i < n && i < SIZER_MAX_ELEMS && ok; ++i) {
        const uint32_t k = vu_fast(b, p, end, ok);
        ok = ok && k > 0 && p < end && json_start_ok(b.u8(p));
        skip_n(p, k, end, ok);
      }
      if (ok && n > SIZER_MAX_ELEMS) return 1;
      break;
    }
    case REF_ANY: {
      const uint32_t n = vu_fast(b, p, end, ok);
      for (uint32_t i = 0; i < n && i < SIZER_MAX_ELEMS && ok; ++i) {
        const uint32_t q0 = p;
        if (any_simple(b, p, end, ok)) continue;
        // a container one level deep with simple members; anything deeper goes to parse_struct
        const bool obj = b.u8(q0) == 118;
        const uint32_t m = vu_fast(b, p, end, ok);
        for (uint32_t j = 0; j < m && j < SIZER_MAX_ELEMS && ok; ++j) {
          if (obj) { const uint32_t k = vu_fast(b, p, end, ok); skip_n(p, k, end, ok); }
          if (!any_simple(b, p, end, ok)) return ok ? 1u : 0u;
        }
        if (ok && m > SIZER_MAX_ELEMS) return 1;
      }
      if (ok && n > SIZER_MAX_ELEMS) return 1;
      break;
    }
    default: {  // ContentDoc: a guid string, then an `any` (handed over when its tag is one)
      const uint32_t n = vu_fast(b, p, end, ok);
      skip_n(p, n, end, ok);
      if (!ok || p >= end) return 0;
      const uint32_t tag = b.u8(p);
      return tag >= 116 && tag <= 127 ? 1u : 0u;
    }
  }
  if (!ok) return 0;
  return p - pos < 0x10000u ? p - pos : 1u;
}

// Direct path: one lane per small update parses it exactly, struct by struct, and writes the
// update's struct-start words of the final bitmap itself (updates are 64-byte aligned, so the
// words are the lane's own: plain stores, each word once, as the lane moves forward). Each lane
// reads its update through a private LDS window of DW bytes, refilled with 16-byte loads when
// fewer than DREFILL bytes are left (the register window of the struct start then always comes
// from LDS): the parse waits on LDS, not on L2 / HBM (a wavefront touches 64 different updates,
// far more lines than L1 keeps). Structs are sized by the register-window sizer, then the
// speculative sizer (both exact on valid structs); what they hand over is parsed by parse_struct.
constexpr uint32_t DW = 128;                    // window bytes per lane
constexpr uint32_t DSTRIDE = DW / 4 + 4;        // words per lane slot (16-byte padded)
constexpr uint32_t DREFILL = WIN_SPAN + 16;
constexpr uint32_t DL = 256;                    // lanes per direct workgroup
// A window refill: all DW/16 loads issued before the first LDS store, so a refill costs one
// memory round trip (a loop bounded by wlen waited on each load in turn). The batch buffer is
// padded past its end, and bytes past wlen are never taken from the window.
template <uint32_t W = DW>
__device__ __forceinline__ void fill_window(uint32_t* slot, const uint4* __restrict__ g) {
  uint4 v[W / 16];
#pragma unroll
  for (uint32_t k = 0; k < W / 16; ++k) v[k] = g[k];
#pragma unroll
  for (uint32_t k = 0; k < W / 16; ++k) ((uint4*)slot)[k] = v[k];
}
// the exact parser out of line: inlined, its nested-`any` walker multiplies the register demand
// of the lane loop (one wavefront per SIMD), and it only runs on the few handed-over structs
__device__ __attribute__((noinline)) uint32_t exact_len(const uint8_t* __restrict__ b, uint32_t p, uint32_t end) {
  uint32_t q = p;
  return parse_struct<false>(b, q, end, 0xFFFFFFFFu, nullptr) > 0 ? q - p : 0u;
}
// (one update's exact walk through the lane's LDS window `slot`)
template <uint32_t DWT>
__device__ __forceinline__ void direct_walk(const Work& w, uint32_t u, uint32_t* slot) {
  const uint32_t uw = upd_win(w, u);  // positions below are relative to the update's window
  const uint8_t* __restrict__ b = win_bytes(w, uw);
  uint64_t* __restrict__ fbits = win_words(w.final_bits, uw);
  uint64_t* __restrict__ sbits = win_words(w.sec_bits, uw);
  const uint32_t ustart = w.uoff[u], uend = ustart + w.ulen[u];
  uint32_t* err = &w.ctr->err;
  LdsSrc src{b, slot, 0, 0};
  auto refill = [&](uint32_t p) {
    src.s0 = p & ~15u;
    src.wlen = min(DWT, (uend + 15u - src.s0) & ~15u);
    const uint4* g = (const uint4*)(b + src.s0);
    fill_window<DWT>(slot, g);
  };
  w.dsstart[u] = NONE;
  bool ok = true;
  uint32_t p = ustart;
  const uint32_t nsec = rd_vu(b, p, uend, ok);
  if (!ok || nsec > (uend - p) / 3 + 1) { raise_err(err, ERR_DECODE); return; }
  const uint32_t sbase = atomicAdd(&w.ctr->nsections, nsec);
  if (sbase + nsec > w.cap_sections) { raise_err(err, ERR_CAPACITY); return; }
  w.usec_start[u] = sbase;
  w.usec_n[u] = nsec;
  refill(p);
  uint32_t word = NONE;
  uint64_t m = 0;
  for (uint32_t sct = 0; sct < nsec; ++sct) {
    const uint32_t n = rd_vu(b, p, uend, ok);  // headers: the walkers' exact reader
    const uint32_t client = rd_vu(b, p, uend, ok);
    const uint32_t clock = rd_vu(b, p, uend, ok);
    if (!ok || n > uend - p) { raise_err(err, ERR_DECODE); return; }
    Section sec;
    sec.upd = u; sec.n = n; sec.client = client; sec.clock = clock;
    sec.first_pos = n ? p : NONE; sec.cidx = NONE; sec.first_idx = NONE; sec.pad = 0;
    w.sections[sbase + sct] = sec;
    if (n) atomicOr((unsigned long long*)&sbits[p >> 6], 1ull << (p & 63));
    for (uint32_t k = 0; k < n; ++k) {
      if (p >= uend) { raise_err(err, ERR_DECODE); w.ctr->err_info = p; return; }
      if ((p >> 6) != word) {
        if (word != NONE) fbits[word] = m;
        word = p >> 6;
        m = 0;
      }
      m |= 1ull << (p & 63);
      // the whole wavefront at once: one stall, not one per lane (a window that already reaches
      // the update end is never refilled)
      if (__ballot(src.wlen == DWT && p - src.s0 + DREFILL > DWT)) refill(p);
      RegWin x;
      src.load_win(p, x);
      uint32_t d = win_len(x, p & 3u, p, uend);
      if (d == NONE) {
        const uint32_t info = src.u8(p), ref = info & 31u;
        d = 0;
        if (ref == REF_GC || ref == REF_SKIP) {
          uint32_t q = p + 1;
          bool okv = true;
          vu_fast(src, q, uend, okv);
          d = okv ? q - p : 0u;
        } else if (ref >= 1 && ref <= REF_DOC) {
          d = spec_len(src, p, uend, (ref - 1) * 8 + (info >> 5));
        }
        if (d <= 1) {  // handed over (long / deep / Doc), or not sized: the exact parser decides
          d = exact_len(b, p, uend);
          if (!d) { raise_err(err, ERR_DECODE); w.ctr->err_info = p; return; }
        }
      }
      p += d;
    }
  }
  if (word != NONE) fbits[word] = m;
  w.dsstart[u] = p;
}
template <uint32_t DWT>
__global__ __launch_bounds__(DL) void k_direct(Work w) {
  constexpr uint32_t DSTR = DWT / 4 + 4;
  __shared__ __attribute__((aligned(16))) uint32_t win[DL * DSTR];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < w.nsmall) direct_walk<DWT>(w, w.ulist[w.nbig + i], win + threadIdx.x * DSTR);
}


// --------------------------------------------------------------------------- 1'. chunk chains
// Struct length at p on the all-struct chain, 0 where no struct parses (the chain then steps one
// byte). The chunk chains and the walker use this one function, so chains that meet stay together.
template <class S>
__device__ __forceinline__ uint32_t chain_len(const S& src, const uint8_t* __restrict__ b, uint32_t p, uint32_t uend,
                                              unsigned long long* dbg = nullptr, const uint8_t* xb = nullptr,
                                              uint32_t xoff = 0) {
  {
    RegWin x;
    src.load_win(p, x);
    const uint32_t f = win_len(x, p & 3u, p, uend);
    if (f != NONE) return f;
  }
  const uint32_t info = src.u8(p), ref = info & 31u;
  uint32_t d = 0;
  if (ref == REF_GC || ref == REF_SKIP) {
    uint32_t q = p + 1;
    bool okv = true;
    vu_fast(src, q, uend, okv);
    d = okv ? q - p : 0u;
  } else if (ref >= 1 && ref <= REF_DOC) {
    d = spec_len(src, p, uend, (ref - 1) * 8 + (info >> 5));
    if (d == 1) {  // handed over (long / deep / Doc)
      // (xb: the update staged in LDS, xoff its first position: the exact parser reads LDS)
      d = xb ? exact_len(xb, p - xoff, uend - xoff) : exact_len(b, p, uend);
      if (dbg) { atomicAdd(&dbg[6], 1ull); atomicAdd(&dbg[7], (unsigned long long)d); }
    }
  }
  return d;
}
struct GlobalSrc {
  const uint8_t* __restrict__ b;
  __device__ __forceinline__ void load_win(uint32_t p, RegWin& x) const { x.load((const uint32_t*)(b + (p & ~3u))); }
  __device__ __forceinline__ uint32_t u8(uint32_t p) const { return b[p]; }
  __device__ __forceinline__ uint64_t w8(uint32_t p) const { return win8(b, p); }
  __device__ __forceinline__ uint32_t w4(uint32_t p) const { return win4(b, p); }
};
// parse_struct's source for k_struct_decode: the struct's first bytes staged in the lane's LDS
// window by one round of loads (SW_WIN bytes from the 16-byte line holding its start), the rest of
// a longer struct read from the batch buffer; varuints / varInts word-wide as in FastSrc. The
// field-by-field parse then waits on LDS instead of on one memory round trip per field.
constexpr uint32_t SD_WIN = 64, SD_STRIDE = SD_WIN / 4 + 4;
struct WinSrc {
  const uint8_t* __restrict__ b;
  const uint32_t* lw;
  uint32_t s0;
  __device__ __forceinline__ uint32_t u8(uint32_t p) const {
    const uint32_t o = p - s0;
    return o < SD_WIN ? (lw[o >> 2] >> ((o & 3u) * 8)) & 0xFFu : (uint32_t)b[p];
  }
  __device__ __forceinline__ uint32_t w4(uint32_t p) const {
    const uint32_t o = p - s0;
    if (o + 4 <= SD_WIN) return __builtin_amdgcn_alignbyte(lw[(o >> 2) + 1], lw[o >> 2], o & 3u);
    return win4(b, p);
  }
  __device__ __forceinline__ uint64_t w8(uint32_t p) const {
    const uint32_t o = p - s0;
    if (o + 8 <= SD_WIN) {
      const uint32_t i = o >> 2, sh = o & 3u;
      const uint32_t lo = __builtin_amdgcn_alignbyte(lw[i + 1], lw[i], sh), hi = __builtin_amdgcn_alignbyte(lw[i + 2], lw[i + 1], sh);
      return (uint64_t)lo | ((uint64_t)hi << 32);
    }
    return win8(b, p);
  }
  __device__ __forceinline__ uint32_t vu(uint32_t& p, uint32_t end, bool& ok) const {
    if (p >= end) { ok = false; return 0; }
    return vu_fast(*this, p, end, ok);
  }
  __device__ __forceinline__ void svi(uint32_t& p, uint32_t end, bool& ok) const {  // readVarInt: at most 7 bytes
    if (p >= end) { ok = false; return; }
    const uint64_t t = ~w8(p) & 0x80808080808080ull;
    const uint32_t len = t ? ((uint32_t)__builtin_ctzll(t) >> 3) + 1 : 8u;
    ok = ok && len <= 7 && end - p >= len;
    p = ok ? p + len : end;
  }
};
// parse_struct's byte source for the exact decode: varuints / varInts read word-wide from the
// batch buffer instead of byte by byte (the same values and the same accept / reject)
struct FastSrc {
  const uint8_t* __restrict__ b;
  __device__ __forceinline__ uint32_t u8(uint32_t p) const { return b[p]; }
  __device__ __forceinline__ uint64_t w8(uint32_t p) const { return win8(b, p); }
  __device__ __forceinline__ uint32_t w4(uint32_t p) const { return win4(b, p); }
  __device__ __forceinline__ uint32_t vu(uint32_t& p, uint32_t end, bool& ok) const {
    if (p >= end) { ok = false; return 0; }
    return vu_fast(*this, p, end, ok);
  }
  __device__ __forceinline__ void svi(uint32_t& p, uint32_t end, bool& ok) const {  // readVarInt: at most 7 bytes
    if (p >= end) { ok = false; return; }
    const uint64_t t = ~win8(b, p) & 0x80808080808080ull;
    const uint32_t len = t ? ((uint32_t)__builtin_ctzll(t) >> 3) + 1 : 8u;
    ok = ok && len <= 7 && end - p >= len;
    p = ok ? p + len : end;
  }
};
__device__ __forceinline__ uint32_t chain_step(const uint8_t* __restrict__ b, uint32_t p, uint32_t uend) {
  const uint32_t d = chain_len(GlobalSrc{b}, b, p, uend);
  return p + (d ? d : 1u);
}
// Step table of a record-mode update (k_rtab): chain_len at every byte, computed once on the whole
// chip, so the chunk chains, the sync rounds, the section-step records and the walkers of that update
// follow the chain by one load per step instead of ~1 500 dependent instructions (k_spec held one
// lane per 512-byte chunk: 16 K lanes, a wavefront per SIMD, 2.5 ms on a C2 document state).
// tab: the update's table (indexed by p - ustart), nullptr for the other updates.
__device__ __forceinline__ const uint32_t* rtab_of(const Work& w, uint32_t u) {
  return w.rtab && w.fwc_off[u] != NONE ? w.rtab + w.fwc_off[u] : nullptr;
}
template <class S>
__device__ __forceinline__ uint32_t tab_len(const uint32_t* __restrict__ tab, uint32_t ustart, const S& src, const uint8_t* __restrict__ b,
                                            uint32_t p, uint32_t uend) {
  return tab && p < uend ? tab[p - ustart] : chain_len(src, b, p, uend);
}
__device__ __forceinline__ uint32_t tab_step(const uint32_t* __restrict__ tab, uint32_t ustart, const uint8_t* __restrict__ b, uint32_t p,
                                             uint32_t uend) {
  const uint32_t d = tab_len(tab, ustart, GlobalSrc{b}, b, p, uend);
  return p + (d ? d : 1u);
}
// one lane per byte of the record-mode updates (grid-stride over the chunk table); a byte whose
// struct-kind bits name no struct (ref > Skip) is chain_len's 0 without a parse
__global__ __launch_bounds__(256) void k_rtab(Work w) {
  const uint32_t CH = w.schunk;
  const uint64_t total = (uint64_t)w.ngroups * CH;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    const Group G = w.groups[t / CH];
    const uint32_t p = G.start + (uint32_t)(t % CH);
    if (p >= G.end) continue;
    const uint32_t off = w.fwc_off[G.upd];
    if (off == NONE) continue;
    const uint8_t* __restrict__ b = win_bytes(w, upd_win(w, G.upd));
    const uint32_t ustart = w.uoff[G.upd];
    w.rtab[off + (p - ustart)] = (b[p] & 31u) > REF_SKIP ? 0u : chain_len(GlobalSrc{b}, b, p, G.uend);
  }
}

// One lane per chunk (SCHUNK bytes of a large update): the chain from the chunk's start (below), every
// visited position inside the chunk set in spec_bits (the lane owns the chunk's words: chunks and
// updates are 64-byte aligned) and the first position at / past the chunk end in cexit. The bytes
// come through the lane's LDS window, as in k_direct.
// k_spec's window is shorter than the direct path's: a chunk path of many chunks needs more
// wavefronts resident per CU than the direct path's one lane per update
constexpr uint32_t SPW = 128, SPSTRIDE = SPW / 4 + 4;
__global__ __launch_bounds__(DL) void k_spec(Work w) {
  __shared__ __attribute__((aligned(16))) uint32_t win[DL * SPSTRIDE];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= w.ngroups) return;
  const Group G = w.groups[i];
  if (w.ufail[G.upd] >= UF_PRE) { w.cexit[i] = G.end; return; }  // (decoded already — by its marks, or whole by k_prewalk: its chunks serve the grid delete-set decode only)
  const uint32_t uw = upd_win(w, G.upd);
  const uint8_t* __restrict__ b = win_bytes(w, uw);
  const uint32_t uend = G.uend;
  const uint32_t* __restrict__ tab = rtab_of(w, G.upd);
  const uint32_t ustart = w.uoff[G.upd];
  uint32_t* slot = win + threadIdx.x * SPSTRIDE;
  LdsSrc src{b, slot, 0, 0};
  auto refill = [&](uint32_t p) {
    src.s0 = p & ~15u;
    src.wlen = min(SPW, (uend + 15u - src.s0) & ~15u);
    const uint4* g = (const uint4*)(b + src.s0);
    fill_window<SPW>(slot, g);
  };
  uint64_t* __restrict__ spec = win_words(w.spec_bits, uw);
  // Where the chain starts. The first chunk of an update: at its first struct (the headers are
  // read exactly). Any other chunk of a single-section update (by default; w.spec_hint): at the
  // first position of its first 96 bytes where three
  // consecutive chain steps start with the info byte of the update's first struct (a stream of
  // similar structs: one replica's pushes, a snapshot) — a guess the walker verifies, which keeps a
  // chunk's chain out of the self-consistent wrong phases such streams lock into (§5.4b); else at
  // the chunk's first byte.
  uint32_t start = G.start;
  {
    const uint32_t u0 = w.uoff[G.upd];
    uint32_t h = u0;
    bool okh = true;
    const uint32_t nsec = rd_vu(b, h, uend, okh);
    const uint32_t n0 = nsec ? rd_vu(b, h, uend, okh) : 0u;
    if (nsec) { rd_vu(b, h, uend, okh); rd_vu(b, h, uend, okh); }
    if (okh && n0 && h < uend) {
      if (G.start == u0) {
        start = min(h, G.end);
      } else if (w.spec_hint == 1u || (w.spec_hint == 2u && nsec == 1)) {
        const uint32_t hint = b[h];
        refill(G.start);
        const uint32_t lim = min(G.start + 96u, G.end);
        for (uint32_t q = G.start; q < lim; ++q) {
          if (src.u8(q) != hint) continue;
          const uint32_t d1 = tab_len(tab, ustart, src, b, q, uend);
          if (!d1 || q + d1 >= uend || src.u8(q + d1) != hint) continue;
          const uint32_t d2 = tab_len(tab, ustart, src, b, q + d1, uend);
          if (!d2 || q + d1 + d2 >= uend || src.u8(q + d1 + d2) != hint) continue;
          start = q;
          break;
        }
      } else if (w.spec_hint == 2u) {
        // several sections (a full state: one section per client): the chunk's own struct kind is
        // unknown, so the hint is SELF-similar — the first of the first 96 bytes where three
        // consecutive chain steps start with the same struct-kind byte. A snapshot section of one
        // client's similar structs (C2's base: 15-byte root map entries; its replicas' 4-byte
        // deleted entries) otherwise locks every chain into a wrong phase for its whole length
        // (else the first position whose chain parses four structs in a row: wrong phases of a
        // stream of text keys run into bytes no struct starts with)
        refill(G.start);
        const uint32_t lim = min(G.start + 96u, G.end);
        uint32_t valid4 = NONE;
        for (uint32_t q = G.start; q < lim; ++q) {
          const uint32_t c = src.u8(q);
          if ((c & 31u) > REF_SKIP) continue;
          const uint32_t d1 = tab_len(tab, ustart, src, b, q, uend);
          if (!d1 || q + d1 >= uend) continue;
          const uint32_t d2 = tab_len(tab, ustart, src, b, q + d1, uend);
          if (!d2 || q + d1 + d2 >= uend) continue;
          if (src.u8(q + d1) == c && src.u8(q + d1 + d2) == c) { start = q; valid4 = NONE; break; }
          if (valid4 == NONE) {
            const uint32_t q3 = q + d1 + d2, d3 = tab_len(tab, ustart, src, b, q3, uend);
            if (d3 && q3 + d3 < uend && tab_len(tab, ustart, src, b, q3 + d3, uend)) valid4 = q;
          }
        }
        if (valid4 != NONE && start == G.start) start = valid4;
      }
    }
  }
  uint32_t p = start, word = G.start >> 6;
  uint64_t m = 0;
  refill(p);
  while (p < G.end) {
    if ((p >> 6) != word) {
      spec[word] = m;
      m = 0;
      while (++word < (p >> 6)) spec[word] = 0;
    }
    m |= 1ull << (p & 63);
    if (__ballot(src.wlen == SPW && p - src.s0 + DREFILL > SPW)) refill(p);  // the whole wavefront at once
    const uint32_t d = tab_len(tab, ustart, src, b, p, uend);
    p += d ? d : 1u;
  }
  const uint32_t wend = (G.end + 63) >> 6;
  spec[word] = m;
  while (++word < wend) spec[word] = 0;
  w.cexit[i] = p;
}

// One lane per chunk re-enters it where the previous chunk's chain leaves (xin of chunk j-1): from
// there the chain is followed until it meets the chunk's own chain, and the chunk's words of
// spec_bits are rewritten to that one chain (walked positions, then the own chain from the meeting
// point); its exit goes to xout. A chain meets the true struct sequence within ~100 bytes of its
// start in the median (C2 snapshots: 90 % within 400 bytes), so after one round nearly every
// chunk's chain is the true sequence from its first struct on; later rounds re-enter the few
// chunks behind a chunk whose chain had not met it, and the walker finds its entries on the chains. A chunk the chain jumps over entirely (one long struct) gets no
// positions. The first chunk of an update keeps its chain (the walker enters it after the update /
// section headers).
// Rounds repeat (SYNC_ROUNDS, xin / xout alternating): a chunk is re-walked only when its entry
// changed since its last walk (sent), and a round after one that changed no exit only copies. A
// chunk whose own chain never met the true sequence passes the true exit on one round later, so
// an isolated such chunk costs one more round, not a hand-over of its update to the walker (an
// 11 MB C4 state has ~11 k chunks: one of them out of phase used to fail the whole fast walk).
constexpr uint32_t SYNC_ROUNDS = 6;  // even: the last round writes cexit
__global__ __launch_bounds__(256) void k_sync(Work w, const uint32_t* __restrict__ xin, uint32_t* __restrict__ xout,
                                              uint32_t round) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= w.ngroups) return;
  uint32_t X = xin[i];
  if (round > 0 && !w.ctr->sync_changed[round - 1]) { xout[i] = X; return; }
  const Group G = w.groups[i];
  if (G.start != w.uoff[G.upd] && w.ufail[G.upd] < UF_PRE) {  // chunks of one update are consecutive
    const uint32_t E = xin[i - 1];
    uint32_t* jumped = w.sent + w.ngroups + 1;
    if (E >= G.end) {
      // the predecessor's chain jumps over the whole chunk: a long struct, or (far more often on
      // a chunk's own chain) garbage parsed as a long string. Passing such an exit on would cascade
      // one chunk per round; the chunk keeps its own chain and is flagged, so the update only
      // reaches the fast walk once a later round enters it from inside the chunk
      w.sent[i] = E;
      jumped[i] = 1u;
    } else if (round == 0 || E != w.sent[i]) {
      w.sent[i] = E;
      jumped[i] = 0u;
      const uint32_t uw = upd_win(w, G.upd);
      const uint8_t* __restrict__ b = win_bytes(w, uw);
      uint64_t* __restrict__ spec = win_words(w.spec_bits, uw);
      const uint32_t* __restrict__ tab = rtab_of(w, G.upd);
      const uint32_t ustart = w.uoff[G.upd];
      uint32_t q = E, word = G.start >> 6;
      uint64_t m = 0;
      while (q < G.end && !((spec[q >> 6] >> (q & 63)) & 1ull)) {
        while ((q >> 6) != word) { spec[word] = m; m = 0; ++word; }
        m |= 1ull << (q & 63);
        q = tab_step(tab, ustart, b, q, G.uend);
      }
      if (q < G.end) {  // met the own chain at q: keep its positions from q on
        while ((q >> 6) != word) { spec[word] = m; m = 0; ++word; }
        spec[word] = m | (spec[word] & (~0ull << (q & 63)));
      } else {
        const uint32_t wend = (G.end + 63) >> 6;
        for (; word < wend; ++word) { spec[word] = m; m = 0; }
        X = q;
      }
    }
  }
  xout[i] = X;
  if (X != xin[i]) atomicOr(&w.ctr->sync_changed[round], 1u);
}


// Fallback for updates whose chunk chains lock into a wrong phase (the walker gave up on them:
// periodic struct streams, e.g. a snapshot of identical structs, hold chains of several phases
// that never meet, so the previous chunk's chain exit is no entry into the next chunk). For each
// chunk of such an update one wavefront tabulates, for every entry offset e < XK, the chain from
// start + e: where it leaves the chunk and how many positions it visits inside. Lane e walks
// offset e over the chunk staged in LDS; every visited position records (lane, step) in an LDS
// word, and a lane landing on a recorded position has merged into that lane's chain (same exit,
// the rest of its count). Merged lanes stop, so a wavefront costs about one chunk walk however
// many phases there are. The walker composes the tables to enter every chunk at its true struct.
constexpr uint32_t SW = SCHUNK / 64;  // bitmap words per chunk
constexpr uint32_t XHALO = 256;       // staged bytes past the chunk end
constexpr uint32_t XFAR = 0xFFFFu;    // exit table: 64 KiB or more past the chunk end
__global__ __launch_bounds__(64) void k_xtab(Work w) {
  __shared__ __attribute__((aligned(16))) uint32_t cb[(SCHUNK + XHALO) / 4];
  __shared__ uint32_t rec[SCHUNK];  // (lane << 16) | step of the first visit, NONE: unvisited
  __shared__ uint32_t res_exit[64], res_cnt[64], res_done[64];
  const uint32_t e = threadIdx.x, nx = w.ctr->xchunks;
  for (uint32_t t = blockIdx.x; t < nx; t += gridDim.x) {
  const uint32_t i = w.xlist[t];
  const Group G = w.groups[i];
  const uint8_t* __restrict__ b = win_bytes(w, upd_win(w, G.upd));
  const uint32_t uend = G.uend, cs = G.start;
  const uint32_t wlen = min(SCHUNK + XHALO, (uend + 15u - cs) & ~15u);
  for (uint32_t k = e; k < wlen / 16; k += 64) ((uint4*)cb)[k] = ((const uint4*)(b + cs))[k];
  for (uint32_t k = e; k < SCHUNK; k += 64) rec[k] = NONE;
  if (e == 0) w.tentry[i] = NONE;
  __syncthreads();
  const LdsSrc src{b, cb, cs, wlen};
  const uint32_t* __restrict__ tab = rtab_of(w, G.upd);
  const uint32_t ustart = w.uoff[G.upd];
  uint32_t q = cs + e, k = 0, tgt = NONE, tidx = 0;
  bool active = true;
  for (;;) {
    bool claim = false;
    if (active) {
      if (q >= G.end) active = false;
      else {
        const uint32_t v = rec[q - cs];
        if (v != NONE) { tgt = v >> 16; tidx = v & 0xFFFFu; active = false; }
        else { rec[q - cs] = (e << 16) | k; claim = true; }
      }
    }
    __syncthreads();
    if (claim) {  // two lanes on one position in the same step: the last writer keeps it
      const uint32_t v = rec[q - cs];
      if ((v >> 16) != e) { tgt = v >> 16; tidx = v & 0xFFFFu; active = false; }
      else {
        const uint32_t d = tab_len(tab, ustart, src, b, q, uend);
        q += d ? d : 1u;
        ++k;
      }
    }
    if (!__ballot(active)) break;
    __syncthreads();
  }
  // resolve merges: a merged lane takes its target's exit and the target's count from the merge
  res_done[e] = tgt == NONE ? 1u : 0u;
  res_exit[e] = q;
  res_cnt[e] = k;
  __syncthreads();
  for (uint32_t round = 0; round < 64; ++round) {
    bool mine = false;
    uint32_t x = 0, c = 0;
    if (!res_done[e] && res_done[tgt]) { x = res_exit[tgt]; c = k + res_cnt[tgt] - tidx; mine = true; }
    __syncthreads();
    if (mine) { res_exit[e] = x; res_cnt[e] = c; res_done[e] = 1u; }
    __syncthreads();
    if (__ballot(!res_done[e]) == 0) break;
  }
  const uint32_t x = res_exit[e];
  const uint32_t dx = res_done[e] ? min(x - G.end, XFAR) : XFAR;
  w.xtab[(size_t)i * XK + e] = (min(res_cnt[e], 0xFFFFu) << 16) | dx;
  __syncthreads();
  }
}

// ---- bitmap ranges [a, e) (e > a): count, OR into the final bitmap, and select
__device__ __forceinline__ uint64_t range_word(const uint64_t* __restrict__ bits, uint32_t wd, uint32_t a, uint32_t e) {
  uint64_t x = bits[wd];
  if (wd == (a >> 6)) x &= ~0ull << (a & 63);
  if (wd == ((e - 1) >> 6)) x &= ~0ull >> (63 - ((e - 1) & 63));
  return x;
}
__device__ __forceinline__ uint32_t popc_range(const uint64_t* __restrict__ bits, uint32_t a, uint32_t e) {
  uint32_t n = 0;
  if (a < e)
    for (uint32_t wd = a >> 6; wd <= (e - 1) >> 6; ++wd) n += (uint32_t)__popcll(range_word(bits, wd, a, e));
  return n;
}
__device__ __forceinline__ void or_range(uint64_t* __restrict__ fin, const uint64_t* __restrict__ bits, uint32_t a, uint32_t e) {
  if (a < e)
    for (uint32_t wd = a >> 6; wd <= (e - 1) >> 6; ++wd) {
      const uint64_t x = range_word(bits, wd, a, e);
      if (x) atomicOr((unsigned long long*)&fin[wd], (unsigned long long)x);
    }
}
// the n-th (n >= 1) set bit at or after a (the caller has counted at least n)
__device__ __forceinline__ uint32_t select_from(const uint64_t* __restrict__ bits, uint32_t a, uint32_t n) {
  uint32_t wd = a >> 6;
  uint64_t x = bits[wd] & (~0ull << (a & 63));
  for (;;) {
    const uint32_t c = (uint32_t)__popcll(x);
    if (c >= n) break;
    n -= c;
    x = bits[++wd];
  }
  for (uint32_t k = 1; k < n; ++k) x &= x - 1;
  return wd * 64 + (uint32_t)__ffsll((long long)x) - 1;
}
// One wavefront per large update follows its true struct sequence through the section headers.
// Per step lane j takes chunk cj + j (cj = the chunk of the current position p). Entries: lane 0
// enters at p; lane 0 composes the chunks' exit tables from p for as long as each entry offset is
// tabulated (lanes up to L get their true entries and exits), beyond that lane j enters at the
// exit of chunk j-1's chain 0 (speculative). Each lane parses exactly from its entry through its
// LDS window, recording the positions, until it meets its chunk's chain 0 (then the rest of the
// chunk's true structs are chain 0's positions: a popcount) or leaves the chunk. Lanes up to the
// first one whose true exit differs from the predicted one have true entries; the step takes
// their chunks, or stops in the chunk where the section ends.
__device__ __forceinline__ void or_words(uint64_t* __restrict__ fin, uint32_t w0, const uint64_t* __restrict__ m, uint32_t nw) {
  for (uint32_t k = 0; k < nw; ++k)
    if (m[k]) atomicOr((unsigned long long*)&fin[w0 + k], (unsigned long long)m[k]);
}
template <bool TABLES>
__global__ __launch_bounds__(64) void k_walk(Work w) {
  __shared__ __attribute__((aligned(16))) uint32_t win[64 * DSTRIDE];
  __shared__ uint64_t walked[64 * (SW + 1)];
  __shared__ uint64_t chain0[64 * (SW + 1)];
  __shared__ __attribute__((aligned(16))) uint32_t tab[TABLES ? 64 * XK : 4];
  __shared__ uint32_t ent[65], cnt[64], nknown;
  if (blockIdx.x >= w.nbig) return;
  const uint32_t u = w.ulist[blockIdx.x];
  if (w.ufail[u] == 2u || w.ufail[u] == 3u || w.ufail[u] >= UF_PRE) return;  // k_fastwalk / k_fastwalk_multi / k_predecoded / k_prewalk did it
  if (TABLES && w.ufail[u] != 1u && w.ufail[u] != 5u) return;
  // k_fastwalk_multi vouched for the first sections (ufail 4; 5 once handed to the tables): the
  // walk resumes at the next one
  const bool resume = TABLES ? w.ufail[u] == 5u : w.ufail[u] == 4u;
  const uint32_t lane = threadIdx.x;
  const uint32_t uw = upd_win(w, u);  // positions below are relative to the update's window
  const uint8_t* __restrict__ b = win_bytes(w, uw);
  const uint64_t* __restrict__ spec = win_words(w.spec_bits, uw);
  uint64_t* __restrict__ fbits = win_words(w.final_bits, uw);
  uint64_t* __restrict__ sbits = win_words(w.sec_bits, uw);
  const uint32_t ustart = w.uoff[u], uend = ustart + w.ulen[u];
  const uint32_t* __restrict__ stab = rtab_of(w, u);  // (step table; `tab` is the exit tables)
  const uint32_t CH = w.schunk;
  const uint32_t c0 = w.ugroup[u], nch = (w.ulen[u] + CH - 1) / CH;
  uint32_t* err = &w.ctr->err;
  const bool L0 = lane == 0;
  uint32_t* slot = win + lane * DSTRIDE;
  uint64_t* mw = walked + lane * (SW + 1);
  uint64_t* mc = chain0 + lane * (SW + 1);
  LdsSrc src{b, slot, 0, 0};
  auto refill = [&](uint32_t p) {
    src.s0 = p & ~15u;
    src.wlen = min(DW, (uend + 15u - src.s0) & ~15u);
    const uint4* g = (const uint4*)(b + src.s0);
    fill_window(slot, g);
  };
  if (L0) w.dsstart[u] = NONE;
  if (w.ulen[u] == 0) { if (L0) raise_err(err, ERR_DECODE); return; }
  uint32_t p = ustart;
  bool ok = true;
  const uint32_t nsec = rd_vu(b, p, uend, ok);
  if (!ok || nsec > (uend - p) / 3 + 1) { if (L0) raise_err(err, ERR_DECODE); return; }
  uint32_t sbase = 0;
  if (TABLES || resume) sbase = w.usec_start[u];  // (the sections were allocated by the first walk)
  else if (L0) sbase = atomicAdd(&w.ctr->nsections, nsec);
  sbase = __shfl(sbase, 0);
  if (sbase + nsec > w.cap_sections) { if (L0) raise_err(err, ERR_CAPACITY); return; }
  if (L0 && !TABLES && !resume) { w.usec_start[u] = sbase; w.usec_n[u] = nsec; }
  uint32_t sfirst = 0;
  if (resume) { sfirst = w.fw[2 * u]; p = w.fw[2 * u + 1]; }
  auto hand_over = [&]() {  // to the exit tables: flag the update, list its chunks (from the resume point's)
    const uint32_t j0 = resume ? (w.fw[2 * u + 1] - ustart) / CH : 0u;
    uint32_t base = 0;
    if (L0) { w.ufail[u] = resume ? 5u : 1u; base = atomicAdd(&w.ctr->xchunks, nch - j0); }
    base = __shfl(base, 0);
    for (uint32_t k = j0 + lane; k < nch; k += 64) w.xlist[base + k - j0] = c0 + k;
  };
  if (!TABLES && w.force_xtab) { hand_over(); return; }
  uint32_t steps = 0, fails = 0;
  for (uint32_t sct = sfirst; sct < nsec; ++sct) {
    const uint32_t n = rd_vu(b, p, uend, ok);
    const uint32_t client = rd_vu(b, p, uend, ok);
    const uint32_t clock = rd_vu(b, p, uend, ok);
    if (!ok || n > uend - p) { if (L0) raise_err(err, ERR_DECODE); return; }
    if (L0) {
      Section sec;
      sec.upd = u; sec.n = n; sec.client = client; sec.clock = clock;
      sec.first_pos = n ? p : NONE; sec.cidx = NONE; sec.first_idx = NONE; sec.pad = 0;
      w.sections[sbase + sct] = sec;
      if (n) atomicOr((unsigned long long*)&sbits[p >> 6], 1ull << (p & 63));
    }
    uint32_t r = n;
    while (r > 0) {
      if (p >= uend) { if (L0) { raise_err(err, ERR_DECODE); w.ctr->err_info = p; } return; }
      const uint32_t j0 = (p - ustart) / CH, j = j0 + lane;
      const bool valid = j < nch;
      const uint32_t cs = ustart + j * CH;
      const uint32_t ce = valid ? min(cs + CH, uend) : 0u;
      if (valid) {
        if (TABLES) {
          const uint4* xt = (const uint4*)(w.xtab + (size_t)(c0 + j) * XK);
          for (uint32_t k = 0; k < XK / 4; ++k) ((uint4*)(tab + lane * XK))[k] = xt[k];
        }
        const uint32_t nwc = (ce - cs + 63) >> 6;  // the chunk's words of spec_bits (no further)
        for (uint32_t k = 0; k <= SW; ++k) { mc[k] = k < nwc ? spec[(cs >> 6) + k] : 0ull; mw[k] = 0; }
      }
      if (!TABLES && L0) nknown = 0;
      __syncthreads();
      if (TABLES && L0) {  // compose the exit tables from p
        uint32_t E = p, L = 0;
        for (uint32_t l = 0; l < 64 && j0 + l < nch; ++l) {
          const uint32_t s_l = ustart + (j0 + l) * CH, e_l = min(s_l + CH, uend);
          const uint32_t off = E - s_l;
          if (E >= e_l) {  // a long struct jumps over the whole chunk: no structs in it
            ent[l + 1] = E;
            cnt[l] = 0;
            L = l + 1;
            continue;
          }
          if (off >= XK) break;
          const uint32_t v = tab[l * XK + off];
          if ((v & 0xFFFFu) == XFAR) break;
          E = e_l + (v & 0xFFFFu);
          ent[l + 1] = E;
          cnt[l] = v >> 16;
          L = l + 1;
        }
        nknown = L;
      }
      __syncthreads();
      const uint32_t L = nknown;
      const uint32_t CX = valid ? w.cexit[c0 + j] : NONE;   // chain 0's exit
      const uint32_t S = valid && lane < L ? ent[lane + 1] : CX;  // predicted exit
      uint32_t E = __shfl_up(S, 1);
      if (L0) E = p;
      // lanes below L hold a tabulated chunk: their count is known and their positions are
      // marked later (k_xmark from the entry); the others parse exactly from their entry
      const bool tabbed = TABLES && valid && lane < L;
      auto walk = [&](uint32_t q0, uint32_t limit, uint32_t& kk) {  // exact, until chain 0 / limit
        uint32_t q = q0;
        if (q < ce) refill(q);
        while (q < ce && kk < limit && !((mc[(q - cs) >> 6] >> (q & 63)) & 1ull)) {
          mw[(q - cs) >> 6] |= 1ull << (q & 63);
          if (src.wlen == DW && q - src.s0 + DREFILL > DW) refill(q);
          const uint32_t d = tab_len(stab, ustart, src, b, q, uend);
          q += d ? d : 1u;
          ++kk;
        }
        return q;
      };
      uint32_t q = E, k = 0;
      bool merged = false;
      if (valid && E >= cs && !tabbed) {
        q = walk(E, NONE, k);
        merged = q < ce;
      }
      const uint32_t C = tabbed ? cnt[lane] : k + (merged ? popc_range(spec, q, ce) : 0u);
      const uint32_t X = tabbed ? S : merged ? CX : q;  // the true exit, given the entry
      const uint64_t bad = __ballot(!(valid && E >= cs && X == S));
      const uint32_t f = bad ? (uint32_t)__ffsll((long long)bad) - 1 : 63u;  // lanes 0..f hold true entries
      uint32_t incl = lane <= f ? C : 0u;
      for (uint32_t off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_up(incl, off);
        if (lane >= off) incl += v;
      }
      const uint32_t excl = incl - (lane <= f ? C : 0u);
      const uint64_t ends = __ballot(lane <= f && valid && incl >= r);
      const uint32_t nw = valid ? (ce - cs + 63) >> 6 : 0u;
      // chains locked into a wrong phase fail (nearly) every speculation: hand the update to the
      // exit tables (k_xtab + k_walk<true>); the marks made so far are true and are made again.
      // A failure where the true exit jumps past the next chunk (a long struct) is no sign of it.
      ++steps;
      const uint32_t Xf = __shfl(X, f), cef = __shfl(ce, f);
      if (!TABLES && !ends && f < 63 && j0 + f + 1 < nch && Xf < cef + CH && ++fails >= 4 && fails * 4 > steps * 3) {
        hand_over();
        return;
      }
      auto mark_all = [&]() {
        if (tabbed) w.tentry[c0 + j] = E;
        else {
          or_words(fbits, cs >> 6, mw, nw);
          if (merged) or_range(fbits, spec, q, ce);
        }
      };
      if (ends) {  // the section ends in lane jl's chunk
        const uint32_t jl = (uint32_t)__ffsll((long long)ends) - 1;
        uint32_t np = 0;
        if (lane < jl) {
          mark_all();
        } else if (lane == jl) {
          const uint32_t rr = r - excl;
          if (tabbed) {  // parse the rr structs exactly (all inside the chunk: the count says so)
            uint32_t kk = 0;
            for (uint32_t x = 0; x <= SW; ++x) mc[x] = 0;
            walk(E, rr, kk);
          }
          uint32_t Lp;
          if (tabbed || rr <= k) {  // the rr-th walked position is the section's last struct
            Lp = select_from(mw, 0, rr) + cs;  // mw is indexed from the chunk start
            const uint32_t lw = (Lp - cs) >> 6;
            for (uint32_t x = 0; x < nw; ++x) {
              const uint64_t v = x < lw ? mw[x] : x == lw ? mw[x] & (~0ull >> (63 - (Lp & 63))) : 0ull;
              if (v) atomicOr((unsigned long long*)&fbits[(cs >> 6) + x], (unsigned long long)v);
            }
          } else {
            or_words(fbits, cs >> 6, mw, nw);
            Lp = select_from(spec, q, rr - k);
            or_range(fbits, spec, q, Lp + 1);
          }
          np = tab_step(stab, ustart, b, Lp, uend);
        }
        p = __shfl(np, jl);
        r = 0;
      } else {
        if (lane <= f) mark_all();
        r -= __shfl(incl, f);
        p = __shfl(X, f);  // NONE / past the update when the section runs past its end
      }
      __syncthreads();
    }
  }
  if (L0) w.dsstart[u] = p;
}

// Fast path of the walk for single-section updates (a snapshot, one replica's own ops): when the
// synced chunk chains form one chain — every chunk's final chain was entered where its
// predecessor's final chain leaves (sexit == cexit after the last k_sync round) — and the exact
// walk from the first struct meets chunk 0's chain inside chunk 0, the chain IS the true struct
// sequence, so the update needs no serial walk: the n-th struct is found by a popcount scan over
// the chunks (64 per wavefront round) and the struct-start words are copied in parallel. Anything
// else (several sections, a chain that never meets, fewer chain positions than structs) is left
// to k_walk, which also reports malformed input.
// The chain positions of the chunks, scanned (cpre, 64-bit), and the chunks whose entry may be off
// the one chain, scanned (opre): k_chunk_counts + two scans. A fast walk's search for the chunk
// holding a section's last struct is then a 64-way search over the scan (two or three rounds of one
// load per lane), not a walk over every chunk's count (C4's 15 MB replica updates: 235 rounds).
// The smallest j in [j0, nch) with cpre[c0 + j + 1] - cpre[c0 + j0] >= need; nch when none.
__device__ __forceinline__ uint32_t chunk_search(const Work& w, uint32_t c0, uint32_t j0, uint32_t nch, uint64_t need, uint32_t lane) {
  const uint64_t base = w.cpre[c0 + j0];
  uint32_t lo = j0, hi = nch;  // the answer is in [lo, hi]; hi == nch: none, else known to hold
  while (lo < hi) {
    const uint32_t step = (hi - lo + 63) / 64;
    const uint32_t pv = lo + lane * step;
    const uint64_t m = __ballot(pv < hi && w.cpre[c0 + pv + 1] - base >= need);
    if (!m) {
      lo += min(63u, (hi - 1 - lo) / step) * step + 1;  // past the last pivot
    } else {
      const uint32_t L = (uint32_t)__ffsll((long long)m) - 1;
      if (L == 0) { hi = lo; break; }
      hi = lo + L * step;
      lo += (L - 1) * step + 1;
    }
  }
  return lo;
}
// The chunk fch holding the target-th (>= 1) chain position counted from q (in chunk jq) and the
// rank rem (>= 1) of that position inside it (counted from q when fch == jq). No chunk after jq up
// to fch may be off the one chain. false: fewer positions (why = 0) or an off chunk (why = 1).
__device__ __forceinline__ bool chain_target(const Work& w, const uint64_t* __restrict__ spec, uint32_t ustart, uint32_t uend, uint32_t c0,
                                             uint32_t nch, uint32_t jq, uint32_t q, uint32_t target, uint32_t lane, uint32_t& fch,
                                             uint32_t& rem, uint32_t& why) {
  const uint32_t cq = popc_range(spec, q, min(ustart + (jq + 1) * w.schunk, uend));
  if (target <= cq) { fch = jq; rem = target; return true; }
  const uint64_t need = target - cq;
  const uint32_t j = jq + 1 < nch ? chunk_search(w, c0, jq + 1, nch, need, lane) : nch;
  if (j >= nch) { why = 0; return false; }
  if (w.opre[c0 + j + 1] != w.opre[c0 + jq + 1]) { why = 1; return false; }
  fch = j;
  rem = (uint32_t)(need - (w.cpre[c0 + j] - w.cpre[c0 + jq + 1]));
  return true;
}
__global__ __launch_bounds__(64) void k_fastwalk(Work w) {
  __shared__ uint64_t walked[SW + 2];
  __shared__ uint32_t sh_q, sh_k0, sh_ok;
  if (blockIdx.x >= w.nbig) return;
  const uint32_t u = w.ulist[blockIdx.x];
  const uint32_t lane = threadIdx.x;
  const uint32_t uw = upd_win(w, u);
  const uint8_t* __restrict__ b = win_bytes(w, uw);
  const uint64_t* __restrict__ spec = win_words(w.spec_bits, uw);
  uint64_t* __restrict__ fbits = win_words(w.final_bits, uw);
  uint64_t* __restrict__ sbits = win_words(w.sec_bits, uw);
  const uint32_t ustart = w.uoff[u], uend = ustart + w.ulen[u];
  const uint32_t CH = w.schunk;
  const uint32_t c0 = w.ugroup[u], nch = (w.ulen[u] + CH - 1) / CH;
  if (!w.ulen[u] || w.ufail[u] >= UF_PRE) return;
  uint32_t p = ustart;
  bool ok = true;
  const uint32_t nsec = rd_vu(b, p, uend, ok);
  auto why = [&](uint32_t k) { if (w.dbg && lane == 0) atomicAdd(&w.dbg[k], 1ull); };
  if (!ok || nsec != 1) { why(1); return; }
  const uint32_t n = rd_vu(b, p, uend, ok);
  const uint32_t client = rd_vu(b, p, uend, ok);
  const uint32_t clock = rd_vu(b, p, uend, ok);
  if (!ok || n == 0 || n > uend - p) return;
  const uint32_t p1 = p, ce0 = min(ustart + CH, uend);
  if (p1 >= ce0) return;
  // one chain through every chunk up to the one holding the last struct (k_chunk_counts flags the
  // chunks whose entry may be off it — C4's replica updates each have one, past their structs)
  // chunk 0: the exact walk from the first struct until it meets chunk 0's chain
  for (uint32_t k = lane; k < SW + 2; k += 64) walked[k] = 0;
  __syncthreads();
  if (lane == 0) {
    uint32_t q = p1, k0 = 0;
    const uint32_t w0 = ustart >> 6;
    while (q < ce0 && !((spec[q >> 6] >> (q & 63)) & 1ull)) {
      walked[(q >> 6) - w0] |= 1ull << (q & 63);
      q = chain_step(b, q, uend);
      ++k0;
    }
    sh_q = q;
    sh_k0 = k0;
    sh_ok = q < ce0 && k0 < n;
  }
  __syncthreads();
  if (!sh_ok) { why(3); return; }
  const uint32_t q = sh_q, target = n - sh_k0;  // the target-th chain position from q is the last struct
  uint32_t fch = 0, rem = 0, wy = 0;
  if (!chain_target(w, spec, ustart, uend, c0, nch, 0, q, target, lane, fch, rem, wy)) { why(wy ? 2 : 4); return; }
  const uint32_t fcs = ustart + fch * CH, fa = fch == 0 ? q : fcs;
  const uint32_t Lp = select_from(spec, fa, rem);
  const uint32_t dsp = chain_step(b, Lp, uend);
  if (Lp >= uend || dsp > uend) { why(5); return; }
  // marks: the walked positions of chunk 0, then every chain position in [q, Lp] — here the words
  // that can hold walked positions, the rest grid-wide (k_fastmark: one wavefront copying a 15 MB
  // update's words took 4 ms of C4's decode)
  const uint32_t wq = q >> 6, wl = min(Lp >> 6, (ustart >> 6) + SW + 1), w0 = ustart >> 6;
  for (uint32_t wd = w0 + lane; wd <= wl; wd += 64) {
    uint64_t x = wd >= wq ? range_word(spec, wd, q, Lp + 1) : 0ull;
    if (wd - w0 < SW + 2) x |= walked[wd - w0];
    fbits[wd] = x;  // the update's own words (updates and chunks are 64-byte aligned)
  }
  if (lane == 0) {
    const uint32_t sbase = atomicAdd(&w.ctr->nsections, 1u);
    if (sbase >= w.cap_sections) { raise_err(&w.ctr->err, ERR_CAPACITY); return; }
    Section sec;
    sec.upd = u; sec.n = n; sec.client = client; sec.clock = clock;
    sec.first_pos = p1; sec.cidx = NONE; sec.first_idx = NONE; sec.pad = 0;
    w.sections[sbase] = sec;
    atomicOr((unsigned long long*)&sbits[p1 >> 6], 1ull << (p1 & 63));
    w.usec_start[u] = sbase;
    w.usec_n[u] = 1;
    w.dsstart[u] = dsp;
    w.fw[2 * u] = q;
    w.fw[2 * u + 1] = Lp + 1;
    w.ufail[u] = 2u;  // done: k_walk leaves the update alone
    if (w.dbg) atomicAdd(&w.dbg[0], 1ull);
  }
}

// Chain positions per chunk of the large updates (one lane per chunk, after the sync rounds): the
// fast walk's search for the n-th position reads one count per chunk instead of popcounting the
// chunk's words from one wavefront (C4: 15 K chunks per update, 16 words each)
// The fast walk for updates of several sections (a snapshot of many clients): the synced chunk
// chains form one chain through the whole update (section headers included, parsed as garbage),
// so for each section in turn: the exact walk from its first struct until it meets the chain
// (inside that struct's chunk), then the section's last struct is the (n - walked)-th chain
// position from the meeting point, and the next header starts where that struct ends. Pass 1
// checks the sections in order without writing anything; pass 2 writes the records of the sections
// it vouched for, their walked positions and chain ranges (k_fastmark copies the ranges grid-wide;
// the header gaps stay clear). A section it cannot vouch for (a chain that never meets, an off
// chunk, more than FWM_MAX sections) ends pass 1: the sections before it are committed and k_walk
// resumes at its header (ufail 4) — one phase-locked section no longer sends a snapshot of a
// thousand clients (a C2 document's state, crdt.js's wire shape) back through the serial walk.
// The sections are a serial chain (a header's position is the end of the section before it), so
// each step is cut to a few rounds of wavefront-wide loads: the bytes from the section's header
// (and the previous section's last struct) and their struct-start words staged in LDS, the exact
// walk from LDS, the meeting chunk's words and the next 64 chunks' count / off prefixes in one
// round, the last struct's chunk words in one more (64-way searches past 64 chunks).
// (C4's base snapshot: 65 sections, 11 MB; C3's merged output: 256 sections, 156 MB.)
constexpr uint32_t FWM_MAX = 1024;    // sections checked per update (LDS records); k_walk resumes past them
constexpr uint32_t FWM_WALK = 256;    // exact steps from a section's first struct to the chain, at most
constexpr uint32_t FWM_STAGE = 512;   // bytes staged per step
template <class S>
__device__ __forceinline__ uint32_t rd_vu_src(const S& b, uint32_t& p, uint32_t end, bool& ok) {  // rd_vu over a source
  uint32_t v = 0, shift = 0;
#pragma unroll 1
  for (;;) {
    if (p >= end) { ok = false; return 0; }
    const uint32_t r = b.u8(p++);
    if (shift < 32) v |= (r & 0x7fu) << shift;
    shift += 7;
    if (r < 0x80u) return v;
    if (shift > 35) { ok = false; return 0; }
  }
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  for (uint32_t off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
__device__ __forceinline__ uint32_t nth_set1(uint64_t x, uint32_t k) {  // position of the k-th (>= 1) set bit
  for (uint32_t i = 1; i < k; ++i) x &= x - 1;
  return (uint32_t)__ffsll((long long)x) - 1;
}
// ---- Record mode of the multi-section fast walk (a full state as ONE update: crdt.js's wire shape,
// crdt.js:288,443; a thousand client sections). A section's step — header, exact walk from its
// first struct to the chain, count search, the last struct's end = the next header — depends only
// on the header's position, and every header after the first lies on the synced chain (the chain
// runs through the previous section's last struct and on into the header bytes). So the step is
// evaluated for EVERY chain position of the update at once (k_fwc: one lane per chain position,
// whole chip), and the serial part shrinks to following the records from header to header: one
// memory round trip per section instead of ~20 dependent parse steps (C2 document state, 1 001
// sections: the walk took ~22 ms). A header off the chain (the update's first; the end of a
// section walked whole) or a record that gave up early is evaluated by the walker itself with the
// same function. The records never vouch for anything the exact walk would not: fwc_eval IS the
// section step (the walk, the off-chunk test, the count search and the select of the old pass).
struct FwcRes { uint32_t next, e, k0, why; };  // next header (NONE: not vouched), chain range end, walked structs, reason
__device__ __forceinline__ bool spec_at(const uint64_t* __restrict__ spec, uint32_t q) { return (spec[q >> 6] >> (q & 63)) & 1ull; }
__device__ __forceinline__ FwcRes fwc_eval(const Work& w, const uint8_t* __restrict__ b, const uint64_t* __restrict__ spec, uint32_t ustart,
                                           uint32_t uend, uint32_t c0, uint32_t nch, uint32_t hdr, uint32_t walk_max,
                                           const uint32_t* __restrict__ tab) {
  FwcRes r{NONE, NONE, 0u, 0u};
  uint32_t p = hdr;
  bool ok = hdr < uend;
  const uint32_t n = rd_vu(b, p, uend, ok);
  rd_vu(b, p, uend, ok);  // client
  rd_vu(b, p, uend, ok);  // clock
  if (!ok || n > uend - p) { r.why = 3; return r; }
  const uint32_t p1 = p;
  if (n == 0) { r.next = p1; r.e = p1; return r; }
  if (p1 >= uend) { r.why = 3; return r; }
  // the exact walk until it meets the chain (or walks the whole section)
  uint32_t q = p1, k0 = 0;
  for (uint32_t steps = 0; q < uend && k0 < n && !spec_at(spec, q); ++steps) {
    if (steps == walk_max) { r.why = walk_max < FWM_WALK ? 8u : 5u; return r; }
    const uint32_t dq = tab_len(tab, ustart, GlobalSrc{b}, b, q, uend);
    if (!dq) { r.why = 4; return r; }  // no struct parses: k_walk reports it
    q += dq;
    ++k0;
  }
  r.k0 = k0;
  if (k0 == n) {  // every struct walked: the next header is where the walk stopped
    if (q > uend) { r.why = 3; return r; }
    r.next = q;
    r.e = q;
    return r;
  }
  if (q >= uend) { r.why = 5; return r; }
  // the target-th chain position from q (q the first) is the section's last struct
  const uint32_t target = n - k0, CH = w.schunk;
  const uint32_t jq = (q - ustart) / CH, ceq = min(ustart + jq * CH + CH, uend);
  const uint32_t cq = popc_range(spec, q, ceq);
  uint32_t fa = q, rem = target;
  if (target > cq) {
    const uint64_t need = target - cq, base = w.cpre[c0 + jq + 1];
    uint32_t lo = jq + 1, hi = nch;  // the first chunk j with cpre[c0 + j + 1] - base >= need
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (w.cpre[c0 + m + 1] - base >= need) hi = m; else lo = m + 1; }
    if (lo >= nch) { r.why = 6; return r; }
    if (w.opre[c0 + lo + 1] != w.opre[c0 + jq + 1]) { r.why = 2; return r; }  // an off chunk between
    rem = (uint32_t)(need - (w.cpre[c0 + lo] - base));
    fa = ustart + lo * CH;
  }
  const uint32_t Lp = select_from(spec, fa, rem);
  const uint32_t dl = Lp < uend ? tab_len(tab, ustart, GlobalSrc{b}, b, Lp, uend) : 0u;
  if (!dl || Lp + dl > uend) { r.why = 7; return r; }  // the last struct's end is unknown
  r.next = Lp + dl;
  r.e = Lp + 1;
  return r;
}
// every chain position of the record-mode updates: its section step as if a header started there
// (one lane per bitmap word of their chunks, grid-stride)
__global__ __launch_bounds__(256) void k_fwc(Work w) {
  const uint32_t wpc = w.schunk / 64;
  const uint64_t total = (uint64_t)w.ngroups * wpc;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    const Group G = w.groups[t / wpc];
    const uint32_t u = G.upd, off = w.fwc_off[u];
    if (off == NONE) continue;
    const uint32_t wd = (G.start >> 6) + (uint32_t)(t % wpc);
    if ((uint64_t)wd * 64 >= G.end) continue;
    const uint32_t uw = upd_win(w, u);
    const uint8_t* __restrict__ b = win_bytes(w, uw);
    const uint64_t* __restrict__ spec = win_words(w.spec_bits, uw);
    const uint32_t ustart = w.uoff[u], uend = ustart + w.ulen[u], c0 = w.ugroup[u], nch = (w.ulen[u] + w.schunk - 1) / w.schunk;
    for (uint64_t x = range_word(spec, wd, G.start, G.end); x; x &= x - 1) {
      const uint32_t c = wd * 64 + (uint32_t)__ffsll((long long)x) - 1;
      const FwcRes r = fwc_eval(w, b, spec, ustart, uend, c0, nch, c, w.fwc_walk, rtab_of(w, u));
      w.fwc[off + (c - ustart)] = make_uint4(r.next, r.e, r.k0, r.why);
    }
  }
}
// ---- The last section of a record-mode update, ranked. A section the records cannot vouch for is
// one whose chunk chains never settle into the true phase (a long snapshot of similar structs: C2's
// 100 k-struct base section, the LAST of a document state's sections); k_walk then resumed at its
// header and composed exit tables, 64 chunks a step (1.5 ms on the C2 state). With the step table
// the section's structs are the first n positions of the chain from its first struct, found by
// pointer doubling over the section's bytes (k_wrank's method on the whole chip): in round k every
// position at distance d < 2^k from the first struct marks the one 2^k steps on (d + 2^k <= n), and
// the jump table advances from 2^k to 2^(k+1) steps (two buffers). Positions at distance < n are the
// structs, the one at distance n starts the delete set. The jump tables and distances live in the
// update's records (free once the walker has followed them). Only the update's last section, and only
// n < 2^RK_ROUNDS; anything else — or a chain that ends short — stays with k_walk.
constexpr uint32_t RK_ROUNDS = 24;
__device__ __forceinline__ uint32_t* rk_base(const Work& w, uint32_t u) { return (uint32_t*)(w.fwc + w.fwc_off[u]); }
// one lane per large update: the ranked section of a record-mode update, if any (rk[u]: first struct,
// n, section index, 1 = ranked)
__global__ void k_rk_setup(Work w) {
  const uint32_t bi = blockIdx.x * blockDim.x + threadIdx.x;
  if (bi >= w.nbig) return;
  const uint32_t u = w.ulist[bi];
  w.rk[u] = make_uint4(0u, 0u, 0u, 0u);
  if (w.fwc_off[u] == NONE || !w.rtab || w.ufail[u] != 4u) return;  // (YCRDT_FWM_MAX = sections - 1: tests take this path)
  const uint32_t done = w.fw[2 * u];
  if (done + 1 != w.usec_n[u]) return;  // (not the last section)
  const uint8_t* __restrict__ b = win_bytes(w, upd_win(w, u));
  const uint32_t uend = w.uoff[u] + w.ulen[u];
  uint32_t p = w.fw[2 * u + 1];
  bool ok = true;
  const uint32_t n = rd_vu(b, p, uend, ok);
  rd_vu(b, p, uend, ok);
  rd_vu(b, p, uend, ok);
  if (!ok || n == 0 || n >= (1u << RK_ROUNDS) || p >= uend) return;
  w.rk[u] = make_uint4(p, n, w.usec_start[u] + done, 1u);
  w.dsstart[u] = NONE;  // (set by the marks only if the chain reaches distance n)
}
// the positions of the record-mode updates (grid-stride over their chunks): (update, position) or false
__device__ __forceinline__ bool rk_pos(const Work& w, uint64_t t, uint32_t& u, uint32_t& p) {
  const Group G = w.groups[t / w.schunk];
  u = G.upd;
  p = G.start + (uint32_t)(t % w.schunk);
  return p < G.end && w.fwc_off[u] != NONE;
}
__global__ __launch_bounds__(256) void k_rk_init(Work w) {
  const uint64_t total = (uint64_t)w.ngroups * w.schunk;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t u, p;
    if (!rk_pos(w, t, u, p)) continue;
    const uint4 d = w.rk[u];
    if (!d.w) continue;
    const uint32_t ustart = w.uoff[u], L = w.ulen[u], uend = ustart + L, i = p - ustart;
    uint32_t* __restrict__ A = rk_base(w, u);
    const uint32_t st = p >= d.x ? rtab_of(w, u)[i] : 0u;
    A[i] = st && p + st < uend ? p + st : (st && p + st == uend ? uend : NONE);  // J_1 (the update end: a sink that counts)
    A[2 * L + i] = p == d.x ? 0u : NONE;                                         // distance from the first struct
  }
}
__global__ __launch_bounds__(256) void k_rk_round(Work w, uint32_t k) {
  const uint64_t total = (uint64_t)w.ngroups * w.schunk;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t u, p;
    if (!rk_pos(w, t, u, p)) continue;
    const uint4 d = w.rk[u];
    if (!d.w || (1u << k) > d.y || p < d.x) continue;  // (no round needed past n)
    const uint32_t ustart = w.uoff[u], L = w.ulen[u], uend = ustart + L, i = p - ustart;
    uint32_t* __restrict__ A = rk_base(w, u);
    const uint32_t* __restrict__ J = A + (k & 1u) * L;
    uint32_t* __restrict__ J2 = A + ((k + 1) & 1u) * L;
    uint32_t* __restrict__ dist = A + 2 * L;
    const uint32_t j = J[i], di = dist[i];
    if (di != NONE && di < (1u << k) && j != NONE && di + (1u << k) <= d.y) {
      if (j < uend) dist[j - ustart] = di + (1u << k);
      else if (j == uend && di + (1u << k) == d.y) w.dsstart[u] = uend;  // (the section ends the update: no delete set)
    }
    J2[i] = j == NONE || j >= uend ? (j == uend ? uend : NONE) : J[j - ustart];
  }
}
// the marks: structs at distance < n, the delete set at n (one lane per bitmap word); the section
// record, its first-struct mark and an empty chain range (k_fastmark), ufail 3
__global__ __launch_bounds__(256) void k_rk_final(Work w) {
  const uint32_t wpc = w.schunk / 64;
  const uint64_t total = (uint64_t)w.ngroups * wpc;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    const Group G = w.groups[t / wpc];
    const uint32_t u = G.upd;
    if (w.fwc_off[u] == NONE) continue;
    const uint4 d = w.rk[u];
    if (!d.w) continue;
    const uint32_t wd = (G.start >> 6) + (uint32_t)(t % wpc);
    if ((uint64_t)wd * 64 >= G.end) continue;
    const uint32_t ustart = w.uoff[u], L = w.ulen[u];
    const uint32_t* __restrict__ dist = rk_base(w, u) + 2 * L;
    uint64_t m = 0;
    for (uint32_t bb = 0; bb < 64; ++bb) {
      const uint32_t p = wd * 64 + bb;
      if (p < max(G.start, d.x) || p >= G.end) continue;
      const uint32_t di = dist[p - ustart];
      if (di < d.y) m |= 1ull << bb;
      else if (di == d.y) w.dsstart[u] = p;
    }
    uint64_t* __restrict__ fbits = win_words(w.final_bits, upd_win(w, u));
    if (m) atomicOr((unsigned long long*)&fbits[wd], (unsigned long long)m);
  }
}
// the section's record once the marks are in (one lane per large update); a chain that ends short
// (no position at distance n) leaves the section to k_walk, which reports it
__global__ void k_rk_commit(Work w) {
  const uint32_t bi = blockIdx.x * blockDim.x + threadIdx.x;
  if (bi >= w.nbig) return;
  const uint32_t u = w.ulist[bi];
  const uint4 d = w.rk[u];
  if (!d.w || w.dsstart[u] == NONE) return;
  const uint8_t* __restrict__ b = win_bytes(w, upd_win(w, u));
  const uint32_t uend = w.uoff[u] + w.ulen[u];
  uint32_t p = w.fw[2 * u + 1];
  bool ok = true;
  const uint32_t n = rd_vu(b, p, uend, ok), client = rd_vu(b, p, uend, ok), clock = rd_vu(b, p, uend, ok);
  Section sec;
  sec.upd = u; sec.n = n; sec.client = client; sec.clock = clock;
  sec.first_pos = d.x; sec.cidx = NONE; sec.first_idx = NONE; sec.pad = 0;
  w.sections[d.z] = sec;
  uint64_t* __restrict__ sbits = win_words(w.sec_bits, upd_win(w, u));
  atomicOr((unsigned long long*)&sbits[d.x >> 6], 1ull << (d.x & 63));
  w.fwsec[2 * d.z] = d.x;  // (an empty chain range: the marks are in)
  w.fwsec[2 * d.z + 1] = d.x;
  w.ufail[u] = 3u;
  if (w.dbg) atomicAdd(&w.dbg[0], 1ull);
}

// the walker's record-mode pass: lane 0 follows the records from header to header; every section
// it vouches for gets (header, chain range end) in fwsec, k_fwc_commit writes the rest
__device__ __forceinline__ void fwm_records(const Work& w, uint32_t u, uint32_t nsec, uint32_t hdr0) {
  const uint32_t uw = upd_win(w, u);
  const uint8_t* __restrict__ b = win_bytes(w, uw);
  const uint64_t* __restrict__ spec = win_words(w.spec_bits, uw);
  const uint32_t ustart = w.uoff[u], uend = ustart + w.ulen[u], c0 = w.ugroup[u], nch = (w.ulen[u] + w.schunk - 1) / w.schunk;
  const uint32_t off = w.fwc_off[u];
  const uint32_t sbase = atomicAdd(&w.ctr->nsections, nsec);
  if (sbase + nsec > w.cap_sections) { raise_err(&w.ctr->err, ERR_CAPACITY); return; }
  uint32_t h = hdr0, done = 0;
  const uint32_t lim = w.fwm_max ? min(nsec, w.fwm_max) : nsec;  // (YCRDT_FWM_MAX: tests cap the vouched prefix)
  for (; done < lim; ++done) {
    FwcRes r{NONE, NONE, 0u, 8u};
    if (h > ustart && h < uend && spec_at(spec, h)) {  // a chain position: k_fwc evaluated it
      const uint4 x = w.fwc[off + (h - ustart)];
      r = FwcRes{x.x, x.y, x.z, x.w};
    }
    if (r.next == NONE && r.why == 8u) {  // off the chain, or walked past k_fwc's bound
      r = fwc_eval(w, b, spec, ustart, uend, c0, nch, h, FWM_WALK, rtab_of(w, u));
      if (w.dbg) atomicAdd(&w.dbg[16], 1ull);
    }
    if (r.next == NONE) {
      if (w.dbg) {
        atomicAdd(&w.dbg[1], 1ull);
        atomicAdd(&w.dbg[8 + min(r.why, 7u)], 1ull);
        w.dbg[14] = done; w.dbg[15] = nsec; w.dbg[17] = h - ustart; w.dbg[18] = uend - ustart;
      }
      break;
    }
    w.fwsec[2 * (sbase + done)] = h;
    w.fwsec[2 * (sbase + done) + 1] = r.e;
    h = r.next;
  }
  w.usec_start[u] = sbase;
  w.usec_n[u] = nsec;
  if (done == nsec) {
    w.dsstart[u] = h;  // (past the last section: the delete set)
    w.ufail[u] = 3u;   // done: k_walk leaves it alone, k_fwc_commit + k_fastmark write it
    if (w.dbg) { atomicAdd(&w.dbg[0], 1ull); atomicAdd(&w.dbg[23], (unsigned long long)done); }
  } else {
    w.fw[2 * u] = done;  // k_walk resumes at section `done`, whose header is at h (section 0: the whole update)
    w.fw[2 * u + 1] = h;
    w.ufail[u] = 4u;
  }
}
// the vouched sections of the record-mode updates, one lane per section (grid-stride): the section
// record, its first-struct mark, the walked positions before the chain, the chain range for k_fastmark
__global__ __launch_bounds__(256) void k_fwc_commit(Work w) {
  const uint32_t gt = blockIdx.x * blockDim.x + threadIdx.x, gs = gridDim.x * blockDim.x;
  for (uint32_t bi = 0; bi < w.nbig; ++bi) {
    const uint32_t u = w.ulist[bi];
    if (w.fwc_off[u] == NONE) continue;
    const uint32_t uf = w.ufail[u];
    if (uf != 3u && uf != 4u) continue;
    const uint32_t sbase = w.usec_start[u], ndone = uf == 3u ? w.usec_n[u] : w.fw[2 * u];
    const uint32_t uw = upd_win(w, u);
    const uint8_t* __restrict__ b = win_bytes(w, uw);
    const uint64_t* __restrict__ spec = win_words(w.spec_bits, uw);
    uint64_t* __restrict__ fbits = win_words(w.final_bits, uw);
    uint64_t* __restrict__ sbits = win_words(w.sec_bits, uw);
    const uint32_t uend = w.uoff[u] + w.ulen[u];
    for (uint32_t s = gt; s < ndone; s += gs) {
      uint32_t p = w.fwsec[2 * (sbase + s)];
      bool ok = true;
      const uint32_t n = rd_vu(b, p, uend, ok), client = rd_vu(b, p, uend, ok), clock = rd_vu(b, p, uend, ok);
      const uint32_t p1 = p;
      Section sec;
      sec.upd = u; sec.n = n; sec.client = client; sec.clock = clock;
      sec.first_pos = n ? p1 : NONE; sec.cidx = NONE; sec.first_idx = NONE; sec.pad = 0;
      w.sections[sbase + s] = sec;
      if (n) atomicOr((unsigned long long*)&sbits[p1 >> 6], 1ull << (p1 & 63));
      // the walked positions (not on the chain): the record's walk again, to where it met the chain
      uint32_t x = p1, k0 = 0;
      while (n && k0 < n && x < uend && !spec_at(spec, x)) {
        atomicOr((unsigned long long*)&fbits[x >> 6], 1ull << (x & 63));
        x = tab_step(rtab_of(w, u), w.uoff[u], b, x, uend);
        ++k0;
      }
      w.fwsec[2 * (sbase + s)] = n ? x : p1;  // the chain range [q, e) (k_fastmark)
    }
  }
}
__global__ __launch_bounds__(64) void k_fastwalk_multi(Work w) {
  __shared__ uint32_t sp1[FWM_MAX], sn[FWM_MAX], scl[FWM_MAX], sck[FWM_MAX], sq[FWM_MAX], se[FWM_MAX], sk0[FWM_MAX], shp[FWM_MAX];
  __shared__ __attribute__((aligned(16))) uint32_t stg[FWM_STAGE / 4 + 4];
  __shared__ uint64_t sspec[FWM_STAGE / 64 + 2];
  __shared__ uint32_t sh_sbase;
  if (blockIdx.x >= w.nbig) return;
  const uint32_t u = w.ulist[blockIdx.x];
  const uint32_t lane = threadIdx.x;
  // (YCRDT_DEBUG_DECODE: updates (partly) left to k_walk, and why — dbg[8 + r]: reason r)
  auto why = [&](uint32_t r) { if (w.dbg && lane == 0) { atomicAdd(&w.dbg[1], 1ull); atomicAdd(&w.dbg[8 + r], 1ull); } };
  if (w.ufail[u] || !w.fwsec) return;
  const uint32_t uw = upd_win(w, u);
  const uint8_t* __restrict__ b = win_bytes(w, uw);
  const uint64_t* __restrict__ spec = win_words(w.spec_bits, uw);
  uint64_t* __restrict__ fbits = win_words(w.final_bits, uw);
  uint64_t* __restrict__ sbits = win_words(w.sec_bits, uw);
  const uint32_t ustart = w.uoff[u], uend = ustart + w.ulen[u];
  const uint32_t CH = w.schunk, SWC = CH / 64;
  const uint32_t c0 = w.ugroup[u], nch = (w.ulen[u] + CH - 1) / CH;
  if (!w.ulen[u] || SWC > 64) return;
  uint32_t p = ustart;
  bool ok = true;
  const uint32_t nsec = rd_vu(b, p, uend, ok);
  if (!ok || nsec < 2) return;
  if (w.fwc_off && w.fwc_off[u] != NONE) {  // record mode (k_fwc ran over the update's chain)
    if (lane == 0) fwm_records(w, u, nsec, p);
    return;
  }
  // pass 1 (every value below is the same in every lane)
  const uint32_t nchk = min(nsec, w.fwm_max ? min(w.fwm_max, FWM_MAX) : FWM_MAX);
  uint32_t done = 0;          // sections vouched for
  uint32_t hdr = p;           // section done's header (unless from_last: then past cur's struct)
  uint32_t cur = p;           // the previous section's last struct when from_last
  bool from_last = false;
  bool broke = false;
  unsigned long long t_stage = 0, t_walk = 0, t_search = 0, n_walk = 0;  // (YCRDT_DEBUG_DECODE: cycles per part)
  for (uint32_t s = 0; s < nchk; ++s) {
    const unsigned long long tc0 = w.dbg ? clock64() : 0ull;
    // ONE round of loads: the bytes from the header (or the previous section's last struct) and
    // their struct-start words staged in LDS; the struct-start words of the two chunks from the
    // stage's start (held in lanes 0 .. 2 SWC - 1); the count and off prefixes of the 64 chunks from
    // there (lane l: through the end of chunk jb + l)
    const uint32_t s0 = (from_last ? cur : hdr) & ~15u;
    const uint32_t wlen = min(FWM_STAGE, (uend + 15u - min(s0, uend)) & ~15u);  // (never past the update)
    const uint32_t jb = (min(s0, uend - 1) - ustart) / CH;
    const uint32_t wb = (ustart + jb * CH) >> 6, wlast = (uend - 1) >> 6;
    __syncthreads();  // (the previous step's reads of the stage are done)
    if (lane * 8 < wlen) ((uint2*)stg)[lane] = ((const uint2*)(b + s0))[lane];
    if (lane < FWM_STAGE / 64 + 2) sspec[lane] = (s0 >> 6) + lane <= wlast ? spec[(s0 >> 6) + lane] : 0ull;
    const uint64_t cw = lane < 2 * SWC && wb + lane <= wlast ? spec[wb + lane] : 0ull;
    const bool pv = jb + lane < nch;
    const uint64_t P = pv ? w.cpre[c0 + jb + lane + 1] : ~0ull;
    const uint32_t O = pv ? w.opre[c0 + jb + lane + 1] : 0u;
    __syncthreads();
    const unsigned long long tc1 = w.dbg ? clock64() : 0ull;
    const LdsSrc src{b, stg, s0, wlen};
    auto spec_bit = [&](uint32_t q) {
      const uint32_t k = (q >> 6) - (s0 >> 6);
      return ((k < FWM_STAGE / 64 + 2 ? sspec[k] : spec[q >> 6]) >> (q & 63)) & 1ull;
    };
    // the chain positions in [a, e) of chunk j's words (lanes' registers when j is jb or jb + 1)
    auto chunk_words = [&](uint32_t jc, uint32_t a, uint32_t e) -> uint64_t {
      const uint32_t cs = ustart + jc * CH;
      uint64_t x = 0;
      if (jc == jb || (jc == jb + 1 && 2 * SWC <= 64)) {
        const uint32_t k = lane - (jc - jb) * SWC;
        if (k < SWC) {
          const uint32_t wd = (cs >> 6) + k;
          if (wd * 64 + 63 >= a && wd * 64 < e) {
            x = cw;
            if (wd == (a >> 6)) x &= ~0ull << (a & 63);
            if (wd == ((e - 1) >> 6)) x &= ~0ull >> (63 - ((e - 1) & 63));
          }
        }
      } else if (lane < SWC) {
        const uint32_t wd = (cs >> 6) + lane;
        if (wd * 64 + 63 >= a && wd * 64 < e) x = range_word(spec, wd, a, e);
      }
      return x;
    };
    if (from_last) {  // the header follows the previous section's last struct
      const uint32_t dl = cur < uend ? chain_len(src, b, cur, uend) : 0u;
      if (!dl || cur + dl > uend) {  // (the previous section's end is unknown: it is not vouched for)
        why(7);
        done = s - 1;
        hdr = shp[s - 1];
        broke = true;
        break;
      }
      hdr = cur + dl;
    }
    if (lane == 0) shp[s] = hdr;
    p = hdr;
    const uint32_t n = rd_vu_src(src, p, uend, ok), client = rd_vu_src(src, p, uend, ok), clock = rd_vu_src(src, p, uend, ok);
    if (!ok || n > uend - p) { why(3); broke = true; break; }
    const uint32_t p1 = p;
    uint32_t q = p1, k0 = 0, e = p1;
    from_last = false;
    if (n) {
      if (p1 >= uend) { why(3); broke = true; break; }
      // the exact walk (lane 0, from the stage) until it meets the chain: a section header breaks
      // the chain's phase, and a section starting near a chunk's end meets it only in a later chunk
      uint32_t walk_bad = 0;
      if (lane == 0) {
        for (uint32_t steps = 0; q < uend && k0 < n && !spec_bit(q); ++steps) {
          if (steps == FWM_WALK) { q = uend; break; }
          const uint32_t dq = chain_len(src, b, q, uend);
          if (!dq) { walk_bad = 1; break; }  // no struct parses: k_walk reports it
          q += dq;
          ++k0;
        }
      }
      if (__shfl(walk_bad, 0)) { why(4); broke = true; break; }
      q = __shfl(q, 0);
      k0 = __shfl(k0, 0);
      const unsigned long long tc2 = w.dbg ? clock64() : 0ull;
      if (w.dbg) { t_stage += tc1 - tc0; t_walk += tc2 - tc1; n_walk += k0; }
      if (k0 == n) {  // every struct walked: the next header is where the walk stopped
        if (q > uend) { why(3); broke = true; break; }
        e = q;  // (an empty chain range [q, q))
        p = q;
      } else {
        if (q >= uend) {  // no meeting within FWM_WALK structs
          if (w.dbg && lane == 0) { w.dbg[14] = s; w.dbg[15] = n; w.dbg[12] = p1 - ustart; w.dbg[11] = uend - ustart; }
          why(5);
          broke = true;
          break;
        }
        // the target-th chain position from q (q the first) is the section's last struct
        const uint32_t target = n - k0;
        const uint32_t jq = (q - ustart) / CH, ceq = min(ustart + jq * CH + CH, uend);
        const uint32_t cq = wave_sum_u32((uint32_t)__popcll(chunk_words(jq, q, ceq)));
        uint32_t fch = jq, rem = target, fa = q;
        if (target > cq) {
          const uint64_t need = target - cq;
          bool found = false;
          if (jq - jb < 2u) {  // the prefixes from the stage's chunk: chunks jq + 1 .. jb + 63
            const uint32_t jr = jq - jb;
            const uint64_t base = __shfl((unsigned long long)P, jr);
            const uint32_t obase = __shfl(O, jr);
            const uint64_t m = __ballot(lane > jr && pv && P - base >= need);
            if (m) {
              const uint32_t L = (uint32_t)__ffsll((long long)m) - 1;
              if (__shfl((uint32_t)(O != obase), L)) { why(2); broke = true; break; }
              const uint64_t before = L > jr + 1 ? (uint64_t)__shfl((unsigned long long)P, L - 1) - base : 0ull;
              fch = jb + L;
              rem = (uint32_t)(need - before);
              found = true;
            }
          }
          if (!found) {  // further on: the 64-way search over the prefixes
            uint32_t wy = 0;
            if (!chain_target(w, spec, ustart, uend, c0, nch, jq, q, target, lane, fch, rem, wy)) { why(wy ? 2 : 6); broke = true; break; }
          }
          fa = ustart + fch * CH;
        }
        // the rem-th chain position at or after fa in chunk fch
        const uint32_t fcs = ustart + fch * CH, fce = min(fcs + CH, uend);
        const uint64_t yw = chunk_words(fch, fa, fce);
        const uint32_t yc = (uint32_t)__popcll(yw);
        uint32_t incl = yc;
        for (uint32_t off = 1; off < 64; off <<= 1) {
          const uint32_t v = __shfl_up(incl, off);
          if (lane >= off) incl += v;
        }
        const uint64_t hit = __ballot(yc && incl >= rem);
        if (!hit) { why(6); broke = true; break; }  // (the counts said the chunk holds it)
        const uint32_t L = (uint32_t)__ffsll((long long)hit) - 1;
        // (the lane's word: from the registers' chunk layout, or lane = word offset in chunk fch)
        const uint32_t kword = (fch == jb || (fch == jb + 1 && 2 * SWC <= 64)) ? L - (fch - jb) * SWC : L;
        const uint32_t Lp = __shfl(lane == L ? ((fcs >> 6) + kword) * 64 + nth_set1(yw, rem - (incl - yc)) : 0u, L);
        e = Lp + 1;
        cur = Lp;
        from_last = true;
        if (w.dbg) t_search += clock64() - tc2;
      }
    }
    if (lane == 0) { sp1[s] = p1; sn[s] = n; scl[s] = client; sck[s] = clock; se[s] = e; sk0[s] = k0; sq[s] = n ? q : p1; }
    done = s + 1;
    if (!from_last) hdr = p;  // the next header (the section ends where its header or walk ended)
  }
  if (!broke && from_last) {  // the last section checked ends at its last struct (cur)
    const uint32_t dl = cur < uend ? chain_len(GlobalSrc{b}, b, cur, uend) : 0u;
    if (!dl || cur + dl > uend) {
      why(7);
      done -= 1;
      hdr = shp[done];
    } else {
      hdr = cur + dl;
    }
  }
  if (w.dbg && lane == 0) {
    atomicAdd(&w.dbg[19], t_stage); atomicAdd(&w.dbg[20], t_walk); atomicAdd(&w.dbg[21], t_search);
    atomicAdd(&w.dbg[22], n_walk); atomicAdd(&w.dbg[23], (unsigned long long)done);
  }
  if (done == 0) return;  // nothing vouched for: k_walk takes the update from its start
  if (!broke && done < nsec) why(1);  // more sections than FWM_MAX
  // pass 2: commit the vouched sections (records for all nsec; k_walk writes the rest)
  __syncthreads();
  if (lane == 0) sh_sbase = atomicAdd(&w.ctr->nsections, nsec);
  __syncthreads();
  const uint32_t sbase = sh_sbase;
  if (sbase + nsec > w.cap_sections) { if (lane == 0) raise_err(&w.ctr->err, ERR_CAPACITY); return; }
  for (uint32_t s = lane; s < done; s += 64) {
    const uint32_t n = sn[s], p1 = sp1[s];
    Section sec;
    sec.upd = u; sec.n = n; sec.client = scl[s]; sec.clock = sck[s];
    sec.first_pos = n ? p1 : NONE; sec.cidx = NONE; sec.first_idx = NONE; sec.pad = 0;
    w.sections[sbase + s] = sec;
    if (n) atomicOr((unsigned long long*)&sbits[p1 >> 6], 1ull << (p1 & 63));
    // the walked positions (not on the chain), again
    uint32_t x = p1;
    for (uint32_t k = 0; k < sk0[s]; ++k) {
      atomicOr((unsigned long long*)&fbits[x >> 6], 1ull << (x & 63));
      x = chain_step(b, x, uend);
    }
    w.fwsec[2 * (sbase + s)] = sq[s];
    w.fwsec[2 * (sbase + s) + 1] = se[s];
  }
  if (lane == 0) {
    w.usec_start[u] = sbase;
    w.usec_n[u] = nsec;
    if (done == nsec) {
      w.dsstart[u] = hdr;  // (past the last section: the delete set)
      w.ufail[u] = 3u;     // done: k_walk leaves it alone, k_fastmark copies the chain ranges
      if (w.dbg) atomicAdd(&w.dbg[0], 1ull);
    } else {
      w.fw[2 * u] = done;  // k_walk resumes at section `done`, whose header is at hdr
      w.fw[2 * u + 1] = hdr;
      w.ufail[u] = 4u;
    }
  }
}
// per chunk: its chain positions, and whether its entry may be off the one chain (coff): it was
// entered past its end (its predecessor's chain jumped over it: it keeps a chain of its own), or
// its predecessor's exit moved in the last sync round (it was walked from an older entry). A fast
// walk trusts the chunk chains from its meeting point to its last struct only when no chunk after
// the meeting chunk is off (checked per section, not per update: a multi-section snapshot's
// headers, parsed as garbage, jump chunks in other sections)
__device__ __forceinline__ bool chunk_moved(const Work& w, uint32_t i) {
  const Group G = w.groups[i];
  return G.end < G.uend && w.cexit[i] != w.sexit[i];
}
__global__ __launch_bounds__(256) void k_chunk_counts(Work w) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > w.ngroups) return;
  if (i == w.ngroups) { w.ccnt[i] = 0; w.coff[i] = 0; return; }  // (the scans' last entries)
  const Group G = w.groups[i];
  const bool first = i == w.ugroup[G.upd];
  const bool jumped = !first && w.sent[w.ngroups + 1 + i];
  const bool moved = !first && chunk_moved(w, i - 1);
  w.ccnt[i] = popc_range(win_words(w.spec_bits, upd_win(w, G.upd)), G.start, G.end);
  w.coff[i] = jumped || moved ? 1u : 0u;
  if (w.dbg) {  // (YCRDT_DEBUG_DECODE, printed as the wave path's "unsettled" / "other")
    if (moved) atomicAdd(&w.dbg[4], 1ull);
    if (jumped) atomicAdd(&w.dbg[5], 1ull);
  }
}

// The chain-position words of the fast-walked updates past their first chunk, one lane per word
// of every chunk (grid-stride).
__global__ __launch_bounds__(256) void k_fastmark(Work w) {
  const uint32_t wpc = w.schunk / 64;  // words per chunk (chunks are 64-byte aligned)
  const uint64_t total = (uint64_t)w.ngroups * wpc;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
    const Group gr = w.groups[t / wpc];
    const uint32_t u = gr.upd;
    const uint32_t uf = w.ufail[u];
    if (uf < 2u || uf >= UF_PRE) continue;
    const uint32_t wd = (gr.start >> 6) + (uint32_t)(t % wpc);
    if (uf >= 3u) {  // several sections (k_fastwalk_multi): the chain ranges meeting this word
      // (ufail 4: only its first fw[2u] sections; k_walk resumes past them)
      if ((uint64_t)wd * 64 >= gr.end) continue;
      const uint32_t s0 = w.usec_start[u], ns = uf == 4u ? w.fw[2 * u] : w.usec_n[u], a = wd * 64;
      uint32_t lo = 0, hi = ns;
      while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (w.fwsec[2 * (s0 + m) + 1] <= a) lo = m + 1; else hi = m; }
      const uint32_t uw = upd_win(w, u);
      const uint64_t* sp = win_words(w.spec_bits, uw);
      uint64_t x = 0;
      for (uint32_t s = lo; s < ns; ++s) {
        const uint32_t q = w.fwsec[2 * (s0 + s)], e = w.fwsec[2 * (s0 + s) + 1];
        if (q >= a + 64) break;
        if (q < e && wd >= (q >> 6) && wd <= ((e - 1) >> 6)) x |= range_word(sp, wd, q, e);
      }
      if (x) win_words(w.final_bits, uw)[wd] |= x;
      continue;
    }
    const uint32_t q = w.fw[2 * u], e = w.fw[2 * u + 1];
    if (wd <= (w.uoff[u] >> 6) + SW + 1 || wd > ((e - 1) >> 6)) continue;  // (k_fastwalk's words; past the last struct)
    const uint32_t uw = upd_win(w, u);
    win_words(w.final_bits, uw)[wd] = range_word(win_words(w.spec_bits, uw), wd, q, e);
  }
}

// Small updates, one wavefront each (k_direct: one lane each). The update (<= DIRECT 16 KiB) is
// staged in LDS with one round of loads; for a single-section update each lane follows the chunk
// chain of 1/64 of it (lane 0 from the first struct, exactly), the lanes re-enter their chunks
// where the previous lane's chain leaves until no exit changes (a wavefront-local k_sync), and the
// n-th chain position from the first struct — a popcount scan across the lanes — is the section's
// last struct. A struct step waits on LDS only, and 64 lanes share an update: an update costs
// ~1/64 of the lane-serial walk's latency, so few updates (one C2 document's 1 000 replicas) no
// longer leave the GPU idle, and many pack 64 x more parallel work. Several sections, a chain that
// does not settle in WD_ROUNDS, or fewer chain positions than structs: lane 0 walks the update
// exactly (as k_direct, from LDS), which also reports malformed input.
// k_wdecode's struct step (inline: an out-of-line step, or only its slow part out of line, was
// slower — the garbage the chunk chains parse takes the slow part often)
__device__ __forceinline__ uint32_t wd_len(const uint32_t* ub, uint32_t ustart, uint32_t wlen,
                                           const uint8_t* __restrict__ b, uint32_t q, uint32_t uend) {
  const LdsSrc src{b, ub, ustart, wlen};
  return chain_len(src, b, q, uend, nullptr, (const uint8_t*)ub, ustart);
}
constexpr uint32_t WD_MAX = 16384, WD_WORDS = WD_MAX / 64, WD_ROUNDS = 64;
constexpr uint32_t WD_LANE_MIN = 1024;  // small updates from which k_direct (a lane each) takes over
constexpr uint32_t WD_HINT = 5;
__global__ __launch_bounds__(64) void k_wdecode(Work w) {
  __shared__ __attribute__((aligned(16))) uint32_t ub[(WD_MAX + 64) / 4];
  __shared__ uint64_t bits[WD_WORDS + 1];
  __shared__ uint64_t walkbuf[64][WD_WORDS / 64];  // a lane's walked positions, before it commits them
  __shared__ uint32_t infoset[8];                   // info bytes on lane 0's exact chain
  const uint32_t lane = threadIdx.x;
  if (blockIdx.x >= w.nsmall) return;
  const uint32_t u = w.ulist[w.nbig + blockIdx.x];
  const uint32_t uw = upd_win(w, u);
  const uint8_t* __restrict__ b = win_bytes(w, uw);
  uint64_t* __restrict__ fbits = win_words(w.final_bits, uw);
  uint64_t* __restrict__ sbits = win_words(w.sec_bits, uw);
  const uint32_t ustart = w.uoff[u], L = w.ulen[u], uend = ustart + L;
  uint32_t* err = &w.ctr->err;
  if (L > WD_MAX) { if (lane == 0) raise_err(err, ERR_CAPACITY); return; }  // (the layout never sends one)
  // stage: the update's 16-byte lines (updates are 64-byte aligned; the buffer is padded)
  const uint32_t nq = (L + 15) / 16;
  for (uint32_t k = lane; k < nq; k += 64) ((uint4*)ub)[k] = ((const uint4*)(b + ustart))[k];
  const uint32_t nw = (L + 63) / 64;
  for (uint32_t k = lane; k < nw; k += 64) bits[k] = 0;
  __syncthreads();
  const LdsSrc src{b, ub, ustart, nq * 16};
  const uint8_t* ubb = (const uint8_t*)ub;  // the staged bytes (update position ustart + k at ubb[k])
  bool ok = true;
  uint32_t p = ustart;
  const uint32_t nsec = rd_vu(b, p, uend, ok);
  if (!ok || nsec > (uend - p) / 3 + 1) { if (lane == 0) { raise_err(err, ERR_DECODE); w.dsstart[u] = NONE; } return; }
  uint32_t sbase = 0;
  if (lane == 0) sbase = atomicAdd(&w.ctr->nsections, nsec);
  sbase = __shfl(sbase, 0);
  if (sbase + nsec > w.cap_sections) { if (lane == 0) { raise_err(err, ERR_CAPACITY); w.dsstart[u] = NONE; } return; }
  auto setbit = [&](uint32_t q) { bits[(q - ustart) >> 6] |= 1ull << (q & 63); };
  uint32_t dsp = NONE;
  bool done = false;
  uint32_t why = 5;  // debug: 4 = not settled / jumped, 5 = several sections or short
  if (nsec == 1) {
    uint32_t q1 = p;
    const uint32_t n = rd_vu(b, q1, uend, ok), client = rd_vu(b, q1, uend, ok), clock = rd_vu(b, q1, uend, ok);
    if (ok && n > 0 && n <= uend - q1) {
      // chunks: CW bytes per lane, 64-byte multiples from the update start (each lane owns words)
      const uint32_t CW = ((L + 63) / 64 + 63) & ~63u;
      const uint32_t cs = ustart + lane * CW, ce = min(cs + CW, uend);
      const bool live = ce > q1 && cs < uend;
      uint32_t x = NONE;  // this lane's chain exit
      // lane 0's chain is exact (from the first struct): the info bytes it meets are the stream's
      // struct kinds; the other lanes start their chains at a run of three chain steps on such
      // bytes (a hint the settling verifies) — a single first-struct byte missed streams whose
      // first struct is of a rarer kind, and their chains locked out of phase
      if (lane == 0) {
        for (uint32_t k = 0; k < 8; ++k) infoset[k] = 0;
        if (live) {
          uint32_t q = q1;
          while (q < ce) {
            setbit(q);
            const uint32_t c = src.u8(q);
            infoset[c >> 5] |= 1u << (c & 31);
            const uint32_t d = wd_len(ub, ustart, nq * 16, b, q, uend);
            q += d ? d : 1u;
          }
          x = q;
        }
      }
      __syncthreads();
      auto kind = [&](uint32_t h) { const uint32_t c = src.u8(h); return (infoset[c >> 5] >> (c & 31)) & 1u; };
      if (live && lane > 0) {
        uint32_t q = max(cs, q1);
        if (cs > q1) {
          const uint32_t lim = min(cs + 96u, ce);
          for (uint32_t h = cs; h < lim; ++h) {
            if (!kind(h)) continue;
            uint32_t t = h, k = 0;  // WD_HINT consecutive chain steps on struct-kind bytes
            for (; k < WD_HINT; ++k) {
              const uint32_t d = wd_len(ub, ustart, nq * 16, b, t, uend);
              if (!d || t + d >= uend || !kind(t + d)) break;
              t += d;
            }
            if (k < WD_HINT && t + 1 < uend) continue;
            q = h;
            break;
          }
        }
        while (q < ce) {
          setbit(q);
          const uint32_t d = wd_len(ub, ustart, nq * 16, b, q, uend);
          q += d ? d : 1u;
        }
        x = q;
      }
      // Settling. A lane re-walks its chunk from its entry E (the previous lane's exit) when E
      // changed, collecting the walked positions aside; meeting its own chain, it keeps the own
      // positions from there (they are the walk's continuation). A walk that does not meet means
      // one of the two chains is out of phase: only the lowest such lane — whose entry is right,
      // every lane before it being consistent — overwrites its chunk with the walk; the others
      // keep their own chains (the next lane's chain is usually the right one: overwriting it
      // with a walk from a wrong entry cascaded one chunk per round to the update's end) and stay
      // "unsettled" until they are the lowest. Settled: no exit changed and every lane consistent.
      bool settled = false;
      bool okc = !(live && lane > 0 && cs >= q1);  // lanes that never re-walk are consistent
      uint32_t sent = NONE;
      uint64_t* wk = walkbuf[lane];
      const uint32_t w0 = (cs - ustart) >> 6, wend = live ? (ce - ustart + 63) >> 6 : w0;
      bool beyond = false;  // this chunk lies past the section's last struct: nothing to settle
      for (uint32_t r = 0; r < WD_ROUNDS; ++r) {
        const uint32_t E = __shfl_up(x, 1);
        {
          // lanes whose predecessors are all consistent and already hold n chain positions are past
          // the last struct (their chunks hold the delete set): they leave the settling, which
          // otherwise cascaded through the delete set's garbage chains a chunk per round
          uint32_t cnt = 0;
          for (uint32_t k = w0; k < wend; ++k) cnt += (uint32_t)__popcll(bits[k]);
          uint32_t inc = cnt;
          for (uint32_t off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(inc, off);
            if (lane >= off) inc += y;
          }
          // (a lane whose entry changed since its walk is not consistent yet, whatever okc says)
          const bool stale = !beyond && live && lane > 0 && cs >= q1 && E != sent;
          const uint64_t b0 = __ballot(!okc || stale);
          const uint32_t fb = b0 ? (uint32_t)__ffsll((long long)b0) - 1 : 64u;
          if (lane > 0 && lane <= fb && inc - cnt >= n) { beyond = true; okc = true; }
        }
        const uint64_t bad = __ballot(!okc);
        const uint32_t first_bad = bad ? (uint32_t)__ffsll((long long)bad) - 1 : 64u;
        uint32_t nx = x;
        bool walked = false, met = false;
        uint32_t q = E;
        if (!beyond && (!okc || (live && lane > 0 && cs >= q1 && E != sent))) {
          if (E != sent || lane == first_bad) {
            sent = E;
            walked = true;
            if (E >= ce) {  // the previous chain jumps over this chunk: no struct starts in it
              for (uint32_t k = w0; k < wend; ++k) bits[k] = 0;
              nx = E;
              met = true;
            } else {
              for (uint32_t k = 0; k < wend - w0; ++k) wk[k] = 0;
              while (q < ce && !((bits[(q - ustart) >> 6] >> (q & 63)) & 1ull)) {
                wk[((q - ustart) >> 6) - w0] |= 1ull << (q & 63);
                const uint32_t d = wd_len(ub, ustart, nq * 16, b, q, uend);
                q += d ? d : 1u;
              }
              met = q < ce;
              if (met) {  // met the own chain at q: walked positions, then the own chain
                const uint32_t qw = (q - ustart) >> 6;
                for (uint32_t k = w0; k < qw; ++k) bits[k] = wk[k - w0];
                bits[qw] = wk[qw - w0] | (bits[qw] & (~0ull << (q & 63)));
              }
            }
          }
        }
        const uint64_t nm = __ballot(walked && !met);
        const uint32_t first_nm = nm ? (uint32_t)__ffsll((long long)nm) - 1 : 64u;
        if (walked && met) okc = true;
        if (walked && !met) {
          if (lane == first_nm) {  // the lowest: its entry is right, its own chain is not
            for (uint32_t k = w0; k < wend; ++k) bits[k] = wk[k - w0];
            nx = q;
            okc = true;
          } else {
            okc = false;
          }
        }
        const bool changed = __ballot(nx != x && !beyond) != 0;
        x = nx;
        if (!changed && !__ballot(!okc)) { settled = true; if (lane == 0 && w.dbg) atomicAdd(&w.dbg[6], (unsigned long long)r + 1); break; }
      }
      const bool jumped = false;
      __syncthreads();
      if (!settled || jumped) why = 4;
      if (settled && !jumped) {
        // the n-th chain position from q1: per-lane counts over the lane's words, a wave scan
        const uint32_t w0 = (cs - ustart) >> 6, w1 = live ? (ce - ustart + 63) >> 6 : w0;
        uint32_t cnt = 0;
        for (uint32_t k = w0; k < w1; ++k) cnt += (uint32_t)__popcll(bits[k]);
        uint32_t inc = cnt;
        for (uint32_t off = 1; off < 64; off <<= 1) {
          const uint32_t y = __shfl_up(inc, off);
          if (lane >= off) inc += y;
        }
        const uint64_t hit = __ballot(inc >= n && inc - cnt < n);
        if (hit) {
          const uint32_t owner = (uint32_t)__ffsll((long long)hit) - 1;
          uint32_t lp = NONE;
          if (lane == owner) {
            uint32_t rem = n - (inc - cnt), k = w0;
            for (;; ++k) { const uint32_t c = (uint32_t)__popcll(bits[k]); if (c >= rem) break; rem -= c; }
            uint64_t m = bits[k];
            for (uint32_t t = 1; t < rem; ++t) m &= m - 1;
            lp = ustart + k * 64 + (uint32_t)__ffsll((long long)m) - 1;
            const uint32_t d = wd_len(ub, ustart, nq * 16, b, lp, uend);
            dsp = d ? lp + d : NONE;
            // drop the chain positions past the last struct (delete-set bytes)
            bits[k] &= ~0ull >> (63 - (lp & 63));
            for (++k; k < w1; ++k) bits[k] = 0;
          }
          dsp = __shfl(dsp, owner);
          if (lane > owner) for (uint32_t k = w0; k < w1; ++k) bits[k] = 0;
          if (dsp != NONE && dsp <= uend) {
            done = true;
            if (lane == 0) {
              Section sec;
              sec.upd = u; sec.n = n; sec.client = client; sec.clock = clock;
              sec.first_pos = q1; sec.cidx = NONE; sec.first_idx = NONE; sec.pad = 0;
              w.sections[sbase] = sec;
              atomicOr((unsigned long long*)&sbits[q1 >> 6], 1ull << (q1 & 63));
            }
          }
        }
      }
      __syncthreads();
      if (!done) for (uint32_t k = lane; k < nw; k += 64) bits[k] = 0;
      __syncthreads();
    }
  }
  if (lane == 0 && w.dbg) atomicAdd(&w.dbg[done ? 3 : why], 1ull);  // (YCRDT_DEBUG_DECODE)
  if (!done && lane == 0) {
    // exact walk of every section (as k_direct), from LDS
    dsp = NONE;
    bool fail = false;
    uint32_t q = p;
    for (uint32_t sct = 0; sct < nsec && !fail; ++sct) {
      const uint32_t n = rd_vu(b, q, uend, ok), client = rd_vu(b, q, uend, ok), clock = rd_vu(b, q, uend, ok);
      if (!ok || n > uend - q) { raise_err(err, ERR_DECODE); fail = true; break; }
      Section sec;
      sec.upd = u; sec.n = n; sec.client = client; sec.clock = clock;
      sec.first_pos = n ? q : NONE; sec.cidx = NONE; sec.first_idx = NONE; sec.pad = 0;
      w.sections[sbase + sct] = sec;
      if (n) atomicOr((unsigned long long*)&sbits[q >> 6], 1ull << (q & 63));
      for (uint32_t k = 0; k < n; ++k) {
        if (q >= uend) { raise_err(err, ERR_DECODE); w.ctr->err_info = q; fail = true; break; }
        setbit(q);
        const uint32_t d = wd_len(ub, ustart, nq * 16, b, q, uend);  // exact on valid structs; 0: none parses
        if (!d) { raise_err(err, ERR_DECODE); w.ctr->err_info = q; fail = true; break; }
        q += d;
      }
    }
    if (!fail) dsp = q;
  }
  __syncthreads();
  if (lane == 0) {
    w.usec_start[u] = sbase;
    w.usec_n[u] = nsec;
  }
  dsp = __shfl(dsp, 0);
  if (lane == 0) w.dsstart[u] = dsp;
  // the update's words of the final bitmap (its own: updates are 64-byte aligned)
  for (uint32_t k = lane; k < nw; k += 64) fbits[(ustart >> 6) + k] = bits[k];
}

// Positions of the chunks the table walk entered without parsing (tentry): one lane per chunk
// parses exactly from the entry to the chunk end through its LDS window and marks them.
__global__ __launch_bounds__(DL) void k_xmark(Work w) {
  __shared__ __attribute__((aligned(16))) uint32_t win[DL * DSTRIDE];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= w.ctr->xchunks) return;
  const uint32_t i = w.xlist[t];
  const Group G = w.groups[i];
  uint32_t p = w.tentry[i];
  if (p == NONE) return;
  const uint32_t uw = upd_win(w, G.upd);
  const uint8_t* __restrict__ b = win_bytes(w, uw);
  uint64_t* __restrict__ fbits = win_words(w.final_bits, uw);
  const uint32_t uend = G.uend;
  uint32_t* slot = win + threadIdx.x * DSTRIDE;
  LdsSrc src{b, slot, 0, 0};
  auto refill = [&](uint32_t x) {
    src.s0 = x & ~15u;
    src.wlen = min(DW, (uend + 15u - src.s0) & ~15u);
    const uint4* g = (const uint4*)(b + src.s0);
    fill_window(slot, g);
  };
  refill(p);
  uint32_t word = p >> 6;
  uint64_t m = 0;
  while (p < G.end) {
    if ((p >> 6) != word) {
      if (m) atomicOr((unsigned long long*)&fbits[word], (unsigned long long)m);
      word = p >> 6;
      m = 0;
    }
    m |= 1ull << (p & 63);
    if (src.wlen == DW && p - src.s0 + DREFILL > DW) refill(p);
    const uint32_t d = tab_len(rtab_of(w, G.upd), w.uoff[G.upd], src, b, p, uend);
    p += d ? d : 1u;
  }
  if (m) atomicOr((unsigned long long*)&fbits[word], (unsigned long long)m);
}

// A doc state decoded by the encode that produced it (PreMarks, k_state_marks): its bitmap words
// copied into the batch's (the state is 64-byte aligned: word for word), its section records
// appended, its delete-set start set. check: the state was decoded the usual way as well — every
// word and the delete-set start must agree (YCRDT_PREDECODE=check, tests).
__global__ void k_predecoded(Work w, uint32_t u, PreMarks m, uint32_t check) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, gs = gridDim.x * blockDim.x;
  const uint32_t uw = upd_win(w, u), w0 = w.uoff[u] >> 6;
  uint64_t* __restrict__ fb = win_words(w.final_bits, uw);
  uint64_t* __restrict__ sb = win_words(w.sec_bits, uw);
  const uint32_t nsec = min(m.meta[0], m.cap_secs);
  if (check) {
    for (uint32_t k = t; k < m.nw; k += gs)
      if (fb[w0 + k] != m.fbits[k] || sb[w0 + k] != m.sbits[k]) {
        raise_err(&w.ctr->err, ERR_DECODE);
        const bool f = fb[w0 + k] != m.fbits[k];
        w.ctr->err_info = 0xC0DE0000u | (f ? 0u : 0x8000u) | min(k, 0x7FFFu);  // (for the message: check() in yc_engine.hip)
        const uint64_t a = f ? fb[w0 + k] : sb[w0 + k], z = f ? m.fbits[k] : m.sbits[k];
        w.ctr->pad[8] = (uint32_t)a; w.ctr->pad[9] = (uint32_t)(a >> 32); w.ctr->pad[10] = (uint32_t)z; w.ctr->pad[11] = (uint32_t)(z >> 32) | (f ? 0u : 0u);
      }
    if (t == 0 && w.dsstart[u] != w.uoff[u] + m.meta[1]) {
      raise_err(&w.ctr->err, ERR_DECODE);
      w.ctr->err_info = 0xC0DF0000u;
      w.ctr->pad[8] = w.dsstart[u]; w.ctr->pad[9] = w.uoff[u] + m.meta[1]; w.ctr->pad[10] = m.meta[0]; w.ctr->pad[11] = m.nw;
    }
    return;
  }
  for (uint32_t k = t; k < m.nw; k += gs) { fb[w0 + k] = m.fbits[k]; sb[w0 + k] = m.sbits[k]; }
  __shared__ uint32_t sbase, part[256];
  if (blockIdx.x == 0) {
    if (threadIdx.x == 0) sbase = atomicAdd(&w.ctr->nsections, nsec);
    __syncthreads();
    if (sbase + nsec > w.cap_sections) { if (threadIdx.x == 0) raise_err(&w.ctr->err, ERR_CAPACITY); return; }
    // the records in the update's byte order (descending client slot), compacted 256 at a time
    const uint32_t nslots = m.meta[2];
    uint32_t out = 0;
    for (uint32_t r0 = 0; r0 < nslots; r0 += 256) {
      const uint32_t r = r0 + threadIdx.x;
      Section sec;
      const bool has = r < nslots && (sec = m.secs[nslots - 1 - r]).n != 0;
      part[threadIdx.x] = has ? 1u : 0u;
      __syncthreads();
      for (uint32_t off = 1; off < 256; off <<= 1) {
        const uint32_t x = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += x;
        __syncthreads();
      }
      if (has && out + part[threadIdx.x] - 1 < nsec) {
        sec.upd = u;
        sec.first_pos += w.uoff[u];
        w.sections[sbase + out + part[threadIdx.x] - 1] = sec;
      }
      out += part[255];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      w.usec_start[u] = sbase;
      w.usec_n[u] = nsec;
      w.ufail[u] = UF_PRE;  // (every walker leaves it alone; its chunks serve the grid delete-set decode)
      w.dsstart[u] = w.uoff[u] + m.meta[1];
    }
  }
}
void launch_predecoded(const Work& w, uint32_t u, const PreMarks& m, bool check, hipStream_t s) {
  hipLaunchKernelGGL(k_predecoded, dim3(std::min<uint32_t>(m.nw / 256 + 1, 1024)), dim3(256), 0, s, w, u, m, check ? 1u : 0u);
}

// Large updates with a short struct section — a delta carrying the doc's whole delete set (the sync
// reply, crdt.js:288, Y.encodeStateAsUpdate(doc, sv) always writes the full delete set), a few
// structs in front of hundreds of KB of ranges: one lane per large update walks the struct section
// exactly for up to PREWALK_STEPS structs. When it reaches the end, the update is decoded (sections,
// struct starts, delete-set start; ufail UF_WALKED) and the chunk chains skip its chunks, whose
// speculative walks over the delete set's bytes were all garbage (a 228 KB delta: k_spec + k_sync
// 2.4 ms at 14 wavefronts). Otherwise it leaves the update to the chunk path untouched.
constexpr uint32_t PREWALK_STEPS = 64;
__global__ void k_prewalk(Work w) {
  const uint32_t bi = blockIdx.x * blockDim.x + threadIdx.x;
  if (bi >= w.nbig) return;
  const uint32_t u = w.ulist[bi];
  if (w.ufail[u] || !w.ulen[u]) return;
  const uint32_t uw = upd_win(w, u);
  const uint8_t* __restrict__ b = win_bytes(w, uw);
  const uint32_t ustart = w.uoff[u], uend = ustart + w.ulen[u];
  uint32_t p = ustart, steps = 0;
  bool ok = true;
  const uint32_t nsec = rd_vu(b, p, uend, ok);
  if (!ok || nsec > 8) return;
  uint32_t hp[8];  // the section headers
  for (uint32_t s = 0; s < nsec; ++s) {
    hp[s] = p;
    const uint32_t n = rd_vu(b, p, uend, ok);
    rd_vu(b, p, uend, ok);
    rd_vu(b, p, uend, ok);
    if (!ok || n > PREWALK_STEPS - steps) return;
    for (uint32_t k = 0; k < n; ++k) {
      const uint32_t d = p < uend ? chain_len(GlobalSrc{b}, b, p, uend) : 0u;
      if (!d || p + d > uend) return;  // (malformed: the walkers report it)
      p += d;
    }
    steps += n;
  }
  // decoded: the records, the marks, the delete-set start
  const uint32_t sbase = atomicAdd(&w.ctr->nsections, nsec);
  if (sbase + nsec > w.cap_sections) { raise_err(&w.ctr->err, ERR_CAPACITY); return; }
  uint64_t* __restrict__ fbits = win_words(w.final_bits, uw);
  uint64_t* __restrict__ sbits = win_words(w.sec_bits, uw);
  for (uint32_t s = 0; s < nsec; ++s) {
    uint32_t q = hp[s];
    const uint32_t n = rd_vu(b, q, uend, ok), client = rd_vu(b, q, uend, ok), clock = rd_vu(b, q, uend, ok);
    Section sec;
    sec.upd = u; sec.n = n; sec.client = client; sec.clock = clock;
    sec.first_pos = n ? q : NONE; sec.cidx = NONE; sec.first_idx = NONE; sec.pad = 0;
    w.sections[sbase + s] = sec;
    if (n) atomicOr((unsigned long long*)&sbits[q >> 6], 1ull << (q & 63));
    for (uint32_t k = 0; k < n; ++k) {
      atomicOr((unsigned long long*)&fbits[q >> 6], 1ull << (q & 63));
      q += chain_len(GlobalSrc{b}, b, q, uend);
    }
  }
  w.usec_start[u] = sbase;
  w.usec_n[u] = nsec;
  w.dsstart[u] = p;
  w.ufail[u] = UF_WALKED;
}

// walk_only: every large update must now be pre-decoded or pre-walked; one that is not (the host's
// struct count and the pre-walk disagree) is a capacity error, and the decode reruns with the walk
__global__ void k_prewalk_check(Work w) {
  const uint32_t bi = blockIdx.x * blockDim.x + threadIdx.x;
  if (bi >= w.nbig) return;
  const uint32_t u = w.ulist[bi], f = w.ufail[u];
  if (w.ulen[u] && f != UF_PRE && f != UF_WALKED) raise_err(&w.ctr->err, ERR_CAPACITY);
}
void launch_chunks(const Work& w, hipStream_t s) {
  if (w.nbig && !w.force_xtab && !env_off("YCRDT_PREWALK")) hipLaunchKernelGGL(k_prewalk, dim3(w.nbig / 64 + 1), dim3(64), 0, s, w);
  if (w.walk_only) {  // (a sync reply's delta behind a doc state: the chunk kernels would find nothing to do)
    hipLaunchKernelGGL(k_prewalk_check, dim3(w.nbig / 64 + 1), dim3(64), 0, s, w);
    return;
  }
  if (w.ngroups) {
    if (w.rtab) hipLaunchKernelGGL(k_rtab, dim3((uint32_t)std::min<uint64_t>((uint64_t)w.ngroups * w.schunk / 256 + 1, 16384)), dim3(256), 0, s, w);
    hipLaunchKernelGGL(k_spec, dim3((w.ngroups + DL - 1) / DL), dim3(DL), 0, s, w);
    for (uint32_t r = 0; r < SYNC_ROUNDS; ++r)
      hipLaunchKernelGGL(k_sync, dim3((w.ngroups + 255) / 256), dim3(256), 0, s, w,
                         (const uint32_t*)(r & 1 ? w.sexit : w.cexit), r & 1 ? w.cexit : w.sexit, r);
  }
  if (w.nbig) {
    // (read per merge: tests compare the fast walks with k_walk alone)
    const bool nofast = getenv("YCRDT_NO_FASTWALK") && getenv("YCRDT_NO_FASTWALK")[0] == '1';
    if (!nofast && !w.force_xtab) {
      hipLaunchKernelGGL(k_chunk_counts, dim3(w.ngroups / 256 + 1), dim3(256), 0, s, w);
      scan_u32_to_u64(w.tmp, w.tmp_bytes, w.ccnt, w.cpre, (uint64_t)w.ngroups + 1, s);
      scan_u32(w.tmp, w.tmp_bytes, w.coff, w.opre, (uint64_t)w.ngroups + 1, s);
      hipLaunchKernelGGL(k_fastwalk, dim3(w.nbig), dim3(64), 0, s, w);
      const uint32_t wgrid = (uint32_t)std::min<uint64_t>((uint64_t)w.ngroups * (w.schunk / 64) / 256 + 1, 8192);
      if (w.fwc) hipLaunchKernelGGL(k_fwc, dim3(wgrid), dim3(256), 0, s, w);  // (record-mode updates only)
      hipLaunchKernelGGL(k_fastwalk_multi, dim3(w.nbig), dim3(64), 0, s, w);
      if (w.fwc) hipLaunchKernelGGL(k_fwc_commit, dim3(64), dim3(256), 0, s, w);
      if (w.rk) {  // the last section the records left, ranked (YCRDT_RANK_LAST=0: k_walk takes it)
        const uint32_t pgrid = (uint32_t)std::min<uint64_t>((uint64_t)w.ngroups * w.schunk / 256 + 1, 16384);
        hipLaunchKernelGGL(k_rk_setup, dim3(w.nbig / 64 + 1), dim3(64), 0, s, w);
        hipLaunchKernelGGL(k_rk_init, dim3(pgrid), dim3(256), 0, s, w);
        for (uint32_t k = 0; k < RK_ROUNDS; ++k) hipLaunchKernelGGL(k_rk_round, dim3(pgrid), dim3(256), 0, s, w, k);
        hipLaunchKernelGGL(k_rk_final, dim3(wgrid), dim3(256), 0, s, w);
        hipLaunchKernelGGL(k_rk_commit, dim3(w.nbig / 64 + 1), dim3(64), 0, s, w);
      }
      hipLaunchKernelGGL(k_fastmark, dim3(std::min<uint64_t>((uint64_t)w.ngroups * (w.schunk / 64) / 256 + 1, 8192)), dim3(256), 0, s, w);
    }
    hipLaunchKernelGGL(k_walk<false>, dim3(w.nbig), dim3(64), 0, s, w);
    // the table path, for updates the speculative walk handed over (grid-stride over xlist)
    hipLaunchKernelGGL(k_xtab, dim3(std::min(w.ngroups, 4096u)), dim3(64), 0, s, w);
    hipLaunchKernelGGL(k_walk<true>, dim3(w.nbig), dim3(64), 0, s, w);
    hipLaunchKernelGGL(k_xmark, dim3((w.ngroups + DL - 1) / DL), dim3(DL), 0, s, w);
  }
}
// ---- Few small updates, ranked: every position's chain step in parallel (k_wlen: one lane per
// byte over the whole chip), then in one workgroup per update the first n positions of each
// section's chain from its first struct are found by pointer doubling in LDS (k_wrank). The result
// is the exact walk's (the same step function from the same start), without its latency: a
// wavefront walking a 9 KB per-op doc state struct by struct (k_wdecode's chains and their
// settling) took 0.5-0.8 ms, one struct step being ~1 000 dependent instructions on one SIMD.
// A workgroup takes WL_SPAN positions: those whose info byte names no struct kind (ref > 10: no
// struct parses there, chain_len's 0) are settled by one byte test; those naming a rare kind
// (JSON, Binary, Embed, Format, Doc) are left unevaluated (WL_LATER: k_wrank sizes them all when a
// chain reaches one); the rest are gathered in LDS and sized by full wavefronts (the sizer is
// VALU-bound, ~1 500 instructions a position: a wavefront with a few live lanes costs as much as a
// full one). The common kinds — GC, Deleted, String, Type, Any, Skip — are 34 of the 256 byte
// values (ref <= 10: 88).
constexpr uint32_t WL_SPAN = 1024;
constexpr uint16_t WL_LATER = 0xFFFFu;  // (a length is at most 16 384)
__device__ __forceinline__ uint32_t wl_class(uint32_t info) {  // 0: no struct, 1: common kind, 2: rare kind
  const uint32_t ref = info & 31u;
  if (ref > REF_SKIP) return 0u;
  return ((1u << REF_GC) | (1u << REF_DELETED) | (1u << REF_STRING) | (1u << REF_TYPE) | (1u << REF_ANY) | (1u << REF_SKIP)) >> ref & 1u ? 1u : 2u;
}
__global__ __launch_bounds__(256) void k_wlen(Work w) {
  __shared__ uint16_t cand[WL_SPAN];
  __shared__ uint32_t ncand;
  const uint32_t j = blockIdx.y;
  const uint32_t u = w.ulist[w.nbig + j];
  const uint32_t ustart = w.uoff[u], L = w.ulen[u];
  const uint32_t k0 = blockIdx.x * WL_SPAN;
  if (k0 >= L || L > WD_MAX) return;
  const uint8_t* __restrict__ b = win_bytes(w, upd_win(w, u));
  uint16_t* __restrict__ out = w.wlen + (size_t)j * WD_MAX;
  if (threadIdx.x == 0) ncand = 0;
  __syncthreads();
  for (uint32_t k = k0 + threadIdx.x; k < min(L, k0 + WL_SPAN); k += 256) {
    const uint32_t c = wl_class(b[ustart + k]);
    if (c == 1u) cand[atomicAdd(&ncand, 1u)] = (uint16_t)(k - k0);
    else out[k] = c ? WL_LATER : 0;
  }
  __syncthreads();
  const uint32_t nc = ncand;
  for (uint32_t i = threadIdx.x; i < nc; i += 256) {
    const uint32_t k = k0 + cand[i];
    out[k] = (uint16_t)chain_len(GlobalSrc{b}, b, ustart + k, ustart + L);
  }
}
constexpr uint32_t WR_LANES = 1024;
constexpr uint16_t WR_INF = 0xFFFFu;
// k_wrank's LDS for updates of at most `cap` bytes: the two jump tables and the distances (u16,
// cap + 3 entries each), then the struct-start bitmap. Sized to the batch's longest small update
// (Work::small_max), not to WD_MAX: at 16 KiB a workgroup takes 100 KB and one fits a CU; a
// replica update of 11 KB takes 67 KB, and two share a CU.
__host__ __device__ constexpr uint32_t wr_tab(uint32_t cap) { return (cap + 3 + 3) & ~3u; }  // (u16 entries, 8-byte multiple)
__host__ __device__ constexpr size_t wr_lds(uint32_t cap) { return 3 * (size_t)wr_tab(cap) * 2 + ((cap + 63) / 64) * 8; }
__global__ __launch_bounds__(WR_LANES) void k_wrank(Work w, uint32_t cap) {
  // [L]: the update end, [L + 1]: no struct parses, [L + 2]: a position k_wlen left unevaluated
  extern __shared__ __attribute__((aligned(16))) uint64_t wr_smem[];
  uint16_t* const ja = (uint16_t*)wr_smem;
  uint16_t* const jb = ja + wr_tab(cap);
  uint16_t* const dist = jb + wr_tab(cap);
  uint64_t* const bits = (uint64_t*)(dist + wr_tab(cap));
  __shared__ uint32_t sh_base, sh_last;
  const uint32_t t = threadIdx.x, j = blockIdx.x;
  const uint32_t u = w.ulist[w.nbig + j];
  const uint32_t uw = upd_win(w, u);
  const uint8_t* __restrict__ b = win_bytes(w, uw);
  uint64_t* __restrict__ fbits = win_words(w.final_bits, uw);
  uint64_t* __restrict__ sbits = win_words(w.sec_bits, uw);
  const uint32_t ustart = w.uoff[u], L = w.ulen[u], uend = ustart + L;
  uint16_t* __restrict__ dl = w.wlen + (size_t)j * WD_MAX;
  bool sized = false;  // every position sized (the rare kinds too)
  uint32_t* err = &w.ctr->err;
  if (L > WD_MAX || L > cap) { if (t == 0) raise_err(err, ERR_CAPACITY); return; }  // (the layout never sends one)
  bool ok = true;
  uint32_t q = ustart;
  const uint32_t nsec = rd_vu(b, q, uend, ok);
  if (!ok || nsec > (uend - q) / 3 + 1) { if (t == 0) { raise_err(err, ERR_DECODE); w.dsstart[u] = NONE; } return; }
  if (t == 0) sh_base = atomicAdd(&w.ctr->nsections, nsec);
  const uint32_t nw = (L + 63) / 64;
  for (uint32_t k = t; k < nw; k += WR_LANES) bits[k] = 0;
  __syncthreads();
  const uint32_t sbase = sh_base;
  if (sbase + nsec > w.cap_sections) { if (t == 0) { raise_err(err, ERR_CAPACITY); w.dsstart[u] = NONE; } return; }
  bool fail = false;
  for (uint32_t sct = 0; sct < nsec; ++sct) {  // (q, n, fail: the same in every lane)
    const uint32_t n = rd_vu(b, q, uend, ok), client = rd_vu(b, q, uend, ok), clock = rd_vu(b, q, uend, ok);
    if (!ok || n > uend - q) { if (t == 0) raise_err(err, ERR_DECODE); fail = true; break; }
    if (t == 0) {
      Section sec;
      sec.upd = u; sec.n = n; sec.client = client; sec.clock = clock;
      sec.first_pos = n ? q : NONE; sec.cidx = NONE; sec.first_idx = NONE; sec.pad = 0;
      w.sections[sbase + sct] = sec;
      if (n) atomicOr((unsigned long long*)&sbits[q >> 6], 1ull << (q & 63));
    }
    if (!n) continue;
  rank:
    // jump tables: ja = one chain step (the end, "no struct" and "not sized" are sinks)
    const uint32_t q1 = q - ustart;
    for (uint32_t i = t; i < L + 3; i += WR_LANES) {
      uint32_t x = i;
      if (i < L) { const uint32_t d = dl[i]; x = d == WL_LATER ? L + 2 : !d ? L + 1 : min(i + d, L); }
      ja[i] = (uint16_t)x;
      dist[i] = i == q1 ? 0 : WR_INF;
    }
    __syncthreads();
    // doubling: in the round of step 2^k every position at distance < 2^k marks the one 2^k steps
    // on (distances below n only), then the table advances to 2^(k+1) steps. The chain's positions
    // increase, so each distance names one position; a sink reached below n is a struct missing.
    uint16_t *A = ja, *B = jb;
    for (uint32_t step = 1; step < n; step <<= 1) {
      for (uint32_t i = t; i < L; i += WR_LANES) {
        const uint32_t dv = dist[i];
        if (dv < step && dv + step < n) dist[A[i]] = (uint16_t)(dv + step);
      }
      __syncthreads();
      if (2 * step < n) {
        for (uint32_t i = t; i < L + 3; i += WR_LANES) B[i] = A[A[i]];
        __syncthreads();
        uint16_t* x = A; A = B; B = x;
      }
    }
    // the section's structs: the positions at distance < n; the last one's end starts the next
    if (t == 0) sh_last = NONE;
    __syncthreads();
    for (uint32_t i = t; i < L; i += WR_LANES)
      if (dist[i] == n - 1) sh_last = i;
    __syncthreads();
    const uint32_t last = sh_last;
    if (!sized && (dist[L + 2] != WR_INF || (last != NONE && dl[last] == WL_LATER))) {
      // the chain reaches a rare struct kind: size every position left unevaluated, rank again
      for (uint32_t i = t; i < L; i += WR_LANES)
        if (dl[i] == WL_LATER) dl[i] = (uint16_t)chain_len(GlobalSrc{b}, b, ustart + i, uend);
      sized = true;
      __syncthreads();
      goto rank;
    }
    for (uint32_t k = t; k < nw; k += WR_LANES) {
      uint64_t m = 0;
      for (uint32_t x = 0; x < 64 && k * 64 + x < L; ++x) m |= (uint64_t)(dist[k * 64 + x] < n) << x;
      bits[k] |= m;
    }
    __syncthreads();
    const bool sunk = dist[L] != WR_INF || dist[L + 1] != WR_INF;
    if (!sunk && last != NONE && dl[last]) {
      q = ustart + last + dl[last];
    } else {
      // a struct missing (malformed input): the exact walk, which reports where
      if (t == 0) {
        uint32_t x = q;
        for (uint32_t k = 0; k < n; ++k) {
          if (x >= uend) { raise_err(err, ERR_DECODE); w.ctr->err_info = x; break; }
          const uint32_t d = dl[x - ustart];
          if (!d) { raise_err(err, ERR_DECODE); w.ctr->err_info = x; break; }
          x += d;
        }
      }
      fail = true;
      break;
    }
    __syncthreads();  // (the tables are rebuilt for the next section)
  }
  __syncthreads();
  if (t == 0) {
    w.usec_start[u] = sbase;
    w.usec_n[u] = nsec;
    w.dsstart[u] = fail ? NONE : q;
    if (w.dbg) atomicAdd(&w.dbg[fail ? 5 : 3], 1ull);  // (YCRDT_DEBUG_DECODE: counted as the wave path's)
  }
  for (uint32_t k = t; k < nw; k += WR_LANES) fbits[(ustart >> 6) + k] = bits[k];
}

bool wave_decode(const Work& w) {
  // one lane per update when there are enough updates to fill wavefronts, else the ranked path;
  // YCRDT_DIRECT_WAVE=1 / 0 forces one (read per merge: tests switch it)
  const char* wd = getenv("YCRDT_DIRECT_WAVE");
  const bool lane_direct = wd && (wd[0] == '1' || wd[0] == '0') ? wd[0] == '0' : w.nsmall >= WD_LANE_MIN;
  return w.nsmall && !lane_direct;
}
void launch_direct(const Work& w, hipStream_t s) {
  // YCRDT_WDECODE=settle: the wavefront-per-update chains of k_wdecode instead of the ranking
  const char* wm = getenv("YCRDT_WDECODE");
  // (a split decode's share may take this path where the whole batch did not: no rank tables)
  if (wave_decode(w) && ((wm && !strcmp(wm, "settle")) || !w.wlen)) hipLaunchKernelGGL(k_wdecode, dim3(w.nsmall), dim3(64), 0, s, w);
  else if (wave_decode(w)) {
    const uint32_t cap = std::min(std::max(w.small_max, 1u), WD_MAX);
    static const bool lds_set = [] {  // (dynamic LDS past 64 KB: up to the WD_MAX table set)
      const bool r = hipFuncSetAttribute((const void*)k_wrank, hipFuncAttributeMaxDynamicSharedMemorySize, (int)wr_lds(WD_MAX)) == hipSuccess;
      if (!r) (void)hipGetLastError();
      return r;
    }();
    (void)lds_set;
    hipLaunchKernelGGL(k_wlen, dim3((cap + WL_SPAN - 1) / WL_SPAN, w.nsmall), dim3(256), 0, s, w);
    hipLaunchKernelGGL(k_wrank, dim3(w.nsmall), dim3(WR_LANES), wr_lds(cap), s, w, cap);
  } else if (w.nsmall) {
    // (one lane per update; 64 / 96 / 256 B windows and 2 / 4 / 8 lanes per update with a
    // wavefront-local chain sync were slower on C2: DESIGN.md §5.1)
    hipLaunchKernelGGL(k_direct<DW>, dim3((w.nsmall + DL - 1) / DL), dim3(DL), 0, s, w);
  }
}

// --------------------------------------------------------------------------- 3. struct positions
__global__ void k_popc(const uint64_t* __restrict__ bits, uint32_t* __restrict__ cnt, uint32_t nwords) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nwords) cnt[i] = (uint32_t)__popcll(bits[i]);
  else if (i == nwords) cnt[i] = 0;
}
// Dense positions of the set bits. A workgroup's 256 words stage their positions in LDS (each
// lane writes its word's bits at its prefix offset) and the workgroup stores them as one
// contiguous run: coalesced stores instead of every lane storing its ~5 positions at its own
// offset, one divergent store per bit of the word with the most.
constexpr uint32_t SCAT_LDS = 4096;
__global__ __launch_bounds__(256) void k_scatter_pos(const uint64_t* __restrict__ bits, const uint32_t* __restrict__ pre, uint32_t nwords,
                                                     uint32_t* __restrict__ out, uint32_t cap, uint32_t* err, uint8_t* __restrict__ swin,
                                                     uint32_t shift) {
  __shared__ uint32_t buf[SCAT_LDS];
  // a fixed grid walks the 256-word tiles (the per-tile work is small: tens of thousands of
  // short workgroups were dispatch-bound, 1.2 ms for C2 x 112)
  const uint32_t ntiles = (nwords + 255) / 256;
  for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint32_t i0 = tile * 256, i = i0 + threadIdx.x;
    const uint32_t iend = min(i0 + 256, nwords);
    const uint32_t base = pre[i0], total = pre[iend] - base;
    if (base + total > cap) {
      if (threadIdx.x == 0) raise_err(err, ERR_CAPACITY);
      return;  // (uniform across the workgroup: no barrier left behind)
    }
    uint64_t x = i < nwords ? bits[i] : 0ull;
    uint32_t k = i < nwords ? pre[i] : 0u;
    // positions within the window; a multi-window batch records the window (a tile's 256 words
    // never straddle a window: windows are 2^14 words or more)
    const uint64_t wmask = (1ull << shift) - 1;
    if (swin) {
      const uint8_t wn = (uint8_t)(((uint64_t)i0 * 64) >> shift);
      for (uint32_t t = threadIdx.x; t < total; t += 256) swin[base + t] = wn;
    }
    const uint32_t rel = (uint32_t)(((uint64_t)i * 64) & wmask);
    if (total > SCAT_LDS) {  // a dense stretch: every lane stores its own positions
      for (; x; x &= x - 1) out[k++] = rel + (uint32_t)__ffsll((long long)x) - 1;
      continue;
    }
    for (k -= base; x; x &= x - 1) buf[k++] = rel + (uint32_t)__ffsll((long long)x) - 1;
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < total; t += 256) out[base + t] = buf[t];
    __syncthreads();  // buf is reused by the next tile
  }
}

__device__ __forceinline__ uint32_t rank_incl(const uint64_t* __restrict__ bits, const uint32_t* __restrict__ pre, uint32_t p) {
  return pre[p >> 6] + (uint32_t)__popcll(bits[p >> 6] & (((2ull << (p & 63)) - 1)));  // bits <= p
}
__device__ __forceinline__ void section_rank_at(const Work& w, uint32_t i) {
  Section* sec = &w.sections[i];
  if (sec->n == 0) return;
  const uint32_t p = sec->first_pos, uw = upd_win(w, sec->upd);  // (bitmap words and prefixes of its window)
  const uint64_t* fbits = win_words(w.final_bits, uw);
  if (!((fbits[p >> 6] >> (p & 63)) & 1ull)) { raise_err(&w.ctr->err, ERR_DECODE); return; }
  sec->first_idx = rank_incl(fbits, win_words(w.wcnt, uw), p) - 1;
  w.sec_sorted[rank_incl(win_words(w.sec_bits, uw), win_words(w.wsec, uw), p) - 1] = i;
  // the struct decode's bound and document, beside the section record (one dependent load fewer
  // per struct than update -> offsets)
  w.sec_uend[i] = w.uoff[sec->upd] + w.ulen[sec->upd];
  w.sec_doc[i] = doc_of_update(w, sec->upd);
}
__global__ void k_section_rank(Work w, uint32_t nsections) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nsections) section_rank_at(w, i);
}
// Small batches: both popcount prefixes in one workgroup and one launch (four launches otherwise):
// a lane sums the popcounts of a contiguous run of words, the run sums are scanned in LDS, each
// lane writes its run's prefixes (n = nwords + 1 entries; the last is the total).
constexpr uint32_t COUNT_LANES = 1024, COUNT_SMALL = COUNT_LANES * 16;
__global__ __launch_bounds__(COUNT_LANES) void k_count_small(const uint64_t* __restrict__ b0, uint32_t* __restrict__ o0,
                                                             const uint64_t* __restrict__ b1, uint32_t* __restrict__ o1, uint32_t nwords) {
  __shared__ uint32_t part[COUNT_LANES];
  const uint32_t t = threadIdx.x, n = nwords + 1, per = (n + COUNT_LANES - 1) / COUNT_LANES;
  const uint32_t a = min(n, t * per), e = min(n, a + per);
  for (int k = 0; k < 2; ++k) {
    const uint64_t* bits = k ? b1 : b0;
    uint32_t* out = k ? o1 : o0;
    uint32_t sum = 0;
    for (uint32_t i = a; i < e; ++i) sum += i < nwords ? (uint32_t)__popcll(bits[i]) : 0u;
    part[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < COUNT_LANES; off <<= 1) {
      const uint32_t v = t >= off ? part[t - off] : 0u;
      __syncthreads();
      part[t] += v;
      __syncthreads();
    }
    uint32_t run = part[t] - sum;
    for (uint32_t i = a; i < e; ++i) { out[i] = run; run += i < nwords ? (uint32_t)__popcll(bits[i]) : 0u; }
    __syncthreads();
  }
}

// before the count sync: struct / section-start counts (popcount prefix of the bitmaps)
void launch_struct_count(const Work& w, hipStream_t s) {
  const uint32_t nwords = (w.nbytes + 63) / 64;
  if (nwords + 1 <= COUNT_SMALL) {
    hipLaunchKernelGGL(k_count_small, dim3(1), dim3(COUNT_LANES), 0, s, w.final_bits, w.wcnt, w.sec_bits, w.wsec, nwords);
    return;
  }
  hipLaunchKernelGGL(k_popc, dim3(nwords / 256 + 1), dim3(256), 0, s, w.final_bits, w.scratch, nwords);
  scan_u32(w.tmp, w.tmp_bytes, w.scratch, w.wcnt, nwords + 1, s);
  hipLaunchKernelGGL(k_popc, dim3(nwords / 256 + 1), dim3(256), 0, s, w.sec_bits, w.scratch, nwords);
  scan_u32(w.tmp, w.tmp_bytes, w.scratch, w.wsec, nwords + 1, s);
}
// after it (the struct table is sized from the count): dense struct positions
void launch_struct_scatter(const Work& w, hipStream_t s) {
  const uint32_t nwords = (w.nbytes + 63) / 64;
  hipLaunchKernelGGL(k_scatter_pos, dim3(std::min<uint32_t>(nwords / 256 + 1, 4096)), dim3(256), 0, s, w.final_bits, w.wcnt, nwords, w.s_pos,
                     w.cap_structs, &w.ctr->err, w.nwin > 1 ? w.s_win : nullptr, w.win_shift);
}

// called once the section count is known on the host
void launch_section_clients(const Work& w, uint32_t nsections, hipStream_t s) {
  if (!nsections) return;
  hipLaunchKernelGGL(k_section_rank, dim3((nsections + 255) / 256), dim3(256), 0, s, w, nsections);
}

// --------------------------------------------------------------------------- 5. delete sets
__device__ __forceinline__ uint32_t nth_lane(uint64_t x, uint32_t n) {  // position of the n-th set bit
  for (uint32_t i = 0; i < n; ++i) x &= x - 1;
  return (uint32_t)__ffsll((long long)x) - 1;
}

__global__ __launch_bounds__(256) void k_ds_decode(Work w) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t u = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (u >= w.nupd) return;
  const uint32_t p0 = w.dsstart[u];
  if (p0 == NONE) return;
  if (w.dsp_b && w.dsp_b[u] != NONE) return;  // decoded grid-wide (k_dsp_*)
  const uint8_t* __restrict__ b = win_bytes(w, upd_win(w, u));
  const uint32_t end = w.uoff[u] + w.ulen[u];
  uint32_t* err = &w.ctr->err;
  enum { PH_N = 0, PH_CLIENT = 1, PH_NR = 2, PH_PAIRS = 3, PH_DONE = 4 };
  uint32_t phase = PH_N, nclients = 0, client = 0, pairs_left = 0, pend_clock = 0;
  // this update's private output region (every range needs >= 2 bytes): no shared counter
  const uint32_t obase0 = w.ds_region[u];
  const uint32_t oend = w.ds_region[u + 1];
  uint32_t obase = obase0;
  uint32_t carry_val = 0, carry_shift = 0, carry_bytes = 0;
  const uint64_t lt_mask = (1ull << lane) - 1;
  for (uint32_t base = p0; base < end && phase != PH_DONE; base += 64) {
    const uint32_t pos = base + lane;
    const bool valid = pos < end;
    const uint32_t byte = valid ? b[pos] : 0x80u;
    const uint64_t term = __ballot(valid && byte < 0x80u);
    const uint64_t below = term & lt_mask;
    const int start = below ? (64 - __clzll((long long)below)) : 0;  // first byte of my varint
    // gather the (<= 6) 7-bit groups of the varint ending at this lane
    uint32_t val = 0;
    for (int k = 0; k < 6; ++k) {
      const int src = start + k;
      const uint32_t bb = (uint32_t)__shfl((int)byte, src & 63);
      if (src <= (int)lane && 7 * k < 32) val |= (bb & 0x7fu) << (7 * k);
    }
    const uint32_t nb_here = lane - start + 1;
    if (start == 0 && carry_bytes) {
      val = carry_shift < 32 ? (carry_val | (val << carry_shift)) : carry_val;
    }
    const uint32_t nb_total = nb_here + (start == 0 ? carry_bytes : 0);
    if (__ballot(((term >> lane) & 1ull) && nb_total > 6)) { raise_err(err, ERR_DECODE); return; }
    const uint32_t prevval = (uint32_t)__shfl((int)val, (start - 1) & 63);
    const uint32_t myk = (uint32_t)__popcll(below);
    const uint32_t m = (uint32_t)__popcll(term);
    uint32_t vi = 0;
    while (vi < m && phase != PH_DONE) {
      if (phase == PH_PAIRS) {
        const uint32_t take = min(pairs_left, m - vi);
        const bool mine = ((term >> lane) & 1ull) && myk >= vi && myk < vi + take;
        const bool is_len = mine && ((pairs_left - (myk - vi)) & 1u);
        const uint64_t lm = __ballot(is_len);
        if (is_len) {
          const uint32_t idx = obase + (uint32_t)__popcll(lm & lt_mask);
          if (idx < oend) {
            DsRange r;
            r.client = client;
            r.clock = myk == vi ? pend_clock : prevval;
            r.len = val;
            r.upd = u;
            w.ds_tmp[idx] = r;
          } else raise_err(err, ERR_CAPACITY);
        }
        obase += (uint32_t)__popcll(lm);
        pairs_left -= take;
        vi += take;
        if (pairs_left & 1u) pend_clock = (uint32_t)__shfl((int)val, (int)nth_lane(term, vi - 1));
        if (pairs_left == 0) { --nclients; phase = nclients ? PH_CLIENT : PH_DONE; }
      } else {
        const uint32_t v = (uint32_t)__shfl((int)val, (int)nth_lane(term, vi));
        ++vi;
        if (phase == PH_N) { nclients = v; phase = v ? PH_CLIENT : PH_DONE; }
        else if (phase == PH_CLIENT) { client = v; phase = PH_NR; }
        else {  // PH_NR
          if (v > 0x7FFFFFFFu) { raise_err(err, ERR_DECODE); return; }
          pairs_left = 2 * v;
          if (v) phase = PH_PAIRS;
          else { --nclients; phase = nclients ? PH_CLIENT : PH_DONE; }
        }
      }
    }
    // partial varint at the end of the window carries into the next one
    const int lt = term ? 63 - __clzll((long long)term) : -1;
    const uint32_t nvalid = min(64u, end - base);
    if ((uint32_t)(lt + 1) < nvalid) {
      uint32_t partial = 0;
      for (int k = 0; k < 6; ++k) {
        const int src = lt + 1 + k;
        const uint32_t bb = (uint32_t)__shfl((int)byte, src & 63);
        if (src < (int)nvalid && 7 * k < 32) partial |= (bb & 0x7fu) << (7 * k);
      }
      const uint32_t nbp = nvalid - (uint32_t)(lt + 1);
      if (lt < 0 && carry_bytes) {
        if (carry_shift < 32) carry_val |= partial << carry_shift;
        carry_shift += 7 * nbp;
        carry_bytes += nbp;
      } else {
        carry_val = partial;
        carry_shift = 7 * nbp;
        carry_bytes = nbp;
      }
      if (carry_bytes > 6) { raise_err(err, ERR_DECODE); return; }
    } else {
      carry_bytes = 0;
      carry_val = 0;
      carry_shift = 0;
    }
  }
  if (phase != PH_DONE) raise_err(err, ERR_DECODE);  // truncated delete set
  if (lane == 0) {
    w.ds_count[u] = obase - obase0;
    if (obase - obase0 > DSA_WAVE) w.ds_biglist[atomicAdd(&w.ctr->ds_big, 1u)] = u;  // (k_units spreads the rest)
  }
}

// ---- Large delete sets, grid-wide. A delete set is a flat varuint stream (readDeleteSet, Y@11105:
// client blocks of {client, n, (clock, len) x n} behind a client count), so its k-th value ends at
// its k-th terminal byte (high bit clear). k_dsp_count counts the terminal bytes of every chunk's
// delete-set part (one wavefront per chunk, 16 bytes a lane), a scan numbers them, k_dsp_vals
// decodes every value where it ends (back to the previous terminal), k_dsp_headers walks the client
// blocks over the decoded values (one lane per update: a block costs two reads), and k_dsp_ranges
// writes every (clock, len) pair into the update's range region. One wavefront stepping 64 bytes at
// a time took 55 ms for the 156 MB C3 state as one update (crdt.js's full-state wire shape).
// Anything irregular — a varuint of more than 6 bytes, a truncated stream, a range count past
// 2^31, more than DSP_MAXBLK client blocks — leaves the update to the wavefront (k_ds_decode),
// which decodes and reports it exactly as before.
constexpr uint32_t DSP_MIN = 4096;  // delete sets of at least this many bytes (to the update end)
__device__ __forceinline__ bool dsp_applies(const Work& w, uint32_t u) {
  const uint32_t ds = w.dsstart[u];
  return ds != NONE && w.uoff[u] + w.ulen[u] - ds >= DSP_MIN;
}
// this lane's 16 bytes of chunk i: the terminal bytes inside the update's delete set (bit k: byte
// p + k), or 0 when the update is not on the grid path
__device__ __forceinline__ uint32_t dsp_terms(const Work& w, const Group& G, uint32_t lane, uint32_t& p) {
  const uint32_t u = G.upd;
  p = G.start + lane * 16;
  if (!dsp_applies(w, u)) return 0u;
  const uint32_t ds = w.dsstart[u];
  if (p >= G.end || p + 16 <= ds) return 0u;
  const uint4 v = *(const uint4*)(win_bytes(w, upd_win(w, u)) + p);  // (chunks are 64-byte aligned; the buffer is padded)
  const uint32_t x[4] = {v.x, v.y, v.z, v.w};
  uint32_t m = 0;
  for (int j = 0; j < 4; ++j)
    for (int k = 0; k < 4; ++k) m |= ((~x[j] >> (8 * k + 7)) & 1u) << (4 * j + k);
  if (ds > p) m &= ~0u << (ds - p);
  if (G.end < p + 16) m &= (1u << (G.end - p)) - 1u;
  return m;
}
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, uint32_t lane, uint32_t& total) {
  uint32_t incl = x;
  for (uint32_t off = 1; off < 64; off <<= 1) {
    const uint32_t v = __shfl_up(incl, off);
    if (lane >= off) incl += v;
  }
  total = __shfl(incl, 63);
  return incl - x;
}
// The chunks the grid path visits: those of the large delete sets only, numbered by one
// workgroup (per big update: its delete set's chunks, scanned). The three grid kernels stride over
// them with a fixed grid: launched over every chunk of every large update, the passes cost a C2
// batch (112 base snapshots, no large delete set) a millisecond beside its struct decode.
constexpr uint32_t DSP_PLAN_LANES = 1024, DSP_GRID = 1024;
__global__ __launch_bounds__(DSP_PLAN_LANES) void k_dsp_plan(Work w) {
  __shared__ uint32_t part[DSP_PLAN_LANES];
  for (uint32_t bi = threadIdx.x; bi <= w.nbig; bi += DSP_PLAN_LANES) {
    uint32_t c = 0;
    if (bi < w.nbig) {
      const uint32_t u = w.ulist[bi];
      if (dsp_applies(w, u)) {
        const uint32_t CH = w.schunk;
        c = (w.ulen[u] + CH - 1) / CH - (w.dsstart[u] - w.uoff[u]) / CH;
      }
    }
    w.dsp_gb[bi] = c;
  }
  __syncthreads();
  block_scan_u32<DSP_PLAN_LANES>(w.dsp_gb, w.dsp_gb, w.nbig + 1, part);
}
// the t-th chunk of the plan: its group index (NONE past the end)
__device__ __forceinline__ uint32_t dsp_group(const Work& w, uint32_t t) {
  if (t >= w.dsp_gb[w.nbig]) return NONE;
  uint32_t lo = 0, hi = w.nbig;  // the last big update whose first planned chunk is <= t
  while (hi - lo > 1) { const uint32_t m = (lo + hi) >> 1; if (w.dsp_gb[m] <= t) lo = m; else hi = m; }
  const uint32_t u = w.ulist[lo];
  return w.ugroup[u] + (w.dsstart[u] - w.uoff[u]) / w.schunk + (t - w.dsp_gb[lo]);
}
__global__ __launch_bounds__(256) void k_dsp_count(Work w) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;; t += gridDim.x * (blockDim.x >> 6)) {
    const uint32_t i = dsp_group(w, t);
    if (i == NONE) return;  // (whole wavefronts)
    const Group G = w.groups[i];
    uint32_t p;
    const uint32_t m = dsp_terms(w, G, lane, p);
    uint32_t total;
    wave_excl_scan((uint32_t)__popc(m), lane, total);
    if (lane == 0) w.dsp_cnt[i] = total;
  }
}
// the value index of this lane's first terminal: terminals before its chunk in the update's delete
// set, then before its lane
__device__ __forceinline__ uint32_t dsp_first_index(const Work& w, const Group& G, uint32_t i, uint32_t m, uint32_t lane) {
  const uint32_t u = G.upd;
  const uint32_t g0 = w.ugroup[u] + (w.dsstart[u] - w.uoff[u]) / w.schunk;
  uint32_t total;
  const uint32_t ex = wave_excl_scan((uint32_t)__popc(m), lane, total);
  return w.dsp_pre[i] - w.dsp_pre[g0] + ex;
}
__device__ __forceinline__ void dsp_vals_group(const Work& w, uint32_t i, uint32_t lane) {
  const Group G = w.groups[i];
  uint32_t p;
  uint32_t m = dsp_terms(w, G, lane, p);
  if (!__ballot(m != 0)) return;
  const uint32_t u = G.upd, ds = w.dsstart[u];
  uint32_t v = dsp_first_index(w, G, i, m, lane);
  const uint8_t* __restrict__ b = win_bytes(w, upd_win(w, u));
  uint32_t* __restrict__ vals = w.dsp_val + 2ull * w.ds_region[u];
  for (; m; m &= m - 1, ++v) {
    const uint32_t e = p + (uint32_t)__ffs(m) - 1;  // the value's last byte
    uint32_t q = e, n = 1;
    while (q > ds && b[q - 1] >= 0x80u && n <= 6) { --q; ++n; }
    if (n > 6) { w.dsp_fail[u] = 1u; return; }  // a varuint of more than 6 bytes (the wavefront reports it)
    uint32_t x = 0;
    for (uint32_t k = 0; k < n && 7 * k < 32; ++k) x |= (uint32_t)(b[q + k] & 0x7Fu) << (7 * k);
    vals[v] = x;
  }
}
__global__ __launch_bounds__(256) void k_dsp_vals(Work w) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;; t += gridDim.x * (blockDim.x >> 6)) {
    const uint32_t i = dsp_group(w, t);
    if (i == NONE) return;
    dsp_vals_group(w, i, lane);
  }
}
// The client blocks of a large delete set without hopping from header to header in one lane (a
// full state's 1 001 blocks were 0.37 ms of dependent loads, on the path of every apply into a large
// doc: crdt.js's sync reply carries the peer's whole delete set). The header after the one at value
// index k is k + 2 + 2 (its run count); k_dsh_jump takes 32 such steps from EVERY value index at once
// (garbage where k is no header, never read), k_dsh_base strides the real chain 32 headers a step
// from value 1, k_dsh_fill walks each stride's 32 headers and writes their blocks, k_dsh_final
// publishes them. Every check of the lane-serial walk (k_dsp_headers) is made on the real chain;
// where one fails the update is left to the wavefront decoder, as there.
__device__ __forceinline__ bool dsh_update(const Work& w, uint32_t bi, uint32_t& u, uint64_t& total, const uint32_t*& vals) {
  u = w.ulist[bi];
  if (!dsp_applies(w, u) || w.dsp_fail[u]) return false;
  const uint32_t CH = w.schunk;
  const uint32_t g0 = w.ugroup[u] + (w.dsstart[u] - w.uoff[u]) / CH, gl = w.ugroup[u] + (w.ulen[u] + CH - 1) / CH;
  total = w.dsp_pre[gl] - w.dsp_pre[g0];
  vals = w.dsp_val + 2ull * w.ds_region[u];
  // (a delete set of few client blocks — C2's snapshots hold one — is walked by k_dsp_headers: the
  // jumps from every value index cost more than a short walk, and they compete with the struct decode)
  return total >= 1 && vals[0] > DSH_MIN_BLOCKS;
}
__global__ __launch_bounds__(256) void k_dsh_jump(Work w) {
  const uint32_t bi = blockIdx.y;
  uint32_t u;
  uint64_t total;
  const uint32_t* vals;
  if (!dsh_update(w, bi, u, total, vals)) return;
  uint32_t* __restrict__ J = w.dsp_j + 2ull * w.ds_region[u];
  uint32_t* __restrict__ S = w.dsp_js + 2ull * w.ds_region[u];
  for (uint64_t i = 1 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t k = i;
    uint32_t sum = 0;
    for (uint32_t h = 0; h < DSH_STRIDE; ++h) {
      if (k + 2 > total) { k = NONE; break; }
      const uint32_t nr = vals[k + 1];
      if (nr > 0x7FFFFFFFu || k + 2 + 2ull * nr > total) { k = NONE; break; }
      sum += nr;
      k += 2 + 2ull * nr;
    }
    J[i] = (uint32_t)k;
    S[i] = sum;
  }
}
__global__ void k_dsh_base(Work w) {
  const uint32_t bi = blockIdx.x * blockDim.x + threadIdx.x;
  if (bi >= w.nbig) return;
  uint2* __restrict__ H = w.dsp_h + (size_t)bi * (DSH_SEG + 1);
  H[DSH_SEG] = make_uint2(1u, 0u);  // (failed until the chain is strided)
  uint32_t u;
  uint64_t total;
  const uint32_t* vals;
  if (!dsh_update(w, bi, u, total, vals)) return;
  const uint32_t nb = vals[0];
  if (nb > DSP_MAXBLK) return;  // (k_dsp_headers gives up there too: the wavefront decodes it)
  const uint32_t* __restrict__ J = w.dsp_j + 2ull * w.ds_region[u];
  const uint32_t* __restrict__ S = w.dsp_js + 2ull * w.ds_region[u];
  const uint32_t nseg = (nb + DSH_STRIDE - 1) / DSH_STRIDE;
  uint32_t k = 1, off = 0;
  for (uint32_t sg = 0; sg < nseg; ++sg) {
    H[sg] = make_uint2(k, off);
    if (sg + 1 < nseg) {  // a full stride of 32 headers: its jump must be valid
      if (k >= total) return;
      const uint32_t j = J[k];
      if (j == NONE) return;
      off += S[k];
      k = j;
    }
  }
  H[DSH_SEG] = make_uint2(0u, 0u);
}
__global__ void k_dsh_fill(Work w) {
  const uint32_t bi = blockIdx.y, sg = threadIdx.x + blockIdx.x * blockDim.x;
  uint32_t u;
  uint64_t total;
  const uint32_t* vals;
  if (!dsh_update(w, bi, u, total, vals)) return;
  uint2* __restrict__ H = w.dsp_h + (size_t)bi * (DSH_SEG + 1);
  const uint32_t nb = vals[0];
  if (nb > DSP_MAXBLK || sg * DSH_STRIDE >= nb || H[DSH_SEG].x) return;
  uint4* __restrict__ blk = w.dsp_blk + (size_t)bi * DSP_MAXBLK;
  uint64_t k = H[sg].x;
  uint32_t off = H[sg].y;
  for (uint32_t c = sg * DSH_STRIDE; c < min(nb, (sg + 1) * DSH_STRIDE); ++c) {
    if (k + 2 > total) { atomicOr(&H[DSH_SEG].x, 1u); return; }
    const uint32_t client = vals[k], nr = vals[k + 1];
    if (nr > 0x7FFFFFFFu || k + 2 + 2ull * nr > total) { atomicOr(&H[DSH_SEG].x, 1u); return; }
    blk[c] = make_uint4((uint32_t)k, client, nr, off);
    off += nr;
    k += 2 + 2ull * nr;
  }
  if (min(nb, (sg + 1) * DSH_STRIDE) == nb) H[DSH_SEG].y = off;  // (the last stride: every run)
}
__global__ void k_dsh_final(Work w) {
  const uint32_t bi = blockIdx.x * blockDim.x + threadIdx.x;
  if (bi >= w.nbig) return;
  uint32_t u;
  uint64_t total;
  const uint32_t* vals;
  if (!dsh_update(w, bi, u, total, vals)) return;
  const uint2 f = w.dsp_h[(size_t)bi * (DSH_SEG + 1) + DSH_SEG];
  if (f.x) return;  // the wavefront decodes it (and reports what is wrong)
  w.dsp_nb[bi] = vals[0];
  w.ds_count[u] = f.y;
  if (f.y > DSA_WAVE) w.ds_biglist[atomicAdd(&w.ctr->ds_big, 1u)] = u;
  w.dsp_b[u] = bi;
}
__global__ void k_dsp_headers(Work w, uint32_t jumps) {
  const uint32_t bi = blockIdx.x * blockDim.x + threadIdx.x;
  if (bi >= w.nbig) return;
  const uint32_t u = w.ulist[bi];
  if (!dsp_applies(w, u) || w.dsp_fail[u]) return;
  if (jumps) {  // (the k_dsh_* kernels take the delete sets of many client blocks)
    const uint32_t CH = w.schunk;
    const uint32_t g0 = w.ugroup[u] + (w.dsstart[u] - w.uoff[u]) / CH, gl = w.ugroup[u] + (w.ulen[u] + CH - 1) / CH;
    if (w.dsp_pre[gl] - w.dsp_pre[g0] >= 1 && w.dsp_val[2ull * w.ds_region[u]] > DSH_MIN_BLOCKS) return;
  }
  const uint32_t CH = w.schunk;
  const uint32_t g0 = w.ugroup[u] + (w.dsstart[u] - w.uoff[u]) / CH, gl = w.ugroup[u] + (w.ulen[u] + CH - 1) / CH;
  const uint64_t total = w.dsp_pre[gl] - w.dsp_pre[g0];
  const uint32_t* __restrict__ vals = w.dsp_val + 2ull * w.ds_region[u];
  uint4* __restrict__ blk = w.dsp_blk + (size_t)bi * DSP_MAXBLK;
  if (total < 1) return;
  const uint32_t ncl = vals[0];
  uint64_t k = 1;
  uint32_t off = 0, c = 0;
  for (; c < ncl; ++c) {
    if (c >= DSP_MAXBLK || k + 2 > total) return;  // (truncated: the wavefront reports it)
    const uint32_t client = vals[k], nr = vals[k + 1];
    if (nr > 0x7FFFFFFFu || k + 2 + 2ull * nr > total) return;
    blk[c] = make_uint4((uint32_t)k, client, nr, off);
    off += nr;
    k += 2 + 2ull * nr;
  }
  w.dsp_nb[bi] = c;
  w.ds_count[u] = off;
  if (off > DSA_WAVE) w.ds_biglist[atomicAdd(&w.ctr->ds_big, 1u)] = u;
  w.dsp_b[u] = bi;
}
__device__ __forceinline__ void dsp_ranges_group(const Work& w, uint32_t i, uint32_t lane) {
  const Group G = w.groups[i];
  const uint32_t u = G.upd;
  const uint32_t bi = w.dsp_b[u];
  if (bi == NONE) return;
  uint32_t p;
  uint32_t m = dsp_terms(w, G, lane, p);
  uint32_t v = dsp_first_index(w, G, i, m, lane);
  if (!m) return;
  const uint32_t nb = w.dsp_nb[bi];
  const uint4* __restrict__ blk = w.dsp_blk + (size_t)bi * DSP_MAXBLK;
  const uint32_t* __restrict__ vals = w.dsp_val + 2ull * w.ds_region[u];
  DsRange* __restrict__ out = w.ds_tmp + w.ds_region[u];
  // the block of the lane's first value (the last block starting at or before it), then onwards
  uint32_t lo = 0, hi = nb;
  while (lo < hi) { const uint32_t mid = (lo + hi) >> 1; if (blk[mid].x <= v) lo = mid + 1; else hi = mid; }
  if (lo == 0) { if (nb == 0) return; lo = 1; }  // (value 0, the client count: no block)
  uint32_t c = lo - 1;
  uint4 B = blk[c];
  for (; m; m &= m - 1, ++v) {
    while (c + 1 < nb && blk[c + 1].x <= v) B = blk[++c];
    if (v < B.x + 2) continue;  // the block's client / count
    const uint32_t rel = v - B.x - 2;
    if (rel >= 2 * B.z) continue;  // past the last block: bytes Yjs never reads
    if (!(rel & 1u)) continue;  // a clock: written with its length
    DsRange r;
    r.client = B.y;
    r.clock = vals[v - 1];
    r.len = vals[v];
    r.upd = u;
    out[B.w + (rel >> 1)] = r;
  }
}
__global__ __launch_bounds__(256) void k_dsp_ranges(Work w) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;; t += gridDim.x * (blockDim.x >> 6)) {
    const uint32_t i = dsp_group(w, t);
    if (i == NONE) return;
    dsp_ranges_group(w, i, lane);
  }
}
void launch_ds_grid(const Work& w, hipStream_t s) {
  if (!w.nbig || !w.dsp_cnt || w.nbig + 1 > DSP_PLAN_LANES * 16) return;
  // YCRDT_DS_GRID=0: every delete set on the wavefront (read per merge: tests compare the two)
  if (const char* g = getenv("YCRDT_DS_GRID")) if (g[0] == '0') return;
  hipMemsetAsync(w.dsp_cnt, 0, sizeof(uint32_t) * ((size_t)w.ngroups + 1), s);
  hipLaunchKernelGGL(k_dsp_plan, dim3(1), dim3(DSP_PLAN_LANES), 0, s, w);
  hipLaunchKernelGGL(k_dsp_count, dim3(DSP_GRID), dim3(256), 0, s, w);
  scan_u32(w.tmp, w.tmp_bytes, w.dsp_cnt, w.dsp_pre, (uint64_t)w.ngroups + 1, s);
  hipLaunchKernelGGL(k_dsp_vals, dim3(DSP_GRID), dim3(256), 0, s, w);
  const uint32_t jumps = w.dsp_j && !env_off("YCRDT_DS_JUMP") ? 1u : 0u;  // (YCRDT_DS_JUMP=0: the lane-serial walk, A/B)
  hipLaunchKernelGGL(k_dsp_headers, dim3(w.nbig / 64 + 1), dim3(64), 0, s, w, jumps);
  if (jumps) {
    hipLaunchKernelGGL(k_dsh_jump, dim3(w.dsh_grid, w.nbig), dim3(256), 0, s, w);
    hipLaunchKernelGGL(k_dsh_base, dim3(w.nbig / 64 + 1), dim3(64), 0, s, w);
    hipLaunchKernelGGL(k_dsh_fill, dim3(1, w.nbig), dim3(DSH_SEG), 0, s, w);
    hipLaunchKernelGGL(k_dsh_final, dim3(w.nbig / 64 + 1), dim3(64), 0, s, w);
  }
  hipLaunchKernelGGL(k_dsp_ranges, dim3(DSP_GRID), dim3(256), 0, s, w);
}

__device__ __forceinline__ void ds_bound_at(const Work& w, uint32_t u) {  // region size per update: (delete-set bytes + 1) / 2
  if (u == w.nupd) {
    w.scratch[u] = 0; w.ds_count[u] = 0;
    w.ctr->nstructs = w.wcnt[(w.nbytes + 63) / 64];  // launch_struct_count's total (no copy launch)
    return;
  }
  const uint32_t st = w.dsstart[u];
  w.scratch[u] = st == NONE ? 0 : (w.uoff[u] + w.ulen[u] - st + 1) / 2;
  w.ds_count[u] = 0;
  // Sections out of strictly descending client order (Yjs never writes them; its readers accept
  // them): mergeUpdates / diffUpdate take the serial loop (ctr->noncanon, yc_lazy.hip), and
  // applyUpdate keeps only the LAST section of a client (readClientsStructRefs' Map.set, Y@19286):
  // an earlier one is marked superseded (pad = 1) and its structs decode as Skips
  const uint32_t a = w.usec_start[u], b = a + w.usec_n[u];
  if (u == w.upre) return;  // a doc state decoded by its marks: its encode wrote descending clients
  bool canon = true;
  // (eight sections' clients per round of loads: a full state's 1 001 sections one dependent load
  // at a time held this pass for 0.13 ms)
  uint32_t prev = b > a ? w.sections[a].client : 0u;
  for (uint32_t i0 = a + 1; i0 < b && canon; i0 += 8) {
    uint32_t c[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = i0 + k < b ? w.sections[i0 + k].client : 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (i0 + k < b) { canon = canon && c[k] < prev; prev = c[k]; }
  }
  if (canon) return;
  w.ctr->noncanon = 1;
  if (w.lazy) return;
  for (uint32_t i = a; i < b; ++i)
    for (uint32_t j = i + 1; j < b; ++j)
      if (w.sections[j].client == w.sections[i].client) { w.sections[i].pad = 1; break; }
}
__global__ void k_ds_bound(Work w) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u <= w.nupd) ds_bound_at(w, u);
}
__global__ void k_ds_compact(Work w) {  // one wave per update: region -> dense ds[]
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t u = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (u >= w.nupd) return;
  const uint32_t n = w.ds_count[u], src = w.ds_region[u], dst = w.ds_dense_off[u];
  for (uint32_t i = lane; i < n; i += 64) w.ds[dst + i] = w.ds_tmp[src + i];
  if (u == w.nupd - 1 && lane == 0) w.ctr->nds = dst + n;
}

// delete-set regions (before the count sync: the range arrays are sized from their total)
void launch_ds_bound(const Work& w, hipStream_t s) {
  if (w.nupd == 0) return;
  hipLaunchKernelGGL(k_ds_bound, dim3(w.nupd / 256 + 1), dim3(256), 0, s, w);
  scan_u32(w.tmp, w.tmp_bytes, w.scratch, w.ds_region, w.nupd + 1, s);
  hipMemcpyAsync(&w.ctr->ds_region, w.ds_region + w.nupd, sizeof(uint32_t), hipMemcpyDeviceToDevice, s);
}
// Small batches: the struct / section-start counts (k_count_small), the delete-set region bounds
// and their scan, and the region total, in ONE workgroup launch (four launches otherwise)
__global__ __launch_bounds__(COUNT_LANES) void k_count_ds_small(Work w, uint32_t nwords) {
  __shared__ uint32_t part[COUNT_LANES];
  const uint32_t t = threadIdx.x, n = nwords + 1, per = (n + COUNT_LANES - 1) / COUNT_LANES;
  const uint32_t a = min(n, t * per), e = min(n, a + per);
  for (int k = 0; k < 2; ++k) {
    const uint64_t* bits = k ? w.sec_bits : w.final_bits;
    uint32_t* out = k ? w.wsec : w.wcnt;
    uint32_t sum = 0;
    for (uint32_t i = a; i < e; ++i) sum += i < nwords ? (uint32_t)__popcll(bits[i]) : 0u;
    part[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < COUNT_LANES; off <<= 1) {
      const uint32_t v = t >= off ? part[t - off] : 0u;
      __syncthreads();
      part[t] += v;
      __syncthreads();
    }
    uint32_t run = part[t] - sum;
    for (uint32_t i = a; i < e; ++i) { out[i] = run; run += i < nwords ? (uint32_t)__popcll(bits[i]) : 0u; }
    __syncthreads();
  }
  for (uint32_t u = t; u <= w.nupd; u += COUNT_LANES) ds_bound_at(w, u);
  __syncthreads();
  block_scan_u32<COUNT_LANES>(w.scratch, w.ds_region, w.nupd + 1, part);
  if (t == 0) w.ctr->ds_region = w.ds_region[w.nupd];
}
bool count_ds_small(const Work& w, hipStream_t s) {
  const uint32_t nwords = (w.nbytes + 63) / 64;
  if (env_off("YCRDT_DECODE_SMALL") || !w.nupd || nwords + 1 > COUNT_SMALL || w.nupd + 1 > COUNT_SMALL) return false;
  hipLaunchKernelGGL(k_count_ds_small, dim3(1), dim3(COUNT_LANES), 0, s, w, nwords);
  return true;
}
// the integrate path reads the ranges in their per-update regions (k_ds_apply); mergeUpdates /
// diffUpdate (lazy) sort them, so there they are compacted into the dense table
void launch_ds_decode(const Work& w, hipStream_t s) {
  if (w.nupd == 0) return;
  launch_ds_grid(w, s);
  hipLaunchKernelGGL(k_ds_decode, dim3((w.nupd + 3) / 4), dim3(256), 0, s, w);
  if (!w.lazy) return;
  scan_u32(w.tmp, w.tmp_bytes, w.ds_count, w.ds_dense_off, w.nupd + 1, s);
  hipLaunchKernelGGL(k_ds_compact, dim3((w.nupd + 3) / 4), dim3(256), 0, s, w);
}

// --------------------------------------------------------------------------- client table
__global__ void k_gather_sec_clients(const Section* __restrict__ sec, uint32_t n, uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = sec[i].n ? sec[i].client : sec[i].client;  // empty sections still name a client
}
__global__ void k_unique_flags(const uint32_t* __restrict__ v, uint32_t n, uint32_t* __restrict__ flags) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) flags[i] = (i == 0 || v[i] != v[i - 1]) ? 1u : 0u;
  else if (i == n) flags[i] = 0;
}
__global__ void k_unique_scatter(const uint32_t* __restrict__ v, const uint32_t* __restrict__ pre, uint32_t n,
                                 uint32_t* __restrict__ out, uint32_t* nout, uint8_t* __restrict__ single) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && (i == 0 || v[i] != v[i - 1])) {
    out[pre[i]] = v[i];
    if (single) single[pre[i]] = (i + 1 == n || v[i + 1] != v[i]) ? 1u : 0u;  // a run of one section
  }
  if (i == n) *nout = pre[n];
}
__global__ void k_section_cidx(Section* __restrict__ sec, uint32_t n, const uint32_t* __restrict__ cl, const uint32_t* nc) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) sec[i].cidx = lower_bound_u32(cl, *nc, sec[i].client);
}
// multi-document batches: clients are (doc, client) pairs, sorted by doc then client id
__global__ void k_gather_sec_keys(Work w, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { w.cl_key2[i] = ((uint64_t)w.udoc[w.sections[i].upd] << 32) | w.sections[i].client; w.cl_tmp[i] = i; }
}
__global__ void k_unique_keys(Work w, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) w.scratch[i] = (i == 0 || w.cl_key[i] != w.cl_key[i - 1]) ? 1u : 0u;
  else if (i == n) w.scratch[i] = 0;
}
__global__ void k_unique_keys_scatter(Work w, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && (i == 0 || w.cl_key[i] != w.cl_key[i - 1])) {
    const uint64_t k = w.cl_key[i];
    const uint32_t c = w.cl_tmp[i];
    w.cl_key2[c] = k;
    w.cl_vals[c] = (uint32_t)k;
    w.cl_doc[c] = (uint32_t)(k >> 32);
    if (w.cl_single) w.cl_single[c] = (i + 1 == n || w.cl_key[i + 1] != k) ? 1u : 0u;  // a run of one section
  }
  if (i == n) w.ctr->nclients = w.cl_tmp[n];
}
__global__ void k_section_cidx_multi(Work w, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) w.sections[i].cidx = find_client(w, w.ctr->nclients, w.udoc[w.sections[i].upd], w.sections[i].client);
}

// Small single-document batches (the per-op path): the client table in ONE workgroup launch
// (seven otherwise): the sections' clients sorted in LDS (bitonic), the distinct ones numbered by a
// scan of the run-start flags, then every section's client index by binary search in LDS.
constexpr uint32_t CT_LANES = 1024, CT_SMALL = 2048;
__device__ __forceinline__ void client_table_small_body(const Work& w, uint32_t n, uint32_t* v, uint32_t* pre, uint32_t* u, uint32_t* part) {
  const uint32_t t = threadIdx.x;
  uint32_t N = 1;
  while (N < n) N <<= 1;
  for (uint32_t i = t; i < N; i += CT_LANES) v[i] = i < n ? w.sections[i].client : 0xFFFFFFFFu;
  __syncthreads();
  for (uint32_t k = 2; k <= N; k <<= 1)
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = t; i < N; i += CT_LANES) {
        const uint32_t l = i ^ j;
        if (l > i) {
          const uint32_t x = v[i], y = v[l];
          if (((i & k) == 0) ? (x > y) : (x < y)) { v[i] = y; v[l] = x; }
        }
      }
      __syncthreads();
    }
  // run starts, scanned: two entries per lane
  const uint32_t i0 = 2 * t, i1 = 2 * t + 1;
  const uint32_t f0 = i0 < n && (i0 == 0 || v[i0] != v[i0 - 1]) ? 1u : 0u;
  const uint32_t f1 = i1 < n && v[i1] != v[i1 - 1] ? 1u : 0u;
  part[t] = f0 + f1;
  __syncthreads();
  for (uint32_t off = 1; off < CT_LANES; off <<= 1) {
    const uint32_t x = t >= off ? part[t - off] : 0u;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  const uint32_t base = part[t] - f0 - f1;
  if (i0 < n) pre[i0] = base;
  if (i1 < n) pre[i1] = base + f0;
  const uint32_t nc = part[CT_LANES - 1];
  __syncthreads();
  for (uint32_t i = t; i < n; i += CT_LANES)
    if (i == 0 || v[i] != v[i - 1]) {
      u[pre[i]] = v[i];
      w.cl_vals[pre[i]] = v[i];
      if (w.cl_single) w.cl_single[pre[i]] = (i + 1 == n || v[i + 1] != v[i]) ? 1u : 0u;  // a run of one section
    }
  if (t == 0) w.ctr->nclients = nc;
  __syncthreads();
  for (uint32_t i = t; i < n; i += CT_LANES) {
    const uint32_t c = w.sections[i].client;
    uint32_t lo = 0, hi = nc;
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (u[m] < c) lo = m + 1; else hi = m; }
    w.sections[i].cidx = lo;
  }
}
__global__ __launch_bounds__(CT_LANES) void k_client_table_small(Work w, uint32_t n) {
  __shared__ uint32_t v[CT_SMALL], pre[CT_SMALL + 1], u[CT_SMALL];
  __shared__ uint32_t part[CT_LANES];
  client_table_small_body(w, n, v, pre, u, part);
}

// NC stays on the device (ctr->nclients) until the struct-decode counter read
void launch_client_table(Work& w, uint32_t nsections, hipStream_t s) {
  const uint32_t grid = nsections / 256 + 1;
  if (!w.udoc && nsections <= CT_SMALL) {
    hipLaunchKernelGGL(k_client_table_small, dim3(1), dim3(CT_LANES), 0, s, w, nsections);
    return;
  }
  if (w.udoc) {
    hipLaunchKernelGGL(k_gather_sec_keys, dim3(grid), dim3(256), 0, s, w, nsections);
    // (doc << 32 | client keys: the radix passes stop past the document bits)
    uint32_t dbits = 0;
    while (dbits < 32 && (w.ndocs - 1) >> dbits) ++dbits;
    sort_pairs_u64_u32(w.tmp, w.tmp_bytes, w.cl_key2, w.cl_key, w.cl_tmp, w.cl_state, nsections, s, 32 + dbits);
    hipLaunchKernelGGL(k_unique_keys, dim3(grid), dim3(256), 0, s, w, nsections);
    scan_u32(w.tmp, w.tmp_bytes, w.scratch, w.cl_tmp, nsections + 1, s);
    hipLaunchKernelGGL(k_unique_keys_scatter, dim3(grid), dim3(256), 0, s, w, nsections);
    // the distinct keys are in cl_key2: the two buffers trade places (a copy back waited ~0.6 ms
    // for compute units beside the delete-set decode on the side stream)
    std::swap(w.cl_key, w.cl_key2);
    hipLaunchKernelGGL(k_section_cidx_multi, dim3(grid), dim3(256), 0, s, w, nsections);
    return;
  }
  hipLaunchKernelGGL(k_gather_sec_clients, dim3(grid), dim3(256), 0, s, w.sections, nsections, w.cl_tmp);
  sort_u32(w.tmp, w.tmp_bytes, w.cl_tmp, w.cl_vals, nsections, s);
  hipLaunchKernelGGL(k_unique_flags, dim3(grid), dim3(256), 0, s, w.cl_vals, nsections, w.scratch);
  scan_u32(w.tmp, w.tmp_bytes, w.scratch, w.cl_tmp, nsections + 1, s);
  // compact in place is unsafe: into cl_state's buffer, and the two trade places (same size)
  hipLaunchKernelGGL(k_unique_scatter, dim3(grid), dim3(256), 0, s, w.cl_vals, w.cl_tmp, nsections, w.cl_state, &w.ctr->nclients, w.cl_single);
  std::swap(w.cl_vals, w.cl_state);
  hipLaunchKernelGGL(k_section_cidx, dim3(grid), dim3(256), 0, s, w.sections, nsections, w.cl_vals, &w.ctr->nclients);
}

// the client hash (find_client), from the finished client table; slots were filled with ~0
__global__ void k_client_hash(Work w, uint64_t* __restrict__ key, uint32_t* __restrict__ val, uint32_t mask) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= w.ctr->nclients) return;
  const uint64_t k = w.udoc ? w.cl_key[i] : (uint64_t)w.cl_vals[i];
  for (uint32_t slot = (uint32_t)client_hash(k) & mask;; slot = (slot + 1) & mask) {
    const unsigned long long old = atomicCAS((unsigned long long*)&key[slot], ~0ull, (unsigned long long)k);
    if (old == ~0ull || old == k) { val[slot] = i; return; }  // keys are distinct
  }
}
void launch_client_hash(const Work& w, uint64_t* key, uint32_t* val, uint32_t mask, hipStream_t s) {
  hipLaunchKernelGGL(k_client_hash, dim3((mask + 1) / 512 + 1), dim3(256), 0, s, w, key, val, mask);
}
// Small single-document batches: the section ranks, the client table and the client hash (its
// fill included) as phases of ONE workgroup (four launches otherwise)
__global__ __launch_bounds__(CT_LANES) void k_sections_small(Work w, uint32_t n, uint64_t* __restrict__ key, uint32_t* __restrict__ val,
                                                             uint32_t mask) {
  __shared__ uint32_t v[CT_SMALL], pre[CT_SMALL + 1], u[CT_SMALL];
  __shared__ uint32_t part[CT_LANES];
  const uint32_t t = threadIdx.x;
  if (n == NONE) {  // (the quick decode: no count synchronisation ran, the count is on the device)
    n = w.ctr->err ? 0u : w.ctr->nsections;  // (the walk failed: the sections are not to be read)
    if (n > CT_SMALL) { if (t == 0) raise_err(&w.ctr->err, ERR_CAPACITY); n = 0; }  // (rerun, counted)
    if (!n) {
      // no client table: the host still hands the hash to find_client (k_units clips a delete-only
      // update's ranges against it), so it must be EMPTY here, not the previous merge's slots
      for (uint32_t i = t; i <= mask; i += CT_LANES) key[i] = ~0ull;
      if (t == 0) w.ctr->nclients = 0;
      return;
    }
  }
  if (w.dbg_bounds && (n > w.cap_sections || n + 1 > w.cap_clients + 1 || 2 * (n + 1) > mask + 1)) {
    if (t == 0) bounds_fail(w.ctr, BOUNDS_SECTIONS);
    return;
  }
  for (uint32_t i = t; i < n; i += CT_LANES) section_rank_at(w, i);
  for (uint32_t i = t; i <= mask; i += CT_LANES) key[i] = ~0ull;
  client_table_small_body(w, n, v, pre, u, part);  // (ends with the sections' client indexes)
  __syncthreads();  // (the key fill's stores reach L2 before the later atomics: one CU's vector L1 forwards in order)
  const uint32_t nc = w.ctr->nclients;
  for (uint32_t i = t; i < nc; i += CT_LANES) {
    const uint64_t k = (uint64_t)w.cl_vals[i];
    for (uint32_t slot = (uint32_t)client_hash(k) & mask;; slot = (slot + 1) & mask) {
      const unsigned long long old = atomicCAS((unsigned long long*)&key[slot], ~0ull, (unsigned long long)k);
      if (old == ~0ull || old == k) { val[slot] = i; break; }  // keys are distinct
    }
  }
}
bool sections_small(const Work& w, uint32_t nsections, uint64_t* key, uint32_t* val, uint32_t mask, hipStream_t s) {
  if (env_off("YCRDT_DECODE_SMALL") || w.udoc || !nsections || (nsections != NONE && nsections > CT_SMALL) || mask + 1 > 16 * CT_SMALL) return false;
  hipLaunchKernelGGL(k_sections_small, dim3(1), dim3(CT_LANES), 0, s, w, nsections, key, val, mask);
  return true;
}

// --------------------------------------------------------------------------- 6. struct decode

// One struct's columns (DEFER: a struct whose content needs the out-of-line `any` reader is
// appended to the deferred list and left to k_struct_decode_deferred). win: the workgroup's LDS.
template <bool DEFER>
__device__ __forceinline__ void struct_decode_one(const Work& w, uint32_t i, uint32_t* win) {
  const uint32_t nclients = w.ctr->nclients;
  uint32_t* err = &w.ctr->err;
  const uint32_t p0 = w.s_pos[i];
  // the struct's section: the section starts at or before it (rank in the section-start bitmap);
  // written here for the later passes (computing it in k_scatter_pos doubled that kernel's LDS
  // and time: 0.32 -> 1.36 ms on the C2 batch)
  const uint32_t si = w.sec_sorted[rank_incl(win_words(w.sec_bits, w.nwin > 1 ? w.s_win[i] : 0u),
                                             win_words(w.wsec, w.nwin > 1 ? w.s_win[i] : 0u), p0) - 1];
  w.s_sec[i] = si;
  // the struct's bytes (they depend on its position only) are fetched beside its section record
  uint32_t* slot = win + threadIdx.x * SD_STRIDE;
  const uint32_t s0 = p0 & ~15u;
  const uint8_t* __restrict__ bw = struct_bytes(w, i);  // the struct's window
  const uint4* g = (const uint4*)(bw + s0);  // the batch buffer is padded past its end
  uint4 v4[SD_WIN / 16];
#pragma unroll
  for (uint32_t k = 0; k < SD_WIN / 16; ++k) v4[k] = g[k];
  const Section sec = w.sections[si];
  const uint32_t uend = w.sec_uend[si];
  const uint32_t doc = w.sec_doc[si];
#pragma unroll
  for (uint32_t k = 0; k < SD_WIN / 16; ++k) ((uint4*)slot)[k] = v4[k];
  StructView v;
  uint32_t p = p0;
  const int pr = parse_struct<true, 32, WinSrc, DEFER>(WinSrc{bw, slot, s0}, p, uend, 0xFFFFFFFFu, &v);
  if (DEFER && pr == PARSE_DEFER) {
    w.sd_defer[atomicAdd(&w.ctr->nsd_defer, 1u)] = i;  // (rare: nested `any` containers, ContentDoc)
    return;
  }
  if (pr <= 0) { raise_err(err, pr == -1 ? ERR_UNSUPPORTED : ERR_DECODE); return; }  // -1: any nested > 32 deep
  const uint32_t ref0 = v.ref;  // (a superseded section's structs are still read: JSON.parse runs on them)
  if (sec.pad && !w.lazy) {  // a superseded section (k_ds_bound): its structs are not integrated
    v.info = (uint8_t)((v.info & 0xE0u) | REF_SKIP);
    v.ref = REF_SKIP;
  }
  w.s_len[i] = v.len;
  w.s_info[i] = v.info;
  w.s_cidx[i] = sec.cidx;
  uint32_t oc = NONE, rc = NONE;
  const bool item = v.ref != REF_GC && v.ref != REF_SKIP;
  // lazy mode (mergeUpdates / diffUpdate): references are copied, never resolved, so the raw
  // client ids are kept (presence = info bits); integrate mode maps them to client indices
  // references to the struct's own client (the common case: a client's consecutive inserts) take
  // the section's client index instead of a binary search over the client table
  if (item && (v.info & 0x80u)) {
    oc = w.lazy ? v.oc : v.oc == sec.client ? sec.cidx : find_client(w, nclients, doc, v.oc);
    if (oc == NONE && !w.lazy) oc = UNKNOWN;  // k_refs decides (pending unless capped away)
  }
  if (item && (v.info & 0x40u)) {
    rc = w.lazy ? v.rc : v.rc == sec.client ? sec.cidx : find_client(w, nclients, doc, v.rc);
    if (rc == NONE && !w.lazy) rc = UNKNOWN;
  }
  // columns a consumer reads only behind their presence test are written only when present
  // (the right origin clock behind s_rcidx != NONE, the parent / parentSub behind s_pk != 0):
  // most structs of a replica update carry neither (C2: 20 of the 57 bytes per struct)
  w.s_ocidx[i] = oc;
  w.s_oclock[i] = v.ok_;
  w.s_rcidx[i] = rc;
  if (rc != NONE) w.s_rclock[i] = v.rk;
  // parent: root type name (varString position/length) or parent item id (client index, clock)
  uint32_t pk = item ? v.pkind : 0u, pa = NONE, pb = 0;
  if (pk == 1) { pa = v.pa; pb = v.pb; }
  else if (pk == 2) {
    pa = w.lazy ? v.pa : v.pa == sec.client ? sec.cidx : find_client(w, nclients, doc, v.pa);
    pb = v.pb;
    if (pa == NONE && !w.lazy) pa = UNKNOWN;
  }
  if (pk != 0 && !v.has_psub) w.ctr->narray_roots = 1;  // a YArray list may exist (flag, plain store)
  if (pk == 2) w.ctr->nested = 1;                        // a nested type's list (flag, plain store)
  wave_flag(&w.ctr->any_rorigin, item && (v.info & 0x40u));  // (a YMap entry may need full YATA)
  wave_count_add_sharded(w.ctr->nroots_sh, pk != 0);
  // the header as Item.write re-encodes it (every varuint in shortest form): an overlong varuint
  // (valid lib0 input) makes the input's header bytes differ from the output's, so such a struct
  // is flagged (s_pk bit 7) and never takes the encoder's byte-copy path
  bool canon_hdr = true;
  if (item) {
    uint32_t h = 0;
    if (v.info & 0x80u) h += vu_size(v.oc) + vu_size(v.ok_);
    if (v.info & 0x40u) h += vu_size(v.rc) + vu_size(v.rk);
    if ((v.info & 0xC0u) == 0) {
      h += 1;  // parent info (1: root type name, 0: parent item id)
      if (v.pkind == 1) h += vu_size(v.pn) + v.pn;
      else h += vu_size(v.pa) + vu_size(v.pb);
      if (v.has_psub) h += vu_size(v.psn) + v.psn;
    }
    canon_hdr = h == v.cpos - p0 - 1;
  }
  // bit 6: the content's `any` values are not in writeAny's form (the encoders re-encode them)
  // bit 5: object keys JS treats specially (ANY_KEYS): the struct is rewritten before the merge
  // (k_json_structs lists it, k_json_canon writes writeAny(readAny(.)) of its content)
  w.s_pk[i] = (uint8_t)(pk | (canon_hdr ? 0u : 0x80u) | ((v.anyf & ANY_REENCODE) ? 0x40u : 0u) | ((v.anyf & ANY_KEYS) ? 0x20u : 0u));
  if (pk != 0) {
    w.s_pa[i] = pa;
    w.s_pb[i] = pb;
    w.s_psub[i] = v.has_psub ? v.psub_pos : NONE;
    w.s_psublen[i] = v.psub_len;
  }
  w.s_cpos[i] = v.cpos;
  w.s_cend[i] = v.cend;
  uint32_t celem = v.cpos;
  if (v.ref == REF_ANY || v.ref == REF_JSON) celem += vu_size(v.nel);
  w.s_celem[i] = celem;
  // a JSON / Embed / Format content: JSON.parse runs in k_json_structs (a call from here, however
  // rare, cost every struct one wave per SIMD: the kernel's registers cover the callee's)
  wave_flag(&w.ctr->any_json, ref0 == REF_JSON || ref0 == REF_EMBED || ref0 == REF_FORMAT || (v.anyf & ANY_KEYS) != 0);
}
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_struct_decode(Work w, uint32_t nstructs) {
  __shared__ __attribute__((aligned(16))) uint32_t win[256 * SD_STRIDE];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nstructs) struct_decode_one<true>(w, i, win);
}
// the structs k_struct_decode deferred (their contents need the out-of-line `any` reader)
constexpr uint32_t SD_DEFER_GRID = 1024;
__global__ __launch_bounds__(256) void k_struct_decode_deferred(Work w) {
  __shared__ __attribute__((aligned(16))) uint32_t win[256 * SD_STRIDE];
  const uint32_t n = w.ctr->nsd_defer;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x)
    struct_decode_one<false>(w, w.sd_defer[k], win);
}
// JSON.parse of the JSON / Embed / Format contents (yc_parse.h json_content), one lane per struct,
// launched only when k_struct_decode saw such a content (Yjs writes ContentAny for JS values)
__global__ __launch_bounds__(256) void k_json_structs(Work w, uint32_t nstructs) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nstructs) return;
  const uint8_t* __restrict__ bw = struct_bytes(w, i);
  const uint32_t ref = bw[w.s_pos[i]] & 31u;  // (the input's info byte: superseded sections' structs too)
  if (w.ntrusted && w.sections[w.s_sec[i]].upd < w.ntrusted) return;  // a doc state: already what Yjs holds
  if (ref == REF_ANY && (w.s_pk[i] & 0x20u)) {  // `any` objects with keys JS treats specially: rewritten
    if (w.jskip_any) return;
    if (!any_keys_exact(bw, w.s_cpos[i], w.s_cend[i])) return;  // (a repeat-mask false alarm)
    const uint32_t k = atomicAdd(&w.ctr->njson, 1u);
    if (k < w.jcap) w.jlist[k] = i;
    return;
  }
  if (ref != REF_JSON && ref != REF_EMBED && ref != REF_FORMAT) return;
  const int jr = json_content(bw, w.s_cpos[i], w.s_cend[i], ref);
  if (jr > 0) raise_err(&w.ctr->err, ERR_DECODE);
  if (jr < 0) {  // not in the form Yjs writes back: listed for k_json_canon (run_decode rewrites the update)
    const uint32_t k = atomicAdd(&w.ctr->njson, 1u);
    if (k < w.jcap) w.jlist[k] = i;
  }
}
void launch_json_structs(const Work& w, uint32_t nstructs, hipStream_t s) {
  if (nstructs) hipLaunchKernelGGL(k_json_structs, dim3(nstructs / 256 + 1), dim3(256), 0, s, w, nstructs);
}
// The canonical contents of the listed structs (yc_parse.h json_content_canon): pass 0 (out null)
// records each one's position, input length, canonical length and verdict; pass 1 writes it at
// out + offs[j] and records whether they differ from the input (JItem.pad). One lane per struct over
// a lane-private arena: these are the rare values a Yjs peer of an old version (or a hand-made
// update) sent outside JSON.stringify's form.
__global__ __launch_bounds__(64) void k_json_canon(Work w, const uint32_t* __restrict__ list, uint32_t n, JItem* __restrict__ items,
                                                   uint32_t* __restrict__ arena, uint32_t acap, uint32_t lanes,
                                                   const unsigned long long* __restrict__ offs, uint8_t* __restrict__ out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= lanes) return;
  uint32_t* a = arena + (uint64_t)t * acap;
  for (uint32_t j = t; j < n; j += lanes) {
    const uint32_t i = list[j];
    const uint8_t* __restrict__ bw = struct_bytes(w, i);
    const uint32_t ref = bw[w.s_pos[i]] & 31u, cp = w.s_cpos[i], ce = w.s_cend[i];
    uint32_t len = 0;
    if (!out) {
      const uint32_t r = json_content_canon(bw, cp, ce, ref, nullptr, a, acap, len);
      const unsigned long long base = w.nwin > 1 ? ((unsigned long long)w.s_win[i] << w.win_shift) : 0ull;
      items[j] = JItem{base + cp, ce - cp, len, r, 0u};
    } else if (items[j].res == JSON_OK) {
      uint8_t* o = out + offs[j];
      json_content_canon(bw, cp, ce, ref, o, a, acap, len);
      // unchanged (a repeat-mask false alarm, a text json_check could not judge): the host keeps
      // the batch as staged when every item says so
      uint32_t same = len == ce - cp;
      for (uint32_t k = 0; same && k < len; ++k) same = o[k] == bw[cp + k];
      items[j].pad = same ? 0u : 1u;
    }
  }
}
void launch_json_canon(const Work& w, const uint32_t* list, uint32_t n, JItem* items, uint32_t* arena, uint32_t acap,
                       uint32_t lanes, const unsigned long long* offs, uint8_t* out, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_json_canon, dim3((lanes + 63) / 64), dim3(64), 0, s, w, list, n, items, arena, acap, lanes, offs, out);
}

// Clocks from the section start and the length prefix; with `states` (integrate mode) also the
// client states (k_states' work, folded in: the clock and length are in registers here)
__device__ __forceinline__ void struct_clock_at(const Work& w, uint32_t i, uint32_t nstructs, uint32_t states) {
  const uint32_t si = w.s_sec[i];
  const Section sec = w.sections[si];
  const uint64_t off = w.s_lenscan[i] - w.s_lenscan[sec.first_idx];
  const uint64_t clock = (uint64_t)sec.clock + off;
  const uint32_t len = w.s_len[i];
  const uint64_t endc = clock + len;
  if (endc > 0xFFFFFFFFull) { raise_err(&w.ctr->err, ERR_DECODE); return; }
  w.s_clock[i] = (uint32_t)clock;
  if (!states) return;
  const uint32_t ref = w.s_info[i] & 31u;
  if (ref == REF_SKIP) {  // rare: Skip lengths are subtracted from the item count
    atomicAdd(&w.ctr->items, (unsigned long long)len);
    return;
  }
  // clocks grow along a section: only the last non-skip struct of a run can hold the max
  const bool last = i + 1 == nstructs || w.s_sec[i + 1] != si || (w.s_info[i + 1] & 31u) == REF_SKIP;
  if (last) atomicMax(&w.cl_state[w.s_cidx[i]], (uint32_t)endc);
}
__global__ void k_struct_clock(Work w, uint32_t nstructs, uint32_t states) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nstructs) struct_clock_at(w, i, nstructs, states);
}

void launch_struct_decode(const Work& w, uint32_t nstructs, hipStream_t s) {
  if (!nstructs) return;
  hipLaunchKernelGGL(k_struct_decode, dim3((nstructs + 255) / 256), dim3(256), 0, s, w, nstructs);
  hipLaunchKernelGGL(k_struct_decode_deferred, dim3(std::min<uint32_t>(nstructs / 256 + 1, SD_DEFER_GRID)), dim3(256), 0, s, w);
}
void launch_struct_lenscan(const Work& w, uint32_t nstructs, hipStream_t s) {
  if (nstructs) scan_u32_to_u64(w.tmp, w.tmp_bytes, w.s_len, w.s_lenscan, nstructs + 1, s);
}

// --------------------------------------------------------------------------- client states
// Yjs pending structs (yc_ingest.h): every client is integrated up to its cap only
__device__ __forceinline__ void apply_caps_at(const Work& w, uint32_t c) {
  const uint32_t v = w.cl_vals[c];
  const uint32_t i = lower_bound_u32(w.cap_client, w.ncaps, v);
  const uint32_t cap = (i < w.ncaps && w.cap_client[i] == v) ? w.cap_clock[i] : 0u;
  if (ld_fresh(&w.cl_state[c]) > cap) w.cl_state[c] = cap;
}
__global__ void k_apply_caps(Work w) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < w.ctr->nclients) apply_caps_at(w, c);
}
__global__ void k_state_totals(Work w, uint32_t nstructs) {  // U and Σ input lengths into the counters
  w.ctr->units = w.cl_base[w.ctr->nclients];
  w.ctr->in_len = w.s_lenscan[nstructs];
}
// NC <= nsections: the states are zero past NC, so a scan over nsections + 1 entries gives cl_base
// cl_state must be zero on entry (the caller's fill)
void launch_struct_clocks(const Work& w, uint32_t nstructs, hipStream_t s) {  // lazy mode: clocks only
  if (nstructs) hipLaunchKernelGGL(k_struct_clock, dim3((nstructs + 255) / 256), dim3(256), 0, s, w, nstructs, 0u);
}
void launch_states(const Work& w, uint32_t nstructs, uint32_t nsections, hipStream_t s) {
  if (nstructs) hipLaunchKernelGGL(k_struct_clock, dim3((nstructs + 255) / 256), dim3(256), 0, s, w, nstructs, 1u);
  if (w.capped && nsections) hipLaunchKernelGGL(k_apply_caps, dim3(nsections / 256 + 1), dim3(256), 0, s, w);
  scan_u32_to_u64(w.tmp, w.tmp_bytes, w.cl_state, w.cl_base, nsections + 1, s);
  hipLaunchKernelGGL(k_state_totals, dim3(1), dim3(1), 0, s, w, nstructs);
}

// Small batches (integrate mode): the struct decode (rare contents inline, no deferred pass), the
// clock-length scan, the clocks and client states, the caps, the state scan and the totals as
// phases of ONE workgroup — one launch for six.
constexpr uint32_t DT_LANES = 256, DT_SMALL = 4096;
__global__ __launch_bounds__(DT_LANES) void k_decode_tail_small(Work w, uint32_t nstructs, uint32_t nsections) {
  __shared__ __attribute__((aligned(16))) uint32_t win[DT_LANES * SD_STRIDE];
  __shared__ uint64_t part[DT_LANES];
  const uint32_t t = threadIdx.x;
  if (nstructs == NONE) {  // (the quick decode: the counts are on the device)
    if (w.ctr->err) return;
    nstructs = w.ctr->nstructs;
    nsections = w.ctr->nsections;
    if (nstructs > DT_SMALL || nsections + 1 > DT_LANES * 16) { if (t == 0) raise_err(&w.ctr->err, ERR_CAPACITY); return; }
  }
  if (w.dbg_bounds && (nstructs > w.cap_structs || nsections + 1 > w.cap_clients + 1)) {
    if (t == 0) bounds_fail(w.ctr, BOUNDS_DECODE_TAIL);
    return;
  }
  for (uint32_t i = t; i <= nsections; i += DT_LANES) { w.cl_start[i] = 0; w.cl_state[i] = 0; }
  for (uint32_t i = t; i < nstructs; i += DT_LANES) struct_decode_one<false>(w, i, win);
  __syncthreads();
  block_scan_u32_u64<DT_LANES>(w.s_len, w.s_lenscan, nstructs + 1, part);
  for (uint32_t i = t; i < nstructs; i += DT_LANES) struct_clock_at(w, i, nstructs, 1u);
  __syncthreads();
  const uint32_t nclients = w.ctr->nclients;
  if (w.capped) {
    for (uint32_t c = t; c < nclients; c += DT_LANES) apply_caps_at(w, c);  // (reads cl_state through L2)
    __syncthreads();
  }
  block_scan_u32_u64<DT_LANES, true>(w.cl_state, w.cl_base, nsections + 1, part);  // (client states: atomicMax)
  if (t == 0) {  // (k_state_totals)
    w.ctr->units = w.cl_base[nclients];
    w.ctr->in_len = w.s_lenscan[nstructs];
  }
}
void launch_decode_tail_small(const Work& w, uint32_t nstructs, uint32_t nsections, hipStream_t s) {
  hipLaunchKernelGGL(k_decode_tail_small, dim3(1), dim3(DT_LANES), 0, s, w, nstructs, nsections);
}
bool decode_tail_small(const Work& w, uint32_t nstructs, uint32_t nsections, hipStream_t s) {
  const bool off = env_off("YCRDT_DECODE_SMALL");  // (read per merge: A/B in one process)
  if (off || !nstructs || nstructs > DT_SMALL || nsections + 1 > DT_LANES * 16) return false;
  hipLaunchKernelGGL(k_decode_tail_small, dim3(1), dim3(DT_LANES), 0, s, w, nstructs, nsections);
  return true;
}

}  // namespace yc
