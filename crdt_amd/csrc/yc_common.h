// yc_common.h — shared definitions for the ycrdt HIP engine (gfx950).
//
// The engine merges a batch of Yjs v1 updates (Y.applyUpdate × n, Y.mergeUpdates) into the
// canonical encoded state (Y.encodeStateAsUpdate) entirely on the GPU. Layout and kernels are
// described in DESIGN.md; reference semantics are those restated in oracle/yref.c (Yjs 13.5.16).
#pragma once
#include <cstring>
#include <cstdlib>
#include <cstdint>
#include <hip/hip_runtime.h>

namespace yc {

constexpr uint32_t NONE = 0xFFFFFFFFu;

// ---------------------------------------------------------------- decode geometry
// A "group" is a ≤16 KiB slice of one update parsed by one 256-lane workgroup; each lane owns
// a 64-byte chunk and speculatively parses the struct chain that starts at the chunk start.
constexpr uint32_t CHUNK = 64;
constexpr uint32_t GROUP_LANES = 256;
constexpr uint32_t GROUP_BYTES = CHUNK * GROUP_LANES;  // 16384
constexpr uint32_t SPEC_STEPS_FAST = 4;               // speculative parse: first pass work cap (elements)
constexpr uint32_t SPEC_MAX_STEPS = 1024;             // second pass (compacted); longer -> exact walker parse
constexpr uint16_t STOPF = 0x8000;                    // table flag: chain stops at an unsized struct

// content refs (low 5 bits of the info byte)
enum : uint8_t {
  REF_GC = 0, REF_DELETED = 1, REF_JSON = 2, REF_BINARY = 3, REF_STRING = 4, REF_EMBED = 5,
  REF_FORMAT = 6, REF_TYPE = 7, REF_ANY = 8, REF_DOC = 9, REF_SKIP = 10
};

// error codes raised on device (first error wins via atomicCAS on the error word)
enum : uint32_t {
  ERR_NONE = 0,
  ERR_DECODE = 1,       // malformed update
  ERR_PENDING = 2,      // missing dependency (Yjs would keep it pending)
  ERR_UNSUPPORTED = 3,  // valid Yjs input outside the engine's current coverage
  ERR_CAPACITY = 4,     // internal capacity exceeded
};

struct Group {          // one decode group
  uint32_t start, end;  // byte range [start,end) inside the batch buffer (start 64-byte aligned)
  uint32_t uend;        // end of the group's update (parses never read past it)
  uint32_t upd;         // update index
};

struct Section {        // one client section of one update's struct section
  uint32_t upd;
  uint32_t n;           // structs in section
  uint32_t client;      // client id (value)
  uint32_t clock;       // first clock
  uint32_t first_pos;   // byte position of the first struct (NONE if n == 0)
  uint32_t cidx;        // dense client index (filled later)
  uint32_t first_idx;   // global struct index of first struct
  uint32_t pad;
};

struct CopyTask {       // verified chain segment: b struct starts along the chain from position a
  uint32_t a, b;
};

// count the lanes of a wavefront for which `pred` holds with ONE atomic (the first such lane adds
// the popcount): per-lane atomics on one counter address serialise at the memory side
__device__ __forceinline__ void wave_count_add(uint32_t* ctr, bool pred) {
  const unsigned long long m = __ballot(pred);
  if (m && (threadIdx.x & 63u) == (uint32_t)__ffsll((long long)m) - 1) atomicAdd(ctr, (uint32_t)__popcll(m));
}

__device__ __forceinline__ void raise_err(uint32_t* err, uint32_t code) {
  atomicCAS(err, 0u, code);
}

// ---------------------------------------------------------------- lib0 readers (L0@1937)
// readVarUint: 7-bit groups with 32-bit shift-or accumulation (lib0 0.2.42). A 6th
// continuation byte or running past `end` is "Integer out of range!".
__device__ __forceinline__ uint32_t rd_vu(const uint8_t* __restrict__ b, uint32_t& p, uint32_t end, bool& ok) {
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
__device__ __forceinline__ void skip_vi(const uint8_t* __restrict__ b, uint32_t& p, uint32_t end, bool& ok) {
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
__device__ __forceinline__ bool json_start_ok(uint32_t c) {
  return c == '{' || c == '[' || c == '"' || c == 't' || c == 'f' || c == 'n' || c == 'u' || c == '-' ||
         (c >= '0' && c <= '9') || c == ' ' || c == '\t' || c == '\n' || c == '\r';
}

__device__ __forceinline__ void skip_bytes(uint32_t& p, uint32_t n, uint32_t end, bool& ok) {
  if (end - p < n) { ok = false; p = end; return; }
  p += n;
}

// readAny (L0@1937 B): iterative skip with an explicit container stack of depth DEPTH (deeper
// nesting fails the parse: speculative callers use a shallow stack, exact callers a deep one).
template <int DEPTH>
__device__ inline bool skip_any(const uint8_t* __restrict__ b, uint32_t& p, uint32_t end, uint32_t& steps) {
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
      case 125: skip_vi(b, p, end, ok); break;
      case 124: skip_bytes(p, 4, end, ok); break;
      case 123: case 122: skip_bytes(p, 8, end, ok); break;
      case 119: case 116: { uint32_t n = rd_vu(b, p, end, ok); if (ok) skip_bytes(p, n, end, ok); break; }
      case 118: case 117: {
        uint32_t n = rd_vu(b, p, end, ok);
        if (!ok) return false;
        if (n > 0) {
          if (d == DEPTH) { steps = 0; return false; }  // too deep: "unknown" (-1), never "malformed"
          rem[d] = n;
          if (tag == 118) objmask |= 1u << d; else objmask &= ~(1u << d);
          ++d;
          if (tag == 118) { uint32_t k = rd_vu(b, p, end, ok); if (ok) skip_bytes(p, k, end, ok); }
          if (!ok) return false;
          continue;  // read the first member value
        }
        break;
      }
      default: return false;
    }
    if (!ok) return false;
    // a value completed: pop finished containers
#pragma unroll 1
    for (;;) {
      if (d == 0) return true;
      if (--rem[d - 1] > 0) {
        if ((objmask >> (d - 1)) & 1u) { uint32_t k = rd_vu(b, p, end, ok); if (ok) skip_bytes(p, k, end, ok); if (!ok) return false; }
        break;  // next member value
      }
      --d;
    }
  }
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
  uint32_t cpos, cend; // content bytes [cpos, cend)
  uint32_t nel;        // Any/JSON element count
};

// Parses one struct starting at p. FULL fills `v`. Speculative callers pass a finite
// step budget; exact callers pass 0xFFFFFFFF. Returns 1 = ok, 0 = malformed, -1 = budget hit,
// -2 = ran past `end` (only distinguishable from 0 when `end` is not the update end).
template <bool FULL, int DEPTH = 32>
__device__ inline int parse_struct(const uint8_t* __restrict__ b, uint32_t& p, uint32_t end, uint32_t steps, StructView* v) {
  bool ok = true;
  if (p >= end) return -2;
  uint32_t info = b[p++];
  uint32_t ref = info & 31u;
  if (FULL) { v->info = (uint8_t)info; v->ref = (uint8_t)ref; v->pkind = 0; v->has_psub = 0; v->nel = 0; }
  if (ref == REF_GC || ref == REF_SKIP) {
    uint32_t len = rd_vu(b, p, end, ok);
    if (FULL) { v->len = len; v->cpos = v->cend = p; }
    return ok ? 1 : (p >= end ? -2 : 0);
  }
  if (ref > REF_DOC) return 0;
  if (info & 0x80u) {
    uint32_t c = rd_vu(b, p, end, ok), k = rd_vu(b, p, end, ok);
    if (FULL) { v->oc = c; v->ok_ = k; }
  }
  if (info & 0x40u) {
    uint32_t c = rd_vu(b, p, end, ok), k = rd_vu(b, p, end, ok);
    if (FULL) { v->rc = c; v->rk = k; }
  }
  if (!ok) return p >= end ? -2 : 0;
  if ((info & 0xC0u) == 0) {
    uint32_t pinfo = rd_vu(b, p, end, ok);
    if (!ok) return p >= end ? -2 : 0;
    if (pinfo == 1) {
      uint32_t st = p;
      uint32_t n = rd_vu(b, p, end, ok);
      if (ok) skip_bytes(p, n, end, ok);
      if (FULL) { v->pkind = 1; v->pa = st; v->pb = p - st; }
    } else {
      uint32_t c = rd_vu(b, p, end, ok), k = rd_vu(b, p, end, ok);
      if (FULL) { v->pkind = 2; v->pa = c; v->pb = k; }
    }
    if (info & 0x20u) {
      uint32_t st = p;
      uint32_t n = rd_vu(b, p, end, ok);
      if (ok) skip_bytes(p, n, end, ok);
      if (FULL) { v->has_psub = 1; v->psub_pos = st; v->psub_len = p - st; }
    }
    if (!ok) return p >= end ? -2 : 0;
  }
  uint32_t cpos = p;
  uint32_t len = 1;
  switch (ref) {
    case REF_DELETED: len = rd_vu(b, p, end, ok); break;
    case REF_JSON: {
      uint32_t n = rd_vu(b, p, end, ok);
      len = n;
      for (uint32_t i = 0; i < n && ok; ++i) {
        if (steps == 0) return -1;
        --steps;
        uint32_t k = rd_vu(b, p, end, ok);
        if (ok && (k == 0 || (p < end && !json_start_ok(b[p])))) return 0;
        if (ok) skip_bytes(p, k, end, ok);
      }
      if (FULL) v->nel = n;
      if (ok && steps == 0) return -1;
      break;
    }
    case REF_BINARY: { uint32_t k = rd_vu(b, p, end, ok); if (ok) skip_bytes(p, k, end, ok); break; }
    case REF_EMBED: {
      uint32_t k = rd_vu(b, p, end, ok);
      if (ok && (k == 0 || (p < end && !json_start_ok(b[p])))) return 0;
      if (ok) skip_bytes(p, k, end, ok);
      break;
    }
    case REF_STRING: {
      uint32_t k = rd_vu(b, p, end, ok);
      uint32_t st = p;
      if (ok) skip_bytes(p, k, end, ok);
      if (ok && FULL) {  // ContentString length counts UTF-16 code units
        uint32_t u = 0;
        for (uint32_t i = st; i < st + k; ++i) {
          uint32_t c = b[i];
          if ((c & 0xC0u) != 0x80u) u += (c >= 0xF0u) ? 2u : 1u;
        }
        len = u;
      }
      break;
    }
    case REF_FORMAT: {
      uint32_t k = rd_vu(b, p, end, ok);
      if (ok) skip_bytes(p, k, end, ok);
      k = rd_vu(b, p, end, ok);
      if (ok && (k == 0 || (p < end && !json_start_ok(b[p])))) return 0;
      if (ok) skip_bytes(p, k, end, ok);
      break;
    }
    case REF_TYPE: {
      uint32_t tr = rd_vu(b, p, end, ok);
      if (ok && (tr == 3 || tr == 5)) { uint32_t k = rd_vu(b, p, end, ok); if (ok) skip_bytes(p, k, end, ok); }
      if (tr > 6) ok = false;
      break;
    }
    case REF_ANY: {
      uint32_t n = rd_vu(b, p, end, ok);
      len = n;
      for (uint32_t i = 0; i < n && ok; ++i) ok = skip_any<DEPTH>(b, p, end, steps);
      if (!ok && steps == 0) return -1;
      if (FULL) v->nel = n;
      break;
    }
    case REF_DOC: {
      uint32_t k = rd_vu(b, p, end, ok);
      if (ok) skip_bytes(p, k, end, ok);
      if (ok) ok = skip_any<DEPTH>(b, p, end, steps);
      if (!ok && steps == 0) return -1;
      break;
    }
    default: return 0;
  }
  if (FULL) { v->len = len; v->cpos = cpos; v->cend = p; }
  if (!ok && p >= end) return -2;  // ran out of input (the struct may continue past `end`)
  return ok ? 1 : 0;
}

// ---------------------------------------------------------------- varuint writer
__device__ __forceinline__ uint32_t vu_size(uint32_t v) {
  return v < (1u << 7) ? 1 : v < (1u << 14) ? 2 : v < (1u << 21) ? 3 : v < (1u << 28) ? 4 : 5;
}
inline uint32_t vu_size_host(uint32_t v) {
  return v < (1u << 7) ? 1 : v < (1u << 14) ? 2 : v < (1u << 21) ? 3 : v < (1u << 28) ? 4 : 5;
}
__device__ __forceinline__ uint32_t wr_vu(uint8_t* __restrict__ o, uint32_t p, uint32_t v) {
  while (v > 127u) { o[p++] = (uint8_t)(0x80u | (v & 0x7fu)); v >>= 7; }
  o[p++] = (uint8_t)v;
  return p;
}

__device__ __forceinline__ uint32_t lower_bound_u32(const uint32_t* __restrict__ a, uint32_t n, uint32_t key) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ uint32_t upper_bound_u32(const uint32_t* __restrict__ a, uint32_t n, uint32_t key) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (a[mid] <= key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

}  // namespace yc
