// yc_decode.hip — K1: decode of Yjs v1 updates on gfx950.
//
// Replaces lib0's sequential readers + readClientsStructRefs (Y@19286) / readDeleteSet
// (Y@11105) with a byte-parallel decode:
//   1. k_group_parse   one 256-lane workgroup per 16 KiB group; every lane speculatively parses the
//                      struct chain starting at its 64-byte chunk, lane 0 stitches the chunk chains
//                      into one deterministic "main chain" bitmap (1 bit per byte of input; a bit
//                      marks every position the chain visits: next(p) on success, p+1 on failure).
//                      From any true struct start the chain IS the true struct sequence.
//   2. k_walker        one lane per update follows the true chain through section headers, jumping a
//                      whole group per step while it is on the main chain (popcount of the bitmap),
//                      parsing exactly only where it is off the chain (after headers).
//   3. k_copy/k_patch  verified main-chain ranges + exact positions -> final struct-start bitmap.
//   4. k_struct_pos    popcount prefix (scan) -> dense struct index for every struct start.
//   5. k_ds_decode     one wavefront per update decodes the delete set, a pure varuint stream, with a
//                      ballot of terminal bytes + in-register gathers (wavefront prefix scan).
//   6. k_struct_decode one lane per struct: full field decode into the SoA struct table.
#include <algorithm>
#include <cstdlib>

#include "yc_work.h"

namespace yc {

// --------------------------------------------------------------------------- 1a. speculative parse
// nxt[p] for every byte position p of every group: the length of the struct that would start at
// p (0 = not a struct, 1 = not sized here: over the work cap, or too long for the 15-bit table
// positions — the walkers parse those exactly). One 256-lane workgroup per 4 KiB slice, reading
// the bytes through the caches (no LDS staging), so many workgroups share a CU and hide the
// latency of the byte-serial parse. Positions are counting-sorted by their would-be info byte
// (content ref x origin/rightOrigin/parentSub bits) and sized by spec_len one class per wavefront;
// what the sizer hands over is re-parsed by parse_struct under a work cap.
constexpr uint32_t PSLICE = 4096;               // bytes per parse workgroup
constexpr uint32_t PL = 256;                    // lanes per parse workgroup
// work cap of the general parser on what the sizer handed over. Most of the queue is garbage
// positions whose would-be element count is large; a long chain of dependent reads there stalls
// the whole workgroup, and a true struct over the cap is parsed exactly by the walkers.
constexpr uint32_t PARSE_QUEUE_STEPS = 96;
constexpr uint32_t PHALO = 1024;
constexpr uint32_t PQUEUE = 1024;              // general-parser queue entries per slice                // bytes staged past the slice (structs crossing its end)
constexpr uint32_t NB = 72;                     // content refs 1..9 x info>>5

// ---- the speculative struct sizer (k_parse). Exact on every valid struct; on other bytes it only
// has to be deterministic: the walkers follow nxt from true struct starts only, and every struct
// on the true chain is re-parsed exactly by k_struct_decode, which reports a malformed one.
// The info byte's class (content ref, origin / right origin / parentSub bits) is wave-uniform
// (positions are tiled per class), so the field layout costs scalar branches, and varuints are
// read branch-free from an 8-byte register window.
__device__ __forceinline__ uint64_t win8(const uint8_t* __restrict__ b, uint32_t p) {
  const uint32_t* d = (const uint32_t*)(b + (p & ~3u));  // the batch buffer is padded past its end
  return ((uint64_t)d[0] | ((uint64_t)d[1] << 32)) >> ((p & 3u) * 8);
}
// Byte sources for the sizer: the slice's bytes staged in LDS (plus a halo past its end), with
// a fallback to the batch buffer (through the caches) for reads beyond the staged window.
struct LdsSrc {
  const uint8_t* __restrict__ b;
  const uint32_t* lw;  // staged words of [s0, wend)
  uint32_t s0, wlen;   // wlen = wend - s0
  __device__ __forceinline__ uint32_t u8(uint32_t p) const {
    const uint32_t o = p - s0;
    return o < wlen ? (lw[o >> 2] >> ((o & 3u) * 8)) & 0xFFu : (uint32_t)b[p];
  }
  __device__ __forceinline__ uint64_t w8(uint32_t p) const {
    const uint32_t o = p - s0;
    if (o + 8 <= wlen) return ((uint64_t)lw[o >> 2] | ((uint64_t)lw[(o >> 2) + 1] << 32)) >> ((o & 3u) * 8);
    return win8(b, p);
  }
};
template <class S>
__device__ __forceinline__ uint32_t vu_fast(const S& b, uint32_t& p, uint32_t end, bool& ok) {
  const uint64_t w = b.w8(p);
  const uint64_t t = ~w & 0x8080808080ull;  // terminal bytes among the first five
  const uint32_t len = t ? ((uint32_t)__builtin_ctzll(t) >> 3) + 1 : 6u;
  uint64_t v = (w & 0x7full) | ((w >> 1) & (0x7full << 7)) | ((w >> 2) & (0x7full << 14)) | ((w >> 3) & (0x7full << 21)) |
               ((w >> 4) & (0x7full << 28));
  v &= len >= 5 ? ~0ull : ((1ull << (7 * len)) - 1);
  ok = ok && len <= 5 && end - p >= len && p < end;
  p += len;
  return (uint32_t)v;  // lib0 0.2.42 accumulates in 32 bits
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
// struct length, 0 = not a struct, 1 = hand over to parse_struct (many elements, deep nesting, Doc)
template <class S>
__device__ __forceinline__ uint32_t spec_len(const S& b, uint32_t pos, uint32_t end, uint32_t cls) {
  const uint32_t ref = cls / 8 + 1, bits = (cls % 8) << 5;
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
    case REF_JSON: {
      const uint32_t n = vu_fast(b, p, end, ok);
      if (ok && n > SIZER_MAX_ELEMS) return 1;
      for (uint32_t i = 0; i < n && ok; ++i) {
        const uint32_t k = vu_fast(b, p, end, ok);
        ok = ok && k > 0 && p < end && json_start_ok(b.u8(p));
        skip_n(p, k, end, ok);
      }
      break;
    }
    case REF_ANY: {
      const uint32_t n = vu_fast(b, p, end, ok);
      if (ok && n > SIZER_MAX_ELEMS) return 1;
      for (uint32_t i = 0; i < n && ok; ++i) {
        const uint32_t q0 = p;
        if (any_simple(b, p, end, ok)) continue;
        // a container one level deep with simple members; anything deeper goes to parse_struct
        const bool obj = b.u8(q0) == 118;
        const uint32_t m = vu_fast(b, p, end, ok);
        if (ok && m > SIZER_MAX_ELEMS) return 1;
        for (uint32_t j = 0; j < m && ok; ++j) {
          if (obj) { const uint32_t k = vu_fast(b, p, end, ok); skip_n(p, k, end, ok); }
          if (!any_simple(b, p, end, ok)) return ok ? 1u : 0u;
        }
      }
      break;
    }
    default: return 1;  // ContentDoc
  }
  if (!ok) return 0;
  return p - pos < 0x10000u ? p - pos : 1u;
}

__global__ __launch_bounds__(PL) void k_parse(Work w) {
  const uint8_t* __restrict__ b = w.bytes;
  const Group G = w.groups[blockIdx.x / (GROUP_BYTES / PSLICE)];
  const uint32_t s0 = G.start + (blockIdx.x % (GROUP_BYTES / PSLICE)) * PSLICE;
  if (s0 >= G.end) return;
  unsigned long long* dbg = w.dbg ? w.dbg + (size_t)w.ngroups * 8 + (size_t)blockIdx.x * 8 : nullptr;
  if (dbg && threadIdx.x == 0) { dbg[0] = wall_clock64(); dbg[1] = clock64(); }
  const uint32_t len = min(G.end - s0, PSLICE), uend = G.uend;
  uint16_t* __restrict__ out = w.tab.nxt + s0;
  __shared__ uint32_t bstart[NB + 1], bcursor[NB], tstart[NB + 1], qn;
  __shared__ uint16_t sorted[PSLICE], queue[PQUEUE];
  __shared__ uint32_t lw[(PSLICE + PHALO) / 4 + 2];
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  // stage the slice + halo in LDS: the byte-serial varuint chains then wait on LDS, not on L2
  const uint32_t wlen = min(uend - s0, PSLICE + PHALO);
  const uint32_t* __restrict__ gw = (const uint32_t*)(b + s0);  // s0 is 64-byte aligned
  for (uint32_t i = tid; i < (wlen + 3) / 4; i += PL) lw[i] = gw[i];
  const LdsSrc src{b, lw, s0, wlen};
  for (uint32_t i = tid; i < NB; i += PL) bcursor[i] = 0;
  if (tid == 0) qn = 0;
  __syncthreads();
  for (uint32_t o = tid; o < len; o += PL) {  // GC / Skip (info + one varuint) resolved on the spot
    const uint32_t info = (lw[o >> 2] >> ((o & 3u) * 8)) & 0xFFu;
    const uint32_t ref = info & 31u;
    uint16_t d = 0;
    if (ref == REF_GC || ref == REF_SKIP) {
      uint32_t q = s0 + o + 1;
      bool okv = true;
      rd_vu(b, q, uend, okv);
      d = okv ? (uint16_t)(q - s0 - o) : (uint16_t)0;
    } else if (ref <= REF_DOC) {
      atomicAdd(&bcursor[(ref - 1) * 8 + (info >> 5)], 1u);
    }
    out[o] = d;
  }
  __syncthreads();
  if (dbg && tid == 0) dbg[2] = clock64();
  if (wave == 0) {  // class starts and 64-position tiles per class: a wavefront scan over NB classes
    uint32_t acc = 0, tiles = 0;
    for (uint32_t base = 0; base < NB; base += 64) {
      const uint32_t i = base + lane;
      const uint32_t c = i < NB ? bcursor[i] : 0u, tc = (c + 63) / 64;
      uint32_t x = c, y = tc;  // inclusive scans
#pragma unroll
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t xo = __shfl_up(x, d), yo = __shfl_up(y, d);
        if (lane >= d) { x += xo; y += yo; }
      }
      if (i < NB) { bstart[i] = acc + x - c; bcursor[i] = acc + x - c; tstart[i] = tiles + y - tc; }
      acc += __shfl(x, 63);
      tiles += __shfl(y, 63);
    }
    if (lane == 0) { bstart[NB] = acc; tstart[NB] = tiles; }
  }
  __syncthreads();
  for (uint32_t o = tid; o < len; o += PL) {
    const uint32_t info = (lw[o >> 2] >> ((o & 3u) * 8)) & 0xFFu;
    const uint32_t ref = info & 31u;
    if (ref >= 1 && ref <= REF_DOC) sorted[atomicAdd(&bcursor[(ref - 1) * 8 + (info >> 5)], 1u)] = (uint16_t)o;
  }
  __syncthreads();
  if (dbg && tid == 0) dbg[3] = clock64();
  // every wavefront sizes tiles of ONE class: the class is a scalar for the whole parse
  const uint32_t ntiles = tstart[NB];
  for (uint32_t t = wave; t < ntiles; t += PL / 64) {
    uint32_t lo = 0, hi = NB;  // last class c with tstart[c] <= t
    while (hi - lo > 1) { const uint32_t m = (lo + hi) >> 1; if (tstart[m] <= t) lo = m; else hi = m; }
    const uint32_t c = __builtin_amdgcn_readfirstlane(lo);
    const uint32_t i = bstart[c] + (t - tstart[c]) * 64 + lane;
    if (i < bstart[c + 1]) {
      const uint32_t o = sorted[i];
      const uint32_t d = spec_len(src, s0 + o, uend, c);
      if (d == 1) {  // over the queue's capacity the position stays handed over (1) to the walkers
        const uint32_t k = atomicAdd(&qn, 1u);
        if (k < PQUEUE) queue[k] = (uint16_t)o;
      }
      out[o] = (uint16_t)d;
    }
  }
  __syncthreads();
  if (dbg && tid == 0) dbg[4] = clock64();
  const uint32_t nq = min(qn, PQUEUE);  // the general parser under a work cap for what the sizer handed over
  for (uint32_t i = tid; i < nq; i += PL) {
    const uint32_t o = queue[i];
    uint32_t q = s0 + o;
    const int r = parse_struct<false, 4>(b, q, uend, PARSE_QUEUE_STEPS, nullptr);
    out[o] = r > 0 ? (q - s0 - o < 0x10000u ? (uint16_t)(q - s0 - o) : (uint16_t)1) : (r == -1 ? (uint16_t)1 : (uint16_t)0);
  }
  if (dbg) {
    __syncthreads();
    if (tid == 0) { dbg[5] = clock64(); dbg[6] = wall_clock64(); dbg[7] = ((unsigned long long)nq << 32) | ntiles; }
  }
}
// --------------------------------------------------------------------------- 1b. chain tables
// For every byte position p of a group, from nxt: the chain summaries (first chain position
// at/after the end of p's chunk / block / group, number of chain positions visited before it)
// computed by backward dynamic programming (list ranking) in LDS. Table positions are 15 bits
// (STOPF marks a chain that stops at a struct the tables could not size).
constexpr uint32_t TL = 1024;                   // lanes per table workgroup
constexpr uint32_t BLOCK = 1024;                // 16 chunks
constexpr uint32_t LDS_NXT = 0, LDS_CEXIT = 32768, LDS_CCNT = 65536, LDS_BEXIT = 81920, LDS_BCNT = 114688;
constexpr uint32_t LDS_BM = 147456, LDS_TASK = LDS_BM + 2048;  // single-group walk: bitmap words, pieces
constexpr uint32_t MAXTASK = 2048;
constexpr uint32_t LDS_TOTAL = LDS_TASK + 4 * MAXTASK;             // 157,696 B of the 160 KiB
static_assert(GROUP_BYTES == 16384, "table layout assumes 16 KiB groups");

__global__ __launch_bounds__(TL) void k_tables(Work w) {
  const uint8_t* __restrict__ b = w.bytes;
  const Group* __restrict__ groups = w.groups;
  const Tables& t = w.tab;
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_TOTAL];
  uint16_t* nxt = (uint16_t*)(lds + LDS_NXT);
  uint16_t* cexit = (uint16_t*)(lds + LDS_CEXIT);
  uint8_t* ccnt = (uint8_t*)(lds + LDS_CCNT);
  uint16_t* bexit = (uint16_t*)(lds + LDS_BEXIT);
  uint16_t* bcnt = (uint16_t*)(lds + LDS_BCNT);
  uint16_t* gexit = nxt;                        // group level overlays nxt / cexit (phase D)
  uint16_t* gcnt = cexit;
  const Group G = groups[blockIdx.x];
  const uint32_t tid = threadIdx.x;
  if (w.dbg && tid == 0) w.dbg[blockIdx.x * 8 + 0] = clock64();
  const uint32_t glen = G.end - G.start;
  for (uint32_t o = tid; o < glen; o += TL) nxt[o] = t.nxt[G.start + o];
  __syncthreads();
  if (w.dbg && tid == 0) { w.dbg[blockIdx.x * 8 + 1] = w.dbg[blockIdx.x * 8 + 2] = w.dbg[blockIdx.x * 8 + 3] = clock64(); }
  // phase B: chunk level by pointer doubling over all positions (6 rounds cover a 64-byte chunk),
  // double-buffered through the block-array region (free again once the bytes are parsed); reads
  // are mostly unit-stride across a wavefront, unlike a lane-per-chunk backward sweep.
  {
    uint16_t* e0 = cexit;
    uint8_t* c0 = ccnt;
    uint16_t* e1 = bexit;
    uint8_t* c1 = (uint8_t*)bcnt;
    for (uint32_t o = tid; o < glen; o += TL) {
      const uint32_t d = nxt[o];
      if (d == 1 || o + d >= STOPF) { e0[o] = (uint16_t)(o | STOPF); c0[o] = 0; }  // sized by an exact parse
      else { e0[o] = (uint16_t)(d == 0 ? o + 1 : o + d); c0[o] = 1; }
    }
    __syncthreads();
#pragma unroll 1
    for (int round = 0; round < 6; ++round) {
      for (uint32_t o = tid; o < glen; o += TL) {
        const uint32_t ce = min((o | (CHUNK - 1)) + 1, glen);
        const uint32_t x = e0[o];
        uint32_t ex = x, cx = c0[o];
        if (!(x & STOPF) && x < ce) { ex = e0[x]; cx += c0[x]; }
        e1[o] = (uint16_t)ex;
        c1[o] = (uint8_t)cx;
      }
      __syncthreads();
      uint16_t* te = e0; e0 = e1; e1 = te;
      uint8_t* tc = c0; c0 = c1; c1 = tc;
    }
    static_assert(6 % 2 == 0, "an even number of rounds leaves the result in cexit/ccnt");
  }
  // phase C: block level (chunk s of every block, s = 15..0), from the chunk level
  for (int s = 15; s >= 0; --s) {
    for (uint32_t i = tid; i < 16 * CHUNK; i += TL) {
      const uint32_t blk = i / CHUNK;
      const uint32_t o = blk * BLOCK + (uint32_t)s * CHUNK + (i % CHUNK);
      if (o >= glen) continue;
      const uint32_t bend = min((blk + 1) * BLOCK, glen);
      const uint32_t x = cexit[o];
      if ((x & STOPF) || x >= bend) { bexit[o] = (uint16_t)x; bcnt[o] = ccnt[o]; }
      else { bexit[o] = bexit[x]; bcnt[o] = (uint16_t)(ccnt[o] + bcnt[x]); }
    }
    __syncthreads();
  }
  if (w.dbg && tid == 0) w.dbg[blockIdx.x * 8 + 4] = clock64();
  // ---- an update that fits in one group is walked right here (its tables never leave LDS): lane 0
  // follows the true chain through the section headers by block exits (1 KiB per step), then chunk
  // exits, queueing (position, count) chain pieces; then one lane per piece marks its struct starts
  // into an LDS copy of the final bitmap (the update owns its 64-byte-aligned words exclusively) —
  // k_walker / k_mark skip it.
  if (G.start == w.uoff[G.upd] && G.end == G.uend) {
    uint64_t* bm = (uint64_t*)(lds + LDS_BM);   // 256 words
    uint32_t* task = (uint32_t*)(lds + LDS_TASK);  // (position << 11 | count), count <= 1024
    __shared__ uint32_t ntask;
    const uint32_t nwords_g = (glen + 63) / 64;
    for (uint32_t i = tid; i < nwords_g; i += TL) bm[i] = 0;
    if (tid == 0) ntask = 0;
    __syncthreads();
    if (tid == 0) {
      const uint32_t u = G.upd, uend = G.uend;
      uint32_t* err = &w.ctr->err;
      w.dsstart[u] = NONE;
      bool ok = true;
      uint32_t p = G.start;
      uint32_t nt = 0;
      // a chain piece: queued while there is room, else marked right here (many tiny sections)
      auto piece = [&](uint32_t o, uint32_t cnt) {
        if (nt < MAXTASK) { task[nt++] = (o << 11) | cnt; return; }
        for (uint32_t k = 0; k < cnt; ++k) {
          bm[o >> 6] |= 1ull << (o & 63);
          const uint32_t d = nxt[o];
          o += d == 0 ? 1 : d;
        }
      };
      const uint32_t nsec = rd_vu(b, p, uend, ok);
      if (!ok || nsec > (uend - p) / 3 + 1) { raise_err(err, ERR_DECODE); goto done; }
      {
        const uint32_t sbase = atomicAdd(&w.ctr->nsections, nsec);
        if (sbase + nsec > w.cap_sections) { raise_err(err, ERR_CAPACITY); goto done; }
        w.usec_start[u] = sbase;
        w.usec_n[u] = nsec;
        for (uint32_t sct = 0; sct < nsec; ++sct) {
          const uint32_t n = rd_vu(b, p, uend, ok);
          const uint32_t client = rd_vu(b, p, uend, ok);
          const uint32_t clock = rd_vu(b, p, uend, ok);
          if (!ok || n > uend - p) { raise_err(err, ERR_DECODE); goto done; }
          Section sec;
          sec.upd = u; sec.n = n; sec.client = client; sec.clock = clock;
          sec.first_pos = n ? p : NONE; sec.cidx = NONE; sec.first_idx = NONE; sec.pad = 0;
          w.sections[sbase + sct] = sec;
          if (n) atomicOr((unsigned long long*)&w.sec_bits[p >> 6], 1ull << (p & 63));
          uint32_t r = n;
          uint32_t o = p - G.start;
          while (r > 0) {
            if (o >= glen) { raise_err(err, ERR_DECODE); goto done; }
            for (;;) {  // whole block pieces of the chain
              const uint32_t be = bexit[o], bc = bcnt[o];
              if ((be & STOPF) || bc >= r || bc == 0) break;
              piece(o, bc);
              r -= bc;
              o = be;
              if (o >= glen) break;
            }
            if (r == 0 || o >= glen) continue;
            for (;;) {  // whole chunk pieces
              const uint32_t ce = cexit[o], cc = ccnt[o];
              if ((ce & STOPF) || cc >= r || cc == 0) break;
              piece(o, cc);
              r -= cc;
              o = ce;
              if (o >= glen) break;
            }
            if (r == 0) break;
            if (o >= glen) { raise_err(err, ERR_DECODE); goto done; }
            // one struct: sized by the table, or parsed exactly (long / unsized struct)
            const uint32_t d = nxt[o];
            uint32_t q = G.start + o;
            if (d == 1) {
              if (parse_struct<false>(b, q, uend, 0xFFFFFFFFu, nullptr) <= 0) { raise_err(err, ERR_DECODE); w.ctr->err_info = G.start + o; goto done; }
            } else if (d == 0) { raise_err(err, ERR_DECODE); goto done; }
            else q += d;
            bm[o >> 6] |= 1ull << (o & 63);
            o = q - G.start;
            --r;
          }
          p = G.start + o;
        }
        w.dsstart[u] = p;
      }
    done:
      ntask = nt;
    }
    __syncthreads();
    const uint32_t nt = ntask;
    for (uint32_t i = tid; i < nt; i += TL) {
      uint32_t x = task[i] >> 11, left = task[i] & 0x7FFu;
      uint32_t word = x >> 6;
      uint64_t m = 0;
      while (left > 0) {
        if ((x >> 6) != word) { atomicOr((unsigned long long*)&bm[word], (unsigned long long)m); word = x >> 6; m = 0; }
        m |= 1ull << (x & 63);
        const uint32_t d = nxt[x];
        x += d == 0 ? 1 : d;
        --left;
      }
      atomicOr((unsigned long long*)&bm[word], (unsigned long long)m);
    }
    __syncthreads();
    for (uint32_t i = tid; i < nwords_g; i += TL) w.final_bits[(G.start >> 6) + i] = bm[i];
    if (w.dbg && tid == 0) w.dbg[blockIdx.x * 8 + 5] = clock64();
    return;
  }
  // exits are stored as forward deltas from the position itself (|STOPF when the chain stops at a
  // struct the tables could not size), so consumers never need the group origin
  for (uint32_t o = tid; o < glen; o += TL) {
    t.cexit[G.start + o] = (uint16_t)(((cexit[o] & 0x7FFFu) - o) | (cexit[o] & STOPF));
    t.ccnt[G.start + o] = ccnt[o];
  }
  for (uint32_t o = tid; o < glen; o += TL) {
    t.bexit[G.start + o] = (uint16_t)(((bexit[o] & 0x7FFFu) - o) | (bexit[o] & STOPF));
    t.bcnt[G.start + o] = bcnt[o];
  }
  // phase D: group level (block s = 15..0); gexit/gcnt overlay nxt/cexit (already written out)
  for (int s = 15; s >= 0; --s) {
    for (uint32_t i = tid; i < BLOCK; i += TL) {
      const uint32_t o = (uint32_t)s * BLOCK + i;
      if (o >= glen) continue;
      const uint32_t x = bexit[o];
      if ((x & STOPF) || x >= glen) { gexit[o] = (uint16_t)x; gcnt[o] = bcnt[o]; }
      else { gexit[o] = gexit[x]; gcnt[o] = (uint16_t)(bcnt[o] + gcnt[x]); }
    }
    __syncthreads();
  }
  for (uint32_t o = tid; o < glen; o += TL) {
    t.gexit[G.start + o] = (uint16_t)(((gexit[o] & 0x7FFFu) - o) | (gexit[o] & STOPF));
    t.gcnt[G.start + o] = gcnt[o];
  }
}

void launch_group_parse(const Work& w, hipStream_t s) {
  if (w.ngroups) hipLaunchKernelGGL(k_parse, dim3(w.ngroups * (GROUP_BYTES / PSLICE)), dim3(PL), 0, s, w);
}
void launch_group_tables(const Work& w, hipStream_t s) {
  if (w.ngroups) hipLaunchKernelGGL(k_tables, dim3(w.ngroups), dim3(TL), 0, s, w);
}

// --------------------------------------------------------------------------- 2. walker
// One lane per update follows the true struct chain through the section headers: a whole group
// per step while the current section continues past it (gexit/gcnt), descending to block /
// chunk / struct granularity only where a section ends. It emits verified chain segments
// (start, count) for k_mark and exact positions (long structs, final steps) as patches.
__device__ __forceinline__ bool emit_seg(const Work& w, uint32_t x, uint32_t n) {
  const uint32_t i = atomicAdd(&w.ctr->ncopy, 1u);
  if (i >= w.cap_copy) { raise_err(&w.ctr->err, ERR_CAPACITY); return false; }
  w.copy[i] = CopyTask{x, n};
  return true;
}
__device__ __forceinline__ bool emit_patch(const Work& w, uint32_t p) {
  const uint32_t i = atomicAdd(&w.ctr->npatch, 1u);
  if (i >= w.cap_patch) { raise_err(&w.ctr->err, ERR_CAPACITY); return false; }
  w.patch[i] = p;
  return true;
}

// One wavefront per multi-group update. The header / descent logic runs uniformly on every lane
// (lane 0 stores); the group-to-group jumps of a long section are speculated 64 groups at a time:
// lane j takes the exit S_j of the chain that starts at its group's first byte; the true chain
// enters group j+1 at S_j as soon as it has synchronised with that chain inside group j, which
// lane j checks by looking up the exit of its (true) entry. The first lane that fails still knows
// its true exit, so a failed speculation costs one group, exactly the sequential step.
__global__ __launch_bounds__(64) void k_walker(Work w) {
  if (blockIdx.x >= w.nbig) return;
  const uint32_t u = w.ulist[blockIdx.x];
  const uint32_t lane = threadIdx.x;
  if (w.ulen[u] > 0 && w.ulen[u] <= GROUP_BYTES) return;  // walked inside k_tables
  const uint8_t* __restrict__ b = w.bytes;
  const Tables& T = w.tab;
  const uint32_t ustart = w.uoff[u];
  const uint32_t uend = ustart + w.ulen[u];
  const uint32_t ngu = (w.ulen[u] + GROUP_BYTES - 1) / GROUP_BYTES;
  uint32_t* err = &w.ctr->err;
  const bool L0 = lane == 0;
  if (L0) w.dsstart[u] = NONE;
  uint32_t p = ustart;
  bool ok = true;
  const uint32_t nsec = rd_vu(b, p, uend, ok);
  if (!ok || nsec > (uend - p) / 3 + 1) { if (L0) raise_err(err, ERR_DECODE); return; }
  uint32_t sbase = 0;
  if (L0) sbase = atomicAdd(&w.ctr->nsections, nsec);
  sbase = __shfl(sbase, 0);
  if (sbase + nsec > w.cap_sections) { if (L0) raise_err(err, ERR_CAPACITY); return; }
  if (L0) { w.usec_start[u] = sbase; w.usec_n[u] = nsec; }
  for (uint32_t sct = 0; sct < nsec; ++sct) {
    const uint32_t n = rd_vu(b, p, uend, ok);
    const uint32_t client = rd_vu(b, p, uend, ok);
    const uint32_t clock = rd_vu(b, p, uend, ok);
    if (!ok || n > uend - p) { if (L0) raise_err(err, ERR_DECODE); return; }
    if (L0) {
      Section sec;
      sec.upd = u; sec.n = n; sec.client = client; sec.clock = clock;
      sec.first_pos = n ? p : NONE; sec.cidx = NONE; sec.first_idx = NONE; sec.pad = 0;
      w.sections[sbase + sct] = sec;
      if (n) atomicOr((unsigned long long*)&w.sec_bits[p >> 6], 1ull << (p & 63));
    }
    uint32_t r = n;
    while (r > 0) {
      if (p >= uend) { if (L0) raise_err(err, ERR_DECODE); return; }
      bool exact = false;
      if (T.gcnt[p] < r) {  // the section continues past this group: speculate 64 groups ahead
        const uint32_t gi = (p - ustart) / GROUP_BYTES + lane;
        uint32_t S = NONE;
        if (gi < ngu) {
          const uint32_t gs = ustart + gi * GROUP_BYTES;
          const uint32_t x = T.gexit[gs];
          if (!(x & STOPF)) S = gs + (x & 0x7FFFu);
        }
        uint32_t E = __shfl_up(S, 1);
        if (lane == 0) E = p;
        uint32_t X = NONE, C = 0;
        bool stop = true;
        if (E != NONE && E < uend && gi < ngu) {
          const uint32_t ge = T.gexit[E];
          C = T.gcnt[E];
          X = E + (ge & 0x7FFFu);
          stop = (ge & STOPF) != 0;
        }
        const bool good = !stop && X == S;
        const uint64_t bad = __ballot(!good);
        const uint32_t f = bad ? (uint32_t)__ffsll((long long)bad) - 1 : 63u;  // lanes 0..f hold true entries
        // inclusive count scan over lanes 0..f
        uint32_t incl = lane <= f ? C : 0u;
        for (uint32_t off = 1; off < 64; off <<= 1) {
          const uint32_t v = __shfl_up(incl, off);
          if (lane >= off) incl += v;
        }
        const uint32_t excl = incl - (lane <= f ? C : 0u);
        const uint64_t ends = __ballot(lane <= f && incl >= r);
        if (ends) {  // the section ends in the group of lane j
          const uint32_t j = (uint32_t)__ffsll((long long)ends) - 1;
          if (lane < j && C && !emit_seg(w, E, C)) return;
          r -= __shfl(excl, j);
          p = __shfl(E, j);
        } else {
          if (lane <= f && C && !emit_seg(w, E, C)) return;
          r -= __shfl(incl, f);
          p = __shfl(X, f);
          exact = __shfl(stop ? 1u : 0u, f) != 0;
          if (p == NONE) { if (L0) raise_err(err, ERR_DECODE); return; }
          if (!exact) continue;
        }
      }
      if (!exact) {  // the section ends inside this group: descend block -> chunk -> struct
        uint32_t rr = r;
        for (;;) {
          const uint32_t be = T.bexit[p], bc = T.bcnt[p];
          if ((be & STOPF) || bc >= rr) break;
          if (L0 && !emit_seg(w, p, bc)) return;
          rr -= bc;
          p += be;
        }
        for (;;) {
          const uint32_t ce = T.cexit[p], cc = T.ccnt[p];
          if ((ce & STOPF) || cc >= rr) break;
          if (L0 && !emit_seg(w, p, cc)) return;
          rr -= cc;
          p += ce;
        }
        while (rr > 0) {
          const uint32_t d = T.nxt[p];
          if (d == 1) { exact = true; break; }
          if (d == 0) { if (L0) raise_err(err, ERR_DECODE); return; }
          if (L0 && !emit_patch(w, p)) return;
          p += d;
          --rr;
        }
        r = rr;
      }
      if (exact && r > 0) {  // a struct the tables could not size: parse it exactly
        if (L0 && !emit_patch(w, p)) return;
        uint32_t q = p;
        if (parse_struct<false>(b, q, uend, 0xFFFFFFFFu, nullptr) <= 0) { if (L0) { raise_err(err, ERR_DECODE); w.ctr->err_info = p; } return; }
        p = q;
        --r;
      }
    }
  }
  if (L0) w.dsstart[u] = p;
}

// Direct path: one lane per small update parses it exactly, struct by struct, and writes the
// update's struct-start words of the final bitmap itself (updates are 64-byte aligned, so the
// words are the lane's own: plain stores, each word once, as the lane moves forward). Each lane
// reads its update through a private LDS window of DW bytes, refilled with 16-byte loads when
// fewer than DREFILL bytes are left: the byte-serial parse then waits on LDS, not on L2 / HBM
// (a wavefront touches 64 different updates, far more lines than L1 keeps). Structs are sized by
// the speculative sizer (exact on valid structs); what it hands over is parsed by parse_struct.
constexpr uint32_t DW = 128;                    // window bytes per lane
constexpr uint32_t DSTRIDE = DW / 4 + 4;        // words per lane slot (16-byte padded)
constexpr uint32_t DREFILL = 48;
constexpr uint32_t DL = 256;                    // lanes per direct workgroup
// the exact parser out of line: inlined, its nested-`any` walker multiplies the register demand
// of the lane loop (one wavefront per SIMD), and it only runs on the few handed-over structs
__device__ __attribute__((noinline)) uint32_t exact_len(const uint8_t* __restrict__ b, uint32_t p, uint32_t end) {
  uint32_t q = p;
  return parse_struct<false>(b, q, end, 0xFFFFFFFFu, nullptr) > 0 ? q - p : 0u;
}
__global__ __launch_bounds__(DL) void k_direct(Work w) {
  __shared__ __attribute__((aligned(16))) uint32_t win[DL * DSTRIDE];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= w.nsmall) return;
  const uint32_t u = w.ulist[w.nbig + i];
  const uint8_t* __restrict__ b = w.bytes;
  const uint32_t ustart = w.uoff[u], uend = ustart + w.ulen[u];
  uint32_t* err = &w.ctr->err;
  uint32_t* slot = win + threadIdx.x * DSTRIDE;
  LdsSrc src{b, slot, 0, 0};
  auto refill = [&](uint32_t p) {
    src.s0 = p & ~15u;
    src.wlen = min(DW, (uend + 15u - src.s0) & ~15u);
    const uint4* g = (const uint4*)(b + src.s0);
    for (uint32_t k = 0; k < src.wlen / 16; ++k) ((uint4*)slot)[k] = g[k];
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
    if (n) atomicOr((unsigned long long*)&w.sec_bits[p >> 6], 1ull << (p & 63));
    for (uint32_t k = 0; k < n; ++k) {
      if (p >= uend) { raise_err(err, ERR_DECODE); w.ctr->err_info = p; return; }
      if ((p >> 6) != word) {
        if (word != NONE) w.final_bits[word] = m;
        word = p >> 6;
        m = 0;
      }
      m |= 1ull << (p & 63);
      if (p - src.s0 + DREFILL > src.wlen) refill(p);
      const uint32_t info = src.u8(p), ref = info & 31u;
      uint32_t d = 0;
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
      p += d;
    }
  }
  if (word != NONE) w.final_bits[word] = m;
  w.dsstart[u] = p;
}

void launch_walker(const Work& w, hipStream_t s) {
  if (w.nbig) hipLaunchKernelGGL(k_walker, dim3(w.nbig), dim3(64), 0, s, w);
}
void launch_direct(const Work& w, hipStream_t s) {
  if (w.nsmall) hipLaunchKernelGGL(k_direct, dim3((w.nsmall + DL - 1) / DL), dim3(DL), 0, s, w);
}

// --------------------------------------------------------------------------- 3. final bitmap
// One wavefront per verified segment (x, n): block hops by lane 0, chunk hops by one lane per
// block, then one lane per chunk walks nxt inside its 64-byte chunk and sets the bits of that
// chunk's bitmap word with a single atomicOr.
__global__ __launch_bounds__(256) void k_mark(Work w) {
  __shared__ uint32_t s_bx[4][16], s_bn[4][16];          // block spans per wave
  __shared__ uint32_t s_cx[4][256], s_cn[4][256];        // chunk spans per wave
  __shared__ uint32_t s_nb[4], s_nc[4][16];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t nseg = min(w.ctr->ncopy, w.cap_copy);  // read on the device: no host sync
  // block-stride loop; the trip count depends on blockIdx only, so every wave reaches the barriers
  for (uint32_t blk = blockIdx.x; blk * 4 < nseg; blk += gridDim.x) {
  const uint32_t si = blk * 4 + wv;
  const bool active = si < nseg;
  CopyTask S{0, 0};
  if (active) S = w.copy[si];
  const Tables& T = w.tab;
  if (lane == 0) {  // block spans of the segment (segments never cross a group)
    uint32_t x = S.a, left = active ? S.b : 0, nb = 0;
    while (left > 0 && nb < 16) {
      const uint32_t take = min((uint32_t)T.bcnt[x], left);
      s_bx[wv][nb] = x;
      s_bn[wv][nb] = take;
      ++nb;
      left -= take;
      if (left) x += T.bexit[x] & 0x7FFFu;
    }
    s_nb[wv] = nb;
  }
  __syncthreads();
  const uint32_t nb = s_nb[wv];
  if (lane < nb) {
    uint32_t x = s_bx[wv][lane], left = s_bn[wv][lane], nc = 0;
    while (left > 0 && nc < 16) {
      const uint32_t cc = T.ccnt[x];
      const uint32_t take = min(cc, left);
      s_cx[wv][lane * 16 + nc] = x; s_cn[wv][lane * 16 + nc] = take; ++nc;
      left -= take;
      if (left) x += T.cexit[x] & 0x7FFFu;
    }
    s_nc[wv][lane] = nc;
  }
  __syncthreads();
  for (uint32_t k = lane; k < nb * 16; k += 64) {
    const uint32_t bi = k >> 4, ci = k & 15;
    if (ci >= s_nc[wv][bi]) continue;
    uint32_t x = s_cx[wv][k], left = s_cn[wv][k];
    uint64_t m = 0;
    const uint32_t word = x >> 6;
    while (left > 0) {
      m |= 1ull << (x & 63);
      const uint32_t d = T.nxt[x];
      x += d == 0 ? 1 : d;
      --left;
    }
    atomicOr((unsigned long long*)&w.final_bits[word], (unsigned long long)m);
  }
  __syncthreads();  // the LDS span lists are reused by the next iteration
  }
}
__global__ void k_patch(const uint32_t* __restrict__ patch, const uint32_t* __restrict__ npatch, uint32_t cap, uint64_t* __restrict__ final_bits) {
  const uint32_t n = min(*npatch, cap);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t p = patch[i];
    atomicOr((unsigned long long*)&final_bits[p >> 6], 1ull << (p & 63));
  }
}

// segment / patch counts are read on the device (grid-stride), so the walker needs no host sync
void launch_build_final_bits(const Work& w, hipStream_t s) {
  const uint32_t grid = std::min<uint32_t>(w.ngroups * 4 + 64, 8192);
  hipLaunchKernelGGL(k_mark, dim3(grid), dim3(256), 0, s, w);
  hipLaunchKernelGGL(k_patch, dim3(std::min<uint32_t>(w.ngroups * 4 + 64, 4096)), dim3(256), 0, s, w.patch, &w.ctr->npatch,
                     w.cap_patch, w.final_bits);
}

// --------------------------------------------------------------------------- 4. struct positions
__global__ void k_popc(const uint64_t* __restrict__ bits, uint32_t* __restrict__ cnt, uint32_t nwords) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nwords) cnt[i] = (uint32_t)__popcll(bits[i]);
  else if (i == nwords) cnt[i] = 0;
}
__global__ void k_scatter_pos(const uint64_t* __restrict__ bits, const uint32_t* __restrict__ pre, uint32_t nwords,
                              uint32_t* __restrict__ out, uint32_t cap, uint32_t* err) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nwords) return;
  uint64_t x = bits[i];
  uint32_t k = pre[i];
  while (x) {
    const uint32_t bit = (uint32_t)__ffsll((long long)x) - 1;
    x &= x - 1;
    if (k >= cap) { raise_err(err, ERR_CAPACITY); return; }
    out[k++] = i * 64 + bit;
  }
}
__device__ __forceinline__ uint32_t rank_incl(const uint64_t* __restrict__ bits, const uint32_t* __restrict__ pre, uint32_t p) {
  return pre[p >> 6] + (uint32_t)__popcll(bits[p >> 6] & (((2ull << (p & 63)) - 1)));  // bits <= p
}
__global__ void k_section_rank(Work w, uint32_t nsections) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsections) return;
  Section* sec = &w.sections[i];
  if (sec->n == 0) return;
  const uint32_t p = sec->first_pos;
  if (!((w.final_bits[p >> 6] >> (p & 63)) & 1ull)) { raise_err(&w.ctr->err, ERR_DECODE); return; }
  sec->first_idx = rank_incl(w.final_bits, w.wcnt, p) - 1;
  w.sec_sorted[rank_incl(w.sec_bits, w.wsec, p) - 1] = i;
}
__global__ void k_struct_sec(Work w, uint32_t nstructs) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nstructs) return;
  const uint32_t p = w.s_pos[i];
  w.s_sec[i] = w.sec_sorted[rank_incl(w.sec_bits, w.wsec, p) - 1];
}

// before the count sync: struct / section-start counts (popcount prefix of the bitmaps)
void launch_struct_count(const Work& w, hipStream_t s) {
  const uint32_t nwords = (w.nbytes + 63) / 64;
  hipLaunchKernelGGL(k_popc, dim3(nwords / 256 + 1), dim3(256), 0, s, w.final_bits, w.scratch, nwords);
  scan_u32(w.tmp, w.tmp_bytes, w.scratch, w.wcnt, nwords + 1, s);
  hipLaunchKernelGGL(k_popc, dim3(nwords / 256 + 1), dim3(256), 0, s, w.sec_bits, w.scratch, nwords);
  scan_u32(w.tmp, w.tmp_bytes, w.scratch, w.wsec, nwords + 1, s);
}
// after it (the struct table is sized from the count): dense struct positions
void launch_struct_scatter(const Work& w, hipStream_t s) {
  const uint32_t nwords = (w.nbytes + 63) / 64;
  hipLaunchKernelGGL(k_scatter_pos, dim3(nwords / 256 + 1), dim3(256), 0, s, w.final_bits, w.wcnt, nwords, w.s_pos,
                     w.cap_structs, &w.ctr->err);
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
  const uint8_t* __restrict__ b = w.bytes;
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
  if (lane == 0) w.ds_count[u] = obase - obase0;
}

__global__ void k_ds_bound(Work w) {  // region size per update: (delete-set bytes + 1) / 2
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u > w.nupd) return;
  if (u == w.nupd) { w.scratch[u] = 0; w.ds_count[u] = 0; return; }
  const uint32_t st = w.dsstart[u];
  w.scratch[u] = st == NONE ? 0 : (w.uoff[u] + w.ulen[u] - st + 1) / 2;
  w.ds_count[u] = 0;
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
void launch_ds_decode(const Work& w, hipStream_t s) {
  if (w.nupd == 0) return;
  hipLaunchKernelGGL(k_ds_decode, dim3((w.nupd + 3) / 4), dim3(256), 0, s, w);
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
                                 uint32_t* __restrict__ out, uint32_t* nout) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && (i == 0 || v[i] != v[i - 1])) out[pre[i]] = v[i];
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
  }
  if (i == n) w.ctr->nclients = w.cl_tmp[n];
}
__global__ void k_section_cidx_multi(Work w, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) w.sections[i].cidx = find_client(w, w.ctr->nclients, w.udoc[w.sections[i].upd], w.sections[i].client);
}

// NC stays on the device (ctr->nclients) until the struct-decode counter read
void launch_client_table(Work& w, uint32_t nsections, hipStream_t s) {
  const uint32_t grid = nsections / 256 + 1;
  if (w.udoc) {
    hipLaunchKernelGGL(k_gather_sec_keys, dim3(grid), dim3(256), 0, s, w, nsections);
    sort_pairs_u64_u32(w.tmp, w.tmp_bytes, w.cl_key2, w.cl_key, w.cl_tmp, w.cl_state, nsections, s);
    hipLaunchKernelGGL(k_unique_keys, dim3(grid), dim3(256), 0, s, w, nsections);
    scan_u32(w.tmp, w.tmp_bytes, w.scratch, w.cl_tmp, nsections + 1, s);
    hipLaunchKernelGGL(k_unique_keys_scatter, dim3(grid), dim3(256), 0, s, w, nsections);
    hipMemcpyAsync(w.cl_key, w.cl_key2, sizeof(uint64_t) * nsections, hipMemcpyDeviceToDevice, s);
    hipLaunchKernelGGL(k_section_cidx_multi, dim3(grid), dim3(256), 0, s, w, nsections);
    return;
  }
  hipLaunchKernelGGL(k_gather_sec_clients, dim3(grid), dim3(256), 0, s, w.sections, nsections, w.cl_tmp);
  sort_u32(w.tmp, w.tmp_bytes, w.cl_tmp, w.cl_vals, nsections, s);
  hipLaunchKernelGGL(k_unique_flags, dim3(grid), dim3(256), 0, s, w.cl_vals, nsections, w.scratch);
  scan_u32(w.tmp, w.tmp_bytes, w.scratch, w.cl_tmp, nsections + 1, s);
  // compact in place is unsafe; use cl_state as scratch output, then copy back
  hipLaunchKernelGGL(k_unique_scatter, dim3(grid), dim3(256), 0, s, w.cl_vals, w.cl_tmp, nsections, w.cl_state, &w.ctr->nclients);
  hipMemcpyAsync(w.cl_vals, w.cl_state, sizeof(uint32_t) * nsections, hipMemcpyDeviceToDevice, s);
  hipLaunchKernelGGL(k_section_cidx, dim3(grid), dim3(256), 0, s, w.sections, nsections, w.cl_vals, &w.ctr->nclients);
}

// --------------------------------------------------------------------------- 6. struct decode

__global__ __launch_bounds__(256) void k_struct_decode(Work w, uint32_t nstructs) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nstructs) return;
  const uint32_t nclients = w.ctr->nclients;
  uint32_t* err = &w.ctr->err;
  const uint32_t p0 = w.s_pos[i];
  const Section sec = w.sections[w.s_sec[i]];
  const uint32_t uend = w.uoff[sec.upd] + w.ulen[sec.upd];
  const uint32_t doc = doc_of_update(w, sec.upd);
  StructView v;
  uint32_t p = p0;
  if (parse_struct<true>(w.bytes, p, uend, 0xFFFFFFFFu, &v) <= 0) { raise_err(err, ERR_DECODE); return; }
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
  w.s_ocidx[i] = oc;
  w.s_oclock[i] = v.ok_;
  w.s_rcidx[i] = rc;
  w.s_rclock[i] = v.rk;
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
  wave_count_add(&w.ctr->nroots, pk != 0);
  w.s_pk[i] = (uint8_t)pk;
  w.s_pa[i] = pa;
  w.s_pb[i] = pb;
  w.s_psub[i] = (item && v.has_psub) ? v.psub_pos : NONE;
  w.s_psublen[i] = v.psub_len;
  w.s_cpos[i] = v.cpos;
  w.s_cend[i] = v.cend;
  uint32_t celem = v.cpos;
  if (v.ref == REF_ANY || v.ref == REF_JSON) celem += vu_size(v.nel);
  w.s_celem[i] = celem;
}

__global__ void k_struct_clock(Work w, uint32_t nstructs) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nstructs) return;
  const Section sec = w.sections[w.s_sec[i]];
  const uint64_t off = w.s_lenscan[i] - w.s_lenscan[sec.first_idx];
  const uint64_t clock = (uint64_t)sec.clock + off;
  const uint64_t endc = clock + w.s_len[i];
  if (endc > 0xFFFFFFFFull) { raise_err(&w.ctr->err, ERR_DECODE); return; }
  w.s_clock[i] = (uint32_t)clock;
}

void launch_struct_decode(const Work& w, uint32_t nstructs, hipStream_t s) {
  if (!nstructs) return;
  hipLaunchKernelGGL(k_struct_sec, dim3((nstructs + 255) / 256), dim3(256), 0, s, w, nstructs);
  hipLaunchKernelGGL(k_struct_decode, dim3((nstructs + 255) / 256), dim3(256), 0, s, w, nstructs);
  scan_u32_to_u64(w.tmp, w.tmp_bytes, w.s_len, w.s_lenscan, nstructs + 1, s);
  hipLaunchKernelGGL(k_struct_clock, dim3((nstructs + 255) / 256), dim3(256), 0, s, w, nstructs);
}

// --------------------------------------------------------------------------- client states
__global__ void k_states(Work w, uint32_t nstructs) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nstructs) return;
  if ((w.s_info[i] & 31u) == REF_SKIP) {  // rare: Skip lengths are subtracted from the item count
    atomicAdd(&w.ctr->items, (unsigned long long)w.s_len[i]);
    return;
  }
  // clocks grow along a section: only the last non-skip struct of a run can hold the max
  const bool last = i + 1 == nstructs || w.s_sec[i + 1] != w.s_sec[i] || (w.s_info[i + 1] & 31u) == REF_SKIP;
  if (last) atomicMax(&w.cl_state[w.s_cidx[i]], w.s_clock[i] + w.s_len[i]);
}
// Yjs pending structs (yc_ingest.h): every client is integrated up to its cap only
__global__ void k_apply_caps(Work w) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= w.ctr->nclients) return;
  const uint32_t v = w.cl_vals[c];
  const uint32_t i = lower_bound_u32(w.cap_client, w.ncaps, v);
  const uint32_t cap = (i < w.ncaps && w.cap_client[i] == v) ? w.cap_clock[i] : 0u;
  if (w.cl_state[c] > cap) w.cl_state[c] = cap;
}
__global__ void k_state_totals(Work w, uint32_t nstructs) {  // U and Σ input lengths into the counters
  w.ctr->units = w.cl_base[w.ctr->nclients];
  w.ctr->in_len = w.s_lenscan[nstructs];
}
// NC <= nsections: the states are zero past NC, so a scan over nsections + 1 entries gives cl_base
void launch_states(const Work& w, uint32_t nstructs, uint32_t nsections, hipStream_t s) {
  hipMemsetAsync(w.cl_state, 0, sizeof(uint32_t) * (nsections + 1), s);
  if (nstructs) hipLaunchKernelGGL(k_states, dim3((nstructs + 255) / 256), dim3(256), 0, s, w, nstructs);
  if (w.capped && nsections) hipLaunchKernelGGL(k_apply_caps, dim3(nsections / 256 + 1), dim3(256), 0, s, w);
  scan_u32_to_u64(w.tmp, w.tmp_bytes, w.cl_state, w.cl_base, nsections + 1, s);
  hipLaunchKernelGGL(k_state_totals, dim3(1), dim3(1), 0, s, w, nstructs);
}

}  // namespace yc
