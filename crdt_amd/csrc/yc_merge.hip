// yc_merge.hip — K2..K6: dedupe, delete sets, segmentation and the YMap winner on gfx950.
//
// All state is indexed by the dense *unit* index g = cl_base[client] + clock (one unit per
// (client, clock) of the merged store), so every step below is a flat, coalesced pass:
//   k_owner        dedupe (integrateStructs offset logic, Y@19963): each unit takes its struct
//                  from the earliest update that carries it (atomicMin over struct index)
//   k_ds_apply     delete-set application (readAndApplyDeleteSet, Y@11619) as unit flags
//   k_refs         split points required by origin / rightOrigin references (getItemCleanEnd /
//                  getItemCleanStart, Y@29100) + min child client per unit (list adjacency)
//   k_cuts         struct boundaries -> bitmap; popcount scan -> segments
//   k_seg_props    per-segment origin / rightOrigin / parent / flags; first pass of the YMap
//                  winner reduction (plain stores of a child into its origin's slot)
//   k_resolve      parent+parentSub resolution (Item.getMissing, Y@76507): climb the origin chain
//                  with path halving; list kind; YATA for map entries (Item.integrate, Y@77594):
//                  children ordered by client ⇒ the rightmost entry is the max-client descent from
//                  the max-client root (settling pass of the max-child reduction)
//   k_winner_walk  per key: descend along the max-client child to the rightmost entry
//   k_overwrite    every non-rightmost entry of a key is deleted (typeMapSet / left.delete)
//   k_merge_flags  Item.mergeWith (Y@79424) / tryToMergeWithLeft (Y@30960) as a pairwise
//                  predicate over adjacent segments ⇒ canonical (maximally merged) structs
#include <algorithm>
#include <cstdlib>

#include "yc_work.h"

namespace yc {



// --------------------------------------------------------------------------- owner / dedupe
// One lane per struct (one per delete-set range below): a struct's units are consecutive in the
// merged store, so a wave's atomics on short structs hit consecutive addresses; structs longer than
// LONG_UNITS are covered by the whole wavefront, one at a time. (A lane per unit pair had to find
// its struct by a binary search over all structs: ~27 dependent loads per lane at C2 x 112.)
constexpr uint32_t LONG_UNITS = 32;
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int l) {
  return ((uint64_t)(uint32_t)__shfl((uint32_t)(v >> 32), l) << 32) | (uint32_t)__shfl((uint32_t)v, l);
}
__device__ __forceinline__ void unit_owner(const Work& w, uint32_t nstructs, uint32_t s) {
  const uint32_t lane = threadIdx.x & 63;
  uint64_t gb = 0;
  uint32_t n = 0, fl = 0;
  if (s < nstructs) {
    const uint32_t ref = w.s_info[s] & 31u, cidx = w.s_cidx[s], clock = w.s_clock[s], len = w.s_len[s];
    const uint32_t st = w.cl_state[cidx];
    const uint64_t cb = w.cl_base[cidx];
    if (ref != REF_SKIP) {
      // units at or past the client's (capped) state stay out of the store
      n = st > clock ? min(len, st - clock) : 0u;
      gb = cb + clock;
      fl = ref == REF_DELETED ? UF_DEL : (ref == REF_GC ? (UF_GC | UF_DEL) : 0u);
    }
  }
  // a client whose structs all come from one section (one update) owns its units alone: plain
  // stores (its structs cover disjoint clock ranges); otherwise the earliest struct wins by atomicMin
  const bool one = n && w.cl_single && w.cl_single[w.s_cidx[s]];
  const bool lng = n > LONG_UNITS;
  if (!lng)
    for (uint32_t k = 0; k < n; ++k) {
      if (one) {
        w.u_owner[(uint32_t)(gb + k)] = s;
        if (fl) reinterpret_cast<uint8_t*>(w.u_flags)[(size_t)(uint32_t)(gb + k) * 4] = (uint8_t)fl;  // byte 0 (UF_DEL | UF_GC)
      } else {
        atomicMin(&w.u_owner[(uint32_t)(gb + k)], s);
        if (fl) atomicOr(&w.u_flags[(uint32_t)(gb + k)], fl);
      }
    }
  for (uint64_t m = __ballot(lng); m; m &= m - 1) {
    const int L = __ffsll((long long)m) - 1;
    const uint64_t g0 = shfl64(gb, L);
    const uint32_t nl = __shfl(n, L), fll = __shfl(fl, L), sl = __shfl(s, L);
    const bool onel = __shfl((int)one, L) != 0;
    for (uint32_t k = lane; k < nl; k += 64) {
      if (onel) {
        w.u_owner[(uint32_t)(g0 + k)] = sl;
        if (fll) reinterpret_cast<uint8_t*>(w.u_flags)[(size_t)(uint32_t)(g0 + k) * 4] = (uint8_t)fll;
      } else {
        atomicMin(&w.u_owner[(uint32_t)(g0 + k)], sl);
        if (fll) atomicOr(&w.u_flags[(uint32_t)(g0 + k)], fll);
      }
    }
  }
}

// --------------------------------------------------------------------------- delete sets
// UF_DS and UF_CUT own a byte of the unit's flag word each, so their writers store that byte
// (no read-modify-write round trip); concurrent stores of the same byte write the same value
__device__ __forceinline__ void set_flag_byte(uint32_t* u_flags, uint32_t g, uint32_t byte) {
  reinterpret_cast<uint8_t*>(u_flags)[(size_t)g * 4 + byte] = 1;
}
// a unit's flag byte (YCRDT_DEBUG_BOUNDS: the unit checked against the unit table first)
__device__ __forceinline__ void unit_flag(const Work& w, uint64_t g, uint32_t byte) {
  if (w.dbg_bounds && g >= w.cap_units) { bounds_fail(w.ctr, BOUNDS_UNIT); return; }
  set_flag_byte(w.u_flags, (uint32_t)g, byte);
}
// The delete sets of a merge, straight from the decoder's per-update regions (no compaction): one
// wavefront per update resolves its ranges' clients, clips them to the known states (pendingDs)
// and marks the units (the prep and mark passes above in one, for the integrate path)
// one range: its units' first index and length, clipped to the client's known state (a range
// past it is Yjs's pendingDs: an error here — the host then takes the pending path —, clipped
// silently when the host already computed the caps)
__device__ __forceinline__ uint32_t ds_range_units(const Work& w, uint32_t nclients, uint32_t doc, const DsRange& r, uint64_t& gb) {
  uint32_t len = r.len;
  gb = 0;
  if (!len) return 0;
  const uint32_t c = find_client(w, nclients, doc, r.client);
  if (c == NONE) {
    if (!w.capped) raise_err(&w.ctr->err, ERR_PENDING);
    return 0;
  }
  const uint32_t st = w.cl_state[c];
  if ((uint64_t)r.clock + len > st) {
    if (!w.capped) raise_err(&w.ctr->err, ERR_PENDING);
    len = r.clock < st ? st - r.clock : 0;
  }
  gb = w.cl_base[c] + r.clock;
  return len;
}
// a run of nl units from g0, by the whole wavefront: with ds_tails (a large delete set) a run past
// DS_TAIL_MIN units flags its first DS_TAIL_MIN and hands the rest to k_ds_tails, which spreads it
// over the grid (a C2 document's state holds runs of ~90 k units: 1 400 steps of one wavefront)
__device__ __forceinline__ void ds_run_wave(const Work& w, uint64_t g0, uint32_t nl, uint32_t lane) {
  if (w.ds_tails && nl > DS_TAIL_MIN) {
    uint32_t slot = 0;
    if (lane == 0) slot = atomicAdd(&w.ctr->ds_ntails, 1u);
    slot = __shfl(slot, 0);
    if (slot < DS_TAILS_CAP) {
      if (lane == 0) {
        const uint64_t gt = g0 + DS_TAIL_MIN;
        w.ds_tails[slot] = make_uint4((uint32_t)gt, (uint32_t)(gt >> 32), nl - DS_TAIL_MIN, 0u);
      }
      nl = DS_TAIL_MIN;
    }
  }
  for (uint32_t k = lane; k < nl; k += 64) unit_flag(w, (uint32_t)(g0 + k), 1);
}
// a wavefront applies the first DSA_WAVE ranges of its update; a large update's delete set (a
// full state as one update: C3's 156 MB state holds a million ranges) is spread over the extra
// workgroups of k_units (unit_ds_apply_big)
__device__ __forceinline__ void unit_ds_apply(const Work& w, uint32_t nclients, uint32_t blk, bool big) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t u = (blk * blockDim.x + threadIdx.x) >> 6;
  if (u >= w.nupd) return;
  // (with the spread apply on, an update past DSA_WAVE ranges is applied by it whole: its first
  // DSA_WAVE ranges were 64 dependent steps of this one wavefront, 0.15 ms on a C2 document's state)
  if (big && w.ds_count[u] > DSA_WAVE) return;
  const uint32_t n = min(w.ds_count[u], DSA_WAVE), base = w.ds_region[u];
  const uint32_t doc = doc_of_update(w, u);
  for (uint32_t i0 = 0; i0 < n; i0 += 64) {
    const uint32_t i = i0 + lane;
    uint64_t gb = 0;
    uint32_t len = 0;
    if (i < n) len = ds_range_units(w, nclients, doc, w.ds_tmp[base + i], gb);
    const bool lng = len > LONG_UNITS;
    if (!lng)
      for (uint32_t k = 0; k < len; ++k) unit_flag(w, (uint32_t)(gb + k), 1);
    for (uint64_t m = __ballot(lng); m; m &= m - 1) {  // (a delete set this size: no tails, ds_run_wave)
      const int L = __ffsll((long long)m) - 1;
      const uint64_t g0 = shfl64(gb, L);
      const uint32_t nl = __shfl(len, L);
      for (uint32_t k = lane; k < nl; k += 64) unit_flag(w, (uint32_t)(g0 + k), 1);
    }
  }
}

// --------------------------------------------------------------------------- reference cuts
__device__ __forceinline__ void unit_refs(const Work& w, uint32_t nstructs, uint32_t i) {
  if (i >= nstructs) return;
  // the struct's columns in one round of loads (the right-origin clock and the parent are written
  // only where present: read, used behind their presence tests), then the clients' states
  const uint32_t clock = w.s_clock[i], cidx = w.s_cidx[i], ref = w.s_info[i] & 31u, pk = w.s_pk[i] & 3u;
  const uint32_t oc = w.s_ocidx[i], ok_ = w.s_oclock[i], rc = w.s_rcidx[i], rk = w.s_rclock[i];
  const bool ov = oc < NONE - 1, rv = rc < NONE - 1;
  const uint32_t st = w.cl_state[cidx], ost = ov ? w.cl_state[oc] : 0u, rst = rv ? w.cl_state[rc] : 0u;
  const uint64_t ob = ov ? w.cl_base[oc] : 0ull, rb = rv ? w.cl_base[rc] : 0ull;
  if (clock >= st || ref == REF_SKIP) return;  // not integrated
  // own-client references at or past the item's own clock (scan_update refuses them on the host)
  if ((oc == cidx && ok_ >= clock) || (rc == cidx && rk >= clock) || (pk == 2 && w.s_pa[i] == cidx && w.s_pb[i] >= clock)) {
    raise_err(&w.ctr->err, ERR_DECODE);
    return;
  }
  // Item.getMissing (Y@76507): every reference of an integrated struct must be in the store
  if (pk == 2 && (w.s_pa[i] == UNKNOWN || w.s_pb[i] >= w.cl_state[w.s_pa[i]])) { raise_err(&w.ctr->err, ERR_PENDING); return; }
  if (oc != NONE) {
    if (oc == UNKNOWN || ok_ >= ost) { raise_err(&w.ctr->err, ERR_PENDING); return; }
    const uint32_t g = (uint32_t)(ob + ok_);
    if (ok_ + 1 < ost) unit_flag(w, g + 1, 2);  // getItemCleanEnd(origin)
  }
  if (rc != NONE) {
    if (rc == UNKNOWN || rk >= rst) { raise_err(&w.ctr->err, ERR_PENDING); return; }
    const uint32_t g = (uint32_t)(rb + rk);
    unit_flag(w, g, 2);                          // getItemCleanStart(rightOrigin)
  }
}
__device__ __forceinline__ bool cut_at(const Work& w, uint64_t g, uint64_t nunits) {
  bool cut = false;
  if (g < nunits) {
    const uint32_t own = w.u_owner[g];
    if (own == NONE) {
      raise_err(&w.ctr->err, ERR_PENDING);  // a gap in a client's clock range
    } else {
      // a struct's first unit needs no test of its own: the unit before it (if any) has another
      // owner — units of one struct are consecutive — and so does a client's first unit
      const uint32_t f = w.u_flags[g];
      cut = (f & UF_CUT) || g == 0;
      if (g > 0) {
        const uint32_t po = w.u_owner[g - 1];
        const uint32_t pf = w.u_flags[g - 1];
        cut |= po != own;
        const bool d = (f & (UF_DEL | UF_DS)) != 0, pd = (pf & (UF_DEL | UF_DS)) != 0;
        cut |= d != pd;
        cut |= ((f ^ pf) & UF_GC) != 0;
      }
    }
  }
  return cut;
}
__global__ __launch_bounds__(256) void k_cuts(Work w, uint64_t nunits) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool cut = cut_at(w, g, nunits);
  const uint64_t word = __ballot(cut);
  if ((threadIdx.x & 63) == 0) {  // the word and its popcount (the scan input of the segment numbering)
    const uint64_t wi = g >> 6;
    if (g < nunits) {
      w.u_cutbits[wi] = word;
      w.scratch[wi] = (uint32_t)__popcll(word);
    } else if (wi == (nunits + 63) / 64) {
      w.scratch[wi] = 0;
    }
  }
}
__device__ __forceinline__ void scatter_seg_at(const Work& w, uint32_t i, uint32_t nwords, uint64_t nunits) {
  if (i == 0) w.ctr->nsegs = w.u_wpre[nwords];  // the scan's total (no copy launch)
  if (i >= nwords) return;
  uint64_t x = w.u_cutbits[i];
  uint32_t k = w.u_wpre[i];
  while (x) {
    const uint32_t bit = (uint32_t)__ffsll((long long)x) - 1;
    x &= x - 1;
    w.g_start[k++] = i * 64 + bit;
  }
  if (i == nwords - 1) w.g_start[w.u_wpre[nwords]] = (uint32_t)nunits;  // sentinel
}
__global__ void k_scatter_seg(Work w, uint32_t nwords, uint64_t nunits) {
  scatter_seg_at(w, blockIdx.x * blockDim.x + threadIdx.x, nwords, nunits);
}
// Small batches: the cut words, their popcount prefix and the segment starts in ONE workgroup launch
// (three otherwise); a wavefront takes 64 consecutive units at a time, as in k_cuts
// (up to 16 K units: a unit's cut test gathers several columns, so one workgroup is only worth it
// while each lane takes a few units — a 900 K-unit C2 document spent 1 ms in it)
constexpr uint32_t SEG_LANES = 1024, SEG_SMALL_WORDS = 256;
template <uint32_t SEG_LANES>
__device__ __forceinline__ void segments_small_body(const Work& w, uint64_t nunits, uint32_t* part) {
  const uint32_t nwords = (uint32_t)((nunits + 63) / 64);
  for (uint32_t base = 0; base < nwords * 64; base += SEG_LANES) {
    const uint32_t g = base + threadIdx.x;
    const uint64_t word = __ballot(cut_at(w, g, nunits));
    if ((threadIdx.x & 63) == 0 && g < nunits) {
      w.u_cutbits[g >> 6] = word;
      w.scratch[g >> 6] = (uint32_t)__popcll(word);
    }
  }
  if (threadIdx.x == 0) w.scratch[nwords] = 0;
  __syncthreads();
  block_scan_u32<SEG_LANES>(w.scratch, w.u_wpre, nwords + 1, part);
  for (uint32_t i = threadIdx.x; i < nwords; i += SEG_LANES) scatter_seg_at(w, i, nwords, nunits);
}
__global__ __launch_bounds__(SEG_LANES) void k_segments_small(Work w, uint64_t nunits) {
  __shared__ uint32_t part[SEG_LANES];
  segments_small_body<SEG_LANES>(w, nunits, part);
}

// One launch for the three unit passes (they touch disjoint bytes of a unit's flag word: byte 0
// UF_DEL / UF_GC from the owner pass, byte 1 UF_DS from the delete sets, byte 2 UF_CUT from the
// references, every one of them a byte store or an atomic): workgroups [0, nb) take a struct each
// lane (owner, then references — the struct's columns are loaded once), the rest one update per
// wavefront (delete sets).
// the delete sets that hold more than DSA_WAVE ranges, whole, one lane per range (grid-stride over the
// extra workgroups). Any update can: a 16 KiB direct-path update of one transaction that deleted
// ~8 000 scattered items carries that many 2-byte ranges, so the list is every such update the
// decoders met (k_ds_decode, k_dsp_headers), not the chunk-path updates
// A wavefront takes 64 consecutive ranges; a long range (a full state's delete set holds runs of
// tens of thousands of units: C2's base client) is flagged by the whole wavefront, 64 units a step,
// as in unit_ds_apply — one lane walking it alone held k_units for 0.8 ms on a C2 document's state.
__device__ __forceinline__ void unit_ds_apply_big(const Work& w, uint32_t nclients, uint32_t blk, uint32_t nx) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = (blk * blockDim.x + threadIdx.x) >> 6, nwaves = nx * blockDim.x / 64;
  const uint32_t nlist = min(w.ctr->ds_big, w.nupd);
  // the 64-range slices of all listed delete sets, dealt to the wavefronts round-robin across the
  // updates (a wave per slice index within each update left most of the grid idle when many
  // updates hold a few thousand ranges each: C2's 112 snapshots)
  uint32_t gs = wave, before = 0;  // the next global slice of this wave; slices of the updates before bi
  for (uint32_t bi = 0; bi < nlist; ++bi) {
    const uint32_t u = w.ds_biglist[bi];
    const uint32_t n = w.ds_count[u];
    if (n <= DSA_WAVE) continue;
    const uint32_t ns = (n + 63) / 64;
    const uint32_t base = w.ds_region[u], doc = doc_of_update(w, u);
    for (; gs < before + ns; gs += nwaves) {  // (wave-uniform; every range: unit_ds_apply left them)
      const uint32_t i = (gs - before) * 64 + lane;
      uint64_t gb = 0;
      uint32_t len = 0;
      if (i < n) len = ds_range_units(w, nclients, doc, w.ds_tmp[base + i], gb);
      const bool lng = len > LONG_UNITS;
      if (!lng)
        for (uint32_t k = 0; k < len; ++k) unit_flag(w, (uint32_t)(gb + k), 1);
      for (uint64_t m = __ballot(lng); m; m &= m - 1) {
        const int L = __ffsll((long long)m) - 1;
        ds_run_wave(w, shfl64(gb, L), __shfl(len, L), lane);
      }
    }
    before += ns;
  }
}
// the tails of the long runs (ds_run_wave), every workgroup striding over each of them
__global__ __launch_bounds__(256) void k_ds_tails(Work w) {
  const uint32_t n = min(w.ctr->ds_ntails, DS_TAILS_CAP);
  for (uint32_t t = 0; t < n; ++t) {
    const uint4 T = w.ds_tails[t];
    const uint64_t g0 = (uint64_t)T.x | ((uint64_t)T.y << 32);
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < T.z; k += gridDim.x * blockDim.x) unit_flag(w, g0 + k, 1);
  }
}
// BIG: the batch holds a delete set of more than DSA_WAVE ranges (the spread workgroups exist). Two
// builds: the spread apply's registers (it walks a list and hands runs to k_ds_tails) cost the
// common case — the C2 headline, no such delete set — 0.15 ms of k_units when compiled in.
template <bool BIG>
__global__ __launch_bounds__(256) void k_units(Work w, uint32_t nstructs, uint32_t nclients, uint32_t nb, uint32_t nd, uint32_t nx) {
  if (blockIdx.x < nb) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    unit_owner(w, nstructs, s);
    unit_refs(w, nstructs, s);
  } else if (blockIdx.x < nb + nd) {
    unit_ds_apply(w, nclients, blockIdx.x - nb, BIG);
  } else if (BIG) {
    unit_ds_apply_big(w, nclients, blockIdx.x - nb - nd, nx);
  }
}
void launch_units_fill(const Work& w, uint64_t nunits, hipStream_t s) {
  fill_u32_multi({{w.u_owner, nunits, NONE}, {w.u_flags, nunits, 0u}}, s);
}
void launch_units(const Work& w, uint32_t nstructs, uint32_t nclients, uint32_t nds, uint64_t nunits, bool ds_big, hipStream_t s) {
  const uint32_t nb = (nstructs + 255) / 256, nd = nds && w.nupd ? (w.nupd + 3) / 4 : 0u;
  const uint32_t nx = nd && ds_big ? 256u : 0u;  // a delete set of more than DSA_WAVE ranges (k_dsp_headers says)
  if (nb + nd) {
    if (nx) hipLaunchKernelGGL(k_units<true>, dim3(nb + nd + nx), dim3(256), 0, s, w, nstructs, nclients, nb, nd, nx);
    else hipLaunchKernelGGL(k_units<false>, dim3(nb + nd), dim3(256), 0, s, w, nstructs, nclients, nb, nd, 0u);
  }
  if (nx && w.ds_tails) hipLaunchKernelGGL(k_ds_tails, dim3(512), dim3(256), 0, s, w);
}

void launch_segments(const Work& w, uint32_t nclients, uint64_t nunits, hipStream_t s) {
  const uint32_t nwords = (uint32_t)((nunits + 63) / 64);
  if (nwords <= SEG_SMALL_WORDS) {
    hipLaunchKernelGGL(k_segments_small, dim3(1), dim3(SEG_LANES), 0, s, w, nunits);
    return;
  }
  hipLaunchKernelGGL(k_cuts, dim3(nwords / 4 + 1), dim3(256), 0, s, w, nunits);
  scan_u32(w.tmp, w.tmp_bytes, w.scratch, w.u_wpre, nwords + 1, s);
  hipLaunchKernelGGL(k_scatter_seg, dim3(nwords / 256 + 1), dim3(256), 0, s, w, nwords, nunits);
}

// --------------------------------------------------------------------------- segment properties
__device__ __forceinline__ uint64_t fnv_bytes(uint64_t h, const uint8_t* __restrict__ p, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) { h ^= p[i]; h *= 1099511628211ull; }
  return h;
}
__device__ __forceinline__ bool bytes_eq(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i)
    if (a[i] != b[i]) return false;
  return true;
}
// Do root structs a and b name the same list? A list is (document, root type name | parent item,
// parentSub) (Item.integrate's parent / parentSub after Item.getMissing, Y@76507; typeMapSet keys,
// crdt.js:434). Names and parentSubs are compared as whole varStrings (length prefix included).
__device__ __forceinline__ bool same_list(const Work& w, uint32_t a, uint32_t b) {  // inline: a Work reference into an out-of-line call copies the whole Work to scratch
  if (a == b) return true;
  const uint32_t pk = w.s_pk[a] & 3u;
  if (pk != (w.s_pk[b] & 3u)) return false;
  if (pk == 1) {
    const uint32_t n = w.s_pb[a];
    if (n != w.s_pb[b]) return false;
    if (w.udoc && w.cl_doc[w.s_cidx[a]] != w.cl_doc[w.s_cidx[b]]) return false;
    if (!bytes_eq(struct_bytes(w, a) + w.s_pa[a], struct_bytes(w, b) + w.s_pa[b], n)) return false;
  } else if (w.s_pa[a] != w.s_pa[b] || w.s_pb[a] != w.s_pb[b]) {  // parent item id (client index, clock)
    return false;
  }
  const uint32_t pa = w.s_psub[a], pb = w.s_psub[b];
  if ((pa == NONE) != (pb == NONE)) return false;
  if (pa == NONE) return true;
  const uint32_t n = w.s_psublen[a];
  return n == w.s_psublen[b] && bytes_eq(struct_bytes(w, a) + pa, struct_bytes(w, b) + pb, n);
}
// Open-addressing insert of the list rooted by struct `own` with hash h. A slot's word is
// (claiming struct + 1) << 32 | low half of h, written by one CAS, so whoever meets a taken slot
// with the same low hash reads the claimer from the same word and compares the two lists' names
// exactly (same_list): equal hashes of different lists keep probing (no hash-only identity).
// Every struct of one list walks the same probe sequence, so the list gets exactly one slot.
__device__ __forceinline__ uint32_t key_insert(const Work& w, uint64_t h, uint32_t own) {
  uint64_t* __restrict__ tab = w.k_hash;
  const uint32_t cap = w.cap_keys;
  const uint64_t mine = ((uint64_t)(own + 1) << 32) | (uint32_t)h;
  uint32_t slot = (uint32_t)(h ^ (h >> 29)) & (cap - 1);
  for (uint32_t probe = 0; probe < cap; ++probe) {
    const unsigned long long old = atomicCAS((unsigned long long*)&tab[slot], 0ull, (unsigned long long)mine);
    if (old == 0ull || old == mine) return slot;
    if ((uint32_t)old == (uint32_t)h && same_list(w, (uint32_t)(old >> 32) - 1u, own)) return slot;
    slot = (slot + 1) & (cap - 1);
  }
  return NONE;
}

__device__ __forceinline__ uint64_t fnv_u32(uint64_t h, uint32_t v) {
  for (int i = 0; i < 4; ++i) { h ^= (v >> (8 * i)) & 0xFFu; h *= 1099511628211ull; }
  return h;
}

// Per segment: item vs GC, origin / right origin units, parent list. A root segment (no origin,
// no right origin) names its list: root type name or parent type item, plus the parentSub for
// YMap entries; every other item inherits the list from its origin (else right origin) by
// pointer jumping (Item.getMissing, Y@76507). An item whose origin / right origin is GC, or
// whose parent item is GC, is integrated as GC (getMissing sets parent = null).
__device__ __forceinline__ void seg_props_at(const Work& w, uint32_t s) {
  // the source struct's columns in one round of loads (the right-origin clock is unwritten when
  // there is none: read, never used), then the client bases
  const uint32_t g0 = seg_start(w, s);
  const uint32_t own = w.u_owner[g0];
  const uint32_t f = w.u_flags[g0];
  const uint32_t cidx = w.s_cidx[own], ref = w.s_info[own] & 31u, sclk = w.s_clock[own];
  const uint32_t socx = w.s_ocidx[own], socl = w.s_oclock[own], srcx = w.s_rcidx[own], srcl = w.s_rclock[own];
  const uint64_t ob = socx < NONE - 1 ? w.cl_base[socx] : 0ull, rb = srcx < NONE - 1 ? w.cl_base[srcx] : 0ull;
  const uint32_t k0 = (uint32_t)(g0 - w.cl_base[cidx]);
  uint32_t sf = 0;
  if (f & (UF_DEL | UF_DS)) sf |= SEG_DEL;
  bool gc = (f & UF_GC) || ref == REF_GC || socx == UNKNOWN || srcx == UNKNOWN;  // (unknown: k_refs raised PENDING)
  const bool expl = k0 == sclk;
  if (expl) sf |= SEG_EXPLICIT;
  uint32_t origin = NONE, rorigin = NONE;
  if (!gc) {
    if (expl) {
      if (socx != NONE) origin = (uint32_t)(ob + socl);
    } else origin = g0 - 1;
    if (srcx != NONE) rorigin = (uint32_t)(rb + srcl);
    // an item whose origin is GC becomes GC in k_resolve (its first hop lands on the GC segment,
    // Item.getMissing drops the parent); only a right origin needs the unit's flag here
    if (rorigin != NONE && (w.u_flags[rorigin] & UF_GC)) gc = true;
  }
  uint32_t key = NONE, link = s;
  if (!gc && origin == NONE && rorigin == NONE) {
    const uint32_t pk = w.s_pk[own] & 3u;
    uint64_t h = 1469598103934665603ull;
    uint32_t parent = NONE;
    if (pk == 1) {
      if (w.udoc) h = fnv_u32(h ^ 0x3Cu, w.cl_doc[cidx]);  // root types are per document
      h = fnv_bytes(h, struct_bytes(w, own) + w.s_pa[own], w.s_pb[own]);
    } else if (pk == 2) {
      const uint32_t pc = w.s_pa[own], pclock = w.s_pb[own];
      if (pc == NONE || pc == UNKNOWN || pclock >= w.cl_state[pc]) { raise_err(&w.ctr->err, ERR_PENDING); gc = true; }
      else {
        parent = (uint32_t)(w.cl_base[pc] + pclock);
        if (w.u_flags[parent] & UF_GC) gc = true;
        h = fnv_u32(h ^ 0xA5u, parent);
      }
    } else {
      raise_err(&w.ctr->err, ERR_DECODE);  // an item without origin, right origin or parent
      gc = true;
    }
    if (!gc) {
      const uint32_t ps = w.s_psub[own];
      if (ps != NONE) { h = fnv_u32(h, 0x5Au); h = fnv_bytes(h, struct_bytes(w, own) + ps, w.s_psublen[own]); }
      h &= w.key_mask;  // tests: YCRDT_KEY_HASH_BITS truncates the hash so distinct lists collide
      key = key_insert(w, h, own);
      if (key != NONE) YC_BOUND(w, key, w.cap_keys, BOUNDS_KEY);
      if (key == NONE) raise_err(&w.ctr->err, ERR_CAPACITY);
      else {
        sf |= SEG_ROOT;
        w.k_parent[key] = parent;  // every root of a list names the same parent
        if (ps != NONE) atomicOr(&w.k_flags[key], KF_PSUB);
      }
    }
  } else if (!gc) {
    link = seg_of_unit(w, origin != NONE ? origin : rorigin);
  }
  if (gc) sf |= SEG_GC | SEG_DEL;
  else sf |= SEG_ITEM;
  if (!gc && rorigin != NONE) sf |= SEG_HASRO;  // (a YMap entry item with one needs full YATA: k_resolve)
  const bool olow = !gc && expl && origin != NONE && socx < NONE - 1 && cidx < socx;
  if (olow) sf |= SEG_OLOW;
  // The YMap winner's max-client child / max-client root, first pass: a plain store of s + 1 into
  // the origin's (the key's) slot — one of the children lands there; k_resolve then raises the
  // slot with an atomicMax only where a child finds it below itself. Plain scattered stores merge
  // in L2 where the one-atomic-per-segment form (98 M memory-side atomics on the C2 batch, 4.9 ms)
  // was bound by the chip's atomic rate. Every item stores: its kind (YMap entry / YArray member)
  // is only known after k_resolve, and a YArray origin's slot is never read. A lower-client child
  // marks its origin unit (UF_LOWCHILD: no merge with the origin's own-client successor; read for
  // entries only).
  if (!gc && origin != NONE) {
    w.g_maxchild[link] = s + 1;
    if (olow) unit_flag(w, origin, 3);  // (UF_LOWCHILD)
  } else if (key != NONE) {
    w.k_rootmax[key] = s + 1;
  }
  w.g_cidx[s] = cidx;
  w.g_src[s] = own;
  w.g_origin[s] = gc ? NONE : origin;
  w.g_rorigin[s] = gc ? NONE : rorigin;
  // the climbing record (k_resolve writes the final flags and keys): a root's key carries its list
  // kind in bit 31 (k_resolve copies it whole down the chains and writes the final keys, without
  // the bit, to g_key); the origin's segment is the winner slot of a YMap entry
  const uint32_t kw = key != NONE && w.s_psub[own] != NONE ? key | KEY_PSUB : key;
  w.g_hop[s] = make_uint4(sf, kw, link, !gc && origin != NONE ? link : NONE);
}
__global__ __launch_bounds__(256) void k_seg_props(Work w, uint32_t nsegs) {
  const uint32_t s = gidx();
  if (s < nsegs) seg_props_at(w, s);
}

void launch_segment_props_fill(const Work& w, uint32_t nsegs, hipStream_t s) {
  fill_u32_multi({{(uint32_t*)w.k_hash, (uint64_t)w.cap_keys * 2, 0u},
                  {w.k_rootmax, (uint64_t)w.cap_keys, 0u},
                  {w.k_flags, w.cap_keys, 0u},
                  {w.k_parent, w.cap_keys, NONE},
                  {w.g_maxchild, (uint64_t)nsegs, 0u}}, s);
}
void launch_segment_props(const Work& w, uint32_t nsegs, uint32_t nclients, uint64_t nunits, hipStream_t s) {
  if (nsegs) hipLaunchKernelGGL(k_seg_props, dim3((nsegs + 255) / 256), dim3(256), 0, s, w, nsegs);
}

// --------------------------------------------------------------------------- key resolution
// One pass (Item.getMissing, Y@76507): every item that is not a list root climbs its origin chain
// to the first segment that knows its list, halving the path it walks (link[x] <- link[link[x]] is
// monotone: it only ever points further up the same chain, so concurrent halving is safe). The
// climb reads the keys of k_seg_props (g_tmp, with the list kind in bit 31); a resolved item
// publishes its key there for later climbers and writes its final key (bit cleared) to g_key, so
// no climber ever reads a key whose kind bit is gone. The item is then tagged YMap entry
// (parentSub) or YArray member, and a YMap entry settles its origin's max-client child slot (the
// second pass of the winner reduction begun in k_seg_props: an atomicMax only where the slot is
// below itself — segments are numbered in client order, so the max child is the max segment).
__device__ __forceinline__ bool resolve_at(const Work& w, uint32_t s, uint32_t nsegs) {
  const uint4 h = w.g_hop[s];  // flags, climbing key, link, origin segment
  uint32_t f = h.x;
  uint32_t kv = h.y;
  bool arr = false;
  if (f & SEG_ITEM) {
    if (kv == NONE) {  // not a root: climb
      uint32_t x = h.z;
      bool done = false;
      for (uint32_t it = 0; it <= nsegs; ++it) {  // more hops than segments: a cycle
        const uint4 hx = w.g_hop[x];  // one 16-B load per hop
        const uint32_t fx = hx.x, k = hx.y, y = hx.z;
        if (!(fx & SEG_ITEM)) {  // the origin chain ends in GC: getMissing drops the parent
          f = (f & ~SEG_ITEM) | SEG_GC | SEG_DEL;
          w.g_hop[s].x = f;
          w.g_origin[s] = NONE;
          w.g_rorigin[s] = NONE;
          done = true;
          break;
        }
        if (k != NONE) { kv = k; w.g_hop[s].y = k; done = true; break; }
        if (y == x) { done = true; break; }  // a chain without a root: reported below
        const uint32_t z = w.g_hop[y].z;
        if (z != y) w.g_hop[x].z = z;
        x = y;
      }
      if (!done) raise_err(&w.ctr->err, ERR_DECODE);  // an origin cycle
    }
    if (f & SEG_ITEM) {
      if (kv == NONE) raise_err(&w.ctr->err, ERR_DECODE);  // origin chain without a root
      else {
        arr = !(kv & KEY_PSUB);
        f |= arr ? SEG_ARRAY : SEG_PSUB;
        // a YMap entry item with a right origin (never written by typeMapSet: crafted input) — or
        // placed by one alone — is not ordered by the max-client descent: the whole entry takes the
        // YATA kernels (launch_mapx_flip / launch_mapx_fix)
        if (!arr && (f & SEG_HASRO)) { atomicOr(&w.k_flags[kv & ~KEY_PSUB], KF_YATA); w.ctr->nmapx = 1u; }
        if (!arr) {  // the winner reduction's settling pass (k_seg_props stored one child)
          uint32_t* slot = h.w != NONE ? &w.g_maxchild[h.w] : (f & SEG_ROOT) ? &w.k_rootmax[kv & ~KEY_PSUB] : nullptr;
          if (slot && *slot < s + 1) atomicMax(slot, s + 1);
        }
      }
    }
  }
  w.g_flags[s] = f & ~SEG_HASRO;
  w.g_key[s] = (f & SEG_ITEM) && kv != NONE ? kv & ~KEY_PSUB : NONE;
  return arr;
}
__global__ __launch_bounds__(256) void k_resolve(Work w, uint32_t nsegs) {
  const uint32_t s = gidx();
  if (s >= nsegs) return;
  wave_flag(&w.ctr->narray, resolve_at(w, s, nsegs));  // read as zero / non-zero (launch_yata)
}

// ---- YMap entries ordered by full YATA (KF_YATA keys). Yjs integrates a map entry's items by the
// same YATA loop as a YArray's (Item.integrate, Y@77594: the list starts at the entry's leftmost
// item), keeps the LAST one as the value (_map.set when right is null) and deletes every other
// (this.delete() when right is not null, left.delete() of the new last one). The descent over
// max-client children orders the origin-only shape typeMapSet writes; an entry with a right origin
// goes through the YArray kernels instead: flipped to SEG_ARRAY before the descent, back to
// SEG_PSUB after YATA with the last member as the winner (g_right == NONE) and every other deleted.
// The origin-tree order (yc_yata.hip) holds for the shapes Yjs's own histories have. One it does
// not: a right origin that is a split piece of another item (a segment starting inside its struct)
// while the item's origin is neither the unit before it — the piece's origin — nor a descendant of
// that unit (an item inserted between the two halves). Yjs integrated such an item before that split
// existed and may place it inside the split item; no replica can create that shape (it would have
// to see the piece without the item), and for a map entry — whose items never carry a right origin
// from typeMapSet — it only comes from corrupted or crafted bytes: refused (YCRDT_E_UNSUPPORTED)
// rather than merged into a state Yjs would not reach.
__device__ __forceinline__ bool origin_below(const Work& w, uint32_t o, uint32_t target, uint32_t nsegs) {
  for (uint32_t it = 0; it <= nsegs && o != NONE; ++it) {  // o: a unit; climb segment by segment
    const uint32_t so = seg_of_unit(w, o);
    if (target >= seg_start(w, so) && target <= o) return true;  // (the units before o in its segment are its ancestors)
    o = w.g_origin[so];
  }
  return false;
}
__global__ void k_mapx_flip(Work w, uint32_t nsegs) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsegs) return;
  const uint32_t f = w.g_flags[s];
  if (!(f & SEG_PSUB) || !(w.k_flags[w.g_key[s]] & KF_YATA)) return;
  const uint32_t r = w.g_rorigin[s];
  if (r != NONE && !(w.g_flags[seg_of_unit(w, r)] & SEG_EXPLICIT) && !origin_below(w, w.g_origin[s], r - 1, nsegs))
    raise_err(&w.ctr->err, ERR_UNSUPPORTED);
  w.g_flags[s] = (f & ~(SEG_PSUB | SEG_WIN)) | SEG_ARRAY | SEG_YMAPX;
}
__global__ void k_mapx_fix(Work w, uint32_t nsegs) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsegs) return;
  uint32_t f = w.g_flags[s];
  if ((f & (SEG_YMAPX | SEG_ITEM | SEG_ARRAY)) != (SEG_YMAPX | SEG_ITEM | SEG_ARRAY)) return;  // (GC / dead / another shard's)
  f = (f & ~(SEG_ARRAY | SEG_WIN)) | SEG_PSUB;
  if (w.g_right[s] == NONE) {
    f |= SEG_WIN;
    w.k_winner[w.g_key[s]] = s;
  } else {
    f |= SEG_DEL;
  }
  w.g_flags[s] = f;
}
void launch_mapx_flip(const Work& w, uint32_t nsegs, hipStream_t s) {
  if (nsegs) hipLaunchKernelGGL(k_mapx_flip, dim3(nsegs / 256 + 1), dim3(256), 0, s, w, nsegs);
}
void launch_mapx_fix(const Work& w, uint32_t nsegs, hipStream_t s) {
  if (nsegs) hipLaunchKernelGGL(k_mapx_fix, dim3(nsegs / 256 + 1), dim3(256), 0, s, w, nsegs);
}

uint32_t run_key_resolution(const Work& w, uint32_t nsegs, hipStream_t s) {
  if (!nsegs) return 0;
  hipLaunchKernelGGL(k_resolve, dim3((nsegs + 255) / 256), dim3(256), 0, s, w, nsegs);
  return 1;
}

// --------------------------------------------------------------------------- map winner
// Per YMap entry: the max-client child of its origin (the winner descent: YATA orders siblings by
// client, Item.integrate Y@77594) is computed by k_seg_props + k_resolve above, and whether its
// origin unit has a child of a lower client than the unit's own (then the origin's own-client
// successor is not adjacent to it: no merge) is marked in k_seg_props.
// the key's value is the rightmost entry: descend from the max-client root through the max-client
// child until a leaf (YATA order of an origin-only tree, SURVEY.md §7 hard part 2)
// (a descent visits every segment at most once: more hops than segments is a cycle, an error)
// (k_rootmax / k_flags / g_maxchild were last written by atomics: ld_fresh, for k_merge_small's
// barrier-separated phases)
__device__ __forceinline__ void winner_at(const Work& w, uint32_t k, uint32_t nsegs) {
  const uint32_t r = ld_fresh(&w.k_rootmax[k]);
  if (!r) { w.k_winner[k] = NONE; return; }
  if (ld_fresh(&w.k_flags[k]) & KF_YATA) { w.k_winner[k] = NONE; return; }  // ordered by the YATA kernels (k_mapx_fix writes the winner)
  uint32_t x = r - 1;
  bool leaf = false;
  for (uint32_t it = 0; it <= nsegs; ++it) {
    const uint32_t m = ld_fresh(&w.g_maxchild[x]);
    if (!m) { leaf = true; break; }
    x = m - 1;
  }
  if (!leaf) { raise_err(&w.ctr->err, ERR_DECODE); return; }
  w.k_winner[k] = x;
  w.g_flags[x] |= SEG_WIN;  // one winner per key: the only writer of x's flags in this kernel
}
__global__ void k_winner_walk(Work w, uint32_t nsegs) {
  const uint32_t k = gidx();
  if (k < w.cap_keys) winner_at(w, k, nsegs);
}
// every entry item but the winner is deleted (overwritten): a flag test, no gather of the key's winner
__global__ void k_overwrite(Work w, uint32_t nsegs) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsegs) return;
  const uint32_t f = w.g_flags[s];
  if ((f & (SEG_PSUB | SEG_WIN)) == SEG_PSUB) w.g_flags[s] = f | SEG_DEL;
}


uint32_t run_descent(const Work& w, uint32_t nsegs, hipStream_t s, bool fold) {
  if (!nsegs) return 0;
  hipLaunchKernelGGL(k_winner_walk, dim3(w.cap_keys / 256 + 1), dim3(256), 0, s, w, nsegs);
  if (!fold) hipLaunchKernelGGL(k_overwrite, dim3((nsegs + 255) / 256), dim3(256), 0, s, w, nsegs);
  return 1;
}

// --------------------------------------------------------------------------- deleted parent types
// ContentType.delete / gc (Y@73441): when a type's item is deleted, every item of that type is
// deleted and garbage-collected into GC structs (Item.gc with parentGCd, Y@75928); nested types
// recurse. A list is dead when its parent item is deleted / GC / not a type, or lies in a dead list.
__global__ void k_dead_init(Work w) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= w.cap_keys || w.k_hash[k] == 0) return;
  const uint32_t pu = w.k_parent[k];
  if (pu == NONE) return;
  const uint32_t p = seg_of_unit(w, pu);
  const uint32_t pf = w.g_flags[p];
  const bool is_type = (w.s_info[w.g_src[p]] & 31u) == REF_TYPE;
  if ((pf & SEG_DEL) || !(pf & SEG_ITEM) || !is_type) w.k_flags[k] |= KF_DEAD;
}
// every list climbs its chain of parent lists (nesting depth) to the first dead one, if any;
// KF_DEAD only ever gets set, so reading a flag another lane is setting is safe
__global__ void k_dead_climb(Work w) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= w.cap_keys || w.k_hash[k] == 0 || (w.k_flags[k] & KF_DEAD)) return;
  uint32_t x = k;
  for (uint32_t depth = 0; depth <= w.cap_keys; ++depth) {  // deeper than the key count: a cycle
    const uint32_t pu = w.k_parent[x];
    if (pu == NONE) return;  // a root type: alive
    const uint32_t pk = w.g_key[seg_of_unit(w, pu)];
    if (pk == NONE) return;
    if (w.k_flags[pk] & KF_DEAD) { atomicOr(&w.k_flags[k], KF_DEAD); return; }
    x = pk;
  }
  raise_err(&w.ctr->err, ERR_DECODE);
}
__global__ void k_dead_apply(Work w, uint32_t nsegs) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsegs) return;
  const uint32_t f = w.g_flags[s];
  if (!(f & SEG_ITEM)) return;
  const uint32_t key = w.g_key[s];
  if (key == NONE || (w.k_flags[key] & KF_DEAD))
    w.g_flags[s] = (f & ~(SEG_ITEM | SEG_ARRAY | SEG_PSUB | SEG_ROOT)) | SEG_GC | SEG_DEL;
}

void run_dead_keys(const Work& w, uint32_t nsegs, hipStream_t s) {
  if (!nsegs) return;
  const uint32_t kg = w.cap_keys / 256 + 1;
  hipLaunchKernelGGL(k_dead_init, dim3(kg), dim3(256), 0, s, w);
  hipLaunchKernelGGL(k_dead_climb, dim3(kg), dim3(256), 0, s, w);
  hipLaunchKernelGGL(k_dead_apply, dim3((nsegs + 255) / 256), dim3(256), 0, s, w, nsegs);
}

// --------------------------------------------------------------------------- merge flags
__device__ __forceinline__ bool seg_deleted(uint32_t f) { return (f & SEG_DEL) || !(f & SEG_ITEM); }  // in a delete set
__device__ __forceinline__ bool content_mergeable(uint32_t ref) {  // ContentX.mergeWith
  return ref == REF_ANY || ref == REF_JSON || ref == REF_STRING || ref == REF_DELETED;
}
// fold = 1: k_overwrite's deletion of the entry items that are not their key's winner is applied
// here, on the flags as they are read (when no dead-type pass sits between the two)
__device__ __forceinline__ uint32_t overwritten(uint32_t f, uint32_t fold) {
  return (fold && (f & (SEG_PSUB | SEG_WIN)) == SEG_PSUB) ? f | SEG_DEL : f;
}
// One lane per segment: the merge flag (s merges into its left neighbour) and the delete-set run
// starts. Either the flags go to g_tmp / r_size and launch_merge_tail / the encoder scan them, or
// (merge_flags_at's caller k_merge_flags_scan, the unsharded merge) their exclusive counts are made
// in the same pass.
__device__ __forceinline__ void merge_flags_at(const Work& w, uint32_t s, uint32_t fold, bool& start, bool& rstart) {
  bool merge = false;
  const uint32_t f0 = w.g_flags[s], fr = overwritten(f0, fold);
  if (s > 0 && w.g_cidx[s - 1] == w.g_cidx[s]) {
    const uint32_t fl = overwritten(w.g_flags[s - 1], fold);
    const uint32_t gs = seg_start(w, s);
    if ((fl & SEG_ITEM) == (fr & SEG_ITEM)) {
      if (!(fr & SEG_ITEM)) merge = true;  // GC + GC
      else if ((fl & SEG_DEL) == (fr & SEG_DEL) && w.g_origin[s] == gs - 1 && w.g_rorigin[s - 1] == w.g_rorigin[s] &&
               (fl & (SEG_ARRAY | SEG_PSUB)) == (fr & (SEG_ARRAY | SEG_PSUB)) &&
               ((fr & (SEG_ARRAY | SEG_YMAPX)) ? w.g_right[s - 1] == s : !(w.u_flags[gs - 1] & UF_LOWCHILD))) {
        if (fr & SEG_DEL) merge = true;  // both become ContentDeleted after GC
        else {
          const uint32_t rl = w.s_info[w.g_src[s - 1]] & 31u, rr = w.s_info[w.g_src[s]] & 31u;
          merge = rl == rr && content_mergeable(rr);
        }
      }
    }
  }
  const uint32_t f1 = merge ? fr | SEG_MERGE : fr;
  if (f1 != f0) w.g_flags[s] = f1;
  // the encode's delete-set runs (createDeleteSetFromStructStore): s starts a run of deleted
  // segments of one client — flagged here, where both final flags are in registers
  const bool del = seg_deleted(fr);
  const bool pdel = s > 0 && w.g_cidx[s - 1] == w.g_cidx[s] && seg_deleted(overwritten(w.g_flags[s - 1], fold));
  start = !merge;
  rstart = del && !pdel;
}
__global__ __launch_bounds__(256) void k_merge_flags(Work w, uint32_t nsegs, uint32_t fold) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s > nsegs) return;
  if (s == nsegs) { w.g_tmp[s] = 0; w.r_size[s] = 0; return; }
  bool start, rstart;
  merge_flags_at(w, s, fold, start, rstart);
  w.g_tmp[s] = start ? 1u : 0u;
  w.r_size[s] = rstart ? 1u : 0u;
}
// The same flags, and their exclusive counts — output struct ids (g_outid) and delete-set run ids
// (g_tmp2), entries [0, NS] (the last: the totals) — by a decoupled look-back per tile of MF_ITEMS
// x 256 segments (two chains), instead of two scan passes over flag columns. Segment
// tile * MF_TILE + k * 256 + t is lane t's k-th: coalesced, and the counts come from ballots.
constexpr uint32_t MF_ITEMS = 16, MF_TILE = 256 * MF_ITEMS;
__global__ __launch_bounds__(256) void k_merge_flags_scan(Work w, uint32_t nsegs, uint32_t fold, LbChains lb) {
  __shared__ uint32_t ca[MF_ITEMS][4], cb[MF_ITEMS][4];
  __shared__ uint32_t pa, pb;
  const uint32_t tile = ordered_block_id(lb.ord, lb.ord_base);
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t bits_a = 0, bits_b = 0;
#pragma unroll 4
  for (uint32_t k = 0; k < MF_ITEMS; ++k) {
    const uint32_t s = tile * MF_TILE + k * 256 + threadIdx.x;
    bool start = false, rstart = false;
    if (s < nsegs) merge_flags_at(w, s, fold, start, rstart);
    bits_a |= (start ? 1u : 0u) << k;
    bits_b |= (rstart ? 1u : 0u) << k;
    const uint64_t ba = __ballot(start), bb = __ballot(rstart);
    if (lane == 0) { ca[k][wv] = (uint32_t)__popcll(ba); cb[k][wv] = (uint32_t)__popcll(bb); }
  }
  __syncthreads();
  if (wv < 2) {
    uint32_t tot = 0;
    for (uint32_t i = lane; i < MF_ITEMS * 4; i += 64) tot += wv == 0 ? (&ca[0][0])[i] : (&cb[0][0])[i];
    for (uint32_t off = 32; off > 0; off >>= 1) tot += __shfl_xor(tot, off);
    const uint32_t p = (uint32_t)lb_wave_lookback(lb.state + (wv ? lb.stride : 0), tile, lb.epoch, tot);
    if (lane == 0) { if (wv == 0) pa = p; else pb = p; }
  }
  __syncthreads();
  uint32_t ra = pa, rb = pb;  // counts before lane t's k-th segment
  for (uint32_t k = 0; k < MF_ITEMS; ++k) {
    const uint64_t ba = __ballot((bits_a >> k) & 1u), bb = __ballot((bits_b >> k) & 1u);
    uint32_t oa = (uint32_t)__popcll(ba & lt), ob = (uint32_t)__popcll(bb & lt);
    for (uint32_t x = 0; x < 4; ++x) {
      if (x < wv) { oa += ca[k][x]; ob += cb[k][x]; }
    }
    const uint32_t s = tile * MF_TILE + k * 256 + threadIdx.x;
    if (s <= nsegs) {
      w.g_outid[s] = ra + oa;
      w.g_tmp2[s] = rb + ob;
    }
    for (uint32_t x = 0; x < 4; ++x) { ra += ca[k][x]; rb += cb[k][x]; }
  }
}
// ---- key-hash sharding of one document (C4). Every list — a YMap entry, a
// YArray — and every mergeWith adjacency lives inside ONE top-level entry of a root type (nested
// lists hang below their parent item's entry), so the integrate phases (map winner, dead types,
// YATA, item merge flags) are shard-local once each segment is owned by hash(top-level list) %
// shards. A shard runs them with the other shards' segments masked out (no YMap / YArray role),
// exports its own segments' final flags, and the flag words of all shards are summed (exactly one
// owner per segment; RCCL all-reduce across GPUs). GC runs merge regardless of lists, so their
// merge flags are settled afterwards on the combined flags (k_merge_final).
__device__ __forceinline__ uint32_t shard_of_hash(uint64_t h, uint32_t n) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  return (uint32_t)(h % n);
}
__global__ void k_key_shard(Work w, uint32_t nshards, uint32_t* __restrict__ key_shard) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= w.cap_keys) return;
  if (w.k_hash[k] == 0) { key_shard[k] = 0; return; }
  uint32_t x = k;  // climb to the top-level list: parent item -> the list that holds it
  bool top = false;
  for (uint32_t depth = 0; depth <= w.cap_keys; ++depth) {  // deeper than the key count: a cycle
    const uint32_t pu = w.k_parent[x];
    if (pu == NONE) { top = true; break; }
    const uint32_t pk = w.g_key[seg_of_unit(w, pu)];
    if (pk == NONE || pk == x) { top = true; break; }
    x = pk;
  }
  if (!top) raise_err(&w.ctr->err, ERR_DECODE);
  key_shard[k] = shard_of_hash((uint32_t)w.k_hash[x], nshards);  // the list's low hash half (slot words, key_insert)
}
__global__ void k_seg_shard(Work w, uint32_t nsegs, const uint32_t* __restrict__ key_shard, uint8_t* __restrict__ owner) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsegs) return;
  const uint32_t key = w.g_key[s];
  owner[s] = key == NONE ? 0 : (uint8_t)key_shard[key];  // keyless (GC) segments: shard 0
}
__global__ void k_shard_mask(Work w, uint32_t nsegs, const uint8_t* __restrict__ owner, uint32_t shard) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsegs || owner[s] == shard) return;
  w.g_flags[s] &= ~(SEG_PSUB | SEG_ARRAY | SEG_ROOT);
}
__global__ void k_shard_export(Work w, uint32_t nsegs, const uint8_t* __restrict__ owner, uint32_t shard, uint32_t* __restrict__ acc) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsegs || owner[s] != shard) return;
  acc[s] = w.g_flags[s];
}
__global__ void k_merge_final(Work w, uint32_t nsegs) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s > nsegs) return;
  if (s == nsegs) { w.g_tmp[s] = 0; w.r_size[s] = 0; return; }
  uint32_t f = w.g_flags[s];
  const bool same = s > 0 && w.g_cidx[s - 1] == w.g_cidx[s];
  const uint32_t fp = same ? w.g_flags[s - 1] : 0u;
  if (!(f & SEG_ITEM)) {  // GC + GC merge (only the MERGE bit changes, so neighbours read ITEM safely)
    const bool m = same && !(fp & SEG_ITEM);
    const uint32_t g = m ? (f | SEG_MERGE) : (f & ~SEG_MERGE);
    if (g != f) w.g_flags[s] = g;
    f = g;
  }
  w.g_tmp[s] = (f & SEG_MERGE) ? 0u : 1u;
  w.r_size[s] = seg_deleted(f) && !(same && seg_deleted(fp)) ? 1u : 0u;  // delete-set run starts (k_merge_flags)
}
void launch_key_shards(const Work& w, uint32_t nsegs, uint32_t nshards, uint32_t* key_shard, uint8_t* owner, hipStream_t s) {
  hipLaunchKernelGGL(k_key_shard, dim3(w.cap_keys / 256 + 1), dim3(256), 0, s, w, nshards, key_shard);
  if (nsegs) hipLaunchKernelGGL(k_seg_shard, dim3(nsegs / 256 + 1), dim3(256), 0, s, w, nsegs, key_shard, owner);
}
void launch_shard_mask(const Work& w, uint32_t nsegs, const uint8_t* owner, uint32_t shard, hipStream_t s) {
  if (nsegs) hipLaunchKernelGGL(k_shard_mask, dim3(nsegs / 256 + 1), dim3(256), 0, s, w, nsegs, owner, shard);
}
void launch_shard_export(const Work& w, uint32_t nsegs, const uint8_t* owner, uint32_t shard, uint32_t* acc, hipStream_t s) {
  if (nsegs) hipLaunchKernelGGL(k_shard_export, dim3(nsegs / 256 + 1), dim3(256), 0, s, w, nsegs, owner, shard, acc);
}
// the combined flags are in place: settle GC merges, then the output-struct numbering
void launch_merge_final(const Work& w, uint32_t nsegs, hipStream_t s) {
  if (!nsegs) return;
  hipLaunchKernelGGL(k_merge_final, dim3(nsegs / 256 + 1), dim3(256), 0, s, w, nsegs);
  launch_merge_tail(w, nsegs, s);
}

// the item-merge predicate only (a shard's part); launch_merge_tail numbers the output structs
void launch_merge_flags_only(const Work& w, uint32_t nsegs, hipStream_t s, bool fold) {
  if (nsegs) hipLaunchKernelGGL(k_merge_flags, dim3(nsegs / 256 + 1), dim3(256), 0, s, w, nsegs, fold ? 1u : 0u);
}
// (the output structs are numbered by the scan; k_out_sizes records their first segments)
void launch_merge_tail(const Work& w, uint32_t nsegs, hipStream_t s) {
  if (!nsegs) return;
  scan_u32(w.tmp, w.tmp_bytes, w.g_tmp, w.g_outid, nsegs + 1, s);
}

// true: the run ids are scanned too (g_tmp2; the encoder skips that scan)
// Small map-only merges (the per-op path: no YArray, no right origin, no nested type, unsharded):
// the key table fill, segment properties, key resolution, winner descent and merge flags with
// their scans as barrier-separated phases of ONE workgroup — one launch for six. The phases hand
// over through atomics (the key table, the winner slots) as well as plain stores (phase_sync).
constexpr uint32_t MS_LANES = 512, MS_SMALL = MS_LANES * 8;
// nunits != 0: the segment cuts and starts (k_segments_small's work) run here first, and the
// segment count is read on the device (the host skipped the count synchronisation)
template <bool FENCE>
__device__ __forceinline__ void ms_sync() {  // FENCE: agent-scope fences around the barrier (A/B)
  if (FENCE) phase_sync();
  else __syncthreads();
}
template <bool FENCE>
__global__ __launch_bounds__(MS_LANES) void k_merge_small(Work w, uint32_t nsegs, uint64_t nunits) {
  __shared__ uint32_t part[MS_LANES];
  __shared__ uint32_t sarr;
  // an error raised before (the unit passes: a missing dependency, a malformed reference) ends the
  // merge here, as the count synchronisation's check does on the other path: past it the unit
  // references are not bounded
  if (w.ctr->err) return;
  if (nunits) {
    segments_small_body<MS_LANES>(w, nunits, part);
    ms_sync<FENCE>();
    if (ld_fresh(&w.ctr->err)) return;  // (ERR_PENDING: an atomic)
    nsegs = w.ctr->nsegs;
  }
  if (w.dbg_bounds && nsegs + 2 > w.cap_units + 1) {  // (the segment columns hold U + 2 entries)
    if (threadIdx.x == 0) bounds_fail(w.ctr, BOUNDS_MERGE_SMALL);
    return;
  }
  const uint32_t t = threadIdx.x, ck = w.cap_keys;
  if (t == 0) sarr = 0;
  for (uint32_t i = t; i < 2 * ck; i += MS_LANES) ((uint32_t*)w.k_hash)[i] = 0;
  for (uint32_t i = t; i < ck; i += MS_LANES) { w.k_rootmax[i] = 0; w.k_flags[i] = 0; w.k_parent[i] = NONE; }
  for (uint32_t i = t; i < nsegs; i += MS_LANES) w.g_maxchild[i] = 0;
  ms_sync<FENCE>();
  for (uint32_t i = t; i < nsegs; i += MS_LANES) seg_props_at(w, i);
  ms_sync<FENCE>();
  bool arr = false;
  for (uint32_t i = t; i < nsegs; i += MS_LANES) arr |= resolve_at(w, i, nsegs);
  if (arr) sarr = 1u;
  ms_sync<FENCE>();
  if (t == 0 && sarr) w.ctr->narray = 1u;
  for (uint32_t k = t; k < ck; k += MS_LANES) winner_at(w, k, nsegs);
  ms_sync<FENCE>();
  // merge flags (fold: no dead-type pass), then the output struct ids and the run starts' scan
  // input, as k_merge_flags + its scan
  for (uint32_t i = t; i <= nsegs; i += MS_LANES) {
    if (i == nsegs) { w.g_tmp[i] = 0; w.r_size[i] = 0; continue; }
    bool start, rstart;
    merge_flags_at(w, i, 1u, start, rstart);
    w.g_tmp[i] = start ? 1u : 0u;
    w.r_size[i] = rstart ? 1u : 0u;
  }
  __syncthreads();
  block_scan_u32<MS_LANES>(w.g_tmp, w.g_outid, nsegs + 1, part);
}
bool merge_small_fits(uint64_t nsegs_bound) {
  const bool off = env_off("YCRDT_MERGE_SMALL");  // (read per merge: A/B in one process)
  return !off && nsegs_bound && nsegs_bound <= MS_SMALL && (nsegs_bound + 63) / 64 <= SEG_SMALL_WORDS && encode_runs_small((uint32_t)nsegs_bound);
}
// (nunits != 0: the segments too, nsegs read on the device)
void launch_merge_small(const Work& w, uint32_t nsegs, uint64_t nunits, hipStream_t s) {
  if (getenv("YCRDT_PHASE_FENCE") && getenv("YCRDT_PHASE_FENCE")[0] == '1')
    hipLaunchKernelGGL(k_merge_small<true>, dim3(1), dim3(MS_LANES), 0, s, w, nsegs, nunits);
  else
    hipLaunchKernelGGL(k_merge_small<false>, dim3(1), dim3(MS_LANES), 0, s, w, nsegs, nunits);
}

bool launch_merge_flags(const Work& w, uint32_t nsegs, hipStream_t s, bool fold) {
  if (!nsegs) return false;
  const uint32_t tiles = (nsegs + 1 + MF_TILE - 1) / MF_TILE;
  LbChains lb;
  if (!encode_runs_small(nsegs) && lb_launch(tiles, 2, s, lb)) {
    hipLaunchKernelGGL(k_merge_flags_scan, dim3(tiles), dim3(256), 0, s, w, nsegs, fold ? 1u : 0u, lb);
    return true;
  }
  hipLaunchKernelGGL(k_merge_flags, dim3(nsegs / 256 + 1), dim3(256), 0, s, w, nsegs, fold ? 1u : 0u);
  scan_u32(w.tmp, w.tmp_bytes, w.g_tmp, w.g_outid, nsegs + 1, s);
  return false;
}

}  // namespace yc
