// yc_encode.hip — K7: state vector + (delta) re-encode of the merged store as a Yjs v1 update.
//
// Restates encodeStateAsUpdate (Y@22505 → writeClientsStructs Y@19025 → writeStructs Y@18809 →
// Item.write Y@80416) and createDeleteSetFromStructStore + writeDeleteSet (Y@10800 / Y@11105):
//   * client blocks are written in descending client order; a client is included when its state
//     exceeds the target state vector, and its first struct is written with offset sv − clock;
//   * the delete set is always the full store's runs of consecutive deleted structs, clients in
//     descending order (Yjs 13.6 canonical order) or, with cl_emit (compat 135), in the store's
//     client insertion order (13.5.16 iterates store.clients, Y@10800), as is the state vector.
// Every size is computed first (one lane per output struct / run / client), positions come from
// exclusive scans, then a second pass writes the bytes.
#include "yc_work.h"

namespace yc {

__device__ __forceinline__ uint32_t* ccol(const Work& w, uint32_t col) { return w.cc + (size_t)col * (w.cap_clients + 1); }
__device__ __forceinline__ uint64_t* ccol64(const Work& w, uint32_t col) { return w.cc64 + (size_t)col * (w.cap_clients + 1); }

__device__ __forceinline__ uint32_t unit_client(const Work& w, uint32_t nclients, uint32_t g) {
  uint32_t lo = 0, hi = nclients;  // last c with cl_base[c] <= g
  while (hi - lo > 1) { const uint32_t mid = (lo + hi) >> 1; if (w.cl_base[mid] <= g) lo = mid; else hi = mid; }
  return lo;
}

// client of unit g, trying the likely candidates first (the segment's own client: an origin inside
// a split struct; the source struct's origin / right-origin client) before the binary search,
// which costs ~10 dependent loads per call
__device__ __forceinline__ uint32_t unit_client_hint(const Work& w, uint32_t nclients, uint32_t g, uint32_t c0, uint32_t c1) {
  if (c0 < nclients && g >= w.cl_base[c0] && g < w.cl_base[c0 + 1]) return c0;
  if (c1 < nclients && g >= w.cl_base[c1] && g < w.cl_base[c1 + 1]) return c1;
  return unit_client(w, nclients, g);
}

__device__ __forceinline__ uint64_t copy_bytes(uint8_t* __restrict__ o, uint64_t p, const uint8_t* __restrict__ src, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) o[p + i] = src[i];
  return p + n;
}

// Encodes output struct `o` (segments [a,b)) at position p when WRITE, returns the size
// (Item.write Y@80416 / GC.write Y@68955 with the writeStructs offset, Y@18809).
template <bool WRITE>
__device__ uint32_t encode_struct_general(const Work& w, uint32_t nclients, uint32_t a, uint32_t b, uint8_t* __restrict__ out, uint64_t p0);

// The common output struct is one WHOLE source item (one segment from the struct's first unit to
// its last, full-state encode): Item.write then emits the input's own bytes — its origin, right
// origin, parent and parentSub fields are the ones it was decoded from — except the info byte
// (content ref -> Deleted when the item is deleted now; the parentSub bit, which lazily merged
// input drops on items with an origin) and, for a deleted item, the content (ContentDeleted: its
// length). So it is a copy of [pos + 1, cpos) and [cpos, cend) — five columns instead of the
// general path's twenty (and its reference-client lookups).
// (output struct = segments [a, b))
// ENC_DEFER: not the whole-item case; the general encoder takes it in a kernel of its own
// (k_out_sizes_general / k_write_general): inlined, the general path's registers — 74 / 94 VGPRs —
// cost the one-pass kernels two to three waves per SIMD for every output struct
constexpr uint32_t ENC_DEFER = 0xFFFFFFFFu;
template <bool WRITE>
__device__ __forceinline__ uint32_t encode_struct_fast(const Work& w, uint32_t a, uint32_t b, uint8_t* __restrict__ out, uint64_t p0) {
  if (b == a + 1 && !w.delta) {
    const uint32_t f = w.g_flags[a], src = w.g_src[a], ga = seg_start(w, a), gb = seg_start(w, b);
    const uint32_t slen = w.s_len[src], spos = w.s_pos[src], scpos = w.s_cpos[src], scend = w.s_cend[src];
    const uint32_t info0 = w.s_info[src], spk = w.s_pk[src];
    if ((f & (SEG_ITEM | SEG_EXPLICIT)) == (SEG_ITEM | SEG_EXPLICIT) && gb - ga == slen && !(spk & 0xC0u)) {
      const bool del = (f & SEG_DEL) != 0;
      const uint32_t hdr = scpos - spos - 1;  // origin / right origin / parent / parentSub bytes
      if (!WRITE) return 1 + hdr + (del ? vu_size(slen) : scend - scpos);
      const uint8_t* __restrict__ sb = struct_bytes(w, src);
      uint64_t p = p0;
      out[p++] = (uint8_t)((del ? (uint32_t)REF_DELETED : (info0 & 31u)) | (info0 & 0xC0u) | ((f & SEG_PSUB) ? 0x20u : 0u));
      p = copy_bytes(out, p, sb + spos + 1, hdr);
      if (del) p = wr_vu(out, p, slen);
      else p = copy_bytes(out, p, sb + scpos, scend - scpos);
      return (uint32_t)(p - p0);
    }
  }
  return ENC_DEFER;
}

template <bool WRITE>
__device__ __forceinline__ uint32_t encode_struct_general(const Work& w, uint32_t nclients, uint32_t a, uint32_t b, uint8_t* __restrict__ out,
                                                                    uint64_t p0) {
  // The columns a struct can need are loaded in three dependent rounds — its first segment's row,
  // then its source struct's and its client's, then the reference clients' — each round issued
  // whole before anything branches on it, instead of one memory round trip per field.
  const uint32_t cidx = w.g_cidx[a], ga = seg_start(w, a), gb = seg_start(w, b), f = w.g_flags[a], src = w.g_src[a];
  const uint32_t go = w.g_origin[a], gr = w.g_rorigin[a];
  const uint64_t base = w.cl_base[cidx], base1 = w.cl_base[cidx + 1];
  const uint32_t cs = w.cl_start[cidx], cval = w.cl_vals[cidx];
  const uint32_t info0 = w.s_info[src], soc = w.s_ocidx[src], src_rc = w.s_rcidx[src];
  const uint32_t sclk = w.s_clock[src], slen = w.s_len[src], scel = w.s_celem[src], scend = w.s_cend[src];
  const uint8_t* __restrict__ sb = struct_bytes(w, src);  // the source struct's window
  const uint32_t k0 = (uint32_t)(ga - base), k1 = (uint32_t)(gb - base);
  if (k1 <= cs) return 0;
  const uint32_t off = cs > k0 ? cs - k0 : 0;
  const uint32_t len = k1 - k0;
  uint64_t p = p0;
  if (!(f & SEG_ITEM)) {  // GC.write
    if (WRITE) { out[p++] = REF_GC; p = wr_vu(out, p, len - off); return (uint32_t)(p - p0); }
    return 1 + vu_size(len - off);
  }
  const bool del = (f & SEG_DEL) != 0;
  const uint32_t ref = del ? (uint32_t)REF_DELETED : (info0 & 31u);
  // the reference clients: the segment's own client first (an origin inside a split struct), then
  // the source struct's recorded origin / right-origin client, a binary search last
  auto client_of = [&](uint32_t g, uint32_t hint) -> uint32_t {
    if (g >= base && g < base1) return cidx;
    if (hint < nclients && g >= w.cl_base[hint] && g < w.cl_base[hint + 1]) return hint;
    return unit_client(w, nclients, g);
  };
  // the origin's likely client (the source struct's recorded one): its base, end and id together
  const bool sh = soc < nclients;
  const uint64_t hb0 = sh ? w.cl_base[soc] : 0ull, hb1 = sh ? w.cl_base[soc + 1] : 0ull;
  const uint32_t hval = sh ? w.cl_vals[soc] : 0u;
  uint32_t oclient = 0, oclock = 0;
  bool has_o = false;
  if (off > 0) { has_o = true; oclient = cval; oclock = k0 + off - 1; }
  else if (go != NONE) {
    has_o = true;
    if (go >= base && go < base1) { oclient = cval; oclock = (uint32_t)(go - base); }
    else if (sh && go >= hb0 && go < hb1) { oclient = hval; oclock = (uint32_t)(go - hb0); }
    else {
      const uint32_t c = unit_client(w, nclients, go);
      oclient = w.cl_vals[c];
      oclock = (uint32_t)(go - w.cl_base[c]);
    }
  }
  bool has_r = false;
  uint32_t rclient = 0, rclock = 0;
  if (gr != NONE) {
    const uint32_t c = client_of(gr, src_rc);
    has_r = true;
    rclient = c == cidx ? cval : w.cl_vals[c];
    rclock = (uint32_t)(gr - (c == cidx ? base : w.cl_base[c]));
  }
  const bool psub = (f & SEG_PSUB) != 0;
  const uint32_t info = ref | (has_o ? 0x80u : 0u) | (has_r ? 0x40u : 0u) | (psub ? 0x20u : 0u);
  uint32_t size = 1;
  if (WRITE) out[p++] = (uint8_t)info;
  if (has_o) {
    if (WRITE) { p = wr_vu(out, p, oclient); p = wr_vu(out, p, oclock); }
    size += vu_size(oclient) + vu_size(oclock);
  }
  if (has_r) {
    if (WRITE) { p = wr_vu(out, p, rclient); p = wr_vu(out, p, rclock); }
    size += vu_size(rclient) + vu_size(rclock);
  }
  if (!has_o && !has_r) {  // parent info (root type name | parent item id) + parentSub
    const uint32_t pa = w.s_pa[src], pb = w.s_pb[src];
    if ((w.s_pk[src] & 3u) == 1) {  // writeVarString(name): the length prefix in shortest form
      uint32_t q = pa;
      bool okq = true;
      const uint32_t n = rd_vu(sb, q, pa + pb, okq);
      if (WRITE) { out[p++] = 1; p = wr_vu(out, p, n); p = copy_bytes(out, p, sb + q, n); }
      size += 1 + vu_size(n) + n;
    } else {
      const uint32_t pc = w.cl_vals[pa];
      if (WRITE) { out[p++] = 0; p = wr_vu(out, p, pc); p = wr_vu(out, p, pb); }
      size += 1 + vu_size(pc) + vu_size(pb);
    }
    if (psub) {
      const uint32_t ps = w.s_psub[src], pl = w.s_psublen[src];
      uint32_t q = ps;
      bool okq = true;
      const uint32_t n = rd_vu(sb, q, ps + pl, okq);
      if (WRITE) { p = wr_vu(out, p, n); p = copy_bytes(out, p, sb + q, n); }
      size += vu_size(n) + n;
    }
  }
  if (del) {
    if (WRITE) p = wr_vu(out, p, len - off);
    size += vu_size(len - off);
  } else if ((ref == REF_ANY || ref == REF_JSON) && b == a + 1 && off == 0 && k0 == sclk && len == slen) {
    // the whole content of one source struct (the common case): its element bytes verbatim (in
    // writeAny's form when the input's were not, s_pk bit 6)
    if (ref == REF_ANY && (w.s_pk[src] & 0x40u)) {
      if (WRITE) p = wr_vu(out, p, len);
      const uint32_t nb = any_canon<WRITE>(sb, scel, scend, 0, len, out, p);
      if (WRITE) p += nb;
      size += vu_size(len) + nb;
    } else {
      const uint32_t nbytes = scend - scel;
      if (WRITE) { p = wr_vu(out, p, len); p = copy_bytes(out, p, sb + scel, nbytes); }
      size += vu_size(len) + nbytes;
    }
  } else if (ref == REF_ANY || ref == REF_JSON || ref == REF_STRING) {
    // elements of every segment from unit k0 + off on, sliced out of their source structs
    uint32_t nbytes = 0;
    for (uint32_t pass = 0; pass < (WRITE ? 2u : 1u); ++pass) {
      if (pass == 1) p = wr_vu(out, p, ref == REF_STRING ? nbytes : len - off);
      for (uint32_t s = a; s < b; ++s) {
        const uint32_t sr = w.g_src[s];
        const uint32_t sb = w.s_clock[sr];  // source struct's first clock
        const uint32_t u0 = max((uint32_t)(seg_start(w, s) - base), k0 + off), u1 = (uint32_t)(seg_start(w, s + 1) - base);
        if (u1 <= u0) continue;
        if (ref == REF_ANY && (w.s_pk[sr] & 0x40u)) {  // flagged content: writeAny's form
          const uint32_t nb = any_canon<WRITE>(struct_bytes(w, sr), w.s_celem[sr], w.s_cend[sr], u0 - sb, u1 - sb, out, p);
          if (pass == 1) p += nb;
          else nbytes += nb;
          continue;
        }
        uint32_t b0 = 0, b1 = 0;
        if (!content_slice(w, sr, u0 - sb, u1 - sb, b0, b1)) { raise_err(&w.ctr->err, ERR_UNSUPPORTED); return size; }
        if (pass == 1) p = copy_bytes(out, p, struct_bytes(w, sr) + b0, b1 - b0);
        else nbytes += b1 - b0;
      }
    }
    size += (ref == REF_STRING ? vu_size(nbytes) : vu_size(len - off)) + nbytes;
  } else {  // Binary / Embed / Format / Type / Doc: one unit, verbatim content bytes
    const uint32_t n = w.s_cend[src] - w.s_cpos[src];
    if (WRITE) p = copy_bytes(out, p, sb + w.s_cpos[src], n);
    size += n;
  }
  return size;
}

// NO (ctr->nout) and the run count (g_tmp2[NS]) stay on the device: grids and scans cover NS + 1.
// One lane per segment: a segment that starts output struct o = g_outid[s] (the exclusive scan of
// the merge flags) records it (o_first, o_cidx) and sizes it, finding the struct's end by stepping
// over the segments merged into it (usually none); the others zero the size slots past NO, so the
// scan over NS + 1 entries sees exactly the NO sizes.
__device__ __forceinline__ bool out_sizes_at(const Work& w, uint32_t s, uint32_t nsegs, uint32_t nout) {
  if (s == nsegs) {
    w.o_first[nout] = nsegs;  // sentinel
    w.o_size[nsegs] = 0;
    w.ctr->nout = nout;
    return false;
  }
  const uint32_t o = w.g_outid[s];
  const bool start = !(w.g_flags[s] & SEG_MERGE);
  uint32_t sz = 0;
  if (!start) {
    w.o_size[nout + (s - o)] = 0;  // (s - o: its rank among the non-starts)
  } else {
    uint32_t b = s + 1;
    while (b < nsegs && (w.g_flags[b] & SEG_MERGE)) ++b;
    w.o_first[o] = s;
    w.o_cidx[o] = w.g_cidx[s];
    sz = encode_struct_fast<false>(w, s, b, nullptr, 0);
    // a deferred one (k_out_sizes_general) is flagged, not listed: one list counter taken by a
    // wavefront of every few took C4 (mostly merged runs) 1.7 -> 7.3 ms, at the one-word atomic rate
    w.o_size[o] = sz == ENC_DEFER ? 0u : sz;
    w.o_gen[o] = sz == ENC_DEFER ? 1u : 0u;
  }
  return sz == ENC_DEFER;
}
__global__ __launch_bounds__(256) void k_out_sizes(Work w, uint32_t nsegs, uint32_t nclients) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s > nsegs) return;
  const bool defer = out_sizes_at(w, s, nsegs, nsegs ? w.g_outid[nsegs] : 0u);
  wave_flag(&w.ctr->pad[6], defer);  // (the general kernels run only when some struct is deferred)
}
// the deferred output structs (split, merged or delta-cut ones), sized by the general encoder
// (a wavefront reads the flags of 1 024 consecutive output structs as 64 quads and skips the whole
// stretch when all are zero, as on C2; otherwise it takes the stretch as 16 steps of 64
// consecutive output structs, a lane each — consecutive, so the general encoder's loads stay
// coalesced: lanes 16 structs apart made them 64 lines per load, C4's general encode 0.8 -> 2.7
// ms. Flags past NO are never taken; the buffer is padded to whole quads.)
template <class F>
__device__ __forceinline__ void for_deferred(const Work& w, uint32_t n, F f) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwaves = (gridDim.x * blockDim.x) >> 6;
  for (uint32_t o0 = wave * 1024; o0 < n; o0 += nwaves * 1024) {
    const uint32_t q = o0 / 16 + lane;
    const uint4 v = q * 16 < n ? ((const uint4*)w.o_gen)[q] : make_uint4(0u, 0u, 0u, 0u);
    if (!__ballot((v.x | v.y | v.z | v.w) != 0u)) continue;
    for (uint32_t k = 0; k < 16; ++k) {
      const uint32_t o = o0 + k * 64 + lane;
      const bool act = o < n && w.o_gen[o];
      if (!__ballot(act)) continue;
      if (act) f(o);
    }
  }
}
__global__ __launch_bounds__(256) void k_out_sizes_general(Work w, uint32_t nclients) {
  if (!w.ctr->pad[6]) return;
  for_deferred(w, w.ctr->nout, [&](uint32_t o) {
    w.o_size[o] = encode_struct_general<false>(w, nclients, w.o_first[o], w.o_first[o + 1], nullptr, 0);
  });
}

// runs of consecutive deleted segments (createDeleteSetFromStructStore): their starts were flagged
// in r_size by k_merge_flags / k_merge_final
__device__ __forceinline__ bool seg_deleted(uint32_t f) { return (f & SEG_DEL) || !(f & SEG_ITEM); }
__device__ __forceinline__ void run_fill_at(const Work& w, uint32_t s, uint32_t nsegs) {
  const uint32_t f = w.g_flags[s];
  if (!seg_deleted(f)) return;
  const uint32_t rid = w.g_tmp2[s + 1] - 1;  // inclusive count of run starts up to s
  if (w.g_tmp2[s + 1] != w.g_tmp2[s]) w.r_seg[rid] = s;  // s starts run rid
  // s ends run rid: the next segment is live or belongs to another client
  const bool last = s + 1 == nsegs || w.g_cidx[s + 1] != w.g_cidx[s] || !seg_deleted(w.g_flags[s + 1]);
  if (last) w.r_len[rid] = seg_start(w, s + 1);  // end unit; the start is subtracted in k_run_sizes
}
__global__ void k_run_fill(Work w, uint32_t nsegs) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < nsegs) run_fill_at(w, s, nsegs);
}
__device__ __forceinline__ void run_sizes_at(const Work& w, uint32_t r, uint32_t nsegs) {
  if (r >= w.g_tmp2[nsegs]) { w.r_size[r] = 0; return; }
  const uint32_t s = w.r_seg[r];
  const uint32_t len = w.r_len[r] - seg_start(w, s);
  w.r_len[r] = len;
  const uint32_t clock = (uint32_t)(seg_start(w, s) - w.cl_base[w.g_cidx[s]]);
  w.r_size[r] = vu_size(clock) + vu_size(len);
}
__global__ void k_run_sizes(Work w, uint32_t nsegs) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r <= nsegs) run_sizes_at(w, r, nsegs);
}
// Small batches: the delete-set runs (scan of the run starts, fill, sizes, scan of the sizes) in
// ONE workgroup launch on the main stream (four launches on the side stream and its fork / join)
constexpr uint32_t RUNS_LANES = 1024, RUNS_SMALL = RUNS_LANES * 16;
__global__ __launch_bounds__(RUNS_LANES) void k_runs_small(Work w, uint32_t nsegs) {
  __shared__ uint32_t part[RUNS_LANES];
  block_scan_u32<RUNS_LANES>(w.r_size, w.g_tmp2, nsegs + 1, part);  // (r_size: k_merge_flags' run starts)
  for (uint32_t s = threadIdx.x; s < nsegs; s += RUNS_LANES) run_fill_at(w, s, nsegs);
  __syncthreads();
  for (uint32_t r = threadIdx.x; r <= nsegs; r += RUNS_LANES) run_sizes_at(w, r, nsegs);
  __syncthreads();
  block_scan_u32<RUNS_LANES>(w.r_size, w.r_pos, nsegs + 1, part);
}

// per client: first output struct and first delete-set run, from the boundaries of the (client-
// sorted) output and run arrays — one parallel pass instead of per-client binary searches, whose
// ~80 dependent loads per lane made the per-client pass latency-bound
__device__ __forceinline__ void client_bounds_at(const Work& w, uint32_t i, uint32_t nclients, uint32_t nout, uint32_t nruns) {
  if (i <= nout) {
    const int64_t a = i == 0 ? -1 : (int64_t)w.o_cidx[i - 1];
    const int64_t b = i == nout ? (int64_t)nclients : (int64_t)w.o_cidx[i];
    for (int64_t c = a + 1; c <= b; ++c) ccol(w, CC_FIRST_OUT)[c] = i;
  }
  if (i <= nruns) {
    const int64_t a = i == 0 ? -1 : (int64_t)w.g_cidx[w.r_seg[i - 1]];
    const int64_t b = i == nruns ? (int64_t)nclients : (int64_t)w.g_cidx[w.r_seg[i]];
    for (int64_t c = a + 1; c <= b; ++c) ccol(w, CC_RUN_LO)[c] = i;
  }
}
__global__ void k_client_bounds(Work w, uint32_t nclients, uint32_t nsegs) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= nsegs) client_bounds_at(w, i, nclients, w.ctr->nout, w.g_tmp2[nsegs]);
}

// per client: struct block + delete-set block + state-vector entry sizes; returns bit 0: the
// client's structs are included, 1: it has delete-set runs, 2: a state-vector entry
__device__ __forceinline__ uint32_t client_sizes_at(const Work& w, uint32_t c, uint32_t nclients) {
  uint32_t* first_out = ccol(w, CC_FIRST_OUT);
  if (c == nclients) {
    ccol(w, CC_BLK)[c] = 0; ccol(w, CC_DSBLK)[c] = 0; ccol(w, CC_SV)[c] = 0;
    return 0u;
  }
  // first output struct of client c and of the next client (outputs are sorted by client)
  const uint32_t fo = first_out[c], eo = first_out[c + 1];
  const uint32_t state = w.cl_state[c];
  const uint32_t cs = w.cl_start[c];
  uint32_t blk = 0, nincl = 0, fi = eo;
  const bool incl = state > cs && eo > fo;
  if (incl) {
    // first included output: the one containing clock cs
    uint32_t lo = fo, hi = cs == 0 ? fo : eo;  // a full-state encode starts at the first output
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      const uint32_t k1 = (uint32_t)(seg_start(w, w.o_first[mid + 1]) - w.cl_base[c]);
      if (k1 <= cs) lo = mid + 1; else hi = mid;
    }
    fi = lo;
    nincl = eo - fi;
    const uint32_t hdr = vu_size(nincl) + vu_size(w.cl_vals[c]) + vu_size(cs);
    ccol(w, CC_HDR)[c] = hdr;
    blk = hdr + (w.o_pos[eo] - w.o_pos[fi]);
  }
  ccol(w, CC_FIRST_INCL)[c] = fi;
  ccol(w, CC_NINCL)[c] = nincl;
  ccol(w, CC_BLK)[c] = blk;
  // delete-set block: runs are ordered by (client, clock)
  const uint32_t lo = ccol(w, CC_RUN_LO)[c], nr = ccol(w, CC_RUN_LO)[c + 1] - lo;
  ccol(w, CC_NRUNS)[c] = nr;
  uint32_t dsblk = 0;
  if (nr) {
    ccol(w, CC_FIRST_RUN)[c] = lo;
    dsblk = vu_size(w.cl_vals[c]) + vu_size(nr) + (w.r_pos[lo + nr] - w.r_pos[lo]);
  }
  ccol(w, CC_DSBLK)[c] = dsblk;
  ccol(w, CC_SV)[c] = state ? vu_size(w.cl_vals[c]) + vu_size(state) : 0;
  return (incl ? 1u : 0u) | (nr ? 2u : 0u) | (state ? 4u : 0u);
}
__global__ void k_client_sizes(Work w, uint32_t nclients, uint32_t nsegs) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c > nclients) return;
  const uint32_t m = client_sizes_at(w, c, nclients);
  wave_count_add(&w.ctr->pad[0], m & 1u);  // included clients
  wave_count_add(&w.ctr->pad[1], m & 2u);  // ds clients
  wave_count_add(&w.ctr->pad[2], m & 4u);  // sv entries
}

// reverse the three per-client size columns (structs, delete set, state vector) so that ascending
// scans yield descending-client positions; one launch each way for all three. With cl_emit
// (compat 135) the delete-set and state-vector columns follow the store insertion order instead.
__device__ __forceinline__ uint32_t emit_slot_client(const Work& w, uint32_t nclients, int k, uint32_t i) {
  return (k > 0 && w.cl_emit) ? w.cl_emit[i] : nclients - 1 - i;
}
__global__ void k_reverse3(Work w, uint32_t nclients) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > nclients) return;
  const uint32_t src[3] = {CC_BLK, CC_DSBLK, CC_SV}, dst[3] = {CC_REV, CC_REV2, CC_REV3};
  for (int k = 0; k < 3; ++k) ccol(w, dst[k])[i] = i < nclients ? ccol(w, src[k])[emit_slot_client(w, nclients, k, i)] : 0;
}
__global__ void k_unreverse3(Work w, uint32_t nclients) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c > nclients) return;
  // position of client c = sum of the blocks written before it = scan[slot of c]; total at [nclients]
  // (64-bit: the sections of a merge past 4 GiB)
  const uint32_t src[3] = {CC64_SCAN, CC64_SCAN2, CC64_SCAN3}, dst[3] = {CC64_BLKPOS, CC64_DSPOS, CC64_SVPOS};
  for (int k = 0; k < 3; ++k) {
    const uint32_t slot = c == nclients ? nclients : (k > 0 && w.cl_emit) ? w.cl_slot[c] : nclients - 1 - c;
    ccol64(w, dst[k])[c] = ccol64(w, src[k])[slot];
  }
}

__device__ __forceinline__ void totals_body(const Work& w, uint32_t nclients) {
  const uint32_t nincl = w.ctr->pad[0], nds = w.ctr->pad[1], nsv = w.ctr->pad[2];
  const uint64_t sblk = ccol64(w, CC64_BLKPOS)[nclients];
  const uint64_t sds = ccol64(w, CC64_DSPOS)[nclients];
  const uint64_t ssv = ccol64(w, CC64_SVPOS)[nclients];
  w.ctr->pad[3] = vu_size(nincl);                 // struct section header size
  w.ctr->ds_base = vu_size(nincl) + sblk;         // delete-set section start
  w.ctr->out_total = vu_size(nincl) + sblk + vu_size(nds) + sds;
  w.ctr->sv_bytes = (uint32_t)(vu_size(nsv) + ssv);
  // the output buffers were sized from a bound before the sizes were known; never write past them
  if (w.ctr->out_total > w.cap_out || vu_size(nsv) + ssv > w.cap_sv) { w.ctr->pad[5] = 1; raise_err(&w.ctr->err, ERR_CAPACITY); }
}
__global__ void k_totals(Work w, uint32_t nclients) { totals_body(w, nclients); }

__device__ __forceinline__ uint64_t out_pos(const Work& w, uint32_t o) {
  const uint32_t c = w.o_cidx[o];
  const uint32_t fi = ccol(w, CC_FIRST_INCL)[c];
  // (o_pos wraps at 2^32: differences within one client's block are exact)
  return w.ctr->pad[3] + ccol64(w, CC64_BLKPOS)[c] + ccol(w, CC_HDR)[c] + (uint32_t)(w.o_pos[o] - w.o_pos[fi]);
}
__global__ __launch_bounds__(256) void k_write_structs(Work w, uint32_t nsegs, uint32_t nclients) {
  const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= w.ctr->nout || w.ctr->pad[5]) return;
  if (w.o_size[o] == 0) return;
  // (the deferred ones decline here, k_write_general writes them)
  encode_struct_fast<true>(w, w.o_first[o], w.o_first[o + 1], w.out, out_pos(w, o));
}
__global__ __launch_bounds__(256) void k_write_general(Work w, uint32_t nclients) {
  if (w.ctr->pad[5] || !w.ctr->pad[6]) return;
  for_deferred(w, w.ctr->nout, [&](uint32_t o) {
    if (w.o_size[o]) encode_struct_general<true>(w, nclients, w.o_first[o], w.o_first[o + 1], w.out, out_pos(w, o));
  });
}
__device__ __forceinline__ void write_clients_at(const Work& w, uint32_t c, uint32_t nclients) {
  if (c == 0) {
    wr_vu(w.out, (uint64_t)0, w.ctr->pad[0]);
    wr_vu(w.out, (uint64_t)w.ctr->ds_base, w.ctr->pad[1]);
    wr_vu(w.sv_out, (uint64_t)0, w.ctr->pad[2]);
  }
  if (c >= nclients) return;
  if (ccol(w, CC_NINCL)[c]) {
    uint64_t p = w.ctr->pad[3] + ccol64(w, CC64_BLKPOS)[c];
    p = wr_vu(w.out, p, ccol(w, CC_NINCL)[c]);
    p = wr_vu(w.out, p, w.cl_vals[c]);
    wr_vu(w.out, p, w.cl_start[c]);
  }
  const uint32_t nr = ccol(w, CC_NRUNS)[c];
  if (nr) {
    const uint64_t dsbase = w.ctr->ds_base + vu_size(w.ctr->pad[1]);
    uint64_t p = dsbase + ccol64(w, CC64_DSPOS)[c];
    p = wr_vu(w.out, p, w.cl_vals[c]);
    wr_vu(w.out, p, nr);
  }
  if (w.cl_state[c]) {
    uint64_t p = vu_size(w.ctr->pad[2]) + ccol64(w, CC64_SVPOS)[c];
    p = wr_vu(w.sv_out, p, w.cl_vals[c]);
    wr_vu(w.sv_out, p, w.cl_state[c]);
  }
}
__global__ void k_write_clients(Work w, uint32_t nclients) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (!w.ctr->pad[5]) write_clients_at(w, c, nclients);
}
__device__ __forceinline__ void write_runs_at(const Work& w, uint32_t r) {
  const uint32_t s = w.r_seg[r];
  const uint32_t c = w.g_cidx[s];
  const uint32_t first = ccol(w, CC_FIRST_RUN)[c];
  const uint32_t nr = ccol(w, CC_NRUNS)[c];
  const uint64_t dsbase = w.ctr->ds_base + vu_size(w.ctr->pad[1]);
  uint64_t p = dsbase + ccol64(w, CC64_DSPOS)[c] + vu_size(w.cl_vals[c]) + vu_size(nr) + (uint32_t)(w.r_pos[r] - w.r_pos[first]);
  p = wr_vu(w.out, p, (uint32_t)(seg_start(w, s) - w.cl_base[c]));
  wr_vu(w.out, p, w.r_len[r]);
}
__global__ void k_write_runs(Work w, uint32_t nsegs) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < w.g_tmp2[nsegs] && !w.ctr->pad[5]) write_runs_at(w, r);
}

// Small client tables (the per-op path, one document): the reverse, the three scans, the
// unreverse and the totals in ONE workgroup and one launch (six launches otherwise). Each scan:
// a lane sums a contiguous run of the emit-order sizes, the run sums are scanned in LDS, each lane
// writes its run's prefixes into the scan column; then every client reads its slot's prefix.
constexpr uint32_t LAYOUT_LANES = 1024, LAYOUT_SMALL = LAYOUT_LANES * 16;
template <uint32_t LAYOUT_LANES>
__device__ __forceinline__ void layout_small_body(const Work& w, uint32_t nclients, uint64_t* part) {
  const uint32_t t = threadIdx.x, n = nclients + 1, per = (n + LAYOUT_LANES - 1) / LAYOUT_LANES;
  const uint32_t a = min(n, t * per), b = min(n, a + per);
  const uint32_t src[3] = {CC_BLK, CC_DSBLK, CC_SV}, scol[3] = {CC64_SCAN, CC64_SCAN2, CC64_SCAN3};
  for (int k = 0; k < 3; ++k) {
    auto val = [&](uint32_t i) -> uint64_t { return i < nclients ? ccol(w, src[k])[emit_slot_client(w, nclients, k, i)] : 0u; };
    uint64_t sum = 0;
    for (uint32_t i = a; i < b; ++i) sum += val(i);
    part[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < LAYOUT_LANES; off <<= 1) {
      const uint64_t v = t >= off ? part[t - off] : 0ull;
      __syncthreads();
      part[t] += v;
      __syncthreads();
    }
    uint64_t run = part[t] - sum;
    for (uint32_t i = a; i < b; ++i) { ccol64(w, scol[k])[i] = run; run += val(i); }
    __syncthreads();
  }
  __threadfence_block();
  const uint32_t dst[3] = {CC64_BLKPOS, CC64_DSPOS, CC64_SVPOS};
  for (uint32_t c = t; c <= nclients; c += LAYOUT_LANES)
    for (int k = 0; k < 3; ++k) {
      const uint32_t slot = c == nclients ? nclients : (k > 0 && w.cl_emit) ? w.cl_slot[c] : nclients - 1 - c;
      ccol64(w, dst[k])[c] = ccol64(w, scol[k])[slot];
    }
  __syncthreads();
  if (t == 0) totals_body(w, nclients);  // (k_totals)
}
__global__ __launch_bounds__(LAYOUT_LANES) void k_layout_small(Work w, uint32_t nclients) {
  __shared__ uint64_t part[LAYOUT_LANES];
  layout_small_body<LAYOUT_LANES>(w, nclients, part);
}

static void rev_scans(const Work& w, uint32_t nclients, hipStream_t s) {
  if (nclients + 1 <= LAYOUT_SMALL) {  // (k_totals included)
    hipLaunchKernelGGL(k_layout_small, dim3(1), dim3(LAYOUT_LANES), 0, s, w, nclients);
    return;
  }
  const uint32_t grid = nclients / 256 + 1;
  hipLaunchKernelGGL(k_reverse3, dim3(grid), dim3(256), 0, s, w, nclients);
  const uint32_t cols[3][2] = {{CC_REV, CC64_SCAN}, {CC_REV2, CC64_SCAN2}, {CC_REV3, CC64_SCAN3}};
  for (auto& c : cols)
    scan_u32_to_u64(w.tmp, w.tmp_bytes, w.cc + (size_t)c[0] * (w.cap_clients + 1), w.cc64 + (size_t)c[1] * (w.cap_clients + 1),
                    nclients + 1, s);
  hipLaunchKernelGGL(k_unreverse3, dim3(grid), dim3(256), 0, s, w, nclients);
}

// Small batches (the per-op path): the whole encode — run starts, fill, sizes and scans, output
// struct sizes (general ones inline), their scan, client bounds and sizes, layout, totals and every
// write — as barrier-separated phases of ONE workgroup: one launch where the phases above take
// twelve (≈4-5 us each at this size). Counters other lanes feed are gathered in LDS, not in the
// counter words (a relaxed L2 atomic is not seen through another wavefront's L1 line).
constexpr uint32_t ENC_SMALL_LANES = 512, ENC_SMALL = ENC_SMALL_LANES * 16;
__global__ __launch_bounds__(ENC_SMALL_LANES) void k_encode_small(Work w, uint32_t nsegs, uint32_t nclients) {
  __shared__ uint64_t part64[ENC_SMALL_LANES];
  __shared__ uint32_t cnt[3];
  if (nsegs == NONE) {  // (a small merge left the count on the device)
    if (w.ctr->err) return;  // (k_merge_small stopped at an earlier error: nothing to encode)
    nsegs = w.ctr->nsegs;
  }
  if (w.dbg_bounds && (nsegs + 2 > w.cap_units + 1 || nclients + 1 > w.cap_clients + 1)) {
    if (threadIdx.x == 0) bounds_fail(w.ctr, BOUNDS_ENCODE_SMALL);
    return;
  }
  uint32_t* part = (uint32_t*)part64;
  const uint32_t t = threadIdx.x;
  for (uint32_t i = t; i < 8; i += ENC_SMALL_LANES) w.ctr->pad[i] = 0;
  for (uint32_t c = t; c <= w.cap_clients; c += ENC_SMALL_LANES) ccol(w, CC_NRUNS)[c] = 0;
  if (t < 3) cnt[t] = 0;
  if (!nsegs && t == 0) w.r_size[0] = 0;
  __syncthreads();
  // delete-set runs (k_runs_small)
  block_scan_u32<ENC_SMALL_LANES>(w.r_size, w.g_tmp2, nsegs + 1, part);
  for (uint32_t s = t; s < nsegs; s += ENC_SMALL_LANES) run_fill_at(w, s, nsegs);
  __syncthreads();
  for (uint32_t r = t; r <= nsegs; r += ENC_SMALL_LANES) run_sizes_at(w, r, nsegs);
  __syncthreads();
  block_scan_u32<ENC_SMALL_LANES>(w.r_size, w.r_pos, nsegs + 1, part);
  // output struct sizes (k_out_sizes, k_out_sizes_general)
  const uint32_t nout = nsegs ? w.g_outid[nsegs] : 0u;
  for (uint32_t s = t; s <= nsegs; s += ENC_SMALL_LANES) out_sizes_at(w, s, nsegs, nout);
  __syncthreads();
  for (uint32_t o = t; o < nout; o += ENC_SMALL_LANES)
    if (w.o_gen[o]) w.o_size[o] = encode_struct_general<false>(w, nclients, w.o_first[o], w.o_first[o + 1], nullptr, 0);
  __syncthreads();
  block_scan_u32<ENC_SMALL_LANES>(w.o_size, w.o_pos, nsegs + 1, part);
  // per-client bounds and sizes (k_client_bounds, k_client_sizes)
  const uint32_t nruns = w.g_tmp2[nsegs];
  for (uint32_t i = t; i <= nsegs; i += ENC_SMALL_LANES) client_bounds_at(w, i, nclients, nout, nruns);
  __syncthreads();
  uint32_t m = 0;
  for (uint32_t c = t; c <= nclients; c += ENC_SMALL_LANES) {
    const uint32_t x = client_sizes_at(w, c, nclients);
    m += (x & 1u) | (x & 2u) << 15;
    if (x & 4u) atomicAdd(&cnt[2], 1u);
  }
  if (m & 0xFFFFu) atomicAdd(&cnt[0], m & 0xFFFFu);
  if (m >> 16) atomicAdd(&cnt[1], m >> 16);
  __syncthreads();
  if (t == 0) { w.ctr->pad[0] = cnt[0]; w.ctr->pad[1] = cnt[1]; w.ctr->pad[2] = cnt[2]; }
  __syncthreads();
  // layout and totals (k_layout_small)
  layout_small_body<ENC_SMALL_LANES>(w, nclients, part64);
  __syncthreads();
  if (w.ctr->pad[5]) return;  // (past the output bound: k_totals raised the error)
  // every write (k_write_structs, k_write_general, k_write_clients, k_write_runs)
  for (uint32_t o = t; o < nout; o += ENC_SMALL_LANES) {
    if (!w.o_size[o]) continue;
    YC_BOUND(w, out_pos(w, o) + w.o_size[o], w.cap_out + 1, BOUNDS_OUTPUT);
    if (w.o_gen[o]) encode_struct_general<true>(w, nclients, w.o_first[o], w.o_first[o + 1], w.out, out_pos(w, o));
    else encode_struct_fast<true>(w, w.o_first[o], w.o_first[o + 1], w.out, out_pos(w, o));
  }
  for (uint32_t c = t; c < max(nclients, 1u); c += ENC_SMALL_LANES) write_clients_at(w, c, nclients);
  for (uint32_t r = t; r < nruns; r += ENC_SMALL_LANES) write_runs_at(w, r);
}
bool encode_small_fits(uint64_t nsegs_bound, uint32_t nclients) {
  const bool off = env_off("YCRDT_ENCODE_SMALL");  // (read per merge: A/B in one process)
  return !off && nsegs_bound + 1 <= ENC_SMALL && nclients + 1 <= ENC_SMALL;
}
// (nsegs: NONE = read on the device)
void launch_encode_small(const Work& w, uint32_t nsegs, uint32_t nclients, hipStream_t s) {
  hipLaunchKernelGGL(k_encode_small, dim3(1), dim3(ENC_SMALL_LANES), 0, s, w, nsegs, nclients);
}

// Phase 1: sizes + layout (ends with out_bytes / sv_bytes in the counters). No host sync: the
// output / run counts are read on the device, grids and scans are sized for NS + 1 entries.
bool encode_runs_small(uint32_t nsegs) { return nsegs + 1 <= RUNS_SMALL; }
// runs_scanned: k_merge_flags already made the run ids (g_tmp2)
void launch_encode_sizes(const Work& w, uint32_t nsegs, uint32_t nclients, hipStream_t s, hipStream_t side,
                         hipEvent_t ev_fork, hipEvent_t ev_join, void* tmp2, size_t tmp2_bytes, bool runs_scanned) {
  fill_u32_multi({{w.ctr->pad, 8, 0u}, {w.cc + (size_t)CC_NRUNS * (w.cap_clients + 1), (uint64_t)w.cap_clients + 1, 0u}}, s);
  const uint32_t grid = nsegs / 256 + 1;
  if (nsegs + 1 <= RUNS_SMALL) {  // (a small batch: one launch, main stream)
    if (!nsegs) fill_u32_multi({{w.r_size, 1, 0u}}, s);
    hipLaunchKernelGGL(k_runs_small, dim3(1), dim3(RUNS_LANES), 0, s, w, nsegs);
    hipEventRecord(ev_join, s);  // (the layout waits on it)
    return;
  }
  // delete-set runs (side stream) || output struct sizes (main stream)
  hipEventRecord(ev_fork, s);
  hipStreamWaitEvent(side, ev_fork, 0);
  if (!nsegs) fill_u32_multi({{w.r_size, 1, 0u}}, side);  // (no merge-flag pass wrote the run starts)
  if (!runs_scanned) scan_u32(tmp2, tmp2_bytes, w.r_size, w.g_tmp2, nsegs + 1, side);
  if (nsegs) hipLaunchKernelGGL(k_run_fill, dim3((nsegs + 255) / 256), dim3(256), 0, side, w, nsegs);
  // (a look-back fused into k_run_sizes ran 2x slower beside k_out_sizes_general: its waiting
  // wavefronts held the CUs the main stream's kernel needed)
  hipLaunchKernelGGL(k_run_sizes, dim3(grid), dim3(256), 0, side, w, nsegs);
  scan_u32(tmp2, tmp2_bytes, w.r_size, w.r_pos, nsegs + 1, side);
  hipEventRecord(ev_join, side);
}
// the output struct sizes (its own phase: the bench times it live when it is the longest kernel)
constexpr uint32_t GEN_GRID = 2048;  // grid-stride over the deferral flags (NO stays on the device)
void launch_out_sizes(const Work& w, uint32_t nsegs, uint32_t nclients, hipStream_t s) {
  hipLaunchKernelGGL(k_out_sizes, dim3(nsegs / 256 + 1), dim3(256), 0, s, w, nsegs, nclients);
  hipLaunchKernelGGL(k_out_sizes_general, dim3(std::min<uint32_t>(nsegs / 256 + 1, GEN_GRID)), dim3(256), 0, s, w, nclients);
}
void launch_encode_layout(const Work& w, uint32_t nsegs, uint32_t nclients, hipStream_t s, hipEvent_t ev_join) {
  const uint32_t grid = nsegs / 256 + 1;
  scan_u32(w.tmp, w.tmp_bytes, w.o_size, w.o_pos, nsegs + 1, s);
  hipStreamWaitEvent(s, ev_join, 0);
  hipLaunchKernelGGL(k_client_bounds, dim3(grid), dim3(256), 0, s, w, nclients, nsegs);
  hipLaunchKernelGGL(k_client_sizes, dim3(nclients / 256 + 1), dim3(256), 0, s, w, nclients, nsegs);
  if (nclients + 1 <= LAYOUT_SMALL) {
    rev_scans(w, nclients, s);  // (with the totals)
  } else {
    rev_scans(w, nclients, s);
    hipLaunchKernelGGL(k_totals, dim3(1), dim3(1), 0, s, w, nclients);
  }
}

// Phase 2: write bytes (buffers sized from a bound, checked in k_totals)
void launch_encode_write(const Work& w, uint32_t nsegs, uint32_t nclients, hipStream_t s) {
  hipLaunchKernelGGL(k_write_clients, dim3(nclients / 256 + 1), dim3(256), 0, s, w, nclients);
  if (nsegs) hipLaunchKernelGGL(k_write_runs, dim3((nsegs + 255) / 256), dim3(256), 0, s, w, nsegs);
}
void launch_write_structs(const Work& w, uint32_t nsegs, uint32_t nclients, hipStream_t s) {
  if (!nsegs) return;
  hipLaunchKernelGGL(k_write_structs, dim3((nsegs + 255) / 256), dim3(256), 0, s, w, nsegs, nclients);
  hipLaunchKernelGGL(k_write_general, dim3(std::min<uint32_t>(nsegs / 256 + 1, GEN_GRID)), dim3(256), 0, s, w, nclients);
}

// The decode of the update just encoded, from the encoder's own layout (a doc's merged state: the
// doc's next merge reads it instead of parsing the state, yc_engine.hip commit_merge): every output
// struct's start (out_pos), every client block's section record and first struct, the delete set's
// start. The bitmaps were zeroed by the caller; the count of sections is meta[0] (atomic).
__global__ void k_state_marks(Work w, uint32_t nout, uint32_t nclients, PreMarks m) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, lane = threadIdx.x & 63;
  // struct starts: positions ascend with t, so a wavefront's bits fall into few words — OR'd across
  // the lanes of a word first (segmented, by shuffles), one atomic per word and wavefront
  uint32_t word = NONE;
  uint64_t bit = 0;
  if (t < nout && w.o_size[t]) {
    const uint32_t p = (uint32_t)out_pos(w, t);
    word = p >> 6;
    bit = 1ull << (p & 63);
  }
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t ow = (uint32_t)__shfl_down((int)word, d);
    const uint64_t ob = ((uint64_t)(uint32_t)__shfl_down((int)(uint32_t)(bit >> 32), d) << 32) | (uint32_t)__shfl_down((int)(uint32_t)bit, d);
    if (lane + d < 64 && ow == word) bit |= ob;
  }
  const uint32_t prev = (uint32_t)__shfl_up((int)word, 1);
  if (word != NONE && (lane == 0 || prev != word)) atomicOr((unsigned long long*)&m.fbits[word], bit);
  // the client blocks: slot c holds client c's record (n = 0: no block); struct blocks are written
  // in descending client order (both compat modes), which k_predecoded restores when it compacts
  if (t < nclients && t < m.cap_secs) {
    const uint32_t n = ccol(w, CC_NINCL)[t];
    Section sec;
    sec.upd = 0; sec.n = n; sec.client = w.cl_vals[t]; sec.clock = w.cl_start[t];
    sec.first_pos = NONE; sec.cidx = NONE; sec.first_idx = NONE; sec.pad = 0;
    if (n) {
      const uint32_t first = (uint32_t)(w.ctr->pad[3] + ccol64(w, CC64_BLKPOS)[t] + ccol(w, CC_HDR)[t]);
      sec.first_pos = first;
      atomicOr((unsigned long long*)&m.sbits[first >> 6], 1ull << (first & 63));
      atomicAdd(&m.meta[0], 1u);
    }
    m.secs[t] = sec;
  }
  if (t == 0) { m.meta[1] = (uint32_t)w.ctr->ds_base; m.meta[2] = min(nclients, m.cap_secs); }
}
void launch_state_marks(const Work& w, uint32_t nout, uint32_t nclients, const PreMarks& m, hipStream_t s) {
  fill_u32_multi({{(uint32_t*)m.fbits, 2ull * m.nw, 0u}, {(uint32_t*)m.sbits, 2ull * m.nw, 0u}, {m.meta, 3, 0u}}, s);
  const uint32_t n = std::max(nout, nclients) + 1;
  hipLaunchKernelGGL(k_state_marks, dim3(n / 256 + 1), dim3(256), 0, s, w, nout, nclients, m);
}

// Per-document byte ranges of a multi-document encode. Clients are laid out in (document, client)
// descending order, so each document's struct blocks, delete-set blocks and state-vector entries
// are contiguous: rng[9d + 0..8] = struct (lo, hi, clients), delete set (lo, hi, clients),
// state vector (lo, hi, entries), relative to each section's first block.
__global__ void k_doc_ranges_init(unsigned long long* rng, uint32_t ndocs) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 9 * ndocs) rng[i] = (i % 3 == 0) ? ~0ull : 0ull;
}
__global__ void k_doc_ranges(Work w, uint32_t nclients, uint32_t ndocs, unsigned long long* rng) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nclients) return;
  const uint32_t d = w.cl_doc[c];
  if (d >= ndocs) { raise_err(&w.ctr->err, ERR_DECODE); return; }
  unsigned long long* r = rng + 9 * (size_t)d;
  if (ccol(w, CC_NINCL)[c]) {
    atomicMin(&r[0], (unsigned long long)ccol64(w, CC64_BLKPOS)[c]);
    atomicMax(&r[1], (unsigned long long)(ccol64(w, CC64_BLKPOS)[c] + ccol(w, CC_BLK)[c]));
    atomicAdd(&r[2], 1ull);
  }
  if (ccol(w, CC_NRUNS)[c]) {
    atomicMin(&r[3], (unsigned long long)ccol64(w, CC64_DSPOS)[c]);
    atomicMax(&r[4], (unsigned long long)(ccol64(w, CC64_DSPOS)[c] + ccol(w, CC_DSBLK)[c]));
    atomicAdd(&r[5], 1ull);
  }
  if (ccol(w, CC_SV)[c]) {
    atomicMin(&r[6], (unsigned long long)ccol64(w, CC64_SVPOS)[c]);
    atomicMax(&r[7], (unsigned long long)(ccol64(w, CC64_SVPOS)[c] + ccol(w, CC_SV)[c]));
    atomicAdd(&r[8], 1ull);
  }
}
void launch_doc_ranges(const Work& w, uint32_t nclients, uint32_t ndocs, unsigned long long* rng, hipStream_t s) {
  hipLaunchKernelGGL(k_doc_ranges_init, dim3(9 * ndocs / 256 + 1), dim3(256), 0, s, rng, ndocs);
  if (nclients) hipLaunchKernelGGL(k_doc_ranges, dim3(nclients / 256 + 1), dim3(256), 0, s, w, nclients, ndocs, rng);
}

}  // namespace yc
