// yc_view.hip — K8: materialised view of a merged doc (the crdt.c cache, reference crdt.js:297-305,
// 372, 494, 528, 555, 581, 607) on gfx950.
//
// After a merge the device already knows, per list (root type / nested type / YMap entry):
//   * YMap entries (k_winner): the rightmost item of the entry is its value (YMap.get / toJSON,
//     typeMapGetAll Y@49897 reads `_map.get(key)`, i.e. that item, and skips it when deleted);
//   * YArray lists (g_right after k_yata): the integrated linked list.
// This pass turns that into an ordered, compacted view the host can read in one copy:
//   k_vkeys       compacts the live lists (not under a deleted type) into ViewKey records
//   k_vrep        one root member per list (the item that names parent / parentSub)
//   k_vkey_fill   parent, names, YMap winner value (last element of the winning item)
//   k_vlist_*     list ranking of every YArray list by pointer jumping over g_right (Wyllie,
//                 double buffered), then a scatter into document order
//   k_vseg_fill   one ViewSeg per array member in document order: id, length, deleted /
//                 countable, content element byte range (ContentX.splice as a byte slice)
// The host (yc_engine.hip) decodes values from those byte ranges (typeListToArray Y@46408,
// YMap.toJSON Y@51558) and encodes local ops against the ids (typeMapSet Y@49334,
// typeListInsertGenerics Y@48365, typeListDelete Y@48835).
#include "yc_work.h"

namespace yc {

__device__ __forceinline__ bool countable_ref(uint32_t ref) { return ref != REF_DELETED && ref != REF_FORMAT; }

// ViewSeg of segment s: every element, or only the last one (a YMap entry's value)
__device__ void fill_seg(const Work& w, uint32_t s, bool last_only, ViewSeg& v) {
  const uint32_t g0 = seg_start(w, s), g1 = seg_start(w, s + 1);
  const uint32_t cidx = w.g_cidx[s], own = w.g_src[s];
  const uint32_t clock = (uint32_t)(g0 - w.cl_base[cidx]);
  const uint32_t f = w.g_flags[s];
  const uint32_t ref = w.s_info[own] & 31u;
  v.client = w.cl_vals[cidx];
  v.clock = clock;
  v.len = g1 - g0;
  v.unit = g0;
  v.ref = ref;
  v.flags = VS_SET | ((f & SEG_DEL) ? VS_DELETED : 0u) | (countable_ref(ref) ? VS_COUNTABLE : 0u) | ((f & SEG_ITEM) ? VS_ITEM : 0u);
  v.b0 = v.b1 = 0;
  if ((f & SEG_DEL) || !(f & SEG_ITEM)) return;
  const uint32_t e1 = clock + v.len - w.s_clock[own];
  const uint32_t e0 = last_only ? e1 - 1 : clock - w.s_clock[own];
  uint32_t b0 = 0, b1 = 0;
  if (!content_slice(w, own, e0, e1, b0, b1)) { raise_err(&w.ctr->err, ERR_DECODE); return; }
  v.b0 = b0;
  v.b1 = b1;
}

__device__ void str_text(const Work& w, uint32_t pos, uint32_t len, uint32_t& tpos, uint32_t& tlen) {
  uint32_t p = pos;
  bool ok = true;
  const uint32_t n = rd_vu(w.bytes, p, pos + len, ok);
  if (!ok || p + n != pos + len) { raise_err(&w.ctr->err, ERR_DECODE); return; }
  tpos = p;
  tlen = n;
}

__global__ void k_vkeys(Work w, uint32_t* __restrict__ kmap, uint32_t* __restrict__ krep, ViewKey* __restrict__ keys,
                        uint32_t* __restrict__ nkeys) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= w.cap_keys) return;
  krep[k] = NONE;
  kmap[k] = NONE;
  if (w.k_hash[k] == 0 || (w.k_flags[k] & KF_DEAD)) return;
  const uint32_t i = atomicAdd(nkeys, 1u);
  kmap[k] = i;
  keys[i].slot = k;
}

__global__ void k_vrep(Work w, uint32_t nsegs, const uint32_t* __restrict__ kmap, uint32_t* __restrict__ krep) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsegs) return;
  const uint32_t f = w.g_flags[s];
  if (!(f & SEG_ROOT) || !(f & SEG_ITEM)) return;
  const uint32_t k = w.g_key[s];
  if (k != NONE && kmap[k] != NONE) atomicMin(&krep[k], s);
}

__device__ __forceinline__ void vkey_fill_at(const Work& w, const uint32_t* __restrict__ krep, ViewKey* __restrict__ keys, uint32_t i) {
  ViewKey& K = keys[i];
  const uint32_t k = K.slot;
  K.flags = (w.k_flags[k] & KF_PSUB) ? VK_PSUB : 0u;
  K.parent_unit = w.k_parent[k];
  K.name_pos = K.name_len = 0;
  K.psub_pos = K.psub_len = 0;
  K.seg0 = K.nseg = 0;
  const uint32_t r = ld_fresh(&krep[k]);  // (atomicMin: read through L2, k_view_small's phases)
  if (r != NONE) {
    const uint32_t own = w.g_src[r];
    // the struct table keeps whole varStrings (length prefix included): the view holds the text
    if ((w.s_pk[own] & 3u) == 1) str_text(w, w.s_pa[own], w.s_pb[own], K.name_pos, K.name_len);
    if (w.s_psub[own] != NONE) str_text(w, w.s_psub[own], w.s_psublen[own], K.psub_pos, K.psub_len);
  } else {
    raise_err(&w.ctr->err, ERR_DECODE);  // every live list has a member that names it
  }
  K.win.client = NONE;
  K.win.flags = 0;
  if (K.flags & VK_PSUB) {
    const uint32_t s = w.k_winner[k];
    if (s != NONE) fill_seg(w, s, true, K.win);
  }
}
__global__ void k_vkey_fill(Work w, const uint32_t* __restrict__ krep, ViewKey* __restrict__ keys,
                            const uint32_t* __restrict__ nkeys) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < *nkeys) vkey_fill_at(w, krep, keys, i);
}
// A small view with no YArray list (the per-op path's map doc): the key compaction, the root
// members and the key records as phases of ONE workgroup (a fill and three launches otherwise)
constexpr uint32_t VS_LANES = 512, VS_SMALL = VS_LANES * 16;
__global__ __launch_bounds__(VS_LANES) void k_view_small(Work w, uint32_t nsegs, uint32_t* __restrict__ kmap, uint32_t* __restrict__ krep,
                                                         ViewKey* __restrict__ keys, uint32_t* __restrict__ nkeys) {
  __shared__ uint32_t n;
  const uint32_t t = threadIdx.x;
  if (t == 0) n = 0;
  __syncthreads();
  for (uint32_t k = t; k < w.cap_keys; k += VS_LANES) {
    krep[k] = NONE;
    kmap[k] = NONE;
    if (w.k_hash[k] == 0 || (w.k_flags[k] & KF_DEAD)) continue;
    const uint32_t i = atomicAdd(&n, 1u);
    kmap[k] = i;
    keys[i].slot = k;
  }
  __syncthreads();
  for (uint32_t s = t; s < nsegs; s += VS_LANES) {
    const uint32_t f = w.g_flags[s];
    if (!(f & SEG_ROOT) || !(f & SEG_ITEM)) continue;
    const uint32_t k = w.g_key[s];
    if (k != NONE && kmap[k] != NONE) atomicMin(&krep[k], s);
  }
  __syncthreads();  // (krep, written by atomicMin, is read with ld_fresh)
  const uint32_t nk = n;
  if (t == 0) *nkeys = nk;
  for (uint32_t i = t; i < nk; i += VS_LANES) vkey_fill_at(w, krep, keys, i);
}

// ---- YArray list ranking. Positions i index the (list, segment)-sorted member array y_seg.
__global__ void k_vlist_init(Work w, uint32_t narr, uint32_t* __restrict__ pos_of) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < narr) pos_of[w.y_seg[i]] = i;
}
__global__ void k_vlist_links(Work w, uint32_t narr, const uint32_t* __restrict__ pos_of, uint32_t* __restrict__ d,
                              uint32_t* __restrict__ nx) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= narr) return;
  const uint32_t r = w.g_right[w.y_seg[i]];
  nx[i] = r == NONE ? NONE : pos_of[r];
  d[i] = r == NONE ? 0u : 1u;
}
// one Wyllie round: distance to the end of the list
__global__ void k_vlist_jump(uint32_t narr, const uint32_t* __restrict__ d0, const uint32_t* __restrict__ n0,
                             uint32_t* __restrict__ d1, uint32_t* __restrict__ n1) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= narr) return;
  const uint32_t n = n0[i];
  if (n == NONE) { d1[i] = d0[i]; n1[i] = NONE; return; }
  d1[i] = d0[i] + d0[n];
  n1[i] = n0[n];
}
__global__ void k_vlist_scatter(Work w, uint32_t narr, uint32_t nlists, const uint32_t* __restrict__ d,
                                uint32_t* __restrict__ order) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= narr) return;
  uint32_t lo = 0, hi = nlists;  // last list l with y_lstart[l] <= i
  while (hi - lo > 1) { const uint32_t m = (lo + hi) >> 1; if (w.y_lstart[m] <= i) lo = m; else hi = m; }
  const uint32_t end = w.y_lstart[lo + 1];
  const uint32_t dist = d[i];
  if (dist >= end - w.y_lstart[lo]) { raise_err(&w.ctr->err, ERR_DECODE); return; }  // not one list
  order[end - 1 - dist] = w.y_seg[i];
}
__global__ void k_vlist_keys(Work w, uint32_t nlists, const uint32_t* __restrict__ kmap, ViewKey* __restrict__ keys) {
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= nlists) return;
  const uint32_t a = w.y_lstart[l], b = w.y_lstart[l + 1];
  const uint32_t i = kmap[w.y_keys[a]];
  if (i == NONE) return;
  keys[i].seg0 = a;
  keys[i].nseg = b - a;
}
__global__ void k_vseg_fill(Work w, uint32_t narr, const uint32_t* __restrict__ order, ViewSeg* __restrict__ segs) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= narr) return;
  fill_seg(w, order[p], false, segs[p]);
}

void launch_view(const Work& w, const ViewBufs& v, uint32_t nsegs, uint32_t nlists, uint32_t narr, hipStream_t s) {
  if ((!nlists || !narr) && w.cap_keys <= VS_SMALL && nsegs <= VS_SMALL && !env_off("YCRDT_VIEW_SMALL")) {
    hipLaunchKernelGGL(k_view_small, dim3(1), dim3(VS_LANES), 0, s, w, nsegs, v.kmap, v.krep, v.keys, v.nkeys);
    return;
  }
  hipMemsetAsync(v.nkeys, 0, sizeof(uint32_t), s);
  hipLaunchKernelGGL(k_vkeys, dim3(w.cap_keys / 256 + 1), dim3(256), 0, s, w, v.kmap, v.krep, v.keys, v.nkeys);
  if (nsegs) hipLaunchKernelGGL(k_vrep, dim3(nsegs / 256 + 1), dim3(256), 0, s, w, nsegs, v.kmap, v.krep);
  hipLaunchKernelGGL(k_vkey_fill, dim3(w.cap_keys / 256 + 1), dim3(256), 0, s, w, v.krep, v.keys, v.nkeys);
  if (!nlists || !narr) return;
  const uint32_t g = narr / 256 + 1;
  hipLaunchKernelGGL(k_vlist_init, dim3(g), dim3(256), 0, s, w, narr, v.pos_of);
  hipLaunchKernelGGL(k_vlist_links, dim3(g), dim3(256), 0, s, w, narr, v.pos_of, v.d0, v.n0);
  uint32_t* d0 = v.d0; uint32_t* n0 = v.n0; uint32_t* d1 = v.d1; uint32_t* n1 = v.n1;
  for (uint64_t span = 1; span < narr; span <<= 1) {
    hipLaunchKernelGGL(k_vlist_jump, dim3(g), dim3(256), 0, s, narr, d0, n0, d1, n1);
    std::swap(d0, d1);
    std::swap(n0, n1);
  }
  hipLaunchKernelGGL(k_vlist_scatter, dim3(g), dim3(256), 0, s, w, narr, nlists, d0, v.order);
  hipLaunchKernelGGL(k_vlist_keys, dim3(nlists / 256 + 1), dim3(256), 0, s, w, nlists, v.kmap, v.keys);
  hipLaunchKernelGGL(k_vseg_fill, dim3(g), dim3(256), 0, s, w, narr, v.order, v.segs);
}

}  // namespace yc
