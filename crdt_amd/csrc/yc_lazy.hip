// yc_lazy.hip — Y.mergeUpdates / Y.diffUpdate on gfx950 (lazy struct merge; no integration).
//
// Restates mergeUpdatesV2 (`ds`, Y@39011) and diffUpdateV2 (`us`, Y@40711) over the struct table
// decoded by yc_decode.hip in lazy mode (references kept as raw client ids):
//
//   mergeUpdates  Yjs re-sorts its readers (one per update) before every step: client desc, clock
//                 asc, stable. Structs of one client only ever meet structs of the same client,
//                 so every client is an independent k-way merge — one wavefront per client —
//                 EXCEPT for the tie order of readers sitting on the same clock: a stable sort
//                 keeps the previous relative order, and the reader that moved last was the front
//                 one, so ties go to the most recent arrival (arrival stamp = processing time).
//                 A reader arrives at its section of client c when it leaves its previous
//                 section (a higher client, processed earlier), so wavefronts run in client-desc
//                 order and pick the arrival stamps of their readers up from the wavefronts of
//                 the higher clients (decoupled look-back: a wave only waits on lower block ids).
//   diffUpdate    a single reader: per section, the first non-Skip struct ending past the state
//                 vector is written with an offset, every later struct of the section as is.
//
// Both produce "events" (struct, offset, length | GC | Skip) per output client block; a size pass,
// scans and a write pass encode them with the lazy Item.write rules (parentSub only on items that
// carry neither origin nor right origin, Y@36564). Delete sets: mergeDeleteSets + sortAndMerge
// (`he`/`le`, Y@10486) as a sort + segmented running-max scan; diffUpdate copies its input's.
#include "yc_work.h"

namespace yc {

constexpr uint32_t LZ_KMAX = 1024;  // readers (updates) per client handled in LDS
constexpr uint32_t END = NONE;

// ---------------------------------------------------------------- section order / reader runs
// key = (client rank) << 32 | update, rank 0 = the highest client
__global__ void k_lz_keys(Work w, uint32_t nsections, uint32_t nclients) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsections) return;
  const Section s = w.sections[i];
  w.lz_key[i] = ((uint64_t)(nclients - 1 - s.cidx) << 32) | s.upd;
  w.lz_iota[i] = i;
}
__global__ void k_lz_runs(Work w, uint32_t nsections, uint32_t nclients) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsections) return;
  const uint64_t k = w.lz_keys[i];
  const uint32_t r = (uint32_t)(k >> 32);
  if (i == 0 || (uint32_t)(w.lz_keys[i - 1] >> 32) != r) w.lz_rstart[r] = i;
  if (i == nsections - 1) w.lz_rstart[nclients] = nsections;
}
// one lane per update: previous non-empty section (arrival source), client-desc check
__device__ __forceinline__ uint32_t first_nonskip(const Work& w, uint32_t a, uint32_t n) {
  for (uint32_t j = a; j < a + n; ++j)
    if ((w.s_info[j] & 31u) != REF_SKIP) return j;
  return END;
}
__global__ void k_lz_prev(Work w, uint32_t nupd) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= nupd) return;
  const uint32_t a = w.usec_start[u], b = a + w.usec_n[u];
  uint32_t prev = NONE;
  for (uint32_t i = a; i < b; ++i) {
    const Section s = w.sections[i];
    w.lz_prev[i] = prev;
    const uint32_t f = s.n ? first_nonskip(w, s.first_idx, s.n) : END;
    w.lz_first[i] = f;
    if (f != END) prev = i;
  }
}
// per client: event capacity (every advance emits at most one struct and one Skip)
__global__ void k_lz_cap(Work w, uint32_t nclients) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r > nclients) return;
  if (r == nclients) { w.lz_cap[r] = 0; return; }
  uint32_t tot = 0;
  for (uint32_t i = w.lz_rstart[r]; i < w.lz_rstart[r + 1]; ++i) tot += w.sections[w.lz_sec[i]].n;
  w.lz_cap[r] = 2 * tot + 2;
}

// ---------------------------------------------------------------- the per-client lazy merge
struct Cur {
  uint32_t kind;   // REF_GC, REF_SKIP or 1 (item)
  uint32_t src;    // source struct (items)
  uint32_t clock;  // first clock (source clock + offset)
  uint32_t len;
};

__global__ __launch_bounds__(64) void k_lz_merge(Work w, uint32_t nclients, unsigned long long* ord, unsigned long long ord_base) {
  __shared__ uint32_t rcur[LZ_KMAX], rend[LZ_KMAX], rhi[LZ_KMAX], rlo[LZ_KMAX];
  // client rank (descending client order) in workgroup start order: the stamps it waits for come
  // from lower ranks, i.e. from workgroups already running (ordered_block_id, yc_work.h)
  const uint32_t r = ordered_block_id(ord, ord_base);
  const uint32_t lane = threadIdx.x;
  const uint32_t a = w.lz_rstart[r], K = w.lz_rstart[r + 1] - a;
  const uint32_t base = w.lz_evbase[r];
  const uint32_t cap = w.lz_cap[r];
  bool fail = K > LZ_KMAX;
  if (fail && lane == 0) raise_err(&w.ctr->err, ERR_CAPACITY);
  // ---- readers: first struct + arrival stamp (look back to the previous section's wave)
  for (uint32_t k = lane; k < K && !fail; k += 64) {
    const uint32_t sec = w.lz_sec[a + k];
    const Section S = w.sections[sec];
    rcur[k] = w.lz_first[sec];
    rend[k] = S.first_idx + S.n;
    const uint32_t p = w.lz_prev[sec];
    if (p == NONE) { rhi[k] = 0; rlo[k] = 0xFFFFFFFFu - S.upd; }  // never moved: update order
    else {
      uint32_t spins = 0;
      while (__hip_atomic_load(&w.lz_flag[p], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1u << 24)) { raise_err(&w.ctr->err, ERR_CAPACITY); break; }
      }
      rhi[k] = w.lz_leave_hi[p];
      rlo[k] = w.lz_leave_lo[p];
    }
  }
  __syncthreads();
  const uint32_t rank_stamp = r + 1;
  uint32_t step = 0, evn = 0;
  Cur cur{0, NONE, 0, 0};
  bool have = false;
  auto emit = [&](const Cur& c) {
    if (evn < cap) {
      if (lane == 0) {
        w.ev_kind[base + evn] = c.kind;
        w.ev_src[base + evn] = c.src;
        w.ev_clock[base + evn] = c.clock;
        w.ev_len[base + evn] = c.len;
      }
      ++evn;
    } else if (lane == 0) raise_err(&w.ctr->err, ERR_CAPACITY);
  };
  auto advance = [&](uint32_t t) {
    uint32_t c = rcur[t] + 1;
    const uint32_t e = rend[t];
    while (c < e && (w.s_info[c] & 31u) == REF_SKIP) ++c;
    ++step;
    __syncthreads();
    if (lane == 0) {
      rcur[t] = c < e ? c : END;
      rhi[t] = rank_stamp;
      rlo[t] = step;
    }
    __syncthreads();
  };
  auto kind_of = [&](uint32_t s) -> uint32_t {
    const uint32_t ref = w.s_info[s] & 31u;
    return ref == REF_GC ? (uint32_t)REF_GC : ref == REF_SKIP ? (uint32_t)REF_SKIP : 1u;
  };
  const uint32_t max_iter = 4 * cap + 16;
  for (uint32_t it = 0; !fail; ++it) {
    if (it > max_iter) { if (lane == 0) raise_err(&w.ctr->err, ERR_CAPACITY); break; }
    // front reader: min (clock), ties → latest arrival (max stamp)
    uint32_t bk = NONE, bc = 0xFFFFFFFFu, bh = 0, bl = 0;
    for (uint32_t k = lane; k < K; k += 64) {
      const uint32_t s = rcur[k];
      if (s == END) continue;
      const uint32_t c = w.s_clock[s], h = rhi[k], l = rlo[k];
      if (bk == NONE || c < bc || (c == bc && (h > bh || (h == bh && l > bl)))) { bk = k; bc = c; bh = h; bl = l; }
    }
    for (int off = 32; off > 0; off >>= 1) {
      const uint32_t ok = __shfl_xor(bk, off), oc = __shfl_xor(bc, off), oh = __shfl_xor(bh, off), ol = __shfl_xor(bl, off);
      if (ok != NONE && (bk == NONE || oc < bc || (oc == bc && (oh > bh || (oh == bh && ol > bl))))) { bk = ok; bc = oc; bh = oh; bl = ol; }
    }
    if (bk == NONE) break;  // every reader of this client is exhausted
    const uint32_t t = bk;
    uint32_t n = rcur[t];
    if (have) {
      bool skipped = false;
      const uint32_t cend = cur.clock + cur.len;
      while (n != END && w.s_clock[n] + w.s_len[n] <= cend) { advance(t); n = rcur[t]; skipped = true; }
      if (n == END || (skipped && w.s_clock[n] > cend)) continue;
      const uint32_t nclock = w.s_clock[n], nlen = w.s_len[n];
      if (cend < nclock) {  // gap
        if (cur.kind == REF_SKIP) cur.len = nclock + nlen - cur.clock;
        else { emit(cur); cur = Cur{REF_SKIP, NONE, cend, nclock - cend}; }
      } else {
        const uint32_t diff = cend - nclock;
        Cur nn{kind_of(n), n, nclock, nlen};
        if (diff > 0) {
          if (cur.kind == REF_SKIP) cur.len -= diff;
          else { nn.clock += diff; nn.len -= diff; }  // sliceStruct
        }
        if (cur.kind == nn.kind && cur.kind != 1u) cur.len += nn.len;  // GC / Skip mergeWith
        else { emit(cur); cur = nn; advance(t); }
      }
    } else {
      cur = Cur{kind_of(n), n, w.s_clock[n], w.s_len[n]};
      have = true;
      advance(t);
    }
    // consecutive structs of the same reader are written without re-sorting
    n = rcur[t];
    while (n != END && w.s_clock[n] == cur.clock + cur.len && kind_of(n) != REF_SKIP) {
      emit(cur);
      cur = Cur{kind_of(n), n, w.s_clock[n], w.s_len[n]};
      advance(t);
      n = rcur[t];
    }
  }
  if (have && !fail) emit(cur);
  if (lane == 0) w.lz_evn[r] = evn;
  // ---- publish the leave stamps of this client's sections
  __syncthreads();
  for (uint32_t k = lane; k < K && k < LZ_KMAX; k += 64) {
    const uint32_t sec = w.lz_sec[a + k];
    w.lz_leave_hi[sec] = rhi[k];
    w.lz_leave_lo[sec] = rlo[k];
    __hip_atomic_store(&w.lz_flag[sec], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (fail) {  // never leave a dependent wave spinning
    for (uint32_t k = lane; k < K; k += 64) __hip_atomic_store(&w.lz_flag[w.lz_sec[a + k]], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---------------------------------------------------------------- non-canonical input: one loop
// An update whose struct section holds two sections of one client, or sections out of the
// descending client order Yjs writes, breaks the per-client split above (a reader may come back to
// a higher client). Such input is valid for Yjs's readers, so it runs mergeUpdatesV2's loop
// (Y@39011) as written, over all readers in one workgroup: each step picks the front reader
// (client desc, clock asc, ties to the latest arrival — the stable re-sort), and the output
// sections follow the lazy writer (a new section whenever the client changes, Y@38735).
// k_ds_bound (yc_decode.hip) flags such input; it is rare, and the loop is serial.
__global__ __launch_bounds__(64) void k_lz_merge_seq(Work w, uint32_t nupd, uint32_t cap_ev, uint32_t cap_blk) {
  __shared__ uint32_t rcur[LZ_KMAX], rend[LZ_KMAX], rhi[LZ_KMAX], rlo[LZ_KMAX];
  const uint32_t lane = threadIdx.x;
  const uint32_t K = nupd;
  if (K > LZ_KMAX) { if (lane == 0) raise_err(&w.ctr->err, ERR_CAPACITY); return; }
  auto skip_of = [&](uint32_t s) { return (w.s_info[s] & 31u) == REF_SKIP; };
  for (uint32_t k = lane; k < K; k += 64) {  // reader k: the structs of update k, Skips filtered
    const uint32_t a = w.usec_start[k], b = a + w.usec_n[k];
    uint32_t first = END, tot = 0;
    for (uint32_t t = a; t < b; ++t) {
      const Section S = w.sections[t];
      if (!S.n) continue;
      if (first == END) first = S.first_idx;
      tot += S.n;
    }
    uint32_t c = first, e = first == END ? END : first + tot;
    if (first != END) while (c < e && skip_of(c)) ++c;
    rcur[k] = (first == END || c >= e) ? END : c;
    rend[k] = e;
    rhi[k] = 0;
    rlo[k] = 0xFFFFFFFFu - k;  // never moved: update order
  }
  __syncthreads();
  auto client_of = [&](uint32_t s) { return w.sections[w.s_sec[s]].client; };
  auto kind_of = [&](uint32_t s) -> uint32_t {
    const uint32_t ref = w.s_info[s] & 31u;
    return ref == REF_GC ? (uint32_t)REF_GC : ref == REF_SKIP ? (uint32_t)REF_SKIP : 1u;
  };
  uint32_t step = 0, evn = 0, nb = 0, last_client = 0;
  bool fail = false;
  auto emit = [&](const Cur& c, uint32_t client) {
    if (evn >= cap_ev || nb >= cap_blk) { fail = true; return; }
    if (evn == 0 || client != last_client) {
      if (lane == 0) { w.lz_evbase[nb] = evn; w.lz_bclient[nb] = client; w.lz_evn[nb] = 0; }
      ++nb;
      last_client = client;
    }
    if (lane == 0) {
      w.ev_kind[evn] = c.kind;
      w.ev_src[evn] = c.src;
      w.ev_clock[evn] = c.clock;
      w.ev_len[evn] = c.len;
      w.lz_evn[nb - 1] += 1;
    }
    ++evn;
  };
  auto advance = [&](uint32_t t) {
    uint32_t c = rcur[t] + 1;
    const uint32_t e = rend[t];
    while (c < e && skip_of(c)) ++c;
    ++step;
    __syncthreads();
    if (lane == 0) {
      rcur[t] = c < e ? c : END;
      rhi[t] = 1;
      rlo[t] = step;
    }
    __syncthreads();
  };
  Cur cur{0, NONE, 0, 0};
  uint32_t cur_client = 0;
  bool have = false;
  uint64_t guard = 0;
  const uint64_t max_iter = 8ull * cap_ev + 64;
  for (;;) {
    if (++guard > max_iter || fail) { fail = true; break; }
    // front reader: max client, then min clock, then the latest arrival (max stamp)
    uint32_t bk = NONE, bcl = 0, bc = 0, bh = 0, bl = 0;
    for (uint32_t k = lane; k < K; k += 64) {
      const uint32_t s = rcur[k];
      if (s == END) continue;
      const uint32_t cl = client_of(s), c = w.s_clock[s], h = rhi[k], l = rlo[k];
      if (bk == NONE || cl > bcl || (cl == bcl && (c < bc || (c == bc && (h > bh || (h == bh && l > bl)))))) {
        bk = k; bcl = cl; bc = c; bh = h; bl = l;
      }
    }
    for (int off = 32; off > 0; off >>= 1) {
      const uint32_t ok = __shfl_xor(bk, off), ocl = __shfl_xor(bcl, off), oc = __shfl_xor(bc, off), oh = __shfl_xor(bh, off),
                     ol = __shfl_xor(bl, off);
      if (ok != NONE && (bk == NONE || ocl > bcl || (ocl == bcl && (oc < bc || (oc == bc && (oh > bh || (oh == bh && ol > bl))))))) {
        bk = ok; bcl = ocl; bc = oc; bh = oh; bl = ol;
      }
    }
    if (bk == NONE) break;  // every reader is exhausted
    const uint32_t t = bk, first_client = bcl;
    uint32_t n = rcur[t];
    if (have) {
      bool iterated = false;
      const uint32_t cend = cur.clock + cur.len;
      while (n != END && w.s_clock[n] + w.s_len[n] <= cend && client_of(n) >= cur_client) { advance(t); n = rcur[t]; iterated = true; }
      if (n == END || client_of(n) != first_client || (iterated && w.s_clock[n] > cend)) continue;
      if (first_client != cur_client) {
        emit(cur, cur_client);
        cur = Cur{kind_of(n), n, w.s_clock[n], w.s_len[n]};
        cur_client = first_client;
        advance(t);
      } else {
        const uint32_t nclock = w.s_clock[n], nlen = w.s_len[n];
        if (cend < nclock) {  // gap
          if (cur.kind == REF_SKIP) cur.len = nclock + nlen - cur.clock;
          else { emit(cur, cur_client); cur = Cur{REF_SKIP, NONE, cend, nclock - cend}; }
        } else {
          const uint32_t diff = cend - nclock;
          Cur nn{kind_of(n), n, nclock, nlen};
          if (diff > 0) {
            if (cur.kind == REF_SKIP) cur.len -= diff;
            else { nn.clock += diff; nn.len -= diff; }  // sliceStruct
          }
          if (cur.kind == nn.kind && cur.kind != 1u) cur.len += nn.len;  // GC / Skip mergeWith (the reader stays)
          else { emit(cur, cur_client); cur = nn; advance(t); }
        }
      }
    } else {
      cur = Cur{kind_of(n), n, w.s_clock[n], w.s_len[n]};
      cur_client = first_client;
      have = true;
      advance(t);
    }
    // consecutive structs of the front reader are written without re-sorting
    n = rcur[t];
    while (n != END && client_of(n) == first_client && w.s_clock[n] == cur.clock + cur.len && kind_of(n) != REF_SKIP) {
      emit(cur, cur_client);
      cur = Cur{kind_of(n), n, w.s_clock[n], w.s_len[n]};
      advance(t);
      n = rcur[t];
    }
  }
  if (have && !fail) emit(cur, cur_client);
  if (lane == 0) {
    if (fail) raise_err(&w.ctr->err, ERR_CAPACITY);
    w.lz_evbase[nb] = evn;
    w.ctr->lz_blocks = nb;
  }
}

// ---------------------------------------------------------------- diffUpdate events
// One lane per section: the section's events live at lz_evbase[section]. Yjs's reader runs on
// while the client stays the same (diffUpdateV2, Y@40711: `while (reader.curr.id.client ===
// currClient)`), so adjacent sections of one client (a layout Yjs never writes, but reads) are one
// run: its first section's lane handles all of them and the others stay empty.
__device__ __forceinline__ bool lz_run_start(const Work& w, uint32_t i) {
  return i == 0 || w.sections[i - 1].upd != w.sections[i].upd || w.sections[i - 1].client != w.sections[i].client;
}
__global__ void k_lz_diff(Work w, uint32_t nsections) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsections) return;
  const Section S = w.sections[i];
  const uint32_t base = w.lz_evbase[i];
  if (!lz_run_start(w, i)) { w.lz_evn[i] = 0; return; }
  uint32_t j = i + 1, nrun = S.n;  // the run: sections [i, j)
  while (j < nsections && !lz_run_start(w, j)) nrun += w.sections[j++].n;
  uint32_t svc = 0;  // target state of this client (lz_multi: in this update's own state vector)
  {
    const uint32_t sv0 = w.lz_multi ? w.sv_off[S.upd] : 0u, sv1 = w.lz_multi ? w.sv_off[S.upd + 1] : w.sv_n;
    uint32_t lo = sv0, hi = sv1;
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (w.sv_client[m] < S.client) lo = m + 1; else hi = m; }
    if (lo < sv1 && w.sv_client[lo] == S.client) svc = w.sv_clock[lo];
  }
  uint32_t evn = 0;
  auto put = [&](uint32_t j2, uint32_t off) {
    const uint32_t ref = w.s_info[j2] & 31u;
    w.ev_kind[base + evn] = ref == REF_GC ? (uint32_t)REF_GC : ref == REF_SKIP ? (uint32_t)REF_SKIP : 1u;
    w.ev_src[base + evn] = j2;
    w.ev_clock[base + evn] = w.s_clock[j2] + off;
    w.ev_len[base + evn] = w.s_len[j2] - off;
    ++evn;
  };
  if (j == i + 1) {
    // one section (clocks ascending): the first struct (non-Skip) that ends past the target state by
    // a binary search, then everything after it
    uint32_t lo = S.first_idx, hi = S.first_idx + S.n;
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (w.s_clock[m] + w.s_len[m] <= svc) lo = m + 1; else hi = m; }
    while (lo < S.first_idx + S.n && (w.s_info[lo] & 31u) == REF_SKIP) ++lo;
    for (uint32_t k = lo; k < S.first_idx + S.n; ++k) put(k, (k == lo && svc > w.s_clock[k]) ? svc - w.s_clock[k] : 0u);
  } else {
    // several sections: Yjs's loop struct by struct (clocks need not ascend across sections)
    uint32_t k = 0;
    for (uint32_t t = i; t < j; ++t)
      if (w.sections[t].n) { k = w.sections[t].first_idx; break; }  // (empty sections have no first struct)
    const uint32_t kend = k + nrun;
    bool writing = false;
    while (k < kend) {
      if (writing) { put(k++, 0); continue; }
      const uint32_t c = w.s_clock[k], l = w.s_len[k];
      if ((w.s_info[k] & 31u) == REF_SKIP) { ++k; continue; }
      if (c + l > svc) { put(k++, svc > c ? svc - c : 0u); writing = true; }
      else while (k < kend && w.s_clock[k] + w.s_len[k] <= svc) ++k;
    }
  }
  w.lz_evn[i] = evn;
}
__global__ void k_lz_diff_cap(Work w, uint32_t nsections) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > nsections) return;
  uint32_t n = 0;
  if (i < nsections && lz_run_start(w, i)) {
    n = w.sections[i].n;
    for (uint32_t j = i + 1; j < nsections && !lz_run_start(w, j); ++j) n += w.sections[j].n;
  }
  w.lz_cap[i] = n;
}

// ---------------------------------------------------------------- event encoding
// Lazy Item.write (Y@80416 on a lazily read item): parentSub survives only on items that carry
// neither origin nor right origin; an offset > 0 turns the origin into (client, clock + off - 1).
template <bool WRITE>
__device__ uint32_t encode_event(const Work& w, uint32_t client, uint32_t e, uint8_t* __restrict__ out, uint32_t p0) {
  const uint32_t kind = w.ev_kind[e], len = w.ev_len[e];
  uint32_t p = p0;
  if (kind != 1u) {
    if (WRITE) { out[p++] = (uint8_t)kind; p = wr_vu(out, p, len); return p - p0; }
    return 1 + vu_size(len);
  }
  const uint32_t src = w.ev_src[e];
  const uint32_t info0 = w.s_info[src];
  const uint32_t ref = info0 & 31u;
  const uint32_t off = w.ev_clock[e] - w.s_clock[src];
  const bool root = (info0 & 0xC0u) == 0;
  const bool has_o = off > 0 || (info0 & 0x80u);
  const bool has_r = (info0 & 0x40u) != 0;
  const bool psub = root && (info0 & 0x20u);
  const uint32_t oc = off > 0 ? client : w.s_ocidx[src], ok = off > 0 ? w.s_clock[src] + off - 1 : w.s_oclock[src];
  uint32_t size = 1;
  if (WRITE) out[p++] = (uint8_t)(ref | (has_o ? 0x80u : 0u) | (has_r ? 0x40u : 0u) | (psub ? 0x20u : 0u));
  if (has_o) {
    if (WRITE) { p = wr_vu(out, p, oc); p = wr_vu(out, p, ok); }
    size += vu_size(oc) + vu_size(ok);
  }
  if (has_r) {
    const uint32_t rc = w.s_rcidx[src], rk = w.s_rclock[src];
    if (WRITE) { p = wr_vu(out, p, rc); p = wr_vu(out, p, rk); }
    size += vu_size(rc) + vu_size(rk);
  }
  if (!has_o && !has_r) {
    const uint32_t pa = w.s_pa[src], pb = w.s_pb[src];
    if ((w.s_pk[src] & 3u) == 1) {
      if (WRITE) { out[p++] = 1; for (uint32_t i = 0; i < pb; ++i) out[p++] = w.bytes[pa + i]; }
      size += 1 + pb;
    } else {
      if (WRITE) { out[p++] = 0; p = wr_vu(out, p, pa); p = wr_vu(out, p, pb); }
      size += 1 + vu_size(pa) + vu_size(pb);
    }
    if (psub) {
      const uint32_t ps = w.s_psub[src], pl = w.s_psublen[src];
      if (WRITE) for (uint32_t i = 0; i < pl; ++i) out[p++] = w.bytes[ps + i];
      size += pl;
    }
  }
  if (ref == REF_DELETED) {
    if (WRITE) p = wr_vu(out, p, len);
    size += vu_size(len);
  } else if (ref == REF_ANY && (w.s_pk[src] & 0x40u)) {  // `any` values not in writeAny's form
    if (WRITE) p = wr_vu(out, p, len);
    const uint32_t nb = any_canon<WRITE>(w.bytes, w.s_celem[src], w.s_cend[src], off, off + len, out, p);
    size += vu_size(len) + nb;
  } else if (ref == REF_ANY || ref == REF_JSON || ref == REF_STRING) {
    uint32_t b0 = 0, b1 = 0;
    if (!content_slice(w, src, off, off + len, b0, b1)) { raise_err(&w.ctr->err, ERR_UNSUPPORTED); return size; }
    const uint32_t pre = ref == REF_STRING ? b1 - b0 : len;
    if (WRITE) { p = wr_vu(out, p, pre); for (uint32_t i = b0; i < b1; ++i) out[p++] = w.bytes[i]; }
    size += vu_size(pre) + (b1 - b0);
  } else {
    const uint32_t n = w.s_cend[src] - w.s_cpos[src];
    if (WRITE) for (uint32_t i = 0; i < n; ++i) out[p++] = w.bytes[w.s_cpos[src] + i];
    size += n;
  }
  return size;
}

// block b (client rank for merge, section for diff): its client id
__device__ __forceinline__ uint32_t blk_client(const Work& w, uint32_t b) {
  if (w.lz_bclient) return w.lz_bclient[b];  // the serial merge's output sections
  return w.lz_diff ? w.sections[b].client : w.cl_vals[w.lz_nblk - 1 - b];
}
// diffUpdate over non-canonical input (k_ds_bound's flag): LazyStructWriter appends a struct to
// the section it is writing when the client is the same (Y@38735), so a non-empty block continues
// the previous non-empty block of its update when both have the same client (a run of one client
// the reader left and came back to, with nothing written in between). Canonical input has distinct
// clients per update: every non-empty block starts a section.
__device__ __forceinline__ bool blk_same_upd(const Work& w, uint32_t a, uint32_t b) {
  return !w.lz_multi || w.sections[a].upd == w.sections[b].upd;
}
__device__ bool blk_continues(const Work& w, uint32_t b) {
  if (!w.lz_diff || !w.ctr->noncanon) return false;
  const uint32_t c = blk_client(w, b);
  for (uint32_t k = b; k-- > 0;) {
    if (!blk_same_upd(w, k, b)) return false;
    if (w.lz_evn[k]) return blk_client(w, k) == c;
  }
  return false;
}
__device__ uint32_t blk_section_n(const Work& w, uint32_t b) {  // structs of the section block b heads
  uint32_t n = w.lz_evn[b];
  if (!w.lz_diff || !w.ctr->noncanon) return n;
  const uint32_t c = blk_client(w, b);
  for (uint32_t k = b + 1; k < w.lz_nblk && blk_same_upd(w, b, k); ++k) {
    const uint32_t e = w.lz_evn[k];
    if (!e) continue;
    if (blk_client(w, k) != c) break;
    n += e;
  }
  return n;
}
// event slots [evbase[b], evbase[b] + cap[b]); slots past evn[b] are empty
__global__ __launch_bounds__(256) void k_ev_sizes(Work w, uint32_t nslots) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e > nslots) return;
  if (e == nslots) { w.ev_size[e] = 0; return; }
  const uint32_t b = upper_bound_u32(w.lz_evbase, w.lz_nblk, e) - 1;
  w.ev_size[e] = (e - w.lz_evbase[b] < w.lz_evn[b]) ? encode_event<false>(w, blk_client(w, b), e, nullptr, 0) : 0u;
}
__global__ void k_blk_sizes(Work w, uint32_t nblk) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b > nblk) return;
  if (b == nblk) { w.blk_size[b] = 0; return; }
  const uint32_t n = w.lz_evn[b];
  uint32_t sz = 0;
  bool head = false;
  if (n) {
    const uint32_t e0 = w.lz_evbase[b];
    head = !blk_continues(w, b);
    sz = w.ev_pos[e0 + n] - w.ev_pos[e0];
    if (head) sz += vu_size(blk_section_n(w, b)) + vu_size(blk_client(w, b)) + vu_size(w.ev_clock[e0]);
  }
  w.blk_size[b] = sz;
  wave_count_add(&w.ctr->pad[0], head);
}
__global__ __launch_bounds__(256) void k_ev_write(Work w, uint32_t nslots) {
  const uint32_t e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nslots) return;
  const uint32_t b = upper_bound_u32(w.lz_evbase, w.lz_nblk, e) - 1;
  const uint32_t e0 = w.lz_evbase[b], n = w.lz_evn[b];
  if (e - e0 >= n) return;
  const uint32_t client = blk_client(w, b);
  const uint32_t hdr = blk_continues(w, b) ? 0u : vu_size(blk_section_n(w, b)) + vu_size(client) + vu_size(w.ev_clock[e0]);
  const uint32_t hoff = w.lz_multi ? 0u : vu_size(w.ctr->pad[0]);  // lz_multi: the host writes per-update headers
  const uint32_t p = hoff + w.blk_pos[b] + hdr + (w.ev_pos[e] - w.ev_pos[e0]);
  encode_event<true>(w, client, e, w.out, p);
}
__global__ void k_blk_write(Work w, uint32_t nblk) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b == 0 && !w.lz_multi) wr_vu(w.out, 0u, w.ctr->pad[0]);
  if (b >= nblk) return;
  const uint32_t n = w.lz_evn[b];
  if (!n || blk_continues(w, b)) return;
  uint32_t p = (w.lz_multi ? 0u : vu_size(w.ctr->pad[0])) + w.blk_pos[b];
  p = wr_vu(w.out, p, blk_section_n(w, b));
  p = wr_vu(w.out, p, blk_client(w, b));
  wr_vu(w.out, p, w.ev_clock[w.lz_evbase[b]]);
}

// ---------------------------------------------------------------- delete sets
// merge: sort (client desc, clock asc), running max of range ends per client, runs
__global__ void k_dsm_keys(Work w, uint32_t nds) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nds) return;
  const DsRange d = w.ds[i];
  w.dsm_key[i] = ((uint64_t)(w.ds_first ? w.ds_fa[i] : ~d.client) << 32) | d.clock;
  w.dsm_len[i] = d.len;
}
__global__ void k_dsm_ends(Work w, uint32_t nds) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nds) return;
  const uint64_t k = w.dsm_keys[i];
  w.dsm_end[i] = (k & 0xFFFFFFFF00000000ull) | (uint64_t)((uint32_t)k + w.dsm_lens[i]);
}
// run starts (sortAndMergeDeleteSet: merge while s.clock + s.len >= r.clock)
__global__ void k_dsm_flags(Work w, uint32_t nds) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > nds) return;
  if (i == nds) { w.dsm_flag[i] = 0; return; }
  const uint64_t k = w.dsm_keys[i];
  bool st = i == 0 || (w.dsm_keys[i - 1] >> 32) != (k >> 32) || (uint32_t)w.dsm_max[i - 1] < (uint32_t)k;
  w.dsm_flag[i] = st ? 1u : 0u;
}
__global__ void k_dsm_runs(Work w, uint32_t nds) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nds) return;
  const uint32_t rid = w.dsm_rid[i] + w.dsm_flag[i] - 1;  // inclusive count of run starts - 1
  const uint64_t k = w.dsm_keys[i];
  if (w.dsm_flag[i]) {
    w.dr_client[rid] = w.ds_first ? w.ds[(uint32_t)(k >> 32)].client : ~(uint32_t)(k >> 32);
    w.dr_clock[rid] = (uint32_t)k;
  }
  if (i + 1 == nds || w.dsm_flag[i + 1]) w.dr_end[rid] = (uint32_t)w.dsm_max[i];
}
// diff: the input's ranges unmerged, clients in descending order (13.6 canonical), wire order
// within a client
__global__ void k_dsd_keys(Work w, uint32_t nds) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nds) return;
  // lz_multi: (update, client desc); the radix sort is stable, so wire order survives within a client.
  // compat 135: first-appearance client order (the range's first-range index; per update for multi)
  const DsRange d = w.ds[i];
  if (w.ds_first)
    w.dsm_key[i] = w.lz_multi ? ((uint64_t)d.upd << 32 | (w.ds_fa[i] - w.ds_dense_off[d.upd])) : ((uint64_t)w.ds_fa[i] << 32) | i;
  else
    w.dsm_key[i] = w.lz_multi ? ((uint64_t)d.upd << 32 | (uint32_t)~d.client) : ((uint64_t)(~d.client) << 32) | i;
  w.dsm_len[i] = i;
}
__global__ void k_dsd_runs(Work w, uint32_t nds) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nds) return;
  const DsRange d = w.ds[w.dsm_lens[i]];
  w.dr_client[i] = d.client;
  w.dr_clock[i] = d.clock;
  w.dr_end[i] = d.clock + d.len;
}

// first appearance of every range's client (compat 135): stable sort by (scope, client), then each
// range takes the smallest original index of its group (the group head, by a running max of heads)
__global__ void k_fa_keys(Work w, uint32_t nds) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nds) return;
  const DsRange d = w.ds[i];
  w.dsm_key[i] = w.lz_multi ? ((uint64_t)d.upd << 32 | d.client) : (uint64_t)d.client;
  w.dsm_len[i] = i;
}
__global__ void k_fa_heads(Work w, uint32_t nds) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nds) return;
  w.dsm_end[p] = (p == 0 || w.dsm_keys[p] != w.dsm_keys[p - 1]) ? p : 0;
}
__global__ void k_fa_set(Work w, uint32_t nds) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= nds) return;
  w.ds_fa[w.dsm_lens[p]] = w.dsm_lens[(uint32_t)w.dsm_max[p]];
}

// writeDeleteSet (Y@11105 `fe`): runs grouped by client in output order
__global__ void k_dw_flags(Work w, uint32_t nr) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > nr) return;
  const bool brk = i > 0 && i < nr && w.lz_multi && (w.dsm_keys[i] >> 32) != (w.dsm_keys[i - 1] >> 32);  // next update
  w.dw_flag[i] = (i < nr && (i == 0 || brk || w.dr_client[i] != w.dr_client[i - 1])) ? 1u : 0u;
}
__global__ void k_dw_gstart(Work w, uint32_t nr) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nr) return;
  if (w.dw_flag[i]) w.dw_gstart[w.dw_gid[i]] = i;
  if (i == nr - 1) w.dw_gstart[w.dw_gid[nr]] = nr;
}
__global__ void k_dw_sizes(Work w, uint32_t nr) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > nr) return;
  if (i == nr) { w.dw_size[i] = 0; return; }
  const uint32_t clock = w.dr_clock[i], len = w.dr_end[i] - clock;
  uint32_t sz = vu_size(clock) + vu_size(len);
  if (w.dw_flag[i]) {
    const uint32_t g = w.dw_gid[i];
    sz += vu_size(w.dr_client[i]) + vu_size(w.dw_gstart[g + 1] - w.dw_gstart[g]);
  }
  w.dw_size[i] = sz;
}
__global__ void k_dw_write(Work w, uint32_t nr, uint32_t dsbase) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t ng = w.dw_gid[nr];
  if (i == 0 && !w.lz_multi) wr_vu(w.out, dsbase, ng);
  if (i >= nr) return;
  uint32_t p = dsbase + (w.lz_multi ? 0u : vu_size(ng)) + w.dw_pos[i];
  if (w.dw_flag[i]) {
    const uint32_t g = w.dw_gid[i];
    p = wr_vu(w.out, p, w.dr_client[i]);
    p = wr_vu(w.out, p, w.dw_gstart[g + 1] - w.dw_gstart[g]);
  }
  const uint32_t clock = w.dr_clock[i];
  p = wr_vu(w.out, p, clock);
  wr_vu(w.out, p, w.dr_end[i] - clock);
}

// ---------------------------------------------------------------- host side
static inline uint32_t G(uint64_t n) { return (uint32_t)(n / 256 + 1); }

// Reader order + per-client merge (mergeUpdates) → events
void launch_lazy_merge(Work& w, uint32_t nsections, uint32_t nclients, hipStream_t s) {
  w.lz_diff = 0;
  w.lz_nblk = nclients;
  hipLaunchKernelGGL(k_lz_keys, dim3(G(nsections)), dim3(256), 0, s, w, nsections, nclients);
  sort_pairs_u64_u32(w.tmp, w.tmp_bytes, w.lz_key, w.lz_keys, w.lz_iota, w.lz_sec, nsections, s);
  hipLaunchKernelGGL(k_lz_runs, dim3(G(nsections)), dim3(256), 0, s, w, nsections, nclients);
  hipLaunchKernelGGL(k_lz_prev, dim3(G(w.nupd)), dim3(256), 0, s, w, w.nupd);
  hipLaunchKernelGGL(k_lz_cap, dim3(G(nclients + 1)), dim3(256), 0, s, w, nclients);
  scan_u32(w.tmp, w.tmp_bytes, w.lz_cap, w.lz_evbase, nclients + 1, s);
  hipMemsetAsync(w.lz_flag, 0, sizeof(uint32_t) * (nsections + 1), s);
  OrderedIds o;
  if (!ordered_ids(nclients, s, o)) { hipMemsetAsync(&w.ctr->err, ERR_CAPACITY, 1, s); return; }
  hipLaunchKernelGGL(k_lz_merge, dim3(nclients), dim3(64), 0, s, w, nclients, o.ctr, o.base);
}
// non-canonical input (k_lz_canon): the serial loop; the block count comes back in ctr->lz_blocks
void launch_lazy_merge_seq(Work& w, uint32_t cap_ev, uint32_t cap_blk, hipStream_t s) {
  w.lz_diff = 0;
  hipLaunchKernelGGL(k_lz_merge_seq, dim3(1), dim3(64), 0, s, w, w.nupd, cap_ev, cap_blk);
}


// diffUpdate: one block per section of the single input update
void launch_lazy_diff(Work& w, uint32_t nsections, hipStream_t s) {
  w.lz_diff = 1;
  w.lz_nblk = nsections;
  hipLaunchKernelGGL(k_lz_diff_cap, dim3(G(nsections + 1)), dim3(256), 0, s, w, nsections);
  scan_u32(w.tmp, w.tmp_bytes, w.lz_cap, w.lz_evbase, nsections + 1, s);
  hipLaunchKernelGGL(k_lz_diff, dim3(G(nsections)), dim3(256), 0, s, w, nsections);
}

// events → struct-section sizes (returns total via counters: pad[0] = non-empty blocks)
uint32_t launch_event_sizes(Work& w, hipStream_t s, uint32_t* nslots_out) {
  uint32_t nslots = 0;
  hipMemcpyAsync(&nslots, w.lz_evbase + w.lz_nblk, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
  hipStreamSynchronize(s);
  *nslots_out = nslots;
  hipMemsetAsync(w.ctr->pad, 0, sizeof(uint32_t) * 8, s);
  hipLaunchKernelGGL(k_ev_sizes, dim3(G(nslots + 1)), dim3(256), 0, s, w, nslots);
  scan_u32(w.tmp, w.tmp_bytes, w.ev_size, w.ev_pos, nslots + 1, s);
  hipLaunchKernelGGL(k_blk_sizes, dim3(G(w.lz_nblk + 1)), dim3(256), 0, s, w, w.lz_nblk);
  scan_u32(w.tmp, w.tmp_bytes, w.blk_size, w.blk_pos, w.lz_nblk + 1, s);
  return nslots;
}

// delete-set runs: merge (union of all inputs) or diff (the input's own)
uint32_t launch_ds_runs(Work& w, uint32_t nds, bool merge, hipStream_t s) {
  if (!nds) return 0;
  if (w.ds_first) {
    hipLaunchKernelGGL(k_fa_keys, dim3(G(nds)), dim3(256), 0, s, w, nds);
    sort_pairs_u64_u32(w.tmp, w.tmp_bytes, w.dsm_key, w.dsm_keys, w.dsm_len, w.dsm_lens, nds, s);
    hipLaunchKernelGGL(k_fa_heads, dim3(G(nds)), dim3(256), 0, s, w, nds);
    scan_segmax_u64(w.tmp, w.tmp_bytes, w.dsm_end, w.dsm_max, nds, s);  // high words 0: a plain running max
    hipLaunchKernelGGL(k_fa_set, dim3(G(nds)), dim3(256), 0, s, w, nds);
  }
  if (!merge) {
    hipLaunchKernelGGL(k_dsd_keys, dim3(G(nds)), dim3(256), 0, s, w, nds);
    sort_pairs_u64_u32(w.tmp, w.tmp_bytes, w.dsm_key, w.dsm_keys, w.dsm_len, w.dsm_lens, nds, s);
    hipLaunchKernelGGL(k_dsd_runs, dim3(G(nds)), dim3(256), 0, s, w, nds);
    return nds;
  }
  hipLaunchKernelGGL(k_dsm_keys, dim3(G(nds)), dim3(256), 0, s, w, nds);
  sort_pairs_u64_u32(w.tmp, w.tmp_bytes, w.dsm_key, w.dsm_keys, w.dsm_len, w.dsm_lens, nds, s);
  hipLaunchKernelGGL(k_dsm_ends, dim3(G(nds)), dim3(256), 0, s, w, nds);
  scan_segmax_u64(w.tmp, w.tmp_bytes, w.dsm_end, w.dsm_max, nds, s);
  hipLaunchKernelGGL(k_dsm_flags, dim3(G(nds + 1)), dim3(256), 0, s, w, nds);
  scan_u32(w.tmp, w.tmp_bytes, w.dsm_flag, w.dsm_rid, nds + 1, s);
  hipLaunchKernelGGL(k_dsm_runs, dim3(G(nds)), dim3(256), 0, s, w, nds);
  uint32_t nr = 0;
  hipMemcpyAsync(&nr, w.dsm_rid + nds, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
  hipStreamSynchronize(s);
  return nr;
}

// delete-set sizes (returns the encoded DS byte count)
uint32_t launch_ds_write_sizes(Work& w, uint32_t nr, hipStream_t s) {
  if (!nr) return 1;  // varuint 0
  hipLaunchKernelGGL(k_dw_flags, dim3(G(nr + 1)), dim3(256), 0, s, w, nr);
  scan_u32(w.tmp, w.tmp_bytes, w.dw_flag, w.dw_gid, nr + 1, s);
  hipLaunchKernelGGL(k_dw_gstart, dim3(G(nr)), dim3(256), 0, s, w, nr);
  hipLaunchKernelGGL(k_dw_sizes, dim3(G(nr + 1)), dim3(256), 0, s, w, nr);
  scan_u32(w.tmp, w.tmp_bytes, w.dw_size, w.dw_pos, nr + 1, s);
  uint32_t v[2] = {0, 0};
  hipMemcpyAsync(&v[0], w.dw_gid + nr, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
  hipMemcpyAsync(&v[1], w.dw_pos + nr, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
  hipStreamSynchronize(s);
  return vu_size_host(v[0]) + v[1];
}

void launch_lazy_write(Work& w, uint32_t nslots, uint32_t nr, uint32_t dsbase, hipStream_t s) {
  hipLaunchKernelGGL(k_blk_write, dim3(G(w.lz_nblk)), dim3(256), 0, s, w, w.lz_nblk);
  if (nslots) hipLaunchKernelGGL(k_ev_write, dim3(G(nslots)), dim3(256), 0, s, w, nslots);
  if (nr) hipLaunchKernelGGL(k_dw_write, dim3(G(nr)), dim3(256), 0, s, w, nr, dsbase);
  else {
    const uint8_t zero = 0;
    hipMemcpyAsync(w.out + dsbase, &zero, 1, hipMemcpyHostToDevice, s);
    hipStreamSynchronize(s);
  }
}

}  // namespace yc
