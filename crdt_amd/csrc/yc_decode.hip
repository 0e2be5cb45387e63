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
#include "yc_work.h"

namespace yc {

// --------------------------------------------------------------------------- 1. group parse
__global__ __launch_bounds__(256) void k_group_parse(const uint8_t* __restrict__ b, const Group* __restrict__ groups,
                                                     uint64_t* __restrict__ main_bits, uint16_t* __restrict__ gpre,
                                                     uint32_t* __restrict__ gexit) {
  __shared__ uint64_t sbits[GROUP_LANES];
  __shared__ uint32_t sexit[GROUP_LANES];
  __shared__ uint8_t strunc[GROUP_LANES];
  __shared__ uint32_t scnt[GROUP_LANES + 1];
  const Group G = groups[blockIdx.x];
  const uint32_t lane = threadIdx.x;
  const uint32_t nchunks = (G.end - G.start + CHUNK - 1) / CHUNK;
  const uint32_t cs = G.start + lane * CHUNK;
  uint64_t bits = 0;
  uint32_t pos = cs;
  uint8_t trunc = 0;
  if (lane < nchunks) {
    const uint32_t ce = min(cs + CHUNK, G.end);
    while (pos < ce) {
      // every position the chain visits is marked (also one that fails to parse: it may be the
      // first byte after a section, which the walker needs to find as "the r-th position")
      bits |= 1ull << (pos - cs);
      uint32_t q = pos;
      int r = parse_struct<false>(b, q, G.uend, SPEC_MAX_STEPS, nullptr);
      if (r > 0) pos = q;
      else if (r == 0) ++pos;          // not a struct start: restart one byte later
      else { trunc = 1; break; }       // long struct: leave it to the exact stitcher
    }
  }
  sbits[lane] = bits;
  sexit[lane] = pos;
  strunc[lane] = trunc;
  __syncthreads();
  if (lane == 0) {
    // stitch: one deterministic chain from the group start (exact where the lanes gave up)
    uint32_t p = G.start;
    for (uint32_t c = 0; c < nchunks; ++c) {
      const uint32_t ccs = G.start + c * CHUNK;
      const uint32_t cce = min(ccs + CHUNK, G.end);
      const uint64_t cb = sbits[c];
      uint64_t m = 0;
      while (p < cce) {
        const uint32_t off = p - ccs;
        if ((cb >> off) & 1ull) {  // on chunk c's chain: adopt it
          m |= cb & (~0ull << off);
          p = sexit[c];
          if (strunc[c]) {         // exact parse of the struct the lane skipped (already marked)
            uint32_t q = p;
            if (parse_struct<false>(b, q, G.uend, 0xFFFFFFFFu, nullptr) > 0) p = q;
            else ++p;
          }
          continue;
        }
        m |= 1ull << off;
        uint32_t q = p;
        if (parse_struct<false>(b, q, G.uend, 0xFFFFFFFFu, nullptr) > 0) p = q;
        else ++p;
      }
      sbits[c] = m;
    }
    gexit[blockIdx.x] = p;
  }
  __syncthreads();
  uint32_t cnt = 0;
  if (lane < nchunks) {
    main_bits[(G.start >> 6) + lane] = sbits[lane];
    cnt = (uint32_t)__popcll(sbits[lane]);
  }
  scnt[lane] = cnt;
  __syncthreads();
  // inclusive Hillis-Steele scan over 256 counts
  for (uint32_t off = 1; off < GROUP_LANES; off <<= 1) {
    uint32_t v = lane >= off ? scnt[lane - off] : 0;
    __syncthreads();
    scnt[lane] += v;
    __syncthreads();
  }
  uint16_t* pre = gpre + (size_t)blockIdx.x * (GROUP_LANES + 1);
  pre[lane + 1] = (uint16_t)scnt[lane];
  if (lane == 0) pre[0] = 0;
}

void launch_group_parse(const Work& w, hipStream_t s) {
  if (w.ngroups == 0) return;
  hipLaunchKernelGGL(k_group_parse, dim3(w.ngroups), dim3(GROUP_LANES), 0, s, w.bytes, w.groups, w.main_bits, w.gpre,
                     w.gexit);
}

// --------------------------------------------------------------------------- 2. walker
__device__ __forceinline__ uint32_t select_bit(uint64_t x, uint32_t n) {  // position of the n-th set bit
  for (uint32_t i = 0; i < n; ++i) x &= x - 1;
  return (uint32_t)__ffsll((long long)x) - 1;
}

__global__ __launch_bounds__(64) void k_walker(Work w) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= w.nupd) return;
  const uint8_t* __restrict__ b = w.bytes;
  const uint32_t ustart = w.uoff[u];
  const uint32_t uend = ustart + w.ulen[u];
  uint32_t* err = &w.ctr->err;
  w.dsstart[u] = NONE;
  uint32_t p = ustart;
  bool ok = true;
  const uint32_t nsec = rd_vu(b, p, uend, ok);
  if (!ok || nsec > (uend - p) / 3 + 1) { raise_err(err, ERR_DECODE); return; }
  const uint32_t sbase = atomicAdd(&w.ctr->nsections, nsec);
  if (sbase + nsec > w.cap_sections) { raise_err(err, ERR_CAPACITY); return; }
  for (uint32_t s = 0; s < nsec; ++s) {
    const uint32_t n = rd_vu(b, p, uend, ok);
    const uint32_t client = rd_vu(b, p, uend, ok);
    const uint32_t clock = rd_vu(b, p, uend, ok);
    if (!ok || n > uend - p) { raise_err(err, ERR_DECODE); return; }
    Section sec;
    sec.upd = u; sec.n = n; sec.client = client; sec.clock = clock;
    sec.first_pos = n ? p : NONE; sec.cidx = NONE; sec.first_idx = NONE; sec.pad = 0;
    w.sections[sbase + s] = sec;
    if (n) atomicOr((unsigned long long*)&w.sec_bits[p >> 6], 1ull << (p & 63));
    uint32_t r = n;
    while (r > 0) {
      if (p >= uend) { raise_err(err, ERR_DECODE); return; }
      const uint32_t g = w.ugroup[u] + (p - ustart) / GROUP_BYTES;
      const uint64_t wb = w.main_bits[p >> 6];
      const uint32_t off = p & 63;
      if ((wb >> off) & 1ull) {
        const Group G = w.groups[g];
        const uint16_t* pre = w.gpre + (size_t)g * (GROUP_LANES + 1);
        const uint32_t c = (p - G.start) >> 6;
        const uint32_t below = pre[c] + (uint32_t)__popcll(wb & ((1ull << off) - 1));
        const uint32_t total = pre[GROUP_LANES];
        const uint32_t k = total - below;
        uint32_t pend;
        if (k < r) {
          pend = w.gexit[g];
          r -= k;
        } else {
          const uint32_t target = below + r;
          if (target == total) pend = w.gexit[g];
          else {
            uint32_t lo = 0, hi = GROUP_LANES;  // last chunk cc with pre[cc] <= target
            while (hi - lo > 1) { uint32_t mid = (lo + hi) >> 1; if (pre[mid] <= target) lo = mid; else hi = mid; }
            const uint64_t cw = w.main_bits[(G.start >> 6) + lo];
            pend = G.start + lo * CHUNK + select_bit(cw, target - pre[lo]);
          }
          r = 0;
        }
        const uint32_t ti = atomicAdd(&w.ctr->ncopy, 1u);
        if (ti >= w.cap_copy) { raise_err(err, ERR_CAPACITY); return; }
        w.copy[ti] = CopyTask{p, min(pend, G.end)};
        p = pend;
      } else {
        const uint32_t pi = atomicAdd(&w.ctr->npatch, 1u);
        if (pi >= w.cap_patch) { raise_err(err, ERR_CAPACITY); return; }
        w.patch[pi] = p;
        uint32_t q = p;
        if (parse_struct<false>(b, q, uend, 0xFFFFFFFFu, nullptr) <= 0) { raise_err(err, ERR_DECODE); w.ctr->err_info = p; return; }
        p = q;
        --r;
      }
    }
  }
  w.dsstart[u] = p;
}

void launch_walker(const Work& w, hipStream_t s) {
  if (w.nupd == 0) return;
  hipLaunchKernelGGL(k_walker, dim3((w.nupd + 63) / 64), dim3(64), 0, s, w);
}

// --------------------------------------------------------------------------- 3. final bitmap
__global__ __launch_bounds__(256) void k_copy(const CopyTask* __restrict__ tasks, const uint32_t* __restrict__ ntasks,
                                              const uint64_t* __restrict__ main_bits, uint64_t* __restrict__ final_bits) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t t = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (t >= *ntasks) return;
  const CopyTask T = tasks[t];
  if (T.a >= T.b) return;
  const uint32_t w0 = T.a >> 6, w1 = (T.b - 1) >> 6;
  for (uint32_t wi = w0 + lane; wi <= w1; wi += 64) {
    uint64_t m = ~0ull;
    if (wi == w0) m &= ~0ull << (T.a & 63);
    if (wi == w1 && (T.b & 63)) m &= (1ull << (T.b & 63)) - 1;
    const uint64_t v = main_bits[wi] & m;
    if (v) atomicOr((unsigned long long*)&final_bits[wi], (unsigned long long)v);
  }
}
__global__ void k_patch(const uint32_t* __restrict__ patch, const uint32_t* __restrict__ npatch, uint64_t* __restrict__ final_bits) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= *npatch) return;
  const uint32_t p = patch[i];
  atomicOr((unsigned long long*)&final_bits[p >> 6], 1ull << (p & 63));
}

void launch_build_final_bits(const Work& w, hipStream_t s) {
  // launch over the capacities; kernels read the real counts from device memory
  hipLaunchKernelGGL(k_copy, dim3((w.cap_copy + 3) / 4), dim3(256), 0, s, w.copy, &w.ctr->ncopy, w.main_bits, w.final_bits);
  hipLaunchKernelGGL(k_patch, dim3((w.cap_patch + 255) / 256), dim3(256), 0, s, w.patch, &w.ctr->npatch, w.final_bits);
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

void launch_struct_positions(const Work& w, hipStream_t s) {
  const uint32_t nwords = (w.nbytes + 63) / 64;
  hipLaunchKernelGGL(k_popc, dim3(nwords / 256 + 1), dim3(256), 0, s, w.final_bits, w.scratch, nwords);
  scan_u32(w.tmp, w.tmp_bytes, w.scratch, w.wcnt, nwords + 1, s);
  hipLaunchKernelGGL(k_scatter_pos, dim3(nwords / 256 + 1), dim3(256), 0, s, w.final_bits, w.wcnt, nwords, w.s_pos,
                     w.cap_structs, &w.ctr->err);
  hipLaunchKernelGGL(k_popc, dim3(nwords / 256 + 1), dim3(256), 0, s, w.sec_bits, w.scratch, nwords);
  scan_u32(w.tmp, w.tmp_bytes, w.scratch, w.wsec, nwords + 1, s);
}

// called once the section count is known on the host
void launch_section_clients(const Work& w, uint32_t nsections, hipStream_t s) {
  if (!nsections) return;
  hipLaunchKernelGGL(k_section_rank, dim3((nsections + 255) / 256), dim3(256), 0, s, w, nsections);
}

// --------------------------------------------------------------------------- 5. delete sets
__device__ __forceinline__ uint32_t nth_lane(uint64_t mask, uint32_t n) { return select_bit(mask, n); }

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
        uint32_t obase = 0;
        if (lane == 0 && lm) obase = atomicAdd(&w.ctr->nds, (uint32_t)__popcll(lm));
        obase = (uint32_t)__shfl((int)obase, 0);
        if (is_len) {
          const uint32_t idx = obase + (uint32_t)__popcll(lm & lt_mask);
          if (idx < w.cap_ds) {
            DsRange r;
            r.client = client;
            r.clock = myk == vi ? pend_clock : prevval;
            r.len = val;
            r.upd = u;
            w.ds[idx] = r;
          } else raise_err(err, ERR_CAPACITY);
        }
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
}

void launch_ds_decode(const Work& w, hipStream_t s) {
  if (w.nupd == 0) return;
  hipLaunchKernelGGL(k_ds_decode, dim3((w.nupd + 3) / 4), dim3(256), 0, s, w);
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
__global__ void k_section_cidx(Section* __restrict__ sec, uint32_t n, const uint32_t* __restrict__ cl, uint32_t nc) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) sec[i].cidx = lower_bound_u32(cl, nc, sec[i].client);
}

void launch_client_table(Work& w, uint32_t nsections, uint32_t* nclients_host, hipStream_t s) {
  const uint32_t grid = nsections / 256 + 1;
  hipLaunchKernelGGL(k_gather_sec_clients, dim3(grid), dim3(256), 0, s, w.sections, nsections, w.cl_tmp);
  sort_u32(w.tmp, w.tmp_bytes, w.cl_tmp, w.cl_vals, nsections, s);
  hipLaunchKernelGGL(k_unique_flags, dim3(grid), dim3(256), 0, s, w.cl_vals, nsections, w.scratch);
  scan_u32(w.tmp, w.tmp_bytes, w.scratch, w.cl_tmp, nsections + 1, s);
  // compact in place is unsafe; use cl_state as scratch output, then copy back
  hipLaunchKernelGGL(k_unique_scatter, dim3(grid), dim3(256), 0, s, w.cl_vals, w.cl_tmp, nsections, w.cl_state, &w.ctr->nclients);
  hipMemcpyAsync(w.cl_vals, w.cl_state, sizeof(uint32_t) * nsections, hipMemcpyDeviceToDevice, s);
  hipMemcpyAsync(nclients_host, &w.ctr->nclients, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
  hipStreamSynchronize(s);
  hipLaunchKernelGGL(k_section_cidx, dim3(grid), dim3(256), 0, s, w.sections, nsections, w.cl_vals, *nclients_host);
}

// --------------------------------------------------------------------------- 6. struct decode
__device__ __forceinline__ uint32_t find_cidx(const uint32_t* __restrict__ cl, uint32_t nc, uint32_t client) {
  const uint32_t i = lower_bound_u32(cl, nc, client);
  return (i < nc && cl[i] == client) ? i : NONE;
}

__global__ __launch_bounds__(256) void k_struct_decode(Work w, uint32_t nstructs, uint32_t nclients) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nstructs) return;
  uint32_t* err = &w.ctr->err;
  const uint32_t p0 = w.s_pos[i];
  const Section sec = w.sections[w.s_sec[i]];
  const uint32_t uend = w.uoff[sec.upd] + w.ulen[sec.upd];
  StructView v;
  uint32_t p = p0;
  if (parse_struct<true>(w.bytes, p, uend, 0xFFFFFFFFu, &v) <= 0) { raise_err(err, ERR_DECODE); return; }
  w.s_len[i] = v.len;
  w.s_info[i] = v.info;
  w.s_cidx[i] = sec.cidx;
  uint32_t oc = NONE, rc = NONE;
  const bool item = v.ref != REF_GC && v.ref != REF_SKIP;
  if (item && (v.info & 0x80u)) {
    oc = find_cidx(w.cl_vals, nclients, v.oc);
    if (oc == NONE) { raise_err(err, ERR_PENDING); w.ctr->err_info = i; }
  }
  if (item && (v.info & 0x40u)) {
    rc = find_cidx(w.cl_vals, nclients, v.rc);
    if (rc == NONE) { raise_err(err, ERR_PENDING); w.ctr->err_info = i; }
  }
  w.s_ocidx[i] = oc;
  w.s_oclock[i] = v.ok_;
  w.s_rcidx[i] = rc;
  w.s_rclock[i] = v.rk;
  w.s_pa[i] = (item && v.pkind == 1) ? v.pa : NONE;
  w.s_pb[i] = v.pb;
  w.s_psub[i] = (item && v.has_psub) ? v.psub_pos : NONE;
  w.s_psublen[i] = v.psub_len;
  w.s_cpos[i] = v.cpos;
  w.s_cend[i] = v.cend;
  uint32_t celem = v.cpos;
  if (v.ref == REF_ANY || v.ref == REF_JSON) celem += vu_size(v.nel);
  w.s_celem[i] = celem;
  // coverage of the engine (round 1): root-level YMap entries
  if (v.ref == REF_GC || v.ref == REF_STRING || v.ref == REF_EMBED || v.ref == REF_FORMAT || v.ref == REF_TYPE)
    raise_err(err, ERR_UNSUPPORTED);
  if (item && ((v.info & 0x40u) || v.pkind == 2)) raise_err(err, ERR_UNSUPPORTED);
  if (item && v.pkind == 1 && !v.has_psub) raise_err(err, ERR_UNSUPPORTED);  // root YArray item
  if (v.ref == REF_ANY && v.len > 1) raise_err(err, ERR_UNSUPPORTED);          // live map items are single values
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

void launch_struct_decode(const Work& w, uint32_t nstructs, uint32_t nsections, uint32_t nclients, hipStream_t s) {
  if (!nstructs) return;
  hipLaunchKernelGGL(k_struct_sec, dim3((nstructs + 255) / 256), dim3(256), 0, s, w, nstructs);
  hipLaunchKernelGGL(k_struct_decode, dim3((nstructs + 255) / 256), dim3(256), 0, s, w, nstructs, nclients);
  scan_u32_to_u64(w.tmp, w.tmp_bytes, w.s_len, w.s_lenscan, nstructs + 1, s);
  hipLaunchKernelGGL(k_struct_clock, dim3((nstructs + 255) / 256), dim3(256), 0, s, w, nstructs);
}

// --------------------------------------------------------------------------- client states
__global__ void k_states(Work w, uint32_t nstructs) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t items = 0;
  if (i < nstructs && (w.s_info[i] & 31u) != REF_SKIP) {
    atomicMax(&w.cl_state[w.s_cidx[i]], w.s_clock[i] + w.s_len[i]);
    items = w.s_len[i];
  }
  // wave-level sum, one 64-bit atomic per wave
  for (int off = 32; off > 0; off >>= 1) items += (uint32_t)__shfl_down((int)items, off);
  if ((threadIdx.x & 63) == 0 && items) atomicAdd(&w.ctr->items, (unsigned long long)items);
}
void launch_states(const Work& w, uint32_t nstructs, uint32_t nclients, hipStream_t s) {
  hipMemsetAsync(w.cl_state, 0, sizeof(uint32_t) * (nclients + 1), s);
  if (nstructs) hipLaunchKernelGGL(k_states, dim3((nstructs + 255) / 256), dim3(256), 0, s, w, nstructs);
  scan_u32_to_u64(w.tmp, w.tmp_bytes, w.cl_state, w.cl_base, nclients + 1, s);
}

}  // namespace yc
