// yc_prims.hip — device-wide scan / sort primitives (rocPRIM) used between the engine's kernels.
#include <algorithm>
#include <cstring>
#include <cstdlib>
#include <rocprim/rocprim.hpp>
#include "yc_work.h"

namespace yc {

struct SegMax64 {  // max of packed (segment << 32 | value) within a segment; a new segment restarts
  __host__ __device__ uint64_t operator()(uint64_t a, uint64_t b) const {
    return (a >> 32) == (b >> 32) ? (a > b ? a : b) : b;
  }
};

// several u32 fills in one launch (blockIdx.y = fill): each hipMemsetAsync is its own ~4.5 us
// dispatch, and a merge issues a dozen of them
__global__ void k_fill_multi(FillBatch b) {
  const FillDesc d = b.d[blockIdx.y];
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < d.n; i += (uint64_t)gridDim.x * blockDim.x)
    d.p[i] = d.v;
}

void fill_u32_multi(std::initializer_list<FillDesc> fills, hipStream_t s) {
  FillBatch b{};
  uint64_t nmax = 0;
  for (const FillDesc& f : fills) {
    if (!f.n) continue;
    if (b.count == FILL_MAX) {  // more than one batch: flush
      hipLaunchKernelGGL(k_fill_multi, dim3((uint32_t)std::min<uint64_t>(nmax / 256 + 1, 2048), b.count), dim3(256), 0, s, b);
      b.count = 0;
      nmax = 0;
    }
    b.d[b.count++] = f;
    nmax = std::max(nmax, f.n);
  }
  if (b.count)
    hipLaunchKernelGGL(k_fill_multi, dim3((uint32_t)std::min<uint64_t>(nmax / 256 + 1, 2048), b.count), dim3(256), 0, s, b);
}

size_t prim_tmp_bytes(uint64_t n) {
  size_t a = 0, b = 0, c = 0;
  rocprim::exclusive_scan(nullptr, a, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)n, rocprim::plus<uint32_t>());
  rocprim::exclusive_scan(nullptr, b, (const uint32_t*)nullptr, (uint64_t*)nullptr, (uint64_t)0, (size_t)n, rocprim::plus<uint64_t>());
  rocprim::radix_sort_keys(nullptr, c, (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)n, 0, 32);
  size_t d = 0;
  rocprim::radix_sort_pairs(nullptr, d, (const uint32_t*)nullptr, (uint32_t*)nullptr, (const uint32_t*)nullptr,
                            (uint32_t*)nullptr, (size_t)n, 0, 32);
  size_t e = 0, f = 0;
  rocprim::radix_sort_pairs(nullptr, e, (const uint64_t*)nullptr, (uint64_t*)nullptr, (const uint32_t*)nullptr,
                            (uint32_t*)nullptr, (size_t)n, 0, 64);
  rocprim::inclusive_scan(nullptr, f, (const uint64_t*)nullptr, (uint64_t*)nullptr, (size_t)n, SegMax64());
  size_t m = a > b ? a : b;
  m = m > c ? m : c;
  m = m > d ? m : d;
  m = m > e ? m : e;
  return (m > f ? m : f) + 256;
}

// A small exclusive scan in one workgroup and one launch (rocPRIM's look-back scan is two: state
// init + scan). Small merges (the per-op path: a doc state and an update) are launch-bound, and a
// merge runs a dozen scans. Each lane sums a contiguous run, the 1 024 run sums are scanned in LDS,
// each lane writes its run's prefixes; a lane reads in[i] before it writes out[i] and runs are
// disjoint, so in == out is safe. Same results as rocprim::exclusive_scan (wrapping plus).
constexpr uint32_t SMALL_SCAN_LANES = 1024, SMALL_SCAN_MAX = SMALL_SCAN_LANES * 16;
template <class T>
__global__ __launch_bounds__(SMALL_SCAN_LANES) void k_scan_small(const uint32_t* in, T* out, uint32_t n) {
  __shared__ T part[SMALL_SCAN_LANES];
  const uint32_t t = threadIdx.x, per = (n + SMALL_SCAN_LANES - 1) / SMALL_SCAN_LANES;
  const uint32_t a = min(n, t * per), b = min(n, a + per);
  T sum = 0;
  for (uint32_t i = a; i < b; ++i) sum += (T)in[i];
  part[t] = sum;
  __syncthreads();
  for (uint32_t off = 1; off < SMALL_SCAN_LANES; off <<= 1) {
    const T v = t >= off ? part[t - off] : (T)0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  T run = part[t] - sum;
  for (uint32_t i = a; i < b; ++i) {
    const T x = (T)in[i];
    out[i] = run;
    run += x;
  }
}

void scan_u32(void* tmp, size_t tmpb, const uint32_t* in, uint32_t* out, uint64_t n, hipStream_t s) {
  if (!n) return;
  if (n <= SMALL_SCAN_MAX) {
    hipLaunchKernelGGL(k_scan_small<uint32_t>, dim3(1), dim3(SMALL_SCAN_LANES), 0, s, in, out, (uint32_t)n);
    return;
  }
  rocprim::exclusive_scan(tmp, tmpb, in, out, 0u, (size_t)n, rocprim::plus<uint32_t>(), s);
}

void scan_u32_to_u64(void* tmp, size_t tmpb, const uint32_t* in, uint64_t* out, uint64_t n, hipStream_t s) {
  if (!n) return;
  if (n <= SMALL_SCAN_MAX) {
    hipLaunchKernelGGL(k_scan_small<uint64_t>, dim3(1), dim3(SMALL_SCAN_LANES), 0, s, in, out, (uint32_t)n);
    return;
  }
  rocprim::exclusive_scan(tmp, tmpb, in, out, (uint64_t)0, (size_t)n, rocprim::plus<uint64_t>(), s);
}

void sort_u32(void* tmp, size_t tmpb, const uint32_t* in, uint32_t* out, uint64_t n, hipStream_t s) {
  if (!n) return;
  rocprim::radix_sort_keys(tmp, tmpb, in, out, (size_t)n, 0, 32, s);
}

void sort_pairs_u32(void* tmp, size_t tmpb, const uint32_t* kin, uint32_t* kout, const uint32_t* vin, uint32_t* vout,
                    uint64_t n, hipStream_t s) {
  if (!n) return;
  rocprim::radix_sort_pairs(tmp, tmpb, kin, kout, vin, vout, (size_t)n, 0, 32, s);
}

void sort_pairs_u64_u32(void* tmp, size_t tmpb, const uint64_t* kin, uint64_t* kout, const uint32_t* vin, uint32_t* vout,
                        uint64_t n, hipStream_t s) {
  if (!n) return;
  rocprim::radix_sort_pairs(tmp, tmpb, kin, kout, vin, vout, (size_t)n, 0, 64, s);
}

void scan_segmax_u64(void* tmp, size_t tmpb, const uint64_t* in, uint64_t* out, uint64_t n, hipStream_t s) {
  if (!n) return;
  rocprim::inclusive_scan(tmp, tmpb, in, out, (size_t)n, SegMax64(), s);
}

// Byte pieces (device -> device, or a few inline bytes) in one launch: one wavefront per piece.
// Doc states are gathered into a multi-document batch and a multi-document result is split back
// into the documents' arena blocks this way (ycrdt_apply_updates_multi), instead of one
// hipMemcpyAsync per document.
__global__ __launch_bounds__(256) void k_copy_pieces(const Piece* __restrict__ pieces, uint32_t n) {
  const uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  if (i >= n) return;
  const Piece P = pieces[i];
  if (!P.src) {
    if (lane < P.len) P.dst[lane] = P.inl[lane];
    return;
  }
  for (uint32_t k = lane; k < P.len; k += 64) P.dst[k] = P.src[k];
}
void copy_pieces(const Piece* pieces, uint32_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_copy_pieces, dim3((n + 3) / 4), dim3(256), 0, s, pieces, n);
}

}  // namespace yc
