// yc_prims.hip — device-wide scan / sort primitives (rocPRIM) used between the engine's kernels.
#include <algorithm>
#include <cstring>
#include <cstdlib>
#include <mutex>
#include <unordered_map>
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

// rocPRIM scratch for scans of up to scan_n items and radix sorts of up to sort_n items. The two
// are sized apart: a sort needs double buffers of its keys and values (12 B per item for the
// 64-bit keys), a scan only its tile states — sized together from the batch bytes, a 15 GB batch
// asked for 187 GB of scratch.
size_t prim_tmp_bytes(uint64_t scan_n, uint64_t sort_n) {
  size_t a = 0, b = 0, f = 0;
  rocprim::exclusive_scan(nullptr, a, (const uint32_t*)nullptr, (uint32_t*)nullptr, 0u, (size_t)scan_n, rocprim::plus<uint32_t>());
  rocprim::exclusive_scan(nullptr, b, (const uint32_t*)nullptr, (uint64_t*)nullptr, (uint64_t)0, (size_t)scan_n, rocprim::plus<uint64_t>());
  rocprim::inclusive_scan(nullptr, f, (const uint64_t*)nullptr, (uint64_t*)nullptr, (size_t)scan_n, SegMax64());
  size_t m = std::max({a, b, f});
  if (sort_n) {
    size_t c = 0, d = 0, e = 0;
    rocprim::radix_sort_keys(nullptr, c, (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)sort_n, 0, 32);
    rocprim::radix_sort_pairs(nullptr, d, (const uint32_t*)nullptr, (uint32_t*)nullptr, (const uint32_t*)nullptr,
                              (uint32_t*)nullptr, (size_t)sort_n, 0, 32);
    rocprim::radix_sort_pairs(nullptr, e, (const uint64_t*)nullptr, (uint64_t*)nullptr, (const uint32_t*)nullptr,
                              (uint32_t*)nullptr, (size_t)sort_n, 0, 64);
    m = std::max({m, c, d, e});
  }
  return m + 256;
}

// A small exclusive scan in one workgroup and one launch (rocPRIM's look-back scan is two: state
// init + scan). Small merges (the per-op path: a doc state and an update) are launch-bound, and a
// merge runs a dozen scans. Each lane sums a contiguous run, the 1 024 run sums are scanned in LDS,
// each lane writes its run's prefixes; a lane reads in[i] before it writes out[i] and runs are
// disjoint, so in == out is safe. Same results as rocprim::exclusive_scan (wrapping plus).
static bool getenv_flag(const char* name) {  // experiments: YCRDT_ROCPRIM_SCAN=1 takes rocPRIM's scans
  static const bool v = getenv(name) && getenv(name)[0] == '1';
  return v;
}
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

// Larger scans: one launch with a decoupled look-back (rocPRIM's is two: the tile-state init and
// the scan; a merge runs about nine large ones). A tile's state is ONE 64-bit word — epoch (22
// bits) | status (2: aggregate / inclusive prefix) | value (40 bits) — stored and loaded as a
// relaxed agent-scope atomic: coherent across the XCDs' L2s without the cache invalidations an
// acquire costs on gfx950 (an acquire-load spin made every kernel beside it 2-5x slower). Tile
// states stay valid across launches without an init pass: every scan on a stream gets a new
// epoch, and a state left by an earlier scan reads as "not yet" (states start zeroed; epoch 0 is
// never used). The states are per stream (work on one stream is ordered; the merge runs scans on
// two streams at once). Each tile is 256 lanes x 16 entries; its first wavefront publishes the
// tile total, then looks back 64 tiles per round (each lane spinning on its own predecessor) until
// a tile with an inclusive prefix, and publishes its own. Tiles wait only on lower tile ids, which
// the dispatcher issued earlier. A lane reads all of its entries before it writes any, and tiles
// are disjoint, so in == out is safe. Values travel mod 2^40: exact for u32 scans (mod 2^32) and
// for u64 scans whose total is below 2^40 (byte and unit positions of a merge: bounded by HBM).
constexpr uint32_t LB_LANES = 256, LB_ITEMS = 16, LB_TILE = LB_LANES * LB_ITEMS;
constexpr uint32_t LB_EPOCHS = 1u << 22;
template <class T>
__global__ __launch_bounds__(LB_LANES) void k_scan_lb(const uint32_t* in, T* out, uint64_t n,
                                                     unsigned long long* __restrict__ state, uint32_t epoch, uint32_t vec,
                                                     unsigned long long* ord, unsigned long long ord_base) {
  __shared__ T wtot[LB_LANES / 64];
  __shared__ T tile_pre;
  // the tile is the order the workgroup STARTED in, not its block id: every tile it waits on has
  // started, so it is resident and finishes (block ids are dealt to the XCDs' dispatchers
  // independently: with another kernel filling one XCD — a second stream, another process — a
  // tile could wait on a lower block id that cannot be dispatched until the waiting tiles leave)
  const uint32_t tile = ordered_block_id(ord, ord_base);
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint64_t base = (uint64_t)tile * LB_TILE + (uint64_t)t * LB_ITEMS;
  uint32_t v[LB_ITEMS];
  if (vec && base + LB_ITEMS <= n) {
#pragma unroll
    for (uint32_t k = 0; k < LB_ITEMS / 4; ++k) {
      const uint4 q = ((const uint4*)(in + base))[k];
      v[4 * k] = q.x; v[4 * k + 1] = q.y; v[4 * k + 2] = q.z; v[4 * k + 3] = q.w;
    }
  } else {
#pragma unroll
    for (uint32_t k = 0; k < LB_ITEMS; ++k) v[k] = base + k < n ? in[base + k] : 0u;
  }
  T sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < LB_ITEMS; ++k) sum += (T)v[k];
  // tile-exclusive prefix of this lane's run
  T inc = sum;
  for (uint32_t off = 1; off < 64; off <<= 1) {
    const T y = __shfl_up(inc, off);
    if (lane >= off) inc += y;
  }
  if (lane == 63) wtot[wv] = inc;
  __syncthreads();
  T wpre = 0, agg = 0;
#pragma unroll
  for (uint32_t k = 0; k < LB_LANES / 64; ++k) {
    wpre += k < wv ? wtot[k] : (T)0;
    agg += wtot[k];
  }
  T run = wpre + inc - sum;
  if (wv == 0) {
    const uint64_t pre = lb_wave_lookback(state, tile, epoch, (uint64_t)agg);
    if (lane == 0) tile_pre = (T)pre;
  }
  __syncthreads();
  run += tile_pre;
  T o[LB_ITEMS];
#pragma unroll
  for (uint32_t k = 0; k < LB_ITEMS; ++k) { o[k] = run; run += (T)v[k]; }
  if (vec && base + LB_ITEMS <= n) {
    if (sizeof(T) == 4) {
#pragma unroll
      for (uint32_t k = 0; k < LB_ITEMS / 4; ++k)
        ((uint4*)(out + base))[k] = make_uint4((uint32_t)o[4 * k], (uint32_t)o[4 * k + 1], (uint32_t)o[4 * k + 2], (uint32_t)o[4 * k + 3]);
    } else {
#pragma unroll
      for (uint32_t k = 0; k < LB_ITEMS / 2; ++k)
        ((ulonglong2*)(out + base))[k] = make_ulonglong2((unsigned long long)o[2 * k], (unsigned long long)o[2 * k + 1]);
    }
  } else {
#pragma unroll
    for (uint32_t k = 0; k < LB_ITEMS; ++k)
      if (base + k < n) out[base + k] = o[k];
  }
}

// per-stream look-back states (zeroed at allocation, then only written by k_scan_lb)
struct LbState {
  unsigned long long* state = nullptr;  // [tiles] tile states, then the ordered-id counter
  uint64_t tiles = 0;
  uint32_t epoch = 0;
  unsigned long long issued = 0;        // ordered ids handed out on this stream (= the counter once they ran)
};
static std::mutex lb_mu;
static std::unordered_map<hipStream_t, LbState> lb_states;
static LbState* lb_state(uint64_t tiles, hipStream_t s) {  // (lb_mu held)
  LbState& st = lb_states[s];
  if (st.tiles < tiles || st.epoch + 1 >= LB_EPOCHS) {
    const uint64_t nt = std::max<uint64_t>(tiles, st.tiles) + 256;
    if (st.state) {  // the stream's earlier scans may still read the old states
      if (hipStreamSynchronize(s) != hipSuccess) return nullptr;
      (void)hipFree(st.state);
    }
    st = LbState{};
    if (hipMalloc((void**)&st.state, (nt + 1) * 8) != hipSuccess || hipMemsetAsync(st.state, 0, (nt + 1) * 8, s) != hipSuccess) {
      (void)hipGetLastError();
      st = LbState{};
      return nullptr;
    }
    st.tiles = nt;
  }
  ++st.epoch;
  return &st;
}
template <class T>
static bool scan_lb(const uint32_t* in, T* out, uint64_t n, hipStream_t s) {
  const uint64_t tiles = (n + LB_TILE - 1) / LB_TILE;
  std::lock_guard<std::mutex> g(lb_mu);
  LbState* st = lb_state(tiles, s);
  if (!st) return false;
  const uint32_t vec = (((uintptr_t)in | (uintptr_t)out) & 15u) == 0;
  hipLaunchKernelGGL(k_scan_lb<T>, dim3((uint32_t)tiles), dim3(LB_LANES), 0, s, in, out, n, st->state, st->epoch, vec,
                     st->state + st->tiles, st->issued);
  st->issued += tiles;
  return true;
}

bool lb_launch(uint64_t tiles, uint32_t chains, hipStream_t s, LbChains& out) {
  std::lock_guard<std::mutex> g(lb_mu);
  LbState* st = lb_state(tiles * chains, s);
  if (!st) return false;
  out.state = st->state;
  out.stride = tiles;
  out.epoch = st->epoch;
  out.ord = st->state + st->tiles;
  out.ord_base = st->issued;
  st->issued += tiles;
  return true;
}

bool ordered_ids(uint64_t nblocks, hipStream_t s, OrderedIds& out) {
  std::lock_guard<std::mutex> g(lb_mu);
  LbState* st = lb_state(1, s);
  if (!st) return false;
  out.ctr = st->state + st->tiles;
  out.base = st->issued;
  st->issued += nblocks;
  return true;
}

void scan_u32(void* tmp, size_t tmpb, const uint32_t* in, uint32_t* out, uint64_t n, hipStream_t s) {
  if (!n) return;
  if (n <= SMALL_SCAN_MAX) {
    hipLaunchKernelGGL(k_scan_small<uint32_t>, dim3(1), dim3(SMALL_SCAN_LANES), 0, s, in, out, (uint32_t)n);
    return;
  }
  if (!getenv_flag("YCRDT_ROCPRIM_SCAN") && scan_lb<uint32_t>(in, out, n, s)) return;
  rocprim::exclusive_scan(tmp, tmpb, in, out, 0u, (size_t)n, rocprim::plus<uint32_t>(), s);
}

void scan_u32_to_u64(void* tmp, size_t tmpb, const uint32_t* in, uint64_t* out, uint64_t n, hipStream_t s) {
  if (!n) return;
  if (n <= SMALL_SCAN_MAX) {
    hipLaunchKernelGGL(k_scan_small<uint64_t>, dim3(1), dim3(SMALL_SCAN_LANES), 0, s, in, out, (uint32_t)n);
    return;
  }
  if (!getenv_flag("YCRDT_ROCPRIM_SCAN") && scan_lb<uint64_t>(in, out, n, s)) return;
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
                        uint64_t n, hipStream_t s, uint32_t end_bit) {
  if (!n) return;
  rocprim::radix_sort_pairs(tmp, tmpb, kin, kout, vin, vout, (size_t)n, 0, end_bit, s);
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
