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
#include "yc_parse.h"

namespace yc {

constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t UNKNOWN = 0xFFFFFFFEu;  // a reference to a client no update of the batch carries

// ---------------------------------------------------------------- decode geometry
// A large update is cut into chunks of SCHUNK bytes (64-byte aligned, so a chunk owns its words of
// the per-byte bitmaps); one lane per chunk follows the struct chain from the chunk's first byte.
constexpr uint32_t SCHUNK = 1024;
constexpr uint32_t XK = 64;  // entry offsets per chunk in the exit table (yc_decode.hip k_xtab)


// error codes raised on device (first error wins via atomicCAS on the error word)
enum : uint32_t {
  ERR_NONE = 0,
  ERR_DECODE = 1,       // malformed update
  ERR_PENDING = 2,      // missing dependency (Yjs would keep it pending)
  ERR_UNSUPPORTED = 3,  // valid Yjs input outside the engine's current coverage
  ERR_CAPACITY = 4,     // internal capacity exceeded
};

struct Group {          // one decode chunk of a large update
  uint32_t start, end;  // byte range [start,end) inside the batch buffer (start 64-byte aligned)
  uint32_t uend;        // end of the chunk's update (parses never read past it)
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

// count the lanes of a wavefront for which `pred` holds with ONE atomic (the first such lane adds
// the popcount): per-lane atomics on one counter address serialise at the memory side
__device__ __forceinline__ void wave_count_add(uint32_t* ctr, bool pred) {
  const unsigned long long m = __ballot(pred);
  if (m && (threadIdx.x & 63u) == (uint32_t)__ffsll((long long)m) - 1) atomicAdd(ctr, (uint32_t)__popcll(m));
}

// the same over NSHARD counter words picked by workgroup: one counter word takes ≈88 atomics per
// µs (MI355X_MICROARCH.md, dequeue row), so a kernel where most wavefronts count would serialise
// on it; the reader sums the shards
constexpr uint32_t NSHARD = 64;
__device__ __forceinline__ void wave_count_add_sharded(uint32_t* shards, bool pred) {
  wave_count_add(shards + (blockIdx.x & (NSHARD - 1)), pred);
}
// a 0 -> 1 flag any lane may raise: plain stores (they merge in L2; no memory-side atomic)
__device__ __forceinline__ void wave_flag(uint32_t* flag, bool pred) {
  if (__ballot(pred) && (threadIdx.x & 63u) == 0) *flag = 1u;
}

// Exclusive scan of n (<= LANES * 16) u32 values in ONE workgroup of LANES threads: a lane sums a
// contiguous run, the run sums are scanned in LDS (part[LANES]), each lane writes its run's prefixes
// (out[i] may alias in[i]: a lane reads its run before writing it). The small-batch kernels use it.
template <uint32_t LANES>
__device__ __forceinline__ void block_scan_u32(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* part) {
  const uint32_t t = threadIdx.x, per = (n + LANES - 1) / LANES;
  const uint32_t a = min(n, t * per), b = min(n, a + per);
  uint32_t sum = 0;
  for (uint32_t i = a; i < b; ++i) sum += in[i];
  part[t] = sum;
  __syncthreads();
  for (uint32_t off = 1; off < LANES; off <<= 1) {
    const uint32_t v = t >= off ? part[t - off] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;
  for (uint32_t i = a; i < b; ++i) { const uint32_t x = in[i]; out[i] = run; run += x; }
  __syncthreads();
}

// a load that never hits a vector-L1 line older than a memory-side atomic (a relaxed agent-scope
// atomic load: served by L2) — the single-workgroup kernels read what other lanes' atomics wrote
__device__ __forceinline__ uint32_t ld_fresh(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the same with 64-bit prefixes (the clock-length and client-state scans)
// (FRESH: the input was written by atomics in the same kernel — read through L2)
template <uint32_t LANES, bool FRESH = false>
__device__ __forceinline__ void block_scan_u32_u64(const uint32_t* in, uint64_t* out, uint32_t n, uint64_t* part) {
  const uint32_t t = threadIdx.x, per = (n + LANES - 1) / LANES;
  const uint32_t a = min(n, t * per), b = min(n, a + per);
  uint64_t sum = 0;
  for (uint32_t i = a; i < b; ++i) sum += FRESH ? ld_fresh(&in[i]) : in[i];
  part[t] = sum;
  __syncthreads();
  for (uint32_t off = 1; off < LANES; off <<= 1) {
    const uint64_t v = t >= off ? part[t - off] : 0ull;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint64_t run = part[t] - sum;
  for (uint32_t i = a; i < b; ++i) { const uint32_t x = FRESH ? ld_fresh(&in[i]) : in[i]; out[i] = run; run += x; }
  __syncthreads();
}
// a phase boundary inside one workgroup where the phase before handed data over through memory-side
// (L2) atomics as well as plain stores: agent-scope fences on both sides of the barrier, so no
// wavefront reads an L1 line older than an atomic of the phase before.
// THE INVARIANT of the single-workgroup kernels (k_merge_small, k_view_small, k_decode_tail_small,
// k_sections_small, k_encode_small), which separate their phases with a plain __syncthreads
// (k_merge_small: by default; YCRDT_PHASE_FENCE=1 puts phase_sync back, A/B): a column written by ATOMICS in one
// phase is read in a later phase only through ld_fresh (or block_scan_*<.., true>), never by a plain
// load — plain stores reach the CU's vector L1 in order, atomics execute in L2 and leave a stale L1
// line behind. The atomically written columns are: the key table's k_hash (CAS) and k_flags (Or),
// the winner slots k_rootmax / g_maxchild (atomicMax settling pass), the client states cl_state
// (atomicMax), the view representatives krep (atomicMin), the counters ctr->* (err, nsegs, ...).
// tests/test_gpu_phase_fence.py runs the small-merge suites under both settings.
__device__ __forceinline__ void phase_sync() {
  __threadfence();
  __syncthreads();
  __threadfence();
}

// a host switch set to 0 (the small-batch kernels' A/B toggles)
inline bool env_off(const char* name) {
  const char* v = getenv(name);
  return v && v[0] == '0';
}

__device__ __forceinline__ void raise_err(uint32_t* err, uint32_t code) {
  atomicCAS(err, 0u, code);
}

// ---------------------------------------------------------------- varuint writer
__device__ __forceinline__ uint32_t vu_size(uint32_t v) {
  return v < (1u << 7) ? 1 : v < (1u << 14) ? 2 : v < (1u << 21) ? 3 : v < (1u << 28) ? 4 : 5;
}
__device__ __forceinline__ uint32_t wr_vu(uint8_t* __restrict__ o, uint32_t p, uint32_t v) {
  while (v > 127u) { o[p++] = (uint8_t)(0x80u | (v & 0x7fu)); v >>= 7; }
  o[p++] = (uint8_t)v;
  return p;
}
// the same at a 64-bit output position (the integrate encoder: outputs past 4 GiB)
__device__ __forceinline__ uint64_t wr_vu(uint8_t* __restrict__ o, uint64_t p, uint32_t v) {
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
