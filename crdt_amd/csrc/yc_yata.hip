// yc_yata.hip — K4: YArray YATA integration (Item.integrate conflict loop, Y@77594) on gfx950.
//
// Every live YArray list (root array or nested array, keyed by the list slot resolved in
// yc_merge.hip) is integrated independently, so lists are the unit of parallelism:
//   k_ykey / sort      segments of live array lists, radix-sorted by (list slot, segment) — a
//                      stable sort, so each list's members stay in (client, clock) order
//   k_ylist_*          list boundaries (flag + scan)
//   k_yata             one wavefront per list runs the exact YATA loop over
//                      segments in a causal order (depth-first on origin / right origin, the
//                      "stack dive" of integrateStructs, Y@19963), producing the final right
//                      neighbour of every segment (g_right) for Item.mergeWith adjacency.
// A segment is a run of consecutive units of one client cut at every referenced unit, so the
// loop's verdict on the first unit of a run holds for the whole run (SURVEY §7 hard part 1,
// per-clock restatement) and the loop can step over segments instead of units.
#include <cstdlib>

#include "yc_work.h"

namespace yc {

__device__ __forceinline__ uint32_t seg_of_unit(const Work& w, uint32_t g) {
  return w.u_wpre[g >> 6] + (uint32_t)__popcll(w.u_cutbits[g >> 6] & ((2ull << (g & 63)) - 1)) - 1;
}

__global__ void k_ykey(Work w, uint32_t nsegs) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsegs) return;
  w.y_key[s] = (w.g_flags[s] & SEG_ARRAY) ? w.g_key[s] : NONE;
  w.y_iota[s] = s;
  w.g_right[s] = NONE;
  w.y_state[s] = 0;
}

// flag list starts; y_before doubles as the flag array, y_confl receives the scan
__global__ void k_ylist_flags(Work w, uint32_t nsegs) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > nsegs) return;
  if (i == nsegs) { w.y_before[i] = 0; return; }
  const uint32_t k = w.y_keys[i];
  w.y_before[i] = (k != NONE && (i == 0 || w.y_keys[i - 1] != k)) ? 1u : 0u;
}
__global__ void k_ylist_starts(Work w, uint32_t nsegs) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsegs) return;
  const uint32_t k = w.y_keys[i];
  if (k == NONE) return;
  if (w.y_before[i]) w.y_lstart[w.y_confl[i]] = i;
  if (i + 1 == nsegs || w.y_keys[i + 1] == NONE) w.y_lstart[w.y_confl[nsegs]] = i + 1;  // sentinel
}

// One wavefront per list; lane 0 runs the sequential loop (the lists of a batch run in parallel).
__global__ __launch_bounds__(64) void k_yata(Work w, uint32_t nlists, uint32_t nmin) {
  const uint32_t l = blockIdx.x;
  if (l >= nlists || threadIdx.x != 0) return;
  const uint32_t a = w.y_lstart[l], b = w.y_lstart[l + 1];
  if (b - a < nmin) return;  // integrated in LDS by k_yata_lds
  const uint32_t key = w.y_keys[a];
  uint32_t* __restrict__ right = w.g_right;
  uint32_t* __restrict__ state = w.y_state;   // 0 = pending, 1 = on the stack, 2 = integrated
  uint32_t* __restrict__ before = w.y_before; // itemsBeforeOrigin stamp
  uint32_t* __restrict__ confl = w.y_confl;   // conflictingItems stamp
  uint32_t* __restrict__ stack = w.y_stack + a;
  uint32_t head = NONE;  // parent._start
  unsigned long long nscan = 0, ndive = 0, nint = 0;  // YCRDT_DEBUG_TABLES statistics
  uint32_t ctr = 0;      // stamps: every (integration, conflicting-set epoch) gets a fresh value
  for (uint32_t i = a; i < b; ++i) {
    const uint32_t s0 = w.y_seg[i];
    if (state[s0] == 2) continue;
    uint32_t sp = 0;
    stack[sp++] = s0;
    state[s0] = 1;
    while (sp > 0) {
      const uint32_t t = stack[sp - 1];
      const uint32_t oU = w.g_origin[t], rU = w.g_rorigin[t];
      const uint32_t oseg = oU != NONE ? seg_of_unit(w, oU) : NONE;
      const uint32_t rseg = rU != NONE ? seg_of_unit(w, rU) : NONE;
      uint32_t dep = NONE;
      if (oseg != NONE && state[oseg] != 2) dep = oseg;
      else if (rseg != NONE && state[rseg] != 2) dep = rseg;
      if (dep != NONE) {
        if (state[dep] == 1 || w.g_key[dep] != key || !(w.g_flags[dep] & SEG_ARRAY) || sp >= b - a) {
          raise_err(&w.ctr->err, ERR_DECODE);  // a reference outside the list, or a cycle
          return;
        }
        state[dep] = 1;
        stack[sp++] = dep;
        ++ndive;
        continue;
      }
      // ---- Item.integrate(t): YATA conflict resolution between origin and right origin
      uint32_t left = oseg;
      const uint32_t ct = w.g_cidx[t];
      uint32_t o = left != NONE ? right[left] : head;
      if (o != rseg) {
        const uint32_t iter = ++ctr;
        uint32_t ep = ++ctr;
        while (o != NONE && o != rseg) {
          ++nscan;
          before[o] = iter;
          confl[o] = ep;
          const uint32_t oo = w.g_origin[o];
          if (oo == oU) {
            if (w.g_cidx[o] < ct) { left = o; ep = ++ctr; }
            else if (w.g_rorigin[o] == rU) break;
          } else if (oo != NONE && before[seg_of_unit(w, oo)] == iter) {
            if (confl[seg_of_unit(w, oo)] != ep) { left = o; ep = ++ctr; }
          } else {
            break;
          }
          o = right[o];
        }
      }
      uint32_t r2;
      if (left != NONE) { r2 = right[left]; right[left] = t; }
      else { r2 = head; head = t; }
      right[t] = r2;
      state[t] = 2;
      ++nint;
      --sp;
    }
  }
  if (w.dbg) {
    unsigned long long* d = w.dbg + (size_t)w.ngroups * 8 + (size_t)w.ngroups * (GROUP_BYTES / 4096) * 8;
    atomicAdd(d + 0, nint);
    atomicAdd(d + 1, nscan);
    atomicAdd(d + 2, ndive);
  }
}

// ---- LDS-resident YATA for lists of at most CAP segments: the same loop over list-local u16
// indices, every array it touches staged in LDS (12 bytes per segment), so each conflict-scan step
// waits on LDS instead of on L2 (~470 ns per step for the global kernel on a 13 K-segment list).
//   lo / lr   local index of the origin / right-origin segment (L_NONE: none, L_OUT: outside the
//             list — an error once it is needed). Origin units are the last unit of their segment
//             and right-origin units the first (k_refs cuts there), so comparing segments is
//             comparing the units the global kernel compares.
//   rt        right neighbour; cs = client index (14 bits) | state << 14 (0 pending, 1 on the
//             stack, 2 integrated) — the four u16 of a segment are one 8-byte record, so a scan
//             step is one LDS read (the next record is fetched while this one is examined);
//             bf / cf the itemsBeforeOrigin / conflictingItems stamps (u16 pair, all cleared when
//             the counter could wrap inside the next integration).
// The dependency stack lives in global memory (y_stack); lists longer than CAP, or batches with
// 16 K clients or more, take k_yata.
constexpr uint32_t L_NONE = 0xFFFFu, L_OUT = 0xFFFEu;
constexpr uint32_t YL_SMALL = 1024, YL_LARGE = 13312;  // 12 B x 13312 = 156 KiB of LDS

__device__ __forceinline__ uint32_t local_of(const Work& w, uint32_t a, uint32_t n, uint32_t g) {
  uint32_t lo = 0, hi = n;  // y_seg[a, a + n) is sorted (stable sort of the identity)
  while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (w.y_seg[a + m] < g) lo = m + 1; else hi = m; }
  return lo < n && w.y_seg[a + lo] == g ? lo : L_OUT;
}

struct __attribute__((aligned(8))) YRec { uint16_t lo, lr, rt, cs; };  // one ds_read_b64 per scan step
struct __attribute__((aligned(4))) YStamp { uint16_t bf, cf; };

template <uint32_t CAP>
__global__ void k_yata_lds(Work w, uint32_t nlists, uint32_t nmin) {
  const uint32_t l = blockIdx.x;
  if (l >= nlists) return;
  const uint32_t a = w.y_lstart[l], n = w.y_lstart[l + 1] - a;
  if (n < nmin || n > CAP) return;
  __shared__ YRec rec[CAP];
  __shared__ YStamp stp[CAP];
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t g = w.y_seg[a + i];
    const uint32_t oU = w.g_origin[g], rU = w.g_rorigin[g];
    YRec r;
    r.lo = (uint16_t)(oU == NONE ? L_NONE : local_of(w, a, n, seg_of_unit(w, oU)));
    r.lr = (uint16_t)(rU == NONE ? L_NONE : local_of(w, a, n, seg_of_unit(w, rU)));
    r.rt = (uint16_t)L_NONE;
    r.cs = (uint16_t)w.g_cidx[g];
    rec[i] = r;
    stp[i] = YStamp{0, 0};
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t* __restrict__ stack = w.y_stack + a;
    uint32_t head = L_NONE, ctr = 0;
    const uint32_t wrap = 0xFFFFu - n - 3;  // an integration issues at most n + 2 stamps
    auto st = [&](uint32_t i) { return (uint32_t)rec[i].cs >> 14; };
    auto set_st = [&](uint32_t i, uint32_t v) { rec[i].cs = (uint16_t)((rec[i].cs & 0x3FFFu) | (v << 14)); };
    for (uint32_t i0 = 0; i0 < n; ++i0) {
      if (st(i0) == 2) continue;
      uint32_t sp = 0;
      stack[sp++] = i0;
      set_st(i0, 1);
      while (sp > 0) {
        const uint32_t t = stack[sp - 1];
        const YRec T = rec[t];
        const uint32_t os = T.lo, rs = T.lr;
        uint32_t dep = L_NONE;
        if (os != L_NONE && (os == L_OUT || st(os) != 2)) dep = os;
        else if (rs != L_NONE && (rs == L_OUT || st(rs) != 2)) dep = rs;
        if (dep != L_NONE) {
          if (dep == L_OUT || st(dep) == 1 || sp >= n) { raise_err(&w.ctr->err, ERR_DECODE); return; }
          set_st(dep, 1);
          stack[sp++] = dep;
          continue;
        }
        if (ctr > wrap) {  // clear the stamps before the counter can wrap
          for (uint32_t k = 0; k < n; ++k) stp[k] = YStamp{0, 0};
          ctr = 0;
        }
        uint32_t left = os;
        const uint32_t ct = T.cs & 0x3FFFu;
        uint32_t o = left != L_NONE ? rec[left].rt : head;
        if (o != rs) {
          const uint32_t iter = ++ctr;
          uint32_t ep = ++ctr;
          YRec R = o != L_NONE ? rec[o] : YRec{0, 0, 0, 0};
          while (o != L_NONE && o != rs) {
            stp[o] = YStamp{(uint16_t)iter, (uint16_t)ep};
            const uint32_t next = R.rt;
            const YRec RN = next != L_NONE ? rec[next] : YRec{0, 0, 0, 0};  // prefetch the next step
            const uint32_t oo = R.lo;
            if (oo == os) {
              if ((R.cs & 0x3FFFu) < ct) { left = o; ep = ++ctr; }
              else if (R.lr == rs) break;
            } else if (oo != L_NONE && oo != L_OUT) {
              const YStamp S = stp[oo];
              if (S.bf != iter) break;
              if (S.cf != ep) { left = o; ep = ++ctr; }
            } else {
              break;
            }
            o = next;
            R = RN;
          }
        }
        uint32_t r2;
        if (left != L_NONE) { r2 = rec[left].rt; rec[left].rt = (uint16_t)t; }
        else { r2 = head; head = t; }
        rec[t].rt = (uint16_t)r2;
        set_st(t, 2);
        --sp;
      }
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t r = rec[i].rt;
    w.g_right[w.y_seg[a + i]] = r == L_NONE ? NONE : w.y_seg[a + r];
  }
}

uint32_t launch_yata(const Work& w, uint32_t nsegs, uint32_t narray, uint32_t nclients, hipStream_t s) {
  if (!nsegs) return 0;
  const uint32_t grid = nsegs / 256 + 1;
  if (!narray) return 0;  // g_right is only read for YArray members (merge predicate, view)
  hipLaunchKernelGGL(k_ykey, dim3(grid), dim3(256), 0, s, w, nsegs);
  sort_pairs_u32(w.tmp, w.tmp_bytes, w.y_key, w.y_keys, w.y_iota, w.y_seg, nsegs, s);
  hipLaunchKernelGGL(k_ylist_flags, dim3(grid), dim3(256), 0, s, w, nsegs);
  scan_u32(w.tmp, w.tmp_bytes, w.y_before, w.y_confl, nsegs + 1, s);
  uint32_t nlists = 0;
  hipMemcpyAsync(&nlists, w.y_confl + nsegs, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
  hipStreamSynchronize(s);
  if (!nlists) return 0;
  hipLaunchKernelGGL(k_ylist_starts, dim3(grid), dim3(256), 0, s, w, nsegs);
  hipMemsetAsync(w.y_before, 0, sizeof(uint32_t) * (nsegs + 1), s);  // stamps: 0 is never issued
  hipMemsetAsync(w.y_confl, 0, sizeof(uint32_t) * (nsegs + 1), s);
  if (nclients < 16384 && !getenv("YCRDT_YATA_GLOBAL")) {  // client index in 14 bits
    hipLaunchKernelGGL(k_yata_lds<YL_SMALL>, dim3(nlists), dim3(64), 0, s, w, nlists, 1u);
    hipLaunchKernelGGL(k_yata_lds<YL_LARGE>, dim3(nlists), dim3(256), 0, s, w, nlists, YL_SMALL + 1);
    hipLaunchKernelGGL(k_yata, dim3(nlists), dim3(64), 0, s, w, nlists, YL_LARGE + 1);
  } else {
    hipLaunchKernelGGL(k_yata, dim3(nlists), dim3(64), 0, s, w, nlists, 0u);
  }
  return nlists;
}

}  // namespace yc
