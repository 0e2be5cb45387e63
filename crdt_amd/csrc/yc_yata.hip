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
#include <cstring>
#include <utility>
#include <vector>

#include "yc_work.h"

namespace yc {


// YATA's per-segment state: the sort values, the final right neighbours, the sequential kernels' stamps
__global__ void k_yinit(Work w, uint32_t nsegs) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsegs) return;
  w.y_iota[s] = s;
  w.g_right[s] = NONE;
  w.y_state[s] = 0;
}
__global__ void k_ykey(Work w, uint32_t nsegs) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsegs) return;
  w.y_key[s] = (w.g_flags[s] & SEG_ARRAY) ? w.g_key[s] : NONE;
  w.y_iota[s] = s;
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
    unsigned long long* d = w.dbg;
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

// ============================================================================================
// Parallel YATA: the list as a pre-order walk of the origin tree.
// In the final Yjs list the origin-descendants of every item form one contiguous block right
// after it: the B.1 loop only ever leaves an item after a whole sibling block (left moves through
// a block's descendants once it is set on the block's root) or right after its origin, and it only
// stops at a block start (the right origin, a same-origin sibling) or past the origin's block. So
// the list is a pre-order walk of the origin tree whose children — items with the same origin
// (segment), each carrying its block — are ordered by the B.1 loop run over the children alone:
//   scan the siblings from the first until c's right origin (if that is a sibling; else to the
//   end): left := o when o.client < c.client, else stop when o.rightOrigin == c.rightOrigin.
// scripts/yata_tree_proto.py checks this against the sequential loop on per-clock items of 234
// seeded / golden histories. Sibling groups are independent: a group of <= TSMALL children runs on
// one lane, larger ones on one workgroup with the group staged in LDS (<= TLDS) or read from
// global memory (sib_loop below: the B.1 scan evaluated backwards). The pre-order successor (g_right) is
// the first child, else the next sibling of the nearest ancestor-or-self that has one: one
// climbing pass with path halving.
constexpr uint32_t TSMALL = 16, TLDS = 6144;  // 20 B per member in LDS

__global__ void k_tkey(Work w, uint32_t nsegs) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nsegs) return;
  uint32_t key = NONE, p = NONE, rs = NONE;
  if (w.g_flags[s] & SEG_ARRAY) {
    const uint32_t list = w.g_key[s];
    const uint32_t o = w.g_origin[s], r = w.g_rorigin[s];
    // (an origin is in the item's list by construction: k_resolve gave the item its origin's key;
    // a right origin is only checked here)
    if (o != NONE) p = seg_of_unit(w, o);
    if (r != NONE) {
      rs = seg_of_unit(w, r);
      // a right origin in another list than the origin's: Yjs takes the RIGHT one's parent
      // (Item.getMissing, Y@76507) but links the item next to its origin in the origin's list —
      // an item in one list's chain that belongs to another. No replica writes that (only corrupted
      // or crafted bytes): refused, as valid Yjs input the engine does not model
      if (!(w.g_flags[rs] & SEG_ARRAY) || w.g_key[rs] != list) raise_err(&w.ctr->err, ERR_UNSUPPORTED);
    }
    key = p != NONE ? p : nsegs + list;
  }
  w.t_key[s] = key;
  w.y_key[s] = rs;  // the right-origin segment, for k_tprep (y_key is free until launch_ylists)
  w.t_first[s] = NONE;  // (t_nsib: every member's group writes it)
  w.t_jump[s] = p;
}
// group starts: t_done = flags, t_next = their exclusive scan (re-initialised by the groups that use them: sib_state_init)
__global__ void k_tgroup_flags(Work w, uint32_t nsegs) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > nsegs) return;
  const uint32_t k = i < nsegs ? w.t_keys[i] : NONE;
  w.t_done[i] = (k != NONE && (i == 0 || w.t_keys[i - 1] != k)) ? 1u : 0u;
}
__global__ void k_tgroup_starts(Work w, uint32_t nsegs) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == nsegs) w.ctr->tgroups = w.t_next[nsegs];
  if (i >= nsegs) return;
  const uint32_t k = w.t_keys[i];
  if (k == NONE) return;
  w.t_pos[w.t_seg[i]] = i;
  if (w.t_done[i]) w.t_gstart[w.t_next[i]] = i;
  if (i + 1 == nsegs || w.t_keys[i + 1] == NONE) w.t_gstart[w.t_next[nsegs]] = i + 1;  // sentinel
}
// per sorted position: client index, right-origin segment, sorted position of a sibling right origin
// (y_state / y_before / y_confl are free once the list table is built)
__global__ void k_tprep(Work w, uint32_t nsegs) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsegs) return;
  const uint32_t k = w.t_keys[i];
  if (k == NONE) return;
  // a one-member group (most of them) needs no loop state (t_done: k_tgroup_flags' start flags)
  if (w.t_done[i] && (i + 1 == nsegs || w.t_keys[i + 1] != k)) return;
  const uint32_t s = w.t_seg[i];
  const uint32_t rs = w.y_key[s];  // (k_tkey)
  uint32_t rp = NONE;
  if (rs != NONE && w.t_key[rs] == k) rp = w.t_pos[rs];
  w.y_state[i] = w.g_cidx[s];
  w.y_before[i] = rs;  // the anchor key: a right-origin unit starts its segment (k_refs), so unit and segment name it alike
  w.y_confl[i] = rp;
}

// The global loop state of a group's members (t_done, t_next, t_prv, t_mprv, t_mtail, t_otail:
// the in-place loop and the chain scratch of the big / huge groups): set by the group's own kernel
// (the small and wavefront groups keep theirs in LDS / registers)
__device__ __forceinline__ void sib_state_init(const Work& w, uint32_t i) {
  w.t_done[i] = 0;
  w.t_next[i] = NONE;
  w.t_prv[i] = NONE;
  w.t_mprv[i] = NONE;
  w.t_mtail[i] = NONE;
  w.t_otail[i] = NONE;
}
__global__ void k_thuge_init(Work w, uint32_t a, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) sib_state_init(w, a + i);
}

// One sibling group (local indices 0..n-1 in ascending client order). The forward B.1 scan
//   from the first sibling until c's right origin: left := o when o.client < c.client, else stop
//   at o when o.rightOrigin == c.rightOrigin
// is evaluated backwards: the members of one right-origin group always stand in ascending client
// order (the stop rule puts every newcomer before the group's first higher client and after its
// lower ones), so the stop is the group's next higher-client member already placed (its member
// list is walked from the top), else the right-origin sibling, else the end; left is then the
// nearest lower-client sibling before the stop. Integrating in ascending client order makes both
// walks O(1) in practice (scripts/yata_tree_proto.py: 49 backward steps where the forward scans
// take 151 k on the same groups, identical orders).
constexpr uint32_t TOUT = 0x8000u;  // LDS trep flag (bit 31 in global memory): the anchor is the first member of an outside right origin
// (stack: global memory for the in-place groups, LDS for the staged ones — a pop reads the new
// top back, and from global memory that read was a memory round trip per pop: C3's list-head loop
// spent 2.6 ms on them)
template <class A, class S>
__device__ uint32_t sib_loop(A& a, uint32_t n, S* __restrict__ stack, uint32_t* err, unsigned long long* dbg = nullptr) {
  uint32_t head = NONE, tail = NONE;
  unsigned long long st_place = 0, st_m = 0, st_left = 0, st_dive = 0;  // (YCRDT_DEBUG_YATA=1: loop statistics)
  for (uint32_t i0 = 0; i0 < n; ++i0) {
    if (a.done(i0) == 2) continue;
    // the stack's top stays in a register (the stack is in global memory: reading back the
    // element just pushed cost a memory round trip per member); it is read only after a pop
    uint32_t sp = 0, c = i0;
    stack[sp++] = i0;
    a.set_done(i0, 1);
    while (sp > 0) {
      // (the reads of a step are issued in rounds of independent loads — c's fields; then its
      // right origin's state and its group's top; each walk step's fields together — since one
      // lane runs the loop and every dependent LDS / memory read is a wait: C3's list head)
      const uint32_t rp = a.rpos(c);
      bool out = false;
      const uint32_t cc = a.cid(c), ta = a.trep(c, out);
      const uint32_t drp = rp != NONE ? a.done(rp) : 2u;
      // member list of c's right-origin group, walked from its top (highest client) down; a group
      // is anchored at its right-origin sibling (mtail) or, for a right origin outside the group,
      // at its first member (otail: a member can anchor both kinds)
      uint32_t m = out ? a.otail(ta) : a.mtail(ta), succ = NONE;
      if (drp != 2) {  // the right origin is a sibling: place it first
        if (drp == 1 || sp >= n) { raise_err(err, ERR_DECODE); return NONE; }
        a.set_done(rp, 1);
        stack[sp++] = rp;
        c = rp;
        ++st_dive;
        continue;
      }
      while (m != NONE) {
        const uint32_t cm = a.cid(m), pm = a.mprv(m);
        if (cm <= cc) break;
        succ = m;
        m = pm;
        ++st_m;
      }
      a.set_mprv(c, m);
      if (succ != NONE) a.set_mprv(succ, c);
      else if (out) a.set_otail(ta, c);
      else a.set_mtail(ta, c);
      const uint32_t stop = succ != NONE ? succ : rp;
      uint32_t left = stop != NONE ? a.prv(stop) : tail, nx = head;
      while (left != NONE) {
        const uint32_t cl = a.cid(left), pl = a.prv(left), nl = a.next(left);
        if (cl < cc) { nx = nl; break; }
        left = pl;
        ++st_left;
      }
      ++st_place;
      a.set_prv(c, left);
      a.set_next(c, nx);
      if (left != NONE) a.set_next(left, c); else head = c;
      if (nx != NONE) a.set_prv(nx, c); else tail = c;
      a.set_done(c, 2);
      if (--sp > 0) c = stack[sp - 1];
    }
  }
  if (dbg) { atomicAdd(&dbg[3], st_place); atomicAdd(&dbg[4], st_m); atomicAdd(&dbg[5], st_left); atomicAdd(&dbg[6], st_dive); }
  return head;
}
struct SibGlobal {  // a group read in place (sorted positions base..base+n); links hold positions
  const Work& w;
  uint32_t base;
  __device__ static uint32_t loc(uint32_t x, uint32_t b) { return x == NONE ? NONE : x - b; }
  __device__ static uint32_t glo(uint32_t x, uint32_t b) { return x == NONE ? NONE : x + b; }
  __device__ uint32_t done(uint32_t i) const { return w.t_done[base + i]; }
  __device__ void set_done(uint32_t i, uint32_t v) { w.t_done[base + i] = v; }
  __device__ uint32_t rpos(uint32_t i) const { return loc(w.y_confl[base + i], base); }
  __device__ uint32_t trep(uint32_t i, bool& out) const { const uint32_t t = w.t_trep[base + i]; out = (t >> 31) != 0; return (t & 0x7FFFFFFFu) - base; }
  __device__ uint32_t cid(uint32_t i) const { return w.y_state[base + i]; }
  __device__ uint32_t next(uint32_t i) const { return loc(w.t_next[base + i], base); }
  __device__ void set_next(uint32_t i, uint32_t v) { w.t_next[base + i] = glo(v, base); }
  __device__ uint32_t prv(uint32_t i) const { return loc(w.t_prv[base + i], base); }
  __device__ void set_prv(uint32_t i, uint32_t v) { w.t_prv[base + i] = glo(v, base); }
  __device__ uint32_t mprv(uint32_t i) const { return loc(w.t_mprv[base + i], base); }
  __device__ void set_mprv(uint32_t i, uint32_t v) { w.t_mprv[base + i] = glo(v, base); }
  __device__ uint32_t mtail(uint32_t i) const { return loc(w.t_mtail[base + i], base); }
  __device__ void set_mtail(uint32_t i, uint32_t v) { w.t_mtail[base + i] = glo(v, base); }
  __device__ uint32_t otail(uint32_t i) const { return loc(w.t_otail[base + i], base); }
  __device__ void set_otail(uint32_t i, uint32_t v) { w.t_otail[base + i] = glo(v, base); }
};
struct __attribute__((aligned(4))) SibRec { uint32_t cid; uint16_t rpos, trep, nxt, prv, mprv, mtail, otail, pad; };
constexpr uint16_t S_NONE = 0xFFFFu;
struct SibLds {  // a group staged in LDS (n <= TLDS)
  SibRec* rec;
  uint8_t* st;
  __device__ static uint32_t w32(uint16_t x) { return x == S_NONE ? NONE : x; }
  __device__ static uint16_t w16(uint32_t x) { return x == NONE ? S_NONE : (uint16_t)x; }
  __device__ uint32_t done(uint32_t i) const { return st[i]; }
  __device__ void set_done(uint32_t i, uint32_t v) { st[i] = (uint8_t)v; }
  __device__ uint32_t rpos(uint32_t i) const { return w32(rec[i].rpos); }
  __device__ uint32_t trep(uint32_t i, bool& out) const { out = (rec[i].trep & TOUT) != 0; return rec[i].trep & ~TOUT; }
  __device__ uint32_t cid(uint32_t i) const { return rec[i].cid; }
  __device__ uint32_t next(uint32_t i) const { return w32(rec[i].nxt); }
  __device__ void set_next(uint32_t i, uint32_t v) { rec[i].nxt = w16(v); }
  __device__ uint32_t prv(uint32_t i) const { return w32(rec[i].prv); }
  __device__ void set_prv(uint32_t i, uint32_t v) { rec[i].prv = w16(v); }
  __device__ uint32_t mprv(uint32_t i) const { return w32(rec[i].mprv); }
  __device__ void set_mprv(uint32_t i, uint32_t v) { rec[i].mprv = w16(v); }
  __device__ uint32_t mtail(uint32_t i) const { return w32(rec[i].mtail); }
  __device__ void set_mtail(uint32_t i, uint32_t v) { rec[i].mtail = w16(v); }
  __device__ uint32_t otail(uint32_t i) const { return w32(rec[i].otail); }
  __device__ void set_otail(uint32_t i, uint32_t v) { rec[i].otail = w16(v); }
};

// sibling order -> first child / next sibling (segment indices)
__device__ __forceinline__ void sib_publish(const Work& w, uint32_t a, uint32_t n, uint32_t nsegs, uint32_t head) {
  const uint32_t key = w.t_keys[a];
  if (key < nsegs && head != NONE) w.t_first[key] = w.t_seg[a + head];
}
// right-origin group anchor of every member: the right-origin sibling itself, or (a right origin
// outside the group, or none) the first member with the same right-origin unit
__device__ __forceinline__ void sib_anchors_small(const Work& w, uint32_t a, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t t = w.y_confl[a + i];
    if (t == NONE) {
      const uint32_t r = w.y_before[a + i];
      t = a + i;
      for (uint32_t j = 0; j < i; ++j)
        if (w.y_confl[a + j] == NONE && w.y_before[a + j] == r) { t = a + j; break; }
      t |= 0x80000000u;
    }
    w.t_trep[a + i] = t;
  }
}

// Groups of at most TSMALL members: one lane each, the group staged in the lane's slice of LDS
// (8-bit links) so the loop's dependent steps wait on LDS, not on memory (it walked the group in
// global memory: C4's 1.4 ms).
struct __attribute__((aligned(4))) SibRec8 { uint32_t cid; uint8_t rpos, trep, nxt, prv, mprv, mtail, otail, pad; };
struct SibLds8 {
  SibRec8* rec;
  uint8_t* st;
  static constexpr uint8_t N8 = 0xFFu, OUT8 = 0x80u;
  __device__ static uint32_t w32(uint8_t x) { return x == N8 ? NONE : x; }
  __device__ static uint8_t w8(uint32_t x) { return x == NONE ? N8 : (uint8_t)x; }
  __device__ uint32_t done(uint32_t i) const { return st[i]; }
  __device__ void set_done(uint32_t i, uint32_t v) { st[i] = (uint8_t)v; }
  __device__ uint32_t rpos(uint32_t i) const { return w32(rec[i].rpos); }
  __device__ uint32_t trep(uint32_t i, bool& out) const { out = (rec[i].trep & OUT8) != 0; return rec[i].trep & ~OUT8; }
  __device__ uint32_t cid(uint32_t i) const { return rec[i].cid; }
  __device__ uint32_t next(uint32_t i) const { return w32(rec[i].nxt); }
  __device__ void set_next(uint32_t i, uint32_t v) { rec[i].nxt = w8(v); }
  __device__ uint32_t prv(uint32_t i) const { return w32(rec[i].prv); }
  __device__ void set_prv(uint32_t i, uint32_t v) { rec[i].prv = w8(v); }
  __device__ uint32_t mprv(uint32_t i) const { return w32(rec[i].mprv); }
  __device__ void set_mprv(uint32_t i, uint32_t v) { rec[i].mprv = w8(v); }
  __device__ uint32_t mtail(uint32_t i) const { return w32(rec[i].mtail); }
  __device__ void set_mtail(uint32_t i, uint32_t v) { rec[i].mtail = w8(v); }
  __device__ uint32_t otail(uint32_t i) const { return w32(rec[i].otail); }
  __device__ void set_otail(uint32_t i, uint32_t v) { rec[i].otail = w8(v); }
};
constexpr uint32_t TS_BLOCK = 64;
__global__ __launch_bounds__(TS_BLOCK) void k_tsib_small(Work w, uint32_t nsegs) {
  __shared__ SibRec8 rec[TS_BLOCK][TSMALL];
  __shared__ uint32_t rr[TS_BLOCK][TSMALL];   // right-origin units (anchors), then the loop's stack
  __shared__ uint8_t st[TS_BLOCK][TSMALL];
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= w.ctr->tgroups) return;
  const uint32_t a = w.t_gstart[g], n = w.t_gstart[g + 1] - a;
  if (n > TSMALL) {
    w.t_big[atomicAdd(&w.ctr->tbig, 1u)] = g;
    return;
  }
  const uint32_t t = threadIdx.x;
  uint32_t head = 0;
  const uint32_t gkey = w.t_keys[a];
  if (n == 1) {  // (most groups: one child)
    const uint32_t s0 = w.t_seg[a];
    if (gkey < nsegs) w.t_first[gkey] = s0;
    w.t_nsib[s0] = NONE;
    return;
  }
  {
    bool plain = true;  // (as in k_tsib_wave: one outside right origin, clients strictly ascending)
    for (uint32_t i = 0; i < n; ++i) {  // independent loads, issued together
      const uint32_t rp = w.y_confl[a + i];
      rec[t][i] = SibRec8{w.y_state[a + i], rp == NONE ? SibLds8::N8 : (uint8_t)(rp - a), 0, SibLds8::N8, SibLds8::N8,
                          SibLds8::N8, SibLds8::N8, SibLds8::N8, 0};
      rr[t][i] = rp == NONE ? w.y_before[a + i] : NONE;
      st[t][i] = 0;
      plain = plain && rp == NONE && rr[t][i] == rr[t][0] && (i == 0 || rec[t][i].cid > rec[t][i - 1].cid);
    }
    if (plain) {
      for (uint32_t i = 0; i < n; ++i) rec[t][i].nxt = i + 1 < n ? (uint8_t)(i + 1) : SibLds8::N8;
      head = 0;
    } else {
      // right-origin group anchors (sib_anchors_small): the sibling itself, else the first member
      // with the same outside right origin
      for (uint32_t i = 0; i < n; ++i) {
        if (rec[t][i].rpos != SibLds8::N8) { rec[t][i].trep = rec[t][i].rpos; continue; }
        uint32_t j = 0;
        while (j < i && !(rec[t][j].rpos == SibLds8::N8 && rr[t][j] == rr[t][i])) ++j;
        rec[t][i].trep = (uint8_t)(j | SibLds8::OUT8);
      }
      SibLds8 acc{rec[t], st[t]};
      head = sib_loop(acc, n, rr[t], &w.ctr->err);  // (the anchors are set: rr is the stack now)
    }
  }
  if (head == NONE) return;  // (a right-origin cycle: reported)
  for (uint32_t i = 0; i < n; ++i) rec[t][i].cid = w.t_seg[a + i];  // the members' segments (cid is done with)
  if (gkey < nsegs) w.t_first[gkey] = rec[t][head].cid;  // (sib_publish)
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t x = rec[t][i].nxt;
    w.t_nsib[rec[t][i].cid] = x == SibLds8::N8 ? NONE : rec[t][x].cid;
  }
}
// one workgroup per large group: anchors of outside right origins through an LDS hash table,
// the group staged in LDS when it fits (else collapsed into chains, else read in place); lane 0
// runs the loop
constexpr uint32_t THASH = 2048, HNONE = 0xFFFFFFFEu;  // the "no right origin" key (units < HNONE)

// Chains. Members c_1..c_m at consecutive sorted positions (one client, ascending clocks) with
// rightOrigin(c_k) = c_{k-1}, where no other member names c_1..c_{m-1} as its right origin, are
// placed by sib_loop as one contiguous block c_m .. c_1: c_k is integrated right
// after c_{k-1} (nothing else can dive into an unreferenced member), lands immediately before it
// (its right-origin group is {c_k}; prv(c_{k-1}) has a lower client), and no later member can
// stop inside the block (its stop would be a referenced interior member) or step left into it
// (a walk from the right crosses the block whole: one client). So the loop runs over chains as
// single members — cid of the client, right origin and anchor of c_1, referenced by c_m — and the
// block is expanded afterwards. The C3 list head (≈790 k unshifts, all origin = the list root)
// collapses to one member per (replica, round).
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t* sh, uint32_t& total) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t x = v;
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) sh[wv] = x;
  __syncthreads();
  uint32_t off = 0;
  for (uint32_t k = 0; k < wv; ++k) off += sh[k];
  total = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  return off + x - v;
}

// Groups of TSMALL+1 .. TWAVE members: one wavefront each, four per workgroup (C4's list heads:
// the pushes of up to 64 replicas after one element, ~10^5 groups). Lane i holds member i and
// finds its anchor with a shuffle scan (the lowest member with the same outside right origin).
// The loop runs on the whole wavefront in position form (sib_wave).
constexpr uint32_t TWAVE = 64;
// The B.1 loop of sib_loop, evaluated by the whole wavefront (lane = member, n <= 64) with the
// list kept in POSITION space instead of lane 0 walking linked lists (scripts/sib_wave_proto.py
// checks the forms equal, ties and right-origin cycles included). Member-space registers (lane =
// member): done, pos, the stack; position-space registers (lane = list position x): the client,
// right-origin group and member at x. Members are placed in sib_loop's order (by index, each
// right-origin sibling first). Placing c:
//   succ = the first position holding a member of c's right-origin group with a client above c's
//          (a group's members stand in ascending client order, equal clients in placement order);
//   stop = succ, else c's right-origin sibling, else the end;
//   left = the last position before stop holding a client below c's;
//   c goes after left: the position-space entries at or past it shift up one lane.
// A step is two ballots, three lane shifts and readlanes of wave-uniform indices. Returns the
// first member (NONE on a right-origin cycle, reported as ERR_DECODE); pos = the lane's member's
// final position, pm = the member at the lane's position.
__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t i) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)i); }
__device__ uint32_t sib_wave(uint32_t n, uint32_t lane, uint32_t cid, uint32_t rp, uint32_t gk, int& pos, uint32_t& pm, uint32_t* err) {
  uint32_t done = 0, stk = 0, placed = 0;
  uint32_t pc = 0, pg = 0xFFFFFFFFu;
  pos = -1;
  pm = NONE;
  for (uint32_t i0 = 0; i0 < n; ++i0) {
    if (rdlane(done, i0) == 2u) continue;
    if (lane == i0) done = 1;
    if (lane == 0) stk = i0;
    uint32_t sp = 1, c = i0;
    while (sp > 0) {
      const uint32_t r = rdlane(rp, c);
      if (r != NONE) {
        const uint32_t dr = rdlane(done, r);
        if (dr != 2u) {  // the right origin is a sibling: place it first
          if (dr == 1u || sp >= n) { if (lane == 0) raise_err(err, ERR_DECODE); return NONE; }
          if (lane == r) done = 1;
          if (lane == sp) stk = r;
          ++sp;
          c = r;
          continue;
        }
      }
      const uint32_t cc = rdlane(cid, c), g = rdlane(gk, c);
      const bool live = lane < placed;
      const uint64_t sm = __ballot(live && pg == g && pc > cc);
      const uint32_t pstop = sm ? (uint32_t)__ffsll((long long)sm) - 1 : r != NONE ? (uint32_t)rdlane((uint32_t)pos, r) : placed;
      const uint64_t lm = __ballot(live && lane < pstop && pc < cc);
      const uint32_t p = lm ? 64u - (uint32_t)__clzll((long long)lm) : 0u;  // past the last such position
      if (done == 2u && pos >= (int)p) ++pos;
      const uint32_t upc = (uint32_t)__shfl_up((int)pc, 1, 64), upg = (uint32_t)__shfl_up((int)pg, 1, 64),
                     upm = (uint32_t)__shfl_up((int)pm, 1, 64);
      if (lane > p) { pc = upc; pg = upg; pm = upm; }
      else if (lane == p) { pc = cc; pg = g; pm = c; }
      if (lane == c) { pos = (int)p; done = 2; }
      ++placed;
      if (--sp > 0) c = rdlane(stk, sp - 1);
    }
  }
  return n ? rdlane(pm, 0) : NONE;
}
__global__ __launch_bounds__(256) void k_tsib_wave(Work w, uint32_t nsegs, uint32_t nbig) {
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t bi = blockIdx.x * 4 + wv;
  if (bi >= nbig) return;  // whole wavefronts only: no workgroup barrier below
  const uint32_t g = w.t_big[bi];
  const uint32_t a = w.t_gstart[g], n = w.t_gstart[g + 1] - a;
  if (n > TWAVE) return;
  const bool in = lane < n;
  // every load the group needs, in one round: the member's columns, its segment, the group key
  const uint32_t rp = in ? w.y_confl[a + lane] : NONE;
  const uint32_t cid = in ? w.y_state[a + lane] : 0u;
  const uint32_t r0 = in ? w.y_before[a + lane] : NONE;
  const uint32_t segl = in ? w.t_seg[a + lane] : NONE;
  const uint32_t gkey = w.t_keys[a];
  const uint32_t rk = !in || rp != NONE ? NONE : r0 == NONE ? HNONE : r0;  // (segments < HNONE)
  uint32_t anc = NONE;
  for (uint32_t j = 0; j < n; ++j) {
    const uint32_t rj = rdlane(rk, j);
    if (anc == NONE && rk != NONE && rj == rk) anc = j;
  }
  // right-origin group: the sibling (local index), or 64 + the anchor of an outside right origin
  const uint32_t lrp = rp != NONE ? rp - a : NONE;
  const uint32_t gk = !in ? 0xFFFFu : lrp != NONE ? lrp : TWAVE + anc;
  int pos;
  uint32_t pm;
  uint32_t head;
  // the common group — every member's right origin the same outside unit (or none), clients
  // strictly ascending (C4's list heads: concurrent pushes after one element) — is ordered by
  // client: each newcomer goes to the end (no higher client is placed yet, no stop before it)
  const uint32_t cprev = (uint32_t)__shfl_up((int)cid, 1, 64);
  const bool plain = !__ballot(in && (rp != NONE || rk != rdlane(rk, 0) || (lane > 0 && cid <= cprev)));
  if (plain) {
    pos = in ? (int)lane : -1;
    pm = lane;
    head = 0;
  } else {
    head = sib_wave(n, lane, in ? cid : 0xFFFFFFFFu, in ? lrp : NONE, gk, pos, pm, &w.ctr->err);
    if (head == NONE) return;
  }
  const uint32_t x = (uint32_t)__shfl((int)pm, (pos + 1) & 63, 64);  // the member after this one
  const uint32_t sx = (uint32_t)__shfl((int)segl, (int)(x & 63), 64);  // ... and its segment
  if (in) w.t_nsib[segl] = pos + 1 < (int)n ? sx : NONE;
  const uint32_t hseg = rdlane(segl, head);
  if (lane == 0 && gkey < nsegs) w.t_first[gkey] = hseg;  // (sib_publish, from registers)
}

// CAP: LDS capacity in members, HS: anchor hash slots. MID = the variant for groups of at most
// CAP members (a small LDS footprint, several workgroups per CU); the other takes the rest.
constexpr uint32_t TMID = 1024;
template <uint32_t CAP, uint32_t HS, bool MID>
__global__ __launch_bounds__(256) void k_tsib_big(Work w, uint32_t nsegs) {
  const uint32_t g = w.t_big[blockIdx.x];
  const uint32_t a = w.t_gstart[g], n = w.t_gstart[g + 1] - a;
  if (MID ? (n > CAP || n <= TWAVE) : (n <= TMID || n > CAP)) return;  // n > TLDS: the grid-wide huge-group path
  // a plain group (k_tsib_wave: one outside right origin, strictly ascending clients) is in
  // ascending order: no staging, no loop
  __shared__ uint32_t notplain;
  if (threadIdx.x == 0) notplain = 0;
  __syncthreads();
  {
    const uint32_t r00 = w.y_before[a];
    bool bad = false;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
      bad |= w.y_confl[a + i] != NONE || w.y_before[a + i] != r00 || (i > 0 && w.y_state[a + i] <= w.y_state[a + i - 1]);
    if (bad) notplain = 1;  // (plain stores of one value)
  }
  __syncthreads();
  if (!notplain) {
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) w.t_nsib[w.t_seg[a + i]] = i + 1 < n ? w.t_seg[a + i + 1] : NONE;
    if (threadIdx.x == 0) {
      const uint32_t key = w.t_keys[a];
      if (key < nsegs) w.t_first[key] = w.t_seg[a];
    }
    return;
  }
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) sib_state_init(w, a + i);
  __syncthreads();  // (workgroup-scope: the stores are visible to the block's later reads)
  __shared__ SibRec rec[CAP];
  __shared__ uint8_t st[CAP];
  __shared__ uint16_t stk[CAP];  // the loop's stack (staged groups)
  __shared__ uint32_t hkey[HS], hval[HS];
  __shared__ uint32_t head_s, scan_sh[4];
  for (uint32_t i = threadIdx.x; i < HS; i += blockDim.x) { hkey[i] = NONE; hval[i] = NONE; }
  __syncthreads();
  // anchors: the first member (lowest position) of every outside right-origin unit
  // (loops over the members take 4 coalesced elements per lane per round: their loads are
  // independent, so a huge group costs rounds of bandwidth, not rounds of latency)
  constexpr uint32_t U4 = 4;
  for (uint32_t i0 = threadIdx.x; i0 < n; i0 += blockDim.x * U4) {
    uint32_t rc[U4];
#pragma unroll
    for (uint32_t u = 0; u < U4; ++u) { const uint32_t i = i0 + u * blockDim.x; rc[u] = i < n ? w.y_confl[a + i] : 0u; }
#pragma unroll
    for (uint32_t u = 0; u < U4; ++u) {
      const uint32_t i = i0 + u * blockDim.x;
      if (i >= n || rc[u] != NONE) continue;
      const uint32_t r0 = w.y_before[a + i], r = r0 == NONE ? HNONE : r0;
      uint32_t slot = (r * 2654435761u) & (HS - 1);
      for (uint32_t probe = 0;; ++probe) {
        if (probe == HS) { raise_err(&w.ctr->err, ERR_CAPACITY); break; }
        const uint32_t old = atomicCAS(&hkey[slot], NONE, r);
        if (old == NONE || old == r) { atomicMin(&hval[slot], i); break; }
        slot = (slot + 1) & (HS - 1);
      }
    }
  }
  __syncthreads();
  for (uint32_t i0 = threadIdx.x; i0 < n; i0 += blockDim.x * U4) {
    uint32_t t[U4];
#pragma unroll
    for (uint32_t u = 0; u < U4; ++u) { const uint32_t i = i0 + u * blockDim.x; t[u] = i < n ? w.y_confl[a + i] : 0u; }
#pragma unroll
    for (uint32_t u = 0; u < U4; ++u) {
      const uint32_t i = i0 + u * blockDim.x;
      if (i >= n) continue;
      if (t[u] == NONE) {
        const uint32_t r0 = w.y_before[a + i], r = r0 == NONE ? HNONE : r0;
        uint32_t slot = (r * 2654435761u) & (HS - 1);
        for (uint32_t probe = 0; probe < HS && hkey[slot] != r; ++probe) slot = (slot + 1) & (HS - 1);
        t[u] = (hkey[slot] == r ? a + hval[slot] : a + i) | 0x80000000u;
      }
      w.t_trep[a + i] = t[u];
    }
  }
  __syncthreads();
  uint32_t nn = NONE;  // member count after collapsing chains (n > CAP only)
  if (n > CAP) {
    // t_mtail / t_prv / t_next hold NONE here (k_tprep) and serve as scratch:
    //   t_mtail[p] = 0   p is named as right origin by a member other than its chain successor
    //   t_prv[i]         the chain (node) of position i;  t_next[k]  first position of node k
    for (uint32_t i0 = threadIdx.x; i0 < n; i0 += blockDim.x * U4) {
      uint32_t rp[U4], ci[U4], cp[U4];
#pragma unroll
      for (uint32_t u = 0; u < U4; ++u) { const uint32_t i = i0 + u * blockDim.x; rp[u] = i < n ? w.y_confl[a + i] : NONE; }
#pragma unroll
      for (uint32_t u = 0; u < U4; ++u) {
        const uint32_t i = i0 + u * blockDim.x;
        const bool chk = rp[u] != NONE && rp[u] - a + 1 == i;  // a chain link candidate: compare clients
        ci[u] = chk ? w.y_state[a + i] : 0u;
        cp[u] = chk ? w.y_state[rp[u]] : 1u;
      }
#pragma unroll
      for (uint32_t u = 0; u < U4; ++u)
        if (rp[u] != NONE && ci[u] != cp[u]) w.t_mtail[rp[u]] = 0;
    }
    __syncthreads();
    // chain numbering: CU consecutive positions per lane per round (vector-width loads, one
    // workgroup scan per 256 x CU positions)
    constexpr uint32_t CU = 8;
    uint32_t carry = 0;
    for (uint32_t base = 0; base < n; base += blockDim.x * CU) {
      const uint32_t i0 = base + threadIdx.x * CU;
      uint32_t fm = 0, cnt = 0;  // bit u: position i0 + u starts a chain
#pragma unroll
      for (uint32_t u = 0; u < CU; ++u) {
        const uint32_t i = i0 + u;
        if (i < n) {
          const bool link = i > 0 && w.y_confl[a + i] == a + i - 1 && w.y_state[a + i] == w.y_state[a + i - 1] &&
                            w.t_mtail[a + i - 1] == NONE;
          if (!link) { fm |= 1u << u; ++cnt; }
        }
      }
      uint32_t tot;
      uint32_t k = carry + block_excl_scan256(cnt, scan_sh, tot);  // chains started before i0
#pragma unroll
      for (uint32_t u = 0; u < CU; ++u) {
        const uint32_t i = i0 + u;
        if (i < n) {
          if ((fm >> u) & 1u) { w.t_next[a + k] = i; ++k; }
          w.t_prv[a + i] = k - 1;
        }
      }
      carry += tot;
    }
    nn = carry;
    __syncthreads();
    if (nn > CAP) {  // no room in LDS even collapsed: restore the scratch, run in place
      for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        w.t_mtail[a + i] = NONE;
        w.t_prv[a + i] = NONE;
        w.t_next[a + i] = NONE;
      }
      __syncthreads();
    }
  }
  if (nn != NONE && nn <= CAP) {
    const uint32_t* node = w.t_prv + a;
    const uint32_t* nfirst = w.t_next + a;
    for (uint32_t k = threadIdx.x; k < nn; k += blockDim.x) {
      const uint32_t f = nfirst[k];
      const uint32_t rp = w.y_confl[a + f];
      const uint32_t t = w.t_trep[a + f];
      const uint32_t tq = node[(t & 0x7FFFFFFFu) - a];
      rec[k] = SibRec{w.y_state[a + f], (uint16_t)(rp == NONE ? S_NONE : node[rp - a]),
                      (uint16_t)(tq | ((t >> 31) ? TOUT : 0u)), S_NONE, S_NONE, S_NONE, S_NONE, S_NONE, 0};
      st[k] = 0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      SibLds acc{rec, st};
      head_s = sib_loop(acc, nn, stk, &w.ctr->err);
    }
    __syncthreads();
    // expand: node k spans positions nfirst[k] .. nfirst[k + 1] - 1, listed from the last down
    auto leftmost = [&](uint32_t k) { return (k + 1 < nn ? nfirst[k + 1] : n) - 1; };
    for (uint32_t i0 = threadIdx.x; i0 < n; i0 += blockDim.x * U4) {
      uint32_t k[U4], f[U4], nx[U4], sg[U4], sx[U4];
#pragma unroll
      for (uint32_t u = 0; u < U4; ++u) { const uint32_t i = i0 + u * blockDim.x; k[u] = i < n ? node[i] : 0u; }
#pragma unroll
      for (uint32_t u = 0; u < U4; ++u) f[u] = nfirst[k[u]];
#pragma unroll
      for (uint32_t u = 0; u < U4; ++u) {
        const uint32_t i = i0 + u * blockDim.x;
        if (i > f[u]) nx[u] = i - 1;
        else {
          const uint32_t kn = rec[k[u]].nxt;
          nx[u] = kn == S_NONE ? NONE : leftmost(kn);
        }
      }
#pragma unroll
      for (uint32_t u = 0; u < U4; ++u) {
        const uint32_t i = i0 + u * blockDim.x;
        sg[u] = i < n ? w.t_seg[a + i] : 0u;
        sx[u] = i < n && nx[u] != NONE ? w.t_seg[a + nx[u]] : NONE;
      }
#pragma unroll
      for (uint32_t u = 0; u < U4; ++u)
        if (i0 + u * blockDim.x < n) w.t_nsib[sg[u]] = sx[u];
    }
    if (threadIdx.x == 0 && head_s != NONE) sib_publish(w, a, n, nsegs, leftmost(head_s));
    return;
  }
  if (n <= CAP) {
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
      const uint32_t rp = w.y_confl[a + i];
      const uint32_t t = w.t_trep[a + i];
      rec[i] = SibRec{w.y_state[a + i], (uint16_t)(rp == NONE ? S_NONE : rp - a),
                      (uint16_t)(((t & 0x7FFFFFFFu) - a) | ((t >> 31) ? TOUT : 0u)), S_NONE, S_NONE, S_NONE, S_NONE, S_NONE, 0};
      st[i] = 0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      SibLds acc{rec, st};
      head_s = sib_loop(acc, n, stk, &w.ctr->err);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
      const uint32_t x = rec[i].nxt;
      w.t_nsib[w.t_seg[a + i]] = x == S_NONE ? NONE : w.t_seg[a + x];
    }
  } else {
    if (threadIdx.x == 0) {
      SibGlobal acc{w, a};
      head_s = sib_loop(acc, n, w.y_stack + a, &w.ctr->err);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
      const uint32_t x = w.t_next[a + i];
      w.t_nsib[w.t_seg[a + i]] = x == NONE ? NONE : w.t_seg[x];
    }
  }
  if (threadIdx.x == 0 && head_s != NONE) sib_publish(w, a, n, nsegs, head_s);
}
// ---- Huge sibling groups (more members than TLDS): the member passes of k_tsib_big — right-origin
// anchors, chain marks, chain numbering, the expansion — run grid-wide over the group, and only the
// loop over the collapsed chains runs on one lane (with the chains in LDS). In one workgroup those
// passes were latency-bound (C3's list head, 790 k members: ≈9.7 ms, of 16 ms of YATA).
// Group descriptors: the host reads (start, size) of the huge groups (> TLDS members) — a count
// and a short compacted list (copying a descriptor for every big group, 800 KB pageable on C4, took
// 0.4 ms of host time between two kernels)
constexpr uint32_t HUGE_DESC_MAX = 62;  // descriptors read with the count in one copy (more: a second copy)
__global__ void k_tbig_desc(Work w, uint32_t* __restrict__ desc) {  // (grid-stride over the big groups: no count on the host)
  const uint32_t nbig = w.ctr->tbig;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nbig; i += gridDim.x * blockDim.x) {
    const uint32_t g = w.t_big[i], a = w.t_gstart[g], n = w.t_gstart[g + 1] - a;
    if (n <= TLDS) continue;
    const uint32_t k = atomicAdd(&desc[0], 1u);
    desc[2 + 2 * k] = a;
    desc[3 + 2 * k] = n;
  }
}
// anchors: the first member of every outside right-origin unit (global open addressing, P slots)
__global__ __launch_bounds__(256) void k_thuge_hash(Work w, uint32_t a, uint32_t n, uint32_t P) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || w.y_confl[a + i] != NONE) return;
  const uint32_t r0 = w.y_before[a + i], r = r0 == NONE ? HNONE : r0;
  uint32_t slot = (r * 2654435761u) & (P - 1);
  for (uint32_t probe = 0; probe < P; ++probe) {
    const uint32_t old = atomicCAS(&w.t_hkey[slot], NONE, r);
    if (old == NONE || old == r) { atomicMin(&w.t_hval[slot], i); return; }
    slot = (slot + 1) & (P - 1);
  }
  raise_err(&w.ctr->err, ERR_CAPACITY);
}
// right-origin group anchor of every member (t_trep, as k_tsib_big) and the chain marks: t_mtail[p]
// = 0 where p is named as right origin by a member other than its chain successor
__global__ __launch_bounds__(256) void k_thuge_anchor(Work w, uint32_t a, uint32_t n, uint32_t P) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t rp = w.y_confl[a + i];
  uint32_t t = rp;
  if (rp == NONE) {
    const uint32_t r0 = w.y_before[a + i], r = r0 == NONE ? HNONE : r0;
    uint32_t slot = (r * 2654435761u) & (P - 1);
    for (uint32_t probe = 0; probe < P && w.t_hkey[slot] != r; ++probe) slot = (slot + 1) & (P - 1);
    t = (w.t_hkey[slot] == r ? a + w.t_hval[slot] : a + i) | 0x80000000u;
  } else if (rp + 1 != a + i || w.y_state[a + i] != w.y_state[rp]) {
    w.t_mtail[rp] = 0;  // (plain stores of the same value)
  }
  w.t_trep[a + i] = t;
}
// chain starts (a member that does not continue the chain of the member before it)
__global__ __launch_bounds__(256) void k_thuge_flags(Work w, uint32_t a, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  if (i == n) { w.t_flag[i] = 0; return; }
  const bool link = i > 0 && w.y_confl[a + i] == a + i - 1 && w.y_state[a + i] == w.y_state[a + i - 1] &&
                    w.t_mtail[a + i - 1] == NONE;
  w.t_flag[i] = link ? 0u : 1u;
}
// node numbering: t_prv[a + i] = node of position i, t_next[a + k] = first position of node k
__global__ __launch_bounds__(256) void k_thuge_nodes(Work w, uint32_t a, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* pre = w.t_flag + n + 1;  // exclusive scan of the flags
  const uint32_t k = pre[i] + w.t_flag[i] - 1;
  w.t_prv[a + i] = k;
  if (w.t_flag[i]) w.t_next[a + k] = i;
}
// the loop over the nn collapsed chains (nn <= TLDS) on one lane, the chains staged in LDS; each
// chain's successor in the sibling order goes to t_mprv[a + k] (NONE: last), the first to head
__global__ __launch_bounds__(256) void k_thuge_loop(Work w, uint32_t a, uint32_t n) {
  __shared__ SibRec rec[TLDS];
  __shared__ uint8_t st[TLDS];
  __shared__ uint16_t stk[TLDS];  // the loop's stack
  __shared__ uint32_t head_s;
  const uint32_t nn = w.t_flag[n + 1 + n];
  if (nn > TLDS) return;  // k_thuge_inplace
  const uint32_t* node = w.t_prv + a;
  const uint32_t* nfirst = w.t_next + a;
  for (uint32_t k = threadIdx.x; k < nn; k += blockDim.x) {
    const uint32_t f = nfirst[k];
    const uint32_t rp = w.y_confl[a + f];
    const uint32_t t = w.t_trep[a + f];
    const uint32_t tq = node[(t & 0x7FFFFFFFu) - a];
    rec[k] = SibRec{w.y_state[a + f], (uint16_t)(rp == NONE ? S_NONE : node[rp - a]),
                    (uint16_t)(tq | ((t >> 31) ? TOUT : 0u)), S_NONE, S_NONE, S_NONE, S_NONE, S_NONE, 0};
    st[k] = 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    SibLds acc{rec, st};
    head_s = sib_loop(acc, nn, stk, &w.ctr->err, w.dbg);
    w.t_flag[2 * n + 2] = head_s;  // (read by the expansion)
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < nn; k += blockDim.x) {
    const uint32_t x = rec[k].nxt;
    w.t_mprv[a + k] = x == S_NONE ? NONE : x;
  }
}
// expansion: node k spans positions nfirst[k] .. nfirst[k + 1] - 1, listed from the last down
__global__ __launch_bounds__(256) void k_thuge_expand(Work w, uint32_t a, uint32_t n, uint32_t nsegs) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nn = w.t_flag[n + 1 + n];
  if (nn > TLDS || i >= n) return;
  const uint32_t* node = w.t_prv + a;
  const uint32_t* nfirst = w.t_next + a;
  auto leftmost = [&](uint32_t k) { return (k + 1 < nn ? nfirst[k + 1] : n) - 1; };
  const uint32_t k = node[i], f = nfirst[k];
  uint32_t nx;
  if (i > f) nx = i - 1;
  else {
    const uint32_t kn = w.t_mprv[a + k];
    nx = kn == NONE ? NONE : leftmost(kn);
  }
  w.t_nsib[w.t_seg[a + i]] = nx == NONE ? NONE : w.t_seg[a + nx];
  if (i == 0) {
    const uint32_t head = w.t_flag[2 * n + 2];
    if (head != NONE) sib_publish(w, a, n, nsegs, leftmost(head));
  }
}
// too many chains for LDS: restore the scratch and run the loop in place over the group (one lane)
__global__ __launch_bounds__(256) void k_thuge_inplace(Work w, uint32_t a, uint32_t n, uint32_t nsegs) {
  __shared__ uint32_t head_s;
  const uint32_t nn = w.t_flag[n + 1 + n];
  if (nn <= TLDS) return;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    w.t_mtail[a + i] = NONE;
    w.t_prv[a + i] = NONE;
    w.t_next[a + i] = NONE;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    SibGlobal acc{w, a};
    head_s = sib_loop(acc, n, w.y_stack + a, &w.ctr->err);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t x = w.t_next[a + i];
    w.t_nsib[w.t_seg[a + i]] = x == NONE ? NONE : w.t_seg[x];
  }
  if (threadIdx.x == 0 && head_s != NONE) sib_publish(w, a, n, nsegs, head_s);
}
void launch_tsib_huge(const Work& w, uint32_t a, uint32_t n, uint32_t nsegs, hipStream_t s) {
  uint32_t P = 64;  // load < 2/3, within the 2 nsegs + 4 slots of t_hkey / t_hval (P > n always)
  while (P < n + n / 2 + 1 && 2ull * P <= 2ull * nsegs + 4) P <<= 1;
  fill_u32_multi({{w.t_hkey, P, NONE}, {w.t_hval, P, NONE}}, s);
  const uint32_t grid = n / 256 + 1;
  hipLaunchKernelGGL(k_thuge_init, dim3(grid), dim3(256), 0, s, w, a, n);
  hipLaunchKernelGGL(k_thuge_hash, dim3(grid), dim3(256), 0, s, w, a, n, P);
  hipLaunchKernelGGL(k_thuge_anchor, dim3(grid), dim3(256), 0, s, w, a, n, P);
  hipLaunchKernelGGL(k_thuge_flags, dim3(grid), dim3(256), 0, s, w, a, n);
  scan_u32(w.tmp, w.tmp_bytes, w.t_flag, w.t_flag + n + 1, n + 1, s);  // [n + 1 + n] = the chain count
  hipLaunchKernelGGL(k_thuge_nodes, dim3(grid), dim3(256), 0, s, w, a, n);
  hipLaunchKernelGGL(k_thuge_loop, dim3(1), dim3(256), 0, s, w, a, n);
  hipLaunchKernelGGL(k_thuge_expand, dim3(grid), dim3(256), 0, s, w, a, n, nsegs);
  hipLaunchKernelGGL(k_thuge_inplace, dim3(1), dim3(256), 0, s, w, a, n, nsegs);
}

// Pre-order successor: the first child, else the next sibling of the nearest ancestor-or-self that
// has one. "The nearest ancestor-or-self with a next sibling" is found by pointer jumping in rounds
// (Wyllie): every array segment holds (ans, nxt) — ans its answer once known, nxt the next ancestor
// to look at — and a round replaces an open pair by its nxt's pair: ans = ans[nxt], nxt =
// nxt[nxt] while that is still open. The distance to the answer halves every round, so a path of
// d only-children closes in at most ceil(log2 d) rounds; each round is a coalesced pass, where the
// lane-serial climb with path halving it replaces walked C3's long push chains at memory latency
// (4.7 ms). A round launched after the last open pair closed returns at once (its predecessor's
// "open" word is zero).
constexpr uint32_t CLIMB_ROUNDS = 34;  // > log2 of any segment count, +1 (<= Counters::climb_open)
// The (answer, next) pair of a segment is one 64-bit word, jumped IN PLACE: a segment's word is
// written only by its own lane, with one 8-byte store, and a lane reading its next's word (one
// 8-byte load) sees either its old or its new pair — both states of the same climb — so a round
// only ever moves a pair further up its chain and no second buffer (nor a copy round) is needed.
// Closed pairs are read and skipped. A fixed grid strides over the segments: a round launched
// after convergence is a few thousand workgroups that read one word and return (one workgroup per
// 256 segments, C4's 27 such rounds cost 70 us each in dispatch alone).
// The first round builds the pairs from the sibling links and jumps once: a segment's initial pair
// is (next sibling, NONE), or (NONE, parent) without one (parent NONE: a child of the list's root);
// its parent's initial pair comes from the same links (no separate init pass).
__device__ __forceinline__ uint2 climb_pair0(const Work& w, uint32_t s) {
  const bool arr = (w.g_flags[s] & SEG_ARRAY) != 0;
  const uint32_t ns = arr ? w.t_nsib[s] : NONE;
  return make_uint2(ns, arr && ns == NONE ? w.t_jump[s] : NONE);
}
__global__ __launch_bounds__(256) void k_tclimb_first(Work w, uint32_t nsegs, uint2* __restrict__ cl, uint32_t* __restrict__ open) {
  const uint32_t stride = gridDim.x * blockDim.x;
  bool any_open = false;
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nsegs; s += stride) {
    uint2 v = climb_pair0(w, s);
    if (v.y != NONE) {
      const uint2 u = climb_pair0(w, v.y);
      v = u.x != NONE ? make_uint2(u.x, NONE) : make_uint2(NONE, u.y);
    }
    cl[s] = v;
    any_open |= v.y != NONE;
  }
  wave_flag(&open[0], any_open);
}
constexpr uint32_t CLIMB_GRID = 4096;
__global__ __launch_bounds__(256) void k_tclimb_round(uint32_t nsegs, uint2* __restrict__ cl, uint32_t* __restrict__ open, uint32_t round) {
  if (round > 0 && __hip_atomic_load(&open[round - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;  // converged
  const uint32_t stride = gridDim.x * blockDim.x;
  // (the pair is read and written as ONE 64-bit atomic: as a uint2 the compiler split the read of
  // the next's pair into two 32-bit loads, and a torn (old answer, new next) pair closed a climb
  // with no answer)
  unsigned long long* w64 = (unsigned long long*)cl;
  bool any_open = false;
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nsegs; s += stride) {
    const unsigned long long v = __hip_atomic_load(&w64[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t vn = (uint32_t)(v >> 32);
    if (vn == NONE) continue;  // closed (ans == the answer)
    const unsigned long long u = __hip_atomic_load(&w64[vn], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t ua = (uint32_t)u, un = (uint32_t)(u >> 32);
    const unsigned long long nv = ua != NONE ? ((unsigned long long)NONE << 32) | ua : ((unsigned long long)un << 32) | NONE;
    __hip_atomic_store(&w64[s], nv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    any_open |= ua == NONE && un != NONE;
  }
  wave_flag(&open[round], any_open);
}
__global__ __launch_bounds__(256) void k_tclimb_done(Work w, uint32_t nsegs, const uint2* __restrict__ cl, const uint32_t* __restrict__ open) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s == 0 && open[CLIMB_ROUNDS - 1]) raise_err(&w.ctr->err, ERR_DECODE);  // still open: an origin cycle
  if (s >= nsegs || !(w.g_flags[s] & SEG_ARRAY)) return;
  const uint32_t fc = w.t_first[s];
  w.g_right[s] = fc != NONE ? fc : cl[s].x;
}
void launch_tclimb(const Work& w, uint32_t nsegs, hipStream_t s) {
  const uint32_t grid = nsegs / 256 + 1;
  // the pairs live in the anchor-hash scratch (2 NS + 4 words), free once the groups are ordered
  uint2* cl = (uint2*)w.t_hkey;
  uint32_t* open = w.ctr->climb_open;
  const uint32_t rgrid = std::min<uint32_t>(grid, CLIMB_GRID);
  hipMemsetAsync(open, 0, sizeof(uint32_t) * CLIMB_ROUNDS, s);  // the per-round "pairs still open" words
  hipLaunchKernelGGL(k_tclimb_first, dim3(rgrid), dim3(256), 0, s, w, nsegs, cl, open);
  // rounds in batches of CLIMB_BATCH, with a look at the last round's word between batches: the
  // converged rounds of one long batch were launched faster than they ran (15 us of dispatch gap
  // each, 0.4 ms per C4 merge), a look costs one synchronisation
  constexpr uint32_t CLIMB_BATCH = 8;
  for (uint32_t r = 1; r < CLIMB_ROUNDS;) {
    const uint32_t r1 = std::min(r + CLIMB_BATCH, CLIMB_ROUNDS);
    for (; r < r1; ++r) hipLaunchKernelGGL(k_tclimb_round, dim3(rgrid), dim3(256), 0, s, nsegs, cl, open, r);
    if (r >= CLIMB_ROUNDS) break;
    uint32_t still = 1;
    hipMemcpyAsync(&still, &open[r - 1], sizeof(uint32_t), hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    if (!still) break;
  }
  hipLaunchKernelGGL(k_tclimb_done, dim3(grid), dim3(256), 0, s, w, nsegs, cl, open);
}

uint32_t launch_yata_tree(const Work& w, uint32_t nsegs, hipStream_t s, hipStream_t side, hipEvent_t ev_fork, hipEvent_t ev_join) {
  const uint32_t grid = nsegs / 256 + 1;
  hipLaunchKernelGGL(k_tkey, dim3(grid), dim3(256), 0, s, w, nsegs);
  sort_pairs_u32(w.tmp, w.tmp_bytes, w.t_key, w.t_keys, w.y_iota, w.t_seg, nsegs, s);
  hipLaunchKernelGGL(k_tgroup_flags, dim3(grid), dim3(256), 0, s, w, nsegs);
  scan_u32(w.tmp, w.tmp_bytes, w.t_done, w.t_next, nsegs + 1, s);
  hipMemsetAsync(&w.ctr->tbig, 0, sizeof(uint32_t), s);
  hipLaunchKernelGGL(k_tgroup_starts, dim3(grid), dim3(256), 0, s, w, nsegs);
  hipLaunchKernelGGL(k_tprep, dim3(grid), dim3(256), 0, s, w, nsegs);
  hipLaunchKernelGGL(k_tsib_small, dim3(nsegs / TS_BLOCK + 1), dim3(TS_BLOCK), 0, s, w, nsegs);
  // the big-group count and the huge groups' (start, size) in ONE synchronisation
  std::vector<uint32_t> desc(2 + 2 * (size_t)HUGE_DESC_MAX);
  uint32_t nbig = 0;
  hipMemsetAsync(w.t_hkey, 0, sizeof(uint32_t), s);
  hipLaunchKernelGGL(k_tbig_desc, dim3(std::min<uint32_t>(grid, 256)), dim3(256), 0, s, w, w.t_hkey);
  hipMemcpyAsync(&nbig, &w.ctr->tbig, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
  hipMemcpyAsync(desc.data(), w.t_hkey, sizeof(uint32_t) * desc.size(), hipMemcpyDeviceToHost, s);
  hipStreamSynchronize(s);
  const uint32_t nhuge = desc[0];
  if (nhuge > HUGE_DESC_MAX) {
    desc.resize(2 + 2 * (size_t)nhuge);
    hipMemcpy(desc.data(), w.t_hkey, sizeof(uint32_t) * desc.size(), hipMemcpyDeviceToHost);
  }
  // The huge groups (> TLDS members; t_hkey turns into their hash table now that the descriptors
  // are read) on the side stream, BESIDE the wavefront / workgroup groups: their loop is one
  // workgroup on one CU (C3's list head: 2.7 ms) and the groups are independent.
  if (nhuge) {
    hipEventRecord(ev_fork, s);
    hipStreamWaitEvent(side, ev_fork, 0);
    for (uint32_t k = 0; k < nhuge; ++k) launch_tsib_huge(w, desc[2 + 2 * k], desc[3 + 2 * k], nsegs, side);
    hipEventRecord(ev_join, side);
  }
  if (nbig) {
    hipLaunchKernelGGL(k_tsib_wave, dim3((nbig + 3) / 4), dim3(256), 0, s, w, nsegs, nbig);
    hipLaunchKernelGGL((k_tsib_big<TMID, 2048, true>), dim3(nbig), dim3(256), 0, s, w, nsegs);
    hipLaunchKernelGGL((k_tsib_big<TLDS, THASH, false>), dim3(nbig), dim3(256), 0, s, w, nsegs);
  }
  if (nhuge) hipStreamWaitEvent(s, ev_join, 0);
  launch_tclimb(w, nsegs, s);
  return nbig;
}

// The YArray lists numbered (members sorted by (list, segment), y_lstart): the view's list table
// and the sequential kernels' work list. The parallel tree path does not need it, so a merge
// without a view skips it (one sort and a host sync: 1.4 ms of C4's merge).
uint32_t launch_ylists(const Work& w, uint32_t nsegs, hipStream_t s) {
  if (!nsegs) return 0;
  const uint32_t grid = nsegs / 256 + 1;
  hipLaunchKernelGGL(k_ykey, dim3(grid), dim3(256), 0, s, w, nsegs);
  sort_pairs_u32(w.tmp, w.tmp_bytes, w.y_key, w.y_keys, w.y_iota, w.y_seg, nsegs, s);
  hipLaunchKernelGGL(k_ylist_flags, dim3(grid), dim3(256), 0, s, w, nsegs);
  scan_u32(w.tmp, w.tmp_bytes, w.y_before, w.y_confl, nsegs + 1, s);
  uint32_t nlists = 0;
  hipMemcpyAsync(&nlists, w.y_confl + nsegs, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
  hipStreamSynchronize(s);
  if (nlists) hipLaunchKernelGGL(k_ylist_starts, dim3(grid), dim3(256), 0, s, w, nsegs);
  return nlists;
}

// Returns the list count, or LISTS_UNNUMBERED when the tree path ran without numbering them
// (launch_ylists, when a view asks).
uint32_t launch_yata(const Work& w, uint32_t nsegs, uint32_t narray, uint32_t nclients, hipStream_t s, hipStream_t side,
                     hipEvent_t ev_fork, hipEvent_t ev_join) {
  if (!nsegs) return 0;
  if (!narray) return 0;  // g_right is only read for YArray members (merge predicate, view)
  hipLaunchKernelGGL(k_yinit, dim3(nsegs / 256 + 1), dim3(256), 0, s, w, nsegs);
  static const bool seq = getenv("YCRDT_YATA") && !strcmp(getenv("YCRDT_YATA"), "seq");
  if (!seq && (uint64_t)nsegs * 5 < 0xFFFFFFF0ull) {  // sibling keys NS + list slot stay below NONE
    static const bool eager = getenv("YCRDT_YLISTS_EAGER") && getenv("YCRDT_YLISTS_EAGER")[0] == '1';
    const uint32_t nl = eager ? launch_ylists(w, nsegs, s) : LISTS_UNNUMBERED;
    launch_yata_tree(w, nsegs, s, side, ev_fork, ev_join);
    return nl;
  }
  const uint32_t nlists = launch_ylists(w, nsegs, s);
  if (!nlists) return 0;
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
