// yc_engine.hip — host orchestration of the batched merge + the C ABI (include/ycrdt.h).
//
// One engine = one HIP device + one stream + a grow-only set of HBM buffers. A merge runs the
// decode → dedupe → delete-set → segmentation → map-winner → encode kernels back to back on the
// engine stream; the host only reads a handful of counters at the sync points where the next
// phase's size depends on data (struct count, unit count, segment count, output bytes).
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <unordered_map>
#include <unordered_set>
#include <algorithm>
#include <memory>
#include <functional>

#include "yc_work.h"
#include "yc_host.h"
#include "yc_ingest.h"
#include "yc_comm.h"
#include <thread>
#include <atomic>
#include "../../include/ycrdt.h"

using namespace yc;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(x)                                                                                    \
  do {                                                                                               \
    hipError_t _e = (x);                                                                             \
    if (_e != hipSuccess) return fail(YCRDT_E_DEVICE, std::string("HIP error: ") + hipGetErrorString(_e) + " at " #x); \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool arena = false;  // a block of the engine's doc-state arena (Arena::release), not a hipMalloc
};

// Doc states live in an engine-owned HBM arena: 64 MiB slabs carved into power-of-two blocks
// (256 B .. 1 MiB) with a free list per size class; larger states get their own hipMalloc. A fleet
// of 100k+ small documents then costs a few slab allocations instead of one hipMalloc per doc.
struct Arena {
  static constexpr size_t MIN_SHIFT = 8, MAX_SHIFT = 20, SLAB = size_t(64) << 20;
  std::vector<void*> slabs;
  std::vector<void*> free_[MAX_SHIFT - MIN_SHIFT + 1];
  uint8_t* cur = nullptr;
  size_t left = 0;
  static int cls(size_t bytes) {
    int c = 0;
    while ((size_t(1) << (MIN_SHIFT + c)) < bytes) ++c;
    return c;
  }
  void* alloc(size_t bytes, size_t& cap) {
    const int c = cls(bytes);
    cap = size_t(1) << (MIN_SHIFT + c);
    if (!free_[c].empty()) { void* p = free_[c].back(); free_[c].pop_back(); return p; }
    if (left < cap) {
      void* s = nullptr;
      if (hipMalloc(&s, SLAB) != hipSuccess) return nullptr;
      slabs.push_back(s);
      cur = (uint8_t*)s;
      left = SLAB;  // the tail of the previous slab (< one block) is abandoned
    }
    void* p = cur;
    cur += cap;
    left -= cap;
    return p;
  }
  void release(void* p, size_t cap) { free_[cls(cap)].push_back(p); }
  ~Arena() { for (void* s : slabs) hipFree(s); }
};

thread_local size_t g_failed_alloc = 0;  // the request of the last failed hipMalloc (error messages)
bool grow(DevBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (bytes <= b.cap) return true;
  if (b.p) hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  // 25 % headroom for the next batch; past 1 GiB (billion-item merges, where the workspace is a
  // large share of HBM) 3 %
  size_t c = bytes + (bytes > (size_t(1) << 30) ? bytes / 32 : bytes / 4) + 256;
  if (hipMalloc(&b.p, c) != hipSuccess) {
    (void)hipGetLastError();
    if (hipMalloc(&b.p, bytes + 256) != hipSuccess) {  // without the headroom
      (void)hipGetLastError();
      b.p = nullptr;
      g_failed_alloc = bytes;
      return false;
    }
    c = bytes + 256;
  }
  b.cap = c;
  return true;
}
thread_local const std::vector<DevBuf>* g_bufs = nullptr;  // the workspace of the merge in progress (oom reports)
// "hipMalloc failed (what)" with the request, the device's free / total memory and the largest
// workspace buffers held at that point (buffer index: the Buf enum below)
std::string oom(const char* what) {
  size_t fr = 0, tot = 0;
  (void)hipMemGetInfo(&fr, &tot);
  char buf[256];
  snprintf(buf, sizeof buf, "hipMalloc failed (%s): request %.2f GB, device free %.2f of %.2f GB", what,
           g_failed_alloc / 1e9, fr / 1e9, tot / 1e9);
  std::string r = buf;
  if (g_bufs) {
    std::vector<std::pair<size_t, size_t>> big;
    size_t sum = 0;
    for (size_t i = 0; i < g_bufs->size(); ++i) {
      sum += (*g_bufs)[i].cap;
      big.emplace_back((*g_bufs)[i].cap, i);
    }
    std::sort(big.rbegin(), big.rend());
    snprintf(buf, sizeof buf, "; workspace %.2f GB, largest (buffer:GB)", sum / 1e9);
    r += buf;
    for (size_t k = 0; k < big.size() && k < 8; ++k) {
      snprintf(buf, sizeof buf, " %zu:%.2f", big[k].second, big[k].first / 1e9);
      r += buf;
    }
  }
  return r;
}

template <class T>
T* take(std::vector<DevBuf>& v, size_t idx, size_t n, bool& ok) {
  if (v.size() <= idx) v.resize(idx + 1);
  if (!grow(v[idx], n * sizeof(T))) { ok = false; return nullptr; }
  return (T*)v[idx].p;
}

uint32_t next_pow2(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return (uint32_t)std::min<uint64_t>(p, 1ull << 31);
}

// decode a state vector (varuint n, (client, clock) × n)
bool parse_sv(const uint8_t* p, size_t n, std::unordered_map<uint32_t, uint32_t>& out) {
  size_t pos = 0;
  auto vu = [&](uint32_t& v) -> bool {
    uint32_t r = 0;
    int shift = 0;
    for (;;) {
      if (pos >= n) return false;
      uint32_t b = p[pos++];
      if (shift < 32) r |= (b & 0x7fu) << shift;
      shift += 7;
      if (b < 0x80) { v = r; return true; }
      if (shift > 35) return false;
    }
  };
  uint32_t k;
  if (!vu(k)) return false;
  for (uint32_t i = 0; i < k; ++i) {
    uint32_t c, cl;
    if (!vu(c) || !vu(cl)) return false;
    out[c] = cl;
  }
  return true;
}

enum Buf {
  B_BYTES, B_META, B_CTR, B_SPECB, B_CEXIT, B_SEXIT, B_FINAL, B_SECB,
  B_DSSTART, B_SECT, B_SECSORT,
  B_WCNT, B_WSEC, B_DS, B_DSTMP, B_DSREG, B_DSCNT, B_DSOFF, B_DSLEN, B_DSSCAN, B_SCRATCH, B_TMP,
  B_SPOS, B_SSEC, B_SLEN, B_SLENSCAN, B_SCLOCK, B_SCIDX, B_SINFO, B_SOC, B_SOK, B_SRC, B_SRK, B_SPA, B_SPB, B_SPS, B_SPL,
  B_SCPOS, B_SCEND, B_SCELEM,
  B_CLVALS, B_CLTMP, B_CLSTATE, B_CLBASE, B_CLSTART, B_CC, B_CC64, B_SWIN,
  B_UOWN, B_UFLAG, B_UCUT, B_UWPRE,
  B_GSTART, B_GCIDX, B_GSRC, B_GFLAGS, B_GORIG, B_GRORIG, B_GLINK, B_GOSEG, B_GKEY, B_GMAXC, B_GNEXT, B_GOUTID, B_GTMP, B_GTMP2,
  B_KHASH, B_KROOT, B_KWIN, B_KPAR, B_KFLAG, B_SPK,
  B_USEC, B_USECN, B_DBG, B_XTAB, B_UFAIL, B_FW, B_CCNT, B_TENTRY, B_XLIST, B_WLEN, B_FWSEC, B_DSPCNT, B_DSPPRE, B_DSPVAL, B_DSPBLK, B_DSPB, B_DSPNB, B_DSPFAIL, B_DSPGB, B_OGEN, B_SDDEFER, B_COFF, B_CPRE, B_OPRE, B_SECUEND, B_SECDOC, B_DSBIGL, B_DSTAILS, B_FWC, B_FWCOFF, B_RTAB, B_RK, B_DSHJ, B_DSHS, B_DSHH, B_JLIST, B_JITEM, B_JARENA, B_JOFF, B_JOUT,
  B_LZKEY, B_LZKEYS, B_LZIOTA, B_LZSEC, B_LZRSTART, B_LZPREV, B_LZFIRST, B_LZCAP, B_LZEVBASE, B_LZEVN, B_LZFLAG,
  B_LZLHI, B_LZLLO, B_EVKIND, B_EVSRC, B_EVCLOCK, B_EVLEN, B_EVSIZE, B_EVPOS, B_BLKSIZE, B_BLKPOS, B_SVC, B_SVK,
  B_DSMKEY, B_DSMKEYS, B_DSMLEN, B_DSMLENS, B_DSMEND, B_DSMMAX, B_DSMFLAG, B_DSMRID, B_DRCLIENT, B_DRCLOCK, B_DREND,
  B_DWFLAG, B_DWGID, B_DWGSTART, B_DWSIZE, B_DWPOS,
  B_GRIGHT, B_YKEY, B_YKEYS, B_YSEG, B_YIOTA, B_YLSTART, B_YSTATE, B_YBEFORE, B_YCONFL, B_YSTACK,
  B_TKEY, B_TKEYS, B_TSEG, B_TPOS, B_TGSTART, B_TNEXT, B_TDONE, B_TFIRST, B_TNSIB, B_TJUMP, B_TBIG,
  B_TPRV, B_TMPRV, B_TMTAIL, B_TTREP, B_TOTAIL, B_THKEY, B_THVAL, B_TFLAG, B_TSCAN, B_SENT,
  B_OFIRST, B_OCIDX, B_OSIZE, B_OPOS, B_RSEG, B_RLEN, B_RSIZE, B_RPOS, B_OUT, B_SVOUT,
  B_VKMAP, B_VKREP, B_VKEYS, B_VNKEYS, B_VPOS, B_VD0, B_VN0, B_VD1, B_VN1, B_VORDER, B_VSEGS,
  B_SCRATCH2, B_TMP2, B_CAPS, B_CLKEY, B_CLKEY2, B_CHKEY, B_CHVAL, B_CLDOC, B_DSFA, B_EMIT, B_DOCRNG, B_PACK, B_PACKPC, B_SPLITMETA, B_CLSINGLE, B_KSHARD, B_SOWNER, B_GFLAGS0, B_GFACC, B_LZBCLIENT,
  B_COUNT
};

}  // namespace

struct Pinned {
  uint8_t* p = nullptr;
  size_t cap = 0;
  hipEvent_t ev[2] = {nullptr, nullptr};
};
constexpr uint64_t PIN_SV = uint64_t(1) << 20;  // pinned state-vector read-back of a small merge
struct ycrdt_engine {
  int device = 0;
  int compat = 136;
  hipStream_t stream = nullptr;
  ycrdt_batch* scratch = nullptr;    // staging batch of the one-shot calls (apply / encode / merge / diff)
  hipStream_t side = nullptr;        // delete-set decode overlaps the client table / struct decode
  hipEvent_t side_done = nullptr, side_fork = nullptr;
  std::vector<DevBuf> bufs;
  Work w;
  bool profiling = false;
  bool debug_sync = false;
  std::vector<std::pair<const char*, hipEvent_t>> marks;  // this merge's phase marks
  std::vector<hipEvent_t> event_pool;                     // reused across merges (no create per mark)
  std::vector<std::pair<const char*, double>> phase_ms;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // pinned host staging (two halves of PIN_PER chunks: the copy of one wave into a half overlaps
  // the copy of the previous wave from the other) and its per-half "copy done" events: one area
  // for batch staging (H2D, on the copy stream) and one for results (D2H, on the engine stream),
  // so a batch can be staged by one host thread while another merges the previous batch
  Pinned pin_in, pin_out;
  // pinned read-back areas of the sync points (a copy into pageable memory goes through the
  // runtime's staging: ~20-30 us per copy on the per-op path): the counters, and a small view
  Counters* ctr_pin = nullptr;
  uint8_t* sv_pin = nullptr;  // [PIN_SV] a small merge's state vector
  uint8_t* rb = nullptr;
  size_t rb_cap = 0;
  // commit_merge's copies (the merged state into the doc's block, the state vector out), queued by
  // run_merge before its last synchronisation so that one wait covers the merge and the copies
  // (cap_out, cap_sv: the bounds the outputs were sized by)
  const std::function<int(uint64_t cap_out, uint64_t cap_sv)>* before_final = nullptr;
  hipStream_t copy = nullptr;  // batch staging (host → HBM)
  hipEvent_t copy_dep = nullptr;
  // result of the last merge (e->w.out / e->w.sv_out): ws_owner is the batch that produced it
  // (nullptr after any other call), so ycrdt_batch_result never returns another call's bytes
  const void* ws_owner = nullptr;
  uint64_t out_bytes = 0;
  uint32_t sv_bytes = 0;
  uint32_t nsegs = 0, nlists = 0;  // segments / YArray lists of the last merge (the view reads them)
  ycrdt_merge_stats last{};
  Arena arena;                      // doc states (alloc_state / release_state)
  std::unordered_set<ycrdt_doc*> docs;  // live docs (ycrdt_engine_trim releases their spare blocks)
};

// a fresh doc state block of at least `bytes` (arena block, or its own hipMalloc when large)
bool alloc_state(ycrdt_engine* e, DevBuf& b, size_t bytes) {
  b = DevBuf();
  if (bytes == 0) bytes = 16;
  if (bytes <= (size_t(1) << Arena::MAX_SHIFT)) {
    b.p = e->arena.alloc(bytes, b.cap);
    b.arena = b.p != nullptr;
    if (!b.p) b.cap = 0;
    return b.p != nullptr;
  }
  return grow(b, bytes);
}
void release_state(ycrdt_engine* e, DevBuf& b) {
  if (b.p) { if (b.arena) e->arena.release(b.p, b.cap); else hipFree(b.p); }
  b = DevBuf();
}
struct ycrdt_doc {
  ycrdt_engine* e = nullptr;
  uint32_t client_id = 0;
  DevBuf state;          // canonical encoded state (Yjs v1 update) in HBM
  DevBuf spare;          // the previous state's block, reused by the next folded merge (commit_merge)
  size_t state_len = 0;  // 0 = empty doc
  std::vector<uint8_t> sv;
  ycrdt_merge_stats last{};
  HostView view;         // materialised view of `state` (crdt.c), rebuilt lazily after a change
  bool wants_view = false;  // a view was read once: build it beside every merge (crdt.js reads after each op)
  // Y.applyUpdate is deferred: validated updates wait here and are merged in one
  // batch by the next read (encode*, toJSON, get, local op). n sequential applies cost one merge.
  struct Queued { std::vector<uint8_t> bytes; bool local; bool ds_error = false; int32_t nst = -1, nsec = -1; };  // ds_error: read_update; nst / nsec: the scan's counts
  std::vector<Queued> queue;
  size_t queue_bytes = 0;
  IngestState ing;       // Yjs pendingStructs / pendingDs / store client order (yc_ingest.h)
  // the decode of `state`, written by the encode that produced it (k_state_marks): the next merge of
  // the doc reads its state's struct / section starts from here instead of parsing it (k_predecoded;
  // YCRDT_PREDECODE=0: off, =check: decoded both ways and compared). marks_len: the state length the
  // marks describe (0: none)
  DevBuf marks;
  size_t marks_len = 0;
  uint32_t marks_nw = 0, marks_cap = 0;
  bool track_local = false;                 // ycrdt_doc_track_local: record local-op updates
  std::vector<std::vector<uint8_t>> local;  // local-op updates since the last ycrdt_doc_take_local_update
  size_t local_bytes = 0;
};

struct ycrdt_batch {
  ycrdt_engine* e = nullptr;
  DevBuf bytes, meta, pieces;
  std::vector<uint32_t> uoff, ulen, ugroup;  // uoff: within the update's window (yc_work.h WIN_SHIFT)
  std::vector<uint32_t> uwin;   // window of every staged update
  uint32_t nwin = 1;
  uint32_t win_shift = WIN_SHIFT;
  size_t uwin_off = 0;          // byte offset of uwin in `meta` (multi-window batches)
  std::vector<uint32_t> udoc;   // multi-document batch: document of every staged update
  uint32_t ndocs = 1;
  size_t udoc_off = 0;          // byte offset of udoc in `meta`
  std::vector<uint32_t> ulist;  // updates parsed through the chain tables, then the direct ones
  uint32_t nbig = 0;
  uint32_t schunk = SCHUNK;     // chunk bytes of the large updates (layout)
  size_t ulist_off = 0;
  std::vector<Group> groups;
  // record mode of the multi-section fast walk (yc_decode.hip k_fwc): per staged update, the base of
  // its records (one per byte) or NONE; fwc_recs records in all
  std::vector<uint32_t> fwc_off;
  uint64_t fwc_recs = 0;
  // a source decoded by its own encode (a doc state with PreMarks): its index among the sources
  // (-1: none), the marks, whether to check them against a real decode instead, its update index
  int pre_src = -1;
  PreMarks pre;
  bool pre_check = false;
  uint32_t pre_u = 0;
  // updates rewritten with their JSON-like contents in JSON.stringify's form (json_rewrite): the
  // host copies the batch was re-staged from, and the rewrite passes so far
  std::vector<std::vector<uint8_t>> jstore;
  uint32_t jpasses = 0;
  uint32_t ntrusted = 0;        // leading staged updates that are doc states the engine wrote (device sources)
  bool walk_only = false;       // every large update is the doc state or pre-walked whole (layout): no chunk walk
  uint64_t nbytes = 0;          // span of the batch buffer (windows before the last are 2^32 bytes)
  uint64_t in_bytes = 0;
  bool merged = false;
  // per-document split of a merged multi-document batch (ycrdt_batch_result_docs_packed):
  // doc d's update = packed[offs[2d], offs[2d+1]), its state vector = [offs[2d+1], offs[2d+2])
  bool packed = false;
  std::vector<uint64_t> pack_offs;
};

namespace {

ycrdt_batch& scratch_batch(ycrdt_engine* e) {
  if (!e->scratch) {
    e->scratch = new ycrdt_batch();
    e->scratch->e = e;
  }
  return *e->scratch;
}

void mark(ycrdt_engine* e, const char* name) {
  if (e->debug_sync) {  // YCRDT_DEBUG_SYNC=1: attribute a device fault to the phase that raised it
    const hipError_t er = hipStreamSynchronize(e->stream);
    if (er != hipSuccess) fprintf(stderr, "[ycrdt] device error before phase %s: %s\n", name, hipGetErrorString(er));
  }
  if (!e->profiling) return;
  if (e->marks.size() == e->event_pool.size()) {
    hipEvent_t ev;
    if (hipEventCreate(&ev) != hipSuccess) return;
    e->event_pool.push_back(ev);
  }
  hipEvent_t ev = e->event_pool[e->marks.size()];
  hipEventRecord(ev, e->stream);
  e->marks.push_back({name, ev});
}

// Small updates are parsed directly, one lane per update walking its structs exactly, when there
// are many of them: a wavefront then parses 64 updates side by side and the batch is read about
// once. A few small updates, and every large one, take the chunk path (k_spec / k_walk), whose
// latency grows with the update only by one wavefront step per 64 KiB. YCRDT_DECODE=chunks|direct
// forces one path for small updates (tests cover both; "tables" is the older name of "chunks");
// xtab = chunks, and every large update walked through the exit tables (yc_decode.hip k_xtab).
constexpr size_t DIRECT_MAX_BYTES = 16384;         // an update the direct lane walks whole
constexpr size_t DIRECT_TINY_BYTES = 1024;         // always direct (a handful of structs)
constexpr size_t DIRECT_MIN_COUNT = 1024;          // enough small updates to fill wavefronts
constexpr size_t SMALL_BATCH_BYTES = size_t(1) << 20;  // chunk-path bytes up to which chunks are short
constexpr uint32_t SCHUNK_SMALL = 256;
constexpr size_t MID_BATCH_BYTES = size_t(64) << 20;  // chunk-path bytes up to which chunks are SCHUNK / 2

// One staged input: host bytes, or a device buffer (a doc state already in HBM).
struct Src {
  const uint8_t* p;
  size_t len;
  bool dev;
  int32_t nst = -1, nsec = -1;  // structs / sections, when the host scan of Y.applyUpdate counted them
};

// Lays out the sources (64-byte aligned, so every update owns its bitmap words; device sources
// first, then the host ones in one contiguous region) + decode group table.
void layout(ycrdt_batch* b, const std::vector<Src>& src, std::vector<uint32_t>& order) {
  b->uoff.clear(); b->ulen.clear(); b->ugroup.clear(); b->groups.clear(); b->ulist.clear(); b->uwin.clear();
  b->fwc_off.clear();
  b->fwc_recs = 0;
  b->in_bytes = 0;
  // A large update of many client sections (a full state sent as one update, crdt.js:288,443) gets
  // the record mode of the multi-section fast walk: 16 bytes of records per update byte, so only
  // updates of >= FWC_MIN_SECTIONS sections (read from the host bytes; a doc state in HBM of
  // >= FWC_MIN_BYTES is taken as one) and at most FWC_MAX_RECS records per batch. YCRDT_FWC=0: off.
  constexpr size_t FWC_MIN_BYTES = size_t(64) << 10;
  constexpr uint32_t FWC_MIN_SECTIONS = 16;
  constexpr uint64_t FWC_MAX_RECS = uint64_t(128) << 20;
  // (YCRDT_FWC=force, tests: every large update of two or more sections, however small)
  const char* fwc_env = getenv("YCRDT_FWC");
  const bool fwc_on = !env_off("YCRDT_FWC"), fwc_force = fwc_env && !strcmp(fwc_env, "force");
  // Sections must also be short on average (<= FWC_MAX_SECTION bytes): the step table and the records
  // cost every byte, the walk they replace costs every section — a C3 state's 256 sections of 300 KB
  // each ran 13.7 -> 25.8 ms in record mode (a C2 document's 1 001 sections of 8 KB: 31 -> 4.5 ms)
  constexpr size_t FWC_MAX_SECTION = size_t(64) << 10;
  auto fwc_wants = [&](const Src& x) {
    if (!fwc_on || (x.len < FWC_MIN_BYTES && !fwc_force)) return false;
    if (x.dev) return fwc_force || x.len <= (size_t(32) << 20);  // (a doc state without marks: its sections are unknown here)
    uint32_t q = 0;
    bool okq = true;
    const uint32_t nsec = rd_vu(x.p, q, (uint32_t)std::min<size_t>(x.len, 16), okq);
    if (fwc_force) return okq && nsec >= 2u;
    return okq && nsec >= FWC_MIN_SECTIONS && x.len <= (size_t)nsec * FWC_MAX_SECTION;
  };
  const char* mode = getenv("YCRDT_DECODE");
  const int force = mode && (!strcmp(mode, "chunks") || !strcmp(mode, "tables") || !strcmp(mode, "xtab")) ? 1
                    : mode && !strcmp(mode, "direct") ? 2 : 0;
  // (decoded by k_predecoded; a large one stays in the big list, its chunks serving the grid
  // delete-set decode only; a small one is in neither list)
  constexpr size_t PRE_GROUPS_MIN = size_t(64) << 10;
  const int pre = b->pre_check ? -1 : b->pre_src;
  size_t nsmall = 0;
  for (size_t i = 0; i < src.size(); ++i) nsmall += src[i].len <= DIRECT_MAX_BYTES && (int)i != pre;
  // small updates are parsed directly however few there are: one lane each (k_direct) when they
  // fill wavefronts, else one wavefront each (k_wdecode); YCRDT_DIRECT_WAVE=0 keeps the lane
  // kernel, and then few small updates take the chunk path as before
  const char* wd = getenv("YCRDT_DIRECT_WAVE");
  const bool lane_only = wd && wd[0] == '0';
  auto direct = [&](size_t len) {
    if (len > DIRECT_MAX_BYTES || force == 1) return false;
    return force == 2 || !lane_only || nsmall >= DIRECT_MIN_COUNT || len <= DIRECT_TINY_BYTES;
  };
  // chunk size: a lane walks its chunk serially, so a batch with little chunk-path input (a doc
  // state and a few updates: the per-op path) takes short chunks; big ones the full SCHUNK
  // (short enough that the walker's 64 lanes still span the largest update in one step)
  size_t big_bytes = 0, big_max = 0;
  for (size_t i = 0; i < src.size(); ++i)
    if (src[i].len && ((int)i == pre ? src[i].len > PRE_GROUPS_MIN : !direct(src[i].len))) { big_bytes += src[i].len; big_max = std::max(big_max, src[i].len); }
  b->schunk = SCHUNK;
  if (big_bytes <= SMALL_BATCH_BYTES)
    while (b->schunk > SCHUNK_SMALL && (size_t)(b->schunk / 2) * 64 >= big_max) b->schunk /= 2;
  else if (big_bytes <= MID_BATCH_BYTES)
    b->schunk = SCHUNK / 2;  // a single document's worth: more, shorter chunk chains (the walk is mostly the fast one)
  if (const char* cs = getenv("YCRDT_SCHUNK")) {  // experiments: a fixed chunk size (64-byte multiple)
    const uint32_t v = (uint32_t)atoi(cs);
    if (v >= 64 && v <= SCHUNK && v % 64 == 0) b->schunk = v;
  }
  order.clear();
  for (size_t i = 0; i < src.size(); ++i) if (src[i].dev) order.push_back((uint32_t)i);
  for (size_t i = 0; i < src.size(); ++i) if (!src[i].dev) order.push_back((uint32_t)i);
  std::vector<uint32_t> small;
  b->win_shift = WIN_SHIFT;
  if (const char* ws = getenv("YCRDT_WIN_SHIFT")) {  // tests: small windows (every multi-window path on MBs)
    const int v = atoi(ws);
    if (v >= 20 && v <= 32) b->win_shift = (uint32_t)v;
  }
  const uint64_t wuse = win_use(b->win_shift);
  uint64_t total = 0, win = 0;  // total: bytes used in window `win`
  bool walk_all = true;
  for (const uint32_t i : order) {
    const size_t len = src[i].len, len64 = (len + 63) & ~size_t(63);
    if (total && total + len64 > wuse) { ++win; total = 0; }  // an update never straddles windows
    const uint64_t off = total;
    const uint32_t u = (uint32_t)b->uoff.size();
    b->uoff.push_back((uint32_t)off);
    b->uwin.push_back((uint32_t)win);
    b->ulen.push_back((uint32_t)len);
    b->fwc_off.push_back(NONE);
    if ((int)i == pre) b->pre_u = u;
    if ((int)i == pre && len <= PRE_GROUPS_MIN) {
      // (a small doc state: no chunks at all — its delete set is short, the wavefront decodes it)
      b->ugroup.push_back(NONE);
    } else if (len && direct(len) && (int)i != pre) {
      b->ugroup.push_back(NONE);
      small.push_back(u);
    } else {
      // (a doc state decoded by its marks keeps its chunks for the grid delete-set decode only)
      if ((int)i != pre && fwc_wants(src[i]) && b->fwc_recs + len <= FWC_MAX_RECS) {
        b->fwc_off.back() = (uint32_t)b->fwc_recs;
        b->fwc_recs += (len + 63) & ~size_t(63);
      }
      // (the chunk walk is needed unless every large update is the doc state or one whose struct
      // section the pre-walk takes whole: <= 64 structs in <= 8 sections, as the host scan counted)
      if ((int)i != pre && !(src[i].nst >= 0 && src[i].nst <= 64 && src[i].nsec >= 0 && src[i].nsec <= 8)) walk_all = false;
      b->ugroup.push_back((uint32_t)b->groups.size());
      b->ulist.push_back(u);
      for (size_t g = 0; g < len; g += b->schunk) {
        Group G;
        G.start = (uint32_t)(off + g);
        G.end = (uint32_t)std::min(off + len, off + g + b->schunk);
        G.uend = (uint32_t)(off + len);
        G.upd = u;
        b->groups.push_back(G);
      }
    }
    b->in_bytes += len;
    total += len64;
  }
  b->nbig = (uint32_t)b->ulist.size();
  b->walk_only = walk_all && b->nbig > 0;
  b->ulist.insert(b->ulist.end(), small.begin(), small.end());
  b->uoff.push_back((uint32_t)total);
  b->nwin = (uint32_t)win + 1;
  b->nbytes = (win << b->win_shift) + total;
}
// absolute byte offset of staged update u in the batch buffer
uint64_t uabs(const ycrdt_batch* b, size_t u) { return ((uint64_t)b->uwin[u] << b->win_shift) + b->uoff[u]; }

// Host bytes → HBM through the engine's pinned staging. The span is cut into PIN_CHUNK chunks;
// a wave of up to PIN_PER chunks is filled by worker threads (each chunk: its pieces copied, the
// bytes between them — slot padding, window gaps — zeroed) and sent with one async H2D, while the
// next wave fills the other half of the staging buffer. Small spans: one memcpy on this thread.
struct HostPiece {
  uint64_t off;   // within the span
  uint64_t len;
  const uint8_t* p;
};
constexpr uint32_t PIN_PER = 4;  // 128 MiB waves: the copy of a wave overlaps the transfer of the previous
// 32 MiB; YCRDT_PIN_CHUNK (tests: e.g. 65536) makes the two-half wave path run on small batches
uint64_t pin_chunk() {
  const char* v = getenv("YCRDT_PIN_CHUNK");
  const uint64_t c = v ? strtoull(v, nullptr, 10) : 0;
  return c >= 4096 && c <= (uint64_t(1) << 30) ? c : uint64_t(32) << 20;
}
// copies the pieces overlapping [lo, hi) of the span to dst (= span byte lo), zero elsewhere
void fill_range(uint8_t* dst, uint64_t lo, uint64_t hi, const std::vector<HostPiece>& hp) {
  size_t i = std::upper_bound(hp.begin(), hp.end(), lo, [](uint64_t v, const HostPiece& x) { return v < x.off; }) - hp.begin();
  if (i > 0) --i;
  uint64_t cur = lo;
  for (; i < hp.size() && hp[i].off < hi; ++i) {
    const uint64_t a = std::max(lo, hp[i].off), z = std::min(hi, hp[i].off + hp[i].len);
    if (z <= a) continue;
    if (a > cur) memset(dst + (cur - lo), 0, a - cur);
    memcpy(dst + (a - lo), hp[i].p + (a - hp[i].off), z - a);
    cur = z;
  }
  if (hi > cur) memset(dst + (cur - lo), 0, hi - cur);
}
int ensure_pinned(Pinned& pin, size_t need, hipStream_t s) {
  if (need <= pin.cap) return YCRDT_OK;
  HIPCHK(hipStreamSynchronize(s));
  if (pin.p) hipHostFree(pin.p);
  pin.p = nullptr;
  pin.cap = 0;
  const size_t c = std::max<size_t>(need, size_t(1) << 20);
  if (hipHostMalloc((void**)&pin.p, c, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    pin.p = nullptr;
    return fail(YCRDT_E_DEVICE, "pinned host staging allocation failed");
  }
  pin.cap = c;
  return YCRDT_OK;
}
int h2d_span(ycrdt_engine* e, uint8_t* dev, uint64_t span, const std::vector<HostPiece>& hp) {
  if (!span) return YCRDT_OK;
  Pinned& pin = e->pin_in;
  const hipStream_t s = e->copy;
  const uint64_t PIN_CHUNK = pin_chunk();
  const uint64_t nch = (span + PIN_CHUNK - 1) / PIN_CHUNK;
  const bool waves = nch > PIN_PER;
  if (const int rc = ensure_pinned(pin, waves ? 2 * PIN_PER * PIN_CHUNK : (size_t)span, s)) return rc;
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const uint32_t T = span < (uint64_t(8) << 20) ? 1u : std::min<uint32_t>({16u, hw, (uint32_t)nch});
  for (uint64_t k0 = 0, wave = 0; k0 < nch; k0 += PIN_PER, ++wave) {
    const uint64_t k1 = std::min<uint64_t>(nch, k0 + PIN_PER);
    const uint32_t half = (uint32_t)(wave & 1);
    uint8_t* base = pin.p + (waves ? half * PIN_PER * PIN_CHUNK : 0);
    if (wave >= 2) HIPCHK(hipEventSynchronize(pin.ev[half]));  // that half's previous H2D is done
    const uint64_t lo = k0 * PIN_CHUNK, hi = std::min(span, k1 * PIN_CHUNK);
    if (T == 1) {
      fill_range(base, lo, hi, hp);
    } else {
      std::atomic<uint64_t> next{k0};
      auto work = [&]() {
        for (uint64_t k; (k = next.fetch_add(1)) < k1;) {
          const uint64_t a = k * PIN_CHUNK, z = std::min(span, a + PIN_CHUNK);
          fill_range(base + (a - lo), a, z, hp);
        }
      };
      std::vector<std::thread> th;
      for (uint32_t t = 1; t < T; ++t) th.emplace_back(work);
      work();
      for (auto& t : th) t.join();
    }
    HIPCHK(hipMemcpyAsync(dev + lo, base, hi - lo, hipMemcpyHostToDevice, s));
    HIPCHK(hipEventRecord(pin.ev[half], s));
  }
  return YCRDT_OK;
}

// Stages the sources into the batch buffer: the host region in one H2D copy, device sources by
// one piece-copy launch. doc_of (one per source) makes it a multi-document batch.
int stage_srcs(ycrdt_batch* b, const std::vector<Src>& src, const uint32_t* doc_of = nullptr, uint32_t ndocs = 1) {
  ycrdt_engine* e = b->e;
  std::vector<uint32_t> order;
  layout(b, src, order);
  for (const Src& x : src)
    if (((x.len + 63) & ~size_t(63)) > win_use(b->win_shift)) return fail(YCRDT_E_CAPACITY, "an update larger than 4 GiB");
  if (b->nwin > 255) return fail(YCRDT_E_CAPACITY, "batch larger than 255 windows of 4 GiB");
  if (!grow(b->bytes, (size_t)b->nbytes + 128)) return fail(YCRDT_E_DEVICE, oom("batch bytes"));
  const size_t nu = b->ulen.size();
  size_t ndev = 0;
  while (ndev < nu && src[order[ndev]].dev) ++ndev;
  b->ntrusted = (uint32_t)ndev;
  // staging runs on the copy stream (a host thread may stage the next batch while another merges
  // on the engine stream); device sources (doc states in HBM) are read after the engine stream's
  // work so far, which may still be writing them
  const hipStream_t cs = e->copy;
  if (ndev) {
    HIPCHK(hipEventRecord(e->copy_dep, e->stream));
    HIPCHK(hipStreamWaitEvent(cs, e->copy_dep, 0));
  }
  // the host updates: their span (window gaps included) through pinned staging
  const uint64_t host0 = ndev < nu ? uabs(b, ndev) : b->nbytes;
  {
    std::vector<HostPiece> hp;
    hp.reserve(nu - ndev);
    for (size_t u = ndev; u < nu; ++u) hp.push_back(HostPiece{uabs(b, u) - host0, b->ulen[u], src[order[u]].p});
    if (const int rc = h2d_span(e, (uint8_t*)b->bytes.p + host0, b->nbytes - host0, hp)) return rc;
  }
  if (ndev == 1) {
    if (b->ulen[0]) HIPCHK(hipMemcpyAsync(b->bytes.p, src[order[0]].p, b->ulen[0], hipMemcpyDeviceToDevice, cs));
  } else if (ndev > 1) {
    std::vector<Piece> pc;
    pc.reserve(ndev);
    for (size_t u = 0; u < ndev; ++u)
      if (b->ulen[u]) pc.push_back(Piece{src[order[u]].p, (uint8_t*)b->bytes.p + uabs(b, u), b->ulen[u], {0}});
    if (!grow(b->pieces, sizeof(Piece) * (pc.size() + 1))) return fail(YCRDT_E_DEVICE, oom("pieces"));
    HIPCHK(hipMemcpyAsync(b->pieces.p, pc.data(), sizeof(Piece) * pc.size(), hipMemcpyHostToDevice, cs));
    copy_pieces((const Piece*)b->pieces.p, (uint32_t)pc.size(), cs);
  }
  // meta: uoff | ulen | ugroup | groups | udoc | ulist
  b->ndocs = doc_of && ndocs > 1 ? ndocs : 1;
  b->udoc.clear();
  if (b->ndocs > 1) {
    b->udoc.resize(nu);
    for (size_t u = 0; u < nu; ++u) {
      b->udoc[u] = doc_of[order[u]];
      if (b->udoc[u] >= b->ndocs) return fail(YCRDT_E_ARG, "document index out of range");
    }
  }
  const size_t meta_bytes = sizeof(uint32_t) * (nu + 1 + nu + nu) + sizeof(Group) * b->groups.size() + 64 +
                            sizeof(uint32_t) * b->udoc.size() + 16 + sizeof(uint32_t) * b->ulist.size() + 16 +
                            sizeof(uint32_t) * b->uwin.size() + 16;
  if (!grow(b->meta, meta_bytes)) return fail(YCRDT_E_DEVICE, oom("meta"));
  std::vector<uint8_t> meta(meta_bytes, 0);
  size_t o = 0;
  memcpy(meta.data() + o, b->uoff.data(), sizeof(uint32_t) * (nu + 1)); o += sizeof(uint32_t) * (nu + 1);
  memcpy(meta.data() + o, b->ulen.data(), sizeof(uint32_t) * nu); o += sizeof(uint32_t) * nu;
  memcpy(meta.data() + o, b->ugroup.data(), sizeof(uint32_t) * nu); o += sizeof(uint32_t) * nu;
  o = (o + 15) & ~size_t(15);
  if (!b->groups.empty()) memcpy(meta.data() + o, b->groups.data(), sizeof(Group) * b->groups.size());
  o += sizeof(Group) * b->groups.size();
  o = (o + 15) & ~size_t(15);
  b->udoc_off = o;
  if (!b->udoc.empty()) memcpy(meta.data() + o, b->udoc.data(), sizeof(uint32_t) * b->udoc.size());
  o += sizeof(uint32_t) * b->udoc.size();
  o = (o + 15) & ~size_t(15);
  b->ulist_off = o;
  if (!b->ulist.empty()) memcpy(meta.data() + o, b->ulist.data(), sizeof(uint32_t) * b->ulist.size());
  o += sizeof(uint32_t) * b->ulist.size();
  o = (o + 15) & ~size_t(15);
  b->uwin_off = o;
  if (!b->uwin.empty()) memcpy(meta.data() + o, b->uwin.data(), sizeof(uint32_t) * b->uwin.size());
  HIPCHK(hipMemcpyAsync(b->meta.p, meta.data(), meta_bytes, hipMemcpyHostToDevice, cs));
  HIPCHK(hipStreamSynchronize(cs));
  b->merged = false;
  return YCRDT_OK;
}

// n host updates, optionally behind a device-resident doc state (`prefix`, the first update)
int stage(ycrdt_batch* b, const ycrdt_buf* ups, size_t n, const DevBuf* prefix, size_t prefix_len,
          const uint32_t* doc_of = nullptr, uint32_t ndocs = 1, const int32_t* hints = nullptr) {
  if (prefix_len && doc_of && ndocs > 1) return fail(YCRDT_E_ARG, "internal: multi-document batch with a state prefix");
  b->jpasses = 0;
  b->jstore.clear();
  std::vector<Src> src;
  src.reserve(n + 1);
  if (prefix_len) src.push_back(Src{(const uint8_t*)prefix->p, prefix_len, true});
  for (size_t i = 0; i < n; ++i) {
    src.push_back(Src{ups[i].ptr, ups[i].len, false});
    if (hints) { src.back().nst = hints[2 * i]; src.back().nsec = hints[2 * i + 1]; }
  }
  return stage_srcs(b, src, doc_of, ndocs);
}

int map_err(uint32_t code, const char* where) {
  switch (code) {
    case ERR_DECODE: return fail(YCRDT_E_DECODE, std::string("Integer out of range! (malformed update, ") + where + ")");
    case ERR_PENDING: return fail(YCRDT_E_PENDING, std::string("update has missing dependencies (pending) at ") + where);
    case ERR_UNSUPPORTED: return fail(YCRDT_E_UNSUPPORTED, std::string("input outside the engine's current coverage (see DESIGN.md) at ") + where);
    case ERR_CAPACITY: return fail(YCRDT_E_CAPACITY, std::string("capacity exceeded at ") + where);
    default: return fail(YCRDT_E_DEVICE, "unknown device error");
  }
}

// Reads the counters (sync) and returns an error if the device raised one.
int check(ycrdt_engine* e, Counters& c, const char* where) {
  if (!e->ctr_pin && hipHostMalloc((void**)&e->ctr_pin, sizeof(Counters), hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    e->ctr_pin = nullptr;
    return fail(YCRDT_E_DEVICE, "pinned counter read-back allocation failed");
  }
  HIPCHK(hipMemcpyAsync(e->ctr_pin, e->w.ctr, sizeof(Counters), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  c = *e->ctr_pin;
  if (c.err && (c.err_info >> 16) >= 0xC0DEu && (c.err_info >> 16) <= 0xC0DFu) {  // YCRDT_PREDECODE=check: marks != decode
    char m[200];
    snprintf(m, sizeof(m), "doc state marks differ from its decode (%s word %u: decode %08x%08x, marks %08x%08x)",
             (c.err_info >> 16) == 0xC0DFu ? "delete-set start" : (c.err_info & 0x8000u) ? "section bitmap" : "struct bitmap",
             c.err_info & 0x7FFFu, c.pad[9], c.pad[8], c.pad[11], c.pad[10]);
    return fail(YCRDT_E_DECODE, m);
  }
  if (c.err == ERR_CAPACITY && (c.err_info >> 16) == 0xB0DEu) {  // YCRDT_DEBUG_BOUNDS
    static const char* what[] = {"?", "unit flag", "key slot", "k_merge_small segments", "k_encode_small segments / clients",
                                 "k_encode_small output struct", "k_decode_tail_small structs / sections", "k_sections_small sections / client hash"};
    const uint32_t k = c.err_info & 0xFFFFu;
    return fail(YCRDT_E_CAPACITY, std::string("bounds check (YCRDT_DEBUG_BOUNDS): an index past its table: ") + what[k < 8 ? k : 0] + " at " + where);
  }
  if (c.err) return map_err(c.err, where);
  return YCRDT_OK;
}

struct ShardSpec {
  uint32_t nshards = 1;
  int32_t shard = -1;  // -1: every shard in turn (logical shards on one GPU)
  ycrdt_comm* comm = nullptr;
  // collective bookkeeping: every data exchange is preceded by a status agreement (a max of one
  // word over the ranks). A rank that fails while its peers head for the next agreement joins that
  // agreement with a failure status (they all stop there); one that fails inside a data exchange
  // aborts the communicator (RCCL) instead.
  mutable bool inside = false;    // between an agreement and the end of its data collectives
  mutable bool finished = false;  // past the last exchange of the merge
};
// the agreement before a data exchange: fails (on every rank) when any rank reports a failure
int shard_agree(const ShardSpec* sh, hipStream_t s) {
  uint32_t any = 0;
  std::string err;
  if (yc::comm_agree(sh->comm, 0u, s, any, err)) return fail(YCRDT_E_DEVICE, err);
  if (any) { sh->finished = true; return fail(YCRDT_E_DEVICE, "another rank failed the sharded merge"); }
  sh->inside = true;
  return YCRDT_OK;
}

struct Decoded {
  uint32_t nstructs = 0, nsections = 0, nclients = 0, nds = 0;
  uint64_t nunits = 0, in_len = 0;
  uint32_t array_roots = 0;  // 1: some item names a parent without a parentSub (a YArray may exist)
  uint32_t any_rorigin = 0;  // 1: some item has a right origin (a YMap entry may need full YATA)
  bool ds_big = false;       // a delete set with more ranges than one wavefront applies
  uint32_t nested = 0;       // 1: some item names a parent item (nested types: dead-type pass needed)
  uint32_t nroots = 0;       // items with an explicit parent (key table bound)
  uint32_t noncanon = 0;     // lazy: some update's sections are not in strictly descending client order
};

// ---- decode split (sharded merge): which updates this rank parses. Updates are dealt to ranks
// by size (largest first onto the least-loaded rank), identically on every rank; the rank's decode
// runs over a filtered update list and chunk table (the other updates are staged but not parsed).
std::vector<uint32_t> split_owners(const ycrdt_batch* b, uint32_t nshards) {
  const size_t nu = b->ulen.size();
  std::vector<uint32_t> idx(nu), owner(nu, 0);
  for (size_t u = 0; u < nu; ++u) idx[u] = (uint32_t)u;
  std::stable_sort(idx.begin(), idx.end(), [&](uint32_t x, uint32_t y) { return b->ulen[x] > b->ulen[y]; });
  std::vector<uint64_t> load(nshards, 0);
  for (const uint32_t u : idx) {
    const uint32_t r = (uint32_t)(std::min_element(load.begin(), load.end()) - load.begin());
    owner[u] = r;
    load[r] += b->ulen[u] + 64;
  }
  return owner;
}
int split_decode_meta(ycrdt_engine* e, ycrdt_batch* b, const ShardSpec* sh, Work& wd) {
  const uint32_t me = (uint32_t)sh->shard;
  const std::vector<uint32_t> owner = split_owners(b, sh->nshards);
  const size_t nu = b->ulen.size();
  std::vector<uint32_t> ul, ug(b->ugroup);
  std::vector<Group> gr;
  uint32_t nbig = 0;
  for (uint32_t i = 0; i < b->ulist.size(); ++i) {
    const uint32_t u = b->ulist[i];
    if (owner[u] != me) continue;
    ul.push_back(u);
    if (i < b->nbig) {  // its chunks, renumbered into this rank's chunk table
      ++nbig;
      const uint32_t g0 = b->ugroup[u];
      ug[u] = (uint32_t)gr.size();
      for (uint32_t g = g0; g < b->groups.size() && b->groups[g].upd == u; ++g) gr.push_back(b->groups[g]);
    }
  }
  const size_t bytes = sizeof(uint32_t) * (nu + 1) * 2 + sizeof(Group) * (gr.size() + 1) + 64;
  bool ok = true;
  uint8_t* m = take<uint8_t>(e->bufs, B_SPLITMETA, bytes, ok);
  if (!ok) return fail(YCRDT_E_DEVICE, oom("decode split"));
  std::vector<uint8_t> h(bytes, 0);
  memcpy(h.data(), ul.data(), sizeof(uint32_t) * ul.size());
  memcpy(h.data() + sizeof(uint32_t) * (nu + 1), ug.data(), sizeof(uint32_t) * nu);
  const size_t goff = (sizeof(uint32_t) * (nu + 1) * 2 + 15) & ~size_t(15);
  if (!gr.empty()) memcpy(h.data() + goff, gr.data(), sizeof(Group) * gr.size());
  HIPCHK(hipMemcpyAsync(m, h.data(), bytes, hipMemcpyHostToDevice, e->stream));
  wd.ulist = (const uint32_t*)m;
  wd.nbig = nbig;
  wd.nsmall = (uint32_t)ul.size() - nbig;
  wd.ugroup = (const uint32_t*)(m + sizeof(uint32_t) * (nu + 1));
  wd.groups = (const Group*)(m + goff);
  wd.ngroups = (uint32_t)gr.size();
  // updates parsed elsewhere leave their delete-set start 0 here (combined by a max)
  HIPCHK(hipMemsetAsync(wd.dsstart, 0, sizeof(uint32_t) * (nu + 1), e->stream));
  return YCRDT_OK;
}
// every rank's parse results combined: struct-start and section-start bitmaps (disjoint words:
// updates are 64-byte aligned, so a sum is the union), delete-set starts (max), the error word
// (max), and the section records (all-gathered, rank after rank)
int split_decode_exchange(ycrdt_engine* e, ycrdt_batch* b, const ShardSpec* sh) {
  Work& w = e->w;
  hipStream_t s = e->stream;
  std::string err;
  if (const int rc = shard_agree(sh, s)) return rc;
  const uint64_t nwords = ((uint64_t)b->nbytes + 64) / 64 + 2;
  const size_t nu = b->ulen.size();
  if (yc::comm_allreduce_u32(sh->comm, (uint32_t*)w.final_bits, 2 * nwords, false, s, err) ||
      yc::comm_allreduce_u32(sh->comm, (uint32_t*)w.sec_bits, 2 * nwords, false, s, err) ||
      yc::comm_allreduce_u32(sh->comm, w.dsstart, nu + 1, true, s, err) ||
      yc::comm_allreduce_u32(sh->comm, &w.ctr->err, 1, true, s, err))
    return fail(YCRDT_E_DEVICE, err);
  uint32_t cw[2] = {0, 0};  // the reduced error word, this rank's section count
  HIPCHK(hipMemcpyAsync(&cw[0], &w.ctr->err, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(&cw[1], &w.ctr->nsections, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  // the walkers bump the count before their capacity test: past the estimate only the first
  // cap_sections records exist (the error word then says ERR_CAPACITY on every rank)
  const uint32_t nsec = std::min(cw[1], w.cap_sections);
  std::vector<Section> mine(nsec);
  if (nsec) HIPCHK(hipMemcpy(mine.data(), w.sections, sizeof(Section) * nsec, hipMemcpyDeviceToHost));
  std::vector<std::vector<uint8_t>> parts;
  if (yc::comm_allgather_updates(sh->comm, (const uint8_t*)mine.data(), sizeof(Section) * nsec, s, parts, err))
    return fail(YCRDT_E_DEVICE, err);
  std::vector<uint8_t> all;
  for (const auto& p : parts) all.insert(all.end(), p.begin(), p.end());
  const uint64_t total = all.size() / sizeof(Section);
  sh->inside = false;  // the exchange is complete on every rank
  // a capacity overflow on any rank (reduced error word) or of the gathered table: the same on
  // every rank, so all of them re-run the decode with the worst-case bound (run_decode)
  if (cw[0] == ERR_CAPACITY || total > w.cap_sections) return fail(YCRDT_E_CAPACITY, "decode split: sections past the estimate");
  if (total) HIPCHK(hipMemcpyAsync(w.sections, all.data(), all.size(), hipMemcpyHostToDevice, s));
  // every update's sections in the gathered table (each walker wrote its update's sections as one
  // run, in byte order): the per-update (first, count) the later passes read (k_ds_bound)
  {
    std::vector<uint32_t> us(2 * (nu + 1), 0);
    const Section* sp = (const Section*)all.data();
    for (uint64_t i = 0; i < total; ++i) {
      const uint32_t u = sp[i].upd;
      if (u >= nu) return fail(YCRDT_E_DEVICE, "decode split: section of an unknown update");
      if (!us[nu + 1 + u]) us[u] = (uint32_t)i;
      ++us[nu + 1 + u];
    }
    HIPCHK(hipMemcpyAsync(w.usec_start, us.data(), sizeof(uint32_t) * (nu + 1), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(w.usec_n, us.data() + nu + 1, sizeof(uint32_t) * (nu + 1), hipMemcpyHostToDevice, s));
  }
  const uint32_t t32 = (uint32_t)total;
  HIPCHK(hipMemcpyAsync(&w.ctr->nsections, &t32, sizeof(uint32_t), hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));
  return YCRDT_OK;
}

// ---- ContentJSON / Embed / Format values outside JSON.stringify's form (Y@72137 readContentJSON
// parses them, Y@71991 writes JSON.stringify of the parsed value back): the decode lists their
// structs (k_json_structs), k_json_canon computes the canonical contents on the device, and the
// batch is staged again with those contents spliced into their updates (host copies of the staged
// updates: byte moves only), so that every later pass sees what Yjs would hold. A pass whose
// canonical contents all equal the input (a text json_check could not judge: nesting past its
// level mask) keeps the batch as it is. Rare by construction: Yjs itself writes ContentAny.
constexpr uint32_t JARENA_WORDS = JSON_ARENA_WORDS;  // arena per lane (yc_parse.h json_canon): 256 KiB
constexpr uint32_t JLANES = 256;
int json_rewrite(ycrdt_engine* e, ycrdt_batch* b, uint32_t n, const ShardSpec* sh, bool& restaged) {
  restaged = false;
  if (++b->jpasses > 8) return fail(YCRDT_E_DEVICE, "internal: the JSON rewrite did not settle");
  Work& w = e->w;
  auto& V = e->bufs;
  hipStream_t s = e->stream;
  bool ok = true;
  const uint32_t lanes = std::min(n, JLANES);
  JItem* items = take<JItem>(V, B_JITEM, n, ok);
  uint32_t* arena = take<uint32_t>(V, B_JARENA, (size_t)lanes * JARENA_WORDS, ok);
  unsigned long long* offs = take<unsigned long long>(V, B_JOFF, n, ok);
  if (!ok) return fail(YCRDT_E_DEVICE, oom("JSON rewrite"));
  launch_json_canon(w, w.jlist, n, items, arena, JARENA_WORDS, lanes, nullptr, nullptr, s);
  std::vector<JItem> it(n);
  HIPCHK(hipMemcpyAsync(it.data(), items, sizeof(JItem) * n, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  std::vector<unsigned long long> off(n);
  unsigned long long total = 0;
  for (uint32_t j = 0; j < n; ++j) {
    if (it[j].res == JSON_BAD) return fail(YCRDT_E_DECODE, "JSON.parse: a ContentJSON / Embed / Format value is not JSON");
    if (it[j].res != JSON_OK) return fail(YCRDT_E_UNSUPPORTED, "a ContentJSON / Embed / Format value past the rewrite arena (nesting or object size)");
    off[j] = total;
    total += it[j].len;
  }
  uint8_t* cout = take<uint8_t>(V, B_JOUT, total + 1, ok);
  if (!ok) return fail(YCRDT_E_DEVICE, oom("JSON rewrite"));
  HIPCHK(hipMemcpyAsync(offs, off.data(), sizeof(unsigned long long) * n, hipMemcpyHostToDevice, s));
  launch_json_canon(w, w.jlist, n, items, arena, JARENA_WORDS, lanes, offs, cout, s);
  HIPCHK(hipMemcpyAsync(it.data(), items, sizeof(JItem) * n, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  bool any_diff = false;
  for (uint32_t j = 0; j < n; ++j) any_diff |= it[j].pad != 0;
  if (!any_diff) return YCRDT_OK;  // already in the form Yjs writes (compared on the device)
  // (a sharded merge parses each update on one rank only: a rewrite would have to be agreed on)
  if (sh) return fail(YCRDT_E_UNSUPPORTED, "a ContentJSON / Embed / Format or `any` value Yjs writes back differently, in a sharded merge");
  std::vector<uint8_t> canon(total);
  if (total) HIPCHK(hipMemcpyAsync(canon.data(), cout, total, hipMemcpyDeviceToHost, s));
  // the updates as staged (layout order), and which of them a content lies in
  const size_t nu = b->ulen.size();
  std::vector<std::vector<uint8_t>> ups(nu);
  for (size_t u = 0; u < nu; ++u) {
    ups[u].resize(b->ulen[u]);
    if (b->ulen[u]) HIPCHK(hipMemcpyAsync(ups[u].data(), (const uint8_t*)b->bytes.p + uabs(b, u), b->ulen[u], hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  std::vector<std::vector<uint32_t>> per(nu);  // items of each update
  bool changed = false;
  for (uint32_t j = 0; j < n; ++j) {
    size_t u = nu;
    for (size_t v = 0; v < nu; ++v)
      if (it[j].cpos >= uabs(b, v) && it[j].cpos + it[j].clen <= uabs(b, v) + b->ulen[v]) { u = v; break; }
    if (u == nu) return fail(YCRDT_E_DEVICE, "internal: a JSON content outside every staged update");
    if (it[j].pad) {
      per[u].push_back(j);
      changed = true;
    }
  }
  if (!changed) return YCRDT_OK;  // already in JSON.stringify's form (a text json_check could not judge)
  std::vector<std::vector<uint8_t>> store(nu);
  std::vector<Src> src(nu);
  for (size_t u = 0; u < nu; ++u) {
    if (per[u].empty()) {
      store[u] = std::move(ups[u]);
    } else {
      std::sort(per[u].begin(), per[u].end(), [&](uint32_t x, uint32_t y) { return it[x].cpos < it[y].cpos; });
      std::vector<uint8_t>& o = store[u];
      uint64_t at = 0;
      for (const uint32_t j : per[u]) {
        const uint64_t rel = it[j].cpos - uabs(b, u);
        o.insert(o.end(), ups[u].begin() + at, ups[u].begin() + rel);
        o.insert(o.end(), canon.begin() + off[j], canon.begin() + off[j] + it[j].len);
        at = rel + it[j].clen;
      }
      o.insert(o.end(), ups[u].begin() + at, ups[u].end());
    }
    src[u] = Src{store[u].data(), store[u].size(), false};
  }
  const std::vector<uint32_t> udoc = b->udoc;
  const uint32_t ndocs = b->ndocs, ntrusted = b->ntrusted;
  b->pre_src = -1;  // (a doc state's marks no longer name a source: it is decoded like the others)
  b->pre_check = false;
  if (const int rc = stage_srcs(b, src, udoc.empty() ? nullptr : udoc.data(), ndocs)) return rc;
  b->ntrusted = ntrusted;  // (the same updates in the same order, now all host copies)
  b->jstore = std::move(store);
  restaged = true;
  return YCRDT_OK;
}

// K1: decode every update of the batch into the struct SoA (+ client table, delete-set ranges).
// lazy = mergeUpdates / diffUpdate mode: references stay raw client ids, no client states.
int run_decode(ycrdt_engine* e, ycrdt_batch* b, bool lazy, Decoded& D, bool generous = false, const ShardSpec* sh = nullptr) {
  Work& w = e->w;
  auto& V = e->bufs;
  g_bufs = &V;
  bool ok = true;
  hipStream_t s = e->stream;
  e->marks.clear();
  e->phase_ms.clear();
  HIPCHK(hipEventRecord(e->ev0, s));
  mark(e, "start");
  // ---- inputs
  const uint32_t nu = (uint32_t)b->ulen.size();
  w.bytes = (const uint8_t*)b->bytes.p;
  w.nbytes = b->nbytes;
  w.nwin = b->nwin;
  w.win_shift = b->win_shift;
  w.uwin = b->nwin > 1 ? (const uint32_t*)((const uint8_t*)b->meta.p + b->uwin_off) : nullptr;
  w.nupd = nu;
  w.uoff = (const uint32_t*)b->meta.p;
  w.ulen = w.uoff + nu + 1;
  w.ugroup = w.ulen + nu;
  {
    size_t o = sizeof(uint32_t) * (nu + 1 + nu + nu);
    o = (o + 15) & ~size_t(15);
    w.groups = (const Group*)((const uint8_t*)b->meta.p + o);
  }
  w.ngroups = (uint32_t)b->groups.size();
  w.udoc = b->ndocs > 1 ? (const uint32_t*)((const uint8_t*)b->meta.p + b->udoc_off) : nullptr;
  w.ndocs = b->ndocs;
  w.ulist = (const uint32_t*)((const uint8_t*)b->meta.p + b->ulist_off);
  w.nbig = b->nbig;
  w.schunk = b->schunk;
  w.nsmall = (uint32_t)b->ulist.size() - b->nbig;
  w.small_max = 0;
  for (size_t i = b->nbig; i < b->ulist.size(); ++i) w.small_max = std::max(w.small_max, b->ulen[b->ulist[i]]);
  w.lazy = lazy ? 1u : 0u;
  {
    const char* mode = getenv("YCRDT_DECODE");
    w.force_xtab = mode && !strcmp(mode, "xtab") ? 1u : 0u;
    // the chunk walk skipped when the pre-walk takes every large update (YCRDT_WALK_ONLY=0: A/B);
    // a pre-walk that stops short raises a capacity error and the generous rerun walks the chunks
    w.walk_only = b->walk_only && !generous && !sh && !w.force_xtab && !env_off("YCRDT_PREWALK") && !env_off("YCRDT_WALK_ONLY") ? 1u : 0u;
    w.fwm_max = getenv("YCRDT_FWM_MAX") ? (uint32_t)atoi(getenv("YCRDT_FWM_MAX")) : 0u;
    const char* sh = getenv("YCRDT_SPEC_HINT");
    // chunk-start hints: single-section updates only by default (a C2 snapshot or replica update
    // syncs with them; multi-section C4 states locked into wrong phases with them, §5.4b);
    // YCRDT_SPEC_HINT=1 / 0: always / never
    w.spec_hint = sh && sh[0] == '1' ? 1u : sh && sh[0] == '0' ? 0u : 2u;
  }
  const uint64_t B = (uint64_t)b->nbytes + 64;
  const uint64_t nwords = B / 64 + 2;
  // The section table is sized from an estimate (a capacity overflow reruns the decode with the
  // worst-case bound); the struct table, the client table and the delete-set ranges are sized
  // after the count sync from the real counts, so the workspace follows the content, not B.
  const uint64_t est_sec = std::min<uint64_t>(generous ? B / 3 + 64 : std::min<uint64_t>(B / 3 + 64, (uint64_t)nu * 16 + B / 256 + 4096),
                                              0x7FFFFFFFull);
  w.cap_sections = (uint32_t)est_sec;
  if (const char* tc = getenv("YCRDT_TEST_SECTION_CAP"))  // tests: a tiny estimate forces the overflow re-run
    if (!generous && atoi(tc) > 0) w.cap_sections = std::min<uint32_t>(w.cap_sections, (uint32_t)atoi(tc));
  w.cap_structs = 0;
  w.cap_ds = 0;
  // ---- decode buffers
  w.ctr = take<Counters>(V, B_CTR, 1, ok);
  w.spec_bits = take<uint64_t>(V, B_SPECB, nwords, ok);
  w.cexit = take<uint32_t>(V, B_CEXIT, (uint64_t)w.ngroups + 1, ok);
  w.sexit = take<uint32_t>(V, B_SEXIT, (uint64_t)w.ngroups + 1, ok);
  w.sent = take<uint32_t>(V, B_SENT, 2 * ((uint64_t)w.ngroups + 1), ok);  // entries, then jumped flags
  w.xtab = take<uint32_t>(V, B_XTAB, ((uint64_t)w.ngroups + 1) * XK, ok);
  w.tentry = take<uint32_t>(V, B_TENTRY, (uint64_t)w.ngroups + 1, ok);
  w.xlist = take<uint32_t>(V, B_XLIST, (uint64_t)w.ngroups + 1, ok);
  w.ufail = take<uint32_t>(V, B_UFAIL, nu + 1, ok);
  w.fw = take<uint32_t>(V, B_FW, 2ull * nu + 2, ok);
  w.ccnt = take<uint32_t>(V, B_CCNT, (uint64_t)w.ngroups + 1, ok);
  w.coff = take<uint32_t>(V, B_COFF, (uint64_t)w.ngroups + 1, ok);
  w.cpre = take<uint64_t>(V, B_CPRE, (uint64_t)w.ngroups + 1, ok);
  w.opre = take<uint32_t>(V, B_OPRE, (uint64_t)w.ngroups + 1, ok);
  w.final_bits = take<uint64_t>(V, B_FINAL, nwords, ok);
  w.sec_bits = take<uint64_t>(V, B_SECB, nwords, ok);
  w.dsstart = take<uint32_t>(V, B_DSSTART, nu + 1, ok);
  w.sections = take<Section>(V, B_SECT, w.cap_sections, ok);
  w.sec_sorted = take<uint32_t>(V, B_SECSORT, w.cap_sections, ok);
  w.sec_uend = take<uint32_t>(V, B_SECUEND, w.cap_sections, ok);
  w.sec_doc = take<uint32_t>(V, B_SECDOC, w.cap_sections, ok);
  w.wcnt = take<uint32_t>(V, B_WCNT, nwords + 1, ok);
  w.wsec = take<uint32_t>(V, B_WSEC, nwords + 1, ok);
  w.ds_region = take<uint32_t>(V, B_DSREG, nu + 2, ok);
  w.ds_count = take<uint32_t>(V, B_DSCNT, nu + 2, ok);
  w.ds_dense_off = take<uint32_t>(V, B_DSOFF, nu + 2, ok);
  w.ds_biglist = take<uint32_t>(V, B_DSBIGL, nu + 1, ok);
  w.jcap = 0;  // (sized when the decode saw a JSON-like content)
  w.jlist = nullptr;
  w.cap_clients = w.cap_sections;
  w.scratch = take<uint32_t>(V, B_SCRATCH, std::max<uint64_t>({nwords + 2, (uint64_t)w.cap_sections + 66, (uint64_t)nu + 2}), ok);
  w.usec_start = take<uint32_t>(V, B_USEC, nu + 1, ok);
  w.usec_n = take<uint32_t>(V, B_USECN, nu + 1, ok);
  w.wlen = wave_decode(w) ? take<uint16_t>(V, B_WLEN, (uint64_t)w.nsmall * 16384, ok) : nullptr;
  w.fwsec = w.nbig ? take<uint32_t>(V, B_FWSEC, 2ull * w.cap_sections + 2, ok) : nullptr;
  w.fwc = nullptr;
  w.fwc_off = nullptr;
  w.rtab = nullptr;
  w.rk = nullptr;
  if (b->fwc_recs && w.fwsec) {  // record mode: the records and each update's base
    w.fwc = take<uint4>(V, B_FWC, b->fwc_recs + 1, ok);
    uint32_t* fo = take<uint32_t>(V, B_FWCOFF, nu + 1, ok);
    if (ok) HIPCHK(hipMemcpyAsync(fo, b->fwc_off.data(), sizeof(uint32_t) * nu, hipMemcpyHostToDevice, e->stream));
    w.fwc_off = fo;
    if (!env_off("YCRDT_RTAB")) w.rtab = take<uint32_t>(V, B_RTAB, b->fwc_recs + 1, ok);  // (YCRDT_RTAB=0: parse every step, A/B)
    if (w.rtab && !env_off("YCRDT_RANK_LAST")) w.rk = take<uint4>(V, B_RK, nu + 1, ok);
    const char* fw = getenv("YCRDT_FWC_WALK");  // (experiments)
    w.fwc_walk = fw && atoi(fw) > 0 ? (uint32_t)atoi(fw) : 256u;
  }
  if (!ok) return fail(YCRDT_E_DEVICE, oom("decode workspace"));
  // rocPRIM scratch sized for the largest scan of this batch (units may grow it later)
  {
    // scans: the bitmap words, per-update and per-struct columns; sorts: the client table (sections)
    size_t tb = prim_tmp_bytes(std::max<uint64_t>({B / 64 + 4, (uint64_t)nu + 2, (uint64_t)w.cap_sections + 2, 1024}),
                               (uint64_t)w.cap_sections + 2);
    w.tmp = take<uint8_t>(V, B_TMP, tb, ok);
    w.tmp_bytes = V[B_TMP].cap;
  }
  if (!ok) return fail(YCRDT_E_DEVICE, oom("scan scratch"));
  static_assert(sizeof(Counters) % 4 == 0, "counters are filled as words");
  fill_u32_multi({{(uint32_t*)w.ctr, sizeof(Counters) / 4, 0u},
                  {w.ufail, (uint64_t)nu + 1, 0u},
                  {w.usec_n, (uint64_t)nu + 1, 0u},  // an update no walker reached has no sections
                  {(uint32_t*)w.final_bits, (uint64_t)nwords * 2, 0u},
                  {(uint32_t*)w.sec_bits, (uint64_t)nwords * 2, 0u}}, s);
  w.dbg_bounds = getenv("YCRDT_DEBUG_BOUNDS") && getenv("YCRDT_DEBUG_BOUNDS")[0] == '1' ? 1u : 0u;
  w.upre = b->pre_src >= 0 && !b->pre_check ? b->pre_u : NONE;
  if (w.upre != NONE) launch_predecoded(w, b->pre_u, b->pre, false, s);  // (a doc state: its own encode's decode)
  const bool dbg_yata = getenv("YCRDT_DEBUG_YATA") && getenv("YCRDT_DEBUG_YATA")[0] == '1';
  const bool dbg_dec = getenv("YCRDT_DEBUG_DECODE") && getenv("YCRDT_DEBUG_DECODE")[0] == '1';
  w.dbg = dbg_yata || dbg_dec ? take<unsigned long long>(V, B_DBG, 24, ok) : nullptr;
  if (w.dbg) HIPCHK(hipMemsetAsync(w.dbg, 0, 192, s));
  // ---- K1 decode
  // large updates (chunk path, mostly latency-bound) on the side stream, beside k_direct
  mark(e, "decode.direct");
  // decode split across the ranks of a sharded merge: each rank parses only
  // its share of the updates (byte-balanced), then the struct / section bitmaps, the delete-set
  // starts and the section records are combined, and every rank continues on the same tables
  const bool split = sh && sh->comm && sh->nshards > 1 && !lazy;
  Work wd = w;
  if (split) {
    const int rc0 = split_decode_meta(e, b, sh, wd);
    if (rc0) return rc0;
  }
  // (no large update: no chunk path, no fork / join — four runtime calls fewer per small merge)
  const bool chunks = wd.ngroups || wd.nbig;
  if (chunks) {
    HIPCHK(hipEventRecord(e->side_fork, s));
    HIPCHK(hipStreamWaitEvent(e->side, e->side_fork, 0));
    launch_chunks(wd, e->side);
    HIPCHK(hipEventRecord(e->side_done, e->side));
  }
  launch_direct(wd, s);
  mark(e, "decode.chunk_wait");  // decode.direct: k_direct alone (the chunk path runs beside it)
  if (chunks) HIPCHK(hipStreamWaitEvent(s, e->side_done, 0));
  if (split) {
    mark(e, "decode.exchange");
    // test hook (tests/test_gpu_exchange.py): this rank fails on the host before the exchange
    const char* fh = getenv("YCRDT_TEST_FAIL_BEFORE_EXCHANGE");
    if (fh && fh[0] == '1') return fail(YCRDT_E_DEVICE, "test hook: failure before the decode exchange");
    const int rc0 = split_decode_exchange(e, b, sh);
    if (rc0 == YCRDT_E_CAPACITY && !generous) return run_decode(e, b, lazy, D, true, sh);  // every rank alike
    if (rc0) return rc0;
  }
  mark(e, "decode.bitmap");
  if (!count_ds_small(w, s)) {  // (small batches: one workgroup)
    launch_struct_count(w, s);
    launch_ds_bound(w, s);
  }
  if (!w.nupd) HIPCHK(hipMemcpyAsync(&w.ctr->nstructs, w.wcnt + (w.nbytes + 63) / 64, sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  Counters c;
  // A small single-document integrate batch skips the count synchronisation: the struct, delete-
  // set and client tables are sized from bounds (a struct starts at a distinct byte; a delete-set
  // region is at most half its bytes; the sections fit the section table), the single-workgroup
  // passes read the counts on the device, and one past their sizes raises a capacity error that
  // reruns the decode the counted way (generous)
  const bool quick = !lazy && !split && !generous && !w.dbg && !w.udoc && w.nupd && b->nwin <= 1 && w.nbytes <= (64u << 10) && w.cap_sections <= 16000 &&
                     !env_off("YCRDT_DECODE_SMALL") && !env_off("YCRDT_DECODE_QUICK");
  if (b->pre_src >= 0 && b->pre_check) launch_predecoded(w, b->pre_u, b->pre, true, s);  // (reported at the next check)
  int rc = quick ? YCRDT_OK : check(e, c, "decode");
  if (quick) {
    c = Counters();
    c.nstructs = (uint32_t)w.nbytes + 1;
    c.nsections = w.cap_sections;
    c.ds_region = (uint32_t)w.nbytes + w.nupd + 1;
  }
  if (dbg_dec && w.dbg) {  // experiments: why k_fastwalk left large updates to k_walk
    unsigned long long h[24];
    HIPCHK(hipMemcpy(h, w.dbg, sizeof(h), hipMemcpyDeviceToHost));
    fprintf(stderr, "[ycrdt decode] multi-section fast walk cycles: stage %llu walk %llu search %llu, walked structs %llu, sections vouched %llu\n",
            h[19], h[20], h[21], h[22], h[23]);
    fprintf(stderr, "[ycrdt decode] fastwalk: done %llu nsec %llu unsynced %llu | wave: done %llu unsettled %llu other %llu (chunk path: moved / jumped chunk entries) | k_spec exact parses %llu (%llu bytes) | multi-section left to k_walk, by reason 1-5: %llu %llu %llu %llu %llu (section %llu of %llu structs) | record mode: %llu sections evaluated by the walker, stopped at byte %llu of %llu\n",
            h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[9], h[10], h[11], h[12], h[13], h[14], h[15], h[16], h[17], h[18]);
    HIPCHK(hipMemsetAsync(w.dbg, 0, 192, s));
  }
  if (rc == YCRDT_E_CAPACITY && !generous) return run_decode(e, b, lazy, D, true, sh);  // past the estimates
  if (rc) return rc;
  const uint32_t nstructs = c.nstructs;
  const uint32_t nsections = c.nsections;
  // ---- tables sized from the counts
  w.cap_structs = nstructs + 64;  // (quick: the bounds)
  w.cap_ds = c.ds_region + 64;
  w.cap_clients = nsections + 64;
  w.ds = lazy ? take<DsRange>(V, B_DS, w.cap_ds, ok) : nullptr;  // dense ranges: mergeUpdates / diffUpdate only
  w.ds_tmp = take<DsRange>(V, B_DSTMP, w.cap_ds, ok);
  w.ds_len = nullptr;  // (no per-range length column: k_ds_apply clips in registers)
  w.s_pos = take<uint32_t>(V, B_SPOS, w.cap_structs, ok);
  w.s_win = b->nwin > 1 ? take<uint8_t>(V, B_SWIN, w.cap_structs, ok) : nullptr;
  w.s_sec = take<uint32_t>(V, B_SSEC, w.cap_structs, ok);
  w.s_len = take<uint32_t>(V, B_SLEN, w.cap_structs + 1, ok);
  w.s_lenscan = take<uint64_t>(V, B_SLENSCAN, w.cap_structs + 1, ok);
  w.s_clock = take<uint32_t>(V, B_SCLOCK, w.cap_structs, ok);
  w.s_cidx = take<uint32_t>(V, B_SCIDX, w.cap_structs, ok);
  w.s_info = take<uint8_t>(V, B_SINFO, w.cap_structs, ok);
  w.s_ocidx = take<uint32_t>(V, B_SOC, w.cap_structs, ok);
  w.s_oclock = take<uint32_t>(V, B_SOK, w.cap_structs, ok);
  w.s_rcidx = take<uint32_t>(V, B_SRC, w.cap_structs, ok);
  w.s_rclock = take<uint32_t>(V, B_SRK, w.cap_structs, ok);
  w.s_pk = take<uint8_t>(V, B_SPK, w.cap_structs, ok);
  w.s_pa = take<uint32_t>(V, B_SPA, w.cap_structs, ok);
  w.s_pb = take<uint32_t>(V, B_SPB, w.cap_structs, ok);
  w.s_psub = take<uint32_t>(V, B_SPS, w.cap_structs, ok);
  w.s_psublen = take<uint32_t>(V, B_SPL, w.cap_structs, ok);
  w.s_cpos = take<uint32_t>(V, B_SCPOS, w.cap_structs, ok);
  w.s_cend = take<uint32_t>(V, B_SCEND, w.cap_structs, ok);
  w.s_celem = take<uint32_t>(V, B_SCELEM, w.cap_structs, ok);
  w.sd_defer = take<uint32_t>(V, B_SDDEFER, w.cap_structs, ok);
  w.cl_vals = take<uint32_t>(V, B_CLVALS, w.cap_clients + 1, ok);
  w.ch_key = nullptr;  // find_client binary-searches until the hash is built below
  const uint32_t ch_slots = (uint32_t)next_pow2(std::max<uint64_t>(2ull * (nsections + 1), 64));
  uint64_t* ch_key = take<uint64_t>(V, B_CHKEY, ch_slots, ok);
  uint32_t* ch_val = take<uint32_t>(V, B_CHVAL, ch_slots, ok);
  w.cl_key = take<uint64_t>(V, B_CLKEY, w.cap_clients + 1, ok);
  w.cl_key2 = take<uint64_t>(V, B_CLKEY2, w.cap_clients + 1, ok);
  w.cl_doc = take<uint32_t>(V, B_CLDOC, w.cap_clients + 1, ok);
  w.cl_tmp = take<uint32_t>(V, B_CLTMP, w.cap_clients + 1, ok);
  w.cl_state = take<uint32_t>(V, B_CLSTATE, w.cap_clients + 1, ok);
  w.cl_single = lazy ? nullptr : take<uint8_t>(V, B_CLSINGLE, w.cap_clients + 16, ok);
  w.cl_base = take<uint64_t>(V, B_CLBASE, w.cap_clients + 2, ok);
  w.cl_start = take<uint32_t>(V, B_CLSTART, w.cap_clients + 1, ok);
  if (!ok) return fail(YCRDT_E_DEVICE, oom("struct table"));
  launch_struct_scatter(w, s);
  // small single-document batches: section ranks, client table and client hash in one launch
  const bool sec_small = quick || (!w.udoc && nsections && nsections <= 2048 && ch_slots <= 8192 && !env_off("YCRDT_DECODE_SMALL"));
  if (!sec_small) launch_section_clients(w, nsections, s);
  mark(e, "decode.sections");
  {  // the delete sets decode on the side stream (own scratch / scan space) while the client
     // table and the struct table are built; both streams only read what the sync above published
    Work wd = w;
    bool okd = true;
    if (quick) {  // (no host synchronisation ordered the walk and the bounds before this stream's work)
      HIPCHK(hipEventRecord(e->side_fork, s));
      HIPCHK(hipStreamWaitEvent(e->side, e->side_fork, 0));
    }
    wd.scratch = take<uint32_t>(V, B_SCRATCH2, (uint64_t)w.nupd + 2, okd);
    wd.tmp = take<uint8_t>(V, B_TMP2, prim_tmp_bytes(std::max<uint64_t>((uint64_t)w.nupd + 2, (uint64_t)w.ngroups + 2), 0), okd);
    wd.tmp_bytes = V[B_TMP2].cap;
    if (w.nbig) {  // large delete sets decode grid-wide (yc_decode.hip k_dsp_*)
      wd.dsp_cnt = take<uint32_t>(V, B_DSPCNT, (uint64_t)w.ngroups + 1, okd);
      wd.dsp_pre = take<uint32_t>(V, B_DSPPRE, (uint64_t)w.ngroups + 1, okd);
      wd.dsp_val = take<uint32_t>(V, B_DSPVAL, 2ull * w.cap_ds, okd);
      wd.dsp_blk = take<uint4>(V, B_DSPBLK, (uint64_t)w.nbig * DSP_MAXBLK, okd);
      wd.dsp_nb = take<uint32_t>(V, B_DSPNB, w.nbig, okd);
      wd.dsp_gb = take<uint32_t>(V, B_DSPGB, (uint64_t)w.nbig + 1, okd);
      wd.dsp_b = take<uint32_t>(V, B_DSPB, (uint64_t)w.nupd + 1, okd);
      wd.dsp_fail = take<uint32_t>(V, B_DSPFAIL, (uint64_t)w.nupd + 1, okd);
      wd.dsp_j = take<uint32_t>(V, B_DSHJ, 2ull * w.cap_ds + 2, okd);
      wd.dsp_js = take<uint32_t>(V, B_DSHS, 2ull * w.cap_ds + 2, okd);
      wd.dsp_h = take<uint2>(V, B_DSHH, (uint64_t)w.nbig * (DSH_SEG + 1), okd);
      {  // k_dsh_jump: about one lane per delete-set value of the largest big update
        uint64_t mx = 0;
        for (uint32_t i = 0; i < b->nbig; ++i) mx = std::max<uint64_t>(mx, b->ulen[b->ulist[i]]);
        wd.dsh_grid = (uint32_t)std::min<uint64_t>(256, mx / 512 + 1);  // (grid-stride past 64 K values)
      }
      if (okd) fill_u32_multi({{wd.dsp_b, (uint64_t)w.nupd + 1, NONE}, {wd.dsp_fail, (uint64_t)w.nupd + 1, 0u}}, e->side);
    } else {
      wd.dsp_cnt = wd.dsp_pre = wd.dsp_val = wd.dsp_nb = wd.dsp_b = wd.dsp_fail = nullptr;
      wd.dsp_blk = nullptr;
      wd.dsp_j = wd.dsp_js = nullptr;
      wd.dsp_h = nullptr;
    }
    if (!okd) return fail(YCRDT_E_DEVICE, oom("delete-set scratch"));
    w.dsp_b = wd.dsp_b;  // (the range apply reads which updates took the grid path)
    launch_ds_decode(wd, e->side);
    HIPCHK(hipEventRecord(e->side_done, e->side));
  }
  if (sec_small) {
    if (!sections_small(w, quick ? NONE : nsections, ch_key, ch_val, ch_slots - 1, s)) return fail(YCRDT_E_DEVICE, "small section pass refused");
    w.ch_key = ch_key;
    w.ch_val = ch_val;
    w.ch_mask = ch_slots - 1;
  } else if (nsections) {
    launch_client_table(w, nsections, s);
    fill_u32_multi({{(uint32_t*)ch_key, 2ull * ch_slots, 0xFFFFFFFFu}}, s);
    launch_client_hash(w, ch_key, ch_val, ch_slots - 1, s);
    w.ch_key = ch_key;
    w.ch_val = ch_val;
    w.ch_mask = ch_slots - 1;
  }
  mark(e, "decode.structs");  // k_struct_decode alone
  if (quick) {
    launch_decode_tail_small(w, NONE, NONE, s);  // (the counts on the device)
    mark(e, "decode.clocks");
  } else if (!lazy && decode_tail_small(w, nstructs, nsections, s)) {
    mark(e, "decode.clocks");  // (one workgroup: structs, clocks, client states, totals)
  } else {
  launch_struct_decode(w, nstructs, s);
  mark(e, "decode.clocks");
  launch_struct_lenscan(w, nstructs, s);
  if (!lazy) {
    fill_u32_multi({{w.cl_start, (uint64_t)nsections + 1, 0u}, {w.cl_state, (uint64_t)nsections + 1, 0u}}, s);
    launch_states(w, nstructs, nsections, s);
  } else {
    HIPCHK(hipMemsetAsync(w.cl_start, 0, sizeof(uint32_t) * (nsections + 1), s));
    launch_struct_clocks(w, nstructs, s);
  }
  }
  HIPCHK(hipStreamWaitEvent(s, e->side_done, 0));
  rc = check(e, c, "struct decode");
  if (quick && rc == YCRDT_E_CAPACITY) return run_decode(e, b, lazy, D, true, sh);  // past a small pass's size
  if (rc) return rc;
  const uint32_t nstructs_q = quick ? c.nstructs : nstructs, nsections_q = quick ? c.nsections : nsections;
  if (c.any_json) {  // ContentJSON / Embed / Format values: JSON.parse (rare: one more pass and sync)
    // room for every struct: one rewrite pass takes all of them (an `any` content is rewritten once)
    w.jcap = std::max<uint32_t>(nstructs_q, 1);
    w.jlist = take<uint32_t>(V, B_JLIST, w.jcap, ok);
    if (!ok) return fail(YCRDT_E_DEVICE, oom("JSON list"));
    w.ntrusted = b->ntrusted;
    w.jskip_any = b->jpasses > 0 ? 1u : 0u;
    launch_json_structs(w, nstructs_q, s);
    rc = check(e, c, "JSON values");
    if (rc) return rc;
    if (c.njson) {  // values Yjs would write back differently: the updates rewritten, then decoded again
      bool restaged = false;
      if ((rc = json_rewrite(e, b, std::min(c.njson, w.jcap), sh, restaged))) return rc;
      if (restaged) return run_decode(e, b, lazy, D, generous, sh);
    }
  }
  D.noncanon = c.noncanon;
  const uint32_t nclients = c.nclients;
  const uint64_t nunits = lazy ? 0 : c.units;
  D.in_len = c.in_len;
  D.array_roots = c.narray_roots;
  D.any_rorigin = c.any_rorigin;
  D.ds_big = c.ds_big != 0;
  D.nested = c.nested;
  D.nroots = 0;
  for (uint32_t k = 0; k < NSHARD; ++k) D.nroots += c.nroots_sh[k];
  if (nunits >= 0xF0000000ull) return fail(YCRDT_E_CAPACITY, "more than 2^32 units in one batch");
  D.nstructs = nstructs_q;
  D.nsections = nsections_q;
  D.nclients = nclients;
  // lazy: the compacted range count; integrate: the ranges stay in their regions (a nonzero
  // region total says there may be some, k_ds_apply reads each update's count)
  D.nds = lazy ? std::min(c.nds, w.cap_ds) : c.ds_region;
  D.nunits = nunits;
  return YCRDT_OK;
}

// The whole batched merge. `target` (optional) selects a delta encode against a state vector;
// `caps` (optional) integrates every client only up to its cap (Yjs pending structs, yc_ingest.h).
// `order` (compat 135): the doc store's client insertion order, the delete-set / state-vector order.
// `sh`: key-hash shards of one document (all of them on this GPU, or this rank's over RCCL).
int comm_allreduce_sum_u32(ycrdt_comm* c, uint32_t* buf, size_t n, hipStream_t s) {
  std::string err;
  if (yc::comm_allreduce_u32(c, buf, n, false, s, err)) return fail(YCRDT_E_DEVICE, err);
  return YCRDT_OK;
}
int run_merge(ycrdt_engine* e, ycrdt_batch* b, const std::unordered_map<uint32_t, uint32_t>* target,
              const ClockMap* caps = nullptr, const std::vector<uint32_t>* order = nullptr, const ShardSpec* sh = nullptr) {
  Work& w = e->w;
  auto& V = e->bufs;
  g_bufs = &V;
  bool ok = true;
  hipStream_t s = e->stream;
  e->ws_owner = nullptr;
  b->packed = false;
  w.capped = 0;
  w.ncaps = 0;
  if (caps) {
    uint32_t* cb = take<uint32_t>(V, B_CAPS, 2 * caps->size() + 2, ok);
    if (!ok) return fail(YCRDT_E_DEVICE, oom("caps"));
    std::vector<uint32_t> h(2 * caps->size() + 2, 0);
    size_t i = 0;
    for (const auto& kv : *caps) { h[i] = kv.first; h[caps->size() + i] = kv.second; ++i; }
    HIPCHK(hipMemcpyAsync(cb, h.data(), sizeof(uint32_t) * h.size(), hipMemcpyHostToDevice, s));
    w.cap_client = cb;
    w.cap_clock = cb + caps->size();
    w.ncaps = (uint32_t)caps->size();
    w.capped = 1;
  }
  Decoded D;
  int rc = run_decode(e, b, false, D, false, sh);
  if (rc) return rc;
  Counters c;
  const uint32_t nstructs = D.nstructs, nclients = D.nclients, nds = D.nds;
  const uint64_t nunits = D.nunits;
  const uint64_t B = (uint64_t)b->nbytes + 64;
  const uint64_t nwords = B / 64 + 2;
  // target state vector → per-client start clocks
  std::vector<uint32_t> vals;
  if (((target && !target->empty()) || order) && nclients) {
    vals.resize(nclients);
    HIPCHK(hipMemcpy(vals.data(), w.cl_vals, sizeof(uint32_t) * nclients, hipMemcpyDeviceToHost));
  }
  w.cl_emit = w.cl_slot = nullptr;
  if (order && nclients) {  // slots: store clients in insertion order, then the rest (no blocks to write)
    std::unordered_map<uint32_t, uint32_t> rank;
    for (size_t i = 0; i < order->size(); ++i) rank.emplace((*order)[i], (uint32_t)i);
    std::vector<uint32_t> h(2 * (size_t)nclients);
    for (uint32_t c = 0; c < nclients; ++c) h[c] = c;
    std::stable_sort(h.begin(), h.begin() + nclients, [&](uint32_t a, uint32_t b2) {
      const auto ia = rank.find(vals[a]), ib = rank.find(vals[b2]);
      const uint32_t ra = ia == rank.end() ? UINT32_MAX : ia->second, rb = ib == rank.end() ? UINT32_MAX : ib->second;
      return ra < rb;
    });
    for (uint32_t i = 0; i < nclients; ++i) h[nclients + h[i]] = i;
    uint32_t* eb = take<uint32_t>(V, B_EMIT, h.size(), ok);
    if (!ok) return fail(YCRDT_E_DEVICE, oom("client order"));
    HIPCHK(hipMemcpyAsync(eb, h.data(), sizeof(uint32_t) * h.size(), hipMemcpyHostToDevice, s));
    w.cl_emit = eb;
    w.cl_slot = eb + nclients;
  }
  w.delta = target && !target->empty() && nclients ? 1u : 0u;
  if (target && !target->empty() && nclients) {
    std::vector<uint32_t> starts(nclients, 0);
    for (uint32_t i = 0; i < nclients; ++i) {
      auto it = target->find(vals[i]);
      if (it != target->end()) starts[i] = it->second;
    }
    HIPCHK(hipMemcpyAsync(w.cl_start, starts.data(), sizeof(uint32_t) * nclients, hipMemcpyHostToDevice, s));
  }
  // ---- per-unit / per-segment buffers
  const uint64_t U = nunits;
  const uint64_t uw = U / 64 + 2;
  w.cap_units = U + 1;
  w.u_owner = take<uint32_t>(V, B_UOWN, U + 1, ok);
  w.u_flags = take<uint32_t>(V, B_UFLAG, U + 1, ok);
  w.u_cutbits = take<uint64_t>(V, B_UCUT, uw, ok);
  w.u_wpre = take<uint32_t>(V, B_UWPRE, uw + 1, ok);
  w.scratch = take<uint32_t>(V, B_SCRATCH, std::max<uint64_t>({nwords + 2, (uint64_t)w.cap_sections + 66, uw + 2, U + 2}), ok);
  w.g_start = take<uint32_t>(V, B_GSTART, U + 2, ok);
  w.g_cidx = take<uint32_t>(V, B_GCIDX, U + 1, ok);
  w.g_src = take<uint32_t>(V, B_GSRC, U + 1, ok);
  w.g_flags = take<uint32_t>(V, B_GFLAGS, U + 1, ok);
  w.g_origin = take<uint32_t>(V, B_GORIG, U + 1, ok);
  w.g_rorigin = take<uint32_t>(V, B_GRORIG, U + 1, ok);
  w.g_hop = take<uint4>(V, B_GLINK, U + 1, ok);
  w.g_key = take<uint32_t>(V, B_GKEY, U + 1, ok);
  w.g_maxchild = take<uint32_t>(V, B_GMAXC, U + 1, ok);
  w.g_outid = take<uint32_t>(V, B_GOUTID, U + 2, ok);
  w.g_tmp = take<uint32_t>(V, B_GTMP, U + 2, ok);
  w.g_tmp2 = take<uint32_t>(V, B_GTMP2, U + 2, ok);
  w.o_first = take<uint32_t>(V, B_OFIRST, U + 2, ok);
  w.o_cidx = take<uint32_t>(V, B_OCIDX, U + 2, ok);
  w.o_size = take<uint32_t>(V, B_OSIZE, U + 2, ok);
  w.o_pos = take<uint32_t>(V, B_OPOS, U + 2, ok);
  w.o_gen = take<uint8_t>(V, B_OGEN, U + 32, ok);  // (whole 16-byte quads: for_deferred)
  w.r_seg = take<uint32_t>(V, B_RSEG, U + 2, ok);
  w.r_len = take<uint32_t>(V, B_RLEN, U + 2, ok);
  w.r_size = take<uint32_t>(V, B_RSIZE, U + 2, ok);
  w.r_pos = take<uint32_t>(V, B_RPOS, U + 2, ok);
  w.cc = take<uint32_t>(V, B_CC, (size_t)CC_N * (w.cap_clients + 1), ok);
  w.cc64 = take<uint64_t>(V, B_CC64, (size_t)CC64_N * (w.cap_clients + 1), ok);
  {
    // scans up to the units; sorts: the client table (YATA's sorts over segments grow it, alloc_lists)
    size_t tb = prim_tmp_bytes(std::max<uint64_t>({B / 64 + 4, U + 2, (uint64_t)nstructs + 2, 1024}), (uint64_t)D.nsections + 2);
    w.tmp = take<uint8_t>(V, B_TMP, tb, ok);
    w.tmp_bytes = V[B_TMP].cap;
  }
  if (!ok) return fail(YCRDT_E_DEVICE, oom("unit workspace"));
  // ---- K2..K5 units
  mark(e, "merge.units_fill");
  if (U || nds) launch_units_fill(w, U, s);
  mark(e, "merge.units");  // k_units alone
  // with no units, delete-set ranges still have to be checked: each one is pending (pendingDs)
  {  // long delete-set runs spread over the grid (k_ds_tails; YCRDT_DS_TAILS=0: A/B); without the
     // buffer every run is flagged by the wavefront that met it
    bool okt = true;
    w.ds_tails = D.ds_big && !env_off("YCRDT_DS_TAILS") ? take<uint4>(V, B_DSTAILS, DS_TAILS_CAP, okt) : nullptr;
    if (!okt) w.ds_tails = nullptr;
  }
  if (U || nds) launch_units(w, nstructs, nclients, nds, U, D.ds_big, s);
  mark(e, "merge.segments");
  uint32_t nsegs = 0;
  // A small map-only merge (the per-op path: no YArray, no right origin, no nested type, one GPU)
  // runs the integrate phases and the encode as two single-workgroup launches that read the
  // segment count on the device: no count synchronisation (a ~25 us round trip per merge), the
  // key table and output sized from the unit count (segments <= units)
  const bool small = U && !sh && !D.array_roots && !D.any_rorigin && !D.nested && merge_small_fits(U) &&
                     encode_small_fits(U, nclients) && (uint64_t)b->in_bytes + 48ull * U + 32ull * nclients + 64 <= (uint64_t(1) << 30);
  if (U && !small) {  // (a small merge cuts its segments in k_merge_small)
    launch_segments(w, nclients, U, s);
    rc = check(e, c, "segments");
    if (rc) return rc;
    nsegs = c.nsegs;
  }
  const uint64_t nseg_bound = small ? U : nsegs;
  // keys
  // every list is rooted by an explicit-parent item (a key per root struct at most): the table is
  // sized from those, not from every segment
  w.cap_keys = next_pow2(std::max<uint64_t>(2ull * std::min<uint64_t>(D.nroots, nseg_bound), 64));
  {  // test hook: keep only the low YCRDT_KEY_HASH_BITS bits of every list hash (collisions certain)
    const int kb = getenv("YCRDT_KEY_HASH_BITS") ? atoi(getenv("YCRDT_KEY_HASH_BITS")) : 64;
    w.key_mask = kb >= 1 && kb < 64 ? (1ull << kb) - 1 : ~0ull;
  }
  w.k_hash = take<uint64_t>(V, B_KHASH, w.cap_keys, ok);
  w.k_rootmax = take<uint32_t>(V, B_KROOT, w.cap_keys, ok);
  w.k_winner = take<uint32_t>(V, B_KWIN, w.cap_keys, ok);
  w.k_parent = take<uint32_t>(V, B_KPAR, w.cap_keys, ok);
  w.k_flags = take<uint32_t>(V, B_KFLAG, w.cap_keys, ok);
  if (!ok) return fail(YCRDT_E_DEVICE, oom("key table"));
  // the YArray arrays (yc_yata.hip, the view's list order) exist only for a merge with YArray
  // members: a map-only merge (C2) never touches them, and at a billion units they would be
  // a hundred gigabytes of HBM
  auto alloc_lists = [&](uint64_t n) -> bool {
    bool okl = true;
    w.g_right = take<uint32_t>(V, B_GRIGHT, n + 2, okl);
    uint32_t** cols[] = {&w.y_key, &w.y_keys, &w.y_seg, &w.y_iota, &w.y_lstart, &w.y_state, &w.y_before, &w.y_confl,
                         &w.y_stack, &w.t_key, &w.t_keys, &w.t_seg, &w.t_pos, &w.t_gstart, &w.t_next, &w.t_done,
                         &w.t_first, &w.t_nsib, &w.t_jump, &w.t_big, &w.t_prv, &w.t_mprv, &w.t_mtail, &w.t_trep, &w.t_otail};
    const int ids[] = {B_YKEY, B_YKEYS, B_YSEG, B_YIOTA, B_YLSTART, B_YSTATE, B_YBEFORE, B_YCONFL, B_YSTACK,
                       B_TKEY, B_TKEYS, B_TSEG, B_TPOS, B_TGSTART, B_TNEXT, B_TDONE, B_TFIRST, B_TNSIB, B_TJUMP,
                       B_TBIG, B_TPRV, B_TMPRV, B_TMTAIL, B_TTREP, B_TOTAIL};
    for (size_t k = 0; k < sizeof(ids) / sizeof(ids[0]); ++k) *cols[k] = take<uint32_t>(V, ids[k], n + 2, okl);
    w.t_hkey = take<uint32_t>(V, B_THKEY, 2 * n + 4, okl);
    w.t_hval = take<uint32_t>(V, B_THVAL, 2 * n + 4, okl);
    w.t_flag = take<uint32_t>(V, B_TFLAG, 2 * n + 4, okl);  // flags, then their scan behind them
    // YATA sorts the segments (sibling groups, list members)
    w.tmp = take<uint8_t>(V, B_TMP, prim_tmp_bytes(std::max<uint64_t>({B / 64 + 4, U + 2, (uint64_t)nstructs + 2, 1024}), n + 2), okl);
    w.tmp_bytes = V[B_TMP].cap;
    return okl;
  };
  uint32_t nout = 0;
  bool runs_scanned = false;  // (k_merge_flags made the delete-set run ids)
  e->nsegs = nsegs;
  e->nlists = 0;
  if (small) {
    // key table, segment properties, resolution, winners and merge flags (yc_merge.hip k_merge_small)
    mark(e, "merge.small");
    launch_merge_small(w, NONE, U, s);
  } else if (nsegs) {
    mark(e, "merge.segment_fill");
    launch_segment_props_fill(w, nsegs, s);
    mark(e, "merge.segment_props");  // k_seg_props alone
    launch_segment_props(w, nsegs, nclients, U, s);
    mark(e, "merge.resolve");  // k_resolve alone
    run_key_resolution(w, nsegs, s);
    uint32_t narray = 0;  // YArray members; only read when the decode saw a possible array root
    uint32_t nmapx = 0;   // a YMap entry that needs full YATA (only with a right origin somewhere)
    if (D.array_roots || D.any_rorigin) {
      uint32_t h2[2];
      static_assert(offsetof(Counters, nmapx) == offsetof(Counters, narray) + 4, "read together");
      HIPCHK(hipMemcpyAsync(h2, &w.ctr->narray, sizeof(h2), hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      narray = h2[0];
      nmapx = h2[1];
    }
    if (nmapx) {
      launch_mapx_flip(w, nsegs, s);
      narray = 1;
    }
    if (narray && !alloc_lists(nsegs)) return fail(YCRDT_E_DEVICE, oom("list workspace"));
    // the integrate phases: once, or once per key-hash shard (sh: C4 sharding, §6 of DESIGN.md)
    uint8_t* owner = nullptr;
    uint32_t *gflags0 = nullptr, *acc = nullptr;
    uint32_t first = 0, last = 1;
    if (sh) {
      uint32_t* key_shard = take<uint32_t>(V, B_KSHARD, w.cap_keys + 1, ok);
      owner = take<uint8_t>(V, B_SOWNER, (size_t)nsegs + 16, ok);
      gflags0 = take<uint32_t>(V, B_GFLAGS0, (size_t)nsegs + 1, ok);
      acc = take<uint32_t>(V, B_GFACC, (size_t)nsegs + 1, ok);
      if (!ok) return fail(YCRDT_E_DEVICE, oom("shards"));
      mark(e, "shard.owners");
      launch_key_shards(w, nsegs, sh->nshards, key_shard, owner, s);
      HIPCHK(hipMemcpyAsync(gflags0, w.g_flags, sizeof(uint32_t) * nsegs, hipMemcpyDeviceToDevice, s));
      HIPCHK(hipMemsetAsync(acc, 0, sizeof(uint32_t) * (nsegs + 1), s));
      first = sh->shard < 0 ? 0u : (uint32_t)sh->shard;
      last = sh->shard < 0 ? sh->nshards : first + 1;
    }
    for (uint32_t shard = first; shard < last; ++shard) {
      if (sh) {
        // a logical shard after the first: the pristine flags (the winner slots were settled for
        // every list in k_resolve: a list's children never leave its shard)
        if (shard != first) HIPCHK(hipMemcpyAsync(w.g_flags, gflags0, sizeof(uint32_t) * nsegs, hipMemcpyDeviceToDevice, s));
        launch_shard_mask(w, nsegs, owner, shard, s);
      }
      mark(e, "merge.descent");
      run_descent(w, nsegs, s, !D.nested);  // no dead-type pass: merge flags apply the overwrite
      mark(e, "merge.dead_types");
      if (D.nested) run_dead_keys(w, nsegs, s);  // only lists under a parent item can die with it
      mark(e, "merge.yata");
      e->nlists = launch_yata(w, nsegs, narray, nclients, s, e->side, e->side_fork, e->side_done);
      if (nmapx) launch_mapx_fix(w, nsegs, s);
      if (w.dbg && e->nlists) {
        unsigned long long h[7];
        HIPCHK(hipStreamSynchronize(s));
        HIPCHK(hipMemcpy(h, w.dbg, sizeof(h), hipMemcpyDeviceToHost));
        fprintf(stderr, "[ycrdt] k_yata: %llu integrations, %llu conflict-scan steps, %llu stack dives | huge sibling loop: %llu placements, %llu group-list steps, %llu left steps, %llu dives\n",
                h[0], h[1], h[2], h[3], h[4], h[5], h[6]);
      }
      mark(e, "merge.merge_flags");
      if (!sh) {
        runs_scanned = launch_merge_flags(w, nsegs, s, !D.nested);
      } else {
        launch_merge_flags_only(w, nsegs, s, !D.nested);
        launch_shard_export(w, nsegs, owner, shard, acc, s);
      }
    }
    if (sh) {  // combine: every segment's flags come from its owner (RCCL sum across GPUs)
      mark(e, "shard.exchange");
      if (sh->comm) {
        // every rank reports before the data collective: a rank that failed earlier joins only
        // this agreement (ycrdt_batch_merge_sharded), so no peer waits in a sum it never enters
        if (const int rc1 = shard_agree(sh, s)) return rc1;
        const int rc2 = comm_allreduce_sum_u32(sh->comm, acc, nsegs, s);
        if (rc2) return rc2;
        sh->inside = false;
        sh->finished = true;  // the merge's last exchange
      }
      HIPCHK(hipMemcpyAsync(w.g_flags, acc, sizeof(uint32_t) * nsegs, hipMemcpyDeviceToDevice, s));
      launch_merge_final(w, nsegs, s);
      e->nlists = 0;  // the view is not built from a sharded merge
    }
  }
  // ---- K7 encode. Output bound: every output struct adds at most 37 bytes of header (info,
  // origin, right origin, parent, length prefix) to content bytes sliced from the input, every
  // delete-set run at most 10, every client block / state-vector entry at most 15 + 10.
  if (!nsegs && !small) HIPCHK(hipMemsetAsync(&w.ctr->nout, 0, sizeof(uint32_t), s));
  w.cap_out = (uint64_t)b->in_bytes + 48ull * nseg_bound + 32ull * nclients + 64;
  w.cap_sv = 16ull + 10ull * nclients;
  // up to 1 GiB of bound the output is allocated before the sizes are known; past it (a merge of
  // billions of items: the bound is several times the input) after them, exactly (one more sync)
  const bool exact_out = w.cap_out > (uint64_t(1) << 30);
  if (!exact_out) w.out = take<uint8_t>(V, B_OUT, (size_t)w.cap_out + 16, ok);
  w.sv_out = take<uint8_t>(V, B_SVOUT, (size_t)w.cap_sv + 16, ok);
  if (!ok) return fail(YCRDT_E_DEVICE, oom("output"));
  uint8_t* tmp2 = take<uint8_t>(V, B_TMP2, prim_tmp_bytes(nseg_bound + 2, 0), ok);
  if (!ok) return fail(YCRDT_E_DEVICE, oom("scan space"));
  mark(e, "encode.runs");
  if (small || (!exact_out && encode_small_fits(nsegs, nclients))) {
    launch_encode_small(w, small ? NONE : nsegs, nclients, s);  // (the whole encode, one workgroup)
    mark(e, "end");
  } else {
  launch_encode_sizes(w, nsegs, nclients, s, e->side, e->side_fork, e->side_done, tmp2, V[B_TMP2].cap, runs_scanned);
  mark(e, "encode.sizes");  // k_out_sizes alone
  launch_out_sizes(w, nsegs, nclients, s);
  mark(e, "encode.layout");
  launch_encode_layout(w, nsegs, nclients, s, e->side_done);
  if (exact_out) {
    rc = check(e, c, "encode sizes");
    if (rc) return rc;
    w.cap_out = c.out_total;
    w.out = take<uint8_t>(V, B_OUT, (size_t)w.cap_out + 16, ok);
    if (!ok) return fail(YCRDT_E_DEVICE, oom("output"));
  }
  mark(e, "encode.write");  // k_write_structs alone
  launch_write_structs(w, nsegs, nclients, s);
  mark(e, "encode.write_tail");
  launch_encode_write(w, nsegs, nclients, s);
  mark(e, "end");
  }
  HIPCHK(hipEventRecord(e->ev1, s));
  if (e->before_final)
    if (const int r = (*e->before_final)(w.cap_out, w.cap_sv)) return r;
  rc = check(e, c, "merge / encode");
  if (rc) return rc;
  if (small) {
    nsegs = c.nsegs;
    e->nsegs = nsegs;
  }
  nout = nsegs ? c.nout : 0;
  e->out_bytes = c.out_total;
  e->sv_bytes = c.sv_bytes;
  float ms = 0;
  hipEventElapsedTime(&ms, e->ev0, e->ev1);
  ycrdt_merge_stats& st = e->last;
  st.in_bytes = b->in_bytes;
  st.items = nstructs ? D.in_len - c.items : 0;  // Item + GC clock lengths (Skip excluded)
  st.structs = nstructs;
  st.units = U;
  st.segments = nsegs;
  st.out_structs = nout;
  st.out_bytes = c.out_total;
  st.clients = nclients;
  st.device_ms = ms;
  if (e->profiling) {
    for (size_t i = 0; i + 1 < e->marks.size(); ++i) {
      float t = 0;
      hipEventElapsedTime(&t, e->marks[i].second, e->marks[i + 1].second);
      e->phase_ms.push_back({e->marks[i].first, (double)t});
    }
  }
  return YCRDT_OK;
}

// K8: materialised view of the doc state just merged into the engine's workspace (yc_view.hip),
// copied to the host with the state bytes its byte ranges point into.
int run_view(ycrdt_engine* e, ycrdt_batch* b, HostView& hv) {
  if (b->nwin > 1) return fail(YCRDT_E_CAPACITY, "a view of a batch over 4 GiB");
  Work& w = e->w;
  auto& V = e->bufs;
  g_bufs = &V;
  bool ok = true;
  hipStream_t s = e->stream;
  if (e->nlists == LISTS_UNNUMBERED) e->nlists = launch_ylists(w, e->nsegs, s);  // (the merge's tree path skipped it)
  const uint32_t nsegs = e->nsegs, nlists = e->nlists;
  uint32_t narr = 0;
  if (nlists) {
    HIPCHK(hipMemcpyAsync(&narr, w.y_lstart + nlists, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
  }
  ViewBufs vb;
  const size_t ck = std::max<uint32_t>(w.cap_keys, 1);
  vb.kmap = take<uint32_t>(V, B_VKMAP, ck, ok);
  vb.krep = take<uint32_t>(V, B_VKREP, ck, ok);
  vb.keys = take<ViewKey>(V, B_VKEYS, ck, ok);
  vb.nkeys = take<uint32_t>(V, B_VNKEYS, 4, ok);
  vb.pos_of = take<uint32_t>(V, B_VPOS, (size_t)nsegs + 1, ok);
  vb.d0 = take<uint32_t>(V, B_VD0, (size_t)narr + 1, ok);
  vb.n0 = take<uint32_t>(V, B_VN0, (size_t)narr + 1, ok);
  vb.d1 = take<uint32_t>(V, B_VD1, (size_t)narr + 1, ok);
  vb.n1 = take<uint32_t>(V, B_VN1, (size_t)narr + 1, ok);
  vb.order = take<uint32_t>(V, B_VORDER, (size_t)narr + 1, ok);
  vb.segs = take<ViewSeg>(V, B_VSEGS, (size_t)narr + 1, ok);
  if (!ok) return fail(YCRDT_E_DEVICE, oom("view"));
  hv.keys.clear();
  hv.segs.clear();
  hv.bytes.assign(b->nbytes, 0);
  if (nsegs) {
    launch_view(w, vb, nsegs, nlists, narr, s);
    // a small view (the per-op path's doc) comes back in ONE synchronisation: counters, key count,
    // the key table up to its capacity, the list segments and the state bytes, queued together
    // (each synchronous copy cost a ~25 us round trip); a large one sizes the key copy first
    static const bool big_only = getenv("YCRDT_VIEW_SYNC") && getenv("YCRDT_VIEW_SYNC")[0] == '1';
    const bool small = !big_only && (uint64_t)ck * sizeof(ViewKey) <= (256u << 10);
    Counters c;
    uint32_t nkeys = 0;
    hv.segs.resize(narr);
    // (the small view's pieces land in the pinned read-back area, 256-byte aligned)
    auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
    const size_t o_keys = al(sizeof(Counters) + 4), o_segs = o_keys + al(sizeof(ViewKey) * ck),
                 o_bytes = o_segs + al(sizeof(ViewSeg) * narr), rb_need = o_bytes + b->nbytes;
    if (small && rb_need > e->rb_cap) {
      if (e->rb) hipHostFree(e->rb);
      e->rb_cap = 0;
      if (hipHostMalloc((void**)&e->rb, std::max<size_t>(rb_need, size_t(1) << 20), hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        e->rb = nullptr;
        return fail(YCRDT_E_DEVICE, "pinned view read-back allocation failed");
      }
      e->rb_cap = std::max<size_t>(rb_need, size_t(1) << 20);
    }
    if (small) {
      HIPCHK(hipMemcpyAsync(e->rb, w.ctr, sizeof(Counters), hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(e->rb + sizeof(Counters), vb.nkeys, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(e->rb + o_keys, vb.keys, sizeof(ViewKey) * ck, hipMemcpyDeviceToHost, s));
      if (narr) HIPCHK(hipMemcpyAsync(e->rb + o_segs, vb.segs, sizeof(ViewSeg) * narr, hipMemcpyDeviceToHost, s));
      if (b->nbytes) HIPCHK(hipMemcpyAsync(e->rb + o_bytes, b->bytes.p, b->nbytes, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      memcpy(&c, e->rb, sizeof(Counters));
      memcpy(&nkeys, e->rb + sizeof(Counters), sizeof(uint32_t));
    } else {
      HIPCHK(hipMemcpyAsync(&c, w.ctr, sizeof(Counters), hipMemcpyDeviceToHost, s));
      HIPCHK(hipMemcpyAsync(&nkeys, vb.nkeys, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
    }
    if (c.err) return map_err(c.err, "view");
    if (nkeys > ck) return fail(YCRDT_E_DEVICE, "view: key count past the key table");
    if (small) {
      hv.keys.resize(nkeys);
      if (nkeys) memcpy(hv.keys.data(), e->rb + o_keys, sizeof(ViewKey) * nkeys);
      if (narr) memcpy(hv.segs.data(), e->rb + o_segs, sizeof(ViewSeg) * narr);
      if (b->nbytes) memcpy(hv.bytes.data(), e->rb + o_bytes, b->nbytes);
    } else {
      hv.keys.resize(nkeys);
      if (nkeys) HIPCHK(hipMemcpy(hv.keys.data(), vb.keys, sizeof(ViewKey) * nkeys, hipMemcpyDeviceToHost));
      if (narr) HIPCHK(hipMemcpy(hv.segs.data(), vb.segs, sizeof(ViewSeg) * narr, hipMemcpyDeviceToHost));
      if (b->nbytes) HIPCHK(hipMemcpy(hv.bytes.data(), b->bytes.p, b->nbytes, hipMemcpyDeviceToHost));
    }
  } else if (b->nbytes) {
    HIPCHK(hipMemcpy(hv.bytes.data(), b->bytes.p, b->nbytes, hipMemcpyDeviceToHost));
  }
  hv.index();
  hv.valid = true;
  return YCRDT_OK;
}

// mergeUpdates (merge = true) or diffUpdate (merge = false, target state vector given) of a
// staged batch; the encoded update is copied to `out`.
// Per-update outputs of a multi diff: [varuint blocks][its sections' blocks, in byte order]
// [varuint delete-set clients][its delete-set groups]. Sections are appended by the walkers per
// update (updates interleave), delete-set rows were sorted by (update, client desc).
int split_multi(ycrdt_engine* e, const Decoded& D, uint32_t nr, uint32_t sbytes, uint32_t total, ycrdt_out* outs) {
  Work& w = e->w;
  const uint32_t nsec = D.nsections;
  std::unique_ptr<uint8_t[]> all(new uint8_t[total ? total : 1]);
  std::vector<Section> sec(nsec);
  std::vector<uint32_t> evn(nsec), bpos(nsec + 1), dflag(nr), dpos(nr + 1);
  std::vector<uint64_t> dkey(nr);
  if (total) HIPCHK(hipMemcpyAsync(all.get(), w.out, total, hipMemcpyDeviceToHost, e->stream));
  if (nsec) {
    HIPCHK(hipMemcpyAsync(sec.data(), w.sections, sizeof(Section) * nsec, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(evn.data(), w.lz_evn, sizeof(uint32_t) * nsec, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(bpos.data(), w.blk_pos, sizeof(uint32_t) * (nsec + 1), hipMemcpyDeviceToHost, e->stream));
  }
  if (nr) {
    HIPCHK(hipMemcpyAsync(dflag.data(), w.dw_flag, sizeof(uint32_t) * nr, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(dpos.data(), w.dw_pos, sizeof(uint32_t) * (nr + 1), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(dkey.data(), w.dsm_keys, sizeof(uint64_t) * nr, hipMemcpyDeviceToHost, e->stream));
  }
  HIPCHK(hipStreamSynchronize(e->stream));
  const uint32_t nupd = w.nupd;
  // non-empty sections grouped by update (counting sort), in byte order within an update
  std::vector<uint32_t> cnt(nupd + 1, 0), idx;
  for (uint32_t i = 0; i < nsec; ++i) {
    if (sec[i].upd >= nupd) return fail(YCRDT_E_DEVICE, "diff batch: section of an unknown update");
    if (evn[i]) ++cnt[sec[i].upd + 1];
  }
  for (uint32_t u = 0; u < nupd; ++u) cnt[u + 1] += cnt[u];
  idx.resize(cnt[nupd]);
  {
    std::vector<uint32_t> cur(cnt.begin(), cnt.end() - 1);
    for (uint32_t i = 0; i < nsec; ++i)
      if (evn[i]) idx[cur[sec[i].upd]++] = i;
  }
  uint8_t hdr[2][5];
  auto vu = [](uint8_t* o, uint32_t v) {
    uint32_t n = 0;
    while (v >= 0x80u) { o[n++] = (uint8_t)(v | 0x80u); v >>= 7; }
    o[n++] = (uint8_t)v;
    return n;
  };
  uint32_t r = 0;
  for (uint32_t u = 0; u < nupd; ++u) {
    uint32_t* a = idx.data() + cnt[u];
    uint32_t* b = idx.data() + cnt[u + 1];
    std::sort(a, b, [&](uint32_t x, uint32_t y) { return sec[x].first_pos < sec[y].first_pos; });
    uint32_t blk = 0;
    for (uint32_t* q = a; q < b; ++q) blk += bpos[*q + 1] - bpos[*q];
    const uint32_t r0 = r;
    uint32_t ng = 0;
    while (r < nr && (uint32_t)(dkey[r] >> 32) == u) { ng += dflag[r]; ++r; }
    uint32_t heads = 0;  // a block of the client of the block before it continues that section (k_blk_sizes)
    for (uint32_t* q = a; q < b; ++q) heads += q == a || sec[*q].client != sec[q[-1]].client;
    const uint32_t h0 = vu(hdr[0], heads), h1 = vu(hdr[1], ng);
    const size_t len = (size_t)h0 + blk + h1 + (dpos[r] - dpos[r0]);
    uint8_t* o = (uint8_t*)malloc(len ? len : 1);
    if (!o) {
      for (uint32_t k = 0; k < u; ++k) { free(outs[k].ptr); outs[k].ptr = nullptr; outs[k].len = 0; }
      return fail(YCRDT_E_CAPACITY, "diff batch: host allocation failed");
    }
    size_t p = 0;
    memcpy(o, hdr[0], h0); p += h0;
    for (uint32_t* q = a; q < b; ++q) { memcpy(o + p, all.get() + bpos[*q], bpos[*q + 1] - bpos[*q]); p += bpos[*q + 1] - bpos[*q]; }
    memcpy(o + p, hdr[1], h1); p += h1;
    memcpy(o + p, all.get() + sbytes + dpos[r0], dpos[r] - dpos[r0]);
    outs[u].ptr = o;
    outs[u].len = len;
  }
  if (r != nr) {
    for (uint32_t u = 0; u < nupd; ++u) { free(outs[u].ptr); outs[u].ptr = nullptr; outs[u].len = 0; }
    return fail(YCRDT_E_DEVICE, "diff batch: delete-set rows out of update order");
  }
  return YCRDT_OK;
}

// With sv_off (diff only): update u is diffed against sv[sv_off[u] .. sv_off[u+1]) and `multi`
// receives one encoded update per input update (the kernels write header-less block and
// delete-set bytes; the per-update headers are written here while the bytes are split).
int run_lazy(ycrdt_engine* e, ycrdt_batch* b, bool merge, const std::vector<std::pair<uint32_t, uint32_t>>& sv,
             ycrdt_out* out, const std::vector<uint32_t>* sv_off = nullptr,
             ycrdt_out* multi = nullptr) {
  if (b->nwin > 1) return fail(YCRDT_E_CAPACITY, "mergeUpdates / diffUpdate of more than 4 GiB");
  Work& w = e->w;
  w.lz_multi = 0;
  w.capped = 0;
  w.ds_first = e->compat == 135 ? 1u : 0u;
  e->ws_owner = nullptr;
  auto& V = e->bufs;
  g_bufs = &V;
  bool ok = true;
  hipStream_t s = e->stream;
  Decoded D;
  int rc = run_decode(e, b, true, D);
  if (rc) return rc;
  Counters c;
  const uint64_t NSEC = D.nsections + 2, NC = D.nclients + 2;
  const bool seq = merge && D.noncanon;  // the serial mergeUpdates loop: output sections follow the events
  const uint64_t NBLK0 = (merge ? D.nclients : D.nsections) + 2;
  const uint64_t SLOTS = 2ull * D.nstructs + 2ull * NBLK0 + 4;
  const uint64_t NBLK = seq ? SLOTS + 2 : NBLK0;
  const uint64_t NDS = D.nds + 2;
  w.lz_key = take<uint64_t>(V, B_LZKEY, NSEC, ok);
  w.lz_keys = take<uint64_t>(V, B_LZKEYS, NSEC, ok);
  w.lz_iota = take<uint32_t>(V, B_LZIOTA, NSEC, ok);
  w.lz_sec = take<uint32_t>(V, B_LZSEC, NSEC, ok);
  w.lz_rstart = take<uint32_t>(V, B_LZRSTART, NC, ok);
  w.lz_prev = take<uint32_t>(V, B_LZPREV, NSEC, ok);
  w.lz_first = take<uint32_t>(V, B_LZFIRST, NSEC, ok);
  w.lz_cap = take<uint32_t>(V, B_LZCAP, NBLK, ok);
  w.lz_evbase = take<uint32_t>(V, B_LZEVBASE, NBLK, ok);
  w.lz_evn = take<uint32_t>(V, B_LZEVN, NBLK, ok);
  w.lz_bclient = seq ? take<uint32_t>(V, B_LZBCLIENT, NBLK, ok) : nullptr;
  w.lz_flag = take<uint32_t>(V, B_LZFLAG, NSEC, ok);
  w.lz_leave_hi = take<uint32_t>(V, B_LZLHI, NSEC, ok);
  w.lz_leave_lo = take<uint32_t>(V, B_LZLLO, NSEC, ok);
  w.ev_kind = take<uint32_t>(V, B_EVKIND, SLOTS, ok);
  w.ev_src = take<uint32_t>(V, B_EVSRC, SLOTS, ok);
  w.ev_clock = take<uint32_t>(V, B_EVCLOCK, SLOTS, ok);
  w.ev_len = take<uint32_t>(V, B_EVLEN, SLOTS, ok);
  w.ev_size = take<uint32_t>(V, B_EVSIZE, SLOTS, ok);
  w.ev_pos = take<uint32_t>(V, B_EVPOS, SLOTS, ok);
  w.blk_size = take<uint32_t>(V, B_BLKSIZE, NBLK, ok);
  w.blk_pos = take<uint32_t>(V, B_BLKPOS, NBLK, ok);
  w.dsm_key = take<uint64_t>(V, B_DSMKEY, NDS, ok);
  w.dsm_keys = take<uint64_t>(V, B_DSMKEYS, NDS, ok);
  w.dsm_len = take<uint32_t>(V, B_DSMLEN, NDS, ok);
  w.dsm_lens = take<uint32_t>(V, B_DSMLENS, NDS, ok);
  w.dsm_end = take<uint64_t>(V, B_DSMEND, NDS, ok);
  w.dsm_max = take<uint64_t>(V, B_DSMMAX, NDS, ok);
  w.dsm_flag = take<uint32_t>(V, B_DSMFLAG, NDS, ok);
  w.dsm_rid = take<uint32_t>(V, B_DSMRID, NDS, ok);
  w.dr_client = take<uint32_t>(V, B_DRCLIENT, NDS, ok);
  w.dr_clock = take<uint32_t>(V, B_DRCLOCK, NDS, ok);
  w.dr_end = take<uint32_t>(V, B_DREND, NDS, ok);
  w.dw_flag = take<uint32_t>(V, B_DWFLAG, NDS, ok);
  w.dw_gid = take<uint32_t>(V, B_DWGID, NDS, ok);
  w.dw_gstart = take<uint32_t>(V, B_DWGSTART, NDS, ok);
  w.dw_size = take<uint32_t>(V, B_DWSIZE, NDS, ok);
  w.dw_pos = take<uint32_t>(V, B_DWPOS, NDS, ok);
  w.ds_fa = w.ds_first ? take<uint32_t>(V, B_DSFA, NDS, ok) : nullptr;
  {
    size_t tb = prim_tmp_bytes(std::max<uint64_t>({((uint64_t)b->nbytes + 64) / 64 + 4, SLOTS, NDS, NSEC, 1024}),
                               std::max<uint64_t>(NSEC, NDS));
    w.tmp = take<uint8_t>(V, B_TMP, tb, ok);
    w.tmp_bytes = V[B_TMP].cap;
  }
  const size_t nsvo = sv_off ? sv_off->size() : 0;
  uint32_t* svbuf = take<uint32_t>(V, B_SVC, 2 * sv.size() + nsvo + 2, ok);
  if (!ok) return fail(YCRDT_E_DEVICE, oom("lazy merge workspace"));
  if (merge) {
    mark(e, "lazy.merge");
    if (seq) launch_lazy_merge_seq(w, (uint32_t)SLOTS, (uint32_t)(NBLK - 1), s);
    else if (D.nsections) launch_lazy_merge(w, D.nsections, D.nclients, s);
    else { w.lz_nblk = 0; w.lz_diff = 0; HIPCHK(hipMemsetAsync(w.lz_evbase, 0, sizeof(uint32_t) * 2, s)); }
  } else {
    std::vector<uint32_t> h(2 * sv.size() + nsvo + 2, 0);
    for (size_t i = 0; i < sv.size(); ++i) { h[i] = sv[i].first; h[sv.size() + i] = sv[i].second; }
    for (size_t i = 0; i < nsvo; ++i) h[2 * sv.size() + i] = (*sv_off)[i];
    HIPCHK(hipMemcpyAsync(svbuf, h.data(), sizeof(uint32_t) * h.size(), hipMemcpyHostToDevice, s));
    w.sv_client = svbuf;
    w.sv_clock = svbuf + sv.size();
    w.sv_n = (uint32_t)sv.size();
    w.sv_off = sv_off ? svbuf + 2 * sv.size() : nullptr;
    w.lz_multi = sv_off ? 1u : 0u;
    mark(e, "lazy.diff");
    if (D.nsections) launch_lazy_diff(w, D.nsections, s);
    else { w.lz_nblk = 0; w.lz_diff = 1; HIPCHK(hipMemsetAsync(w.lz_evbase, 0, sizeof(uint32_t) * 2, s)); }
  }
  rc = check(e, c, merge ? "mergeUpdates" : "diffUpdate");
  if (rc) return rc;
  if (seq) w.lz_nblk = c.lz_blocks;
  mark(e, "lazy.sizes");
  uint32_t nslots = 0;
  if (w.lz_nblk) launch_event_sizes(w, s, &nslots);
  else HIPCHK(hipMemsetAsync(w.ctr->pad, 0, sizeof(uint32_t) * 8, s));
  const uint32_t nr = launch_ds_runs(w, D.nds, merge, s);
  const uint32_t dsbytes = launch_ds_write_sizes(w, nr, s);
  rc = check(e, c, "lazy sizes");
  if (rc) return rc;
  uint32_t blk_total = 0;
  if (w.lz_nblk) {
    HIPCHK(hipMemcpyAsync(&blk_total, w.blk_pos + w.lz_nblk, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
  }
  const uint32_t sbytes = vu_size_host(c.pad[0]) + blk_total;
  const uint32_t total = sbytes + dsbytes;
  w.out = take<uint8_t>(V, B_OUT, (size_t)total + 16, ok);
  if (!ok) return fail(YCRDT_E_DEVICE, oom("output"));
  mark(e, "lazy.write");
  if (w.lz_nblk) launch_lazy_write(w, nslots, nr, sbytes, s);
  else {
    const uint8_t zero[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(w.out, zero, 1, hipMemcpyHostToDevice, s));
    if (nr) launch_lazy_write(w, 0, nr, sbytes, s);
    else HIPCHK(hipMemcpyAsync(w.out + 1, zero, 1, hipMemcpyHostToDevice, s));
  }
  mark(e, "end");
  HIPCHK(hipEventRecord(e->ev1, s));
  rc = check(e, c, "lazy write");
  if (rc) return rc;
  if (e->profiling) {  // phase times of the lazy pipeline (stage .. last kernel, host syncs included)
    for (size_t i = 0; i + 1 < e->marks.size(); ++i) {
      float t = 0;
      hipEventElapsedTime(&t, e->marks[i].second, e->marks[i + 1].second);
      e->phase_ms.push_back({e->marks[i].first, (double)t});
    }
  }
  if (multi) return split_multi(e, D, nr, sbytes, total, multi);
  out->len = total;
  out->ptr = (uint8_t*)malloc(total ? total : 1);
  if (!out->ptr) { out->len = 0; return fail(YCRDT_E_CAPACITY, "host allocation failed"); }
  HIPCHK(hipMemcpy(out->ptr, w.out, total, hipMemcpyDeviceToHost));
  return YCRDT_OK;
}

// Multi-document merge result, split per document on the host. The encoder lays clients out in
// descending (document, client) order, so every document's struct blocks, delete-set blocks and
// state-vector entries are contiguous; each document's update is its blocks behind its own
// varuint counts (writeClientsStructs / writeDeleteSet / writeStateVector headers).
// Device-side split of a merged multi-document batch: every document's update ([varuint struct
// blocks][its blocks][varuint delete-set clients][its delete-set groups]) and state vector laid
// out back to back in one HBM buffer (B_PACK) by one piece-copy launch, the varuint headers
// written inline; b->pack_offs holds the boundaries. Clients are encoded in (document, client)
// descending order, so each document's sections are contiguous ranges (k_doc_ranges).
constexpr uint32_t PIECE_MAX = 16384;  // large ranges are cut so no wavefront copies megabytes alone
int pack_docs(ycrdt_engine* e, ycrdt_batch* b) {
  if (b->packed) return YCRDT_OK;
  Work& w = e->w;
  auto& V = e->bufs;
  g_bufs = &V;
  bool ok = true;
  hipStream_t s = e->stream;
  const uint32_t nd = b->ndocs;
  unsigned long long* rng = take<unsigned long long>(V, B_DOCRNG, 9 * (size_t)nd + 9, ok);
  if (!ok) return fail(YCRDT_E_DEVICE, oom("document ranges"));
  launch_doc_ranges(w, (uint32_t)e->last.clients, nd, rng, s);
  std::vector<unsigned long long> r(9 * (size_t)nd);
  Counters c;
  HIPCHK(hipMemcpyAsync(r.data(), rng, sizeof(unsigned long long) * r.size(), hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(&c, w.ctr, sizeof(Counters), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (c.err) return map_err(c.err, "document split");
  const uint64_t sbase = c.pad[3], dsbase = c.ds_base + vu_size_host(c.pad[1]), svbase = vu_size_host(c.pad[2]);
  std::vector<uint64_t>& offs = b->pack_offs;
  offs.assign(2 * (size_t)nd + 1, 0);
  uint64_t pos = 0;
  for (uint32_t d = 0; d < nd; ++d) {
    const unsigned long long* x = &r[9 * (size_t)d];
    offs[2 * d] = pos;
    pos += vu_size_host((uint32_t)x[2]) + (x[2] ? x[1] - x[0] : 0) + vu_size_host((uint32_t)x[5]) + (x[5] ? x[4] - x[3] : 0);
    offs[2 * d + 1] = pos;
    pos += vu_size_host((uint32_t)x[8]) + (x[8] ? x[7] - x[6] : 0);
  }
  offs[2 * (size_t)nd] = pos;
  uint8_t* dst0 = take<uint8_t>(V, B_PACK, pos + 16, ok);
  if (!ok) return fail(YCRDT_E_DEVICE, oom("document split"));
  std::vector<Piece> pc;
  pc.reserve(8 * (size_t)nd);
  auto hdr = [&](uint8_t* dst, uint32_t v) -> uint8_t* {
    Piece P{};
    while (v > 127u) { P.inl[P.len++] = (uint8_t)(0x80u | (v & 0x7fu)); v >>= 7; }
    P.inl[P.len++] = (uint8_t)v;
    P.dst = dst;
    pc.push_back(P);
    return dst + P.len;
  };
  auto range = [&](uint8_t* dst, const uint8_t* src, uint64_t n) -> uint8_t* {
    for (uint64_t k = 0; k < n; k += PIECE_MAX)
      pc.push_back(Piece{src + k, dst + k, (uint32_t)std::min<uint64_t>(PIECE_MAX, n - k), {0}});
    return dst + n;
  };
  for (uint32_t d = 0; d < nd; ++d) {
    const unsigned long long* x = &r[9 * (size_t)d];
    uint8_t* dst = dst0 + offs[2 * d];
    dst = hdr(dst, (uint32_t)x[2]);
    if (x[2]) dst = range(dst, w.out + sbase + x[0], x[1] - x[0]);
    dst = hdr(dst, (uint32_t)x[5]);
    if (x[5]) dst = range(dst, w.out + dsbase + x[3], x[4] - x[3]);
    dst = hdr(dst, (uint32_t)x[8]);
    if (x[8]) range(dst, w.sv_out + svbase + x[6], x[7] - x[6]);
  }
  if (pc.size() >= 0xFFFFFFF0ull) return fail(YCRDT_E_CAPACITY, "document split: too many pieces");
  Piece* dpc = take<Piece>(V, B_PACKPC, pc.size() + 1, ok);
  if (!ok) return fail(YCRDT_E_DEVICE, oom("document split pieces"));
  HIPCHK(hipMemcpyAsync(dpc, pc.data(), sizeof(Piece) * pc.size(), hipMemcpyHostToDevice, s));
  copy_pieces(dpc, (uint32_t)pc.size(), s);
  HIPCHK(hipStreamSynchronize(s));
  b->packed = true;
  return YCRDT_OK;
}

// HBM → host memory through the engine's pinned staging: a wave of chunks is copied D2H into one
// half while worker threads move the previous wave out of the other half.
int d2h_span(ycrdt_engine* e, uint8_t* host, const uint8_t* dev, uint64_t span) {
  if (!span) return YCRDT_OK;
  const uint64_t PIN_CHUNK = pin_chunk();
  const uint64_t nch = (span + PIN_CHUNK - 1) / PIN_CHUNK;
  const bool waves = nch > PIN_PER;
  Pinned& pin = e->pin_out;
  if (const int rc = ensure_pinned(pin, waves ? 2 * PIN_PER * PIN_CHUNK : (size_t)span, e->stream)) return rc;
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const uint32_t T = span < (uint64_t(8) << 20) ? 1u : std::min<uint32_t>({16u, hw, (uint32_t)nch});
  const uint64_t nw = (nch + PIN_PER - 1) / PIN_PER;
  auto issue = [&](uint64_t wave) -> int {
    const uint64_t lo = wave * PIN_PER * PIN_CHUNK, hi = std::min(span, lo + PIN_PER * PIN_CHUNK);
    uint8_t* base = pin.p + (waves ? (wave & 1) * PIN_PER * PIN_CHUNK : 0);
    HIPCHK(hipMemcpyAsync(base, dev + lo, hi - lo, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipEventRecord(pin.ev[wave & 1], e->stream));
    return YCRDT_OK;
  };
  if (const int rc = issue(0)) return rc;
  for (uint64_t wave = 0; wave < nw; ++wave) {
    HIPCHK(hipEventSynchronize(pin.ev[wave & 1]));
    if (wave + 1 < nw)
      if (const int rc = issue(wave + 1)) return rc;  // into the other half, beside the copy-out below
    const uint64_t lo = wave * PIN_PER * PIN_CHUNK, hi = std::min(span, lo + PIN_PER * PIN_CHUNK);
    const uint8_t* base = pin.p + (waves ? (wave & 1) * PIN_PER * PIN_CHUNK : 0);
    if (T == 1) {
      memcpy(host + lo, base, hi - lo);
    } else {
      std::atomic<uint64_t> next{lo};
      auto work = [&]() {
        for (uint64_t a; (a = next.fetch_add(PIN_CHUNK)) < hi;) memcpy(host + a, base + (a - lo), std::min(hi, a + PIN_CHUNK) - a);
      };
      std::vector<std::thread> th;
      for (uint32_t t = 1; t < T; ++t) th.emplace_back(work);
      work();
      for (auto& t : th) t.join();
    }
  }
  return YCRDT_OK;
}

int split_docs(ycrdt_engine* e, ycrdt_batch* b, ycrdt_out* outs, ycrdt_out* svs) {
  if (const int rc = pack_docs(e, b)) return rc;
  const std::vector<uint64_t>& offs = b->pack_offs;
  std::vector<uint8_t> all(offs.back());
  if (const int rc = d2h_span(e, all.data(), (const uint8_t*)e->bufs[B_PACK].p, all.size())) return rc;
  for (uint32_t d = 0; d < b->ndocs; ++d) {
    const uint64_t a = offs[2 * d], m = offs[2 * d + 1], z = offs[2 * d + 2];
    outs[d].ptr = (uint8_t*)malloc(m - a);
    if (!outs[d].ptr) return fail(YCRDT_E_CAPACITY, "host allocation failed");  // the caller frees the rest
    outs[d].len = m - a;
    memcpy(outs[d].ptr, all.data() + a, m - a);
    if (svs) {
      svs[d].ptr = (uint8_t*)malloc(z - m);
      if (!svs[d].ptr) return fail(YCRDT_E_CAPACITY, "host allocation failed");
      svs[d].len = z - m;
      memcpy(svs[d].ptr, all.data() + m, z - m);
    }
  }
  return YCRDT_OK;
}

int empty_update(ycrdt_out* out) {
  out->ptr = (uint8_t*)malloc(2);
  if (!out->ptr) { out->len = 0; return fail(YCRDT_E_CAPACITY, "host allocation failed"); }
  out->ptr[0] = 0;
  out->ptr[1] = 0;
  out->len = 2;
  return YCRDT_OK;
}

}  // namespace

// =========================================================================================== C ABI
extern "C" {

const char* ycrdt_last_error(void) { return g_err.c_str(); }
const char* ycrdt_version(void) { return "ycrdt-mi355x 0.1 (gfx950)"; }

void ycrdt_free(ycrdt_out* o) {
  if (o && o->ptr) free(o->ptr);
  if (o) { o->ptr = nullptr; o->len = 0; }
}

int ycrdt_engine_create(int device, int compat, ycrdt_engine** out) {
  if (!out) return fail(YCRDT_E_ARG, "null out");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(YCRDT_E_DEVICE, "no HIP device available");
  if (device < 0 || device >= n) return fail(YCRDT_E_DEVICE, "bad device ordinal");
  HIPCHK(hipSetDevice(device));
  auto* e = new ycrdt_engine();
  e->device = device;
  e->compat = compat == 135 ? 135 : 136;
  e->debug_sync = getenv("YCRDT_DEBUG_SYNC") && getenv("YCRDT_DEBUG_SYNC")[0] == '1';
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) { delete e; return fail(YCRDT_E_DEVICE, "stream"); }
  if (hipStreamCreateWithFlags(&e->side, hipStreamNonBlocking) != hipSuccess) { delete e; return fail(YCRDT_E_DEVICE, "stream"); }
  hipEventCreateWithFlags(&e->side_done, hipEventDisableTiming);
  hipEventCreateWithFlags(&e->side_fork, hipEventDisableTiming);
  hipEventCreate(&e->ev0);
  hipEventCreate(&e->ev1);
  if (hipStreamCreateWithFlags(&e->copy, hipStreamNonBlocking) != hipSuccess) { delete e; return fail(YCRDT_E_DEVICE, "stream"); }
  hipEventCreateWithFlags(&e->copy_dep, hipEventDisableTiming);
  for (Pinned* pin : {&e->pin_in, &e->pin_out}) {
    hipEventCreateWithFlags(&pin->ev[0], hipEventDisableTiming);
    hipEventCreateWithFlags(&pin->ev[1], hipEventDisableTiming);
  }
  e->bufs.resize(B_COUNT);
  *out = e;
  return YCRDT_OK;
}

void ycrdt_engine_destroy(ycrdt_engine* e) {
  if (!e) return;
  hipSetDevice(e->device);
  hipStreamSynchronize(e->stream);
  for (auto& b : e->bufs) if (b.p) hipFree(b.p);
  if (e->scratch) {
    if (e->scratch->bytes.p) hipFree(e->scratch->bytes.p);
    if (e->scratch->pieces.p) hipFree(e->scratch->pieces.p);
    if (e->scratch->meta.p) hipFree(e->scratch->meta.p);
    delete e->scratch;
  }
  for (auto& ev : e->event_pool) hipEventDestroy(ev);
  hipEventDestroy(e->ev0);
  hipEventDestroy(e->ev1);
  hipStreamSynchronize(e->copy);
  for (Pinned* pin : {&e->pin_in, &e->pin_out}) {
    hipEventDestroy(pin->ev[0]);
    hipEventDestroy(pin->ev[1]);
    if (pin->p) hipHostFree(pin->p);
  }
  if (e->ctr_pin) hipHostFree(e->ctr_pin);
  if (e->sv_pin) hipHostFree(e->sv_pin);
  if (e->rb) hipHostFree(e->rb);
  hipEventDestroy(e->copy_dep);
  hipStreamDestroy(e->copy);
  hipStreamSynchronize(e->side);
  hipEventDestroy(e->side_done);
  hipEventDestroy(e->side_fork);
  hipStreamDestroy(e->side);
  hipStreamDestroy(e->stream);
  delete e;
}

int ycrdt_engine_set_profiling(ycrdt_engine* e, int on) {
  if (!e) return fail(YCRDT_E_ARG, "null engine");
  e->profiling = on != 0;
  return YCRDT_OK;
}

int ycrdt_engine_phase_times(ycrdt_engine* e, const char** names, double* ms, int cap) {
  if (!e) return 0;
  int n = 0;
  for (auto& p : e->phase_ms) {
    if (n >= cap) break;
    names[n] = p.first;
    ms[n] = p.second;
    ++n;
  }
  return n;
}

int ycrdt_engine_device_bytes(ycrdt_engine* e, uint64_t* bytes) {
  if (!e || !bytes) return fail(YCRDT_E_ARG, "null arg");
  uint64_t n = 0;
  for (const auto& b : e->bufs) n += b.cap;
  n += (uint64_t)e->arena.slabs.size() * Arena::SLAB;
  if (e->scratch) n += e->scratch->bytes.cap + e->scratch->meta.cap + e->scratch->pieces.cap;
  *bytes = n;
  return YCRDT_OK;
}

int ycrdt_engine_trim(ycrdt_engine* e) {
  if (!e) return fail(YCRDT_E_ARG, "null arg");
  hipSetDevice(e->device);
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipStreamSynchronize(e->side));
  for (auto& b : e->bufs)
    if (b.p && !b.arena) { hipFree(b.p); b = DevBuf{}; }
  // the docs' spare blocks (a folded merge keeps the previous state block, up to FOLD_MAX, for the
  // next one: about twice the state bytes of every small doc until trimmed)
  for (ycrdt_doc* d : e->docs) release_state(e, d->spare);
  e->ws_owner = nullptr;  // no doc's merge results are held any more: its next read merges again
  e->nsegs = 0;
  e->nlists = 0;
  return YCRDT_OK;
}

int ycrdt_doc_create(ycrdt_engine* e, uint32_t client_id, ycrdt_doc** out) {
  if (!e || !out) return fail(YCRDT_E_ARG, "null arg");
  auto* d = new ycrdt_doc();
  d->e = e;
  d->client_id = client_id;
  d->sv = {0};
  e->docs.insert(d);
  *out = d;
  return YCRDT_OK;
}

void ycrdt_doc_destroy(ycrdt_doc* d) {
  if (!d) return;
  hipSetDevice(d->e->device);
  if (d->e->ws_owner == d) d->e->ws_owner = nullptr;
  if (d->state.p) { if (d->state.arena) d->e->arena.release(d->state.p, d->state.cap); else hipFree(d->state.p); }
  if (d->marks.p) { if (d->marks.arena) d->e->arena.release(d->marks.p, d->marks.cap); else hipFree(d->marks.p); }
  if (d->spare.p) { if (d->spare.arena) d->e->arena.release(d->spare.p, d->spare.cap); else hipFree(d->spare.p); }
  d->e->docs.erase(d);
  delete d;
}

}  // extern "C"

namespace {

constexpr size_t QUEUE_FLUSH_BYTES = size_t(1) << 30;  // deferred updates past this are merged at once

// YCRDT_PREDECODE: 0 off, "check" decode the state the usual way and compare with its marks
int predecode_mode() {
  const char* v = getenv("YCRDT_PREDECODE");
  return v && v[0] == '0' ? 0 : v && !strcmp(v, "check") ? 2 : 1;
}
// the doc's state goes into the next batch as source 0: decoded from its marks when they describe it
void doc_pre(ycrdt_doc* d, ycrdt_batch& b) {
  b.pre_src = -1;
  b.pre_check = false;
  const int mode = predecode_mode();
  if (!mode || !d->state_len || d->marks_len != d->state_len || !d->marks.p) return;
  uint8_t* m = (uint8_t*)d->marks.p;
  b.pre.fbits = (uint64_t*)m;
  b.pre.sbits = (uint64_t*)(m + 8ull * d->marks_nw);
  b.pre.secs = (Section*)(m + 16ull * d->marks_nw);
  b.pre.meta = (uint32_t*)(m + 16ull * d->marks_nw + sizeof(Section) * d->marks_cap);
  b.pre.nw = d->marks_nw;
  b.pre.cap_secs = d->marks_cap;
  b.pre_src = 0;
  b.pre_check = mode == 2;
}
// after a successful merge of the doc (the workspace holds its encode): the marks of the new state
void doc_marks(ycrdt_doc* d) {
  ycrdt_engine* e = d->e;
  d->marks_len = 0;
  if (!predecode_mode() || !e->out_bytes || e->out_bytes >= (uint64_t(1) << 31)) return;
  // (exactly the state's own 64-byte slot: the next staged update's words follow it)
  const uint32_t nw = (uint32_t)((e->out_bytes + 63) / 64), cap = (uint32_t)e->last.clients + 1;
  const size_t bytes = 16ull * nw + sizeof(Section) * cap + 16;
  if (d->marks.cap < bytes) {
    release_state(e, d->marks);
    if (!alloc_state(e, d->marks, bytes)) { (void)hipGetLastError(); d->marks = DevBuf(); return; }
  }
  d->marks_nw = nw;
  d->marks_cap = cap;
  {
    uint8_t* m = (uint8_t*)d->marks.p;
    PreMarks pm;
    pm.fbits = (uint64_t*)m;
    pm.sbits = (uint64_t*)(m + 8ull * nw);
    pm.secs = (Section*)(m + 16ull * nw);
    pm.meta = (uint32_t*)(m + 16ull * nw + sizeof(Section) * cap);
    pm.nw = nw;
    pm.cap_secs = cap;
    launch_state_marks(e->w, (uint32_t)e->last.out_structs, (uint32_t)e->last.clients, pm, e->stream);
  }
  d->marks_len = e->out_bytes;
}

// Merges `extra` (host updates) behind the doc's state in one device pass and makes the result the
// doc's state. caps: integrate only below the per-client caps (the pending path).
int commit_merge(ycrdt_doc* d, const std::vector<ycrdt_buf>& extra, const ClockMap* caps,
                 const std::vector<uint32_t>* order = nullptr, const std::vector<int32_t>* hints = nullptr) {
  ycrdt_engine* e = d->e;
  ycrdt_batch& b = scratch_batch(e);  // engine-owned: no hipMalloc / hipFree per call
  doc_pre(d, b);
  int rc = stage(&b, extra.data(), extra.size(), d->state_len ? &d->state : nullptr, d->state_len, nullptr, 1,
                 hints && hints->size() == 2 * extra.size() ? hints->data() : nullptr);
  // The merged state goes to a block of its own (or the doc's, when it fits and is not the source
  // of this merge any more: the batch holds a copy once staged); the doc changes only once it is
  // there. A small merge queues the copies before its last synchronisation (run_merge's
  // before_final) — its output bound, not yet its size, is known then: the bound is copied.
  constexpr uint64_t FOLD_MAX = uint64_t(4) << 20;
  DevBuf nb = d->state;
  bool fresh = false, folded = false;
  const std::function<int(uint64_t, uint64_t)> fold = [&](uint64_t cap_out, uint64_t cap_sv) -> int {
    if (cap_out > FOLD_MAX || cap_sv > PIN_SV) return YCRDT_OK;
    if (!e->sv_pin && hipHostMalloc((void**)&e->sv_pin, PIN_SV, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      e->sv_pin = nullptr;
      return YCRDT_OK;  // (the copies after the merge)
    }
    // never the doc's own block (the merge may still fail at its last check, and the doc's state
    // must then be what it was): the spare block when it is large enough, else a new one
    fresh = true;
    if (d->spare.p && d->spare.cap >= cap_out + 16) { nb = d->spare; d->spare = DevBuf(); }
    else if (!alloc_state(e, nb, cap_out + 16)) return fail(YCRDT_E_DEVICE, oom("doc state"));
    HIPCHK(hipMemcpyAsync(nb.p, e->w.out, cap_out, hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(hipMemcpyAsync(e->sv_pin, e->w.sv_out, cap_sv, hipMemcpyDeviceToHost, e->stream));
    folded = true;
    return YCRDT_OK;
  };
  static const bool nofold = getenv("YCRDT_NO_FOLD") && getenv("YCRDT_NO_FOLD")[0] == '1';  // (A/B)
  if (rc == YCRDT_OK) {
    e->before_final = nofold ? nullptr : &fold;
    rc = run_merge(e, &b, nullptr, caps, order);
    e->before_final = nullptr;
  }
  b.pre_src = -1;
  if (rc == YCRDT_OK) doc_marks(d);  // (the new state's decode, from this encode: queued on the stream)
  if (rc) {
    if (fresh && !d->spare.p) d->spare = nb;  // (kept for the next merge)
    else if (fresh) release_state(e, nb);
    return rc;
  }
  std::vector<uint8_t> sv(e->sv_bytes);
  if (folded) {
    if (!sv.empty()) memcpy(sv.data(), e->sv_pin, e->sv_bytes);
  } else {
    fresh = e->out_bytes + 16 > d->state.cap;
    if (fresh && !alloc_state(e, nb, e->out_bytes + 16)) return fail(YCRDT_E_DEVICE, oom("doc state"));
    hipError_t er = hipMemcpyAsync(nb.p, e->w.out, e->out_bytes, hipMemcpyDeviceToDevice, e->stream);
    if (er == hipSuccess && !sv.empty()) er = hipMemcpyAsync(sv.data(), e->w.sv_out, e->sv_bytes, hipMemcpyDeviceToHost, e->stream);
    if (er == hipSuccess) er = hipStreamSynchronize(e->stream);
    if (er != hipSuccess) {
      if (fresh) release_state(e, nb);
      return fail(YCRDT_E_DEVICE, std::string("HIP error: ") + hipGetErrorString(er) + " (doc state copy)");
    }
  }
  if (fresh && folded) {  // the old block becomes the spare
    release_state(e, d->spare);
    d->spare = d->state;
    d->state = nb;
  } else if (fresh) {
    release_state(e, d->state);
    d->state = nb;
  }
  d->state_len = e->out_bytes;
  d->sv.swap(sv);
  d->last = e->last;
  d->view.valid = false;
  e->ws_owner = d;  // the workspace now holds this doc's merged store (ensure_view reuses it)
  // a doc that is read through its view (local ops, toJSON, get) takes the view now, while the
  // workspace holds its merge: another doc's merge in between would otherwise force a re-merge
  if (d->wants_view) return run_view(e, &b, d->view);
  return YCRDT_OK;
}

// Y.mergeUpdates of host buffers on the device (the pending path's merges)
int lazy_merge_host(ycrdt_engine* e, const std::vector<const std::vector<uint8_t>*>& ins, std::vector<uint8_t>& out) {
  std::vector<ycrdt_buf> bufs;
  for (const auto* v : ins) bufs.push_back(ycrdt_buf{v->data(), v->size()});
  ycrdt_out o{nullptr, 0};
  const int rc = ycrdt_merge_updates(e, bufs.data(), bufs.size(), &o);
  if (rc) return rc;
  out.assign(o.ptr, o.ptr + o.len);
  ycrdt_free(&o);
  return YCRDT_OK;
}

// Runs the deferred Y.applyUpdate calls. Fast path: no pending state before, and the device merge
// of (state ∪ queue) finds every dependency — then sequential Yjs ends with nothing pending either
// (every parked struct is retried once the client it waits on advances), so the merge IS the
// result. Otherwise the queue is replayed through Yjs's readUpdateV2 on struct headers
// (yc_ingest.cpp), which yields the pending structs / delete set byte for byte and the state every
// client reaches; one capped device merge then integrates exactly that.
int flush(ycrdt_doc* d) {
  if (d->queue.empty()) return YCRDT_OK;
  ycrdt_engine* e = d->e;
  HIPCHK(hipSetDevice(e->device));
  std::vector<ycrdt_buf> bufs;
  bool ds_errors = false;  // a cut-short delete set takes effect against the state of its time: replay
  std::vector<int32_t> hints;  // the scan's struct / section counts (a large update with few structs: no chunk walk)
  for (const auto& q : d->queue) {
    bufs.push_back(ycrdt_buf{q.bytes.data(), q.bytes.size()});
    ds_errors |= q.ds_error;
    hints.push_back(q.nst);
    hints.push_back(q.nsec);
  }
  if (!d->ing.has_pending && !d->ing.has_ds && e->compat != 135 && !ds_errors) {
    const int rc = commit_merge(d, bufs, nullptr, nullptr, &hints);
    if (rc != YCRDT_E_PENDING) {
      if (rc == YCRDT_OK) { d->queue.clear(); d->queue_bytes = 0; }
      return rc;
    }
  }
  IngestState S = d->ing;
  S.state.clear();
  if (!parse_state_vector(d->sv.data(), d->sv.size(), S.state)) return fail(YCRDT_E_DEVICE, "internal: doc state vector");
  const MergeFn mf = [e](const std::vector<const std::vector<uint8_t>*>& ins, std::vector<uint8_t>& out) {
    return lazy_merge_host(e, ins, out);
  };
  std::string err;
  std::vector<std::vector<uint8_t>> eff(d->queue.size());  // ds_error entries as they take effect
  for (size_t i = 0; i < d->queue.size(); ++i) {
    const auto& q = d->queue[i];
    const int rc = read_update(S, q.bytes.data(), q.bytes.size(), q.local, mf, err, q.ds_error, q.ds_error ? &eff[i] : nullptr);
    if (rc) return fail(rc, err);
    if (q.ds_error) bufs[i] = ycrdt_buf{eff[i].data(), eff[i].size()};
  }
  if (d->ing.has_pending) bufs.push_back(ycrdt_buf{d->ing.pending.data(), d->ing.pending.size()});
  if (d->ing.has_ds) bufs.push_back(ycrdt_buf{d->ing.pending_ds.data(), d->ing.pending_ds.size()});
  // compat 135: the stored state is written with the store's client order (what 13.5.16 emits)
  int rc = commit_merge(d, bufs, &S.state, e->compat == 135 ? &S.order : nullptr);
  if (rc) return rc;
  ClockMap got;
  parse_state_vector(d->sv.data(), d->sv.size(), got);
  for (auto it = S.state.begin(); it != S.state.end();) it = it->second ? std::next(it) : S.state.erase(it);
  if (got != S.state) return fail(YCRDT_E_DEVICE, "internal: capped merge disagrees with the pending emulation");
  d->ing = std::move(S);
  d->queue.clear();
  d->queue_bytes = 0;
  return YCRDT_OK;
}

void enqueue(ycrdt_doc* d, const uint8_t* p, size_t n, bool local, bool ds_error = false, int32_t nst = -1, int32_t nsec = -1) {
  d->queue.push_back(ycrdt_doc::Queued{std::vector<uint8_t>(p, p + n), local, ds_error, nst, nsec});
  d->queue_bytes += n;
  d->view.valid = false;
}

// Multi-document flush (ycrdt_apply_updates_multi): the documents on the fast path (nothing
// pending, 13.6 client order) are merged in ONE device pass — each document's state (HBM, read in
// place) and its queued updates form one multi-document batch (yc_work.h: (doc, client) keys) —
// and the result is split back into each document's arena block on the device, headers written
// inline (k_doc_ranges + copy_pieces): no per-document merge, copy or hipMalloc. A missing
// dependency anywhere sends every document through its own flush (the pending emulation is per
// document), as does any document on the slow path.
int flush_multi(ycrdt_engine* e, const std::vector<ycrdt_doc*>& docs) {
  std::vector<ycrdt_doc*> fast;
  for (ycrdt_doc* d : docs) {
    if (d->queue.empty()) continue;
    bool ds_errors = false;
    for (const auto& q : d->queue) ds_errors |= q.ds_error;
    if (!d->ing.has_pending && !d->ing.has_ds && e->compat != 135 && !ds_errors) fast.push_back(d);
    else if (const int rc = flush(d)) return rc;
  }
  if (fast.size() < 2) return fast.empty() ? YCRDT_OK : flush(fast[0]);
  HIPCHK(hipSetDevice(e->device));
  const uint32_t nd = (uint32_t)fast.size();
  std::vector<Src> src;
  std::vector<uint32_t> doc_of;
  for (uint32_t j = 0; j < nd; ++j) {
    ycrdt_doc* d = fast[j];
    if (d->state_len) { src.push_back(Src{(const uint8_t*)d->state.p, d->state_len, true}); doc_of.push_back(j); }
    for (const auto& q : d->queue) { src.push_back(Src{q.bytes.data(), q.bytes.size(), false}); doc_of.push_back(j); }
  }
  ycrdt_batch& b = scratch_batch(e);
  int rc = stage_srcs(&b, src, doc_of.data(), nd);
  if (rc == YCRDT_OK) rc = run_merge(e, &b, nullptr);
  if (rc == YCRDT_E_PENDING) {
    for (ycrdt_doc* d : fast)
      if (const int r2 = flush(d)) return r2;
    return YCRDT_OK;
  }
  if (rc) return rc;
  // per-document ranges of the encode, then every document's state assembled on the device
  Work& w = e->w;
  auto& V = e->bufs;
  g_bufs = &V;
  bool ok = true;
  unsigned long long* rng = take<unsigned long long>(V, B_DOCRNG, 9 * (size_t)nd + 9, ok);
  if (!ok) return fail(YCRDT_E_DEVICE, oom("document ranges"));
  hipStream_t s = e->stream;
  launch_doc_ranges(w, (uint32_t)e->last.clients, nd, rng, s);
  std::vector<unsigned long long> r(9 * (size_t)nd);
  std::vector<uint8_t> svall(e->sv_bytes);
  Counters c;
  HIPCHK(hipMemcpyAsync(r.data(), rng, sizeof(unsigned long long) * r.size(), hipMemcpyDeviceToHost, s));
  if (!svall.empty()) HIPCHK(hipMemcpyAsync(svall.data(), w.sv_out, svall.size(), hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(&c, w.ctr, sizeof(Counters), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (c.err) return map_err(c.err, "document split");
  const uint64_t sbase = c.pad[3], dsbase = c.ds_base + vu_size_host(c.pad[1]), svbase = vu_size_host(c.pad[2]);
  std::vector<Piece> pc;
  pc.reserve(4 * (size_t)nd);
  std::vector<size_t> len(nd);
  // every document's new block and state vector are prepared first; the documents change only
  // after the copy has succeeded (a failed allocation or copy leaves all of them as they were)
  std::vector<DevBuf> nblk(nd);
  std::vector<char> fresh(nd, 0);
  std::vector<std::vector<uint8_t>> nsv(nd);
  auto drop_fresh = [&]() { for (uint32_t j = 0; j < nd; ++j) if (fresh[j]) release_state(e, nblk[j]); };
  auto hdr = [](Piece& P, uint32_t v) {
    P.src = nullptr;
    P.len = 0;
    while (v > 127u) { P.inl[P.len++] = (uint8_t)(0x80u | (v & 0x7fu)); v >>= 7; }
    P.inl[P.len++] = (uint8_t)v;
  };
  for (uint32_t j = 0; j < nd; ++j) {
    const unsigned long long* x = &r[9 * (size_t)j];
    const uint32_t ns = x[2] ? (uint32_t)(x[1] - x[0]) : 0, ndb = x[5] ? (uint32_t)(x[4] - x[3]) : 0;
    len[j] = vu_size_host((uint32_t)x[2]) + ns + vu_size_host((uint32_t)x[5]) + ndb;
    ycrdt_doc* d = fast[j];
    // the batch holds a copy of every document's old state, so a block that fits is rewritten
    // in place (untouched until the copy below), a bigger one is allocated beside the old
    nblk[j] = d->state;
    if (len[j] + 16 > d->state.cap) {
      if (!alloc_state(e, nblk[j], len[j] + 16)) { drop_fresh(); return fail(YCRDT_E_DEVICE, oom("doc state")); }
      fresh[j] = 1;
    }
    uint8_t* dst = (uint8_t*)nblk[j].p;
    Piece P{};
    hdr(P, (uint32_t)x[2]); P.dst = dst; dst += P.len; pc.push_back(P);
    if (ns) { pc.push_back(Piece{w.out + sbase + x[0], dst, ns, {0}}); dst += ns; }
    hdr(P, (uint32_t)x[5]); P.dst = dst; dst += P.len; pc.push_back(P);
    if (ndb) pc.push_back(Piece{w.out + dsbase + x[3], dst, ndb, {0}});
    // state vector: its entries (host copy of the encode's state vector section)
    std::vector<uint8_t>& sv = nsv[j];
    put_vu(sv, (uint32_t)x[8]);
    if (x[8]) sv.insert(sv.end(), svall.begin() + svbase + x[6], svall.begin() + svbase + x[7]);
  }
  if (!grow(b.pieces, sizeof(Piece) * (pc.size() + 1))) { drop_fresh(); return fail(YCRDT_E_DEVICE, oom("pieces")); }
  hipError_t er = hipMemcpyAsync(b.pieces.p, pc.data(), sizeof(Piece) * pc.size(), hipMemcpyHostToDevice, s);
  if (er == hipSuccess) { copy_pieces((const Piece*)b.pieces.p, (uint32_t)pc.size(), s); er = hipStreamSynchronize(s); }
  if (er != hipSuccess) {
    // a block rewritten in place may be partly written: those documents cannot be trusted
    drop_fresh();
    return fail(YCRDT_E_DEVICE, std::string("HIP error: ") + hipGetErrorString(er) + " (document split)");
  }
  for (uint32_t j = 0; j < nd; ++j) {
    ycrdt_doc* d = fast[j];
    if (fresh[j]) { release_state(e, d->state); d->state = nblk[j]; }
    d->sv.swap(nsv[j]);
    d->state_len = len[j];
    d->marks_len = 0;  // (assembled from a multi-document encode: no marks)
    d->last = e->last;  // the whole pass
    d->view.valid = false;
    d->queue.clear();
    d->queue_bytes = 0;
  }
  e->ws_owner = nullptr;  // the workspace holds many documents: a view re-merges its own
  return YCRDT_OK;
}

}  // namespace

extern "C" {

// Y.applyUpdate × n. Each update is validated now (Yjs decodes the struct section before it
// changes anything, and throws on malformed input); the merge itself is deferred to the next read.
int ycrdt_apply_updates(ycrdt_doc* d, const ycrdt_buf* ups, size_t n) {
  if (!d || (!ups && n)) return fail(YCRDT_E_ARG, "null arg");
  if (n == 0) return YCRDT_OK;
  std::vector<UpdScan> sc(n);
  std::vector<char> ok(n, 0);
  size_t total = 0;
  for (size_t i = 0; i < n; ++i) total += ups[i].len;
  const size_t nt = total > (size_t(4) << 20) && n > 1 ? std::min<size_t>({n, 16, std::max(1u, std::thread::hardware_concurrency())}) : 1;
  auto work = [&](size_t t) {
    for (size_t i = t; i < n; i += nt) ok[i] = scan_update(ups[i].ptr, ups[i].len, false, sc[i]) ? 1 : 0;
  };
  if (nt > 1) {
    std::vector<std::thread> th;
    for (size_t t = 0; t < nt; ++t) th.emplace_back(work, t);
    for (auto& t : th) t.join();
  } else {
    work(0);
  }
  for (size_t i = 0; i < n; ++i) {
    if (!ok[i] && sc[i].unsupported)
      return fail(YCRDT_E_UNSUPPORTED, "update " + std::to_string(i) + ": an any value nests deeper than 32 levels (engine limit)");
    if (!ok[i]) {
      // Yjs integrates a well-formed struct section and the delete-set ranges read before the error
      if (sc[i].structs_ok) {
        const std::vector<uint8_t> r = repaired_update(ups[i].ptr, sc[i]);
        enqueue(d, r.data(), r.size(), false, true);
      }
      return fail(YCRDT_E_DECODE, "Integer out of range! (malformed update " + std::to_string(i) + ")");
    }
    enqueue(d, ups[i].ptr, ups[i].len, false, false, (int32_t)std::min<uint64_t>(sc[i].nstructs, 0x7FFFFFFF), (int32_t)sc[i].secs.size());
  }
  if (d->queue_bytes > QUEUE_FLUSH_BYTES) return flush(d);
  return YCRDT_OK;
}

int ycrdt_apply_update(ycrdt_doc* d, ycrdt_buf update) { return ycrdt_apply_updates(d, &update, 1); }

// Y.applyUpdate(docs[i], ups[i]) for i = 0..n-1 (a fleet ingest batch: many documents, any number
// of updates each), validated like ycrdt_apply_updates and then merged at once: one device pass
// for every document on the fast path (flush_multi).
int ycrdt_apply_updates_multi(ycrdt_engine* e, ycrdt_doc* const* docs, const ycrdt_buf* ups, size_t n) {
  if (!e || (n && (!docs || !ups))) return fail(YCRDT_E_ARG, "null arg");
  for (size_t i = 0; i < n; ++i)
    if (!docs[i] || docs[i]->e != e) return fail(YCRDT_E_ARG, "document of another engine (or null) at " + std::to_string(i));
  std::vector<UpdScan> sc(n);
  std::vector<char> ok(n, 0);
  size_t total = 0;
  for (size_t i = 0; i < n; ++i) total += ups[i].len;
  const size_t nt = total > (size_t(4) << 20) && n > 1 ? std::min<size_t>({n, 16, std::max(1u, std::thread::hardware_concurrency())}) : 1;
  auto work = [&](size_t t) {
    for (size_t i = t; i < n; i += nt) ok[i] = scan_update(ups[i].ptr, ups[i].len, false, sc[i]) ? 1 : 0;
  };
  if (nt > 1) {
    std::vector<std::thread> th;
    for (size_t t = 0; t < nt; ++t) th.emplace_back(work, t);
    for (auto& t : th) t.join();
  } else {
    work(0);
  }
  std::vector<ycrdt_doc*> touched;
  int rc = YCRDT_OK;
  std::string err;
  for (size_t i = 0; i < n; ++i) {
    ycrdt_doc* d = docs[i];
    touched.push_back(d);
    if (!ok[i] && sc[i].unsupported) {  // the earlier updates are applied; this one is refused
      rc = YCRDT_E_UNSUPPORTED;
      err = "update " + std::to_string(i) + ": an any value nests deeper than 32 levels (engine limit)";
      break;
    }
    if (!ok[i]) {  // sequential semantics: what came before is applied, then Yjs throws
      if (sc[i].structs_ok) {
        const std::vector<uint8_t> r = repaired_update(ups[i].ptr, sc[i]);
        enqueue(d, r.data(), r.size(), false, true);
      }
      rc = YCRDT_E_DECODE;
      err = "Integer out of range! (malformed update " + std::to_string(i) + ")";
      break;
    }
    enqueue(d, ups[i].ptr, ups[i].len, false);
  }
  std::sort(touched.begin(), touched.end());
  touched.erase(std::unique(touched.begin(), touched.end()), touched.end());
  const int frc = flush_multi(e, touched);
  if (rc) return fail(rc, err);
  return frc;
}

// Every document's Y.encodeStateAsUpdate + Y.encodeStateVector in one call (a fleet's LevelDB
// storeUpdate / sync snapshot, crdt.js:33-40,260,288): deferred applies flushed as one batched
// merge, the states gathered from their arena blocks by one piece-copy launch and copied to the
// host through the pipelined pinned D2H. A document with pending structs takes its own encode.
int ycrdt_docs_states_packed(ycrdt_engine* e, ycrdt_doc* const* docs, size_t n, uint8_t* dst, uint64_t cap, uint64_t* offs,
                             uint64_t* total) {
  if (!e || (n && !docs)) return fail(YCRDT_E_ARG, "null arg");
  for (size_t i = 0; i < n; ++i)
    if (!docs[i] || docs[i]->e != e) return fail(YCRDT_E_ARG, "document of another engine (or null) at " + std::to_string(i));
  HIPCHK(hipSetDevice(e->device));
  {
    std::vector<ycrdt_doc*> q;
    for (size_t i = 0; i < n; ++i) if (!docs[i]->queue.empty()) q.push_back(docs[i]);
    std::sort(q.begin(), q.end());
    q.erase(std::unique(q.begin(), q.end()), q.end());
    if (const int rc = flush_multi(e, q)) return rc;
  }
  std::vector<uint64_t> o(2 * n + 1, 0);
  std::vector<std::vector<uint8_t>> slow(n);  // pending documents: their encode (host)
  uint64_t pos = 0;
  for (size_t i = 0; i < n; ++i) {
    ycrdt_doc* d = docs[i];
    o[2 * i] = pos;
    if (d->ing.has_pending || d->ing.has_ds) {
      ycrdt_out u{nullptr, 0};
      if (const int rc = ycrdt_encode_state_as_update(d, ycrdt_buf{nullptr, 0}, &u)) return rc;
      slow[i].assign(u.ptr, u.ptr + u.len);
      ycrdt_free(&u);
      pos += slow[i].size();
    } else {
      pos += d->state_len ? d->state_len : 2;
    }
    o[2 * i + 1] = pos;
    pos += d->sv.size();
  }
  o[2 * n] = pos;
  if (total) *total = pos;
  if (offs) memcpy(offs, o.data(), sizeof(uint64_t) * o.size());
  if (!dst) return YCRDT_OK;
  if (cap < pos) return fail(YCRDT_E_ARG, "destination smaller than the packed states");
  // device states: one gather into B_PACK, one pipelined D2H; the rest is written on the host
  std::vector<Piece> pc;
  uint64_t dev = 0;
  std::vector<uint64_t> at(n, ~0ull);
  for (size_t i = 0; i < n; ++i) {
    ycrdt_doc* d = docs[i];
    if (slow[i].empty() && d->state_len) {
      at[i] = dev;
      for (uint64_t k = 0; k < d->state_len; k += PIECE_MAX)
        pc.push_back(Piece{(const uint8_t*)d->state.p + k, nullptr, (uint32_t)std::min<uint64_t>(PIECE_MAX, d->state_len - k), {0}});
      dev += d->state_len;
    }
  }
  if (dev) {
    auto& V = e->bufs;
  g_bufs = &V;
    bool ok = true;
    uint8_t* buf = take<uint8_t>(V, B_PACK, dev + 16, ok);
    Piece* dpc = ok ? take<Piece>(V, B_PACKPC, pc.size() + 1, ok) : nullptr;
    if (!ok) return fail(YCRDT_E_DEVICE, oom("document states"));
    uint64_t w = 0;
    for (Piece& P : pc) { P.dst = buf + w; w += P.len; }
    HIPCHK(hipMemcpyAsync(dpc, pc.data(), sizeof(Piece) * pc.size(), hipMemcpyHostToDevice, e->stream));
    copy_pieces(dpc, (uint32_t)pc.size(), e->stream);
    std::vector<uint8_t> host(dev);
    if (const int rc = d2h_span(e, host.data(), buf, dev)) return rc;
    e->ws_owner = nullptr;  // B_PACK held a batch's split
    for (size_t i = 0; i < n; ++i)
      if (at[i] != ~0ull) memcpy(dst + o[2 * i], host.data() + at[i], docs[i]->state_len);
  }
  for (size_t i = 0; i < n; ++i) {
    ycrdt_doc* d = docs[i];
    if (!slow[i].empty()) memcpy(dst + o[2 * i], slow[i].data(), slow[i].size());
    else if (!d->state_len) { dst[o[2 * i]] = 0; dst[o[2 * i] + 1] = 0; }
    if (!d->sv.empty()) memcpy(dst + o[2 * i + 1], d->sv.data(), d->sv.size());
  }
  return YCRDT_OK;
}

int ycrdt_doc_flush(ycrdt_doc* d) {
  if (!d) return fail(YCRDT_E_ARG, "null doc");
  return flush(d);
}

int ycrdt_doc_pending(ycrdt_doc* d, int* structs, int* delete_set) {
  if (!d) return fail(YCRDT_E_ARG, "null doc");
  const int rc = flush(d);
  if (rc) return rc;
  if (structs) *structs = d->ing.has_pending ? 1 : 0;
  if (delete_set) *delete_set = d->ing.has_ds ? 1 : 0;
  return YCRDT_OK;
}

int ycrdt_encode_state_as_update(ycrdt_doc* d, ycrdt_buf sv, ycrdt_out* out) {
  if (!d || !out) return fail(YCRDT_E_ARG, "null arg");
  out->ptr = nullptr;
  out->len = 0;
  std::unordered_map<uint32_t, uint32_t> target;
  if (sv.len && !parse_sv(sv.ptr, sv.len, target)) return fail(YCRDT_E_DECODE, "Integer out of range! (state vector)");
  int rc = flush(d);
  if (rc) return rc;
  ycrdt_engine* e = d->e;
  HIPCHK(hipSetDevice(e->device));
  // writeStateAsUpdate (the integrated store)
  std::vector<uint8_t> main;
  if (!d->state_len) {
    main = {0, 0};
  } else if (target.empty()) {
    main.resize(d->state_len);
    HIPCHK(hipMemcpy(main.data(), d->state.p, d->state_len, hipMemcpyDeviceToHost));
  } else {  // delta: re-run the (idempotent) merge of the canonical state with per-client start clocks
    ycrdt_batch& b = scratch_batch(e);
    doc_pre(d, b);  // (the state's own decode: crdt.js's sync reply, crdt.js:288)
    rc = stage(&b, nullptr, 0, &d->state, d->state_len);
    if (rc == YCRDT_OK) rc = run_merge(e, &b, &target, nullptr, e->compat == 135 ? &d->ing.order : nullptr);
    b.pre_src = -1;
    if (rc) return rc;
    main.resize(e->out_bytes);
    HIPCHK(hipMemcpy(main.data(), e->w.out, e->out_bytes, hipMemcpyDeviceToHost));
  }
  if (!d->ing.has_pending && !d->ing.has_ds) {
    out->len = main.size();
    out->ptr = (uint8_t*)malloc(out->len);
    if (!out->ptr) return fail(YCRDT_E_CAPACITY, "host allocation failed");
    memcpy(out->ptr, main.data(), out->len);
    return YCRDT_OK;
  }
  // encodeStateAsUpdateV2 (Y@22155): mergeUpdates([main, pendingDs, diffUpdate(pending, sv)])
  std::vector<ycrdt_buf> parts{ycrdt_buf{main.data(), main.size()}};
  if (d->ing.has_ds) parts.push_back(ycrdt_buf{d->ing.pending_ds.data(), d->ing.pending_ds.size()});
  ycrdt_out pd{nullptr, 0};
  if (d->ing.has_pending) {
    static const uint8_t empty_sv[1] = {0};
    const ycrdt_buf svb = sv.len ? sv : ycrdt_buf{empty_sv, 1};
    rc = ycrdt_diff_update(e, ycrdt_buf{d->ing.pending.data(), d->ing.pending.size()}, svb, &pd);
    if (rc) return rc;
    parts.push_back(ycrdt_buf{pd.ptr, pd.len});
  }
  rc = ycrdt_merge_updates(e, parts.data(), parts.size(), out);
  ycrdt_free(&pd);
  return rc;
}

int ycrdt_encode_state_vector(ycrdt_doc* d, ycrdt_out* out) {
  if (!d || !out) return fail(YCRDT_E_ARG, "null arg");
  out->ptr = nullptr;
  out->len = 0;
  const int rc = flush(d);
  if (rc) return rc;
  const std::vector<uint8_t>* src = &d->sv;  // device-written: descending, or store order (compat 135)
  out->len = src->size();
  out->ptr = (uint8_t*)malloc(out->len ? out->len : 1);
  if (!out->ptr) { out->len = 0; return fail(YCRDT_E_CAPACITY, "host allocation failed"); }
  if (out->len) memcpy(out->ptr, src->data(), out->len);
  return YCRDT_OK;
}

int ycrdt_doc_last_stats(ycrdt_doc* d, ycrdt_merge_stats* st) {
  if (!d || !st) return fail(YCRDT_E_ARG, "null arg");
  const int rc = flush(d);
  if (rc) return rc;
  *st = d->last;
  return YCRDT_OK;
}

int ycrdt_batch_stage(ycrdt_engine* e, const ycrdt_buf* ups, size_t n, ycrdt_batch** out) {
  if (!e || !out || (!ups && n)) return fail(YCRDT_E_ARG, "null arg");
  HIPCHK(hipSetDevice(e->device));
  auto* b = new ycrdt_batch();
  b->e = e;
  int rc = stage(b, ups, n, nullptr, 0);
  if (rc) { ycrdt_batch_destroy(b); return rc; }
  *out = b;
  return YCRDT_OK;
}

int ycrdt_batch_stage_docs(ycrdt_engine* e, const ycrdt_buf* ups, const uint32_t* doc_of, size_t n, uint32_t ndocs,
                           ycrdt_batch** out) {
  if (!e || !out || (n && (!ups || !doc_of)) || !ndocs) return fail(YCRDT_E_ARG, "null arg");
  HIPCHK(hipSetDevice(e->device));
  auto* b = new ycrdt_batch();
  b->e = e;
  int rc = stage(b, ups, n, nullptr, 0, doc_of, ndocs);
  if (rc) { ycrdt_batch_destroy(b); return rc; }
  b->ndocs = ndocs;
  *out = b;
  return YCRDT_OK;
}

int ycrdt_batch_result_docs(ycrdt_batch* b, ycrdt_out* updates, ycrdt_out* svs) {
  if (!b || !b->merged || !updates) return fail(YCRDT_E_ARG, "batch not merged");
  ycrdt_engine* e = b->e;
  if (e->ws_owner != b) return fail(YCRDT_E_ARG, "batch result no longer available (another engine call ran since ycrdt_batch_merge)");
  HIPCHK(hipSetDevice(e->device));
  for (uint32_t d = 0; d < b->ndocs; ++d) { updates[d] = ycrdt_out{nullptr, 0}; if (svs) svs[d] = ycrdt_out{nullptr, 0}; }
  if (b->ndocs == 1) return ycrdt_batch_result(b, updates, svs);
  const int rc = split_docs(e, b, updates, svs);
  if (rc) for (uint32_t d = 0; d < b->ndocs; ++d) { ycrdt_free(&updates[d]); if (svs) ycrdt_free(&svs[d]); }
  return rc;
}

int ycrdt_batch_result_docs_packed(ycrdt_batch* b, uint8_t* dst, uint64_t cap, uint64_t* offs, uint64_t* total) {
  if (!b || !b->merged) return fail(YCRDT_E_ARG, "batch not merged");
  ycrdt_engine* e = b->e;
  if (e->ws_owner != b) return fail(YCRDT_E_ARG, "batch result no longer available (another engine call ran since ycrdt_batch_merge)");
  HIPCHK(hipSetDevice(e->device));
  if (b->ndocs == 1 && !b->packed) {  // one document: the update and the state vector as they are
    b->pack_offs = {0, e->out_bytes, e->out_bytes + e->sv_bytes};
  } else if (const int rc = pack_docs(e, b)) {
    return rc;
  }
  const std::vector<uint64_t>& o = b->pack_offs;
  if (total) *total = o.back();
  if (offs) memcpy(offs, o.data(), sizeof(uint64_t) * o.size());
  if (!dst) return YCRDT_OK;
  if (cap < o.back()) return fail(YCRDT_E_ARG, "destination smaller than the packed result");
  if (b->ndocs == 1) {
    if (const int rc = d2h_span(e, dst, e->w.out, e->out_bytes)) return rc;
    return d2h_span(e, dst + e->out_bytes, e->w.sv_out, e->sv_bytes);
  }
  return d2h_span(e, dst, (const uint8_t*)e->bufs[B_PACK].p, o.back());
}
int ycrdt_merge_docs(ycrdt_engine* e, const ycrdt_buf* ups, const uint32_t* doc_of, size_t n, uint32_t ndocs,
                     ycrdt_out* updates, ycrdt_out* svs) {
  if (!e || !updates || (n && (!ups || !doc_of)) || !ndocs) return fail(YCRDT_E_ARG, "null arg");
  HIPCHK(hipSetDevice(e->device));
  ycrdt_batch& b = scratch_batch(e);
  int rc = stage(&b, ups, n, nullptr, 0, doc_of, ndocs);
  if (rc == YCRDT_OK) rc = run_merge(e, &b, nullptr);
  if (rc) return rc;
  b.merged = true;
  e->ws_owner = &b;
  const uint32_t nd = b.ndocs;
  b.ndocs = ndocs;
  rc = ycrdt_batch_result_docs(&b, updates, svs);
  b.ndocs = nd;
  return rc;
}

int ycrdt_batch_merge(ycrdt_batch* b, ycrdt_merge_stats* st) {
  if (!b) return fail(YCRDT_E_ARG, "null batch");
  HIPCHK(hipSetDevice(b->e->device));
  int rc = run_merge(b->e, b, nullptr);
  if (rc == YCRDT_OK) {
    b->merged = true;
    b->e->ws_owner = b;
    if (st) *st = b->e->last;
  }
  return rc;
}

int ycrdt_comm_unique_id(uint8_t id[YCRDT_COMM_ID_BYTES]) {
  if (!id) return fail(YCRDT_E_ARG, "null arg");
  std::string err;
  if (yc::comm_unique_id(id, err)) return fail(YCRDT_E_DEVICE, err);
  return YCRDT_OK;
}

int ycrdt_comm_create(ycrdt_engine* e, int nranks, int rank, const uint8_t id[YCRDT_COMM_ID_BYTES], ycrdt_comm** out) {
  if (!e || !id || !out) return fail(YCRDT_E_ARG, "null arg");
  std::string err;
  *out = yc::comm_create(e->device, nranks, rank, id, err);
  if (!*out) return fail(YCRDT_E_DEVICE, err);
  return YCRDT_OK;
}

void ycrdt_comm_destroy(ycrdt_comm* c) { yc::comm_destroy(c); }

int ycrdt_comm_create_exchange(ycrdt_engine* e, int nranks, int rank, const ycrdt_exchange* x, ycrdt_comm** out) {
  if (!e || !x || !out) return fail(YCRDT_E_ARG, "null arg");
  std::string err;
  *out = yc::comm_create_exchange(e->device, nranks, rank, x, err);
  if (!*out) return fail(YCRDT_E_ARG, err);
  return YCRDT_OK;
}

uint32_t ycrdt_route(const uint8_t* id, size_t len, uint32_t world) {
  if (!world) return 0;
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < len; ++i) { h ^= id[i]; h *= 1099511628211ull; }
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  h ^= h >> 33;
  return (uint32_t)(h % world);
}

int ycrdt_comm_fleet_sv_allreduce_max(ycrdt_comm* c, ycrdt_engine* e, const uint32_t* docs, const ycrdt_buf* svs, size_t n,
                                      ycrdt_out* doc_ids, ycrdt_out* offs, ycrdt_out* blob) {
  if (!c || !e || !doc_ids || !offs || !blob || (n && (!docs || !svs))) return fail(YCRDT_E_ARG, "null arg");
  *doc_ids = ycrdt_out{nullptr, 0};
  *offs = ycrdt_out{nullptr, 0};
  *blob = ycrdt_out{nullptr, 0};
  HIPCHK(hipSetDevice(e->device));
  std::string err;
  std::vector<uint32_t> d;
  std::vector<uint64_t> o;
  std::vector<uint8_t> b;
  const int r = yc::comm_fleet_sv_allreduce_max(c, docs, svs, n, e->stream, d, o, b, err);
  if (r) return fail(r == -2 ? YCRDT_E_DECODE : r == -3 ? YCRDT_E_ARG : YCRDT_E_DEVICE, err);
  auto give = [](ycrdt_out* x, const void* p, size_t len) -> bool {
    x->ptr = (uint8_t*)malloc(len ? len : 1);
    if (!x->ptr) return false;
    x->len = len;
    if (len) memcpy(x->ptr, p, len);
    return true;
  };
  if (!give(doc_ids, d.data(), 4 * d.size()) || !give(offs, o.data(), 8 * o.size()) || !give(blob, b.data(), b.size())) {
    ycrdt_free(doc_ids);
    ycrdt_free(offs);
    ycrdt_free(blob);
    return fail(YCRDT_E_CAPACITY, "host allocation failed");
  }
  return YCRDT_OK;
}

int ycrdt_batch_merge_sharded(ycrdt_batch* b, ycrdt_comm* comm, uint32_t nshards, ycrdt_merge_stats* st) {
  if (!b || !nshards || nshards > 255) return fail(YCRDT_E_ARG, "bad batch / shard count (1..255)");
  if (b->ndocs > 1) return fail(YCRDT_E_ARG, "sharded merge of a multi-document batch");
  ShardSpec sh;
  sh.nshards = nshards;
  if (comm) {
    if ((uint32_t)yc::comm_size(comm) != nshards) return fail(YCRDT_E_ARG, "nshards must equal the communicator size");
    sh.shard = yc::comm_rank(comm);
    sh.comm = comm;
  }
  HIPCHK(hipSetDevice(b->e->device));
  int rc = run_merge(b->e, b, nullptr, nullptr, nullptr, &sh);
  if (rc != YCRDT_OK && comm && !sh.finished) {
    const std::string keep = g_err;
    if (sh.inside) {
      yc::comm_abort(comm);  // inside a data exchange: the peers' collectives return
    } else {                 // the peers wait in the next agreement: join it with a failure status
      uint32_t any = 0;
      std::string err;
      if (yc::comm_agree(comm, 1u, b->e->stream, any, err)) yc::comm_abort(comm);
    }
    g_err = keep;
  }
  if (rc == YCRDT_OK) {
    b->merged = true;
    b->e->ws_owner = b;
    if (st) *st = b->e->last;
  }
  return rc;
}

int ycrdt_comm_sv_allreduce_max(ycrdt_comm* c, ycrdt_engine* e, ycrdt_buf sv, ycrdt_out* out) {
  if (!c || !e || !out || (sv.len && !sv.ptr)) return fail(YCRDT_E_ARG, "null arg");
  out->ptr = nullptr;
  out->len = 0;
  HIPCHK(hipSetDevice(e->device));
  std::string err;
  std::vector<uint8_t> o;
  const int r = yc::comm_sv_allreduce_max(c, sv.ptr, sv.len, e->stream, o, err);
  if (r) return fail(r == -2 ? YCRDT_E_DECODE : YCRDT_E_DEVICE, err);
  out->len = o.size();
  out->ptr = (uint8_t*)malloc(o.size() ? o.size() : 1);
  if (!out->ptr) { out->len = 0; return fail(YCRDT_E_CAPACITY, "host allocation failed"); }
  memcpy(out->ptr, o.data(), o.size());
  return YCRDT_OK;
}

int ycrdt_comm_allgather(ycrdt_comm* c, ycrdt_engine* e, ycrdt_buf mine, ycrdt_out* blob, ycrdt_out* offs) {
  if (!c || !e || !blob || !offs || (mine.len && !mine.ptr)) return fail(YCRDT_E_ARG, "null arg");
  blob->ptr = offs->ptr = nullptr;
  blob->len = offs->len = 0;
  HIPCHK(hipSetDevice(e->device));
  std::string err;
  std::vector<std::vector<uint8_t>> parts;
  if (yc::comm_allgather_updates(c, mine.ptr, mine.len, e->stream, parts, err)) return fail(YCRDT_E_DEVICE, err);
  std::vector<uint64_t> o(1, 0);
  for (const auto& p : parts) o.push_back(o.back() + p.size());
  blob->ptr = (uint8_t*)malloc(o.back() ? o.back() : 1);
  offs->ptr = (uint8_t*)malloc(sizeof(uint64_t) * o.size());
  if (!blob->ptr || !offs->ptr) {
    free(blob->ptr);
    free(offs->ptr);
    blob->ptr = offs->ptr = nullptr;
    return fail(YCRDT_E_CAPACITY, "host allocation failed");
  }
  for (size_t r = 0; r < parts.size(); ++r)
    if (!parts[r].empty()) memcpy(blob->ptr + o[r], parts[r].data(), parts[r].size());
  memcpy(offs->ptr, o.data(), sizeof(uint64_t) * o.size());
  blob->len = o.back();
  offs->len = sizeof(uint64_t) * o.size();
  return YCRDT_OK;
}

int ycrdt_device_count(int* count) {
  if (!count) return fail(YCRDT_E_ARG, "null arg");
  *count = 0;
  if (hipGetDeviceCount(count) != hipSuccess) {
    (void)hipGetLastError();
    *count = 0;
    return fail(YCRDT_E_DEVICE, "no HIP device");
  }
  return YCRDT_OK;
}

int ycrdt_comm_ds_allgather(ycrdt_comm* c, ycrdt_engine* e, ycrdt_buf update, ycrdt_out* out) {
  if (!c || !e || !out || (update.len && !update.ptr)) return fail(YCRDT_E_ARG, "null arg");
  out->ptr = nullptr;
  out->len = 0;
  HIPCHK(hipSetDevice(e->device));
  std::string err;
  std::vector<std::vector<uint8_t>> parts;
  if (yc::comm_allgather_updates(c, update.ptr, update.len, e->stream, parts, err)) return fail(YCRDT_E_DEVICE, err);
  // the union: Y.mergeUpdates of the gathered updates on this engine (delete sets: sort + segmented max)
  std::vector<ycrdt_buf> bufs;
  for (const auto& p : parts) bufs.push_back(ycrdt_buf{p.data(), p.size()});
  return ycrdt_merge_updates(e, bufs.data(), bufs.size(), out);
}

int ycrdt_batch_result(ycrdt_batch* b, ycrdt_out* update, ycrdt_out* sv) {
  if (!b || !b->merged) return fail(YCRDT_E_ARG, "batch not merged");
  ycrdt_engine* e = b->e;
  // the result lives in the engine workspace until the next engine call overwrites it
  if (e->ws_owner != b) return fail(YCRDT_E_ARG, "batch result no longer available (another engine call ran since ycrdt_batch_merge)");
  HIPCHK(hipSetDevice(e->device));
  if (update) { update->ptr = nullptr; update->len = 0; }
  if (sv) { sv->ptr = nullptr; sv->len = 0; }
  if (update) {
    update->ptr = (uint8_t*)malloc(e->out_bytes ? e->out_bytes : 1);
    if (!update->ptr) return fail(YCRDT_E_CAPACITY, "host allocation failed");
    update->len = e->out_bytes;
    HIPCHK(hipMemcpy(update->ptr, e->w.out, update->len, hipMemcpyDeviceToHost));
  }
  if (sv) {
    sv->ptr = (uint8_t*)malloc(e->sv_bytes ? e->sv_bytes : 1);
    if (!sv->ptr) { ycrdt_free(update); return fail(YCRDT_E_CAPACITY, "host allocation failed"); }
    sv->len = e->sv_bytes;
    HIPCHK(hipMemcpy(sv->ptr, e->w.sv_out, sv->len, hipMemcpyDeviceToHost));
  }
  return YCRDT_OK;
}

int ycrdt_merge_updates(ycrdt_engine* e, const ycrdt_buf* ups, size_t n, ycrdt_out* out) {
  if (!e || !out || (!ups && n)) return fail(YCRDT_E_ARG, "null arg");
  out->ptr = nullptr;
  out->len = 0;
  if (n == 1) {  // mergeUpdatesV2 returns its single input unchanged (Y@39011)
    out->len = ups[0].len;
    out->ptr = (uint8_t*)malloc(out->len ? out->len : 1);
    if (out->len) memcpy(out->ptr, ups[0].ptr, out->len);
    return YCRDT_OK;
  }
  HIPCHK(hipSetDevice(e->device));
  ycrdt_batch& b = scratch_batch(e);  // engine-owned: no hipMalloc / hipFree per call
  int rc = stage(&b, ups, n, nullptr, 0);
  if (rc == YCRDT_OK) rc = run_lazy(e, &b, true, {}, out);
  return rc;
}

int ycrdt_diff_update(ycrdt_engine* e, ycrdt_buf update, ycrdt_buf sv, ycrdt_out* out) {
  if (!e || !out) return fail(YCRDT_E_ARG, "null arg");
  out->ptr = nullptr;
  out->len = 0;
  std::unordered_map<uint32_t, uint32_t> m;
  if (!parse_sv(sv.ptr, sv.len, m)) return fail(YCRDT_E_DECODE, "Integer out of range! (state vector)");
  std::vector<std::pair<uint32_t, uint32_t>> v(m.begin(), m.end());
  std::sort(v.begin(), v.end());
  HIPCHK(hipSetDevice(e->device));
  ycrdt_batch& b = scratch_batch(e);  // engine-owned: no hipMalloc / hipFree per call
  int rc = stage(&b, &update, 1, nullptr, 0);
  if (rc == YCRDT_OK) rc = run_lazy(e, &b, false, v, out);
  return rc;
}

int ycrdt_diff_updates(ycrdt_engine* e, const ycrdt_buf* updates, const ycrdt_buf* svs, size_t n, ycrdt_out* outs) {
  if (!e || (n && (!updates || !svs || !outs))) return fail(YCRDT_E_ARG, "null arg");
  for (size_t i = 0; i < n; ++i) { outs[i].ptr = nullptr; outs[i].len = 0; }
  if (!n) return YCRDT_OK;
  std::vector<std::pair<uint32_t, uint32_t>> v;
  std::vector<uint32_t> off(n + 1, 0);
  for (size_t i = 0; i < n; ++i) {
    std::unordered_map<uint32_t, uint32_t> m;
    if (!parse_sv(svs[i].ptr, svs[i].len, m)) return fail(YCRDT_E_DECODE, "Integer out of range! (state vector)");
    const size_t v0 = v.size();
    v.insert(v.end(), m.begin(), m.end());
    std::sort(v.begin() + v0, v.end());
    off[i + 1] = (uint32_t)v.size();
  }
  HIPCHK(hipSetDevice(e->device));
  ycrdt_batch& b = scratch_batch(e);  // engine-owned: no hipMalloc / hipFree per call
  int rc = stage(&b, updates, n, nullptr, 0);
  if (rc == YCRDT_OK) rc = run_lazy(e, &b, false, v, nullptr, &off, outs);
  return rc;
}

void ycrdt_batch_destroy(ycrdt_batch* b) {
  if (!b) return;
  hipSetDevice(b->e->device);
  if (b->e->ws_owner == b) b->e->ws_owner = nullptr;
  if (b->bytes.p) hipFree(b->bytes.p);
  if (b->pieces.p) hipFree(b->pieces.p);
  if (b->meta.p) hipFree(b->meta.p);
  delete b;
}

// ---- crdt.c materialisation + local ops (yc_view.hip, yc_host.cpp)

static int ensure_view(ycrdt_doc* d) {
  d->wants_view = true;
  int rc = flush(d);
  if (rc) return rc;
  if (d->view.valid) return YCRDT_OK;
  if (!d->state_len) {
    d->view = HostView();
    d->view.valid = true;
    return YCRDT_OK;
  }
  ycrdt_engine* e = d->e;
  HIPCHK(hipSetDevice(e->device));
  ycrdt_batch& b = scratch_batch(e);  // engine-owned: no hipMalloc / hipFree per call
  if (e->ws_owner != d) {  // the workspace no longer holds this doc's merge: redo it (idempotent)
    doc_pre(d, b);
    rc = stage(&b, nullptr, 0, &d->state, d->state_len);
    if (rc == YCRDT_OK) rc = run_merge(e, &b, nullptr);
    b.pre_src = -1;
    if (rc) return rc;
    e->ws_owner = d;
  }
  return run_view(e, &b, d->view);
}

static uint32_t next_clock(ycrdt_doc* d) {
  std::unordered_map<uint32_t, uint32_t> sv;
  parse_sv(d->sv.data(), d->sv.size(), sv);
  auto it = sv.find(d->client_id);
  return it == sv.end() ? 0u : it->second;
}

// A local op's update joins the ingest queue as a local transaction (no pending retry / pendingDs
// pass, like Yjs's local transact) and, when the host opted in, the incremental-delta list.
static int apply_local(ycrdt_doc* d, const std::vector<uint8_t>& u) {
  enqueue(d, u.data(), u.size(), true);
  if (!d->track_local) return YCRDT_OK;
  d->local.push_back(u);
  d->local_bytes += u.size();
  if (d->local.size() > 4096 || d->local_bytes > (size_t(64) << 20)) {  // bound the list: fold it into one update
    std::vector<ycrdt_buf> bufs;
    for (const auto& x : d->local) bufs.push_back(ycrdt_buf{x.data(), x.size()});
    ycrdt_out o{nullptr, 0};
    const int rc = ycrdt_merge_updates(d->e, bufs.data(), bufs.size(), &o);
    if (rc) return rc;
    d->local.assign(1, std::vector<uint8_t>(o.ptr, o.ptr + o.len));
    d->local_bytes = o.len;
    ycrdt_free(&o);
  }
  return YCRDT_OK;
}

int ycrdt_doc_track_local(ycrdt_doc* d, int on) {
  if (!d) return fail(YCRDT_E_ARG, "null doc");
  d->track_local = on != 0;
  if (!on) { d->local.clear(); d->local_bytes = 0; }
  return YCRDT_OK;
}

int ycrdt_doc_take_local_update(ycrdt_doc* d, ycrdt_out* out) {
  if (!d || !out) return fail(YCRDT_E_ARG, "null arg");
  out->ptr = nullptr;
  out->len = 0;
  d->track_local = true;  // from now on local ops are recorded for the next take
  const std::vector<std::vector<uint8_t>>& ops = d->local;
  if (ops.empty()) return empty_update(out);
  int rc = YCRDT_OK;
  if (ops.size() == 1) {  // Y.mergeUpdates returns a single input unchanged
    out->ptr = (uint8_t*)malloc(ops[0].size() ? ops[0].size() : 1);
    if (!out->ptr) return fail(YCRDT_E_CAPACITY, "host allocation failed");
    out->len = ops[0].size();
    memcpy(out->ptr, ops[0].data(), out->len);
  } else {
    std::vector<ycrdt_buf> bufs;
    for (const auto& u : ops) bufs.push_back(ycrdt_buf{u.data(), u.size()});
    rc = ycrdt_merge_updates(d->e, bufs.data(), bufs.size(), out);  // one update for the transaction
  }
  if (rc == YCRDT_OK) { d->local.clear(); d->local_bytes = 0; }  // on failure the ops stay for the next take
  return rc;
}

static OpTarget target_of(const char* root, const char* parent_key) {
  OpTarget t;
  t.root = root;
  t.nested = parent_key != nullptr;
  if (parent_key) t.key = parent_key;
  return t;
}

int ycrdt_type_json(ycrdt_doc* d, const char* root, const char* parent_key, int kind, ycrdt_out* out) {
  if (!d || !root || !out || kind < 0 || kind > 1) return fail(YCRDT_E_ARG, "bad arg");
  out->ptr = nullptr;
  out->len = 0;
  int rc = ensure_view(d);
  if (rc) return rc;
  std::string j, err;
  if (!view_type_json(d->view, target_of(root, parent_key), kind, j, err)) return fail(YCRDT_E_DECODE, err);
  out->len = j.size();
  out->ptr = (uint8_t*)malloc(j.size() + 1);
  if (!out->ptr) { out->len = 0; return fail(YCRDT_E_CAPACITY, "host allocation failed"); }
  memcpy(out->ptr, j.data(), j.size());
  out->ptr[j.size()] = 0;
  return YCRDT_OK;
}
static int read_out(const std::string& j, ycrdt_out* out);
int ycrdt_map_entries(ycrdt_doc* d, const char* root, const char* parent_key, ycrdt_out* out) {
  if (!d || !root || !out) return fail(YCRDT_E_ARG, "null arg");
  out->ptr = nullptr;
  out->len = 0;
  const int rc = ensure_view(d);
  if (rc) return rc;
  std::string j;
  view_map_entries(d->view, target_of(root, parent_key), j);
  return read_out(j, out);
}
int ycrdt_doc_json(ycrdt_doc* d, const char* root, int kind, ycrdt_out* out) {
  if (!d || !root || !out || kind < 0 || kind > 1) return fail(YCRDT_E_ARG, "bad arg");
  out->ptr = nullptr;
  out->len = 0;
  int rc = ensure_view(d);
  if (rc) return rc;
  std::string j, err;
  if (!view_root_json(d->view, root, kind, j, err)) return fail(YCRDT_E_DECODE, err);
  out->len = j.size();
  out->ptr = (uint8_t*)malloc(j.size() + 1);
  memcpy(out->ptr, j.data(), j.size());
  out->ptr[j.size()] = 0;
  return YCRDT_OK;
}

int ycrdt_map_type_at(ycrdt_doc* d, const char* root, const char* key, int32_t* type_ref) {
  if (!d || !root || !key || !type_ref) return fail(YCRDT_E_ARG, "null arg");
  int rc = ensure_view(d);
  if (rc) return rc;
  *type_ref = view_type_at(d->view, root, key);
  return YCRDT_OK;
}

int ycrdt_map_set(ycrdt_doc* d, const char* root, const char* parent_key, const char* key, const uint8_t* any,
                  size_t anylen) {
  if (!d || !root || !key || (!any && anylen)) return fail(YCRDT_E_ARG, "null arg");
  if (!any_values_ok(any, anylen, 1)) return fail(YCRDT_E_ARG, "bad any value");
  int rc = ensure_view(d);
  if (rc) return rc;
  std::vector<uint8_t> content{1};  // ContentAny([value])
  content.insert(content.end(), any, any + anylen);
  std::vector<uint8_t> u;
  std::string err;
  rc = encode_map_set(d->view, target_of(root, parent_key), key, d->client_id, next_clock(d), 8, content.data(),
                      content.size(), u, err);
  if (rc) return fail(rc, err);
  return apply_local(d, u);
}

int ycrdt_map_set_type(ycrdt_doc* d, const char* root, const char* parent_key, const char* key, uint32_t type_ref) {
  if (!d || !root || !key || type_ref > 1) return fail(YCRDT_E_ARG, "bad arg (type_ref: 0 = YArray, 1 = YMap)");
  int rc = ensure_view(d);
  if (rc) return rc;
  std::vector<uint8_t> content{(uint8_t)type_ref};  // ContentType: writeTypeRef
  std::vector<uint8_t> u;
  std::string err;
  rc = encode_map_set(d->view, target_of(root, parent_key), key, d->client_id, next_clock(d), 7, content.data(),
                      content.size(), u, err);
  if (rc) return fail(rc, err);
  return apply_local(d, u);
}

int ycrdt_map_delete(ycrdt_doc* d, const char* root, const char* parent_key, const char* key) {
  if (!d || !root || !key) return fail(YCRDT_E_ARG, "null arg");
  int rc = ensure_view(d);
  if (rc) return rc;
  std::vector<uint8_t> u;
  std::string err;
  bool nothing = false;
  rc = encode_map_delete(d->view, target_of(root, parent_key), key, u, nothing, err);
  if (rc) return fail(rc, err);
  return nothing ? YCRDT_OK : apply_local(d, u);
}

int ycrdt_array_insert(ycrdt_doc* d, const char* root, const char* parent_key, uint32_t index, const uint8_t* anys,
                       size_t len, uint32_t count) {
  if (!d || !root || (!anys && len)) return fail(YCRDT_E_ARG, "null arg");
  if (!any_values_ok(anys, len, count)) return fail(YCRDT_E_ARG, "bad any value");
  int rc = ensure_view(d);
  if (rc) return rc;
  std::vector<uint8_t> u;
  std::string err;
  bool nothing = false;
  rc = encode_array_insert(d->view, target_of(root, parent_key), index, anys, len, count, d->client_id, next_clock(d), u,
                           nothing, err);
  if (rc) return fail(rc, err);
  return nothing ? YCRDT_OK : apply_local(d, u);
}

int ycrdt_array_delete(ycrdt_doc* d, const char* root, const char* parent_key, uint32_t index, uint32_t length) {
  if (!d || !root) return fail(YCRDT_E_ARG, "null arg");
  int rc = ensure_view(d);
  if (rc) return rc;
  std::vector<uint8_t> u;
  std::string err;
  bool nothing = false;
  rc = encode_array_delete(d->view, target_of(root, parent_key), index, length, u, nothing, err);
  // like Yjs, what exists is deleted even when the range runs past the end (then it throws)
  if (!nothing && !u.empty()) {
    const int rc2 = apply_local(d, u);
    if (rc2) return rc2;
  }
  if (rc) return fail(rc, err);
  return YCRDT_OK;
}

// Per-key reads (YMap.get / has / size, YArray.length / get): the view's hash index, no JSON of
// the whole type. The first read after a change merges the queue and rebuilds the view, as toJSON.
static int read_out(const std::string& j, ycrdt_out* out) {
  out->len = j.size();
  out->ptr = (uint8_t*)malloc(j.size() + 1);
  if (!out->ptr) { out->len = 0; return fail(YCRDT_E_CAPACITY, "host allocation failed"); }
  memcpy(out->ptr, j.data(), j.size());
  return YCRDT_OK;
}

int ycrdt_map_get(ycrdt_doc* d, const char* root, const char* parent_key, const char* key, int* state, ycrdt_out* json) {
  if (!d || !root || !key || !state || !json) return fail(YCRDT_E_ARG, "null arg");
  json->ptr = nullptr;
  json->len = 0;
  const int rc = ensure_view(d);
  if (rc) return rc;
  std::string j;
  view_map_get(d->view, target_of(root, parent_key), key, *state, j);
  return read_out(j, json);
}

int ycrdt_map_size(ycrdt_doc* d, const char* root, const char* parent_key, uint32_t* size) {
  if (!d || !root || !size) return fail(YCRDT_E_ARG, "null arg");
  const int rc = ensure_view(d);
  if (rc) return rc;
  *size = view_map_size(d->view, target_of(root, parent_key));
  return YCRDT_OK;
}

int ycrdt_array_length(ycrdt_doc* d, const char* root, const char* parent_key, uint64_t* length) {
  if (!d || !root || !length) return fail(YCRDT_E_ARG, "null arg");
  const int rc = ensure_view(d);
  if (rc) return rc;
  *length = view_array_length(d->view, target_of(root, parent_key));
  return YCRDT_OK;
}

int ycrdt_array_get(ycrdt_doc* d, const char* root, const char* parent_key, uint64_t index, int* state, ycrdt_out* json) {
  if (!d || !root || !state || !json) return fail(YCRDT_E_ARG, "null arg");
  json->ptr = nullptr;
  json->len = 0;
  const int rc = ensure_view(d);
  if (rc) return rc;
  std::string j;
  view_array_get(d->view, target_of(root, parent_key), index, *state, j);
  return read_out(j, json);
}

int ycrdt_validate_update(ycrdt_buf update, int* structs_ok) {
  UpdScan sc;
  const bool ok = scan_update(update.ptr, update.len, false, sc);
  if (structs_ok) *structs_ok = sc.structs_ok ? 1 : 0;
  if (!ok && sc.unsupported) return fail(YCRDT_E_UNSUPPORTED, "an any value nests deeper than 32 levels (engine limit)");
  return ok ? YCRDT_OK : fail(YCRDT_E_DECODE, "Integer out of range!");
}

static int out_copy(ycrdt_out* o, const std::vector<uint8_t>& v) {
  if (!o) return YCRDT_OK;
  o->ptr = (uint8_t*)malloc(v.size() ? v.size() : 1);
  if (!o->ptr) { o->len = 0; return fail(YCRDT_E_CAPACITY, "host allocation failed"); }
  o->len = v.size();
  if (!v.empty()) memcpy(o->ptr, v.data(), v.size());
  return YCRDT_OK;
}

int ycrdt_debug_replay(const ycrdt_buf* ups, size_t n, ycrdt_merge_fn merge, void* ctx, ycrdt_out* sv, ycrdt_out* pending,
                       ycrdt_out* pending_ds) {
  if ((!ups && n) || !merge) return fail(YCRDT_E_ARG, "null arg");
  IngestState S;
  const MergeFn mf = [merge, ctx](const std::vector<const std::vector<uint8_t>*>& ins, std::vector<uint8_t>& out) -> int {
    std::vector<ycrdt_buf> b;
    for (const auto* v : ins) b.push_back(ycrdt_buf{v->data(), v->size()});
    ycrdt_out o{nullptr, 0};
    const int rc = merge(ctx, b.data(), b.size(), &o);
    if (rc) return rc;
    out.assign(o.ptr, o.ptr + o.len);
    return (int)YCRDT_OK;
  };
  std::string err;
  for (size_t i = 0; i < n; ++i) {
    UpdScan sc;
    if (!scan_update(ups[i].ptr, ups[i].len, false, sc)) return fail(YCRDT_E_DECODE, "Integer out of range!");
    const int rc = read_update(S, ups[i].ptr, ups[i].len, false, mf, err);
    if (rc) return fail(rc, err);
  }
  std::vector<uint8_t> s;
  uint32_t k = 0;
  std::vector<uint8_t> body;
  for (const auto& kv : S.state) { put_vu(body, kv.first); put_vu(body, kv.second); ++k; }
  put_vu(s, k);
  s.insert(s.end(), body.begin(), body.end());
  int rc = out_copy(sv, s);
  if (!rc) rc = out_copy(pending, S.has_pending ? S.pending : std::vector<uint8_t>());
  if (!rc) rc = out_copy(pending_ds, S.has_ds ? S.pending_ds : std::vector<uint8_t>());
  return rc;
}

int ycrdt_doc_client_id(ycrdt_doc* d, uint32_t* out) {
  if (!d || !out) return fail(YCRDT_E_ARG, "null arg");
  *out = d->client_id;
  return YCRDT_OK;
}

}  // extern "C"
