// yc_comm.hip — the exchanges of the multi-GPU path inside libycrdt, reachable from the C ABI and
// so from the Node addon (north_star "RCCL over xGMI does allreduce-max on state
// vectors and allgather of delete sets"):
//   * the flag-word sum that combines the key-hash shards of one document (ycrdt_batch_merge_sharded),
//   * the fleet state-vector all-reduce(MAX): every (document, client) clock of the topics the ranks
//     hold, as one dense all-reduce over the fleet's sorted key space (crdt.js:239,289 per topic,
//     batched over the fleet),
//   * the state-vector all-reduce of one document and the delete-set all-gather (its union is the
//     engine's own HIP mergeUpdates).
// Transport: RCCL (ncclCommInitRank from a unique id that rank 0 creates and the caller hands out
// over any byte channel; collectives on the caller's stream, device buffers) — or a host exchange
// the caller supplies (ycrdt_exchange: allreduce / allgather over host buffers), which runs the same
// library code over any transport (the world-size-2 gloo tests drive it with two processes on one
// GPU). Every primitive below goes through xg_allreduce / xg_allgather.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <rccl/rccl.h>
#include <rocprim/rocprim.hpp>

#include "yc_comm.h"

struct ycrdt_comm {
  ncclComm_t comm = nullptr;   // RCCL transport
  ycrdt_exchange x{};          // host transport (x.allreduce_u32 != nullptr)
  int nranks = 1, rank = 0, device = 0;
};

namespace yc {

namespace {
std::string nccl_msg(const char* what, ncclResult_t r) { return std::string(what) + ": " + ncclGetErrorString(r); }

// device scratch of the exchanges (counts, padded payloads); grown, never shrunk
struct Scratch {
  void* p = nullptr;
  size_t cap = 0;
  bool grow(size_t n) {
    if (n <= cap) return true;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, n ? n : 16) != hipSuccess) { (void)hipGetLastError(); return false; }
    cap = n;
    return true;
  }
  ~Scratch() { if (p) hipFree(p); }
};

bool host_xchg(const ycrdt_comm* c) { return c->x.allreduce_u32 != nullptr; }

// in-place all-reduce of n device words (op: sum / max)
int xg_allreduce(ycrdt_comm* c, uint32_t* dbuf, size_t n, bool max, hipStream_t s, std::string& err) {
  if (!n) return 0;
  if (!host_xchg(c)) {
    const ncclResult_t r = ncclAllReduce(dbuf, dbuf, n, ncclUint32, max ? ncclMax : ncclSum, c->comm, s);
    if (r != ncclSuccess) { err = nccl_msg("ncclAllReduce", r); return -1; }
    return 0;
  }
  std::vector<uint32_t> h(n);
  if (hipMemcpyAsync(h.data(), dbuf, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) { err = "exchange copy"; return -1; }
  if (c->x.allreduce_u32(c->x.ctx, h.data(), n, max ? 1 : 0) != 0) { err = "host exchange: allreduce failed"; return -1; }
  if (hipMemcpyAsync(dbuf, h.data(), sizeof(uint32_t) * n, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) { err = "exchange copy"; return -1; }
  return 0;
}
// drecv[r * bytes ..) = rank r's dsend (device buffers)
int xg_allgather(ycrdt_comm* c, const void* dsend, size_t bytes, void* drecv, hipStream_t s, std::string& err) {
  if (!host_xchg(c)) {
    const ncclResult_t r = ncclAllGather(dsend, drecv, bytes, ncclUint8, c->comm, s);
    if (r != ncclSuccess) { err = nccl_msg("ncclAllGather", r); return -1; }
    return 0;
  }
  std::vector<uint8_t> snd(bytes), rcv(bytes * c->nranks);
  if ((bytes && hipMemcpyAsync(snd.data(), dsend, bytes, hipMemcpyDeviceToHost, s) != hipSuccess) ||
      hipStreamSynchronize(s) != hipSuccess) { err = "exchange copy"; return -1; }
  if (c->x.allgather(c->x.ctx, snd.data(), bytes, rcv.data()) != 0) { err = "host exchange: allgather failed"; return -1; }
  if ((!rcv.empty() && hipMemcpyAsync(drecv, rcv.data(), rcv.size(), hipMemcpyHostToDevice, s) != hipSuccess) ||
      hipStreamSynchronize(s) != hipSuccess) { err = "exchange copy"; return -1; }
  return 0;
}

// all-gather of one variable-length byte string per rank: lengths first, then the payloads padded
// to the longest (the collectives need equal sizes)
int allgather_bytes(ycrdt_comm* c, const uint8_t* p, size_t n, hipStream_t s, std::vector<std::vector<uint8_t>>& out,
                    std::string& err) {
  Scratch lens, pay;
  const int R = c->nranks;
  if (!lens.grow(sizeof(uint64_t) * (R + 1))) { err = "hipMalloc failed (exchange)"; return -1; }
  uint64_t mine = n;
  if (hipMemcpyAsync((uint64_t*)lens.p + R, &mine, sizeof(uint64_t), hipMemcpyHostToDevice, s) != hipSuccess) { err = "copy"; return -1; }
  if (xg_allgather(c, (uint64_t*)lens.p + R, sizeof(uint64_t), lens.p, s, err)) return -1;
  std::vector<uint64_t> L(R);
  if (hipMemcpyAsync(L.data(), lens.p, sizeof(uint64_t) * R, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) { err = "copy"; return -1; }
  uint64_t mx = 0;
  for (uint64_t x : L) mx = x > mx ? x : mx;
  const size_t slot = (size_t)((mx + 15) & ~15ull) + 16;
  if (!pay.grow(slot * (R + 1))) { err = "hipMalloc failed (exchange)"; return -1; }
  uint8_t* send = (uint8_t*)pay.p + slot * R;
  if (n && hipMemcpyAsync(send, p, n, hipMemcpyHostToDevice, s) != hipSuccess) { err = "copy"; return -1; }
  if (xg_allgather(c, send, slot, pay.p, s, err)) return -1;
  std::vector<uint8_t> all(slot * R);
  if (hipMemcpyAsync(all.data(), pay.p, all.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) { err = "copy"; return -1; }
  out.assign(R, {});
  for (int i = 0; i < R; ++i) out[i].assign(all.begin() + slot * i, all.begin() + slot * i + L[i]);
  return 0;
}

struct MaxU32 {
  __host__ __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a > b ? a : b; }
};
constexpr uint64_t KEY_PAD = ~0ull;  // padding of the gathered key lists (document id 0xFFFFFFFF is refused)

// dense[pos(key)] = clock for every local (key, clock): keys are unique locally and present in the
// sorted key space
__global__ void k_sv_scatter(const uint64_t* __restrict__ space, uint64_t nspace, const uint64_t* __restrict__ keys,
                             const uint32_t* __restrict__ clocks, uint64_t n, uint32_t* __restrict__ dense) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t k = keys[i];
  uint64_t lo = 0, hi = nspace;
  while (lo < hi) { const uint64_t m = (lo + hi) >> 1; if (space[m] < k) lo = m + 1; else hi = m; }
  if (lo < nspace) dense[lo] = clocks[i];
}
}  // namespace

int comm_unique_id(uint8_t* id, std::string& err) {
  ncclUniqueId u;
  const ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) { err = nccl_msg("ncclGetUniqueId", r); return -1; }
  static_assert(sizeof(u.internal) == YCRDT_COMM_ID_BYTES, "unique id size");
  memcpy(id, u.internal, YCRDT_COMM_ID_BYTES);
  return 0;
}

ycrdt_comm* comm_create(int device, int nranks, int rank, const uint8_t* id, std::string& err) {
  if (nranks < 1 || rank < 0 || rank >= nranks || nranks > 255) { err = "bad rank / size"; return nullptr; }
  if (hipSetDevice(device) != hipSuccess) { err = "hipSetDevice failed"; return nullptr; }
  ncclUniqueId u;
  memcpy(u.internal, id, YCRDT_COMM_ID_BYTES);
  auto* c = new ycrdt_comm();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) { err = nccl_msg("ncclCommInitRank", r); delete c; return nullptr; }
  return c;
}

ycrdt_comm* comm_create_exchange(int device, int nranks, int rank, const ycrdt_exchange* x, std::string& err) {
  if (nranks < 1 || rank < 0 || rank >= nranks || nranks > 255) { err = "bad rank / size"; return nullptr; }
  if (!x || !x->allreduce_u32 || !x->allgather) { err = "exchange without allreduce_u32 / allgather"; return nullptr; }
  auto* c = new ycrdt_comm();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  c->x = *x;
  return c;
}

void comm_destroy(ycrdt_comm* c) {
  if (!c) return;
  if (c->comm) ncclCommDestroy(c->comm);
  delete c;
}

void comm_abort(ycrdt_comm* c) {
  if (c && c->comm) {
    ncclCommAbort(c->comm);
    c->comm = nullptr;
  }
}

int comm_rank(const ycrdt_comm* c) { return c->rank; }
int comm_size(const ycrdt_comm* c) { return c->nranks; }
int comm_device(const ycrdt_comm* c) { return c->device; }

int comm_allreduce_u32(ycrdt_comm* c, uint32_t* buf, size_t n, bool max, hipStream_t s, std::string& err) {
  return xg_allreduce(c, buf, n, max, s, err);
}

int comm_agree(ycrdt_comm* c, uint32_t mine, hipStream_t s, uint32_t& all, std::string& err) {
  Scratch w;
  if (!w.grow(sizeof(uint32_t))) { err = "hipMalloc failed (exchange)"; return -1; }
  if (hipMemcpyAsync(w.p, &mine, sizeof(uint32_t), hipMemcpyHostToDevice, s) != hipSuccess) { err = "copy"; return -1; }
  if (xg_allreduce(c, (uint32_t*)w.p, 1, true, s, err)) return -1;
  if (hipMemcpyAsync(&all, w.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) { err = "copy"; return -1; }
  return 0;
}

// State vector of the union: every rank's (client, clock) pairs all-gathered, max per client
// (allreduce-max over the union of client ids); written in descending client order (13.6).
int comm_sv_allreduce_max(ycrdt_comm* c, const uint8_t* sv, size_t n, hipStream_t s, std::vector<uint8_t>& out,
                          std::string& err) {
  std::vector<std::vector<uint8_t>> parts;
  if (allgather_bytes(c, sv, n, s, parts, err)) return -1;
  std::vector<std::pair<uint32_t, uint32_t>> cc;
  for (const auto& p : parts) {
    uint32_t pos = 0;
    bool ok = true;
    const uint32_t k = rd_vu(p.data(), pos, (uint32_t)p.size(), ok);
    for (uint32_t i = 0; i < k && ok; ++i) {
      const uint32_t cl = rd_vu(p.data(), pos, (uint32_t)p.size(), ok);
      const uint32_t ck = rd_vu(p.data(), pos, (uint32_t)p.size(), ok);
      if (ok) cc.push_back({cl, ck});
    }
    if (!ok) { err = "Integer out of range! (state vector)"; return -2; }
  }
  std::sort(cc.begin(), cc.end(), [](const auto& a, const auto& b) { return a.first != b.first ? a.first > b.first : a.second > b.second; });
  std::vector<std::pair<uint32_t, uint32_t>> u;
  for (const auto& x : cc)
    if (u.empty() || u.back().first != x.first) u.push_back(x);
  out.clear();
  put_vu(out, (uint32_t)u.size());
  for (const auto& x : u) { put_vu(out, x.first); put_vu(out, x.second); }
  return 0;
}

// Fleet state vectors: this rank holds `n` documents (ids docs[i], state
// vectors svs[i]) — any subset of the fleet, overlapping other ranks' or not. Result: for every
// document any rank holds, the state vector of the union (per client the max clock), in ascending
// document order, 13.6 client order inside each. Device work: the local (document << 32 | client,
// clock) pairs are sorted and reduced (max), the distinct keys of all ranks all-gathered, sorted
// and uniqued into the fleet's key space (identical on every rank), the clocks scattered into one
// dense u32 vector over it and combined by ONE all-reduce(MAX).
int comm_fleet_sv_allreduce_max(ycrdt_comm* c, const uint32_t* docs, const ycrdt_buf* svs, size_t n, hipStream_t s,
                                std::vector<uint32_t>& out_docs, std::vector<uint64_t>& out_offs,
                                std::vector<uint8_t>& out, std::string& err) {
  // ---- parse (host): one pass over the state vector bytes
  std::vector<uint64_t> keys;
  std::vector<uint32_t> clocks;
  int bad = 0;
  for (size_t i = 0; i < n && !bad; ++i) {
    if (docs[i] == 0xFFFFFFFFu) { bad = 1; err = "document id 0xFFFFFFFF is reserved"; break; }
    uint32_t pos = 0;
    bool ok = true;
    const uint8_t* p = svs[i].ptr;
    const uint32_t len = (uint32_t)svs[i].len;
    const uint32_t k = rd_vu(p, pos, len, ok);
    for (uint32_t j = 0; j < k && ok; ++j) {
      const uint32_t cl = rd_vu(p, pos, len, ok);
      const uint32_t ck = rd_vu(p, pos, len, ok);
      if (ok) { keys.push_back((uint64_t)docs[i] << 32 | cl); clocks.push_back(ck); }
    }
    if (!ok) { bad = 2; err = "Integer out of range! (state vector)"; }
  }
  // every rank learns whether any rank failed before the first data collective (a failing rank
  // must not leave its peers blocked in a collective it never joins)
  uint32_t any = 0;
  std::string e2;
  if (comm_agree(c, (uint32_t)bad, s, any, e2)) { err = e2; return -1; }
  if (bad) return bad == 2 ? -2 : -3;
  if (any) { err = "another rank failed the fleet state-vector exchange"; return -1; }
  const uint64_t m = keys.size();
  const int R = c->nranks;
  Scratch kin, vin, kout, vout, tmp, cnt, lens, gk, gks, space, dense;
  size_t tb = 0, tb2 = 0, tb3 = 0;
  // ---- local sort + max per key
  uint64_t u = 0;
  if (!kin.grow(8 * (m + 1)) || !vin.grow(4 * (m + 1)) || !kout.grow(8 * (m + 1)) || !vout.grow(4 * (m + 1)) ||
      !cnt.grow(16)) { err = "hipMalloc failed (fleet exchange)"; return -1; }
  uint64_t* lk = (uint64_t*)kin.p;  // reduced keys end up here
  uint32_t* lc = (uint32_t*)vin.p;
  if (m) {
    if (hipMemcpyAsync(kin.p, keys.data(), 8 * m, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(vin.p, clocks.data(), 4 * m, hipMemcpyHostToDevice, s) != hipSuccess) { err = "copy"; return -1; }
    rocprim::radix_sort_pairs(nullptr, tb, (const uint64_t*)kin.p, (uint64_t*)kout.p, (const uint32_t*)vin.p, (uint32_t*)vout.p,
                              (size_t)m, 0, 64, s);
    rocprim::reduce_by_key(nullptr, tb2, (const uint64_t*)kout.p, (const uint32_t*)vout.p, (size_t)m, (uint64_t*)kin.p,
                           (uint32_t*)vin.p, (uint64_t*)cnt.p, MaxU32(), rocprim::equal_to<uint64_t>(), s);
    if (!tmp.grow(std::max(tb, tb2) + 256)) { err = "hipMalloc failed (fleet exchange)"; return -1; }
    rocprim::radix_sort_pairs(tmp.p, tb, (const uint64_t*)kin.p, (uint64_t*)kout.p, (const uint32_t*)vin.p, (uint32_t*)vout.p,
                              (size_t)m, 0, 64, s);
    tb2 = tmp.cap;
    rocprim::reduce_by_key(tmp.p, tb2, (const uint64_t*)kout.p, (const uint32_t*)vout.p, (size_t)m, lk, lc, (uint64_t*)cnt.p,
                           MaxU32(), rocprim::equal_to<uint64_t>(), s);
    if (hipMemcpyAsync(&u, cnt.p, 8, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {
      err = "copy";
      return -1;
    }
  }
  // ---- the fleet's key space: all-gather of every rank's distinct keys (padded), sort, unique
  if (!lens.grow(8 * (R + 1))) { err = "hipMalloc failed (fleet exchange)"; return -1; }
  if (hipMemcpyAsync((uint64_t*)lens.p + R, &u, 8, hipMemcpyHostToDevice, s) != hipSuccess) { err = "copy"; return -1; }
  if (xg_allgather(c, (uint64_t*)lens.p + R, 8, lens.p, s, err)) return -1;
  std::vector<uint64_t> L(R);
  if (hipMemcpyAsync(L.data(), lens.p, 8 * R, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {
    err = "copy";
    return -1;
  }
  uint64_t mx = 0;
  for (uint64_t x : L) mx = std::max(mx, x);
  const uint64_t G = mx * R;
  if (!gk.grow(8 * (G + mx + 1)) || !gks.grow(8 * (G + 1)) || !space.grow(8 * (G + 1))) { err = "hipMalloc failed (fleet exchange)"; return -1; }
  uint64_t* send = (uint64_t*)gk.p + G;
  if (mx) {
    std::vector<uint64_t> pad(mx - u, KEY_PAD);
    if (u && hipMemcpyAsync(send, lk, 8 * u, hipMemcpyDeviceToDevice, s) != hipSuccess) { err = "copy"; return -1; }
    if (mx > u && hipMemcpyAsync(send + u, pad.data(), 8 * (mx - u), hipMemcpyHostToDevice, s) != hipSuccess) { err = "copy"; return -1; }
  }
  if (xg_allgather(c, send, 8 * mx, gk.p, s, err)) return -1;
  uint64_t K = 0;
  if (G) {
    size_t t1 = 0, t2 = 0;
    rocprim::radix_sort_keys(nullptr, t1, (const uint64_t*)gk.p, (uint64_t*)gks.p, (size_t)G, 0, 64, s);
    rocprim::unique(nullptr, t2, (const uint64_t*)gks.p, (uint64_t*)space.p, (uint64_t*)cnt.p, (size_t)G,
                    rocprim::equal_to<uint64_t>(), s);
    if (!tmp.grow(std::max(t1, t2) + 256)) { err = "hipMalloc failed (fleet exchange)"; return -1; }
    t1 = tmp.cap;
    rocprim::radix_sort_keys(tmp.p, t1, (const uint64_t*)gk.p, (uint64_t*)gks.p, (size_t)G, 0, 64, s);
    t2 = tmp.cap;
    rocprim::unique(tmp.p, t2, (const uint64_t*)gks.p, (uint64_t*)space.p, (uint64_t*)cnt.p, (size_t)G,
                    rocprim::equal_to<uint64_t>(), s);
    uint64_t last = 0;
    if (hipMemcpyAsync(&K, cnt.p, 8, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) { err = "copy"; return -1; }
    if (K && hipMemcpy(&last, (uint64_t*)space.p + K - 1, 8, hipMemcpyDeviceToHost) != hipSuccess) { err = "copy"; return -1; }
    if (K && last == KEY_PAD) --K;  // the padding sorts last
  }
  (void)tb3;
  // ---- dense clocks over the key space, one all-reduce(MAX)
  if (!dense.grow(4 * (K + 1))) { err = "hipMalloc failed (fleet exchange)"; return -1; }
  if (K && hipMemsetAsync(dense.p, 0, 4 * K, s) != hipSuccess) { err = "memset"; return -1; }
  if (u && K) hipLaunchKernelGGL(k_sv_scatter, dim3((uint32_t)(u / 256 + 1)), dim3(256), 0, s, (const uint64_t*)space.p, K, lk, lc, u,
                                 (uint32_t*)dense.p);
  if (xg_allreduce(c, (uint32_t*)dense.p, K, true, s, err)) return -1;
  std::vector<uint64_t> hk(K);
  std::vector<uint32_t> hc(K);
  if (K && (hipMemcpyAsync(hk.data(), space.p, 8 * K, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipMemcpyAsync(hc.data(), dense.p, 4 * K, hipMemcpyDeviceToHost, s) != hipSuccess)) { err = "copy"; return -1; }
  if (hipStreamSynchronize(s) != hipSuccess) { err = "copy"; return -1; }
  // ---- the documents any rank holds (a document whose state vector is empty on every rank has
  // no key above, yet it is held: its result is the empty state vector, encodeStateVector = [0])
  std::vector<uint32_t> held(docs, docs + n);
  std::sort(held.begin(), held.end());
  held.erase(std::unique(held.begin(), held.end()), held.end());
  std::vector<std::vector<uint8_t>> hparts;
  if (allgather_bytes(c, (const uint8_t*)held.data(), 4 * held.size(), s, hparts, err)) return -1;
  std::vector<uint32_t> all_docs;
  for (const auto& p : hparts) {
    const size_t k0 = all_docs.size();
    all_docs.resize(k0 + p.size() / 4);
    if (!p.empty()) memcpy(all_docs.data() + k0, p.data(), p.size() / 4 * 4);
  }
  std::sort(all_docs.begin(), all_docs.end());
  all_docs.erase(std::unique(all_docs.begin(), all_docs.end()), all_docs.end());
  // ---- per document: writeStateVector, clients descending (the keys of one document are a run)
  out_docs.clear();
  out_offs.clear();
  out.clear();
  uint64_t a = 0;
  for (const uint32_t d : all_docs) {
    uint64_t z = a;
    while (z < K && (uint32_t)(hk[z] >> 32) == d) ++z;
    out_docs.push_back(d);
    out_offs.push_back(out.size());
    put_vu(out, (uint32_t)(z - a));
    for (uint64_t i = z; i-- > a;) { put_vu(out, (uint32_t)hk[i]); put_vu(out, hc[i]); }
    a = z;
  }
  if (a != K) { err = "fleet exchange: a key of a document no rank holds"; return -1; }
  out_offs.push_back(out.size());
  return 0;
}

int comm_allgather_updates(ycrdt_comm* c, const uint8_t* p, size_t n, hipStream_t s, std::vector<std::vector<uint8_t>>& out,
                           std::string& err) {
  return allgather_bytes(c, p, n, s, out, err);
}

}  // namespace yc
