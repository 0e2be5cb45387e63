// yc_comm.hip — RCCL (over xGMI) inside libycrdt: the exchanges of the multi-GPU path, reachable
// from the C ABI and so from the Node addon (north_star "RCCL over xGMI does
// allreduce-max on state vectors and allgather of delete sets"):
//   * the flag-word sum that combines the key-hash shards of one document (ycrdt_batch_merge_sharded),
//   * the state-vector all-reduce(MAX) of one document held in parts by several ranks,
//   * the delete-set all-gather (its union is the engine's own HIP mergeUpdates).
// One communicator per engine device (ncclCommInitRank), bootstrapped from a unique id that rank 0
// creates and the caller distributes (a file, the launcher's store, torch.distributed — any byte
// channel). Every collective runs on the caller's stream.
#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <vector>

#include "yc_comm.h"

struct ycrdt_comm {
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0, device = 0;
};

namespace yc {

namespace {
std::string nccl_msg(const char* what, ncclResult_t r) { return std::string(what) + ": " + ncclGetErrorString(r); }

// device scratch of the small exchanges (counts, padded payloads); grown, never shrunk
struct Scratch {
  void* p = nullptr;
  size_t cap = 0;
  bool grow(size_t n) {
    if (n <= cap) return true;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, n) != hipSuccess) return false;
    cap = n;
    return true;
  }
  ~Scratch() { if (p) hipFree(p); }
};

// all-gather of one variable-length byte string per rank: lengths first, then the payloads padded
// to the longest (ncclAllGather needs equal sizes)
int allgather_bytes(ycrdt_comm* c, const uint8_t* p, size_t n, hipStream_t s, std::vector<std::vector<uint8_t>>& out,
                    std::string& err) {
  Scratch lens, pay;
  const int R = c->nranks;
  if (!lens.grow(sizeof(uint64_t) * (R + 1))) { err = "hipMalloc failed (exchange)"; return -1; }
  uint64_t mine = n;
  if (hipMemcpyAsync((uint64_t*)lens.p + R, &mine, sizeof(uint64_t), hipMemcpyHostToDevice, s) != hipSuccess) { err = "copy"; return -1; }
  ncclResult_t r = ncclAllGather((uint64_t*)lens.p + R, lens.p, 1, ncclUint64, c->comm, s);
  if (r != ncclSuccess) { err = nccl_msg("ncclAllGather", r); return -1; }
  std::vector<uint64_t> L(R);
  if (hipMemcpyAsync(L.data(), lens.p, sizeof(uint64_t) * R, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) { err = "copy"; return -1; }
  uint64_t mx = 0;
  for (uint64_t x : L) mx = x > mx ? x : mx;
  const size_t slot = (size_t)((mx + 15) & ~15ull) + 16;
  if (!pay.grow(slot * (R + 1))) { err = "hipMalloc failed (exchange)"; return -1; }
  uint8_t* send = (uint8_t*)pay.p + slot * R;
  if (n && hipMemcpyAsync(send, p, n, hipMemcpyHostToDevice, s) != hipSuccess) { err = "copy"; return -1; }
  r = ncclAllGather(send, pay.p, slot, ncclUint8, c->comm, s);
  if (r != ncclSuccess) { err = nccl_msg("ncclAllGather", r); return -1; }
  std::vector<uint8_t> all(slot * R);
  if (hipMemcpyAsync(all.data(), pay.p, all.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) { err = "copy"; return -1; }
  out.assign(R, {});
  for (int i = 0; i < R; ++i) out[i].assign(all.begin() + slot * i, all.begin() + slot * i + L[i]);
  return 0;
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

void comm_destroy(ycrdt_comm* c) {
  if (!c) return;
  if (c->comm) ncclCommDestroy(c->comm);
  delete c;
}

int comm_rank(const ycrdt_comm* c) { return c->rank; }
int comm_size(const ycrdt_comm* c) { return c->nranks; }

int comm_allreduce_u32(ycrdt_comm* c, uint32_t* buf, size_t n, bool max, hipStream_t s, std::string& err) {
  const ncclResult_t r = ncclAllReduce(buf, buf, n, ncclUint32, max ? ncclMax : ncclSum, c->comm, s);
  if (r != ncclSuccess) { err = nccl_msg("ncclAllReduce", r); return -1; }
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

int comm_allgather_updates(ycrdt_comm* c, const uint8_t* p, size_t n, hipStream_t s, std::vector<std::vector<uint8_t>>& out,
                           std::string& err) {
  return allgather_bytes(c, p, n, s, out, err);
}

}  // namespace yc
