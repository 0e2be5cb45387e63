// yc_comm.h — the engine's RCCL layer (yc_comm.hip): communicator lifetime and the collectives of
// the multi-GPU path. Only this header and yc_comm.hip see RCCL types.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/ycrdt.h"
#include "yc_ingest.h"  // lib0 readers / writers

namespace yc {

int comm_unique_id(uint8_t* id, std::string& err);
ycrdt_comm* comm_create(int device, int nranks, int rank, const uint8_t* id, std::string& err);
// a communicator whose collectives run over the caller's host exchange (ycrdt_exchange)
ycrdt_comm* comm_create_exchange(int device, int nranks, int rank, const ycrdt_exchange* x, std::string& err);
void comm_destroy(ycrdt_comm* c);
// ncclCommAbort (RCCL transport): peers blocked in a collective this rank will not join return
void comm_abort(ycrdt_comm* c);
int comm_rank(const ycrdt_comm* c);
int comm_size(const ycrdt_comm* c);
int comm_device(const ycrdt_comm* c);
// max of one status word over the ranks (every rank calls it exactly once per exchange)
int comm_agree(ycrdt_comm* c, uint32_t mine, hipStream_t s, uint32_t& all, std::string& err);
// fleet state vectors: (document, state vector) pairs of this rank -> the union over the ranks,
// per document (ascending), clients descending; out_offs has one entry per document + 1
int comm_fleet_sv_allreduce_max(ycrdt_comm* c, const uint32_t* docs, const ycrdt_buf* svs, size_t n, hipStream_t s,
                                std::vector<uint32_t>& out_docs, std::vector<uint64_t>& out_offs,
                                std::vector<uint8_t>& out, std::string& err);
// in-place all-reduce of n u32 words on stream s (sum or max)
int comm_allreduce_u32(ycrdt_comm* c, uint32_t* buf, size_t n, bool max, hipStream_t s, std::string& err);
// state vector of the union of every rank's `sv` (max clock per client, 13.6 order)
int comm_sv_allreduce_max(ycrdt_comm* c, const uint8_t* sv, size_t n, hipStream_t s, std::vector<uint8_t>& out,
                          std::string& err);
// every rank's byte string, in rank order
int comm_allgather_updates(ycrdt_comm* c, const uint8_t* p, size_t n, hipStream_t s, std::vector<std::vector<uint8_t>>& out,
                           std::string& err);

}  // namespace yc
