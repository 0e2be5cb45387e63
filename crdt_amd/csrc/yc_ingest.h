// yc_ingest.h — host side of Y.applyUpdate: the update scanner (validation + struct headers) and
// Yjs's pending-struct machinery restated on struct headers.
//
// Yjs never throws on missing dependencies. readUpdateV2 (Y@21330) integrates what it can
// (integrateStructs, Y@19963: clients high → low, stack dives into the client a struct waits on),
// parks the rest as store.pendingStructs {update, missing state vector}, parks delete-set ranges
// beyond the known state as store.pendingDs (readAndApplyDeleteSet, Y@11619), merges new leftovers
// into the parked ones with mergeUpdates, and retries the parked structs once a later update
// advances a missing client. None of this needs the item contents: only ids, lengths and the
// origin / right origin / parent ids, which scan_update extracts. The device merge then only has
// to integrate every client up to the state this emulation reaches (per-client caps).
#pragma once
#include <cstdint>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include "yc_parse.h"

namespace yc {

struct ScanStruct {
  uint32_t client, clock;  // struct id
  uint32_t pos;            // byte offset of the info byte
  StructView v;            // decoded header; content = byte range [v.cpos, v.cend)
};
struct ScanSection { uint32_t client, clock, first, n; };  // structs [first, first + n)
struct ScanDs { uint32_t client, first, n; };              // ranges [first, first + n)
struct UpdScan {
  std::vector<ScanSection> secs;
  std::vector<ScanStruct> st;                          // per struct (headers == true)
  std::vector<ScanDs> ds;                              // delete-set clients in wire order
  std::vector<std::pair<uint32_t, uint32_t>> ranges;   // (clock, len) of every fully read range
  size_t struct_end = 0;     // byte offset of the delete set
  bool structs_ok = false;   // struct section decoded (else Yjs throws before changing anything)
  bool ds_ok = false;        // delete set decoded (else Yjs throws after integrating the structs)
  bool unsupported = false;  // an `any` value nests deeper than the decoder's 32 levels: valid Yjs
                             // input the engine refuses (YCRDT_E_UNSUPPORTED), never "malformed"
  uint64_t nstructs = 0;
};
// readClientsStructRefs (Y@19286) + readDeleteSet over one v1 update, with lib0 0.2.42's error
// behaviour (yc_parse.h, the same grammar the gfx950 decoder uses). Returns structs_ok && ds_ok.
bool scan_update(const uint8_t* p, size_t n, bool headers, UpdScan& out);
// What Yjs has applied when the delete set of an update is malformed: the struct section plus the
// delete-set ranges read before the error (readAndApplyDeleteSet applies range by range).
std::vector<uint8_t> repaired_update(const uint8_t* p, const UpdScan& sc);

using ClockMap = std::map<uint32_t, uint32_t>;  // client -> clock

struct IngestState {
  ClockMap state;                    // getStateVector(store): integrated structs only
  bool has_pending = false;          // store.pendingStructs
  std::vector<uint8_t> pending;      //   .update (v1 image of Yjs's v2 bytes)
  ClockMap missing;                  //   .missing
  bool has_ds = false;               // store.pendingDs
  std::vector<uint8_t> pending_ds;   //   (v1 image)
  std::vector<uint32_t> order;       // store client insertion order (Yjs 13.5.16 DS / SV order)
};

// Y.mergeUpdates(ups) — supplied by the engine (the device lazy merge)
using MergeFn = std::function<int(const std::vector<const std::vector<uint8_t>*>&, std::vector<uint8_t>&)>;

// One Y.applyUpdate(doc, u) (local = false) or one local transaction's update (local = true: it
// integrates, but Yjs runs no pending retry and no pendingDs pass for local transactions).
// Advances S; returns 0 or a YCRDT_E_* code (err says why).
// ds_error: the update's delete set was cut short by a decode error (the queued bytes are the
// struct section + the ranges read before it, repaired_update): Yjs threw inside
// readAndApplyDeleteSet, so its ranges at or past the state are dropped (not store.pendingDs), the
// parked delete set is not re-applied and nothing is retried. `effective` (ds_error only) receives
// the update as it takes effect: the struct section + the ranges clipped to the state.
int read_update(IngestState& S, const uint8_t* u, size_t n, bool local, const MergeFn& merge, std::string& err,
                bool ds_error = false, std::vector<uint8_t>* effective = nullptr);

// varuint writer
inline void put_vu(std::vector<uint8_t>& o, uint32_t v) {
  while (v > 127u) { o.push_back((uint8_t)(0x80u | (v & 0x7fu))); v >>= 7; }
  o.push_back((uint8_t)v);
}
// decodes an encoded state vector (varuint n, (client, clock) × n)
bool parse_state_vector(const uint8_t* p, size_t n, ClockMap& out);

}  // namespace yc
