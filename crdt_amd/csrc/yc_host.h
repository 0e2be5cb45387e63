// yc_host.h — host side of the materialised view: crdt.c JSON (YMap.toJSON / YArray.toJSON) and
// the encoders of local ops (YMap.set / delete, YArray.insert / delete) as Yjs v1 updates.
// Pure host C++ (no HIP): the device computes winners and list order (yc_view.hip); this file only
// decodes the values at the byte ranges the view hands over and writes new structs.
#pragma once
#include <cstdint>
#include <string>
#include <vector>
#include <unordered_map>

#include "yc_view.h"

namespace yc {

struct HostView {
  std::vector<ViewKey> keys;
  std::vector<ViewSeg> segs;
  std::vector<uint8_t> bytes;  // the merged doc state the byte ranges point into
  std::unordered_map<uint32_t, std::vector<uint32_t>> by_parent;  // parent unit (VNONE = root) -> keys
  // (parent, root name, entry key | array) -> list: the per-key lookups of YMap.get / has and the
  // local ops, O(1) instead of a scan of the parent's lists
  std::unordered_map<std::string, uint32_t> entry;
  std::unordered_map<std::string, std::vector<uint32_t>> root_entries;  // root name -> its YMap entries
  bool valid = false;

  void index();
  std::string str(uint32_t pos, uint32_t len) const { return std::string((const char*)bytes.data() + pos, len); }
  // the list of root `name` (psub null: the YArray list; else the YMap entry `psub`)
  const ViewKey* root_list(const std::string& name, const std::string* psub) const;
  // the list of the nested type whose item is `unit`
  const ViewKey* child_list(uint32_t unit, const std::string* psub) const;
};

// toJSON of root `name`: kind 0 = YMap, 1 = YArray (JSON.stringify text)
bool view_root_json(const HostView& v, const std::string& name, int kind, std::string& out, std::string& err);

// type_ref of the live shared type stored in root map `root` under `key` (YMap.get returning a
// Y.AbstractType), or -1 when the key holds a plain value or nothing
int view_type_at(const HostView& v, const std::string& root, const std::string& key);

// Where a local op writes: a root type, or the type stored in root map `root` under `key`.
struct OpTarget {
  std::string root;
  bool nested = false;
  std::string key;
};
// toJSON of a root type or of the type stored in a root map entry (its own list only); kind 0 map, 1 array
bool view_type_json(const HostView& v, const OpTarget& t, int kind, std::string& out, std::string& err);
// a YMap's live entries with their winning item ids: {"key": ["client:clock", value], ...}
bool view_map_entries(const HostView& v, const OpTarget& t, std::string& out);

// Per-key reads of the view (YMap.get / has / size, YArray.length / get) without building the
// type's JSON: state 0 = absent, 1 = present (`json` holds the value), 2 = present but `undefined`
// (YMap.has is true, toJSON drops it). A nested target whose type does not exist reads as empty.
void view_map_get(const HostView& v, const OpTarget& t, const std::string& key, int& state, std::string& json);
uint32_t view_map_size(const HostView& v, const OpTarget& t);
uint64_t view_array_length(const HostView& v, const OpTarget& t);
void view_array_get(const HostView& v, const OpTarget& t, uint64_t index, int& state, std::string& json);

// Local ops as one Yjs v1 update each (client, clock = the doc's next clock for its client).
// Values are lib0 `any` encodings (concatenated for inserts). Return 0 or a YCRDT_E_* code with
// `err` set; *nothing* = true when the op changes nothing (Yjs writes no struct either).
int encode_map_set(const HostView& v, const OpTarget& t, const std::string& key, uint32_t client, uint32_t clock,
                   uint32_t content_ref, const uint8_t* content, size_t content_len, std::vector<uint8_t>& out,
                   std::string& err);
int encode_map_delete(const HostView& v, const OpTarget& t, const std::string& key, std::vector<uint8_t>& out,
                      bool& nothing, std::string& err);
int encode_array_insert(const HostView& v, const OpTarget& t, uint32_t index, const uint8_t* anys, size_t len,
                        uint32_t count, uint32_t client, uint32_t clock, std::vector<uint8_t>& out, bool& nothing,
                        std::string& err);
int encode_array_delete(const HostView& v, const OpTarget& t, uint32_t index, uint32_t length,
                        std::vector<uint8_t>& out, bool& nothing, std::string& err);
// lib0 `any` value check (the whole buffer is `count` values)
bool any_values_ok(const uint8_t* p, size_t n, uint32_t count);

}  // namespace yc
