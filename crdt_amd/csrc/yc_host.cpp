// yc_host.cpp — crdt.c materialisation and local-op encoding over the device view (yc_view.hip).
//
// JSON follows Yjs 13.5.16 toJSON + JSON.stringify: YMap.toJSON (Y@51558, typeMapGetAll Y@49897:
// the entry's item, skipped when deleted, value = last element of its content), YArray.toJSON
// (typeListToArray Y@46408: every countable, undeleted element in list order), nested types
// recurse; lib0 readAny (L0@1937) for ContentAny values, JSON.parse text for ContentJSON.
// Local ops restate typeMapSet (Y@49334), typeMapDelete (Y@49261), typeListInsertGenerics
// (Y@48365) + typeListInsertGenericsAfter (Y@47498) and typeListDelete (Y@48835): the new item's
// origin / right origin are read off the view, and the struct is written as Item.write (Y@80416).
#include "yc_host.h"
#include "yc_parse.h"  // (yc_num.h: Number::toString for the JSON output)

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "ycrdt.h"

namespace yc {

namespace {

enum : uint32_t {
  R_GC = 0, R_DELETED = 1, R_JSON = 2, R_BINARY = 3, R_STRING = 4, R_EMBED = 5, R_FORMAT = 6, R_TYPE = 7,
  R_ANY = 8, R_DOC = 9
};

struct Rd {
  const uint8_t* b;
  size_t p, end;
  bool ok = true;
  uint32_t u8() {
    if (p >= end) { ok = false; return 0; }
    return b[p++];
  }
  uint32_t vu() {  // lib0 0.2.42 readVarUint (32-bit accumulation)
    uint32_t v = 0, shift = 0;
    for (;;) {
      if (p >= end) { ok = false; return 0; }
      const uint32_t r = b[p++];
      if (shift < 32) v |= (r & 0x7fu) << shift;
      shift += 7;
      if (r < 0x80u) return v;
      if (shift > 35) { ok = false; return 0; }
    }
  }
  double vi() {  // readVarInt: JS 32-bit shifts, `num >>> 0` on multi-byte values
    uint32_t r = u8();
    int32_t num = (int32_t)(r & 63u);
    const double sign = (r & 64u) ? -1.0 : 1.0;
    if (!(r & 128u)) return sign * num;
    uint32_t len = 6;
    for (;;) {
      r = u8();
      if (!ok) return 0;
      num = num | (int32_t)((r & 127u) << (len & 31u));
      len += 7;
      if (r < 128u) return sign * (double)(uint32_t)num;
      if (len > 41) { ok = false; return 0; }
    }
  }
  const uint8_t* take(size_t n) {
    if (end - p < n || p > end) { ok = false; p = end; return b; }
    const uint8_t* q = b + p;
    p += n;
    return q;
  }
};

void put_json_str(std::string& o, const uint8_t* s, size_t n) {
  o.push_back('"');
  for (size_t i = 0; i < n; ++i) {
    const unsigned char c = s[i];
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\b': o += "\\b"; break;
      case '\f': o += "\\f"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default:
        if (c < 0x20) {
          char t[8];
          snprintf(t, sizeof t, "\\u%04x", c);
          o += t;
        } else {
          o.push_back((char)c);
        }
    }
  }
  o.push_back('"');
}

void put_number(std::string& o, double x) {  // JSON.stringify(Number): Number::toString's text (yc_num.h)
  if (!std::isfinite(x)) { o += "null"; return; }
  if (x == 0) { o += "0"; return; }
  char d[20], t[40];
  int32_t n;
  const uint32_t k = f64_shortest(x < 0 ? -x : x, d, n);
  o.append(t, num_text(x < 0, d, k, n, t));
}

double be_f64(const uint8_t* p) {
  uint64_t u = 0;
  for (int i = 0; i < 8; ++i) u = (u << 8) | p[i];
  double d;
  memcpy(&d, &u, 8);
  return d;
}
float be_f32(const uint8_t* p) {
  uint32_t u = 0;
  for (int i = 0; i < 4; ++i) u = (u << 8) | p[i];
  float f;
  memcpy(&f, &u, 4);
  return f;
}

void put_uint8array(std::string& o, const uint8_t* p, size_t n) {  // JSON.stringify(Uint8Array)
  o.push_back('{');
  for (size_t i = 0; i < n; ++i) {
    char t[32];
    snprintf(t, sizeof t, "%s\"%zu\":%u", i ? "," : "", i, p[i]);
    o += t;
  }
  o.push_back('}');
}

// lib0 readAny -> JSON text; returns false for `undefined` (the caller omits / nulls it)
bool any_json(Rd& r, std::string& o, int depth) {
  if (depth > 4000) { r.ok = false; return false; }  // lib0 readAny recurses without a limit (V8 overflows its stack near here)
  const uint32_t tag = r.u8();
  switch (tag) {
    case 127: return false;  // undefined
    case 126: o += "null"; return true;
    case 125: put_number(o, r.vi()); return true;
    case 124: { const uint8_t* q = r.take(4); if (r.ok) put_number(o, (double)be_f32(q)); return true; }
    case 123: { const uint8_t* q = r.take(8); if (r.ok) put_number(o, be_f64(q)); return true; }
    case 122: {  // BigInt64 (JSON.stringify would throw; written as its decimal value)
      const uint8_t* q = r.take(8);
      if (!r.ok) return true;
      uint64_t u = 0;
      for (int i = 0; i < 8; ++i) u = (u << 8) | q[i];
      o += std::to_string((long long)u);
      return true;
    }
    case 121: o += "false"; return true;
    case 120: o += "true"; return true;
    case 119: { const uint32_t n = r.vu(); const uint8_t* q = r.take(n); if (r.ok) put_json_str(o, q, n); return true; }
    case 118: {
      const uint32_t n = r.vu();
      o.push_back('{');
      bool first = true;
      for (uint32_t i = 0; i < n && r.ok; ++i) {
        const uint32_t kl = r.vu();
        const uint8_t* k = r.take(kl);
        std::string v;
        if (!any_json(r, v, depth + 1)) continue;  // undefined members are dropped
        if (!first) o.push_back(',');
        first = false;
        put_json_str(o, k, kl);
        o.push_back(':');
        o += v;
      }
      o.push_back('}');
      return true;
    }
    case 117: {
      const uint32_t n = r.vu();
      o.push_back('[');
      for (uint32_t i = 0; i < n && r.ok; ++i) {
        if (i) o.push_back(',');
        std::string v;
        if (any_json(r, v, depth + 1)) o += v;
        else o += "null";
      }
      o.push_back(']');
      return true;
    }
    case 116: { const uint32_t n = r.vu(); const uint8_t* q = r.take(n); if (r.ok) put_uint8array(o, q, n); return true; }
    default: r.ok = false; return false;
  }
}

bool skip_any(Rd& r, int depth) {
  if (depth > 4000) { r.ok = false; return false; }  // lib0 readAny recurses without a limit (V8 overflows its stack near here)
  const uint32_t tag = r.u8();
  switch (tag) {
    case 127: case 126: case 121: case 120: return r.ok;
    case 125: r.vi(); return r.ok;
    case 124: r.take(4); return r.ok;
    case 123: case 122: r.take(8); return r.ok;
    case 119: case 116: { const uint32_t n = r.vu(); r.take(n); return r.ok; }
    case 118: { const uint32_t n = r.vu(); for (uint32_t i = 0; i < n && r.ok; ++i) { r.take(r.vu()); skip_any(r, depth + 1); } return r.ok; }
    case 117: { const uint32_t n = r.vu(); for (uint32_t i = 0; i < n && r.ok; ++i) skip_any(r, depth + 1); return r.ok; }
    default: r.ok = false; return false;
  }
}

uint32_t utf8_len(unsigned char c) { return c < 0x80u ? 1u : c < 0xE0u ? 2u : c < 0xF0u ? 3u : 4u; }

struct JsonCtx {
  const HostView& v;
  int depth = 0;
};

void type_json(JsonCtx& c, uint32_t parent_unit, uint32_t type_ref, const ViewKey* array_list, std::string& o);

// every element of a visible view segment, as JSON values (undefined kept as a flag)
void seg_elements(JsonCtx& c, const ViewSeg& s, std::vector<std::pair<bool, std::string>>& out, bool last_only) {
  const HostView& v = c.v;
  Rd r{v.bytes.data(), s.b0, s.b1};
  const uint32_t n = last_only ? 1u : s.len;
  switch (s.ref) {
    case R_ANY:
      for (uint32_t i = 0; i < n && r.ok; ++i) {
        std::string e;
        const bool def = any_json(r, e, 0);
        out.push_back({def, e});
      }
      return;
    case R_JSON:
      for (uint32_t i = 0; i < n && r.ok; ++i) {
        const uint32_t k = r.vu();
        const uint8_t* q = r.take(k);
        if (!r.ok) return;
        const std::string t((const char*)q, k);
        out.push_back({t != "undefined", t});
      }
      return;
    case R_STRING: {  // one element per UTF-16 code unit; astral characters stay whole
      size_t p = s.b0;
      while (p < s.b1) {
        const uint32_t l = std::min<uint32_t>(utf8_len(v.bytes[p]), (uint32_t)(s.b1 - p));
        std::string e;
        put_json_str(e, v.bytes.data() + p, l);
        out.push_back({true, e});
        p += l;
      }
      return;
    }
    case R_BINARY: {
      const uint32_t k = r.vu();
      const uint8_t* q = r.take(k);
      std::string e;
      if (r.ok) put_uint8array(e, q, k);
      out.push_back({true, e});
      return;
    }
    case R_TYPE: {
      const uint32_t tr = r.vu();
      std::string e;
      if (c.depth < 512) {
        ++c.depth;
        type_json(c, s.unit + s.len - 1, tr, nullptr, e);
        --c.depth;
      }
      out.push_back({true, e});
      return;
    }
    case R_EMBED: {
      const uint32_t k = r.vu();
      const uint8_t* q = r.take(k);
      out.push_back({true, r.ok ? std::string((const char*)q, k) : std::string("null")});
      return;
    }
    case R_FORMAT:  // ContentFormat.getContent() is [] (Y@72137 area): a map entry's value is undefined
      out.push_back({false, std::string()});
      return;
    default:
      out.push_back({true, "null"});  // ContentDoc is outside crdt.c
  }
}

void map_json(JsonCtx& c, uint32_t parent_unit, std::string& o) {
  const HostView& v = c.v;
  o.push_back('{');
  bool first = true;
  auto it = v.by_parent.find(parent_unit);
  if (it != v.by_parent.end()) {
    for (uint32_t ki : it->second) {
      const ViewKey& K = v.keys[ki];
      if (!(K.flags & VK_PSUB) || !(K.win.flags & VS_SET) || (K.win.flags & VS_DELETED) || !(K.win.flags & VS_ITEM)) continue;
      std::vector<std::pair<bool, std::string>> el;
      seg_elements(c, K.win, el, true);
      if (el.empty() || !el.back().first) continue;
      if (!first) o.push_back(',');
      first = false;
      put_json_str(o, v.bytes.data() + K.psub_pos, K.psub_len);
      o.push_back(':');
      o += el.back().second;
    }
  }
  o.push_back('}');
}

const ViewKey* list_of(const HostView& v, uint32_t parent_unit) {
  auto it = v.by_parent.find(parent_unit);
  if (it == v.by_parent.end()) return nullptr;
  for (uint32_t ki : it->second)
    if (!(v.keys[ki].flags & VK_PSUB)) return &v.keys[ki];
  return nullptr;
}

void array_json(JsonCtx& c, const ViewKey* L, std::string& o) {
  o.push_back('[');
  bool first = true;
  if (L) {
    for (uint32_t i = 0; i < L->nseg; ++i) {
      const ViewSeg& s = c.v.segs[L->seg0 + i];
      if ((s.flags & VS_DELETED) || !(s.flags & VS_COUNTABLE) || !(s.flags & VS_ITEM)) continue;
      std::vector<std::pair<bool, std::string>> el;
      seg_elements(c, s, el, false);
      for (auto& e : el) {
        if (!first) o.push_back(',');
        first = false;
        o += e.first ? e.second : std::string("null");
      }
    }
  }
  o.push_back(']');
}

void text_json(JsonCtx& c, const ViewKey* L, std::string& o) {  // YText.toJSON: the visible string
  std::string s;
  if (L)
    for (uint32_t i = 0; i < L->nseg; ++i) {
      const ViewSeg& g = c.v.segs[L->seg0 + i];
      if ((g.flags & VS_DELETED) || !(g.flags & VS_ITEM) || g.ref != R_STRING) continue;
      s.append((const char*)c.v.bytes.data() + g.b0, g.b1 - g.b0);
    }
  put_json_str(o, (const uint8_t*)s.data(), s.size());
}

// YMap (1) -> object, YText (2) -> string, XML types -> "" (XmlElement.toJSON is its XML text,
// outside crdt.c), everything else (YArray) -> array
void type_json(JsonCtx& c, uint32_t parent_unit, uint32_t type_ref, const ViewKey* array_list, std::string& o) {
  if (type_ref == 1) { map_json(c, parent_unit, o); return; }
  const ViewKey* L = array_list ? array_list : list_of(c.v, parent_unit);
  if (type_ref == 2) { text_json(c, L, o); return; }
  if (type_ref >= 3 && type_ref <= 6) { o += "\"\""; return; }
  array_json(c, L, o);
}

// ---- lib0 writers
void w_vu(std::vector<uint8_t>& o, uint32_t v) {
  while (v > 0x7fu) { o.push_back((uint8_t)(0x80u | (v & 0x7fu))); v >>= 7; }
  o.push_back((uint8_t)v);
}
void w_str(std::vector<uint8_t>& o, const std::string& s) {
  w_vu(o, (uint32_t)s.size());
  o.insert(o.end(), s.begin(), s.end());
}

// an item id; `set` marks presence (client ids use all 32 bits: 0xFFFFFFFF is a valid client)
struct Id {
  uint32_t client = 0, clock = 0;
  bool set = false;
  Id() = default;
  Id(uint32_t c, uint32_t k) : client(c), clock(k), set(true) {}
  bool some() const { return set; }
};

// Parent of the op's target type: root name, or the type item stored under root map `key`
struct ParentRef {
  bool root = true;
  Id item;            // nested: the type item's id
  uint32_t unit = VNONE;  // nested: its merged-store unit (for child lookup); root: VNONE
};

int resolve_parent(const HostView& v, const OpTarget& t, uint32_t want_type, ParentRef& pr, std::string& err) {
  if (!t.nested) { pr.root = true; pr.unit = VNONE; return YCRDT_OK; }
  const ViewKey* e = v.root_list(t.root, &t.key);
  if (!e || !(e->win.flags & VS_SET) || (e->win.flags & VS_DELETED) || e->win.ref != R_TYPE) {
    err = "no shared type at " + t.root + "." + t.key;
    return YCRDT_E_ARG;
  }
  Rd r{v.bytes.data(), e->win.b0, e->win.b1};
  const uint32_t tr = r.vu();
  if (!r.ok || tr != want_type) { err = "type mismatch at " + t.root + "." + t.key; return YCRDT_E_ARG; }
  pr.root = false;
  pr.item = {e->win.client, e->win.clock + e->win.len - 1};
  pr.unit = e->win.unit + e->win.len - 1;
  return YCRDT_OK;
}

const ViewKey* target_list(const HostView& v, const OpTarget& t, const ParentRef& pr, const std::string* psub) {
  return pr.root ? v.root_list(t.root, psub) : v.child_list(pr.unit, psub);
}

// One-struct update: numClients 1, numStructs 1, client, clock, Item.write, empty delete set
void write_item_update(std::vector<uint8_t>& o, uint32_t client, uint32_t clock, uint32_t ref, Id origin, Id rorigin,
                       const OpTarget& t, const ParentRef& pr, const std::string* psub, const uint8_t* content,
                       size_t content_len) {
  o.clear();
  w_vu(o, 1);
  w_vu(o, 1);
  w_vu(o, client);
  w_vu(o, clock);
  const uint32_t info = (ref & 31u) | (origin.some() ? 0x80u : 0u) | (rorigin.some() ? 0x40u : 0u) | (psub ? 0x20u : 0u);
  o.push_back((uint8_t)info);
  if (origin.some()) { w_vu(o, origin.client); w_vu(o, origin.clock); }
  if (rorigin.some()) { w_vu(o, rorigin.client); w_vu(o, rorigin.clock); }
  if (!origin.some() && !rorigin.some()) {
    if (pr.root) { w_vu(o, 1); w_str(o, t.root); }
    else { w_vu(o, 0); w_vu(o, pr.item.client); w_vu(o, pr.item.clock); }
    if (psub) w_str(o, *psub);
  }
  o.insert(o.end(), content, content + content_len);
  w_vu(o, 0);  // delete set: no clients
}

// delete-set-only update from (client, clock, len) element ranges
void write_ds_update(std::vector<uint8_t>& o, std::vector<std::array<uint32_t, 3>> r) {
  std::sort(r.begin(), r.end());
  std::vector<std::array<uint32_t, 3>> m;
  for (auto& x : r) {
    if (!m.empty() && m.back()[0] == x[0] && m.back()[1] + m.back()[2] == x[1]) m.back()[2] += x[2];
    else m.push_back(x);
  }
  o.clear();
  w_vu(o, 0);  // no structs
  std::vector<size_t> starts;
  for (size_t i = 0; i < m.size(); ++i)
    if (i == 0 || m[i][0] != m[i - 1][0]) starts.push_back(i);
  starts.push_back(m.size());
  w_vu(o, (uint32_t)(starts.size() - 1));
  for (size_t c = 0; c + 1 < starts.size(); ++c) {
    w_vu(o, m[starts[c]][0]);
    w_vu(o, (uint32_t)(starts[c + 1] - starts[c]));
    for (size_t i = starts[c]; i < starts[c + 1]; ++i) { w_vu(o, m[i][1]); w_vu(o, m[i][2]); }
  }
}

bool visible(const ViewSeg& s) { return (s.flags & VS_ITEM) && !(s.flags & VS_DELETED) && (s.flags & VS_COUNTABLE); }

}  // namespace

namespace {
std::string entry_key(uint32_t parent_unit, const uint8_t* name, uint32_t name_len, const uint8_t* psub, uint32_t psub_len,
                      bool has_psub) {
  std::string k;
  k.reserve(10 + name_len + psub_len);
  k.append((const char*)&parent_unit, 4);
  k.append((const char*)name, name_len);
  k.push_back('\0');
  k.push_back(has_psub ? 'P' : 'A');
  k.append((const char*)psub, psub_len);
  return k;
}
}  // namespace

void HostView::index() {
  by_parent.clear();
  entry.clear();
  root_entries.clear();
  for (uint32_t i = 0; i < keys.size(); ++i) by_parent[keys[i].parent_unit].push_back(i);
  for (auto& kv : by_parent) {  // deterministic member order: by entry name, then slot
    std::sort(kv.second.begin(), kv.second.end(), [&](uint32_t a, uint32_t b) {
      const std::string sa = str(keys[a].psub_pos, keys[a].psub_len), sb = str(keys[b].psub_pos, keys[b].psub_len);
      return sa != sb ? sa < sb : keys[a].slot < keys[b].slot;
    });
    // the first list (lowest slot) of every (parent, name, entry) is the one the lookups return
    for (uint32_t ki : kv.second) {
      const ViewKey& K = keys[ki];
      const bool root = K.parent_unit == VNONE, ps = (K.flags & VK_PSUB) != 0;
      entry.emplace(entry_key(K.parent_unit, root ? bytes.data() + K.name_pos : nullptr, root ? K.name_len : 0,
                              bytes.data() + K.psub_pos, ps ? K.psub_len : 0, ps),
                    ki);
      if (root && ps) root_entries[str(K.name_pos, K.name_len)].push_back(ki);
    }
  }
}

const ViewKey* HostView::root_list(const std::string& name, const std::string* psub) const {
  const auto it = entry.find(entry_key(VNONE, (const uint8_t*)name.data(), (uint32_t)name.size(),
                                       psub ? (const uint8_t*)psub->data() : nullptr, psub ? (uint32_t)psub->size() : 0, psub != nullptr));
  return it == entry.end() ? nullptr : &keys[it->second];
}

const ViewKey* HostView::child_list(uint32_t unit, const std::string* psub) const {
  const auto it = entry.find(entry_key(unit, nullptr, 0, psub ? (const uint8_t*)psub->data() : nullptr,
                                       psub ? (uint32_t)psub->size() : 0, psub != nullptr));
  return it == entry.end() ? nullptr : &keys[it->second];
}

int view_type_at(const HostView& v, const std::string& root, const std::string& key) {
  const ViewKey* e = v.root_list(root, &key);
  if (!e || !(e->win.flags & VS_SET) || (e->win.flags & VS_DELETED) || e->win.ref != R_TYPE) return -1;
  Rd r{v.bytes.data(), e->win.b0, e->win.b1};
  const uint32_t tr = r.vu();
  return r.ok ? (int)tr : -1;
}

bool view_root_json(const HostView& v, const std::string& name, int kind, std::string& out, std::string& err) {
  JsonCtx c{v};
  out.clear();
  if (kind == 0) {
    // root map entries: every root list named `name` with a parentSub
    out.push_back('{');
    bool first = true;
    auto it = v.root_entries.find(name);
    if (it != v.root_entries.end())
      for (uint32_t ki : it->second) {
        const ViewKey& K = v.keys[ki];
        if (!(K.win.flags & VS_SET) || (K.win.flags & VS_DELETED) || !(K.win.flags & VS_ITEM)) continue;
        std::vector<std::pair<bool, std::string>> el;
        seg_elements(c, K.win, el, true);
        if (el.empty() || !el.back().first) continue;
        if (!first) out.push_back(',');
        first = false;
        put_json_str(out, v.bytes.data() + K.psub_pos, K.psub_len);
        out.push_back(':');
        out += el.back().second;
      }
    out.push_back('}');
    return true;
  }
  array_json(c, v.root_list(name, nullptr), out);
  return true;
}

// toJSON of one shared type: a root type (view_root_json), or the YMap / YArray stored in root map
// `t.root` under `t.key` — only that type's own list is read (a nested YArray's toJSON no longer
// builds the JSON of the whole root map). A key that holds no type of `kind` gives {} / [].
bool view_type_json(const HostView& v, const OpTarget& t, int kind, std::string& out, std::string& err) {
  if (!t.nested) return view_root_json(v, t.root, kind, out, err);
  out.clear();
  ParentRef pr;
  std::string e2;
  if (resolve_parent(v, t, kind == 0 ? 1u : 0u, pr, e2) != YCRDT_OK) {
    out = kind == 0 ? "{}" : "[]";
    return true;
  }
  JsonCtx c{v};
  type_json(c, pr.unit, kind == 0 ? 1u : 0u, nullptr, out);
  return true;
}

// The live entries of a YMap with the id of each entry's winning item: {"key": ["client:clock",
// value], ...}. A key changed in a transaction (YMapEvent.keysChanged, Y@51190) is a key whose
// winning item changed — the same value set again is a new item — so the facade's map observers
// compare these ids, not the values (and nested-type contents never count, as in YMap.observe).
bool view_map_entries(const HostView& v, const OpTarget& t, std::string& out) {
  out = "{";
  std::vector<uint32_t> ks;
  if (!t.nested) {
    auto it = v.root_entries.find(t.root);
    if (it != v.root_entries.end()) ks = it->second;
  } else {
    ParentRef pr;
    std::string err;
    if (resolve_parent(v, t, 1, pr, err) == YCRDT_OK) {
      auto it = v.by_parent.find(pr.unit);
      if (it != v.by_parent.end()) ks = it->second;
    }
  }
  JsonCtx c{v};
  bool first = true;
  for (uint32_t ki : ks) {
    const ViewKey& K = v.keys[ki];
    if (!(K.flags & VK_PSUB) || !(K.win.flags & VS_SET) || (K.win.flags & VS_DELETED) || !(K.win.flags & VS_ITEM)) continue;
    std::vector<std::pair<bool, std::string>> el;
    seg_elements(c, K.win, el, true);
    if (el.empty() || !el.back().first) continue;
    if (!first) out.push_back(',');
    first = false;
    put_json_str(out, v.bytes.data() + K.psub_pos, K.psub_len);
    out += ":[\"" + std::to_string(K.win.client) + ":" + std::to_string(K.win.clock + K.win.len - 1) + "\",";
    out += el.back().second;
    out.push_back(']');
  }
  out.push_back('}');
  return true;
}

namespace {
// the list a read addresses (nullptr: it does not exist), `want` = 1 YMap, 0 YArray
const ViewKey* read_list(const HostView& v, const OpTarget& t, uint32_t want, const std::string* psub) {
  ParentRef pr;
  std::string err;
  if (resolve_parent(v, t, want, pr, err) != YCRDT_OK) return nullptr;
  return target_list(v, t, pr, psub);
}
}  // namespace

void view_map_get(const HostView& v, const OpTarget& t, const std::string& key, int& state, std::string& json) {
  state = 0;
  json.clear();
  const ViewKey* K = read_list(v, t, 1, &key);
  if (!K || !(K->win.flags & VS_SET) || (K->win.flags & VS_DELETED) || !(K->win.flags & VS_ITEM)) return;
  // typeMapGet (Y@49897): the last element of the entry's winning item
  JsonCtx c{v};
  std::vector<std::pair<bool, std::string>> el;
  seg_elements(c, K->win, el, true);
  if (el.empty()) return;
  state = el.back().first ? 1 : 2;
  if (state == 1) json = el.back().second;
}

uint32_t view_map_size(const HostView& v, const OpTarget& t) {
  uint32_t n = 0;
  auto count = [&](const ViewKey& K) {
    if ((K.flags & VK_PSUB) && (K.win.flags & VS_SET) && !(K.win.flags & VS_DELETED) && (K.win.flags & VS_ITEM)) ++n;
  };
  if (!t.nested) {
    const auto it = v.root_entries.find(t.root);
    if (it != v.root_entries.end())
      for (uint32_t ki : it->second) count(v.keys[ki]);
    return n;
  }
  ParentRef pr;
  std::string err;
  if (resolve_parent(v, t, 1, pr, err) != YCRDT_OK) return 0;
  const auto it = v.by_parent.find(pr.unit);
  if (it != v.by_parent.end())
    for (uint32_t ki : it->second) count(v.keys[ki]);
  return n;
}

uint64_t view_array_length(const HostView& v, const OpTarget& t) {
  const ViewKey* L = read_list(v, t, 0, nullptr);
  uint64_t n = 0;
  if (L)
    for (uint32_t i = 0; i < L->nseg; ++i)
      if (visible(v.segs[L->seg0 + i])) n += v.segs[L->seg0 + i].len;
  return n;
}

void view_array_get(const HostView& v, const OpTarget& t, uint64_t index, int& state, std::string& json) {
  state = 0;
  json.clear();
  const ViewKey* L = read_list(v, t, 0, nullptr);
  if (!L) return;
  for (uint32_t i = 0; i < L->nseg; ++i) {
    const ViewSeg& s = v.segs[L->seg0 + i];
    if (!visible(s)) continue;
    if (index >= s.len) { index -= s.len; continue; }
    JsonCtx c{v};
    std::vector<std::pair<bool, std::string>> el;
    seg_elements(c, s, el, false);
    if (index >= el.size()) return;
    // YArray.get of an `undefined` element: toJSON writes null there, get returns undefined
    state = el[index].first ? 1 : 2;
    if (state == 1) json = el[index].second;
    return;
  }
}

bool any_values_ok(const uint8_t* p, size_t n, uint32_t count) {
  Rd r{p, 0, n};
  for (uint32_t i = 0; i < count && r.ok; ++i) skip_any(r, 0);
  return r.ok && r.p == n;
}

int encode_map_set(const HostView& v, const OpTarget& t, const std::string& key, uint32_t client, uint32_t clock,
                   uint32_t content_ref, const uint8_t* content, size_t content_len, std::vector<uint8_t>& out,
                   std::string& err) {
  ParentRef pr;
  int rc = resolve_parent(v, t, 1, pr, err);
  if (rc) return rc;
  // typeMapSet: left = parent._map.get(key) (the entry's rightmost item, deleted or not)
  const ViewKey* e = target_list(v, t, pr, &key);
  Id origin;
  if (e && (e->win.flags & VS_SET)) origin = {e->win.client, e->win.clock + e->win.len - 1};
  write_item_update(out, client, clock, content_ref, origin, Id{}, t, pr, &key, content, content_len);
  return YCRDT_OK;
}

int encode_map_delete(const HostView& v, const OpTarget& t, const std::string& key, std::vector<uint8_t>& out,
                      bool& nothing, std::string& err) {
  ParentRef pr;
  int rc = resolve_parent(v, t, 1, pr, err);
  if (rc) return rc;
  const ViewKey* e = target_list(v, t, pr, &key);
  nothing = !e || !(e->win.flags & VS_SET) || (e->win.flags & VS_DELETED);
  if (nothing) return YCRDT_OK;
  write_ds_update(out, {{e->win.client, e->win.clock, e->win.len}});
  return YCRDT_OK;
}

int encode_array_insert(const HostView& v, const OpTarget& t, uint32_t index, const uint8_t* anys, size_t len,
                        uint32_t count, uint32_t client, uint32_t clock, std::vector<uint8_t>& out, bool& nothing,
                        std::string& err) {
  ParentRef pr;
  int rc = resolve_parent(v, t, 0, pr, err);
  if (rc) return rc;
  const ViewKey* L = target_list(v, t, pr, nullptr);
  uint64_t length = 0;
  if (L)
    for (uint32_t i = 0; i < L->nseg; ++i)
      if (visible(v.segs[L->seg0 + i])) length += v.segs[L->seg0 + i].len;
  if (index > length) { err = "Length exceeded!"; return YCRDT_E_ARG; }
  nothing = count == 0;
  if (nothing) return YCRDT_OK;
  // left = the element at index - 1 (split there), right = whatever follows it in the list,
  // deleted or not (typeListInsertGenericsAfter: right = left.right / parent._start)
  Id origin, rorigin;
  if (L && L->nseg) {
    if (index == 0) {
      const ViewSeg& s = v.segs[L->seg0];
      rorigin = {s.client, s.clock};
    } else {
      uint64_t acc = 0;
      for (uint32_t i = 0; i < L->nseg; ++i) {
        const ViewSeg& s = v.segs[L->seg0 + i];
        if (!visible(s)) continue;
        if (index <= acc + s.len) {
          const uint32_t off = (uint32_t)(index - acc) - 1;
          origin = {s.client, s.clock + off};
          if (off + 1 < s.len) rorigin = {s.client, s.clock + off + 1};
          else if (i + 1 < L->nseg) rorigin = {v.segs[L->seg0 + i + 1].client, v.segs[L->seg0 + i + 1].clock};
          break;
        }
        acc += s.len;
      }
    }
  }
  std::vector<uint8_t> content;
  w_vu(content, count);
  content.insert(content.end(), anys, anys + len);
  write_item_update(out, client, clock, R_ANY, origin, rorigin, t, pr, nullptr, content.data(), content.size());
  return YCRDT_OK;
}

int encode_array_delete(const HostView& v, const OpTarget& t, uint32_t index, uint32_t length,
                        std::vector<uint8_t>& out, bool& nothing, std::string& err) {
  ParentRef pr;
  int rc = resolve_parent(v, t, 0, pr, err);
  if (rc) return rc;
  nothing = length == 0;
  if (nothing) return YCRDT_OK;
  const ViewKey* L = target_list(v, t, pr, nullptr);
  std::vector<std::array<uint32_t, 3>> ranges;
  uint64_t acc = 0, left = length;
  if (L)
    for (uint32_t i = 0; i < L->nseg && left; ++i) {
      const ViewSeg& s = v.segs[L->seg0 + i];
      if (!visible(s)) continue;
      const uint64_t a = std::max<uint64_t>(acc, index), b = std::min<uint64_t>(acc + s.len, (uint64_t)index + length);
      if (a < b) {
        ranges.push_back({s.client, s.clock + (uint32_t)(a - acc), (uint32_t)(b - a)});
        left -= b - a;
      }
      acc += s.len;
    }
  if (ranges.empty()) nothing = true;
  else write_ds_update(out, ranges);
  if (left) { err = "Length exceeded!"; return YCRDT_E_ARG; }  // Yjs throws after deleting what exists
  return YCRDT_OK;
}

}  // namespace yc
