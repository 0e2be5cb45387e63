// yc_ingest.cpp — Y.applyUpdate on the host side: update scanner + Yjs pending-struct semantics
// (see yc_ingest.h). Plain C++; the device merge is reached only through the MergeFn callback.
#include "yc_ingest.h"

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/ycrdt.h"

namespace yc {

// ------------------------------------------------------------------------------------ scanner
bool scan_update(const uint8_t* b, size_t n, bool headers, UpdScan& o) {
  o = UpdScan();
  if (n >= 0xFFFFFFF0ull) return false;
  const uint32_t end = (uint32_t)n;
  uint32_t p = 0;
  bool ok = true;
  const uint32_t nc = rd_vu(b, p, end, ok);
  if (!ok) return false;
  for (uint32_t i = 0; i < nc; ++i) {
    const uint32_t ns = rd_vu(b, p, end, ok);
    const uint32_t client = rd_vu(b, p, end, ok);
    const uint32_t clock = rd_vu(b, p, end, ok);
    if (!ok) return false;
    ScanSection sec{client, clock, (uint32_t)o.st.size(), 0};
    uint64_t ck = clock;
    for (uint32_t k = 0; k < ns; ++k) {
      StructView v;
      const uint32_t pos = p;
      int r = parse_struct<true>(b, p, end, 0xFFFFFFFFu, &v);
      if (r > 0 && (v.ref == REF_JSON || v.ref == REF_EMBED || v.ref == REF_FORMAT)) {  // JSON.parse (k_struct_decode alike)
        const int jr = json_content(b, v.cpos, v.cend, v.ref);
        if (jr > 0) r = 0;
        if (jr < 0) {  // not in JSON.stringify's form: valid if JSON.parse takes it (the merge rewrites it, k_json_canon)
          thread_local std::vector<uint32_t> arena(JSON_ARENA_WORDS);
          uint32_t len = 0;
          const uint32_t cr = json_content_canon(b, v.cpos, v.cend, v.ref, nullptr, arena.data(), JSON_ARENA_WORDS, len);
          if (cr == JSON_BAD) r = 0;
          else if (cr != JSON_OK) r = -1;  // past the rewrite arena: refused
        }
      }
      if (r == -1) o.unsupported = true;  // skip_any's depth limit (exact budget: never the step count)
      if (r <= 0) return false;
      if (ck + v.len > 0xFFFFFFFFull) return false;  // clocks are u32 (k_struct_clock refuses the same)
      // an item whose origin, right origin or parent item is of its own client at or past its own
      // clock: Yjs takes own-client references as present (getMissing skips them) and then fails
      // to find the item (a TypeError inside integrateStructs); the engine refuses the update
      if (v.ref != REF_GC && v.ref != REF_SKIP &&
          (((v.info & 0x80u) && v.oc == client && v.ok_ >= ck) || ((v.info & 0x40u) && v.rc == client && v.rk >= ck) ||
           ((v.info & 0xC0u) == 0 && v.pkind == 2 && v.pa == client && v.pb >= ck)))
        return false;
      if (headers) o.st.push_back(ScanStruct{client, (uint32_t)ck, pos, v});
      ck += v.len;
      ++o.nstructs;
    }
    sec.n = headers ? ns : 0;
    o.secs.push_back(sec);
  }
  o.struct_end = p;
  o.structs_ok = true;
  // readAndApplyDeleteSet reads (and applies) range by range. The ranges are kept only where a
  // caller reads them (headers: the pending emulation) or where the set is cut short (the part read
  // before the error still applies: repaired_update); a valid set is only checked — a sync reply
  // carries the peer's whole delete set, 70 k ranges for a C2 document, on every Y.applyUpdate
  const uint32_t ds0 = p;
  // Checking skips t varuints eight bytes a load: a byte below 0x80 ends one (rd_vu), so a word is
  // passed whole while it ends at most t of them; rd_vu's only other error — a sixth continuation
  // byte in a row — sends the set to the exact reader (it ends no valid set: u32 values take five)
  auto skip_vus = [&](uint32_t& q, uint32_t t) -> bool {
    uint32_t run = 0;  // continuation bytes carried over from the words passed
    while (t && q + 8 <= end) {
      uint64_t w;
      std::memcpy(&w, b + q, 8);
      const uint64_t cont = w & 0x8080808080808080ull;
      const uint32_t ends = (uint32_t)(((~w & 0x8080808080808080ull) >> 7) * 0x0101010101010101ull >> 56);
      if (ends > t) break;
      if (cont & (cont >> 8) & (cont >> 16) & (cont >> 24) & (cont >> 32) & (cont >> 40)) return false;
      const uint32_t lead = cont == 0x8080808080808080ull ? 8u : (uint32_t)__builtin_ctzll(~cont & 0x8080808080808080ull) >> 3;
      if (run + lead >= 6) return false;
      run = cont == 0x8080808080808080ull ? run + 8 : (uint32_t)__builtin_clzll(~cont & 0x8080808080808080ull) >> 3;
      t -= ends;
      q += 8;
    }
    q -= run;  // back to the start of the varuint the last word passed ended inside of
    bool okd = true;
    for (; t; --t) {
      rd_vu(b, q, end, okd);
      if (!okd) return false;
    }
    return true;
  };
  auto check_ds = [&]() -> bool {
    uint32_t q = ds0;
    bool okd = true;
    const uint32_t nd = rd_vu(b, q, end, okd);
    if (!okd) return false;
    for (uint32_t i = 0; i < nd; ++i) {
      rd_vu(b, q, end, okd);
      const uint32_t nr = rd_vu(b, q, end, okd);
      if (!okd) return false;
      if (nr >= 0x80000000u || !skip_vus(q, 2 * nr)) return false;
    }
    return true;
  };
  auto read_ds = [&](bool keep) -> bool {
    uint32_t q = ds0;
    bool okd = true;
    const uint32_t nd = rd_vu(b, q, end, okd);
    if (!okd) return false;
    for (uint32_t i = 0; i < nd; ++i) {
      const uint32_t client = rd_vu(b, q, end, okd);
      const uint32_t nr = rd_vu(b, q, end, okd);
      if (!okd) return false;
      ScanDs e{client, (uint32_t)o.ranges.size(), 0};
      for (uint32_t k = 0; k < nr; ++k) {
        const uint32_t clock = rd_vu(b, q, end, okd);
        const uint32_t len = rd_vu(b, q, end, okd);
        if (!okd) { if (keep) o.ds.push_back(e); return false; }
        if (keep) o.ranges.push_back({clock, len});
        ++e.n;
      }
      if (keep) o.ds.push_back(e);
    }
    return true;
  };
  if (headers ? !read_ds(true) : !check_ds() && !read_ds(false)) {
    if (!headers) read_ds(true);  // (again, keeping what was read before the error)
    return false;
  }
  o.ds_ok = true;
  return true;
}

static void put_ds(std::vector<uint8_t>& o, const std::vector<std::pair<uint32_t, std::vector<std::pair<uint32_t, uint32_t>>>>& ds) {
  put_vu(o, (uint32_t)ds.size());
  for (const auto& c : ds) {
    put_vu(o, c.first);
    put_vu(o, (uint32_t)c.second.size());
    for (const auto& r : c.second) { put_vu(o, r.first); put_vu(o, r.second); }
  }
}

std::vector<uint8_t> repaired_update(const uint8_t* p, const UpdScan& sc) {
  std::vector<uint8_t> o(p, p + sc.struct_end);
  std::vector<std::pair<uint32_t, std::vector<std::pair<uint32_t, uint32_t>>>> ds;
  for (const auto& e : sc.ds) {
    if (!e.n) continue;
    ds.push_back({e.client, std::vector<std::pair<uint32_t, uint32_t>>(sc.ranges.begin() + e.first, sc.ranges.begin() + e.first + e.n)});
  }
  put_ds(o, ds);
  return o;
}

bool parse_state_vector(const uint8_t* p, size_t n, ClockMap& out) {
  if (n >= 0xFFFFFFF0ull) return false;
  uint32_t pos = 0;
  bool ok = true;
  const uint32_t k = rd_vu(p, pos, (uint32_t)n, ok);
  for (uint32_t i = 0; i < k && ok; ++i) {
    const uint32_t c = rd_vu(p, pos, (uint32_t)n, ok);
    const uint32_t cl = rd_vu(p, pos, (uint32_t)n, ok);
    if (ok) out[c] = cl;
  }
  return ok;
}

// ------------------------------------------------------------------------------------ rest encode
static void put_vstring(std::vector<uint8_t>& o, const uint8_t* b, uint32_t pos, uint32_t total) {
  uint32_t p = pos;
  bool ok = true;
  const uint32_t n = rd_vu(b, p, pos + total, ok);
  put_vu(o, n);
  o.insert(o.end(), b + p, b + p + n);
}

// Item.write / GC.write / Skip.write with offset 0 (Y@80416, Y@68955) of a decoded, NOT integrated
// struct: the parentSub of an item with an origin was never read (Y@19286), so its 0x20 bit is
// dropped; the parent of an origin-less item is the root name (parentInfo 1) or the parent id.
static void write_struct(std::vector<uint8_t>& o, const uint8_t* u, const ScanStruct& s) {
  const StructView& v = s.v;
  if (v.ref == REF_GC || v.ref == REF_SKIP) {
    o.push_back(v.ref);
    put_vu(o, v.len);
    return;
  }
  const bool ho = (v.info & 0x80u) != 0, hr = (v.info & 0x40u) != 0;
  const bool psub = !ho && !hr && (v.info & 0x20u);
  o.push_back((uint8_t)((v.ref & 31u) | (ho ? 0x80u : 0u) | (hr ? 0x40u : 0u) | (psub ? 0x20u : 0u)));
  if (ho) { put_vu(o, v.oc); put_vu(o, v.ok_); }
  if (hr) { put_vu(o, v.rc); put_vu(o, v.rk); }
  if (!ho && !hr) {
    if (v.pkind == 1) { o.push_back(1); put_vstring(o, u, v.pa, v.pb); }
    else { o.push_back(0); put_vu(o, v.pa); put_vu(o, v.pb); }
    if (psub) put_vstring(o, u, v.psub_pos, v.psub_len);
  }
  o.insert(o.end(), u + v.cpos, u + v.cend);
}

// ------------------------------------------------------------------------------------ integrateStructs
namespace {

struct RefList {
  uint32_t first = 0, n = 0, i = 0;
  bool dead = false;  // deleted from clientsStructRefs (parked)
};

uint32_t state_of(const ClockMap& m, uint32_t c) {
  const auto it = m.find(c);
  return it == m.end() ? 0u : it->second;
}

// Item.getMissing (Y@76507): the first referenced client whose state does not cover the reference
bool get_missing(const ClockMap& state, const ScanStruct& s, uint32_t& m) {
  const StructView& v = s.v;
  if (v.ref == REF_GC || v.ref == REF_SKIP) return false;  // GC.getMissing() = null
  if ((v.info & 0x80u) && v.oc != s.client && v.ok_ >= state_of(state, v.oc)) { m = v.oc; return true; }
  if ((v.info & 0x40u) && v.rc != s.client && v.rk >= state_of(state, v.rc)) { m = v.rc; return true; }
  if (!(v.info & 0xC0u) && v.pkind == 2 && v.pa != s.client && v.pb >= state_of(state, v.pa)) { m = v.pa; return true; }
  return false;
}

// Y@19963, over headers. Integrating a struct = advancing the client's state (and, the first time,
// appending the client to the store's insertion order). Returns true if structs were parked.
bool integrate_structs(IngestState& S, const uint8_t* u, const UpdScan& sc, std::vector<uint8_t>& rest, ClockMap& missing) {
  std::map<uint32_t, RefList> refs;  // Map.set: a second section of the same client replaces the first
  for (const auto& s : sc.secs) refs[s.client] = RefList{s.first, s.n, 0, false};
  std::vector<uint32_t> ids;
  for (const auto& kv : refs) ids.push_back(kv.first);  // ascending
  auto next_target = [&]() -> RefList* {
    while (!ids.empty()) {
      RefList& t = refs[ids.back()];
      if (t.i < t.n) return &t;
      ids.pop_back();
    }
    return nullptr;
  };
  RefList* cur = next_target();
  if (!cur) return false;
  std::vector<uint32_t> stack;
  std::map<uint32_t, std::pair<uint32_t, uint32_t>> parked;  // client -> [first struct, count)
  auto upd_missing = [&](uint32_t c, uint32_t k) {
    const auto it = missing.find(c);
    if (it == missing.end() || it->second > k) missing[c] = k;
  };
  auto add_stack_to_rest = [&]() {
    for (const uint32_t si : stack) {
      const uint32_t c = sc.st[si].client;
      const auto it = refs.find(c);
      if (it != refs.end() && !it->second.dead) {
        RefList& t = it->second;
        t.i--;  // the stack item was the last one taken from this client
        parked[c] = {t.first + t.i, t.n - t.i};
        t.dead = true;
        t.i = t.n = 0;
      } else {
        parked[c] = {si, 1};
      }
      ids.erase(std::remove(ids.begin(), ids.end(), c), ids.end());
    }
    stack.clear();
  };
  uint32_t h = cur->first + cur->i++;
  for (;;) {
    const ScanStruct& x = sc.st[h];
    if (x.v.ref != REF_SKIP) {
      const uint32_t local = state_of(S.state, x.client);
      const int64_t off = (int64_t)local - (int64_t)x.clock;
      if (off < 0) {
        stack.push_back(h);
        upd_missing(x.client, x.clock - 1);
        add_stack_to_rest();
      } else {
        uint32_t m = 0;
        if (get_missing(S.state, x, m)) {
          stack.push_back(h);
          const auto it = refs.find(m);
          if (it == refs.end() || it->second.dead || it->second.i == it->second.n) {
            upd_missing(m, state_of(S.state, m));
            add_stack_to_rest();
          } else {
            h = it->second.first + it->second.i++;
            continue;
          }
        } else if (off == 0 || off < (int64_t)x.v.len) {
          if (!S.state.count(x.client)) S.order.push_back(x.client);
          S.state[x.client] = x.clock + x.v.len;
        }
      }
    }
    if (!stack.empty()) {
      h = stack.back();
      stack.pop_back();
    } else if (cur && cur->i < cur->n) {
      h = cur->first + cur->i++;
    } else {
      cur = next_target();
      if (!cur) break;
      h = cur->first + cur->i++;
    }
  }
  if (parked.empty()) return false;
  // writeClientsStructs(restStructs) (Y@19025: clients descending) + an empty delete set
  rest.clear();
  put_vu(rest, (uint32_t)parked.size());
  for (auto it = parked.rbegin(); it != parked.rend(); ++it) {
    const uint32_t first = it->second.first, cnt = it->second.second;
    put_vu(rest, cnt);
    put_vu(rest, it->first);
    put_vu(rest, sc.st[first].clock);
    for (uint32_t k = 0; k < cnt; ++k) write_struct(rest, u, sc.st[first + k]);
  }
  put_vu(rest, 0);
  return true;
}

// readAndApplyDeleteSet (Y@11619): ranges (or their tails) at or beyond the client's state are not
// applied; they come back as a delete-set-only update (store.pendingDs), clients in first-add order
bool pending_ds_of(const UpdScan& sc, const ClockMap& state, std::vector<uint8_t>& out) {
  std::vector<std::pair<uint32_t, std::vector<std::pair<uint32_t, uint32_t>>>> ds;
  std::map<uint32_t, size_t> at;
  auto add = [&](uint32_t c, uint32_t clock, uint32_t len) {
    auto it = at.find(c);
    if (it == at.end()) { it = at.emplace(c, ds.size()).first; ds.push_back({c, {}}); }
    ds[it->second].second.push_back({clock, len});
  };
  for (const auto& e : sc.ds) {
    const uint32_t st = state_of(state, e.client);  // getState once per client
    for (uint32_t k = 0; k < e.n; ++k) {
      const uint32_t clock = sc.ranges[e.first + k].first, len = sc.ranges[e.first + k].second;
      const uint64_t endc = (uint64_t)clock + len;
      if (clock < st) {
        if ((uint64_t)st < endc) add(e.client, st, (uint32_t)(endc - st));
      } else {
        add(e.client, clock, len);
      }
    }
  }
  if (ds.empty()) return false;
  out.clear();
  put_vu(out, 0);  // no structs
  put_ds(out, ds);
  return true;
}

}  // namespace

// ------------------------------------------------------------------------------------ readUpdateV2
int read_update(IngestState& S, const uint8_t* u, size_t n, bool local, const MergeFn& merge, std::string& err, bool ds_error,
                std::vector<uint8_t>* effective) {
  UpdScan sc;
  if (!scan_update(u, n, true, sc)) {
    err = "internal: a queued update no longer decodes";
    return YCRDT_E_DECODE;
  }
  std::vector<uint8_t> rest;
  ClockMap rmissing;
  const bool parked = integrate_structs(S, u, sc, rest, rmissing);
  if (local) {
    if (parked) { err = "internal: a local transaction has missing dependencies"; return YCRDT_E_ARG; }
    return YCRDT_OK;
  }
  bool retry = false;
  if (S.has_pending) {
    for (const auto& kv : S.missing)
      if (kv.second < state_of(S.state, kv.first)) { retry = true; break; }
    if (parked) {
      for (const auto& kv : rmissing) {
        const auto it = S.missing.find(kv.first);
        if (it == S.missing.end() || it->second > kv.second) S.missing[kv.first] = kv.second;
      }
      std::vector<uint8_t> merged;
      const int rc = merge({&S.pending, &rest}, merged);
      if (rc) { err = "pending merge failed"; return rc; }
      S.pending.swap(merged);
    }
  } else if (parked) {
    S.has_pending = true;
    S.pending.swap(rest);
    S.missing.swap(rmissing);
  }
  if (ds_error) {  // readAndApplyDeleteSet threw: the ranges within the state are applied, no more
    if (effective) {
      std::vector<std::pair<uint32_t, std::vector<std::pair<uint32_t, uint32_t>>>> ds;
      for (const auto& e : sc.ds) {
        const uint32_t st = state_of(S.state, e.client);
        std::vector<std::pair<uint32_t, uint32_t>> rs;
        for (uint32_t k = 0; k < e.n; ++k) {
          const uint32_t clock = sc.ranges[e.first + k].first, len = sc.ranges[e.first + k].second;
          if (clock < st) rs.push_back({clock, (uint32_t)std::min<uint64_t>(len, st - clock)});
        }
        if (!rs.empty()) ds.push_back({e.client, rs});
      }
      effective->assign(u, u + sc.struct_end);
      put_ds(*effective, ds);
    }
    return YCRDT_OK;
  }
  // the update's delete set, then the parked delete set again (Y@21330)
  std::vector<uint8_t> ds1, ds2;
  const bool h1 = pending_ds_of(sc, S.state, ds1);
  if (S.has_ds) {
    UpdScan ps;
    if (!scan_update(S.pending_ds.data(), S.pending_ds.size(), true, ps)) { err = "internal: pendingDs"; return YCRDT_E_DECODE; }
    const bool h2 = pending_ds_of(ps, S.state, ds2);
    if (h1 && h2) {
      std::vector<uint8_t> merged;
      const int rc = merge({&ds1, &ds2}, merged);
      if (rc) { err = "pendingDs merge failed"; return rc; }
      S.pending_ds.swap(merged);
    } else if (h1) {
      S.pending_ds.swap(ds1);
    } else if (h2) {
      S.pending_ds.swap(ds2);
    } else {
      S.has_ds = false;
      S.pending_ds.clear();
    }
  } else if (h1) {
    S.has_ds = true;
    S.pending_ds.swap(ds1);
  }
  if (retry) {
    std::vector<uint8_t> p;
    p.swap(S.pending);
    S.has_pending = false;
    S.missing.clear();
    return read_update(S, p.data(), p.size(), false, merge, err);
  }
  return YCRDT_OK;
}

}  // namespace yc
