// ycw.cpp — seeded synthetic replica-update workloads.
//
// Emulates N Yjs replicas doing local YMap set/delete ops (typeMapSet Y@49334 / typeMapDelete
// Y@49261 semantics) on one root map, optionally starting from a base snapshot written by one
// client, and emits exactly the bytes Yjs would send: the base snapshot update plus every replica's
// encodeStateAsUpdate(replica, baseSV) (13.6 canonical delete-set order). The op script can be
// exported as JSON so tests/golden/gen/pin_workload.js can replay it through real Yjs and pin the
// generator byte for byte.
//
// This is benchmark/test input generation, not part of the merge path.
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>

namespace {

struct Rng {  // mulberry32
  uint32_t a;
  explicit Rng(uint32_t s) : a(s) {}
  uint32_t next_u32() {
    a += 0x6D2B79F5u;
    uint32_t t = a;
    t = (t ^ (t >> 15)) * (1u | t);
    t = (t + ((t ^ (t >> 7)) * (61u | t))) ^ t;
    return t ^ (t >> 14);
  }
  double next() { return next_u32() / 4294967296.0; }
  uint32_t below(uint32_t n) { return (uint32_t)(next() * n); }
};

struct W {
  std::vector<uint8_t> b;
  void u8(uint8_t v) { b.push_back(v); }
  void vu(uint32_t v) {
    while (v > 127) { b.push_back((uint8_t)(0x80 | (v & 0x7f))); v >>= 7; }
    b.push_back((uint8_t)v);
  }
  void vstr(const std::string& s) { vu((uint32_t)s.size()); b.insert(b.end(), s.begin(), s.end()); }
  void raw(const std::vector<uint8_t>& r) { b.insert(b.end(), r.begin(), r.end()); }
};

// lib0 writeAny for the three value shapes used by the workloads
std::vector<uint8_t> any_int(uint32_t v) {  // 0 <= v < 2^31: tag 125 + varInt
  std::vector<uint8_t> o{125};
  o.push_back((uint8_t)((v > 63 ? 0x80 : 0) | (v & 63)));
  v >>= 6;
  while (v > 0) { o.push_back((uint8_t)((v > 127 ? 0x80 : 0) | (v & 127))); v >>= 7; }
  return o;
}
std::vector<uint8_t> any_str(const std::string& s) {
  W w; w.u8(119); w.vstr(s); return w.b;
}
std::vector<uint8_t> any_obj(const std::vector<std::pair<std::string, std::vector<uint8_t>>>& kv) {
  W w; w.u8(118); w.vu((uint32_t)kv.size());
  for (auto& p : kv) { w.vstr(p.first); w.raw(p.second); }
  return w.b;
}

std::string rand_ascii(Rng& g, uint32_t lo, uint32_t hi) {
  const uint32_t n = lo + g.below(hi - lo + 1);
  std::string s(n, 'a');
  for (auto& c : s) c = (char)('a' + g.below(26));
  return s;
}

struct Cfg {
  uint32_t n_keys;
  uint32_t n_replicas;
  uint32_t ops_per_replica;
  double zipf_s;          // 0 = uniform
  double p_set;           // probability of set (else delete)
  int base_snapshot;      // 1 = one client writes every key first
  uint32_t base_client;
  uint32_t client_mode;   // 0: (r+1)*2654435761 mod 2^32, 1: r+1
  uint32_t value_mode;    // 0: C2 mixed, 1: C1 {name, v}
  uint32_t seed;
  int export_script;
};

struct Ref { uint32_t client, clock; };

struct Item {
  uint32_t key;
  bool deleted;
  bool has_origin;
  Ref origin;
  std::vector<uint8_t> value;
};

std::vector<uint8_t> gen_value(Rng& g, uint32_t mode, uint32_t key, std::string* json) {
  char buf[96];
  if (mode == 1) {
    const uint32_t v = g.below(1u << 20);
    snprintf(buf, sizeof buf, "{\"name\":\"user%u\",\"v\":%u}", key, v);
    if (json) *json = buf;
    return any_obj({{"name", any_str("user" + std::to_string(key))}, {"v", any_int(v)}});
  }
  const double x = g.next();
  if (x < 0.5) {
    const uint32_t v = g.below(1u << 20);
    if (json) { snprintf(buf, sizeof buf, "%u", v); *json = buf; }
    return any_int(v);
  }
  if (x < 0.8) {
    const std::string s = rand_ascii(g, 4, 16);
    if (json) *json = "\"" + s + "\"";
    return any_str(s);
  }
  const std::string s = rand_ascii(g, 4, 16);
  if (json) *json = "{\"name\":\"" + s + "\"}";
  return any_obj({{"name", any_str(s)}});
}

void write_item(W& w, const Item& it, bool merged_deleted, uint32_t run_len, const std::string& root) {
  const uint8_t ref = merged_deleted ? 1 : 8;
  uint8_t info = ref | 0x20;
  if (it.has_origin) info |= 0x80;
  w.u8(info);
  if (it.has_origin) { w.vu(it.origin.client); w.vu(it.origin.clock); }
  else {
    w.vu(1);
    w.vstr(root);
    w.vstr("user" + std::to_string(it.key));
  }
  if (merged_deleted) w.vu(run_len);
  else { w.vu(1); w.raw(it.value); }
}

struct Out {
  std::vector<uint8_t> data;
  std::vector<uint64_t> offs;
  std::string script;
};

void generate(const Cfg& cfg, Out& out) {
  const std::string root = "users";
  const uint32_t K = cfg.n_keys;
  // key sampler
  std::vector<double> cdf;
  if (cfg.zipf_s > 0) {
    cdf.resize(K);
    double acc = 0;
    for (uint32_t k = 0; k < K; ++k) { acc += 1.0 / std::pow((double)(k + 1), cfg.zipf_s); cdf[k] = acc; }
    for (auto& c : cdf) c /= acc;
  }
  auto sample_key = [&](Rng& g) -> uint32_t {
    const double u = g.next();
    if (cfg.zipf_s <= 0) return (uint32_t)(u * K);
    const uint32_t i = (uint32_t)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
    return std::min(i, K - 1);
  };
  auto emit = [&](const std::vector<uint8_t>& u) {
    out.offs.push_back(out.data.size());
    out.data.insert(out.data.end(), u.begin(), u.end());
  };
  std::string& js = out.script;
  const bool S = cfg.export_script != 0;
  if (S) {
    js = "{\"root\":\"users\",\"n_keys\":" + std::to_string(K) + ",\"base_client\":" + std::to_string(cfg.base_client) +
         ",\"base\":[";
  }
  // base snapshot: base client sets every key once (keys in order)
  std::vector<std::vector<uint8_t>> base_vals;
  if (cfg.base_snapshot) {
    Rng g(cfg.seed ^ 0xB5E0000Bu);
    W w;
    w.vu(1);
    w.vu(K);
    w.vu(cfg.base_client);
    w.vu(0);
    base_vals.resize(K);
    for (uint32_t k = 0; k < K; ++k) {
      std::string j;
      base_vals[k] = gen_value(g, cfg.value_mode, k, S ? &j : nullptr);
      if (S) { if (k) js += ","; js += j; }
      Item it{k, false, false, {0, 0}, base_vals[k]};
      write_item(w, it, false, 1, root);
    }
    w.vu(0);  // empty delete set
    emit(w.b);
  }
  if (S) js += "],\"replicas\":[";
  std::vector<Ref> cur(K);
  std::vector<uint8_t> has(K), del(K), base_del(K);
  for (uint32_t r = 0; r < cfg.n_replicas; ++r) {
    const uint32_t client = cfg.client_mode == 0 ? (uint32_t)((uint64_t)(r + 1) * 2654435761ull) : r + 1;
    Rng g(cfg.seed * 0x9E3779B1u + r * 0x85EBCA77u + 1);
    std::fill(base_del.begin(), base_del.end(), 0);
    for (uint32_t k = 0; k < K; ++k) {
      has[k] = cfg.base_snapshot ? 1 : 0;
      cur[k] = Ref{cfg.base_client, k};
      del[k] = 0;
    }
    std::vector<Item> own;
    own.reserve(cfg.ops_per_replica);
    if (S) { if (r) js += ","; js += "{\"client\":" + std::to_string(client) + ",\"ops\":["; }
    for (uint32_t o = 0; o < cfg.ops_per_replica; ++o) {
      const uint32_t k = sample_key(g);
      const bool set = g.next() < cfg.p_set;
      if (S && o) js += ",";
      if (set) {
        std::string j;
        Item it;
        it.key = k;
        it.deleted = false;
        it.has_origin = has[k] != 0;
        it.origin = cur[k];
        it.value = gen_value(g, cfg.value_mode, k, S ? &j : nullptr);
        if (has[k] && !del[k]) {  // the previous entry is overwritten (left.delete)
          if (cur[k].client == client) own[cur[k].clock].deleted = true;
          else base_del[k] = 1;
        }
        cur[k] = Ref{client, (uint32_t)own.size()};
        has[k] = 1;
        del[k] = 0;
        own.push_back(std::move(it));
        if (S) js += "[\"s\"," + std::to_string(k) + "," + j + "]";
      } else {
        if (has[k] && !del[k]) {
          if (cur[k].client == client) own[cur[k].clock].deleted = true;
          else base_del[k] = 1;
          del[k] = 1;
        }
        if (S) js += "[\"d\"," + std::to_string(k) + "]";
      }
    }
    if (S) js += "]}";
    // encodeStateAsUpdate(replica, baseSV): own structs (merged runs) + full delete set
    W w;
    std::vector<std::pair<uint32_t, uint32_t>> own_runs;  // deleted runs (clock,len) over own structs
    if (own.empty()) w.vu(0);
    else {
      // count structs first: consecutive items merge when same key, origin = previous, both deleted
      std::vector<uint32_t> heads;
      for (uint32_t i = 0; i < own.size(); ++i) {
        const bool merge = i > 0 && own[i].deleted && own[i - 1].deleted && own[i].key == own[i - 1].key &&
                           own[i].has_origin && own[i].origin.client == client && own[i].origin.clock == i - 1;
        if (!merge) heads.push_back(i);
      }
      w.vu(1);
      w.vu((uint32_t)heads.size());
      w.vu(client);
      w.vu(0);
      for (size_t h = 0; h < heads.size(); ++h) {
        const uint32_t a = heads[h], b = h + 1 < heads.size() ? heads[h + 1] : (uint32_t)own.size();
        write_item(w, own[a], own[a].deleted, b - a, root);
      }
      for (uint32_t i = 0; i < own.size(); ++i) {
        if (!own[i].deleted) continue;
        uint32_t j = i;
        while (j + 1 < own.size() && own[j + 1].deleted) ++j;
        own_runs.push_back({i, j - i + 1});
        i = j;
      }
    }
    std::vector<std::pair<uint32_t, uint32_t>> base_runs;
    for (uint32_t k = 0; k < K; ++k) {
      if (!base_del[k]) continue;
      uint32_t j = k;
      while (j + 1 < K && base_del[j + 1]) ++j;
      base_runs.push_back({k, j - k + 1});
      k = j;
    }
    // delete set, clients in descending order (Yjs 13.6)
    std::vector<std::pair<uint32_t, std::vector<std::pair<uint32_t, uint32_t>>*>> dsc;
    if (!own_runs.empty()) dsc.push_back({client, &own_runs});
    if (!base_runs.empty()) dsc.push_back({cfg.base_client, &base_runs});
    std::sort(dsc.begin(), dsc.end(), [](auto& x, auto& y) { return x.first > y.first; });
    w.vu((uint32_t)dsc.size());
    for (auto& c : dsc) {
      w.vu(c.first);
      w.vu((uint32_t)c.second->size());
      for (auto& rr : *c.second) { w.vu(rr.first); w.vu(rr.second); }
    }
    emit(w.b);
  }
  if (S) js += "]}";
  out.offs.push_back(out.data.size());
}

}  // namespace

extern "C" {

// Generates a map workload; returns 0. data/offs (n_updates+1 offsets) and script are malloc'ed.
int ycw_gen_map(uint32_t n_keys, uint32_t n_replicas, uint32_t ops_per_replica, double zipf_s, double p_set,
                int base_snapshot, uint32_t base_client, uint32_t client_mode, uint32_t value_mode, uint32_t seed,
                int export_script, uint8_t** data, size_t* data_len, uint64_t** offs, size_t* n_updates, char** script) {
  Cfg cfg{n_keys, n_replicas, ops_per_replica, zipf_s, p_set, base_snapshot, base_client, client_mode, value_mode, seed,
          export_script};
  if (!n_keys) return -1;
  Out out;
  generate(cfg, out);
  *data_len = out.data.size();
  *data = (uint8_t*)malloc(out.data.size() ? out.data.size() : 1);
  if (!out.data.empty()) memcpy(*data, out.data.data(), out.data.size());
  *n_updates = out.offs.size() - 1;
  *offs = (uint64_t*)malloc(sizeof(uint64_t) * out.offs.size());
  memcpy(*offs, out.offs.data(), sizeof(uint64_t) * out.offs.size());
  if (script) {
    *script = (char*)malloc(out.script.size() + 1);
    memcpy(*script, out.script.c_str(), out.script.size() + 1);
  }
  return 0;
}

void ycw_free(void* p) { free(p); }
}
