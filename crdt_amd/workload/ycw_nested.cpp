// ycw_nested.cpp — seeded C4-shaped workloads: a root YMap 'docs' whose keys
// hold nested YArrays, replicas appending to them concurrently, overwriting keys with fresh arrays
// (the old array and everything in it becomes garbage: nested-type GC) and deleting elements.
//
// A base client first writes every key (ContentType YArray, parent 'docs', parentSub "d<k>") and an
// initial run of elements into each array (explicit parent = the type item's id). Then every replica
// works from the base (no gossip: maximal concurrency) with Yjs's local-op semantics:
//   * push m values onto array k: origin = the last element of k in the replica's view, no right
//     origin (typeListPushGenerics → insert at the end); an empty array takes the type item as its
//     explicit parent (Item.write: parent info 0 + the item id);
//   * overwrite key k (p_over): a new ContentType item whose origin is k's current entry item (the
//     map's typeMapSet); pushes then go into the replica's own new array;
//   * delete (p_del): one base element of k's base array (a delete-set range).
// Each replica's update is its structs in clock order (one struct per push; Yjs would have merged
// consecutive pushes in its store — unmerged structs are equally valid input and merge to the same
// state) plus its delete set. Benchmark / test input generation only, not part of the merge path.
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
};

void any_value(W& w, Rng& g) {  // lib0 writeAny: small ints and short strings
  if (g.below(2)) {
    const uint32_t v = g.below(64);
    w.u8(125);
    w.u8((uint8_t)v);
  } else {
    w.u8(119);
    w.vstr("v" + std::to_string(g.below(1000)));
  }
}

struct Id { uint32_t client, clock; };
constexpr uint8_t REF_ANY = 8, REF_TYPE = 7;

struct Cfg {
  uint32_t n_replicas, n_keys, pushes, init_len;
  double p_over, p_del;
  uint32_t seed;
};

// an ANY struct of m values: origin or explicit parent item
void put_elems(W& w, Rng& g, bool has_origin, Id origin, Id parent, uint32_t m) {
  w.u8((uint8_t)(REF_ANY | (has_origin ? 0x80 : 0)));
  if (has_origin) { w.vu(origin.client); w.vu(origin.clock); }
  else { w.u8(0); w.vu(parent.client); w.vu(parent.clock); }
  w.vu(m);
  for (uint32_t i = 0; i < m; ++i) any_value(w, g);
}

}  // namespace

extern "C" {

// data / offs (n_updates + 1 offsets) malloc'ed; stats[0] = items, [1] = structs, [2] = deletes
int ycw_gen_nested(uint32_t n_replicas, uint32_t n_keys, uint32_t pushes, uint32_t init_len, double p_over, double p_del,
                   uint32_t seed, uint8_t** data, size_t* data_len, uint64_t** offs, size_t* n_updates, uint64_t* stats) {
  if (!n_keys || !init_len) return -1;
  Cfg cfg{n_replicas, n_keys, pushes, init_len, p_over, p_del, seed};
  Rng g(seed);
  std::vector<uint8_t> all;
  std::vector<uint64_t> off{0};
  uint64_t items = 0, structs = 0, dels = 0;
  const uint32_t B = 1;  // base client
  // ---- base: every key's type item (clock k), then its initial elements (one struct each)
  {
    W w;
    w.vu(1);
    w.vu(2 * cfg.n_keys);
    w.vu(B);
    w.vu(0);
    for (uint32_t k = 0; k < cfg.n_keys; ++k) {
      w.u8((uint8_t)(REF_TYPE | 0x20));  // parentSub, no origin: parent = root name
      w.u8(1);
      w.vstr("docs");
      w.vstr("d" + std::to_string(k));
      w.vu(0);  // typeRef YArray
    }
    for (uint32_t k = 0; k < cfg.n_keys; ++k) put_elems(w, g, false, Id{0, 0}, Id{B, k}, cfg.init_len);
    w.vu(0);  // empty delete set
    all.insert(all.end(), w.b.begin(), w.b.end());
    off.push_back(all.size());
    items += 2ull * cfg.n_keys + (uint64_t)cfg.n_keys * (cfg.init_len - 1);
    structs += 2ull * cfg.n_keys;
  }
  auto base_elem0 = [&](uint32_t k) { return cfg.n_keys + k * cfg.init_len; };  // first clock of k's base elements
  // ---- replicas
  std::vector<Id> entry(cfg.n_keys), last(cfg.n_keys), type(cfg.n_keys);
  std::vector<uint8_t> has_last(cfg.n_keys), own(cfg.n_keys);
  for (uint32_t r = 0; r < cfg.n_replicas; ++r) {
    const uint32_t client = 1000u + 7919u * r;  // distinct, above the base client
    for (uint32_t k = 0; k < cfg.n_keys; ++k) {
      entry[k] = Id{B, k};
      type[k] = Id{B, k};
      last[k] = Id{B, base_elem0(k) + cfg.init_len - 1};
      has_last[k] = 1;
      own[k] = 0;
    }
    W body;
    uint32_t clock = 0, nst = 0;
    std::vector<std::pair<uint32_t, uint32_t>> ds;  // base clocks deleted
    for (uint32_t i = 0; i < cfg.pushes; ++i) {
      // skewed key choice: half the ops on the first 1 % of the keys
      const uint32_t hot = std::max(1u, cfg.n_keys / 100);
      const uint32_t k = g.below(2) ? g.below(hot) : g.below(cfg.n_keys);
      const double x = g.next();
      if (x < cfg.p_over) {  // overwrite the key with a new array
        body.u8((uint8_t)(REF_TYPE | 0x80 | 0x20));
        body.vu(entry[k].client);
        body.vu(entry[k].clock);
        body.vu(0);
        entry[k] = type[k] = Id{client, clock};
        has_last[k] = 0;
        own[k] = 1;
        ++clock;
        ++nst;
        ++items;
      } else if (x < cfg.p_over + cfg.p_del) {
        if (!own[k]) {  // delete one base element of k (a range of the base client)
          ds.push_back({base_elem0(k) + g.below(cfg.init_len), 1});
          ++dels;
        }
      } else {
        const uint32_t m = 1 + g.below(4);
        put_elems(body, g, has_last[k] != 0, last[k], type[k], m);
        last[k] = Id{client, clock + m - 1};
        has_last[k] = 1;
        clock += m;
        ++nst;
        items += m;
      }
    }
    W w;
    w.vu(nst ? 1 : 0);
    if (nst) {
      w.vu(nst);
      w.vu(client);
      w.vu(0);
      w.b.insert(w.b.end(), body.b.begin(), body.b.end());
    }
    std::sort(ds.begin(), ds.end());
    std::vector<std::pair<uint32_t, uint32_t>> m;
    for (auto& d : ds) {
      if (!m.empty() && m.back().first + m.back().second >= d.first) {
        m.back().second = std::max(m.back().first + m.back().second, d.first + d.second) - m.back().first;
      } else {
        m.push_back(d);
      }
    }
    if (m.empty()) {
      w.vu(0);
    } else {
      w.vu(1);
      w.vu(B);
      w.vu((uint32_t)m.size());
      for (auto& d : m) { w.vu(d.first); w.vu(d.second); }
    }
    all.insert(all.end(), w.b.begin(), w.b.end());
    off.push_back(all.size());
    structs += nst;
  }
  *data_len = all.size();
  *data = (uint8_t*)malloc(all.size() ? all.size() : 1);
  if (!all.empty()) memcpy(*data, all.data(), all.size());
  *n_updates = off.size() - 1;
  *offs = (uint64_t*)malloc(sizeof(uint64_t) * off.size());
  memcpy(*offs, off.data(), sizeof(uint64_t) * off.size());
  stats[0] = items;
  stats[1] = structs;
  stats[2] = dels;
  return 0;
}

}  // extern "C"
