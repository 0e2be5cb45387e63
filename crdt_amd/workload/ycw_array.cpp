// ycw_array.cpp — seeded synthetic YArray replica workload at scale (BASELINE.json config C3).
//
// 256 replicas edit YArray 'messages' with the C3 op mix (push 40 % / unshift 15 % / insert at a
// random position 30 %, 1-4 values each / cut of 1-3 values 15 %) over `rounds` rounds. Within a
// round every replica works on its own view: the merged list of the previous round plus its own
// new items; at the end of a round all replicas exchange everything. The wire output is every
// replica's per-round update (its new items, one struct per op, plus the delete-set ranges of its
// cuts) — the messages crdt.js broadcasts.
//
// Replica views need the exact Yjs list order of the previous round. It is kept as the origin tree
// with children ordered by the backward-evaluated B.1 sibling rule (the formulation checked against
// the sequential loop in scripts/yata_tree_proto.py, re-implemented here independently of the HIP
// kernels), linearised once per round. Every generated item therefore names an origin and right
// origin that are adjacent in its creator's view, as a real Yjs replica would.
//
// This is benchmark/test input generation, not part of the merge path.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

constexpr uint32_t NIL = 0xFFFFFFFFu;

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

struct Unit {
  uint32_t client;   // client id (value)
  uint32_t clock;
  uint32_t right;    // right origin unit (NIL = none)
  uint32_t parent;   // origin unit (NIL = the list start)
  uint8_t deleted;
};

struct Item {        // one op's struct
  uint32_t first;    // first unit
  uint32_t n;
  uint32_t origin, right;
  std::string vals;  // lib0 `any` values, concatenated
};

struct Tree {
  // per node (unit index; ROOT = the list start): ordered children, right-origin member lists
  std::vector<uint32_t> first, last, nxt, prv, mprv, mtail;
  std::unordered_map<uint64_t, uint32_t> otail;  // (parent, outside right origin) -> last member
  uint32_t root;
  void grow(size_t n) {
    for (auto* v : {&first, &last, &nxt, &prv, &mprv, &mtail}) v->resize(n, NIL);
  }
};

// Inserts unit c into its origin's children (Item.integrate restricted to the siblings, evaluated
// backwards: see yc_yata.hip sib_loop). Its right origin, if a sibling, is already placed.
void tree_insert(Tree& T, const std::vector<Unit>& U, uint32_t c) {
  const uint32_t p = U[c].parent == NIL ? T.root : U[c].parent;
  const uint32_t r = U[c].right;
  const uint32_t cc = U[c].client;
  const bool sib = r != NIL && (U[r].parent == NIL ? T.root : U[r].parent) == p;  // unit 0 is the root
  uint32_t* tail;
  if (sib) tail = &T.mtail[r];
  else tail = &T.otail.emplace(((uint64_t)p << 32) | r, NIL).first->second;
  uint32_t m = *tail, succ = NIL;
  while (m != NIL && U[m].client > cc) { succ = m; m = T.mprv[m]; }
  T.mprv[c] = m;
  if (succ != NIL) T.mprv[succ] = c;
  else *tail = c;
  const uint32_t stop = succ != NIL ? succ : (sib ? r : NIL);
  uint32_t left = stop != NIL ? T.prv[stop] : T.last[p];
  while (left != NIL && U[left].client >= cc) left = T.prv[left];
  const uint32_t nx = left != NIL ? T.nxt[left] : T.first[p];
  T.prv[c] = left;
  T.nxt[c] = nx;
  if (left != NIL) T.nxt[left] = c; else T.first[p] = c;
  if (nx != NIL) T.prv[nx] = c; else T.last[p] = c;
}

// pre-order of the origin tree = the list order
void linearize(const Tree& T, std::vector<uint32_t>& out) {
  out.clear();
  std::vector<uint32_t> stack;
  uint32_t x = T.first[T.root];
  while (x != NIL) {
    out.push_back(x);
    if (T.first[x] != NIL) {
      stack.push_back(x);
      x = T.first[x];
      continue;
    }
    while (x != NIL && T.nxt[x] == NIL) {
      if (stack.empty()) { x = NIL; break; }
      x = stack.back();
      stack.pop_back();
    }
    if (x != NIL) x = T.nxt[x];
  }
}

void any_value(Rng& g, uint32_t r, uint32_t seq, uint32_t i, std::string& o) {
  if (g.next() < 0.6) {
    const std::string s = "m" + std::to_string(r) + "_" + std::to_string(seq) + "_" + std::to_string(i);
    o.push_back((char)119);
    o.push_back((char)s.size());
    o += s;
  } else {  // 0 <= v < 2^20: tag 125 + varInt
    uint32_t v = g.below(1u << 20);
    o.push_back((char)125);
    o.push_back((char)((v > 63 ? 0x80 : 0) | (v & 63)));
    v >>= 6;
    while (v > 0) { o.push_back((char)((v > 127 ? 0x80 : 0) | (v & 127))); v >>= 7; }
  }
}

struct View {  // one replica's view in a round: the base list plus its own new units in the gaps
  std::unordered_map<int64_t, std::vector<uint32_t>> gap;  // after base position i (-1: before the first)
  std::unordered_map<uint32_t, std::pair<int64_t, uint32_t>> where;  // own unit -> (gap, index)
  std::vector<uint32_t> own;
};

}  // namespace

extern "C" {

// C3-shaped YArray workload: n_replicas x rounds, about items_target values in total.
// data/offs (n_updates+1 offsets) are malloc'ed; stats[4] = {ops, items, deleted items, list length}.
// order (optional): the final list's live values as (client, clock) pairs, malloc'ed (test check).
int ycw_gen_array(uint32_t n_replicas, uint32_t rounds, uint64_t items_target, uint32_t seed, uint8_t** data,
                  size_t* data_len, uint64_t** offs, size_t* n_updates, uint64_t* stats, uint32_t** order_out,
                  size_t* norder) {
  if (!n_replicas || !rounds) return -1;
  Rng g(seed);
  std::vector<uint32_t> client(n_replicas), nclock(n_replicas, 0);
  for (uint32_t r = 0; r < n_replicas; ++r) client[r] = (uint32_t)(((uint64_t)(r + 1) * 2654435761ull) & 0xFFFFFFFFull) ?: 1u;
  // ops per replica per round from the target: ~1.9 values per op (push / insert 1-4, unshift 1)
  const uint64_t ops_total = items_target / 19 * 10 + 1;
  const uint32_t ops = (uint32_t)std::max<uint64_t>(1, ops_total / ((uint64_t)n_replicas * rounds));
  std::vector<Unit> U;
  U.reserve(items_target + items_target / 4 + 16);
  U.push_back(Unit{0, 0, NIL, NIL, 1});  // unit 0: the list start (root of the origin tree)
  Tree T;
  T.root = 0;
  std::vector<int64_t> bpos;             // unit -> position in `base`
  std::vector<uint32_t> base;  // the merged list of the previous round
  std::vector<uint8_t> outb;
  std::vector<uint64_t> off{0};
  std::vector<uint32_t> order(n_replicas);
  for (uint32_t r = 0; r < n_replicas; ++r) order[r] = r;
  std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return client[a] < client[b]; });
  uint64_t nops = 0, nitems = 0, ndel = 0, seq = 0;
  for (uint32_t round = 0; round < rounds; ++round) {
    const int64_t N = (int64_t)base.size();
    std::vector<std::vector<Item>> items(n_replicas);
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> dels(n_replicas);  // (client, clock)
    for (uint32_t r = 0; r < n_replicas; ++r) {
      View v;
      // next unit after a view position
      auto succ_of = [&](int64_t gi, uint32_t j) -> uint32_t {  // j = index in gap gi, or NIL: the base unit gi itself
        auto it = v.gap.find(gi);
        const uint32_t k = j == NIL ? 0 : j + 1;
        if (it != v.gap.end() && k < it->second.size()) return it->second[k];
        return gi + 1 < N ? base[gi + 1] : NIL;
      };
      auto locate = [&](uint32_t u, int64_t& gi, uint32_t& j) {  // view position of a unit
        auto it = v.where.find(u);
        if (it != v.where.end()) { gi = it->second.first; j = it->second.second; }
        else { gi = -2; j = NIL; }
      };
      auto base_index = [&](uint32_t u) -> int64_t { return u < bpos.size() ? bpos[u] : -1; };
      auto random_live = [&](uint32_t& u) -> bool {  // a live unit of the view, uniformly
        const uint64_t tot = (uint64_t)N + v.own.size();
        if (!tot) return false;
        for (int t = 0; t < 64; ++t) {
          const uint64_t i = (uint64_t)(g.next() * (double)tot);
          u = i < (uint64_t)N ? base[i] : v.own[i - N];
          if (!U[u].deleted) return true;
        }
        return false;
      };
      auto next_in_view = [&](uint32_t u) -> uint32_t {
        int64_t gi; uint32_t j;
        locate(u, gi, j);
        if (gi == -2) return succ_of(base_index(u), NIL);
        return succ_of(gi, j);
      };
      auto insert_after = [&](uint32_t o, const std::vector<uint32_t>& units) {  // o = NIL: the front
        int64_t gi; uint32_t j, k;
        if (o == NIL) { gi = -1; k = 0; }
        else {
          locate(o, gi, j);
          if (gi == -2) { gi = base_index(o); k = 0; } else k = j + 1;
        }
        auto& lst = v.gap[gi];
        lst.insert(lst.begin() + k, units.begin(), units.end());
        for (uint32_t x = k; x < lst.size(); ++x) v.where[lst[x]] = {gi, x};
        v.own.insert(v.own.end(), units.begin(), units.end());
      };
      auto last_live = [&]() -> uint32_t {  // walk the view backwards from its end
        for (int64_t gi = N - 1; gi >= -1; --gi) {
          auto it = v.gap.find(gi);
          if (it != v.gap.end())
            for (size_t k = it->second.size(); k-- > 0;)
              if (!U[it->second[k]].deleted) return it->second[k];
          if (gi >= 0 && !U[base[gi]].deleted) return base[gi];
        }
        return NIL;
      };
      for (uint32_t o = 0; o < ops; ++o, ++nops) {
        const double x = g.next();
        uint32_t n = 1 + g.below(4), origin = NIL, right = NIL;
        const bool empty = N == 0 && v.own.empty();
        if (x < 0.85 || empty) {
          if (x < 0.40 || empty) {                    // push: after the last live value
            origin = last_live();
            if (origin != NIL) right = next_in_view(origin);
            else { auto it = v.gap.find(-1); right = it != v.gap.end() && !it->second.empty() ? it->second[0] : (N ? base[0] : NIL); }
          } else if (x < 0.55) {                      // unshift: before the first item
            n = 1;
            auto it = v.gap.find(-1);
            right = it != v.gap.end() && !it->second.empty() ? it->second[0] : (N ? base[0] : NIL);
          } else {                                    // insert after a random live value
            uint32_t u;
            if (random_live(u)) { origin = u; right = next_in_view(u); }
            else { auto it = v.gap.find(-1); right = it != v.gap.end() && !it->second.empty() ? it->second[0] : (N ? base[0] : NIL); }
          }
          Item it{(uint32_t)U.size(), n, origin, right, {}};
          std::vector<uint32_t> units;
          for (uint32_t i = 0; i < n; ++i) {
            U.push_back(Unit{client[r], nclock[r]++, right, i == 0 ? origin : (uint32_t)U.size() - 1, 0});
            units.push_back((uint32_t)U.size() - 1);
            any_value(g, r, (uint32_t)seq, i, it.vals);
          }
          ++seq;
          nitems += n;
          insert_after(origin, units);
          items[r].push_back(std::move(it));
        } else {                                      // cut: 1-3 live values from a random one
          uint32_t u;
          if (!random_live(u)) continue;
          const uint32_t k = 1 + g.below(3);
          for (uint32_t d = 0; d < k && u != NIL;) {
            if (!U[u].deleted) {
              U[u].deleted = 1;
              dels[r].push_back({U[u].client, U[u].clock});
              ++ndel;
              ++d;
            }
            u = next_in_view(u);
          }
        }
      }
    }
    // the round's wire updates
    for (uint32_t r = 0; r < n_replicas; ++r) {
      W w;
      if (items[r].empty()) w.vu(0);
      else {
        w.vu(1);
        w.vu((uint32_t)items[r].size());
        w.vu(client[r]);
        w.vu(U[items[r][0].first].clock);
        for (const Item& it : items[r]) {
          const uint8_t info = 8 | (it.origin != NIL ? 0x80 : 0) | (it.right != NIL ? 0x40 : 0);
          w.u8(info);
          if (it.origin != NIL) { w.vu(U[it.origin].client); w.vu(U[it.origin].clock); }
          if (it.right != NIL) { w.vu(U[it.right].client); w.vu(U[it.right].clock); }
          if (it.origin == NIL && it.right == NIL) { w.vu(1); w.vstr("messages"); }
          w.vu(it.n);
          w.b.insert(w.b.end(), it.vals.begin(), it.vals.end());
        }
      }
      auto& ds = dels[r];
      std::sort(ds.begin(), ds.end());
      std::vector<std::pair<uint32_t, std::vector<std::pair<uint32_t, uint32_t>>>> groups;
      for (const auto& d : ds) {
        if (groups.empty() || groups.back().first != d.first) groups.push_back({d.first, {}});
        auto& rg = groups.back().second;
        if (!rg.empty() && rg.back().first + rg.back().second == d.second) ++rg.back().second;
        else rg.push_back({d.second, 1});
      }
      std::sort(groups.begin(), groups.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
      w.vu((uint32_t)groups.size());
      for (const auto& gr : groups) {
        w.vu(gr.first);
        w.vu((uint32_t)gr.second.size());
        for (const auto& rg : gr.second) { w.vu(rg.first); w.vu(rg.second); }
      }
      outb.insert(outb.end(), w.b.begin(), w.b.end());
      off.push_back(outb.size());
    }
    // everyone receives everything: integrate the round into the tree (causal: per replica in
    // creation order, replicas by ascending client) and linearise the merged list
    T.grow(U.size());
    for (const uint32_t r : order)
      for (const Item& it : items[r])
        for (uint32_t i = 0; i < it.n; ++i) tree_insert(T, U, it.first + i);
    linearize(T, base);
    bpos.assign(U.size(), -1);
    for (size_t i = 0; i < base.size(); ++i) bpos[base[i]] = (int64_t)i;
  }
  *data_len = outb.size();
  *data = (uint8_t*)malloc(outb.size() ? outb.size() : 1);
  if (!outb.empty()) memcpy(*data, outb.data(), outb.size());
  *n_updates = off.size() - 1;
  *offs = (uint64_t*)malloc(sizeof(uint64_t) * off.size());
  memcpy(*offs, off.data(), sizeof(uint64_t) * off.size());
  if (stats) { stats[0] = nops; stats[1] = nitems; stats[2] = ndel; stats[3] = base.size(); }
  if (order_out && norder) {
    std::vector<uint32_t> o;
    for (const uint32_t u : base)
      if (!U[u].deleted) { o.push_back(U[u].client); o.push_back(U[u].clock); }
    *norder = o.size() / 2;
    *order_out = (uint32_t*)malloc(sizeof(uint32_t) * (o.size() + 1));
    if (!o.empty()) memcpy(*order_out, o.data(), sizeof(uint32_t) * o.size());
  }
  return 0;
}

}  // extern "C"
