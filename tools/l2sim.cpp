// l2sim.cpp -- CPU model of the per-XCD L2 reuse of the PLANES backward's
// neighbour-row reads (diagnostic tool, not product code).
//
// Per plane level (one launch), the level's list is dealt to the 8 XCDs as
// plane_share does (one contiguous chunk each); an XCD's waves take its
// chunk's planes in list order, `window` planes resident at a time.  Every
// plane reads its 8 neighbour planes (1 KiB each); the model keeps, per XCD,
// an LRU of `cap` planes (4 MiB = 4096 planes) that starts EMPTY at every
// launch (a kernel boundary), and counts neighbour-plane reads that miss.
//
//   g++ -O2 -std=c++17 tools/l2sim.cpp -o /tmp/l2sim && /tmp/l2sim order [cap]
// order: 0 plane index; 8 the product's 8^3 tiles; t (>1) t^3 tiles;
//        -1 Morton over the three upper digits; -2 tiles dealt round robin to XCDs
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <list>
#include <unordered_map>
#include <vector>

struct LRU {
  size_t cap;
  std::list<uint32_t> l;
  std::unordered_map<uint32_t, std::list<uint32_t>::iterator> m;
  bool touch(uint32_t k) {
    auto it = m.find(k);
    if (it != m.end()) {
      l.splice(l.begin(), l, it->second);
      return true;
    }
    l.push_front(k);
    m[k] = l.begin();
    if (l.size() > cap) {
      m.erase(l.back());
      l.pop_back();
    }
    return false;
  }
  void clear() {
    l.clear();
    m.clear();
  }
};

int main(int argc, char** argv) {
  const int order = argc > 1 ? atoi(argv[1]) : 8;
  const size_t cap = argc > 2 ? (size_t)atoi(argv[2]) : 4096;
  const int NO = 4, S = 124;
  const uint32_t np = 1u << 20;
  auto dig = [](uint32_t P, int j) { return (P >> (5 * j)) & 31u; };
  std::vector<std::vector<uint32_t>> lev(S + 1);
  for (uint32_t P = 0; P < np; P++) {
    int s = 0;
    for (int j = 0; j < NO; j++) s += dig(P, j);
    lev[s].push_back(P);
  }
  auto key = [&](uint32_t P) -> uint64_t {
    uint32_t d[4];
    for (int j = 0; j < 4; j++) d[j] = dig(P, j);
    uint64_t k = 0;
    if (order == -1) {
      for (int b = 4; b >= 0; b--)
        for (int j = 3; j >= 1; j--) k = k * 2 + ((d[j] >> b) & 1);
      return k * 64 + d[0];
    }
    const int t = order > 1 ? order : (order == -2 ? 8 : 32);
    for (int j = 3; j >= 1; j--) k = k * 64 + d[j] / t;
    for (int j = 3; j >= 1; j--) k = k * 64 + d[j] % t;
    return k * 64 + d[0];
  };
  if (order != 0)
    for (auto& L : lev) std::sort(L.begin(), L.end(), [&](uint32_t a, uint32_t b) { return key(a) < key(b); });
  uint64_t reads = 0, miss = 0, wide_reads = 0, wide_miss = 0;
  std::vector<LRU> l2(8);
  for (auto& c : l2) c.cap = cap;
  for (int s = 0; s <= S; s++) {
    const auto& L = lev[s];
    const size_t n = L.size();
    for (auto& c : l2) c.clear();
    std::vector<std::vector<uint32_t>> part(8);
    if (order == -2) {  // whole 8^3 tiles round robin over the XCDs
      uint64_t prev = ~0ull;
      int x = -1;
      for (uint32_t P : L) {
        const uint64_t tk = key(P) >> (6 * 3 + 6);
        if (tk != prev) x = (x + 1) % 8, prev = tk;
        part[x].push_back(P);
      }
    } else {
      const size_t chunk = ((n + 7) / 8 + 3) / 4 * 4;
      for (size_t i = 0; i < n; i++) part[std::min<size_t>(i / std::max<size_t>(chunk, 1), 7)].push_back(L[i]);
    }
    for (int x = 0; x < 8; x++)
      for (uint32_t P : part[x])
        for (int j = 0; j < NO; j++)
          for (uint32_t k = 1; k <= 2; k++) {
            if (dig(P, j) < k) continue;
            const uint32_t Q = P - (k << (5 * j));
            reads++;
            const bool hit = l2[x].touch(Q);
            miss += !hit;
            if (n > 8192) wide_reads++, wide_miss += !hit;
          }
  }
  printf("order %d cap %zu: %llu neighbour-plane reads, hit rate %.3f (levels > 8192 planes: %.3f), "
         "misses per plane %.3f (compulsory ~2)\n",
         order, cap, (unsigned long long)reads, 1.0 - (double)miss / reads, 1.0 - (double)wide_miss / wide_reads,
         (double)miss / np);
  return 0;
}
