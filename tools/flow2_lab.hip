// flow2_lab.hip -- measurement harness (diagnostic tool, not product code):
// the PLANES backward (one GPU, 8-bit absolute words, sum_four_to_one 31^6)
// as ONE launch in which waves take 4-plane items by TICKET in level order and
// wait for each item's neighbours by per-plane ready flags, against the
// product's one launch per plane level.  Round 6 successor of flow_lab.hip:
//   * the item body is the PRODUCT's visit (plane_x2_visit, write-through
//     rows in 16-B pieces), so the two sides differ only in the schedule;
//   * items are dealt by tickets, one counter per XCD: each level's items are
//     cut into 8 contiguous chunks (the product's plane_share locality) and
//     XCD x's waves (blockIdx % 8 == x) take chunk x of level 0, then of
//     level 1, ...  Deadlock-free for any grid: a wave only waits for items of
//     lower levels, every taken item is held by a resident wave, and the
//     lowest unfinished item's neighbours are final;
//   * a plane waits for its four k = 1 neighbours only: its k = 2 neighbour
//     along digit j is the k = 1 neighbour of its k = 1 neighbour, final
//     before that one started;
//   * neighbour rows come through PLAIN loads, no acquire: a line is first
//     read only after its plane's flag is set (written through, sc1, drained
//     before the flag), so no L1 / L2 can hold an older copy of it within
//     the launch (the launch's own acquire cleared them).  Checked on a
//     poisoned table, every rep.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/flow2_lab.hip -o tools/flow2_lab
//   ./tools/flow2_lab variant [reps] [blocks_per_cu]
// variants: 0 product launches (k_plane_resolve_x2 per level); 1 ticketed flow
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../gamesmanmpi_amd/csrc/gm_plane.h"
using namespace gm;

#define CK(x)                                                                             \
  do {                                                                                    \
    hipError_t evt = (x);                                                                 \
    if (evt != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(evt)); \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

typedef __attribute__((address_space(1))) uint32_t gu32;
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kSpinLimit = 1u << 20;  // a stuck wave gives up (tmo) after ~0.1-0.5 s

// NSUB: sequences per XCD; SLP: s_sleep between polls (x 64 clocks)
template <int NO, uint32_t NSUB, int SLP>
__global__ __launch_bounds__(256) void k_flow2(uint8_t* __restrict__ tab, const uint32_t* __restrict__ items,
                                               const uint32_t* __restrict__ xoff, uint32_t* __restrict__ ctr,
                                               uint32_t* __restrict__ flags, uint32_t epoch, uint32_t* __restrict__ tmo,
                                               PlaneGeom g, const uint4* __restrict__ zero,
                                               uint64_t* __restrict__ stamp) {
  // sequence q: XCD x = blockIdx % 8, sub-sequence (blockIdx / 8) % NSUB;
  // its counter on a line (and channel) of its own
  const uint32_t lane = threadIdx.x & 63, q = (blockIdx.x & 7u) + 8u * ((blockIdx.x >> 3) % NSUB);
  const uint32_t base = xoff[q], n = xoff[q + 1] - base;
  uint32_t* const c = ctr + 64u * q;
  uint32_t t = 0;
  if (lane == 0) t = atomicAdd(c, 1u);
  t = __builtin_amdgcn_readfirstlane(__shfl(t, 0));
  while (t < n) {
    uint32_t tn = 0;  // the next ticket, in flight during this item
    if (lane == 0) tn = atomicAdd(c, 1u);
    const uint32_t* ip = items + (size_t)(base + t) * 4;
    // wait: lane l < 4 NO polls the k = 1 neighbour along digit l % NO of plane l / NO
    uint32_t nbp = kNone;
    if (lane < 4u * NO) {
      const uint32_t pq = ip[lane / NO], j = lane % NO;
      if (pq != kNone && ((pq >> g.shift[j]) & (g.base[j] - 1u)) >= 1u) nbp = pq - g.stride[j];
    }
    bool ok = nbp == kNone;
    for (uint32_t spins = 0;; spins++) {
      if (!ok) ok = __hip_atomic_load((gu32*)(flags + nbp), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
      if (__all(ok)) break;
      if (spins >= kSpinLimit || __hip_atomic_load((gu32*)tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        if (lane == 0) __hip_atomic_store((gu32*)tmo, 1u + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
      __builtin_amdgcn_s_sleep(SLP);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler order only: the rows load after the polls
    const uint32_t p0 = ip[0];
    PlaneEntry ex, ey;
    ex.p = ip[2 * (lane >> 5)];
    ey.p = ip[2 * (lane >> 5) + 1];
    const bool livex = ex.p != kNone, livey = ey.p != kNone;
    if (!livex) ex.p = p0;
    if (!livey) ey.p = p0;
    plane_x2_visit<1, NO, false, 0, true, true>(tab, g, zero, nullptr, nullptr, ex, ey, livex, livey);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every lane's rows written through before any flag
    if ((lane & 31) < 2) {
      const uint32_t p = (lane & 1) ? ey.p : ex.p;
      const bool live = (lane & 1) ? livey : livex;
      if (live) __hip_atomic_store((gu32*)(flags + p), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (live && stamp) stamp[p] = __builtin_amdgcn_s_memrealtime();  // (var 2: when each plane became final)
    }
    t = __builtin_amdgcn_readfirstlane(__shfl(tn, 0));
  }
}

int main(int argc, char** argv) {
  const int var = argc > 1 ? atoi(argv[1]) : 1;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const int bpc = argc > 3 ? atoi(argv[3]) : 0;
  const uint32_t NSUB = argc > 4 ? (uint32_t)atoi(argv[4]) : 4;
  const int SLP = argc > 5 ? atoi(argv[5]) : 8;
  constexpr int K = 6, NO = K - 2;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  PlaneGeom g{};
  g.no = NO;
  g.pow2 = 1;
  g.world = 1;
  uint64_t np = 1;
  for (int j = 0; j < NO; j++) {
    g.base[j] = 32;
    g.rlim[2 + j] = 31;
    g.stride[j] = (uint32_t)np;
    g.shift[j] = __builtin_ctzll(np);
    np *= 32;
  }
  g.rlim[0] = g.rlim[1] = 31;
  g.nplanes = (uint32_t)np;
  const int S = 31 * NO;
  auto osum = [&](uint64_t P) {
    int s = 0;
    for (int j = 0; j < NO; j++) s += (int)((P >> (5 * j)) & 31);
    return s;
  };
  // level lists in the product's tile order (8^3 tiles over the digits above the lowest)
  std::vector<std::vector<uint32_t>> lev(S + 1);
  for (uint64_t P = 0; P < np; P++) lev[osum(P)].push_back((uint32_t)P);
  auto key = [&](uint32_t P) {
    uint64_t k = 0;
    for (int j = NO - 1; j >= 1; j--) k = k * 64 + ((P >> (5 * j)) & 31) / 8;
    for (int j = NO - 1; j >= 1; j--) k = k * 64 + ((P >> (5 * j)) & 31) % 8;
    return k * 64 + (P & 31);
  };
  for (auto& v : lev) std::sort(v.begin(), v.end(), [&](uint32_t a, uint32_t b) { return key(a) < key(b); });
  // item sequences: level s's groups of 4 cut into 8 contiguous XCD chunks,
  // each dealt round robin over the XCD's NSUB sequences (q = x + 8 sub)
  const uint32_t NQ = 8 * NSUB;
  std::vector<std::vector<uint32_t>> xi(NQ);
  for (int s = 0; s <= S; s++) {
    std::vector<uint32_t> v = lev[s];
    while (v.size() % 4) v.push_back(kNone);
    const size_t ng = v.size() / 4, chunk = (ng + 7) / 8;
    for (int x = 0; x < 8; x++)
      for (size_t gi = x * chunk; gi < std::min(ng, (x + 1) * chunk); gi++)
        for (int c = 0; c < 4; c++) xi[x + 8 * ((gi - x * chunk) % NSUB)].push_back(v[gi * 4 + c]);
  }
  std::vector<uint32_t> items, xoff(NQ + 1, 0);
  for (uint32_t x = 0; x < NQ; x++) {
    xoff[x + 1] = xoff[x] + (uint32_t)(xi[x].size() / 4);
    items.insert(items.end(), xi[x].begin(), xi[x].end());
  }
  std::vector<uint32_t> flat_list, off(S + 2, 0);
  for (int s = 0; s <= S; s++) {
    off[s + 1] = off[s] + (uint32_t)lev[s].size();
    for (uint32_t P : lev[s]) flat_list.push_back(P);
  }
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_flow2<NO, 4, 8>, 256, 0));
  const int per_cu = bpc > 0 ? bpc : occ;
  const uint32_t blocks = (uint32_t)(cus * per_cu);
  const size_t tbytes = np * 1024;
  uint8_t* tab;
  void* zero;
  uint32_t *dlist, *ditems, *dxoff, *flags, *ctr, *tmo;
  CK(hipMalloc(&tab, tbytes));
  CK(hipMalloc(&zero, 4096));
  CK(hipMemset(zero, 0, 4096));
  CK(hipMalloc(&dlist, flat_list.size() * 4));
  CK(hipMemcpy(dlist, flat_list.data(), flat_list.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&ditems, items.size() * 4));
  CK(hipMemcpy(ditems, items.data(), items.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&dxoff, (NQ + 1) * 4));
  CK(hipMemcpy(dxoff, xoff.data(), (NQ + 1) * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&flags, np * 4 + 64 * 4 * (NQ + 1)));
  ctr = flags + np;
  tmo = ctr + 64 * NQ;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  uint64_t* dstamp = nullptr;
  CK(hipMalloc(&dstamp, np * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run_levels = [&]() {
    for (int s = 0; s <= S; s++) {
      const uint32_t n = off[s + 1] - off[s];
      const uint32_t waves = (n + 3) / 4;
      uint32_t b = (waves + 3) / 4;
      b = std::min<uint32_t>((b + 7) / 8 * 8, (uint32_t)cus * 32);
      hipLaunchKernelGGL((k_plane_resolve_x2<1, NO, false, 0>), dim3(b), dim3(256), 0, st, tab,
                         (const void*)(dlist + off[s]), n, g, (const uint4*)zero, (const uint8_t*)nullptr,
                         (uint8_t*)nullptr, (const uint32_t*)nullptr, 0u);
    }
  };
  uint32_t epoch = 0;
  auto run_flow = [&]() {
    epoch++;
    CK(hipMemsetAsync(ctr, 0, 64 * 4 * NQ, st));
    auto go = [&](auto ns, auto sl) {
      hipLaunchKernelGGL((k_flow2<NO, decltype(ns)::value, decltype(sl)::value>), dim3(blocks), dim3(256), 0, st, tab,
                         (const uint32_t*)ditems, (const uint32_t*)dxoff, ctr, flags, epoch, tmo, g,
                         (const uint4*)zero, var == 2 ? dstamp : (uint64_t*)nullptr);
    };
    auto sel = [&](auto ns) {
      switch (SLP) {
        case 1: go(ns, std::integral_constant<int, 1>()); break;
        case 2: go(ns, std::integral_constant<int, 2>()); break;
        case 4: go(ns, std::integral_constant<int, 4>()); break;
        case 16: go(ns, std::integral_constant<int, 16>()); break;
        default: go(ns, std::integral_constant<int, 8>()); break;
      }
    };
    switch (NSUB) {
      case 1: sel(std::integral_constant<uint32_t, 1>()); break;
      case 2: sel(std::integral_constant<uint32_t, 2>()); break;
      case 8: sel(std::integral_constant<uint32_t, 8>()); break;
      case 16: sel(std::integral_constant<uint32_t, 16>()); break;
      default: sel(std::integral_constant<uint32_t, 4>()); break;
    }
  };
  printf("flow2_lab var %d: %llu planes, %d levels, %u items, grid %u blocks (%d per CU, occupancy API %d), %u sequences per XCD, sleep %d\n", var,
         (unsigned long long)np, S + 1, xoff[NQ], blocks, per_cu, occ, NSUB, SLP);
  fflush(stdout);
  CK(hipMemset(flags, 0, np * 4 + 64 * 4 * (NQ + 1)));
  run_levels();
  CK(hipStreamSynchronize(st));
  std::vector<uint8_t> ref(tbytes), got(tbytes);
  CK(hipMemcpy(ref.data(), tab, tbytes, hipMemcpyDeviceToHost));
  std::vector<float> ts;
  for (int r = 0; r <= reps; r++) {  // r = 0: warm-up
    CK(hipMemsetAsync(tab, 0xAA, tbytes, st));  // poison: a stale read shows
    CK(hipEventRecord(e0, st));
    if (var == 0) run_levels();
    else run_flow();
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r) ts.push_back(ms);
    uint32_t tm = 0;
    CK(hipMemcpy(&tm, tmo, 4, hipMemcpyDeviceToHost));
    if (tm) {
      printf("GAVE UP: a wave timed out waiting (ticket %u)\n", tm - 1);
      return 3;
    }
    CK(hipMemcpy(got.data(), tab, tbytes, hipMemcpyDeviceToHost));
    size_t bad = 0, first = 0;
    for (size_t i = 0; i < tbytes; i++)
      if (got[i] != ref[i]) {
        if (!bad) first = i;
        bad++;
      }
    if (bad) {
      printf("rep %d: %zu differing bytes, first at %zu (plane %zu): got %02x want %02x MISMATCH\n", r, bad, first,
             first / 1024, got[first], ref[first]);
      return 2;
    }
  }
  if (var == 2) {  // per plane level: when its first / last plane became final (100 MHz ticks from the first)
    std::vector<uint64_t> h(np);
    CK(hipMemcpy(h.data(), dstamp, np * 8, hipMemcpyDeviceToHost));
    uint64_t t0 = ~0ull;
    for (uint64_t P = 0; P < np; P++) t0 = std::min(t0, h[P]);
    printf("level first_us last_us planes\n");
    for (int s = 0; s <= S; s++) {
      uint64_t a = ~0ull, b = 0;
      for (uint32_t P : lev[s]) a = std::min(a, h[P]), b = std::max(b, h[P]);
      printf("%d %.2f %.2f %zu\n", s, (a - t0) / 100.0, (b - t0) / 100.0, lev[s].size());
    }
  }
  float best = 1e9, sum = 0;
  for (float t : ts) {
    best = std::min(best, t);
    sum += t;
  }
  printf("var %d backward best %.4f ms mean %.4f ms (%d reps, every rep byte-exact vs the product's per-level launches)\n",
         var, best, sum / reps, reps);
  return 0;
}
