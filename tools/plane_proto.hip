// Standalone harness for the PLANES backward kernel (gm_plane.h): builds the
// per-level plane lists, runs the backward pass of a sum_four_to_one shape
// heaps = 31 x K (optionally a different top heap), times it with HIP events
// and checks every word against a CPU retrograde for small shapes (rank
// order is a topological order: every move lowers the rank) and the root
// line for the bench shape.  Diagnostic tool, not product code.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/plane_proto.hip -o tools/plane_proto
//   ./tools/plane_proto K [top] [wb] [reps]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "plane_variants.h"
using namespace gm;

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

static int g_x2 = 1;
template <int WB, int NO>
static void launch(void* tab, const uint32_t* list, uint32_t n, const PlaneGeom& g, const uint4* zero,
                   hipStream_t st) {
  typedef typename PlaneWord<WB>::T T;
  const uint32_t waves = g_x2 ? (n + 3) / 4 : (n + 1) / 2;
  uint32_t blocks = (waves + 3) / 4;
  blocks = (blocks + 7) / 8 * 8;
  if (g_x2 == 10 && WB == 1)
    hipLaunchKernelGGL((k_plane_resolve_x2d<1, NO, false>), dim3(blocks), dim3(256), 0, st, (uint8_t*)tab, list, n, g,
                       zero, (const uint8_t*)nullptr, (uint8_t*)nullptr);
  else if (g_x2 == 9 && WB == 1)
    hipLaunchKernelGGL((k_plane_resolve_x2c<1, NO, false>), dim3(blocks), dim3(256), 0, st, (uint8_t*)tab, list, n, g,
                       zero, (const uint8_t*)nullptr, (uint8_t*)nullptr);
  else if (g_x2 == 8 && WB == 1)
    hipLaunchKernelGGL((k_plane_resolve_x2w<1, NO, false>), dim3(blocks), dim3(256), 0, st, (uint8_t*)tab, list, n, g,
                       zero, (const uint8_t*)nullptr, (uint8_t*)nullptr);
  else if (g_x2 == 7 && WB == 1)
    hipLaunchKernelGGL((k_plane_resolve_x2b<1, NO, false>), dim3(blocks), dim3(256), 0, st, (uint8_t*)tab, list, n, g,
                       zero, (const uint8_t*)nullptr, (uint8_t*)nullptr);
  else if (g_x2 == 6 && WB == 1)
    hipLaunchKernelGGL((k_plane_resolve_x2f<NO, false>), dim3(blocks), dim3(256), 0, st, (uint8_t*)tab, list, n, g,
                       zero, (const uint8_t*)nullptr, (uint8_t*)nullptr);
  else if (g_x2 == 4 && WB == 1)  // diagnostic: no neighbour loads
    hipLaunchKernelGGL((k_plane_resolve_x2h<NO, false, 1>), dim3(blocks), dim3(256), 0, st, (uint8_t*)tab, list, n, g,
                       zero, (const uint8_t*)nullptr, (uint8_t*)nullptr);
  else if (g_x2 == 5 && WB == 1)  // diagnostic: no wavefront
    hipLaunchKernelGGL((k_plane_resolve_x2h<NO, false, 2>), dim3(blocks), dim3(256), 0, st, (uint8_t*)tab, list, n, g,
                       zero, (const uint8_t*)nullptr, (uint8_t*)nullptr);
  else if (g_x2 == 3 && WB == 1)
    hipLaunchKernelGGL((k_plane_resolve_x2h<NO, false>), dim3(blocks), dim3(256), 0, st, (uint8_t*)tab, list, n, g,
                       zero, (const uint8_t*)nullptr, (uint8_t*)nullptr);
  else if (g_x2 == 2 && WB == 1)
    hipLaunchKernelGGL((k_plane_resolve_x2l<NO, false>), dim3(blocks), dim3(256), 0, st, (uint8_t*)tab, list, n, g,
                       zero, (const uint8_t*)nullptr, (uint8_t*)nullptr);
  else if (g_x2)
    hipLaunchKernelGGL((k_plane_resolve_x2<WB, NO, false>), dim3(blocks), dim3(256), 0, st, (T*)tab, list, n, g, zero,
                       (const T*)nullptr, (T*)nullptr, (const uint32_t*)nullptr, 0u);
  else
    hipLaunchKernelGGL((k_plane_resolve<WB, NO, false>), dim3(blocks), dim3(256), 0, st, (T*)tab, list, n, g, zero,
                       (const T*)nullptr, (T*)nullptr, (const uint32_t*)nullptr, 0u);
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 6;
  const int top = argc > 2 ? atoi(argv[2]) : 31;
  const int WB = argc > 3 ? atoi(argv[3]) : 1;
  const int reps = argc > 4 ? atoi(argv[4]) : 10;
  g_x2 = argc > 5 ? atoi(argv[5]) : 1;
  std::vector<int> heaps(K, 31);
  heaps[K - 1] = top;
  PlaneGeom g{};
  g.no = K - 2;
  g.pow2 = 1;
  g.world = 1;
  uint64_t np = 1;
  int root_sum = 0;
  for (int h : heaps) root_sum += h;
  for (int j = 0; j < K - 2; j++) {
    g.base[j] = heaps[j + 2] + 1;
    g.stride[j] = (uint32_t)np;
    g.shift[j] = __builtin_ctzll(np);
    if (g.base[j] & (g.base[j] - 1)) g.pow2 = 0;
    np *= g.base[j];
  }
  g.nplanes = (uint32_t)np;
  if (WB == 1 && root_sum > 253) {
    fprintf(stderr, "8-bit words need root_sum <= 253\n");
    return 1;
  }
  // per-level lists
  int S = 0;
  for (int j = 0; j < K - 2; j++) S += heaps[j + 2];
  std::vector<uint32_t> cnt(S + 2, 0), off(S + 2, 0), list(np);
  auto osum = [&](uint64_t P) {
    int s = 0;
    for (int j = 0; j < K - 2; j++) {
      s += (int)(P % g.base[j]);
      P /= g.base[j];
    }
    return s;
  };
  for (uint64_t P = 0; P < np; P++) cnt[osum(P)]++;
  for (int s = 0; s <= S; s++) off[s + 1] = off[s] + cnt[s];
  {
    std::vector<uint32_t> pos(off.begin(), off.end());
    for (uint64_t P = 0; P < np; P++) list[pos[osum(P)]++] = (uint32_t)P;
  }
  const size_t tbytes = np * 1024 * (size_t)WB;
  void *tab, *zero;
  uint32_t* dlist;
  CK(hipMalloc(&tab, tbytes));
  CK(hipMalloc(&zero, 4096));
  CK(hipMemset(zero, 0, 4096));
  CK(hipMalloc(&dlist, np * 4));
  CK(hipMemcpy(dlist, list.data(), np * 4, hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<hipEvent_t> lev_ev;
  bool lev_timing = false;
  auto run = [&]() {
    for (int s = 0; s <= S; s++) {
      if (lev_timing) CK(hipEventRecord(lev_ev[s], st));
      const uint32_t n = cnt[s];
      const uint32_t* l = dlist + off[s];
      switch (WB * 10 + (K - 2)) {
#define C(wb, no)                                                   \
  case wb * 10 + no:                                                \
    launch<wb, no>(tab, l, n, g, (const uint4*)zero, st); \
    break;
        C(1, 0) C(1, 1) C(1, 2) C(1, 3) C(1, 4) C(1, 5) C(2, 0) C(2, 1) C(2, 2) C(2, 3) C(2, 4) C(2, 5)
#undef C
        default:
          fprintf(stderr, "unsupported\n");
          exit(1);
      }
    }
    if (lev_timing) CK(hipEventRecord(lev_ev[S + 1], st));
  };
  run();
  CK(hipStreamSynchronize(st));
  CK(hipGetLastError());
  std::vector<float> ts;
  for (int r = 0; r < reps; r++) {
    CK(hipEventRecord(e0, st));
    run();
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ts.push_back(ms);
  }
  if (getenv("LEVEL_TIMES")) {  // per-level times of one more solve (an event between launches)
    lev_ev.resize(S + 2);
    for (auto& ev : lev_ev) CK(hipEventCreate(&ev));
    lev_timing = true;
    run();
    CK(hipStreamSynchronize(st));
    lev_timing = false;
    printf("level_us");
    for (int s = 0; s <= S; s++) {
      float ms;
      CK(hipEventElapsedTime(&ms, lev_ev[s], lev_ev[s + 1]));
      printf(" %.1f", ms * 1e3);
    }
    printf("\n");
  }
  float best = 1e9, sum = 0;
  for (float t : ts) {
    best = t < best ? t : best;
    sum += t;
  }
  const double P = (double)np * 1024;
  printf("v%d K=%d top=%d wb=%d planes=%llu levels=%d positions=%.0f backward best %.3f ms mean %.3f ms (%.3g pos/s)\n",
         g_x2, K, top, WB, (unsigned long long)np, S + 1, P, best, sum / reps, P / (best * 1e-3));
  // root
  std::vector<uint8_t> host(tbytes);
  CK(hipMemcpy(host.data(), tab, tbytes, hipMemcpyDeviceToHost));
  auto word_at = [&](const std::vector<int>& h) {
    uint64_t Pl = 0, m = 1;
    for (int j = 0; j < K - 2; j++) {
      Pl += (uint64_t)h[j + 2] * m;
      m *= g.base[j];
    }
    const size_t idx = Pl * 1024 + h[1] * 32 + ((h[0] + h[1]) & 31);
    return WB == 1 ? (uint32_t)host[idx] : (uint32_t)((uint16_t*)host.data())[idx];
  };
  const uint32_t rw = plane_word_to_vr(word_at(heaps), WB);
  printf("root: %s in %u moves\n", (rw & 3) ? "LOSS" : "WIN", rw >> 2);
  // full CPU check for small shapes
  if (P <= (double)(1 << 26)) {
    const uint64_t N = (uint64_t)P;
    std::vector<uint32_t> vr(N);  // value | rem << 2
    std::vector<uint64_t> strides(K);
    uint64_t s = 1;
    for (int i = 0; i < K; i++) {
      strides[i] = s;
      s *= heaps[i] + 1;
    }
    uint64_t bad = 0;
    std::vector<int> h(K);
    for (uint64_t r = 0; r < N; r++) {
      uint64_t x = r;
      for (int i = 0; i < K; i++) {
        h[i] = (int)(x % (heaps[i] + 1));
        x /= heaps[i] + 1;
      }
      uint32_t w;
      if (r == 0) {
        w = 1u;
      } else {
        bool win = false;
        uint32_t minl = ~0u, maxr = 0;
        for (int i = 0; i < K; i++)
          for (int k = 1; k <= 2 && k <= h[i]; k++) {
            const uint32_t c = vr[r - k * strides[i]];
            if ((c & 3) == 1) {
              win = true;
              minl = std::min(minl, c >> 2);
            }
            maxr = std::max(maxr, c >> 2);
          }
        w = win ? (0u | ((minl + 1) << 2)) : (1u | ((maxr + 1) << 2));
      }
      vr[r] = w;
      const uint32_t gw = plane_word_to_vr(word_at(h), WB);
      if (gw != w && bad++ < 5)
        printf("MISMATCH at rank %llu: gpu %u/%u cpu %u/%u\n", (unsigned long long)r, gw & 3, gw >> 2, w & 3, w >> 2);
    }
    printf("full check: %llu mismatches of %llu\n", (unsigned long long)bad, (unsigned long long)N);
    if (bad) return 2;
  }
  return 0;
}
