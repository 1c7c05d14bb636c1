// pad_lab.hip -- does the PLANES table's natural placement cost L2 hits?
// Diagnostic tool, not product code.
//
// In the natural layout plane P = d0 + 32 d1 + 1024 d2 + 32768 d3 (outer
// digits) sits at byte P * 1024, so its lines fall in L2 set (8 P + i) mod
// 2^k: only the low digits choose the set, while one launch reads, from one
// XCD's L2, planes that differ in the HIGH digits at equal low ones (a
// level's tile: d0 = s - d1 - d2 - d3).  This lab runs the product's visit
// (8-bit absolute forms, four planes per wave, write-through row stores) with
// the plane base taken from per-digit strides in 128-B lines, padded by `pad`
// lines at every digit boundary (S0 = 8, S(j+1) = 32 S(j) + pad), so the
// high digits move the set index too, and compares every byte with the
// product kernel (k_plane_resolve_x2 over the natural table).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/pad_lab.hip -o tools/pad_lab
//   ./tools/pad_lab pad [reps] [level_times] [check] [diag] [plain] [single_level]
// diag: 0 full visit; 1 neighbour rows = the plane's own rows (L1/L2-hot);
//       2 no neighbour loads; 3 no wavefront (stores the folded E); 4 neither
//       (list entry + stores); 5 an empty kernel (the launch alone)
// plain: 1 = plain row stores (write-back, the line stays in L2) instead of sc1
// single_level = s >= 0: launch level s 200 times back to back instead (the
// per-launch time of one level in steady state)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../gamesmanmpi_amd/csrc/gm_plane.h"
using namespace gm;

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

struct PadGeom {
  uint32_t S[4];  // line stride of outer digit j
};

template <int DIAG, bool PLAIN = false>
__global__ __launch_bounds__(256) void k_pad(uint8_t* __restrict__ tab, const uint32_t* __restrict__ list,
                                             uint32_t n, PadGeom pg, const uint4* __restrict__ zero) {
  if (DIAG == 5) return;  // the empty launch
  const PlaneShare sh = plane_share(n, 4);
  const uint32_t lane = threadIdx.x & 63, L = lane & 31;
  for (uint32_t i0 = sh.first; i0 < sh.end; i0 += sh.stride) {
    const uint32_t ix = i0 + 2 * (lane >> 5), iy = ix + 1;
    const bool livex = ix < sh.end, livey = iy < sh.end;
    const uint32_t px = list[livex ? ix : i0], py = list[livey ? iy : i0];
    uint32_t dx[4], dy[4], bx = 0, by = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      dx[j] = (px >> (5 * j)) & 31u;
      dy[j] = (py >> (5 * j)) & 31u;
      bx += dx[j] * pg.S[j];
      by += dy[j] * pg.S[j];
    }
    const size_t ox = (size_t)bx * 128u + L * 16u, oy = (size_t)by * 128u + L * 16u;
    uint32_t Xh[8], Xl[8], Yh[8], Yl[8];
#pragma unroll
    for (int d = 0; d < 8; d++) Xh[d] = Xl[d] = Yh[d] = Yl[d] = 0;
    auto nb = [&](const uint32_t* dig, size_t off, int j, int k) -> const uint4* {
      if (DIAG == 1) return (const uint4*)(tab + off);
      return dig[j] >= (uint32_t)k ? (const uint4*)(tab + off - (size_t)k * pg.S[j] * 128u) : zero;
    };
    if (DIAG != 2 && DIAG != 4) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint4 *sx1 = nb(dx, ox, j, 1), *sy1 = nb(dy, oy, j, 1), *sx2 = nb(dx, ox, j, 2),
                    *sy2 = nb(dy, oy, j, 2);
        uint4 vx1[2], vy1[2], vx2[2], vy2[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
          vx1[q] = sx1[q * kPieceU4];
          vy1[q] = sy1[q * kPieceU4];
          vx2[q] = sx2[q * kPieceU4];
          vy2[q] = sy2[q * kPieceU4];
        }
#pragma unroll
        for (int q = 0; q < 2; q++) {
          const uint32_t a1[4] = {vx1[q].x, vx1[q].y, vx1[q].z, vx1[q].w};
          const uint32_t b1[4] = {vy1[q].x, vy1[q].y, vy1[q].z, vy1[q].w};
          const uint32_t a2[4] = {vx2[q].x, vx2[q].y, vx2[q].z, vx2[q].w};
          const uint32_t b2[4] = {vy2[q].x, vy2[q].y, vy2[q].z, vy2[q].w};
#pragma unroll
          for (int c = 0; c < 4; c++) {
            const int d = 4 * q + c;
            Xh[d] = pk_max16(pk_max16(Xh[d], a1[c]), a2[c]);
            Yh[d] = pk_max16(pk_max16(Yh[d], b1[c]), b2[c]);
            Xl[d] = pk_max3w<true>(Xl[d], a1[c] & 0x00FF00FFu, a2[c] & 0x00FF00FFu);
            Yl[d] = pk_max3w<true>(Yl[d], b1[c] & 0x00FF00FFu, b2[c] & 0x00FF00FFu);
          }
        }
      }
    }
    uint32_t ox_[8], oy_[8];
    if (DIAG == 3 || DIAG == 4) {
#pragma unroll
      for (int d = 0; d < 8; d++) {
        ox_[d] = perm(Xh[d], Xl[d], 0x07020500u);
        oy_[d] = perm(Yh[d], Yl[d], 0x07020500u);
      }
    } else {
      const uint32_t primv = L == 0 ? ((px == 0 ? 0xFFu : 0u) | (py == 0 ? 0xFFu << 16 : 0u)) : 0u;
      uint32_t cur = 0, prev = 0, u1p = 0;
      uint32_t op[32];
      const uint32_t A0 = ~0u << L;
      auto phase = [&](auto PHc) {
        constexpr int PH = decltype(PHc)::value;
        const uint32_t A = PH ? ~A0 : A0;
#pragma unroll
        for (int q = 0; q < 32; q++) {
          const int d = q >> 2, b = q & 3;
          const uint32_t sel = 0x0C000C00u | ((4u + (uint32_t)b) << 16) | (uint32_t)b;
          const uint32_t a = (b & 1) ? perm(Yh[d], Xh[d], sel) : perm(Yl[d], Xl[d], sel);
          const uint32_t u2r = from_lane_below(u1p);
          const uint32_t pre = pk_max3w<true>(a, prev, u2r);
          const uint32_t u1r = from_lane_below(cur);
          const uint32_t pre_ = PH == 0 ? ((__builtin_amdgcn_sbfe((int)A, q, 1) != 0) ? pre : 0x00FF00FFu) : pre;
          const uint32_t m = pk_max3w<true>(pre_, cur, u1r);
          uint32_t f = parent_x2<1>(m);
          if (PH == 0) {
            if (q == 0) f = pk_max16(f, primv);
            op[q] = f;
          } else {
            op[q] = __builtin_amdgcn_sbfe((int)A, q, 1) ? f : op[q];
          }
          prev = cur;
          cur = f;
          u1p = u1r;
        }
      };
      phase(std::integral_constant<int, 0>());
      phase(std::integral_constant<int, 1>());
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint32_t t1 = perm(op[4 * k + 1], op[4 * k], 0x06020400u);
        const uint32_t t2 = perm(op[4 * k + 3], op[4 * k + 2], 0x06020400u);
        ox_[k] = perm(t2, t1, 0x05040100u);
        oy_[k] = perm(t2, t1, 0x07060302u);
      }
    }
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    auto store = [&](uint8_t* dst, const uint32_t* o) {
      uint4* p = (uint4*)dst;
#pragma unroll
      for (int q = 0; q < 2; q++) {
        if (PLAIN) {
          p[q * kPieceU4] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
        } else {
          const v4u v = {o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]};
          asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p + q * kPieceU4), "v"(v) : "memory");
        }
      }
    };
    if (livex) store(tab + ox, ox_);
    if (livey) store(tab + oy, oy_);
  }
}

int main(int argc, char** argv) {
  const int pad = argc > 1 ? atoi(argv[1]) : 0;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const bool lev_times = argc > 3 && atoi(argv[3]);
  const bool check = argc > 4 ? atoi(argv[4]) != 0 : true;
  const int diag = argc > 5 ? atoi(argv[5]) : 0;
  const int plain = argc > 6 ? atoi(argv[6]) : 0;
  const int single = argc > 7 ? atoi(argv[7]) : -1;
  const int NO = 4, S = 124;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const uint32_t gridcap = prop.multiProcessorCount * 8 * 4;
  PlaneGeom g{};
  g.no = NO;
  g.pow2 = 1;
  g.world = 1;
  uint64_t np = 1;
  for (int j = 0; j < NO; j++) {
    g.base[j] = 32;
    g.stride[j] = (uint32_t)np;
    g.shift[j] = 5 * j;
    np *= 32;
  }
  g.nplanes = (uint32_t)np;
  PadGeom pg;
  pg.S[0] = 8;
  for (int j = 1; j < 4; j++) pg.S[j] = 32 * pg.S[j - 1] + (uint32_t)pad;
  const size_t lines = (size_t)31 * (pg.S[0] + pg.S[1] + pg.S[2] + pg.S[3]) + 8;
  std::vector<uint32_t> cnt(S + 2, 0), off(S + 2, 0), list(np);
  auto osum = [&](uint64_t P) {
    int s = 0;
    for (int j = 0; j < NO; j++) s += (int)((P >> (5 * j)) & 31);
    return s;
  };
  for (uint64_t P = 0; P < np; P++) cnt[osum(P)]++;
  for (int s = 0; s <= S; s++) off[s + 1] = off[s] + cnt[s];
  {
    std::vector<uint32_t> pos(off.begin(), off.end());
    for (uint64_t P = 0; P < np; P++) list[pos[osum(P)]++] = (uint32_t)P;
  }
  {  // the product's order: 8^3 tiles over the digits above the lowest
    auto key = [&](uint32_t P) {
      uint64_t k = 0;
      uint32_t d[4];
      for (int j = 0; j < 4; j++) d[j] = (P >> (5 * j)) & 31;
      for (int j = 3; j >= 1; j--) k = k * 64 + d[j] / 8;
      for (int j = 3; j >= 1; j--) k = k * 64 + d[j] % 8;
      return k * 64 + d[0];
    };
    for (int s = 0; s <= S; s++)
      std::sort(list.begin() + off[s], list.begin() + off[s + 1],
                [&](uint32_t a, uint32_t b) { return key(a) < key(b); });
  }
  const size_t tbytes = np * 1024, pbytes = lines * 128;
  uint8_t *tab, *ptab;
  void* zero;
  uint32_t* dlist;
  CK(hipMalloc(&tab, tbytes));
  CK(hipMalloc(&ptab, pbytes));
  CK(hipMalloc(&zero, 4096));
  CK(hipMemset(zero, 0, 4096));
  CK(hipMalloc(&dlist, np * 4));
  CK(hipMemcpy(dlist, list.data(), np * 4, hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  std::vector<hipEvent_t> ev(S + 2);
  for (auto& evt : ev) CK(hipEventCreate(&evt));
  auto launch = [&](int v, uint32_t s) {
    const uint32_t n = cnt[s];
    const uint32_t* l = dlist + off[s];
    const uint32_t waves = (n + 3) / 4;
    uint32_t blocks = (waves + 3) / 4;
    blocks = std::min<uint32_t>((blocks + 7) / 8 * 8, gridcap);
    const dim3 G(blocks), B(256);
    if (v == 0) {
      hipLaunchKernelGGL((k_plane_resolve_x2<1, 4, false, 0>), G, B, 0, st, tab, (const void*)l, n, g,
                         (const uint4*)zero, (const uint8_t*)nullptr, (uint8_t*)nullptr, (const uint32_t*)nullptr, 0u);
    } else {
      auto go = [&](auto PL) {
        constexpr bool P_ = decltype(PL)::value;
        switch (diag) {
          case 1: hipLaunchKernelGGL((k_pad<1, P_>), G, B, 0, st, ptab, l, n, pg, (const uint4*)zero); break;
          case 2: hipLaunchKernelGGL((k_pad<2, P_>), G, B, 0, st, ptab, l, n, pg, (const uint4*)zero); break;
          case 3: hipLaunchKernelGGL((k_pad<3, P_>), G, B, 0, st, ptab, l, n, pg, (const uint4*)zero); break;
          case 4: hipLaunchKernelGGL((k_pad<4, P_>), G, B, 0, st, ptab, l, n, pg, (const uint4*)zero); break;
          case 5: hipLaunchKernelGGL((k_pad<5, P_>), G, B, 0, st, ptab, l, n, pg, (const uint4*)zero); break;
          default: hipLaunchKernelGGL((k_pad<0, P_>), G, B, 0, st, ptab, l, n, pg, (const uint4*)zero); break;
        }
      };
      if (plain) go(std::true_type());
      else go(std::false_type());
    }
  };
  auto run = [&](int v, bool per_level) {
    for (int s = 0; s <= S; s++) {
      if (per_level || s == 0) CK(hipEventRecord(ev[s], st));
      launch(v, s);
    }
    CK(hipEventRecord(ev[S + 1], st));
  };
  auto timeit = [&](int v, const char* name) {
    run(v, false);
    CK(hipStreamSynchronize(st));
    CK(hipGetLastError());
    std::vector<float> ts;
    for (int r = 0; r < reps; r++) {
      run(v, false);
      CK(hipEventSynchronize(ev[S + 1]));
      float ms;
      CK(hipEventElapsedTime(&ms, ev[0], ev[S + 1]));
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    printf("%s pad=%d diag=%d plain=%d backward best %.4f ms median %.4f ms\n", name, pad, diag, plain, ts[0], ts[ts.size() / 2]);
    if (lev_times) {
      run(v, true);
      CK(hipStreamSynchronize(st));
      printf("level_us %s:", name);
      for (int s = 0; s <= S; s++) {
        float ms;
        CK(hipEventElapsedTime(&ms, ev[s], ev[s + 1]));
        printf(" %.1f", ms * 1e3);
      }
      printf("\n");
    }
    fflush(stdout);
  };
  if (single >= 0) {  // one level, 200 launches back to back
    for (int w = 0; w < 2; w++) {
      CK(hipEventRecord(ev[0], st));
      for (int r = 0; r < 200; r++) launch(pad < 0 ? 0 : 1, (uint32_t)single);
      CK(hipEventRecord(ev[1], st));
      CK(hipEventSynchronize(ev[1]));
    }
    float ms;
    CK(hipEventElapsedTime(&ms, ev[0], ev[1]));
    printf("single level %d (%u planes) %s pad=%d diag=%d plain=%d: %.2f us per launch\n", single, cnt[single],
           pad < 0 ? "product" : "padlab", pad, diag, plain, ms * 1e3 / 200);
    return 0;
  }
  if (pad >= 0) timeit(1, "padlab");
  if (check || pad < 0) timeit(0, "product");
  if (check && diag == 0 && pad >= 0) {
    std::vector<uint8_t> ref(tbytes), got(pbytes);
    CK(hipMemset(tab, 0x5A, tbytes));
    CK(hipMemset(ptab, 0xA5, pbytes));
    run(0, false);
    run(1, false);
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(ref.data(), tab, tbytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(got.data(), ptab, pbytes, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (uint64_t P = 0; P < np; P++) {
      size_t b = 0;
      for (int j = 0; j < 4; j++) b += ((P >> (5 * j)) & 31) * pg.S[j];
      if (memcmp(ref.data() + P * 1024, got.data() + b * 128, 1024)) bad++;
    }
    printf("check pad=%d: %zu planes differ of %llu%s\n", pad, bad, (unsigned long long)np, bad ? " MISMATCH" : "");
    if (bad) return 2;
  }
  return 0;
}
