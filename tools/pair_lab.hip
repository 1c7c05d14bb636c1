// pair_lab.hip -- two plane levels per launch for the narrow levels of the
// PLANES backward (diagnostic tool; the product form is k_plane_pair in
// gm_plane.h once it wins).
//
// A narrow plane level costs about one dependent launch (~4.5 us: boundary,
// list entry, neighbour rows, 64-step wavefront, row stores) however few
// planes it holds.  Here ONE launch resolves levels s and s + 1: each wave
// takes one plane P of level s + 1, first resolves its four k = 1 neighbours
// P - e_j (level s) in its four channels (one visit: lane halves x 16-bit
// halves), then P itself, its k = 1 rows taken from the first visit's
// registers (the upper lane half's through LDS) and its k = 2 rows (level
// s - 1) from memory.  Every level-s plane is resolved by each of its
// level-(s + 1) parents (redundant work, nothing at narrow levels) and
// STORED by exactly one: the parent P = Q + e_j whose j is the lowest digit
// with P's digits below j all at their maximum (so Q + e_j exists).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/pair_lab.hip -o tools/pair_lab
//   ./tools/pair_lab lo hi lo2 hi2 [reps] [level_times]
// pairs (s, s + 1) for s = lo, lo + 2, ... while s + 1 <= hi, and likewise in
// [lo2, hi2]; every other level is a product launch.  Checked byte for byte
// against the product kernel at every level.
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

// The product visit's arithmetic (8-bit absolute forms, four planes per wave)
// as a device function over per-lane plane indices: lanes 0-31 resolve
// planes px (low halves) and py (high halves) of their row L, lanes 32-63
// theirs; E rows come from `fold` (the caller's), results come back as the
// lane's two rows in byte form (ox, oy).
template <class Fold>
__device__ __forceinline__ void pair_wavefront(uint32_t L, uint32_t primv, Fold fold, uint32_t* ox, uint32_t* oy) {
  uint32_t Xh[8], Xl[8], Yh[8], Yl[8];
#pragma unroll
  for (int d = 0; d < 8; d++) Xh[d] = Xl[d] = Yh[d] = Yl[d] = 0;
  fold(Xh, Xl, Yh, Yl);
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
    ox[k] = perm(t2, t1, 0x05040100u);
    oy[k] = perm(t2, t1, 0x07060302u);
  }
}

// fold one neighbour row pair (X's row a, Y's row b: 8 dwords each) into the E rows
__device__ __forceinline__ void fold_rows(uint32_t* Xh, uint32_t* Xl, uint32_t* Yh, uint32_t* Yl, const uint32_t* a,
                                          const uint32_t* b) {
#pragma unroll
  for (int d = 0; d < 8; d++) {
    Xh[d] = pk_max16(Xh[d], a[d]);
    Yh[d] = pk_max16(Yh[d], b[d]);
    Xl[d] = pk_max16(Xl[d], a[d] & 0x00FF00FFu);
    Yl[d] = pk_max16(Yl[d], b[d] & 0x00FF00FFu);
  }
}
__device__ __forceinline__ void load_row(const uint8_t* tab, bool has, uint32_t P, uint32_t L, const uint4* zero,
                                         uint32_t* r) {
  const uint4* src = has ? (const uint4*)(tab + (size_t)P * 1024u + L * 16u) : zero;
  const uint4 v0 = src[0], v1 = src[kPieceU4];
  r[0] = v0.x, r[1] = v0.y, r[2] = v0.z, r[3] = v0.w;
  r[4] = v1.x, r[5] = v1.y, r[6] = v1.z, r[7] = v1.w;
}
__device__ __forceinline__ void store_row(uint8_t* tab, uint32_t P, uint32_t L, const uint32_t* o) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  uint4* p = (uint4*)(tab + (size_t)P * 1024u + L * 16u);
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const v4u v = {o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p + q * kPieceU4), "v"(v) : "memory");
  }
}

// One wave per plane P of level s + 1 (list = level s + 1's planes; four
// outer digits of 32 values, plane index = d0 + 32 d1 + 1024 d2 + 32768 d3).
__global__ __launch_bounds__(256) void k_pair(uint8_t* __restrict__ tab, const uint32_t* __restrict__ list, uint32_t n,
                                              const uint4* __restrict__ zero) {
  __shared__ uint32_t xch[4][32][16];  // per wave: the upper lane half's two rows for the lower half
  const uint32_t lane = threadIdx.x & 63, L = lane & 31, hi = lane >> 5, w = threadIdx.x >> 6;
  const uint32_t stride[4] = {1u, 32u, 1024u, 32768u};
  for (uint32_t i0 = blockIdx.x * 4; i0 < n; i0 += gridDim.x * 4) {  // uniform per block: the barriers below
    const uint32_t i = i0 + w;
    const bool valid = i < n;
    const uint32_t P = list[valid ? i : i0];
    uint32_t dP[4];
#pragma unroll
    for (int j = 0; j < 4; j++) dP[j] = (P >> (5 * j)) & 31u;
    // visit 1: channel (hi, half) = digit j = 2 hi + half: plane Q_j = P - e_j
    const uint32_t jx = 2 * hi, jy = 2 * hi + 1;
    const bool hx = dP[jx] >= 1, hy = dP[jy] >= 1;
    const uint32_t qx = hx ? P - stride[jx] : 0u, qy = hy ? P - stride[jy] : 0u;
    uint32_t dx[4], dy[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      dx[j] = (qx >> (5 * j)) & 31u;
      dy[j] = (qy >> (5 * j)) & 31u;
    }
    const uint32_t primv1 = L == 0 ? (((hx && qx == 0) ? 0xFFu : 0u) | ((hy && qy == 0) ? 0xFFu << 16 : 0u)) : 0u;
    uint32_t rx[8], ry[8];
    pair_wavefront(
        L, primv1,
        [&](uint32_t* Xh, uint32_t* Xl, uint32_t* Yh, uint32_t* Yl) {
#pragma unroll
          for (int j = 0; j < 4; j++)
#pragma unroll
            for (uint32_t k = 1; k <= 2; k++) {
              uint32_t a[8], b[8];
              load_row(tab, hx && dx[j] >= k, qx - k * stride[j], L, zero, a);
              load_row(tab, hy && dy[j] >= k, qy - k * stride[j], L, zero, b);
              fold_rows(Xh, Xl, Yh, Yl, a, b);
            }
        },
        rx, ry);
    // the designated writer of Q_j: digits of P below j all 31
    auto writes = [&](uint32_t j) {
      bool ok = true;
      for (uint32_t t = 0; t < j; t++) ok = ok && dP[t] == 31u;
      return ok;
    };
    if (valid && hx && writes(jx)) store_row(tab, qx, L, rx);
    if (valid && hy && writes(jy)) store_row(tab, qy, L, ry);
    // the k = 1 rows of P: Q_0, Q_1 in this lane (lower half) / Q_2, Q_3 in lane L + 32
    if (hi) {
#pragma unroll
      for (int d = 0; d < 8; d++) {
        xch[w][L][d] = hx ? rx[d] : 0u;
        xch[w][L][8 + d] = hy ? ry[d] : 0u;
      }
    }
    __syncthreads();
    uint32_t q2[8], q3[8];
#pragma unroll
    for (int d = 0; d < 8; d++) {
      q2[d] = xch[w][L][d];
      q3[d] = xch[w][L][8 + d];
    }
    __syncthreads();
    // visit 2: P in the lower half's low channel (the other channels idle)
    const uint32_t primv2 = (L == 0 && P == 0) ? 0xFFu : 0u;
    uint32_t rp[8], rz[8];
    pair_wavefront(
        L, primv2,
        [&](uint32_t* Xh, uint32_t* Xl, uint32_t* Yh, uint32_t* Yl) {
          uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0}, a[8];
          uint32_t r0[8], r1[8];
#pragma unroll
          for (int d = 0; d < 8; d++) {
            r0[d] = hx ? rx[d] : 0u;  // lower half: Q_0, Q_1
            r1[d] = hy ? ry[d] : 0u;
          }
          fold_rows(Xh, Xl, Yh, Yl, r0, z);
          fold_rows(Xh, Xl, Yh, Yl, r1, z);
          fold_rows(Xh, Xl, Yh, Yl, q2, z);
          fold_rows(Xh, Xl, Yh, Yl, q3, z);
#pragma unroll
          for (int j = 0; j < 4; j++) {
            load_row(tab, dP[j] >= 2, P - 2 * stride[j], L, zero, a);
            fold_rows(Xh, Xl, Yh, Yl, a, z);
          }
        },
        rp, rz);
    if (valid && !hi) store_row(tab, P, L, rp);
  }
}

int main(int argc, char** argv) {
  const int lo = argc > 1 ? atoi(argv[1]) : 4, hi = argc > 2 ? atoi(argv[2]) : 17;
  const int lo2 = argc > 3 ? atoi(argv[3]) : 107, hi2 = argc > 4 ? atoi(argv[4]) : 120;
  const int reps = argc > 5 ? atoi(argv[5]) : 10;
  const bool lev_times = argc > 6 && atoi(argv[6]);
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
  {
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
  // the schedule: pair starts (level s of a pair (s, s + 1))
  std::vector<int> pair_at(S + 2, 0);
  for (int s = lo; s + 1 <= hi; s += 2) pair_at[s] = 1;
  for (int s = lo2; s + 1 <= hi2; s += 2) pair_at[s] = 1;
  const size_t tbytes = np * 1024;
  uint8_t* tab;
  void* zero;
  uint32_t* dlist;
  CK(hipMalloc(&tab, tbytes));
  CK(hipMalloc(&zero, 4096));
  CK(hipMemset(zero, 0, 4096));
  CK(hipMalloc(&dlist, np * 4));
  CK(hipMemcpy(dlist, list.data(), np * 4, hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  std::vector<hipEvent_t> ev(S + 2);
  for (auto& evt : ev) CK(hipEventCreate(&evt));
  int launches = 0;
  auto product = [&](int s) {
    const uint32_t n = cnt[s];
    const uint32_t waves = (n + 3) / 4;
    uint32_t blocks = (waves + 3) / 4;
    blocks = std::min<uint32_t>((blocks + 7) / 8 * 8, gridcap);
    hipLaunchKernelGGL((k_plane_resolve_x2<1, 4, false, 0>), dim3(blocks), dim3(256), 0, st, tab,
                       (const void*)(dlist + off[s]), n, g, (const uint4*)zero, (const uint8_t*)nullptr, (uint8_t*)nullptr,
                       (const uint32_t*)nullptr, 0u);
  };
  auto run = [&](bool pairs, bool per_level) {
    launches = 0;
    for (int s = 0; s <= S; s++) {
      if (per_level || s == 0) CK(hipEventRecord(ev[s], st));
      if (pairs && pair_at[s]) {
        const uint32_t n = cnt[s + 1];
        const uint32_t blocks = std::min<uint32_t>((n + 3) / 4, gridcap);
        hipLaunchKernelGGL(k_pair, dim3(blocks), dim3(256), 0, st, tab, dlist + off[s + 1], n, (const uint4*)zero);
        launches++;
        if (per_level) CK(hipEventRecord(ev[s + 1], st));
        s++;
        continue;
      }
      product(s);
      launches++;
    }
    CK(hipEventRecord(ev[S + 1], st));
  };
  auto timeit = [&](bool pairs, const char* name) {
    run(pairs, false);
    CK(hipStreamSynchronize(st));
    CK(hipGetLastError());
    std::vector<float> ts;
    for (int r = 0; r < reps; r++) {
      run(pairs, false);
      CK(hipEventSynchronize(ev[S + 1]));
      float ms;
      CK(hipEventElapsedTime(&ms, ev[0], ev[S + 1]));
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    printf("%s [%d,%d] [%d,%d]: %d launches, backward best %.4f ms median %.4f ms\n", name, lo, hi, lo2, hi2, launches,
           ts[0], ts[ts.size() / 2]);
    if (lev_times) {
      run(pairs, true);
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
  timeit(false, "product");
  timeit(true, "pairs");
  timeit(false, "product");
  timeit(true, "pairs");
  std::vector<uint8_t> ref(tbytes), got(tbytes);
  CK(hipMemset(tab, 0x5A, tbytes));
  run(false, false);
  CK(hipStreamSynchronize(st));
  CK(hipMemcpy(ref.data(), tab, tbytes, hipMemcpyDeviceToHost));
  CK(hipMemset(tab, 0xA5, tbytes));
  run(true, false);
  CK(hipStreamSynchronize(st));
  CK(hipMemcpy(got.data(), tab, tbytes, hipMemcpyDeviceToHost));
  size_t bad = 0, first = 0;
  for (size_t i = 0; i < tbytes; i++)
    if (got[i] != ref[i]) {
      if (!bad) first = i;
      bad++;
    }
  printf("check pairs vs product: %zu differing bytes of %zu%s\n", bad, tbytes, bad ? " MISMATCH" : "");
  if (bad) {
    printf("first at plane %zu (level %d) byte %zu: got %02x want %02x\n", first / 1024, osum(first / 1024),
           first % 1024, got[first], ref[first]);
    return 2;
  }
  return 0;
}
