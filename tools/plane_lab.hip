// plane_lab.hip -- measurement harness for the PLANES backward (one GPU,
// sum_four_to_one heaps 31^K).  Diagnostic tool, not product code.
//
// Runs the product kernel (gm_plane.h, k_plane_resolve_x2<1, NO, false>) and
// lab variants of it over the same per-level lists, times whole backward
// passes with HIP events (optionally one event pair per level) and compares
// every table byte of the real variants with the product kernel's table.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/plane_lab.hip -o tools/plane_lab
//   ./tools/plane_lab K variant [reps] [level_times]
//
// variants: 0 product kernel; 1 lab kernel (lean step chain); 10+d lab
// kernel with diagnostic d (results wrong on purpose): 11 neighbour loads
// read the plane's own rows (L1/L2-hot, same instruction stream), 12 no
// neighbour loads, 13 no wavefront (store the folded E), 14 neither (store
// zeros: the launch + store floor).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
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

// Lab form of plane_x2_range (8-bit words, one table).  LEAN: the step chain
// without the lane-32 masks (lane 31's idle steps already read 0 there), the
// in-lane and lane-below-by-two children folded off the chain first, and the
// active-row mask one bit extract of a per-lane word.
template <int NO, int DIAG, bool LEAN, bool OPQ = false, int MINW = 1, bool ELDS = false, bool IMAX = false,
          bool PPAR = false>
__global__ __launch_bounds__(256, MINW) void lab_x2(uint8_t* __restrict__ tab, const uint32_t* __restrict__ list,
                                                    uint32_t n, PlaneGeom g, const uint4* __restrict__ zero,
                                                    uint64_t* __restrict__ stamps = nullptr) {
  uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, items = 0;
  if (DIAG == 5) t0 = __builtin_amdgcn_s_memtime();
  const PlaneShare sh = plane_share(n, 4);
  const uint32_t lane = threadIdx.x & 63, L = lane & 31;
  const bool l32 = lane == 32;
  for (uint32_t i0 = sh.first; i0 < sh.end; i0 += sh.stride) {
    const uint32_t ix = i0 + 2 * (lane >> 5), iy = ix + 1;
    const bool livex = ix < sh.end, livey = iy < sh.end;
    const uint32_t px = list[livex ? ix : i0], py = list[livey ? iy : i0];
    if (DIAG == 5) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (!items) t1 = __builtin_amdgcn_s_memtime() + (px & 0 ? 1 : 0);
      items++;
    }
    uint32_t dx[NO > 0 ? NO : 1], dy[NO > 0 ? NO : 1];
    plane_digits<NO>(g, px, dx);
    plane_digits<NO>(g, py, dy);
    const size_t ox = (size_t)px * 1024u + L * 32u, oy = (size_t)py * 1024u + L * 32u;
    uint32_t Xh[8], Xl[8], Yh[8], Yl[8];
#pragma unroll
    for (int d = 0; d < 8; d++) Xh[d] = Yh[d] = Xl[d] = Yl[d] = 0;
    if (DIAG != 2 && DIAG != 4) {
#pragma unroll
      for (int j = 0; j < NO; j++) {
#pragma unroll
        for (int k = 1; k <= 2; k++) {
          const uint4* sx = DIAG == 1 ? (const uint4*)(tab + ox)
                            : dx[j] >= (uint32_t)k ? (const uint4*)(tab + ox - (size_t)k * g.stride[j] * 1024u) : zero;
          const uint4* sy = DIAG == 1 ? (const uint4*)(tab + oy)
                            : dy[j] >= (uint32_t)k ? (const uint4*)(tab + oy - (size_t)k * g.stride[j] * 1024u) : zero;
          uint4 vx[2], vy[2];
#pragma unroll
          for (int q = 0; q < 2; q++) {
            vx[q] = sx[q];
            vy[q] = sy[q];
          }
#pragma unroll
          for (int q = 0; q < 2; q++) {
            const uint32_t a[4] = {vx[q].x, vx[q].y, vx[q].z, vx[q].w};
            const uint32_t b[4] = {vy[q].x, vy[q].y, vy[q].z, vy[q].w};
#pragma unroll
            for (int c = 0; c < 4; c++) {
              Xh[4 * q + c] = pk_max16(Xh[4 * q + c], a[c]);
              Yh[4 * q + c] = pk_max16(Yh[4 * q + c], b[c]);
              Xl[4 * q + c] = pk_max16(Xl[4 * q + c], pk_shl8(a[c]));
              Yl[4 * q + c] = pk_max16(Yl[4 * q + c], pk_shl8(b[c]));
            }
          }
        }
      }
    }
    if (DIAG == 5 && items == 1) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      t2 = __builtin_amdgcn_s_memtime();
    }
    uint32_t ox_[8], oy_[8];
    if (DIAG == 3 || DIAG == 4) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        ox_[k] = Xh[k] | (Xl[k] >> 8);
        oy_[k] = Yh[k] | (Yl[k] >> 8);
      }
    } else {
      // ELDS: the folded E rows go to LDS as interleaved bytes [X0 Y0 X1 Y1
      // ...] (64 B per lane, 4 KiB per wave) and come back 4 steps at a time
      // during the wavefront, so the 32 E registers die before it starts
      __shared__ uint2 elds[ELDS ? 4 * 8 * 64 : 1];  // [wave][quad of steps][lane]
      uint2* ew = elds + (threadIdx.x >> 6) * (8 * 64) + (threadIdx.x & 63);
      if (ELDS) {
#pragma unroll
        for (int d = 0; d < 8; d++) {
          // bytes 0-3 of X's and Y's rows at dword d: even bytes from the
          // high bytes of the low-shifted fold, odd bytes from the other
          const uint32_t xb = perm(Xh[d], Xl[d], 0x07030501u), yb = perm(Yh[d], Yl[d], 0x07030501u);
          ew[d * 64] = make_uint2(perm(yb, xb, 0x05010400u), perm(yb, xb, 0x07030602u));
        }
      }
      const uint32_t primv = L == 0 ? ((px == 0 ? 0xFFu : 0u) | (py == 0 ? 0xFFu << 16 : 0u)) : 0u;
      uint32_t cur = 0, prev = 0, u1p = 0;
      uint32_t op[32];
#pragma unroll
      for (int q = 0; q < 32; q++) op[q] = 0;
      const uint32_t A0 = ~0u << L;  // bit q: row L is active at step q of phase 0
#pragma unroll 1
      for (uint32_t ph = 0; ph < 2; ph++) {
        const uint32_t flip = ph ? 0xFFFFFFFFu : 0u;
        const uint32_t A = A0 ^ flip;
        if (OPQ) {
#pragma unroll
          for (int d = 0; d < 8; d++) asm volatile("" : "+v"(Xh[d]), "+v"(Xl[d]), "+v"(Yh[d]), "+v"(Yl[d]));
        }
        uint2 eq = make_uint2(0, 0);
#pragma unroll
        for (int q = 0; q < 32; q++) {
          const int d = q >> 2, b = q & 3;
          uint32_t a;
          if (ELDS) {
            if (b == 0) eq = ew[d * 64];
            const uint32_t w2 = b < 2 ? eq.x : eq.y;  // [Xq Yq Xq+1 Yq+1]
            a = (b & 1) ? perm(0u, w2, 0x0C030C02u) : perm(0u, w2, 0x0C010C00u);
          } else {
            const uint32_t bx = (b & 1) ? (uint32_t)b : (uint32_t)b + 1;
            const uint32_t sel = 0x0C000C00u | ((4u + bx) << 16) | bx;
            a = (b & 1) ? perm(Yh[d], Xh[d], sel) : perm(Yl[d], Xl[d], sel);
          }
          uint32_t f;
          if (LEAN && IMAX) {
            // idle rows: max with 0xFF per half, whose parent is 0 -- the mask
            // leaves the chain (folded into the off-chain max)
            const uint32_t idle = (uint32_t)__builtin_amdgcn_sbfe((int)~A, q, 1) & 0x00FF00FFu;
            const uint32_t u2r = from_lane_below(u1p);
            const uint32_t pre = pk_max16(pk_max16(a, prev), pk_max16(u2r, idle));
            const uint32_t u1r = from_lane_below(cur);
            const uint32_t m = pk_max16(pk_max16(pre, cur), u1r);
            f = parent_x2<1>(m);
            u1p = u1r;
          } else if (LEAN) {
            const uint32_t u2r = from_lane_below(u1p);
            const uint32_t pre = pk_max16(pk_max16(a, prev), u2r);
            const uint32_t u1r = from_lane_below(cur);
            const uint32_t m = pk_max16(pk_max16(pre, cur), u1r);
            const uint32_t keep = (uint32_t)__builtin_amdgcn_sbfe((int)A, q, 1);
            if (PPAR) {
              // parent as (0xFE - m) and (m >> 7) side by side, then one add:
              // the asm keeps the compiler from re-associating it into
              // ((m >> 7) - m) + 0xFE, one dependent op longer
              uint32_t t1;
              asm("v_pk_sub_u16 %0, %1, %2" : "=v"(t1) : "s"(0x00FE00FEu), "v"(m));
              f = pk_add16(t1, pk_shr16(m, 7)) & keep;
            } else {
              f = parent_x2<1>(m) & keep;
            }
            u1p = u1r;
          } else {
            const uint32_t u1r = from_lane_below(cur), u2r = from_lane_below(u1p);
            uint32_t m = pk_max16(pk_max16(a, cur), prev);
            const uint32_t m2 = pk_max16(pk_max16(m, u1r), u2r);
            m = l32 ? m : m2;
            const uint32_t am = (uint32_t)(q == 31 ? 0xFFFFFFFFull : ((2ull << q) - 1)) ^ flip;
            f = keep_rows(am, L, parent_x2<1>(m));
            u1p = l32 ? 0u : u1r;
          }
          if (q == 0) f = pk_max16(f, ph ? 0u : primv);
          op[q] |= f;
          prev = cur;
          cur = f;
        }
      }
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint32_t t1 = perm(op[4 * k + 1], op[4 * k], 0x06020400u);
        const uint32_t t2 = perm(op[4 * k + 3], op[4 * k + 2], 0x06020400u);
        ox_[k] = perm(t2, t1, 0x05040100u);
        oy_[k] = perm(t2, t1, 0x07060302u);
      }
    }
    if (DIAG == 4) {
#pragma unroll
      for (int k = 0; k < 8; k++) ox_[k] = oy_[k] = 0;
    }
    auto store = [&](uint8_t* dst, const uint32_t* o) {
      uint4* p = (uint4*)dst;
      p[0] = make_uint4(o[0], o[1], o[2], o[3]);
      p[1] = make_uint4(o[4], o[5], o[6], o[7]);
    };
    if (DIAG == 5 && items == 1) t3 = __builtin_amdgcn_s_memtime() + (ox_[0] & 0 ? 1 : 0);
    if (livex) store(tab + ox, ox_);
    if (livey) store(tab + oy, oy_);
  }
  if (DIAG == 5 && stamps) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t t4 = __builtin_amdgcn_s_memtime();
    const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0 && w < 65536 && items) {
      uint64_t* o = stamps + (size_t)w * 6;
      o[0] = t0;
      o[1] = t1;
      o[2] = t2;
      o[3] = t3;
      o[4] = t4;
      o[5] = items;
    }
  }
}

// Lab form with both phases unrolled (MODE 0: the lean chain, phase 0
// assigns op[q] instead of OR-ing into it) and (MODE 1) the active-row mask
// as ONE v_cndmask per step against a per-step constant lane mask in SGPRs
// instead of a per-lane bit extract + and.
template <int NO, int MODE>
__global__ __launch_bounds__(256) void lab_x2u(uint8_t* __restrict__ tab, const uint32_t* __restrict__ list, uint32_t n,
                                               PlaneGeom g, const uint4* __restrict__ zero) {
  const PlaneShare sh = plane_share(n, 4);
  const uint32_t lane = threadIdx.x & 63, L = lane & 31;
  for (uint32_t i0 = sh.first; i0 < sh.end; i0 += sh.stride) {
    const uint32_t ix = i0 + 2 * (lane >> 5), iy = ix + 1;
    const bool livex = ix < sh.end, livey = iy < sh.end;
    const uint32_t px = list[livex ? ix : i0], py = list[livey ? iy : i0];
    uint32_t dx[NO], dy[NO];
    plane_digits<NO>(g, px, dx);
    plane_digits<NO>(g, py, dy);
    const size_t ox = (size_t)px * 1024u + L * 32u, oy = (size_t)py * 1024u + L * 32u;
    uint32_t Xh[8], Xl[8], Yh[8], Yl[8];
#pragma unroll
    for (int d = 0; d < 8; d++) Xh[d] = Yh[d] = Xl[d] = Yl[d] = 0;
#pragma unroll
    for (int j = 0; j < NO; j++) {
#pragma unroll
      for (int k = 1; k <= 2; k++) {
        const uint4* sx = dx[j] >= (uint32_t)k ? (const uint4*)(tab + ox - (size_t)k * g.stride[j] * 1024u) : zero;
        const uint4* sy = dy[j] >= (uint32_t)k ? (const uint4*)(tab + oy - (size_t)k * g.stride[j] * 1024u) : zero;
        uint4 vx[2], vy[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
          vx[q] = sx[q];
          vy[q] = sy[q];
        }
#pragma unroll
        for (int q = 0; q < 2; q++) {
          const uint32_t a[4] = {vx[q].x, vx[q].y, vx[q].z, vx[q].w};
          const uint32_t b[4] = {vy[q].x, vy[q].y, vy[q].z, vy[q].w};
#pragma unroll
          for (int c = 0; c < 4; c++) {
            Xh[4 * q + c] = pk_max16(Xh[4 * q + c], a[c]);
            Yh[4 * q + c] = pk_max16(Yh[4 * q + c], b[c]);
            Xl[4 * q + c] = pk_max16(Xl[4 * q + c], pk_shl8(a[c]));
            Yl[4 * q + c] = pk_max16(Yl[4 * q + c], pk_shl8(b[c]));
          }
        }
      }
    }
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
        const uint32_t bx = (b & 1) ? (uint32_t)b : (uint32_t)b + 1;
        const uint32_t sel = 0x0C000C00u | ((4u + bx) << 16) | bx;
        const uint32_t a = (b & 1) ? perm(Yh[d], Xh[d], sel) : perm(Yl[d], Xl[d], sel);
        const uint32_t u2r = from_lane_below(u1p);
        const uint32_t pre = pk_max16(pk_max16(a, prev), u2r);
        const uint32_t u1r = from_lane_below(cur);
        const uint32_t m = pk_max16(pk_max16(pre, cur), u1r);
        uint32_t f = parent_x2<1>(m);
        if (MODE == 1) {
          // lanes active at step q: phase 0 rows 0..q, phase 1 rows q+1..31, in both halves
          const uint32_t m32 = q == 31 ? 0xFFFFFFFFu : ((2u << q) - 1u);
          const uint64_t mk = PH ? ~(((uint64_t)m32 << 32) | m32) : (((uint64_t)m32 << 32) | m32);
          uint32_t fo;
          asm("v_cndmask_b32 %0, 0, %1, %2" : "=v"(fo) : "v"(f), "s"(mk));
          f = fo;
        } else {
          f &= (uint32_t)__builtin_amdgcn_sbfe((int)A, q, 1);
        }
        if (q == 0 && PH == 0) f = pk_max16(f, primv);
        if (PH == 0) op[q] = f;
        else op[q] |= f;
        prev = cur;
        cur = f;
        u1p = u1r;
      }
    };
    phase(std::integral_constant<int, 0>());
    phase(std::integral_constant<int, 1>());
    uint32_t ox_[8], oy_[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t t1 = perm(op[4 * k + 1], op[4 * k], 0x06020400u);
      const uint32_t t2 = perm(op[4 * k + 3], op[4 * k + 2], 0x06020400u);
      ox_[k] = perm(t2, t1, 0x05040100u);
      oy_[k] = perm(t2, t1, 0x07060302u);
    }
    if (livex) {
      uint4* p = (uint4*)(tab + ox);
      p[0] = make_uint4(ox_[0], ox_[1], ox_[2], ox_[3]);
      p[1] = make_uint4(ox_[4], ox_[5], ox_[6], ox_[7]);
    }
    if (livey) {
      uint4* p = (uint4*)(tab + oy);
      p[0] = make_uint4(oy_[0], oy_[1], oy_[2], oy_[3]);
      p[1] = make_uint4(oy_[4], oy_[5], oy_[6], oy_[7]);
    }
  }
}

static int g_grid_blocks = 2048;
static uint64_t* g_stamps = nullptr;  // variant 15: per-wave s_memtime stamps of the level being traced

template <int NO>
static void launch(int var, uint8_t* tab, const uint32_t* list, uint32_t n, const PlaneGeom& g, const uint4* zero,
                   hipStream_t st) {
  const uint32_t waves = (n + 3) / 4;
  uint32_t blocks = (waves + 3) / 4;
  blocks = std::min<uint32_t>((blocks + 7) / 8 * 8, (uint32_t)g_grid_blocks * 4);
  const dim3 G(blocks), B(256);
  switch (var) {
    case 0:
      hipLaunchKernelGGL((k_plane_resolve_x2<1, NO, false, 0>), G, B, 0, st, tab, (const void*)list, n, g, zero,
                         (const uint8_t*)nullptr, (uint8_t*)nullptr, (const uint32_t*)nullptr, 0u);
      break;
    case 1: hipLaunchKernelGGL((lab_x2<NO, 0, true>), G, B, 0, st, tab, list, n, g, zero); break;
    case 10: hipLaunchKernelGGL((lab_x2<NO, 0, false>), G, B, 0, st, tab, list, n, g, zero); break;
    case 11: hipLaunchKernelGGL((lab_x2<NO, 1, false>), G, B, 0, st, tab, list, n, g, zero); break;
    case 12: hipLaunchKernelGGL((lab_x2<NO, 2, false>), G, B, 0, st, tab, list, n, g, zero); break;
    case 13: hipLaunchKernelGGL((lab_x2<NO, 3, false>), G, B, 0, st, tab, list, n, g, zero); break;
    case 14: hipLaunchKernelGGL((lab_x2<NO, 4, false>), G, B, 0, st, tab, list, n, g, zero); break;
    case 21: hipLaunchKernelGGL((lab_x2<NO, 1, true>), G, B, 0, st, tab, list, n, g, zero); break;
    case 22: hipLaunchKernelGGL((lab_x2<NO, 2, true>), G, B, 0, st, tab, list, n, g, zero); break;
    case 2: hipLaunchKernelGGL((lab_x2<NO, 0, true, true>), G, B, 0, st, tab, list, n, g, zero); break;
    case 3: hipLaunchKernelGGL((lab_x2<NO, 0, true, true, 5>), G, B, 0, st, tab, list, n, g, zero); break;
    case 15: hipLaunchKernelGGL((lab_x2<NO, 5, true, true>), G, B, 0, st, tab, list, n, g, zero, g_stamps); break;
    case 4: hipLaunchKernelGGL((lab_x2<NO, 0, true, false, 1, true>), G, B, 0, st, tab, list, n, g, zero); break;
    case 5: hipLaunchKernelGGL((lab_x2<NO, 0, true, false, 5, true>), G, B, 0, st, tab, list, n, g, zero); break;
    case 6: hipLaunchKernelGGL((lab_x2<NO, 0, true, false, 6, true>), G, B, 0, st, tab, list, n, g, zero); break;
    case 7: hipLaunchKernelGGL((lab_x2<NO, 0, true, false, 1, false, true>), G, B, 0, st, tab, list, n, g, zero); break;
    case 8: hipLaunchKernelGGL((lab_x2<NO, 0, true, false, 1, true, true>), G, B, 0, st, tab, list, n, g, zero); break;
    case 9: hipLaunchKernelGGL((lab_x2<NO, 0, true, false, 1, false, false, true>), G, B, 0, st, tab, list, n, g, zero); break;
    case 30: hipLaunchKernelGGL((lab_x2u<NO, 0>), G, B, 0, st, tab, list, n, g, zero); break;
    case 31: hipLaunchKernelGGL((lab_x2u<NO, 1>), G, B, 0, st, tab, list, n, g, zero); break;
    default: fprintf(stderr, "unknown variant %d\n", var); exit(1);
  }
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 6;
  const int var = argc > 2 ? atoi(argv[2]) : 0;
  const int reps = argc > 3 ? atoi(argv[3]) : 10;
  const bool lev_times = argc > 4 && atoi(argv[4]);
  if (K < 3 || K > 6) {
    fprintf(stderr, "K in [3, 6]\n");
    return 1;
  }
  int dev = 0;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, dev));
  g_grid_blocks = prop.multiProcessorCount * 8;
  PlaneGeom g{};
  g.no = K - 2;
  g.pow2 = 1;
  g.world = 1;
  uint64_t np = 1;
  for (int j = 0; j < K - 2; j++) {
    g.base[j] = 32;
    g.stride[j] = (uint32_t)np;
    g.shift[j] = __builtin_ctzll(np);
    np *= 32;
  }
  g.nplanes = (uint32_t)np;
  const int S = 31 * (K - 2);
  std::vector<uint32_t> cnt(S + 2, 0), off(S + 2, 0), list(np);
  auto osum = [&](uint64_t P) {
    int s = 0;
    for (int j = 0; j < K - 2; j++) {
      s += (int)(P % 32);
      P /= 32;
    }
    return s;
  };
  for (uint64_t P = 0; P < np; P++) cnt[osum(P)]++;
  for (int s = 0; s <= S; s++) off[s + 1] = off[s] + cnt[s];
  {
    std::vector<uint32_t> pos(off.begin(), off.end());
    for (uint64_t P = 0; P < np; P++) list[pos[osum(P)]++] = (uint32_t)P;
  }
  // LAB_ORDER=t (t > 1): within each level, planes in 3-D tiles of t^3 over
  // the outer digits above the lowest (tiles lexicographic, planes inside a
  // tile lexicographic); default: plane index order
  const int tile = getenv("LAB_ORDER") ? atoi(getenv("LAB_ORDER")) : 0;
  if (tile > 1) {
    auto key = [&](uint32_t P) {
      uint64_t k = 0;
      uint32_t d[6];
      for (int j = 0; j < K - 2; j++) d[j] = (P >> (5 * j)) & 31;
      for (int j = K - 3; j >= 1; j--) k = k * 64 + d[j] / tile;
      for (int j = K - 3; j >= 1; j--) k = k * 64 + d[j] % tile;
      return k * 64 + d[0];
    };
    for (int s = 0; s <= S; s++)
      std::sort(list.begin() + off[s], list.begin() + off[s + 1], [&](uint32_t a, uint32_t b) { return key(a) < key(b); });
  }
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
  if (var == 15) CK(hipMalloc(&g_stamps, 65536 * 6 * 8));
  std::vector<uint64_t> hst(65536 * 6);
  auto trace = [&](int s) {  // per-wave stamps of level s's launch (variant 15): first item's phases
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(hst.data(), g_stamps, hst.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> ph[5];  // start offset, list, fold, wavefront, (store + later items)
    uint64_t t0min = ~0ull, t4max = 0, multi = 0;
    for (uint32_t w = 0; w < 65536; w++) {
      const uint64_t* o = &hst[(size_t)w * 6];
      if (!o[5]) continue;
      t0min = std::min(t0min, o[0]);
      t4max = std::max(t4max, o[4]);
      multi += o[5] > 1;
    }
    for (uint32_t w = 0; w < 65536; w++) {
      const uint64_t* o = &hst[(size_t)w * 6];
      if (!o[5]) continue;
      ph[0].push_back((double)(o[0] - t0min));
      for (int k = 1; k < 5; k++) ph[k].push_back((double)(o[k] - o[k - 1]));
    }
    auto q = [](std::vector<double>& v, double f) {
      std::sort(v.begin(), v.end());
      return v[(size_t)std::min<double>(v.size() - 1, f * v.size())];
    };
    const char* nm[5] = {"start", "list", "fold", "wavefront", "store+rest"};
    printf("trace level %d: %u planes, %zu waves (%llu with >1 item), span %llu cycles;", s, cnt[s], ph[0].size(),
           (unsigned long long)multi, (unsigned long long)(t4max - t0min));
    for (int k = 0; k < 5; k++) printf(" %s p50 %.0f p90 %.0f max %.0f;", nm[k], q(ph[k], 0.5), q(ph[k], 0.9), q(ph[k], 1.0));
    printf("\n");
  };
  const char* tl = getenv("LAB_TRACE");  // levels to trace, "10,40,62"
  std::vector<int> traced;
  if (tl)
    for (const char* p = tl; *p;) {
      traced.push_back(atoi(p));
      while (*p && *p != ',') p++;
      if (*p) p++;
    }
  auto run = [&](int v, bool per_level) {
    for (int s = 0; s <= S; s++) {
      if (per_level || s == 0) CK(hipEventRecord(ev[s], st));
      const uint32_t n = cnt[s];
      const uint32_t* l = dlist + off[s];
      const bool tr = v == 15 && !per_level && std::find(traced.begin(), traced.end(), s) != traced.end();
      if (tr) CK(hipMemsetAsync(g_stamps, 0, 65536 * 6 * 8, st));
      switch (K) {
        case 3: launch<1>(v, tab, l, n, g, (const uint4*)zero, st); break;
        case 4: launch<2>(v, tab, l, n, g, (const uint4*)zero, st); break;
        case 5: launch<3>(v, tab, l, n, g, (const uint4*)zero, st); break;
        default: launch<4>(v, tab, l, n, g, (const uint4*)zero, st); break;
      }
      if (tr) trace(s);
    }
    CK(hipEventRecord(ev[S + 1], st));
  };
  // reference table: the round-3 step chain (lab kernel, LEAN = false,
  // bit-exact with the round-3 product kernel: profiles/r04a_plane_lab_diag.txt)
  std::vector<uint8_t> ref, got;
  if (var < 11 || var > 15) {
    run(10, false);
    CK(hipStreamSynchronize(st));
    ref.resize(tbytes);
    CK(hipMemcpy(ref.data(), tab, tbytes, hipMemcpyDeviceToHost));
  }
  std::vector<int> traced_keep;
  traced_keep.swap(traced);  // no tracing in the timed runs
  run(var, false);  // warm-up
  CK(hipStreamSynchronize(st));
  CK(hipGetLastError());
  std::vector<float> ts;
  for (int r = 0; r < reps; r++) {
    run(var, false);
    CK(hipEventSynchronize(ev[S + 1]));
    float ms;
    CK(hipEventElapsedTime(&ms, ev[0], ev[S + 1]));
    ts.push_back(ms);
  }
  float best = 1e9, sum = 0;
  for (float t : ts) {
    best = std::min(best, t);
    sum += t;
  }
  printf("var %d K=%d planes=%llu levels=%d backward best %.4f ms mean %.4f ms\n", var, K, (unsigned long long)np,
         S + 1, best, sum / reps);
  if (lev_times) {
    run(var, true);
    CK(hipStreamSynchronize(st));
    printf("level_us var %d:", var);
    double tot = 0;
    for (int s = 0; s <= S; s++) {
      float ms;
      CK(hipEventElapsedTime(&ms, ev[s], ev[s + 1]));
      tot += ms;
      printf(" %.1f", ms * 1e3);
    }
    printf("  (sum %.3f ms)\n", tot);
  }
  if (var == 15 && !traced_keep.empty()) {
    traced.swap(traced_keep);
    run(var, false);
    CK(hipStreamSynchronize(st));
  }
  if (!ref.empty() && var != 10) {
    got.resize(tbytes);
    CK(hipMemcpy(got.data(), tab, tbytes, hipMemcpyDeviceToHost));
    size_t bad = 0, first = ~(size_t)0;
    for (size_t i = 0; i < tbytes; i++)
      if (got[i] != ref[i]) {
        if (!bad) first = i;
        bad++;
      }
    printf("check var %d vs the round-3 chain: %zu differing bytes of %zu%s\n", var, bad, tbytes, bad ? " MISMATCH" : "");
    if (bad) {
      printf("first at %zu: got %02x want %02x\n", first, got[first], ref[first]);
      return 2;
    }
  }
  return 0;
}
