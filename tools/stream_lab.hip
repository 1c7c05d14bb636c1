// stream_lab.hip -- measurement harness for a STREAMED PLANES backward (one
// GPU, sum_four_to_one heaps 31^K, 8-bit absolute order-form words).
// Diagnostic tool, not product code.
//
// The product kernel (gm_plane.h, k_plane_resolve_x2) resolves a plane by a
// 63-step skewed wavefront in which lane h1 is busy for 32 steps only: lane
// h1 handles column t - h1 at step t.  Here each of a wave's four channels
// (lane half x 16-bit register half) resolves K planes of the SAME plane
// level back to back: lane h1 starts plane i+1 at the step after it finished
// plane i, so after the first plane every lane is busy at every step
// (32 (K + 1) steps for K planes instead of 63 K).  The step is the product
// chain plus two lane masks (a lane's first two columns of a plane must not
// see the previous plane's last two columns) and the lane-32 DPP guard.
//
// Window m = 32 consecutive steps.  At step j of window m lane L works on
// plane m (j >= L) or plane m - 1 (j < L); with rows rotated by L the byte it
// needs is byte j of the plane's row in either case, so the window's E row is
// one per-lane byte merge of the two planes' folded rows, and the results of
// plane m - 1 are the merge of windows m - 1 (j >= L) and m (j < L).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stream_lab.hip -o tools/stream_lab
//   ./tools/stream_lab K variant [reps] [level_times] [threshold]
// variants: 0 product kernel at every level; 2 / 4 / 8: the streamed kernel
// with K planes per channel at levels of >= threshold planes (default 4096),
// the product kernel below.
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

// bytes of a where m is set, of b elsewhere (v_bfi_b32; written so that no
// ~m is formed and hoisted out of the loops)
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}
// v where the lane's bit of the wave-uniform mask is set, else 0 (one
// v_cndmask against an SGPR pair)
__device__ __forceinline__ uint32_t lsel(uint64_t m, uint32_t v) {
  return __builtin_amdgcn_inverse_ballot_w64(m) ? v : 0u;
}

template <int NO, int K, int DIAG = 0>
__global__ __launch_bounds__(256, 3) void k_stream(uint8_t* __restrict__ tab, const uint32_t* __restrict__ list,
                                                uint32_t n, PlaneGeom g, const uint4* __restrict__ zero,
                                                uint8_t* __restrict__ dump) {
  static_assert(NO <= 4, "one neighbour digit per 8 steps");
  const uint32_t lane = threadIdx.x & 63, L = lane & 31, half = lane >> 5;
  const PlaneShare sh = plane_share(n, 4 * K);
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)tab, (short)0, (int)(g.nplanes * 1024u), 0x00020000);
  uint32_t m32 = lane == 32 ? 0u : 0xFFFFFFFFu;  // no row below row 0 of the upper channel pair
  asm volatile("" : "+v"(m32));  // (opaque: kept as a v_and the DPP move folds into)
  // byte j of dword d is plane m's (not plane m - 1's) when j >= L
  uint32_t mhi[8];
#pragma unroll
  for (int d = 0; d < 8; d++) {
    const int s = (int)L - 4 * d;
    mhi[d] = s <= 0 ? 0xFFFFFFFFu : (s >= 4 ? 0u : (0xFFFFFFFFu << (8 * s)));
  }
  for (uint32_t i0 = sh.first; i0 < sh.end; i0 += sh.stride) {
    // channel planes: X = entry i0 + 4 i + 2 half, Y = the next one (an
    // absent entry resolves the visit's first plane and stores nothing)
    auto entry = [&](int i, uint32_t& pX, uint32_t& pY, bool& lX, bool& lY) {
      const uint32_t ix = i0 + 4 * i + 2 * half, iy = ix + 1;
      lX = ix < sh.end;
      lY = iy < sh.end;
      pX = list[lX ? ix : i0];
      pY = list[lY ? iy : i0];
    };
    // external E of a plane pair: per neighbour digit j, the rows at k = 1,
    // 2 (zero rows when absent), folded in split form (odd bytes exact in
    // the high bytes of Xh / Yh, even bytes in the low bytes of Xl / Yl)
    // rows through a buffer resource: 32-bit offsets, an absent neighbour
    // reads 0 from an out-of-range offset
    struct Src {
      uint32_t x1, y1, x2, y2;
    };
    auto srcs = [&](uint32_t pX, uint32_t pY, bool real, int j) -> Src {
      const uint32_t djx = (pX >> g.shift[j]) & 31u, djy = (pY >> g.shift[j]) & 31u;
      const uint32_t ox = pX * 1024u + L * 32u, oy = pY * 1024u + L * 32u;
      const uint32_t st = g.stride[j] * 1024u;
      Src s;
      if (DIAG == 1) {  // diagnostic: the plane's own rows (cache-hot, results wrong)
        s.x1 = s.x2 = ox;
        s.y1 = s.y2 = oy;
        return s;
      }
      if (DIAG == 2) {  // diagnostic: no memory at all (out-of-range offsets read 0 without a fetch)
        s.x1 = s.x2 = s.y1 = s.y2 = 0xFFFFFFE0u;
        return s;
      }
      s.x1 = real && djx >= 1u ? ox - st : 0xFFFFFFE0u;
      s.y1 = real && djy >= 1u ? oy - st : 0xFFFFFFE0u;
      s.x2 = real && djx >= 2u ? ox - 2u * st : 0xFFFFFFE0u;
      s.y2 = real && djy >= 2u ? oy - 2u * st : 0xFFFFFFE0u;
      return s;
    };
    struct Rows {
      uint4 x1[2], y1[2], x2[2], y2[2];
    };
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    auto ld = [&](uint32_t off) -> uint4 {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
      return make_uint4(v.x, v.y, v.z, v.w);
    };
    auto load = [&](const Src& s) -> Rows {
      Rows r;
#pragma unroll
      for (int q = 0; q < 2; q++) {
        r.x1[q] = ld(s.x1 + 16u * q);
        r.y1[q] = ld(s.y1 + 16u * q);
        r.x2[q] = ld(s.x2 + 16u * q);
        r.y2[q] = ld(s.y2 + 16u * q);
      }
      return r;
    };
    uint32_t Xh[8], Xl[8], Yh[8], Yl[8];
    auto acc_zero = [&]() {
#pragma unroll
      for (int d = 0; d < 8; d++) Xh[d] = Xl[d] = Yh[d] = Yl[d] = 0;
    };
    auto fold = [&](const Rows& r) {
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const uint32_t a1[4] = {r.x1[q].x, r.x1[q].y, r.x1[q].z, r.x1[q].w};
        const uint32_t b1[4] = {r.y1[q].x, r.y1[q].y, r.y1[q].z, r.y1[q].w};
        const uint32_t a2[4] = {r.x2[q].x, r.x2[q].y, r.x2[q].z, r.x2[q].w};
        const uint32_t b2[4] = {r.y2[q].x, r.y2[q].y, r.y2[q].z, r.y2[q].w};
#pragma unroll
        for (int c = 0; c < 4; c++) {
          const int d = 4 * q + c;
          Xh[d] = pk_max16(pk_max16(Xh[d], a1[c]), a2[c]);
          Yh[d] = pk_max16(pk_max16(Yh[d], b1[c]), b2[c]);
          Xl[d] = pk_max3w<true>(Xl[d], a1[c] & 0x00FF00FFu, a2[c] & 0x00FF00FFu);
          Yl[d] = pk_max3w<true>(Yl[d], b1[c] & 0x00FF00FFu, b2[c] & 0x00FF00FFu);
        }
      }
    };
    uint32_t EwX[8], EwY[8];  // the window's merged E bytes
    uint32_t EpX[8], EpY[8];  // the last folded plane's E bytes (its low bytes feed the next merge)
    uint32_t WX[8], WY[8];    // results of the previous window, replaced dword by dword
    acc_zero();
    uint32_t cx, cy, nx_ = 0, ny_ = 0;  // planes of this window (m) and of the next (m + 1)
    bool clx, cly, nlx = false, nly = false;
    entry(0, cx, cy, clx, cly);
#pragma unroll
    for (int j = 0; j < NO; j++) fold(load(srcs(cx, cy, true, j)));
    if (K > 1) entry(1, nx_, ny_, nlx, nly);
#pragma unroll
    for (int d = 0; d < 8; d++) {
      EpX[d] = perm(Xh[d], Xl[d], 0x07020500u);  // bytes Xl.b0, Xh.b1, Xl.b2, Xh.b3
      EpY[d] = perm(Yh[d], Yl[d], 0x07020500u);
      EwX[d] = EpX[d];  // window 0: the lanes with j < L have no plane (their results are never used)
      EwY[d] = EpY[d];
      WX[d] = WY[d] = 0;
    }
    uint32_t cur = 0, prev = 0, u1p = 0;
    uint32_t px_prev = 0, py_prev = 0;
    bool plx_prev = false, ply_prev = false;
#pragma unroll 1
    for (int m = 0; m <= K; m++) {
      // plane m + 1 (if any) is folded during this window, one neighbour
      // digit per 8 steps; plane m - 1 (if any) is stored
      const bool more = m + 1 < K;
      const uint32_t qx = nx_, qy = ny_;
      // (window m stores plane m - 1: the previous window's plane)
      const uint32_t ox = px_prev, oy = py_prev;
      const bool sx = m >= 1 && plx_prev, sy = m >= 1 && ply_prev;
      // masks as opaque SGPR values per window: the compiler would hoist all
      // 64 step constants out of the window loop and spill them
      uint64_t zz = 0;
      asm volatile("" : "+s"(zz));
      uint4* dx = (uint4*)(sx ? tab + (size_t)ox * 1024u + L * 32u : dump + lane * 32u);
      uint4* dy = (uint4*)(sy ? tab + (size_t)oy * 1024u + L * 32u : dump + 2048u + lane * 32u);
      acc_zero();
      Rows rw;
      uint32_t rX[4], rY[4];
      uint32_t op[4];
#pragma unroll
      for (int j = 0; j < 32; j++) {
        if ((j & 7) == 0 && j / 8 < NO) rw = load(srcs(qx, qy, more, j / 8));
        const int d = j >> 2, b = j & 3;
        const uint32_t sel = 0x0C000C00u | ((4u + b) << 16) | (uint32_t)b;  // [X_b, 0, Y_b, 0]
        const uint32_t a = perm(EwY[d], EwX[d], sel);
        // lanes at column 0 (L == j) and 1 (L == j - 1) of their plane
        const uint64_t c0 = (1ull << j) | (1ull << (j + 32));
        const uint64_t c1 = (1ull << ((j + 31) & 31)) | (1ull << (((j + 31) & 31) + 32));
        const uint64_t kpv = ~(c0 | c1) ^ zz, kcv = ~c0 ^ zz;
        const uint32_t u2r = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)u1p, 0x138, 0xF, 0xF, true) & m32;
        const uint32_t pv = lsel(kpv, prev);
        const uint32_t pre = pk_max3w<true>(a, pv, u2r);
        const uint32_t u1r = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)cur, 0x138, 0xF, 0xF, true) & m32;
        const uint32_t cv = lsel(kcv, cur);
        const uint32_t mm = pk_max3w<true>(pre, cv, u1r);
        const uint32_t f = parent_x2<1>(mm);
        op[b] = f;
        if (b == 3) {
          const uint32_t t1 = perm(op[1], op[0], 0x06020400u);  // [X0 X1 Y0 Y1]
          const uint32_t t2 = perm(op[3], op[2], 0x06020400u);  // [X2 X3 Y2 Y3]
          const uint32_t wx = perm(t2, t1, 0x05040100u), wy = perm(t2, t1, 0x07060302u);
          // plane m - 1's row: bytes >= L from window m - 1, < L from window m
          rX[d & 3] = bsel(mhi[d], WX[d], wx);
          rY[d & 3] = bsel(mhi[d], WY[d], wy);
          WX[d] = wx;
          WY[d] = wy;
          if ((d & 3) == 3) {
            dx[d >> 2] = make_uint4(rX[0], rX[1], rX[2], rX[3]);
            dy[d >> 2] = make_uint4(rY[0], rY[1], rY[2], rY[3]);
          }
        }
        if ((j & 7) == 7 && j / 8 < NO) fold(rw);
        prev = cur;
        cur = f;
        u1p = u1r;
      }
      // next window: bytes >= L from plane m + 1, < L from plane m
#pragma unroll
      for (int d = 0; d < 8; d++) {
        const uint32_t nx = perm(Xh[d], Xl[d], 0x07020500u), ny = perm(Yh[d], Yl[d], 0x07020500u);
        EwX[d] = bsel(mhi[d], nx, EpX[d]);
        EwY[d] = bsel(mhi[d], ny, EpY[d]);
        EpX[d] = nx;
        EpY[d] = ny;
      }
      px_prev = cx, py_prev = cy, plx_prev = clx, ply_prev = cly;
      cx = nx_, cy = ny_, clx = nlx, cly = nly;
      if (m + 2 < K) entry(m + 2, nx_, ny_, nlx, nly);
    }
  }
}

// LEAN product form: the visit of k_plane_resolve_x2 (4 planes per wave,
// 63-step skewed wavefront, both phases unrolled) with the E rows in BYTE form
// after the fold (16 registers instead of 32) and the results packed four
// steps at a time (phase 0 -> P0, phase 1 merged into it by a per-lane byte
// mask: step q's result is row byte q in both phases, phase 0 owning bytes
// >= L) instead of 32 per-step registers: fewer VGPRs, more waves per SIMD.
// NB: neighbour digits per load batch (each digit = 8 x 16-B loads).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 bld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return make_uint4(v.x, v.y, v.z, v.w);
}
template <int NO, int MINW, int NB, bool STFULL = false>
__global__ __launch_bounds__(256, MINW) void k_lean(uint8_t* __restrict__ tab, const uint32_t* __restrict__ list,
                                                    uint32_t n, PlaneGeom g, const uint4* __restrict__ zero) {
  const uint32_t lane = threadIdx.x & 63, L = lane & 31;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)tab, (short)0, (int)(g.nplanes * 1024u), 0x00020000);
  const PlaneShare sh = plane_share(n, 4);
  for (uint32_t i0 = sh.first; i0 < sh.end; i0 += sh.stride) {
    const uint32_t ix = i0 + 2 * (lane >> 5), iy = ix + 1;
    const bool livex = ix < sh.end, livey = iy < sh.end;
    const uint32_t px = list[livex ? ix : i0], py = list[livey ? iy : i0];
    const size_t ox = (size_t)px * 1024u + L * 32u, oy = (size_t)py * 1024u + L * 32u;
    const uint32_t ox32 = (uint32_t)ox, oy32 = (uint32_t)oy;
    uint32_t Xh[8], Xl[8], Yh[8], Yl[8];
#pragma unroll
    for (int d = 0; d < 8; d++) Xh[d] = Xl[d] = Yh[d] = Yl[d] = 0;
#pragma unroll
    for (int j0 = 0; j0 < NO; j0 += NB) {
      // (a compiler barrier per batch: the loads of the next batch may not be
      // hoisted above this batch's fold, which would keep both in registers)
      if (j0) asm volatile("" ::: "memory");
      uint4 v[NB][8];
#pragma unroll
      for (int jj = 0; jj < NB; jj++) {
        const int j = j0 + jj;
        if (j >= NO) break;
        const uint32_t djx = (px >> g.shift[j]) & 31u, djy = (py >> g.shift[j]) & 31u;
        const uint32_t st = g.stride[j] * 1024u;
        const uint32_t o[4] = {djx >= 1u ? ox32 - st : 0xFFFFFFE0u, djy >= 1u ? oy32 - st : 0xFFFFFFE0u,
                               djx >= 2u ? ox32 - 2u * st : 0xFFFFFFE0u, djy >= 2u ? oy32 - 2u * st : 0xFFFFFFE0u};
#pragma unroll
        for (int r = 0; r < 4; r++) {
          v[jj][2 * r] = bld(rsrc, o[r]);
          v[jj][2 * r + 1] = bld(rsrc, o[r] + 16u);
        }
      }
#pragma unroll
      for (int jj = 0; jj < NB; jj++) {
        if (j0 + jj >= NO) break;
#pragma unroll
        for (int q = 0; q < 2; q++) {
          const uint32_t a1[4] = {v[jj][q].x, v[jj][q].y, v[jj][q].z, v[jj][q].w};
          const uint32_t b1[4] = {v[jj][2 + q].x, v[jj][2 + q].y, v[jj][2 + q].z, v[jj][2 + q].w};
          const uint32_t a2[4] = {v[jj][4 + q].x, v[jj][4 + q].y, v[jj][4 + q].z, v[jj][4 + q].w};
          const uint32_t b2[4] = {v[jj][6 + q].x, v[jj][6 + q].y, v[jj][6 + q].z, v[jj][6 + q].w};
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
      // the batch's fold is done before the next batch's loads issue: one
      // batch of rows in registers at a time
#define GM_PIN8(A) asm volatile("" : "+v"(A[0]), "+v"(A[1]), "+v"(A[2]), "+v"(A[3]), "+v"(A[4]), "+v"(A[5]), "+v"(A[6]), "+v"(A[7])::"memory")
      GM_PIN8(Xh);
      GM_PIN8(Xl);
      GM_PIN8(Yh);
      GM_PIN8(Yl);
#undef GM_PIN8
    }
    uint32_t EX[8], EY[8];
#pragma unroll
    for (int d = 0; d < 8; d++) {
      EX[d] = perm(Xh[d], Xl[d], 0x07020500u);
      EY[d] = perm(Yh[d], Yl[d], 0x07020500u);
    }
    const uint32_t primv = L == 0 ? ((px == 0 ? 0xFFu : 0u) | (py == 0 ? 0xFFu << 16 : 0u)) : 0u;
    uint32_t cur = 0, prev = 0, u1p = 0;
    uint32_t PX[8], PY[8], op[4];
    // an opaque copy of the row number per visit: the per-step masks below are
    // functions of the lane only, and the compiler would otherwise hoist all
    // of them out of the visit loop into registers (and spill)
    uint32_t Lv = L;
    asm volatile("" : "+v"(Lv));
    const uint32_t A0 = ~0u << Lv;  // bit q: row L is active at step q of phase 0
    auto phase = [&](auto PHc) {
      constexpr int PH = decltype(PHc)::value;
#pragma unroll
      for (int q = 0; q < 32; q++) {
        const int d = q >> 2, b = q & 3;
        const uint32_t sel = 0x0C000C00u | ((4u + b) << 16) | (uint32_t)b;  // [X_b, 0, Y_b, 0]
        const uint32_t a = perm(EY[d], EX[d], sel);
        const uint32_t u2r = from_lane_below(u1p);
        const uint32_t pre = pk_max3w<true>(a, prev, u2r);
        const uint32_t u1r = from_lane_below(cur);
        // phase 0: a row that has not started takes pre = 0xFF, whose parent is 0
        const uint32_t pre_ = PH == 0 ? ((__builtin_amdgcn_sbfe((int)A0, q, 1) != 0) ? pre : 0x00FF00FFu) : pre;
        const uint32_t m = pk_max3w<true>(pre_, cur, u1r);
        uint32_t f = parent_x2<1>(m);
        if (PH == 0 && q == 0) f = pk_max16(f, primv);
        op[b] = f;
        if (b == 3) {
          const uint32_t t1 = perm(op[1], op[0], 0x06020400u);
          const uint32_t t2 = perm(op[3], op[2], 0x06020400u);
          const uint32_t wx = perm(t2, t1, 0x05040100u), wy = perm(t2, t1, 0x07060302u);
          if (PH == 0) {
            PX[d] = wx;
            PY[d] = wy;
          } else {
            const int s = (int)Lv - 4 * d;  // phase 0 owns row bytes >= L
            const uint32_t mh = s <= 0 ? 0xFFFFFFFFu : (s >= 4 ? 0u : (0xFFFFFFFFu << (8 * s)));
            PX[d] = bsel(mh, PX[d], wx);
            PY[d] = bsel(mh, PY[d], wy);
          }
        }
        prev = cur;
        cur = f;
        u1p = u1r;
      }
    };
    phase(std::integral_constant<int, 0>());
    phase(std::integral_constant<int, 1>());
    if (STFULL) {
      // timing diagnostic (wrong layout): each store instruction writes whole
      // 128-B lines (a half-wave's 16-B pieces contiguous), halves of every
      // row 512 B apart
      if (livex) {
        uint4* p = (uint4*)(tab + (size_t)px * 1024u + L * 16u);
        p[0] = make_uint4(PX[0], PX[1], PX[2], PX[3]);
        p[32] = make_uint4(PX[4], PX[5], PX[6], PX[7]);
      }
      if (livey) {
        uint4* p = (uint4*)(tab + (size_t)py * 1024u + L * 16u);
        p[0] = make_uint4(PY[0], PY[1], PY[2], PY[3]);
        p[32] = make_uint4(PY[4], PY[5], PY[6], PY[7]);
      }
      continue;
    }
    if (livex) {
      uint4* p = (uint4*)(tab + ox);
      p[0] = make_uint4(PX[0], PX[1], PX[2], PX[3]);
      p[1] = make_uint4(PX[4], PX[5], PX[6], PX[7]);
    }
    if (livey) {
      uint4* p = (uint4*)(tab + oy);
      p[0] = make_uint4(PY[0], PY[1], PY[2], PY[3]);
      p[1] = make_uint4(PY[4], PY[5], PY[6], PY[7]);
    }
  }
}

static int g_grid_blocks = 2048;
static uint8_t* g_dump = nullptr;  // stores of absent planes (4 KiB)

template <int NO>
static void launch(int var, uint8_t* tab, const uint32_t* list, uint32_t n, const PlaneGeom& g, const uint4* zero,
                   hipStream_t st, uint32_t thr) {
  const int vk = var % 100, diag = var / 100;  // 1xx / 2xx: diagnostics of the streamed kernel
  const int KK = (vk == 2 || vk == 4 || vk == 8) && n >= thr ? vk : 1;
  const uint32_t waves = (n + 4 * KK - 1) / (4 * KK);
  uint32_t blocks = (waves + 3) / 4;
  blocks = std::min<uint32_t>((blocks + 7) / 8 * 8, (uint32_t)g_grid_blocks * 4);
  static const uint32_t cap = getenv("LAB_GRIDCAP") ? (uint32_t)atoi(getenv("LAB_GRIDCAP")) : 0u;
  if (cap) blocks = std::min(blocks, cap);  // fewer waves in flight: they loop (plane_share) over the level
  const dim3 G(blocks), B(256);
  switch (KK) {
    case 1:
      switch (vk) {  // 11..16: the lean form, minimum waves per SIMD 4 / 5 / 6, batches of 1 or 2 digits
        case 11: hipLaunchKernelGGL((k_lean<NO, 4, 2>), G, B, 0, st, tab, list, n, g, zero); break;
        case 12: hipLaunchKernelGGL((k_lean<NO, 5, 2>), G, B, 0, st, tab, list, n, g, zero); break;
        case 13: hipLaunchKernelGGL((k_lean<NO, 6, 2>), G, B, 0, st, tab, list, n, g, zero); break;
        case 14: hipLaunchKernelGGL((k_lean<NO, 4, 1>), G, B, 0, st, tab, list, n, g, zero); break;
        case 15: hipLaunchKernelGGL((k_lean<NO, 5, 1>), G, B, 0, st, tab, list, n, g, zero); break;
        case 16: hipLaunchKernelGGL((k_lean<NO, 6, 1>), G, B, 0, st, tab, list, n, g, zero); break;
        case 17: hipLaunchKernelGGL((k_lean<NO, 7, 1>), G, B, 0, st, tab, list, n, g, zero); break;
        case 18: hipLaunchKernelGGL((k_lean<NO, 8, 1>), G, B, 0, st, tab, list, n, g, zero); break;
        case 19: hipLaunchKernelGGL((k_lean<NO, 4, 1, true>), G, B, 0, st, tab, list, n, g, zero); break;
        default:
          hipLaunchKernelGGL((k_plane_resolve_x2<1, NO, false, 0>), G, B, 0, st, tab, (const void*)list, n, g, zero,
                             (const uint8_t*)nullptr, (uint8_t*)nullptr, (const uint32_t*)nullptr, 0u);
      }
      break;
    case 2: hipLaunchKernelGGL((k_stream<NO, 2>), G, B, 0, st, tab, list, n, g, zero, g_dump); break;
    case 4:
      if (diag == 1) hipLaunchKernelGGL((k_stream<NO, 4, 1>), G, B, 0, st, tab, list, n, g, zero, g_dump);
      else if (diag == 2) hipLaunchKernelGGL((k_stream<NO, 4, 2>), G, B, 0, st, tab, list, n, g, zero, g_dump);
      else hipLaunchKernelGGL((k_stream<NO, 4>), G, B, 0, st, tab, list, n, g, zero, g_dump);
      break;
    case 8: hipLaunchKernelGGL((k_stream<NO, 8>), G, B, 0, st, tab, list, n, g, zero, g_dump); break;
  }
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 6;
  const int var = argc > 2 ? atoi(argv[2]) : 0;
  const int reps = argc > 3 ? atoi(argv[3]) : 10;
  const bool lev_times = argc > 4 && atoi(argv[4]);
  const uint32_t thr = argc > 5 ? (uint32_t)atoi(argv[5]) : 4096u;
  if (K < 3 || K > 6) {
    fprintf(stderr, "K in [3, 6]\n");
    return 1;
  }
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
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
  // the product's tile order: planes in 8^3 tiles over the digits above the lowest
  {
    // LAB_ORDER=t: 3-D tiles of t^3 over the digits above the lowest; -1:
    // Morton (bit-interleaved) order of those digits; -2: Morton over all
    // four outer digits
    const int tile = getenv("LAB_ORDER") ? atoi(getenv("LAB_ORDER")) : 8;
    auto key = [&](uint32_t P) {
      uint64_t k = 0;
      uint32_t d[6];
      for (int j = 0; j < K - 2; j++) d[j] = (P >> (5 * j)) & 31;
      if (tile == -1 || tile == -2) {
        const int lo = tile == -1 ? 1 : 0;
        for (int b = 4; b >= 0; b--)
          for (int j = K - 3; j >= lo; j--) k = k * 2 + ((d[j] >> b) & 1);
        return tile == -1 ? k * 64 + d[0] : k;
      }
      for (int j = K - 3; j >= 1; j--) k = k * 64 + d[j] / tile;
      for (int j = K - 3; j >= 1; j--) k = k * 64 + d[j] % tile;
      return k * 64 + d[0];
    };
    if (tile > 1 || tile < 0)
      for (int s = 0; s <= S; s++)
        std::sort(list.begin() + off[s], list.begin() + off[s + 1],
                  [&](uint32_t a, uint32_t b) { return key(a) < key(b); });
  }
  const size_t tbytes = np * 1024;
  uint8_t* tab;
  void* zero;
  uint32_t* dlist;
  CK(hipMalloc(&tab, tbytes));
  CK(hipMalloc(&zero, 4096));
  CK(hipMalloc(&g_dump, 4096));
  CK(hipMemset(zero, 0, 4096));
  CK(hipMalloc(&dlist, np * 4));
  CK(hipMemcpy(dlist, list.data(), np * 4, hipMemcpyHostToDevice));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  std::vector<hipEvent_t> ev(S + 2);
  for (auto& evt : ev) CK(hipEventCreate(&evt));
  auto run = [&](int v, bool per_level) {
    for (int s = 0; s <= S; s++) {
      if (per_level || s == 0) CK(hipEventRecord(ev[s], st));
      const uint32_t n = cnt[s];
      const uint32_t* l = dlist + off[s];
      switch (K) {
        case 3: launch<1>(v, tab, l, n, g, (const uint4*)zero, st, thr); break;
        case 4: launch<2>(v, tab, l, n, g, (const uint4*)zero, st, thr); break;
        case 5: launch<3>(v, tab, l, n, g, (const uint4*)zero, st, thr); break;
        default: launch<4>(v, tab, l, n, g, (const uint4*)zero, st, thr); break;
      }
    }
    CK(hipEventRecord(ev[S + 1], st));
  };
  // reference table: the product kernel at every level
  std::vector<uint8_t> ref, got;
  if (var != 0 && var < 100) {
    CK(hipMemset(tab, 0x5A, tbytes));
    run(0, false);
    CK(hipStreamSynchronize(st));
    ref.resize(tbytes);
    CK(hipMemcpy(ref.data(), tab, tbytes, hipMemcpyDeviceToHost));
    CK(hipMemset(tab, 0xA5, tbytes));  // poison: every byte must be rewritten
  }
  run(var, false);  // warm-up (and the checked result)
  CK(hipStreamSynchronize(st));
  CK(hipGetLastError());
  if (!ref.empty()) {
    got.resize(tbytes);
    CK(hipMemcpy(got.data(), tab, tbytes, hipMemcpyDeviceToHost));
  }
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
  printf("var %d K=%d thr=%u planes=%llu levels=%d backward best %.4f ms mean %.4f ms\n", var, K, thr,
         (unsigned long long)np, S + 1, best, sum / reps);
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
  if (!ref.empty()) {
    size_t bad = 0, first = ~(size_t)0;
    for (size_t i = 0; i < tbytes; i++)
      if (got[i] != ref[i]) {
        if (!bad) first = i;
        bad++;
      }
    printf("check var %d vs the product kernel: %zu differing bytes of %zu%s\n", var, bad, tbytes,
           bad ? " MISMATCH" : "");
    if (bad) {
      printf("first at %zu (plane %zu row %zu byte %zu): got %02x want %02x\n", first, first / 1024, first / 32 % 32,
             first % 32, got[first], ref[first]);
      return 2;
    }
  }
  return 0;
}
