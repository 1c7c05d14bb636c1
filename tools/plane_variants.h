// tools/plane_variants.h -- measured-and-not-kept variants of the PLANES
// backward kernel (gamesmanmpi_amd/csrc/gm_plane.h), kept for the A/B harness
// tools/plane_proto.hip only; results in profiles/r03g_plane_ab.txt and
// DESIGN.md §2a.  Not part of the library.
#pragma once
#include "../gamesmanmpi_amd/csrc/gm_plane.h"

namespace gm {

// Lean packed form (8-bit words only): the wave shape and results of
// k_plane_resolve_x2, built for more waves per SIMD and a shorter per-step
// dependency chain (the wide levels are latency-bound: ~27 % VALU busy at
// 3 waves/SIMD, profiles/r03c_pmc):
//  * neighbour rows folded one at a time, the next one's loads in flight,
//    and the odd/even fold registers compressed back to raw bytes (v_perm)
//    before the wavefront: 8 dwords of E per plane instead of 16;
//  * results packed into row dwords every four steps (no 32-entry buffer);
//  * idle lanes are not masked after the parent map: they feed 0xFF into
//    the off-chain max (parent(0xFF) = 0), so the chain from one step's
//    result to the next is dpp -> select -> max -> parent.
template <int NO, bool SH>
__global__ __launch_bounds__(256, 5) void k_plane_resolve_x2l(uint8_t* __restrict__ tab,
                                                              const void* __restrict__ list, uint32_t n,
                                                              PlaneGeom g, const uint4* __restrict__ zero,
                                                              const uint8_t* __restrict__ recv,
                                                              uint8_t* __restrict__ send) {
  const uint32_t lane = threadIdx.x & 63, L = lane & 31;
  const bool l32 = lane == 32, l3132 = lane == 31 || lane == 32;
  const PlaneShare sh = plane_share(n, 4);
  for (uint32_t i0 = sh.first; i0 < sh.end; i0 += sh.stride) {
    const uint32_t ix = i0 + 2 * (lane >> 5), iy = ix + 1;
    const bool livex = ix < sh.end, livey = iy < sh.end;
    PlaneEntry ex, ey;
    if (SH) {
      ex = ((const PlaneEntry*)list)[livex ? ix : i0];
      ey = ((const PlaneEntry*)list)[livey ? iy : i0];
    } else {
      ex.p = ((const uint32_t*)list)[livex ? ix : i0];
      ey.p = ((const uint32_t*)list)[livey ? iy : i0];
    }
    uint32_t dx[NO > 0 ? NO : 1], dy[NO > 0 ? NO : 1];
    plane_digits<NO>(g, ex.p, dx);
    plane_digits<NO>(g, ey.p, dy);
    const size_t ox = (size_t)ex.p * 1024u + L * 32u, oy = (size_t)ey.p * 1024u + L * 32u;
    auto nb = [&](const PlaneEntry& e, const uint32_t* dig, size_t off, int j, int k) -> const uint4* {
      if (SH && j == NO - 1) {
        const uint32_t w = k == 1 ? e.top1 : e.top2;
        return w == kPlaneAbsent ? zero
               : w == kPlaneLocal ? (const uint4*)(tab + off - (size_t)k * g.Z * 1024u)
                                  : (const uint4*)(recv + (size_t)w * 1024u + L * 32u);
      }
      return dig[j] >= (uint32_t)k ? (const uint4*)(tab + off - (size_t)k * g.stride[j] * 1024u) : zero;
    };
    // E rows (odd bytes exact in Xh, even bytes in the high bytes of Xl)
    uint32_t Xh[8], Xl[8], Yh[8], Yl[8];
#pragma unroll
    for (int d = 0; d < 8; d++) Xh[d] = Xl[d] = Yh[d] = Yl[d] = 0;
    uint4 vx[2], vy[2];
    if (NO > 0) {
      const uint4 *sx = nb(ex, dx, ox, 0, 1), *sy = nb(ey, dy, oy, 0, 1);
      vx[0] = sx[0], vx[1] = sx[1], vy[0] = sy[0], vy[1] = sy[1];
    }
#pragma unroll
    for (int t = 0; t < 2 * NO; t++) {
      uint4 wx[2], wy[2];
      if (t + 1 < 2 * NO) {
        const int j = (t + 1) >> 1, k = 1 + ((t + 1) & 1);
        const uint4 *sx = nb(ex, dx, ox, j, k), *sy = nb(ey, dy, oy, j, k);
        wx[0] = sx[0], wx[1] = sx[1], wy[0] = sy[0], wy[1] = sy[1];
      }
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const uint32_t a[4] = {vx[q].x, vx[q].y, vx[q].z, vx[q].w};
        const uint32_t b[4] = {vy[q].x, vy[q].y, vy[q].z, vy[q].w};
#pragma unroll
        for (int c = 0; c < 4; c++) {
          Xh[4 * q + c] = pk_max16(Xh[4 * q + c], a[c]);
          Xl[4 * q + c] = pk_max16(Xl[4 * q + c], pk_shl8(a[c]));
          Yh[4 * q + c] = pk_max16(Yh[4 * q + c], b[c]);
          Yl[4 * q + c] = pk_max16(Yl[4 * q + c], pk_shl8(b[c]));
        }
      }
      if (t + 1 < 2 * NO) {
        vx[0] = wx[0], vx[1] = wx[1], vy[0] = wy[0], vy[1] = wy[1];
      }
    }
    uint32_t EX[8], EY[8];  // raw E bytes: byte q of dword q / 4
#pragma unroll
    for (int d = 0; d < 8; d++) {
      EX[d] = perm(Xh[d], Xl[d], 0x07030501u);
      EY[d] = perm(Yh[d], Yl[d], 0x07030501u);
    }
    const uint32_t primv = (g.rank == 0 && L == 0) ? ((ex.p == 0 ? 0xFFu : 0u) | (ey.p == 0 ? 0xFF0000u : 0u)) : 0u;
    uint32_t cur = 0, prev = 0, u1p = 0;
    uint32_t RX[8], RY[8];
#pragma unroll
    for (int d = 0; d < 8; d++) RX[d] = RY[d] = 0;
#pragma unroll 1
    for (uint32_t ph = 0; ph < 2; ph++) {
      const uint32_t flip = ph ? 0xFFFFFFFFu : 0u;
      uint32_t f4[4];
#pragma unroll
      for (int q = 0; q < 32; q++) {
        const int d = q >> 2, b = q & 3;
        const uint32_t a = perm(EY[d], EX[d], 0x0C000C00u | ((4u + b) << 16) | (uint32_t)b);  // [X_q, Y_q]
        const uint32_t u1r = from_lane_below(cur), u2r = from_lane_below(u1p);
        // idle rows of this step: phase 0 rows q+1..31, phase 1 rows 0..q
        const uint32_t im = ~((uint32_t)(q == 31 ? 0xFFFFFFFFull : ((2ull << q) - 1)) ^ flip);
        const uint32_t idle = 0x00FF00FFu & (uint32_t)__builtin_amdgcn_sbfe((int)im, (int)L, 1);
        const uint32_t e = pk_max16(pk_max16(pk_max16(a, prev), u2r), idle);  // lane 32: u2r = 0 (lane 31's u1p)
        const uint32_t u1 = l32 ? 0u : u1r;
        uint32_t f = parent_x2<1>(pk_max16(pk_max16(cur, e), u1));
        if (q == 0) f = pk_max16(f, ph ? 0u : primv);
        prev = cur;
        cur = f;
        u1p = l3132 ? 0u : u1r;
        f4[b] = f;
        if (b == 3) {
          const uint32_t t1 = perm(f4[1], f4[0], 0x06020400u), t2 = perm(f4[3], f4[2], 0x06020400u);
          RX[d] |= perm(t2, t1, 0x05040100u);
          RY[d] |= perm(t2, t1, 0x07060302u);
        }
      }
    }
    auto store = [&](uint8_t* dst, const uint32_t* o) {
      uint4* p = (uint4*)dst;
      p[0] = make_uint4(o[0], o[1], o[2], o[3]);
      p[1] = make_uint4(o[4], o[5], o[6], o[7]);
    };
    if (livex) {
      store(tab + ox, RX);
      if (SH && ex.send != kPlaneAbsent) store(send + (size_t)ex.send * 1024u + L * 32u, RX);
    }
    if (livey) {
      store(tab + oy, RY);
      if (SH && ey.send != kPlaneAbsent) store(send + (size_t)ey.send * 1024u + L * 32u, RY);
    }
  }
}

// One skewed-wavefront step of the packed 8-bit kernels: results of planes
// X / Y in the low bytes of the two 16-bit halves.  Step q of phase PH
// (0: rows 0..q active, 1: rows q+1..31 active); idle rows feed 0xFF into
// the off-chain max and so produce 0 (parent(0xFF) = 0); lane 32 (row 0 of
// the upper plane pair) takes nothing from lane 31, lane 33 nothing two
// rows down (u1p is zeroed on lanes 31 and 32).
struct PlaneChain {
  uint32_t cur, prev, u1p;
};
__device__ __forceinline__ uint32_t plane_step8(PlaneChain& c, uint32_t a, int q, int ph, uint32_t L, bool l32,
                                                bool l3132, uint32_t primv) {
  const uint32_t u1r = from_lane_below(c.cur), u2r = from_lane_below(c.u1p);
  const uint32_t act = q == 31 ? 0xFFFFFFFFu : ((2u << q) - 1u);
  const uint32_t im = ph ? act : ~act;
  const uint32_t idle = 0x00FF00FFu & (uint32_t)__builtin_amdgcn_sbfe((int)im, (int)L, 1);
  const uint32_t e = pk_max16(pk_max16(pk_max16(a, c.prev), u2r), idle);
  const uint32_t u1 = l32 ? 0u : u1r;
  uint32_t f = parent_x2<1>(pk_max16(pk_max16(c.cur, e), u1));
  if (q == 0 && ph == 0) f = pk_max16(f, primv);
  c.prev = c.cur;
  c.cur = f;
  c.u1p = l3132 ? 0u : u1r;
  return f;
}
// byte q of the raw E rows of X and Y -> [X_q, 0, Y_q, 0]
__device__ __forceinline__ uint32_t plane_e8(const uint32_t* EX, const uint32_t* EY, int q) {
  const int d = q >> 2, b = q & 3;
  return perm(EY[d], EX[d], 0x0C000C00u | ((4u + b) << 16) | (uint32_t)b);
}
// four packed step results -> the X and Y row dwords they fill
__device__ __forceinline__ void plane_pack8(const uint32_t* f4, uint32_t& rx, uint32_t& ry) {
  const uint32_t t1 = perm(f4[1], f4[0], 0x06020400u), t2 = perm(f4[3], f4[2], 0x06020400u);
  rx |= perm(t2, t1, 0x05040100u);
  ry |= perm(t2, t1, 0x07060302u);
}
// fold the 16-B loads of every neighbour row half into raw E dwords
template <int NN>
__device__ __forceinline__ void plane_fold_half8(const uint4* v, uint32_t* E) {
  uint32_t h[4] = {0, 0, 0, 0}, l[4] = {0, 0, 0, 0};
#pragma unroll
  for (int t = 0; t < NN; t++) {
    const uint32_t a[4] = {v[t].x, v[t].y, v[t].z, v[t].w};
#pragma unroll
    for (int c = 0; c < 4; c++) {
      h[c] = pk_max16(h[c], a[c]);          // odd bytes exact
      l[c] = pk_max16(l[c], pk_shl8(a[c]));  // even bytes, exact in the high bytes
    }
  }
#pragma unroll
  for (int c = 0; c < 4; c++) E[c] = perm(h[c], l[c], 0x07030501u);
}

// Half-split packed form (8-bit words; the default): k_plane_resolve_x2's
// wave shape and results, with the neighbour rows fetched in two halves.
// The first 16 bytes of every neighbour row (E bytes 0..15) are loaded and
// folded, then the second halves are issued and stay in flight during the
// first 16 wavefront steps, which need only bytes 0..15 -- all loads of a
// half in flight at once (one memory round before the wavefront instead of
// the whole fetch), in <= 128 VGPRs (4 waves / SIMD instead of 3).  Phase 1
// stops at step 30 (step 31 has no active row).
// DIAG (diagnostic builds only, tools/plane_proto.hip): 1 = no neighbour
// loads (E = 0), 2 = no wavefront (the folded E rows are stored)
template <int NO, bool SH, int DIAG = 0>
__global__ __launch_bounds__(256, 4) void k_plane_resolve_x2h(uint8_t* __restrict__ tab,
                                                              const void* __restrict__ list, uint32_t n,
                                                              PlaneGeom g, const uint4* __restrict__ zero,
                                                              const uint8_t* __restrict__ recv,
                                                              uint8_t* __restrict__ send) {
  constexpr int NN = NO > 0 ? 2 * NO : 1;
  const uint32_t lane = threadIdx.x & 63, L = lane & 31;
  const bool l32 = lane == 32, l3132 = lane == 31 || lane == 32;
  const PlaneShare sh = plane_share(n, 4);
  for (uint32_t i0 = sh.first; i0 < sh.end; i0 += sh.stride) {
    const uint32_t ix = i0 + 2 * (lane >> 5), iy = ix + 1;
    const bool livex = ix < sh.end, livey = iy < sh.end;
    PlaneEntry ex, ey;
    if (SH) {
      ex = ((const PlaneEntry*)list)[livex ? ix : i0];
      ey = ((const PlaneEntry*)list)[livey ? iy : i0];
    } else {
      ex.p = ((const uint32_t*)list)[livex ? ix : i0];
      ey.p = ((const uint32_t*)list)[livey ? iy : i0];
    }
    uint32_t dx[NO > 0 ? NO : 1], dy[NO > 0 ? NO : 1];
    plane_digits<NO>(g, ex.p, dx);
    plane_digits<NO>(g, ey.p, dy);
    const size_t ox = (size_t)ex.p * 1024u + L * 32u, oy = (size_t)ey.p * 1024u + L * 32u;
    auto nb = [&](const PlaneEntry& e, const uint32_t* dig, size_t off, int j, int k) -> const uint4* {
      if (SH && j == NO - 1) {
        const uint32_t w = k == 1 ? e.top1 : e.top2;
        return w == kPlaneAbsent ? zero
               : w == kPlaneLocal ? (const uint4*)(tab + off - (size_t)k * g.Z * 1024u)
                                  : (const uint4*)(recv + (size_t)w * 1024u + L * 32u);
      }
      return dig[j] >= (uint32_t)k ? (const uint4*)(tab + off - (size_t)k * g.stride[j] * 1024u) : zero;
    };
    uint4 vx[NN], vy[NN];
    uint32_t EX[8], EY[8];
#pragma unroll
    for (int t = 0; t < NN; t++) {
      vx[t] = NO > 0 && DIAG != 1 ? nb(ex, dx, ox, t >> 1, 1 + (t & 1))[0] : make_uint4(0, 0, 0, 0);
      vy[t] = NO > 0 && DIAG != 1 ? nb(ey, dy, oy, t >> 1, 1 + (t & 1))[0] : make_uint4(0, 0, 0, 0);
    }
    plane_fold_half8<NN>(vx, EX);
    plane_fold_half8<NN>(vy, EY);
    // the second halves' addresses are recomputed from the plane offsets
    // (an opaque copy stops the compiler from keeping the first halves' 16
    // pointers live across the fold: 32 VGPRs)
    size_t ox2 = ox, oy2 = oy;
    asm volatile("" : "+v"(ox2), "+v"(oy2) : "v"(EX[3]), "v"(EY[3]));  // after the fold
#pragma unroll
    for (int t = 0; t < NN; t++) {
      vx[t] = NO > 0 && DIAG != 1 ? nb(ex, dx, ox2, t >> 1, 1 + (t & 1))[1] : make_uint4(0, 0, 0, 0);
      vy[t] = NO > 0 && DIAG != 1 ? nb(ey, dy, oy2, t >> 1, 1 + (t & 1))[1] : make_uint4(0, 0, 0, 0);
    }
    const uint32_t primv = (g.rank == 0 && L == 0) ? ((ex.p == 0 ? 0xFFu : 0u) | (ey.p == 0 ? 0xFF0000u : 0u)) : 0u;
    PlaneChain c{0, 0, 0};
    uint32_t RX[8], RY[8], f4[4];
#pragma unroll
    for (int d = 0; d < 8; d++) RX[d] = RY[d] = 0;
    // an opaque copy of the row number per section: the 63 idle-row masks
    // depend on it alone and would otherwise be hoisted out of the plane
    // loop into 63 live VGPRs
    uint32_t Lv = L;
    asm volatile("" : "+v"(Lv));
#pragma unroll
    for (int q = 0; q < 16; q++) {
      f4[q & 3] = plane_step8(c, plane_e8(EX, EY, q), q, 0, Lv, l32, l3132, primv);
      if ((q & 3) == 3) plane_pack8(f4, RX[q >> 2], RY[q >> 2]);
    }
    plane_fold_half8<NN>(vx, EX + 4);
    plane_fold_half8<NN>(vy, EY + 4);
    Lv = L;
    asm volatile("" : "+v"(Lv));
#pragma unroll
    for (int q = 16; q < 32; q++) {
      f4[q & 3] = plane_step8(c, plane_e8(EX, EY, q), q, 0, Lv, l32, l3132, primv);
      if ((q & 3) == 3) plane_pack8(f4, RX[q >> 2], RY[q >> 2]);
    }
    Lv = L;
    asm volatile("" : "+v"(Lv));
#pragma unroll
    for (int q = 0; q < 31; q++) {
      f4[q & 3] = plane_step8(c, plane_e8(EX, EY, q), q, 1, Lv, l32, l3132, primv);
      if ((q & 3) == 3) plane_pack8(f4, RX[q >> 2], RY[q >> 2]);
    }
    f4[3] = 0;
    plane_pack8(f4, RX[7], RY[7]);
    if (DIAG == 2) {
#pragma unroll
      for (int d = 0; d < 8; d++) RX[d] = EX[d], RY[d] = EY[d];
    }
    auto store = [&](uint8_t* dst, const uint32_t* o) {
      uint4* p = (uint4*)dst;
      p[0] = make_uint4(o[0], o[1], o[2], o[3]);
      p[1] = make_uint4(o[4], o[5], o[6], o[7]);
    };
    if (livex) {
      store(tab + ox, RX);
      if (SH && ex.send != kPlaneAbsent) store(send + (size_t)ex.send * 1024u + L * 32u, RX);
    }
    if (livey) {
      store(tab + oy, RY);
      if (SH && ey.send != kPlaneAbsent) store(send + (size_t)ey.send * 1024u + L * 32u, RY);
    }
  }
}

template <int NO, bool SH, int DIAG = 0>
__global__ __launch_bounds__(256, 3) void k_plane_resolve_x2f(uint8_t* __restrict__ tab,
                                                              const void* __restrict__ list, uint32_t n,
                                                              PlaneGeom g, const uint4* __restrict__ zero,
                                                              const uint8_t* __restrict__ recv,
                                                              uint8_t* __restrict__ send) {
  constexpr int NN = NO > 0 ? 2 * NO : 1;
  const uint32_t lane = threadIdx.x & 63, L = lane & 31;
  const bool l32 = lane == 32, l3132 = lane == 31 || lane == 32;
  const PlaneShare sh = plane_share(n, 4);
  for (uint32_t i0 = sh.first; i0 < sh.end; i0 += sh.stride) {
    const uint32_t ix = i0 + 2 * (lane >> 5), iy = ix + 1;
    const bool livex = ix < sh.end, livey = iy < sh.end;
    PlaneEntry ex, ey;
    if (SH) {
      ex = ((const PlaneEntry*)list)[livex ? ix : i0];
      ey = ((const PlaneEntry*)list)[livey ? iy : i0];
    } else {
      ex.p = ((const uint32_t*)list)[livex ? ix : i0];
      ey.p = ((const uint32_t*)list)[livey ? iy : i0];
    }
    uint32_t dx[NO > 0 ? NO : 1], dy[NO > 0 ? NO : 1];
    plane_digits<NO>(g, ex.p, dx);
    plane_digits<NO>(g, ey.p, dy);
    const size_t ox = (size_t)ex.p * 1024u + L * 32u, oy = (size_t)ey.p * 1024u + L * 32u;
    auto nb = [&](const PlaneEntry& e, const uint32_t* dig, size_t off, int j, int k) -> const uint4* {
      if (SH && j == NO - 1) {
        const uint32_t w = k == 1 ? e.top1 : e.top2;
        return w == kPlaneAbsent ? zero
               : w == kPlaneLocal ? (const uint4*)(tab + off - (size_t)k * g.Z * 1024u)
                                  : (const uint4*)(recv + (size_t)w * 1024u + L * 32u);
      }
      return dig[j] >= (uint32_t)k ? (const uint4*)(tab + off - (size_t)k * g.stride[j] * 1024u) : zero;
    };
    uint4 vx[NN], vy[NN], wx[NN], wy[NN];
    uint32_t EX[8], EY[8];
#pragma unroll
    for (int t = 0; t < NN; t++) {
      const uint4* sx = NO > 0 && DIAG != 1 ? nb(ex, dx, ox, t >> 1, 1 + (t & 1)) : zero;
      const uint4* sy = NO > 0 && DIAG != 1 ? nb(ey, dy, oy, t >> 1, 1 + (t & 1)) : zero;
      vx[t] = sx[0], wx[t] = sx[1], vy[t] = sy[0], wy[t] = sy[1];
    }
    plane_fold_half8<NN>(vx, EX);
    plane_fold_half8<NN>(vy, EY);
    plane_fold_half8<NN>(wx, EX + 4);
    plane_fold_half8<NN>(wy, EY + 4);
    const uint32_t primv = (g.rank == 0 && L == 0) ? ((ex.p == 0 ? 0xFFu : 0u) | (ey.p == 0 ? 0xFF0000u : 0u)) : 0u;
    PlaneChain c{0, 0, 0};
    uint32_t RX[8], RY[8], f4[4];
#pragma unroll
    for (int d = 0; d < 8; d++) RX[d] = RY[d] = 0;
    // an opaque copy of the row number per section: the 63 idle-row masks
    // depend on it alone and would otherwise be hoisted out of the plane
    // loop into 63 live VGPRs
    uint32_t Lv = L;
    asm volatile("" : "+v"(Lv));
#pragma unroll
    for (int q = 0; q < 16; q++) {
      f4[q & 3] = plane_step8(c, plane_e8(EX, EY, q), q, 0, Lv, l32, l3132, primv);
      if ((q & 3) == 3) plane_pack8(f4, RX[q >> 2], RY[q >> 2]);
    }
    Lv = L;
    asm volatile("" : "+v"(Lv));
#pragma unroll
    for (int q = 16; q < 32; q++) {
      f4[q & 3] = plane_step8(c, plane_e8(EX, EY, q), q, 0, Lv, l32, l3132, primv);
      if ((q & 3) == 3) plane_pack8(f4, RX[q >> 2], RY[q >> 2]);
    }
    Lv = L;
    asm volatile("" : "+v"(Lv));
#pragma unroll
    for (int q = 0; q < 31; q++) {
      f4[q & 3] = plane_step8(c, plane_e8(EX, EY, q), q, 1, Lv, l32, l3132, primv);
      if ((q & 3) == 3) plane_pack8(f4, RX[q >> 2], RY[q >> 2]);
    }
    f4[3] = 0;
    plane_pack8(f4, RX[7], RY[7]);
    if (DIAG == 2) {
#pragma unroll
      for (int d = 0; d < 8; d++) RX[d] = EX[d], RY[d] = EY[d];
    }
    auto store = [&](uint8_t* dst, const uint32_t* o) {
      uint4* p = (uint4*)dst;
      p[0] = make_uint4(o[0], o[1], o[2], o[3]);
      p[1] = make_uint4(o[4], o[5], o[6], o[7]);
    };
    if (livex) {
      store(tab + ox, RX);
      if (SH && ex.send != kPlaneAbsent) store(send + (size_t)ex.send * 1024u + L * 32u, RX);
    }
    if (livey) {
      store(tab + oy, RY);
      if (SH && ey.send != kPlaneAbsent) store(send + (size_t)ey.send * 1024u + L * 32u, RY);
    }
  }
}

// k_plane_resolve_x2 held to 4 waves / SIMD (<= 128 VGPRs)
template <int WB, int NO, bool SH>
__global__ __launch_bounds__(256, 4) void k_plane_resolve_x2b(typename PlaneWord<WB>::T* __restrict__ tab,
                                                          const void* __restrict__ list, uint32_t n, PlaneGeom g,
                                                          const uint4* __restrict__ zero,
                                                          const typename PlaneWord<WB>::T* __restrict__ recv,
                                                          typename PlaneWord<WB>::T* __restrict__ send) {
  typedef PlaneWord<WB> W;
  typedef typename W::T T;
  constexpr int DW = W::DW, NQ = DW / 4;
  const uint32_t lane = threadIdx.x & 63, L = lane & 31;
  const bool l32 = lane == 32;
  const PlaneShare sh = plane_share(n, 4);
  for (uint32_t i0 = sh.first; i0 < sh.end; i0 += sh.stride) {
    const uint32_t ix = i0 + 2 * (lane >> 5), iy = ix + 1;
    const bool livex = ix < sh.end, livey = iy < sh.end;
    PlaneEntry ex, ey;
    if (SH) {
      ex = ((const PlaneEntry*)list)[livex ? ix : i0];
      ey = ((const PlaneEntry*)list)[livey ? iy : i0];
    } else {
      ex.p = ((const uint32_t*)list)[livex ? ix : i0];
      ey.p = ((const uint32_t*)list)[livey ? iy : i0];
    }
    uint32_t dx[NO > 0 ? NO : 1], dy[NO > 0 ? NO : 1];
    plane_digits<NO>(g, ex.p, dx);
    plane_digits<NO>(g, ey.p, dy);
    const size_t ox = (size_t)ex.p * 1024u + L * 32u, oy = (size_t)ey.p * 1024u + L * 32u;
    // E rows of both planes (8-bit: odd bytes exact in Ehi, even bytes in
    // the high bytes of Elo; 16-bit: Ehi exact)
    uint32_t Xh[DW], Xl[WB == 1 ? DW : 1], Yh[DW], Yl[WB == 1 ? DW : 1];
#pragma unroll
    for (int d = 0; d < DW; d++) {
      Xh[d] = Yh[d] = 0;
      if (WB == 1) Xl[d] = Yl[d] = 0;
    }
    auto nb = [&](const PlaneEntry& e, const uint32_t* dig, size_t off, int j, int k) -> const uint4* {
      if (SH && j == NO - 1) {
        const uint32_t w = k == 1 ? e.top1 : e.top2;
        return w == kPlaneAbsent ? zero
               : w == kPlaneLocal ? (const uint4*)(tab + off - (size_t)k * g.Z * 1024u)
                                  : (const uint4*)(recv + (size_t)w * 1024u + L * 32u);
      }
      return dig[j] >= (uint32_t)k ? (const uint4*)(tab + off - (size_t)k * g.stride[j] * 1024u) : zero;
    };
#pragma unroll
    for (int j = 0; j < NO; j++) {
#pragma unroll
      for (int k = 1; k <= 2; k++) {
        const uint4* sx = nb(ex, dx, ox, j, k);
        const uint4* sy = nb(ey, dy, oy, j, k);
        uint4 vx[NQ], vy[NQ];
#pragma unroll
        for (int q = 0; q < NQ; q++) {
          vx[q] = sx[q];
          vy[q] = sy[q];
        }
#pragma unroll
        for (int q = 0; q < NQ; q++) {
          const uint32_t a[4] = {vx[q].x, vx[q].y, vx[q].z, vx[q].w};
          const uint32_t b[4] = {vy[q].x, vy[q].y, vy[q].z, vy[q].w};
#pragma unroll
          for (int c = 0; c < 4; c++) {
            Xh[4 * q + c] = pk_max16(Xh[4 * q + c], a[c]);
            Yh[4 * q + c] = pk_max16(Yh[4 * q + c], b[c]);
            if (WB == 1) {
              Xl[4 * q + c] = pk_max16(Xl[4 * q + c], pk_shl8(a[c]));
              Yl[4 * q + c] = pk_max16(Yl[4 * q + c], pk_shl8(b[c]));
            }
          }
        }
      }
    }
    const uint32_t primv =
        (g.rank == 0 && L == 0) ? ((ex.p == 0 ? W::kPrim : 0u) | (ey.p == 0 ? W::kPrim << 16 : 0u)) : 0u;
    // step q's results of both planes stay packed [X | Y] in op[q] (OR of
    // the two phases: an idle lane contributes 0) and are unpacked into the
    // two rows once, after the wavefront
    uint32_t cur = 0, prev = 0, u1p = 0;
    uint32_t op[32];
#pragma unroll
    for (int q = 0; q < 32; q++) op[q] = 0;
#pragma unroll 1
    for (uint32_t ph = 0; ph < 2; ph++) {
      const uint32_t flip = ph ? 0xFFFFFFFFu : 0u;
#pragma unroll
      for (int q = 0; q < 32; q++) {
        uint32_t a;
        if (WB == 1) {
          // byte q of X's and Y's E rows -> [X, 0, Y, 0]
          const int d = q >> 2, b = q & 3;
          const uint32_t bx = (b & 1) ? (uint32_t)b : (uint32_t)b + 1;  // byte inside the split dword
          const uint32_t sel = 0x0C000C00u | ((4u + bx) << 16) | bx;     // hi = Y (bytes 4-7), lo = X
          a = (b & 1) ? perm(Yh[d], Xh[d], sel) : perm(Yl[d], Xl[d], sel);
        } else {
          const int d = q >> 1, h = q & 1;
          const uint32_t b0 = 2 * h;
          const uint32_t sel = ((5u + b0) << 24) | ((4u + b0) << 16) | ((1u + b0) << 8) | b0;
          a = perm(Yh[d], Xh[d], sel);
        }
        const uint32_t u1r = from_lane_below(cur), u2r = from_lane_below(u1p);
        uint32_t m = pk_max16(pk_max16(a, cur), prev);
        const uint32_t m2 = pk_max16(pk_max16(m, u1r), u2r);
        m = l32 ? m : m2;  // row 0 of the upper pair has no row below
        const uint32_t am = (uint32_t)(q == 31 ? 0xFFFFFFFFull : ((2ull << q) - 1)) ^ flip;
        uint32_t f = keep_rows(am, L, parent_x2<WB>(m));
        if (q == 0) f = pk_max16(f, ph ? 0u : primv);
        op[q] |= f;
        prev = cur;
        cur = f;
        u1p = l32 ? 0u : u1r;
      }
    }
    uint32_t ox_[DW], oy_[DW];
    if (WB == 1) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint32_t t1 = perm(op[4 * k + 1], op[4 * k], 0x06020400u);      // [X0 X1 Y0 Y1]
        const uint32_t t2 = perm(op[4 * k + 3], op[4 * k + 2], 0x06020400u);  // [X2 X3 Y2 Y3]
        ox_[k] = perm(t2, t1, 0x05040100u);
        oy_[k] = perm(t2, t1, 0x07060302u);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 16; k++) {
        ox_[k] = perm(op[2 * k + 1], op[2 * k], 0x05040100u);
        oy_[k] = perm(op[2 * k + 1], op[2 * k], 0x07060302u);
      }
    }
    auto store = [&](T* dst, const uint32_t* o) {
      uint4* p = (uint4*)dst;
#pragma unroll
      for (int q = 0; q < NQ; q++) p[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
    };
    if (livex) {
      store(tab + ox, ox_);
      if (SH && ex.send != kPlaneAbsent) store(send + (size_t)ex.send * 1024u + L * 32u, ox_);
    }
    if (livey) {
      store(tab + oy, oy_);
      if (SH && ey.send != kPlaneAbsent) store(send + (size_t)ey.send * 1024u + L * 32u, oy_);
    }
  }
}

// k_plane_resolve_x2 with a plain grid-stride share (no XCD chunking of the level list)
template <int WB, int NO, bool SH>
__global__ __launch_bounds__(256) void k_plane_resolve_x2d(typename PlaneWord<WB>::T* __restrict__ tab,
                                                          const void* __restrict__ list, uint32_t n, PlaneGeom g,
                                                          const uint4* __restrict__ zero,
                                                          const typename PlaneWord<WB>::T* __restrict__ recv,
                                                          typename PlaneWord<WB>::T* __restrict__ send) {
  typedef PlaneWord<WB> W;
  typedef typename W::T T;
  constexpr int DW = W::DW, NQ = DW / 4;
  const uint32_t lane = threadIdx.x & 63, L = lane & 31;
  const bool l32 = lane == 32;
  const uint32_t gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const PlaneShare sh{gw * 4u, n, gridDim.x * (blockDim.x >> 6) * 4u};
  for (uint32_t i0 = sh.first; i0 < sh.end; i0 += sh.stride) {
    const uint32_t ix = i0 + 2 * (lane >> 5), iy = ix + 1;
    const bool livex = ix < sh.end, livey = iy < sh.end;
    PlaneEntry ex, ey;
    if (SH) {
      ex = ((const PlaneEntry*)list)[livex ? ix : i0];
      ey = ((const PlaneEntry*)list)[livey ? iy : i0];
    } else {
      ex.p = ((const uint32_t*)list)[livex ? ix : i0];
      ey.p = ((const uint32_t*)list)[livey ? iy : i0];
    }
    uint32_t dx[NO > 0 ? NO : 1], dy[NO > 0 ? NO : 1];
    plane_digits<NO>(g, ex.p, dx);
    plane_digits<NO>(g, ey.p, dy);
    const size_t ox = (size_t)ex.p * 1024u + L * 32u, oy = (size_t)ey.p * 1024u + L * 32u;
    // E rows of both planes (8-bit: odd bytes exact in Ehi, even bytes in
    // the high bytes of Elo; 16-bit: Ehi exact)
    uint32_t Xh[DW], Xl[WB == 1 ? DW : 1], Yh[DW], Yl[WB == 1 ? DW : 1];
#pragma unroll
    for (int d = 0; d < DW; d++) {
      Xh[d] = Yh[d] = 0;
      if (WB == 1) Xl[d] = Yl[d] = 0;
    }
    auto nb = [&](const PlaneEntry& e, const uint32_t* dig, size_t off, int j, int k) -> const uint4* {
      if (SH && j == NO - 1) {
        const uint32_t w = k == 1 ? e.top1 : e.top2;
        return w == kPlaneAbsent ? zero
               : w == kPlaneLocal ? (const uint4*)(tab + off - (size_t)k * g.Z * 1024u)
                                  : (const uint4*)(recv + (size_t)w * 1024u + L * 32u);
      }
      return dig[j] >= (uint32_t)k ? (const uint4*)(tab + off - (size_t)k * g.stride[j] * 1024u) : zero;
    };
#pragma unroll
    for (int j = 0; j < NO; j++) {
#pragma unroll
      for (int k = 1; k <= 2; k++) {
        const uint4* sx = nb(ex, dx, ox, j, k);
        const uint4* sy = nb(ey, dy, oy, j, k);
        uint4 vx[NQ], vy[NQ];
#pragma unroll
        for (int q = 0; q < NQ; q++) {
          vx[q] = sx[q];
          vy[q] = sy[q];
        }
#pragma unroll
        for (int q = 0; q < NQ; q++) {
          const uint32_t a[4] = {vx[q].x, vx[q].y, vx[q].z, vx[q].w};
          const uint32_t b[4] = {vy[q].x, vy[q].y, vy[q].z, vy[q].w};
#pragma unroll
          for (int c = 0; c < 4; c++) {
            Xh[4 * q + c] = pk_max16(Xh[4 * q + c], a[c]);
            Yh[4 * q + c] = pk_max16(Yh[4 * q + c], b[c]);
            if (WB == 1) {
              Xl[4 * q + c] = pk_max16(Xl[4 * q + c], pk_shl8(a[c]));
              Yl[4 * q + c] = pk_max16(Yl[4 * q + c], pk_shl8(b[c]));
            }
          }
        }
      }
    }
    const uint32_t primv =
        (g.rank == 0 && L == 0) ? ((ex.p == 0 ? W::kPrim : 0u) | (ey.p == 0 ? W::kPrim << 16 : 0u)) : 0u;
    // step q's results of both planes stay packed [X | Y] in op[q] (OR of
    // the two phases: an idle lane contributes 0) and are unpacked into the
    // two rows once, after the wavefront
    uint32_t cur = 0, prev = 0, u1p = 0;
    uint32_t op[32];
#pragma unroll
    for (int q = 0; q < 32; q++) op[q] = 0;
#pragma unroll 1
    for (uint32_t ph = 0; ph < 2; ph++) {
      const uint32_t flip = ph ? 0xFFFFFFFFu : 0u;
#pragma unroll
      for (int q = 0; q < 32; q++) {
        uint32_t a;
        if (WB == 1) {
          // byte q of X's and Y's E rows -> [X, 0, Y, 0]
          const int d = q >> 2, b = q & 3;
          const uint32_t bx = (b & 1) ? (uint32_t)b : (uint32_t)b + 1;  // byte inside the split dword
          const uint32_t sel = 0x0C000C00u | ((4u + bx) << 16) | bx;     // hi = Y (bytes 4-7), lo = X
          a = (b & 1) ? perm(Yh[d], Xh[d], sel) : perm(Yl[d], Xl[d], sel);
        } else {
          const int d = q >> 1, h = q & 1;
          const uint32_t b0 = 2 * h;
          const uint32_t sel = ((5u + b0) << 24) | ((4u + b0) << 16) | ((1u + b0) << 8) | b0;
          a = perm(Yh[d], Xh[d], sel);
        }
        const uint32_t u1r = from_lane_below(cur), u2r = from_lane_below(u1p);
        uint32_t m = pk_max16(pk_max16(a, cur), prev);
        const uint32_t m2 = pk_max16(pk_max16(m, u1r), u2r);
        m = l32 ? m : m2;  // row 0 of the upper pair has no row below
        const uint32_t am = (uint32_t)(q == 31 ? 0xFFFFFFFFull : ((2ull << q) - 1)) ^ flip;
        uint32_t f = keep_rows(am, L, parent_x2<WB>(m));
        if (q == 0) f = pk_max16(f, ph ? 0u : primv);
        op[q] |= f;
        prev = cur;
        cur = f;
        u1p = l32 ? 0u : u1r;
      }
    }
    uint32_t ox_[DW], oy_[DW];
    if (WB == 1) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint32_t t1 = perm(op[4 * k + 1], op[4 * k], 0x06020400u);      // [X0 X1 Y0 Y1]
        const uint32_t t2 = perm(op[4 * k + 3], op[4 * k + 2], 0x06020400u);  // [X2 X3 Y2 Y3]
        ox_[k] = perm(t2, t1, 0x05040100u);
        oy_[k] = perm(t2, t1, 0x07060302u);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 16; k++) {
        ox_[k] = perm(op[2 * k + 1], op[2 * k], 0x05040100u);
        oy_[k] = perm(op[2 * k + 1], op[2 * k], 0x07060302u);
      }
    }
    auto store = [&](T* dst, const uint32_t* o) {
      uint4* p = (uint4*)dst;
#pragma unroll
      for (int q = 0; q < NQ; q++) p[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
    };
    if (livex) {
      store(tab + ox, ox_);
      if (SH && ex.send != kPlaneAbsent) store(send + (size_t)ex.send * 1024u + L * 32u, ox_);
    }
    if (livey) {
      store(tab + oy, oy_);
      if (SH && ey.send != kPlaneAbsent) store(send + (size_t)ey.send * 1024u + L * 32u, oy_);
    }
  }
}

// k_plane_resolve_x2 held to 5 waves / SIMD (<= 96 VGPRs): the widest levels hold ~4.2 K waves
template <int WB, int NO, bool SH>
__global__ __launch_bounds__(256, 5) void k_plane_resolve_x2c(typename PlaneWord<WB>::T* __restrict__ tab,
                                                          const void* __restrict__ list, uint32_t n, PlaneGeom g,
                                                          const uint4* __restrict__ zero,
                                                          const typename PlaneWord<WB>::T* __restrict__ recv,
                                                          typename PlaneWord<WB>::T* __restrict__ send) {
  typedef PlaneWord<WB> W;
  typedef typename W::T T;
  constexpr int DW = W::DW, NQ = DW / 4;
  const uint32_t lane = threadIdx.x & 63, L = lane & 31;
  const bool l32 = lane == 32;
  const PlaneShare sh = plane_share(n, 4);
  for (uint32_t i0 = sh.first; i0 < sh.end; i0 += sh.stride) {
    const uint32_t ix = i0 + 2 * (lane >> 5), iy = ix + 1;
    const bool livex = ix < sh.end, livey = iy < sh.end;
    PlaneEntry ex, ey;
    if (SH) {
      ex = ((const PlaneEntry*)list)[livex ? ix : i0];
      ey = ((const PlaneEntry*)list)[livey ? iy : i0];
    } else {
      ex.p = ((const uint32_t*)list)[livex ? ix : i0];
      ey.p = ((const uint32_t*)list)[livey ? iy : i0];
    }
    uint32_t dx[NO > 0 ? NO : 1], dy[NO > 0 ? NO : 1];
    plane_digits<NO>(g, ex.p, dx);
    plane_digits<NO>(g, ey.p, dy);
    const size_t ox = (size_t)ex.p * 1024u + L * 32u, oy = (size_t)ey.p * 1024u + L * 32u;
    // E rows of both planes (8-bit: odd bytes exact in Ehi, even bytes in
    // the high bytes of Elo; 16-bit: Ehi exact)
    uint32_t Xh[DW], Xl[WB == 1 ? DW : 1], Yh[DW], Yl[WB == 1 ? DW : 1];
#pragma unroll
    for (int d = 0; d < DW; d++) {
      Xh[d] = Yh[d] = 0;
      if (WB == 1) Xl[d] = Yl[d] = 0;
    }
    auto nb = [&](const PlaneEntry& e, const uint32_t* dig, size_t off, int j, int k) -> const uint4* {
      if (SH && j == NO - 1) {
        const uint32_t w = k == 1 ? e.top1 : e.top2;
        return w == kPlaneAbsent ? zero
               : w == kPlaneLocal ? (const uint4*)(tab + off - (size_t)k * g.Z * 1024u)
                                  : (const uint4*)(recv + (size_t)w * 1024u + L * 32u);
      }
      return dig[j] >= (uint32_t)k ? (const uint4*)(tab + off - (size_t)k * g.stride[j] * 1024u) : zero;
    };
#pragma unroll
    for (int j = 0; j < NO; j++) {
#pragma unroll
      for (int k = 1; k <= 2; k++) {
        const uint4* sx = nb(ex, dx, ox, j, k);
        const uint4* sy = nb(ey, dy, oy, j, k);
        uint4 vx[NQ], vy[NQ];
#pragma unroll
        for (int q = 0; q < NQ; q++) {
          vx[q] = sx[q];
          vy[q] = sy[q];
        }
#pragma unroll
        for (int q = 0; q < NQ; q++) {
          const uint32_t a[4] = {vx[q].x, vx[q].y, vx[q].z, vx[q].w};
          const uint32_t b[4] = {vy[q].x, vy[q].y, vy[q].z, vy[q].w};
#pragma unroll
          for (int c = 0; c < 4; c++) {
            Xh[4 * q + c] = pk_max16(Xh[4 * q + c], a[c]);
            Yh[4 * q + c] = pk_max16(Yh[4 * q + c], b[c]);
            if (WB == 1) {
              Xl[4 * q + c] = pk_max16(Xl[4 * q + c], pk_shl8(a[c]));
              Yl[4 * q + c] = pk_max16(Yl[4 * q + c], pk_shl8(b[c]));
            }
          }
        }
      }
    }
    const uint32_t primv =
        (g.rank == 0 && L == 0) ? ((ex.p == 0 ? W::kPrim : 0u) | (ey.p == 0 ? W::kPrim << 16 : 0u)) : 0u;
    // step q's results of both planes stay packed [X | Y] in op[q] (OR of
    // the two phases: an idle lane contributes 0) and are unpacked into the
    // two rows once, after the wavefront
    uint32_t cur = 0, prev = 0, u1p = 0;
    uint32_t op[32];
#pragma unroll
    for (int q = 0; q < 32; q++) op[q] = 0;
#pragma unroll 1
    for (uint32_t ph = 0; ph < 2; ph++) {
      const uint32_t flip = ph ? 0xFFFFFFFFu : 0u;
#pragma unroll
      for (int q = 0; q < 32; q++) {
        uint32_t a;
        if (WB == 1) {
          // byte q of X's and Y's E rows -> [X, 0, Y, 0]
          const int d = q >> 2, b = q & 3;
          const uint32_t bx = (b & 1) ? (uint32_t)b : (uint32_t)b + 1;  // byte inside the split dword
          const uint32_t sel = 0x0C000C00u | ((4u + bx) << 16) | bx;     // hi = Y (bytes 4-7), lo = X
          a = (b & 1) ? perm(Yh[d], Xh[d], sel) : perm(Yl[d], Xl[d], sel);
        } else {
          const int d = q >> 1, h = q & 1;
          const uint32_t b0 = 2 * h;
          const uint32_t sel = ((5u + b0) << 24) | ((4u + b0) << 16) | ((1u + b0) << 8) | b0;
          a = perm(Yh[d], Xh[d], sel);
        }
        const uint32_t u1r = from_lane_below(cur), u2r = from_lane_below(u1p);
        uint32_t m = pk_max16(pk_max16(a, cur), prev);
        const uint32_t m2 = pk_max16(pk_max16(m, u1r), u2r);
        m = l32 ? m : m2;  // row 0 of the upper pair has no row below
        const uint32_t am = (uint32_t)(q == 31 ? 0xFFFFFFFFull : ((2ull << q) - 1)) ^ flip;
        uint32_t f = keep_rows(am, L, parent_x2<WB>(m));
        if (q == 0) f = pk_max16(f, ph ? 0u : primv);
        op[q] |= f;
        prev = cur;
        cur = f;
        u1p = l32 ? 0u : u1r;
      }
    }
    uint32_t ox_[DW], oy_[DW];
    if (WB == 1) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint32_t t1 = perm(op[4 * k + 1], op[4 * k], 0x06020400u);      // [X0 X1 Y0 Y1]
        const uint32_t t2 = perm(op[4 * k + 3], op[4 * k + 2], 0x06020400u);  // [X2 X3 Y2 Y3]
        ox_[k] = perm(t2, t1, 0x05040100u);
        oy_[k] = perm(t2, t1, 0x07060302u);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 16; k++) {
        ox_[k] = perm(op[2 * k + 1], op[2 * k], 0x05040100u);
        oy_[k] = perm(op[2 * k + 1], op[2 * k], 0x07060302u);
      }
    }
    auto store = [&](T* dst, const uint32_t* o) {
      uint4* p = (uint4*)dst;
#pragma unroll
      for (int q = 0; q < NQ; q++) p[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
    };
    if (livex) {
      store(tab + ox, ox_);
      if (SH && ex.send != kPlaneAbsent) store(send + (size_t)ex.send * 1024u + L * 32u, ox_);
    }
    if (livey) {
      store(tab + oy, oy_);
      if (SH && ey.send != kPlaneAbsent) store(send + (size_t)ey.send * 1024u + L * 32u, oy_);
    }
  }
}

// k_plane_resolve_x2 with every neighbour row of the wave's four planes
// loaded before any is folded (32 x 16 B in flight per lane; the shipped
// kernel keeps a window of ~6 under its 128-VGPR budget), at <= 2 waves /
// SIMD (256 VGPRs)
template <int WB, int NO, bool SH>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) void k_plane_resolve_x2w(typename PlaneWord<WB>::T* __restrict__ tab,
                                                          const void* __restrict__ list, uint32_t n, PlaneGeom g,
                                                          const uint4* __restrict__ zero,
                                                          const typename PlaneWord<WB>::T* __restrict__ recv,
                                                          typename PlaneWord<WB>::T* __restrict__ send) {
  typedef PlaneWord<WB> W;
  typedef typename W::T T;
  constexpr int DW = W::DW, NQ = DW / 4;
  const uint32_t lane = threadIdx.x & 63, L = lane & 31;
  const bool l32 = lane == 32;
  const PlaneShare sh = plane_share(n, 4);
  for (uint32_t i0 = sh.first; i0 < sh.end; i0 += sh.stride) {
    const uint32_t ix = i0 + 2 * (lane >> 5), iy = ix + 1;
    const bool livex = ix < sh.end, livey = iy < sh.end;
    PlaneEntry ex, ey;
    if (SH) {
      ex = ((const PlaneEntry*)list)[livex ? ix : i0];
      ey = ((const PlaneEntry*)list)[livey ? iy : i0];
    } else {
      ex.p = ((const uint32_t*)list)[livex ? ix : i0];
      ey.p = ((const uint32_t*)list)[livey ? iy : i0];
    }
    uint32_t dx[NO > 0 ? NO : 1], dy[NO > 0 ? NO : 1];
    plane_digits<NO>(g, ex.p, dx);
    plane_digits<NO>(g, ey.p, dy);
    const size_t ox = (size_t)ex.p * 1024u + L * 32u, oy = (size_t)ey.p * 1024u + L * 32u;
    // E rows of both planes (8-bit: odd bytes exact in Ehi, even bytes in
    // the high bytes of Elo; 16-bit: Ehi exact)
    uint32_t Xh[DW], Xl[WB == 1 ? DW : 1], Yh[DW], Yl[WB == 1 ? DW : 1];
#pragma unroll
    for (int d = 0; d < DW; d++) {
      Xh[d] = Yh[d] = 0;
      if (WB == 1) Xl[d] = Yl[d] = 0;
    }
    auto nb = [&](const PlaneEntry& e, const uint32_t* dig, size_t off, int j, int k) -> const uint4* {
      if (SH && j == NO - 1) {
        const uint32_t w = k == 1 ? e.top1 : e.top2;
        return w == kPlaneAbsent ? zero
               : w == kPlaneLocal ? (const uint4*)(tab + off - (size_t)k * g.Z * 1024u)
                                  : (const uint4*)(recv + (size_t)w * 1024u + L * 32u);
      }
      return dig[j] >= (uint32_t)k ? (const uint4*)(tab + off - (size_t)k * g.stride[j] * 1024u) : zero;
    };
    constexpr int NN = NO > 0 ? NO : 1;
    uint4 VX[NN][2][NQ], VY[NN][2][NQ];
#pragma unroll
    for (int j = 0; j < NO; j++) {
#pragma unroll
      for (int k = 1; k <= 2; k++) {
        const uint4* sx = nb(ex, dx, ox, j, k);
        const uint4* sy = nb(ey, dy, oy, j, k);
#pragma unroll
        for (int q = 0; q < NQ; q++) {
          VX[j][k - 1][q] = sx[q];
          VY[j][k - 1][q] = sy[q];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NO; j++) {
#pragma unroll
      for (int k = 1; k <= 2; k++) {
#pragma unroll
        for (int q = 0; q < NQ; q++) {
          const uint4 xv = VX[j][k - 1][q], yv = VY[j][k - 1][q];
          const uint32_t a[4] = {xv.x, xv.y, xv.z, xv.w};
          const uint32_t b[4] = {yv.x, yv.y, yv.z, yv.w};
#pragma unroll
          for (int c = 0; c < 4; c++) {
            Xh[4 * q + c] = pk_max16(Xh[4 * q + c], a[c]);
            Yh[4 * q + c] = pk_max16(Yh[4 * q + c], b[c]);
            if (WB == 1) {
              Xl[4 * q + c] = pk_max16(Xl[4 * q + c], pk_shl8(a[c]));
              Yl[4 * q + c] = pk_max16(Yl[4 * q + c], pk_shl8(b[c]));
            }
          }
        }
      }
    }
    const uint32_t primv =
        (g.rank == 0 && L == 0) ? ((ex.p == 0 ? W::kPrim : 0u) | (ey.p == 0 ? W::kPrim << 16 : 0u)) : 0u;
    // step q's results of both planes stay packed [X | Y] in op[q] (OR of
    // the two phases: an idle lane contributes 0) and are unpacked into the
    // two rows once, after the wavefront
    uint32_t cur = 0, prev = 0, u1p = 0;
    uint32_t op[32];
#pragma unroll
    for (int q = 0; q < 32; q++) op[q] = 0;
#pragma unroll 1
    for (uint32_t ph = 0; ph < 2; ph++) {
      const uint32_t flip = ph ? 0xFFFFFFFFu : 0u;
#pragma unroll
      for (int q = 0; q < 32; q++) {
        uint32_t a;
        if (WB == 1) {
          // byte q of X's and Y's E rows -> [X, 0, Y, 0]
          const int d = q >> 2, b = q & 3;
          const uint32_t bx = (b & 1) ? (uint32_t)b : (uint32_t)b + 1;  // byte inside the split dword
          const uint32_t sel = 0x0C000C00u | ((4u + bx) << 16) | bx;     // hi = Y (bytes 4-7), lo = X
          a = (b & 1) ? perm(Yh[d], Xh[d], sel) : perm(Yl[d], Xl[d], sel);
        } else {
          const int d = q >> 1, h = q & 1;
          const uint32_t b0 = 2 * h;
          const uint32_t sel = ((5u + b0) << 24) | ((4u + b0) << 16) | ((1u + b0) << 8) | b0;
          a = perm(Yh[d], Xh[d], sel);
        }
        const uint32_t u1r = from_lane_below(cur), u2r = from_lane_below(u1p);
        uint32_t m = pk_max16(pk_max16(a, cur), prev);
        const uint32_t m2 = pk_max16(pk_max16(m, u1r), u2r);
        m = l32 ? m : m2;  // row 0 of the upper pair has no row below
        const uint32_t am = (uint32_t)(q == 31 ? 0xFFFFFFFFull : ((2ull << q) - 1)) ^ flip;
        uint32_t f = keep_rows(am, L, parent_x2<WB>(m));
        if (q == 0) f = pk_max16(f, ph ? 0u : primv);
        op[q] |= f;
        prev = cur;
        cur = f;
        u1p = l32 ? 0u : u1r;
      }
    }
    uint32_t ox_[DW], oy_[DW];
    if (WB == 1) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint32_t t1 = perm(op[4 * k + 1], op[4 * k], 0x06020400u);      // [X0 X1 Y0 Y1]
        const uint32_t t2 = perm(op[4 * k + 3], op[4 * k + 2], 0x06020400u);  // [X2 X3 Y2 Y3]
        ox_[k] = perm(t2, t1, 0x05040100u);
        oy_[k] = perm(t2, t1, 0x07060302u);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 16; k++) {
        ox_[k] = perm(op[2 * k + 1], op[2 * k], 0x05040100u);
        oy_[k] = perm(op[2 * k + 1], op[2 * k], 0x07060302u);
      }
    }
    auto store = [&](T* dst, const uint32_t* o) {
      uint4* p = (uint4*)dst;
#pragma unroll
      for (int q = 0; q < NQ; q++) p[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
    };
    if (livex) {
      store(tab + ox, ox_);
      if (SH && ex.send != kPlaneAbsent) store(send + (size_t)ex.send * 1024u + L * 32u, ox_);
    }
    if (livey) {
      store(tab + oy, oy_);
      if (SH && ey.send != kPlaneAbsent) store(send + (size_t)ey.send * 1024u + L * 32u, oy_);
    }
  }
}

}  // namespace gm
