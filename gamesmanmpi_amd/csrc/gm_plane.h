// gm_plane.h -- PLANES layout of the dense (rank-indexable) sum games:
// natural rank order, 1 or 2 bytes per position, no holes.  Kernels for
// gfx950 (MI355X).
//
// Replaces, for sum_four_to_one with heaps 0 and 1 of 32 values, the
// reference's per-position job loop (src/process.py:109-267: lookup ->
// distribute -> resolve with _res_red/_remote_red) by a sweep over PLANES:
//
//   position (h0, h1, P), P = mixed-radix index of the outer heaps
//   h2..h(K-1) ("plane"): planes of 32 x 32 positions, rows of 32, each row
//   ROTATED left by its row number -- byte b = (h0 + h1) & 31 of row h1 --
//   and every row cut into 16-B PIECES, piece c of all 32 rows side by side:
//       byte  P * 1024 + c * 512 + h1 * 16 + (b & 15),  c = b >> 4  (8-bit)
//       word  P * 1024 + c * 256 + h1 * 8 + (b & 7),    c = b >> 3  (16-bit)
//   (plane_word_index).  A plane is 1 KiB (8-bit words) or 2 KiB (16-bit).
//   Lane h1 still loads and stores its row as 16-B pieces, but a half-wave's
//   32 pieces of one instruction are now 512 CONTIGUOUS bytes: four whole
//   128-B lines.  With rows contiguous instead (round 4), each store
//   instruction wrote half of 8 lines, and the L2 filled every line from
//   memory before the second half arrived: +1 KiB of fetch per plane written
//   (FETCH_SIZE 4.26 -> 3.70 GB per 2^30 backward in tools/stream_lab.hip
//   var 14 vs 19), a third of the fabric reads of the wide plane levels.
//
// One move lowers ONE heap by 1 or 2 (test_games/four_to_one.py:7-22), so a
// position's children lie in its own plane (h0 / h1 lowered) or at the same
// (h0, h1) of one of 2 (K - 2) neighbour planes P - k * stride_j (k = 1, 2).
// Planes of equal outer digit sum s are independent of each other; plane
// level s needs levels s - 1 and s - 2 only.  The backward pass is one launch
// per plane level (outer digit sums 0 .. sum of outer heaps; 125 launches
// for 31^6 instead of 187 levels of the level-major DENSE layout).
//
// k_plane_resolve: one wave = two planes (lanes 0-31 and 32-63, lane = row
// h1).  Each lane loads its row of the neighbour planes (16-B loads, a
// wave's load = 1 KiB of contiguous rows), folds them into E, the per-
// position max of the external children, with packed 16-bit maxes, and then
// resolves its row by a 63-step skewed wavefront: at step t lane h1 handles
// h0 = t - h1, whose children (h0-1, h1), (h0-2, h1) are the lane's last two
// results and (h0, h1-1), (h0, h1-2) the last results of lanes h1-1 / h1-2
// one and two steps ago (DPP wave_shr:1).  Because every row is rotated by
// its row number, the byte a lane needs at step t sits at register byte
// t & 31 in EVERY lane: all extracts and inserts are static.
//
// Order-form words (the unsigned max over the children is the reduction of
// _res_red/_remote_red; absent children read 0, neutral):
//   8-bit (every value WIN/LOSS, remoteness < 255, value = parity of the
//          remoteness): WIN r -> (r - 1) / 2, LOSS r -> 0x80 | (0x7F - r / 2);
//          parent of max m: h(m) = 0xFE - m + (m >> 7)
//   16-bit: WIN r -> r, LOSS r -> 0x8000 | (0x7FFF - r);
//          parent of max m: h(m) = 0xFFFE - m + 2 (m >> 15)
// The only primitive (every heap 0, a LOSS) is LOSS 0 = 0xFF / 0xFFFF.
//
// Relative 8-bit forms (word form 3; root digit sums 254 .. 505, e.g. the
// sharded bench shapes 31^5 x 127 and 31^5 x 255): a position of digit sum e
// (all heaps) has remoteness in [ceil(e / 2), e], a window of e / 2 + 1
// values, so its word is taken relative to an offset o(e) = (e + 1) / 4 - 1:
//   WIN r -> (r - 1) / 2 - o(e),  LOSS r -> 0xFF - r / 2 + o(e)
// (o is one below the smallest (r - 1) / 2 of the window: every real WIN
// word is >= 1, so 0 still reads as "no child" after the shift below; the
// primitive is LOSS 0 = 0xFE).  A parent at e = d reduces its children in
// the frame of d - 1: children at d - 1 are already in it, children at
// d - 2 (a heap lowered by 2) are shifted by o(d - 1) - o(d - 2), which is 1
// exactly when d % 4 == 0 (WIN w -> w - 1, LOSS l -> l + 1, 0 stays 0: a
// saturating subtract); the parent word from the frame-(d - 1) max m is
// h(m) above when o(d) == o(d - 1), and 0xFF - m - (m >> 7) when
// o(d) = o(d - 1) + 1 (d % 4 == 3).  d % 4 = (s + t) % 4 for outer digit sum
// s and wavefront step t, so with s % 4 (RS) a template parameter of the
// launch every shift and parent form is static per step.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace gm {

constexpr int kPlaneMaxOuter = 6;  // K <= 8 heaps

// Geometry of one PLANES table (a whole game, or one shard of it).  A shard
// (world > 1) owns blocks of B consecutive values of the TOP outer digit
// (heap K-1), dealt in rounds of `world` blocks: round j = blocks
// [j * world, (j + 1) * world) gives each rank one block (plane_owner); its
// table holds only its own slices, block after block: local plane =
// (j * B + o) * Z + lower, where j is the rank's block number (= the round),
// o the value's offset in the block, Z = planes per top value and lower =
// the index of the digits below the top.  Neighbours along the top digit
// that belong to the previous block come from a halo buffer (PlaneEntry).
struct PlaneGeom {
  uint32_t no;     // outer digits (heaps 2 .. K-1)
  uint32_t pow2;   // every outer base a power of two
  uint32_t nplanes;  // planes of this table (local)
  uint32_t world, rank, B, Z;  // shards (world 1: B = Z = 0)
  uint32_t spread;  // shards: the link-spreading deal (plane_owner), else round robin
  // the row deal (shards of heap 1, plane_shape): this shard's rows are heap-1
  // values [h1off, h1off + 32); the outer digits are the whole table's
  uint32_t rowdeal, h1off;
  uint32_t base[kPlaneMaxOuter];
  uint32_t shift[kPlaneMaxOuter];   // log2(stride[j]) when pow2
  uint32_t stride[kPlaneMaxOuter];  // global plane-index stride of outer digit j
  uint32_t rlim[kPlaneMaxOuter + 2];  // reach: heap i reachable up to rlim[i] (heaps 0, 1, then outer)
};

// Which rank owns global block b, and which global block is a rank's local
// block j.  Round robin: block c of a round goes to rank c, so every block's
// successor lives on rank + 1 and a shard's whole halo crosses ONE xGMI link.
// The spreading deal (world a power of two >= 4, whole rounds): round j
// gives block c to rank c * (2j + 1) mod world -- an odd multiplier, so a
// permutation -- and the successor of a rank's round-j block sits 2j + 1
// ranks further on: the rounds' halos leave on up to world / 2 different
// links.  Block 0 stays rank 0's local block 0 (the primitive plane).
__host__ __device__ inline uint32_t plane_owner(const PlaneGeom& g, uint32_t b) {
  const uint32_t c = b % g.world;
  return g.spread ? (c * (2u * (b / g.world) + 1u)) & (g.world - 1u) : c;
}
__host__ __device__ inline uint32_t plane_gblock(const PlaneGeom& g, uint32_t j) {
  if (!g.spread) return g.rank + j * g.world;
  const uint32_t m = 2u * j + 1u;
  uint32_t inv = m;  // m^-1 mod 2^32 by Newton steps (each doubles the good bits)
  for (int i = 0; i < 5; i++) inv *= 2u - m * inv;
  return j * g.world + ((g.rank * inv) & (g.world - 1u));
}

// Sharded level lists: per plane, where its top-digit neighbours are and
// where its words go besides the table.
constexpr uint32_t kPlaneAbsent = 0xFFFFFFFFu;  // no such neighbour (top value < k): reads 0
constexpr uint32_t kPlaneLocal = 0xFFFFFFFEu;   // the neighbour is local: plane - k * Z
struct PlaneEntry {
  uint32_t p;      // local plane
  uint32_t top1;   // neighbour at top value - 1: kPlaneAbsent / kPlaneLocal / halo plane index
  uint32_t top2;   // neighbour at top value - 2: the same
  uint32_t send;   // halo plane index in the send buffer (boundary slices), or kPlaneAbsent
};

// element index of byte / word b (rotated row position) of row h1 of plane
// P (T = 8- or 16-bit words)
__host__ __device__ inline uint64_t plane_word_index(uint64_t P, uint32_t h1, uint32_t b, uint32_t wb) {
  return wb == 2 ? P * 1024u + (uint64_t)(b >> 3) * 256u + h1 * 8u + (b & 7u)
                 : P * 1024u + (uint64_t)(b >> 4) * 512u + h1 * 16u + (b & 15u);
}
// in elements of T: a lane's first piece in its plane, and the piece stride
template <typename T>
__host__ __device__ constexpr uint32_t plane_row0(uint32_t h1) { return h1 * (16u / (uint32_t)sizeof(T)); }
template <typename T>
__host__ __device__ constexpr uint32_t plane_piece() { return 512u / (uint32_t)sizeof(T); }
constexpr int kPieceU4 = 32;  // piece stride in uint4 (512 B)

template <int WB>
struct PlaneWord;
template <>
struct PlaneWord<1> {
  typedef uint8_t T;
  static constexpr int DW = 8;  // dwords of one 32-position row
  static constexpr uint32_t kPrim = 0xFFu;
  __device__ static __forceinline__ uint32_t parent(uint32_t m) { return 0xFEu - m + (m >> 7); }
};
template <>
struct PlaneWord<3> {  // relative 8-bit forms (above)
  typedef uint8_t T;
  static constexpr int DW = 8;
  static constexpr uint32_t kPrim = 0xFEu;
};
template <>
struct PlaneWord<2> {
  typedef uint16_t T;
  static constexpr int DW = 16;
  static constexpr uint32_t kPrim = 0xFFFFu;
  __device__ static __forceinline__ uint32_t parent(uint32_t m) { return 0xFFFEu - m + ((m >> 15) << 1); }
};

// host + device: the order-form word of a value/remoteness and back
__host__ __device__ inline uint32_t plane_word_to_vr(uint32_t w, int wb) {
  // -> value | remoteness << 2 (GM_WIN 0 / GM_LOSS 1)
  if (wb == 1) {
    if (w & 0x80u) return 1u | ((2u * (0x7Fu - (w & 0x7Fu))) << 2);
    return 0u | ((2u * w + 1u) << 2);
  }
  if (w & 0x8000u) return 1u | ((0x7FFFu - (w & 0x7FFFu)) << 2);
  return 0u | (w << 2);
}

// relative forms: the offset at digit sum e, the word -> value | remoteness
// << 2, and the largest root digit sum whose every window fits a byte
__host__ __device__ inline int plane_rel_off(uint32_t e) { return (int)((e + 1) / 4) - 1; }
__host__ __device__ inline uint32_t plane_rel_to_vr(uint32_t w, uint32_t e) {
  const int o = plane_rel_off(e);
  if (w & 0x80u) return 1u | ((uint32_t)(2 * (0xFF - (int)w + o)) << 2);
  return 0u | ((uint32_t)(2 * ((int)w + o) + 1) << 2);
}
constexpr uint32_t kPlaneRelMaxSum = 505;  // e = 506: the WIN window's top word reaches 0x80

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk_max16(uint32_t a, uint32_t b) {
  u16x2 x = __builtin_bit_cast(u16x2, a), y = __builtin_bit_cast(u16x2, b);
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(x, y));
}
// max of three packed step values.  The 8-bit word forms keep every step
// value in [0, 0xFF] per 16-bit half (words in the low byte, the high byte 0:
// the E byte extract, the parent forms and the frame shift all map [0, 0xFF]
// into itself), and there the f16 bit patterns are +0 and positive
// subnormals, ordered as the integers are: gfx950's v_pk_maximum3_f16 is an
// exact three-input packed u16 max, one instruction for two v_pk_max_u16
// (the kernels run with f16 denormals preserved, float_denorm_mode_16_64 = 3;
// no NaN pattern can arise).  16-bit words: two integer maxes.
template <bool B8V>
__device__ __forceinline__ uint32_t pk_max3w(uint32_t a, uint32_t b, uint32_t c) {
  if constexpr (B8V) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    const h2 x = __builtin_bit_cast(h2, a), y = __builtin_bit_cast(h2, b), z = __builtin_bit_cast(h2, c);
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_maximum(__builtin_elementwise_maximum(x, y), z));
  } else {
    return pk_max16(pk_max16(a, b), c);
  }
}
__device__ __forceinline__ uint32_t pk_shl8(uint32_t a) {
  u16x2 x = __builtin_bit_cast(u16x2, a);
  return __builtin_bit_cast(uint32_t, (u16x2)(x << (unsigned short)8));
}
// v if bit `row` of the wave-uniform row mask m is set, else 0: a
// sign-extended bit extract (v_bfe_i32, SGPR mask) and an and.  (An inline
// v_cndmask with an "s"-constrained 64-bit mask was miscompiled under SGPR
// pressure: the mask landed in a VGPR pair.)
__device__ __forceinline__ uint32_t keep_rows(uint32_t m, uint32_t row, uint32_t v) {
  return v & (uint32_t)__builtin_amdgcn_sbfe((int)m, (int)row, 1);
}
// value of lane - 1 (lane 0: 0)
__device__ __forceinline__ uint32_t from_lane_below(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138 /* wave_shr:1 */, 0xF, 0xF, true);
}

template <int NO>
__device__ __forceinline__ void plane_digits(const PlaneGeom& g, uint32_t P, uint32_t* dig) {
  if (g.pow2) {
#pragma unroll
    for (int j = 0; j < NO; j++) dig[j] = (P >> g.shift[j]) & (g.base[j] - 1u);
  } else {
    uint32_t x = P;
#pragma unroll
    for (int j = 0; j < NO; j++) {
      dig[j] = x % g.base[j];
      x /= g.base[j];
    }
  }
}

// global digits of a local plane: outer digits j < NO - 1 from the lower
// index, the top one from the shard's block layout (world 1: plain digits)
template <int NO>
__device__ __forceinline__ void plane_global_digits(const PlaneGeom& g, uint32_t P, uint32_t* dig) {
  plane_digits<NO>(g, P, dig);
  if (g.B && NO > 0) {  // the top-heap deals (the row deal's outer digits are global)
    const uint32_t u = P / g.Z, j = u / g.B, o = u - j * g.B;
    dig[NO - 1] = plane_gblock(g, j) * g.B + o;
  }
}

// XCD-chunked share of n items for this wave (blocks b -> XCD b % 8):
// the wave handles items [first, end) with the given stride
struct PlaneShare {
  uint32_t first, end, stride;
};
__device__ __forceinline__ PlaneShare plane_share(uint32_t n, uint32_t per_wave) {
  const uint32_t G = gridDim.x, waves = blockDim.x >> 6;
  const uint32_t nx = (G >= 8 && G % 8 == 0) ? 8u : 1u;
  const uint32_t x = blockIdx.x % nx, lb = blockIdx.x / nx;
  const uint32_t chunk = ((n + nx - 1) / nx + per_wave - 1) / per_wave * per_wave;
  const uint32_t b = min(n, x * chunk);
  PlaneShare s;
  s.end = min(n, b + chunk);
  s.first = b + (lb * waves + (threadIdx.x >> 6)) * per_wave;
  s.stride = (G / nx) * waves * per_wave;
  return s;
}

// One plane level: list[0 .. n) are the level's planes (uint32 plane index,
// or PlaneEntry for shards).  tab: the table (plane P at tab + P * 1024
// words); zero: >= 64 zero bytes; recv / send: the shard's halo buffers.
// the wave's share of list entries [first, end), two planes per wave
// visit, `stride` apart (k_plane_resolve: plane_share; k_plane_run: the
// workgroup's waves)
template <int WB, int NO, bool SH>
__device__ __forceinline__ void plane_x1_range(typename PlaneWord<WB>::T* __restrict__ tab,
                                               const void* __restrict__ list, const PlaneShare sh,
                                               const PlaneGeom& g, const uint4* __restrict__ zero,
                                               const typename PlaneWord<WB>::T* __restrict__ recv,
                                               typename PlaneWord<WB>::T* __restrict__ send) {
  typedef PlaneWord<WB> W;
  static_assert(WB != 3, "relative words: the packed form only");
  constexpr int DW = W::DW, NQ = DW / 4;  // dwords / 16-B loads per row
  const uint32_t lane = threadIdx.x & 63, L = lane & 31;
  for (uint32_t i0 = sh.first; i0 < sh.end; i0 += sh.stride) {
    const uint32_t idx = i0 + (lane >> 5);
    const bool live = idx < sh.end;
    PlaneEntry e;
    if (SH) {
      e = ((const PlaneEntry*)list)[live ? idx : i0];
    } else {
      e.p = ((const uint32_t*)list)[live ? idx : i0];
    }
    const uint32_t P = e.p;
    uint32_t dig[NO > 0 ? NO : 1];
    plane_digits<NO>(g, P, dig);
    const size_t rowoff = (size_t)P * 1024u + plane_row0<typename W::T>(L);  // in words: the row's first piece
    // external children: rows of the neighbour planes, folded into E
    uint32_t Ehi[DW], Elo[WB == 1 ? DW : 1];
#pragma unroll
    for (int d = 0; d < DW; d++) {
      Ehi[d] = 0;
      if (WB == 1) Elo[d] = 0;
    }
#pragma unroll
    for (int j = 0; j < NO; j++) {
#pragma unroll
      for (int k = 1; k <= 2; k++) {
        const uint4* src;
        if (SH && j == NO - 1) {  // the sharded top digit: local, halo or absent
          const uint32_t w = k == 1 ? e.top1 : e.top2;
          src = w == kPlaneAbsent ? zero
                : w == kPlaneLocal ? (const uint4*)(tab + rowoff - (size_t)k * g.Z * 1024u)
                                   : (const uint4*)(recv + (size_t)w * 1024u + plane_row0<typename W::T>(L));
        } else {
          src = dig[j] >= (uint32_t)k ? (const uint4*)(tab + rowoff - (size_t)k * g.stride[j] * 1024u) : zero;
        }
        uint4 v[NQ];
#pragma unroll
        for (int q = 0; q < NQ; q++) v[q] = src[q * kPieceU4];
#pragma unroll
        for (int q = 0; q < NQ; q++) {
          const uint32_t x[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
          for (int c = 0; c < 4; c++) {
            Ehi[4 * q + c] = pk_max16(Ehi[4 * q + c], x[c]);  // 8-bit: odd bytes exact in the high halves
            if (WB == 1) Elo[4 * q + c] = pk_max16(Elo[4 * q + c], pk_shl8(x[c]));  // even bytes
          }
        }
      }
    }
    // the skewed wavefront over the plane: step t = 32 ph + q handles
    // h0 = t - h1; lanes outside [t - 31, t] are idle and produce 0.  The
    // active-row mask is formed in SALU per step (a table of 63 constants
    // would be hoisted into SGPRs and spill).
    const bool prim = g.rank == 0 && P == 0 && L == 0;  // every heap 0: the primitive LOSS
    // (the lean step chain of plane_x2_range: no lane-32 masks, ready
    // children folded off the chain, active rows from a per-lane word)
    uint32_t cur = 0, prev = 0, u1p = 0;
    uint32_t out[DW];
#pragma unroll
    for (int d = 0; d < DW; d++) out[d] = 0;
    const uint32_t A0 = ~0u << L;  // bit q set: row L is active at step q of phase 0
#pragma unroll 1
    for (uint32_t ph = 0; ph < 2; ph++) {
      const uint32_t A = ph ? ~A0 : A0;  // phase 1: the lanes past their row's start
#pragma unroll
      for (int q = 0; q < 32; q++) {
        uint32_t a;
        if (WB == 1) {
          const int d = q >> 2, b = q & 3;
          a = (b & 1) ? __builtin_amdgcn_ubfe(Ehi[d], 8 * b, 8) : __builtin_amdgcn_ubfe(Elo[d], 8 * b + 8, 8);
        } else {
          a = __builtin_amdgcn_ubfe(Ehi[q >> 1], 16 * (q & 1), 16);
        }
        const uint32_t u2 = from_lane_below(u1p);
        const uint32_t pre = max(max(a, prev), u2);
        const uint32_t u1 = from_lane_below(cur);
        const uint32_t m = max(max(pre, cur), u1);
        uint32_t f = W::parent(m) & (uint32_t)__builtin_amdgcn_sbfe((int)A, q, 1);
        if (q == 0) f = (prim && ph == 0) ? W::kPrim : f;
        if (WB == 1)
          out[q >> 2] |= f << (8 * (q & 3));
        else
          out[q >> 1] |= f << (16 * (q & 1));
        prev = cur;
        cur = f;
        u1p = u1;
      }
    }
    if (live) {
      uint4* dst = (uint4*)(tab + rowoff);
#pragma unroll
      for (int q = 0; q < NQ; q++)
        dst[q * kPieceU4] = make_uint4(out[4 * q], out[4 * q + 1], out[4 * q + 2], out[4 * q + 3]);
      if (SH && e.send != kPlaneAbsent) {  // a boundary slice: also into the send buffer
        uint4* sd = (uint4*)(send + (size_t)e.send * 1024u + plane_row0<typename W::T>(L));
#pragma unroll
        for (int q = 0; q < NQ; q++)
          sd[q * kPieceU4] = make_uint4(out[4 * q], out[4 * q + 1], out[4 * q + 2], out[4 * q + 3]);
      }
    }
  }
}

// Warm the caches with the NEXT launch's list entries: one 128-B line per
// thread, issued before this wave's own loads so its wait overlaps theirs;
// the value is kept live to the end of the kernel (a dead load is dropped).
// The line lands in this XCD's L2 and the memory-side Infinity Cache, so
// the next level's first, dependent load (list entry -> neighbour rows)
// does not go to HBM.
__device__ __forceinline__ uint32_t plane_prefetch(const uint32_t* __restrict__ pf, uint32_t lines) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  return t < lines ? pf[(size_t)t * 32u] : 0u;
}
__device__ __forceinline__ void plane_keep(uint32_t v) { asm volatile("; keep %0" ::"v"(v)); }

template <int WB, int NO, bool SH>
__global__ __launch_bounds__(256) void k_plane_resolve(typename PlaneWord<WB>::T* __restrict__ tab,
                                                       const void* __restrict__ list, uint32_t n, PlaneGeom g,
                                                       const uint4* __restrict__ zero,
                                                       const typename PlaneWord<WB>::T* __restrict__ recv,
                                                       typename PlaneWord<WB>::T* __restrict__ send,
                                                       const uint32_t* __restrict__ pf, uint32_t pflines) {
  const uint32_t v = plane_prefetch(pf, pflines);
  plane_x1_range<WB, NO, SH>(tab, list, plane_share(n, 2), g, zero, recv, send);
  plane_keep(v);
}

// Packed form: a wave resolves FOUR planes -- each lane carries two planes'
// rows in the 16-bit halves of its registers (X low, Y high; lanes 0-31 one
// pair, 32-63 another), so every step of the skewed wavefront advances two
// positions per lane with packed 16-bit maxes / adds (v_pk_*): about half
// the VALU of k_plane_resolve per position.  Same layout, lists and results.
__device__ __forceinline__ uint32_t pk_add16(uint32_t a, uint32_t b) {
  u16x2 x = __builtin_bit_cast(u16x2, a), y = __builtin_bit_cast(u16x2, b);
  return __builtin_bit_cast(uint32_t, (u16x2)(x + y));
}
__device__ __forceinline__ uint32_t pk_sub16(uint32_t a, uint32_t b) {
  u16x2 x = __builtin_bit_cast(u16x2, a), y = __builtin_bit_cast(u16x2, b);
  return __builtin_bit_cast(uint32_t, (u16x2)(x - y));
}
__device__ __forceinline__ uint32_t pk_shr16(uint32_t a, int n) {
  u16x2 x = __builtin_bit_cast(u16x2, a);
  return __builtin_bit_cast(uint32_t, (u16x2)(x >> (unsigned short)n));
}
// parent order form of packed child maxima (both halves)
template <int WB>
__device__ __forceinline__ uint32_t parent_x2(uint32_t m) {
  if (WB == 1) return pk_add16(pk_sub16(0x00FE00FEu, m), pk_shr16(m, 7));
  return pk_add16(pk_sub16(0xFFFEFFFEu, m), pk_shr16(m, 15) << 1);  // (m>>15)<<1 stays in its half
}
__device__ __forceinline__ uint32_t pk_sub_sat16(uint32_t a, uint32_t b) {
  u16x2 x = __builtin_bit_cast(u16x2, a), y = __builtin_bit_cast(u16x2, b);
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(x, y));
}
// relative forms, the d - 2 -> d - 1 frame shift of byte B0 (a HIGH byte of
// its 16-bit half, B0 odd) of a folded E dword (WIN w -> w - 1, LOSS l ->
// l + 1).  The byte is 0 only when every folded row was a zero row (absent
// neighbour: real WIN words are >= 1), and then so is the half's low byte:
// the saturating 16-bit subtract leaves 0 there and never borrows otherwise.
template <int B0>
__device__ __forceinline__ uint32_t rel_shift_byte(uint32_t x) {
  const uint32_t t = pk_sub_sat16(x, 1u << (8 * B0));
  return t + (__builtin_amdgcn_ubfe(x, 8 * B0 + 7, 1) << (8 * B0 + 1));
}
// the same shift of packed step values (one word in the low byte of each
// 16-bit half; 0 -- no child, an idle lane -- stays 0)
__device__ __forceinline__ uint32_t rel_shift_pk(uint32_t v) {
  return pk_sub_sat16(v, 0x00010001u) + (pk_shr16(v, 7) << 1);
}
// relative forms, parent word when o(d) = o(d - 1) + 1
__device__ __forceinline__ uint32_t parent_rel_up(uint32_t m) {
  return pk_sub16(pk_sub16(0x00FF00FFu, m), pk_shr16(m, 7));
}
// v_perm_b32 selector bytes
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}

// One visit: planes ex / ey resolved by one wave (the lower / upper half
// wave each holds one plane's 32 rows).  A function of its own, not a
// lambda inside the list loop: the lambda form cost the NO = 4 kernel 12
// VGPRs (119 -> 131, one wave per SIMD less).
#ifndef GM_PLANE_MAX3  // 0: the step's maxima as v_pk_max_u16 pairs (A/B)
#define GM_PLANE_MAX3 1
#endif
#ifndef GM_PLANE_OFFMASK  // 0: phase 0 masks f on the chain (A/B)
#define GM_PLANE_OFFMASK 1
#endif
#ifndef GM_PLANE_FOLD3  // 0: even bytes folded as shift + max (A/B)
#define GM_PLANE_FOLD3 1
#endif
#ifndef GM_PLANE_RSV_UNR
#define GM_PLANE_RSV_UNR false
#endif
// (mid: called once the neighbour rows are folded, before the wavefront --
// the one-launch backward issues its next visit's polls there)
struct PlaneNoMid {
  __device__ void operator()() const {}
};
template <int WB, int NO, bool SH, int RS_, bool UNR = true, bool WT = false, bool HR = false, class Mid = PlaneNoMid>
__device__ __forceinline__ void plane_x2_visit(typename PlaneWord<WB>::T* __restrict__ tab, const PlaneGeom& g,
                                               const uint4* __restrict__ zero,
                                               const typename PlaneWord<WB>::T* __restrict__ recv,
                                               typename PlaneWord<WB>::T* __restrict__ send, const PlaneEntry ex,
                                               const PlaneEntry ey, const bool livex, const bool livey,
                                               Mid mid = Mid()) {
  typedef PlaneWord<WB> W;
  typedef typename W::T T;
  constexpr int DW = W::DW, NQ = DW / 4;
  constexpr bool B8 = DW == 8, REL = WB == 3;
  const uint32_t L = threadIdx.x & 31;
  constexpr int B0 = (4 - RS_) & 3;  // relative: row bytes j = B0 mod 4 are parents with d % 4 == 0
  uint32_t dx[NO > 0 ? NO : 1], dy[NO > 0 ? NO : 1];
  plane_digits<NO>(g, ex.p, dx);
  plane_digits<NO>(g, ey.p, dy);
  const size_t ox = (size_t)ex.p * 1024u + plane_row0<T>(L), oy = (size_t)ey.p * 1024u + plane_row0<T>(L);
  // E rows of both planes (8-bit: odd bytes exact in Ehi, even bytes in
  // the high bytes of Elo; 16-bit: Ehi exact)
  uint32_t Xh[DW], Xl[B8 ? DW : 1], Yh[DW], Yl[B8 ? DW : 1];
#pragma unroll
  for (int d = 0; d < DW; d++) {
    Xh[d] = Yh[d] = 0;
    if (B8) Xl[d] = Yl[d] = 0;
  }
  auto nb = [&](const PlaneEntry& e, const uint32_t* dig, size_t off, int j, int k) -> const uint4* {
    if (SH && j == NO - 1) {
      const uint32_t w = k == 1 ? e.top1 : e.top2;
      return w == kPlaneAbsent ? zero
             : w == kPlaneLocal ? (const uint4*)(tab + off - (size_t)k * g.Z * 1024u)
                                : (const uint4*)(recv + (size_t)w * 1024u + plane_row0<T>(L));
    }
    return dig[j] >= (uint32_t)k ? (const uint4*)(tab + off - (size_t)k * g.stride[j] * 1024u) : zero;
  };
  // FL3 (8-bit forms): the even bytes fold in LOW-byte form (masked with
  // 0x00FF00FF, two neighbours per v_pk_maximum3_f16, exact on [0, 0xFF] as
  // in the step), the odd ones raw in the high bytes (one v_pk_max_u16 each):
  // 2.5 operations per neighbour dword and plane instead of 3 (shift + max)
  constexpr bool FL3 = GM_PLANE_FOLD3 && B8;
  auto lowb = [](uint32_t v) { return FL3 ? (v & 0x00FF00FFu) : pk_shl8(v); };
  // the neighbour rows' values (v*2: when `two`) into the E rows
  auto foldv = [&](const uint4* vx1, const uint4* vy1, const uint4* vx2, const uint4* vy2, const bool two) {
#pragma unroll
    for (int q = 0; q < NQ; q++) {
      const uint32_t a1[4] = {vx1[q].x, vx1[q].y, vx1[q].z, vx1[q].w};
      const uint32_t b1[4] = {vy1[q].x, vy1[q].y, vy1[q].z, vy1[q].w};
      uint32_t a2[4] = {0, 0, 0, 0}, b2[4] = {0, 0, 0, 0};
      if (two) {
        a2[0] = vx2[q].x, a2[1] = vx2[q].y, a2[2] = vx2[q].z, a2[3] = vx2[q].w;
        b2[0] = vy2[q].x, b2[1] = vy2[q].y, b2[2] = vy2[q].z, b2[3] = vy2[q].w;
      }
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const int d = 4 * q + c;
        Xh[d] = pk_max16(Xh[d], a1[c]);
        Yh[d] = pk_max16(Yh[d], b1[c]);
        if (two) {
          Xh[d] = pk_max16(Xh[d], a2[c]);
          Yh[d] = pk_max16(Yh[d], b2[c]);
        }
        if (B8) {
          if (FL3 && two) {
            Xl[d] = pk_max3w<true>(Xl[d], lowb(a1[c]), lowb(a2[c]));
            Yl[d] = pk_max3w<true>(Yl[d], lowb(b1[c]), lowb(b2[c]));
          } else {
            Xl[d] = pk_max16(Xl[d], lowb(a1[c]));
            Yl[d] = pk_max16(Yl[d], lowb(b1[c]));
            if (two) {
              Xl[d] = pk_max16(Xl[d], lowb(a2[c]));
              Yl[d] = pk_max16(Yl[d], lowb(b2[c]));
            }
          }
        }
      }
    }
  };
  auto fold2 = [&](int j1, int k1, int j2, int k2) {  // j2 < 0: one neighbour
    const bool two = j2 >= 0;
    const uint4* sx1 = nb(ex, dx, ox, j1, k1);
    const uint4* sy1 = nb(ey, dy, oy, j1, k1);
    const uint4* sx2 = two ? nb(ex, dx, ox, j2, k2) : sx1;
    const uint4* sy2 = two ? nb(ey, dy, oy, j2, k2) : sy1;
    uint4 vx1[NQ], vy1[NQ], vx2[NQ], vy2[NQ];
#pragma unroll
    for (int q = 0; q < NQ; q++) {
      vx1[q] = sx1[q * kPieceU4];
      vy1[q] = sy1[q * kPieceU4];
      if (two) {
        vx2[q] = sx2[q * kPieceU4];
        vy2[q] = sy2[q * kPieceU4];
      }
    }
    foldv(vx1, vy1, vx2, vy2, two);
  };
  // HR (the row deal, shards of heap 1): the first two rows' neighbours below
  // the shard -- heap-1 values h1off - 1 and h1off - 2 -- are the previous
  // shard's rows 31 and 30, from the halo buffer (recv: per list entry
  // [row 30 | row 31] as that shard stored them, each rotated by its own row).
  // Row L's neighbour at h1 - k (L < k) is halo row L - k + 2, and in row L's
  // rotation its byte j is their byte j - k: every other lane reads zeros.
  auto hrow = [&](const PlaneEntry& e, int k, uint4* v) {
    const bool has = HR && e.top1 != kPlaneAbsent && L < (uint32_t)k;
    const uint4* src = has ? (const uint4*)(recv + (size_t)e.top1 * 64u + (L + 2u - (uint32_t)k) * 32u) : zero;
    uint32_t x[DW], y[DW];
#pragma unroll
    for (int q = 0; q < NQ; q++) {
      const uint4 t = src[q];
      x[4 * q] = t.x, x[4 * q + 1] = t.y, x[4 * q + 2] = t.z, x[4 * q + 3] = t.w;
    }
#pragma unroll
    for (int d = 0; d < DW; d++) {
      const uint32_t lo = x[(d + DW - 1) % DW];
      y[d] = B8 ? __builtin_amdgcn_alignbit(x[d], lo, 32u - 8u * (uint32_t)k)
                : (k == 2 ? lo : __builtin_amdgcn_alignbit(x[d], lo, 16u));
    }
#pragma unroll
    for (int q = 0; q < NQ; q++) v[q] = make_uint4(y[4 * q], y[4 * q + 1], y[4 * q + 2], y[4 * q + 3]);
  };
  auto hfold = [&](int k1, int k2) {  // k2 = 0: one neighbour row
    uint4 x1[NQ], y1[NQ], x2[NQ], y2[NQ];
    hrow(ex, k1, x1);
    hrow(ey, k1, y1);
    if (k2) {
      hrow(ex, k2, x2);
      hrow(ey, k2, y2);
    }
    foldv(x1, y1, x2, y2, k2 != 0);
  };
  if constexpr (REL) {
    // children at d - 2 first, then their frame shift -- ONCE on the
    // folded maxima (the shift is monotone: it commutes with max), on the
    // one split array that holds row bytes B0 mod 4 (Xh: odd bytes, high in
    // their halves; Xl: even ones, low with FL3), half B0 / 2 of every
    // dword -- then the children at d - 1
#pragma unroll
    for (int j = 0; j < NO; j += 2) fold2(j, 2, j + 1 < NO ? j + 1 : -1, 2);
    if constexpr (HR) hfold(2, 0);
#pragma unroll
    for (int d = 0; d < DW; d++) {
      if (B0 & 1) {
        Xh[d] = rel_shift_byte<2 * (B0 >> 1) + 1>(Xh[d]);
        Yh[d] = rel_shift_byte<2 * (B0 >> 1) + 1>(Yh[d]);
      } else {
        Xl[d] = rel_shift_byte<2 * (B0 >> 1) + (FL3 ? 0 : 1)>(Xl[d]);
        Yl[d] = rel_shift_byte<2 * (B0 >> 1) + (FL3 ? 0 : 1)>(Yl[d]);
      }
    }
#pragma unroll
    for (int j = 0; j < NO; j += 2) fold2(j, 1, j + 1 < NO ? j + 1 : -1, 1);
    if constexpr (HR) hfold(1, 0);
  } else {
#pragma unroll
    for (int j = 0; j < NO; j++) fold2(j, 1, j, 2);
    if constexpr (HR) hfold(1, 2);
  }
  mid();
  const uint32_t primv =
      (g.rank == 0 && L == 0) ? ((ex.p == 0 ? W::kPrim : 0u) | (ey.p == 0 ? W::kPrim << 16 : 0u)) : 0u;
  // step q's results of both planes stay packed [X | Y] in op[q] (OR of
  // the two phases: an idle lane contributes 0) and are unpacked into the
  // two rows once, after the wavefront
  // The step chain (lean form, round 4: backward 1.624 -> 1.540 ms per
  // 2^30 in tools/plane_lab, bit-exact): the children that are ready a
  // step early -- the E byte, this row's h0 - 2 result, the h1 - 2 row's
  // -- are folded off the chain, so cur -> (lane below) -> max -> parent
  // -> active mask is the whole dependency per step.  No lane-32 masks:
  // the upper pair's row 0 (lane 32) reads lane 31 (the lower pair's row
  // 31) only at steps <= 31, where row 31 is still idle and holds 0, and
  // row 1 reads lane 31's u1 of step <= 30, also 0.  Active rows: bit q of
  // A, one bit extract per step (phase 0: rows 0..q; phase 1: q+1..31).
  uint32_t cur = 0, prev = 0, u1p = 0;
  uint32_t op[32];
  const uint32_t A0 = ~0u << L;  // bit q set: row L is active at step q of phase 0
  // both phases unrolled (phase 0 assigns op[q], phase 1 ORs into it):
  // 1.549 -> 1.512 ms per 2^30 backward in tools/plane_lab (var 30), 98
  // VGPRs in the lab form against 119 for a rolled phase loop
  // (UNR false, the per-visit RS dispatch: a rolled phase loop, so the
  // kernel's four visit bodies stay within the instruction cache)
  auto phase = [&](auto PHc) {
    const int PH = PHc;  // a constant when unrolled
    const uint32_t A = PH ? ~A0 : A0;
#pragma unroll
    for (int q = 0; q < 32; q++) {
      uint32_t a;
      if (B8) {
        // byte q of X's and Y's E rows -> [X, 0, Y, 0]
        const int d = q >> 2, b = q & 3;
        const uint32_t bx = (b & 1) || FL3 ? (uint32_t)b : (uint32_t)b + 1;  // byte inside the split dword
        const uint32_t sel = 0x0C000C00u | ((4u + bx) << 16) | bx;     // hi = Y (bytes 4-7), lo = X
        a = (b & 1) ? perm(Yh[d], Xh[d], sel) : perm(Yl[d], Xl[d], sel);
      } else {
        const int d = q >> 1, h = q & 1;
        const uint32_t b0 = 2 * h;
        const uint32_t sel = ((5u + b0) << 24) | ((4u + b0) << 16) | ((1u + b0) << 8) | b0;
        a = perm(Yh[d], Xh[d], sel);
      }
      const uint32_t u2r = from_lane_below(u1p);
      const int dcls = (RS_ + q) & 3;  // relative forms: d % 4 of this step's positions (32 = 0 mod 4)
      const uint32_t pre = REL && dcls == 0 ? pk_max16(a, rel_shift_pk(pk_max16(prev, u2r)))
                                            : pk_max3w<GM_PLANE_MAX3 && B8>(a, prev, u2r);
      const uint32_t u1r = from_lane_below(cur);
      // phase 0, 8-bit forms: a row that has not started takes pre = the word
      // whose parent is 0 (0xFF; 0xFE for the relative up form) -- its cur
      // and the row below's are still 0, so m = pre and f = 0 with no mask
      // on the chain (cur -> DPP -> max3 -> parent -> cur, five operations)
      const bool offm = GM_PLANE_OFFMASK && UNR && B8 && PH == 0;
      const uint32_t pre_ =
          offm ? ((__builtin_amdgcn_sbfe((int)A, q, 1) != 0) ? pre : (REL && dcls == 3 ? 0x00FE00FEu : 0x00FF00FFu))
               : pre;
      const uint32_t m = pk_max3w<GM_PLANE_MAX3 && B8>(pre_, cur, u1r);
      uint32_t f = REL && dcls == 3 ? parent_rel_up(m) : parent_x2<WB == 2 ? 2 : 1>(m);
      if (offm) {
        if (q == 0) f = pk_max16(f, primv);
        op[q] = f;
      } else if (UNR && PH == 1) {
        // phase 1: a finished row's value is never read by an active row
        // (row L, active at steps q < L, reads rows L - 1 / L - 2 at steps
        // q - 1 / q - 2, when they were active too), so it needs no zeroing:
        // the mask only merges the step into the row's output, one
        // v_cndmask in place of and + or
        op[q] = __builtin_amdgcn_sbfe((int)A, q, 1) ? f : op[q];
      } else {
        f &= (uint32_t)__builtin_amdgcn_sbfe((int)A, q, 1);
        if (q == 0) f = pk_max16(f, PH ? 0u : primv);
        if (UNR && PH == 0) op[q] = f;
        else op[q] |= f;
      }
      prev = cur;
      cur = f;
      u1p = u1r;
    }
  };
  if constexpr (UNR) {
    phase(std::integral_constant<int, 0>());
    phase(std::integral_constant<int, 1>());
  } else {
#pragma unroll
    for (int q = 0; q < 32; q++) op[q] = 0;
#pragma unroll 1
    for (int ph = 0; ph < 2; ph++) phase(ph);
  }
  uint32_t ox_[DW], oy_[DW];
  if (B8) {
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
  // WT (the per-level grid launches): write-through (sc1) vector stores --
  // the next level is a new launch whose readers find nothing of this one in
  // their L2 anyway, and the lines leave while the kernel still runs instead
  // of in the write-back at its end: 1.342 -> 1.283-1.292 ms per 2^30
  // backward (tools/stream_lab.hip, GM_PLANE_STORE_POLICY builds; nt stores
  // 1.42 ms).  (An inline-asm store the compiler does not count in vmcnt only
  // makes its later waits stricter: it is the youngest operation.)
  auto store = [&](T* dst, const uint32_t* o) {
    uint4* p = (uint4*)dst;
#pragma unroll
    for (int q = 0; q < NQ; q++) {
      if constexpr (WT) {
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        const v4u v = {o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]};
        asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p + q * kPieceU4), "v"(v) : "memory");
      } else {
        p[q * kPieceU4] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
      }
    }
  };
  // HR: rows 30 and 31 also go to the next shard's halo, one entry per plane
  auto hstore = [&](const PlaneEntry& e, const uint32_t* o) {
    if (!HR || e.send == kPlaneAbsent || L < 30) return;
    uint4* p = (uint4*)(send + (size_t)e.send * 64u + (L - 30u) * 32u);
#pragma unroll
    for (int q = 0; q < NQ; q++) p[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
  };
  if (livex) {
    store(tab + ox, ox_);
    if (SH && ex.send != kPlaneAbsent) store(send + (size_t)ex.send * 1024u + plane_row0<T>(L), ox_);
    hstore(ex, ox_);
  }
  if (livey) {
    store(tab + oy, oy_);
    if (SH && ey.send != kPlaneAbsent) store(send + (size_t)ey.send * 1024u + plane_row0<T>(L), oy_);
    hstore(ey, oy_);
  }
}

// (RS: with WB = 3, the launch's outer digit sum s mod 4; -1: per wave
// visit, from its first plane -- the list deals every four consecutive
// entries one s mod 4, padding with kPlaneAbsent entries)
template <int WB, int NO, bool SH, int RS = 0, bool WT = false, bool HR = false>
__device__ __forceinline__ void plane_x2_range(typename PlaneWord<WB>::T* __restrict__ tab,
                                               const void* __restrict__ list, const PlaneShare sh,
                                               const PlaneGeom& g, const uint4* __restrict__ zero,
                                               const typename PlaneWord<WB>::T* __restrict__ recv,
                                               typename PlaneWord<WB>::T* __restrict__ send) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint32_t i0 = sh.first; i0 < sh.end; i0 += sh.stride) {
    const uint32_t ix = i0 + 2 * (lane >> 5), iy = ix + 1;
    bool livex = ix < sh.end, livey = iy < sh.end;
    PlaneEntry ex, ey;
    if (SH) {
      ex = ((const PlaneEntry*)list)[livex ? ix : i0];
      ey = ((const PlaneEntry*)list)[livey ? iy : i0];
      if (RS < 0) {  // padding entries: compute on the visit's first plane, store nothing
        const PlaneEntry e0 = ((const PlaneEntry*)list)[i0];
        if (ex.p == kPlaneAbsent) ex = e0, livex = false;
        if (ey.p == kPlaneAbsent) ey = e0, livey = false;
      }
    } else {
      const uint32_t jx = livex ? ix : i0, jy = livey ? iy : i0;
      ex.p = ((const uint32_t*)list)[jx];
      ey.p = ((const uint32_t*)list)[jy];
      if (HR) {  // the row deal: halo entries in list order
        ex.top1 = recv ? jx : kPlaneAbsent;
        ey.top1 = recv ? jy : kPlaneAbsent;
        ex.send = send ? jx : kPlaneAbsent;
        ey.send = send ? jy : kPlaneAbsent;
      }
    }
    if constexpr (RS >= 0) {
      plane_x2_visit<WB, NO, SH, RS, true, WT, HR>(tab, g, zero, recv, send, ex, ey, livex, livey);
    } else {  // the visit's outer digit sum (global digits) mod 4, wave-uniform
      uint32_t dg[NO > 0 ? NO : 1], sum = 0;
      plane_global_digits<NO>(g, ex.p, dg);
#pragma unroll
      for (int j = 0; j < NO; j++) sum += dg[j];
      switch (__builtin_amdgcn_readfirstlane(sum) & 3u) {
        case 0: plane_x2_visit<WB, NO, SH, 0, GM_PLANE_RSV_UNR, WT>(tab, g, zero, recv, send, ex, ey, livex, livey); break;
        case 1: plane_x2_visit<WB, NO, SH, 1, GM_PLANE_RSV_UNR, WT>(tab, g, zero, recv, send, ex, ey, livex, livey); break;
        case 2: plane_x2_visit<WB, NO, SH, 2, GM_PLANE_RSV_UNR, WT>(tab, g, zero, recv, send, ex, ey, livex, livey); break;
        default: plane_x2_visit<WB, NO, SH, 3, GM_PLANE_RSV_UNR, WT>(tab, g, zero, recv, send, ex, ey, livex, livey); break;
      }
    }
  }
}

template <int WB, int NO, bool SH, int RS, bool HR = false>
__global__ __launch_bounds__(256) void k_plane_resolve_x2(typename PlaneWord<WB>::T* __restrict__ tab,
                                                          const void* __restrict__ list, uint32_t n, PlaneGeom g,
                                                          const uint4* __restrict__ zero,
                                                          const typename PlaneWord<WB>::T* __restrict__ recv,
                                                          typename PlaneWord<WB>::T* __restrict__ send,
                                                          const uint32_t* __restrict__ pf, uint32_t pflines) {
  const uint32_t v = plane_prefetch(pf, pflines);
  plane_x2_range<WB, NO, SH, RS, true, HR>(tab, list, plane_share(n, 4), g, zero, recv, send);
  plane_keep(v);
}

// The one-table backward as ONE launch (round 6, the default for one-table
// 8-bit absolute solves): every plane level in it, a plane resolved as soon
// as its neighbours are final instead of at a kernel boundary per level.
//   Items: a wave visit of four planes.  Every level's visits are cut into 8
// contiguous chunks (XCD x's waves, blockIdx % 8 == x, take chunk x: the
// per-level launches' plane_share locality) and each chunk is dealt round
// robin over the XCD's kPlaneFlowSeq sequences; a sequence holds its visits
// level after level, and its waves take them by ticket (one device counter
// per sequence, each on a line of its own).  Deadlock-free for any grid: a
// wave waits only for planes of lower levels, every taken visit is held by a
// wave that runs, and the lowest unfinished visit's neighbours are final.
//   Hand-off: a visit stores its rows write-through (sc1, the per-level
// launches' stores), drains them (s_waitcnt vmcnt(0)), then sets its planes'
// flags to the solve's epoch (relaxed device-scope stores).  A plane waits
// for the flags of its four k = 1 neighbours only: its k = 2 neighbour along
// digit j is the k = 1 neighbour of its k = 1 neighbour along j, final
// before that one started.  The neighbour rows then come through PLAIN
// loads: a plane's lines (1 KiB, 8 lines of its own) are first read only
// after its flag is set, so no L1 or L2 holds an older copy of them within
// the launch (the launch's acquire cleared what the previous solve left).
//   Exit: a wave that finds its sequence empty leaves; a wave that waits past
// kPlaneFlowSpin polls sets the give-up word and ERR bit `stall` and leaves
// (every other wave sees the word and leaves: the launch always drains).
// The last wave out resets the counters and the give-up word for the next
// solve.  tools/flow2_lab.hip: 1.06-1.09 vs 1.34 ms per 2^30 backward for
// the same visits launched per level, byte-exact on a poisoned table
// (profiles/r06/flow2_lab.txt).
constexpr uint32_t kPlaneFlowSeq = 8;      // ticket sequences per XCD (PlaneFlow::nseq; lab A/B up to kPlaneFlowSeqMax)
constexpr uint32_t kPlaneFlowSeqMax = 16;
constexpr uint32_t kPlaneFlowQ = 8 * kPlaneFlowSeqMax;  // counter lines / sequence offsets provisioned
constexpr uint32_t kPlaneFlowLine = 64;    // u32 per counter line
constexpr uint32_t kPlaneFlowSpin = 1u << 20;
constexpr uint32_t kPlaneFlowBlocksPerCU = 3;
struct PlaneFlow {
  const uint32_t* items;  // visits: 4 planes each (kPlaneAbsent pads), sequence after sequence
  const uint32_t* qoff;   // [kPlaneFlowQ + 1]: first visit of each sequence
  uint32_t* ctr;          // [kPlaneFlowQ + 2] lines: tickets, then the exit count and the give-up word
  uint32_t* flags;        // per plane: the epoch of the solve that finished it
  uint32_t* err;          // DevState::err
  uint32_t epoch, stall;
  uint32_t skip;  // (the lab build's fault injector, GM_FAULT_FLOW: this plane's flag is never set; else kPlaneAbsent)
  uint32_t nseq;  // ticket sequences per XCD (kPlaneFlowSeq)
  uint32_t mode;  // (lab A/B, GM_PLANE_FLOW_MODE: 1 agent release fence before the flags, 4 agent acquire after the polls)
};
typedef __attribute__((address_space(1))) uint32_t plane_gu32;
__device__ __forceinline__ uint32_t plane_flow_ld(uint32_t* p) {
  return __hip_atomic_load((plane_gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void plane_flow_st(uint32_t* p, uint32_t v) {
  __hip_atomic_store((plane_gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// (the kernel, k_plane_flow in gm_plane_run.h, runs this body and then the
// forward's reach map and counts in the same launch)
template <int NO, bool PIPE>
__device__ __forceinline__ void plane_flow_body(uint8_t* __restrict__ tab, const PlaneGeom& g,
                                                const uint4* __restrict__ zero, const PlaneFlow& f) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t q = (blockIdx.x & 7u) + 8u * ((blockIdx.x >> 3) % f.nseq);
  const uint32_t base = f.qoff[q], n = f.qoff[q + 1] - base;
  uint32_t* const c = f.ctr + kPlaneFlowLine * q;
  uint32_t* const nout = f.ctr + kPlaneFlowLine * kPlaneFlowQ;
  uint32_t* const gave = nout + kPlaneFlowLine;
  constexpr uint32_t NW = NO > 0 ? NO : 1;
  // lane l < 4 NO watches the k = 1 neighbour along digit l % NO of the
  // visit's plane l / NO (kPlaneAbsent: nothing to wait for)
  auto nbr = [&](uint32_t pq) -> uint32_t {
    uint32_t nbp = kPlaneAbsent;
    if (NO > 0 && lane < 4u * NO && pq != kPlaneAbsent) {
      const uint32_t j = lane % NW;
      uint32_t dg[NW];
      plane_digits<NO>(g, pq, dg);
#pragma unroll
      for (int i = 0; i < NO; i++)
        if ((uint32_t)i == j && dg[i] >= 1u) nbp = pq - g.stride[i];
    }
    return nbp;
  };
  // a visit's planes: this lane's X and Y, the first (padding lanes compute
  // it again, storing nothing) and the plane this lane watches
  struct Visit {
    uint32_t x, y, p0, pq;
  };
  auto visit_of = [&](uint32_t tk) -> Visit {
    const uint32_t* ip = f.items + (size_t)(base + tk) * 4u;
    Visit v;
    v.x = ip[2 * (lane >> 5)];
    v.y = ip[2 * (lane >> 5) + 1];
    v.p0 = ip[0];
    v.pq = (NO > 0 && lane < 4u * NO) ? ip[lane / NW] : kPlaneAbsent;
    return v;
  };
  const Visit none{kPlaneAbsent, kPlaneAbsent, kPlaneAbsent, kPlaneAbsent};
  auto ticket = [&]() -> uint32_t {  // (lane 0's device atomic; read with readfirstlane(__shfl(., 0)))
    uint32_t v = 0;
    if (lane == 0) v = atomicAdd(c, 1u);
    return v;
  };
  auto uni = [](uint32_t v) { return __builtin_amdgcn_readfirstlane(__shfl(v, 0)); };
  uint32_t t = uni(ticket());
  Visit cv = t < n ? visit_of(t) : none;
  // PIPE: the ticket after next is in flight during a visit (requested after
  // the previous drain, read after this one); the next visit's planes load
  // after the previous drain, and its polls go out once this visit's rows are
  // folded (mid) -- at the drain their answers are in, usually "final", so
  // the next visit loads its rows at once.  Not PIPE: the next ticket and the
  // next visit's planes are requested after the drain (issued before the row
  // loads, a device-scope atomic held up their first wait: 1.062-1.066 ->
  // 1.022 ms per step) and each visit polls before its rows.
  uint32_t tn = ticket(), tn2 = 0;
  Visit nv = none;
  if (PIPE) {
    tn = uni(tn);
    nv = tn < n ? visit_of(tn) : none;
    tn2 = ticket();
  }
  bool ready = false;  // (PIPE) this visit's neighbours seen final during the previous one
  while (t < n) {
    if (!ready) {
      const uint32_t nbp = nbr(cv.pq);
      bool ok = nbp == kPlaneAbsent;
      for (uint32_t spins = 0;; spins++) {
        if (!ok) ok = plane_flow_ld(f.flags + nbp) == f.epoch;
        if (__all(ok)) break;
        if (spins >= kPlaneFlowSpin || plane_flow_ld(gave)) {
          if (lane == 0) {
            plane_flow_st(gave, 1u);
            atomicOr(f.err, f.stall);
          }
          t = n;
          break;
        }
        if (f.mode & 16u) __builtin_amdgcn_s_sleep(1);  // (lab A/B: GM_PLANE_FLOW_MODE bit 16)
        else __builtin_amdgcn_s_sleep(4);
      }
      if (t >= n) break;
    }
    if (f.mode & 4u) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    // the polls complete before anything below issues, and no load below may
    // be moved above them (a compiler barrier, not only a hardware wait)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    PlaneEntry ex, ey;
    ex.p = cv.x;
    ey.p = cv.y;
    const bool livex = ex.p != kPlaneAbsent, livey = ey.p != kPlaneAbsent;
    if (!livex) ex.p = cv.p0;
    if (!livey) ey.p = cv.p0;
    uint32_t nflag = 0, nbn = kPlaneAbsent;
    auto mid = [&]() {
      if (PIPE) {
        nbn = nbr(nv.pq);
        if (nbn != kPlaneAbsent) nflag = plane_flow_ld(f.flags + nbn);
      }
    };
    plane_x2_visit<1, NO, false, 0, true, true, false>(tab, g, zero, nullptr, nullptr, ex, ey, livex, livey, mid);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every lane's rows written through before any flag
    if (f.mode & 1u) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if ((lane & 31) < 2) {
      const bool live = (lane & 1) ? livey : livex;
      const uint32_t p = (lane & 1) ? ey.p : ex.p;
      if (live && p != f.skip) plane_flow_st(f.flags + p, f.epoch);
    }
    if (PIPE) {
      ready = __all(nbn == kPlaneAbsent || nflag == f.epoch);
      t = tn;
      cv = nv;
      tn = uni(tn2);
      if (t < n) {
        nv = tn < n ? visit_of(tn) : none;
        tn2 = ticket();
      }
    } else {
      t = uni(tn);
      if (t < n) {
        cv = visit_of(t);
        tn = ticket();
      }
    }
  }
  if (lane == 0) {  // the last wave out resets the counters for the next solve
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    if (atomicAdd(nout, 1u) == waves - 1u) {
      for (uint32_t i = 0; i < kPlaneFlowQ; i++) plane_flow_st(f.ctr + kPlaneFlowLine * i, 0u);
      plane_flow_st(gave, 0u);
      plane_flow_st(nout, 0u);
    }
  }
}

// A run of narrow plane levels (or staged keys) in ONE workgroup: the
// groups [off[i], off[i + 1]) one after another, a workgroup barrier
// between them.  One CU suffices for a group of a few dozen planes, and the
// run pays one launch instead of one per group (a narrow launch costs
// ~5 us of kernel plus ~2-3 us of boundary: profiles/r03c_trace_levels.txt).
// Coherence: the waves share the CU's L1 and write through to its XCD's L2;
// a plane's lines are first loaded by this CU only after the group that
// writes them (neighbours lie in earlier groups), so the barrier's
// workgroup-scope release / acquire is all a later group needs.
constexpr int kPlaneRunMax = 32;      // groups per run
constexpr int kPlaneRunThreads = 512;  // 8 waves: <= 256 VGPRs, every kernel variant fits
struct PlaneRun {
  uint32_t n;
  uint32_t off[kPlaneRunMax + 1];  // list entries, absolute
  uint64_t rs;                     // relative forms: group i's outer digit sum mod 4 in bits 2i, 2i + 1
  uint32_t visit;                  // relative forms: per wave visit instead (staged lists)
};
template <int WB, int NO, bool SH, bool X1>
__global__ __launch_bounds__(kPlaneRunThreads) void k_plane_run(typename PlaneWord<WB>::T* __restrict__ tab,
                                                                const void* __restrict__ list, PlaneRun run,
                                                                PlaneGeom g, const uint4* __restrict__ zero,
                                                                const typename PlaneWord<WB>::T* __restrict__ recv,
                                                                typename PlaneWord<WB>::T* __restrict__ send) {
  constexpr uint32_t per = X1 ? 2u : 4u;  // planes per wave visit
  const uint32_t w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (uint32_t i = 0; i < run.n; i++) {
    const PlaneShare sh{run.off[i] + w * per, run.off[i + 1], nw * per};
    if constexpr (WB == 3) {
      bool done = false;
      if constexpr (SH) {
        if (run.visit) {
          plane_x2_range<WB, NO, SH, -1>(tab, list, sh, g, zero, recv, send);
          done = true;
        }
      }
      if (!done) switch ((run.rs >> (2 * i)) & 3u) {
        case 0: plane_x2_range<WB, NO, SH, 0>(tab, list, sh, g, zero, recv, send); break;
        case 1: plane_x2_range<WB, NO, SH, 1>(tab, list, sh, g, zero, recv, send); break;
        case 2: plane_x2_range<WB, NO, SH, 2>(tab, list, sh, g, zero, recv, send); break;
        default: plane_x2_range<WB, NO, SH, 3>(tab, list, sh, g, zero, recv, send); break;
      }
    } else if constexpr (X1) {
      plane_x1_range<WB, NO, SH>(tab, list, sh, g, zero, recv, send);
    } else {
      plane_x2_range<WB, NO, SH>(tab, list, sh, g, zero, recv, send);
    }
    __syncthreads();
  }
}


// Two plane levels in ONE launch (round 6; the narrow levels of a one-table
// solve, 8-bit absolute words, at most four outer digits).  A narrow plane
// level costs about one dependent launch -- boundary, list entry, neighbour
// rows, the 64-step wavefront, row stores, ~4.5 us -- however few planes it
// holds, and the solve has ~60 of them.  k_plane_pair resolves levels s and
// s + 1 together: a wave takes one plane P of level s + 1, FIRST resolves
// P's k = 1 neighbours Q_j = P - e_j (level s) in its four channels (lane
// half x 16-bit half: one visit, channel j = outer digit j), THEN P itself,
// its k = 1 rows straight from the first visit's registers (the upper lane
// half's through LDS) and its k = 2 rows (level s - 1) from memory.  Every
// level-s plane is resolved by each of its level-(s + 1) parents (up to four:
// redundant work, nothing at a narrow level) and STORED by exactly one: the
// parent P = Q + e_j with j the lowest digit that Q can be raised in (P's
// digits below j all at their top value).  The dependent chain of the pair is
// one launch and two wavefronts instead of two launches.  Measured in
// tools/pair_lab.hip: pairs over levels 4-17 and 107-120 (14 launches fewer)
// 1.282-1.286 -> 1.225-1.231 ms per 2^30 backward, byte-exact
// (profiles/r06/pair_lab.txt).
template <class Fold>
__device__ __forceinline__ void plane_pair_wavefront(uint32_t L, uint32_t primv, Fold fold, uint32_t* ox,
                                                     uint32_t* oy) {
  uint32_t Xh[8], Xl[8], Yh[8], Yl[8];
#pragma unroll
  for (int d = 0; d < 8; d++) Xh[d] = Xl[d] = Yh[d] = Yl[d] = 0;
  fold(Xh, Xl, Yh, Yl);  // E rows: odd bytes raw in Xh / Yh, even bytes low-masked in Xl / Yl
  uint32_t cur = 0, prev = 0, u1p = 0;
  uint32_t op[32];
  const uint32_t A0 = ~0u << L;
  auto phase = [&](auto PHc) {  // the step chain of plane_x2_visit (8-bit absolute forms)
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
__device__ __forceinline__ void plane_pair_fold(uint32_t* Xh, uint32_t* Xl, uint32_t* Yh, uint32_t* Yl,
                                                const uint32_t* a, const uint32_t* b) {
#pragma unroll
  for (int d = 0; d < 8; d++) {
    Xh[d] = pk_max16(Xh[d], a[d]);
    Yh[d] = pk_max16(Yh[d], b[d]);
    Xl[d] = pk_max16(Xl[d], a[d] & 0x00FF00FFu);
    Yl[d] = pk_max16(Yl[d], b[d] & 0x00FF00FFu);
  }
}
// row L of plane P (both 16-B pieces), or zeros
__device__ __forceinline__ void plane_pair_row(const uint8_t* tab, bool has, uint32_t P, uint32_t L,
                                               const uint4* zero, uint32_t* r) {
  const uint4* src = has ? (const uint4*)(tab + (size_t)P * 1024u + L * 16u) : zero;
  const uint4 v0 = src[0], v1 = src[kPieceU4];
  r[0] = v0.x, r[1] = v0.y, r[2] = v0.z, r[3] = v0.w;
  r[4] = v1.x, r[5] = v1.y, r[6] = v1.z, r[7] = v1.w;
}
__device__ __forceinline__ void plane_pair_store(uint8_t* tab, uint32_t P, uint32_t L, const uint32_t* o) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  uint4* p = (uint4*)(tab + (size_t)P * 1024u + L * 16u);
#pragma unroll
  for (int q = 0; q < 2; q++) {  // write-through, as the grid launches' rows (plane_x2_visit)
    const v4u v = {o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p + q * kPieceU4), "v"(v) : "memory");
  }
}
// list: level s + 1's planes (uint32 plane indices), n of them; one wave per
// plane, four waves per workgroup (the grid loop is uniform per workgroup:
// the LDS exchange's barriers)
template <int NO>
__global__ __launch_bounds__(256) void k_plane_pair(uint8_t* __restrict__ tab, const uint32_t* __restrict__ list,
                                                    uint32_t n, PlaneGeom g, const uint4* __restrict__ zero) {
  static_assert(NO >= 1 && NO <= 4, "one channel per outer digit");
  __shared__ uint32_t xch[4][32][16];  // per wave: the upper lane half's two rows, for the lower half
  const uint32_t lane = threadIdx.x & 63, L = lane & 31, hi = lane >> 5, w = threadIdx.x >> 6;
  for (uint32_t i0 = blockIdx.x * 4u; i0 < n; i0 += gridDim.x * 4u) {
    const uint32_t i = i0 + w;
    const bool valid = i < n;
    const uint32_t P = list[valid ? i : i0];
    uint32_t dP[4];
#pragma unroll
    for (int j = 0; j < 4; j++) dP[j] = j < NO ? (P >> g.shift[j]) & (g.base[j] - 1u) : 0u;
    // visit 1: channel (hi, half) = outer digit j = 2 hi + half, plane Q_j = P - e_j
    const uint32_t jx = 2 * hi, jy = 2 * hi + 1;
    const bool hx = (int)jx < NO && dP[jx] >= 1, hy = (int)jy < NO && dP[jy] >= 1;
    const uint32_t qx = hx ? P - g.stride[jx] : 0u, qy = hy ? P - g.stride[jy] : 0u;
    uint32_t dx[4], dy[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      dx[j] = j < NO ? (qx >> g.shift[j]) & (g.base[j] - 1u) : 0u;
      dy[j] = j < NO ? (qy >> g.shift[j]) & (g.base[j] - 1u) : 0u;
    }
    const uint32_t primv1 = L == 0 ? (((hx && qx == 0) ? 0xFFu : 0u) | ((hy && qy == 0) ? 0xFFu << 16 : 0u)) : 0u;
    uint32_t rx[8], ry[8];
    plane_pair_wavefront(
        L, primv1,
        [&](uint32_t* Xh, uint32_t* Xl, uint32_t* Yh, uint32_t* Yl) {
#pragma unroll
          for (int j = 0; j < NO; j++)
#pragma unroll
            for (uint32_t k = 1; k <= 2; k++) {
              uint32_t a[8], b[8];
              plane_pair_row(tab, hx && dx[j] >= k, qx - k * g.stride[j], L, zero, a);
              plane_pair_row(tab, hy && dy[j] >= k, qy - k * g.stride[j], L, zero, b);
              plane_pair_fold(Xh, Xl, Yh, Yl, a, b);
            }
        },
        rx, ry);
    // Q_j's one writer: every digit of P below j at its top value
    auto writer = [&](uint32_t j) {
      bool ok = true;
#pragma unroll
      for (uint32_t t = 0; t < 4; t++) ok = ok && (t >= j || dP[t] == g.base[t] - 1u);
      return ok;
    };
    if (valid && hx && writer(jx)) plane_pair_store(tab, qx, L, rx);
    if (valid && hy && writer(jy)) plane_pair_store(tab, qy, L, ry);
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
    __syncthreads();  // (the next item's writes)
    // visit 2: P in the lower lane half's low channel; the other channels idle
    const uint32_t primv2 = (L == 0 && P == 0) ? 0xFFu : 0u;
    uint32_t rp[8], rz[8];
    plane_pair_wavefront(
        L, primv2,
        [&](uint32_t* Xh, uint32_t* Xl, uint32_t* Yh, uint32_t* Yl) {
          uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0}, a[8], r0[8], r1[8];
#pragma unroll
          for (int d = 0; d < 8; d++) {
            r0[d] = hx ? rx[d] : 0u;  // (lower half: Q_0, Q_1)
            r1[d] = hy ? ry[d] : 0u;
          }
          plane_pair_fold(Xh, Xl, Yh, Yl, r0, z);
          plane_pair_fold(Xh, Xl, Yh, Yl, r1, z);
          plane_pair_fold(Xh, Xl, Yh, Yl, q2, z);
          plane_pair_fold(Xh, Xl, Yh, Yl, q3, z);
#pragma unroll
          for (int j = 0; j < NO; j++) {
            plane_pair_row(tab, dP[j] >= 2, P - 2 * g.stride[j], L, zero, a);
            plane_pair_fold(Xh, Xl, Yh, Yl, a, z);
          }
        },
        rp, rz);
    if (valid && !hi) plane_pair_store(tab, P, L, rp);
  }
}

// Forward pass: the reach map and the counts.  Moves act on one heap at a
// time and the only primitive (every heap 0) has no moves, so the positions
// reachable from the root are the product of each heap's values reachable by
// its own moves (x -> x-1 for x >= 1, x -> x-2 for x >= 2: every value up to
// the start, rlim[i]).  A reached row (plane P, heap-1 value h1) therefore
// holds exactly the positions h0 = 0..rlim[0], and the map keeps ONE bit per
// row: bit h1 of the 32-bit word bits[P] (4 MiB -> 128 KiB on the 2^30
// table; k_plane_reach 26 -> a few us).  plane_row_bits expands it back to
// the row's 32 position bits for the readers.  One thread per plane (its
// digits decoded once for 32 rows); counts per block into its BlockCount
// slot (block_count), summed once per solve (k_fill_red).
__host__ __device__ __forceinline__ uint32_t plane_row_full(const PlaneGeom& g) {
  return g.rlim[0] >= 31 ? 0xFFFFFFFFu : ((2u << g.rlim[0]) - 1u);
}

// the position bits (bit h0) of local row (P, h1): the full row or none
__device__ __forceinline__ uint32_t plane_row_bits(const uint32_t* __restrict__ bits, const PlaneGeom& g, uint64_t P,
                                                   uint32_t h1) {
  return ((bits[P] >> h1) & 1u) ? plane_row_full(g) : 0u;
}

template <int NO, class CountFn>
__device__ __forceinline__ void plane_reach_body(uint32_t* __restrict__ bits, const PlaneGeom& g, CountFn count) {
  const uint32_t full = plane_row_full(g);
  const uint32_t c = __builtin_popcount(full), c12 = __builtin_popcount(full >> 1) + __builtin_popcount(full >> 2);
  // rows this shard reaches in a reached plane: heap-1 values h1off + h1 <= rlim[1]
  const uint32_t nrow = g.rlim[1] >= g.h1off ? (g.rlim[1] - g.h1off + 1u < 32u ? g.rlim[1] - g.h1off + 1u : 32u) : 0u;
  const uint32_t rows = nrow >= 32u ? 0xFFFFFFFFu : ((1u << nrow) - 1u);
  // edges of a reached plane's rows without the outer heaps: sum over its rows
  // of c * min(h1 + h1off, 2) + c12
  uint64_t e01 = 0;
  for (uint32_t h1 = 0; h1 < nrow; h1++) {
    const uint32_t v = h1 + g.h1off;
    e01 += (uint64_t)c * (v < 2 ? v : 2u) + c12;
  }
  uint64_t npos = 0, edges = 0;
  for (uint64_t P = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; P < g.nplanes;
       P += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t dig[NO > 0 ? NO : 1];
    plane_global_digits<NO>(g, (uint32_t)P, dig);
    bool in = true;
    uint32_t ext = 0;  // moves of the heaps other than heaps 0 and 1
#pragma unroll
    for (int j = 0; j < NO; j++) {
      in = in && dig[j] <= g.rlim[2 + j];
      ext += dig[j] < 2 ? dig[j] : 2u;
    }
    bits[P] = in ? rows : 0u;
    if (in) {
      npos += (uint64_t)c * nrow;
      edges += (uint64_t)c * nrow * ext + e01;
    }
  }
  count(npos, edges);
}

}  // namespace gm
