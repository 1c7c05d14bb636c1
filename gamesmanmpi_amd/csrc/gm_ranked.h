// gm_ranked.h -- RANKED layout (GM_MODE_RANKED): toot_and_otto_bitstring
// positions at COMPUTED indices -- no keys stored, no dedup, no hash.
// Included by gm_solver.hip after the solver object, the count helpers and
// the keyed layouts (inside its extern "C" block: templates need C++ linkage,
// see the extern "C++" below).
//
// Replaces, for toot-and-otto, the keyed pipeline of the reference's
// per-position job loop (src/process.py:109-267: expand, look up, dedup in
// the resolved/remote CacheDicts, resolve) the way PLANES replaces it for the
// sum game: the state space is rank-indexable.  A position is
//   * per column x: its height h_x in [0, H] and the letters of its stack,
//     bit y = 1 for T (gravity: do_move fills the lowest blank cell,
//     toot_and_otto_bitstring.py:106-116, so a column is a contiguous stack);
//   * a = how many T's the first mover has placed, in [0, 6].
// Everything else in the key follows: pieces on the board L = sum h_x (the
// level; the first mover moves at even L), the T's on the board nT (the
// popcount of the stacks), hence every hand (6 each at the start, :38-40:
// first mover T = 6 - a, O = 6 - (ceil(L/2) - a); second mover T =
// 6 - (nT - a), O = 6 - (floor(L/2) - (nT - a))) and the turn bit.  The
// first mover is the reference's player 2: is_player1_turn reads board[-1]
// (:218-222), a padding bit that starts 0 (the key's turn bit, gm_games.h;
// the root's, gm_solver.hip), so player 2's hands (key bits 2A+6..) go first.
//
// Index space: the height vectors (h_0 .. h_{C-1}) of one level in ascending
// code order (hvcode = sum h_x (H+1)^x), each a BLOCK of 8 x 2^L slots
// [a][stack bits] -- a-major, the stacks' L bits concatenated column after
// column (column x at bits [off_x, off_x + h_x), off_x = sum_{c<x} h_c) --
// and the levels one after another, each padded to 64 slots.  toot 6x4:
// 8 x 31^6 = 7.1e9 slots, one byte of word each (value | remoteness << 2,
// remoteness <= 24) + a reach and an "expandable" bit = 8.9 GB against the
// BUCKETED layout's ~70 GB of keys, in-edges and partitions.
//
// A move in column x with letter l: child block = hvcode + (H+1)^x, child
// stack bits = the parent's with bit l inserted at off_x + h_x, a + 1 if the
// first player placed a T.  Consecutive lanes take consecutive stack bits of
// one block, so for a fixed move their children are consecutive bytes too
// (one or two lines per wave): every access is coalesced, and the only
// random access left is none.
//
// Forward, level L (pull): a slot is reached iff its hands are valid and one
// of its parents -- remove the top piece of some column -- is reached and not
// primitive ("expandable" bit); primitive = the reference rule on the key
// (toot_prim).  Backward, level L: every reached slot gathers its children's
// words (the legal moves: a column not full, a letter left in the mover's
// hand) and applies the reference reduction (_res_red/_remote_red, SURVEY
// §8a A8/A9) -- the same words, counts and fingerprint as the keyed layouts
// (tests/test_gpu_ranked.py).
extern "C++" {

constexpr uint32_t kRankHand = 6;  // every hand starts at 6 (toot_and_otto_bitstring.py:38-40)

// (RankGeom: gm_solver.hip, before the solver object that holds one)

struct RankPos {
  uint32_t h[kRankMaxCols], off[kRankMaxCols];
};
__device__ __forceinline__ void rk_unpack(const RankGeom& g, uint32_t ph, RankPos& p) {
  uint32_t o = 0;
#pragma unroll
  for (int x = 0; x < kRankMaxCols; x++) {
    p.h[x] = x < (int)g.C ? (ph >> (4 * x)) & 15u : 0u;
    p.off[x] = o;
    o += p.h[x];
  }
}
// pieces used from each hand, all in [0, 6]: the first mover's T's = a, O's =
// ceil(L/2) - a; the second mover's T's = nT - a, O's = floor(L/2) - (nT - a)
struct RankHands {
  int t1, o1, t2, o2;
};
__device__ __forceinline__ RankHands rk_hands(uint32_t L, uint32_t nT, uint32_t a) {
  RankHands u;
  u.t1 = (int)a;
  u.o1 = (int)((L + 1) / 2) - (int)a;
  u.t2 = (int)nT - (int)a;
  u.o2 = (int)(L / 2) - u.t2;
  return u;
}
__device__ __forceinline__ bool rk_valid(const RankHands& u) {
  return u.t1 >= 0 && u.t1 <= (int)kRankHand && u.o1 >= 0 && u.o1 <= (int)kRankHand && u.t2 >= 0 &&
         u.t2 <= (int)kRankHand && u.o2 >= 0 && u.o2 <= (int)kRankHand;
}
// the toot key (gm_games.h layout) of a slot with valid hands
__device__ __forceinline__ u64 rk_key(const RankGeom& g, const RankPos& p, uint32_t pat, uint32_t L, const RankHands& u) {
  u64 t = 0, o = 0;
#pragma unroll
  for (int x = 0; x < kRankMaxCols; x++) {
    if (x >= (int)g.C) break;
    const uint32_t hb = p.h[x], col = (pat >> p.off[x]) & ((1u << hb) - 1u);
    for (uint32_t y = 0; y < hb; y++) {
      const u64 cell = 1ull << (g.C * y + (uint32_t)x);
      if ((col >> y) & 1u) t |= cell;
      else o |= cell;
    }
  }
  // key hands: player 1 (the second mover) at 2A, 2A+3; player 2 (the first
  // mover) at 2A+6, 2A+9; turn bit 1 = player 1 to move = odd levels
  const uint32_t A = g.A;
  return t | (o << A) | ((u64)(kRankHand - u.t2) << (2 * A)) | ((u64)(kRankHand - u.o2) << (2 * A + 3)) |
         ((u64)(kRankHand - u.t1) << (2 * A + 6)) | ((u64)(kRankHand - u.o1) << (2 * A + 9)) |
         ((u64)(L & 1u) << (2 * A + 12));
}
// key -> slot (false: not a gravity board with consistent hands)
__device__ __forceinline__ bool rk_slot_of(const RankGeom& g, u64 key, u64* slot, uint32_t* level) {
  const uint32_t A = g.A;
  const u64 full = (A >= 64) ? ~0ull : ((1ull << A) - 1);
  const u64 t = key & full, o = (key >> A) & full;
  if (t & o) return false;
  if (key >> (2 * A + 13)) return false;
  uint32_t hv = 0, pat = 0, L = 0;
  for (uint32_t x = 0; x < g.C; x++) {
    uint32_t h = 0;
    while (h < g.H && (((t | o) >> (g.C * h + x)) & 1)) h++;
    for (uint32_t y = h; y < g.H; y++)
      if (((t | o) >> (g.C * y + x)) & 1) return false;  // a gap under a piece
    for (uint32_t y = 0; y < h; y++) pat |= (uint32_t)((t >> (g.C * y + x)) & 1) << (L + y);
    hv += h * g.stride[x];
    L += h;
  }
  const uint32_t nT = __builtin_popcount(pat);
  // second mover (player 1) at 2A, first mover (player 2) at 2A+6 (rk_key)
  const uint32_t sT = (uint32_t)((key >> (2 * A)) & 7), sO = (uint32_t)((key >> (2 * A + 3)) & 7);
  const uint32_t fT = (uint32_t)((key >> (2 * A + 6)) & 7), fO = (uint32_t)((key >> (2 * A + 9)) & 7);
  const uint32_t turn = (uint32_t)((key >> (2 * A + 12)) & 1);
  if (fT > kRankHand) return false;
  const uint32_t a = kRankHand - fT;
  const RankHands u = rk_hands(L, nT, a);
  if (!rk_valid(u) || kRankHand - u.o1 != fO || kRankHand - u.t2 != sT || kRankHand - u.o2 != sO ||
      turn != (L & 1u))
    return false;
  *slot = g.base[hv] + ((u64)a << L) + pat;
  *level = L;
  return true;
}

// The level's slots as one index space: item i of level L = slot lvstart + i,
// block i >> (L + 3) of the level's list (lvoff + that), a = (i >> L) & 7,
// stack bits = i & (2^L - 1).  Levels start 512-aligned, so a level's boards
// (the a = 0 view: board lvstart / 8 + (i >> (L + 3) << L) + bits) start
// 64-aligned and every 64-slot / 64-board word belongs to one level.

// The t / o planes of a board from its stacks.  C > H: a column's h <= H
// bits land on cells x + C y by one multiply (bit y times 2^((C-1) y) sits at
// C y; no two products meet), else a loop.
template <int CC, int HH>
__device__ __forceinline__ u64 rk_board_key(const RankGeom& g, uint32_t ph, uint32_t pat, uint32_t L) {
  u64 t = 0, o = 0;
  uint32_t off = 0;
  if constexpr (CC > HH && CC * HH <= 32) {
    constexpr uint32_t mul = [] {
      uint32_t m = 0;
      for (int y = 0; y < HH; y++) m |= 1u << ((CC - 1) * y);
      return m;
    }();
    constexpr uint32_t msk = [] {
      uint32_t m = 0;
      for (int y = 0; y < HH; y++) m |= 1u << (CC * y);
      return m;
    }();
    uint32_t t32 = 0, o32 = 0;
#pragma unroll
    for (int x = 0; x < CC; x++) {
      const uint32_t h = (ph >> (4 * x)) & 15u, full = (1u << h) - 1u;
      const uint32_t col = (pat >> off) & full;
      off += h;
      t32 |= ((col * mul) & msk) << x;
      o32 |= (((~col & full) * mul) & msk) << x;
    }
    t = t32;
    o = o32;
  } else {
    for (uint32_t x = 0; x < g.C; x++) {
      const uint32_t h = (ph >> (4 * x)) & 15u, col = (pat >> off) & ((1u << h) - 1u);
      off += h;
      for (uint32_t y = 0; y < h; y++) {
        const u64 cell = 1ull << (g.C * y + x);
        if ((col >> y) & 1u) t |= cell;
        else o |= cell;
      }
    }
  }
  return t | (o << g.A) | ((u64)(L & 1u) << (2 * g.A + 12));  // hands: unread by the rule
}

// F0: every board of level L (its stacks; the hands do not enter the rule):
// the reference's primitive value (toot_prim) or UNDECIDED in bstat, and the
// primitive bit in pbits.  One thread per board; a wave = one pbits word.
template <int KIND, int CC, int HH>
__global__ __launch_bounds__(256) void k_rk_boards(Desc d, RankGeom g, uint32_t L, u64 bstart, uint32_t lvoff,
                                                   u64 nboards, u64 nreal) {
  const uint32_t lane = threadIdx.x & 63;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i0 = (u64)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); i0 < nboards; i0 += stride) {
    const u64 i = i0 + lane;
    bool prim = false;
    if (i < nreal) {
      const u64 blk = i >> L;
      const uint32_t pat = (uint32_t)(i & ((1ull << L) - 1));
      const int pr = Game<KIND>::prim(d, rk_board_key<CC, HH>(g, g.lvph[lvoff + blk], pat, L));
      g.bstat[bstart + i] = (uint8_t)pr;
      prim = pr != UNDECIDED;
    }
    const u64 bp = __ballot(prim);
    if (lane == 0) reinterpret_cast<u64*>(g.pbits)[(bstart + i0) >> 6] = bp;
  }
}

// F0, bit-sliced (boards of <= 32 cells with <= 31 windows: the BASELINE 6x4
// and the 5x4 / 4x4 test boards; levels L >= 5): a thread takes 32 boards of
// one block -- stack patterns pat0 + b, b = 0..31 -- as bit b of 32-bit words.
// Cell (x, y) holds stack bit j = off_x + y, and across the 32 boards that
// bit is the constant 0xAAAAAAAA, 0xCCCCCCCC, .. for j < 5 and all-zero / all-
// one from pat0 above; a window's TOOT (OTTO) bits are the AND of its four
// cells' T / O words, the counts are a Harley-Seal carry-save sum of the
// window words (v_bitop3: one instruction per sum, one per carry), and the
// comparison is a 5-bit bit-sliced one.  bstat bytes and pbits words come
// out as k_rk_boards writes them (tests/test_gpu_ranked.py: word for word
// against BUCKETED; the 5x4 / 6x4 goldens).  ~15 operations a board where
// the per-board kernel issues ~150.
template <int CC, int HH>
struct RkWindows {
  static constexpr int NC = CC * HH;
  int n = 0, c[64] = {}, s[64] = {};
  constexpr RkWindows() {
    const int dxs[4] = {1, 0, 1, 1}, dys[4] = {0, 1, 1, -1};
    for (int i = 0; i < 4; i++)
      for (int y = 0; y < HH; y++)
        for (int x = 0; x < CC; x++) {
          const int ex = x + 3 * dxs[i], ey = y + 3 * dys[i];
          if (ex >= 0 && ex < CC && ey >= 0 && ey < HH) {
            c[n] = CC * y + x;
            s[n] = dxs[i] + CC * dys[i];
            n++;
          }
        }
  }
};
// v_bitop3_b32 truth tables over (a, b, c) = (0xF0, 0xCC, 0xAA)
__device__ __forceinline__ uint32_t rk_xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t rk_maj(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}
__device__ __forceinline__ uint32_t rk_and3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x80);
}
// Harley-Seal: the 5-bit bit-sliced count of up to 32 window words (zeros fold away)
__device__ __forceinline__ void rk_count32(const uint32_t (&x)[32], uint32_t (&cnt)[5]) {
  uint32_t ones = 0, twos = 0, fours = 0, eights = 0, sixteens = 0;
#pragma unroll
  for (int i = 0; i < 32; i += 16) {
    uint32_t twosA, twosB, foursA, foursB, eightsA, eightsB, t;
    auto csa = [](uint32_t& h, uint32_t& l, uint32_t a, uint32_t b, uint32_t c) {
      h = rk_maj(a, b, c);
      l = rk_xor3(a, b, c);
    };
    csa(twosA, ones, ones, x[i + 0], x[i + 1]);
    csa(twosB, ones, ones, x[i + 2], x[i + 3]);
    csa(foursA, twos, twos, twosA, twosB);
    csa(twosA, ones, ones, x[i + 4], x[i + 5]);
    csa(twosB, ones, ones, x[i + 6], x[i + 7]);
    csa(foursB, twos, twos, twosA, twosB);
    csa(eightsA, fours, fours, foursA, foursB);
    csa(twosA, ones, ones, x[i + 8], x[i + 9]);
    csa(twosB, ones, ones, x[i + 10], x[i + 11]);
    csa(foursA, twos, twos, twosA, twosB);
    csa(twosA, ones, ones, x[i + 12], x[i + 13]);
    csa(twosB, ones, ones, x[i + 14], x[i + 15]);
    csa(foursB, twos, twos, twosA, twosB);
    csa(eightsB, fours, fours, foursA, foursB);
    csa(t, eights, eights, eightsA, eightsB);
    sixteens |= t;  // the total is <= 31: one sixteen at most
  }
  cnt[0] = ones, cnt[1] = twos, cnt[2] = fours, cnt[3] = eights, cnt[4] = sixteens;
}
template <int CC, int HH>
__global__ __launch_bounds__(256) void k_rk_boards_sl(RankGeom g, uint32_t L, u64 bstart, uint32_t lvoff,
                                                      u64 nslices, u64 nreal) {
  constexpr RkWindows<CC, HH> W{};
  static_assert(CC * HH <= 32 && W.n <= 31, "bit-sliced boards: <= 32 cells, <= 31 windows");
  constexpr int NCELL = CC * HH;
  // stack bit j's word over the 32 boards for j < 5 (0 above: pat0 gives those)
  __shared__ uint32_t kLow[32];
  if (threadIdx.x < 32) {
    const uint32_t j = threadIdx.x;
    kLow[j] = j == 0 ? 0xAAAAAAAAu : j == 1 ? 0xCCCCCCCCu : j == 2 ? 0xF0F0F0F0u : j == 3 ? 0xFF00FF00u
              : j == 4 ? 0xFFFF0000u : 0u;
  }
  __syncthreads();
  const bool p1 = (L & 1u) != 0, full = L == (uint32_t)NCELL;
  const uint32_t eqv = full ? 1u : 2u;  // eq -> TIE (2) on a full board, else UNDECIDED (4)
  for (u64 sl = (u64)blockIdx.x * blockDim.x + threadIdx.x; sl < nslices; sl += (u64)gridDim.x * blockDim.x) {
    const u64 ib0 = sl << 5;
    uint32_t pm = 0;
    if (ib0 < nreal) {
      const u64 blk = ib0 >> L;
      const uint32_t pat0 = (uint32_t)(ib0 & ((1ull << L) - 1));
      const uint32_t ph = g.lvph[lvoff + blk];
      uint32_t Tm[NCELL], Om[NCELL];
      uint32_t off = 0;
#pragma unroll
      for (int x = 0; x < CC; x++) {
        const uint32_t h = (ph >> (4 * x)) & 15u, hm = (1u << h) - 1u;
#pragma unroll
        for (int y = 0; y < HH; y++) {
          const uint32_t j = (off + (uint32_t)y) & 31u;
          // bits >= 5 of the stacks: pat0's, the same for all 32 (all 0 / all 1)
          const uint32_t S = kLow[j] | (uint32_t)__builtin_amdgcn_sbfe((int)pat0, j, 1);
          const uint32_t vm = (uint32_t)__builtin_amdgcn_sbfe((int)hm, y, 1);  // cell (x, y) occupied
          Tm[CC * y + x] = S & vm;
          Om[CC * y + x] = ~S & vm;
        }
        off += h;
      }
      uint32_t xt[32], xo[32];
#pragma unroll
      for (int w = 0; w < 32; w++) {
        if (w < W.n) {
          const int c = W.c[w], st = W.s[w];
          xt[w] = rk_and3(Tm[c], Om[c + st], Om[c + 2 * st]) & Tm[c + 3 * st];
          xo[w] = rk_and3(Om[c], Tm[c + st], Tm[c + 2 * st]) & Om[c + 3 * st];
        } else {
          xt[w] = xo[w] = 0;
        }
      }
      uint32_t ct[5], co[5];
      rk_count32(xt, ct);
      rk_count32(xo, co);
      // bit-sliced compare, least significant bit first
      uint32_t gt = ct[0] & ~co[0], eq = ~(ct[0] ^ co[0]);
#pragma unroll
      for (int k = 1; k < 5; k++) {
        // gt' = t & ~o | ~(t ^ o) & gt over (t, o, gt): table 0xB2; eq' = eq & ~(t ^ o) over (eq, t, o): 0x90
        gt = __builtin_amdgcn_bitop3_b32(ct[k], co[k], gt, 0xB2);
        eq = __builtin_amdgcn_bitop3_b32(eq, ct[k], co[k], 0x90);
      }
      // toot_prim: equal counts -> TIE on a full board, else UNDECIDED;
      // otherwise LOSS iff (toot > otto) != p1, else WIN (gm_games.h)
      const uint32_t loss = ~eq & (p1 ? ~gt : gt);
      pm = full ? ~0u : ~eq;
      uint32_t by[8];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint32_t e4 = (eq >> (4 * k)) & 15u, l4 = (loss >> (4 * k)) & 15u;
        const uint32_t es = (e4 * 0x00204081u) & 0x01010101u;
        const uint32_t ls = (l4 * 0x00204081u) & 0x01010101u;
        by[k] = (es << eqv) | ls;  // WIN 0 / LOSS 1 / TIE 2 / UNDECIDED 4
      }
      uint4* bp = reinterpret_cast<uint4*>(g.bstat + bstart + ib0);
      bp[0] = make_uint4(by[0], by[1], by[2], by[3]);
      bp[1] = make_uint4(by[4], by[5], by[6], by[7]);
    }
    reinterpret_cast<uint32_t*>(g.pbits)[(bstart + ib0) >> 5] = pm;
  }
}

// bits j of a 64-slot word (consecutive stack bits p0 + j, p0 a multiple of
// 64) whose hands are valid: nT = popc(p0) + popc(j) in [lo, hi]
__device__ __forceinline__ u64 rk_valid_mask(const RankGeom& g, uint32_t L, uint32_t a, uint32_t p0) {
  if (a > kRankHand) return 0;
  const int o1 = (int)((L + 1) / 2) - (int)a;
  if (o1 < 0 || o1 > (int)kRankHand) return 0;
  const int half = (int)(L / 2);
  const int lo = (int)a + max(0, half - (int)kRankHand) - __builtin_popcount(p0);
  const int hi = (int)a + min((int)kRankHand, half) - __builtin_popcount(p0);
  if (hi < 0 || lo > 6) return 0;
  const u64 up = hi >= 6 ? ~0ull : g.le[hi];
  const u64 dn = lo <= 0 ? 0ull : g.le[lo - 1];
  return up & ~dn;
}
// 32 bits -> 64: insert a 0 at bit q of every index (runs of 2^q bits, each
// followed by a gap of 2^q)
__device__ __forceinline__ u64 rk_spread(uint32_t e, uint32_t q) {
  u64 x = e;
  if (q <= 4) x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
  if (q <= 3) x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
  if (q <= 2) x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
  if (q <= 1) x = (x | (x << 2)) & 0x3333333333333333ull;
  if (q == 0) x = (x | (x << 1)) & 0x5555555555555555ull;
  return x;
}

// F1 (levels L >= 6): reach and expandable bits 64 slots at a time -- a slot
// is reached iff its hands are valid and a parent (its stacks with one
// column's top piece removed, the first mover's T count one lower if it
// placed that T) is expandable.  For a column whose top sits at bit q >= 6 of
// the stacks the 64 slots' parents are 64 consecutive slots (one word); for
// q < 6 the children with letter l at bit q have 32 consecutive parents, half
// a word, spread back to the child bits (rk_spread).  expandable = reached
// and not a primitive board (pbits).
// Four consecutive words per thread per step (a height-vector block is >= 8
// words at L >= 6, so an aligned group of four shares one block, its metadata
// and its parents' bases): the four words' parent loads are in flight
// together instead of one word's three dependent round trips (block metadata
// -> parent base -> parent bits) after another -- the toot 6x4 forward
// 2.01 -> 1.91 ms against one word per thread (round 5, tools/rk_anatomy.sh).
// (nwords: the level's 512-slot padded extent in words -- every bitmap word
// of the level is written, the padding's as 0; nreal: its slots)
__global__ __launch_bounds__(256) void k_rk_reach4(RankGeom g, uint32_t L, u64 lvstart, uint32_t lvoff, u64 nwords,
                                                   u64 nreal, BlockCount* bc, DevState* st, u64 plvstart) {
  u64 npos = 0, prims = 0;
  const bool fmoved = ((L - 1) & 1u) == 0;  // the move into level L was the first mover's
  for (u64 w0 = ((u64)blockIdx.x * blockDim.x + threadIdx.x) * 4; w0 < nwords; w0 += (u64)gridDim.x * blockDim.x * 4) {
    const u64 b0 = w0 << 6;
    u64* rout = reinterpret_cast<u64*>(g.reach) + ((lvstart + b0) >> 6);
    u64* xout = reinterpret_cast<u64*>(g.expd) + ((lvstart + b0) >> 6);
    if (b0 >= nreal) {  // padding (nreal: whole blocks, a multiple of four words)
      reinterpret_cast<uint4*>(rout)[0] = reinterpret_cast<uint4*>(rout)[1] = make_uint4(0, 0, 0, 0);
      reinterpret_cast<uint4*>(xout)[0] = reinterpret_cast<uint4*>(xout)[1] = make_uint4(0, 0, 0, 0);
      continue;
    }
    const u64 blk = b0 >> (L + 3);
    RankPos p;
    rk_unpack(g, g.lvph[lvoff + blk], p);
    // the parent blocks' offsets (lvpa), loaded beside the stacks: two
    // dependent round trips per group (metadata, parent bits) instead of
    // three (hvcode, parent base, parent bits)
    const uint4* pp = reinterpret_cast<const uint4*>(g.lvpa + (u64)(lvoff + blk) * kRankMaxCols);
    const uint4 pa0 = pp[0], pa1 = pp[1];
    const uint32_t pao[kRankMaxCols] = {pa0.x, pa0.y, pa0.z, pa0.w, pa1.x, pa1.y, pa1.z, pa1.w};
    uint32_t a[4], p0[4];
    u64 valid[4], r[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const u64 i0 = b0 + ((u64)k << 6);
      a[k] = (uint32_t)((i0 >> L) & 7u);
      p0[k] = (uint32_t)(i0 & ((1ull << L) - 1));
      valid[k] = rk_valid_mask(g, L, a[k], p0[k]);
      r[k] = 0;
    }
#pragma unroll
    for (int x = 0; x < kRankMaxCols; x++) {
      if (x >= (int)g.C || p.h[x] == 0) continue;
      const uint32_t q = p.off[x] + p.h[x] - 1;
      const u64 pb = plvstart + pao[x];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (!valid[k]) continue;
        if (q >= 6) {
          const uint32_t l = (p0[k] >> q) & 1u;
          if (fmoved && l && a[k] == 0) continue;
          const uint32_t pa = a[k] - (fmoved && l ? 1u : 0u);
          const uint32_t pp0 = (p0[k] & ((1u << q) - 1u)) | ((p0[k] >> (q + 1)) << q);
          r[k] |= reinterpret_cast<const u64*>(g.expd)[(pb + ((u64)pa << (L - 1)) + pp0) >> 6];
        } else {
#pragma unroll
          for (uint32_t l = 0; l < 2; l++) {
            if (fmoved && l && a[k] == 0) continue;
            const uint32_t pa = a[k] - (fmoved && l ? 1u : 0u);
            const u64 ps0 = pb + ((u64)pa << (L - 1)) + (p0[k] >> 1);  // a multiple of 32
            r[k] |= rk_spread(g.expd[ps0 >> 5], q) << (l << q);
          }
        }
      }
    }
    u64 e[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      r[k] &= valid[k];
      const u64 pm = reinterpret_cast<const u64*>(g.pbits)[((lvstart >> 3) + (blk << L) + p0[k]) >> 6];
      e[k] = r[k] & ~pm;
      npos += (u64)__builtin_popcountll(r[k]);
      prims += (u64)__builtin_popcountll(r[k] & pm);
    }
    reinterpret_cast<uint4*>(rout)[0] = make_uint4((uint32_t)r[0], (uint32_t)(r[0] >> 32), (uint32_t)r[1], (uint32_t)(r[1] >> 32));
    reinterpret_cast<uint4*>(rout)[1] = make_uint4((uint32_t)r[2], (uint32_t)(r[2] >> 32), (uint32_t)r[3], (uint32_t)(r[3] >> 32));
    reinterpret_cast<uint4*>(xout)[0] = make_uint4((uint32_t)e[0], (uint32_t)(e[0] >> 32), (uint32_t)e[1], (uint32_t)(e[1] >> 32));
    reinterpret_cast<uint4*>(xout)[1] = make_uint4((uint32_t)e[2], (uint32_t)(e[2] >> 32), (uint32_t)e[3], (uint32_t)(e[3] >> 32));
  }
  block_count(bc, npos, 0);
  block_add(&st->prims, prims);
}

// F1 for levels L < 6 (blocks narrower than a word): one thread per slot
// (nitems: the level's slots rounded up to 64, so every bitmap word of the
// level is written -- no clearing -- nreal: its slots)
__global__ __launch_bounds__(256) void k_rk_forward(RankGeom g, uint32_t L, u64 lvstart, uint32_t lvoff, u64 nitems,
                                                    u64 nreal, BlockCount* bc, DevState* st) {
  u64 npos = 0, prims = 0;
  const uint32_t lane = threadIdx.x & 63;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 i0 = (u64)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); i0 < nitems; i0 += stride) {
    const u64 i = i0 + lane;
    bool reach = false, ex = false;
    if (i < nreal) {
      const u64 blk = i >> (L + 3);
      const uint32_t a = (uint32_t)((i >> L) & 7u), pat = (uint32_t)(i & ((1ull << L) - 1));
      const uint32_t hvc = g.lvhv[lvoff + blk];
      RankPos p;
      rk_unpack(g, g.lvph[lvoff + blk], p);
      const RankHands u = rk_hands(L, (uint32_t)__builtin_popcount(pat), a);
      if (rk_valid(u)) {
        if (L == 0) {
          reach = true;  // the root (hands 6 / 6 / 6 / 6, the first mover to move)
        } else {
          const bool fmoved = ((L - 1) & 1u) == 0;
#pragma unroll
          for (int x = 0; x < kRankMaxCols; x++) {
            if (x >= (int)g.C || p.h[x] == 0) continue;
            const uint32_t q = p.off[x] + p.h[x] - 1, l = (pat >> q) & 1u;
            if (fmoved && l && a == 0) continue;
            const uint32_t pp = (pat & ((1u << q) - 1u)) | ((pat >> (q + 1)) << q);
            const uint32_t pa = a - (fmoved && l ? 1u : 0u);
            const u64 ps = g.base[hvc - g.stride[x]] + ((u64)pa << (L - 1)) + pp;
            if ((g.expd[ps >> 5] >> (ps & 31)) & 1u) {
              reach = true;
              break;
            }
          }
        }
        if (reach) {
          const int pr = g.bstat[(lvstart >> 3) + (blk << L) + pat];
          ex = pr == UNDECIDED;
          prims += !ex;
          npos++;
        }
      }
    }
    const u64 br = __ballot(reach), be = __ballot(ex);
    if (lane == 0) {
      const u64 w = (lvstart + i0) >> 6;  // aligned: lvstart and i0 are multiples of 64
      reinterpret_cast<u64*>(g.reach)[w] = br;
      reinterpret_cast<u64*>(g.expd)[w] = be;
    }
  }
  block_count(bc, npos, 0);
  block_add(&st->prims, prims);
}

// B: the reached slots of level L gather their children's words.  A
// workgroup takes a tile of 256 x 32 slots: each thread reads one 32-slot
// reach word, the workgroup lays the reached slots' offsets out in LDS
// (exclusive scan of the words' popcounts), then every thread resolves list
// entries -- waves carry reached slots only (about 1 in 6 of all slots on
// toot 6x4), and a primitive's value comes from bstat.  The 16 KB list lets
// 9 workgroups share a CU (then bound by VGPRs); a list of 256 x 64 slots
// (4 per CU) was slower (profiles/r05d: SQ_WAIT_ANY 59 %).
// The children's words come through a buffer resource over level L + 1: a
// move that is not legal reads an offset past the level's end, i.e. 0 = WIN
// in 0, neutral in the reduction -- so all 2C loads of an entry, two entries
// per lane, issue back to back with no branches.  CC / HH: the board at
// compile time (0: from g).  A tile inside one height-vector block (L >= 10)
// reads its block's stacks / child bases once, wave-uniform.
// md5 owners of 32 slots as three bit planes (gm_ranked_shard.h: ownb[w] =
// bits 0, 1, 2 of the owners of slots 32w .. 32w + 31 in x, y, z): bit j of
// the result = slot j's owner is v (< 8)
__device__ __forceinline__ uint32_t rko_own_mask(const uint4 o, uint32_t v) {
  return ((v & 1u) ? o.x : ~o.x) & ((v & 2u) ? o.y : ~o.y) & ((v & 4u) ? o.z : ~o.z);
}

typedef unsigned short rk_u16x2 __attribute__((ext_vector_type(2)));

// Offsets of an illegal move.  A board compiled in (CC > 0: every level
// <= 1 GiB, rank_backward_level checks) marks a full column by a child base of
// 2^30 and an empty hand by a slot base of 2^31: one add3 per child, and any
// sum holding a mark lands in [2^30, 2^32), past the level's end -- then
// clamped to 2^30, one address for every illegal move of a wave (distinct
// out-of-range addresses cost the gathers as much as real ones: toot 6x4
// backward 7.6 -> 8.9 ms without the clamp).  The generic kernel (levels up
// to 4 GB) adds with unsigned saturation instead: a mark of 2^32 - 1 stays
// there.
constexpr uint32_t kRkColMark = 0x40000000u, kRkHandMark = 0x80000000u;

// OWN (md5 shards, gm_ranked_shard.h): only the slots whose md5 owner
// (ownb: bit planes, 16 B per 32 slots) is `orank` are resolved here; the
// others arrive from their owners before the level above reads them.
// DBG (A/B timing only, the words are wrong): 1 = no gathers, 2 = no entries.
template <int CC, int HH, bool OWN = false, int DBG = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void k_rk_backward(RankGeom g, uint32_t L, u64 lvstart, uint32_t lvoff,
                                                     u64 nwords, u64 cstart, u64 csize, BlockCount* bc, DevState* st,
                                                     const uint4* __restrict__ ownb = nullptr, uint32_t orank = 0) {
  constexpr int U = 2;  // entries per lane per pass: U x 2C child loads in flight before any reduction
  constexpr int NC = CC > 0 ? CC : kRankMaxCols;
  constexpr bool NARROW = CC > 0;
  const uint32_t C = CC > 0 ? (uint32_t)CC : g.C, H = HH > 0 ? (uint32_t)HH : g.H;
  const uint32_t colmark = NARROW ? kRkColMark : 0xFFFFFFFFu, handmark = NARROW ? kRkHandMark : 0xFFFFFFFFu;
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc(g.words + cstart, 0, (int)(uint32_t)csize, 0x00020000);
  __shared__ uint16_t list[256 * 32];
  __shared__ uint4 tw[256 * 2];  // the tile's words (L >= 5): 32 B per tile word, in slot order
  __shared__ uint32_t wsum[4];
  u64 edges = 0, resolved = 0;
  uint32_t err = 0;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool fmoves = (L & 1u) == 0;  // the first mover moves at even levels
  const uint32_t dT = fmoves ? (1u << (L + 1)) : 0u;  // the first mover's T: one a-row on
  for (u64 t0 = (u64)blockIdx.x * 256; t0 < nwords; t0 += (u64)gridDim.x * 256) {
    const u64 wi = t0 + threadIdx.x;
    // the list holds the EXPANDABLE slots (reached, not primitive: one kind of
    // work per lane); the reached primitives take their board's value below
    uint32_t m = wi < nwords ? g.expd[(lvstart >> 5) + wi] : 0u;
    uint32_t mp = wi < nwords ? g.reach[(lvstart >> 5) + wi] & ~m : 0u;
    if constexpr (OWN) {
      const uint32_t om = wi < nwords ? rko_own_mask(ownb[(lvstart >> 5) + wi], orank) : 0u;
      m &= om;
      mp &= om;
      resolved += (u64)__builtin_popcount(m | mp);
    }
    // the reached primitives take their board's value (process.py:120-123).
    // From L = 5 on, a 32-slot word's slots are 32 consecutive boards (one
    // block, one a): their bstat bytes -- bstat's byte is the word
    // (remoteness 0) -- come in as two 16-B loads into the tile's LDS row,
    // the entries below write the expandable slots' bytes into the same row,
    // and the row goes out whole (two 16-B stores) once the tile is resolved:
    // no byte store reaches memory, the unreached slots' bytes are never
    // read.  A loop of one dependent load and store per primitive cost 2.6 of
    // the 10.3 ms backward (GM_RK_DBG A/B, round 5).
    const bool rows = L >= 5;
    if (rows) {
      if (mp) {
        const u64 i0 = wi << 5, blk = i0 >> (L + 3);
        const uint32_t pat0 = (uint32_t)(i0 & ((1ull << L) - 1));
        const uint4* src = reinterpret_cast<const uint4*>(g.bstat + (lvstart >> 3) + (blk << L) + pat0);
        const uint4 v0 = src[0], v1 = src[1];
        tw[2 * threadIdx.x] = v0;
        tw[2 * threadIdx.x + 1] = v1;
      }
    } else {
      for (uint32_t pm = mp; pm; pm &= pm - 1) {
        const u64 i = (wi << 5) + (u64)__builtin_ctz(pm);
        const u64 blk = i >> (L + 3);
        const uint32_t pat = (uint32_t)(i & ((1ull << L) - 1));
        g.words[lvstart + i] = (uint8_t)make_word(g.bstat[(lvstart >> 3) + (blk << L) + pat], 0);
      }
    }
    // exclusive scan of the popcounts over the workgroup
    const uint32_t c = (uint32_t)__builtin_popcount(m);
    uint32_t incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(incl, o);
      if (lane >= (uint32_t)o) incl += y;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (uint32_t k = 0; k < 4; k++) {
      if (k < wv) before += wsum[k];
      total += wsum[k];
    }
    uint32_t at = before + incl - c;
    for (uint32_t mm = m; mm; mm &= mm - 1) list[at++] = (uint16_t)(threadIdx.x * 32 + __builtin_ctz(mm));
    // one block for the whole tile: its stacks and child bases, read once
    const u64 tb0 = (t0 << 5) >> (L + 3);
    const bool oneblk = ((((t0 + 255) << 5) + 31) >> (L + 3)) == tb0;
    uint32_t tph = 0, tcho[kRankMaxCols] = {};
    if (oneblk) {
      tph = g.lvph[lvoff + tb0];
      const uint4* cp = reinterpret_cast<const uint4*>(g.lvch + (u64)(lvoff + tb0) * kRankMaxCols);
      const uint4 c0 = cp[0], c1 = cp[1];
      tcho[0] = c0.x, tcho[1] = c0.y, tcho[2] = c0.z, tcho[3] = c0.w;
      tcho[4] = c1.x, tcho[5] = c1.y, tcho[6] = c1.z, tcho[7] = c1.w;
    }
    __syncthreads();
    // A tile inside one block knows its full columns (wave-uniform): it runs
    // a copy of the pass over its NV columns with room only, compacted in
    // order (base cb[k], top bit cq[k]) -- no loads or reduction for a full
    // column, whose move is illegal for every slot of the tile (at the deep
    // levels two to three of six).  Other tiles run the NC-column pass with
    // per-lane stacks, a full column's offsets at the mark.
    uint32_t nv = 0, cb[NC], cq[NC];
    {
      uint32_t off = 0;
#pragma unroll
      for (int x = 0; x < NC; x++) {
        const uint32_t h = (tph >> (4 * x)) & 15u, q = off + h;
        off += h;
        const bool col = (CC > 0 || (uint32_t)x < C) && h < H;
#pragma unroll
        for (int k = 0; k <= x; k++)
          if (col && nv == (uint32_t)k) cb[k] = tcho[x], cq[k] = q;
        nv += col ? 1u : 0u;
      }
#pragma unroll
      for (int k = 0; k < NC; k++)
        if ((uint32_t)k >= nv) cb[k] = colmark, cq[k] = 0u;  // (the NC-column copy's extra columns: marked)
    }
    auto pass = [&](auto NVc, const uint32_t e0, const bool uni) {
      constexpr int NV = decltype(NVc)::value;
      uint32_t offu[U][2 * NV], nchu[U];
      u64 slotu[U];
      bool liveu[U];
      // the children's offsets: lo | hi (the stacks with a 0 inserted at bit
      // q = the column's top) is pat + (pat & ~(2^q - 1)); the T child adds
      // 2^q and, if the first mover placed it, one a-row (dT).  Per column:
      // its child base (or colmark when full) and 2^q; per entry: the slot's
      // own part for the O and the T children (or handmark when that hand is
      // empty)
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t e = e0 + 256u * (uint32_t)u;
        liveu[u] = e < total;
        const u64 i = (t0 << 5) + list[liveu[u] ? e : e0];
        slotu[u] = lvstart + i;
        const u64 blk = i >> (L + 3);
        const uint32_t a = (uint32_t)((i >> L) & 7u), pat = (uint32_t)(i & ((1ull << L) - 1));
        const RankHands h_ = rk_hands(L, (uint32_t)__builtin_popcount(pat), a);
        const bool hasT = fmoves ? h_.t1 < (int)kRankHand : h_.t2 < (int)kRankHand;
        const bool hasO = fmoves ? h_.o1 < (int)kRankHand : h_.o2 < (int)kRankHand;
        const uint32_t rp = (a << (L + 1)) + pat;
        const uint32_t bO = hasO ? rp : handmark, bT = hasT ? rp + dT : handmark;
        uint32_t ncol = 0;
        if (uni) {
#pragma unroll
          for (int k = 0; k < NV; k++) {
            const uint32_t q = cq[k], base = cb[k], hi = pat & (0xFFFFFFFFu << q);
            if constexpr (NARROW) {
              offu[u][2 * k] = min(base + (1u << q) + hi + bT, kRkColMark);
              offu[u][2 * k + 1] = min(base + hi + bO, kRkColMark);
            } else {
              const uint32_t bh = __builtin_elementwise_add_sat(base, hi);
              offu[u][2 * k] = __builtin_elementwise_add_sat(__builtin_elementwise_add_sat(bh, 1u << q), bT);
              offu[u][2 * k + 1] = __builtin_elementwise_add_sat(bh, bO);
            }
          }
          ncol = nv;
        } else {
          const uint32_t ph = g.lvph[lvoff + blk];
          const uint4* cp = reinterpret_cast<const uint4*>(g.lvch + (u64)(lvoff + blk) * kRankMaxCols);
          const uint4 c0 = cp[0], c1 = cp[1];
          const uint32_t cho[kRankMaxCols] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
          uint32_t off = 0;
#pragma unroll
          for (int x = 0; x < NV; x++) {
            const uint32_t h = (ph >> (4 * x)) & 15u;
            const bool col = (CC > 0 || (uint32_t)x < C) && h < H;
            const uint32_t q = off + h;
            off += h;
            const uint32_t base = col ? cho[x] : colmark, hi = pat & (0xFFFFFFFFu << q);
            if constexpr (NARROW) {
              offu[u][2 * x] = min(base + (1u << q) + hi + bT, kRkColMark);
              offu[u][2 * x + 1] = min(base + hi + bO, kRkColMark);
            } else {
              const uint32_t bh = __builtin_elementwise_add_sat(base, hi);
              offu[u][2 * x] = __builtin_elementwise_add_sat(__builtin_elementwise_add_sat(bh, 1u << q), bT);
              offu[u][2 * x + 1] = __builtin_elementwise_add_sat(bh, bO);
            }
            ncol += (uint32_t)col;
          }
        }
        nchu[u] = liveu[u] ? ncol * ((uint32_t)hasT + (uint32_t)hasO) : 0u;
      }
      uint32_t wu[U][2 * NV];
#pragma unroll
      for (int u = 0; u < U; u++)
#pragma unroll
        for (int k = 0; k < 2 * NV; k++)
          wu[u][k] = DBG == 1 ? (offu[u][k] & 0x7Du)  // (A/B only: no gathers, a word from the offset)
                              : __builtin_amdgcn_raw_buffer_load_b8(rw, offu[u][k], 0, 0);
#pragma unroll
      for (int u = 0; u < U; u++) {
        // reference-canonical _res_red / _remote_red over the children (an
        // absent child reads 0: WIN in 0, changes none of the four;
        // SURVEY §8a A8/A9), a column's T and O children side by side in the
        // 16-bit halves of one register (v_pk_min_u16 / v_pk_max_u16):
        //   t = (v ^ 1) & 3 -- LOSS 0, WIN 1, DRAW 2, TIE 3: its maximum is
        //       the best non-losing value (TIE over DRAW over WIN);
        //   min of w + (t << 8): below 256 iff a child is a LOSS, then the
        //       smallest LOSS child's word;  max of w: the largest remoteness
        rk_u16x2 mn = {0xFFFFu, 0xFFFFu}, mx = {0, 0}, pr = {0, 0};
#pragma unroll
        for (int x = 0; x < NV; x++) {
          const uint32_t p = wu[u][2 * x] | (wu[u][2 * x + 1] << 16);
          const uint32_t t = (p ^ 0x00010001u) & 0x00030003u;
          mn = __builtin_elementwise_min(mn, __builtin_bit_cast(rk_u16x2, p + (t << 8)));
          mx = __builtin_elementwise_max(mx, __builtin_bit_cast(rk_u16x2, p));
          pr = __builtin_elementwise_max(pr, __builtin_bit_cast(rk_u16x2, t));
        }
        const uint32_t mn1 = min((uint32_t)mn.x, (uint32_t)mn.y), mx1 = max((uint32_t)mx.x, (uint32_t)mx.y);
        const uint32_t pr1 = max((uint32_t)pr.x, (uint32_t)pr.y);
        if (!liveu[u]) continue;
        if (nchu[u] == 0) err |= ERR_NO_MOVES;
        edges += nchu[u];
        const uint32_t word = mn1 < 256u ? make_word(WIN, (mn1 >> 2) + 1)
                                         : make_word(pr1 == 3u ? TIE : pr1 == 2u ? DRAW : LOSS, (mx1 >> 2) + 1);
        if (rows) reinterpret_cast<uint8_t*>(tw)[slotu[u] - lvstart - (t0 << 5)] = (uint8_t)word;
        else g.words[slotu[u]] = (uint8_t)word;
      }
    };
    const uint32_t nvu = __builtin_amdgcn_readfirstlane(nv);
    for (uint32_t e0 = threadIdx.x; e0 < (DBG == 2 ? 0u : total); e0 += 256u * U) {
      if (!oneblk || nvu == 0) {
        pass(std::integral_constant<int, NC>(), e0, false);
      } else if constexpr (CC > 0 && DBG == 0) {
        // (the compiled-in boards: one copy per count of columns with room)
        if (nvu >= (uint32_t)NC) pass(std::integral_constant<int, NC>(), e0, true);
        else if (nvu == 1) pass(std::integral_constant<int, 1>(), e0, true);
        else if (nvu == 2) pass(std::integral_constant<int, NC >= 2 ? 2 : 1>(), e0, true);
        else if (nvu == 3) pass(std::integral_constant<int, NC >= 3 ? 3 : 1>(), e0, true);
        else if (nvu == 4) pass(std::integral_constant<int, NC >= 4 ? 4 : 1>(), e0, true);
        else if (nvu == 5) pass(std::integral_constant<int, NC >= 5 ? 5 : 1>(), e0, true);
        else pass(std::integral_constant<int, NC>(), e0, true);
      } else {
        pass(std::integral_constant<int, NC>(), e0, true);
      }
    }
    if (rows) {  // the tile's rows with a reached slot, whole
      __syncthreads();
      if ((m | mp) && wi < nwords) {
        uint4* dst = reinterpret_cast<uint4*>(g.words + lvstart + (wi << 5));
        uint4 v0 = tw[2 * threadIdx.x], v1 = tw[2 * threadIdx.x + 1];
        if constexpr (OWN) {
          // md5 shards: only this shard's reached slots (m | mp, both
          // already masked to the owned ones) are written; every other byte
          // of the row keeps what the table holds (other owners' words come
          // in through the level exchange, k_rko_unpack), so the backward
          // never depends on running before the unpack
          const uint4 o0 = dst[0], o1 = dst[1];
          uint32_t nv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
          const uint32_t ov[8] = {o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w};
          const uint32_t mine = m | mp;
#pragma unroll
          for (int d = 0; d < 8; d++) {
            const uint32_t nib = (mine >> (4 * d)) & 15u;
            const uint32_t bm = ((nib & 1u) ? 0xFFu : 0u) | ((nib & 2u) ? 0xFF00u : 0u) |
                                ((nib & 4u) ? 0xFF0000u : 0u) | ((nib & 8u) ? 0xFF000000u : 0u);
            nv[d] = (nv[d] & bm) | (ov[d] & ~bm);
          }
          v0 = make_uint4(nv[0], nv[1], nv[2], nv[3]);
          v1 = make_uint4(nv[4], nv[5], nv[6], nv[7]);
        }
        dst[0] = v0;
        dst[1] = v1;
      }
    }
    __syncthreads();  // the list and the rows are rewritten by the next tile
  }
  if (err) atomicOr(&st->err, err);
  block_count(bc, 0, edges);
  if constexpr (OWN) {  // slots this shard resolved (gm_rk_shard_stats)
    for (int o = 32; o > 0; o >>= 1) resolved += __shfl_xor(resolved, o);
    if ((threadIdx.x & 63) == 0 && resolved) atomicAdd((unsigned long long*)&st->ks_cursor, (unsigned long long)resolved);
  }
}

// the end of a solve: the root's word, then the counts (fill_red_body)
__global__ __launch_bounds__(1024) void k_rk_finish(RankGeom g, u64 root_slot, DevState* st, const BlockCount* bc) {
  if (threadIdx.x == 0)
    st->root_word = ((g.reach[root_slot >> 5] >> (root_slot & 31)) & 1u) ? (uint32_t)g.words[root_slot] : NO_WORD;
  __syncthreads();
  fill_red_body(st, bc);
}

__global__ void k_rk_query(Desc d, RankGeom g, const u64* keys, u64 n, uint32_t* out) {
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
    u64 s;
    uint32_t L, w = NO_WORD;
    if (rk_slot_of(g, keys[i], &s, &L) && ((g.reach[s >> 5] >> (s & 31)) & 1u)) w = g.words[s];
    out[i] = w;
  }
}

// every reached slot of every level: its key (positions) or its fingerprint
// term (checksum); one thread per 64-slot word of the reach bitmap
// (lvt: the levels' first slots [0, T], then their first block entries [T + 1, 2T + 1])
template <bool CK>
__global__ __launch_bounds__(256) void k_rk_scan(Desc d, RankGeom g, const u64* lvt, uint32_t T, u64 nwords, u64* keys,
                                                 u64 cap, u64* count, u64* acc) {
  const u64* lvstart = lvt;
  const u64* lvoff = lvt + T + 1;
  u64 v[6] = {0, 0, 0, 0, 0, 0};
  for (u64 wi = (u64)blockIdx.x * blockDim.x + threadIdx.x; wi < nwords; wi += (u64)gridDim.x * blockDim.x) {
    u64 m = reinterpret_cast<const u64*>(g.reach)[wi];
    if (!m) continue;
    const u64 s0 = wi << 6;
    uint32_t L = 0;
    while (L + 1 < T && lvstart[L + 1] <= s0) L++;
    u64 k = 0;
    if (!CK) k = atomicAdd(count, (u64)__builtin_popcountll(m));
    for (; m; m &= m - 1, k++) {
      const u64 i = s0 + (u64)__builtin_ctzll(m) - lvstart[L];
      const u64 blk = i >> (L + 3);
      const uint32_t a = (uint32_t)((i >> L) & 7u), pat = (uint32_t)(i & ((1ull << L) - 1));
      RankPos p;
      rk_unpack(g, g.lvph[lvoff[L] + blk], p);
      const u64 key = rk_key(g, p, pat, L, rk_hands(L, (uint32_t)__builtin_popcount(pat), a));
      if (CK) ck_add(d, key, g.words[lvstart[L] + i], v);
      else if (k < cap) keys[k] = key;
    }
  }
  if (CK) ck_block_add(acc, v);
}

// ---------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------

struct RankShape {
  RankGeom g;
  std::vector<u64> base;                // per hvcode
  std::vector<uint32_t> lvhv, lvph;     // hvcodes level by level, packed heights
  std::vector<uint32_t> lvch;           // per entry: child block offsets in the next level (RankGeom::lvch)
  std::vector<uint32_t> lvpa;           // per entry: parent block offsets in the level below (RankGeom::lvpa)
  std::vector<uint32_t> lvoff;          // per level: first entry in lvhv (T + 1)
  std::vector<u64> lvstart, lvitems;    // per level: first slot, slots
  u64 words_off, reach_off, expd_off, bstat_off, pbits_off, base_off, lvhv_off, lvph_off, lvch_off, lvpa_off, table_bytes;
};

static int rank_shape(const Desc* d, RankShape* rs) {
  RankGeom& g = rs->g;
  memset(&g, 0, sizeof g);
  g.C = (uint32_t)d->L;
  g.H = (uint32_t)d->H;
  g.R = g.H + 1;
  g.A = g.C * g.H;
  g.T = g.A + 1;
  uint32_t nhv = 1;
  for (uint32_t x = 0; x < g.C; x++) {
    g.stride[x] = nhv;
    nhv *= g.R;
  }
  std::vector<std::vector<uint32_t>> byl(g.T);
  for (uint32_t c = 0; c < nhv; c++) {
    uint32_t s = 0, v = c;
    for (uint32_t x = 0; x < g.C; x++) {
      s += v % g.R;
      v /= g.R;
    }
    byl[s].push_back(c);
  }
  // Block order inside a level.  A child block (hv + e_x) is read by up to C
  // parent blocks, one per column; in ascending code order those are up to
  // (H+1)^(C-1) codes apart, so a child block's lines are fetched again by
  // parents far away in time.  GM_RK_ORDER=morton orders a level's blocks by
  // the bit-interleaved height digits instead (neighbours along any column
  // mostly close together) -- A/B
  if (const char* e = lab_env("GM_RK_ORDER")) {
    if (!strcmp(e, "morton")) {
      auto key = [&](uint32_t c) {
        uint32_t dig[kRankMaxCols] = {}, v = c;
        for (uint32_t x = 0; x < g.C; x++) {
          dig[x] = v % g.R;
          v /= g.R;
        }
        u64 k = 0;
        for (int b = 3; b >= 0; b--)
          for (int x = (int)g.C - 1; x >= 0; x--) k = k * 2 + ((dig[x] >> b) & 1u);
        return k;
      };
      for (auto& v : byl) std::sort(v.begin(), v.end(), [&](uint32_t a, uint32_t b) { return key(a) < key(b); });
    }
  }
  rs->base.assign(nhv, 0);
  rs->lvhv.clear();
  rs->lvph.clear();
  rs->lvoff.assign(g.T + 1, 0);
  rs->lvstart.assign(g.T + 1, 0);
  rs->lvitems.assign(g.T, 0);
  u64 at = 0;
  for (uint32_t L = 0; L < g.T; L++) {
    rs->lvoff[L] = (uint32_t)rs->lvhv.size();
    rs->lvstart[L] = at;
    const u64 nb = 8ull << L;
    for (size_t j = 0; j < byl[L].size(); j++) {
      const uint32_t c = byl[L][j];
      rs->base[c] = at + j * nb;
      uint32_t ph = 0, v = c;
      for (uint32_t x = 0; x < g.C; x++) {
        ph |= (v % g.R) << (4 * x);
        v /= g.R;
      }
      rs->lvhv.push_back(c);
      rs->lvph.push_back(ph);
    }
    rs->lvitems[L] = (u64)byl[L].size() * nb;
    at += (rs->lvitems[L] + 511) & ~511ull;  // boards (slots / 8) 64-aligned
  }
  rs->lvoff[g.T] = (uint32_t)rs->lvhv.size();
  rs->lvstart[g.T] = at;
  rs->lvch.assign(rs->lvhv.size() * kRankMaxCols, 0xFFFFFFFFu);
  for (uint32_t L = 0; L < g.T; L++)
    for (uint32_t j = rs->lvoff[L]; j < rs->lvoff[L + 1]; j++)
      for (uint32_t x = 0; x < g.C; x++)
        if (((rs->lvph[j] >> (4 * x)) & 15u) < g.H)
          rs->lvch[(size_t)j * kRankMaxCols + x] = (uint32_t)(rs->base[rs->lvhv[j] + g.stride[x]] - rs->lvstart[L + 1]);
  rs->lvpa.assign(rs->lvhv.size() * kRankMaxCols, 0xFFFFFFFFu);
  for (uint32_t L = 1; L < g.T; L++)
    for (uint32_t j = rs->lvoff[L]; j < rs->lvoff[L + 1]; j++)
      for (uint32_t x = 0; x < g.C; x++)
        if (((rs->lvph[j] >> (4 * x)) & 15u) > 0)
          rs->lvpa[(size_t)j * kRankMaxCols + x] = (uint32_t)(rs->base[rs->lvhv[j] - g.stride[x]] - rs->lvstart[L - 1]);
  g.nslots = at;
  rs->words_off = 0;
  rs->reach_off = rup256(at);
  rs->expd_off = rs->reach_off + rup256(at / 8);
  rs->bstat_off = rs->expd_off + rup256(at / 8);
  rs->pbits_off = rs->bstat_off + rup256(at / 8);
  rs->base_off = rs->pbits_off + rup256(at / 64);
  rs->lvhv_off = rs->base_off + rup256((u64)nhv * 8);
  rs->lvph_off = rs->lvhv_off + rup256((u64)nhv * 4);
  rs->lvch_off = rs->lvph_off + rup256((u64)nhv * 4);
  rs->lvpa_off = rs->lvch_off + rup256((u64)nhv * 4 * kRankMaxCols);
  rs->table_bytes = rs->lvpa_off + rup256((u64)nhv * 4 * kRankMaxCols);
  return 0;
}

static bool rank_ok(const Desc* d) {
  if (d->kind != K_TOOT || d->L < 1 || d->L > kRankMaxCols || d->H < 1 || d->H > 7) return false;
  if (d->max_levels > 64 || (int)d->max_levels != d->L * d->H + 1) return false;  // remoteness in 6 bits
  double n = 8;
  for (int x = 0; x < d->L; x++) n *= (double)((2u << d->H) - 1);
  if (n > (double)(1ull << 36)) return false;
  // every level's slots addressable by one 32-bit buffer offset (k_rk_backward)
  RankShape rs;
  if (rank_shape(d, &rs)) return false;
  for (uint32_t L = 0; L < rs.g.T; L++)
    if (rs.lvstart[L + 1] - rs.lvstart[L] >= 0xFFFFFFFFull) return false;
  return true;
}
static bool rank_wanted(const Desc* d, uint32_t flags) {
  return rank_ok(d) && !(flags & (GM_F_FORCE_HASHED | GM_F_HASH_TABLE));
}

static int plan_ranked(const Desc* d, uint64_t max_table_bytes, gm_plan_t* out, bool* fits) {
  RankShape rs;
  int rc = rank_shape(d, &rs);
  if (rc) return rc;
  *fits = max_table_bytes == 0 || rs.table_bytes <= max_table_bytes;
  out->mode = GM_MODE_RANKED;
  out->table_slots = rs.g.nslots;
  out->table_bytes = rs.table_bytes;
  out->level_capacity = 1;
  out->scratch_bytes = scratch_bytes_for(d->max_levels);
  out->max_levels = (uint32_t)d->max_levels;
  return 0;
}

static int rko_setup(gm_solver* s, const gm_buffers* buf, const RankShape& rs);  // gm_ranked_shard.h
static int rank_setup(gm_solver* s, const gm_buffers* buf) {
  RankShape rs;
  int rc = rank_shape(&s->d, &rs);
  if (rc) return rc;
  if (buf->table_bytes < rs.table_bytes)
    return fail(GM_EINVAL, "ranked table of %llu bytes, the plan needs %llu", (unsigned long long)buf->table_bytes,
                (unsigned long long)rs.table_bytes);
  char* t = (char*)buf->table;
  rs.g.words = (uint8_t*)(t + rs.words_off);
  rs.g.reach = (uint32_t*)(t + rs.reach_off);
  rs.g.expd = (uint32_t*)(t + rs.expd_off);
  rs.g.base = (const u64*)(t + rs.base_off);
  rs.g.lvhv = (const uint32_t*)(t + rs.lvhv_off);
  rs.g.lvph = (const uint32_t*)(t + rs.lvph_off);
  rs.g.lvch = (const uint32_t*)(t + rs.lvch_off);
  rs.g.lvpa = (const uint32_t*)(t + rs.lvpa_off);
  rs.g.bstat = (uint8_t*)(t + rs.bstat_off);
  rs.g.pbits = (u64*)(t + rs.pbits_off);
  for (int c = 0; c < 7; c++) {
    u64 m = 0;
    for (int j = 0; j < 64; j++)
      if (__builtin_popcount((unsigned)j) <= c) m |= 1ull << j;
    rs.g.le[c] = m;
  }
  HIPCHK(hipMemcpy((void*)rs.g.base, rs.base.data(), rs.base.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy((void*)rs.g.lvhv, rs.lvhv.data(), rs.lvhv.size() * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy((void*)rs.g.lvph, rs.lvph.data(), rs.lvph.size() * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy((void*)rs.g.lvch, rs.lvch.data(), rs.lvch.size() * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy((void*)rs.g.lvpa, rs.lvpa.data(), rs.lvpa.size() * 4, hipMemcpyHostToDevice));
  s->rg = rs.g;
  s->rlvoff = rs.lvoff;
  s->rlvstart = rs.lvstart;
  s->rlvitems = rs.lvitems;
  // the per-level tables the scans read on the device (k_rk_scan's lvt)
  if (!s->rlv_dev) HIPCHK(hipMalloc((void**)&s->rlv_dev, (size_t)(2 * (rs.g.T + 1)) * 8));
  std::vector<u64> tabs(2 * (rs.g.T + 1), 0);
  for (uint32_t L = 0; L <= rs.g.T; L++) {
    tabs[L] = rs.lvstart[L];
    tabs[rs.g.T + 1 + L] = rs.lvoff[L];
  }
  HIPCHK(hipMemcpy(s->rlv_dev, tabs.data(), tabs.size() * 8, hipMemcpyHostToDevice));
  if (s->world > 1) return rko_setup(s, buf, rs);  // md5 shards: owners, exchange buffers
  return 0;
}

template <class F>
static void rank_kind_dispatch(const Desc& d, F&& f) {
  switch (fixed_kind(d)) {
    case K_TOOT_6x4: f(std::integral_constant<int, K_TOOT_6x4>()); break;
    case K_TOOT_5x4: f(std::integral_constant<int, K_TOOT_5x4>()); break;
    case K_TOOT_4x4: f(std::integral_constant<int, K_TOOT_4x4>()); break;
    default: f(std::integral_constant<int, K_TOOT>()); break;
  }
}

// GM_RK_DBG=1 / 2: the backward without its gathers / without its entries
// (timing A/B only: the words are wrong)
static int rk_dbg() {
  static const int v = [] {
    const char* e = lab_env("GM_RK_DBG");
    return e ? atoi(e) : 0;
  }();
  return v;
}
// the bit-sliced board kernel (k_rk_boards_sl) where it applies; GM_RK_SLICED=0
// keeps the per-board one (A/B runs)
static bool rk_sliced() {
  static const bool on = [] {
    const char* e = lab_env("GM_RK_SLICED");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

static int rank_grid(const gm_solver* s, u64 nitems) {
  return (int)std::max<u64>(1, std::min<u64>((nitems + 255) / 256, (u64)std::min(s->grid * 2, kCountSlots)));
}

// one forward level of the RANKED solve: the board pass, then reach / counts
static void rank_forward_level(gm_solver* s, hipStream_t st, uint32_t L) {
  const Desc& d = s->d;
  const RankGeom& g = s->rg;
  rank_kind_dispatch(d, [&](auto KC) {
    constexpr int KIND = decltype(KC)::value;
    const u64 nreal = s->rlvitems[L] >> 3, nb = (s->rlvstart[L + 1] - s->rlvstart[L]) >> 3;  // boards
    auto boards = [&](auto CH) {
      constexpr int CC = decltype(CH)::value / 16, HH = decltype(CH)::value % 16;
      hipLaunchKernelGGL((k_rk_boards<KIND, CC, HH>), dim3(rank_grid(s, nb)), dim3(256), 0, st, d, g, L,
                         s->rlvstart[L] >> 3, s->rlvoff[L], nb, nreal);
    };
    auto boards_sl = [&](auto CH) {
      constexpr int CC = decltype(CH)::value / 16, HH = decltype(CH)::value % 16;
      hipLaunchKernelGGL((k_rk_boards_sl<CC, HH>), dim3(rank_grid(s, nb / 32)), dim3(256), 0, st, g, L,
                         s->rlvstart[L] >> 3, s->rlvoff[L], nb / 32, nreal);
    };
    const bool sliced = L >= 5 && rk_sliced();
    if (g.C == 6 && g.H == 4) {
      if (sliced) boards_sl(std::integral_constant<int, 6 * 16 + 4>());
      else boards(std::integral_constant<int, 6 * 16 + 4>());
    } else if (g.C == 5 && g.H == 4) {
      if (sliced) boards_sl(std::integral_constant<int, 5 * 16 + 4>());
      else boards(std::integral_constant<int, 5 * 16 + 4>());
    } else if (g.C == 4 && g.H == 4 && sliced) {
      boards_sl(std::integral_constant<int, 4 * 16 + 4>());
    } else {
      boards(std::integral_constant<int, 0>());
    }
    const u64 n = s->rlvstart[L + 1] - s->rlvstart[L];  // 512-padded: every bitmap word written
    if (L >= 6)
      hipLaunchKernelGGL(k_rk_reach4, dim3(rank_grid(s, n / 256)), dim3(256), 0, st, g, L, s->rlvstart[L],
                         s->rlvoff[L], n / 64, s->rlvitems[L], s->bcount, s->st, s->rlvstart[L - 1]);
    else
      hipLaunchKernelGGL(k_rk_forward, dim3(rank_grid(s, n)), dim3(256), 0, st, g, L, s->rlvstart[L], s->rlvoff[L],
                         n, s->rlvitems[L], s->bcount, s->st);
  });
}

// one backward level (ownb: md5 shards -- only the slots `orank` owns, in
// 32-slot tile words)
static void rank_backward_level(gm_solver* s, hipStream_t st, uint32_t L, const uint4* ownb = nullptr,
                                uint32_t orank = 0) {
  const RankGeom& g = s->rg;
  const uint32_t T = g.T;
  const u64 nw = (s->rlvitems[L] + 31) / 32;  // 32-slot tile words
  // level L + 1's slots (the last level has no children: an empty range)
  const u64 cs = s->rlvstart[std::min<uint32_t>(L + 1, T)];
  const u64 cn = L + 1 < T ? s->rlvstart[L + 2] - cs : 0;
  const dim3 grid(rank_grid(s, nw)), blk(256);
  auto go = [&](auto CH) {
    constexpr int CC = decltype(CH)::value / 16, HH = decltype(CH)::value % 16;
    if (ownb)
      hipLaunchKernelGGL((k_rk_backward<CC, HH, true>), grid, blk, 0, st, g, L, s->rlvstart[L], s->rlvoff[L], nw, cs,
                         cn, s->bcount, s->st, ownb, orank);
    else if (rk_dbg() == 1)
      hipLaunchKernelGGL((k_rk_backward<CC, HH, false, 1>), grid, blk, 0, st, g, L, s->rlvstart[L], s->rlvoff[L], nw,
                         cs, cn, s->bcount, s->st, nullptr, 0u);
    else if (rk_dbg() == 2)
      hipLaunchKernelGGL((k_rk_backward<CC, HH, false, 2>), grid, blk, 0, st, g, L, s->rlvstart[L], s->rlvoff[L], nw,
                         cs, cn, s->bcount, s->st, nullptr, 0u);
    else
      hipLaunchKernelGGL((k_rk_backward<CC, HH>), grid, blk, 0, st, g, L, s->rlvstart[L], s->rlvoff[L], nw, cs, cn,
                         s->bcount, s->st, nullptr, 0u);
  };
  // the compiled-in boards' marks need the child level <= 1 GiB (kRkColMark)
  const bool narrow = cn <= kRkColMark;
  if (narrow && g.C == 6 && g.H == 4) go(std::integral_constant<int, 6 * 16 + 4>());
  else if (narrow && g.C == 5 && g.H == 4) go(std::integral_constant<int, 5 * 16 + 4>());
  else if (narrow && g.C == 4 && g.H == 4) go(std::integral_constant<int, 4 * 16 + 4>());
  else go(std::integral_constant<int, 0>());
}

// Steps (gm_solver_set_steps): forward level L is step L, backward level L
// step 2T - 1 - L, as for the other layouts.
static int run_ranked(gm_solver* s, gm_result* out) {
  const RankGeom& g = s->rg;
  const int T = (int)g.T;
  const int first = (int)s->step_first, stop = s->step_stop ? (int)s->step_stop : 2 * T;
  s->step_first = s->step_stop = 0;
  const bool timing = (s->flags & GM_F_KERNEL_TIMING) && first == 0 && stop == 2 * T;
  hipStream_t st = s->stream;
  if (first > 0) {
    uint32_t wb = 0;
    HIPCHK(hipMemcpy(&wb, &s->st->word_bits, sizeof wb, hipMemcpyDeviceToHost));
    if (wb != 0x208u) return fail(GM_EINVAL, "resume: the scratch holds no ranked solve");
  }
  hipEvent_t ev[4];
  for (auto& e : ev) HIPCHK(hipEventCreate(&e));
  auto t0 = std::chrono::steady_clock::now();
  HIPCHK(hipEventRecord(ev[0], st));
  if (first == 0) {
    HIPCHK(hipMemsetAsync(s->st, 0, devstate_bytes(T), st));
    HIPCHK(hipMemsetAsync(s->bcount, 0, kCountSlots * sizeof(BlockCount), st));
    HIPCHK(hipMemsetD32Async((hipDeviceptr_t)&s->st->word_bits, 0x208, 1, st));  // the solve in progress: ranked
  }
  u64 nl_f = 0, nl_b = 0;
  for (int k = std::max(first, 0); k < std::min(stop, T); k++) {
    rank_forward_level(s, st, (uint32_t)k);
    nl_f += 2;
  }
  HIPCHK(hipEventRecord(ev[1], st));
  for (int k = std::max(first, T); k < stop; k++) {
    rank_backward_level(s, st, (uint32_t)(2 * T - 1 - k));
    nl_b++;
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ev[2], st));
  if (stop < 2 * T) {
    HIPCHK(hipStreamSynchronize(st));
    for (auto& e : ev) (void)hipEventDestroy(e);
    out->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    out->word_bits = 8;
    return GM_PARTIAL;
  }
  hipLaunchKernelGGL(k_rk_finish, dim3(1), dim3(1024), 0, st, g, s->rlvstart[0], s->st, (const BlockCount*)s->bcount);
  HIPCHK(hipGetLastError());
  u64 red[5];
  HIPCHK(hipMemcpyAsync(red, s->st->red, sizeof red, hipMemcpyDeviceToHost, st));
  HIPCHK(hipEventRecord(ev[3], st));
  HIPCHK(hipStreamSynchronize(st));
  float f = 0, b = 0;
  HIPCHK(hipEventElapsedTime(&f, ev[0], ev[1]));
  HIPCHK(hipEventElapsedTime(&b, ev[1], ev[2]));
  for (auto& e : ev) (void)hipEventDestroy(e);
  out->ms_forward = f;
  out->ms_backward = b;
  out->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (timing) {
    out->ms_expand_kernels = f;
    out->ms_resolve_kernels = b;
    out->n_expand_launches = nl_f;
    out->n_resolve_launches = nl_b;
  }
  out->positions = red[0];
  out->edges = red[1];
  out->primitives = red[2];
  out->levels = (uint32_t)T;
  out->max_level_width = 0;
  out->word_bits = 8;
  out->kernels = RK_RANKED;
  const uint32_t word = red[3] ? (uint32_t)(red[3] - 1) : NO_WORD;
  out->root_word = word;
  if (red[4]) return fail(GM_ECORRUPT, "solve failed:%s", err_text((uint32_t)red[4]).c_str());
  if (word == NO_WORD) return fail(GM_ECORRUPT, "root unresolved");
  out->root_value = (int32_t)(word & 3u);
  out->root_remoteness = word >> 2;
  return 0;
}

static int rank_query(gm_solver* s, const uint64_t* keys_dev, uint64_t n, uint32_t* words_dev) {
  const int grid = (int)std::min<u64>((n + kBlock - 1) / kBlock, (u64)s->grid);
  hipLaunchKernelGGL(k_rk_query, dim3(grid), dim3(kBlock), 0, s->stream, s->d, s->rg, (const u64*)keys_dev, n,
                     words_dev);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s->stream));
  return 0;
}

static int rank_scan(gm_solver* s, bool ck, u64* keys_dev, u64 cap, u64* acc) {
  const RankGeom& g = s->rg;
  const u64 nwords = g.nslots / 64;
  if (ck)
    hipLaunchKernelGGL((k_rk_scan<true>), dim3(s->grid), dim3(256), 0, s->stream, s->d, g, (const u64*)s->rlv_dev, g.T,
                       nwords, (u64*)nullptr, (u64)0, (u64*)nullptr, acc);
  else
    hipLaunchKernelGGL((k_rk_scan<false>), dim3(s->grid), dim3(256), 0, s->stream, s->d, g, (const u64*)s->rlv_dev, g.T,
                       nwords, keys_dev, cap, &s->st->cursor_back, (u64*)nullptr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s->stream));
  return 0;
}

static int rank_positions(gm_solver* s, uint64_t* keys_dev, uint64_t cap, uint64_t* n) {
  u64 cnt = 0;
  HIPCHK(hipStreamSynchronize(s->stream));
  HIPCHK(hipMemcpy(&cnt, &s->st->cursor_front, sizeof cnt, hipMemcpyDeviceToHost));
  *n = cnt;
  if (cnt > cap || !keys_dev) return cap < cnt ? fail(GM_EFULL, "need %llu slots", (unsigned long long)cnt) : 0;
  HIPCHK(hipMemsetAsync(&s->st->cursor_back, 0, sizeof(u64), s->stream));
  return rank_scan(s, false, (u64*)keys_dev, cap, nullptr);
}

}  // extern "C++"
