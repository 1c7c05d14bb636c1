// gm_games.h -- device-side game descriptors for the MI355X solver.
//
// Each reference game module (test_games/*.py) is paired with a descriptor
// over a packed 64-bit state ("key").  A descriptor provides, for one key:
//   prim(key)                      -> WIN/LOSS/TIE/DRAW or UNDECIDED
//                                     (the module's primitive())
//   children(key, emit)            -> calls emit(child, step) for each child
//                                     in gen_moves() order, each do_move()'d,
//                                     with the child's level step (1 or 2)
//                                     for the tier pipeline
// These are __host__ __device__ so the same code serves the GPU kernels and
// gm_host_expand (the C-ABI's host-side parity probe).  Canonical-bytes
// <-> key conversion lives in gm_codec.cpp.
//
// Value codes follow src/utils.py:3 (WIN=0, LOSS=1, TIE=2, DRAW=3,
// UNDECIDED=4).  A resolved position is stored as one 32-bit word:
//   bits [0,2) value, bits [2,32) remoteness  (remoteness needs >= 30 bits:
//   the Four-To-One 2^30 chain reaches 715,827,883; SURVEY.md §7 "Hard
//   parts").
#pragma once
#include <stdint.h>

#ifndef __HIP_DEVICE_COMPILE__
#include <string.h>
#endif

#if defined(__HIPCC__)
#define GM_HD __host__ __device__ __forceinline__
#else
#define GM_HD inline
#endif

namespace gm {

enum : int { WIN = 0, LOSS = 1, TIE = 2, DRAW = 3, UNDECIDED = 4 };

enum GameKind : int {
  K_SUM = 1,     // four_to_one.py (1 heap) and sum_four_to_one.py (K heaps)
  K_TTT = 2,     // tic_tac_toe_np.py and mttt.py (same graph)
  K_TOOT = 3,    // toot_and_otto_bitstring.py
  K_OTHELLO = 4  // othello_bit_new.py (square boards)
};

constexpr int MAXCHILD = 32;
constexpr uint64_t EMPTY_KEY = ~0ull;
constexpr uint32_t NO_WORD = 0xFFFFFFFFu;

GM_HD uint32_t make_word(int value, uint32_t rem) { return (uint32_t)value | (rem << 2); }

// ---------------------------------------------------------------------------
// Descriptor parameter block (passed to kernels by value).
// ---------------------------------------------------------------------------
struct Desc {
  int kind;
  int variant;     // K_TTT: 0 = tic_tac_toe_np, 1 = mttt; K_SUM: 0 = sum, 1 = four_to_one
  int L, H, A;     // board games
  int nbits;       // bitstring length (toot/othello canonical form)
  // K_SUM
  int nheaps;
  int pow2;        // every base is a power of two -> shift/mask digits
  uint32_t heap[16];
  uint32_t base[16];
  uint32_t shift[16];
  uint64_t stride[16];
  uint32_t root_sum;
  // K_TOOT word-start masks (directions (1,0),(0,1),(1,1),(1,-1))
  uint64_t tmask[4];
  int tstep[4];
  uint64_t full;   // all-cells mask
  uint64_t col0;   // K_TOOT: the cells of column 0 (bit L*y for every y)
  uint64_t root;   // root key
  int max_levels;  // levels the pipeline must provision (root level = 0)
  // K_SUM dense (perfect-hash) layout: slot = level * W + prefix, where
  // prefix = rank / base[0] (heap digits 1..K-1) and heap 0 is recovered
  // from the level: h0 = (root_sum - level) - digitsum(prefix).
  int dense_ok;
  int wshift;      // log2(W) when W is a power of two, else -1
  uint64_t W;      // prefixes per level = prod_{i>=1} base[i]
  uint64_t pstride[16];  // stride of heap digit i inside the prefix (i >= 1)
  uint32_t pshift[16];   // log2(pstride[i]) when pow2
  // symmetry hooks (params "symmetry=1"): keys are
  // canonical representatives of their orbit under the game module's
  // symmetry_functions() (othello_bit_new.py:224-226: player_flip, order 2)
  int sym;
};

// Which part of a DENSE table's global prefix space one table holds, and
// which part a launch sweeps.  A single-GPU table holds everything (local
// prefix = global prefix).  A shard (blk = 1) owns
// BLOCKS of B consecutive values of the TOP prefix digit, block k owned by
// rank k mod world, and lays them out one after another, each as
// [2 halo slices | B own slices | 2 halo slices] of Z prefixes (Z = the top
// digit's stride): local slice u is slice o = u mod (B + 4) of its rank's
// block j = u / (B + 4), i.e. top value t = (rank + j world) B + o - 2.
// p_lo/p_hi bound the local prefixes a launch sweeps; a launch processes
// only slices with olo <= o < ohi (own slices: [2, B + 2)).  Wl = local
// words per level, Wbl = local reach bits per level (Wl rounded up to 64).
constexpr int kMaxSweepSlices = 192;
struct DenseView {
  uint64_t p_lo, p_hi;
  uint64_t base_off;  // always 0 (local addressing starts at 0)
  uint64_t Wl, Wbl;
  uint32_t blk, B, world, rank;
  uint64_t Z, E;
  int32_t zshift;     // log2(Z) when Z is a power of two, else -1
  uint32_t olo, ohi;
  // compact sweep (blk, nsl > 0): a launch sweeps only the nsl local slices
  // listed in sl[] -- sweep index i is slice sl[i / Z], prefix i % Z
  uint32_t nsl;
  uint16_t sl[kMaxSweepSlices];  // local slice
  uint16_t st[kMaxSweepSlices];  // its global top value
};

// local prefix of sweep index i (identity unless the view lists slices)
GM_HD uint64_t dense_sweep_q(const DenseView& v, uint64_t i) {
  if (!v.nsl) return i;
  const uint64_t si = v.zshift >= 0 ? (i >> v.zshift) : i / v.Z;
  return (uint64_t)v.sl[si] * v.Z + (i - si * v.Z);
}

// sweep index qi -> local prefix *q and global prefix (returned); *run =
// this launch processes the slice.  Listed slices carry their global top
// value, so the common case is two table reads and shifts.
GM_HD uint64_t dense_global(const DenseView& v, uint64_t q, bool* run);
GM_HD uint64_t dense_sweep(const DenseView& v, uint64_t qi, uint64_t* q, bool* run) {
  if (v.nsl) {
    const uint64_t si = v.zshift >= 0 ? (qi >> v.zshift) : qi / v.Z;
    const uint64_t base = v.zshift >= 0 ? (si << v.zshift) : si * v.Z;
    const uint64_t r = qi - base;
    *run = true;
    if (v.zshift >= 0) {
      *q = ((uint64_t)v.sl[si] << v.zshift) + r;
      return ((uint64_t)v.st[si] << v.zshift) + r;
    }
    *q = (uint64_t)v.sl[si] * v.Z + r;
    return (uint64_t)v.st[si] * v.Z + r;
  }
  *q = qi;
  return dense_global(v, qi, run);
}

// global prefix of local prefix q; *run = this launch processes its slice
// (q's slice must be the same for every lane of a wave: Z % 64 == 0)
GM_HD uint64_t dense_global(const DenseView& v, uint64_t q, bool* run) {
  if (!v.blk) {
    *run = true;
    return q;
  }
  const uint64_t u = v.zshift >= 0 ? (q >> v.zshift) : q / v.Z;
  const uint32_t j = (uint32_t)u / (v.B + 4), o = (uint32_t)u - j * (v.B + 4);
  const int64_t t = (int64_t)(((uint64_t)v.rank + (uint64_t)j * v.world) * v.B + o) - 2;
  *run = o >= v.olo && o < v.ohi && t >= 0 && (uint64_t)t < v.E;
  return (uint64_t)t * v.Z + (q - u * v.Z);
}

// local prefix of global prefix p, if this table owns it
GM_HD bool dense_local(const DenseView& v, uint64_t p, uint64_t* q) {
  if (!v.blk) {
    if (p >= v.Wl) return false;
    *q = p;
    return true;
  }
  const uint64_t t = p / v.Z, k = t / v.B;
  if (t >= v.E || k % v.world != v.rank) return false;
  const uint64_t u = (k / v.world) * (v.B + 4) + 2 + (t - k * v.B);
  *q = u * v.Z + (p - t * v.Z);
  return true;
}

GM_HD int popc64(uint64_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __popcll(v);
#else
  return __builtin_popcountll(v);
#endif
}

// ---------------------------------------------------------------------------
// Sum of Four-To-One heaps (four_to_one.py:7-22 per heap;
// gamesmanmpi_amd/games/sum_four_to_one.py).  key = mixed-radix rank, heap 0
// least significant.  Level = root_sum - digit sum; a -1 move steps one
// level, a -2 move two.
// ---------------------------------------------------------------------------
GM_HD uint32_t sum_digit(const Desc& d, uint64_t r, int i) {
  if (d.pow2) return (uint32_t)((r >> d.shift[i]) & (d.base[i] - 1));
  return (uint32_t)((r / d.stride[i]) % d.base[i]);
}
GM_HD int sum_prim(const Desc&, uint64_t r) { return r == 0 ? LOSS : UNDECIDED; }
template <class F>
GM_HD int sum_children(const Desc& d, uint64_t r, F&& emit) {
  int n = 0;
  if (d.pow2) {
    for (int i = 0; i < d.nheaps; i++) {
      uint32_t h = (uint32_t)((r >> d.shift[i]) & (d.base[i] - 1));
      if (h >= 1) { emit(r - d.stride[i], 1); n++; }
      if (h >= 2) { emit(r - 2 * d.stride[i], 2); n++; }
    }
  } else {
    uint64_t rest = r;
    for (int i = 0; i < d.nheaps; i++) {
      uint64_t q = rest / d.base[i];
      uint32_t h = (uint32_t)(rest - q * d.base[i]);
      rest = q;
      if (h >= 1) { emit(r - d.stride[i], 1); n++; }
      if (h >= 2) { emit(r - 2 * d.stride[i], 2); n++; }
    }
  }
  return n;
}
GM_HD int sum_level(const Desc& d, uint64_t r) {
  uint32_t s = 0;
  for (int i = 0; i < d.nheaps; i++) s += sum_digit(d, r, i);
  return (int)(d.root_sum - s);
}

// ---------------------------------------------------------------------------
// Tic-tac-toe (tic_tac_toe_np.py:7-61 / mttt.py:11-127).  key: 2 bits per
// cell in reading order (np cell [x][y] -> 3x+y; mttt char i -> i);
// 1 = first mover (np 1 / mttt 'X'), 2 = second (np 2 / mttt 'O').
// ---------------------------------------------------------------------------
GM_HD uint32_t ttt_plane(uint64_t k, uint32_t who) {
  uint32_t m = 0;
  for (int c = 0; c < 9; c++) m |= (uint32_t)(((k >> (2 * c)) & 3) == who) << c;
  return m;
}
GM_HD bool ttt_line(uint32_t m) {
  // rows, columns, diagonals of the 3x3 reading-order grid: every line the
  // reference's 4-direction scan can find (tic_tac_toe_np.py:50-56)
  const uint32_t L8[8] = {0007, 0070, 0700, 0111, 0222, 0444, 0421, 0124};
  for (int i = 0; i < 8; i++)
    if ((m & L8[i]) == L8[i]) return true;
  return false;
}
GM_HD int ttt_prim(const Desc&, uint64_t k) {
  uint32_t a = ttt_plane(k, 1), b = ttt_plane(k, 2);
  if (ttt_line(a) || ttt_line(b)) return LOSS;  // checked before fullness
  return ((a | b) == 0777) ? TIE : UNDECIDED;
}
template <class F>
GM_HD int ttt_children(const Desc&, uint64_t k, F&& emit) {
  uint32_t a = ttt_plane(k, 1), b = ttt_plane(k, 2);
  uint64_t who = popc64(a) > popc64(b) ? 2 : 1;  // tic_tac_toe_np.py:13-25
  int n = 0;
  for (int c = 0; c < 9; c++)
    if (!(((a | b) >> c) & 1)) { emit(k | (who << (2 * c)), 1); n++; }
  return n;
}
GM_HD int ttt_level(const Desc&, uint64_t k) {
  return popc64(ttt_plane(k, 1) | ttt_plane(k, 2));
}

// ---------------------------------------------------------------------------
// Toot-and-Otto (toot_and_otto_bitstring.py).  key bits:
//   [0,A) T plane, [A,2A) O plane (cell index L*y+x as in board_get :179-185)
//   [2A, 2A+12) hands, 3 bits each: P1-T, P1-O, P2-T, P2-O (0..6)
//   2A+12: the live turn bit (board[-1], :218-222), 1 = player 1 to move
// Level = pieces on the board.
// ---------------------------------------------------------------------------
GM_HD uint64_t shr_s(uint64_t v, int s) { return s >= 0 ? (v >> s) : (v << (-s)); }
GM_HD int toot_count(const Desc& d, uint64_t first, uint64_t mid) {
  // word = first, mid, mid, first along each direction (TOOT: T,O,O,T)
  int n = 0;
  for (int i = 0; i < 4; i++) {
    int s = d.tstep[i];
    n += popc64(d.tmask[i] & first & shr_s(mid, s) & shr_s(mid, 2 * s) & shr_s(first, 3 * s));
  }
  return n;
}
GM_HD int toot_prim(const Desc& d, uint64_t k) {
  uint64_t t = k & d.full, o = (k >> d.A) & d.full;
  int toot = toot_count(d, t, o), otto = toot_count(d, o, t);
  bool p1 = (k >> (2 * d.A + 12)) & 1;
  if (toot == otto) return ((t | o) == d.full) ? TIE : UNDECIDED;  // :80-81
  return ((toot > otto) != p1) ? LOSS : WIN;                         // :82-85
}
template <class F>
GM_HD int toot_children(const Desc& d, uint64_t k, F&& emit) {
  const int A = d.A, L = d.L, H = d.H;
  uint64_t t = k & d.full, o = (k >> A) & d.full, occ = t | o;
  int p1 = (int)((k >> (2 * A + 12)) & 1);
  int hb = 2 * A + (p1 ? 0 : 6);  // player 1 hands at 2A, player 2 at 2A+6
  uint32_t nT = (uint32_t)((k >> hb) & 7), nO = (uint32_t)((k >> (hb + 3)) & 7);
  uint64_t turn = 1ull << (2 * A + 12);
  int n = 0;
  for (int x = 0; x < L; x++) {
    if ((occ >> (L * (H - 1) + x)) & 1) continue;  // column full (:95)
    // lowest blank cell of column x (:112-115): the lowest clear bit of the
    // column's cells, isolated (no loop; exact for any key)
    const uint64_t blank = ~(occ >> x) & d.col0;
    const uint64_t cell = (blank & (~blank + 1)) << x;
    if (nT > 0) { emit((k - (1ull << hb)) ^ turn ^ cell, 1); n++; }
    if (nO > 0) { emit((k - (1ull << (hb + 3))) ^ turn ^ (cell << A), 1); n++; }
  }
  return n;
}
GM_HD int toot_level(const Desc& d, uint64_t k) {
  return popc64((k | (k >> d.A)) & d.full);
}

// The same rules with the board size fixed at compile time (the bucketed
// kernels instantiate it for the BASELINE board, 6x4, and the test boards):
// every mask, shift and the column loop fold to constants.  Bit-identical
// to toot_prim / toot_children (tests: both forms solve to the same
// fingerprints).
template <int L, int H>
struct TootFixed {
  static constexpr int A = L * H;
  static constexpr uint64_t full = (1ull << A) - 1;
  static constexpr uint64_t col0() {
    uint64_t m = 0;
    for (int y = 0; y < H; y++) m |= 1ull << (L * y);
    return m;
  }
  static constexpr uint64_t tmask(int i) {
    const int dxs[4] = {1, 0, 1, 1}, dys[4] = {0, 1, 1, -1};
    uint64_t m = 0;
    for (int x = 0; x < L; x++)
      for (int y = 0; y < H; y++) {
        const int ex = x + 3 * dxs[i], ey = y + 3 * dys[i];
        if (ex >= 0 && ex < L && ey >= 0 && ey < H) m |= 1ull << (L * y + x);
      }
    return m;
  }
  static constexpr int tstep(int i) {
    const int dxs[4] = {1, 0, 1, 1}, dys[4] = {0, 1, 1, -1};
    return dxs[i] + L * dys[i];
  }
  template <int S>
  static GM_HD uint64_t shr(uint64_t v) {
    if constexpr (S >= 0) return v >> S;
    else return v << (-S);
  }
  template <int I>
  static GM_HD int count_dir(uint64_t first, uint64_t mid) {
    constexpr int s = tstep(I);
    constexpr uint64_t m = tmask(I);
    if constexpr (m == 0) return 0;
    else return popc64(m & first & shr<s>(mid) & shr<2 * s>(mid) & shr<3 * s>(first));
  }
  static GM_HD int count(uint64_t first, uint64_t mid) {
    return count_dir<0>(first, mid) + count_dir<1>(first, mid) + count_dir<2>(first, mid) + count_dir<3>(first, mid);
  }
  static GM_HD int prim(const Desc&, uint64_t k) {
    const uint64_t t = k & full, o = (k >> A) & full;
    const int toot = count(t, o), otto = count(o, t);
    const bool p1 = (k >> (2 * A + 12)) & 1;
    if (toot == otto) return ((t | o) == full) ? TIE : UNDECIDED;
    return ((toot > otto) != p1) ? LOSS : WIN;
  }
  template <class F>
  static GM_HD int children(const Desc&, uint64_t k, F&& emit) {
    const uint64_t occ = (k | (k >> A)) & full;
    const int p1 = (int)((k >> (2 * A + 12)) & 1);
    const int hb = 2 * A + (p1 ? 0 : 6);
    const bool hasT = ((k >> hb) & 7) != 0, hasO = ((k >> (hb + 3)) & 7) != 0;
    constexpr uint64_t turn = 1ull << (2 * A + 12);
    const uint64_t kT = (k - (1ull << hb)) ^ turn, kO = (k - (1ull << (hb + 3))) ^ turn;
    int n = 0;
#pragma unroll
    for (int x = 0; x < L; x++) {
      if ((occ >> (L * (H - 1) + x)) & 1) continue;  // column full
      const uint64_t blank = ~(occ >> x) & col0();
      const uint64_t cell = (blank & (~blank + 1)) << x;
      if (hasT) { emit(kT ^ cell, 1); n++; }
      if (hasO) { emit(kO ^ (cell << A), 1); n++; }
    }
    return n;
  }
  static GM_HD int level(const Desc&, uint64_t k) { return popc64((k | (k >> A)) & full); }
};

// ---------------------------------------------------------------------------
// Othello (othello_bit_new.py), square boards.  key bits:
//   [0,A) WHITE plane, [A,2A) BLACK plane (board_get :251-257)
//   2A: 1 = BLACK to move (turn_count == 1), 0 = WHITE (turn_count == 2)
//   [2A+1, 2A+3): pass_count (0..2)
// Level = pieces - 4 + pass_count (every edge steps one level, passes
// included; a pass never switches the turn, :122-124).
// ---------------------------------------------------------------------------
GM_HD int oth_prim(const Desc& d, uint64_t k) {
  const int A = d.A;
  uint64_t w = k & d.full, b = (k >> A) & d.full;
  uint32_t passes = (uint32_t)((k >> (2 * A + 1)) & 3);
  if ((w | b) == d.full || passes >= 2) {  // :82-83
    int wc = popc64(w), bc = popc64(b);
    if (bc == wc) return TIE;
    bool black_to_move = (k >> (2 * A)) & 1;
    return ((bc > wc) != black_to_move) ? LOSS : WIN;  // :71-73
  }
  return UNDECIDED;
}
// pieces flipped by `me` playing cell (x,y); 0 if the move is not legal
GM_HD uint64_t oth_flips(const Desc& d, uint64_t me, uint64_t opp, int x, int y) {
  const int L = d.L, H = d.H;
  uint64_t flips = 0;
  for (int dx = -1; dx <= 1; dx++)
    for (int dy = -1; dy <= 1; dy++) {
      if (dx == 0 && dy == 0) continue;
      uint64_t run = 0;
      int cx = x + dx, cy = y + dy;
      while (cx >= 0 && cx < L && cy >= 0 && cy < H) {
        uint64_t bit = 1ull << (L * cy + cx);
        if (opp & bit) { run |= bit; cx += dx; cy += dy; continue; }
        if ((me & bit) && run) flips |= run;
        break;
      }
    }
  return flips;
}
// player_flip (othello_bit_new.py:228-235): every piece changes colour
// (flip :274-275 maps BLANK to BLANK), incr_turn toggles the side to move,
// the pass count stays.  Values and remoteness are invariant under it:
// oth_prim, the move rules and the level only see (mover, opponent) planes.
GM_HD uint64_t oth_flip(const Desc& d, uint64_t k) {
  const int A = d.A;
  const uint64_t w = k & d.full, b = (k >> A) & d.full, hi = ~((1ull << (2 * A)) - 1);
  return b | (w << A) | ((k ^ (1ull << (2 * A))) & hi);
}
// canonical representative: the smaller key of {k, player_flip(k)}
GM_HD uint64_t oth_canon(const Desc& d, uint64_t k) {
  if (!d.sym) return k;
  const uint64_t f = oth_flip(d, k);
  return f < k ? f : k;
}
template <class F>
GM_HD int oth_children(const Desc& d, uint64_t k, F&& emit) {
  const int A = d.A, L = d.L, H = d.H;
  uint64_t w = k & d.full, b = (k >> A) & d.full;
  bool black = (k >> (2 * A)) & 1;
  uint64_t me = black ? b : w, opp = black ? w : b;
  int n = 0;
  for (int x = 0; x < L; x++)       // gen_moves: x outer, y inner (:163-166)
    for (int y = 0; y < H; y++) {
      uint64_t cell = 1ull << (L * y + x);
      if ((w | b) & cell) continue;
      uint64_t f = oth_flips(d, me, opp, x, y);
      if (!f) continue;
      uint64_t nme = me | cell | f, nopp = opp & ~f;
      uint64_t nw = black ? nopp : nme, nb = black ? nme : nopp;
      // reset_pass, place + flip, incr_turn (:125-129)
      emit(oth_canon(d, nw | (nb << A) | ((uint64_t)(!black) << (2 * A))), 1);
      n++;
    }
  if (n == 0) {  // [None]: incr_pass only (:122-124)
    emit(oth_canon(d, k + (1ull << (2 * A + 1))), 1);
    n = 1;
  }
  return n;
}
GM_HD int oth_level(const Desc& d, uint64_t k) {
  return popc64((k | (k >> d.A)) & d.full) - 4 + (int)((k >> (2 * d.A + 1)) & 3);
}

// ---------------------------------------------------------------------------
// Static dispatch.  children(d, key, emit) calls emit(child, level_step) in
// gen_moves() order and returns the child count.
// ---------------------------------------------------------------------------
template <int KIND> struct Game;
template <> struct Game<K_SUM> {
  static GM_HD int prim(const Desc& d, uint64_t k) { return sum_prim(d, k); }
  template <class F> static GM_HD int children(const Desc& d, uint64_t k, F&& f) { return sum_children(d, k, f); }
  static GM_HD int level(const Desc& d, uint64_t k) { return sum_level(d, k); }
};
template <> struct Game<K_TTT> {
  static GM_HD int prim(const Desc& d, uint64_t k) { return ttt_prim(d, k); }
  template <class F> static GM_HD int children(const Desc& d, uint64_t k, F&& f) { return ttt_children(d, k, f); }
  static GM_HD int level(const Desc& d, uint64_t k) { return ttt_level(d, k); }
};
template <> struct Game<K_TOOT> {
  static GM_HD int prim(const Desc& d, uint64_t k) { return toot_prim(d, k); }
  template <class F> static GM_HD int children(const Desc& d, uint64_t k, F&& f) { return toot_children(d, k, f); }
  static GM_HD int level(const Desc& d, uint64_t k) { return toot_level(d, k); }
};
// compile-time toot boards (kernel instantiation ids, not descriptor kinds)
constexpr int K_TOOT_6x4 = 64, K_TOOT_5x4 = 54, K_TOOT_4x4 = 44;
template <> struct Game<K_TOOT_6x4> : TootFixed<6, 4> { static constexpr bool kFixed = true; };
template <> struct Game<K_TOOT_5x4> : TootFixed<5, 4> { static constexpr bool kFixed = true; };
template <> struct Game<K_TOOT_4x4> : TootFixed<4, 4> { static constexpr bool kFixed = true; };
// the instantiation id for a descriptor: a fixed toot board where one exists
GM_HD int fixed_kind(const Desc& d) {
  if (d.kind == K_TOOT && d.H == 4 && d.L >= 4 && d.L <= 6) return d.L * 10 + 4;
  return d.kind;
}
template <> struct Game<K_OTHELLO> {
  static GM_HD int prim(const Desc& d, uint64_t k) { return oth_prim(d, k); }
  template <class F> static GM_HD int children(const Desc& d, uint64_t k, F&& f) { return oth_children(d, k, f); }
  static GM_HD int level(const Desc& d, uint64_t k) { return oth_level(d, k); }
};

GM_HD int any_prim(const Desc& d, uint64_t k) {
  switch (d.kind) {
    case K_SUM: return sum_prim(d, k);
    case K_TTT: return ttt_prim(d, k);
    case K_TOOT: return toot_prim(d, k);
    default: return oth_prim(d, k);
  }
}
template <class F>
GM_HD int any_children(const Desc& d, uint64_t k, F&& f) {
  switch (d.kind) {
    case K_SUM: return sum_children(d, k, f);
    case K_TTT: return ttt_children(d, k, f);
    case K_TOOT: return toot_children(d, k, f);
    default: return oth_children(d, k, f);
  }
}
// canonical key of any position (identity without symmetry hooks)
GM_HD uint64_t any_canon(const Desc& d, uint64_t k) { return d.kind == K_OTHELLO ? oth_canon(d, k) : k; }
GM_HD int any_level(const Desc& d, uint64_t k) {
  switch (d.kind) {
    case K_SUM: return sum_level(d, k);
    case K_TTT: return ttt_level(d, k);
    case K_TOOT: return toot_level(d, k);
    default: return oth_level(d, k);
  }
}

}  // namespace gm
