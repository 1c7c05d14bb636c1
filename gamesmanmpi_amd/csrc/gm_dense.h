// gm_dense.h -- dense (perfect-hash) tier pipeline for rank-indexable games.
// Included by gm_solver.hip after the shared device helpers.
//
// For descriptors whose positions have a computable rank (K_SUM:
// four_to_one and the sum of Four-To-One heaps) the open-addressing table
// degenerates to a perfect hash, laid out LEVEL-MAJOR so that every child
// access of a wave is one contiguous stream:
//
//   slot(key) = level(key) * W + prefix(key)
//     prefix = rank / base[0]        (heap digits 1..K-1)
//     level  = root_sum - digit sum  (so heap 0 = (root_sum - level) - digitsum(prefix))
//
// A position at (L, p) has its children at (L+1, p) / (L+2, p) (heap 0 -1/-2)
// and (L+d, p - d*pstride[i]) (heap i>=1, -d): for 64 consecutive prefixes
// of one wave each child kind is 64 consecutive words.  Slots whose heap-0
// digit would fall outside [0, heap0] are holes: never read or written.
// Per slot: one reach bit (bitmap, written by the forward pass) and one
// 32-bit word value | remoteness << 2 (src/utils.py:3 value codes), written
// by the backward pass for reached slots only.  The key is implicit in the
// slot, so the traffic is ~0.2 B per position forward and 8 B per position
// + 4 B per edge backward instead of the 36 + 20 B of
// the keyed table.  ABSENT (0xFFFFFFFD) is a register-only "no such child"
// marker; W_REACHED/W_UNREACHED never appear in resolved words.

constexpr uint32_t W_UNREACHED = 0xFFFFFFFFu;

// Dense tables hold only WIN/LOSS positions (K_SUM: every primitive is a
// LOSS, four_to_one.py:19-22), stored in an ORDER form y whose unsigned max
// over a position's children is the whole reduction (reference-canonical
// _res_red/_remote_red, process.py:187-220):
//   WIN  remoteness r -> y = r                          (top bit 0)
//   LOSS remoteness r -> y = 0x80000000 | (0x7FFFFFFF - r)
// max over children: any LOSS child -> top bit set, low bits = 0x7FFFFFFF -
// (smallest LOSS remoteness) -> parent WIN, 1 + that; else max WIN
// remoteness -> parent LOSS, 1 + that.  An absent child reads 0 (a WIN of
// remoteness 0, which no position holds): neutral.  Converted to the
// value | remoteness << 2 word only where words leave the table (root,
// query).  W_UNREACHED marks reached-bit-clear slots (never read as
// children; readers check the reach bit first).
__host__ __device__ __forceinline__ uint32_t dense_word(uint32_t y) {
  return (y & 0x80000000u) ? make_word(LOSS, 0x7FFFFFFFu - (y & 0x7FFFFFFFu)) : make_word(WIN, y);
}
// parent order form from the max m over its children's order forms
__device__ __forceinline__ uint32_t dense_parent(uint32_t m) {
  return (m & 0x80000000u) ? (0x7FFFFFFFu - (m & 0x7FFFFFFFu)) + 1u : 0x80000000u | (0x7FFFFFFFu - (m + 1u));
}
constexpr uint32_t DENSE_PRIMITIVE = 0xFFFFFFFFu;  // LOSS, remoteness 0 (all heaps empty)

// digit i (i >= 1) of a prefix
__device__ __forceinline__ uint32_t pdigit(const Desc& d, u64 p, int i) {
  if (d.pow2) return (uint32_t)((p >> d.pshift[i]) & (d.base[i] - 1));
  return (uint32_t)((p / d.pstride[i]) % d.base[i]);
}

// prefix digits into registers.  MAXH is the compile-time heap count (exact
// for 1..8 heaps; 16 = generic bound with runtime checks) so every loop over
// heaps unrolls and all child/parent loads issue before the first wait
template <int MAXH>
__device__ __forceinline__ uint32_t prefix_digits(const Desc& d, u64 p, uint32_t (&h)[MAXH]) {
  uint32_t s = 0;
#pragma unroll
  for (int i = 1; i < MAXH; i++) {
    h[i] = ((MAXH <= 8) || i < d.nheaps) ? pdigit(d, p, i) : 0u;
    s += h[i];
  }
  return s;
}

// Digits of the 64 prefixes a wave covers.  For power-of-two bases and a
// 64-aligned wave base, digit_i(p_base | lane) = digit_i(p_base) +
// digit_i(lane): the first term is wave-uniform (computed on the scalar
// unit), the second a per-lane constant computed once per kernel.  For
// other bases every lane decomposes its own prefix.
template <int MAXH, bool POW2>
struct WaveDigits {
  uint32_t hl[MAXH];  // POW2: digits of the lane offset
  uint32_t sl;
  __device__ __forceinline__ void init(const Desc& d) {
    const uint32_t lane = __lane_id();
    sl = 0;
#pragma unroll
    for (int i = 1; i < MAXH; i++) {
      hl[i] = (POW2 && ((MAXH <= 8) || i < d.nheaps)) ? ((lane >> d.pshift[i]) & (d.base[i] - 1)) : 0u;
      sl += hl[i];
    }
  }
  // digits of p = wave_base + lane into h, returns the digit sum
  __device__ __forceinline__ uint32_t digits(const Desc& d, u64 wave_base, u64 p, uint32_t (&h)[MAXH]) const {
    if (!POW2) return prefix_digits<MAXH>(d, p, h);
    const u64 wb = __builtin_amdgcn_readfirstlane((uint32_t)wave_base) |
                   ((u64)__builtin_amdgcn_readfirstlane((uint32_t)(wave_base >> 32)) << 32);
    uint32_t s = sl;
#pragma unroll
    for (int i = 1; i < MAXH; i++) {
      uint32_t hb = ((MAXH <= 8) || i < d.nheaps) ? (uint32_t)((wb >> d.pshift[i]) & (d.base[i] - 1)) : 0u;
      h[i] = hb + hl[i];
      s += hb;
    }
    return s;
  }
};

__device__ __forceinline__ uint32_t prefix_digit_sum(const Desc& d, u64 p) {
  uint32_t s = 0;
  for (int i = 1; i < d.nheaps; i++) s += pdigit(d, p, i);
  return s;
}

__device__ __forceinline__ void slot_split(const Desc& d, u64 slot, u64* L, u64* p) {
  if (d.wshift >= 0) {
    *L = slot >> d.wshift;
    *p = slot & (d.W - 1);
  } else {
    *L = slot / d.W;
    *p = slot - *L * d.W;
  }
}

// heap-0 digit of (L, p), or -1 for a hole
__device__ __forceinline__ int64_t dense_h0(const Desc& d, u64 L, u64 p) {
  int64_t h0 = (int64_t)d.root_sum - (int64_t)L - (int64_t)prefix_digit_sum(d, p);
  return (h0 >= 0 && h0 <= (int64_t)d.heap[0]) ? h0 : -1;
}

__device__ __forceinline__ bool dense_slot_of(const Desc& d, u64 key, u64* slot) {
  u64 rest = key, p = key / d.base[0];
  uint32_t s = 0;
  for (int i = 0; i < d.nheaps; i++) {
    u64 q = rest / d.base[i];
    s += (uint32_t)(rest - q * d.base[i]);
    rest = q;
  }
  if (rest != 0 || s > d.root_sum) return false;  // outside the state space
  *slot = (u64)(d.root_sum - s) * d.W + p;
  return true;
}

// Reach marks live in a bitmap beside the words: level L's bit for local
// prefix q is bit (L * Wbl + q), so every 64-prefix group of one level owns
// one 64-bit word (written whole by one lane after a ballot).
__device__ __forceinline__ bool reach_bit(const u64* bits, u64 pos) {
  return (bits[pos >> 6] >> (pos & 63)) & 1ull;
}


// Forward, PULL form, target level L: each non-hole slot of level L ORs the
// reach bits of its parents -- the positions one move away, i.e. one heap +1
// (level L-1) or +2 (level L-2), the undo-moves of four_to_one.py:10-17 --
// and the wave writes its 64 bits at once.  Every bitmap word of a level is
// written by exactly one lane: no initialisation, no races.
template <int MAXH, bool POW2>
__global__ __launch_bounds__(256) void k_dense_pull(Desc d, DenseView v, u64* bits, u64 L, u64 root_p) {
  const uint32_t S = d.root_sum - (uint32_t)L;
  const u64 b0 = L * v.Wbl, b1 = (L - 1) * v.Wbl, b2 = (L - 2) * v.Wbl;  // b1/b2 used only when L >= 1/2
  const u64 stride = (u64)gridDim.x * blockDim.x;
  // whole waves over [p_lo, p_hi rounded up to 64): every lane reaches the
  // ballot (p_lo is a multiple of 64)
  const u64 n = (v.p_hi - v.p_lo + 63) & ~63ull;
  WaveDigits<MAXH, POW2> wd;
  wd.init(d);
  for (u64 i0 = (u64)blockIdx.x * blockDim.x + threadIdx.x; i0 < n; i0 += stride) {
    const u64 qi = v.p_lo + i0;  // sweep index
    const u64 qiw = __builtin_amdgcn_readfirstlane((uint32_t)(qi & ~63ull)) |
                    ((u64)__builtin_amdgcn_readfirstlane((uint32_t)(qi >> 32)) << 32);
    uint64_t qw;  // local prefix of the wave's lane 0
    bool run;
    const u64 pw = dense_sweep(v, qiw, &qw, &run);
    const u64 q = qw + (qi - qiw);
    if (!run) continue;  // wave-uniform: another launch's slice, or a halo
    const u64 p = pw + (q - qw);  // global prefix
    bool reached = false;
    uint32_t h[MAXH];
    const uint32_t s = wd.digits(d, pw, p, h);
    if (qi < v.p_hi && s <= S && S - s <= d.heap[0]) {  // not a hole
      if (L == 0) {
        reached = p == root_p;  // level 0 holds only the root
      } else {
        const uint32_t h0 = S - s;
        reached = (h0 + 1 <= d.heap[0] && reach_bit(bits, b1 + q)) ||
                  (L >= 2 && h0 + 2 <= d.heap[0] && reach_bit(bits, b2 + q));
#pragma unroll
        for (int i = 1; i < MAXH; i++) {
          const bool live = (MAXH <= 8) || i < d.nheaps;  // exact heap count when MAXH <= 8
          reached = reached || (live && h[i] + 1 <= d.heap[i] && reach_bit(bits, b1 + q + d.pstride[i])) ||
                    (live && L >= 2 && h[i] + 2 <= d.heap[i] && reach_bit(bits, b2 + q + 2 * d.pstride[i]));
        }
      }
    }
    const u64 m = __ballot(reached);
    if (__lane_id() == 0) bits[(b0 + qw) >> 6] = m;
  }
}

// ---------------------------------------------------------------------------
// Word-parallel pull (power-of-two layouts): one THREAD per 64-prefix group,
// i.e. per output bitmap word.  With pow2 bases and a 64-aligned group base
// pg, digit_i(pg + j) = digit_i(pg) + digit_i(j) for j < 64, so every
// per-prefix condition of the group is a 64-bit mask read from small
// tables (staged in LDS) indexed by the group's (uniform) digits:
//   TS[t]    = { j : sum_i digit_i(j) <= t }      (slot validity, heap-0 moves)
//   TD[i][t] = { j : digit_i(j) <= t }            (heap-i moves, i >= 1)
// and each parent kind contributes (64 parent bits, one or two word loads)
// AND (mask of j whose parent exists).  A level needs W/64 threads, each
// doing ~2K+2 word loads: no per-lane bit probes, no grid-stride rounds.
// ---------------------------------------------------------------------------
__device__ __forceinline__ u64 mask_le(const u64* T, int t) {
  return t < 0 ? 0ull : (t >= 63 ? ~0ull : T[t]);
}
// 64 bits of the bitmap starting at bit position pos
__device__ __forceinline__ u64 bits64_at(const u64* bits, u64 pos) {
  const u64 w = pos >> 6;
  const unsigned sh = (unsigned)(pos & 63);
  u64 lo = bits[w];
  return sh ? (lo >> sh) | (bits[w + 1] << (64 - sh)) : lo;
}

// Column-job tables (k_dense_resolve8c / k_dense_resolve4c)
constexpr int kMaxColJobs = 96;
struct ColJobs {
  uint32_t n;                     // slices
  uint32_t cum[kMaxColJobs + 1];  // groups before slice i (cum[n] = total)
  uint32_t lo[kMaxColJobs];       // first colperm entry of slice i
  uint32_t u[kMaxColJobs];        // local slice
  uint32_t t[kMaxColJobs];        // global top value
};
struct RowGeom {
  u64 Wl, Wbl, Z;
};

// One 64-prefix bitmap word of level L: reach bits = OR of the parents'
// bits (undo-moves +1/+2 on one heap), masked to the word's non-holes.  q =
// local prefix of lane-bit 0 (multiple of 64), pg = its global prefix, V0 =
// extra validity mask (band end), TS/TD = the mask tables in LDS.  Split in
// two: pull_issue loads every parent word the word can need (raw, no
// combining, so no wait is implied), pull_finish masks and ORs them -- the
// kernel issues the first item's loads BEFORE it fills the mask tables, so
// both memory rounds overlap.  Unneeded words are read but masked off; every
// index stays inside the bitmap (rows L-1 / L-2 plus at most two pstrides,
// i.e. at most into row L - 1 / L).
template <int MAXH>
struct PullLd {
  u64 w1, w2;                         // heap 0: same prefix, one / two levels up
  u64 a1[MAXH], b1[MAXH], a2[MAXH], b2[MAXH];  // heap i: the two words around the +1 / +2 parents
};
__device__ __forceinline__ u64 bits64_join(u64 lo, u64 hi, unsigned sh) {
  return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
}
template <int MAXH>
__device__ __forceinline__ void pull_issue(const Desc& d, u64 Wbl, const u64* bits, u64 L, u64 q, PullLd<MAXH>& X) {
  if (L == 0) return;
  const u64 p1 = (L - 1) * Wbl + q;
  X.w1 = bits[p1 >> 6];
#pragma unroll
  for (int i = 1; i < MAXH; i++) {
    if (!((MAXH <= 8) || i < d.nheaps)) continue;
    const u64 w = (p1 + d.pstride[i]) >> 6;
    X.a1[i] = bits[w];
    X.b1[i] = (d.pstride[i] & 63) ? bits[w + 1] : 0ull;
  }
  if (L < 2) return;
  const u64 p2 = (L - 2) * Wbl + q;
  X.w2 = bits[p2 >> 6];
#pragma unroll
  for (int i = 1; i < MAXH; i++) {
    if (!((MAXH <= 8) || i < d.nheaps)) continue;
    const u64 w = (p2 + 2 * d.pstride[i]) >> 6;
    X.a2[i] = bits[w];
    X.b2[i] = ((2 * d.pstride[i]) & 63) ? bits[w + 1] : 0ull;
  }
}
template <int MAXH>
__device__ __forceinline__ void pull_finish(const Desc& d, u64 Wbl, u64* bits, u64 L, u64 root_p, u64 q, u64 pg,
                                            u64 V0, const u64* TS, const u64* M, const PullLd<MAXH>& X) {
#define TD(i) (M + 64 * ((i) + 1))
  const int S = (int)(d.root_sum - (uint32_t)L);
  const int H0 = (int)d.heap[0];
  int dg[MAXH];
  int sg = 0;
#pragma unroll
  for (int i = 1; i < MAXH; i++) {
    const bool live = (MAXH <= 8) || i < d.nheaps;
    dg[i] = live ? (int)((pg >> d.pshift[i]) & (d.base[i] - 1)) : 0;
    sg += dg[i];
  }
  // valid: S - H0 <= sg + sj <= S
  const int lo_s = S - H0 - sg, hi_s = S - sg;
  const u64 V = mask_le(TS, hi_s) & ~mask_le(TS, lo_s - 1) & V0;
  u64 reached = 0;
  if (L == 0) {
    if (root_p >= pg && root_p < pg + 64) reached = 1ull << (root_p - pg);
  } else {
    // heap 0 +1 / +2: parent at the same prefix, one / two levels up;
    // exists iff h0 + d <= H0  <=>  sj >= lo_s + d
    reached |= X.w1 & ~mask_le(TS, lo_s);
    if (L >= 2) reached |= X.w2 & ~mask_le(TS, lo_s + 1);
#pragma unroll
    for (int i = 1; i < MAXH; i++) {
      const bool live = (MAXH <= 8) || i < d.nheaps;
      if (!live) continue;
      // heap i +1 / +2: exists iff dg + dj <= H_i - d
      const int Hi = (int)d.heap[i];
      reached |= bits64_join(X.a1[i], X.b1[i], (unsigned)(d.pstride[i] & 63)) & mask_le(TD(i), Hi - 1 - dg[i]);
      if (L >= 2)
        reached |= bits64_join(X.a2[i], X.b2[i], (unsigned)((2 * d.pstride[i]) & 63)) & mask_le(TD(i), Hi - 2 - dg[i]);
    }
  }
  bits[(L * Wbl + q) >> 6] = reached & V;
#undef TD
}

constexpr uint32_t kXcds = 8;
// Per-level XCD shares of a live-group list: share x = entries [o[x], o[x+1])
// (contiguous column ranges of ~equal live count, built at solver creation)
struct XcdShares {
  uint32_t o[9];
};

template <int MAXH>
__global__ __launch_bounds__(256) void k_dense_pull_words(Desc d, DenseView v, u64* bits, u64 L, u64 root_p,
                                                          const u64* __restrict__ masks,
                                                          const uint32_t* __restrict__ glist, XcdShares xs) {
  // mask tables (built once on the host at solver creation, gm_solver.hip
  // build_mask_tables): M[0..63] = TS, M[64 (i + 1) + t] = TD[i][t]
  __shared__ u64 M[64 * (MAXH + 1)];
  // one thread per 64-prefix bitmap word of the band, or of the level's
  // live 256-prefix groups (glist, world 1: words of groups without a
  // non-hole are never read unmasked, so they are not written).  List
  // sweeps are XCD-chunked (workgroup b runs on XCD b % 8, the host launches
  // a multiple of 8): the blocks of one XCD take one share, so the parent
  // words that neighbouring groups share (heap-3..5 parents 128 B - 128 KB
  // away) are fetched into one L2 instead of all eight.
  u64 g_first, ngroups, stride;
  if (glist) {
    const uint32_t x = blockIdx.x % kXcds;
    g_first = (u64)xs.o[x] * 4 + (u64)(blockIdx.x / kXcds) * blockDim.x + threadIdx.x;
    ngroups = (u64)xs.o[x + 1] * 4;
    stride = (u64)(gridDim.x / kXcds) * blockDim.x;
  } else {
    g_first = (u64)blockIdx.x * blockDim.x + threadIdx.x;
    ngroups = (v.p_hi - v.p_lo + 63) >> 6;
    stride = (u64)gridDim.x * blockDim.x;
  }
  // the first item (most launches give a thread a single one): its list
  // entry, then its parent words, are loaded before the table fill and
  // barrier, so the parent loads and the table loads share one memory round
  auto item = [&](u64 gi, uint32_t e, uint64_t* q, u64* pg, u64* V0) -> bool {
    const u64 qi = glist ? ((u64)e << 8) + ((gi & 3) << 6) : v.p_lo + (gi << 6);  // sweep index of lane-bit 0
    bool run;
    *pg = dense_sweep(v, qi, q, &run);  // global prefix of lane-bit 0; q = its local prefix
    *V0 = qi + 64 > v.p_hi ? (1ull << (v.p_hi - qi)) - 1 : ~0ull;
    return run;  // false: another launch's slice, or a halo
  };
  const bool has1 = g_first < ngroups;
  uint64_t q1 = 0;
  u64 pg1 = 0, V01 = 0;
  bool run1 = false;
  PullLd<MAXH> X;
  if (has1) {
    run1 = item(g_first, glist ? glist[g_first >> 2] : 0u, &q1, &pg1, &V01);
    if (run1) pull_issue<MAXH>(d, v.Wbl, bits, L, q1, X);
  }
  for (int k = threadIdx.x; k < 64 * (MAXH + 1); k += blockDim.x) M[k] = masks[k];
  __syncthreads();
  if (run1) pull_finish<MAXH>(d, v.Wbl, bits, L, root_p, q1, pg1, V01, M, M, X);
  for (u64 gi = g_first + stride; gi < ngroups; gi += stride) {
    uint64_t q;
    u64 pg, V0;
    if (!item(gi, glist ? glist[gi >> 2] : 0u, &q, &pg, &V0)) continue;
    pull_issue<MAXH>(d, v.Wbl, bits, L, q, X);
    pull_finish<MAXH>(d, v.Wbl, bits, L, root_p, q, pg, V0, M, M, X);
  }
}

// XCD-aware split of [0, n) (MI355X dispatches workgroup b to XCD b % 8):
// the blocks of one XCD grid-stride over one contiguous, 64-aligned chunk,
// so the child words that neighbouring prefixes share are fetched into ONE
// XCD's L2 instead of all eight.  Grids that are not a multiple of 8 blocks
// fall back to one plain grid-stride range.
struct XcdRange {
  u64 first, end, stride;
};
__device__ __forceinline__ XcdRange xcd_range(u64 n) {
  const uint32_t G = gridDim.x;
  const uint32_t nx = (G >= kXcds && G % kXcds == 0) ? kXcds : 1;
  const uint32_t x = blockIdx.x % nx, lb = blockIdx.x / nx;
  const u64 chunk = ((n + nx - 1) / nx + 63) & ~63ull;
  const u64 b = min(n, (u64)x * chunk);
  XcdRange r;
  r.end = min(n, b + chunk);
  r.first = b + (u64)lb * blockDim.x + threadIdx.x;
  r.stride = (u64)(G / nx) * blockDim.x;
  return r;
}

// One level row of words for child loads.  BUF: a raw buffer resource
// (32-bit byte offsets, hardware range check): an absent child is given an
// out-of-range offset and reads 0 with no memory access; a missing row
// (level past the table) has zero records.  !BUF: 64-bit global loads for
// rows of 2^30 words or more.
template <bool BUF>
struct WordRow;
template <>
struct WordRow<true> {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ void init(const uint32_t* base, u64 nwords) {
    r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(uint32_t)(nwords * 4u), 0x00020000);
  }
  __device__ __forceinline__ uint32_t at(u64 idx, bool ok) const {
    return __builtin_amdgcn_raw_buffer_load_b32(r, ok ? (uint32_t)idx * 4u : 0xFFFFFFFCu, 0, 0);
  }
};
template <>
struct WordRow<false> {
  const uint32_t* p;
  u64 n;
  __device__ __forceinline__ void init(const uint32_t* base, u64 nwords) {
    p = base;
    n = nwords;
  }
  // the range check mirrors the buffer form (wrapped indices read 0)
  __device__ __forceinline__ uint32_t at(u64 idx, bool ok) const { return (ok && idx < n) ? p[idx] : 0u; }
};

// backward, level L: resolve every reached owned position from its children.
// Absent children read as 0 (= WIN, remoteness 0, which no resolved
// position holds), neutral for every term of the reduction, so each child
// costs a load and a few ALU ops (reference-canonical _res_red/_remote_red):
//   value       WIN if any child LOSS, else TIE if any TIE, else DRAW if any
//               DRAW, else LOSS      (min / max of the remapped value codes)
//   remoteness  WIN: 1 + min rem over LOSS children, else 1 + max rem over
//               all children         (min of LOSS words, max of words)
// The reach-bit word is loaded with the child words (children of a non-hole
// slot are never holes), so a round costs one memory latency.
template <int MAXH, bool POW2, bool BUF, int U, bool BLK>
__global__ __launch_bounds__(256) void k_dense_resolve(Desc d, DenseView v, uint32_t* words, const u64* bits, u64 L,
                                                       DevState* st) {
  const uint32_t S = d.root_sum - (uint32_t)L;
  uint32_t* mine = words + L * v.Wl;
  WordRow<BUF> n1, n2;  // levels L+1, L+2 (empty rows past the last level)
  n1.init(words + (L + 1) * v.Wl, S >= 1 ? v.Wl : 0);
  n2.init(words + (L + 2) * v.Wl, S >= 2 ? v.Wl : 0);
  u64 npos = 0, edges = 0, prims = 0;
  WaveDigits<MAXH, POW2> wd;
  wd.init(d);
  const XcdRange r = xcd_range(v.p_hi - v.p_lo);
  for (u64 i0 = r.first; i0 < r.end; i0 += U * r.stride) {
    // U grid-stride rounds per iteration: all their loads issue before the
    // first wait
    uint32_t c[U][2 * MAXH];
    u64 rw[U], qs[U];
    uint32_t nch[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      ok[u] = false;
      rw[u] = 0;
      nch[u] = 0;
      const u64 iu = i0 + (u64)u * r.stride;
      u64 q = v.p_lo + iu;  // local prefix (world 1) / sweep index (shards)
      u64 qw = q & ~63ull;
      bool run = true;
      u64 pw = qw;  // world 1: local = global
      if (BLK) {
        const u64 qiw = __builtin_amdgcn_readfirstlane((uint32_t)qw) |
                        ((u64)__builtin_amdgcn_readfirstlane((uint32_t)(qw >> 32)) << 32);
        uint64_t lq;
        pw = dense_sweep(v, qiw, &lq, &run);
        q = lq + (q - qw);
        qw = lq;
      }
      qs[u] = q;
      const u64 p = pw + (q - qw);  // global prefix
      uint32_t h[MAXH];
      const uint32_t s = wd.digits(d, pw, p, h);
      const bool valid = run && iu < r.end && s <= S && S - s <= d.heap[0];  // not a hole
      if (!__ballot(valid)) continue;                                 // a wave of holes
      if (!valid) continue;
      ok[u] = true;
      // the wave's 64 reach bits (one uniform word), loaded with the children
      rw[u] = bits[__builtin_amdgcn_readfirstlane((uint32_t)((L * v.Wbl + q) >> 6)) |
                   ((u64)__builtin_amdgcn_readfirstlane((uint32_t)(((L * v.Wbl + q) >> 6) >> 32)) << 32)];
      const uint32_t h0 = S - s;
      nch[u] = min(h0, 2u);
      c[u][0] = n1.at(q, h0 >= 1);
      c[u][1] = n2.at(q, h0 >= 2);
#pragma unroll
      for (int i = 1; i < MAXH; i++) {
        const bool live = (MAXH <= 8) || i < d.nheaps;
        c[u][2 * i] = n1.at(q - d.pstride[i], live && h[i] >= 1);
        c[u][2 * i + 1] = n2.at(q - 2 * d.pstride[i], live && h[i] >= 2);
        nch[u] += live ? min(h[i], 2u) : 0u;
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (!ok[u]) continue;
      // order forms: the max over the children is the reduction (absent
      // children read 0, neutral)
      uint32_t m = 0;
#pragma unroll
      for (int j = 0; j < 2 * MAXH; j++) m = max(m, c[u][j]);
      const uint32_t word = S == 0 ? DENSE_PRIMITIVE : dense_parent(m);
      // Every non-hole slot is written (the word is consumed unconditionally,
      // so the child loads issue together with the reach word); unreached
      // slots get W_UNREACHED and are never read as children.
      const u64 q = qs[u];
      const bool reached = (rw[u] >> (q & 63)) & 1ull;
      mine[q] = reached ? word : W_UNREACHED;
      if (reached) {
        npos++;
        edges += (u64)nch[u];
        prims += S == 0;
      }
    }
  }
  block_add(&st->cursor_front, npos);  // positions resolved
  block_add(&st->edges, edges);
  block_add(&st->prims, prims);
}

// ---------------------------------------------------------------------------
// Four prefixes per lane (power-of-two tables with base[1] >= 4): a lane
// resolves prefixes q..q+3 (q 4-aligned), which share every digit but the
// lowest (h1 + e), so every child stream of the lane is ONE 16-B load:
//   heap 0 -d : row L+d words [q, q+4)                      (A_d)
//   heap 1 -d : row L+d words [q-d, q-d+4) = tail of the aligned quad
//               [q-4, q) (P_d) followed by the head of A_d
//   heap i -d : row L+d words [q - d stride_i, +4)           (i >= 2, aligned)
// 2K+1 memory instructions per four positions instead of per position, and
// four times the bytes in flight per instruction: the k_dense_resolve
// kernel is latency/issue-bound, this one is not.  Per
// element e the digit sum is s + e, so validity (not a hole) and child
// existence are per-element compares; quads touching hole slots are loaded
// whole and the hole words (never written, so garbage) masked to 0 before
// the reduction.  Stores are one 16-B store when all four are non-holes,
// else per-element stores (holes stay untouched).
// ---------------------------------------------------------------------------
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// a level's live-group list split into 8 XCD shares: share x = entries
// [o[x], o[x + 1]) (blocks b with b % 8 == x sweep it)
struct WordRow4 {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ void init(const uint32_t* base, u64 nwords) {
    r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(uint32_t)(nwords * 4u), 0x00020000);
  }
  // words [idx, idx + 4), idx 4-aligned; !ok reads zeros with no memory access
  __device__ __forceinline__ u32x4 at(u64 idx, bool ok) const {
    return __builtin_amdgcn_raw_buffer_load_b128(r, ok ? (uint32_t)idx * 4u : 0xFFFFFFF0u, 0, 0);
  }
};

// Body shared by the quad kernels: one lane, four prefixes.  q = local
// prefix of element 0 (4-aligned), pw = global prefix of the wave's element
// 0 (256-aligned), qi/qlo/qhi = sweep index of element 0 and the launch's
// sweep range (elements outside are skipped).
struct Quad4 {
  WordRow4 n1, n2;  // levels L+1, L+2 (empty rows past the last level)
  uint32_t* mine;
  const u64* bits;
  u64 Lb;  // L * Wbl
  uint32_t S, H0;
  uint32_t npos = 0, edges = 0;  // per thread: far below 2^32
};
template <int MAXH>
__device__ __forceinline__ void lane_digits4(const Desc& d, uint32_t (&hl)[MAXH], uint32_t& sl) {
  const uint32_t lane = __lane_id();
  sl = 0;
#pragma unroll
  for (int i = 1; i < MAXH; i++) {
    hl[i] = ((MAXH <= 8) || i < d.nheaps) ? (((4u * lane) >> d.pshift[i]) & (d.base[i] - 1)) : 0u;
    sl += hl[i];
  }
}
template <int MAXH>
__device__ __forceinline__ void resolve_quad(const Desc& d, Quad4& Q, const uint32_t (&hl)[MAXH], uint32_t sl, u64 q,
                                             u64 pw, u64 qi, u64 qlo, u64 qhi) {
  const uint32_t S = Q.S;
  uint32_t h[MAXH];
  uint32_t s = sl;
#pragma unroll
  for (int i = 1; i < MAXH; i++) {
    const uint32_t hb = ((MAXH <= 8) || i < d.nheaps) ? (uint32_t)((pw >> d.pshift[i]) & (d.base[i] - 1)) : 0u;
    h[i] = hb + hl[i];
    s += hb;
  }
  // element e: digit sum s + e, heap 0 = S - s - e
  uint32_t valid = 0;
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const uint32_t se = s + e;
    const bool ok = qi + e >= qlo && qi + e < qhi && se <= S && S - se <= Q.H0;
    valid |= (uint32_t)ok << e;
  }
  if (!__ballot(valid != 0)) return;  // a wave of holes
  if (!valid) return;
  const u64 bw = (Q.Lb + q) >> 6;
  const uint32_t rbits = (uint32_t)(Q.bits[bw] >> ((Q.Lb + q) & 63)) & 15u;
  const u32x4 A1 = Q.n1.at(q, true), A2 = Q.n2.at(q, true);
#ifdef GM_DIAG_SKIP
  constexpr uint32_t kDiag = GM_DIAG_SKIP;
#else
  constexpr uint32_t kDiag = 0;
#endif
  u32x4 P1 = Q.n1.at(q - 4, !(kDiag & 64) && q >= 4), P2 = Q.n2.at(q - 4, !(kDiag & 64) && q >= 4);
  u32x4 C1[MAXH], C2[MAXH];
#pragma unroll
  for (int i = 2; i < MAXH; i++) {
    const bool live = (MAXH <= 8) || i < d.nheaps;
    const bool on = !((kDiag >> i) & 1u);
    C1[i] = Q.n1.at(q - d.pstride[i], on && live && h[i] >= 1);
    C2[i] = Q.n2.at(q - 2 * d.pstride[i], on && live && h[i] >= 2);
  }
  uint32_t nch_hi = 0;  // children through heaps >= 2 (same for the four)
#pragma unroll
  for (int i = 2; i < MAXH; i++) nch_hi += ((MAXH <= 8) || i < d.nheaps) ? min(h[i], 2u) : 0u;
  uint32_t out[4];
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const uint32_t h0 = S - (s + e), h1 = h[1] + e;
    // heap 0: same prefix; heap 1: one / two prefixes down.  Order forms
    // (see dense_word): the max over the children is the reduction;
    // heap-0/1 quads may hold hole words (masked to 0)
    uint32_t m = max(h0 >= 1 ? A1[e] : 0u, h0 >= 2 ? A2[e] : 0u);
    m = max(m, max(h1 >= 1 ? (e >= 1 ? A1[e - 1] : P1[3]) : 0u, h1 >= 2 ? (e >= 2 ? A2[e - 2] : P2[2 + e]) : 0u));
#pragma unroll
    for (int i = 2; i < MAXH; i++) m = max(m, max(C1[i][e], C2[i][e]));
    const uint32_t word = S == 0 ? DENSE_PRIMITIVE : dense_parent(m);
    const bool reached = (rbits >> e) & 1u;
    out[e] = reached ? word : W_UNREACHED;
    if (reached && ((valid >> e) & 1u)) {
      Q.npos++;
      Q.edges += min(h0, 2u) + min(h1, 2u) + nch_hi;
    }
  }
  if (kDiag & 128) {
  } else if (valid == 15u) {
    u32x4 o4 = {out[0], out[1], out[2], out[3]};
    *(u32x4*)(Q.mine + q) = o4;
  } else {
#pragma unroll
    for (int e = 0; e < 4; e++)
      if ((valid >> e) & 1u) Q.mine[q + e] = out[e];
  }
}
// Software-pipelined form (k_dense_resolve4p): quad_issue computes a
// lane's digits and issues every load of one group; quad_finish reduces and
// stores.  A wave issues group k+1's loads before finishing group k, so the
// wait for group k's data never covers group k-1's store (gfx9 counts
// loads and stores in one in-order vmcnt: without the pipeline every
// group's loads also waited for the previous group's store acknowledgement;
// skipping the stores altogether measured 14.3 -> 10.6 ms per solve).
template <int MAXH>
struct QuadLoads {
  u32x4 A1, A2, P1, P2, C1[MAXH], C2[MAXH];
  u64 bitsw;
  u64 q;
  uint32_t h1, s, valid, nch_hi;
};
template <int MAXH>
__device__ __forceinline__ void quad_issue(const Desc& d, const Quad4& Q, const uint32_t (&hl)[MAXH], uint32_t sl,
                                           u64 q, u64 pw, bool on, QuadLoads<MAXH>& X) {
  const uint32_t S = Q.S;
  uint32_t h[MAXH];
  uint32_t s = sl;
#pragma unroll
  for (int i = 1; i < MAXH; i++) {
    const uint32_t hb = ((MAXH <= 8) || i < d.nheaps) ? (uint32_t)((pw >> d.pshift[i]) & (d.base[i] - 1)) : 0u;
    h[i] = hb + hl[i];
    s += hb;
  }
  uint32_t valid = 0;
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const uint32_t se = s + e;
    valid |= (uint32_t)(on && se <= S && S - se <= Q.H0) << e;
  }
  X.q = q;
  X.h1 = h[1];
  X.s = s;
  X.valid = valid;
  uint32_t nch_hi = 0;
#pragma unroll
  for (int i = 2; i < MAXH; i++) nch_hi += ((MAXH <= 8) || i < d.nheaps) ? min(h[i], 2u) : 0u;
  X.nch_hi = nch_hi;
  // lanes (and waves) without a non-hole issue nothing: out-of-range
  // buffer offsets read zeros without a memory access
  const bool any = valid != 0;
  X.bitsw = any ? Q.bits[(Q.Lb + q) >> 6] : 0ull;
  X.A1 = Q.n1.at(q, any);
  X.A2 = Q.n2.at(q, any);
  X.P1 = Q.n1.at(q - 4, any && q >= 4);
  X.P2 = Q.n2.at(q - 4, any && q >= 4);
#pragma unroll
  for (int i = 2; i < MAXH; i++) {
    const bool live = (MAXH <= 8) || i < d.nheaps;
    X.C1[i] = Q.n1.at(q - d.pstride[i], any && live && h[i] >= 1);
    X.C2[i] = Q.n2.at(q - 2 * d.pstride[i], any && live && h[i] >= 2);
  }
}
template <int MAXH>
__device__ __forceinline__ void quad_finish(Quad4& Q, const QuadLoads<MAXH>& X) {
  const uint32_t valid = X.valid;
  if (!valid) return;
  const uint32_t S = Q.S;
  const uint32_t rbits = (uint32_t)(X.bitsw >> ((Q.Lb + X.q) & 63)) & 15u;
  uint32_t out[4];
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const uint32_t h0 = S - (X.s + e), h1 = X.h1 + e;
    uint32_t m = max(h0 >= 1 ? X.A1[e] : 0u, h0 >= 2 ? X.A2[e] : 0u);
    m = max(m, max(h1 >= 1 ? (e >= 1 ? X.A1[e - 1] : X.P1[3]) : 0u,
                   h1 >= 2 ? (e >= 2 ? X.A2[e - 2] : X.P2[2 + e]) : 0u));
#pragma unroll
    for (int i = 2; i < MAXH; i++) m = max(m, max(X.C1[i][e], X.C2[i][e]));
    const uint32_t word = S == 0 ? DENSE_PRIMITIVE : dense_parent(m);
    const bool reached = (rbits >> e) & 1u;
    out[e] = reached ? word : W_UNREACHED;
    if (reached && ((valid >> e) & 1u)) {
      Q.npos++;
      Q.edges += min(h0, 2u) + min(h1, 2u) + X.nch_hi;
    }
  }
  if (valid == 15u) {
    u32x4 o4 = {out[0], out[1], out[2], out[3]};
    *(u32x4*)(Q.mine + X.q) = o4;
  } else {
#pragma unroll
    for (int e = 0; e < 4; e++)
      if ((valid >> e) & 1u) Q.mine[X.q + e] = out[e];
  }
}

__device__ __forceinline__ void quad_init(Quad4& Q, const Desc& d, uint32_t* words, const u64* bits, u64 L, u64 Wl,
                                          u64 Wbl) {
  Q.S = d.root_sum - (uint32_t)L;
  Q.H0 = d.heap[0];
  Q.mine = words + L * Wl;
  Q.n1.init(words + (L + 1) * Wl, Q.S >= 1 ? Wl : 0);
  Q.n2.init(words + (L + 2) * Wl, Q.S >= 2 ? Wl : 0);
  Q.bits = bits;
  Q.Lb = L * Wbl;
}
__device__ __forceinline__ void quad_done(const Quad4& Q, DevState* st) {
  block_add(&st->cursor_front, (u64)Q.npos);  // positions resolved
  block_add(&st->edges, (u64)Q.edges);
  block_add(&st->prims, Q.S == 0 ? (u64)Q.npos : 0ull);
}

// Sweep forms: the level's band (world 1), the level's live-group list
// (world 1, XCD shares), or a shard's listed slices (BLK).
template <int MAXH, bool BLK>
__global__ __launch_bounds__(256) void k_dense_resolve4(Desc d, DenseView v, uint32_t* words, const u64* bits, u64 L,
                                                        DevState* st, const uint32_t* __restrict__ glist,
                                                        XcdShares xs) {
  Quad4 Q;
  quad_init(Q, d, words, bits, L, v.Wl, v.Wbl);
  uint32_t hl[MAXH], sl;
  lane_digits4<MAXH>(d, hl, sl);
  // units of four prefixes over [p_lo rounded down to 256, p_hi), or over
  // the level's live 256-prefix groups (glist, 64 units each)
  const u64 lo = v.p_lo & ~255ull;
  XcdRange r;
  if (glist) {  // grid is a multiple of 8 blocks (host)
    const uint32_t x = blockIdx.x % kXcds;
    r.first = (u64)xs.o[x] * 64 + (u64)(blockIdx.x / kXcds) * blockDim.x + threadIdx.x;
    r.end = (u64)xs.o[x + 1] * 64;
    r.stride = (u64)(gridDim.x / kXcds) * blockDim.x;
  } else {
    r = xcd_range((v.p_hi - lo + 3) >> 2);
  }
  for (u64 iu = r.first; iu < r.end; iu += r.stride) {
    // sweep index of element 0 (the wave's 64 units are one group)
    const u64 qi = glist ? ((u64)glist[__builtin_amdgcn_readfirstlane((uint32_t)(iu >> 6))] << 8) + 4 * (iu & 63)
                         : lo + 4 * iu;
    const u64 qiw = __builtin_amdgcn_readfirstlane((uint32_t)(qi & ~255ull)) |
                    ((u64)__builtin_amdgcn_readfirstlane((uint32_t)(qi >> 32)) << 32);
    u64 qw = qiw, pw = qiw;  // local / global prefix of the wave's element 0
    bool run = true;
    if (BLK) {
      uint64_t lq;
      pw = dense_sweep(v, qiw, &lq, &run);
      qw = lq;
    }
    if (!run) continue;  // wave-uniform: another launch's slice, or a halo
    resolve_quad<MAXH>(d, Q, hl, sl, qw + (qi - qiw), pw, qi, v.p_lo, v.p_hi);
  }
  quad_done(Q, st);
}

// Live-group list sweep (world 1), software-pipelined: see quad_issue.
#ifndef GM_R4P_PIPE
#define GM_R4P_PIPE 1
#endif
template <int MAXH>
__global__ __launch_bounds__(256) void k_dense_resolve4p(Desc d, DenseView v, uint32_t* words, const u64* bits, u64 L,
                                                         DevState* st, const uint32_t* __restrict__ glist,
                                                         XcdShares xs) {
  Quad4 Q;
  quad_init(Q, d, words, bits, L, v.Wl, v.Wbl);
  uint32_t hl[MAXH], sl;
  lane_digits4<MAXH>(d, hl, sl);
  const uint32_t x = blockIdx.x % kXcds;
  const u64 first = (u64)xs.o[x] * 64 + (u64)(blockIdx.x / kXcds) * blockDim.x + threadIdx.x;
  const u64 end = (u64)xs.o[x + 1] * 64, stride = (u64)(gridDim.x / kXcds) * blockDim.x;
  auto issue = [&](u64 iu, QuadLoads<MAXH>& X) {
    const bool on = iu < end;  // wave-uniform (64-unit aligned ranges)
    const uint32_t gi = __builtin_amdgcn_readfirstlane((uint32_t)((on ? iu : first) >> 6));
    const u64 pw = (u64)glist[gi] << 8;  // world 1: local = global prefix
    quad_issue<MAXH>(d, Q, hl, sl, pw + 4 * (iu & 63), pw, on, X);
  };
#if GM_R4P_PIPE
  if (first < end) {
    // two register sets, statically named (a dynamically indexed pair
    // would live in scratch)
    QuadLoads<MAXH> X0, X1;
    issue(first, X0);
    for (u64 iu = first; iu < end; iu += 2 * stride) {
      issue(iu + stride, X1);  // next group's loads before this group's store
      quad_finish<MAXH>(Q, X0);
      if (iu + stride >= end) break;
      issue(iu + 2 * stride, X0);
      quad_finish<MAXH>(Q, X1);
    }
  }
#else
  for (u64 iu = first; iu < end; iu += stride) {
    QuadLoads<MAXH> X;
    issue(iu, X);
    quad_finish<MAXH>(Q, X);
  }
#endif
  quad_done(Q, st);
}

// ---------------------------------------------------------------------------
// 16-bit tables (world 1, k_dense_resolve8p).  K_SUM remoteness never exceeds
// root_sum, so below 2^15 the order form fits 16 bits: WIN r -> r, LOSS r ->
// 0x8000 | (0x7FFF - r) -- the same ordering, so the unsigned max over the
// children is still the whole reduction, and an absent child (0) is still
// neutral.  Half the bytes per child stream, and a 16-B load now carries
// EIGHT consecutive prefixes: a lane owns an octet (the eight share every
// digit but the lowest, base[1] >= 8), a wave two 256-prefix groups of the
// level's live-group list, so each group costs half the memory instructions
// of the quad form.  Converted to value | remoteness << 2 at the root and in
// queries (dense_word16).  Octet stores are whole 16-B stores: the hole
// slots they overwrite are never read unmasked (heap-0/1 children of a
// valid parent are masked when they would be holes; heap >= 2 children of a
// valid parent are never holes).
// ---------------------------------------------------------------------------
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
constexpr uint32_t W16_UNREACHED = 0xFFFFu;
constexpr uint32_t DENSE_PRIMITIVE16 = 0xFFFFu;  // LOSS, remoteness 0
__device__ __forceinline__ uint32_t dense_parent16(uint32_t m) {
  return (m & 0x8000u) ? (0x7FFFu - (m & 0x7FFFu)) + 1u : 0x8000u | (0x7FFFu - (m + 1u));
}
__host__ __device__ __forceinline__ uint32_t dense_word16(uint32_t h) {
  return dense_word((h & 0x8000u) ? (0xFFFF8000u | h) : h);
}
// 8-bit order form (k_dense_resolve16p) -> the 32-bit one -> value | rem << 2
__host__ __device__ __forceinline__ uint32_t dense_word8(uint32_t h) {
  return dense_word((h & 0x80u) ? 0x80000000u | (0x7FFFFFFFu - 2u * (0x7Fu - (h & 0x7Fu))) : 2u * h + 1u);
}
// the word at index i of a table of wbits-bit words
__host__ __device__ __forceinline__ uint32_t dense_word_at(const void* words, u64 i, uint32_t wbits) {
  return wbits == 8 ? dense_word8(((const uint8_t*)words)[i])
         : wbits == 16 ? dense_word16(((const uint16_t*)words)[i])
                       : dense_word(((const uint32_t*)words)[i]);
}
struct WordRow8 {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ void init(const uint16_t* base, u64 nwords) {
    r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(uint32_t)(nwords * 2u), 0x00020000);
  }
  // words [idx, idx + 8), idx 8-aligned; !ok reads zeros with no memory access
  __device__ __forceinline__ u16x8 at(u64 idx, bool ok) const {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, ok ? (uint32_t)idx * 2u : 0xFFFFFFF0u, 0, 0);
    return __builtin_bit_cast(u16x8, v);
  }
};
struct Oct8 {
  WordRow8 n1, n2;  // levels L+1, L+2 (empty rows past the last level)
  uint16_t* mine;
  const u64* bits;
  u64 Lb;  // L * Wbl
  uint32_t S, H0;
  uint32_t npos = 0, edges = 0;
};
template <int MAXH>
struct OctLoads {
  u16x8 A1, A2, P1, P2, C1[MAXH], C2[MAXH];
  u64 bitsw;
  u64 q;
  uint32_t h1, s, valid, nch_hi;
};
__device__ __forceinline__ void oct_init(Oct8& Q, const Desc& d, uint16_t* words, const u64* bits, u64 L, u64 Wl,
                                         u64 Wbl) {
  Q.S = d.root_sum - (uint32_t)L;
  Q.H0 = d.heap[0];
  Q.mine = words + L * Wl;
  Q.n1.init(words + (L + 1) * Wl, Q.S >= 1 ? Wl : 0);
  Q.n2.init(words + (L + 2) * Wl, Q.S >= 2 ? Wl : 0);
  Q.bits = bits;
  Q.Lb = L * Wbl;
}
// digits of the lane's global prefix pg and every load of its octet at local
// prefix q (both 8-aligned; world 1: q = pg)
template <int MAXH>
__device__ __forceinline__ void oct_issue(const Desc& d, const Oct8& Q, u64 q, u64 pg, bool on, OctLoads<MAXH>& X) {
  const uint32_t S = Q.S;
  uint32_t h[MAXH];
  uint32_t s = 0;
#pragma unroll
  for (int i = 1; i < MAXH; i++) {
    h[i] = ((MAXH <= 8) || i < d.nheaps) ? (uint32_t)((pg >> d.pshift[i]) & (d.base[i] - 1)) : 0u;
    s += h[i];
  }
  uint32_t valid = 0;
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const uint32_t se = s + e;
    valid |= (uint32_t)(on && se <= S && S - se <= Q.H0) << e;
  }
  X.q = q;
  X.h1 = h[1];
  X.s = s;
  X.valid = valid;
  uint32_t nch_hi = 0;
#pragma unroll
  for (int i = 2; i < MAXH; i++) nch_hi += ((MAXH <= 8) || i < d.nheaps) ? min(h[i], 2u) : 0u;
  X.nch_hi = nch_hi;
  const bool any = valid != 0;
  X.bitsw = any ? Q.bits[(Q.Lb + q) >> 6] : 0ull;
  X.A1 = Q.n1.at(q, any);
  X.A2 = Q.n2.at(q, any);
  X.P1 = Q.n1.at(q - 8, any && q >= 8);
  X.P2 = Q.n2.at(q - 8, any && q >= 8);
#pragma unroll
  for (int i = 2; i < MAXH; i++) {
    const bool live = (MAXH <= 8) || i < d.nheaps;
    X.C1[i] = Q.n1.at(q - d.pstride[i], any && live && h[i] >= 1);
    X.C2[i] = Q.n2.at(q - 2 * d.pstride[i], any && live && h[i] >= 2);
  }
}
template <int MAXH>
__device__ __forceinline__ void oct_finish(Oct8& Q, const OctLoads<MAXH>& X) {
  const uint32_t valid = X.valid;
  if (!valid) return;
  const uint32_t S = Q.S;
  const uint32_t rbits = (uint32_t)(X.bitsw >> ((Q.Lb + X.q) & 63)) & 0xFFu;
  u16x8 mc = {0, 0, 0, 0, 0, 0, 0, 0};  // heaps >= 2: never holes under a valid parent
#pragma unroll
  for (int i = 2; i < MAXH; i++) mc = __builtin_elementwise_max(mc, __builtin_elementwise_max(X.C1[i], X.C2[i]));
  u16x8 o;
#pragma unroll
  for (int e = 0; e < 8; e++) {
    const uint32_t h0 = S - (X.s + e), h1 = X.h1 + e;
    uint32_t m = max(h0 >= 1 ? (uint32_t)X.A1[e] : 0u, h0 >= 2 ? (uint32_t)X.A2[e] : 0u);
    m = max(m, max(h1 >= 1 ? (uint32_t)(e >= 1 ? X.A1[e - 1] : X.P1[7]) : 0u,
                   h1 >= 2 ? (uint32_t)(e >= 2 ? X.A2[e - 2] : X.P2[6 + e]) : 0u));
    m = max(m, (uint32_t)mc[e]);
    const uint32_t word = S == 0 ? DENSE_PRIMITIVE16 : dense_parent16(m);
    const bool reached = (rbits >> e) & 1u;
    o[e] = (uint16_t)(reached ? word : W16_UNREACHED);
    if (reached && ((valid >> e) & 1u)) {
      Q.npos++;
      Q.edges += min(h0, 2u) + min(h1, 2u) + X.nch_hi;
    }
  }
  *(u16x8*)(Q.mine + X.q) = o;
}
// Live-group list sweep over a 16-bit table (software-pipelined like
// k_dense_resolve4p when GM_R8P_PIPE).  Units of 8 prefixes, 32 per group; the host starts
// every XCD share at an even list entry, so a wave's 64 units are two whole
// groups (lanes 0-31 / 32-63), read with two scalar loads.
// one unit in flight per lane (88 VGPRs, 5 waves per SIMD) against the
// two-stage pipeline (GM_R8P_PIPE 1: 3 waves): GM_F_WORDS16 bench backward
// 5.35 -> 5.08 ms (tools/ab_dense.sh default:64 against a variant)
#ifndef GM_R8P_PIPE
#define GM_R8P_PIPE 0
#endif
template <int MAXH>
__device__ __forceinline__ void resolve8p_body(const Desc& d, const DenseView& v, uint16_t* words, const u64* bits,
                                               u64 L, DevState* st, const uint32_t* __restrict__ glist,
                                               const XcdShares& xs, BlockCount* bc) {
  Oct8 Q;
  oct_init(Q, d, words, bits, L, v.Wl, v.Wbl);
  const uint32_t lane = __lane_id();
  const uint32_t x = blockIdx.x % kXcds;
  const u64 first = (u64)xs.o[x] * 32 + (u64)(blockIdx.x / kXcds) * blockDim.x + threadIdx.x;
  const u64 end = (u64)xs.o[x + 1] * 32, stride = (u64)(gridDim.x / kXcds) * blockDim.x;
  const uint32_t last = xs.o[8] - 1;  // last entry of the level's list (the host launches only non-empty lists)
  auto issue = [&](u64 iu, OctLoads<MAXH>& X) {
    const bool on = iu < end;
    const uint32_t g0 = min(__builtin_amdgcn_readfirstlane((uint32_t)((iu - lane) >> 5)), last);
    const uint32_t g1 = min(g0 + 1, last);
    const uint32_t e0 = glist[g0], e1 = glist[g1];
    const u64 pg = ((u64)(lane < 32 ? e0 : e1) << 8) + 8 * (lane & 31);
    oct_issue<MAXH>(d, Q, pg, pg, on, X);
  };
#if GM_R8P_PIPE
  if (first < end) {
    OctLoads<MAXH> X0, X1;
    issue(first, X0);
    for (u64 iu = first; iu < end; iu += 2 * stride) {
      issue(iu + stride, X1);
      oct_finish<MAXH>(Q, X0);
      if (iu + stride >= end) break;
      issue(iu + 2 * stride, X0);
      oct_finish<MAXH>(Q, X1);
    }
  }
#else
  for (u64 iu = first; iu < end; iu += stride) {
    OctLoads<MAXH> X;
    issue(iu, X);
    oct_finish<MAXH>(Q, X);
  }
#endif
  block_count(bc, (u64)Q.npos, (u64)Q.edges);
  if (Q.S == 0) block_add(&st->prims, (u64)Q.npos);  // one launch per solve
}

// Column jobs (shards, and any table whose top digit sits above 256-prefix
// groups): within a top-digit slice, group k (a "column") holds digit sums
// gsc[k] + t + [0, mj] at top value t, so the live columns of slice t at
// level L are those with gsc in [S - t - heap0 - mj, S - t] -- ONE range of
// the columns sorted by gsc (colperm, built once).  A launch lists its
// slices with their colperm ranges; wave w of the concatenation finds its
// slice by a scalar binary search over the prefix counts (kernel
// arguments).  No per-level tables, no hole groups.
template <int MAXH>
__global__ __launch_bounds__(256) void k_dense_resolve4c(Desc d, RowGeom g, uint32_t* words, const u64* bits, u64 L,
                                                         DevState* st, const uint32_t* __restrict__ colperm,
                                                         ColJobs J) {
  Quad4 Q;
  quad_init(Q, d, words, bits, L, g.Wl, g.Wbl);
  uint32_t hl[MAXH], sl;
  lane_digits4<MAXH>(d, hl, sl);
  const XcdRange r = xcd_range((u64)J.cum[J.n] * 64);
  // software-pipelined like k_dense_resolve4p
  auto issue = [&](u64 iu, QuadLoads<MAXH>& X) {
    const bool on = iu < r.end;
    const uint32_t w = __builtin_amdgcn_readfirstlane((uint32_t)((on ? iu : r.first) >> 6));
    uint32_t a = 0, b = J.n;  // slice i: cum[i] <= w < cum[i + 1]
    while (b - a > 1) {
      const uint32_t m = (a + b) >> 1;
      if (J.cum[m] <= w) a = m;
      else b = m;
    }
    const u64 k = colperm[J.lo[a] + (w - J.cum[a])];
    const u64 qw = (u64)J.u[a] * g.Z + k * 256, pw = (u64)J.t[a] * g.Z + k * 256;
    quad_issue<MAXH>(d, Q, hl, sl, qw + 4 * (iu & 63), pw, on, X);
  };
  if (r.first < r.end) {
    QuadLoads<MAXH> X0, X1;
    issue(r.first, X0);
    for (u64 iu = r.first; iu < r.end; iu += 2 * r.stride) {
      issue(iu + r.stride, X1);
      quad_finish<MAXH>(Q, X0);
      if (iu + r.stride >= r.end) break;
      issue(iu + 2 * r.stride, X0);
      quad_finish<MAXH>(Q, X1);
    }
  }
  quad_done(Q, st);
}

template <int MAXH>
__global__ __launch_bounds__(256) void k_dense_resolve8p(Desc d, DenseView v, uint16_t* words, const u64* bits, u64 L,
                                                         DevState* st, const uint32_t* __restrict__ glist,
                                                         XcdShares xs, BlockCount* bc) {
  resolve8p_body<MAXH>(d, v, words, bits, L, st, glist, xs, bc);
}
// (held to 128 VGPRs for 4 waves per SIMD it spills 88 B per lane and runs
// 1.5x slower: profiles/r01_ab_occupancy.jsonl)

// ---------------------------------------------------------------------------
// 8-bit tables (k_dense_resolve16p): SIXTEEN consecutive prefixes per lane,
// one 16-B load per child row, a wave four 256-prefix groups of the level's
// live-group list.  Half the bytes of the 16-bit octet form per position.
// In a game of WIN / LOSS positions only (every K_SUM table) the parity of
// the remoteness carries the value -- a LOSS has even remoteness (0 at a
// primitive, 1 + an odd WIN remoteness), a WIN odd (1 + an even one) -- so
// a byte holds remoteness up to 255 as an order form:
//   WIN  r (odd)  -> y = (r - 1) / 2             (0x00 .. 0x7F)
//   LOSS r (even) -> y = 0x80 | (0x7F - r / 2)   (0x80 .. 0xFF)
// The unsigned max over a parent's children picks the LOSS child of least
// remoteness if there is one, else the WIN child of greatest (0 = WIN 1 is
// the least element, so an absent child read as 0 never wins the max).
// Plan-time condition: every remoteness < 255 (root_sum <= 253).
// ---------------------------------------------------------------------------
typedef uint8_t u8x16 __attribute__((ext_vector_type(16)));
constexpr uint32_t W8_UNREACHED = 0xFFu;
constexpr uint32_t DENSE_PRIMITIVE8 = 0xFFu;  // LOSS, remoteness 0
__device__ __forceinline__ uint32_t dense_parent8(uint32_t m) {
  return (m & 0x80u) ? 0x7Fu - (m & 0x7Fu) : 0x80u | (0x7Fu - (m + 1u));
}
struct WordRow16 {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ void init(const uint8_t* base, u64 nwords) {
    r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)(uint32_t)nwords, 0x00020000);
  }
  // words [idx, idx + 16), idx 16-aligned; !ok reads zeros with no memory access
  __device__ __forceinline__ u8x16 at(uint32_t idx, bool ok) const {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, ok ? idx : 0xFFFFFFF0u, 0, 0);
    return __builtin_bit_cast(u8x16, v);
  }
};
struct Hex16 {
  WordRow16 n1, n2;  // levels L+1, L+2 (empty rows past the last level)
  uint8_t* mine;
  const u64* bits;
  u64 Lb;  // L * Wbl
  uint32_t S, H0;
  uint32_t npos = 0, edges = 0;
};
template <int MAXH>
struct HexLoads {
  u8x16 A1, A2, P1, P2, C1[MAXH], C2[MAXH];
  u64 bitsw;
  u64 q;
  uint32_t h1, s, valid, nch_hi;
};
__device__ __forceinline__ void hex_init(Hex16& Q, const Desc& d, uint8_t* words, const u64* bits, u64 L, u64 Wl,
                                         u64 Wbl) {
  Q.S = d.root_sum - (uint32_t)L;
  Q.H0 = d.heap[0];
  Q.mine = words + L * Wl;
  Q.n1.init(words + (L + 1) * Wl, Q.S >= 1 ? Wl : 0);
  Q.n2.init(words + (L + 2) * Wl, Q.S >= 2 ? Wl : 0);
  Q.bits = bits;
  Q.Lb = L * Wbl;
}
// q: the unit's first prefix in the row (8-bit tables have rows below 2^31
// words, dense_plan_bits, so prefixes and buffer offsets are 32-bit)
template <int MAXH>
__device__ __forceinline__ void hex_issue(const Desc& d, const Hex16& Q, uint32_t q, bool on, HexLoads<MAXH>& X) {
  const uint32_t S = Q.S;
  uint32_t h[MAXH];
  uint32_t s = 0;
#pragma unroll
  for (int i = 1; i < MAXH; i++) {
    h[i] = ((MAXH <= 8) || i < d.nheaps) ? (q >> d.pshift[i]) & ((uint32_t)d.base[i] - 1u) : 0u;
    s += h[i];
  }
  // valid e: s + e <= S and S - (s + e) <= H0, i.e. e in [S - s - H0, S - s]
  const int hi = min((int)S - (int)s, 15), lo = max((int)S - (int)s - (int)Q.H0, 0);
  const uint32_t valid = (on && hi >= lo) ? ((2u << hi) - 1u) & ~((1u << lo) - 1u) : 0u;
  X.q = q;
  X.h1 = h[1];
  X.s = s;
  X.valid = valid;
  uint32_t nch_hi = 0;
#pragma unroll
  for (int i = 2; i < MAXH; i++) nch_hi += ((MAXH <= 8) || i < d.nheaps) ? min(h[i], 2u) : 0u;
  X.nch_hi = nch_hi;
  const bool any = valid != 0;
  X.bitsw = any ? Q.bits[(Q.Lb + q) >> 6] : 0ull;
  X.A1 = Q.n1.at(q, any);
  X.A2 = Q.n2.at(q, any);
  X.P1 = Q.n1.at(q - 16, any && h[1] >= 16);
  X.P2 = Q.n2.at(q - 16, any && h[1] >= 16);
#pragma unroll
  for (int i = 2; i < MAXH; i++) {
    const bool live = (MAXH <= 8) || i < d.nheaps;
    const uint32_t ps = (uint32_t)d.pstride[i];
    X.C1[i] = Q.n1.at(q - ps, any && live && h[i] >= 1);
    X.C2[i] = Q.n2.at(q - 2 * ps, any && live && h[i] >= 2);
  }
}
// Byte arithmetic on the packed 16-B vectors (SWAR), so a lane keeps 4 VGPRs
// per vector and a byte max costs half a packed instruction: the even bytes
// (v & 0x00FF00FF: the LOW byte of each 16-bit lane) and the odd bytes (the
// HIGH byte, left in place) are reduced with v_pk_max_u16 -- a 16-bit max of
// x << 8 is the byte max of x, so the odd half needs no shift, and since the
// high byte of a 16-bit max does not depend on the low bytes, its operands
// need no mask either (one AND at the end) -- and the parent words are formed
// in place and OR-ed for the store.
// The byte masks reach the ANDs through an empty asm: with a visible
// constant the compiler rewrites (v & 0x00FF00FF) feeding 16-bit maxes as
// per-16-bit-lane ops (v_and + v_and_sdwa + v_perm: three VALU per dword
// instead of one v_and_b32 with an SGPR operand)
__device__ __forceinline__ uint32_t opaque_u32(uint32_t x) {
  asm("" : "+s"(x));
  return x;
}
__device__ __forceinline__ u32x4 splat4(uint32_t m) { return u32x4{m, m, m, m}; }

__device__ __forceinline__ u32x4 hmax(u32x4 a, u32x4 b) {
  typedef uint16_t h16x8 __attribute__((ext_vector_type(8)));
  return __builtin_bit_cast(u32x4, __builtin_elementwise_max(__builtin_bit_cast(h16x8, a), __builtin_bit_cast(h16x8, b)));
}
// 16-bit lanes shifted up one lane, lane 0 from the top lane of prev
// (SH = 16); with SH = 24 the HIGH bytes of v (an odd half) arrive as the
// LOW bytes of the next lane: byte 2k+1 -> byte 2k+2 (high bytes of the
// result are v's even bytes, zero in an odd half)
template <int SH>
__device__ __forceinline__ u32x4 hshift(u32x4 v, u32x4 prev) {
  u32x4 r;
  r[0] = __builtin_amdgcn_alignbit(v[0], prev[3], SH);
#pragma unroll
  for (int k = 1; k < 4; k++) r[k] = __builtin_amdgcn_alignbit(v[k], v[k - 1], SH);
  return r;
}
// 16-bit lanes [0, n) all ones (n clamped to [0, 8]): two 64-bit halves of
// (1 << 16 n) - 1 (compares and selects per dword cost 4x the VALU)
__device__ __forceinline__ u32x4 hprefix(int n) {
  const uint32_t c = (uint32_t)min(max(n, 0), 8);
  const u64 lo = c >= 4 ? ~0ull : (1ull << (16 * c)) - 1;
  const u64 hi = c <= 4 ? 0ull : c >= 8 ? ~0ull : (1ull << (16 * (c - 4))) - 1;
  return u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
}
// dense_parent8 in each 16-bit lane, on the byte at bit B of the lane (B = 0:
// low byte, B = 8: high byte); never 0x7F: remoteness < 255.  No borrow
// crosses a lane: 0xFE - m >= 0 for the WIN-only (m <= 0x7F) lanes.
template <int B>
__device__ __forceinline__ uint32_t parent8x2(uint32_t m) {
  constexpr uint32_t top = 0x00800080u << B, low7 = 0x007F007Fu << B, fe = 0x00FE00FEu << B;
  const uint32_t L = ((m & top) >> (7 + B)) * (0xFFu << B);  // lanes with a LOSS child
  return ((~m & low7) & L) | ((fe - (m & ~L)) & ~L);
}
__device__ __forceinline__ uint32_t bits4_to_bytes(uint32_t b4) {  // 4 bits -> 4 byte masks
  return ((b4 * 0x00204081u) & 0x01010101u) * 0xFFu;
}
// the unit's parent words into o (false: no valid slot, nothing to store)
template <int MAXH>
__device__ __forceinline__ bool hex_reduce(Hex16& Q, const HexLoads<MAXH>& X, u32x4& o) {
  const uint32_t valid = X.valid;
  if (!valid) return false;
  const uint32_t S = Q.S;
  const uint32_t rbits = (uint32_t)(X.bitsw >> ((Q.Lb + X.q) & 63)) & 0xFFFFu;
  const u32x4 EM = splat4(opaque_u32(0x00FF00FFu)), OM = splat4(opaque_u32(0xFF00FF00u));
  const u32x4 a1 = __builtin_bit_cast(u32x4, X.A1), a2 = __builtin_bit_cast(u32x4, X.A2);
  const u32x4 a1e = a1 & EM, a1o = a1 & OM, a2e = a2 & EM;
  const u32x4 p1 = __builtin_bit_cast(u32x4, X.P1), p2 = __builtin_bit_cast(u32x4, X.P2);
  // Odd outputs (high bytes) accumulate RAW 16-bit maxes: the high byte of
  // a 16-bit max is the max of the high bytes whatever the low bytes hold,
  // so their operands need no mask and the sum is masked once at the end.
  // Even outputs (low bytes) need every operand's high byte cleared.
  // heap 1: byte e -1 / -2 (P = 0 when the unit starts the digit: no child
  // there).  Even outputs: -1 = the odd byte below (hshift<24> of the odd
  // half), -2 = the even byte below; odd outputs: -1 = the even byte of the
  // same lane moved up, -2 = the odd byte below (hshift<16>, raw).
  u32x4 me = hshift<24>(a1o, p1 & OM), mo = a1e << 8;
  me = hmax(me, hshift<16>(a2e, p2 & EM));
  mo = hmax(mo, hshift<16>(a2, p2));
  // heaps >= 2: never holes under a valid parent
#pragma unroll
  for (int i = 2; i < MAXH; i++) {
    const u32x4 c1 = __builtin_bit_cast(u32x4, X.C1[i]), c2 = __builtin_bit_cast(u32x4, X.C2[i]);
    me = hmax(me, hmax(c1 & EM, c2 & EM));
    mo = hmax(mo, hmax(c1, c2));
  }
  // heap 0 -1 / -2 where h0 = S - s - e >= 1 / >= 2, i.e. e <= t1 / e <= t1 - 1
  const int t1 = (int)S - (int)X.s - 1;
  me = hmax(me, hmax(a1e & hprefix((t1 + 2) >> 1), a2e & hprefix((t1 + 1) >> 1)));
  mo = hmax(mo, hmax(a1 & hprefix((t1 + 1) >> 1), a2 & hprefix(t1 >> 1))) & OM;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t w = S == 0 ? 0xFFFFFFFFu : parent8x2<0>(me[k]) | parent8x2<8>(mo[k]);  // DENSE_PRIMITIVE8
    o[k] = w | ~bits4_to_bytes((rbits >> (4 * k)) & 0xFu);  // unreached -> W8_UNREACHED
  }
  const uint32_t V = rbits & valid;
  if (V) {
    const uint32_t n = (uint32_t)__popc(V);
    auto pre = [](int t) -> uint32_t { return t < 0 ? 0u : t >= 15 ? 0xFFFFu : (2u << t) - 1u; };
    Q.npos += n;
    // min(h0, 2) + min(h1, 2) + heaps >= 2 per reached valid position
    // (h1 = the unit's first heap-1 digit: 0, or a multiple of 16)
    Q.edges += n * X.nch_hi + (uint32_t)__popc(V & pre(t1)) + (uint32_t)__popc(V & pre(t1 - 1)) +
               (X.h1 >= 2 ? 2 * n : (uint32_t)__popc(V & 0xFFFEu) + (uint32_t)__popc(V & 0xFFFCu));
  }
  return true;
}
template <int MAXH>
__device__ __forceinline__ void hex_finish(Hex16& Q, const HexLoads<MAXH>& X) {
  u32x4 o;
  if (hex_reduce<MAXH>(Q, X, o)) *(u32x4*)(Q.mine + X.q) = o;
}
// Live-group list sweep; the host starts every XCD share at an entry
// divisible by 4, so a wave's 64 units are four whole groups (lanes 16k ..
// 16k+15), read with four scalar loads.  Not software-pipelined: one unit in
// flight per lane keeps 91 VGPRs (5 waves per SIMD) and measured 3.90 ms per
// 2^30 backward pass against 4.25 ms for the two-stage pipeline at 166 VGPRs
// (3 waves per SIMD).
// six resident 256-thread blocks per CU (6 waves per SIMD: the compiler keeps
// the kernel at <= 80 VGPRs, no spills): backward 3.17 -> 3.06 ms against the
// unconstrained 84 VGPRs / 5 waves; prefetching the next unit's list entries
// measured no gain (tools/ab_dense.sh)
#ifndef GM_R16_MINB
#define GM_R16_MINB 6
#endif
#ifndef GM_R16_DEFER
#define GM_R16_DEFER 0
#endif
template <int MAXH>
__global__ __launch_bounds__(256, GM_R16_MINB) void k_dense_resolve16p(Desc d, DenseView v, uint8_t* words,
                                                                       const u64* bits, u64 L, DevState* st,
                                                                       const uint32_t* __restrict__ glist,
                                                                       XcdShares xs, BlockCount* bc) {
  Hex16 Q;
  hex_init(Q, d, words, bits, L, v.Wl, v.Wbl);
  const uint32_t lane = __lane_id();
  const uint32_t x = blockIdx.x % kXcds;
  // units (16 prefixes each) of this XCD's share; a level has < 2^28 of them
  const uint32_t first = xs.o[x] * 16 + (blockIdx.x / kXcds) * blockDim.x + threadIdx.x;
  const uint32_t end = xs.o[x + 1] * 16, stride = (gridDim.x / kXcds) * blockDim.x;
  const uint32_t last = xs.o[8] - 1;  // last entry of the level's list (the host launches only non-empty lists)
  // the wave's four list entries (scalar loads), lane's group = entry lane >> 4
  auto fetch = [&](uint32_t iu) -> uint32_t {
    const uint32_t g0 = min(__builtin_amdgcn_readfirstlane((iu - lane) >> 4), last);
    const uint32_t e0 = glist[g0], e1 = glist[min(g0 + 1, last)], e2 = glist[min(g0 + 2, last)],
                   e3 = glist[min(g0 + 3, last)];
    const uint32_t k = lane >> 4;
    return k == 0 ? e0 : k == 1 ? e1 : k == 2 ? e2 : e3;
  };
#if GM_R16_DEFER
  // each unit's store is issued after the NEXT unit's loads: gfx9 counts
  // loads and stores in one in-order vmcnt, so a store issued before the
  // loads would make their wait cover its write acknowledgement too
  u32x4 po;
  uint32_t pq = 0;
  bool pend = false;
  for (uint32_t iu = first; iu < end; iu += stride) {
    HexLoads<MAXH> X;
    hex_issue<MAXH>(d, Q, (fetch(iu) << 8) + 16 * (lane & 15), true, X);
    if (pend) *(u32x4*)(Q.mine + pq) = po;
    pend = hex_reduce<MAXH>(Q, X, po);
    pq = (uint32_t)X.q;
  }
  if (pend) *(u32x4*)(Q.mine + pq) = po;
#else
  for (uint32_t iu = first; iu < end; iu += stride) {
    HexLoads<MAXH> X;
    hex_issue<MAXH>(d, Q, (fetch(iu) << 8) + 16 * (lane & 15), true, X);
    hex_finish<MAXH>(Q, X);
  }
#endif

  block_count(bc, (u64)Q.npos, (u64)Q.edges);
  if (Q.S == 0) block_add(&st->prims, (u64)Q.npos);  // one launch per solve
}

// ---------------------------------------------------------------------------
// Tail runs (world 1, live-group lists): the narrow ends of the tier sequence
// hold a few hundred live groups per level, where a launch costs its fixed
// ~4-6 us (dispatch, list entry, parent / child loads, store drain) for well
// under a microsecond of work.  One 1024-thread workgroup walks a run of such
// levels instead, a barrier between levels: its stores reach its own later
// loads through the CU's L1 / its XCD's L2 (workgroup-scope release/acquire
// of __syncthreads), so a level costs about one L2 round trip.  Same per-word
// (pull_issue / pull_finish) and per-unit (hex_issue / hex_finish) bodies as
// the per-level kernels.
// ---------------------------------------------------------------------------
constexpr int kTailMax = 40;       // levels per run
constexpr int kTailThreads = 1024;
// thresholds measured (tools/ab_dense.sh): 1024 / 256 and 2048 / 512 groups
// were slower (+0.05, +0.3 ms): past two passes a workgroup's serial passes
// cost more than the launch they save.  Staging the run's list in LDS saved
// nothing (a tail level costs ~4 us: its data round, store drain, barrier).
#ifndef GM_TAIL_PULL_GROUPS
#define GM_TAIL_PULL_GROUPS 512
#define GM_TAIL_RESOLVE_GROUPS 128
#endif
constexpr uint64_t kTailPullGroups = GM_TAIL_PULL_GROUPS;        // two passes of 1024 bitmap words
constexpr uint64_t kTailResolveGroups = GM_TAIL_RESOLVE_GROUPS;  // two passes of 1024 sixteen-prefix units
struct TailRun {
  uint32_t n;                      // levels in the run
  uint32_t L[kTailMax];            // the levels, in solve order
  uint32_t off[kTailMax];          // first list entry of the level (relative to glist)
  uint32_t cnt[kTailMax];          // live groups of the level
  u64 phi[kTailMax];               // band end of the level (dense_band p_hi)
};
template <int MAXH>
__global__ __launch_bounds__(kTailThreads) void k_dense_pull_tail(Desc d, DenseView v, u64* bits, u64 root_p,
                                                                  const u64* __restrict__ masks,
                                                                  const uint32_t* __restrict__ glist, TailRun R) {
  __shared__ u64 M[64 * (MAXH + 1)];
  for (int k = threadIdx.x; k < 64 * (MAXH + 1); k += blockDim.x) M[k] = masks[k];
  __syncthreads();
  for (uint32_t i = 0; i < R.n; i++) {
    const u64 L = R.L[i];
    const uint32_t nw = R.cnt[i] * 4;  // one thread per 64-prefix bitmap word
    for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x) {
      const u64 qi = ((u64)glist[R.off[i] + (w >> 2)] << 8) + ((w & 3) << 6);
      uint64_t q;
      bool run;
      const u64 pg = dense_sweep(v, qi, &q, &run);
      if (!run) continue;
      const u64 V0 = qi + 64 > R.phi[i] ? (qi >= R.phi[i] ? 0ull : (1ull << (R.phi[i] - qi)) - 1) : ~0ull;
      PullLd<MAXH> X;
      pull_issue<MAXH>(d, v.Wbl, bits, L, q, X);
      pull_finish<MAXH>(d, v.Wbl, bits, L, root_p, q, pg, V0, M, M, X);
    }
    __syncthreads();  // level L's words visible to level L + 1's parents
  }
}
template <int MAXH>
__global__ __launch_bounds__(kTailThreads) void k_dense_resolve16_tail(Desc d, DenseView v, uint8_t* words,
                                                                       const u64* bits, DevState* st,
                                                                       const uint32_t* __restrict__ glist, TailRun R,
                                                                       BlockCount* bc) {
  u64 npos = 0, edges = 0, prims = 0;
  for (uint32_t i = 0; i < R.n; i++) {
    const u64 L = R.L[i];
    Hex16 Q;
    hex_init(Q, d, words, bits, L, v.Wl, v.Wbl);
    const uint32_t nu = R.cnt[i] * 16;  // sixteen prefixes per unit
    for (uint32_t u = threadIdx.x; u < nu; u += blockDim.x) {
      HexLoads<MAXH> X;
      hex_issue<MAXH>(d, Q, (glist[R.off[i] + (u >> 4)] << 8) + 16 * (u & 15), true, X);
      hex_finish<MAXH>(Q, X);
    }
    npos += Q.npos;
    edges += Q.edges;
    if (Q.S == 0) prims += Q.npos;
    __syncthreads();  // level L's words visible to levels L - 1 and L - 2
  }
  block_count(bc, npos, edges);
  block_add(&st->prims, prims);
}

// Column jobs over a 16-bit table (shards): the octet body of
// k_dense_resolve8p, a wave = two consecutive columns of the jobs'
// concatenation (lanes 0-31 / 32-63; each half finds its slice by a scalar
// search), software-pipelined.
#ifndef GM_R8C_MINB
#define GM_R8C_MINB 1
#endif
// One unit in flight per lane (86 VGPRs, 5 waves per SIMD) against the
// two-stage software pipeline (GM_R8C_PIPE 1: 138 VGPRs, 3 waves): the
// 2-shard group solve's backward 22.4 -> 20.1 ms (tools/ab_group.sh), the
// same trade the 8-bit list kernel made
#ifndef GM_R8C_PIPE
#define GM_R8C_PIPE 0
#endif
template <int MAXH>
__global__ __launch_bounds__(256, GM_R8C_MINB) void k_dense_resolve8c(Desc d, RowGeom g, uint16_t* words, const u64* bits, u64 L,
                                                         DevState* st, const uint32_t* __restrict__ colperm,
                                                         ColJobs J, BlockCount* bc) {
  Oct8 Q;
  oct_init(Q, d, words, bits, L, g.Wl, g.Wbl);
  const uint32_t lane = __lane_id();
  const uint32_t total = J.cum[J.n];  // columns (host: > 0)
  const XcdRange r = xcd_range((u64)((total + 1) / 2) * 64);
  auto find = [&](uint32_t w, u64* q, u64* pg) {  // column w of the concatenation (scalar)
    uint32_t a = 0, b = J.n;  // slice i: cum[i] <= w < cum[i + 1]
    while (b - a > 1) {
      const uint32_t m = (a + b) >> 1;
      if (J.cum[m] <= w) a = m;
      else b = m;
    }
    const u64 k = colperm[J.lo[a] + (w - J.cum[a])];
    *q = (u64)J.u[a] * g.Z + k * 256;
    *pg = (u64)J.t[a] * g.Z + k * 256;
  };
  auto issue = [&](u64 iu, OctLoads<MAXH>& X) {
    const uint32_t c0 = min(__builtin_amdgcn_readfirstlane((uint32_t)((iu - lane) >> 6)) * 2, total - 1);
    const uint32_t c1 = min(c0 + 1, total - 1);
    const bool on = iu < r.end && (lane < 32 || c0 + 1 < total);
    u64 q0, p0, q1, p1;
    find(c0, &q0, &p0);
    find(c1, &q1, &p1);
    const u64 o = 8 * (lane & 31);
    oct_issue<MAXH>(d, Q, (lane < 32 ? q0 : q1) + o, (lane < 32 ? p0 : p1) + o, on, X);
  };
#if GM_R8C_PIPE
  if (r.first < r.end) {
    OctLoads<MAXH> X0, X1;
    issue(r.first, X0);
    for (u64 iu = r.first; iu < r.end; iu += 2 * r.stride) {
      issue(iu + r.stride, X1);
      oct_finish<MAXH>(Q, X0);
      if (iu + r.stride >= r.end) break;
      issue(iu + 2 * r.stride, X0);
      oct_finish<MAXH>(Q, X1);
    }
  }
#else
  for (u64 iu = r.first; iu < r.end; iu += r.stride) {
    OctLoads<MAXH> X;
    issue(iu, X);
    oct_finish<MAXH>(Q, X);
  }
#endif
  block_count(bc, (u64)Q.npos, (u64)Q.edges);
  if (Q.S == 0) block_add(&st->prims, (u64)Q.npos);  // one launch per solve
}

// Packed word halos (shards, gm_solver.hip exchange_words): the non-hole
// words of a halo slice at level L move between the table and a dense
// buffer in COLUMN order -- live columns in colperm order (digit sum gs
// ascending), slots ascending inside a column.  With x = S - t and y = x -
// gs, column position i of slice x starts at
//   PB[x][gs] + (i - CS[gs]) * NY[y]
// (PB[x][g] = non-holes of all columns with smaller sum, NY[y] = non-holes
// of a column at y, CS = colperm's sum starts; host tables built once), and
// a slot's rank inside its column comes from four ballots.  Both ends
// derive the same order from (L, t) alone.  W16: words travel as 16 bits
// (order form: top bit + 15 low bits; exact while every remoteness is below
// 2^15, which K_SUM's remoteness <= root_sum guarantees when root_sum is).
constexpr int kMaxHaloColJobs = 64;
struct HaloColJobs {
  uint32_t n;
  uint32_t cum[kMaxHaloColJobs + 1];  // columns before job i
  uint32_t lo[kMaxHaloColJobs];       // first colperm entry
  uint32_t u[kMaxHaloColJobs];        // local slice
  int32_t x[kMaxHaloColJobs];         // S - t
  uint32_t base[kMaxHaloColJobs];     // buffer offset of the slice's first word
};
struct HaloTabs {
  const uint32_t* PB;  // [XN][NG]
  const uint32_t* NY;  // [NYn]
  const uint32_t* CS;  // [NG]
  int NG, NYn, top;
};
__device__ __forceinline__ uint32_t halo16(uint32_t y) { return ((y >> 16) & 0x8000u) | (y & 0x7FFFu); }
__device__ __forceinline__ uint32_t unhalo16(uint32_t h) { return (h & 0x8000u) ? (0xFFFF8000u | h) : h; }

// T16: the table itself holds 16-bit order forms (k_dense_resolve8c; implies
// W16), which are already the halo's 16-bit form.
template <bool PACK, bool W16, bool T16 = false>
__global__ __launch_bounds__(256) void k_halo_cols(Desc d, HaloColJobs J, u64 Z, const uint32_t* __restrict__ colperm,
                                                   HaloTabs T, void* level_words_v, void* buf) {
  static_assert(!T16 || W16, "a 16-bit table travels as 16-bit words");
  uint32_t* level_words = (uint32_t*)level_words_v;
  uint16_t* level_words16 = (uint16_t*)level_words_v;
  typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
  const uint32_t lane = __lane_id();
  uint32_t sl = 0;  // digit sum of the lane's first slot offset 4 * lane (below the top digit)
  for (int i = 1; i < T.top; i++) sl += ((4u * lane) >> d.pshift[i]) & (d.base[i] - 1);
  const int H0 = (int)d.heap[0];
  const u64 ltmask = (1ull << lane) - 1ull;
  const XcdRange r = xcd_range((u64)J.cum[J.n] * 64);
  for (u64 iu = r.first; iu < r.end; iu += r.stride) {
    const uint32_t w = __builtin_amdgcn_readfirstlane((uint32_t)(iu >> 6));
    uint32_t a = 0, b = J.n;
    while (b - a > 1) {
      const uint32_t m = (a + b) >> 1;
      if (J.cum[m] <= w) a = m;
      else b = m;
    }
    const uint32_t i = J.lo[a] + (w - J.cum[a]);
    const uint32_t k = colperm[i];
    int gs = 0;
    for (int h = 1; h < T.top; h++) gs += (int)(((u64)k * 256 >> d.pshift[h]) & (d.base[h] - 1));
    const int x = J.x[a], y = x - gs;
    const uint32_t ny = (y >= 0 && y < T.NYn) ? T.NY[y] : 0u;
    const u64 base = (u64)J.base[a] + T.PB[(u64)x * T.NG + gs] + (u64)(i - T.CS[gs]) * ny;
    // element e of the lane: slot 4 lane + e, digit sum sl + e
    uint32_t valid = 0;
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const int ds = (int)sl + e;
      valid |= (uint32_t)(ds <= y && ds >= y - H0) << e;
    }
    u64 bl[4];
#pragma unroll
    for (int e = 0; e < 4; e++) bl[e] = __ballot((valid >> e) & 1u);
    uint32_t before = 0;  // valid slots in lower lanes
#pragma unroll
    for (int e = 0; e < 4; e++) before += (uint32_t)__popcll(bl[e] & ltmask);
    const u64 q = (u64)J.u[a] * Z + (u64)k * 256 + 4 * lane;
    if (T16) {
      if (!valid) continue;
      uint32_t rk = before;
      if (PACK) {
        const u16x4 v4 = *(const u16x4*)(level_words16 + q);
#pragma unroll
        for (int e = 0; e < 4; e++) {
          if (!((valid >> e) & 1u)) continue;
          ((uint16_t*)buf)[base + rk] = v4[e];
          rk++;
        }
      } else {
        u16x4 v4 = {0, 0, 0, 0};
#pragma unroll
        for (int e = 0; e < 4; e++) {
          if (!((valid >> e) & 1u)) continue;
          v4[e] = ((const uint16_t*)buf)[base + rk];
          rk++;
        }
        *(u16x4*)(level_words16 + q) = v4;  // holes of a live lane get 0 (never read unmasked)
      }
      continue;
    }
    if (PACK) {
      if (!valid) continue;
      const u32x4 v4 = *(const u32x4*)(level_words + q);
      uint32_t rk = before;
#pragma unroll
      for (int e = 0; e < 4; e++) {
        if (!((valid >> e) & 1u)) continue;
        if (W16) ((uint16_t*)buf)[base + rk] = (uint16_t)halo16(v4[e]);
        else ((uint32_t*)buf)[base + rk] = v4[e];
        rk++;
      }
    } else {
      if (!valid) continue;
      u32x4 v4 = {0u, 0u, 0u, 0u};
      uint32_t rk = before;
#pragma unroll
      for (int e = 0; e < 4; e++) {
        if (!((valid >> e) & 1u)) continue;
        v4[e] = W16 ? unhalo16(((const uint16_t*)buf)[base + rk]) : ((const uint32_t*)buf)[base + rk];
        rk++;
      }
      *(u32x4*)(level_words + q) = v4;  // holes of a live lane get 0 (never read unmasked)
    }
  }
}

// 16-bit tables (k_dense_resolve8c shards): the same column-order packing,
// two columns per wave (lanes 0-31 / 32-63) and eight slots per lane (one
// 16-B access), so a level's halo is one pass of the grid instead of two.
// Each half finds its column with scalar searches; a slot's rank is the
// valid slots of lower lanes in its half (eight ballots) plus the lower
// valid elements of its own lane.  Needs base[1] >= 8 (w16 tables do).
template <bool PACK>
__global__ __launch_bounds__(256) void k_halo_cols16(Desc d, HaloColJobs J, u64 Z, const uint32_t* __restrict__ colperm,
                                                     HaloTabs T, uint16_t* level_words, uint16_t* buf) {
  const uint32_t lane = __lane_id(), hl = lane & 31;
  uint32_t sl = 0;  // digit sum of the lane's first slot offset 8 hl (below the top digit)
  for (int i = 1; i < T.top; i++) sl += ((8u * hl) >> d.pshift[i]) & (d.base[i] - 1);
  const int H0 = (int)d.heap[0];
  const u64 below = ((1ull << lane) - 1ull) & (lane < 32 ? 0x00000000FFFFFFFFull : 0xFFFFFFFF00000000ull);
  const uint32_t total = J.cum[J.n];  // columns (host: > 0)
  const XcdRange r = xcd_range((u64)((total + 1) / 2) * 64);
  struct Col {
    u64 q, base;
    int y;
  };
  auto find = [&](uint32_t c) {  // column c of the concatenation (scalar)
    uint32_t a = 0, b = J.n;
    while (b - a > 1) {
      const uint32_t m = (a + b) >> 1;
      if (J.cum[m] <= c) a = m;
      else b = m;
    }
    const uint32_t i = J.lo[a] + (c - J.cum[a]);
    const uint32_t k = colperm[i];
    int gs = 0;
    for (int h = 1; h < T.top; h++) gs += (int)(((u64)k * 256 >> d.pshift[h]) & (d.base[h] - 1));
    const int x = J.x[a], y = x - gs;
    const uint32_t ny = (y >= 0 && y < T.NYn) ? T.NY[y] : 0u;
    Col col;
    col.base = (u64)J.base[a] + T.PB[(u64)x * T.NG + gs] + (u64)(i - T.CS[gs]) * ny;
    col.q = (u64)J.u[a] * Z + (u64)k * 256;
    col.y = y;
    return col;
  };
  for (u64 iu = r.first; iu < r.end; iu += r.stride) {
    const uint32_t c0 = __builtin_amdgcn_readfirstlane((uint32_t)(iu >> 6)) * 2;
    const Col A = find(c0), B = find(min(c0 + 1, total - 1));
    const bool on = lane < 32 || c0 + 1 < total;
    const int y = lane < 32 ? A.y : B.y;
    const u64 base = lane < 32 ? A.base : B.base;
    const u64 q = (lane < 32 ? A.q : B.q) + 8 * hl;
    uint32_t valid = 0;
#pragma unroll
    for (int e = 0; e < 8; e++) {
      const int ds = (int)sl + e;
      valid |= (uint32_t)(on && ds <= y && ds >= y - H0) << e;
    }
    uint32_t rk = 0;  // valid slots of lower lanes in this half
#pragma unroll
    for (int e = 0; e < 8; e++) rk += (uint32_t)__popcll(__ballot((valid >> e) & 1u) & below);
    if (!valid) continue;
    if (PACK) {
      const u16x8 v = *(const u16x8*)(level_words + q);
#pragma unroll
      for (int e = 0; e < 8; e++)
        if ((valid >> e) & 1u) buf[base + rk++] = v[e];
    } else {
      u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};  // holes of a live lane get 0 (never read unmasked)
#pragma unroll
      for (int e = 0; e < 8; e++)
        if ((valid >> e) & 1u) v[e] = buf[base + rk++];
      *(u16x8*)(level_words + q) = v;
    }
  }
}

// root word (on the shard that owns the root, root_q = its local prefix;
// others pass ~0 and report NO_WORD)
__global__ void k_dense_root(DenseView v, const uint32_t* words, const u64* bits, u64 root_q, DevState* st,
                             uint32_t wbits) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    uint32_t w = NO_WORD;
    if (root_q != ~0ull && reach_bit(bits, root_q))  // level 0
      w = dense_word_at(words, root_q, wbits);
    st->root_word = w;
  }
}

// word of each key this table owns (NO_WORD for unreachable / not owned)
__global__ void k_dense_query(Desc d, DenseView v, const uint32_t* words, const u64* bits, const u64* keys, u64 n,
                              uint32_t* out, uint32_t wbits) {
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
    u64 slot, L, p;
    uint32_t w = NO_WORD;
    if (dense_slot_of(d, keys[i], &slot)) {
      slot_split(d, slot, &L, &p);
      uint64_t q;
      if (dense_local(v, p, &q) && reach_bit(bits, L * v.Wbl + q))
        w = dense_word_at(words, L * v.Wl + q, wbits);
    }
    out[i] = w;
  }
}

// every reachable owned position -> its key (order arbitrary); v sweeps the
// whole local range with the own-slice filter
__global__ void k_dense_positions(Desc d, DenseView v, const u64* bits, u64 levels, u64* out, u64 cap, u64* count) {
  const u64 n = v.Wl;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < levels * n; i += (u64)gridDim.x * blockDim.x) {
    const u64 L = i / n, q = i - L * n;
    bool run;
    const u64 p = dense_global(v, q, &run);
    if (!run) continue;
    int64_t h0 = dense_h0(d, L, p);
    if (h0 < 0 || !reach_bit(bits, L * v.Wbl + q)) continue;
    u64 k = atomicAdd(count, 1ull);
    if (k < cap) out[k] = p * d.base[0] + (u64)h0;
  }
}
