// gm_solver.hip -- tier-synchronous retrograde solver for gfx950 (MI355X)
// behind the C-ABI of include/gamesman.h.
//
// Replaces the reference's asynchronous per-state job machinery
// (src/process.py:37-267, src/job.py) with a level-synchronous pipeline:
//
//   forward, level L = 0..T-1   K1+K2  k_expand<G>: every position of level L
//                                      is tested with primitive(); the
//                                      non-primitive ones generate their
//                                      children (gen_moves+do_move fused),
//                                      which are inserted into the HBM hash
//                                      table by 64-bit CAS; a child inserted
//                                      for the first time is appended
//                                      (wave-aggregated atomics) to the
//                                      position store of level L+1 or L+2.
//   backward, level L = T-1..0  K3     k_resolve<G>: each position of level L
//                                      re-generates its children, probes
//                                      their 32-bit words and reduces them
//                                      with the reference-canonical rule of
//                                      _res_red/_remote_red (SURVEY §8a
//                                      A8/A9), then stores its own word.
//
// HBM layout (caller-allocated, gamesman.h):
//   table  : gm_slot[2^k] {u64 key, u32 word, u32 spare}, open addressing,
//            linear probing, EMPTY key = ~0.  Replaces the resolved/remote
//            CacheDicts (src/cache_dict.py) -- one 16-B line per probe
//            serves both key compare and word.
//   levels : u64 keys of every reachable position grouped by level.  +1
//            children grow a stack from the front, +2 children a stack from
//            the back, so each level is at most two contiguous segments.
//   scratch: DevState (cursors, counters, error bits, per-level segments).
// No host synchronisation inside the level loops: segment bounds travel
// through device memory (k_finalize), so a whole solve is enqueued at once.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "gm_solver.hip is written for gfx950 (MI355X) only: v_bitop3_b32, v_pk_maximum3_f16 on f16 subnormals"
#endif

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>
#include <memory>
#include <type_traits>
#include <map>
#include <mutex>
#include <thread>
#include <atomic>

#include "../../include/gamesman.h"
#include "gm_codec.h"
#include "gm_games.h"
#include "gm_md5.h"
#include "gm_plane.h"

using namespace gm;
typedef unsigned long long u64;

// A/B knobs of the measurement labs (tools/*.sh): environment variables read
// ONLY by a library built with -DGM_LAB=1 (make lab ->
// libgamesman_hip_lab.so).  In the shipped library every knob reads as unset,
// so no environment can select a timing-only variant (some of them write
// wrong words on purpose, e.g. GM_RK_DBG) or change the product's schedule.
#ifndef GM_LAB
#define GM_LAB 0
#endif
static const char* lab_env(const char* name) {
#if GM_LAB
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
static thread_local std::string g_err;
static int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) return fail(GM_EHIP, "%s: %s", #x, hipGetErrorString(e_)); \
  } while (0)

// queued one-table PLANES solves (gm_solver_solve_async): a ring slot holds
// one solve's events (start, forward end, backward end, its completion --
// recorded after the counts' copy -- and the forward's start) and its counts
// in pinned host memory
constexpr int kPlaneRing = 8;
struct PlaneSlot {
  hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};  // (4: the forward's start, no timing)
  u64* host = nullptr;
  double t_enq = 0;  // host clock at enqueue (ms)
  bool lite = false;  // only ev[0] and ev[3] recorded (a queued one-launch solve)
};

// an in-process multi-GPU group aborted (solve_multi's abort_all): no RCCL
// call may use the aborted communicators
#define RCCL_LIVE(S)                                                                              \
  do {                                                                                            \
    if ((S)->gabort && (S)->gabort->load(std::memory_order_acquire))                              \
      return fail(GM_EHIP, "RCCL group aborted: a peer shard failed (shard %d/%d)", (S)->rank, (S)->world); \
  } while (0)

enum : uint32_t {
  ERR_TABLE_FULL = 1u,
  ERR_LEVELS_FULL = 2u,
  ERR_BAD_STEP = 4u,
  ERR_CHILD_MISSING = 8u,
  ERR_CHILD_UNRESOLVED = 16u,
  ERR_NO_MOVES = 32u,
  ERR_SELF_MISSING = 64u,
  // a shard failed on its host side (a deferred error: it kept serving its
  // halo transfers so that its peers finished, then reported through the
  // end-of-solve reduction; gm_plane_run.h plane_backward_staged)
  ERR_SHARD_FAILED = 512u,
  // the one-launch PLANES backward (k_plane_flow) gave up waiting for a
  // neighbour plane: the launch drained, the words are incomplete
  ERR_PLANE_STALL = 1024u,
};

// ---------------------------------------------------------------------------
// game registry
// ---------------------------------------------------------------------------
static std::mutex g_mu;
static std::vector<Desc> g_games;


static int kv(const char* params, const char* key, int dflt) {
  if (!params) return dflt;
  size_t kl = strlen(key);
  for (const char* p = params; (p = strstr(p, key)); p += kl) {
    if ((p == params || p[-1] == ',') && p[kl] == '=') return atoi(p + kl + 1);
  }
  return dflt;
}

static int build_desc(const char* name, const char* params, Desc* out) {
  Desc d;
  memset(&d, 0, sizeof d);
  if (!strcmp(name, "four_to_one") || !strcmp(name, "sum_four_to_one")) {
    d.kind = K_SUM;
    if (name[0] == 'f') {
      d.variant = 1;
      int start = kv(params, "start", 4);  // four_to_one.py:7-8
      if (start < 0) return fail(GM_EINVAL, "four_to_one start must be >= 0");
      d.nheaps = 1;
      d.heap[0] = (uint32_t)start;
    } else {
      const char* p = params ? strstr(params, "heaps=") : nullptr;
      if (!p) return fail(GM_EINVAL, "sum_four_to_one needs heaps=h0:h1:...");
      p += 6;
      while (*p && *p != ',') {
        if (d.nheaps >= 16) return fail(GM_EINVAL, "at most 16 heaps");
        long h = strtol(p, nullptr, 10);
        if (h < 0 || h > (1L << 30)) return fail(GM_EINVAL, "bad heap %ld", h);
        d.heap[d.nheaps++] = (uint32_t)h;
        while (*p && *p != ':' && *p != ',') p++;
        if (*p == ':') p++;
      }
      if (d.nheaps == 0) return fail(GM_EINVAL, "no heaps");
    }
    unsigned __int128 stride = 1;
    d.pow2 = 1;
    d.root = 0;
    d.root_sum = 0;
    for (int i = 0; i < d.nheaps; i++) {
      d.base[i] = d.heap[i] + 1;
      d.stride[i] = (uint64_t)stride;
      if (d.base[i] & (d.base[i] - 1)) d.pow2 = 0;
      int sh = 0;
      while ((1ull << sh) < (uint64_t)stride) sh++;
      d.shift[i] = (uint32_t)sh;
      d.root += (uint64_t)d.heap[i] * d.stride[i];
      d.root_sum += d.heap[i];
      stride *= d.base[i];
      if (stride > ((unsigned __int128)1 << 62)) return fail(GM_EINVAL, "state space exceeds 2^62");
    }
    if (d.root_sum >= (1u << 30) - 2) return fail(GM_EINVAL, "remoteness would exceed 30 bits");
    d.max_levels = (int)d.root_sum + 1;
    // dense layout (see gm_dense.h)
    d.W = 1;
    for (int i = 1; i < d.nheaps; i++) {
      d.pstride[i] = d.W;
      int sh = 0;
      while ((1ull << sh) < d.W) sh++;
      d.pshift[i] = (uint32_t)sh;
      d.W *= d.base[i];
    }
    d.wshift = -1;
    if ((d.W & (d.W - 1)) == 0) {
      int sh = 0;
      while ((1ull << sh) < d.W) sh++;
      d.wshift = sh;
    }
    d.dense_ok = 1;
  } else if (!strcmp(name, "tic_tac_toe_np") || !strcmp(name, "mttt")) {
    d.kind = K_TTT;
    d.variant = name[0] == 'm';
    d.root = 0;
    d.max_levels = 10;
  } else if (!strcmp(name, "toot_and_otto_bitstring")) {
    d.kind = K_TOOT;
    d.L = kv(params, "length", 6);  // toot_and_otto_bitstring.py:8
    d.H = kv(params, "height", 4);
    d.A = d.L * d.H;
    if (d.L < 1 || d.H < 1 || 2 * d.A + 13 > 64)
      return fail(GM_EINVAL, "toot board %dx%d does not fit a 64-bit key (area <= 25)", d.L, d.H);
    d.nbits = (2 * d.A + 17 + 7) / 8 * 8;
    d.full = (1ull << d.A) - 1;
    for (int y = 0; y < d.H; y++) d.col0 |= 1ull << (d.L * y);
    // word starts per direction: (1,0) (0,1) (1,1) (1,-1); steps in cell index
    const int dxs[4] = {1, 0, 1, 1}, dys[4] = {0, 1, 1, -1};
    for (int i = 0; i < 4; i++) {
      uint64_t m = 0;
      for (int x = 0; x < d.L; x++)
        for (int y = 0; y < d.H; y++) {
          int ex = x + 3 * dxs[i], ey = y + 3 * dys[i];
          if (ex >= 0 && ex < d.L && ey >= 0 && ey < d.H) m |= 1ull << (d.L * y + x);
        }
      d.tmask[i] = m;
      d.tstep[i] = dxs[i] + d.L * dys[i];
    }
    // initial_position (:36-44): hands 6,6,6,6; turn bit 0 (player 2 first)
    d.root = 0;
    for (int j = 0; j < 4; j++) d.root |= 6ull << (2 * d.A + 3 * j);
    d.max_levels = d.A + 1;
  } else if (!strcmp(name, "othello_bit_new")) {
    d.kind = K_OTHELLO;
    d.L = kv(params, "length", 8);  // othello_bit_new.py:8
    d.H = kv(params, "height", 8);
    d.A = d.L * d.H;
    if (d.L != d.H)
      return fail(GM_EINVAL, "othello descriptor supports square boards only (reference flip bounds "
                             "are transposed for non-square boards, othello_bit_new.py:101,110)");
    if (d.L < 2 || 2 * d.A + 3 > 64)
      return fail(GM_EINVAL, "othello board %dx%d does not fit a 64-bit key (area <= 30)", d.L, d.H);
    d.nbits = (2 * d.A + 16 + 7) / 8 * 8;
    d.full = (1ull << d.A) - 1;
    // initial_position (:37-48) with the module's float coordinates
    // (length / 2 - 1): board index int(length*y + x)
    auto put = [&](double x, double y, int white) {
      int idx = (int)(d.L * y + x);
      d.root |= 1ull << (white ? idx : d.A + idx);
    };
    double hx = d.L / 2.0, hy = d.H / 2.0;
    d.root = 0;
    put(hx - 1, hy - 1, 1);
    put(hx - 1, hy, 0);
    put(hx, hy - 1, 0);
    put(hx, hy, 1);
    // two incr_turn calls from 0 -> turn_count 2 (WHITE): bit 2A = 0
    d.max_levels = d.A + 3;
    d.sym = kv(params, "symmetry", 0) ? 1 : 0;  // player_flip orbits (symmetry_functions, :224-226)
    d.root = oth_canon(d, d.root);
  } else {
    return fail(GM_EINVAL, "no device descriptor for game '%s'", name);
  }
  if (kv(params, "symmetry", 0) && d.kind != K_OTHELLO)
    return fail(GM_EINVAL, "'%s' defines no symmetry_functions() to reduce by", name);
  *out = d;
  return 0;
}

// Shard geometry of a dense table.  world == 1: the whole prefix space.
// world > 1: the values [0, E) of the TOP prefix digit (heap K-1) are cut
// into blocks of B and block k is owned by rank k mod world (round robin:
// every rank's top values spread over the whole range, so the ranks'
// per-level work stays close -- DESIGN.md §Multi-GPU).  Each block keeps
// halo slices [kB-2, kB) (children: one move lowers a heap by 1 or 2) and
// [kB+B, kB+B+2) (parents, for the pull-form forward pass).  B = 8 when
// every rank gets at least two blocks, else ceil(E / world) (one block per
// rank).  The geometry is a function of (descriptor, rank, world) alone, so
// every rank derives the same halo sizes.
struct DenseGeom {
  DenseView v;
  u64 nblocks, nb;
};
static int dense_geom(const Desc* d, int rank, int world, DenseGeom* g) {
  memset(g, 0, sizeof *g);
  if (world <= 1) {
    g->v.p_lo = 0;
    g->v.p_hi = d->W;
    g->v.Wl = d->W;
    g->v.Wbl = (d->W + 63) & ~63ull;
    g->v.world = 1;
    g->v.zshift = -1;
    g->nblocks = g->nb = 1;
    return 0;
  }
  if (d->nheaps < 2) return fail(GM_EINVAL, "sharding needs at least 2 heaps");
  if (rank < 0 || rank >= world) return fail(GM_EINVAL, "bad shard %d/%d", rank, world);
  const int k = d->nheaps - 1;
  const u64 E = d->base[k], Z = d->pstride[k];
  if (Z % 64) return fail(GM_EINVAL, "shard slices must hold a multiple of 64 prefixes (got %llu)", (unsigned long long)Z);
  const u64 B = E >= 16 * (u64)world ? 8 : (E + world - 1) / world;
  const u64 nblocks = B ? (E + B - 1) / B : 0;
  if (B < 2 || nblocks < (u64)world)
    return fail(GM_EINVAL, "top heap of %llu values cannot give %d ranks blocks of >= 2", (unsigned long long)E, world);
  g->nblocks = nblocks;
  g->nb = (nblocks - (u64)rank + world - 1) / world;
  DenseView& v = g->v;
  v.blk = 1;
  v.B = (uint32_t)B;
  v.world = (uint32_t)world;
  v.rank = (uint32_t)rank;
  v.Z = Z;
  v.E = E;
  v.zshift = (Z & (Z - 1)) ? -1 : __builtin_ctzll(Z);
  v.olo = 2;
  v.ohi = (uint32_t)B + 2;
  v.Wl = g->nb * (B + 4) * Z;
  v.Wbl = v.Wl;  // multiple of 64
  if (v.Wl * 4 > 0xFFFFFFF0ull)  // the shard resolve addresses a level with 32-bit buffer offsets
    return fail(GM_EINVAL, "shard of %llu prefixes per level: more than 2^30 (use more ranks)",
                (unsigned long long)v.Wl);
  v.p_lo = 0;
  v.p_hi = v.Wl;
  return 0;
}
static uint32_t dense_plan_bits(const Desc* d, int world, uint32_t flags);
// word area of a dense table: 8- or 16-bit order forms when the plan chose
// them (dense_plan_bits: one-GPU K_SUM tables the 16- / 8-prefix kernels
// handle), else 32-bit
static u64 dense_words_bytes(const Desc* d, const DenseGeom& g, uint32_t wbits) {
  return ((u64)d->max_levels * g.v.Wl * (wbits / 8) + 255) & ~255ull;
}
static u64 dense_bits_bytes(const Desc* d, const DenseGeom& g) {
  return (u64)d->max_levels * g.v.Wbl / 8;
}

struct gm_solver;
struct PlaneShape;
static bool plane_ok(const Desc* d, int world);
static bool plane_wanted(const Desc* d, uint32_t flags, int world);
static int plan_planes(const Desc* d, int rank, int world, uint32_t flags, uint64_t max_table_bytes, gm_plan_t* out,
                       bool* fits);
static int plane_setup(gm_solver* s, const gm_buffers* buf);
static int run_planes(std::vector<gm_solver*> ss, gm_result* out, bool async = false);
static int plane_collect(gm_solver* s, u64 ticket, gm_result* out);
static int plane_query(gm_solver* s, const uint64_t* keys_dev, uint64_t n, uint32_t* words_dev);
static int plane_positions(gm_solver* s, uint64_t* keys_dev, uint64_t cap, uint64_t* n);
static void plane_checksum_launch(gm_solver* s, u64* acc);
static bool rank_wanted(const Desc* d, uint32_t flags);
static bool rank_ok(const Desc* d);
static int plan_ranked(const Desc* d, uint64_t max_table_bytes, gm_plan_t* out, bool* fits);
static int rank_setup(gm_solver* s, const gm_buffers* buf);
static int plan_ranked_shard(const Desc* d, int world, uint64_t max_table_bytes, gm_plan_t* out);
static int run_ranked_shards(std::vector<gm_solver*> ss, gm_result* out);
static int run_ranked(gm_solver* s, gm_result* out);
static int rank_query(gm_solver* s, const uint64_t* keys_dev, uint64_t n, uint32_t* words_dev);
static int rank_positions(gm_solver* s, uint64_t* keys_dev, uint64_t cap, uint64_t* n);
static int rank_scan(gm_solver* s, bool ck, u64* keys_dev, u64 cap, u64* acc);

static const Desc* get_game(int id) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (id < 0 || id >= (int)g_games.size()) return nullptr;
  return &g_games[id];
}

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
struct LevelSeg {
  u64 fb, fe;      // front segment [fb, fe) of the level store
  u64 c2lo, c2hi;  // back segment: back-stack counts [c2lo, c2hi)
};
struct DevState {
  u64 cursor_front;
  u64 cursor_back;
  u64 edges;
  u64 prims;
  u64 max_width;
  uint32_t err;
  uint32_t root_word;
  u64 ks_cursor;    // keyed shards: children emitted by k_ks_expand
  u64 red[5];     // cross-shard reduction: positions, edges, prims, root word + 1, err
  uint32_t word_bits;  // dense: table word width of the solve in progress (resume reads it back)
  uint32_t pad_;
  u64 ck[6];        // gm_solver_checksum: checksum, positions, W, L, T, D
  LevelSeg seg[1];  // [max_levels + 2]
};
static size_t devstate_bytes(int max_levels) {
  return sizeof(DevState) + sizeof(LevelSeg) * (size_t)(max_levels + 2);
}
// Scratch = DevState (cleared per solve) + the dense mask tables (written
// once at solver creation): TS[64] then TD[16][64], u64 each.
constexpr size_t kMaskTableWords = 64 * 17;
static size_t mask_tables_offset(int max_levels) { return (devstate_bytes(max_levels) + 255) / 256 * 256; }
// then per-block position/edge counts of the octet resolves (block_count):
// one plain read-modify-write per block and launch instead of device-scope
// atomics on one line, which serialise at ~12 ns each (MI355X_MICROARCH.md
// "fanin"): 768 resident blocks x 2 counters cost ~18 us at the end of every
// launch.  Cleared per solve, summed by k_fill_red.
struct BlockCount {
  u64 npos, edges;
};
constexpr int kCountSlots = 4096;  // >= any octet-resolve grid (host clamps)
static size_t count_slots_offset(int max_levels) { return mask_tables_offset(max_levels) + kMaskTableWords * sizeof(u64); }
static size_t scratch_bytes_for(int max_levels) {
  return count_slots_offset(max_levels) + kCountSlots * sizeof(BlockCount);
}
// Packed word halos of sharded power-of-two dense tables (exchange_words):
// after the mask tables, the group offset table off[XN][G] (u32; G = Z/64
// groups of a slice, XN = values of x = S - t that leave any slot valid),
// then a send and a receive buffer of 2 slices of words each.
struct HaloGeom {
  u64 Z = 0, nb = 0;
  int XN = 0, NG = 0, NYn = 0, mj = 0, top = 0;
  bool on = false;
};
static HaloGeom halo_geom(const Desc* d, int world, u64 nb) {
  HaloGeom h;
  if (world <= 1 || !d->pow2 || d->nheaps < 3 || d->base[1] < 4) return h;
  const int k = d->nheaps - 1;
  h.Z = d->pstride[k];
  if (h.Z % 256) return h;
  h.nb = nb;
  h.top = k;
  int slow = 0;
  for (int i = 1; i < k; i++) {
    slow += (int)d->heap[i];
    h.mj += (int)((255u >> d->pshift[i]) & (d->base[i] - 1));
  }
  h.XN = slow + (int)d->heap[0] + 1;  // x = S - t with any non-hole
  h.NG = slow + 2;                    // column digit sums 0..slow, plus the total
  h.NYn = h.mj + (int)d->heap[0] + 1;
  h.on = true;
  return h;
}
// column tables PB[XN][NG], NY[NYn], CS[NG] (u32) + send and receive
// buffers of 2 slices per local block
static size_t halo_tab_bytes(const HaloGeom& h) {
  auto r = [](size_t b) { return (b + 255) / 256 * 256; };
  return r((size_t)h.XN * h.NG * 4) + r((size_t)h.NYn * 4) + r((size_t)h.NG * 4);
}
static size_t halo_bytes(const HaloGeom& h) {
  if (!h.on) return 0;
  return halo_tab_bytes(h) + 2 * (h.nb * 2 * h.Z * 4);
}

// Active-group lists of single-table power-of-two dense layouts
// (k_dense_resolve4): per level, the 256-prefix groups holding at least one
// non-hole.  A level's band (dense_band) is a loose bound -- at the narrow
// ends of the tier sequence it spans nearly the whole row while a few
// percent of its groups hold positions -- and XCD chunks of a band split the
// level's work unevenly; a launch over the list sweeps only live groups.
// Group g (base 256 g) holds digit sums [gs, gs + mj] with gs =
// digitsum(256 g), mj = digitsum(255) (pow2 digits are bit fields), so it is
// live at level L iff [gs, gs + mj] meets [S - heap0, S].
//
// Order (L2 reuse): a group's children lie in the same group or in groups
// one or two steps down one digit.  With g = column + top * C (C = groups
// per top-digit slice), the level's columns are cut into 8 contiguous
// ranges of equal live-group count, one per XCD, and each XCD walks its
// range TOP-MAJOR (all its columns at top value t, then t + 1, ...): the
// top-digit children (4-8 MB away in address order) were touched one or two
// steps earlier, the other digits' children are neighbouring columns of the
// same step -- both still in that XCD's L2.  Tables without a top digit
// above the group fall back to address order in 8 equal shares.
struct GroupGeom {
  bool on = false;
  u64 groups = 0;
  int mj = 0;
};
static GroupGeom group_geom(const Desc* d, int world) {
  GroupGeom g;
  if (world != 1 || !d->pow2 || d->nheaps < 2 || d->base[1] < 4 || d->W % 256 || d->W * 4 > 0xFFFFFFF0ull)
    return g;
  g.groups = d->W / 256;
  for (int i = 1; i < d->nheaps; i++) g.mj += (int)((255u >> d->pshift[i]) & (d->base[i] - 1));
  g.on = true;
  return g;
}
// Plan-time choice of 16-bit table words (half the HBM of the word area):
// one-GPU tables the octet kernel (k_dense_resolve8p) can solve, unless the
// plan flags ask for 32-bit words or the one-prefix kernel.  The same flags
// must reach gm_solver_create_shard (gm_buffers.flags), which sizes the
// table against them: a table planned with 16-bit words cannot be handed a
// 32-bit kernel (GM_EINVAL at creation, never a fault).
static uint32_t dense_plan_bits(const Desc* d, int world, uint32_t flags) {
  if (world != 1 || d->kind != K_SUM || !d->pow2 || d->nheaps < 2 || d->nheaps > 8 || d->base[1] < 8 ||
      d->root_sum >= 0x7FFF || d->W * 2 > 0xFFFFFFF0ull || !group_geom(d, 1).on ||
      (flags & (GM_F_WORDS32 | GM_F_RESOLVE_SCALAR)))
    return 32;
  // 8-bit words (k_dense_resolve16p): 16 prefixes per lane, every
  // remoteness < 255 (dense_parent8)
  if (d->base[1] >= 16 && d->root_sum <= 253 && !(flags & GM_F_WORDS16)) return 8;
  return 16;
}
static void group_sums(const Desc* d, const GroupGeom& g, std::vector<uint16_t>& gs) {
  gs.resize(g.groups);
  for (u64 k = 0; k < g.groups; k++) {
    int s = 0;
    for (int i = 1; i < d->nheaps; i++) s += (int)(((k * 256) >> d->pshift[i]) & (d->base[i] - 1));
    gs[k] = (uint16_t)s;
  }
}
static bool group_live(const Desc* d, const GroupGeom& g, int gs, int L) {
  const int S = (int)d->root_sum - L;
  return gs <= S && gs + g.mj >= S - (int)d->heap[0];
}
static u64 group_entries(const Desc* d, const GroupGeom& g) {
  if (!g.on) return 0;
  std::vector<uint16_t> gs;
  group_sums(d, g, gs);
  std::vector<u64> hist(1 << 16, 0);
  for (uint16_t x : gs) hist[x]++;
  u64 n = 0;
  for (int L = 0; L < d->max_levels; L++)
    for (int x = 0; x < (1 << 16); x++)
      if (hist[x] && group_live(d, g, x, L)) n += hist[x];
  return n;
}
static size_t group_bytes(const Desc* d, int world) {
  const GroupGeom g = group_geom(d, world);
  return g.on ? (group_entries(d, g) * 4 + 255) / 256 * 256 : 0;
}

// Column permutation (k_dense_resolve4c): the Z / 256 groups ("columns") of
// a top-digit slice sorted by their digit sum over the digits below the
// top; cstart[x] = first position with sum >= x.  Any world.
struct ColGeom {
  bool on = false;
  int top = 0, mj = 0, maxgs = 0;
  u64 C = 0;
};
static ColGeom col_geom(const Desc* d) {
  ColGeom c;
  if (!d->pow2 || d->nheaps < 3 || d->base[1] < 4) return c;
  c.top = d->nheaps - 1;
  const u64 Z = d->pstride[c.top];
  if (Z % 256 || Z * 4 > 0xFFFFFFF0ull) return c;
  c.C = Z / 256;
  for (int i = 1; i < c.top; i++) {
    c.mj += (int)((255u >> d->pshift[i]) & (d->base[i] - 1));
    c.maxgs += (int)d->heap[i];
  }
  c.on = true;
  return c;
}
static size_t col_bytes(const Desc* d) {
  const ColGeom c = col_geom(d);
  return c.on ? (c.C * 4 + 255) / 256 * 256 : 0;
}
static void build_colperm(const Desc* d, const ColGeom& c, std::vector<uint32_t>& perm, std::vector<uint32_t>& cstart) {
  std::vector<int> gs(c.C);
  for (u64 k = 0; k < c.C; k++) {
    int x = 0;
    for (int i = 1; i < c.top; i++) x += (int)(((k * 256) >> d->pshift[i]) & (d->base[i] - 1));
    gs[k] = x;
  }
  cstart.assign((size_t)c.maxgs + 2, 0);
  for (u64 k = 0; k < c.C; k++) cstart[(size_t)gs[k] + 1]++;
  for (size_t x = 1; x < cstart.size(); x++) cstart[x] += cstart[x - 1];
  perm.assign(c.C, 0);
  std::vector<uint32_t> at(cstart.begin(), cstart.end() - 1);
  for (u64 k = 0; k < c.C; k++) perm[at[gs[k]]++] = (uint32_t)k;  // stable: address order within a sum
}

__device__ __forceinline__ u64 mix64(u64 x) {  // splitmix64 finaliser
  x ^= x >> 31;
  x *= 0x7fb5d329728ea185ull;
  x ^= x >> 27;
  x *= 0x81dadef4bc2dd44dull;
  x ^= x >> 33;
  return x;
}

__device__ __forceinline__ u64 lanemask_lt() {
  return (1ull << __lane_id()) - 1ull;
}

// Wave-aggregated append: one atomic per wave per call site.
__device__ __forceinline__ u64 wave_reserve(u64* cursor, bool pred) {
  u64 mask = __ballot(pred);
  if (mask == 0) return 0;
  int leader = __ffsll((long long)mask) - 1;
  u64 base = 0;
  if ((int)__lane_id() == leader) base = atomicAdd(cursor, (u64)__popcll(mask));
  base = __shfl(base, leader);
  return base + (u64)__popcll(mask & lanemask_lt());
}

// insert key; true iff this call created the slot
__device__ __forceinline__ bool table_insert(gm_slot* tab, u64 mask, u64 key, uint32_t* err) {
  u64 h = mix64(key) & mask;
  for (u64 probe = 0; probe <= mask; probe++) {
    u64 k = __hip_atomic_load(&tab[h].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == key) return false;
    if (k == EMPTY_KEY) {
      u64 old = atomicCAS((u64*)&tab[h].key, (u64)EMPTY_KEY, key);
      if (old == EMPTY_KEY) return true;
      if (old == key) return false;
    }
    h = (h + 1) & mask;
  }
  atomicOr(err, ERR_TABLE_FULL);
  return false;
}

// slot index of key, or ~0 if absent
__device__ __forceinline__ u64 table_find(const gm_slot* tab, u64 mask, u64 key) {
  u64 h = mix64(key) & mask;
  for (u64 probe = 0; probe <= mask; probe++) {
    u64 k = tab[h].key;
    if (k == key) return h;
    if (k == EMPTY_KEY) return ~0ull;
    h = (h + 1) & mask;
  }
  return ~0ull;
}

__device__ __forceinline__ u64 level_key(const u64* lv, u64 lcap, const LevelSeg& s, u64 i) {
  u64 nf = s.fe - s.fb;
  return i < nf ? lv[s.fb + i] : lv[lcap - 1 - (s.c2lo + (i - nf))];
}

// block-wide sum then one atomic per block
// per-block counts into this block's own slot (no atomics; launches on one
// stream run in order, so slot b has one writer at a time)
__device__ __forceinline__ void block_count(BlockCount* bc, u64 npos, u64 edges) {
  __shared__ u64 rn[16], re[16];
  for (int o = 32; o > 0; o >>= 1) {
    npos += __shfl_xor(npos, o);
    edges += __shfl_xor(edges, o);
  }
  const int w = threadIdx.x >> 6;
  if (__lane_id() == 0) {
    rn[w] = npos;
    re[w] = edges;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 sn = 0, se = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); i++) {
      sn += rn[i];
      se += re[i];
    }
    if (sn | se) {
      bc[blockIdx.x].npos += sn;
      bc[blockIdx.x].edges += se;
    }
  }
  __syncthreads();
}
__device__ __forceinline__ void block_add(u64* dst, u64 v) {
  __shared__ u64 red[16];
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  int w = threadIdx.x >> 6;
  if (__lane_id() == 0) red[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 s = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); i++) s += red[i];
    if (s) atomicAdd(dst, s);
  }
  __syncthreads();
}

// Block-staged appends to up to two global stacks (Guideline 12).  Every
// new key used to cost one wave-aggregated atomic on ONE global cursor; a
// device-scope counter saturates near 90 adds/us, which bounded the hashed
// forward (toot 6x4: 324 ms on the widest level).  Keys now go to LDS with
// LDS atomics and a block reserves global space once per flush.  A key that
// finds its LDS queue full is appended straight to global memory (rare).
constexpr uint32_t kStageCap = 1024;  // keys per queue (2 queues: 16 KB, 8+ blocks per CU)
struct StageLDS {
  u64 key[2][kStageCap];
  uint32_t n[2];
  u64 base[2];
};

__device__ __forceinline__ void stage_init(StageLDS& s) {
  if (threadIdx.x == 0) s.n[0] = s.n[1] = 0;
  __syncthreads();
}

// queue q: true if staged, false if the caller must append directly
__device__ __forceinline__ bool stage_push(StageLDS& s, int q, u64 key) {
  const uint32_t j = atomicAdd(&s.n[q], 1u);
  if (j < kStageCap) {
    s.key[q][j] = key;
    return true;
  }
  return false;
}

// Block-uniform: true when a queue is at least 3/4 full.  Both barriers
// are needed so every thread reads the same counts before the next pushes.
__device__ __forceinline__ bool stage_should_flush(StageLDS& s) {
  __syncthreads();
  const bool f = s.n[0] >= kStageCap * 3 / 4 || s.n[1] >= kStageCap * 3 / 4;
  __syncthreads();
  return f;
}

// Reserve [base, base + n) on cursor q with one atomic per queue and copy
// the staged keys out with coalesced stores: store(q, global_index, key).
template <class Store>
__device__ __forceinline__ void stage_flush(StageLDS& s, u64* cur0, u64* cur1, Store store) {
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 0; q < 2; q++) {
      const uint32_t c = min(s.n[q], kStageCap);
      s.n[q] = c;
      s.base[q] = c ? atomicAdd(q ? cur1 : cur0, (u64)c) : 0;
    }
  }
  __syncthreads();
  for (int q = 0; q < 2; q++)
    for (uint32_t j = threadIdx.x; j < s.n[q]; j += blockDim.x) store(q, s.base[q] + j, s.key[q][j]);
  __syncthreads();
  if (threadIdx.x == 0) s.n[0] = s.n[1] = 0;
  __syncthreads();
}

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
__global__ void k_seed(gm_slot* tab, u64 mask, u64* lv, DevState* st, u64 root) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    table_insert(tab, mask, root, &st->err);
    lv[0] = root;
    st->cursor_front = 1;
    st->cursor_back = 0;
    st->seg[0].fb = 0;
    st->seg[0].fe = 1;
    st->seg[0].c2lo = 0;
    st->seg[0].c2hi = 0;
    st->seg[1].c2lo = 0;
    st->seg[1].c2hi = 0;
  }
}

// append a new level-(L+1) key (q = 0, front stack) or level-(L+2) key
// (q = 1, back stack) at global stack index g
__device__ __forceinline__ void level_store(u64* lv, u64 lcap, int q, u64 g, u64 key) {
  if (g < lcap) lv[q ? lcap - 1 - g : g] = key;
}

// K1+K2: expand level L, insert children, append new ones to L+1 / L+2
// through the block's LDS stage (one global atomic per block flush).
template <int KIND>
__global__ __launch_bounds__(256) void k_expand(Desc d, gm_slot* tab, u64 mask, u64* lv, u64 lcap,
                                                DevState* st, int L) {
  __shared__ StageLDS stage;
  stage_init(stage);
  const LevelSeg s = st->seg[L];
  const u64 n = (s.fe - s.fb) + (s.c2hi - s.c2lo);
  const u64 stride = (u64)gridDim.x * blockDim.x;
  uint32_t err = 0;
  auto store = [&](int q, u64 g, u64 key) { level_store(lv, lcap, q, g, key); };
  for (u64 base = (u64)blockIdx.x * blockDim.x; base < n; base += stride) {  // block-uniform
    const u64 i = base + threadIdx.x;
    if (i < n) {
      const u64 key = level_key(lv, lcap, s, i);
      if (Game<KIND>::prim(d, key) == UNDECIDED)  // lookup(): primitive, no children
        Game<KIND>::children(d, key, [&](u64 child, int step) {
          if (!table_insert(tab, mask, child, &st->err)) return;
          if (step != 1 && step != 2) {
            err |= ERR_BAD_STEP;
            return;
          }
          const int q = step - 1;
          if (!stage_push(stage, q, child))
            store(q, atomicAdd(q ? &st->cursor_back : &st->cursor_front, 1ull), child);
        });
    }
    if (stage_should_flush(stage)) stage_flush(stage, &st->cursor_front, &st->cursor_back, store);
  }
  stage_flush(stage, &st->cursor_front, &st->cursor_back, store);
  if (err) atomicOr(&st->err, err);
}

// level bookkeeping after expanding level L (one thread)
__global__ void k_finalize(DevState* st, int L, u64 lcap) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    LevelSeg& nx = st->seg[L + 1];
    nx.fb = st->seg[L].fe;
    nx.fe = st->cursor_front;
    LevelSeg& nn = st->seg[L + 2];
    nn.c2lo = nx.c2hi;
    nn.c2hi = st->cursor_back;
    if (st->cursor_front + st->cursor_back > lcap) st->err |= ERR_LEVELS_FULL;
    u64 w = (nx.fe - nx.fb) + (nx.c2hi - nx.c2lo);
    if (w > st->max_width) st->max_width = w;
  }
}

// K3: resolve level L from its children's words
template <int KIND>
__global__ __launch_bounds__(256) void k_resolve(Desc d, gm_slot* tab, u64 mask, const u64* lv, u64 lcap,
                                                 DevState* st, int L) {
  const LevelSeg s = st->seg[L];
  const u64 n = (s.fe - s.fb) + (s.c2hi - s.c2lo);
  const u64 stride = (u64)gridDim.x * blockDim.x;
  u64 edges = 0, prims = 0;
  uint32_t err = 0;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    u64 key = level_key(lv, lcap, s, i);
    int p = Game<KIND>::prim(d, key);
    uint32_t word;
    if (p != UNDECIDED) {
      word = make_word(p, 0);  // process.py:120-123: primitive, remoteness 0
      prims++;
    } else {
      bool any_loss = false, any_tie = false, any_draw = false;
      uint32_t min_loss = 0xFFFFFFFFu, max_all = 0;
      int nch = Game<KIND>::children(d, key, [&](u64 c, int) {
        u64 h = table_find(tab, mask, c);
        if (h == ~0ull) { err |= ERR_CHILD_MISSING; return; }
        uint32_t w = tab[h].word;
        if (w == NO_WORD) { err |= ERR_CHILD_UNRESOLVED; return; }
        uint32_t v = w & 3u, r = w >> 2;
        if (v == LOSS) { any_loss = true; min_loss = min(min_loss, r); }
        any_tie |= (v == TIE);
        any_draw |= (v == DRAW);
        max_all = max(max_all, r);
      });
      if (nch == 0) err |= ERR_NO_MOVES;
      edges += (u64)nch;
      // reference-canonical _res_red / _remote_red
      if (any_loss) word = make_word(WIN, min_loss + 1);
      else word = make_word(any_tie ? TIE : any_draw ? DRAW : LOSS, max_all + 1);
    }
    u64 h = table_find(tab, mask, key);
    if (h == ~0ull) err |= ERR_SELF_MISSING;
    else tab[h].word = word;
  }
  if (err) atomicOr(&st->err, err);
  block_add(&st->edges, edges);
  block_add(&st->prims, prims);
}

__global__ void k_query(Desc d, const gm_slot* tab, u64 mask, const u64* keys, u64 n, uint32_t* words) {
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
    u64 h = table_find(tab, mask, any_canon(d, keys[i]));  // symmetry hooks: the orbit's representative
    words[i] = h == ~0ull ? NO_WORD : tab[h].word;
  }
}

__global__ void k_root_word(const gm_slot* tab, u64 mask, u64 root, DevState* st) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    u64 h = table_find(tab, mask, root);
    st->root_word = h == ~0ull ? NO_WORD : tab[h].word;
  }
}

__global__ void k_gather_positions(const u64* lv, u64 lcap, const DevState* st, u64* out) {
  u64 nf = st->cursor_front, nb = st->cursor_back;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < nf + nb; i += (u64)gridDim.x * blockDim.x)
    out[i] = i < nf ? lv[i] : lv[lcap - 1 - (i - nf)];
}


#include "gm_dense.h"
#include "gm_keyed_shard.h"

// K4 owner kernel: md5(str(pos)) % P per key (GameState.get_hash,
// src/game_state.py:22-30), the register-resident form where it applies
__global__ void k_owner(Desc d, const u64* keys, u64 n, uint32_t P, uint32_t* owners) {
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x)
    owners[i] = owner_dev(d, keys[i], P);
}
#include "gm_bucketed.h"

// ---------------------------------------------------------------------------
// whole-solve fingerprint (gm_solver_checksum): per block partial sums of
// pos_checksum and the value histogram, one atomic per block and field
// ---------------------------------------------------------------------------
__device__ __forceinline__ void ck_block_add(u64* acc, u64 (&v)[6]) {
  __shared__ u64 part[16][6];
#pragma unroll
  for (int f = 0; f < 6; f++)
    for (int o = 32; o > 0; o >>= 1) v[f] += __shfl_xor(v[f], o);
  const int w = threadIdx.x >> 6;
  if (__lane_id() == 0)
    for (int f = 0; f < 6; f++) part[w][f] = v[f];
  __syncthreads();
  if (threadIdx.x < 6) {
    u64 t = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); i++) t += part[i][threadIdx.x];
    if (t) atomicAdd(&acc[threadIdx.x], t);
  }
}
__device__ __forceinline__ void ck_add(const Desc& d, u64 key, uint32_t word, u64 (&v)[6]) {
  uint8_t c[40];
  const int n = canon_from_key(d, key, c);
  v[0] += pos_checksum(c, n, word & 3u, word >> 2);
  v[1] += 1;
  v[2 + (word & 3u)] += 1;
}
__global__ __launch_bounds__(256) void k_checksum_hashed(Desc d, const gm_slot* tab, u64 mask, const u64* lv, u64 lcap,
                                                         const DevState* st, u64* acc) {
  u64 v[6] = {0, 0, 0, 0, 0, 0};
  const u64 nf = st->cursor_front, nb = st->cursor_back;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < nf + nb; i += (u64)gridDim.x * blockDim.x) {
    const u64 key = i < nf ? lv[i] : lv[lcap - 1 - (i - nf)];
    const u64 h = table_find(tab, mask, key);
    ck_add(d, key, h == ~0ull ? NO_WORD : tab[h].word, v);
  }
  ck_block_add(acc, v);
}
__global__ __launch_bounds__(256) void k_checksum_flat(Desc d, const u64* K, const uint32_t* W, u64 n, u64* acc) {
  u64 v[6] = {0, 0, 0, 0, 0, 0};
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x)
    ck_add(d, K[i], W[i], v);
  ck_block_add(acc, v);
}
__global__ __launch_bounds__(256) void k_checksum_dense(Desc d, DenseView v, const uint32_t* words, const u64* bits,
                                                        u64 levels, uint32_t wbits, u64* acc) {
  u64 a[6] = {0, 0, 0, 0, 0, 0};
  const u64 n = v.Wl;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < levels * n; i += (u64)gridDim.x * blockDim.x) {
    const u64 L = i / n, q = i - L * n;
    bool run;
    const u64 p = dense_global(v, q, &run);
    if (!run) continue;
    const int64_t h0 = dense_h0(d, L, p);
    if (h0 < 0 || !reach_bit(bits, L * v.Wbl + q)) continue;
    const uint32_t w = dense_word_at(words, L * v.Wl + q, wbits);
    ck_add(d, p * d.base[0] + (u64)h0, w, a);
  }
  ck_block_add(acc, a);
}

// ---------------------------------------------------------------------------
// solver object
// ---------------------------------------------------------------------------
// Dense kernel families, fixed when the solver is created (dense_choose,
// from the descriptor, the shard geometry and the GM_F_* flags of
// gm_buffers): nothing later -- no environment variable, no flag change --
// can hand a table a kernel of another word width.  The codes are reported
// in gm_result.kernels (resolve | pull << 16).
// RANKED layout geometry (gm_ranked.h): toot-and-otto positions at computed
// indices
constexpr int kRankMaxCols = 8;
struct RankGeom {
  uint32_t C, H, R, A;     // columns, rows, height radix H + 1, cells
  uint32_t T;              // levels (pieces 0 .. A)
  uint32_t stride[kRankMaxCols];  // hvcode stride of column x: R^x
  u64 nslots;
  uint8_t* words;          // [nslots]
  uint32_t* reach;         // [nslots / 32] reached
  uint32_t* expd;          // [nslots / 32] reached and not primitive
  const u64* base;         // [R^C] hvcode -> first slot of its block
  const uint32_t* lvhv;    // hvcodes level by level
  const uint32_t* lvph;    // the same, heights packed 4 bits per column
  const uint32_t* lvch;    // per block entry, kRankMaxCols u32: child block x's first slot - its level's
                           // first slot (0xFFFFFFFF: column x full)
  const uint32_t* lvpa;    // per block entry, kRankMaxCols u32: parent block x (column x's top piece
                           // removed)'s first slot - its level's first slot (0xFFFFFFFF: column x empty)
  uint8_t* bstat;          // [nslots / 8] per board (stacks): primitive value or UNDECIDED
  u64* pbits;              // [nslots / 512] per board: primitive
  u64 le[7];               // bits j < 64 with popcount(j) <= c
};

enum DenseResolveKind : uint32_t {
  RK_NONE = 0,
  RK_OCT_LIST = 1,   // k_dense_resolve8p: world 1, 16-bit table, live-group lists
  RK_OCT_COLS = 2,   // k_dense_resolve8c: shards, 16-bit table, column jobs
  RK_QUAD_LIST = 3,  // k_dense_resolve4p: world 1, 32-bit table, live-group lists
  RK_QUAD_COLS = 4,  // k_dense_resolve4c: shards, 32-bit table, column jobs
  RK_QUAD_BAND = 5,  // k_dense_resolve4: 32-bit band sweeps (no list)
  RK_SCALAR = 6,     // k_dense_resolve: one prefix per lane (any bases; GM_F_RESOLVE_SCALAR)
  RK_HEX_LIST = 7,   // k_dense_resolve16p: world 1, 8-bit table, live-group lists
  RK_PLANE = 8,      // k_plane_resolve: PLANES layout (gm_plane.h), one plane per half-wave
  RK_PLANE_X2 = 9,   // k_plane_resolve_x2: two planes per half-wave, packed 16-bit lanes
  RK_RANKED = 10,    // k_rk_backward: RANKED layout (gm_ranked.h)
  RK_PLANE_FLOW = 11,  // k_plane_flow: the one-launch PLANES backward (gm_plane.h)
};
enum DensePullKind : uint32_t { PK_NONE = 0, PK_WORDS = 1, PK_LANE = 2, PK_PLANE = 3 };

struct gm_solver {
  Desc d;
  uint32_t mode;
  uint32_t* words;  // DENSE table: levels * Wl words ...
  u64* bits;        // ... followed by the reach bitmap (levels * Wbl bits)
  DenseView view;   // owned prefix range + local addressing
  u64 nslots;       // DENSE: levels * Wl
  // dense sharding over the top prefix digit
  int rank, world;
  u64 nblocks;  // blocks of the top digit over all ranks (view.B values each)
  ncclComm_t comm;  // RCCL communicator (world > 1), or null
  u64* errg = nullptr;  // RCCL: every rank's error mask, all-gathered (world u64, device)
  gm_xfer_fn xfer = nullptr;  // host-staged transport (gm_solver_set_transport), replaces comm
  void* xfer_ctx = nullptr;
  bool halo_ok = false;       // the exchange plan was checked against the other ranks'
  std::vector<uint8_t> hstage;  // host staging of the transport
  gm_slot* tab;
  u64 mask;
  u64* lv;
  u64 lcap;
  DevState* st;
  const u64* masks;  // dense pow2 mask tables in scratch (k_dense_pull_words)
  // sharded dense solves: halo exchanges run on their own stream, ordered
  // against the compute stream by events (created on first use)
  hipStream_t cstream = nullptr;
  std::vector<hipEvent_t> pev;
  // packed word halos (HaloGeom): device offset table, buffers, host totals
  HaloGeom hg;
  HaloTabs ht{};
  bool halo16 = false;  // words travel as 16 bits (k_halo_cols)
  bool w16 = false;     // this solve's table holds 16-bit order-form words (k_dense_resolve8p / 8c)
  bool w8 = false;      // 8-bit order-form words (k_dense_resolve16p)
  uint32_t wbits() const { return w8 ? 8u : w16 ? 16u : 32u; }
  uint32_t plan_bits = 32;  // the table's word width as planned (dense_plan_bits)
  BlockCount* bcount = nullptr;  // per-block counts in scratch (block_count)
  uint32_t* halo_send = nullptr;
  uint32_t* halo_recv = nullptr;
  std::vector<uint32_t> halo_tot;
  // active-group lists (GroupGeom): device list, per-level offsets and
  // per-level XCD shares (host)
  const uint32_t* glist = nullptr;
  std::vector<u64> goff;
  std::vector<uint32_t> gxcd;  // [L * 9 + x]: share x of level L starts at entry gxcd (relative to goff[L])
  // column permutation (ColGeom): device perm, host cstart
  const uint32_t* colperm = nullptr;
  ColGeom cg;
  std::vector<uint32_t> cstart;
  hipStream_t stream;
  bool own_stream;
  uint32_t flags;
  int grid;
  uint32_t step_first = 0, step_stop = 0;  // gm_solver_set_steps (one solve)
  uint32_t rk = RK_NONE, pk = PK_NONE;      // dense kernel families (dense_choose)
  bool launch_err = false;                  // a launch found no kernel of the table's word width
  // whole-solve HIP graphs of a one-table dense solve (run_dense): the
  // forward and the backward launches, captured on the first full solve
  hipGraphExec_t gfwd = nullptr, gbwd = nullptr;
  // one-table PLANES: the counts of a solve in pinned host memory, the
  // solve's timing events, and the ring of queued solves
  // (gm_solver_solve_async / gm_solver_collect)
  u64* phost = nullptr;
  hipEvent_t pse[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};  // run_planes' events (as PlaneSlot::ev)
  PlaneSlot pring[kPlaneRing];
  u64 pq_next = 0, pq_done = 0;  // tickets issued / collected
  // BUCKETED (gm_bucketed.h): level store, words, in-edges, partition scratch
  u64* bkK = nullptr;
  uint32_t* bkW = nullptr;
  uint32_t* REp = nullptr;
  uint16_t* REc = nullptr;  // child index inside its bucket (< kBkMaxUnique)
  u64* S1k = nullptr;
  uint32_t* S1p = nullptr;
  u64* S2k = nullptr;
  uint8_t* S1f = nullptr;  // per staged child: the byte under mix64's top byte (fine bucket bits)
  u64 *XSk = nullptr, *XRk = nullptr;  // md5-sharded bucketed levels: exchange buffers
  uint32_t *XSr = nullptr, *XRr = nullptr;
  std::vector<std::vector<u64>> bks_sc, bks_rc;  // per forward level: records sent to / received from each rank
  uint32_t* REpl = nullptr;  // md5 shards, local-dedup form: in-edges of the rank's own parents' children
  uint16_t* REcl = nullptr;
  struct BksLocal {
    u64 rb = 0, ein = 0, nu = 0;  // local in-edges [rb, rb + ein), unique local children
    uint32_t nbits = 0, cst_off = 0;
    bool used = false;  // this level's children went out in the local-dedup form
  };
  std::vector<BksLocal> bksl;  // per parent level
  u64* xdev = nullptr;  // RCCL all-gather staging of the sharded bucketed loop
  size_t xdev_n = 0;
  u64 Pcap = 0, Ecap = 0, Emax = 0;
  BkLevel* bkL = nullptr;  // device level table (scratch)
  uint32_t *pbase = nullptr, *bh = nullptr, *ph = nullptr, *boff = nullptr, *tot = nullptr, *cbase = nullptr;
  uint32_t *bkcur = nullptr, *bkah = nullptr, *ucnt = nullptr, *meta = nullptr;
  uint32_t* bkgc = nullptr;  // [256 partition cursors | 256 parent-range totals | overflow flag]
  u64* bktotal = nullptr;
  u64 meta_cap = 0;
  std::vector<BkLevel> lvh;  // host copy of the level table
  // PLANES (gm_plane.h, gm_plane_run.h)
  PlaneGeom pg{};
  uint32_t pwb = 1;     // word bytes
  uint32_t pform = 1;   // word form: 1 8-bit, 2 16-bit, 3 relative 8-bit (gm_plane.h)
  // DevState::word_bits of a planes solve in progress (a resume checks it):
  // the word width, 0x100 set for the relative forms
  uint32_t pmark() const { return 8u * pwb | (pform == 3 ? 0x100u : 0u); }
  uint32_t pS = 0;      // last plane level
  void* ptab = nullptr;  // words
  uint32_t* pbits = nullptr;  // reach map, 32 bits per plane row
  void* precv = nullptr;  // shard halo planes received / sent (all levels)
  void* psend = nullptr;
  u64 pnrecv = 0, pnsend = 0;
  const uint4* pzero = nullptr;  // 4 KB of zeros (absent neighbours)
  const void* plist = nullptr;   // level lists (uint32 planes, or PlaneEntry for shards)
  std::vector<u64> ploff;        // per level: first list entry
  std::vector<u64> pbnd;         // shards, per level: first entry that reads a halo plane (they come last)
  std::vector<u64> prcv_off, psnd_off;  // shards, per level: first halo plane received / sent
  // the one-launch backward (k_plane_flow; one-table 8-bit absolute solves):
  // visit lists, counters and per-plane flags in the scratch buffer
  PlaneFlow pflow{};
  bool pflow_ok = false;
  bool pflow_last = false;  // the last solve's backward was k_plane_flow
  uint32_t pflow_grid = 0;
  // staged PLANES shards (run_planes_staged): ploff / prcv_off / psnd_off are
  // per key / per row; k = key skew, K keys, rows 0..smax
  uint32_t pstage_k = 0, pkeys = 0, prows = 0;
  ncclComm_t comm2 = nullptr;        // second communicator (ncclCommSplit): the other halo direction
  // the group's abort flag (solve_multi): once set, its communicators are
  // being aborted and this shard issues no further RCCL call
  std::atomic<int>* gabort = nullptr;
  int defer_rc = 0;                  // a deferred failure of this shard's last solve (0: none)
  std::string defer_msg;
  hipStream_t cstream2 = nullptr;    // receive stream of the staged exchange
  // RANKED (gm_ranked.h)
  RankGeom rg{};
  std::vector<uint32_t> rlvoff;        // per level: first entry of its block list
  std::vector<u64> rlvstart, rlvitems;  // per level: first slot, slots
  u64* rlv_dev = nullptr;              // device: rlvstart then rlvoff (k_rk_scan)
  // md5 shards of the RANKED layout (gm_ranked_shard.h), inside the table
  // buffer: every slot's owner, the level pack / receive buffers, per-level
  // tile counts, their offsets and totals (device; the totals also on the host)
  uint4* rko_own = nullptr;  // owner bit planes, 16 B per 32 slots
  uint8_t *rko_pk = nullptr, *rko_rb = nullptr;
  uint32_t *rko_cnt = nullptr, *rko_toff = nullptr;
  u64* rko_tot = nullptr;
  std::vector<u64> rko_tile0, rko_tot_h;
};

static const int kBlock = 256;

static int launch_grid() {
  static int g = 0;
  if (!g) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
      hipDeviceProp_t p;
      if (hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0) cus = p.multiProcessorCount;
    }
    g = cus * 8;  // Guideline 11: 8 blocks/CU, grid-stride the rest
  }
  return g;
}

template <int KIND>
static void enqueue_level_expand(gm_solver* s, int L) {
  hipLaunchKernelGGL(k_expand<KIND>, dim3(s->grid), dim3(kBlock), 0, s->stream, s->d, s->tab, s->mask, s->lv,
                     s->lcap, s->st, L);
}
template <int KIND>
static void enqueue_level_resolve(gm_solver* s, int L) {
  hipLaunchKernelGGL(k_resolve<KIND>, dim3(s->grid), dim3(kBlock), 0, s->stream, s->d, s->tab, s->mask, s->lv,
                     s->lcap, s->st, L);
}
static void do_expand(gm_solver* s, int L) {
  switch (s->d.kind) {
    case K_SUM: enqueue_level_expand<K_SUM>(s, L); break;
    case K_TTT: enqueue_level_expand<K_TTT>(s, L); break;
    case K_TOOT: enqueue_level_expand<K_TOOT>(s, L); break;
    default: enqueue_level_expand<K_OTHELLO>(s, L); break;
  }
}
static void do_resolve(gm_solver* s, int L) {
  switch (s->d.kind) {
    case K_SUM: enqueue_level_resolve<K_SUM>(s, L); break;
    case K_TTT: enqueue_level_resolve<K_TTT>(s, L); break;
    case K_TOOT: enqueue_level_resolve<K_TOOT>(s, L); break;
    default: enqueue_level_resolve<K_OTHELLO>(s, L); break;
  }
}

// Blocks of 256 threads of `kernel` that fit on the device at once (a
// multiple of 8, one share per XCD): list sweeps launch exactly that many,
// since blocks that start late would sweep their grid-stride items out of
// order.  Cached per kernel.
static int resident_blocks(const void* kernel) {
  static std::mutex mu;
  static std::map<const void*, int> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(kernel);
  if (it != cache.end()) return it->second;
  int per_cu = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, 0) != hipSuccess || per_cu < 1) per_cu = 2;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
  const int r = std::max(8, (per_cu * cus) & ~7);
  cache[kernel] = r;
  return r;
}

// Column jobs of level L over a shard view's listed slices: each slice's
// live columns are one range of the digit-sum-sorted permutation.  False
// if no column is live.
static bool build_col_jobs(const gm_solver* s, const DenseView& v, u64 L, ColJobs& J) {
  J.n = 0;
  J.cum[0] = 0;
  const int64_t S = (int64_t)s->d.root_sum - (int64_t)L;
  for (uint32_t i = 0; i < v.nsl; i++) {
    const int64_t t = (int64_t)v.st[i];
    const int64_t hi = std::min<int64_t>(S - t, s->cg.maxgs);
    const int64_t lo = std::max<int64_t>(S - t - (int64_t)s->d.heap[0] - s->cg.mj, 0);
    if (hi < lo) continue;
    const uint32_t a = s->cstart[(size_t)lo], b = s->cstart[(size_t)hi + 1];
    if (a == b) continue;
    J.lo[J.n] = a;
    J.u[J.n] = (uint32_t)v.sl[i];
    J.t[J.n] = (uint32_t)t;
    J.cum[J.n + 1] = J.cum[J.n] + (b - a);
    J.n++;
  }
  return J.n > 0;
}

// Forward (pull): power-of-two tables run one thread per 64-prefix bitmap
// word (k_dense_pull_words; world 1 over the level's live-group list), other
// bases one prefix per lane (k_dense_pull).
template <int MAXH, bool POW2>
static void dense_launch_pull_t(gm_solver* s, const DenseView& v, int grid, u64 L, u64 root_p) {
  if (POW2 && s->pk == PK_WORDS) {
    const uint32_t* gl = nullptr;
    u64 groups = (v.p_hi - v.p_lo + 63) / 64;
    XcdShares xs{};
    int g;
    if (s->glist && !v.blk) {  // the level's live 256-prefix groups, one share per XCD
      gl = s->glist + s->goff[L];
      if (s->goff[L + 1] == s->goff[L]) return;
      uint32_t widest = 0;
      for (int x = 0; x < 9; x++) xs.o[x] = s->gxcd[(size_t)L * 9 + x];
      for (int x = 0; x < 8; x++) widest = std::max(widest, xs.o[x + 1] - xs.o[x]);
      const u64 per = ((u64)widest * 4 + kBlock - 1) / kBlock;  // blocks per XCD
      g = (int)(kXcds * std::min<u64>(per, (u64)s->grid / kXcds));
    } else {
      g = (int)std::min<u64>((groups + kBlock - 1) / kBlock, (u64)s->grid);
    }
    hipLaunchKernelGGL((k_dense_pull_words<MAXH>), dim3(g), dim3(kBlock), 0, s->stream, s->d, v, s->bits, L,
                       root_p, s->masks, gl, xs);
    return;
  }
  hipLaunchKernelGGL((k_dense_pull<MAXH, POW2>), dim3(grid), dim3(kBlock), 0, s->stream, s->d, v, s->bits, L,
                     root_p);
}
// Backward (resolve) by the family fixed at creation (s->rk, dense_choose).
template <int MAXH, bool POW2>
static void dense_launch_resolve_t(gm_solver* s, const DenseView& v, int grid, u64 L) {
  if constexpr (POW2 && MAXH >= 2) {
    if (s->rk != RK_SCALAR) {
      const uint32_t* gl = nullptr;
      u64 units = (v.p_hi - (v.p_lo & ~255ull) + 3) / 4;
      if (s->glist && !v.blk) {  // live groups of level L, 64 units each
        gl = s->glist + s->goff[L];
        units = (s->goff[L + 1] - s->goff[L]) * 64;
        if (!units) return;
      }
      const int resident = resident_blocks((const void*)k_dense_resolve4<MAXH, false>);
      // shards: column jobs over the level's listed slices (a view that
      // lists no slices -- too many to list -- takes the band sweep)
      if constexpr (MAXH >= 3) {
        if (v.blk && s->colperm && v.nsl > 0 && v.nsl <= (uint32_t)kMaxColJobs) {
          ColJobs J;
          if (!build_col_jobs(s, v, L, J)) return;
          const RowGeom rg{v.Wl, v.Wbl, v.Z};
          if (s->w16) {  // 16-bit shard table: octets, two columns per wave
            const u64 cu8 = (u64)((J.cum[J.n] + 1) / 2) * 64;
            const int g8 = (int)std::min<u64>(
                std::min<u64>(((cu8 + kBlock - 1) / kBlock + 7) & ~7ull,
                              (u64)resident_blocks((const void*)k_dense_resolve8c<MAXH>)),
                (u64)kCountSlots);
            hipLaunchKernelGGL((k_dense_resolve8c<MAXH>), dim3(g8), dim3(kBlock), 0, s->stream, s->d, rg,
                               (uint16_t*)s->words, s->bits, L, s->st, s->colperm, J, s->bcount);
            return;
          }
          const u64 cu = (u64)J.cum[J.n] * 64;
          const int gc = (int)std::min<u64>(((cu + kBlock - 1) / kBlock + 7) & ~7ull,
                                            (u64)resident_blocks((const void*)k_dense_resolve4c<MAXH>));
          hipLaunchKernelGGL((k_dense_resolve4c<MAXH>), dim3(gc), dim3(kBlock), 0, s->stream, s->d, rg, s->words,
                             s->bits, L, s->st, s->colperm, J);
          return;
        }
      }
      if (s->w8) {  // 8-bit table: sixteen prefixes per lane over the live-group list (world 1)
        if (!gl) {
          s->launch_err = true;
          return;
        }
        XcdShares xs;
        for (int x = 0; x < 9; x++) xs.o[x] = s->gxcd[(size_t)L * 9 + x];
        for (int x = 1; x < 8; x++) xs.o[x] &= ~3u;  // shares start at entries divisible by 4: a wave = four groups
        const u64 u16 = (u64)xs.o[8] * 16;
        const int rp = resident_blocks((const void*)k_dense_resolve16p<MAXH>);
        const int gp = (int)std::min<u64>(std::min<u64>(((u16 + kBlock - 1) / kBlock + 7) & ~7ull, (u64)rp),
                                          (u64)kCountSlots);
        hipLaunchKernelGGL((k_dense_resolve16p<MAXH>), dim3(gp), dim3(kBlock), 0, s->stream, s->d, v,
                           (uint8_t*)s->words, s->bits, L, s->st, gl, xs, s->bcount);
        return;
      }
      if (s->w16) {
        // 16-bit table: octets over the live-group list (world 1).  A 16-bit
        // shard table always lists its slices (dense_choose), so reaching
        // here without a list is a bug: flag it instead of running a kernel
        // of the wrong word width.
        if (!gl) {
          s->launch_err = true;
          return;
        }
        XcdShares xs;
        for (int x = 0; x < 9; x++) xs.o[x] = s->gxcd[(size_t)L * 9 + x];
        for (int x = 1; x < 8; x++) xs.o[x] &= ~1u;  // shares start at even entries: a wave = two whole groups
        const u64 u8 = (u64)xs.o[8] * 32;
        const int rp = resident_blocks((const void*)k_dense_resolve8p<MAXH>);
        const int gp = (int)std::min<u64>(std::min<u64>(((u8 + kBlock - 1) / kBlock + 7) & ~7ull, (u64)rp),
                                          (u64)kCountSlots);
        hipLaunchKernelGGL((k_dense_resolve8p<MAXH>), dim3(gp), dim3(kBlock), 0, s->stream, s->d, v,
                           (uint16_t*)s->words, s->bits, L, s->st, gl, xs, s->bcount);
        return;
      }
      const int g = (int)std::min<u64>(((units + kBlock - 1) / kBlock + 7) & ~7ull, (u64)resident);
      if (gl) {  // 32-bit words over the list, software-pipelined
        XcdShares xs;
        for (int x = 0; x < 9; x++) xs.o[x] = s->gxcd[(size_t)L * 9 + x];
        const int rp = resident_blocks((const void*)k_dense_resolve4p<MAXH>);
        const int gp = (int)std::min<u64>(((units + kBlock - 1) / kBlock + 7) & ~7ull, (u64)rp);
        hipLaunchKernelGGL((k_dense_resolve4p<MAXH>), dim3(gp), dim3(kBlock), 0, s->stream, s->d, v, s->words,
                           s->bits, L, s->st, gl, xs);
      } else if (v.blk)
        hipLaunchKernelGGL((k_dense_resolve4<MAXH, true>), dim3(g), dim3(kBlock), 0, s->stream, s->d, v, s->words,
                           s->bits, L, s->st, nullptr, XcdShares{});
      else
        hipLaunchKernelGGL((k_dense_resolve4<MAXH, false>), dim3(g), dim3(kBlock), 0, s->stream, s->d, v, s->words,
                           s->bits, L, s->st, nullptr, XcdShares{});
      return;
    }
  }
  if (s->w16 || s->w8) {  // never chosen with the one-prefix kernel (dense_choose)
    s->launch_err = true;
    return;
  }
  if (v.blk)
    hipLaunchKernelGGL((k_dense_resolve<MAXH, POW2, true, 1, true>), dim3(grid), dim3(kBlock), 0, s->stream, s->d,
                       v, s->words, s->bits, L, s->st);
  else if (v.Wl * 4 <= 0xFFFFFFF0ull)
    hipLaunchKernelGGL((k_dense_resolve<MAXH, POW2, true, 1, false>), dim3(grid), dim3(kBlock), 0, s->stream, s->d,
                       v, s->words, s->bits, L, s->st);
  else
    hipLaunchKernelGGL((k_dense_resolve<MAXH, POW2, false, 1, false>), dim3(grid), dim3(kBlock), 0, s->stream, s->d,
                       v, s->words, s->bits, L, s->st);
}
// kernels are instantiated per exact heap count 1..8 (16 = generic)
template <bool POW2>
static void dense_launch_pull_p(gm_solver* s, const DenseView& v, int grid, u64 L, u64 root_p) {
  switch (s->d.nheaps) {
    case 1: dense_launch_pull_t<1, POW2>(s, v, grid, L, root_p); break;
    case 2: dense_launch_pull_t<2, POW2>(s, v, grid, L, root_p); break;
    case 3: dense_launch_pull_t<3, POW2>(s, v, grid, L, root_p); break;
    case 4: dense_launch_pull_t<4, POW2>(s, v, grid, L, root_p); break;
    case 5: dense_launch_pull_t<5, POW2>(s, v, grid, L, root_p); break;
    case 6: dense_launch_pull_t<6, POW2>(s, v, grid, L, root_p); break;
    case 7: dense_launch_pull_t<7, POW2>(s, v, grid, L, root_p); break;
    case 8: dense_launch_pull_t<8, POW2>(s, v, grid, L, root_p); break;
    default: dense_launch_pull_t<16, POW2>(s, v, grid, L, root_p); break;
  }
}
template <bool POW2>
static void dense_launch_resolve_p(gm_solver* s, const DenseView& v, int grid, u64 L) {
  switch (s->d.nheaps) {
    case 1: dense_launch_resolve_t<1, POW2>(s, v, grid, L); break;
    case 2: dense_launch_resolve_t<2, POW2>(s, v, grid, L); break;
    case 3: dense_launch_resolve_t<3, POW2>(s, v, grid, L); break;
    case 4: dense_launch_resolve_t<4, POW2>(s, v, grid, L); break;
    case 5: dense_launch_resolve_t<5, POW2>(s, v, grid, L); break;
    case 6: dense_launch_resolve_t<6, POW2>(s, v, grid, L); break;
    case 7: dense_launch_resolve_t<7, POW2>(s, v, grid, L); break;
    case 8: dense_launch_resolve_t<8, POW2>(s, v, grid, L); break;
    default: dense_launch_resolve_t<16, POW2>(s, v, grid, L); break;
  }
}
static void dense_launch_pull(gm_solver* s, const DenseView& v, int grid, u64 L, u64 root_p) {
  if (s->d.pow2) dense_launch_pull_p<true>(s, v, grid, L, root_p);
  else dense_launch_pull_p<false>(s, v, grid, L, root_p);
}
static void dense_launch_resolve(gm_solver* s, const DenseView& v, int grid, u64 L) {
  if (s->d.pow2) dense_launch_resolve_p<true>(s, v, grid, L);
  else dense_launch_resolve_p<false>(s, v, grid, L);
}

// Tail runs (world 1, lists; gm_dense.h k_dense_pull_tail /
// k_dense_resolve16_tail): one workgroup walks the run's levels
template <int MAXH>
static void dense_launch_tail_t(gm_solver* s, const TailRun& R, bool pull, u64 root_p) {
  if (pull) {
    hipLaunchKernelGGL((k_dense_pull_tail<MAXH>), dim3(1), dim3(kTailThreads), 0, s->stream, s->d, s->view, s->bits,
                       root_p, s->masks, s->glist, R);
    return;
  }
  if constexpr (MAXH >= 2)
    hipLaunchKernelGGL((k_dense_resolve16_tail<MAXH>), dim3(1), dim3(kTailThreads), 0, s->stream, s->d, s->view,
                       (uint8_t*)s->words, s->bits, s->st, s->glist, R, s->bcount);
  else
    s->launch_err = true;
}
static void dense_launch_tail(gm_solver* s, const TailRun& R, bool pull, u64 root_p) {
  if (!R.n) return;
  switch (s->d.nheaps) {
    case 1: dense_launch_tail_t<1>(s, R, pull, root_p); break;
    case 2: dense_launch_tail_t<2>(s, R, pull, root_p); break;
    case 3: dense_launch_tail_t<3>(s, R, pull, root_p); break;
    case 4: dense_launch_tail_t<4>(s, R, pull, root_p); break;
    case 5: dense_launch_tail_t<5>(s, R, pull, root_p); break;
    case 6: dense_launch_tail_t<6>(s, R, pull, root_p); break;
    case 7: dense_launch_tail_t<7>(s, R, pull, root_p); break;
    case 8: dense_launch_tail_t<8>(s, R, pull, root_p); break;
    default: dense_launch_tail_t<16>(s, R, pull, root_p); break;
  }
}

static std::string err_text(uint32_t e) {
  std::string s;
  if (e & ERR_TABLE_FULL) s += " table-full";
  if (e & ERR_LEVELS_FULL) s += " level-store-full";
  if (e & ERR_BAD_STEP) s += " bad-level-step";
  if (e & ERR_CHILD_MISSING) s += " child-missing";
  if (e & ERR_CHILD_UNRESOLVED) s += " child-unresolved";
  if (e & ERR_NO_MOVES) s += " non-primitive-without-moves";
  if (e & ERR_SELF_MISSING) s += " self-missing";
  if (e & ERR_BUCKET_FULL) s += " hash-bucket-over-capacity";
  if (e & ERR_EDGE_COUNT) s += " edge-count-mismatch";
  if (e & ERR_SHARD_FAILED) s += " shard-failed";
  if (e & ERR_PLANE_STALL) s += " plane-flow-stalled";
  return s;
}

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
extern "C" {

const char* gm_last_error(void) { return g_err.c_str(); }
const char* gm_version(void) { return "gamesmanmpi_amd 0.1 (gfx950)"; }

int gm_abi_sizes(uint32_t out[3]) {
  if (!out) return fail(GM_EINVAL, "null argument");
  out[0] = (uint32_t)sizeof(gm_plan_t);
  out[1] = (uint32_t)sizeof(gm_buffers);
  out[2] = (uint32_t)sizeof(gm_result);
  return 0;
}

int gm_game_lookup(const char* name, const char* params, int* game_id) {
  if (!name || !game_id) return fail(GM_EINVAL, "null argument");
  Desc d;
  int rc = build_desc(name, params ? params : "", &d);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(g_mu);
  for (size_t i = 0; i < g_games.size(); i++)
    if (!memcmp(&g_games[i], &d, sizeof d)) { *game_id = (int)i; return 0; }
  g_games.push_back(d);
  *game_id = (int)g_games.size() - 1;
  return 0;
}

int gm_game_info(int game, uint64_t* positions_bound, uint32_t* max_levels, uint32_t* key_bits) {
  const Desc* d = get_game(game);
  if (!d) return fail(GM_EINVAL, "bad game id %d", game);
  uint64_t bound = 0;
  uint32_t bits = 0;
  switch (d->kind) {
    case K_SUM: {
      unsigned __int128 p = 1;
      for (int i = 0; i < d->nheaps; i++) p *= d->base[i];
      bound = (uint64_t)p;
      bits = 64 - __builtin_clzll(bound | 1);
      break;
    }
    case K_TTT: bound = 5478; bits = 18; break;
    case K_TOOT: {
      // reachable counts measured by the survey (Appendix B) where known
      if (d->L == 3 && d->H == 3) bound = 11097;
      else if (d->L == 4 && d->H == 3) bound = 200127;
      else if (d->L == 3 && d->H == 4) bound = 126559;
      else if (d->L == 4 && d->H == 4) bound = 3468773;
      else if (d->L == 5 && d->H == 4) bound = 70184763;
      else if (d->L == 6 && d->H == 4) bound = 1187212827ull;
      else bound = 0;  // unknown: caller must pass an estimate to gm_plan
      bits = 2 * d->A + 13;
      break;
    }
    default:
      if (d->L == 4) bound = 54089;
      else bound = 0;
      bits = 2 * d->A + 3;
  }
  if (positions_bound) *positions_bound = bound;
  if (max_levels) *max_levels = (uint32_t)d->max_levels;
  if (key_bits) *key_bits = bits;
  return 0;
}

int gm_root(int game, uint64_t* key) {
  const Desc* d = get_game(game);
  if (!d || !key) return fail(GM_EINVAL, "bad game id %d", game);
  *key = d->root;
  return 0;
}

int gm_encode(int game, const uint8_t* canon, size_t n, uint64_t* key) {
  const Desc* d = get_game(game);
  if (!d || !canon || !key) return fail(GM_EINVAL, "bad argument");
  if (d->kind == K_TOOT || d->kind == K_OTHELLO) {
    if (key_from_bits(*d, canon, (int)n, key)) return fail(GM_EINVAL, "bytes are not a %s position", d->kind == K_TOOT ? "toot" : "othello");
    return 0;
  }
  if (d->kind == K_TTT) {
    if (n != 9) return fail(GM_EINVAL, "tic-tac-toe positions are 9 bytes");
    uint64_t k = 0;
    for (int c = 0; c < 9; c++) {
      uint32_t v;
      if (d->variant == 1) {
        if (canon[c] == '_') v = 0;
        else if (canon[c] == 'X') v = 1;
        else if (canon[c] == 'O') v = 2;
        else return fail(GM_EINVAL, "mttt cell must be _ X or O");
      } else {
        if (canon[c] > 2) return fail(GM_EINVAL, "tic_tac_toe_np cell must be 0, 1 or 2");
        v = canon[c];
      }
      k |= (uint64_t)v << (2 * c);
    }
    *key = k;
    return 0;
  }
  if (n == 0 || n > 20) return fail(GM_EINVAL, "bad integer position");
  unsigned __int128 v = 0;
  for (size_t i = 0; i < n; i++) {
    if (canon[i] < '0' || canon[i] > '9') return fail(GM_EINVAL, "integer positions are non-negative decimals");
    v = v * 10 + (canon[i] - '0');
  }
  unsigned __int128 space = 1;
  for (int i = 0; i < d->nheaps; i++) space *= d->base[i];
  if (v >= space) return fail(GM_EINVAL, "position outside the game's state space");
  *key = (uint64_t)v;
  return 0;
}

int gm_decode(int game, uint64_t key, uint8_t* canon, size_t cap, size_t* n) {
  const Desc* d = get_game(game);
  if (!d || !canon || !n) return fail(GM_EINVAL, "bad argument");
  uint8_t tmp[64];
  int m = canon_from_key(*d, key, tmp);
  if ((size_t)m > cap) return fail(GM_EINVAL, "buffer too small");
  memcpy(canon, tmp, (size_t)m);
  *n = (size_t)m;
  return 0;
}

int gm_encode_batch(int game, const uint8_t* canon, size_t stride, const uint8_t* lens, size_t n,
                    uint64_t* keys) {
  for (size_t i = 0; i < n; i++) {
    int rc = gm_encode(game, canon + i * stride, lens[i], &keys[i]);
    if (rc) return rc;
  }
  return 0;
}

int gm_decode_batch(int game, const uint64_t* keys, size_t n, uint8_t* canon, size_t stride, uint8_t* lens) {
  const Desc* d = get_game(game);
  if (!d || (n && (!keys || !canon || !lens))) return fail(GM_EINVAL, "bad argument");
  for (size_t i = 0; i < n; i++) {
    uint8_t tmp[64];
    int m = canon_from_key(*d, keys[i], tmp);
    if ((size_t)m > stride) return fail(GM_EINVAL, "stride too small");
    memset(canon + i * stride, 0, stride);
    memcpy(canon + i * stride, tmp, (size_t)m);
    lens[i] = (uint8_t)m;
  }
  return 0;
}

int gm_str_utf8(int game, uint64_t key, uint8_t* out, size_t cap, size_t* n) {
  const Desc* d = get_game(game);
  if (!d || !out || !n) return fail(GM_EINVAL, "bad argument");
  uint8_t tmp[64];
  int m = str_utf8_from_key(*d, key, tmp);
  if ((size_t)m > cap) return fail(GM_EINVAL, "buffer too small");
  memcpy(out, tmp, (size_t)m);
  *n = (size_t)m;
  return 0;
}

int gm_host_expand(int game, const uint64_t* keys, size_t n, uint64_t* children, uint8_t* nchild, uint8_t* prim) {
  const Desc* d = get_game(game);
  if (!d || (n && (!keys || !children || !nchild || !prim))) return fail(GM_EINVAL, "bad argument");
  for (size_t i = 0; i < n; i++) {
    prim[i] = (uint8_t)any_prim(*d, keys[i]);
    int c = 0;
    if (prim[i] == UNDECIDED)
      any_children(*d, keys[i], [&](uint64_t ck, int) {
        if (c < GM_MAXCHILD) children[i * GM_MAXCHILD + c] = ck;
        c++;
      });
    if (c > GM_MAXCHILD) return fail(GM_ECORRUPT, "more than %d children", GM_MAXCHILD);
    nchild[i] = (uint8_t)c;
  }
  return 0;
}

int gm_host_level(int game, const uint64_t* keys, size_t n, int32_t* levels) {
  const Desc* d = get_game(game);
  if (!d || (n && (!keys || !levels))) return fail(GM_EINVAL, "bad argument");
  for (size_t i = 0; i < n; i++) levels[i] = any_level(*d, keys[i]);
  return 0;
}

int gm_symmetry(int game, int which, const uint64_t* keys, size_t n, uint64_t* out) {
  const Desc* d = get_game(game);
  if (!d || (n && (!keys || !out))) return fail(GM_EINVAL, "bad argument");
  if (which == -1) {
    for (size_t i = 0; i < n; i++) out[i] = any_canon(*d, keys[i]);
    return 0;
  }
  if (which != 0 || d->kind != K_OTHELLO) return fail(GM_EINVAL, "no symmetry function %d for this game", which);
  for (size_t i = 0; i < n; i++) out[i] = oth_flip(*d, keys[i]);
  return 0;
}

int gm_owner_host(int game, const uint64_t* keys, size_t n, int world_size, uint32_t* owners) {
  const Desc* d = get_game(game);
  if (!d || world_size < 1 || (n && (!keys || !owners))) return fail(GM_EINVAL, "bad argument");
  for (size_t i = 0; i < n; i++) {
    uint8_t s[64], dig[16];
    int len = str_utf8_from_key(*d, keys[i], s);
    md5_block(s, len, dig);
    owners[i] = md5_mod(dig, (uint32_t)world_size);
  }
  return 0;
}

static int plan_dense(const Desc* d, int rank, int world, uint32_t flags, uint64_t max_table_bytes, gm_plan_t* out,
                      bool* fits) {
  DenseGeom g;
  int rc = dense_geom(d, rank, world, &g);
  if (rc) return rc;
  const u64 bytes = dense_words_bytes(d, g, dense_plan_bits(d, world, flags)) + dense_bits_bytes(d, g);
  *fits = max_table_bytes == 0 || bytes <= max_table_bytes;
  out->mode = GM_MODE_DENSE;
  out->table_slots = (u64)d->max_levels * g.v.Wl;
  out->table_bytes = bytes;
  out->level_capacity = 1;
  return 0;
}

int gm_shard_info(int game, int rank, int world, uint64_t out[8]) {
  const Desc* d = get_game(game);
  if (!d || !out) return fail(GM_EINVAL, "bad argument");
  if (!d->dense_ok) return fail(GM_EINVAL, "game has no dense layout");
  DenseGeom g;
  int rc = dense_geom(d, rank, world, &g);
  if (rc) return rc;
  const uint64_t v[8] = {g.v.B, g.nblocks, g.nb, (uint64_t)rank, g.v.Z, g.v.E, g.v.Wl, (uint64_t)world};
  memcpy(out, v, sizeof v);
  return 0;
}

int gm_plan_shard(int game, int rank, int world, uint32_t flags, uint64_t max_table_bytes, gm_plan_t* out) {
  const Desc* d = get_game(game);
  if (!d || !out) return fail(GM_EINVAL, "bad argument");
  memset(out, 0, sizeof *out);
  out->max_levels = (uint32_t)d->max_levels;
  out->scratch_bytes = scratch_bytes_for(d->max_levels);
  if (!d->dense_ok || (flags & GM_F_FORCE_HASHED))
    return fail(GM_EINVAL, "only DENSE layouts shard by prefix blocks; keyed tables shard by md5 owner");
  if (plane_wanted(d, flags, world)) {
    bool fits = false;
    int rc = plan_planes(d, rank, world, flags, max_table_bytes, out, &fits);
    if (rc) return rc;
    if (!fits) return fail(GM_EFULL, "planes shard needs %llu bytes", (unsigned long long)out->table_bytes);
    return 0;
  }
  DenseGeom g;
  int grc = dense_geom(d, rank, world, &g);
  if (grc) return grc;
  out->scratch_bytes += halo_bytes(halo_geom(d, world, g.nb)) + col_bytes(d);
  bool fits = false;
  int rc = plan_dense(d, rank, world, flags, max_table_bytes, out, &fits);
  if (rc) return rc;
  if (!fits) return fail(GM_EFULL, "dense shard needs %llu bytes", (unsigned long long)out->table_bytes);
  return 0;
}

// ---- BUCKETED plan ---------------------------------------------------------
// keyed games whose every move advances one level (the tier is the number
// of pieces placed): the bucketed pipeline applies (gm_bucketed.h)
// every move advances one level, and remoteness < 256 (packed backward answers)
static bool bk_ok(const Desc* d) {
  return (d->kind == K_TTT || d->kind == K_TOOT || d->kind == K_OTHELLO) && d->max_levels <= 256;
}
// edges bound for a positions bound: the known counts where the board and
// bound match (SURVEY Appendix B / tests/golden), else a branching factor
// above every known board's
struct BkKnown {
  int kind, L, H;
  u64 P, E;
};
static const BkKnown* bk_known(const Desc* d) {
  static const BkKnown kn[] = {
      {K_TOOT, 3, 3, 11097ull, 27774ull},          {K_TOOT, 4, 3, 200127ull, 640648ull},
      {K_TOOT, 4, 4, 3468773ull, 9932808ull},      {K_TOOT, 5, 4, 70184763ull, 226547754ull},
      {K_TOOT, 6, 4, 1187212827ull, 4243234712ull}, {K_OTHELLO, 4, 4, 54089ull, 69916ull},
      {K_TTT, 0, 0, 5478ull, 16167ull}};
  for (const BkKnown& k : kn)
    if (k.kind == d->kind && (d->kind == K_TTT || (k.L == d->L && k.H == d->H))) return &k;
  return nullptr;
}
static u64 bk_edges_bound(const Desc* d, u64 P) {
  const BkKnown* k = bk_known(d);
  if (k && P <= k->P) return k->E + 1024;
  const double ratio = d->kind == K_TOOT ? 3.6 : d->kind == K_TTT ? 3.0 : 2.0;
  return (u64)(ratio * (double)P) + 1024;
}
// out-edges of the P positions an md5 shard owns: the md5 partition spreads
// positions evenly and regardless of their move counts, so a shard's share of
// the edges is its share of the positions -- the board's known edge / position
// ratio (+2 %), else the per-kind ratio; not the whole board's edges, which
// sized every shard of toot 6x4 for the full 4.2e9 (4 shards: out of memory)
static u64 bk_shard_edges_bound(const Desc* d, u64 P) {
  const BkKnown* k = bk_known(d);
  if (k && P < k->P) return std::min<u64>(k->E, (u64)((double)k->E / (double)k->P * (double)P * 1.02)) + 1024;
  return bk_edges_bound(d, P);
}
// in-edges of the widest level: a quarter of all edges (every known board
// is below a fifth; a level over it returns GM_EFULL and the host re-plans)
// (+5% and a run per partition: the count-free expand provisions each of the
// 256 coarse partitions a 1/256 share of it, k_bk_expand<OVER>)
static u64 bk_emax_bound(u64 E) { return std::min<u64>(E, std::max<u64>(E / 4, 1u << 20)) / 20 * 21 + (u64)kBkC * 4096; }
struct BkScratch {
  size_t lv, pbase, bh, ph, boff, tot, cbase, ah, cur, ucnt, total, gc, meta, end;
};
static BkScratch bk_scratch(int T) {
  auto r = [](size_t b) { return (b + 255) / 256 * 256; };
  BkScratch x;
  size_t o = r(devstate_bytes(T));
  x.lv = o; o += r(sizeof(BkLevel) * (size_t)T);
  x.pbase = o; o += r((size_t)T * (kBkC + 1) * 4);
  x.bh = o; o += r((size_t)kBkExpandBlocks * kBkC * 4);
  x.ph = o; o += r((size_t)kBkExpandBlocks * kBkC * 4);
  x.boff = o; o += r((size_t)kBkExpandBlocks * kBkC * 4);
  x.tot = o; o += r(2 * kBkC * 4);
  x.cbase = o; o += r((kBkC + 1) * 4);
  const size_t NBmax = (size_t)kBkC << kBkMaxFineBits;
  x.ah = o; o += r((size_t)T * kBkC * kBkC * 4);  // per level: answers per (child partition, parent range)
  x.cur = o; o += r((kBkC + ((size_t)1 << (29 - kBkRangeBits)) + 1) * 4);  // B3 / B4 run cursors
  x.ucnt = o; o += r(NBmax * 4);
  x.total = o; o += r(2 * 8);
  x.gc = o; o += r((2 * kBkC + 4) * 4);  // k_bk_expand<OVER>: partition cursors, parent-range totals, overflow flag
  const size_t NRmax = (size_t)1 << (29 - kBkRangeBits);
  // per level: cst, fo, rfo (twice: md5 shards' local-dedup form keeps a second cst / fo per level)
  x.meta = o; o += r((size_t)T * 2 * (2 * (NBmax + 1) + NRmax + 1) * 4);
  x.end = o;
  return x;
}

int gm_plan(int game, uint64_t positions, uint32_t flags, uint64_t max_table_bytes, gm_plan_t* out) {
  const Desc* d = get_game(game);
  if (!d || !out) return fail(GM_EINVAL, "bad argument");
  memset(out, 0, sizeof *out);
  out->max_levels = (uint32_t)d->max_levels;
  out->scratch_bytes = scratch_bytes_for(d->max_levels);
  if (d->dense_ok && plane_wanted(d, flags, 1)) {
    bool fits = false;
    int rc = plan_planes(d, 0, 1, flags, max_table_bytes, out, &fits);
    if (rc) return rc;
    if (fits) return 0;
    memset(out, 0, sizeof *out);
    out->max_levels = (uint32_t)d->max_levels;
    out->scratch_bytes = scratch_bytes_for(d->max_levels);
  }
  if (d->dense_ok && !(flags & GM_F_FORCE_HASHED)) {
    bool fits = false;
    int rc = plan_dense(d, 0, 1, flags, max_table_bytes, out, &fits);
    if (rc) return rc;
    out->scratch_bytes += col_bytes(d) + group_bytes(d, 1);
    if (fits) return 0;
    memset(out, 0, sizeof *out);
    out->max_levels = (uint32_t)d->max_levels;
    out->scratch_bytes = scratch_bytes_for(d->max_levels);
  }
  if (rank_wanted(d, flags)) {  // toot-and-otto: positions at computed indices (gm_ranked.h)
    bool fits = false;
    int rc = plan_ranked(d, max_table_bytes, out, &fits);
    if (rc) return rc;
    if (fits) return 0;
    memset(out, 0, sizeof *out);
    out->max_levels = (uint32_t)d->max_levels;
    out->scratch_bytes = scratch_bytes_for(d->max_levels);
  }
  if (positions == 0) {
    gm_game_info(game, &positions, nullptr, nullptr);
    if (positions == 0) return fail(GM_EINVAL, "no known position bound for this board; pass an estimate");
  }
  if (bk_ok(d) && !(flags & GM_F_HASH_TABLE)) {
    // bucketed levels: keys (levels buffer), words + in-edges + two
    // partition buffers of the widest level's in-edges (table buffer)
    const u64 P = positions + 64, E = bk_edges_bound(d, positions), Em = bk_emax_bound(E);
    if (Em >= 0xFFFFFFF0ull) return fail(GM_EINVAL, "a level of more than 2^32 edges: not supported");
    const u64 bytes = 4 * P + 6 * E + 24 * Em;  // words, in-edges (u32 parent + u16 child), staging
    // over the caller's byte budget: the keyed hash table instead (as a
    // dense table over budget falls back above)
    if (max_table_bytes == 0 || bytes <= max_table_bytes) {
      out->mode = GM_MODE_BUCKETED;
      out->level_capacity = P;
      out->table_slots = E;
      out->table_bytes = bytes;
      out->scratch_bytes = bk_scratch(d->max_levels).end;
      return 0;
    }
  }
  uint64_t slots = 1024;
  while (slots < 2 * positions) slots <<= 1;  // load factor <= 0.5
  out->mode = GM_MODE_HASHED;
  out->table_slots = slots;
  out->table_bytes = slots * sizeof(gm_slot);
  out->level_capacity = positions + 64;
  return 0;
}

int gm_plan_keyed_shard(int game, int rank, int world, uint64_t positions, uint32_t flags, uint64_t max_table_bytes,
                        gm_plan_t* out) {
  const Desc* d = get_game(game);
  if (!d || !out) return fail(GM_EINVAL, "bad argument");
  if (world < 2 || world > 8 || rank < 0 || rank >= world) return fail(GM_EINVAL, "bad shard %d/%d (2..8 ranks)", rank, world);
  if (flags & GM_F_RANKED_SHARD) {  // the RANKED index space, md5-owned slots (gm_ranked_shard.h)
    memset(out, 0, sizeof *out);
    return plan_ranked_shard(d, world, max_table_bytes, out);
  }
  if (!bk_ok(d) || (flags & GM_F_HASH_TABLE))
    return fail(GM_EINVAL, "md5-sharded bucketed levels need every move to advance one level");
  memset(out, 0, sizeof *out);
  out->max_levels = (uint32_t)d->max_levels;
  if (positions == 0) {
    gm_game_info(game, &positions, nullptr, nullptr);
    if (positions == 0) return fail(GM_EINVAL, "no known position bound for this board; pass an estimate");
  }
  const u64 P = positions + 64, E = bk_shard_edges_bound(d, positions), Em = bk_emax_bound(E);
  if (Em >= 0xFFFFFFF0ull) return fail(GM_EINVAL, "a level of more than 2^32 edges: not supported");
  const u64 bytes = 4 * P + 12 * E + 48 * Em + 64;  // the one-GPU layout + local in-edges + the exchange buffers
  if (max_table_bytes && bytes > max_table_bytes)
    return fail(GM_EFULL, "bucketed shard needs %llu bytes", (unsigned long long)bytes);
  out->mode = GM_MODE_BUCKETED;
  out->level_capacity = P;
  out->table_slots = E;
  out->table_bytes = bytes;
  out->scratch_bytes = bk_scratch(d->max_levels).end;
  return 0;
}

// Per-lane condition masks of a 64-prefix group for power-of-two layouts
// (k_dense_pull_words): with j the lane's offset in the group,
//   M[t]              = { j : sum_i digit_i(j) <= t }   (TS)
//   M[64 (i + 1) + t] = { j : digit_i(j) <= t }         (TD[i], i >= 1)
// They depend only on the descriptor, so they are built once here.
static void build_mask_tables(const Desc& d, u64* M) {
  memset(M, 0, kMaskTableWords * sizeof(u64));
  for (int j = 0; j < 64; j++) {
    uint32_t dj[16] = {0}, sj = 0;
    for (int i = 1; i < d.nheaps; i++) {
      dj[i] = (uint32_t)((j >> d.pshift[i]) & (d.base[i] - 1));
      sj += dj[i];
    }
    for (int t = 0; t < 64; t++) {
      if (sj <= (uint32_t)t) M[t] |= 1ull << j;
      for (int i = 1; i < d.nheaps; i++)
        if (dj[i] <= (uint32_t)t) M[64 * (i + 1) + t] |= 1ull << j;
    }
  }
}

// Column tables of the packed halos (k_halo_cols).  Slot j of a column
// (j < 256, digit sum ds(j) over the digits below the top) is a non-hole of
// slice x iff ds(j) in [y - heap0, y], y = x - gs: NY[y] counts them,
// PB[x][g] sums NY over the columns of smaller sum, and tot[x] = PB[x][NG-1]
// is the slice's non-hole total.
static void build_halo_cols(const Desc& d, const HaloGeom& h, const std::vector<uint32_t>& cstart,
                            std::vector<uint32_t>& PB, std::vector<uint32_t>& NY, std::vector<uint32_t>& CS,
                            std::vector<uint32_t>& tot) {
  const int H0 = (int)d.heap[0];
  NY.assign((size_t)h.NYn, 0);
  for (int j = 0; j < 256; j++) {
    int ds = 0;
    for (int i = 1; i < h.top; i++) ds += (int)(((uint32_t)j >> d.pshift[i]) & (d.base[i] - 1));
    for (int y = ds; y <= ds + H0 && y < h.NYn; y++) NY[(size_t)y]++;
  }
  CS.assign((size_t)h.NG, 0);
  std::vector<uint32_t> cnt((size_t)h.NG, 0);
  for (int g = 0; g < h.NG; g++) {
    CS[(size_t)g] = g + 1 < (int)cstart.size() ? cstart[(size_t)g] : cstart.back();
    if (g + 1 < (int)cstart.size()) cnt[(size_t)g] = cstart[(size_t)g + 1] - cstart[(size_t)g];
  }
  PB.assign((size_t)h.XN * h.NG, 0);
  tot.assign((size_t)h.XN, 0);
  for (int x = 0; x < h.XN; x++) {
    uint32_t run = 0;
    for (int g = 0; g < h.NG; g++) {
      PB[(size_t)x * h.NG + g] = run;
      const int y = x - g;
      if (y >= 0 && y < h.NYn) run += cnt[(size_t)g] * NY[(size_t)y];
    }
    tot[(size_t)x] = run;
  }
}

static u64 blk_count(const gm_solver* s);
// Kernel families of a dense solver (DenseResolveKind / DensePullKind),
// chosen once from the descriptor, the geometry, the scratch the caller
// provided and the flags.  16-bit tables: world 1 needs the live-group
// lists (octets sweep only listed groups); shards need the column
// permutation, packed 16-bit halos and every level's slices in one job list.
static int dense_choose(gm_solver* s) {
  const Desc& d = s->d;
  const DenseView& v = s->view;
  s->pk = d.pow2 ? PK_WORDS : PK_LANE;
  const bool scalar = (s->flags & GM_F_RESOLVE_SCALAR) != 0;
  const bool quad = d.pow2 && d.nheaps >= 2 && d.base[1] >= 4 && v.Wl * 4 <= 0xFFFFFFF0ull && (!v.blk || v.Z % 256 == 0);
  const bool base16 = d.pow2 && d.kind == K_SUM && d.nheaps >= 2 && d.nheaps <= 8 && d.base[1] >= 8 &&
                      d.root_sum < 0x7FFF && v.Wl * 2 <= 0xFFFFFFF0ull &&
                      !(s->flags & (GM_F_WORDS32 | GM_F_RESOLVE_SCALAR));
  s->w8 = false;
  if (!v.blk) {
    if (s->plan_bits < 32) {
      if (!s->glist)
        return fail(GM_EINVAL, "%u-bit dense table without live-group lists: scratch smaller than gm_plan's",
                    s->plan_bits);
      s->w16 = s->plan_bits == 16;
      s->w8 = s->plan_bits == 8;
      s->rk = s->w8 ? RK_HEX_LIST : RK_OCT_LIST;
      return 0;
    }
    s->w16 = false;
    s->rk = (scalar || !quad) ? RK_SCALAR : s->glist ? RK_QUAD_LIST : RK_QUAD_BAND;
    return 0;
  }
  s->w16 = base16 && d.nheaps >= 3 && s->colperm && s->hg.on && s->halo16 && v.Z % 256 == 0 && v.E <= 0xFFFF &&
           blk_count(s) * (v.B + 4) <= (u64)kMaxColJobs;
  s->rk = s->w16 ? RK_OCT_COLS : (scalar || !quad) ? RK_SCALAR : s->colperm ? RK_QUAD_COLS : RK_QUAD_BAND;
  return 0;
}

int gm_solver_create_shard(int game, int rank, int world, const gm_buffers* buf, gm_solver** out) {
  const Desc* d = get_game(game);
  if (!d || !buf || !out) return fail(GM_EINVAL, "bad argument");
  if (!buf->table || !buf->scratch) return fail(GM_EINVAL, "null device buffer");
  if (buf->scratch_bytes < scratch_bytes_for(d->max_levels)) return fail(GM_EINVAL, "scratch too small (use gm_plan)");
  DenseGeom g;
  memset(&g, 0, sizeof g);
  if (buf->mode == GM_MODE_DENSE) {
    if (!d->dense_ok) return fail(GM_EINVAL, "game has no dense layout");
    int rc = dense_geom(d, rank, world, &g);
    if (rc) return rc;
    if (buf->table_slots != (u64)d->max_levels * g.v.Wl) return fail(GM_EINVAL, "dense table must hold levels * Wl words (use gm_plan_shard)");
    // the word width follows from the flags: a table planned with 16-bit
    // words is too small for the 32-bit kernels other flags select
    const u64 need = dense_words_bytes(d, g, dense_plan_bits(d, world, buf->flags)) + dense_bits_bytes(d, g);
    if (buf->table_bytes < need)
      return fail(GM_EINVAL, "dense table of %llu bytes, these flags need %llu (plan with the flags the solver is "
                             "created with)", (unsigned long long)buf->table_bytes, (unsigned long long)need);
  } else if (buf->mode == GM_MODE_PLANES) {
    if (!d->dense_ok || !plane_ok(d, world)) return fail(GM_EINVAL, "game has no planes layout");
    if (world > 1 && (rank < 0 || rank >= world)) return fail(GM_EINVAL, "bad shard %d/%d", rank, world);
  } else if (buf->mode == GM_MODE_RANKED) {
    if (world != 1 && !(buf->flags & GM_F_RANKED_SHARD))
      return fail(GM_EINVAL, "ranked md5 shards are planned with GM_F_RANKED_SHARD (gm_plan_keyed_shard)");
    if (world > 8 || rank < 0 || rank >= world) return fail(GM_EINVAL, "bad ranked shard %d/%d (2..8 ranks)", rank, world);
    if (!rank_ok(d)) return fail(GM_EINVAL, "game has no ranked layout");
  } else if (buf->mode == GM_MODE_BUCKETED) {
    if (world < 1 || rank < 0 || rank >= world) return fail(GM_EINVAL, "bad shard %d/%d", rank, world);
    if (world > 8) return fail(GM_EINVAL, "md5-sharded bucketed levels support up to 8 ranks");
    if (!bk_ok(d)) return fail(GM_EINVAL, "bucketed levels need every move to advance one level");
    if (!buf->levels || buf->level_capacity < 2) return fail(GM_EINVAL, "null level store");
    if (buf->scratch_bytes < bk_scratch(d->max_levels).end) return fail(GM_EINVAL, "scratch too small (use gm_plan)");
    const u64 fixed = 4 * buf->level_capacity + 6 * buf->table_slots;
    if (buf->table_bytes < fixed + (world > 1 ? 48 : 24) * 1024ull)
      return fail(GM_EINVAL, "bucketed table too small (use gm_plan / gm_plan_keyed_shard)");
  } else if (buf->mode == GM_MODE_HASHED) {
    if (world < 1 || rank < 0 || rank >= world) return fail(GM_EINVAL, "bad shard %d/%d", rank, world);
    if (!buf->levels || buf->level_capacity < 1) return fail(GM_EINVAL, "null level store");
    if (buf->table_slots < 2 || (buf->table_slots & (buf->table_slots - 1)))
      return fail(GM_EINVAL, "table_slots must be a power of two");
    if (buf->table_bytes < buf->table_slots * sizeof(gm_slot))
      return fail(GM_EINVAL, "keyed table of %llu bytes holds fewer than %llu slots",
                  (unsigned long long)buf->table_bytes, (unsigned long long)buf->table_slots);
  } else {
    return fail(GM_EINVAL, "unknown mode %u", buf->mode);
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(GM_ENOGPU, "no HIP device");
  gm_solver* s = new gm_solver();
  s->d = *d;
  s->mode = buf->mode;
  s->words = (uint32_t*)buf->table;
  s->nslots = buf->table_slots;
  s->view = g.v;
  s->plan_bits = buf->mode == GM_MODE_DENSE ? dense_plan_bits(d, world, buf->flags) : 32;
  s->bits = (u64*)((char*)buf->table + (buf->mode == GM_MODE_DENSE ? dense_words_bytes(d, g, s->plan_bits) : 0));
  s->rank = rank;
  s->world = world;
  s->nblocks = g.nblocks;
  s->comm = nullptr;
  s->tab = (gm_slot*)buf->table;
  s->mask = buf->table_slots - 1;
  s->lv = (u64*)buf->levels;
  s->lcap = buf->level_capacity;
  s->st = (DevState*)buf->scratch;
  s->masks = (const u64*)((char*)buf->scratch + mask_tables_offset(d->max_levels));
  s->bcount = (BlockCount*)((char*)buf->scratch + count_slots_offset(d->max_levels));
  s->flags = buf->flags;
  s->grid = launch_grid();
  if (buf->stream) {
    s->stream = (hipStream_t)buf->stream;
    s->own_stream = false;
  } else {
    hipError_t e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
      delete s;
      return fail(GM_EHIP, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    s->own_stream = true;
  }
  if (s->mode == GM_MODE_DENSE && d->pow2) {
    std::vector<u64> m(kMaskTableWords);
    build_mask_tables(*d, m.data());
    hipError_t e = hipMemcpy((void*)s->masks, m.data(), m.size() * sizeof(u64), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      gm_solver_destroy(s);
      return fail(GM_EHIP, "mask tables: %s", hipGetErrorString(e));
    }
    const ColGeom cg = col_geom(d);
    std::vector<uint32_t> perm;
    if (cg.on) build_colperm(d, cg, perm, s->cstart);
    s->hg = halo_geom(d, world, (u64)(s->view.blk ? s->view.Wl / ((s->view.B + 4) * s->view.Z) : 1));
    size_t off = scratch_bytes_for(d->max_levels);
    const size_t hbytes = s->hg.on ? halo_bytes(s->hg) : 0;
    // scratch: [halo tables + buffers | column permutation | group lists]
    if (cg.on && buf->scratch_bytes >= off + hbytes + col_bytes(d)) {
      uint32_t* dp = (uint32_t*)((char*)buf->scratch + off + hbytes);
      e = hipMemcpy(dp, perm.data(), perm.size() * 4, hipMemcpyHostToDevice);
      if (e != hipSuccess) {
        gm_solver_destroy(s);
        return fail(GM_EHIP, "column permutation: %s", hipGetErrorString(e));
      }
      s->colperm = dp;
      s->cg = cg;
    }
    if (s->hg.on && s->colperm) {
      char* base = (char*)buf->scratch + off;
      auto r = [](size_t b) { return (b + 255) / 256 * 256; };
      std::vector<uint32_t> PB, NY, CS;
      build_halo_cols(*d, s->hg, s->cstart, PB, NY, CS, s->halo_tot);
      uint32_t* pb = (uint32_t*)base;
      uint32_t* ny = (uint32_t*)(base + r(PB.size() * 4));
      uint32_t* cs = (uint32_t*)(base + r(PB.size() * 4) + r(NY.size() * 4));
      e = hipMemcpy(pb, PB.data(), PB.size() * 4, hipMemcpyHostToDevice);
      if (e == hipSuccess) e = hipMemcpy(ny, NY.data(), NY.size() * 4, hipMemcpyHostToDevice);
      if (e == hipSuccess) e = hipMemcpy(cs, CS.data(), CS.size() * 4, hipMemcpyHostToDevice);
      if (e != hipSuccess) {
        gm_solver_destroy(s);
        return fail(GM_EHIP, "halo tables: %s", hipGetErrorString(e));
      }
      s->ht = HaloTabs{pb, ny, cs, s->hg.NG, s->hg.NYn, s->hg.top};
      s->halo_send = (uint32_t*)(base + halo_tab_bytes(s->hg));
      s->halo_recv = s->halo_send + s->hg.nb * 2 * s->hg.Z;
      s->halo16 = d->kind == K_SUM && d->root_sum < 32768;
    } else {
      s->hg.on = false;  // scratch from an older plan: whole-slice halos
    }
    off += hbytes + (s->colperm ? col_bytes(d) : 0);
    const GroupGeom gg = group_geom(d, world);
    const size_t gbytes = gg.on ? (group_entries(d, gg) * 4 + 255) / 256 * 256 : 0;
    if (gg.on && !s->view.blk && buf->scratch_bytes >= off + gbytes) {
      std::vector<uint16_t> gsum;
      group_sums(d, gg, gsum);
      std::vector<uint32_t> list;
      list.reserve(gbytes / 4);
      s->goff.assign((size_t)d->max_levels + 1, 0);
      s->gxcd.assign((size_t)d->max_levels * 9, 0);
      const int top = d->nheaps - 1;
      const u64 C = d->pstride[top] / 256;  // groups per top-digit slice
      bool cols = top >= 2 && d->pstride[top] % 256 == 0 && C >= 8;
      const u64 tile = 0;  // columns per top-major tile (0: the XCD's whole range; tiles measured no gain)
      const u64 NT = cols ? gg.groups / C : 1, NC = cols ? C : gg.groups;
      std::vector<u64> live(NC);
      for (int L = 0; L < d->max_levels; L++) {
        s->goff[L] = list.size();
        u64 tot = 0;
        for (u64 c = 0; c < NC; c++) {
          u64 n = 0;
          for (u64 t = 0; t < NT; t++) n += group_live(d, gg, gsum[c + t * NC], L);
          live[c] = n;
          tot += n;
        }
        // 8 contiguous column ranges of ~equal live count, each walked
        // top-major in tiles of `tile` columns
        u64 c0 = 0, acc = 0;
        for (int x = 0; x < 8; x++) {
          s->gxcd[(size_t)L * 9 + x] = (uint32_t)(list.size() - s->goff[L]);
          u64 c1 = c0;
          const u64 want = tot * (u64)(x + 1) / 8;
          while (c1 < NC && (acc < want || x == 7)) acc += live[c1++];
          const u64 tw = tile ? tile : std::max<u64>(1, c1 - c0);
          for (u64 ta = c0; ta < c1; ta += tw)
            for (u64 t = 0; t < NT; t++)
              for (u64 c = ta; c < std::min(c1, ta + tw); c++)
                if (group_live(d, gg, gsum[c + t * NC], L)) list.push_back((uint32_t)(c + t * NC));
          c0 = c1;
        }
        s->gxcd[(size_t)L * 9 + 8] = (uint32_t)(list.size() - s->goff[L]);
      }
      s->goff[d->max_levels] = list.size();
      uint32_t* dl = (uint32_t*)((char*)buf->scratch + off);
      e = list.empty() ? hipSuccess : hipMemcpy(dl, list.data(), list.size() * 4, hipMemcpyHostToDevice);
      if (e != hipSuccess) {
        gm_solver_destroy(s);
        return fail(GM_EHIP, "group lists: %s", hipGetErrorString(e));
      }
      s->glist = dl;
    }
  }
  if (s->mode == GM_MODE_BUCKETED) {
    char* t = (char*)buf->table;
    s->Pcap = buf->level_capacity;
    s->Ecap = buf->table_slots;
    // a shard of a world > 1 job also holds the md5 exchange buffers (24 B per staged record)
    // (world > 1 also: the local-dedup form's in-edges, another 6 B per edge)
    s->Emax = std::min<u64>((buf->table_bytes - 4 * s->Pcap - (world > 1 ? 12 : 6) * s->Ecap) / (world > 1 ? 48 : 24),
                            0xFFFFFFF0ull);
    s->bkK = (u64*)buf->levels;
    s->bkW = (uint32_t*)t;
    t += (4 * s->Pcap + 7) & ~7ull;
    s->REp = (uint32_t*)t;
    t += 4 * s->Ecap;
    s->REc = (uint16_t*)t;
    t += (2 * s->Ecap + 7) & ~7ull;
    if (world > 1) {
      s->REpl = (uint32_t*)t;
      t += 4 * s->Ecap;
      s->REcl = (uint16_t*)t;
      t += (2 * s->Ecap + 7) & ~7ull;
    }
    // staging: [S1k | S1p | S1f] (the count-free expand writes the first 13
    // Emax bytes of it in its chunked layout, BkChunked) then S2k
    s->S1k = (u64*)t;
    t += 8 * s->Emax;
    s->S1p = (uint32_t*)t;
    t += 4 * s->Emax;
    s->S1f = (uint8_t*)t;  // (4 Emax bytes of the plan; one is used)
    t += 4 * s->Emax;
    s->S2k = (u64*)t;
    t += 8 * s->Emax;
    if (world > 1) {  // md5 exchange: records sent / received (keys, refs; answers reuse the key arrays)
      s->XSk = (u64*)t;
      t += 8 * s->Emax;
      s->XSr = (uint32_t*)t;
      t += 4 * s->Emax;
      s->XRk = (u64*)t;
      t += 8 * s->Emax;
      s->XRr = (uint32_t*)t;
    }
    const BkScratch x = bk_scratch(d->max_levels);
    char* sc = (char*)buf->scratch;
    s->bkL = (BkLevel*)(sc + x.lv);
    s->pbase = (uint32_t*)(sc + x.pbase);
    s->bh = (uint32_t*)(sc + x.bh);
    s->ph = (uint32_t*)(sc + x.ph);
    s->boff = (uint32_t*)(sc + x.boff);
    s->tot = (uint32_t*)(sc + x.tot);
    s->cbase = (uint32_t*)(sc + x.cbase);
    s->bkcur = (uint32_t*)(sc + x.cur);
    s->bkah = (uint32_t*)(sc + x.ah);
    s->bkgc = (uint32_t*)(sc + x.gc);
    s->ucnt = (uint32_t*)(sc + x.ucnt);
    s->bktotal = (u64*)(sc + x.total);
    s->meta = (uint32_t*)(sc + x.meta);
    s->meta_cap = (x.end - x.meta) / 4;
  }
  if (s->mode == GM_MODE_DENSE) {
    int rc = dense_choose(s);
    if (rc) {
      gm_solver_destroy(s);
      return rc;
    }
  }
  if (s->mode == GM_MODE_PLANES) {
    int rc = plane_setup(s, buf);
    if (rc) {
      gm_solver_destroy(s);
      return rc;
    }
  }
  if (s->mode == GM_MODE_RANKED) {
    int rc = rank_setup(s, buf);
    if (rc) {
      gm_solver_destroy(s);
      return rc;
    }
  }
  *out = s;
  return 0;
}

int gm_solver_create(int game, const gm_buffers* buf, gm_solver** out) {
  return gm_solver_create_shard(game, 0, 1, buf, out);
}

int gm_comm_unique_id(void* id_out) {
  if (!id_out) return fail(GM_EINVAL, "null argument");
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return fail(GM_EHIP, "ncclGetUniqueId: %s", ncclGetErrorString(r));
  memcpy(id_out, &id, sizeof id);
  return 0;
}

int gm_solver_comm_init(gm_solver* s, const void* id) {
  if (!s || !id) return fail(GM_EINVAL, "bad argument");
  if (s->world <= 1) return 0;
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof uid);
  ncclComm_t c;
  ncclResult_t r = ncclCommInitRank(&c, s->world, uid, s->rank);
  if (r != ncclSuccess) return fail(GM_EHIP, "ncclCommInitRank: %s", ncclGetErrorString(r));
  s->comm = c;
  if (!s->errg && hipMalloc((void**)&s->errg, (size_t)s->world * sizeof(u64)) != hipSuccess)
    return fail(GM_EHIP, "error-mask gather buffer");
  return 0;
}

static void halo_sigs(const gm_solver* s, u64 L, u64 out[4]);
// host half of a dense shard's halo geometry, as gm_solver_create_shard
// builds it from a gm_plan_shard scratch (column permutation present)
static int shard_host_geom(const Desc* d, int rank, int world, gm_solver* s) {
  DenseGeom g;
  memset(&g, 0, sizeof g);
  int rc = dense_geom(d, rank, world, &g);
  if (rc) return rc;
  s->d = *d;
  s->mode = GM_MODE_DENSE;
  s->view = g.v;
  s->rank = rank;
  s->world = world;
  s->nblocks = g.nblocks;
  s->hg.on = false;
  if (d->pow2) {
    const ColGeom cg = col_geom(d);
    std::vector<uint32_t> perm;
    if (cg.on) build_colperm(d, cg, perm, s->cstart);
    s->hg = halo_geom(d, world, (u64)(s->view.blk ? s->view.Wl / ((s->view.B + 4) * s->view.Z) : 1));
    if (s->hg.on && cg.on) {
      std::vector<uint32_t> PB, NY, CS;
      build_halo_cols(*d, s->hg, s->cstart, PB, NY, CS, s->halo_tot);
      s->halo16 = d->kind == K_SUM && d->root_sum < 32768;
    } else {
      s->hg.on = false;
    }
  }
  return 0;
}

int gm_shard_halo_sigs(int game, int rank, int world, uint32_t flags, uint64_t* out, uint32_t levels) {
  (void)flags;  // the halo geometry does not depend on the kernel families
  const Desc* d = get_game(game);
  if (!d || !out || world < 1 || rank < 0 || rank >= world) return fail(GM_EINVAL, "bad argument");
  if (!d->dense_ok) return fail(GM_EINVAL, "game has no dense layout");
  if (levels < (uint32_t)d->max_levels) return fail(GM_EINVAL, "out holds %u levels, the game has %d", levels, d->max_levels);
  std::unique_ptr<gm_solver> s(new gm_solver());
  int rc = shard_host_geom(d, rank, world, s.get());
  if (rc) return rc;
  for (int L = 0; L < d->max_levels; L++) halo_sigs(s.get(), (u64)L, (u64*)out + (size_t)L * 4);
  return 0;
}

int gm_solver_set_transport(gm_solver* s, gm_xfer_fn fn, void* ctx) {
  if (!s) return fail(GM_EINVAL, "bad argument");
  if ((s->mode != GM_MODE_DENSE && s->mode != GM_MODE_PLANES && s->mode != GM_MODE_BUCKETED &&
       s->mode != GM_MODE_RANKED) || s->world <= 1)
    return fail(GM_EINVAL, "a transport serves dense / planes / bucketed / ranked shards of a world > 1");
  s->xfer = fn;
  s->xfer_ctx = ctx;
  return 0;
}

int gm_solver_set_steps(gm_solver* s, uint32_t first, uint32_t stop) {
  if (!s) return fail(GM_EINVAL, "bad argument");
  const uint32_t n = 2u * (uint32_t)s->d.max_levels;
  if (s->world > 1) return fail(GM_EINVAL, "stop/resume drives one-GPU solves only");
  if (first > n || (stop && (stop <= first || stop > n))) return fail(GM_EINVAL, "bad step range [%u, %u) of %u", first, stop, n);
  s->step_first = first;
  s->step_stop = stop;
  return 0;
}

int gm_solver_set_flags(gm_solver* s, uint32_t flags) {
  if (!s) return fail(GM_EINVAL, "null solver");
  if ((flags & ~GM_F_KERNEL_TIMING) != (s->flags & ~GM_F_KERNEL_TIMING))
    return fail(GM_EINVAL, "only GM_F_KERNEL_TIMING changes after creation: the kernel families and word width "
                           "are fixed by the flags the solver was planned and created with");
  s->flags = flags;
  return 0;
}

void gm_solver_destroy(gm_solver* s) {
  if (!s) return;
  for (hipEvent_t e : s->pev) (void)hipEventDestroy(e);
  if (s->gfwd) (void)hipGraphExecDestroy(s->gfwd);
  if (s->gbwd) (void)hipGraphExecDestroy(s->gbwd);
  for (hipEvent_t e : s->pse)
    if (e) (void)hipEventDestroy(e);
  for (PlaneSlot& q : s->pring) {
    for (hipEvent_t e : q.ev)
      if (e) (void)hipEventDestroy(e);
    if (q.host) (void)hipHostFree(q.host);
  }
  if (s->phost) (void)hipHostFree(s->phost);
  if (s->cstream) (void)hipStreamDestroy(s->cstream);
  if (s->cstream2) (void)hipStreamDestroy(s->cstream2);
  if (s->comm2) (void)ncclCommDestroy(s->comm2);
  if (s->comm) (void)ncclCommDestroy(s->comm);
  if (s->errg) (void)hipFree(s->errg);
  if (s->xdev) (void)hipFree(s->xdev);
  if (s->rlv_dev) (void)hipFree(s->rlv_dev);
  if (s->own_stream) (void)hipStreamDestroy(s->stream);
  delete s;
}

static int solve_dense(gm_solver* s, gm_result* out);
static int solve_bucketed(gm_solver* s, gm_result* out);
static int run_bucketed_shards(std::vector<gm_solver*> ss, gm_result* out);

// Queued one-table PLANES solves: enqueue without waiting, collect later
// (in order).  Solves queued back to back run back to back on the solver's
// stream with no host round trip between them.
int gm_solver_solve_async(gm_solver* s, uint64_t* ticket) {
  if (!s || !ticket) return fail(GM_EINVAL, "bad argument");
  if (s->mode != GM_MODE_PLANES || s->world > 1) return fail(GM_EINVAL, "queued solves: one-table PLANES solvers only");
  if (s->pq_next - s->pq_done >= (u64)kPlaneRing)
    return fail(GM_EINVAL, "%d solves queued: collect one first", kPlaneRing);
  const u64 t = s->pq_next;
  gm_result scratch;
  memset(&scratch, 0, sizeof scratch);
  const int rc = run_planes({s}, &scratch, true);
  if (rc) return rc;
  *ticket = t;
  return 0;
}

int gm_solver_collect(gm_solver* s, uint64_t ticket, gm_result* out) {
  if (!s || !out) return fail(GM_EINVAL, "bad argument");
  memset(out, 0, sizeof *out);
  if (s->mode != GM_MODE_PLANES || s->world > 1) return fail(GM_EINVAL, "queued solves: one-table PLANES solvers only");
  return plane_collect(s, ticket, out);
}

int gm_solver_solve(gm_solver* s, gm_result* out) {
  if (!s || !out) return fail(GM_EINVAL, "bad argument");
  memset(out, 0, sizeof *out);
  if (s->mode == GM_MODE_DENSE) return solve_dense(s, out);
  if (s->mode == GM_MODE_PLANES) return run_planes({s}, out);
  if (s->mode == GM_MODE_RANKED) return s->world > 1 ? run_ranked_shards({s}, out) : run_ranked(s, out);
  if (s->mode == GM_MODE_BUCKETED) return s->world > 1 ? run_bucketed_shards({s}, out) : solve_bucketed(s, out);
  if (s->world > 1) return fail(GM_EINVAL, "keyed-table shard %d/%d: drive it with gm_ks_* (md5 exchange)", s->rank, s->world);
  const int T = s->d.max_levels;
  // steps [first, stop) of the 2T (gm_solver_set_steps); forward level L is
  // step L (level T-1 expands nothing), backward level L is step 2T-1-L
  const int first = (int)s->step_first, stop = s->step_stop ? (int)s->step_stop : 2 * T;
  s->step_first = s->step_stop = 0;
  const bool timing = (s->flags & GM_F_KERNEL_TIMING) && first == 0 && stop == 2 * T;
  std::vector<hipEvent_t> ev;
  auto new_event = [&](hipEvent_t* e) -> int {
    HIPCHK(hipEventCreate(e));
    ev.push_back(*e);
    return 0;
  };
  hipEvent_t e0, e1, e2;
  if (new_event(&e0) || new_event(&e1) || new_event(&e2)) return GM_EHIP;
  std::vector<hipEvent_t> kx, kr;  // per-launch start/stop pairs
  if (timing) {
    kx.resize(2 * (size_t)T);
    kr.resize(2 * (size_t)T);
    for (auto& e : kx)
      if (new_event(&e)) return GM_EHIP;
    for (auto& e : kr)
      if (new_event(&e)) return GM_EHIP;
  }
  auto t0 = std::chrono::steady_clock::now();
  HIPCHK(hipEventRecord(e0, s->stream));
  if (first == 0) {
    // fresh table: keys EMPTY, words NO_WORD
    HIPCHK(hipMemsetAsync(s->tab, 0xFF, (s->mask + 1) * sizeof(gm_slot), s->stream));
    HIPCHK(hipMemsetAsync(s->st, 0, devstate_bytes(T), s->stream));
    hipLaunchKernelGGL(k_seed, dim3(1), dim3(64), 0, s->stream, s->tab, s->mask, s->lv, s->st, s->d.root);
  }
  for (int L = std::max(first, 0); L + 1 < T && L < stop; L++) {
    if (timing) HIPCHK(hipEventRecord(kx[2 * L], s->stream));
    do_expand(s, L);
    if (timing) HIPCHK(hipEventRecord(kx[2 * L + 1], s->stream));
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(64), 0, s->stream, s->st, L, s->lcap);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(e1, s->stream));
  for (int L = T - 1; L >= 0; L--) {
    const int k = 2 * T - 1 - L;
    if (k < first) continue;
    if (k >= stop) break;
    if (timing) HIPCHK(hipEventRecord(kr[2 * L], s->stream));
    do_resolve(s, L);
    if (timing) HIPCHK(hipEventRecord(kr[2 * L + 1], s->stream));
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(e2, s->stream));
  if (stop < 2 * T) {  // stopped early: the state stays on the device for a resume
    HIPCHK(hipStreamSynchronize(s->stream));
    for (auto e : ev) (void)hipEventDestroy(e);
    out->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return GM_PARTIAL;
  }
  hipLaunchKernelGGL(k_root_word, dim3(1), dim3(64), 0, s->stream, s->tab, s->mask, s->d.root, s->st);
  HIPCHK(hipGetLastError());
  std::vector<unsigned char> host(devstate_bytes(T));
  HIPCHK(hipMemcpyAsync(host.data(), s->st, host.size(), hipMemcpyDeviceToHost, s->stream));
  HIPCHK(hipStreamSynchronize(s->stream));
  auto t1 = std::chrono::steady_clock::now();
  const DevState* hs = (const DevState*)host.data();
  const uint32_t word = hs->root_word;
  float f = 0, b = 0;
  HIPCHK(hipEventElapsedTime(&f, e0, e1));
  HIPCHK(hipEventElapsedTime(&b, e1, e2));
  out->ms_forward = f;
  out->ms_backward = b;
  out->ms_total = std::chrono::duration<double, std::milli>(t1 - t0).count();
  if (timing) {
    double sx = 0, sr = 0;
    for (int L = 0; L + 1 < T; L++) {
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, kx[2 * L], kx[2 * L + 1]));
      sx += ms;
    }
    for (int L = 0; L < T; L++) {
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, kr[2 * L], kr[2 * L + 1]));
      sr += ms;
    }
    out->ms_expand_kernels = sx;
    out->ms_resolve_kernels = sr;
    out->n_expand_launches = (uint64_t)(T - 1);
    out->n_resolve_launches = (uint64_t)T;
  }
  for (auto e : ev) (void)hipEventDestroy(e);
  out->positions = hs->cursor_front + hs->cursor_back;
  out->edges = hs->edges;
  out->primitives = hs->prims;
  out->max_level_width = (uint32_t)std::max<u64>(hs->max_width, 1);
  uint32_t lv = 0;
  for (int L = 0; L < T; L++) {
    const LevelSeg& g = hs->seg[L];
    if ((g.fe - g.fb) + (g.c2hi - g.c2lo) > 0) lv++;
  }
  out->levels = lv;
  out->root_word = word;
  if (hs->err) {
    bool full = hs->err & (ERR_TABLE_FULL | ERR_LEVELS_FULL);
    return fail(full ? GM_EFULL : GM_ECORRUPT, "solve failed:%s", err_text(hs->err).c_str());
  }
  if (word == NO_WORD) return fail(GM_ECORRUPT, "root unresolved");
  out->root_value = (int32_t)(word & 3u);
  out->root_remoteness = word >> 2;
  return 0;
}

// the per-block counts summed into the table's totals and the solve's
// reduction words (one block of 1024 threads; also the tail of the PLANES
// finish kernel, k_plane_finish)
__device__ __forceinline__ void fill_red_body(DevState* st, const BlockCount* bc) {
  __shared__ u64 rn[16], re[16];
  u64 sn = 0, se = 0;
  for (int i = (int)threadIdx.x; i < kCountSlots; i += (int)blockDim.x) {
    sn += bc[i].npos;
    se += bc[i].edges;
  }
  for (int o = 32; o > 0; o >>= 1) {
    sn += __shfl_xor(sn, o);
    se += __shfl_xor(se, o);
  }
  if (__lane_id() == 0) {
    rn[threadIdx.x >> 6] = sn;
    re[threadIdx.x >> 6] = se;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    sn = se = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); w++) {
      sn += rn[w];
      se += re[w];
    }
    st->cursor_front += sn;  // this table's totals (gm_solver_positions reads them)
    st->edges += se;
    st->red[0] = st->cursor_front;
    st->red[1] = st->edges;
    st->red[2] = st->prims;
    st->red[3] = st->root_word == NO_WORD ? 0 : (u64)st->root_word + 1;
    st->red[4] = st->err;
  }
}
__global__ __launch_bounds__(1024) void k_fill_red(DevState* st, const BlockCount* bc) { fill_red_body(st, bc); }

// Band of level L: every non-hole slot has digit sum s(p) in [S - H0, S]
// (S = root_sum - L), so its prefix lies between the smallest prefix with
// s >= S - H0 (fill the low digits first) and the largest with s <= S (fill
// the high digits first).  Narrowing a launch to the band skips whole
// stretches of holes at both ends of the tier sequence.  Returns the view
// clipped to the band (64-aligned start) or one with p_lo == p_hi.
static DenseView dense_band(const Desc& d, const DenseView& v, u64 L) {
  const int64_t S = (int64_t)d.root_sum - (int64_t)L;
  int64_t T = S - (int64_t)d.heap[0];
  u64 pmin = 0, pmax = 0;
  int64_t rem = S;
  for (int i = d.nheaps - 1; i >= 1; i--) {
    const int64_t h = std::min<int64_t>(rem, d.heap[i]);
    pmax += (u64)h * d.pstride[i];
    rem -= h;
  }
  for (int i = 1; i < d.nheaps && T > 0; i++) {
    const int64_t h = std::min<int64_t>(T, d.heap[i]);
    pmin += (u64)h * d.pstride[i];
    T -= h;
  }
  DenseView b = v;
  if (S < 0 || T > 0) {  // no slot of this level exists
    b.p_hi = b.p_lo;
    return b;
  }
  b.p_lo = std::max<u64>(v.p_lo, pmin & ~63ull);
  b.p_hi = std::min<u64>(v.p_hi, pmax + 1);
  if (b.p_hi < b.p_lo) b.p_hi = b.p_lo;
  return b;
}

// Halo exchanges of a dense shard group (block layout, DenseView).  Block
// k's bottom two own slices (top values kB, kB+1) are the upper halo of
// block k-1 (reach bits, after the pull); its top two own slices are the
// lower halo of block k+1 (words, after the resolve).  With blocks dealt
// round robin every block of rank r sends to the same neighbour rank
// (r -/+ 1 mod world), in block order, and the receiver walks its blocks in
// the same order.  Only the part of a slice pair inside level L's band
// travels: bits as whole 64-bit words, words packed to their non-hole slots
// (power-of-two tables, k_halo_move) or as the band's 4-B run.  `cs` is the
// stream the copies / RCCL calls run on.  mode: 1 = RCCL (one process per
// GPU), 2 = in-process group (device-to-device copies).

// local slice index of slice o of local block j
static u64 blk_slice(const gm_solver* s, u64 j, u64 o) { return j * (s->view.B + 4) + o; }
// global top value of slice o of local block j
static int64_t blk_top(const gm_solver* s, u64 j, u64 o) {
  return (int64_t)(((u64)s->view.rank + j * s->view.world) * s->view.B + o) - 2;
}
static u64 blk_count(const gm_solver* s) { return s->view.Wl / ((s->view.B + 4) * s->view.Z); }
static u64 blk_global(const gm_solver* s, u64 j) { return (u64)s->view.rank + j * s->view.world; }

// prefixes [lo, hi) (offsets inside the slice pair starting at top value
// t0) of level L's band; false if none
static bool band_pair(const gm_solver* s, u64 L, int64_t t0, u64* lo, u64* hi) {
  const DenseView all{0, ~0ull, 0, 0, 0};
  const DenseView band = dense_band(s->d, all, L);
  const int64_t Z = (int64_t)s->view.Z;
  const int64_t a = std::max<int64_t>(t0 * Z, (int64_t)band.p_lo);
  const int64_t b = std::min<int64_t>((t0 + 2) * Z, (int64_t)std::min<u64>(band.p_hi, (u64)INT64_MAX));
  if (b <= a) return false;
  *lo = (u64)(a - t0 * Z);
  *hi = (u64)(b - t0 * Z);
  return true;
}

static int xfer_call(gm_solver* s, int op, const void* sb, u64 sn, int sp, void* rb, u64 rn, int rp) {
  const int rc = s->xfer(s->xfer_ctx, op, sb, sn, sp, rb, rn, rp);
  return rc ? fail(GM_EHIP, "transport callback failed (%d) on rank %d", rc, s->rank) : 0;
}
// host-staged copy of device ranges into / out of s->hstage
struct HostRange {
  void* dev;
  u64 bytes;
};
static int stage_out(gm_solver* s, const std::vector<HostRange>& rs, u64 at, hipStream_t cs) {
  for (const HostRange& r : rs) {
    HIPCHK(hipMemcpyAsync(s->hstage.data() + at, r.dev, r.bytes, hipMemcpyDeviceToHost, cs));
    at += r.bytes;
  }
  HIPCHK(hipStreamSynchronize(cs));
  return 0;
}
static int stage_in(gm_solver* s, const std::vector<HostRange>& rs, u64 at, hipStream_t cs) {
  for (const HostRange& r : rs) {
    HIPCHK(hipMemcpyAsync(r.dev, s->hstage.data() + at, r.bytes, hipMemcpyHostToDevice, cs));
    at += r.bytes;
  }
  HIPCHK(hipStreamSynchronize(cs));
  return 0;
}
static u64 ranges_bytes(const std::vector<HostRange>& rs) {
  u64 n = 0;
  for (const HostRange& r : rs) n += r.bytes;
  return n;
}
// one paired transfer through the host: send ranges `out` to rank sp, receive
// ranges `in` from rank rp
static int xfer_ranges(gm_solver* s, const std::vector<HostRange>& out, int sp, const std::vector<HostRange>& in, int rp,
                       hipStream_t cs) {
  const u64 ns = ranges_bytes(out), nr = ranges_bytes(in);
  if (s->hstage.size() < ns + nr) s->hstage.resize(ns + nr);
  int rc = stage_out(s, out, 0, cs);
  if (rc) return rc;
  rc = xfer_call(s, GM_XFER_SENDRECV, s->hstage.data(), ns, sp, s->hstage.data() + ns, nr, rp);
  if (rc) return rc;
  return stage_in(s, in, ns, cs);
}

#include "gm_plane_run.h"
#include "gm_ranked.h"
#include "gm_ranked_shard.h"

int gm_rk_shard_stats(gm_solver* s, uint64_t out[2]) {
  if (!s || !out) return fail(GM_EINVAL, "bad argument");
  if (s->mode != GM_MODE_RANKED || s->world < 2 || !s->rko_own) return fail(GM_EINVAL, "not a ranked md5 shard");
  HIPCHK(hipStreamSynchronize(s->stream));
  HIPCHK(hipMemcpy(&out[0], &s->st->ks_cursor, sizeof(u64), hipMemcpyDeviceToHost));
  out[1] = 0;
  for (size_t L = 0; L < s->rko_tot_h.size() / (size_t)s->world; L++) out[1] += s->rko_tot_h[L * s->world + s->rank];
  return 0;
}

int gm_plane_halo_plan(int game, int rank, int world, uint32_t flags, uint64_t* out, uint32_t levels) {
  const Desc* d = get_game(game);
  if (!d || !out || world < 2 || rank < 0 || rank >= world) return fail(GM_EINVAL, "bad argument");
  if (!plane_ok(d, world)) return fail(GM_EINVAL, "game has no planes layout");
  PlaneShape ps;
  int rc = plane_shape(d, rank, world, flags, &ps);
  if (rc) return rc;
  const uint32_t steps = ps.stage_k ? ps.nrows : ps.S + 1;
  if (levels < steps) return fail(GM_EINVAL, "out holds %u steps, the plan has %u", levels, steps);
  memset(out, 0, (size_t)levels * world * 2 * sizeof(uint64_t));
  std::unique_ptr<gm_solver> s(new gm_solver());
  s->world = world;
  s->rank = rank;
  std::vector<uint8_t> lb;
  rc = plane_lists(s.get(), ps, lb);
  if (rc) return rc;
  if (ps.stage_k) {  // staged: step = halo row, to rank + 1 / from rank - 1
    for (uint32_t r = 0; r < ps.nrows; r++) {
      if (rank + 1 < world) out[((size_t)r * world + rank + 1) * 2] = s->psnd_off[r + 1] - s->psnd_off[r];
      if (rank > 0) out[((size_t)r * world + rank - 1) * 2 + 1] = s->prcv_off[r + 1] - s->prcv_off[r];
    }
    return 0;
  }
  for (uint32_t l = 0; l <= ps.S; l++)
    for (int p = 0; p < world; p++) {
      u64 n;
      plane_seg(s->psnd_off, l, world, p, &n);
      out[((size_t)l * world + p) * 2] = n;
      plane_seg(s->prcv_off, l, world, p, &n);
      out[((size_t)l * world + p) * 2 + 1] = n;
    }
  return 0;
}

// after pull(L): bits of every block's bottom two own slices go down
static int exchange_bits(std::vector<gm_solver*>& ss, u64 L, int mode, hipStream_t cs) {
  auto bits_at = [&](gm_solver* s, u64 j, u64 o, u64 off) {
    return s->bits + (L * s->view.Wbl + blk_slice(s, j, o) * s->view.Z + off) / 64;
  };
  if (mode == 3) {  // host-staged: the same ranges, in the same order as the RCCL form
    gm_solver* s = ss[0];
    const int down = (s->rank + s->world - 1) % s->world, up = (s->rank + 1) % s->world;
    const u64 nb = blk_count(s), B = s->view.B;
    std::vector<HostRange> out, in;
    for (u64 j = 0; j < nb; j++) {
      u64 lo, hi;
      if (blk_global(s, j) >= 1 && band_pair(s, L, blk_top(s, j, 2), &lo, &hi)) {
        lo &= ~63ull;
        hi = (hi + 63) & ~63ull;
        out.push_back({bits_at(s, j, 2, lo), (hi - lo) / 8});
      }
      if (blk_global(s, j) + 1 < s->nblocks && band_pair(s, L, blk_top(s, j, B + 2), &lo, &hi)) {
        lo &= ~63ull;
        hi = (hi + 63) & ~63ull;
        in.push_back({bits_at(s, j, B + 2, lo), (hi - lo) / 8});
      }
    }
    return xfer_ranges(s, out, down, in, up, cs);
  }
  if (mode == 1) {
    gm_solver* s = ss[0];
    const int down = (s->rank + s->world - 1) % s->world, up = (s->rank + 1) % s->world;
    const u64 nb = blk_count(s), B = s->view.B;
    RCCL_LIVE(s);
    ncclGroupStart();
    for (u64 j = 0; j < nb; j++) {
      u64 lo, hi;
      if (blk_global(s, j) >= 1 && band_pair(s, L, blk_top(s, j, 2), &lo, &hi)) {  // to block k-1
        lo &= ~63ull;
        hi = (hi + 63) & ~63ull;
        ncclSend(bits_at(s, j, 2, lo), (hi - lo) / 8, ncclUint8, down, s->comm, cs);
      }
    }
    for (u64 j = 0; j < nb; j++) {
      u64 lo, hi;
      if (blk_global(s, j) + 1 < s->nblocks && band_pair(s, L, blk_top(s, j, B + 2), &lo, &hi)) {  // from block k+1
        lo &= ~63ull;
        hi = (hi + 63) & ~63ull;
        ncclRecv(bits_at(s, j, B + 2, lo), (hi - lo) / 8, ncclUint8, up, s->comm, cs);
      }
    }
    ncclResult_t r = ncclGroupEnd();
    if (r != ncclSuccess) return fail(GM_EHIP, "RCCL bits halo: %s", ncclGetErrorString(r));
    return 0;
  }
  const int W = (int)ss.size();
  for (gm_solver* s : ss) {
    const u64 nb = blk_count(s), B = s->view.B;
    for (u64 j = 0; j < nb; j++) {
      const u64 k = blk_global(s, j);
      u64 lo, hi;
      if (k < 1 || !band_pair(s, L, blk_top(s, j, 2), &lo, &hi)) continue;
      gm_solver* dst = ss[(k - 1) % W];
      const u64 jd = (k - 1) / W;
      lo &= ~63ull;
      hi = (hi + 63) & ~63ull;
      HIPCHK(hipMemcpyAsync(bits_at(dst, jd, B + 2, lo), bits_at(s, j, 2, lo), (hi - lo) / 8,
                            hipMemcpyDeviceToDevice, cs));
    }
  }
  return 0;
}

// packed halo helpers: non-hole words of the slice pair whose first slice
// has top value t0 at level L
static uint32_t halo_total(const gm_solver* s, int64_t x) {
  return (x < 0 || x >= s->hg.XN) ? 0u : s->halo_tot[(size_t)x];
}
static uint32_t halo_count(const gm_solver* s, u64 L, int64_t t0) {
  const int64_t x0 = (int64_t)s->d.root_sum - (int64_t)L - t0;
  return halo_total(s, x0) + halo_total(s, x0 - 1);
}
// Pack (send side: every block's top pair, o = B) or unpack (receive side:
// every block's lower halo, o = 0) all of a rank's halo pairs of level L
// between the table and buf; returns the words moved.  Blocks without a
// neighbour on that side are skipped, in the same order on both ends.
static u64 halo_move_all(gm_solver* s, u64 L, int pack, uint32_t* buf, hipStream_t cs) {
  const u64 nb = blk_count(s), B = s->view.B;
  const int64_t S = (int64_t)s->d.root_sum - (int64_t)L;
  const int H0 = (int)s->d.heap[0];
  HaloColJobs J;
  J.n = 0;
  J.cum[0] = 0;
  u64 at = 0;
  auto flush = [&]() {
    if (!J.n) return;
    const u64 units = (u64)J.cum[J.n] * 64;
    const int grid = (int)std::min<u64>(((units + kBlock - 1) / kBlock + 7) & ~7ull, (u64)s->grid);
    uint32_t* lw = s->words + L * s->view.Wl;
    uint16_t* lw16 = (uint16_t*)s->words + L * s->view.Wl;
    if (s->w16) {  // two columns per wave, eight slots per lane
      const u64 u2 = (u64)((J.cum[J.n] + 1) / 2) * 64;
      const int g2 = (int)std::min<u64>(((u2 + kBlock - 1) / kBlock + 7) & ~7ull, (u64)s->grid);
      if (pack)
        hipLaunchKernelGGL((k_halo_cols16<true>), dim3(g2), dim3(kBlock), 0, cs, s->d, J, s->view.Z, s->colperm,
                           s->ht, lw16, (uint16_t*)buf);
      else
        hipLaunchKernelGGL((k_halo_cols16<false>), dim3(g2), dim3(kBlock), 0, cs, s->d, J, s->view.Z, s->colperm,
                           s->ht, lw16, (uint16_t*)buf);
    } else if (pack && s->halo16)
      hipLaunchKernelGGL((k_halo_cols<true, true>), dim3(grid), dim3(kBlock), 0, cs, s->d, J, s->view.Z, s->colperm,
                         s->ht, lw, (void*)buf);
    else if (pack)
      hipLaunchKernelGGL((k_halo_cols<true, false>), dim3(grid), dim3(kBlock), 0, cs, s->d, J, s->view.Z, s->colperm,
                         s->ht, lw, (void*)buf);
    else if (s->halo16)
      hipLaunchKernelGGL((k_halo_cols<false, true>), dim3(grid), dim3(kBlock), 0, cs, s->d, J, s->view.Z, s->colperm,
                         s->ht, lw, (void*)buf);
    else
      hipLaunchKernelGGL((k_halo_cols<false, false>), dim3(grid), dim3(kBlock), 0, cs, s->d, J, s->view.Z,
                         s->colperm, s->ht, lw, (void*)buf);
    J.n = 0;
  };
  for (u64 j = 0; j < nb; j++) {
    const u64 k = blk_global(s, j);
    if (pack ? k + 1 >= s->nblocks : k < 1) continue;
    const u64 o = pack ? B : 0;
    for (u64 m = 0; m < 2; m++) {
      const int64_t t = blk_top(s, j, o + m), x = S - t;
      const uint32_t n = halo_total(s, x);
      if (!n) continue;
      // live columns of slice x: sums gs in [x - heap0 - mj, x]
      const int64_t glo = std::max<int64_t>(0, x - H0 - s->hg.mj), ghi = std::min<int64_t>(x, s->hg.NG - 2);
      const uint32_t ca = s->cstart[(size_t)glo], cb = s->cstart[(size_t)ghi + 1];
      if (J.n == (uint32_t)kMaxHaloColJobs) flush();
      J.lo[J.n] = ca;
      J.u[J.n] = (uint32_t)blk_slice(s, j, o + m);
      J.x[J.n] = (int32_t)x;
      J.base[J.n] = (uint32_t)at;
      J.cum[J.n + 1] = J.cum[J.n] + (cb - ca);
      J.n++;
      at += n;
    }
  }
  flush();
  return at;
}
static u64 halo_recv_count(const gm_solver* s, u64 L) {
  u64 n = 0;
  for (u64 j = 0; j < blk_count(s); j++)
    if (blk_global(s, j) >= 1) n += halo_count(s, L, blk_top(s, j, 0));
  return n;
}
// words halo_move_all packs on the send side (its count, without the kernels)
static u64 halo_send_count(const gm_solver* s, u64 L) {
  u64 n = 0;
  for (u64 j = 0; j < blk_count(s); j++)
    if (blk_global(s, j) + 1 < s->nblocks) n += halo_count(s, L, blk_top(s, j, s->view.B));
  return n;
}

// Fail-fast check of a sharded solve's exchange plan.  Every message of
// every level is fixed by the geometry, so before level 0 each rank
// fingerprints, per level, the ordered byte counts it will send and receive
// for the bits (down) and words (up) halos; the fingerprints are gathered
// and a sender's must equal its receiver's.  A mismatch -- which under RCCL
// would leave a receive of the wrong size waiting forever -- is GM_ECORRUPT
// on every rank at once, before any transfer.
struct SigAcc {
  u64 h = 1469598103934665603ull, n = 0;
  void add(u64 bytes) {
    h = (h ^ bytes) * 1099511628211ull;
    n++;
  }
  u64 get() const { return h ^ (n << 56); }
};
static void halo_sigs(const gm_solver* s, u64 L, u64 out[4]) {
  SigAcc bs, br, ws, wr;
  const u64 nb = blk_count(s), B = s->view.B;
  for (u64 j = 0; j < nb; j++) {
    u64 lo, hi;
    if (blk_global(s, j) >= 1 && band_pair(s, L, blk_top(s, j, 2), &lo, &hi))
      bs.add(((hi + 63) & ~63ull) / 8 - (lo & ~63ull) / 8);
    if (blk_global(s, j) + 1 < s->nblocks && band_pair(s, L, blk_top(s, j, B + 2), &lo, &hi))
      br.add(((hi + 63) & ~63ull) / 8 - (lo & ~63ull) / 8);
  }
  if (s->hg.on) {
    const u64 wb = s->halo16 ? 2 : 4;
    const u64 ns = halo_send_count(s, L), nr = halo_recv_count(s, L);
    if (ns) ws.add(ns * wb);
    if (nr) wr.add(nr * wb);
  } else {
    for (u64 j = 0; j < nb; j++) {
      u64 lo, hi;
      if (blk_global(s, j) + 1 < s->nblocks && band_pair(s, L, blk_top(s, j, B), &lo, &hi)) ws.add((hi - lo) * 4);
      if (blk_global(s, j) >= 1 && band_pair(s, L, blk_top(s, j, 0), &lo, &hi)) wr.add((hi - lo) * 4);
    }
  }
  out[0] = bs.get();
  out[1] = br.get();
  out[2] = ws.get();
  out[3] = wr.get();
}
// all ranks' fingerprints, rank-major [world][T][4]: bits go down (rank r
// sends what r - 1 receives), words go up
static int halo_sigs_match(const std::vector<u64>& all, int world, int T) {
  auto at = [&](int r, int L, int k) { return all[((size_t)r * T + L) * 4 + k]; };
  for (int r = 0; r < world; r++) {
    const int down = (r + world - 1) % world, up = (r + 1) % world;
    for (int L = 0; L < T; L++) {
      if (at(r, L, 0) != at(down, L, 1))
        return fail(GM_ECORRUPT, "bits halo of level %d: rank %d would send what rank %d does not expect", L, r, down);
      if (at(r, L, 2) != at(up, L, 3))
        return fail(GM_ECORRUPT, "words halo of level %d: rank %d would send what rank %d does not expect", L, r, up);
    }
  }
  return 0;
}
// gather every rank's fingerprints and compare (once per solver: the
// geometry never changes)
static int check_halo_plan(std::vector<gm_solver*>& ss, int mode, hipStream_t st) {
  gm_solver* s0 = ss[0];
  if (s0->halo_ok) return 0;
  const int T = s0->d.max_levels, W = s0->world;
  std::vector<u64> all((size_t)W * T * 4);
  if (mode == 2) {
    for (gm_solver* s : ss)
      for (int L = 0; L < T; L++) halo_sigs(s, (u64)L, &all[((size_t)s->rank * T + L) * 4]);
  } else {
    std::vector<u64> mine((size_t)T * 4);
    for (int L = 0; L < T; L++) halo_sigs(s0, (u64)L, &mine[(size_t)L * 4]);
    if (mode == 3) {
      int rc = xfer_call(s0, GM_XFER_ALLGATHER, mine.data(), mine.size() * 8, -1, all.data(), all.size() * 8, -1);
      if (rc) return rc;
    } else {
      void* dev = nullptr;
      HIPCHK(hipMalloc(&dev, (all.size() + mine.size()) * 8));
      u64* dall = (u64*)dev;
      u64* dmine = dall + all.size();
      hipError_t e = hipMemcpyAsync(dmine, mine.data(), mine.size() * 8, hipMemcpyHostToDevice, st);
      ncclResult_t r = ncclSuccess;
      if (s0->gabort && s0->gabort->load(std::memory_order_acquire)) r = ncclInvalidUsage;
      if (e == hipSuccess && r == ncclSuccess) r = ncclAllGather(dmine, dall, mine.size(), ncclUint64, s0->comm, st);
      if (e == hipSuccess && r == ncclSuccess) e = hipMemcpyAsync(all.data(), dall, all.size() * 8, hipMemcpyDeviceToHost, st);
      if (e == hipSuccess) e = hipStreamSynchronize(st);
      (void)hipFree(dev);
      if (r != ncclSuccess) return fail(GM_EHIP, "RCCL allgather of the halo plan: %s", ncclGetErrorString(r));
      if (e != hipSuccess) return fail(GM_EHIP, "halo plan: %s", hipGetErrorString(e));
    }
  }
  int rc = halo_sigs_match(all, W, T);
  if (rc) return rc;
  for (gm_solver* s : ss) s->halo_ok = true;
  return 0;
}

// after resolve(L): words of every block's top two own slices go up.
// Power-of-two tables send only the non-hole words (about a fifth of the
// two slices, averaged over the levels).
static int exchange_words(std::vector<gm_solver*>& ss, u64 L, int mode, hipStream_t cs) {
  bool packed = true;
  for (gm_solver* s : ss) packed = packed && s->hg.on;
  auto words_at = [&](gm_solver* s, u64 j, u64 o, u64 off) {
    return s->words + L * s->view.Wl + blk_slice(s, j, o) * s->view.Z + off;
  };
  if (mode == 3) {  // host-staged: the RCCL form's buffers and order
    gm_solver* s = ss[0];
    const int down = (s->rank + s->world - 1) % s->world, up = (s->rank + 1) % s->world;
    const u64 nb = blk_count(s), B = s->view.B;
    std::vector<HostRange> out, in;
    u64 nrecv = 0;
    if (packed) {
      const u64 wb = s->halo16 ? 2 : 4;
      const u64 nsend = halo_move_all(s, L, 1, s->halo_send, cs);
      HIPCHK(hipGetLastError());
      nrecv = halo_recv_count(s, L);
      if (nsend) out.push_back({s->halo_send, nsend * wb});
      if (nrecv) in.push_back({s->halo_recv, nrecv * wb});
    } else {
      for (u64 j = 0; j < nb; j++) {
        u64 lo, hi;
        if (blk_global(s, j) + 1 < s->nblocks && band_pair(s, L, blk_top(s, j, B), &lo, &hi))
          out.push_back({words_at(s, j, B, lo), (hi - lo) * 4});
        if (blk_global(s, j) >= 1 && band_pair(s, L, blk_top(s, j, 0), &lo, &hi))
          in.push_back({words_at(s, j, 0, lo), (hi - lo) * 4});
      }
    }
    int rc = xfer_ranges(s, out, up, in, down, cs);
    if (rc) return rc;
    if (packed && nrecv) halo_move_all(s, L, 0, s->halo_recv, cs);
    HIPCHK(hipGetLastError());
    return 0;
  }
  if (mode == 1) {
    gm_solver* s = ss[0];
    const int down = (s->rank + s->world - 1) % s->world, up = (s->rank + 1) % s->world;
    const u64 nb = blk_count(s), B = s->view.B;
    RCCL_LIVE(s);
    if (packed) {
      const u64 nsend = halo_move_all(s, L, 1, s->halo_send, cs);
      const u64 nrecv = halo_recv_count(s, L);
      ncclGroupStart();
      const u64 wb = s->halo16 ? 2 : 4;  // bytes per packed word
      if (nsend) ncclSend(s->halo_send, nsend * wb, ncclUint8, up, s->comm, cs);
      if (nrecv) ncclRecv(s->halo_recv, nrecv * wb, ncclUint8, down, s->comm, cs);
      ncclResult_t r = ncclGroupEnd();
      if (r != ncclSuccess) return fail(GM_EHIP, "RCCL words halo: %s", ncclGetErrorString(r));
      if (nrecv) halo_move_all(s, L, 0, s->halo_recv, cs);
      HIPCHK(hipGetLastError());
      return 0;
    }
    ncclGroupStart();
    for (u64 j = 0; j < nb; j++) {
      u64 lo, hi;
      if (blk_global(s, j) + 1 < s->nblocks && band_pair(s, L, blk_top(s, j, B), &lo, &hi))
        ncclSend(words_at(s, j, B, lo), (hi - lo) * 4, ncclUint8, up, s->comm, cs);
    }
    for (u64 j = 0; j < nb; j++) {
      u64 lo, hi;
      if (blk_global(s, j) >= 1 && band_pair(s, L, blk_top(s, j, 0), &lo, &hi))
        ncclRecv(words_at(s, j, 0, lo), (hi - lo) * 4, ncclUint8, down, s->comm, cs);
    }
    ncclResult_t r = ncclGroupEnd();
    if (r != ncclSuccess) return fail(GM_EHIP, "RCCL words halo: %s", ncclGetErrorString(r));
    return 0;
  }
  const int W = (int)ss.size();
  if (packed) {
    // every block of shard g sends to shard g + 1 (mod W): pack straight
    // into the receiver's buffer, then unpack there -- the RCCL path's
    // kernels and order, with the transfer left out
    for (int g = 0; g < W; g++) {
      gm_solver* dst = ss[(g + 1) % W];
      const u64 n = halo_move_all(ss[g], L, 1, dst->halo_recv, cs);
      // the RCCL path posts a receive of halo_recv_count words for the
      // sender's count: a mismatch would hang it, so the group checks it
      if (n != halo_recv_count(dst, L))
        return fail(GM_ECORRUPT, "halo count mismatch at level %llu: shard %d packs %llu, shard %d expects %llu",
                    (unsigned long long)L, g, (unsigned long long)n, (g + 1) % W,
                    (unsigned long long)halo_recv_count(dst, L));
      if (n) halo_move_all(dst, L, 0, dst->halo_recv, cs);
    }
    HIPCHK(hipGetLastError());
    return 0;
  }
  for (gm_solver* s : ss) {
    const u64 nb = blk_count(s), B = s->view.B;
    for (u64 j = 0; j < nb; j++) {
      const u64 k = blk_global(s, j);
      if (k + 1 >= s->nblocks) continue;
      gm_solver* dst = ss[(k + 1) % W];
      const u64 jd = (k + 1) / W;
      const int64_t t0 = blk_top(s, j, B);
      u64 lo, hi;
      if (!band_pair(s, L, t0, &lo, &hi)) continue;
      HIPCHK(hipMemcpyAsync(words_at(dst, jd, 0, lo), words_at(s, j, B, lo), (hi - lo) * 4,
                            hipMemcpyDeviceToDevice, cs));
    }
  }
  HIPCHK(hipGetLastError());
  return 0;
}

// Dense solve of one table (world 1), one shard of an RCCL job, or every
// shard of an in-process group (all on one stream), level-synchronously.
static int run_dense(std::vector<gm_solver*> ss, gm_result* out) {
  gm_solver* s0 = ss[0];
  const Desc& d = s0->d;
  const int T = d.max_levels;
  // 0: one table; 1: one shard per process over RCCL; 2: in-process group;
  // 3: one shard per process over a host-staged transport
  const int mode = s0->world <= 1 ? 0 : ss.size() != 1 ? 2 : s0->xfer ? 3 : 1;
  if (mode == 1 && !s0->comm) return fail(GM_EINVAL, "shard %d/%d has no communicator (gm_solver_comm_init)", s0->rank, s0->world);
  if (mode == 2) {
    if ((int)ss.size() != s0->world) return fail(GM_EINVAL, "group solve needs all %d shards", s0->world);
    for (size_t g = 0; g < ss.size(); g++)
      if (ss[g]->rank != (int)g || ss[g]->stream != s0->stream || ss[g]->mode != GM_MODE_DENSE)
        return fail(GM_EINVAL, "group shards must be ranks 0..n-1 on one stream");
  }
  // steps [first, stop) (gm_solver_set_steps, world 1 only): forward level L
  // is step L, backward level L is step 2T-1-L
  const int first = mode == 0 ? (int)s0->step_first : 0;
  const int stop = mode == 0 && s0->step_stop ? (int)s0->step_stop : 2 * T;
  s0->step_first = s0->step_stop = 0;
  const bool timing = (s0->flags & GM_F_KERNEL_TIMING) && first == 0 && stop == 2 * T;
  hipStream_t st = s0->stream;
  // the kernel families and word width were fixed at creation (dense_choose);
  // a resume checks the interrupted solve used the same width
  for (gm_solver* s : ss) {
    s->launch_err = false;
    if (first > 0) {
      uint32_t wb = 0;
      HIPCHK(hipMemcpy(&wb, &s->st->word_bits, sizeof wb, hipMemcpyDeviceToHost));
      if (wb != 8 && wb != 16 && wb != 32) return fail(GM_EINVAL, "resume: scratch holds no solve in progress");
      if (wb != s->wbits())
        return fail(GM_EINVAL, "resume: the interrupted solve used %u-bit words, this solver %u", wb, s->wbits());
    }
  }
  std::vector<hipEvent_t> ev;
  auto new_event = [&](hipEvent_t* e) -> int {
    HIPCHK(hipEventCreate(e));
    ev.push_back(*e);
    return 0;
  };
  hipEvent_t e0, e1, e2;
  if (new_event(&e0) || new_event(&e1) || new_event(&e2)) return GM_EHIP;
  std::vector<hipEvent_t> kx, kr;  // per-level kernel start/stop (shard 0's launches)
  if (timing) {
    kx.resize(2 * (size_t)T);
    kr.resize(2 * (size_t)T);
    for (auto& e : kx)
      if (new_event(&e)) return GM_EHIP;
    for (auto& e : kr)
      if (new_event(&e)) return GM_EHIP;
  }
  const u64 root_p = d.root / d.base[0];  // global prefix of the root (level 0)
  // launches cover only the level's band of prefixes (dense_band); the
  // grid is a multiple of 8 blocks for the XCD-chunked kernels
  auto grid_of = [&](gm_solver* s, const DenseView& b) {
    const u64 blocks = (b.p_hi - b.p_lo + kBlock - 1) / kBlock;
    return (int)std::min<u64>((blocks + 7) & ~7ull, (u64)s->grid);
  };
  auto t0 = std::chrono::steady_clock::now();
  // Sharded solves overlap each level's halo exchange with compute: a
  // level's launch is split into the part whose parents (pull) / children
  // (resolve) lie inside the shard's own block -- which includes the two
  // slices the exchange sends -- and the two boundary slices that read the
  // halo.  Per level: own part -> event -> exchange on the comm stream ->
  // event; the boundary part of the NEXT level waits for that exchange.  A
  // block narrower than 4 top values has no such split: exchange in order.
  bool pipe = mode == 1 || mode == 2;  // the host-staged transport runs in order
  for (gm_solver* s : ss)
    if (s->view.B < 4) pipe = false;
  if (s0->flags & GM_F_SHARD_INORDER) pipe = false;  // A/B: exchange in order
  hipStream_t cs = st;
  hipEvent_t* E = nullptr;  // [0, T): own part done, [T, 2T): exchange done (forward); reused backward
  if (pipe) {
    if (!s0->cstream) HIPCHK(hipStreamCreateWithFlags(&s0->cstream, hipStreamNonBlocking));
    while (s0->pev.size() < 2 * (size_t)T) {
      hipEvent_t e;
      HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      s0->pev.push_back(e);
    }
    cs = s0->cstream;
    E = s0->pev.data();
  }
  // the launch view of level L: world 1 sweeps the level's band; a shard
  // sweeps its whole local range, processing the own slices o in [olo, ohi)
  // of every block
  int slow = 0;  // largest digit sum of the prefix digits below the top
  for (int i = 1; i + 1 < d.nheaps; i++) slow += (int)d.heap[i];
  auto level_view = [&](gm_solver* s, int L, uint32_t olo, uint32_t ohi) {
    if (!s->view.blk) return dense_band(d, s->view, (u64)L);
    // a shard sweeps only the listed slices of its blocks that hold a
    // non-hole at level L: top value t with 0 <= S - t <= slow + heap0
    DenseView c = s->view;
    c.olo = olo;
    c.ohi = ohi;
    const int64_t S = (int64_t)d.root_sum - L;
    uint32_t n = 0;
    bool over = false;
    for (u64 j = 0; j < blk_count(s); j++)
      for (uint32_t o = olo; o < ohi; o++) {
        const int64_t t = blk_top(s, j, o);
        if (t < 0 || (u64)t >= c.E || S - t < 0 || S - t > slow + (int64_t)d.heap[0]) continue;
        if (n == (uint32_t)kMaxSweepSlices || t > 0xFFFF || blk_slice(s, j, o) > 0xFFFF) {
          over = true;
        } else {
          c.sl[n] = (uint16_t)blk_slice(s, j, o);
          c.st[n++] = (uint16_t)t;
        }
      }
    c.p_lo = 0;
    if (over) {  // too many to list: sweep everything, filter per wave
      c.nsl = 0;
      c.p_hi = c.Wl;
    } else {
      c.nsl = n;
      c.p_hi = (u64)n * c.Z;
    }
    return c;
  };
  if (mode != 0) {
    int rc = check_halo_plan(ss, mode, st);
    if (rc) return rc;
  }
  // Tail runs (one table, whole solves, live-group lists, 8-bit words): the
  // levels at both ends whose live groups fit a workgroup in a pass or two
  // run as one single-workgroup launch each (k_dense_pull_tail,
  // k_dense_resolve16_tail).  A kernel-timing solve keeps one launch per
  // level, so per-launch figures (bench roofline, PMC passes of a timed solve)
  // describe the per-level kernels alone.
  const bool tails = mode == 0 && !timing && first == 0 && stop == 2 * T && s0->glist && !s0->view.blk &&
                     s0->pk == PK_WORDS && s0->w8 && d.pow2;
  int pa = 0, pb = T, ra = T, rb = 0;  // per-level pulls [pa, pb); per-level resolves [rb, ra)
  TailRun pull_head{}, pull_end{}, res_head{}, res_end{};
  if (tails) {
    auto groups = [&](int L) { return s0->goff[(size_t)L + 1] - s0->goff[(size_t)L]; };
    auto add = [&](TailRun& R, int L) {
      R.L[R.n] = (uint32_t)L;
      R.off[R.n] = (uint32_t)s0->goff[(size_t)L];
      R.cnt[R.n] = (uint32_t)groups(L);
      R.phi[R.n] = dense_band(d, s0->view, (u64)L).p_hi;
      R.n++;
    };
    while (pa < T && pa < kTailMax && groups(pa) <= kTailPullGroups) add(pull_head, pa++);
    while (pb > pa && T - pb < kTailMax && groups(pb - 1) <= kTailPullGroups) pb--;
    for (int L = pb; L < T; L++) add(pull_end, L);
    while (ra > 0 && T - ra < kTailMax && groups(ra - 1) <= kTailResolveGroups) add(res_head, --ra);
    while (rb < ra && rb < kTailMax && groups(rb) <= kTailResolveGroups) rb++;
    for (int L = rb - 1; L >= 0; L--) add(res_end, L);
  }
  // forward (pull): level 0 .. T-1, each level's bitmap written exactly once.
  // Parents are one or two top values ABOVE: the boundary is the top two
  // slices [b-2, b), whose parents sit in the halo [b, b+2) sent down by the
  // rank above.
  auto issue_forward = [&]() -> int {
  if (first == 0) {
    for (gm_solver* s : ss) {
      HIPCHK(hipMemsetAsync(s->st, 0, devstate_bytes(T), st));
      HIPCHK(hipMemsetAsync(s->bcount, 0, kCountSlots * sizeof(BlockCount), st));
      HIPCHK(hipMemsetD32Async((hipDeviceptr_t)&s->st->word_bits, (int)s->wbits(), 1, st));
    }
  }
  dense_launch_tail(s0, pull_head, true, root_p);
  for (int L = first; L < T && L < stop; L++) {
    if (L < pa || L >= pb) continue;  // in a tail run
    if (timing) HIPCHK(hipEventRecord(kx[2 * L], st));
    for (gm_solver* s : ss) {
      const uint32_t B = s->view.B;  // pull: the top two own slices read the upper halo
      const DenseView own = level_view(s, L, 2, pipe ? B : B + 2);
      if (own.p_hi > own.p_lo) dense_launch_pull(s, own, grid_of(s, own), (u64)L, root_p);
    }
    if (mode) {
      if (pipe) {
        HIPCHK(hipEventRecord(E[L], st));
        HIPCHK(hipStreamWaitEvent(cs, E[L], 0));
      }
      int rc = exchange_bits(ss, (u64)L, mode, cs);
      if (rc) return rc;
      if (pipe) {
        HIPCHK(hipEventRecord(E[T + L], cs));
        if (L >= 1) HIPCHK(hipStreamWaitEvent(st, E[T + L - 1], 0));  // halos of L-1 (L-2 waited before)
        for (gm_solver* s : ss) {
          const DenseView bd = level_view(s, L, s->view.B, s->view.B + 2);
          if (bd.p_hi > bd.p_lo) dense_launch_pull(s, bd, grid_of(s, bd), (u64)L, root_p);
        }
      }
    }
    if (timing) HIPCHK(hipEventRecord(kx[2 * L + 1], st));
  }
  dense_launch_tail(s0, pull_end, true, root_p);
  HIPCHK(hipGetLastError());
  return 0;
  };
  // backward (resolve): children are one or two top values BELOW: the
  // boundary is the bottom two slices [a, a+2), whose children sit in the
  // halo [a-2, a) sent up by the rank below.
  auto issue_backward = [&]() -> int {
  dense_launch_tail(s0, res_head, false, root_p);
  for (int L = T - 1; L >= 0; L--) {
    if (2 * T - 1 - L < first) continue;
    if (2 * T - 1 - L >= stop) break;
    if (L >= ra || L < rb) continue;  // in a tail run
    if (timing) HIPCHK(hipEventRecord(kr[2 * L], st));
    for (gm_solver* s : ss) {
      const uint32_t B = s->view.B;  // resolve: the bottom two own slices read the lower halo
      const DenseView own = level_view(s, L, pipe ? 4 : 2, B + 2);
      if (own.p_hi > own.p_lo) dense_launch_resolve(s, own, grid_of(s, own), (u64)L);
    }
    if (mode) {
      if (pipe) {
        HIPCHK(hipEventRecord(E[L], st));
        HIPCHK(hipStreamWaitEvent(cs, E[L], 0));
      }
      int rc = exchange_words(ss, (u64)L, mode, cs);
      if (rc) return rc;
      if (pipe) {
        HIPCHK(hipEventRecord(E[T + L], cs));
        if (L + 1 < T) HIPCHK(hipStreamWaitEvent(st, E[T + L + 1], 0));  // halos of L+1 (L+2 waited before)
        for (gm_solver* s : ss) {
          const DenseView bd = level_view(s, L, 2, 4);
          if (bd.p_hi > bd.p_lo) dense_launch_resolve(s, bd, grid_of(s, bd), (u64)L);
        }
      }
    }
    if (timing) HIPCHK(hipEventRecord(kr[2 * L + 1], st));
  }
  dense_launch_tail(s0, res_end, false, root_p);
  HIPCHK(hipGetLastError());
  return 0;
  };
  // GM_F_GRAPH: one-table full solves replay HIP graphs of these launches,
  // captured on the first such solve of the solver (every argument -- level
  // views, group lists, XCD shares, tail runs, grids -- is fixed when the
  // solver is made), so the host enqueues two graph launches instead of ~350
  // kernels.  Measured on the bench workload: 4.47-4.49 ms against
  // 4.44-4.48 ms with plain launches (the host already runs ahead of the
  // GPU; what remains between levels is the device-side kernel boundary), so
  // it is not the default.
  const bool graphed = (s0->flags & GM_F_GRAPH) && mode == 0 && !timing && first == 0 && stop == 2 * T;
  if (graphed && !s0->gfwd) {
    auto capture = [&](auto&& issue, hipGraphExec_t* exec) -> int {
      hipGraph_t g = nullptr;
      HIPCHK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
      const int rc = issue();
      const hipError_t e = hipStreamEndCapture(st, &g);
      if (rc || e != hipSuccess || s0->launch_err) {
        if (g) (void)hipGraphDestroy(g);
        return rc ? rc : e != hipSuccess ? fail(GM_EHIP, "graph capture: %s", hipGetErrorString(e)) : 0;
      }
      const hipError_t ei = hipGraphInstantiate(exec, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      if (ei != hipSuccess) {
        *exec = nullptr;
        return fail(GM_EHIP, "graph instantiate: %s", hipGetErrorString(ei));
      }
      return 0;
    };
    int rc = capture(issue_forward, &s0->gfwd);
    if (!rc) rc = capture(issue_backward, &s0->gbwd);
    if (rc || !s0->gfwd || !s0->gbwd) {  // a launch error is reported by the plain path below
      if (s0->gfwd) (void)hipGraphExecDestroy(s0->gfwd);
      if (s0->gbwd) (void)hipGraphExecDestroy(s0->gbwd);
      s0->gfwd = s0->gbwd = nullptr;
      s0->launch_err = false;
      if (rc) return rc;
    }
  }
  const bool replay = graphed && s0->gfwd && s0->gbwd;
  HIPCHK(hipEventRecord(e0, st));
  if (replay) {
    HIPCHK(hipGraphLaunch(s0->gfwd, st));
  } else {
    const int rc = issue_forward();
    if (rc) return rc;
  }
  if (pipe) {  // the backward pass reuses the events: drain the forward exchanges first
    HIPCHK(hipEventRecord(E[0], cs));
    HIPCHK(hipStreamWaitEvent(st, E[0], 0));
  }
  HIPCHK(hipEventRecord(e1, st));
  if (replay) {
    HIPCHK(hipGraphLaunch(s0->gbwd, st));
  } else {
    const int rc = issue_backward();
    if (rc) return rc;
  }
  if (pipe) {  // every exchange done before the reduction and the host read-back
    HIPCHK(hipEventRecord(E[0], cs));
    HIPCHK(hipStreamWaitEvent(st, E[0], 0));
  }
  HIPCHK(hipEventRecord(e2, st));
  if (stop < 2 * T) {  // stopped early (world 1): the state stays on the device for a resume
    HIPCHK(hipStreamSynchronize(st));
    for (auto e : ev) (void)hipEventDestroy(e);
    out->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    out->word_bits = s0->wbits();
    return GM_PARTIAL;
  }
  for (gm_solver* s : ss) {
    uint64_t root_q = ~0ull;
    if (!dense_local(s->view, root_p, &root_q)) root_q = ~0ull;
    hipLaunchKernelGGL(k_dense_root, dim3(1), dim3(64), 0, st, s->view, s->words, s->bits, root_q, s->st, s->wbits());
    hipLaunchKernelGGL(k_fill_red, dim3(1), dim3(1024), 0, st, s->st, s->bcount);
  }
  if (mode == 1) {  // counts and root word summed; every rank's error mask gathered, OR-ed on the host
    RCCL_LIVE(s0);
    ncclGroupStart();
    ncclResult_t r = ncclAllReduce(s0->st->red, s0->st->red, 4, ncclUint64, ncclSum, s0->comm, st);
    ncclResult_t r2 = ncclAllGather(s0->st->red + 4, s0->errg, 1, ncclUint64, s0->comm, st);
    ncclResult_t r3 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess || r3 != ncclSuccess)
      return fail(GM_EHIP, "RCCL allreduce: %s", ncclGetErrorString(r != ncclSuccess ? r : r2 != ncclSuccess ? r2 : r3));
  }
  // totals (host): RCCL has already reduced red[] across ranks; a group and
  // the host-staged transport reduce here (counts summed, error masks OR-ed)
  u64 red[5] = {0, 0, 0, 0, 0};
  for (gm_solver* s : ss) {
    u64 r[5];
    HIPCHK(hipMemcpyAsync(r, s->st->red, sizeof r, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (mode == 3) {
      std::vector<u64> all((size_t)5 * s->world);
      int rc = xfer_call(s, GM_XFER_ALLGATHER, r, sizeof r, -1, all.data(), all.size() * 8, -1);
      if (rc) return rc;
      for (int g = 0; g < s->world; g++)
        for (int i = 0; i < 5; i++) red[i] = (i == 4) ? (red[i] | all[(size_t)g * 5 + i]) : red[i] + all[(size_t)g * 5 + i];
      continue;
    }
    if (mode == 1) {
      std::vector<u64> e((size_t)s->world);
      HIPCHK(hipMemcpy(e.data(), s->errg, e.size() * sizeof(u64), hipMemcpyDeviceToHost));
      r[4] = 0;
      for (u64 x : e) r[4] |= x;
    }
    for (int i = 0; i < 5; i++) red[i] = (i == 4) ? (red[i] | r[i]) : red[i] + r[i];
  }
  auto t1 = std::chrono::steady_clock::now();
  float f = 0, b = 0;
  HIPCHK(hipEventElapsedTime(&f, e0, e1));
  HIPCHK(hipEventElapsedTime(&b, e1, e2));
  out->ms_forward = f;
  out->ms_backward = b;
  out->ms_total = std::chrono::duration<double, std::milli>(t1 - t0).count();
  if (timing) {
    double sx = 0, sr = 0;
    for (int L = 0; L < T; L++) {
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, kx[2 * L], kx[2 * L + 1]));
      sx += ms;
      HIPCHK(hipEventElapsedTime(&ms, kr[2 * L], kr[2 * L + 1]));
      sr += ms;
    }
    out->ms_expand_kernels = sx;
    out->ms_resolve_kernels = sr;
    out->n_expand_launches = (uint64_t)T;
    out->n_resolve_launches = (uint64_t)T;
  }
  for (auto e : ev) (void)hipEventDestroy(e);
  out->positions = red[0];
  out->edges = red[1];
  out->primitives = red[2];
  out->levels = (uint32_t)T;
  out->max_level_width = 0;
  out->word_bits = s0->wbits();
  out->kernels = s0->rk | (s0->pk << 16);
  for (gm_solver* s : ss)
    if (s->launch_err) return fail(GM_ECORRUPT, "a level found no resolve kernel of the table's word width");
  const uint32_t word = red[3] ? (uint32_t)(red[3] - 1) : NO_WORD;
  out->root_word = word;
  if (red[4]) return fail(GM_ECORRUPT, "solve failed:%s", err_text((uint32_t)red[4]).c_str());
  if (word == NO_WORD) return fail(GM_ECORRUPT, "root unresolved");
  out->root_value = (int32_t)(word & 3u);
  out->root_remoteness = word >> 2;
  return 0;
}

static int solve_dense(gm_solver* s, gm_result* out) { return run_dense({s}, out); }

// ---------------------------------------------------------------------------
// BUCKETED solve (gm_bucketed.h).  Steps as in the other layouts: forward
// step L (L < T - 1) builds level L + 1 from level L; backward step
// 2T - 1 - L resolves level L.  The host reads back two small arrays per
// forward level (partition sizes, then the level's unique count) to size
// the next launches and check capacities BEFORE any kernel writes past
// them; the backward pass is enqueued without host round trips.
// ---------------------------------------------------------------------------
static uint32_t bitlen64(u64 x) { return x ? 64u - (uint32_t)__builtin_clzll(x) : 0u; }
// parent-range geometry of a level of n positions (B3-B5): coarse ranges
// index >> pshift (< 256 of them), fine ranges index >> fb (<= 2^13 parents,
// <= 256 per coarse range)
static bool bk_ranges(u64 n, uint32_t* pshift, uint32_t* fb) {
  const uint32_t bl = bitlen64(n ? n - 1 : 0);
  *pshift = bl > 8 ? bl - 8 : 0;
  *fb = std::min<uint32_t>(*pshift, (uint32_t)kBkRangeBits);
  return *pshift - *fb <= (uint32_t)kBkMaxFineBits;
}
}  // extern "C"
// the bucketed kernels' instantiation for a descriptor (fixed_kind: the
// compile-time toot boards where one exists)
template <class Fn>
static void bk_dispatch(const Desc& d, Fn&& fn) {
  switch (fixed_kind(d)) {
    case K_TTT: fn(std::integral_constant<int, K_TTT>{}); break;
    case K_TOOT_6x4: fn(std::integral_constant<int, K_TOOT_6x4>{}); break;
    case K_TOOT_5x4: fn(std::integral_constant<int, K_TOOT_5x4>{}); break;
    case K_TOOT_4x4: fn(std::integral_constant<int, K_TOOT_4x4>{}); break;
    case K_TOOT: fn(std::integral_constant<int, K_TOOT>{}); break;
    default: fn(std::integral_constant<int, K_OTHELLO>{}); break;
  }
}
extern "C" {
#define BK_KIND_LAUNCH(KERNEL, GRID, BLOCK, S, ...)                                                      \
  bk_dispatch((S)->d, [&](auto kind_) {                                                                  \
    constexpr int K_ = decltype(kind_)::value;                                                           \
    hipLaunchKernelGGL(KERNEL<K_>, dim3(GRID), dim3(BLOCK), 0, (S)->stream, __VA_ARGS__);               \
  })

// parents per expand round for a mean branching avg: the round's children
// should fill about 3/4 of the 8192-record stage (whole waves, 256..4096)
static uint32_t bk_ppr(double avg) {
  const double p = 0.75 * kBkExpandCap / std::max(avg, 0.25);
  return (uint32_t)std::min<double>(4.0 * kBkExpandThreads, std::max<double>(256.0, std::floor(p / 64.0) * 64.0));
}

static int solve_bucketed(gm_solver* s, gm_result* out) {
  const Desc& d = s->d;
  const int T = d.max_levels;
  const int first = (int)s->step_first, stop = s->step_stop ? (int)s->step_stop : 2 * T;
  s->step_first = s->step_stop = 0;
  const bool timing = (s->flags & GM_F_KERNEL_TIMING) && first == 0 && stop == 2 * T;
  hipStream_t st = s->stream;
  std::vector<hipEvent_t> ev;
  auto new_event = [&](hipEvent_t* e) -> int {
    HIPCHK(hipEventCreate(e));
    ev.push_back(*e);
    return 0;
  };
  auto cleanup = [&]() {
    for (auto e : ev) (void)hipEventDestroy(e);
    ev.clear();
  };
  hipEvent_t e0, e1, e2;
  if (new_event(&e0) || new_event(&e1) || new_event(&e2)) return GM_EHIP;
  // kernel-time spans (timing): [start, stop, forward?]
  struct Span {
    hipEvent_t a, b;
    bool fwd;
  };
  std::vector<Span> spans;
  u64 nfwd = 0, nbwd = 0;
  auto span = [&](bool fwd) -> hipEvent_t* {  // opens a span; returns its stop event to record later
    if (!timing) return nullptr;
    Span x{};
    x.fwd = fwd;
    if (new_event(&x.a) || new_event(&x.b)) return nullptr;
    if (hipEventRecord(x.a, st) != hipSuccess) return nullptr;
    spans.push_back(x);
    return &spans.back().b;
  };
  auto span_end = [&](hipEvent_t* b) -> int {
    if (b) HIPCHK(hipEventRecord(*b, st));
    return 0;
  };
  int rc = 0;
  auto bail = [&](int code) {
    (void)hipStreamSynchronize(st);
    cleanup();
    return code;
  };
  auto t0 = std::chrono::steady_clock::now();
  HIPCHK(hipEventRecord(e0, st));
  std::vector<BkLevel>& lv = s->lvh;
  if (first == 0) {
    HIPCHK(hipMemsetAsync(s->st, 0, devstate_bytes(T), st));
    HIPCHK(hipMemsetAsync(s->bkL, 0, sizeof(BkLevel) * (size_t)T, st));
    lv.assign((size_t)T, BkLevel{});
    lv[0].n = 1;
    HIPCHK(hipMemcpyAsync(s->bkK, &s->d.root, sizeof(u64), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(s->bkL, lv.data(), sizeof(BkLevel), hipMemcpyHostToDevice, st));
  } else {
    lv.assign((size_t)T, BkLevel{});
    HIPCHK(hipMemcpyAsync(lv.data(), s->bkL, sizeof(BkLevel) * (size_t)T, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  std::vector<uint32_t> htot(2 * kBkC);
  std::vector<std::vector<uint32_t>> keep;  // host arrays of async H2D copies, alive until the end
  uint32_t herr = 0;
  // ---- forward ----
  for (int L = first; L < T && L < stop; L++) {
    if (L + 1 >= T) continue;  // the last level expands nothing (backward checks it holds only primitives)
    BkLevel& P = lv[(size_t)L];
    BkLevel& X = lv[(size_t)L + 1];
    u64 re_used = P.rb + P.ein;
    u64 meta_used = 0;  // end of the meta tables of the levels so far
    for (int i = 0; i <= L; i++) {
      const BkLevel& Q = lv[(size_t)i];
      if (Q.nbits) meta_used = std::max<u64>(meta_used, Q.cst_off + 2 * ((1ull << Q.nbits) + 1));
      if (i < L && Q.eout) meta_used = std::max<u64>(meta_used, Q.rfo_off + ((Q.n + (1ull << Q.fb) - 1) >> Q.fb) + 1);
    }
    X = BkLevel{};
    X.lb = P.lb + P.n;
    X.rb = re_used;
    if (!bk_ranges(P.n, &P.pshift, &P.fb))
      return bail(fail(GM_ELIMIT, "level %d holds %llu positions: more than the 2^29 a bucketed level supports", L,
                       (unsigned long long)P.n));
    P.eout = 0;
    if (P.n) {
      const u64 nblk = std::min<u64>(kBkExpandBlocks, (P.n + kBkExpandThreads - 1) / kBkExpandThreads),
                chunk = (P.n + nblk - 1) / nblk;
      const uint32_t NR = (uint32_t)((P.n + (1ull << P.fb) - 1) >> P.fb);
      if (meta_used + NR + 1 > s->meta_cap) return bail(fail(GM_ECORRUPT, "bucket tables exceed the scratch"));
      P.rfo_off = (uint32_t)meta_used;
      meta_used += NR + 1;
      uint32_t* rfo = s->meta + P.rfo_off;  // answers per fine parent range -> their starts
      keep.emplace_back(2 * (kBkC + 1));
      std::vector<uint32_t>& hb = keep.back();  // [coarse bases | parent-range bases]
      u64 E = 0, Ep = 0;
      // Count-free form first (k_bk_expand<OVER>): children go straight to
      // provisioned partitions; a partition past its share -> the exact
      // form (F0 counts, then k_bk_expand<false>) for this level.
      // a partition's provisioned share, whole chunks of the chunked staging
      uint32_t ck_sh = 14;
      while (ck_sh > 6 && (s->Emax / kBkC) < (1ull << ck_sh)) ck_sh--;
      const uint32_t cap = (uint32_t)((s->Emax / kBkC) >> ck_sh << ck_sh);
      const BkChunked ck{(char*)s->S1k, ck_sh};
      uint32_t incap = 0;
      bool exact = true;
      hipEvent_t* sp = nullptr;
      if (!(s->flags & GM_F_BK_EXACT)) {
        HIPCHK(hipMemsetAsync(rfo, 0, (NR + 1) * 4, st));
        HIPCHK(hipMemsetAsync(s->bkgc, 0, (2 * kBkC + 4) * 4, st));
        // parents per round from the previous level's branching (a round's
        // children should fill most of the 8192-record stage)
        const double avg = (L > 0 && lv[(size_t)L - 1].n) ? std::max(1.0, (double)P.ein / (double)lv[(size_t)L - 1].n) : 4.0;
        const uint32_t ppr = bk_ppr(avg);
        sp = span(true);
        bk_dispatch(s->d, [&](auto kind_) {
          constexpr int K_ = decltype(kind_)::value;
          hipLaunchKernelGGL((k_bk_expand<K_, true>), dim3(nblk), dim3(kBkExpandThreads), 0, st, s->d, s->bkK + P.lb, P.n,
                             chunk, (const uint32_t*)nullptr, (const uint32_t*)nullptr, ppr, s->S1k, s->S1p, s->S1f, cap,
                             s->bkgc, P.pshift, P.fb, s->bkgc + kBkC, rfo, s->bkgc + 2 * kBkC, s->st, ck);
        });
        hipLaunchKernelGGL(k_bk_scan, dim3(1), dim3(1024), 0, st, rfo, NR + 1, rfo, s->bktotal + 1);
        if ((rc = span_end(sp))) return bail(rc);
        nfwd += 2;
        HIPCHK(hipGetLastError());
        std::vector<uint32_t> g(2 * kBkC + 1);
        HIPCHK(hipMemcpyAsync(g.data(), s->bkgc, g.size() * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(&herr, &s->st->err, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (herr) return bail(fail(GM_ECORRUPT, "level %d:%s", L, err_text(herr).c_str()));
        if (!g[2 * kBkC]) {
          exact = false;
          incap = cap;
          for (int j = 0; j < kBkC; j++) {
            hb[(size_t)j] = (uint32_t)E;
            hb[(size_t)kBkC + 1 + j] = (uint32_t)Ep;
            E += g[(size_t)j];
            Ep += g[(size_t)kBkC + j];
          }
        }
      }
      if (exact) {
        HIPCHK(hipMemsetAsync(rfo, 0, (NR + 1) * 4, st));
        sp = span(true);
        BK_KIND_LAUNCH(k_bk_count, nblk, kBkStreamThreads, s, s->d, s->bkK + P.lb, P.n, chunk, P.pshift, P.fb, s->bh,
                       s->ph, rfo, s->st);
        hipLaunchKernelGGL(k_bk_colscan, dim3(kBkC), dim3(256), 0, st, s->bh, (uint32_t)nblk, s->boff, s->tot);
        hipLaunchKernelGGL(k_bk_colscan, dim3(kBkC), dim3(256), 0, st, s->ph, (uint32_t)nblk, s->ph, s->tot + kBkC);
        hipLaunchKernelGGL(k_bk_scan, dim3(1), dim3(1024), 0, st, rfo, NR + 1, rfo, s->bktotal + 1);
        if ((rc = span_end(sp))) return bail(rc);
        nfwd += 4;
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(htot.data(), s->tot, 2 * kBkC * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(&herr, &s->st->err, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (herr) return bail(fail(GM_ECORRUPT, "level %d:%s", L, err_text(herr).c_str()));
        for (int j = 0; j < kBkC; j++) {
          hb[(size_t)j] = (uint32_t)E;
          hb[(size_t)kBkC + 1 + j] = (uint32_t)Ep;
          E += htot[(size_t)j];
          Ep += htot[(size_t)kBkC + j];
        }
      }
      if (E != Ep) return bail(fail(GM_ECORRUPT, "level %d: %llu children by partition, %llu by parent", L,
                                    (unsigned long long)E, (unsigned long long)Ep));
      if (E > s->Emax) return bail(fail(GM_EFULL, "level %d emits %llu children; the plan holds %llu per level", L,
                                        (unsigned long long)E, (unsigned long long)s->Emax));
      if (re_used + E > s->Ecap) return bail(fail(GM_EFULL, "edges exceed the plan's %llu", (unsigned long long)s->Ecap));
      hb[(size_t)kBkC] = (uint32_t)E;
      hb[(size_t)2 * kBkC + 1] = (uint32_t)Ep;
      P.eout = E;
      X.ein = E;
      HIPCHK(hipMemcpyAsync(s->cbase, hb.data(), (kBkC + 1) * 4, hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(s->pbase + (size_t)L * (kBkC + 1), hb.data() + kBkC + 1, (kBkC + 1) * 4,
                            hipMemcpyHostToDevice, st));
      if (E) {
        uint32_t f = 0;
        while (f < (uint32_t)kBkMaxFineBits && (E >> f) > (u64)kBkC * 4096) f++;
        const uint32_t F = 1u << f, NB = (uint32_t)kBkC << f;
        X.nbits = 8 + f;
        if (meta_used + 2 * (NB + 1) > s->meta_cap) return bail(fail(GM_ECORRUPT, "bucket tables exceed the scratch"));
        X.cst_off = (uint32_t)meta_used;
        uint32_t* cst = s->meta + X.cst_off;
        uint32_t* fo = cst + NB + 1;  // kept: the backward pass walks the level's in-edges bucket by bucket
        const int gd = (int)std::min<uint32_t>(NB, 512);  // two workgroups per CU
        sp = span(true);
        if (exact) {  // parents per expand round: about a stage (8192 records) of children
          const double avg = (double)E / (double)P.n;
          const uint32_t ppr = bk_ppr(avg);
          bk_dispatch(s->d, [&](auto kind_) {
            constexpr int K_ = decltype(kind_)::value;
            hipLaunchKernelGGL((k_bk_expand<K_, false>), dim3(nblk), dim3(kBkExpandThreads), 0, st, s->d, s->bkK + P.lb,
                               P.n, chunk, (const uint32_t*)s->boff, (const uint32_t*)s->cbase, ppr, s->S1k, s->S1p,
                               s->S1f, 0u, (uint32_t*)nullptr, 0u, 0u, (uint32_t*)nullptr, (uint32_t*)nullptr,
                               (uint32_t*)nullptr, s->st, BkChunked{nullptr, 0});
          });
          nfwd++;
        }
        // the fine partition writes the parents straight into the level's
        // in-edge parents (REp); F3 adds the child indices (REc)
        hipLaunchKernelGGL(k_bk_fine, dim3(kBkC), dim3(kBkFineThreads), 0, st, (const u64*)s->S1k,
                           (const uint32_t*)s->S1p, (const uint8_t*)s->S1f, (const uint32_t*)s->cbase, 8u - f, F, s->S2k,
                           s->REp + X.rb, fo, P.pshift, s->bkah + (size_t)L * kBkC * kBkC, incap, ck);
        // unique keys of bucket b to S1k[fo[b] ..), compacted into the level
        hipLaunchKernelGGL(k_bk_dedup, dim3(gd), dim3(kBkDedupThreads), 0, st, s->S2k, (const uint32_t*)fo, NB, s->S1k,
                           s->ucnt, s->REc + X.rb, s->st);
        hipLaunchKernelGGL(k_bk_scan, dim3(1), dim3(1024), 0, st, s->ucnt, NB, cst, s->bktotal);
        if ((rc = span_end(sp))) return bail(rc);
        nfwd += 3;
        HIPCHK(hipGetLastError());
        u64 n1 = 0;
        HIPCHK(hipMemcpyAsync(&n1, s->bktotal, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(&herr, &s->st->err, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (herr) {
          // a fine bucket over kBkMaxUnique keys follows from the level's
          // real edges, not from the buffers: more memory cannot fix it
          const bool lim = herr & ERR_BUCKET_FULL;
          return bail(fail(lim ? GM_ELIMIT : GM_ECORRUPT, "level %d:%s", L + 1, err_text(herr).c_str()));
        }
        if (X.lb + n1 > s->Pcap) return bail(fail(GM_EFULL, "positions exceed the plan's %llu", (unsigned long long)s->Pcap));
        X.n = n1;
        sp = span(true);
        hipLaunchKernelGGL(k_bk_compact, dim3(std::min<uint32_t>(NB, 4096)), dim3(256), 0, st, (const u64*)s->S1k,
                           (const uint32_t*)fo, (const uint32_t*)cst, NB, s->bkK + X.lb);
        if ((rc = span_end(sp))) return bail(rc);
        nfwd++;
        HIPCHK(hipGetLastError());
      }
    }
    HIPCHK(hipMemcpyAsync(s->bkL + L, &lv[(size_t)L], 2 * sizeof(BkLevel), hipMemcpyHostToDevice, st));
  }
  HIPCHK(hipEventRecord(e1, st));
  // ---- backward ----
  for (int L = T - 1; L >= 0; L--) {
    const int k = 2 * T - 1 - L;
    if (k < first) continue;
    if (k >= stop) break;
    BkLevel& P = lv[(size_t)L];
    if (!P.n) continue;
    if (!bk_ranges(P.n, &P.pshift, &P.fb)) return bail(fail(GM_ELIMIT, "level %d too wide for bucketed levels", L));
    const uint32_t NR = (uint32_t)((P.n + (1ull << P.fb) - 1) >> P.fb);
    const int gr = (int)std::min<uint32_t>(NR, 512);
    hipEvent_t* sp = span(false);
    if (L + 1 < T && P.eout) {
      const BkLevel& X = lv[(size_t)L + 1];
      const uint32_t NB = 1u << X.nbits, F = NB / kBkC;
      const uint32_t* cst = s->meta + X.cst_off;
      const uint32_t* fo = cst + NB + 1;
      const uint32_t* rfo = s->meta + P.rfo_off;
      const uint32_t* pb = s->pbase + (size_t)L * (kBkC + 1);
      uint32_t* Ap = (uint32_t*)s->S1k;
      constexpr uint32_t K = kBkSplitK;  // B4 workgroups per range
      // B3: one workgroup per children's partition, exact offsets per
      // (partition, parent range) from the counts F2 kept (ah).  (Measured:
      // K = 4 workgroups of 512 threads per partition on device run cursors
      // took 50.5 ms of backward against 48.2 for this form.)
      hipLaunchKernelGGL(k_bk_colscan, dim3(kBkC), dim3(256), 0, st, s->bkah + (size_t)L * kBkC * kBkC, (uint32_t)kBkC,
                         s->boff, s->tot);
      hipLaunchKernelGGL(k_bk_answer, dim3(kBkC), dim3(kBkStreamThreads), 0, st, s->REp + X.rb, s->REc + X.rb, fo, cst,
                         NB, F, P.pshift, s->boff, pb, s->bkW + X.lb, Ap, s->st);
      nbwd += 2;
      const uint32_t Fp = 1u << (P.pshift - P.fb);
      const uint32_t* ap = Ap;
      if (Fp > 1) {
        HIPCHK(hipMemcpyAsync(s->bkcur + kBkC, rfo, (size_t)NR * 4, hipMemcpyDeviceToDevice, st));
        hipLaunchKernelGGL(k_bk_split, dim3(kBkC * K), dim3(kBkStreamThreads), 0, st, (const uint32_t*)Ap, pb,
                           10u + P.fb, Fp, K, s->bkcur + kBkC, (uint32_t*)s->S2k);
        ap = (uint32_t*)s->S2k;
        nbwd++;
      }
      BK_KIND_LAUNCH(k_bk_reduce, gr, kBkReduceThreads, s, s->d, s->bkK + P.lb, P.n, ap, rfo, P.fb, Fp - 1, NR,
                     s->bkW + P.lb, s->st);
    } else {
      BK_KIND_LAUNCH(k_bk_reduce, gr, kBkReduceThreads, s, s->d, s->bkK + P.lb, P.n, (const uint32_t*)nullptr,
                     (const uint32_t*)nullptr, P.fb, 0u, NR, s->bkW + P.lb, s->st);
    }
    nbwd++;
    if ((rc = span_end(sp))) return bail(rc);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipEventRecord(e2, st));
  if (stop < 2 * T) {  // stopped early: the state stays in the buffers for a resume
    HIPCHK(hipMemcpyAsync(s->bkL, lv.data(), sizeof(BkLevel) * (size_t)T, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
    cleanup();
    out->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return GM_PARTIAL;
  }
  HIPCHK(hipMemcpyAsync(s->bkL, lv.data(), sizeof(BkLevel) * (size_t)T, hipMemcpyHostToDevice, st));
  uint32_t root_word = NO_WORD;
  HIPCHK(hipMemcpyAsync(&root_word, s->bkW, 4, hipMemcpyDeviceToHost, st));
  std::vector<unsigned char> host(devstate_bytes(T));
  HIPCHK(hipMemcpyAsync(host.data(), s->st, host.size(), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  auto t1 = std::chrono::steady_clock::now();
  const DevState* hs = (const DevState*)host.data();
  float f = 0, b = 0;
  HIPCHK(hipEventElapsedTime(&f, e0, e1));
  HIPCHK(hipEventElapsedTime(&b, e1, e2));
  out->ms_forward = f;
  out->ms_backward = b;
  out->ms_total = std::chrono::duration<double, std::milli>(t1 - t0).count();
  if (timing) {
    double sx = 0, sr = 0;
    for (const Span& x : spans) {
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, x.a, x.b));
      (x.fwd ? sx : sr) += ms;
    }
    out->ms_expand_kernels = sx;
    out->ms_resolve_kernels = sr;
    out->n_expand_launches = nfwd;
    out->n_resolve_launches = nbwd;
  }
  cleanup();
  u64 pos = 0, wmax = 0;
  uint32_t nlev = 0;
  for (const BkLevel& x : lv) {
    pos += x.n;
    wmax = std::max<u64>(wmax, x.n);
    nlev += x.n > 0;
  }
  out->positions = pos;
  out->edges = hs->edges;
  out->primitives = hs->prims;
  out->levels = nlev;
  out->max_level_width = (uint32_t)std::min<u64>(wmax, 0xFFFFFFFFull);
  out->root_word = root_word;
  if (hs->err) {
    const bool full = hs->err & (ERR_TABLE_FULL | ERR_LEVELS_FULL);
    const bool lim = hs->err & ERR_BUCKET_FULL;
    return fail(lim ? GM_ELIMIT : full ? GM_EFULL : GM_ECORRUPT, "solve failed:%s", err_text(hs->err).c_str());
  }
  if (root_word == NO_WORD) return fail(GM_ECORRUPT, "root unresolved");
  out->root_value = (int32_t)(root_word & 3u);
  out->root_remoteness = root_word >> 2;
  return 0;
}

#include "gm_bucketed_shard.h"

int gm_solve_group(gm_solver** shards, int n, gm_result* out) {
  if (!shards || n < 1 || !out) return fail(GM_EINVAL, "bad argument");
  memset(out, 0, sizeof *out);
  std::vector<gm_solver*> ss(shards, shards + n);
  for (gm_solver* s : ss)
    if (!s) return fail(GM_EINVAL, "null shard");
  if (ss[0]->mode == GM_MODE_PLANES) return run_planes(ss, out);
  if (ss[0]->mode == GM_MODE_BUCKETED) return run_bucketed_shards(ss, out);
  if (ss[0]->mode == GM_MODE_RANKED) return ss[0]->world > 1 ? run_ranked_shards(ss, out) : run_ranked(ss[0], out);
  return run_dense(ss, out);
}

int gm_solver_query(gm_solver* s, const uint64_t* keys_dev, uint64_t n, uint32_t* words_dev) {
  if (!s || (n && (!keys_dev || !words_dev))) return fail(GM_EINVAL, "bad argument");
  if (!n) return 0;
  if (s->mode == GM_MODE_PLANES) return plane_query(s, keys_dev, n, words_dev);
  if (s->mode == GM_MODE_RANKED) return rank_query(s, keys_dev, n, words_dev);
  int grid = (int)std::min<u64>((n + kBlock - 1) / kBlock, (u64)s->grid);
  if (s->mode == GM_MODE_DENSE)
    hipLaunchKernelGGL(k_dense_query, dim3(grid), dim3(kBlock), 0, s->stream, s->d, s->view, s->words, s->bits,
                       (const u64*)keys_dev, n, words_dev, s->wbits());
  else if (s->mode == GM_MODE_BUCKETED)
    hipLaunchKernelGGL(k_bk_query, dim3(grid), dim3(kBlock), 0, s->stream, s->d, s->bkK, s->bkW, s->bkL,
                       s->d.max_levels, s->meta, (const u64*)keys_dev, n, words_dev);
  else
    hipLaunchKernelGGL(k_query, dim3(grid), dim3(kBlock), 0, s->stream, s->d, s->tab, s->mask, (const u64*)keys_dev, n,
                       words_dev);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s->stream));
  return 0;
}

int gm_solver_positions(gm_solver* s, uint64_t* keys_dev, uint64_t cap, uint64_t* n) {
  if (!s || !n) return fail(GM_EINVAL, "bad argument");
  if (s->mode == GM_MODE_PLANES) return plane_positions(s, keys_dev, cap, n);
  if (s->mode == GM_MODE_RANKED) return rank_positions(s, keys_dev, cap, n);
  if (s->mode == GM_MODE_BUCKETED) {  // every level's keys, contiguous
    u64 tot = 0;
    for (const BkLevel& x : s->lvh) tot += x.n;
    *n = tot;
    if (tot > cap || !keys_dev) return cap < tot ? fail(GM_EFULL, "need %llu slots", (unsigned long long)tot) : 0;
    HIPCHK(hipMemcpyAsync(keys_dev, s->bkK, tot * sizeof(u64), hipMemcpyDeviceToDevice, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return 0;
  }
  u64 cur[2];
  HIPCHK(hipStreamSynchronize(s->stream));
  HIPCHK(hipMemcpy(cur, s->st, sizeof cur, hipMemcpyDeviceToHost));
  *n = s->mode == GM_MODE_DENSE ? cur[0] : cur[0] + cur[1];
  if (s->mode == GM_MODE_DENSE) {
    if (*n > cap || !keys_dev) return cap < *n ? fail(GM_EFULL, "need %llu slots", (unsigned long long)*n) : 0;
    HIPCHK(hipMemsetAsync(&s->st->cursor_back, 0, sizeof(u64), s->stream));
    hipLaunchKernelGGL(k_dense_positions, dim3(s->grid), dim3(kBlock), 0, s->stream, s->d, s->view, s->bits,
                       (u64)s->d.max_levels, (u64*)keys_dev, cap, &s->st->cursor_back);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s->stream));
    return 0;
  }
  if (*n > cap || !keys_dev) return cap < *n ? fail(GM_EFULL, "need %llu slots", (unsigned long long)*n) : 0;
  hipLaunchKernelGGL(k_gather_positions, dim3(s->grid), dim3(kBlock), 0, s->stream, s->lv, s->lcap, s->st,
                     (u64*)keys_dev);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s->stream));
  return 0;
}

int gm_solver_checksum(gm_solver* s, uint64_t out[6]) {
  if (!s || !out) return fail(GM_EINVAL, "bad argument");
  u64* acc = s->st->ck;
  HIPCHK(hipMemsetAsync(acc, 0, 6 * sizeof(u64), s->stream));
  if (s->mode == GM_MODE_PLANES)
    plane_checksum_launch(s, acc);
  else if (s->mode == GM_MODE_RANKED) {
    int rc = rank_scan(s, true, nullptr, 0, acc);
    if (rc) return rc;
  }
  else if (s->mode == GM_MODE_DENSE)
    hipLaunchKernelGGL(k_checksum_dense, dim3(s->grid), dim3(kBlock), 0, s->stream, s->d, s->view, s->words, s->bits,
                       (u64)s->d.max_levels, s->wbits(), acc);
  else if (s->mode == GM_MODE_BUCKETED) {
    u64 tot = 0;
    for (const BkLevel& x : s->lvh) tot += x.n;
    hipLaunchKernelGGL(k_checksum_flat, dim3(s->grid), dim3(kBlock), 0, s->stream, s->d, s->bkK, s->bkW, tot, acc);
  } else
    hipLaunchKernelGGL(k_checksum_hashed, dim3(s->grid), dim3(kBlock), 0, s->stream, s->d, s->tab, s->mask, s->lv,
                       s->lcap, s->st, acc);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, acc, 6 * sizeof(u64), hipMemcpyDeviceToHost, s->stream));
  HIPCHK(hipStreamSynchronize(s->stream));
  return 0;
}

// gm_solve keeps its solver per game id until the next gm_solve of that game
// or gm_release(game), so gm_query(game, ...) reads the table it left in the
// caller's buffers (SURVEY §8b's one-shot pair)
static std::mutex g_solved_mu;
static std::map<int, gm_solver*> g_solved;

// gm_solve over several GPUs of this process (SURVEY §8b's `ngpus`; the
// reference's `mpiexec -n P`, solver_launcher.py:30,76-84): shard i of the
// plan gm_plan_multi gives lives on device i in buf[i]; one RCCL
// communicator per device (ncclCommInitAll) and one host thread per device
// driving its shard's gm_solver_solve -- the halo rows (PLANES / DENSE) and
// the md5 all-to-alls (BUCKETED) are RCCL calls every rank's thread must
// enter.  Every rank ends with the job's totals and root word.
struct MultiSolve {
  std::vector<gm_solver*> ss;
};
static std::map<int, MultiSolve> g_multi;  // under g_solved_mu

static void multi_destroy(MultiSolve& m) {
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (size_t i = 0; i < m.ss.size(); i++)
    if (m.ss[i]) {
      (void)hipSetDevice((int)i);
      gm_solver_destroy(m.ss[i]);
      m.ss[i] = nullptr;
    }
  (void)hipSetDevice(cur);
}

// Failure in bounded time: every early return goes through bail (shards and
// communicators freed, the caller's device restored).  A shard whose solve
// fails on its own side defers the error to the end-of-solve reduction (the
// staged PLANES backward, the md5 BUCKETED levels), so its peers finish; a
// shard whose solve returns while its peers may still wait in an RCCL call
// (an early return) aborts EVERY communicator of the group (ncclCommAbort:
// the peers' pending calls return with an error), so join() always returns.
static int solve_multi(int game, int ngpus, const gm_buffers* buf, gm_result* out) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
  if (ngpus > ndev) return fail(GM_EINVAL, "ngpus %d: %d GPU(s) visible", ngpus, ndev);
  for (int i = 0; i < ngpus; i++)
    if (buf[i].mode != buf[0].mode) return fail(GM_EINVAL, "buf[%d]: every shard needs the mode of gm_plan_multi", i);
  int cur = 0;
  HIPCHK(hipGetDevice(&cur));
  MultiSolve m;
  m.ss.assign((size_t)ngpus, nullptr);
  std::vector<ncclComm_t> comms((size_t)ngpus, nullptr);
  std::vector<int> devs((size_t)ngpus);
  for (int i = 0; i < ngpus; i++) devs[(size_t)i] = i;
  bool aborted = false;  // every communicator aborted (and detached from its shard)
  auto bail = [&](int rc) {
    if (!aborted)
      for (size_t i = 0; i < comms.size(); i++)
        if (comms[i] && !(m.ss[i] && m.ss[i]->comm == comms[i])) (void)ncclCommDestroy(comms[i]);
    multi_destroy(m);
    (void)hipSetDevice(cur);
    return rc;
  };
  for (int i = 0; i < ngpus; i++) {
    if (hipSetDevice(i) != hipSuccess) return bail(fail(GM_EHIP, "hipSetDevice(%d)", i));
    const int rc = gm_solver_create_shard(game, i, ngpus, &buf[i], &m.ss[(size_t)i]);
    if (rc) return bail(fail(rc, "shard %d: %s", i, gm_last_error()));
  }
  const ncclResult_t r = ncclCommInitAll(comms.data(), ngpus, devs.data());
  if (r != ncclSuccess) return bail(fail(GM_EHIP, "ncclCommInitAll: %s", ncclGetErrorString(r)));
  for (int i = 0; i < ngpus; i++) {
    gm_solver* sh = m.ss[(size_t)i];
    sh->comm = comms[(size_t)i];
    if (hipSetDevice(i) != hipSuccess) return bail(fail(GM_EHIP, "hipSetDevice(%d)", i));
    if (!sh->errg && hipMalloc((void**)&sh->errg, (size_t)ngpus * sizeof(u64)) != hipSuccess)
      return bail(fail(GM_EHIP, "error-mask gather buffer"));
  }
  // The staged PLANES deal sends its odd-direction halos on a second
  // communicator per shard (gm_plane_run.h): split here, before any shard
  // thread runs, one group call over every rank -- so abort_all below knows
  // every communicator a thread can wait in (a shard that split its own on
  // first use could be blocked in comm2 while the abort missed it).
  bool staged_deal = false;
  for (gm_solver* sh : m.ss) staged_deal = staged_deal || (sh->mode == GM_MODE_PLANES && sh->pstage_k);
  if (staged_deal) {
    ncclResult_t r1 = ncclGroupStart();
    for (int i = 0; i < ngpus && r1 == ncclSuccess; i++) {
      gm_solver* sh = m.ss[(size_t)i];
      if (!sh->comm2) r1 = ncclCommSplit(sh->comm, 0, sh->rank, &sh->comm2, nullptr);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r1 != ncclSuccess || r2 != ncclSuccess)
      return bail(fail(GM_EHIP, "ncclCommSplit (staged deal): %s", ncclGetErrorString(r1 != ncclSuccess ? r1 : r2)));
  }
  std::vector<gm_result> res((size_t)ngpus);
  std::vector<int> rcs((size_t)ngpus, 0);
  std::vector<std::string> msg((size_t)ngpus);
  std::mutex abort_mu;  // one abort of the whole group, by the first thread that fails
  std::atomic<int> gabort{0};
  for (gm_solver* sh : m.ss) sh->gabort = &gabort;
  auto abort_all = [&]() {
    std::lock_guard<std::mutex> lk(abort_mu);
    if (aborted) return;
    aborted = true;
    // published first: a shard that checks it (RCCL_LIVE, before every RCCL
    // call) issues nothing more on these communicators; then every one of
    // them -- the primary ones and the staged deal's second ones -- is
    // aborted, so a peer waiting in any RCCL call on any of them returns
    gabort.store(1, std::memory_order_release);
    for (size_t i = 0; i < comms.size(); i++)
      if (comms[i]) (void)ncclCommAbort(comms[i]);
    for (gm_solver* sh : m.ss)
      if (sh && sh->comm2) (void)ncclCommAbort(sh->comm2);
  };
  std::vector<std::thread> th;
  for (int i = 0; i < ngpus; i++)
    th.emplace_back([&, i]() {
      if (hipSetDevice(i) != hipSuccess) {
        rcs[(size_t)i] = GM_EHIP;
        msg[(size_t)i] = "hipSetDevice";
        abort_all();
        return;
      }
      rcs[(size_t)i] = gm_solver_solve(m.ss[(size_t)i], &res[(size_t)i]);
      if (rcs[(size_t)i]) {
        msg[(size_t)i] = gm_last_error();
        // a deferred failure has already taken every peer through the
        // reduction; any other failure may leave them waiting: abort
        if (!m.ss[(size_t)i]->defer_rc) abort_all();
      }
    });
  for (auto& t : th) t.join();
  (void)hipSetDevice(cur);
  for (gm_solver* sh : m.ss) sh->gabort = nullptr;
  if (aborted)  // the aborted communicators are not destroyed again with the shards
    for (gm_solver* sh : m.ss)
      if (sh) sh->comm = sh->comm2 = nullptr;
  for (int i = 0; i < ngpus; i++)
    if (rcs[(size_t)i]) return bail(fail(rcs[(size_t)i], "shard %d: %s", i, msg[(size_t)i].c_str()));
  *out = res[0];
  std::lock_guard<std::mutex> lk(g_solved_mu);
  g_multi[game] = std::move(m);
  return 0;
}

int gm_plan_multi(int game, int ngpus, uint64_t positions, uint32_t flags, uint64_t max_table_bytes,
                  gm_plan_t* plans) {
  const Desc* d = get_game(game);
  if (!d || !plans || ngpus < 1) return fail(GM_EINVAL, "bad argument");
  if (ngpus == 1) return gm_plan(game, positions, flags, max_table_bytes, plans);
  if (d->dense_ok) {  // sum games: PLANES (or level-major DENSE) blocks of the last heap
    for (int r = 0; r < ngpus; r++) {
      const int rc = gm_plan_shard(game, r, ngpus, flags, max_table_bytes, &plans[r]);
      if (rc) return rc;
    }
    return 0;
  }
  if (!bk_ok(d)) return fail(GM_EINVAL, "%d GPUs in one process: the game needs a dense or bucketed shard layout "
                                        "(keyed games of other shapes: one process per GPU, keyed.py)", ngpus);
  if (positions == 0) {
    gm_game_info(game, &positions, nullptr, nullptr);
    if (positions == 0) return fail(GM_EINVAL, "no known position bound for this board; pass an estimate");
  }
  // the md5 shard bound of keyed._shard_bound: the share + 3 % + 64 K
  const u64 per = (u64)((double)positions * 1.03) / (u64)ngpus + 65536;
  for (int r = 0; r < ngpus; r++) {
    const int rc = gm_plan_keyed_shard(game, r, ngpus, per, flags, max_table_bytes, &plans[r]);
    if (rc) return rc;
  }
  return 0;
}

int gm_solve(int game, uint64_t root, int ngpus, const gm_buffers* buf, gm_result* out) {
  const Desc* d = get_game(game);
  if (!d) return fail(GM_EINVAL, "bad game id %d", game);
  if (ngpus < 1 || !buf || !out) return fail(GM_EINVAL, "bad argument");
  if (root != d->root) return fail(GM_EINVAL, "root must be the game's initial position");
  (void)gm_release(game);
  if (ngpus > 1) return solve_multi(game, ngpus, buf, out);
  gm_solver* s = nullptr;
  int rc = gm_solver_create(game, buf, &s);
  if (rc) return rc;
  rc = gm_solver_solve(s, out);
  if (rc) {
    gm_solver_destroy(s);
    return rc;
  }
  std::lock_guard<std::mutex> lk(g_solved_mu);
  g_solved[game] = s;
  return 0;
}

int gm_query(int game, const uint64_t* keys_dev, size_t n, uint32_t* words_dev) {
  gm_solver* s = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_solved_mu);
    auto it = g_solved.find(game);
    if (it != g_solved.end()) s = it->second;
  }
  if (!s) {
    std::lock_guard<std::mutex> lk(g_solved_mu);
    if (g_multi.count(game))
      return fail(GM_EINVAL, "game %d was solved on several GPUs: query its shards (gm_solver_query per device)", game);
    return fail(GM_EINVAL, "game %d has no finished gm_solve to query", game);
  }
  int rc = gm_solver_query(s, keys_dev, (uint64_t)n, words_dev);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(s->stream));
  return 0;
}

int gm_release(int game) {
  gm_solver* s = nullptr;
  MultiSolve m;
  {
    std::lock_guard<std::mutex> lk(g_solved_mu);
    auto it = g_solved.find(game);
    if (it != g_solved.end()) {
      s = it->second;
      g_solved.erase(it);
    }
    auto jt = g_multi.find(game);
    if (jt != g_multi.end()) {
      m = std::move(jt->second);
      g_multi.erase(jt);
    }
  }
  if (s) gm_solver_destroy(s);
  multi_destroy(m);
  return 0;
}

int gm_owner(int game, const uint64_t* keys_dev, uint64_t n, int world_size, uint32_t* owners_dev, void* stream) {
  const Desc* d = get_game(game);
  if (!d || world_size < 1 || (n && (!keys_dev || !owners_dev))) return fail(GM_EINVAL, "bad argument");
  if (!n) return 0;
  int grid = (int)std::min<u64>((n + kBlock - 1) / kBlock, (u64)launch_grid());
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_owner, dim3(grid), dim3(kBlock), 0, st, *d, (const u64*)keys_dev, n, (uint32_t)world_size,
                     owners_dev);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// md5-sharded keyed tables (gm_keyed_shard.h): the host moves keys/words
// between ranks between these steps (gamesmanmpi_amd/keyed.py)
// ---------------------------------------------------------------------------
#define GM_KIND_DISPATCH(KERNEL, GRID, S, ...)                                                      \
  switch ((S)->d.kind) {                                                                           \
    case K_SUM: hipLaunchKernelGGL(KERNEL<K_SUM>, dim3(GRID), dim3(kBlock), 0, (S)->stream, __VA_ARGS__); break; \
    case K_TTT: hipLaunchKernelGGL(KERNEL<K_TTT>, dim3(GRID), dim3(kBlock), 0, (S)->stream, __VA_ARGS__); break; \
    case K_TOOT: hipLaunchKernelGGL(KERNEL<K_TOOT>, dim3(GRID), dim3(kBlock), 0, (S)->stream, __VA_ARGS__); break; \
    default: hipLaunchKernelGGL(KERNEL<K_OTHELLO>, dim3(GRID), dim3(kBlock), 0, (S)->stream, __VA_ARGS__); break; \
  }

static int ks_check(gm_solver* s, int level) {
  if (!s) return fail(GM_EINVAL, "null solver");
  if (s->mode != GM_MODE_HASHED) return fail(GM_EINVAL, "gm_ks_* drive keyed (HASHED) tables only");
  if (level < 0 || level >= s->d.max_levels) return fail(GM_EINVAL, "level %d out of range", level);
  return 0;
}

static int ks_grid(gm_solver* s, u64 n) {
  return (int)std::max<u64>(1, std::min<u64>((n + kBlock - 1) / kBlock, (u64)s->grid));
}

static int ks_errors(gm_solver* s) {
  uint32_t err = 0;
  HIPCHK(hipMemcpyAsync(&err, &s->st->err, sizeof err, hipMemcpyDeviceToHost, s->stream));
  HIPCHK(hipStreamSynchronize(s->stream));
  if (err) {
    bool full = err & (ERR_TABLE_FULL | ERR_LEVELS_FULL);
    return fail(full ? GM_EFULL : GM_ECORRUPT, "shard %d/%d:%s", s->rank, s->world, err_text(err).c_str());
  }
  return 0;
}

int gm_ks_begin(gm_solver* s, int root_owned) {
  int rc = ks_check(s, 0);
  if (rc) return rc;
  HIPCHK(hipMemsetAsync(s->tab, 0xFF, (s->mask + 1) * sizeof(gm_slot), s->stream));
  HIPCHK(hipMemsetAsync(s->st, 0, devstate_bytes(s->d.max_levels), s->stream));
  hipLaunchKernelGGL(k_ks_seed, dim3(1), dim3(64), 0, s->stream, s->tab, s->mask, s->lv, s->st, s->d.root,
                     root_owned ? 1 : 0);
  HIPCHK(hipGetLastError());
  return 0;
}

int gm_ks_level_size(gm_solver* s, int level, uint64_t* n) {
  int rc = ks_check(s, level);
  if (rc) return rc;
  if (!n) return fail(GM_EINVAL, "null argument");
  LevelSeg g;
  HIPCHK(hipMemcpyAsync(&g, &s->st->seg[level], sizeof g, hipMemcpyDeviceToHost, s->stream));
  HIPCHK(hipStreamSynchronize(s->stream));
  *n = (g.fe - g.fb) + (g.c2hi - g.c2lo);
  return 0;
}

int gm_ks_expand(gm_solver* s, int level, uint64_t* keys_dev, uint32_t* owners_dev, uint64_t cap, int world,
                 uint64_t* n) {
  int rc = ks_check(s, level);
  if (rc) return rc;
  if (!n || world < 1 || (cap && (!keys_dev || !owners_dev))) return fail(GM_EINVAL, "bad argument");
  uint64_t width = 0;
  if ((rc = gm_ks_level_size(s, level, &width))) return rc;
  HIPCHK(hipMemsetAsync(&s->st->ks_cursor, 0, sizeof(u64), s->stream));
  GM_KIND_DISPATCH(k_ks_expand, ks_grid(s, width), s, s->d, s->lv, s->lcap, s->st, level, (u64*)keys_dev, cap,
                   &s->st->ks_cursor);
  HIPCHK(hipGetLastError());
  u64 got = 0;
  HIPCHK(hipMemcpyAsync(&got, &s->st->ks_cursor, sizeof got, hipMemcpyDeviceToHost, s->stream));
  HIPCHK(hipStreamSynchronize(s->stream));
  *n = got;
  if (got > cap) return fail(GM_EFULL, "expand of level %d emits %llu children (cap %llu)", level,
                             (unsigned long long)got, (unsigned long long)cap);
  if (got)
    hipLaunchKernelGGL(k_owner, dim3(ks_grid(s, got)), dim3(kBlock), 0, s->stream, s->d, (const u64*)keys_dev, got,
                       (uint32_t)world, owners_dev);
  HIPCHK(hipGetLastError());
  return 0;
}

int gm_ks_insert(gm_solver* s, int level, const uint64_t* keys_dev, uint64_t n) {
  int rc = ks_check(s, level);
  if (rc) return rc;
  if (n && !keys_dev) return fail(GM_EINVAL, "null keys");
  if (n) GM_KIND_DISPATCH(k_ks_insert, ks_grid(s, n), s, s->d, s->tab, s->mask, s->lv, s->lcap, s->st, level,
                          (const u64*)keys_dev, (u64)n);
  HIPCHK(hipGetLastError());
  return 0;
}

int gm_ks_finalize(gm_solver* s, int level) {
  int rc = ks_check(s, level);
  if (rc) return rc;
  if (level + 1 >= s->d.max_levels) return fail(GM_EINVAL, "level %d is the last level", level);
  hipLaunchKernelGGL(k_finalize, dim3(1), dim3(64), 0, s->stream, s->st, level, s->lcap);
  HIPCHK(hipGetLastError());
  return ks_errors(s);
}

int gm_ks_counts(gm_solver* s, int level, uint64_t* counts_dev) {
  int rc = ks_check(s, level);
  if (rc) return rc;
  uint64_t width = 0;
  if ((rc = gm_ks_level_size(s, level, &width))) return rc;
  if (!width) return 0;
  if (!counts_dev) return fail(GM_EINVAL, "null counts");
  GM_KIND_DISPATCH(k_ks_counts, ks_grid(s, width), s, s->d, s->lv, s->lcap, s->st, level, counts_dev);
  HIPCHK(hipGetLastError());
  return 0;
}

int gm_ks_children(gm_solver* s, int level, const uint64_t* offsets_dev, uint64_t* keys_dev, uint32_t* owners_dev,
                   int world) {
  int rc = ks_check(s, level);
  if (rc) return rc;
  uint64_t width = 0;
  if ((rc = gm_ks_level_size(s, level, &width))) return rc;
  if (!width) return 0;
  if (!offsets_dev || !keys_dev || !owners_dev || world < 1) return fail(GM_EINVAL, "bad argument");
  GM_KIND_DISPATCH(k_ks_children, ks_grid(s, width), s, s->d, s->lv, s->lcap, s->st, level, offsets_dev,
                   (u64*)keys_dev, owners_dev, (uint32_t)world);
  HIPCHK(hipGetLastError());
  return 0;
}

int gm_ks_reduce(gm_solver* s, int level, const uint64_t* offsets_dev, const uint32_t* child_words_dev) {
  int rc = ks_check(s, level);
  if (rc) return rc;
  uint64_t width = 0;
  if ((rc = gm_ks_level_size(s, level, &width))) return rc;
  if (!width) return 0;
  if (!offsets_dev || !child_words_dev) return fail(GM_EINVAL, "bad argument");
  GM_KIND_DISPATCH(k_ks_reduce, ks_grid(s, width), s, s->d, s->tab, s->mask, s->lv, s->lcap, s->st, level,
                   offsets_dev, child_words_dev);
  HIPCHK(hipGetLastError());
  return ks_errors(s);
}

int gm_ks_end(gm_solver* s, gm_result* out) {
  int rc = ks_check(s, 0);
  if (rc) return rc;
  if (!out) return fail(GM_EINVAL, "null result");
  memset(out, 0, sizeof *out);
  const int T = s->d.max_levels;
  hipLaunchKernelGGL(k_root_word, dim3(1), dim3(64), 0, s->stream, s->tab, s->mask, s->d.root, s->st);
  HIPCHK(hipGetLastError());
  std::vector<unsigned char> host(devstate_bytes(T));
  HIPCHK(hipMemcpyAsync(host.data(), s->st, host.size(), hipMemcpyDeviceToHost, s->stream));
  HIPCHK(hipStreamSynchronize(s->stream));
  const DevState* hs = (const DevState*)host.data();
  out->positions = hs->cursor_front + hs->cursor_back;
  out->edges = hs->edges;
  out->primitives = hs->prims;
  out->max_level_width = (uint32_t)hs->max_width;
  uint32_t lv = 0;
  for (int L = 0; L < T; L++) {
    const LevelSeg& g = hs->seg[L];
    if ((g.fe - g.fb) + (g.c2hi - g.c2lo) > 0) lv++;
  }
  out->levels = lv;
  out->root_word = hs->root_word;  // NO_WORD on every rank but the root's owner
  if (hs->root_word != NO_WORD) {
    out->root_value = (int32_t)(hs->root_word & 3u);
    out->root_remoteness = hs->root_word >> 2;
  }
  if (hs->err) {
    bool full = hs->err & (ERR_TABLE_FULL | ERR_LEVELS_FULL);
    return fail(full ? GM_EFULL : GM_ECORRUPT, "shard %d/%d:%s", s->rank, s->world, err_text(hs->err).c_str());
  }
  return 0;
}

// ---------------------------------------------------------------------------
// Explicit-graph retrograde for game files without a device descriptor
// (SURVEY §8f row 3): the host enumerates the positions with the module's
// own gen_moves/do_move/primitive (gamesmanmpi_amd/generic.py) and hands
// over a CSR graph; the device resolves it in rounds.  A round resolves
// every position whose children are all resolved (any order of positions
// inside a round is fine: a word, once written, is final), so the number of
// rounds is the height of the DAG.  No progress with the root unresolved
// means a cycle (the reference's job loop would never finish either).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_graph_round(const uint8_t* prim, const uint64_t* offsets,
                                                     const uint32_t* children, uint64_t n, uint32_t* words,
                                                     DevState* st) {
  u64 done = 0, edges = 0, prims = 0;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
    if (words[i] != NO_WORD) continue;
    const int p = prim[i];
    uint32_t word;
    if (p != UNDECIDED) {
      word = make_word(p, 0);  // process.py:120-123: primitive, remoteness 0
      prims++;
    } else {
      const u64 a = offsets[i], b = offsets[i + 1];
      bool ready = true, any_loss = false, any_tie = false, any_draw = false;
      uint32_t min_loss = 0xFFFFFFFFu, max_all = 0;
      for (u64 j = a; j < b && ready; j++) {
        const uint32_t w = __hip_atomic_load(&words[children[j]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (w == NO_WORD) {
          ready = false;
          break;
        }
        const uint32_t v = w & 3u, r = w >> 2;
        if (v == LOSS) { any_loss = true; min_loss = min(min_loss, r); }
        any_tie |= (v == TIE);
        any_draw |= (v == DRAW);
        max_all = max(max_all, r);
      }
      if (!ready) continue;
      if (a == b) {  // no moves but not primitive: the reference's job never resolves
        atomicOr(&st->err, ERR_NO_MOVES);
        continue;
      }
      // reference-canonical _res_red / _remote_red
      if (any_loss) word = make_word(WIN, min_loss + 1);
      else word = make_word(any_tie ? TIE : any_draw ? DRAW : LOSS, max_all + 1);
      edges += b - a;
    }
    __hip_atomic_store(&words[i], word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    done++;
  }
  block_add(&st->cursor_front, done);
  block_add(&st->edges, edges);
  block_add(&st->prims, prims);
}

int gm_graph_solve(const uint8_t* prim_dev, const uint64_t* offsets_dev, const uint32_t* children_dev, uint64_t n,
                   uint64_t root, uint32_t* words_dev, void* scratch_dev, void* stream, gm_result* out) {
  if (!out || !n || root >= n || !prim_dev || !offsets_dev || !words_dev || !scratch_dev)
    return fail(GM_EINVAL, "bad argument");
  memset(out, 0, sizeof *out);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(GM_ENOGPU, "no HIP device");
  hipStream_t s = (hipStream_t)stream;
  DevState* st = (DevState*)scratch_dev;
  const int grid = (int)std::max<u64>(1, std::min<u64>((n + kBlock - 1) / kBlock, (u64)launch_grid()));
  auto t0 = std::chrono::steady_clock::now();
  HIPCHK(hipMemsetAsync(words_dev, 0xFF, n * sizeof(uint32_t), s));
  HIPCHK(hipMemsetAsync(st, 0, sizeof(DevState), s));
  u64 resolved = 0, rounds = 0;
  uint32_t root_word = NO_WORD;
  for (;;) {
    hipLaunchKernelGGL(k_graph_round, dim3(grid), dim3(kBlock), 0, s, prim_dev, offsets_dev, children_dev, n,
                       words_dev, st);
    HIPCHK(hipGetLastError());
    rounds++;
    u64 now = 0;
    uint32_t err = 0;
    HIPCHK(hipMemcpyAsync(&now, &st->cursor_front, sizeof now, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&err, &st->err, sizeof err, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (err) return fail(GM_ECORRUPT, "graph solve:%s", err_text(err).c_str());
    if (now == resolved) break;  // no progress: done, or a cycle
    resolved = now;
    if (resolved == n) break;
  }
  HIPCHK(hipMemcpyAsync(&root_word, words_dev + root, sizeof root_word, hipMemcpyDeviceToHost, s));
  DevState hs;
  HIPCHK(hipMemcpyAsync(&hs, st, sizeof hs, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  out->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  out->positions = hs.cursor_front;
  out->edges = hs.edges;
  out->primitives = hs.prims;
  out->levels = (uint32_t)rounds;
  out->n_resolve_launches = rounds;
  out->root_word = root_word;
  if (resolved != n)
    return fail(GM_ECORRUPT, "%llu of %llu positions never resolve (cycle)", (unsigned long long)(n - resolved),
                (unsigned long long)n);
  out->root_value = (int32_t)(root_word & 3u);
  out->root_remoteness = root_word >> 2;
  return 0;
}
