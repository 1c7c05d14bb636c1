// gm_ranked_shard.h -- md5 shards of the RANKED layout (toot-and-otto on
// several GPUs).  Included by gm_solver.hip after gm_ranked.h.
//
// Replaces, for toot-and-otto, the reference's multi-rank job
// (src/process.py:109-267 with ownership src/game_state.py:22-30 --
// owner = md5(str(pos)) % world -- and /root/reference/run_savio.sh's many
// ranks): every position is RESOLVED by its md5 owner, exactly the
// reference's partition; what travels between ranks is each level's words,
// not per-edge LOOK_UP / RESOLVE messages.
//
//   setup   every rank holds the whole RANKED index space (gm_ranked.h) and,
//           per slot, its md5 owner as three bit planes (ownb: 16 B per 32
//           slots) -- computed once, it depends on the game alone
//   forward replicated: the 2 ms RANKED forward on every rank (reach bits,
//           counts); then per level and owner, the reached slots each rank
//           owns per tile of 8192 slots (k_rko_count) and their exclusive
//           scan (k_rko_scan) -- the offsets at which the owners' words
//           travel, identical on every rank, so no sizes are exchanged
//   backward, level L (top down):
//           k_rk_backward<.., OWN> resolves only this rank's slots (the
//           children's words at L + 1 are complete on every rank);
//           k_rko_pack packs them in slot order; every rank sends its pack
//           to every other (RCCL send / receive pairs in one group, or the
//           one-GPU rehearsal's device copies, or the host transport);
//           k_rko_unpack writes the others' words into their slots
//   finish  counts: positions and primitives from the forward (rank 0's),
//           edges summed over the ranks (each counts its own slots' moves)
// Bytes per rank and solve: the replicated forward, 1/world of the backward,
// and the level words of the other ranks in (~(world - 1) / world of the
// 1.19 GB of toot 6x4's words) -- DESIGN.md §6c.
extern "C++" {

constexpr uint32_t kRkoMaxWorld = 8;

// per lane, bits of this 32-slot tile word (level-local word wi < nw): the
// reached slots each owner p < P holds
__device__ __forceinline__ void rko_masks(const RankGeom& g, const uint4* __restrict__ ownb, u64 lvstart, u64 wi,
                                          u64 nw, uint32_t P, uint32_t (&mk)[kRkoMaxWorld]) {
  const uint32_t r = wi < nw ? g.reach[(lvstart >> 5) + wi] : 0u;
  const uint4 o = r ? ownb[(lvstart >> 5) + wi] : make_uint4(0, 0, 0, 0);
#pragma unroll
  for (uint32_t p = 0; p < kRkoMaxWorld; p++) mk[p] = p < P ? r & rko_own_mask(o, p) : 0u;
}

// exclusive prefix over the block (256 threads) of c[p] and the block's
// totals, two counters per 32-bit lane (each total <= 8192 < 2^16)
__device__ __forceinline__ void rko_scan8(const uint32_t (&c)[kRkoMaxWorld], uint32_t (&ex)[kRkoMaxWorld],
                                          uint32_t (&tot)[kRkoMaxWorld]) {
  __shared__ uint32_t ws[4][kRkoMaxWorld / 2];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t v[kRkoMaxWorld / 2], x[kRkoMaxWorld / 2];
#pragma unroll
  for (int k = 0; k < (int)kRkoMaxWorld / 2; k++) x[k] = v[k] = c[2 * k] | (c[2 * k + 1] << 16);
#pragma unroll
  for (int o = 1; o < 64; o <<= 1)
#pragma unroll
    for (int k = 0; k < (int)kRkoMaxWorld / 2; k++) {
      const uint32_t y = __shfl_up(x[k], o);
      if (lane >= (uint32_t)o) x[k] += y;
    }
  if (lane == 63)
#pragma unroll
    for (int k = 0; k < (int)kRkoMaxWorld / 2; k++) ws[w][k] = x[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < (int)kRkoMaxWorld / 2; k++) {
    uint32_t before = 0, all = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
      const uint32_t t = ws[j][k];
      if (j < w) before += t;
      all += t;
    }
    const uint32_t e = before + x[k] - v[k];
    ex[2 * k] = e & 0xFFFFu;
    ex[2 * k + 1] = e >> 16;
    tot[2 * k] = all & 0xFFFFu;
    tot[2 * k + 1] = all >> 16;
  }
  __syncthreads();
}

// the md5 owner of every slot of level L (setup), as bit planes: a wave
// takes 64 slots, three ballots, lanes 0 and 32 write their 32-slot words
// (slots that are no position -- hands out of range -- and the padding: 0)
__global__ __launch_bounds__(256) void k_rko_owner(Desc d, RankGeom g, uint32_t L, u64 lvstart, uint32_t lvoff,
                                                   u64 nitems, u64 nspan, uint32_t P, uint4* __restrict__ ownb) {
  const uint32_t lane = threadIdx.x & 63;
  for (u64 i0 = (u64)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); i0 < nspan; i0 += (u64)gridDim.x * blockDim.x) {
    const u64 i = i0 + lane;
    uint32_t o = 0;
    if (i < nitems) {
      const u64 blk = i >> (L + 3);
      const uint32_t a = (uint32_t)((i >> L) & 7u), pat = (uint32_t)(i & ((1ull << L) - 1));
      RankPos p;
      rk_unpack(g, g.lvph[lvoff + blk], p);
      const RankHands u = rk_hands(L, (uint32_t)__builtin_popcount(pat), a);
      if (rk_valid(u)) o = owner_dev(d, rk_key(g, p, pat, L, u), P);
    }
    const u64 b0 = __ballot(o & 1u), b1 = __ballot(o & 2u), b2 = __ballot(o & 4u);
    if ((lane & 31) == 0 && i < nspan) {
      const uint32_t sh = lane;  // 0 or 32
      ownb[(lvstart + i) >> 5] = make_uint4((uint32_t)(b0 >> sh), (uint32_t)(b1 >> sh), (uint32_t)(b2 >> sh), 0u);
    }
  }
}

// per tile of 256 words: the reached slots each owner holds
__global__ __launch_bounds__(256) void k_rko_count(RankGeom g, const uint4* __restrict__ ownb, u64 lvstart, u64 nw,
                                                   uint32_t P, uint32_t* __restrict__ cnt, u64 ntiles) {
  for (u64 tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    uint32_t mk[kRkoMaxWorld], c[kRkoMaxWorld], ex[kRkoMaxWorld], tot[kRkoMaxWorld];
    rko_masks(g, ownb, lvstart, tile * 256 + threadIdx.x, nw, P, mk);
#pragma unroll
    for (uint32_t p = 0; p < kRkoMaxWorld; p++) c[p] = (uint32_t)__builtin_popcount(mk[p]);
    rko_scan8(c, ex, tot);
    if (threadIdx.x == 0)
#pragma unroll
      for (uint32_t p = 0; p < kRkoMaxWorld; p++)
        if (p < P) cnt[p * ntiles + tile] = tot[p];
  }
}

// per owner (one block each): exclusive scan of the tile counts, and the total
__global__ __launch_bounds__(1024) void k_rko_scan(const uint32_t* __restrict__ cnt, uint32_t* __restrict__ off,
                                                   u64 ntiles, u64* __restrict__ total) {
  const uint32_t p = blockIdx.x;
  const uint32_t* c = cnt + p * ntiles;
  uint32_t* o = off + p * ntiles;
  const u64 ch = (ntiles + blockDim.x - 1) / blockDim.x, a = threadIdx.x * ch, b = min(ntiles, a + ch);
  uint32_t sum = 0;
  for (u64 i = a; i < b; i++) sum += c[i];
  uint32_t all;
  uint32_t run = bk_block_scan(sum, &all);
  for (u64 i = a; i < b; i++) {
    const uint32_t v = c[i];
    o[i] = run;
    run += v;
  }
  if (threadIdx.x == 0) total[p] = all;
}

// this rank's words of level L, in slot order, to pk
__global__ __launch_bounds__(256) void k_rko_pack(RankGeom g, const uint4* __restrict__ ownb, u64 lvstart, u64 nw,
                                                  uint32_t me, const uint32_t* __restrict__ off, u64 ntiles,
                                                  uint8_t* __restrict__ pk) {
  for (u64 tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const u64 wi = tile * 256 + threadIdx.x;
    const uint32_t r = wi < nw ? g.reach[(lvstart >> 5) + wi] : 0u;
    const uint32_t m = r ? r & rko_own_mask(ownb[(lvstart >> 5) + wi], me) : 0u;
    uint32_t all;
    u64 at = (u64)off[me * ntiles + tile] + bk_block_scan((uint32_t)__builtin_popcount(m), &all);
    for (uint32_t mm = m; mm; mm &= mm - 1) pk[at++] = g.words[lvstart + (wi << 5) + __builtin_ctz(mm)];
  }
}

// the other owners' words of level L, from rb (owner p's pack at base[p])
struct RkoBases {
  u64 b[kRkoMaxWorld];
};
__global__ __launch_bounds__(256) void k_rko_unpack(RankGeom g, const uint4* __restrict__ ownb, u64 lvstart, u64 nw,
                                                    uint32_t P, uint32_t me, const uint32_t* __restrict__ off,
                                                    u64 ntiles, const uint8_t* __restrict__ rb, RkoBases base) {
  for (u64 tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const u64 wi = tile * 256 + threadIdx.x;
    uint32_t mk[kRkoMaxWorld], c[kRkoMaxWorld], ex[kRkoMaxWorld], tot[kRkoMaxWorld];
    rko_masks(g, ownb, lvstart, wi, nw, P, mk);
#pragma unroll
    for (uint32_t p = 0; p < kRkoMaxWorld; p++)
      if (p == me) mk[p] = 0u;  // (its own words are in place)
#pragma unroll
    for (uint32_t p = 0; p < kRkoMaxWorld; p++) c[p] = (uint32_t)__builtin_popcount(mk[p]);
    rko_scan8(c, ex, tot);
#pragma unroll
    for (uint32_t p = 0; p < kRkoMaxWorld; p++) {
      if (!mk[p]) continue;
      u64 at = base.b[p] + off[p * ntiles + tile] + ex[p];
      for (uint32_t mm = mk[p]; mm; mm &= mm - 1) g.words[lvstart + (wi << 5) + __builtin_ctz(mm)] = rb[at++];
    }
  }
}

// ---------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------
// tile words (32 slots) and tiles (256 words) of level L
static u64 rko_words(const RankShape& rs, uint32_t L) { return (rs.lvitems[L] + 31) / 32; }
static u64 rko_tiles(const RankShape& rs, uint32_t L) { return (rko_words(rs, L) + 255) / 256; }

// The shard's buffers after the RANKED table: the owner bit planes (16 B per
// 32 slots), the pack and
// receive buffers (the largest level's slots each), the per-level tile
// counts and offsets (P rows of the level's tiles), the per-level totals.
struct RkoLayout {
  u64 own_off, pk_off, rb_off, cnt_off, toff_off, tot_off, table_bytes, tiles;
  std::vector<u64> tile0;  // per level: first tile row index
};
static RkoLayout rko_layout(const RankShape& rs, int world) {
  RkoLayout l;
  u64 maxlev = 0;
  l.tile0.assign(rs.g.T + 1, 0);
  for (uint32_t L = 0; L < rs.g.T; L++) {
    maxlev = std::max<u64>(maxlev, rs.lvstart[L + 1] - rs.lvstart[L]);
    l.tile0[L + 1] = l.tile0[L] + rko_tiles(rs, L);
  }
  l.tiles = l.tile0[rs.g.T];
  l.own_off = rup256(rs.table_bytes);
  l.pk_off = l.own_off + rup256(rs.g.nslots / 32 * 16);
  l.rb_off = l.pk_off + rup256(maxlev);
  l.cnt_off = l.rb_off + rup256(maxlev);
  l.toff_off = l.cnt_off + rup256(l.tiles * (u64)world * 4);
  l.tot_off = l.toff_off + rup256(l.tiles * (u64)world * 4);
  l.table_bytes = l.tot_off + rup256((u64)rs.g.T * world * 8);
  return l;
}

static int plan_ranked_shard(const Desc* d, int world, uint64_t max_table_bytes, gm_plan_t* out) {
  if (!rank_ok(d)) return fail(GM_EINVAL, "game has no ranked layout");
  if (world < 2 || world > (int)kRkoMaxWorld) return fail(GM_EINVAL, "ranked md5 shards: 2..%u ranks", kRkoMaxWorld);
  RankShape rs;
  int rc = rank_shape(d, &rs);
  if (rc) return rc;
  const RkoLayout l = rko_layout(rs, world);
  if (max_table_bytes && l.table_bytes > max_table_bytes)
    return fail(GM_EFULL, "ranked shard needs %llu bytes", (unsigned long long)l.table_bytes);
  out->mode = GM_MODE_RANKED;
  out->table_slots = rs.g.nslots;
  out->table_bytes = l.table_bytes;
  out->level_capacity = 1;
  out->scratch_bytes = scratch_bytes_for(d->max_levels);
  out->max_levels = (uint32_t)d->max_levels;
  return 0;
}

// rank_setup's shard part: the buffers and every slot's owner
static int rko_setup(gm_solver* s, const gm_buffers* buf, const RankShape& rs) {
  const RkoLayout l = rko_layout(rs, s->world);
  if (buf->table_bytes < l.table_bytes)
    return fail(GM_EINVAL, "ranked shard table of %llu bytes, the plan needs %llu",
                (unsigned long long)buf->table_bytes, (unsigned long long)l.table_bytes);
  char* t = (char*)buf->table;
  s->rko_own = (uint4*)(t + l.own_off);
  s->rko_pk = (uint8_t*)(t + l.pk_off);
  s->rko_rb = (uint8_t*)(t + l.rb_off);
  s->rko_cnt = (uint32_t*)(t + l.cnt_off);
  s->rko_toff = (uint32_t*)(t + l.toff_off);
  s->rko_tot = (u64*)(t + l.tot_off);
  s->rko_tile0 = l.tile0;
  s->rko_tot_h.assign((size_t)rs.g.T * s->world, 0);
  for (uint32_t L = 0; L < rs.g.T; L++) {
    const u64 span = rs.lvstart[L + 1] - rs.lvstart[L];
    hipLaunchKernelGGL(k_rko_owner, dim3(rank_grid(s, span)), dim3(256), 0, s->stream, s->d, s->rg, L, rs.lvstart[L],
                       rs.lvoff[L], rs.lvitems[L], span, (uint32_t)s->world, s->rko_own);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s->stream));
  return 0;
}

// level L's tile rows of owner p (counts / offsets)
static uint32_t* rko_rows(const gm_solver* s, uint32_t* base, uint32_t L) {
  return base + s->rko_tile0[L] * (u64)s->world;
}
static u64 rko_ntiles(const gm_solver* s, uint32_t L) { return s->rko_tile0[L + 1] - s->rko_tile0[L]; }
static u64 rko_nw(const gm_solver* s, uint32_t L) { return (s->rlvitems[L] + 31) / 32; }
static int rko_tgrid(const gm_solver* s, u64 ntiles) {
  return (int)std::max<u64>(1, std::min<u64>(ntiles, (u64)s->grid * 2));
}
// where owner p's words of level L sit in rank `me`'s receive buffer
static u64 rko_roff(const gm_solver* s, uint32_t L, int me, int p) {
  u64 o = 0;
  for (int q = 0; q < p; q++)
    if (q != me) o += s->rko_tot_h[(size_t)L * s->world + q];
  return o;
}

// The md5-sharded RANKED solve: ss = every shard (one GPU: the rehearsal --
// each shard on its own stream, device copies for the transfers; or on one
// stream) or this process's one shard (RCCL, or the host transport).
static int run_ranked_shards(std::vector<gm_solver*> ss, gm_result* out) {
  gm_solver* s0 = ss[0];
  const int W = s0->world;
  const uint32_t T = s0->rg.T;
  const bool group = ss.size() > 1;
  if (group && (int)ss.size() != W) return fail(GM_EINVAL, "group solve needs all %d shards", W);
  for (size_t i = 0; i < ss.size(); i++) {
    gm_solver* s = ss[i];
    if (s->mode != GM_MODE_RANKED || s->world != W || !s->rko_own || (group && s->rank != (int)i))
      return fail(GM_EINVAL, "ranked md5 shards: ranks 0..%d of one plan", W - 1);
  }
  const int mode = group ? 4 : s0->xfer ? 3 : 1;
  if (mode == 1 && !s0->comm) return fail(GM_EINVAL, "shard %d/%d has no communicator (gm_solver_comm_init)", s0->rank, W);
  // the solve's events, destroyed on EVERY return (the HIPCHK early
  // returns included: they used to skip cleanup() and leak them)
  struct Events {
    std::vector<hipEvent_t> v;
    void clear() {
      for (auto e : v) (void)hipEventDestroy(e);
      v.clear();
    }
    ~Events() { clear(); }
  } ev;
  auto cleanup = [&]() { ev.clear(); };
  auto new_event = [&](hipEvent_t* e, unsigned fl) -> int {
    HIPCHK(hipEventCreateWithFlags(e, fl));
    ev.v.push_back(*e);
    return 0;
  };
  hipEvent_t e0, e1, e2;
  if (new_event(&e0, 0) || new_event(&e1, 0) || new_event(&e2, 0)) return GM_EHIP;
  std::vector<hipEvent_t> PE(ss.size()), CE(ss.size()), JE(ss.size());
  for (size_t i = 0; i < ss.size(); i++)
    if (new_event(&PE[i], hipEventDisableTiming) || new_event(&CE[i], hipEventDisableTiming) ||
        new_event(&JE[i], hipEventDisableTiming))
      return GM_EHIP;
  hipStream_t st = s0->stream;
  auto t0 = std::chrono::steady_clock::now();
  HIPCHK(hipEventRecord(e0, st));
  for (gm_solver* s : ss)
    if (s->stream != st) HIPCHK(hipStreamWaitEvent(s->stream, e0, 0));
  // forward (replicated) and the per-level owner counts
  for (gm_solver* s : ss) {
    hipStream_t ss_ = s->stream;
    HIPCHK(hipMemsetAsync(s->st, 0, devstate_bytes((int)T), ss_));
    HIPCHK(hipMemsetAsync(s->bcount, 0, kCountSlots * sizeof(BlockCount), ss_));
    HIPCHK(hipMemsetD32Async((hipDeviceptr_t)&s->st->word_bits, 0x208, 1, ss_));
    for (uint32_t L = 0; L < T; L++) rank_forward_level(s, ss_, L);
    for (uint32_t L = 0; L < T; L++) {
      const u64 nt = rko_ntiles(s, L);
      if (!nt) continue;
      hipLaunchKernelGGL(k_rko_count, dim3(rko_tgrid(s, nt)), dim3(256), 0, ss_, s->rg, (const uint4*)s->rko_own,
                         s->rlvstart[L], rko_nw(s, L), (uint32_t)W, rko_rows(s, s->rko_cnt, L), nt);
      hipLaunchKernelGGL(k_rko_scan, dim3(W), dim3(1024), 0, ss_, (const uint32_t*)rko_rows(s, s->rko_cnt, L),
                         rko_rows(s, s->rko_toff, L), nt, s->rko_tot + (u64)L * W);
    }
    HIPCHK(hipMemcpyAsync(s->rko_tot_h.data(), s->rko_tot, s->rko_tot_h.size() * 8, hipMemcpyDeviceToHost, ss_));
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(e1, st));
  for (gm_solver* s : ss) HIPCHK(hipStreamSynchronize(s->stream));  // the exchange sizes, on the host
  // backward
  for (uint32_t k = 0; k < T; k++) {
    const uint32_t L = T - 1 - k;
    const u64 nt = rko_ntiles(s0, L);
    for (size_t i = 0; i < ss.size(); i++) {
      gm_solver* s = ss[i];
      if (group && k > 0)  // every receiver has copied this shard's previous pack
        for (size_t j = 0; j < ss.size(); j++)
          if (j != i) HIPCHK(hipStreamWaitEvent(s->stream, CE[j], 0));
      rank_backward_level(s, s->stream, L, s->rko_own, (uint32_t)s->rank);
      if (nt)
        hipLaunchKernelGGL(k_rko_pack, dim3(rko_tgrid(s, nt)), dim3(256), 0, s->stream, s->rg,
                           (const uint4*)s->rko_own, s->rlvstart[L], rko_nw(s, L), (uint32_t)s->rank,
                           (const uint32_t*)rko_rows(s, s->rko_toff, L), nt, s->rko_pk);
      if (group) HIPCHK(hipEventRecord(PE[i], s->stream));
    }
    HIPCHK(hipGetLastError());
    // every rank's pack to every other
    if (mode == 4) {
      for (size_t i = 0; i < ss.size(); i++) {
        gm_solver* t = ss[i];
        for (size_t j = 0; j < ss.size(); j++) {
          if (j == i) continue;
          const u64 n = t->rko_tot_h[(size_t)L * W + j];
          HIPCHK(hipStreamWaitEvent(t->stream, PE[j], 0));
          if (n)
            HIPCHK(hipMemcpyAsync(t->rko_rb + rko_roff(t, L, (int)i, (int)j), ss[j]->rko_pk, n,
                                  hipMemcpyDeviceToDevice, t->stream));
        }
        HIPCHK(hipEventRecord(CE[i], t->stream));
      }
    } else if (mode == 1) {
      gm_solver* s = s0;
      if (s->gabort && s->gabort->load(std::memory_order_acquire)) {
        cleanup();
        return fail(GM_EHIP, "RCCL group aborted: a peer shard failed (shard %d/%d)", s->rank, s->world);
      }
      ncclGroupStart();
      ncclResult_t r = ncclSuccess;
      for (int p = 0; p < W && r == ncclSuccess; p++) {
        if (p == s->rank) continue;
        const u64 ns = s->rko_tot_h[(size_t)L * W + s->rank], nr = s->rko_tot_h[(size_t)L * W + p];
        if (ns) r = ncclSend(s->rko_pk, ns, ncclUint8, p, s->comm, s->stream);
        if (nr && r == ncclSuccess)
          r = ncclRecv(s->rko_rb + rko_roff(s, L, s->rank, p), nr, ncclUint8, p, s->comm, s->stream);
      }
      const ncclResult_t r2 = ncclGroupEnd();
      if (r != ncclSuccess || r2 != ncclSuccess) {
        cleanup();
        return fail(GM_EHIP, "RCCL level exchange: %s", ncclGetErrorString(r != ncclSuccess ? r : r2));
      }
    } else {  // mode 3: pairwise rounds, send to rank + d, receive from rank - d
      gm_solver* s = s0;
      for (int dd = 1; dd < W; dd++) {
        const int sp = (s->rank + dd) % W, rp = (s->rank - dd + W) % W;
        std::vector<HostRange> o, in;
        const u64 ns = s->rko_tot_h[(size_t)L * W + s->rank], nr = s->rko_tot_h[(size_t)L * W + rp];
        if (ns) o.push_back({s->rko_pk, ns});
        if (nr) in.push_back({s->rko_rb + rko_roff(s, L, s->rank, rp), nr});
        int rc = xfer_ranges(s, o, sp, in, rp, s->stream);
        if (rc) {
          cleanup();
          return rc;
        }
      }
    }
    for (gm_solver* s : ss) {
      if (!nt) continue;
      RkoBases b{};
      for (int p = 0; p < W; p++) b.b[p] = rko_roff(s, L, s->rank, p);
      hipLaunchKernelGGL(k_rko_unpack, dim3(rko_tgrid(s, nt)), dim3(256), 0, s->stream, s->rg,
                         (const uint4*)s->rko_own, s->rlvstart[L], rko_nw(s, L), (uint32_t)W, (uint32_t)s->rank,
                         (const uint32_t*)rko_rows(s, s->rko_toff, L), nt, (const uint8_t*)s->rko_rb, b);
    }
    HIPCHK(hipGetLastError());
  }
  for (gm_solver* s : ss) {
    hipLaunchKernelGGL(k_rk_finish, dim3(1), dim3(1024), 0, s->stream, s->rg, s->rlvstart[0], s->st,
                       (const BlockCount*)s->bcount);
    // positions, primitives and the root word once (rank 0's, replicated);
    // edges from every rank (each counted its own slots' moves)
    if (s->rank != 0) HIPCHK(hipMemsetAsync(&s->st->red[2], 0, 2 * sizeof(u64), s->stream));
    if (s->rank != 0) HIPCHK(hipMemsetAsync(&s->st->red[0], 0, sizeof(u64), s->stream));
  }
  HIPCHK(hipGetLastError());
  if (mode == 1) {
    if (s0->gabort && s0->gabort->load(std::memory_order_acquire)) {
      cleanup();
      return fail(GM_EHIP, "RCCL group aborted: a peer shard failed (shard %d/%d)", s0->rank, s0->world);
    }
    ncclGroupStart();
    ncclResult_t r = ncclAllReduce(s0->st->red, s0->st->red, 4, ncclUint64, ncclSum, s0->comm, st);
    ncclResult_t r2 = ncclAllGather(s0->st->red + 4, s0->errg, 1, ncclUint64, s0->comm, st);
    ncclResult_t r3 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess || r3 != ncclSuccess) {
      cleanup();
      return fail(GM_EHIP, "RCCL allreduce: %s", ncclGetErrorString(r != ncclSuccess ? r : r2 != ncclSuccess ? r2 : r3));
    }
  }
  for (size_t i = 0; i < ss.size(); i++)
    if (ss[i]->stream != st) {
      HIPCHK(hipEventRecord(JE[i], ss[i]->stream));
      HIPCHK(hipStreamWaitEvent(st, JE[i], 0));
    }
  HIPCHK(hipEventRecord(e2, st));
  u64 red[5] = {0, 0, 0, 0, 0};
  for (gm_solver* s : ss) {
    u64 r[5];
    HIPCHK(hipMemcpyAsync(r, s->st->red, sizeof r, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (mode == 3) {
      std::vector<u64> all((size_t)5 * W);
      int rc = xfer_call(s, GM_XFER_ALLGATHER, r, sizeof r, -1, all.data(), all.size() * 8, -1);
      if (rc) {
        cleanup();
        return rc;
      }
      for (int q = 0; q < W; q++)
        for (int i = 0; i < 5; i++) red[i] = (i == 4) ? (red[i] | all[(size_t)q * 5 + i]) : red[i] + all[(size_t)q * 5 + i];
      continue;
    }
    if (mode == 1) {
      std::vector<u64> e((size_t)W);
      HIPCHK(hipMemcpy(e.data(), s->errg, e.size() * sizeof(u64), hipMemcpyDeviceToHost));
      r[4] = 0;
      for (u64 x : e) r[4] |= x;
    }
    for (int i = 0; i < 5; i++) red[i] = (i == 4) ? (red[i] | r[i]) : red[i] + r[i];
  }
  float f = 0, b = 0;
  HIPCHK(hipEventElapsedTime(&f, e0, e1));
  HIPCHK(hipEventElapsedTime(&b, e1, e2));
  cleanup();
  out->ms_forward = f;
  out->ms_backward = b;
  out->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  out->positions = red[0];
  out->edges = red[1];
  out->primitives = red[2];
  out->levels = T;
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

}  // extern "C++"
