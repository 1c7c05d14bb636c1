// gm_bucketed_shard.h -- BUCKETED levels sharded by the reference's own
// ownership rule, owner(pos) = md5(str(pos)) % P (GameState.get_hash,
// src/game_state.py:22-30; used by src/process.py:157-160 to route every
// LOOK_UP).  Included by gm_solver.hip after solve_bucketed.
//
// Every rank keeps the one-GPU BUCKETED structures (gm_bucketed.h) for the
// positions it owns -- unique keys per level grouped by fine bucket, words,
// in-edges -- and the per-edge LOOK_UP / RESOLVE messages of
// src/process.py:146-185 become two bulk all-to-alls per level:
//
// Forward, level L -> X = L + 1 (each rank, its own level-L positions):
//   k_bk_count<OWN>   children per OWNER rank (md5) and per parent range
//   k_bk_expand<OWN>  (child key, ref = rank << 29 | parent index) to the
//                     owner's segment of the send buffer
//   [all-to-all of keys and refs; one host read of the size matrix]
//   k_bks_hist / k_bks_part   the received records to coarse partitions
//   k_bk_fine, k_bk_dedup, k_bk_scan, k_bk_compact   as on one GPU: the
//                     owner's level X, its in-edges (ref, child in bucket)
// Backward, level L (parents) from X:
//   k_bks_answer      the owner streams X's in-edges: (parent index, child
//                     word) to the parent's rank (the ref's top bits)
//   [all-to-all back along the forward's pairs]
//   k_bks_answer_in   the parent's rank: answers to its coarse parent ranges
//   k_bk_split, k_bk_reduce   as on one GPU
// Transfers: RCCL send / recv pairs (one process per GPU), device copies (all
// shards in one process: gm_solve_group), or the host-staged transport.

extern "C++" {
// owner rank of a key on the host (the root's owner seeds level 0)
static uint32_t owner_host(const Desc& d, u64 key, uint32_t W) {
  if (W <= 1) return 0;
  uint8_t s[64], dig[16];
  const int len = str_utf8_from_key(d, key, s);
  md5_block(s, len, dig);
  return md5_mod(dig, W);
}

// received occurrences of one block's chunk -> per coarse partition counts
__global__ __launch_bounds__(kBkStreamThreads) void k_bks_hist(const u64* __restrict__ keys, u64 n, u64 chunk,
                                                              uint32_t* bh) {
  __shared__ uint32_t hc[kBkC];
  if (threadIdx.x < kBkC) hc[threadIdx.x] = 0;
  __syncthreads();
  const u64 a = (u64)blockIdx.x * chunk, e = min(n, a + chunk);
  for (u64 i = a + threadIdx.x; i < e; i += blockDim.x) atomicAdd(&hc[bk_coarse(keys[i])], 1u);
  __syncthreads();
  if (threadIdx.x < kBkC) bh[(u64)blockIdx.x * kBkC + threadIdx.x] = hc[threadIdx.x];
}

// the same chunks to their coarse partitions at exact offsets (base[c] +
// off[b][c]), with the fine byte k_bk_fine bins by, staged run by run
constexpr int kBksPartCap = 4096;
__global__ __launch_bounds__(kBkStreamThreads) void k_bks_part(const u64* __restrict__ keys,
                                                              const uint32_t* __restrict__ refs, u64 n, u64 chunk,
                                                              const uint32_t* __restrict__ off,
                                                              const uint32_t* __restrict__ base, u64* outk,
                                                              uint32_t* outp, uint8_t* outf) {
  __shared__ BkStage<u64, true, kBksPartCap> S;
  __shared__ uint32_t at[kBkC];
  if (threadIdx.x < kBkC) at[threadIdx.x] = base[threadIdx.x] + off[(u64)blockIdx.x * kBkC + threadIdx.x];
  bk_stage_init(S);
  const u64 a = (u64)blockIdx.x * chunk, e = min(n, a + chunk);
  constexpr int U = kBksPartCap / kBkStreamThreads;
  for (u64 i0 = a; i0 < e; i0 += (u64)U * blockDim.x) {  // block-uniform rounds
#pragma unroll
    for (int u = 0; u < U; u++) {
      const u64 i = i0 + (u64)u * blockDim.x + threadIdx.x;
      if (i < e) {
        const u64 k = keys[i], h = mix64(k);
        bk_stage_put(S, k, refs[i], (uint32_t)(h >> 56), (uint32_t)(h >> 48) & 0xFFu);
      }
    }
    bk_stage_flush(S, at, outk, outp, outf);
  }
}

// Owner side of the backward: block j over the in-edges of level X's fine
// buckets [j bpb, (j + 1) bpb) (bucket of a record by binary search, as
// k_bk_answer); one answer per in-edge, (parent index << 32 | child's word),
// to the parent's rank (ref >> 29), runs reserved on cur[rank]
constexpr int kBksAnswerCap = 4096;
// local-dedup refs: rank << 29 | unique local child index
constexpr uint32_t kBksRefLimit = 1u << 29;
__global__ __launch_bounds__(kBkStreamThreads) void k_bks_answer(const uint32_t* __restrict__ REp,
                                                                const uint16_t* __restrict__ REc,
                                                                const uint32_t* __restrict__ fo,
                                                                const uint32_t* __restrict__ cst, uint32_t NB,
                                                                uint32_t bpb, const uint32_t* __restrict__ WX,
                                                                uint32_t* cur, u64* out, DevState* st) {
  __shared__ BkStage<u64, false, kBksAnswerCap> S;
  __shared__ uint32_t at[kBkC], lfo[kBkC + 1], lcs[kBkC];
  const uint32_t b0 = blockIdx.x * bpb, b1 = min(NB, b0 + bpb), nb = b1 > b0 ? b1 - b0 : 0u;
  if (threadIdx.x <= nb) lfo[threadIdx.x] = fo[b0 + threadIdx.x];
  if (threadIdx.x < nb) lcs[threadIdx.x] = cst[b0 + threadIdx.x];
  bk_stage_init(S);
  if (nb == 0) return;  // block-uniform
  const uint32_t a = lfo[0], e = lfo[nb];
  constexpr int UA = kBksAnswerCap / kBkStreamThreads;
  uint32_t err = 0;
  for (uint32_t i0 = a; i0 < e; i0 += UA * blockDim.x) {  // block-uniform rounds
#pragma unroll
    for (int u = 0; u < UA; u++) {
      const uint32_t i = i0 + u * blockDim.x + threadIdx.x;
      if (i >= e) continue;
      const uint32_t ref = REp[i], c = REc[i];
      uint32_t lo = 0, hi = nb;  // bucket: lfo[lo] <= i < lfo[lo + 1]
      while (hi - lo > 1) {
        const uint32_t m = (lo + hi) >> 1;
        if (lfo[m] <= i) lo = m;
        else hi = m;
      }
      const uint32_t w = bk_pack_word(WX[lcs[lo] + c], &err);
      bk_stage_put_few(S, ((u64)(ref & 0x1FFFFFFFu) << 32) | w, 0u, ref >> 29);
    }
    bk_stage_reserve(S, at, cur, [](uint32_t b) { return b; });
    bk_stage_flush(S, at, out, (uint32_t*)nullptr);
  }
  if (err) atomicOr(&st->err, err);
}

// Parent side: the received answers [0, n) to their coarse parent ranges as
// k_bk_answer's packed records ((offset in the range << 10) | word), runs
// reserved on cur[range] (set to the ranges' first answers)
__global__ __launch_bounds__(kBkStreamThreads) void k_bks_answer_in(const u64* __restrict__ in, u64 n, u64 chunk,
                                                                   uint32_t pshift, uint32_t* cur, uint32_t* out) {
  __shared__ BkStage<uint32_t, false, kBksAnswerCap> S;
  __shared__ uint32_t at[kBkC];
  bk_stage_init(S);
  const u64 a = (u64)blockIdx.x * chunk, e = min(n, a + chunk);
  const uint32_t omask = (1u << pshift) - 1u;
  constexpr int UA = kBksAnswerCap / kBkStreamThreads;
  for (u64 i0 = a; i0 < e; i0 += (u64)UA * blockDim.x) {  // block-uniform rounds
#pragma unroll
    for (int u = 0; u < UA; u++) {
      const u64 i = i0 + (u64)u * blockDim.x + threadIdx.x;
      if (i >= e) continue;
      const u64 r = in[i];
      const uint32_t pidx = (uint32_t)(r >> 32), w = (uint32_t)r & 0x3FFu;
      bk_stage_put(S, ((pidx & omask) << 10) | w, 0u, pidx >> pshift);
    }
    bk_stage_reserve(S, at, cur, [](uint32_t b) { return b; });
    bk_stage_flush(S, at, out, (uint32_t*)nullptr);
  }
}

// Local-dedup form (GM_F_BKS_LOCAL): a rank first builds the UNIQUE children
// of its own parents with the one-GPU passes (expand, fine, LDS dedup), then
// hashes and sends each of them once.  k_bks_ownbin: block j over the local
// unique children of fine buckets [j bpb, (j + 1) bpb) -- compact index u in
// [cst[b0], cst[b1]), key at U[fo[b] + u - cst[b]] -- staged by owner rank
// (md5) and written to the owner's region [o cap, (o + 1) cap) of the send
// buffer at runs reserved on cur[o]: (key, ref = rank << 29 | u).  A region
// past cap sets *oflag (the level fails with GM_EFULL).
template <int KIND>
__global__ __launch_bounds__(kBkStreamThreads) void k_bks_ownbin(Desc d, const u64* __restrict__ U,
                                                                const uint32_t* __restrict__ fo,
                                                                const uint32_t* __restrict__ cst, uint32_t NB,
                                                                uint32_t bpb, uint32_t W, uint32_t pref, uint32_t cap,
                                                                uint32_t* cur, u64* outk, uint32_t* outr,
                                                                uint32_t* oflag) {
  __shared__ BkStage<u64, true, kBksAnswerCap> S;
  __shared__ uint32_t at[kBkC], lfo[kBkC + 1], lcs[kBkC + 1];
  const uint32_t b0 = blockIdx.x * bpb, b1 = min(NB, b0 + bpb), nb = b1 > b0 ? b1 - b0 : 0u;
  if (threadIdx.x <= nb) {
    lfo[threadIdx.x] = fo[b0 + threadIdx.x];
    lcs[threadIdx.x] = cst[b0 + threadIdx.x];
  }
  bk_stage_init(S);
  if (nb == 0) return;  // block-uniform
  const uint32_t a = lcs[0], e = lcs[nb];
  constexpr int UA = kBksAnswerCap / kBkStreamThreads;
  for (uint32_t i0 = a; i0 < e; i0 += UA * blockDim.x) {  // block-uniform rounds
#pragma unroll
    for (int u = 0; u < UA; u++) {
      const uint32_t i = i0 + u * blockDim.x + threadIdx.x;
      if (i >= e) continue;
      uint32_t lo = 0, hi = nb;  // bucket: lcs[lo] <= i < lcs[lo + 1]
      while (hi - lo > 1) {
        const uint32_t m = (lo + hi) >> 1;
        if (lcs[m] <= i) lo = m;
        else hi = m;
      }
      const u64 key = U[lfo[lo] + (i - lcs[lo])];
      if (i >= kBksRefLimit) atomicOr(&S.stop, 2u);  // the index would spill into the rank bits (the host refuses first)
      bk_stage_put_few(S, key, pref | (i & (kBksRefLimit - 1u)), owner_k<KIND>(d, key, W));
    }
    __syncthreads();
    if (threadIdx.x < W) {
      const uint32_t v = S.binc[threadIdx.x];
      if (v) {
        const uint32_t p = atomicAdd(&cur[threadIdx.x], v);
        if (p + v > cap) atomicOr(&S.stop, 1u);
        at[threadIdx.x] = threadIdx.x * cap + p;
      }
    }
    bk_stage_flush(S, at, outk, outr);
  }
  if (threadIdx.x == 0 && S.stop) atomicOr(oflag, S.stop);
}

// sender side of the local-dedup backward: the owners' answers (u << 32 |
// word) -> the words of the local unique children, Wu[u]
__global__ void k_bks_wu(const u64* __restrict__ in, u64 n, uint32_t* Wu) {
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
    const u64 r = in[i];
    Wu[r >> 32] = (uint32_t)r & 0x3FFu;
  }
}

// ---------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------
// One all-to-all of eb-byte elements: shard r sends sbuf[so[p] ..) (sc[p]
// elements) to p and receives rbuf[ro[p] ..) (rc[p]) from p.  mode 1 RCCL,
// 2 in-process copies (every shard in ss), 3 host-staged transport, 4 the
// rehearsal of mode 1 (every shard in ss, each on its own stream).
struct BksA2A {
  char* sbuf;
  char* rbuf;
  std::vector<u64> sc, so, rc, ro;
};
static int bks_alltoall(std::vector<gm_solver*>& ss, int mode, hipStream_t st, std::vector<BksA2A>& a, u64 eb) {
  const int W = ss[0]->world;
  if (mode == 4) {
    // RCCL's grouped send / receive on each rank's own stream (mode 1),
    // rehearsed with the shards on streams of their own: every sender's
    // records are final on its stream (ready[r]); each receiver's stream
    // waits for every sender and copies its incoming segments; every
    // stream then waits for every receiver (done[p]) -- a send completes
    // only with the transfer, so no rank reuses its buffers early
    for (gm_solver* s : ss)
      while (s->pev.size() < 2) {
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        s->pev.push_back(e);
      }
    for (gm_solver* s : ss) HIPCHK(hipEventRecord(s->pev[0], s->stream));
    for (int p = 0; p < W; p++) {
      gm_solver* t = ss[(size_t)p];
      for (int r = 0; r < W; r++) {
        const u64 n = a[(size_t)r].sc[(size_t)p];
        if (n != a[(size_t)p].rc[(size_t)r])
          return fail(GM_ECORRUPT, "exchange: shard %d sends %llu to %d, which expects %llu", r, (unsigned long long)n,
                      p, (unsigned long long)a[(size_t)p].rc[(size_t)r]);
        if (!n) continue;
        if (r != p) HIPCHK(hipStreamWaitEvent(t->stream, ss[(size_t)r]->pev[0], 0));
        HIPCHK(hipMemcpyAsync(a[(size_t)p].rbuf + a[(size_t)p].ro[(size_t)r] * eb,
                              a[(size_t)r].sbuf + a[(size_t)r].so[(size_t)p] * eb, n * eb, hipMemcpyDeviceToDevice,
                              t->stream));
      }
      HIPCHK(hipEventRecord(t->pev[1], t->stream));
    }
    for (gm_solver* s : ss)
      for (gm_solver* t : ss)
        if (t != s) HIPCHK(hipStreamWaitEvent(s->stream, t->pev[1], 0));
    return 0;
  }
  if (mode == 2) {
    for (int r = 0; r < W; r++)
      for (int p = 0; p < W; p++) {
        const u64 n = a[(size_t)r].sc[(size_t)p];
        if (n != a[(size_t)p].rc[(size_t)r])
          return fail(GM_ECORRUPT, "exchange: shard %d sends %llu to %d, which expects %llu", r, (unsigned long long)n,
                      p, (unsigned long long)a[(size_t)p].rc[(size_t)r]);
        if (n)
          HIPCHK(hipMemcpyAsync(a[(size_t)p].rbuf + a[(size_t)p].ro[(size_t)r] * eb,
                                a[(size_t)r].sbuf + a[(size_t)r].so[(size_t)p] * eb, n * eb, hipMemcpyDeviceToDevice, st));
      }
    return 0;
  }
  gm_solver* s = ss[0];
  BksA2A& x = a[0];
  const int r = s->rank;
  if (x.sc[(size_t)r] != x.rc[(size_t)r]) return fail(GM_ECORRUPT, "exchange: self counts differ");
  if (x.sc[(size_t)r])
    HIPCHK(hipMemcpyAsync(x.rbuf + x.ro[(size_t)r] * eb, x.sbuf + x.so[(size_t)r] * eb, x.sc[(size_t)r] * eb,
                          hipMemcpyDeviceToDevice, st));
  if (mode == 1) {
    RCCL_LIVE(s);
    ncclGroupStart();
    ncclResult_t e1 = ncclSuccess, e2 = ncclSuccess;
    for (int p = 0; p < W; p++) {
      if (p == r) continue;
      if (x.sc[(size_t)p] && e1 == ncclSuccess)
        e1 = ncclSend(x.sbuf + x.so[(size_t)p] * eb, x.sc[(size_t)p] * eb, ncclUint8, p, s->comm, st);
      if (x.rc[(size_t)p] && e2 == ncclSuccess)
        e2 = ncclRecv(x.rbuf + x.ro[(size_t)p] * eb, x.rc[(size_t)p] * eb, ncclUint8, p, s->comm, st);
    }
    const ncclResult_t e3 = ncclGroupEnd();
    if (e1 != ncclSuccess || e2 != ncclSuccess || e3 != ncclSuccess)
      return fail(GM_EHIP, "RCCL all-to-all: %s",
                  ncclGetErrorString(e1 != ncclSuccess ? e1 : e2 != ncclSuccess ? e2 : e3));
    return 0;
  }
  // host-staged: W - 1 rounds, round k pairs r -> r + k with r - k -> r
  for (int k = 1; k < W; k++) {
    const int to = (r + k) % W, from = (r - k + W) % W;
    std::vector<HostRange> out, in;
    if (x.sc[(size_t)to]) out.push_back({x.sbuf + x.so[(size_t)to] * eb, x.sc[(size_t)to] * eb});
    if (x.rc[(size_t)from]) in.push_back({x.rbuf + x.ro[(size_t)from] * eb, x.rc[(size_t)from] * eb});
    int rc = xfer_ranges(s, out, to, in, from, st);
    if (rc) return rc;
  }
  return 0;
}

// every shard's row of a W-wide u64 vector, all-gathered: out[r * W + p]
static int bks_allgather(std::vector<gm_solver*>& ss, int mode, hipStream_t st, const std::vector<std::vector<u64>>& mine,
                         std::vector<u64>& out) {
  const int W = ss[0]->world;
  const size_t m = mine[0].size();
  out.assign((size_t)W * m, 0);
  if (mode == 2 || mode == 4) {
    for (int r = 0; r < W; r++) std::copy(mine[(size_t)r].begin(), mine[(size_t)r].end(), out.begin() + (size_t)r * m);
    return 0;
  }
  gm_solver* s = ss[0];
  if (mode == 3) return xfer_call(s, GM_XFER_ALLGATHER, mine[0].data(), m * 8, -1, out.data(), out.size() * 8, -1);
  if (s->xdev_n < m + out.size()) {  // kept across levels and solves (freed with the solver)
    if (s->xdev) (void)hipFree(s->xdev);
    s->xdev = nullptr;
    s->xdev_n = 0;
    HIPCHK(hipMalloc((void**)&s->xdev, (m + out.size()) * 8));
    s->xdev_n = m + out.size();
  }
  u64* dev = s->xdev;
  RCCL_LIVE(s);
  HIPCHK(hipMemcpyAsync(dev, mine[0].data(), m * 8, hipMemcpyHostToDevice, st));
  const ncclResult_t r = ncclAllGather(dev, dev + m, m, ncclUint64, s->comm, st);
  hipError_t e = hipMemcpyAsync(out.data(), dev + m, out.size() * 8, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (r != ncclSuccess) return fail(GM_EHIP, "RCCL all-gather: %s", ncclGetErrorString(r));
  if (e != hipSuccess) return fail(GM_EHIP, "all-gather: %s", hipGetErrorString(e));
  return 0;
}

static std::vector<u64> bks_prefix(const std::vector<u64>& c) {
  std::vector<u64> o(c.size() + 1, 0);
  for (size_t i = 0; i < c.size(); i++) o[i + 1] = o[i] + c[i];
  return o;
}

// The sharded BUCKETED solve: every shard of the job in ss (mode 2), or
// this process's one shard (mode 1 RCCL / 3 host transport).  Whole solves
// only (no steps, no kernel timing).
static int run_bucketed_shards(std::vector<gm_solver*> ss, gm_result* out) {
  gm_solver* s0 = ss[0];
  const Desc& d = s0->d;
  const int T = d.max_levels, W = s0->world;
  // mode 2: a group on one stream; mode 4: a group whose shards run on
  // streams of their own -- mode 1's per-rank stream order, the all-to-alls
  // as device copies between the shards' streams (bks_alltoall)
  const bool own_streams = ss.size() > 1 && ss[1]->stream != s0->stream;
  const int mode = ss.size() != 1 ? (own_streams ? 4 : 2) : s0->xfer ? 3 : 1;
  if (mode == 1 && !s0->comm) return fail(GM_EINVAL, "shard %d/%d has no communicator (gm_solver_comm_init)", s0->rank, W);
  if (mode == 2 || mode == 4) {
    if ((int)ss.size() != W) return fail(GM_EINVAL, "group solve needs all %d shards", W);
    for (size_t g = 0; g < ss.size(); g++) {
      if (ss[g]->rank != (int)g || ss[g]->mode != GM_MODE_BUCKETED)
        return fail(GM_EINVAL, "group shards must be ranks 0..n-1");
      for (size_t h = 0; h < g; h++)
        if ((mode == 2) != (ss[g]->stream == ss[h]->stream))
          return fail(GM_EINVAL, "group shards share one stream, or (the RCCL rehearsal) each has its own");
    }
  }
  if (s0->step_first || s0->step_stop) return fail(GM_EINVAL, "sharded bucketed solves run whole (no steps)");
  // Which form a level's children take: the local-dedup form pays an extra
  // host sync and a second dedup per level, won back where a shard expands
  // many parents (toot 6x4 on 2 shards 500 -> 356 ms; toot 5x4 on 8 shards,
  // ~0.5 M parents per level and shard, 64 -> 74 ms).  Default: local for a
  // level whose largest shard expands >= kBksLocalMin parents (2 M: toot 5x4 on 4 and 8 shards ran 1-4 ms
  // slower with 1 M); GM_F_BKS_LOCAL:
  // every level.  Ranks may decide differently (the owners' side is the same
  // in both forms; each rank reads its answers by its own choice).
  constexpr u64 kBksLocalMin = 1ull << 21;
  const bool local_all = (s0->flags & GM_F_BKS_LOCAL) != 0;
  // lmax[L]: the largest shard's level L, known to EVERY rank (all-gathered
  // with the level sizes in modes 1 / 3), so all ranks pick the same form --
  // the one the in-process group, which the tests run, picks
  std::vector<u64> lmax((size_t)T, 0);
  lmax[0] = 1;
  auto local_level = [&](int L) { return local_all || lmax[(size_t)L] >= kBksLocalMin; };
  hipStream_t st = s0->stream;
  auto sync_all = [&]() -> hipError_t {  // every shard's stream (one stream in modes 1-3)
    for (gm_solver* s : ss) {
      const hipError_t e = hipStreamSynchronize(s->stream);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  };
  auto t0 = std::chrono::steady_clock::now();
  hipEvent_t e0, e1, e2;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  HIPCHK(hipEventCreate(&e2));
  auto done_events = [&]() {
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipEventDestroy(e2);
  };
  auto bail = [&](int code) {
    (void)sync_all();
    done_events();
    return code;
  };
  HIPCHK(hipEventRecord(e0, st));
  if (mode == 4) HIPCHK(sync_all());  // the shards' streams start after e0 (host order)
  // the root's owner seeds level 0
  const uint32_t root_owner = owner_host(d, d.root, (uint32_t)W);
  for (gm_solver* s : ss) {
    HIPCHK(hipMemsetAsync(s->st, 0, devstate_bytes(T), s->stream));
    HIPCHK(hipMemsetAsync(s->bkL, 0, sizeof(BkLevel) * (size_t)T, s->stream));
    s->lvh.assign((size_t)T, BkLevel{});
    s->lvh[0].n = s->rank == (int)root_owner ? 1 : 0;
    HIPCHK(hipMemcpyAsync(s->bkK, &s->d.root, sizeof(u64), hipMemcpyHostToDevice, s->stream));
    s->bks_sc.assign((size_t)T, std::vector<u64>((size_t)W, 0));
    s->bksl.assign((size_t)T, gm_solver::BksLocal{});
    s->bks_rc.assign((size_t)T, std::vector<u64>((size_t)W, 0));
  }
  std::vector<std::vector<uint32_t>> keep;  // host arrays of async H2D copies
  // A failure on one rank must not leave the others waiting in an exchange:
  // it is recorded (prc / perr) and travels in the next all-gathered row, and
  // every rank returns together.
  int prc = 0;
  std::string perr;
  u64 host_err = 0;  // error bits found on the host (sent with the final totals)
  auto defer = [&](int code) {
    if (!prc) {
      prc = code;
      perr = g_err;
    }
  };
  // row of the per-level all-gather: sends per rank, status, Emax, edge room
  auto status_of = [&](const std::vector<u64>& all, size_t m) -> int {
    for (int r = 0; r < W; r++)
      if (all[(size_t)r * m + (size_t)W]) {
        const int code = (int)(int64_t)all[(size_t)r * m + (size_t)W];
        if (prc) g_err = perr;
        return prc ? prc : fail(code, "shard %d failed", r);
      }
    return 0;
  };
  // Local-dedup forward of level L (GM_F_BKS_LOCAL): per shard the one-GPU
  // count-free expand of its own parents into coarse partitions, the fine
  // pass (the local in-edges' parents, REpl), the LDS dedup (REcl) and the
  // unique local children binned by owner (k_bks_ownbin, one MD5 each) into
  // the send regions; then the size matrix and the all-to-all as the
  // occurrence form.  Two host syncs for all shards, plus the size matrix.
  auto forward_local = [&](int L, std::vector<u64>& meta_at) -> int {
    struct Q {
      std::vector<uint32_t> g;
      uint32_t herr = 0, cap = 0;
      u64 NR = 0, nblk = 0, chunk = 0;
      bool active = false;
    };
    std::vector<Q> q(ss.size());
    for (size_t gi = 0; gi < ss.size(); gi++) {
      gm_solver* s = ss[gi];
      std::vector<BkLevel>& lv = s->lvh;
      BkLevel& P = lv[(size_t)L];
      BkLevel& X = lv[(size_t)L + 1];
      u64 meta_used = 0;
      for (int i = 0; i <= L; i++) {
        const BkLevel& Qv = lv[(size_t)i];
        if (Qv.nbits) meta_used = std::max<u64>(meta_used, Qv.cst_off + 2 * ((1ull << Qv.nbits) + 1));
        if (i < L && Qv.eout) meta_used = std::max<u64>(meta_used, Qv.rfo_off + ((Qv.n + (1ull << Qv.fb) - 1) >> Qv.fb) + 1);
        const gm_solver::BksLocal& B = s->bksl[(size_t)i];
        if (i < L && B.nbits) meta_used = std::max<u64>(meta_used, B.cst_off + 2 * ((1ull << B.nbits) + 1));
      }
      X = BkLevel{};
      X.lb = P.lb + P.n;
      X.rb = P.rb + P.ein;
      P.eout = 0;
      gm_solver::BksLocal& B = s->bksl[(size_t)L];
      B = gm_solver::BksLocal{};
      B.used = true;
      for (int i = 0; i < L; i++) B.rb = std::max<u64>(B.rb, s->bksl[(size_t)i].rb + s->bksl[(size_t)i].ein);
      Q& z = q[gi];
      z.g.assign(2 * kBkC + 1, 0);
      if (!bk_ranges(P.n, &P.pshift, &P.fb))
        defer(fail(GM_ELIMIT, "level %d holds %llu positions: more than a bucketed level supports", L,
                   (unsigned long long)P.n));
      meta_at[gi] = meta_used;
      if (!P.n || prc) continue;
      z.nblk = std::min<u64>(kBkExpandBlocks, (P.n + kBkExpandThreads - 1) / kBkExpandThreads);
      z.chunk = (P.n + z.nblk - 1) / z.nblk;
      z.NR = (P.n + (1ull << P.fb) - 1) >> P.fb;
      if (meta_used + z.NR + 1 > s->meta_cap) {
        defer(fail(GM_ECORRUPT, "bucket tables exceed the scratch"));
        continue;
      }
      P.rfo_off = (uint32_t)meta_used;
      meta_used += z.NR + 1;
      meta_at[gi] = meta_used;
      z.active = true;
      uint32_t* rfo = s->meta + P.rfo_off;
      uint32_t ck_sh = 14;
      while (ck_sh > 6 && (s->Emax / kBkC) < (1ull << ck_sh)) ck_sh--;
      z.cap = (uint32_t)((s->Emax / kBkC) >> ck_sh << ck_sh);
      const BkChunked ck{(char*)s->S1k, ck_sh};
      HIPCHK(hipMemsetAsync(rfo, 0, (z.NR + 1) * 4, s->stream));
      HIPCHK(hipMemsetAsync(s->bkgc, 0, (2 * kBkC + 4) * 4, s->stream));
      const double avg =
          (L > 0 && s->lvh[(size_t)L - 1].n) ? std::max(1.0, (double)s->lvh[(size_t)L - 1].eout / (double)s->lvh[(size_t)L - 1].n)
                                              : 4.0;
      bk_dispatch(s->d, [&](auto kind_) {
        constexpr int K_ = decltype(kind_)::value;
        hipLaunchKernelGGL((k_bk_expand<K_, true>), dim3(z.nblk), dim3(kBkExpandThreads), 0, s->stream, s->d, s->bkK + P.lb,
                           P.n, z.chunk, (const uint32_t*)nullptr, (const uint32_t*)nullptr, bk_ppr(avg), s->S1k, s->S1p,
                           s->S1f, z.cap, s->bkgc, P.pshift, P.fb, s->bkgc + kBkC, rfo, s->bkgc + 2 * kBkC, s->st, ck);
      });
      hipLaunchKernelGGL(k_bk_scan, dim3(1), dim3(1024), 0, s->stream, rfo, (uint32_t)z.NR + 1, rfo, s->bktotal + 1);
      HIPCHK(hipGetLastError());
      HIPCHK(hipMemcpyAsync(z.g.data(), s->bkgc, z.g.size() * 4, hipMemcpyDeviceToHost, s->stream));
      HIPCHK(hipMemcpyAsync(&z.herr, &s->st->err, 4, hipMemcpyDeviceToHost, s->stream));
    }
    HIPCHK(sync_all());
    std::vector<std::vector<uint32_t>> oc(ss.size(), std::vector<uint32_t>((size_t)W + 1, 0));
    std::vector<u64> nu(ss.size(), 0);
    std::vector<uint32_t> derr(ss.size(), 0);
    for (size_t gi = 0; gi < ss.size(); gi++) {
      gm_solver* s = ss[gi];
      Q& z = q[gi];
      if (!z.active) continue;
      BkLevel& P = s->lvh[(size_t)L];
      gm_solver::BksLocal& B = s->bksl[(size_t)L];
      if (z.herr) {
        defer(fail(GM_ECORRUPT, "shard %d level %d:%s", s->rank, L, err_text(z.herr).c_str()));
        z.active = false;
        continue;
      }
      if (z.g[2 * kBkC]) {  // a coarse partition past its provisioned share
        defer(fail(GM_EFULL, "shard %d level %d: a partition of the local children exceeds its share", s->rank, L));
        z.active = false;
        continue;
      }
      keep.emplace_back(2 * (kBkC + 1));
      std::vector<uint32_t>& hb = keep.back();
      u64 E = 0, Ep = 0;
      for (int j = 0; j < kBkC; j++) {
        hb[(size_t)j] = (uint32_t)E;
        hb[(size_t)kBkC + 1 + j] = (uint32_t)Ep;
        E += z.g[(size_t)j];
        Ep += z.g[(size_t)kBkC + j];
      }
      hb[(size_t)kBkC] = (uint32_t)E;
      hb[(size_t)2 * kBkC + 1] = (uint32_t)Ep;
      if (E != Ep) defer(fail(GM_ECORRUPT, "shard %d level %d: %llu children by partition, %llu by parent", s->rank, L,
                              (unsigned long long)E, (unsigned long long)Ep));
      if (E > s->Emax || B.rb + E > s->Ecap)
        defer(fail(GM_EFULL, "shard %d level %d: %llu local children exceed the plan", s->rank, L, (unsigned long long)E));
      // the refs sent to the owners pack rank << 29 | unique index, and the
      // unique children are at most the E occurrences
      if (E >= kBksRefLimit)
        defer(fail(GM_ELIMIT, "shard %d level %d: %llu local children; the local-dedup form indexes fewer than 2^29",
                   s->rank, L, (unsigned long long)E));
      if (prc || !E) {
        z.active = false;
        continue;
      }
      P.eout = E;
      B.ein = E;
      HIPCHK(hipMemcpyAsync(s->cbase, hb.data(), (kBkC + 1) * 4, hipMemcpyHostToDevice, s->stream));
      HIPCHK(hipMemcpyAsync(s->pbase + (size_t)L * (kBkC + 1), hb.data() + kBkC + 1, (kBkC + 1) * 4,
                            hipMemcpyHostToDevice, s->stream));
      uint32_t f = 0;
      while (f < (uint32_t)kBkMaxFineBits && (E >> f) > (u64)kBkC * 4096) f++;
      const uint32_t F = 1u << f, NB = (uint32_t)kBkC << f;
      if (meta_at[gi] + 2 * (NB + 1) > s->meta_cap) {
        defer(fail(GM_ECORRUPT, "bucket tables exceed the scratch"));
        z.active = false;
        continue;
      }
      B.nbits = 8 + f;
      B.cst_off = (uint32_t)meta_at[gi];
      meta_at[gi] += 2 * (NB + 1);
      uint32_t* cst = s->meta + B.cst_off;
      uint32_t* fo = cst + NB + 1;
      uint32_t ck_sh = 14;
      while (ck_sh > 6 && (s->Emax / kBkC) < (1ull << ck_sh)) ck_sh--;
      const BkChunked ck{(char*)s->S1k, ck_sh};
      hipLaunchKernelGGL(k_bk_fine, dim3(kBkC), dim3(kBkFineThreads), 0, s->stream, (const u64*)s->S1k, (const uint32_t*)s->S1p,
                         (const uint8_t*)s->S1f, (const uint32_t*)s->cbase, 8u - f, F, s->S2k, s->REpl + B.rb, fo,
                         P.pshift, s->bkah + (size_t)L * kBkC * kBkC, z.cap, ck);
      const int gd = (int)std::min<uint32_t>(NB, 512);
      hipLaunchKernelGGL(k_bk_dedup, dim3(gd), dim3(kBkDedupThreads), 0, s->stream, s->S2k, (const uint32_t*)fo, NB, s->S1k,
                         s->ucnt, s->REcl + B.rb, s->st);
      hipLaunchKernelGGL(k_bk_scan, dim3(1), dim3(1024), 0, s->stream, s->ucnt, NB, cst, s->bktotal);
      HIPCHK(hipMemsetAsync(s->bkgc, 0, (2 * kBkC + 4) * 4, s->stream));
      const uint32_t capd = (uint32_t)(s->Emax / (u64)W);
      bk_dispatch(s->d, [&](auto kind_) {
        constexpr int K_ = decltype(kind_)::value;
        hipLaunchKernelGGL((k_bks_ownbin<K_>), dim3(kBkC), dim3(kBkStreamThreads), 0, s->stream, s->d, (const u64*)s->S1k,
                           (const uint32_t*)fo, (const uint32_t*)cst, NB, F, (uint32_t)W, (uint32_t)s->rank << 29, capd,
                           s->bkgc, s->XSk, s->XSr, s->bkgc + 2 * kBkC);
      });
      HIPCHK(hipGetLastError());
      HIPCHK(hipMemcpyAsync(oc[gi].data(), s->bkgc, (size_t)W * 4, hipMemcpyDeviceToHost, s->stream));
      HIPCHK(hipMemcpyAsync(&oc[gi][(size_t)W], s->bkgc + 2 * kBkC, 4, hipMemcpyDeviceToHost, s->stream));
      HIPCHK(hipMemcpyAsync(&nu[gi], s->bktotal, 8, hipMemcpyDeviceToHost, s->stream));
      HIPCHK(hipMemcpyAsync(&derr[gi], &s->st->err, 4, hipMemcpyDeviceToHost, s->stream));
    }
    HIPCHK(sync_all());
    std::vector<std::vector<u64>> sendc(ss.size(), std::vector<u64>((size_t)W + 3, 0));
    for (size_t gi = 0; gi < ss.size(); gi++) {
      gm_solver* s = ss[gi];
      Q& z = q[gi];
      if (z.active) {
        if (derr[gi]) {
          const bool lim = derr[gi] & ERR_BUCKET_FULL;
          defer(fail(lim ? GM_ELIMIT : GM_ECORRUPT, "shard %d level %d:%s", s->rank, L + 1, err_text(derr[gi]).c_str()));
        } else if (oc[gi][(size_t)W] & 2u) {
          defer(fail(GM_ELIMIT, "shard %d level %d: a unique child index reached 2^29", s->rank, L));
        } else if (oc[gi][(size_t)W]) {
          defer(fail(GM_EFULL, "shard %d level %d: an owner's region of unique children overflowed", s->rank, L));
        } else {
          u64 t = 0;
          for (int p = 0; p < W; p++) t += oc[gi][(size_t)p];
          if (t != nu[gi]) defer(fail(GM_ECORRUPT, "shard %d level %d: %llu unique children, %llu binned", s->rank, L,
                                      (unsigned long long)nu[gi], (unsigned long long)t));
          s->bksl[(size_t)L].nu = nu[gi];
          for (int p = 0; p < W; p++) sendc[gi][(size_t)p] = oc[gi][(size_t)p];
        }
      }
      sendc[gi][(size_t)W] = (u64)(int64_t)prc;
      sendc[gi][(size_t)W + 1] = s->Emax;
      sendc[gi][(size_t)W + 2] = s->Ecap - std::min(s->Ecap, s->lvh[(size_t)L + 1].rb);
    }
    // the size matrix (with every rank's status and room), then the records
    std::vector<u64> MA;
    int rc = bks_allgather(ss, mode, st, sendc, MA);
    if (rc) return rc;
    if ((rc = status_of(MA, (size_t)W + 3))) return rc;
    const size_t m3 = (size_t)W + 3;
    for (int p = 0; p < W; p++) {
      u64 in = 0, outn = 0;
      for (int r = 0; r < W; r++) {
        in += MA[(size_t)r * m3 + p];
        outn += MA[(size_t)p * m3 + r];
      }
      const u64 emax = MA[(size_t)p * m3 + W + 1], room = MA[(size_t)p * m3 + W + 2];
      if (in > emax || outn > emax || in > room)
        return fail(GM_EFULL, "level %d: shard %d sends %llu / receives %llu records; its plan holds %llu per level and "
                              "%llu more edges", L, p, (unsigned long long)outn, (unsigned long long)in,
                    (unsigned long long)emax, (unsigned long long)room);
    }
    std::vector<BksA2A> ak(ss.size()), ar(ss.size());
    for (size_t gi = 0; gi < ss.size(); gi++) {
      gm_solver* s = ss[gi];
      const int r = s->rank;
      std::vector<u64>& sc = s->bks_sc[(size_t)L];
      std::vector<u64>& rcv = s->bks_rc[(size_t)L];
      for (int p = 0; p < W; p++) {
        sc[(size_t)p] = MA[(size_t)r * m3 + p];
        rcv[(size_t)p] = MA[(size_t)p * m3 + r];
      }
      std::vector<u64> so((size_t)W + 1, 0);
      for (int p = 0; p < W; p++) so[(size_t)p] = (u64)p * (s->Emax / (u64)W);  // owner p's records at [p cap, ...)
      const std::vector<u64> ro = bks_prefix(rcv);
      s->lvh[(size_t)L + 1].ein = ro[(size_t)W];
      ak[gi] = BksA2A{(char*)s->XSk, (char*)s->XRk, sc, std::vector<u64>(so.begin(), so.end() - 1), rcv,
                      std::vector<u64>(ro.begin(), ro.end() - 1)};
      ar[gi] = ak[gi];
      ar[gi].sbuf = (char*)s->XSr;
      ar[gi].rbuf = (char*)s->XRr;
    }
    if ((rc = bks_alltoall(ss, mode, st, ak, 8)) || (rc = bks_alltoall(ss, mode, st, ar, 4))) return rc;
    return 0;
  };
  // ---- forward ----
  for (int L = 0; L + 1 < T; L++) {
    // (a) per shard: children per owner and per parent range
    std::vector<u64> meta_at(ss.size(), 0);
    const bool local = local_level(L);
    for (gm_solver* s : ss) s->bksl[(size_t)L].used = local;
    if (local) {
      int rc = forward_local(L, meta_at);
      if (rc) return bail(rc);
    } else {
    std::vector<std::vector<u64>> sendc(ss.size());
    std::vector<u64> ptot_all(ss.size() * kBkC, 0);
    std::vector<char> over(ss.size(), 0);  // the count-free expand already filled the send regions
    // every shard's launches first, then ONE host sync for all of them (and
    // a second only when some owner region overflowed)
    struct Pending {
      std::vector<uint32_t> htot;
      uint32_t herr = 0;
      bool active = false, exact = false;
      u64 nblk = 0, chunk = 0;
      uint32_t NR = 0;
    };
    std::vector<Pending> pd(ss.size());
    for (size_t g = 0; g < ss.size(); g++) {
      gm_solver* s = ss[g];
      std::vector<BkLevel>& lv = s->lvh;
      BkLevel& P = lv[(size_t)L];
      BkLevel& X = lv[(size_t)L + 1];
      u64 meta_used = 0;
      for (int i = 0; i <= L; i++) {
        const BkLevel& Q = lv[(size_t)i];
        if (Q.nbits) meta_used = std::max<u64>(meta_used, Q.cst_off + 2 * ((1ull << Q.nbits) + 1));
        if (i < L && Q.eout) meta_used = std::max<u64>(meta_used, Q.rfo_off + ((Q.n + (1ull << Q.fb) - 1) >> Q.fb) + 1);
        const gm_solver::BksLocal& B = s->bksl[(size_t)i];  // an earlier level's local-dedup tables
        if (i < L && B.nbits) meta_used = std::max<u64>(meta_used, B.cst_off + 2 * ((1ull << B.nbits) + 1));
      }
      X = BkLevel{};
      X.lb = P.lb + P.n;
      X.rb = P.rb + P.ein;
      P.eout = 0;
      sendc[g].assign((size_t)W + 3, 0);
      Pending& q = pd[g];
      q.htot.assign(2 * kBkC + 1, 0);
      if (!bk_ranges(P.n, &P.pshift, &P.fb))
        defer(fail(GM_ELIMIT, "level %d holds %llu positions: more than a bucketed level supports", L,
                   (unsigned long long)P.n));
      if (P.n && !prc) {
        q.nblk = std::min<u64>(kBkExpandBlocks, (P.n + kBkExpandThreads - 1) / kBkExpandThreads);
        q.chunk = (P.n + q.nblk - 1) / q.nblk;
        q.NR = (uint32_t)((P.n + (1ull << P.fb) - 1) >> P.fb);
        if (meta_used + q.NR + 1 > s->meta_cap) defer(fail(GM_ECORRUPT, "bucket tables exceed the scratch"));
        P.rfo_off = (uint32_t)meta_used;
        meta_used += q.NR + 1;
        q.active = !prc;
        q.exact = (s->flags & GM_F_BK_EXACT) != 0;
      }
      meta_at[g] = meta_used;
      if (!q.active || q.exact) continue;
      // Count-free form first: the children go straight to per-owner
      // regions of the send buffer (one MD5 per child); an owner past its
      // region (Emax / W records) -> count, then the exact form in (c).
      uint32_t* rfo = s->meta + P.rfo_off;
      HIPCHK(hipMemsetAsync(rfo, 0, (q.NR + 1) * 4, s->stream));
      HIPCHK(hipMemsetAsync(s->bkgc, 0, (2 * kBkC + 4) * 4, s->stream));
      const double avg =  // children per parent of the level before (this shard's own)
          (L > 0 && s->lvh[(size_t)L - 1].n) ? std::max(1.0, (double)s->lvh[(size_t)L - 1].eout / (double)s->lvh[(size_t)L - 1].n)
                                              : 4.0;
      const uint32_t capd = (uint32_t)(s->Emax / (u64)W);
      bk_dispatch(s->d, [&](auto kind_) {
        constexpr int K_ = decltype(kind_)::value;
        hipLaunchKernelGGL((k_bk_expand<K_, true, true>), dim3(q.nblk), dim3(kBkExpandThreads), 0, s->stream, s->d,
                           s->bkK + P.lb, P.n, q.chunk, (const uint32_t*)nullptr, (const uint32_t*)nullptr, bk_ppr(avg),
                           s->XSk, s->XSr, (uint8_t*)nullptr, capd, s->bkgc, P.pshift, P.fb, s->bkgc + kBkC, rfo,
                           s->bkgc + 2 * kBkC, s->st, BkChunked{nullptr, 0}, (uint32_t)W, (uint32_t)s->rank << 29);
      });
      hipLaunchKernelGGL(k_bk_scan, dim3(1), dim3(1024), 0, s->stream, rfo, q.NR + 1, rfo, s->bktotal + 1);
      HIPCHK(hipGetLastError());
      HIPCHK(hipMemcpyAsync(q.htot.data(), s->bkgc, q.htot.size() * 4, hipMemcpyDeviceToHost, s->stream));
      HIPCHK(hipMemcpyAsync(&q.herr, &s->st->err, 4, hipMemcpyDeviceToHost, s->stream));
    }
    HIPCHK(sync_all());
    bool any_exact = false;
    for (size_t g = 0; g < ss.size(); g++) {
      gm_solver* s = ss[g];
      Pending& q = pd[g];
      if (!q.active) continue;
      if (!q.exact) {
        if (q.htot[2 * kBkC] && !q.herr) q.exact = true;  // an owner region overflowed: redo the level counted
        else over[g] = 1;
      }
      if (!q.exact || q.herr) continue;
      any_exact = true;
      BkLevel& P = s->lvh[(size_t)L];
      uint32_t* rfo = s->meta + P.rfo_off;
      HIPCHK(hipMemsetAsync(rfo, 0, (q.NR + 1) * 4, s->stream));
      bk_dispatch(s->d, [&](auto kind_) {
        constexpr int K_ = decltype(kind_)::value;
        hipLaunchKernelGGL((k_bk_count<K_, true>), dim3(q.nblk), dim3(kBkStreamThreads), 0, s->stream, s->d, s->bkK + P.lb,
                           P.n, q.chunk, P.pshift, P.fb, s->bh, s->ph, rfo, s->st, (uint32_t)W);
      });
      hipLaunchKernelGGL(k_bk_colscan, dim3(kBkC), dim3(256), 0, s->stream, s->bh, (uint32_t)q.nblk, s->boff, s->tot);
      hipLaunchKernelGGL(k_bk_colscan, dim3(kBkC), dim3(256), 0, s->stream, s->ph, (uint32_t)q.nblk, s->ph, s->tot + kBkC);
      hipLaunchKernelGGL(k_bk_scan, dim3(1), dim3(1024), 0, s->stream, rfo, q.NR + 1, rfo, s->bktotal + 1);
      HIPCHK(hipGetLastError());
      HIPCHK(hipMemcpyAsync(q.htot.data(), s->tot, 2 * kBkC * 4, hipMemcpyDeviceToHost, s->stream));
      HIPCHK(hipMemcpyAsync(&q.herr, &s->st->err, 4, hipMemcpyDeviceToHost, s->stream));
    }
    if (any_exact) HIPCHK(sync_all());
    for (size_t g = 0; g < ss.size(); g++) {
      gm_solver* s = ss[g];
      Pending& q = pd[g];
      if (q.active) {
        if (q.herr) defer(fail(GM_ECORRUPT, "shard %d level %d:%s", s->rank, L, err_text(q.herr).c_str()));
        for (int p = 0; p < W; p++) sendc[g][(size_t)p] = q.htot[(size_t)p];
        for (int j = 0; j < kBkC; j++) ptot_all[g * kBkC + (size_t)j] = q.htot[(size_t)kBkC + j];
      }
      sendc[g][(size_t)W] = (u64)(int64_t)prc;
      sendc[g][(size_t)W + 1] = s->Emax;
      sendc[g][(size_t)W + 2] = s->Ecap - std::min(s->Ecap, s->lvh[(size_t)L + 1].rb);
    }
    // (b) the size matrix (with every rank's status and room)
    std::vector<u64> MA;
    int rc = bks_allgather(ss, mode, st, sendc, MA);
    if (rc) return bail(rc);
    if ((rc = status_of(MA, (size_t)W + 3))) return bail(rc);
    const size_t m3 = (size_t)W + 3;
    for (int p = 0; p < W; p++) {  // every rank checks every rank's room: all fail together
      u64 in = 0, outn = 0;
      for (int r = 0; r < W; r++) {
        in += MA[(size_t)r * m3 + p];
        outn += MA[(size_t)p * m3 + r];
      }
      const u64 emax = MA[(size_t)p * m3 + W + 1], room = MA[(size_t)p * m3 + W + 2];
      if (in > emax || outn > emax || in > room)
        return bail(fail(GM_EFULL, "level %d: shard %d sends %llu / receives %llu records; its plan holds %llu per "
                                   "level and %llu more edges", L, p, (unsigned long long)outn, (unsigned long long)in,
                         (unsigned long long)emax, (unsigned long long)room));
    }
    std::vector<u64> M((size_t)W * W);
    for (int r = 0; r < W; r++)
      for (int p = 0; p < W; p++) M[(size_t)r * W + p] = MA[(size_t)r * m3 + p];
    // (c) per shard: expand into the owners' segments
    std::vector<BksA2A> ak(ss.size()), ar(ss.size());
    for (size_t g = 0; g < ss.size(); g++) {
      gm_solver* s = ss[g];
      const int r = s->rank;
      BkLevel& P = s->lvh[(size_t)L];
      BkLevel& X = s->lvh[(size_t)L + 1];
      std::vector<u64>& sc = s->bks_sc[(size_t)L];
      std::vector<u64>& rcv = s->bks_rc[(size_t)L];
      for (int p = 0; p < W; p++) {
        sc[(size_t)p] = M[(size_t)r * W + p];
        rcv[(size_t)p] = M[(size_t)p * W + r];
      }
      std::vector<u64> so = bks_prefix(sc);
      const std::vector<u64> ro = bks_prefix(rcv);
      const u64 Eout = so[(size_t)W], Ein = ro[(size_t)W];
      if (over[g])  // owner p's records sit at [p cap, ...) of the send buffer
        for (int p = 0; p < W; p++) so[(size_t)p] = (u64)p * (s->Emax / (u64)W);
      u64 Ep = 0;
      for (int j = 0; j < kBkC; j++) Ep += ptot_all[g * kBkC + (size_t)j];
      if (Eout != Ep)  // an internal inconsistency of this rank's own counts: recorded, reported at the end
        defer(fail(GM_ECORRUPT, "shard %d level %d: %llu children by owner, %llu by parent", r, L,
                   (unsigned long long)Eout, (unsigned long long)Ep));
      P.eout = Eout;
      X.ein = Ein;
      // parent-range bases (backward: where each coarse range's answers go)
      keep.emplace_back(2 * (kBkC + 1));
      std::vector<uint32_t>& hb = keep.back();  // [owner-segment bases | parent-range bases]
      u64 acc = 0;
      for (int j = 0; j < kBkC; j++) {
        hb[(size_t)j] = (uint32_t)(j < W ? so[(size_t)j] : Eout);
        hb[(size_t)kBkC + 1 + j] = (uint32_t)acc;
        acc += ptot_all[g * kBkC + (size_t)j];
      }
      hb[(size_t)kBkC] = (uint32_t)Eout;
      hb[(size_t)2 * kBkC + 1] = (uint32_t)acc;
      HIPCHK(hipMemcpyAsync(s->cbase, hb.data(), (kBkC + 1) * 4, hipMemcpyHostToDevice, s->stream));
      HIPCHK(hipMemcpyAsync(s->pbase + (size_t)L * (kBkC + 1), hb.data() + kBkC + 1, (kBkC + 1) * 4,
                            hipMemcpyHostToDevice, s->stream));
      if (P.n && Eout && !over[g]) {
        const u64 nblk = std::min<u64>(kBkExpandBlocks, (P.n + kBkExpandThreads - 1) / kBkExpandThreads),
                  chunk = (P.n + nblk - 1) / nblk;
        const uint32_t ppr = bk_ppr((double)Eout / (double)P.n);
        bk_dispatch(s->d, [&](auto kind_) {
          constexpr int K_ = decltype(kind_)::value;
          hipLaunchKernelGGL((k_bk_expand<K_, false, true>), dim3(nblk), dim3(kBkExpandThreads), 0, s->stream, s->d,
                             s->bkK + P.lb, P.n, chunk, (const uint32_t*)s->boff, (const uint32_t*)s->cbase, ppr, s->XSk,
                             s->XSr, (uint8_t*)nullptr, 0u, (uint32_t*)nullptr, 0u, 0u, (uint32_t*)nullptr,
                             (uint32_t*)nullptr, (uint32_t*)nullptr, s->st, BkChunked{nullptr, 0}, (uint32_t)W,
                             (uint32_t)r << 29);
        });
        HIPCHK(hipGetLastError());
      }
      ak[g] = BksA2A{(char*)s->XSk, (char*)s->XRk, sc, std::vector<u64>(so.begin(), so.end() - 1), rcv,
                     std::vector<u64>(ro.begin(), ro.end() - 1)};
      ar[g] = ak[g];
      ar[g].sbuf = (char*)s->XSr;
      ar[g].rbuf = (char*)s->XRr;
    }
    if ((rc = bks_alltoall(ss, mode, st, ak, 8)) || (rc = bks_alltoall(ss, mode, st, ar, 4))) return bail(rc);
    }  // !local
    // (d) per shard: the received occurrences -> level X
    std::vector<u64> ncnt(ss.size(), 0);
    for (size_t g = 0; g < ss.size(); g++) {
      gm_solver* s = ss[g];
      BkLevel& P = s->lvh[(size_t)L];
      BkLevel& X = s->lvh[(size_t)L + 1];
      const u64 E = X.ein;
      u64 meta_used = meta_at[g];
      if (!E) continue;
      if (prc) {  // a failed rank moves no more data: its level stays empty until the status travels
        X.ein = 0;
        continue;
      }
      uint32_t f = 0;
      while (f < (uint32_t)kBkMaxFineBits && (E >> f) > (u64)kBkC * 4096) f++;
      const uint32_t F = 1u << f, NB = (uint32_t)kBkC << f;
      X.nbits = 8 + f;
      if (meta_used + 2 * (NB + 1) > s->meta_cap) {
        defer(fail(GM_ECORRUPT, "bucket tables exceed the scratch"));
        X.ein = 0;
        continue;
      }
      X.cst_off = (uint32_t)meta_used;
      uint32_t* cst = s->meta + X.cst_off;
      uint32_t* fo = cst + NB + 1;
      const u64 nblk = std::min<u64>(kBkExpandBlocks, (E + kBksPartCap - 1) / kBksPartCap), chunk = (E + nblk - 1) / nblk;
      hipLaunchKernelGGL(k_bks_hist, dim3(nblk), dim3(kBkStreamThreads), 0, s->stream, (const u64*)s->XRk, E, chunk, s->bh);
      hipLaunchKernelGGL(k_bk_colscan, dim3(kBkC), dim3(256), 0, s->stream, s->bh, (uint32_t)nblk, s->boff, s->tot);
      hipLaunchKernelGGL(k_bk_scan, dim3(1), dim3(1024), 0, s->stream, s->tot, (uint32_t)kBkC, s->cbase, s->bktotal + 1);
      hipLaunchKernelGGL(k_bks_part, dim3(nblk), dim3(kBkStreamThreads), 0, s->stream, (const u64*)s->XRk,
                         (const uint32_t*)s->XRr, E, chunk, (const uint32_t*)s->boff, (const uint32_t*)s->cbase, s->S1k,
                         s->S1p, s->S1f);
      // refs ride in the parent slot: pshift 31 puts every record in parent range 0 of ah, whose counts
      // nothing reads -- the last level's ah (no level expands from it), so the local-dedup form's
      // parent-range counts of level L stay intact
      hipLaunchKernelGGL(k_bk_fine, dim3(kBkC), dim3(kBkFineThreads), 0, s->stream, (const u64*)s->S1k, (const uint32_t*)s->S1p,
                         (const uint8_t*)s->S1f, (const uint32_t*)s->cbase, 8u - f, F, s->S2k, s->REp + X.rb, fo, 31u,
                         s->bkah + (size_t)(T - 1) * kBkC * kBkC, 0u, BkChunked{nullptr, 0});
      const int gd = (int)std::min<uint32_t>(NB, 512);
      hipLaunchKernelGGL(k_bk_dedup, dim3(gd), dim3(kBkDedupThreads), 0, s->stream, s->S2k, (const uint32_t*)fo, NB, s->S1k,
                         s->ucnt, s->REc + X.rb, s->st);
      hipLaunchKernelGGL(k_bk_scan, dim3(1), dim3(1024), 0, s->stream, s->ucnt, NB, cst, s->bktotal);
      HIPCHK(hipGetLastError());
      (void)P;
    }
    std::vector<uint32_t> derr(ss.size(), 0);
    for (size_t g = 0; g < ss.size(); g++) {
      gm_solver* s = ss[g];
      if (!s->lvh[(size_t)L + 1].ein) continue;
      HIPCHK(hipMemcpyAsync(&ncnt[g], s->bktotal, 8, hipMemcpyDeviceToHost, s->stream));
      HIPCHK(hipMemcpyAsync(&derr[g], &s->st->err, 4, hipMemcpyDeviceToHost, s->stream));
    }
    HIPCHK(sync_all());  // one host sync for every shard's level size
    for (size_t g = 0; g < ss.size(); g++) {
      gm_solver* s = ss[g];
      BkLevel& X = s->lvh[(size_t)L + 1];
      if (!X.ein) continue;
      const uint32_t herr = derr[g];
      if (herr) {
        const bool lim = herr & ERR_BUCKET_FULL;
        defer(fail(lim ? GM_ELIMIT : GM_ECORRUPT, "shard %d level %d:%s", s->rank, L + 1, err_text(herr).c_str()));
        ncnt[g] = 0;
      }
      if (X.lb + ncnt[g] > s->Pcap) {
        defer(fail(GM_EFULL, "shard %d: positions exceed the plan's %llu", s->rank, (unsigned long long)s->Pcap));
        ncnt[g] = 0;
      }
      X.n = ncnt[g];
      if (!X.n) continue;
      const uint32_t NB = 1u << X.nbits;
      const uint32_t* cst = s->meta + X.cst_off;
      hipLaunchKernelGGL(k_bk_compact, dim3(std::min<uint32_t>(NB, 4096)), dim3(256), 0, s->stream, (const u64*)s->S1k,
                         (const uint32_t*)(cst + NB + 1), cst, NB, s->bkK + X.lb);
      HIPCHK(hipGetLastError());
    }
    if (L + 2 < T) {  // the largest shard of level L + 1 (the next level's form)
      std::vector<std::vector<u64>> row(ss.size(), std::vector<u64>(1, 0));
      for (size_t g = 0; g < ss.size(); g++) row[g][0] = ss[g]->lvh[(size_t)L + 1].n;
      std::vector<u64> all;
      int rc = bks_allgather(ss, mode, st, row, all);
      if (rc) return bail(rc);
      for (u64 v : all) lmax[(size_t)L + 1] = std::max(lmax[(size_t)L + 1], v);
    }
  }
  {  // the last level's status, before any rank starts the backward exchanges
    std::vector<std::vector<u64>> row(ss.size(), std::vector<u64>((size_t)W + 3, 0));
    for (size_t g = 0; g < ss.size(); g++) row[g][(size_t)W] = (u64)(int64_t)prc;
    std::vector<u64> MA;
    int rc = bks_allgather(ss, mode, st, row, MA);
    if (!rc) rc = status_of(MA, (size_t)W + 3);
    if (rc) return bail(rc);
  }
  if (mode == 4) HIPCHK(sync_all());  // e1 after every shard's forward
  HIPCHK(hipEventRecord(e1, st));
  // ---- backward ----
  for (int L = T - 1; L >= 0; L--) {
    const bool edges = L + 1 < T;
    // (a) owners answer along level X's in-edges
    std::vector<BksA2A> aa(ss.size());
    for (size_t g = 0; g < ss.size(); g++) {
      gm_solver* s = ss[g];
      if (!edges) continue;
      const BkLevel& X = s->lvh[(size_t)L + 1];
      const std::vector<u64>& sc = s->bks_sc[(size_t)L];
      const std::vector<u64>& rcv = s->bks_rc[(size_t)L];
      const std::vector<u64> so = bks_prefix(sc), ro = bks_prefix(rcv);
      if (X.ein) {
        keep.emplace_back((size_t)W);
        std::vector<uint32_t>& cb = keep.back();
        for (int p = 0; p < W; p++) cb[(size_t)p] = (uint32_t)ro[(size_t)p];
        HIPCHK(hipMemcpyAsync(s->bkcur, cb.data(), (size_t)W * 4, hipMemcpyHostToDevice, s->stream));
        const uint32_t NB = 1u << X.nbits, F = NB / kBkC;
        const uint32_t* cst = s->meta + X.cst_off;
        hipLaunchKernelGGL(k_bks_answer, dim3(kBkC), dim3(kBkStreamThreads), 0, s->stream, s->REp + X.rb, s->REc + X.rb,
                           cst + NB + 1, cst, NB, F, s->bkW + X.lb, s->bkcur, s->XSk, s->st);
        HIPCHK(hipGetLastError());
      }
      // back along the forward's pairs: what came from p goes to p
      aa[g] = BksA2A{(char*)s->XSk, (char*)s->XRk, rcv, std::vector<u64>(ro.begin(), ro.end() - 1), sc,
                     std::vector<u64>(so.begin(), so.end() - 1)};
    }
    if (edges) {
      int rc = bks_alltoall(ss, mode, st, aa, 8);
      if (rc) return bail(rc);
    }
    // (b) parents reduce
    for (size_t g = 0; g < ss.size(); g++) {
      gm_solver* s = ss[g];
      BkLevel& P = s->lvh[(size_t)L];
      if (!P.n) continue;
      bk_ranges(P.n, &P.pshift, &P.fb);  // checked in the forward
      const uint32_t NR = (uint32_t)((P.n + (1ull << P.fb) - 1) >> P.fb);
      const int gr = (int)std::min<uint32_t>(NR, 512);
      if (edges && P.eout && s->bksl[(size_t)L].used) {
        // the owners' words of this rank's unique children, then the one-GPU
        // backward over its local in-edges
        const gm_solver::BksLocal& B = s->bksl[(size_t)L];
        const uint32_t* rfo = s->meta + P.rfo_off;
        const uint32_t* pb = s->pbase + (size_t)L * (kBkC + 1);
        uint32_t* Ap = (uint32_t*)s->S1k;
        uint32_t* Wu = (uint32_t*)s->XSk;  // the answers it held have left in the exchange
        u64 na = 0;
        for (int p = 0; p < W; p++) na += s->bks_sc[(size_t)L][(size_t)p];
        if (na != B.nu) {
          // recorded, not returned: the other ranks are about to enter the
          // next level's exchange with this one; the error travels in the
          // final totals (error mask OR-ed over ranks) and every rank
          // returns together
          defer(fail(GM_ECORRUPT, "shard %d level %d: %llu answers for %llu unique children", s->rank, L,
                     (unsigned long long)na, (unsigned long long)B.nu));
          host_err |= ERR_EDGE_COUNT;
          continue;
        }
        if (na)
          hipLaunchKernelGGL(k_bks_wu, dim3((uint32_t)std::min<u64>((na + 255) / 256, 4096)), dim3(256), 0, s->stream,
                             (const u64*)s->XRk, na, Wu);
        const uint32_t NB = 1u << B.nbits, F = NB / kBkC;
        const uint32_t* cst = s->meta + B.cst_off;
        hipLaunchKernelGGL(k_bk_colscan, dim3(kBkC), dim3(256), 0, s->stream, s->bkah + (size_t)L * kBkC * kBkC, (uint32_t)kBkC,
                           s->boff, s->tot);
        hipLaunchKernelGGL(k_bk_answer, dim3(kBkC), dim3(kBkStreamThreads), 0, s->stream, s->REpl + B.rb, s->REcl + B.rb,
                           cst + NB + 1, cst, NB, F, P.pshift, s->boff, pb, (const uint32_t*)Wu, Ap, s->st);
        const uint32_t Fp = 1u << (P.pshift - P.fb);
        const uint32_t* ap = Ap;
        if (Fp > 1) {
          constexpr uint32_t K = kBkSplitK;
          HIPCHK(hipMemcpyAsync(s->bkcur + kBkC, rfo, (size_t)NR * 4, hipMemcpyDeviceToDevice, s->stream));
          hipLaunchKernelGGL(k_bk_split, dim3(kBkC * K), dim3(kBkStreamThreads), 0, s->stream, (const uint32_t*)Ap, pb,
                             10u + P.fb, Fp, K, s->bkcur + kBkC, (uint32_t*)s->S2k);
          ap = (uint32_t*)s->S2k;
        }
        BK_KIND_LAUNCH(k_bk_reduce, gr, kBkReduceThreads, s, s->d, s->bkK + P.lb, P.n, ap, rfo, P.fb, Fp - 1, NR,
                       s->bkW + P.lb, s->st);
      } else if (edges && P.eout) {
        const uint32_t* rfo = s->meta + P.rfo_off;
        const uint32_t* pb = s->pbase + (size_t)L * (kBkC + 1);
        uint32_t* Ap = (uint32_t*)s->S1k;
        HIPCHK(hipMemcpyAsync(s->bkcur, pb, kBkC * 4, hipMemcpyDeviceToDevice, s->stream));
        const u64 nblk = std::min<u64>(kBkExpandBlocks, (P.eout + kBksAnswerCap - 1) / kBksAnswerCap),
                  chunk = (P.eout + nblk - 1) / nblk;
        hipLaunchKernelGGL(k_bks_answer_in, dim3(nblk), dim3(kBkStreamThreads), 0, s->stream, (const u64*)s->XRk, P.eout, chunk,
                           P.pshift, s->bkcur, Ap);
        const uint32_t Fp = 1u << (P.pshift - P.fb);
        const uint32_t* ap = Ap;
        if (Fp > 1) {
          constexpr uint32_t K = kBkSplitK;
          HIPCHK(hipMemcpyAsync(s->bkcur + kBkC, rfo, (size_t)NR * 4, hipMemcpyDeviceToDevice, s->stream));
          hipLaunchKernelGGL(k_bk_split, dim3(kBkC * K), dim3(kBkStreamThreads), 0, s->stream, (const uint32_t*)Ap, pb,
                             10u + P.fb, Fp, K, s->bkcur + kBkC, (uint32_t*)s->S2k);
          ap = (uint32_t*)s->S2k;
        }
        BK_KIND_LAUNCH(k_bk_reduce, gr, kBkReduceThreads, s, s->d, s->bkK + P.lb, P.n, ap, rfo, P.fb, Fp - 1, NR,
                       s->bkW + P.lb, s->st);
      } else {
        BK_KIND_LAUNCH(k_bk_reduce, gr, kBkReduceThreads, s, s->d, s->bkK + P.lb, P.n, (const uint32_t*)nullptr,
                       (const uint32_t*)nullptr, P.fb, 0u, NR, s->bkW + P.lb, s->st);
      }
      HIPCHK(hipGetLastError());
    }
  }
  if (mode == 4) HIPCHK(sync_all());  // e2 after every shard's backward
  HIPCHK(hipEventRecord(e2, st));
  // ---- totals: positions, edges, primitives, root word + 1, error bits, per-level sizes ----
  std::vector<std::vector<u64>> mine(ss.size(), std::vector<u64>(5 + (size_t)T, 0));
  for (size_t g = 0; g < ss.size(); g++) {
    gm_solver* s = ss[g];
    HIPCHK(hipMemcpyAsync(s->bkL, s->lvh.data(), sizeof(BkLevel) * (size_t)T, hipMemcpyHostToDevice, s->stream));
    uint32_t root_word = NO_WORD;
    if (s->lvh[0].n) HIPCHK(hipMemcpyAsync(&root_word, s->bkW, 4, hipMemcpyDeviceToHost, s->stream));
    std::vector<unsigned char> host(devstate_bytes(T));
    HIPCHK(hipMemcpyAsync(host.data(), s->st, host.size(), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(sync_all());
    const DevState* hs = (const DevState*)host.data();
    std::vector<u64>& m = mine[g];
    for (int L = 0; L < T; L++) {
      m[0] += s->lvh[(size_t)L].n;
      m[5 + (size_t)L] = s->lvh[(size_t)L].n;
    }
    m[1] = hs->edges;
    m[2] = hs->prims;
    m[3] = root_word != NO_WORD ? (u64)root_word + 1 : 0;
    m[4] = hs->err | host_err;
  }
  std::vector<u64> all;
  int rc = bks_allgather(ss, mode, st, mine, all);
  if (rc) return bail(rc);
  std::vector<u64> tot(5 + (size_t)T, 0);
  for (int r = 0; r < W; r++)
    for (size_t i = 0; i < tot.size(); i++) {
      const u64 v = all[(size_t)r * tot.size() + i];
      tot[i] = i == 4 ? (tot[i] | v) : i == 3 ? std::max(tot[i], v) : tot[i] + v;
    }
  auto t1 = std::chrono::steady_clock::now();
  float fms = 0, bms = 0;
  HIPCHK(hipEventElapsedTime(&fms, e0, e1));
  HIPCHK(hipEventElapsedTime(&bms, e1, e2));
  done_events();
  out->ms_forward = fms;
  out->ms_backward = bms;
  out->ms_total = std::chrono::duration<double, std::milli>(t1 - t0).count();
  out->positions = tot[0];
  out->edges = tot[1];
  out->primitives = tot[2];
  u64 wmax = 0;
  uint32_t nlev = 0;
  for (int L = 0; L < T; L++) {
    wmax = std::max<u64>(wmax, tot[5 + (size_t)L]);
    nlev += tot[5 + (size_t)L] > 0;
  }
  out->levels = nlev;
  out->max_level_width = (uint32_t)std::min<u64>(wmax, 0xFFFFFFFFull);
  const uint32_t word = tot[3] ? (uint32_t)(tot[3] - 1) : NO_WORD;
  out->root_word = word;
  if (prc) {  // this rank's own deferred failure (its bits are in tot[4] too)
    g_err = perr;
    return prc;
  }
  if (tot[4]) {
    const bool full = tot[4] & (ERR_TABLE_FULL | ERR_LEVELS_FULL);
    const bool lim = tot[4] & ERR_BUCKET_FULL;
    return fail(lim ? GM_ELIMIT : full ? GM_EFULL : GM_ECORRUPT, "solve failed:%s", err_text((uint32_t)tot[4]).c_str());
  }
  if (word == NO_WORD) return fail(GM_ECORRUPT, "root unresolved");
  out->root_value = (int32_t)(word & 3u);
  out->root_remoteness = word >> 2;
  return 0;
}
}  // extern "C++"
