// gm_plane_run.h -- host side of the PLANES layout (gm_plane.h): planning,
// level lists, the solve loop (one table, an in-process shard group, or one
// shard per process over RCCL / a host-staged transport), and the table
// readers (query, positions, checksum).  Included by gm_solver.hip after the
// solver object and the dense helpers it shares (BlockCount slots,
// k_fill_red, the transport helpers).
//
// Reference path replaced: src/process.py:37-267 (the per-state job loop)
// and src/game_state.py:22-30 (which rank owns a state): a shard owns
// blocks of the last heap's values (plane_owner); the per-edge LOOK_UP /
// RESOLVE messages become, per plane level, one grouped send of the rank's
// boundary slices to the ranks owning its blocks' successors (the planes
// their first two slices need).

// (gm_solver.hip includes this inside its extern "C" block: templates need
// C++ linkage)
extern "C++" {
// ---------------------------------------------------------------------------
// kernels (need DevState / BlockCount / Desc from gm_solver.hip)
// ---------------------------------------------------------------------------
template <int NO>
__global__ __launch_bounds__(256) void k_plane_reach(uint32_t* bits, PlaneGeom g, BlockCount* bc, DevState* st,
                                                     uint32_t word_bits) {
  plane_reach_body<NO>(bits, g, [&](u64 npos, u64 edges) { block_count(bc, npos, edges); });
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st->word_bits = word_bits;  // the solve in progress (a resume checks it)
    // the only primitive, every heap 0: global plane 0 of rank 0, row 0, bit 0
    if (g.rank == 0) atomicAdd(&st->prims, 1ull);
  }
}

// word of local position (h0, h1, P) in value | remoteness << 2 form; e:
// the position's digit sum (all heaps; read by the relative forms only)
template <int WB>
__device__ __forceinline__ uint32_t plane_vr(const void* tab, u64 P, uint32_t h0, uint32_t h1, uint32_t e) {
  const u64 i = plane_word_index(P, h1, (h0 + h1) & 31u, WB == 2 ? 2u : 1u);
  const uint32_t w = WB == 2 ? ((const uint16_t*)tab)[i] : ((const uint8_t*)tab)[i];
  return WB == 3 ? plane_rel_to_vr(w, e) : plane_word_to_vr(w, WB);
}

// rank (key) -> local plane, h0, h1 and the key's digit sum; false if
// another shard owns it or the key lies outside the heaps
__device__ __forceinline__ bool plane_locate(const Desc& d, const PlaneGeom& g, u64 key, u64* P, uint32_t* h0,
                                             uint32_t* h1, uint32_t* esum) {
  u64 x = key;
  uint32_t dig[16], e = 0;
  for (int i = 0; i < d.nheaps; i++) {
    dig[i] = (uint32_t)(x % d.base[i]);
    e += dig[i];
    x /= d.base[i];
  }
  if (x) return false;
  *esum = e;
  *h0 = dig[0];
  *h1 = dig[1];
  u64 p = 0;
  const int no = d.nheaps - 2;
  if (g.rowdeal) {  // this shard holds heap-1 values [h1off, h1off + 32)
    if (dig[1] < g.h1off || dig[1] >= g.h1off + 32u) return false;
    *h1 = dig[1] - g.h1off;
    for (int j = 0; j < no; j++) p += (u64)dig[2 + j] * g.stride[j];
  } else if (g.world > 1) {
    const uint32_t t = dig[d.nheaps - 1], blk = t / g.B, o = t - blk * g.B;
    if (plane_owner(g, blk) != g.rank) return false;
    for (int j = 0; j + 1 < no; j++) p += (u64)dig[2 + j] * g.stride[j];
    p += ((u64)(blk / g.world) * g.B + o) * g.Z;
  } else {
    for (int j = 0; j < no; j++) p += (u64)dig[2 + j] * g.stride[j];
  }
  *P = p;
  return true;
}

template <int WB>
__global__ void k_plane_query(Desc d, PlaneGeom g, const void* tab, const uint32_t* bits, const u64* keys, u64 n,
                              uint32_t* out) {
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
    u64 P;
    uint32_t h0, h1, e, w = NO_WORD;
    if (plane_locate(d, g, keys[i], &P, &h0, &h1, &e) && ((plane_row_bits(bits, g, P, h1) >> h0) & 1u))
      w = plane_vr<WB>(tab, P, h0, h1, e);
    out[i] = w;
  }
}

// the end of a solve, one launch: the root's word (only the shard that owns
// it; DevState::root_word), then the counts and reduction words (k_fill_red's
// body) -- one block of 1024 threads.  After the one-launch backward
// (FLOW, k_plane_flow): the count slots [0, nslots) were STORED by that
// launch's workgroups, the totals are assigned, not added, the reduction
// words also go straight into the caller's pinned host buffer (no copy),
// and the error word is cleared once reported -- so the next one-launch
// solve needs neither the state fills nor the copy.  (Doing this in the
// flow launch's last workgroup instead was slower: 1.077-1.082 vs
// 1.041-1.043 ms per step, profiles/r06/flow_selffin_ab.txt.)
template <int WB, bool FLOW = false>
__global__ __launch_bounds__(1024) void k_plane_finish(Desc d, PlaneGeom g, const void* tab, const uint32_t* bits,
                                                       DevState* st, const BlockCount* bc, uint32_t nslots = 0,
                                                       u64* host = nullptr) {
  if (threadIdx.x == 0) {
    u64 P;
    uint32_t h0, h1, e, w = NO_WORD;
    if (plane_locate(d, g, d.root, &P, &h0, &h1, &e) && ((plane_row_bits(bits, g, P, h1) >> h0) & 1u))
      w = plane_vr<WB>(tab, P, h0, h1, e);
    st->root_word = w;
  }
  __syncthreads();
  if (!FLOW) {
    fill_red_body(st, bc);
    return;
  }
  __shared__ u64 rn[16], re[16];
  u64 sn = 0, se = 0;
  for (uint32_t i = threadIdx.x; i < nslots; i += blockDim.x) {
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
    for (int w = 0; w < (int)(blockDim.x >> 6); w++) sn += rn[w], se += re[w];
    const u64 red[5] = {sn, se, st->prims, st->root_word == NO_WORD ? 0ull : (u64)st->root_word + 1ull, (u64)st->err};
    st->cursor_front = sn;
    st->edges = se;
    for (int k = 0; k < 5; k++) st->red[k] = red[k];
    if (host)
      for (int k = 0; k < 5; k++) __hip_atomic_store(host + k, red[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    st->err = 0;  // (reported above: the next one-launch solve starts clean)
  }
}

// The one-launch backward (gm_plane.h plane_flow_body) and, in the same
// launch, the forward: once a wave's ticket sequence is empty it writes its
// grid-stride share of the reach map and the counts (k_plane_reach's body);
// the narrow tail levels leave most waves idle, so the forward costs no
// launch of its own.  Each workgroup STORES its count slot (no reset before
// the solve; k_plane_finish<., true> sums the grid's slots).
template <int NO, bool PIPE = true>
__global__ __launch_bounds__(256) void k_plane_flow(uint8_t* tab, PlaneGeom g, const uint4* zero, PlaneFlow f,
                                                    uint32_t* bits, BlockCount* bc, DevState* st, uint32_t word_bits) {
  plane_flow_body<NO, PIPE>(tab, g, zero, f);
  __shared__ u64 rn[4], re[4];
  plane_reach_body<NO>(bits, g, [&](u64 npos, u64 edges) {
    for (int o = 32; o > 0; o >>= 1) {
      npos += __shfl_xor(npos, o);
      edges += __shfl_xor(edges, o);
    }
    if (__lane_id() == 0) {
      rn[threadIdx.x >> 6] = npos;
      re[threadIdx.x >> 6] = edges;
    }
  });
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 sn = 0, se = 0;
    for (int w = 0; w < 4; w++) sn += rn[w], se += re[w];
    bc[blockIdx.x].npos = sn;
    bc[blockIdx.x].edges = se;
    if (blockIdx.x == 0) {
      st->word_bits = word_bits;
      st->prims = g.rank == 0 ? 1ull : 0ull;  // every heap 0: global plane 0 of rank 0
    }
  }
}

// global rank of local position (h0, h1, P); *osum: its outer digit sum
template <int NO>
__device__ __forceinline__ u64 plane_key(const Desc& d, const PlaneGeom& g, uint32_t P, uint32_t h0, uint32_t h1,
                                         uint32_t* osum = nullptr) {
  uint32_t dig[NO > 0 ? NO : 1];
  plane_global_digits<NO>(g, P, dig);
  u64 k = (u64)h0 + (u64)(h1 + g.h1off) * d.stride[1];
  uint32_t t = 0;
#pragma unroll
  for (int j = 0; j < NO; j++) {
    k += (u64)dig[j] * d.stride[2 + j];
    t += dig[j];
  }
  if (osum) *osum = t;
  return k;
}

template <int NO>
__global__ void k_plane_positions(Desc d, PlaneGeom g, const uint32_t* bits, u64* out, u64 cap, u64* count) {
  const u64 nw = (u64)g.nplanes * 32u;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += (u64)gridDim.x * blockDim.x) {
    uint32_t w = plane_row_bits(bits, g, i >> 5, (uint32_t)i & 31u);
    if (!w) continue;
    u64 k = atomicAdd(count, (u64)__builtin_popcount(w));
    const u64 base = plane_key<NO>(d, g, (uint32_t)(i >> 5), 0, (uint32_t)i & 31u);
    for (; w; w &= w - 1, k++)
      if (k < cap) out[k] = base + (u64)__builtin_ctz(w);
  }
}

template <int NO, int WB>
__global__ __launch_bounds__(256) void k_plane_checksum(Desc d, PlaneGeom g, const void* tab, const uint32_t* bits,
                                                        u64* acc) {
  u64 a[6] = {0, 0, 0, 0, 0, 0};
  const u64 nw = (u64)g.nplanes * 32u;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += (u64)gridDim.x * blockDim.x) {
    const uint32_t P = (uint32_t)(i >> 5), h1 = (uint32_t)i & 31u;
    uint32_t w = plane_row_bits(bits, g, P, h1);
    if (!w) continue;
    uint32_t os;
    const u64 base = plane_key<NO>(d, g, P, 0, h1, &os);
    for (; w; w &= w - 1) {
      const uint32_t h0 = (uint32_t)__builtin_ctz(w);
      ck_add(d, base + h0, plane_vr<WB>(tab, P, h0, h1, os + h0 + h1 + g.h1off), a);
    }
  }
  ck_block_add(acc, a);
}

// ---------------------------------------------------------------------------
// host: shape, plan, lists
// ---------------------------------------------------------------------------
// PLANES applies to sum_four_to_one whose heaps 0 and 1 hold 32 values (a
// plane is 32 x 32), with at most kPlaneMaxOuter further heaps and every
// remoteness below 2^15 (16-bit order forms).
static uint32_t plane_form(const Desc* d, uint32_t flags);
// The row deal (shards of heap 1): heap 1 holds 32 values per rank, each rank
// a 32-row slab of every plane (plane_shape); 8-bit words only (the packed
// kernels carry its halo rows)
static bool plane_row_deal(const Desc* d, int world) {
  return world > 1 && d->nheaps >= 3 && d->heap[0] == 31 && d->heap[1] + 1 == 32u * (uint32_t)world &&
         plane_form(d, 0) != 2;
}
static bool plane_ok(const Desc* d, int world) {
  if (d->kind != K_SUM || d->variant != 0 || d->nheaps < 2 || d->nheaps - 2 > kPlaneMaxOuter) return false;
  if (d->heap[0] != 31 || (d->heap[1] != 31 && !plane_row_deal(d, world)) || d->root_sum >= 0x7FFF) return false;
  u64 np = 1;
  for (int i = 2; i < d->nheaps; i++) np *= d->base[i];
  return np <= 0xFFFFFFF0ull;
}
// Word form: 8-bit order forms when every remoteness < 255 (they carry the
// value in the remoteness parity: every K_SUM position is WIN or LOSS); the
// relative 8-bit forms (gm_plane.h) up to root digit sum kPlaneRelMaxSum;
// else (or GM_F_WORDS16) 16-bit
static uint32_t plane_form(const Desc* d, uint32_t flags) {
  if (flags & GM_F_WORDS16) return 2u;
  return d->root_sum <= 253 ? 1u : d->root_sum <= kPlaneRelMaxSum ? 3u : 2u;
}
static bool plane_wanted(const Desc* d, uint32_t flags, int world) {
  if (plane_row_deal(d, world) && (flags & (GM_F_WORDS16 | GM_F_PLANE_X1))) return false;
  return plane_ok(d, world) && !(flags & (GM_F_LEVEL_MAJOR | GM_F_FORCE_HASHED | GM_F_WORDS32 | GM_F_RESOLVE_SCALAR));
}

struct PlaneShape {
  PlaneGeom g;
  uint32_t wb;           // word bytes
  uint32_t form;         // plane_form
  uint32_t S;            // largest plane level (sum of the outer heaps)
  uint32_t nblocks, nb;  // shards: blocks of the top digit over all ranks / of this rank
  u64 nlocal;            // planes of this table
  u64 nrecv, nsend;      // halo planes of this shard (all levels)
  u64 words_off, bits_off, recv_off, send_off, table_bytes;  // table buffer layout
  u64 zero_off, list_off, scratch_bytes;                      // scratch layout
  // the one-launch backward (k_plane_flow): one-table 8-bit absolute forms;
  // scratch: visits, sequence offsets, counter lines, per-plane flags
  bool flow;
  u64 flow_off, flow_qoff_off, flow_ctr_off, flow_flags_off;
  // the staged deal (shards; 0: level-synchronous): key skew k, keys, rows
  uint32_t stage_k, nkeys, nrows;
};

// Staged PLANES shards.  Rank r owns ONE block: the top
// values [r B, (r + 1) B), B = E / world.  A plane (top offset o, lower
// digits of sum s) depends only on planes at o - 1, o - 2 (same lower digits)
// and at lower sums s - 1, s - 2 (same o); so key(o, s) = o + k s, k >= 1,
// orders every plane after its children and a rank resolves its planes key
// by key with NO level barrier across ranks.  The only cross-rank edge: the
// planes of top offsets 0, 1 read the previous rank's last two slices at the
// same lower digits.  Those leave rank r - 1 row by row -- row s (slices
// B - 2, B - 1 at lower sum s) is final after key B - 1 + k s -- and rank r
// first needs row s at key k s: the ranks form a pipeline in which rank r
// trails rank r - 1 by about B keys, and the transfers hide under B - 1 keys
// of compute.  Larger k shortens the trail (fewer planes per key) but adds
// launches.  Measured per-shard sweeps of the 4- and 8-GPU bench shapes
// (8-bit relative words, profiles/r04j/): 2.32 / 2.89 / 3.51 / 4.01 ms (N = 4)
// and 2.35 / 2.92 / 3.54 / 4.03 ms (N = 8) at k = 2 / 3 / 4 / 5 -- every key
// costs ~4.5 us beyond its planes, while the trail is B - 1 keys whatever k
// is (narrower keys only shorten each of them) -- so k = 2; at N = 2, k = 1
// (profiles/r04zn/: a shard's sweep and its widest window of B keys -- the
// trail each rank adds -- from kernel traces: 2.24 + 0.83 ms at k = 1 against
// 3.12 + 0.54 ms at k = 2 under the profiler; equal at N = 4, k = 2 ahead at
// N = 8).  A
// key's planes have outer digit sums s = rB + o + c = rB + key - (k - 1) c of
// several residues mod 4: with the relative word forms the staged lists deal
// each key's planes by s mod 4 in whole wave visits (padded) and the kernel
// picks its specialisation per visit (plane_x2_range, RS = -1).
// GM_PLANE_STAGE_K overrides k (A/B).
static uint32_t plane_stage_k(int world) {
  if (const char* e = lab_env("GM_PLANE_STAGE_K")) {
    const int k = atoi(e);
    if (k >= 1 && k <= 64) return (uint32_t)k;
  }
  return world == 2 ? 1u : 2u;
}
// list padding of the relative forms' staged deal: at most 3 entries per
// (key, s mod 4) class
static u64 plane_stage_pad(const PlaneShape* ps) { return ps->form == 3 && !ps->g.rowdeal ? 12ull * ps->nkeys : 0ull; }

static u64 rup256(u64 x) { return (x + 255) & ~255ull; }


static int plane_shape(const Desc* d, int rank, int world, uint32_t flags, PlaneShape* ps) {
  memset(ps, 0, sizeof *ps);
  PlaneGeom& g = ps->g;
  g.no = (uint32_t)(d->nheaps - 2);
  g.pow2 = 1;
  g.world = (uint32_t)std::max(world, 1);
  g.rank = (uint32_t)rank;
  u64 np = 1;
  for (uint32_t j = 0; j < g.no; j++) {
    g.base[j] = d->base[2 + j];
    g.stride[j] = (uint32_t)np;
    g.shift[j] = (uint32_t)__builtin_ctzll(np);
    if (g.base[j] & (g.base[j] - 1)) g.pow2 = 0;
    np *= g.base[j];
  }
  // reach: the values each heap reaches by its own moves from its start
  // (four_to_one.py:10-15: x -> x-1 for x >= 1, x -> x-2 for x >= 2), a 1-D
  // closure; the layout needs it to be [0, r] (it is: [0, start])
  for (int i = 0; i < d->nheaps; i++) {
    std::vector<uint8_t> seen((size_t)d->heap[i] + 1, 0);
    std::vector<uint32_t> todo{d->heap[i]};
    seen[d->heap[i]] = 1;
    while (!todo.empty()) {
      const uint32_t x = todo.back();
      todo.pop_back();
      for (uint32_t k = 1; k <= 2 && k <= x; k++)
        if (!seen[x - k]) {
          seen[x - k] = 1;
          todo.push_back(x - k);
        }
    }
    uint32_t r = 0;
    while (r + 1 < seen.size() && seen[r + 1]) r++;
    for (size_t v = 0; v < seen.size(); v++)
      if (seen[v] != (v <= r)) return fail(GM_EINVAL, "heap %d: reachable values are not a prefix", i);
    g.rlim[i] = r;
  }
  ps->form = plane_form(d, flags);
  ps->wb = ps->form == 2 ? 2u : 1u;
  ps->S = 0;
  for (int i = 2; i < d->nheaps; i++) ps->S += d->heap[i];
  const bool rows = plane_row_deal(d, world);
  if (rows && (ps->form == 2 || (flags & GM_F_PLANE_X1)))
    return fail(GM_EINVAL, "the row deal runs the packed 8-bit kernels only");
  if (world <= 1) {
    g.nplanes = (uint32_t)np;
    ps->nlocal = np;
  } else if (rows) {
    // The row deal: every rank holds all 2^(5 * outer) planes, rows = heap-1
    // values [32 r, 32 r + 32).  Plane levels are the one-table levels; a
    // plane's rows 0 and 1 read the previous rank's rows 30 and 31 of the
    // SAME plane (heap 1 - 1, - 2), so rank r's level l waits only for rank
    // r - 1's level l: the pipeline trails by one level (+ its transfer)
    // instead of B keys.  As staged keys: key = row = level, both with lag 0.
    if (rank < 0 || rank >= world) return fail(GM_EINVAL, "bad shard %d/%d", rank, world);
    g.rowdeal = 1;
    g.h1off = 32u * (uint32_t)rank;
    g.nplanes = (uint32_t)np;
    ps->nlocal = np;
    ps->stage_k = 1;
    ps->nkeys = ps->nrows = ps->S + 1;
    ps->nrecv = rank > 0 ? np : 0;          // halo entries: two rows per plane
    ps->nsend = rank + 1 < world ? np : 0;
  } else {
    if (g.no < 1) return fail(GM_EINVAL, "sharded planes need at least 3 heaps");
    if (rank < 0 || rank >= world) return fail(GM_EINVAL, "bad shard %d/%d", rank, world);
    const u64 E = d->base[d->nheaps - 1], Z = g.stride[g.no - 1];
    const bool staged = !(flags & GM_F_PLANE_LEVEL_SYNC) && E % (u64)world == 0 && E / (u64)world >= 2;
    const u64 B = staged ? E / world : E >= 16 * (u64)world ? 8 : (E + world - 1) / world;
    if (B < 2 || E % B || E / B < (u64)world)
      return fail(GM_EINVAL, "last heap of %llu values cannot give %d ranks whole blocks of >= 2", (unsigned long long)E,
                  world);
    ps->nblocks = (uint32_t)(E / B);
    ps->nb = (uint32_t)((ps->nblocks - (u64)rank + world - 1) / world);
    g.B = (uint32_t)B;
    g.Z = (uint32_t)Z;
    g.spread = !staged && world >= 4 && !(world & (world - 1)) && ps->nblocks % world == 0 &&
               ps->nblocks > (u64)world && !(flags & GM_F_PLANE_ROUND_ROBIN);
    if (staged) {
      uint32_t smax = 0;  // largest digit sum below the top
      for (uint32_t j = 0; j + 1 < g.no; j++) smax += g.base[j] - 1;
      ps->stage_k = plane_stage_k(world);
      ps->nrows = smax + 1;
      ps->nkeys = (uint32_t)(B - 1) + ps->stage_k * smax + 1;
    }
    ps->nlocal = (u64)ps->nb * B * Z;
    g.nplanes = (uint32_t)ps->nlocal;
    for (uint32_t j = 0; j < ps->nb; j++) {
      const u64 gb = plane_gblock(g, j);
      if (gb >= 1) ps->nrecv += 2 * Z;
      if (gb + 1 < ps->nblocks) ps->nsend += 2 * Z;
    }
  }
  const u64 pb = 1024ull * ps->wb, hb = g.rowdeal ? 64ull * ps->wb : pb;  // halo entry: plane / two rows
  ps->words_off = 0;
  ps->bits_off = rup256(ps->nlocal * pb);
  ps->recv_off = ps->bits_off + rup256(ps->nlocal * 4);  // one reach bit per row
  ps->send_off = ps->recv_off + rup256(ps->nrecv * hb);
  ps->table_bytes = ps->send_off + rup256(ps->nsend * hb);
  ps->zero_off = rup256(scratch_bytes_for(d->max_levels));
  ps->list_off = ps->zero_off + 4096;
  ps->scratch_bytes =
      ps->list_off + rup256((ps->nlocal + plane_stage_pad(ps)) * (world > 1 && !g.rowdeal ? sizeof(PlaneEntry) : 4));
  ps->flow = world <= 1 && ps->form == 1 && g.no >= 1;
  if (ps->flow) {  // visits: every level padded to whole visits of 4 planes
    ps->flow_off = ps->scratch_bytes;
    ps->flow_qoff_off = ps->flow_off + rup256((ps->nlocal + 24ull * (ps->S + 1)) * 4);  // (<= 3 pads per level and XCD)
    ps->flow_ctr_off = ps->flow_qoff_off + rup256((kPlaneFlowQ + 1) * 4);
    ps->flow_flags_off = ps->flow_ctr_off + rup256((u64)kPlaneFlowLine * (kPlaneFlowQ + 2) * 4);
    ps->scratch_bytes = ps->flow_flags_off + rup256(ps->nlocal * 4);
  }
  return 0;
}

static int plan_planes(const Desc* d, int rank, int world, uint32_t flags, uint64_t max_table_bytes, gm_plan_t* out,
                       bool* fits) {
  PlaneShape ps;
  int rc = plane_shape(d, rank, world, flags, &ps);
  if (rc) return rc;
  *fits = max_table_bytes == 0 || ps.table_bytes <= max_table_bytes;
  out->mode = GM_MODE_PLANES;
  out->table_slots = ps.nlocal * 1024;
  out->table_bytes = ps.table_bytes;
  out->level_capacity = 1;
  out->scratch_bytes = ps.scratch_bytes;
  out->max_levels = (uint32_t)d->max_levels;
  return 0;
}

// Level lists (host, once per solver).  World 1: the planes of each level
// (outer digit sum s) in index order.  Shards: PlaneEntry per own plane,
// level by level, and within a level block by block, slice by slice, lower
// index ascending -- the canonical order in which the boundary slices travel:
// the sender's (level s, peer p) segment lists, for each of its blocks whose
// successor p owns, slices B-2 and B-1; the receiver's (s, q), for each of
// its blocks whose predecessor q owns, the two slices below it (local block
// order is global block order, so both walk the same blocks in the same
// order).  Segments are level-major, peer-minor.  A halo plane's index is its
// group's start plus the rank of its lower digits within their digit-sum
// class, which is also the rank of the receiving plane in its own group.
// Staged lists: PlaneEntry per own plane, key by key (key = o + k s, s the
// lower digit sum).  Halo buffers (send and receive alike) are row-major:
// row s = [2 R(s), 2 R(s + 1)) with R the prefix of the lower-digit class
// sizes, slice h (top value rB - 2 + h / the sender's B - 2 + h) at
// 2 R(s) + h ncl(s) + the lower digits' rank in their class -- so a row is one
// contiguous message.  ploff: per key; prcv_off / psnd_off: per row.
static int plane_lists_staged(gm_solver* s, const PlaneShape& ps, const std::vector<uint32_t>& sig,
                              const std::vector<uint32_t>& rk, const std::vector<u64>& ncl,
                              std::vector<uint8_t>& bytes) {
  const PlaneGeom& g = ps.g;
  const u64 Z = g.Z, B = g.B, k = ps.stage_k, K = ps.nkeys, R = ps.nrows;
  if (ncl.size() != R) return fail(GM_ECORRUPT, "staged lists: %zu digit-sum classes, %llu rows", ncl.size(),
                                   (unsigned long long)R);
  const bool rx = g.rank > 0, tx = g.rank + 1 < g.world;
  std::vector<u64> row(R + 1, 0);
  for (u64 r = 0; r < R; r++) row[r + 1] = row[r] + 2 * ncl[r];
  s->prcv_off.assign(R + 1, 0);
  s->psnd_off.assign(R + 1, 0);
  if (rx) s->prcv_off = row;
  if (tx) s->psnd_off = row;
  if (s->prcv_off[R] != ps.nrecv || s->psnd_off[R] != ps.nsend)
    return fail(GM_ECORRUPT, "staged halo plan: %llu / %llu planes, sized %llu / %llu",
                (unsigned long long)s->prcv_off[R], (unsigned long long)s->psnd_off[R],
                (unsigned long long)ps.nrecv, (unsigned long long)ps.nsend);
  // entries per key; relative forms: per (key, s mod 4) class, each class
  // padded to whole wave visits of 4 entries (plane_x2_range, RS = -1)
  const bool rel = ps.form == 3;
  const u64 t0 = (u64)g.rank * B;
  const u64 ncls = rel ? 4 : 1;
  auto cls_of = [&](u64 o, uint32_t c) -> u64 { return rel ? (t0 + o + c) & 3u : 0u; };
  std::vector<u64> cnt(K * ncls, 0);
  for (u64 o = 0; o < B; o++)
    for (u64 l = 0; l < Z; l++) cnt[(o + k * sig[l]) * ncls + cls_of(o, sig[l])]++;
  s->ploff.assign(K + 1, 0);
  std::vector<u64> cpos(K * ncls, 0);  // first entry of each (key, class)
  u64 at = 0;
  for (u64 q = 0; q < K; q++) {
    s->ploff[q] = at;
    for (u64 c = 0; c < ncls; c++) {
      cpos[q * ncls + c] = at;
      at += rel ? (cnt[q * ncls + c] + 3) / 4 * 4 : cnt[q * ncls + c];
    }
  }
  s->ploff[K] = at;
  if (at < ps.nlocal || at > ps.nlocal + plane_stage_pad(&ps))
    return fail(GM_ECORRUPT, "staged lists: %llu entries for %llu planes", (unsigned long long)at,
                (unsigned long long)ps.nlocal);
  bytes.assign(at * sizeof(PlaneEntry), 0xFF);  // padding: every field kPlaneAbsent
  PlaneEntry* E = (PlaneEntry*)bytes.data();
  std::vector<u64>& pos = cpos;
  for (u64 o = 0; o < B; o++)
    for (u64 l = 0; l < Z; l++) {
      const uint32_t c = sig[l];
      PlaneEntry e;
      e.p = (uint32_t)(o * Z + l);
      auto halo = [&](u64 kk) -> uint32_t {  // neighbour at top value t0 + o - kk
        if (t0 + o < kk) return kPlaneAbsent;
        if (o >= kk) return kPlaneLocal;
        return (uint32_t)(row[c] + (o + 2 - kk) * ncl[c] + rk[l]);
      };
      e.top1 = halo(1);
      e.top2 = halo(2);
      e.send = (tx && o + 2 >= B) ? (uint32_t)(row[c] + (o + 2 - B) * ncl[c] + rk[l]) : kPlaneAbsent;
      E[pos[(o + k * c) * ncls + cls_of(o, c)]++] = e;
    }
  s->pbnd.clear();
  return 0;
}

static int plane_lists(gm_solver* s, const PlaneShape& ps, std::vector<uint8_t>& bytes) {
  const PlaneGeom& g = ps.g;
  const uint32_t S = ps.S;
  auto digsum = [&](u64 P, uint32_t ndig) {
    uint32_t t = 0;
    for (uint32_t j = 0; j < ndig; j++) {
      t += (uint32_t)(P % g.base[j]);
      P /= g.base[j];
    }
    return t;
  };
  s->ploff.assign((size_t)S + 2, 0);
  if (g.world <= 1 || g.rowdeal) {
    std::vector<uint32_t> lev(ps.nlocal);
    for (u64 P = 0; P < ps.nlocal; P++) {
      lev[P] = digsum(P, g.no);
      s->ploff[lev[P] + 1]++;
    }
    for (uint32_t l = 0; l <= S; l++) s->ploff[l + 1] += s->ploff[l];
    bytes.resize(ps.nlocal * 4);
    uint32_t* L = (uint32_t*)bytes.data();
    std::vector<u64> pos(s->ploff.begin(), s->ploff.end());
    for (u64 P = 0; P < ps.nlocal; P++) L[pos[lev[P]]++] = (uint32_t)P;
    // Within a level: the planes in 3-D tiles of kPlaneTile^3 over the outer
    // digits above the lowest (the lowest follows from the level), tiles and
    // the planes inside a tile lexicographic.  A child plane's four parents
    // at the next level (one outer digit + 1) then mostly share its tile, so
    // they run on one XCD close together and its lines are fetched into that
    // L2 about once per level (plane index order: -2 % backward time,
    // tools/plane_lab LAB_ORDER=8, profiles/r04b_plane_lab.txt).
    if (g.no >= 2) {
      constexpr uint32_t kPlaneTile = 8;
      auto key = [&](uint32_t P) {
        uint32_t dig[kPlaneMaxOuter];
        u64 x = P;
        for (uint32_t j = 0; j < g.no; j++) {
          dig[j] = (uint32_t)(x % g.base[j]);
          x /= g.base[j];
        }
        u64 k = 0;  // mixed radix: < 8^5 * 2^32 (the plane index is 32-bit)
        for (int j = (int)g.no - 1; j >= 1; j--) k = k * ((g.base[j] + kPlaneTile - 1) / kPlaneTile) + dig[j] / kPlaneTile;
        for (int j = (int)g.no - 1; j >= 1; j--) k = k * kPlaneTile + dig[j] % kPlaneTile;
        return k * g.base[0] + dig[0];
      };
      std::vector<std::pair<u64, uint32_t>> tmp;
      for (uint32_t l = 0; l <= S; l++) {
        const u64 a = s->ploff[l], b = s->ploff[(size_t)l + 1];
        tmp.resize(b - a);
        for (u64 i = a; i < b; i++) tmp[i - a] = {key(L[i]), L[i]};
        std::sort(tmp.begin(), tmp.end());
        for (u64 i = a; i < b; i++) L[i] = tmp[i - a].second;
      }
    }
    if (g.rowdeal) {  // halo row r = level r's entries, in list order, both ways
      s->prcv_off.assign((size_t)S + 2, 0);
      s->psnd_off.assign((size_t)S + 2, 0);
      if (g.rank > 0) s->prcv_off = s->ploff;
      if (g.rank + 1 < g.world) s->psnd_off = s->ploff;
      s->pbnd.clear();
    }
    return 0;
  }
  const u64 Z = g.Z, B = g.B;
  const uint32_t nlow = g.no - 1;  // digits below the top
  std::vector<uint32_t> sig(Z), rk(Z);
  uint32_t smax = 0;
  for (u64 l = 0; l < Z; l++) smax = std::max(smax, sig[l] = digsum(l, nlow));
  std::vector<u64> ncl(smax + 1, 0);
  for (u64 l = 0; l < Z; l++) rk[l] = (uint32_t)ncl[sig[l]]++;
  auto cls = [&](int64_t c) -> u64 { return c < 0 || c > (int64_t)smax ? 0 : ncl[(size_t)c]; };
  if (ps.stage_k) return plane_lists_staged(s, ps, sig, rk, ncl, bytes);
  const u64 nb = ps.nb, W = g.world;
  auto gblk = [&](u64 j) { return (u64)plane_gblock(g, (uint32_t)j); };
  // halo groups per level and peer (the rank the slices come from / go to):
  // recv (j, h) = top value gB - 2 + h; send (j, h) = top value gB + B - 2 + h
  std::vector<u64> rgb(((size_t)S + 1) * nb * 2, ~0ull), sgb(((size_t)S + 1) * nb * 2, ~0ull);
  s->prcv_off.assign(((size_t)S + 1) * W + 1, 0);
  s->psnd_off.assign(((size_t)S + 1) * W + 1, 0);
  u64 ra = 0, sa = 0;
  for (uint32_t l = 0; l <= S; l++)
    for (u64 p = 0; p < W; p++) {
      s->prcv_off[(size_t)l * W + p] = ra;
      s->psnd_off[(size_t)l * W + p] = sa;
      for (u64 j = 0; j < nb; j++) {
        const u64 gb = gblk(j);
        const bool rx = gb >= 1 && plane_owner(g, (uint32_t)(gb - 1)) == p;
        const bool tx = gb + 1 < ps.nblocks && plane_owner(g, (uint32_t)(gb + 1)) == p;
        for (u64 h = 0; h < 2; h++) {
          if (rx) {
            rgb[((size_t)l * nb + j) * 2 + h] = ra;
            ra += cls((int64_t)l - (int64_t)(gb * B - 2 + h));
          }
          if (tx) {
            sgb[((size_t)l * nb + j) * 2 + h] = sa;
            sa += cls((int64_t)l - (int64_t)(gb * B + B - 2 + h));
          }
        }
      }
    }
  s->prcv_off[((size_t)S + 1) * W] = ra;
  s->psnd_off[((size_t)S + 1) * W] = sa;
  if (ra != ps.nrecv || sa != ps.nsend) return fail(GM_ECORRUPT, "halo plan: %llu / %llu planes, sized %llu / %llu",
                                                   (unsigned long long)ra, (unsigned long long)sa,
                                                   (unsigned long long)ps.nrecv, (unsigned long long)ps.nsend);
  // entries by level
  for (u64 j = 0; j < nb; j++)
    for (u64 o = 0; o < B; o++) {
      const u64 t = gblk(j) * B + o;
      for (uint32_t c = 0; c <= smax; c++)
        if (t + c <= S) s->ploff[t + c + 1] += ncl[c];
    }
  for (uint32_t l = 0; l <= S; l++) s->ploff[l + 1] += s->ploff[l];
  if (s->ploff[S + 1] != ps.nlocal) return fail(GM_ECORRUPT, "plane lists: %llu entries for %llu planes",
                                               (unsigned long long)s->ploff[S + 1], (unsigned long long)ps.nlocal);
  bytes.resize(ps.nlocal * sizeof(PlaneEntry));
  PlaneEntry* E = (PlaneEntry*)bytes.data();
  std::vector<u64> pos(s->ploff.begin(), s->ploff.end());
  for (u64 j = 0; j < nb; j++) {
    const u64 gb = gblk(j);
    for (u64 o = 0; o < B; o++) {
      const u64 t = gb * B + o;
      for (u64 l = 0; l < Z; l++) {
        const u64 lev = t + sig[l];
        PlaneEntry e;
        e.p = (uint32_t)((j * B + o) * Z + l);
        auto halo = [&](u64 k) -> uint32_t {  // neighbour at top value t - k
          if (t < k) return kPlaneAbsent;
          if (o >= k) return kPlaneLocal;
          const u64 h = o + 2 - k;  // halo slice: top value gB - 2 + h
          return (uint32_t)(rgb[((size_t)(lev - k) * nb + j) * 2 + h] + rk[l]);
        };
        e.top1 = halo(1);
        e.top2 = halo(2);
        e.send = (o + 2 >= B && gb + 1 < ps.nblocks) ? (uint32_t)(sgb[((size_t)lev * nb + j) * 2 + (o + 2 - B)] + rk[l])
                                                     : kPlaneAbsent;
        E[pos[lev]++] = e;
      }
    }
  }
  // per level, the planes that read a halo plane (top values gB, gB + 1 of
  // blocks with a predecessor) last: the launch can be split into an own
  // part and a boundary part that waits for the exchange (run_planes)
  s->pbnd.assign((size_t)S + 1, 0);
  auto reads_halo = [](const PlaneEntry& e) { return e.top1 < kPlaneLocal || e.top2 < kPlaneLocal; };
  for (uint32_t l = 0; l <= S; l++) {
    PlaneEntry* a = E + s->ploff[l];
    PlaneEntry* b = E + s->ploff[l + 1];
    s->pbnd[l] = s->ploff[l] + (u64)(std::stable_partition(a, b, [&](const PlaneEntry& e) { return !reads_halo(e); }) - a);
  }
  return 0;
}

template <class F>
static void plane_no_dispatch(uint32_t no, F&& f);

// solver set-up for PLANES buffers (gm_solver_create_shard)
static int plane_setup(gm_solver* s, const gm_buffers* buf) {
  PlaneShape ps;
  int rc = plane_shape(&s->d, s->rank, s->world, buf->flags, &ps);
  if (rc) return rc;
  if (buf->table_bytes < ps.table_bytes || buf->scratch_bytes < ps.scratch_bytes)
    return fail(GM_EINVAL, "planes table / scratch of %llu / %llu bytes, the plan needs %llu / %llu (plan with the same "
                           "flags)", (unsigned long long)buf->table_bytes, (unsigned long long)buf->scratch_bytes,
                (unsigned long long)ps.table_bytes, (unsigned long long)ps.scratch_bytes);
  s->pg = ps.g;
  s->pwb = ps.wb;
  s->pform = ps.form;
  s->pS = ps.S;
  char* t = (char*)buf->table;
  s->ptab = t + ps.words_off;
  s->pbits = (uint32_t*)(t + ps.bits_off);
  s->precv = t + ps.recv_off;
  s->psend = t + ps.send_off;
  char* sc = (char*)buf->scratch;
  s->pzero = (const uint4*)(sc + ps.zero_off);
  s->plist = sc + ps.list_off;
  s->pnrecv = ps.nrecv;
  s->pnsend = ps.nsend;
  s->pstage_k = ps.stage_k;
  s->pkeys = ps.nkeys;
  s->prows = ps.nrows;
  std::vector<uint8_t> lb;
  rc = plane_lists(s, ps, lb);
  if (rc) return rc;
  HIPCHK(hipMemset((void*)s->pzero, 0, 4096));
  HIPCHK(hipMemcpy((void*)s->plist, lb.data(), lb.size(), hipMemcpyHostToDevice));
  s->pflow_ok = false;
  if (ps.flow) {
    // k_plane_flow's visits (gm_plane.h): each level's planes in list order,
    // padded to whole visits; the level's visits cut into 8 contiguous XCD
    // chunks, a chunk dealt round robin over its XCD's sequences
    const uint32_t* L = (const uint32_t*)lb.data();
    // (lab knob GM_PLANE_FLOW_SEQ: sequences per XCD, 1..kPlaneFlowSeqMax; A/B)
    uint32_t nseq = kPlaneFlowSeq;
    if (const char* e = lab_env("GM_PLANE_FLOW_SEQ")) nseq = std::max(1u, std::min(kPlaneFlowSeqMax, (uint32_t)atoi(e)));
    const uint32_t nq = 8 * nseq;
    std::vector<std::vector<uint32_t>> qv(nq);
    // (lab knob GM_PLANE_FLOW_DEAL=1: XCD x takes the planes whose top outer
    // digit lies in slab x of 8 -- the same XCD for a plane at every level,
    // so neighbours along the other digits share its L2 -- instead of an
    // even chunk of every level; A/B)
    const char* deal_e = lab_env("GM_PLANE_FLOW_DEAL");
    const bool slabs = deal_e && atoi(deal_e) == 1 && ps.g.no >= 2;
    const uint32_t tb = ps.g.base[ps.g.no > 0 ? ps.g.no - 1 : 0];
    for (uint32_t l = 0; l <= ps.S; l++) {
      std::vector<uint32_t> v(L + s->ploff[l], L + s->ploff[(size_t)l + 1]);
      if (slabs) {
        std::vector<std::vector<uint32_t>> xv(8);
        for (uint32_t P : v) {
          const uint32_t top = (uint32_t)((P / ps.g.stride[ps.g.no - 1]) % tb);
          xv[std::min(7u, top * 8u / tb)].push_back(P);
        }
        for (uint32_t x = 0; x < 8; x++) {
          while (xv[x].size() % 4) xv[x].push_back(kPlaneAbsent);
          for (u64 i = 0; i < xv[x].size() / 4; i++) {
            auto& q = qv[x + 8 * (i % nseq)];
            q.insert(q.end(), xv[x].begin() + 4 * i, xv[x].begin() + 4 * i + 4);
          }
        }
        continue;
      }
      while (v.size() % 4) v.push_back(kPlaneAbsent);
      const u64 nv = v.size() / 4, chunk = (nv + 7) / 8;
      for (u64 x = 0; x < 8; x++)
        for (u64 i = x * chunk; i < std::min(nv, (x + 1) * chunk); i++) {
          auto& q = qv[x + 8 * ((i - x * chunk) % nseq)];
          q.insert(q.end(), v.begin() + 4 * i, v.begin() + 4 * i + 4);
        }
    }
    std::vector<uint32_t> items, qoff(kPlaneFlowQ + 1, 0);
    for (uint32_t q = 0; q < nq; q++) {
      qoff[q + 1] = qoff[q] + (uint32_t)(qv[q].size() / 4);
      items.insert(items.end(), qv[q].begin(), qv[q].end());
    }
    if (items.size() > ps.nlocal + 24ull * (ps.S + 1)) return fail(GM_ECORRUPT, "plane flow: %zu visit entries", items.size());
    PlaneFlow& f = s->pflow;
    f.items = (const uint32_t*)(sc + ps.flow_off);
    f.qoff = (const uint32_t*)(sc + ps.flow_qoff_off);
    f.ctr = (uint32_t*)(sc + ps.flow_ctr_off);
    f.flags = (uint32_t*)(sc + ps.flow_flags_off);
    f.err = &s->st->err;
    f.epoch = 0;
    f.stall = ERR_PLANE_STALL;
    f.nseq = nseq;
    f.skip = kPlaneAbsent;
    f.mode = 0;
    HIPCHK(hipMemcpy((void*)f.items, items.data(), items.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy((void*)f.qoff, qoff.data(), qoff.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemset(f.ctr, 0, (size_t)kPlaneFlowLine * (kPlaneFlowQ + 2) * 4));
    HIPCHK(hipMemset(f.flags, 0, ps.nlocal * 4));
    // the grid: kPlaneFlowBlocksPerCU workgroups per CU (at most what the
    // CU holds at once -- every workgroup resident), whole rounds of the 64
    // sequences
    int occ = 0;
    plane_no_dispatch(ps.g.no, [&](auto NO) {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_plane_flow<decltype(NO)::value, true>, 256, 0) != hipSuccess)
        occ = 0;
    });
    const u64 cus = (u64)launch_grid() / 8;
    u64 bpc = std::min<u64>(kPlaneFlowBlocksPerCU, (u64)std::max(occ, 0));
    if (const char* e = lab_env("GM_PLANE_FLOW_BPC")) bpc = std::min<u64>(bpc, (u64)std::max(1, atoi(e)));  // (lab A/B)
    const u64 blocks = cus * bpc / nq * nq;
    s->pflow_grid = (uint32_t)blocks;
    s->pflow_ok = blocks >= nq;
  }
  s->w8 = ps.wb == 1;  // (the dense flags; the planes paths read pform)
  s->w16 = ps.wb == 2;
  return 0;
}

// ---------------------------------------------------------------------------
// host: launches
// ---------------------------------------------------------------------------
// kernel family: two planes per half-wave in packed 16-bit lanes for 8-bit
// words (1.65 vs 1.87 ms per 2^30 backward); one plane per half-wave for
// 16-bit words, where the packed form's register and byte footprint made it
// slower (3.80 vs 2.77 ms; profiles/r03b_plane_proto.txt); GM_F_PLANE_X1
// forces the one-plane form (A/B) of the absolute 8-bit forms; the relative
// forms have the packed form only
static bool plane_x1(const gm_solver* s) { return s->pform == 2 || (s->pform == 1 && (s->flags & GM_F_PLANE_X1)); }

// rs: the launch's outer digit sum mod 4 (the relative forms' kernels are
// specialised for it), or kPlaneRsVisit: per wave visit (staged lists)
constexpr uint32_t kPlaneRsVisit = 4;
template <int WB, int NO, bool SH>
static void plane_launch_t(gm_solver* s, u64 a, u64 n, u64 pa, u64 pn, uint32_t rs) {
  if (!n) return;
  // next launch's entries [pa, pa + pn): lines to prefetch (none: pn = 0)
  const size_t esz = SH ? sizeof(PlaneEntry) : 4;
  const uint32_t* pf = (const uint32_t*)((const char*)s->plist + ((pa * esz) & ~(size_t)127));
  const uint32_t pfl = pn ? (uint32_t)(((pa + pn) * esz - ((pa * esz) & ~(size_t)127) + 127) / 128) : 0u;
  const bool x1 = plane_x1(s);
  const u64 waves = x1 ? (n + 1) / 2 : (n + 3) / 4;
  u64 blocks = (waves + 3) / 4;
  blocks = std::min<u64>((blocks + 7) & ~7ull, (u64)s->grid * 4);  // plane_share loops past the grid
  typedef typename PlaneWord<WB>::T T;
  const void* list = (const char*)s->plist + a * (SH ? sizeof(PlaneEntry) : 4);
  const dim3 grid((uint32_t)blocks), blk(256);
  // the row deal: uint32 lists, halo rows from rank - 1 / to rank + 1, one
  // entry (two rows) per list entry: the kernel indexes them from the launch's
  // first entry, a
  const bool hr = !SH && s->pg.rowdeal;
  const T* hrecv = hr && s->rank > 0 ? (const T*)s->precv + a * 64u : nullptr;
  T* hsend = hr && s->rank + 1 < s->world ? (T*)s->psend + a * 64u : nullptr;
  if constexpr (WB == 3) {
    auto go = [&](auto RS) {
      if constexpr (!SH) {
        if (hr) {
          hipLaunchKernelGGL((k_plane_resolve_x2<3, NO, false, decltype(RS)::value, true>), grid, blk, 0, s->stream,
                             (T*)s->ptab, list, (uint32_t)n, s->pg, s->pzero, hrecv, hsend, pf, pfl);
          return;
        }
      }
      hipLaunchKernelGGL((k_plane_resolve_x2<3, NO, SH, decltype(RS)::value>), grid, blk, 0, s->stream, (T*)s->ptab,
                         list, (uint32_t)n, s->pg, s->pzero, (const T*)s->precv, (T*)s->psend, pf, pfl);
    };
    if (SH && rs == kPlaneRsVisit) {
      go(std::integral_constant<int, -1>());
      return;
    }
    switch (rs & 3u) {
      case 0: go(std::integral_constant<int, 0>()); break;
      case 1: go(std::integral_constant<int, 1>()); break;
      case 2: go(std::integral_constant<int, 2>()); break;
      default: go(std::integral_constant<int, 3>()); break;
    }
  } else if (x1) {
    hipLaunchKernelGGL((k_plane_resolve<WB, NO, SH>), grid, blk, 0, s->stream, (T*)s->ptab, list, (uint32_t)n, s->pg,
                       s->pzero, (const T*)s->precv, (T*)s->psend, pf, pfl);
  } else {
    if constexpr (!SH && WB == 1) {
      if (hr) {
        hipLaunchKernelGGL((k_plane_resolve_x2<1, NO, false, 0, true>), grid, blk, 0, s->stream, (T*)s->ptab, list,
                           (uint32_t)n, s->pg, s->pzero, hrecv, hsend, pf, pfl);
        return;
      }
    }
    hipLaunchKernelGGL((k_plane_resolve_x2<WB, NO, SH, 0>), grid, blk, 0, s->stream, (T*)s->ptab, list, (uint32_t)n,
                       s->pg, s->pzero, (const T*)s->precv, (T*)s->psend, pf, pfl);
  }
}
template <int WB, bool SH>
static void plane_launch_w(gm_solver* s, u64 a, u64 n, u64 pa, u64 pn, uint32_t rs) {
  switch (s->pg.no) {
    case 0: if (!SH) plane_launch_t<WB, 0, false>(s, a, n, pa, pn, rs); break;
    case 1: plane_launch_t<WB, 1, SH>(s, a, n, pa, pn, rs); break;
    case 2: plane_launch_t<WB, 2, SH>(s, a, n, pa, pn, rs); break;
    case 3: plane_launch_t<WB, 3, SH>(s, a, n, pa, pn, rs); break;
    case 4: plane_launch_t<WB, 4, SH>(s, a, n, pa, pn, rs); break;
    case 5: plane_launch_t<WB, 5, SH>(s, a, n, pa, pn, rs); break;
    default: plane_launch_t<WB, 6, SH>(s, a, n, pa, pn, rs); break;
  }
}
// the solver's word form and shard flag as template arguments
template <class F>
static void plane_form_dispatch(const gm_solver* s, F&& f) {
  const bool sh = s->world > 1 && !s->pg.rowdeal;  // PlaneEntry lists (the top-heap deals)
  auto w = [&](auto WB) {
    if (sh) f(WB, std::true_type());
    else f(WB, std::false_type());
  };
  if (s->pform == 3) w(std::integral_constant<int, 3>());
  else if (s->pform == 2) w(std::integral_constant<int, 2>());
  else w(std::integral_constant<int, 1>());
}
// list entries [a, a + n) of the solver's level lists, all of outer digit
// sum = rs mod 4; [pa, pa + pn): the entries the next launch starts with,
// prefetched (pn = 0: none)
static void plane_launch_range(gm_solver* s, u64 a, u64 n, uint32_t rs, u64 pa = 0, u64 pn = 0) {
  plane_form_dispatch(s, [&](auto WB, auto SH) {
    plane_launch_w<decltype(WB)::value, decltype(SH)::value>(s, a, n, pa, pn, rs);
  });
}
template <int WB, int NO, bool SH>
static void plane_run_t(gm_solver* s, const PlaneRun& run) {
  typedef typename PlaneWord<WB>::T T;
  if (WB != 3 && plane_x1(s))
    hipLaunchKernelGGL((k_plane_run<WB, NO, SH, true>), dim3(1), dim3(kPlaneRunThreads), 0, s->stream, (T*)s->ptab,
                       s->plist, run, s->pg, s->pzero, (const T*)s->precv, (T*)s->psend);
  else
    hipLaunchKernelGGL((k_plane_run<WB, NO, SH, false>), dim3(1), dim3(kPlaneRunThreads), 0, s->stream, (T*)s->ptab,
                       s->plist, run, s->pg, s->pzero, (const T*)s->precv, (T*)s->psend);
}
template <int WB, bool SH>
static void plane_run_w(gm_solver* s, const PlaneRun& run) {
  switch (s->pg.no) {
    case 0: if (!SH) plane_run_t<WB, 0, false>(s, run); break;
    case 1: plane_run_t<WB, 1, SH>(s, run); break;
    case 2: plane_run_t<WB, 2, SH>(s, run); break;
    case 3: plane_run_t<WB, 3, SH>(s, run); break;
    case 4: plane_run_t<WB, 4, SH>(s, run); break;
    case 5: plane_run_t<WB, 5, SH>(s, run); break;
    default: plane_run_t<WB, 6, SH>(s, run); break;
  }
}
// Batches consecutive groups of list entries (plane levels, staged keys)
// into launches: a group of at most `narrow` planes joins the open run
// (k_plane_run, one workgroup), a wider one flushes the run and gets its own
// grid-wide launch.  flush() before anything that must see the groups so
// far done on the stream (an event, an exchange).
#ifndef GM_PLANE_RUN_PASSES
#define GM_PLANE_RUN_PASSES 1  // (A/B builds, tools/ab_runs.sh: 1 pass 1.607 ms, 2: 1.631, 3: 1.657, 4: 1.697)
#endif
struct PlaneBatcher {
  gm_solver* s;
  PlaneRun run{};
  u64 narrow;
  u64 launches = 0;  // grid launches + runs issued
  explicit PlaneBatcher(gm_solver* sv) : s(sv) {
    // one pass of the run's waves: one CU beats a grid launch up to about there
    narrow = (s->flags & GM_F_PLANE_NO_RUNS) || s->pg.rowdeal  // (k_plane_run carries no halo rows)
                 ? 0
                 : (u64)((double)(kPlaneRunThreads / 64) * (plane_x1(s) ? 2 : 4) * GM_PLANE_RUN_PASSES);
    run.n = 0;
  }
  void flush() {
    launches += run.n ? 1 : 0;
    if (run.n == 1) plane_launch_range(s, run.off[0], run.off[1] - run.off[0], run.visit ? kPlaneRsVisit : (uint32_t)run.rs & 3u);
    else if (run.n > 1) {
      plane_form_dispatch(s, [&](auto WB, auto SH) { plane_run_w<decltype(WB)::value, decltype(SH)::value>(s, run); });
    }
    run.n = 0;
    run.rs = 0;
    run.visit = 0;
  }
  // list entries [a, b), outer digit sum = rs mod 4; the next group's size
  // (prefetch)
  void add(u64 a, u64 b, uint32_t rs, u64 next = 0) {
    if (b == a) return;
    if (b - a > narrow) {
      flush();
      plane_launch_range(s, a, b - a, rs, b, next);
      launches++;
      return;
    }
    if (run.n == (uint32_t)kPlaneRunMax || (run.n && run.off[run.n] != a)) flush();
    if (run.n == 0) run.off[0] = (uint32_t)a;
    run.rs |= (u64)(rs & 3u) << (2 * run.n);
    run.visit = rs == kPlaneRsVisit;
    run.off[++run.n] = (uint32_t)b;
  }
};

// plane level l; part 0: all of it, 1: the planes that read no halo plane,
// 2: the ones that do
static void plane_launch(gm_solver* s, uint32_t l, int part = 0) {
  const u64 a = s->ploff[l], b = s->ploff[(size_t)l + 1];
  const u64 m = s->world > 1 ? s->pbnd[l] : b;
  if (part == 0) plane_launch_range(s, a, b - a, l);
  else if (part == 1) plane_launch_range(s, a, m - a, l);
  else plane_launch_range(s, m, b - m, l);
}
template <class F>
static void plane_no_dispatch(uint32_t no, F&& f) {
  switch (no) {
    case 0: f(std::integral_constant<int, 0>()); break;
    case 1: f(std::integral_constant<int, 1>()); break;
    case 2: f(std::integral_constant<int, 2>()); break;
    case 3: f(std::integral_constant<int, 3>()); break;
    case 4: f(std::integral_constant<int, 4>()); break;
    case 5: f(std::integral_constant<int, 5>()); break;
    default: f(std::integral_constant<int, 6>()); break;
  }
}
static void plane_reach_launch(gm_solver* s, hipStream_t stream = nullptr) {
  const u64 nq = (u64)s->pg.nplanes;  // one thread per plane (its 32 row bits)
  const int grid = (int)std::max<u64>(1, std::min<u64>((nq + 255) / 256, (u64)std::min(s->grid, kCountSlots)));
  plane_no_dispatch(s->pg.no, [&](auto NO) {
    hipLaunchKernelGGL((k_plane_reach<decltype(NO)::value>), dim3(grid), dim3(256), 0, stream ? stream : s->stream,
                       s->pbits, s->pg, s->bcount, s->st, s->pmark());
  });
}

// Pairs of narrow plane levels in one launch (k_plane_pair, gm_plane.h):
// one-table solves of the 8-bit absolute forms with 1-4 outer digits of
// power-of-two bases, levels (l, l + 1) both wider than a one-workgroup run
// and both at most kPlanePairMax planes (the pair's redundant first visits
// grow with the width: 14 pairs over levels 4-17 and 107-120 of the 2^30
// bench table at the default).  (lab knob GM_PLANE_PAIR_MAX; 0: no pairs)
constexpr u64 kPlanePairMax = 1200;
// (A/B, GM_PLANE_FWD=3) the forward's side-stream start: the first level
// past the widest with at most this many planes (run_planes)
constexpr u64 kPlaneFwdTail = 2048;
static u64 plane_pair_max(const gm_solver* s) {
  static const long long v = [] {
    const char* e = lab_env("GM_PLANE_PAIR_MAX");
    return e ? atoll(e) : -1ll;
  }();
  const bool ok = s->world <= 1 && s->pform == 1 && !plane_x1(s) && s->pg.no >= 1 && s->pg.no <= 4 && s->pg.pow2;
  return !ok ? 0 : v >= 0 ? (u64)v : kPlanePairMax;
}
// levels l and l + 1 of a one-table solve in one launch
static void plane_pair_launch(gm_solver* s, uint32_t l) {
  const u64 a = s->ploff[(size_t)l + 1], n = s->ploff[(size_t)l + 2] - a;  // level l + 1's planes
  const u64 blocks = std::min<u64>((n + 3) / 4, (u64)s->grid * 4);
  const uint32_t* list = (const uint32_t*)s->plist + a;
  plane_no_dispatch(s->pg.no, [&](auto NO) {
    constexpr int no = decltype(NO)::value;
    if constexpr (no >= 1 && no <= 4)
      hipLaunchKernelGGL((k_plane_pair<no>), dim3((uint32_t)blocks), dim3(256), 0, s->stream, (uint8_t*)s->ptab, list,
                         (uint32_t)n, s->pg, s->pzero);
  });
}

// halo segment (level l, peer p) of a shard's send / receive plan: first
// plane and plane count
static u64 plane_seg(const std::vector<u64>& off, uint32_t l, int W, int p, u64* n) {
  const size_t i = (size_t)l * W + p;
  *n = off[i + 1] - off[i];
  return off[i];
}

// per-peer send / receive plane counts of a shard over all levels, as
// fingerprints out[2p] (sends to p), out[2p + 1] (receives from p) --
// checked against the peers' before the first exchange: a mismatched
// receive would wait forever
static void plane_sigs(const gm_solver* s, u64* out) {
  const int W = s->world;
  const uint32_t nl = (uint32_t)((s->psnd_off.size() - 1) / W);
  for (int p = 0; p < W; p++) {
    u64 a = 0xcbf29ce484222325ull, b = a, n;
    for (uint32_t l = 0; l < nl; l++) {
      plane_seg(s->psnd_off, l, W, p, &n);
      a = (a ^ n) * 0x100000001b3ull;
      plane_seg(s->prcv_off, l, W, p, &n);
      b = (b ^ n) * 0x100000001b3ull;
    }
    out[2 * p] = a;
    out[2 * p + 1] = b;
  }
}

// exchange the boundary planes of level l: every shard sends its (l, p)
// send segment to each peer p and receives each peer q's into its (l, q)
// receive segment (mode 1 RCCL, one grouped send/recv set; 2 in-process
// copies; 3 host-staged, world - 1 shifted pairwise rounds)
static int plane_exchange(std::vector<gm_solver*>& ss, uint32_t l, int mode, hipStream_t cs) {
  const u64 pb = 1024ull * ss[0]->pwb;
  const int W = ss[0]->world;
  if (mode == 2) {
    for (int r = 0; r < W; r++)
      for (int p = 0; p < W; p++) {
        gm_solver* a = ss[(size_t)r];
        gm_solver* b = ss[(size_t)p];
        u64 ns, nr;
        const u64 so = plane_seg(a->psnd_off, l, W, p, &ns), ro = plane_seg(b->prcv_off, l, W, r, &nr);
        if (ns != nr) return fail(GM_ECORRUPT, "level %u: shard %d sends %llu planes, shard %d expects %llu", l, r,
                                  (unsigned long long)ns, p, (unsigned long long)nr);
        if (ns)
          HIPCHK(hipMemcpyAsync((char*)b->precv + ro * pb, (const char*)a->psend + so * pb, ns * pb,
                                hipMemcpyDeviceToDevice, cs));
      }
    return 0;
  }
  gm_solver* s = ss[0];
  auto sbuf = [&](int p, u64* n) { return (void*)((char*)s->psend + plane_seg(s->psnd_off, l, W, p, n) * pb); };
  auto rbuf = [&](int p, u64* n) { return (void*)((char*)s->precv + plane_seg(s->prcv_off, l, W, p, n) * pb); };
  if (mode == 1) {
    RCCL_LIVE(s);
    ncclResult_t r = ncclGroupStart();
    for (int p = 0; p < W && r == ncclSuccess; p++) {
      u64 ns, nr;
      void* sb = sbuf(p, &ns);
      void* rb = rbuf(p, &nr);
      if (ns) r = ncclSend(sb, ns * pb, ncclUint8, p, s->comm, cs);
      if (nr && r == ncclSuccess) r = ncclRecv(rb, nr * pb, ncclUint8, p, s->comm, cs);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
      return fail(GM_EHIP, "RCCL halo exchange: %s", ncclGetErrorString(r != ncclSuccess ? r : r2));
    return 0;
  }
  for (int k = 1; k < W; k++) {
    const int to = (s->rank + k) % W, from = (s->rank + W - k) % W;
    u64 ns, nr;
    void* sb = sbuf(to, &ns);
    void* rb = rbuf(from, &nr);
    std::vector<HostRange> out, in;
    if (ns) out.push_back({sb, ns * pb});
    if (nr) in.push_back({rb, nr * pb});
    int rc = xfer_ranges(s, out, to, in, from, cs);
    if (rc) return rc;
  }
  return 0;
}

// before the first sharded solve: every shard's sends to each peer must
// match that peer's receives from it (fingerprints all-gathered)
static int plane_check_plan(std::vector<gm_solver*>& ss, int mode, hipStream_t st) {
  const int W = ss[0]->world;
  const size_t m = (size_t)2 * W;  // fingerprints per shard
  std::vector<u64> all(m * W);
  if (mode == 2) {
    for (gm_solver* s : ss) plane_sigs(s, &all[m * s->rank]);
  } else {
    std::vector<u64> mine(m);
    plane_sigs(ss[0], mine.data());
    if (mode == 3) {
      int rc = xfer_call(ss[0], GM_XFER_ALLGATHER, mine.data(), m * 8, -1, all.data(), all.size() * 8, -1);
      if (rc) return rc;
    } else {
      RCCL_LIVE(ss[0]);
      u64* dev = nullptr;
      HIPCHK(hipMalloc((void**)&dev, (m + all.size()) * 8));
      HIPCHK(hipMemcpyAsync(dev, mine.data(), m * 8, hipMemcpyHostToDevice, st));
      ncclResult_t r = ncclAllGather(dev, dev + m, m, ncclUint64, ss[0]->comm, st);
      hipError_t e = hipMemcpyAsync(all.data(), dev + m, all.size() * 8, hipMemcpyDeviceToHost, st);
      if (e == hipSuccess) e = hipStreamSynchronize(st);
      (void)hipFree(dev);
      if (r != ncclSuccess) return fail(GM_EHIP, "RCCL plan check: %s", ncclGetErrorString(r));
      if (e != hipSuccess) return fail(GM_EHIP, "plan check: %s", hipGetErrorString(e));
    }
  }
  for (int r = 0; r < W; r++)
    for (int p = 0; p < W; p++)
      if (all[m * r + 2 * p] != all[m * p + 2 * r + 1])
        return fail(GM_ECORRUPT, "halo plan mismatch: shard %d's sends vs shard %d's receives", r, p);
  for (gm_solver* s : ss) s->halo_ok = true;
  return 0;
}

// Staged shards: every rank's geometry must be the same staged deal (the
// row messages pair by construction then: both sides size row s from the
// lower digits alone)
static u64 plane_stage_sig(const gm_solver* s) {
  u64 h = 0xcbf29ce484222325ull;
  auto mix = [&](u64 v) { h = (h ^ v) * 0x100000001b3ull; };
  mix(s->pstage_k);
  mix(s->pkeys);
  mix(s->prows);
  mix(s->pg.B);
  mix(s->pg.Z);
  mix(s->pg.rowdeal);
  mix(s->world);
  const std::vector<u64>& rows = s->rank > 0 ? s->prcv_off : s->psnd_off;
  for (u64 v : rows) mix(v);
  return h;
}
static int plane_check_stage(std::vector<gm_solver*>& ss, int mode, hipStream_t st) {
  const int W = ss[0]->world;
  std::vector<u64> all((size_t)W);
  if (mode == 2 || mode == 4) {
    for (gm_solver* s : ss) all[(size_t)s->rank] = plane_stage_sig(s);
  } else {
    u64 mine = plane_stage_sig(ss[0]);
    if (mode == 3) {
      int rc = xfer_call(ss[0], GM_XFER_ALLGATHER, &mine, 8, -1, all.data(), all.size() * 8, -1);
      if (rc) return rc;
    } else {
      RCCL_LIVE(ss[0]);
      u64* dev = nullptr;
      HIPCHK(hipMalloc((void**)&dev, (size_t)(1 + W) * 8));
      HIPCHK(hipMemcpyAsync(dev, &mine, 8, hipMemcpyHostToDevice, st));
      ncclResult_t r = ncclAllGather(dev, dev + 1, 1, ncclUint64, ss[0]->comm, st);
      hipError_t e = hipMemcpyAsync(all.data(), dev + 1, all.size() * 8, hipMemcpyDeviceToHost, st);
      if (e == hipSuccess) e = hipStreamSynchronize(st);
      (void)hipFree(dev);
      if (r != ncclSuccess) return fail(GM_EHIP, "RCCL plan check: %s", ncclGetErrorString(r));
      if (e != hipSuccess) return fail(GM_EHIP, "plan check: %s", hipGetErrorString(e));
    }
  }
  for (int r = 1; r < W; r++)
    if (all[(size_t)r] != all[0])
      return fail(GM_ECORRUPT, "staged plan mismatch: shard %d's geometry differs from shard 0's", r);
  for (gm_solver* s : ss) s->halo_ok = true;
  return 0;
}

// Fault injection for the failure tests only: GM_FAULT_STAGED="rank:key"
// makes shard `rank` fail at key `key` of the staged backward as a DEFERRED
// error (below); "rank:key:early" returns at once instead -- the path that
// solve_multi's communicator abort has to bound.  Unset: no effect.
struct StagedFault {
  int rank = -1;
  uint32_t key = 0;
  bool early = false;
};
static StagedFault staged_fault() {
  StagedFault f;
  const char* e = lab_env("GM_FAULT_STAGED");
  if (!e || !*e) return f;
  unsigned r = 0, k = 0;
  char tail[16] = {0};
  const int n = sscanf(e, "%u:%u:%15s", &r, &k, tail);
  if (n >= 2) {
    f.rank = (int)r;
    f.key = k;
    f.early = n == 3 && strcmp(tail, "early") == 0;
  }
  return f;
}
__global__ void k_err_or(DevState* st, uint32_t e) {
  if (threadIdx.x == 0) st->err |= e;
}
// a deferred failure (herr, already reported through fail()): remembered on
// the shard, and ERR_SHARD_FAILED set in its error word for the reduction
static int staged_defer(gm_solver* s, int herr, hipStream_t st) {
  if (!herr) return 0;
  s->defer_rc = herr;
  s->defer_msg = gm_last_error();
  hipLaunchKernelGGL(k_err_or, dim3(1), dim3(64), 0, st, s->st, (uint32_t)ERR_SHARD_FAILED);
  return 0;
}

// The staged backward (see plane_stage_k): every rank walks its keys; row s
// of the halo is waited for before key k s and sent after key B - 1 + k s.
//  mode 2 (in-process group, one stream): shard after shard, rows copied to
//    the next shard as they complete (the next shard runs after this one).
//  mode 1 (RCCL): transfers r -> r + 1 travel on comm when r is even and on
//    comm2 (ncclCommSplit: up front for an in-process group, solve_multi;
//    on first use by a one-process-per-GPU rank) when odd, so on every rank one
//    communicator carries only its receives and the other only its sends:
//    receives are posted ahead (a window of rows) on the receive stream and
//    can never hold up the sends, which follow the rank's own keys on the
//    send stream.
//  mode 3 (host-staged transport): blocking row transfers in key order.
//  mode 4 (one-GPU rehearsal of mode 1, every shard in one process on its
//    own streams): mode 1's code path -- key loop, receive window, send /
//    receive streams, SE / RE events, end-of-solve joins -- with a device
//    copy on the receiver's receive stream in place of each ncclSend /
//    ncclRecv pair.  What only RCCL itself exercises: ncclCommSplit, the
//    send / receive matching on the two communicators, RCCL's own progress.
// Failures of a rank's own work (a stream / event call, a launch) are
// DEFERRED in modes 1, 3 and 4: the rank stops computing but keeps posting
// every halo send and receive of its schedule, so its peers finish their
// keys instead of waiting forever in a receive, marks ERR_SHARD_FAILED in its
// error word, which the end-of-solve reduction hands to every rank, and
// reports its own error there (s->defer_rc).  Only a failed transfer call
// returns at once: the exchange itself is then broken.
static int plane_backward_staged(std::vector<gm_solver*>& ss, int mode, hipStream_t st, u64* nlaunch) {
  gm_solver* s0 = ss[0];
  // (the row deal: key = row = plane level, each final after its own key --
  // a lag of B - 1 = 0 -- and two rows per plane in the halo)
  const bool rowdeal = s0->pg.rowdeal != 0;
  const uint32_t k = s0->pstage_k, K = s0->pkeys, R = s0->prows, B = rowdeal ? 1u : s0->pg.B;
  const int W = s0->world;
  const u64 pb = (rowdeal ? 64ull : 1024ull) * s0->pwb;
  auto row_done = [&](uint32_t key, uint32_t* r) {  // key completes row *r (its last slice)
    if (key + 1 < B || (key - (B - 1)) % k) return false;
    *r = (key - (B - 1)) / k;
    return *r < R;
  };
  auto row_need = [&](uint32_t key, uint32_t* r) {  // key is the first to read row *r
    if (key % k) return false;
    *r = key / k;
    return *r < R;
  };
  auto seg = [](const std::vector<u64>& off, uint32_t r, u64* n) {
    *n = off[r + 1] - off[r];
    return off[r];
  };
  auto launch_key = [K, rowdeal](PlaneBatcher& pb_, uint32_t key) {
    const std::vector<u64>& o = pb_.s->ploff;
    // relative forms: s mod 4 per wave visit (plane_lists_staged); the row
    // deal's keys are plane levels, of one s each
    const uint32_t rs = rowdeal ? key & 3u : kPlaneRsVisit;
    pb_.add(o[key], o[(size_t)key + 1], rs, key + 1 < K ? o[(size_t)key + 2] - o[(size_t)key + 1] : 0);
  };
  if (mode == 2) {
    for (int c = 0; c < W; c++) {
      gm_solver* s = ss[(size_t)c];
      PlaneBatcher bat(s);
      for (uint32_t key = 0; key < K; key++) {
        launch_key(bat, key);
        uint32_t r;
        if (c + 1 < W && row_done(key, &r)) {
          bat.flush();
          gm_solver* t = ss[(size_t)c + 1];
          u64 ns, nr;
          const u64 so = seg(s->psnd_off, r, &ns), ro = seg(t->prcv_off, r, &nr);
          if (ns != nr) return fail(GM_ECORRUPT, "row %u: shard %d sends %llu planes, shard %d expects %llu", r, c,
                                    (unsigned long long)ns, c + 1, (unsigned long long)nr);
          if (ns)
            HIPCHK(hipMemcpyAsync((char*)t->precv + ro * pb, (const char*)s->psend + so * pb, ns * pb,
                                  hipMemcpyDeviceToDevice, st));
        }
      }
      bat.flush();
      if (c == 0) *nlaunch = bat.launches;
    }
    return 0;
  }
  if (mode == 3) {
    gm_solver* s = s0;
    PlaneBatcher bat(s);
    const int rank = s->rank;
    const bool rx = rank > 0, tx = rank + 1 < W;
    auto rbuf = [&](uint32_t r, u64* n) { return (void*)((char*)s->precv + seg(s->prcv_off, r, n) * pb); };
    auto sbuf = [&](uint32_t r, u64* n) { return (void*)((char*)s->psend + seg(s->psnd_off, r, n) * pb); };
    const StagedFault fault = staged_fault();
    int herr = 0;  // deferred failure (see above)
    for (uint32_t key = 0; key < K; key++) {
      uint32_t r;
      if (!herr && fault.rank == rank && fault.key == key) {
        herr = fail(GM_EHIP, "injected fault: shard %d at key %u", rank, key);
        if (fault.early) return herr;
      }
      if (rx && row_need(key, &r)) {
        bat.flush();
        u64 n;
        void* b = rbuf(r, &n);
        std::vector<HostRange> out, in;
        if (n) in.push_back({b, n * pb});
        int rc = xfer_ranges(s, out, -1, in, rank - 1, st);
        if (rc) return rc;
      }
      if (!herr) launch_key(bat, key);
      if (tx && row_done(key, &r)) {
        bat.flush();
        u64 n;
        void* b = sbuf(r, &n);
        std::vector<HostRange> out, in;
        if (n) out.push_back({b, n * pb});
        int rc = xfer_ranges(s, out, rank + 1, in, -1, st);
        if (rc) return rc;
      }
    }
    bat.flush();
    *nlaunch = bat.launches;
    return staged_defer(s, herr, st);
  }
  // mode 1 (RCCL) and mode 4 (its one-GPU rehearsal): the same key loop,
  // receive window, streams, events and joins per shard; only the two
  // transfer calls differ.  Per shard: compute stream s->stream, send
  // stream ts, receive stream rs; RE[r] row r received, SE[r] row r final
  // here, XS[r] row r handed to the send stream's transfer.
  const StagedFault fault = staged_fault();
  auto staged_rank = [&](gm_solver* s, auto&& recv_op, auto&& send_op) -> int {
    PlaneBatcher bat(s);
    const int rank = s->rank;
    const bool rx = rank > 0, tx = rank + 1 < W;
    hipStream_t cst = s->stream;
    // set-up (before any transfer of this rank: a failure here is returned
    // at once, as a mode-1 peer's matching calls have not been posted either)
    if (!s->cstream) HIPCHK(hipStreamCreateWithFlags(&s->cstream, hipStreamNonBlocking));
    if (!s->cstream2) HIPCHK(hipStreamCreateWithFlags(&s->cstream2, hipStreamNonBlocking));
    while (s->pev.size() < 3 * (size_t)R + 3) {
      hipEvent_t e;
      HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      s->pev.push_back(e);
    }
    hipEvent_t* RE = s->pev.data();      // row r received
    hipEvent_t* SE = RE + R;             // row r final on this rank
    hipEvent_t* XS = SE + R;             // row r's send issued on the send stream
    hipEvent_t* XE = XS + R;             // [0] start, [1] sends done, [2] receives done
    hipStream_t ts = s->cstream, rs = s->cstream2;
    int herr = 0;  // deferred failure: compute stops, the transfers go on
    auto dchk = [&](hipError_t e, const char* what) {
      if (e != hipSuccess && !herr) herr = fail(GM_EHIP, "%s: %s", what, hipGetErrorString(e));
    };
    dchk(hipEventRecord(XE[0], cst), "hipEventRecord");
    dchk(hipStreamWaitEvent(ts, XE[0], 0), "hipStreamWaitEvent");
    dchk(hipStreamWaitEvent(rs, XE[0], 0), "hipStreamWaitEvent");
    constexpr uint32_t kAhead = 8;  // rows whose receives are posted ahead of the key that reads them
    uint32_t posted = 0;            // rows [0, posted) have their receive posted
    auto post_to = [&](uint32_t lim) -> int {
      for (; rx && posted < std::min(lim, R); posted++) {
        u64 n;
        void* b = (void*)((char*)s->precv + seg(s->prcv_off, posted, &n) * pb);
        int rc = recv_op(s, posted, b, n, rs);
        if (rc) return rc;
        dchk(hipEventRecord(RE[posted], rs), "hipEventRecord");
      }
      return 0;
    };
    for (uint32_t key = 0; key < K; key++) {
      uint32_t r;
      if (!herr && fault.rank == rank && fault.key == key) {
        herr = fail(GM_EHIP, "injected fault: shard %d at key %u", rank, key);
        if (fault.early) return herr;
      }
      if (rx && row_need(key, &r)) {
        bat.flush();
        int rc = post_to(r + 1 + kAhead);
        if (rc) return rc;
        dchk(hipStreamWaitEvent(cst, RE[r], 0), "hipStreamWaitEvent");
      }
      if (!herr) launch_key(bat, key);
      if (tx && row_done(key, &r)) {
        bat.flush();
        dchk(hipEventRecord(SE[r], cst), "hipEventRecord");
        dchk(hipStreamWaitEvent(ts, SE[r], 0), "hipStreamWaitEvent");
        u64 n;
        void* b = (void*)((char*)s->psend + seg(s->psnd_off, r, &n) * pb);
        int rc = send_op(s, r, b, n, ts);
        if (rc) return rc;
        dchk(hipEventRecord(XS[r], ts), "hipEventRecord");
      }
    }
    bat.flush();
    if (rank == 0 || mode == 1) *nlaunch = bat.launches;
    int rc = post_to(R);
    if (rc) return rc;
    dchk(hipEventRecord(XE[1], ts), "hipEventRecord");
    dchk(hipEventRecord(XE[2], rs), "hipEventRecord");
    dchk(hipStreamWaitEvent(cst, XE[1], 0), "hipStreamWaitEvent");
    dchk(hipStreamWaitEvent(cst, XE[2], 0), "hipStreamWaitEvent");
    return staged_defer(s, herr, cst);
  };
  if (mode == 4) {
    // the ranks' host loops in pipeline order (a row's XS event exists before
    // the next rank's receive waits on it); every rank on its own streams of
    // the one GPU, so its keys overlap the ranks before it as on separate
    // GPUs; a device copy on the receiver's receive stream stands in for the
    // ncclSend / ncclRecv pair: it waits for the sender's XS[r], i.e. row r
    // final there and handed to its send stream
    for (int c = 0; c < W; c++) {
      int rc = staged_rank(
          ss[(size_t)c],
          [&](gm_solver* t, uint32_t row, void* b, u64 n, hipStream_t rs) -> int {
            gm_solver* f = ss[(size_t)t->rank - 1];
            u64 ns;
            const u64 so = seg(f->psnd_off, row, &ns);
            if (ns != n) return fail(GM_ECORRUPT, "row %u: shard %d sends %llu planes, shard %d expects %llu", row,
                                     f->rank, (unsigned long long)ns, t->rank, (unsigned long long)n);
            if (!n) return 0;
            HIPCHK(hipStreamWaitEvent(rs, f->pev[2 * (size_t)R + row], 0));
            HIPCHK(hipMemcpyAsync(b, (const char*)f->psend + so * pb, n * pb, hipMemcpyDeviceToDevice, rs));
            return 0;
          },
          [&](gm_solver*, uint32_t, void*, u64, hipStream_t) -> int { return 0; });
      if (rc) return rc;
    }
    return 0;
  }
  // mode 1: transfers r -> r + 1 on comm when r is even and on comm2 when odd
  gm_solver* s = s0;
  if (!s->comm2) {
    ncclResult_t e = ncclCommSplit(s->comm, 0, s->rank, &s->comm2, nullptr);
    if (e != ncclSuccess) return fail(GM_EHIP, "ncclCommSplit: %s", ncclGetErrorString(e));
  }
  ncclComm_t csend = (s->rank % 2 == 0) ? s->comm : s->comm2, crecv = (s->rank % 2 == 1) ? s->comm : s->comm2;
  return staged_rank(
      s,
      [&](gm_solver* t, uint32_t, void* b, u64 n, hipStream_t rs) -> int {
        if (!n) return 0;
        RCCL_LIVE(t);
        const ncclResult_t e = ncclRecv(b, n * pb, ncclUint8, t->rank - 1, crecv, rs);
        if (e != ncclSuccess) return fail(GM_EHIP, "RCCL halo receive: %s", ncclGetErrorString(e));
        return 0;
      },
      [&](gm_solver* t, uint32_t, void* b, u64 n, hipStream_t ts) -> int {
        if (!n) return 0;
        RCCL_LIVE(t);
        const ncclResult_t e = ncclSend(b, n * pb, ncclUint8, t->rank + 1, csend, ts);
        if (e != ncclSuccess) return fail(GM_EHIP, "RCCL halo send: %s", ncclGetErrorString(e));
        return 0;
      });
}

// The PLANES solve.  Steps (gm_solver_set_steps, one table only): 2T like
// the other layouts; step 0 is the forward pass (reach map + counts), steps
// 1..T-1 are empty, step T + l is plane level l (l <= S), later steps empty.
// The end of a one-table solve: the host polls the stream for a bounded
// time (up to kPlaneSpinUs, about a narrow plane level: the solve's last
// launches), then sleeps in hipStreamSynchronize -- a solve's wake-up is not
// paid on every call, and no core is pinned for a long solve (round 5 spun
// without a bound: 1.325 vs 1.329 ms per bench step, within noise).  Queued
// solves (gm_solver_solve_async) do not wait here at all.
constexpr double kPlaneSpinUs = 100.0;
static hipError_t plane_wait(hipStream_t st) {
  const auto t0 = std::chrono::steady_clock::now();
  hipError_t e;
  while ((e = hipStreamQuery(st)) == hipErrorNotReady) {
    if (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() > kPlaneSpinUs)
      return hipStreamSynchronize(st);
    __builtin_ia32_pause();
  }
  return e;
}

// the counts of a finished solve (red: positions, edges, primitives, root
// word + 1, error bits) into the result
static int plane_result(const std::vector<gm_solver*>& ss, const u64* red, gm_result* out) {
  gm_solver* s0 = ss[0];
  out->positions = red[0];
  out->edges = red[1];
  out->primitives = red[2];
  out->levels = (uint32_t)s0->d.max_levels;
  out->max_level_width = 0;
  out->word_bits = 8 * s0->pwb;
  out->kernels = (plane_x1(s0) ? RK_PLANE : s0->pflow_last ? RK_PLANE_FLOW : RK_PLANE_X2) | (PK_PLANE << 16);
  const uint32_t word = red[3] ? (uint32_t)(red[3] - 1) : NO_WORD;
  out->root_word = word;
  if (red[4]) {
    for (gm_solver* s : ss)  // this process's shard failed: its own error
      if (s->defer_rc) return fail(s->defer_rc, "shard %d/%d: %s", s->rank, s->world, s->defer_msg.c_str());
    return fail(GM_ECORRUPT, "solve failed:%s", err_text((uint32_t)red[4]).c_str());
  }
  if (word == NO_WORD) return fail(GM_ECORRUPT, "root unresolved");
  out->root_value = (int32_t)(word & 3u);
  out->root_remoteness = word >> 2;
  return 0;
}

static int run_planes(std::vector<gm_solver*> ss, gm_result* out, bool async) {
  gm_solver* s0 = ss[0];
  const Desc& d = s0->d;
  const int T = d.max_levels;
  const uint32_t S = s0->pS;
  // mode 2: a group on ONE stream; mode 4: a group whose shards have their
  // own streams -- the rehearsal of mode 1's staged schedule
  const bool own_streams = ss.size() > 1 && ss[1]->stream != s0->stream;
  const int mode = s0->world <= 1 ? 0 : ss.size() != 1 ? (own_streams ? 4 : 2) : s0->xfer ? 3 : 1;
  if (mode == 1 && !s0->comm) return fail(GM_EINVAL, "shard %d/%d has no communicator (gm_solver_comm_init)", s0->rank, s0->world);
  if (mode == 2 || mode == 4) {
    if ((int)ss.size() != s0->world) return fail(GM_EINVAL, "group solve needs all %d shards", s0->world);
    for (size_t g = 0; g < ss.size(); g++) {
      if (ss[g]->rank != (int)g || ss[g]->mode != GM_MODE_PLANES)
        return fail(GM_EINVAL, "group shards must be ranks 0..n-1");
      for (size_t h = 0; h < g; h++)
        if ((mode == 2) != (ss[g]->stream == ss[h]->stream))
          return fail(GM_EINVAL, "group shards share one stream, or (the staged rehearsal) each has its own");
    }
    if (mode == 4 && !s0->pstage_k)
      return fail(GM_EINVAL, "shards on their own streams rehearse the staged deal only (this shape is level-synchronous)");
  }
  const int first = mode == 0 ? (int)s0->step_first : 0;
  const int stop = mode == 0 && s0->step_stop ? (int)s0->step_stop : 2 * T;
  s0->step_first = s0->step_stop = 0;
  const bool timing = (s0->flags & GM_F_KERNEL_TIMING) && first == 0 && stop == 2 * T;
  if (async && (mode != 0 || first != 0 || stop != 2 * T || timing))
    return fail(GM_EINVAL, "queued solves: one-table PLANES full solves without kernel timing only");
  hipStream_t st = s0->stream;
  if (first > 0) {
    uint32_t wb = 0;
    HIPCHK(hipMemcpy(&wb, &s0->st->word_bits, sizeof wb, hipMemcpyDeviceToHost));
    if (wb != s0->pmark())
      return fail(GM_EINVAL, "resume: the scratch holds no %u-bit%s planes solve", 8 * s0->pwb,
                  s0->pform == 3 ? " relative" : "");
  }
  const bool staged = mode != 0 && s0->pstage_k;
  for (gm_solver* s : ss) {
    s->defer_rc = 0;
    s->defer_msg.clear();
  }
  if (mode != 0 && !s0->halo_ok) {
    int rc = staged ? plane_check_stage(ss, mode, st) : plane_check_plan(ss, mode, st);
    if (rc) return rc;
  }
  std::vector<hipEvent_t> ev;
  auto new_event = [&](hipEvent_t* e) -> int {
    HIPCHK(hipEventCreate(e));
    ev.push_back(*e);
    return 0;
  };
  auto cleanup = [&]() {
    for (auto e : ev) (void)hipEventDestroy(e);
  };
  // the solve's three timing events live with the solver (created once: a
  // create + destroy per event per solve was host time between solves); a
  // queued solve (gm_solver_solve_async) uses its ring slot's own
  hipEvent_t e0, e1, e2, etail;
  {
    hipEvent_t* se = async ? s0->pring[s0->pq_next % kPlaneRing].ev : s0->pse;
    for (int i = 0; i < 3; i++)
      if (!se[i]) HIPCHK(hipEventCreate(&se[i]));
    if (!se[4]) HIPCHK(hipEventCreate(&se[4]));
    e0 = se[0], e1 = se[1], e2 = se[2], etail = se[4];
  }
  std::vector<hipEvent_t> kr;  // per-level start/stop (shard 0's launches)
  hipEvent_t kx[2];
  if (timing) {
    kr.resize(2 * ((size_t)S + 1));
    for (auto& e : kr)
      if (new_event(&e)) return GM_EHIP;
    if (new_event(&kx[0]) || new_event(&kx[1])) return GM_EHIP;
  }
  // mode 4: the shards' own streams fork from st after e0 and join it
  // before e1, fork again for the backward and join before e2 (other modes:
  // every shard runs on st)
  hipEvent_t ef = nullptr;
  std::vector<hipEvent_t> ej;
  if (mode == 4) {
    if (new_event(&ef)) return GM_EHIP;
    ej.resize(ss.size());
    for (auto& e : ej)
      if (new_event(&e)) return GM_EHIP;
  }
  auto fork = [&]() -> int {
    if (mode != 4) return 0;
    HIPCHK(hipEventRecord(ef, st));
    for (gm_solver* s : ss)
      if (s->stream != st) HIPCHK(hipStreamWaitEvent(s->stream, ef, 0));
    return 0;
  };
  auto join = [&]() -> int {
    if (mode != 4) return 0;
    for (size_t g = 0; g < ss.size(); g++)
      if (ss[g]->stream != st) {
        HIPCHK(hipEventRecord(ej[g], ss[g]->stream));
        HIPCHK(hipStreamWaitEvent(st, ej[g], 0));
      }
    return 0;
  };
  // One table, whole solve: the forward -- state and count-slot resets,
  // reach map + counts -- runs on a side stream BESIDE the backward, which
  // never reads any of it (a plane's words follow from its neighbours'
  // words alone); the finish kernel waits for both.  The reach launch then
  // overlaps the first, narrow plane levels instead of preceding them.
  // A QUEUED solve (gm_solver_solve_async) runs its forward on the solve
  // stream before the backward instead: with the next solves already in the
  // queues, a side-stream forward made every queued solve 0.10-0.14 ms
  // longer on the device, whether it started with the backward (1.37-1.46
  // vs 1.27-1.31 ms per 2^30 solve) or at its narrow tail (1.40 ms);
  // profiles/r06/forward_placement_probe.txt.  (lab knob GM_PLANE_FWD:
  // 1 = always on the solve stream, 2 = always on the side stream from the
  // start, 3 = always on the side stream from the narrow tail -- the first
  // level past the widest with <= kPlaneFwdTail planes; A/B)
  static const int fwd_mode = [] {
    const char* e = lab_env("GM_PLANE_FWD");
    return e ? atoi(e) : 0;
  }();
  // one table, whole solve: the backward as ONE launch (k_plane_flow,
  // gm_plane.h) -- GM_F_PLANE_LEVELS keeps the per-level launches (A/B; lab
  // knob GM_PLANE_FLOW=0 too), and partial / resumed solves take them
  static const bool flow_knob = [] {
    const char* e = lab_env("GM_PLANE_FLOW");
    return !(e && atoi(e) == 0);
  }();
  const bool flow = mode == 0 && s0->pflow_ok && first == 0 && stop == 2 * T && flow_knob &&
                    !(s0->flags & (GM_F_PLANE_LEVELS | GM_F_PLANE_X1));
  // (the one-launch backward runs after the forward on the solve stream:
  // the forward's state reset must not race its error bit)
  const bool overlap = mode == 0 && first == 0 && stop == 2 * T && !timing && fwd_mode != 1 &&
                       (!async || fwd_mode >= 2) && !flow;
  uint32_t fwd_at = 0;  // the level whose launch the side-stream forward is enqueued after
  if (overlap && fwd_mode == 3) {
    uint32_t pk = 0;
    for (uint32_t l = 0; l <= S; l++)
      if (s0->ploff[(size_t)l + 1] - s0->ploff[l] > s0->ploff[(size_t)pk + 1] - s0->ploff[pk]) pk = l;
    fwd_at = S;
    for (uint32_t l = pk + 1; l <= S; l++)
      if (s0->ploff[(size_t)l + 1] - s0->ploff[l] <= kPlaneFwdTail) {
        fwd_at = l;
        break;
      }
  }
  hipStream_t fs = st;  // the forward's stream
  if (overlap) {
    if (!s0->cstream) {
      HIPCHK(hipStreamCreateWithFlags(&s0->cstream, hipStreamNonBlocking));
    }
    fs = s0->cstream;
  }
  // a queued one-launch solve records only its start and its completion:
  // the forward has no launch of its own and every timing marker between
  // solves is a gap on the device (the trace: ~20 us between one solve's
  // finish and the next launch); ms_forward 0, ms_backward = the whole span
  // (lab knob GM_PLANE_FLOW_LITE=0: all five events; A/B)
  static const bool lite_knob = [] {
    const char* e = lab_env("GM_PLANE_FLOW_LITE");
    return !(e && atoi(e) == 0);
  }();
  const bool lite = async && flow && lite_knob;
  if (async) s0->pring[s0->pq_next % kPlaneRing].lite = lite;
  auto t0 = std::chrono::steady_clock::now();
  HIPCHK(hipEventRecord(e0, st));
  if (fork()) return GM_EHIP;
  auto issue_forward = [&]() -> int {
    if (first == 0) {
      for (gm_solver* s : ss) {
        hipStream_t ws = overlap ? fs : s->stream;
        // (a one-launch solve after another one: that launch left the state
        // it needs clean -- error word 0, its count slots stored, not added)
        if (flow && s->pflow_last) continue;
        HIPCHK(hipMemsetAsync(s->st, 0, devstate_bytes(T), ws));
        HIPCHK(hipMemsetAsync(s->bcount, 0, kCountSlots * sizeof(BlockCount), ws));
        // the word width: written by k_plane_reach below (no reach: here)
        if (stop == 0) HIPCHK(hipMemsetD32Async((hipDeviceptr_t)&s->st->word_bits, (int)s->pmark(), 1, ws));
      }
      if (stop > 0) {
        if (timing) HIPCHK(hipEventRecord(kx[0], st));
        // (the one-launch backward writes the reach map and counts itself)
        if (!flow)
          for (gm_solver* s : ss) plane_reach_launch(s, overlap ? fs : nullptr);
        if (timing && join()) return GM_EHIP;
        if (timing) HIPCHK(hipEventRecord(kx[1], st));
      }
    }
    HIPCHK(hipGetLastError());
    if (join()) return GM_EHIP;
    if (!lite) HIPCHK(hipEventRecord(e1, fs));  // overlap: the forward's end on its own stream
    if (fork()) return GM_EHIP;
    return 0;
  };
  // overlap: the forward (resets, reach map, counts) is enqueued on its side
  // stream right after the backward's first launch (GM_PLANE_FWD=3: at its
  // narrow tail, fwd_at), so the host's first enqueue is a resolve launch
  // (the forward is read by the finish only)
  bool fwd_pending = overlap;
  if (!fwd_pending) {
    if (!lite) HIPCHK(hipEventRecord(etail, st));  // (the forward's start: ms_forward)
    const int rc = issue_forward();
    if (rc) return rc;
  }
  // kernel timing: one table -- the backward is nothing but the resolve
  // launches, so one event pair around all of them (no events between
  // launches: they would add their own gaps to what they time); shards --
  // a pair around each level's launches (exchanges sit between them)
  const bool per_level = timing && mode != 0 && !staged;
  // Shards (RCCL or in-process copies): each level's launch is split into
  // the planes that read no halo plane -- the boundary slices the exchange
  // sends are among them when blocks hold >= 4 top values -- and the ones
  // that do.  Own part -> event -> exchange on the comm stream -> event;
  // the boundary part of the NEXT level waits for it, so the exchange of
  // level l overlaps the boundary part of l and the own part of l + 1.  The
  // host-staged transport (mode 3) and blocks of < 4 values exchange in
  // order.
  bool pipe = (mode == 1 || mode == 2) && !staged;
  if (s0->pg.B < 4 || (s0->flags & GM_F_SHARD_INORDER)) pipe = false;
  hipStream_t cs = st;
  hipEvent_t* PE = nullptr;  // [0, S]: own part of level l done; [S+1, 2S+2): exchange of l done
  if (pipe) {
    if (!s0->cstream) HIPCHK(hipStreamCreateWithFlags(&s0->cstream, hipStreamNonBlocking));
    while (s0->pev.size() < 2 * ((size_t)S + 1)) {
      hipEvent_t e;
      HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      s0->pev.push_back(e);
    }
    cs = s0->cstream;
    PE = s0->pev.data();
  }
  int last_x = -1;  // last level exchanged on the comm stream
  PlaneBatcher bat0(s0);  // one table: narrow levels in one-workgroup runs
  const u64 pair_max = mode == 0 ? plane_pair_max(s0) : 0;  // and pairs of narrow levels in one launch
  static const bool pair_runs = [] {  // (lab knob GM_PLANE_PAIR_RUNS=1: pairs replace the runs; A/B)
    const char* e = lab_env("GM_PLANE_PAIR_RUNS");
    return e && atoi(e) == 1;
  }();
  u64 nlaunch = 0;        // resolve launches of this solve (shard 0's)
  s0->pflow_last = flow;
  // the one-launch solve writes its reduction words straight into pinned host
  // memory: the queued slot's, or the solver's own for a blocking solve
  u64* flow_host = nullptr;
  if (flow) {
    u64** hp = async ? &s0->pring[s0->pq_next % kPlaneRing].host : &s0->phost;
    if (!*hp) HIPCHK(hipHostMalloc((void**)hp, 8 * sizeof(u64), hipHostMallocDefault));
    flow_host = *hp;
  }
  if (flow) {
    if (timing) HIPCHK(hipEventRecord(kr[0], st));
    PlaneFlow f = s0->pflow;
    f.skip = kPlaneAbsent;
    if (const char* e = lab_env("GM_FAULT_FLOW")) f.skip = (uint32_t)atoi(e);  // (read per solve)
    f.mode = 0;
    if (const char* e = lab_env("GM_PLANE_FLOW_MODE")) f.mode = (uint32_t)atoi(e);
    f.epoch = ++s0->pflow.epoch;
    if (f.epoch == 0) {  // (2^32 solves: the flags start over)
      HIPCHK(hipMemsetAsync(f.flags, 0, (size_t)s0->pg.nplanes * 4, st));
      f.epoch = s0->pflow.epoch = 1;
    }
    plane_no_dispatch(s0->pg.no, [&](auto NO) {
      // (lab knob GM_PLANE_FLOW_PIPE=0: each visit polls before its rows;
      // the pipelined form -- the next visit's polls mid-visit, tickets two
      // ahead -- 1.017-1.021 vs 1.029-1.034 ms per step on one box,
      // profiles/r06/flow_pipe_ab.txt; A/B)
      if (const char* e = lab_env("GM_PLANE_FLOW_PIPE"); !(e && atoi(e) == 0))
        hipLaunchKernelGGL((k_plane_flow<decltype(NO)::value, true>), dim3(s0->pflow_grid), dim3(256), 0, st,
                           (uint8_t*)s0->ptab, s0->pg, s0->pzero, f, s0->pbits, s0->bcount, s0->st, s0->pmark());
      else
        hipLaunchKernelGGL((k_plane_flow<decltype(NO)::value, false>), dim3(s0->pflow_grid), dim3(256), 0, st,
                           (uint8_t*)s0->ptab, s0->pg, s0->pzero, f, s0->pbits, s0->bcount, s0->st, s0->pmark());
    });
    nlaunch = 1;
    if (timing) HIPCHK(hipEventRecord(kr[2 * (size_t)S + 1], st));
  }
  if (staged && stop == 2 * T) {
    if (timing) HIPCHK(hipEventRecord(kr[0], st));
    int rc = plane_backward_staged(ss, mode, st, &nlaunch);
    if (rc) {
      cleanup();
      return rc;
    }
    if (timing && join()) return GM_EHIP;
    if (timing) HIPCHK(hipEventRecord(kr[2 * (size_t)S + 1], st));
  }
  for (uint32_t l = 0; l <= S && !staged && !flow; l++) {
    const int k = T + (int)l;
    if (k < first) continue;
    if (k >= stop) break;
    if (per_level || (timing && l == 0)) HIPCHK(hipEventRecord(kr[2 * l], st));
    if (mode == 0 && !per_level) {
      const u64 n0 = s0->ploff[(size_t)l + 1] - s0->ploff[l];
      const u64 n1 = l < S ? s0->ploff[(size_t)l + 2] - s0->ploff[(size_t)l + 1] : 0;
      const u64 pmin = pair_runs ? 1 : bat0.narrow + 1;  // (pairs of run-narrow levels too: A/B)
      if (l < S && k + 1 < stop && n0 >= pmin && n1 >= pmin && n0 <= pair_max && n1 <= pair_max) {
        bat0.flush();  // levels l and l + 1 in one launch (k_plane_pair)
        plane_pair_launch(s0, l);
        bat0.launches++;
        l++;
      } else {
        bat0.add(s0->ploff[l], s0->ploff[(size_t)l + 1], l, n1);
      }
      if (l == S) bat0.flush();
      if (fwd_pending && bat0.launches > 0 && l >= fwd_at) {
        fwd_pending = false;
        bat0.flush();  // the side stream starts behind this level's launch
        HIPCHK(hipEventRecord(etail, st));
        HIPCHK(hipStreamWaitEvent(fs, etail, 0));
        const int rc = issue_forward();
        if (rc) return rc;
      }
    } else if (!pipe) {
      for (gm_solver* s : ss) plane_launch(s, l);
    } else {
      for (gm_solver* s : ss) plane_launch(s, l, 1);
      HIPCHK(hipEventRecord(PE[l], st));
      HIPCHK(hipStreamWaitEvent(cs, PE[l], 0));
    }
    if (mode != 0) {
      int rc = plane_exchange(ss, l, mode, cs);
      if (rc) {
        cleanup();
        return rc;
      }
    }
    if (pipe) {
      HIPCHK(hipEventRecord(PE[S + 1 + l], cs));
      last_x = (int)l;
      // the boundary planes read the halos of levels l - 1 and l - 2
      if (l >= 1) HIPCHK(hipStreamWaitEvent(st, PE[S + l], 0));
      for (gm_solver* s : ss) plane_launch(s, l, 2);
    }
    if (per_level || (timing && l == S)) HIPCHK(hipEventRecord(kr[2 * l + 1], st));
  }
  bat0.flush();  // a stop inside a run
  if (fwd_pending) {  // (not reached in the loop)
    fwd_pending = false;
    HIPCHK(hipEventRecord(etail, st));
    HIPCHK(hipStreamWaitEvent(fs, etail, 0));
    const int rc = issue_forward();
    if (rc) return rc;
  }
  if (!staged && !flow) nlaunch = mode == 0 && !per_level ? bat0.launches : (u64)(S + 1) * (pipe ? 2 : 1);
  if (last_x >= 0) HIPCHK(hipStreamWaitEvent(st, PE[S + 1 + last_x], 0));  // join the comm stream
  {
    const hipError_t e = hipGetLastError();  // (a failed launch of the backward)
    if (e != hipSuccess) {
      if (!staged || mode == 2) return fail(GM_EHIP, "plane backward: %s", hipGetErrorString(e));
      // staged shards: deferred, so the end-of-solve reduction is still entered
      if (!s0->defer_rc) staged_defer(s0, fail(GM_EHIP, "plane backward: %s", hipGetErrorString(e)), st);
    }
  }
  if (join()) return GM_EHIP;
  if (!lite) HIPCHK(hipEventRecord(e2, st));
  if (overlap) HIPCHK(hipStreamWaitEvent(st, e1, 0));  // the counts and state resets before the finish
  if (stop < 2 * T) {
    HIPCHK(hipStreamSynchronize(st));
    cleanup();
    out->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    out->word_bits = 8 * s0->pwb;
    return GM_PARTIAL;
  }
  for (gm_solver* s : ss)
    plane_form_dispatch(s, [&](auto WB, auto) {
      if (flow)  // (the one-launch solve: its own count slots, the result straight to pinned memory)
        hipLaunchKernelGGL((k_plane_finish<decltype(WB)::value, true>), dim3(1), dim3(1024), 0, st, s->d, s->pg,
                           (const void*)s->ptab, s->pbits, s->st, (const BlockCount*)s->bcount, s->pflow_grid,
                           flow_host);
      else
        hipLaunchKernelGGL((k_plane_finish<decltype(WB)::value, false>), dim3(1), dim3(1024), 0, st, s->d, s->pg,
                           (const void*)s->ptab, s->pbits, s->st, (const BlockCount*)s->bcount, 0u, (u64*)nullptr);
    });
  HIPCHK(hipGetLastError());
  if (async) {  // queued: the counts into the slot's pinned memory, then its completion event
    PlaneSlot& q = s0->pring[s0->pq_next % kPlaneRing];
    if (!q.host) HIPCHK(hipHostMalloc((void**)&q.host, 8 * sizeof(u64), hipHostMallocDefault));
    if (!q.ev[3]) HIPCHK(hipEventCreate(&q.ev[3]));
    if (!flow) HIPCHK(hipMemcpyAsync(q.host, s0->st->red, 5 * sizeof(u64), hipMemcpyDeviceToHost, st));
    HIPCHK(hipEventRecord(q.ev[3], st));
    s0->pq_next++;
    cleanup();
    return 0;
  }
  if (mode == 1) {
    RCCL_LIVE(s0);
    ncclGroupStart();
    ncclResult_t r = ncclAllReduce(s0->st->red, s0->st->red, 4, ncclUint64, ncclSum, s0->comm, st);
    ncclResult_t r2 = ncclAllGather(s0->st->red + 4, s0->errg, 1, ncclUint64, s0->comm, st);
    ncclResult_t r3 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess || r3 != ncclSuccess)
      return fail(GM_EHIP, "RCCL allreduce: %s", ncclGetErrorString(r != ncclSuccess ? r : r2 != ncclSuccess ? r2 : r3));
  }
  u64 red[5] = {0, 0, 0, 0, 0};
  for (gm_solver* s : ss) {
    u64 r[5];
    // (into pinned host memory: a pageable destination is staged and waited
    // for inside the copy call)
    if (!s->phost) HIPCHK(hipHostMalloc((void**)&s->phost, 8 * sizeof(u64), hipHostMallocDefault));
    if (!flow) HIPCHK(hipMemcpyAsync(s->phost, s->st->red, sizeof r, hipMemcpyDeviceToHost, st));
    HIPCHK(mode == 0 ? plane_wait(st) : hipStreamSynchronize(st));
    memcpy(r, s->phost, sizeof r);
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
  HIPCHK(hipEventElapsedTime(&f, etail, e1));  // the forward's own span (it starts at etail)
  HIPCHK(hipEventElapsedTime(&b, overlap ? e0 : e1, e2));  // overlap: the backward starts at e0
  out->ms_forward = f;
  out->ms_backward = b;
  out->ms_total = std::chrono::duration<double, std::milli>(t1 - t0).count();
  if (timing) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, kx[0], kx[1]));
    out->ms_expand_kernels = ms;
    out->n_expand_launches = 1;
    double sr = 0;
    if (per_level) {
      for (uint32_t l = 0; l <= S; l++) {
        HIPCHK(hipEventElapsedTime(&ms, kr[2 * l], kr[2 * l + 1]));
        sr += ms;
      }
    } else {
      HIPCHK(hipEventElapsedTime(&ms, kr[0], kr[2 * (size_t)S + 1]));
      sr = ms;
    }
    out->ms_resolve_kernels = sr;
    out->n_resolve_launches = nlaunch;
  }
  cleanup();
  return plane_result(ss, red, out);
}

// A queued solve's result (gm_solver_collect): wait for its completion
// event (bounded spin, then a blocking wait), read its counts from the slot
static int plane_collect(gm_solver* s, u64 ticket, gm_result* out) {
  if (ticket < s->pq_done || ticket >= s->pq_next)
    return fail(GM_EINVAL, "ticket %llu: queued solves %llu..%llu are outstanding", (unsigned long long)ticket,
                (unsigned long long)s->pq_done, (unsigned long long)s->pq_next);
  if (ticket != s->pq_done) return fail(GM_EINVAL, "collect queued solves in order (next: %llu)", (unsigned long long)s->pq_done);
  PlaneSlot& q = s->pring[ticket % kPlaneRing];
  const auto t0 = std::chrono::steady_clock::now();
  hipError_t e;
  while ((e = hipEventQuery(q.ev[3])) == hipErrorNotReady) {
    if (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() > kPlaneSpinUs) {
      e = hipEventSynchronize(q.ev[3]);
      break;
    }
    __builtin_ia32_pause();
  }
  s->pq_done++;
  if (e != hipSuccess) return fail(GM_EHIP, "queued solve %llu: %s", (unsigned long long)ticket, hipGetErrorString(e));
  u64 red[5];
  memcpy(red, q.host, sizeof red);
  float f = 0, b = 0, t = 0;
  HIPCHK(hipEventElapsedTime(&t, q.ev[0], q.ev[3]));
  if (q.lite) {  // (a one-launch solve: start and completion only)
    b = t;
  } else {
    HIPCHK(hipEventElapsedTime(&f, q.ev[4], q.ev[1]));
    HIPCHK(hipEventElapsedTime(&b, q.ev[0], q.ev[2]));
  }
  out->ms_forward = f;
  out->ms_backward = b;
  out->ms_total = t;  // device span of the queued solve (its host wall overlaps other solves)
  out->ms_expand_kernels = out->ms_resolve_kernels = 0;
  out->n_expand_launches = out->n_resolve_launches = 0;
  return plane_result({s}, red, out);
}

static int plane_query(gm_solver* s, const uint64_t* keys_dev, uint64_t n, uint32_t* words_dev) {
  const int grid = (int)std::min<u64>((n + kBlock - 1) / kBlock, (u64)s->grid);
  plane_form_dispatch(s, [&](auto WB, auto) {
    hipLaunchKernelGGL(k_plane_query<decltype(WB)::value>, dim3(grid), dim3(kBlock), 0, s->stream, s->d, s->pg,
                       (const void*)s->ptab, s->pbits, (const u64*)keys_dev, n, words_dev);
  });
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s->stream));
  return 0;
}

static int plane_positions(gm_solver* s, uint64_t* keys_dev, uint64_t cap, uint64_t* n) {
  u64 cnt = 0;
  HIPCHK(hipStreamSynchronize(s->stream));
  HIPCHK(hipMemcpy(&cnt, &s->st->cursor_front, sizeof cnt, hipMemcpyDeviceToHost));
  *n = cnt;
  if (cnt > cap || !keys_dev) return cap < cnt ? fail(GM_EFULL, "need %llu slots", (unsigned long long)cnt) : 0;
  HIPCHK(hipMemsetAsync(&s->st->cursor_back, 0, sizeof(u64), s->stream));
  plane_no_dispatch(s->pg.no, [&](auto NO) {
    hipLaunchKernelGGL((k_plane_positions<decltype(NO)::value>), dim3(s->grid), dim3(kBlock), 0, s->stream, s->d,
                       s->pg, (const uint32_t*)s->pbits, (u64*)keys_dev, cap, &s->st->cursor_back);
  });
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s->stream));
  return 0;
}

static void plane_checksum_launch(gm_solver* s, u64* acc) {
  plane_no_dispatch(s->pg.no, [&](auto NO) {
    plane_form_dispatch(s, [&](auto WB, auto) {
      hipLaunchKernelGGL((k_plane_checksum<decltype(NO)::value, decltype(WB)::value>), dim3(s->grid), dim3(kBlock), 0,
                         s->stream, s->d, s->pg, (const void*)s->ptab, (const uint32_t*)s->pbits, acc);
    });
  });
}

}  // extern "C++"
