// gm_keyed_shard.h -- per-level building blocks of the md5-sharded solve of
// keyed (HASHED) tables.  Included by gm_solver.hip after the shared device
// helpers and the single-table kernels.
//
// Ownership is the reference's own rule, owner(pos) = md5(str(pos)) % P
// (GameState.get_hash, src/game_state.py:22-30).  Each rank's table holds
// the positions it owns; the host moves keys and words between ranks with
// all-to-all(v) (gamesmanmpi_amd/keyed.py).  Per level L:
//   forward   k_ks_expand   own level-L positions -> (child key, owner) pairs
//             [exchange keys to their owners]
//             k_ks_insert   owner: CAS-insert, new keys appended to level
//                           L+1 / L+2 of ITS store (level from the descriptor)
//             k_finalize    level bookkeeping (shared with the 1-GPU path)
//   backward  k_ks_counts   children per own level-L position
//             [host: exclusive scan -> offsets]
//             k_ks_children children in gen_moves order at offsets, + owners
//             [exchange queries; owners k_query their words; reply]
//             k_ks_reduce   canonical reduction of each
//                           position's contiguous child words, own word stored
// This replaces the per-edge LOOK_UP / RESOLVE message pairs of
// src/process.py:146-185 by two bulk exchanges per level.

__device__ __forceinline__ uint32_t owner_of(const Desc& d, u64 key, uint32_t P) {
  if (P <= 1) return 0;
  uint8_t s[56], dig[16];
  const int len = str_utf8_from_key(d, key, s);
  md5_block(s, len, dig);
  return md5_mod(dig, P);
}

// the same as a call: the bucketed kernels ask for owners inside the
// unrolled move generators, where an inlined MD5 per move site multiplies the
// code (and the compile time) by the number of sites
__device__ __noinline__ uint32_t owner_of_call(const Desc& d, u64 key, uint32_t P) { return owner_of(d, key, P); }

// rank owning the root seeds its table and level 0; every rank zeroes state
__global__ void k_ks_seed(gm_slot* tab, u64 mask, u64* lv, DevState* st, u64 root, int owned) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (owned) {
      table_insert(tab, mask, root, &st->err);
      lv[0] = root;
    }
    st->cursor_front = owned ? 1 : 0;
    st->cursor_back = 0;
    st->seg[0].fb = 0;
    st->seg[0].fe = owned ? 1 : 0;
    st->seg[0].c2lo = 0;
    st->seg[0].c2hi = 0;
    st->seg[1].c2lo = 0;
    st->seg[1].c2hi = 0;
  }
}

// children of the own level-L positions (LDS-staged appends at `cursor`);
// owners are filled afterwards by k_owner over the emitted keys
template <int KIND>
__global__ __launch_bounds__(256) void k_ks_expand(Desc d, const u64* lv, u64 lcap, DevState* st, int L,
                                                   u64* keys_out, u64 cap, u64* cursor) {
  __shared__ StageLDS stage;
  stage_init(stage);
  const LevelSeg s = st->seg[L];
  const u64 n = (s.fe - s.fb) + (s.c2hi - s.c2lo);
  const u64 stride = (u64)gridDim.x * blockDim.x;
  auto store = [&](int, u64 g, u64 key) {
    if (g < cap) keys_out[g] = key;
  };
  for (u64 base = (u64)blockIdx.x * blockDim.x; base < n; base += stride) {  // block-uniform
    const u64 i = base + threadIdx.x;
    if (i < n) {
      const u64 key = level_key(lv, lcap, s, i);
      if (Game<KIND>::prim(d, key) == UNDECIDED)
        Game<KIND>::children(d, key, [&](u64 child, int) {
          if (!stage_push(stage, 0, child)) store(0, atomicAdd(cursor, 1ull), child);
        });
    }
    if (stage_should_flush(stage)) stage_flush(stage, cursor, cursor, store);
  }
  stage_flush(stage, cursor, cursor, store);
}

// insert received keys (all owned by this rank); new ones join the level
// store at their own level, which must be L+1 or L+2
template <int KIND>
__global__ __launch_bounds__(256) void k_ks_insert(Desc d, gm_slot* tab, u64 mask, u64* lv, u64 lcap, DevState* st,
                                                   int L, const u64* keys, u64 n) {
  __shared__ StageLDS stage;
  stage_init(stage);
  uint32_t err = 0;
  const u64 stride = (u64)gridDim.x * blockDim.x;
  auto store = [&](int q, u64 g, u64 key) { level_store(lv, lcap, q, g, key); };
  for (u64 base = (u64)blockIdx.x * blockDim.x; base < n; base += stride) {  // block-uniform
    const u64 i = base + threadIdx.x;
    if (i < n) {
      const u64 key = keys[i];
      if (table_insert(tab, mask, key, &st->err)) {
        const int step = Game<KIND>::level(d, key) - L;
        if (step == 1 || step == 2) {
          const int q = step - 1;
          if (!stage_push(stage, q, key))
            store(q, atomicAdd(q ? &st->cursor_back : &st->cursor_front, 1ull), key);
        } else {
          err |= ERR_BAD_STEP;
        }
      }
    }
    if (stage_should_flush(stage)) stage_flush(stage, &st->cursor_front, &st->cursor_back, store);
  }
  stage_flush(stage, &st->cursor_front, &st->cursor_back, store);
  if (err) atomicOr(&st->err, err);
}

template <int KIND>
__global__ __launch_bounds__(256) void k_ks_counts(Desc d, const u64* lv, u64 lcap, DevState* st, int L,
                                                   uint64_t* counts) {
  const LevelSeg s = st->seg[L];
  const u64 n = (s.fe - s.fb) + (s.c2hi - s.c2lo);
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
    const u64 key = level_key(lv, lcap, s, i);
    counts[i] = Game<KIND>::prim(d, key) != UNDECIDED ? 0 : (u64)Game<KIND>::children(d, key, [](u64, int) {});
  }
}

template <int KIND>
__global__ __launch_bounds__(256) void k_ks_children(Desc d, const u64* lv, u64 lcap, DevState* st, int L,
                                                     const uint64_t* offsets, u64* keys_out, uint32_t* owners_out,
                                                     uint32_t P) {
  const LevelSeg s = st->seg[L];
  const u64 n = (s.fe - s.fb) + (s.c2hi - s.c2lo);
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
    const u64 key = level_key(lv, lcap, s, i);
    if (Game<KIND>::prim(d, key) != UNDECIDED) continue;
    u64 j = offsets[i];
    Game<KIND>::children(d, key, [&](u64 child, int) {
      keys_out[j] = child;
      owners_out[j] = owner_of(d, child, P);
      j++;
    });
  }
}

// offsets: n + 1 entries (exclusive scan of k_ks_counts, last = total)
template <int KIND>
__global__ __launch_bounds__(256) void k_ks_reduce(Desc d, gm_slot* tab, u64 mask, const u64* lv, u64 lcap,
                                                   DevState* st, int L, const uint64_t* offsets,
                                                   const uint32_t* child_words) {
  const LevelSeg s = st->seg[L];
  const u64 n = (s.fe - s.fb) + (s.c2hi - s.c2lo);
  u64 edges = 0, prims = 0;
  uint32_t err = 0;
  for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
    const u64 key = level_key(lv, lcap, s, i);
    const int p = Game<KIND>::prim(d, key);
    uint32_t word;
    if (p != UNDECIDED) {
      word = make_word(p, 0);  // process.py:120-123
      prims++;
    } else {
      bool any_loss = false, any_tie = false, any_draw = false;
      uint32_t min_loss = 0xFFFFFFFFu, max_all = 0;
      const u64 a = offsets[i], b = offsets[i + 1];
      if (a == b) err |= ERR_NO_MOVES;
      for (u64 j = a; j < b; j++) {
        const uint32_t w = child_words[j];
        if (w == NO_WORD) { err |= ERR_CHILD_MISSING; continue; }
        const uint32_t v = w & 3u, r = w >> 2;
        if (v == LOSS) { any_loss = true; min_loss = min(min_loss, r); }
        any_tie |= (v == TIE);
        any_draw |= (v == DRAW);
        max_all = max(max_all, r);
      }
      edges += b - a;
      // reference-canonical _res_red / _remote_red
      if (any_loss) word = make_word(WIN, min_loss + 1);
      else word = make_word(any_tie ? TIE : any_draw ? DRAW : LOSS, max_all + 1);
    }
    const u64 h = table_find(tab, mask, key);
    if (h == ~0ull) err |= ERR_SELF_MISSING;
    else tab[h].word = word;
  }
  if (err) atomicOr(&st->err, err);
  block_add(&st->edges, edges);
  block_add(&st->prims, prims);
}
