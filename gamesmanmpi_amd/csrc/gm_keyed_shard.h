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

// ---- register-resident owners (device) ----------------------------------
// owner_of renders str(pos) into a byte array and runs the generic MD5 over
// it; on the GPU both arrays are indexed by data-dependent positions and live
// in scratch memory, ~1.5 ns of the whole chip per owner (the md5-sharded
// bucketed forward spent 97 % of its time there).  For the kinds the bucketed
// shards serve (tic-tac-toe, mttt, toot-and-otto, othello) the message is
// built straight into the 16 MD5 words -- static byte positions, or for the
// UTF-8 expansion of the bitstring bytes a select over the few words a byte
// can land in -- and the 64 rounds are unrolled (K, shifts and message
// indices become constants).  Bit-exact with owner_of: tests check both
// against the owners the reference's own GameState.get_hash produced.
__device__ __forceinline__ void md5_put_byte(uint32_t* M, uint32_t n, uint32_t b, int wlo, int whi) {
#pragma unroll
  for (int w = 0; w < 16; w++)
    if (w >= wlo && w <= whi) M[w] |= (n >> 2) == (uint32_t)w ? b << (8 * (n & 3)) : 0u;
}
__device__ __forceinline__ uint32_t md5_mod_words(const uint32_t M[16], uint32_t P) {
  constexpr uint32_t K[64] = {
      0xd76aa478u, 0xe8c7b756u, 0x242070dbu, 0xc1bdceeeu, 0xf57c0fafu, 0x4787c62au, 0xa8304613u, 0xfd469501u,
      0x698098d8u, 0x8b44f7afu, 0xffff5bb1u, 0x895cd7beu, 0x6b901122u, 0xfd987193u, 0xa679438eu, 0x49b40821u,
      0xf61e2562u, 0xc040b340u, 0x265e5a51u, 0xe9b6c7aau, 0xd62f105du, 0x02441453u, 0xd8a1e681u, 0xe7d3fbc8u,
      0x21e1cde6u, 0xc33707d6u, 0xf4d50d87u, 0x455a14edu, 0xa9e3e905u, 0xfcefa3f8u, 0x676f02d9u, 0x8d2a4c8au,
      0xfffa3942u, 0x8771f681u, 0x6d9d6122u, 0xfde5380cu, 0xa4beea44u, 0x4bdecfa9u, 0xf6bb4b60u, 0xbebfbc70u,
      0x289b7ec6u, 0xeaa127fau, 0xd4ef3085u, 0x04881d05u, 0xd9d4d039u, 0xe6db99e5u, 0x1fa27cf8u, 0xc4ac5665u,
      0xf4292244u, 0x432aff97u, 0xab9423a7u, 0xfc93a039u, 0x655b59c3u, 0x8f0ccc92u, 0xffeff47du, 0x85845dd1u,
      0x6fa87e4fu, 0xfe2ce6e0u, 0xa3014314u, 0x4e0811a1u, 0xf7537e82u, 0xbd3af235u, 0x2ad7d2bbu, 0xeb86d391u};
  constexpr int R[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};
  uint32_t a = 0x67452301u, b = 0xefcdab89u, c = 0x98badcfeu, e = 0x10325476u;
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t f;
    int g;
    if (i < 16) { f = (b & c) | (~b & e); g = i; }
    else if (i < 32) { f = (e & b) | (~e & c); g = (5 * i + 1) & 15; }
    else if (i < 48) { f = b ^ c ^ e; g = (3 * i + 5) & 15; }
    else { f = c ^ (b | ~e); g = (7 * i) & 15; }
    f = f + a + K[i] + M[g];
    a = e; e = c; c = b;
    b = b + __builtin_amdgcn_alignbit(f, f, 32 - R[(i >> 4) * 4 + (i & 3)]);
  }
  const uint32_t h[4] = {a + 0x67452301u, b + 0xefcdab89u, c + 0x98badcfeu, e + 0x10325476u};
  // int(hexdigest, 16) % P: the 16 digest bytes as a big-endian integer.  A
  // power-of-two P (every bench world) keeps the low bits of the last byte;
  // otherwise Horner over the bytes (< P <= 2^23: acc << 8 | byte fits 32
  // bits), sixteen dependent 32-bit remainders
  if ((P & (P - 1)) == 0 && P <= 256u) return (h[3] >> 24) & (P - 1u);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) acc = ((acc << 8) | ((h[i >> 2] >> (8 * (i & 3))) & 0xFFu)) % P;
  return acc;
}
// (the descriptor fields the rule reads, as values: a call passes them in
// registers instead of materialising the whole Desc in scratch)
struct OwnerGeom {
  int kind, variant, A, nbits;
};
__device__ __forceinline__ uint32_t owner_fast_g(const OwnerGeom d, u64 k, uint32_t P);
__device__ __forceinline__ uint32_t owner_fast(const Desc& d, u64 k, uint32_t P) {
  return owner_fast_g(OwnerGeom{d.kind, d.variant, d.A, d.nbits}, k, P);
}
__device__ __forceinline__ uint32_t owner_fast_g(const OwnerGeom d, u64 k, uint32_t P) {
  if (P <= 1) return 0;
  uint32_t M[16];
#pragma unroll
  for (int w = 0; w < 16; w++) M[w] = 0;
  uint32_t len;
  if (d.kind == K_TTT && d.variant == 0) {  // numpy str() of a 3x3 int8 array: "[[a b c]\n [d e f]\n [g h i]]"
    const char* t = "[[0 0 0]\n [0 0 0]\n [0 0 0]]";
#pragma unroll
    for (int i = 0; i < 27; i++) {
      uint32_t ch = (uint8_t)t[i];
      const int r = i / 9, q = i % 9;
      if (q == 2 || q == 4 || q == 6) ch += (uint32_t)((k >> (2 * (3 * r + (q - 2) / 2))) & 3);
      M[i >> 2] |= ch << (8 * (i & 3));
    }
    len = 27;
  } else if (d.kind == K_TTT) {  // mttt: the 9-character string
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const uint32_t v = (uint32_t)((k >> (2 * i)) & 3);
      M[i >> 2] |= (v == 0 ? (uint32_t)'_' : v == 1 ? (uint32_t)'X' : (uint32_t)'O') << (8 * (i & 3));
    }
    len = 9;
  } else {  // toot / othello: the MSB-first bitstring bytes (bits_from_key), latin-1 -> UTF-8
    const int A = d.A, nb = d.nbits / 8;  // wave-uniform; 2A <= 48 and nb <= 16 for every served board
    // string bit i <-> bit 127 - i of hi:lo
    u64 hi = 0, lo = 0;
    const u64 cells = k & ((1ull << (2 * A)) - 1);
    hi = __builtin_bitreverse64(cells);  // bits 0..2A-1 of the string
    auto put = [&](int at, int w, uint32_t v) {  // field v of w bits at string bit at
      const int sh = 128 - at - w;  // its lowest bit's position in hi:lo
      const u64 x = (u64)v;
      if (sh >= 64) hi |= x << (sh - 64);
      else if (sh + w <= 64) lo |= x << sh;
      else {
        lo |= x << sh;
        hi |= x >> (64 - sh);
      }
    };
    if (d.kind == K_TOOT) {
#pragma unroll
      for (int j = 0; j < 4; j++) put(2 * A + 4 * j, 4, (uint32_t)((k >> (2 * A + 3 * j)) & 7));
      put(2 * A + 16, 1, 1u);
      put(d.nbits - 1, 1, (uint32_t)((k >> (2 * A + 12)) & 1));
    } else {
      put(2 * A, 8, ((k >> (2 * A)) & 1) ? 1u : 2u);
      put(2 * A + 8, 8, (uint32_t)((k >> (2 * A + 1)) & 3));
    }
    uint32_t n = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) {
      if (j >= nb) break;  // wave-uniform
      const uint32_t b = (uint32_t)((j < 8 ? hi >> (56 - 8 * j) : lo >> (120 - 8 * j)) & 0xFFu);
      if (b < 0x80u) {
        md5_put_byte(M, n, b, j >> 2, (2 * j) >> 2);
        n += 1;
      } else {
        md5_put_byte(M, n, 0xC0u | (b >> 6), j >> 2, (2 * j) >> 2);
        md5_put_byte(M, n + 1, 0x80u | (b & 0x3Fu), (j + 1) >> 2, (2 * j + 1) >> 2);
        n += 2;
      }
    }
    len = n;
    md5_put_byte(M, len, 0x80u, nb >> 2, (2 * nb) >> 2);
    M[14] = len * 8u;
    return md5_mod_words(M, P);
  }
  M[len >> 2] |= 0x80u << (8 * (len & 3));
  M[14] = len * 8u;
  return md5_mod_words(M, P);
}
// the owner rule on the device: the register-resident form where it applies
__device__ __forceinline__ uint32_t owner_dev(const Desc& d, u64 key, uint32_t P) {
  if (d.kind == K_TTT || d.kind == K_TOOT || d.kind == K_OTHELLO) return owner_fast(d, key, P);
  return owner_of(d, key, P);
}

// the owner rule for a kernel specialised to game kind KIND: the kinds the
// bucketed shards serve get the register-resident MD5 with no runtime branch
// to owner_of, whose byte arrays live in scratch (inlined beside the fast
// form they cost the sharded expand 672 B of scratch per lane and half its
// occupancy)
template <int KIND>
__device__ __forceinline__ uint32_t owner_k(const Desc& d, u64 key, uint32_t P) {
  if constexpr (KIND == K_TTT || KIND == K_TOOT || KIND == K_OTHELLO || KIND == K_TOOT_6x4 || KIND == K_TOOT_5x4 ||
                KIND == K_TOOT_4x4)
    return owner_fast(d, key, P);
  else
    return owner_dev(d, key, P);
}

// the same as a call: the bucketed kernels ask for owners inside the
// unrolled move generators, where an inlined MD5 per move site multiplies the
// code (and the compile time) by the number of sites
__device__ __noinline__ uint32_t owner_of_call(const Desc& d, u64 key, uint32_t P) { return owner_dev(d, key, P); }
__device__ __noinline__ uint32_t owner_fast_call(const OwnerGeom d, u64 key, uint32_t P) { return owner_fast_g(d, key, P); }
// as a call, for a kernel specialised to KIND (no scratch-array path for the fast kinds)
template <int KIND>
__device__ __forceinline__ uint32_t owner_call_k(const Desc& d, u64 key, uint32_t P) {
  if constexpr (KIND == K_TTT || KIND == K_TOOT || KIND == K_OTHELLO || KIND == K_TOOT_6x4 || KIND == K_TOOT_5x4 ||
                KIND == K_TOOT_4x4)
    return owner_fast_call(OwnerGeom{d.kind, d.variant, d.A, d.nbits}, key, P);
  else
    return owner_of_call(d, key, P);
}

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
      owners_out[j] = owner_dev(d, child, P);
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
