/*
 * gamesman.h -- C-ABI of the MI355X-native GamesmanMPI solver
 * (libgamesman_hip.so, built from gamesmanmpi_amd/csrc/).
 *
 * The reference's hot path is the solve of a game module behind the
 * game-module API (initial_position / gen_moves / do_move / primitive,
 * README.md:28-88, called only through src/game_state.py:14,37-40,65,84).
 * Each entry point below replaces one piece of that path; the reference
 * interface it stands in for is cited beside it.  The Python host
 * (gamesmanmpi_amd/) binds these with ctypes.
 *
 * Conventions: plain pointers and sizes, no torch/HIP types.  Every call
 * returns 0 on success and a negative GM_E* code on failure; gm_last_error()
 * gives the thread's last message.  No exception crosses the ABI.  The
 * library never frees caller memory.  Device buffers are allocated by the
 * caller (PyTorch-ROCm in the shipped host) and passed as addresses.
 */
#ifndef GAMESMAN_H
#define GAMESMAN_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* value codes, identical to src/utils.py:3 */
#define GM_WIN 0
#define GM_LOSS 1
#define GM_TIE 2
#define GM_DRAW 3
#define GM_UNDECIDED 4

/* one resolved position = 32-bit word: value in bits [0,2), remoteness in
 * bits [2,32); GM_NO_WORD = unknown/unresolved */
#define GM_NO_WORD 0xFFFFFFFFu
#define GM_EMPTY_KEY 0xFFFFFFFFFFFFFFFFull

#define GM_EINVAL (-1)    /* bad argument / unknown game / bad canonical bytes */
#define GM_EHIP (-2)      /* HIP runtime error */
#define GM_EFULL (-3)     /* table or level storage too small: re-plan larger */
#define GM_ECORRUPT (-4)  /* internal consistency check failed (bug) */
#define GM_ENOGPU (-5)    /* no usable gfx950 device */
#define GM_ELIMIT (-6)    /* a layout limit more memory cannot lift (a BUCKETED
                             hash bucket over capacity, a level wider than
                             the layout supports): re-planning larger does
                             not help, use another layout */
#define GM_PARTIAL 1      /* gm_solver_solve stopped at the step set by gm_solver_set_steps (not an error) */

/* layout of one hash-table slot (16 B): key, word, spare */
typedef struct gm_slot {
  uint64_t key;
  uint32_t word;
  uint32_t spare;
} gm_slot;

/* Table layouts.  HASHED: open-addressing gm_slot table + per-level key
 * store (any descriptor).  DENSE: level-major perfect-hash array of 32-bit
 * words, slot = level * W + prefix (rank-indexable descriptors only:
 * four_to_one, sum_four_to_one). */
#define GM_MODE_HASHED 0u
#define GM_MODE_DENSE 1u
/* BUCKETED (keyed games whose every move advances one level: tic-tac-toe,
 * toot-and-otto, othello; one GPU): no hash table.  Each level's unique keys
 * grouped by hash bucket in the levels buffer (level_capacity keys), 32-bit
 * words + the level's in-edges + partition scratch in the table buffer
 * (table_slots = edge capacity); dedup and lookups happen in LDS
 * (gamesmanmpi_amd/csrc/gm_bucketed.h). */
#define GM_MODE_BUCKETED 2u
/* PLANES (sum_four_to_one with heaps 0 and 1 of 32 values; the default for
 * those): no levels at all in the layout -- every position's 8- or 16-bit
 * order-form word in natural rank order, planes of 32 x 32 positions (heaps
 * 0 and 1) with each row rotated by its row number, plus a 1-bit reach map;
 * table_slots = positions.  The backward pass runs once per sum of the outer
 * heaps (gamesmanmpi_amd/csrc/gm_plane.h).  Shards own blocks of the last
 * heap's values -- one block per rank, resolved as a pipeline with the
 * boundary slices streamed to the next rank row by row (the staged deal), or
 * round-robin blocks with one exchange per plane level (GM_F_PLANE_LEVEL_SYNC
 * or uneven splits); their table buffer also holds the halo send / receive
 * areas. */
#define GM_MODE_PLANES 3u
/* RANKED (toot_and_otto_bitstring; the default for it on one GPU): no keys
 * and no dedup -- every position at a computed index.  A position is its
 * column stacks (heights and letters: gravity boards) plus the first
 * player's T count; the level's height vectors are blocks of 8 x 2^L slots
 * [T count][stack bits], levels one after another.  One byte of word per
 * slot (value | remoteness << 2) + a reach and an expandable bit; a move is
 * index arithmetic (gamesmanmpi_amd/csrc/gm_ranked.h).  table_slots = slots;
 * the levels buffer is unused.  GM_F_FORCE_HASHED / GM_F_HASH_TABLE keep
 * the keyed layouts. */
#define GM_MODE_RANKED 4u

/* Sizes the caller must allocate for a solve (see gm_plan). */
typedef struct gm_plan_t {
  uint64_t table_bytes;      /* bytes of the table buffer */
  uint64_t table_slots;      /* HASHED: gm_slot entries (power of two);
                                DENSE: table words (levels * W): 16-bit for
                                one-GPU tables the octet kernels solve, else
                                32-bit (table_bytes holds the choice) */
  uint64_t level_capacity;   /* HASHED: uint64 keys in the per-level store */
  uint64_t scratch_bytes;    /* device scratch (counters, level table) */
  uint32_t max_levels;       /* tiers the pipeline provisions */
  uint32_t mode;             /* GM_MODE_* chosen */
} gm_plan_t;

/* Device buffers (addresses in the current HIP device's memory). */
typedef struct gm_buffers {
  void *table;               /* plan.table_bytes */
  uint64_t table_slots;      /* plan.table_slots */
  void *levels;              /* uint64_t[level_capacity] (HASHED only) */
  uint64_t level_capacity;
  void *scratch;             /* scratch_bytes */
  uint64_t scratch_bytes;
  void *stream;              /* hipStream_t to run on (NULL: library's own) */
  uint32_t flags;            /* GM_F*: the same flags gm_plan was given */
  uint32_t mode;             /* GM_MODE_* from gm_plan */
  uint64_t table_bytes;      /* bytes of the table buffer (>= plan.table_bytes) */
} gm_buffers;

#define GM_F_KERNEL_TIMING 1u  /* time every kernel with HIP events (the only
                                  flag gm_solver_set_flags may change) */
#define GM_F_FORCE_HASHED 2u   /* gm_plan: keyed table even when DENSE fits */
/* Kernel-family flags (A/B runs).  They are given to gm_plan (they decide
 * the dense word width, hence the table size) AND in gm_buffers.flags to
 * gm_solver_create*, which fixes the kernels for the solver's lifetime and
 * refuses a table sized for other flags with GM_EINVAL. */
#define GM_F_WORDS32 4u        /* dense: 32-bit table words (quad kernels) */
#define GM_F_RESOLVE_SCALAR 8u /* dense: one-prefix-per-lane resolve, 32-bit */
#define GM_F_SHARD_INORDER 16u /* dense / planes shards: exchange each level's
                                  halo in order instead of overlapping it */
#define GM_F_HASH_TABLE 32u    /* gm_plan, keyed games: the open-addressing
                                  hash table (HASHED) instead of BUCKETED */
#define GM_F_WORDS16 64u       /* dense: 16-bit table words (octet kernels)
                                  where 8-bit ones would be chosen */
#define GM_F_BK_EXACT 128u     /* BUCKETED: count every level's children first
                                  (exact partition offsets) instead of writing
                                  into provisioned partitions */
#define GM_F_LEVEL_MAJOR 512u /* gm_plan / gm_plan_shard: the level-major DENSE
                                  layout even where PLANES applies (A/B runs) */
#define GM_F_PLANE_X1 1024u   /* PLANES: one plane per half-wave in 32-bit lanes
                                  (k_plane_resolve) instead of two per half-wave
                                  in packed 16-bit lanes (A/B runs) */
#define GM_F_PLANE_ROUND_ROBIN 2048u /* PLANES shards: deal the top-digit blocks
                                  round robin (every halo to rank + 1, one link)
                                  instead of the link-spreading deal used for
                                  power-of-two worlds >= 4 (A/B runs) */
#define GM_F_PLANE_LEVEL_SYNC 4096u /* PLANES shards: the level-synchronous deal
                                  (blocks of 8 top values, one halo exchange
                                  per plane level) even where the staged
                                  pipeline applies (A/B runs) */
#define GM_F_PLANE_NO_RUNS 8192u /* PLANES: one launch per narrow plane level /
                                  staged key instead of one-workgroup runs of
                                  them (A/B runs) */
#define GM_F_BKS_LOCAL 16384u /* md5-sharded BUCKETED levels: dedup each rank's
                                  children locally first and hash / send each
                                  unique child once (A/B against hashing and
                                  sending every child occurrence) */
#define GM_F_RANKED_SHARD 32768u /* gm_plan_keyed_shard: toot-and-otto as md5
                                  shards of the RANKED index space (every
                                  slot resolved by its md5 owner, level words
                                  exchanged; gm_ranked_shard.h) instead of
                                  BUCKETED levels */
#define GM_F_PLANE_LEVELS 65536u /* PLANES one-table solves: one launch per
                                  plane level (narrow levels in runs and
                                  pairs) instead of the one-launch backward
                                  (k_plane_flow; A/B, and the schedule of
                                  partial / resumed solves) */
#define GM_F_GRAPH 256u      /* dense one-table full solves: capture the
                                  forward and backward launches as HIP graphs
                                  on the first solve, replay them after
                                  (measured: no faster than plain launches) */

typedef struct gm_result {
  uint32_t root_word;
  int32_t root_value;        /* GM_WIN.. */
  uint64_t root_remoteness;
  uint64_t positions;        /* reachable positions solved */
  uint64_t edges;            /* children generated by non-primitive positions */
  uint64_t primitives;
  uint32_t levels;           /* non-empty tiers */
  uint32_t max_level_width;
  double ms_total;           /* host wall: first launch -> root word on host */
  double ms_forward;         /* device time, forward expansion (events) */
  double ms_backward;        /* device time, retrograde pass (events) */
  /* per-kernel device time (GM_F_KERNEL_TIMING): sums and launch counts */
  double ms_expand_kernels;
  double ms_resolve_kernels;
  uint64_t n_expand_launches;
  uint64_t n_resolve_launches;
  uint32_t word_bits;        /* DENSE: bits per table word this solve used (8, 16 or 32); 0 keyed */
  uint32_t kernels;          /* DENSE: resolve family | pull family << 16 (gm_solver.hip DenseResolveKind) */
} gm_result;

/* sizeof(gm_plan_t), sizeof(gm_buffers), sizeof(gm_result) as compiled into
 * the library: bindings check their struct layouts against it (host-only). */
int gm_abi_sizes(uint32_t out[3]);

/* Game lookup: name = reference game-file stem ("four_to_one",
 * "sum_four_to_one", "tic_tac_toe_np", "mttt", "toot_and_otto_bitstring",
 * "othello_bit_new"); params "length=6,height=4" / "start=20" /
 * "heaps=31:31:31".  Replaces solver_launcher.py:41-42,55-66 (load +
 * validate the game module). */
int gm_game_lookup(const char *name, const char *params, int *game_id);

/* Number of tiers and a default capacity bound for the game. */
int gm_game_info(int game, uint64_t *positions_bound, uint32_t *max_levels,
                 uint32_t *key_bits);

/* Root key: initial_position() (src/game_state.py:14). */
int gm_root(int game, uint64_t *key);

/* Canonical bytes <-> packed key.  Canonical bytes are str(pos) for int
 * positions (four_to_one, sum_four_to_one), the latin-1 bytes of the
 * bitstring games' str positions, the 9 chars of mttt and the 9 int8 cells
 * (ndarray.tobytes()) of tic_tac_toe_np. */
int gm_encode(int game, const uint8_t *canon, size_t n, uint64_t *key);
int gm_decode(int game, uint64_t key, uint8_t *canon, size_t cap,
              size_t *n);

/* batch forms: canon rows of `stride` bytes, lengths in lens[] */
int gm_encode_batch(int game, const uint8_t *canon, size_t stride,
                    const uint8_t *lens, size_t n, uint64_t *keys);
int gm_decode_batch(int game, const uint64_t *keys, size_t n, uint8_t *canon,
                    size_t stride, uint8_t *lens);

/* str(pos).encode('utf-8') -- the md5 partition input of
 * GameState.get_hash (src/game_state.py:22-30). */
int gm_str_utf8(int game, uint64_t key, uint8_t *out, size_t cap,
                size_t *n);

/* Host-side run of the product's own descriptor (primitive + ordered
 * children, GameState.expand / .primitive, src/game_state.py:32-40,58-84)
 * for parity probes.  children: n * GM_MAXCHILD keys. */
#define GM_MAXCHILD 32
int gm_host_expand(int game, const uint64_t *keys, size_t n,
                   uint64_t *children, uint8_t *nchild, uint8_t *prim);
/* host run of the descriptor's level function (tier of each key: the
 * number of moves from the root, counting a two-tier step as two) */
int gm_host_level(int game, const uint64_t *keys, size_t n, int32_t *levels);
/* Symmetry hooks (params "symmetry=1"): the game
 * module's symmetry_functions() (othello_bit_new.py:224-235, unused by the
 * reference's solvers) as key maps, host-run.  which = -1: canonical
 * representative of each key's orbit (what a symmetric solve stores and
 * gm_solver_query looks up); which = i >= 0: symmetry function i itself
 * (othello: 0 = player_flip), for checking a module against its descriptor. */
int gm_symmetry(int game, int which, const uint64_t *keys, size_t n,
                uint64_t *out);

/* Buffer sizes for a solve of at most `positions` reachable positions
 * (0 = the game's own bound).  DENSE is chosen when the descriptor supports
 * it, its table fits in `max_table_bytes` (0 = no limit) and flags lacks
 * GM_F_FORCE_HASHED. */
int gm_plan(int game, uint64_t positions, uint32_t flags,
            uint64_t max_table_bytes, gm_plan_t *out);

/* Stateful solver on the current HIP device.  Replaces Process
 * (src/process.py:10-267): run() is gm_solver_solve; the resolved/remote
 * CacheDicts (src/cache_dict.py) are the HBM table read by gm_solver_query. */
typedef struct gm_solver gm_solver;
int gm_solver_create(int game, const gm_buffers *buf, gm_solver **out);
int gm_solver_solve(gm_solver *s, gm_result *out);
/* Queued full solves (one-table PLANES solvers): gm_solver_solve_async
 * enqueues a whole solve on the solver's stream and returns at once with a
 * ticket; gm_solver_collect waits for that solve and fills *out as
 * gm_solver_solve would (ms_total = the solve's device span).  Up to 8 may
 * be queued; collect them in ticket order.  Solves queued back to back run
 * back to back on the device with no host round trip between them -- the
 * throughput form of the reference's one-job-at-a-time run()
 * (src/process.py:37-60). */
int gm_solver_solve_async(gm_solver *s, uint64_t *ticket);
int gm_solver_collect(gm_solver *s, uint64_t ticket, gm_result *out);
/* words_dev[i] = word of keys_dev[i] (GM_NO_WORD if not reachable) */
int gm_solver_query(gm_solver *s, const uint64_t *keys_dev, uint64_t n,
                    uint32_t *words_dev);
/* copy every reachable key into keys_dev (capacity cap); *n = count */
int gm_solver_positions(gm_solver *s, uint64_t *keys_dev, uint64_t cap,
                        uint64_t *n);
void gm_solver_destroy(gm_solver *s);
/* Whole-solve fingerprint of a finished solve: out[0] = sum (mod 2^64) over
 * every reachable position this table holds of a mix of its canonical bytes
 * (gm_decode), value and remoteness; out[1] = positions; out[2..5] = WIN /
 * LOSS / TIE / DRAW counts.  Order- and layout-independent (md5 shards add
 * up), so a solve can be compared with a CPU restatement of any size
 * without dumping it (the reference's equivalent is reading every
 * resolved/remote shelve entry, src/cache_dict.py:44-60). */
int gm_solver_checksum(gm_solver *s, uint64_t out[6]);
/* change GM_F_* flags of an existing solver (e.g. kernel timing) */
int gm_solver_set_flags(gm_solver *s, uint32_t flags);
/* Level-granular stop / resume (checkpoints; SURVEY.md §8f rank 2 -- the
 * reference's only persistence is its write-through shelve files,
 * src/cache_dict.py:38-60).  A one-GPU solve is 2T steps (T = max_levels):
 * step k < T is forward level k, step T + j is backward level T-1-j.  The
 * next gm_solver_solve starts at step `first` and stops before step `stop`
 * (0 = run to the end), returning GM_PARTIAL when it stopped early.
 * first = 0 starts fresh (clears table and state); first > 0 resumes: the
 * table, level store and scratch buffers must hold exactly what a solve that
 * stopped before step `first` left in them (the same solver, or buffers
 * restored from a checkpoint of the same plan).  The setting applies to one
 * gm_solver_solve call.  Sharded solves refuse it. */
int gm_solver_set_steps(gm_solver *s, uint32_t first, uint32_t stop);

/* ---- multi-GPU ----------------------------------
 * Replaces the reference's md5-partitioned ranks + per-edge mpi4py messages
 * (src/game_state.py:22-30, src/process.py:146-185).  DENSE tables cut the
 * values of the top prefix digit (the last heap) into blocks of >= 2 dealt
 * round robin to the ranks, and exchange two boundary slices per block and
 * level (RCCL send/recv on a comm stream, overlapped with compute).  Sizes
 * for rank `rank` of `world`: */
int gm_plan_shard(int game, int rank, int world, uint32_t flags,
                  uint64_t max_table_bytes, gm_plan_t *out);
int gm_solver_create_shard(int game, int rank, int world,
                           const gm_buffers *buf, gm_solver **out);
/* Keyed games whose every move advances one level (tic-tac-toe, toot-and-
 * otto, othello): one shard of an md5-partitioned BUCKETED solve -- the
 * positions with md5(str(pos)) % world == rank (GameState.get_hash,
 * src/game_state.py:22-30; the routing of src/process.py:157-160), each
 * level's child occurrences moved to their owners and the answers back in
 * two all-to-alls per level (gm_solve_group for every shard in one process;
 * gm_solver_solve per process over RCCL or a transport).  `positions`:
 * bound on this shard's positions (0: the game's own).  Replaces the
 * per-edge LOOK_UP / RESOLVE messages of src/process.py:146-185. */
int gm_plan_keyed_shard(int game, int rank, int world, uint64_t positions,
                        uint32_t flags, uint64_t max_table_bytes,
                        gm_plan_t *out);
/* host-only: geometry of shard `rank` -- out[0..7] = block width B (values
 * of the top digit per block), blocks over all ranks, blocks of this rank
 * (global blocks rank, rank + world, ...), rank, slice size Z (prefixes
 * per top value), top extent E, local prefixes per level (each block with
 * two halo slices on either side), world */
int gm_shard_info(int game, int rank, int world, uint64_t out[8]);
/* RCCL bootstrap: rank 0 calls gm_comm_unique_id (128 bytes), the host
 * broadcasts them (torch.distributed), every rank calls
 * gm_solver_comm_init; gm_solver_solve then exchanges halos over RCCL. */
#define GM_COMM_ID_BYTES 128
int gm_comm_unique_id(void *id_out);
int gm_solver_comm_init(gm_solver *s, const void *id);
/* Host-staged transport (one shard per process without RCCL, e.g.
 * torch.distributed over gloo): the solver stages every halo in host memory
 * and calls fn, which returns 0 once the transfer is complete.
 *   GM_XFER_SENDRECV  send sbytes of sbuf to rank speer and receive rbytes
 *                     into rbuf from rank rpeer (either may be 0 bytes)
 *   GM_XFER_ALLGATHER every rank's sbytes of sbuf into rbuf, rank order
 *                     (world * sbytes; speer / rpeer unused)
 * Replaces the communicator for gm_solver_solve; NULL fn restores RCCL. */
#define GM_XFER_SENDRECV 0
#define GM_XFER_ALLGATHER 1
typedef int (*gm_xfer_fn)(void *ctx, int op, const void *sbuf, uint64_t sbytes, int speer, void *rbuf,
                          uint64_t rbytes, int rpeer);
int gm_solver_set_transport(gm_solver *s, gm_xfer_fn fn, void *ctx);
/* The per-level halo fingerprints a shard checks against its neighbours'
 * before level 0 (gm_solver.hip halo_sigs): out[T][4] = bits sent down,
 * bits received from above, words sent up, words received from below.
 * Host only: no device memory, no GPU needed. */
int gm_shard_halo_sigs(int game, int rank, int world, uint32_t flags, uint64_t *out, uint32_t levels);
/* PLANES shards: the halo plan of shard `rank` (gm_plane_run.h
 * plane_lists), host only.  out[(step * world + p) * 2 + 0] = boundary planes
 * the shard sends to rank p at that step, [.. + 1] = planes it receives from
 * p (the rest of out[levels][world][2] zeroed).  A step is a plane level for
 * the level-synchronous deal (GM_F_PLANE_LEVEL_SYNC, or shapes the staged
 * deal does not fit) and a halo row -- the boundary planes of one lower-digit
 * sum, sent to rank + 1 -- for the staged pipeline.  `levels` >= the steps
 * (the game's levels always suffice), else GM_EINVAL.  Replaces the per-edge
 * message fan-out of the reference's shards (src/process.py:37-267). */
int gm_plane_halo_plan(int game, int rank, int world, uint32_t flags, uint64_t *out, uint32_t levels);
/* md5 shards of the RANKED layout: out[0] = the slots this shard resolved in
 * its last solve (k_rk_backward<OWN>), out[1] = the reached positions its md5
 * owner rule gives it (src/game_state.py:22-30).  Equal on every shard, and
 * the out[1] add up to the positions, when every position was resolved on
 * its owner. */
int gm_rk_shard_stats(gm_solver *s, uint64_t out[2]);
/* All `n` shards of one job in ONE process on one stream, halos moved by
 * device-to-device copies: the same kernels and halo geometry as the RCCL
 * path, runnable on a single GPU (parity tests). */
int gm_solve_group(gm_solver **shards, int n, gm_result *out);

/* ---- md5-sharded keyed (HASHED) tables ---------------------------------
 * The reference's own partition, owner(pos) = md5(str(pos)) % world
 * (src/game_state.py:22-30), with the per-edge LOOK_UP / RESOLVE messages
 * of src/process.py:146-185 replaced by two bulk all-to-all(v) exchanges
 * per level that the host performs between these steps (keyed.py).  A
 * shard is gm_solver_create_shard(game, rank, world, HASHED buffers).
 * Forward, for L = 0 .. max_levels-2:
 *   gm_ks_expand   children of own level-L positions + their owners
 *                  (GM_EFULL with *n = needed when cap is short)
 *   gm_ks_insert   keys received from every rank (all owned here)
 *   gm_ks_finalize level bookkeeping; reports table/level overflow
 * Backward, for L = max_levels-1 .. 0:
 *   gm_ks_counts   children per own level-L position (uint64 each)
 *   gm_ks_children children at offsets[i] (exclusive scan, n+1 entries)
 *   gm_solver_query  (owner side) words of the keys other ranks sent
 *   gm_ks_reduce   value/remoteness of each position from the words of
 *                  its children, in gm_ks_children order
 * gm_ks_end: this shard's counts; root_word is GM_NO_WORD except on the
 * root's owner. */
int gm_ks_begin(gm_solver *s, int root_owned);
int gm_ks_level_size(gm_solver *s, int level, uint64_t *n);
int gm_ks_expand(gm_solver *s, int level, uint64_t *keys_dev,
                 uint32_t *owners_dev, uint64_t cap, int world, uint64_t *n);
int gm_ks_insert(gm_solver *s, int level, const uint64_t *keys_dev,
                 uint64_t n);
int gm_ks_finalize(gm_solver *s, int level);
int gm_ks_counts(gm_solver *s, int level, uint64_t *counts_dev);
int gm_ks_children(gm_solver *s, int level, const uint64_t *offsets_dev,
                   uint64_t *keys_dev, uint32_t *owners_dev, int world);
int gm_ks_reduce(gm_solver *s, int level, const uint64_t *offsets_dev,
                 const uint32_t *child_words_dev);
int gm_ks_end(gm_solver *s, gm_result *out);

/* ---- game files without a device descriptor ------------
 * The host enumerates the positions with the module's own functions
 * (GameState.expand / .primitive, src/game_state.py:32-40,58-84; Python in
 * gamesmanmpi_amd/generic.py) into a CSR graph: prim[n] (GM_WIN..
 * GM_UNDECIDED), children of position i at children[offsets[i] ..
 * offsets[i+1]) in gen_moves order (uint32 ids), root id.  The device
 * resolves it in rounds (each round resolves every position whose children
 * are all resolved) with the same reduction as gm_solve; words_dev[n]
 * receives value | remoteness << 2.  scratch_dev: gm_plan's scratch_bytes
 * for any game, or >= 4 KB.  result.levels = rounds (the DAG height + 1).
 * GM_ECORRUPT if positions never resolve (a cycle). */
int gm_graph_solve(const uint8_t *prim_dev, const uint64_t *offsets_dev,
                   const uint32_t *children_dev, uint64_t n, uint64_t root,
                   uint32_t *words_dev, void *scratch_dev, void *stream,
                   gm_result *out);

/* One-shot pair: gm_solve creates a solver on the caller's
 * buffers and solves from the game's root; the solver is kept per game id
 * (the buffers must stay valid) until the next gm_solve of that game or
 * gm_release(game).  Replaces solver_launcher.py:68-72 (Process
 * construction + run) and the rank count of `mpiexec -n P`
 * (solver_launcher.py:30,76-84).
 * ngpus > 1: buf points to ngpus gm_buffers, buf[i] allocated on device i
 * with the sizes gm_plan_multi gives for shard i; the library makes one RCCL
 * communicator per device (ncclCommInitAll) and drives every shard from its
 * own host thread; *out holds the whole job's counts and root.  GM_EINVAL
 * when fewer than ngpus devices are visible.  gm_query serves one-GPU
 * solves (shards: gm_solver_query per device). */
int gm_solve(int game, uint64_t root, int ngpus, const gm_buffers *buf,
             gm_result *out);
/* Plans of the ngpus shards gm_solve(.., ngpus, ..) runs, plans[0..ngpus):
 * ngpus 1 is gm_plan; sum games: gm_plan_shard per rank (PLANES blocks of
 * the last heap, or level-major DENSE); keyed games whose moves advance one
 * level: gm_plan_keyed_shard per rank, each bounded by its md5 share of
 * `positions` (0: the board's own count) + 3 % + 64 K.  Host only. */
int gm_plan_multi(int game, int ngpus, uint64_t positions, uint32_t flags,
                  uint64_t max_table_bytes, gm_plan_t *plans);
/* words_dev[i] = word of keys_dev[i] in the table of the game's last
 * gm_solve (GM_NO_WORD if unreachable); device pointers, synchronous.
 * Replaces the resolved/remote CacheDict lookups (src/cache_dict.py:62-79). */
int gm_query(int game, const uint64_t *keys_dev, size_t n,
             uint32_t *words_dev);
/* drop the solver gm_solve kept for `game` (0 if none) */
int gm_release(int game);

/* md5(str(pos).encode('utf-8')) mod world_size for n device keys
 * (GameState.get_hash, src/game_state.py:22-30). */
int gm_owner(int game, const uint64_t *keys_dev, uint64_t n, int world_size,
             uint32_t *owners_dev, void *stream);
/* host version of the same (for parity tests and the launcher) */
int gm_owner_host(int game, const uint64_t *keys, size_t n, int world_size,
                  uint32_t *owners);

const char *gm_last_error(void);
const char *gm_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GAMESMAN_H */
