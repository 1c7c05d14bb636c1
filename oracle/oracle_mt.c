/*
 * oracle/oracle_mt.c -- MULTI-THREADED CPU RESTATEMENTS (#included at the end
 * of oracle.c, same translation unit: it reuses the literal game functions).
 *
 *   *** TEST INFRASTRUCTURE / CPU BASELINE ONLY. ***  Same rule as oracle.c:
 *   only tests/, tests/golden/ generators, __graft_entry__.smoke() and
 *   bench.py's cpu_baseline leg load it.
 *
 * Two solvers, both the reference-canonical retrograde of oracle.c
 * (src/process.py:109-267), parallel over all host
 * cores with OpenMP:
 *
 *   or_solve_levels   any game: tier-synchronous forward expansion (children
 *                     of level L deduplicated into level L+1 / L+2 by sorting)
 *                     then a backward pass that looks each child's word up in
 *                     its level.  Positions are stored as a 64-bit packing of
 *                     the literal byte image (storage only: every game
 *                     function still runs on the reference's representation),
 *                     sorted by a bijective mix so a level is bucket-indexable.
 *   or_solve_rows     sum_four_to_one / four_to_one: the state space is the
 *                     box prod(h_i + 1) ranked in mixed radix (the rank IS the
 *                     int position, four_to_one.py:7-22 per heap), solved row
 *                     by row: a row holds every heap-0 value of one setting of
 *                     heaps 1..K-1, rows are processed in order of their digit
 *                     sum (children of a row lie in the same row or in rows of
 *                     digit sum one or two lower), rows of one digit sum in
 *                     parallel.  Reachability is computed, not assumed.
 *
 * Both produce an order-independent checksum of every reachable position's
 * (canonical bytes, value, remoteness) -- the same function as
 * gm_solver_checksum in the product (gamesmanmpi_amd/csrc/gm_codec.h) --
 * so a GPU solve can be compared position-for-position with a CPU solve of
 * any size without dumping tables.
 */
#include <omp.h>

/* order-independent per-position checksum term (== gm::pos_checksum) */
static uint64_t ck_term(const uint8_t *c, int n, uint32_t value, uint32_t rem) {
  uint64_t a = 0xcbf29ce484222325ull;
  for (int i = 0; i < n; i++) {
    a ^= c[i];
    a *= 0x100000001b3ull;
  }
  a ^= (uint64_t)n << 56;
  a = a * 0x9E3779B97F4A7C15ull + ((uint64_t)value << 40) + rem;
  a ^= a >> 29;
  a *= 0xBF58476D1CE4E5B9ull;
  a ^= a >> 32;
  return a;
}

int or_threads(void) { return omp_get_max_threads(); }

/* ------------------------------------------------------------------------ */
/* storage packing of the literal byte image                                */
/* ------------------------------------------------------------------------ */
static uint64_t mix64(uint64_t x) { /* splitmix64 finaliser (bijective) */
  x ^= x >> 31;
  x *= 0x7fb5d329728ea185ull;
  x ^= x >> 27;
  x *= 0x81dadef4bc2dd44dull;
  x ^= x >> 33;
  return x;
}
static uint64_t inv_odd(uint64_t a) { /* a^-1 mod 2^64 (Newton) */
  uint64_t x = a;
  for (int i = 0; i < 6; i++) x *= 2 - a * x;
  return x;
}
static uint64_t unmix64(uint64_t x) {
  static uint64_t i1, i2;
  if (!i1) {
    i2 = inv_odd(0x81dadef4bc2dd44dull);
    i1 = inv_odd(0x7fb5d329728ea185ull);
  }
  x ^= x >> 33;
  x *= i2;
  x ^= (x >> 27) ^ (x >> 54);
  x *= i1;
  x ^= (x >> 31) ^ (x >> 62);
  return x;
}

static int pack_blob(const game *g, const blob *s, uint64_t *k) {
  uint64_t v = 0;
  switch (g->kind) {
    case G_FTO:
    case G_SUM: *k = (uint64_t)blob_i64(s); return 0;
    case G_TTTNP:
      for (int i = 0; i < 9; i++) {
        if (s->b[i] > 2) return -1;
        v |= (uint64_t)s->b[i] << (2 * i);
      }
      *k = v;
      return 0;
    case G_MTTT:
      for (int i = 0; i < 9; i++) {
        uint64_t c = s->b[i] == '_' ? 0 : s->b[i] == 'X' ? 1 : s->b[i] == 'O' ? 2 : 3;
        if (c == 3) return -1;
        v |= c << (2 * i);
      }
      *k = v;
      return 0;
    case G_TOOT: {
      const int A = g->area;
      for (int i = 0; i < 2 * A; i++) v |= (uint64_t)bget(s->b, i) << i;
      for (int j = 0; j < 4; j++) {
        int h = bint(s->b, 2 * A + 4 * j, 4);
        if (h < 0 || h > 7) return -1;
        v |= (uint64_t)h << (2 * A + 3 * j);
      }
      if (!bget(s->b, 2 * A + 16)) return -1;
      for (int i = 2 * A + 17; i < g->nbits - 1; i++)
        if (bget(s->b, i)) return -1;
      v |= (uint64_t)bget(s->b, g->nbits - 1) << (2 * A + 12);
      *k = v;
      return 0;
    }
    default: { /* othello */
      const int A = g->area;
      for (int i = 0; i < 2 * A; i++) v |= (uint64_t)bget(s->b, i) << i;
      int t = ot_turncount(g, s->b), p = ot_passes(g, s->b);
      if ((t != 1 && t != 2) || p < 0 || p > 3) return -1;
      for (int i = 2 * A + 16; i < g->nbits; i++)
        if (bget(s->b, i)) return -1;
      v |= (uint64_t)(t == 1) << (2 * A);
      v |= (uint64_t)p << (2 * A + 1);
      *k = v;
      return 0;
    }
  }
}

static void unpack_blob(const game *g, uint64_t k, blob *s) {
  memset(s, 0, sizeof *s);
  switch (g->kind) {
    case G_FTO:
    case G_SUM: i64_blob(s, (int64_t)k); return;
    case G_TTTNP:
      for (int i = 0; i < 9; i++) s->b[i] = (uint8_t)((k >> (2 * i)) & 3);
      return;
    case G_MTTT:
      for (int i = 0; i < 9; i++) {
        int c = (int)((k >> (2 * i)) & 3);
        s->b[i] = (uint8_t)(c == 0 ? '_' : c == 1 ? 'X' : 'O');
      }
      return;
    case G_TOOT: {
      const int A = g->area;
      for (int i = 0; i < 2 * A; i++)
        if ((k >> i) & 1) bset(s->b, i, 1);
      for (int j = 0; j < 4; j++) bput(s->b, 2 * A + 4 * j, 4, (int)((k >> (2 * A + 3 * j)) & 7));
      bset(s->b, 2 * A + 16, 1);
      if ((k >> (2 * A + 12)) & 1) bset(s->b, g->nbits - 1, 1);
      return;
    }
    default: {
      const int A = g->area;
      for (int i = 0; i < 2 * A; i++)
        if ((k >> i) & 1) bset(s->b, i, 1);
      bput(s->b, 2 * A, 8, ((k >> (2 * A)) & 1) ? 1 : 2);
      bput(s->b, 2 * A + 8, 8, (int)((k >> (2 * A + 1)) & 3));
      return;
    }
  }
}

/* tier of a position: moves from the root (a -2 move of the int games
 * counts two) -- pieces placed, pieces - 4 + passes for othello */
static int level_of(const game *g, const blob *s) {
  switch (g->kind) {
    case G_FTO: return (int)(g->fto_start - blob_i64(s));
    case G_SUM: {
      int64_t r = blob_i64(s), sum = 0, root = 0;
      for (int i = 0; i < g->nheaps; i++) {
        sum += r % (g->heaps[i] + 1);
        r /= g->heaps[i] + 1;
        root += g->heaps[i];
      }
      return (int)(root - sum);
    }
    case G_TTTNP: {
      int n = 0;
      for (int i = 0; i < 9; i++) n += s->b[i] != 0;
      return n;
    }
    case G_MTTT: {
      int n = 0;
      for (int i = 0; i < 9; i++) n += s->b[i] != '_';
      return n;
    }
    case G_TOOT: {
      int n = 0;
      for (int i = 0; i < g->area; i++) n += bget(s->b, i) | bget(s->b, g->area + i);
      return n;
    }
    default: {
      int n = 0;
      for (int i = 0; i < g->area; i++) n += bget(s->b, i) | bget(s->b, g->area + i);
      return n - 4 + ot_passes(g, s->b);
    }
  }
}

static int max_levels_of(const game *g) {
  switch (g->kind) {
    case G_FTO: return (int)g->fto_start + 1;
    case G_SUM: {
      int root = 0;
      for (int i = 0; i < g->nheaps; i++) root += g->heaps[i];
      return root + 1;
    }
    case G_TTTNP:
    case G_MTTT: return 10;
    case G_TOOT: return g->area + 1;
    default: return g->area + 3;
  }
}

/* ------------------------------------------------------------------------ */
/* sorted levels                                                             */
/* ------------------------------------------------------------------------ */
typedef struct {
  uint64_t *a;
  uint64_t n, cap;
} vec64;

static int v_push(vec64 *v, uint64_t x) {
  if (v->n == v->cap) {
    uint64_t c = v->cap ? 2 * v->cap : 1024;
    uint64_t *p = realloc(v->a, c * sizeof *p);
    if (!p) return -1;
    v->a = p;
    v->cap = c;
  }
  v->a[v->n++] = x;
  return 0;
}

static int cmp_u64(const void *x, const void *y) {
  uint64_t a = *(const uint64_t *)x, b = *(const uint64_t *)y;
  return a < b ? -1 : a > b;
}

#define SB 12 /* sort buckets: top SB bits of the mixed key */

/* sort + dedup `n` mixed keys in place (parallel MSD bucket + qsort);
 * returns the unique count */
static uint64_t sort_unique(uint64_t *a, uint64_t n) {
  if (n < (1u << 16)) {
    qsort(a, n, sizeof *a, cmp_u64);
    uint64_t m = 0;
    for (uint64_t i = 0; i < n; i++)
      if (!m || a[m - 1] != a[i]) a[m++] = a[i];
    return m;
  }
  const int NBK = 1 << SB, T = omp_get_max_threads();
  uint64_t *cnt = calloc((size_t)T * NBK, sizeof *cnt), *tmp = malloc(n * sizeof *tmp);
  uint64_t *start = malloc((NBK + 1) * sizeof *start), *uq = calloc(NBK, sizeof *uq);
#pragma omp parallel
  {
    const int t = omp_get_thread_num();
    uint64_t *c = cnt + (size_t)t * NBK;
#pragma omp for schedule(static)
    for (uint64_t i = 0; i < n; i++) c[a[i] >> (64 - SB)]++;
#pragma omp single
    {
      uint64_t run = 0;
      for (int b = 0; b < NBK; b++) {
        start[b] = run;
        for (int u = 0; u < T; u++) {
          uint64_t x = cnt[(size_t)u * NBK + b];
          cnt[(size_t)u * NBK + b] = run;
          run += x;
        }
      }
      start[NBK] = run;
    }
#pragma omp for schedule(static)
    for (uint64_t i = 0; i < n; i++) tmp[c[a[i] >> (64 - SB)]++] = a[i];
#pragma omp for schedule(dynamic, 16)
    for (int b = 0; b < NBK; b++) {
      uint64_t *s = tmp + start[b], m = 0, k = start[b + 1] - start[b];
      qsort(s, k, sizeof *s, cmp_u64);
      for (uint64_t i = 0; i < k; i++)
        if (!m || s[m - 1] != s[i]) s[m++] = s[i];
      uq[b] = m;
    }
  }
  uint64_t out = 0;
  for (int b = 0; b < NBK; b++) {
    memcpy(a + out, tmp + start[b], uq[b] * sizeof *a);
    out += uq[b];
  }
  free(cnt);
  free(tmp);
  free(start);
  free(uq);
  return out;
}

/* a sorted level with a bucket index over the top `ib` bits */
typedef struct {
  uint64_t *k;   /* mixed packed keys, ascending */
  uint64_t n;
  uint32_t *w;   /* words (value | remoteness << 2) */
  uint64_t *ix;  /* ix[b] = first index with top ib bits >= b; ix[1 << ib] = n */
  int ib;
} olevel;

static void level_index(olevel *L) {
  int ib = 1;
  while (ib < 30 && (1ull << ib) < L->n / 4 + 1) ib++;
  L->ib = ib;
  const uint64_t NB = 1ull << ib;
  L->ix = malloc((NB + 1) * sizeof *L->ix);
#pragma omp parallel for schedule(static)
  for (uint64_t b = 0; b <= NB; b++) {
    /* first i with a[i] >> (64 - ib) >= b: binary search */
    uint64_t lo = 0, hi = L->n;
    while (lo < hi) {
      uint64_t m = (lo + hi) / 2;
      if ((L->k[m] >> (64 - ib)) < b) lo = m + 1;
      else hi = m;
    }
    L->ix[b] = lo;
  }
}

static int64_t level_find(const olevel *L, uint64_t h) {
  if (!L->n) return -1;
  const uint64_t b = h >> (64 - L->ib);
  for (uint64_t i = L->ix[b], e = L->ix[b + 1]; i < e; i++)
    if (L->k[i] == h) return (int64_t)i;
  return -1;
}

typedef struct {
  int game, T;
  olevel *lv;
  uint64_t count, edges, prims, checksum, hist[4];
  uint32_t root_word;
  int keep; /* keep every level (lookups) or free them as the pass goes */
} lsolve_t;

static void lfree(lsolve_t *S) {
  if (!S) return;
  if (S->lv)
    for (int L = 0; L < S->T; L++) {
      free(S->lv[L].k);
      free(S->lv[L].w);
      free(S->lv[L].ix);
    }
  free(S->lv);
  free(S);
}

/* Tier-synchronous solve of any game on all OpenMP threads.  keep = 1 keeps
 * every level for or_lsolve_lookup; 0 frees keys as soon as the backward
 * pass no longer needs them (large games). */
void *or_solve_levels(int h, int keep) {
  const game *g = G(h);
  if (!g) { snprintf(g_err, sizeof g_err, "bad game handle"); return NULL; }
  lsolve_t *S = calloc(1, sizeof *S);
  S->game = h;
  S->T = max_levels_of(g);
  S->keep = keep;
  S->lv = calloc((size_t)S->T, sizeof *S->lv);
  const int T = S->T, NT = omp_get_max_threads();
  vec64 *pend = calloc((size_t)T + 2, sizeof *pend); /* children awaiting dedup */
  vec64 *tb = NULL;
  blob root;
  root_of(g, &root);
  uint64_t rk;
  if (pack_blob(g, &root, &rk)) { snprintf(g_err, sizeof g_err, "root does not pack"); goto fail; }
  v_push(&pend[0], mix64(rk));
  tb = calloc((size_t)NT * 2, sizeof *tb);
  volatile int bad = 0;
  /* ---- forward ---- */
  for (int L = 0; L < T; L++) {
    olevel *lv = &S->lv[L];
    lv->n = sort_unique(pend[L].a, pend[L].n);
    lv->k = pend[L].n ? realloc(pend[L].a, (lv->n ? lv->n : 1) * sizeof(uint64_t)) : pend[L].a;
    memset(&pend[L], 0, sizeof pend[L]);
    S->count += lv->n;
    if (L + 1 == T || !lv->n) continue;
#pragma omp parallel
    {
      const int t = omp_get_thread_num();
      blob s, ch[OR_MAXCHILD];
#pragma omp for schedule(dynamic, 4096)
      for (uint64_t i = 0; i < lv->n; i++) {
        unpack_blob(g, unmix64(lv->k[i]), &s);
        if (prim_of(g, &s) != UNDECIDED) continue;
        int nc = children_of(g, &s, ch);
        for (int c = 0; c < nc; c++) {
          uint64_t k;
          int step = level_of(g, &ch[c]) - L;
          if ((step != 1 && step != 2) || L + step >= T || pack_blob(g, &ch[c], &k)) { bad = 1; continue; }
          if (v_push(&tb[2 * t + step - 1], mix64(k))) bad = 1;
        }
      }
    }
    if (bad) { snprintf(g_err, sizeof g_err, "child outside levels L+1/L+2, or not packable"); goto fail; }
    for (int q = 0; q < 2; q++) {
      vec64 *dst = &pend[L + 1 + q];
      uint64_t add = 0;
      for (int t = 0; t < NT; t++) add += tb[2 * t + q].n;
      if (!add) continue;
      uint64_t *p = realloc(dst->a, (dst->n + add) * sizeof *p);
      if (!p) { snprintf(g_err, sizeof g_err, "oom"); goto fail; }
      dst->a = p;
      for (int t = 0; t < NT; t++) {
        memcpy(dst->a + dst->n, tb[2 * t + q].a, tb[2 * t + q].n * sizeof *p);
        dst->n += tb[2 * t + q].n;
        tb[2 * t + q].n = 0;
      }
      dst->cap = dst->n;
    }
    for (int t = 0; t < 2 * NT; t++) {
      free(tb[t].a);
      memset(&tb[t], 0, sizeof tb[t]);
    }
  }
  free(tb);
  tb = NULL;
  /* ---- backward ---- */
  for (int L = T - 1; L >= 0; L--) {
    olevel *lv = &S->lv[L];
    level_index(lv);
    lv->w = malloc((lv->n ? lv->n : 1) * sizeof(uint32_t));
    uint64_t edges = 0, prims = 0, ck = 0, h0 = 0, h1 = 0, h2 = 0, h3 = 0;
#pragma omp parallel for schedule(dynamic, 4096) reduction(+ : edges, prims, ck, h0, h1, h2, h3)
    for (uint64_t i = 0; i < lv->n; i++) {
      blob s, ch[OR_MAXCHILD];
      unpack_blob(g, unmix64(lv->k[i]), &s);
      int p = prim_of(g, &s);
      uint32_t word;
      if (p != UNDECIDED) {
        word = (uint32_t)p; /* process.py:120-123 */
        prims++;
      } else {
        int nc = children_of(g, &s, ch);
        if (!nc) bad = 1;
        int any_loss = 0, any_tie = 0, any_draw = 0;
        uint32_t min_loss = 0xFFFFFFFFu, max_all = 0;
        for (int c = 0; c < nc; c++) {
          uint64_t k;
          pack_blob(g, &ch[c], &k);
          const olevel *cl = &S->lv[level_of(g, &ch[c])];
          int64_t j = level_find(cl, mix64(k));
          if (j < 0) { bad = 1; continue; }
          uint32_t cw = cl->w[j], v = cw & 3, r = cw >> 2;
          if (v == LOSS) { any_loss = 1; if (r < min_loss) min_loss = r; }
          if (v == TIE) any_tie = 1;
          if (v == DRAW) any_draw = 1;
          if (r > max_all) max_all = r;
        }
        edges += (uint64_t)nc;
        /* reference-canonical _res_red / _remote_red */
        if (any_loss) word = WIN | ((min_loss + 1) << 2);
        else word = (uint32_t)(any_tie ? TIE : any_draw ? DRAW : LOSS) | ((max_all + 1) << 2);
      }
      lv->w[i] = word;
      uint8_t cb[32];
      int cn = to_canon(g, &s, cb);
      ck += ck_term(cb, cn, word & 3, word >> 2);
      switch (word & 3) {
        case 0: h0++; break;
        case 1: h1++; break;
        case 2: h2++; break;
        default: h3++;
      }
    }
    if (bad) { snprintf(g_err, sizeof g_err, "child missing or non-primitive position without moves"); goto fail; }
    S->edges += edges;
    S->prims += prims;
    S->checksum += ck;
    S->hist[0] += h0;
    S->hist[1] += h1;
    S->hist[2] += h2;
    S->hist[3] += h3;
    if (!keep && L + 2 < T) { /* levels >= L+2 are never read again */
      olevel *o = &S->lv[L + 2];
      free(o->k); free(o->w); free(o->ix);
      o->k = NULL; o->w = NULL; o->ix = NULL;
    }
  }
  S->root_word = S->lv[0].n ? S->lv[0].w[0] : 0xFFFFFFFFu;
  free(pend);
  return S;
fail:
  if (tb) {
    for (int t = 0; t < 2 * NT; t++) free(tb[t].a);
    free(tb);
  }
  for (int L = 0; L < T + 2; L++) free(pend[L].a);
  free(pend);
  lfree(S);
  return NULL;
}

/* out[0..8] = positions, edges, primitives, root word, checksum, W, L, T, D */
void or_lsolve_stats(void *hs, uint64_t *out) {
  lsolve_t *S = hs;
  out[0] = S->count;
  out[1] = S->edges;
  out[2] = S->prims;
  out[3] = S->root_word;
  out[4] = S->checksum;
  for (int i = 0; i < 4; i++) out[5 + i] = S->hist[i];
}

uint32_t or_lsolve_lookup(void *hs, const uint8_t *canon, int len) {
  lsolve_t *S = hs;
  const game *g = G(S->game);
  blob s;
  uint64_t k;
  if (from_canon(g, canon, len, &s) || pack_blob(g, &s, &k)) return 0xFFFFFFFFu;
  int L = level_of(g, &s);
  if (L < 0 || L >= S->T || !S->lv[L].k || !S->lv[L].ix) return 0xFFFFFFFFu;
  int64_t j = level_find(&S->lv[L], mix64(k));
  return j < 0 ? 0xFFFFFFFFu : S->lv[L].w[j];
}

void or_lsolve_free(void *hs) { lfree(hs); }

/* ------------------------------------------------------------------------ */
/* row solver for the int games (sum_four_to_one / four_to_one)              */
/* ------------------------------------------------------------------------ */
typedef struct {
  int game;
  uint64_t N, base0, P;   /* positions of the box, heap-0 base, rows */
  uint32_t *w;            /* word per rank, 0xFFFFFFFF = unreachable */
  uint64_t count, edges, prims;
  uint32_t root_word;
} rsolve_t;

void *or_solve_rows(int h) {
  const game *g = G(h);
  if (!g || (g->kind != G_SUM && g->kind != G_FTO)) {
    snprintf(g_err, sizeof g_err, "row solver: sum_four_to_one / four_to_one only");
    return NULL;
  }
  int K = g->kind == G_FTO ? 1 : g->nheaps;
  int64_t H[16] = {0}, st[16] = {0};
  for (int i = 0; i < K; i++) {
    H[i] = g->kind == G_FTO ? g->fto_start : g->heaps[i];
    st[i] = g->kind == G_FTO ? 1 : g->strides[i];
  }
  rsolve_t *S = calloc(1, sizeof *S);
  S->game = h;
  S->base0 = (uint64_t)H[0] + 1;
  S->P = 1;
  int dmax = 0;
  for (int i = 1; i < K; i++) {
    S->P *= (uint64_t)H[i] + 1;
    dmax += (int)H[i];
  }
  S->N = S->base0 * S->P;
  S->w = malloc(S->N * sizeof(uint32_t));
  uint8_t *reach = calloc((S->N + 7) / 8, 1);
  uint16_t *ds = malloc(S->P * sizeof(uint16_t));
  uint64_t *cs = calloc((size_t)dmax + 2, sizeof(uint64_t));
  uint32_t *order = malloc(S->P * sizeof(uint32_t));
  if (!S->w || !reach || !ds || !cs || !order || S->P > 0xFFFFFFFFull) {
    snprintf(g_err, sizeof g_err, "oom");
    free(S->w); free(reach); free(ds); free(cs); free(order); free(S);
    return NULL;
  }
  /* rows grouped by the digit sum of heaps 1..K-1 (counting sort) */
#pragma omp parallel for schedule(static)
  for (uint64_t p = 0; p < S->P; p++) {
    uint64_t r = p;
    int s = 0;
    for (int i = 1; i < K; i++) {
      s += (int)(r % (uint64_t)(H[i] + 1));
      r /= (uint64_t)(H[i] + 1);
    }
    ds[p] = (uint16_t)s;
  }
  for (uint64_t p = 0; p < S->P; p++) cs[ds[p] + 1]++;
  for (int s = 0; s <= dmax; s++) cs[s + 1] += cs[s];
  {
    uint64_t *at = malloc(((size_t)dmax + 1) * sizeof *at);
    memcpy(at, cs, ((size_t)dmax + 1) * sizeof *at);
    for (uint64_t p = 0; p < S->P; p++) order[at[ds[p]]++] = (uint32_t)p;
    free(at);
  }
  uint64_t root = 0;
  for (int i = 0; i < K; i++) root += (uint64_t)H[i] * (uint64_t)st[i];
  const uint64_t B0 = S->base0;
#define RBIT(r) ((reach[(r) >> 3] >> ((r) & 7)) & 1)
  /* forward: reach(r) = r is the root, or a parent (one heap one or two
   * higher, four_to_one.py:10-17 undone) is reached; rows from the highest
   * digit sum down, each row from heap 0 = H0 down */
  for (int s = dmax; s >= 0; s--) {
#pragma omp parallel for schedule(dynamic, 64)
    for (uint64_t j = cs[s]; j < cs[s + 1]; j++) {
      const uint64_t p = order[j];
      int64_t dig[16];
      uint64_t r0 = p;
      for (int i = 1; i < K; i++) {
        dig[i] = (int64_t)(r0 % (uint64_t)(H[i] + 1));
        r0 /= (uint64_t)(H[i] + 1);
      }
      for (int64_t h0 = H[0]; h0 >= 0; h0--) {
        const uint64_t r = (uint64_t)h0 + B0 * p;
        int on = r == root;
        if (!on && h0 + 1 <= H[0]) on = RBIT(r + 1);
        if (!on && h0 + 2 <= H[0]) on = RBIT(r + 2);
        for (int i = 1; i < K && !on; i++) {
          if (dig[i] + 1 <= H[i] && RBIT(r + (uint64_t)st[i])) on = 1;
          else if (dig[i] + 2 <= H[i] && RBIT(r + 2 * (uint64_t)st[i])) on = 1;
        }
        if (on) __atomic_fetch_or(&reach[r >> 3], (uint8_t)(1u << (r & 7)), __ATOMIC_RELAXED);
      }
    }
  }
  /* backward: rows from the lowest digit sum up, each row from heap 0 = 0 */
  uint64_t count = 0, edges = 0, prims = 0;
  for (int s = 0; s <= dmax; s++) {
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : count, edges, prims)
    for (uint64_t j = cs[s]; j < cs[s + 1]; j++) {
      const uint64_t p = order[j];
      int64_t dig[16];
      uint64_t r0 = p;
      for (int i = 1; i < K; i++) {
        dig[i] = (int64_t)(r0 % (uint64_t)(H[i] + 1));
        r0 /= (uint64_t)(H[i] + 1);
      }
      for (int64_t h0 = 0; h0 <= H[0]; h0++) {
        const uint64_t r = (uint64_t)h0 + B0 * p;
        if (!RBIT(r)) {
          S->w[r] = 0xFFFFFFFFu;
          continue;
        }
        count++;
        if (r == 0) { /* every heap empty: LOSS, remoteness 0 */
          S->w[r] = LOSS;
          prims++;
          continue;
        }
        int any_loss = 0, nc = 0;
        uint32_t min_loss = 0xFFFFFFFFu, max_all = 0;
#define CHILD(c)                                                \
  do {                                                          \
    uint32_t cw = S->w[(c)], v = cw & 3, rr = cw >> 2;          \
    nc++;                                                       \
    if (v == LOSS) { any_loss = 1; if (rr < min_loss) min_loss = rr; } \
    if (rr > max_all) max_all = rr;                             \
  } while (0)
        if (h0 >= 1) CHILD(r - 1);
        if (h0 >= 2) CHILD(r - 2);
        for (int i = 1; i < K; i++) {
          if (dig[i] >= 1) CHILD(r - (uint64_t)st[i]);
          if (dig[i] >= 2) CHILD(r - 2 * (uint64_t)st[i]);
        }
#undef CHILD
        edges += (uint64_t)nc;
        /* only WIN / LOSS occur (every primitive is a LOSS) */
        S->w[r] = any_loss ? (WIN | ((min_loss + 1) << 2)) : (LOSS | ((max_all + 1) << 2));
      }
    }
  }
#undef RBIT
  S->count = count;
  S->edges = edges;
  S->prims = prims;
  S->root_word = S->w[root];
  free(reach);
  free(ds);
  free(cs);
  free(order);
  return S;
}

/* out[0..8] as or_lsolve_stats (checksum computed on demand: it renders
 * every reachable rank in decimal, which costs more than the solve) */
void or_rsolve_stats(void *hs, int with_checksum, uint64_t *out) {
  rsolve_t *S = hs;
  memset(out, 0, 9 * sizeof *out);
  out[0] = S->count;
  out[1] = S->edges;
  out[2] = S->prims;
  out[3] = S->root_word;
  if (!with_checksum) return;
  uint64_t ck = 0, h0 = 0, h1 = 0;
#pragma omp parallel for schedule(static) reduction(+ : ck, h0, h1)
  for (uint64_t r = 0; r < S->N; r++) {
    uint32_t w = S->w[r];
    if (w == 0xFFFFFFFFu) continue;
    char tmp[24];
    int n = snprintf(tmp, sizeof tmp, "%llu", (unsigned long long)r);
    ck += ck_term((const uint8_t *)tmp, n, w & 3, w >> 2);
    if ((w & 3) == 0) h0++;
    else h1++;
  }
  out[4] = ck;
  out[5] = h0;
  out[6] = h1;
}

uint32_t or_rsolve_word(void *hs, uint64_t rank) {
  rsolve_t *S = hs;
  return rank < S->N ? S->w[rank] : 0xFFFFFFFFu;
}

void or_rsolve_free(void *hs) {
  rsolve_t *S = hs;
  if (!S) return;
  free(S->w);
  free(S);
}
