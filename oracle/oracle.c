/*
 * oracle/oracle.c -- CPU RESTATEMENT OF THE REFERENCE'S HOT PATH.
 *
 *   *** TEST INFRASTRUCTURE ONLY. ***  Only tests/, __graft_entry__.smoke()
 *   and bench.py's cpu_baseline leg may load this library, and only as the
 *   checker / the timed CPU baseline.  The product (gamesmanmpi_amd/) never
 *   links or calls it.
 *
 * What it restates (swerwath/GamesmanMPI @ /root/reference):
 *   - the game modules' initial_position / gen_moves / do_move / primitive,
 *     written LITERALLY against the reference's own representations (raw
 *     MSB-first bitstrings for the bitstring games, the 3x3 int8 array for
 *     tic_tac_toe_np, the 9-char string for mttt, ints for Four-To-One), so
 *     board-layout quirks are reproduced rather than re-derived;
 *   - the solve itself (src/process.py:109-267): every reachable position is
 *     expanded once and resolved from its children with the
 *     REFERENCE-CANONICAL reduction of _res_red/_remote_red (SURVEY.md §8a
 *     rows A8/A9): value = WIN if any child LOSS, else TIE if any TIE, else
 *     DRAW if any DRAW, else LOSS; remoteness = 1 + min{rem(c): c LOSS} for
 *     WIN, otherwise 1 + max{rem(c)}; primitives have remoteness 0
 *     (src/process.py:122,243);
 *   - the md5 partition of GameState.get_hash (src/game_state.py:22-30) is
 *     restated in tests/ with hashlib (it is not arithmetic of ours).
 *
 * Parity pinning: checked against tests/golden/ (tables generated from the
 * reference's own game modules and root lines printed by the reference's own
 * job loop; see tests/golden/make_golden.py) by tests/test_oracle.py.
 *
 * The solver is a memoised, explicit-stack depth-first retrograde over an
 * open-addressing hash map -- the order-independent reading of the
 * reference's recursive LOOK_UP/DISTRIBUTE/RESOLVE protocol.  It is
 * deliberately scalar and simple (one core): it is the checker, not a
 * competitor.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define WIN 0
#define LOSS 1
#define TIE 2
#define DRAW 3
#define UNDECIDED 4 /* src/utils.py:3 */

#define OR_MAXCHILD 64
#define OR_BLOB 16

enum { G_FTO = 1, G_SUM, G_TTTNP, G_MTTT, G_TOOT, G_OTH };

typedef struct {
  uint8_t b[OR_BLOB];
} blob;

typedef struct {
  int kind;
  int length, height, area; /* bitstring games */
  int nbits, nbytes;         /* bitstring length after byte padding */
  int64_t fto_start;
  int nheaps;
  int heaps[16];
  int64_t strides[16];
} game;

static __thread char g_err[256];
const char *or_last_error(void) { return g_err; }

/* ------------------------------------------------------------------------ */
/* MSB-first bit access on the bitstring byte image                          */
/* ------------------------------------------------------------------------ */
static inline int bget(const uint8_t *b, int i) { return (b[i >> 3] >> (7 - (i & 7))) & 1; }
static inline void bset(uint8_t *b, int i, int v) {
  if (v)
    b[i >> 3] |= (uint8_t)(0x80 >> (i & 7));
  else
    b[i >> 3] &= (uint8_t)~(0x80 >> (i & 7));
}
/* board[a:a+w].int -- signed two's complement (bitstring .int) */
static int bint(const uint8_t *b, int a, int w) {
  int v = 0;
  for (int i = 0; i < w; i++) v = (v << 1) | bget(b, a + i);
  if (v & (1 << (w - 1))) v -= (1 << w);
  return v;
}
/* board[a:a+w] = v  (uint if v>=0 else int of width w) */
static void bput(uint8_t *b, int a, int w, int v) {
  unsigned u = (unsigned)v & ((1u << w) - 1);
  for (int i = 0; i < w; i++) bset(b, a + i, (u >> (w - 1 - i)) & 1);
}

/* ------------------------------------------------------------------------ */
/* Four-To-One: test_games/four_to_one.py:7-22                               */
/* ------------------------------------------------------------------------ */
static int64_t blob_i64(const blob *s) { int64_t v; memcpy(&v, s->b, 8); return v; }
static void i64_blob(blob *s, int64_t v) { memset(s, 0, sizeof *s); memcpy(s->b, &v, 8); }

static int fto_prim(const game *g, const blob *s) {
  (void)g;
  return blob_i64(s) <= 0 ? LOSS : UNDECIDED; /* four_to_one.py:19-22 */
}
static int fto_children(const game *g, const blob *s, blob *out) {
  (void)g;
  int64_t x = blob_i64(s);
  int n = 0;
  i64_blob(&out[n++], x - 1); /* gen_moves: [-1] at 1 else [-1,-2] (:10-14) */
  if (x != 1) i64_blob(&out[n++], x - 2);
  return n;
}

/* Sum of Four-To-One heaps: gamesmanmpi_amd/games/sum_four_to_one.py
 * (each heap follows four_to_one.py:10-14; primitive iff all heaps 0). */
static int sum_prim(const game *g, const blob *s) {
  (void)g;
  return blob_i64(s) == 0 ? LOSS : UNDECIDED;
}
static int sum_children(const game *g, const blob *s, blob *out) {
  int64_t r = blob_i64(s), rest = r;
  int n = 0;
  for (int i = 0; i < g->nheaps; i++) {
    int64_t h = rest % (g->heaps[i] + 1);
    rest /= (g->heaps[i] + 1);
    if (h >= 1) i64_blob(&out[n++], r - g->strides[i]);
    if (h >= 2) i64_blob(&out[n++], r - 2 * g->strides[i]);
  }
  return n;
}

/* ------------------------------------------------------------------------ */
/* tic_tac_toe_np: test_games/tic_tac_toe_np.py:7-61 (state[x][y] = b[3x+y]) */
/* ------------------------------------------------------------------------ */
static int tnp_conn(const uint8_t *st, int x, int y, int player, int dx, int dy, int left) {
  /* connectionTest (:43-48) */
  while (1) {
    if (left <= 0) return 1;
    if (x < 0 || x > 2 || y < 0 || y > 2 || st[3 * x + y] != player) return 0;
    x += dx; y += dy; left--;
  }
}
static int tnp_prim(const game *g, const blob *s) {
  (void)g;
  const uint8_t *st = s->b;
  int full = 1;
  for (int x = 0; x < 3; x++)
    for (int y = 0; y < 3; y++) {
      int p = st[3 * x + y];
      if (p != 0) {
        if (tnp_conn(st, x + 1, y, p, 1, 0, 2) || tnp_conn(st, x, y + 1, p, 0, 1, 2) ||
            tnp_conn(st, x + 1, y + 1, p, 1, 1, 2) || tnp_conn(st, x + 1, y - 1, p, 1, -1, 2))
          return LOSS; /* :50-56 */
      } else
        full = 0;
    }
  return full ? TIE : UNDECIDED; /* :57-61 */
}
static int tnp_children(const game *g, const blob *s, blob *out) {
  (void)g;
  int n1 = 0, n2 = 0, n = 0;
  for (int i = 0; i < 9; i++) { n1 += s->b[i] == 1; n2 += s->b[i] == 2; }
  int player = n1 > n2 ? 2 : 1; /* :13-25 */
  for (int x = 0; x < 3; x++)
    for (int y = 0; y < 3; y++)
      if (s->b[3 * x + y] == 0) { /* :27-31 row-major, x outer */
        out[n] = *s;
        out[n].b[3 * x + y] = (uint8_t)player; /* do_move :35-39 */
        n++;
      }
  return n;
}

/* ------------------------------------------------------------------------ */
/* mttt: test_games/mttt.py:11-127 (9-char string, index x + 3y)             */
/* ------------------------------------------------------------------------ */
static char mt_piece(const uint8_t *p, int x, int y) {
  if (x < 0 || x > 2 || y < 0 || y > 2) return 'B'; /* get_piece :33-37 */
  return (char)p[x + 3 * y];
}
static int mt_prim(const game *g, const blob *s) {
  (void)g;
  const uint8_t *p = s->b;
  int blank = 0;
  for (int i = 0; i < 9; i++) {
    if (p[i] == '_') { blank = 1; continue; }
    int x = i % 3, y = i / 3;
    char c = (char)p[i];
    if ((mt_piece(p, x + 1, y) == c && mt_piece(p, x + 2, y) == c) ||
        (mt_piece(p, x, y + 1) == c && mt_piece(p, x, y + 2) == c) ||
        (mt_piece(p, x + 1, y + 1) == c && mt_piece(p, x + 2, y + 2) == c) ||
        (mt_piece(p, x - 1, y + 1) == c && mt_piece(p, x - 2, y + 2) == c))
      return LOSS; /* :72-83 */
  }
  return blank ? UNDECIDED : TIE; /* :84-87 */
}
static int mt_children(const game *g, const blob *s, blob *out) {
  (void)g;
  int nx = 0, no = 0, n = 0;
  for (int i = 0; i < 9; i++) { nx += s->b[i] == 'X'; no += s->b[i] == 'O'; }
  char player = no >= nx ? 'X' : 'O'; /* get_player :39-43 */
  for (int i = 0; i < 9; i++)
    if (s->b[i] == '_') { out[n] = *s; out[n].b[i] = (uint8_t)player; n++; }
  return n;
}

/* ------------------------------------------------------------------------ */
/* Toot-and-Otto: test_games/toot_and_otto_bitstring.py                      */
/* ------------------------------------------------------------------------ */
#define T_ 1
#define O_ (-1)
#define BL 0
static int tt_get(const game *g, const uint8_t *b, int x, int y) { /* :179-185 */
  if (bget(b, g->length * y + x)) return T_;
  if (bget(b, g->area + g->length * y + x)) return O_;
  return BL;
}
static void tt_set(const game *g, uint8_t *b, int x, int y, int letter) { /* :188-199 */
  int ti = g->length * y + x, oi = g->area + g->length * y + x;
  bset(b, ti, letter == T_);
  bset(b, oi, letter == O_);
}
static int tt_p1turn(const game *g, const uint8_t *b) { return bget(b, g->nbits - 1); } /* :218-219 */
static int tt_hand_at(const game *g, int player, int letter) {
  return g->area * 2 + 8 * (player - 1) + (letter == T_ ? 0 : 4); /* :202-205 */
}
static int tt_full(const game *g, const uint8_t *b) { /* :224-227 */
  for (int i = 0; i < g->area; i++)
    if (!(bget(b, i) | bget(b, g->area + i))) return 0;
  return 1;
}
static int tt_word(const game *g, const uint8_t *b, int x, int y, const char *w, int dx, int dy) {
  for (int pos = 1; pos < 4; pos++, x += dx, y += dy) { /* word_test :70-77 */
    if (x < 0 || y < 0 || x >= g->length || y >= g->height) return 0;
    int c = tt_get(g, b, x, y);
    char ch = c == T_ ? 'T' : c == O_ ? 'O' : '-';
    if (ch != w[pos]) return 0;
  }
  return 1;
}
static int tt_prim(const game *g, const blob *s) { /* :46-85 */
  const uint8_t *b = s->b;
  int toot = 0, otto = 0;
  for (int x = 0; x < g->length; x++)
    for (int y = 0; y < g->height; y++) {
      int c = tt_get(g, b, x, y);
      if (c == BL) continue;
      const char *w = c == T_ ? "TOOT" : "OTTO";
      int *sc = c == T_ ? &toot : &otto;
      *sc += tt_word(g, b, x + 1, y, w, 1, 0);
      *sc += tt_word(g, b, x, y + 1, w, 0, 1);
      *sc += tt_word(g, b, x + 1, y + 1, w, 1, 1);
      *sc += tt_word(g, b, x + 1, y - 1, w, 1, -1);
    }
  if (otto == toot) return tt_full(g, b) ? TIE : UNDECIDED;
  if ((toot > otto) ^ tt_p1turn(g, b)) return LOSS;
  return WIN;
}
static int tt_children(const game *g, const blob *s, blob *out) { /* :87-115 */
  const uint8_t *b = s->b;
  int player = tt_p1turn(g, b) ? 1 : 2;
  int nT = bint(b, tt_hand_at(g, player, T_), 4);
  int nO = bint(b, tt_hand_at(g, player, O_), 4);
  int n = 0;
  for (int x = 0; x < g->length; x++) {
    if (tt_get(g, b, x, g->height - 1) != BL) continue;
    for (int k = 0; k < 2; k++) {
      int letter = k == 0 ? T_ : O_;
      if ((letter == T_ ? nT : nO) <= 0) continue;
      blob c = *s;
      int at = tt_hand_at(g, player, letter);
      bput(c.b, at, 4, bint(c.b, at, 4) - 1);           /* decr_hand_count */
      bset(c.b, g->nbits - 1, !bget(c.b, g->nbits - 1)); /* incr_turn */
      for (int y = 0; y < g->height; y++)
        if (tt_get(g, c.b, x, y) == BL) { tt_set(g, c.b, x, y, letter); break; }
      out[n++] = c;
    }
  }
  return n;
}
static void tt_root(const game *g, blob *s) { /* initial_position :36-44 */
  memset(s, 0, sizeof *s);
  for (int p = 0; p < 4; p++) bput(s->b, 2 * g->area + 4 * p, 4, 6);
  bset(s->b, 2 * g->area + 16, 1);
}

/* ------------------------------------------------------------------------ */
/* Othello: test_games/othello_bit_new.py (WHITE=2, BLACK=1)                 */
/* ------------------------------------------------------------------------ */
#define WHITE 2
#define BLACK 1
static int ot_get(const game *g, const uint8_t *b, int x, int y) { /* :251-257 */
  if (bget(b, g->length * y + x)) return WHITE;
  if (bget(b, g->area + g->length * y + x)) return BLACK;
  return 0;
}
static void ot_set(const game *g, uint8_t *b, int x, int y, int color) { /* :260-271 */
  int wi = g->length * y + x, bi = g->area + g->length * y + x;
  if (color == WHITE) { bset(b, wi, 1); bset(b, bi, 0); }
  else if (color == BLACK) { bset(b, bi, 1); bset(b, wi, 0); }
  else { bset(b, wi, 0); bset(b, bi, 0); }
}
static int ot_opp(int c) { return c == BLACK ? WHITE : c == WHITE ? BLACK : 0; }
static int ot_turncount(const game *g, const uint8_t *b) { return bint(b, 2 * g->area, 8); }
static int ot_cur(const game *g, const uint8_t *b) { return ot_turncount(g, b) == 1 ? BLACK : WHITE; }
static int ot_passes(const game *g, const uint8_t *b) { return bint(b, 2 * g->area + 8, 8); }
static void ot_incr_turn(const game *g, uint8_t *b) { /* :283-288 */
  bput(b, 2 * g->area, 8, ot_turncount(g, b) % 2 + 1);
}
static int ot_prim(const game *g, const blob *s) { /* :57-84 */
  const uint8_t *b = s->b;
  int nz = 0, bc = 0, wc = 0;
  for (int x = 0; x < g->length; x++)
    for (int y = 0; y < g->height; y++) {
      int c = ot_get(g, b, x, y);
      nz += c != 0; bc += c == BLACK; wc += c == WHITE;
    }
  if (nz == g->area || ot_passes(g, b) >= 2) {
    if (bc == wc) return TIE;
    if ((bc > wc) ^ (ot_turncount(g, b) == 1)) return LOSS;
    return WIN;
  }
  return UNDECIDED;
}
static int ot_legit_helper(const game *g, const uint8_t *b, int x, int y, int dx, int dy) {
  /* legit_helper :148-160, iterative */
  int opp = ot_opp(ot_cur(g, b));
  int first = 1;
  while (1) {
    if (x >= g->length || y >= g->height || x < 0 || y < 0) return 0;
    int c = ot_get(g, b, x, y);
    if (first) {
      if (c != opp) return 0;
      first = 0;
    } else {
      if (c == ot_cur(g, b)) return 1;
      if (c != opp) return 0;
    }
    x += dx; y += dy;
  }
}
static int ot_legit(const game *g, const uint8_t *b, int x, int y) { /* :134-146 */
  if (ot_get(g, b, x, y) != 0) return 0;
  for (int dx = -1; dx <= 1; dx++)
    for (int dy = -1; dy <= 1; dy++)
      if (!(dx == 0 && dy == 0) && ot_legit_helper(g, b, x + dx, y + dy, dx, dy)) return 1;
  return 0;
}
static void ot_flip_dir(const game *g, uint8_t *st, int x, int y, int dx, int dy) {
  /* flip_helper / flip_helper2 :100-118 (note the swapped bounds
   * `x >= height or y >= length`, kept verbatim) */
  if (x >= g->height || y >= g->length || x < 0 || y < 0) return;
  int cur = ot_cur(g, st);
  if (ot_get(g, st, x, y) != ot_opp(cur)) return;
  int fx[64], fy[64], nf = 0;
  fx[nf] = x; fy[nf] = y; nf++;
  x += dx; y += dy;
  while (1) {
    if (x >= g->height || y >= g->length || x < 0 || y < 0) return;
    int c = ot_get(g, st, x, y);
    if (c == cur) {
      for (int i = 0; i < nf; i++) ot_set(g, st, fx[i], fy[i], ot_opp(ot_get(g, st, fx[i], fy[i])));
      return;
    }
    if (c == ot_opp(cur)) { fx[nf] = x; fy[nf] = y; nf++; x += dx; y += dy; continue; }
    return;
  }
}
static int ot_children(const game *g, const blob *s, blob *out) { /* gen_moves :132-170 + do_move :86-130 */
  const uint8_t *b = s->b;
  int n = 0;
  for (int x = 0; x < g->length; x++)
    for (int y = 0; y < g->height; y++) {
      if (!ot_legit(g, b, x, y)) continue;
      blob c = *s;
      bput(c.b, 2 * g->area + 8, 8, 0);          /* reset_pass */
      ot_set(g, c.b, x, y, ot_cur(g, b));        /* flip_pieces: place */
      for (int dx = -1; dx <= 1; dx++)
        for (int dy = -1; dy <= 1; dy++)
          if (!(dx == 0 && dy == 0)) ot_flip_dir(g, c.b, x + dx, y + dy, dx, dy);
      ot_incr_turn(g, c.b);
      out[n++] = c;
    }
  if (n == 0) { /* [None] -> incr_pass only, turn NOT switched (:122-124) */
    blob c = *s;
    bput(c.b, 2 * g->area + 8, 8, ot_passes(g, c.b) + 1);
    out[n++] = c;
  }
  return n;
}
static void ot_root(const game *g, blob *s) { /* initial_position :36-55 */
  memset(s, 0, sizeof *s);
  /* the module passes float coordinates (length / 2 - 1) and board_set
   * indexes int(length * y + x) (:42-45, :260-262) */
  double hx = g->length / 2.0, hy = g->height / 2.0;
  const double px[4] = {hx - 1, hx - 1, hx, hx}, py[4] = {hy - 1, hy, hy - 1, hy};
  const int col[4] = {WHITE, BLACK, BLACK, WHITE};
  for (int i = 0; i < 4; i++) {
    int idx = (int)(g->length * py[i] + px[i]);
    bset(s->b, idx, col[i] == WHITE);
    bset(s->b, g->area + idx, col[i] == BLACK);
  }
  ot_incr_turn(g, s->b);
  ot_incr_turn(g, s->b);
}

/* ------------------------------------------------------------------------ */
/* Game registry                                                             */
/* ------------------------------------------------------------------------ */
#define MAXGAMES 64
static game g_games[MAXGAMES];
static int g_ngames;

static int parse_kv(const char *params, const char *key, int dflt) {
  if (!params) return dflt;
  const char *p = strstr(params, key);
  if (!p) return dflt;
  p += strlen(key);
  if (*p != '=') return dflt;
  return atoi(p + 1);
}

/* name: four_to_one | sum_four_to_one | tic_tac_toe_np | mttt |
 *       toot_and_otto_bitstring | othello_bit_new
 * params: "length=4,height=4" / "start=20" / "heaps=31:31:31" */
static char g_keys[MAXGAMES][256]; /* "name|params" of each registered game */

int or_game(const char *name, const char *params) {
  /* a game already described returns its handle: descriptors are immutable,
   * so a test process may ask for the same game any number of times */
  char key[256];
  snprintf(key, sizeof key, "%s|%s", name, params ? params : "");
  for (int i = 0; i < g_ngames; i++)
    if (!strcmp(g_keys[i], key)) return i;
  if (g_ngames >= MAXGAMES) { snprintf(g_err, sizeof g_err, "too many games"); return -1; }
  game g;
  memset(&g, 0, sizeof g);
  if (!strcmp(name, "four_to_one")) {
    g.kind = G_FTO;
    g.fto_start = parse_kv(params, "start", 4); /* four_to_one.py:7-8 */
  } else if (!strcmp(name, "sum_four_to_one")) {
    g.kind = G_SUM;
    const char *p = params ? strstr(params, "heaps=") : NULL;
    if (!p) { snprintf(g_err, sizeof g_err, "sum_four_to_one needs heaps="); return -1; }
    p += 6;
    int64_t stride = 1;
    while (*p && *p != ',') {
      if (g.nheaps >= 16) { snprintf(g_err, sizeof g_err, "too many heaps"); return -1; }
      g.heaps[g.nheaps] = atoi(p);
      g.strides[g.nheaps] = stride;
      stride *= g.heaps[g.nheaps] + 1;
      g.nheaps++;
      while (*p && *p != ':' && *p != ',') p++;
      if (*p == ':') p++;
    }
  } else if (!strcmp(name, "tic_tac_toe_np")) {
    g.kind = G_TTTNP;
  } else if (!strcmp(name, "mttt")) {
    g.kind = G_MTTT;
  } else if (!strcmp(name, "toot_and_otto_bitstring") || !strcmp(name, "othello_bit_new")) {
    int toot = name[0] == 't';
    g.kind = toot ? G_TOOT : G_OTH;
    g.length = parse_kv(params, "length", toot ? 6 : 8);
    g.height = parse_kv(params, "height", toot ? 4 : 8);
    g.area = g.length * g.height;
    int bits = toot ? 2 * g.area + 17 : 2 * g.area + 16;
    g.nbits = (bits + 7) / 8 * 8;
    g.nbytes = g.nbits / 8;
    if (g.nbytes > OR_BLOB) { snprintf(g_err, sizeof g_err, "board too large for the oracle"); return -1; }
  } else {
    snprintf(g_err, sizeof g_err, "unknown game '%s'", name);
    return -1;
  }
  g_games[g_ngames] = g;
  memcpy(g_keys[g_ngames], key, sizeof key);
  return g_ngames++;
}

static const game *G(int h) { return (h >= 0 && h < g_ngames) ? &g_games[h] : NULL; }

static int prim_of(const game *g, const blob *s) {
  switch (g->kind) {
    case G_FTO: return fto_prim(g, s);
    case G_SUM: return sum_prim(g, s);
    case G_TTTNP: return tnp_prim(g, s);
    case G_MTTT: return mt_prim(g, s);
    case G_TOOT: return tt_prim(g, s);
    default: return ot_prim(g, s);
  }
}
static int children_of(const game *g, const blob *s, blob *out) {
  switch (g->kind) {
    case G_FTO: return fto_children(g, s, out);
    case G_SUM: return sum_children(g, s, out);
    case G_TTTNP: return tnp_children(g, s, out);
    case G_MTTT: return mt_children(g, s, out);
    case G_TOOT: return tt_children(g, s, out);
    default: return ot_children(g, s, out);
  }
}
static void root_of(const game *g, blob *s) {
  memset(s, 0, sizeof *s);
  switch (g->kind) {
    case G_FTO: i64_blob(s, g->fto_start); break;
    case G_SUM: {
      int64_t r = 0;
      for (int i = 0; i < g->nheaps; i++) r += g->heaps[i] * g->strides[i];
      i64_blob(s, r);
      break;
    }
    case G_TTTNP: break;
    case G_MTTT: memset(s->b, '_', 9); break; /* mttt.py:11-12 */
    case G_TOOT: tt_root(g, s); break;
    default: ot_root(g, s);
  }
}

/* canonical bytes <-> blob.  Int games: ASCII decimal (str(pos)); others:
 * the raw byte image (latin-1 string bytes / ndarray.tobytes()). */
static int canon_len(const game *g) {
  switch (g->kind) {
    case G_TTTNP: case G_MTTT: return 9;
    case G_TOOT: case G_OTH: return g->nbytes;
    default: return -1;
  }
}
static int to_canon(const game *g, const blob *s, uint8_t *out) {
  int n = canon_len(g);
  if (n >= 0) { memcpy(out, s->b, (size_t)n); return n; }
  char tmp[32];
  int k = snprintf(tmp, sizeof tmp, "%lld", (long long)blob_i64(s));
  memcpy(out, tmp, (size_t)k);
  return k;
}
static int from_canon(const game *g, const uint8_t *in, int len, blob *s) {
  memset(s, 0, sizeof *s);
  int n = canon_len(g);
  if (n >= 0) {
    if (len != n) return -1;
    memcpy(s->b, in, (size_t)n);
    return 0;
  }
  if (len <= 0 || len > 20) return -1;
  char tmp[32];
  memcpy(tmp, in, (size_t)len);
  tmp[len] = 0;
  i64_blob(s, strtoll(tmp, NULL, 10));
  return 0;
}

int or_root(int h, uint8_t *canon, int *len) {
  const game *g = G(h);
  if (!g) return -1;
  blob s;
  root_of(g, &s);
  *len = to_canon(g, &s, canon);
  return 0;
}

/* primitive + ordered children of one position (gen_moves order).
 * children: nchild rows of 32 bytes, lens in clens. */
int or_expand(int h, const uint8_t *canon, int len, int *prim, uint8_t *children, int *clens, int *nchild) {
  const game *g = G(h);
  if (!g) return -1;
  blob s, ch[OR_MAXCHILD];
  if (from_canon(g, canon, len, &s)) { snprintf(g_err, sizeof g_err, "bad canonical bytes"); return -2; }
  *prim = prim_of(g, &s);
  *nchild = 0;
  if (*prim != UNDECIDED) return 0;
  int n = children_of(g, &s, ch);
  for (int i = 0; i < n; i++) clens[i] = to_canon(g, &ch[i], children + 32 * i);
  *nchild = n;
  return 0;
}

/* ------------------------------------------------------------------------ */
/* Solver: memoised explicit-stack DFS over an open-addressing map           */
/* ------------------------------------------------------------------------ */
typedef struct {
  blob key;
  uint32_t word; /* value | remoteness << 2 ; 0xFFFFFFFF = in progress */
  uint8_t used;
} slot;

typedef struct {
  int game;
  uint64_t cap, n, edges;
  slot *tab;
  uint32_t root_word;
} solve_t;

static uint64_t blob_hash(const blob *k) {
  uint64_t a, b;
  memcpy(&a, k->b, 8);
  memcpy(&b, k->b + 8, 8);
  uint64_t x = a * 0x9E3779B97F4A7C15ull ^ (b + 0x632BE59BD9B4E019ull);
  x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 29; x *= 0x94D049BB133111EBull; x ^= x >> 32;
  return x;
}

static slot *find_or_add(solve_t *S, const blob *k, int *added) {
  uint64_t m = S->cap - 1, i = blob_hash(k) & m;
  while (S->tab[i].used) {
    if (!memcmp(S->tab[i].key.b, k->b, OR_BLOB)) { *added = 0; return &S->tab[i]; }
    i = (i + 1) & m;
  }
  *added = 1;
  S->tab[i].used = 1;
  S->tab[i].key = *k;
  S->tab[i].word = 0xFFFFFFFFu;
  S->n++;
  return &S->tab[i];
}

typedef struct {
  blob s;
  slot *me;
  int nch, it;
  blob ch[OR_MAXCHILD];
} frame;

/* Returns a handle (or NULL); max_positions bounds the table. */
void *or_solve(int h, uint64_t max_positions) {
  const game *g = G(h);
  if (!g) { snprintf(g_err, sizeof g_err, "bad game handle"); return NULL; }
  solve_t *S = calloc(1, sizeof *S);
  S->game = h;
  S->cap = 1024;
  while (S->cap < 2 * max_positions) S->cap <<= 1;
  S->tab = calloc(S->cap, sizeof(slot));
  if (!S->tab) { free(S); snprintf(g_err, sizeof g_err, "oom"); return NULL; }
  size_t depth_cap = 1024, sp = 0;
  frame *st = malloc(depth_cap * sizeof(frame));
  blob root;
  root_of(g, &root);
  int added;
  st[sp].s = root;
  st[sp].me = find_or_add(S, &root, &added);
  st[sp].nch = -1;
  sp++;
  while (sp) {
    frame *f = &st[sp - 1];
    if (f->nch < 0) {
      int p = prim_of(g, &f->s);
      if (p != UNDECIDED) { f->me->word = (uint32_t)p; sp--; continue; } /* process.py:120-123 */
      f->nch = children_of(g, &f->s, f->ch);
      if (f->nch == 0) { snprintf(g_err, sizeof g_err, "non-primitive position with no moves"); goto fail; }
      S->edges += (uint64_t)f->nch;
      f->it = 0;
    }
    /* descend into the first unresolved child */
    while (f->it < f->nch) {
      slot *c = find_or_add(S, &f->ch[f->it], &added);
      if (S->n * 10 > S->cap * 9) { snprintf(g_err, sizeof g_err, "table full (raise max_positions)"); goto fail; }
      if (added) {
        if (sp == depth_cap) {
          depth_cap *= 2;
          st = realloc(st, depth_cap * sizeof(frame));
          f = &st[sp - 1];
        }
        st[sp].s = f->ch[f->it];
        st[sp].me = c;
        st[sp].nch = -1;
        sp++;
        break;
      }
      if (c->word == 0xFFFFFFFFu) { snprintf(g_err, sizeof g_err, "cycle in game graph"); goto fail; }
      f->it++;
    }
    if (f != &st[sp - 1]) continue; /* pushed a child */
    if (f->it < f->nch) continue;
    /* all children resolved: canonical reduction */
    int any_loss = 0, any_tie = 0, any_draw = 0;
    uint32_t min_loss = 0xFFFFFFFFu, max_all = 0;
    for (int i = 0; i < f->nch; i++) {
      slot *c = find_or_add(S, &f->ch[i], &added);
      uint32_t v = c->word & 3, r = c->word >> 2;
      if (v == LOSS) { any_loss = 1; if (r < min_loss) min_loss = r; }
      if (v == TIE) any_tie = 1;
      if (v == DRAW) any_draw = 1;
      if (r > max_all) max_all = r;
    }
    uint32_t v, r;
    if (any_loss) { v = WIN; r = min_loss + 1; }
    else { v = any_tie ? TIE : any_draw ? DRAW : LOSS; r = max_all + 1; }
    f->me->word = v | (r << 2);
    sp--;
  }
  free(st);
  {
    slot *rs = find_or_add(S, &root, &added);
    S->root_word = rs->word;
  }
  return S;
fail:
  free(st);
  free(S->tab);
  free(S);
  return NULL;
}

uint64_t or_count(void *hs) { return ((solve_t *)hs)->n; }
uint64_t or_edges(void *hs) { return ((solve_t *)hs)->edges; }
uint32_t or_root_word(void *hs) { return ((solve_t *)hs)->root_word; }

/* Dump every solved position: canon rows of `stride` bytes, lengths, value,
 * remoteness (table order; callers sort). */
int or_dump(void *hs, uint8_t *canon, int stride, uint8_t *clen, uint8_t *value, uint32_t *rem) {
  solve_t *S = hs;
  const game *g = G(S->game);
  uint64_t j = 0;
  uint8_t tmp[32];
  for (uint64_t i = 0; i < S->cap; i++) {
    if (!S->tab[i].used) continue;
    int n = to_canon(g, &S->tab[i].key, tmp);
    if (n > stride) return -1;
    memset(canon + j * (uint64_t)stride, 0, (size_t)stride);
    memcpy(canon + j * (uint64_t)stride, tmp, (size_t)n);
    clen[j] = (uint8_t)n;
    value[j] = (uint8_t)(S->tab[i].word & 3);
    rem[j] = S->tab[i].word >> 2;
    j++;
  }
  return 0;
}

/* Look up one position's word (or 0xFFFFFFFF if unknown). */
uint32_t or_lookup(void *hs, const uint8_t *canon, int len) {
  solve_t *S = hs;
  const game *g = G(S->game);
  blob k;
  if (from_canon(g, canon, len, &k)) return 0xFFFFFFFFu;
  uint64_t m = S->cap - 1, i = blob_hash(&k) & m;
  while (S->tab[i].used) {
    if (!memcmp(S->tab[i].key.b, k.b, OR_BLOB)) return S->tab[i].word;
    i = (i + 1) & m;
  }
  return 0xFFFFFFFFu;
}

void or_free(void *hs) {
  solve_t *S = hs;
  if (!S) return;
  free(S->tab);
  free(S);
}

/* multi-threaded restatements (same translation unit: reuses the game code) */
#include "oracle_mt.c"
