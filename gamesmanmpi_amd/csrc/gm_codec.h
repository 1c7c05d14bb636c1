// gm_codec.h -- packed key <-> canonical bytes of the reference's positions.
//
// Canonical bytes (what the C-ABI's gm_encode/gm_decode exchange with the
// Python host):
//   four_to_one / sum_four_to_one : str(int) in ASCII         (four_to_one.py:7-8)
//   tic_tac_toe_np                : ndarray.tobytes(), 9 int8  (tic_tac_toe_np.py:7-8)
//   mttt                          : the 9-char string          (mttt.py:11-12)
//   toot_and_otto_bitstring       : latin-1 bytes of the MSB-first bitstring
//                                   (board_to_bytes, toot_and_otto_bitstring.py:229-236)
//   othello_bit_new               : same (othello_bit_new.py:241-248)
// __host__ __device__ so the owner kernel can render str(pos) on device.
#pragma once
#include "gm_games.h"

namespace gm {

GM_HD int cb_get(const uint8_t* b, int i) { return (b[i >> 3] >> (7 - (i & 7))) & 1; }
GM_HD void cb_set(uint8_t* b, int i) { b[i >> 3] |= (uint8_t)(0x80 >> (i & 7)); }
GM_HD uint32_t cb_field(const uint8_t* b, int at, int w) {
  uint32_t v = 0;
  for (int i = 0; i < w; i++) v = (v << 1) | (uint32_t)cb_get(b, at + i);
  return v;
}
GM_HD void cb_put(uint8_t* b, int at, int w, uint32_t v) {
  for (int i = 0; i < w; i++)
    if ((v >> (w - 1 - i)) & 1) cb_set(b, at + i);
}

// key -> bitstring bytes (toot/othello); returns byte count
GM_HD int bits_from_key(const Desc& d, uint64_t k, uint8_t* out) {
  const int A = d.A, nb = d.nbits / 8;
  for (int i = 0; i < nb; i++) out[i] = 0;
  for (int i = 0; i < 2 * A; i++)
    if ((k >> i) & 1) cb_set(out, i);
  if (d.kind == K_TOOT) {
    for (int j = 0; j < 4; j++) cb_put(out, 2 * A + 4 * j, 4, (uint32_t)((k >> (2 * A + 3 * j)) & 7));
    cb_set(out, 2 * A + 16);                             // constant '0b1' (:41)
    if ((k >> (2 * A + 12)) & 1) cb_set(out, d.nbits - 1);  // turn = board[-1]
  } else {
    cb_put(out, 2 * A, 8, ((k >> (2 * A)) & 1) ? 1u : 2u);         // turn_count
    cb_put(out, 2 * A + 8, 8, (uint32_t)((k >> (2 * A + 1)) & 3));  // pass_count
  }
  return nb;
}

// bitstring bytes -> key; returns 0 or -1 when the bytes are not a state
// the descriptor can represent
GM_HD int key_from_bits(const Desc& d, const uint8_t* b, int n, uint64_t* key) {
  const int A = d.A;
  if (n != d.nbits / 8) return -1;
  uint64_t k = 0;
  for (int i = 0; i < A; i++) {
    int p = cb_get(b, i), q = cb_get(b, A + i);
    if (p && q) return -1;  // a cell cannot hold both letters/colours
    k |= (uint64_t)p << i;
    k |= (uint64_t)q << (A + i);
  }
  if (d.kind == K_TOOT) {
    for (int j = 0; j < 4; j++) {
      uint32_t v = cb_field(b, 2 * A + 4 * j, 4);
      if (v > 7) return -1;  // negative (signed .int) or > 7 hands
      k |= (uint64_t)v << (2 * A + 3 * j);
    }
    if (!cb_get(b, 2 * A + 16)) return -1;
    for (int i = 2 * A + 17; i < d.nbits - 1; i++)
      if (cb_get(b, i)) return -1;
    k |= (uint64_t)cb_get(b, d.nbits - 1) << (2 * A + 12);
  } else {
    uint32_t turn = cb_field(b, 2 * A, 8), pass = cb_field(b, 2 * A + 8, 8);
    if (turn != 1 && turn != 2) return -1;
    if (pass > 3) return -1;
    for (int i = 2 * A + 16; i < d.nbits; i++)
      if (cb_get(b, i)) return -1;
    k |= (uint64_t)(turn == 1) << (2 * A);
    k |= (uint64_t)pass << (2 * A + 1);
  }
  *key = k;
  return 0;
}

// key -> canonical bytes; returns the length
GM_HD int canon_from_key(const Desc& d, uint64_t k, uint8_t* out) {
  if (d.kind == K_TOOT || d.kind == K_OTHELLO) return bits_from_key(d, k, out);
  if (d.kind == K_TTT) {
    for (int c = 0; c < 9; c++) {
      uint32_t v = (uint32_t)((k >> (2 * c)) & 3);
      out[c] = d.variant == 1 ? (uint8_t)(v == 0 ? '_' : v == 1 ? 'X' : 'O') : (uint8_t)v;
    }
    return 9;
  }
  char tmp[24];
  int m = 0, n = 0;
  do { tmp[m++] = (char)('0' + k % 10); k /= 10; } while (k);
  while (m) out[n++] = (uint8_t)tmp[--m];
  return n;
}

// str(pos).encode('utf-8'); returns the length (<= 55)
GM_HD int str_utf8_from_key(const Desc& d, uint64_t k, uint8_t* out) {
  if (d.kind == K_TOOT || d.kind == K_OTHELLO) {
    uint8_t raw[16];
    int nb = bits_from_key(d, k, raw), n = 0;
    for (int i = 0; i < nb; i++) {  // latin-1 str -> UTF-8
      if (raw[i] < 0x80) out[n++] = raw[i];
      else { out[n++] = (uint8_t)(0xC0 | (raw[i] >> 6)); out[n++] = (uint8_t)(0x80 | (raw[i] & 0x3F)); }
    }
    return n;
  }
  if (d.kind == K_TTT && d.variant == 1) return canon_from_key(d, k, out);
  if (d.kind == K_TTT) {  // numpy str() of a 3x3 int8 array
    int n = 0;
    for (int r = 0; r < 3; r++) {
      out[n++] = r == 0 ? '[' : ' ';
      out[n++] = '[';
      for (int c = 0; c < 3; c++) {
        if (c) out[n++] = ' ';
        out[n++] = (uint8_t)('0' + ((k >> (2 * (3 * r + c))) & 3));
      }
      out[n++] = ']';
      if (r < 2) out[n++] = '\n';
    }
    out[n++] = ']';
    return n;
  }
  return canon_from_key(d, k, out);  // str(int)
}

// Order-independent fingerprint of one solved position: FNV-1a over its
// canonical bytes, then a mix with its value and remoteness.  A solve's
// checksum is the sum (mod 2^64) over every reachable position, so it is
// independent of storage order, layout and sharding (shards add up), and
// equal to oracle/oracle_mt.c's ck_term sum over the same positions.
GM_HD uint64_t pos_checksum(const uint8_t* c, int n, uint32_t value, uint32_t rem) {
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

}  // namespace gm
