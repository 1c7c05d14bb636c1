// gm_md5.h -- single-block MD5 (RFC 1321) for the shard-owner rule of
// GameState.get_hash (src/game_state.py:22-30):
//   owner = int(md5(str(pos).encode('utf-8')).hexdigest(), 16) % world_size
// Every str(pos) the descriptors render is <= 55 bytes, so one 64-byte block
// suffices.  __host__ __device__: the K4 owner kernel and the host ABI share
// it.
#pragma once
#include <stdint.h>
#include "gm_games.h"

namespace gm {

GM_HD uint32_t md5_rotl(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }

// digest (16 bytes) of msg[0..len), len <= 55
GM_HD void md5_block(const uint8_t* msg, int len, uint8_t* digest) {
  const uint32_t K[64] = {
      0xd76aa478u, 0xe8c7b756u, 0x242070dbu, 0xc1bdceeeu, 0xf57c0fafu, 0x4787c62au, 0xa8304613u, 0xfd469501u,
      0x698098d8u, 0x8b44f7afu, 0xffff5bb1u, 0x895cd7beu, 0x6b901122u, 0xfd987193u, 0xa679438eu, 0x49b40821u,
      0xf61e2562u, 0xc040b340u, 0x265e5a51u, 0xe9b6c7aau, 0xd62f105du, 0x02441453u, 0xd8a1e681u, 0xe7d3fbc8u,
      0x21e1cde6u, 0xc33707d6u, 0xf4d50d87u, 0x455a14edu, 0xa9e3e905u, 0xfcefa3f8u, 0x676f02d9u, 0x8d2a4c8au,
      0xfffa3942u, 0x8771f681u, 0x6d9d6122u, 0xfde5380cu, 0xa4beea44u, 0x4bdecfa9u, 0xf6bb4b60u, 0xbebfbc70u,
      0x289b7ec6u, 0xeaa127fau, 0xd4ef3085u, 0x04881d05u, 0xd9d4d039u, 0xe6db99e5u, 0x1fa27cf8u, 0xc4ac5665u,
      0xf4292244u, 0x432aff97u, 0xab9423a7u, 0xfc93a039u, 0x655b59c3u, 0x8f0ccc92u, 0xffeff47du, 0x85845dd1u,
      0x6fa87e4fu, 0xfe2ce6e0u, 0xa3014314u, 0x4e0811a1u, 0xf7537e82u, 0xbd3af235u, 0x2ad7d2bbu, 0xeb86d391u};
  const int R[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};
  uint32_t M[16];
  for (int i = 0; i < 16; i++) M[i] = 0;
  for (int i = 0; i < len; i++) M[i >> 2] |= (uint32_t)msg[i] << (8 * (i & 3));
  M[len >> 2] |= 0x80u << (8 * (len & 3));
  M[14] = (uint32_t)len * 8u;
  uint32_t a = 0x67452301u, b = 0xefcdab89u, c = 0x98badcfeu, d = 0x10325476u;
  for (int i = 0; i < 64; i++) {
    uint32_t f;
    int g;
    if (i < 16) { f = (b & c) | (~b & d); g = i; }
    else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
    else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) & 15; }
    else { f = c ^ (b | ~d); g = (7 * i) & 15; }
    f = f + a + K[i] + M[g];
    a = d; d = c; c = b;
    b = b + md5_rotl(f, R[(i >> 4) * 4 + (i & 3)]);
  }
  uint32_t h[4] = {a + 0x67452301u, b + 0xefcdab89u, c + 0x98badcfeu, d + 0x10325476u};
  for (int i = 0; i < 16; i++) digest[i] = (uint8_t)(h[i >> 2] >> (8 * (i & 3)));
}

// int(hexdigest, 16) % P: the digest read as a big-endian 128-bit integer
GM_HD uint32_t md5_mod(const uint8_t* digest, uint32_t P) {
  uint64_t acc = 0;
  for (int i = 0; i < 16; i++) acc = ((acc << 8) | digest[i]) % P;
  return (uint32_t)acc;
}

}  // namespace gm
