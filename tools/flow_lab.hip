// flow_lab.hip -- measurement harness: the PLANES backward (one GPU, 8-bit
// words, sum_four_to_one heaps 31^K) as ONE persistent launch in which every
// wave waits for its planes' neighbours by per-plane ready flags, against the
// product's one launch per plane level.  Diagnostic tool, not product code.
//
// Why: the level-synchronous backward pays a dependent kernel boundary per
// level (~1.5-1.9 us + the level's dirty bytes / 6 TB/s, MI355X_MICROARCH.md
// "boundary") and every level waits for its slowest wave.  Here a plane
// starts as soon as its 2 (K - 2) neighbour planes are final.
//
// Protocol (cdna_hip_programming.md Guideline 16, R1 with sc1 loads): a wave
// stores its four planes' rows WRITE-THROUGH (buffer store, aux sc1), drains
// (s_waitcnt vmcnt(0)), then lanes 0/1/32/33 store the planes' flags with
// relaxed agent-scope atomic stores; a consumer wave polls the flags of all
// neighbours (one lane per flag, relaxed agent loads, s_sleep between passes,
// bounded: a give-up word), then reads the neighbour rows with sc1 buffer
// loads (variant 1) or sc0|sc1 loads (variant 2).  Flags are zeroed before
// every launch; the table is poisoned (0xAA) before every timed run so a
// stale read shows as a mismatch.
//
// Work assignment: static, grid = resident capacity (census below), wave w
// takes items w, w + W, w + 2W, ... of a level-ordered item sequence (4
// planes per item); every item depends only on items earlier in the
// sequence, and every wave is resident, so the wave holding the lowest
// unfinished item can always proceed.  Within each level the items are dealt
// so each XCD's waves get one contiguous chunk of the level (the product's
// plane_share locality).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/flow_lab.hip -o tools/flow_lab
//   ./tools/flow_lab K variant [reps] [blocks_per_cu]
// variants: 0 product launches (k_plane_resolve_x2, per level); 1 flow, sc1
// loads; 2 flow, sc0|sc1 loads; 3 flow, plain loads behind an agent acquire;
// 9 flow, plain buffer loads and NO acquire (round 6: a line is first read
// only after its plane's flag is set, so no L1/L2 can hold a stale copy of it
// -- checked empirically on the poisoned table, every rep)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../gamesmanmpi_amd/csrc/gm_plane.h"
using namespace gm;

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

typedef __attribute__((address_space(1))) uint32_t gu32;
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kSpinLimit = 1u << 21;  // passes of ~0.1 us: a stuck wave gives up after ~0.2 s

// ST: 1 write-through (sc1) stores; 0 plain stores (timing only: not a
// valid hand-off).  TR: s_memtime stamps of each wave's first 16 items.
// LEVEL: one launch per plane level instead (items = the level's planes in
// groups of 4, dealt by plane_share as the product does; no flags).
template <int NO, int LD, int ST = 1, bool TR = false, bool LEVEL = false>
__global__ __launch_bounds__(256) void k_flow(uint8_t* __restrict__ tab, const uint32_t* __restrict__ items,
                                              uint32_t nitems, uint32_t W, uint32_t* __restrict__ flags,
                                              uint32_t* __restrict__ tmo, PlaneGeom g, const uint4* __restrict__ zero,
                                              uint32_t tabbytes, uint64_t* __restrict__ stamps = nullptr) {
  uint32_t nit = 0;
  uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
  const uint32_t lane = threadIdx.x & 63, L = lane & 31;
  const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(tab, 0, tabbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rz = __builtin_amdgcn_make_buffer_rsrc((void*)zero, 0, 4096, 0x00020000);
  constexpr int AUX = LD == 1 ? 16 : LD == 2 ? 17 : 0;
  const PlaneShare shr = plane_share(nitems, 1);
  for (uint32_t it = LEVEL ? shr.first : w; it < (LEVEL ? shr.end : nitems); it += LEVEL ? shr.stride : W, nit++) {
    if (TR) t0 = __builtin_amdgcn_s_memtime();
    const uint32_t* ip = items + (size_t)it * 4;
    // the wave's four planes: [X0, Y0] on lanes 0-31, [X1, Y1] on 32-63
    const uint32_t px = ip[2 * (lane >> 5)], py = ip[2 * (lane >> 5) + 1];
    const bool livex = px != kNone, livey = py != kNone;
    // dependency wait: lane l < 8 NO polls neighbour (l % (2 NO)) of plane l / (2 NO)
    if constexpr (!LEVEL) {
      uint32_t nbp = kNone;
      if (lane < 8 * NO) {
        const uint32_t pq = ip[lane / (2 * NO)], n = lane % (2 * NO), j = n >> 1, k = (n & 1) + 1;
        if (pq != kNone) {
          const uint32_t dj = (pq >> g.shift[j]) & (g.base[j] - 1u);
          if (dj >= k) nbp = pq - k * g.stride[j];
        }
      }
      bool ok = nbp == kNone;
      for (uint32_t spins = 0;; spins++) {
        if (!ok) ok = __hip_atomic_load((gu32*)(flags + nbp), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
        if (__all(ok)) break;
        if (spins >= kSpinLimit || __hip_atomic_load((gu32*)tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          if (lane == 0) __hip_atomic_store((gu32*)tmo, 1u + it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          return;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      if (LD == 3) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
    if (TR) t1 = __builtin_amdgcn_s_memtime();
    uint32_t dx[NO], dy[NO];
    plane_digits<NO>(g, livex ? px : 0u, dx);
    plane_digits<NO>(g, livey ? py : 0u, dy);
    const uint32_t ox = (livex ? px : 0u) * 1024u + L * 32u, oy = (livey ? py : 0u) * 1024u + L * 32u;
    uint32_t Xh[8], Xl[8], Yh[8], Yl[8];
#pragma unroll
    for (int d = 0; d < 8; d++) Xh[d] = Yh[d] = Xl[d] = Yl[d] = 0;
#pragma unroll
    for (int j = 0; j < NO; j++) {
#pragma unroll
      for (int k = 1; k <= 2; k++) {
        const bool hx = livex && dx[j] >= (uint32_t)k, hy = livey && dy[j] >= (uint32_t)k;
        const uint32_t sx = hx ? ox - k * g.stride[j] * 1024u : 0u, sy = hy ? oy - k * g.stride[j] * 1024u : 0u;
        uint4 vx[2], vy[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
          if (LD == 3) {
            vx[q] = hx ? *(const uint4*)(tab + sx + 16 * q) : make_uint4(0, 0, 0, 0);
            vy[q] = hy ? *(const uint4*)(tab + sy + 16 * q) : make_uint4(0, 0, 0, 0);
          } else {
            const __amdgpu_buffer_rsrc_t r1 = hx ? rt : rz, r2 = hy ? rt : rz;
            const auto a = __builtin_amdgcn_raw_buffer_load_b128(r1, hx ? sx + 16 * q : 0u, 0, AUX);
            const auto b = __builtin_amdgcn_raw_buffer_load_b128(r2, hy ? sy + 16 * q : 0u, 0, AUX);
            vx[q] = make_uint4(a[0], a[1], a[2], a[3]);
            vy[q] = make_uint4(b[0], b[1], b[2], b[3]);
          }
        }
#pragma unroll
        for (int q = 0; q < 2; q++) {
          const uint32_t a[4] = {vx[q].x, vx[q].y, vx[q].z, vx[q].w};
          const uint32_t b[4] = {vy[q].x, vy[q].y, vy[q].z, vy[q].w};
#pragma unroll
          for (int c = 0; c < 4; c++) {
            Xh[4 * q + c] = pk_max16(Xh[4 * q + c], a[c]);
            Yh[4 * q + c] = pk_max16(Yh[4 * q + c], b[c]);
            Xl[4 * q + c] = pk_max16(Xl[4 * q + c], pk_shl8(a[c]));
            Yl[4 * q + c] = pk_max16(Yl[4 * q + c], pk_shl8(b[c]));
          }
        }
      }
    }
    if (TR) t2 = __builtin_amdgcn_s_memtime() + (Xh[0] & Yl[7] & 0 ? 1 : 0);
    const uint32_t primv = L == 0 ? ((px == 0 ? 0xFFu : 0u) | (py == 0 ? 0xFFu << 16 : 0u)) : 0u;
    uint32_t cur = 0, prev = 0, u1p = 0;
    uint32_t op[32];
#pragma unroll
    for (int q = 0; q < 32; q++) op[q] = 0;
    const uint32_t A0 = ~0u << L;
#pragma unroll 1
    for (uint32_t ph = 0; ph < 2; ph++) {
      const uint32_t A = ph ? ~A0 : A0;
#pragma unroll
      for (int q = 0; q < 32; q++) {
        const int d = q >> 2, b = q & 3;
        const uint32_t bx = (b & 1) ? (uint32_t)b : (uint32_t)b + 1;
        const uint32_t sel = 0x0C000C00u | ((4u + bx) << 16) | bx;
        const uint32_t a = (b & 1) ? perm(Yh[d], Xh[d], sel) : perm(Yl[d], Xl[d], sel);
        const uint32_t u2r = from_lane_below(u1p);
        const uint32_t pre = pk_max16(pk_max16(a, prev), u2r);
        const uint32_t u1r = from_lane_below(cur);
        const uint32_t m = pk_max16(pk_max16(pre, cur), u1r);
        const uint32_t keep = (uint32_t)__builtin_amdgcn_sbfe((int)A, q, 1);
        uint32_t f = parent_x2<1>(m) & keep;
        if (q == 0) f = pk_max16(f, ph ? 0u : primv);
        op[q] |= f;
        prev = cur;
        cur = f;
        u1p = u1r;
      }
    }
    uint32_t ox_[8], oy_[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t t1 = perm(op[4 * k + 1], op[4 * k], 0x06020400u);
      const uint32_t t2 = perm(op[4 * k + 3], op[4 * k + 2], 0x06020400u);
      ox_[k] = perm(t2, t1, 0x05040100u);
      oy_[k] = perm(t2, t1, 0x07060302u);
    }
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    if (TR) t3 = __builtin_amdgcn_s_memtime() + (ox_[0] & oy_[7] & 0 ? 1 : 0);
    constexpr int SAUX = ST == 1 ? 16 : ST == 2 ? 2 : 0;
    if (livex) {
      __builtin_amdgcn_raw_buffer_store_b128((v4u){ox_[0], ox_[1], ox_[2], ox_[3]}, rt, ox, 0, SAUX);
      __builtin_amdgcn_raw_buffer_store_b128((v4u){ox_[4], ox_[5], ox_[6], ox_[7]}, rt, ox + 16, 0, SAUX);
    }
    if (livey) {
      __builtin_amdgcn_raw_buffer_store_b128((v4u){oy_[0], oy_[1], oy_[2], oy_[3]}, rt, oy, 0, SAUX);
      __builtin_amdgcn_raw_buffer_store_b128((v4u){oy_[4], oy_[5], oy_[6], oy_[7]}, rt, oy + 16, 0, SAUX);
    }
    if (LEVEL) continue;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every lane's rows written through before any flag
    if (TR && nit < 16 && lane == 0) {
      const uint64_t t4 = __builtin_amdgcn_s_memtime();
      uint64_t* o = stamps + ((size_t)w * 16 + nit) * 5;
      o[0] = t0;
      o[1] = t1;
      o[2] = t2;
      o[3] = t3;
      o[4] = t4;
    }
    if ((lane & 31) < 2) {
      const uint32_t p = (lane & 1) ? py : px;
      if (p != kNone) __hip_atomic_store((gu32*)(flags + p), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? atoi(argv[1]) : 6;
  const int var = argc > 2 ? atoi(argv[2]) : 1;
  const int reps = argc > 3 ? atoi(argv[3]) : 10;
  const int bpc = argc > 4 ? atoi(argv[4]) : 0;
  if (K < 3 || K > 6) {
    fprintf(stderr, "K in [3, 6]\n");
    return 1;
  }
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  PlaneGeom g{};
  g.no = K - 2;
  g.pow2 = 1;
  g.world = 1;
  uint64_t np = 1;
  for (int j = 0; j < K - 2; j++) {
    g.base[j] = 32;
    g.stride[j] = (uint32_t)np;
    g.shift[j] = __builtin_ctzll(np);
    np *= 32;
  }
  g.nplanes = (uint32_t)np;
  const int S = 31 * (K - 2);
  auto osum = [&](uint64_t P) {
    int s = 0;
    for (int j = 0; j < K - 2; j++) s += (int)((P >> (5 * j)) & 31);
    return s;
  };
  // level lists in the product's tile order (8^3 tiles over the digits above the lowest)
  std::vector<std::vector<uint32_t>> lev(S + 1);
  for (uint64_t P = 0; P < np; P++) lev[osum(P)].push_back((uint32_t)P);
  auto key = [&](uint32_t P) {
    uint64_t k = 0;
    for (int j = K - 3; j >= 1; j--) k = k * 64 + ((P >> (5 * j)) & 31) / 8;
    for (int j = K - 3; j >= 1; j--) k = k * 64 + ((P >> (5 * j)) & 31) % 8;
    return k * 64 + (P & 31);
  };
  for (auto& v : lev) std::sort(v.begin(), v.end(), [&](uint32_t a, uint32_t b) { return key(a) < key(b); });
  // the grid: resident capacity (occupancy API, capped by the SGPR rule of
  // MI355X_MICROARCH.md "Residency"), or blocks_per_cu from the command line
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_flow<4, 1>, 256, 0));
  const int per_cu = bpc > 0 ? bpc : std::max(1, occ - 1);
  const uint32_t blocks = (uint32_t)(cus * per_cu), W = blocks * 4;
  // item sequence: per level, groups of 4 planes; position m belongs to wave
  // m % W, whose block (m % W) / 4 sits on XCD ((m % W) / 4) % 8; each XCD's
  // positions in the level take one contiguous chunk of the level's groups
  std::vector<uint32_t> items;
  uint64_t pos = 0;
  for (int s = 0; s <= S; s++) {
    std::vector<uint32_t>& v = lev[s];
    while (v.size() % 4) v.push_back(kNone);
    const uint64_t ng = v.size() / 4;
    std::vector<std::vector<uint64_t>> xpos(8);
    for (uint64_t m = pos; m < pos + ng; m++) xpos[((m % W) / 4) % 8].push_back(m);
    items.resize((pos + ng) * 4, kNone);
    uint64_t gi = 0;
    for (int x = 0; x < 8; x++)
      for (uint64_t m : xpos[x]) {
        for (int c = 0; c < 4; c++) items[m * 4 + c] = v[gi * 4 + c];
        gi++;
      }
    pos += ng;
  }
  const uint32_t nitems = (uint32_t)pos;
  std::vector<uint32_t> flat_list, off(S + 2, 0);
  for (int s = 0; s <= S; s++) {
    off[s + 1] = off[s] + (uint32_t)lev[s].size();
    for (uint32_t P : lev[s]) flat_list.push_back(P);
  }
  const size_t tbytes = np * 1024;
  uint8_t* tab;
  void* zero;
  uint32_t *dlist, *ditems, *flags, *tmo;
  CK(hipMalloc(&tab, tbytes));
  CK(hipMalloc(&zero, 4096));
  CK(hipMemset(zero, 0, 4096));
  CK(hipMalloc(&dlist, flat_list.size() * 4));
  CK(hipMemcpy(dlist, flat_list.data(), flat_list.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&ditems, items.size() * 4));
  CK(hipMemcpy(ditems, items.data(), items.size() * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&flags, np * 4 + 256));
  tmo = flags + np;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  uint64_t* dstamps = nullptr;
  CK(hipMalloc(&dstamps, (size_t)W * 16 * 5 * 8));
  CK(hipMemset(dstamps, 0, (size_t)W * 16 * 5 * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // the reference: the product kernel, one launch per level (padded sentinels skipped: real planes only)
  auto run_levels = [&]() {
    for (int s = 0; s <= S; s++) {
      uint32_t n = 0;
      for (uint32_t i = off[s]; i < off[s + 1]; i++) n += flat_list[i] != kNone;
      const uint32_t waves = (n + 3) / 4;
      uint32_t b = (waves + 3) / 4;
      b = std::min<uint32_t>((b + 7) / 8 * 8, (uint32_t)cus * 32);
      const uint32_t* l = dlist + off[s];
      switch (K) {
        case 3: hipLaunchKernelGGL((k_plane_resolve_x2<1, 1, false, 0>), dim3(b), dim3(256), 0, st, tab, (const void*)l, n, g, (const uint4*)zero, (const uint8_t*)nullptr, (uint8_t*)nullptr, (const uint32_t*)nullptr, 0u); break;
        case 4: hipLaunchKernelGGL((k_plane_resolve_x2<1, 2, false, 0>), dim3(b), dim3(256), 0, st, tab, (const void*)l, n, g, (const uint4*)zero, (const uint8_t*)nullptr, (uint8_t*)nullptr, (const uint32_t*)nullptr, 0u); break;
        case 5: hipLaunchKernelGGL((k_plane_resolve_x2<1, 3, false, 0>), dim3(b), dim3(256), 0, st, tab, (const void*)l, n, g, (const uint4*)zero, (const uint8_t*)nullptr, (uint8_t*)nullptr, (const uint32_t*)nullptr, 0u); break;
        default: hipLaunchKernelGGL((k_plane_resolve_x2<1, 4, false, 0>), dim3(b), dim3(256), 0, st, tab, (const void*)l, n, g, (const uint4*)zero, (const uint8_t*)nullptr, (uint8_t*)nullptr, (const uint32_t*)nullptr, 0u); break;
      }
    }
  };
  auto run_level_lab = [&](int v) {  // per-level launches of the lab body: 6 plain, 7 sc1, 8 nt stores
    for (int s = 0; s <= S; s++) {
      const uint32_t ng = (off[s + 1] - off[s]) / 4;
      uint32_t b = (ng + 3) / 4;
      b = std::min<uint32_t>((b + 7) / 8 * 8, (uint32_t)cus * 32);
      const uint32_t* l = dlist + off[s];
      auto go = [&](auto NOc) {
        constexpr int NO = decltype(NOc)::value;
        if (v == 6) hipLaunchKernelGGL((k_flow<NO, 3, 0, false, true>), dim3(b), dim3(256), 0, st, tab, l, ng, 0u, flags, tmo, g, (const uint4*)zero, (uint32_t)tbytes, (uint64_t*)nullptr);
        else if (v == 7) hipLaunchKernelGGL((k_flow<NO, 3, 1, false, true>), dim3(b), dim3(256), 0, st, tab, l, ng, 0u, flags, tmo, g, (const uint4*)zero, (uint32_t)tbytes, (uint64_t*)nullptr);
        else hipLaunchKernelGGL((k_flow<NO, 3, 2, false, true>), dim3(b), dim3(256), 0, st, tab, l, ng, 0u, flags, tmo, g, (const uint4*)zero, (uint32_t)tbytes, (uint64_t*)nullptr);
      };
      switch (K) {
        case 3: go(std::integral_constant<int, 1>()); break;
        case 4: go(std::integral_constant<int, 2>()); break;
        case 5: go(std::integral_constant<int, 3>()); break;
        default: go(std::integral_constant<int, 4>()); break;
      }
    }
  };
  auto run_flow = [&](int v) {
    CK(hipMemsetAsync(flags, 0, np * 4 + 256, st));
    auto go = [&](auto NOc) {
      constexpr int NO = decltype(NOc)::value;
      if (v == 1) hipLaunchKernelGGL((k_flow<NO, 1>), dim3(blocks), dim3(256), 0, st, tab, ditems, nitems, W, flags, tmo, g, (const uint4*)zero, (uint32_t)tbytes, (uint64_t*)nullptr);
      else if (v == 4) hipLaunchKernelGGL((k_flow<NO, 1, 0>), dim3(blocks), dim3(256), 0, st, tab, ditems, nitems, W, flags, tmo, g, (const uint4*)zero, (uint32_t)tbytes, (uint64_t*)nullptr);
      else if (v == 5) hipLaunchKernelGGL((k_flow<NO, 1, 1, true>), dim3(blocks), dim3(256), 0, st, tab, ditems, nitems, W, flags, tmo, g, (const uint4*)zero, (uint32_t)tbytes, dstamps);
      else if (v == 9) hipLaunchKernelGGL((k_flow<NO, 0>), dim3(blocks), dim3(256), 0, st, tab, ditems, nitems, W, flags, tmo, g, (const uint4*)zero, (uint32_t)tbytes, (uint64_t*)nullptr);
      else if (v == 2) hipLaunchKernelGGL((k_flow<NO, 2>), dim3(blocks), dim3(256), 0, st, tab, ditems, nitems, W, flags, tmo, g, (const uint4*)zero, (uint32_t)tbytes, (uint64_t*)nullptr);
      else hipLaunchKernelGGL((k_flow<NO, 3>), dim3(blocks), dim3(256), 0, st, tab, ditems, nitems, W, flags, tmo, g, (const uint4*)zero, (uint32_t)tbytes, (uint64_t*)nullptr);
    };
    switch (K) {
      case 3: go(std::integral_constant<int, 1>()); break;
      case 4: go(std::integral_constant<int, 2>()); break;
      case 5: go(std::integral_constant<int, 3>()); break;
      default: go(std::integral_constant<int, 4>()); break;
    }
  };
  printf("flow_lab K=%d var %d: %llu planes, %d levels, %u items, grid %u blocks (%d per CU, occupancy API %d), %u waves\n", K,
         var, (unsigned long long)np, S + 1, nitems, blocks, per_cu, occ, W);
  fflush(stdout);
  // the byte reference: the product's launches for var 0, the lab body's own
  // per-level launches (var 7) otherwise -- the lab body keeps the round-4
  // contiguous-row layout, the product the round-5 16-B pieces
  if (var == 0) run_levels();
  else run_level_lab(7);
  CK(hipStreamSynchronize(st));
  std::vector<uint8_t> ref(tbytes), got(tbytes);
  CK(hipMemcpy(ref.data(), tab, tbytes, hipMemcpyDeviceToHost));
  std::vector<float> ts;
  for (int r = 0; r <= reps; r++) {  // r = 0: warm-up
    CK(hipMemsetAsync(tab, 0xAA, tbytes, st));  // poison: a stale read shows
    if (var == 0) {
      CK(hipEventRecord(e0, st));
      run_levels();
    } else if (var >= 6 && var != 9) {
      CK(hipEventRecord(e0, st));
      run_level_lab(var);
    } else {
      CK(hipMemsetAsync(flags, 0, np * 4 + 256, st));
      CK(hipEventRecord(e0, st));
      run_flow(var);
    }
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r) ts.push_back(ms);
    if (var != 0 && (var < 6 || var == 9)) {
      uint32_t t = 0;
      CK(hipMemcpy(&t, tmo, 4, hipMemcpyDeviceToHost));
      if (t) {
        printf("GAVE UP: a wave timed out waiting (item %u)\n", t - 1);
        return 3;
      }
    }
    CK(hipMemcpy(got.data(), tab, tbytes, hipMemcpyDeviceToHost));
    size_t bad = 0, first = 0;
    for (size_t i = 0; i < tbytes; i++)
      if (got[i] != ref[i]) {
        if (!bad) first = i;
        bad++;
      }
    if (bad) {
      printf("rep %d: %zu differing bytes, first at %zu (plane %zu): got %02x want %02x MISMATCH%s\n", r, bad, first,
             first / 1024, got[first], ref[first], var == 4 ? " (expected: plain stores are no hand-off)" : "");
      if (var != 4) return 2;
    }
  }
  if (var == 5) {  // per-item phases (cycles of the wave's XCD clock): wait, load+fold, wavefront, store+drain, gap to the next item
    std::vector<uint64_t> h((size_t)W * 16 * 5);
    CK(hipMemcpy(h.data(), dstamps, h.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> ph[5];
    for (uint32_t w = 0; w < W; w++)
      for (int n = 0; n < 16; n++) {
        const uint64_t* o = &h[((size_t)w * 16 + n) * 5];
        if (!o[4]) continue;
        for (int k = 0; k < 4; k++) ph[k].push_back((double)(o[k + 1] - o[k]));
        const uint64_t* nx = o + 5;
        if (n + 1 < 16 && nx[4]) ph[4].push_back((double)(nx[0] - o[4]));
      }
    const char* nm[5] = {"wait", "load+fold", "wavefront", "store+drain", "gap"};
    printf("item phases (memtime ticks, 100 MHz):");
    for (int k = 0; k < 5; k++) {
      std::sort(ph[k].begin(), ph[k].end());
      if (ph[k].empty()) continue;
      printf(" %s p10 %.0f p50 %.0f p90 %.0f;", nm[k], ph[k][ph[k].size() / 10], ph[k][ph[k].size() / 2],
             ph[k][ph[k].size() * 9 / 10]);
    }
    printf("\n");
  }
  float best = 1e9, sum = 0;
  for (float t : ts) {
    best = std::min(best, t);
    sum += t;
  }
  printf("var %d K=%d backward best %.4f ms mean %.4f ms (%d reps, every rep byte-exact vs per-level launches)\n", var, K,
         best, sum / reps, reps);
  return 0;
}
