// mall_probe.hip -- does data written by one kernel come back from the
// Infinity Cache (MALL) in the next?  Diagnostic tool, not product code.
//
// A plane level of the 2^30 PLANES backward writes ~22 MB and the next two
// levels read it back (each 1 KiB plane by up to 8 waves on several XCDs).
// This probe times, on HIP events:
//   W: write S bytes (16 B per lane, whole 1 KiB chunks per wave)
//   R1: read them back right after (1 KiB chunks in a scattered order)
//   R2: the same read after 1 GiB of other writes (the chunk is HBM-cold)
//   R3: the same read again right after R2 (hot in MALL if it caches reads)
//   ./tools/mall_probe [MB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

__global__ void k_write(uint4* p, size_t n16, uint32_t v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_uint4(v, (uint32_t)i, v ^ 1u, (uint32_t)(i >> 32));
}

// each wave reads whole 1 KiB chunks, chunk c -> (c * 2654435761) mod nchunks
template <int ILP>
__global__ void k_read(const uint4* __restrict__ p, size_t nch, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63;
  const size_t w = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  uint32_t acc = 0;
  for (size_t c0 = w * ILP; c0 < nch; c0 += nw * ILP) {
    uint4 v[ILP];
#pragma unroll
    for (int i = 0; i < ILP; i++) {
      const size_t c = c0 + i < nch ? c0 + i : c0;
      const size_t ch = (c * 2654435761ull) % nch;
      v[i] = p[ch * 64 + lane];
    }
#pragma unroll
    for (int i = 0; i < ILP; i++) acc += v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
static int g_ilp = 1;
static void rd(const uint4* p, size_t nch, uint32_t* out, int grid) {
  if (g_ilp == 8) hipLaunchKernelGGL(k_read<8>, dim3(grid), dim3(256), 0, 0, p, nch, out);
  else if (g_ilp == 4) hipLaunchKernelGGL(k_read<4>, dim3(grid), dim3(256), 0, 0, p, nch, out);
  else hipLaunchKernelGGL(k_read<1>, dim3(grid), dim3(256), 0, 0, p, nch, out);
}

int main(int argc, char** argv) {
  const size_t mb = argc > 1 ? (size_t)atoi(argv[1]) : 24;
  g_ilp = argc > 2 ? atoi(argv[2]) : 1;
  const size_t S = mb << 20, BIG = (size_t)1 << 30;
  uint4 *a, *b;
  uint32_t* out;
  CK(hipMalloc(&a, S));
  CK(hipMalloc(&b, BIG));
  CK(hipMalloc(&out, 64));
  hipEvent_t ev[8];
  for (auto& x : ev) CK(hipEventCreate(&x));
  const size_t n16 = S / 16, nch = S / 1024;
  const int grid = 256 * 8;
  for (int rep = 0; rep < 3; rep++) {
    CK(hipEventRecord(ev[0]));
    hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, a, n16, 7u + rep);
    CK(hipEventRecord(ev[1]));
    rd(a, nch, out, grid);
    CK(hipEventRecord(ev[2]));
    hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, b, BIG / 16, 3u);
    CK(hipEventRecord(ev[3]));
    rd(a, nch, out, grid);
    CK(hipEventRecord(ev[4]));
    rd(a, nch, out, grid);
    CK(hipEventRecord(ev[5]));
    CK(hipEventSynchronize(ev[5]));
    float t[5];
    for (int k = 0; k < 5; k++) CK(hipEventElapsedTime(&t[k], ev[k], ev[k + 1]));
    printf("ILP %d S=%zu MB  W %.1f us (%.2f TB/s)  R1 after write %.1f us (%.2f TB/s)  big write %.1f us  "
           "R2 cold %.1f us (%.2f TB/s)  R3 again %.1f us (%.2f TB/s)\n",
           g_ilp, mb, t[0] * 1e3, S / (t[0] * 1e-3) / 1e12, t[1] * 1e3, S / (t[1] * 1e-3) / 1e12, t[2] * 1e3, t[3] * 1e3,
           S / (t[3] * 1e-3) / 1e12, t[4] * 1e3, S / (t[4] * 1e-3) / 1e12);
  }
  return 0;
}
