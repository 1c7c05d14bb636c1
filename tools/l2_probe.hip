// l2_probe.hip -- does a line written by one kernel stay in the writing
// XCD's L2 for the next kernel?  Diagnostic tool, not product code.
//
// W: block b writes its own 4 KiB chunk (2048 blocks, 8 MiB: 1 MiB per XCD,
// well inside one XCD's 4 MiB L2).  Then a read kernel in which block b reads
// chunk (b + shift) mod 2048 several times: shift 0 = the chunk its own XCD
// wrote (blocks b and b + 8k share an XCD under round-robin dispatch), shift 1
// = a chunk another XCD wrote.  If the writer's L2 keeps the lines across the
// kernel boundary, shift 0 reads at L2 speed.
//   ./tools/l2_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t err_ = (x);                                                             \
    if (err_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(err_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr int kBlocks = 2048, kChunk16 = 256;  // 4 KiB per block

__global__ void k_w(uint4* p, uint32_t v) {
  p[(size_t)blockIdx.x * kChunk16 + threadIdx.x] = make_uint4(v, blockIdx.x, threadIdx.x, v);
}
// per block: the cycles of its first (dependent) load, thread 0's view
__global__ void k_r(const uint4* __restrict__ p, int shift, uint32_t* out, uint64_t* cyc) {
  const uint32_t c = (blockIdx.x + shift) % kBlocks;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint4 v = p[(size_t)c * kChunk16 + threadIdx.x];
  const uint32_t acc = v.x ^ v.y ^ v.w;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint64_t t1 = __builtin_amdgcn_s_memtime() + (acc & 0 ? 1 : 0);
  if (acc == 0x9876543u) out[0] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  uint4* a;
  uint32_t* out;
  uint64_t* cyc;
  CK(hipMalloc(&a, (size_t)kBlocks * kChunk16 * 16));
  CK(hipMalloc(&out, 64));
  CK(hipMalloc(&cyc, kBlocks * 8));
  static uint64_t h[kBlocks];
  for (int rep = 0; rep < 3; rep++)
    for (int shift : {0, 1, 8, 3, 16}) {
      hipLaunchKernelGGL(k_w, dim3(kBlocks), dim3(256), 0, 0, a, 5u + rep);
      hipLaunchKernelGGL(k_r, dim3(kBlocks), dim3(256), 0, 0, a, shift, out, cyc);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost));
      double s1 = 0;
      for (int b = 0; b < kBlocks; b++) s1 += (double)h[b];
      hipLaunchKernelGGL(k_r, dim3(kBlocks), dim3(256), 0, 0, a, shift, out, cyc);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost));
      double s2 = 0;
      for (int b = 0; b < kBlocks; b++) s2 += (double)h[b];
      printf("rep %d shift %2d: first-load cycles after the write %.0f, on a second read %.0f\n", rep, shift,
             s1 / kBlocks, s2 / kBlocks);
    }
  return 0;
}
