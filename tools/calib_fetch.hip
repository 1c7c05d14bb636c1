// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the access widths
// the solver's kernels use (MI355X_MICROARCH.md §HBM: only 16-B-per-lane
// streaming reads are calibrated there).  Each kernel touches a known byte
// count of a 1 GiB buffer (past the 256 MiB Infinity Cache); the PMC pass
// divides the counter by that count.
//   hipcc --offload-arch=gfx950 -O3 tools/calib_fetch.hip -o tools/calib_fetch
//   rocprofv3 --pmc FETCH_SIZE -- tools/calib_fetch
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x)                                                        \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      return 1;                                                       \
    }                                                                 \
  } while (0)

// 4 B per lane, contiguous per wave (the dense resolve's child loads)
__global__ void read_b32(const uint32_t* __restrict__ p, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  if (acc == 0x12345678u) out[0] = acc;
}
// 8 B per lane (bitmap words, hashed-table keys)
__global__ void read_b64(const uint64_t* __restrict__ p, size_t n, uint32_t* out) {
  uint64_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  if (acc == 0x12345678u) out[0] = (uint32_t)acc;
}
// 16 B per lane (the guide's calibrated case)
__global__ void read_b128(const uint4* __restrict__ p, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
// 4 B per lane stores (the resolve's word stores)
__global__ void write_b32(uint32_t* __restrict__ p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)i;
}

// 64 B of every 128-B line (16 lanes x 4 B, lines 128 B apart): does a
// partial-line read fetch 64 or 128 B?  n = lines
__global__ void read_half_lines(const uint32_t* __restrict__ p, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (size_t i = t; i < n * 16; i += (size_t)gridDim.x * blockDim.x) acc ^= p[(i >> 4) * 32 + (i & 15)];
  if (acc == 0x12345678u) out[0] = acc;
}
// resolve-shaped stream: two 16-B-per-lane reads and one 16-B-per-lane
// write per element (achievable rate of the dense resolve's compulsory
// traffic); n = elements of 16 B per stream
__global__ void triad_b128(const uint4* __restrict__ a, const uint4* __restrict__ b, uint4* __restrict__ c,
                           size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint4 x = a[i], y = b[i];
    c[i] = make_uint4(max(x.x, y.x), max(x.y, y.y), max(x.z, y.z), max(x.w, y.w));
  }
}

// Reuse at large strides (the dense resolve's top-digit children): a sweep
// reads every quad at i, i - o1, i - o2, so each line is requested three
// times, o1 / o2 quads apart in time.  With L2 reuse the misses stay near one
// per line.  Power-of-two strides against padded ones tests channel / set
// aliasing.  n = quads swept.
__global__ void reuse3(const uint4* __restrict__ a, size_t n, size_t o1, size_t o2, uint32_t* out) {
  uint32_t acc = 0;
  const size_t G = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += G) {
    const size_t j = i + o2;
    const uint4 x = a[j], y = a[j - o1], z = a[j - o2];
    acc ^= x.x ^ y.y ^ z.z;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const size_t bytes = (size_t)1 << 30;
  void* buf = nullptr;
  uint32_t* out = nullptr;
  CHK(hipMalloc(&buf, bytes));
  CHK(hipMalloc(&out, 64));
  CHK(hipMemset(buf, 1, bytes));
  const int grid = 256 * 8, block = 256;
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(read_b32, dim3(grid), dim3(block), 0, 0, (const uint32_t*)buf, bytes / 4, out);
    hipLaunchKernelGGL(read_b64, dim3(grid), dim3(block), 0, 0, (const uint64_t*)buf, bytes / 8, out);
    hipLaunchKernelGGL(read_b128, dim3(grid), dim3(block), 0, 0, (const uint4*)buf, bytes / 16, out);
    hipLaunchKernelGGL(write_b32, dim3(grid), dim3(block), 0, 0, (uint32_t*)buf, bytes / 4);
  }
  CHK(hipDeviceSynchronize());
  // timed: half-line reads and the resolve-shaped triad over 3 x 1/3 GiB
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  float ms_half = 0, ms_triad = 0;
  for (int rep = 0; rep < 3; rep++) {
    CHK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(read_half_lines, dim3(grid), dim3(block), 0, 0, (const uint32_t*)buf, bytes / 128, out);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms_half, e0, e1));
    const size_t third = bytes / 3 / 16;
    const uint4* a = (const uint4*)buf;
    CHK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(triad_b128, dim3(grid), dim3(block), 0, 0, a, a + third, (uint4*)(a + 2 * third), third);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    CHK(hipEventElapsedTime(&ms_triad, e0, e1));
  }
  // reuse3: pow2 vs padded strides (quads; 2^18 quads = 4 MB)
  float ms_pow2 = 0, ms_pad = 0;
  {
    const size_t n = ((size_t)1 << 30) / 16 - ((size_t)1 << 20);
    for (int rep = 0; rep < 3; rep++) {
      CHK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(reuse3, dim3(grid), dim3(block), 0, 0, (const uint4*)buf, n, (size_t)1 << 18,
                         (size_t)1 << 19, out);
      CHK(hipEventRecord(e1, 0));
      CHK(hipEventSynchronize(e1));
      CHK(hipEventElapsedTime(&ms_pow2, e0, e1));
      CHK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(reuse3, dim3(grid), dim3(block), 0, 0, (const uint4*)buf, n, ((size_t)1 << 18) + 40,
                         ((size_t)1 << 19) + 88, out);
      CHK(hipEventRecord(e1, 0));
      CHK(hipEventSynchronize(e1));
      CHK(hipEventElapsedTime(&ms_pad, e0, e1));
    }
  }
  printf("{\"reuse3_pow2_ms\": %.4f, \"reuse3_pad_ms\": %.4f}\n", ms_pow2, ms_pad);
  printf("{\"bytes_per_kernel\": %zu, \"half_lines_ms\": %.4f, \"half_lines_requested_GBps\": %.1f, "
         "\"triad_ms\": %.4f, \"triad_GBps\": %.1f}\n",
         bytes, ms_half, bytes / 2 / ms_half / 1e6, ms_triad, (double)(bytes / 3 / 16 * 16 * 3) / ms_triad / 1e6);
  CHK(hipFree(buf));
  CHK(hipFree(out));
  return 0;
}
