// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access patterns of the
// merge kernels (random 4 B / 16 B gathers and 4 B scattered stores), against a known request
// count. MI355X_MICROARCH.md calibrates only 16-B-per-lane streaming reads (FETCH_SIZE = half the
// bytes) and asks for a calibration of any other width before trusting an absolute.
// Build: hipcc --offload-arch=gfx950 -O3 -o calib_fetch calib_fetch.hip
// Run:   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./calib_fetch   (then WRITE_SIZE)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}
__global__ void k_cal_stream16(const uint4* __restrict__ a, uint64_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ void k_cal_gather4(const uint32_t* __restrict__ a, uint64_t words, uint64_t n, uint32_t* out) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t v = a[mix(i) % words];
  if (v == 0x12345678u) out[0] = v;
}
__global__ void k_cal_gather16(const uint4* __restrict__ a, uint64_t quads, uint64_t n, uint32_t* out) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 v = a[mix(i) % quads];
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) out[0] = v.x;
}
__global__ void k_cal_scatter4(uint32_t* __restrict__ a, uint64_t words, uint64_t n) {
  const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  a[mix(i + 77) % words] = (uint32_t)i;
}
__global__ void k_cal_stream_store16(uint4* __restrict__ a, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    a[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

int main() {
  const uint64_t bytes = uint64_t(4) << 30;  // 4 GiB: far past the 256 MiB last-level cache
  uint32_t* a = nullptr;
  uint32_t* out = nullptr;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) { fprintf(stderr, "alloc failed\n"); return 1; }
  hipMemset(a, 1, bytes);
  const uint64_t n = uint64_t(64) << 20;  // 64 Mi random requests per gather kernel
  const uint64_t stream_quads = (uint64_t(1) << 30) / 16;  // 1 GiB streamed
  hipLaunchKernelGGL(k_cal_stream16, dim3(8192), dim3(256), 0, 0, (const uint4*)a, stream_quads, out);
  hipLaunchKernelGGL(k_cal_gather4, dim3(n / 256), dim3(256), 0, 0, (const uint32_t*)a, bytes / 4, n, out);
  hipLaunchKernelGGL(k_cal_gather16, dim3(n / 256), dim3(256), 0, 0, (const uint4*)a, bytes / 16, n, out);
  hipLaunchKernelGGL(k_cal_scatter4, dim3(n / 256), dim3(256), 0, 0, a, bytes / 4, n);
  hipLaunchKernelGGL(k_cal_stream_store16, dim3(8192), dim3(256), 0, 0, (uint4*)a, stream_quads);
  if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "kernel failed\n"); return 1; }
  printf("requests per gather/scatter kernel: %llu; streamed bytes: %llu\n", (unsigned long long)n,
         (unsigned long long)(stream_quads * 16));
  hipFree(a);
  hipFree(out);
  return 0;
}
