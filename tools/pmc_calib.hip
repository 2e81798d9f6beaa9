// pmc_calib.hip -- calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE for the access width the
// stencil kernels use (8-byte fp64 loads and stores, one per lane, coalesced along i).
// MI355X_MICROARCH.md (HBM section) calibrates only 16-B-per-lane streams (FETCH_SIZE
// reads half the bytes there); this copies a known byte count so that
// tools/pmc_summary.py can apply the factor measured for our own pattern.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/pmc_calib tools/pmc_calib.hip
//   rocprofv3 --pmc FETCH_SIZE -d OUT -o run --output-format csv -- tools/pmc_calib
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(256) k_calib_copy8(double *__restrict__ dst, const double *__restrict__ src, long n) {
  const long q = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < n) dst[q] = src[q] * 1.0000001;
}

int main() {
  const long n = 96L << 20;   // 96 Mi doubles = 768 MiB per array: far beyond the 256 MiB Infinity Cache
  double *a = nullptr, *b = nullptr;
  if (hipMalloc(&a, n * 8) != hipSuccess || hipMalloc(&b, n * 8) != hipSuccess) { fprintf(stderr, "alloc\n"); return 1; }
  hipMemset(a, 0, n * 8);
  hipMemset(b, 0, n * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int r = 0; r < 4; r++) {
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_calib_copy8, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, b, a, n);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    printf("k_calib_copy8: read %ld B, wrote %ld B, %.3f ms, %.1f GB/s\n", n * 8, n * 8, ms, 2.0 * n * 8 / (ms * 1e-3) / 1e9);
  }
  hipFree(a);
  hipFree(b);
  return 0;
}
