// Dev tool (not shipped): Σ-pass access patterns without the arithmetic — which load/store shape
// streams a row-major n × ld matrix fastest, one 32×32 fp32 tile per wave, 4 waves per block.
// Build: hipcc -O3 --offload-arch=gfx950 pattern_bench.hip -o pattern_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

// (a) the 32x32x2 f32 MFMA D layout: 16 dword loads / stores, each instruction 2 rows × 128 B
__global__ __launch_bounds__(256) void k_dlayout(const float* __restrict__ in, float* __restrict__ out, int n, int ld, int tiles) {
  const int lane = threadIdx.x & 63, t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= tiles * tiles) return;
  const int R0 = (t / tiles) * 32, C0 = (t % tiles) * 32, kr = lane >> 5, kc = lane & 31;
  float v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = R0 + (r & 3) + 8 * (r >> 2) + 4 * kr;
    v[r] = in[(size_t)min(row, n - 1) * ld + min(C0 + kc, n - 1)];
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = R0 + (r & 3) + 8 * (r >> 2) + 4 * kr;
    if (row < n && C0 + kc < n) out[(size_t)row * ld + C0 + kc] = v[r] * 1.0001f;
  }
}

// (b) the same tile as 4 dwordx4 loads / stores per lane, each instruction 8 rows × 128 B
__global__ __launch_bounds__(256) void k_vec4(const float* __restrict__ in, float* __restrict__ out, int n, int ld, int tiles) {
  const int lane = threadIdx.x & 63, t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= tiles * tiles) return;
  const int R0 = (t / tiles) * 32, C0 = (t % tiles) * 32, c4 = (lane & 7) * 4, rr = lane >> 3;
  float4 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = min(R0 + rr + 8 * i, n - 1);
    v[i] = *reinterpret_cast<const float4*>(in + (size_t)row * ld + C0 + c4);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = R0 + rr + 8 * i;
    float4 w = v[i];
    w.x *= 1.0001f; w.y *= 1.0001f; w.z *= 1.0001f; w.w *= 1.0001f;
    if (row < n) *reinterpret_cast<float4*>(out + (size_t)row * ld + C0 + c4) = w;
  }
}

// (c) 1-D streaming copy of the same bytes, one float4 per thread
__global__ void k_copy(const float4* __restrict__ in, float4* __restrict__ out, size_t nv) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nv) out[i] = in[i];
}

// (d) (a) with the tile row-band per block: 4 waves = 4 consecutive tile rows of one tile column
__global__ __launch_bounds__(256) void k_dlayout_col(const float* __restrict__ in, float* __restrict__ out, int n, int ld, int tiles) {
  const int lane = threadIdx.x & 63, t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= tiles * tiles) return;
  const int C0 = (t / tiles) * 32, R0 = (t % tiles) * 32, kr = lane >> 5, kc = lane & 31;
  float v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = R0 + (r & 3) + 8 * (r >> 2) + 4 * kr;
    v[r] = in[(size_t)min(row, n - 1) * ld + min(C0 + kc, n - 1)];
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = R0 + (r & 3) + 8 * (r >> 2) + 4 * kr;
    if (row < n && C0 + kc < n) out[(size_t)row * ld + C0 + kc] = v[r] * 1.0001f;
  }
}

int main() {
  for (int n : {2051, 1030, 4099}) {
    const int ld = (n + 31) / 32 * 32, tiles = (n + 31) / 32;
    const size_t elems = (size_t)n * ld;
    float *a, *b;
    CK(hipMalloc(&a, elems * 4 + 64));
    CK(hipMalloc(&b, elems * 4 + 64));
    CK(hipMemset(a, 0, elems * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 200, blocks = (tiles * tiles + 3) / 4;
    const double bytes = 2.0 * elems * 4;
    auto timeit = [&](const char* name, auto fn) {
      for (int i = 0; i < 5; ++i) fn();
      CK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i) fn();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / reps;
      printf("n=%d %-12s %7.2f us %6.0f GB/s\n", n, name, us, bytes / us / 1e3);
    };
    timeit("dlayout", [&] { hipLaunchKernelGGL(k_dlayout, dim3(blocks), dim3(256), 0, 0, a, b, n, ld, tiles); });
    timeit("dlayout_col", [&] { hipLaunchKernelGGL(k_dlayout_col, dim3(blocks), dim3(256), 0, 0, a, b, n, ld, tiles); });
    timeit("vec4", [&] { hipLaunchKernelGGL(k_vec4, dim3(blocks), dim3(256), 0, 0, a, b, n, ld, tiles); });
    const size_t nv = elems / 4;
    timeit("copy", [&] { hipLaunchKernelGGL(k_copy, dim3((nv + 255) / 256), dim3(256), 0, 0, (const float4*)a, (float4*)b, nv); });
    CK(hipFree(a));
    CK(hipFree(b));
  }
  return 0;
}
