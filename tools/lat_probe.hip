// Dev tool: dependent-latency probe for the chain kernel's building blocks on gfx950
// (one wave, s_memtime). Build: hipcc --offload-arch=gfx950 -O3 tools/lat_probe.hip -o tools/lat_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ double readlane_f64(double v, int l) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane(static_cast<int>(x), l);
  const int hi = __builtin_amdgcn_readlane(static_cast<int>(x >> 32), l);
  return __hiloint2double(hi, lo);
}

__global__ void probe(double* out, unsigned long long* t, double a, double b, int n) {
  double x = threadIdx.x * 1e-3 + a;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {  // 8 dependent FMAs per iteration
#pragma unroll
    for (int k = 0; k < 8; ++k) x = fma(x, b, a);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double y = x;
  for (int i = 0; i < n; ++i) {  // 8 dependent readlane_f64 + add
#pragma unroll
    for (int k = 0; k < 8; ++k) y = readlane_f64(y, k + 1) + b;
  }
  unsigned long long t2 = __builtin_amdgcn_s_memtime();
  double z = y;
  for (int i = 0; i < n; ++i) {  // 8 dependent divisions
#pragma unroll
    for (int k = 0; k < 8; ++k) z = a / (z + b);
  }
  unsigned long long t3 = __builtin_amdgcn_s_memtime();
  __shared__ double lds[64];
  double w = z;
  for (int i = 0; i < n; ++i) {  // 8 dependent LDS write+read round trips
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      lds[threadIdx.x] = w;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      w = lds[(threadIdx.x + 1) & 63] + b;
    }
  }
  unsigned long long t4 = __builtin_amdgcn_s_memtime();
  double u = w;
  for (int i = 0; i < n; ++i) {  // 8 independent FMA chains interleaved (throughput)
    double p0 = u, p1 = u + 1, p2 = u + 2, p3 = u + 3, p4 = u + 4, p5 = u + 5, p6 = u + 6, p7 = u + 7;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      p0 = fma(p0, b, a); p1 = fma(p1, b, a); p2 = fma(p2, b, a); p3 = fma(p3, b, a);
      p4 = fma(p4, b, a); p5 = fma(p5, b, a); p6 = fma(p6, b, a); p7 = fma(p7, b, a);
    }
    u = p0 + p1 + p2 + p3 + p4 + p5 + p6 + p7;
  }
  unsigned long long t5 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x + y + z + w + u;
  if (threadIdx.x == 0) {
    t[0] = t1 - t0; t[1] = t2 - t1; t[2] = t3 - t2; t[3] = t4 - t3; t[4] = t5 - t4;
  }
}

int main() {
  double* out; unsigned long long* t;
  hipMalloc(&out, 64 * sizeof(double));
  hipMalloc(&t, 8 * sizeof(unsigned long long));
  const int n = 1000;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, out, t, 0.5, 0.999, n);
    hipDeviceSynchronize();
  }
  unsigned long long h[8];
  hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
  const double ops = 8.0 * n;
  printf("cycles per dependent f64 fma        %.2f\n", h[0] / ops);
  printf("cycles per dependent readlane_f64+add %.2f\n", h[1] / ops);
  printf("cycles per dependent f64 division    %.2f\n", h[2] / ops);
  printf("cycles per LDS write->read round trip %.2f\n", h[3] / ops);
  printf("cycles per f64 fma, 8 chains         %.2f\n", h[4] / (ops * 8));
  return 0;
}
