// Dev tool: issue and dependent-latency costs of the chain's wave-0 building blocks on gfx950, one
// wave alone on its SIMD (s_memtime cycles). Each probe runs 8·n operations; "dep" = each op uses
// the previous result, "ind" = 8 independent chains interleaved (issue throughput).
// Build: hipcc --offload-arch=gfx950 -O3 tools/lat_probe2.hip -o tools/lat_probe2
#include <hip/hip_runtime.h>

#include <cstdio>

#define PROBE(name, init, body)                                                   \
  {                                                                              \
    init;                                                                        \
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();                  \
    for (int i = 0; i < n; ++i) {                                                \
      _Pragma("unroll") for (int k = 0; k < 8; ++k) { body; }                   \
    }                                                                            \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();                  \
    if (threadIdx.x == 0) t[np] = t1 - t0;                                       \
    ++np;                                                                        \
  }

__device__ __forceinline__ double rl(double v, int l) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane(static_cast<int>(x), l);
  const int hi = __builtin_amdgcn_readlane(static_cast<int>(x >> 32), l);
  return __hiloint2double(hi, lo);
}

__global__ void probe(double* out, unsigned long long* t, double a, double b, int n) {
  __shared__ double lds[256];
  int np = 0;
  double acc = threadIdx.x * 1e-3 + a;
  double p[8];
  for (int k = 0; k < 8; ++k) p[k] = acc + k;
  lds[threadIdx.x] = acc;
  lds[threadIdx.x + 64] = acc;
  __syncthreads();
  PROBE("dep fma", , acc = fma(acc, b, a));
  PROBE("dep mul", , acc = acc * b);
  PROBE("dep add", , acc = acc + b);
  PROBE("dep rcp", , acc = __builtin_amdgcn_rcp(acc + 2.0));
  PROBE("dep rsq", , acc = __builtin_amdgcn_rsq(acc + 2.0));
  PROBE("dep readlane", , acc = rl(acc, k + 1) + b);
  PROBE("ind fma x8", , {
    p[0] = fma(p[0], b, a); p[1] = fma(p[1], b, a); p[2] = fma(p[2], b, a); p[3] = fma(p[3], b, a);
    p[4] = fma(p[4], b, a); p[5] = fma(p[5], b, a); p[6] = fma(p[6], b, a); p[7] = fma(p[7], b, a);
  });
  PROBE("ind readlane x8", double s = 0.0, {
    s += rl(p[0], k) ; s += rl(p[1], k + 1); s += rl(p[2], k + 2); s += rl(p[3], k + 3);
  });
  PROBE("dep lds rt", , {
    lds[threadIdx.x] = acc;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    acc = lds[(threadIdx.x + 1) & 63] + b;
  });
  PROBE("dep lds read (addr chain)", int ix = threadIdx.x, {
    ix = static_cast<int>(lds[ix & 127]) & 63;
  });
  PROBE("ind cndmask x8", int q = threadIdx.x, {
    q = (q & 1) ? q + 3 : q - 1; q = (q & 2) ? q + 3 : q - 1; q = (q & 4) ? q + 3 : q - 1;
    q = (q & 8) ? q + 3 : q - 1;
  });
  for (int k = 0; k < 8; ++k) acc += p[k];
  out[threadIdx.x] = acc;
}

int main() {
  double* out;
  unsigned long long* t;
  hipMalloc(&out, 64 * sizeof(double));
  hipMalloc(&t, 32 * sizeof(unsigned long long));
  const int n = 2000;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, out, t, 0.5, 0.999, n);
    hipDeviceSynchronize();
  }
  unsigned long long h[32];
  hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[] = {"dep v_fma_f64", "dep v_mul_f64", "dep v_add_f64", "dep v_rcp_f64",
                         "dep v_rsq_f64", "dep readlane_f64 + add", "ind fma (per fma, 8 chains)",
                         "ind readlane_f64 + add (per op, 4/iter)", "dep LDS write->read",
                         "dep LDS read (address chain)", "32-bit select chain (per 4 ops)"};
  const double per[] = {8, 8, 8, 8, 8, 8, 64, 32, 8, 8, 8};
  for (int i = 0; i < 11; ++i) printf("%-42s %8.2f cycles\n", names[i], h[i] / (per[i] * 2000.0));
  return 0;
}
