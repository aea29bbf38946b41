// Dev tool (not shipped): Σ-pass bandwidth vs a plain vectorised copy of the same bytes.
// Build: hipcc -O3 --offload-arch=gfx950 -I../include -I../ekf-slam_amd/csrc sigma_bench.hip
#include "../ekf-slam_amd/csrc/ekf_kernels.hip"

#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>
#include <algorithm>

using namespace ekfslam;
static int g_pingpong = 0;
static int g_m = 16;
static unsigned* sync_buf(int nf) {  // device epochs (kSync*), zeroed
  unsigned* p = nullptr;
  const size_t bytes = sizeof(unsigned) * (kSyncChain + nf);
  if (hipMalloc(&p, bytes) != hipSuccess || hipMemset(p, 0, bytes) != hipSuccess) abort();
  return p;
}
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

template <typename V>
__global__ void k_copy(const V* __restrict__ in, V* __restrict__ out, size_t nv) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += gridDim.x * blockDim.x) out[i] = in[i];
}

template <typename T>
void run(int N, int F, int reps) {
  const int n = 3 + 2 * N;
  const int per_line = 128 / sizeof(T);
  const int ld = (n + per_line - 1) / per_line * per_line, ldk = (n + 63) / 64 * 64;
  const size_t stride = static_cast<size_t>(n) * ld;
  T *S0, *S1, *kc, *mc;
  CK(hipMalloc(&S0, stride * F * sizeof(T)));
  CK(hipMalloc(&S1, stride * F * sizeof(T)));
  CK(hipMemset(S0, 0, stride * F * sizeof(T)));
  CK(hipMalloc(&kc, static_cast<size_t>(kMaxKW) * ldk * F * sizeof(T)));
  CK(hipMalloc(&mc, static_cast<size_t>(kMaxKW) * ldk * F * sizeof(T)));
  std::vector<T> h(static_cast<size_t>(kMaxKW) * ldk * F);
  for (auto& v : h) v = static_cast<T>((rand() % 1000) * 1e-5);
  CK(hipMemcpy(kc, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  CK(hipMemcpy(mc, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  std::vector<MsgDesc> d(F);
  for (int f = 0; f < F; ++f) { std::memset(&d[f], 0, sizeof(MsgDesc)); d[f].m = g_m; d[f].flags = kActive | kFirst; }
  MsgDesc* dd;  // [2][F]: parity 0 and parity 1 descriptors (ping-pong like the product)
  CK(hipMalloc(&dd, 2 * F * sizeof(MsgDesc)));
  CK(hipMemcpy(dd, d.data(), F * sizeof(MsgDesc), hipMemcpyHostToDevice));
  for (int f = 0; f < F; ++f) d[f].parity = 1;
  CK(hipMemcpy(dd + F, d.data(), F * sizeof(MsgDesc), hipMemcpyHostToDevice));
  FilterCtl* ctl;
  CK(hipMalloc(&ctl, F * sizeof(FilterCtl)));
  ChunkRec* rec;  // [2][F], nu = 0: no U block to write back (the fp32 pass reads rec->u / nu)
  CK(hipMalloc(&rec, 2 * F * sizeof(ChunkRec)));
  CK(hipMemset(rec, 0, 2 * F * sizeof(ChunkRec)));
  PassArgs<T> a{};
  a.rec = rec; a.rec_stride = F;
  a.sig[0] = S0; a.sig[1] = S1; a.sig_stride = stride;
  a.kcat = kc; a.mcat = mc; a.km_stride = static_cast<size_t>(kMaxKW) * ldk; a.ldk = ldk;
  a.ctl = ctl; a.sync = sync_buf(4096); a.desc = dd; a.n = n; a.ld = ld; a.N = N; a.f0 = 0; a.q = 1e-2;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = 2.0 * n * n * sizeof(T) * F;
  float ms;
  // copy of the same buffer (16-B vectors)
  using V = float4;
  const size_t nv = stride * F * sizeof(T) / sizeof(V);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k_copy<V>, dim3(4096), dim3(256), 0, s, (const V*)S0, (V*)S1, nv);
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k_copy<V>, dim3(4096), dim3(256), 0, s, (const V*)S0, (V*)S1, nv);
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double cbytes = 2.0 * stride * F * sizeof(T);
  printf("N=%d F=%d %s: copy %.2f us (%.0f GB/s)", N, F, sizeof(T) == 4 ? "f32" : "f64", ms * 1e3 / reps, cbytes / (ms / reps * 1e-3) / 1e9);
  for (int i = 0; i < 3; ++i) CK(launch_sigma_pass<T>(a, F, false, false, s));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < reps; ++i) {
    if (g_pingpong) a.desc = dd + (i & 1) * F;
    CK(launch_sigma_pass<T>(a, F, false, false, s));
  }
  a.desc = dd;
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf(" | sigma pass %.2f us (%.0f GB/s algorithmic)\n", ms * 1e3 / reps, bytes / (ms / reps * 1e-3) / 1e9);
#ifdef EKF_DIAG_STAMPS
  {
    const int tiles = ((n + SigmaTile<T>::kRows - 1) / SigmaTile<T>::kRows * ((n + SigmaTile<T>::kCols - 1) / SigmaTile<T>::kCols) + 3) / 4, nb = std::min(tiles, 4096);
    CK(launch_sigma_pass<T>(a, F, false, false, s));
    CK(launch_sigma_pass<T>(a, F, false, false, s));
    CK(hipStreamSynchronize(s));
    std::vector<unsigned long long> st(4096 * 5);
    CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_sig_stamps), st.size() * sizeof(unsigned long long)));
    unsigned long long t0 = ~0ull, tend = 0;
    std::vector<double> e, d1, d2, d3;
    for (int b = 0; b < nb; ++b) t0 = std::min(t0, st[5 * b]);
    for (int b = 0; b < nb; ++b) {
      const unsigned long long* x = &st[5 * b];
      tend = std::max(tend, x[3]);
      e.push_back((x[0] - t0) * 0.01); d1.push_back((x[1] - x[0]) * 0.01);
      d2.push_back((x[2] - x[1]) * 0.01); d3.push_back((x[3] - x[2]) * 0.01);
    }
    auto q = [](std::vector<double> v, double f) { std::sort(v.begin(), v.end()); return v[(size_t)(f * (v.size() - 1))]; };
    printf("   stamps(us): entry med %.2f max %.2f | desc med %.2f max %.2f | loads+mfma med %.2f max %.2f | "
           "stores med %.2f max %.2f | span %.2f\n", q(e, .5), q(e, 1), q(d1, .5), q(d1, 1), q(d2, .5), q(d2, 1),
           q(d3, .5), q(d3, 1), (tend - t0) * 0.01);
    if (n == 1024 && sizeof(T) == 4)
      for (int b = 0; b < nb; ++b) {
        const unsigned long long* x = &st[5 * b];
        const unsigned hw = x[4] & 0xffffffffu, xcc = x[4] >> 32;
        printf("   b%3d xcc %u se %u cu %2u simd %u wave %u entry %.2f end %.2f\n", b, xcc & 0xf, (hw >> 13) & 7,
               (hw >> 8) & 15, (hw >> 4) & 3, hw & 15, (x[0] - t0) * 0.01, (x[3] - t0) * 0.01);
      }
  }
#endif
  CK(hipFree(S0)); CK(hipFree(S1)); CK(hipFree(kc)); CK(hipFree(mc)); CK(hipFree(dd)); CK(hipFree(ctl)); CK(hipFree(rec));
}

int main(int argc, char** argv) {
  if (argc > 1) g_pingpong = atoi(argv[1]);
  if (argc > 2) g_m = atoi(argv[2]);
  run<float>(1024, 1, 200);
  run<double>(1024, 1, 200);
  run<double>(256, 1, 200);
  run<double>(256, 64, 50);
  run<double>(256, 512, 10);
  run<float>(4096, 1, 20);
  return 0;
}
