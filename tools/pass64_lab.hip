// Dev tool (not shipped): the swarm's fp64 Σ pass (512 filters, N = 256: n = 515, 2.2 GB of Σ per
// message) A/B'd standalone against the product's k_sigma_pass<double, true> on the same buffers,
// outputs (Σ_out and the kRowsOut rows) compared bit for bit.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../include -I../ekf-slam_amd/csrc pass64_lab.hip -o pass64_lab
#include "../ekf-slam_amd/csrc/ekf_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace ekfslam;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

// the product's wide tile with ablations: MODE 1 = no MFMA (a VALU product keeps the operands
// live), 2 = no operand loads (constants), both = Σ_in → Σ_out only
enum { kNoMfma = 1, kNoOps = 2 };
template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_ablate(PassArgs<double> A, int tcols, int xcd_b, int nf) {
  const int L = blockIdx.x, j = L >> 3;
  const int fb = (L & 7) + 8 * (j / xcd_b), bx = j % xcd_b;
  if (fb >= nf) return;
  const MsgDesc& d = A.desc[fb];
  const int lane = threadIdx.x & 63;
  const int trows = (A.n + 31) / 32;
  const int t = __builtin_amdgcn_readfirstlane(bx * 4 + (threadIdx.x >> 6));
  if (t >= trows * tcols || !(d.flags & kActive)) return;
  const int R0 = (t / tcols) * 32, C0 = (t % tcols) * 64;
  const int f = A.f0 + fb;
  const int n = A.n, ld = A.ld, ldk = A.ldk;
  const double* Sin = A.sig[d.parity] + f * A.sig_stride;
  double* Sout = A.sig[d.parity ^ 1] + f * A.sig_stride;
  const double* kc = A.kcat + f * A.km_stride;
  const double* mc = A.mcat + f * A.km_stride;
  constexpr int TJ = 4;
  const int kr = lane >> 4, kcol = lane & 15;
  const size_t pbase = static_cast<size_t>(R0) * ld;
  const unsigned sbytes = static_cast<unsigned>(min(n - R0, 32)) * ld * 8u;
  const unsigned kbytes = static_cast<unsigned>(kMaxKW) * ldk * 8u;
  const auto rin = buf_rsrc(Sin + pbase, sbytes), rout = buf_rsrc(Sout + pbase, sbytes);
  const auto rk = buf_rsrc(kc, kbytes), rm = buf_rsrc(mc, kbytes);
  double a[2][9], b[TJ][9], sv[2][TJ][4];
  const unsigned ko = static_cast<unsigned>(kr * ldk + R0 + kcol) * 8u;
  unsigned mo[TJ], so[TJ];
  const unsigned rstride = static_cast<unsigned>(ld) * 8u;
#pragma unroll
  for (int tj = 0; tj < TJ; ++tj) {
    const int col = C0 + 16 * tj + kcol;
    mo[tj] = static_cast<unsigned>(kr * ldk + min(col, n - 1)) * 8u;
    so[tj] = col < n ? static_cast<unsigned>(kr * ld + col) * 8u : kOOB;
  }
  const unsigned kstep = 4u * ldk * 8u;
  if (MODE & kNoOps) {
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      a[0][s] = 1e-3 * (s + 1);
      a[1][s] = 2e-3 * (s + 1);
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj) b[tj][s] = 1e-3 * (tj + s);
    }
  } else {
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      a[0][s] = ld_f64(rk, ko, s * kstep);
      a[1][s] = ld_f64(rk, ko + 16 * 8, s * kstep);
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj) b[tj][s] = ld_f64(rm, mo[tj], s * kstep);
    }
  }
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        sv[ti][tj][r] = __builtin_bit_cast(
            double, __builtin_amdgcn_raw_buffer_load_b64(rin, so[tj] + (16 * ti + 4 * r) * rstride, 0, 2));
  d4 acc[2][TJ];
  if (MODE & kNoMfma) {
    double s0 = 0.0;
#pragma unroll
    for (int s = 0; s < 9; ++s) s0 += a[0][s] * a[1][s] + b[0][s] * b[1][s] + b[2][s] * b[3][s];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj) acc[ti][tj] = d4{s0, s0, s0, s0};
  } else {
    const int kw = ((2 + 2 * d.m + 3) / 4) * 4;
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj) acc[ti][tj] = d4{0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      const bool live = 4 * s < kw;
#pragma unroll
      for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < TJ; ++tj)
          acc[ti][tj] = mfma_f64(live ? a[ti][s] : 0.0, live ? b[tj][s] : 0.0, acc[ti][tj]);
    }
  }
#pragma unroll
  for (int ti = 0; ti < 2; ++ti)
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double v = sv[ti][tj][r] - acc[ti][tj][r];
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v), rout,
                                              so[tj] + (16 * ti + 4 * r) * rstride, 0, 2);
      }
}


template <typename V>
__global__ void k_copy(const V* __restrict__ in, V* __restrict__ out, size_t nv) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += gridDim.x * blockDim.x) out[i] = in[i];
}

int main(int argc, char** argv) {
  const int F = argc > 1 ? atoi(argv[1]) : 512, reps = argc > 2 ? atoi(argv[2]) : 20;
  const int N = 256, n = 3 + 2 * N, ld = (n + 15) / 16 * 16, ldk = (n + 63) / 64 * 64;
  const size_t stride = static_cast<size_t>(n) * ld, km = static_cast<size_t>(kMaxKW) * ldk;
  double *S0, *S1, *kc, *mc, *rows;
  CK(hipMalloc(&S0, stride * F * 8));
  CK(hipMalloc(&S1, stride * F * 8));
  CK(hipMalloc(&kc, km * F * 8));
  CK(hipMalloc(&mc, km * F * 8));
  CK(hipMalloc(&rows, static_cast<size_t>(kRowW) * ldk * F * 8));
  {
    std::vector<double> h(stride * F);
    srand(7);
    for (auto& v : h) v = (rand() % 100000) * 1e-3;
    CK(hipMemcpy(S0, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    std::vector<double> k(km * F);
    for (auto& v : k) v = (rand() % 2000 - 1000) * 1e-4;
    CK(hipMemcpy(kc, k.data(), k.size() * 8, hipMemcpyHostToDevice));
    for (auto& v : k) v = (rand() % 2000 - 1000) * 1e-4;
    CK(hipMemcpy(mc, k.data(), k.size() * 8, hipMemcpyHostToDevice));
  }
  std::vector<MsgDesc> hd(F);
  for (int f = 0; f < F; ++f) {
    MsgDesc& d = hd[f];
    std::memset(&d, 0, sizeof d);
    d.m = 16;
    d.flags = kActive | kFirst | ((f % 3) ? kRowsOut : 0);
    d.parity = 0;
    d.nxt_nu = 35;
    for (int b = 0; b <= kMaxU; ++b) d.nxt_u[b] = b < 3 ? b : 3 + ((f * 37 + b * 11) % (n - 3));
  }
  MsgDesc* dd;
  CK(hipMalloc(&dd, sizeof(MsgDesc) * F));
  CK(hipMemcpy(dd, hd.data(), sizeof(MsgDesc) * F, hipMemcpyHostToDevice));
  PassArgs<double> a{};
  a.sig[0] = S0; a.sig[1] = S1; a.sig_stride = stride;
  a.kcat = kc; a.mcat = mc; a.km_stride = km; a.ldk = ldk;
  a.rows = rows; a.rows_stride = static_cast<size_t>(kRowW) * ldk;
  a.desc = dd; a.n = n; a.ld = ld; a.N = N; a.q = 1e-2;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = 2.0 * n * n * 8 * F;
  std::vector<double> ref(stride * F), out(stride * F), rref(a.rows_stride * F), rout(a.rows_stride * F);
  const int trows = (n + 31) / 32, tcols = (n + 63) / 64, per_filter = (trows * tcols + 3) / 4;
  auto prod = [&](hipStream_t st) {
    hipLaunchKernelGGL((k_sigma_pass<double, true>), dim3(8 * ((F + 7) / 8) * per_filter), dim3(256), 0, st,
                       a, tcols, per_filter, F);
  };
  auto time_it = [&](const char* name, auto&& fn, bool check_rows) {
    CK(hipMemset(S1, 0, stride * F * 8));
    CK(hipMemset(rows, 0, a.rows_stride * F * 8));
    for (int i = 0; i < 3; ++i) fn(s);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(out.data(), S1, stride * F * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(rout.data(), rows, a.rows_stride * F * 8, hipMemcpyDeviceToHost));
    float best = 1e30f, sum = 0;
    for (int rep = 0; rep < 3; ++rep) {
      float ms;
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < reps; ++i) fn(s);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms);
      sum += ms;
    }
    size_t bad = 0, rbad = 0;
    for (int f = 0; f < F; ++f)
      for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) {
          const size_t o = f * stride + static_cast<size_t>(r) * ld + c;
          if (std::memcmp(&out[o], &ref[o], 8)) ++bad;
        }
    if (check_rows)
      for (int f = 0; f < F; ++f)
        for (int b = 0; b < kMaxU; ++b)
          for (int r = 0; r < n; ++r) {
            const size_t o = f * a.rows_stride + static_cast<size_t>(b) * ldk + r;
            if (std::memcmp(&rout[o], &rref[o], 8)) ++rbad;
          }
    printf("%-26s %8.2f us (best of 3; mean %8.2f)  %6.0f GB/s  frac %.3f  mismatches %zu rows %zu\n", name,
           best * 1e3 / reps, sum / 3 * 1e3 / reps, bytes / (best / reps * 1e-3) / 1e9,
           bytes / (best / reps * 1e-3) / 8e12, bad, rbad);
    fflush(stdout);
  };
  CK(hipMemset(rows, 0, a.rows_stride * F * 8));
  prod(s);
  CK(hipStreamSynchronize(s));
  CK(hipMemcpy(ref.data(), S1, stride * F * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(rref.data(), rows, a.rows_stride * F * 8, hipMemcpyDeviceToHost));
  {
    using F4 = float4;
    const size_t nv = stride * F * 8 / sizeof(F4);
    time_it("copy float4", [&](hipStream_t st) {
      hipLaunchKernelGGL(k_copy<F4>, dim3(8192), dim3(256), 0, st, (const F4*)S0, (F4*)S1, nv);
    }, false);
  }
  auto abl = [&](auto kern) {
    return [&, kern](hipStream_t st) {
      hipLaunchKernelGGL(kern, dim3(8 * ((F + 7) / 8) * per_filter), dim3(256), 0, st, a, tcols, per_filter, F);
    };
  };
  int dev_cus = 0;
  CK(hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, 0));
  auto stream = [&](int blocks) {
    return [&, blocks](hipStream_t st) {
      hipLaunchKernelGGL(k_sigma_stream, dim3(blocks), dim3(256), 0, st, a, tcols, trows * tcols, F);
    };
  };
  for (int round = 0; round < 2; ++round) {
    time_it("stream 1 wg/cu", stream(dev_cus), true);
    time_it("stream 0.75 wg/cu", stream(dev_cus * 3 / 4 / 8 * 8), true);
    time_it("product k_sigma_pass", prod, true);
    time_it("ablate: copy of product", abl(k_ablate<0>), false);
    time_it("ablate: no mfma", abl(k_ablate<kNoMfma>), false);
    time_it("ablate: no operands", abl(k_ablate<kNoOps>), false);
    time_it("ablate: sigma only", abl(k_ablate<kNoMfma | kNoOps>), false);
  }
  return 0;
}
