// Dev tool (not shipped): the fp32 / fp64 Σ pass against a CPU Σ_in + Q̄ − Kcatᵀ·Mcat on random
// operands; prints the max error and the first wrong element.
// Build: hipcc -O3 --offload-arch=gfx950 -I../include -I../ekf-slam_amd/csrc sigma_check.hip
#include "../ekf-slam_amd/csrc/ekf_kernels.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace ekfslam;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

template <typename T>
int check(int N, int m = 16) {
  const int n = 3 + 2 * N, per_line = 128 / sizeof(T);
  const int ld = (n + per_line - 1) / per_line * per_line, ldk = (n + 63) / 64 * 64;
  const size_t ss = static_cast<size_t>(n) * ld, ks = static_cast<size_t>(kMaxKW) * ldk;
  std::vector<T> S(ss, 0), K(ks, 0), M(ks, 0), out(ss, 0);
  srand(7);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) S[static_cast<size_t>(i) * ld + j] = static_cast<T>((rand() % 2001 - 1000) * 1e-3);
  // the factor kernel writes the rank's 2 + 2m rows; the padding rows up to kw stay zero
  const int kw = ((2 + 2 * m + 3) / 4) * 4, rank = m >= 0 ? 2 + 2 * m : 0;
  for (int k = 0; k < rank && k < kw; ++k)
    for (int i = 0; i < n; ++i) {
      K[static_cast<size_t>(k) * ldk + i] = static_cast<T>((rand() % 2001 - 1000) * 1e-3);
      M[static_cast<size_t>(k) * ldk + i] = static_cast<T>((rand() % 2001 - 1000) * 1e-3);
    }
  T *dS0, *dS1, *dK, *dM;
  CK(hipMalloc(&dS0, ss * sizeof(T))); CK(hipMalloc(&dS1, ss * sizeof(T)));
  CK(hipMalloc(&dK, ks * sizeof(T))); CK(hipMalloc(&dM, ks * sizeof(T)));
  CK(hipMemcpy(dS0, S.data(), ss * sizeof(T), hipMemcpyHostToDevice));
  CK(hipMemset(dS1, 0, ss * sizeof(T)));
  CK(hipMemcpy(dK, K.data(), ks * sizeof(T), hipMemcpyHostToDevice));
  CK(hipMemcpy(dM, M.data(), ks * sizeof(T), hipMemcpyHostToDevice));
  MsgDesc d{};
  d.m = m;
  d.flags = kActive | kFirst;
  MsgDesc* dd;
  CK(hipMalloc(&dd, sizeof(MsgDesc)));
  CK(hipMemcpy(dd, &d, sizeof(MsgDesc), hipMemcpyHostToDevice));
  ChunkRec* rec;
  CK(hipMalloc(&rec, 2 * sizeof(ChunkRec)));
  CK(hipMemset(rec, 0, 2 * sizeof(ChunkRec)));
  PassArgs<T> a{};
  a.sig[0] = dS0; a.sig[1] = dS1; a.sig_stride = ss;
  a.kcat = dK; a.mcat = dM; a.km_stride = ks; a.ldk = ldk;
  a.rec = rec; a.rec_stride = 1; a.desc = dd;
  a.n = n; a.ld = ld; a.N = N; a.q = 0.01;
  CK(launch_sigma_pass<T>(a, 1, false, false, nullptr));
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(out.data(), dS1, ss * sizeof(T), hipMemcpyDeviceToHost));
  double worst = 0;
  int wi = -1, wj = -1;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double v = S[static_cast<size_t>(i) * ld + j];
      for (int k = 0; k < kw; ++k) v -= double(K[static_cast<size_t>(k) * ldk + i]) * M[static_cast<size_t>(k) * ldk + j];
      if (i == j && i < 3) v += 0.01;
      const double e = std::fabs(v - out[static_cast<size_t>(i) * ld + j]);
      if (e > worst) { worst = e; wi = i; wj = j; }
    }
  if (sizeof(T) == 4 && N == 50) {
    for (int i = 0; i < 3; ++i) {
      printf("row %d:", i);
      for (int j = 0; j < 40; ++j) {
        double v = S[static_cast<size_t>(i) * ld + j], km = 0;
        for (int k = 0; k < kw; ++k) km += double(K[static_cast<size_t>(k) * ldk + i]) * M[static_cast<size_t>(k) * ldk + j];
        if (i == j && i < 3) v += 0.01;
        const double o = out[static_cast<size_t>(i) * ld + j];
        // classify: ok, = S only (no KM), = -KM only (S lost), other
        const char* c = std::fabs(o - (v - km)) < 1e-3 ? "." : std::fabs(o - v) < 1e-3 ? "S" : std::fabs(o + km) < 1e-3 ? "k" : "x";
        printf("%s", c);
      }
      printf("\n");
    }
  }
  printf("%s N=%d n=%d m=%d: max |err| %.3e at (%d, %d)\n", sizeof(T) == 4 ? "fp32" : "fp64", N, n, m, worst, wi, wj);
  return worst < (sizeof(T) == 4 ? 1e-3 : 1e-10) ? 0 : 1;
}

int main() {
  int bad = 0;
  bad |= check<float>(50, -1);  // kw = 0: Σ_in + Q̄ only
  bad |= check<float>(50);
  bad |= check<float>(1024);
  bad |= check<double>(256);
  return bad;
}
