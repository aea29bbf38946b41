// Dev tool (not shipped): times the gain kernel alone and prints per-phase s_memtime stamps of
// block (0,0) thread 0. Build: hipcc -O3 --offload-arch=gfx950 -DEKF_DIAG_STAMPS -I../include
//   -I../ekf-slam_amd/csrc gain_bench.hip -o gain_bench
#include "../ekf-slam_amd/csrc/ekf_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace ekfslam;
static int g_look = 0;

static unsigned* sync_buf(int nf) {  // device epochs (kSync*), zeroed
  unsigned* p = nullptr;
  const size_t bytes = sizeof(unsigned) * (kSyncChain + nf);
  if (hipMalloc(&p, bytes) != hipSuccess || hipMemset(p, 0, bytes) != hipSuccess) abort();
  return p;
}
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

template <typename T>
void run(int N, int m, int reps) {
  const int n = 3 + 2 * N;
  const int per_line = 128 / sizeof(T);
  const int ld = (n + per_line - 1) / per_line * per_line, ldk = (n + 63) / 64 * 64;
  std::vector<T> S(static_cast<size_t>(n) * ld, 0);
  std::vector<double> x(n, 0);
  srand(1);
  for (int i = 0; i < n; ++i) S[static_cast<size_t>(i) * ld + i] = i < 3 ? 1e-2 : 1e-2;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < i; ++j) {
      T v = static_cast<T>(1e-4 * ((rand() % 1000) / 1000.0 - 0.5));
      S[static_cast<size_t>(i) * ld + j] = v;
      S[static_cast<size_t>(j) * ld + i] = v;
    }
  for (int k = 0; k < N; ++k) { x[3 + 2 * k] = 1.0 + 0.1 * k; x[4 + 2 * k] = 0.5 - 0.05 * k; }
  T *dS[2], *kc, *mc;
  double* dx[2];
  FilterCtl* ctl;
  ChunkRec* rec;
  MsgDesc* dd;
  for (int p = 0; p < 2; ++p) {
    CK(hipMalloc(&dS[p], S.size() * sizeof(T)));
    CK(hipMemcpy(dS[p], S.data(), S.size() * sizeof(T), hipMemcpyHostToDevice));
    CK(hipMalloc(&dx[p], n * sizeof(double)));
    CK(hipMemcpy(dx[p], x.data(), n * sizeof(double), hipMemcpyHostToDevice));
  }
  CK(hipMalloc(&kc, kMaxKW * ldk * sizeof(T)));
  CK(hipMalloc(&mc, kMaxKW * ldk * sizeof(T)));
  CK(hipMalloc(&ctl, sizeof(FilterCtl)));
  CK(hipMemset(ctl, 0, sizeof(FilterCtl)));
  CK(hipMalloc(&rec, 2 * sizeof(ChunkRec)));
  MsgDesc d{};
  d.m = m;
  d.flags = kActive | kFirst | kLast;
  d.parity = 0;
  for (int c = 0; c < m; ++c) {
    d.ids[c] = (c * 7) % N;
    const double lx = x[3 + 2 * d.ids[c]], ly = x[4 + 2 * d.ids[c]];
    d.z[c][0] = sqrt(lx * lx + ly * ly) + 0.001;
    d.z[c][1] = atan2(ly, lx) + 0.001;
  }
  CK(hipMalloc(&dd, sizeof(MsgDesc)));
  // record at parity 1 first (no kLook), then the timed chains rebuild from it (kLook, parity 0)
  d.parity = 1;
  CK(hipMemcpy(dd, &d, sizeof(MsgDesc), hipMemcpyHostToDevice));
  PassArgs<T> a{};
  a.sig[0] = dS[0]; a.sig[1] = dS[1]; a.sig_stride = 0;
  a.x[0] = dx[0]; a.x[1] = dx[1]; a.x_stride = 0;
  a.kcat = kc; a.mcat = mc; a.km_stride = 0; a.ldk = ldk;
  a.ctl = ctl; a.sync = sync_buf(4096); a.desc_stride = 1; a.rec = rec; a.rec_stride = 1; a.desc = dd; a.n = n; a.ld = ld; a.N = N; a.f0 = 0;
  a.q = 1e-2; a.r = 1e-2; a.gate = 2.0;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  CK(launch_chain<T>(a, 1, 1, s));
  CK(hipStreamSynchronize(s));
  if (g_look) {
    d.parity = 0;
    d.flags |= kLook;
    d.prev_m = m;
    for (int c = 0; c < m; ++c) d.prev_ids[c] = d.ids[c];
    CK(hipMemcpy(dd, &d, sizeof(MsgDesc), hipMemcpyHostToDevice));
  }
  for (int i = 0; i < 5; ++i) CK(launch_chain<T>(a, 1, 1, s));
  CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < reps; ++i) CK(launch_chain<T>(a, 1, 1, s));
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long st[160];
  CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof(st)));
  printf("N=%d m=%d %s: chain %.2f us/launch | A0 %llu A1 %llu endA %llu | per step (avg cycles):",
         N, m, sizeof(T) == 4 ? "f32" : "f64", ms * 1e3 / reps, st[1] - st[0], st[2] - st[0],
         st[40] - st[0]);
  const char* nm[6] = {"rb", "S+inv+xpre", "KMx+pub", "kx", "cross", "loop"};
  const int pts[7] = {64, 65, 66, 67, 68, 69, 70};
  for (int p = 0; p < 6; ++p) {
    double acc = 0;
    const int steps = m > 1 ? m - 1 : 1;  // stamps 68/69 exist only when a next step follows
    for (int c = 0; c < steps; ++c) {
      const unsigned long long a0 = st[pts[p] + 6 * c];
      const unsigned long long a1 = p < 5 ? st[pts[p + 1] + 6 * c] : (c + 1 < m ? st[64 + 6 * (c + 1)] : st[40]);
      acc += static_cast<double>(a1 - a0);
    }
    printf(" %s %.0f", nm[p], acc / (m > 1 ? m - 1 : 1));
  }
  printf("\n    prologue stamps (cycles from 0): A0 %llu loads+transform %llu K'M'-tiles %llu +x %llu P %llu\n",
         st[1] - st[0], st[3] - st[0], st[7] - st[0], st[5] - st[0], st[6] - st[0]);
  if (g_look == 2) {  // one launch walking C chunks (carry path), same markers every chunk
    const int C = 8;
    std::vector<MsgDesc> dv(C, d);
    for (int i = 0; i < C; ++i) {
      dv[i].parity = i & 1;
      dv[i].flags = (d.flags & ~kLook) | kLook;
    }
    MsgDesc* dm;
    CK(hipMalloc(&dm, C * sizeof(MsgDesc)));
    CK(hipMemcpy(dm, dv.data(), C * sizeof(MsgDesc), hipMemcpyHostToDevice));
    unsigned big = 0x40000000u;  // every Σ-pass epoch poll passes at once
    CK(hipMemcpy(a.sync + kSyncSigma, &big, sizeof(unsigned), hipMemcpyHostToDevice));
    PassArgs<T> ac = a;
    ac.desc = dm;
    CK(launch_chain<T>(ac, 1, C, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < reps / C; ++i) CK(launch_chain<T>(ac, 1, C, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("    carry: %.2f us/chunk (launches of %d chunks)\n", ms * 1e3 / (reps / C * C), C);
    CK(hipFree(dm));
  }
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < reps; ++i) CK(launch_factors<T>(a, 1, s));
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("    factors %.2f us/launch\n", ms * 1e3 / reps);
}

int main(int argc, char** argv) {
  if (argc > 1) g_look = atoi(argv[1]);
  printf("kLook %d\n", g_look);
  run<double>(50, 4, 200);
  run<double>(256, 16, 200);
  run<float>(1024, 16, 200);
  run<float>(1024, 1, 200);
  return 0;
}
