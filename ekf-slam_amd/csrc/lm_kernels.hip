// HIP kernels (gfx950 / CDNA4) for the lidar landmark front-end of maxipalay/ekf-slam:
// nuslam/src/landmarks.cpp (getClusters :58-106, laserCallback :109-156) and
// turtlelib/src/landmark_detection.cpp (checkCircle :5-48, fitCircle :50-135).
//
// lm_detect is three launches:
//   k_clusters    one wavefront per scan: beams → points (LDS + global); break flags by ballot,
//                 break positions compacted in order (prefix popcount): cluster c is the run
//                 between breaks c−1 and c, the breaking point itself dropped (landmarks.cpp:81-86),
//                 the last run appended to cluster 0 when the scan closes on itself (:94-103);
//                 clusters of 4..39 points go to a dense batch-wide candidate list;
//   k_candidates  one lane per candidate of the whole batch: checkCircle, then the Hyper fit (a
//                 scan has ≈ 20 candidates, so per-scan lanes would leave two thirds of a wave idle);
//   k_markers     one wavefront per scan: ids (index among circle clusters, :147) and the publish
//                 filter (:145), compacted by ballot in cluster order.
// The fit never forms ZᵀZ: Z (n × 4) is reduced row by row to its 4 × 4 R factor with Givens
// rotations (orthogonal, registers only), the SVD of R comes from one-sided Jacobi (same singular
// values and V as Z's), and the 4 × 4 eigenproblem of Q = Y·H⁻¹·Y from cyclic Jacobi. Y⁻¹ = V·S⁻¹·Vᵀ
// replaces arma::solve (same vector in exact arithmetic; tolerances in tests/test_gpu_landmarks.py).
#include <hip/hip_runtime.h>

#include <cmath>

#include "geom.hpp"
#include "landmarks.h"
#include "lm_launch.hpp"

namespace lmk {

using ekfslam::normalize_angle;

constexpr double kLidarX = 0.032;   // landmarks.cpp:69
constexpr double kMaxR = 0.2;       // landmarks.cpp:145
constexpr double kMaxDist = 2.0;    // landmarks.cpp:145

__device__ __forceinline__ double sq(double v) { return v * v; }  // std::pow(v, 2): exact square

// 1/√x: hardware estimate + two Newton steps (≤ 1 ulp); replaces sqrt + two divisions in the
// rotations of the fit, whose latency chain bounds the front-end (one lane per cluster)
__device__ __forceinline__ double rsq_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
  double e = fma(-h * y, y, 0.5);
  y = fma(y, e, y);
  e = fma(-h * y, y, 0.5);
  return fma(y, e, y);
}

// arma accumulate / mean: two interleaved accumulators (even, odd), then (acc1 + acc2) / n
struct PairSum {
  double a = 0.0, b = 0.0;
  int k = 0;
  __device__ void add(double v) {
    if (k & 1) b += v; else a += v;
    ++k;
  }
  __device__ double sum() const { return a + b; }
};

// turtlelib::checkCircle (landmark_detection.cpp:5-48). pt(k) → (x, y) of the cluster's k-th point.
template <class P>
__device__ bool check_circle(int n, const P& pt) {
  const double2 p0 = pt(0), p1 = pt(n - 1);
  const double c = sqrt(sq(p0.x - p1.x) + sq(p0.y - p1.y));
  auto angle = [&](int j) {
    const double2 q = pt(j);
    const double a = sqrt(sq(p0.x - q.x) + sq(p0.y - q.y));
    const double b = sqrt(sq(p1.x - q.x) + sq(p1.y - q.y));
    return acos((c * c - a * a - b * b) / (-2.0 * a * b));
  };
  const int m = n - 2;
  // one pass (each acos once): sums of the angles shifted by the first one, then the mean and
  // the N − 1 variance from them; the same quantities as arma::mean / op_var::direct_var (whose
  // acc2, acc3 are these sums shifted by the mean), equal up to rounding of a 1e-16 relative size
  const double k0 = angle(1);
  PairSum s1, s2;
  for (int j = 2; j <= m; ++j) {
    const double t = angle(j) - k0;
    s1.add(t);
    s2.add(t * t);
  }
  const double mean = k0 + s1.sum() / m;  // arma::mean
  double var = 0.0;                       // arma::stddev (N − 1)
  if (m > 1) var = (s2.sum() - s1.sum() * s1.sum() / m) / (m - 1);
  const double sd = sqrt(var);
  return sd < 0.2 && 1.3 < mean && mean < 2.6;
}

// Streaming Givens QR: fold row w into the upper-triangular R (R ← the R factor of [R; w]).
__device__ __forceinline__ void givens_row(double (&R)[4][4], double (&w)[4]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (w[c] != 0.0) {
      const double r2 = fma(R[c][c], R[c][c], w[c] * w[c]);
      const double ir = rsq_nr(r2);
      const double cs = R[c][c] * ir, sn = w[c] * ir;
      R[c][c] = r2 * ir;
#pragma unroll
      for (int j = c + 1; j < 4; ++j) {
        const double t = R[c][j];
        R[c][j] = cs * t + sn * w[j];
        w[j] = cs * w[j] - sn * t;
      }
    }
  }
}

// turtlelib::fitCircle (landmark_detection.cpp:50-135): (c_x, c_y, R).
template <class P>
__device__ double3 fit_circle(int n, const P& pt) {
  PairSum sx, sy;
  for (int k = 0; k < n; ++k) {
    const double2 p = pt(k);
    sx.add(p.x);
    sy.add(p.y);
  }
  const double mx = sx.sum() / n, my = sy.sum() / n;  // arma::mean(cluster, 0)
  double B[4][4] = {};
  PairSum sz;
  for (int k = 0; k < n; ++k) {
    const double2 p = pt(k);
    const double x = p.x - mx, y = p.y - my, z = x * x + y * y;
    sz.add(z);
    double w[4] = {z, x, y, 1.0};  // the row of Z (:63-68)
    givens_row(B, w);
  }
  const double z_mean = sz.sum() / n;
  // one-sided Jacobi on R: B·V has orthogonal columns, their norms are Z's singular values
  double V[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
  for (int sweep = 0; sweep < 40; ++sweep) {
    bool rotated = false;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int q = p + 1; q < 4; ++q) {
        double al = 0.0, be = 0.0, ga = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          al = fma(B[i][p], B[i][p], al);
          be = fma(B[i][q], B[i][q], be);
          ga = fma(B[i][p], B[i][q], ga);
        }
        if (fabs(ga) > 1e-15 * sqrt(al * be)) {
          rotated = true;
          const double zeta = (be - al) / (2.0 * ga);
          const double t = copysign(1.0, zeta) / (fabs(zeta) + sqrt(fma(zeta, zeta, 1.0)));
          const double cs = rsq_nr(fma(t, t, 1.0)), sn = cs * t;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const double bp = B[i][p], bq = B[i][q];
            B[i][p] = cs * bp - sn * bq;
            B[i][q] = sn * bp + cs * bq;
            const double vp = V[i][p], vq = V[i][q];
            V[i][p] = cs * vp - sn * vq;
            V[i][q] = sn * vp + cs * vq;
          }
        }
      }
    if (!rotated) break;
  }
  double s[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) s[j] = sqrt(sq(B[0][j]) + sq(B[1][j]) + sq(B[2][j]) + sq(B[3][j]));
  // descending, like arma::svd's s (V's columns follow)
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3 - i; ++j) {
      const bool sw = s[j] < s[j + 1];
      const double a = s[j], b = s[j + 1];
      s[j] = sw ? b : a;
      s[j + 1] = sw ? a : b;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double u = V[k][j], v = V[k][j + 1];
        V[k][j] = sw ? v : u;
        V[k][j + 1] = sw ? u : v;
      }
    }
  double A[4];
  if (s[3] < 10.0e-12) {  // :97-98
#pragma unroll
    for (int k = 0; k < 4; ++k) A[k] = V[k][3];
  } else {
    // Y = V·diag(s)·Vᵀ (:100); Q = Y·H⁻¹·Y (:104) with H⁻¹ = [[0,0,0,½],[0,1,0,0],[0,0,1,0],[½,0,0,−2z̄]]
    double Y[4][4], YH[4][4], Q[4][4], E[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) acc = fma(V[i][k] * s[k], V[j][k], acc);
        Y[i][j] = acc;
      }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      YH[i][0] = 0.5 * Y[i][3];
      YH[i][1] = Y[i][1];
      YH[i][2] = Y[i][2];
      YH[i][3] = 0.5 * Y[i][0] - 2.0 * z_mean * Y[i][3];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) acc = fma(YH[i][k], Y[k][j], acc);
        Q[i][j] = acc;
        E[i][j] = i == j ? 1.0 : 0.0;
      }
#pragma unroll
    for (int i = 0; i < 4; ++i)  // exact symmetry for the two-sided rotations
#pragma unroll
      for (int j = i + 1; j < 4; ++j) Q[i][j] = Q[j][i] = 0.5 * (Q[i][j] + Q[j][i]);
    // cyclic Jacobi: eig_sym(Q) (:111)
    for (int sweep = 0; sweep < 50; ++sweep) {
      bool rotated = false;
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int q = p + 1; q < 4; ++q) {
          const double apq = Q[p][q];
          if (fabs(apq) > 1e-17 * (fabs(Q[p][p]) + fabs(Q[q][q])) && apq != 0.0) {
            rotated = true;
            const double th = (Q[q][q] - Q[p][p]) / (2.0 * apq);
            const double t = copysign(1.0, th) / (fabs(th) + sqrt(fma(th, th, 1.0)));
            const double cs = rsq_nr(fma(t, t, 1.0)), sn = t * cs;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const double kp = Q[k][p], kq = Q[k][q];
              Q[k][p] = cs * kp - sn * kq;
              Q[k][q] = sn * kp + cs * kq;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const double pk = Q[p][k], qk = Q[q][k];
              Q[p][k] = cs * pk - sn * qk;
              Q[q][k] = sn * pk + cs * qk;
            }
            Q[p][q] = Q[q][p] = 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const double ep = E[k][p], eq = E[k][q];
              E[k][p] = cs * ep - sn * eq;
              E[k][q] = sn * ep + cs * eq;
            }
          }
        }
      if (!rotated) break;
    }
    double w[4] = {Q[0][0], Q[1][1], Q[2][2], Q[3][3]};
    // ascending, like arma::eig_sym
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3 - i; ++j) {
        const bool sw = w[j] > w[j + 1];
        const double a = w[j], b = w[j + 1];
        w[j] = sw ? b : a;
        w[j + 1] = sw ? a : b;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const double u = E[k][j], v = E[k][j + 1];
          E[k][j] = sw ? v : u;
          E[k][j + 1] = sw ? u : v;
        }
      }
    // :113-121: the smallest positive eigenvalue below 1e7 (index 0 when there is none)
    int idx = 0;
    double mn = 10.0e6;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool take = w[i] < mn && w[i] > 0.0;
      mn = take ? w[i] : mn;
      idx = take ? i : idx;
    }
    double e[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      e[k] = idx == 0 ? E[k][0] : (idx == 1 ? E[k][1] : (idx == 2 ? E[k][2] : E[k][3]));
    // A = Y⁻¹·e = V·S⁻¹·Vᵀ·e (:122)
    double g[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      double acc = 0.0;
#pragma unroll
      for (int i = 0; i < 4; ++i) acc = fma(V[i][k], e[i], acc);
      g[k] = acc / s[k];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      double acc = 0.0;
#pragma unroll
      for (int k = 0; k < 4; ++k) acc = fma(V[i][k], g[k], acc);
      A[i] = acc;
    }
  }
  const double a = -A[1] / 2.0 / A[0];
  const double b = -A[2] / 2.0 / A[0];
  const double r2 = (A[1] * A[1] + A[2] * A[2] - 4.0 * A[0] * A[3]) / 4.0 / A[0] / A[0];
  return make_double3(a + mx, b + my, sqrt(r2));
}

// A cluster of the scan: up to two index runs (cluster 0 may wrap around the scan's end).
// A cluster of the scan: up to two index runs (cluster 0 may wrap around the scan's end).
struct Run2 {
  const double* px;
  const double* py;
  int s0, n0, s1;
  __device__ double2 operator()(int k) const {
    const int i = k < n0 ? s0 + k : s1 + (k - n0);
    return make_double2(px[i], py[i]);
  }
};

__device__ __forceinline__ unsigned long long lanes_below() {
  const int lane = threadIdx.x & 63;
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// Stage 1, one wavefront per scan: points (LDS and global), breaks, clusters; clusters of 4..39
// points are appended, in cluster order, to the candidate list of region s mod kRegions (one
// atomic per scan; a single counter for 4096 scans serialised ≈ 40 µs of same-address atomics).
__global__ __launch_bounds__(64) void k_clusters(const float* __restrict__ ranges, int B,
                                                const double* __restrict__ amin,
                                                const double* __restrict__ ainc, double thr,
                                                double* __restrict__ gpx, double* __restrict__ gpy,
                                                Cand* __restrict__ cand, int* __restrict__ gcount,
                                                int regcap, int* __restrict__ sbase,
                                                int* __restrict__ sncand) {
  // dynamic LDS sized to the scan (B·20 bytes: 7.2 KB at 360 beams), so a CU holds many scans
  extern __shared__ double lds[];
  const int s = blockIdx.x, lane = threadIdx.x;
  double* px = lds;
  double* py = lds + B;
  int* bpos = reinterpret_cast<int*>(lds + 2 * B);
  const float* rs = ranges + static_cast<size_t>(s) * B;
  double* gx = gpx + static_cast<size_t>(s) * B;
  double* gy = gpy + static_cast<size_t>(s) * B;
  const double a0 = amin[s], inc = ainc[s];
  for (int i = lane; i < B; i += 64) {  // landmarks.cpp:66-70
    const double r = static_cast<double>(rs[i]);
    const double a = normalize_angle(static_cast<double>(i) * inc) + a0;
    double sa, ca;
    sincos(a, &sa, &ca);
    const double x = r * ca - kLidarX, y = r * sa;
    px[i] = x;
    py[i] = y;
    gx[i] = x;
    gy[i] = y;
  }
  __syncthreads();
  int nb = 0;  // breaks, compacted in scan order (:78-86)
  for (int base = 0; base < B; base += 64) {
    const int i = base + lane;
    bool brk = false;
    if (i >= 1 && i < B) brk = !(sqrt(sq(px[i] - px[i - 1]) + sq(py[i] - py[i - 1])) <= thr);
    const unsigned long long bal = __ballot(brk);
    if (brk) bpos[nb + __popcll(bal & lanes_below())] = i;
    nb += __popcll(bal);
  }
  __syncthreads();
  if (nb == 0) {  // clusters.at(0) on an empty list throws in the reference (:94)
    if (lane == 0) sncand[s] = LM_NO_BREAK;
    return;
  }
  const bool merged = sqrt(sq(px[0] - px[B - 1]) + sq(py[0] - py[B - 1])) <= thr;  // :96
  const int ncl = merged ? nb : nb + 1;
  auto cluster = [&](int c, int* s0, int* n0, int* s1) {  // cluster c's runs; returns its size
    *s0 = c == 0 ? 0 : bpos[c - 1] + 1;
    *n0 = (c == nb ? B : bpos[c]) - *s0;
    *s1 = bpos[nb - 1] + 1;
    const int n1 = (c == 0 && merged) ? B - *s1 : 0;
    return *n0 + n1;
  };
  int total = 0;  // pass 1: how many candidates (:122, the size test)
  for (int cb = 0; cb < ncl; cb += 64) {
    int s0, n0, s1, n = 0;
    if (cb + lane < ncl) n = cluster(cb + lane, &s0, &n0, &s1);
    total += __popcll(__ballot(n > 3 && n < 40));
  }
  int base = 0;
  const int reg = s % kRegions;
  if (lane == 0) base = reg * regcap + atomicAdd(gcount + reg, total);
  base = __shfl(base, 0);
  if (lane == 0) {
    sbase[s] = base;
    sncand[s] = total;
  }
  int k = base;  // pass 2: the candidates, in cluster order
  for (int cb = 0; cb < ncl; cb += 64) {
    int s0 = 0, n0 = 0, s1 = 0, n = 0;
    if (cb + lane < ncl) n = cluster(cb + lane, &s0, &n0, &s1);
    const bool cd = n > 3 && n < 40;
    const unsigned long long bal = __ballot(cd);
    if (cd) {
      Cand e;
      e.scan = s;
      e.s0 = s0;
      e.n0 = n0;
      e.s1 = s1;
      e.n = n;
      e.pass = 0;
      e.cx = e.cy = e.r = 0.0;
      cand[k + __popcll(bal & lanes_below())] = e;
    }
    k += __popcll(bal);
  }
}

// Stage 2, one lane per candidate over the whole batch (dense per region): checkCircle, then the
// Hyper fit.
__global__ __launch_bounds__(64) void k_candidates(int B, const double* __restrict__ gpx,
                                                  const double* __restrict__ gpy,
                                                  Cand* __restrict__ cand,
                                                  const int* __restrict__ gcount, int regcap) {
  // lanes interleave the regions (lane → region idx mod kRegions, entry idx / kRegions), so the
  // occupied entries of every region come first in the grid and the empty tail retires at once
  const int idx = blockIdx.x * 64 + threadIdx.x;
  const int reg = idx % kRegions, k = idx / kRegions;
  if (k >= regcap || k >= gcount[reg]) return;
  const int slot = reg * regcap + k;
  Cand e = cand[slot];
  const size_t o = static_cast<size_t>(e.scan) * B;
  const Run2 g{gpx + o, gpy + o, e.s0, e.n0, e.s1};
  e.pass = check_circle(e.n, g) ? 1 : 0;  // :123
  if (e.pass) {
    const double3 f = fit_circle(e.n, g);  // :144
    e.cx = f.x;
    e.cy = f.y;
    e.r = f.z;
  }
  cand[slot] = e;
}

// Stage 3, one wavefront per scan: marker ids (index among circle clusters, :147) and the publish
// filter (R < 0.2, centre within 2 m, :145), compacted by ballot in cluster order.
__global__ __launch_bounds__(64) void k_markers(const Cand* __restrict__ cand,
                                               const int* __restrict__ sbase,
                                               const int* __restrict__ sncand,
                                               lm_marker* __restrict__ out, int max_markers,
                                               int* __restrict__ counts) {
  const int s = blockIdx.x, lane = threadIdx.x;
  const int nc = sncand[s];
  if (nc < 0) {
    if (lane == 0) counts[s] = LM_NO_BREAK;
    return;
  }
  const Cand* cs = cand + sbase[s];
  lm_marker* o = out + static_cast<size_t>(s) * max_markers;
  int id_base = 0, pub_base = 0;
  for (int cb = 0; cb < nc; cb += 64) {
    Cand e;
    e.pass = 0;
    if (cb + lane < nc) e = cs[cb + lane];
    const bool cand_ok = e.pass != 0;
    const unsigned long long bc = __ballot(cand_ok);
    const int id = id_base + __popcll(bc & lanes_below());
    const bool pub = cand_ok && e.r < kMaxR && sqrt(sq(e.cx) + sq(e.cy)) < kMaxDist;
    const unsigned long long bp = __ballot(pub);
    const int slot = pub_base + __popcll(bp & lanes_below());
    if (pub && slot < max_markers) {
      lm_marker m;
      m.x = e.cx;
      m.y = e.cy;
      m.r = e.r;
      m.id = id;
      m.pad = 0;
      o[slot] = m;
    }
    id_base += __popcll(bc);
    pub_base += __popcll(bp);
  }
  if (lane == 0) counts[s] = pub_base;
}

// Arbitrary point sets (lm_fit_circles / lm_check_circles): one lane per cluster.
struct Flat {
  const double* xy;
  int off;
  __device__ double2 operator()(int k) const {
    return make_double2(xy[2 * (off + k)], xy[2 * (off + k) + 1]);
  }
};

__global__ __launch_bounds__(64) void k_fit(int nc, const int* __restrict__ offs,
                                           const double* __restrict__ xy, double* __restrict__ out) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (c >= nc) return;
  const int n = offs[c + 1] - offs[c];
  const double3 f = fit_circle(n, Flat{xy, offs[c]});
  out[3 * c] = f.x;
  out[3 * c + 1] = f.y;
  out[3 * c + 2] = f.z;
}

__global__ __launch_bounds__(64) void k_check(int nc, const int* __restrict__ offs,
                                             const double* __restrict__ xy, int* __restrict__ out) {
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (c >= nc) return;
  const int n = offs[c + 1] - offs[c];
  out[c] = check_circle(n, Flat{xy, offs[c]}) ? 1 : 0;
}

hipError_t launch_detect(const float* ranges, int S, int B, const double* amin,
                         const double* ainc, double thr, lm_marker* out, int max_markers,
                         int* counts, const DetectWork& w, hipStream_t st) {
  if (hipMemsetAsync(w.gcount, 0, sizeof(int) * kRegions, st) != hipSuccess)
    return hipErrorUnknown;
  const int regcap = (S + kRegions - 1) / kRegions * max_candidates(B);
  const size_t lds = static_cast<size_t>(B) * (2 * sizeof(double) + sizeof(int));
  hipLaunchKernelGGL(k_clusters, dim3(S), dim3(64), lds, st, ranges, B, amin, ainc, thr, w.px,
                     w.py, w.cand, w.gcount, regcap, w.sbase, w.sncand);
  const size_t cap = static_cast<size_t>(kRegions) * regcap;  // bound of the regions' lists
  hipLaunchKernelGGL(k_candidates, dim3((cap + 63) / 64), dim3(64), 0, st, B, w.px, w.py, w.cand,
                     w.gcount, regcap);
  hipLaunchKernelGGL(k_markers, dim3(S), dim3(64), 0, st, w.cand, w.sbase, w.sncand, out,
                     max_markers, counts);
  return hipGetLastError();
}

hipError_t launch_fit(int nc, const int* offs, const double* xy, double* out, hipStream_t st) {
  hipLaunchKernelGGL(k_fit, dim3((nc + 63) / 64), dim3(64), 0, st, nc, offs, xy, out);
  return hipGetLastError();
}

hipError_t launch_check(int nc, const int* offs, const double* xy, int* out, hipStream_t st) {
  hipLaunchKernelGGL(k_check, dim3((nc + 63) / 64), dim3(64), 0, st, nc, offs, xy, out);
  return hipGetLastError();
}

}  // namespace lmk
