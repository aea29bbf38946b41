// HIP kernels (gfx950 / CDNA4) for the lidar landmark front-end of maxipalay/ekf-slam:
// nuslam/src/landmarks.cpp (getClusters :58-106, laserCallback :109-156) and
// turtlelib/src/landmark_detection.cpp (checkCircle :5-48, fitCircle :50-135).
//
// k_detect: one wavefront per scan.
//   1. beams → points in LDS (64 lanes stride the scan);
//   2. break flags by ballot, break positions compacted in order (prefix popcount): cluster c is
//      the run between breaks c−1 and c, the breaking point itself dropped (landmarks.cpp:81-86),
//      the last run appended to cluster 0 when the scan closes on itself (:94-103);
//   3. one lane per cluster: checkCircle, then the Hyper fit, numbered and compacted by ballot in
//      cluster order (the marker id of :147 and the publish filter of :145).
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
  PairSum s;
  for (int j = 1; j <= m; ++j) s.add(angle(j));
  const double mean = s.sum() / m;  // arma::mean
  double var = 0.0;                 // arma::stddev (N − 1), op_var::direct_var
  if (m > 1) {
    PairSum a2, a3;
    for (int j = 1; j <= m; ++j) {
      const double t = mean - angle(j);
      a2.add(t * t);
      a3.add(t);
    }
    // the pair sums of direct_var add tmpi² + tmpj² per pair; same terms, rounding-level order
    var = (a2.sum() - a3.sum() * a3.sum() / m) / (m - 1);
  }
  const double sd = sqrt(var);
  return sd < 0.2 && 1.3 < mean && mean < 2.6;
}

// Streaming Givens QR: fold row w into the upper-triangular R (R ← the R factor of [R; w]).
__device__ __forceinline__ void givens_row(double (&R)[4][4], double (&w)[4]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (w[c] != 0.0) {
      const double r = sqrt(fma(R[c][c], R[c][c], w[c] * w[c]));
      const double cs = R[c][c] / r, sn = w[c] / r;
      R[c][c] = r;
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
          const double cs = 1.0 / sqrt(fma(t, t, 1.0)), sn = cs * t;
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
            const double cs = 1.0 / sqrt(fma(t, t, 1.0)), sn = t * cs;
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

__global__ __launch_bounds__(64) void k_detect(const float* __restrict__ ranges, int nb_beams,
                                              const double* __restrict__ amin,
                                              const double* __restrict__ ainc, double thr,
                                              lm_marker* __restrict__ out, int max_markers,
                                              int* __restrict__ counts) {
  // dynamic LDS sized to the scan (B·20 bytes: 7.2 KB at 360 beams), so a CU holds many scans
  extern __shared__ double lds[];
  const int s = blockIdx.x, lane = threadIdx.x;
  const int B = nb_beams;
  double* px = lds;
  double* py = lds + B;
  int* bpos = reinterpret_cast<int*>(lds + 2 * B);
  const float* rs = ranges + static_cast<size_t>(s) * B;
  const double a0 = amin[s], inc = ainc[s];
  for (int i = lane; i < B; i += 64) {  // landmarks.cpp:66-70
    const double r = static_cast<double>(rs[i]);
    const double a = normalize_angle(static_cast<double>(i) * inc) + a0;
    px[i] = r * cos(a) - kLidarX;
    py[i] = r * sin(a);
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
    if (lane == 0) counts[s] = LM_NO_BREAK;
    return;
  }
  const bool merged = sqrt(sq(px[0] - px[B - 1]) + sq(py[0] - py[B - 1])) <= thr;  // :96
  const int ncl = merged ? nb : nb + 1;
  int id_base = 0, pub_base = 0;
  lm_marker* o = out + static_cast<size_t>(s) * max_markers;
  for (int cb = 0; cb < ncl; cb += 64) {
    const int c = cb + lane;
    Run2 g{px, py, 0, 0, 0};
    int n = 0;
    if (c < ncl) {
      g.s0 = c == 0 ? 0 : bpos[c - 1] + 1;
      g.n0 = (c == nb ? B : bpos[c]) - g.s0;
      const int n1 = (c == 0 && merged) ? B - (bpos[nb - 1] + 1) : 0;
      g.s1 = bpos[nb - 1] + 1;
      n = g.n0 + n1;
    }
    const bool cand = n > 3 && n < 40 && check_circle(n, g);  // :122-123
    const unsigned long long bc = __ballot(cand);
    const int id = id_base + __popcll(bc & lanes_below());
    double3 f = make_double3(0.0, 0.0, 0.0);
    if (cand) f = fit_circle(n, g);
    const bool pub = cand && f.z < kMaxR && sqrt(sq(f.x) + sq(f.y)) < kMaxDist;  // :145
    const unsigned long long bp = __ballot(pub);
    const int slot = pub_base + __popcll(bp & lanes_below());
    if (pub && slot < max_markers) {
      lm_marker m;
      m.x = f.x;
      m.y = f.y;
      m.r = f.z;
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
                         int* counts, hipStream_t st) {
  const size_t lds = static_cast<size_t>(B) * (2 * sizeof(double) + sizeof(int));
  hipLaunchKernelGGL(k_detect, dim3(S), dim3(64), lds, st, ranges, B, amin, ainc, thr, out,
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
