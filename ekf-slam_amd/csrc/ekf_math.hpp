// Device math shared by the EKF kernels (ekf_kernels.hip, ekf_resident.hip): the predict's
// pose and At entries, refined reciprocals, the range-bearing model and the 2×2 inverse.
#pragma once
#include <hip/hip_runtime.h>

#include "ekf_device.hpp"
#include "geom.hpp"

namespace ekfslam {

#define EKF_FLAG_RANGE_D 1u
#define EKF_FLAG_NUMERIC_D 2u

__device__ __forceinline__ double alpha_of(int idx, double a1, double a2) {
  return idx == 1 ? a1 : (idx == 2 ? a2 : 0.0);
}

// Predicted pose and the two nonzeros of At (slam.cpp:184-196). xin = posterior of the last
// message = filter_previous_configuration (slam.cpp:291).
__device__ __forceinline__ void predicted_pose(const double* tmo, int flags, const double* odom,
                                               const double* xin, double* pose, double* a1,
                                               double* a2) {
  if (flags & kFirst) {
    const Pose2 cur = compose(Pose2{tmo[0], tmo[1], tmo[2]},
                              Pose2{odom[0], odom[1], odom[2]});
    *a1 = -(cur.y - xin[2]);
    *a2 = cur.x - xin[1];
    pose[0] = normalize_angle(cur.theta);
    pose[1] = cur.x;
    pose[2] = cur.y;
  } else {
    *a1 = 0.0;
    *a2 = 0.0;
    pose[0] = xin[0];
    pose[1] = xin[1];
    pose[2] = xin[2];
  }
}
__device__ __forceinline__ void predicted_pose(const double* tmo, const MsgDesc& d,
                                               const double* xin, double* pose, double* a1,
                                               double* a2) {
  predicted_pose(tmo, d.flags, d.odom, xin, pose, a1, a2);
}

// 1/x and 1/√x from the hardware estimate plus two Newton steps (≤ 1 ulp; the f64 division
// sequence is ~3× longer and sits on the correction chain).
__device__ __forceinline__ double rcp_refined(double x) {
  double y = __builtin_amdgcn_rcp(x);
  double e = fma(-x, y, 1.0);
  y = fma(y, e, y);
  e = fma(-x, y, 1.0);
  return fma(y, e, y);
}
__device__ __forceinline__ double rsq_refined(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double h = 0.5 * x;
  double e = fma(-h * y, y, 0.5);
  y = fma(y, e, y);
  e = fma(-h * y, y, 0.5);
  return fma(y, e, y);
}

// Range-bearing model for landmark at (lx, ly) seen from pose: ẑ and the 2×5 H over
// {θ, x, y, jx, jy} (slam.cpp:219-249).
// bear_raw / bear_ok: the bearing before normalisation and whether the branch-free normalisation
// applied (|θ| ≤ π keeps it so); when not, the caller sets zhat[1] = normalize_angle(bear_raw).
__device__ __forceinline__ void range_bearing(const double* pose, double lx, double ly,
                                              double* zhat, double* H0, double* H1,
                                              double* bear_raw, bool* bear_ok) {
  const double ex = lx - pose[1], ey = ly - pose[2];
  const double d = ex * ex + ey * ey;
  const double isd = rsq_refined(d), id = isd * isd;
  zhat[0] = d * isd;
  *bear_raw = atan2_fast(ey, ex) - pose[0];
  zhat[1] = normalize_angle_near(*bear_raw, bear_ok);
  H0[0] = 0.0;
  H0[1] = -ex * isd;
  H0[2] = -ey * isd;
  H0[3] = ex * isd;
  H0[4] = ey * isd;
  H1[0] = -1.0;
  H1[1] = ey * id;
  H1[2] = -ex * id;
  H1[3] = -ey * id;
  H1[4] = ex * id;
}

// arma::inv on a 2×2 (closed form: adjugate / det, one reciprocal). false if singular / non-finite.
// inv2_calc: the adjugate / det without a test (returns det); inv2_ok: whether it was a valid inverse.
__device__ __forceinline__ double inv2_calc(const double* A, double* o) {
  const double det = A[0] * A[3] - A[1] * A[2];
  const double idet = rcp_refined(det);
  o[0] = A[3] * idet;
  o[1] = -A[1] * idet;
  o[2] = -A[2] * idet;
  o[3] = A[0] * idet;
  return det;
}
__device__ __forceinline__ bool inv2_ok(double det, const double* o) {
  return fabs(det) > 0.0 && isfinite(o[0]) && isfinite(o[1]) && isfinite(o[2]) && isfinite(o[3]);
}
__device__ __forceinline__ bool inv2(const double* A, double* o) {
  const double det = A[0] * A[3] - A[1] * A[2];
  if (!(fabs(det) > 0.0)) return false;
  inv2_calc(A, o);
  return inv2_ok(det, o);
}

// slam.cpp:364-401: d_k = νᵀ ψ⁻¹ ν for a landmark at (lx, ly) with P the 5×5 block of Σ over
// {θ, x, y, kx, ky}: ψ = (H·P)·Hᵀ + R (arma's left-to-right triple product), ν = z − ẑ with the
// bearing normalised; NaN when ψ is singular (never selected by the strict argmin). One expression
// for every association kernel (k_assoc, k_assoc_msg), so they decide alike.
__device__ __forceinline__ double assoc_dist(const double (&P)[5][5], const double* pose,
                                             double lx, double ly, double z0, double z1,
                                             double r_noise) {
  double zhat[2], H0[5], H1[5];
  double braw;
  bool bok;
  range_bearing(pose, lx, ly, zhat, H0, H1, &braw, &bok);
  if (!bok) zhat[1] = normalize_angle(braw);
  double HP0[5], HP1[5];
  for (int bb = 0; bb < 5; ++bb) {
    double s0 = 0.0, s1 = 0.0;
    for (int a = 0; a < 5; ++a) {
      s0 += H0[a] * P[a][bb];
      s1 += H1[a] * P[a][bb];
    }
    HP0[bb] = s0;
    HP1[bb] = s1;
  }
  double psi[4] = {0, 0, 0, 0};
  for (int b = 0; b < 5; ++b) {
    psi[0] += HP0[b] * H0[b];
    psi[1] += HP0[b] * H1[b];
    psi[2] += HP1[b] * H0[b];
    psi[3] += HP1[b] * H1[b];
  }
  psi[0] += r_noise;
  psi[3] += r_noise;
  const double nu0 = z0 - zhat[0];
  const double nu1 = normalize_angle(z1 - zhat[1]);
  // νᵀ·adj(ψ)·ν / det(ψ): arma's inv (adjugate / det) with the one division taken last
  double dist = NAN;
  const double det = psi[0] * psi[3] - psi[1] * psi[2];
  if (fabs(det) > 0.0) {
    const double t0 = nu0 * psi[3] - nu1 * psi[2];
    const double t1 = nu1 * psi[0] - nu0 * psi[1];
    dist = (t0 * nu0 + t1 * nu1) / det;
  }
  return dist;
}

// v − k0·m0 − k1·m1 with one fixed evaluation order (two FMAs), so a value rebuilt on the fly
// from the previous buffer is bit-identical to the one the block update stores.
__device__ __forceinline__ double rank2_sub(double v, double k0, double k1, double m0, double m1) {
  return fma(-k1, m1, fma(-k0, m0, v));
}

// geom.hpp's compose / inverse with one sincos (one argument reduction for both) — the same
// expressions, for device code where the trig sits on a latency chain
__device__ __forceinline__ Pose2 compose_sc(const Pose2& a, const Pose2& b) {
  double s, c;
  sincos(a.theta, &s, &c);
  Pose2 r;
  r.theta = a.theta + b.theta;
  r.x = c * b.x - s * b.y + a.x;
  r.y = s * b.x + c * b.y + a.y;
  return r;
}
__device__ __forceinline__ Pose2 inverse_sc(const Pose2& t) {
  double s, c;
  sincos(t.theta, &s, &c);
  Pose2 r;
  r.theta = -t.theta;
  r.x = -t.x * c - t.y * s;
  r.y = -t.y * c + t.x * s;
  return r;
}

// lane l's double, wave-uniform (v_readlane ×2)
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane(static_cast<int>(x), l);
  const int hi = __builtin_amdgcn_readlane(static_cast<int>(x >> 32), l);
  return __hiloint2double(hi, lo);
}

// wave argmin of (d, k): the smaller d, ties (and two +inf) to the lower k. A strict total order
// on the pairs, so any reduction tree gives the same pair: DPP row shifts 1, 2, 4, 8 (lane 15 of
// each row holds its row's minimum), row_bcast15 / row_bcast31 (lane 63 holds the wave's), then a
// broadcast — six steps of three 32-bit DPP moves instead of six rounds of three ds_bpermutes. A
// lane whose DPP source lies outside its row (or whose row the step masks off) combines with
// itself. Every lane of the wave must be active.
template <int CTRL, int ROWS>
__device__ __forceinline__ void argmin_dpp(double& d, int& k) {
  const long long b = __double_as_longlong(d);
  const int lo = static_cast<int>(b), hi = static_cast<int>(b >> 32);
  const int olo = __builtin_amdgcn_update_dpp(lo, lo, CTRL, ROWS, 0xf, false);
  const int ohi = __builtin_amdgcn_update_dpp(hi, hi, CTRL, ROWS, 0xf, false);
  const int ok = __builtin_amdgcn_update_dpp(k, k, CTRL, ROWS, 0xf, false);
  const double od = __longlong_as_double(static_cast<long long>(
      (static_cast<unsigned long long>(static_cast<unsigned>(ohi)) << 32) | static_cast<unsigned>(olo)));
  if (od < d || (od == d && ok < k)) {
    d = od;
    k = ok;
  }
}
__device__ __forceinline__ void wave_argmin(double& d, int& k) {
  argmin_dpp<0x111, 0xf>(d, k);  // row_shr:1
  argmin_dpp<0x112, 0xf>(d, k);  // row_shr:2
  argmin_dpp<0x114, 0xf>(d, k);  // row_shr:4
  argmin_dpp<0x118, 0xf>(d, k);  // row_shr:8
  argmin_dpp<0x142, 0xa>(d, k);  // row_bcast:15 into rows 1, 3
  argmin_dpp<0x143, 0xc>(d, k);  // row_bcast:31 into rows 2, 3
  d = readlane_f64(d, 63);
  k = __builtin_amdgcn_readlane(k, 63);
}

}  // namespace ekfslam
