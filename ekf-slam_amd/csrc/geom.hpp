// SE(2) geometry and differential-drive odometry, host + device.
//
// Same semantics as the reference's turtlelib (maxipalay/ekf-slam), written fresh for use on both
// sides of the HIP boundary:
//   normalize_angle   turtlelib/src/geometry2d.cpp:5-14   (fmod based, maps into (-π, π], -π → π)
//   Pose2 compose     turtlelib/src/se2d.cpp:66-75        (Transform2D::operator*=; θ not wrapped)
//   Pose2 inverse     turtlelib/src/se2d.cpp:57-63        (Transform2D::inv)
//   integrate_twist   turtlelib/src/se2d.cpp:127-138
//   DiffDrive::fkin   turtlelib/src/diff_drive.cpp:10-28
//   DiffDrive::ikin   turtlelib/src/diff_drive.cpp:30-38  (host only; throws on lateral twist)
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

namespace ekfslam {

constexpr double kPi = 3.14159265358979323846;

// fmod(x, 2π) without the generic frexp loop: for |x| < 5π the result x − k·2π (k ≤ 2) is exact in
// floating point (Sterbenz), so this returns fmod's bits, sign of zero included.
__host__ __device__ inline double fmod_2pi(double x) {
  const double y = 2.0 * kPi;
  const double ax = fabs(x);
  if (ax < y) return x;
  if (ax < 2.0 * y) return copysign(ax - y, x);
  if (ax < 2.5 * y) return copysign(ax - 2.0 * y, x);
  return fmod(x, y);
}

__host__ __device__ inline double normalize_angle(double rad) {
  const double d = fmod_2pi(rad + kPi);
  return d <= 0.0 ? d + kPi : d - kPi;
}

// normalize_angle for |rad + π| < 5π, branch-free (selects): the same bits as normalize_angle
// there; *ok is false outside, where the caller falls back to normalize_angle.
__host__ __device__ inline double normalize_angle_near(double rad, bool* ok) {
  const double y = 2.0 * kPi;
  const double x = rad + kPi, ax = fabs(x);
  *ok = ax < 2.5 * y;
  const double d = ax < y ? x : copysign(ax < 2.0 * y ? ax - y : ax - 2.0 * y, x);
  return d <= 0.0 ? d + kPi : d - kPi;
}

// atan2 in ~40 f64 operations (one reciprocal) for the bearing of every EKF step; max error
// 0.59 ulp for the reduced atan polynomial (fitted at 60 digits by tools/fit_atan.py), a few ulp
// overall (Estrin evaluation and the refined reciprocal each add rounding).
// ocml's atan2 costs ~190 f64 operations and sits on the correction chain's critical path.
__host__ __device__ inline double atan2_fast(double y, double x) {
  constexpr double kC[11] = {
      -0.3333333333333333,   0.19999999999995652,  -0.1428571428469138,   0.11111111017100327,
      -0.0909090464769568,   0.07692184699371778,  -0.06664531369805009,  0.05858311810501153,
      -0.05086254885823143,  0.039253696320618564, -0.01920252926841228};
  const double ax = fabs(x), ay = fabs(y);
  const bool swap = ay > ax;
  const double num = swap ? ax : ay, den = swap ? ay : ax;  // t = num/den ∈ [0, 1]
  // atan(t) = π/4 + atan((t−1)/(t+1)) above tan(π/8); selects, one division, no branch
  const bool hi = num > 0.41421356237309503 * den;
  const double tn = hi ? num - den : num, td = hi ? num + den : (den > 0.0 ? den : 1.0);
#ifdef __HIP_DEVICE_COMPILE__
  // reciprocal with two Newton steps (≤ 1 ulp) and a product: 6 operations against the 10 of the
  // IEEE division sequence on the correction chain
  double ri = __builtin_amdgcn_rcp(td);
  ri = fma(ri, fma(-td, ri, 1.0), ri);
  ri = fma(ri, fma(-td, ri, 1.0), ri);
  const double tq = tn * ri;
#else
  const double tq = tn / td;
#endif
  const double t = hi || den > 0.0 ? tq : 0.0;
  const double off = hi ? 0.78539816339744831 : 0.0;
  const double z = t * t;
  // Estrin's scheme: independent pairs, then powers of z (fewer dependent steps than Horner)
  const double z2 = z * z, z4 = z2 * z2, z8 = z4 * z4;
  const double p01 = fma(kC[1], z, kC[0]), p23 = fma(kC[3], z, kC[2]);
  const double p45 = fma(kC[5], z, kC[4]), p67 = fma(kC[7], z, kC[6]);
  const double p89 = fma(kC[9], z, kC[8]);
  const double p03 = fma(p23, z2, p01), p47 = fma(p67, z2, p45);
  const double p8a = fma(kC[10], z2, p89);
  const double r = fma(p8a, z8, fma(p47, z4, p03));
  double a = off + fma(t * z, r, t);
  if (swap) a = 1.5707963267948966 - a;
  if (x < 0.0) a = kPi - a;
  return copysign(a, y);
}

// A planar rigid transform {θ, x, y} (turtlelib Transform2D).
struct Pose2 {
  double theta = 0.0, x = 0.0, y = 0.0;
};

struct Twist2 {
  double omega = 0.0, vx = 0.0, vy = 0.0;
};

__host__ __device__ inline Pose2 compose(const Pose2& a, const Pose2& b) {
  const double c = cos(a.theta), s = sin(a.theta);
  Pose2 r;
  r.theta = a.theta + b.theta;
  r.x = c * b.x - s * b.y + a.x;
  r.y = s * b.x + c * b.y + a.y;
  return r;
}

__host__ __device__ inline Pose2 inverse(const Pose2& t) {
  const double c = cos(t.theta), s = sin(t.theta);
  Pose2 r;
  r.theta = -t.theta;
  r.x = -t.x * c - t.y * s;
  r.y = -t.y * c + t.x * s;
  return r;
}

// Exact integration of a body twist over unit time.
__host__ __device__ inline Pose2 integrate_twist(const Twist2& tw) {
  if (tw.omega == 0.0) return Pose2{0.0, tw.vx, tw.vy};
  const Pose2 tsb{0.0, tw.vy / tw.omega, -tw.vx / tw.omega};
  return compose(compose(inverse(tsb), Pose2{tw.omega, 0.0, 0.0}), tsb);
}

struct WheelSpeeds {
  double left = 0.0, right = 0.0;
};

class DiffDrive {
 public:
  __host__ __device__ DiffDrive(double track = 0.160, double radius = 0.033)
      : track_(track), radius_(radius) {}

  // Wheel angles → body twist → exact arc → config ← config · Δ.
  __host__ __device__ Pose2 fkin(double rad_left, double rad_right) {
    const double dl = rad_left - phi_l_, dr = rad_right - phi_r_;
    const Twist2 tw{radius_ / track_ * (-dl + dr), radius_ / 2.0 * (dl + dr), 0.0};
    config_ = compose(config_, integrate_twist(tw));
    phi_l_ = rad_left;
    phi_r_ = rad_right;
    return config_;
  }

  // Body twist → wheel velocities. Returns false on a twist with lateral velocity (the reference
  // throws std::logic_error there, diff_drive.cpp:31-33).
  __host__ bool ikin(const Twist2& tw, WheelSpeeds* out) const {
    if (std::fabs(tw.vy) > 1e-12) return false;
    out->left = -track_ / 2.0 / radius_ * tw.omega + 1.0 / radius_ * tw.vx;
    out->right = track_ / 2.0 / radius_ * tw.omega + 1.0 / radius_ * tw.vx;
    return true;
  }

  __host__ __device__ Pose2 config() const { return config_; }
  __host__ __device__ void set_config(const Pose2& p) { config_ = p; }

 private:
  double track_, radius_;
  double phi_l_ = 0.0, phi_r_ = 0.0;
  Pose2 config_{};
};

}  // namespace ekfslam
