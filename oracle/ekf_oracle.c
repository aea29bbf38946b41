/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see ekf_oracle.h for the parity status and the rules on who
 * may load this file). CPU restatement of nuslam/src/slam.cpp (maxipalay/ekf-slam) in plain C.
 *
 * Two arithmetic modes of the same filter:
 *   literal    — the dense algebra exactly as slam.cpp writes it: At*Σ*Atᵀ (slam.cpp:194-198),
 *                K = Σ Hᵀ inv(HΣHᵀ+R) with a dense 2×n H (slam.cpp:240-252), Σ ← (I−KH)Σ as a dense
 *                n×n×n product (slam.cpp:264-265). O(n³) per correction. This is the CPU baseline
 *                "the reference's own algorithm" (bench.py cpu_baseline).
 *   structured — the same math with the zeros of At and H skipped: O(n) predict, O(n²) rank-2
 *                correction. Same results up to rounding.
 *
 * Layout: Σ row-major n×n (the reference uses Armadillo column-major; layout does not change the
 * math). State order [θ, x, y, m1x, m1y, …] (slam.cpp:186-188).
 */
#include "ekf_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define ORC_MARKER_DELETE 2 /* visualization_msgs::msg::Marker::DELETE */

static const double PI = 3.14159265358979323846;  /* turtlelib/include/turtlelib/geometry2d.hpp PI */

/* turtlelib/src/geometry2d.cpp:5-14 */
double orc_normalize_angle(double rad) {
  double diff = fmod(rad + PI, 2.0 * PI);
  if (diff <= 0.0) return diff + PI;
  return diff - PI;
}

/* turtlelib/src/se2d.cpp:66-75 (operator*=), :123-125 (operator*). Transforms are {θ, x, y}. */
void orc_tf_compose(const double* lhs, const double* rhs, double* out) {
  const double c = cos(lhs[0]), s = sin(lhs[0]);
  const double th = lhs[0] + rhs[0];
  const double x = c * rhs[1] - s * rhs[2] + lhs[1];
  const double y = s * rhs[1] + c * rhs[2] + lhs[2];
  out[0] = th;
  out[1] = x;
  out[2] = y;
}

/* turtlelib/src/se2d.cpp:57-63 */
void orc_tf_inv(const double* t, double* out) {
  const double c = cos(t[0]), s = sin(t[0]);
  const double x = -t[1] * c - t[2] * s;
  const double y = -t[2] * c + t[1] * s;
  out[0] = -t[0];
  out[1] = x;
  out[2] = y;
}

/* turtlelib/src/se2d.cpp:127-138 */
void orc_integrate_twist(double omega, double vx, double vy, double* out) {
  if (omega == 0.0) {
    out[0] = 0.0;
    out[1] = vx;
    out[2] = vy;
    return;
  }
  const double tsb[3] = {0.0, vy / omega, -vx / omega};
  double tbs[3], tss[3] = {omega, 0.0, 0.0}, tmp[3];
  orc_tf_inv(tsb, tbs);
  orc_tf_compose(tbs, tss, tmp); /* Tbs * Tssprime */
  orc_tf_compose(tmp, tsb, out); /* (...) * Tsb    */
}

/* turtlelib/src/diff_drive.cpp:10-28. dd = {track, radius, phi_l, phi_r, θ, x, y}. */
void orc_fkin(double* dd, double rad_left, double rad_right, double* out) {
  const double track = dd[0], radius = dd[1];
  const double dl = rad_left - dd[2];
  const double dr = rad_right - dd[3];
  const double omega = radius / track * (-dl + dr);
  const double vx = radius / 2.0 * (dl + dr);
  double tf[3], cfg[3] = {dd[4], dd[5], dd[6]}, ncfg[3];
  orc_integrate_twist(omega, vx, 0.0, tf);
  orc_tf_compose(cfg, tf, ncfg); /* config *= tf */
  dd[4] = ncfg[0];
  dd[5] = ncfg[1];
  dd[6] = ncfg[2];
  dd[2] = rad_left;
  dd[3] = rad_right;
  out[0] = ncfg[0];
  out[1] = ncfg[1];
  out[2] = ncfg[2];
}

/* ------------------------------------------------------------------------------------------ */

struct orc_ekf {
  int N, n;
  double q, r, init_var, gate;
  int literal;
  int joseph;     /* Joseph-form Σ update (opt-in; the reference uses (I − KH)Σ) */
  double* x;      /* n    */
  double* S;      /* n×n  */
  double* T1;     /* n×n scratch (literal mode) */
  double* T2;     /* n×n scratch (literal mode) */
  double* PHt;    /* n×2  */
  double* HP;     /* 2×n  */
  double* H;      /* 2×n dense (literal mode) */
  double* PH0;    /* n×2 : Σ·Hᵀ kept for the Joseph form (PHt is overwritten by K) */
  unsigned counter;      /* counter_obstacles, slam.cpp:670 */
  double last_dmin;      /* the last association's smallest existing d_k (test diagnostics) */
  double tmo[3];         /* t_map_odom, slam.cpp:659 */
  double prev[3];        /* filter_previous_configuration, slam.cpp:660 */
  double todom[3];       /* t_odom_robot, slam.cpp:650 */
};

/* Row-major C = A·B, n×n, blocked; OpenMP over row blocks when compiled with -fopenmp. */
static void gemm_nn(int n, const double* A, const double* B, double* C) {
  const int BI = 64, BK = 128;
#pragma omp parallel for schedule(static)
  for (int i0 = 0; i0 < n; i0 += BI) {
    const int i1 = i0 + BI < n ? i0 + BI : n;
    for (int i = i0; i < i1; ++i) memset(C + (size_t)i * n, 0, sizeof(double) * n);
    for (int k0 = 0; k0 < n; k0 += BK) {
      const int k1 = k0 + BK < n ? k0 + BK : n;
      for (int i = i0; i < i1; ++i) {
        double* c = C + (size_t)i * n;
        for (int k = k0; k < k1; ++k) {
          const double a = A[(size_t)i * n + k];
          const double* b = B + (size_t)k * n;
          for (int j = 0; j < n; ++j) c[j] += a * b[j];
        }
      }
    }
  }
}

orc_ekf* orc_ekf_create(int n_landmarks, double q_noise, double r_noise, double init_var,
                        double mah_gate, int literal) {
  orc_ekf* f = (orc_ekf*)calloc(1, sizeof(orc_ekf));
  const int n = 3 + 2 * n_landmarks;
  f->N = n_landmarks;
  f->n = n;
  f->q = q_noise;
  f->r = r_noise;
  f->init_var = init_var;
  f->gate = mah_gate;
  f->literal = literal;
  f->x = (double*)calloc(n, sizeof(double));
  f->S = (double*)calloc((size_t)n * n, sizeof(double));
  f->PHt = (double*)calloc((size_t)n * 2, sizeof(double));
  f->HP = (double*)calloc((size_t)n * 2, sizeof(double));
  f->H = (double*)calloc((size_t)n * 2, sizeof(double));
  f->PH0 = (double*)calloc((size_t)n * 2, sizeof(double));
  if (literal) {
    f->T1 = (double*)calloc((size_t)n * n, sizeof(double));
    f->T2 = (double*)calloc((size_t)n * n, sizeof(double));
  }
  /* Σ₀ = diag(0,0,0, init_var·I_2N): slam.cpp:128-132 (init_var is the literal 10e6 = 1e7) */
  for (int i = 3; i < n; ++i) f->S[(size_t)i * n + i] = init_var;
  return f;
}

void orc_ekf_destroy(orc_ekf* f) {
  if (!f) return;
  free(f->x); free(f->S); free(f->PHt); free(f->HP); free(f->H); free(f->T1); free(f->T2);
  free(f->PH0);
  free(f);
}

int orc_ekf_dim(const orc_ekf* f) { return f->n; }

/* Joseph form, opt-in (BASELINE.json north_star; SURVEY.md §8b `joseph`): Σ ← (I−KH)Σ(I−KH)ᵀ + KRKᵀ
 * in place of slam.cpp:264-265's (I−KH)Σ. Equal in exact arithmetic with the optimal gain. */
void orc_ekf_set_joseph(orc_ekf* f, int on) {
  f->joseph = on;
  if (on && f->literal && !f->T1) {
    f->T1 = (double*)calloc((size_t)f->n * f->n, sizeof(double));
    f->T2 = (double*)calloc((size_t)f->n * f->n, sizeof(double));
  }
}

void orc_ekf_set_odom(orc_ekf* f, double theta, double x, double y) {
  f->todom[0] = theta; f->todom[1] = x; f->todom[2] = y;
}

/* slam.cpp:184-198 (identical block at :321-335). */
void orc_ekf_predict(orc_ekf* f) {
  const int n = f->n;
  double cur[3];
  orc_tf_compose(f->tmo, f->todom, cur);                /* :184 t_map_odom * t_odom_robot */
  f->x[0] = orc_normalize_angle(cur[0]);                /* :186 */
  f->x[1] = cur[1];                                     /* :187 */
  f->x[2] = cur[2];                                     /* :188 */
  const double dx = cur[1] - f->prev[1];                /* :190 */
  const double dy = cur[2] - f->prev[2];                /* :191 */
  double* S = f->S;
  if (f->literal) {
    /* At = I; At(1,0) = -dy; At(2,0) = dx; Σ = At*Σ*Atᵀ + Q̄  (:194-198) */
    double* At = f->T1;
    memset(At, 0, sizeof(double) * (size_t)n * n);
    for (int i = 0; i < n; ++i) At[(size_t)i * n + i] = 1.0;
    At[(size_t)1 * n + 0] = -dy;
    At[(size_t)2 * n + 0] = dx;
    gemm_nn(n, At, S, f->T2);                 /* T2 = At*Σ */
    /* Atᵀ in place of At */
    At[(size_t)1 * n + 0] = 0.0; At[(size_t)2 * n + 0] = 0.0;
    At[1] = -dy; At[2] = dx;
    gemm_nn(n, f->T2, At, S);                 /* Σ = (At*Σ)*Atᵀ */
  } else {
    /* Structured: A = I + a·e0ᵀ, a = (0,-dy,dx,0…): rows 1,2 += a_i·row0, then cols 1,2 += X[:,0]·a_j */
    const double a1 = -dy, a2 = dx;
    for (int j = 0; j < n; ++j) {
      const double r0 = S[j];
      S[(size_t)1 * n + j] += a1 * r0;
      S[(size_t)2 * n + j] += a2 * r0;
    }
    for (int i = 0; i < n; ++i) {
      const double xi0 = S[(size_t)i * n + 0];
      S[(size_t)i * n + 1] += xi0 * a1;
      S[(size_t)i * n + 2] += xi0 * a2;
    }
  }
  /* + Q̄ = q·I₃ on the pose block (:135-136) */
  for (int i = 0; i < 3; ++i) S[(size_t)i * n + i] += f->q;
}

/* Armadillo's closed-form tiny 2×2 inverse (det = ad − bc; adjugate / det), used by arma::inv on the
 * 2×2 innovation covariance at slam.cpp:252, :395/:401, :476. Returns 0 if singular. */
static int inv2(const double* A, double* out) {
  const double a = A[0], b = A[1], c = A[2], d = A[3];
  const double det = a * d - b * c;
  if (!(fabs(det) > 0.0)) return 0;
  out[0] = d / det;
  out[1] = -b / det;
  out[2] = -c / det;
  out[3] = a / det;
  return 1;
}

/* Range-bearing model for landmark slot k: ẑ (:219-227 / :364-370 / :444-451) and the 9 nonzeros of
 * H (:234-249 / :377-392 / :458-473). hrow0 = {H01,H02,H0j,H0j1}, hrow1 = {H10,H11,H12,H1j,H1j1}. */
static void model(const double* x, int k, double* zhat, double* h0, double* h1) {
  const int j = 3 + 2 * k;
  const double ex = x[j] - x[1], ey = x[j + 1] - x[2];
  zhat[0] = sqrt(pow(ex, 2) + pow(ey, 2));
  zhat[1] = orc_normalize_angle(atan2(ey, ex) - x[0]);
  const double dX = x[j] - x[1], dY = x[j + 1] - x[2];
  const double d = dX * dX + dY * dY;
  h0[0] = -dX / sqrt(d); h0[1] = -dY / sqrt(d); h0[2] = dX / sqrt(d); h0[3] = dY / sqrt(d);
  h1[0] = -1.0; h1[1] = dY / d; h1[2] = -dX / d; h1[3] = -dY / d; h1[4] = dX / d;
}

/* One EKF correction against landmark slot k with measurement (range, bearing):
 * slam.cpp:251-267 (and the identical :475-488). Returns 0, or -4 if S is singular/non-finite. */
static int correct_slot(orc_ekf* f, int k, double zr, double zb) {
  const int n = f->n, j = 3 + 2 * k;
  double zhat[2], h0[4], h1[5];
  model(f->x, k, zhat, h0, h1);
  const int idx[5] = {0, 1, 2, j, j + 1};
  /* H as 2×5 over idx */
  const double H[2][5] = {{0.0, h0[0], h0[1], h0[2], h0[3]}, {h1[0], h1[1], h1[2], h1[3], h1[4]}};
  double* S = f->S;
  double* PHt = f->PHt; /* n×2 : Σ·Hᵀ */
  double* HP = f->HP;   /* 2×n : H·Σ  */
  if (f->literal) {
    double* Hd = f->H;
    memset(Hd, 0, sizeof(double) * 2 * (size_t)n);
    for (int a = 0; a < 5; ++a) { Hd[idx[a]] = H[0][a]; Hd[n + idx[a]] = H[1][a]; }
    for (int i = 0; i < n; ++i) {           /* Σ*Hjᵀ over the full row (zeros included) */
      double s0 = 0.0, s1 = 0.0;
      for (int c = 0; c < n; ++c) { s0 += S[(size_t)i * n + c] * Hd[c]; s1 += S[(size_t)i * n + c] * Hd[n + c]; }
      PHt[2 * i] = s0; PHt[2 * i + 1] = s1;
    }
    for (int c = 0; c < n; ++c) {           /* Hj*Σ */
      double s0 = 0.0, s1 = 0.0;
      for (int a = 0; a < n; ++a) { s0 += Hd[a] * S[(size_t)a * n + c]; s1 += Hd[n + a] * S[(size_t)a * n + c]; }
      HP[c] = s0; HP[n + c] = s1;
    }
  } else {
    for (int i = 0; i < n; ++i) {
      double s0 = 0.0, s1 = 0.0;
      for (int a = 0; a < 5; ++a) { const double v = S[(size_t)i * n + idx[a]]; s0 += v * H[0][a]; s1 += v * H[1][a]; }
      PHt[2 * i] = s0; PHt[2 * i + 1] = s1;
    }
    for (int c = 0; c < n; ++c) {
      double s0 = 0.0, s1 = 0.0;
      for (int a = 0; a < 5; ++a) { const double v = S[(size_t)idx[a] * n + c]; s0 += H[0][a] * v; s1 += H[1][a] * v; }
      HP[c] = s0; HP[n + c] = s1;
    }
  }
  /* Sinn = (Hj*Σ)*Hjᵀ + R (:252; arma evaluates the triple product left to right) */
  double Sm[4] = {0, 0, 0, 0};
  for (int a = 0; a < 5; ++a) {
    Sm[0] += HP[idx[a]] * H[0][a];
    Sm[1] += HP[idx[a]] * H[1][a];
    Sm[2] += HP[n + idx[a]] * H[0][a];
    Sm[3] += HP[n + idx[a]] * H[1][a];
  }
  Sm[0] += f->r; Sm[3] += f->r;
  double Si[4];
  if (!inv2(Sm, Si) || !isfinite(Si[0]) || !isfinite(Si[1]) || !isfinite(Si[2]) || !isfinite(Si[3]))
    return -4;
  /* ν = z − ẑ, bearing normalized (:255-256) */
  const double nu0 = zr - zhat[0];
  const double nu1 = orc_normalize_angle(zb - zhat[1]);
  /* K = (Σ*Hᵀ)*inv(S) (n×2), state += K·ν (:261) */
  if (f->joseph) memcpy(f->PH0, PHt, sizeof(double) * 2 * (size_t)n);
  for (int i = 0; i < n; ++i) {
    const double p0 = PHt[2 * i], p1 = PHt[2 * i + 1];
    const double k0 = p0 * Si[0] + p1 * Si[2];
    const double k1 = p0 * Si[1] + p1 * Si[3];
    PHt[2 * i] = k0; PHt[2 * i + 1] = k1;   /* PHt now holds K */
    f->x[i] = f->x[i] + (k0 * nu0 + k1 * nu1);
  }
  /* Σ = (I − K*Hj)*Σ (:264-265) */
  if (f->joseph && f->literal) {
    /* (I − KH)·Σ·(I − KH)ᵀ + K·R·Kᵀ as dense products */
    double* IKH = f->T1;
    const double* Hd = f->H;
    for (int i = 0; i < n; ++i)
      for (int c = 0; c < n; ++c)
        IKH[(size_t)i * n + c] = (i == c ? 1.0 : 0.0) - (PHt[2 * i] * Hd[c] + PHt[2 * i + 1] * Hd[n + c]);
    gemm_nn(n, IKH, S, f->T2);                       /* T2 = (I − KH)Σ */
    for (int i = 0; i < n; ++i)                      /* T1 ← (I − KH)ᵀ */
      for (int c = i + 1; c < n; ++c) {
        const double t = IKH[(size_t)i * n + c];
        IKH[(size_t)i * n + c] = IKH[(size_t)c * n + i];
        IKH[(size_t)c * n + i] = t;
      }
    gemm_nn(n, f->T2, IKH, S);                       /* Σ = T2 (I − KH)ᵀ */
    for (int i = 0; i < n; ++i)                      /* + K R Kᵀ, R = r·I₂ */
      for (int c = 0; c < n; ++c)
        S[(size_t)i * n + c] += f->r * (PHt[2 * i] * PHt[2 * c] + PHt[2 * i + 1] * PHt[2 * c + 1]);
  } else if (f->joseph) {
    /* Σ − K·(HΣ) − (ΣHᵀ)·Kᵀ + K·S·Kᵀ, S = HΣHᵀ + R (the expansion of the Joseph form) */
    const double* P0 = f->PH0;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
      const double k0 = PHt[2 * i], k1 = PHt[2 * i + 1];
      const double p0 = P0[2 * i], p1 = P0[2 * i + 1];
      double* row = S + (size_t)i * n;
      for (int c = 0; c < n; ++c) {
        const double q0 = PHt[2 * c], q1 = PHt[2 * c + 1];
        const double ks = k0 * (Sm[0] * q0 + Sm[1] * q1) + k1 * (Sm[2] * q0 + Sm[3] * q1);
        row[c] = row[c] - (k0 * HP[c] + k1 * HP[n + c]) - (p0 * q0 + p1 * q1) + ks;
      }
    }
  } else if (f->literal) {
    double* IKH = f->T1;
    const double* Hd = f->H;
    for (int i = 0; i < n; ++i)
      for (int c = 0; c < n; ++c)
        IKH[(size_t)i * n + c] = (i == c ? 1.0 : 0.0) - (PHt[2 * i] * Hd[c] + PHt[2 * i + 1] * Hd[n + c]);
    gemm_nn(n, IKH, S, f->T2);
    memcpy(S, f->T2, sizeof(double) * (size_t)n * n);
  } else {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
      const double k0 = PHt[2 * i], k1 = PHt[2 * i + 1];
      double* row = S + (size_t)i * n;
      for (int c = 0; c < n; ++c) row[c] -= k0 * HP[c] + k1 * HP[n + c];
    }
  }
  f->x[0] = orc_normalize_angle(f->x[0]); /* :267 */
  return 0;
}

/* slam.cpp:208-216 then correct_slot. Returns 0, -2 (id out of range), -4 (numeric). */
int orc_ekf_correct(orc_ekf* f, int id, double rel_x, double rel_y) {
  if (id < 0 || id >= f->N) return -2;
  const double zr = sqrt(pow(rel_x, 2) + pow(rel_y, 2)); /* :208-209 */
  const double zb = atan2(rel_y, rel_x);                   /* :210 */
  const int j = 3 + 2 * id;
  if (f->x[j] == 0.0 && f->x[j + 1] == 0.0) {              /* :213-216 first sighting */
    f->x[j] = f->x[1] + zr * cos(zb + f->x[0]);
    f->x[j + 1] = f->x[2] + zr * sin(zb + f->x[0]);
  }
  return correct_slot(f, id, zr, zb);
}

/* Mahalanobis distance νᵀ ψ⁻¹ ν for landmark slot k (slam.cpp:364-401). */
static double mahalanobis(orc_ekf* f, int k, double zr, double zb) {
  const int n = f->n, j = 3 + 2 * k;
  double zhat[2], h0[4], h1[5];
  model(f->x, k, zhat, h0, h1);
  const int idx[5] = {0, 1, 2, j, j + 1};
  const double H[2][5] = {{0.0, h0[0], h0[1], h0[2], h0[3]}, {h1[0], h1[1], h1[2], h1[3], h1[4]}};
  const double* S = f->S;
  double HP[2][5]; /* (H*Σ) restricted to the columns idx — the only ones Hᵀ picks up */
  if (f->literal) {
    /* dense (Hk*Σ) over the full inner dimension, then *Hkᵀ */
    double* Hd = f->H;
    memset(Hd, 0, sizeof(double) * 2 * (size_t)n);
    for (int a = 0; a < 5; ++a) { Hd[idx[a]] = H[0][a]; Hd[n + idx[a]] = H[1][a]; }
    for (int b = 0; b < 5; ++b) {
      double s0 = 0.0, s1 = 0.0;
      for (int a = 0; a < n; ++a) { s0 += Hd[a] * S[(size_t)a * n + idx[b]]; s1 += Hd[n + a] * S[(size_t)a * n + idx[b]]; }
      HP[0][b] = s0; HP[1][b] = s1;
    }
  } else {
    for (int b = 0; b < 5; ++b) {
      double s0 = 0.0, s1 = 0.0;
      for (int a = 0; a < 5; ++a) { const double v = S[(size_t)idx[a] * n + idx[b]]; s0 += H[0][a] * v; s1 += H[1][a] * v; }
      HP[0][b] = s0; HP[1][b] = s1;
    }
  }
  double psi[4] = {0, 0, 0, 0};
  for (int b = 0; b < 5; ++b) {
    psi[0] += HP[0][b] * H[0][b]; psi[1] += HP[0][b] * H[1][b];
    psi[2] += HP[1][b] * H[0][b]; psi[3] += HP[1][b] * H[1][b];
  }
  psi[0] += f->r; psi[3] += f->r;                       /* :395 */
  const double nu0 = zr - zhat[0];
  const double nu1 = orc_normalize_angle(zb - zhat[1]); /* :398-399 */
  double pi[4];
  if (!inv2(psi, pi)) return NAN;
  const double t0 = nu0 * pi[0] + nu1 * pi[2];          /* (z_diffᵀ * inv(ψ)) * z_diff (:401) */
  const double t1 = nu0 * pi[1] + nu1 * pi[3];
  return t0 * nu0 + t1 * nu1;
}

/* slam.cpp:345-488 for one marker. Returns 0, -2 (capacity: the reference indexes state out of
 * range and throws), -4 (numeric). */
int orc_ekf_associate_correct(orc_ekf* f, double rel_x, double rel_y, int* jout, int* is_new) {
  if (f->counter >= (unsigned)f->N) return -2;
  const double zr = sqrt(pow(rel_x, 2) + pow(rel_y, 2)); /* :345-346 */
  const double zb = atan2(rel_y, rel_x);                   /* :347 */
  const unsigned s = f->counter;
  const int js = 3 + 2 * (int)s;
  f->x[js] = f->x[1] + zr * cos(zb + f->x[0]);             /* :351-354 temporary add */
  f->x[js + 1] = f->x[2] + zr * sin(zb + f->x[0]);
  f->counter++;                                            /* :356 */
  /* :361-416; index_min = first minimum; NaN never wins (strict <) */
  int best = -1;
  double bestd = INFINITY;
  double dnew = f->gate;                                   /* :406-408 */
  double dm = INFINITY; /* the smallest existing d_k (test diagnostics, orc_ekf_last_dmin) */
  for (unsigned k = 0; k < f->counter; ++k) {
    const double d = (k == f->counter - 1) ? dnew : mahalanobis(f, (int)k, zr, zb);
    if (d < bestd) { bestd = d; best = (int)k; }
    if (k + 1 < f->counter && d < dm) dm = d;
  }
  f->last_dmin = dm;
  int jsel = best;
  int nw = 0;
  if (best == (int)f->counter - 1 && bestd >= f->gate) {  /* :421 new landmark */
    nw = 1;
  } else {
    if (best == (int)f->counter - 1 && bestd < f->gate) { /* :423-427 (unreachable: d_new == gate) */
      bestd = INFINITY; best = -1;
      for (unsigned k = 0; k + 1 < f->counter; ++k) {
        const double d = mahalanobis(f, (int)k, zr, zb);
        if (d < bestd) { bestd = d; best = (int)k; }
      }
      if (best < 0) best = 0;
      jsel = best;
    }
    f->counter--;                                          /* :429 / :435 */
    f->x[js] = 0.0;                                        /* :431-432 / :437-438 */
    f->x[js + 1] = 0.0;
  }
  if (jout) *jout = jsel;
  if (is_new) *is_new = nw;
  return correct_slot(f, jsel, zr, zb);                    /* :443-488 */
}

/* slam.cpp:273-277 and :291 */
void orc_ekf_posterior(orc_ekf* f) {
  const double filt[3] = {f->x[0], f->x[1], f->x[2]};
  double inv[3];
  orc_tf_inv(f->todom, inv);
  orc_tf_compose(filt, inv, f->tmo);
  f->prev[0] = filt[0]; f->prev[1] = filt[1]; f->prev[2] = filt[2];
}

/* slam.cpp:180-316 with the ROS publishing left out. Ids are validated before any change (the
 * reference would throw from Armadillo's bounds check part way through the message). */
int orc_ekf_fake_sensor_cb(orc_ekf* f, int m, const int* ids, const int* actions,
                           const double* rel_xy) {
  if (m <= 0) return -3; /* msg.markers.at(0) throws on an empty array (:281) */
  for (int i = 0; i < m; ++i)
    if (actions[i] != ORC_MARKER_DELETE && (ids[i] < 0 || ids[i] >= f->N)) return -2;
  orc_ekf_predict(f);
  int rc = 0;
  for (int i = 0; i < m; ++i) {
    /* only DELETE (= 2) is skipped (:205); ADD, MODIFY and DELETEALL markers are corrections */
    if (actions[i] == ORC_MARKER_DELETE) continue;
    const int e = orc_ekf_correct(f, ids[i], rel_xy[2 * i], rel_xy[2 * i + 1]);
    if (e && !rc) rc = e;
  }
  orc_ekf_posterior(f);
  return rc;
}

/* slam.cpp:318-530 with the ROS publishing left out. */
int orc_ekf_sensor_cb(orc_ekf* f, int m, const double* rel_xy, int* assoc_out, int* new_out) {
  if (m <= 0) return -3; /* :498 */
  orc_ekf_predict(f);
  int rc = 0;
  for (int i = 0; i < m; ++i) {
    int j = -1, nw = 0;
    const int e = orc_ekf_associate_correct(f, rel_xy[2 * i], rel_xy[2 * i + 1], &j, &nw);
    if (assoc_out) assoc_out[i] = j;
    if (new_out) new_out[i] = nw;
    if (e && !rc) rc = e;
  }
  orc_ekf_posterior(f);
  return rc;
}

void orc_ekf_get(const orc_ekf* f, double* state, double* sigma, double* tmo, unsigned* counter) {
  if (state) memcpy(state, f->x, sizeof(double) * f->n);
  if (sigma) memcpy(sigma, f->S, sizeof(double) * (size_t)f->n * f->n);
  if (tmo) memcpy(tmo, f->tmo, sizeof(double) * 3);
  if (counter) *counter = f->counter;
}

void orc_ekf_get_prev(const orc_ekf* f, double* prev) { memcpy(prev, f->prev, sizeof(double) * 3); }

double orc_ekf_last_dmin(const orc_ekf* f) { return f->last_dmin; }

void orc_ekf_set(orc_ekf* f, const double* state, const double* sigma, const double* tmo,
                 const double* prev, unsigned counter) {
  if (state) memcpy(f->x, state, sizeof(double) * f->n);
  if (sigma) memcpy(f->S, sigma, sizeof(double) * (size_t)f->n * f->n);
  if (tmo) memcpy(f->tmo, tmo, sizeof(double) * 3);
  if (prev) memcpy(f->prev, prev, sizeof(double) * 3);
  f->counter = counter;
}
