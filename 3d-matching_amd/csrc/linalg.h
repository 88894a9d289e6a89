// linalg.h — small fp64 linear algebra shared by the device kernels and the host test hooks.
//
//  * svd3_top2 / rotation_from_cov: Kabsch rotation from a 3×3 cross-covariance
//      ransac.py:161-173 (H = pᵀq, svd, R = V Uᵀ, reflection fix) and Eigen::umeyama's
//      S = diag(1,1,±1) (Open3D TransformationEstimationPointToPoint).  For rank ≥ 2 the
//      reflection-fixed rotation is unique:  R = v1 u1ᵀ + v2 u2ᵀ + (v1×v2)(u1×u2)ᵀ,
//      so only the two leading singular pairs are needed; a one-sided (Hestenes) Jacobi SVD
//      gives them to high relative accuracy.  Rank 1 completes both bases with the same
//      deterministic rule (collinear KAT of test_ransac_crash.py:114-139 → I), rank 0 → I
//      (duplicate-points KAT → I, as LAPACK returns).
//  * ldlt6_solve: Eigen::LDLT (diagonal pivoting; zero pivots give zero components) as used by
//      Open3D SolveLinearSystemPSD(JTJ, -JTr); ldlt6_solve_spd: the same system unpivoted,
//      for full-rank JTJ (the device solve's fast path, falling back to ldlt6_solve).
//  * vec6_to_matrix: Open3D TransformVector6dToMatrix4d, R = Rz(x2)·Ry(x1)·Rx(x0).
#pragma once

#include <math.h>

#ifdef __HIPCC__
#define M3D_HD __host__ __device__ inline
#else
#define M3D_HD inline
#endif

namespace m3d {

M3D_HD void cross3(const double a[3], const double b[3], double o[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

M3D_HD double dot3(const double a[3], const double b[3]) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

M3D_HD void normalize3(double a[3]) {
  double n = sqrt(dot3(a, a));
  if (n > 0.0) {
    a[0] /= n;
    a[1] /= n;
    a[2] /= n;
  }
}

// Unit vector orthogonal to unit `a`: normalize(a × e_k), e_k the axis least aligned with a.
M3D_HD void ortho_completion(const double a[3], double o[3]) {
  double ax = fabs(a[0]), ay = fabs(a[1]), az = fabs(a[2]);
  double e[3] = {0.0, 0.0, 0.0};
  if (ax <= ay && ax <= az)
    e[0] = 1.0;
  else if (ay <= az)
    e[1] = 1.0;
  else
    e[2] = 1.0;
  cross3(a, e, o);
  normalize3(o);
}

// Kabsch rotation from the 3×3 cross-covariance H (row-major, H = Σ p qᵀ with p in the
// source frame and q in the target frame).  Writes R (row-major) mapping source → target.
// Returns the numerical rank used (0, 1, 2 or 3 → reported as 2 for ≥2).
M3D_HD int rotation_from_cov(const double Hm[9], double R[9]) {
  // columns of A = H
  double a[3][3], v[3][3];
  for (int c = 0; c < 3; ++c) {
    for (int r = 0; r < 3; ++r) a[c][r] = Hm[r * 3 + c];
    for (int r = 0; r < 3; ++r) v[c][r] = (r == c) ? 1.0 : 0.0;
  }
  for (int sweep = 0; sweep < 16; ++sweep) {
    bool rotated = false;
    for (int pr = 0; pr < 3; ++pr) {
      const int i = (pr == 2) ? 1 : 0;
      const int j = (pr == 0) ? 1 : 2;
      double alpha = dot3(a[i], a[i]);
      double beta = dot3(a[j], a[j]);
      double gamma = dot3(a[i], a[j]);
      if (gamma == 0.0 || fabs(gamma) <= 1e-15 * sqrt(alpha * beta)) continue;
      double zeta = (beta - alpha) / (2.0 * gamma);
      double t;
      if (fabs(zeta) > 1e150)
        t = 0.5 / zeta;
      else
        t = copysign(1.0, zeta) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
      double c = 1.0 / sqrt(1.0 + t * t);
      double s = c * t;
      for (int r = 0; r < 3; ++r) {
        double ai = a[i][r], aj = a[j][r];
        a[i][r] = c * ai - s * aj;
        a[j][r] = s * ai + c * aj;
        double vi = v[i][r], vj = v[j][r];
        v[i][r] = c * vi - s * vj;
        v[j][r] = s * vi + c * vj;
      }
      rotated = true;
    }
    if (!rotated) break;
  }
  double sg[3] = {sqrt(dot3(a[0], a[0])), sqrt(dot3(a[1], a[1])), sqrt(dot3(a[2], a[2]))};
  // order indices by singular value, descending (stable)
  int o0 = 0, o1 = 1, o2 = 2, tmp;
  if (sg[o1] > sg[o0]) { tmp = o0; o0 = o1; o1 = tmp; }
  if (sg[o2] > sg[o1]) { tmp = o1; o1 = o2; o2 = tmp; }
  if (sg[o1] > sg[o0]) { tmp = o0; o0 = o1; o1 = tmp; }
  (void)o2;
  const double s0 = sg[o0], s1 = sg[o1];
  if (!(s0 > 1e-300)) {  // H == 0 (duplicates) or non-finite
    for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0) ? 1.0 : 0.0;
    return (s0 == s0) ? 0 : -1;
  }
  // H V = U Σ: u_k = a_k / σ_k (source frame), v_k (target frame).  The columns o0 / o1 are
  // picked by selects, not by a runtime index: a dynamically indexed a[][] / v[][] lives in
  // scratch memory on the device.
  double u0[3], u1[3], v0[3], v1[3];
  for (int r = 0; r < 3; ++r) {
    u0[r] = (o0 == 0 ? a[0][r] : (o0 == 1 ? a[1][r] : a[2][r])) / s0;
    v0[r] = o0 == 0 ? v[0][r] : (o0 == 1 ? v[1][r] : v[2][r]);
  }
  int rank;
  if (s1 > 1e-14 * s0) {
    for (int r = 0; r < 3; ++r) {
      u1[r] = (o1 == 0 ? a[0][r] : (o1 == 1 ? a[1][r] : a[2][r])) / s1;
      v1[r] = o1 == 0 ? v[0][r] : (o1 == 1 ? v[1][r] : v[2][r]);
    }
    double d = dot3(u0, u1);  // re-orthogonalise (Jacobi leaves it ~eps, harmless)
    for (int r = 0; r < 3; ++r) u1[r] -= d * u0[r];
    normalize3(u1);
    rank = 2;
  } else {
    ortho_completion(u0, u1);
    ortho_completion(v0, v1);
    rank = 1;
  }
  double u2[3], v2[3];
  cross3(u0, u1, u2);
  cross3(v0, v1, v2);
  // R = V Uᵀ restricted to the proper rotation: Σ_k v_k u_kᵀ
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) R[r * 3 + c] = v0[r] * u0[c] + v1[r] * u1[c] + v2[r] * u2[c];
  return rank;
}

// Kabsch on three pairs exactly in the order of ransac.py:153-188: centroids ((a+b)+c)/3,
// H = pᵀq (numpy dot: fma chain), R from the SVD with reflection fix, t = c_t − R c_s.
// Returns 0 ok, 2 non-finite (identity written).
M3D_HD int kabsch3(const double ps[3][3], const double qs[3][3], double T[16]) {
  double cp[3], cq[3], P[3][3], Q[3][3], Hm[9], R[9];
  for (int k = 0; k < 3; ++k) {
    cp[k] = ((ps[0][k] + ps[1][k]) + ps[2][k]) / 3.0;
    cq[k] = ((qs[0][k] + qs[1][k]) + qs[2][k]) / 3.0;
  }
  for (int n = 0; n < 3; ++n)
    for (int k = 0; k < 3; ++k) {
      P[n][k] = ps[n][k] - cp[k];
      Q[n][k] = qs[n][k] - cq[k];
    }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Hm[i * 3 + j] = fma(P[2][i], Q[2][j], fma(P[1][i], Q[1][j], P[0][i] * Q[0][j]));
  rotation_from_cov(Hm, R);
  bool finite = true;
  for (int i = 0; i < 3; ++i) {
    double t = cq[i] - fma(R[i * 3 + 2], cp[2], fma(R[i * 3 + 1], cp[1], R[i * 3 + 0] * cp[0]));
    for (int j = 0; j < 3; ++j) T[i * 4 + j] = R[i * 3 + j];
    T[i * 4 + 3] = t;
  }
  T[12] = T[13] = T[14] = 0.0;
  T[15] = 1.0;
  for (int k = 0; k < 12; ++k) finite = finite && isfinite(T[k]);
  if (!finite) {
    for (int k = 0; k < 16; ++k) T[k] = (k % 5 == 0) ? 1.0 : 0.0;
    return 2;
  }
  return 0;
}

M3D_HD void swapd(double& a, double& b) {
  const double t = a;
  a = b;
  b = t;
}

// Eigen::LDLT-style solve of a symmetric 6×6 system A x = b (A row-major, full).
// Every loop is unrolled and the pivot swap is predicated on compile-time row indices, so on
// the device the factorisation lives in registers (a dynamically indexed pivot row would put
// M, L and the permutation in scratch memory: 720 B and ~10 µs of serial scratch latency).
M3D_HD void ldlt6_solve(const double A_in[36], const double b_in[6], double x[6]) {
  double M[6][6], L[6][6], D[6], y[6];
  int perm[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    perm[i] = i;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      M[i][j] = A_in[i * 6 + j];
      L[i][j] = (i == j) ? 1.0 : 0.0;
    }
  }
  const double tiny = 2.2250738585072014e-308;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    int p = k;
    double best = fabs(M[k][k]);
#pragma unroll
    for (int i = k + 1; i < 6; ++i)
      if (fabs(M[i][i]) > best) {
        best = fabs(M[i][i]);
        p = i;
      }
#pragma unroll
    for (int q = k + 1; q < 6; ++q) {
      if (q == p) {
#pragma unroll
        for (int j = 0; j < 6; ++j) swapd(M[k][j], M[q][j]);
#pragma unroll
        for (int i = 0; i < 6; ++i) swapd(M[i][k], M[i][q]);
#pragma unroll
        for (int j = 0; j < k; ++j) swapd(L[k][j], L[q][j]);
        const int t = perm[k];
        perm[k] = perm[q];
        perm[q] = t;
      }
    }
    D[k] = M[k][k];
    const bool ok = fabs(D[k]) > tiny;
#pragma unroll
    for (int i = k + 1; i < 6; ++i) L[i][k] = ok ? M[i][k] / D[k] : 0.0;
#pragma unroll
    for (int i = k + 1; i < 6; ++i)
#pragma unroll
      for (int j = k + 1; j < 6; ++j) M[i][j] -= L[i][k] * M[k][j];
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) s = (perm[i] == j) ? b_in[j] : s;  // b[perm[i]]
#pragma unroll
    for (int j = 0; j < i; ++j) s -= L[i][j] * y[j];
    y[i] = s;
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) y[i] = (fabs(D[i]) > tiny) ? y[i] / D[i] : 0.0;
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    double s = y[i];
#pragma unroll
    for (int j = i + 1; j < 6; ++j) s -= L[j][i] * y[j];
    y[i] = s;
  }
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j)
      if (perm[i] == j) x[j] = y[i];
}

// The same system without pivoting, for the device solve's common case: JᵀJ is symmetric
// positive semi-definite, so while every pivot stays well away from zero the unpivoted
// factorisation is as stable as the pivoted one and gives the same x up to rounding.  Returns
// false — x untouched — when a pivot falls below 1e-9 of the largest diagonal entry (a rank-
// deficient or near-deficient system): the caller then runs ldlt6_solve, whose pivot order
// decides which components a singular system zeroes, as Eigen's does.
M3D_HD bool ldlt6_solve_spd(const double A[36], const double b[6], double x[6]) {
  double M[6][6], D[6], Di[6], y[6];
  double dmax = 0.0;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    dmax = fmax(dmax, A[i * 6 + i]);
#pragma unroll
    for (int j = 0; j <= i; ++j) M[i][j] = A[i * 6 + j];
  }
  const double lo = 1e-9 * dmax;
  bool ok = dmax > 0.0 && isfinite(dmax);
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    D[k] = M[k][k];
    ok = ok && D[k] > lo;
    Di[k] = 1.0 / D[k];
    // M[i][k] becomes L[i][k]; the trailing lower triangle takes the rank-1 update
#pragma unroll
    for (int i = k + 1; i < 6; ++i) {
      const double c = M[i][k];
      M[i][k] = c * Di[k];
#pragma unroll
      for (int j = k + 1; j <= i; ++j) M[i][j] -= c * M[j][k];  // L[i][k]·D[k]·L[j][k]
    }
  }
  if (!ok) return false;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double s = b[i];
#pragma unroll
    for (int j = 0; j < i; ++j) s -= M[i][j] * y[j];
    y[i] = s;
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {
    double s = y[i] * Di[i];
#pragma unroll
    for (int j = i + 1; j < 6; ++j) s -= M[j][i] * x[j];
    x[i] = s;
  }
  return true;
}

// Open3D TransformVector6dToMatrix4d: R = Rz(x2) Ry(x1) Rx(x0), t = x[3..5].
// (the sines/cosines of x[0..2] given: the device solve computes them in three lanes at once)
M3D_HD void vec6_to_matrix_sc(const double x[6], double ca, double sa, double cb, double sb,
                              double cc, double sc, double T[16]) {
  const double rx[9] = {1, 0, 0, 0, ca, -sa, 0, sa, ca};
  const double ry[9] = {cb, 0, sb, 0, 1, 0, -sb, 0, cb};
  const double rz[9] = {cc, -sc, 0, sc, cc, 0, 0, 0, 1};
  double zy[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      zy[i * 3 + j] = rz[i * 3 + 0] * ry[0 * 3 + j] + rz[i * 3 + 1] * ry[1 * 3 + j] + rz[i * 3 + 2] * ry[2 * 3 + j];
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j)
      T[i * 4 + j] = zy[i * 3 + 0] * rx[0 * 3 + j] + zy[i * 3 + 1] * rx[1 * 3 + j] + zy[i * 3 + 2] * rx[2 * 3 + j];
    T[i * 4 + 3] = x[3 + i];
  }
  T[12] = T[13] = T[14] = 0.0;
  T[15] = 1.0;
}

M3D_HD void vec6_to_matrix(const double x[6], double T[16]) {
  vec6_to_matrix_sc(x, cos(x[0]), sin(x[0]), cos(x[1]), sin(x[1]), cos(x[2]), sin(x[2]), T);
}

// C = A · B for row-major 4×4.
M3D_HD void matmul4(const double A[16], const double B[16], double C[16]) {
  double t[16];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      t[i * 4 + j] = A[i * 4 + 0] * B[0 * 4 + j] + A[i * 4 + 1] * B[1 * 4 + j] +
                     A[i * 4 + 2] * B[2 * 4 + j] + A[i * 4 + 3] * B[3 * 4 + j];
  for (int k = 0; k < 16; ++k) C[k] = t[k];
}

// C = A · B for row-major affine 4×4 (bottom rows 0 0 0 1): matmul4's sums in its order, without
// the terms that multiply by the bottom row's exact 0 / 1 (equal values; the sign of an exact zero
// entry may differ)
M3D_HD void matmul4_affine(const double A[16], const double B[16], double C[16]) {
  double t[12];
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j)
      t[i * 4 + j] = A[i * 4 + 0] * B[0 * 4 + j] + A[i * 4 + 1] * B[1 * 4 + j] + A[i * 4 + 2] * B[2 * 4 + j];
    t[i * 4 + 3] = A[i * 4 + 0] * B[3] + A[i * 4 + 1] * B[7] + A[i * 4 + 2] * B[11] + A[i * 4 + 3];
  }
  for (int k = 0; k < 12; ++k) C[k] = t[k];
  C[12] = C[13] = C[14] = 0.0;
  C[15] = 1.0;
}

}  // namespace m3d
