// Bundle adjustment on the device, gfx950: the reference's Ceres problem
// (bundle_adjustment/custom_cpp_cost_functions.cpp:56-222, driven by code/utils/ba_functions.py and
// ceres_utils.py) solved by a trust-region Levenberg-Marquardt with the points eliminated (Schur
// complement, as Ceres' DENSE_SCHUR), in fp64.  The host loop is gasfm_amd/ba.py; these kernels
// are its passes over the E observations (edges, camera-major) and the n points (point CSR):
//
//   ba_eval      per edge: residual r, Huber(0.1) corrector w = sqrt(rho'(|r|^2)), corrected and
//                Jacobi-scaled Jacobians Jc [2 x CP] / Jp [2 x 3]; cost 1/2 rho per workgroup
//                (Euclidean CP = 6: angle-axis + t deltas, the rotation differentiated through
//                ceres::AngleAxisRotatePoint with 3-partial dual numbers, like Ceres' autodiff;
//                projective CP = 12: column-major P deltas)
//   ba_cam_normal  one wave per camera: U = Jc^T Jc, gc = Jc^T f over its contiguous edges
//   ba_pt_normal   one thread per point: V = Jp^T Jp, gp = Jp^T f over its CSR slots
//   ba_damp      LM diagonal: U + clamp(diag U, 1e-6, 1e32) / radius, V likewise, V^-1
//   ba_edge_y    Y_e = (Jc^T Jp)_e V^-1_p                                     [E x CP x 3]
//   ba_rhs       one wave per camera: rhs_c = -gc + sum_e Y_e gp
//   ba_pairs     one wave per camera pair block (a <= b) of the reduced camera matrix:
//                S_ab = [a == b] U'_a - sum over shared points of Y_(a,p) W_(b,p)^T, written to
//                the dense [m CP]^2 matrix (and its transpose); the pair lists are sorted once
//                per problem, so every sum runs in a fixed order (no atomics, deterministic)
//   ba_backsub   one thread per point: dp = V'^-1 (-gp - sum_e W_e^T dc_c)
//   ba_model     per edge: model residual Jc dc + Jp dp, -(m . (f + m / 2)) per workgroup
//   ba_sum       fixed-order sum of per-workgroup partials (one workgroup)
//   ba_dlt       one thread per point: the DLT null vector of [P_j | -x_j e_j] (geo_utils.py:611-656)
//                through the secular equation of its normal matrix (4x4 Jacobi eigen-solves
//                inside a safeguarded Newton iteration), X / X[3]
// The dense factorisation of the reduced camera system runs in rocSOLVER (torch.linalg.cholesky_ex).
#include <hip/hip_runtime.h>

#include <cmath>

#include "common.hpp"

namespace gasfm {
namespace {

constexpr double kHuberA = 0.1;  // ceres::HuberLoss(0.1), custom_cpp_cost_functions.cpp:211
constexpr int kT = 256;

struct J3 {  // value + partials w.r.t. the 3 angle-axis components
  double v, d[3];
};
__device__ __forceinline__ J3 jc(double v) { return {v, {0.0, 0.0, 0.0}}; }
__device__ __forceinline__ J3 operator+(J3 a, J3 b) { return {a.v + b.v, {a.d[0] + b.d[0], a.d[1] + b.d[1], a.d[2] + b.d[2]}}; }
__device__ __forceinline__ J3 operator-(J3 a, J3 b) { return {a.v - b.v, {a.d[0] - b.d[0], a.d[1] - b.d[1], a.d[2] - b.d[2]}}; }
__device__ __forceinline__ J3 operator*(J3 a, J3 b) {
  return {a.v * b.v, {a.d[0] * b.v + a.v * b.d[0], a.d[1] * b.v + a.v * b.d[1], a.d[2] * b.v + a.v * b.d[2]}};
}
__device__ __forceinline__ J3 operator*(J3 a, double s) { return {a.v * s, {a.d[0] * s, a.d[1] * s, a.d[2] * s}}; }
__device__ __forceinline__ J3 operator/(J3 a, J3 b) {
  const double q = a.v / b.v, ib = 1.0 / b.v;
  return {q, {(a.d[0] - q * b.d[0]) * ib, (a.d[1] - q * b.d[1]) * ib, (a.d[2] - q * b.d[2]) * ib}};
}
__device__ __forceinline__ J3 jsqrt(J3 a) {
  const double s = sqrt(a.v), h = 0.5 / s;
  return {s, {a.d[0] * h, a.d[1] * h, a.d[2] * h}};
}
__device__ __forceinline__ J3 jsin(J3 a) {
  const double s = sin(a.v), c = cos(a.v);
  return {s, {a.d[0] * c, a.d[1] * c, a.d[2] * c}};
}
__device__ __forceinline__ J3 jcos(J3 a) {
  const double s = sin(a.v), c = cos(a.v);
  return {c, {-a.d[0] * s, -a.d[1] * s, -a.d[2] * s}};
}

// ceres::AngleAxisRotatePoint (rotation.h) with the angle-axis as dual numbers: result[i] and
// d result[i] / d aa; dRdX[i][j] = d result[i] / d pt[j] (the same formula's derivative).
__device__ void aa_rotate(const double aa[3], const double pt[3], J3 out[3], double dRdX[3][3]) {
  J3 w[3] = {{aa[0], {1, 0, 0}}, {aa[1], {0, 1, 0}}, {aa[2], {0, 0, 1}}};
  const J3 t2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  if (t2.v > 2.220446049250313e-16) {
    const J3 th = jsqrt(t2), c = jcos(th), s = jsin(th), ith = jc(1.0) / th;
    J3 u[3] = {w[0] * ith, w[1] * ith, w[2] * ith};
    const J3 uxp[3] = {u[1] * pt[2] - u[2] * pt[1], u[2] * pt[0] - u[0] * pt[2], u[0] * pt[1] - u[1] * pt[0]};
    const J3 omc = jc(1.0) - c;
    const J3 tmp = (u[0] * pt[0] + u[1] * pt[1] + u[2] * pt[2]) * omc;
    for (int i = 0; i < 3; ++i) out[i] = c * pt[i] + uxp[i] * s + u[i] * tmp;
    // d/dpt: c I + s [u]x + (1 - c) u u^T
    const double uv[3] = {u[0].v, u[1].v, u[2].v};
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) dRdX[i][j] = (i == j ? c.v : 0.0) + omc.v * uv[i] * uv[j];
    dRdX[0][1] -= s.v * uv[2];
    dRdX[0][2] += s.v * uv[1];
    dRdX[1][0] += s.v * uv[2];
    dRdX[1][2] -= s.v * uv[0];
    dRdX[2][0] -= s.v * uv[1];
    dRdX[2][1] += s.v * uv[0];
  } else {  // first order: pt + aa x pt
    const J3 axp[3] = {w[1] * pt[2] - w[2] * pt[1], w[2] * pt[0] - w[0] * pt[2], w[0] * pt[1] - w[1] * pt[0]};
    for (int i = 0; i < 3; ++i) out[i] = jc(pt[i]) + axp[i];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) dRdX[i][j] = i == j ? 1.0 : 0.0;
    dRdX[0][1] -= aa[2];
    dRdX[0][2] += aa[1];
    dRdX[1][0] += aa[2];
    dRdX[1][2] -= aa[0];
    dRdX[2][0] -= aa[1];
    dRdX[2][1] += aa[0];
  }
}

// eucReprojectionError (custom_cpp_cost_functions.cpp:105-155): camera = (aa, t) (+ K, fixed)
__device__ void euc_residual(const double* c, const double* K, const double X[3], double ox, double oy, double r[2],
                             double Jc[2][12], double Jp[2][3], bool jac) {
  J3 xr[3];
  double dRdX[3][3];
  aa_rotate(c, X, xr, dRdX);
  const double xc0 = xr[0].v + c[3], xc1 = xr[1].v + c[4], xc2 = xr[2].v + c[5];
  const double iz = 1.0 / xc2;
  const double nu = xc0 * K[0] + xc1 * K[1] + xc2 * K[2];
  const double nv = xc1 * K[3] + xc2 * K[4];
  r[0] = nu * iz - ox;
  r[1] = nv * iz - oy;
  if (!jac) return;
  // d r / d Xc
  const double du[3] = {K[0] * iz, K[1] * iz, K[2] * iz - nu * iz * iz};
  const double dv[3] = {0.0, K[3] * iz, K[4] * iz - nv * iz * iz};
  for (int k = 0; k < 3; ++k) {  // angle-axis
    Jc[0][k] = du[0] * xr[0].d[k] + du[1] * xr[1].d[k] + du[2] * xr[2].d[k];
    Jc[1][k] = dv[0] * xr[0].d[k] + dv[1] * xr[1].d[k] + dv[2] * xr[2].d[k];
  }
  for (int k = 0; k < 3; ++k) {  // translation
    Jc[0][3 + k] = du[k];
    Jc[1][3 + k] = dv[k];
  }
  for (int k = 0; k < 3; ++k) {
    Jp[0][k] = du[0] * dRdX[0][k] + du[1] * dRdX[1][k] + du[2] * dRdX[2][k];
    Jp[1][k] = dv[0] * dRdX[0][k] + dv[1] * dRdX[1][k] + dv[2] * dRdX[2][k];
  }
}

// projReprojectionError (custom_cpp_cost_functions.cpp:56-102): P column-major (P[r + 3 c]), X_w = 1
__device__ void proj_residual(const double* P, const double X[3], double ox, double oy, double r[2], double Jc[2][12],
                              double Jp[2][3], bool jac) {
  const double Xh[4] = {X[0], X[1], X[2], 1.0};
  double q[3];
  for (int i = 0; i < 3; ++i) q[i] = P[i] * Xh[0] + P[3 + i] * Xh[1] + P[6 + i] * Xh[2] + P[9 + i] * Xh[3];
  const double iz = 1.0 / q[2];
  const double u = q[0] * iz, v = q[1] * iz;
  r[0] = u - ox;
  r[1] = v - oy;
  if (!jac) return;
  for (int c = 0; c < 4; ++c) {
    Jc[0][3 * c + 0] = Xh[c] * iz;
    Jc[0][3 * c + 1] = 0.0;
    Jc[0][3 * c + 2] = -u * iz * Xh[c];
    Jc[1][3 * c + 0] = 0.0;
    Jc[1][3 * c + 1] = Xh[c] * iz;
    Jc[1][3 * c + 2] = -v * iz * Xh[c];
  }
  for (int c = 0; c < 3; ++c) {
    Jp[0][c] = (P[3 * c] - u * P[3 * c + 2]) * iz;
    Jp[1][c] = (P[3 * c + 1] - v * P[3 * c + 2]) * iz;
  }
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// fixed-order workgroup sum of one double per thread -> part[blockIdx.x]
__device__ __forceinline__ void block_partial(double v, double* part) {
  __shared__ double red[kT / 64];
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < kT / 64; ++w) s += red[w];
    part[blockIdx.x] = s;
  }
}

template <int CP>
__global__ __launch_bounds__(kT) void ba_eval_kernel(const double* __restrict__ cam0, const double* __restrict__ K,
                                                     const double* __restrict__ X0, const double* __restrict__ dcam,
                                                     const double* __restrict__ dX, const int* __restrict__ cidx,
                                                     const int* __restrict__ pidx, const double* __restrict__ obs,
                                                     int64_t E, const double* __restrict__ sc,
                                                     const double* __restrict__ sp, int jac, double* __restrict__ fres,
                                                     double* __restrict__ Jc, double* __restrict__ Jp,
                                                     double* __restrict__ part) {
  const int64_t e = int64_t(blockIdx.x) * kT + threadIdx.x;
  double half_rho = 0.0;
  if (e < E) {
    const int c = cidx[e], p = pidx[e];
    double cv[CP], X[3];
    for (int k = 0; k < CP; ++k) cv[k] = cam0[int64_t(c) * CP + k] + dcam[int64_t(c) * CP + k];
    for (int k = 0; k < 3; ++k) X[k] = X0[int64_t(p) * 3 + k] + dX[int64_t(p) * 3 + k];
    double r[2], jc_[2][12], jp_[2][3];
    if constexpr (CP == 6)
      euc_residual(cv, K + int64_t(c) * 5, X, obs[2 * e], obs[2 * e + 1], r, jc_, jp_, jac != 0);
    else
      proj_residual(cv, X, obs[2 * e], obs[2 * e + 1], r, jc_, jp_, jac != 0);
    const double s = r[0] * r[0] + r[1] * r[1];
    // ceres::HuberLoss::Evaluate: rho, rho'; the corrector scales residual and Jacobian by sqrt(rho')
    const double b = kHuberA * kHuberA;
    double rho, d1;
    if (s > b) {
      const double rr = sqrt(s);
      rho = 2.0 * kHuberA * rr - b;
      d1 = fmax(2.2250738585072014e-308, kHuberA / rr);
    } else {
      rho = s;
      d1 = 1.0;
    }
    half_rho = 0.5 * rho;
    if (jac) {
      const double w = sqrt(d1);
      fres[2 * e] = w * r[0];
      fres[2 * e + 1] = w * r[1];
      for (int i = 0; i < 2; ++i) {
        for (int k = 0; k < CP; ++k) Jc[(e * 2 + i) * CP + k] = w * jc_[i][k] * (sc ? sc[int64_t(c) * CP + k] : 1.0);
        for (int k = 0; k < 3; ++k) Jp[(e * 2 + i) * 3 + k] = w * jp_[i][k] * (sp ? sp[int64_t(p) * 3 + k] : 1.0);
      }
    }
  }
  block_partial(half_rho, part);
}

// one wave per camera: U (full CP x CP) and gc
template <int CP>
__global__ __launch_bounds__(kT) void ba_cam_normal_kernel(const int* __restrict__ cam_ptr, int m,
                                                           const double* __restrict__ fres,
                                                           const double* __restrict__ Jc, double* __restrict__ U,
                                                           double* __restrict__ gc) {
  constexpr int NU = CP * (CP + 1) / 2;
  const int c = blockIdx.x * (kT / 64) + (threadIdx.x >> 6);
  if (c >= m) return;
  const int lane = threadIdx.x & 63;
  double u[NU], g[CP];
  for (int k = 0; k < NU; ++k) u[k] = 0.0;
  for (int k = 0; k < CP; ++k) g[k] = 0.0;
  for (int e = cam_ptr[c] + lane; e < cam_ptr[c + 1]; e += 64) {
    for (int i = 0; i < 2; ++i) {
      double j[CP];
      for (int k = 0; k < CP; ++k) j[k] = Jc[(int64_t(e) * 2 + i) * CP + k];
      const double f = fres[2 * int64_t(e) + i];
      int q = 0;
      for (int a = 0; a < CP; ++a) {
        g[a] += j[a] * f;
        for (int b2 = a; b2 < CP; ++b2) u[q++] += j[a] * j[b2];
      }
    }
  }
  int q = 0;
  for (int a = 0; a < CP; ++a) {
    const double ga = wave_sum(g[a]);
    if (lane == 0) gc[int64_t(c) * CP + a] = ga;
    for (int b2 = a; b2 < CP; ++b2) {
      const double s = wave_sum(u[q++]);
      if (lane == 0) {
        U[(int64_t(c) * CP + a) * CP + b2] = s;
        U[(int64_t(c) * CP + b2) * CP + a] = s;
      }
    }
  }
}

// one thread per point: V (3 x 3) and gp over its CSR slots
__global__ __launch_bounds__(kT) void ba_pt_normal_kernel(const int* __restrict__ pt_ptr,
                                                          const int* __restrict__ perm, int n,
                                                          const double* __restrict__ fres,
                                                          const double* __restrict__ Jp, double* __restrict__ V,
                                                          double* __restrict__ gp) {
  const int p = blockIdx.x * kT + threadIdx.x;
  if (p >= n) return;
  double v[6] = {0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
  for (int s = pt_ptr[p]; s < pt_ptr[p + 1]; ++s) {
    const int64_t e = perm ? perm[s] : s;
    for (int i = 0; i < 2; ++i) {
      const double j0 = Jp[(e * 2 + i) * 3], j1 = Jp[(e * 2 + i) * 3 + 1], j2 = Jp[(e * 2 + i) * 3 + 2];
      const double f = fres[2 * e + i];
      g[0] += j0 * f;
      g[1] += j1 * f;
      g[2] += j2 * f;
      v[0] += j0 * j0;
      v[1] += j0 * j1;
      v[2] += j0 * j2;
      v[3] += j1 * j1;
      v[4] += j1 * j2;
      v[5] += j2 * j2;
    }
  }
  double* o = V + int64_t(p) * 9;
  o[0] = v[0], o[1] = v[1], o[2] = v[2];
  o[3] = v[1], o[4] = v[3], o[5] = v[4];
  o[6] = v[2], o[7] = v[4], o[8] = v[5];
  gp[3 * int64_t(p)] = g[0], gp[3 * int64_t(p) + 1] = g[1], gp[3 * int64_t(p) + 2] = g[2];
}

__device__ __forceinline__ double lm_diag(double d, double radius) {
  return fmin(fmax(d, 1e-6), 1e32) / radius;  // LevenbergMarquardtStrategy: clamp(diag J^T J) / radius
}

// cameras: Ud = U + D; points: Vinv = (V + D)^-1 (explicit 3 x 3 inverse; singular -> bad[0] = 1)
template <int CP>
__global__ __launch_bounds__(kT) void ba_damp_kernel(const double* __restrict__ U, const double* __restrict__ V, int m,
                                                     int n, double radius, double* __restrict__ Ud,
                                                     double* __restrict__ Vinv, int* __restrict__ bad) {
  const int t = blockIdx.x * kT + threadIdx.x;
  if (t < m) {
    for (int a = 0; a < CP; ++a)
      for (int b = 0; b < CP; ++b) {
        const int64_t o = (int64_t(t) * CP + a) * CP + b;
        Ud[o] = U[o] + (a == b ? lm_diag(U[o], radius) : 0.0);
      }
  } else if (t < m + n) {
    const int64_t p = t - m;
    const double* v = V + p * 9;
    const double a00 = v[0] + lm_diag(v[0], radius), a11 = v[4] + lm_diag(v[4], radius),
                 a22 = v[8] + lm_diag(v[8], radius);
    const double a01 = v[1], a02 = v[2], a12 = v[5];
    const double c00 = a11 * a22 - a12 * a12, c01 = a02 * a12 - a01 * a22, c02 = a01 * a12 - a02 * a11;
    const double det = a00 * c00 + a01 * c01 + a02 * c02;
    double* o = Vinv + p * 9;
    if (!(det > 0.0) || !isfinite(det)) {
      bad[0] = 1;
      for (int i = 0; i < 9; ++i) o[i] = 0.0;
      return;
    }
    const double id = 1.0 / det;
    const double c11 = a00 * a22 - a02 * a02, c12 = a01 * a02 - a00 * a12, c22 = a00 * a11 - a01 * a01;
    o[0] = c00 * id, o[1] = c01 * id, o[2] = c02 * id;
    o[3] = c01 * id, o[4] = c11 * id, o[5] = c12 * id;
    o[6] = c02 * id, o[7] = c12 * id, o[8] = c22 * id;
  }
}

// Y_e = (Jc^T Jp)_e Vinv_p   [E x CP x 3]
template <int CP>
__global__ __launch_bounds__(kT) void ba_edge_y_kernel(const int* __restrict__ pidx, int64_t E,
                                                       const double* __restrict__ Jc, const double* __restrict__ Jp,
                                                       const double* __restrict__ Vinv, double* __restrict__ Y) {
  const int64_t e = int64_t(blockIdx.x) * kT + threadIdx.x;
  if (e >= E) return;
  const double* vi = Vinv + int64_t(pidx[e]) * 9;
  double jp[2][3];
  for (int i = 0; i < 2; ++i)
    for (int k = 0; k < 3; ++k) jp[i][k] = Jp[(e * 2 + i) * 3 + k];
  for (int a = 0; a < CP; ++a) {
    const double c0 = Jc[(e * 2) * CP + a], c1 = Jc[(e * 2 + 1) * CP + a];
    const double w[3] = {c0 * jp[0][0] + c1 * jp[1][0], c0 * jp[0][1] + c1 * jp[1][1], c0 * jp[0][2] + c1 * jp[1][2]};
    for (int k = 0; k < 3; ++k) Y[(e * CP + a) * 3 + k] = w[0] * vi[k] + w[1] * vi[3 + k] + w[2] * vi[6 + k];
  }
}

// one wave per camera: rhs_c = -gc + sum_e Y_e gp
template <int CP>
__global__ __launch_bounds__(kT) void ba_rhs_kernel(const int* __restrict__ cam_ptr, const int* __restrict__ pidx,
                                                    int m, const double* __restrict__ Y,
                                                    const double* __restrict__ gc, const double* __restrict__ gp,
                                                    double* __restrict__ rhs) {
  const int c = blockIdx.x * (kT / 64) + (threadIdx.x >> 6);
  if (c >= m) return;
  const int lane = threadIdx.x & 63;
  double acc[CP];
  for (int a = 0; a < CP; ++a) acc[a] = 0.0;
  for (int e = cam_ptr[c] + lane; e < cam_ptr[c + 1]; e += 64) {
    const double* g = gp + int64_t(pidx[e]) * 3;
    const double g0 = g[0], g1 = g[1], g2 = g[2];
    for (int a = 0; a < CP; ++a) {
      const double* y = Y + (int64_t(e) * CP + a) * 3;
      acc[a] += y[0] * g0 + y[1] * g1 + y[2] * g2;
    }
  }
  for (int a = 0; a < CP; ++a) {
    const double s = wave_sum(acc[a]);
    if (lane == 0) rhs[int64_t(c) * CP + a] = -gc[int64_t(c) * CP + a] + s;
  }
}

// one wave per camera-pair block: lane = entries (i, j) of the CP x CP block, pairs in list order
template <int CP>
__global__ __launch_bounds__(kT) void ba_pairs_kernel(const int* __restrict__ blk_ptr, const int* __restrict__ blk_ab,
                                                      int64_t nblk, int m, const int* __restrict__ pe1,
                                                      const int* __restrict__ pe2, const double* __restrict__ Y,
                                                      const double* __restrict__ Jc, const double* __restrict__ Jp,
                                                      const double* __restrict__ Ud, double* __restrict__ S) {
  constexpr int NE = CP * CP, PER = (NE + 63) / 64;
  const int64_t b = int64_t(blockIdx.x) * (kT / 64) + (threadIdx.x >> 6);
  if (b >= nblk) return;
  const int lane = threadIdx.x & 63;
  const int ca = blk_ab[2 * b], cb = blk_ab[2 * b + 1];
  double acc[PER];
  int ei[PER], ej[PER];
  for (int u = 0; u < PER; ++u) {
    acc[u] = 0.0;
    const int q = lane + 64 * u;
    ei[u] = q < NE ? q / CP : 0;
    ej[u] = q < NE ? q % CP : 0;
  }
  for (int q = blk_ptr[b]; q < blk_ptr[b + 1]; ++q) {
    const int64_t e1 = pe1[q], e2 = pe2[q];
    const double* jp = Jp + e2 * 6;
    for (int u = 0; u < PER; ++u) {
      const double* y = Y + (e1 * CP + ei[u]) * 3;
      const double c0 = Jc[(e2 * 2) * CP + ej[u]], c1 = Jc[(e2 * 2 + 1) * CP + ej[u]];
      acc[u] += y[0] * (c0 * jp[0] + c1 * jp[3]) + y[1] * (c0 * jp[1] + c1 * jp[4]) + y[2] * (c0 * jp[2] + c1 * jp[5]);
    }
  }
  const int64_t ld = int64_t(m) * CP;
  for (int u = 0; u < PER; ++u) {
    if (lane + 64 * u >= NE) break;
    const int i = ei[u], j = ej[u];
    double v = -acc[u];
    if (ca == cb) v += Ud[(int64_t(ca) * CP + i) * CP + j];
    S[(int64_t(ca) * CP + i) * ld + int64_t(cb) * CP + j] = v;
    if (ca != cb) S[(int64_t(cb) * CP + j) * ld + int64_t(ca) * CP + i] = v;
  }
}

// one thread per point: dp = Vinv (-gp - sum_e W_e^T dc)
template <int CP>
__global__ __launch_bounds__(kT) void ba_backsub_kernel(const int* __restrict__ pt_ptr, const int* __restrict__ perm,
                                                        const int* __restrict__ cidx, int n,
                                                        const double* __restrict__ Jc, const double* __restrict__ Jp,
                                                        const double* __restrict__ Vinv,
                                                        const double* __restrict__ gp, const double* __restrict__ dc,
                                                        double* __restrict__ dp) {
  const int p = blockIdx.x * kT + threadIdx.x;
  if (p >= n) return;
  double t[3] = {-gp[3 * int64_t(p)], -gp[3 * int64_t(p) + 1], -gp[3 * int64_t(p) + 2]};
  for (int s = pt_ptr[p]; s < pt_ptr[p + 1]; ++s) {
    const int64_t e = perm ? perm[s] : s;
    const double* d = dc + int64_t(cidx[e]) * CP;
    for (int i = 0; i < 2; ++i) {
      double jd = 0.0;
      for (int k = 0; k < CP; ++k) jd += Jc[(e * 2 + i) * CP + k] * d[k];
      for (int k = 0; k < 3; ++k) t[k] -= Jp[(e * 2 + i) * 3 + k] * jd;
    }
  }
  const double* vi = Vinv + int64_t(p) * 9;
  for (int k = 0; k < 3; ++k) dp[3 * int64_t(p) + k] = vi[3 * k] * t[0] + vi[3 * k + 1] * t[1] + vi[3 * k + 2] * t[2];
}

// per edge: model residual mr = Jc dc + Jp dp; -(mr . (f + mr / 2)) per workgroup
template <int CP>
__global__ __launch_bounds__(kT) void ba_model_kernel(const int* __restrict__ cidx, const int* __restrict__ pidx,
                                                      int64_t E, const double* __restrict__ Jc,
                                                      const double* __restrict__ Jp, const double* __restrict__ fres,
                                                      const double* __restrict__ dc, const double* __restrict__ dp,
                                                      double* __restrict__ part) {
  const int64_t e = int64_t(blockIdx.x) * kT + threadIdx.x;
  double v = 0.0;
  if (e < E) {
    const double* d = dc + int64_t(cidx[e]) * CP;
    const double* q = dp + int64_t(pidx[e]) * 3;
    for (int i = 0; i < 2; ++i) {
      double mr = 0.0;
      for (int k = 0; k < CP; ++k) mr += Jc[(e * 2 + i) * CP + k] * d[k];
      for (int k = 0; k < 3; ++k) mr += Jp[(e * 2 + i) * 3 + k] * q[k];
      v -= mr * (fres[2 * e + i] + 0.5 * mr);
    }
  }
  block_partial(v, part);
}

__global__ __launch_bounds__(kT) void ba_sum_kernel(const double* __restrict__ part, int64_t count,
                                                    double* __restrict__ out) {
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < count; i += kT) s += part[i];
  __shared__ double red[kT];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = kT / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

// ---------------------------------------------------------------- DLT triangulation
// smallest eigenpair of a symmetric 4x4 by cyclic Jacobi
__device__ void eig4_min(double A[4][4], double& lam, double x[4]) {
  double Vm[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) Vm[i][j] = i == j ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 12; ++sweep) {
    double off = 0.0, tot = 0.0;
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) {
        tot += A[i][j] * A[i][j];
        if (i != j) off += A[i][j] * A[i][j];
      }
    if (off <= 1e-32 * tot) break;
    for (int p = 0; p < 3; ++p)
      for (int q = p + 1; q < 4; ++q) {
        if (A[p][q] == 0.0) continue;
        const double th = (A[q][q] - A[p][p]) / (2.0 * A[p][q]);
        const double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 4; ++k) {  // A <- A J
          const double akp = A[k][p], akq = A[k][q];
          A[k][p] = c * akp - s * akq;
          A[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < 4; ++k) {  // A <- J^T A
          const double apk = A[p][k], aqk = A[q][k];
          A[p][k] = c * apk - s * aqk;
          A[q][k] = s * apk + c * aqk;
        }
        for (int k = 0; k < 4; ++k) {
          const double vkp = Vm[k][p], vkq = Vm[k][q];
          Vm[k][p] = c * vkp - s * vkq;
          Vm[k][q] = s * vkp + c * vkq;
        }
      }
  }
  int imin = 0;
  for (int i = 1; i < 4; ++i)
    if (A[i][i] < A[imin][imin]) imin = i;
  lam = A[imin][imin];
  for (int k = 0; k < 4; ++k) x[k] = Vm[k][imin];
}

// one thread per point.  A = [P_j | -x~_j e_j] (x~ = (x, y, 1)); its normal matrix is [[B, C], [C^T, D]]
// with B = sum P_j^T P_j, C_j = -P_j^T x~_j, D = diag |x~_j|^2, so the smallest eigenpair (mu, (X, l))
// satisfies (B - sum_j C_j C_j^T / (d_j - mu)) X = mu X: a safeguarded Newton iteration on mu in
// [0, min d_j) with h(mu) = lambda_min(M(mu)) - mu, h' = -(1 + |l|^2 / |X|^2).
__global__ __launch_bounds__(kT) void ba_dlt_kernel(const int* __restrict__ pt_ptr, const int* __restrict__ perm,
                                                    const int* __restrict__ cidx, int n,
                                                    const double* __restrict__ nP, const double* __restrict__ nx,
                                                    double* __restrict__ X) {
  const int p = blockIdx.x * kT + threadIdx.x;
  if (p >= n) return;
  const int s0 = pt_ptr[p], s1 = pt_ptr[p + 1];
  double* out = X + 4 * int64_t(p);
  if (s1 - s0 < 2) {
    for (int k = 0; k < 4; ++k) out[k] = __builtin_nan("");
    return;
  }
  double B[4][4] = {};
  double dmin = 1e300;
  for (int s = s0; s < s1; ++s) {
    const int64_t e = perm ? perm[s] : s;
    const double* P = nP + int64_t(cidx[e]) * 12;
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) B[i][j] += P[i] * P[j] + P[4 + i] * P[4 + j] + P[8 + i] * P[8 + j];
    const double x0 = nx[2 * e], x1 = nx[2 * e + 1];
    dmin = fmin(dmin, x0 * x0 + x1 * x1 + 1.0);
  }
  double lo = 0.0, hi = dmin, mu = 0.0, lam = 0.0, v[4] = {0, 0, 0, 1};
  for (int it = 0; it < 80; ++it) {
    double M[4][4];
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) M[i][j] = B[i][j];
    for (int s = s0; s < s1; ++s) {
      const int64_t e = perm ? perm[s] : s;
      const double* P = nP + int64_t(cidx[e]) * 12;
      const double x0 = nx[2 * e], x1 = nx[2 * e + 1];
      double Cj[4];
      for (int i = 0; i < 4; ++i) Cj[i] = -(P[i] * x0 + P[4 + i] * x1 + P[8 + i]);
      const double inv = 1.0 / (x0 * x0 + x1 * x1 + 1.0 - mu);
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) M[i][j] -= Cj[i] * Cj[j] * inv;
    }
    eig4_min(M, lam, v);
    const double h = lam - mu;
    if (h >= 0.0) lo = mu; else hi = mu;
    double l2 = 0.0;  // |l|^2 for |X| = 1
    for (int s = s0; s < s1; ++s) {
      const int64_t e = perm ? perm[s] : s;
      const double* P = nP + int64_t(cidx[e]) * 12;
      const double x0 = nx[2 * e], x1 = nx[2 * e + 1];
      double cx = 0.0;
      for (int i = 0; i < 4; ++i) cx -= (P[i] * x0 + P[4 + i] * x1 + P[8 + i]) * v[i];
      const double l = -cx / (x0 * x0 + x1 * x1 + 1.0 - mu);
      l2 += l * l;
    }
    double nmu = mu + h / (1.0 + l2);
    if (!(nmu > lo && nmu < hi)) nmu = 0.5 * (lo + hi);
    if (fabs(nmu - mu) <= 1e-15 * fmax(fabs(mu), 1e-300) || h == 0.0) break;
    mu = nmu;
  }
  for (int k = 0; k < 4; ++k) out[k] = v[k] / v[3];
}

}  // namespace
}  // namespace gasfm

using namespace gasfm;

static unsigned blocks_of(int64_t n) { return unsigned((n + kT - 1) / kT); }

extern "C" int64_t gasfm_ba_partials(int64_t E) { return E <= 0 ? 1 : (E + kT - 1) / kT; }

extern "C" int gasfm_ba_eval(int32_t cp, const double* cam0, const double* K, const double* X0, const double* dcam,
                             const double* dX, const int32_t* cidx, const int32_t* pidx, const double* obs, int64_t E,
                             const double* sc, const double* sp, int32_t jac, double* fres, double* Jc, double* Jp,
                             double* part, void* stream) {
  GASFM_REQUIRE(cp == 6 || cp == 12, "gasfm_ba_eval: camera block size %d (6 or 12)", cp);
  GASFM_REQUIRE(E >= 0 && part, "gasfm_ba_eval: E=%lld", (long long)E);
  GASFM_REQUIRE(E == 0 || (cam0 && X0 && dcam && dX && cidx && pidx && obs && (cp == 12 || K)),
                "gasfm_ba_eval: null pointer");
  GASFM_REQUIRE(!jac || (fres && Jc && Jp), "gasfm_ba_eval: jacobian outputs missing");
  hipStream_t st = (hipStream_t)stream;
  const unsigned g = unsigned(gasfm_ba_partials(E));
  if (cp == 6)
    hipLaunchKernelGGL(ba_eval_kernel<6>, dim3(g), dim3(kT), 0, st, cam0, K, X0, dcam, dX, cidx, pidx, obs, E, sc, sp,
                       jac, fres, Jc, Jp, part);
  else
    hipLaunchKernelGGL(ba_eval_kernel<12>, dim3(g), dim3(kT), 0, st, cam0, K, X0, dcam, dX, cidx, pidx, obs, E, sc, sp,
                       jac, fres, Jc, Jp, part);
  return launch_status("gasfm_ba_eval");
}

extern "C" int gasfm_ba_sum(const double* part, int64_t count, double* out, void* stream) {
  GASFM_REQUIRE(part && out && count >= 0, "gasfm_ba_sum: bad args");
  hipLaunchKernelGGL(ba_sum_kernel, dim3(1), dim3(kT), 0, (hipStream_t)stream, part, count, out);
  return launch_status("gasfm_ba_sum");
}

extern "C" int gasfm_ba_normals(int32_t cp, int32_t m, int32_t n, const int32_t* cam_ptr, const int32_t* pt_ptr,
                                const int32_t* perm, const double* fres, const double* Jc, const double* Jp, double* U,
                                double* gc, double* V, double* gp, void* stream) {
  GASFM_REQUIRE(cp == 6 || cp == 12, "gasfm_ba_normals: camera block size %d", cp);
  GASFM_REQUIRE(m > 0 && n > 0 && cam_ptr && pt_ptr && fres && Jc && Jp && U && gc && V && gp,
                "gasfm_ba_normals: bad args");
  hipStream_t st = (hipStream_t)stream;
  const unsigned gw = unsigned((m + 3) / 4);
  if (cp == 6)
    hipLaunchKernelGGL(ba_cam_normal_kernel<6>, dim3(gw), dim3(kT), 0, st, cam_ptr, m, fres, Jc, U, gc);
  else
    hipLaunchKernelGGL(ba_cam_normal_kernel<12>, dim3(gw), dim3(kT), 0, st, cam_ptr, m, fres, Jc, U, gc);
  hipLaunchKernelGGL(ba_pt_normal_kernel, dim3(blocks_of(n)), dim3(kT), 0, st, pt_ptr, perm, n, fres, Jp, V, gp);
  return launch_status("gasfm_ba_normals");
}

extern "C" int gasfm_ba_damp(int32_t cp, int32_t m, int32_t n, const double* U, const double* V, double radius,
                             double* Ud, double* Vinv, int32_t* bad, void* stream) {
  GASFM_REQUIRE((cp == 6 || cp == 12) && m > 0 && n > 0 && radius > 0, "gasfm_ba_damp: bad args");
  GASFM_REQUIRE(U && V && Ud && Vinv && bad, "gasfm_ba_damp: null pointer");
  hipStream_t st = (hipStream_t)stream;
  if (cp == 6)
    hipLaunchKernelGGL(ba_damp_kernel<6>, dim3(blocks_of(int64_t(m) + n)), dim3(kT), 0, st, U, V, m, n, radius, Ud,
                       Vinv, bad);
  else
    hipLaunchKernelGGL(ba_damp_kernel<12>, dim3(blocks_of(int64_t(m) + n)), dim3(kT), 0, st, U, V, m, n, radius, Ud,
                       Vinv, bad);
  return launch_status("gasfm_ba_damp");
}

extern "C" int gasfm_ba_schur(int32_t cp, int32_t m, const int32_t* cam_ptr, const int32_t* cidx,
                              const int32_t* pidx, int64_t E, const double* Jc, const double* Jp, const double* Vinv,
                              const double* gc, const double* gp, const double* Ud, const int32_t* blk_ptr,
                              const int32_t* blk_ab, int64_t nblk, const int32_t* pe1, const int32_t* pe2, double* Y,
                              double* S, double* rhs, void* stream) {
  GASFM_REQUIRE((cp == 6 || cp == 12) && m > 0 && E > 0 && nblk > 0, "gasfm_ba_schur: bad sizes");
  GASFM_REQUIRE(cam_ptr && cidx && pidx && Jc && Jp && Vinv && gc && gp && Ud && blk_ptr && blk_ab && pe1 && pe2 && Y &&
                    S && rhs,
                "gasfm_ba_schur: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const int64_t ld = int64_t(m) * cp;
  int s = hip_status(hipMemsetAsync(S, 0, sizeof(double) * size_t(ld * ld), st), "gasfm_ba_schur");
  if (s) return s;
  const unsigned gw = unsigned((m + 3) / 4), gb = unsigned((nblk + 3) / 4);
  if (cp == 6) {
    hipLaunchKernelGGL(ba_edge_y_kernel<6>, dim3(blocks_of(E)), dim3(kT), 0, st, pidx, E, Jc, Jp, Vinv, Y);
    hipLaunchKernelGGL(ba_rhs_kernel<6>, dim3(gw), dim3(kT), 0, st, cam_ptr, pidx, m, Y, gc, gp, rhs);
    hipLaunchKernelGGL(ba_pairs_kernel<6>, dim3(gb), dim3(kT), 0, st, blk_ptr, blk_ab, nblk, m, pe1, pe2, Y, Jc, Jp,
                       Ud, S);
  } else {
    hipLaunchKernelGGL(ba_edge_y_kernel<12>, dim3(blocks_of(E)), dim3(kT), 0, st, pidx, E, Jc, Jp, Vinv, Y);
    hipLaunchKernelGGL(ba_rhs_kernel<12>, dim3(gw), dim3(kT), 0, st, cam_ptr, pidx, m, Y, gc, gp, rhs);
    hipLaunchKernelGGL(ba_pairs_kernel<12>, dim3(gb), dim3(kT), 0, st, blk_ptr, blk_ab, nblk, m, pe1, pe2, Y, Jc, Jp,
                       Ud, S);
  }
  return launch_status("gasfm_ba_schur");
}

extern "C" int gasfm_ba_backsub(int32_t cp, int32_t n, const int32_t* pt_ptr, const int32_t* perm,
                                const int32_t* cidx, const double* Jc, const double* Jp, const double* Vinv,
                                const double* gp, const double* dc, double* dp, void* stream) {
  GASFM_REQUIRE((cp == 6 || cp == 12) && n > 0, "gasfm_ba_backsub: bad sizes");
  GASFM_REQUIRE(pt_ptr && cidx && Jc && Jp && Vinv && gp && dc && dp, "gasfm_ba_backsub: null pointer");
  hipStream_t st = (hipStream_t)stream;
  if (cp == 6)
    hipLaunchKernelGGL(ba_backsub_kernel<6>, dim3(blocks_of(n)), dim3(kT), 0, st, pt_ptr, perm, cidx, n, Jc, Jp, Vinv,
                       gp, dc, dp);
  else
    hipLaunchKernelGGL(ba_backsub_kernel<12>, dim3(blocks_of(n)), dim3(kT), 0, st, pt_ptr, perm, cidx, n, Jc, Jp,
                       Vinv, gp, dc, dp);
  return launch_status("gasfm_ba_backsub");
}

extern "C" int gasfm_ba_model(int32_t cp, const int32_t* cidx, const int32_t* pidx, int64_t E, const double* Jc,
                              const double* Jp, const double* fres, const double* dc, const double* dp, double* part,
                              void* stream) {
  GASFM_REQUIRE((cp == 6 || cp == 12) && E >= 0 && part, "gasfm_ba_model: bad args");
  GASFM_REQUIRE(E == 0 || (cidx && pidx && Jc && Jp && fres && dc && dp), "gasfm_ba_model: null pointer");
  hipStream_t st = (hipStream_t)stream;
  const unsigned g = unsigned(gasfm_ba_partials(E));
  if (cp == 6)
    hipLaunchKernelGGL(ba_model_kernel<6>, dim3(g), dim3(kT), 0, st, cidx, pidx, E, Jc, Jp, fres, dc, dp, part);
  else
    hipLaunchKernelGGL(ba_model_kernel<12>, dim3(g), dim3(kT), 0, st, cidx, pidx, E, Jc, Jp, fres, dc, dp, part);
  return launch_status("gasfm_ba_model");
}

extern "C" int gasfm_ba_dlt(int32_t n, const int32_t* pt_ptr, const int32_t* perm, const int32_t* cidx,
                            const double* nP, const double* nx, double* X, void* stream) {
  GASFM_REQUIRE(n > 0 && pt_ptr && cidx && nP && nx && X, "gasfm_ba_dlt: bad args");
  hipLaunchKernelGGL(ba_dlt_kernel, dim3(blocks_of(n)), dim3(kT), 0, (hipStream_t)stream, pt_ptr, perm, cidx, n, nP,
                     nx, X);
  return launch_status("gasfm_ba_dlt");
}
