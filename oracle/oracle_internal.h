/* oracle_internal.h -- small vector/quaternion helpers shared by the oracle sources (TEST INFRA). */
#ifndef FM_ORACLE_INTERNAL_H
#define FM_ORACLE_INTERNAL_H
#include <math.h>
#include <string.h>

#define OR_MINVAL 1e-15
#define OR_MINIMP 0.0001
#define OR_MAXIMP 0.9999

static inline double or_dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline void or_cross(double* r, const double* a, const double* b) {
  double t[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  r[0] = t[0];
  r[1] = t[1];
  r[2] = t[2];
}
static inline double or_norm3(const double* a) { return sqrt(or_dot3(a, a)); }

/* mju_normalize4: unit quaternion, (1,0,0,0) if degenerate, untouched if already unit */
static inline double or_quat_normalize(double* q) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < OR_MINVAL) {
    q[0] = 1;
    q[1] = q[2] = q[3] = 0;
  } else if (fabs(n - 1.0) > OR_MINVAL) {
    q[0] /= n;
    q[1] /= n;
    q[2] /= n;
    q[3] /= n;
  }
  return n;
}
/* mju_normalize3 */
static inline double or_normalize3(double* v) {
  double n = or_norm3(v);
  if (n < OR_MINVAL) {
    v[0] = 1;
    v[1] = v[2] = 0;
  } else {
    v[0] /= n;
    v[1] /= n;
    v[2] /= n;
  }
  return n;
}
/* Hamilton product r = a*b, (w,x,y,z) */
static inline void or_quat_mul(double* r, const double* a, const double* b) {
  double t[4] = {a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                 a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                 a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
                 a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]};
  memcpy(r, t, sizeof t);
}
static inline void or_quat2mat(double* R, const double* q) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = w * w + x * x - y * y - z * z;
  R[1] = 2 * (x * y - w * z);
  R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z);
  R[4] = w * w - x * x + y * y - z * z;
  R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y);
  R[7] = 2 * (y * z + w * x);
  R[8] = w * w - x * x - y * y + z * z;
}
static inline void or_axis_angle_quat(double* q, const double* axis, double angle) {
  if (angle == 0.0) {
    q[0] = 1;
    q[1] = q[2] = q[3] = 0;
    return;
  }
  double s = sin(angle * 0.5);
  q[0] = cos(angle * 0.5);
  q[1] = axis[0] * s;
  q[2] = axis[1] * s;
  q[3] = axis[2] * s;
}
/* r = R * v  (R row-major 3x3) */
static inline void or_mulmv3(double* r, const double* R, const double* v) {
  double t[3] = {R[0] * v[0] + R[1] * v[1] + R[2] * v[2], R[3] * v[0] + R[4] * v[1] + R[5] * v[2],
                 R[6] * v[0] + R[7] * v[1] + R[8] * v[2]};
  r[0] = t[0];
  r[1] = t[1];
  r[2] = t[2];
}
/* r = R^T * v */
static inline void or_mulmtv3(double* r, const double* R, const double* v) {
  double t[3] = {R[0] * v[0] + R[3] * v[1] + R[6] * v[2], R[1] * v[0] + R[4] * v[1] + R[7] * v[2],
                 R[2] * v[0] + R[5] * v[1] + R[8] * v[2]};
  r[0] = t[0];
  r[1] = t[1];
  r[2] = t[2];
}
static inline void or_mulmm3(double* C, const double* A, const double* B) {
  double t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
  memcpy(C, t, sizeof t);
}

/* internal entry points */
void or_model_setconst(or_model* m);
void or_cholesky(double* A, int n);                         /* in-place lower Cholesky, row-major n x n */
void or_chol_solve(const double* L, int n, double* x);      /* solve L L^T x = b in place */
void or_cholesky_env(double* A, int n, int* f);               /* the same factor, envelope f[] skipped (kin.c) */
void or_chol_solve_env(const double* L, int n, const int* f, double* x);
void or_body_jac(const or_model* m, const or_data* d, int body, const double p[3], double* jacp, double* jacr);
void or_solve(const or_model* m, or_data* d);               /* Newton constraint solver (solver.c) */
void or_fwd_actuation(const or_model* m, or_data* d);
void or_fwd_acceleration(const or_model* m, or_data* d);
void or_velocity_stage(const or_model* m, or_data* d);
void or_implicit(const or_model* m, or_data* d);

#endif
