// fm_dev.hpp -- device-side data structures and small math helpers for the env-step kernel.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace fm {

constexpr int WAVE = 64;
constexpr int MAXCON = 64;    // per-arena contact capacity (64-bit tree masks)
constexpr int CJ = 18;        // Jacobian columns per contact (two trees of <= 9 dofs)
constexpr int MAXSURV = 512;  // broadphase survivors per chunk
constexpr int MAXPC = 8;      // contacts per geom pair (box-box)

// Flat per-arena record layouts (strides in elements)
struct Dims {
  int N, A, K, nq, nv, nu, ngc, nbox, npair, nparam, ntree, obs_dim, act_dim, frame_skip;
  int ncb, ncbp;  // collision bodies, allowed collision-body pairs
  int maxcon, maxrow;
  int phys_stride;  // T:      qpos nq | qvel nv | qpos_s nq | qvel_s nv | qacc_ws nv
  int dbl_stride;   // double: ctrl_target nu | spawn_freq | speed | play_time | last_grip A | last_bucket A | ep_return
  int int_stride;   // int32:  in_scene K | out_scene K | n_in n_out step since fail hidden score0 score1 last0 last1 ep_len
};

// indices into the int block after the two lists
enum { I_NIN = 0, I_NOUT, I_STEP, I_SINCE, I_FAIL, I_HIDDEN, I_S0, I_S1, I_LS0, I_LS1, I_EPLEN, I_NINT };

template <typename T>
struct Model {
  Dims dm;
  // scene scalars
  T dt, grav;
  T belt_mass, belt_kv, belt_damp, belt_invw_t;
  double init_speed, accel, pt_time, force_thr, spawn_freq0, spawn_inc;
  double w_grip, w_bucket, w_action, base_reward;
  double bucket_x0, bucket_x1, bucket_y, bucket_z;
  int env_class, solver_iter;
  double solver_tol;
  // arm template
  const T* arm_base;  // [A][12]  world pos(3), R(9) of the iiwa frame
  const T* body;      // [10][32] local pos(3) local R(9) mass ipos(3) iR(9) I(3) invw_t invw_r pad(2)
  const T* dof;       // [9][4]   range lo, hi, dof_invweight0, pad
  const T* ctrlrange; // [nu][2]
  // geoms (compact, collidable)
  const T* geom;      // [ngc][16]  pos(3) R(9) size(3) rbound
  const int* geom_i;  // [ngc][4]   mjid, type, kbody, box slot
  const uint32_t* pair;  // [npair]  c1 | c2 << 12 | param << 24 (reference list; the kernel uses cb*)
  const int* ginfo;      // [ngc] packed: type code | arm << 2 | pclass << 3 | kbody << 8
  const int* cbi;        // [ncb][4] kbody, flags, first index in cbg, geom count
  const T* cbs;          // [ncb][8] static AABB centre(3), radius, half extents(3), pad
  const uint16_t* cbg;   // geoms grouped by collision body
  const uint32_t* cbp;   // [ncbp] allowed collision-body pairs b1 | b2 << 8
  int ptab[25];          // param index by (pclass g1, pclass g2)
  const T* param;     // [nparam][8] mu, solref(2), solimp(5)
  // per arena
  const T* cube;      // [N][K][4] h, m, I, pad
  const T* meaninertia;  // [N]
  const uint32_t* tri;   // [nv (nv+1) / 2]  column-major lower triangle: i | j << 16
  unsigned long long* prof;  // [16] phase clocks (fm_profile), NULL when profiling is off
};

template <typename T>
struct State {
  T* phys;
  double* dbl;
  int32_t* ints;
  uint64_t* rng;      // [N][4]
  int64_t* counters;  // [N][4]
};

struct StepIO {
  const float* actions;
  float* obs;
  float* reward;
  uint8_t* terminated;
  uint8_t* truncated;
  int32_t* scores;
  int32_t* num_obj;
  double* play_time;
  double* conveyor_speed;
  uint8_t* out_of_reach;
  uint8_t* force_terminate;
  float* terminal_obs;
  double* ep_return;
  int32_t* ep_len;
  int32_t* terminal_scores;
  const uint8_t* reset_mask;
};

// byte offsets of the per-arena LDS workspace (computed on the host, see lds_layout())
struct Lay {
  int q, v, a, as, fs, fc, pb, g, dir, Ma, tmp, fa;
  int ctrl;   // double
  int alen, avel, aforce;
  int bpos, bR, bcom, bIw, bF, bN, dax, danc, site;
  int cR;
  int Marm, Larm, LBarm;
  int gx;     // T [ngc][4]  geom world centre, rbound
  int ginfo, cbi, cbw, cbg;  // LDS copies of the geom / collision-body tables, body bounds T [ncb][8]
  int sp, spoff, gsurv;      // broadphase work lists
  int stage, skey, spw;      // staged contacts T [maxcon][8], keys, pair words
  int cube;                  // T [K][4] this arena's cube h, m, I
  int H;
  int c_i;    // int [maxcon][4]: g1 | g2 << 12, tree1, tree2, flags
  int c_r;    // T [maxcon][CR]
  int r_i;    // int [maxrow][4]
  int r_r;    // T [maxrow][8]
  int tmask;  // uint64 [ntree]
  int misc;   // int [16]
  int sort;   // int [K]
  int uctl;   // double [nu]  clipped control of this env-step
  int scal;   // double [4]   per-step scalars broadcast from lane 0
  int prof;   // uint64 [16]  phase clocks of this arena (profiling only)
  int total;
};

// per-contact real record
enum { CR_DIST = 0, CR_MU, CR_D, CR_KD, CR_BD, CR_POS, CR_FR = CR_POS + 3, CR_J = CR_FR + 9, CR_VEL = CR_J + 3 * CJ,
       CR_JA = CR_VEL + 3, CR_JD = CR_JA + 3, CR_F = CR_JD + 3, CR_N = CR_F + 4 };
// generic row record (equality / joint limit)
enum { RR_C0 = 0, RR_C1, RR_POS, RR_D, RR_AREF, RR_JAR, RR_JD, RR_F, RR_N };
// phase slots of the optional wall-clock profile (fm_profile)
enum { PH_FK = 0, PH_GEOM, PH_COLL, PH_ROWS, PH_SMOOTH, PH_NSETUP, PH_NGRAD, PH_NHESS, PH_NCHOL, PH_NSOLVE, PH_NLS,
       PH_NFINAL, PH_INT, PH_TAIL, PH_NCON, PH_LAST };
enum { MISC_NCON = 0, MISC_NROW, MISC_NSURV, MISC_DROP, MISC_ITER, MISC_MAXIT, MISC_FLAG, MISC_NSTAGE };
// packed geom info
enum { GC_PLANE = 0, GC_SPHERE = 1, GC_BOX = 2, GI_ARM = 2, GI_PC = 3 };

// ------------------------------------------------------------------------------------------------
// math helpers
// ------------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T dsqrt(T x) {
  return sqrt(x);
}

template <typename T>
__device__ __forceinline__ void cross3(const T* a, const T* b, T* r) {
  T t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0;
  r[1] = t1;
  r[2] = t2;
}
template <typename T>
__device__ __forceinline__ T dot3(const T* a, const T* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
template <typename T>
__device__ __forceinline__ void matvec3(const T* R, const T* v, T* r) {
  T t0 = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
  T t1 = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
  T t2 = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
  r[0] = t0;
  r[1] = t1;
  r[2] = t2;
}
template <typename T>
__device__ __forceinline__ void mattvec3(const T* R, const T* v, T* r) {
  T t0 = R[0] * v[0] + R[3] * v[1] + R[6] * v[2];
  T t1 = R[1] * v[0] + R[4] * v[1] + R[7] * v[2];
  T t2 = R[2] * v[0] + R[5] * v[1] + R[8] * v[2];
  r[0] = t0;
  r[1] = t1;
  r[2] = t2;
}
template <typename T>
__device__ __forceinline__ void matmul3(const T* A, const T* B, T* C) {
  T t[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
#pragma unroll
  for (int k = 0; k < 9; k++) C[k] = t[k];
}

template <typename T>
__device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}
template <typename T>
__device__ __forceinline__ T wave_min(T x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T y = __shfl_xor(x, o);
    x = y < x ? y : x;
  }
  return x;
}
template <typename T>
__device__ __forceinline__ T wave_max(T x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T y = __shfl_xor(x, o);
    x = y > x ? y : x;
  }
  return x;
}

}  // namespace fm
