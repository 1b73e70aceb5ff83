// fm_ik.hpp -- the IK base policy of the IK env classes on the GPU (float64, one arena per workgroup).
//
// Reference: IKPolicy (challenge_env/challenge_env/ik_policy.py:28-282) inside
// FactoryManipulationEnv._compose_control (src/environments.py:104-127) and the env classes that use it
// (environments.py:386-459, 498-645).  Per env-step and arena:
//   1. one lane per arm: forward kinematics of the 7-hinge chain + gripper base in float64 from the master
//      state -> the between_gripper_plates site (site_xpos the reference reads);
//   2. lane 0: IKPolicy.act() up to the IK call for every arm IN ARM ORDER (target selection reads the
//      ignore map the previous arms of this compose just wrote), exactly the FSM of ik_policy.py:141-264;
//   3. one lane per arm: qpos_from_site_pose (dm_control, max_steps=10, tol 1e-14, damped least squares with
//      regularisation 3e-2 above error 0.1, minimum-norm step below, progress threshold 20, step cap 2) on a
//      private copy of the arm's hinge angles; the solves of different arms are independent;
//   4. one lane per arm: ctrl = [q*, gripper 0 / 2] on success else last_ctrl, clipped to ctrlrange[1:9].
// Float64 throughout (the IK success test is err < 1e-14): the fp32 physics build runs the same code.
// Parity: the FSM, target choice, grasp orientation and composition follow the oracle (oracle/ik.c), which is
// pinned by golden vectors from the reference's own ik_policy.py; the DLS solve is parity unpinned
// (dm_control absent) and matches the oracle's restatement.
#pragma once

namespace fm {

// the IK env classes (environments.py): which compose the step runs, and whether the reward is the score delta
__host__ __device__ constexpr bool env_toggle(int ec) { return ec == FM_ENV_PAUSE_IK_TOGGLE || ec == FM_ENV_BACKUP_IK_TOGGLE; }
__host__ __device__ constexpr bool env_ik_at_step(int ec) { return ec != FM_ENV_ALLFULLRL_PROGRESS && !env_toggle(ec); }
__host__ __device__ constexpr bool env_score_reward(int ec) { return ec == FM_ENV_FACTORY || env_toggle(ec); }

// scipy Rotation.create_group("O").as_quat(), scalar-last (oracle/ik.c OCT_GROUP)
__device__ __forceinline__ void oct_quat(int k, double q[4]) {
  const double h = 0.5, r = 0.7071067811865476;
  switch (k) {
    case 0: q[0] = 1, q[1] = 0, q[2] = 0, q[3] = 0; break;
    case 1: q[0] = 0, q[1] = 1, q[2] = 0, q[3] = 0; break;
    case 2: q[0] = 0, q[1] = 0, q[2] = 1, q[3] = 0; break;
    case 3: q[0] = 0, q[1] = 0, q[2] = 0, q[3] = 1; break;
    case 4: q[0] = h, q[1] = -h, q[2] = -h, q[3] = h; break;
    case 5: q[0] = h, q[1] = -h, q[2] = h, q[3] = h; break;
    case 6: q[0] = h, q[1] = h, q[2] = -h, q[3] = h; break;
    case 7: q[0] = h, q[1] = h, q[2] = h, q[3] = h; break;
    case 8: q[0] = h, q[1] = -h, q[2] = -h, q[3] = -h; break;
    case 9: q[0] = h, q[1] = -h, q[2] = h, q[3] = -h; break;
    case 10: q[0] = h, q[1] = h, q[2] = -h, q[3] = -h; break;
    case 11: q[0] = h, q[1] = h, q[2] = h, q[3] = -h; break;
    case 12: q[0] = r, q[1] = 0, q[2] = 0, q[3] = r; break;
    case 13: q[0] = 0, q[1] = r, q[2] = 0, q[3] = r; break;
    case 14: q[0] = 0, q[1] = 0, q[2] = r, q[3] = r; break;
    case 15: q[0] = 0, q[1] = 0, q[2] = -r, q[3] = r; break;
    case 16: q[0] = 0, q[1] = -r, q[2] = 0, q[3] = r; break;
    case 17: q[0] = -r, q[1] = 0, q[2] = 0, q[3] = r; break;
    case 18: q[0] = 0, q[1] = r, q[2] = r, q[3] = 0; break;
    case 19: q[0] = 0, q[1] = -r, q[2] = r, q[3] = 0; break;
    case 20: q[0] = r, q[1] = 0, q[2] = r, q[3] = 0; break;
    case 21: q[0] = -r, q[1] = 0, q[2] = r, q[3] = 0; break;
    case 22: q[0] = r, q[1] = r, q[2] = 0, q[3] = 0; break;
    default: q[0] = -r, q[1] = r, q[2] = 0, q[3] = 0; break;
  }
}

// ik_policy.py:53-72
constexpr double IK_DEFAULT_POSE[8] = {-0.5, -0.5, 0.0, 1.0, 0.0, -1.6, 0.0, 0.06};
enum { IK_IDLE = 0, IK_GO_TO_GRASP, IK_GRASP_APPROACH, IK_GRASP_CLOSE, IK_POST_GRASP, IK_GO_TO_RELEASE, IK_RELEASE };

// per-arena IK block in the state arrays (the oracle's export order, oracle/capi.c):
//   double  td + 4 + 2A + 27 i : last_ctrl 8 | move_start 3 | ik_actions 8 | pause_last 8
//   int32   ti + 2K + I_NINT + (3 + A) i : state | counter | target | ignore[A]
struct IkArm {
  double* d;
  int32_t* s;
  __device__ double* last_ctrl() const { return d; }
  __device__ double* move_start() const { return d + 8; }
  __device__ double* ik_actions() const { return d + 11; }
  __device__ double* pause_last() const { return d + 19; }
};
template <typename DD>
__device__ __forceinline__ IkArm ik_arm(const DD& dm, int32_t* ti, double* td, int i) {
  return IkArm{td + 4 + 2 * dm.A + 27 * i, ti + 2 * dm.K + I_NINT + (3 + dm.A) * i};
}

__device__ __forceinline__ double norm3(double a, double b, double c) { return sqrt(a * a + b * b + c * c); }

// scipy _compose_quat (scalar-last) r = p * q, then normalised (Rotation.__mul__)
__device__ __forceinline__ void sp_compose_norm(const double* p, const double* q, double* r) {
  const double c0 = p[1] * q[2] - p[2] * q[1], c1 = p[2] * q[0] - p[0] * q[2], c2 = p[0] * q[1] - p[1] * q[0];
  double t0 = p[3] * q[0] + q[3] * p[0] + c0, t1 = p[3] * q[1] + q[3] * p[1] + c1, t2 = p[3] * q[2] + q[3] * p[2] + c2;
  double t3 = p[3] * q[3] - (p[0] * q[0] + p[1] * q[1] + p[2] * q[2]);
  const double n = sqrt(t0 * t0 + t1 * t1 + t2 * t2 + t3 * t3);
  r[0] = t0 / n;
  r[1] = t1 / n;
  r[2] = t2 / n;
  r[3] = t3 / n;
}

// ik_policy.py:154-162: the cube-symmetric orientation nearest the default gripper orientation (w, x, y, z)
__device__ __forceinline__ void grasp_quat(const double* obj_wxyz, double* out) {
  double qo[4] = {obj_wxyz[1], obj_wxyz[2], obj_wxyz[3], obj_wxyz[0]};
  const double n = sqrt(qo[0] * qo[0] + qo[1] * qo[1] + qo[2] * qo[2] + qo[3] * qo[3]);
  for (int k = 0; k < 4; k++) qo[k] /= n;
  const double def[4] = {0.0, 1.0, 0.0, 0.0};
  double best = 0.0, bq[4] = {0, 0, 0, 1};
  for (int k = 0; k < 24; k++) {
    double g[4], s[4], d[4];
    oct_quat(k, g);
    sp_compose_norm(qo, g, s);
    const double inv[4] = {-s[0], -s[1], -s[2], s[3]};
    sp_compose_norm(def, inv, d);
    const double mag = 2.0 * atan2(norm3(d[0], d[1], d[2]), fabs(d[3]));
    if (k == 0 || mag < best) {
      best = mag;
      for (int c = 0; c < 4; c++) bq[c] = s[c];
    }
  }
  out[0] = bq[3];
  out[1] = bq[0];
  out[2] = bq[1];
  out[3] = bq[2];
}

// forward kinematics of one arm (iiwa14.xml:62-139 links 1..7, gripper.xml gripper base) in float64:
// hinge anchors / world axes and the between_gripper_plates site (pos, frame).  base = world pose of the
// iiwa frame (pos 3, R 9, world frame).
__device__ __forceinline__ void ik_fk(const double* base, const double* q, double* sp, double* sR, double (*anc)[3],
                                      double (*ax)[3]) {
  double P[3] = {base[0], base[1], base[2]}, R[9];
  for (int k = 0; k < 9; k++) R[k] = base[3 + k];
  for (int b = 0; b < 8; b++) {
    const double* bl = ARM_BODY[b];
    double o[3], Rp[9];
    for (int r = 0; r < 3; r++) {
      o[r] = P[r] + R[3 * r] * bl[0] + R[3 * r + 1] * bl[1] + R[3 * r + 2] * bl[2];
      for (int c = 0; c < 3; c++) Rp[3 * r + c] = R[3 * r] * bl[3 + c] + R[3 * r + 1] * bl[6 + c] + R[3 * r + 2] * bl[9 + c];
    }
    if (b < 7) {
      if (anc) {
        for (int k = 0; k < 3; k++) {
          anc[b][k] = o[k];
          ax[b][k] = Rp[3 * k + 2];
        }
      }
      double s, c;
      sincos(q[b], &s, &c);
      for (int r = 0; r < 3; r++) {
        const double x = Rp[3 * r], y = Rp[3 * r + 1];
        Rp[3 * r] = x * c + y * s;
        Rp[3 * r + 1] = -x * s + y * c;
      }
    }
    for (int k = 0; k < 3; k++) P[k] = o[k];
    for (int k = 0; k < 9; k++) R[k] = Rp[k];
  }
  for (int r = 0; r < 3; r++)
    sp[r] = P[r] + R[3 * r] * ARM_GRIP_SITE[0] + R[3 * r + 1] * ARM_GRIP_SITE[1] + R[3 * r + 2] * ARM_GRIP_SITE[2];
  for (int k = 0; k < 9; k++) sR[k] = R[k];
}

// MuJoCo mju_mat2Quat
__device__ __forceinline__ void mat2quat_d(double* q, const double* m) {
  if (m[0] + m[4] + m[8] > 0) {
    q[0] = 0.5 * sqrt(1 + m[0] + m[4] + m[8]);
    q[1] = 0.25 * (m[7] - m[5]) / q[0];
    q[2] = 0.25 * (m[2] - m[6]) / q[0];
    q[3] = 0.25 * (m[3] - m[1]) / q[0];
  } else if (m[0] > m[4] && m[0] > m[8]) {
    q[1] = 0.5 * sqrt(1 + m[0] - m[4] - m[8]);
    q[0] = 0.25 * (m[7] - m[5]) / q[1];
    q[2] = 0.25 * (m[1] + m[3]) / q[1];
    q[3] = 0.25 * (m[2] + m[6]) / q[1];
  } else if (m[4] > m[8]) {
    q[2] = 0.5 * sqrt(1 - m[0] + m[4] - m[8]);
    q[0] = 0.25 * (m[2] - m[6]) / q[2];
    q[1] = 0.25 * (m[1] + m[3]) / q[2];
    q[3] = 0.25 * (m[5] + m[7]) / q[2];
  } else {
    q[3] = 0.5 * sqrt(1 - m[0] - m[4] + m[8]);
    q[0] = 0.25 * (m[3] - m[1]) / q[3];
    q[1] = 0.25 * (m[2] + m[6]) / q[3];
    q[2] = 0.25 * (m[5] + m[7]) / q[3];
  }
  const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < 1e-15) {
    q[0] = 1;
    q[1] = q[2] = q[3] = 0;
  } else if (fabs(n - 1.0) > 1e-15) {
    for (int k = 0; k < 4; k++) q[k] /= n;
  }
}

// in-place Cholesky solve of an n x n SPD matrix (row-major, n <= 7), the oracle's or_cholesky / or_chol_solve
template <int N>
__device__ __forceinline__ void chol_solve_d(double* A, double* x) {
  for (int j = 0; j < N; j++) {
    double s = A[N * j + j];
    for (int k = 0; k < j; k++) s -= A[N * j + k] * A[N * j + k];
    const double d = sqrt(s);
    A[N * j + j] = d;
    for (int i = j + 1; i < N; i++) {
      double t = A[N * i + j];
      for (int k = 0; k < j; k++) t -= A[N * i + k] * A[N * j + k];
      A[N * i + j] = t / d;
    }
  }
  for (int i = 0; i < N; i++) {
    double t = x[i];
    for (int k = 0; k < i; k++) t -= A[N * i + k] * x[k];
    x[i] = t / A[N * i + i];
  }
  for (int i = N - 1; i >= 0; i--) {
    double t = x[i];
    for (int k = i + 1; k < N; k++) t -= A[N * k + i] * x[k];
    x[i] = t / A[N * i + i];
  }
}

// qpos_from_site_pose on the arm's 7 hinges (oracle or_ik_solve); q is updated in place, returns success.
// Not inlined: base is the scene table (constant address space), q / tpos / tquat the compose scratch (address
// space SAS: LDS, or the arena's global block in the spill layouts) -- no generic pointer, no FLAT access
template <int SAS>
__device__ __noinline__ int ik_solve(const double FM_AS(4)* base_, double FM_AS(SAS)* q_, const double FM_AS(SAS)* tpos_,
                                     const double FM_AS(SAS)* tquat_) {
  const double* base = (const double*)base_;
  double* q = (double*)q_;
  const double* tpos = (const double*)tpos_;
  const double* tquat = (const double*)tquat_;
  int success = 0;
  for (int steps = 0; steps < 10; steps++) {
    double sp[3], sR[9], anc[7][3], ax[7][3];
    ik_fk(base, q, sp, sR, anc, ax);
    double err[6];
    for (int k = 0; k < 3; k++) err[k] = tpos[k] - sp[k];
    double en = norm3(err[0], err[1], err[2]);
    {
      double sq[4];
      mat2quat_d(sq, sR);
      const double ng[4] = {sq[0], -sq[1], -sq[2], -sq[3]};
      const double* a = tquat;
      const double e0 = a[0] * ng[0] - a[1] * ng[1] - a[2] * ng[2] - a[3] * ng[3];
      double e1 = a[0] * ng[1] + a[1] * ng[0] + a[2] * ng[3] - a[3] * ng[2];
      double e2 = a[0] * ng[2] - a[1] * ng[3] + a[2] * ng[0] + a[3] * ng[1];
      double e3 = a[0] * ng[3] + a[1] * ng[2] - a[2] * ng[1] + a[3] * ng[0];
      // mju_quat2Vel(dt = 1)
      double s = norm3(e1, e2, e3);
      if (s < 1e-15) {
        e1 = 1;
        e2 = e3 = 0;
      } else {
        e1 /= s;
        e2 /= s;
        e3 /= s;
      }
      double speed = 2.0 * atan2(s, e0);
      if (speed > M_PI) speed -= 2.0 * M_PI;
      err[3] = e1 * speed;
      err[4] = e2 * speed;
      err[5] = e3 * speed;
    }
    en += norm3(err[3], err[4], err[5]);
    if (en < 1e-14) {
      success = 1;
      break;
    }
    double J[6][7];
    for (int j = 0; j < 7; j++) {
      const double r[3] = {sp[0] - anc[j][0], sp[1] - anc[j][1], sp[2] - anc[j][2]};
      J[0][j] = ax[j][1] * r[2] - ax[j][2] * r[1];
      J[1][j] = ax[j][2] * r[0] - ax[j][0] * r[2];
      J[2][j] = ax[j][0] * r[1] - ax[j][1] * r[0];
      J[3][j] = ax[j][0];
      J[4][j] = ax[j][1];
      J[5][j] = ax[j][2];
    }
    double x[7];
    if (en > 0.1) {
      double H[49];
      for (int i = 0; i < 7; i++) {
        double g = 0;
        for (int k = 0; k < 6; k++) g += J[k][i] * err[k];
        x[i] = g;
        for (int j = 0; j < 7; j++) {
          double h = 0;
          for (int k = 0; k < 6; k++) h += J[k][i] * J[k][j];
          H[7 * i + j] = h + (i == j ? 3e-2 : 0.0);
        }
      }
      chol_solve_d<7>(H, x);
    } else {
      double G[36], y[6];
      for (int a = 0; a < 6; a++) {
        y[a] = err[a];
        for (int b = 0; b < 6; b++) {
          double g = 0;
          for (int j = 0; j < 7; j++) g += J[a][j] * J[b][j];
          G[6 * a + b] = g;
        }
      }
      chol_solve_d<6>(G, y);
      for (int j = 0; j < 7; j++) {
        double t = 0;
        for (int a = 0; a < 6; a++) t += J[a][j] * y[a];
        x[j] = t;
      }
    }
    double un = 0;
    for (int j = 0; j < 7; j++) un += x[j] * x[j];
    un = sqrt(un);
    if (en / un > 20.0) break;
    if (un > 2.0)
      for (int j = 0; j < 7; j++) x[j] *= 2.0 / un;
    for (int j = 0; j < 7; j++) q[j] += x[j];
  }
  return success;
}

// IKPolicy.act() up to the IK call (oracle or_ik_plan, ik_policy.py:141-254) for arm i; lane 0.
// Returns 1 when an IK solve for (tp, tq) follows, 0 when act() returned idle_ctrl().
__device__ __forceinline__ int ik_plan(int A, int i, IkArm p, const int32_t* in_scene, int n_in, const double* qd,
                                       const double* vd, int K, const double* grip, const double* base,
                                       const IkTiming& tm, double* tp, double* tq, int* close) {
  int32_t* st = p.s;  // state, counter, target, ignore[A]
  const int qa = 1 + 7 * K + 9 * i;
  // select_target_object (ik_policy.py:92-118): candidates = in-scene cubes not in ignore_objects.values()
  int target = -1;
  {
    const int cur = st[2];
    bool cur_ok = false;
    double best = 0.0;
    int bi = -1;
    for (int c = 0; c < n_in; c++) {
      const int obj = in_scene[c];
      bool ign = false;
      for (int o = 0; o < A; o++) ign |= st[3 + o] == obj;
      if (ign) continue;
      const double* q = qd + 1 + 7 * obj;
      if (obj == cur) cur_ok = norm3(q[0] - base[0], q[1] - base[1], q[2] - base[2]) < 1.0;
      const double dd = norm3(q[0] - base[0], (q[1] - 0.2) - base[1], q[2] - base[2]);
      if (bi < 0 || dd < best) {
        best = dd;
        bi = obj;
      }
    }
    if (cur >= 0 && cur_ok)
      target = cur;
    else if (bi >= 0 && best < 0.8)
      target = bi;
  }
  auto idle = [&]() {  // idle_ctrl(): IDLE, counter 0, target None, last_ctrl = default pose
    st[0] = IK_IDLE;
    st[1] = 0;
    st[2] = -1;
    for (int j = 0; j < 8; j++) p.last_ctrl()[j] = IK_DEFAULT_POSE[j];
  };
  st[2] = target;
  if (target < 0) {
    idle();
    return 0;
  }
  const double* op = qd + 1 + 7 * target;
  const double* ov = vd + 1 + 6 * target;
  double quat[4];
  grasp_quat(op + 3, quat);
  const double pre[3] = {op[0], op[1], op[2] + 0.15};
  const double grasp[3] = {op[0], op[1], op[2] + 0.04};
  const bool near = norm3(grip[0] - op[0], grip[1] - op[1], grip[2] - op[2]) < 0.04;
  const double rel[3] = {(i % 2) == 0 ? 0.9 : -0.9, 0.7 - (A / 2 - 1), 1.3};
  int state = st[0], counter = st[1];
  double* ms = p.move_start();
  auto set_state = [&](int s) {
    counter = 0;
    state = s;
  };
  switch (state) {
    case IK_IDLE: {
      double s = 0.0;
      for (int j = 0; j < 7; j++) {
        const double dj = qd[qa + j] - IK_DEFAULT_POSE[j];
        s += dj * dj;
      }
      if (sqrt(s) < 0.1) set_state(IK_GO_TO_GRASP);
      break;
    }
    case IK_GO_TO_GRASP:
      if (norm3(grip[0] - pre[0], grip[1] - pre[1], grip[2] - pre[2]) < 0.05) set_state(IK_GRASP_APPROACH);
      break;
    case IK_GRASP_APPROACH:
      if (near) set_state(IK_GRASP_CLOSE);
      break;
    case IK_GRASP_CLOSE:
      if (near && counter > tm.grasp_wait) {
        for (int k = 0; k < 3; k++) ms[k] = grip[k];
        set_state(IK_POST_GRASP);
      } else if (!near) {
        set_state(IK_IDLE);
      }
      break;
    case IK_POST_GRASP:
      if (!near) {
        set_state(IK_IDLE);
      } else if (fabs(grip[2] - (ms[2] + 0.18)) < 0.05) {
        for (int k = 0; k < 3; k++) ms[k] = grip[k];
        set_state(IK_GO_TO_RELEASE);
      }
      break;
    case IK_GO_TO_RELEASE:
      if (!near)
        set_state(IK_IDLE);
      else if (norm3(grip[0] - rel[0], grip[1] - rel[1], grip[2] - rel[2]) < 0.1)
        set_state(IK_RELEASE);
      break;
    default:  // RELEASE
      if (counter > tm.release_wait) set_state(IK_IDLE);
      break;
  }
  const double t = (double)counter / tm.move_steps;
  bool comp = false;
  int cl = 0;
  const double defq[4] = {0, 0, 1, 0};
  switch (state) {
    case IK_IDLE:
      idle();
      return 0;
    case IK_GO_TO_GRASP:
      for (int k = 0; k < 3; k++) tp[k] = pre[k];
      comp = true;
      break;
    case IK_GRASP_APPROACH:
      for (int k = 0; k < 3; k++) tp[k] = grasp[k];
      comp = true;
      break;
    case IK_GRASP_CLOSE:
      cl = 1;
      for (int k = 0; k < 3; k++) tp[k] = grasp[k];
      comp = true;
      break;
    case IK_POST_GRASP: {
      cl = 1;
      const double end[3] = {ms[0], ms[1], ms[2] + 0.18};
      for (int k = 0; k < 3; k++) tp[k] = ms[k] + (end[k] - ms[k]) * t;
      for (int k = 0; k < 4; k++) quat[k] = defq[k];
      break;
    }
    case IK_GO_TO_RELEASE:
      cl = 1;
      for (int k = 0; k < 3; k++) tp[k] = ms[k] + (rel[k] - ms[k]) * t;
      for (int k = 0; k < 4; k++) quat[k] = defq[k];
      break;
    default:
      for (int k = 0; k < 3; k++) tp[k] = rel[k];
      for (int k = 0; k < 4; k++) quat[k] = defq[k];
      break;
  }
  counter++;
  if (counter > tm.timeout_steps) {
    idle();
    return 0;
  }
  if (comp) {
    tp[0] += ov[0] * tm.pt_comp;  // env.pt_time * env.dt * 15.0
    tp[1] += ov[1] * tm.pt_comp;
  }
  for (int k = 0; k < 4; k++) tq[k] = quat[k];
  st[0] = state;
  st[1] = counter;
  *close = cl;
  return 1;
}

}  // namespace fm
