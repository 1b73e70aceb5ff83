/* ik.c -- IK base policy and the env classes that compose it (TEST INFRASTRUCTURE).
 *
 * Restates, per arm:
 *   IKPolicy.select_target_object / act / idle_ctrl / ignore   challenge_env/challenge_env/ik_policy.py:85-282
 *     (FSM IDLE -> GO_TO_GRASP -> GRASP_APPROACH -> GRASP_CLOSE -> POST_GRASP -> GO_TO_RELEASE -> RELEASE,
 *      constants ik_policy.py:53-72, octahedral grasp orientation ik_policy.py:154-162 with scipy's
 *      Rotation algebra: from_quat normalises, p * q = Hamilton product, magnitude = 2 atan2(|xyz|, |w|))
 *   dm_control qpos_from_site_pose (3rd party, dm_control 1.0.21, not vendored; called at ik_policy.py:257-264
 *     with max_steps=10 and the library defaults tol 1e-14, rot_weight 1, regularization_threshold 0.1,
 *     regularization_strength 3e-2, max_update_norm 2, progress_thresh 20) over this oracle's own
 *     kinematics (mj_fwdPosition) and site Jacobian (mj_jacSite), rotation error by mju_mat2Quat /
 *     mju_negQuat / mju_mulQuat / mju_quat2Vel
 *   FactoryManipulationEnv._compose_control (environments.py:104-127): act() per arm in order, clip to
 *     actuator_ctrlrange[1:9], then every other arm ignores this arm's target
 * The FSM / target selection / symmetry choice / compensation / timeout are pinned by golden vectors from the
 * reference's own ik_policy.py (tests/golden/gen_golden.py, fake IK); the damped-least-squares solve is
 * PARITY UNPINNED (dm_control absent).  One deliberate definition: dm_control's unregularised step solves the
 * rank-6 7x7 normal equations with numpy lstsq(rcond=-1), whose null-space component is set by rounding;
 * this oracle (and the product) take the minimum-norm step J^T (J J^T)^-1 e, the value lstsq converges to
 * when that rounding residue is cut.
 */
#include <stdlib.h>

#include "oracle.h"
#include "oracle_internal.h"

/* scipy.spatial.transform.Rotation.create_group("O").as_quat() (scalar-last), scipy 1.15.3 */
static const double OCT_GROUP[24][4] = {
    {1.0, 0.0, 0.0, 0.0}, {0.0, 1.0, 0.0, 0.0}, {0.0, 0.0, 1.0, 0.0}, {0.0, 0.0, 0.0, 1.0},
    {0.5, -0.5, -0.5, 0.5}, {0.5, -0.5, 0.5, 0.5}, {0.5, 0.5, -0.5, 0.5}, {0.5, 0.5, 0.5, 0.5},
    {0.5, -0.5, -0.5, -0.5}, {0.5, -0.5, 0.5, -0.5}, {0.5, 0.5, -0.5, -0.5}, {0.5, 0.5, 0.5, -0.5},
    {0.7071067811865476, 0.0, 0.0, 0.7071067811865476}, {0.0, 0.7071067811865476, 0.0, 0.7071067811865476},
    {0.0, 0.0, 0.7071067811865476, 0.7071067811865476}, {0.0, 0.0, -0.7071067811865476, 0.7071067811865476},
    {0.0, -0.7071067811865476, 0.0, 0.7071067811865476}, {-0.7071067811865476, 0.0, 0.0, 0.7071067811865476},
    {0.0, 0.7071067811865476, 0.7071067811865476, 0.0}, {0.0, -0.7071067811865476, 0.7071067811865476, 0.0},
    {0.7071067811865476, 0.0, 0.7071067811865476, 0.0}, {-0.7071067811865476, 0.0, 0.7071067811865476, 0.0},
    {0.7071067811865476, 0.7071067811865476, 0.0, 0.0}, {-0.7071067811865476, 0.7071067811865476, 0.0, 0.0},
};

/* ik_policy.py:53-72 (env.dt = 0.1, env.pt_time = 0.2) */
const double OR_IK_DEFAULT_POSE[8] = {-0.5, -0.5, 0.0, 1.0, 0.0, -1.6, 0.0, 0.06};
#define WORKSPACE_RADIUS 1.0
#define GRASP_RADIUS 0.8
#define PRE_GRASP_HEIGHT 0.15
#define POST_GRASP_HEIGHT 0.18
#define TARGET_THRESHOLD 0.05
#define RELEASE_THRESHOLD 0.1
#define GRASP_OFFSET 0.04
/* the step counts and the velocity compensation follow env.dt and env.pt_time (ik_policy.py:56-67); at the
 * defaults (dt = 0.001 * 100 = 0.1, pt_time 0.2): release 5, grasp 10, move 10, timeout 30, 0.30000000000000004 */
#define RELEASE_WAIT ((int)(0.5 / in->dt))
#define GRASP_WAIT ((int)(1.0 / in->dt))
#define MOVE_STEPS ((int)(1.0 / in->dt))
#define TIMEOUT_STEPS ((int)(3.0 / in->dt))
#define PT_COMPENSATION (in->pt_time * in->dt * 15.0) /* env.pt_time * env.dt * 15.0 */

static double norm3d(const double* a) { return sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]); }

/* scipy _compose_quat (scalar-last): r = p * q */
static void sp_compose(const double* p, const double* q, double* r) {
  double c[3] = {p[1] * q[2] - p[2] * q[1], p[2] * q[0] - p[0] * q[2], p[0] * q[1] - p[1] * q[0]};
  double t[4] = {p[3] * q[0] + q[3] * p[0] + c[0], p[3] * q[1] + q[3] * p[1] + c[1], p[3] * q[2] + q[3] * p[2] + c[2],
                 p[3] * q[3] - (p[0] * q[0] + p[1] * q[1] + p[2] * q[2])};
  memcpy(r, t, sizeof t);
}
static void sp_normalize(double* q) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  for (int k = 0; k < 4; k++) q[k] /= n;
}

/* ik_policy.py:154-162: the cube-symmetric orientation closest to the default gripper orientation,
 * returned MuJoCo-ordered (w, x, y, z) */
void or_ik_grasp_quat(const double obj_quat_wxyz[4], double out_wxyz[4]) {
  double qo[4] = {obj_quat_wxyz[1], obj_quat_wxyz[2], obj_quat_wxyz[3], obj_quat_wxyz[0]};
  sp_normalize(qo);
  const double def[4] = {0.0, 1.0, 0.0, 0.0}; /* quat_mujoco2scipy([0, 0, 1, 0]) */
  double best = 0.0, bq[4] = {0, 0, 0, 1};
  for (int k = 0; k < 24; k++) {
    double s[4], inv[4], d[4];
    sp_compose(qo, OCT_GROUP[k], s);
    sp_normalize(s);
    inv[0] = -s[0];
    inv[1] = -s[1];
    inv[2] = -s[2];
    inv[3] = s[3];
    sp_compose(def, inv, d);
    sp_normalize(d);
    double mag = 2.0 * atan2(norm3d(d), fabs(d[3]));
    if (k == 0 || mag < best) {
      best = mag;
      memcpy(bq, s, sizeof bq);
    }
  }
  out_wxyz[0] = bq[3];
  out_wxyz[1] = bq[0];
  out_wxyz[2] = bq[1];
  out_wxyz[3] = bq[2];
}

void or_ik_arm_reset(or_ik_arm* p) { /* IKPolicy.reset -> idle_ctrl (ik_policy.py:120-127) */
  p->state = OR_IK_IDLE;
  p->counter = 0;
  p->target = -1;
  memcpy(p->last_ctrl, OR_IK_DEFAULT_POSE, sizeof p->last_ctrl);
}

void or_ik_arm_init(or_ik_arm* p) {
  memset(p, 0, sizeof *p);
  for (int i = 0; i < OR_IK_MAXA; i++) p->ignore[i] = -1;
  or_ik_arm_reset(p);
}

static void set_state(or_ik_arm* p, int s) {
  p->counter = 0;
  p->state = s;
}

static int ignored(const or_ik_arm* p, int A, int obj) {
  for (int i = 0; i < A; i++)
    if (p->ignore[i] == obj) return 1;
  return 0;
}

/* select_target_object (ik_policy.py:92-118) */
static int select_target(const or_ik_in* in, const or_ik_arm* p) {
  int cand[64], nc = 0;
  for (int c = 0; c < in->n_in; c++)
    if (!ignored(p, in->A, in->in_scene[c])) cand[nc++] = in->in_scene[c];
  if (p->target >= 0) {
    const double* q = in->cube_qpos + 7 * p->target;
    double dv[3] = {q[0] - in->base[0], q[1] - in->base[1], q[2] - in->base[2]};
    int inc = 0;
    for (int c = 0; c < nc; c++) inc |= cand[c] == p->target;
    if (norm3d(dv) < WORKSPACE_RADIUS && inc) return p->target;
  }
  if (nc == 0) return -1;
  double best = 0.0;
  int bi = 0;
  for (int c = 0; c < nc; c++) {
    const double* q = in->cube_qpos + 7 * cand[c];
    double dv[3] = {q[0] - in->base[0], (q[1] - 0.2) - in->base[1], q[2] - in->base[2]};
    double dd = norm3d(dv);
    if (c == 0 || dd < best) {
      best = dd;
      bi = c;
    }
  }
  return best < GRASP_RADIUS ? cand[bi] : -1;
}

/* IKPolicy.act up to the IK call (ik_policy.py:141-254).  Returns 0 when act() returns idle_ctrl()
 * (ctrl = default pose, already written to p->last_ctrl), 1 when an IK solve for (tpos, tquat) follows. */
int or_ik_plan(const or_ik_in* in, or_ik_arm* p, double tpos[3], double tquat[4], int* close_gripper) {
  p->target = select_target(in, p);
  if (p->target < 0) {
    set_state(p, OR_IK_IDLE);
    or_ik_arm_reset(p);
    return 0;
  }
  const double* op = in->cube_qpos + 7 * p->target;
  const double* ov = in->cube_qvel + 6 * p->target;
  double target_quat[4];
  or_ik_grasp_quat(op + 3, target_quat);
  const double* g = in->grip;
  double pre[3] = {op[0], op[1], op[2] + PRE_GRASP_HEIGHT};
  double grasp[3] = {op[0], op[1], op[2] + GRASP_OFFSET};
  double dgo[3] = {g[0] - op[0], g[1] - op[1], g[2] - op[2]};
  int near = norm3d(dgo) < GRASP_OFFSET;
  const double pre_release[3] = {in->bucket[0], in->bucket[1], 1.3};
  switch (p->state) {
    case OR_IK_IDLE: {
      double s = 0.0;
      for (int j = 0; j < 7; j++) {
        double dj = in->arm_q[j] - OR_IK_DEFAULT_POSE[j];
        s += dj * dj;
      }
      if (sqrt(s) < 0.1) set_state(p, OR_IK_GO_TO_GRASP);
      break;
    }
    case OR_IK_GO_TO_GRASP: {
      double d[3] = {g[0] - pre[0], g[1] - pre[1], g[2] - pre[2]};
      if (norm3d(d) < TARGET_THRESHOLD) set_state(p, OR_IK_GRASP_APPROACH);
      break;
    }
    case OR_IK_GRASP_APPROACH:
      if (near) set_state(p, OR_IK_GRASP_CLOSE);
      break;
    case OR_IK_GRASP_CLOSE:
      if (near && p->counter > GRASP_WAIT) {
        memcpy(p->move_start, g, sizeof p->move_start);
        set_state(p, OR_IK_POST_GRASP);
      } else if (!near) {
        set_state(p, OR_IK_IDLE);
      }
      break;
    case OR_IK_POST_GRASP:
      if (!near) {
        set_state(p, OR_IK_IDLE);
      } else if (fabs(g[2] - (p->move_start[2] + POST_GRASP_HEIGHT)) < TARGET_THRESHOLD) {
        memcpy(p->move_start, g, sizeof p->move_start);
        set_state(p, OR_IK_GO_TO_RELEASE);
      }
      break;
    case OR_IK_GO_TO_RELEASE:
      if (!near) {
        set_state(p, OR_IK_IDLE);
      } else {
        double d[3] = {g[0] - pre_release[0], g[1] - pre_release[1], g[2] - pre_release[2]};
        if (norm3d(d) < RELEASE_THRESHOLD) set_state(p, OR_IK_RELEASE);
      }
      break;
    case OR_IK_RELEASE:
      if (p->counter > RELEASE_WAIT) set_state(p, OR_IK_IDLE);
      break;
  }
  int close = 0, comp = 0;
  double tp[3];
  const double def_quat[4] = {0, 0, 1, 0};
  double t = (double)p->counter / MOVE_STEPS; /* lin_interp reads the counter before the increment */
  switch (p->state) {
    case OR_IK_IDLE:
      or_ik_arm_reset(p);
      p->target = -1;
      return 0;
    case OR_IK_GO_TO_GRASP:
      memcpy(tp, pre, sizeof tp);
      comp = 1;
      break;
    case OR_IK_GRASP_APPROACH:
      memcpy(tp, grasp, sizeof tp);
      comp = 1;
      break;
    case OR_IK_GRASP_CLOSE:
      close = 1;
      memcpy(tp, grasp, sizeof tp);
      comp = 1;
      break;
    case OR_IK_POST_GRASP: {
      close = 1;
      double end[3] = {p->move_start[0], p->move_start[1], p->move_start[2] + POST_GRASP_HEIGHT};
      for (int k = 0; k < 3; k++) tp[k] = p->move_start[k] + (end[k] - p->move_start[k]) * t;
      memcpy(target_quat, def_quat, sizeof target_quat);
      break;
    }
    case OR_IK_GO_TO_RELEASE:
      close = 1;
      for (int k = 0; k < 3; k++) tp[k] = p->move_start[k] + (pre_release[k] - p->move_start[k]) * t;
      memcpy(target_quat, def_quat, sizeof target_quat);
      break;
    default: /* RELEASE */
      memcpy(tp, pre_release, sizeof tp);
      memcpy(target_quat, def_quat, sizeof target_quat);
      break;
  }
  p->counter++;
  if (p->counter > TIMEOUT_STEPS) {
    set_state(p, OR_IK_IDLE);
    p->target = -1;
    or_ik_arm_reset(p);
    return 0;
  }
  if (comp) {
    tp[0] += ov[0] * PT_COMPENSATION;
    tp[1] += ov[1] * PT_COMPENSATION;
  }
  memcpy(tpos, tp, sizeof tp);
  memcpy(tquat, target_quat, sizeof target_quat);
  *close_gripper = close;
  return 1;
}

/* ik_policy.py:266-282 */
void or_ik_finish(or_ik_arm* p, int success, const double q7[7], int close_gripper, double ctrl[8]) {
  if (!success) {
    memcpy(ctrl, p->last_ctrl, 8 * sizeof(double));
    return;
  }
  for (int j = 0; j < 7; j++) ctrl[j] = q7[j];
  ctrl[7] = close_gripper ? 0.0 : 2.0;
  memcpy(p->last_ctrl, ctrl, 8 * sizeof(double));
}

/* MuJoCo mju_mat2Quat (engine_util_spatial.c) */
static void mat2quat(double q[4], const double* m) {
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
  or_quat_normalize(q);
}

/* MuJoCo mju_quat2Vel with dt = 1 */
static void quat2vel(double res[3], const double q[4]) {
  double ax[3] = {q[1], q[2], q[3]};
  double s = or_normalize3(ax);
  double speed = 2.0 * atan2(s, q[0]);
  if (speed > M_PI) speed -= 2.0 * M_PI;
  for (int k = 0; k < 3; k++) res[k] = ax[k] * speed;
}

/* symmetric positive definite solve, n <= 7 (Cholesky) */
static void spd_solve(double* A, int n, double* x) {
  or_cholesky(A, n);
  or_chol_solve(A, n, x);
}

/* err / Jacobian of the gripper site of `arm` at the kinematics in d */
static double site_error(const or_model* m, const or_data* d, int arm, const double tpos[3], const double tquat[4],
                         double err[6]) {
  int s = m->grip_site[arm];
  const double* sp = d->site_xpos + 3 * s;
  for (int k = 0; k < 3; k++) err[k] = tpos[k] - sp[k];
  double en = norm3d(err);
  double sq[4], neg[4], eq[4];
  mat2quat(sq, d->site_xmat + 9 * s);
  neg[0] = sq[0];
  neg[1] = -sq[1];
  neg[2] = -sq[2];
  neg[3] = -sq[3];
  or_quat_mul(eq, tquat, neg);
  quat2vel(err + 3, eq);
  return en + norm3d(err + 3);
}

/* qpos_from_site_pose(physics, gripper site, target_pos, target_quat, joint_names=7 arm hinges, max_steps=10)
 * on a copy of the data (inplace=False).  Returns success; q7 = the arm hinges of the result. */
int or_ik_solve(const or_model* m, or_data* scratch, const double* qpos, int arm, const double tpos[3],
                const double tquat[4], double q7[7], int* steps_out) {
  const int nv = m->nv, K = m->K;
  const int qa = 1 + 7 * K + 9 * arm, da = 1 + 6 * K + 9 * arm;
  memcpy(scratch->qpos, qpos, m->nq * sizeof(double));
  or_kinematics(m, scratch); /* mj_fwdPosition: only the kinematics reach the site */
  double* jp = malloc(6 * nv * sizeof(double));
  double* jr = jp + 3 * nv;
  int success = 0, steps = 0;
  for (steps = 0; steps < 10; steps++) {
    double err[6];
    double en = site_error(m, scratch, arm, tpos, tquat, err);
    if (en < 1e-14) {
      success = 1;
      break;
    }
    int s = m->grip_site[arm];
    or_jac_point(m, scratch, m->site_body[s], scratch->site_xpos + 3 * s, jp, jr);
    double J[6][7];
    for (int j = 0; j < 7; j++)
      for (int k = 0; k < 3; k++) {
        J[k][j] = jp[k * nv + da + j];
        J[3 + k][j] = jr[k * nv + da + j];
      }
    double x[7];
    if (en > 0.1) { /* (J^T J + 3e-2 I) x = J^T e */
      double H[49];
      for (int i = 0; i < 7; i++) {
        x[i] = 0;
        for (int k = 0; k < 6; k++) x[i] += J[k][i] * err[k];
        for (int j = 0; j < 7; j++) {
          double h = 0;
          for (int k = 0; k < 6; k++) h += J[k][i] * J[k][j];
          H[7 * i + j] = h + (i == j ? 3e-2 : 0.0);
        }
      }
      spd_solve(H, 7, x);
    } else { /* minimum-norm step x = J^T (J J^T)^-1 e */
      double G[36], y[6];
      for (int a = 0; a < 6; a++) {
        y[a] = err[a];
        for (int b = 0; b < 6; b++) {
          double g = 0;
          for (int j = 0; j < 7; j++) g += J[a][j] * J[b][j];
          G[6 * a + b] = g;
        }
      }
      spd_solve(G, 6, y);
      for (int j = 0; j < 7; j++) {
        x[j] = 0;
        for (int a = 0; a < 6; a++) x[j] += J[a][j] * y[a];
      }
    }
    double un = 0;
    for (int j = 0; j < 7; j++) un += x[j] * x[j];
    un = sqrt(un);
    if (en / un > 20.0) break; /* insufficient progress */
    if (un > 2.0)
      for (int j = 0; j < 7; j++) x[j] *= 2.0 / un;
    for (int j = 0; j < 7; j++) scratch->qpos[qa + j] += x[j]; /* mj_integratePos on hinges */
    or_kinematics(m, scratch);
  }
  free(jp);
  for (int j = 0; j < 7; j++) q7[j] = scratch->qpos[qa + j];
  if (steps_out) *steps_out = steps;
  return success;
}
