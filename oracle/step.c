/* step.c -- one dm_control legacy physics.step() = mj_step2 ; mj_step1 (TEST INFRASTRUCTURE).
 *
 * base_env.py:217-218 calls physics.set_control(ctrl_target) then physics.step().  dm_control's
 * legacy step finishes the step whose position/velocity stage the previous mj_step1 computed
 * (mj_step2: actuation, smooth acceleration, constraint solve, implicitfast integration) and then
 * recomputes the stage at the new state (mj_step1: kinematics, inertia, collision, constraints,
 * passive/bias forces, efc_vel/aref).  Consequence reproduced here: a cube teleported by the
 * TaskManager between two env-steps (task_utils.py:54-60,115-129) is integrated from its new qpos/qvel
 * with the acceleration of the stale stage.
 *
 * implicitfast (MuJoCo mj_implicit): qacc = (M - dt*qDeriv)^-1 (qfrc_smooth + qfrc_constraint) with
 * qDeriv = actuator velocity gains (biasprm[2] * moment^T moment; skipped when the actuator force is
 * clamped by forcerange) - joint damping; qvel += dt*qacc; qpos integrated with the new qvel
 * (free-joint quaternion: normalise, then rotate by dt*omega in the body frame: mju_quatIntegrate).
 */
#include <stdlib.h>

#include "oracle.h"
#include "oracle_internal.h"

void or_reference(const or_model* m, or_data* d);

/* fixed-tendon / joint transmission: actuator length and velocity */
static void transmission(const or_model* m, or_data* d) {
  for (int u = 0; u < m->nu; u++) {
    int d0 = m->act_dof0[u], d1 = m->act_dof1[u];
    int j0 = m->dof_jnt[d0];
    double L = m->act_coef0[u] * d->qpos[m->jnt_qposadr[j0]];
    if (d1 >= 0) L += m->act_coef1[u] * d->qpos[m->jnt_qposadr[m->dof_jnt[d1]]];
    d->act_length[u] = L;
  }
}

void or_velocity_stage(const or_model* m, or_data* d) {
  for (int i = 0; i < m->nv; i++) d->qfrc_passive[i] = -m->dof_damping[i] * d->qvel[i];
  for (int u = 0; u < m->nu; u++) {
    int d0 = m->act_dof0[u], d1 = m->act_dof1[u];
    double v = m->act_coef0[u] * d->qvel[d0];
    if (d1 >= 0) v += m->act_coef1[u] * d->qvel[d1];
    d->act_velocity[u] = v;
  }
  or_reference(m, d);
  or_bias(m, d);
}

/* data-precision probe (tools/fp32_floor.py --probe, not part of the restated algorithm): a relative perturbation
 * amp*U(-1,1) of chosen inputs of the substep's dynamics, modelling one fp32 rounding of each entry -- bit 1 the
 * constraint Jacobian, 2 the mass matrix (symmetric), 4 qacc_smooth, 8 efc_D, 16 efc_aref, 32 qfrc_bias; 64 the
 * arm / gripper geoms' world positions (absolute noise amp metres: float forward kinematics) before the collision,
 * 128 their orientation matrices (absolute noise amp) */
static double g_probe_amp = 0.0;
static int g_probe_mask = 0;
static double noise_u(void);
void or_set_probe(int mask, double amp, uint64_t seed);
static void probe(double* x, int n, int bit) {
  if (!(g_probe_mask & bit)) return;
  for (int i = 0; i < n; i++) x[i] *= 1.0 + g_probe_amp * noise_u();
}
static void probe_sym(double* A, int n, int bit) {
  if (!(g_probe_mask & bit)) return;
  for (int i = 0; i < n; i++)
    for (int j = 0; j <= i; j++) {
      A[i * n + j] *= 1.0 + g_probe_amp * noise_u();
      A[j * n + i] = A[i * n + j];
    }
}

void or_step1(const or_model* m, or_data* d) {
  or_kinematics(m, d);
  or_mass(m, d);
  if (g_probe_mask & (64 | 128))
    for (int a = 0; a < m->A; a++)
      for (int g = m->arm_geom_lo[a]; g < m->arm_geom_hi[a]; g++) {
        if (g_probe_mask & 64)
          for (int k = 0; k < 3; k++) d->geom_xpos[3 * g + k] += g_probe_amp * noise_u();
        if (g_probe_mask & 128)
          for (int k = 0; k < 9; k++) d->geom_xmat[9 * g + k] += g_probe_amp * noise_u();
      }
  or_collision(m, d);
  or_make_constraint(m, d);
  transmission(m, d);
  or_velocity_stage(m, d);
}

void or_fwd_actuation(const or_model* m, or_data* d) {
  memset(d->qfrc_actuator, 0, m->nv * sizeof(double));
  for (int u = 0; u < m->nu; u++) {
    if (d->actuation_disabled) {
      d->act_force[u] = 0;
      continue;
    }
    double c = d->ctrl[u];
    const double* cr = m->act_ctrlrange + 2 * u;
    c = c < cr[0] ? cr[0] : (c > cr[1] ? cr[1] : c);
    const double* bp = m->act_bias + 3 * u;
    double f = m->act_gain[u] * c + bp[0] + bp[1] * d->act_length[u] + bp[2] * d->act_velocity[u];
    if (m->act_forcelimited[u]) {
      const double* fr = m->act_forcerange + 2 * u;
      f = f < fr[0] ? fr[0] : (f > fr[1] ? fr[1] : f);
    }
    d->act_force[u] = f;
    d->qfrc_actuator[m->act_dof0[u]] += m->act_coef0[u] * f;
    if (m->act_dof1[u] >= 0) d->qfrc_actuator[m->act_dof1[u]] += m->act_coef1[u] * f;
  }
}

void or_fwd_acceleration(const or_model* m, or_data* d) {
  int nv = m->nv;
  for (int i = 0; i < nv; i++) d->qfrc_smooth[i] = d->qfrc_passive[i] - d->qfrc_bias[i] + d->qfrc_actuator[i];
  double* L = d->scratch + 4 * nv * nv;
  memcpy(L, d->M, nv * nv * sizeof(double));
  int f[nv];
  or_cholesky_env(L, nv, f);
  memcpy(d->qacc_smooth, d->qfrc_smooth, nv * sizeof(double));
  or_chol_solve_env(L, nv, f, d->qacc_smooth);
}

static void fwd_constraint(const or_model* m, or_data* d) {
  int nv = m->nv;
  probe(d->efc_J, d->nefc * nv, 1);
  probe(d->efc_D, d->nefc, 8);
  probe(d->efc_aref, d->nefc, 16);
  if (d->nefc == 0) {
    memcpy(d->qacc, d->qacc_smooth, nv * sizeof(double));
    memcpy(d->qacc_warmstart, d->qacc_smooth, nv * sizeof(double));
    memset(d->qfrc_constraint, 0, nv * sizeof(double));
    d->solver_niter = 0;
    return;
  }
  or_solve(m, d);
}

static void quat_integrate(double* q, const double* w, double dt) {
  double ax[3] = {w[0], w[1], w[2]};
  double ang = dt * or_normalize3(ax);
  double qr[4];
  or_axis_angle_quat(qr, ax, ang);
  or_quat_normalize(q);
  or_quat_mul(q, q, qr);
}

/* sensitivity probe (tools/fp32_floor.py, not part of the restated algorithm): each substep's acceleration
 * is multiplied by 1 + amp*U(-1,1), amp = 2^-24 modelling a single fp32 rounding per component; 0 = off */
static double g_acc_noise = 0.0;
static uint64_t g_noise_state = 0x9E3779B97F4A7C15ull;
void or_set_accel_noise(double amp, uint64_t seed) {
  g_acc_noise = amp;
  g_noise_state = seed * 0x9E3779B97F4A7C15ull + 1;
}
void or_set_probe(int mask, double amp, uint64_t seed) {
  g_probe_mask = mask;
  g_probe_amp = amp;
  g_noise_state = seed * 0x9E3779B97F4A7C15ull + 1;
}
static double noise_u(void) { /* xorshift64*, uniform in [-1, 1) */
  g_noise_state ^= g_noise_state >> 12;
  g_noise_state ^= g_noise_state << 25;
  g_noise_state ^= g_noise_state >> 27;
  return (double)((g_noise_state * 0x2545F4914F6CDD1Dull) >> 11) * (2.0 / 9007199254740992.0) - 1.0;
}

void or_implicit(const or_model* m, or_data* d) {
  int nv = m->nv;
  double dt = m->timestep;
  double* MhB = d->scratch + 4 * nv * nv;
  memcpy(MhB, d->M, nv * nv * sizeof(double));
  for (int i = 0; i < nv; i++) MhB[i * nv + i] += dt * m->dof_damping[i];
  for (int u = 0; u < m->nu && !d->actuation_disabled; u++) {
    if (m->act_forcelimited[u]) {
      const double* fr = m->act_forcerange + 2 * u;
      if (d->act_force[u] <= fr[0] || d->act_force[u] >= fr[1]) continue;
    }
    double dv = m->act_bias[3 * u + 2];
    int dd[2] = {m->act_dof0[u], m->act_dof1[u]};
    double cc[2] = {m->act_coef0[u], m->act_coef1[u]};
    for (int a = 0; a < 2; a++)
      for (int b = 0; b < 2; b++)
        if (dd[a] >= 0 && dd[b] >= 0) MhB[dd[a] * nv + dd[b]] -= dt * dv * cc[a] * cc[b];
  }
  int f[nv];
  or_cholesky_env(MhB, nv, f);
  double* qa = d->scratch + 5 * nv * nv;
  for (int i = 0; i < nv; i++) qa[i] = d->qfrc_smooth[i] + d->qfrc_constraint[i];
  or_chol_solve_env(MhB, nv, f, qa);
  if (g_acc_noise > 0)
    for (int i = 0; i < nv; i++) qa[i] *= 1.0 + g_acc_noise * noise_u();
  for (int i = 0; i < nv; i++) d->qvel[i] += dt * qa[i];
  for (int j = 0; j < m->njnt; j++) {
    int qa_ = m->jnt_qposadr[j], da = m->jnt_dofadr[j];
    if (m->jnt_type[j] == OR_JNT_FREE) {
      for (int k = 0; k < 3; k++) d->qpos[qa_ + k] += dt * d->qvel[da + k];
      quat_integrate(d->qpos + qa_ + 3, d->qvel + da + 3, dt);
    } else {
      d->qpos[qa_] += dt * d->qvel[da];
    }
  }
}

void or_step2(const or_model* m, or_data* d) {
  or_fwd_actuation(m, d);
  probe(d->qfrc_bias, m->nv, 32);
  probe_sym(d->M, m->nv, 2);
  or_fwd_acceleration(m, d);
  probe(d->qacc_smooth, m->nv, 4);
  fwd_constraint(m, d);
  or_implicit(m, d);
}

/* mj_forward: full forward dynamics at the current state, no integration */
void or_forward(const or_model* m, or_data* d) {
  or_step1(m, d);
  or_fwd_actuation(m, d);
  or_fwd_acceleration(m, d);
  fwd_constraint(m, d);
}
