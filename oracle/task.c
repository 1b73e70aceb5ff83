/* task.c -- BaseEnv / TaskManager / environment wrappers restated (TEST INFRASTRUCTURE; see oracle.h).
 *
 *   or_task_reset          TaskManager.reset (task_utils.py:146-156) + BaseEnv.reset_sim (base_env.py:177-198)
 *   or_task_process_action FactoryManipulationEnv._process_action (environments.py:84-102), float32 tanh
 *   or_task_clip_ctrl      BaseEnv.step_sim ctrl = clip([speed, arm actions]) (base_env.py:240-262)
 *   or_task_lowpass        _step_sim_unscaled low-pass + conveyor override (base_env.py:207-215)
 *   or_task_force_check    contact-force termination (base_env.py:225-236)
 *   or_task_step           TaskManager.step: spawn schedule, _spawn_object, _check_states (incl. the
 *                          reference's bucket-loop index reuse, task_utils.py:103-113), _hide_object
 *   or_task_after_step     play_time / conveyor speed / spawn_freq updates (base_env.py:266-272)
 *   or_task_obs            _get_state + get_valid_object_vectors + _process_observation
 *                          (base_env.py:149-175, task_utils.py:62-77, environments.py:55-82)
 *   or_task_reward         FactoryManipulationEnv._get_reward / ProgressRewardEnv._get_reward
 *                          (environments.py:129-149, 284-383)
 * Python float64 semantics are reproduced with IEEE double in the same operation order
 * (e.g. int(1.0 / (0.1 * spawn_freq)), spawn_freq *= 1.001, 0.2 * counter).
 */
#include <stdlib.h>

#include "oracle.h"
#include "oracle_internal.h"

#define BX 0.6

void or_task_init(or_task* t, int A, int K, uint64_t seed) {
  memset(t, 0, sizeof *t);
  t->A = A;
  t->K = K;
  t->initial_conveyor_speed = 0.1;
  t->conveyor_acceleration = 0.001;
  t->pt_time = 0.2;
  t->force_contact_threshold = 200.0;
  t->spawn_freq_increase = 1.001;
  t->init_spawn_freq = (1.0 / 10) * A;
  t->spawn_freq = t->init_spawn_freq;
  t->frame_skip = (int)((1.0 / 10.0) / 0.001);
  or_pcg64_seed(&t->rng, seed);
  t->conveyor_speed = t->initial_conveyor_speed;
  for (int i = 0; i < 16; i++)
    for (int j = 0; j < 16; j++) t->ik_ignore[i][j] = -1;
  t->act_dim = 8 * A;
}

static int cube_qadr(const or_model* m, int k) { return m->jnt_qposadr[m->body_jntadr[m->cube_body0 + k]]; }
static int cube_dadr(const or_model* m, int k) { return m->jnt_dofadr[m->body_jntadr[m->cube_body0 + k]]; }

void or_task_reset(or_task* t, const or_model* m, double* qpos, double* qvel) {
  for (int k = 0; k < t->K; k++) {
    double* q = qpos + cube_qadr(m, k);
    q[0] = 4.0;
    q[1] = 0.0 + k * 0.2;
    q[2] = 1.0;
    q[3] = 1.0;
    q[4] = q[5] = q[6] = 0.0;
    double* v = qvel + cube_dadr(m, k);
    for (int i = 0; i < 6; i++) v[i] = 0.0;
    t->out_scene[k] = k;
  }
  t->n_out = t->K;
  t->n_in = 0;
  t->step_counter = t->steps_since_spawn = t->failure_counter = t->hidden_counter = 0;
  t->scores[0] = t->scores[1] = 0;
  t->conveyor_speed = t->initial_conveyor_speed;
  t->spawn_freq = t->init_spawn_freq;
  memset(t->ctrl_target, 0, sizeof t->ctrl_target);
  t->play_time = 0.0;
  t->last_score[0] = t->last_score[1] = 0;
  t->force_terminate = t->out_of_reach = 0;
}

void or_task_process_action(const or_model* m, const float* action, double* arm_ctrl) {
  for (int i = 0; i < m->A; i++)
    for (int j = 0; j < 8; j++) {
      float a = (float)tanh((double)action[8 * i + j]); /* correctly rounded float32 tanh */
      float s = (a + 1.0f) * 0.5f;
      double lo = m->act_ctrlrange[2 * (1 + j)], hi = m->act_ctrlrange[2 * (1 + j) + 1];
      arm_ctrl[8 * i + j] = lo + (double)s * (hi - lo);
    }
}

void or_task_clip_ctrl(const or_task* t, const or_model* m, const double* arm_ctrl, double* ctrl) {
  ctrl[0] = t->conveyor_speed;
  for (int i = 0; i < 8 * m->A; i++) ctrl[1 + i] = arm_ctrl[i];
  for (int u = 0; u < m->nu; u++) {
    double lo = m->act_ctrlrange[2 * u], hi = m->act_ctrlrange[2 * u + 1];
    ctrl[u] = ctrl[u] < lo ? lo : (ctrl[u] > hi ? hi : ctrl[u]);
  }
}

void or_task_lowpass(or_task* t, const or_model* m, const double* ctrl, int substep, double* out) {
  (void)substep;
  double f = m->timestep / (m->timestep + t->pt_time);
  for (int u = 0; u < m->nu; u++) t->ctrl_target[u] += (ctrl[u] - t->ctrl_target[u]) * f;
  t->ctrl_target[0] = -t->conveyor_speed;
  if (out) memcpy(out, t->ctrl_target, m->nu * sizeof(double));
}

int or_task_force_check(const or_task* t, const or_model* m, int ncon, const int* con_geom,
                        const double* con_force) {
  double mx = -1.0;
  int any = 0;
  for (int c = 0; c < ncon; c++) {
    int arm = 0;
    for (int s = 0; s < 2 && !arm; s++) {
      int g = con_geom[2 * c + s];
      for (int i = 0; i < m->A; i++)
        if (g >= m->arm_geom_lo[i] && g < m->arm_geom_hi[i]) arm = 1;
    }
    if (!arm) continue;
    any = 1;
    for (int k = 0; k < 6; k++) {
      double a = fabs(con_force[6 * c + k]);
      if (a > mx) mx = a;
    }
  }
  return any && mx > t->force_contact_threshold;
}

static void hide(or_task* t, const or_model* m, int obj, double* qpos, double* qvel) {
  t->out_scene[t->n_out++] = obj;
  double* q = qpos + cube_qadr(m, obj);
  q[0] = 4.0 + 1.0;
  q[1] = t->hidden_counter * 0.2;
  q[2] = 1.0;
  q[3] = 1.0;
  q[4] = q[5] = q[6] = 0.0;
  double* v = qvel + cube_dadr(m, obj);
  for (int i = 0; i < 6; i++) v[i] = 0.0;
  t->hidden_counter++;
}

static void pop_at(int* list, int* n, int idx) {
  for (int i = idx; i < *n - 1; i++) list[i] = list[i + 1];
  (*n)--;
}

void or_task_step(or_task* t, const or_model* m, double* qpos, double* qvel) {
  int spawn_steps = (int)(1.0 / (0.1 * t->spawn_freq));
  if (t->step_counter == 0 || t->steps_since_spawn >= spawn_steps) {
    if (t->n_out > 0) {
      int obj = t->out_scene[0];
      pop_at(t->out_scene, &t->n_out, 0);
      double* q = qpos + cube_qadr(m, obj);
      q[0] = 0.0;
      q[1] = 1.0;
      q[2] = 2.0;
      for (int k = 0; k < 4; k++) q[3 + k] = 0.0 + 1.0 * or_pcg64_double(&t->rng);
      t->in_scene[t->n_in++] = obj;
    }
    t->steps_since_spawn = 0;
  }
  /* _check_states */
  if (t->n_in > 0) {
    int n = t->n_in;
    int oob[64];
    for (int i = 0; i < n; i++) {
      const double* q = qpos + cube_qadr(m, t->in_scene[i]);
      oob[i] = fabs(q[0]) > 1.2 || q[1] < -1.5 || q[2] < 0.9;
    }
    for (int i = n - 1; i >= 0; i--) {
      if (!oob[i]) continue;
      int obj = t->in_scene[i];
      pop_at(t->in_scene, &t->n_in, i);
      hide(t, m, obj, qpos, qvel);
      t->failure_counter++;
    }
    if (t->n_in > 0) {
      /* obj_pos is read once, before both bucket loops (task_utils.py:103) */
      int n2 = t->n_in;
      double pos[64][3];
      for (int i = 0; i < n2; i++) memcpy(pos[i], qpos + cube_qadr(m, t->in_scene[i]), 3 * sizeof(double));
      for (int b = 0; b < 2; b++) {
        double bx = b == 0 ? 0.9 : -0.9, by = 0.7 - (m->A / 2 - 1), bz = 1.05 - 0.04;
        const double bs[3] = {0.29, 0.29, 0.02};
        for (int i = n2 - 1; i >= 0; i--) {
          int in_x = fabs(pos[i][0] - bx) <= BX * bs[0];
          int in_y = fabs(pos[i][1] - by) <= BX * bs[1];
          int in_z = pos[i][2] - bz - bs[2] / 2 <= 0.07;
          if (!(in_x && in_y && in_z)) continue;
          if (i >= t->n_in) continue; /* the reference raises IndexError here (list.pop out of range) */
          int obj = t->in_scene[i];
          pop_at(t->in_scene, &t->n_in, i);
          hide(t, m, obj, qpos, qvel);
          t->scores[b]++;
        }
      }
    }
  }
  t->step_counter++;
  t->steps_since_spawn++;
}

void or_task_after_step(or_task* t) {
  double dt = 0.001 * t->frame_skip;
  t->play_time += dt;
  t->conveyor_speed += t->conveyor_acceleration * dt;
  t->spawn_freq *= t->spawn_freq_increase;
}

void or_task_obs(const or_task* t, const or_model* m, const double* qpos, const double* qvel, float* obs) {
  int o = 0;
  for (int i = 0; i < m->A; i++) {
    /* arm joints 1..7 + left plate: the first 8 dofs of arm i */
    int jq = 1 + 7 * t->K + 9 * i; /* qpos layout: belt, cubes, arms */
    int jd = 1 + 6 * t->K + 9 * i;
    for (int j = 0; j < 8; j++) obs[o++] = (float)qpos[jq + j];
    for (int j = 0; j < 8; j++) obs[o++] = (float)qvel[jd + j];
    for (int j = 0; j < 8; j++) obs[o++] = (float)t->ctrl_target[1 + 8 * i + j];
  }
  /* objects sorted by x (stable), zero padded */
  int n = t->n_in, idx[64];
  for (int i = 0; i < n; i++) idx[i] = t->in_scene[i];
  for (int i = 1; i < n; i++) {
    int v = idx[i];
    double x = qpos[cube_qadr(m, v)];
    int j = i - 1;
    while (j >= 0 && qpos[cube_qadr(m, idx[j])] > x) {
      idx[j + 1] = idx[j];
      j--;
    }
    idx[j + 1] = v;
  }
  for (int k = 0; k < t->K; k++)
    for (int c = 0; c < 7; c++) obs[o + 7 * k + c] = k < n ? (float)qpos[cube_qadr(m, idx[k]) + c] : 0.0f;
  o += 7 * t->K;
  for (int k = 0; k < t->K; k++)
    for (int c = 0; c < 6; c++) obs[o + 6 * k + c] = k < n ? (float)qvel[cube_dadr(m, idx[k]) + c] : 0.0f;
}

double or_task_reward(or_task* t, const or_model* m, const double* qpos, const double* grip_site,
                      const float* action) {
  int score_delta = (t->scores[0] + t->scores[1]) - (t->last_score[0] + t->last_score[1]);
  double reward;
  if (t->reward_kind == 0) {
    reward = score_delta;
  } else {
    double gc = 0.0, bc = 0.0;
    int closest[16];
    for (int i = 0; i < m->A; i++) {
      const double* gp = grip_site + 3 * i;
      if (t->n_in == 0) {
        closest[i] = -1;
        gc += 0.0;
        continue;
      }
      double best = 0;
      int bi = -1;
      for (int c = 0; c < t->n_in; c++) {
        /* candidates: in-scene cubes this arm's IK policy does not ignore (environments.py:303-304) */
        int ign = 0;
        for (int o = 0; o < m->A; o++) ign |= t->ik_ignore[i][o] == t->in_scene[c];
        if (ign) continue;
        const double* q = qpos + cube_qadr(m, t->in_scene[c]);
        double dv[3] = {q[0] - gp[0], q[1] - gp[1], q[2] - gp[2]};
        double dd = sqrt(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2]);
        if (bi < 0 || dd < best) {
          best = dd;
          bi = c;
        }
      }
      if (bi < 0) { /* every candidate ignored: (None, last distance, 0) */
        closest[i] = -1;
        continue;
      }
      closest[i] = t->in_scene[bi];
      double change = t->last_grip_dist[i] - best;
      t->last_grip_dist[i] = best;
      gc += change;
    }
    for (int i = 0; i < m->A; i++) {
      if (closest[i] < 0) {
        bc += 0.0;
        continue;
      }
      const double* q = qpos + cube_qadr(m, closest[i]);
      double bx = (i % 2) == 0 ? 0.9 : -0.9, by = 0.7 - (m->A / 2 - 1), bz = 1.05 - 0.04;
      double dv[3] = {q[0] - bx, q[1] - by, q[2] - bz};
      double dd = sqrt(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2]);
      double change = t->last_bucket_dist[i] - dd;
      t->last_bucket_dist[i] = dd;
      bc += change;
    }
    /* np.exp(-np.linalg.norm(float32 actions)) stays float32; the sum is float64 (numpy 1.26,
       environment.yml:200, scalar promotion) */
    float ss = 0.0f;
    for (int i = 0; i < t->act_dim; i++)
      if (i % 8 != 7) ss += action[i] * action[i];
    float an = expf(-sqrtf(ss));
    double progress = t->base_reward + t->w_grip * gc + t->w_bucket * bc + t->w_action * (double)an;
    reward = score_delta > 0 ? (double)score_delta : progress;
  }
  t->last_score[0] = t->scores[0];
  t->last_score[1] = t->scores[1];
  return reward;
}

/* ------------------------------------------------------------------------------------------------
 * full environment: the env classes of src/environments.py (OR_ENV_*)
 * ------------------------------------------------------------------------------------------------ */
static int is_toggle(int c) { return c == OR_ENV_PAUSE_TOGGLE || c == OR_ENV_BACKUP_TOGGLE; }

or_env* or_env_create(int A, int K, uint64_t seed, int env_class, const double* w) {
  if (env_class < OR_ENV_FACTORY || env_class > OR_ENV_BACKUP_TOGGLE || A > OR_IK_MAXA) return NULL;
  or_env* e = calloc(1, sizeof(or_env));
  e->m = or_model_create(A, K, seed);
  if (!e->m) {
    free(e);
    return NULL;
  }
  e->d = or_data_create(e->m);
  e->ik_d = or_data_create(e->m);
  or_task_init(&e->t, A, K, seed);
  e->env_class = env_class;
  /* FactoryManipulationEnv and the IK-toggling envs keep the score-delta reward (environments.py:129-149,
   * 538-645); the other classes derive from ProgressRewardEnv (environments.py:251-535) */
  e->t.reward_kind = (env_class == OR_ENV_FACTORY || is_toggle(env_class)) ? 0 : 1;
  if (w) {
    e->t.w_grip = w[0];
    e->t.w_bucket = w[1];
    e->t.w_action = w[2];
    e->t.base_reward = w[3];
  }
  e->obs_dim = 24 * A + 13 * K + (is_toggle(env_class) ? 8 * A : 0);
  switch (env_class) {
    case OR_ENV_FACTORY: e->act_dim = 0; break;
    case OR_ENV_SINGLEFULLRL:
    case OR_ENV_SINGLEDELTA: e->act_dim = 8; break;
    case OR_ENV_PAUSE_TOGGLE:
    case OR_ENV_BACKUP_TOGGLE: e->act_dim = A; break;
    default: e->act_dim = 8 * A;
  }
  e->t.act_dim = e->act_dim;
  for (int i = 0; i < A; i++) {
    or_ik_arm_init(&e->ik[i]); /* IKPolicy(env, arm_id=i, bucket_idx=i % 2) (environments.py:39) */
    memset(e->pause_last[i], 0, sizeof e->pause_last[i]); /* np.zeros(dof) (environments.py:592) */
  }
  e->stage_qpos = calloc(e->m->nq, sizeof(double));
  e->stage_qvel = calloc(e->m->nv, sizeof(double));
  return e;
}

/* FactoryManipulationEnv._compose_control (environments.py:104-127): each arm's IKPolicy.act() in arm
 * order, clipped to actuator_ctrlrange[1:9]; then every other arm ignores this arm's target.  The IK solve
 * is a callback: qpos_from_site_pose in the env (or_ik_solve), recorded results in the golden replay. */
void or_ik_compose(const or_model* m, or_ik_arm* ik, const double* qpos, const double* qvel, const double* grip,
                   const double* base, const int* in_scene, int n_in, or_ik_solver solve, void* ctx,
                   double pt_time, double dt, double* arm_ctrl /* 8A */) {
  const int A = m->A, K = m->K;
  double cq[64 * 7], cv[64 * 6];
  for (int k = 0; k < K; k++) {
    memcpy(cq + 7 * k, qpos + cube_qadr(m, k), 7 * sizeof(double));
    memcpy(cv + 6 * k, qvel + cube_dadr(m, k), 6 * sizeof(double));
  }
  for (int i = 0; i < A; i++) {
    or_ik_arm* p = &ik[i];
    const double bucket[3] = {(i % 2) == 0 ? 0.9 : -0.9, 0.7 - (A / 2 - 1), 1.05 - 0.04};
    or_ik_in in = {A, n_in, in_scene, cq, cv, grip + 3 * i, base + 3 * i, bucket, qpos + 1 + 7 * K + 9 * i,
                   pt_time, dt};
    double tp[3], tq[4], ctrl[8];
    int close = 0;
    if (or_ik_plan(&in, p, tp, tq, &close)) {
      double q7[7];
      int ok = solve(ctx, i, tp, tq, q7);
      or_ik_finish(p, ok, q7, close, ctrl);
    } else {
      memcpy(ctrl, p->last_ctrl, sizeof ctrl);
    }
    for (int j = 0; j < 8; j++) {
      const double lo = m->act_ctrlrange[2 * (1 + j)], hi = m->act_ctrlrange[2 * (1 + j) + 1];
      arm_ctrl[8 * i + j] = ctrl[j] < lo ? lo : (ctrl[j] > hi ? hi : ctrl[j]);
    }
    for (int j = 0; j < A; j++)
      if (j != i) ik[j].ignore[i] = p->target;
  }
}

static int env_ik_solve(void* ctx, int arm, const double* tp, const double* tq, double* q7) {
  or_env* e = ctx;
  int steps = 0;
  int ok = or_ik_solve(e->m, e->ik_d, e->d->qpos, arm, tp, tq, q7, &steps);
  e->ik_steps += steps;
  e->ik_calls[arm]++;
  if (!ok) e->ik_fails[arm]++;
  return ok;
}

static void ik_compose(or_env* e, double* arm_ctrl) {
  const or_model* m = e->m;
  double grip[3 * OR_IK_MAXA], base[3 * OR_IK_MAXA];
  for (int i = 0; i < m->A; i++) {
    memcpy(grip + 3 * i, e->d->site_xpos + 3 * m->grip_site[i], 3 * sizeof(double));
    memcpy(base + 3 * i, e->d->site_xpos + 3 * m->base_site[i], 3 * sizeof(double));
  }
  e->ik_steps = 0;
  or_ik_compose(m, e->ik, e->d->qpos, e->d->qvel, grip, base, e->t.in_scene, e->t.n_in, env_ik_solve, e, e->t.pt_time,
                0.001 * e->t.frame_skip, arm_ctrl);
  for (int i = 0; i < m->A; i++)
    for (int o = 0; o < m->A; o++) e->t.ik_ignore[i][o] = e->ik[i].ignore[o];
}

/* _process_action of one arm's 8 action entries (environments.py:84-102) */
static void process8(const or_model* m, const float* a, double* out) {
  for (int j = 0; j < 8; j++) {
    float th = (float)tanh((double)a[j]);
    float s = (th + 1.0f) * 0.5f;
    double lo = m->act_ctrlrange[2 * (1 + j)], hi = m->act_ctrlrange[2 * (1 + j) + 1];
    out[j] = lo + (double)s * (hi - lo);
  }
}

/* _compose_control of the env class (environments.py:104-127, 405-420, 442-459, 481-495, 517-535,
 * 594-612, 628-645) -> the A arm commands handed to step_sim.  `ik` = the IK proposals of this compose
 * (non-toggle IK classes, already computed by or_ik_compose), `ik_state` = the policies' states after it;
 * toggles read the proposals of the last observation and update pause_last. */
void or_compose_class(const or_model* m, int env_class, const float* action, const double* ik, const int* ik_state,
                      const double* ik_actions /* 8A */, double* pause_last /* 8A */, double* arm_ctrl) {
  const int A = m->A;
  double pa[8];
  switch (env_class) {
    case OR_ENV_ALLFULLRL:
      or_task_process_action(m, action, arm_ctrl);
      break;
    case OR_ENV_FACTORY:
      memcpy(arm_ctrl, ik, 8 * A * sizeof(double));
      break;
    case OR_ENV_SINGLEFULLRL:
      memcpy(arm_ctrl, ik, 8 * A * sizeof(double));
      process8(m, action, arm_ctrl);
      break;
    case OR_ENV_SINGLEDELTA:
      memcpy(arm_ctrl, ik, 8 * A * sizeof(double));
      if (ik_state[0] != OR_IK_IDLE) {
        process8(m, action, pa);
        for (int j = 0; j < 8; j++) arm_ctrl[j] += 0.5 * pa[j];
      }
      break;
    case OR_ENV_ALLDELTA:
      memcpy(arm_ctrl, ik, 8 * A * sizeof(double));
      for (int i = 0; i < A; i++)
        if (ik_state[i] != OR_IK_IDLE) {
          process8(m, action + 8 * i, pa);
          for (int j = 0; j < 8; j++) arm_ctrl[8 * i + j] += 0.5 * pa[j];
        }
      break;
    case OR_ENV_PAUSE_TOGGLE:
      for (int i = 0; i < A; i++)
        memcpy(arm_ctrl + 8 * i, action[i] == 1.0f ? ik_actions + 8 * i : pause_last + 8 * i, 8 * sizeof(double));
      memcpy(pause_last, arm_ctrl, 8 * A * sizeof(double));
      break;
    case OR_ENV_BACKUP_TOGGLE:
      for (int i = 0; i < A; i++)
        memcpy(arm_ctrl + 8 * i, action[i] == 1.0f ? ik_actions + 8 * i : OR_IK_DEFAULT_POSE, 8 * sizeof(double));
      break;
  }
}

static void compose(or_env* e, const float* action, double* arm_ctrl) {
  const int A = e->m->A;
  double ik[8 * OR_IK_MAXA], ika[8 * OR_IK_MAXA], pl[8 * OR_IK_MAXA];
  int st[OR_IK_MAXA];
  const int c = e->env_class;
  if (c != OR_ENV_ALLFULLRL && !is_toggle(c)) ik_compose(e, ik);
  for (int i = 0; i < A; i++) {
    st[i] = e->ik[i].state;
    memcpy(ika + 8 * i, e->ik_actions[i], 8 * sizeof(double));
    memcpy(pl + 8 * i, e->pause_last[i], 8 * sizeof(double));
  }
  or_compose_class(e->m, c, action, ik, st, ika, pl, arm_ctrl);
  for (int i = 0; i < A; i++) memcpy(e->pause_last[i], pl + 8 * i, 8 * sizeof(double));
}

/* _process_observation (environments.py:55-82), IKTogglingEnv adds the proposals of a fresh
 * FactoryManipulationEnv._compose_control (environments.py:560-577) */
static void env_obs(or_env* e, float* obs) {
  if (is_toggle(e->env_class)) {
    double prop[8 * OR_IK_MAXA];
    ik_compose(e, prop);
    for (int i = 0; i < e->m->A; i++) memcpy(e->ik_actions[i], prop + 8 * i, 8 * sizeof(double));
  }
  if (!obs) return;
  or_task_obs(&e->t, e->m, e->d->qpos, e->d->qvel, obs);
  if (is_toggle(e->env_class)) {
    float* o = obs + 24 * e->m->A + 13 * e->m->K;
    for (int i = 0; i < e->m->A; i++)
      for (int j = 0; j < 8; j++) o[8 * i + j] = (float)e->ik_actions[i][j];
  }
}

void or_env_free(or_env* e) {
  if (!e) return;
  or_data_free(e->d);
  or_data_free(e->ik_d);
  or_model_free(e->m);
  free(e->stage_qpos);
  free(e->stage_qvel);
  free(e);
}

void or_env_reset(or_env* e, float* obs) {
  or_reset_data(e->m, e->d);
  or_task_reset(&e->t, e->m, e->d->qpos, e->d->qvel);
  e->d->actuation_disabled = 1;
  or_forward(e->m, e->d); /* physics.after_reset(): forward with actuation disabled */
  e->d->actuation_disabled = 0;
  memcpy(e->stage_qpos, e->d->qpos, e->m->nq * sizeof(double));
  memcpy(e->stage_qvel, e->d->qvel, e->m->nv * sizeof(double));
  e->ep_return = 0;
  e->ep_len = 0;
  for (int i = 0; i < e->m->A; i++) or_ik_arm_reset(&e->ik[i]); /* environments.py:243-244 */
  env_obs(e, obs);
}

int or_env_step(or_env* e, const float* action, float* obs, double* reward, double* info) {
  or_model* m = e->m;
  or_data* d = e->d;
  or_task* t = &e->t;
  double arm_ctrl[128], ctrl[128];
  compose(e, action, arm_ctrl);
  or_task_clip_ctrl(t, m, arm_ctrl, ctrl);
  int force_term = 0;
  for (int s = 0; s < t->frame_skip; s++) {
    or_task_lowpass(t, m, ctrl, s, d->ctrl);
    or_step2(m, d);
    if (s == t->frame_skip - 1) {
      /* contact-force check on the contacts + forces of the final solve */
      int cg[2 * 4096];
      double* cf = malloc(6 * (size_t)(d->ncon > 0 ? d->ncon : 1) * sizeof(double));
      for (int c = 0; c < d->ncon; c++) {
        cg[2 * c] = d->con[c].geom[0];
        cg[2 * c + 1] = d->con[c].geom[1];
        or_contact_force(m, d, c, cf + 6 * c);
      }
      force_term = or_task_force_check(t, m, d->ncon, cg, cf);
      free(cf);
    }
    or_step1(m, d);
  }
  or_task_step(t, m, d->qpos, d->qvel);
  or_task_after_step(t);
  /* the TaskManager's teleports (spawn / hide) are seen by the next substep's dynamics: MuJoCo's own outputs in
   * the reference show a cube spawned from rest on the floor falling freely from its first substep (its
   * (z, vz) after n env-steps is exact free fall over 100 n substeps, tests/test_physics_pins.py), not held for one
   * substep by the pre-teleport floor contact -- so the stage is recomputed at the post-teleport state */
  or_step1(m, d);
  memcpy(e->stage_qpos, d->qpos, m->nq * sizeof(double));
  memcpy(e->stage_qvel, d->qvel, m->nv * sizeof(double));
  int terminated = t->failure_counter > 0 || force_term;
  double grip[48];
  for (int i = 0; i < m->A; i++) memcpy(grip + 3 * i, d->site_xpos + 3 * m->grip_site[i], 3 * sizeof(double));
  *reward = or_task_reward(t, m, d->qpos, grip, action);
  e->ep_return += *reward;
  e->ep_len++;
  env_obs(e, obs);
  if (info) {
    info[0] = t->scores[0];
    info[1] = t->scores[1];
    info[2] = t->play_time;
    info[3] = t->conveyor_speed;
    info[4] = t->failure_counter > 0;
    info[5] = force_term;
    info[6] = t->n_in;
  }
  return terminated;
}
