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
        const double* q = qpos + cube_qadr(m, t->in_scene[c]);
        double dv[3] = {q[0] - gp[0], q[1] - gp[1], q[2] - gp[2]};
        double dd = sqrt(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2]);
        if (bi < 0 || dd < best) {
          best = dd;
          bi = c;
        }
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
    for (int i = 0; i < 8 * m->A; i++)
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
 * full environment: AllFullRLProgressRewardEnv / FactoryManipulationEnv-style score reward
 * ------------------------------------------------------------------------------------------------ */
or_env* or_env_create(int A, int K, uint64_t seed, int reward_kind, const double* w) {
  or_env* e = calloc(1, sizeof(or_env));
  e->m = or_model_create(A, K, seed);
  if (!e->m) {
    free(e);
    return NULL;
  }
  e->d = or_data_create(e->m);
  or_task_init(&e->t, A, K, seed);
  e->t.reward_kind = reward_kind;
  if (w) {
    e->t.w_grip = w[0];
    e->t.w_bucket = w[1];
    e->t.w_action = w[2];
    e->t.base_reward = w[3];
  }
  e->obs_dim = 24 * A + 13 * K;
  e->act_dim = 8 * A;
  e->stage_qpos = calloc(e->m->nq, sizeof(double));
  e->stage_qvel = calloc(e->m->nv, sizeof(double));
  return e;
}

void or_env_free(or_env* e) {
  if (!e) return;
  or_data_free(e->d);
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
  if (obs) or_task_obs(&e->t, e->m, e->d->qpos, e->d->qvel, obs);
}

int or_env_step(or_env* e, const float* action, float* obs, double* reward, double* info) {
  or_model* m = e->m;
  or_data* d = e->d;
  or_task* t = &e->t;
  double arm_ctrl[128], ctrl[128];
  or_task_process_action(m, action, arm_ctrl);
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
  memcpy(e->stage_qpos, d->qpos, m->nq * sizeof(double));
  memcpy(e->stage_qvel, d->qvel, m->nv * sizeof(double));
  or_task_step(t, m, d->qpos, d->qvel);
  or_task_after_step(t);
  int terminated = t->failure_counter > 0 || force_term;
  double grip[48];
  for (int i = 0; i < m->A; i++) memcpy(grip + 3 * i, d->site_xpos + 3 * m->grip_site[i], 3 * sizeof(double));
  *reward = or_task_reward(t, m, d->qpos, grip, action);
  e->ep_return += *reward;
  e->ep_len++;
  if (obs) or_task_obs(t, m, d->qpos, d->qvel, obs);
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
