/* capi.c -- flat accessors so tests can drive the oracle through ctypes (TEST INFRASTRUCTURE). */
#include <stdlib.h>

#include "oracle.h"
#include "oracle_internal.h"

int or_m_int(const or_model* m, const char* what) {
#define F(x) if (!strcmp(what, #x)) return m->x
  F(A); F(K); F(nbody); F(njnt); F(nq); F(nv); F(ngeom); F(nsite); F(nu); F(neq); F(nexclude); F(cube_body0);
#undef F
  return -1;
}

double or_m_meaninertia(const or_model* m) { return m->meaninertia; }
const double* or_m_body_invweight0(const or_model* m) { return m->body_invweight0; }
const double* or_m_dof_invweight0(const or_model* m) { return m->dof_invweight0; }
const double* or_m_cube_size(const or_model* m) { return m->cube_size; }
const double* or_m_body_mass(const or_model* m) { return m->body_mass; }
const int* or_m_geom_body(const or_model* m) { return m->geom_body; }
const int* or_m_geom_type(const or_model* m) { return m->geom_type; }
const double* or_m_geom_size(const or_model* m) { return m->geom_size; }
const int* or_m_arm_geom_lo(const or_model* m) { return m->arm_geom_lo; }
const int* or_m_arm_geom_hi(const or_model* m) { return m->arm_geom_hi; }
const double* or_m_act_ctrlrange(const or_model* m) { return m->act_ctrlrange; }
int or_m_grip_site(const or_model* m, int i) { return m->grip_site[i]; }

or_model* or_env_model(or_env* e) { return e->m; }
or_data* or_env_data(or_env* e) { return e->d; }
or_task* or_env_task(or_env* e) { return &e->t; }
int or_env_obs_dim(const or_env* e) { return e->obs_dim; }

double* or_d_qpos(or_data* d) { return d->qpos; }
double* or_d_qvel(or_data* d) { return d->qvel; }
double* or_d_ctrl(or_data* d) { return d->ctrl; }
double* or_d_qacc(or_data* d) { return d->qacc; }
double* or_d_qacc_warmstart(or_data* d) { return d->qacc_warmstart; }
double* or_d_M(or_data* d) { return d->M; }
double* or_d_qfrc_bias(or_data* d) { return d->qfrc_bias; }
double* or_d_qfrc_constraint(or_data* d) { return d->qfrc_constraint; }
double* or_d_xpos(or_data* d) { return d->xpos; }
double* or_d_xmat(or_data* d) { return d->xmat; }
double* or_d_xipos(or_data* d) { return d->xipos; }
double* or_d_geom_xpos(or_data* d) { return d->geom_xpos; }
double* or_d_geom_xmat(or_data* d) { return d->geom_xmat; }
double* or_d_site_xpos(or_data* d) { return d->site_xpos; }
double* or_d_efc_force(or_data* d) { return d->efc_force; }
double* or_d_qacc_smooth(or_data* d) { return d->qacc_smooth; }
double* or_d_qfrc_smooth(or_data* d) { return d->qfrc_smooth; }
double* or_d_qfrc_passive(or_data* d) { return d->qfrc_passive; }
int* or_d_efc_type(or_data* d) { return d->efc_type; }
double* or_d_efc_pos(or_data* d) { return d->efc_pos; }
double* or_d_efc_D(or_data* d) { return d->efc_D; }
double* or_d_efc_aref(or_data* d) { return d->efc_aref; }
double* or_d_efc_J(or_data* d) { return d->efc_J; }
double* or_d_stage_fwd(const or_model* m, or_data* d, int actuated) {
  /* mj_step1 at the current qpos/qvel + actuation + smooth acceleration + solve (no integration) */
  d->actuation_disabled = !actuated;
  or_forward(m, d);
  d->actuation_disabled = 0;
  return d->qacc;
}
int or_d_ncon(const or_data* d) { return d->ncon; }
int or_d_nefc(const or_data* d) { return d->nefc; }
int or_d_niter(const or_data* d) { return d->solver_niter; }
void or_d_set_actuation_disabled(or_data* d, int v) { d->actuation_disabled = v; }

/* contact i: geom1, geom2, dist, pos[3], frame[9], mu */
void or_d_contact(const or_data* d, int i, int* geoms, double* out) {
  const or_contact* c = d->con + i;
  geoms[0] = c->geom[0];
  geoms[1] = c->geom[1];
  out[0] = c->dist;
  memcpy(out + 1, c->pos, 3 * sizeof(double));
  memcpy(out + 4, c->frame, 9 * sizeof(double));
  out[13] = c->mu;
}

/* one dm_control legacy physics.step() with the given ctrl */
void or_physics_step(const or_model* m, or_data* d, const double* ctrl) {
  memcpy(d->ctrl, ctrl, m->nu * sizeof(double));
  or_step2(m, d);
  or_step1(m, d);
}

/* task state accessors */
int or_t_int(const or_task* t, const char* what) {
#define F(x) if (!strcmp(what, #x)) return t->x
  F(n_in); F(n_out); F(step_counter); F(steps_since_spawn); F(failure_counter); F(hidden_counter);
#undef F
  if (!strcmp(what, "score0")) return t->scores[0];
  if (!strcmp(what, "score1")) return t->scores[1];
  return -1;
}
const int* or_t_in_scene(const or_task* t) { return t->in_scene; }
double or_t_double(const or_task* t, const char* what) {
#define F(x) if (!strcmp(what, #x)) return t->x
  F(spawn_freq); F(conveyor_speed); F(play_time);
#undef F
  return 0.0 / 0.0;
}
double* or_t_ctrl_target(or_task* t) { return t->ctrl_target; }
void or_t_set_reward(or_task* t, int kind, const double* w) {
  t->reward_kind = kind;
  t->w_grip = w[0];
  t->w_bucket = w[1];
  t->w_action = w[2];
  t->base_reward = w[3];
}
or_task* or_task_new(int A, int K, uint64_t seed) {
  or_task* t = malloc(sizeof(or_task));
  or_task_init(t, A, K, seed);
  return t;
}
void or_task_free(or_task* t) { free(t); }

/* ---- exchange of the full arena state with the product's record layout (include/factorysim.h,
 *      fm_get_state / fm_set_state): doubles [qpos nq | qvel nv | qpos_stage nq | qvel_stage nv |
 *      qacc_warmstart nv | ctrl_target nu | spawn_freq | speed | play_time | last_grip A |
 *      last_bucket A | ep_return], int32 [in K | out K | n_in n_out step since fail hidden s0 s1 ls0 ls1 eplen],
 *      uint64 [state_hi state_lo inc_hi inc_lo]
 *      IK block (every env class): doubles A x [last_ctrl 8 | move_start 3 | ik_actions 8 | pause_last 8]
 *      after ep_return, int32 A x [state counter target ignore[A]] after eplen */
void or_env_export(const or_env* e, double* dbl, int32_t* ints, uint64_t* rng) {
  const or_model* m = e->m;
  const or_data* d = e->d;
  const or_task* t = &e->t;
  int nq = m->nq, nv = m->nv, nu = m->nu, A = m->A, K = m->K;
  double* p = dbl;
  memcpy(p, d->qpos, nq * sizeof(double)); p += nq;
  memcpy(p, d->qvel, nv * sizeof(double)); p += nv;
  memcpy(p, e->stage_qpos, nq * sizeof(double)); p += nq;
  memcpy(p, e->stage_qvel, nv * sizeof(double)); p += nv;
  memcpy(p, d->qacc_warmstart, nv * sizeof(double)); p += nv;
  memcpy(p, t->ctrl_target, nu * sizeof(double)); p += nu;
  *p++ = t->spawn_freq;
  *p++ = t->conveyor_speed;
  *p++ = t->play_time;
  for (int i = 0; i < A; i++) *p++ = t->last_grip_dist[i];
  for (int i = 0; i < A; i++) *p++ = t->last_bucket_dist[i];
  *p++ = e->ep_return;
  for (int i = 0; i < A; i++) {
    memcpy(p, e->ik[i].last_ctrl, 8 * sizeof(double)); p += 8;
    memcpy(p, e->ik[i].move_start, 3 * sizeof(double)); p += 3;
    memcpy(p, e->ik_actions[i], 8 * sizeof(double)); p += 8;
    memcpy(p, e->pause_last[i], 8 * sizeof(double)); p += 8;
  }
  int32_t* q = ints;
  for (int k = 0; k < K; k++) q[k] = k < t->n_in ? t->in_scene[k] : -1;
  for (int k = 0; k < K; k++) q[K + k] = k < t->n_out ? t->out_scene[k] : -1;
  q += 2 * K;
  q[0] = t->n_in; q[1] = t->n_out; q[2] = t->step_counter; q[3] = t->steps_since_spawn;
  q[4] = t->failure_counter; q[5] = t->hidden_counter; q[6] = t->scores[0]; q[7] = t->scores[1];
  q[8] = t->last_score[0]; q[9] = t->last_score[1]; q[10] = e->ep_len;
  q += 11;
  for (int i = 0; i < A; i++) {
    *q++ = e->ik[i].state; *q++ = e->ik[i].counter; *q++ = e->ik[i].target;
    for (int o = 0; o < A; o++) *q++ = e->ik[i].ignore[o];
  }
  rng[0] = t->rng.state_hi; rng[1] = t->rng.state_lo; rng[2] = t->rng.inc_hi; rng[3] = t->rng.inc_lo;
}

/* set the oracle from a record; the position/velocity stage is recomputed at qpos_stage/qvel_stage */
void or_env_import(or_env* e, const double* dbl, const int32_t* ints, const uint64_t* rng) {
  const or_model* m = e->m;
  or_data* d = e->d;
  or_task* t = &e->t;
  int nq = m->nq, nv = m->nv, nu = m->nu, A = m->A, K = m->K;
  const double* p = dbl;
  const double* q_now = p; p += nq;
  const double* v_now = p; p += nv;
  memcpy(e->stage_qpos, p, nq * sizeof(double)); p += nq;
  memcpy(e->stage_qvel, p, nv * sizeof(double)); p += nv;
  memcpy(d->qacc_warmstart, p, nv * sizeof(double)); p += nv;
  memcpy(t->ctrl_target, p, nu * sizeof(double)); p += nu;
  t->spawn_freq = *p++;
  t->conveyor_speed = *p++;
  t->play_time = *p++;
  for (int i = 0; i < A; i++) t->last_grip_dist[i] = *p++;
  for (int i = 0; i < A; i++) t->last_bucket_dist[i] = *p++;
  e->ep_return = *p++;
  for (int i = 0; i < A; i++) {
    memcpy(e->ik[i].last_ctrl, p, 8 * sizeof(double)); p += 8;
    memcpy(e->ik[i].move_start, p, 3 * sizeof(double)); p += 3;
    memcpy(e->ik_actions[i], p, 8 * sizeof(double)); p += 8;
    memcpy(e->pause_last[i], p, 8 * sizeof(double)); p += 8;
  }
  const int32_t* q = ints + 2 * K;
  t->n_in = q[0]; t->n_out = q[1]; t->step_counter = q[2]; t->steps_since_spawn = q[3];
  t->failure_counter = q[4]; t->hidden_counter = q[5]; t->scores[0] = q[6]; t->scores[1] = q[7];
  t->last_score[0] = q[8]; t->last_score[1] = q[9]; e->ep_len = q[10];
  {
    const int32_t* r = q + 11;
    for (int i = 0; i < A; i++) {
      e->ik[i].state = *r++; e->ik[i].counter = *r++; e->ik[i].target = *r++;
      for (int o = 0; o < A; o++) e->ik[i].ignore[o] = *r++;
    }
    for (int i = 0; i < A; i++)
      for (int o = 0; o < A; o++) t->ik_ignore[i][o] = e->ik[i].ignore[o];
  }
  for (int k = 0; k < K; k++) t->in_scene[k] = ints[k];
  for (int k = 0; k < K; k++) t->out_scene[k] = ints[K + k];
  t->rng.state_hi = rng[0]; t->rng.state_lo = rng[1]; t->rng.inc_hi = rng[2]; t->rng.inc_lo = rng[3];
  /* stage at the stage state, then the current state on top (legacy-step semantics) */
  memcpy(d->qpos, e->stage_qpos, nq * sizeof(double));
  memcpy(d->qvel, e->stage_qvel, nv * sizeof(double));
  or_step1(m, d);
  memcpy(d->qpos, q_now, nq * sizeof(double));
  memcpy(d->qvel, v_now, nv * sizeof(double));
}

/* CPU baseline leg of bench.py: n arenas x `steps` env-steps of the oracle with uniform random
 * AllFullRL actions, OpenMP over arenas (one arena per thread at a time), auto-reset on termination.
 * Returns wall seconds of the stepping (env creation and reset excluded). */
#include <omp.h>
double or_batch_bench(int A, int K, int n, int steps, int threads, uint64_t seed, int64_t* env_steps_out) {
  or_env** envs = malloc(n * sizeof(or_env*));
  const double w[4] = {0.2, 0.4, 0.0, 0.4};
  for (int i = 0; i < n; i++) {
    envs[i] = or_env_create(A, K, 42, 1, w);
    or_env_reset(envs[i], NULL);
  }
  int64_t total = 0;
  double t0 = omp_get_wtime();
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1) reduction(+ : total)
  for (int i = 0; i < n; i++) {
    uint64_t s = seed * 0x9E3779B97F4A7C15ULL + (uint64_t)i * 0xD1B54A32D192ED03ULL + 1;
    float act[128];
    double rew, info[7];
    for (int t = 0; t < steps; t++) {
      for (int j = 0; j < 8 * A; j++) {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        act[j] = (float)((double)(s >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0);
      }
      if (or_env_step(envs[i], act, NULL, &rew, info)) or_env_reset(envs[i], NULL);
      total++;
    }
  }
  double dt = omp_get_wtime() - t0;
  for (int i = 0; i < n; i++) or_env_free(envs[i]);
  free(envs);
  if (env_steps_out) *env_steps_out = total;
  return dt;
}

/* ---- IK policy pieces on flat arrays (tests/test_oracle_golden.py replays the reference's FSM) ----
 * arm_i = [state, counter, target, ignore[16]], arm_d = [last_ctrl 8, move_start 3] */
static void arm_from_flat(or_ik_arm* p, const int* ai, const double* ad) {
  p->state = ai[0];
  p->counter = ai[1];
  p->target = ai[2];
  for (int o = 0; o < OR_IK_MAXA; o++) p->ignore[o] = ai[3 + o];
  memcpy(p->last_ctrl, ad, 8 * sizeof(double));
  memcpy(p->move_start, ad + 8, 3 * sizeof(double));
}
static void arm_to_flat(const or_ik_arm* p, int* ai, double* ad) {
  ai[0] = p->state;
  ai[1] = p->counter;
  ai[2] = p->target;
  for (int o = 0; o < OR_IK_MAXA; o++) ai[3 + o] = p->ignore[o];
  memcpy(ad, p->last_ctrl, 8 * sizeof(double));
  memcpy(ad + 8, p->move_start, 3 * sizeof(double));
}
void or_ik_arm_init_flat(int* ai, double* ad) {
  or_ik_arm p;
  or_ik_arm_init(&p);
  arm_to_flat(&p, ai, ad);
}
void or_ik_arm_reset_flat(int* ai, double* ad) {
  or_ik_arm p;
  arm_from_flat(&p, ai, ad);
  or_ik_arm_reset(&p);
  arm_to_flat(&p, ai, ad);
}
int or_ik_plan_flat(int A, int n_in, const int* in_scene, const double* cube_qpos, const double* cube_qvel,
                    const double* grip, const double* base, const double* bucket, const double* arm_q, int* ai,
                    double* ad, double* tpos, double* tquat, int* close) {
  or_ik_arm p;
  arm_from_flat(&p, ai, ad);
  or_ik_in in = {A, n_in, in_scene, cube_qpos, cube_qvel, grip, base, bucket, arm_q, 0.2, 0.001 * 100};
  int r = or_ik_plan(&in, &p, tpos, tquat, close);
  arm_to_flat(&p, ai, ad);
  return r;
}
void or_ik_finish_flat(int* ai, double* ad, int success, const double* q7, int close, double* ctrl) {
  or_ik_arm p;
  arm_from_flat(&p, ai, ad);
  or_ik_finish(&p, success, q7, close, ctrl);
  arm_to_flat(&p, ai, ad);
}
int or_env_act_dim(const or_env* e) { return e->act_dim; }
/* BaseEnv(pt_time=..., control_frequency=...) (base_env.py:28-31,133-135): the low-pass time constant, frame_skip
 * = int((1 / control_frequency) / timestep), and everything that follows env.dt (play time, conveyor speed, the IK
 * policy's step counts and compensation) */
void or_env_set_timing(or_env* e, double pt_time, double control_frequency) {
  e->t.pt_time = pt_time;
  e->t.frame_skip = (int)((1.0 / control_frequency) / 0.001);
}
int or_env_ik_steps(const or_env* e) { return e->ik_steps; }
long or_env_ik_calls(const or_env* e, int arm) { return e->ik_calls[arm]; }
long or_env_ik_fails(const or_env* e, int arm) { return e->ik_fails[arm]; }
void or_env_ik_arm(const or_env* e, int i, int* ai, double* ad) { arm_to_flat(&e->ik[i], ai, ad); }

/* golden replay of FactoryManipulationEnv._compose_control with the reference's (fake) IK results in call
 * order; the IK arguments of each call are written to args (tpos 3 | tquat 4 per call) */
typedef struct {
  const int* success;
  const double* q7;
  int n, calls;
  double* args;
} rec_solver;
static int rec_solve(void* ctx, int arm, const double* tp, const double* tq, double* q7) {
  rec_solver* r = ctx;
  (void)arm;
  if (r->calls >= r->n) return 0;
  memcpy(r->args + 7 * r->calls, tp, 3 * sizeof(double));
  memcpy(r->args + 7 * r->calls + 3, tq, 4 * sizeof(double));
  memcpy(q7, r->q7 + 7 * r->calls, 7 * sizeof(double));
  return r->success[r->calls++];
}
int or_ik_compose_replay(const or_model* m, int* arm_i /* A x 19 */, double* arm_d /* A x 11 */, const double* qpos,
                         const double* qvel, const double* grip, const double* base, const int* in_scene, int n_in,
                         const int* rec_success, const double* rec_q7, int n_rec, double* args_out,
                         double* arm_ctrl) {
  or_ik_arm ik[OR_IK_MAXA];
  for (int i = 0; i < m->A; i++) arm_from_flat(&ik[i], arm_i + 19 * i, arm_d + 11 * i);
  rec_solver r = {rec_success, rec_q7, n_rec, 0, args_out};
  or_ik_compose(m, ik, qpos, qvel, grip, base, in_scene, n_in, rec_solve, &r, 0.2, 0.001 * 100, arm_ctrl);
  for (int i = 0; i < m->A; i++) arm_to_flat(&ik[i], arm_i + 19 * i, arm_d + 11 * i);
  return r.calls;
}
void or_t_set_ignore(or_task* t, int arm, const int* values, int n) {
  for (int o = 0; o < 16; o++) t->ik_ignore[arm][o] = o < n ? values[o] : -1;
}
void or_t_set_act_dim(or_task* t, int act_dim) { t->act_dim = act_dim; }
void or_t_set_in_scene(or_task* t, const int* list, int n) {
  t->n_in = n;
  for (int i = 0; i < n; i++) t->in_scene[i] = list[i];
}
void or_t_set_scores(or_task* t, int s0, int s1) {
  t->scores[0] = s0;
  t->scores[1] = s1;
}
void or_t_reset_reward_state(or_task* t) { t->last_score[0] = t->last_score[1] = 0; } /* reset(): last_score */
