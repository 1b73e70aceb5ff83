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
