/* model.c -- scene model for the oracle (TEST INFRASTRUCTURE; see oracle.h header).
 *
 * Transcribes the compiled MuJoCo model of build_scene(num_objects=K, seed, num_arms=A)
 * (challenge_env/challenge_env/scene.py:109-169) from the MJCF assets:
 *   scene.xml:2 (implicitfast, dt=1 ms), scene.xml:21 (floor plane)
 *   scene.py:26-38 (table), conveyor_belt.xml:4-12 (belt, slide joint, velocity actuator)
 *   scene.py:9-23,121-134 (cubes: half size ~U(0.03,0.05) from default_rng(seed), mass 1000 h^3, freejoint)
 *   scene.py:64-106,136-145 (buckets: target_area + 4 fences at euler z = f*1.57 rad)
 *   scene.py:41-61,147-161 (arms: player_site pos/euler, iiwa14 attached to the site, gripper to attachment_site)
 *   iiwa14.xml:1-170 (links, inertials, 46 collision spheres, joint classes, excludes, PD actuators)
 *   gripper.xml:1-66 (gripper base, plates, joint equality, fixed tendon "split", tendon actuator)
 * Body / geom / joint numbering follows MuJoCo's preorder of the dm_control-generated MJCF
 * (DESIGN.md §2), so geom ids line up with BaseEnv.arm_geom_ids (base_env.py:121-130).
 * Compile-time constants that MuJoCo derives in mj_setConst (body_invweight0, dof_invweight0,
 * meaninertia) are computed here at qpos0 (see or_model_setconst).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "oracle_internal.h"

#define MAXB 256
#define MAXG 1024

typedef struct builder {
  or_model* m;
  int nb, nj, ng, ns, nu, ne, nx;
  int nq, nv;
} builder;

static void* zalloc(size_t n) { return calloc(n ? n : 1, 1); }

static int add_body(builder* b, int parent, const double pos[3], const double quat[4]) {
  or_model* m = b->m;
  int id = b->nb++;
  m->body_parent[id] = parent;
  memcpy(m->body_pos + 3 * id, pos, 3 * sizeof(double));
  double q[4] = {quat[0], quat[1], quat[2], quat[3]};
  or_quat_normalize(q);
  memcpy(m->body_quat + 4 * id, q, 4 * sizeof(double));
  m->body_iquat[4 * id] = 1.0;
  m->body_jntadr[id] = -1;
  m->body_dofadr[id] = -1;
  return id;
}

static void set_inertial(builder* b, int body, double mass, const double ipos[3], const double diag[3],
                         const double* iquat) {
  or_model* m = b->m;
  m->body_mass[body] = mass;
  memcpy(m->body_ipos + 3 * body, ipos, 3 * sizeof(double));
  memcpy(m->body_inertia + 3 * body, diag, 3 * sizeof(double));
  double q[4] = {1, 0, 0, 0};
  if (iquat) memcpy(q, iquat, 4 * sizeof(double));
  or_quat_normalize(q);
  memcpy(m->body_iquat + 4 * body, q, 4 * sizeof(double));
}

static int add_joint(builder* b, int body, int type, const double axis[3], int limited, double lo, double hi,
                     double damping) {
  or_model* m = b->m;
  int id = b->nj++;
  m->jnt_type[id] = type;
  m->jnt_body[id] = body;
  m->jnt_qposadr[id] = b->nq;
  m->jnt_dofadr[id] = b->nv;
  m->jnt_limited[id] = limited;
  m->jnt_range[2 * id] = lo;
  m->jnt_range[2 * id + 1] = hi;
  if (axis) memcpy(m->jnt_axis + 3 * id, axis, 3 * sizeof(double));
  m->jnt_solref[2 * id] = 0.02; /* MuJoCo default solreflimit */
  m->jnt_solref[2 * id + 1] = 1.0;
  const double si[5] = {0.9, 0.95, 0.001, 0.5, 2.0};
  memcpy(m->jnt_solimp + 5 * id, si, sizeof si);
  int nd = type == OR_JNT_FREE ? 6 : 1;
  int nqj = type == OR_JNT_FREE ? 7 : 1;
  if (m->body_jntadr[body] < 0) {
    m->body_jntadr[body] = id;
    m->body_dofadr[body] = b->nv;
  }
  m->body_jntnum[body]++;
  m->body_dofnum[body] += nd;
  for (int k = 0; k < nd; k++) {
    m->dof_body[b->nv + k] = body;
    m->dof_jnt[b->nv + k] = id;
    m->dof_damping[b->nv + k] = damping;
  }
  if (type == OR_JNT_FREE) {
    m->qpos0[b->nq + 3] = 1.0;
  }
  b->nq += nqj;
  b->nv += nd;
  return id;
}

/* geom defaults = MuJoCo defaults (friction 1 .005 .0001, solref .02 1, solimp .9 .95 .001 .5 2) */
static int add_geom(builder* b, int body, int type, const double size[3], const double pos[3], const double* quat,
                    int collide) {
  or_model* m = b->m;
  int id = b->ng++;
  m->geom_type[id] = type;
  m->geom_body[id] = body;
  m->geom_contype[id] = collide ? 1 : 0;
  m->geom_conaffinity[id] = collide ? 1 : 0;
  m->geom_condim[id] = 3;
  m->geom_priority[id] = 0;
  memcpy(m->geom_size + 3 * id, size, 3 * sizeof(double));
  if (pos) memcpy(m->geom_pos + 3 * id, pos, 3 * sizeof(double));
  double q[4] = {1, 0, 0, 0};
  if (quat) memcpy(q, quat, 4 * sizeof(double));
  or_quat_normalize(q);
  memcpy(m->geom_quat + 4 * id, q, 4 * sizeof(double));
  const double fr[3] = {1.0, 0.005, 0.0001};
  memcpy(m->geom_friction + 3 * id, fr, sizeof fr);
  m->geom_solref[2 * id] = 0.02;
  m->geom_solref[2 * id + 1] = 1.0;
  const double si[5] = {0.9, 0.95, 0.001, 0.5, 2.0};
  memcpy(m->geom_solimp + 5 * id, si, sizeof si);
  m->geom_solmix[id] = 1.0;
  m->geom_margin[id] = 0.0;
  if (type == OR_GEOM_SPHERE)
    m->geom_rbound[id] = size[0];
  else if (type == OR_GEOM_BOX)
    m->geom_rbound[id] = sqrt(size[0] * size[0] + size[1] * size[1] + size[2] * size[2]);
  else
    m->geom_rbound[id] = 0.0;
  return id;
}

static void geom_params(or_model* m, int g, const double* friction, const double* solref, const double* solimp3,
                        int priority) {
  if (friction) memcpy(m->geom_friction + 3 * g, friction, 3 * sizeof(double));
  if (solref) memcpy(m->geom_solref + 2 * g, solref, 2 * sizeof(double));
  if (solimp3) memcpy(m->geom_solimp + 5 * g, solimp3, 3 * sizeof(double));
  m->geom_priority[g] = priority;
}

static int add_site(builder* b, int body, const double pos[3], const double* quat) {
  or_model* m = b->m;
  int id = b->ns++;
  m->site_body[id] = body;
  memcpy(m->site_pos + 3 * id, pos, 3 * sizeof(double));
  double q[4] = {1, 0, 0, 0};
  if (quat) memcpy(q, quat, 4 * sizeof(double));
  or_quat_normalize(q);
  memcpy(m->site_quat + 4 * id, q, 4 * sizeof(double));
  return id;
}

static void add_exclude(builder* b, int b0, int b1) {
  int lo = b0 < b1 ? b0 : b1, hi = b0 < b1 ? b1 : b0;
  b->m->exclude[2 * b->nx] = lo;
  b->m->exclude[2 * b->nx + 1] = hi;
  b->nx++;
}

static void euler_z(double a, double q[4]) {
  q[0] = cos(a / 2);
  q[1] = 0;
  q[2] = 0;
  q[3] = sin(a / 2);
}

static void sphere(builder* b, int body, double r, double x, double y, double z) {
  const double s[3] = {r, 0, 0}, p[3] = {x, y, z};
  add_geom(b, body, OR_GEOM_SPHERE, s, p, NULL, 1);
}

static void visual(builder* b, int body) {
  const double s[3] = {0, 0, 0};
  add_geom(b, body, OR_GEOM_SPHERE, s, NULL, NULL, 0); /* mesh geom of class "visual": never collides */
}

static void alloc_model(or_model* m) {
#define A_(f, n) m->f = zalloc((n) * sizeof(*m->f))
  A_(body_parent, MAXB); A_(body_jntadr, MAXB); A_(body_jntnum, MAXB); A_(body_dofadr, MAXB);
  A_(body_dofnum, MAXB); A_(body_weldid, MAXB);
  A_(body_pos, 3 * MAXB); A_(body_quat, 4 * MAXB); A_(body_ipos, 3 * MAXB); A_(body_iquat, 4 * MAXB);
  A_(body_mass, MAXB); A_(body_inertia, 3 * MAXB); A_(body_invweight0, 2 * MAXB);
  A_(jnt_type, MAXB); A_(jnt_body, MAXB); A_(jnt_qposadr, MAXB); A_(jnt_dofadr, MAXB); A_(jnt_limited, MAXB);
  A_(jnt_axis, 3 * MAXB); A_(jnt_range, 2 * MAXB); A_(jnt_solref, 2 * MAXB); A_(jnt_solimp, 5 * MAXB);
  A_(dof_body, 4 * MAXB); A_(dof_jnt, 4 * MAXB); A_(dof_damping, 4 * MAXB); A_(dof_invweight0, 4 * MAXB);
  A_(geom_type, MAXG); A_(geom_body, MAXG); A_(geom_contype, MAXG); A_(geom_conaffinity, MAXG);
  A_(geom_condim, MAXG); A_(geom_priority, MAXG);
  A_(geom_size, 3 * MAXG); A_(geom_pos, 3 * MAXG); A_(geom_quat, 4 * MAXG); A_(geom_friction, 3 * MAXG);
  A_(geom_solref, 2 * MAXG); A_(geom_solimp, 5 * MAXG); A_(geom_solmix, MAXG); A_(geom_margin, MAXG);
  A_(geom_rbound, MAXG);
  A_(site_body, MAXB); A_(site_pos, 3 * MAXB); A_(site_quat, 4 * MAXB);
  A_(act_dof0, MAXB); A_(act_dof1, MAXB); A_(act_forcelimited, MAXB); A_(act_coef0, MAXB); A_(act_coef1, MAXB);
  A_(act_gain, MAXB); A_(act_bias, 3 * MAXB); A_(act_ctrlrange, 2 * MAXB); A_(act_forcerange, 2 * MAXB);
  A_(eq_dof0, 64); A_(eq_dof1, 64); A_(eq_solref, 2 * 64); A_(eq_solimp, 5 * 64);
  A_(exclude, 2 * MAXB); A_(qpos0, 4 * MAXB);
  A_(arm_geom_lo, 64); A_(arm_geom_hi, 64); A_(grip_site, 64); A_(base_site, 64); A_(cube_size, 256);
#undef A_
}

void or_model_free(or_model* m) {
  if (!m) return;
  void** fields[] = {
      (void**)&m->body_parent, (void**)&m->body_jntadr, (void**)&m->body_jntnum, (void**)&m->body_dofadr,
      (void**)&m->body_dofnum, (void**)&m->body_weldid, (void**)&m->body_pos, (void**)&m->body_quat,
      (void**)&m->body_ipos, (void**)&m->body_iquat, (void**)&m->body_mass, (void**)&m->body_inertia,
      (void**)&m->body_invweight0, (void**)&m->jnt_type, (void**)&m->jnt_body, (void**)&m->jnt_qposadr,
      (void**)&m->jnt_dofadr, (void**)&m->jnt_limited, (void**)&m->jnt_axis, (void**)&m->jnt_range,
      (void**)&m->jnt_solref, (void**)&m->jnt_solimp, (void**)&m->dof_body, (void**)&m->dof_jnt,
      (void**)&m->dof_damping, (void**)&m->dof_invweight0, (void**)&m->geom_type, (void**)&m->geom_body,
      (void**)&m->geom_contype, (void**)&m->geom_conaffinity, (void**)&m->geom_condim, (void**)&m->geom_priority,
      (void**)&m->geom_size, (void**)&m->geom_pos, (void**)&m->geom_quat, (void**)&m->geom_friction,
      (void**)&m->geom_solref, (void**)&m->geom_solimp, (void**)&m->geom_solmix, (void**)&m->geom_margin,
      (void**)&m->geom_rbound, (void**)&m->site_body, (void**)&m->site_pos, (void**)&m->site_quat,
      (void**)&m->act_dof0, (void**)&m->act_dof1, (void**)&m->act_forcelimited, (void**)&m->act_coef0,
      (void**)&m->act_coef1, (void**)&m->act_gain, (void**)&m->act_bias, (void**)&m->act_ctrlrange,
      (void**)&m->act_forcerange, (void**)&m->eq_dof0, (void**)&m->eq_dof1, (void**)&m->eq_solref,
      (void**)&m->eq_solimp, (void**)&m->exclude, (void**)&m->qpos0, (void**)&m->arm_geom_lo,
      (void**)&m->arm_geom_hi, (void**)&m->grip_site, (void**)&m->base_site, (void**)&m->cube_size, (void**)&m->cpair,
      (void**)&m->run_lo, (void**)&m->run_geom, (void**)&m->run_body, (void**)&m->run_margin};
  for (size_t i = 0; i < sizeof fields / sizeof fields[0]; i++) free(*fields[i]);
  free(m);
}

/* one KUKA iiwa14 + gripper (iiwa14.xml:55-147, gripper.xml:4-64) attached at a site frame */
static void build_arm(builder* b, int arm, const double site_pos[3], double yaw) {
  or_model* m = b->m;
  const double z3[3] = {0, 0, 0}, id4[4] = {1, 0, 0, 0}, zax[3] = {0, 0, 1};
  double sq[4];
  euler_z(yaw, sq);
  int frame = add_body(b, 0, z3, id4);             /* "arm{i}/" */
  m->base_site[arm] = add_site(b, frame, site_pos, sq); /* player_site */
  int iiwa = add_body(b, frame, site_pos, sq);      /* "arm{i}/iiwa14/" frame at the site */
  m->arm_geom_lo[arm] = b->ng;
  /* base (iiwa14.xml:55-61) -- static */
  int base = add_body(b, iiwa, z3, id4);
  set_inertial(b, base, 5.0, (double[3]){-0.1, 0, 0.07}, (double[3]){0.05, 0.06, 0.03}, NULL);
  visual(b, base);
  sphere(b, base, 0.12, 0, 0, 0.03);
  sphere(b, base, 0.08, -0.08, 0, 0.103);
  sphere(b, base, 0.08, -0.08, 0, 0.04);
  sphere(b, base, 0.1, 0, 0, 0.14);
  const double r1 = 2.96706, r2 = 2.0944, r3 = 3.05433;
  /* link1 (iiwa14.xml:62-71) */
  int l1 = add_body(b, base, (double[3]){0, 0, 0.1575}, id4);
  set_inertial(b, l1, 5.76, (double[3]){0, -0.03, 0.12}, (double[3]){0.0333, 0.033, 0.0123}, NULL);
  add_joint(b, l1, OR_JNT_HINGE, zax, 1, -r1, r1, 0);
  visual(b, l1);
  sphere(b, l1, 0.08, 0, 0, -0.0005);
  sphere(b, l1, 0.075, 0.01, -0.025, 0.0425);
  sphere(b, l1, 0.075, -0.01, -0.025, 0.0425);
  sphere(b, l1, 0.07, 0.01, -0.045, 0.1025);
  sphere(b, l1, 0.07, -0.01, -0.045, 0.1025);
  /* link2 (iiwa14.xml:71-84) */
  int l2 = add_body(b, l1, (double[3]){0, 0, 0.2025}, (double[4]){0, 0, 1, 1});
  set_inertial(b, l2, 6.35, (double[3]){0.0003, 0.059, 0.042}, (double[3]){0.0305, 0.0304, 0.011},
               (double[4]){0, 0, 1, 1});
  add_joint(b, l2, OR_JNT_HINGE, zax, 1, -r2, r2, 0);
  visual(b, l2);
  visual(b, l2);
  sphere(b, l2, 0.095, 0, 0, -0.01);
  sphere(b, l2, 0.09, 0, 0, 0.045);
  sphere(b, l2, 0.07, -0.01, 0.04, 0.054);
  sphere(b, l2, 0.065, -0.01, 0.09, 0.04);
  sphere(b, l2, 0.065, -0.01, 0.13, 0.02);
  sphere(b, l2, 0.07, 0.01, 0.04, 0.054);
  sphere(b, l2, 0.065, 0.01, 0.09, 0.04);
  sphere(b, l2, 0.065, 0.01, 0.13, 0.02);
  sphere(b, l2, 0.075, 0, 0.18, 0);
  /* link3 (iiwa14.xml:85-99) */
  int l3 = add_body(b, l2, (double[3]){0, 0.2045, 0}, (double[4]){0, 0, 1, 1});
  set_inertial(b, l3, 3.5, (double[3]){0, 0.03, 0.13}, (double[3]){0.025, 0.0238, 0.0076}, NULL);
  add_joint(b, l3, OR_JNT_HINGE, zax, 1, -r1, r1, 0);
  visual(b, l3);
  visual(b, l3);
  visual(b, l3);
  sphere(b, l3, 0.075, 0, 0, 0.0355);
  sphere(b, l3, 0.06, 0.01, 0.023, 0.0855);
  sphere(b, l3, 0.055, 0.01, 0.048, 0.1255);
  sphere(b, l3, 0.06, 0.01, 0.056, 0.1755);
  sphere(b, l3, 0.06, -0.01, 0.023, 0.0855);
  sphere(b, l3, 0.055, -0.01, 0.048, 0.1255);
  sphere(b, l3, 0.06, -0.01, 0.056, 0.1755);
  sphere(b, l3, 0.075, 0, 0.045, 0.2155);
  sphere(b, l3, 0.075, 0, 0, 0.2155);
  /* link4 (iiwa14.xml:100-111) */
  int l4 = add_body(b, l3, (double[3]){0, 0, 0.2155}, (double[4]){1, 1, 0, 0});
  set_inertial(b, l4, 3.5, (double[3]){0, 0.067, 0.034}, (double[3]){0.017, 0.0164, 0.006},
               (double[4]){1, 1, 0, 0});
  add_joint(b, l4, OR_JNT_HINGE, zax, 1, -r2, r2, 0);
  visual(b, l4);
  visual(b, l4);
  sphere(b, l4, 0.078, 0, 0.01, 0.046);
  sphere(b, l4, 0.06, 0.01, 0.06, 0.052);
  sphere(b, l4, 0.065, 0.01, 0.12, 0.034);
  sphere(b, l4, 0.06, -0.01, 0.06, 0.052);
  sphere(b, l4, 0.065, -0.01, 0.12, 0.034);
  sphere(b, l4, 0.075, 0, 0.184, 0);
  /* link5 (iiwa14.xml:111-125) */
  int l5 = add_body(b, l4, (double[3]){0, 0.1845, 0}, (double[4]){0, 0, 1, 1});
  set_inertial(b, l5, 3.5, (double[3]){0.0001, 0.021, 0.076}, (double[3]){0.01, 0.0087, 0.00449}, NULL);
  add_joint(b, l5, OR_JNT_HINGE, zax, 1, -r1, r1, 0);
  visual(b, l5);
  visual(b, l5);
  visual(b, l5);
  sphere(b, l5, 0.075, 0, 0, 0.0335);
  sphere(b, l5, 0.05, -0.012, 0.031, 0.0755);
  sphere(b, l5, 0.05, 0.012, 0.031, 0.0755);
  sphere(b, l5, 0.04, -0.012, 0.06, 0.1155);
  sphere(b, l5, 0.04, 0.012, 0.06, 0.1155);
  sphere(b, l5, 0.04, -0.01, 0.065, 0.1655);
  sphere(b, l5, 0.04, 0.01, 0.065, 0.1655);
  sphere(b, l5, 0.035, -0.012, 0.065, 0.1855);
  sphere(b, l5, 0.035, 0.012, 0.065, 0.1855);
  /* link6 (iiwa14.xml:126-133) */
  int l6 = add_body(b, l5, (double[3]){0, 0, 0.2155}, (double[4]){1, 1, 0, 0});
  set_inertial(b, l6, 1.8, (double[3]){0, 0.0006, 0.0004}, (double[3]){0.0049, 0.0047, 0.0036},
               (double[4]){1, 1, 0, 0});
  add_joint(b, l6, OR_JNT_HINGE, zax, 1, -r2, r2, 0);
  visual(b, l6);
  visual(b, l6);
  sphere(b, l6, 0.055, 0, 0, -0.059);
  sphere(b, l6, 0.065, 0, -0.03, 0.011);
  sphere(b, l6, 0.08, 0, 0, 0);
  /* link7 (iiwa14.xml:134-140) */
  int l7 = add_body(b, l6, (double[3]){0, 0.081, 0}, (double[4]){0, 0, 1, 1});
  set_inertial(b, l7, 1.2, (double[3]){0, 0, 0.02}, (double[3]){0.001, 0.001, 0.001}, NULL);
  add_joint(b, l7, OR_JNT_HINGE, zax, 1, -r3, r3, 0);
  visual(b, l7);
  sphere(b, l7, 0.06, 0, 0, 0.001);
  /* gripper attached at attachment_site (iiwa14.xml:139; scene.py:57-61) */
  int gframe = add_body(b, l7, (double[3]){0, 0, 0.045}, id4);
  int gb = add_body(b, gframe, z3, id4);
  set_inertial(b, gb, 0.73, (double[3]){0.035, 0.0125, 0.015}, (double[3]){0.001, 0.0025, 0.0017}, NULL);
  const double gfr[3] = {2.0, 0.01, 0.01}, gsr[2] = {0.002, 1.0}, gsi[3] = {0.99, 0.9999, 0.001};
  int g = add_geom(b, gb, OR_GEOM_BOX, (double[3]){0.07, 0.025, 0.015}, (double[3]){0, 0, 0.015}, NULL, 1);
  geom_params(m, g, gfr, gsr, gsi, 1);
  m->grip_site[arm] = add_site(b, gb, (double[3]){0, 0, 0.05}, NULL);
  const double xax[3] = {1, 0, 0}, pl[3] = {0.005, 0.0075, 0.01};
  const double pd[3] = {2.375e-6, 2.375e-6, 7.5e-7};
  int plates[2];
  for (int s = 0; s < 2; s++) {
    double ppos[3] = {s == 0 ? 0.005 : -0.005, 0, 0.05};
    double pq[4] = {1, 0, 0, 0};
    if (s == 1) { pq[0] = 0; pq[3] = 1; }
    int pb = add_body(b, gb, ppos, pq);
    plates[s] = pb;
    set_inertial(b, pb, 0.015, z3, pd, NULL);
    const double gp[4][3] = {{0, -0.0075, -0.01}, {0, -0.0075, 0.01}, {0, 0.0075, -0.01}, {0, 0.0075, 0.01}};
    for (int k = 0; k < 4; k++) {
      g = add_geom(b, pb, OR_GEOM_BOX, pl, gp[k], NULL, 1);
      geom_params(m, g, gfr, gsr, gsi, 1);
    }
    add_joint(b, pb, OR_JNT_SLIDE, xax, 1, 0.0, 0.060000000000000005, 0);
  }
  m->arm_geom_hi[arm] = b->ng;
  /* contact excludes (iiwa14.xml:150-158, gripper.xml:50-54) */
  add_exclude(b, base, l1);
  add_exclude(b, base, l2);
  add_exclude(b, base, l3);
  add_exclude(b, l1, l3);
  add_exclude(b, l3, l5);
  add_exclude(b, l4, l7);
  add_exclude(b, l5, l7);
  add_exclude(b, gb, plates[0]);
  add_exclude(b, gb, plates[1]);
  add_exclude(b, plates[0], plates[1]);
  /* joint equality left = right (gripper.xml:46-49) */
  int e = b->ne++;
  int dl = m->body_dofadr[plates[0]], dr = m->body_dofadr[plates[1]];
  m->eq_dof0[e] = dl;
  m->eq_dof1[e] = dr;
  m->eq_solref[2 * e] = 0.002;
  m->eq_solref[2 * e + 1] = 1.0;
  const double esi[5] = {0.98, 0.9999, 0.001, 0.5, 2.0};
  memcpy(m->eq_solimp + 5 * e, esi, sizeof esi);
  /* actuators (iiwa14.xml:160-168, classes 10-21): general, gain 2000, bias (0,-2000,-200) */
  const double rng[7] = {r1, r2, r1, r2, r1, r2, r3};
  int d0 = m->body_dofadr[l1];
  for (int j = 0; j < 7; j++) {
    int u = b->nu++;
    m->act_dof0[u] = d0 + j;
    m->act_dof1[u] = -1;
    m->act_coef0[u] = 1.0;
    m->act_gain[u] = 2000.0;
    m->act_bias[3 * u] = 0;
    m->act_bias[3 * u + 1] = -2000.0;
    m->act_bias[3 * u + 2] = -200.0;
    m->act_ctrlrange[2 * u] = -rng[j];
    m->act_ctrlrange[2 * u + 1] = rng[j];
  }
  /* gripper actuator on tendon split = 0.5 ql + 0.5 qr (gripper.xml:55-64) */
  int u = b->nu++;
  m->act_dof0[u] = dl;
  m->act_dof1[u] = dr;
  m->act_coef0[u] = 0.5;
  m->act_coef1[u] = 0.5;
  m->act_gain[u] = 100.0;
  m->act_bias[3 * u] = 0;
  m->act_bias[3 * u + 1] = -100.0;
  m->act_bias[3 * u + 2] = -10.0;
  m->act_ctrlrange[2 * u] = 0.0;
  m->act_ctrlrange[2 * u + 1] = 0.060000000000000005;
  m->act_forcelimited[u] = 1;
  m->act_forcerange[2 * u] = -100.0;
  m->act_forcerange[2 * u + 1] = 100.0;
}

static void build_bucket(builder* b, double x, double y) {
  or_model* m = b->m;
  const double z3[3] = {0, 0, 0}, id4[4] = {1, 0, 0, 0};
  const double sr[2] = {0.002, 1.0}, si[3] = {0.98, 0.9999, 0.001};
  int frame = add_body(b, 0, z3, id4);
  int bk = add_body(b, frame, (double[3]){x, y, 1.05}, id4);
  int g = add_geom(b, bk, OR_GEOM_BOX, (double[3]){0.29, 0.29, 0.02}, (double[3]){0, 0, -0.04}, NULL, 1);
  geom_params(m, g, NULL, sr, si, 1);
  if (m->bucket_geom[0] < 0)
    m->bucket_geom[0] = g;
  else
    m->bucket_geom[1] = g;
  for (int f = 0; f < 4; f++) {
    double q[4];
    euler_z(f * 1.57, q);
    int fb = add_body(b, bk, z3, q);
    g = add_geom(b, fb, OR_GEOM_BOX, (double[3]){0.05, 0.3, 0.05}, (double[3]){0.3 - 0.05, 0, 0}, NULL, 1);
    geom_params(m, g, NULL, sr, si, 1);
  }
}

or_model* or_model_create(int A, int K, uint64_t seed) {
  if (A < 2 || A % 2 || A > 16 || K < 1 || K > 64) return NULL;
  or_model* m = zalloc(sizeof(or_model));
  alloc_model(m);
  m->A = A;
  m->K = K;
  m->timestep = 0.001;
  m->gravity[2] = -9.81;
  m->bucket_geom[0] = m->bucket_geom[1] = -1;
  builder bb = {0};
  builder* b = &bb;
  b->m = m;
  const double z3[3] = {0, 0, 0}, id4[4] = {1, 0, 0, 0};
  /* world + floor plane (scene.xml:21) */
  add_body(b, -1, z3, id4);
  add_geom(b, 0, OR_GEOM_PLANE, (double[3]){0, 0, 0.05}, NULL, NULL, 1);
  /* table (scene.py:26-38, 113-115) */
  int tb = add_body(b, 0, z3, id4);
  double L = 1.0 + 0.5 * ((A - 2) / 2.0);
  int g = add_geom(b, tb, OR_GEOM_BOX, (double[3]){1.2, L, 0.5}, (double[3]){0, 0, 0.5}, NULL, 1);
  geom_params(m, g, NULL, (double[2]){0.002, 1}, (double[3]){0.98, 0.9999, 0.001}, 1);
  /* conveyor (conveyor_belt.xml:4-12) */
  int cf = add_body(b, 0, z3, id4);
  int cb = add_body(b, cf, (double[3]){0, 0, 1.05}, id4);
  add_joint(b, cb, OR_JNT_SLIDE, (double[3]){0, 1, 0}, 0, 0, 0, 5e-4);
  g = add_geom(b, cb, OR_GEOM_BOX, (double[3]){0.3, 100.0, 0.04}, NULL, NULL, 1);
  geom_params(m, g, (double[3]){0.8, 0.01, 0.01}, (double[2]){0.004, 1.0}, (double[3]){0.95, 0.9999, 0.001}, 1);
  m->body_mass[cb] = 1000.0;
  m->body_inertia[3 * cb] = 1000.0 / 3 * (100.0 * 100.0 + 0.04 * 0.04);
  m->body_inertia[3 * cb + 1] = 1000.0 / 3 * (0.3 * 0.3 + 0.04 * 0.04);
  m->body_inertia[3 * cb + 2] = 1000.0 / 3 * (0.3 * 0.3 + 100.0 * 100.0);
  /* velocity actuator, kv = 1e4 */
  {
    int u = b->nu++;
    m->act_dof0[u] = m->body_dofadr[cb];
    m->act_dof1[u] = -1;
    m->act_coef0[u] = 1.0;
    m->act_gain[u] = 1e4;
    m->act_bias[3 * u + 2] = -1e4;
    m->act_ctrlrange[2 * u] = -1;
    m->act_ctrlrange[2 * u + 1] = 1;
  }
  /* cubes (scene.py:9-23, 121-134): draw order per cube = size, rgba[4] */
  or_pcg64 rng;
  or_pcg64_seed(&rng, seed);
  m->cube_body0 = b->nb;
  for (int k = 0; k < K; k++) {
    double h = 0.03 + (0.05 - 0.03) * or_pcg64_double(&rng);
    for (int c = 0; c < 4; c++) (void)or_pcg64_double(&rng);
    m->cube_size[k] = h;
    int body = add_body(b, 0, z3, id4);
    add_joint(b, body, OR_JNT_FREE, NULL, 0, 0, 0, 0);
    g = add_geom(b, body, OR_GEOM_BOX, (double[3]){h, h, h}, NULL, NULL, 1);
    geom_params(m, g, (double[3]){1.0, 0.01, 0.01}, NULL, NULL, 0);
    double mass = 1000.0 * pow(h, 3.0); /* PickableObject: mass = 1000 * size**3 (scene.py:13) */
    m->body_mass[body] = mass;
    double I = mass / 3.0 * (h * h + h * h);
    m->body_inertia[3 * body] = m->body_inertia[3 * body + 1] = m->body_inertia[3 * body + 2] = I;
  }
  /* buckets (scene.py:136-145) */
  double by = 0.7 - (A / 2 - 1);
  build_bucket(b, 0.9, by);
  build_bucket(b, -0.9, by);
  /* arms (scene.py:147-161) */
  for (int i = 0; i < A; i++) {
    double x = 0.7 * ((i % 2) ? -1.0 : 1.0);
    double y = 1.4 * (i / 2) - (A / 2 - 1);
    if (i == 4 || i == 5) {
      y = 0.5 * 1.4 * ((i - 2) / 2);
      x *= 0.9;
    }
    double pos[3] = {x, y, 1.0};
    build_arm(b, i, pos, (i % 2) ? M_PI : 0.0);
  }
  m->nbody = b->nb;
  m->njnt = b->nj;
  m->ngeom = b->ng;
  m->nsite = b->ns;
  m->nu = b->nu;
  m->neq = b->ne;
  m->nexclude = b->nx;
  m->nq = b->nq;
  m->nv = b->nv;
  /* weld ids: a body without joints is welded to its parent (world = 0) */
  for (int i = 0; i < m->nbody; i++) {
    if (i == 0)
      m->body_weldid[i] = 0;
    else if (m->body_jntnum[i] > 0)
      m->body_weldid[i] = i;
    else
      m->body_weldid[i] = m->body_weldid[m->body_parent[i]];
  }
  or_collision_pairs(m);
  or_model_setconst(m);
  return m;
}
