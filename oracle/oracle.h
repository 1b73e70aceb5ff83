/* oracle.h -- CPU restatement of the reference env-step path.  TEST INFRASTRUCTURE ONLY.
 *
 * This library is the parity CHECKER for the HIP product in factory_marl_amd/.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  It is never linked into,
 * or called by, the product path.
 *
 * What it restates (fp64 throughout, like the reference's MuJoCo mjtNum):
 *   - the scene of challenge_env/challenge_env/scene.py:109-169 + assets/ XML (model.c)
 *   - one dm_control legacy physics.step() = mj_step2 + mj_step1 (MuJoCo 3.1.x defaults:
 *     implicitfast, Newton solver, pyramidal cones; step.c, kin.c, collide.c, solver.c)
 *   - BaseEnv.step_sim / reset_sim, TaskManager, and the src/environments.py wrappers
 *     (task.c, pcg64.c)
 *
 * Parity status: the task layer is pinned by golden vectors produced by running the
 * reference's own Python (tests/golden/gen_golden.py).  The physics is "parity unpinned": MuJoCo is
 * not available in this image or on the GPU box, so the MuJoCo algorithms are restated from their
 * published definitions and pinned only by analytic known-answer tests (tests/test_oracle_physics.py).
 */
#ifndef FM_ORACLE_H
#define FM_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_JNT_FREE = 0, OR_JNT_SLIDE = 2, OR_JNT_HINGE = 3 };
enum { OR_GEOM_PLANE = 0, OR_GEOM_SPHERE = 2, OR_GEOM_BOX = 6 };
enum { OR_CNSTR_EQUALITY = 0, OR_CNSTR_LIMIT = 3, OR_CNSTR_PYRAMIDAL = 6 };

typedef struct or_model {
  int A, K;
  int nbody, njnt, nq, nv, ngeom, nsite, nu, nexclude;
  /* bodies (MuJoCo preorder numbering) */
  int *body_parent, *body_jntadr, *body_jntnum, *body_dofadr, *body_dofnum, *body_weldid;
  double *body_pos, *body_quat, *body_ipos, *body_iquat, *body_mass, *body_inertia;
  double *body_invweight0; /* 2 per body */
  /* joints */
  int *jnt_type, *jnt_body, *jnt_qposadr, *jnt_dofadr, *jnt_limited;
  double *jnt_axis, *jnt_range, *jnt_solref, *jnt_solimp;
  /* dofs */
  int *dof_body, *dof_jnt;
  double *dof_damping, *dof_invweight0;
  /* geoms */
  int *geom_type, *geom_body, *geom_contype, *geom_conaffinity, *geom_condim, *geom_priority;
  double *geom_size, *geom_pos, *geom_quat, *geom_friction, *geom_solref, *geom_solimp, *geom_solmix,
      *geom_margin, *geom_rbound;
  /* sites */
  int *site_body;
  double *site_pos, *site_quat;
  /* actuators: trn = joint dof (single) or fixed tendon (two dofs with coefficients) */
  int *act_dof0, *act_dof1, *act_forcelimited;
  double *act_coef0, *act_coef1, *act_gain, *act_bias, *act_ctrlrange, *act_forcerange;
  /* joint equality (one per gripper) */
  int neq;
  int *eq_dof0, *eq_dof1;
  double *eq_solref, *eq_solimp;
  /* contact excludes (body pairs, b0 < b1) */
  int *exclude;
  /* misc */
  double timestep, gravity[3], meaninertia;
  double *qpos0;
  /* task-level ids */
  int *arm_geom_lo, *arm_geom_hi; /* [A]: geom id range [lo, hi) of the 70 arm+gripper geoms */
  int *grip_site;                  /* [A]: site id of "between_gripper_plates" */
  int *base_site;                  /* [A]: site id of "player_site" */
  int bucket_geom[2];              /* target_area geoms */
  int cube_body0;                  /* body id of cube 0 */
  double *cube_size;               /* [K] half sizes */
  /* geom pairs passing mj_collision's static filter (contype/conaffinity, weld/parent, excludes), type-ordered,
   * g1 | g2 << 16, in its loop order: built once by or_collision_pairs so a substep only tests bounds */
  int ncpair;
  int *cpair;
  /* runs of cpair sharing the loop's first geom and the second geom's body: [run_lo[r], run_lo[r + 1]) against
   * geom run_geom[r] and body run_body[r], run_margin[r] the largest pair margin of the run */
  int nrun;
  int *run_lo, *run_geom, *run_body;
  double *run_margin;
} or_model;

typedef struct or_contact {
  double dist, pos[3], frame[9], mu, solref[2], solimp[5], margin;
  int geom[2], dim, efc_adr;
} or_contact;

typedef struct or_data {
  /* state */
  double *qpos, *qvel, *ctrl, *qacc_warmstart, *qacc;
  /* position/velocity stage (mj_step1 products) */
  double *xpos, *xquat, *xmat, *xipos, *ximat, *geom_xpos, *geom_xmat, *site_xpos, *site_xmat;
  double *cvel_ang, *cvel_lin;  /* body angular velocity (world) and com linear velocity */
  double *M, *qfrc_bias, *qfrc_passive, *act_length, *act_velocity;
  int ncon, maxcon;
  or_contact *con;
  int nefc, maxefc;
  int *efc_type, *efc_id;
  double *efc_J, *efc_pos, *efc_margin, *efc_vel, *efc_aref, *efc_R, *efc_D, *efc_diag, *efc_force;
  double *efc_K, *efc_B, *efc_imp;
  /* acceleration stage */
  double *qfrc_actuator, *act_force, *qfrc_smooth, *qacc_smooth, *qfrc_constraint;
  int solver_niter;
  int actuation_disabled;
  double *scratch; /* nv*nv*4 + ... */
} or_data;

/* ---------------- model / data ---------------- */
or_model* or_model_create(int A, int K, uint64_t seed);
void or_model_free(or_model* m);
or_data* or_data_create(const or_model* m);
void or_data_free(or_data* d);
void or_reset_data(const or_model* m, or_data* d); /* mj_resetData */

/* ---------------- physics stages ---------------- */
void or_kinematics(const or_model* m, or_data* d);
void or_mass(const or_model* m, or_data* d);
void or_bias(const or_model* m, or_data* d);
void or_collision(const or_model* m, or_data* d);
void or_collision_pairs(or_model* m);
void or_make_constraint(const or_model* m, or_data* d);
void or_step1(const or_model* m, or_data* d);
void or_step2(const or_model* m, or_data* d);
void or_set_accel_noise(double amp, uint64_t seed); /* sensitivity probe only (tools/fp32_floor.py) */
void or_set_probe(int mask, double amp, uint64_t seed); /* data-precision probe only (tools/fp32_floor.py) */
void or_set_solver_tol(double tol);                /* Newton tolerance study only (tools/tolerance_floor.py) */
void or_forward(const or_model* m, or_data* d); /* step1 + acceleration stage, no integration */
void or_jac_point(const or_model* m, const or_data* d, int body, const double p[3], double* jacp, double* jacr);
void or_contact_force(const or_model* m, const or_data* d, int i, double out[6]);
int or_collide_geoms(const or_model* m, const or_data* d, int g1, int g2, or_contact* out, int maxout);
double or_impedance(const double solimp[5], double x);

/* narrowphase primitives exposed for known-answer tests (frame: normal from geom1 to geom2) */
int or_box_box(const double* p1, const double* R1, const double* h1, const double* p2, const double* R2,
               const double* h2, double margin, or_contact* out);
int or_sphere_box(const double* c, double r, const double* p, const double* R, const double* h, double margin,
                  or_contact* out);
int or_plane_box(const double* pp, const double* pR, const double* p, const double* R, const double* h,
                 double margin, or_contact* out);

/* ---------------- task layer (BaseEnv + TaskManager + wrappers) ---------------- */
typedef struct or_pcg64 {
  uint64_t state_hi, state_lo, inc_hi, inc_lo;
} or_pcg64;
void or_pcg64_seed(or_pcg64* r, uint64_t seed);
uint64_t or_pcg64_next64(or_pcg64* r);
double or_pcg64_double(or_pcg64* r);

typedef struct or_task {
  int A, K;
  /* TaskManager */
  int in_scene[64], n_in, out_scene[64], n_out;
  int step_counter, steps_since_spawn, failure_counter, hidden_counter;
  int scores[2];
  double spawn_freq, init_spawn_freq;
  or_pcg64 rng;
  /* BaseEnv */
  double conveyor_speed, play_time;
  double ctrl_target[128];
  int force_terminate, out_of_reach;
  /* ProgressRewardEnv */
  double last_grip_dist[16], last_bucket_dist[16];
  int last_score[2];
  double w_grip, w_bucket, w_action, base_reward;
  int reward_kind; /* 0: score delta (FactoryManipulationEnv), 1: progress (ProgressRewardEnv) */
  int ik_ignore[16][16]; /* IKPolicy.ignore_objects of arm i: owner arm -> cube index, -1 = none (reward candidates) */
  int act_dim;           /* action_space.shape[0] of the env class (progress-reward action norm) */
  /* config (BaseEnv.__init__ kwargs, base_env.py:15-35) */
  double initial_conveyor_speed, conveyor_acceleration, pt_time, force_contact_threshold, spawn_freq_increase;
  int frame_skip;
} or_task;

/* ---------------- IK base policy (ik.c; ik_policy.py) ---------------- */
#define OR_IK_MAXA 16
enum { OR_IK_IDLE = 0, OR_IK_GO_TO_GRASP, OR_IK_GRASP_APPROACH, OR_IK_GRASP_CLOSE, OR_IK_POST_GRASP,
       OR_IK_GO_TO_RELEASE, OR_IK_RELEASE };
typedef struct or_ik_arm {
  int state, counter, target; /* PolicyState, state_counter, target_object (cube index, -1 = None) */
  int ignore[OR_IK_MAXA];     /* ignore_objects: owner arm -> cube index, -1 = None / never set */
  double last_ctrl[8], move_start[3];
} or_ik_arm;
/* what IKPolicy.act reads from the physics (all world frame, float64) */
typedef struct or_ik_in {
  int A, n_in;
  const int* in_scene;      /* TaskManager._in_scene order */
  const double* cube_qpos;  /* [K][7] */
  const double* cube_qvel;  /* [K][6] */
  const double* grip;       /* site_xpos of between_gripper_plates */
  const double* base;       /* site_xpos of player_site */
  const double* bucket;     /* xpos of this arm's bucket (buckets[i % 2]) */
  const double* arm_q;      /* the 7 hinge qpos */
  double pt_time, dt;       /* env.pt_time, env.dt = timestep * frame_skip (ik_policy.py:56-67) */
} or_ik_in;
extern const double OR_IK_DEFAULT_POSE[8];
void or_ik_arm_init(or_ik_arm* p);
void or_ik_arm_reset(or_ik_arm* p);
void or_ik_grasp_quat(const double obj_quat_wxyz[4], double out_wxyz[4]);
int or_ik_plan(const or_ik_in* in, or_ik_arm* p, double tpos[3], double tquat[4], int* close_gripper);
void or_ik_finish(or_ik_arm* p, int success, const double q7[7], int close_gripper, double ctrl[8]);
int or_ik_solve(const or_model* m, or_data* scratch, const double* qpos, int arm, const double tpos[3],
                const double tquat[4], double q7[7], int* steps_out);
typedef int (*or_ik_solver)(void* ctx, int arm, const double* tpos, const double* tquat, double* q7);
void or_ik_compose(const or_model* m, or_ik_arm* ik, const double* qpos, const double* qvel, const double* grip /*3A*/,
                   const double* base /*3A*/, const int* in_scene, int n_in, or_ik_solver solve, void* ctx,
                   double pt_time, double dt, double* arm_ctrl /* 8A */);
void or_compose_class(const or_model* m, int env_class, const float* action, const double* ik, const int* ik_state,
                      const double* ik_actions, double* pause_last, double* arm_ctrl);

/* env classes (environments.py), same numbering as the product's FM_ENV_* (include/factorysim.h) */
enum { OR_ENV_FACTORY = 0, OR_ENV_ALLFULLRL = 1, OR_ENV_SINGLEFULLRL = 2, OR_ENV_SINGLEDELTA = 3,
       OR_ENV_ALLDELTA = 4, OR_ENV_PAUSE_TOGGLE = 5, OR_ENV_BACKUP_TOGGLE = 6 };

typedef struct or_env {
  or_model* m;
  or_data* d;
  or_task t;
  int obs_dim, act_dim, env_class;
  or_ik_arm ik[OR_IK_MAXA];
  double ik_actions[OR_IK_MAXA][8]; /* IKTogglingEnv.ik_actions (proposals of the last observation) */
  double pause_last[OR_IK_MAXA][8]; /* PauseIKToggleEnv.last_arm_actions */
  or_data* ik_d;                    /* scratch physics copy of qpos_from_site_pose (inplace=False) */
  int ik_steps;                     /* diagnostics: IK iterations summed over the last compose */
  long ik_calls[OR_IK_MAXA];        /* diagnostics (tools/base_policy_study.py): IK solves per arm since creation, */
  long ik_fails[OR_IK_MAXA];        /* and the ones that did not converge (act() returns last_ctrl) */
  double* stage_qpos; /* state at which the current position/velocity stage was computed (last mj_step1) */
  double* stage_qvel;
  double ep_return;
  int ep_len;
} or_env;
void or_env_set_timing(or_env* e, double pt_time, double control_frequency);

or_env* or_env_create(int A, int K, uint64_t seed, int env_class, const double* reward_w /*4*/);
void or_env_free(or_env* e);
void or_env_reset(or_env* e, float* obs);
/* one FactoryManipulationEnv.step(): returns terminated; info_out = [score0, score1, play_time,
 * conveyor_speed, out_of_reach, force_terminate, num_obj] */
int or_env_step(or_env* e, const float* action, float* obs, double* reward, double* info_out);

/* task-layer pieces, driveable from recorded (fake-physics) state for the golden-vector tests */
void or_task_init(or_task* t, int A, int K, uint64_t seed);
void or_task_reset(or_task* t, const or_model* m, double* qpos, double* qvel);
void or_task_process_action(const or_model* m, const float* action, double* arm_ctrl /*8A*/);
void or_task_lowpass(or_task* t, const or_model* m, const double* ctrl_in /*nu, clipped*/, int substep,
                     double* ctrl_out);
void or_task_clip_ctrl(const or_task* t, const or_model* m, const double* arm_ctrl, double* ctrl);
int or_task_force_check(const or_task* t, const or_model* m, int ncon, const int* con_geom,
                        const double* con_force);
void or_task_step(or_task* t, const or_model* m, double* qpos, double* qvel);
void or_task_after_step(or_task* t);
void or_task_obs(const or_task* t, const or_model* m, const double* qpos, const double* qvel, float* obs);
double or_task_reward(or_task* t, const or_model* m, const double* qpos, const double* grip_site /*3A*/,
                      const float* action);

#ifdef __cplusplus
}
#endif
#endif
