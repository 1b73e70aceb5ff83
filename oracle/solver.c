/* solver.c -- constraint assembly and Newton solver (TEST INFRASTRUCTURE; see oracle.h).
 *
 * Restates MuJoCo 3.1 engine_core_constraint.c / engine_solver.c for this scene:
 *   rows: joint equality (gripper.xml:46-49), joint limits (autolimits ranges), pyramidal contacts
 *   (condim 3 -> 4 edge rows J_n +- mu J_t); pos = violation, margin 0.
 *   solref -> K = 1/(dmax^2 tc^2 dr^2), B = 2/(dmax tc) with tc >= 2 dt (refsafe);
 *   solimp -> impedance d(|pos - margin|) (getimpedance);  R = max(MINVAL, (1-d)/d * diagApprox);
 *   diagApprox from body/dof invweight0 (mj_diagApprox; pyramid edges: tran*(1 + mu^2));
 *   pyramid edges: the position term of aref uses K / (4 mu^2) -- PINNED by MuJoCo's own outputs in the reference
 *   (runs/[run].zip _last_obs, tests/test_physics_pins.py): cubes resting on the belt (mu 0.8, solref 0.004,
 *   solimp 0.95) sit 2.29e-6 m deep and on the table (mu 1, solref 0.002, solimp 0.98) 4.19e-7 m deep, where
 *   K imp pos alone gives 2.56x / 4.1x shallower equilibria, while the belt-carried cube velocities (set by the
 *   edges' R, B and J) already match MuJoCo to 1 float32 ulp.  The 1 / (4 mu^2) position stiffness reproduces all
 *   three to float32 resolution; scaling R by 4 mu^2 instead fits the depths but moves the carried velocities by
 *   3-4 ulps.  MuJoCo's source is not available to state the general form (OR_PYR_KSCALE);
 *   aref = -B*efc_vel - K*d*(pos - margin).
 * Solver: minimises the MuJoCo primal cost
 *   f(a) = 1/2 (a - a0)^T M (a - a0) + sum_i 1/2 D_i (J_i a - aref_i)^2 [eq, or ineq with J_i a < aref_i]
 * by Newton's method (H = M + J^T D_active J, dense Cholesky) with an EXACT piecewise-quadratic line
 * search (breakpoints sorted), warm-started from qacc_warmstart when that is cheaper than a0.  The
 * optimum is unique (strictly convex), so the result does not depend on solver path; tolerance is set
 * tighter than MuJoCo's 1e-8 so this checker sits at the optimum MuJoCo's Newton approximates.
 */
#include <stdlib.h>

#include "oracle.h"
#include "oracle_internal.h"

#ifndef OR_SOLVER_TOL
#define OR_SOLVER_TOL 1e-12 /* liboracle_f32.so (fp32 floor study) overrides it */
#endif
#define OR_SOLVER_ITER 100
/* the tolerance in use: OR_SOLVER_TOL unless a study sets another (or_set_solver_tol, tools/tolerance_floor.py) */
static double or_solver_tol = OR_SOLVER_TOL;
void or_set_solver_tol(double tol) { or_solver_tol = tol > 0 ? tol : OR_SOLVER_TOL; }
#ifndef OR_PYR_KSCALE
#define OR_PYR_KSCALE(mu) (4.0 * (mu) * (mu)) /* pyramid edges: aref position stiffness K / this (header comment) */
#endif

double or_impedance(const double si[5], double x) {
  double dmin = si[0], dmax = si[1], width = si[2], mid = si[3], power = si[4];
  dmin = dmin < OR_MINIMP ? OR_MINIMP : (dmin > OR_MAXIMP ? OR_MAXIMP : dmin);
  dmax = dmax < OR_MINIMP ? OR_MINIMP : (dmax > OR_MAXIMP ? OR_MAXIMP : dmax);
  if (dmin == dmax || width <= OR_MINVAL) return 0.5 * (dmin + dmax);
  x = fabs(x) / width;
  if (x >= 1) return dmax;
  if (x <= 0) return dmin;
  double y;
  if (power == 1)
    y = x;
  else if (x <= mid)
    y = pow(x, power) / pow(mid, power - 1);
  else
    y = 1 - pow(1 - x, power) / pow(1 - mid, power - 1);
  return dmin + y * (dmax - dmin);
}

static void kbip(const or_model* m, const double solref[2], const double solimp[5], double* K, double* B) {
  double tc = solref[0], dr = solref[1];
  double dmax = solimp[1];
  dmax = dmax < OR_MINIMP ? OR_MINIMP : (dmax > OR_MAXIMP ? OR_MAXIMP : dmax);
  if (tc > 0) {
    if (tc < 2 * m->timestep) tc = 2 * m->timestep;
    double k = dmax * dmax * tc * tc * dr * dr;
    double b = dmax * tc;
    *K = 1.0 / (k > OR_MINVAL ? k : OR_MINVAL);
    *B = 2.0 / (b > OR_MINVAL ? b : OR_MINVAL);
  } else {
    *K = -tc / (dmax * dmax);
    *B = -dr / dmax;
  }
}

static int add_row(const or_model* m, or_data* d, int type, int id, double pos, double margin, double diag,
                   const double solref[2], const double solimp[5], double kscale) {
  int r = d->nefc++;
  d->efc_type[r] = type;
  d->efc_id[r] = id;
  d->efc_pos[r] = pos;
  d->efc_margin[r] = margin;
  d->efc_diag[r] = diag;
  double imp = or_impedance(solimp, pos - margin);
  double K, B;
  kbip(m, solref, solimp, &K, &B);
  d->efc_imp[r] = imp;
  d->efc_K[r] = K / kscale;
  d->efc_B[r] = B;
  double R = (1 - imp) * diag / imp;
  d->efc_R[r] = R > OR_MINVAL ? R : OR_MINVAL;
  d->efc_D[r] = 1.0 / d->efc_R[r];
  return r;
}

/* mj_makeConstraint (+ mj_diagApprox, mj_makeImpedance) at the current position stage */
void or_make_constraint(const or_model* m, or_data* d) {
  int nv = m->nv;
  d->nefc = 0;
  /* equality */
  for (int e = 0; e < m->neq; e++) {
    int d0 = m->eq_dof0[e], d1 = m->eq_dof1[e];
    int j0 = m->dof_jnt[d0], j1 = m->dof_jnt[d1];
    double pos = (d->qpos[m->jnt_qposadr[j0]] - m->qpos0[m->jnt_qposadr[j0]]) -
                 (d->qpos[m->jnt_qposadr[j1]] - m->qpos0[m->jnt_qposadr[j1]]);
    double diag = m->dof_invweight0[d0] + m->dof_invweight0[d1];
    int r = add_row(m, d, OR_CNSTR_EQUALITY, e, pos, 0.0, diag, m->eq_solref + 2 * e, m->eq_solimp + 5 * e, 1.0);
    double* J = d->efc_J + (size_t)r * nv;
    memset(J, 0, nv * sizeof(double));
    J[d0] = 1.0;
    J[d1] = -1.0;
  }
  /* joint limits */
  for (int j = 0; j < m->njnt; j++) {
    if (!m->jnt_limited[j] || m->jnt_type[j] == OR_JNT_FREE) continue;
    double q = d->qpos[m->jnt_qposadr[j]];
    int da = m->jnt_dofadr[j];
    for (int side = 0; side < 2; side++) {
      double dist = side == 0 ? q - m->jnt_range[2 * j] : m->jnt_range[2 * j + 1] - q;
      if (dist < 0.0) {
        int r = add_row(m, d, OR_CNSTR_LIMIT, j, dist, 0.0, m->dof_invweight0[da], m->jnt_solref + 2 * j,
                        m->jnt_solimp + 5 * j, 1.0);
        double* J = d->efc_J + (size_t)r * nv;
        memset(J, 0, nv * sizeof(double));
        J[da] = side == 0 ? 1.0 : -1.0;
      }
    }
  }
  /* contacts, pyramidal */
  double* jp1 = d->scratch;
  double* jp2 = jp1 + 3 * nv;
  for (int c = 0; c < d->ncon; c++) {
    or_contact* con = d->con + c;
    int b1 = m->geom_body[con->geom[0]], b2 = m->geom_body[con->geom[1]];
    or_body_jac(m, d, b1, con->pos, jp1, NULL);
    or_body_jac(m, d, b2, con->pos, jp2, NULL);
    double tran = m->body_invweight0[2 * b1] + m->body_invweight0[2 * b2];
    double mu = con->mu;
    double diag = tran + mu * mu * tran;
    con->efc_adr = d->nefc;
    double Jf[3][256];
    for (int k = 0; k < 3; k++) {
      const double* f = con->frame + 3 * k;
      for (int i = 0; i < nv; i++)
        Jf[k][i] = f[0] * (jp2[i] - jp1[i]) + f[1] * (jp2[nv + i] - jp1[nv + i]) + f[2] * (jp2[2 * nv + i] - jp1[2 * nv + i]);
    }
    for (int e = 0; e < 4; e++) {
      int r = add_row(m, d, OR_CNSTR_PYRAMIDAL, c, con->dist, con->margin, diag, con->solref, con->solimp,
                      OR_PYR_KSCALE(mu));
      double* J = d->efc_J + (size_t)r * nv;
      int t = 1 + e / 2;
      double sg = (e & 1) ? -mu : mu;
      for (int i = 0; i < nv; i++) J[i] = Jf[0][i] + sg * Jf[t][i];
    }
  }
}

/* mj_referenceConstraint: efc_vel = J qvel, aref */
void or_reference(const or_model* m, or_data* d) {
  int nv = m->nv;
  for (int r = 0; r < d->nefc; r++) {
    const double* J = d->efc_J + (size_t)r * nv;
    double v = 0;
    for (int i = 0; i < nv; i++) v += J[i] * d->qvel[i];
    d->efc_vel[r] = v;
    d->efc_aref[r] = -d->efc_B[r] * v - d->efc_K[r] * d->efc_imp[r] * (d->efc_pos[r] - d->efc_margin[r]);
  }
}

typedef struct lsrow {
  double t;
  int r;
} lsrow;

static int cmp_lsrow(const void* a, const void* b) {
  double x = ((const lsrow*)a)->t, y = ((const lsrow*)b)->t;
  return x < y ? -1 : (x > y ? 1 : 0);
}

static double cost_at(const or_model* m, const or_data* d, const double* a, double* jar, double* Ma) {
  int nv = m->nv;
  double c = 0;
  for (int i = 0; i < nv; i++) {
    double s = 0;
    for (int k = 0; k < nv; k++) s += d->M[i * nv + k] * (a[k] - d->qacc_smooth[k]);
    Ma[i] = s;
    c += 0.5 * (a[i] - d->qacc_smooth[i]) * s;
  }
  for (int r = 0; r < d->nefc; r++) {
    const double* J = d->efc_J + (size_t)r * nv;
    double v = -d->efc_aref[r];
    for (int i = 0; i < nv; i++) v += J[i] * a[i];
    jar[r] = v;
    if (d->efc_type[r] == OR_CNSTR_EQUALITY || v < 0) c += 0.5 * d->efc_D[r] * v * v;
  }
  return c;
}

/* Newton solver on the primal cost (mj_solNewton) */
void or_solve(const or_model* m, or_data* d) {
  int nv = m->nv, ne = d->nefc;
  double* a = d->qacc;
  double* jar = d->scratch;
  double* Ma = jar + ne;
  double* g = Ma + nv;
  double* dir = g + nv;
  double* Jd = dir + nv;
  double* H = Jd + ne;
  lsrow* bp = (lsrow*)(H + nv * nv);
  double scale = 1.0 / (m->meaninertia * (nv > 1 ? nv : 1));
  /* warmstart: keep the cheaper of qacc_warmstart and qacc_smooth */
  double c_ws = cost_at(m, d, d->qacc_warmstart, jar, Ma);
  double c_sm = cost_at(m, d, d->qacc_smooth, jar, Ma);
  memcpy(a, c_ws < c_sm ? d->qacc_warmstart : d->qacc_smooth, nv * sizeof(double));
  double cost = cost_at(m, d, a, jar, Ma);
  int it;
  int nz[nv]; /* nonzero columns of a constraint row; then the Hessian's envelope */
  for (it = 0; it < OR_SOLVER_ITER; it++) {
    /* gradient and Hessian at a */
    memcpy(g, Ma, nv * sizeof(double));
    memcpy(H, d->M, nv * nv * sizeof(double));
    for (int r = 0; r < ne; r++) {
      if (!(d->efc_type[r] == OR_CNSTR_EQUALITY || jar[r] < 0)) continue;
      const double* J = d->efc_J + (size_t)r * nv;
      double Dr = d->efc_D[r];
      int nnz = 0; /* the row's nonzero columns: the products with J[k] == 0 add exact zeros */
      for (int i = 0; i < nv; i++)
        if (J[i] != 0) nz[nnz++] = i;
      for (int a_ = 0; a_ < nnz; a_++) {
        const int i = nz[a_];
        g[i] += Dr * jar[r] * J[i];
        for (int b_ = 0; b_ < nnz; b_++) H[i * nv + nz[b_]] += Dr * J[i] * J[nz[b_]];
      }
    }
    double gn = 0;
    for (int i = 0; i < nv; i++) gn += g[i] * g[i];
    if (scale * sqrt(gn) < or_solver_tol) break;
    or_cholesky_env(H, nv, nz);
    for (int i = 0; i < nv; i++) dir[i] = -g[i];
    or_chol_solve_env(H, nv, nz, dir);
    /* exact line search along dir: f'(t) = c0 + c1 t on each active-set segment */
    double dMd = 0, dMa = 0;
    for (int i = 0; i < nv; i++) {
      double s = 0;
      for (int k = 0; k < nv; k++) s += d->M[i * nv + k] * dir[k];
      dMd += dir[i] * s;
      dMa += dir[i] * Ma[i];
    }
    double c0 = dMa, c1 = dMd;
    int nbp = 0;
    for (int r = 0; r < ne; r++) {
      const double* J = d->efc_J + (size_t)r * nv;
      double v = 0;
      for (int i = 0; i < nv; i++) v += J[i] * dir[i];
      Jd[r] = v;
      int eq = d->efc_type[r] == OR_CNSTR_EQUALITY;
      int act = eq || jar[r] < 0 || (jar[r] == 0 && v < 0);
      if (act) {
        c0 += d->efc_D[r] * jar[r] * v;
        c1 += d->efc_D[r] * v * v;
      }
      if (!eq && v != 0) {
        double t = -jar[r] / v;
        if (t > 0) {
          bp[nbp].t = t;
          bp[nbp].r = r;
          nbp++;
        }
      }
    }
    qsort(bp, nbp, sizeof(lsrow), cmp_lsrow);
    double alpha = 0;
    if (c0 < 0) {
      int k = 0;
      double tprev = 0;
      for (;;) {
        double tnext = k < nbp ? bp[k].t : 1e300;
        double fnext = c0 + c1 * tnext;
        if (k >= nbp || fnext >= 0) {
          alpha = c1 > 0 ? -c0 / c1 : tnext;
          if (alpha < tprev) alpha = tprev;
          break;
        }
        /* cross breakpoint: toggle row */
        int r = bp[k].r;
        double v = Jd[r];
        /* contribution of row r on the segment before/after tnext */
        double contrib0 = d->efc_D[r] * jar[r] * v, contrib1 = d->efc_D[r] * v * v;
        if (v < 0) { /* becomes active (jar goes negative) */
          c0 += contrib0;
          c1 += contrib1;
        } else { /* becomes inactive */
          c0 -= contrib0;
          c1 -= contrib1;
        }
        tprev = tnext;
        k++;
      }
    }
    for (int i = 0; i < nv; i++) a[i] += alpha * dir[i];
    double newcost = cost_at(m, d, a, jar, Ma);
    double improvement = scale * (cost - newcost);
    cost = newcost;
    if (improvement < or_solver_tol) {
      it++;
      break;
    }
  }
  d->solver_niter = it;
  /* forces */
  memset(d->qfrc_constraint, 0, nv * sizeof(double));
  for (int r = 0; r < ne; r++) {
    int act = d->efc_type[r] == OR_CNSTR_EQUALITY || jar[r] < 0;
    d->efc_force[r] = act ? -d->efc_D[r] * jar[r] : 0.0;
    const double* J = d->efc_J + (size_t)r * nv;
    for (int i = 0; i < nv; i++) d->qfrc_constraint[i] += J[i] * d->efc_force[r];
  }
  memcpy(d->qacc_warmstart, a, nv * sizeof(double));
}

/* mj_contactForce for a pyramidal contact: decode edge forces into (normal, t1, t2, 0, 0, 0) */
void or_contact_force(const or_model* m, const or_data* d, int i, double out[6]) {
  (void)m;
  memset(out, 0, 6 * sizeof(double));
  const or_contact* c = d->con + i;
  if (c->efc_adr < 0) return;
  const double* f = d->efc_force + c->efc_adr;
  out[0] = f[0] + f[1] + f[2] + f[3];
  out[1] = (f[0] - f[1]) * c->mu;
  out[2] = (f[2] - f[3]) * c->mu;
}
