/* kin.c -- kinematics, Jacobians, joint-space inertia and bias forces (TEST INFRASTRUCTURE).
 *
 * Restates MuJoCo 3.1 mj_kinematics / mj_jac / mj_crb / mj_rne at definition level (dense, fp64):
 *   M         = sum_b  m_b Jc_b^T Jc_b + Jr_b^T I_b Jr_b
 *   qfrc_bias = sum_b  Jc_b^T m_b (a_c,b - g) + Jr_b^T (I_b alpha_b + w_b x I_b w_b)   (qacc = 0)
 * where a_c,b / alpha_b are the velocity-product accelerations.  Every joint of this scene has its
 * anchor at its body origin (jnt pos = 0: iiwa14.xml, gripper.xml, conveyor_belt.xml), which the
 * recursion below relies on.  Free-joint dofs: 3 world-frame translations then 3 body-frame
 * rotations (MuJoCo convention).  The product (HIP) uses an independent recursive formulation.
 */
#include <stdlib.h>

#include "oracle.h"
#include "oracle_internal.h"

static void* zalloc(size_t n) { return calloc(n ? n : 1, 1); }

or_data* or_data_create(const or_model* m) {
  or_data* d = zalloc(sizeof(or_data));
  int nv = m->nv, nb = m->nbody, ng = m->ngeom, ns = m->nsite;
  d->qpos = zalloc(m->nq * sizeof(double));
  d->qvel = zalloc(nv * sizeof(double));
  d->ctrl = zalloc(m->nu * sizeof(double));
  d->qacc_warmstart = zalloc(nv * sizeof(double));
  d->qacc = zalloc(nv * sizeof(double));
  d->xpos = zalloc(3 * nb * sizeof(double));
  d->xquat = zalloc(4 * nb * sizeof(double));
  d->xmat = zalloc(9 * nb * sizeof(double));
  d->xipos = zalloc(3 * nb * sizeof(double));
  d->ximat = zalloc(9 * nb * sizeof(double));
  d->cvel_ang = zalloc(3 * nb * sizeof(double));
  d->cvel_lin = zalloc(3 * nb * sizeof(double));
  d->geom_xpos = zalloc(3 * ng * sizeof(double));
  d->geom_xmat = zalloc(9 * ng * sizeof(double));
  d->site_xpos = zalloc(3 * ns * sizeof(double));
  d->site_xmat = zalloc(9 * ns * sizeof(double));
  d->M = zalloc(nv * nv * sizeof(double));
  d->qfrc_bias = zalloc(nv * sizeof(double));
  d->qfrc_passive = zalloc(nv * sizeof(double));
  d->act_length = zalloc(m->nu * sizeof(double));
  d->act_velocity = zalloc(m->nu * sizeof(double));
  d->maxcon = 4096;
  d->con = zalloc(d->maxcon * sizeof(or_contact));
  d->maxefc = 4 * d->maxcon + 4 * nv + 64;
  int me = d->maxefc;
  d->efc_type = zalloc(me * sizeof(int));
  d->efc_id = zalloc(me * sizeof(int));
  d->efc_J = zalloc((size_t)me * nv * sizeof(double));
  d->efc_pos = zalloc(me * sizeof(double));
  d->efc_margin = zalloc(me * sizeof(double));
  d->efc_vel = zalloc(me * sizeof(double));
  d->efc_aref = zalloc(me * sizeof(double));
  d->efc_R = zalloc(me * sizeof(double));
  d->efc_D = zalloc(me * sizeof(double));
  d->efc_diag = zalloc(me * sizeof(double));
  d->efc_force = zalloc(me * sizeof(double));
  d->efc_K = zalloc(me * sizeof(double));
  d->efc_B = zalloc(me * sizeof(double));
  d->efc_imp = zalloc(me * sizeof(double));
  d->qfrc_actuator = zalloc(nv * sizeof(double));
  d->act_force = zalloc(m->nu * sizeof(double));
  d->qfrc_smooth = zalloc(nv * sizeof(double));
  d->qacc_smooth = zalloc(nv * sizeof(double));
  d->qfrc_constraint = zalloc(nv * sizeof(double));
  d->scratch = zalloc((size_t)(8 * nv * nv + 64 * nv + 4 * me) * sizeof(double));
  or_reset_data(m, d);
  return d;
}

void or_data_free(or_data* d) {
  if (!d) return;
  void* p[] = {d->qpos, d->qvel, d->ctrl, d->qacc_warmstart, d->qacc, d->xpos, d->xquat, d->xmat, d->xipos,
               d->ximat, d->cvel_ang, d->cvel_lin, d->geom_xpos, d->geom_xmat, d->site_xpos, d->site_xmat, d->M,
               d->qfrc_bias, d->qfrc_passive, d->act_length, d->act_velocity, d->con, d->efc_type, d->efc_id,
               d->efc_J, d->efc_pos, d->efc_margin, d->efc_vel, d->efc_aref, d->efc_R, d->efc_D, d->efc_diag,
               d->efc_force, d->efc_K, d->efc_B, d->efc_imp, d->qfrc_actuator, d->act_force, d->qfrc_smooth,
               d->qacc_smooth, d->qfrc_constraint, d->scratch};
  for (size_t i = 0; i < sizeof p / sizeof p[0]; i++) free(p[i]);
  free(d);
}

void or_reset_data(const or_model* m, or_data* d) {
  memcpy(d->qpos, m->qpos0, m->nq * sizeof(double));
  memset(d->qvel, 0, m->nv * sizeof(double));
  memset(d->ctrl, 0, m->nu * sizeof(double));
  memset(d->qacc_warmstart, 0, m->nv * sizeof(double));
  memset(d->qacc, 0, m->nv * sizeof(double));
  d->ncon = 0;
  d->nefc = 0;
}

/* mj_kinematics (+ mj_comPos's xipos/ximat, geom and site poses) */
void or_kinematics(const or_model* m, or_data* d) {
  d->xquat[0] = 1;
  for (int k = 1; k < 4; k++) d->xquat[k] = 0;
  for (int k = 0; k < 3; k++) d->xpos[k] = 0;
  or_quat2mat(d->xmat, d->xquat);
  memcpy(d->xipos, d->xpos, 3 * sizeof(double));
  memcpy(d->ximat, d->xmat, 9 * sizeof(double));
  for (int b = 1; b < m->nbody; b++) {
    double* xp = d->xpos + 3 * b;
    double* xq = d->xquat + 4 * b;
    int ja = m->body_jntadr[b];
    if (ja >= 0 && m->jnt_type[ja] == OR_JNT_FREE) {
      const double* q = d->qpos + m->jnt_qposadr[ja];
      memcpy(xp, q, 3 * sizeof(double));
      memcpy(xq, q + 3, 4 * sizeof(double));
      or_quat_normalize(xq);
    } else {
      int p = m->body_parent[b];
      double R[9];
      or_quat2mat(R, d->xquat + 4 * p);
      double off[3];
      or_mulmv3(off, R, m->body_pos + 3 * b);
      for (int k = 0; k < 3; k++) xp[k] = d->xpos[3 * p + k] + off[k];
      or_quat_mul(xq, d->xquat + 4 * p, m->body_quat + 4 * b);
      for (int j = ja; ja >= 0 && j < ja + m->body_jntnum[b]; j++) {
        double qv = d->qpos[m->jnt_qposadr[j]] - m->qpos0[m->jnt_qposadr[j]];
        if (m->jnt_type[j] == OR_JNT_SLIDE) {
          double Rb[9], ax[3];
          or_quat2mat(Rb, xq);
          or_mulmv3(ax, Rb, m->jnt_axis + 3 * j);
          for (int k = 0; k < 3; k++) xp[k] += ax[k] * qv;
        } else {
          double ql[4];
          or_axis_angle_quat(ql, m->jnt_axis + 3 * j, qv);
          or_quat_mul(xq, xq, ql);
        }
      }
      or_quat_normalize(xq);
    }
    or_quat2mat(d->xmat + 9 * b, xq);
    double off[3], Ri[9];
    or_mulmv3(off, d->xmat + 9 * b, m->body_ipos + 3 * b);
    for (int k = 0; k < 3; k++) d->xipos[3 * b + k] = xp[k] + off[k];
    or_quat2mat(Ri, m->body_iquat + 4 * b);
    or_mulmm3(d->ximat + 9 * b, d->xmat + 9 * b, Ri);
  }
  for (int g = 0; g < m->ngeom; g++) {
    int b = m->geom_body[g];
    double off[3], Rg[9];
    or_mulmv3(off, d->xmat + 9 * b, m->geom_pos + 3 * g);
    for (int k = 0; k < 3; k++) d->geom_xpos[3 * g + k] = d->xpos[3 * b + k] + off[k];
    or_quat2mat(Rg, m->geom_quat + 4 * g);
    or_mulmm3(d->geom_xmat + 9 * g, d->xmat + 9 * b, Rg);
  }
  for (int s = 0; s < m->nsite; s++) {
    int b = m->site_body[s];
    double off[3], Rs[9];
    or_mulmv3(off, d->xmat + 9 * b, m->site_pos + 3 * s);
    for (int k = 0; k < 3; k++) d->site_xpos[3 * s + k] = d->xpos[3 * b + k] + off[k];
    or_quat2mat(Rs, m->site_quat + 4 * s);
    or_mulmm3(d->site_xmat + 9 * s, d->xmat + 9 * b, Rs);
  }
}

/* world axis of a hinge/slide joint: R(parent frame composed with body_quat) * axis.  The axis of a
 * hinge is invariant under its own rotation, so the body's final xmat gives the same vector. */
static void joint_axis(const or_model* m, const or_data* d, int j, double ax[3]) {
  or_mulmv3(ax, d->xmat + 9 * m->jnt_body[j], m->jnt_axis + 3 * j);
}

/* mj_jac: translational (3 x nv) and rotational (3 x nv) Jacobian of point p fixed to body */
void or_body_jac(const or_model* m, const or_data* d, int body, const double p[3], double* jacp, double* jacr) {
  int nv = m->nv;
  if (jacp) memset(jacp, 0, 3 * nv * sizeof(double));
  if (jacr) memset(jacr, 0, 3 * nv * sizeof(double));
  for (int b = body; b > 0; b = m->body_parent[b]) {
    int ja = m->body_jntadr[b];
    if (ja < 0) continue;
    for (int j = ja; j < ja + m->body_jntnum[b]; j++) {
      int da = m->jnt_dofadr[j];
      const double* anchor = d->xpos + 3 * b;
      double rel[3] = {p[0] - anchor[0], p[1] - anchor[1], p[2] - anchor[2]};
      if (m->jnt_type[j] == OR_JNT_FREE) {
        for (int k = 0; k < 3; k++) {
          if (jacp) jacp[k * nv + da + k] = 1.0;
          double ax[3] = {d->xmat[9 * b + k], d->xmat[9 * b + 3 + k], d->xmat[9 * b + 6 + k]};
          double c[3];
          or_cross(c, ax, rel);
          for (int r = 0; r < 3; r++) {
            if (jacp) jacp[r * nv + da + 3 + k] = c[r];
            if (jacr) jacr[r * nv + da + 3 + k] = ax[r];
          }
        }
      } else if (m->jnt_type[j] == OR_JNT_SLIDE) {
        double ax[3];
        joint_axis(m, d, j, ax);
        for (int r = 0; r < 3; r++)
          if (jacp) jacp[r * nv + da] = ax[r];
      } else {
        double ax[3], c[3];
        joint_axis(m, d, j, ax);
        or_cross(c, ax, rel);
        for (int r = 0; r < 3; r++) {
          if (jacp) jacp[r * nv + da] = c[r];
          if (jacr) jacr[r * nv + da] = ax[r];
        }
      }
    }
  }
}

void or_jac_point(const or_model* m, const or_data* d, int body, const double p[3], double* jacp, double* jacr) {
  or_body_jac(m, d, body, p, jacp, jacr);
}

static void inertia_world(const or_model* m, const or_data* d, int b, double I[9]) {
  const double* R = d->ximat + 9 * b;
  const double* di = m->body_inertia + 3 * b;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      I[3 * i + j] = R[3 * i] * di[0] * R[3 * j] + R[3 * i + 1] * di[1] * R[3 * j + 1] + R[3 * i + 2] * di[2] * R[3 * j + 2];
}

/* joint-space inertia, dense nv x nv (the definition mj_crb evaluates recursively) */
void or_mass(const or_model* m, or_data* d) {
  int nv = m->nv;
  double* jp = d->scratch;
  double* jr = jp + 3 * nv;
  memset(d->M, 0, nv * nv * sizeof(double));
  for (int b = 1; b < m->nbody; b++) {
    if (m->body_weldid[b] == 0 || m->body_mass[b] == 0.0) continue;
    or_body_jac(m, d, b, d->xipos + 3 * b, jp, jr);
    double I[9];
    inertia_world(m, d, b, I);
    double mb = m->body_mass[b];
    for (int i = 0; i < nv; i++) {
      double ji[3] = {jp[i], jp[nv + i], jp[2 * nv + i]};
      double ri[3] = {jr[i], jr[nv + i], jr[2 * nv + i]};
      if (ji[0] == 0 && ji[1] == 0 && ji[2] == 0 && ri[0] == 0 && ri[1] == 0 && ri[2] == 0) continue;
      double Iri[3];
      or_mulmv3(Iri, I, ri);
      for (int j = 0; j < nv; j++) {
        double v = mb * (ji[0] * jp[j] + ji[1] * jp[nv + j] + ji[2] * jp[2 * nv + j]) +
                   Iri[0] * jr[j] + Iri[1] * jr[nv + j] + Iri[2] * jr[2 * nv + j];
        d->M[i * nv + j] += v;
      }
    }
  }
}

/* qfrc_bias = RNE(q, qdot, qacc = 0) incl. gravity */
void or_bias(const or_model* m, or_data* d) {
  int nv = m->nv, nb = m->nbody;
  double* jp = d->scratch;
  double* jr = jp + 3 * nv;
  double* w = jr + 3 * nv;  /* 3 nb: angular velocity */
  double* al = w + 3 * nb;  /* 3 nb: angular vp acceleration */
  double* vo = al + 3 * nb; /* 3 nb: velocity of body origin */
  double* ao = vo + 3 * nb; /* 3 nb: vp acceleration of body origin */
  memset(w, 0, 12 * nb * sizeof(double));
  memset(d->qfrc_bias, 0, nv * sizeof(double));
  for (int b = 1; b < nb; b++) {
    int p = m->body_parent[b];
    double* wb = w + 3 * b;
    double* ab = al + 3 * b;
    double* vb = vo + 3 * b;
    double* aob = ao + 3 * b;
    const double* wp = w + 3 * p;
    double r[3];
    for (int k = 0; k < 3; k++) r[k] = d->xpos[3 * b + k] - d->xpos[3 * p + k];
    double t1[3], t2[3], t3[3];
    or_cross(t1, wp, r);
    or_cross(t2, al + 3 * p, r);
    or_cross(t3, wp, t1);
    for (int k = 0; k < 3; k++) {
      wb[k] = wp[k];
      ab[k] = al[3 * p + k];
      vb[k] = vo[3 * p + k] + t1[k];
      aob[k] = ao[3 * p + k] + t2[k] + t3[k];
    }
    int ja = m->body_jntadr[b];
    for (int j = ja; ja >= 0 && j < ja + m->body_jntnum[b]; j++) {
      int da = m->jnt_dofadr[j];
      if (m->jnt_type[j] == OR_JNT_FREE) {
        double wl[3] = {d->qvel[da + 3], d->qvel[da + 4], d->qvel[da + 5]};
        or_mulmv3(wb, d->xmat + 9 * b, wl);
        for (int k = 0; k < 3; k++) {
          ab[k] = 0;
          vb[k] = d->qvel[da + k];
          aob[k] = 0;
        }
      } else {
        double ax[3], c[3];
        joint_axis(m, d, j, ax);
        double qd = d->qvel[da];
        if (m->jnt_type[j] == OR_JNT_SLIDE) {
          or_cross(c, wb, ax);
          for (int k = 0; k < 3; k++) {
            vb[k] += ax[k] * qd;
            aob[k] += 2.0 * c[k] * qd;
          }
        } else {
          or_cross(c, wb, ax);
          for (int k = 0; k < 3; k++) {
            ab[k] += c[k] * qd;
            wb[k] += ax[k] * qd;
          }
        }
      }
    }
    if (m->body_weldid[b] == 0 || m->body_mass[b] == 0.0) continue;
    double rc[3];
    for (int k = 0; k < 3; k++) rc[k] = d->xipos[3 * b + k] - d->xpos[3 * b + k];
    double u1[3], u2[3], u3[3];
    or_cross(u1, ab, rc);
    or_cross(u2, wb, rc);
    or_cross(u3, wb, u2);
    double mb = m->body_mass[b];
    double Flin[3];
    for (int k = 0; k < 3; k++) {
      d->cvel_ang[3 * b + k] = wb[k];
      d->cvel_lin[3 * b + k] = vb[k] + u2[k];
      double ac = aob[k] + u1[k] + u3[k];
      Flin[k] = mb * (ac - m->gravity[k]);
    }
    double I[9], Iw[3], Ia[3], gy[3], Fang[3];
    inertia_world(m, d, b, I);
    or_mulmv3(Iw, I, wb);
    or_mulmv3(Ia, I, ab);
    or_cross(gy, wb, Iw);
    for (int k = 0; k < 3; k++) Fang[k] = Ia[k] + gy[k];
    or_body_jac(m, d, b, d->xipos + 3 * b, jp, jr);
    for (int i = 0; i < nv; i++)
      d->qfrc_bias[i] += jp[i] * Flin[0] + jp[nv + i] * Flin[1] + jp[2 * nv + i] * Flin[2] + jr[i] * Fang[0] +
                         jr[nv + i] * Fang[1] + jr[2 * nv + i] * Fang[2];
  }
}

/* dense Cholesky L L^T (lower triangle written, row-major) */
void or_cholesky(double* A, int n) {
  for (int j = 0; j < n; j++) {
    double s = A[j * n + j];
    for (int k = 0; k < j; k++) s -= A[j * n + k] * A[j * n + k];
    double ljj = sqrt(s > 1e-300 ? s : 1e-300);
    A[j * n + j] = ljj;
    for (int i = j + 1; i < n; i++) {
      double t = A[i * n + j];
      for (int k = 0; k < j; k++) t -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = t / ljj;
    }
  }
}

void or_chol_solve(const double* L, int n, double* x) {
  for (int i = 0; i < n; i++) {
    double t = x[i];
    for (int k = 0; k < i; k++) t -= L[i * n + k] * x[k];
    x[i] = t / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double t = x[i];
    for (int k = i + 1; k < n; k++) t -= L[k * n + i] * x[k];
    x[i] = t / L[i * n + i];
  }
}

/* Envelope (profile) Cholesky, the CPU-baseline speed-up of or_cholesky: row i of L is zero left of f[i], the
 * first nonzero of row i of A's lower triangle (fill-in stays inside the envelope), so every product skipped is
 * an exact zero and the factor equals or_cholesky's bit for bit (up to the sign of zero entries).  M is block
 * diagonal by kinematic tree and the Newton Hessian keeps tree-block sparsity (MuJoCo factors both sparsely). */
void or_cholesky_env(double* A, int n, int* f) {
  for (int i = 0; i < n; i++) {
    int k = 0;
    while (k < i && A[i * n + k] == 0) k++;
    f[i] = k;
  }
  for (int j = 0; j < n; j++) {
    double s = A[j * n + j];
    for (int k = f[j]; k < j; k++) s -= A[j * n + k] * A[j * n + k];
    double ljj = sqrt(s > 1e-300 ? s : 1e-300);
    A[j * n + j] = ljj;
    for (int i = j + 1; i < n; i++) {
      if (j < f[i]) continue; /* L[i][j] stays the exact zero of A */
      double t = A[i * n + j];
      for (int k = f[i] > f[j] ? f[i] : f[j]; k < j; k++) t -= A[i * n + k] * A[j * n + k];
      A[i * n + j] = t / ljj;
    }
  }
}

void or_chol_solve_env(const double* L, int n, const int* f, double* x) {
  for (int i = 0; i < n; i++) {
    double t = x[i];
    for (int k = f[i]; k < i; k++) t -= L[i * n + k] * x[k];
    x[i] = t / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double t = x[i];
    for (int k = i + 1; k < n; k++)
      if (f[k] <= i) t -= L[k * n + i] * x[k];
    x[i] = t / L[i * n + i];
  }
}

/* mj_setConst at qpos0: body_invweight0, dof_invweight0, meaninertia (engine_setconst.c set0) */
void or_model_setconst(or_model* m) {
  or_data* d = or_data_create(m);
  int nv = m->nv;
  or_kinematics(m, d);
  or_mass(m, d);
  double tr = 0;
  for (int i = 0; i < nv; i++) tr += d->M[i * nv + i];
  m->meaninertia = tr / (nv > 0 ? nv : 1);
  double* L = malloc(nv * nv * sizeof(double));
  double* Minv = malloc(nv * nv * sizeof(double));
  double* col = malloc(nv * sizeof(double));
  memcpy(L, d->M, nv * nv * sizeof(double));
  or_cholesky(L, nv);
  for (int j = 0; j < nv; j++) {
    memset(col, 0, nv * sizeof(double));
    col[j] = 1.0;
    or_chol_solve(L, nv, col);
    for (int i = 0; i < nv; i++) Minv[i * nv + j] = col[i];
  }
  double* J = malloc(6 * nv * sizeof(double));
  double* T = malloc(6 * nv * sizeof(double));
  for (int b = 0; b < m->nbody; b++) {
    if (b == 0 || m->body_weldid[b] == 0) {
      m->body_invweight0[2 * b] = m->body_invweight0[2 * b + 1] = 0;
      continue;
    }
    or_body_jac(m, d, b, d->xipos + 3 * b, J, J + 3 * nv);
    for (int r = 0; r < 6; r++)
      for (int i = 0; i < nv; i++) {
        double s = 0;
        for (int k = 0; k < nv; k++) s += Minv[i * nv + k] * J[r * nv + k];
        T[r * nv + i] = s;
      }
    double diag[6];
    for (int r = 0; r < 6; r++) {
      double s = 0;
      for (int i = 0; i < nv; i++) s += J[r * nv + i] * T[r * nv + i];
      diag[r] = s;
    }
    double t = (diag[0] + diag[1] + diag[2]) / 3, rr = (diag[3] + diag[4] + diag[5]) / 3;
    m->body_invweight0[2 * b] = t > OR_MINVAL ? t : OR_MINVAL;
    m->body_invweight0[2 * b + 1] = rr > OR_MINVAL ? rr : OR_MINVAL;
  }
  for (int j = 0; j < m->njnt; j++) {
    int da = m->jnt_dofadr[j];
    if (m->jnt_type[j] == OR_JNT_FREE) {
      double t = (Minv[da * nv + da] + Minv[(da + 1) * nv + da + 1] + Minv[(da + 2) * nv + da + 2]) / 3;
      double r = (Minv[(da + 3) * nv + da + 3] + Minv[(da + 4) * nv + da + 4] + Minv[(da + 5) * nv + da + 5]) / 3;
      for (int k = 0; k < 3; k++) {
        m->dof_invweight0[da + k] = t;
        m->dof_invweight0[da + 3 + k] = r;
      }
    } else {
      m->dof_invweight0[da] = Minv[da * nv + da];
    }
  }
  free(L);
  free(Minv);
  free(col);
  free(J);
  free(T);
  or_data_free(d);
}
