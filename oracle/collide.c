/* collide.c -- collision detection (TEST INFRASTRUCTURE; see oracle.h).
 *
 * Restates MuJoCo 3.1 mj_collision for the geom types this scene uses (plane, sphere, box):
 *   pair filter: contype/conaffinity, same weld body, weld parent-child (filterparent), explicit
 *   <exclude> body pairs (iiwa14.xml:150-158, gripper.xml:50-54), bounding spheres (geom_rbound+margin);
 *   parameter mixing by priority / solmix (mj_contactParam); contact frame via mju_makeFrame.
 * Narrowphase: mjc_PlaneSphere, mjc_PlaneBox and mjc_SphereSphere follow MuJoCo's published formulas.
 * Sphere-box and box-box are this project's own definitions: MuJoCo's mjc_BoxBox
 * is not available here, so box-box is SAT over 15 axes; a face contact yields the vertices of the
 * incident-face / reference-face intersection (<= 8 points), edge-edge a single point; the HIP kernel
 * implements the same definition.
 */
#include <stdlib.h>

#include "oracle.h"
#include "oracle_internal.h"

static void col(const double* R, int k, double* v) {
  v[0] = R[k];
  v[1] = R[3 + k];
  v[2] = R[6 + k];
}

/* mju_makeFrame: complete an orthonormal frame from the normal in frame[0:3] */
static void make_frame(double* f) {
  or_normalize3(f);
  f[3] = f[4] = f[5] = 0;
  if (f[1] < 0.5 && f[1] > -0.5)
    f[4] = 1;
  else
    f[5] = 1;
  double t = or_dot3(f, f + 3);
  for (int k = 0; k < 3; k++) f[3 + k] -= t * f[k];
  or_normalize3(f + 3);
  or_cross(f + 6, f, f + 3);
}

static void set_con(or_contact* c, double dist, const double pos[3], const double n[3]) {
  memset(c, 0, sizeof *c);
  c->dist = dist;
  memcpy(c->pos, pos, 3 * sizeof(double));
  memcpy(c->frame, n, 3 * sizeof(double));
  make_frame(c->frame);
}

static int plane_sphere(const double* pp, const double* pR, const double* c, double r, double margin,
                        or_contact* out) {
  double n[3] = {pR[2], pR[5], pR[8]};
  double v[3] = {c[0] - pp[0], c[1] - pp[1], c[2] - pp[2]};
  double dist = or_dot3(v, n) - r;
  if (dist > margin) return 0;
  double pos[3];
  for (int k = 0; k < 3; k++) pos[k] = c[k] - n[k] * (r + dist / 2);
  set_con(out, dist, pos, n);
  return 1;
}

int or_plane_box(const double* pp, const double* pR, const double* p, const double* R, const double* h,
                 double margin, or_contact* out) {
  double n[3] = {pR[2], pR[5], pR[8]};
  double v[3] = {p[0] - pp[0], p[1] - pp[1], p[2] - pp[2]};
  double dist = or_dot3(v, n);
  int cnt = 0;
  for (int i = 0; i < 8; i++) {
    double cl[3] = {(i & 1) ? h[0] : -h[0], (i & 2) ? h[1] : -h[1], (i & 4) ? h[2] : -h[2]};
    double cw[3];
    or_mulmv3(cw, R, cl);
    double ld = or_dot3(n, cw);
    if (dist + ld > margin || ld > 0) continue;
    double cd = dist + ld;
    double pos[3];
    for (int k = 0; k < 3; k++) pos[k] = cw[k] + p[k] - n[k] * cd / 2;
    set_con(out + cnt, cd, pos, n);
    if (++cnt >= 4) return 4;
  }
  return cnt;
}

static int sphere_sphere(const double* c1, double r1, const double* c2, double r2, double margin,
                         or_contact* out) {
  double n[3] = {c2[0] - c1[0], c2[1] - c1[1], c2[2] - c1[2]};
  double len = or_norm3(n);
  double dist = len - r1 - r2;
  if (dist > margin) return 0;
  if (len < OR_MINVAL) {
    n[0] = 1;
    n[1] = n[2] = 0;
  } else {
    for (int k = 0; k < 3; k++) n[k] /= len;
  }
  double pos[3];
  for (int k = 0; k < 3; k++) pos[k] = c1[k] + n[k] * (r1 + dist / 2);
  set_con(out, dist, pos, n);
  return 1;
}

/* sphere (geom1) vs box (geom2): closest point; centre inside -> least-penetration face */
int or_sphere_box(const double* c, double r, const double* p, const double* R, const double* h, double margin,
                  or_contact* out) {
  double d[3] = {c[0] - p[0], c[1] - p[1], c[2] - p[2]};
  double pl[3];
  or_mulmtv3(pl, R, d);
  double q[3];
  int inside = 1;
  for (int k = 0; k < 3; k++) {
    q[k] = pl[k] < -h[k] ? -h[k] : (pl[k] > h[k] ? h[k] : pl[k]);
    if (q[k] != pl[k]) inside = 0;
  }
  double nl[3], dist;
  if (!inside) {
    double dl[3] = {q[0] - pl[0], q[1] - pl[1], q[2] - pl[2]};
    double len = or_norm3(dl);
    dist = len - r;
    if (dist > margin) return 0;
    for (int k = 0; k < 3; k++) nl[k] = dl[k] / len;
  } else {
    int best = 0;
    double bd = h[0] - fabs(pl[0]);
    for (int k = 1; k < 3; k++) {
      double dk = h[k] - fabs(pl[k]);
      if (dk < bd) {
        bd = dk;
        best = k;
      }
    }
    nl[0] = nl[1] = nl[2] = 0;
    nl[best] = pl[best] >= 0 ? -1.0 : 1.0;
    dist = -bd - r;
  }
  double n[3];
  or_mulmv3(n, R, nl);
  double pos[3];
  for (int k = 0; k < 3; k++) pos[k] = c[k] + n[k] * (r + dist / 2);
  set_con(out, dist, pos, n);
  return 1;
}

/* box1 vs box2: SAT (15 axes) + reference-face clipping.  Normal from box1 to box2. */
int or_box_box(const double* p1, const double* R1, const double* h1, const double* p2, const double* R2,
               const double* h2, double margin, or_contact* out) {
  double a[3][3], b[3][3];
  for (int k = 0; k < 3; k++) {
    col(R1, k, a[k]);
    col(R2, k, b[k]);
  }
  double d[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  double best_face = 1e300, best_edge = 1e300;
  int face_id = -1, edge_id = -1;
  double face_u[3] = {0}, edge_u[3] = {0};
  double face_s = 0, edge_s = 0;
  for (int ax = 0; ax < 15; ax++) {
    double u[3];
    if (ax < 3) {
      memcpy(u, a[ax], sizeof u);
    } else if (ax < 6) {
      memcpy(u, b[ax - 3], sizeof u);
    } else {
      int i = (ax - 6) / 3, j = (ax - 6) % 3;
      or_cross(u, a[i], b[j]);
      double n = or_norm3(u);
      if (n < 1e-6) continue;
      for (int k = 0; k < 3; k++) u[k] /= n;
    }
    double ra = 0, rb = 0;
    for (int k = 0; k < 3; k++) {
      ra += h1[k] * fabs(or_dot3(u, a[k]));
      rb += h2[k] * fabs(or_dot3(u, b[k]));
    }
    double s = or_dot3(u, d);
    double ov = ra + rb - fabs(s);
    if (ov < -margin) return 0;
    if (ax < 6) {
      if (ov < best_face) {
        best_face = ov;
        face_id = ax;
        memcpy(face_u, u, sizeof u);
        face_s = s;
      }
    } else if (ov < best_edge) {
      best_edge = ov;
      edge_id = ax;
      memcpy(edge_u, u, sizeof u);
      edge_s = s;
    }
  }
  if (edge_id >= 0 && best_edge < 0.95 * best_face) {
    double n[3];
    double sg = edge_s >= 0 ? 1.0 : -1.0;
    for (int k = 0; k < 3; k++) n[k] = edge_u[k] * sg;
    int i = (edge_id - 6) / 3, j = (edge_id - 6) % 3;
    double e1[3], e2[3];
    memcpy(e1, p1, sizeof e1);
    memcpy(e2, p2, sizeof e2);
    for (int k = 0; k < 3; k++) {
      if (k != i) {
        double sgn = or_dot3(n, a[k]) >= 0 ? 1.0 : -1.0;
        for (int r = 0; r < 3; r++) e1[r] += h1[k] * sgn * a[k][r];
      }
      if (k != j) {
        double sgn = or_dot3(n, b[k]) >= 0 ? -1.0 : 1.0;
        for (int r = 0; r < 3; r++) e2[r] += h2[k] * sgn * b[k][r];
      }
    }
    double w[3] = {e1[0] - e2[0], e1[1] - e2[1], e1[2] - e2[2]};
    double bb = or_dot3(a[i], b[j]), dd = or_dot3(a[i], w), ee = or_dot3(b[j], w);
    double den = 1.0 - bb * bb;
    double s = 0, t = 0;
    if (den > 1e-12) {
      s = (bb * ee - dd) / den;
      t = (ee - bb * dd) / den;
    }
    s = s < -h1[i] ? -h1[i] : (s > h1[i] ? h1[i] : s);
    t = t < -h2[j] ? -h2[j] : (t > h2[j] ? h2[j] : t);
    double pos[3];
    for (int r = 0; r < 3; r++) pos[r] = 0.5 * (e1[r] + s * a[i][r] + e2[r] + t * b[j][r]);
    set_con(out, -best_edge, pos, n);
    return 1;
  }
  /* face contact: the vertices of the intersection of the incident face with the reference face,
   * enumerated as (1) incident vertices inside the reference rectangle, (2) reference corners inside
   * the incident quad (projected along the reference normal), (3) proper crossings of incident edges
   * with the rectangle's sides; each kept if it penetrates.  Boundary conventions make every polygon
   * vertex appear once: (1) closed rectangle, (2) open quad, (3) u-sides closed / v-sides open.  Worked in reference-face coordinates
   * (u along ar[t1], v along ar[t2], w along nref, origin at the face centre). */
  double sg = face_s >= 0 ? 1.0 : -1.0;
  double n[3];
  for (int k = 0; k < 3; k++) n[k] = face_u[k] * sg;
  const double *pr, *hr, *pi, *hi;
  double(*ar)[3], (*ai)[3];
  double nref[3];
  int kr;
  if (face_id < 3) {
    pr = p1; hr = h1; ar = a; pi = p2; hi = h2; ai = b; kr = face_id;
    memcpy(nref, n, sizeof nref);
  } else {
    pr = p2; hr = h2; ar = b; pi = p1; hi = h1; ai = a; kr = face_id - 3;
    for (int k = 0; k < 3; k++) nref[k] = -n[k];
  }
  double fc[3];
  for (int k = 0; k < 3; k++) fc[k] = pr[k] + nref[k] * hr[kr];
  int t1 = (kr + 1) % 3, t2 = (kr + 2) % 3;
  const double *ta = ar[t1], *tb = ar[t2];
  double e1 = hr[t1], e2 = hr[t2];
  /* incident face: the incident box axis most anti-parallel to nref */
  int mi = 0;
  double bestdot = -1;
  for (int k = 0; k < 3; k++) {
    double dk = fabs(or_dot3(nref, ai[k]));
    if (dk > bestdot) {
      bestdot = dk;
      mi = k;
    }
  }
  double sgn = or_dot3(nref, ai[mi]) > 0 ? -1.0 : 1.0;
  int u1 = (mi + 1) % 3, u2 = (mi + 2) % 3;
  double icr[3];
  for (int k = 0; k < 3; k++) icr[k] = pi[k] + sgn * hi[mi] * ai[mi][k] - fc[k];
  double cu = or_dot3(icr, ta), cv = or_dot3(icr, tb), cw = or_dot3(icr, nref);
  double a1u = hi[u1] * or_dot3(ai[u1], ta), a1v = hi[u1] * or_dot3(ai[u1], tb), a1w = hi[u1] * or_dot3(ai[u1], nref);
  double a2u = hi[u2] * or_dot3(ai[u2], ta), a2v = hi[u2] * or_dot3(ai[u2], tb), a2w = hi[u2] * or_dot3(ai[u2], nref);
  const double sx[4] = {1, -1, -1, 1}, sy[4] = {1, 1, -1, -1};
  double U[4], V[4], W[4];
  for (int k = 0; k < 4; k++) {
    U[k] = cu + sx[k] * a1u + sy[k] * a2u;
    V[k] = cv + sx[k] * a1v + sy[k] * a2v;
    W[k] = cw + sx[k] * a1w + sy[k] * a2w;
  }
  double cand[24][3];
  int nc = 0;
  /* (1) */
  for (int k = 0; k < 4; k++)
    if (fabs(U[k]) <= e1 && fabs(V[k]) <= e2) {
      cand[nc][0] = U[k];
      cand[nc][1] = V[k];
      cand[nc][2] = W[k];
      nc++;
    }
  /* (2) */
  double det = a1u * a2v - a2u * a1v;
  double ia = a1w * a2v - a2w * a1v, ib = a1u * a2w - a2u * a1w;
  for (int k = 0; k < 4; k++) {
    double cu_ = sx[k] * e1, cv_ = sy[k] * e2;
    int in = det != 0;
    for (int m = 0; m < 4; m++) {
      int m1 = (m + 1) & 3;
      double cr = (U[m1] - U[m]) * (cv_ - V[m]) - (V[m1] - V[m]) * (cu_ - U[m]);
      in = in && (det >= 0 ? cr > 0 : cr < 0);
    }
    if (in) {
      cand[nc][0] = cu_;
      cand[nc][1] = cv_;
      cand[nc][2] = cw + (ia * (cu_ - cu) + ib * (cv_ - cv)) / det;
      nc++;
    }
  }
  /* (3) */
  for (int m = 0; m < 4; m++) {
    int m1 = (m + 1) & 3;
    for (int sd = 0; sd < 4; sd++) {
      int onu = sd < 2;
      double ss = (sd & 1) ? -1.0 : 1.0;
      double e = onu ? e1 : e2;
      double dp = e - ss * (onu ? U[m] : V[m]);
      double dq = e - ss * (onu ? U[m1] : V[m1]);
      if ((dp > 0 && dq < 0) || (dp < 0 && dq > 0)) {
        double f = dp / (dp - dq);
        double xu = U[m] + (U[m1] - U[m]) * f, xv = V[m] + (V[m1] - V[m]) * f, xw = W[m] + (W[m1] - W[m]) * f;
        if (onu ? fabs(xv) <= e2 : fabs(xu) < e1) {
          cand[nc][0] = xu;
          cand[nc][1] = xv;
          cand[nc][2] = xw;
          nc++;
        }
      }
    }
  }
  int cnt = 0;
  for (int c = 0; c < nc && cnt < 8; c++) {
    double u = cand[c][0], v = cand[c][1], w = cand[c][2];
    if (w > margin) continue;
    double hw = 0.5 * w, pos[3];
    for (int k = 0; k < 3; k++) pos[k] = fc[k] + u * ta[k] + v * tb[k] + hw * nref[k];
    set_con(out + cnt, w, pos, n);
    cnt++;
  }
  return cnt;
}

static int excluded(const or_model* m, int b1, int b2) {
  int lo = b1 < b2 ? b1 : b2, hi = b1 < b2 ? b2 : b1;
  for (int i = 0; i < m->nexclude; i++)
    if (m->exclude[2 * i] == lo && m->exclude[2 * i + 1] == hi) return 1;
  return 0;
}

/* pair filter of mj_collision; returns 1 if the pair may collide */
static int pair_allowed(const or_model* m, int g1, int g2) {
  if (!((m->geom_contype[g1] & m->geom_conaffinity[g2]) || (m->geom_contype[g2] & m->geom_conaffinity[g1])))
    return 0;
  int b1 = m->geom_body[g1], b2 = m->geom_body[g2];
  int w1 = m->body_weldid[b1], w2 = m->body_weldid[b2];
  if (w1 == w2) return 0;
  int wp1 = w1 > 0 ? m->body_weldid[m->body_parent[w1]] : 0;
  int wp2 = w2 > 0 ? m->body_weldid[m->body_parent[w2]] : 0;
  if (w1 != 0 && w2 != 0 && (w1 == wp2 || w2 == wp1)) return 0;
  if (excluded(m, b1, b2)) return 0;
  return 1;
}

/* narrowphase for one (ordered) pair; fills geometry only */
int or_collide_geoms(const or_model* m, const or_data* d, int g1, int g2, or_contact* out, int maxout) {
  (void)maxout;
  int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
  const double *p1 = d->geom_xpos + 3 * g1, *p2 = d->geom_xpos + 3 * g2;
  const double *R1 = d->geom_xmat + 9 * g1, *R2 = d->geom_xmat + 9 * g2;
  const double *s1 = m->geom_size + 3 * g1, *s2 = m->geom_size + 3 * g2;
  double margin = m->geom_margin[g1] > m->geom_margin[g2] ? m->geom_margin[g1] : m->geom_margin[g2];
  if (t1 == OR_GEOM_PLANE && t2 == OR_GEOM_SPHERE) return plane_sphere(p1, R1, p2, s2[0], margin, out);
  if (t1 == OR_GEOM_PLANE && t2 == OR_GEOM_BOX) return or_plane_box(p1, R1, p2, R2, s2, margin, out);
  if (t1 == OR_GEOM_SPHERE && t2 == OR_GEOM_SPHERE) return sphere_sphere(p1, s1[0], p2, s2[0], margin, out);
  if (t1 == OR_GEOM_SPHERE && t2 == OR_GEOM_BOX) return or_sphere_box(p1, s1[0], p2, R2, s2, margin, out);
  if (t1 == OR_GEOM_BOX && t2 == OR_GEOM_BOX) return or_box_box(p1, R1, s1, p2, R2, s2, margin, out);
  return 0;
}

/* mj_contactParam: priority, else solmix-weighted mixing (friction = max) */
static void contact_param(const or_model* m, int g1, int g2, or_contact* c) {
  int pr1 = m->geom_priority[g1], pr2 = m->geom_priority[g2];
  if (pr1 != pr2) {
    int g = pr1 > pr2 ? g1 : g2;
    c->dim = m->geom_condim[g];
    c->mu = m->geom_friction[3 * g];
    memcpy(c->solref, m->geom_solref + 2 * g, 2 * sizeof(double));
    memcpy(c->solimp, m->geom_solimp + 5 * g, 5 * sizeof(double));
  } else {
    c->dim = m->geom_condim[g1] > m->geom_condim[g2] ? m->geom_condim[g1] : m->geom_condim[g2];
    double s1 = m->geom_solmix[g1], s2 = m->geom_solmix[g2];
    double mix;
    if (s1 < OR_MINVAL && s2 < OR_MINVAL)
      mix = 0.5;
    else if (s1 < OR_MINVAL)
      mix = 0.0;
    else if (s2 < OR_MINVAL)
      mix = 1.0;
    else
      mix = s1 / (s1 + s2);
    double f1 = m->geom_friction[3 * g1], f2 = m->geom_friction[3 * g2];
    c->mu = f1 > f2 ? f1 : f2;
    const double *r1 = m->geom_solref + 2 * g1, *r2 = m->geom_solref + 2 * g2;
    if (r1[0] > 0 && r2[0] > 0) {
      for (int k = 0; k < 2; k++) c->solref[k] = mix * r1[k] + (1 - mix) * r2[k];
    } else {
      for (int k = 0; k < 2; k++) c->solref[k] = r1[k] < r2[k] ? r1[k] : r2[k];
    }
    for (int k = 0; k < 5; k++) c->solimp[k] = mix * m->geom_solimp[5 * g1 + k] + (1 - mix) * m->geom_solimp[5 * g2 + k];
  }
  c->margin = m->geom_margin[g1] > m->geom_margin[g2] ? m->geom_margin[g1] : m->geom_margin[g2];
}

void or_collision_pairs(or_model* m) {
  const size_t np = (size_t)(m->ngeom * (m->ngeom - 1) / 2 + 1);
  free(m->cpair);
  free(m->run_lo);
  free(m->run_geom);
  free(m->run_body);
  free(m->run_margin);
  m->ncpair = m->nrun = 0;
  m->cpair = (int*)malloc(sizeof(int) * np);
  m->run_lo = (int*)malloc(sizeof(int) * (np + 1));
  m->run_geom = (int*)malloc(sizeof(int) * np);
  m->run_body = (int*)malloc(sizeof(int) * np);
  m->run_margin = (double*)malloc(sizeof(double) * np);
  for (int ga = 0; ga < m->ngeom; ga++)
    for (int gb = ga + 1; gb < m->ngeom; gb++) {
      if (!pair_allowed(m, ga, gb)) continue;
      const int bb = m->geom_body[gb];
      const double mg = m->geom_margin[ga] > m->geom_margin[gb] ? m->geom_margin[ga] : m->geom_margin[gb];
      if (m->nrun == 0 || m->run_geom[m->nrun - 1] != ga || m->run_body[m->nrun - 1] != bb) {
        m->run_lo[m->nrun] = m->ncpair;
        m->run_geom[m->nrun] = ga;
        m->run_body[m->nrun] = bb;
        m->run_margin[m->nrun++] = mg;
      } else if (mg > m->run_margin[m->nrun - 1]) {
        m->run_margin[m->nrun - 1] = mg;
      }
      int sw = m->geom_type[ga] > m->geom_type[gb];
      m->cpair[m->ncpair++] = sw ? (gb | ga << 16) : (ga | gb << 16);
    }
  m->run_lo[m->nrun] = m->ncpair;
}

/* mj_collision over the static pair list.  CPU-baseline speed-up (not in the restated algorithm's results): a run
 * of pairs (one geom against the geoms of one body) is skipped when the geom's bounding sphere misses the body's
 * bounding sphere of its geoms' spheres -- then every pair of the run fails the per-pair rbound test below, which
 * still decides each pair, so the contact list is the same, in the same order */
void or_collision(const or_model* m, or_data* d) {
  d->ncon = 0;
  or_contact tmp[16];
  double bc[3 * m->nbody], br[m->nbody];
  for (int b = 0; b < m->nbody; b++) {
    br[b] = 0;
    for (int k = 0; k < 3; k++) bc[3 * b + k] = d->xpos[3 * b + k];
  }
  for (int g = 0; g < m->ngeom; g++) {
    const int b = m->geom_body[g];
    double v[3];
    for (int k = 0; k < 3; k++) v[k] = d->geom_xpos[3 * g + k] - bc[3 * b + k];
    const double r = m->geom_rbound[g] > 0 ? or_norm3(v) + m->geom_rbound[g] : INFINITY;
    if (r > br[b]) br[b] = r;
  }
  for (int run = 0; run < m->nrun; run++) {
    const int ga = m->run_geom[run], bb = m->run_body[run];
    if (m->geom_rbound[ga] > 0 && br[bb] < INFINITY) {
      double v[3];
      for (int k = 0; k < 3; k++) v[k] = d->geom_xpos[3 * ga + k] - bc[3 * bb + k];
      const double lim = m->geom_rbound[ga] + br[bb] + m->run_margin[run];
      if (or_norm3(v) > lim * (1 + 1e-9) + 1e-9) continue;
    }
    for (int p = m->run_lo[run]; p < m->run_lo[run + 1]; p++) {
      const int g1 = m->cpair[p] & 0xFFFF, g2 = m->cpair[p] >> 16;
      double margin = m->geom_margin[g1] > m->geom_margin[g2] ? m->geom_margin[g1] : m->geom_margin[g2];
      if (m->geom_rbound[g1] > 0 && m->geom_rbound[g2] > 0) {
        double v[3];
        for (int k = 0; k < 3; k++) v[k] = d->geom_xpos[3 * g1 + k] - d->geom_xpos[3 * g2 + k];
        if (or_norm3(v) > m->geom_rbound[g1] + m->geom_rbound[g2] + margin) continue;
      }
      int n = or_collide_geoms(m, d, g1, g2, tmp, 16);
      for (int i = 0; i < n && d->ncon < d->maxcon; i++) {
        or_contact* c = d->con + d->ncon++;
        *c = tmp[i];
        c->geom[0] = g1;
        c->geom[1] = g2;
        contact_param(m, g1, g2, c);
        c->efc_adr = -1;
      }
    }
  }
}
