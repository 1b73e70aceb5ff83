// fm_scene.cpp -- host-side scene compiler (see fm_scene.hpp).
//
// Sources transcribed (reference, read-only):
//   challenge_env/challenge_env/scene.py:9-23    PickableObject: box half-size h, mass 1000*h**3, friction (1,.01,.01)
//   challenge_env/challenge_env/scene.py:26-38   Table: box (1.2, L, 0.5) at z=0.5, solref (.002,1), solimp (.98,.9999,.001), priority 1
//   challenge_env/challenge_env/scene.py:41-61   Arm: player_site pos/euler (yaw pi for odd arms), iiwa14 + gripper attached
//   challenge_env/challenge_env/scene.py:64-106  Bucket: target_area (0.29,0.29,0.02) at z-0.04, 4 fences at euler z=f*1.57
//   challenge_env/challenge_env/scene.py:109-161 build_scene: table length, cube draws, bucket / arm placement
//   assets/conveyor_belt.xml:4-12                belt box (0.3,100,0.04) mass 1000, slide y, damping 5e-4, velocity kv 1e4
//   assets/kuka_iiwa_14/iiwa14.xml:55-168        link frames, inertials, collision spheres, joint/ctrl ranges, excludes
//   assets/gripper.xml:4-64                      gripper base / plates, equality, tendon actuator
//   assets/scene.xml:2,21                        implicitfast, dt=1e-3, floor plane
#include "fm_scene.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <tuple>

namespace fm {

namespace {

constexpr double MINVAL = 1e-15;

void quat_norm(double q[4]) {
  double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MINVAL) {
    q[0] = 1;
    q[1] = q[2] = q[3] = 0;
  } else if (std::fabs(n - 1.0) > MINVAL) {
    for (int k = 0; k < 4; k++) q[k] /= n;
  }
}

void quat2mat(const double qin[4], double R[9]) {
  double q[4] = {qin[0], qin[1], qin[2], qin[3]};
  quat_norm(q);
  double w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = w * w + x * x - y * y - z * z;
  R[1] = 2 * (x * y - w * z);
  R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z);
  R[4] = w * w - x * x + y * y - z * z;
  R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y);
  R[7] = 2 * (y * z + w * x);
  R[8] = w * w - x * x - y * y + z * z;
}

void matmul3(const double A[9], const double B[9], double C[9]) {
  double t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
  std::memcpy(C, t, sizeof t);
}

void matvec3(const double A[9], const double v[3], double r[3]) {
  double t[3] = {A[0] * v[0] + A[1] * v[1] + A[2] * v[2], A[3] * v[0] + A[4] * v[1] + A[5] * v[2],
                 A[6] * v[0] + A[7] * v[1] + A[8] * v[2]};
  std::memcpy(r, t, sizeof t);
}

void cross3(const double a[3], const double b[3], double r[3]) {
  double t[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  std::memcpy(r, t, sizeof t);
}

const double I9[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};

struct SphereDef {
  int link;  // 0 = static base, 1..7
  double r, x, y, z;
};

// iiwa14.xml:58-138 collision spheres (class "collision", default sphere type), XML order
const SphereDef kSpheres[NSPH] = {
    {0, 0.12, 0, 0, 0.03},         {0, 0.08, -0.08, 0, 0.103},     {0, 0.08, -0.08, 0, 0.04},
    {0, 0.1, 0, 0, 0.14},          {1, 0.08, 0, 0, -0.0005},       {1, 0.075, 0.01, -0.025, 0.0425},
    {1, 0.075, -0.01, -0.025, 0.0425}, {1, 0.07, 0.01, -0.045, 0.1025}, {1, 0.07, -0.01, -0.045, 0.1025},
    {2, 0.095, 0, 0, -0.01},       {2, 0.09, 0, 0, 0.045},         {2, 0.07, -0.01, 0.04, 0.054},
    {2, 0.065, -0.01, 0.09, 0.04}, {2, 0.065, -0.01, 0.13, 0.02},  {2, 0.07, 0.01, 0.04, 0.054},
    {2, 0.065, 0.01, 0.09, 0.04},  {2, 0.065, 0.01, 0.13, 0.02},   {2, 0.075, 0, 0.18, 0},
    {3, 0.075, 0, 0, 0.0355},      {3, 0.06, 0.01, 0.023, 0.0855}, {3, 0.055, 0.01, 0.048, 0.1255},
    {3, 0.06, 0.01, 0.056, 0.1755}, {3, 0.06, -0.01, 0.023, 0.0855}, {3, 0.055, -0.01, 0.048, 0.1255},
    {3, 0.06, -0.01, 0.056, 0.1755}, {3, 0.075, 0, 0.045, 0.2155}, {3, 0.075, 0, 0, 0.2155},
    {4, 0.078, 0, 0.01, 0.046},    {4, 0.06, 0.01, 0.06, 0.052},   {4, 0.065, 0.01, 0.12, 0.034},
    {4, 0.06, -0.01, 0.06, 0.052}, {4, 0.065, -0.01, 0.12, 0.034}, {4, 0.075, 0, 0.184, 0},
    {5, 0.075, 0, 0, 0.0335},      {5, 0.05, -0.012, 0.031, 0.0755}, {5, 0.05, 0.012, 0.031, 0.0755},
    {5, 0.04, -0.012, 0.06, 0.1155}, {5, 0.04, 0.012, 0.06, 0.1155}, {5, 0.04, -0.01, 0.065, 0.1655},
    {5, 0.04, 0.01, 0.065, 0.1655}, {5, 0.035, -0.012, 0.065, 0.1855}, {5, 0.035, 0.012, 0.065, 0.1855},
    {6, 0.055, 0, 0, -0.059},      {6, 0.065, 0, -0.03, 0.011},    {6, 0.08, 0, 0, 0},
    {7, 0.06, 0, 0, 0.001}};
// MuJoCo geom offset (within the arm's 70 geoms) of each sphere: visual mesh geoms interleave
const int kSphereMjOff[NSPH] = {1,  2,  3,  4,  6,  7,  8,  9,  10, 13, 14, 15, 16, 17, 18, 19,
                                20, 21, 25, 26, 27, 28, 29, 30, 31, 32, 33, 36, 37, 38, 39, 40,
                                41, 45, 46, 47, 48, 49, 50, 51, 52, 53, 56, 57, 58, 60};

}  // namespace

// ------------------------------------------------------------------------------------------------
// numpy default_rng(seed) = PCG64(SeedSequence(seed))
// ------------------------------------------------------------------------------------------------
Pcg64 Pcg64::from_seed(uint64_t seed) {
  auto hashmix = [](uint32_t v, uint32_t& hc) {
    v ^= hc;
    hc *= 0x931e8875u;
    v *= hc;
    v ^= v >> 16;
    return v;
  };
  auto mix = [](uint32_t x, uint32_t y) {
    uint32_t r = 0xca01f9ddu * x - 0x4973f715u * y;
    r ^= r >> 16;
    return r;
  };
  uint32_t ent[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  int nent = (seed >> 32) ? 2 : 1;
  uint32_t pool[4];
  uint32_t hc = 0x43b0d7e5u;
  for (int i = 0; i < 4; i++) pool[i] = hashmix(i < nent ? ent[i] : 0u, hc);
  for (int s = 0; s < 4; s++)
    for (int d = 0; d < 4; d++)
      if (s != d) pool[d] = mix(pool[d], hashmix(pool[s], hc));
  uint32_t w[8];
  uint32_t hb = 0x8b51f9ddu;
  for (int i = 0; i < 8; i++) {
    uint32_t v = pool[i % 4];
    v ^= hb;
    hb *= 0x58f38dedu;
    v *= hb;
    v ^= v >> 16;
    w[i] = v;
  }
  uint64_t val[4];
  for (int i = 0; i < 4; i++) val[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  using u128 = unsigned __int128;
  const u128 mult = ((u128)0x2360ED051FC65DA4ULL << 64) | 0x4385DF649FCCF645ULL;
  u128 initstate = ((u128)val[0] << 64) | val[1];
  u128 inc = ((((u128)val[2] << 64) | val[3]) << 1) | 1;
  u128 st = inc;  // 0 * mult + inc
  st += initstate;
  st = st * mult + inc;
  Pcg64 r;
  r.s_hi = (uint64_t)(st >> 64);
  r.s_lo = (uint64_t)st;
  r.i_hi = (uint64_t)(inc >> 64);
  r.i_lo = (uint64_t)inc;
  return r;
}

uint64_t Pcg64::next64() {
  using u128 = unsigned __int128;
  const u128 mult = ((u128)0x2360ED051FC65DA4ULL << 64) | 0x4385DF649FCCF645ULL;
  u128 st = (((u128)s_hi << 64) | s_lo) * mult + (((u128)i_hi << 64) | i_lo);
  s_hi = (uint64_t)(st >> 64);
  s_lo = (uint64_t)st;
  uint64_t x = s_hi ^ s_lo;
  unsigned rot = (unsigned)(s_hi >> 58);
  return (x >> rot) | (x << ((-rot) & 63));
}

double Pcg64::next_double() { return (double)(next64() >> 11) * (1.0 / 9007199254740992.0); }

// ------------------------------------------------------------------------------------------------
// arm template constants and mj_setConst quantities
// ------------------------------------------------------------------------------------------------
static void arm_template(SceneHost& s) {
  struct L {
    double pos[3], quat[4], mass, ipos[3], I[3], iquat[4];
  };
  // iiwa14.xml:62-140 (link1..link7)
  const L links[7] = {
      {{0, 0, 0.1575}, {1, 0, 0, 0}, 5.76, {0, -0.03, 0.12}, {0.0333, 0.033, 0.0123}, {1, 0, 0, 0}},
      {{0, 0, 0.2025}, {0, 0, 1, 1}, 6.35, {0.0003, 0.059, 0.042}, {0.0305, 0.0304, 0.011}, {0, 0, 1, 1}},
      {{0, 0.2045, 0}, {0, 0, 1, 1}, 3.5, {0, 0.03, 0.13}, {0.025, 0.0238, 0.0076}, {1, 0, 0, 0}},
      {{0, 0, 0.2155}, {1, 1, 0, 0}, 3.5, {0, 0.067, 0.034}, {0.017, 0.0164, 0.006}, {1, 1, 0, 0}},
      {{0, 0.1845, 0}, {0, 0, 1, 1}, 3.5, {0.0001, 0.021, 0.076}, {0.01, 0.0087, 0.00449}, {1, 0, 0, 0}},
      {{0, 0, 0.2155}, {1, 1, 0, 0}, 1.8, {0, 0.0006, 0.0004}, {0.0049, 0.0047, 0.0036}, {1, 1, 0, 0}},
      {{0, 0.081, 0}, {0, 0, 1, 1}, 1.2, {0, 0, 0.02}, {0.001, 0.001, 0.001}, {1, 0, 0, 0}}};
  for (int k = 0; k < 7; k++) {
    std::memcpy(s.body_local[k], links[k].pos, 3 * sizeof(double));
    quat2mat(links[k].quat, s.body_local[k] + 3);
    s.body_mass[k] = links[k].mass;
    std::memcpy(s.body_ipos[k], links[k].ipos, 3 * sizeof(double));
    std::memcpy(s.body_I[k], links[k].I, 3 * sizeof(double));
    quat2mat(links[k].iquat, s.body_iR[k]);
  }
  // gripper frame at attachment_site (0,0,0.045) of link7; gripper_base at its origin (gripper.xml:4-5)
  double gb_pos[3] = {0, 0, 0.045};
  std::memcpy(s.body_local[7], gb_pos, sizeof gb_pos);
  std::memcpy(s.body_local[7] + 3, I9, sizeof I9);
  s.body_mass[7] = 0.73;
  double gbi[3] = {0.035, 0.0125, 0.015}, gbI[3] = {0.001, 0.0025, 0.0017};
  std::memcpy(s.body_ipos[7], gbi, sizeof gbi);
  std::memcpy(s.body_I[7], gbI, sizeof gbI);
  std::memcpy(s.body_iR[7], I9, sizeof I9);
  // plates (gripper.xml:9-42): left (0.005,0,0.05) identity, right (-0.005,0,0.05) quat (0,0,0,1)
  for (int p = 0; p < 2; p++) {
    double pos[3] = {p == 0 ? 0.005 : -0.005, 0, 0.05};
    double q[4] = {p == 0 ? 1.0 : 0.0, 0, 0, p == 0 ? 0.0 : 1.0};
    std::memcpy(s.body_local[8 + p], pos, sizeof pos);
    quat2mat(q, s.body_local[8 + p] + 3);
    s.body_mass[8 + p] = 0.015;
    double I[3] = {2.375e-6, 2.375e-6, 7.5e-7};
    std::memcpy(s.body_I[8 + p], I, sizeof I);
    s.body_ipos[8 + p][0] = s.body_ipos[8 + p][1] = s.body_ipos[8 + p][2] = 0;
    std::memcpy(s.body_iR[8 + p], I9, sizeof I9);
  }
  const double rng[7] = {2.96706, 2.0944, 2.96706, 2.0944, 2.96706, 2.0944, 3.05433};
  for (int j = 0; j < 7; j++) {
    s.dof_range[j][0] = -rng[j];
    s.dof_range[j][1] = rng[j];
  }
  for (int j = 7; j < 9; j++) {
    s.dof_range[j][0] = 0.0;
    s.dof_range[j][1] = 0.060000000000000005;
  }
  s.grip_site[0] = s.grip_site[1] = 0;
  s.grip_site[2] = 0.05;

  // ---- M(q=0) of one arm and its inverse -> invweight0 (engine_setconst.c set0 semantics)
  double bp[ARM_NB][3], bR[ARM_NB][9], com[ARM_NB][3], Iw[ARM_NB][9];
  double ax[ARM_ND][3], anc[ARM_ND][3];
  double p[3] = {0, 0, 0}, R[9];
  std::memcpy(R, I9, sizeof R);
  for (int b = 0; b < ARM_NB; b++) {
    const double* par_p = b == 0 ? p : (b <= 7 ? bp[b - 1] : bp[7]);
    const double* par_R = b == 0 ? R : (b <= 7 ? bR[b - 1] : bR[7]);
    double off[3];
    matvec3(par_R, s.body_local[b], off);
    for (int k = 0; k < 3; k++) bp[b][k] = par_p[k] + off[k];
    matmul3(par_R, s.body_local[b] + 3, bR[b]);
    if (b < 7) {
      for (int k = 0; k < 3; k++) {
        ax[b][k] = bR[b][3 * k + 2];
        anc[b][k] = bp[b][k];
      }
    } else if (b >= 8) {
      for (int k = 0; k < 3; k++) {
        ax[b - 1][k] = bR[b][3 * k];
        anc[b - 1][k] = bp[b][k];
      }
    }
    double o2[3];
    matvec3(bR[b], s.body_ipos[b], o2);
    for (int k = 0; k < 3; k++) com[b][k] = bp[b][k] + o2[k];
    double Ri[9];
    matmul3(bR[b], s.body_iR[b], Ri);
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++)
        Iw[b][3 * i + j] = Ri[3 * i] * s.body_I[b][0] * Ri[3 * j] + Ri[3 * i + 1] * s.body_I[b][1] * Ri[3 * j + 1] +
                           Ri[3 * i + 2] * s.body_I[b][2] * Ri[3 * j + 2];
  }
  auto in_chain = [](int b, int d) {
    if (d < 7) return (b < 7 ? d <= b : true);
    return (d == 7 && b == 8) || (d == 8 && b == 9);
  };
  double Jc[ARM_NB][3][ARM_ND], Jr[ARM_NB][3][ARM_ND];
  std::memset(Jc, 0, sizeof Jc);
  std::memset(Jr, 0, sizeof Jr);
  for (int b = 0; b < ARM_NB; b++)
    for (int d = 0; d < ARM_ND; d++) {
      if (!in_chain(b, d)) continue;
      if (d < 7) {
        double rel[3] = {com[b][0] - anc[d][0], com[b][1] - anc[d][1], com[b][2] - anc[d][2]}, c[3];
        cross3(ax[d], rel, c);
        for (int k = 0; k < 3; k++) {
          Jc[b][k][d] = c[k];
          Jr[b][k][d] = ax[d][k];
        }
      } else {
        for (int k = 0; k < 3; k++) Jc[b][k][d] = ax[d][k];
      }
    }
  double M[ARM_ND][ARM_ND] = {};
  for (int b = 0; b < ARM_NB; b++)
    for (int i = 0; i < ARM_ND; i++)
      for (int j = 0; j < ARM_ND; j++) {
        double v = 0;
        for (int k = 0; k < 3; k++) v += s.body_mass[b] * Jc[b][k][i] * Jc[b][k][j];
        for (int k = 0; k < 3; k++)
          for (int l = 0; l < 3; l++) v += Jr[b][k][i] * Iw[b][3 * k + l] * Jr[b][l][j];
        M[i][j] += v;
      }
  s.arm_trace_M = 0;
  for (int i = 0; i < ARM_ND; i++) s.arm_trace_M += M[i][i];
  // inverse by Gauss-Jordan
  double Minv[ARM_ND][ARM_ND], W[ARM_ND][2 * ARM_ND];
  for (int i = 0; i < ARM_ND; i++)
    for (int j = 0; j < 2 * ARM_ND; j++) W[i][j] = j < ARM_ND ? M[i][j] : (j - ARM_ND == i ? 1.0 : 0.0);
  for (int c = 0; c < ARM_ND; c++) {
    int piv = c;
    for (int r = c + 1; r < ARM_ND; r++)
      if (std::fabs(W[r][c]) > std::fabs(W[piv][c])) piv = r;
    for (int j = 0; j < 2 * ARM_ND; j++) std::swap(W[c][j], W[piv][j]);
    double d = W[c][c];
    for (int j = 0; j < 2 * ARM_ND; j++) W[c][j] /= d;
    for (int r = 0; r < ARM_ND; r++)
      if (r != c) {
        double f = W[r][c];
        for (int j = 0; j < 2 * ARM_ND; j++) W[r][j] -= f * W[c][j];
      }
  }
  for (int i = 0; i < ARM_ND; i++)
    for (int j = 0; j < ARM_ND; j++) Minv[i][j] = W[i][ARM_ND + j];
  for (int d = 0; d < ARM_ND; d++) s.dof_invw[d] = Minv[d][d];
  for (int b = 0; b < ARM_NB; b++) {
    double t = 0, r = 0;
    for (int k = 0; k < 3; k++)
      for (int i = 0; i < ARM_ND; i++)
        for (int j = 0; j < ARM_ND; j++) {
          t += Jc[b][k][i] * Minv[i][j] * Jc[b][k][j];
          r += Jr[b][k][i] * Minv[i][j] * Jr[b][k][j];
        }
    s.body_invw[b][0] = std::max(MINVAL, t / 3);
    s.body_invw[b][1] = std::max(MINVAL, r / 3);
  }
}

// contact parameter classes: 0 default (floor, arm spheres), 1 table/bucket, 2 belt, 3 cube, 4 gripper
struct PClass {
  double fr, solref[2], solimp[5];
  int priority;
};
static const PClass kPClass[5] = {
    {1.0, {0.02, 1.0}, {0.9, 0.95, 0.001, 0.5, 2.0}, 0},       // MuJoCo defaults
    {1.0, {0.002, 1.0}, {0.98, 0.9999, 0.001, 0.5, 2.0}, 1},   // scene.py:35-37, 75-77, 95-97
    {0.8, {0.004, 1.0}, {0.95, 0.9999, 0.001, 0.5, 2.0}, 1},   // conveyor_belt.xml:6-7
    {1.0, {0.02, 1.0}, {0.9, 0.95, 0.001, 0.5, 2.0}, 0},       // scene.py:22 friction (1,.01,.01)
    {2.0, {0.002, 1.0}, {0.99, 0.9999, 0.001, 0.5, 2.0}, 1}};  // gripper.xml:6-39

static ParamRec mix_params(int c1, int c2) {
  const PClass& a = kPClass[c1];
  const PClass& b = kPClass[c2];
  ParamRec p;
  if (a.priority != b.priority) {
    const PClass& w = a.priority > b.priority ? a : b;
    p.mu = w.fr;
    std::memcpy(p.solref, w.solref, sizeof p.solref);
    std::memcpy(p.solimp, w.solimp, sizeof p.solimp);
  } else {
    double mix = 0.5;  // solmix 1 : 1
    p.mu = std::max(a.fr, b.fr);
    for (int k = 0; k < 2; k++) p.solref[k] = mix * a.solref[k] + (1 - mix) * b.solref[k];
    for (int k = 0; k < 5; k++) p.solimp[k] = mix * a.solimp[k] + (1 - mix) * b.solimp[k];
  }
  return p;
}

bool build_scene(int A, int K, int N, const uint64_t* seeds, SceneHost& s, std::string& err) {
  if (A < 2 || A % 2 != 0 || A > 16) {
    err = "num_arms must be even and in [2, 16] (scene.py:149)";
    return false;
  }
  if (K < 1 || K > 64) {
    err = "max_num_objects must be in [1, 64]";
    return false;
  }
  if (N < 1) {
    err = "num_arenas must be >= 1";
    return false;
  }
  s.A = A;
  s.K = K;
  s.N = N;
  s.nq = 1 + 7 * K + 9 * A;
  s.nv = 1 + 6 * K + 9 * A;
  s.nu = 1 + 8 * A;
  s.obs_dim = 24 * A + 13 * K;
  s.act_dim = 8 * A;
  arm_template(s);
  // arm placement (scene.py:147-161)
  for (int i = 0; i < A; i++) {
    double x = 0.7 * ((i % 2) ? -1.0 : 1.0);
    double y = 1.4 * (i / 2) - (A / 2 - 1);
    if (i == 4 || i == 5) {
      y = 0.5 * 1.4 * ((i - 2) / 2);
      x *= 0.9;
    }
    double yaw = (i % 2) ? M_PI : 0.0;
    double q[4] = {std::cos(yaw / 2), 0, 0, std::sin(yaw / 2)};
    s.arm_base[i][0] = x;
    s.arm_base[i][1] = y;
    s.arm_base[i][2] = 1.0;
    quat2mat(q, s.arm_base[i] + 3);
  }
  // ctrl ranges: belt, then per arm 7 joints + gripper (actuator order of the compiled model)
  s.ctrlrange[0][0] = -1;
  s.ctrlrange[0][1] = 1;
  for (int i = 0; i < A; i++)
    for (int j = 0; j < 8; j++) {
      s.ctrlrange[1 + 8 * i + j][0] = s.dof_range[j][0];
      s.ctrlrange[1 + 8 * i + j][1] = s.dof_range[j][1];
    }
  s.bucket_x[0] = 0.9;
  s.bucket_x[1] = -0.9;
  s.bucket_y = 0.7 - (A / 2 - 1);
  s.bucket_z = 1.05 + (-0.04);

  // ---- geoms (collidable only), MuJoCo numbering
  s.geoms.clear();
  auto add = [&](int mjid, int type, int kbody, int mjbody, int weld, int wparent, int pc, const double* pos,
                 const double* R, const double* size) {
    GeomRec g;
    g.mjid = mjid;
    g.type = type;
    g.kbody = kbody;
    g.mjbody = mjbody;
    g.weld = weld;
    g.weldparent = wparent;
    g.pclass = pc;
    std::memcpy(g.pos, pos, 3 * sizeof(double));
    std::memcpy(g.R, R ? R : I9, 9 * sizeof(double));
    std::memcpy(g.size, size, 3 * sizeof(double));
    g.rbound = type == GT_SPHERE ? size[0]
               : type == GT_BOX  ? std::sqrt(size[0] * size[0] + size[1] * size[1] + size[2] * size[2])
                                 : 0.0;
    s.geoms.push_back(g);
  };
  const double z3[3] = {0, 0, 0};
  {
    double sz[3] = {0, 0, 0.05};
    add(0, GT_PLANE, 0, 0, 0, 0, 0, z3, I9, sz);
    double tp[3] = {0, 0, 0.5}, ts[3] = {1.2, 1.0 + 0.5 * ((A - 2) / 2.0), 0.5};
    add(1, GT_BOX, 0, 1, 0, 0, 1, tp, I9, ts);
    double bs[3] = {0.3, 100.0, 0.04};
    add(2, GT_BOX, 1, 3, 3, 0, 2, z3, I9, bs);
  }
  for (int k = 0; k < K; k++) {
    double hs[3] = {0.04, 0.04, 0.04};  // per-arena half sizes live in s.cube; placeholder here
    add(3 + k, GT_BOX, 2 + k, 4 + k, 4 + k, 0, 3, z3, I9, hs);
  }
  for (int b = 0; b < 2; b++) {
    double bx = s.bucket_x[b];
    double tpos[3] = {bx, s.bucket_y, 1.05 + (-0.04)}, ts[3] = {0.29, 0.29, 0.02};
    add(3 + K + 5 * b, GT_BOX, 0, 5 + K + 6 * b, 0, 0, 1, tpos, I9, ts);
    for (int f = 0; f < 4; f++) {
      double a = f * 1.57;
      double q[4] = {std::cos(a / 2), 0, 0, std::sin(a / 2)}, R[9];
      quat2mat(q, R);
      double lp[3] = {0.3 - 0.05, 0, 0}, off[3];
      matvec3(R, lp, off);
      double wp[3] = {bx + off[0], s.bucket_y + off[1], 1.05 + off[2]}, fs[3] = {0.05, 0.3, 0.05};
      add(4 + K + 5 * b + f, GT_BOX, 0, 6 + K + 6 * b + f, 0, 0, 1, wp, R, fs);
    }
  }
  for (int i = 0; i < A; i++) {
    int mj0 = 13 + K + 70 * i;
    int B = 16 + K + 14 * i;  // MuJoCo body id of the arm frame
    int kb0 = 2 + K + 10 * i;
    for (int sI = 0; sI < NSPH; sI++) {
      const SphereDef& sd = kSpheres[sI];
      double lp[3] = {sd.x, sd.y, sd.z}, sz[3] = {sd.r, 0, 0};
      if (sd.link == 0) {
        double off[3];
        matvec3(s.arm_base[i] + 3, lp, off);
        double wp[3] = {s.arm_base[i][0] + off[0], s.arm_base[i][1] + off[1], s.arm_base[i][2] + off[2]};
        add(mj0 + kSphereMjOff[sI], GT_SPHERE, 0, B + 2, 0, 0, 0, wp, I9, sz);
      } else {
        int mjb = B + 2 + sd.link;
        int wparent = sd.link == 1 ? 0 : mjb - 1;
        add(mj0 + kSphereMjOff[sI], GT_SPHERE, kb0 + sd.link - 1, mjb, mjb, wparent, 0, lp, I9, sz);
      }
    }
    // gripper base box (gripper.xml:6-8), body gripper_base welded into link7
    {
      double lp[3] = {0, 0, 0.015}, sz[3] = {0.07, 0.025, 0.015};
      add(mj0 + 61, GT_BOX, kb0 + 7, B + 11, B + 9, B + 8, 4, lp, I9, sz);
    }
    const double plate_gp[4][3] = {{0, -0.0075, -0.01}, {0, -0.0075, 0.01}, {0, 0.0075, -0.01}, {0, 0.0075, 0.01}};
    for (int p = 0; p < 2; p++)
      for (int g = 0; g < 4; g++) {
        double sz[3] = {0.005, 0.0075, 0.01};
        add(mj0 + 62 + 4 * p + g, GT_BOX, kb0 + 8 + p, B + 12 + p, B + 12 + p, B + 9, 4, plate_gp[g], I9, sz);
      }
  }
  // box slots
  s.box_slot.assign(s.geoms.size(), -1);
  s.nbox = 0;
  for (size_t g = 0; g < s.geoms.size(); g++)
    if (s.geoms[g].type == GT_BOX) s.box_slot[g] = s.nbox++;

  // ---- collision candidates: MuJoCo's static pair filters (mj_collision)
  std::vector<std::pair<int, int>> excl;
  for (int i = 0; i < A; i++) {
    int B = 16 + K + 14 * i;
    int base = B + 2, l1 = B + 3, l2 = B + 4, l3 = B + 5, l4 = B + 6, l5 = B + 7, l7 = B + 9;
    int gb = B + 11, pl = B + 12, pr = B + 13;
    int ex[10][2] = {{base, l1}, {base, l2}, {base, l3}, {l1, l3}, {l3, l5},
                     {l4, l7}, {l5, l7}, {gb, pl}, {gb, pr}, {pl, pr}};
    for (auto& e : ex) excl.push_back({std::min(e[0], e[1]), std::max(e[0], e[1])});
  }
  std::map<std::tuple<long long, long long, long long>, int> pidx;
  s.params.clear();
  s.pairs.clear();
  int ng = (int)s.geoms.size();
  for (int a = 0; a < ng; a++)
    for (int b = a + 1; b < ng; b++) {
      const GeomRec& ga = s.geoms[a];
      const GeomRec& gbr = s.geoms[b];
      if (ga.weld == gbr.weld) continue;
      if (ga.weld != 0 && gbr.weld != 0 && (ga.weld == gbr.weldparent || gbr.weld == ga.weldparent)) continue;
      std::pair<int, int> bp{std::min(ga.mjbody, gbr.mjbody), std::max(ga.mjbody, gbr.mjbody)};
      if (std::find(excl.begin(), excl.end(), bp) != excl.end()) continue;
      int c1 = a, c2 = b;
      if (s.geoms[c1].type > s.geoms[c2].type) std::swap(c1, c2);
      ParamRec p = mix_params(s.geoms[c1].pclass, s.geoms[c2].pclass);
      auto key = std::make_tuple((long long)std::llround(p.mu * 1e9), (long long)std::llround(p.solref[0] * 1e12),
                                 (long long)std::llround(p.solimp[0] * 1e9 + p.solimp[1] * 1e3));
      int pi;
      auto it = pidx.find(key);
      if (it == pidx.end()) {
        pi = (int)s.params.size();
        s.params.push_back(p);
        pidx[key] = pi;
      } else {
        pi = it->second;
      }
      s.pairs.push_back((uint32_t)c1 | ((uint32_t)c2 << 12) | ((uint32_t)pi << 24));
    }
  // (geom-pair indices of one broadphase sweep are kept in 16 bits)
  if (ng >= 4096 || s.params.size() > 255 || s.pairs.size() >= 65536) {
    err = "scene too large for the pair encoding";
    return false;
  }
  for (int a = 0; a < 5; a++)
    for (int b = 0; b < 5; b++) {
      ParamRec p = mix_params(a, b);
      auto key = std::make_tuple((long long)std::llround(p.mu * 1e9), (long long)std::llround(p.solref[0] * 1e12),
                                 (long long)std::llround(p.solimp[0] * 1e9 + p.solimp[1] * 1e3));
      auto it = pidx.find(key);
      if (it == pidx.end()) {
        s.ptab[a][b] = (int)s.params.size();
        pidx[key] = s.ptab[a][b];
        s.params.push_back(p);
      } else {
        s.ptab[a][b] = it->second;
      }
    }

  // ---- collision bodies: each moving kernel body; static geoms grouped (floor, table, bucket b, arm base i)
  {
    std::vector<int> cb_of(ng, -1);
    std::vector<std::vector<int>> members;
    std::map<long long, int> idx;
    auto group = [&](long long key, int kb, int flags) {
      auto it = idx.find(key);
      if (it != idx.end()) return it->second;
      CBody c{};
      c.kbody = kb;
      c.flags = flags;
      s.cbodies.push_back(c);
      members.emplace_back();
      idx[key] = (int)s.cbodies.size() - 1;
      return (int)s.cbodies.size() - 1;
    };
    for (int g = 0; g < ng; g++) {
      const GeomRec& G = s.geoms[g];
      int cb;
      if (G.kbody == 0) {
        if (G.type == GT_PLANE)
          cb = group(-1, 0, CB_STATIC | CB_PLANE);
        else if (G.mjid == 1)
          cb = group(-2, 0, CB_STATIC);
        else if (G.mjid >= 3 + K && G.mjid < 13 + K)
          cb = group(-3 - (G.mjid - 3 - K) / 5, 0, CB_STATIC);
        else
          cb = group(-10 - (G.mjid - 13 - K) / 70, 0, CB_STATIC);
      } else {
        cb = group(G.kbody, G.kbody, G.kbody == 1 ? CB_BELT : 0);
      }
      cb_of[g] = cb;
      members[cb].push_back(g);
    }
    if (s.cbodies.size() > 255) {
      err = "too many collision bodies";
      return false;
    }
    s.cb_geoms.clear();
    for (size_t b = 0; b < s.cbodies.size(); b++) {
      CBody& c = s.cbodies[b];
      c.g0 = (int)s.cb_geoms.size();
      c.ng = (int)members[b].size();
      for (int g : members[b]) s.cb_geoms.push_back((uint16_t)g);
      double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
      c.r = 0;
      for (int g : members[b]) {
        const GeomRec& G = s.geoms[g];
        if (c.flags & CB_STATIC) {
          if (G.type == GT_PLANE) continue;
          for (int i = 0; i < 8; i++) {
            double cl[3] = {0, 0, 0}, cw[3];
            if (G.type == GT_BOX) {
              cl[0] = (i & 1) ? G.size[0] : -G.size[0];
              cl[1] = (i & 2) ? G.size[1] : -G.size[1];
              cl[2] = (i & 4) ? G.size[2] : -G.size[2];
            } else {
              cl[0] = (i & 1) ? G.size[0] : -G.size[0];
              cl[1] = (i & 2) ? G.size[0] : -G.size[0];
              cl[2] = (i & 4) ? G.size[0] : -G.size[0];
            }
            matvec3(G.R, cl, cw);
            for (int k = 0; k < 3; k++) {
              lo[k] = std::min(lo[k], G.pos[k] + cw[k]);
              hi[k] = std::max(hi[k], G.pos[k] + cw[k]);
            }
          }
        } else if (c.flags & CB_BELT) {
          for (int k = 0; k < 3; k++) c.e[k] = G.size[k];
        } else if (G.kbody >= 2 && G.kbody < 2 + K) {
          c.r = std::sqrt(3.0) * 0.05;  // largest cube (h <= 0.05), about the cube centre
        } else {
          double d = std::sqrt(G.pos[0] * G.pos[0] + G.pos[1] * G.pos[1] + G.pos[2] * G.pos[2]);
          c.r = std::max(c.r, d + G.rbound);
        }
      }
      if ((c.flags & CB_STATIC) && !(c.flags & CB_PLANE))
        for (int k = 0; k < 3; k++) {
          c.c[k] = 0.5 * (lo[k] + hi[k]);
          c.e[k] = 0.5 * (hi[k] - lo[k]);
        }
    }
    // allowed body pairs: MuJoCo's filters are per body, so every geom pair of a body pair agrees
    auto allowed = [&](int a, int b) {
      const GeomRec& ga = s.geoms[a];
      const GeomRec& gbr = s.geoms[b];
      if (ga.weld == gbr.weld) return false;
      if (ga.weld != 0 && gbr.weld != 0 && (ga.weld == gbr.weldparent || gbr.weld == ga.weldparent)) return false;
      std::pair<int, int> bp{std::min(ga.mjbody, gbr.mjbody), std::max(ga.mjbody, gbr.mjbody)};
      return std::find(excl.begin(), excl.end(), bp) == excl.end();
    };
    s.cb_pairs.clear();
    int ncb = (int)s.cbodies.size();
    for (int x = 0; x < ncb; x++)
      for (int y = x + 1; y < ncb; y++) {
        if ((s.cbodies[x].flags & CB_STATIC) && (s.cbodies[y].flags & CB_STATIC)) continue;
        int na = 0, nt = 0;
        for (int g : members[x])
          for (int h : members[y]) {
            nt++;
            na += allowed(g, h) ? 1 : 0;
          }
        if (na == 0) continue;
        if (na != nt) {
          err = "collision filter is not uniform over a body pair";
          return false;
        }
        s.cb_pairs.push_back((uint32_t)x | ((uint32_t)y << 8));
      }
  }

  // ---- per-arena cubes (scene.py:121-131: draws size, rgba[4] per cube) and constants
  s.cube.assign((size_t)N * K * 4, 0.0);
  s.cube_rgba.assign((size_t)N * K * 4, 0.0f);
  s.meaninertia.assign(N, 0.0);
  s.rng_init.assign((size_t)N * 4, 0);
  for (int n = 0; n < N; n++) {
    uint64_t seed = seeds ? seeds[n] : 42;
    Pcg64 r = Pcg64::from_seed(seed);
    double tr = 1000.0 + A * s.arm_trace_M;
    for (int k = 0; k < K; k++) {
      double h = 0.03 + (0.05 - 0.03) * r.next_double();
      float* rgba = &s.cube_rgba[((size_t)n * K + k) * 4];
      for (int c = 0; c < 4; c++) rgba[c] = (float)r.next_double();
      rgba[3] = 1.0f;
      double m = 1000.0 * std::pow(h, 3.0);
      double I = m / 3.0 * (h * h + h * h);
      double* c = &s.cube[((size_t)n * K + k) * 4];
      c[0] = h;
      c[1] = m;
      c[2] = I;
      tr += 3 * m + 3 * I;
    }
    s.meaninertia[n] = tr / s.nv;
    Pcg64 t = Pcg64::from_seed(seed);  // TaskManager's own default_rng(seed) (task_utils.py:19)
    s.rng_init[4 * n + 0] = t.s_hi;
    s.rng_init[4 * n + 1] = t.s_lo;
    s.rng_init[4 * n + 2] = t.i_hi;
    s.rng_init[4 * n + 3] = t.i_lo;
  }
  s.tri.clear();
  for (int j = 0; j < s.nv; j++)
    for (int i = j; i < s.nv; i++) s.tri.push_back((uint32_t)i | ((uint32_t)j << 16));
  return true;
}

}  // namespace fm

// ------------------------------------------------------------------------------------------------
// MJCF export: the scene this compiler builds, as one flat MJCF document that
// MuJoCo loads without dm_control, for the optional MuJoCo cross-check.  The element tree follows
// dm_control's attach semantics of build_scene (scene.py:109-161): every attached model becomes an
// attachment-frame body named "<model>/", element names carry the namescope prefixes base_env.py and
// ik_policy.py look up (base_env.py:114-126, ik_policy.py:41-45), and unnamed geoms get dm_control's
// "<scope>//unnamed_geom_<j>" names -- so body, joint, geom and actuator ids are those of the
// reference's compiled model.  Kinematics, inertias, contact parameters and ranges are written from
// the SceneHost tables the kernel runs on (angles as quaternions; limits spelled out, since the flat
// document has no per-file compiler settings).  Visual meshes (iiwa14.xml, contype 0) are written as
// mesh geoms when a mesh directory is given and otherwise as non-colliding 1 mm spheres in the same
// slots, which keeps the geom numbering without the mesh files.
// ------------------------------------------------------------------------------------------------
namespace fm {

namespace {

void mat2quat(const double R[9], double q[4]) {
  const double tr = R[0] + R[4] + R[8];
  if (tr > 0) {
    double s = 0.5 / std::sqrt(tr + 1.0);
    q[0] = 0.25 / s;
    q[1] = (R[7] - R[5]) * s;
    q[2] = (R[2] - R[6]) * s;
    q[3] = (R[3] - R[1]) * s;
  } else if (R[0] > R[4] && R[0] > R[8]) {
    double s = 2.0 * std::sqrt(1.0 + R[0] - R[4] - R[8]);
    q[0] = (R[7] - R[5]) / s;
    q[1] = 0.25 * s;
    q[2] = (R[1] + R[3]) / s;
    q[3] = (R[2] + R[6]) / s;
  } else if (R[4] > R[8]) {
    double s = 2.0 * std::sqrt(1.0 + R[4] - R[0] - R[8]);
    q[0] = (R[2] - R[6]) / s;
    q[1] = (R[1] + R[3]) / s;
    q[2] = 0.25 * s;
    q[3] = (R[5] + R[7]) / s;
  } else {
    double s = 2.0 * std::sqrt(1.0 + R[8] - R[0] - R[4]);
    q[0] = (R[3] - R[1]) / s;
    q[1] = (R[2] + R[6]) / s;
    q[2] = (R[5] + R[7]) / s;
    q[3] = 0.25 * s;
  }
  if (q[0] < 0)
    for (int k = 0; k < 4; k++) q[k] = -q[k];
}

std::string num(double x) {
  char b[40];
  std::snprintf(b, sizeof b, "%.17g", x == 0.0 ? 0.0 : x);
  return b;
}
std::string vec(const double* v, int n) {
  std::string s;
  for (int i = 0; i < n; i++) s += (i ? " " : "") + num(v[i]);
  return s;
}

struct Doc {
  std::string out;
  int depth = 0;
  void open(const std::string& tag_attrs) {
    out += std::string(2 * depth, ' ') + "<" + tag_attrs + ">\n";
    depth++;
  }
  void close(const char* tag) {
    depth--;
    out += std::string(2 * depth, ' ') + "</" + tag + ">\n";
  }
  void leaf(const std::string& tag_attrs) { out += std::string(2 * depth, ' ') + "<" + tag_attrs + "/>\n"; }
};

// contact attributes of a parameter class (kPClass; priority 1 classes carry solref/solimp)
std::string contact_attrs(int pc) {
  const PClass& p = kPClass[pc];
  if (pc == 0) return "";
  return " solref=\"" + vec(p.solref, 2) + "\" solimp=\"" + vec(p.solimp, 5) + "\" priority=\"" +
         std::to_string(p.priority) + "\"";
}

// iiwa14.xml visual meshes per body (base, link1..7) in XML order, with their material
struct Vis {
  int body;
  const char* mesh;
  const char* material;
};
const Vis kVis[] = {{0, "link_0", "gray"},         {1, "link_1", "gray"},        {2, "link_2_orange", "orange"},
                    {2, "link_2_grey", "gray"},    {3, "link_3", "gray"},        {3, "band", "light_gray"},
                    {3, "kuka", "black"},          {4, "link_4_orange", "orange"}, {4, "link_4_grey", "gray"},
                    {5, "link_5", "gray"},         {5, "band", "light_gray"},    {5, "kuka", "black"},
                    {6, "link_6_orange", "orange"}, {6, "link_6_grey", "gray"},  {7, "link_7", "gray"}};

}  // namespace

std::string export_mjcf(const SceneHost& s, uint64_t seed, const char* meshdir) {
  const int A = s.A, K = s.K;
  const bool mesh = meshdir && meshdir[0];
  Doc d;
  d.open("mujoco model=\"factory_scene_A" + std::to_string(A) + "_K" + std::to_string(K) + "_seed" +
         std::to_string((unsigned long long)seed) + "\"");
  d.leaf(std::string("compiler angle=\"radian\" autolimits=\"true\"") +
         (mesh ? " meshdir=\"" + std::string(meshdir) + "\"" : ""));
  // scene.xml:2 integrator / timestep; MuJoCo's defaults for the rest, spelled out (the kernel's solver)
  d.leaf("option timestep=\"0.001\" integrator=\"implicitfast\" cone=\"pyramidal\" solver=\"Newton\" "
         "iterations=\"100\" tolerance=\"1e-08\" ls_iterations=\"50\"");
  d.open("visual");
  d.leaf("headlight diffuse=\"0.6 0.6 0.6\" ambient=\"0.3 0.3 0.3\" specular=\"0 0 0\"");
  d.leaf("rgba haze=\"0.15 0.25 0.35 1\"");
  d.leaf("global azimuth=\"120\" elevation=\"-20\"");
  d.close("visual");
  d.leaf("statistic center=\"0 0 0\" extent=\"3\"");
  d.open("asset");
  d.leaf("texture type=\"skybox\" builtin=\"gradient\" rgb1=\"0.3 0.5 0.7\" rgb2=\"0 0 0\" width=\"512\" height=\"3072\"");
  d.leaf("texture type=\"2d\" name=\"groundplane\" builtin=\"checker\" mark=\"edge\" rgb1=\"0.2 0.3 0.4\" "
         "rgb2=\"0.1 0.2 0.3\" markrgb=\"0.8 0.8 0.8\" width=\"300\" height=\"300\"");
  d.leaf("material name=\"groundplane\" texture=\"groundplane\" texuniform=\"true\" texrepeat=\"5 5\" "
         "reflectance=\"0.2\"");
  d.leaf("material name=\"iiwa14/gray\" specular=\"0.5\" shininess=\"0.25\" rgba=\"0.4 0.4 0.4 1\"");
  d.leaf("material name=\"iiwa14/light_gray\" specular=\"0.5\" shininess=\"0.25\" rgba=\"0.6 0.6 0.6 1\"");
  d.leaf("material name=\"iiwa14/black\" specular=\"0.5\" shininess=\"0.25\" rgba=\"0 0 0 1\"");
  d.leaf("material name=\"iiwa14/orange\" specular=\"0.5\" shininess=\"0.25\" rgba=\"1 0.423529 0.0392157 1\"");
  if (mesh) {
    const char* meshes[] = {"link_0", "link_1", "link_2_orange", "link_2_grey", "link_3",  "band",
                            "kuka",   "link_4_orange", "link_4_grey", "link_5", "link_6_orange", "link_6_grey",
                            "link_7"};
    for (const char* m : meshes) d.leaf(std::string("mesh name=\"iiwa14/") + m + "\" file=\"" + m + ".obj\"");
  }
  d.close("asset");

  d.open("worldbody");
  d.leaf("light pos=\"0 0 1.5\" dir=\"0 0 -1\" directional=\"true\"");
  d.leaf("geom name=\"floor\" type=\"plane\" size=\"0 0 0.05\" material=\"groundplane\"");
  const GeomRec& tg = s.geoms[1];
  d.open("body name=\"table/\"");
  d.leaf("geom name=\"table/table\" type=\"box\" pos=\"" + vec(tg.pos, 3) + "\" size=\"" + vec(tg.size, 3) + "\"" +
         contact_attrs(1));
  d.close("body");
  // conveyor_belt.xml:4-12
  d.open("body name=\"conveyor_belt/\"");
  d.open("body name=\"conveyor_belt/conveyor\" pos=\"0 0 1.05\"");
  d.leaf("joint name=\"conveyor_belt/conveyor_linear\" type=\"slide\" axis=\"0 1 0\" solreflimit=\"0.08 1\" "
         "damping=\"0.0005\"");
  d.leaf("geom name=\"conveyor_belt/belt\" type=\"box\" size=\"" + vec(s.geoms[2].size, 3) +
         "\" mass=\"1000\" rgba=\"0.3 0.3 0.3 1\" friction=\"" + num(kPClass[2].fr) + " 0.01 0.01\"" +
         contact_attrs(2));
  d.close("body");
  d.close("body");
  // cubes (scene.py:121-133): the seed's draws -- size, then rgba[4] with alpha forced to 1
  {
    Pcg64 r = Pcg64::from_seed(seed);
    for (int k = 0; k < K; k++) {
      double h = 0.03 + (0.05 - 0.03) * r.next_double();
      double rgba[4];
      for (int c = 0; c < 4; c++) rgba[c] = r.next_double();
      rgba[3] = 1.0;
      const double sz[3] = {h, h, h};
      std::string nm = "cube" + std::to_string(k) + "/";
      d.open("body name=\"" + nm + "\"");
      d.leaf("freejoint name=\"" + nm + "unnamed_joint_0\"");
      d.leaf("geom name=\"" + nm + "cube\" type=\"box\" size=\"" + vec(sz, 3) + "\" mass=\"" +
             num(1000.0 * std::pow(h, 3.0)) + "\" rgba=\"" + vec(rgba, 4) + "\" friction=\"1 0.01 0.01\"");
      d.close("body");
    }
  }
  // buckets (scene.py:64-106, 136-145)
  for (int b = 0; b < 2; b++) {
    std::string nm = std::string("bucket") + (b ? "_1" : "") + "/";
    const double bp[3] = {s.bucket_x[b], s.bucket_y, 1.05};
    const GeomRec& ta = s.geoms[3 + K + 5 * b];
    d.open("body name=\"" + nm + "\"");
    d.open("body name=\"" + nm + "bucket\" pos=\"" + vec(bp, 3) + "\"");
    d.leaf("geom name=\"" + nm + "target_area\" type=\"box\" pos=\"0 0 -0.040000000000000001\" size=\"" +
           vec(ta.size, 3) + "\" rgba=\"1 1 1 1\"" + contact_attrs(1));
    for (int f = 0; f < 4; f++) {
      const GeomRec& fg = s.geoms[4 + K + 5 * b + f];
      double q[4];
      mat2quat(fg.R, q);
      std::string fn = nm + "bucket_fence" + (f ? "_" + std::to_string(f) : std::string()) + "/";
      d.leaf("site name=\"" + nm + "fence_site" + std::to_string(f) + "\" quat=\"" + vec(q, 4) + "\"");
      d.open("body name=\"" + fn + "\" quat=\"" + vec(q, 4) + "\"");
      d.leaf("geom name=\"" + fn + "fence\" type=\"box\" pos=\"0.25 0 0\" size=\"" + vec(fg.size, 3) +
             "\" rgba=\"0.2 0.2 0.2 1\"" + contact_attrs(1));
      d.close("body");
    }
    d.close("body");
    d.close("body");
  }
  // arms (scene.py:41-61, 147-161; iiwa14.xml; gripper.xml)
  for (int i = 0; i < A; i++) {
    const std::string an = "arm" + std::to_string(i) + "/", iw = an + "iiwa14/", gr = iw + "single_gripper/";
    double q[4];
    mat2quat(s.arm_base[i] + 3, q);
    d.open("body name=\"" + an + "\"");
    d.leaf("site name=\"" + an + "player_site\" pos=\"" + vec(s.arm_base[i], 3) + "\" quat=\"" + vec(q, 4) + "\"");
    d.open("body name=\"" + iw + "\" pos=\"" + vec(s.arm_base[i], 3) + "\" quat=\"" + vec(q, 4) + "\"");
    int gj = 0;  // iiwa14 unnamed-geom counter
    auto geoms_of = [&](int link) {
      for (const Vis& v : kVis) {
        if (v.body != link) continue;
        std::string g = "geom name=\"" + iw + "/unnamed_geom_" + std::to_string(gj++) + "\" ";
        if (mesh)
          g += std::string("type=\"mesh\" mesh=\"iiwa14/") + v.mesh + "\" material=\"iiwa14/" + v.material + "\"";
        else
          g += std::string("type=\"sphere\" size=\"0.001\" material=\"iiwa14/") + v.material + "\"";
        d.leaf(g + " contype=\"0\" conaffinity=\"0\" group=\"2\"");
      }
      for (int sI = 0; sI < NSPH; sI++) {
        const SphereDef& sd = kSpheres[sI];
        if (sd.link != link) continue;
        const double p[3] = {sd.x, sd.y, sd.z};
        d.leaf("geom name=\"" + iw + "/unnamed_geom_" + std::to_string(gj++) + "\" type=\"sphere\" size=\"" +
               num(sd.r) + "\" pos=\"" + vec(p, 3) + "\" group=\"3\"");
      }
    };
    d.open("body name=\"" + iw + "base\"");
    d.leaf("inertial mass=\"5\" pos=\"-0.10000000000000001 0 0.070000000000000007\" diaginertia=\"0.050000000000000003 "
           "0.059999999999999998 0.029999999999999999\"");
    geoms_of(0);
    for (int b = 0; b < 7; b++) {
      double bq[4], iq[4];
      mat2quat(s.body_local[b] + 3, bq);
      mat2quat(s.body_iR[b], iq);
      d.open("body name=\"" + iw + "link" + std::to_string(b + 1) + "\" pos=\"" + vec(s.body_local[b], 3) +
             "\" quat=\"" + vec(bq, 4) + "\"");
      d.leaf("inertial mass=\"" + num(s.body_mass[b]) + "\" pos=\"" + vec(s.body_ipos[b], 3) + "\" quat=\"" +
             vec(iq, 4) + "\" diaginertia=\"" + vec(s.body_I[b], 3) + "\"");
      d.leaf("joint name=\"" + iw + "joint" + std::to_string(b + 1) + "\" type=\"hinge\" axis=\"0 0 1\" limited=\"true\" "
             "range=\"" + vec(s.dof_range[b], 2) + "\"");
      geoms_of(b + 1);
    }
    d.leaf("site name=\"" + iw + "attachment_site\" pos=\"" + vec(s.body_local[7], 3) + "\"");
    // gripper.xml attached at attachment_site
    d.open("body name=\"" + gr + "\" pos=\"" + vec(s.body_local[7], 3) + "\"");
    d.open("body name=\"" + gr + "gripper_base\"");
    d.leaf("inertial mass=\"" + num(s.body_mass[7]) + "\" pos=\"" + vec(s.body_ipos[7], 3) + "\" diaginertia=\"" +
           vec(s.body_I[7], 3) + "\"");
    int gg = 0;
    const std::string gattr = " condim=\"3\" friction=\"" + num(kPClass[4].fr) + " 0.01 0.01\"" + contact_attrs(4);
    d.leaf("geom name=\"" + gr + "/unnamed_geom_" + std::to_string(gg++) +
           "\" type=\"box\" pos=\"0 0 0.014999999999999999\" size=\"0.070000000000000007 0.025000000000000001 "
           "0.014999999999999999\"" + gattr);
    for (int p = 0; p < 2; p++) {
      double pq[4];
      mat2quat(s.body_local[8 + p] + 3, pq);
      const std::string pn = gr + (p ? "right_plate" : "left_plate");
      d.open("body name=\"" + pn + "\" pos=\"" + vec(s.body_local[8 + p], 3) + "\" quat=\"" + vec(pq, 4) + "\"");
      d.leaf("inertial mass=\"" + num(s.body_mass[8 + p]) + "\" pos=\"0 0 0\" diaginertia=\"" + vec(s.body_I[8 + p], 3) +
             "\"");
      const double gp[4][3] = {{0, -0.0075, -0.01}, {0, -0.0075, 0.01}, {0, 0.0075, -0.01}, {0, 0.0075, 0.01}};
      for (int g = 0; g < 4; g++)
        d.leaf("geom name=\"" + gr + "/unnamed_geom_" + std::to_string(gg++) + "\" type=\"box\" pos=\"" +
               vec(gp[g], 3) + "\" size=\"0.0050000000000000001 0.0074999999999999997 0.01\"" + gattr);
      d.leaf("joint name=\"" + pn + "_slide_joint\" type=\"slide\" axis=\"1 0 0\" limited=\"true\" range=\"" +
             vec(s.dof_range[7 + p], 2) + "\"");
      d.close("body");
    }
    d.leaf("site name=\"" + gr + "between_gripper_plates\" pos=\"" + vec(s.grip_site, 3) + "\"");
    d.close("body");  // gripper_base
    d.close("body");  // gripper frame
    for (int b = 0; b < 7; b++) d.close("body");
    d.close("body");  // base
    d.close("body");  // iiwa14 frame
    d.close("body");  // arm frame
  }
  d.close("worldbody");

  // contact excludes (iiwa14.xml:143-151, gripper.xml:50-54)
  d.open("contact");
  for (int i = 0; i < A; i++) {
    const std::string iw = "arm" + std::to_string(i) + "/iiwa14/", gr = iw + "single_gripper/";
    const char* ex[7][2] = {{"base", "link1"}, {"base", "link2"}, {"base", "link3"}, {"link1", "link3"},
                            {"link3", "link5"}, {"link4", "link7"}, {"link5", "link7"}};
    for (auto& e : ex) d.leaf("exclude body1=\"" + iw + e[0] + "\" body2=\"" + iw + e[1] + "\"");
    d.leaf("exclude body1=\"" + gr + "gripper_base\" body2=\"" + gr + "left_plate\"");
    d.leaf("exclude body1=\"" + gr + "gripper_base\" body2=\"" + gr + "right_plate\"");
    d.leaf("exclude body1=\"" + gr + "left_plate\" body2=\"" + gr + "right_plate\"");
  }
  d.close("contact");
  d.open("equality");
  for (int i = 0; i < A; i++) {
    const std::string gr = "arm" + std::to_string(i) + "/iiwa14/single_gripper/";
    d.leaf("joint joint1=\"" + gr + "left_plate_slide_joint\" joint2=\"" + gr +
           "right_plate_slide_joint\" solref=\"0.002 1\" solimp=\"0.97999999999999998 0.99990000000000001 0.001\"");
  }
  d.close("equality");
  d.open("tendon");
  for (int i = 0; i < A; i++) {
    const std::string gr = "arm" + std::to_string(i) + "/iiwa14/single_gripper/";
    d.open("fixed name=\"" + gr + "split\"");
    d.leaf("joint joint=\"" + gr + "left_plate_slide_joint\" coef=\"0.5\"");
    d.leaf("joint joint=\"" + gr + "right_plate_slide_joint\" coef=\"0.5\"");
    d.close("fixed");
  }
  d.close("tendon");
  // actuators in the compiled order the kernel's ctrl vector follows: belt, then per arm 7 joints + gripper
  d.open("actuator");
  d.leaf("velocity name=\"conveyor_belt/slide\" joint=\"conveyor_belt/conveyor_linear\" kv=\"10000\" "
         "ctrllimited=\"true\" ctrlrange=\"" + vec(s.ctrlrange[0], 2) + "\"");
  for (int i = 0; i < A; i++) {
    const std::string iw = "arm" + std::to_string(i) + "/iiwa14/", gr = iw + "single_gripper/";
    for (int j = 0; j < 7; j++)
      d.leaf("general name=\"" + iw + "actuator" + std::to_string(j + 1) + "\" joint=\"" + iw + "joint" +
             std::to_string(j + 1) + "\" gaintype=\"fixed\" biastype=\"affine\" gainprm=\"2000\" "
             "biasprm=\"0 -2000 -200\" ctrllimited=\"true\" ctrlrange=\"" + vec(s.ctrlrange[1 + 8 * i + j], 2) + "\"");
    d.leaf("general name=\"" + gr + "gripper_linear_actuator\" tendon=\"" + gr + "split\" dyntype=\"none\" "
           "biastype=\"affine\" forcelimited=\"true\" forcerange=\"-100 100\" ctrllimited=\"true\" ctrlrange=\"" +
           vec(s.ctrlrange[8 + 8 * i], 2) + "\" gainprm=\"100 0 0\" biasprm=\"0 -100 -10\"");
  }
  d.close("actuator");
  d.close("mujoco");
  return d.out;
}

}  // namespace fm
