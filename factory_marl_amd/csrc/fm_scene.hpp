// fm_scene.hpp -- host-side scene compiler for the MI355X env-step kernel.
//
// Turns (num_arms A, max_num_objects K, per-arena seeds) into the flat, specialised tables the HIP
// kernel reads: the KUKA iiwa14 + gripper template (iiwa14.xml, gripper.xml), the static world
// (scene.xml floor, scene.py Table / Bucket / BucketFence), the conveyor (conveyor_belt.xml), the
// per-arena cube half-sizes drawn by build_scene's default_rng(seed) (scene.py:121-131), the
// collision candidate list after MuJoCo's static pair filters, mixed contact parameters, and the
// mj_setConst constants (body/dof invweight0, meaninertia) the soft-constraint model needs.
// Everything here runs once per fm_create, in double precision.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace fm {

constexpr int ARM_NB = 10;  // link1..7, gripper base, left plate, right plate
constexpr int ARM_ND = 9;   // joint1..7, left slide, right slide
constexpr int NSPH = 46;    // collision spheres per arm (4 on the static base)
constexpr int NGBOX = 9;    // gripper boxes per arm

enum GeomType : int { GT_PLANE = 0, GT_SPHERE = 2, GT_BOX = 6 };

// kernel body codes: 0 static world, 1 belt, 2..1+K cubes, 2+K+10*i+b arm i body b
struct GeomRec {
  int mjid;      // MuJoCo geom id (preorder numbering of the compiled scene)
  int type;      // GT_*
  int kbody;     // kernel body code
  int mjbody;    // MuJoCo body id
  int weld;      // MuJoCo weld body id (0 = world)
  int weldparent;
  int pclass;    // parameter class 0..4
  double pos[3]; // local (or world for static)
  double R[9];
  double size[3];
  double rbound;
};

// collision body: the unit of the broadphase (one moving kernel body, or a group of static geoms)
enum { CB_STATIC = 1, CB_PLANE = 2, CB_BELT = 4 };
struct CBody {
  int kbody;      // kernel body code (0 for static groups)
  int flags;      // CB_*
  double c[3];    // static: world AABB centre
  double e[3];    // static / belt: AABB half extents
  double r;       // moving: bounding radius about the body origin (cubes: about the centre)
  int g0, ng;     // range in cb_geoms
};

struct ParamRec {
  double mu, solref[2], solimp[5];
};

struct SceneHost {
  int A = 0, K = 0, N = 0;
  int nq = 0, nv = 0, nu = 0;
  int obs_dim = 0, act_dim = 0;
  // arm template
  double arm_base[16][12];           // world pose of each arm's iiwa frame: pos(3) R(9)
  double body_local[ARM_NB][12];     // pose in parent frame
  double body_mass[ARM_NB], body_ipos[ARM_NB][3], body_iR[ARM_NB][9], body_I[ARM_NB][3];
  double body_invw[ARM_NB][2];
  double dof_range[ARM_ND][2], dof_invw[ARM_ND];
  double grip_site[3];  // in gripper-base frame
  double arm_trace_M;   // trace of the arm block of M at qpos0
  // geoms (collidable only)
  std::vector<GeomRec> geoms;
  std::vector<ParamRec> params;
  std::vector<uint32_t> pairs;  // c1 | c2 << 12 | param << 24  (compact geom indices, type-ordered)
  int nbox = 0;
  std::vector<int> box_slot;    // per compact geom, -1 for non-box
  // two-level broadphase: collision bodies, their geoms, the body pairs MuJoCo's filters allow
  std::vector<CBody> cbodies;
  std::vector<uint16_t> cb_geoms;
  std::vector<uint32_t> cb_pairs;  // b1 | b2 << 8 (b1 < b2)
  int ptab[5][5];                  // params index for (pclass g1, pclass g2)
  // per arena
  std::vector<double> cube;     // [N][K][4]: h, m, I, pad
  std::vector<float> cube_rgba;  // [N][K][4]: the seed's colour draws (alpha 1), for rendering only
  std::vector<double> meaninertia;  // [N]
  std::vector<uint64_t> rng_init;   // [N][4]: PCG64 state hi, lo, inc hi, lo (TaskManager rng)
  std::vector<uint32_t> tri;        // column-major lower triangle (i | j << 16)
  double ctrlrange[64][2];
  double bucket_x[2], bucket_y, bucket_z;
};

// numpy default_rng(seed): SeedSequence + PCG64 (numpy/random/bit_generator.pyx, src/pcg64)
struct Pcg64 {
  uint64_t s_hi, s_lo, i_hi, i_lo;
  static Pcg64 from_seed(uint64_t seed);
  uint64_t next64();
  double next_double();
};

bool build_scene(int A, int K, int N, const uint64_t* seeds, SceneHost& out, std::string& err);

// flat MJCF document of a built scene with the cubes of arena seed `seed` (scene.py:109-161 as
// dm_control compiles it); meshdir = directory of the iiwa14 .obj meshes, or null/empty for placeholders
std::string export_mjcf(const SceneHost& s, uint64_t seed, const char* meshdir);

}  // namespace fm
