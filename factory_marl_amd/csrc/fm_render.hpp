// fm_render.hpp -- batched offscreen rgb_array rendering of arenas.
//
// The reference renders one env at a time with MuJoCo's OpenGL renderer (rendering.py:153-305 OffScreenViewer,
// 653-789 MujocoRenderer.render("rgb_array"); base_env.py:288-306), a visual-only side path for videos and
// debugging.  Here the arenas resident in HBM are ray cast on the GPU, many at once, with no host round trip:
//   1. render_frames_kernel -- one wave per requested arena: forward kinematics of the arena's stored state
//      (the step kernel's own FK: hinge sin/cos, arm chains, cube rotations) and the world frame + colour of
//      every collidable geom -> a [count][ngc][20] float table (optionally the caller's buffer).
//   2. render_pixels_kernel -- a 16x16 pixel tile per workgroup (4 pixels per lane), grid (tiles, count): the
//      arena's geom table staged in LDS, one primary ray per pixel against planes / spheres / boxes (slab test
//      in the box frame), Lambert shading with the scene's headlight and top light, the floor checker and the
//      skybox gradient of assets/scene.xml.
// What is drawn is the collision geometry the physics uses: the arms appear as their collision spheres and
// gripper boxes (the iiwa14 visual meshes are not loaded), coloured like the meshes they stand for.
#pragma once
#include "fm_device.hpp"

namespace fm {

// geom table row of the renderer: mjid, type (GC_*), world pos(3), R(9), size(3), rgb(3)
constexpr int RF_N = 20;
constexpr int RTILE = 16;

struct RenderParams {
  float eye[3], fwd[3], right[3], up[3];  // world frame
  float tan_y, aspect;
  int width, height, tiles_x;
  const int* arenas;       // [count]
  const float* geom_rgb;   // [ngc][4] base colour (cubes: from cube_rgba)
  const float* cube_rgba;  // [N][K][4]
  float* frames;           // [count][ngc][RF_N]
  uint8_t* rgb;            // [count][height][width][3], row 0 = top
};

template <typename T, typename DIM>
__global__ void __launch_bounds__(64) render_frames_kernel(Model<T> M, State<T> S, Lay L, RenderParams rp) {
  FM_SMEM_DECL(smem);
  const DIM dm(M.dm);
  Ws<T, DIM> w{lds_base(smem), &L};
  const int slot = blockIdx.x, arena = rp.arenas[slot];
  const int K = dm.K;
  init_arena(M, w, arena);
  SYNC();
  load_state(M, S, w, arena, false);
  SYNC();
  arm_hinge_sincos(M, w);
  SYNC();
  if (LANE < dm.A) arm_chain<T, DIM, false>(M, w, LANE);
  for (int k = LANE; k < K; k += WAVE) {  // cube rotations as in stage(): normalised quaternion -> R
    const T* qq = w.q() + 1 + 7 * k;
    T qu[4] = {qq[3], qq[4], qq[5], qq[6]};
    T n = sqrt(qu[0] * qu[0] + qu[1] * qu[1] + qu[2] * qu[2] + qu[3] * qu[3]);
    if (n < T(1e-15)) {
      qu[0] = 1;
      qu[1] = qu[2] = qu[3] = 0;
    } else {
      for (int c = 0; c < 4; c++) qu[c] /= n;
    }
    T* R = w.cR() + 9 * k;
    T ww = qu[0], x = qu[1], y = qu[2], z = qu[3];
    R[0] = ww * ww + x * x - y * y - z * z;
    R[1] = T(2) * (x * y - ww * z);
    R[2] = T(2) * (x * z + ww * y);
    R[3] = T(2) * (x * y + ww * z);
    R[4] = ww * ww - x * x + y * y - z * z;
    R[5] = T(2) * (y * z - ww * x);
    R[6] = T(2) * (x * z - ww * y);
    R[7] = T(2) * (y * z + ww * x);
    R[8] = ww * ww - x * x - y * y + z * z;
  }
  SYNC();
  const T* q = w.q();
  const double zs = zshift<T>();
  float* out = rp.frames + (size_t)slot * dm.ngc * RF_N;
  for (int g = LANE; g < dm.ngc; g += WAVE) {
    const int gi = w.ginfo()[g];
    const int type = gi & 3, kb = (gi >> 8) & 255;
    const T* gg = M.geom + 16 * g;
    T p[3], R[9], h[3];
    if (kb == 0) {
      for (int k = 0; k < 3; k++) p[k] = gg[k];
    } else if (kb == 1) {
      p[0] = 0;
      p[1] = q[0];
      p[2] = T(1.05 - zs);
    } else if (kb < 2 + K) {
      for (int k = 0; k < 3; k++) p[k] = q[1 + 7 * (kb - 2) + k];
    } else {
      const int arm = (kb - 2 - K) / 10, b = (kb - 2 - K) % 10;
      T off[3];
      matvec3(w.bR() + 90 * arm + 9 * b, gg, off);
      for (int k = 0; k < 3; k++) p[k] = w.bpos()[30 * arm + 3 * b + k] + off[k];
    }
    if (type == GC_SPHERE) {
      for (int k = 0; k < 9; k++) R[k] = (k % 4 == 0) ? T(1) : T(0);
      h[0] = h[1] = h[2] = gg[12];
    } else {
      geom_frame(M, w, g, kb, R, h);
    }
    float* o = out + RF_N * g;
    o[0] = (float)M.geom_i[4 * g];
    o[1] = (float)type;
    o[2] = (float)p[0];
    o[3] = (float)p[1];
    o[4] = (float)((double)p[2] + zs);
    for (int k = 0; k < 9; k++) o[5 + k] = (float)R[k];
    for (int k = 0; k < 3; k++) o[14 + k] = (float)h[k];
    const float* c = (kb >= 2 && kb < 2 + K) ? rp.cube_rgba + ((size_t)arena * K + (kb - 2)) * 4 : rp.geom_rgb + 4 * g;
    for (int k = 0; k < 3; k++) o[17 + k] = c[k];
  }
}

// one primary ray against the arena's geoms; returns the hit distance (or a large value), normal and geom
__device__ __forceinline__ float cast_ray(const float* tab, int ngc, const float o[3], const float d[3], float n[3],
                                          int& hit) {
  float best = 3.0e30f;
  hit = -1;
  for (int g = 0; g < ngc; g++) {
    const float* r = tab + RF_N * g;
    const int type = (int)r[1];
    const float c[3] = {r[2], r[3], r[4]};
    const float oc[3] = {o[0] - c[0], o[1] - c[1], o[2] - c[2]};
    if (type == GC_PLANE) {  // z-up plane through c (the floor)
      if (d[2] < -1e-7f) {
        const float t = -oc[2] / d[2];
        if (t > 1e-4f && t < best) {
          best = t;
          hit = g;
          n[0] = 0.f;
          n[1] = 0.f;
          n[2] = 1.f;
        }
      }
      continue;
    }
    if (type == GC_SPHERE) {
      const float rad = r[14];
      const float b = oc[0] * d[0] + oc[1] * d[1] + oc[2] * d[2];
      const float cc = oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2] - rad * rad;
      const float disc = b * b - cc;
      if (disc <= 0.f) continue;
      const float t = -b - sqrtf(disc);
      if (t > 1e-4f && t < best) {
        best = t;
        hit = g;
        const float inv = 1.f / rad;
        for (int k = 0; k < 3; k++) n[k] = (oc[k] + t * d[k]) * inv;
      }
      continue;
    }
    // box: slab test in the box frame (local = R^T (x - c))
    const float* R = r + 5;
    float lo[3], ld[3];
    for (int k = 0; k < 3; k++) {
      lo[k] = R[k] * oc[0] + R[3 + k] * oc[1] + R[6 + k] * oc[2];
      ld[k] = R[k] * d[0] + R[3 + k] * d[1] + R[6 + k] * d[2];
    }
    float tn = -3.0e30f, tf = 3.0e30f;
    int ax = 0;
    float sg = 1.f;
    bool miss = false;
    for (int k = 0; k < 3; k++) {
      const float hk = r[14 + k];
      if (fabsf(ld[k]) < 1e-12f) {
        if (fabsf(lo[k]) > hk) miss = true;
        continue;
      }
      const float inv = 1.f / ld[k];
      float t1 = (-hk - lo[k]) * inv, t2 = (hk - lo[k]) * inv;
      const float s = ld[k] > 0.f ? -1.f : 1.f;  // the face entered first
      if (t1 > t2) {
        const float tt = t1;
        t1 = t2;
        t2 = tt;
      }
      if (t1 > tn) {
        tn = t1;
        ax = k;
        sg = s;
      }
      tf = fminf(tf, t2);
    }
    if (miss || tn > tf || tn <= 1e-4f || tn >= best) continue;
    best = tn;
    hit = g;
    for (int k = 0; k < 3; k++) n[k] = sg * R[3 * k + ax];
  }
  return best;
}

__global__ void __launch_bounds__(64) render_pixels_kernel(RenderParams rp, int ngc) {
  FM_SMEM_DECL(smem);
  float* tab = (float*)smem;
  const int slot = blockIdx.y;
  const float* src = rp.frames + (size_t)slot * ngc * RF_N;
  for (int i = LANE; i < ngc * RF_N; i += WAVE) tab[i] = src[i];
  __syncthreads();
  const int tx = blockIdx.x % rp.tiles_x, ty = blockIdx.x / rp.tiles_x;
  uint8_t* img = rp.rgb + (size_t)slot * rp.height * rp.width * 3;
#pragma unroll 1
  for (int s = 0; s < RTILE * RTILE / WAVE; s++) {
    const int p = s * WAVE + LANE;
    const int px = tx * RTILE + (p % RTILE), py = ty * RTILE + (p / RTILE);
    if (px >= rp.width || py >= rp.height) continue;
    const float sx = (2.f * (px + 0.5f) / rp.width - 1.f) * rp.tan_y * rp.aspect;
    const float sy = (1.f - 2.f * (py + 0.5f) / rp.height) * rp.tan_y;
    float d[3];
    for (int k = 0; k < 3; k++) d[k] = rp.fwd[k] + sx * rp.right[k] + sy * rp.up[k];
    const float dn = rsqrtf(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    for (int k = 0; k < 3; k++) d[k] *= dn;
    float n[3];
    int hit;
    const float t = cast_ray(tab, ngc, rp.eye, d, n, hit);
    float col[3];
    if (hit < 0) {  // skybox gradient rgb1 (0.3 0.5 0.7) above, rgb2 (0 0 0) below
      const float u = 0.5f * (d[2] + 1.f);
      col[0] = 0.3f * u;
      col[1] = 0.5f * u;
      col[2] = 0.7f * u;
    } else {
      const float* r = tab + RF_N * hit;
      float base[3] = {r[17], r[18], r[19]};
      if ((int)r[1] == GC_PLANE) {  // groundplane checker, 0.1 m squares
        const float x = rp.eye[0] + t * d[0], y = rp.eye[1] + t * d[1];
        const int cx = (int)floorf(x * 10.f), cy = (int)floorf(y * 10.f);
        const bool a = ((cx + cy) & 1) == 0;
        base[0] = a ? 0.2f : 0.1f;
        base[1] = a ? 0.3f : 0.2f;
        base[2] = a ? 0.4f : 0.3f;
      }
      const float head = fmaxf(0.f, -(n[0] * d[0] + n[1] * d[1] + n[2] * d[2]));
      const float top = fmaxf(0.f, n[2]);
      const float lum = 0.3f + 0.6f * head + 0.4f * top;
      for (int k = 0; k < 3; k++) col[k] = fminf(1.f, base[k] * lum);
    }
    uint8_t* o = img + ((size_t)py * rp.width + px) * 3;
    for (int k = 0; k < 3; k++) o[k] = (uint8_t)(col[k] * 255.f + 0.5f);
  }
}

}  // namespace fm
