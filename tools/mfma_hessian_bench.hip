// Microbenchmark (measurement infrastructure, not product): the Newton Hessian's contact term
// H += sum_c B_c' K_c B_c of the (2,4) scene (nv = 43; per contact a 3 x 18 Jacobian block over <= 2 trees and a
// symmetric 3 x 3 K_c), assembled two ways on one wave64 per arena-like workgroup:
//   A  the product's path (fm_device.hpp, Newton "contact blocks"): one lane per (contact, block column), the
//      column's 18 products added to H with LDS atomics;
//   B  matrix cores: the blocks scattered into dense 48 x 48 operands Bd (rows = contact rows, columns = dofs)
//      and Pd = K_c B_c, then H = Bd' Pd as 3 x 3 tiles of 12 chained v_mfma_f32_16x16x4_f32.
// Both run on the same synthetic contacts (16 per arena, random cube/arm/belt tree pairs, the (2,4) dof
// numbering); the kernel times each variant with s_memtime over REPS repetitions and checks A == B.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/mfma_hessian_bench tools/mfma_hessian_bench.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int NV = 43, NCON = 16, CJ = 18, NP = 48, REPS = 200;

struct Con {
  int oa, ob, nda, ndb;
  float J[3 * CJ];
  float K[6];  // xx yy zz xy xz yz
};

__device__ inline float kij(const float* K, int i, int j) {
  if (i == j) return K[i];
  const int s = i + j;  // 1: xy, 2: xz, 3: yz
  return K[2 + s];
}

__global__ void __launch_bounds__(64) bench(const Con* cons, float* outA, float* outB, unsigned long long* cyc) {
  __shared__ float H[NV * NV];
  __shared__ float Bd[NP * NP];
  __shared__ float Pd[NP * NP];
  __shared__ Con C[NCON];
  const int l = threadIdx.x;
  const Con* src = cons + (size_t)blockIdx.x * NCON;
  for (int i = l; i < NCON * (int)(sizeof(Con) / 4); i += 64) ((float*)C)[i] = ((const float*)src)[i];
  __syncthreads();
  // ---- A: product path
  unsigned long long t0 = clock64();
  for (int rep = 0; rep < REPS; rep++) {
    for (int e = l; e < NV * NV; e += 64) H[e] = 0.f;
    __syncthreads();
    for (int e = l; e < CJ * NCON; e += 64) {
      const int c = e / CJ, ii = e - CJ * c;
      const Con& k = C[c];
      const int ncol = k.nda + k.ndb;
      if (ii >= ncol) continue;
      const float* J = k.J;
      const float b0 = J[ii], b1 = J[CJ + ii], b2 = J[2 * CJ + ii];
      const float q0 = k.K[0] * b0 + k.K[3] * b1 + k.K[4] * b2;
      const float q1 = k.K[3] * b0 + k.K[1] * b1 + k.K[5] * b2;
      const float q2 = k.K[4] * b0 + k.K[5] * b1 + k.K[2] * b2;
      const int gi = ii < k.nda ? k.oa + ii : k.ob + ii - k.nda;
      float* Hrow = H + gi * NV;
#pragma unroll
      for (int jj = 0; jj < CJ; jj++) {
        const int gj = jj < k.nda ? k.oa + jj : k.ob + jj - k.nda;
        const float val = q0 * J[jj] + q1 * J[CJ + jj] + q2 * J[2 * CJ + jj];
        if (jj < ncol) atomicAdd(Hrow + gj, val);
      }
    }
    __syncthreads();
  }
  unsigned long long t1 = clock64();
  for (int e = l; e < NV * NV; e += 64) outA[(size_t)blockIdx.x * NV * NV + e] = H[e];
  __syncthreads();
  // ---- B: dense operands + MFMA
  unsigned long long t2 = clock64();
  for (int rep = 0; rep < REPS; rep++) {
    for (int e = l; e < NP * NP; e += 64) {
      Bd[e] = 0.f;
      Pd[e] = 0.f;
    }
    __syncthreads();
    for (int e = l; e < CJ * NCON; e += 64) {  // scatter: lane per (contact, block column)
      const int c = e / CJ, ii = e - CJ * c;
      const Con& k = C[c];
      if (ii >= k.nda + k.ndb) continue;
      const int gi = ii < k.nda ? k.oa + ii : k.ob + ii - k.nda;
      const float b0 = k.J[ii], b1 = k.J[CJ + ii], b2 = k.J[2 * CJ + ii];
      Bd[(3 * c + 0) * NP + gi] = b0;
      Bd[(3 * c + 1) * NP + gi] = b1;
      Bd[(3 * c + 2) * NP + gi] = b2;
      Pd[(3 * c + 0) * NP + gi] = kij(k.K, 0, 0) * b0 + kij(k.K, 0, 1) * b1 + kij(k.K, 0, 2) * b2;
      Pd[(3 * c + 1) * NP + gi] = kij(k.K, 1, 0) * b0 + kij(k.K, 1, 1) * b1 + kij(k.K, 1, 2) * b2;
      Pd[(3 * c + 2) * NP + gi] = kij(k.K, 2, 0) * b0 + kij(k.K, 2, 1) * b1 + kij(k.K, 2, 2) * b2;
    }
    __syncthreads();
    // H (48 x 48) = Bd' Pd: A operand (16 x 4) = Bd'[m0.., k0..] = Bd[k0 + l/16][m0 + l%16],
    // B operand (4 x 16) = Pd[k0 + l/16][n0 + l%16]; D lane l holds column l%16, rows 4 (l/16) + i
    for (int tm = 0; tm < 3; tm++)
      for (int tn = 0; tn < 3; tn++) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k0 = 0; k0 < NP; k0 += 4) {
          const float a = Bd[(k0 + l / 16) * NP + 16 * tm + l % 16];
          const float b = Pd[(k0 + l / 16) * NP + 16 * tn + l % 16];
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const int r = 16 * tm + 4 * (l / 16) + i, cidx = 16 * tn + l % 16;
          if (r < NV && cidx < NV) H[r * NV + cidx] = acc[i];
        }
      }
    __syncthreads();
  }
  unsigned long long t3 = clock64();
  for (int e = l; e < NV * NV; e += 64) outB[(size_t)blockIdx.x * NV * NV + e] = H[e];
  if (l == 0) {
    cyc[2 * blockIdx.x] = (t1 - t0) / REPS;
    cyc[2 * blockIdx.x + 1] = (t3 - t2) / REPS;
  }
}

int main(int argc, char** argv) {
  const int nblk = argc > 1 ? atoi(argv[1]) : 1024;
  std::vector<Con> h((size_t)nblk * NCON);
  srand(7);
  auto U = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
  for (auto& c : h) {
    // tree a: a cube (dofs 1 + 6k) or the belt (dof 0); tree b: an arm (25 or 34) or another cube
    const int cube = rand() % 4, kind = rand() % 3;
    c.oa = kind == 0 ? 0 : 1 + 6 * cube;
    c.nda = kind == 0 ? 1 : 6;
    if (kind == 2) {
      c.ob = 25 + 9 * (rand() % 2);
      c.ndb = 9;
    } else {
      c.ob = 1 + 6 * ((cube + 1) % 4);
      c.ndb = 6;
    }
    for (int i = 0; i < 3 * CJ; i++) c.J[i] = (i % CJ) < c.nda + c.ndb ? U() : 0.f;
    const float d = 1.f + std::fabs(U());
    c.K[0] = d;
    c.K[1] = d;
    c.K[2] = d;
    c.K[3] = 0.1f * U();
    c.K[4] = 0.1f * U();
    c.K[5] = 0.1f * U();
  }
  Con* dc;
  float *dA, *dB;
  unsigned long long* dcyc;
  hipMalloc(&dc, h.size() * sizeof(Con));
  hipMalloc(&dA, (size_t)nblk * NV * NV * 4);
  hipMalloc(&dB, (size_t)nblk * NV * NV * 4);
  hipMalloc(&dcyc, (size_t)nblk * 2 * 8);
  hipMemcpy(dc, h.data(), h.size() * sizeof(Con), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(bench, dim3(nblk), dim3(64), 0, 0, dc, dA, dB, dcyc);
  if (hipDeviceSynchronize() != hipSuccess) {
    printf("kernel failed\n");
    return 1;
  }
  std::vector<float> A((size_t)nblk * NV * NV), B(A.size());
  std::vector<unsigned long long> cyc((size_t)nblk * 2);
  hipMemcpy(A.data(), dA, A.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(B.data(), dB, B.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(cyc.data(), dcyc, cyc.size() * 8, hipMemcpyDeviceToHost);
  double err = 0, ref = 0, ca = 0, cb = 0;
  for (size_t i = 0; i < A.size(); i++) {
    err = std::fmax(err, std::fabs(A[i] - B[i]));
    ref = std::fmax(ref, std::fabs(A[i]));
  }
  for (int b = 0; b < nblk; b++) {
    ca += cyc[2 * b];
    cb += cyc[2 * b + 1];
  }
  printf("{\"arenas\": %d, \"contacts\": %d, \"nv\": %d, \"atomics_cycles\": %.1f, \"mfma_cycles\": %.1f, "
         "\"max_abs_diff\": %.3e, \"max_abs\": %.3e, \"clock\": \"s_memtime (clock64) per assembly, mean over "
         "workgroups\"}\n",
         nblk, NCON, NV, ca / nblk, cb / nblk, err, ref);
  return err <= 1e-4 * (ref + 1) ? 0 : 2;
}
