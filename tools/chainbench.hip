// Microbenchmark of the 16-step register pivot chain (wave_chol_inv16, common.h) that bounds
// the grouped polish's LDS Cholesky (k_pg_solve) and k_gcap_prep's H_b: cycles per chain for
// one wave alone, one wave per SIMD and four waves per SIMD, for the library's chain and for
// variants (row kk by gfx950 permlane swaps instead of ds_bpermute; fewer Newton steps).
// Checks each variant's L and L^-1 against the library chain.  Experiment tooling:
//   hipcc --offload-arch=gfx950 -O3 -I porqua_amd/csrc tools/chainbench.hip -o /tmp/chainbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include "common.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

using namespace pq;

// row (K & 3) of the 4 x 16-lane rows broadcast to every row: permlane16_swap pairs rows
// (0,1) / (2,3), permlane32_swap the halves -- VALU only, no LDS round trip
template <int K>
__device__ __forceinline__ int row_to_all_b32(int v) {
  const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);   // {rows 0,0,2,2 ; 1,1,3,3}
  const int e = (K & 1) ? (int)p[1] : (int)p[0];
  const auto h = __builtin_amdgcn_permlane32_swap(e, e, false, false);   // {lo,lo ; hi,hi}
  return (K & 2) ? (int)h[1] : (int)h[0];
}
template <int K>
__device__ __forceinline__ double row_to_all(double v) {
  return __hiloint2double(row_to_all_b32<K>(__double2hiint(v)), row_to_all_b32<K>(__double2loint(v)));
}

// variant: the library chain with row kk by permlane swaps; NEWTON = Newton steps on rsq
template <int NEWTON>
__device__ __forceinline__ int chain_pl(double (&A)[4], double (&Bv)[4]) {
  const int l = lane_id();
  const int cc = l & 15, gg = l >> 4;
  int bad = 0;
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) {
    const int src = ((kk & 3) << 4);
    const double akk = A[kk >> 2];
    const double piv = readlane_f64(akk, src | kk);
    double rowk, bkr;
    switch (kk & 3) {   // (compile time)
      case 0: rowk = row_to_all<0>(akk); bkr = row_to_all<0>(Bv[kk >> 2]); break;
      case 1: rowk = row_to_all<1>(akk); bkr = row_to_all<1>(Bv[kk >> 2]); break;
      case 2: rowk = row_to_all<2>(akk); bkr = row_to_all<2>(Bv[kk >> 2]); break;
      default: rowk = row_to_all<3>(akk); bkr = row_to_all<3>(Bv[kk >> 2]); break;
    }
    double colv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) colv[q] = row_bcast16(A[q], kk);
    if (!(piv > 0.0) || !isfinite(piv)) bad = 1;
    double rs = __builtin_amdgcn_rsq(piv);
#pragma unroll
    for (int s = 0; s < NEWTON; ++s) rs = rs * fma(-0.5 * piv * rs, rs, 1.5);
    const double bk = bkr * rs;
    const double lck = cc > kk ? rowk * rs : 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (4 * q + 3 < kk) continue;
      const int r = gg + 4 * q;
      const double lrk = colv[q] * rs;
      const double lrt = r > kk ? lrk : 0.0;
      const double upd = fma(-lrt, lck, A[q]);
      A[q] = (cc == kk && r >= kk) ? lrk : upd;
      const double bu = fma(-lrt, bk, Bv[q]);
      Bv[q] = r == kk ? bk : bu;
    }
  }
  return bad;
}

template <int V>
__global__ __launch_bounds__(64) void k_chain(const double* M, double* out, long long* cyc, int reps) {
  const int l = threadIdx.x & 63;
  const double* Mb = M + (blockIdx.x & 255) * 256;
  double A0[4], A[4], Bv[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) A0[q] = Mb[((l >> 4) + 4 * q) * 16 + (l & 15)];
  double acc = 0.0;
  int bad = 0;
  const long long t0 = wall_clock64();
  for (int it = 0; it < reps; ++it) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      A[q] = A0[q] + acc * 1e-300;   // (dependency on the previous chain)
      Bv[q] = ((l >> 4) + 4 * q) == (l & 15) ? 1.0 : 0.0;
    }
    if (V == 0) bad |= wave_chol_inv16(A, Bv);
    else if (V == 1) bad |= chain_pl<2>(A, Bv);
    else bad |= chain_pl<1>(A, Bv);
    acc += A[0] + Bv[3];
  }
  const long long t1 = wall_clock64();
  if (blockIdx.x < 256) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      out[(blockIdx.x * 2) * 256 + q * 64 + l] = A[q];
      out[(blockIdx.x * 2 + 1) * 256 + q * 64 + l] = Bv[q];
    }
  }
  if (l == 0) cyc[blockIdx.x] = (t1 - t0) + (bad ? (1ll << 40) : 0) + (acc == 12345.0 ? 1 : 0);
}

int main() {
  std::vector<double> h(256 * 256);
  srand(7);
  for (int b = 0; b < 256; ++b) {   // SPD: G G' / 16 + I
    double G[16][16];
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) G[i][j] = (rand() / (double)RAND_MAX) - 0.5;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double s = i == j ? 1.0 : 0.0;
        for (int k = 0; k < 16; ++k) s += G[i][k] * G[j][k] / 16.0;
        h[b * 256 + i * 16 + j] = s;
      }
  }
  double *dM, *dO;
  long long* dC;
  const int maxg = 256 * 16;
  CK(hipMalloc(&dM, h.size() * 8));
  CK(hipMalloc(&dO, 512 * 256 * 8));
  CK(hipMalloc(&dC, maxg * 8));
  CK(hipMemcpy(dM, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  const int reps = 2000;
  std::vector<double> ref(512 * 256), got(512 * 256);
  std::vector<long long> cyc(maxg);
  const char* names[3] = {"library (ds_bpermute row, 2 Newton)", "permlane row, 2 Newton", "permlane row, 1 Newton"};
  for (int v = 0; v < 3; ++v) {
    for (int grid : {1, 1024, 4096}) {
      for (int rep = 0; rep < 2; ++rep) {
        if (v == 0) hipLaunchKernelGGL(k_chain<0>, dim3(grid), dim3(64), 0, 0, dM, dO, dC, reps);
        if (v == 1) hipLaunchKernelGGL(k_chain<1>, dim3(grid), dim3(64), 0, 0, dM, dO, dC, reps);
        if (v == 2) hipLaunchKernelGGL(k_chain<2>, dim3(grid), dim3(64), 0, 0, dM, dO, dC, reps);
        CK(hipDeviceSynchronize());
      }
      CK(hipMemcpy(cyc.data(), dC, grid * 8, hipMemcpyDeviceToHost));
      double mean = 0;
      int bad = 0;
      for (int g = 0; g < grid; ++g) {
        bad |= (cyc[g] >> 40) != 0;
        mean += (double)(cyc[g] & ((1ll << 40) - 1));
      }
      mean /= grid;
      // wall_clock64 runs at 100 MHz: ns per chain step
      printf("%-40s grid %5d (%s): %.1f ns per chain, %.2f ns per pivot step%s\n", names[v], grid,
             grid == 1 ? "alone" : grid == 1024 ? "1 wave/SIMD" : "4 waves/SIMD", mean * 10.0 / reps,
             mean * 10.0 / reps / 16, bad ? " BAD PIVOT" : "");
    }
    CK(hipMemcpy(v == 0 ? ref.data() : got.data(), dO, 512 * 256 * 8, hipMemcpyDeviceToHost));
    if (v > 0) {
      double md = 0;
      for (int b = 0; b < 256; ++b)
        for (int q = 0; q < 4; ++q)
          for (int l = 0; l < 64; ++l) {
            const int r = (l >> 4) + 4 * q, c = l & 15;
            if (c > r) continue;   // L / L^-1 are lower triangular (strict upper of A is stale)
            for (int s = 0; s < 2; ++s) {
              const int i = (b * 2 + s) * 256 + q * 64 + l;
              md = fmax(md, fabs(ref[i] - got[i]) / (1.0 + fabs(ref[i])));
            }
          }
      printf("  max rel diff vs library chain: %.3e\n", md);
    }
  }
  return 0;
}
