// Microbenchmarks that calibrate the roofline peaks used by bench.py on gfx950:
//  (1) v_mfma_f64_16x16x4_f64 operand/result lane maps (exact integer check),
//  (2) FP64 MFMA and FP64 VALU FMA peak rate (one workgroup per CU, 4 waves),
//  (3) HBM streaming read bandwidth (16 B per lane loads, 1 GiB buffer).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef double f64x4 __attribute__((ext_vector_type(4)));

// A is 16x4 (row-major), B is 4x16 (row-major). Guide: A[i=l&15][k=l>>4], B[k=l>>4][j=l&15],
// C/D col=lane&15, row=(lane>>4)+4*reg.
__global__ void mfma_layout(const double* A, const double* B, double* C) {
  int l = threadIdx.x;
  double a = A[(l & 15) * 4 + (l >> 4)];
  double b = B[(l >> 4) * 16 + (l & 15)];
  f64x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) C[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
}

__global__ __launch_bounds__(256) void mfma_rate(double* out, int iters) {
  double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
  f64x4 c0 = {0,0,0,0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  double s = 0; for (int r = 0; r < 4; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  if (s == 12345.0) out[0] = s;
}

__global__ __launch_bounds__(256) void valu_rate(double* out, int iters) {
  double x[8]; for (int j = 0; j < 8; ++j) x[j] = threadIdx.x + j;
  double a = 1.0000001, b = 1e-9;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = fma(x[j], a, b);
  }
  double s = 0; for (int j = 0; j < 8; ++j) s += x[j];
  if (s == 12345.0) out[0] = s;
}

__global__ __launch_bounds__(256) void stream_read(const double2* __restrict__ p, size_t n2, double* out) {
  double acc = 0;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += stride) {
    double2 v = p[i]; acc += v.x + v.y;
  }
  if (acc == 12345.0) out[0] = acc;
}

int main() {
  // (1) layout
  std::vector<double> A(64), B(64), C(256), R(256, 0.0);
  srand(7);
  for (int i = 0; i < 64; ++i) { A[i] = rand() % 7 - 3; B[i] = rand() % 5 - 2; }
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) for (int k = 0; k < 4; ++k) R[i*16+j] += A[i*4+k] * B[k*16+j];
  double *dA, *dB, *dC, *dout; CK(hipMalloc(&dA, 512)); CK(hipMalloc(&dB, 512)); CK(hipMalloc(&dC, 2048)); CK(hipMalloc(&dout, 64));
  CK(hipMemcpy(dA, A.data(), 512, hipMemcpyHostToDevice)); CK(hipMemcpy(dB, B.data(), 512, hipMemcpyHostToDevice));
  mfma_layout<<<1, 64>>>(dA, dB, dC); CK(hipDeviceSynchronize());
  CK(hipMemcpy(C.data(), dC, 2048, hipMemcpyDeviceToHost));
  int bad = 0; for (int i = 0; i < 256; ++i) bad += (C[i] != R[i]);
  printf("{\"mfma_f64_layout_mismatches\": %d}\n", bad);

  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); float ms;
  int ncu = 256; hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0)); ncu = prop.multiProcessorCount;
  // (2) MFMA rate: grid = 2 blocks per CU
  for (int rep = 0; rep < 2; ++rep) {
    int iters = 20000, grid = ncu * 2;
    mfma_rate<<<grid, 256>>>(dout, 100); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); mfma_rate<<<grid, 256>>>(dout, iters); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    double fl = (double)grid * 4 /*waves*/ * iters * 4 * 2048.0;
    printf("{\"mfma_f64_tflops\": %.2f, \"ms\": %.3f}\n", fl / (ms * 1e-3) / 1e12, ms);
    CK(hipEventRecord(e0)); valu_rate<<<grid, 256>>>(dout, iters); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    fl = (double)grid * 256 * iters * 8 * 2.0;
    printf("{\"valu_f64_tflops\": %.2f, \"ms\": %.3f}\n", fl / (ms * 1e-3) / 1e12, ms);
  }
  // (3) stream
  size_t bytes = (size_t)1 << 30; double2* p; CK(hipMalloc(&p, bytes)); CK(hipMemset(p, 0, bytes));
  for (int g : {ncu * 4, ncu * 8, ncu * 16}) {
    stream_read<<<g, 256>>>(p, bytes / 16, dout); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) stream_read<<<g, 256>>>(p, bytes / 16, dout);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"stream_read_GBps\": %.1f, \"grid\": %d}\n", 5.0 * bytes / (ms * 1e-3) / 1e9, g);
  }
  printf("{\"cus\": %d, \"clock_khz\": %d}\n", ncu, prop.clockRate);
  return 0;
}
