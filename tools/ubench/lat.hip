// Latency microbenchmark (dev tool): one wave, s_memtime around dependent
// chains of the primitives the fit's serial path is built from.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "pf_common.h"
#define N 64
// timer read ordered after `x` is ready (v_mov issue interlocks on it) and
// the chain that follows ordered after the read ("+v" makes x an output)
__device__ __forceinline__ unsigned long long tick(double &x) {
  unsigned long long t;
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
  asm volatile("v_mov_b32 %1, %1\n v_mov_b32 %2, %2\n s_memtime %0\n s_waitcnt lgkmcnt(0)"
               : "=s"(t), "+v"(lo), "+v"(hi) : : "memory");
  x = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
  return t;
}
__global__ void k_lat(double *out, unsigned long long *cyc, const double *in) {
  __shared__ double lds[256];
  const int lane = threadIdx.x;
  double x = in[lane], y = in[lane + 64];
  lds[lane] = x; lds[lane + 64] = y;
  __syncthreads();
  unsigned long long t0, t1;
  // 1: dependent fma chain
  t0 = tick(x);
  for (int i = 0; i < N; ++i) x = fma(x, y, 0.5);
  t1 = tick(x); if (lane == 0) cyc[0] = t1 - t0;
  // 2: wave_sum chain
  t0 = tick(x);
  for (int i = 0; i < N; ++i) x = wave_sum(x * 1e-3) + y;
  t1 = tick(x); if (lane == 0) cyc[1] = t1 - t0;
  // 3: LDS read chain (address depends on value)
  int idx = lane;
  t0 = tick(x);
  for (int i = 0; i < N; ++i) { const double v = lds[idx]; idx = ((int)v & 63) ^ lane; x += v; }
  t1 = tick(x); if (lane == 0) cyc[2] = t1 - t0;
  // 4: division chain
  t0 = tick(x);
  for (int i = 0; i < N; ++i) x = 1.0 / (x + 2.0);
  t1 = tick(x); if (lane == 0) cyc[3] = t1 - t0;
  // 5: readlane -> valu chain
  t0 = tick(x);
  for (int i = 0; i < N; ++i) x = readlane_f64(x, (i * 7) & 63) * 0.999 + y;
  t1 = tick(x); if (lane == 0) cyc[4] = t1 - t0;
  // 6: one DPP f64 step chain (row_shr:1)
  t0 = tick(x);
  for (int i = 0; i < N; ++i) x = x + dpp_f64<PF_DPP_SHR(1)>(x) * 0.5;
  t1 = tick(x); if (lane == 0) cyc[5] = t1 - t0;
  // 7: permlane32 f64 xor step chain
  t0 = tick(x);
  for (int i = 0; i < N; ++i) x = x + shfl_xor_f64<32>(x) * 0.5;
  t1 = tick(x); if (lane == 0) cyc[6] = t1 - t0;
  // 7b/7c: xor-16 (permlane16_swap) and xor-8 (DPP ror) f64 steps
  t0 = tick(x);
  for (int i = 0; i < N; ++i) x = x + shfl_xor_f64<16>(x) * 0.5;
  t1 = tick(x); if (lane == 0) cyc[13] = t1 - t0;
  t0 = tick(x);
  for (int i = 0; i < N; ++i) x = x + shfl_xor_f64<8>(x) * 0.5;
  t1 = tick(x); if (lane == 0) cyc[14] = t1 - t0;
  t0 = tick(x);
  for (int i = 0; i < N; ++i) x = x + shfl_xor_f64<4>(x) * 0.5;
  t1 = tick(x); if (lane == 0) cyc[15] = t1 - t0;
  // 8: ds_bpermute (__shfl) chain
  t0 = tick(x);
  for (int i = 0; i < N; ++i) x = __shfl(x, (lane + 5) & 63, 64) * 0.5 + y;
  t1 = tick(x); if (lane == 0) cyc[7] = t1 - t0;
  // 9: independent fma throughput (8 chains)
  double c[8];
  t0 = tick(x);
  for (int j = 0; j < 8; ++j) c[j] = x + j;
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = fma(c[j], y, 0.5);
  { double cc = c[0] + c[7]; t1 = tick(cc); x += cc; } if (lane == 0) cyc[8] = t1 - t0;
  for (int j = 0; j < 8; ++j) x += c[j];
  // 10: wave_sum_multi<22>
  double v[22], r[22];
  for (int j = 0; j < 22; ++j) v[j] = x * (j + 1);
  t0 = tick(x);
  for (int i = 0; i < 8; ++i) { wave_sum_multi<22>(v, r); v[0] = r[21] * 1e-9 + v[1]; }
  x += v[0];
  t1 = tick(x); if (lane == 0) cyc[9] = (t1 - t0) * N / 8;
  // 11: exp / log / sqrt chains
  t0 = tick(x);
  for (int i = 0; i < N; ++i) x = exp(x * 1e-3);
  t1 = tick(x); if (lane == 0) cyc[10] = t1 - t0;
  t0 = tick(x);
  for (int i = 0; i < N; ++i) x = sqrt(x + 1.0);
  t1 = tick(x); if (lane == 0) cyc[11] = t1 - t0;
  // 12: s_barrier alone (1 wave)
  t0 = tick(x);
  for (int i = 0; i < N; ++i) __syncthreads();
  t1 = tick(x); if (lane == 0) cyc[12] = t1 - t0;
  // 13: f64 MFMA 16x16x4, dependent (same accumulator) and 4 independent chains
  {
    typedef double d4 __attribute__((ext_vector_type(4)));
    d4 acc = d4{x, y, x, y}, a1 = acc, a2 = acc, a3 = acc;
    t0 = tick(x);
    for (int i = 0; i < N; ++i) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0);
    double s = acc[0] + acc[3];
    t1 = tick(s); if (lane == 0) cyc[16] = t1 - t0;
    x += s * 1e-30;
    t0 = tick(x);
    for (int i = 0; i < N; ++i) {
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, x, a1, 0, 0, 0);
      a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, a2, 0, 0, 0);
      a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, y, a3, 0, 0, 0);
    }
    s = acc[0] + a1[1] + a2[2] + a3[3];
    t1 = tick(s); if (lane == 0) cyc[17] = t1 - t0;
    x += s * 1e-30;
  }
  out[lane] = x;
}
int main() {
  double *out, *in; unsigned long long *cyc;
  hipMalloc(&out, 64 * 8); hipMalloc(&in, 128 * 8); hipMalloc(&cyc, 18 * 8);
  double h[128]; for (int i = 0; i < 128; ++i) h[i] = 1.0 + i * 1e-3;
  hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, out, cyc, in);
  unsigned long long c[18]; (void)hipMemcpy(c, cyc, sizeof(c[0]) * 18, hipMemcpyDeviceToHost);
  const char *nm[] = {"fma_f64 dep", "wave_sum f64", "lds read dep", "div f64", "readlane f64 -> valu",
                      "dpp row_shr f64 step", "permlane32 f64 step", "ds_bpermute f64", "fma_f64 8 indep chains (per iter)",
                      "wave_sum_multi<22>", "exp f64", "sqrt f64", "s_barrier (1 wave)",
                      "xor16 (permlane16_swap) f64 step", "xor8 (dpp ror) f64 step", "xor4 (dpp shl/shr+sel) f64 step",
                      "mfma f64 16x16x4 dependent", "mfma f64 16x16x4 x4 indep (per iter)"};
  for (int i = 0; i < 18; ++i) printf("%-34s %8.1f cycles/op\n", nm[i], (double)c[i] / N);
  return 0;
}
