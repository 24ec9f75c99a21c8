// pf_common.h — device-side helpers shared by the engine's HIP kernels (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PF_WAVE 64

// ---------------------------------------------------------------- wave math
// All cross-lane traffic uses DPP / gfx950 permlane{16,32}_swap (VALU, a few
// cycles) instead of __shfl (ds_bpermute: an LDS-unit round trip per step).
// Callers must have all 64 lanes active.
__device__ __forceinline__ int pf_lane() { return threadIdx.x & 63; }
__device__ __forceinline__ int pf_wave() { return threadIdx.x >> 6; }

// DPP controls (GFX9 encoding)
#define PF_DPP_QXOR1 0xB1    // quad_perm [1,0,3,2]
#define PF_DPP_QXOR2 0x4E    // quad_perm [2,3,0,1]
#define PF_DPP_SHL(n) (0x100 + (n))
#define PF_DPP_SHR(n) (0x110 + (n))
#define PF_DPP_ROR(n) (0x120 + (n))
#define PF_DPP_MIRROR 0x140
#define PF_DPP_HMIRROR 0x141
#define PF_DPP_BCAST15 0x142
#define PF_DPP_BCAST31 0x143

template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ int dpp_i32(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, ROW_MASK, 0xF, true);
}
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(dpp_i32<CTRL, ROW_MASK>(__float_as_int(v)));
}
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ double dpp_f64(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const int lo = dpp_i32<CTRL, ROW_MASK>((int)(unsigned)b);
  const int hi = dpp_i32<CTRL, ROW_MASK>((int)(unsigned)(b >> 32));
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)b, l);
  const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(b >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ float readlane_f32(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// value of lane (lane ^ J), J in {1,2,4,8,16,32}
template <int J>
__device__ __forceinline__ float shfl_xor_f32(float x) {
  if constexpr (J == 1) {
    return dpp_f32<PF_DPP_QXOR1>(x);
  } else if constexpr (J == 2) {
    return dpp_f32<PF_DPP_QXOR2>(x);
  } else if constexpr (J == 4) {
    const float up = dpp_f32<PF_DPP_SHL(4)>(x);   // lane i <- i+4
    const float dn = dpp_f32<PF_DPP_SHR(4)>(x);   // lane i <- i-4
    return (pf_lane() & 4) ? dn : up;
  } else if constexpr (J == 8) {
    return dpp_f32<PF_DPP_ROR(8)>(x);             // within a row of 16: i ^ 8
  } else if constexpr (J == 16) {
    const unsigned u = __float_as_uint(x);
    const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    return __uint_as_float((pf_lane() & 16) ? r[0] : r[1]);
  } else {
    static_assert(J == 32, "xor distance");
    const unsigned u = __float_as_uint(x);
    const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    return __uint_as_float((pf_lane() & 32) ? r[0] : r[1]);
  }
}
template <int J>
__device__ __forceinline__ double shfl_xor_f64(double x) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  const float lo = shfl_xor_f32<J>(__uint_as_float((unsigned)b));
  const float hi = shfl_xor_f32<J>(__uint_as_float((unsigned)(b >> 32)));
  return __longlong_as_double((long long)(((unsigned long long)__float_as_uint(hi) << 32) |
                                          __float_as_uint(lo)));
}

// Pairwise cross-half/cross-row adds: one permlane swap per dword exchanges
// the halves of two registers, so no keep/send selects are needed.
//   pair_add32(a, b): lanes 0..31 -> a_l + a_{l+32}, lanes 32..63 -> b_{l-32} + b_l
//   pair_add16(a, b): rows 0,2 -> a_l + a_{l+16}, rows 1,3 -> b_{l-16} + b_l
__device__ __forceinline__ double pair_add32(double a, double b) {
  const unsigned long long ua = (unsigned long long)__double_as_longlong(a);
  const unsigned long long ub = (unsigned long long)__double_as_longlong(b);
  const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)ua, (unsigned)ub, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
  const double x = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));
  const double y = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));
  return x + y;
}
__device__ __forceinline__ double pair_add16(double a, double b) {
  const unsigned long long ua = (unsigned long long)__double_as_longlong(a);
  const unsigned long long ub = (unsigned long long)__double_as_longlong(b);
  const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)ua, (unsigned)ub, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
  const double x = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));
  const double y = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));
  return x + y;
}

// full-wave sum, result uniform in every lane
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp_f64<PF_DPP_QXOR1>(v);
  v += dpp_f64<PF_DPP_QXOR2>(v);
  v += dpp_f64<PF_DPP_HMIRROR>(v);
  v += dpp_f64<PF_DPP_MIRROR>(v);
  v += dpp_f64<PF_DPP_BCAST15, 0xA>(v);
  v += dpp_f64<PF_DPP_BCAST31, 0xC>(v);
  return readlane_f64(v, 63);
}

__device__ __forceinline__ float wave_minf(float v) {
  v = fminf(v, shfl_xor_f32<1>(v));
  v = fminf(v, shfl_xor_f32<2>(v));
  v = fminf(v, shfl_xor_f32<4>(v));
  v = fminf(v, shfl_xor_f32<8>(v));
  v = fminf(v, shfl_xor_f32<16>(v));
  v = fminf(v, shfl_xor_f32<32>(v));
  return v;
}

// inclusive prefix sum across the wave (lane l gets sum_{l' <= l})
__device__ __forceinline__ double wave_prefix_sum(double v) {
  v += dpp_f64<PF_DPP_SHR(1)>(v);
  v += dpp_f64<PF_DPP_SHR(2)>(v);
  v += dpp_f64<PF_DPP_SHR(4)>(v);
  v += dpp_f64<PF_DPP_SHR(8)>(v);
  v += dpp_f64<PF_DPP_BCAST15, 0xA>(v);
  v += dpp_f64<PF_DPP_BCAST31, 0xC>(v);
  return v;
}

// value of lane l-1 (0 for lane 0): exclusive-scan helper
__device__ __forceinline__ double wave_shift_up1(double v) {
  // wave_shr:1 (0x138) is GFX8/9 only; gfx950 keeps it
  return dpp_f64<0x138>(v);
}

// inclusive suffix sum (lane l gets sum_{l' >= l}); total returned in `tot`
__device__ __forceinline__ double wave_suffix_sum(double v, double &tot) {
  const double p = wave_prefix_sum(v);
  tot = readlane_f64(p, 63);
  return tot - p + v;
}

// Sum N <= 32 independent per-lane values over the wave by recursive halving
// (32 shuffle+add pairs instead of 6*N); out[v] is the uniform total of v.
template <int N>
__device__ __forceinline__ void wave_sum_multi(const double (&v)[N], double (&out)[N]) {
  static_assert(N <= 32, "wave_sum_multi: N <= 32");
  const int lane = pf_lane();
  double w16[16], w8[8], w4[4], w2[2], w1;
  // level xor 32: value pair (2k, 2k+1) -> lanes <32 keep 2k, >=32 keep 2k+1
  // (pairs whose value indices are all >= N are skipped at compile time)
  const bool h3 = lane & 8, h2 = lane & 4, h1 = lane & 2;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (2 * k >= N) { w16[k] = 0.0; continue; }
    const double a = v[2 * k], b = (2 * k + 1 < N) ? v[2 * k + 1] : 0.0;
    w16[k] = pair_add32(a, b);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (4 * k >= N) { w8[k] = 0.0; continue; }
    w8[k] = pair_add16(w16[2 * k], w16[2 * k + 1]);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (8 * k >= N) { w4[k] = 0.0; continue; }
    const double keep = h3 ? w8[2 * k + 1] : w8[2 * k], send = h3 ? w8[2 * k] : w8[2 * k + 1];
    w4[k] = keep + shfl_xor_f64<8>(send);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    if (16 * k >= N) { w2[k] = 0.0; continue; }
    const double keep = h2 ? w4[2 * k + 1] : w4[2 * k], send = h2 ? w4[2 * k] : w4[2 * k + 1];
    w2[k] = keep + shfl_xor_f64<4>(send);
  }
  {
    const double keep = h1 ? w2[1] : w2[0], send = h1 ? w2[0] : w2[1];
    w1 = keep + shfl_xor_f64<2>(send);
  }
  w1 += shfl_xor_f64<1>(w1);
  // value index held by lane l: bit0 <- lane bit5, bit1 <- bit4, ... bit4 <- bit1
#pragma unroll
  for (int idx = 0; idx < N; ++idx) {
    const int l = ((idx & 1) << 5) | (((idx >> 1) & 1) << 4) | (((idx >> 2) & 1) << 3) |
                  (((idx >> 3) & 1) << 2) | (((idx >> 4) & 1) << 1);
    out[idx] = readlane_f64(w1, l);
  }
}

// Transposed wave reduction of N <= 64 per-lane values by recursive halving
// (about N shuffle+add pairs instead of 6 per value).  Returns, in every
// lane, the wave total of value index transpose_index<N>(lane); for N <= 32
// the two lanes of each (2k, 2k+1) pair hold the same total.
template <int N>
__device__ __forceinline__ int transpose_index(int lane) {
  if constexpr (N <= 32)
    return ((lane >> 5) & 1) | (((lane >> 4) & 1) << 1) | (((lane >> 3) & 1) << 2) |
           (((lane >> 2) & 1) << 3) | (((lane >> 1) & 1) << 4);
  else
    return ((lane >> 5) & 1) | (((lane >> 4) & 1) << 1) | (((lane >> 3) & 1) << 2) |
           (((lane >> 2) & 1) << 3) | (((lane >> 1) & 1) << 4) | ((lane & 1) << 5);
}
template <int M, int D, int N>
__device__ __forceinline__ void transpose_level(const double (&w)[M], double (&o)[M / 2]) {
  const bool h = pf_lane() & D;
  constexpr int SPAN = (M == 64) ? 1 : 32 / M;  // value indices per input entry
#pragma unroll
  for (int k = 0; k < M / 2; ++k) {
    // value indices carried by w[2k], w[2k+1] are all >= N: compile-time zero
    if (2 * k * SPAN >= N) { o[k] = 0.0; continue; }
    const double a = w[2 * k], b = w[2 * k + 1];
    if constexpr (D == 32) {
      o[k] = pair_add32(a, b);
    } else if constexpr (D == 16) {
      o[k] = pair_add16(a, b);
    } else {
      const double keep = h ? b : a, send = h ? a : b;
      o[k] = keep + shfl_xor_f64<D>(send);
    }
  }
}
template <int N>
__device__ __forceinline__ double wave_transpose_sum(const double (&v)[N]) {
  static_assert(N >= 1 && N <= 64, "wave_transpose_sum: 1 <= N <= 64");
  if constexpr (N <= 32) {
    double w32[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) w32[i] = (i < N) ? v[i] : 0.0;
    double w16[16], w8[8], w4[4], w2[2], w1[1];
    transpose_level<32, 32, N>(w32, w16);
    transpose_level<16, 16, N>(w16, w8);
    transpose_level<8, 8, N>(w8, w4);
    transpose_level<4, 4, N>(w4, w2);
    transpose_level<2, 2, N>(w2, w1);
    return w1[0] + shfl_xor_f64<1>(w1[0]);
  } else {
    double w64[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) w64[i] = (i < N) ? v[i] : 0.0;
    double w32[32], w16[16], w8[8], w4[4], w2[2], w1[1];
    transpose_level<64, 32, N>(w64, w32);
    transpose_level<32, 16, N>(w32, w16);
    transpose_level<16, 8, N>(w16, w8);
    transpose_level<8, 4, N>(w8, w4);
    transpose_level<4, 2, N>(w4, w2);
    transpose_level<2, 1, N>(w2, w1);
    return w1[0];
  }
}

// ---------------------------------------------------------------- Philox4x32-10
struct pf_u4 { uint32_t x, y, z, w; };

__device__ __forceinline__ pf_u4 philox4x32_10(pf_u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = pf_u4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// uniform in (0,1) from 24 random bits (never 0, never 1)
__device__ __forceinline__ float pf_u01f(uint32_t x) {
  return ((float)(x >> 8) + 0.5f) * (1.0f / 16777216.0f);
}
// uniform in (0,1) in double from 53 bits of two words
__device__ __forceinline__ double pf_u01d(uint32_t a, uint32_t b) {
  const uint64_t v = ((uint64_t)a << 21) ^ (uint64_t)(b >> 11);
  return ((double)(v & ((1ull << 53) - 1)) + 0.5) * (1.0 / 9007199254740992.0);
}

// Box-Muller: two normals from two uniforms (v_sin/v_cos take revolutions).
// -2 ln u1 = -2 ln2 log2 u1 on the hardware log2 and sqrt (v_log_f32,
// v_sqrt_f32, ~1 ulp): pf_u01f's uniforms are >= 2^-25, never denormal, so
// the library forms' denormal scaling and ln2 extension (~17 instructions
// per pair) buy nothing here.
__device__ __forceinline__ void pf_box_muller(float u1, float u2, float &z0, float &z1) {
  const float r = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));
  z0 = r * __builtin_amdgcn_cosf(u2);
  z1 = r * __builtin_amdgcn_sinf(u2);
}

// ---------------------------------------------------------------- bitonic sort across a wave (1 value / lane, ascending)
template <int J>
__device__ __forceinline__ float bitonic_step(float x, bool up) {
  const float p = shfl_xor_f32<J>(x);
  const bool lower = (pf_lane() & J) == 0;
  return (lower == up) ? fminf(x, p) : fmaxf(x, p);
}
template <int K>
__device__ __forceinline__ float bitonic_merge(float x) {
  const bool up = (pf_lane() & K) == 0 || K == 64;
  if constexpr (K >= 64) x = bitonic_step<32>(x, up);
  if constexpr (K >= 32) x = bitonic_step<16>(x, up);
  if constexpr (K >= 16) x = bitonic_step<8>(x, up);
  if constexpr (K >= 8) x = bitonic_step<4>(x, up);
  if constexpr (K >= 4) x = bitonic_step<2>(x, up);
  x = bitonic_step<1>(x, up);
  return x;
}
__device__ __forceinline__ float wave_bitonic_sort_asc(float x) {
  x = bitonic_merge<2>(x);
  x = bitonic_merge<4>(x);
  x = bitonic_merge<8>(x);
  x = bitonic_merge<16>(x);
  x = bitonic_merge<32>(x);
  x = bitonic_merge<64>(x);
  return x;
}

__device__ __forceinline__ uint32_t pf_f2ord(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float pf_ord2f(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
}

// uniform pointer (both halves from the first active lane: kept in SGPRs)
__device__ __forceinline__ const void *rfl_ptr(const void *p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (const void *)(((uint64_t)hi << 32) | lo);
}
