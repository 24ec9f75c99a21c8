// pf_ostat.h — exact order-statistic sampling for the forecast intervals.
//
// UPSTREAM predict_uncertainty (called from 02_training.py:205 and
// model_wrapper.py:61) draws N predictive samples per row and takes
// np.nanpercentile(·, 2.5 / 97.5) with linear interpolation, i.e. a lerp of
// the sorted samples at positions (k_lo, k_lo+1) and (k_hi, k_hi+1).
// On every row whose trend is deterministic (t <= 1, flat growth: the
// history), the samples are yhat + sd·z_i with z_i iid N(0,1), so the
// interval endpoints are yhat + sd·lerp(z_(k), z_(k+1)).  The joint law of
// the four needed normal order statistics is drawn EXACTLY (not
// approximated) from uniform spacings (Rényi):  with G_0..G_m independent
// Gamma(r_0), Gamma(r_1 - r_0), ..., Gamma(N + 1 - r_{m-1}),
//     U_(r_i) = (G_0 + ... + G_i) / (G_0 + ... + G_m),
//     z_(r_i) = Φ^{-1}(U_(r_i))          (Wichura AS241, |rel err| ~ 1e-16).
// (Computed in single precision by default — the fp32 outputs cannot
// resolve the difference; -DPF_OSTAT_F64 selects the fp64 routines.)
// The output therefore has the same distribution as the N-sample estimate
// (rows independent of each other and of the future rows, as in the
// reference), at O(1) work per row instead of O(N).
#pragma once
#include "pf_common.h"

// Wichura (1988) AS241 PPND16: Φ^{-1}(p) given p and q = 1 - p (both
// accurate, so the upper tail does not lose digits to 1 - p).
__device__ __forceinline__ double pf_ppnd16(double p, double q) {
  const double d = p - 0.5;
  if (fabs(d) <= 0.425) {
    const double r = 0.180625 - d * d;
    const double num = (((((((2.5090809287301226727e+3 * r + 3.3430575583588128105e+4) * r +
                             6.7265770927008700853e+4) * r + 4.5921953931549871457e+4) * r +
                           1.3731693765509461125e+4) * r + 1.9715909503065514427e+3) * r +
                         1.3314166789178437745e+2) * r + 3.3871328727963666080e0);
    const double den = (((((((5.2264952788528545610e+3 * r + 2.8729085735721942674e+4) * r +
                             3.9307895800092710610e+4) * r + 2.1213794301586595867e+4) * r +
                           5.3941960214247511077e+3) * r + 6.8718700749205790830e+2) * r +
                         4.2313330701600911252e+1) * r + 1.0);
    return d * num / den;
  }
  double r = sqrt(-log(fmin(p, q)));
  double v;
  if (r <= 5.0) {
    r -= 1.6;
    const double num = (((((((7.74545014278341407640e-4 * r + 2.27238449892691845833e-2) * r +
                             2.41780725177450611770e-1) * r + 1.27045825245236838258e0) * r +
                           3.64784832476320460504e0) * r + 5.76949722146069140550e0) * r +
                         4.63033784615654529590e0) * r + 1.42343711074968357734e0);
    const double den = (((((((1.05075007164441684324e-9 * r + 5.47593808499534494600e-4) * r +
                             1.51986665636164571966e-2) * r + 1.48103976427480074590e-1) * r +
                           6.89767334985100004550e-1) * r + 1.67638483018380384940e0) * r +
                         2.05319162663775882187e0) * r + 1.0);
    v = num / den;
  } else {
    r -= 5.0;
    const double num = (((((((2.01033439929228813265e-7 * r + 2.71155556874348757815e-5) * r +
                             1.24266094738807843860e-3) * r + 2.65321895265761230930e-2) * r +
                           2.96560571828504891230e-1) * r + 1.78482653991729133580e0) * r +
                         5.46378491116411436990e0) * r + 6.65790464350110377720e0);
    const double den = (((((((2.04426310338993978564e-15 * r + 1.42151175831644588870e-7) * r +
                             1.84631831751005468180e-5) * r + 7.86869131145613259100e-4) * r +
                           1.48753612908506148525e-2) * r + 1.36929880922735805310e-1) * r +
                         5.99832206555887937690e-1) * r + 1.0);
    v = num / den;
  }
  return d < 0.0 ? -v : v;
}

// Counter-based stream for one row: every call consumes one Philox block.
struct pf_rowrng {
  uint32_t row, sid, k0, k1, ctr;
  __device__ __forceinline__ pf_u4 next() {
    return philox4x32_10(pf_u4{row, 0x05A70000u + (ctr++), sid, 0x0DD5EEDu}, k0, k1);
  }
};

// Gamma(alpha, 1) for integer-valued alpha >= 1: Exp(1) by inversion when
// alpha == 1, Marsaglia–Tsang (2000) squeeze/rejection otherwise.
__device__ __noinline__ double pf_gamma(double alpha, pf_rowrng &rng) {
  if (alpha <= 1.0) {
    const pf_u4 r = rng.next();
    return -log(pf_u01d(r.x, r.y));
  }
  const double dd = alpha - 1.0 / 3.0;
  const double c = 1.0 / sqrt(9.0 * dd);
  for (int it = 0; it < 64; ++it) {
    const pf_u4 ra = rng.next();
    const pf_u4 rb = rng.next();
    // two normals (Box–Muller, fp64), two acceptance uniforms
    const double u1 = pf_u01d(ra.x, ra.y), u2 = pf_u01d(ra.z, ra.w);
    const double rad = sqrt(-2.0 * log(u1));
    double sn, cs;
    sincospi(2.0 * u2, &sn, &cs);
    const double xs[2] = {rad * cs, rad * sn};
    const double us[2] = {pf_u01d(rb.x, rb.y), pf_u01d(rb.z, rb.w)};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const double x = xs[h];
      double v = 1.0 + c * x;
      if (v <= 0.0) continue;
      v = v * v * v;
      const double u = us[h];
      const double x2 = x * x;
      if (u < 1.0 - 0.0331 * x2 * x2) return dd * v;
      if (log(u) < 0.5 * x2 + dd * (1.0 - v + log(v))) return dd * v;
    }
  }
  return dd;  // unreachable in practice (acceptance >= 95% per proposal)
}

// ---- single-precision arithmetic for the same exact law (the default):
// the interval endpoints are fp32 outputs, and the fp32 draw moves an
// endpoint by ~1e-7 sd, far below their Monte-Carlo spread; hardware
// v_log_f32 / v_sqrt_f32 / v_sin_f32 instead of the fp64 software routines.
__device__ __forceinline__ float pf_ppnd16f(float p, float q) {
  const float d = p - 0.5f;
  if (fabsf(d) <= 0.425f) {
    const float r = 0.180625f - d * d;
    const float num = (((((((2.5090809287301226727e+3f * r + 3.3430575583588128105e+4f) * r +
                            6.7265770927008700853e+4f) * r + 4.5921953931549871457e+4f) * r +
                          1.3731693765509461125e+4f) * r + 1.9715909503065514427e+3f) * r +
                        1.3314166789178437745e+2f) * r + 3.3871328727963666080e0f);
    const float den = (((((((5.2264952788528545610e+3f * r + 2.8729085735721942674e+4f) * r +
                            3.9307895800092710610e+4f) * r + 2.1213794301586595867e+4f) * r +
                          5.3941960214247511077e+3f) * r + 6.8718700749205790830e+2f) * r +
                        4.2313330701600911252e+1f) * r + 1.0f);
    return d * num / den;
  }
  float r = sqrtf(-logf(fminf(p, q)));
  float v;
  if (r <= 5.0f) {
    r -= 1.6f;
    const float num = (((((((7.74545014278341407640e-4f * r + 2.27238449892691845833e-2f) * r +
                            2.41780725177450611770e-1f) * r + 1.27045825245236838258e0f) * r +
                          3.64784832476320460504e0f) * r + 5.76949722146069140550e0f) * r +
                        4.63033784615654529590e0f) * r + 1.42343711074968357734e0f);
    const float den = (((((((1.05075007164441684324e-9f * r + 5.47593808499534494600e-4f) * r +
                            1.51986665636164571966e-2f) * r + 1.48103976427480074590e-1f) * r +
                          6.89767334985100004550e-1f) * r + 1.67638483018380384940e0f) * r +
                        2.05319162663775882187e0f) * r + 1.0f);
    v = num / den;
  } else {
    r -= 5.0f;
    const float num = (((((((2.01033439929228813265e-7f * r + 2.71155556874348757815e-5f) * r +
                            1.24266094738807843860e-3f) * r + 2.65321895265761230930e-2f) * r +
                          2.96560571828504891230e-1f) * r + 1.78482653991729133580e0f) * r +
                        5.46378491116411436990e0f) * r + 6.65790464350110377720e0f);
    const float den = (((((((2.04426310338993978564e-15f * r + 1.42151175831644588870e-7f) * r +
                            1.84631831751005468180e-5f) * r + 7.86869131145613259100e-4f) * r +
                          1.48753612908506148525e-2f) * r + 1.36929880922735805310e-1f) * r +
                        5.99832206555887937690e-1f) * r + 1.0f);
    v = num / den;
  }
  return d < 0.0f ? -v : v;
}

// Gamma(alpha, 1), integer-valued alpha >= 1, single precision: Exp(1) by
// inversion when alpha == 1, Marsaglia–Tsang otherwise (one Philox block
// per two proposals: Box–Muller pair + two acceptance uniforms)
__device__ __forceinline__ float pf_gamma_f(float alpha, pf_rowrng &rng) {
  if (alpha <= 1.0f) {
    const pf_u4 r = rng.next();
    return -logf(pf_u01f(r.x));
  }
  const float dd = alpha - 1.0f / 3.0f;
  const float c = 1.0f / sqrtf(9.0f * dd);
  for (int it = 0; it < 64; ++it) {
    const pf_u4 ra = rng.next();
    const float rad = sqrtf(-2.0f * logf(pf_u01f(ra.x)));
    float sn, cs;
    sincospif(2.0f * pf_u01f(ra.y), &sn, &cs);
    const float xs[2] = {rad * cs, rad * sn};
    const float us[2] = {pf_u01f(ra.z), pf_u01f(ra.w)};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float x = xs[h];
      float v = 1.0f + c * x;
      if (v <= 0.0f) continue;
      v = v * v * v;
      const float u = us[h];
      const float x2 = x * x;
      if (u < 1.0f - 0.0331f * x2 * x2) return dd * v;
      if (logf(u) < 0.5f * x2 + dd * (1.0f - v + logf(v))) return dd * v;
    }
  }
  return dd;  // unreachable in practice (acceptance >= 95% per proposal)
}

// Exact joint draw of the standard-normal order statistics of ranks
// (1-indexed, 1 <= r <= N) r[0..3] out of N samples; r need not be
// distinct or sorted.  Equal ranks give a zero-length spacing (G = 0).
__device__ __forceinline__ void pf_normal_order_stats(const int (&r)[4], int N, pf_rowrng &rng,
                                                      double (&z)[4]) {
  // sort the four ranks (5-comparator network, static indices)
  int s[4] = {r[0], r[1], r[2], r[3]};
#define PF_CSWAP(i, j) { const int lo_ = min(s[i], s[j]), hi_ = max(s[i], s[j]); s[i] = lo_; s[j] = hi_; }
  PF_CSWAP(0, 1) PF_CSWAP(2, 3) PF_CSWAP(0, 2) PF_CSWAP(1, 3) PF_CSWAP(1, 2)
#undef PF_CSWAP
  double G[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int shape = (i < 4 ? s[i] : N + 1) - (i > 0 ? s[i - 1] : 0);
#ifdef PF_OSTAT_F64
    G[i] = shape > 0 ? pf_gamma((double)shape, rng) : 0.0;
#else
    G[i] = shape > 0 ? (double)pf_gamma_f((float)shape, rng) : 0.0;
#endif
  }
  double zs[4];
  double pre = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    pre += G[i];
    double suf = 0.0;
#pragma unroll
    for (int j = i + 1; j < 5; ++j) suf += G[j];
    const double tot = pre + suf;
#ifdef PF_OSTAT_F64
    zs[i] = pf_ppnd16(pre / tot, suf / tot);
#else
    zs[i] = (double)pf_ppnd16f((float)(pre / tot), (float)(suf / tot));
#endif
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double v = zs[0];
#pragma unroll
    for (int i = 1; i < 4; ++i)
      if (s[i] == r[j]) v = zs[i];
    z[j] = v;
  }
}
