// pf_cv.h — K6: batched cross-validation metrics.
//
// Replaces UPSTREAM diagnostics.performance_metrics(rolling_window=0.1) +
// the notebook's per-metric mean over horizons (02_training.py:178-188).
// Rows of one series are the concatenated CV fold predictions, pre-sorted by
// horizon so that equal-horizon rows are contiguous (the host computes that
// permutation once per bucket: every series of a bucket shares the dates).
//
// One wave per series.  Lane g sums the rows of horizon groups g, g+64, ...
// into LDS; then lanes 0..5 run UPSTREAM rolling_mean_by_h's backward sweep
// for one metric each (the sweep's control flow depends only on the shared
// group counts, so the six lanes never diverge).  Included by pf_engine.hip.
#pragma once

#define PF_CV_GMAX 512

struct CvKArgs {
  int n_series, n_rows, n_groups, window, ld_y, ld_f, skip_mdape;
  const int32_t *group_start;
  const double *y;
  const float *yhat, *ylo, *yhi;
  double *metrics;
};

// k-th smallest (0-based) of n non-negative doubles by MSB-first radix
// select on their bit patterns (monotone for x >= 0, +inf included): 8
// passes of an 8-bit LDS histogram.  keys: LDS cache of the bits (n <= ncache)
// or NULL to recompute from y / yh.  One wave; every lane returns the value.
__device__ __forceinline__ double cv_radix_select(const unsigned long long *keys, int n, int k,
                                                  const double *y, const float *yh, int *hist) {
  const int lane = pf_lane();
  unsigned long long prefix = 0ull, mask = 0ull;
  for (int pass = 7; pass >= 0; --pass) {
    const int sh = 8 * pass;
    for (int b = lane; b < 256; b += 64) hist[b] = 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (int r = lane; r < n; r += 64) {
      const unsigned long long key = keys ? keys[r]
          : (unsigned long long)__double_as_longlong(fabs((y[r] - (double)yh[r]) / y[r]));
      if ((key & mask) == prefix) atomicAdd(&hist[(int)((key >> sh) & 255ull)], 1);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    int c[4], lsum = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) { c[q] = hist[4 * lane + q]; lsum += c[q]; }
    const double incl = wave_prefix_sum((double)lsum);
    const double excl = incl - (double)lsum;
    const unsigned long long hit = __ballot(incl > (double)k);
    const int L = __ffsll((long long)hit) - 1;
    int bsel = 0, below = 0;
    if (lane == L) {
      int acc = (int)excl;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (acc + c[q] > k) { bsel = 4 * lane + q; below = acc; break; }
        acc += c[q];
      }
    }
    bsel = __shfl(bsel, L, 64);
    below = __shfl(below, L, 64);
    prefix |= (unsigned long long)bsel << sh;
    mask |= 255ull << sh;
    k -= below;
  }
  return __longlong_as_double((long long)prefix);
}

// One horizon group holding every row (in-sample metrics: rolling_mean_by_h
// with w = n is the plain mean, rolling_median_by_h the median): a block of
// PF_CV_INS_WAVES waves per series strides over the rows (four independent
// row loads in flight per thread), each wave reduces its sums, and wave 0 adds
// the wave totals in a fixed order; the MDAPE median comes from two radix
// selects (ranks (n-1)/2 and n/2) over the APE bit patterns cached in LDS.
#define PF_CV_INS_WAVES 4
#define PF_CV_INS_CACHE 3072
// One series' in-sample metrics by a block of PF_CV_INS_WAVES waves.  LDS:
// s_cache [PF_CV_INS_CACHE] (MDAPE only), s_part [PF_CV_INS_WAVES][6],
// s_hist [256], s_bad [1].  Waves other than 0 return after the block
// barrier.  Shared by k_cv_insample and the fused forecast epilogue.
__device__ __forceinline__ void cv_insample_block(const CvKArgs &a, int series, unsigned long long *s_cache,
                                                  double (*s_part)[6], int *s_hist, int *s_bad_) {
  int &s_bad = *s_bad_;
  constexpr int NT = PF_CV_INS_WAVES * 64;
  const int lane = pf_lane(), wave = pf_wave(), tid = threadIdx.x;
  const double *y = a.y + (size_t)series * a.ld_y;
  const float *yh = a.yhat + (size_t)series * a.ld_f;
  const float *lo = a.ylo ? a.ylo + (size_t)series * a.ld_f : nullptr;
  const float *hi = a.yhi ? a.yhi + (size_t)series * a.ld_f : nullptr;
  const int n = a.n_rows;
  const bool cached = n <= PF_CV_INS_CACHE;
  if (tid == 0) s_bad = 0;
  double se = 0.0, ae = 0.0, ape = 0.0, sape = 0.0, cov = 0.0, ymin = INFINITY;
  bool bad = false;
  for (int r0 = tid; r0 < n; r0 += 4 * NT) {
    double yv[4], fv[4];
    bool in[4], ci[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = r0 + u * NT;
      in[u] = r < n;
      yv[u] = in[u] ? y[r] : 1.0;
      fv[u] = in[u] ? (double)yh[r] : 1.0;
      ci[u] = in[u] && lo && (yv[u] >= (double)lo[r] && yv[u] <= (double)hi[r]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (!in[u]) continue;
      const double e = yv[u] - fv[u];
      se = fma(e, e, se);
      ae += fabs(e);
      const double q = fabs(e / yv[u]);
      ape += q;
      sape += 2.0 * fabs(e) / (fabs(yv[u]) + fabs(fv[u]));
      cov += ci[u] ? 1.0 : 0.0;
      ymin = fmin(ymin, fabs(yv[u]));
      if (!a.skip_mdape) {
        bad |= (q != q);
        if (cached) s_cache[r0 + u * NT] = (unsigned long long)__double_as_longlong(q);
      }
    }
  }
  se = wave_sum(se);
  ae = wave_sum(ae);
  ape = wave_sum(ape);
  sape = wave_sum(sape);
  cov = wave_sum(cov);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) ymin = fmin(ymin, __shfl_xor(ymin, o, 64));
  if (lane == 0) {
    s_part[wave][0] = se;
    s_part[wave][1] = ae;
    s_part[wave][2] = ape;
    s_part[wave][3] = sape;
    s_part[wave][4] = cov;
    s_part[wave][5] = ymin;
  }
  if (__ballot(bad) != 0ull && lane == 0) s_bad = 1;
  __syncthreads();
  if (wave != 0) return;   // no block-level sync below
  double t[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  double tmin = INFINITY;
#pragma unroll
  for (int w = 0; w < PF_CV_INS_WAVES; ++w) {
#pragma unroll
    for (int k = 0; k < 5; ++k) t[k] += s_part[w][k];
    tmin = fmin(tmin, s_part[w][5]);
  }
  const bool anybad = s_bad != 0;
  double v0 = NAN, v1 = NAN;
  if (!anybad && !a.skip_mdape) {
    v0 = cv_radix_select(cached ? s_cache : nullptr, n, (n - 1) / 2, y, yh, s_hist);
    v1 = (n % 2) ? v0 : cv_radix_select(cached ? s_cache : nullptr, n, n / 2, y, yh, s_hist);
  }
  if (lane == 0) {
    double *m = a.metrics + (size_t)series * PF_CV_NMETRICS;
    const double w = (double)n;
    m[PF_CV_MSE] = t[0] / w;
    m[PF_CV_RMSE] = sqrt(t[0] / w);
    m[PF_CV_MAE] = t[1] / w;
    m[PF_CV_MAPE] = (tmin >= 1e-8) ? t[2] / w : NAN;
    m[PF_CV_SMAPE] = t[3] / w;
    m[PF_CV_COVERAGE] = lo ? t[4] / w : NAN;
    m[PF_CV_MDAPE] = (!anybad && !a.skip_mdape) ? (v0 + v1) * 0.5 : NAN;
  }
}

// the kernels live in the main unit only (the fit units use the device
// functions above through the fused forecast epilogue)
#if PF_MAIN
__global__ __launch_bounds__(PF_CV_INS_WAVES * 64) void k_cv_insample(CvKArgs a) {
  __shared__ unsigned long long s_cache[PF_CV_INS_CACHE];
  __shared__ double s_part[PF_CV_INS_WAVES][6];
  __shared__ int s_hist[256];
  __shared__ int s_bad;
  cv_insample_block(a, blockIdx.x, s_cache, s_part, s_hist, &s_bad);
}

__global__ __launch_bounds__(64) void k_cv_metrics(CvKArgs a) {
  __shared__ double s_sum[PF_CV_MDAPE][PF_CV_GMAX];
  __shared__ int s_cnt[PF_CV_GMAX];
  const int series = blockIdx.x, lane = pf_lane();
  const double *y = a.y + (size_t)series * a.ld_y;
  const float *yh = a.yhat + (size_t)series * a.ld_f;
  const float *lo = a.ylo ? a.ylo + (size_t)series * a.ld_f : nullptr;
  const float *hi = a.yhi ? a.yhi + (size_t)series * a.ld_f : nullptr;
  double ymin = INFINITY;
  for (int g = lane; g < a.n_groups; g += 64) {
    double se = 0.0, ae = 0.0, ape = 0.0, sape = 0.0, cov = 0.0;
    const int r0 = a.group_start[g], r1 = a.group_start[g + 1];
    for (int r = r0; r < r1; ++r) {
      const double yv = y[r], fv = (double)yh[r];
      const double e = yv - fv;
      se += e * e;
      ae += fabs(e);
      ape += fabs(e / yv);                      // inf/nan only matter if MAPE is kept
      sape += 2.0 * fabs(e) / (fabs(yv) + fabs(fv));
      if (lo) cov += (yv >= (double)lo[r] && yv <= (double)hi[r]) ? 1.0 : 0.0;
      ymin = fmin(ymin, fabs(yv));
    }
    s_sum[PF_CV_MSE][g] = se;
    s_sum[PF_CV_RMSE][g] = se;
    s_sum[PF_CV_MAE][g] = ae;
    s_sum[PF_CV_MAPE][g] = ape;
    s_sum[PF_CV_SMAPE][g] = sape;
    s_sum[PF_CV_COVERAGE][g] = cov;
    s_cnt[g] = r1 - r0;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) ymin = fmin(ymin, __shfl_xor(ymin, o, 64));
  __syncthreads();
  // MDAPE (UPSTREAM rolling_median_by_h): lane g takes horizon groups g,
  // g+64, ...; group i's sample is its rows extended backwards (rows are
  // sorted by horizon) until the window is filled; a group is kept iff
  // rows up to its end >= window (monotone: UPSTREAM's backward sweep stops
  // at the first group that cannot fill it).  Median by rank counting.
  if (a.skip_mdape) {
    if (lane == 0) a.metrics[(size_t)series * PF_CV_NMETRICS + PF_CV_MDAPE] = NAN;
  } else {
    double macc = 0.0, mcnt = 0.0;
    for (int g = lane; g < a.n_groups; g += 64) {
      const int gs = a.group_start[g], r1 = a.group_start[g + 1];
      if (r1 < a.window) continue;
      const int r0 = (r1 - gs >= a.window) ? gs : r1 - a.window;
      const int n = r1 - r0, k0 = (n - 1) / 2, k1 = n / 2;
      double v0 = NAN, v1 = NAN;
      bool bad = false;
      for (int j = r0; j < r1 && !bad; ++j) {
        const double vj = fabs((y[j] - (double)yh[j]) / y[j]);
        if (vj != vj) { bad = true; break; }
        int lt = 0, le = 0;
        for (int q = r0; q < r1; ++q) {
          const double vq = fabs((y[q] - (double)yh[q]) / y[q]);
          lt += (vq < vj);
          le += (vq <= vj);
        }
        if (lt <= k0 && k0 < le) v0 = vj;
        if (lt <= k1 && k1 < le) v1 = vj;
      }
      macc += bad ? NAN : (v0 + v1) * 0.5;
      mcnt += 1.0;
    }
    macc = wave_sum(macc);
    mcnt = wave_sum(mcnt);
    if (lane == 0)
      a.metrics[(size_t)series * PF_CV_NMETRICS + PF_CV_MDAPE] = (mcnt > 0.0) ? macc / mcnt : NAN;
  }
  if (lane < PF_CV_MDAPE) {
    const int m = lane;
    const double w = (double)a.window;
    double x_sum = 0.0, acc = 0.0;
    long n_sum = 0;
    int trailing = a.n_groups - 1, n_out = 0;
    for (int i = a.n_groups - 1; i >= 0; --i) {
      x_sum += s_sum[m][i];
      n_sum += s_cnt[i];
      while (n_sum >= a.window) {
        const double excess_n = (double)(n_sum - a.window);
        const double excess_x = excess_n * s_sum[m][i] / (double)s_cnt[i];
        const double r = (x_sum - excess_x) / w;
        acc += (m == PF_CV_RMSE) ? sqrt(r) : r;
        ++n_out;
        x_sum -= s_sum[m][trailing];
        n_sum -= s_cnt[trailing];
        --trailing;
      }
    }
    double v = (n_out > 0) ? acc / (double)n_out : NAN;
    if (m == PF_CV_MAPE && ymin < 1e-8) v = NAN;   // UPSTREAM: skip MAPE when y ~ 0
    if (m == PF_CV_COVERAGE && !lo) v = NAN;
    a.metrics[(size_t)series * PF_CV_NMETRICS + m] = v;
  }
}
#endif  // PF_MAIN
