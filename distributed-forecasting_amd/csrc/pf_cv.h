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
  int n_series, n_rows, n_groups, window;
  const int32_t *group_start;
  const double *y;
  const float *yhat, *ylo, *yhi;
  double *metrics;
};

__global__ __launch_bounds__(64) void k_cv_metrics(CvKArgs a) {
  __shared__ double s_sum[PF_CV_MDAPE][PF_CV_GMAX];
  __shared__ int s_cnt[PF_CV_GMAX];
  const int series = blockIdx.x, lane = pf_lane();
  const double *y = a.y + (size_t)series * a.n_rows;
  const float *yh = a.yhat + (size_t)series * a.n_rows;
  const float *lo = a.ylo ? a.ylo + (size_t)series * a.n_rows : nullptr;
  const float *hi = a.yhi ? a.yhi + (size_t)series * a.n_rows : nullptr;
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
  {
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
