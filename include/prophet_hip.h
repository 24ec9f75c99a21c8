/*
 * prophet_hip.h — C ABI of the MI355X (gfx950) batched Prophet engine.
 *
 * This is the drop-in boundary for the reference's per-group hot path
 * (SURVEY.md §8b).  The reference binds Prophet through Python only:
 *   - fit:      Prophet(...).fit(history_pd)           notebooks/prophet/02_training.py:162-172
 *               (→ PyStan optimizing(LBFGS), UPSTREAM)
 *   - forecast: make_future_dataframe(90,'d') + predict  notebooks/prophet/02_training.py:201-205
 *               and model.predict(future_df)             notebooks/prophet/model_wrapper.py:58-61
 * Each entry point below replaces one of those upstream calls for a whole
 * batch of series at once.  The Python host layer (distributed-forecasting_amd/)
 * binds them with ctypes exactly as INTEGRATION.md shows.
 *
 * Conventions
 *   - Every buffer is a caller-owned DEVICE pointer (e.g. torch tensor
 *     data_ptr()).  The library never frees caller memory; scratch lives in
 *     the opaque context.
 *   - Every call is asynchronous on the caller's hipStream_t (passed as void*).
 *   - Return value: 0 = ok, <0 = argument / HIP error (pf_last_error() has
 *     the message).  Per-series outcomes are reported in status arrays, never
 *     as a non-zero return.
 *   - A context is per device and must not be shared between host threads.
 *
 * Parameter vector per series (Stan unconstrained order, fp64):
 *   theta = [k, m, delta[S], log(sigma_obs), beta[K]],  P = 3 + S + K.
 */
#ifndef PROPHET_HIP_H
#define PROPHET_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pf_ctx pf_ctx;

enum pf_growth { PF_GROWTH_LINEAR = 0, PF_GROWTH_LOGISTIC = 1, PF_GROWTH_FLAT = 2 };

/* Per-series fit status (Stan bfgs.hpp TERM_* codes + engine extras). */
enum pf_status {
  PF_ST_SUCCESS = 0, PF_ST_ABSX = 10, PF_ST_ABSF = 20, PF_ST_RELF = 21,
  PF_ST_ABSGRAD = 30, PF_ST_RELGRAD = 31, PF_ST_MAXIT = 40,
  PF_ST_LSFAIL = -1, PF_ST_BADINIT = -2,
  PF_ST_CONSTANT = 50,         /* min y == max y: optimizer skipped (Prophet rule) */
  PF_ST_WARMUP = 60,           /* L-BFGS stopped at the warm-up cap (lbfgs_warmup)  */
  PF_ST_MAP = 70               /* exact-MAP polish certified the optimum            */
};

/* One Fourier seasonality block: columns sin/cos(2π(i+1)d/period), i<order. */
typedef struct { double period; int32_t order; int32_t _pad; } pf_season;

/* A shared date grid (all series of a batch share their non-NaN dates).
 * Rows are padded to T_pad = round_up(T, 128); buffers use stride T_pad. */
typedef struct {
  int32_t T;            /* valid rows                                       */
  int32_t T_pad;        /* row stride of XT / y buffers (multiple of 128)   */
  int32_t K;            /* feature columns                                  */
  int32_t S;            /* changepoints (>= 1; dummy t_change=[0] if none)  */
  const double *t;      /* [T_pad]   (ds - start)/t_scale                   */
  const double *XT;     /* [K*T_pad] features, feature-major                */
  const double *t_change;  /* [S]                                           */
  const int32_t *seg;   /* [T_pad]   #{j : t_change[j] <= t[i]}             */
  const int32_t *cp_first; /* [S]    first row with t >= t_change[j]         */
} pf_grid;

/* The Stan data block for a batch of n_series series on one grid. */
typedef struct {
  int32_t n_series;
  int32_t growth;       /* pf_growth */
  double tau;           /* changepoint_prior_scale                          */
  pf_grid grid;
  const double *sigmas; /* [K] prior scales                                 */
  const double *s_a;    /* [K] additive indicator                           */
  const double *s_m;    /* [K] multiplicative indicator                     */
  const double *y_scaled; /* [n_series*T_pad] y / y_scale (pad rows ignored) */
  const double *cap_scaled; /* [n_series*T_pad] or NULL (logistic only)     */
  /* Layout hints (host-known, avoid device reads):
   *   fourier_orders: orders of the Fourier blocks occupying the first
   *     2*sum(orders) columns of X (e.g. {10,3,0} = yearly+weekly); lets the
   *     kernel regenerate harmonics in-register. {0,0,0} = read X densely.
   *   season_mode: 0 = every column multiplicative (s_m=1,s_a=0),
   *                1 = every column additive, 2 = mixed.                   */
  int32_t fourier_orders[3];
  int32_t season_mode;
  /* Hyperparameter batching (the AutoML ProphetHyperoptEstimator search over
   * changepoint / seasonality / holidays prior scales, notebooks/automl/
   * 22-09-26-06:54-Prophet-...py:111-123, run as extra batch rows): per-series
   * prior scales, or NULL to use the shared tau / sigmas above.            */
  const double *tau_series;     /* [n_series]      changepoint_prior_scale   */
  const double *sigmas_series;  /* [n_series * K]  per-column prior scales   */
  /* Ragged batches (series with different date grids in one launch; the
   * reference's applyInPandas groups each carry their own history,
   * notebooks/prophet/02_training.py:277-307): grids is a DEVICE array of
   * n_grids pf_grid descriptors (device pointers inside), grid_of a DEVICE
   * [n_series] index into it.  Every grid shares T_pad, K, S and the
   * seasonality layout; `grid` above is then the envelope: T = max T over the
   * grids, T_pad / K / S the shared values (its pointers are not read).
   * n_grids = 0: every series uses `grid`.                                  */
  int32_t n_grids;
  const pf_grid *grids;
  const int32_t *grid_of;
} pf_problem;

typedef struct {
  /* Stan optimizing() defaults as PyStan 2.19 / Prophet pass them */
  double init_alpha, tol_obj, tol_rel_obj, tol_grad, tol_rel_grad, tol_param;
  int32_t max_iter, history;
  /* engine: exact-MAP proximal-Newton polish after the Stan phase (0/1) */
  int32_t polish, polish_max_iter;
  /* engine: with polish, the Stan L-BFGS phase runs at most lbfgs_warmup
   * iterations before the polish takes it to the MAP (Stan's zig-zag at the
   * |delta| kink adds hundreds of evaluations that do not move the MAP); a
   * series whose polish does not certify convergence resumes L-BFGS (once
   * more for lbfgs_warmup iterations, then with Stan's full termination
   * rules) and is polished again.  0 = run Stan's full termination rules
   * first (the reference's behaviour), then polish.  lbfgs_warmup_evals > 0
   * also ends a warm-up pass once it has used that many evaluations (at the
   * next accepted iterate, or inside a line search at the last accepted
   * iterate once lbfgs_warmup_ls_slack more were used).  Defaults: 40 iterations, 60
   * evaluations.                                                           */
  int32_t lbfgs_warmup, lbfgs_warmup_evals;
  /* engine: batches of at least tile_min_series series run the first L-BFGS
   * pass in the tiled kernel (16 series per workgroup, FP64 MFMA row pass,
   * 16 lanes of L-BFGS per series) when the layout allows it (linear, flat
   * or logistic growth, P <= 72, K <= 48, shared prior scales); < 0 never. */
  int32_t tile_min_series;
  /* engine polish: after a full undamped Newton step the next QP reuses the
   * swept Hessian (at most polish_max_lag times in a row) as long as each
   * lagged QP's predicted decrease is below polish_lag_ratio times the
   * previous one; otherwise the exact Hessian is recomputed.  Defaults 4,
   * 1e-2.                                                                  */
  int32_t polish_max_lag;
  double polish_lag_ratio;
  /* engine polish: the first QP's model is H + polish_lam0 * max|diag H| * I
   * (one Levenberg-Marquardt-damped step; later steps undamped unless a
   * non-positive pivot asks for damping).  An undamped first Newton step from
   * the warm-up hand-off can jump to a neighbouring, worse local optimum of
   * the non-convex MAP objective.  Default 1e-2; 0 = undamped.             */
  double polish_lam0;
  /* engine warm-up: inside a line search the pass ends (at the last accepted
   * iterate) once it has used lbfgs_warmup_evals + lbfgs_warmup_ls_slack
   * evaluations.  Default 4.                                               */
  int32_t lbfgs_warmup_ls_slack;
} pf_fit_opts;

/* component blocks pf_predict can report (seasonalities, holidays, ...) */
#define PF_MAX_COMP 32

/* ---------------------------------------------------------------- context */
int pf_ctx_create(int device, pf_ctx **out);
int pf_ctx_destroy(pf_ctx *ctx);
const char *pf_last_error(pf_ctx *ctx);
/* Defaults every caller should start from (Stan optimizing() + the engine's
 * polish settings); a zero-initialised pf_fit_opts is not a valid default. */
void pf_default_fit_opts(pf_fit_opts *o);
/* Build id: 32 hex digits of SHA-256 over the library's sources and compile
 * flags (no reference counterpart; the Python loader refuses a library whose
 * id does not match the sources it ships with).                            */
const char *pf_build_id(void);

/* Per-kernel timing (measurement only; no reference counterpart).  When
 * enabled, every launch is bracketed by HIP events on its own stream;
 * pf_read_timings synchronises on them, returns the number of records
 * written (<= max_out, at most 1024 per read) and clears the list.         */
typedef struct {
  char name[32];
  float ms;
  int32_t grid;   /* workgroups launched */
} pf_kernel_time;
int pf_set_timing(pf_ctx *ctx, int enable);
int pf_read_timings(pf_ctx *ctx, pf_kernel_time *out, int max_out);

/* Host-side helper (no GPU): number of changepoints Prophet will place for a
 * history of T rows (set_changepoints clamp: n_cp+1 > floor(T*range) → floor-1). */
int pf_num_changepoints(int T, int n_changepoints, double changepoint_range);

/* ----------------------------------------------------- K1: design builder
 * Replaces UPSTREAM setup_dataframe (t), make_all_seasonality_features (X)
 * and set_changepoints + Stan get_changepoint_matrix (t_change, segments).
 *   ds_ns [T] sorted int64 ns; start_ns / t_scale_ns from the fit history.
 *   extra_cols [n_extra*T] (holidays / regressors, feature-major) or NULL.
 *   n_changepoints < 0  → do not place changepoints (predict grids reuse the
 *   fit's t_change and only get seg[]).                                     */
int pf_build_grid(pf_ctx *ctx, const int64_t *ds_ns, int T, int T_pad,
                  int64_t start_ns, int64_t t_scale_ns,
                  const pf_season *seasons_host, int n_season,
                  const double *extra_cols, int n_extra,
                  int n_changepoints, double changepoint_range,
                  double *t_out, double *XT_out,
                  double *t_change_io, int32_t *cp_idx_out,
                  int32_t *seg_out, int32_t *cp_first_out, int S,
                  void *stream);

/* Ragged design builder: n_grids grids (one per distinct history, all with
 * the same seasonalities, T_pad and S) in three launches, for pf_problem.grids
 * / pf_predict_args.grids.  DEVICE inputs: grid_params[n_grids*6] int64 =
 * {offset into ds_ns, T, start_ns, t_scale_ns, first_ns, step_ns} per grid
 * (step_ns > 0: dates first + i*step generated on the device, ds_ns unread
 * for that grid; else ds_ns[offset + i]).  T_max = max T (host).  DEVICE
 * outputs, grid g at: t_out[g*T_pad], XT_out[g*K*T_pad], t_change_io[g*S]
 * (input when n_changepoints < 0: forecast grids on their fit's
 * changepoints), cp_idx_out[g*S], seg_out[g*T_pad], cp_first_out[g*S], and
 * grids_out[g] = the pf_grid descriptor pointing into them.  No extra
 * (holiday) columns: use pf_build_grid per grid for those.                 */
int pf_build_grids(pf_ctx *ctx, int n_grids, const int64_t *grid_params, const int64_t *ds_ns,
                   int T_max, int T_pad, const pf_season *seasons_host, int n_season,
                   int n_changepoints, double changepoint_range,
                   double *t_out, double *XT_out, double *t_change_io, int32_t *cp_idx_out,
                   int32_t *seg_out, int32_t *cp_first_out, int S, pf_grid *grids_out,
                   void *stream);

/* ------------------------------------------ scaling + Prophet init (a1, a4)
 * y [n_series*T_pad] raw (pad rows ignored) → y_scale[n], y_scaled[n*T_pad],
 * theta0[n*P] (linear_growth_init; delta=beta=0; sigma_obs=1) and
 * status[n] = PF_ST_CONSTANT where min y == max y (else 0).               */
int pf_prepare(pf_ctx *ctx, int n_series, const pf_grid *grid, int growth,
               const double *y, const double *cap,
               double *y_scale, double *y_scaled, double *cap_scaled,
               double *theta0, int32_t *status, void *stream);

/* pf_prepare for a ragged batch: series s is scaled and initialised on its
 * own grid grids_dev[grid_of[s]] (DEVICE arrays, see pf_problem.grids);
 * envelope as in pf_problem.grid.                                          */
int pf_prepare_ragged(pf_ctx *ctx, int n_series, const pf_grid *envelope, int n_grids,
                      const pf_grid *grids_dev, const int32_t *grid_of, int growth,
                      const double *y, const double *cap,
                      double *y_scale, double *y_scaled, double *cap_scaled,
                      double *theta0, int32_t *status, void *stream);

/* ------------------------------------------- K2: batched objective + grad
 * f[n] = -log posterior (Stan propto), g[n*P] = its gradient.            */
int pf_objective_grad(pf_ctx *ctx, const pf_problem *pb, const double *theta,
                      double *f, double *g, void *stream);

/* ------------------------------------------- exact Hessian (polish model)
 * H[n*P*P] (row-major per series) = Hessian of the smooth part of the
 * -log posterior at theta (the L1 term on delta excluded): the model the
 * exact-MAP polish of pf_fit solves its QP with, and what Stan's Newton
 * optimizer (PyStan optimizing(algorithm='Newton'), Prophet's fallback when
 * L-BFGS fails, UPSTREAM) would form.  Linear, flat and logistic growth;
 * needs 2 + S <= 32 and K <= 48.                                          */
int pf_hessian(pf_ctx *ctx, const pf_problem *pb, const double *theta, double *H, void *stream);

/* -------------------------------------------------- K3: batched fit (MAP)
 * theta_inout[n*P]: init in, optimum out.  f_out[n] final -log posterior,
 * f_stan[n] objective where the (first) L-BFGS phase stopped, status[n]
 * (in: PF_ST_CONSTANT rows are skipped; out: PF_ST_MAP when the polish
 * certified the optimum, else the Stan termination code), n_iter[n]
 * (L-BFGS iterations), n_eval[n] (L-BFGS objective+gradient evaluations,
 * all passes; the polish's few line-search evaluations are not counted).
 * Scratch is stream-ordered in the context.                              */
int pf_fit(pf_ctx *ctx, const pf_problem *pb, const pf_fit_opts *opts,
           double *theta_inout, double *f_out, double *f_stan,
           int32_t *status, int32_t *n_iter, int32_t *n_eval, void *stream);

/* ------------------------------ K4+K5: forecast + Monte-Carlo intervals
 * Future grid fg (t relative to the fit's start/t_scale; seg vs the fit's
 * t_change).  Outputs fp32 [n*fg.T_pad] (stride T_pad).  n_samples <= 1024;
 * n_samples == 0 skips the intervals (lower/upper = point).  trend_* and
 * the component outputs may be NULL.                                     */
/* Interval estimator (pf_predict_args.interval_method).
 *  EXACT  (0, default): rows whose trend is deterministic (the history, flat
 *         growth) draw the needed order statistics of the N noise samples
 *         exactly (uniform spacings + inverse normal CDF): the same
 *         distribution as N materialised samples, O(1) work per row.  Rows
 *         with future trend uncertainty are always sampled N times.
 *  SAMPLE (1): every row materialises N samples (UPSTREAM's literal loop). */
enum { PF_INTERVAL_EXACT = 0, PF_INTERVAL_SAMPLE = 1 };

typedef struct {
  int32_t n_series, growth, n_samples, interval_method;
  pf_grid fg;
  const double *s_a, *s_m;
  const double *theta;        /* [n*P] */
  const double *y_scale;      /* [n]   */
  const double *cap_scaled;   /* [n*fg.T_pad] or NULL */
  double interval_width;
  uint64_t seed;
  float *yhat, *yhat_lower, *yhat_upper;
  float *trend, *trend_lower, *trend_upper;
  float *mult_terms, *add_terms;
  /* optional per-seasonality components (Prophet's 'yearly', 'weekly', ...):
   * block b covers columns [comp_col0[b], comp_col0[b]+comp_ncol[b]); output
   * comp[(b*n + s)*T_pad + row] (additive blocks already x y_scale).      */
  int32_t n_comp;
  int32_t comp_col0[PF_MAX_COMP], comp_ncol[PF_MAX_COMP];
  float *comp;
  /* optional [n_series] RNG stream key per series (e.g. a hash of
   * (store, item)) so samples do not depend on batch position; NULL: use
   * the batch index.                                                      */
  const uint32_t *series_id;
  /* ragged forecasts (see pf_problem.grids): DEVICE pf_grid[n_grids] of
   * forecast grids (each relative to its fit's start / t_scale / t_change)
   * and DEVICE grid_of[n_series]; fg is the envelope (T = max rows, shared
   * T_pad / K / S).  Rows past a series' own T are not written.            */
  int32_t n_grids;
  const pf_grid *grids;
  const int32_t *grid_of;
  /* which kernels to launch: 0 = all; PF_PREDICT_DET = the point forecast,
   * components and deterministic-row intervals (K4); PF_PREDICT_MC = the
   * Monte-Carlo rows (K5).  The two parts write disjoint rows and depend only
   * on theta, so a caller may run them on two streams (join before reading
   * the intervals).                                                        */
  int32_t parts;
} pf_predict_args;
enum { PF_PREDICT_DET = 1, PF_PREDICT_MC = 2 };

int pf_predict(pf_ctx *ctx, const pf_predict_args *args, void *stream);

/* ------------------------------------------ K6: cross-validation metrics
 * Replaces UPSTREAM diagnostics.performance_metrics(df_cv, rolling_window=0.1)
 * followed by the notebook's mean over horizons (02_training.py:178-188):
 * per series, rolling_mean_by_h over the CV rows with window w, then the mean
 * of the rolled values.  Rows (the concatenated fold predictions) must be
 * sorted by horizon; group_start[n_groups+1] delimits equal-horizon runs and
 * is shared by all series.  MAPE is NaN when min|y| < 1e-8 (UPSTREAM skips
 * it); coverage is NaN when yhat_lower/upper are NULL.  MDAPE follows UPSTREAM
 * rolling_median_by_h (AutoML logs it, notebooks/automl/...:163): per
 * horizon group from the last, the median of the group's rows extended
 * backwards to the window; groups that cannot fill the window are dropped. */
enum { PF_CV_MSE = 0, PF_CV_RMSE = 1, PF_CV_MAE = 2, PF_CV_MAPE = 3, PF_CV_SMAPE = 4,
       PF_CV_COVERAGE = 5, PF_CV_MDAPE = 6, PF_CV_NMETRICS = 7 };
typedef struct {
  int32_t n_series, n_rows, n_groups, window;
  const int32_t *group_start;          /* [n_groups + 1], n_groups <= 512;
                                          NULL with n_groups = 1: one group of
                                          every row (in-sample metrics)     */
  const double *y;                     /* [n_series, ld_y] actuals         */
  const float *yhat, *yhat_lower, *yhat_upper;   /* [n_series, ld_f]       */
  double *metrics;                     /* [n_series, PF_CV_NMETRICS]       */
  int32_t ld_y, ld_f;                  /* row strides in elements (0: n_rows),
                                          e.g. the padded history / forecast
                                          buffers read in place             */
  int32_t skip_mdape;                  /* 1: MDAPE not computed (NaN): the
                                          reference logs mse / mae / mape    */
} pf_cv_args;
int pf_cv_metrics(pf_ctx *ctx, const pf_cv_args *args, void *stream);

/* ------------------------------------ K3+K4+K5+K6: fit, forecast, metrics
 * The results of pf_fit, then pf_predict(pred), then (cv != NULL)
 * pf_cv_metrics(cv) on one stream — the training stage of
 * 02_training.py:150-205 for a batch — with pred->theta == theta_inout and
 * every part covering the pb->n_series fitted series.  Where the layout
 * allows (one grid, PF_INTERVAL_EXACT, every forecast part, in-sample metrics
 * (cv: n_groups = 1, window = n_rows), the warm-up hand-off fit path) it is
 * ONE launch: each series' forecast rows and metrics run in its fit
 * workgroup as soon as its own fit ends (bitwise the separate launches'
 * outputs); *fused (may be NULL) says whether it was.  flags
 * PF_FF_ONLY_FUSED: launch nothing unless fused (*fused = 0: the caller runs
 * the parts itself, e.g. on two streams).  The metrics' y / yhat rows are
 * read after this series' forecast rows are written (yhat = pred->yhat).   */
enum { PF_FF_ONLY_FUSED = 1 };
int pf_fit_forecast(pf_ctx *ctx, const pf_problem *pb, const pf_fit_opts *opts,
                    double *theta_inout, double *f_out, double *f_stan,
                    int32_t *status, int32_t *n_iter, int32_t *n_eval,
                    const pf_predict_args *pred, const pf_cv_args *cv, int flags,
                    int32_t *fused, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* PROPHET_HIP_H */
