// pf_engine.hip — MI355X (gfx950) batched Prophet fit + forecast engine.
//
// Kernels:
//   K1 k_grid_*      a1/a2/a3  t, Fourier features X^T, changepoints, segments
//   -- k_prepare     a1/a4     y_scale, y_scaled, Prophet linear/flat init
//   K2 k_objgrad     a5        Stan log-posterior (propto) + analytic gradient
//   K3 k_fit         a6        Stan-faithful L-BFGS (+ exact-MAP polish, pf_polish.h)
//   K4/K5 k_predict  a7/a8     point forecast + Poisson-process MC intervals
//
// One workgroup owns one series for the whole optimisation (persistent per
// series): the series' y lives in LDS, every objective evaluation is a
// collective pass over the rows (4 waves), and the L-BFGS state machine runs
// redundantly in every wave (lane p holds parameter p), so the only
// synchronisation is the handful of barriers inside each evaluation.
// No CPU fallback exists: every entry point launches HIP kernels.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "pf_common.h"
#include "prophet_hip.h"

// Split compilation (build.py): PF_TU = 0 compiles the host API and every
// kernel outside the fit family; PF_TU = k >= 1 compiles the fit-kernel
// instantiations of group k (launch_fitlike, listed at the end of the file),
// so the groups build in parallel.  PF_TU undefined: one translation unit
// with everything (diagnostic builds).
#ifdef PF_TU
#define PF_MAIN (PF_TU == 0)
#else
#define PF_MAIN 1
#endif

#include "pf_cv.h"
#include "pf_ostat.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

// Per-launch timing (pf_set_timing): a fixed pool of HIP event pairs recorded
// on the launch stream around every kernel, read back by pf_read_timings.
#define PF_MAX_TIMED 1024
struct pf_timed {
  const char *name;
  hipEvent_t start, stop;
  int grid;
};

struct pf_ctx {
  int device;
  int n_cu;         // compute units of the device (persistent K3T grid)
  char err[512];
  void *ws;         // scratch owned by the context (lane-blocked grid copy)
  size_t ws_bytes;
  void *ws2;        // fused launch's work-sharing counters (pf_fit_forecast)
  size_t ws2_bytes;
  int timing;       // record events around launches
  int n_timed;      // records since the last pf_read_timings
  int n_events;     // event pairs created so far
  pf_timed timed[PF_MAX_TIMED];
};

static char g_err_noctx[512] = "";

// Diagnostic build only (-DPF_STAMPS, tools/stamps.py): s_memtime sums at
// phase boundaries of block 0 / thread 0.  Never compiled into the product.
#ifdef PF_STAMPS
__device__ unsigned long long pf_dbg[32];
#define PF_STAMP(i)                                                              \
  do {                                                                           \
    if (blockIdx.x == 0 && threadIdx.x == 0)                                     \
      atomicAdd(&pf_dbg[i], (unsigned long long)__builtin_amdgcn_s_memtime());   \
  } while (0)
#define PF_COUNT(i)                                                              \
  do {                                                                           \
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&pf_dbg[i], 1ull);        \
  } while (0)
#define PF_STAMP1(i)                                                             \
  do {                                                                           \
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)                  \
      atomicAdd(&pf_dbg[i], (unsigned long long)__builtin_amdgcn_s_memtime());   \
  } while (0)
// every wave of every block (lane 0): path counters
#define PF_COUNTW(i)                                                             \
  do {                                                                           \
    if (pf_lane() == 0) atomicAdd(&pf_dbg[i], 1ull);                             \
  } while (0)
#else
#define PF_COUNTW(i) do { } while (0)
#define PF_STAMP1(i) do { } while (0)
#define PF_STAMP(i) do { } while (0)
#define PF_COUNT(i) do { } while (0)
#endif

#if defined(PF_STAMPS) && !defined(PF_TIMELINE)
#define PF_TIMELINE
#endif
// Diagnostic build only (-DPF_TIMELINE, tools/block_timeline.py): no other
// instrumentation, so the timeline is the product kernel's.
#ifdef PF_TIMELINE
// per-block timeline of the fused launch: [start, fit end, end] s_memrealtime
// (100 MHz, one clock for every XCD)
// [3]: the first L-BFGS phase's end (the polish starts); blocks < 4096
// [4] / [5]: the polish's Newton steps / exact Hessians (all passes, summed)
// [6] / [7]: time in the polish's Hessian assembly / sweep-in (memrealtime ticks)
// [8] / [9] / [10]: time in the QP (wave 0) / the polish's line-search
// evaluations / the stash restore
__device__ unsigned long long pf_blk[11][4096];
#define PF_BLK(i)                                                                \
  do {                                                                           \
    if (threadIdx.x == 0 && blockIdx.x < 4096)                                   \
      pf_blk[i][blockIdx.x] = (unsigned long long)__builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define PF_RT() ((unsigned long long)__builtin_amdgcn_s_memrealtime())
#define PF_BLKV(i, v)                                                            \
  do {                                                                           \
    if (threadIdx.x == 0 && blockIdx.x < 4096) pf_blk[i][blockIdx.x] += (unsigned long long)(v); \
  } while (0)
#else
#define PF_BLK(i) do { } while (0)
#define PF_BLKV(i, v) do { } while (0)
#define PF_RT() 0ull
#endif

// Wave priorities.  Two fit workgroups share each CU and the SIMD arbiter
// otherwise prefers the older one's waves, so the younger workgroup's serial
// steps (one wave works, the other three wait at the next barrier) queue
// behind the older one's row pass and its fit ends up to ~50% later
// (tools/block_timeline.py).  Serial sections run at 3, the rest of a fit
// at 1, and the fused forecast epilogue (k_fit_forecast) at 0: the critical
// path first on every SIMD, the epilogue in the gaps the fits leave.
__device__ __forceinline__ void pf_serial_prio(bool on) {
#ifndef PF_NO_PRIO
  if (on) __builtin_amdgcn_s_setprio(3);
  else __builtin_amdgcn_s_setprio(1);
#else
  (void)on;
#endif
}
__device__ __forceinline__ void pf_base_prio(int p) {
#ifndef PF_NO_PRIO
  if (p == 0) __builtin_amdgcn_s_setprio(0);
  else __builtin_amdgcn_s_setprio(1);
#else
  (void)p;
#endif
}

// diagnostic switch (environment): "1" enables
static bool getenv_flag(const char *name) {
  const char *v = getenv(name);
  return v && v[0] == '1';
}

static int set_err(pf_ctx *ctx, const char *msg) {
  char *dst = ctx ? ctx->err : g_err_noctx;
  snprintf(dst, 512, "%s", msg);
  return -1;
}

#define PF_HIP(ctx, call)                                                        \
  do {                                                                           \
    hipError_t e_ = (call);                                                      \
    if (e_ != hipSuccess) {                                                      \
      char b_[480];                                                              \
      snprintf(b_, sizeof b_, "%s failed: %s", #call, hipGetErrorString(e_));    \
      set_err(ctx, b_);                                                          \
      return -2;                                                                 \
    }                                                                            \
  } while (0)

// bracket a launch with the context's timing events (no-op unless enabled)
static int timed_begin(pf_ctx *ctx, const char *name, int grid, hipStream_t st) {
  if (!ctx || !ctx->timing || ctx->n_timed >= PF_MAX_TIMED) return -1;
  const int i = ctx->n_timed;
  if (i >= ctx->n_events) {
    if (hipEventCreate(&ctx->timed[i].start) != hipSuccess) return -1;
    if (hipEventCreate(&ctx->timed[i].stop) != hipSuccess) return -1;
    ctx->n_events = i + 1;
  }
  ctx->timed[i].name = name;
  ctx->timed[i].grid = grid;
  if (hipEventRecord(ctx->timed[i].start, st) != hipSuccess) return -1;
  ctx->n_timed = i + 1;
  return i;
}
static void timed_end(pf_ctx *ctx, int i, hipStream_t st) {
  if (i >= 0) (void)hipEventRecord(ctx->timed[i].stop, st);
}
#define PF_TIMED_LAUNCH(ctx, name, grid_n, st, ...)                              \
  do {                                                                           \
    const int ti_ = timed_begin(ctx, name, (int)(grid_n), st);                   \
    hipLaunchKernelGGL(__VA_ARGS__);                                             \
    timed_end(ctx, ti_, st);                                                     \
  } while (0)

#if PF_MAIN
// ============================================================================
// K1: design builder
// ============================================================================
#define PF_MAX_SEASONS 8
struct SeasonSpec {
  int n;
  double period[PF_MAX_SEASONS];
  int order[PF_MAX_SEASONS];
};

// t = (ds - start)/t_scale (numpy m8/m8 -> double/double);
// d = (ns / 1e9) / 86400  (pandas total_seconds()/(3600*24.));
// X col (2i, 2i+1) = sin, cos of ((2.0*(i+1))*pi*d)/period evaluated
// left to right like UPSTREAM fourier_series.
__device__ __forceinline__ void grid_features_row(int i, bool valid, int64_t ns, int Tp,
                                                  int64_t start, int64_t tscale,
                                                  const SeasonSpec &ss,
                                                  const double *__restrict__ extra, int n_extra,
                                                  int T, double *__restrict__ t_out,
                                                  double *__restrict__ XT) {
  int col = 0;
  if (!valid) {
    if (t_out) t_out[i] = 0.0;
    for (int b = 0; b < ss.n; ++b)
      for (int r = 0; r < 2 * ss.order[b]; ++r) XT[(size_t)(col++) * Tp + i] = 0.0;
    for (int e = 0; e < n_extra; ++e) XT[(size_t)(col++) * Tp + i] = 0.0;
    return;
  }
  if (t_out) t_out[i] = __ddiv_rn((double)(ns - start), (double)tscale);
  const double d = __ddiv_rn(__ddiv_rn((double)ns, 1e9), 86400.0);
  for (int b = 0; b < ss.n; ++b) {
    for (int r = 0; r < ss.order[b]; ++r) {
      const double c = __dmul_rn(2.0 * (double)(r + 1), M_PI);
      const double arg = __ddiv_rn(__dmul_rn(c, d), ss.period[b]);
      double sn, cs;
      sincos(arg, &sn, &cs);
      XT[(size_t)(col++) * Tp + i] = sn;
      XT[(size_t)(col++) * Tp + i] = cs;
    }
  }
  for (int e = 0; e < n_extra; ++e) XT[(size_t)(col++) * Tp + i] = extra[(size_t)e * T + i];
}

// One harmonic per blockIdx.y (the seasons' harmonics in column order; the
// last y writes t and the extra columns): each thread evaluates one sincos
// instead of all of them (13 at the default seasons; 7.8 us on 8 CUs before),
// with grid_features_row's arithmetic, bitwise.  The seasons are walked with
// constant indices so the by-value SeasonSpec stays out of scratch.
__global__ void k_grid_features(const int64_t *__restrict__ ds, int T, int Tp, int64_t start,
                                int64_t tscale, SeasonSpec ss, const double *__restrict__ extra,
                                int n_extra, double *__restrict__ t_out, double *__restrict__ XT) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Tp) return;
  const bool valid = i < T;
  int h = blockIdx.y, col = 0, rsel = -1;
  double per = 1.0;
#pragma unroll
  for (int b = 0; b < PF_MAX_SEASONS; ++b) {
    if (b < ss.n && rsel < 0) {
      if (h < ss.order[b]) {
        rsel = h;
        per = ss.period[b];
        col += 2 * h;
      } else {
        h -= ss.order[b];
        col += 2 * ss.order[b];
      }
    }
  }
  if (rsel >= 0) {
    double sn = 0.0, cs = 0.0;
    if (valid) {
      const double d = __ddiv_rn(__ddiv_rn((double)ds[i], 1e9), 86400.0);
      const double c = __dmul_rn(2.0 * (double)(rsel + 1), M_PI);
      sincos(__ddiv_rn(__dmul_rn(c, d), per), &sn, &cs);
    }
    XT[(size_t)col * Tp + i] = sn;
    XT[(size_t)(col + 1) * Tp + i] = cs;
    return;
  }
  if (t_out) t_out[i] = valid ? __ddiv_rn((double)(ds[i] - start), (double)tscale) : 0.0;
  for (int e = 0; e < n_extra; ++e)
    XT[(size_t)(col + e) * Tp + i] = valid ? extra[(size_t)e * T + i] : 0.0;
}

// Ragged design builder (pf_build_grids): grid g = blockIdx.y, its parameters
// prm[g*6 ..] = {ds offset, T, start, t_scale, first, step}; dates first +
// i*step when step > 0 (generated here), else ds[offset + i].
__global__ void k_grids_features(const int64_t *__restrict__ prm, const int64_t *__restrict__ ds,
                                 int Tp, int K, SeasonSpec ss, double *__restrict__ t_out,
                                 double *__restrict__ XT) {
  const int g = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Tp) return;
  const int64_t *p = prm + (size_t)g * 6;
  const int T = (int)p[1];
  const int64_t step = p[5];
  int64_t ns = 0;
  if (i < T) ns = step > 0 ? p[4] + (int64_t)i * step : ds[p[0] + i];
  grid_features_row(i, i < T, ns, Tp, p[2], p[3], ss, nullptr, 0, T, t_out + (size_t)g * Tp,
                    XT + (size_t)g * K * Tp);
}

// UPSTREAM set_changepoints: linspace(0, hist_size-1, n_cp+1).round()[1:]
// (numpy: step = (stop-start)/div; y = arange*step; y[-1] = stop; rint)
__device__ void grid_changepoints(const double *__restrict__ t, int T, int n_cp_req, double range,
                                  double *__restrict__ t_change, int32_t *__restrict__ cp_idx) {
  const int hist_size = (int)floor((double)T * range);
  int n_cp = n_cp_req;
  if (n_cp + 1 > hist_size) n_cp = hist_size - 1;
  if (n_cp > 0) {
    const double stop = (double)(hist_size - 1);
    const double step = stop / (double)n_cp;
    for (int j = 1; j <= n_cp; ++j) {
      const double v = (j == n_cp) ? stop : __dmul_rn((double)j, step);
      const int idx = (int)rint(v);
      cp_idx[j - 1] = idx;
      t_change[j - 1] = t[idx];
    }
    // sort (stable insertion; already sorted for sorted t)
    for (int a = 1; a < n_cp; ++a) {
      double v = t_change[a];
      int b = a - 1;
      while (b >= 0 && t_change[b] > v) { t_change[b + 1] = t_change[b]; --b; }
      t_change[b + 1] = v;
    }
  } else {
    t_change[0] = 0.0;  // dummy changepoint, S = 1
    cp_idx[0] = -1;
  }
}
#define PF_GRID_CP_LDS 4096  // changepoints k_grid_segments places in LDS (32 KB)
__global__ void k_grid_changepoints(const double *__restrict__ t, int T, int n_cp_req, double range,
                                    double *__restrict__ t_change, int32_t *__restrict__ cp_idx) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  grid_changepoints(t, T, n_cp_req, range, t_change, cp_idx);
}
// ragged: one thread per grid (grid g's t at t + g*Tp, S slots per grid)
__global__ void k_grids_changepoints(const int64_t *__restrict__ prm, int G, int Tp, int S,
                                     int n_cp_req, double range, const double *__restrict__ t,
                                     double *__restrict__ t_change, int32_t *__restrict__ cp_idx) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  grid_changepoints(t + (size_t)g * Tp, (int)prm[(size_t)g * 6 + 1], n_cp_req, range,
                    t_change + (size_t)g * S, cp_idx + (size_t)g * S);
}

// seg[i] = #{j : t_change[j] <= t[i]} (Stan A[i,j] = t_i >= t_change_j);
// cp_first[j] = first row with t >= t_change[j].
__device__ __forceinline__ void grid_segments(int i, const double *__restrict__ t, int T, int Tp,
                                              const double *__restrict__ t_change, int S,
                                              int32_t *__restrict__ seg,
                                              int32_t *__restrict__ cp_first) {
  if (i < Tp) {
    int c = S;
    if (i < T) {
      const double ti = t[i];
      c = 0;
      for (int j = 0; j < S; ++j) c += (ti >= t_change[j]) ? 1 : 0;
    }
    seg[i] = c;
  }
  if (cp_first && i < S) {
    const double tc = t_change[i];
    int lo = 0, hi = T;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (t[mid] >= tc) hi = mid; else lo = mid + 1;
    }
    cp_first[i] = lo;
  }
}
// With n_cp_req >= 0 every block first places the changepoints itself (the
// rule of grid_changepoints, one index per thread, then the same stable
// insertion sort, in LDS) and block 0 writes t_change / cp_idx: one launch
// instead of a single-thread k_grid_changepoints (~12 us of serial loads on
// the headline step's critical path) followed by this one.  Bitwise the
// two-kernel form.  n_cp_req < 0: t_change is the caller's (read only).
__global__ __launch_bounds__(256) void k_grid_segments(const double *__restrict__ t, int T, int Tp,
                                                       double *__restrict__ t_change, int S,
                                                       int n_cp_req, double range,
                                                       int32_t *__restrict__ cp_idx,
                                                       int32_t *__restrict__ seg,
                                                       int32_t *__restrict__ cp_first) {
  extern __shared__ double s_tc[];
  const double *tc = t_change;
  if (n_cp_req >= 0) {
    const int hist_size = (int)floor((double)T * range);
    int n_cp = n_cp_req;
    if (n_cp + 1 > hist_size) n_cp = hist_size - 1;
    if (n_cp > 0) {
      const double stop = (double)(hist_size - 1);
      const double step = stop / (double)n_cp;
      for (int j = 1 + (int)threadIdx.x; j <= n_cp; j += blockDim.x) {
        const double v = (j == n_cp) ? stop : __dmul_rn((double)j, step);
        const int idx = (int)rint(v);
        if (blockIdx.x == 0) cp_idx[j - 1] = idx;
        s_tc[j - 1] = t[idx];
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        for (int a = 1; a < n_cp; ++a) {
          double v = s_tc[a];
          int b = a - 1;
          while (b >= 0 && s_tc[b] > v) { s_tc[b + 1] = s_tc[b]; --b; }
          s_tc[b + 1] = v;
        }
      }
    } else if (threadIdx.x == 0) {
      s_tc[0] = 0.0;  // dummy changepoint, S = 1
      if (blockIdx.x == 0) cp_idx[0] = -1;
    }
    __syncthreads();
    if (blockIdx.x == 0)
      for (int j = threadIdx.x; j < S; j += blockDim.x) t_change[j] = s_tc[j];
    tc = s_tc;
  }
  grid_segments(blockIdx.x * blockDim.x + threadIdx.x, t, T, Tp, tc, S, seg, cp_first);
}
// ragged: grid g = blockIdx.y; also writes grid g's pf_grid descriptor
__global__ void k_grids_segments(const int64_t *__restrict__ prm, int Tp, int K, int S,
                                 const double *__restrict__ t, const double *__restrict__ XT,
                                 const double *__restrict__ t_change, int32_t *__restrict__ seg,
                                 int32_t *__restrict__ cp_first, pf_grid *__restrict__ desc) {
  const int g = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int T = (int)prm[(size_t)g * 6 + 1];
  grid_segments(i, t + (size_t)g * Tp, T, Tp, t_change + (size_t)g * S, S, seg + (size_t)g * Tp,
                cp_first + (size_t)g * S);
  if (desc && i == 0) {
    pf_grid d;
    d.T = T;
    d.T_pad = Tp;
    d.K = K;
    d.S = S;
    d.t = t + (size_t)g * Tp;
    d.XT = XT + (size_t)g * K * Tp;
    d.t_change = t_change + (size_t)g * S;
    d.seg = seg + (size_t)g * Tp;
    d.cp_first = cp_first + (size_t)g * S;
    desc[g] = d;
  }
}

// ============================================================================
// prepare: y_scale, y_scaled, init (UPSTREAM initialize_scales, *_growth_init)
// ============================================================================
__global__ __launch_bounds__(256) void k_prepare(int T, int Tp, const double *__restrict__ t,
                                                 int growth, const double *__restrict__ y,
                                                 const double *__restrict__ cap,
                                                 double *__restrict__ y_scale,
                                                 double *__restrict__ y_scaled,
                                                 double *__restrict__ cap_scaled,
                                                 double *__restrict__ theta0,
                                                 int32_t *__restrict__ status, int P, int S,
                                                 const pf_grid *__restrict__ grids,
                                                 const int32_t *__restrict__ grid_of) {
  __shared__ double red[3][4];
  const int s = blockIdx.x;
  if (grid_of) {
    // ragged batch: this series' own rows and t
    const int g = __builtin_amdgcn_readfirstlane(grid_of[s]);
    T = __builtin_amdgcn_readfirstlane(grids[g].T);
    t = (const double *)rfl_ptr(grids[g].t);
  }
  const double *ys = y + (size_t)s * Tp;
  double amax = 0.0, vmin = INFINITY, vmax = -INFINITY, vsum = 0.0;
  // rows up to PF_PREP_REG * 256 stay in registers between the two passes
  // (one read of y instead of two)
  constexpr int PF_PREP_REG = 8;
  const bool in_reg = Tp <= PF_PREP_REG * 256;
  double yr[PF_PREP_REG];
  if (in_reg) {
#pragma unroll
    for (int k = 0; k < PF_PREP_REG; ++k) {
      const int i = threadIdx.x + k * 256;
      yr[k] = i < T ? ys[i] : 0.0;
      if (i < T) {
        amax = fmax(amax, fabs(yr[k]));
        vmin = fmin(vmin, yr[k]);
        vmax = fmax(vmax, yr[k]);
      }
    }
  } else {
    for (int i = threadIdx.x; i < T; i += blockDim.x) {
      const double v = ys[i];
      amax = fmax(amax, fabs(v));
      vmin = fmin(vmin, v);
      vmax = fmax(vmax, v);
    }
  }
  for (int o = 32; o >= 1; o >>= 1) {
    amax = fmax(amax, __shfl_xor(amax, o, 64));
    vmin = fmin(vmin, __shfl_xor(vmin, o, 64));
    vmax = fmax(vmax, __shfl_xor(vmax, o, 64));
  }
  const int w = pf_wave(), lane = pf_lane();
  if (lane == 0) { red[0][w] = amax; red[1][w] = vmin; red[2][w] = vmax; }
  __syncthreads();
  amax = fmax(fmax(red[0][0], red[0][1]), fmax(red[0][2], red[0][3]));
  vmin = fmin(fmin(red[1][0], red[1][1]), fmin(red[1][2], red[1][3]));
  vmax = fmax(fmax(red[2][0], red[2][1]), fmax(red[2][2], red[2][3]));
  double scale = amax == 0.0 ? 1.0 : amax;
  double *out = y_scaled + (size_t)s * Tp;
  if (in_reg) {
#pragma unroll
    for (int k = 0; k < PF_PREP_REG; ++k) {
      const int i = threadIdx.x + k * 256;
      if (i < Tp) {
        const double v = (i < T) ? yr[k] / scale : 0.0;
        out[i] = v;
        if (i < T) vsum += v;
      }
    }
  } else {
    for (int i = threadIdx.x; i < Tp; i += blockDim.x) {
      const double v = (i < T) ? ys[i] / scale : 0.0;
      out[i] = v;
      if (i < T) vsum += v;
    }
  }
  if (growth == PF_GROWTH_LOGISTIC) {
    // UPSTREAM initialize_scales: cap_scaled = (cap - floor) / y_scale, floor 0
    const double *cs = cap + (size_t)s * Tp;
    double *co = cap_scaled + (size_t)s * Tp;
    for (int i = threadIdx.x; i < Tp; i += blockDim.x) co[i] = (i < T) ? cs[i] / scale : 0.0;
  }
  vsum = wave_sum(vsum);
  __syncthreads();
  if (lane == 0) red[0][w] = vsum;
  __syncthreads();
  if (threadIdx.x == 0) {
    vsum = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    y_scale[s] = scale;
    double *th = theta0 + (size_t)s * P;
    for (int p = 0; p < P; ++p) th[p] = 0.0;
    const double y0 = ys[0] / scale, y1 = ys[T - 1] / scale;
    double k = 0.0, m = 0.0;
    if (growth == PF_GROWTH_LINEAR) {
      k = (y1 - y0) / (t[T - 1] - t[0]);
      m = y0 - k * t[0];
    } else if (growth == PF_GROWTH_FLAT) {
      k = 0.0;
      m = vsum / (double)T;
    } else {
      // UPSTREAM logistic_growth_init
      const double *cs = cap + (size_t)s * Tp;
      const double Tt = t[T - 1] - t[0];
      const double C0 = cs[0] / scale, C1 = cs[T - 1] / scale;
      const double yy0 = fmax(0.01 * C0, fmin(0.99 * C0, y0));
      const double yy1 = fmax(0.01 * C1, fmin(0.99 * C1, y1));
      double r0 = C0 / yy0;
      const double r1 = C1 / yy1;
      if (fabs(r0 - r1) <= 0.01) r0 = 1.05 * r0;
      const double L0 = log(r0 - 1.0), L1 = log(r1 - 1.0);
      m = L0 * Tt / (L0 - L1);
      k = (L0 - L1) / Tt;
    }
    th[0] = k;
    th[1] = m;
    th[2 + S] = 0.0;  // log(sigma_obs = 1)
    status[s] = (vmin == vmax && growth != PF_GROWTH_LOGISTIC) ? PF_ST_CONSTANT : 0;
  }
}

#endif  // PF_MAIN (K1, prepare)

// ============================================================================
// K2/K3: objective + gradient (collective over one workgroup) and L-BFGS
// ============================================================================
enum { MODE_MULT = 0, MODE_ADD = 1, MODE_MIXED = 2 };
// bit 2 of the MODE template argument selects the logistic-growth variant
// (compiled separately so the linear kernels carry none of its registers)
#define PF_MODE_LOGI 4
// bit 3: wide variant, P up to 128 — two parameter words per lane, parameter
// p = lane + 64 h in word h (word 1 holds only beta's: 3 + S <= 64)
#define PF_MODE_WIDE 8
template <int MODE>
struct ModeTr {
  static constexpr int PW = (MODE & PF_MODE_WIDE) ? 2 : 1;
};
// this lane's parameter words
template <int PW>
struct PV {
  double v[PW];
  __device__ __forceinline__ double &operator[](int i) { return v[i]; }
  __device__ __forceinline__ double operator[](int i) const { return v[i]; }
};
template <int PW>
__device__ __forceinline__ PV<PW> pv_zero() {
  PV<PW> r;
#pragma unroll
  for (int h = 0; h < PW; ++h) r[h] = 0.0;
  return r;
}

// a warm-up pass (pf_fit_opts.lbfgs_warmup_evals > 0) ends at its next accepted
// iterate once it has used that many evaluations, or inside a line search at
// the last accepted iterate once it has used pf_fit_opts.lbfgs_warmup_ls_slack more

struct FitKArgs {
  int T, Tp, K, S, growth, P, NB;
  const double *t, *XT, *t_change;
  const int32_t *seg;
  // lane-blocked copy of the grid (k_permute_grid): thread L of the
  // workgroup owns natural rows [L*R, L*R+R); position r*NL + L holds row
  // L*R + r, so step r of the row pass is a coalesced load across lanes.
  int R, TQ;                 // rows per thread, TQ = NL*R
  const double *tP, *XTP;    // [TQ], [K][TQ]
  const int32_t *sgP;        // [TQ] seg | (#changepoints first active at this row) << 16
  // row-major copy of the features for the tiled kernel K3T: [Tp][XR_width]
  // (32 or 48), features >= K zero (NULL unless the tiled path may run)
  const double *XR;
  int XR_width;
  int *queue;                // K3T work-queue counter (context scratch)
  const double *sigmas, *s_a, *s_m;
  double tau;
  // hyperparameter batching: per-series prior scales (NULL: the shared
  // tau / sigmas[K] above); sigmas_series is [n][K]
  const double *tau_series, *sigmas_series;
  const double *y_scaled;
  const double *cap_scaled;  // [n][Tp] logistic capacity / y_scale (natural rows), else NULL
  // fit
  double *theta;
  double *f_out, *f_stan, *g_out;
  int32_t *status, *n_iter, *n_eval;
  pf_fit_opts o;
  int pass;      // 0: first L-BFGS pass; >0: resume series the polish did not certify
  int warm_cap;  // this pass's iteration cap is the warm-up cap (MAXIT -> WARMUP)
  int hstash;    // polish LDS holds the undamped-Hessian stash (FitSmem::hst)
  // ragged batch (pf_problem.grids): series s fits on grids[grid_of[s]]; that
  // grid's lane-blocked copy sits at rg_base + g * rg_stride bytes (same
  // layout as tP / XTP / sgP with the grid's own R, TQ); NULL: one grid
  const pf_grid *grids;
  const int32_t *grid_of;
  const char *rg_base;
  size_t rg_stride;
};


// Ragged batch: point the grid fields of `a` at series s's own grid (uniform
// per workgroup).  Rows owned per thread R = ceil(T / NL) as for a batch of
// that grid alone, so a series fitted in a ragged batch follows the same
// arithmetic as in a batch of its own grid.
template <int NL>
__device__ __forceinline__ void bind_grid(FitKArgs &a, int s) {
  const int g = __builtin_amdgcn_readfirstlane(a.grid_of[s]);
  const pf_grid *G = a.grids + g;
  a.T = __builtin_amdgcn_readfirstlane(G->T);
  a.t = (const double *)rfl_ptr(G->t);
  a.XT = (const double *)rfl_ptr(G->XT);
  a.t_change = (const double *)rfl_ptr(G->t_change);
  a.seg = (const int32_t *)rfl_ptr(G->seg);
  a.R = (a.T + NL - 1) / NL;
  a.TQ = NL * a.R;
  const double *base = (const double *)(a.rg_base + (size_t)g * a.rg_stride);
  a.tP = base;
  a.XTP = base + a.TQ;
  a.sgP = (const int32_t *)(base + (size_t)a.TQ * (1 + a.K));
}

// Generated Fourier block: harmonics r >= 1 from the first harmonic column
// pair by the angle-addition recurrence (|err| ~ r ulp), so a pass reads two
// columns per block instead of 2*order.
template <int O, int OFF, int KMAX>
__device__ __forceinline__ void gen_block(const double *__restrict__ XT, int Tp, int i,
                                          double (&x)[KMAX]) {
  if constexpr (O > 0) {
    const double s1 = XT[(size_t)OFF * Tp + i];
    const double c1 = XT[(size_t)(OFF + 1) * Tp + i];
    x[OFF] = s1;
    x[OFF + 1] = c1;
    double sr = s1, cr = c1;
#pragma unroll
    for (int r = 1; r < O; ++r) {
      const double sn = fma(sr, c1, cr * s1);
      const double cn = fma(cr, c1, -(sr * s1));
      sr = sn;
      cr = cn;
      x[OFF + 2 * r] = sr;
      x[OFF + 2 * r + 1] = cr;
    }
  }
}

// Per-row inputs of one evaluation pass, loaded one batch ahead (prefetch).
struct RowIn {
  double t;
  int seg, sprev;
  double f[6];  // first-harmonic (sin, cos) of up to three Fourier blocks
};

// lane-blocked layout: position q of the permuted grid
template <int O0, int O1, int O2>
__device__ __forceinline__ void load_rowp(const FitKArgs &a, int q, RowIn &r) {
  const int TQ = a.TQ;
  r.t = a.tP[q];
  const int pk = a.sgP[q];
  r.seg = pk & 0xFFFF;
  r.sprev = r.seg - (pk >> 16);
  const double *X = a.XTP;
  if constexpr (O0 > 0) { r.f[0] = X[q]; r.f[1] = X[(size_t)TQ + q]; }
  if constexpr (O1 > 0) { r.f[2] = X[(size_t)(2 * O0) * TQ + q]; r.f[3] = X[(size_t)(2 * O0 + 1) * TQ + q]; }
  if constexpr (O2 > 0) {
    r.f[4] = X[(size_t)(2 * (O0 + O1)) * TQ + q];
    r.f[5] = X[(size_t)(2 * (O0 + O1) + 1) * TQ + q];
  }
}

template <int O0, int O1, int O2>
__device__ __forceinline__ void load_row(const double *__restrict__ t, const int32_t *__restrict__ seg,
                                         const double *__restrict__ XT, int Tp, int i, RowIn &r) {
  r.t = t[i];
  r.seg = seg[i];
  r.sprev = (i == 0) ? 0 : seg[i - 1];
  if constexpr (O0 > 0) { r.f[0] = XT[i]; r.f[1] = XT[(size_t)Tp + i]; }
  if constexpr (O1 > 0) { r.f[2] = XT[(size_t)(2 * O0) * Tp + i]; r.f[3] = XT[(size_t)(2 * O0 + 1) * Tp + i]; }
  if constexpr (O2 > 0) {
    r.f[4] = XT[(size_t)(2 * (O0 + O1)) * Tp + i];
    r.f[5] = XT[(size_t)(2 * (O0 + O1) + 1) * Tp + i];
  }
}

template <int O, int OFF, int KMAX>
__device__ __forceinline__ void gen_block_from(double s1, double c1, double (&x)[KMAX]) {
  if constexpr (O > 0) {
    x[OFF] = s1;
    x[OFF + 1] = c1;
    double sr = s1, cr = c1;
#pragma unroll
    for (int r = 1; r < O; ++r) {
      const double sn = fma(sr, c1, cr * s1);
      const double cn = fma(cr, c1, -(sr * s1));
      sr = sn;
      cr = cn;
      x[OFF + 2 * r] = sr;
      x[OFF + 2 * r + 1] = cr;
    }
  }
}

template <int KMAX, int O0, int O1, int O2>
__device__ __forceinline__ void row_features_from(const RowIn &r, const double *__restrict__ XT,
                                                  int Tp, int K, int i, double (&x)[KMAX]) {
  constexpr int KF = 2 * (O0 + O1 + O2);
  gen_block_from<O0, 0, KMAX>(r.f[0], r.f[1], x);
  gen_block_from<O1, 2 * O0, KMAX>(r.f[2], r.f[3], x);
  gen_block_from<O2, 2 * (O0 + O1), KMAX>(r.f[4], r.f[5], x);
#pragma unroll
  for (int f = KF; f < KMAX; ++f) x[f] = (f < K) ? XT[(size_t)f * Tp + i] : 0.0;
}

template <int KMAX, int O0, int O1, int O2>
__device__ __forceinline__ void row_features(const double *__restrict__ XT, int Tp, int K, int i,
                                             double (&x)[KMAX]) {
  constexpr int KF = 2 * (O0 + O1 + O2);
  gen_block<O0, 0, KMAX>(XT, Tp, i, x);
  gen_block<O1, 2 * O0, KMAX>(XT, Tp, i, x);
  gen_block<O2, 2 * (O0 + O1), KMAX>(XT, Tp, i, x);
#pragma unroll
  for (int f = KF; f < KMAX; ++f) x[f] = (f < K) ? XT[(size_t)f * Tp + i] : 0.0;
}

template <int PW>
struct LbLds;
// LDS layout of the fit kernels.  Fixed part + a union region U that holds
// the L-BFGS state during the Stan phase (k_fit) and {Hessian tile
// reduction, H, Cholesky workspace} during the polish (k_polish).
template <int NW, int KMAX, int MODE = 2>
struct FitSmem {
  static constexpr int NSET = ((MODE & 3) == 2) ? 2 : 1;  // (mult, add) gradient sets
  static constexpr int NL = NW * 64;                 // row-pass threads
  // polish Hessian: beta column blocks of 16 and output tiles over
  // [trend 2 blocks | beta NBB blocks] (pf_polish.h)
  static constexpr int NBB = (KMAX + 15) / 16;
  static constexpr int NTILE = (2 + NBB) * (3 + NBB) / 2;
  double *y;        // [ny] lane-blocked y_scaled (position r*NL + L)
  double *th;       // [128]
  double *kseg;     // [64]
  double *mseg;     // [64]
  double *bm, *ba;  // [KMAX]
  double *sfx0, *sfx1;    // [NL] inclusive within-wave suffix of per-thread sums of G, G*t
  double *wt0, *wt1;      // [NW] per-wave totals of G, G*t
  double *cpre0, *cpre1;  // [64] per changepoint: owner thread's sum before its first row
  double *rrw;      // [NW]
  double *gout;     // [128]
  double *fout;     // [4]
  double *sig;      // [4] sigma, 1/sigma^2 of the published point; [2] = this series' tau
  double *gpart;    // [NW][NSET*KMAX] per-wave beta-gradient totals
  double *pd, *pz;  // [128] polish direction / scratch (two parameter words)
  int *cpl;         // [64] per changepoint: owner thread
  int *qmap;        // [64]
  int *flag;        // [4] loop control
  double *ctc, *csg, *csm, *csa;  // [64] t_change[j], sigmas[f], s_m[f], s_a[f] (0 past the end)
  double *U;        // union region
  LbLds<ModeTr<MODE>::PW> *lb; // U view (Stan phase)
  int LD;           // stride of the polish matrix A in U
  double *pmt, *prho;  // polish, logistic: [32][32] d m_s / d theta, [32] segment sums
  double *hst;         // polish: packed upper triangle of the undamped Hessian (FitKArgs.hstash)
  static __host__ __device__ size_t fixed_doubles(int ny) {
    return (size_t)ny + 64 * 4 + 2 * KMAX + 2 * NL + 2 * NW + 128 + NW + 128 + 4 + 4 +
           (size_t)NW * NSET * KMAX + 256 + 32 + 32 + 4 + 4 * 64;
  }
  // polish region: A (P rows + 8 padding rows, stride LD) overlapping the
  // tile-reduction buffer, then the logistic tables
  static __host__ __device__ size_t polish_head_doubles(int P) {
    const size_t a = (size_t)(P + 8) * (size_t)(P | 1);
    const size_t red = (size_t)NTILE * 4 * 64;
    return ((a > red ? a : red) + 1) & ~(size_t)1;
  }
  // logistic tables after the polish matrix, then (optional) the stash of the
  // undamped Hessian's upper triangle (polish_run: the damped first step's
  // Hessian serves the next, undamped QP without a recomputation)
  static __host__ __device__ size_t logi_doubles() {
    return ((MODE & PF_MODE_LOGI) != 0) ? (32 * 32 + 32) : 0;
  }
  static __host__ __device__ size_t stash_doubles(int P) { return (size_t)P * (P + 1) / 2; }
  static __host__ __device__ size_t union_bytes(int P, int S, bool polish, bool stash = false) {
    (void)S;
    const size_t lbb = sizeof(LbLds<ModeTr<MODE>::PW>) + 16;
    if (!polish) return lbb;
    const size_t hm = (polish_head_doubles(P) + logi_doubles() + (stash ? stash_doubles(P) : 0)) *
                      sizeof(double);
    return lbb > hm ? lbb : hm;
  }
  static __host__ __device__ size_t bytes(int ny, int P, int S, bool polish, bool stash = false) {
    return fixed_doubles(ny) * sizeof(double) + union_bytes(P, S, polish, stash) + 64;
  }
  __device__ void carve(char *base, int ny, int P) {
    double *p = reinterpret_cast<double *>(base);
    y = p; p += ny;
    th = p; p += 128;
    kseg = p; p += 64;
    mseg = p; p += 64;
    bm = p; p += KMAX;
    ba = p; p += KMAX;
    sfx0 = p; p += NL;
    sfx1 = p; p += NL;
    wt0 = p; p += NW;
    wt1 = p; p += NW;
    cpre0 = p; p += 64;
    cpre1 = p; p += 64;
    rrw = p; p += NW;
    gout = p; p += 128;
    fout = p; p += 4;
    sig = p; p += 4;
    gpart = p; p += (size_t)NW * NSET * KMAX;
    pd = p; p += 128;
    pz = p; p += 128;
    cpl = reinterpret_cast<int *>(p); p += 32;
    qmap = reinterpret_cast<int *>(p); p += 32;
    flag = reinterpret_cast<int *>(p); p += 4;
    ctc = p; p += 64;
    csg = p; p += 64;
    csm = p; p += 64;
    csa = p; p += 64;
    // 16-byte align U via offsets from the LDS base (keeps the address space)
    size_t off = (size_t)(reinterpret_cast<char *>(p) - base);
    off = (off + 15) & ~(size_t)15;
    U = reinterpret_cast<double *>(base + off);
    lb = reinterpret_cast<LbLds<ModeTr<MODE>::PW> *>(U);
    LD = P | 1;
    pmt = U + polish_head_doubles(P);
    prho = pmt + 32 * 32;
    hst = pmt + logi_doubles();
  }
};

// UPSTREAM logistic_gamma (prophet.stan): with k_s = k + sum_{j<s} delta_j in
// lane s (s <= S) and t_change_s in lane s, returns the segment offsets
// m_0 = m, m_{s+1} = m_s + (t_s - m_s)(1 - k_s/k_{s+1}) in lane s — Stan's
// sequential order (one uniform FP64 chain; the ratios are lane-parallel).
__device__ __forceinline__ double logistic_mseg(double kl, double tcl, double m, int S) {
  const int lane = pf_lane();
  const double kn = __shfl(kl, (lane + 1) & 63, 64);
  const double rho = (lane < S) ? kl / kn : 0.0;
  double mcur = m, ml = (lane == 0) ? m : 0.0;
  for (int s = 0; s < S; ++s) {
    const double tcs = readlane_f64(tcl, s), r = readlane_f64(rho, s);
    mcur = mcur + (tcs - mcur) * (1.0 - r);
    if (lane == s + 1) ml = mcur;
  }
  return ml;
}

template <int NW, int KMAX, int MODE>
__device__ __forceinline__ void publish_theta(const FitKArgs &a, FitSmem<NW, KMAX, MODE> &sm,
                                              const PV<ModeTr<MODE>::PW> &xv) {
  constexpr int PW = ModeTr<MODE>::PW;
  const int lane = pf_lane();
  if (pf_wave() != 0) return;
  const int P = a.P, S = a.S, K = a.K;
  const double x = xv[0];
#pragma unroll
  for (int h = 0; h < PW; ++h)
    if (lane + 64 * h < P) sm.th[lane + 64 * h] = xv[h];
  const double k = readlane_f64(x, 0), m = readlane_f64(x, 1);
  // delta_j sits in lane 2+j
  const double dj = __shfl(x, (lane + 2) & 63, 64);
  const double dval = (lane < S) ? dj : 0.0;
  const double tcd = sm.ctc[lane] * dval;
  const double cd = wave_prefix_sum(dval);   // inclusive: sum_{j<=lane}
  const double ctd = wave_prefix_sum(tcd);
  // kseg[s] = k + sum_{j<s} delta_j ; mseg[s] = m - sum_{j<s} tc_j delta_j
  const double cd_ex = wave_shift_up1(cd);
  const double ctd_ex = wave_shift_up1(ctd);
  const double kl = k + (lane == 0 ? 0.0 : cd_ex);
  if constexpr ((MODE & PF_MODE_LOGI) != 0) {
    const double ml = logistic_mseg(kl, sm.ctc[lane], m, S);
    if (lane <= S) {
      sm.kseg[lane] = kl;
      sm.mseg[lane] = ml;
    }
  } else if (lane <= S) {
    sm.kseg[lane] = kl;
    sm.mseg[lane] = m - (lane == 0 ? 0.0 : ctd_ex);
  }
  double bval = __shfl(x, (lane + 3 + S) & 63, 64);
  if constexpr (PW > 1) {
    const double b1 = __shfl(xv[1], (lane + 3 + S) & 63, 64);
    if (lane + 3 + S >= 64) bval = b1;
  }
  if (lane < KMAX) {
    const double bv = (lane < K) ? bval : 0.0;
    sm.bm[lane] = bv * sm.csm[lane];
    sm.ba[lane] = bv * sm.csa[lane];
  }
  if (lane == 2 + S) {
    const double sigma = exp(x);
    sm.sig[0] = sigma;
    sm.sig[1] = 1.0 / (sigma * sigma);
  }
}

// per-lane problem constants -> LDS once per kernel (every thread calls; the
// caller's next barrier publishes them)
template <int NW, int KMAX, int MODE>
__device__ __forceinline__ void load_consts(const FitKArgs &a, FitSmem<NW, KMAX, MODE> &sm) {
  const int i = threadIdx.x;
  if (i < 64) {
    sm.ctc[i] = (i < a.S) ? a.t_change[i] : 0.0;
    const double *sg = a.sigmas_series ? a.sigmas_series + (size_t)blockIdx.x * a.K : a.sigmas;
    sm.csg[i] = (i < a.K) ? sg[i] : 1.0;
    if (i == 0) sm.sig[2] = a.tau_series ? a.tau_series[blockIdx.x] : a.tau;
    sm.csm[i] = (i < a.K) ? a.s_m[i] : 0.0;
    sm.csa[i] = (i < a.K) ? a.s_a[i] : 0.0;
  }
}

// Wave totals of N per-lane values stored to dst[0..N) (chunks of <= 64).
template <int N, int C0>
__device__ __forceinline__ void transpose_store(const double (&v)[N], double *dst) {
  constexpr int CH = (N - C0 > 64) ? 64 : N - C0;
  double w[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) w[i] = v[C0 + i];
  const double t = wave_transpose_sum<CH>(w);
  const int lane = pf_lane();
  const int idx = transpose_index<CH>(lane);
  if (idx < CH && (CH > 32 || (lane & 1) == 0)) dst[C0 + idx] = t;
  if constexpr (C0 + CH < N) transpose_store<N, C0 + CH>(v, dst);
}

// Row pass of one evaluation (every wave; theta already published).
// Thread L owns the contiguous natural rows [L*R, L*R + R) (lane-blocked
// grid, coalesced loads) and accumulates, in registers: the residual sum of
// squares, its beta-gradient partials, and the running sums of
// G = r(1 + Xb_m) and G*t.  The changepoint gradient needs suffix sums of
// G / G*t from each changepoint's first row; the owner thread records its
// running sums just before that row (cpre), and one scan over thread totals
// per evaluation (sfx, wt) completes them in eval_assemble.  Leaves its
// partial results in LDS; the caller synchronises.
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__device__ __forceinline__ void eval_rows(const FitKArgs &a, FitSmem<NW, KMAX, MODE> &sm) {
  const int lane = pf_lane(), wave = pf_wave();
  constexpr int NL = NW * 64;
  const int L = threadIdx.x;
  const int K = a.K, T = a.T, R = a.R, TQ = a.TQ;
  PF_STAMP(1);
  double gbm[KMAX], gba[KMAX];
#pragma unroll
  for (int f2 = 0; f2 < KMAX; ++f2) {
    gbm[f2] = 0.0;
    gba[f2] = 0.0;
  }
  // beta coefficients in registers for the whole pass (uniform values)
  double lbm[KMAX], lba[KMAX];
#pragma unroll
  for (int f2 = 0; f2 < KMAX; ++f2) {
    lbm[f2] = ((MODE & 3) != MODE_ADD) ? sm.bm[f2] : 0.0;
    lba[f2] = ((MODE & 3) != MODE_MULT) ? sm.ba[f2] : 0.0;
  }
  const double th_m = sm.th[1];
  const bool linear = (a.growth == PF_GROWTH_LINEAR);
  constexpr bool logistic = (MODE & PF_MODE_LOGI) != 0;
  const double *capr = logistic ? a.cap_scaled + (size_t)blockIdx.x * a.Tp : nullptr;
  double rr = 0.0, acc0 = 0.0, acc1 = 0.0;
  RowIn cur;
  if (R > 0) load_rowp<O0, O1, O2>(a, L, cur);
#ifdef PF_ROW_PF2
  // rows loaded two ahead (the grid copy is an L2 hit; one row of FP64 work
  // does not cover its latency)
  RowIn nx1;
  if (R > 1) load_rowp<O0, O1, O2>(a, NL + L, nx1);
#endif
  for (int r = 0; r < R; ++r) {
    const int q = r * NL + L;       // lane-blocked position
    const int i = L * R + r;        // natural row
    RowIn nxt;
#ifdef PF_ROW_PF2
    if (r + 2 < R) load_rowp<O0, O1, O2>(a, q + 2 * NL, nxt);
#else
    if (r + 1 < R) load_rowp<O0, O1, O2>(a, q + NL, nxt);
#endif
    const bool valid = i < T;
    const double ti = cur.t;
    const int sg = cur.seg;
    double xf[KMAX];
    row_features_from<KMAX, O0, O1, O2>(cur, a.XTP, TQ, K, q, xf);
    double xm[4] = {0.0, 0.0, 0.0, 0.0}, xa[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int f2 = 0; f2 < KMAX; ++f2) {
      if constexpr ((MODE & 3) != MODE_ADD) xm[f2 & 3] = fma(xf[f2], lbm[f2], xm[f2 & 3]);
      if constexpr ((MODE & 3) != MODE_MULT) xa[f2 & 3] = fma(xf[f2], lba[f2], xa[f2 & 3]);
    }
    const double xbm = (xm[0] + xm[1]) + (xm[2] + xm[3]);
    const double xba = (xa[0] + xa[1]) + (xa[2] + xa[3]);
    // trend: linear k_s t + m_s; logistic cap sigma(k_s (t - m_s)); flat m
    double tr, lgs = 0.0, capi = 0.0;
    if constexpr (logistic) {
      capi = valid ? capr[i] : 0.0;
      lgs = 1.0 / (1.0 + exp(-(sm.kseg[sg] * (ti - sm.mseg[sg]))));
      tr = capi * lgs;
    } else {
      tr = linear ? fma(sm.kseg[sg], ti, sm.mseg[sg]) : th_m;
    }
    const double u = 1.0 + xbm;
    const double mu = fma(tr, u, xba);
    const double res = valid ? (sm.y[q] - mu) : 0.0;
    rr = fma(res, res, rr);
    const double G = res * u;
    const double cm = res * tr;
    // per-row terms of the changepoint-block gradient, summed from each
    // changepoint's first row (linear: G, G t; logistic, oracle PM/PK:
    // -a k_s, a (t - m_s) with a = G cap sigma (1 - sigma))
    double A0 = G, A1 = G * ti;
    if constexpr (logistic) {
      const double aa = G * capi * lgs * (1.0 - lgs);
      A0 = -aa * sm.kseg[sg];
      A1 = aa * (ti - sm.mseg[sg]);
    }
#pragma unroll
    for (int f2 = 0; f2 < KMAX; ++f2) {
      if constexpr ((MODE & 3) != MODE_ADD) gbm[f2] = fma(xf[f2], cm, gbm[f2]);
      if constexpr ((MODE & 3) != MODE_MULT) gba[f2] = fma(xf[f2], res, gba[f2]);
    }
    // changepoints j in [sprev, sg) are first active at this row
    if (valid && sg > cur.sprev) {
      for (int j = cur.sprev; j < sg; ++j) {
        sm.cpre0[j] = acc0;
        sm.cpre1[j] = acc1;
        sm.cpl[j] = L;
      }
    }
    acc0 += A0;
    acc1 += A1;
#ifdef PF_ROW_PF2
    cur = nx1;
    nx1 = nxt;
#else
    cur = nxt;
#endif
  }
  PF_STAMP(2);
  // thread totals -> inclusive suffix within the wave + wave totals
  double w0, w1;
  const double s0 = wave_suffix_sum(acc0, w0);
  const double s1 = wave_suffix_sum(acc1, w1);
  sm.sfx0[L] = s0;
  sm.sfx1[L] = s1;
  rr = wave_sum(rr);
  if (lane == 0) {
    sm.wt0[wave] = w0;
    sm.wt1[wave] = w1;
    sm.rrw[wave] = rr;
  }
  // beta-gradient partials: transposed in-register reduction, one total per lane
  constexpr int NS = ((MODE & 3) == MODE_MIXED) ? 2 : 1;
  double vv[NS * KMAX];
#pragma unroll
  for (int f2 = 0; f2 < KMAX; ++f2) {
    if constexpr ((MODE & 3) == MODE_MULT) vv[f2] = gbm[f2];
    else if constexpr ((MODE & 3) == MODE_ADD) vv[f2] = gba[f2];
    else { vv[f2] = gbm[f2]; vv[KMAX + f2] = gba[f2]; }
  }
  transpose_store<NS * KMAX, 0>(vv, sm.gpart + (size_t)wave * NS * KMAX);
  PF_STAMP(3);
}

// Sums of two per-lane values over the wave in one 6-level pass (a is
// reduced in lanes 0..31, b in lanes 32..63); uniform results via readlane.
__device__ __forceinline__ void wave_sum2(double a, double b, double &ta, double &tb) {
  double w = pair_add32(a, b);
  w += shfl_xor_f64<16>(w);
  w += shfl_xor_f64<8>(w);
  w += shfl_xor_f64<4>(w);
  w += shfl_xor_f64<2>(w);
  w += shfl_xor_f64<1>(w);
  ta = readlane_f64(w, 0);
  tb = readlane_f64(w, 32);
}

// Wave 0 after the row pass (and a barrier): objective f and gradient g at
// this lane's parameter x (lane p < P), and gp = g . pdir (the line search's
// directional derivative; pass pdir = 0 if unused).  Returns true if f or g
// is not finite (Stan ModelAdaptor error -> line-search retreat).
template <int NW, int KMAX, int MODE>
__device__ __forceinline__ bool eval_assemble(const FitKArgs &a, FitSmem<NW, KMAX, MODE> &sm,
                                              const PV<ModeTr<MODE>::PW> &xv,
                                              const PV<ModeTr<MODE>::PW> &pdir, double &f,
                                              PV<ModeTr<MODE>::PW> &g, double &gp) {
  constexpr int PW = ModeTr<MODE>::PW;
  const int lane = pf_lane();
  const double x = xv[0];
  const int P = a.P, S = a.S, T = a.T;
  const bool linear = (a.growth == PF_GROWTH_LINEAR);
  double rrt = 0.0, tot0 = 0.0, tot1 = 0.0;
#pragma unroll
  for (int w2 = 0; w2 < NW; ++w2) {
    rrt += sm.rrw[w2];
    tot0 += sm.wt0[w2];
    tot1 += sm.wt1[w2];
  }
  const double sigma = sm.sig[0], inv_s2 = sm.sig[1], tau = sm.sig[2];
  const double ls = x;  // meaningful in lane 2+S only
  double gv = 0.0, fterm = 0.0;
  const int p = lane;
  // logistic: segment sums PM_s, PK_s (lane s) from the changepoint suffix
  // sums, then reverse mode through logistic_gamma exactly in the oracle's
  // order (orc_objective): uniform chains over s, lane-parallel otherwise.
  constexpr bool logistic = (MODE & PF_MODE_LOGI) != 0;
  double gkL = 0.0, gmL = 0.0, gdL = 0.0;
  if constexpr (logistic) {
    double su0 = 0.0, su1 = 0.0;
    if (lane < S) {
      const int Lj = sm.cpl[lane];
      const int wj = Lj >> 6;
      double l0 = 0.0, l1 = 0.0;
#pragma unroll
      for (int w2 = 0; w2 < NW; ++w2)
        if (w2 > wj) { l0 += sm.wt0[w2]; l1 += sm.wt1[w2]; }
      su0 = (sm.sfx0[Lj] + l0) - sm.cpre0[lane];
      su1 = (sm.sfx1[Lj] + l1) - sm.cpre1[lane];
    }
    // segment s = [first row of cp s-1, first row of cp s)
    const double pu0 = wave_shift_up1(su0), pu1 = wave_shift_up1(su1);
    const double PMs = (lane == 0 ? tot0 : pu0) - (lane < S ? su0 : 0.0);
    const double PKs = (lane == 0 ? tot1 : pu1) - (lane < S ? su1 : 0.0);
    const double ks = (lane <= S) ? sm.kseg[lane] : 1.0;
    const double kn = __shfl(ks, (lane + 1) & 63, 64);
    const double ms = (lane <= S) ? sm.mseg[lane] : 0.0;
    const double tcs = sm.ctc[lane];
    const double rho = (lane < S) ? ks / kn : 0.0;
    double PMt = readlane_f64(PMs, S), bar_l = 0.0;
    for (int i = S - 1; i >= 0; --i) {
      const double bar = PMt;
      if (lane == i) bar_l = bar;
      PMt = readlane_f64(PMs, i) + bar;
      PMt += bar * (-(1.0 - readlane_f64(rho, i)));
    }
    gmL = PMt;
    // PK[i] += bar_i (-(t_i - m_i)/k_{i+1});  PK[i+1] += bar_i (t_i - m_i) k_i / k_{i+1}^2
    const double dtm = tcs - ms;
    const double t1 = (lane < S) ? bar_l * (-dtm / kn) : 0.0;
    const double t2 = (lane < S) ? bar_l * (dtm * ks / (kn * kn)) : 0.0;
    const double PKf = (PKs + t1) + wave_shift_up1(t2);
    // gd[s-1] = sum_{s' >= s} PK[s'] (s = S..1), gk = that + PK[0]
    double sk = 0.0;
    for (int s2 = S; s2 >= 1; --s2) {
      sk += readlane_f64(PKf, s2);
      if (lane == s2 + 1) gdL = sk;
    }
    gkL = sk + readlane_f64(PKf, 0);
  }
  if (p == 0) {
    const double k = x;
    const double gk = logistic ? gkL : (linear ? tot1 : 0.0);
    gv = -inv_s2 * gk + k / 25.0;
    fterm = k * k / 50.0;
  } else if (p == 1) {
    const double m = x;
    const double gm = logistic ? gmL : tot0;
    gv = -inv_s2 * gm + m / 25.0;
    fterm = m * m / 50.0;
  } else if (p < 2 + S && logistic) {
    const double d = x;
    const double sg = (d > 0.0) - (d < 0.0);
    gv = -inv_s2 * gdL + sg / tau;
    fterm = fabs(d) / tau;
  } else if (p < 2 + S) {
    // suffix sums from changepoint j's first row: owner thread's inclusive
    // within-wave suffix + later waves - the owner's sum before that row
    const int j = p - 2;
    const int Lj = sm.cpl[j];
    const int wj = Lj >> 6;
    double l0 = 0.0, l1 = 0.0;
#pragma unroll
    for (int w2 = 0; w2 < NW; ++w2)
      if (w2 > wj) { l0 += sm.wt0[w2]; l1 += sm.wt1[w2]; }
    const double su0 = (sm.sfx0[Lj] + l0) - sm.cpre0[j];
    const double su1 = (sm.sfx1[Lj] + l1) - sm.cpre1[j];
    const double gdel = su1 - sm.ctc[j] * su0;
    const double d = x;
    const double sg = (d > 0.0) - (d < 0.0);
    gv = (linear ? -inv_s2 * gdel : 0.0) + sg / tau;
    fterm = fabs(d) / tau;
  } else if (p == 2 + S) {
    gv = (double)T - inv_s2 * rrt + 4.0 * sigma * sigma;
    fterm = 2.0 * sigma * sigma + (double)T * ls;
  }
  // beta f2 (parameter 3 + S + f2): Xb prior + the per-wave partials
  auto beta_term = [&](int f2, double bv, double &gb, double &fb) {
    constexpr int NS = ((MODE & 3) == MODE_MIXED) ? 2 : 1;
    const double sgm = sm.csg[f2];
    double gm = 0.0, ga = 0.0;
#pragma unroll
    for (int w2 = 0; w2 < NW; ++w2) {
      const double *gq = sm.gpart + (size_t)w2 * NS * KMAX;
      if constexpr ((MODE & 3) == MODE_MULT) gm += gq[f2];
      else if constexpr ((MODE & 3) == MODE_ADD) ga += gq[f2];
      else { gm += gq[f2]; ga += gq[KMAX + f2]; }
    }
    double gl = 0.0;
    if ((MODE & 3) != MODE_ADD) gl += sm.csm[f2] * gm;
    if ((MODE & 3) != MODE_MULT) gl += sm.csa[f2] * ga;
    gb = -inv_s2 * gl + bv / (sgm * sgm);
    fb = bv * bv / (2.0 * sgm * sgm);
  };
  if (p > 2 + S && p < P) beta_term(p - 3 - S, x, gv, fterm);
  g[0] = (p < P) ? gv : 0.0;
  bool bad = (p < P && !isfinite(gv));
  double gpl = g[0] * pdir[0];
  if constexpr (PW > 1) {
    const int p1 = lane + 64;
    double g1 = 0.0, f1 = 0.0;
    if (p1 < P) beta_term(p1 - 3 - S, xv[1], g1, f1);
    g[1] = (p1 < P) ? g1 : 0.0;
    if (p1 < P && !isfinite(g1)) bad = true;
    fterm += f1;
    gpl = fma(g[1], pdir[1], gpl);
  }
  double fs;
  wave_sum2(fterm, gpl, fs, gp);
  f = fs + 0.5 * rrt * inv_s2;
  if (!isfinite(f)) bad = true;
  return __ballot(bad) != 0ull;
}

// One collective evaluation of f(theta) = -log posterior and its gradient
// (K2 / polish).  Every thread of the workgroup must call it.  `x` is this
// lane's parameter (lane p < P); returns f in every thread and g (lane p).
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__device__ bool eval_collective(const FitKArgs &a, FitSmem<NW, KMAX, MODE> &sm,
                                const PV<ModeTr<MODE>::PW> &x, double &f, PV<ModeTr<MODE>::PW> &g) {
  constexpr int PW = ModeTr<MODE>::PW;
  const int lane = pf_lane(), wave = pf_wave();
  PF_STAMP(0);
  publish_theta<NW, KMAX, MODE>(a, sm, x);
  __syncthreads();
  eval_rows<NW, KMAX, O0, O1, O2, MODE>(a, sm);
  __syncthreads();
  if (wave == 0) {
    double fw, gpw;
    PV<PW> gw;
    const bool badw = eval_assemble<NW, KMAX, MODE>(a, sm, x, pv_zero<PW>(), fw, gw, gpw);
#pragma unroll
    for (int h = 0; h < PW; ++h) sm.gout[lane + 64 * h] = gw[h];
    if (lane == 0) {
      sm.fout[0] = fw;
      sm.fout[1] = badw ? 1.0 : 0.0;
    }
  }
  __syncthreads();
  f = sm.fout[0];
#pragma unroll
  for (int h = 0; h < PW; ++h) g[h] = sm.gout[lane + 64 * h];
  const bool bad = sm.fout[1] != 0.0;
  __syncthreads();
  PF_STAMP(4);
  return bad;
}
// single-word form (polish: P <= 64)
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__device__ __forceinline__ bool eval_collective1(const FitKArgs &a, FitSmem<NW, KMAX, MODE> &sm, double x,
                                                 double &f, double &g) {
  static_assert(ModeTr<MODE>::PW == 1, "polish is single-word");
  PV<1> xv, gv;
  xv[0] = x;
  const bool bad = eval_collective<NW, KMAX, O0, O1, O2, MODE>(a, sm, xv, f, gv);
  g = gv[0];
  return bad;
}

template <int NW, int KMAX, int MODE>
__device__ __forceinline__ void load_y(const FitKArgs &a, FitSmem<NW, KMAX, MODE> &sm, int s) {
  // lane-blocked copy: position r*NL + L holds natural row L*R + r
  const double *ys = a.y_scaled + (size_t)s * a.Tp;
  constexpr int NL = NW * 64;
  const int L = threadIdx.x;
  for (int r = 0; r < a.R; ++r) {
    const int i = L * a.R + r;
    sm.y[r * NL + L] = (i < a.T) ? ys[i] : 0.0;
  }
  load_consts<NW, KMAX, MODE>(a, sm);
}

// ---------------------------------------------------------------- K2 kernel
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__global__ __launch_bounds__(NW * 64) void k_objgrad(FitKArgs a0) {
  FitKArgs a = a0;
  if (a0.grid_of) bind_grid<NW * 64>(a, blockIdx.x);
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  FitSmem<NW, KMAX, MODE> sm;
  sm.carve(smem_raw, a.TQ, a.P);
  const int s = blockIdx.x, lane = pf_lane();
  constexpr int PW = ModeTr<MODE>::PW;
  load_y<NW, KMAX, MODE>(a, sm, s);
  PV<PW> x, g;
#pragma unroll
  for (int h = 0; h < PW; ++h) x[h] = (lane + 64 * h < a.P) ? a.theta[(size_t)s * a.P + lane + 64 * h] : 0.0;
  __syncthreads();
  double f;
  const bool bad = eval_collective<NW, KMAX, O0, O1, O2, MODE>(a, sm, x, f, g);
  if (threadIdx.x < 64) {
#pragma unroll
    for (int h = 0; h < PW; ++h)
      if (lane + 64 * h < a.P) a.g_out[(size_t)s * a.P + lane + 64 * h] = g[h];
    if (lane == 0) a.f_out[s] = bad ? NAN : f;
  }
}

// ---------------------------------------------------------------- L-BFGS (Stan 2.19 restatement)
__device__ __forceinline__ double cubic_interp0(double df0, double x1, double f1, double df1,
                                                double loX, double hiX) {
#ifdef PF_FAST_CUBIC
  // two reciprocals instead of nine divisions (Stan's CubicInterp values up
  // to rounding)
  const double ix = 1.0 / x1;
  const double c3 = (-12 * f1 + 6 * x1 * (df0 + df1)) * (ix * ix * ix);
  const double c2 = -(4 * df0 + 2 * df1) * ix + 6 * f1 * (ix * ix);
  const double c1 = df0;
  const double t_s = sqrt(c2 * c2 - 2.0 * c1 * c3);
  const double ic3 = 1.0 / c3;
  const double s1 = -(c2 + t_s) * ic3;
  const double s2 = -(c2 - t_s) * ic3;
  const double c33 = c3 * (1.0 / 3.0);
  auto poly = [&](double x) { return x * (x * (x * c33 + c2) * 0.5 + c1); };
#else
  const double c3 = (-12 * f1 + 6 * x1 * (df0 + df1)) / (x1 * x1 * x1);
  const double c2 = -(4 * df0 + 2 * df1) / x1 + 6 * f1 / (x1 * x1);
  const double c1 = df0;
  const double t_s = sqrt(c2 * c2 - 2.0 * c1 * c3);
  const double s1 = -(c2 + t_s) / c3;
  const double s2 = -(c2 - t_s) / c3;
  auto poly = [&](double x) { return x * (x * (x * c3 / 3.0 + c2) / 2.0 + c1); };
#endif
  double tmpF, minF, minX;
  minF = poly(loX);
  minX = loX;
  tmpF = poly(hiX);
  if (tmpF < minF) { minF = tmpF; minX = hiX; }
  if (loX < s1 && s1 < hiX) {
    tmpF = poly(s1);
    if (tmpF < minF) { minF = tmpF; minX = s1; }
  }
  if (loX < s2 && s2 < hiX) {
    tmpF = poly(s2);
    if (tmpF < minF) { minF = tmpF; minX = s2; }
  }
  return minX;
}

__device__ __forceinline__ double cubic_interp(double x0, double f0, double df0, double x1,
                                               double f1, double df1, double loX, double hiX) {
  return x0 + cubic_interp0(df0, x1 - x0, f1 - f0, df1, loX - x0, hiX - x0);
}

#define PF_HIST 5

// Reverse-communication restatement of Stan's BFGSMinimizer<LBFGSUpdate>::step
// + WolfeLineSearch + WolfLSZoom (same control flow as oracle/stan_lbfgs.c),
// written as a state machine so that the collective evaluation has exactly
// one call site (keeps the workgroup's register budget at 2+ waves/SIMD).
// All waves run it redundantly; vectors are one parameter per lane.
enum LbState {
  LB_INIT = 0, LB_NEW_ITER, LB_LS_START, LB_TRY, LB_TRY_RES, LB_ZOOM_ITER, LB_ZOOM_RES,
  LB_LS_FAIL, LB_LS_OK, LB_DONE
};

struct LbScalars {
  double fk, fk1, fq, alpha, alphak_1, gammak;
  double dfp, c1dfp, c2dfp, alpha0, alpha1, prevF, prevDFp;
  double alo, aloF, aloDFp, ahi, ahiF, ahiDFp;
  double lastDFp;   // g_k . p_{k-1}  (directional derivative at acceptance)
  double dfp_prev;  // g_{k-1} . p_{k-1} (dfp of the accepted line search)
  double dfp_next;  // g_k . p_k = -g' H g of the new direction
  int itNum, resetB, nits, lsRestarts, zit, hcount, ret, n_eval, head;
};

template <int PW>
__device__ __forceinline__ double ddot(const PV<PW> &u, const PV<PW> &v) {
  double s = u[0] * v[0];
#pragma unroll
  for (int h = 1; h < PW; ++h) s = fma(u[h], v[h], s);
  return wave_sum(s);
}
// (a mod H) for 0 <= a < 2H without an integer division
__device__ __forceinline__ int pf_wrap(int a, int H) {
  a = (a >= H) ? a - H : a;
  return (a >= H) ? a - H : a;
}

// Optimizer state kept in LDS (wave 0 only) so it does not compete with the
// evaluation's registers.
template <int PW>
struct LbLds {
  double xk[64 * PW], gk[64 * PW], pk[64 * PW];        // parameter lane + 64 h at [lane + 64 h]
  double hs[PF_HIST][64 * PW], hy[PF_HIST][64 * PW];   // circular, logical j at (head + j) % H
  // compact-form blocks in logical order (oldest = 0), zero beyond the
  // history length so the 5x5 solves run branch-free
  double Rm[PF_HIST][PF_HIST];                // Rm[i][j] = s_i . y_j (i <= j used)
  double YYm[PF_HIST][PF_HIST];               // y_i . y_j
  double rinv[PF_HIST];                       // 1 / (s_i . y_i)
  double av[PF_HIST], bv[PF_HIST];            // s_i . g_k, y_i . g_k at the current iterate
  LbScalars z;
  int state;
  int need;
};

// Advance the machine until it needs an evaluation (returns true, trial point
// in xq) or terminates (returns false).  `bad` / fq / gq are the result of the
// evaluation requested last time.
template <int PW>
__device__ __forceinline__ bool lbfgs_step(const pf_fit_opts &o, LbLds<PW> &L, int &state, LbScalars &z,
                                           PV<PW> &xk, PV<PW> &gk, PV<PW> &pk, PV<PW> &xq, const PV<PW> &gq,
                                           double gpq, bool bad) {
  const int lane = pf_lane();
  const int H = o.history < PF_HIST ? o.history : PF_HIST;
  while (true) {
    switch (state) {
      case LB_INIT:
        if (bad) { z.ret = PF_ST_BADINIT; state = LB_DONE; return false; }
        z.fk = z.fq;
        gk = gq;
#pragma unroll
        for (int h = 0; h < PW; ++h) pk[h] = -gk[h];
        z.itNum = 0;
        z.hcount = 0;
        z.head = 0;
        state = LB_NEW_ITER;
        break;
      case LB_NEW_ITER:
        z.itNum++;
        z.resetB = (z.itNum == 1) ? 1 : 0;
        state = LB_LS_START;
        break;
      case LB_LS_START:
        if (z.itNum > 1 && z.resetB != 2) {
          // Stan: CubicInterp(g_{k-1}.p_{k-1}, alpha_{k-1}, f_k - f_{k-1}, g_k.p_{k-1})
          z.alpha = fmin(1.0, 1.01 * cubic_interp0(z.dfp_prev, z.alphak_1, z.fk - z.fk1, z.lastDFp,
                                                   1e-12, 1.0));
        } else {
          z.alpha = o.init_alpha;
        }
        if (z.resetB) {
#pragma unroll
          for (int h = 0; h < PW; ++h) pk[h] = -gk[h];
          z.dfp = ddot(gk, pk);
        } else {
          z.dfp = z.dfp_next;
        }
        z.c1dfp = 1e-4 * z.dfp;
        z.c2dfp = 0.9 * z.dfp;
        z.alpha0 = 1e-12;
        z.alpha1 = z.alpha;
        z.prevF = z.fk;
        z.prevDFp = z.dfp;
        z.nits = 0;
        z.lsRestarts = 0;
        state = LB_TRY;
        break;
      case LB_TRY:
        if (o.lbfgs_warmup_evals > 0 && z.n_eval >= o.lbfgs_warmup_evals + o.lbfgs_warmup_ls_slack) {
          // warm-up pass out of evaluations inside a line search: end it at
          // the last accepted iterate (the polish takes it from there)
          z.ret = PF_ST_MAXIT; state = LB_DONE; return false;
        }
        if (z.nits >= 20) { state = LB_LS_FAIL; break; }
#pragma unroll
        for (int h = 0; h < PW; ++h) xq[h] = xk[h] + z.alpha1 * pk[h];
        state = LB_TRY_RES;
        return true;
      case LB_TRY_RES: {
        if (bad) {
          if (z.lsRestarts >= 10) { state = LB_LS_FAIL; break; }
          z.alpha1 = 0.5 * (z.alpha0 + z.alpha1);
          z.lsRestarts++;
          state = LB_TRY;
          break;
        }
        z.lsRestarts = 0;
        const double f1 = z.fq;
        const double newDFp = gpq;  // g(x + alpha p) . p, fused into the evaluation
        if ((f1 > z.fk + z.alpha1 * z.c1dfp) || (f1 >= z.prevF && z.nits > 0)) {
          z.alo = z.alpha0; z.aloF = z.prevF; z.aloDFp = z.prevDFp;
          z.ahi = z.alpha1; z.ahiF = f1; z.ahiDFp = newDFp;
          z.zit = 0;
          state = LB_ZOOM_ITER;
        } else if (fabs(newDFp) <= -z.c2dfp) {
          z.alpha = z.alpha1;
          z.lastDFp = newDFp;
          state = LB_LS_OK;
        } else if (newDFp >= 0) {
          z.alo = z.alpha1; z.aloF = f1; z.aloDFp = newDFp;
          z.ahi = z.alpha0; z.ahiF = z.prevF; z.ahiDFp = z.prevDFp;
          z.zit = 0;
          state = LB_ZOOM_ITER;
        } else {
          z.alpha0 = z.alpha1;
          z.prevF = f1;
          z.prevDFp = newDFp;
          z.alpha1 *= 10.0;
          z.nits++;
          state = LB_TRY;
        }
        break;
      }
      case LB_ZOOM_ITER: {
        if (o.lbfgs_warmup_evals > 0 && z.n_eval >= o.lbfgs_warmup_evals + o.lbfgs_warmup_ls_slack) {
          z.ret = PF_ST_MAXIT; state = LB_DONE; return false;
        }
        z.zit++;
        if (fabs(z.alo - z.ahi) < 1e-16) { state = LB_LS_FAIL; break; }
        if (z.zit % 5 == 0) {
          z.alpha = 0.5 * (z.alo + z.ahi);
        } else {
          const double lo = fmin(z.alo, z.ahi), hi = fmax(z.alo, z.ahi);
          z.alpha = cubic_interp(z.alo, z.aloF, z.aloDFp, z.ahi, z.ahiF, z.ahiDFp, lo, hi);
          if (z.alpha < lo + 0.01 * (hi - lo) || z.alpha > hi - 0.01 * (hi - lo))
            z.alpha = 0.5 * (z.alo + z.ahi);
        }
#pragma unroll
        for (int h = 0; h < PW; ++h) xq[h] = xk[h] + z.alpha * pk[h];
        state = LB_ZOOM_RES;
        return true;
      }
      case LB_ZOOM_RES: {
        if (bad) {
          const double lo = fmin(z.alo, z.ahi);
          z.alpha = 0.5 * (z.alpha + lo);
          if (fabs(lo - z.alpha) < 1e-16) { state = LB_LS_FAIL; break; }
#pragma unroll
          for (int h = 0; h < PW; ++h) xq[h] = xk[h] + z.alpha * pk[h];
          return true;  // stay in LB_ZOOM_RES
        }
        const double f1 = z.fq;
        const double newDFp = gpq;
        if (f1 > (z.fk + z.alpha * z.c1dfp) || f1 >= z.aloF) {
          z.ahi = z.alpha; z.ahiF = f1; z.ahiDFp = newDFp;
          state = LB_ZOOM_ITER;
        } else {
          if (fabs(newDFp) <= -z.c2dfp) { z.lastDFp = newDFp; state = LB_LS_OK; break; }
          if (newDFp * (z.ahi - z.alo) >= 0) { z.ahi = z.alo; z.ahiF = z.aloF; z.ahiDFp = z.aloDFp; }
          z.alo = z.alpha; z.aloF = f1; z.aloDFp = newDFp;
          state = LB_ZOOM_ITER;
        }
        break;
      }
      case LB_LS_FAIL:
        if (z.resetB) { z.ret = PF_ST_LSFAIL; state = LB_DONE; return false; }
        z.resetB = 2;
        state = LB_LS_START;
        break;
      case LB_LS_OK: {
        PF_STAMP(10);
        // accepted point = last evaluated (xq, fq, gq); k becomes the newest
        z.fk1 = z.fk;
        z.fk = z.fq;
        PV<PW> sk, yk;
#pragma unroll
        for (int h = 0; h < PW; ++h) {
          sk[h] = xq[h] - xk[h];
          yk[h] = gq[h] - gk[h];
        }
        xk = xq;
        gk = gq;
        z.alphak_1 = z.alpha;
        z.dfp_prev = z.dfp;
        // LBFGSUpdate history after this update: cleared on reset, oldest pair
        // dropped when full; kept pairs are old logical j + drop
        const int m_old = z.resetB ? 0 : z.hcount;
        const int drop = (m_old == H) ? 1 : 0;
        const int nw = m_old - drop;  // logical index of the new pair
        // one fused reduction: gg, ss, sy, yy, s.g, y.g of the new pair and
        // s_j.y, y_j.y of the kept pairs (their s_j.g, y_j.g follow by
        // a_j += s_j.y, b_j += y_j.y since g_new = g_old + y)
        double v[14], r[14];
#pragma unroll
        for (int i = 0; i < 14; ++i) v[i] = 0.0;
#pragma unroll
        for (int h = 0; h < PW; ++h) {
          v[0] = fma(gq[h], gq[h], v[0]);
          v[1] = fma(sk[h], sk[h], v[1]);
          v[2] = fma(sk[h], yk[h], v[2]);
          v[3] = fma(yk[h], yk[h], v[3]);
          v[4] = fma(sk[h], gq[h], v[4]);
          v[5] = fma(yk[h], gq[h], v[5]);
        }
#pragma unroll
        for (int j = 0; j < PF_HIST - 1; ++j) {
#pragma unroll
          for (int h = 0; h < PW; ++h) {
            double sj = 0.0, yj = 0.0;
            if (j < nw) {
              const int slot = pf_wrap(z.head + j + drop, H);
              sj = L.hs[slot][lane + 64 * h];
              yj = L.hy[slot][lane + 64 * h];
            }
            v[6 + 2 * j] = fma(sj, yk[h], v[6 + 2 * j]);
            v[7 + 2 * j] = fma(yj, yk[h], v[7 + 2 * j]);
          }
        }
        wave_sum_multi<14>(v, r);
        PF_STAMP(11);
        const double gg = r[0];
        if (fabs(z.fk1 - z.fk) < o.tol_obj) {
          z.ret = PF_ST_ABSF;
        } else if (sqrt(gg) < o.tol_grad) {
          z.ret = PF_ST_ABSGRAD;
        } else if (sqrt(r[1]) < o.tol_param) {
          z.ret = PF_ST_ABSX;
        } else if (z.itNum >= o.max_iter || (o.lbfgs_warmup_evals > 0 && z.n_eval >= o.lbfgs_warmup_evals)) {
          z.ret = PF_ST_MAXIT;
        } else if (((z.fk1 - z.fk) / fmax(fabs(z.fk1), fmax(fabs(z.fk), 1.0))) <
                   o.tol_rel_obj * 2.220446049250313e-16) {
          z.ret = PF_ST_RELF;
        } else {
          // ---- LBFGSUpdate::update + search_direction in compact
          //      (Byrd-Nocedal-Schnabel) form, equal to Stan's two-loop
          //      recursion in exact arithmetic:
          //        H g = gamma g + S p' - gamma Y u,  u = R^-1 a,
          //        p' = R^-T ((D + gamma Y'Y) u - gamma b),  a = S'g, b = Y'g,
          //      R = upper(S'Y), D = diag(S'Y), gamma = s'y / y'y (newest).
          z.gammak = r[2] / r[3];
          const double gam = z.gammak;
          {
            // lanes (i, j) < 25 rebuild the logical blocks: reset -> zero,
            // drop -> shift up-left by one (zero fill), then the new column
            const int i0 = lane / PF_HIST, j0 = lane - i0 * PF_HIST;
            double rv = 0.0, yv = 0.0, iv = 0.0, aj = 0.0, bj = 0.0;
            if (lane < PF_HIST * PF_HIST && !z.resetB) {
              const int si = i0 + drop, sj = j0 + drop;
              if (si < PF_HIST && sj < PF_HIST) { rv = L.Rm[si][sj]; yv = L.YYm[si][sj]; }
            }
            if (lane < PF_HIST && !z.resetB && lane + drop < PF_HIST) {
              iv = L.rinv[lane + drop];
              aj = L.av[lane + drop];
              bj = L.bv[lane + drop];
            }
            // new column nw / diagonal, and a_j, b_j moved to g_new
            double syi = 0.0, yyi = 0.0, yyj = 0.0;
#pragma unroll
            for (int j = 0; j < PF_HIST - 1; ++j) {
              if (i0 == j) { syi = r[6 + 2 * j]; yyi = r[7 + 2 * j]; }
              if (j0 == j) yyj = r[7 + 2 * j];
            }
            if (lane < PF_HIST * PF_HIST) {
              if (j0 == nw && i0 < nw) { rv = syi; yv = yyi; }
              if (i0 == nw && j0 < nw) { yv = yyj; }
              if (i0 == nw && j0 == nw) { rv = r[2]; yv = r[3]; }
            }
            if (lane < PF_HIST) {
              double sy_l = 0.0, yy_l = 0.0;
#pragma unroll
              for (int j = 0; j < PF_HIST - 1; ++j)
                if (lane == j) { sy_l = r[6 + 2 * j]; yy_l = r[7 + 2 * j]; }
              if (lane < nw) { aj += sy_l; bj += yy_l; }
              if (lane == nw) { aj = r[4]; bj = r[5]; iv = 1.0 / r[2]; }
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (lane < PF_HIST * PF_HIST) { L.Rm[i0][j0] = rv; L.YYm[i0][j0] = yv; }
            if (lane < PF_HIST) { L.rinv[lane] = iv; L.av[lane] = aj; L.bv[lane] = bj; }
          }
          if (drop) z.head = pf_wrap(z.head + 1, H);
          const int slot_new = pf_wrap(z.head + nw, H);
#pragma unroll
          for (int h = 0; h < PW; ++h) {
            L.hs[slot_new][lane + 64 * h] = sk[h];
            L.hy[slot_new][lane + 64 * h] = yk[h];
          }
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
          __builtin_amdgcn_wave_barrier();
          z.hcount = nw + 1;
          // branch-free padded solves (entries past the history are zero)
          double Rr[PF_HIST][PF_HIST], Yr[PF_HIST][PF_HIST], ri[PF_HIST], av[PF_HIST], bv[PF_HIST];
#pragma unroll
          for (int i = 0; i < PF_HIST; ++i) {
            ri[i] = L.rinv[i];
            av[i] = L.av[i];
            bv[i] = L.bv[i];
#pragma unroll
            for (int j = i; j < PF_HIST; ++j) { Rr[i][j] = L.Rm[i][j]; Yr[i][j] = L.YYm[i][j]; }
          }
          double uu[PF_HIST], pp[PF_HIST];
          // u = R^-1 a (back substitution)
#pragma unroll
          for (int i = PF_HIST - 1; i >= 0; --i) {
            double t = av[i];
#pragma unroll
            for (int j = i + 1; j < PF_HIST; ++j) t = fma(-Rr[i][j], uu[j], t);
            uu[i] = t * ri[i];
          }
          // w = (D + gamma Y'Y) u - gamma b ; p' = R^-T w (forward substitution)
#pragma unroll
          for (int i = 0; i < PF_HIST; ++i) {
            double yu = 0.0;
#pragma unroll
            for (int j = 0; j < PF_HIST; ++j) yu = fma(j >= i ? Yr[i][j] : Yr[j][i], uu[j], yu);
            double w = fma(Rr[i][i], uu[i], gam * (yu - bv[i]));
#pragma unroll
            for (int j = 0; j < i; ++j) w = fma(-Rr[j][i], pp[j], w);
            pp[i] = w * ri[i];
          }
          PV<PW> Hg;
#pragma unroll
          for (int h = 0; h < PW; ++h) Hg[h] = gam * gq[h];
          double gHg = gam * gg;
#pragma unroll
          for (int j = 0; j < PF_HIST; ++j) {
            const int sl = pf_wrap(z.head + j, H);
#pragma unroll
            for (int h = 0; h < PW; ++h)
              Hg[h] = fma(pp[j], L.hs[sl][lane + 64 * h], fma(-gam * uu[j], L.hy[sl][lane + 64 * h], Hg[h]));
            gHg = fma(pp[j], av[j], fma(-gam * uu[j], bv[j], gHg));
          }
#pragma unroll
          for (int h = 0; h < PW; ++h) pk[h] = -Hg[h];
          z.dfp_next = -gHg;
          PF_STAMP(12);
          if (gHg / fmax(fabs(z.fk), 1.0) < o.tol_rel_grad * 2.220446049250313e-16)
            z.ret = PF_ST_RELGRAD;
          else
            z.ret = PF_ST_SUCCESS;
        }
        if (z.ret != PF_ST_SUCCESS) { state = LB_DONE; return false; }
        state = LB_NEW_ITER;
        break;
      }
      default:
        return false;
    }
  }
}


// State lives in LDS between evaluations; copy it into registers for the
// step (one batch of independent LDS loads) and write it back at the end.
template <int PW>
__device__ __forceinline__ bool lbfgs_advance(const pf_fit_opts &o, LbLds<PW> &L, PV<PW> &xq, const PV<PW> &gq,
                                              double gpq, bool bad) {
  const int lane = pf_lane();
  PF_STAMP(6);
  LbScalars z = L.z;
  int state = __builtin_amdgcn_readfirstlane(L.state);
  // every scalar of the optimizer is wave-uniform: say so (SGPRs + scalar
  // branches instead of exec-masked control flow)
#ifndef PF_NO_RFL_Z
  {
    static_assert(sizeof(LbScalars) % 4 == 0, "LbScalars words");
    int *w = reinterpret_cast<int *>(&z);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(LbScalars) / 4); ++i) w[i] = __builtin_amdgcn_readfirstlane(w[i]);
  }
#endif
  PV<PW> xk, gk, pk;
#pragma unroll
  for (int h = 0; h < PW; ++h) {
    xk[h] = L.xk[lane + 64 * h];
    gk[h] = L.gk[lane + 64 * h];
    pk[h] = L.pk[lane + 64 * h];
  }
  PF_STAMP(7);
  const bool need = lbfgs_step<PW>(o, L, state, z, xk, gk, pk, xq, gq, gpq, bad);
  PF_STAMP(8);
#pragma unroll
  for (int h = 0; h < PW; ++h) {
    L.xk[lane + 64 * h] = xk[h];
    L.gk[lane + 64 * h] = gk[h];
    L.pk[lane + 64 * h] = pk[h];
  }
  if (lane == 0) {
    L.z = z;
    L.state = state;
  }
  return need;
}


#include "pf_polish.h"
#include "pf_tile.h"

// ---------------------------------------------------------------- K3 kernel
// pass 0: first L-BFGS run; pass > 0: resume the series the polish did not
// certify.  o: this pass's options (iteration cap); warm: the cap is the
// warm-up cap (MAXIT -> WARMUP).
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__device__ __forceinline__ void fit_body(const FitKArgs &a, int pass, const pf_fit_opts &o, bool warm) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  FitSmem<NW, KMAX, MODE> sm;
  sm.carve(smem_raw, a.TQ, a.P);
  const int s = blockIdx.x, lane = pf_lane();
  const int P = a.P;
  double *th_out = a.theta + (size_t)s * P;
  const int st_in = a.status[s];
  if (pass > 0) {
    // resume pass: only series whose polish did not certify the MAP
    if (st_in == PF_ST_CONSTANT || st_in == PF_ST_BADINIT || st_in == PF_ST_MAP) return;
  } else if (st_in == PF_ST_CONSTANT) {
    // Prophet: params = init, sigma_obs = 1e-9; optimizer skipped
    if (threadIdx.x == 0) {
      th_out[2 + a.S] = log(1e-9);
      a.f_out[s] = NAN;
      a.f_stan[s] = NAN;
      a.n_iter[s] = 0;
      a.n_eval[s] = 0;
    }
    return;
  }
  constexpr int PW = ModeTr<MODE>::PW;
  load_y<NW, KMAX, MODE>(a, sm, s);
  LbLds<PW> &L = *sm.lb;
  PV<PW> xq;
#pragma unroll
  for (int h = 0; h < PW; ++h) xq[h] = (lane + 64 * h < P) ? th_out[lane + 64 * h] : 0.0;
  if (pf_wave() == 0) {
    L.state = LB_INIT;
    if (lane == 0) memset(&L.z, 0, sizeof(LbScalars));
#pragma unroll
    for (int h = 0; h < PW; ++h) {
      const int e = lane + 64 * h;
      L.xk[e] = xq[h];
      L.pk[e] = 0.0;
#pragma unroll
      for (int q = 0; q < PF_HIST; ++q) { L.hs[q][e] = 0.0; L.hy[q][e] = 0.0; }
    }
    if (lane < PF_HIST * PF_HIST) { (&L.Rm[0][0])[lane] = 0.0; (&L.YYm[0][0])[lane] = 0.0; }
    if (lane < PF_HIST) { L.rinv[lane] = 0.0; L.av[lane] = 0.0; L.bv[lane] = 0.0; }
    publish_theta<NW, KMAX, MODE>(a, sm, xq);
  }
  __syncthreads();
  // ---- phase A: Stan-faithful L-BFGS (reverse communication).  Per
  // evaluation: row pass (all waves) | barrier | wave 0: assemble f, g ->
  // optimizer step -> publish the next trial point | barrier.
  int n_eval = 0;
  while (true) {
    eval_rows<NW, KMAX, O0, O1, O2, MODE>(a, sm);
    __syncthreads();
    if (pf_wave() == 0) {
      // the workgroup's serial section: the other workgroup on this CU is
      // in its row pass meanwhile (pf_serial_prio)
      pf_serial_prio(true);
      double fq, gpq;
      PV<PW> gq, pkc;
#pragma unroll
      for (int h = 0; h < PW; ++h) pkc[h] = L.pk[lane + 64 * h];
      const bool bad = eval_assemble<NW, KMAX, MODE>(a, sm, xq, pkc, fq, gq, gpq);
      ++n_eval;
      PF_STAMP(4);
      if (lane == 0) { L.z.fq = fq; L.z.n_eval = n_eval; }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const bool need = lbfgs_advance(o, L, xq, gq, gpq, bad);
      if (need) publish_theta<NW, KMAX, MODE>(a, sm, xq);
      if (lane == 0) sm.flag[0] = need ? 1 : 0;
      pf_serial_prio(false);
    }
    __syncthreads();
    PF_STAMP(5);
    if (!__builtin_amdgcn_readfirstlane(sm.flag[0])) break;
  }
  double f = L.z.fk;
  const double f_stan = f;
  int st_stan = L.z.ret;
  const int it_stan = L.z.itNum;
  if (warm && st_stan == PF_ST_MAXIT) st_stan = PF_ST_WARMUP;
  if (threadIdx.x < 64) {
#pragma unroll
    for (int h = 0; h < PW; ++h)
      if (lane + 64 * h < P) th_out[lane + 64 * h] = L.xk[lane + 64 * h];
    if (lane == 0) {
      a.f_out[s] = f;
      if (pass == 0) {
        a.f_stan[s] = f_stan;
        a.n_iter[s] = it_stan;
        a.n_eval[s] = n_eval;
      } else {
        a.n_iter[s] += it_stan;
        a.n_eval[s] += n_eval;
      }
      a.status[s] = st_stan;
    }
  }
}

// ---------------------------------------------------------------- K3b polish kernel
// Separate launch so the Hessian's MFMA accumulators get their own register
// budget (the L-BFGS kernel stays at 2 waves/SIMD).  Reads the Stan-phase
// optimum from theta, re-evaluates f/g there, runs the proximal-Newton polish.
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__device__ __forceinline__ void polish_body(const FitKArgs &a) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  FitSmem<NW, KMAX, MODE> sm;
  sm.carve(smem_raw, a.TQ, a.P);
  constexpr int PW = ModeTr<MODE>::PW;
  const int s = blockIdx.x, lane = pf_lane();
  const int P = a.P;
  const int st = a.status[s];
  if (st == PF_ST_CONSTANT || st == PF_ST_BADINIT || st == PF_ST_MAP) return;
  double *th_out = a.theta + (size_t)s * P;
  load_y<NW, KMAX, MODE>(a, sm, s);
  PV<PW> x, g;
#pragma unroll
  for (int h = 0; h < PW; ++h) x[h] = (lane + 64 * h < P) ? th_out[lane + 64 * h] : 0.0;
  __syncthreads();
  double f;
  const bool bad = eval_collective<NW, KMAX, O0, O1, O2, MODE>(a, sm, x, f, g);
  if (bad) return;
  int n_eval = 1, n_newton = 0;  // polish evaluations are not counted in n_eval[]
  const bool cert = polish_run<NW, KMAX, O0, O1, O2, MODE>(a, sm, x, f, g, n_eval, n_newton);
  PF_BLKV(4, n_newton);
  if (threadIdx.x < 64) {
#pragma unroll
    for (int h = 0; h < PW; ++h)
      if (lane + 64 * h < P) th_out[lane + 64 * h] = x[h];
    if (lane == 0) {
      a.f_out[s] = f;
      if (cert) a.status[s] = PF_ST_MAP;
    }
  }
}

// Exact Hessian of the smooth part at theta (pf_hessian; the polish's model
// without damping): H_out[s][P][P].
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__global__ __launch_bounds__(NW * 64) void k_hessian(FitKArgs a0, double *H_out) {
  FitKArgs a = a0;
  if (a0.grid_of) bind_grid<NW * 64>(a, blockIdx.x);
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  FitSmem<NW, KMAX, MODE> sm;
  sm.carve(smem_raw, a.TQ, a.P);
  constexpr int PW = ModeTr<MODE>::PW;
  const int s = blockIdx.x, lane = pf_lane();
  const int P = a.P, S = a.S;
  load_y<NW, KMAX, MODE>(a, sm, s);
  PV<PW> x, g;
#pragma unroll
  for (int h = 0; h < PW; ++h) x[h] = (lane + 64 * h < P) ? a.theta[(size_t)s * P + lane + 64 * h] : 0.0;
  __syncthreads();
  double f;
  (void)eval_collective<NW, KMAX, O0, O1, O2, MODE>(a, sm, x, f, g);
  PV<PW> gh = g;
  const double c = 1.0 / sm.sig[2];
  if (lane >= 2 && lane < 2 + S) gh[0] = g[0] - c * (double)((x[0] > 0.0) - (x[0] < 0.0));
  hessian_collective<NW, KMAX, O0, O1, O2, MODE>(a, sm, x, gh, 0.0);
  __syncthreads();
  const int LD = sm.LD;
  double *Ho = H_out + (size_t)s * P * P;
  for (int e = threadIdx.x; e < P * P; e += NW * 64) {
    const int i = e / P, j = e - i * P;
    Ho[e] = sm.U[i * LD + j];
  }
}

// Entry points: the first pass and the resume passes are distinct kernels so
// that traces and counters attribute them separately.
// waves per SIMD the register budget targets: 2 for the reference layouts; 1
// (512 registers, no spills) for the holiday / wide layouts, whose long
// (hourly) grids hold one workgroup per CU in LDS anyway
template <int KMAX>
struct FitOcc {
  static constexpr int W = KMAX > 34 ? 1 : 2;
};
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__global__ __launch_bounds__(NW * 64, FitOcc<KMAX>::W) void k_fit(FitKArgs a0) {
  FitKArgs a = a0;
  if (a0.grid_of) bind_grid<NW * 64>(a, blockIdx.x);
  fit_body<NW, KMAX, O0, O1, O2, MODE>(a, a.pass, a.o, a.warm_cap != 0);
}
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__global__ __launch_bounds__(NW * 64, FitOcc<KMAX>::W) void k_fit_resume(FitKArgs a0) {
  FitKArgs a = a0;
  if (a0.grid_of) bind_grid<NW * 64>(a, blockIdx.x);
  fit_body<NW, KMAX, O0, O1, O2, MODE>(a, a.pass, a.o, a.warm_cap != 0);
}
// (The standalone polish at one workgroup per CU with 512 registers — no
// spills — or at three with 168: configs[2] k_polish 24.9 -> 47.4 / 46.4 ms,
// tools/polish_occ_ab.sh; the spilling two-per-CU budget stays.)
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__global__ __launch_bounds__(NW * 64, FitOcc<KMAX>::W) void k_polish(FitKArgs a0) {
  FitKArgs a = a0;
  if (a0.grid_of) bind_grid<NW * 64>(a, blockIdx.x);
  polish_body<NW, KMAX, O0, O1, O2, MODE>(a);
}
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__global__ __launch_bounds__(NW * 64, FitOcc<KMAX>::W) void k_polish_resume(FitKArgs a0) {
  FitKArgs a = a0;
  if (a0.grid_of) bind_grid<NW * 64>(a, blockIdx.x);
  polish_body<NW, KMAX, O0, O1, O2, MODE>(a);
}
// The warm-up hand-off of launch_fitlike — L-BFGS warm-up -> polish, once
// more for uncertified series, then Stan's full rules -> polish — per series
// in one launch: each series moves on to its polish as soon as its own
// L-BFGS phase ends, so the batch's slow fits overlap other series' polish
// instead of the two phases being separated by a grid-wide kernel boundary.
// The two phases are separate (non-inlined) functions so each gets its own
// register allocation: inlined together, the polish's pressure spilled
// values of the L-BFGS evaluation loop.
#ifdef PF_FUSE_INLINE
#define PF_PHASE_ATTR __forceinline__
#else
#define PF_PHASE_ATTR __noinline__
#endif
#ifdef PF_FUSE_INLINE_FIT
#define PF_FIT_PHASE_ATTR __forceinline__
#else
#define PF_FIT_PHASE_ATTR PF_PHASE_ATTR
#endif
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__device__ PF_FIT_PHASE_ATTR void fit_phase(const FitKArgs &a, int pass, int max_iter, bool warm) {
  pf_fit_opts o = a.o;
  o.max_iter = max_iter;
  if (!warm) o.lbfgs_warmup_evals = 0;
  fit_body<NW, KMAX, O0, O1, O2, MODE>(a, pass, o, warm);
}
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__device__ PF_PHASE_ATTR void polish_phase(const FitKArgs &a) {
  polish_body<NW, KMAX, O0, O1, O2, MODE>(a);
}
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__device__ __forceinline__ void fit_polish_passes(const FitKArgs &a) {
  const int W = a.o.lbfgs_warmup;
  for (int ps = 0; ps < 3; ++ps) {
    const bool warm = ps < 2;
    fit_phase<NW, KMAX, O0, O1, O2, MODE>(a, ps, warm ? W : a.o.max_iter, warm);
    __syncthreads();
    if (ps == 0) PF_BLK(3);
    polish_phase<NW, KMAX, O0, O1, O2, MODE>(a);
    __syncthreads();
    const int st = __builtin_amdgcn_readfirstlane(__atomic_load_n(&a.status[blockIdx.x], __ATOMIC_RELAXED));
    if (st == PF_ST_MAP || st == PF_ST_CONSTANT || st == PF_ST_BADINIT) break;
  }
}
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__global__ __launch_bounds__(NW * 64, FitOcc<KMAX>::W) void k_fit_polish(FitKArgs a) {
  if (a.grid_of) {
    // ragged batch: the phases read this series' grid from a private copy
    FitKArgs b = a;
    bind_grid<NW * 64>(b, blockIdx.x);
    fit_polish_passes<NW, KMAX, O0, O1, O2, MODE>(b);
  } else {
    fit_polish_passes<NW, KMAX, O0, O1, O2, MODE>(a);
  }
}

// ============================================================================
// K4+K5: forecast + Monte-Carlo uncertainty (UPSTREAM predict / 0.7.1-1.0
//        sample_predictive_trend Poisson process / nanpercentile 'linear')
// ============================================================================
#define PF_NQ 16  // samples per lane (n_samples <= 1024)

struct PredKArgs {
  int n_series, growth, N, Tf, Tp, K, S, P;
  const double *t, *XT, *t_change;
  const int32_t *seg;
  const double *s_a, *s_m;
  const double *theta, *y_scale;
  int k_lo, k_hi_neg;  // order statistics: lower k_lo,k_lo+1; upper via negation
  float fr_lo, fr_hi;
  uint32_t seed0, seed1;
  float *yhat, *ylo, *yhi, *tr, *trlo, *trhi, *mult, *add;
  int n_comp;
  int comp_col0[PF_MAX_COMP], comp_ncol[PF_MAX_COMP];
  float *comp;
  const uint32_t *series_id;  // RNG stream key per series (NULL: batch index)
  int method;                 // PF_INTERVAL_EXACT / PF_INTERVAL_SAMPLE
  const double *cap;          // [n][Tp] logistic capacity / y_scale on the predicted rows
  float zthr;                 // deterministic-trend rows: tail threshold on the standard
                              // normal draws (0: always the general selection)
  const pf_grid *grids;       // ragged forecasts: series s predicts on grids[grid_of[s]]
  const int32_t *grid_of;     // (NULL: every series on t / XT / seg above)
};

// Ragged forecast: rows / t / features / segments / changepoints of series s's
// own forecast grid (uniform per workgroup).
__device__ __forceinline__ void bind_pred_grid(PredKArgs &a, int s) {
  const int g = __builtin_amdgcn_readfirstlane(a.grid_of[s]);
  const pf_grid *G = a.grids + g;
  a.Tf = __builtin_amdgcn_readfirstlane(G->T);
  a.t = (const double *)rfl_ptr(G->t);
  a.XT = (const double *)rfl_ptr(G->XT);
  a.t_change = (const double *)rfl_ptr(G->t_change);
  a.seg = (const int32_t *)rfl_ptr(G->seg);
}

// numpy _lerp: a + (b-a)*t, or b - (b-a)*(1-t) when t >= 0.5
__device__ __forceinline__ float np_lerp(float a, float b, float t) {
  const float d = b - a;
  return (t >= 0.5f) ? (b - d * (1.0f - t)) : (a + d * t);
}

// Per-series forecast state shared by the two forecast kernels (LDS).
struct PredSeries {
  double kseg[64], mseg[64], bm[64], ba[64];
  double sigma, ysc, lam;
};

// wave 0: theta -> segment rates/offsets, beta*s_m / beta*s_a, sigma, lambda
__device__ __forceinline__ void pred_setup(const PredKArgs &a, int series, PredSeries &ps) {
  const int lane = pf_lane();
  if (pf_wave() != 0) return;
  const int P = a.P, S = a.S, K = a.K;
  const double x = (lane < P) ? a.theta[(size_t)series * P + lane] : 0.0;
  const double x1 = (lane + 64 < P) ? a.theta[(size_t)series * P + 64 + lane] : 0.0;  // P > 64: betas
  const double k = readlane_f64(x, 0), m = readlane_f64(x, 1);
  const double dj = __shfl(x, (lane + 2) & 63, 64);
  const double dval = (lane < S) ? dj : 0.0;
  const double tcd = (lane < S) ? a.t_change[lane] * dval : 0.0;
  const double cd = wave_prefix_sum(dval), ctd = wave_prefix_sum(tcd);
  const double cd_ex = wave_shift_up1(cd), ctd_ex = wave_shift_up1(ctd);
  const double kl = k + (lane == 0 ? 0.0 : cd_ex);
  if (a.growth == PF_GROWTH_LOGISTIC) {
    const double ml = logistic_mseg(kl, (lane < S) ? a.t_change[lane] : 0.0, m, S);
    if (lane <= S) {
      ps.kseg[lane] = kl;
      ps.mseg[lane] = ml;
    }
  } else if (lane <= S) {
    ps.kseg[lane] = kl;
    ps.mseg[lane] = m - (lane == 0 ? 0.0 : ctd_ex);
  }
  const double b0 = __shfl(x, (lane + 3 + S) & 63, 64), b1 = __shfl(x1, (lane + 3 + S) & 63, 64);
  const double bval = (lane + 3 + S < 64) ? b0 : b1;
  const double bv = (lane < K) ? bval : 0.0;
  ps.bm[lane] = bv * ((lane < K) ? a.s_m[lane] : 0.0);
  ps.ba[lane] = bv * ((lane < K) ? a.s_a[lane] : 0.0);
  const double absd = wave_sum(fabs(dval));
  const double ls = readlane_f64(x, 2 + S);
  if (lane == 0) {
    ps.sigma = exp(ls);                   // sigma_obs
    ps.ysc = a.y_scale[series];
    ps.lam = absd / (double)S + 1e-8;     // lambda = mean|delta| + 1e-8 (UPSTREAM)
  }
}

// UPSTREAM sample_predictive_trend: T = t.max() of the frame being predicted
// (rows sorted: the last valid row); the trend of a row is random iff
// growth is linear or logistic, T > 1 and t > 1 (new changepoints live on
// (1, T]).
__device__ __forceinline__ bool pred_row_random(const PredKArgs &a, double ti, double t_max) {
  return a.growth != PF_GROWTH_FLAT && ti > 1.0 && t_max > 1.0;
}

// point trend (scaled units) of a row on the fitted segments
__device__ __forceinline__ double pred_trend(const PredKArgs &a, const PredSeries &ps, int series,
                                             int row, double ti, int sg) {
  if (a.growth == PF_GROWTH_LINEAR) return ps.kseg[sg] * ti + ps.mseg[sg];
  if (a.growth == PF_GROWTH_LOGISTIC)
    return a.cap[(size_t)series * a.Tp + row] / (1.0 + exp(-(ps.kseg[sg] * (ti - ps.mseg[sg]))));
  return ps.mseg[0];
}

// x . (beta s_m) and x . (beta s_a) over the K features of one row, in
// feature order; the loads are issued 16 at a time (one memory latency per
// 16 features instead of one per feature)
__device__ __forceinline__ void pred_row_dot(const PredKArgs &a, const PredSeries &ps, int row,
                                             double &xbm, double &xba) {
  constexpr int CH = 16;
  const int K = a.K;
  for (int f0 = 0; f0 < K; f0 += CH) {
    double xv[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) xv[j] = (f0 + j < K) ? a.XT[(size_t)(f0 + j) * a.Tp + row] : 0.0;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      if (f0 + j < K) {
        xbm += xv[j] * ps.bm[f0 + j];
        xba += xv[j] * ps.ba[f0 + j];
      }
    }
  }
}

// ---- K4: point forecast + components + deterministic-row intervals.
// Grid (ceil(Tf/256), n_series), thread per row.  Under PF_INTERVAL_EXACT
// the interval endpoints of deterministic rows are exact order-statistic
// draws (pf_ostat.h); rows left to k_predict_mc are not written here.
__device__ __forceinline__ void det_row(const PredKArgs &a, const PredSeries &ps, int series,
                                        uint32_t sid, int row, double t_max,
                                        const int *__restrict__ comp_col0,
                                        const int *__restrict__ comp_ncol) {
  const double ysc = ps.ysc;
  const double ti = a.t[row];
  const int sg = a.seg[row];
  double xbm = 0.0, xba = 0.0;
  pred_row_dot(a, ps, row, xbm, xba);
  if (a.comp) {
    // component blocks: contiguous column ranges (UPSTREAM
    // predict_seasonal_components, MAP: the mean); additive parts x y_scale
    for (int b = 0; b < a.n_comp; ++b) {
      double cb = 0.0;
      const int c0 = comp_col0[b], c1 = c0 + comp_ncol[b];
      for (int f = c0; f < c1; ++f) {
        const double xv = a.XT[(size_t)f * a.Tp + row];
        cb += xv * ps.bm[f] + xv * ps.ba[f] * ysc;
      }
      a.comp[((size_t)b * a.n_series + series) * a.Tp + row] = (float)cb;
    }
  }
  const double trs = pred_trend(a, ps, series, row, ti, sg);
  const double trend = trs * ysc;
  const double addt = xba * ysc;
  const double yhat = trend * (1.0 + xbm) + addt;
  const size_t o = (size_t)series * a.Tp + row;
  a.yhat[o] = (float)yhat;
  if (a.tr) a.tr[o] = (float)trend;
  if (a.mult) a.mult[o] = (float)xbm;
  if (a.add) a.add[o] = (float)addt;
  const bool mc = (a.N > 0) && (a.method == PF_INTERVAL_SAMPLE || pred_row_random(a, ti, t_max));
  if (mc) return;
  float ylo = (float)yhat, yhi = (float)yhat;
  if (a.N > 0) {
    // exact joint order statistics of the N noise draws (pf_ostat.h)
    int rk[4] = {a.k_lo + 1, a.k_lo + 2, a.N - a.k_hi_neg - 1, a.N - a.k_hi_neg};
#pragma unroll
    for (int q = 0; q < 4; ++q) rk[q] = min(max(rk[q], 1), a.N);
    pf_rowrng rng{(uint32_t)row, sid, a.seed0, a.seed1, 0u};
    double z[4];
    pf_normal_order_stats(rk, a.N, rng, z);
    const double sd = ps.sigma * ysc;
    const double fl = (double)a.fr_lo, fh = (double)a.fr_hi;
    // numpy _lerp on the sorted samples yhat + sd*z
    const double l0 = yhat + sd * z[0], l1 = yhat + sd * z[1];
    const double h0 = yhat + sd * z[2], h1 = yhat + sd * z[3];
    ylo = (float)((fl >= 0.5) ? l1 - (l1 - l0) * (1.0 - fl) : l0 + (l1 - l0) * fl);
    yhi = (float)((fh >= 0.5) ? h1 - (h1 - h0) * (1.0 - fh) : h0 + (h1 - h0) * fh);
  }
  a.ylo[o] = ylo;
  a.yhi[o] = yhi;
  if (a.tr) { a.trlo[o] = (float)trend; a.trhi[o] = (float)trend; }}

// PF_DET_RPT rows per thread (strided by the block): the per-series setup is
// paid once per 256 * PF_DET_RPT rows
#define PF_DET_RPT 4
// The component column table is indexed at run time: it is read from the
// kernel argument block (a0), never from the thread's copy `a` (a dynamically
// indexed local array lives in scratch: the whole argument struct was
// written to scratch by every thread — 5x the kernel's output bytes).
template <int KMAX>
__global__ __launch_bounds__(256) void k_predict_det(PredKArgs a0) {
  __shared__ PredSeries ps;
  const int series = blockIdx.y;
  PredKArgs a = a0;
  if (a0.grid_of) bind_pred_grid(a, series);
  const uint32_t sid = a.series_id ? a.series_id[series] : (uint32_t)series;
  pred_setup(a, series, ps);
  __syncthreads();
  const double t_max = a.t[a.Tf - 1];
#pragma unroll 1
  for (int r = 0; r < PF_DET_RPT; ++r) {
    const int row = (blockIdx.x * PF_DET_RPT + r) * 256 + threadIdx.x;
    if (row < a.Tf) det_row(a, ps, series, sid, row, t_max, a0.comp_col0, a0.comp_ncol);
  }
}

#include "pf_mc.h"

// ============================================================================
// K3 + K4 + K5 + K6 in one launch (pf_fit_forecast): each series' forecast
// rows and in-sample metrics run in its own fit workgroup as soon as its fit
// + polish ends, so they fill the time the batch's slowest fits leave the
// other CUs idle instead of waiting for the whole fit launch to drain.  The
// rows are computed by the very device functions k_predict_det /
// k_predict_mc / k_cv_insample run (same arithmetic, same RNG streams keyed by
// (series id, row, sample)): the outputs are bitwise those of the separate
// launches.  Exact intervals, one grid, the warm-up hand-off fit path.
// ============================================================================
struct FuseArgs {
  PredKArgs p;
  CvKArgs cv;
  int metrics;  // run K6 (in-sample: one group of every history row)
  // K5 work sharing: a series' random rows are PF_FF_BLOCKS row blocks; its
  // own workgroup claims them first, workgroups whose series are done claim
  // the rest.  ctl (zeroed per launch): [0] workgroups started, [1] blocks
  // not yet claimed (set by the host to n * PF_FF_BLOCKS), then ready[n],
  // claimed[n], finished[n]
  int *ctl;
};
#ifndef PF_FF_BLOCKS
#define PF_FF_BLOCKS 4
#endif
#define PF_FF_SPIN 4000   // a helper's bounded wait for work (x ~1 us of s_sleep)
// what pf_fit_forecast asks of the fit launcher: fuse when the fit takes the
// fused fit + polish path (done = 1); only = 1: launch nothing otherwise
struct FuseReq {
  const FuseArgs *args;
  int only;
  int done;
};
// epilogue LDS, from the dynamic LDS base (the fit's layout is dead by then)
struct FuseSmem {
  static constexpr size_t cp_off = (sizeof(PredSeries) + 15) & ~(size_t)15;
  static constexpr size_t meta_off = cp_off + PF_MC_CPCAP * sizeof(float2);
  static constexpr size_t buf_off = meta_off + 64 * PF_NQ * sizeof(uint32_t);
  static constexpr size_t wsum_off = buf_off + PF_MC_WAVES * 4 * 64 * sizeof(float);
  static constexpr size_t r0_off = wsum_off + PF_MC_WAVES * sizeof(double);
  // K6 runs after the Monte-Carlo rows: its APE cache reuses s_cp
  static constexpr size_t cache_off = cp_off;
  static constexpr size_t part_off = r0_off + 16;
  static constexpr size_t hist_off = part_off + PF_CV_INS_WAVES * 6 * sizeof(double);
  static constexpr size_t bad_off = hist_off + 256 * sizeof(int);
  static constexpr size_t bytes = bad_off + 32;   // K6's s_bad, then 4 broadcast slots
};
static_assert(PF_CV_INS_CACHE * sizeof(unsigned long long) <= PF_MC_CPCAP * sizeof(float2),
              "K6 cache must fit the changepoint slots it aliases");

// The K5 setup of series t (ps holds its PredSeries): first random row and
// every sample's changepoints packed in LDS.  Every thread calls it.
__device__ __forceinline__ void ff_setup(const FuseArgs &e, const PredSeries &ps, int t, char *smem_raw) {
  const PredKArgs &pa = e.p;
  const uint32_t sid = pa.series_id ? pa.series_id[t] : (uint32_t)t;
  int *s_r0 = reinterpret_cast<int *>(smem_raw + FuseSmem::r0_off);
  if (threadIdx.x == 0) *s_r0 = pa.Tf;
  __syncthreads();
  mc_setup(pa, ps, sid, reinterpret_cast<float2 *>(smem_raw + FuseSmem::cp_off),
           reinterpret_cast<uint32_t *>(smem_raw + FuseSmem::meta_off),
           reinterpret_cast<double *>(smem_raw + FuseSmem::wsum_off), s_r0);
}

// Row block b of series t (after ff_setup of t), then — for the workgroup
// that finishes the series' last block — its K6 row.  Returns true when K6
// ran (its APE cache overwrote the packed changepoints).  Every thread calls it.
#ifdef PF_FF_ROWS_NOINLINE
__device__ __noinline__
#else
__device__ __forceinline__
#endif
bool ff_rows(const FuseArgs &e, const PredSeries &ps, int t, int b, char *smem_raw, int *s_bcast) {
  const PredKArgs &pa = e.p;
  const int n = pa.n_series;
  int *finished = e.ctl + 2 + 2 * n;
  const uint32_t sid = pa.series_id ? pa.series_id[t] : (uint32_t)t;
  const float2 *s_cp = reinterpret_cast<const float2 *>(smem_raw + FuseSmem::cp_off);
  const uint32_t *s_meta = reinterpret_cast<const uint32_t *>(smem_raw + FuseSmem::meta_off);
  float *s_buf = reinterpret_cast<float *>(smem_raw + FuseSmem::buf_off);
  const double *s_wsum = reinterpret_cast<const double *>(smem_raw + FuseSmem::wsum_off);
  const int *s_r0 = reinterpret_cast<const int *>(smem_raw + FuseSmem::r0_off);
  if (pa.tr) mc_block_rows<true>(pa, ps, t, sid, b, PF_FF_BLOCKS, s_cp, s_meta, s_buf, s_wsum, s_r0);
  else mc_block_rows<false>(pa, ps, t, sid, b, PF_FF_BLOCKS, s_cp, s_meta, s_buf, s_wsum, s_r0);
  __syncthreads();   // this block's rows written by every wave
  if (threadIdx.x == 0) {
    __threadfence();  // the rows visible device-wide before the count says so
    s_bcast[0] = atomicAdd(&finished[t], 1);
  }
  __syncthreads();
  const int done_before = s_bcast[0];
  __syncthreads();
  if (!(e.metrics && done_before == PF_FF_BLOCKS - 1)) return false;
  // the series' last block: every row of t is written (its K4 rows before it
  // was published, the other blocks before their counts)
  __threadfence();
  cv_insample_block(e.cv, t, reinterpret_cast<unsigned long long *>(smem_raw + FuseSmem::cache_off),
                    reinterpret_cast<double (*)[6]>(smem_raw + FuseSmem::part_off),
                    reinterpret_cast<int *>(smem_raw + FuseSmem::hist_off),
                    reinterpret_cast<int *>(smem_raw + FuseSmem::bad_off));
  __syncthreads();
  return true;
}

template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__global__ __launch_bounds__(NW * 64, FitOcc<KMAX>::W) void k_fit_forecast(FitKArgs a, FuseArgs e) {
  static_assert(NW == PF_MC_WAVES && NW == PF_CV_INS_WAVES, "fused epilogue: one block shape");
  const int n = e.p.n_series;
  int *ready = e.ctl + 2, *claimed = e.ctl + 2 + n;
  if (threadIdx.x == 0) atomicAdd(&e.ctl[0], 1);   // started
  PF_BLK(0);
  pf_base_prio(1);
  fit_polish_passes<NW, KMAX, O0, O1, O2, MODE>(a);
  __syncthreads();   // theta of this series written (wave 0), the fit's LDS dead
  PF_BLK(1);
  pf_base_prio(0);
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  PredSeries &ps = *reinterpret_cast<PredSeries *>(smem_raw);
  int *s_bcast = reinterpret_cast<int *>(smem_raw + FuseSmem::bad_off + 8);
  const int series = blockIdx.x;
  const PredKArgs &pa = e.p;
  const uint32_t sid = pa.series_id ? pa.series_id[series] : (uint32_t)series;
  pred_setup(pa, series, ps);
  __syncthreads();
  // K4: every row's point forecast (+ components), the deterministic rows'
  // exact intervals
  const double t_max = pa.t[pa.Tf - 1];
  for (int row = threadIdx.x; row < pa.Tf; row += NW * 64)
    det_row(pa, ps, series, sid, row, t_max, e.p.comp_col0, e.p.comp_ncol);
  if (pa.N == 0) {
    if (e.metrics) {
      __syncthreads();
      cv_insample_block(e.cv, series, reinterpret_cast<unsigned long long *>(smem_raw + FuseSmem::cache_off),
                        reinterpret_cast<double (*)[6]>(smem_raw + FuseSmem::part_off),
                        reinterpret_cast<int *>(smem_raw + FuseSmem::hist_off),
                        reinterpret_cast<int *>(smem_raw + FuseSmem::bad_off));
    }
    PF_BLK(2);
    return;
  }
  // publish: theta and the K4 rows of this series are final
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    atomicExch(&ready[series], 1);
  }
  // K5: row blocks claimed one at a time — this series' first (helpers may
  // take some), then other published series' blocks while any are left.  A
  // workgroup waits for work only once every workgroup of the launch has
  // started (the series it waits on are resident, so they finish), and only
  // for a bounded time; the owner of a series always takes its unclaimed
  // blocks itself, so the results never depend on helping.  One call site
  // of the block body (its registers are allocated once).
  int cur = series;   // the series whose PredSeries is in ps
  int cur_setup = -1; // the series whose K5 setup is in LDS
  bool own = true;
  int spin = 0;
  while (true) {
    if (threadIdx.x < 64) {
      const int lane = pf_lane();
      int t = -1, b = PF_FF_BLOCKS, act = 2;
      if (own) {
        if (lane == 0) {
          b = atomicAdd(&claimed[series], 1);
          if (b < PF_FF_BLOCKS) atomicSub(&e.ctl[1], 1);
        }
        b = __shfl(b, 0, 64);
        t = series;
        act = b < PF_FF_BLOCKS ? 0 : 3;   // 3: own blocks done, look for others
      } else {
        // wave 0 scans for an unclaimed block of a published series,
        // starting after its own index
        for (int base = 0; base < n && t < 0; base += 64) {
          const int u = (series + 1 + base + lane) % n;
          const bool cand = (base + lane < n - 1) &&
                            __atomic_load_n(&ready[u], __ATOMIC_RELAXED) != 0 &&
                            __atomic_load_n(&claimed[u], __ATOMIC_RELAXED) < PF_FF_BLOCKS;
          const unsigned long long m = __ballot(cand);
          if (m) t = __shfl(u, __ffsll((long long)m) - 1, 64);
        }
        if (lane == 0) {
          if (t >= 0) {
            b = atomicAdd(&claimed[t], 1);
            if (b < PF_FF_BLOCKS) atomicSub(&e.ctl[1], 1);
          }
          const int left = __atomic_load_n(&e.ctl[1], __ATOMIC_RELAXED);
          const int started = __atomic_load_n(&e.ctl[0], __ATOMIC_RELAXED);
          act = (t >= 0 && b < PF_FF_BLOCKS) ? 0 : 1;   // 0: work; 1: wait; 2: exit
          if (act == 1 && (left <= 0 || started < n || spin >= PF_FF_SPIN)) act = 2;
        }
      }
      if (lane == 0) {
        s_bcast[1] = act;
        s_bcast[2] = t;
        s_bcast[3] = b;
      }
    }
    __syncthreads();
    const int act = s_bcast[1], tt = s_bcast[2], bb = s_bcast[3];
    __syncthreads();
    if (act == 2) break;
    if (act == 3) {
      own = false;
      continue;
    }
    if (act == 1) {
      ++spin;
      __builtin_amdgcn_s_sleep(127);
      continue;
    }
    spin = 0;
    if (tt != cur) {
      __threadfence();   // acquire: the series' theta and K4 rows
      pred_setup(pa, tt, ps);
      cur = tt;
      __syncthreads();
    }
    if (tt != cur_setup) {
      ff_setup(e, ps, tt, smem_raw);
      cur_setup = tt;
    }
    if (ff_rows(e, ps, tt, bb, smem_raw, s_bcast)) cur_setup = -1;
  }
  PF_BLK(2);
}

#if PF_MAIN
// ============================================================================
// C ABI
// ============================================================================
extern "C" {

int pf_ctx_create(int device, pf_ctx **out) {
  if (!out) return set_err(nullptr, "pf_ctx_create: out is NULL");
  pf_ctx *c = new pf_ctx();
  c->device = device;
  c->err[0] = 0;
  c->ws = nullptr;
  c->ws2 = nullptr;
  c->ws2_bytes = 0;
  c->ws_bytes = 0;
  c->timing = 0;
  c->n_timed = 0;
  c->n_events = 0;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device);
  if (e != hipSuccess) {
    snprintf(g_err_noctx, sizeof g_err_noctx, "hipSetDevice(%d): %s", device, hipGetErrorString(e));
    delete c;
    return -2;
  }
  if (c->n_cu < 1) c->n_cu = 256;
  *out = c;
  return 0;
}

int pf_set_timing(pf_ctx *ctx, int enable) {
  if (!ctx) return set_err(nullptr, "pf_set_timing: NULL ctx");
  ctx->timing = enable ? 1 : 0;
  ctx->n_timed = 0;
  return 0;
}

int pf_read_timings(pf_ctx *ctx, pf_kernel_time *out, int max_out) {
  if (!ctx) return set_err(nullptr, "pf_read_timings: NULL ctx");
  const int n = ctx->n_timed;
  for (int i = 0; i < n && i < max_out; ++i) {
    PF_HIP(ctx, hipEventSynchronize(ctx->timed[i].stop));
    float ms = 0.f;
    PF_HIP(ctx, hipEventElapsedTime(&ms, ctx->timed[i].start, ctx->timed[i].stop));
    snprintf(out[i].name, sizeof out[i].name, "%s", ctx->timed[i].name);
    out[i].ms = ms;
    out[i].grid = ctx->timed[i].grid;
  }
  ctx->n_timed = 0;
  return n < max_out ? n : max_out;
}

int pf_ctx_destroy(pf_ctx *ctx) {
  if (ctx)
    for (int i = 0; i < ctx->n_events; ++i) {
      (void)hipEventDestroy(ctx->timed[i].start);
      (void)hipEventDestroy(ctx->timed[i].stop);
    }
  if (ctx && ctx->ws) (void)hipFree(ctx->ws);
  if (ctx && ctx->ws2) (void)hipFree(ctx->ws2);
  delete ctx;
  return 0;
}

// grow the context scratch (synchronises the device when it has to grow;
// steady-state calls with the same shapes never allocate)
static int ctx_workspace(pf_ctx *ctx, size_t bytes, void **out) {
  if (bytes > ctx->ws_bytes) {
    if (ctx->ws) PF_HIP(ctx, hipFree(ctx->ws));
    ctx->ws = nullptr;
    ctx->ws_bytes = 0;
    PF_HIP(ctx, hipMalloc(&ctx->ws, bytes));
    ctx->ws_bytes = bytes;
  }
  *out = ctx->ws;
  return 0;
}

static int ctx_workspace2(pf_ctx *ctx, size_t bytes, void **out) {
  if (bytes > ctx->ws2_bytes) {
    if (ctx->ws2) PF_HIP(ctx, hipFree(ctx->ws2));
    ctx->ws2 = nullptr;
    ctx->ws2_bytes = 0;
    PF_HIP(ctx, hipMalloc(&ctx->ws2, bytes));
    ctx->ws2_bytes = bytes;
  }
  *out = ctx->ws2;
  return 0;
}

const char *pf_last_error(pf_ctx *ctx) { return ctx ? ctx->err : g_err_noctx; }

// build id: SHA-256 (32 hex digits) of csrc/ + include/ + the compile flags,
// passed by build.py; _lib.load() compares it with the sources on disk
#ifndef PF_BUILD_ID
#define PF_BUILD_ID "unversioned"
#endif
static const char pf_build_id_str[] = "PF_BUILD_ID:" PF_BUILD_ID;
const char *pf_build_id(void) { return pf_build_id_str + 12; }

void pf_default_fit_opts(pf_fit_opts *o) {
  o->init_alpha = 1e-3;
  o->tol_obj = 1e-12;
  o->tol_rel_obj = 1e4;
  o->tol_grad = 1e-8;
  o->tol_rel_grad = 1e7;
  o->tol_param = 1e-8;
  o->max_iter = 10000;
  o->history = 5;
  o->polish = 1;
  o->polish_max_iter = 100;  // Newton steps (damped logistic fits from far away need up to ~52)
  o->lbfgs_warmup = 40;       // with the damped first polish step (tools/sweep_warmup_damped.py)
  o->lbfgs_warmup_evals = 60;  // also end a warm-up pass at 60 evaluations
  o->tile_min_series = 2048;
  o->polish_max_lag = 4;
  o->polish_lag_ratio = 1e-2;
  o->polish_lam0 = 1e-2;    // damped first polish step (tools/diag_basin_floor.py)
  o->lbfgs_warmup_ls_slack = 4;
  if (const char *e = getenv("PF_POLISH_LAM0")) o->polish_lam0 = atof(e);   // diagnostic override
}

int pf_num_changepoints(int T, int n_changepoints, double changepoint_range) {
  const int hist_size = (int)floor((double)T * changepoint_range);
  int n = n_changepoints;
  if (n + 1 > hist_size) n = hist_size - 1;
  return n > 0 ? n : 0;
}

int pf_build_grid(pf_ctx *ctx, const int64_t *ds_ns, int T, int T_pad, int64_t start_ns,
                  int64_t t_scale_ns, const pf_season *seasons_host, int n_season,
                  const double *extra_cols, int n_extra, int n_changepoints,
                  double changepoint_range, double *t_out, double *XT_out, double *t_change_io,
                  int32_t *cp_idx_out, int32_t *seg_out, int32_t *cp_first_out, int S,
                  void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (T < 1 || T_pad < T || (T_pad % 128) != 0) return set_err(ctx, "pf_build_grid: bad T/T_pad");
  if (n_season < 0 || n_season > PF_MAX_SEASONS) return set_err(ctx, "pf_build_grid: n_season");
  if (t_scale_ns <= 0) return set_err(ctx, "pf_build_grid: t_scale must be > 0");
  if (!ds_ns || !t_out || !XT_out || !t_change_io || !seg_out) return set_err(ctx, "pf_build_grid: NULL buffer");
  if (S < 1) return set_err(ctx, "pf_build_grid: S must be >= 1");
  SeasonSpec ss;
  ss.n = n_season;
  for (int b = 0; b < n_season; ++b) {
    ss.period[b] = seasons_host[b].period;
    ss.order[b] = seasons_host[b].order;
    if (ss.order[b] < 0) return set_err(ctx, "pf_build_grid: negative fourier order");
  }
  const int nb = (T_pad + 255) / 256;
  int n_harm = 0;
  for (int b = 0; b < n_season; ++b) n_harm += ss.order[b];
  PF_TIMED_LAUNCH(ctx, "k_grid_features", nb * (n_harm + 1), st, k_grid_features,
                  dim3(nb, n_harm + 1), dim3(256), 0, st,
                  ds_ns, T, T_pad, start_ns, t_scale_ns, ss, extra_cols, n_extra, t_out, XT_out);
  PF_HIP(ctx, hipGetLastError());
  // changepoints placed inside k_grid_segments while they fit in LDS
  const bool fused_cp = n_changepoints >= 0 && S <= PF_GRID_CP_LDS;
  if (n_changepoints >= 0) {
    if (!cp_idx_out) return set_err(ctx, "pf_build_grid: cp_idx_out NULL");
    const int n_expect = pf_num_changepoints(T, n_changepoints, changepoint_range);
    if ((n_expect > 0 ? n_expect : 1) != S)
      return set_err(ctx, "pf_build_grid: S does not match pf_num_changepoints");
    if (!fused_cp) {
      PF_TIMED_LAUNCH(ctx, "k_grid_changepoints", 1, st, k_grid_changepoints, dim3(1), dim3(64), 0,
                      st, t_out, T, n_changepoints, changepoint_range, t_change_io, cp_idx_out);
      PF_HIP(ctx, hipGetLastError());
    }
  }
  const int ns = ((T_pad > S ? T_pad : S) + 255) / 256;
  PF_TIMED_LAUNCH(ctx, "k_grid_segments", ns, st, k_grid_segments, dim3(ns), dim3(256),
                  fused_cp ? (size_t)S * sizeof(double) : 0, st, t_out, T, T_pad, t_change_io, S,
                  fused_cp ? n_changepoints : -1, changepoint_range,
                  fused_cp ? cp_idx_out : nullptr, seg_out, cp_first_out);
  PF_HIP(ctx, hipGetLastError());
  return 0;
}

int pf_build_grids(pf_ctx *ctx, int n_grids, const int64_t *grid_params, const int64_t *ds_ns,
                   int T_max, int T_pad, const pf_season *seasons_host, int n_season,
                   int n_changepoints, double changepoint_range, double *t_out, double *XT_out,
                   double *t_change_io, int32_t *cp_idx_out, int32_t *seg_out,
                   int32_t *cp_first_out, int S, pf_grid *grids_out, void *stream) {
  hipStream_t st = (hipStream_t)stream;
  if (n_grids < 0) return set_err(ctx, "pf_build_grids: n_grids < 0");
  if (n_grids == 0) return 0;
  if (T_max < 1 || T_pad < T_max || (T_pad % 128) != 0) return set_err(ctx, "pf_build_grids: bad T_max/T_pad");
  if (n_season < 0 || n_season > PF_MAX_SEASONS) return set_err(ctx, "pf_build_grids: n_season");
  if (!grid_params || !t_out || !XT_out || !t_change_io || !seg_out || !cp_first_out || !grids_out)
    return set_err(ctx, "pf_build_grids: NULL buffer");
  if (n_changepoints >= 0 && !cp_idx_out) return set_err(ctx, "pf_build_grids: cp_idx_out NULL");
  if (S < 1) return set_err(ctx, "pf_build_grids: S must be >= 1");
  SeasonSpec ss;
  ss.n = n_season;
  int K = 0;
  for (int b = 0; b < n_season; ++b) {
    ss.period[b] = seasons_host[b].period;
    ss.order[b] = seasons_host[b].order;
    K += 2 * ss.order[b];
  }
  if (K < 1) return set_err(ctx, "pf_build_grids: no seasonality columns");
  const int nb = (T_pad + 255) / 256;
  PF_TIMED_LAUNCH(ctx, "k_grids_features", nb * n_grids, st, k_grids_features, dim3(nb, n_grids),
                  dim3(256), 0, st, grid_params, ds_ns, T_pad, K, ss, t_out, XT_out);
  PF_HIP(ctx, hipGetLastError());
  if (n_changepoints >= 0) {
    const int nc = (n_grids + 63) / 64;
    PF_TIMED_LAUNCH(ctx, "k_grids_changepoints", nc, st, k_grids_changepoints, dim3(nc), dim3(64),
                    0, st, grid_params, n_grids, T_pad, S, n_changepoints, changepoint_range,
                    t_out, t_change_io, cp_idx_out);
    PF_HIP(ctx, hipGetLastError());
  }
  const int ns = ((T_pad > S ? T_pad : S) + 255) / 256;
  PF_TIMED_LAUNCH(ctx, "k_grids_segments", ns * n_grids, st, k_grids_segments, dim3(ns, n_grids),
                  dim3(256), 0, st, grid_params, T_pad, K, S, t_out, XT_out, t_change_io, seg_out,
                  cp_first_out, grids_out);
  PF_HIP(ctx, hipGetLastError());
  return 0;
}

int pf_prepare_ragged(pf_ctx *ctx, int n_series, const pf_grid *grid, int n_grids,
                      const pf_grid *grids_dev, const int32_t *grid_of, int growth,
                      const double *y, const double *cap, double *y_scale, double *y_scaled,
                      double *cap_scaled, double *theta0, int32_t *status, void *stream) {
  if (n_series < 0 || !grid || !y || !y_scale || !y_scaled || !theta0 || !status)
    return set_err(ctx, "pf_prepare: bad arguments");
  if (n_grids < 0 || (n_grids > 0 && (!grids_dev || !grid_of)))
    return set_err(ctx, "pf_prepare_ragged: n_grids > 0 needs grids and grid_of");
  if (n_grids == 0 && !grid->t) return set_err(ctx, "pf_prepare: NULL grid.t");
  if (grid->T < 2 || grid->T > grid->T_pad) return set_err(ctx, "pf_prepare: bad T / T_pad");
  if (growth == PF_GROWTH_LOGISTIC && (!cap || !cap_scaled))
    return set_err(ctx, "pf_prepare: logistic growth needs cap and cap_scaled");
  if (n_series == 0) return 0;
  const int P = 3 + grid->S + grid->K;
  PF_TIMED_LAUNCH(ctx, "k_prepare", n_series, (hipStream_t)stream, k_prepare, dim3(n_series),
                  dim3(256), 0, (hipStream_t)stream, grid->T, grid->T_pad, grid->t, growth, y,
                  cap, y_scale, y_scaled, cap_scaled, theta0, status, P, grid->S,
                  n_grids > 0 ? grids_dev : nullptr, n_grids > 0 ? grid_of : nullptr);
  PF_HIP(ctx, hipGetLastError());
  return 0;
}

int pf_prepare(pf_ctx *ctx, int n_series, const pf_grid *grid, int growth, const double *y,
               const double *cap, double *y_scale, double *y_scaled, double *cap_scaled,
               double *theta0, int32_t *status, void *stream) {
  return pf_prepare_ragged(ctx, n_series, grid, 0, nullptr, nullptr, growth, y, cap, y_scale,
                           y_scaled, cap_scaled, theta0, status, stream);
}

}  // extern "C"

// ---------------------------------------------------------------- lane-blocked grid
// Position q = r*NL + L of the copy holds natural row i = L*R + r (rows past
// T: t = 0, X = 0, seg = S, no changepoint starts).  Built per fit call into
// the context workspace (K+1 doubles + 1 int per position; ~0.4 MB at 1826
// days), read by every series of the batch.  One column per blockIdx.y, so
// the copy spreads over (K + 1) x ceil(TQ / 256) workgroups rather than
// ceil(TQ / 256) threads each walking the K strided columns (11 -> ~4 us at
// 1826 days; the copy sits on the fit's critical path).
__global__ __launch_bounds__(256) void k_permute_grid(const double *__restrict__ t,
                                                      const int32_t *__restrict__ seg,
                                                      const double *__restrict__ XT, int T, int Tp,
                                                      int K, int S, int R, int NL,
                                                      double *__restrict__ tP,
                                                      int32_t *__restrict__ sgP,
                                                      double *__restrict__ XTP) {
  const int TQ = NL * R;
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= TQ) return;
  const int r = q / NL, L = q - r * NL;
  const int i = L * R + r;
  const bool v = i < T;
  const int f = (int)blockIdx.y - 1;  // y = 0: t and seg; y = f + 1: column f
  if (f < 0) {
    tP[q] = v ? t[i] : 0.0;
    const int sg = v ? seg[i] : S;
    const int sp = v ? (i > 0 ? seg[i - 1] : 0) : S;
    sgP[q] = sg | ((sg - sp) << 16);
  } else {
    XTP[(size_t)f * TQ + q] = v ? XT[(size_t)f * Tp + i] : 0.0;
  }
}

// Ragged batch: the lane-blocked copy of every grid (blockIdx.y = grid), each
// with its own R = ceil(T / NL), at base + g * stride bytes.
__global__ __launch_bounds__(256) void k_permute_grid_ragged(const pf_grid *__restrict__ grids,
                                                             int Tp, int K, int S, int NL,
                                                             char *__restrict__ base, size_t stride) {
  const int g = blockIdx.y;  // blockIdx.z: which column, as in k_permute_grid
  const int T = __builtin_amdgcn_readfirstlane(grids[g].T);
  const int R = (T + NL - 1) / NL, TQ = NL * R;
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= TQ) return;
  const double *__restrict__ t = grids[g].t;
  const int32_t *__restrict__ seg = grids[g].seg;
  const double *__restrict__ XT = grids[g].XT;
  double *tP = (double *)(base + (size_t)g * stride);
  double *XTP = tP + TQ;
  int32_t *sgP = (int32_t *)(tP + (size_t)TQ * (1 + K));
  const int r = q / NL, L = q - r * NL;
  const int i = L * R + r;
  const bool v = i < T;
  const int f = (int)blockIdx.z - 1;  // z = 0: t and seg; z = f + 1: column f
  if (f < 0) {
    tP[q] = v ? t[i] : 0.0;
    const int sg = v ? seg[i] : S;
    const int sp = v ? (i > 0 ? seg[i - 1] : 0) : S;
    sgP[q] = sg | ((sg - sp) << 16);
  } else {
    XTP[(size_t)f * TQ + q] = v ? XT[(size_t)f * Tp + i] : 0.0;
  }
}

// Row-major feature copy for K3T: XR[r][f] = X[r][f] (f < K), 0 for K <= f < W
// (W = 32 or 48, the tile's padded feature count).
__global__ __launch_bounds__(256) void k_grid_rowmajor(const double *__restrict__ XT, int Tp, int K,
                                                       int W, double *__restrict__ XR) {
  const size_t q = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= (size_t)Tp * W) return;
  const int r = (int)(q / W), f = (int)(q - (size_t)r * W);
  XR[q] = f < K ? XT[(size_t)f * Tp + r] : 0.0;
}

#endif  // PF_MAIN (C ABI part 1, grid copies)

// ---------------------------------------------------------------- dispatch
#define PF_FIT_NW 4
#if PF_MAIN
namespace {

FitKArgs make_fit_args(const pf_problem *pb) {
  FitKArgs a;
  memset(&a, 0, sizeof a);
  a.T = pb->grid.T;
  a.Tp = pb->grid.T_pad;
  a.K = pb->grid.K;
  a.S = pb->grid.S;
  a.growth = pb->growth;
  a.P = 3 + a.S + a.K;
  a.NB = a.Tp / 64;
  a.R = (a.T + PF_FIT_NW * 64 - 1) / (PF_FIT_NW * 64);
  a.TQ = PF_FIT_NW * 64 * a.R;
  a.t = pb->grid.t;
  a.XT = pb->grid.XT;
  a.t_change = pb->grid.t_change;
  a.seg = pb->grid.seg;
  a.sigmas = pb->sigmas;
  a.s_a = pb->s_a;
  a.s_m = pb->s_m;
  a.tau = pb->tau;
  a.tau_series = pb->tau_series;
  a.sigmas_series = pb->sigmas_series;
  a.y_scaled = pb->y_scaled;
  a.cap_scaled = pb->cap_scaled;
  if (pb->n_grids > 0) {
    a.grids = pb->grids;
    a.grid_of = pb->grid_of;
  }
  return a;
}

}  // namespace
#endif  // PF_MAIN

enum { PF_LAUNCH_OBJGRAD = 0, PF_LAUNCH_FIT = 1, PF_LAUNCH_HESSIAN = 2 };
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
int launch_fitlike_impl(pf_ctx *ctx, int what, const FitKArgs &a, int n, hipStream_t st, double *H_out,
                        size_t smem, size_t smem_p, FuseReq *fz);
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
int launch_fitlike(pf_ctx *ctx, int what, const FitKArgs &a, int n, hipStream_t st, double *H_out,
                   FuseReq *fz) {
  // the polish handles K <= 48 (three 16-column beta blocks) and 2 + S <= 32
  constexpr bool HAS_POLISH = KMAX <= 48;
  const size_t smem = FitSmem<NW, KMAX, MODE>::bytes(a.TQ, a.P, a.S, false);
  size_t smem_p = FitSmem<NW, KMAX, MODE>::bytes(a.TQ, a.P, a.S, HAS_POLISH);
  FitKArgs a2 = a;
  a2.hstash = 0;
  if (HAS_POLISH && a.o.polish_lam0 > 0.0) {
    // the stash only where it keeps the workgroups per CU the kernel is built
    // for (two at <= 80 KB each for the 2-waves/SIMD layouts)
    const size_t with = FitSmem<NW, KMAX, MODE>::bytes(a.TQ, a.P, a.S, true, true);
    const size_t cap = (FitOcc<KMAX>::W >= 2 && smem_p <= 80 * 1024) ? 80 * 1024 : 160 * 1024;
    if (with <= cap) {
      smem_p = with;
      a2.hstash = 1;
    }
  }
  return launch_fitlike_impl<NW, KMAX, O0, O1, O2, MODE>(ctx, what, a2, n, st, H_out, smem, smem_p, fz);
}
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
int launch_fitlike_impl(pf_ctx *ctx, int what, const FitKArgs &a, int n, hipStream_t st, double *H_out,
                        size_t smem, size_t smem_p, FuseReq *fz) {
  constexpr bool HAS_POLISH = KMAX <= 48;
  if (smem > 160 * 1024) return set_err(ctx, "fit: series too long for the LDS budget");
  if (what == PF_LAUNCH_HESSIAN) {
    if constexpr (HAS_POLISH) {
      if (2 + a.S > 32 || smem_p > 160 * 1024) return set_err(ctx, "pf_hessian: needs 2 + S <= 32 and the polish LDS budget");
      auto kh = k_hessian<NW, KMAX, O0, O1, O2, MODE>;
      PF_HIP(ctx, hipFuncSetAttribute((const void *)kh, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem_p));
      PF_TIMED_LAUNCH(ctx, "k_hessian", n, st, kh, dim3(n), dim3(NW * 64), smem_p, st, a, H_out);
      PF_HIP(ctx, hipGetLastError());
      return 0;
    } else {
      return set_err(ctx, "pf_hessian: layout has no polish (K > 48)");
    }
  }
  if (what == PF_LAUNCH_FIT) {
    void (*kf[2])(FitKArgs) = {k_fit<NW, KMAX, O0, O1, O2, MODE>,
                               k_fit_resume<NW, KMAX, O0, O1, O2, MODE>};
    for (int v = 0; v < 2; ++v)
      PF_HIP(ctx, hipFuncSetAttribute((const void *)kf[v],
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
    bool polish = a.o.polish && a.K <= 48 && 2 + a.S <= 32 && smem_p <= 160 * 1024;
    void (*kpl[2])(FitKArgs) = {nullptr, nullptr};
    if constexpr (HAS_POLISH) {
      kpl[0] = k_polish<NW, KMAX, O0, O1, O2, MODE>;
      kpl[1] = k_polish_resume<NW, KMAX, O0, O1, O2, MODE>;
      if (polish)
        for (int v = 0; v < 2; ++v)
          PF_HIP(ctx, hipFuncSetAttribute((const void *)kpl[v],
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem_p));
    } else {
      polish = false;
    }
    const int W = a.o.lbfgs_warmup;
    // passes: (cap, warm?) — warm-up, one more warm-up for uncertified
    // series, then Stan's full rules; each followed by the polish
    int caps[3], warm[3], npass = 1;
    if (polish && W > 0 && W < a.o.max_iter) {
      caps[0] = W; warm[0] = 1;
      caps[1] = W; warm[1] = 1;
      caps[2] = a.o.max_iter; warm[2] = 0;
      npass = 3;
    } else {
      caps[0] = a.o.max_iter; warm[0] = 0;
    }
    // tiled first pass (K3T, 16 series per workgroup, MFMA row pass) for
    // large batches of the layouts it covers (K <= 48, P <= 72, S + 1 <= 32,
    // shared prior scales, one grid); the per-series kernels finish
    constexpr int TKP = KMAX <= 32 ? 32 : 48;
    constexpr bool TILE_OK = KMAX <= 48;
    bool tile = false;
    size_t smem_t = 0;
    if constexpr (TILE_OK) {
      smem_t = TileSmem<MODE, TKP>::bytes();
      tile = a.o.tile_min_series >= 0 && n >= a.o.tile_min_series && a.P <= TileTr<MODE, TKP>::TV &&
             a.K <= TKP && a.S + 1 <= 32 && !a.tau_series && !a.sigmas_series && a.XR &&
             a.XR_width == TKP && !a.grid_of && smem_t <= 160 * 1024;
    }
    if (npass == 3 && !tile && !getenv_flag("PF_SPLIT_POLISH")) {
      if constexpr (HAS_POLISH) {
        if (fz) {
          // fused forecast epilogue: the fit's LDS, grown to the epilogue's
          // when needed only while that keeps the workgroups per CU
          const size_t sf0 = smem_p > smem ? smem_p : smem;
          const size_t sf = sf0 > FuseSmem::bytes ? sf0 : FuseSmem::bytes;
          const size_t cap = (FitOcc<KMAX>::W >= 2 && sf0 <= 80 * 1024) ? 80 * 1024 : 160 * 1024;
          if (sf <= cap) {
            auto kff = k_fit_forecast<NW, KMAX, O0, O1, O2, MODE>;
            PF_HIP(ctx, hipFuncSetAttribute((const void *)kff, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (int)sf));
            PF_TIMED_LAUNCH(ctx, "k_fit_forecast", n, st, kff, dim3(n), dim3(NW * 64), sf, st, a, *fz->args);
            PF_HIP(ctx, hipGetLastError());
            fz->done = 1;
            return 0;
          }
          if (fz->only) return 0;
        }
        auto kfp = k_fit_polish<NW, KMAX, O0, O1, O2, MODE>;
        PF_HIP(ctx, hipFuncSetAttribute((const void *)kfp, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)(smem_p > smem ? smem_p : smem)));
        PF_TIMED_LAUNCH(ctx, "k_fit_polish", n, st, kfp, dim3(n), dim3(NW * 64),
                        smem_p > smem ? smem_p : smem, st, a);
        PF_HIP(ctx, hipGetLastError());
        return 0;
      }
    }
    if (fz && fz->only) return 0;   // not the fused path: the caller launches the parts
    for (int ps = 0; ps < npass; ++ps) {
      FitKArgs b = a;
      b.o.max_iter = caps[ps];
      b.warm_cap = warm[ps];
      if (!warm[ps]) b.o.lbfgs_warmup_evals = 0;
      b.pass = ps;
      const int v = ps == 0 ? 0 : 1;
      if (ps == 0 && tile) {
        if constexpr (TILE_OK) {
          auto kt = k_fit_tile<MODE, TKP>;
          PF_HIP(ctx, hipFuncSetAttribute((const void *)kt, hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)smem_t));
          // persistent tiles: one workgroup per CU (the LDS budget), series
          // handed out by the queue counter after the first 16 per tile
          const int nt = (n + PF_TS - 1) / PF_TS;
          const int grid = nt < ctx->n_cu ? nt : ctx->n_cu;
          PF_HIP(ctx, hipMemsetD32Async((hipDeviceptr_t)b.queue, grid * PF_TS, 1, st));
          PF_TIMED_LAUNCH(ctx, "k_fit_tile", grid, st, kt, dim3(grid), dim3(PF_TNW * 64), smem_t, st, b, n);
        }
      } else {
        PF_TIMED_LAUNCH(ctx, v ? "k_fit_resume" : "k_fit", n, st, kf[v], dim3(n), dim3(NW * 64),
                        smem, st, b);
      }
      PF_HIP(ctx, hipGetLastError());
      if (polish) {
        PF_TIMED_LAUNCH(ctx, v ? "k_polish_resume" : "k_polish", n, st, kpl[v], dim3(n),
                        dim3(NW * 64), smem_p, st, b);
        PF_HIP(ctx, hipGetLastError());
      }
    }
  } else {
    auto kern = k_objgrad<NW, KMAX, O0, O1, O2, MODE>;
    PF_HIP(ctx, hipFuncSetAttribute((const void *)kern,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
    PF_TIMED_LAUNCH(ctx, "k_objgrad", n, st, kern, dim3(n), dim3(NW * 64), smem, st, a);
  }
  PF_HIP(ctx, hipGetLastError());
  return 0;
}

// The instantiations, grouped by translation unit (PF_TU = group): LG =
// logistic, WD = wide (two parameter words).
#define PF_LG PF_MODE_LOGI
#define PF_WD PF_MODE_WIDE
#define PF_FIT_INSTANCES(X)                                   \
  X(1, 26, 10, 3, 0, MODE_MULT)                               \
  X(2, 26, 10, 3, 0, MODE_ADD)                                \
  X(2, 26, 10, 3, 0, MODE_MIXED)                              \
  X(3, 36, 10, 3, 0, MODE_MULT | PF_LG)                       \
  X(3, 36, 10, 3, 0, MODE_MULT)                               \
  X(4, 44, 10, 3, 4, MODE_MULT | PF_LG | PF_WD)               \
  X(4, 44, 10, 3, 4, MODE_MULT | PF_WD)                       \
  X(5, 26, 10, 3, 0, MODE_MULT | PF_LG)                       \
  X(5, 34, 10, 3, 4, MODE_MULT | PF_LG)                       \
  X(6, 32, 0, 0, 0, MODE_MIXED | PF_LG)                       \
  X(6, 32, 0, 0, 0, MODE_MIXED)                               \
  X(7, 34, 10, 3, 4, MODE_MULT)                               \
  X(7, 61, 0, 0, 0, MODE_MIXED)
#define PF_FIT_NTU 8
#ifdef PF_TU
#if PF_TU == 0
// the main unit uses the instances the fit units define
#define PF_EXTERN_INST(G, K, O0, O1, O2, M)                                               \
  extern template int launch_fitlike<PF_FIT_NW, K, O0, O1, O2, M>(pf_ctx *, int, const FitKArgs &, \
                                                                  int, hipStream_t, double *,      \
                                                                  FuseReq *);
PF_FIT_INSTANCES(PF_EXTERN_INST)
#endif
#endif

#if PF_MAIN
namespace {
// Template instances:
//   (26, 10,3,0, MULT) — the reference's configuration (yearly 10 + weekly 3,
//                        multiplicative): features regenerated in-register
//   (26, 10,3,0, ADD/MIXED) — same grid, other seasonality modes
//   (34, 10,3,4, MULT) — sub-daily data (yearly + weekly + daily 4; config 5)
//   dense fallbacks KMAX 32 / 61 (any K <= KMAX), features read from X^T.
int dispatch_fitlike(pf_ctx *ctx, int fit, const FitKArgs &a, int n, const int32_t *orders, int mode,
                     hipStream_t st, double *H_out = nullptr, FuseReq *fz = nullptr) {
  const bool o1030 = orders[0] == 10 && orders[1] == 3 && orders[2] == 0;
  const bool o1034 = orders[0] == 10 && orders[1] == 3 && orders[2] == 4;
  constexpr int LG = PF_MODE_LOGI, WD = PF_MODE_WIDE;
  // extra (holiday / regressor) columns after the Fourier blocks: up to 10
  // with yearly + weekly (P <= 64), up to 10 with yearly + weekly + daily
  // (P <= 72: two parameter words per lane) — SURVEY.md §8d configs[4]
  if (o1030 && a.K > 26 && a.K <= 36 && mode == MODE_MULT) {
    if (a.growth == PF_GROWTH_LOGISTIC)
      return launch_fitlike<PF_FIT_NW, 36, 10, 3, 0, MODE_MULT | LG>(ctx, fit, a, n, st, H_out, fz);
    return launch_fitlike<PF_FIT_NW, 36, 10, 3, 0, MODE_MULT>(ctx, fit, a, n, st, H_out, fz);
  }
  if (o1034 && a.K > 34 && a.K <= 44 && mode == MODE_MULT) {
    if (a.growth == PF_GROWTH_LOGISTIC)
      return launch_fitlike<PF_FIT_NW, 44, 10, 3, 4, MODE_MULT | LG | WD>(ctx, fit, a, n, st, H_out, fz);
    return launch_fitlike<PF_FIT_NW, 44, 10, 3, 4, MODE_MULT | WD>(ctx, fit, a, n, st, H_out, fz);
  }
  if (a.P > 64) return set_err(ctx, "fit: P > 64 is supported for yearly+weekly+daily (10,3,4) plus <= 10 extra columns, multiplicative");
  if (a.growth == PF_GROWTH_LOGISTIC) {
    if (o1030 && a.K == 26 && mode == MODE_MULT)
      return launch_fitlike<PF_FIT_NW, 26, 10, 3, 0, MODE_MULT | LG>(ctx, fit, a, n, st, H_out, fz);
    if (o1034 && a.K == 34 && mode == MODE_MULT)
      return launch_fitlike<PF_FIT_NW, 34, 10, 3, 4, MODE_MULT | LG>(ctx, fit, a, n, st, H_out, fz);
    if (a.K <= 32) return launch_fitlike<PF_FIT_NW, 32, 0, 0, 0, MODE_MIXED | LG>(ctx, fit, a, n, st, H_out, fz);
    return set_err(ctx, "fit: logistic growth supports K <= 32, or yearly+weekly+daily (K = 34) multiplicative");
  }
  if (o1030 && a.K == 26) {
    if (mode == MODE_MULT) return launch_fitlike<PF_FIT_NW, 26, 10, 3, 0, MODE_MULT>(ctx, fit, a, n, st, H_out, fz);
    if (mode == MODE_ADD) return launch_fitlike<PF_FIT_NW, 26, 10, 3, 0, MODE_ADD>(ctx, fit, a, n, st, H_out, fz);
    return launch_fitlike<PF_FIT_NW, 26, 10, 3, 0, MODE_MIXED>(ctx, fit, a, n, st, H_out, fz);
  }
  if (o1034 && a.K == 34 && mode == MODE_MULT)
    return launch_fitlike<PF_FIT_NW, 34, 10, 3, 4, MODE_MULT>(ctx, fit, a, n, st, H_out, fz);
  if (a.K <= 32) return launch_fitlike<PF_FIT_NW, 32, 0, 0, 0, MODE_MIXED>(ctx, fit, a, n, st, H_out, fz);
  if (a.K <= 61) return launch_fitlike<PF_FIT_NW, 61, 0, 0, 0, MODE_MIXED>(ctx, fit, a, n, st, H_out, fz);
  return set_err(ctx, "fit: K > 61 not supported");
}

}  // namespace

extern "C" {

// Context scratch for one fit-like call: [lane-blocked grid | polish rows],
// then the permutation launch (stream-ordered with the fit that reads it).
static int prepare_fit_scratch(pf_ctx *ctx, FitKArgs &a, hipStream_t st, bool rowmajor = false,
                               int n_grids = 0) {
  const size_t TQ = (size_t)a.TQ;
  size_t gbytes = TQ * sizeof(double) * (1 + (size_t)a.K) + TQ * sizeof(int32_t);
  gbytes = (gbytes + 255) & ~(size_t)255;
  if (a.grid_of) {
    // ragged: one lane-blocked copy per grid (envelope-sized slots)
    void *w = nullptr;
    const int rc = ctx_workspace(ctx, gbytes * (size_t)n_grids, &w);
    if (rc) return rc;
    a.rg_base = (const char *)w;
    a.rg_stride = gbytes;
    a.tP = a.XTP = nullptr;
    a.sgP = nullptr;
    a.XR = nullptr;
    const int nb = (int)((TQ + 255) / 256);
    PF_TIMED_LAUNCH(ctx, "k_permute_grid_ragged", nb * n_grids * (a.K + 1), st,
                    k_permute_grid_ragged, dim3(nb, n_grids, a.K + 1), dim3(256), 0, st, a.grids, a.Tp, a.K, a.S, PF_FIT_NW * 64,
                    (char *)w, gbytes);
    PF_HIP(ctx, hipGetLastError());
    return 0;
  }
  const int W = a.K <= 32 ? 32 : 48;
  const size_t rbytes = rowmajor ? (size_t)a.Tp * W * sizeof(double) + 256 : 0;
  void *w = nullptr;
  const int rc = ctx_workspace(ctx, gbytes + rbytes, &w);
  if (rc) return rc;
  double *base = (double *)w;
  a.tP = base;
  a.XTP = base + TQ;
  a.sgP = (int32_t *)(base + TQ * (1 + (size_t)a.K));
  a.XR = nullptr;
  a.XR_width = 0;
  const int nb = (int)((TQ + 255) / 256);
  PF_TIMED_LAUNCH(ctx, "k_permute_grid", nb * (a.K + 1), st, k_permute_grid, dim3(nb, a.K + 1),
                  dim3(256), 0, st,
                  a.t, a.seg, a.XT, a.T, a.Tp, a.K, a.S, a.R, PF_FIT_NW * 64,
                  const_cast<double *>(a.tP), const_cast<int32_t *>(a.sgP),
                  const_cast<double *>(a.XTP));
  PF_HIP(ctx, hipGetLastError());
  if (rowmajor) {
    double *xr = (double *)((char *)w + gbytes);
    const int nr = (int)(((size_t)a.Tp * W + 255) / 256);
    PF_TIMED_LAUNCH(ctx, "k_grid_rowmajor", nr, st, k_grid_rowmajor, dim3(nr), dim3(256), 0, st,
                    a.XT, a.Tp, a.K, W, xr);
    PF_HIP(ctx, hipGetLastError());
    a.XR = xr;
    a.XR_width = W;
    a.queue = (int *)((char *)xr + (size_t)a.Tp * W * sizeof(double));
  }
  return 0;
}

static int mode_of(const pf_problem *pb) {
  return (pb->season_mode == 0) ? MODE_MULT : (pb->season_mode == 1) ? MODE_ADD : MODE_MIXED;
}

static int check_problem(pf_ctx *ctx, const pf_problem *pb) {
  if (!pb) return set_err(ctx, "NULL problem");
  if (pb->growth == PF_GROWTH_LOGISTIC && !pb->cap_scaled)
    return set_err(ctx, "logistic growth needs cap_scaled");
  const int P = 3 + pb->grid.S + pb->grid.K;
  if (P > 128) return set_err(ctx, "P = 3 + S + K must be <= 128");
  if (pb->grid.S < 1 || pb->grid.S > 62) return set_err(ctx, "S out of range");
  if (pb->grid.T < 2 || pb->grid.T_pad % 128 || pb->grid.T > pb->grid.T_pad)
    return set_err(ctx, "bad T / T_pad");
  if (pb->n_grids < 0 || (pb->n_grids > 0 && (!pb->grids || !pb->grid_of)))
    return set_err(ctx, "n_grids > 0 needs grids and grid_of");
  if (pb->n_grids == 0 && (!pb->grid.t || !pb->grid.XT || !pb->grid.t_change || !pb->grid.seg))
    return set_err(ctx, "NULL grid buffer in problem");
  if (!pb->sigmas || !pb->s_a || !pb->s_m || !pb->y_scaled)
    return set_err(ctx, "NULL buffer in problem");
  return 0;
}

int pf_objective_grad(pf_ctx *ctx, const pf_problem *pb, const double *theta, double *f,
                      double *g, void *stream) {
  int rc = check_problem(ctx, pb);
  if (rc) return rc;
  if (pb->n_series == 0) return 0;
  FitKArgs a = make_fit_args(pb);
  a.theta = const_cast<double *>(theta);
  a.f_out = f;
  a.g_out = g;
  rc = prepare_fit_scratch(ctx, a, (hipStream_t)stream, false, pb->n_grids);
  if (rc) return rc;
  return dispatch_fitlike(ctx, PF_LAUNCH_OBJGRAD, a, pb->n_series, pb->fourier_orders, mode_of(pb),
                          (hipStream_t)stream);
}

int pf_fit(pf_ctx *ctx, const pf_problem *pb, const pf_fit_opts *opts, double *theta_inout,
           double *f_out, double *f_stan, int32_t *status, int32_t *n_iter, int32_t *n_eval,
           void *stream) {
  int rc = check_problem(ctx, pb);
  if (rc) return rc;
  if (!opts || !theta_inout || !f_out || !f_stan || !status || !n_iter || !n_eval)
    return set_err(ctx, "pf_fit: NULL output");
  if (pb->n_series == 0) return 0;
  FitKArgs a = make_fit_args(pb);
  a.theta = theta_inout;
  a.f_out = f_out;
  a.f_stan = f_stan;
  a.status = status;
  a.n_iter = n_iter;
  a.n_eval = n_eval;
  a.o = *opts;
  // the tiled first pass reads a row-major feature copy
  const bool maybe_tile = opts->tile_min_series >= 0 && pb->n_series >= opts->tile_min_series &&
                          pb->grid.K <= 48 && pb->n_grids == 0 && !pb->tau_series &&
                          !pb->sigmas_series;
  rc = prepare_fit_scratch(ctx, a, (hipStream_t)stream, maybe_tile, pb->n_grids);
  if (rc) return rc;
  return dispatch_fitlike(ctx, PF_LAUNCH_FIT, a, pb->n_series, pb->fourier_orders, mode_of(pb),
                          (hipStream_t)stream);
}

int pf_hessian(pf_ctx *ctx, const pf_problem *pb, const double *theta, double *H, void *stream) {
  int rc = check_problem(ctx, pb);
  if (rc) return rc;
  if (!theta || !H) return set_err(ctx, "pf_hessian: NULL buffer");
  if (pb->n_series == 0) return 0;
  FitKArgs a = make_fit_args(pb);
  a.theta = const_cast<double *>(theta);
  rc = prepare_fit_scratch(ctx, a, (hipStream_t)stream, false, pb->n_grids);
  if (rc) return rc;
  return dispatch_fitlike(ctx, PF_LAUNCH_HESSIAN, a, pb->n_series, pb->fourier_orders, mode_of(pb),
                          (hipStream_t)stream, H);
}

// pf_predict's checks and kernel arguments (shared with pf_fit_forecast)
static int make_pred_args(pf_ctx *ctx, const pf_predict_args *p, PredKArgs &a) {
  if (!p) return set_err(ctx, "pf_predict: NULL args");
  if (p->n_samples < 0 || p->n_samples > 64 * PF_NQ) return set_err(ctx, "pf_predict: n_samples must be in [0, 1024]");
  const int P = 3 + p->fg.S + p->fg.K;
  if (P > 128 || p->fg.K > 64) return set_err(ctx, "pf_predict: P must be <= 128 and K <= 64");
  if (p->n_grids < 0 || (p->n_grids > 0 && (!p->grids || !p->grid_of)))
    return set_err(ctx, "pf_predict: n_grids > 0 needs grids and grid_of");
  if (p->n_grids == 0 && (!p->fg.t || !p->fg.XT || !p->fg.t_change || !p->fg.seg))
    return set_err(ctx, "pf_predict: NULL grid buffer");
  if (p->fg.T < 1 || p->fg.T > p->fg.T_pad) return set_err(ctx, "pf_predict: bad T / T_pad");
  if (!p->theta || !p->y_scale || !p->yhat || !p->yhat_lower || !p->yhat_upper)
    return set_err(ctx, "pf_predict: NULL buffer");
  if ((p->trend != nullptr) != (p->trend_lower != nullptr) ||
      (p->trend != nullptr) != (p->trend_upper != nullptr))
    return set_err(ctx, "pf_predict: trend/trend_lower/trend_upper must be all set or all NULL");
  memset(&a, 0, sizeof a);
  a.n_series = p->n_series;
  a.growth = p->growth;
  a.N = p->n_samples;
  a.Tf = p->fg.T;
  a.Tp = p->fg.T_pad;
  a.K = p->fg.K;
  a.S = p->fg.S;
  a.P = P;
  a.t = p->fg.t;
  a.XT = p->fg.XT;
  a.t_change = p->fg.t_change;
  a.seg = p->fg.seg;
  a.s_a = p->s_a;
  a.s_m = p->s_m;
  a.theta = p->theta;
  a.y_scale = p->y_scale;
  a.seed0 = (uint32_t)(p->seed & 0xFFFFFFFFu);
  a.seed1 = (uint32_t)(p->seed >> 32);
  a.yhat = p->yhat;
  a.ylo = p->yhat_lower;
  a.yhi = p->yhat_upper;
  a.tr = p->trend;
  a.trlo = p->trend_lower;
  a.trhi = p->trend_upper;
  a.mult = p->mult_terms;
  a.add = p->add_terms;
  a.comp = p->comp;
  a.series_id = p->series_id;
  if (p->n_grids > 0) {
    a.grids = p->grids;
    a.grid_of = p->grid_of;
  }
  a.n_comp = p->comp ? p->n_comp : 0;
  if (a.n_comp < 0 || a.n_comp > PF_MAX_COMP) return set_err(ctx, "pf_predict: n_comp must be in [0, PF_MAX_COMP]");
  for (int b = 0; b < a.n_comp; ++b) {
    if (p->comp_col0[b] < 0 || p->comp_ncol[b] < 0 || p->comp_col0[b] + p->comp_ncol[b] > p->fg.K)
      return set_err(ctx, "pf_predict: component block outside [0, K)");
    a.comp_col0[b] = p->comp_col0[b];
    a.comp_ncol[b] = p->comp_ncol[b];
  }
  if (a.N > 0) {
    // percentile positions exactly as numpy: q = 100*(1 -/+ w)/2; idx = q/100*(n-1)
    const double lo_p = 100.0 * (1.0 - p->interval_width) / 2.0;
    const double hi_p = 100.0 * (1.0 + p->interval_width) / 2.0;
    const double qlo = lo_p / 100.0, qhi = hi_p / 100.0;
    const double ilo = a.N * qlo + (1.0 - qlo) - 1.0;  // numpy _compute_virtual_index
    const double ihi = a.N * qhi + (1.0 - qhi) - 1.0;
    int klo = (int)floor(ilo), khi = (int)floor(ihi);
    if (klo > a.N - 2) klo = a.N - 2;
    if (khi > a.N - 2) khi = a.N - 2;
    if (klo < 0) klo = 0;
    if (khi < 0) khi = 0;
    a.k_lo = klo;
    a.fr_lo = (float)(ilo - klo);
    a.k_hi_neg = a.N - 2 - khi;
    a.fr_hi = (float)(ihi - khi);
    if (a.N == 1) { a.k_lo = 0; a.fr_lo = 0.f; a.k_hi_neg = 0; a.fr_hi = 0.f; }
    // threshold selection on the normal draws of deterministic-trend rows
    // (k_predict_mc_hist): z* with N Phi(-z*) = k + 22 expected keys beyond
    // it — exact whenever between k + 2 and 64 keys fall beyond (else the
    // general selection runs): ~99% of rows at N = 1000.  Random-trend rows
    // (k_predict_mc) use the same z* on their own sample mean / sd first
    a.zthr = 0.0f;
    const int kmax = a.k_lo > a.k_hi_neg ? a.k_lo : a.k_hi_neg;
    if (a.N >= 200 && kmax + 22 <= 60 && !getenv_flag("PF_MC_GENERAL_SELECT")) {
      const double target = (double)(kmax + 22) / (double)a.N;  // tail mass
      double lo = 0.0, hi = 10.0;
      for (int it = 0; it < 80; ++it) {
        const double mid = 0.5 * (lo + hi);
        if (0.5 * erfc(mid / sqrt(2.0)) > target) lo = mid; else hi = mid;
      }
      a.zthr = (float)(0.5 * (lo + hi));
    }
  }
  a.method = p->interval_method;
  a.cap = p->cap_scaled;
  if (a.growth == PF_GROWTH_LOGISTIC && !a.cap)
    return set_err(ctx, "pf_predict: logistic growth needs cap_scaled on the predicted rows");
  if (a.method != PF_INTERVAL_EXACT && a.method != PF_INTERVAL_SAMPLE)
    return set_err(ctx, "pf_predict: interval_method must be PF_INTERVAL_EXACT or PF_INTERVAL_SAMPLE");
  const int parts = p->parts == 0 ? (PF_PREDICT_DET | PF_PREDICT_MC) : p->parts;
  if (parts & ~(PF_PREDICT_DET | PF_PREDICT_MC)) return set_err(ctx, "pf_predict: bad parts");
  return 0;
}

int pf_predict(pf_ctx *ctx, const pf_predict_args *p, void *stream) {
  PredKArgs a;
  const int rc = make_pred_args(ctx, p, a);
  if (rc) return rc;
  if (p->n_series == 0) return 0;
  const int parts = p->parts == 0 ? (PF_PREDICT_DET | PF_PREDICT_MC) : p->parts;
  const dim3 grid((a.Tf + 256 * PF_DET_RPT - 1) / (256 * PF_DET_RPT), a.n_series);
  if (parts & PF_PREDICT_DET) {
    PF_TIMED_LAUNCH(ctx, "k_predict_det", grid.x * grid.y, (hipStream_t)stream,
                    (k_predict_det<64>), grid, dim3(256), 0, (hipStream_t)stream, a);
    PF_HIP(ctx, hipGetLastError());
  }
  if (a.N > 0 && (parts & PF_PREDICT_MC)) {
    // exact mode: one block (PF_MC_WAVES waves) per series over the random
    // rows (the horizon); sample mode: every row, <= 64 rows per wave
    // sample mode: every row; a block per (series, row range) while the
    // batch is small, one block per series (its per-sample changepoint setup
    // done once) when the series alone fill the GPU
    int gx = 1;
    if (a.method == PF_INTERVAL_SAMPLE) {
      gx = (a.Tf + 64 * PF_MC_WAVES - 1) / (64 * PF_MC_WAVES);
      const int want = (8192 + a.n_series - 1) / a.n_series;  // blocks per series for ~8k blocks
      if (gx > want) gx = want;
      if (gx < 1) gx = 1;
    }
    // (exact mode: one block per series.  More blocks per series repeat the
    // per-sample changepoint setup and were slower at every batch size
    // measured: 500 series, 1/2/4/8 blocks -> 0.198 / 0.236 / 0.316 / 0.449 ms,
    // tools/time_tail.py, profiles/r04a_tail.log)
    if (const char *e = getenv("PF_MC_GX")) {   // diagnostic override
      const int v = atoi(e);
      if (v >= 1 && v <= 64) gx = v;
    }
    const dim3 gmc(gx, a.n_series);
    if (a.tr)
      PF_TIMED_LAUNCH(ctx, "k_predict_mc", gmc.x * gmc.y, (hipStream_t)stream,
                      (k_predict_mc<64, true>), gmc, dim3(PF_MC_WAVES * 64), 0, (hipStream_t)stream, a);
    else
      PF_TIMED_LAUNCH(ctx, "k_predict_mc", gmc.x * gmc.y, (hipStream_t)stream,
                      (k_predict_mc<64, false>), gmc, dim3(PF_MC_WAVES * 64), 0, (hipStream_t)stream, a);
    PF_HIP(ctx, hipGetLastError());
    if (a.method == PF_INTERVAL_SAMPLE) {
      // the deterministic-trend rows' samples (k_predict_mc walks the random rows)
      // a block per series (its setup once) when the series alone fill the
      // GPU, more blocks (each wave a strided set of 64-row chunks) otherwise
      int hx = (a.Tf + 64 * PF_MC_WAVES - 1) / (64 * PF_MC_WAVES);
      const int hwant = (16384 + a.n_series - 1) / a.n_series;
      if (hx > hwant) hx = hwant;
      const dim3 gh(hx, a.n_series);
      PF_TIMED_LAUNCH(ctx, "k_predict_mc_hist", gh.x * gh.y, (hipStream_t)stream,
                      (k_predict_mc_hist<64>), gh, dim3(PF_MC_WAVES * 64), 0, (hipStream_t)stream, a);
      PF_HIP(ctx, hipGetLastError());
    }
  }
  return 0;
}

// pf_cv_metrics's checks and kernel arguments (shared with pf_fit_forecast)
static int make_cv_args(pf_ctx *ctx, const pf_cv_args *p, CvKArgs &a) {
  if (!p) return set_err(ctx, "pf_cv_metrics: NULL args");
  if (p->n_series < 0 || p->n_rows < 1 || p->n_groups < 1 || p->n_groups > PF_CV_GMAX ||
      p->window < 1)
    return set_err(ctx, "pf_cv_metrics: bad sizes (need n_rows >= 1, 1 <= n_groups <= 512, window >= 1)");
  if ((!p->group_start && p->n_groups != 1) || !p->y || !p->yhat || !p->metrics)
    return set_err(ctx, "pf_cv_metrics: NULL buffer");
  if (p->ld_y < 0 || p->ld_f < 0 || (p->ld_y > 0 && p->ld_y < p->n_rows) ||
      (p->ld_f > 0 && p->ld_f < p->n_rows))
    return set_err(ctx, "pf_cv_metrics: row strides must be 0 or >= n_rows");
  if (!p->group_start && p->window != p->n_rows)
    return set_err(ctx, "pf_cv_metrics: group_start NULL needs window = n_rows (one group)");
  if ((p->yhat_lower == nullptr) != (p->yhat_upper == nullptr))
    return set_err(ctx, "pf_cv_metrics: yhat_lower/yhat_upper must be both set or both NULL");
  a.n_series = p->n_series;
  a.n_rows = p->n_rows;
  a.n_groups = p->n_groups;
  a.window = p->window;
  a.ld_y = p->ld_y > 0 ? p->ld_y : p->n_rows;
  a.ld_f = p->ld_f > 0 ? p->ld_f : p->n_rows;
  a.skip_mdape = p->skip_mdape ? 1 : 0;
  a.group_start = p->group_start;
  a.y = p->y;
  a.yhat = p->yhat;
  a.ylo = p->yhat_lower;
  a.yhi = p->yhat_upper;
  a.metrics = p->metrics;
  return 0;
}

int pf_cv_metrics(pf_ctx *ctx, const pf_cv_args *p, void *stream) {
  CvKArgs a;
  const int rc = make_cv_args(ctx, p, a);
  if (rc) return rc;
  if (p->n_series == 0) return 0;
  if (p->n_groups == 1 && p->window == p->n_rows)   // one group of every row: in-sample
    PF_TIMED_LAUNCH(ctx, "k_cv_metrics", p->n_series, (hipStream_t)stream, k_cv_insample,
                    dim3(p->n_series), dim3(PF_CV_INS_WAVES * 64), 0, (hipStream_t)stream, a);
  else
    PF_TIMED_LAUNCH(ctx, "k_cv_metrics", p->n_series, (hipStream_t)stream, k_cv_metrics,
                    dim3(p->n_series), dim3(64), 0, (hipStream_t)stream, a);
  PF_HIP(ctx, hipGetLastError());
  return 0;
}

int pf_fit_forecast(pf_ctx *ctx, const pf_problem *pb, const pf_fit_opts *opts, double *theta_inout,
                    double *f_out, double *f_stan, int32_t *status, int32_t *n_iter, int32_t *n_eval,
                    const pf_predict_args *pred, const pf_cv_args *cv, int flags, int32_t *fused,
                    void *stream) {
  if (fused) *fused = 0;
  int rc = check_problem(ctx, pb);
  if (rc) return rc;
  if (!opts || !theta_inout || !f_out || !f_stan || !status || !n_iter || !n_eval)
    return set_err(ctx, "pf_fit_forecast: NULL fit output");
  if (flags & ~PF_FF_ONLY_FUSED) return set_err(ctx, "pf_fit_forecast: bad flags");
  FuseArgs fa;
  memset(&fa, 0, sizeof fa);
  rc = make_pred_args(ctx, pred, fa.p);
  if (rc) return rc;
  if (cv) {
    rc = make_cv_args(ctx, cv, fa.cv);
    if (rc) return rc;
    fa.metrics = 1;
  }
  if (pred->n_series != pb->n_series || pred->theta != theta_inout || (cv && cv->n_series != pb->n_series))
    return set_err(ctx, "pf_fit_forecast: the forecast and metrics must cover the fitted series (theta = theta_inout)");
  if (pb->n_series == 0) return 0;
  const hipStream_t st = (hipStream_t)stream;
  // one launch: one grid, exact intervals, every forecast part, in-sample metrics
  const bool can = pb->n_grids == 0 && pred->n_grids == 0 && fa.p.method == PF_INTERVAL_EXACT &&
                   (pred->parts == 0 || pred->parts == (PF_PREDICT_DET | PF_PREDICT_MC)) &&
                   (!cv || (cv->n_groups == 1 && cv->window == cv->n_rows)) && !getenv_flag("PF_NO_FUSE");
  const bool only = (flags & PF_FF_ONLY_FUSED) != 0;
  if (!can && only) return 0;
  const hipStream_t st0 = (hipStream_t)stream;
  if (can) {
    // K5 work-sharing counters (FuseArgs.ctl), zeroed on the stream
    const int n = pb->n_series;
    void *w = nullptr;
    rc = ctx_workspace2(ctx, sizeof(int) * (size_t)(2 + 3 * n), &w);
    if (rc) return rc;
    fa.ctl = (int *)w;
    PF_HIP(ctx, hipMemsetAsync(fa.ctl, 0, sizeof(int) * (size_t)(2 + 3 * n), st0));
    PF_HIP(ctx, hipMemsetD32Async((hipDeviceptr_t)(fa.ctl + 1), n * PF_FF_BLOCKS, 1, st0));
  }
  FuseReq fz{&fa, only ? 1 : 0, 0};
  FitKArgs a = make_fit_args(pb);
  a.theta = theta_inout;
  a.f_out = f_out;
  a.f_stan = f_stan;
  a.status = status;
  a.n_iter = n_iter;
  a.n_eval = n_eval;
  a.o = *opts;
  const bool maybe_tile = opts->tile_min_series >= 0 && pb->n_series >= opts->tile_min_series &&
                          pb->grid.K <= 48 && pb->n_grids == 0 && !pb->tau_series &&
                          !pb->sigmas_series;
  rc = prepare_fit_scratch(ctx, a, st, maybe_tile, pb->n_grids);
  if (rc) return rc;
  rc = dispatch_fitlike(ctx, PF_LAUNCH_FIT, a, pb->n_series, pb->fourier_orders, mode_of(pb), st, nullptr,
                        can ? &fz : nullptr);
  if (rc) return rc;
  if (fz.done) {
    if (fused) *fused = 1;
    return 0;
  }
  if (can && only) return 0;   // the fit took another path: nothing launched
  rc = pf_predict(ctx, pred, stream);
  if (rc) return rc;
  return cv ? pf_cv_metrics(ctx, cv, stream) : 0;
}

}  // extern "C"
#endif  // PF_MAIN (dispatch, C ABI part 2)

// explicit instantiations of this fit unit's group (PF_EMIT_g expands to the
// instantiation only in unit g)
#if defined(PF_TU) && PF_TU >= 1
#define PF_INST_BODY(K, O0, O1, O2, M)                                                     \
  template int launch_fitlike<PF_FIT_NW, K, O0, O1, O2, M>(pf_ctx *, int, const FitKArgs &, int, \
                                                           hipStream_t, double *, FuseReq *);
#define PF_SKIP(K, O0, O1, O2, M)
#define PF_EMIT_1 PF_SKIP
#define PF_EMIT_2 PF_SKIP
#define PF_EMIT_3 PF_SKIP
#define PF_EMIT_4 PF_SKIP
#define PF_EMIT_5 PF_SKIP
#define PF_EMIT_6 PF_SKIP
#define PF_EMIT_7 PF_SKIP
#if PF_TU == 1
#undef PF_EMIT_1
#define PF_EMIT_1 PF_INST_BODY
#elif PF_TU == 2
#undef PF_EMIT_2
#define PF_EMIT_2 PF_INST_BODY
#elif PF_TU == 3
#undef PF_EMIT_3
#define PF_EMIT_3 PF_INST_BODY
#elif PF_TU == 4
#undef PF_EMIT_4
#define PF_EMIT_4 PF_INST_BODY
#elif PF_TU == 5
#undef PF_EMIT_5
#define PF_EMIT_5 PF_INST_BODY
#elif PF_TU == 6
#undef PF_EMIT_6
#define PF_EMIT_6 PF_INST_BODY
#elif PF_TU == 7
#undef PF_EMIT_7
#define PF_EMIT_7 PF_INST_BODY
#endif
#define PF_DEF_INST(G, K, O0, O1, O2, M) PF_EMIT_##G(K, O0, O1, O2, M)
PF_FIT_INSTANCES(PF_DEF_INST)
#endif

// diagnostic stamps read-back: defined in the unit whose kernels write the
// stamps (each split unit has its own device copy of pf_dbg) — the
// reference-layout fit unit, or the single unit
#if defined(PF_TIMELINE) && (!defined(PF_TU) || PF_TU == 1)
extern "C" int pf_debug_blocks(unsigned long long *out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pf_blk), sizeof(unsigned long long) * 11 * 4096) != hipSuccess) return -2;
  unsigned long long *z = (unsigned long long *)calloc(11 * 4096, sizeof(unsigned long long));
  const hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(pf_blk), z, sizeof(unsigned long long) * 11 * 4096);
  free(z);
  return e == hipSuccess ? 0 : -2;
}
#endif
#if defined(PF_STAMPS) && (!defined(PF_TU) || PF_TU == 1)
extern "C" int pf_debug_stamps(unsigned long long *out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pf_dbg), sizeof(unsigned long long) * 32) != hipSuccess) return -2;
  if (reset) {
    unsigned long long z[32] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(pf_dbg), z, sizeof z) != hipSuccess) return -2;
  }
  return 0;
}
#endif
