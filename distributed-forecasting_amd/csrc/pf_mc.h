// pf_mc.h — K5: Monte-Carlo forecast rows.
//
// UPSTREAM predict_uncertainty → sample_posterior_predictive →
// sample_predictive_trend (Prophet 0.7.1 / 1.0): per
// sample, n ~ Poisson(S (T - 1)) new changepoints at t_c ~ U(1, T] with
// delta ~ Laplace(0, lambda = mean|delta| + 1e-8); the trend is the fitted
// piecewise trend continued over the concatenated changepoints; yhat sample
// = trend_s (1 + Xb_m) + Xb_a + N(0, sigma_obs) y_scale; the interval ends are
// np.nanpercentile(·, 2.5 / 97.5) with linear interpolation.
//
// Layout: one block of PF_MC_WAVES waves per (series, row range); a wave walks
// a contiguous run of rows in time order; 16 samples per lane (sample
// lane + 64 q).
//   * Setup (block): every sample's changepoints are drawn once from its
//     counter-based stream and packed into LDS in time order (prefix offsets;
//     ~1.2 per sample at T = 1826).
//   * Rows: a sample's trend is piecewise in t, so each lane keeps per-sample
//     running state (linear: A = sum delta, B = sum delta tau_c, trend offset
//     A tau - B with tau = t - 1; logistic: the logistic_gamma walk (k, m))
//     and absorbs a changepoint only when t passes it — O(1) per sample-row.
//   * The row's deterministic part (Xb, point trend) is computed lane-per-row
//     for 64 rows at once and broadcast by readlane.
//   * Selection: exact order statistics of up to four key sets (yhat lower /
//     upper tail, trend lower / upper tail) with interleaved wave sorts
//     (wave_tail_select).
#pragma once

#define PF_MC_WAVES 4        // waves per block
#define PF_MC_CPCAP 4096     // packed changepoint slots per block (E = N S (T-1): 1.2k at T = 1826, 3.1k at 730)
#define PF_MC_ABS (1u << 26)  // per-sample state: a changepoint was absorbed

// ---- NS independent ascending wave sorts, interleaved step by step (ILP)
template <int J, int NS>
__device__ __forceinline__ void bitonic_step_n(float (&x)[NS], bool up) {
  const bool tmin = ((pf_lane() & J) == 0) == up;
  float p[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) p[s] = shfl_xor_f32<J>(x[s]);
#pragma unroll
  for (int s = 0; s < NS; ++s) x[s] = tmin ? fminf(x[s], p[s]) : fmaxf(x[s], p[s]);
}
template <int K, int NS>
__device__ __forceinline__ void bitonic_merge_n(float (&x)[NS]) {
  const bool up = (pf_lane() & K) == 0 || K == 64;
  if constexpr (K >= 64) bitonic_step_n<32>(x, up);
  if constexpr (K >= 32) bitonic_step_n<16>(x, up);
  if constexpr (K >= 16) bitonic_step_n<8>(x, up);
  if constexpr (K >= 8) bitonic_step_n<4>(x, up);
  if constexpr (K >= 4) bitonic_step_n<2>(x, up);
  bitonic_step_n<1>(x, up);
}
template <int NS>
__device__ __forceinline__ void wave_sort_asc_n(float (&x)[NS]) {
  bitonic_merge_n<2>(x);
  bitonic_merge_n<4>(x);
  bitonic_merge_n<8>(x);
  bitonic_merge_n<16>(x);
  bitonic_merge_n<32>(x);
  bitonic_merge_n<64>(x);
}

// inclusive prefix sum of an int across the wave
__device__ __forceinline__ int wave_prefix_i32(int v) {
  v += dpp_i32<PF_DPP_SHR(1)>(v);
  v += dpp_i32<PF_DPP_SHR(2)>(v);
  v += dpp_i32<PF_DPP_SHR(4)>(v);
  v += dpp_i32<PF_DPP_SHR(8)>(v);
  v += dpp_i32<PF_DPP_BCAST15, 0xA>(v);
  v += dpp_i32<PF_DPP_BCAST31, 0xC>(v);
  return v;
}

// NV float sums across the wave (butterflies interleaved), lane 0's value
// broadcast: one uniform result per sum
template <int NV>
__device__ __forceinline__ void wave_sums_f32(float (&x)[NV]) {
#define PF_BFLY(J) _Pragma("unroll") for (int i = 0; i < NV; ++i) x[i] += shfl_xor_f32<J>(x[i]);
  PF_BFLY(1) PF_BFLY(2) PF_BFLY(4) PF_BFLY(8) PF_BFLY(16) PF_BFLY(32)
#undef PF_BFLY
#pragma unroll
  for (int i = 0; i < NV; ++i) x[i] = readlane_f32(x[i], 0);
}

// Ranks kk[s] and kk[s] + 1 (0-indexed, ascending) of NS key sets held 16 per
// lane: set s reads src[s >> 1 ? 1 : 0] (yhat / trend samples), negated for
// odd s (upper tail); absent samples are NaN (ignored by fminf/fmaxf, never
// below a threshold).  The keys strictly below a threshold U_s (M_s of them)
// are compacted into LDS (lane-local counts, one wave prefix scan, no
// per-key ballots) and sorted; a rank k < M_s is read off the sorted keys.
//   1. zc > 0 (large N): U_s = mean -/+ zc sd of the set's source, so that
//      ~k + 22 keys fall below for a normal-like law (zc = k_predict_mc's
//      zthr); exact whenever k + 2 <= M_s <= 64 for every set, else step 2;
//   2. U_s = the (kk+2)-th smallest lane minimum, so at least kk+2 keys are
//      <= U_s, and every rank >= M_s equals U_s (exact under ties — trend
//      samples without a new changepoint all equal the point trend); a
//      bisection on the ordered bit patterns when kk + 2 > 64 or more than
//      64 keys fall below U_s.
// Both steps return the exact order statistics (the same bits).
// buf: NS * 64 floats of wave-private LDS.
template <int NS>
__device__ __forceinline__ void wave_tail_select(const float (&v)[PF_NQ], const float (&tv)[PF_NQ],
                                                 const int (&kk)[NS], float *buf, float (&o0)[NS],
                                                 float (&o1)[NS], float zc = 0.0f, int N = 0) {
  const int lane = pf_lane();
  auto src = [&](int s, int q) -> float { return (s < 2) ? v[q] : tv[q]; };
  constexpr int NSRC = NS > 2 ? 2 : 1;
  float U[NS];
  int M[NS], cl[NS], pre[NS];
  for (int step = (zc > 0.0f && N > 0) ? 1 : 2; step <= 2; ++step) {
    if (step == 1) {
      float m[2 * NSRC];
#pragma unroll
      for (int i = 0; i < 2 * NSRC; ++i) m[i] = 0.0f;
#pragma unroll
      for (int q = 0; q < PF_NQ; ++q) {
#pragma unroll
        for (int r = 0; r < NSRC; ++r) {
          const float x = src(2 * r, q);
          const bool ok = x == x;
          m[2 * r] += ok ? x : 0.0f;
          m[2 * r + 1] = ok ? fmaf(x, x, m[2 * r + 1]) : m[2 * r + 1];
        }
      }
      wave_sums_f32(m);
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const float mean = m[2 * (s >> 1)] / (float)N;
        const float sd = sqrtf(fmaxf(m[2 * (s >> 1) + 1] / (float)N - mean * mean, 0.0f));
        U[s] = (s & 1) ? -(mean + zc * sd) : mean - zc * sd;
      }
    } else {
      float lm[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        if (s & 1) {
          float mx = -INFINITY;
#pragma unroll
          for (int q = 0; q < PF_NQ; ++q) mx = fmaxf(mx, src(s, q));
          lm[s] = -mx;
        } else {
          float mn = INFINITY;
#pragma unroll
          for (int q = 0; q < PF_NQ; ++q) mn = fminf(mn, src(s, q));
          lm[s] = mn;
        }
      }
      wave_sort_asc_n(lm);
#pragma unroll
      for (int s = 0; s < NS; ++s) U[s] = (kk[s] + 1 < 64) ? readlane_f32(lm[s], kk[s] + 1) : INFINITY;
    }
    PF_STAMP1(10);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      int c = 0;
#pragma unroll
      for (int q = 0; q < PF_NQ; ++q) {
        const float x = src(s, q);
        c += ((s & 1) ? (x > -U[s]) : (x < U[s])) ? 1 : 0;
      }
      cl[s] = c;
      pre[s] = wave_prefix_i32(c);
      M[s] = __builtin_amdgcn_readlane(pre[s], 63);
    }
    if (step == 1) {
      bool ok = true;
#pragma unroll
      for (int s = 0; s < NS; ++s) ok = ok && M[s] >= kk[s] + 2 && M[s] <= 64;
      if (ok) { PF_COUNTW(13); break; }
    }
  }
  PF_COUNTW(14);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    int w = pre[s] - cl[s];
#pragma unroll
    for (int q = 0; q < PF_NQ; ++q) {
      const float x = src(s, q);
      const bool pr = (s & 1) ? (x > -U[s]) : (x < U[s]);
      if (pr && w < 64) buf[s * 64 + w] = (s & 1) ? -x : x;
      w += pr ? 1 : 0;
    }
  }
  PF_STAMP1(11);
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  float c[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) c[s] = (lane < M[s]) ? buf[s * 64 + lane] : INFINITY;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  wave_sort_asc_n(c);
  PF_STAMP1(12);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int k = kk[s];
    if (k + 1 < 64 && M[s] <= 64) {
      o0[s] = (k < M[s]) ? readlane_f32(c[s], k) : U[s];
      o1[s] = (k + 1 < M[s]) ? readlane_f32(c[s], k + 1) : U[s];
    } else {
      PF_COUNTW(25);
      for (int want = 0; want < 2; ++want) {
        uint32_t lo = 0u, hi = 0xFFFFFFFFu;
        while (lo < hi) {
          const uint32_t mid = lo + ((hi - lo) >> 1);
          int cnt = 0;
#pragma unroll
          for (int q = 0; q < PF_NQ; ++q) {
            const float x = src(s, q);
            const float kx = (x != x) ? INFINITY : ((s & 1) ? -x : x);
            cnt += __popcll(__ballot(pf_f2ord(kx) <= mid));
          }
          if (cnt >= k + want + 1) hi = mid; else lo = mid + 1;
        }
        if (want == 0) o0[s] = pf_ord2f(lo); else o1[s] = pf_ord2f(lo);
      }
    }
  }
}

// Deterministic-trend rows: the samples are yhat + sd z with z standard
// normal, a monotone map, so the order statistics are those of z.  Ranks
// kk[0], kk[0]+1 of z (lower tail) and kk[1], kk[1]+1 of -z (upper tail)
// from the keys beyond the fixed threshold zthr: exact when each tail holds
// between kk + 2 and 64 keys (returns false otherwise: the caller runs the
// general wave_tail_select).  Absent samples are NaN (never beyond).
__device__ __forceinline__ bool wave_tail_select_z(const float (&z)[PF_NQ], const int (&kk)[2], float zthr,
                                                   float *buf, float (&o0)[2], float (&o1)[2]) {
  // buf: 2 * 64 floats of wave-private LDS
  const int lane = pf_lane();
  int c0 = 0, c1 = 0;
#pragma unroll
  for (int q = 0; q < PF_NQ; ++q) {
    c0 += (z[q] < -zthr) ? 1 : 0;
    c1 += (z[q] > zthr) ? 1 : 0;
  }
  const int p0 = wave_prefix_i32(c0), p1 = wave_prefix_i32(c1);
  const int M0 = __builtin_amdgcn_readlane(p0, 63), M1 = __builtin_amdgcn_readlane(p1, 63);
  if (M0 < kk[0] + 2 || M0 > 64 || M1 < kk[1] + 2 || M1 > 64) return false;
  int w0 = p0 - c0, w1 = 64 + p1 - c1;
#pragma unroll
  for (int q = 0; q < PF_NQ; ++q) {
    if (z[q] < -zthr) buf[w0++] = z[q];
    if (z[q] > zthr) buf[w1++] = -z[q];
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  float c[2];
  c[0] = (lane < M0) ? buf[lane] : INFINITY;
  c[1] = (lane < M1) ? buf[64 + lane] : INFINITY;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  wave_sort_asc_n(c);
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    o0[s] = readlane_f32(c[s], kk[s]);
    o1[s] = readlane_f32(c[s], kk[s] + 1);
  }
  return true;
}

// sample smp's c-th new changepoint: tau = t_c - 1 ~ U(0, T - 1], delta ~ Laplace(0, lam)
__device__ __forceinline__ void mc_sample_cp(uint32_t seed0, uint32_t seed1, uint32_t series, int smp,
                                             int c, double t_max, double lam, double &tau, double &dl) {
  const pf_u4 rc = philox4x32_10(pf_u4{(uint32_t)smp, (uint32_t)(c + 1), (uint32_t)series, 0x7EE2D00Du},
                                 seed0 ^ 0x5A5A5A5Au, seed1);
  tau = pf_u01d(rc.x, rc.y) * (t_max - 1.0);
  const double ul = pf_u01d(rc.z, rc.w);
  dl = (ul >= 0.5) ? -lam * log(2.0 - ul - ul) : lam * log(ul + ul);
}

// Poisson(lam_pois) count of sample smp by inversion (e_neg = exp(-lam_pois))
__device__ __forceinline__ int mc_sample_count(uint32_t seed0, uint32_t seed1, uint32_t series, int smp,
                                               double lam_pois, double e_neg) {
  const pf_u4 r0 = philox4x32_10(pf_u4{(uint32_t)smp, 0u, (uint32_t)series, 0x7EE2D00Du},
                                 seed0 ^ 0x5A5A5A5Au, seed1);
  const double u0 = pf_u01d(r0.x, r0.y);
  int n = 0;
  if (lam_pois > 0.0) {
    double p = e_neg, F = p;
    while (u0 > F && n < 100000) {
      ++n;
      p *= lam_pois / (double)n;
      F += p;
      if (p == 0.0 && F < u0) break;
    }
  }
  return n;
}

// Trend sample at tau re-derived from the counter-based stream (blocks whose
// changepoints overflow the LDS slots: horizons far beyond the history).
__device__ __forceinline__ float mc_trend_direct(uint32_t seed0, uint32_t seed1, uint32_t series, int smp, int n,
                                                 double t_max, double lam, double tau, bool logi, double trend,
                                                 double ysc, double capy, double k0, double m0) {
  if (!logi) {
    double off = 0.0;
    for (int c = 0; c < n; ++c) {
      double tc, dl;
      mc_sample_cp(seed0, seed1, series, smp, c, t_max, lam, tc, dl);
      if (tau >= tc) off += dl * (tau - tc);
    }
    return (float)(trend + ysc * off);
  }
  // logistic: absorb the changepoints before tau in time order (selection by
  // repeated minimum; no per-sample storage)
  double kc = k0, mc = m0, last = -1.0;
  bool any = false;
  for (int it = 0; it < n; ++it) {
    double best = INFINITY, bdl = 0.0;
    for (int c = 0; c < n; ++c) {
      double tc, dl;
      mc_sample_cp(seed0, seed1, series, smp, c, t_max, lam, tc, dl);
      if (tc > last && tc < best) { best = tc; bdl = dl; }
    }
    if (!(best <= tau)) break;
    const double kn = kc + bdl;
    mc = mc + (1.0 + best - mc) * (1.0 - kc / kn);
    kc = kn;
    last = best;
    any = true;
  }
  if (!any) return (float)trend;
  return (float)(capy / (1.0 + exp(-(kc * (1.0 + tau - mc)))));
}

// The lane's PF_NQ standard-normal noise draws of one row (sample lane + 64 q;
// absent samples, lane + 64 q >= N, are NaN): 16 uniforms of 24 bits from 12
// Philox words (three calls keyed (call, lane, row, series); each word's top
// 24 bits, the fourth uniform of a group of three words from their low
// bytes), Box-Muller pairs.
__device__ __forceinline__ void mc_row_normals(const PredKArgs &a, uint32_t sid, int row, float (&z)[PF_NQ]) {
  const int lane = pf_lane();
  uint32_t uw[PF_NQ];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const pf_u4 rr = philox4x32_10(pf_u4{(uint32_t)c, (uint32_t)lane, (uint32_t)row, sid}, a.seed0, a.seed1);
    const uint32_t w[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // words 4c + j: groups g = (4c + j) / 3 of three words
      const int wi = 4 * c + j, g = wi / 3, m = wi % 3;
      uw[4 * g + m] = w[j];
      if (m == 0) uw[4 * g + 3] = (w[j] & 0xFFu) << 8;
      else uw[4 * g + 3] |= (w[j] & 0xFFu) << (8 + 8 * m);
    }
  }
#pragma unroll
  for (int c = 0; c < PF_NQ / 4; ++c) {
    pf_box_muller(pf_u01f(uw[4 * c]), pf_u01f(uw[4 * c + 1]), z[4 * c], z[4 * c + 1]);
    pf_box_muller(pf_u01f(uw[4 * c + 2]), pf_u01f(uw[4 * c + 3]), z[4 * c + 2], z[4 * c + 3]);
  }
#pragma unroll
  for (int q = 0; q < PF_NQ; ++q)
    if (lane + 64 * q >= a.N) z[q] = __builtin_nanf("");
}

// The wave's rows [row_b, row_e), every one a random-trend row (t > 1; the
// deterministic-trend rows are k_predict_det's (exact) or k_predict_mc_hist's
// (sample)).  DIRECT: every trend sample re-derived from the stream (s_meta =
// count); otherwise the per-sample running state over the packed changepoints.
template <bool DIRECT, bool TR>
__device__ __forceinline__ void mc_rows(const PredKArgs &a, const PredSeries &ps, const float2 *s_cp,
                                        const uint32_t *s_meta, float *buf, int series, uint32_t sid,
                                        double t_max, int row_b, int row_e) {
  const int lane = pf_lane();
  const int N = a.N;
  const bool logi = a.growth == PF_GROWTH_LOGISTIC;
  const double ysc = ps.ysc, lam = ps.lam;
  const float sd = (float)(ps.sigma * ysc);
  const double k0 = ps.kseg[a.S], m0 = ps.mseg[a.S];
  // per-sample trend state: st = index of the next changepoint (its tau /
  // delta held in nxt / nxd) | end << 13 | PF_MC_ABS once one was absorbed
  uint32_t st[PF_NQ];
  float nxt[PF_NQ], nxd[PF_NQ], s1[PF_NQ], s2[PF_NQ];
  if constexpr (!DIRECT) {
#pragma unroll
    for (int q = 0; q < PF_NQ; ++q) {
      const int smp = lane + 64 * q;
      const uint32_t meta = (smp < N) ? s_meta[smp] : 0u;
      const uint32_t p0 = meta & 0x1FFFu, e0 = (meta >> 13) & 0x1FFFu;
      st[q] = meta;
      const float2 cp0 = (p0 < e0) ? s_cp[p0] : make_float2(INFINITY, 0.0f);
      nxt[q] = cp0.x;
      nxd[q] = cp0.y;
      s1[q] = logi ? (float)k0 : 0.0f;
      s2[q] = logi ? (float)m0 : 0.0f;
    }
  }
  const int kk4[4] = {a.k_lo, a.k_hi_neg, a.k_lo, a.k_hi_neg};
  const int kk2[2] = {a.k_lo, a.k_hi_neg};
  for (int c0 = row_b; c0 < row_e; c0 += 64) {
    const int nr = min(64, row_e - c0);
    // lane-per-row deterministic part (same arithmetic as k_predict_det)
    const int myrow = c0 + lane;
    const bool rv = lane < nr;
    double ti = 0.0, xbm = 0.0, xba = 0.0, trs = 0.0, capr = 0.0;
    if (rv) {
      ti = a.t[myrow];
      const int sg = a.seg[myrow];
      pred_row_dot(a, ps, myrow, xbm, xba);
      trs = pred_trend(a, ps, series, myrow, ti, sg);
      if (logi) capr = a.cap[(size_t)series * a.Tp + myrow];
    }
    const double l_trend = trs * ysc, l_add = xba * ysc;
    const float lf_tau = (float)(ti - 1.0), lf_trend = (float)l_trend, lf_u1 = (float)(1.0 + xbm);
    const float lf_add = (float)l_add;
    const float lf_capy = (float)(ysc * capr);
    float o_ylo = 0.f, o_yhi = 0.f, o_tlo = 0.f, o_thi = 0.f;
    PF_STAMP1(2);
    // the samples of row c0 + r: v (yhat) and, with TR, tv (trend); advances
    // the per-sample changepoint state to the row's time
    auto gen_row = [&](int r, float (&v)[PF_NQ], float (&tv)[TR ? PF_NQ : 1]) {
      const int row = c0 + r;
      const float tau = readlane_f32(lf_tau, r);
      const float trendf = readlane_f32(lf_trend, r);
      const float u1 = readlane_f32(lf_u1, r), addf = readlane_f32(lf_add, r);
      float z[PF_NQ];
      const float capy = readlane_f32(lf_capy, r);
      if constexpr (DIRECT) {
        mc_row_normals(a, sid, row, z);
#pragma unroll
        for (int q = 0; q < PF_NQ; ++q) {
          const int smp = lane + 64 * q;
          const float ts = (smp < N) ? mc_trend_direct(a.seed0, a.seed1, sid, smp, (int)s_meta[smp], t_max, lam,
                                                       (double)tau, logi, (double)trendf, ysc, (double)capy, k0, m0)
                                     : __builtin_nanf("");
          if constexpr (TR) tv[q] = ts;
          v[q] = (smp < N) ? fmaf(sd, z[q], fmaf(ts, u1, addf)) : __builtin_nanf("");
        }
      } else {
        // absorb the changepoints passed since the previous row: one pass
        // over the samples with the next changepoint held in registers (the
        // LDS loads of different samples overlap), repeated only if a sample
        // passed two changepoints since the previous row
        while (true) {
#pragma unroll
          for (int q = 0; q < PF_NQ; ++q) {
            const bool cr = tau >= nxt[q];
            if (__ballot(cr) != 0ull) {
              if (cr) {
                const uint32_t p = (st[q] & 0x1FFFu) + 1u, e = (st[q] >> 13) & 0x1FFFu;
                if (!logi) {
                  s1[q] += nxd[q];
                  s2[q] = fmaf(nxd[q], nxt[q], s2[q]);
                } else {
                  const float kn = s1[q] + nxd[q];
                  s2[q] = s2[q] + (1.0f + nxt[q] - s2[q]) * (1.0f - s1[q] / kn);
                  s1[q] = kn;
                }
                st[q] = (st[q] & ~0x1FFFu) | p | PF_MC_ABS;
                const float2 cp = (p < e) ? s_cp[p] : make_float2(INFINITY, 0.0f);
                nxt[q] = cp.x;
                nxd[q] = cp.y;
              }
            }
          }
          unsigned long long more = 0ull;
#pragma unroll
          for (int q = 0; q < PF_NQ; ++q) more |= __ballot(tau >= nxt[q]);
          if (more == 0ull) break;
        }
        PF_STAMP1(4);
        mc_row_normals(a, sid, row, z);
        PF_STAMP1(5);
        const float ysf = (float)ysc;
#pragma unroll
        for (int q = 0; q < PF_NQ; ++q) {
          float trs_s;
          if (!logi) trs_s = fmaf(ysf, fmaf(s1[q], tau, -s2[q]), trendf);
          else trs_s = (st[q] & PF_MC_ABS) ? capy / (1.0f + __expf(-(s1[q] * (1.0f + tau - s2[q])))) : trendf;
          const bool on = lane + 64 * q < N;
          if constexpr (TR) tv[q] = on ? trs_s : __builtin_nanf("");
          v[q] = on ? fmaf(sd, z[q], fmaf(trs_s, u1, addf)) : __builtin_nanf("");
        }
      }
    };
    if constexpr (TR) {
      for (int r = 0; r < nr; ++r) {
        PF_STAMP1(3);
        if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) PF_COUNT(9);
        float v[PF_NQ], tv[PF_NQ];
        gen_row(r, v, tv);
        PF_STAMP1(6);
        float o0[4], o1[4];
        // (the trend sets are tie-heavy: the moment threshold rarely fits them)
        wave_tail_select<4>(v, tv, kk4, buf, o0, o1);
        if (N == 1) { for (int s = 0; s < 4; ++s) o1[s] = o0[s]; }
        const float ylo = np_lerp(o0[0], o1[0], a.fr_lo);
        const float yhi = np_lerp(-o1[1], -o0[1], a.fr_hi);
        const float tlo = np_lerp(o0[2], o1[2], a.fr_lo);
        const float thi = np_lerp(-o1[3], -o0[3], a.fr_hi);
        PF_STAMP1(7);
        if (lane == r) { o_ylo = ylo; o_yhi = yhi; o_tlo = tlo; o_thi = thi; }
      }
    } else {
      // yhat tails only (no trend bands requested): two rows per selection
      // (four interleaved key sets: more independent work per step)
      for (int r = 0; r < nr; r += 2) {
        PF_STAMP1(3);
        if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) PF_COUNT(9);
        float v0[PF_NQ], v1[PF_NQ], unused[1];
        gen_row(r, v0, unused);
        const bool two = r + 1 < nr;
        if (two) gen_row(r + 1, v1, unused);
        PF_STAMP1(6);
        if (two) {
          float o0[4], o1[4];
          wave_tail_select<4>(v0, v1, kk4, buf, o0, o1, a.zthr, N);
          if (N == 1) { for (int s = 0; s < 4; ++s) o1[s] = o0[s]; }
          const float ylo0 = np_lerp(o0[0], o1[0], a.fr_lo), yhi0 = np_lerp(-o1[1], -o0[1], a.fr_hi);
          const float ylo1 = np_lerp(o0[2], o1[2], a.fr_lo), yhi1 = np_lerp(-o1[3], -o0[3], a.fr_hi);
          if (lane == r) { o_ylo = ylo0; o_yhi = yhi0; }
          if (lane == r + 1) { o_ylo = ylo1; o_yhi = yhi1; }
        } else {
          float o0[2], o1[2];
          wave_tail_select<2>(v0, v0, kk2, buf, o0, o1, a.zthr, N);
          if (N == 1) { o1[0] = o0[0]; o1[1] = o0[1]; }
          if (lane == r) { o_ylo = np_lerp(o0[0], o1[0], a.fr_lo); o_yhi = np_lerp(-o1[1], -o0[1], a.fr_hi); }
        }
        PF_STAMP1(7);
      }
    }
    if (rv) {
      const size_t o = (size_t)series * a.Tp + myrow;
      a.ylo[o] = o_ylo;
      a.yhi[o] = o_yhi;
      if (a.tr) { a.trlo[o] = o_tlo; a.trhi[o] = o_thi; }
    }
  }
}

template <bool TR>
__device__ __forceinline__ void mc_block_rows(const PredKArgs &a, const PredSeries &ps, int series, uint32_t sid,
                                              int bx, int gdx, const float2 *s_cp, const uint32_t *s_meta,
                                              float *s_buf, const double *s_wsum, const int *s_r0);

// One block's share of a series' Monte-Carlo rows (block bx of gdx over the
// random rows), the series' PredSeries already set up in ps (pred_setup +
// a block barrier).  LDS: s_cp [PF_MC_CPCAP], s_meta [64 PF_NQ], s_buf
// [PF_MC_WAVES][4 * 64], s_wsum [PF_MC_WAVES], s_r0 [1].  A wave without rows
// returns early (no block-level sync after the setup).  Shared by
// k_predict_mc and the fused forecast epilogue (k_fit_forecast).
__device__ __forceinline__ void mc_setup(const PredKArgs &a, const PredSeries &ps, uint32_t sid,
                                         float2 *s_cp, uint32_t *s_meta, double *s_wsum, int *s_r0) {
  constexpr int NT = PF_MC_WAVES * 64;
  constexpr int SPT = (64 * PF_NQ) / NT;  // samples per thread in the setup
  const int lane = pf_lane(), wave = pf_wave(), tid = threadIdx.x;
  const int N = a.N;
  const double t_max = a.t[a.Tf - 1];
  {
    // first random-trend row (rows sorted by t): independent loads, min
    int loc = a.Tf;
    for (int b0 = 0; b0 < a.Tf; b0 += 8 * NT) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = b0 + i * NT + tid;
        if (r < a.Tf && pred_row_random(a, a.t[r], t_max)) loc = min(loc, r);
      }
    }
    if (loc < a.Tf) atomicMin(s_r0, loc);
  }
  // ---- per-sample new changepoints, packed in time order
  const double lam = ps.lam;
  const bool any_random = pred_row_random(a, t_max, t_max);
  const double lam_pois = any_random ? (double)a.S * (t_max - 1.0) : 0.0;
  int cnt[SPT];
  int tot = 0;
  {
    const double e_neg = exp(-lam_pois);
#pragma unroll
    for (int i = 0; i < SPT; ++i) {
      const int smp = tid + i * NT;
      cnt[i] = (any_random && smp < N) ? mc_sample_count(a.seed0, a.seed1, sid, smp, lam_pois, e_neg) : 0;
      tot += cnt[i];
    }
  }
  const double inc = wave_prefix_sum((double)tot);
  if (lane == 63) s_wsum[wave] = inc;
  __syncthreads();
  double total = 0.0, base = inc - (double)tot;
  for (int w = 0; w < PF_MC_WAVES; ++w) {
    total += s_wsum[w];
    if (w < wave) base += s_wsum[w];
  }
  const bool ovf = total > (double)PF_MC_CPCAP;  // uniform
  int off = (int)base;
#pragma unroll
  for (int i = 0; i < SPT; ++i) {
    const int smp = tid + i * NT;
    const int n = cnt[i];
    if (!ovf) {
      for (int c = 0; c < n; ++c) {
        double tau, dl;
        mc_sample_cp(a.seed0, a.seed1, sid, smp, c, t_max, lam, tau, dl);
        const float tf = (float)tau;
        int q = c;
        while (q > 0 && s_cp[off + q - 1].x > tf) { s_cp[off + q] = s_cp[off + q - 1]; --q; }
        s_cp[off + q] = make_float2(tf, (float)dl);
      }
      s_meta[smp] = (uint32_t)off | ((uint32_t)(off + n) << 13);
    } else {
      s_meta[smp] = (uint32_t)n;
    }
    off += n;
  }
  __syncthreads();
  PF_STAMP1(1);
}

template <bool TR>
__device__ __forceinline__ void mc_block(const PredKArgs &a, const PredSeries &ps, int series, uint32_t sid,
                                         int bx, int gdx, float2 *s_cp, uint32_t *s_meta, float *s_buf,
                                         double *s_wsum, int *s_r0) {
  mc_setup(a, ps, sid, s_cp, s_meta, s_wsum, s_r0);
  mc_block_rows<TR>(a, ps, series, sid, bx, gdx, s_cp, s_meta, s_buf, s_wsum, s_r0);
}

// The row part of mc_block (after its setup: s_r0, s_cp / s_meta packed,
// s_wsum's total): block bx of gdx over the random rows.  A workgroup that
// ran the setup once can walk several of its series' blocks.
template <bool TR>
__device__ __forceinline__ void mc_block_rows(const PredKArgs &a, const PredSeries &ps, int series, uint32_t sid,
                                              int bx, int gdx, const float2 *s_cp, const uint32_t *s_meta,
                                              float *s_buf, const double *s_wsum, const int *s_r0) {
  const int wave = pf_wave();
  const double t_max = a.t[a.Tf - 1];
  double total = 0.0;
  for (int w = 0; w < PF_MC_WAVES; ++w) total += s_wsum[w];
  const bool ovf = total > (double)PF_MC_CPCAP;  // uniform
  const int r0 = *s_r0;
  const int nrows = a.Tf - r0;
  if (nrows <= 0) return;
  const int nw = gdx * PF_MC_WAVES;
  const int rpw = (nrows + nw - 1) / nw;
  const int row_b = r0 + (bx * PF_MC_WAVES + wave) * rpw;
  const int row_e = min(row_b + rpw, a.Tf);
  if (row_b >= row_e) return;  // no block-level sync below
  float *buf = s_buf + wave * 4 * 64;
  if (ovf) mc_rows<true, TR>(a, ps, s_cp, s_meta, buf, series, sid, t_max, row_b, row_e);
  else mc_rows<false, TR>(a, ps, s_cp, s_meta, buf, series, sid, t_max, row_b, row_e);
}

template <int KMAX, bool TR>
__global__ __launch_bounds__(PF_MC_WAVES * 64) void k_predict_mc(PredKArgs a0) {
  PredKArgs a = a0;
  if (a0.grid_of) bind_pred_grid(a, blockIdx.y);
  __shared__ PredSeries ps;
  __shared__ float2 s_cp[PF_MC_CPCAP];     // (tau_c, delta), each sample's run in time order
  __shared__ uint32_t s_meta[64 * PF_NQ];  // first slot | end << 13  (overflow: count)
  __shared__ float s_buf[PF_MC_WAVES][4 * 64];
  __shared__ double s_wsum[PF_MC_WAVES];
  __shared__ int s_r0;
  const int series = blockIdx.y;
  const uint32_t sid = a.series_id ? a.series_id[series] : (uint32_t)series;
  PF_STAMP1(0);
  if (threadIdx.x == 0) s_r0 = a.Tf;
  pred_setup(a, series, ps);
  __syncthreads();
  mc_block<TR>(a, ps, series, sid, blockIdx.x, gridDim.x, s_cp, s_meta, &s_buf[0][0], s_wsum, &s_r0);
}

// ---- sample mode, deterministic-trend rows (the history: t <= 1, or every
// row under flat growth).  UPSTREAM's samples of such a row are yhat + sd z_i
// (no new changepoints), so nothing carries from row to row: a wave walks
// 64-row chunks (chunk = wave index + k x the grid's waves) with no
// per-sample changepoint state, setup or block-level sync in the row loop,
// which keeps the kernel far below k_predict_mc's registers (more waves per
// SIMD to hide the Philox / Box-Muller / selection latency chains).  The
// draws and the selection are k_predict_mc's row arithmetic (mc_row_normals,
// the threshold selection on z, the general wave_tail_select otherwise):
// the intervals are bitwise those of one kernel walking every row.  Rows are
// sorted by t, so the deterministic rows are a prefix: a wave stops at its
// first chunk without one (k_predict_mc writes the random rows).
// Grid (<= ceil(Tf / (64 PF_MC_WAVES)), n_series).
template <int KMAX>
__global__ __launch_bounds__(PF_MC_WAVES * 64) void k_predict_mc_hist(PredKArgs a0) {
  PredKArgs a = a0;
  if (a0.grid_of) bind_pred_grid(a, blockIdx.y);
  __shared__ PredSeries ps;
  __shared__ float s_buf[PF_MC_WAVES][2 * 64];
  const int series = blockIdx.y, lane = pf_lane(), wave = pf_wave();
  const int nchunk = (a.Tf + 63) / 64;
  if ((int)blockIdx.x * PF_MC_WAVES >= nchunk) return;  // uniform per block (ragged grids)
  const uint32_t sid = a.series_id ? a.series_id[series] : (uint32_t)series;
  const int N = a.N;
  pred_setup(a, series, ps);
  __syncthreads();
  const double t_max = a.t[a.Tf - 1];
  const double ysc = ps.ysc;
  const float sd = (float)(ps.sigma * ysc);
  const int kk2[2] = {a.k_lo, a.k_hi_neg};
  float *buf = s_buf[wave];
  for (int ch = blockIdx.x * PF_MC_WAVES + wave; ch < nchunk; ch += gridDim.x * PF_MC_WAVES) {
    const int c0 = ch * 64;
    const int nr = min(64, a.Tf - c0);
    const int myrow = c0 + lane;
    const bool rv = lane < nr;
    // lane-per-row deterministic part (k_predict_mc's arithmetic)
    double ti = 0.0, xbm = 0.0, xba = 0.0, trs = 0.0;
    if (rv) {
      ti = a.t[myrow];
      pred_row_dot(a, ps, myrow, xbm, xba);
      trs = pred_trend(a, ps, series, myrow, ti, a.seg[myrow]);
    }
    const double l_trend = trs * ysc, l_add = xba * ysc;
    const float lf_trend = (float)l_trend, lf_yhat = (float)(l_trend * (1.0 + xbm) + l_add);
    const bool mine = rv && !pred_row_random(a, ti, t_max);
    unsigned long long todo = __ballot(mine);
    if (todo == 0ull) break;
    float o_ylo = 0.f, o_yhi = 0.f;
    while (todo) {
      const int r = __builtin_ctzll(todo);
      todo &= todo - 1ull;
      const int row = c0 + r;
      const float yh = readlane_f32(lf_yhat, r);
      float z[PF_NQ];
      mc_row_normals(a, sid, row, z);
      float ylo, yhi;
      float zo0[2], zo1[2];
      if (a.zthr > 0.0f && wave_tail_select_z(z, kk2, a.zthr, buf, zo0, zo1)) {
        // order statistics of yhat + sd z: the same monotone map of z's
        ylo = np_lerp(fmaf(sd, zo0[0], yh), fmaf(sd, zo1[0], yh), a.fr_lo);
        yhi = np_lerp(fmaf(sd, -zo1[1], yh), fmaf(sd, -zo0[1], yh), a.fr_hi);
      } else {
        float v[PF_NQ], o0[2], o1[2];
#pragma unroll
        for (int q = 0; q < PF_NQ; ++q) v[q] = (lane + 64 * q < N) ? fmaf(sd, z[q], yh) : __builtin_nanf("");
        wave_tail_select<2>(v, v, kk2, buf, o0, o1);
        if (N == 1) { o1[0] = o0[0]; o1[1] = o0[1]; }
        ylo = np_lerp(o0[0], o1[0], a.fr_lo);
        yhi = np_lerp(-o1[1], -o0[1], a.fr_hi);
      }
      if (lane == r) { o_ylo = ylo; o_yhi = yhi; }
    }
    if (mine) {
      const size_t o = (size_t)series * a.Tp + myrow;
      a.ylo[o] = o_ylo;
      a.yhi[o] = o_yhi;
      if (a.tr) { a.trlo[o] = lf_trend; a.trhi[o] = lf_trend; }
    }
  }
}
