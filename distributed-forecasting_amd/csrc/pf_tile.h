// pf_tile.h — K3T: tiled batched Stan L-BFGS, 16 series per workgroup.
//
// The throughput form of K3 (north_star (2)/(3)):
// a workgroup owns a tile of PF_TS = 16 series that share one date grid.
// Every objective evaluation evaluates all 16 series at their own trial
// points at once, and the seasonal contractions are dense GEMMs on the FP64
// matrix cores:
//   X[T x K] . B[K x 16]  (B = beta o s_m per series)       -> Xb, C layout
//   X'[K x T] . W[T x 16] (W = r o trend per series)        -> beta gradient
// both v_mfma_f64_16x16x4f64 over 16-row chunks (the first product's
// accumulator registers are the second product's B operand: the C layout's
// rows are the next MFMA's k index).  The changepoint contraction A[T x C]
// . Delta[C x 16] is a step matrix: the trend reads per-series segment
// tables (k_s, m_s) — the exact contraction at O(1) per element — and its
// adjoint is a segment sum of G = r(1 + Xb_m), G t per series.
// Residuals, likelihood and prior terms are elementwise in the C layout.
//
// L-BFGS: each series owns a lane quad of wave 0 (16 parameters per lane,
// p = q + 4i) running Stan 2.19's BFGSMinimizer<LBFGSUpdate> + Wolfe line
// search (same control flow as oracle/stan_lbfgs.c, two-loop recursion),
// with per-series convergence masking: a series that terminates stops
// moving and the tile exits when all 16 have.  State lives in LDS.
//
// Scope: linear / flat growth, P = 3 + S + K <= 60, shared prior scales
// (the reference layout and the fallback-free configs[2]/[3] shapes); the
// per-series kernel K3 covers the rest.  The exact-MAP polish runs after it
// (k_polish, one workgroup per series).
#pragma once

#define PF_TS 16   // series per tile (MFMA N)
#define PF_TNW 4   // waves per tile workgroup
#define PF_TH 5    // L-BFGS history (Stan default)

struct TileZ {
  double fk, fk1, fq, gpq, alpha, alphak_1, dfp, c1dfp, c2dfp, alpha0, alpha1, prevF, prevDFp;
  double alo, aloF, aloDFp, ahi, ahiF, ahiDFp, lastDFp, dfp_prev, gammak;
  int state, itNum, resetB, nits, lsRestarts, zit, hcount, head, ret, n_eval, bad, done;
};

template <int MODE>
struct TileSmem {
  static constexpr int NSET = ((MODE & 3) == 2) ? 2 : 1;
  static constexpr int KP = 32;  // padded feature count (K <= 32)
  int V;                         // per-series vector stride (doubles)
  double *xk, *gk, *pk, *xq, *gq;  // [16][V]
  double *hs, *hy;               // [H][16][V]
  double *hrho;                  // [16][H]
  double *kseg, *mseg;           // [16][32]
  double *bm, *ba;               // [KP][16]
  double *gb;                    // [NSET][KP][16]
  double *sg0, *sg1;             // [32][16] segment sums of G, G t
  double *rr;                    // [16]
  double *sig;                   // [16][2] sigma, 1/sigma^2
  double *ctc, *csg, *csm, *csa; // [64]
  TileZ *z;                      // [16]
  int *flag;                     // [4]
  static __host__ __device__ int vstride(int P) { return 4 * ((P + 3) / 4) + 4; }
  static __host__ __device__ size_t bytes(int P) {
    const size_t V = (size_t)vstride(P);
    const size_t d = (5 + 2 * PF_TH) * PF_TS * V + PF_TS * PF_TH + 2 * PF_TS * 32 +
                     2 * KP * PF_TS + NSET * KP * PF_TS + 2 * 32 * PF_TS + PF_TS + 2 * PF_TS + 4 * 64;
    return d * sizeof(double) + PF_TS * sizeof(TileZ) + 64;
  }
  __device__ void carve(char *base, int P) {
    V = vstride(P);
    double *p = reinterpret_cast<double *>(base);
    const size_t vec = (size_t)PF_TS * V;
    xk = p; p += vec;
    gk = p; p += vec;
    pk = p; p += vec;
    xq = p; p += vec;
    gq = p; p += vec;
    hs = p; p += PF_TH * vec;
    hy = p; p += PF_TH * vec;
    hrho = p; p += PF_TS * PF_TH;
    kseg = p; p += PF_TS * 32;
    mseg = p; p += PF_TS * 32;
    bm = p; p += KP * PF_TS;
    ba = p; p += KP * PF_TS;
    gb = p; p += NSET * KP * PF_TS;
    sg0 = p; p += 32 * PF_TS;
    sg1 = p; p += 32 * PF_TS;
    rr = p; p += PF_TS;
    sig = p; p += 2 * PF_TS;
    ctc = p; p += 64;
    csg = p; p += 64;
    csm = p; p += 64;
    csa = p; p += 64;
    z = reinterpret_cast<TileZ *>(p);
    flag = reinterpret_cast<int *>(z + PF_TS);
  }
};

// sum over the 4 lanes of a quad (uniform within the quad)
__device__ __forceinline__ double quad_sum(double v) {
  v += dpp_f64<PF_DPP_QXOR1>(v);
  v += dpp_f64<PF_DPP_QXOR2>(v);
  return v;
}

// Publish series j's trial point xq: segment tables, beta o s_m / s_a, sigma.
// Lane quad of series j; q = lane & 3.
template <int MODE>
__device__ __forceinline__ void tile_publish(const FitKArgs &a, TileSmem<MODE> &sm, int j, int q) {
  const int S = a.S, K = a.K, V = sm.V;
  const double *x = sm.xq + (size_t)j * V;
  if (q == 0) {
    const double k = x[0], m = x[1];
    double cd = 0.0, ctd = 0.0;
    sm.kseg[j * 32] = k;
    sm.mseg[j * 32] = m;
    for (int jj = 0; jj < S; ++jj) {
      const double d = x[2 + jj];
      cd += d;
      ctd = fma(sm.ctc[jj], d, ctd);
      sm.kseg[j * 32 + jj + 1] = k + cd;
      sm.mseg[j * 32 + jj + 1] = m - ctd;
    }
    const double sg = exp(x[2 + S]);
    sm.sig[2 * j] = sg;
    sm.sig[2 * j + 1] = 1.0 / (sg * sg);
  }
  for (int f = q; f < TileSmem<MODE>::KP; f += 4) {
    const double bv = (f < K) ? x[3 + S + f] : 0.0;
    sm.bm[f * PF_TS + j] = bv * sm.csm[f];
    sm.ba[f * PF_TS + j] = bv * sm.csa[f];
  }
}

// Row pass of one evaluation (all waves): per 16-row chunk, Xb on MFMA,
// elementwise residual / likelihood terms in the C layout, the beta
// gradient on MFMA, segment sums of G and G t.  Accumulates into LDS
// (gb, sg0/sg1, rr), which the caller zeroed.
// one chunk's global inputs (loaded a chunk ahead: with one wave per SIMD
// nothing else hides the L2 / HBM latency)
struct TileIn {
  double xa[8];      // Xb A operand, k-step kk: X[row r0 + (lane & 15)][4kk + (lane >> 4)]
  double xg[2][4];   // X'W A operand: X[row r0 + (lane >> 4) + 4q][16 ft + (lane & 15)]
  double t[4], y[4]; // C-layout rows r0 + (lane >> 4) + 4 rg
  int sg[4];
  int sfirst, slast;
};

template <int MODE>
__device__ __forceinline__ void tile_rows(const FitKArgs &a, TileSmem<MODE> &sm, int tile, int n) {
  constexpr int NSET = TileSmem<MODE>::NSET;
  const int lane = pf_lane(), wave = pf_wave();
  const int T = a.T, Tp = a.Tp, K = a.K;
  const int j = lane & 15, rq = lane >> 4;
  const bool linear = a.growth == PF_GROWTH_LINEAR;
  const int s_g = tile * PF_TS + j;
  const bool svalid = s_g < n;
  const double *ys = a.y_scaled + (size_t)(svalid ? s_g : 0) * Tp;
  const double *XT = a.XT;
  // B operands of Xb: k-step kk covers features 4kk..4kk+3 (lane: k = rq)
  double bmr[8], bar_[8];
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    bmr[kk] = ((MODE & 3) != MODE_ADD) ? sm.bm[(4 * kk + rq) * PF_TS + j] : 0.0;
    bar_[kk] = ((MODE & 3) != MODE_MULT) ? sm.ba[(4 * kk + rq) * PF_TS + j] : 0.0;
  }
  const int nkk = (K + 3) >> 2;
  auto tload = [&](int c, TileIn &in) {
    const int r0 = 16 * c;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int f = 4 * kk + rq;
      in.xa[kk] = (kk < nkk && f < K) ? XT[(size_t)f * Tp + r0 + j] : 0.0;
    }
#pragma unroll
    for (int ft = 0; ft < 2; ++ft) {
      const int f = 16 * ft + j;
#pragma unroll
      for (int q = 0; q < 4; ++q) in.xg[ft][q] = (f < K) ? XT[(size_t)f * Tp + r0 + rq + 4 * q] : 0.0;
    }
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      const int row = r0 + rq + 4 * rg;
      in.t[rg] = a.t[row];
      in.sg[rg] = a.seg[row];
      in.y[rg] = (svalid && row < T) ? ys[row] : 0.0;
    }
    in.sfirst = a.seg[r0];
    in.slast = a.seg[min(r0 + 15, T - 1)];
  };
  pf_d4 gbm[2], gba[2];
#pragma unroll
  for (int ft = 0; ft < 2; ++ft) { gbm[ft] = pf_d4{0.0, 0.0, 0.0, 0.0}; gba[ft] = pf_d4{0.0, 0.0, 0.0, 0.0}; }
  double rr = 0.0, a0 = 0.0, a1 = 0.0;
  int cur = -1;
  const int nch = (T + 15) >> 4;
  const int c0 = (nch * wave) / PF_TNW, c1 = (nch * (wave + 1)) / PF_TNW;
  TileIn nx;
  if (c0 < c1) tload(c0, nx);
  for (int c = c0; c < c1; ++c) {
    const TileIn cu = nx;
    if (c + 1 < c1) tload(c + 1, nx);
    const int r0 = 16 * c;
    // Xb = X[16 rows x K] . B[K x 16]
    pf_d4 xbm = pf_d4{0.0, 0.0, 0.0, 0.0}, xba = pf_d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      if (kk < nkk) {
        if constexpr ((MODE & 3) != MODE_ADD) xbm = __builtin_amdgcn_mfma_f64_16x16x4f64(cu.xa[kk], bmr[kk], xbm, 0, 0, 0);
        if constexpr ((MODE & 3) != MODE_MULT) xba = __builtin_amdgcn_mfma_f64_16x16x4f64(cu.xa[kk], bar_[kk], xba, 0, 0, 0);
      }
    }
    // elementwise on the C layout: element rg is (row r0 + rq + 4 rg, series j)
    double W[4], Wa[4], G[4], Gt[4];
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      const int row = r0 + rq + 4 * rg;
      const bool v = svalid && row < T;
      const double ti = cu.t[rg];
      const int sg = cu.sg[rg];
      const double tr = linear ? fma(sm.kseg[j * 32 + sg], ti, sm.mseg[j * 32 + sg]) : sm.mseg[j * 32];
      const double u = 1.0 + (((MODE & 3) != MODE_ADD) ? xbm[rg] : 0.0);
      const double mu = fma(tr, u, ((MODE & 3) != MODE_MULT) ? xba[rg] : 0.0);
      const double r = v ? cu.y[rg] - mu : 0.0;
      rr = fma(r, r, rr);
      W[rg] = r * tr;
      Wa[rg] = r;
      G[rg] = r * u;
      Gt[rg] = G[rg] * ti;
    }
    // beta gradient X'[K x 16 rows] . W[16 rows x 16]: k-step q is register q
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int ft = 0; ft < 2; ++ft) {
        if constexpr ((MODE & 3) != MODE_ADD) gbm[ft] = __builtin_amdgcn_mfma_f64_16x16x4f64(cu.xg[ft][q], W[q], gbm[ft], 0, 0, 0);
        if constexpr ((MODE & 3) != MODE_MULT) gba[ft] = __builtin_amdgcn_mfma_f64_16x16x4f64(cu.xg[ft][q], Wa[q], gba[ft], 0, 0, 0);
      }
    }
    // changepoint adjoint: segment sums of G, G t per series
    if (cu.sfirst == cu.slast) {
      const double g0 = (G[0] + G[1]) + (G[2] + G[3]), g1 = (Gt[0] + Gt[1]) + (Gt[2] + Gt[3]);
      if (cu.sfirst != cur) {
        if (cur >= 0) {
          double b0 = a0 + shfl_xor_f64<16>(a0), b1 = a1 + shfl_xor_f64<16>(a1);
          b0 += shfl_xor_f64<32>(b0);
          b1 += shfl_xor_f64<32>(b1);
          if (rq == 0) {
            atomicAdd(&sm.sg0[cur * PF_TS + j], b0);
            atomicAdd(&sm.sg1[cur * PF_TS + j], b1);
          }
        }
        cur = cu.sfirst;
        a0 = 0.0;
        a1 = 0.0;
      }
      a0 += g0;
      a1 += g1;
    } else {
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const int row = r0 + rq + 4 * rg;
        if (row < T) {
          atomicAdd(&sm.sg0[cu.sg[rg] * PF_TS + j], G[rg]);
          atomicAdd(&sm.sg1[cu.sg[rg] * PF_TS + j], Gt[rg]);
        }
      }
    }
  }
  if (cur >= 0) {
    double b0 = a0 + shfl_xor_f64<16>(a0), b1 = a1 + shfl_xor_f64<16>(a1);
    b0 += shfl_xor_f64<32>(b0);
    b1 += shfl_xor_f64<32>(b1);
    if (rq == 0) {
      atomicAdd(&sm.sg0[cur * PF_TS + j], b0);
      atomicAdd(&sm.sg1[cur * PF_TS + j], b1);
    }
  }
  rr += shfl_xor_f64<16>(rr);
  rr += shfl_xor_f64<32>(rr);
  if (rq == 0) atomicAdd(&sm.rr[j], rr);
  // gradient tiles: C[feature 16 ft + rq + 4 rg][series j]
#pragma unroll
  for (int ft = 0; ft < 2; ++ft)
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      const int f = 16 * ft + rq + 4 * rg;
      if constexpr ((MODE & 3) != MODE_ADD) atomicAdd(&sm.gb[f * PF_TS + j], gbm[ft][rg]);
      if constexpr ((MODE & 3) != MODE_MULT)
        atomicAdd(&sm.gb[(NSET - 1) * TileSmem<MODE>::KP * PF_TS + f * PF_TS + j], gba[ft][rg]);
    }
}

// wave 0, lane quad of series j: f and g at xq (this lane's parameters
// p = q + 4i -> gq), gpq = g . pk.  Returns true if not finite.
template <int MODE>
__device__ __forceinline__ bool tile_assemble(const FitKArgs &a, TileSmem<MODE> &sm, int j, int q,
                                              double &f, double &gpq) {
  constexpr int NSET = TileSmem<MODE>::NSET;
  const int S = a.S, K = a.K, P = a.P, T = a.T, V = sm.V;
  const bool linear = a.growth == PF_GROWTH_LINEAR;
  const double *x = sm.xq + (size_t)j * V;
  double *g = sm.gq + (size_t)j * V;
  const double *pk = sm.pk + (size_t)j * V;
  const double sigma = sm.sig[2 * j], inv = sm.sig[2 * j + 1], tau = a.tau;
  const double rrt = sm.rr[j];
  // totals and suffix sums over segments (redundant in the quad's lanes)
  double tot0 = 0.0, tot1 = 0.0;
  for (int s = 0; s <= S; ++s) { tot0 += sm.sg0[s * PF_TS + j]; tot1 += sm.sg1[s * PF_TS + j]; }
  double fl = 0.0, gp = 0.0;
  bool bad = false;
  // delta_jj: sum over segments s > jj of (G t - tc_jj G)
  {
    double su0 = 0.0, su1 = 0.0;
    for (int s = S; s >= 1; --s) {
      su0 += sm.sg0[s * PF_TS + j];
      su1 += sm.sg1[s * PF_TS + j];
      const int p = 2 + (s - 1);
      if ((p & 3) == q) {
        const double d = x[p];
        const double sgn = (d > 0.0) - (d < 0.0);
        const double gv = (linear ? -inv * (su1 - sm.ctc[s - 1] * su0) : 0.0) + sgn / tau;
        g[p] = gv;
        fl += fabs(d) / tau;
        gp = fma(gv, pk[p], gp);
        bad |= !isfinite(gv);
      }
    }
  }
  for (int p = q; p < P; p += 4) {
    if (p >= 2 && p < 2 + S) continue;
    double gv, ft;
    const double xv = x[p];
    if (p == 0) {
      gv = -inv * (linear ? tot1 : 0.0) + xv / 25.0;
      ft = xv * xv / 50.0;
    } else if (p == 1) {
      gv = -inv * tot0 + xv / 25.0;
      ft = xv * xv / 50.0;
    } else if (p == 2 + S) {
      gv = (double)T - inv * rrt + 4.0 * sigma * sigma;
      ft = 2.0 * sigma * sigma + (double)T * xv;
    } else {
      const int f2 = p - 3 - S;
      const double sgm = sm.csg[f2];
      double gl = 0.0;
      if constexpr ((MODE & 3) != MODE_ADD) gl += sm.csm[f2] * sm.gb[f2 * PF_TS + j];
      if constexpr ((MODE & 3) != MODE_MULT)
        gl += sm.csa[f2] * sm.gb[(NSET - 1) * TileSmem<MODE>::KP * PF_TS + f2 * PF_TS + j];
      gv = -inv * gl + xv / (sgm * sgm);
      ft = xv * xv / (2.0 * sgm * sgm);
    }
    g[p] = gv;
    fl += ft;
    gp = fma(gv, pk[p], gp);
    bad |= !isfinite(gv);
  }
  f = quad_sum(fl) + 0.5 * rrt * inv;
  gpq = quad_sum(gp);
  bad |= !isfinite(f);
  // quad-uniform
  const int b = bad ? 1 : 0;
  return (b | __shfl_xor(b, 1, 64) | __shfl_xor(b, 2, 64)) != 0;
}

#define PF_TNP 15  // parameters per lane (p = q + 4i, P <= 60)
typedef double TVec[PF_TNP];

__device__ __forceinline__ double tvdot(const TVec &u, const TVec &v) {
  double s0 = 0.0, s1 = 0.0;
#pragma unroll
  for (int i = 0; i < PF_TNP; i += 2) {
    s0 = fma(u[i], v[i], s0);
    if (i + 1 < PF_TNP) s1 = fma(u[i + 1], v[i + 1], s1);
  }
  return quad_sum(s0 + s1);
}
// LDS vector (series stride V) <-> registers; entries past P read as 0
__device__ __forceinline__ void tvload(TVec &r, const double *v, int P, int q) {
#pragma unroll
  for (int i = 0; i < PF_TNP; ++i) {
    const int p = q + 4 * i;
    r[i] = (p < P) ? v[p] : 0.0;
  }
}
__device__ __forceinline__ void tvstore(double *v, const TVec &r, int P, int q) {
#pragma unroll
  for (int i = 0; i < PF_TNP; ++i) {
    const int p = q + 4 * i;
    if (p < P) v[p] = r[i];
  }
}

// Stan 2.19 BFGSMinimizer<LBFGSUpdate>::step + WolfeLineSearch as a per-series
// state machine (lane quad): advance until the series needs an evaluation
// at xq (returns true) or terminates (false, z.ret set).  Same control flow
// as lbfgs_step (pf_engine.hip) and oracle/stan_lbfgs.c; the search direction
// by Stan's two-loop recursion.  The working vectors live in registers for
// the step (one batched LDS read per history vector).
template <int MODE>
__device__ __forceinline__ bool tile_lbfgs(const pf_fit_opts &o, TileSmem<MODE> &sm, TileZ &z, int j,
                                           int q, int P) {
  const int V = sm.V;
  double *xkL = sm.xk + (size_t)j * V, *gkL = sm.gk + (size_t)j * V, *pkL = sm.pk + (size_t)j * V;
  double *xqL = sm.xq + (size_t)j * V;
  const int H = o.history < PF_TH ? o.history : PF_TH;
  const size_t hstep = (size_t)PF_TS * V;
  TVec xk, gk, pk, xq, gq;
  tvload(xk, xkL, P, q);
  tvload(gk, gkL, P, q);
  tvload(pk, pkL, P, q);
  tvload(xq, xqL, P, q);
  tvload(gq, sm.gq + (size_t)j * V, P, q);
  bool need = false;
  bool run = true;
  while (run) {
    switch (z.state) {
      case LB_INIT:
        if (z.bad) { z.ret = PF_ST_BADINIT; z.state = LB_DONE; run = false; break; }
        z.fk = z.fq;
#pragma unroll
        for (int i = 0; i < PF_TNP; ++i) { xk[i] = xq[i]; gk[i] = gq[i]; pk[i] = -gq[i]; }
        z.itNum = 0;
        z.hcount = 0;
        z.head = 0;
        z.state = LB_NEW_ITER;
        break;
      case LB_NEW_ITER:
        z.itNum++;
        z.resetB = (z.itNum == 1) ? 1 : 0;
        z.state = LB_LS_START;
        break;
      case LB_LS_START:
        if (z.itNum > 1 && z.resetB != 2) {
          z.alpha = fmin(1.0, 1.01 * cubic_interp0(z.dfp_prev, z.alphak_1, z.fk - z.fk1, z.lastDFp,
                                                   1e-12, 1.0));
        } else {
          z.alpha = o.init_alpha;
        }
        if (z.resetB) {
#pragma unroll
          for (int i = 0; i < PF_TNP; ++i) pk[i] = -gk[i];
        }
        z.dfp = tvdot(gk, pk);
        z.c1dfp = 1e-4 * z.dfp;
        z.c2dfp = 0.9 * z.dfp;
        z.alpha0 = 1e-12;
        z.alpha1 = z.alpha;
        z.prevF = z.fk;
        z.prevDFp = z.dfp;
        z.nits = 0;
        z.lsRestarts = 0;
        z.state = LB_TRY;
        break;
      case LB_TRY:
        if (z.nits >= 20) { z.state = LB_LS_FAIL; break; }
#pragma unroll
        for (int i = 0; i < PF_TNP; ++i) xq[i] = xk[i] + z.alpha1 * pk[i];
        z.state = LB_TRY_RES;
        need = true;
        run = false;
        break;
      case LB_TRY_RES: {
        if (z.bad) {
          if (z.lsRestarts >= 10) { z.state = LB_LS_FAIL; break; }
          z.alpha1 = 0.5 * (z.alpha0 + z.alpha1);
          z.lsRestarts++;
          z.state = LB_TRY;
          break;
        }
        z.lsRestarts = 0;
        const double f1 = z.fq, newDFp = z.gpq;
        if ((f1 > z.fk + z.alpha1 * z.c1dfp) || (f1 >= z.prevF && z.nits > 0)) {
          z.alo = z.alpha0; z.aloF = z.prevF; z.aloDFp = z.prevDFp;
          z.ahi = z.alpha1; z.ahiF = f1; z.ahiDFp = newDFp;
          z.zit = 0;
          z.state = LB_ZOOM_ITER;
        } else if (fabs(newDFp) <= -z.c2dfp) {
          z.alpha = z.alpha1;
          z.lastDFp = newDFp;
          z.state = LB_LS_OK;
        } else if (newDFp >= 0) {
          z.alo = z.alpha1; z.aloF = f1; z.aloDFp = newDFp;
          z.ahi = z.alpha0; z.ahiF = z.prevF; z.ahiDFp = z.prevDFp;
          z.zit = 0;
          z.state = LB_ZOOM_ITER;
        } else {
          z.alpha0 = z.alpha1;
          z.prevF = f1;
          z.prevDFp = newDFp;
          z.alpha1 *= 10.0;
          z.nits++;
          z.state = LB_TRY;
        }
        break;
      }
      case LB_ZOOM_ITER: {
        z.zit++;
        if (fabs(z.alo - z.ahi) < 1e-16) { z.state = LB_LS_FAIL; break; }
        if (z.zit % 5 == 0) {
          z.alpha = 0.5 * (z.alo + z.ahi);
        } else {
          const double lo = fmin(z.alo, z.ahi), hi = fmax(z.alo, z.ahi);
          z.alpha = cubic_interp(z.alo, z.aloF, z.aloDFp, z.ahi, z.ahiF, z.ahiDFp, lo, hi);
          if (z.alpha < lo + 0.01 * (hi - lo) || z.alpha > hi - 0.01 * (hi - lo))
            z.alpha = 0.5 * (z.alo + z.ahi);
        }
#pragma unroll
        for (int i = 0; i < PF_TNP; ++i) xq[i] = xk[i] + z.alpha * pk[i];
        z.state = LB_ZOOM_RES;
        need = true;
        run = false;
        break;
      }
      case LB_ZOOM_RES: {
        if (z.bad) {
          const double lo = fmin(z.alo, z.ahi);
          z.alpha = 0.5 * (z.alpha + lo);
          if (fabs(lo - z.alpha) < 1e-16) { z.state = LB_LS_FAIL; break; }
#pragma unroll
          for (int i = 0; i < PF_TNP; ++i) xq[i] = xk[i] + z.alpha * pk[i];
          need = true;   // stay in LB_ZOOM_RES
          run = false;
          break;
        }
        const double f1 = z.fq, newDFp = z.gpq;
        if (f1 > (z.fk + z.alpha * z.c1dfp) || f1 >= z.aloF) {
          z.ahi = z.alpha; z.ahiF = f1; z.ahiDFp = newDFp;
          z.state = LB_ZOOM_ITER;
        } else {
          if (fabs(newDFp) <= -z.c2dfp) { z.lastDFp = newDFp; z.state = LB_LS_OK; break; }
          if (newDFp * (z.ahi - z.alo) >= 0) { z.ahi = z.alo; z.ahiF = z.aloF; z.ahiDFp = z.aloDFp; }
          z.alo = z.alpha; z.aloF = f1; z.aloDFp = newDFp;
          z.state = LB_ZOOM_ITER;
        }
        break;
      }
      case LB_LS_FAIL:
        if (z.resetB) { z.ret = PF_ST_LSFAIL; z.state = LB_DONE; run = false; break; }
        z.resetB = 2;
        z.state = LB_LS_START;
        break;
      case LB_LS_OK: {
        // accepted point = last evaluated (xq, fq, gq); k becomes the newest
        z.fk1 = z.fk;
        z.fk = z.fq;
        z.alphak_1 = z.alpha;
        z.dfp_prev = z.dfp;
        if (z.resetB) { z.hcount = 0; z.head = 0; }
        const int slot = (z.hcount < H) ? pf_wrap(z.head + z.hcount, H) : z.head;
        TVec sk, yk;
#pragma unroll
        for (int i = 0; i < PF_TNP; ++i) {
          sk[i] = xq[i] - xk[i];
          yk[i] = gq[i] - gk[i];
          xk[i] = xq[i];
          gk[i] = gq[i];
        }
        const double gg = tvdot(gk, gk), ss = tvdot(sk, sk), sy = tvdot(sk, yk), yy = tvdot(yk, yk);
        if (fabs(z.fk1 - z.fk) < o.tol_obj) {
          z.ret = PF_ST_ABSF;
        } else if (sqrt(gg) < o.tol_grad) {
          z.ret = PF_ST_ABSGRAD;
        } else if (sqrt(ss) < o.tol_param) {
          z.ret = PF_ST_ABSX;
        } else if (z.itNum >= o.max_iter || (o.lbfgs_warmup_evals > 0 && z.n_eval >= o.lbfgs_warmup_evals)) {
          z.ret = PF_ST_MAXIT;
        } else if (((z.fk1 - z.fk) / fmax(fabs(z.fk1), fmax(fabs(z.fk), 1.0))) <
                   o.tol_rel_obj * 2.220446049250313e-16) {
          z.ret = PF_ST_RELF;
        } else {
          // LBFGSUpdate::update (store the pair) + search_direction (two loops)
          z.gammak = sy / yy;
          tvstore(sm.hs + slot * hstep + (size_t)j * V, sk, P, q);
          tvstore(sm.hy + slot * hstep + (size_t)j * V, yk, P, q);
          if (q == 0) sm.hrho[j * PF_TH + slot] = 1.0 / sy;
          if (z.hcount < H) z.hcount++;
          else z.head = pf_wrap(z.head + 1, H);
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
          for (int i = 0; i < PF_TNP; ++i) pk[i] = -gk[i];
          double al[PF_TH];
#pragma unroll
          for (int c = PF_TH - 1; c >= 0; --c) {
            al[c] = 0.0;
            if (c < z.hcount) {
              const int sl = pf_wrap(z.head + c, H);
              TVec sv, yv;
              if (c == z.hcount - 1) {    // newest pair: still in registers
#pragma unroll
                for (int i = 0; i < PF_TNP; ++i) { sv[i] = sk[i]; yv[i] = yk[i]; }
              } else {
                tvload(sv, sm.hs + sl * hstep + (size_t)j * V, P, q);
                tvload(yv, sm.hy + sl * hstep + (size_t)j * V, P, q);
              }
              al[c] = sm.hrho[j * PF_TH + sl] * tvdot(sv, pk);
#pragma unroll
              for (int i = 0; i < PF_TNP; ++i) pk[i] = fma(-al[c], yv[i], pk[i]);
            }
          }
#pragma unroll
          for (int i = 0; i < PF_TNP; ++i) pk[i] *= z.gammak;
#pragma unroll
          for (int c = 0; c < PF_TH; ++c) {
            if (c < z.hcount) {
              const int sl = pf_wrap(z.head + c, H);
              TVec sv, yv;
              tvload(sv, sm.hs + sl * hstep + (size_t)j * V, P, q);
              tvload(yv, sm.hy + sl * hstep + (size_t)j * V, P, q);
              const double b = sm.hrho[j * PF_TH + sl] * tvdot(yv, pk);
#pragma unroll
              for (int i = 0; i < PF_TNP; ++i) pk[i] = fma(al[c] - b, sv[i], pk[i]);
            }
          }
          const double gp = tvdot(pk, gk);
          if (-gp / fmax(fabs(z.fk), 1.0) < o.tol_rel_grad * 2.220446049250313e-16)
            z.ret = PF_ST_RELGRAD;
          else
            z.ret = PF_ST_SUCCESS;
        }
        if (z.ret != PF_ST_SUCCESS) { z.state = LB_DONE; run = false; break; }
        z.state = LB_NEW_ITER;
        break;
      }
      default:
        run = false;
        break;
    }
  }
  tvstore(xkL, xk, P, q);
  tvstore(gkL, gk, P, q);
  tvstore(pkL, pk, P, q);
  tvstore(xqL, xq, P, q);
  return need;
}

// K3T kernel: grid = ceil(n / 16) tiles.  Pass-0 semantics of fit_body
// (theta in: init; out: the L-BFGS endpoint, f, f_stan, status, n_iter,
// n_eval), warm = the iteration cap is the warm-up cap (MAXIT -> WARMUP).
template <int MODE>
__global__ __launch_bounds__(PF_TNW * 64, 1) void k_fit_tile(FitKArgs a, int n) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  TileSmem<MODE> sm;
  sm.carve(smem_raw, a.P);
  const int tile = blockIdx.x, lane = pf_lane(), wave = pf_wave();
  const int P = a.P, S = a.S, V = sm.V;
  const int j = lane >> 2, q = lane & 3;  // wave 0: lane quad of series j
  const int sgl = tile * PF_TS + j;
  const bool warm = a.warm_cap != 0;
  const pf_fit_opts o = a.o;
  // constants
  if (threadIdx.x < 64) {
    const int i = threadIdx.x;
    sm.ctc[i] = (i < S) ? a.t_change[i] : 0.0;
    sm.csg[i] = (i < a.K) ? a.sigmas[i] : 1.0;
    sm.csm[i] = (i < a.K) ? a.s_m[i] : 0.0;
    sm.csa[i] = (i < a.K) ? a.s_a[i] : 0.0;
  }
  __syncthreads();
  if (wave == 0) {
    TileZ &z = sm.z[j];
    const bool live = sgl < n && a.status[sgl] != PF_ST_CONSTANT;
    double *xq = sm.xq + (size_t)j * V, *xk = sm.xk + (size_t)j * V;
    for (int p = q; p < V; p += 4) {
      const double v = (sgl < n && p < P) ? a.theta[(size_t)sgl * P + p] : 0.0;
      xq[p] = v;
      xk[p] = v;
    }
    if (q == 0) {
      memset(&z, 0, sizeof(TileZ));
      z.state = LB_INIT;
      z.done = live ? 0 : 1;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    tile_publish<MODE>(a, sm, j, q);
  }
  for (int e = threadIdx.x; e < TileSmem<MODE>::NSET * TileSmem<MODE>::KP * PF_TS; e += PF_TNW * 64) sm.gb[e] = 0.0;
  for (int e = threadIdx.x; e < 32 * PF_TS; e += PF_TNW * 64) { sm.sg0[e] = 0.0; sm.sg1[e] = 0.0; }
  if (threadIdx.x < PF_TS) sm.rr[threadIdx.x] = 0.0;
  __syncthreads();
  while (true) {
    PF_STAMP(0);
    tile_rows<MODE>(a, sm, tile, n);
    PF_STAMP(1);
    __syncthreads();
    PF_STAMP(2);
    PF_COUNT(7);
    if (wave == 0) {
      TileZ &z = sm.z[j];
      double fq, gpq;
      const bool bad = tile_assemble<MODE>(a, sm, j, q, fq, gpq);
      PF_STAMP(3);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      bool need = false;
      if (!z.done) {
        TileZ zl = z;          // quad-local copy; lane q == 0 writes it back
        zl.fq = fq;
        zl.gpq = gpq;
        zl.bad = bad ? 1 : 0;
        zl.n_eval++;
        need = tile_lbfgs<MODE>(o, sm, zl, j, q, P);
        if (!need) zl.done = 1;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (q == 0) z = zl;
      }
      PF_STAMP(4);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (need) tile_publish<MODE>(a, sm, j, q);
      const unsigned long long any = __ballot(need);
      if (lane == 0) sm.flag[0] = any != 0ull ? 1 : 0;
      // zero the accumulators for the next evaluation (wave 0 has read them)
      for (int e = lane; e < TileSmem<MODE>::NSET * TileSmem<MODE>::KP * PF_TS; e += 64) sm.gb[e] = 0.0;
      for (int e = lane; e < 32 * PF_TS; e += 64) { sm.sg0[e] = 0.0; sm.sg1[e] = 0.0; }
      if (lane < PF_TS) sm.rr[lane] = 0.0;
      PF_STAMP(5);
    }
    __syncthreads();
    PF_STAMP(6);
    if (!__builtin_amdgcn_readfirstlane(sm.flag[0])) break;
  }
  // outputs (pass-0 semantics of fit_body)
  if (wave == 0 && sgl < n) {
    TileZ &z = sm.z[j];
    double *th = a.theta + (size_t)sgl * P;
    const int st_in = a.status[sgl];
    if (st_in == PF_ST_CONSTANT) {
      if (q == 0) {
        th[2 + S] = log(1e-9);
        a.f_out[sgl] = NAN;
        a.f_stan[sgl] = NAN;
        a.n_iter[sgl] = 0;
        a.n_eval[sgl] = 0;
      }
    } else {
      const double *xk = sm.xk + (size_t)j * V;
      for (int p = q; p < P; p += 4) th[p] = xk[p];
      if (q == 0) {
        int st = z.ret;
        if (warm && st == PF_ST_MAXIT) st = PF_ST_WARMUP;
        a.f_out[sgl] = z.fk;
        a.f_stan[sgl] = z.fk;
        a.n_iter[sgl] = z.itNum;
        a.n_eval[sgl] = z.n_eval;
        a.status[sgl] = st;
      }
    }
  }
}
