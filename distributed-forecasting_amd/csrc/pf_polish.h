// pf_polish.h — exact-MAP polish after the Stan-faithful L-BFGS phase.
//
// Engine extension (NOT part of Stan): Stan's smooth L-BFGS stalls at the L1
// kink of delta ~ double_exponential(0, tau) up to ~3e-5 relative short of the
// MAP (linear growth; up to 2e-4 for logistic growth).  From where it stops we
// run proximal Newton on f = h + c*||delta||_1 (c = 1/tau):
//   1. exact Hessian of the smooth part h.  Its data term sum_i (dmu dmu' -
//      r d2mu)/sigma^2 is a genuine GEMM over the T rows: per row one column
//      vector per parameter block [trend: 32 | beta: 16*NBB], NT 16x16 output
//      tiles accumulated on FP64 MFMA (v_mfma_f64_16x16x4f64).  Per-row
//      quantities (u, trend, residual) are recomputed inside the MFMA loop by
//      the 16 lanes of each row (nothing goes to HBM).  Logistic growth adds
//      the curvature of the sigmoid per row and of UPSTREAM logistic_gamma per
//      segment (oracle/stan_lbfgs.c orc_hessian states the formulas);
//   2. the lasso-QP subproblem min gh.d + d'Hd/2 + c||x_delta + d_delta||_1,
//      solved exactly by an active-set method on the swept matrix (LDS, wave 0);
//      a non-positive pivot (non-convex region) damps the model to
//      H + lam*max|diag H|*I, lam x10 per retry, /10 after each accepted step;
//   3. Armijo backtracking on the true objective (collective evaluations);
//   4. after a full undamped step the next QP reuses the swept matrix (lagged
//      Hessian, see polish_run).
// Same algorithm as oracle/stan_lbfgs.c:orc_polish_ex (the CPU check).
// Linear, flat and logistic growth; 2 + S <= 32; K <= 16*NBB (NBB <= 3, so
// K <= 48: P up to 3 + 30 + 48); P > 64 uses two parameter words per lane.
#pragma once

typedef double pf_d4 __attribute__((ext_vector_type(4)));

// tile q of the upper block triangle over NB column blocks -> (bi, bj), bi <= bj
__host__ __device__ constexpr int ptile_bi(int q, int NB) {
  int bi = 0;
  while (q >= NB - bi) { q -= NB - bi; ++bi; }
  return bi;
}
__host__ __device__ constexpr int ptile_bj(int q, int NB) {
  int bi = 0;
  while (q >= NB - bi) { q -= NB - bi; ++bi; }
  return bi + q;
}

// column of the J space [trend 0..31 | beta 32..] -> parameter index (or -1)
__device__ __forceinline__ int pcolmap(int c, int S, int K) {
  if (c < 32) return (c < 2 + S) ? c : -1;
  const int f = c - 32;
  return (f < K) ? 3 + S + f : -1;
}

// E_s[c] = d k_s / d theta_c: k, and delta_j for j < s
__device__ __forceinline__ double pf_Ecol(int c, int s) {
  return (c == 0 || (c >= 2 && c - 2 < s)) ? 1.0 : 0.0;
}

// One k-step's MFMAs, tile Q..NT-1 (template recursion: every tile's block
// pair is a compile-time constant, so the operand arrays stay in registers —
// a runtime index would put them in scratch).
template <int Q, int NB, int NT, int NBB>
__device__ __forceinline__ void mfma_tiles(pf_d4 (&acc)[NT], const double (&lt)[2], const double (&rt)[2],
                                           const double (&gt)[2], const double (&V)[NBB],
                                           const double (&W)[NBB]) {
  if constexpr (Q < NT) {
    constexpr int bi = ptile_bi(Q, NB), bj = ptile_bj(Q, NB);
    double A_, B_;
    if constexpr (bj < 2) { A_ = lt[bi]; B_ = rt[bj]; }
    else if constexpr (bi < 2) { A_ = gt[bi]; B_ = W[bj - 2]; }
    else { A_ = V[bi - 2]; B_ = V[bj - 2]; }
    acc[Q] = __builtin_amdgcn_mfma_f64_16x16x4f64(A_, B_, acc[Q], 0, 0, 0);
    mfma_tiles<Q + 1, NB, NT, NBB>(acc, lt, rt, gt, V, W);
  }
}

// Hessian of the smooth part at x, assembled into A = sm.U (stride LD, P
// rows + 8 zero padding rows), damped by lam * max|diag| when lam > 0.
// gh: smooth gradient at x (this lane's words).  Every thread calls it.
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__device__ __forceinline__ void hessian_collective(const FitKArgs &a, FitSmem<NW, KMAX, MODE> &sm,
                                                   const PV<ModeTr<MODE>::PW> &x,
                                                   const PV<ModeTr<MODE>::PW> &gh, double lam,
                                                   bool stash = false) {
  constexpr int PW = ModeTr<MODE>::PW;
  constexpr int NBB = FitSmem<NW, KMAX, MODE>::NBB;
  constexpr int NB = 2 + NBB;
  constexpr int NT = NB * (NB + 1) / 2;
  constexpr bool logistic = (MODE & PF_MODE_LOGI) != 0;
  const int lane = pf_lane(), wave = pf_wave();
  const int S = __builtin_amdgcn_readfirstlane(a.S), K = __builtin_amdgcn_readfirstlane(a.K);
  const int T = __builtin_amdgcn_readfirstlane(a.T), Tp = __builtin_amdgcn_readfirstlane(a.Tp);
  const int P = __builtin_amdgcn_readfirstlane(a.P);
  const int R = __builtin_amdgcn_readfirstlane(a.R);
  const int nt = 2 + S;
  const int growth = a.growth;
  double *Mt = sm.pmt;    // [32][32] d m_s / d theta_c (logistic)
  double *rho = sm.prho;  // [32]     sum_{i in s} r u cap s'
  publish_theta<NW, KMAX, MODE>(a, sm, x);
  // logistic: per row-group partial segment sums rho in U ([16][32]; U is
  // free while the Hessian is rebuilt: the previous swept matrix is dead).
  // Each row group (wave, rq) visits every segment in one run and writes its
  // sum once; the totals are added in a fixed order below (bitwise
  // reproducible, no atomics)
  double *rslot = sm.U;
  if constexpr (logistic) {
    static_assert(NW <= 4, "rho slots: 4 row groups per wave, 16 slots");
    for (int e = threadIdx.x; e < 16 * 32; e += NW * 64) rslot[e] = 0.0;
  }
  if constexpr (logistic) {
    if (wave == 0) {
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      // M_{s+1} = q_s M_s + (m_s - tc_s) dq_s, q_s = k_s / k_{s+1}
      // (UPSTREAM logistic_gamma differentiated; lane = parameter column)
      if (lane < 32) {
        const int c = lane;
        double Mc = (c == 1) ? 1.0 : 0.0;
        Mt[c] = Mc;
        for (int s = 0; s < S; ++s) {
          const double ks = sm.kseg[s], ks1 = sm.kseg[s + 1];
          const double q = ks / ks1;
          const double dq = pf_Ecol(c, s) / ks1 - ks * pf_Ecol(c, s + 1) / (ks1 * ks1);
          Mc = q * Mc + (sm.mseg[s] - sm.ctc[s]) * dq;
          Mt[(s + 1) * 32 + c] = Mc;
        }
        rho[c] = 0.0;
      }
    }
  }
  __syncthreads();
  // ---- MFMA pass: k-steps of 4 rows (row = lane >> 4), column = lane & 15
  pf_d4 acc[NT];
#pragma unroll
  for (int q = 0; q < NT; ++q) acc[q] = pf_d4{0.0, 0.0, 0.0, 0.0};
  const int c16 = lane & 15, rq = lane >> 4;
  const int cA = c16, cB = 16 + c16;  // this lane's trend columns (blocks 0, 1)
  double bmv[NBB], bav[NBB], smv[NBB], sav[NBB];
#pragma unroll
  for (int b = 0; b < NBB; ++b) {
    const int f = 16 * b + c16;
    const bool ok = f < K;
    bmv[b] = ok ? sm.bm[f < KMAX ? f : 0] : 0.0;
    bav[b] = ok ? sm.ba[f < KMAX ? f : 0] : 0.0;
    smv[b] = ok ? sm.csm[f] : 0.0;
    sav[b] = ok ? sm.csa[f] : 0.0;
  }
  const double tcA = (cA >= 2 && cA - 2 < S) ? sm.ctc[cA - 2] : 0.0;
  const double tcB = (cB - 2 < S) ? sm.ctc[cB - 2] : 0.0;
  const double th_m = sm.th[1];
  const double *capr = logistic ? a.cap_scaled + (size_t)blockIdx.x * Tp : nullptr;
  constexpr int NL = NW * 64;
  const int nks = (T + 3) >> 2;
  struct HIn { double t, y, cap, X[NBB]; int sg; };
  auto hload = [&](int s_, HIn &h) {
    const int row = 4 * s_ + rq;
    const bool v = row < T;
    const int rr = v ? row : 0;
    h.t = a.t[rr];
    h.sg = a.seg[rr];
    // lane-blocked y: natural row L*R + r sits at r*NL + L
    const int Lr = rr / R;
    h.y = v ? sm.y[(rr - Lr * R) * NL + Lr] : 0.0;
    h.cap = logistic ? capr[rr] : 0.0;
#pragma unroll
    for (int b = 0; b < NBB; ++b) {
      const int f = 16 * b + c16;
      h.X[b] = (v && f < K) ? a.XT[(size_t)f * Tp + rr] : 0.0;
    }
  };
  double Q = 0.0;
  int cur_seg = 0;
  double rho_acc = 0.0;
  HIn nx;
  if (wave < nks) hload(wave, nx);
  for (int s = wave; s < nks; s += NW) {
    const HIn cu = nx;
    if (s + NW < nks) hload(s + NW, nx);
    const int row = 4 * s + rq;
    const bool valid = row < T;
    // u = 1 + X(beta s_m), additive part: partial over this lane's columns,
    // reduced over the 16 lanes of the row
    double pm = 0.0, pa = 0.0;
#pragma unroll
    for (int b = 0; b < NBB; ++b) {
      if constexpr ((MODE & 3) != MODE_ADD) pm = fma(cu.X[b], bmv[b], pm);
      if constexpr ((MODE & 3) != MODE_MULT) pa = fma(cu.X[b], bav[b], pa);
    }
    if constexpr ((MODE & 3) != MODE_ADD) {
      pm += shfl_xor_f64<1>(pm);
      pm += shfl_xor_f64<2>(pm);
      pm += shfl_xor_f64<4>(pm);
      pm += shfl_xor_f64<8>(pm);
    }
    if constexpr ((MODE & 3) != MODE_MULT) {
      pa += shfl_xor_f64<1>(pa);
      pa += shfl_xor_f64<2>(pa);
      pa += shfl_xor_f64<4>(pa);
      pa += shfl_xor_f64<8>(pa);
    }
    const double u = 1.0 + pm;
    const double ti = cu.t;
    const int sg = cu.sg;
    double tr, dzA, dzB, wt, gf = 1.0, sp = 0.0, sgm = 0.0;
    if constexpr (logistic) {
      const double ks = sm.kseg[sg], ms = sm.mseg[sg];
      sgm = 1.0 / (1.0 + exp(-(ks * (ti - ms))));
      sp = sgm * (1.0 - sgm);
      tr = cu.cap * sgm;
      dzA = (cA < nt) ? (ti - ms) * pf_Ecol(cA, sg) - ks * Mt[sg * 32 + cA] : 0.0;
      dzB = (cB < nt) ? (ti - ms) * pf_Ecol(cB, sg) - ks * Mt[sg * 32 + cB] : 0.0;
      gf = cu.cap * sp;
    } else if (growth == PF_GROWTH_LINEAR) {
      tr = fma(sm.kseg[sg], ti, sm.mseg[sg]);
      dzA = (cA == 0) ? ti : (cA == 1) ? 1.0 : ((cA - 2 < S && sg > cA - 2) ? ti - tcA : 0.0);
      dzB = (cB - 2 < S && sg > cB - 2) ? ti - tcB : 0.0;
    } else {  // flat: trend = m
      tr = th_m;
      dzA = (cA == 1) ? 1.0 : 0.0;
      dzB = 0.0;
    }
    const double r = valid ? (cu.y - fma(tr, u, pa)) : 0.0;
    if constexpr (logistic) {
      const double aa = u * cu.cap * sp;
      wt = aa * aa - r * u * cu.cap * sp * (1.0 - 2.0 * sgm);
      // rho_s: one lane per row, flushed to LDS when the (monotone) segment changes
      if (c16 == 0 && valid) {
        if (sg != cur_seg) {
          rslot[(wave * 4 + rq) * 32 + cur_seg] = rho_acc;
          rho_acc = 0.0;
          cur_seg = sg;
        }
        rho_acc = fma(r, u * cu.cap * sp, rho_acc);
      }
    } else {
      wt = u * u;
    }
    if (!valid) { dzA = 0.0; dzB = 0.0; wt = 0.0; gf = 0.0; }
    if (c16 == 0) Q = fma(r, r, Q);
    double V[NBB], W[NBB];
#pragma unroll
    for (int b = 0; b < NBB; ++b) {
      const double kf = fma(tr, smv[b], sav[b]);
      V[b] = cu.X[b] * kf;
      W[b] = cu.X[b] * fma(u, kf, -r * smv[b]);
    }
    const double lt[2] = {wt * dzA, wt * dzB}, rt[2] = {dzA, dzB}, gt[2] = {gf * dzA, gf * dzB};
    mfma_tiles<0, NB, NT, NBB>(acc, lt, rt, gt, V, W);
  }
  if constexpr (logistic) {
    if (c16 == 0) rslot[(wave * 4 + rq) * 32 + cur_seg] = rho_acc;
    __syncthreads();
    if (threadIdx.x < 32) {
      double tot = 0.0;
#pragma unroll
      for (int g2 = 0; g2 < 16; ++g2) tot += rslot[g2 * 32 + threadIdx.x];
      rho[threadIdx.x] = tot;
    }
    __syncthreads();  // U becomes the tile-reduction buffer below
  }
  // ---- chained reduction of the tiles over waves through one LDS buffer
  Q = wave_sum(Q);
  if (lane == 0) sm.rrw[wave] = Q;
  double *red = sm.U;  // [NT][4][64]
  for (int w2 = NW - 1; w2 >= 1; --w2) {
    if (wave == w2) {
#pragma unroll
      for (int q = 0; q < NT; ++q)
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) red[((size_t)q * 4 + rg) * 64 + lane] = acc[q][rg];
    }
    __syncthreads();
    if (wave == w2 - 1) {
#pragma unroll
      for (int q = 0; q < NT; ++q)
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) acc[q][rg] += red[((size_t)q * 4 + rg) * 64 + lane];
    }
    __syncthreads();
  }
  // ---- wave 0 assembles A (LDS, stride LD): data term / sigma^2, logistic
  //      segment terms, priors, the l row, damping
  if (wave == 0) {
    double *A = sm.U;
    const int LD = sm.LD;
    for (int e = lane; e < (P + 8) * LD; e += 64) A[e] = 0.0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    Q = 0.0;
    for (int w2 = 0; w2 < NW; ++w2) Q += sm.rrw[w2];
    const int il = 2 + S;
    const double ls = (il < 64) ? readlane_f64(x[0], il) : 0.0;
    const double sig2 = exp(2.0 * ls);
    const double inv = 1.0 / sig2;
#pragma unroll
    for (int q = 0; q < NT; ++q) {
      const int bi = ptile_bi(q, NB), bj = ptile_bj(q, NB);
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const int ci = bi * 16 + (lane >> 4) + 4 * rg;
        const int cj = bj * 16 + (lane & 15);
        const int pi = pcolmap(ci, S, K), pj = pcolmap(cj, S, K);
        // diagonal-block tiles hold (i, j) and (j, i) with different product
        // rounding: take the upper entry for both, so A is exactly symmetric
        if (pi >= 0 && pj >= 0 && (bi != bj || ci <= cj)) {
          const double v = acc[q][rg] * inv;
          A[pi * LD + pj] = v;
          A[pj * LD + pi] = v;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if constexpr (logistic) {
      // sum_s rho_s (E_s M_s' + M_s E_s' + k_s D2M_s) over the trend block;
      // D2M_{s+1} = q D2M_s + dq dm' + dm dq' + (m_s - tc_s) d2q, lane
      // (c = lane & 31, h = lane >> 5) holds rows a = 2i + h of column c
      const int c = lane & 31, h = lane >> 5;
      double D2[16], corr[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) { D2[i] = 0.0; corr[i] = 0.0; }
      for (int s = 0; s <= S; ++s) {
        if (s > 0) {
          const int sp_ = s - 1;
          const double k0 = sm.kseg[sp_], b = sm.kseg[s];
          const double q = k0 / b, ib = 1.0 / b, ib2 = ib * ib;
          const double dmt = sm.mseg[sp_] - sm.ctc[sp_];
          const double Ec = pf_Ecol(c, sp_), Ec1 = pf_Ecol(c, s);
          const double dqc = Ec * ib - k0 * Ec1 * ib2;
          const double Mc = Mt[sp_ * 32 + c];
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int r_ = 2 * i + h;
            const double Ea = pf_Ecol(r_, sp_), Ea1 = pf_Ecol(r_, s);
            const double dqa = Ea * ib - k0 * Ea1 * ib2;
            const double d2q = -(Ea * Ec1 + Ea1 * Ec) * ib2 + 2.0 * k0 * Ea1 * Ec1 * ib2 * ib;
            D2[i] = fma(q, D2[i], fma(dqa, Mc, fma(Mt[sp_ * 32 + r_], dqc, dmt * d2q)));
          }
        }
        const double rs = rho[s], kss = sm.kseg[s];
        const double Ec = pf_Ecol(c, s), Mc = Mt[s * 32 + c];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int r_ = 2 * i + h;
          const double v = pf_Ecol(r_, s) * Mc + Mt[s * 32 + r_] * Ec + kss * D2[i];
          corr[i] = fma(rs, v, corr[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int r_ = 2 * i + h;
        if (r_ < nt && c < nt) A[r_ * LD + c] += corr[i] * inv;
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    // priors, l row/col: d2h/dl2 = 8 sigma^2 + 2Q/sigma^2;
    // d2h/dl dp = (2/sigma^2) sum r dmu/dp = -2 (gh_p - prior'_p)
    double dmax = 0.0;
#pragma unroll
    for (int hw = 0; hw < PW; ++hw) {
      const int p = lane + 64 * hw;
      if (p < P) {
        const double xp = x[hw];
        double prior1 = 0.0, prior2 = 0.0;
        if (p == 0 || p == 1) { prior1 = xp / 25.0; prior2 = 1.0 / 25.0; }
        else if (p > il) {
          const double sg2 = sm.csg[p - il - 1];
          prior1 = xp / (sg2 * sg2);
          prior2 = 1.0 / (sg2 * sg2);
        }
        if (p != il) {
          A[p * LD + p] += prior2;
          const double v = -2.0 * (gh[hw] - prior1);
          A[il * LD + p] = v;
          A[p * LD + il] = v;
        } else {
          A[il * LD + il] = 8.0 * sig2 + 2.0 * Q * inv;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (stash) {
      // the undamped H (packed upper triangle, row i from i (2P - i + 1) / 2)
      // for the QP after the damped first step (polish_run)
      for (int e = lane; e < P * P; e += 64) {
        const int i = e / P, j = e - i * P;
        if (j >= i) sm.hst[i * (2 * P - i + 1) / 2 + (j - i)] = A[i * LD + j];
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    if (lam > 0.0) {
#pragma unroll
      for (int hw = 0; hw < PW; ++hw) {
        const int p = lane + 64 * hw;
        if (p < P) dmax = fmax(dmax, fabs(A[p * LD + p]));
      }
      for (int o = 32; o >= 1; o >>= 1) dmax = fmax(dmax, __shfl_xor(dmax, o, 64));
#pragma unroll
      for (int hw = 0; hw < PW; ++hw) {
        const int p = lane + 64 * hw;
        if (p < P) A[p * LD + p] += lam * dmax;
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// The matrix stride re-materialised inside a loop body: keeps the compiler
// from hoisting one LDS address per matrix row out of the QP loops (16+ live
// VGPRs that end up spilled to scratch and reloaded on every row access).
__device__ __forceinline__ int pf_opaque(int v) {
  int r;
  asm volatile("s_mov_b32 %0, %1" : "=s"(r) : "s"(__builtin_amdgcn_readfirstlane(v)));
  return r;
}

// element i of a vector held one entry per lane in PW words (uniform result)
template <int PW>
__device__ __forceinline__ double pv_read(const PV<PW> &v, int i) {
  if constexpr (PW == 1) {
    return readlane_f64(v[0], i & 63);
  } else {
    return (i < 64) ? readlane_f64(v[0], i) : readlane_f64(v[1], (i - 64) & 63);
  }
}

// Symmetric sweep operator on A (P x P, stride LD, LDS; wave-local, lane =
// column j in each word).  Sweeping k in (rev = false) or out (rev = true)
// with pivot d = A[k][k]:  A[i][j] -= A[i][k] A[k][j] / d  (i, j != k),
//               A[i][k] = A[k][i] = +-A[i][k] / d,  A[k][k] = -1/d.
// After sweeping the set F, A_FF = -(H_FF)^-1, A_FZ = (H_FF)^-1 H_FZ and
// A_ZZ is the Schur complement, so each active-set change costs one O(P^2)
// sweep instead of a refactorisation.  A sweep-in needs d > 0 (H_FF PD).
template <int PW>
__device__ __forceinline__ bool wave_sweep(double *A, int LD_, int P_, int k_, bool rev) {
  const int lane = pf_lane();
  const int LD = pf_opaque(LD_);
  const int P = __builtin_amdgcn_readfirstlane(P_), k = __builtin_amdgcn_readfirstlane(k_);
  const double d = A[k * LD + k];
  if (!rev && !(d > 0.0)) return false;
  if (rev && !(d < 0.0)) return false;
  const double inv = 1.0 / d;
  PV<PW> akj, sj;
#pragma unroll
  for (int h = 0; h < PW; ++h) {
    const int j = lane + 64 * h;
    akj[h] = (j < P) ? A[k * LD + j] : 0.0;
    sj[h] = akj[h] * inv;
  }
  // row k (= column k) is held across lanes in akj: A[k][i] = element i.
  // Rows in blocks of 8, all loads of a block before its stores, no per-row
  // conditions: A carries 8 padding rows past P (their values are don't-care)
  // and row / column k are rewritten below.
#pragma unroll
  for (int h = 0; h < PW; ++h) {
    const int j = lane + 64 * h;
    if (j < P) {
      double *Aj = A + j;
      for (int i0 = 0; i0 < P; i0 += 8) {
        double av[8], ak[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          ak[q] = pv_read<PW>(akj, i0 + q);
          av[q] = Aj[(i0 + q) * LD];
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) Aj[(i0 + q) * LD] = fma(-ak[q], sj[h], av[q]);
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int h = 0; h < PW; ++h) {
    const int j = lane + 64 * h;
    if (j < P && j != k) {
      const double v = rev ? -sj[h] : sj[h];
      A[k * LD + j] = v;
      A[j * LD + k] = v;
    }
    if (j == k) A[k * LD + k] = -inv;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  return true;
}

// Workgroup version of the initial sweep-in: A already holds H (+ damping);
// sweep every coordinate free under the QP's starting active set (|gh| > c
// for delta, always for the rest).  Rows are split across the NW waves (lane
// = column); two barriers per sweep.  Every wave derives the same free set
// from its own copy of gh (lane = parameter).  flag[1] = 1 on a non-positive
// pivot.
template <int NW, int KMAX, int MODE>
__device__ __forceinline__ void sweep_in_free(const FitKArgs &a, FitSmem<NW, KMAX, MODE> &sm,
                                              const PV<ModeTr<MODE>::PW> &gh, double c) {
  constexpr int PW = ModeTr<MODE>::PW;
  const int lane = pf_lane(), wave = pf_wave();
  const int P = __builtin_amdgcn_readfirstlane(a.P), S = __builtin_amdgcn_readfirstlane(a.S);
  const int LD = __builtin_amdgcn_readfirstlane(sm.LD);
  double *A = sm.U;
  constexpr int RW = (64 * PW + NW - 1) / NW;  // rows per wave
  const int r0 = wave * RW;
  if (threadIdx.x == 0) sm.flag[1] = 0;
  __syncthreads();
  const bool isd = (lane >= 2 && lane < 2 + S);
  const bool zero = isd && fabs(gh[0]) <= c;
  unsigned long long fm[PW];
  fm[0] = __ballot(lane < P && !zero);
  if constexpr (PW > 1) fm[1] = __ballot(lane + 64 < P);
  bool failed = false;
#pragma unroll
  for (int h0 = 0; h0 < PW; ++h0) {
    while (!failed && fm[h0]) {
      const int k = (__ffsll((long long)fm[h0]) - 1) + 64 * h0;
      fm[h0] &= fm[h0] - 1;
      const int LDl = pf_opaque(LD);
      const double d = A[k * LDl + k];
      if (!(d > 0.0)) {  // uniform across the workgroup
        if (threadIdx.x == 0) sm.flag[1] = 1;
        failed = true;
        break;
      }
      const double inv = 1.0 / d;
      PV<PW> akj, sj;
#pragma unroll
      for (int h = 0; h < PW; ++h) {
        const int j = lane + 64 * h;
        akj[h] = (j < P) ? A[k * LDl + j] : 0.0;
        sj[h] = akj[h] * inv;
      }
#pragma unroll
      for (int h = 0; h < PW; ++h) {
        const int j = lane + 64 * h;
        if (j < P) {
          // this wave's rows: every load issued before the first store (one
          // LDS latency per pivot instead of one per row); rows past P read
          // row P - 1 and are not stored; row k is left for wave 0 below
          double av[RW];
#pragma unroll
          for (int q = 0; q < RW; ++q) {
            const int i = min(r0 + q, P - 1);
            av[q] = A[i * LDl + j];
          }
#pragma unroll
          for (int q = 0; q < RW; ++q) {
            const int i = r0 + q;
            if (i < P && i != k) A[i * LDl + j] = fma(-pv_read<PW>(akj, i), sj[h], av[q]);
          }
        }
      }
      __syncthreads();
      if (wave == 0) {
#pragma unroll
        for (int h = 0; h < PW; ++h) {
          const int j = lane + 64 * h;
          if (j < P && j != k) {
            A[k * LDl + j] = sj[h];
            A[j * LDl + k] = sj[h];
          }
          if (j == k) A[k * LDl + k] = -inv;
        }
      }
      __syncthreads();
      PF_COUNT(26);
    }
  }
  __syncthreads();
}

// Block form of sweep_in_free: up to PF_SWEEP_BLK pivots K per round, in the
// same order.  With B = A[K][K] (current values) and W = B^-1 A[K][:],
//   A'[i][j] = A[i][j] - A[i][K] W[:][j]   (i, j not in K)
//   A'[K][j] = A'[j][K] = W[:][j],  A'[K][K] = -B^-1,
// which is the sequential sweep of K in exact arithmetic; B^-1 comes from the
// sequential sweeps of the small block, so the positive-pivot checks are the
// sequential ones.  Two barriers per round instead of two per pivot, and one
// read + write of each matrix entry per round instead of per pivot.
#ifndef PF_SWEEP_BLK
#define PF_SWEEP_BLK 2
#endif
template <int NW, int KMAX, int MODE>
__device__ __forceinline__ void sweep_in_free_blk(const FitKArgs &a, FitSmem<NW, KMAX, MODE> &sm,
                                                  const PV<ModeTr<MODE>::PW> &gh, double c) {
  constexpr int PW = ModeTr<MODE>::PW;
  constexpr int BK = PF_SWEEP_BLK > 0 ? PF_SWEEP_BLK : 1;
  const int lane = pf_lane(), wave = pf_wave();
  const int P = __builtin_amdgcn_readfirstlane(a.P), S = __builtin_amdgcn_readfirstlane(a.S);
  const int LD = __builtin_amdgcn_readfirstlane(sm.LD);
  double *A = sm.U;
  constexpr int RW = (64 * PW + NW - 1) / NW;  // rows per wave
  const int r0 = wave * RW;
  if (threadIdx.x == 0) sm.flag[1] = 0;
  __syncthreads();
  const bool isd = (lane >= 2 && lane < 2 + S);
  const bool zero = isd && fabs(gh[0]) <= c;
  unsigned long long fm[PW];
  fm[0] = __ballot(lane < P && !zero);
  if constexpr (PW > 1) fm[1] = __ballot(lane + 64 < P);
  while (true) {
    int ks[BK];
    int nb = 0;
#pragma unroll
    for (int h0 = 0; h0 < PW; ++h0) {
#pragma unroll
      for (int t = 0; t < BK; ++t) {
        if (nb < BK && fm[h0]) {
          ks[nb++] = (__ffsll((long long)fm[h0]) - 1) + 64 * h0;
          fm[h0] &= fm[h0] - 1;
        }
      }
    }
    if (nb == 0) break;
#pragma unroll
    for (int t = 0; t < BK; ++t)
      if (t >= nb) ks[t] = ks[0];
    const int LDl = pf_opaque(LD);
    PV<PW> R[BK];
#pragma unroll
    for (int t = 0; t < BK; ++t)
#pragma unroll
      for (int h = 0; h < PW; ++h) {
        const int j = lane + 64 * h;
        R[t][h] = (t < nb && j < P) ? A[ks[t] * LDl + j] : 0.0;
      }
    // M <- the sequential sweep of B = A[K][K]: -B^-1 (identity padding)
    double M[BK][BK];
#pragma unroll
    for (int t = 0; t < BK; ++t)
#pragma unroll
      for (int u = 0; u < BK; ++u)
        M[t][u] = (t < nb && u < nb) ? pv_read<PW>(R[t], ks[u]) : (t == u ? -1.0 : 0.0);
    bool ok = true;
#pragma unroll
    for (int p = 0; p < BK; ++p) {
      if (p < nb) {
        const double d = M[p][p];
        if (!(d > 0.0)) { ok = false; break; }
        const double inv = 1.0 / d;
#pragma unroll
        for (int i = 0; i < BK; ++i)
#pragma unroll
          for (int j = 0; j < BK; ++j)
            if (i != p && j != p) M[i][j] = fma(-M[i][p] * inv, M[p][j], M[i][j]);
#pragma unroll
        for (int i = 0; i < BK; ++i)
          if (i != p) { M[i][p] *= inv; M[p][i] = M[i][p]; }
        M[p][p] = -inv;
      }
    }
    if (!ok) {  // uniform across the workgroup
      if (threadIdx.x == 0) sm.flag[1] = 1;
      break;
    }
    // W[t][j] = (B^-1 A[K][:])[t][j] = -sum_u M[t][u] R[u][j]
    PV<PW> W[BK];
    bool inK[PW];
#pragma unroll
    for (int h = 0; h < PW; ++h) {
      const int j = lane + 64 * h;
      inK[h] = false;
#pragma unroll
      for (int t = 0; t < BK; ++t) {
        inK[h] |= (t < nb) && (j == ks[t]);
        double v = 0.0;
#pragma unroll
        for (int u = 0; u < BK; ++u) v = fma(-M[t][u], R[u][h], v);
        W[t][h] = (t < nb) ? v : 0.0;
      }
    }
#pragma unroll
    for (int h = 0; h < PW; ++h) {
      const int j = lane + 64 * h;
      if (j < P && !inK[h]) {
        double av[RW];
#pragma unroll
        for (int q = 0; q < RW; ++q) {
          const int i = min(r0 + q, P - 1);
          av[q] = A[i * LDl + j];
        }
#pragma unroll
        for (int q = 0; q < RW; ++q) {
          const int i = r0 + q;
          bool ik = false;
#pragma unroll
          for (int t = 0; t < BK; ++t) ik |= (t < nb) && (i == ks[t]);
          if (i < P && !ik) {
            double v = av[q];
#pragma unroll
            for (int t = 0; t < BK; ++t) v = fma(-pv_read<PW>(R[t], min(i, 64 * PW - 1)), W[t][h], v);
            A[i * LDl + j] = v;
          }
        }
      }
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int h = 0; h < PW; ++h) {
        const int j = lane + 64 * h;
        if (j < P) {
#pragma unroll
          for (int t = 0; t < BK; ++t) {
            if (t < nb) {
              if (!inK[h]) {
                A[ks[t] * LDl + j] = W[t][h];
                A[j * LDl + ks[t]] = W[t][h];
              } else {
#pragma unroll
                for (int u = 0; u < BK; ++u)
                  if (u < nb && j == ks[u]) A[ks[t] * LDl + j] = M[t][u];
              }
            }
          }
        }
      }
    }
    __syncthreads();
    PF_COUNT(26);
  }
  __syncthreads();
}

// u = A v for the symmetric swept matrix (lane p: u_p = sum_q A[q][p] v_q;
// v staged in LDS, read by uniform broadcast)
template <int PW>
__device__ __forceinline__ PV<PW> wave_symv(const double *A, int LD_, int P_, const double *v) {
  const int lane = pf_lane();
  const int LD = pf_opaque(LD_);
  const int P = __builtin_amdgcn_readfirstlane(P_);
  PV<PW> out;
#pragma unroll
  for (int h = 0; h < PW; ++h) {
    const int p = lane + 64 * h;
    double u[4] = {0.0, 0.0, 0.0, 0.0};
    if (p < P) {
      // 8 rows per batch, all loads issued before the FMAs (one LDS latency
      // per batch); rows past P read the zeroed padding rows with v = 0
      const double *Ap = A + p;
      for (int q0 = 0; q0 < P; q0 += 8) {
        double av[8], vv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          av[j] = Ap[(q0 + j) * LD];
          vv[j] = v[q0 + j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) u[j & 3] = fma(av[j], vv[j], u[j & 3]);
      }
    }
    out[h] = (u[0] + u[1]) + (u[2] + u[3]);
  }
  return out;
}

// Active-set solution of min gh.(z-x) + (z-x)'H(z-x)/2 + c||z_delta||_1 (wave 0).
// Returns z (lane p, word h); false if a pivot failed or the active set did
// not settle.  Only delta coordinates (word 0, lanes 2..S+1) change activity.
//
// Cold start (warm = false): the starting active set is {delta: |gh| <= c}
// and A holds H with its complement swept in (sweep_in_free).  Warm start:
// A and the active set (zero, sgn_: lane-local, wave 0) are the ones the
// previous QP ended with — the swept matrix depends only on H and the free
// set, so a QP at a new (x, gh) under the same H needs no initial sweeps.
template <int NW, int KMAX, int MODE>
__device__ __forceinline__ bool qp_active(const FitKArgs &a, FitSmem<NW, KMAX, MODE> &sm,
                                          const PV<ModeTr<MODE>::PW> &x, const PV<ModeTr<MODE>::PW> &gh,
                                          double c, PV<ModeTr<MODE>::PW> &z, int &nsolve, bool &zero,
                                          double &sgn_, bool warm) {
  constexpr int PW = ModeTr<MODE>::PW;
  const int lane = pf_lane();
  const int P = __builtin_amdgcn_readfirstlane(a.P), S = __builtin_amdgcn_readfirstlane(a.S);
  const int LD = __builtin_amdgcn_readfirstlane(sm.LD);
  double *A = sm.U;
  const bool isd = (lane >= 2 && lane < 2 + S);
  if (isd) {
    const double sgx = (x[0] > 0.0) - (x[0] < 0.0), sgg = (gh[0] > 0.0) - (gh[0] < 0.0);
    if (!warm) {
      zero = false;
      sgn_ = 0.0;
      if (fabs(gh[0]) <= c) zero = true;
      else if (x[0] != 0.0 && sgx == -sgg) sgn_ = sgx;
      else sgn_ = -sgg;
    } else if (!zero) {
      sgn_ = (x[0] != 0.0) ? sgx : -sgg;
    }
  } else {
    zero = false;
    sgn_ = 0.0;
  }
  // cold: A holds H with every initially free coordinate swept in
  // (sweep_in_free, all waves); a failed pivot there leaves flag[1] set
  if (!warm && sm.flag[1]) return false;
  z = x;
  const int max_as = 2 * S + 16;
  for (int it = 0; it < max_as; ++it) {
    // v: free -> gh + c s ; zero -> x  (so u_F = d_F, u_Z = gh_Z - model grad)
#pragma unroll
    for (int h = 0; h < PW; ++h) {
      const int p = lane + 64 * h;
      const bool zh = (h == 0) && zero;
      sm.pz[p] = (p < P) ? (zh ? x[h] : gh[h] + ((h == 0) ? c * sgn_ : 0.0)) : 0.0;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    PF_COUNT(27);
    const PV<PW> u = wave_symv<PW>(A, LD, P, sm.pz);
    ++nsolve;
    PV<PW> zn;
#pragma unroll
    for (int h = 0; h < PW; ++h) {
      const int p = lane + 64 * h;
      const bool fr = (p < P) && !((h == 0) && zero);
      zn[h] = fr ? x[h] + u[h] : 0.0;
    }
    // first sign crossing among free delta coordinates along z -> zn
    const bool viol = isd && !zero && (zn[0] * sgn_ < 0.0);
    const double tt = viol ? ((z[0] != zn[0]) ? z[0] / (z[0] - zn[0]) : 0.0) : 2.0;
    double tmin = tt;
    tmin = fmin(tmin, shfl_xor_f64<1>(tmin));
    tmin = fmin(tmin, shfl_xor_f64<2>(tmin));
    tmin = fmin(tmin, shfl_xor_f64<4>(tmin));
    tmin = fmin(tmin, shfl_xor_f64<8>(tmin));
    tmin = fmin(tmin, shfl_xor_f64<16>(tmin));
    tmin = fmin(tmin, shfl_xor_f64<32>(tmin));
    if (tmin < 2.0) {
      const unsigned long long hit = __ballot(viol && tt == tmin);
      const int jmin = __ffsll((long long)hit) - 1;
#pragma unroll
      for (int h = 0; h < PW; ++h) {
        const int p = lane + 64 * h;
        z[h] = (p < P) ? z[h] + tmin * (zn[h] - z[h]) : 0.0;
      }
      if (lane == jmin) { z[0] = 0.0; zero = true; sgn_ = 0.0; }
      if (!wave_sweep<PW>(A, LD, P, jmin, true)) return false;
      continue;
    }
#pragma unroll
    for (int h = 0; h < PW; ++h) z[h] = (lane + 64 * h < P) ? zn[h] : 0.0;
    // KKT of zero delta coordinates: |gh + H (z - x)| <= c
    const bool cand = isd && zero;
    const double gq = cand ? gh[0] - u[0] : 0.0;
    const double sc = (cand && fabs(gq) > c * (1.0 + 1e-12)) ? fabs(gq) : -1.0;
    double smax = sc;
    smax = fmax(smax, shfl_xor_f64<1>(smax));
    smax = fmax(smax, shfl_xor_f64<2>(smax));
    smax = fmax(smax, shfl_xor_f64<4>(smax));
    smax = fmax(smax, shfl_xor_f64<8>(smax));
    smax = fmax(smax, shfl_xor_f64<16>(smax));
    smax = fmax(smax, shfl_xor_f64<32>(smax));
    if (smax < 0.0) return true;
    const unsigned long long hit = __ballot(sc == smax && sc >= 0.0);
    const int jadd = __ffsll((long long)hit) - 1;
    if (lane == jadd) { zero = false; sgn_ = -((gq > 0.0) - (gq < 0.0)); }
    if (!wave_sweep<PW>(A, LD, P, jadd, false)) return false;
  }
  return false;  // active set did not settle
}

// Returns true when the polish certifies the optimum: the last lasso-QP
// (solved to KKT under a positive-definite model) predicts no decrease
// beyond 1e-15 |f|.
//
// Lagged Hessian: after a full undamped Newton step (alpha = 1) the next QP
// reuses the swept matrix of the previous one (warm start) instead of
// recomputing it, as long as each lagged step shrinks the predicted
// decrease by >= 1 / pf_fit_opts.polish_lag_ratio (default 100x: measured,
// 0.1 .. 0.5 save 5-6 % of k_polish at configs[4] but certify fewer series,
// tools/lag_experiment.sh) at most polish_max_lag times in a row (default
// 4); otherwise, or after a backtracked step
// or a failed warm QP, the exact Hessian is recomputed.  A cold QP that hits
// a non-positive pivot recomputes the Hessian with Levenberg-Marquardt
// damping (x10 per retry).  A QP under any positive definite model predicts
// zero decrease exactly at a KKT point, so the certificate holds either way;
// oracle/stan_lbfgs.c:orc_polish_ex recomputes every iteration and reaches
// the same MAP.
// A <- the stashed undamped Hessian (hessian_collective with stash), padding
// rows zeroed as the assembly leaves them.  Wave 0; the caller synchronises.
template <int NW, int KMAX, int MODE>
__device__ __forceinline__ void restore_hessian(const FitKArgs &a, FitSmem<NW, KMAX, MODE> &sm) {
  if (pf_wave() != 0) return;
  const int lane = pf_lane();
  const int P = __builtin_amdgcn_readfirstlane(a.P);
  const int LD = __builtin_amdgcn_readfirstlane(sm.LD);
  double *A = sm.U;
  for (int e = lane; e < (P + 8) * LD; e += 64) A[e] = 0.0;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  for (int e = lane; e < P * P; e += 64) {
    const int i = e / P, j = e - i * P;
    if (j >= i) {
      const double v = sm.hst[i * (2 * P - i + 1) / 2 + (j - i)];
      A[i * LD + j] = v;
      A[j * LD + i] = v;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

#define PF_POLISH_MAXDAMP 24
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__device__ __forceinline__ bool polish_run(const FitKArgs &a, FitSmem<NW, KMAX, MODE> &sm,
                                           PV<ModeTr<MODE>::PW> &x, double &f, PV<ModeTr<MODE>::PW> &g,
                                           int &n_eval, int &n_newton) {
  constexpr int PW = ModeTr<MODE>::PW;
  const int lane = pf_lane(), wave = pf_wave();
  const int S = a.S, P = a.P;
  const double c = 1.0 / sm.sig[2];
  const bool isd = (lane >= 2 && lane < 2 + S);
  n_newton = 0;
  PF_COUNT(23);
  bool cert = false;
  bool need_h = true;
  int lag = 0, ndamp = 0;
  // the first QP's model is damped (pf_fit_opts.polish_lam0): an undamped
  // first Newton step from the warm-up hand-off can jump into a neighbouring,
  // worse local optimum (tools/diag_basin_floor.py / diag_basin_commit.py)
  const double lam0 = a.o.polish_lam0 > 0.0 ? a.o.polish_lam0 : 0.0;
  double lam = lam0;
  double dec_prev = 0.0;
  bool zero = false;    // QP active set (wave 0, lane = parameter)
  double sgn_ = 0.0;
  // the damped first step's Hessian is stashed undamped (FitKArgs.hstash):
  // the next QP sweeps it in again instead of recomputing H at the new point
  // (a lagged Hessian one short step old; the certificate holds for any
  // positive-definite model)
  bool stashed = false, restore = false;
  for (int it = 0; it < a.o.polish_max_iter;) {
    PV<PW> gh = g;
    if (isd) gh[0] = g[0] - c * (double)((x[0] > 0.0) - (x[0] < 0.0));
    const bool fresh = need_h;
    const bool restored = fresh && restore;
    if (fresh) {
      PF_STAMP(20);
      if (restored) {
        const unsigned long long t_r0 = PF_RT();
        restore_hessian<NW, KMAX, MODE>(a, sm);
        PF_BLKV(10, PF_RT() - t_r0);
        restore = false;
      } else {
        PF_COUNT(15);
        const bool st = a.hstash && n_newton == 0 && lam > 0.0 && lam <= lam0;
        const unsigned long long t_h0 = PF_RT();
        hessian_collective<NW, KMAX, O0, O1, O2, MODE>(a, sm, x, gh, lam, st);
        PF_BLKV(5, 1);
        PF_BLKV(6, PF_RT() - t_h0);
        stashed = st;
      }
      __syncthreads();
      PF_STAMP(21);
      const unsigned long long t_s0 = PF_RT();
#if PF_SWEEP_BLK > 1
      sweep_in_free_blk<NW, KMAX, MODE>(a, sm, gh, c);
#else
      sweep_in_free<NW, KMAX, MODE>(a, sm, gh, c);
#endif
      PF_BLKV(7, PF_RT() - t_s0);
      PF_STAMP(24);
    }
    PF_STAMP(19);
    const unsigned long long t_q0 = PF_RT();
    if (wave == 0) {
      pf_serial_prio(true);
      PV<PW> z;
      int ns = 0;
      const bool ok = qp_active<NW, KMAX, MODE>(a, sm, x, gh, c, z, ns, zero, sgn_, !fresh);
      PF_STAMP(22);
      double dl = 0.0, l1 = 0.0;
#pragma unroll
      for (int h = 0; h < PW; ++h) {
        const int p = lane + 64 * h;
        const double d = (p < P) ? z[h] - x[h] : 0.0;
        dl = fma(gh[h], d, dl);
        sm.pd[p] = d;
      }
      if (isd) l1 = fabs(z[0]) - fabs(x[0]);
      double dec, l1s;
      wave_sum2(dl, l1, dec, l1s);
      dec += c * l1s;
      if (lane == 0) { sm.fout[2] = ok ? dec : 0.0; sm.fout[3] = ok ? 1.0 : 0.0; }
      pf_serial_prio(false);
    }
    __syncthreads();
    PF_BLKV(8, PF_RT() - t_q0);
    const double dec = sm.fout[2];
    const bool qp_ok = sm.fout[3] != 0.0;
    PV<PW> d;
#pragma unroll
    for (int h = 0; h < PW; ++h) d[h] = sm.pd[lane + 64 * h];
    __syncthreads();
    if (!qp_ok) {
      // warm QP failed: recompute the Hessian at the same point; cold QP
      // failed (non-positive pivot): damp the model and recompute (a failed
      // QP on the restored stash first recomputes the exact Hessian)
      if (fresh) PF_COUNT(28); else PF_COUNT(29);
      if (fresh && !restored) {
        if (++ndamp > PF_POLISH_MAXDAMP) break;
        lam = (lam == 0.0) ? 1e-10 : lam * 10.0;
      }
      need_h = true;
      lag = 0;
      continue;
    }
    if (!fresh && !(fabs(dec) < a.o.polish_lag_ratio * fabs(dec_prev))) {
      PF_COUNT(30);
      // the lagged model stopped converging fast: recompute the Hessian
      need_h = true;
      lag = 0;
      continue;
    }
    ++it;
    if (!(dec < -1e-15 * fabs(f))) {
      cert = dec == dec;
      break;
    }
    ++n_newton;
    PF_COUNT(18);
    PF_STAMP(16);
    double alpha = 1.0, fn = 0.0;
    PV<PW> gn = pv_zero<PW>(), xn = x;
    bool acc = false;
    for (int ls = 0; ls < 30; ++ls) {
#pragma unroll
      for (int h = 0; h < PW; ++h) xn[h] = x[h] + alpha * d[h];
      const unsigned long long t_e0 = PF_RT();
      const bool bad = eval_collective<NW, KMAX, O0, O1, O2, MODE>(a, sm, xn, fn, gn);
      PF_BLKV(9, PF_RT() - t_e0);
      ++n_eval;
      if (!bad && fn <= f + 1e-4 * alpha * dec) { acc = true; break; }
      alpha *= 0.5;
    }
    PF_STAMP(17);
    if (!acc) break;
    if (alpha < 1.0) PF_COUNT(31);
    x = xn;
    f = fn;
    g = gn;
    // the first step's damping ends with it; damping a non-positive pivot
    // raised relaxes /10 per accepted step (oracle orc_polish_cfg2)
    if (n_newton == 1 && lam <= lam0) {
      lam = 0.0;
      restore = stashed;
    } else {
      lam = (lam < 1e-9) ? 0.0 : lam * 0.1;
    }
    stashed = false;
    if (restore) {
      need_h = true;   // the restored stash (a lagged Hessian: lag 1 after it)
      lag = 0;
    } else {
      need_h = !(alpha == 1.0 && lag < a.o.polish_max_lag && lam == 0.0);
      lag = need_h ? 0 : lag + 1;
    }
    if (restored) lag = need_h ? 0 : lag + 1;
    dec_prev = dec;
  }
  return cert;
}
