// pf_polish.h — exact-MAP polish after the Stan-faithful L-BFGS phase.
//
// Engine extension (NOT part of Stan): Stan's smooth L-BFGS stalls at the L1
// kink of delta ~ double_exponential(0, tau) up to ~3e-5 relative short of the
// MAP (yhat off by up to ~2e-3*y_scale).  From where it stops we run proximal
// Newton on f = h + c*||delta||_1 (c = 1/tau):
//   1. exact Hessian of the smooth part h.  Its data term (J^T J - R)/sigma^2
//      is a genuine GEMM over the T rows: J[T x 64] with 10 16x16 output tiles,
//      accumulated on FP64 MFMA (v_mfma_f64_16x16x4f64);
//   2. the lasso-QP subproblem min gh.d + d'Hd/2 + c||x_delta + d_delta||_1,
//      solved exactly by an active-set method (Cholesky solves in LDS, wave 0);
//   3. Armijo backtracking on the true objective (collective evaluations);
//   4. after a full step the next QP reuses H and its swept matrix (lagged
//      Hessian, see polish_run).
// Same algorithm as oracle/stan_lbfgs.c:orc_polish (the CPU check).
// Linear growth, K <= 32, 2 + S <= 32 (the reference configuration).
#pragma once

typedef double pf_d4 __attribute__((ext_vector_type(4)));

#define PF_NTILE 10
// tile (row block, col block) in the 64-column space [a: 0..31 | beta: 32..63]
__device__ __forceinline__ int tile_ti(int q) {
  constexpr int T_I[PF_NTILE] = {0, 0, 1, 2, 2, 3, 0, 0, 1, 1};
  return T_I[q];
}
__device__ __forceinline__ int tile_tj(int q) {
  constexpr int T_J[PF_NTILE] = {0, 1, 1, 2, 3, 3, 2, 3, 2, 3};
  return T_J[q];
}

// column of the 64-wide J space -> parameter index (or -1)
__device__ __forceinline__ int colmap(int c, int S, int K) {
  if (c < 32) return (c < 2 + S) ? c : -1;
  const int f = c - 32;
  return (f < K) ? 3 + S + f : -1;
}

// publish theta (wave 0) — same as the evaluation's phase 0

template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__device__ __forceinline__ void hessian_collective(const FitKArgs &a, FitSmem<NW, KMAX, MODE> &sm, double x,
                                   double gh, double *ws) {
  const int lane = pf_lane(), wave = pf_wave();
  const int S = __builtin_amdgcn_readfirstlane(a.S), K = __builtin_amdgcn_readfirstlane(a.K);
  const int T = __builtin_amdgcn_readfirstlane(a.T), Tp = __builtin_amdgcn_readfirstlane(a.Tp);
  const int P = __builtin_amdgcn_readfirstlane(a.P);
  {
    PV<1> xv;
    xv[0] = x;
    publish_theta<NW, KMAX, MODE>(a, sm, xv);
  }
  __syncthreads();
  // ---- H1: per-row u, tr, r into the workspace (row per lane)
  double Q = 0.0;
  const double th_m = sm.th[1];
  const bool linear = (a.growth == PF_GROWTH_LINEAR);
  constexpr int NL = NW * 64;
  for (int rr = 0; rr < a.R; ++rr) {
    const int q = rr * NL + threadIdx.x;        // lane-blocked position
    const int i = threadIdx.x * a.R + rr;       // natural row
    const bool valid = i < T;
    RowIn cur;
    load_rowp<O0, O1, O2>(a, q, cur);
    double xf[KMAX];
    row_features_from<KMAX, O0, O1, O2>(cur, a.XTP, a.TQ, K, q, xf);
    double xm[4] = {0.0, 0.0, 0.0, 0.0}, xa[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int f2 = 0; f2 < KMAX; ++f2) {
      if constexpr ((MODE & 3) != MODE_ADD) xm[f2 & 3] = fma(xf[f2], sm.bm[f2], xm[f2 & 3]);
      if constexpr ((MODE & 3) != MODE_MULT) xa[f2 & 3] = fma(xf[f2], sm.ba[f2], xa[f2 & 3]);
      if ((f2 & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    }
    const double xbm = (xm[0] + xm[1]) + (xm[2] + xm[3]);
    const double xba = (xa[0] + xa[1]) + (xa[2] + xa[3]);
    const double tr = linear ? fma(sm.kseg[cur.seg], cur.t, sm.mseg[cur.seg]) : th_m;
    const double u = 1.0 + xbm;
    const double r = valid ? (sm.y[q] - fma(tr, u, xba)) : 0.0;
    Q = fma(r, r, Q);
    if (i < Tp) {
      ws[i] = valid ? u : 0.0;
      ws[Tp + i] = valid ? tr : 0.0;
      ws[2 * Tp + i] = r;
    }
  }
  Q = wave_sum(Q);
  if (lane == 0) sm.rrw[wave] = Q;
  __syncthreads();
  PF_STAMP(13);
  PF_COUNT(15);
  // ---- H2: J^T J - R on FP64 MFMA.  k-steps of 4 rows, split over waves.
  pf_d4 acc[PF_NTILE];
#pragma unroll
  for (int q = 0; q < PF_NTILE; ++q) acc[q] = pf_d4{0.0, 0.0, 0.0, 0.0};
  const int c16 = lane & 15;
  const int c1 = 16 + c16;
  const double tc0 = (c16 >= 2 && c16 - 2 < S) ? a.t_change[c16 - 2] : 0.0;
  const double tc1 = (c1 - 2 < S) ? a.t_change[c1 - 2] : 0.0;
  const bool f2v = c16 < K, f3v = c1 < K;
  const double cm2 = f2v ? a.s_m[c16] : 0.0, ca2 = f2v ? a.s_a[c16] : 0.0;
  const double cm3 = f3v ? a.s_m[c1] : 0.0, ca3 = f3v ? a.s_a[c1] : 0.0;
  const int nks = (T + 3) >> 2;  // k-steps holding a valid row
  // operands of the next k-step are loaded before this step's MFMAs
  // (global/L2 latency would otherwise stall every step)
  struct HIn { double u, tr, r, ti, X2, X3; int sg; };
  auto hload = [&](int s_, HIn &h) {
    const int rho = 4 * s_ + (lane >> 4);
    h.u = ws[rho];
    h.tr = ws[Tp + rho];
    h.r = ws[2 * Tp + rho];
    h.ti = a.t[rho];
    h.sg = a.seg[rho];
    h.X2 = f2v ? a.XT[(size_t)c16 * Tp + rho] : 0.0;
    h.X3 = f3v ? a.XT[(size_t)c1 * Tp + rho] : 0.0;
  };
  HIn nx;
  if (wave < nks) hload(wave, nx);
  for (int s = wave; s < nks; s += NW) {
    const HIn cu = nx;
    if (s + NW < nks) hload(s + NW, nx);
    const int rho = 4 * s + (lane >> 4);
    const double u = cu.u, tr = cu.tr, r = cu.r;
    const double ti = cu.ti;
    const int sg = cu.sg;
    // a columns (tile 0: c16, tile 1: 16 + c16)
    double D0, D1;
    if (c16 == 0) D0 = ti;
    else if (c16 == 1) D0 = 1.0;
    else D0 = (c16 - 2 < S && sg > c16 - 2) ? ti - tc0 : 0.0;
    D1 = (c1 - 2 < S && sg > c1 - 2) ? ti - tc1 : 0.0;
    if (rho >= T) { D0 = 0.0; D1 = 0.0; }
    const double Du0 = D0 * u, Du1 = D1 * u;
    // beta columns (tile 2: f = c16, tile 3: f = 16 + c16)
    const double X2 = cu.X2, X3 = cu.X3;
    const double k2 = fma(tr, cm2, ca2), k3 = fma(tr, cm3, ca3);
    const double V2 = X2 * k2, V3 = X3 * k3;
    const double W2 = X2 * fma(u, k2, -r * cm2), W3 = X3 * fma(u, k3, -r * cm3);
    acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(Du0, Du0, acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(Du0, Du1, acc[1], 0, 0, 0);
    acc[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(Du1, Du1, acc[2], 0, 0, 0);
    acc[3] = __builtin_amdgcn_mfma_f64_16x16x4f64(V2, V2, acc[3], 0, 0, 0);
    acc[4] = __builtin_amdgcn_mfma_f64_16x16x4f64(V2, V3, acc[4], 0, 0, 0);
    acc[5] = __builtin_amdgcn_mfma_f64_16x16x4f64(V3, V3, acc[5], 0, 0, 0);
    acc[6] = __builtin_amdgcn_mfma_f64_16x16x4f64(D0, W2, acc[6], 0, 0, 0);
    acc[7] = __builtin_amdgcn_mfma_f64_16x16x4f64(D0, W3, acc[7], 0, 0, 0);
    acc[8] = __builtin_amdgcn_mfma_f64_16x16x4f64(D1, W2, acc[8], 0, 0, 0);
    acc[9] = __builtin_amdgcn_mfma_f64_16x16x4f64(D1, W3, acc[9], 0, 0, 0);
  }
  PF_STAMP(14);
  // ---- H3: chained reduction of the tiles over waves through one
  // wave-sized LDS buffer (NW-1 hops; keeps the union region small)
  double *red = sm.U;  // [PF_NTILE][4][64]
  for (int w2 = NW - 1; w2 >= 1; --w2) {
    if (wave == w2) {
#pragma unroll
      for (int q = 0; q < PF_NTILE; ++q)
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) red[((size_t)q * 4 + rg) * 64 + lane] = acc[q][rg];
    }
    __syncthreads();
    if (wave == w2 - 1) {
#pragma unroll
      for (int q = 0; q < PF_NTILE; ++q)
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) acc[q][rg] += red[((size_t)q * 4 + rg) * 64 + lane];
    }
    __syncthreads();
  }
  // ---- H4: wave 0 assembles H (LDS, stride LD) incl. priors and the l row
  if (wave == 0) {
    double *H = sm.U;
    const int LD = sm.LD;
    for (int e = lane; e < P * LD; e += 64) H[e] = 0.0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    Q = 0.0;
    for (int w2 = 0; w2 < NW; ++w2) Q += sm.rrw[w2];
    const double ls = readlane_f64(x, 2 + S);
    const double sig2 = exp(2.0 * ls);
    const double inv = 1.0 / sig2;
#pragma unroll
    for (int q = 0; q < PF_NTILE; ++q) {
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const int ci = tile_ti(q) * 16 + (lane >> 4) + 4 * rg;
        const int cj = tile_tj(q) * 16 + (lane & 15);
        const int pi = colmap(ci, S, K), pj = colmap(cj, S, K);
        if (pi >= 0 && pj >= 0) {
          const double v = acc[q][rg] * inv;
          H[pi * LD + pj] = v;
          H[pj * LD + pi] = v;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // priors, l row/col: d2h/dl2 = 8 sigma^2 + 2Q/sigma^2;
    // d2h/dl dp = (2/sigma^2) sum r dmu/dp = -2 (gh_p - prior'_p)
    const int il = 2 + S;
    const int p = lane;
    if (p < P) {
      double prior1 = 0.0, prior2 = 0.0;
      if (p == 0 || p == 1) { prior1 = x / 25.0; prior2 = 1.0 / 25.0; }
      else if (p > il) {
        const double sg2 = sm.csg[p - il - 1];
        prior1 = x / (sg2 * sg2);
        prior2 = 1.0 / (sg2 * sg2);
      }
      if (p != il) {
        H[p * LD + p] += prior2;
        const double v = -2.0 * (gh - prior1);
        H[il * LD + p] = v;
        H[p * LD + il] = v;
      } else {
        H[il * LD + il] = 8.0 * sig2 + 2.0 * Q * inv;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
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

// Symmetric sweep operator on A (P x P, stride LD, LDS; wave-local, lane =
// column j).  Sweeping k in (rev = false) or out (rev = true) with pivot
// d = A[k][k]:  A[i][j] -= A[i][k] A[k][j] / d  (i, j != k),
//               A[i][k] = A[k][i] = +-A[i][k] / d,  A[k][k] = -1/d.
// After sweeping the set F, A_FF = -(H_FF)^-1, A_FZ = (H_FF)^-1 H_FZ and
// A_ZZ is the Schur complement, so each active-set change costs one O(P^2)
// sweep instead of a refactorisation.  A sweep-in needs d > 0 (H_FF PD).
__device__ __forceinline__ bool wave_sweep(double *A, int LD_, int P_, int k_, bool rev) {
  const int j = pf_lane();
  const int LD = pf_opaque(LD_);
  const int P = __builtin_amdgcn_readfirstlane(P_), k = __builtin_amdgcn_readfirstlane(k_);
  const double d = A[k * LD + k];
  if (!rev && !(d > 0.0)) return false;
  if (rev && !(d < 0.0)) return false;
  const double inv = 1.0 / d;
  const double akj = (j < P) ? A[k * LD + j] : 0.0;
  const double sj = akj * inv;
  // row k (= column k) is held across lanes in akj: A[k][i] = readlane(akj, i).
  // Rows in blocks of 8, all loads of a block before its stores, no per-row
  // conditions: A carries 8 padding rows past P (their values are don't-care)
  // and row / column k are rewritten below.
  if (j < P) {
    double *Aj = A + j;
    for (int i0 = 0; i0 < P; i0 += 8) {
      double av[8], ak[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        ak[q] = readlane_f64(akj, (i0 + q) & 63);
        av[q] = Aj[(i0 + q) * LD];
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) Aj[(i0 + q) * LD] = fma(-ak[q], sj, av[q]);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (j < P && j != k) {
    const double v = rev ? -sj : sj;
    A[k * LD + j] = v;
    A[j * LD + k] = v;
  }
  if (j == k) A[k * LD + k] = -inv;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  return true;
}

// Workgroup version of the initial sweep-in: A = H, then sweep every
// coordinate free under the QP's starting active set (|gh| > c for delta,
// always for the rest).  Rows are split across the NW waves (lane =
// column); two barriers per sweep.  Every wave derives the same free set
// from its own copy of x and gh (lane = parameter).  flag[1] = 1 on a
// non-positive pivot.
template <int NW, int KMAX, int MODE>
__device__ __forceinline__ void sweep_in_free(const FitKArgs &a, FitSmem<NW, KMAX, MODE> &sm, double gh,
                                              double c) {
  const int lane = pf_lane(), wave = pf_wave();
  const int P = __builtin_amdgcn_readfirstlane(a.P), S = __builtin_amdgcn_readfirstlane(a.S);
  const int LD = __builtin_amdgcn_readfirstlane(sm.LD);
  const double *H = sm.U;
  double *A = sm.U + (size_t)P * LD;
  constexpr int RW = (64 + NW - 1) / NW;  // rows per wave
  const int r0 = wave * RW;
  if (lane < P)
    for (int i = r0; i < r0 + RW && i < P; ++i) A[i * LD + lane] = H[i * LD + lane];
  // 8 zeroed padding rows past P (read unconditionally by the batched
  // sweep / symv loops)
  if (lane < LD)
    for (int i = P + wave; i < P + 8; i += NW) A[i * LD + lane] = 0.0;
  if (threadIdx.x == 0) sm.flag[1] = 0;
  __syncthreads();
  const bool isd = (lane >= 2 && lane < 2 + S);
  const bool zero = isd && fabs(gh) <= c;
  unsigned long long fm = __ballot(lane < P && !zero);
  while (fm) {
    const int k = __ffsll((long long)fm) - 1;
    fm &= fm - 1;
    const int LDl = pf_opaque(LD);
    const double d = A[k * LDl + k];
    if (!(d > 0.0)) {  // uniform across the workgroup
      if (threadIdx.x == 0) sm.flag[1] = 1;
      break;
    }
    const double inv = 1.0 / d;
    const double akj = (lane < P) ? A[k * LDl + lane] : 0.0;
    const double sj = akj * inv;
    if (lane < P) {
      double *Ar = A + r0 * LDl + lane;
#pragma unroll
      for (int q = 0; q < RW; ++q) {
        const int i = r0 + q;
        if (i < P && i != k) Ar[q * LDl] = fma(-readlane_f64(akj, i), sj, Ar[q * LDl]);
      }
    }
    __syncthreads();
    if (wave == 0) {
      if (lane < P && lane != k) {
        A[k * LDl + lane] = sj;
        A[lane * LDl + k] = sj;
      }
      if (lane == k) A[k * LDl + k] = -inv;
    }
    __syncthreads();
    PF_COUNT(26);
  }
  __syncthreads();
}

// u = A v for the symmetric swept matrix (lane p: u_p = sum_q A[q][p] v_q;
// v staged in LDS, read by uniform broadcast)
__device__ __forceinline__ double wave_symv(const double *A, int LD_, int P_, const double *v) {
  const int p = pf_lane();
  const int LD = pf_opaque(LD_);
  const int P = __builtin_amdgcn_readfirstlane(P_);
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
  return (u[0] + u[1]) + (u[2] + u[3]);
}

// Active-set solution of min gh.(z-x) + (z-x)'H(z-x)/2 + c||z_delta||_1 (wave 0).
// Returns z in lane p; false if a pivot failed or the active set did not settle.
//
// Cold start (warm = false): the starting active set is {delta: |gh| <= c}
// and A holds H with its complement swept in (sweep_in_free).  Warm start:
// A and the active set (zero, sgn_: lane-local, wave 0) are the ones the
// previous QP ended with — the swept matrix depends only on H and the free
// set, so a QP at a new (x, gh) under the same H needs no initial sweeps.
template <int NW, int KMAX, int MODE>
__device__ __forceinline__ bool qp_active(const FitKArgs &a, FitSmem<NW, KMAX, MODE> &sm, double x, double gh, double c,
                          double &z, int &nsolve, bool &zero, double &sgn_, bool warm) {
  const int lane = pf_lane();
  const int P = __builtin_amdgcn_readfirstlane(a.P), S = __builtin_amdgcn_readfirstlane(a.S);
  const int LD = __builtin_amdgcn_readfirstlane(sm.LD);
  double *A = sm.U + (size_t)P * LD;
  const bool isd = (lane >= 2 && lane < 2 + S);
  if (isd) {
    const double sgx = (x > 0.0) - (x < 0.0), sgg = (gh > 0.0) - (gh < 0.0);
    if (!warm) {
      zero = false;
      sgn_ = 0.0;
      if (fabs(gh) <= c) zero = true;
      else if (x != 0.0 && sgx == -sgg) sgn_ = sgx;
      else sgn_ = -sgg;
    } else if (!zero) {
      sgn_ = (x != 0.0) ? sgx : -sgg;
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
    const bool fr = (lane < P) && !zero;
    // v: free -> gh + c s ; zero -> x  (so u_F = d_F, u_Z = gh_Z - model grad)
    sm.pz[lane] = (lane < P) ? (zero ? x : gh + c * sgn_) : 0.0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    PF_COUNT(27);
    PF_STAMP(28);
    const double u = wave_symv(A, LD, P, sm.pz);
    PF_STAMP(29);
    ++nsolve;
    const double zn = fr ? x + u : 0.0;
    // first sign crossing among free delta coordinates along z -> zn
    const bool viol = isd && fr && (zn * sgn_ < 0.0);
    const double tt = viol ? ((z != zn) ? z / (z - zn) : 0.0) : 2.0;
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
      z = (lane < P) ? z + tmin * (zn - z) : 0.0;
      if (lane == jmin) { z = 0.0; zero = true; sgn_ = 0.0; }
      PF_STAMP(30);
      if (!wave_sweep(A, LD, P, jmin, true)) return false;
      PF_STAMP(31);
      continue;
    }
    z = (lane < P) ? zn : 0.0;
    // KKT of zero delta coordinates: |gh + H (z - x)| <= c
    const bool cand = isd && zero;
    const double gq = cand ? gh - u : 0.0;
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
    if (!wave_sweep(A, LD, P, jadd, false)) return false;
  }
  return false;  // active set did not settle
}

// Returns true when the polish certifies the optimum: the last lasso-QP
// (solved to KKT) predicts no decrease beyond 1e-15 |f|.
//
// Lagged Hessian: after a full Newton step (alpha = 1) the next QP reuses the
// Hessian and the swept matrix of the previous one (warm start) instead of
// recomputing them, as long as each lagged step shrinks the predicted
// decrease by >= 100x (superlinear); otherwise, or after a backtracked step or
// a failed warm QP, the exact Hessian is recomputed.  A QP under any positive
// definite model predicts zero decrease exactly at a KKT point, so the
// certificate is unchanged; oracle/stan_lbfgs.c:orc_polish recomputes every
// iteration and reaches the same MAP.
#define PF_POLISH_MAXLAG 4
template <int NW, int KMAX, int O0, int O1, int O2, int MODE>
__device__ __forceinline__ bool polish_run(const FitKArgs &a, FitSmem<NW, KMAX, MODE> &sm, double &x, double &f,
                           double &g, int &n_eval, int &n_newton) {
  const int lane = pf_lane(), wave = pf_wave();
  const int S = a.S;
  const double c = 1.0 / sm.sig[2];
  const bool isd = (lane >= 2 && lane < 2 + S);
  double *ws = a.ws + (size_t)blockIdx.x * 3 * a.Tp;
  n_newton = 0;
  bool cert = false;
  bool need_h = true;
  int lag = 0;
  double dec_prev = 0.0;
  bool zero = false;    // QP active set (wave 0, lane = parameter)
  double sgn_ = 0.0;
  for (int it = 0; it < a.o.polish_max_iter; ++it) {
    const double gh = isd ? g - c * (double)((x > 0.0) - (x < 0.0)) : g;
    const bool fresh = need_h;
    if (fresh) {
      PF_STAMP(20);
      hessian_collective<NW, KMAX, O0, O1, O2, MODE>(a, sm, x, gh, ws);
      __syncthreads();
      PF_STAMP(21);
      sweep_in_free<NW, KMAX, MODE>(a, sm, gh, c);
      PF_STAMP(24);
    }
    PF_STAMP(19);
    if (wave == 0) {
      double z;
      int ns = 0;
      const bool ok = qp_active<NW, KMAX, MODE>(a, sm, x, gh, c, z, ns, zero, sgn_, !fresh);
      PF_STAMP(22);
      const double d = (lane < a.P) ? z - x : 0.0;
      double dec = wave_sum(gh * d);
      const double l1 = wave_sum(isd ? fabs(z) - fabs(x) : 0.0);
      dec += c * l1;
      sm.pd[lane] = d;
      if (lane == 0) { sm.fout[2] = ok ? dec : 0.0; sm.fout[3] = ok ? 1.0 : 0.0; }
    }
    __syncthreads();
    const double dec = sm.fout[2];
    const bool qp_ok = sm.fout[3] != 0.0;
    const double d = sm.pd[lane];
    __syncthreads();
    if (!fresh && (!qp_ok || !(fabs(dec) < 1e-2 * fabs(dec_prev)))) {
      // warm QP failed or the lagged model stopped converging fast:
      // recompute the Hessian at the same point
      need_h = true;
      lag = 0;
      continue;
    }
    if (!(dec < -1e-15 * fabs(f))) {
      cert = qp_ok && dec == dec;
      break;
    }
    ++n_newton;
    PF_COUNT(18);
    PF_STAMP(16);
    double alpha = 1.0, fn = 0.0, gn = 0.0, xn = x;
    bool acc = false;
    for (int ls = 0; ls < 30; ++ls) {
      xn = x + alpha * d;
      const bool bad = eval_collective1<NW, KMAX, O0, O1, O2, MODE>(a, sm, xn, fn, gn);
      ++n_eval;
      if (!bad && fn <= f + 1e-4 * alpha * dec) { acc = true; break; }
      alpha *= 0.5;
    }
    PF_STAMP(17);
    if (!acc) break;
    x = xn;
    f = fn;
    g = gn;
    need_h = !(alpha == 1.0 && lag < PF_POLISH_MAXLAG);
    lag = need_h ? 0 : lag + 1;
    dec_prev = dec;
  }
  return cert;
}
