// pf_tile.h — K3T: tiled batched Stan L-BFGS, 16 series per workgroup.
//
// The throughput form of K3 (north_star (2)/(3)):
// a workgroup owns a tile of PF_TS = 16 series that share one date grid.
// Every objective evaluation evaluates all 16 series at their own trial
// points at once, and the seasonal contractions are dense GEMMs on the FP64
// matrix cores:
//   X[T x K] . B[K x 16]  (B = beta o s_m per series)       -> Xb, C layout
//   X'[K x T] . W[T x 16] (W = r o trend per series)        -> beta gradient
// both v_mfma_f64_16x16x4f64 over 16-row chunks (the C layout's rows are
// the second product's k index, so the elementwise results feed it from
// registers).  The changepoint contraction A[T x C] . Delta[C x 16] is a
// step matrix: the trend reads per-series segment tables (k_s, m_s) — the
// exact contraction at O(1) per element — and its adjoint is a segment sum
// per series.  Residuals, likelihood and prior terms are elementwise in the
// C layout.
//
// Growth: linear / flat (trend k_s t + m_s; adjoint sums of G = r(1 + Xb_m)
// and G t), and logistic (trend cap sigma(k_s (t - m_s)), the offsets m_s by
// UPSTREAM logistic_gamma's recursion in the publish step; adjoint sums of
// -a k_s and a (t - m_s), a = G cap sigma (1 - sigma), then the reverse mode
// through logistic_gamma in the assemble step — the oracle's order,
// orc_objective).  Layouts: features padded to KP = 32 or 48 (K <= 48:
// yearly + weekly (+ daily) + holiday columns); parameters p = g + 16 i in
// lane g of the series' 16 lanes, NP = 4 (P <= 64) or 5 (wide, P <= 72).
//
// Row pass: each wave takes a contiguous quarter of the 16-row chunks,
// software-pipelined — the Xb MFMAs of chunk c+1 are issued before chunk c's
// elementwise VALU work, and global loads run two chunks ahead (one wave per
// SIMD: nothing else hides L2 / HBM latency).
//
// Reproducibility: every LDS accumulator has exactly one writer wave.
// Segment sums go to per-wave slots (wave w adds segment s at slot s + w;
// the waves' segment ranges are contiguous and ordered, so the slots are
// disjoint) — LDS adds of one wave to its own addresses apply in program
// order —, the beta gradient and residual sums to per-wave slots, and the
// assemble step adds the slots in a fixed order: a tile's iterates are
// bitwise identical run to run.
//
// L-BFGS: every series owns 16 lanes (4 series per wave, all 4 waves busy)
// running Stan 2.19's BFGSMinimizer<LBFGSUpdate> + Wolfe line search (same
// control flow as oracle/stan_lbfgs.c, two-loop recursion), with per-series
// convergence masking: a series that terminates stops moving and the tile
// exits when all 16 have.  The iterate, gradient and direction stay in the
// lanes' registers across evaluations; the trial point, history and scalar
// state live in LDS.
//
// Scope: P <= 72, K <= 48, S + 1 <= 32, shared prior scales; the
// per-series kernel K3 covers the rest.  The exact-MAP polish runs after it
// (k_polish, one workgroup per series).
#pragma once

#define PF_TS 16   // series per tile (MFMA N)
#define PF_TNW 4   // waves per tile workgroup (one per SIMD; 8 waves, two per SIMD, measured
                   // no faster: the row pass is bound by the SIMD's FP64 pipe, shared by
                   // MFMA and VALU, and the register cap of two waves spills the step)
#define PF_TH 5    // L-BFGS history (Stan default)
#define PF_TSEG 33 // per-series stride of the segment tables (odd: conflict-free LDS reads)
#define PF_TSLOT 36  // segment-sum slots: segment s of wave w at s + w (S + 1 <= 32)

template <int MODE, int KP_>
struct TileTr {
  static constexpr bool LOGI = (MODE & PF_MODE_LOGI) != 0;
  static constexpr bool WIDE = (MODE & PF_MODE_WIDE) != 0;
  static constexpr bool HM = (MODE & 3) != MODE_ADD, HA = (MODE & 3) != MODE_MULT;
  static constexpr int NSET = ((MODE & 3) == MODE_MIXED) ? 2 : 1;
  static constexpr int KP = KP_;          // padded feature count (32 or 48)
  static constexpr int NKS = KP / 4;      // Xb k-steps
  static constexpr int NFT = KP / 16;     // X'W output tiles
  static constexpr int NP = WIDE ? 5 : 4; // parameters per lane (p = g + 16 i)
  static constexpr int TV = WIDE ? 72 : 64;  // LDS stride of a parameter vector (P <= TV)
  static_assert(KP == 32 || KP == 48, "KP");
};

struct TileZ {
  double fk, fk1, fq, gpq, alpha, alphak_1, dfp, c1dfp, c2dfp, alpha0, alpha1, prevF, prevDFp;
  double alo, aloF, aloDFp, ahi, ahiF, ahiDFp, lastDFp, dfp_prev, gammak;
  int state, itNum, resetB, nits, lsRestarts, zit, hcount, head, ret, n_eval, bad, done;
};

template <int MODE, int KP>
struct TileSmem {
  using Tr = TileTr<MODE, KP>;
  static constexpr int TV = Tr::TV;
  double *xq;                    // [16][TV] trial points
  double *hs, *hy;               // [H][16][TV]
  double *hrho;                  // [16][H]
  double *kseg, *mseg;           // [16][PF_TSEG]
  double *bm, *ba;               // [KP][16] (ba only with additive terms)
  double *gb;                    // [4 waves][NSET][KP][16] beta-gradient partials
  double *sg0, *sg1;             // [PF_TSLOT][16] per-wave segment-sum slots
  double *rr;                    // [4 waves][16]
  double *sig;                   // [16][2] sigma, 1/sigma^2
  double *ctc, *csg, *csm, *csa; // [64]
  TileZ *z;                      // [16]
  int *flag;                     // [4]
  int *wseg;                     // [2][4] first / last segment of each wave's rows
  int *sidx;                     // [16] series of each slot (-1: retired)
  static constexpr size_t bytes() {
    const size_t vec = (size_t)PF_TS * TV;
    const size_t d = (1 + 2 * PF_TH) * vec + PF_TS * PF_TH + 2 * PF_TS * PF_TSEG +
                     (Tr::HA ? 2 : 1) * KP * PF_TS + 4 * Tr::NSET * KP * PF_TS +
                     2 * PF_TSLOT * PF_TS + 4 * PF_TS + 2 * PF_TS + 4 * 64;
    return d * sizeof(double) + PF_TS * sizeof(TileZ) + (4 + 8 + PF_TS) * sizeof(int) + 64;
  }
  __device__ void carve(char *base) {
    double *p = reinterpret_cast<double *>(base);
    constexpr size_t vec = (size_t)PF_TS * TV;
    xq = p; p += vec;
    hs = p; p += PF_TH * vec;
    hy = p; p += PF_TH * vec;
    hrho = p; p += PF_TS * PF_TH;
    kseg = p; p += PF_TS * PF_TSEG;
    mseg = p; p += PF_TS * PF_TSEG;
    bm = p; p += KP * PF_TS;
    ba = Tr::HA ? p : bm;
    if (Tr::HA) p += KP * PF_TS;
    gb = p; p += 4 * Tr::NSET * KP * PF_TS;
    sg0 = p; p += PF_TSLOT * PF_TS;
    sg1 = p; p += PF_TSLOT * PF_TS;
    rr = p; p += 4 * PF_TS;
    sig = p; p += 2 * PF_TS;
    ctc = p; p += 64;
    csg = p; p += 64;
    csm = p; p += 64;
    csa = p; p += 64;
    z = reinterpret_cast<TileZ *>(p);
    flag = reinterpret_cast<int *>(z + PF_TS);
    wseg = flag + 4;
    sidx = wseg + 8;
  }
};

// sum over the 16 lanes of a series group (bitwise uniform within the group:
// each butterfly stage adds the same two partial sums in both lanes)
__device__ __forceinline__ double grp_sum(double v) {
  v += shfl_xor_f64<1>(v);
  v += shfl_xor_f64<2>(v);
  v += shfl_xor_f64<4>(v);
  v += shfl_xor_f64<8>(v);
  return v;
}

// DPP row (16-lane) scans, zero fill at the row edge: inclusive prefix
// (lane g: sum over g' <= g) and inclusive suffix (sum over g' >= g)
#define PF_DPP_ROWBCAST(n) (0x150 + (n))  // row_newbcast: lane n of each row
__device__ __forceinline__ double row_prefix(double v) {
  v += dpp_f64<PF_DPP_SHR(1)>(v);
  v += dpp_f64<PF_DPP_SHR(2)>(v);
  v += dpp_f64<PF_DPP_SHR(4)>(v);
  v += dpp_f64<PF_DPP_SHR(8)>(v);
  return v;
}
__device__ __forceinline__ double row_suffix(double v) {
  v += dpp_f64<PF_DPP_SHL(1)>(v);
  v += dpp_f64<PF_DPP_SHL(2)>(v);
  v += dpp_f64<PF_DPP_SHL(4)>(v);
  v += dpp_f64<PF_DPP_SHL(8)>(v);
  return v;
}
// value of segment / changepoint I (compile time) of this series: held in
// lane I of the a-half (I < 16) or lane I - 16 of the b-half
template <int I>
__device__ __forceinline__ double row_bcast2(double va, double vb) {
  return dpp_f64<PF_DPP_ROWBCAST(I & 15)>(I < 16 ? va : vb);
}

template <int NP>
struct TVec {
  double v[NP];
  __device__ __forceinline__ double &operator[](int i) { return v[i]; }
  __device__ __forceinline__ double operator[](int i) const { return v[i]; }
};

template <int NP>
__device__ __forceinline__ double tvdot(const TVec<NP> &u, const TVec<NP> &v) {
  double s = 0.0;
  if constexpr (NP == 4) {
    s = fma(u[0], v[0], u[1] * v[1]) + fma(u[2], v[2], u[3] * v[3]);
  } else {
    s = (fma(u[0], v[0], u[1] * v[1]) + fma(u[2], v[2], u[3] * v[3])) + u[4] * v[4];
  }
  return grp_sum(s);
}
// LDS vector <-> registers; entries past P read as 0
template <int NP>
__device__ __forceinline__ void tvload(TVec<NP> &r, const double *v, int P, int g) {
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int p = g + 16 * i;
    r[i] = (p < P) ? v[p] : 0.0;
  }
}
template <int NP>
__device__ __forceinline__ void tvstore(double *v, const TVec<NP> &r, int P, int g) {
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int p = g + 16 * i;
    if (p < P) v[p] = r[i];
  }
}

// Publish series j's trial point xq: segment tables, beta o s_m / s_a, sigma
// (the 16 lanes of series j; g = lane & 15).
template <int MODE, int KP>
__device__ __forceinline__ void tile_publish(const FitKArgs &a, TileSmem<MODE, KP> &sm, int j, int g) {
  using Tr = TileTr<MODE, KP>;
  constexpr int TV = Tr::TV;
  const int S = a.S, K = a.K;
  const double *x = sm.xq + (size_t)j * TV;
  // segment tables k_s = k + sum_{c < s} delta_c (lane g: segments g + 1 and
  // g + 17 by a row-parallel inclusive prefix; the 16 lanes of series j are
  // one DPP row).  Linear: m_s = m - sum_{c < s} t_c delta_c.  Logistic:
  // m_s by UPSTREAM logistic_gamma.  Flat: k = 0, trend = m.
  const bool lin = a.growth == PF_GROWTH_LINEAR || Tr::LOGI;
  const double k = lin ? x[0] : 0.0, m = x[1];
  const double da = (lin && g < S) ? x[2 + g] : 0.0, db = (lin && g + 16 < S) ? x[18 + g] : 0.0;
  double pa = row_prefix(da);
  const double pb = row_prefix(db) + dpp_f64<PF_DPP_ROWBCAST(15)>(pa);
  const double ka1 = k + pa, kb1 = k + pb;   // k_{g+1}, k_{g+17}
  if (g == 0) {
    sm.kseg[j * PF_TSEG] = k;
    sm.mseg[j * PF_TSEG] = m;
  }
  if (g < S) sm.kseg[j * PF_TSEG + g + 1] = ka1;
  if (g + 16 < S) sm.kseg[j * PF_TSEG + g + 17] = kb1;
  if constexpr (Tr::LOGI) {
    // m_0 = m, m_{s+1} = m_s + (t_s - m_s)(1 - k_s / k_{s+1}): the ratios
    // lane-parallel (changepoints g, g + 16), the chain uniform per series
    const double kb0 = dpp_f64<PF_DPP_ROWBCAST(15)>(ka1);            // k_16
    double ka0 = dpp_f64<PF_DPP_SHR(1)>(ka1);                         // k_g (g >= 1)
    double kbp = dpp_f64<PF_DPP_SHR(1)>(kb1);                         // k_{g+16} (g >= 1)
    if (g == 0) { ka0 = k; kbp = kb0; }
    const double ra = (g < S) ? ka0 / ka1 : 0.0, rb = (g + 16 < S) ? kbp / kb1 : 0.0;
    const double tca = sm.ctc[g], tcb = sm.ctc[g + 16];
    double mcur = m, mla = 0.0, mlb = 0.0;
#define PF_LG_STEP(I)                                                           \
    if (I < S) {                                                                \
      const double ri = row_bcast2<I>(ra, rb), ti = row_bcast2<I>(tca, tcb);    \
      mcur = mcur + (ti - mcur) * (1.0 - ri);                                   \
      if ((I & 15) == g) { if (I < 16) mla = mcur; else mlb = mcur; }           \
    }
    PF_LG_STEP(0) PF_LG_STEP(1) PF_LG_STEP(2) PF_LG_STEP(3) PF_LG_STEP(4) PF_LG_STEP(5)
    PF_LG_STEP(6) PF_LG_STEP(7) PF_LG_STEP(8) PF_LG_STEP(9) PF_LG_STEP(10) PF_LG_STEP(11)
    PF_LG_STEP(12) PF_LG_STEP(13) PF_LG_STEP(14) PF_LG_STEP(15) PF_LG_STEP(16) PF_LG_STEP(17)
    PF_LG_STEP(18) PF_LG_STEP(19) PF_LG_STEP(20) PF_LG_STEP(21) PF_LG_STEP(22) PF_LG_STEP(23)
    PF_LG_STEP(24) PF_LG_STEP(25) PF_LG_STEP(26) PF_LG_STEP(27) PF_LG_STEP(28) PF_LG_STEP(29)
    PF_LG_STEP(30)
#undef PF_LG_STEP
    if (g < S) sm.mseg[j * PF_TSEG + g + 1] = mla;
    if (g + 16 < S) sm.mseg[j * PF_TSEG + g + 17] = mlb;
  } else {
    const double qa = row_prefix(sm.ctc[g] * da);
    const double qb = row_prefix(sm.ctc[g + 16] * db) + dpp_f64<PF_DPP_ROWBCAST(15)>(qa);
    if (g < S) sm.mseg[j * PF_TSEG + g + 1] = m - qa;
    if (g + 16 < S) sm.mseg[j * PF_TSEG + g + 17] = m - qb;
  }
  if (g == 1) {
    const double sg = exp(x[2 + S]);
    sm.sig[2 * j] = sg;
    sm.sig[2 * j + 1] = 1.0 / (sg * sg);
  }
#pragma unroll
  for (int h = 0; h < Tr::NFT; ++h) {
    const int f = g + 16 * h;
    const double bv = (f < K) ? x[3 + S + f] : 0.0;
    sm.bm[f * PF_TS + j] = bv * sm.csm[f];
    if constexpr (Tr::HA) sm.ba[f * PF_TS + j] = bv * sm.csa[f];
  }
}

typedef double pf_d2 __attribute__((ext_vector_type(2)));
typedef int pf_i4 __attribute__((ext_vector_type(4)));

// Row mapping inside a 16-row chunk: C-layout row i (lane (j, rq) register
// rg holds C-row rq + 4 rg) is data row r0 + 4 (i & 3) + (i >> 2), so each
// lane's four rows are contiguous (t, y, cap, seg in two / one wide loads)
// and k-step q of X'W covers data rows r0 + 4 rq + q.  Feature maps (row-
// major copy XR, row stride KP): Xb k-step kk < 8 at lane k index rq <->
// feature 8 rq + kk, kk >= 8 <-> 32 + 4 rq + kk - 8; X'W tiles 0/1: output
// row i <-> feature 2 i + ft, tile 2: 32 + i (all contiguous per lane).
template <bool LOGI, int KP>
struct TileIn {
  pf_d2 xa[KP / 8];  // X[r0 + 4 (j & 3) + (j >> 2)][Xb k-step features]
  pf_d2 xg[4];       // X[r0 + 4 rq + q][2 j .. 2 j + 1]     (X'W k-step q, tiles 0/1)
  double xg2[KP == 48 ? 4 : 1];  // X[r0 + 4 rq + q][32 + j]  (tile 2)
  pf_d2 t[2], y[2];  // data rows r0 + 4 rq + rg
  pf_d2 cp[LOGI ? 2 : 1];
  pf_i4 sg;
};

// Row pass of one evaluation (all waves): each wave leaves its beta-gradient
// partials, segment sums and residual sums of squares in its LDS slots
// (gb[wave], sg0/sg1 at segment + wave, rr[wave]); the segment slots were
// zeroed by the caller.
template <int MODE, int KP>
__device__ __forceinline__ void tile_rows(const FitKArgs &a, TileSmem<MODE, KP> &sm) {
  using Tr = TileTr<MODE, KP>;
  constexpr int NSET = Tr::NSET, NKS = Tr::NKS, NFT = Tr::NFT;
  constexpr bool HM = Tr::HM, HA = Tr::HA, LOGI = Tr::LOGI;
  const int lane = pf_lane(), wave = __builtin_amdgcn_readfirstlane(pf_wave());
  const int T = a.T, Tp = a.Tp;
  const int j = lane & 15, rq = lane >> 4;
  const int s_g = sm.sidx[j];          // this slot's series (-1: empty slot)
  const bool svalid = s_g >= 0;
  const double *kseg = sm.kseg + j * PF_TSEG, *mseg = sm.mseg + j * PF_TSEG;
  const int jrow = 4 * (j & 3) + (j >> 2);
  // feature of Xb k-step kk at lane k index rq
  auto xb_feat = [&](int kk) { return kk < 8 ? 8 * rq + kk : 32 + 4 * rq + (kk - 8); };
  double bmr[NKS], bar_[NKS];
#pragma unroll
  for (int kk = 0; kk < NKS; ++kk) {
    bmr[kk] = HM ? sm.bm[xb_feat(kk) * PF_TS + j] : 0.0;
    bar_[kk] = HA ? sm.ba[xb_feat(kk) * PF_TS + j] : 0.0;
  }
  // Chunk loads as buffer loads: lane-constant byte offsets (voffset) plus
  // the chunk's uniform offset (soffset), no per-load address arithmetic;
  // unconditional (T_pad % 128 == 0 keeps every chunk row in range, XR is
  // zero past K, rows of series past n read 0 from the y buffer's range
  // check), so no predicated load drains the prefetch.
  const __amdgpu_buffer_rsrc_t rXR = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double *>(a.XR), (short)0, Tp * KP * 8, 0x00020000);
  const __amdgpu_buffer_rsrc_t rT = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double *>(a.t), (short)0, Tp * 8, 0x00020000);
  const __amdgpu_buffer_rsrc_t rS = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<int32_t *>(a.seg), (short)0, Tp * 4, 0x00020000);
  // y / cap rows of the slot's series (any series of the batch; an empty
  // slot reads series 0 and masks it)
  const size_t srow = (size_t)(svalid ? s_g : 0) * Tp + 4 * rq;
  const pf_d2 *yb = reinterpret_cast<const pf_d2 *>(a.y_scaled + srow);
  const pf_d2 *cb = reinterpret_cast<const pf_d2 *>((LOGI ? a.cap_scaled : a.y_scaled) + srow);
  const int oxa = (jrow * KP + 8 * rq) * 8, oxa2 = (jrow * KP + 32 + 4 * rq) * 8;
  const int oxg = (4 * rq * KP + 2 * j) * 8, oxg2 = (4 * rq * KP + 32 + j) * 8;
  const int ot = 4 * rq * 8, os = 4 * rq * 4;
  auto ld2 = [](__amdgpu_buffer_rsrc_t r, int vo, int so) {
    return __builtin_bit_cast(pf_d2, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0));
  };
  auto tload = [&](int c, TileIn<LOGI, KP> &in) {
    const int r0 = 16 * c;
#pragma unroll
    for (int h = 0; h < 4; ++h) in.xa[h] = ld2(rXR, oxa + 16 * h, r0 * KP * 8);
    if constexpr (KP == 48) {
      in.xa[4] = ld2(rXR, oxa2, r0 * KP * 8);
      in.xa[5] = ld2(rXR, oxa2 + 16, r0 * KP * 8);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) in.xg[q] = ld2(rXR, oxg + KP * 8 * q, r0 * KP * 8);
    if constexpr (KP == 48) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        in.xg2[q] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                                    rXR, oxg2 + KP * 8 * q, r0 * KP * 8, 0));
    }
    in.t[0] = ld2(rT, ot, r0 * 8);
    in.t[1] = ld2(rT, ot + 16, r0 * 8);
    in.y[0] = yb[r0 / 2];
    in.y[1] = yb[r0 / 2 + 1];
    if constexpr (LOGI) {
      in.cp[0] = cb[r0 / 2];
      in.cp[1] = cb[r0 / 2 + 1];
    }
    in.sg = __builtin_bit_cast(pf_i4, __builtin_amdgcn_raw_buffer_load_b128(rS, os, r0 * 4, 0));
  };
  auto xb_mfma = [&](const TileIn<LOGI, KP> &in, pf_d4 &xm, pf_d4 &xa) {
    // two independent accumulation chains per product (even / odd k-steps)
    pf_d4 m0 = pf_d4{0.0, 0.0, 0.0, 0.0}, m1 = m0, a0_ = m0, a1_ = m0;
#pragma unroll
    for (int h = 0; h < NKS / 2; ++h) {
      if constexpr (HM) {
        m0 = __builtin_amdgcn_mfma_f64_16x16x4f64(in.xa[h][0], bmr[2 * h], m0, 0, 0, 0);
        m1 = __builtin_amdgcn_mfma_f64_16x16x4f64(in.xa[h][1], bmr[2 * h + 1], m1, 0, 0, 0);
      }
      if constexpr (HA) {
        a0_ = __builtin_amdgcn_mfma_f64_16x16x4f64(in.xa[h][0], bar_[2 * h], a0_, 0, 0, 0);
        a1_ = __builtin_amdgcn_mfma_f64_16x16x4f64(in.xa[h][1], bar_[2 * h + 1], a1_, 0, 0, 0);
      }
    }
    xm = m0 + m1;
    xa = a0_ + a1_;
  };
  pf_d4 gbm[NFT], gba[NFT];
#pragma unroll
  for (int ft = 0; ft < NFT; ++ft) { gbm[ft] = pf_d4{0.0, 0.0, 0.0, 0.0}; gba[ft] = gbm[ft]; }
  double rr = 0.0, a0 = 0.0, a1 = 0.0;
  int cur = -1;
  double *sl0 = sm.sg0 + wave * PF_TS + j, *sl1 = sm.sg1 + wave * PF_TS + j;  // slot s + wave
  // running sums of the current segment -> its slot (this wave is the only
  // writer of slots s + wave, so its LDS adds — no return value, no wait —
  // apply in program order; lane rq = 0 adds)
  auto flush = [&]() {
    double b0 = a0 + shfl_xor_f64<16>(a0), b1 = a1 + shfl_xor_f64<16>(a1);
    b0 += shfl_xor_f64<32>(b0);
    b1 += shfl_xor_f64<32>(b1);
    if (rq == 0) {
      atomicAdd(&sl0[cur * PF_TS], b0);
      atomicAdd(&sl1[cur * PF_TS], b1);
    }
  };
  const int nch = (T + 15) >> 4;
  const int c0 = (nch * wave) / PF_TNW, c1 = (nch * (wave + 1)) / PF_TNW;
  // one chunk: loads of chunk c + 2 into `nn`, Xb of chunk c + 1 (`nx`)
  // issued before chunk c's (`cu`, Xb in `xc`) elementwise work and X'W.
  // Input and Xb buffers rotate three ways: no register copies of in-flight
  // loads or MFMA results.  (A four-buffer ring, loads three chunks ahead,
  // measured no faster.)
  auto step = [&](int c, const TileIn<LOGI, KP> &cu, const TileIn<LOGI, KP> &nx, TileIn<LOGI, KP> &nn,
                  const pf_d4 &xcm, const pf_d4 &xca, pf_d4 &xnm, pf_d4 &xna) {
    const int r0 = 16 * c;
    const int rbase = r0 + 4 * rq;
    // trend from the per-series segment tables; reads issued before the Xb
    // MFMAs of the next chunk
    double ks[4], ms[4];
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      ks[rg] = kseg[cu.sg[rg]];
      ms[rg] = mseg[cu.sg[rg]];
    }
    tload(min(c + 2, c1 - 1), nn);
    xb_mfma(nx, xnm, xna);
    // chunk-uniform segment (all valid rows in one segment): register sums
    const int s0 = __builtin_amdgcn_readfirstlane(cu.sg[0]);
    const bool same = (cu.sg[0] == s0 || rbase >= T) && (cu.sg[1] == s0 || rbase + 1 >= T) &&
                      (cu.sg[2] == s0 || rbase + 2 >= T) && (cu.sg[3] == s0 || rbase + 3 >= T);
    const bool uni = __ballot(!same) == 0ull;
    double W[4], Wa[4], A0[4], A1[4];
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      const int row = rbase + rg;
      const bool v = svalid && row < T;
      const double ti = cu.t[rg >> 1][rg & 1];
      double tr, capi = 0.0, lgs = 0.0;
      if constexpr (LOGI) {
        capi = cu.cp[rg >> 1][rg & 1];
        lgs = 1.0 / (1.0 + exp(-(ks[rg] * (ti - ms[rg]))));
        tr = capi * lgs;
      } else {
        tr = fma(ks[rg], ti, ms[rg]);
      }
      const double u = 1.0 + (HM ? xcm[rg] : 0.0);
      const double mu = fma(tr, u, HA ? xca[rg] : 0.0);
      const double r = v ? cu.y[rg >> 1][rg & 1] - mu : 0.0;
      rr = fma(r, r, rr);
      W[rg] = r * tr;
      Wa[rg] = r;
      const double G = r * u;
      if constexpr (LOGI) {
        // oracle PM / PK terms: -a k_s, a (t - m_s), a = G cap sigma (1 - sigma)
        const double aa = G * capi * lgs * (1.0 - lgs);
        A0[rg] = -aa * ks[rg];
        A1[rg] = aa * (ti - ms[rg]);
      } else {
        A0[rg] = G;
        A1[rg] = G * ti;
      }
    }
    // beta gradient X'[K x 16 rows] . W[16 rows x 16]: k-step q is register q
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int ft = 0; ft < 2; ++ft) {
        if constexpr (HM) gbm[ft] = __builtin_amdgcn_mfma_f64_16x16x4f64(cu.xg[q][ft], W[q], gbm[ft], 0, 0, 0);
        if constexpr (HA) gba[ft] = __builtin_amdgcn_mfma_f64_16x16x4f64(cu.xg[q][ft], Wa[q], gba[ft], 0, 0, 0);
      }
      if constexpr (NFT == 3) {
        if constexpr (HM) gbm[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(cu.xg2[q], W[q], gbm[2], 0, 0, 0);
        if constexpr (HA) gba[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(cu.xg2[q], Wa[q], gba[2], 0, 0, 0);
      }
    }
    // changepoint adjoint: segment sums per series
    if (uni) {
      if (s0 != cur) {
        if (cur >= 0) flush();
        cur = s0;
        a0 = 0.0;
        a1 = 0.0;
      }
      a0 += (A0[0] + A0[1]) + (A0[2] + A0[3]);
      a1 += (A1[0] + A1[1]) + (A1[2] + A1[3]);
    } else {
      // a chunk across segment boundaries (at most one per changepoint):
      // per-row adds into this wave's slots (a wave's LDS adds apply in
      // instruction order, and the lanes of one add in lane order)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        if (rbase + rg < T) {
          atomicAdd(&sl0[cu.sg[rg] * PF_TS], A0[rg]);
          atomicAdd(&sl1[cu.sg[rg] * PF_TS], A1[rg]);
        }
      }
    }
  };
  if (c0 < c1) {
    TileIn<LOGI, KP> A, B, C;
    pf_d4 XAm, XAa, XBm, XBa, XCm, XCa;
    tload(c0, A);
    tload(min(c0 + 1, c1 - 1), B);
    xb_mfma(A, XAm, XAa);
    for (int c = c0; c < c1; c += 3) {
      step(c, A, B, C, XAm, XAa, XBm, XBa);
      if (c + 1 < c1) step(c + 1, B, C, A, XBm, XBa, XCm, XCa);
      if (c + 2 < c1) step(c + 2, C, A, B, XCm, XCa, XAm, XAa);
    }
  }
  if (cur >= 0) flush();
  rr += shfl_xor_f64<16>(rr);
  rr += shfl_xor_f64<32>(rr);
  if (rq == 0) sm.rr[wave * PF_TS + j] = rr;
  // gradient tiles: C[row i = rq + 4 rg][series j] of tile ft is feature
  // 2 i + ft (ft < 2) or 32 + i (ft = 2), stored into this wave's slot
  double *gsl = sm.gb + wave * (NSET * KP * PF_TS);
#pragma unroll
  for (int ft = 0; ft < NFT; ++ft)
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      const int i = rq + 4 * rg;
      const int f = ft < 2 ? 2 * i + ft : 32 + i;
      if constexpr (HM) gsl[f * PF_TS + j] = gbm[ft][rg];
      if constexpr (HA) gsl[(NSET - 1) * KP * PF_TS + f * PF_TS + j] = gba[ft][rg];
    }
}

// f and g of series j at xq (lane g: parameters g + 16 i -> gq), gpq =
// g . pk.  Returns true if not finite (group-uniform).
template <int MODE, int KP>
__device__ __forceinline__ bool tile_assemble(const FitKArgs &a, TileSmem<MODE, KP> &sm, int j, int g,
                                              const TVec<TileTr<MODE, KP>::NP> &pk,
                                              TVec<TileTr<MODE, KP>::NP> &gq, double &f, double &gpq) {
  using Tr = TileTr<MODE, KP>;
  constexpr int NSET = Tr::NSET, NP = Tr::NP;
  const int S = a.S, P = a.P, T = a.T;
  const bool linear = a.growth == PF_GROWTH_LINEAR;
  const double *x = sm.xq + (size_t)j * Tr::TV;
  const double sigma = sm.sig[2 * j], inv = sm.sig[2 * j + 1], tau = a.tau;
  const double rrt = (sm.rr[j] + sm.rr[PF_TS + j]) + (sm.rr[2 * PF_TS + j] + sm.rr[3 * PF_TS + j]);
  // segment totals, lane g: segments g and g + 16 (S + 1 <= 32), from the
  // per-wave slots in wave order (wave w holds segment s at slot s + w when
  // s is in its row range)
  auto seg_total = [&](const double *slot, int s) {
    double v = 0.0;
#pragma unroll
    for (int w = 0; w < PF_TNW; ++w)
      if (s >= sm.wseg[w] && s <= sm.wseg[4 + w]) v += slot[(s + w) * PF_TS + j];
    return v;
  };
  const double s0a = (g <= S) ? seg_total(sm.sg0, g) : 0.0;
  const double s1a = (g <= S) ? seg_total(sm.sg1, g) : 0.0;
  const double s0b = (g + 16 <= S) ? seg_total(sm.sg0, g + 16) : 0.0;
  const double s1b = (g + 16 <= S) ? seg_total(sm.sg1, g + 16) : 0.0;
  // per-segment values whose suffix sums give the changepoint gradients
  // (changepoint jj is active in the segments s > jj): linear G, G t;
  // logistic: PK after the reverse mode through logistic_gamma
  double v0a = s0a, v1a = s1a, v0b = s0b, v1b = s1b, gm_log = 0.0;
  if constexpr (Tr::LOGI) {
    // PMt = PM_S; for i = S-1..0: bar_i = PMt, PMt = PM_i + bar_i - bar_i (1 - rho_i)
    const double kA = sm.kseg[j * PF_TSEG + g], kA1 = sm.kseg[j * PF_TSEG + g + 1];
    const double kB = sm.kseg[j * PF_TSEG + g + 16], kB1 = sm.kseg[j * PF_TSEG + g + 17];
    const double rA = (g < S) ? kA / kA1 : 0.0, rB = (g + 16 < S) ? kB / kB1 : 0.0;
    double PMt = 0.0, barA = 0.0, barB = 0.0;
#define PF_LG_BACK(I)                                                           \
    {                                                                           \
      const double pmi = row_bcast2<I>(s0a, s0b);                               \
      if (I == S) PMt = pmi;                                                    \
      if (I < S) {                                                              \
        const double ri = row_bcast2<I>(rA, rB);                                \
        const double bar = PMt;                                                 \
        if ((I & 15) == g) { if (I < 16) barA = bar; else barB = bar; }         \
        PMt = pmi + bar;                                                        \
        PMt += bar * (-(1.0 - ri));                                             \
      }                                                                         \
    }
    PF_LG_BACK(31) PF_LG_BACK(30) PF_LG_BACK(29) PF_LG_BACK(28) PF_LG_BACK(27) PF_LG_BACK(26)
    PF_LG_BACK(25) PF_LG_BACK(24) PF_LG_BACK(23) PF_LG_BACK(22) PF_LG_BACK(21) PF_LG_BACK(20)
    PF_LG_BACK(19) PF_LG_BACK(18) PF_LG_BACK(17) PF_LG_BACK(16) PF_LG_BACK(15) PF_LG_BACK(14)
    PF_LG_BACK(13) PF_LG_BACK(12) PF_LG_BACK(11) PF_LG_BACK(10) PF_LG_BACK(9) PF_LG_BACK(8)
    PF_LG_BACK(7) PF_LG_BACK(6) PF_LG_BACK(5) PF_LG_BACK(4) PF_LG_BACK(3) PF_LG_BACK(2)
    PF_LG_BACK(1) PF_LG_BACK(0)
#undef PF_LG_BACK
    gm_log = PMt;
    // PK_i += bar_i (-(t_i - m_i) / k_{i+1});  PK_{i+1} += bar_i (t_i - m_i) k_i / k_{i+1}^2
    const double dA = sm.ctc[g] - sm.mseg[j * PF_TSEG + g];
    const double dB = sm.ctc[g + 16] - sm.mseg[j * PF_TSEG + g + 16];
    const double t1a = (g < S) ? barA * (-dA / kA1) : 0.0, t2a = (g < S) ? barA * (dA * kA / (kA1 * kA1)) : 0.0;
    const double t1b = (g + 16 < S) ? barB * (-dB / kB1) : 0.0, t2b = (g + 16 < S) ? barB * (dB * kB / (kB1 * kB1)) : 0.0;
    // (every cross-lane read is issued by all 16 lanes before any select: a
    // DPP inside a ?: operand runs only in the lanes taking that branch and
    // reads 0 from the others)
    const double t2a_prev = dpp_f64<PF_DPP_SHR(1)>(t2a);                       // segment g - 1
    const double t2a_15 = dpp_f64<PF_DPP_ROWBCAST(15)>(t2a), t2b_sh = dpp_f64<PF_DPP_SHR(1)>(t2b);
    const double t2b_prev = (g == 0) ? t2a_15 : t2b_sh;
    v1a = (s1a + t1a) + t2a_prev;
    v1b = (s1b + t1b) + t2b_prev;
  }
  // suffix sums over segments by a DPP row scan; parameter p = 2 + jj needs
  // the suffix at s = p - 1: lane g - 1 of the same half (row_shr:1), or row
  // lane 15 across halves
  const double u0b = row_suffix(v0b), u1b = row_suffix(v1b);
  const double u0a = row_suffix(v0a) + dpp_f64<PF_DPP_ROWBCAST(0)>(u0b);
  const double u1a = row_suffix(v1a) + dpp_f64<PF_DPP_ROWBCAST(0)>(u1b);
  const double tot0 = dpp_f64<PF_DPP_ROWBCAST(0)>(u0a), tot1 = dpp_f64<PF_DPP_ROWBCAST(0)>(u1a);
  double su0[3], su1[3];
  {
    const double h0a = dpp_f64<PF_DPP_SHR(1)>(u0a), h1a = dpp_f64<PF_DPP_SHR(1)>(u1a);
    const double h0b = dpp_f64<PF_DPP_SHR(1)>(u0b), h1b = dpp_f64<PF_DPP_SHR(1)>(u1b);
    const double e0a = dpp_f64<PF_DPP_ROWBCAST(15)>(u0a), e1a = dpp_f64<PF_DPP_ROWBCAST(15)>(u1a);
    su0[0] = h0a;
    su1[0] = h1a;
    su0[1] = g == 0 ? e0a : h0b;
    su1[1] = g == 0 ? e1a : h1b;
    su0[2] = dpp_f64<PF_DPP_ROWBCAST(15)>(u0b);
    su1[2] = dpp_f64<PF_DPP_ROWBCAST(15)>(u1b);
  }
  constexpr int GS = NSET * KP * PF_TS;
  const double *gbw = sm.gb;
  // beta-gradient slots of the four waves, added in wave order
  auto gsum = [&](int off) { return (gbw[off] + gbw[GS + off]) + (gbw[2 * GS + off] + gbw[3 * GS + off]); };
  double fl = 0.0, gp = 0.0;
  bool bad = false;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int p = g + 16 * i;
    double gv = 0.0, ft = 0.0;
    if (p < P) {
      const double xv = x[p];
      if (p == 0) {
        const double gk = Tr::LOGI ? tot1 : (linear ? tot1 : 0.0);
        gv = -inv * gk + xv / 25.0;
        ft = xv * xv / 50.0;
      } else if (p == 1) {
        gv = -inv * (Tr::LOGI ? gm_log : tot0) + xv / 25.0;
        ft = xv * xv / 50.0;
      } else if (p < 2 + S) {
        // changepoint jj is active in segments s > jj
        const int jj = p - 2;
        const int ii = i < 3 ? i : 2;
        const double sgn = (xv > 0.0) - (xv < 0.0);
        double gd = 0.0;
        if constexpr (Tr::LOGI) gd = -inv * su1[ii];
        else gd = linear ? -inv * (su1[ii] - sm.ctc[jj] * su0[ii]) : 0.0;
        gv = gd + sgn / tau;
        ft = fabs(xv) / tau;
      } else if (p == 2 + S) {
        gv = (double)T - inv * rrt + 4.0 * sigma * sigma;
        ft = 2.0 * sigma * sigma + (double)T * xv;
      } else {
        const int f2 = p - 3 - S;
        const double sgm = sm.csg[f2];
        double gl = 0.0;
        if constexpr (Tr::HM) gl += sm.csm[f2] * gsum(f2 * PF_TS + j);
        if constexpr (Tr::HA) gl += sm.csa[f2] * gsum((NSET - 1) * KP * PF_TS + f2 * PF_TS + j);
        gv = -inv * gl + xv / (sgm * sgm);
        ft = xv * xv / (2.0 * sgm * sgm);
      }
      bad |= !isfinite(gv);
    }
    gq[i] = gv;
    fl += ft;
    gp = fma(gv, pk[i], gp);
  }
  f = grp_sum(fl) + 0.5 * rrt * inv;
  gpq = grp_sum(gp);
  bad |= !isfinite(f);
  return grp_sum(bad ? 1.0 : 0.0) != 0.0;
}

// Stan 2.19 BFGSMinimizer<LBFGSUpdate>::step + WolfeLineSearch as a per-series
// state machine (16 lanes): advance until the series needs an evaluation at
// xq (returns true) or terminates (false, z.ret set).  Same control flow as
// lbfgs_step (pf_engine.hip) and oracle/stan_lbfgs.c; the search direction
// by Stan's two-loop recursion.  xk / gk / pk live in the caller's
// registers across evaluations (NP entries per lane).
template <int MODE, int KP>
__device__ __forceinline__ bool tile_lbfgs(const pf_fit_opts &o, TileSmem<MODE, KP> &sm, TileZ &z, int j,
                                           int g, int P, TVec<TileTr<MODE, KP>::NP> &xk,
                                           TVec<TileTr<MODE, KP>::NP> &gk, TVec<TileTr<MODE, KP>::NP> &pk,
                                           const TVec<TileTr<MODE, KP>::NP> &gq) {
  using Tr = TileTr<MODE, KP>;
  constexpr int NP = Tr::NP, TV = Tr::TV;
  using V = TVec<NP>;
  double *xqL = sm.xq + (size_t)j * TV;
  const int H = o.history < PF_TH ? o.history : PF_TH;
  constexpr size_t hstep = (size_t)PF_TS * TV;
  V xq;
  tvload(xq, xqL, P, g);
  bool need = false, run = true;
  while (run) {
    switch (z.state) {
      case LB_INIT:
        if (z.bad) { z.ret = PF_ST_BADINIT; z.state = LB_DONE; run = false; break; }
        z.fk = z.fq;
#pragma unroll
        for (int i = 0; i < NP; ++i) { xk[i] = xq[i]; gk[i] = gq[i]; pk[i] = -gq[i]; }
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
          for (int i = 0; i < NP; ++i) pk[i] = -gk[i];
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
        for (int i = 0; i < NP; ++i) xq[i] = xk[i] + z.alpha1 * pk[i];
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
        for (int i = 0; i < NP; ++i) xq[i] = xk[i] + z.alpha * pk[i];
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
          for (int i = 0; i < NP; ++i) xq[i] = xk[i] + z.alpha * pk[i];
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
        V sk, yk;
#pragma unroll
        for (int i = 0; i < NP; ++i) {
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
          const double rho_new = 1.0 / sy;
          tvstore(sm.hs + slot * hstep + (size_t)j * TV, sk, P, g);
          tvstore(sm.hy + slot * hstep + (size_t)j * TV, yk, P, g);
          if (g == 0) sm.hrho[j * PF_TH + slot] = rho_new;
          if (z.hcount < H) z.hcount++;
          else z.head = pf_wrap(z.head + 1, H);
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int i = 0; i < NP; ++i) pk[i] = -gk[i];
          double al[PF_TH];
#pragma unroll
          for (int c = PF_TH - 1; c >= 0; --c) {
            al[c] = 0.0;
            if (c < z.hcount) {
              const int sl = pf_wrap(z.head + c, H);
              V sv, yv;
              double rho_c;
              if (c == z.hcount - 1) {    // newest pair: still in registers
#pragma unroll
                for (int i = 0; i < NP; ++i) { sv[i] = sk[i]; yv[i] = yk[i]; }
                rho_c = rho_new;
              } else {
                tvload(sv, sm.hs + sl * hstep + (size_t)j * TV, P, g);
                tvload(yv, sm.hy + sl * hstep + (size_t)j * TV, P, g);
                rho_c = sm.hrho[j * PF_TH + sl];
              }
              al[c] = rho_c * tvdot(sv, pk);
#pragma unroll
              for (int i = 0; i < NP; ++i) pk[i] = fma(-al[c], yv[i], pk[i]);
            }
          }
#pragma unroll
          for (int i = 0; i < NP; ++i) pk[i] *= z.gammak;
#pragma unroll
          for (int c = 0; c < PF_TH; ++c) {
            if (c < z.hcount) {
              const int sl = pf_wrap(z.head + c, H);
              V sv, yv;
              double rho_c;
              if (c == z.hcount - 1) {
#pragma unroll
                for (int i = 0; i < NP; ++i) { sv[i] = sk[i]; yv[i] = yk[i]; }
                rho_c = rho_new;
              } else {
                tvload(sv, sm.hs + sl * hstep + (size_t)j * TV, P, g);
                tvload(yv, sm.hy + sl * hstep + (size_t)j * TV, P, g);
                rho_c = sm.hrho[j * PF_TH + sl];
              }
              const double b = rho_c * tvdot(yv, pk);
#pragma unroll
              for (int i = 0; i < NP; ++i) pk[i] = fma(al[c] - b, sv[i], pk[i]);
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
  tvstore(xqL, xq, P, g);
  return need;
}

// Load series idx into slot j (the 16 lanes of the slot's group): theta0
// into the registers and the LDS trial point, a fresh L-BFGS state.  Returns
// false for a constant series (outputs written here: the optimizer is
// skipped, Prophet's rule).
template <int MODE, int KP>
__device__ __forceinline__ bool tile_load_series(const FitKArgs &a, TileSmem<MODE, KP> &sm, int j, int g,
                                                 int idx, TileZ &zl, TVec<TileTr<MODE, KP>::NP> &xk,
                                                 TVec<TileTr<MODE, KP>::NP> &gk,
                                                 TVec<TileTr<MODE, KP>::NP> &pk,
                                                 TVec<TileTr<MODE, KP>::NP> &gq) {
  using Tr = TileTr<MODE, KP>;
  const int P = a.P, S = a.S;
  double *xq = sm.xq + (size_t)j * Tr::TV;
  double *th = a.theta + (size_t)idx * P;
#pragma unroll
  for (int i = 0; i < Tr::NP; ++i) {
    const int p = g + 16 * i;
    const double v = (p < P) ? th[p] : 0.0;
    if (p < Tr::TV) xq[p] = v;
    xk[i] = v;
    gk[i] = 0.0;
    pk[i] = 0.0;
    gq[i] = 0.0;
  }
  memset(&zl, 0, sizeof(TileZ));
  zl.state = LB_INIT;
  if (a.status[idx] == PF_ST_CONSTANT) {
    if (g == 0) {
      th[2 + S] = log(1e-9);
      a.f_out[idx] = NAN;
      a.f_stan[idx] = NAN;
      a.n_iter[idx] = 0;
      a.n_eval[idx] = 0;
    }
    zl.done = 1;
    return false;
  }
  return true;
}

// K3T kernel, persistent: grid = min(tiles, CUs) workgroups of 16 series
// slots.  Slot j of workgroup b starts on series 16 b + j; a slot whose
// series terminates writes that series' outputs and takes the next series
// from the batch's work queue (a global counter, one atomic per refill), so
// a tile no longer waits for the slowest of 16 fixed series — it runs until
// the queue is empty and its last series have finished.  A series computes
// the same arithmetic in any slot (the MFMA columns, segment slots and DPP
// rows are per series), so results do not depend on the schedule.
// Pass-0 semantics of fit_body (theta in: init; out: the L-BFGS endpoint,
// f, f_stan, status, n_iter, n_eval); warm = the iteration cap is the
// warm-up cap (MAXIT -> WARMUP).
// Per evaluation: row pass (all waves) | barrier |
// assemble (16 lanes per series) | barrier | zero segment slots + L-BFGS
// step (+ outputs and refill) + publish | barrier.
template <int MODE, int KP>
__global__ __launch_bounds__(PF_TNW * 64, 1) void k_fit_tile(FitKArgs a, int n) {
  using Tr = TileTr<MODE, KP>;
  constexpr int NP = Tr::NP;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  TileSmem<MODE, KP> sm;
  sm.carve(smem_raw);
  const int lane = pf_lane(), wave = __builtin_amdgcn_readfirstlane(pf_wave());
  const int P = a.P, S = a.S, T = a.T;
  const int j = (4 * wave + (lane >> 4)) & 15, g = lane & 15;  // slot j's 16 lanes
  const bool warm = a.warm_cap != 0;
  const pf_fit_opts o = a.o;
  if (threadIdx.x < 64) {
    const int i = threadIdx.x;
    sm.ctc[i] = (i < S) ? a.t_change[i] : 0.0;
    sm.csg[i] = (i < a.K) ? a.sigmas[i] : 1.0;
    sm.csm[i] = (i < a.K) ? a.s_m[i] : 0.0;
    sm.csa[i] = (i < a.K) ? a.s_a[i] : 0.0;
  }
  if (threadIdx.x < PF_TNW) {
    // segment range of each wave's rows (the same chunk split as tile_rows)
    const int w = threadIdx.x;
    const int nch = (T + 15) >> 4;
    const int c0 = (nch * w) / PF_TNW, c1 = (nch * (w + 1)) / PF_TNW;
    if (c0 < c1) {
      sm.wseg[w] = a.seg[16 * c0];
      sm.wseg[4 + w] = a.seg[min(16 * c1, T) - 1];
    } else {
      sm.wseg[w] = 1;
      sm.wseg[4 + w] = 0;
    }
  }
  for (int e = threadIdx.x; e < 2 * PF_TSLOT * PF_TS; e += PF_TNW * 64) sm.sg0[e] = 0.0;
  TVec<NP> xk, gk, pk, gq;
  // take series from the queue until one needs fitting (or the queue is
  // empty: the slot retires with sidx = -1); group-uniform loop
  auto refill = [&](TileZ &zl, int first) {
    int idx = first;
    while (true) {
      if (idx < 0) {
        int t = 0;
        if (g == 0) t = atomicAdd(a.queue, 1);
        idx = dpp_i32<PF_DPP_ROWBCAST(0)>(t);
      }
      if (idx >= n) {
        memset(&zl, 0, sizeof(TileZ));
        zl.done = 1;
        return -1;
      }
      if (tile_load_series<MODE, KP>(a, sm, j, g, idx, zl, xk, gk, pk, gq)) return idx;
      idx = -1;
    }
  };
  int sidx;
  {
    TileZ zl;
    sidx = refill(zl, (int)blockIdx.x * PF_TS + j);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (g == 0) {
      sm.z[j] = zl;
      sm.sidx[j] = sidx;
    }
  }
  __syncthreads();
  if (sidx < 0) {
    // an empty slot (last tile, n % 16 != 0) still runs the row pass: give
    // it a finite model (k = 1, every other parameter 0; k != 0 keeps the
    // logistic offsets' ratios k_s / k_{s+1} finite) once
    constexpr int TV = TileTr<MODE, KP>::TV;
    for (int p = g; p < TV; p += 16) sm.xq[(size_t)j * TV + p] = (p == 0) ? 1.0 : 0.0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  tile_publish<MODE, KP>(a, sm, j, g);
  __syncthreads();
  {
    const unsigned long long any = __ballot(sidx >= 0);
    if (lane == 0) sm.flag[wave] = any != 0ull ? 1 : 0;
  }
  __syncthreads();
  if (!__builtin_amdgcn_readfirstlane(sm.flag[0] | sm.flag[1] | sm.flag[2] | sm.flag[3])) return;
  while (true) {
    PF_STAMP(0);
    tile_rows<MODE, KP>(a, sm);
    PF_STAMP(1);
    __syncthreads();
    PF_STAMP(2);
    PF_COUNT(7);
    double fq = 0.0, gpq = 0.0;
    const bool bad = tile_assemble<MODE, KP>(a, sm, j, g, pk, gq, fq, gpq);
    PF_STAMP(3);
    __syncthreads();       // every wave has read the accumulators
    for (int e = threadIdx.x; e < 2 * PF_TSLOT * PF_TS; e += PF_TNW * 64) sm.sg0[e] = 0.0;
    bool need = false;
    {
      TileZ &z = sm.z[j];
      TileZ zl = z;        // group-local copy; lane g == 0 writes it back
      if (!zl.done) {
        zl.fq = fq;
        zl.gpq = gpq;
        zl.bad = bad ? 1 : 0;
        zl.n_eval++;
        need = tile_lbfgs<MODE, KP>(o, sm, zl, j, g, P, xk, gk, pk, gq);
        if (!need) {
          // series finished: its outputs, then the slot's next series
          double *th = a.theta + (size_t)sidx * P;
#pragma unroll
          for (int i = 0; i < NP; ++i) {
            const int p = g + 16 * i;
            if (p < P) th[p] = xk[i];
          }
          if (g == 0) {
            int st = zl.ret;
            if (warm && st == PF_ST_MAXIT) st = PF_ST_WARMUP;
            a.f_out[sidx] = zl.fk;
            a.f_stan[sidx] = zl.fk;
            a.n_iter[sidx] = zl.itNum;
            a.n_eval[sidx] = zl.n_eval;
            a.status[sidx] = st;
          }
          sidx = refill(zl, -1);
          need = sidx >= 0;
        }
      }
      PF_STAMP(4);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (g == 0) {
        z = zl;
        sm.sidx[j] = sidx;
      }
      if (need) tile_publish<MODE, KP>(a, sm, j, g);
      const unsigned long long any = __ballot(need);
      if (lane == 0) sm.flag[wave] = any != 0ull ? 1 : 0;
    }
    PF_STAMP(5);
    __syncthreads();
    PF_STAMP(6);
    const int more = sm.flag[0] | sm.flag[1] | sm.flag[2] | sm.flag[3];
    if (!__builtin_amdgcn_readfirstlane(more)) break;
  }
}
