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
// of G = r(1 + Xb_m), G t per series.  Residuals, likelihood and prior terms
// are elementwise in the C layout.
//
// Row pass: each wave takes a contiguous quarter of the 16-row chunks,
// software-pipelined — the Xb MFMAs of chunk c+1 are issued before chunk c's
// elementwise VALU work (matrix and vector pipes overlap within the wave),
// and global loads run two chunks ahead (one wave per SIMD: nothing else
// hides L2 / HBM latency).
//
// L-BFGS: every series owns 16 lanes (4 series per wave, all 4 waves busy;
// parameter p = g + 16 i in lane g) running Stan 2.19's
// BFGSMinimizer<LBFGSUpdate> + Wolfe line search (same control flow as
// oracle/stan_lbfgs.c, two-loop recursion), with per-series convergence
// masking: a series that terminates stops moving and the tile exits when
// all 16 have.  State lives in LDS between evaluations.
//
// Scope: linear / flat growth, P = 3 + S + K <= 64, K <= 32, S + 1 <= 32,
// shared prior scales (the reference layout and the configs[2]/[3]
// shapes); the per-series kernel K3 covers the rest.  The exact-MAP polish
// runs after it (k_polish, one workgroup per series).
#pragma once

#define PF_TS 16   // series per tile (MFMA N)
#define PF_TNW 4   // waves per tile workgroup (one per SIMD; 8 waves, two per SIMD, measured
                   // no faster: the row pass is bound by the SIMD's FP64 pipe, shared by
                   // MFMA and VALU, and the register cap of two waves spills the step)
#define PF_TSW 4   // waves that run the per-series phases (16 lanes per series)
#define PF_TH 5    // L-BFGS history (Stan default)
#define PF_TV 64   // LDS stride of a per-series parameter vector
#define PF_TNP 4   // parameters per lane (p = g + 16 i)
#define PF_TSEG 33 // per-series stride of the segment tables (odd: conflict-free LDS reads)

struct TileZ {
  double fk, fk1, fq, gpq, alpha, alphak_1, dfp, c1dfp, c2dfp, alpha0, alpha1, prevF, prevDFp;
  double alo, aloF, aloDFp, ahi, ahiF, ahiDFp, lastDFp, dfp_prev, gammak;
  int state, itNum, resetB, nits, lsRestarts, zit, hcount, head, ret, n_eval, bad, done;
};

template <int MODE>
struct TileSmem {
  static constexpr int NSET = ((MODE & 3) == 2) ? 2 : 1;
  static constexpr int KP = 32;  // padded feature count (K <= 32)
  double *xk, *gk, *pk, *xq, *gq;  // [16][PF_TV]
  double *hs, *hy;               // [H][16][PF_TV]
  double *hrho;                  // [16][H]
  double *kseg, *mseg;           // [16][PF_TSEG]
  double *bm, *ba;               // [KP][16]
  double *gb;                    // [NSET][KP][16]
  double *sg0, *sg1;             // [32][16] segment sums of G, G t
  double *rr;                    // [16]
  double *sig;                   // [16][2] sigma, 1/sigma^2
  double *ctc, *csg, *csm, *csa; // [64]
  TileZ *z;                      // [16]
  int *flag;                     // [4]
  // gb, sg0, sg1, rr are contiguous: zeroed as one block per evaluation
  static constexpr size_t acc_doubles() { return NSET * KP * PF_TS + 2 * 32 * PF_TS + PF_TS; }
  static __host__ __device__ size_t bytes() {
    const size_t d = (5 + 2 * PF_TH) * PF_TS * PF_TV + PF_TS * PF_TH + 2 * PF_TS * PF_TSEG +
                     2 * KP * PF_TS + acc_doubles() + 2 * PF_TS + 4 * 64;
    return d * sizeof(double) + PF_TS * sizeof(TileZ) + 64;
  }
  __device__ void carve(char *base) {
    double *p = reinterpret_cast<double *>(base);
    constexpr size_t vec = (size_t)PF_TS * PF_TV;
    xk = p; p += vec;
    gk = p; p += vec;
    pk = p; p += vec;
    xq = p; p += vec;
    gq = p; p += vec;
    hs = p; p += PF_TH * vec;
    hy = p; p += PF_TH * vec;
    hrho = p; p += PF_TS * PF_TH;
    kseg = p; p += PF_TS * PF_TSEG;
    mseg = p; p += PF_TS * PF_TSEG;
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

typedef double TVec[PF_TNP];

__device__ __forceinline__ double tvdot(const TVec &u, const TVec &v) {
  const double s = fma(u[0], v[0], u[1] * v[1]) + fma(u[2], v[2], u[3] * v[3]);
  return grp_sum(s);
}
// LDS vector <-> registers; entries past P read as 0
__device__ __forceinline__ void tvload(TVec &r, const double *v, int P, int g) {
#pragma unroll
  for (int i = 0; i < PF_TNP; ++i) {
    const int p = g + 16 * i;
    r[i] = (p < P) ? v[p] : 0.0;
  }
}
__device__ __forceinline__ void tvstore(double *v, const TVec &r, int P, int g) {
#pragma unroll
  for (int i = 0; i < PF_TNP; ++i) {
    const int p = g + 16 * i;
    if (p < P) v[p] = r[i];
  }
}

// Publish series j's trial point xq: segment tables, beta o s_m / s_a, sigma
// (the 16 lanes of series j; g = lane & 15).
template <int MODE>
__device__ __forceinline__ void tile_publish(const FitKArgs &a, TileSmem<MODE> &sm, int j, int g) {
  const int S = a.S, K = a.K;
  const double *x = sm.xq + (size_t)j * PF_TV;
  // segment tables k_s = k + sum_{c < s} delta_c, m_s = m - sum_{c < s}
  // t_c delta_c: row-parallel inclusive prefix (lane g: changepoints g and
  // g + 16; the 16 lanes of series j are one DPP row).  Flat growth: k = 0
  // and no slope changes (trend = m).
  const bool lin = a.growth == PF_GROWTH_LINEAR;
  const double k = lin ? x[0] : 0.0, m = x[1];
  const double da = (lin && g < S) ? x[2 + g] : 0.0, db = (lin && g + 16 < S) ? x[18 + g] : 0.0;
  double pa = da, qa = sm.ctc[g] * da, pb = db, qb = sm.ctc[g + 16] * db;
  pa = row_prefix(pa);
  qa = row_prefix(qa);
  pb = row_prefix(pb) + dpp_f64<PF_DPP_ROWBCAST(15)>(pa);
  qb = row_prefix(qb) + dpp_f64<PF_DPP_ROWBCAST(15)>(qa);
  if (g == 0) {
    sm.kseg[j * PF_TSEG] = k;
    sm.mseg[j * PF_TSEG] = m;
  }
  if (g < S) {
    sm.kseg[j * PF_TSEG + g + 1] = k + pa;
    sm.mseg[j * PF_TSEG + g + 1] = m - qa;
  }
  if (g + 16 < S) {
    sm.kseg[j * PF_TSEG + g + 17] = k + pb;
    sm.mseg[j * PF_TSEG + g + 17] = m - qb;
  }
  if (g == 1) {
    const double sg = exp(x[2 + S]);
    sm.sig[2 * j] = sg;
    sm.sig[2 * j + 1] = 1.0 / (sg * sg);
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int f = g + 16 * h;
    const double bv = (f < K) ? x[3 + S + f] : 0.0;
    sm.bm[f * PF_TS + j] = bv * sm.csm[f];
    sm.ba[f * PF_TS + j] = bv * sm.csa[f];
  }
}

typedef double pf_d2 __attribute__((ext_vector_type(2)));
typedef int pf_i4 __attribute__((ext_vector_type(4)));

// Row mapping inside a 16-row chunk: C-layout row i (lane (j, rq) register
// rg holds C-row rq + 4 rg) is data row r0 + 4 (i & 3) + (i >> 2), so each
// lane's four rows are contiguous (t, y, seg in two / one wide loads) and
// k-step q of X'W covers data rows r0 + 4 rq + q.  Feature maps: Xb k-step
// kk, lane k index rq <-> feature 8 rq + kk; X'W tile ft, output row i <->
// feature 2 i + ft (both contiguous per lane in the row-major copy XR).
struct TileIn {
  pf_d2 xa[4];  // X[r0 + 4 (j & 3) + (j >> 2)][8 rq + 2h .. +1]  (Xb k-steps 2h, 2h+1)
  pf_d2 xg[4];  // X[r0 + 4 rq + q][2 j .. 2 j + 1]             (X'W k-step q, tiles 0/1)
  pf_d2 t[2], y[2];  // data rows r0 + 4 rq + rg
  pf_i4 sg;
};

// Row pass of one evaluation (all waves): accumulates the beta gradient
// tiles, segment sums of G / G t and the residual sum of squares into LDS
// (gb, sg0/sg1, rr), which the caller zeroed.
template <int MODE>
__device__ __forceinline__ void tile_rows(const FitKArgs &a, TileSmem<MODE> &sm, int tile, int n) {
  constexpr int NSET = TileSmem<MODE>::NSET;
  constexpr bool HM = (MODE & 3) != MODE_ADD, HA = (MODE & 3) != MODE_MULT;
  const int lane = pf_lane(), wave = __builtin_amdgcn_readfirstlane(pf_wave());
  const int T = a.T, Tp = a.Tp;
  const int j = lane & 15, rq = lane >> 4;
  const int s_g = tile * PF_TS + j;
  const bool svalid = s_g < n;
  const double *kseg = sm.kseg + j * PF_TSEG, *mseg = sm.mseg + j * PF_TSEG;
  const int jrow = 4 * (j & 3) + (j >> 2);
  // B operands of Xb: k-step kk, lane k index rq <-> feature 8 rq + kk
  double bmr[8], bar_[8];
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    bmr[kk] = HM ? sm.bm[(8 * rq + kk) * PF_TS + j] : 0.0;
    bar_[kk] = HA ? sm.ba[(8 * rq + kk) * PF_TS + j] : 0.0;
  }
  // Chunk loads as buffer loads: lane-constant byte offsets (voffset) plus
  // the chunk's uniform offset (soffset), no per-load address arithmetic;
  // unconditional (T_pad % 128 == 0 keeps every chunk row in range, XR is
  // zero past K, rows of series past n read 0 from the y buffer's range
  // check), so no predicated load drains the prefetch.
  const int nvalid = min(n - tile * PF_TS, PF_TS);
  const __amdgpu_buffer_rsrc_t rXR = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double *>(a.XR), (short)0, Tp * 32 * 8, 0x00020000);
  const __amdgpu_buffer_rsrc_t rT = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double *>(a.t), (short)0, Tp * 8, 0x00020000);
  const __amdgpu_buffer_rsrc_t rS = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<int32_t *>(a.seg), (short)0, Tp * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rY = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double *>(a.y_scaled + (size_t)tile * PF_TS * Tp), (short)0, nvalid * Tp * 8,
      0x00020000);
  const int oxa = (jrow * 32 + 8 * rq) * 8, oxg = (4 * rq * 32 + 2 * j) * 8;
  const int ot = 4 * rq * 8, oy = (j * Tp + 4 * rq) * 8, os = 4 * rq * 4;
  auto ld2 = [](__amdgpu_buffer_rsrc_t r, int vo, int so) {
    return __builtin_bit_cast(pf_d2, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0));
  };
  auto tload = [&](int c, TileIn &in) {
    const int r0 = 16 * c;
#pragma unroll
    for (int h = 0; h < 4; ++h) in.xa[h] = ld2(rXR, oxa + 16 * h, r0 * 256);
#pragma unroll
    for (int q = 0; q < 4; ++q) in.xg[q] = ld2(rXR, oxg + 256 * q, r0 * 256);
    in.t[0] = ld2(rT, ot, r0 * 8);
    in.t[1] = ld2(rT, ot + 16, r0 * 8);
    in.y[0] = ld2(rY, oy, r0 * 8);
    in.y[1] = ld2(rY, oy + 16, r0 * 8);
    in.sg = __builtin_bit_cast(pf_i4, __builtin_amdgcn_raw_buffer_load_b128(rS, os, r0 * 4, 0));
  };
  auto xb_mfma = [&](const TileIn &in, pf_d4 &xm, pf_d4 &xa) {
    // two independent accumulation chains per product (even / odd k-steps)
    pf_d4 m0 = pf_d4{0.0, 0.0, 0.0, 0.0}, m1 = m0, a0_ = m0, a1_ = m0;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
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
  pf_d4 gbm[2], gba[2];
#pragma unroll
  for (int ft = 0; ft < 2; ++ft) { gbm[ft] = pf_d4{0.0, 0.0, 0.0, 0.0}; gba[ft] = gbm[ft]; }
  double rr = 0.0, a0 = 0.0, a1 = 0.0;
  int cur = -1;
  auto flush = [&]() {
    double b0 = a0 + shfl_xor_f64<16>(a0), b1 = a1 + shfl_xor_f64<16>(a1);
    b0 += shfl_xor_f64<32>(b0);
    b1 += shfl_xor_f64<32>(b1);
    if (rq == 0) {
      atomicAdd(&sm.sg0[cur * PF_TS + j], b0);
      atomicAdd(&sm.sg1[cur * PF_TS + j], b1);
    }
  };
  const int nch = (T + 15) >> 4;
  const int c0 = (nch * wave) / PF_TNW, c1 = (nch * (wave + 1)) / PF_TNW;
  // one chunk: loads of chunk c + 2 into `nn`, Xb of chunk c + 1 (`nx`)
  // issued before chunk c's (`cu`, Xb in `xc`) elementwise work and X'W.
  // Input and Xb buffers rotate three ways: no register copies of in-flight
  // loads or MFMA results.  (A four-buffer ring, loads three chunks ahead,
  // measured no faster.)
  auto step = [&](int c, const TileIn &cu, const TileIn &nx, TileIn &nn, const pf_d4 &xcm,
                  const pf_d4 &xca, pf_d4 &xnm, pf_d4 &xna) {
    const int r0 = 16 * c;
    const int rbase = r0 + 4 * rq;
    // trend k_s t + m_s from the per-series segment tables (flat growth:
    // k = 0, one m); reads issued before the Xb MFMAs of the next chunk
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
    double W[4], Wa[4], G[4], Gt[4];
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      const int row = rbase + rg;
      const bool v = svalid && row < T;
      const double ti = cu.t[rg >> 1][rg & 1];
      const double tr = fma(ks[rg], ti, ms[rg]);
      const double u = 1.0 + (HM ? xcm[rg] : 0.0);
      const double mu = fma(tr, u, HA ? xca[rg] : 0.0);
      const double r = v ? cu.y[rg >> 1][rg & 1] - mu : 0.0;
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
        if constexpr (HM) gbm[ft] = __builtin_amdgcn_mfma_f64_16x16x4f64(cu.xg[q][ft], W[q], gbm[ft], 0, 0, 0);
        if constexpr (HA) gba[ft] = __builtin_amdgcn_mfma_f64_16x16x4f64(cu.xg[q][ft], Wa[q], gba[ft], 0, 0, 0);
      }
    }
    // changepoint adjoint: segment sums of G, G t per series
    if (uni) {
      if (s0 != cur) {
        if (cur >= 0) flush();
        cur = s0;
        a0 = 0.0;
        a1 = 0.0;
      }
      a0 += (G[0] + G[1]) + (G[2] + G[3]);
      a1 += (Gt[0] + Gt[1]) + (Gt[2] + Gt[3]);
    } else {
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        if (rbase + rg < T) {
          atomicAdd(&sm.sg0[cu.sg[rg] * PF_TS + j], G[rg]);
          atomicAdd(&sm.sg1[cu.sg[rg] * PF_TS + j], Gt[rg]);
        }
      }
    }
  };
  if (c0 < c1) {
    TileIn A, B, C;
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
  if (rq == 0) atomicAdd(&sm.rr[j], rr);
  // gradient tiles: C[row i = rq + 4 rg][series j] of tile ft is feature 2 i + ft
#pragma unroll
  for (int ft = 0; ft < 2; ++ft)
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      const int f = 2 * (rq + 4 * rg) + ft;
      if constexpr (HM) atomicAdd(&sm.gb[f * PF_TS + j], gbm[ft][rg]);
      if constexpr (HA) atomicAdd(&sm.gb[(NSET - 1) * TileSmem<MODE>::KP * PF_TS + f * PF_TS + j], gba[ft][rg]);
    }
}

// f and g of series j at xq (lane g: parameters g + 16 i -> sm.gq), gpq =
// g . pk.  Returns true if not finite (group-uniform).
template <int MODE>
__device__ __forceinline__ bool tile_assemble(const FitKArgs &a, TileSmem<MODE> &sm, int j, int g,
                                              double &f, double &gpq) {
  constexpr int NSET = TileSmem<MODE>::NSET;
  const int S = a.S, P = a.P, T = a.T;
  const bool linear = a.growth == PF_GROWTH_LINEAR;
  const double *x = sm.xq + (size_t)j * PF_TV;
  double *gv_out = sm.gq + (size_t)j * PF_TV;
  const double *pk = sm.pk + (size_t)j * PF_TV;
  const double sigma = sm.sig[2 * j], inv = sm.sig[2 * j + 1], tau = a.tau;
  const double rrt = sm.rr[j];
  // segment sums, lane g: segments g and g + 16 (S + 1 <= 32).  Suffix
  // sums over segments by a DPP row scan; changepoint jj is active in the
  // segments s > jj, so parameter p = 2 + jj needs the suffix at s = p - 1:
  // lane g - 1 of the same half (row_shr:1), or row lane 15 across halves.
  const double s0a = (g <= S) ? sm.sg0[g * PF_TS + j] : 0.0;
  const double s1a = (g <= S) ? sm.sg1[g * PF_TS + j] : 0.0;
  const double s0b = (g + 16 <= S) ? sm.sg0[(g + 16) * PF_TS + j] : 0.0;
  const double s1b = (g + 16 <= S) ? sm.sg1[(g + 16) * PF_TS + j] : 0.0;
  const double u0b = row_suffix(s0b), u1b = row_suffix(s1b);
  const double u0a = row_suffix(s0a) + dpp_f64<PF_DPP_ROWBCAST(0)>(u0b);
  const double u1a = row_suffix(s1a) + dpp_f64<PF_DPP_ROWBCAST(0)>(u1b);
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
  double fl = 0.0, gp = 0.0;
  bool bad = false;
#pragma unroll
  for (int i = 0; i < PF_TNP; ++i) {
    const int p = g + 16 * i;
    if (p >= P) continue;
    const double xv = x[p];
    double gv, ft;
    if (p == 0) {
      gv = -inv * (linear ? tot1 : 0.0) + xv / 25.0;
      ft = xv * xv / 50.0;
    } else if (p == 1) {
      gv = -inv * tot0 + xv / 25.0;
      ft = xv * xv / 50.0;
    } else if (p < 2 + S) {
      // changepoint jj is active in segments s > jj
      const int jj = p - 2;
      const double sgn = (xv > 0.0) - (xv < 0.0);
      gv = (linear ? -inv * (su1[i < 3 ? i : 2] - sm.ctc[jj] * su0[i < 3 ? i : 2]) : 0.0) + sgn / tau;
      ft = fabs(xv) / tau;
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
    gv_out[p] = gv;
    fl += ft;
    gp = fma(gv, pk[p], gp);
    bad |= !isfinite(gv);
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
// by Stan's two-loop recursion.  The working vectors live in registers for
// the step (4 entries per lane).
template <int MODE>
__device__ __forceinline__ bool tile_lbfgs(const pf_fit_opts &o, TileSmem<MODE> &sm, TileZ &z, int j,
                                           int g, int P) {
  double *xkL = sm.xk + (size_t)j * PF_TV, *gkL = sm.gk + (size_t)j * PF_TV, *pkL = sm.pk + (size_t)j * PF_TV;
  double *xqL = sm.xq + (size_t)j * PF_TV;
  const int H = o.history < PF_TH ? o.history : PF_TH;
  constexpr size_t hstep = (size_t)PF_TS * PF_TV;
  TVec xk, gk, pk, xq, gq;
  tvload(xk, xkL, P, g);
  tvload(gk, gkL, P, g);
  tvload(pk, pkL, P, g);
  tvload(xq, xqL, P, g);
  tvload(gq, sm.gq + (size_t)j * PF_TV, P, g);
  bool need = false, run = true;
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
          const double rho_new = 1.0 / sy;
          tvstore(sm.hs + slot * hstep + (size_t)j * PF_TV, sk, P, g);
          tvstore(sm.hy + slot * hstep + (size_t)j * PF_TV, yk, P, g);
          if (g == 0) sm.hrho[j * PF_TH + slot] = rho_new;
          if (z.hcount < H) z.hcount++;
          else z.head = pf_wrap(z.head + 1, H);
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int i = 0; i < PF_TNP; ++i) pk[i] = -gk[i];
          double al[PF_TH];
#pragma unroll
          for (int c = PF_TH - 1; c >= 0; --c) {
            al[c] = 0.0;
            if (c < z.hcount) {
              const int sl = pf_wrap(z.head + c, H);
              TVec sv, yv;
              double rho_c;
              if (c == z.hcount - 1) {    // newest pair: still in registers
#pragma unroll
                for (int i = 0; i < PF_TNP; ++i) { sv[i] = sk[i]; yv[i] = yk[i]; }
                rho_c = rho_new;
              } else {
                tvload(sv, sm.hs + sl * hstep + (size_t)j * PF_TV, P, g);
                tvload(yv, sm.hy + sl * hstep + (size_t)j * PF_TV, P, g);
                rho_c = sm.hrho[j * PF_TH + sl];
              }
              al[c] = rho_c * tvdot(sv, pk);
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
              double rho_c;
              if (c == z.hcount - 1) {
#pragma unroll
                for (int i = 0; i < PF_TNP; ++i) { sv[i] = sk[i]; yv[i] = yk[i]; }
                rho_c = rho_new;
              } else {
                tvload(sv, sm.hs + sl * hstep + (size_t)j * PF_TV, P, g);
                tvload(yv, sm.hy + sl * hstep + (size_t)j * PF_TV, P, g);
                rho_c = sm.hrho[j * PF_TH + sl];
              }
              const double b = rho_c * tvdot(yv, pk);
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
  tvstore(xkL, xk, P, g);
  tvstore(gkL, gk, P, g);
  tvstore(pkL, pk, P, g);
  tvstore(xqL, xq, P, g);
  return need;
}

// K3T kernel: grid = ceil(n / 16) tiles.  Pass-0 semantics of fit_body
// (theta in: init; out: the L-BFGS endpoint, f, f_stan, status, n_iter,
// n_eval); warm = the iteration cap is the warm-up cap (MAXIT -> WARMUP).
// Per evaluation: row pass (all waves) | barrier | assemble (16 lanes per
// series) | barrier | zero accumulators + L-BFGS step + publish | barrier.
template <int MODE>
__global__ __launch_bounds__(PF_TNW * 64, 1) void k_fit_tile(FitKArgs a, int n) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  TileSmem<MODE> sm;
  sm.carve(smem_raw);
  const int tile = blockIdx.x, lane = pf_lane(), wave = __builtin_amdgcn_readfirstlane(pf_wave());
  const int P = a.P, S = a.S;
  const bool stepper = wave < PF_TSW;                   // per-series phases: waves 0..3
  const int j = (4 * wave + (lane >> 4)) & 15, g = lane & 15;  // series j's 16 lanes
  const int sgl = tile * PF_TS + j;
  const bool warm = a.warm_cap != 0;
  const pf_fit_opts o = a.o;
  constexpr int NACC = (int)TileSmem<MODE>::acc_doubles();
  if (threadIdx.x < 64) {
    const int i = threadIdx.x;
    sm.ctc[i] = (i < S) ? a.t_change[i] : 0.0;
    sm.csg[i] = (i < a.K) ? a.sigmas[i] : 1.0;
    sm.csm[i] = (i < a.K) ? a.s_m[i] : 0.0;
    sm.csa[i] = (i < a.K) ? a.s_a[i] : 0.0;
  }
  for (int e = threadIdx.x; e < NACC; e += PF_TNW * 64) sm.gb[e] = 0.0;
  if (stepper) {
    TileZ &z = sm.z[j];
    const bool live = sgl < n && a.status[sgl] != PF_ST_CONSTANT;
    double *xq = sm.xq + (size_t)j * PF_TV, *xk = sm.xk + (size_t)j * PF_TV;
    for (int p = g; p < PF_TV; p += 16) {
      const double v = (sgl < n && p < P) ? a.theta[(size_t)sgl * P + p] : 0.0;
      xq[p] = v;
      xk[p] = v;
    }
    if (g == 0) {
      memset(&z, 0, sizeof(TileZ));
      z.state = LB_INIT;
      z.done = live ? 0 : 1;
    }
  }
  __syncthreads();
  if (stepper) tile_publish<MODE>(a, sm, j, g);
  __syncthreads();
  while (true) {
    PF_STAMP(0);
    tile_rows<MODE>(a, sm, tile, n);
    PF_STAMP(1);
    __syncthreads();
    PF_STAMP(2);
    PF_COUNT(7);
    double fq = 0.0, gpq = 0.0;
    bool bad = false;
    if (stepper) bad = tile_assemble<MODE>(a, sm, j, g, fq, gpq);
    PF_STAMP(3);
    __syncthreads();       // every wave has read the accumulators
    for (int e = threadIdx.x; e < NACC; e += PF_TNW * 64) sm.gb[e] = 0.0;
    if (stepper) {
      TileZ &z = sm.z[j];
      bool need = false;
      TileZ zl = z;        // group-local copy; lane g == 0 writes it back
      if (!zl.done) {
        zl.fq = fq;
        zl.gpq = gpq;
        zl.bad = bad ? 1 : 0;
        zl.n_eval++;
        need = tile_lbfgs<MODE>(o, sm, zl, j, g, P);
        if (!need) zl.done = 1;
      }
      PF_STAMP(4);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (g == 0) z = zl;
      if (need) tile_publish<MODE>(a, sm, j, g);
      const unsigned long long any = __ballot(need);
      if (lane == 0) sm.flag[wave] = any != 0ull ? 1 : 0;
    }
    PF_STAMP(5);
    __syncthreads();
    PF_STAMP(6);
    const int more = sm.flag[0] | sm.flag[1] | sm.flag[2] | sm.flag[3];
    if (!__builtin_amdgcn_readfirstlane(more)) break;
  }
  // outputs (pass-0 semantics of fit_body)
  if (stepper && sgl < n) {
    const TileZ &z = sm.z[j];
    double *th = a.theta + (size_t)sgl * P;
    const int st_in = a.status[sgl];
    if (st_in == PF_ST_CONSTANT) {
      if (g == 0) {
        th[2 + S] = log(1e-9);
        a.f_out[sgl] = NAN;
        a.f_stan[sgl] = NAN;
        a.n_iter[sgl] = 0;
        a.n_eval[sgl] = 0;
      }
    } else {
      const double *xk = sm.xk + (size_t)j * PF_TV;
      for (int p = g; p < P; p += 16) th[p] = xk[p];
      if (g == 0) {
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
