// CDNA4 kernels of the Metropolis-Hastings baseline (mcmc.py) and the SRTM2
// forward model (kinetic_model.py), fp64 like the reference (mcmc.py:22).
//
// One 64-lane wavefront per chain.  Lane f (< 54) owns frame f of the TAC being
// evaluated; lane r (< 48) owns ROI r of the chain state (DVR_r, R1_r, the prior
// gradient g = P (x - mu) and the ROI log-likelihood).  An element-wise
// Metropolis update of ROI i touches only ROI i's TAC (SRTM2 is per ROI), so a
// proposal costs one 54 x 54 operator application + 54 truncated-normal terms;
// the MvNormal prior change is 2 d g_i + d^2 P_ii (g kept current on accept).
#include "mh_internal.h"
#include "logphi_coef.h"
#include "fp64_math.h"

#include <cstdlib>

// Tuning knobs (the product uses the defaults; scripts/micro/build_mh.sh builds variants)
#ifndef MH_EXP_MODE
#define MH_EXP_MODE 0     // timing experiments only: bits drop exp / log / log_ndtr / sqrt / divisions
#endif
#ifndef MH_MV_UNROLL
#define MH_MV_UNROLL 28   // operator-row matvec: 16-B steps unrolled
#endif

// log Phi of the truncated-normal normaliser: 1 = the piecewise polynomial of logphi_coef.h
// (scripts/gen_logphi.py; |err| <= 1.2e-16 on [0, 10)), 0 = ocml log(erfc) (A/B)
#ifndef MH_LOGPHI_POLY
#define MH_LOGPHI_POLY 1
#endif

namespace petmh {

constexpr int NR = kNRoi, NF = kNFrames;
constexpr int LPNI = PETMH_LOGPHI_NI, LPLD = 18;   // LDS row: 16 coefficients (c15 = 0) + 2 pad doubles,
static_assert(PETMH_LOGPHI_DEG == 14, "8 x 16-B pieces per row");   // 144-B rows: conflict-free ds_read_b128
__constant__ double c_logphi[LPNI][PETMH_LOGPHI_DEG + 1] = PETMH_LOGPHI_COEF;

#ifndef MH_ESTRIN
#define MH_ESTRIN 0
#endif
// log Phi(x) for 0 <= x < 10 (x = NaN: NaN): interval k = floor(x), Horner in u = x - (k + 0.5)
// from the LDS copy of the coefficients (row k: pieces (c_2j, c_2j+1)).
__device__ __forceinline__ double log_phi_poly(const double* tab, double x) {
  int k = (int)x;
  k = k < 0 ? 0 : (k > LPNI - 1 ? LPNI - 1 : k);
  const double u = x - ((double)k + 0.5);
  const double2* row = reinterpret_cast<const double2*>(tab + k * LPLD);
#if MH_ESTRIN
  // Estrin's scheme: depth 5 instead of Horner's 14 dependent FMAs (the update is latency-bound at 2 waves / SIMD)
  double q[8];
#pragma unroll
  for (int j = 0; j < 7; ++j) q[j] = fma(row[j].y, u, row[j].x);
  q[7] = row[7].x;
  const double u2 = u * u, u4 = u2 * u2, u8 = u4 * u4;
  const double r0 = fma(q[1], u2, q[0]), r1 = fma(q[3], u2, q[2]), r2 = fma(q[5], u2, q[4]), r3 = fma(q[7], u2, q[6]);
  return fma(fma(r3, u4, r2), u8, fma(r1, u4, r0));
#else
  double p = row[7].x;
#pragma unroll
  for (int j = 6; j >= 0; --j) {
    const double2 cc = row[j];
    p = fma(p, u, cc.y);
    p = fma(p, u, cc.x);
  }
  return p;
#endif
}

// 1/sqrt(x) for a positive normal x: v_rsq_f64, then two Newton steps y (1 + (1/2 - x y^2 / 2)) in fma form
__device__ __forceinline__ double rsq_f64(double x) {
  double y = __builtin_amdgcn_rsq(x);
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const double r = fma(-(x * y), 0.5 * y, 0.5);
    y = fma(y, r, y);
  }
  return y;
}

// Round 6: e^x of the per-frame exponentials from a 64-entry table of 2^(j/64) in LDS: x = (64 m + j) ln 2 / 64 + r,
// |r| <= ln 2 / 128, e^r by its degree-5 Taylor polynomial (truncation 3e-17), 2^m by ldexp (<= 2 ulp); about
// 16 instructions and one LDS read against ocml's ~30.  Outside (-708, 709) and NaN: ocml's exp.  0: ocml's exp
#ifndef MH_TEXP
#define MH_TEXP 1
#endif
constexpr int kE2 = 64;
#ifndef MH_BRANCHLESS
#define MH_BRANCHLESS 1
#endif
#ifndef MH_SEL_BCAST
#define MH_SEL_BCAST 1
#endif
#ifndef MH_FRAME_SELECT
#define MH_FRAME_SELECT 1     // the update's frame terms on every lane, masked by a select (roi_loglik_r)
#endif
__device__ __forceinline__ double exp_tab(const double* E2, double x) {
#if MH_BRANCHLESS
  // x clamped to [-746, 710] instead of a branch to ocml: below, e^x rounds to 0 (ldexp), above it overflows
  // to inf; NaN passes the clamp and the reduction as NaN; (-745, -708) gives denormals by ldexp
  x = x < -746.0 ? -746.0 : (x > 710.0 ? 710.0 : x);
#else
  if (!(x > -708.0 && x < 709.0)) return exp(x);
#endif
  const double kf = rint(x * 92.332482616893656);                 // 64 / ln 2
  double r = fma(-kf, 6.93147180369123816490e-01 / 64, x);       // fdlibm's ln 2 split (kf ln2_hi exact), / 64
  r = fma(-kf, 1.90821492927058770002e-10 / 64, r);
  const int k = (int)kf, j = k & (kE2 - 1), m = k >> 6;
  double q = 8.3333333333333333e-03;                              // 1/5!
  q = fma(q, r, 4.1666666666666667e-02);
  q = fma(q, r, 1.6666666666666667e-01);
  q = fma(q, r, 0.5);
  q = fma(q, r, 1.0);
  q = fma(q, r, 1.0);
  return ldexp(E2[j] * q, m);
}
__device__ __forceinline__ void load_e2(double* E2) {
  for (int j = threadIdx.x; j < kE2; j += blockDim.x) E2[j] = exp2((double)j / kE2);
}

// Round 6: log x (x > 0 finite) from a 64-entry table over the mantissa: m = x 2^-e in [1, 2), row j = floor(64 (m - 1))
// holds (1/c_j rounded, -log of that), c_j = 1 + (j + 1/2) / 64; r = m / c_j - 1 by one fma (|r| <= 1/128), log(1 + r)
// by its degree-8 Taylor polynomial (truncation 5e-20).  Absolute error < 1 ulp of max(|log x|, 1) (numpy check in
// DESIGN.md §3), the measure that matters in a sum of 54 frame terms.  Replaces fdlibm's division f / (2 + f) and its
// 14 polynomial / combination steps.  Otherwise (0, negative, inf, NaN, denormal): ocml's log.  0: log_pos
#ifndef MH_TLOG
#define MH_TLOG 1
#endif
constexpr int kLT = 64;
__device__ __forceinline__ double log_tab(const double2* LT, double x) {
#if !MH_BRANCHLESS
  if (!(x >= 2.2250738585072014e-308 && x < __builtin_huge_val())) return log(x);
#endif
  const int e = __builtin_amdgcn_frexp_exp(x) - 1;                     // x = m 2^e, m in [1, 2)
  const double m = __builtin_amdgcn_frexp_mant(x) * 2.0;
#if MH_BRANCHLESS
  const int j = min(max((int)((m - 1.0) * 64.0), 0), 63);            // rows 0..63 for 0 / inf / NaN too
#else
  const int j = (int)((m - 1.0) * 64.0);                               // exact: m - 1 and the scaling
#endif
  const double2 t = LT[j];                                             // (1/c, -log(1/c))
  const double r = fma(m, t.x, -1.0);
  double p = -0.125;                                                   // -1/8
  p = fma(p, r, 1.4285714285714285e-01);
  p = fma(p, r, -1.6666666666666666e-01);
  p = fma(p, r, 0.2);
  p = fma(p, r, -0.25);
  p = fma(p, r, 3.3333333333333333e-01);
  p = fma(p, r, -0.5);
  const double l1p = fma(p * r, r, r);                                 // r - r^2/2 + ... - r^8/8
  const double res = fma((double)e, 6.93147180369123816490e-01, fma((double)e, 1.90821492927058770002e-10, t.y + l1p));
#if MH_BRANCHLESS
  // denormals take the table path (frexp normalises them); 0 -> -inf, < 0 -> NaN, inf -> inf, NaN -> NaN
  return x > 0.0 ? (x < __builtin_huge_val() ? res : x) : (x == 0.0 ? -__builtin_huge_val() : __builtin_nan(""));
#else
  return res;
#endif
}
__device__ __forceinline__ void load_lt(double2* LT) {
  for (int j = threadIdx.x; j < kLT; j += blockDim.x) {
    const double inv = 1.0 / (1.0 + (j + 0.5) / kLT);
    LT[j] = make_double2(inv, -log(inv));
  }
}

// e^{-k2a t} of the update kernel by fp64_math.h exp_fast (<= 1 ulp) instead of ocml's exp
#ifndef MH_FAST_EXP
#define MH_FAST_EXP 0
#endif
// log of the noise scale sigma > 0 (MH_FAST_LOG): fp64_math.h log_pos
#ifndef MH_FAST_LOG
#define MH_FAST_LOG 1
#endif
// Round 6: the per-frame noise terms from r = 1/sqrt(sn) (v_rsq_f64 + two Newton steps) and a table of 1/SIG
// (exact, formed at LDS load): 1/sig = r / SIG, z = (y - sn) / sig, xs = sn / sig, log sig = -log(1/sig).
// It replaces ocml's correctly rounded sqrt and the IEEE division 1 / sig (about 20 fp64 instructions a
// frame) by 8; the terms move by an ulp or two, so accept / reject paths can differ from the oracles' only
// where log u lies within ~1e-15 of the ratio.  0: sqrt and divide (the oracles' expression order)
#ifndef MH_RSQ
#define MH_RSQ 1
#endif
// Round 6: the sweep's per-element LDS operands (the next element's index, proposal draw, log u and prior
// diagonal) read one element ahead, so their LDS round trips overlap the current element's likelihood
#ifndef MH_PF
#define MH_PF 1
#endif

// Round 6: the update's operator matvec on DPP row broadcasts of e (conv_dpp) instead of an LDS round trip
// of e (a write and 28 broadcast ds_read_b128, about three in flight).  0: the LDS matvec
#ifndef MH_DPP
#define MH_DPP 1
#endif

// LDS copy of the coefficient table (one element per thread)
__device__ __forceinline__ void load_logphi(double* tab) {
  for (int e = threadIdx.x; e < LPNI * LPLD; e += blockDim.x) {
    const int k = e / LPLD, j = e - k * LPLD;
    tab[e] = j <= PETMH_LOGPHI_DEG ? c_logphi[k][j] : 0.0;
  }
}
#ifndef MH_WAVES
#define MH_WAVES 8
#endif
constexpr int kWaves = MH_WAVES;      // chains per workgroup (64 * kWaves threads)

constexpr int MLD = 56;               // padded operator row (16-B aligned pairs)

struct Lds {
  double M[NF * MLD];                 // SRTM2 operator, [f][g] (row per frame, g padded to 56)
  double PD[NR * NR], PR[NR * NR];    // prior precision matrices
  double Y[NR * NF], SIG[NR * NF];    // observed TAC / dt and noise sigma, [roi][frame]
  double CR[NF], TV[NF];
  double MUD[NR], MUR[NR];
  alignas(16) double LPHI[LPNI * LPLD];   // log Phi polynomial (16-B aligned rows)
  double E2[kE2];                         // 2^(j/64) (MH_TEXP)
  double2 LT[kLT];                        // (1/c_j, -log(1/c_j)) (MH_TLOG)
  double E[kWaves][64];               // per-wave exponential scratch
  double Z[kWaves][2 * NR];           // per-wave sweep draws: N(0,1) proposal per element
  double LU[kWaves][2 * NR];          //   log accept-uniform per element
  uint32_t KEY[kWaves][2 * NR];       //   sort key of the shuffled order
  int ORD[kWaves][2 * NR];            //   the sweep's element order
};

// DPP move of a double (two 32-bit halves); lanes without a source read 0.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), CTRL, ROW_MASK, 0xf, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROW_MASK, 0xf, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// Wave sum with DPP row shifts + row broadcasts (gfx9), total in lane 63, returned to
// every lane through an SGPR (readlane): one wave-uniform value, so every accept /
// reject decision is taken identically by all lanes.
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp_f64<0x111>(v);          // row_shr:1
  v += dpp_f64<0x112>(v);          // row_shr:2
  v += dpp_f64<0x114>(v);          // row_shr:4
  v += dpp_f64<0x118>(v);          // row_shr:8   -> lane 15 of each row: the row's sum
  v += dpp_f64<0x142, 0xa>(v);     // row_bcast:15 into rows 1, 3
  v += dpp_f64<0x143, 0xc>(v);     // row_bcast:31 into rows 2, 3 -> lane 63: total
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), 63);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// Value of a double held by lane `src` (wave-uniform index), as an SGPR broadcast.
__device__ __forceinline__ double lane_bcast(double v, int src) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), src);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}

// log Phi(x) (scipy.special.log_ndtr), via erfc / erfcx for the left tail
__device__ __forceinline__ double log_ndtr(double x) {
  if (x > -1.0) return log(0.5 * erfc(-x * 0.7071067811865476));
  return log(0.5 * erfcx(-x * 0.7071067811865476)) - 0.5 * x * x;
}

// Sum over frames of the TruncatedNormal(lower=0) log density of ROI i with
// parameters (DVR, R1); every lane returns the total (mcmc.py:151-155).
// MH_MROW_REG: the lane's operator row lives in registers for the whole kernel (28 x 16 B) instead
// of being re-read from LDS every update
#ifndef MH_MROW_REG
#define MH_MROW_REG 1
#endif
#if MH_DPP
// conv_f = sum_g M[f][g] e[g] with e[g] held by lane g, no LDS round trip: two permlane swaps replicate each
// 16-lane row j of e into every row (X_j), and v_fmac_f64 with DPP row_newbcast:k hands every lane
// e[16 j + k] as its first operand.  The lane's operator row M[f][0..53] lives in registers.
using MRow = double[NF];
template <int K, bool FIRST>
__device__ __forceinline__ void fma_nb(double& acc, double x, double m) {
  // FIRST: 2 wait states between the VALU write of x (the permlane swaps) and its DPP read
  if constexpr (FIRST)
    asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
        : "+v"(acc) : "v"(x), "v"(m), "i"(K));
  else
    asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(x), "v"(m), "i"(K));
}
template <int K>
__device__ __forceinline__ void conv_terms(const MRow& mr, const double (&X)[4], double (&a)[4]) {
  if constexpr (K < 16) {
    fma_nb<K, K == 0>(a[0], X[0], mr[K]);
    fma_nb<K, K == 0>(a[1], X[1], mr[16 + K]);
    fma_nb<K, K == 0>(a[2], X[2], mr[32 + K]);
    if constexpr (48 + K < NF) fma_nb<K, K == 0>(a[3], X[3], mr[48 + K]);
    conv_terms<K + 1>(mr, X, a);
  }
}
__device__ __forceinline__ double conv_dpp(const MRow& mr, double ev) {   // every lane active
  const unsigned long long b = (unsigned long long)__double_as_longlong(ev);
  const unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
  // permlane16_swap(x, x): odd rows of the first copy <-> even rows of the second: {[E0 E0 E2 E2], [E1 E1 E3 E3]}
  const auto l16 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h16 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  // permlane32_swap(y, y): rows 2-3 of the first copy <-> rows 0-1 of the second: {[Ea x4], [Eb x4]}
  const auto l02 = __builtin_amdgcn_permlane32_swap(l16[0], l16[0], false, false);
  const auto h02 = __builtin_amdgcn_permlane32_swap(h16[0], h16[0], false, false);
  const auto l13 = __builtin_amdgcn_permlane32_swap(l16[1], l16[1], false, false);
  const auto h13 = __builtin_amdgcn_permlane32_swap(h16[1], h16[1], false, false);
  auto mk = [](unsigned l, unsigned h) { return __longlong_as_double((long long)(((unsigned long long)h << 32) | l)); };
  const double X[4] = {mk(l02[0], h02[0]), mk(l13[0], h13[0]), mk(l02[1], h02[1]), mk(l13[1], h13[1])};
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  conv_terms<0>(mr, X, a);
  return (a[0] + a[1]) + (a[2] + a[3]);
}
__device__ __forceinline__ void load_mrow(const Lds& s, MRow& mr, int lane) {
#pragma unroll
  for (int g = 0; g < NF; ++g) mr[g] = s.M[(lane < NF ? lane : 0) * MLD + g];
}
#else
using MRow = double2[MLD / 2];
__device__ __forceinline__ void load_mrow(const Lds& s, MRow& mr, int lane) {
#pragma unroll
  for (int q = 0; q < MLD / 2; ++q) mr[q] = reinterpret_cast<const double2*>(s.M + (lane < NF ? lane : 0) * MLD)[q];
}
#endif

#if MH_DPP
static_assert(MH_RSQ, "the DPP update path takes 1/SIG");
// One ROI's log-likelihood from the lane's frame operands: t_f and C_R(t_f) (fixed per lane) and Y_{i,f},
// 1/SIG_{i,f} of ROI i (the sweep reads them one element ahead)
__device__ __forceinline__ double roi_loglik_r(const Lds& s, const MRow& mreg, int lane, double tv, double cr,
                                              double y, double rsig, double dvr, double r1, double k2p) {
  const double k2 = k2p * r1;           // kinetic_model.py:153-154
  const double k2a = k2 / dvr;
  const double ex = -k2a * tv;
#if MH_FRAME_SELECT && MH_BRANCHLESS && MH_TEXP && MH_TLOG && MH_LOGPHI_POLY
  // every lane runs the frame terms (lanes 54..63 on frame 0's operands) and the frame mask is a select at
  // the end: no exec-mask branches on the update's critical path
  const double ev = exp_tab(s.E2, ex);                            // lanes 54..63: never read by conv_dpp
  const double conv = conv_dpp(mreg, ev);
  const double tac = r1 * cr + (k2 - r1 * k2a) * conv;            // :157-158
  const double sn = tac < 0.0 ? 1e-6 : tac;                       // mcmc.py:152
  const double inv = rsq_f64(sn) * rsig;                          // 1 / (sqrt(sn) SIG), :153
  const double z = (y - sn) * inv;
  const double xs = sn * inv;
  const double lp = log_phi_poly(s.LPHI, xs);                     // row clamped to [0, 9] for any xs
  const double lnd = xs < 10.0 ? lp : 0.0;
  const double lf = -0.5 * z * z - 0.9189385332046727 + log_tab(s.LT, inv) - lnd;   // - log sig
  const double l = lane < NF ? lf : 0.0;
#else
  const double ev = lane < NF ? (MH_TEXP ? exp_tab(s.E2, ex) : exp(ex)) : 0.0;   // lanes 54..63: never read
  const double conv = conv_dpp(mreg, ev);
  double l = 0.0;
  if (lane < NF) {
    const double tac = r1 * cr + (k2 - r1 * k2a) * conv;            // :157-158
    const double sn = tac < 0.0 ? 1e-6 : tac;                       // mcmc.py:152
    const double inv = rsq_f64(sn) * rsig;                          // 1 / (sqrt(sn) SIG), :153
    const double z = (y - sn) * inv;
    const double xs = sn * inv;
    const double lnd = xs < 10.0 ? (MH_LOGPHI_POLY ? log_phi_poly(s.LPHI, xs) : log_ndtr(xs)) : 0.0;
    l = -0.5 * z * z - 0.9189385332046727 + (MH_TLOG ? log_tab(s.LT, inv) : log_pos(inv)) - lnd;   // - log sig
  }
#endif
  __builtin_amdgcn_wave_barrier();
  return wave_sum(l);
}
__device__ __forceinline__ double roi_loglik(const Lds& s, const MRow& mreg, double*, int lane, int i,
                                            double dvr, double r1, double k2p) {
  const int fl = lane < NF ? lane : 0;
  return roi_loglik_r(s, mreg, lane, s.TV[fl], s.CR[fl], s.Y[i * NF + fl], s.SIG[i * NF + fl], dvr, r1, k2p);
}
#else
__device__ __forceinline__ double roi_loglik(const Lds& s, const MRow& mreg, double* e, int lane, int i,
                                            double dvr, double r1, double k2p) {
  const double k2 = k2p * r1;           // kinetic_model.py:153-154
  const double k2a = k2 / dvr;
#if MH_EXP_MODE & 1
  e[lane] = lane < NF ? 1.0 - k2a * s.TV[lane < NF ? lane : 0] : 0.0;
#else
  const double ex = -k2a * s.TV[lane < NF ? lane : 0];
  e[lane] = lane < NF ? (MH_TEXP ? exp_tab(s.E2, ex) : MH_FAST_EXP ? exp_fast(ex) : exp(ex)) : 0.0;   // e[54..63] = 0
#endif
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  double l = 0.0;
  if (lane < NF) {
    // conv_f = sum_g M[f][g] e[g]: own operator row, e broadcast, 16-B reads, 2 chains
    const double2* mrow = reinterpret_cast<const double2*>(s.M + lane * MLD);
    const double2* ev = reinterpret_cast<const double2*>(e);
    double c0 = 0.0, c1 = 0.0;
#pragma unroll MH_MV_UNROLL
    for (int q = 0; q < MLD / 2; ++q) {
      const double2 m = MH_MROW_REG ? mreg[q] : mrow[q], x = ev[q];
      c0 = fma(m.x, x.x, c0);
      c1 = fma(m.y, x.y, c1);
    }
    const double conv = c0 + c1;
    const double tac = r1 * s.CR[lane] + (k2 - r1 * k2a) * conv;   // :157-158
    const double sn = tac < 0.0 ? 1e-6 : tac;                       // mcmc.py:152
#if MH_RSQ
    const double inv = rsq_f64(sn) * s.SIG[i * NF + lane];         // SIG holds 1/SIG (load_lds)
#else
#if MH_EXP_MODE & 8
    const double sig = sn * s.SIG[i * NF + lane];
#else
    const double sig = sqrt(sn) * s.SIG[i * NF + lane];             // :153
#endif
#if MH_EXP_MODE & 16
    const double inv = sig;
#else
    const double inv = 1.0 / sig;
#endif
#endif
    const double z = (s.Y[i * NF + lane] - sn) * inv;
    const double xs = sn * inv;
    // log Phi(x) for x >= 10 is -7.6e-24 or smaller: 0 at the precision of the sum
#if MH_EXP_MODE & 4
    const double lnd = 0.0;
#else
    const double lnd = xs < 10.0 ? (MH_LOGPHI_POLY ? log_phi_poly(s.LPHI, xs) : log_ndtr(xs)) : 0.0;
#endif
#if MH_RSQ
    l = -0.5 * z * z - 0.9189385332046727 + log_pos(inv) - lnd;      // - log sig = log(1 / sig)
#elif MH_EXP_MODE & 2
    l = -0.5 * z * z - 0.9189385332046727 - sig - lnd;
#else
    l = -0.5 * z * z - 0.9189385332046727 - (MH_FAST_LOG ? log_pos(sig) : log(sig)) - lnd;
#endif
  }
  __builtin_amdgcn_wave_barrier();
  return wave_sum(l);
}
#endif

__device__ void load_lds(Lds& s, const MHConst& c) {
  for (int k = threadIdx.x; k < NF * MLD; k += blockDim.x) {
    const int f = k / MLD, g = k - f * MLD;
    s.M[k] = g < NF ? c.M[g * NF + f] : 0.0;   // global operator is [g][f]
  }
  for (int k = threadIdx.x; k < NR * NR; k += blockDim.x) { s.PD[k] = c.PD[k]; s.PR[k] = c.PR[k]; }
  for (int k = threadIdx.x; k < NR * NF; k += blockDim.x) { s.Y[k] = c.Y[k]; s.SIG[k] = MH_RSQ ? 1.0 / c.SIG[k] : c.SIG[k]; }
  for (int k = threadIdx.x; k < NF; k += blockDim.x) { s.CR[k] = c.CR[k]; s.TV[k] = c.TV[k]; }
  for (int k = threadIdx.x; k < NR; k += blockDim.x) { s.MUD[k] = c.MUD[k]; s.MUR[k] = c.MUR[k]; }
  load_logphi(s.LPHI);
  load_e2(s.E2);
  load_lt(s.LT);
  __syncthreads();
}

__device__ __forceinline__ double tune_scale(double s, double rate) {   // pymc Metropolis tune()
  if (rate < 0.001) return s * 0.1;
  if (rate < 0.05) return s * 0.5;
  if (rate < 0.2) return s * 0.9;
  if (rate > 0.95) return s * 10.0;
  if (rate > 0.75) return s * 2.0;
  if (rate > 0.5) return s * 1.1;
  return s;
}

// One chain per wavefront.  Per draw (pymc 5.12 Metropolis.astep, elemwise_update):
// tune, draw the proposal vector + accept uniforms + the shuffled element order for
// all 96 elements in parallel (lane k: Philox block of element k), then the sequential
// element-wise sweep.  Element k = (v, i): v = 0 DVR / 1 R1, ROI i.  A proposal for
// ROI i changes only ROI i's TAC, so its log ratio vs the running state is
// d_prior + ll_i(new) - ll_i; pymc compares against the sweep-START point, i.e. adds
// the running sum `run` of the sweep's accepted ratios (vs_sweep_start).
__global__ __launch_bounds__(kWaves * 64) void mh_chain_kernel(MHConst c, MHRun r) {
  __shared__ Lds s;
  load_lds(s, c);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  MRow mreg;
  load_mrow(s, mreg, lane);
  double* e = s.E[w];
  double* Zw = s.Z[w];
  double* LUw = s.LU[w];
  uint32_t* KEYw = s.KEY[w];
  int* ORDw = s.ORD[w];
  const bool own = lane < NR;
  const int li = own ? lane : 0;
  const uint32_t sk0 = (uint32_t)(r.seed & 0xffffffffull), sk1 = (uint32_t)(r.seed >> 32);
#if MH_DPP && MH_PF
  const int fl = lane < NF ? lane : 0;
  const double tvr = s.TV[fl], crr = s.CR[fl];   // the lane's frame time and reference TAC, in registers
#endif
  for (int chain = blockIdx.x * kWaves + w; chain < r.n_chains; chain += gridDim.x * kWaves) {
    // ---- state: lane l < 48 holds ROI l
    double D = r.x0 ? r.x0[(size_t)chain * 2 * NR + li] : s.MUD[li];
    double R = r.x0 ? r.x0[(size_t)chain * 2 * NR + NR + li] : s.MUR[li];
    // prior gradients g = P (x - mu)
    e[lane] = own ? D - s.MUD[lane] : 0.0;
    __builtin_amdgcn_wave_barrier();
    double gD = 0.0;
#pragma unroll 1
    for (int k = 0; k < NR; ++k) gD = fma(s.PD[li * NR + k], e[k], gD);
    __builtin_amdgcn_wave_barrier();
    e[lane] = own ? R - s.MUR[lane] : 0.0;
    __builtin_amdgcn_wave_barrier();
    double gR = 0.0;
#pragma unroll 1
    for (int k = 0; k < NR; ++k) gR = fma(s.PR[li * NR + k], e[k], gR);
    __builtin_amdgcn_wave_barrier();
    double ll = 0.0;
#pragma unroll 1
    for (int i = 0; i < NR; ++i) {
      const double di = lane_bcast(D, i), ri = lane_bcast(R, i);
      const double v = roi_loglik(s, mreg, e, lane, i, di, ri, c.k2p);
      if (lane == i) ll = v;
    }
    double sD = r.scaling, sR = r.scaling;
    int aD = 0, aR = 0;                  // accepts in the current tune window
    double accD = 0.0, accR = 0.0;       // accepts over kept draws
    double mD = 0.0, m2D = 0.0, mR = 0.0, m2R = 0.0;
    long long nk = 0;
    const uint32_t ch_lo = (uint32_t)((unsigned long long)chain & 0xffffffffull);
    const uint32_t ch_hi = (uint32_t)((unsigned long long)chain >> 32);
    const int total = r.n_tune + r.n_draws;
    for (int it = 0; it < total; ++it) {
      if (it < r.n_tune && it > 0 && it % r.tune_interval == 0) {
        sD = tune_scale(sD, (double)aD / r.tune_interval);
        sR = tune_scale(sR, (double)aR / r.tune_interval);
        aD = aR = 0;
      }
      // ---- the draw's random numbers, element k on lane k (and k - 64 for k >= 64)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = lane + 64 * h;
        if (k < 2 * NR) {
          uint32_t q[4] = {(uint32_t)k, (uint32_t)it, ch_lo, ch_hi};
          philox(q, sk0, sk1);
          const double u1 = ((double)q[0] + 1.0) * 2.3283064365386963e-10;
          const double u2 = ((double)q[1] + 0.5) * 2.3283064365386963e-10;
          Zw[k] = sqrt(-2.0 * log(u1)) * cospi(2.0 * u2);
          LUw[k] = log(((double)q[2] + 0.5) * 2.3283064365386963e-10);
          KEYw[k] = q[3];
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      // ---- shuffled order: rank of (key, k) among the 96 elements
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = lane + 64 * h;
        if (k < 2 * NR) {
          const uint32_t kk = KEYw[k];
          int rank = 0;
#pragma unroll 8
          for (int j = 0; j < 2 * NR; ++j) {
            const uint32_t kj = KEYw[j];
            rank += (kj < kk) | ((kj == kk) & (j < k));
          }
          ORDw[rank] = k;
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      double run = 0.0;                  // log p(running) - log p(sweep start)
#if MH_PF
      // element j's (k, Z_k, log u_k) were read during element j - 1, element j + 1's order index during j - 1
      int k_cur = __builtin_amdgcn_readfirstlane(ORDw[0]);
      int k_nxt = __builtin_amdgcn_readfirstlane(ORDw[1]);
      double z_cur = Zw[k_cur], lu_cur = LUw[k_cur];
#if MH_DPP
      const int ic0 = k_cur >= NR ? k_cur - NR : k_cur;   // ROI i's Y and 1/SIG rows, also one element ahead
      double y_cur = s.Y[ic0 * NF + fl], g_cur = s.SIG[ic0 * NF + fl];
#endif
#endif
#pragma unroll 1
      for (int j = 0; j < 2 * NR; ++j) {
#if MH_PF
        const int k = k_cur;
        const int ord2 = ORDw[j + 2 < 2 * NR ? j + 2 : 2 * NR - 1];
        const double z_nxt = Zw[k_nxt], lu_nxt = LUw[k_nxt];
        const double zk = z_cur, luk = lu_cur;
#if MH_DPP
        const int inx = k_nxt >= NR ? k_nxt - NR : k_nxt;
        const double y_nxt = s.Y[inx * NF + fl], g_nxt = s.SIG[inx * NF + fl];
#endif
#else
        const int k = __builtin_amdgcn_readfirstlane(ORDw[j]);
#endif
        const int v = k >= NR, i = v ? k - NR : k;
        const double* P = v ? s.PR : s.PD;
#if MH_PF
        const double pii = P[i * NR + i], pli = P[li * NR + i];
#endif
        const double Di = lane_bcast(D, i), Ri = lane_bcast(R, i);
        const double xi = v ? Ri : Di;
#if MH_SEL_BCAST
        // the element's scale and prior gradient: per-lane select on the (uniform) v, then one broadcast each
        // (no branch between two readlane pairs)
        const double si = lane_bcast(v ? sR : sD, i);
        const double gi = lane_bcast(v ? gR : gD, i);
#else
        const double si = v ? lane_bcast(sR, i) : lane_bcast(sD, i);
        const double gi = v ? lane_bcast(gR, i) : lane_bcast(gD, i);
#endif
        const double lli = lane_bcast(ll, i);
#if MH_PF
        const double delta = zk * si;
#else
        const double delta = Zw[k] * si;
#endif
        const double xp = xi + delta;
#if MH_DPP && MH_PF
        const double lln = roi_loglik_r(s, mreg, lane, tvr, crr, y_cur, g_cur, v ? Di : xp, v ? xp : Ri, c.k2p);
#else
        const double lln = roi_loglik(s, mreg, e, lane, i, v ? Di : xp, v ? xp : Ri, c.k2p);
#endif
#if MH_PF
        const double dprior = -0.5 * (2.0 * delta * gi + delta * delta * pii);
#else
        const double dprior = -0.5 * (2.0 * delta * gi + delta * delta * P[i * NR + i]);
#endif
        const double step = dprior + lln - lli;
        const double mr = r.vs_sweep_start ? run + step : step;
#if MH_PF
        const bool acc_ = isfinite(mr) && luk < mr;
        k_cur = k_nxt;
        z_cur = z_nxt;
        lu_cur = lu_nxt;
#if MH_DPP
        y_cur = y_nxt;
        g_cur = g_nxt;
#endif
        k_nxt = __builtin_amdgcn_readfirstlane(ord2);
#else
        const bool acc_ = isfinite(mr) && LUw[k] < mr;
#endif
        if (acc_) {   // wave-uniform decision (metrop_select)
          run += step;
          if (lane == i) {
            if (v == 0) { D = xp; aD += 1; if (it >= r.n_tune) accD += 1.0; }
            else { R = xp; aR += 1; if (it >= r.n_tune) accR += 1.0; }
            ll = lln;
          }
          if (own) {
#if MH_PF
            if (v == 0) gD = fma(delta, pli, gD);
            else gR = fma(delta, pli, gR);
#else
            if (v == 0) gD = fma(delta, P[lane * NR + i], gD);
            else gR = fma(delta, P[lane * NR + i], gR);
#endif
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
      if (it >= r.n_tune) {              // Welford over kept draws
        if (r.draws && own) {            // optional trace [chain][draw][DVR 48 | R1 48] (mcmc.py idata)
          double* dr = r.draws + ((size_t)chain * r.n_draws + (it - r.n_tune)) * 2 * NR;
          dr[lane] = D;
          dr[NR + lane] = R;
        }
        ++nk;
        const double dd = D - mD;
        mD += dd / (double)nk;
        m2D = fma(dd, D - mD, m2D);
        const double dr = R - mR;
        mR += dr / (double)nk;
        m2R = fma(dr, R - mR, m2R);
      }
    }
    if (own) {
      double* st = r.stats + (size_t)chain * 2 * NR * 3;
      st[lane * 3 + 0] = (double)nk;
      st[lane * 3 + 1] = mD;
      st[lane * 3 + 2] = m2D;
      st[(NR + lane) * 3 + 0] = (double)nk;
      st[(NR + lane) * 3 + 1] = mR;
      st[(NR + lane) * 3 + 2] = m2R;
      if (r.accept) {
        r.accept[(size_t)chain * 2 * NR + lane] = accD;
        r.accept[(size_t)chain * 2 * NR + NR + lane] = accR;
      }
      if (r.last) {
        r.last[(size_t)chain * 2 * NR + lane] = D;
        r.last[(size_t)chain * 2 * NR + NR + lane] = R;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Batched-proposal sampler (the default chain kernel).
//
// Within one draw every proposal is known before the sweep starts: element (v, i) proposes
// x_i + Z_k s_k, whatever happened earlier in the sweep.  Its ROI-i likelihood depends on the
// sweep only through the OTHER element of ROI i (proposed-and-accepted earlier, or not).  So the
// three likelihoods a sweep can ask of ROI i,
//   c = 0: (DVR', R1)   c = 1: (DVR, R1')   c = 2: (DVR', R1')
// are evaluated up front for all 48 ROIs (144 evaluations, no sequential dependence: batches of
// kQ evaluations share one operator-row read per frame and keep kQ independent FMA chains in
// flight), and the sweep itself (pymc order, vs the sweep start) becomes a scan over
// wave-uniform scalars that picks the evaluation each element needs.  Same expressions per
// evaluation as roi_loglik (the operator row FMAs in the same order), so the chain path is the
// oracle's up to the summation order over frames.
//
// WPC waves cooperate on one chain (the 144 evaluations are dealt to them, the scan runs
// redundantly in every wave, identical decisions): WPC = 1 for throughput (10k chains),
// WPC = kBW for few chains (the reference's 4-chain protocol is latency bound).
// ---------------------------------------------------------------------------
// diagnostic builds only (scripts/micro/build_mh.sh): bit 1 drops the per-frame transcendentals,
// 2 the exponentials of e, 4 the operator FMAs, 8 the sweep scan, 16 the sweep's RNG + sort
#ifndef MH_BEXP
#define MH_BEXP 0
#endif
// scan: 0 = branch-free state updates, 1 = updates behind a branch on the decision (faster: 0.67
// vs 0.74 us per element at 4 chains, profiles/r02/mh)
#ifndef MH_SCAN_BRANCH
#define MH_SCAN_BRANCH 1
#endif
// per-frame transcendental loop: evaluations in flight per wave
#ifndef MH_T_UNROLL
#define MH_T_UNROLL 1
#endif
#ifndef MH_P_UNROLL
#define MH_P_UNROLL 1
#endif
#ifndef MH_Q
#define MH_Q 4
#endif
constexpr int kQ = MH_Q;              // evaluations per batch (144 = 36 batches of 4: 3 per wave at 12 waves)
static_assert(kQ == 4 || kQ == 8, "frame-sum lane groups of 16 or 8");
#ifndef MH_BW
#define MH_BW 12
#endif
constexpr int kBW = MH_BW;            // waves per workgroup
constexpr int kNE = 3 * NR;           // evaluations per draw
// per-wave scratch (doubles): the batch's e rows / frame terms, or the sweep draws Z[96] LU[96]
// KEY[96] (u32) ORD[96] (i32)
constexpr int kWD = kQ * 64 > 6 * NR ? kQ * 64 : 6 * NR;
static_assert(kQ * MLD <= kWD && kQ * 64 <= kWD && 6 * NR <= kWD, "per-wave scratch");

struct LdsB {
  double M[NF * MLD];
  double PD[NR * NR], PR[NR * NR];    // prior precisions (the sweep's prior-gradient updates)
  double Y[NR * NF], SIG[NR * NF];
  double CR[NF], TV[NF];
  double MUD[NR], MUR[NR];
  alignas(16) double LPHI[LPNI * LPLD];   // log Phi polynomial (16-B aligned rows)
  double E2[kE2];                         // 2^(j/64) (MH_TEXP)
  double2 LT[kLT];                        // (1/c_j, -log(1/c_j)) (MH_TLOG)
  double W[kBW][kWD];                 // per wave: e rows [q][MLD] / frame terms [q][64] / sweep draws
  double P[kBW][kQ * 4];              // per wave: the batch's (R1, k2, k2a, roi)
  double LL[kBW][kNE];                // per chain group: the draw's evaluations
  double SH[kBW / 2][4 * NR];         // waves_per_chain > 1: the leader's D, R, D', R' per draw
};

// kQ log-likelihoods.  Lane q < kQ brings evaluation q's (roi, DVR, R1) in (my_roi, my_dvr,
// my_r1); the results come back wave-uniform in out[q].  W / P: this wave's scratch.
// mcmc.py:151-155 per frame; the 54-frame sum is a strided partial per lane plus a DPP tree
// inside each group of 64 / kQ lanes (the group's last lane ends with its evaluation).  The transcendental part
// runs one evaluation at a time (not unrolled: the fp64 exp / log / erfc constants would
// otherwise be hoisted into registers kQ times over); the operator FMAs run kQ chains at once.
__device__ __forceinline__ void eval_batch(const LdsB& s, double* W, double* P, int lane, int my_roi, double my_dvr,
                                           double my_r1, double k2p, double (&out)[kQ]) {
  if (lane < kQ) {
    const double k2 = k2p * my_r1;       // kinetic_model.py:153-154
    P[lane * 4 + 0] = my_r1;
    P[lane * 4 + 1] = k2;
    P[lane * 4 + 2] = k2 / my_dvr;
    P[lane * 4 + 3] = (double)my_roi;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  const int f = lane < NF ? lane : 0;
  if (lane < MLD) {
    const double tv = s.TV[f];
#pragma unroll 1
    for (int q = 0; q < kQ; ++q)
      W[q * MLD + lane] = lane < NF ? ((MH_BEXP & 2) ? 1.0 - P[q * 4 + 2] * tv
                                                     : MH_TEXP ? exp_tab(s.E2, -P[q * 4 + 2] * tv) : exp(-P[q * 4 + 2] * tv))
                                    : 0.0;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  double c0[kQ], c1[kQ];
#pragma unroll
  for (int q = 0; q < kQ; ++q) c0[q] = c1[q] = 0.0;
  if (lane < NF && !(MH_BEXP & 4)) {
    const double2* mrow = reinterpret_cast<const double2*>(s.M + lane * MLD);
#pragma unroll MH_P_UNROLL
    for (int p = 0; p < MLD / 2; ++p) {
      const double2 m = mrow[p];
#pragma unroll
      for (int q = 0; q < kQ; ++q) {
        const double2 x = reinterpret_cast<const double2*>(W + q * MLD)[p];
        c0[q] = fma(m.x, x.x, c0[q]);
        c1[q] = fma(m.y, x.y, c1[q]);
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
  for (int q = 0; q < kQ; ++q) W[q * 64 + lane] = c0[q] + c1[q];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  const double crf = s.CR[f];
#pragma unroll MH_T_UNROLL
  for (int q = 0; q < kQ; ++q) {
    double l = 0.0;
    if (lane < NF) {
      const double r1 = P[q * 4 + 0], k2 = P[q * 4 + 1], k2a = P[q * 4 + 2];
      const int i = (int)P[q * 4 + 3];
      const double conv = W[q * 64 + lane];
      const double tac = r1 * crf + (k2 - r1 * k2a) * conv;                // :157-158
      const double sn = tac < 0.0 ? 1e-6 : tac;                           // mcmc.py:152
#if MH_BEXP & 1
      const double sig = sn * s.SIG[i * NF + lane];
      const double z = (s.Y[i * NF + lane] - sn) * sig;
      l = -0.5 * z * z - 0.9189385332046727 - sig;
#else
#if MH_RSQ
      const double inv = rsq_f64(sn) * s.SIG[i * NF + lane];             // SIG holds 1/SIG
#else
      const double sig = sqrt(sn) * s.SIG[i * NF + lane];                 // :153
      const double inv = 1.0 / sig;
#endif
      const double z = (s.Y[i * NF + lane] - sn) * inv;
      const double xs = sn * inv;
      // log Phi(xs) (log_ndtr): xs = sqrt(sn) / SIG >= 0 or NaN, so only its x > -1 branch
      // log(erfc(-x / sqrt 2) / 2) is reachable (NaN falls through to NaN either way)
      const double lnd = xs < 10.0 ? (MH_LOGPHI_POLY ? log_phi_poly(s.LPHI, xs)
                                                      : log(0.5 * erfc(-xs * 0.7071067811865476))) : 0.0;
#if MH_RSQ
      l = -0.5 * z * z - 0.9189385332046727 + (MH_TLOG ? log_tab(s.LT, inv) : log_pos(inv)) - lnd;
#else
      l = -0.5 * z * z - 0.9189385332046727 - (MH_FAST_LOG ? log_pos(sig) : log(sig)) - lnd;
#endif
#endif
    }
    W[q * 64 + lane] = l;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  constexpr int G = 64 / kQ;            // lanes per evaluation
  const int qq = lane / G, pp = lane % G;
  double sum = 0.0;
#pragma unroll
  for (int m = 0; m < kQ; ++m) sum += W[qq * 64 + pp + G * m];
  sum += dpp_f64<0x111>(sum);          // row_shr:1
  sum += dpp_f64<0x112>(sum);          // row_shr:2
  sum += dpp_f64<0x114>(sum);          // row_shr:4 -> lanes 7 / 15 of each row: their 8-lane group
  if constexpr (G == 16) sum += dpp_f64<0x118>(sum);   // row_shr:8 -> lane 15: the row
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int q = 0; q < kQ; ++q) out[q] = lane_bcast(sum, G * q + G - 1);
}

template <int WPC>
__global__ __launch_bounds__(kBW * 64) void mh_chain_batched(MHConst c, MHRun r) {
  constexpr int CPG = kBW / WPC;       // chains per workgroup
  __shared__ LdsB s;
  for (int k = threadIdx.x; k < NF * MLD; k += blockDim.x) {
    const int f = k / MLD, g = k - f * MLD;
    s.M[k] = g < NF ? c.M[g * NF + f] : 0.0;   // global operator is [g][f]
  }
  for (int k = threadIdx.x; k < NR * NF; k += blockDim.x) { s.Y[k] = c.Y[k]; s.SIG[k] = MH_RSQ ? 1.0 / c.SIG[k] : c.SIG[k]; }
  for (int k = threadIdx.x; k < NR * NR; k += blockDim.x) { s.PD[k] = c.PD[k]; s.PR[k] = c.PR[k]; }
  for (int k = threadIdx.x; k < NF; k += blockDim.x) { s.CR[k] = c.CR[k]; s.TV[k] = c.TV[k]; }
  for (int k = threadIdx.x; k < NR; k += blockDim.x) { s.MUD[k] = c.MUD[k]; s.MUR[k] = c.MUR[k]; }
  load_logphi(s.LPHI);
  load_e2(s.E2);
  load_lt(s.LT);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int grp = w / WPC, rk = w - grp * WPC;
  double* W = s.W[w];
  double* Pw = s.P[w];
  double* LLg = s.LL[grp];
  const bool own = lane < NR;
  const int li = own ? lane : 0;
  const uint32_t sk0 = (uint32_t)(r.seed & 0xffffffffull), sk1 = (uint32_t)(r.seed >> 32);
  const double PDd = s.PD[li * NR + li], PRd = s.PR[li * NR + li];
  // the chain loop is uniform over the workgroup (its barriers): groups past the last chain
  // run a copy of the last one and store nothing
  for (int base = blockIdx.x * CPG; base < r.n_chains; base += gridDim.x * CPG) {
    const bool live = base + grp < r.n_chains;
    if constexpr (WPC == 1) {          // no workgroup barriers: a wave past the end just leaves
      if (!live) break;
    }
    const int chain = live ? base + grp : r.n_chains - 1;
    const bool store = live && rk == 0;
    double D = r.x0 ? r.x0[(size_t)chain * 2 * NR + li] : s.MUD[li];
    double R = r.x0 ? r.x0[(size_t)chain * 2 * NR + NR + li] : s.MUR[li];
    // prior gradients g = P (x - mu) (same FMA order as mh_chain_kernel)
    W[lane] = own ? D - s.MUD[lane] : 0.0;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    double gD = 0.0;
#pragma unroll 1
    for (int k = 0; k < NR; ++k) gD = fma(s.PD[li * NR + k], W[k], gD);
    __builtin_amdgcn_wave_barrier();
    W[lane] = own ? R - s.MUR[lane] : 0.0;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    double gR = 0.0;
#pragma unroll 1
    for (int k = 0; k < NR; ++k) gR = fma(s.PR[li * NR + k], W[k], gR);
    __builtin_amdgcn_wave_barrier();
    // the state's per-ROI log-likelihoods: 48 evaluations
#pragma unroll 1
    for (int b = rk; b < NR / kQ; b += WPC) {
      // lane q < kQ: ROI b kQ + q at the state
      const int mi = b * kQ + (lane & (kQ - 1));
      double out[kQ];
      eval_batch(s, W, Pw, lane, mi, __shfl(D, mi), __shfl(R, mi), c.k2p, out);
      double o = out[0];
#pragma unroll
      for (int q = 1; q < kQ; ++q) o = lane == q ? out[q] : o;
      if (lane < kQ) LLg[b * kQ + lane] = o;
    }
    if constexpr (WPC > 1) __syncthreads();
    else { __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); }
    double ll = LLg[li];
    if constexpr (WPC > 1) __syncthreads();
    double sD = r.scaling, sR = r.scaling;
    int aD = 0, aR = 0;
    double accD = 0.0, accR = 0.0;
    double mD = 0.0, m2D = 0.0, mR = 0.0, m2R = 0.0;
    long long nk = 0;
    const uint32_t ch_lo = (uint32_t)((unsigned long long)chain & 0xffffffffull);
    const uint32_t ch_hi = (uint32_t)((unsigned long long)chain >> 32);
    const int total = r.n_tune + r.n_draws;
    double* Zw = W;                    // sweep draws in the wave's scratch: Z[96] LU[96] KEY[96] ORD[96]
    double* LUw = W + 2 * NR;
    uint32_t* KEYw = reinterpret_cast<uint32_t*>(W + 4 * NR);
    int* ORDw = reinterpret_cast<int*>(W + 5 * NR);
    // waves_per_chain > 1: the group's first wave (the leader) alone tunes, draws the sweep's random
    // numbers, scans and keeps the statistics; it hands D, R and the proposals to the others
    // through LDS once per draw (a redundant scan in every wave would triple its issue cost)
    const bool lead = WPC == 1 || rk == 0;
    // the sweep's random numbers of draw `itn` (N(0,1) proposals, log accept uniforms, shuffled
    // order) into the scratch of the wave that runs it
    auto draw_rng = [&](int itn, double* Zx, double* LUx, uint32_t* KEYx, int* ORDx) {
      if (MH_BEXP & 16) {                  // diagnostic: identity order, no RNG
        for (int h = 0; h < 2; ++h) {
          const int k = lane + 64 * h;
          if (k < 2 * NR) { Zx[k] = 0.5; LUx[k] = -1.0; ORDx[k] = k; }
        }
        return;
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = lane + 64 * h;
        if (k < 2 * NR) {
          uint32_t q[4] = {(uint32_t)k, (uint32_t)itn, ch_lo, ch_hi};
          philox(q, sk0, sk1);
          const double u1 = ((double)q[0] + 1.0) * 2.3283064365386963e-10;
          const double u2 = ((double)q[1] + 0.5) * 2.3283064365386963e-10;
          Zx[k] = sqrt(-2.0 * log(u1)) * cospi(2.0 * u2);
          LUx[k] = log(((double)q[2] + 0.5) * 2.3283064365386963e-10);
          KEYx[k] = q[3];
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = lane + 64 * h;
        if (k < 2 * NR) {
          const uint32_t kk = KEYx[k];
          int rank = 0;
#pragma unroll 8
          for (int j = 0; j < 2 * NR; ++j) {
            const uint32_t kj = KEYx[j];
            rank += (kj < kk) | ((kj == kk) & (j < k));
          }
          ORDx[rank] = k;
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    };
    // waves_per_chain > 1: the group's second wave draws the NEXT draw's random numbers while the
    // leader scans (they do not depend on the sweep), into its own scratch; the leader reads them
    // after the end-of-draw barrier
    double* Wh = s.W[grp * WPC + (WPC > 1 ? 1 : 0)];
    if constexpr (WPC > 1) {               // the first draw's numbers come from the helper too
      if (rk == 1 && total > 0)
        draw_rng(0, Wh, Wh + 2 * NR, reinterpret_cast<uint32_t*>(Wh + 4 * NR), reinterpret_cast<int*>(Wh + 5 * NR));
      __syncthreads();
    }
    for (int it = 0; it < total; ++it) {
      double dD = 0.0, dR = 0.0, luD = 0.0, luR = 0.0;
      int ordA = 0, ordB = 0;
      if (lead) {
        if (it < r.n_tune && it > 0 && it % r.tune_interval == 0) {
          sD = tune_scale(sD, (double)aD / r.tune_interval);
          sR = tune_scale(sR, (double)aR / r.tune_interval);
          aD = aR = 0;
        }
        double* Zs = Wh;                   // waves_per_chain > 1: the helper's draw
        if constexpr (WPC == 1) {
          draw_rng(it, Zw, LUw, KEYw, ORDw);
          Zs = Zw;
        }
        const double* LUs = Zs + 2 * NR;
        const int* ORDs = reinterpret_cast<const int*>(Zs + 5 * NR);
        // to registers: lane i holds its ROI's two proposals / accept uniforms, lane j the order
        dD = Zs[li] * sD;
        dR = Zs[NR + li] * sR;
        luD = LUs[li];
        luR = LUs[NR + li];
        ordA = ORDs[lane];
        ordB = ORDs[64 + (lane & 31)];
        __builtin_amdgcn_wave_barrier();
      }
      double pD = D + dD, pR = R + dR;
      if constexpr (WPC > 1) {
        double* SHg = s.SH[grp];
        if (lead && own) {
          SHg[lane] = D;
          SHg[NR + lane] = R;
          SHg[2 * NR + lane] = pD;
          SHg[3 * NR + lane] = pR;
        }
        __syncthreads();
        if (!lead) {
          D = SHg[li];
          R = SHg[NR + li];
          pD = SHg[2 * NR + li];
          pR = SHg[3 * NR + li];
        }
      }
      // the 144 evaluations, dealt to the chain's waves by batch
#pragma unroll 1
      for (int b = rk; b < kNE / kQ; b += WPC) {
        // lane q < kQ: evaluation n = b kQ + q = 3 i + cc
        const int n = b * kQ + (lane & (kQ - 1)), mi = n / 3, cc = n - 3 * mi;
        const double sd = __shfl(D, mi), spd = __shfl(pD, mi), sr = __shfl(R, mi), spr = __shfl(pR, mi);
        double out[kQ];
        eval_batch(s, W, Pw, lane, mi, cc == 1 ? sd : spd, cc == 0 ? sr : spr, c.k2p, out);
        double o = out[0];
#pragma unroll
        for (int q = 1; q < kQ; ++q) o = lane == q ? out[q] : o;
        if (lane < kQ) LLg[b * kQ + lane] = o;
      }
      if constexpr (WPC > 1) __syncthreads();
      else { __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); }
      if (WPC > 1 && rk == 1 && it + 1 < total) {
        uint32_t* KEYh = reinterpret_cast<uint32_t*>(Wh + 4 * NR);
        draw_rng(it + 1, Wh, Wh + 2 * NR, KEYh, reinterpret_cast<int*>(Wh + 5 * NR));
      }
      // (the leader reads LLg below; the others next write it after the next draw's hand-off
      // barrier, which the leader joins only after its scan)
      // ---- the sweep: wave-uniform scan over the shuffled order.  An accept adds delta times
      // column i of P to g (P is exactly symmetric, spd_inverse: column i = row i, read from LDS).
      double run = 0.0;
      unsigned long long fD = 0ull, fR = 0ull;   // elements accepted so far in this sweep
      // scan-order tables: lane j holds element ORD[j]'s (ORD[64 + j]'s in the *B set) proposal
      // step, P_ii, log accept uniform and its two candidate likelihoods (the other element of
      // its ROI not accepted / accepted), so a step broadcasts them by its own index j and only
      // g_i and ll_i wait on the previous decisions
#define PETMH_TAB(ordX, kX, dlX, piX, uX, lnX, lyX)                                            \
  const int kX = ordX;                                                                        \
  double dlX, piX, uX, lnX, lyX;                                                              \
  {                                                                                           \
    const bool v_ = kX >= NR;                                                                 \
    const int i_ = v_ ? kX - NR : kX;                                                         \
    const double dd_ = __shfl(dD, i_), dr_ = __shfl(dR, i_);                                  \
    const double pd_ = __shfl(PDd, i_), pr_ = __shfl(PRd, i_);                                \
    const double ud_ = __shfl(luD, i_), ur_ = __shfl(luR, i_);                                \
    dlX = v_ ? dr_ : dd_;                                                                     \
    piX = v_ ? pr_ : pd_;                                                                     \
    uX = v_ ? ur_ : ud_;                                                                      \
    lnX = LLg[3 * i_ + (v_ ? 1 : 0)];                                                         \
    lyX = LLg[3 * i_ + 2];                                                                    \
  }
      PETMH_TAB(ordA, kA, dlA, piA, uA, lnA, lyA)
      PETMH_TAB(ordB, kB, dlB, piB, uB, lnB, lyB)
#undef PETMH_TAB
// one element of the sweep; the state updates sit behind the (wave-uniform) decision
#define PETMH_STEP(jl, kX, dlX, piX, uX, lnX, lyX)                                             \
  {                                                                                           \
    const int k = __builtin_amdgcn_readlane(kX, (jl));                                        \
    const bool v = k >= NR;                                                                   \
    const int i = v ? k - NR : k;                                                             \
    const double prw = (v ? s.PR : s.PD)[i * NR + li];   /* column i = row i (P symmetric) */ \
    const double delta = lane_bcast(dlX, (jl));                                               \
    const double pii = lane_bcast(piX, (jl));                                                 \
    const double lu = lane_bcast(uX, (jl));                                                   \
    const double lno = lane_bcast(lnX, (jl)), lyes = lane_bcast(lyX, (jl));                   \
    const double gi = lane_bcast(v ? gR : gD, i);                                             \
    const double lli = lane_bcast(ll, i);                                                     \
    const bool oth = ((v ? fD : fR) >> i) & 1ull;                                             \
    const double lln = oth ? lyes : lno;                                                      \
    const double dprior = -0.5 * (2.0 * delta * gi + delta * delta * pii);                    \
    const double step = dprior + lln - lli;                                                   \
    const double mr = r.vs_sweep_start ? run + step : step;                                   \
    const bool acc = isfinite(mr) && lu < mr; /* wave-uniform decision (metrop_select) */     \
    if (!MH_SCAN_BRANCH || acc) {                                                             \
      run = acc ? run + step : run;                                                           \
      const unsigned long long bit = acc ? 1ull << i : 0ull;                                  \
      fR |= v ? bit : 0ull;                                                                   \
      fD |= v ? 0ull : bit;                                                                   \
      const bool mine = acc && lane == i;                                                     \
      D = (mine && !v) ? pD : D;                                                              \
      R = (mine && v) ? pR : R;                                                               \
      ll = mine ? lln : ll;                                                                   \
      aD += (mine && !v) ? 1 : 0;                                                             \
      aR += (mine && v) ? 1 : 0;                                                              \
      accD += (mine && !v && kept) ? 1.0 : 0.0;                                               \
      accR += (mine && v && kept) ? 1.0 : 0.0;                                                \
      /* fma(0, finite row, g) == g: the unselected g is unchanged */                          \
      gD = fma((acc && !v) ? delta : 0.0, prw, gD);                                           \
      gR = fma((acc && v) ? delta : 0.0, prw, gR);                                            \
    }                                                                                         \
  }
      if (lead && !(MH_BEXP & 8)) {
        const bool kept = it >= r.n_tune;
#pragma unroll 1
        for (int j = 0; j < 64; j += 4) {
          PETMH_STEP(j, kA, dlA, piA, uA, lnA, lyA)
          PETMH_STEP(j + 1, kA, dlA, piA, uA, lnA, lyA)
          PETMH_STEP(j + 2, kA, dlA, piA, uA, lnA, lyA)
          PETMH_STEP(j + 3, kA, dlA, piA, uA, lnA, lyA)
        }
#pragma unroll 1
        for (int j = 0; j < 2 * NR - 64; j += 4) {
          PETMH_STEP(j, kB, dlB, piB, uB, lnB, lyB)
          PETMH_STEP(j + 1, kB, dlB, piB, uB, lnB, lyB)
          PETMH_STEP(j + 2, kB, dlB, piB, uB, lnB, lyB)
          PETMH_STEP(j + 3, kB, dlB, piB, uB, lnB, lyB)
        }
      }
#undef PETMH_STEP
      if (lead && it >= r.n_tune) {
        if (r.draws && own && store) {
          double* dr = r.draws + ((size_t)chain * r.n_draws + (it - r.n_tune)) * 2 * NR;
          dr[lane] = D;
          dr[NR + lane] = R;
        }
        ++nk;
        const double dd = D - mD;
        mD += dd / (double)nk;
        m2D = fma(dd, D - mD, m2D);
        const double dr = R - mR;
        mR += dr / (double)nk;
        m2R = fma(dr, R - mR, m2R);
      }
      if constexpr (WPC > 1) __syncthreads();   // the helper's next draw is in its scratch
    }
    if (own && store) {
      double* st = r.stats + (size_t)chain * 2 * NR * 3;
      st[lane * 3 + 0] = (double)nk;
      st[lane * 3 + 1] = mD;
      st[lane * 3 + 2] = m2D;
      st[(NR + lane) * 3 + 0] = (double)nk;
      st[(NR + lane) * 3 + 1] = mR;
      st[(NR + lane) * 3 + 2] = m2R;
      if (r.accept) {
        r.accept[(size_t)chain * 2 * NR + lane] = accD;
        r.accept[(size_t)chain * 2 * NR + NR + lane] = accR;
      }
      if (r.last) {
        r.last[(size_t)chain * 2 * NR + lane] = D;
        r.last[(size_t)chain * 2 * NR + NR + lane] = R;
      }
    }
  }
}

// Joint log density at n points (one wave per point).
__global__ __launch_bounds__(kWaves * 64) void mh_logp_kernel(MHConst c, const double* x, int n, double* out) {
  __shared__ Lds s;
  load_lds(s, c);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  MRow mreg;
  load_mrow(s, mreg, lane);
  double* e = s.E[w];
  const int li = lane < NR ? lane : 0;
  for (int pt = blockIdx.x * kWaves + w; pt < n; pt += gridDim.x * kWaves) {
    const double D = x[(size_t)pt * 2 * NR + li], R = x[(size_t)pt * 2 * NR + NR + li];
    double ll = 0.0;
    for (int i = 0; i < NR; ++i) ll += roi_loglik(s, mreg, e, lane, i, lane_bcast(D, i), lane_bcast(R, i), c.k2p);
    // MvNormal quadratic forms
    double q = 0.0;
    for (int v = 0; v < 2; ++v) {
      const double* P = v == 0 ? s.PD : s.PR;
      const double* mu = v == 0 ? s.MUD : s.MUR;
      const double xv = v == 0 ? D : R;
      e[lane] = lane < NR ? xv - mu[lane] : 0.0;
      __builtin_amdgcn_wave_barrier();
      double gi = 0.0;
      if (lane < NR)
        for (int k = 0; k < NR; ++k) gi = fma(P[lane * NR + k], e[k], gi);
      q += wave_sum(lane < NR ? gi * e[lane] : 0.0);
      __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0) out[pt] = ll - 0.5 * q + c.prior_const;
  }
}

// Batched SRTM2 forward: one wave per (row, roi); tac [n][n_roi][NF].
__global__ void srtm2_kernel(const double* M, const double* cr, const double* tv, const double* dvr,
                             const double* r1, const double* k2p, int n, int n_roi, double* tac) {
  __shared__ double e[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int item = blockIdx.x * 4 + w;
  if (item >= n * n_roi) return;
  const int row = item / n_roi;
  const double R = r1[item], D = dvr[item];
  const double k2 = k2p[row] * R, k2a = k2 / D;
  if (lane < NF) e[w][lane] = exp(-k2a * tv[lane]);
  __builtin_amdgcn_wave_barrier();
  if (lane < NF) {
    double conv = 0.0;
    for (int g = 0; g < NF; ++g) conv = fma(M[g * NF + lane], e[w][g], conv);
    tac[(size_t)item * NF + lane] = R * cr[lane] + (k2 - R * k2a) * conv;
  }
}

template <int WPC>
static hipError_t launch_batched(const MHConst& c, const MHRun& r, hipStream_t st) {
  constexpr int CPG = kBW / WPC;
  int grid = (r.n_chains + CPG - 1) / CPG;
  if (grid > 256 * 16) grid = 256 * 16;
  hipLaunchKernelGGL(mh_chain_batched<WPC>, dim3(grid), dim3(kBW * 64), 0, st, c, r);
  return hipGetLastError();
}

// Kernel choice: MHRun.kernel / .wpc (petmh_set_kernel), else the environment (PETMH_KERNEL=wave |
// batched, PETMH_WPC; A/B scripts), else automatic: the batched kernel for up to 256 chains
// (12 waves per chain: the reference's 4-chain protocol is latency bound), one update at a time
// above (one wave per chain fills the chip; it issues fewer instructions per chain-step).
hipError_t launch_mh_chains(const MHConst& c, const MHRun& r, hipStream_t st) {
  if (r.n_chains <= 0) return hipSuccess;
  static const int kind_env = [] {
    const char* e = getenv("PETMH_KERNEL");
    return !e ? 0 : e[0] == 'w' ? 1 : e[0] == 'b' ? 2 : 0;
  }();
  static const int wpc_env = [] {
    const char* e = getenv("PETMH_WPC");
    return e ? atoi(e) : 0;
  }();
  int kind = r.kernel ? r.kernel : kind_env;
  if (kind == 0) kind = r.n_chains <= 256 ? 2 : 1;
  if (kind == 2) {
    static_assert(kBW % 4 == 0 && kBW > 4, "waves per chain 1, 2, 4 or kBW");
    int wpc = r.wpc ? r.wpc : wpc_env;
    if (wpc <= 0) {
      wpc = 1;
      for (const int nx : {2, 4, kBW})
        if ((long long)r.n_chains * nx <= 256LL * kBW) wpc = nx;
    }
    switch (wpc) {
      case 1: return launch_batched<1>(c, r, st);
      case 2: return launch_batched<2>(c, r, st);
      case 4: return launch_batched<4>(c, r, st);
      default: return launch_batched<kBW>(c, r, st);
    }
  }
  int grid = (r.n_chains + kWaves - 1) / kWaves;
  if (grid > 256 * 4) grid = 256 * 4;
  hipLaunchKernelGGL(mh_chain_kernel, dim3(grid), dim3(kWaves * 64), 0, st, c, r);
  return hipGetLastError();
}

hipError_t launch_mh_logp(const MHConst& c, const double* x, int n, double* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  int grid = (n + kWaves - 1) / kWaves;
  if (grid > 1024) grid = 1024;
  hipLaunchKernelGGL(mh_logp_kernel, dim3(grid), dim3(kWaves * 64), 0, st, c, x, n, out);
  return hipGetLastError();
}

hipError_t launch_srtm2(const double* M, const double* cr, const double* tv, const double* dvr, const double* r1,
                        const double* k2p, int n, int n_roi, double* tac, hipStream_t st) {
  const int items = n * n_roi;
  if (items <= 0) return hipSuccess;
  hipLaunchKernelGGL(srtm2_kernel, dim3((items + 3) / 4), dim3(256), 0, st, M, cr, tv, dvr, r1, k2p, n, n_roi, tac);
  return hipGetLastError();
}

}  // namespace petmh
