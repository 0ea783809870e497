// CDNA4 (gfx950) kernels of the iDDPM posterior sampler hot path.
//
// Reference being replaced (yanisdjebra/PET_posterior_distribution):
//   UnetConditional.call           networks.py:994-1093  (conv blocks, skips, cond concat)
//   ConvBlock.call                 networks.py:679-691   (relu(conv_k6 + conv_1x1))
//   SinusoidalPosEmb / GELU        networks.py:189-198, 236-241
//   Encoder_v3_noskip              networks.py:574-586
//   ImprovedDDPM.p_mean_variance   diffusion_model.py:424-496
//   ImprovedDDPM.ddpm (p_sample)   diffusion_model.py:651-663
//
// Design: activations are channels-last rows [sample*L + l][C] in
// HBM.  Every x-dependent Conv1D is an implicit GEMM  M = B*L, N = Cout,
// K = taps*Cin  on MFMA (bf16 32x32x16 or exact-f32 32x32x2).  A workgroup owns
// 192 rows = whole samples, so the 'same'-padding halo of all taps is served
// from ONE LDS copy of the input rows (tap j = row shift, out-of-range rows read
// a zero row).  The label / time channels of every concat are constant per
// (TAC) / per (t): their contribution is folded into per-level maps computed
// once (fold_map_kernel) and added in the epilogue together with the biases.
// The 1x1 residual conv is folded into the centre tap of the packed weights.
#include "petdiff_internal.h"

namespace petdiff {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));


__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(bf16 v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float v) { return (bf16)v; }

// ---------------------------------------------------------------------------
// Counter-based RNG: Philox4x32-10 + Box-Muller (restated in oracle/iddpm_ref.py)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}

__device__ __forceinline__ float philox_normal(unsigned long long seed, unsigned long long g, int step,
                                               int roi, int which) {
  uint32_t c[4] = {(uint32_t)roi, (uint32_t)step, (uint32_t)(g & 0xffffffffull), (uint32_t)(g >> 32)};
  philox4x32_10(c, (uint32_t)(seed & 0xffffffffull), (uint32_t)(seed >> 32));
  const double u1 = ((double)c[0] + 1.0) * 2.3283064365386963e-10;
  const double u2 = ((double)c[1] + 0.5) * 2.3283064365386963e-10;
  const double r = sqrt(-2.0 * log(u1));
  const double ang = 6.283185307179586 * u2;
  return (float)(which == 0 ? r * cos(ang) : r * sin(ang));
}

// ---------------------------------------------------------------------------
// p_sample epilogue (diffusion_model.py:424-496, 651-663), fp32, no FMA
// contraction so every op rounds like the TF graph.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void p_sample_elem(const FinalArgs& f, int t, float x, float mo,
                                                        float vv, float z, float* mean_o, float* var_o,
                                                        float* var_t_o) {
#pragma clang fp contract(off)
  const float* tab = f.tab;
  const int T = f.T;
  float logvar, logvar_t;
  if (f.learn_mode == 2) {          // learn_ranged (:447-452)
    const float min_log = tab[TAB_PLVC * T + t];
    const float max_log = tab[TAB_LOG_BETA * T + t];
    const float frac = (vv + 1.0f) / 2.0f;
    logvar = frac * max_log + (1.0f - frac) * min_log;
    logvar_t = logvar;
  } else if (f.learn_mode == 1) {   // learn (:443-445)
    logvar = vv;
    logvar_t = vv;
  } else {                          // fixed (:455-462)
    logvar = tab[TAB_LOG_BETA * T + t];
    logvar_t = tab[TAB_PLVC * T + t];
  }
  float mean;
  if (f.param_mode == 3) {          // x_prev (:476-479)
    mean = mo;
  } else {
    float x0;
    if (f.param_mode == 0) {        // eps (:370-374)
      const float a = tab[TAB_INV_SQRT_AB * T + t] * x;
      const float b = tab[TAB_SQRT_RECIP_M1 * T + t] * mo;
      x0 = a - b;
    } else if (f.param_mode == 2) { // v (:380-386)
      const float a = tab[TAB_SQRT_AB * T + t] * x;
      const float b = tab[TAB_SQRT_1M_AB * T + t] * mo;
      x0 = a - b;
    } else {                        // x0
      x0 = mo;
    }
    const float m1 = tab[TAB_C1 * T + t] * x0;   // q_posterior_mean_variance (:415)
    const float m2 = tab[TAB_C2 * T + t] * x;
    mean = m1 + m2;
  }
  const float mask = (t == 0) ? 0.0f : 1.0f;
  const float e = expf(0.5f * logvar);
  const float et = expf(0.5f * logvar_t);
  *mean_o = mean;
  *var_o = (mask * e) * z;
  *var_t_o = (mask * et) * z;
}

// ---------------------------------------------------------------------------
// Implicit-GEMM Conv1D on MFMA.  See DESIGN.md for the tiling.
//   M tile = 192 rows = S whole samples, N tile = 128 channels, 4 waves (2x2),
//   96 x 64 per wave (3 x 2 MFMA 32x32 tiles).  K loop over chunks of
//   ROWB bytes of input channels; per chunk all TAPS taps are served from one
//   LDS copy of the chunk's input rows.
// ---------------------------------------------------------------------------
template <typename T, int L, bool UPS, int TAPS, int PADL, int EPI, int ROWB>
struct ConvGeom {
  static constexpr int S = kMT / L;                 // samples per workgroup
  static constexpr int LIN = UPS ? L / 2 : L;       // input rows per sample
  static constexpr int AROWS = S * LIN;
  static constexpr int ZROW = AROWS;                // always-zero LDS row
  static constexpr int CPR = ROWB / 16;             // 16-B pieces per LDS row
  static constexpr int KC = ROWB / (int)sizeof(T);  // input channels per chunk
  static constexpr int EPC = 16 / (int)sizeof(T);   // elements per 16-B piece
  static constexpr int A_BYTES = ((AROWS + 1) * ROWB + 255) / 256 * 256;
  static constexpr int B_BYTES = TAPS * kNT * ROWB;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static constexpr int APIECES = AROWS * CPR;
  static constexpr int APT = (APIECES + kThreads - 1) / kThreads;
  static constexpr int BPT = B_BYTES / 16 / kThreads;
  static constexpr int CT_LD = kNT + 4;             // fp32 C tile row (non-final epilogue)
  static constexpr int FIN_LD = 129;                 // fp32 C tile row (final epilogue)
  static constexpr int EPI_BYTES = (EPI == EPI_FINAL) ? kMT * FIN_LD * 4 + 128 * 4 * 4 + 64 : kMT * CT_LD * 4;
  static constexpr int SMEM = EPI_BYTES > 2 * STAGE ? EPI_BYTES : 2 * STAGE;
  static_assert(kMT % L == 0, "tile must hold whole samples");
  static_assert(B_BYTES % (16 * kThreads) == 0, "B tile split");
  static_assert(ROWB == 64 || ROWB == 128, "row width");
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  // XOR key of the 16-B piece index within a row: conflict-free ds_read_b128 for
  // 16 consecutive rows (lane groups of MI355X_MICROARCH.md LDS table)
  static __device__ __forceinline__ int key(int row) { return CPR == 4 ? ((row >> 2) & 3) : ((row >> 1) & 7); }
};

// Global -> LDS staging of chunk kc into stage buf by LDS-DMA
// (global_load_lds_dwordx4).  Piece p of a stage lands at byte 16*p; the pieces
// of one wave instruction are the 64 consecutive p = q*256 + wave*64 + lane, so
// the LDS destination is wave-uniform base + lane*16 and the XOR swizzle lives
// in the SOURCE address.
template <typename T, int L, bool UPS, int TAPS, int PADL, int EPI, int ROWB>
__device__ __forceinline__ void stage_issue(const ConvArgs<T>& a, char* smem, int kc, int buf, int n1, int NC,
                                            int m0, int n_tile, int wv, int lane) {
  using G = ConvGeom<T, L, UPS, TAPS, PADL, EPI, ROWB>;
  const T* src;
  int stride, ch;
  if (kc < n1) { src = a.src1; stride = a.c1; ch = kc * G::KC; }
  else { src = a.src2; stride = a.c2; ch = (kc - n1) * G::KC; }
  char* sbase = smem + buf * G::STAGE;
#pragma unroll
  for (int qq = 0; qq < G::APT; ++qq) {
    const int p0 = qq * kThreads + wv * 64;
    if (p0 < G::APIECES) {
      const int p = p0 + lane;
      if (p < G::APIECES) {
        const int row = p / G::CPR, cp = p - row * G::CPR;
        const int c = cp ^ G::key(row);
        const int s = row / G::LIN, li = row - s * G::LIN;
        const int b = min(m0 + s, a.B - 1);   // rows of absent samples only feed unstored outputs
        const T* g = src + (size_t)(b * G::LIN + li) * stride + ch + c * G::EPC;
        __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(sbase + p0 * 16), 16, 0, 0);
      }
    }
  }
  const char* wp = reinterpret_cast<const char*>(a.wpack) + (size_t)(n_tile * NC + kc) * G::B_BYTES;
#pragma unroll
  for (int qq = 0; qq < G::BPT; ++qq) {
    const int p0 = qq * kThreads + wv * 64;
    __builtin_amdgcn_global_load_lds(wp + (size_t)(p0 + lane) * 16,
                                     (__attribute__((address_space(3))) void*)(sbase + G::A_BYTES + p0 * 16), 16,
                                     0, 0);
  }
}

template <typename T> struct Vec8;
template <> struct Vec8<bf16> {
  static __device__ __forceinline__ void store(bf16* p, const float* v) {
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)v[e];
    *reinterpret_cast<bf16x8*>(p) = o;
  }
};
template <> struct Vec8<float> {
  static __device__ __forceinline__ void store(float* p, const float* v) {
    *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4*>(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
  }
};

template <typename T, int L, bool UPS, int TAPS, int PADL, int EPI, int ROWB>
__global__ __launch_bounds__(kThreads, 1) void conv_kernel(ConvArgs<T> a) {
  using G = ConvGeom<T, L, UPS, TAPS, PADL, EPI, ROWB>;
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM];

  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int h = lane >> 5, lr = lane & 31;

  // XCD-aware bijective block remap: the blocks sharing an XCD (bid % 8) get a
  // contiguous slot range, i.e. (mostly) the same N tile -> weight slice stays in that L2.
  const int B = a.B;
  const int nM = (B + G::S - 1) / G::S;
  const int nN = a.cout / kNT;
  const int total = nM * nN;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, loc = bid >> 3, q8 = total >> 3, r8 = total & 7;
  const int slot = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int n_tile = slot / nM, m_tile = slot - n_tile * nM;
  const int m0 = m_tile * G::S;

  const int n1 = a.c1 / G::KC;
  const int NC = n1 + a.c2 / G::KC;

  // zero row of both stages
  if (tid < 2 * G::CPR) {
    const int st = tid / G::CPR, pc = tid - st * G::CPR;
    *reinterpret_cast<uint4*>(smem + st * G::STAGE + G::ZROW * ROWB + pc * 16) = make_uint4(0, 0, 0, 0);
  }

  // per-lane LDS byte offsets of the A fragment rows (tap j, m-subtile i) and B rows
  const int c0 = (sizeof(T) == 2) ? h : 2 * h;
  int aoff[TAPS][3];
#pragma unroll
  for (int j = 0; j < TAPS; ++j) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int r = wm * 96 + i * 32 + lr;
      const int s = r / L, l = r - s * L;
      const int p = l + j - PADL;
      int row;
      if (!UPS) row = (p >= 0 && p < L) ? s * L + p : G::ZROW;
      else row = (p < L) ? s * G::LIN + (p >> 1) : G::ZROW;
      aoff[j][i] = row * ROWB + ((c0 ^ G::key(row)) << 4);
    }
  }
  int boff[2];
#pragma unroll
  for (int jn = 0; jn < 2; ++jn) {
    const int n = wn * 64 + jn * 32 + lr;
    boff[jn] = G::A_BYTES + n * ROWB + ((c0 ^ G::key(n)) << 4);
  }
  const int wv = __builtin_amdgcn_readfirstlane(w);

  f32x16 acc[3][2];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int jn = 0; jn < 2; ++jn)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][jn][e] = 0.f;

  stage_issue<T, L, UPS, TAPS, PADL, EPI, ROWB>(a, smem, 0, 0, n1, NC, m0, n_tile, wv, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kc = 0; kc < NC; ++kc) {
    if (kc + 1 < NC)
      stage_issue<T, L, UPS, TAPS, PADL, EPI, ROWB>(a, smem, kc + 1, (kc + 1) & 1, n1, NC, m0, n_tile, wv, lane);
    const char* base = smem + (kc & 1) * G::STAGE;
    if constexpr (sizeof(T) == 2) {
      // step = (tap j, 16-k group g); fragments of step+1 are read while step's MFMAs run
      constexpr int NG = ROWB / 32;
      constexpr int NS = TAPS * NG;
      bf16x8 av[2][3], bv[2][2];
#pragma unroll
      for (int st = 0; st < NS + 1; ++st) {
        if (st < NS) {
          const int j = st / NG, g = st % NG, sb = st & 1;
#pragma unroll
          for (int i = 0; i < 3; ++i) av[sb][i] = *reinterpret_cast<const bf16x8*>(base + (aoff[j][i] ^ (g << 5)));
#pragma unroll
          for (int jn = 0; jn < 2; ++jn)
            bv[sb][jn] = *reinterpret_cast<const bf16x8*>(base + ((boff[jn] + j * kNT * ROWB) ^ (g << 5)));
        }
        if (st > 0) {
          const int pb = (st - 1) & 1;
#pragma unroll
          for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int jn = 0; jn < 2; ++jn)
              acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[pb][i], bv[pb][jn], acc[i][jn], 0, 0, 0);
        }
      }
    } else {
      constexpr int NG = ROWB / 64;
#pragma unroll
      for (int j = 0; j < TAPS; ++j) {
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          f32x4 av0[3], av1[3], bv0[2], bv1[2];
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            av0[i] = *reinterpret_cast<const f32x4*>(base + (aoff[j][i] ^ (g << 6)));
            av1[i] = *reinterpret_cast<const f32x4*>(base + (aoff[j][i] ^ (g << 6) ^ 16));
          }
#pragma unroll
          for (int jn = 0; jn < 2; ++jn) {
            bv0[jn] = *reinterpret_cast<const f32x4*>(base + ((boff[jn] + j * kNT * ROWB) ^ (g << 6)));
            bv1[jn] = *reinterpret_cast<const f32x4*>(base + ((boff[jn] + j * kNT * ROWB) ^ (g << 6) ^ 16));
          }
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
              for (int jn = 0; jn < 2; ++jn)
                acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x2f32(av0[i][s4], bv0[jn][s4], acc[i][jn], 0, 0, 0);
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
              for (int jn = 0; jn < 2; ++jn)
                acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x2f32(av1[i][s4], bv1[jn][s4], acc[i][jn], 0, 0, 0);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ------------------------------- epilogue --------------------------------
  const int cout = a.cout;
  if constexpr (EPI != EPI_FINAL) {
    // accumulators -> fp32 C tile in LDS -> row-wise: + maps (float4), act, 16-B stores
    float* ct = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int jn = 0; jn < 2; ++jn)
#pragma unroll
        for (int rg = 0; rg < 16; ++rg) {
          const int r = wm * 96 + i * 32 + (rg & 3) + 8 * (rg >> 2) + 4 * h;
          ct[r * G::CT_LD + wn * 64 + jn * 32 + lr] = acc[i][jn][rg];
        }
    __syncthreads();
    const int cg = tid & 15;                 // 8-column group
    const int nloc = cg * 8, n = n_tile * kNT + nloc;
    for (int rp = tid >> 4; rp < kMT / 2; rp += kThreads / 16) {
      const int r = 2 * rp;
      const int s = r / L, l = r - s * L, b = m0 + s;
      if (b >= B) continue;
      const int tac = a.tac ? a.tac[b] : 0;
      const int t = a.t_uniform >= 0 ? a.t_uniform : a.tvec[b];
      float v[2][8];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const f32x4 c0v = *reinterpret_cast<const f32x4*>(ct + (r + e) * G::CT_LD + nloc);
        const f32x4 c1v = *reinterpret_cast<const f32x4*>(ct + (r + e) * G::CT_LD + nloc + 4);
        f32x4 m0v, m1v;
        if (a.tmap) {
          const float* mp = a.tmap + ((size_t)t * L + l + e) * cout + n;
          m0v = *reinterpret_cast<const f32x4*>(mp);
          m1v = *reinterpret_cast<const f32x4*>(mp + 4);
        } else {
          m0v = *reinterpret_cast<const f32x4*>(a.bias + n);
          m1v = *reinterpret_cast<const f32x4*>(a.bias + n + 4);
        }
        if (a.cmap) {
          const float* cp = a.cmap + ((size_t)tac * L + l + e) * cout + n;
          m0v += *reinterpret_cast<const f32x4*>(cp);
          m1v += *reinterpret_cast<const f32x4*>(cp + 4);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[e][q] = c0v[q] + m0v[q];
          v[e][4 + q] = c1v[q] + m1v[q];
        }
        if constexpr (EPI != EPI_LIN) {
#pragma unroll
          for (int q = 0; q < 8; ++q) v[e][q] = fmaxf(v[e][q], 0.f);
        }
        Vec8<T>::store(a.out + ((size_t)b * L + l + e) * cout + n, v[e]);
      }
      if constexpr (EPI == EPI_POOL) {
        float pv[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) pv[q] = fmaxf(v[0][q], v[1][q]);
        Vec8<T>::store(a.out_pool + ((size_t)b * (L / 2) + (l >> 1)) * cout + n, pv);
      }
    }
  } else {
    // up2 ConvBlock output (relu) -> LDS -> final 1x1 conv (networks.py:1074) -> p_sample
    float* fin = reinterpret_cast<float*>(smem);
    float* wfl = fin + kMT * G::FIN_LD;
    const FinalArgs& f = a.fin;
    const int n_out = f.n_out;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
      for (int jn = 0; jn < 2; ++jn) {
        const int n = wn * 64 + jn * 32 + lr;
#pragma unroll
        for (int rg = 0; rg < 16; ++rg) {
          const int r = wm * 96 + i * 32 + (rg & 3) + 8 * (rg >> 2) + 4 * h;
          const int s = r / L, l = r - s * L, b = m0 + s;
          float v = 0.f;
          if (b < B) {
            const int tac = a.tac ? a.tac[b] : 0;
            const int t = a.t_uniform >= 0 ? a.t_uniform : a.tvec[b];
            float m = a.tmap ? a.tmap[((size_t)t * L + l) * cout + n] : a.bias[n];
            if (a.cmap) m += a.cmap[((size_t)tac * L + l) * cout + n];
            v = fmaxf(acc[i][jn][rg] + m, 0.f);
          }
          fin[r * G::FIN_LD + n] = v;
        }
      }
    }
    for (int e = tid; e < 128 * n_out; e += kThreads) wfl[e] = f.wf[e];
    __syncthreads();
    if (f.net_out) {
      for (int it = tid; it < kMT * n_out; it += kThreads) {
        const int r = it / n_out, o = it - r * n_out;
        const int s = r / L, l = r - s * L, b = m0 + s;
        if (b >= B) continue;
        float accf = 0.f;
        for (int n = 0; n < 128; ++n) accf = fmaf(fin[r * G::FIN_LD + n], wfl[n * n_out + o], accf);
        f.net_out[((size_t)b * L + l) * n_out + o] = accf + f.bf[o];
      }
    } else {
      const unsigned long long seed = f.rng ? f.rng[0] : 0ull;
      const unsigned long long goff = f.rng ? f.rng[1] : 0ull;
      const int half = n_out / 2;   // eps channels = 2, var channels follow when learned
      for (int it = tid; it < kMT * 2; it += kThreads) {
        const int r = it >> 1, c = it & 1;
        const int s = r / L, l = r - s * L, b = m0 + s;
        if (b >= B) continue;
        float mo = 0.f, vv = 0.f;
        for (int n = 0; n < 128; ++n) mo = fmaf(fin[r * G::FIN_LD + n], wfl[n * n_out + c], mo);
        mo += f.bf[c];
        if (n_out == 4) {
          for (int n = 0; n < 128; ++n) vv = fmaf(fin[r * G::FIN_LD + n], wfl[n * n_out + half + c], vv);
          vv += f.bf[half + c];
        }
        const int t = a.t_uniform >= 0 ? a.t_uniform : a.tvec[b];
        const size_t idx = ((size_t)b * L + l) * 2 + c;
        const float x = f.x_t[idx];
        const float z = f.z ? f.z[idx] : philox_normal(seed, goff + (unsigned long long)b, f.rng_step, l, c);
        float mean, var, var_t;
        p_sample_elem(f, t, x, mo, vv, z, &mean, &var, &var_t);
        if (f.mean_out) f.mean_out[idx] = mean;
        if (f.var_out) f.var_out[idx] = var;
        if (f.var_tilde_out) f.var_tilde_out[idx] = var_t;
        if (f.x_next) {
          const float xn = mean + (f.flag_var_tilde ? var_t : var);
          f.x_next[idx] = xn;
          if (f.x_all) f.x_all[idx] = xn;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// down0 block: K = 6 taps x 2 x-channels (label/time folded into maps) -> VALU.
// Writes the skip s0 (B*48 x 128) and the pooled p0 (B*24 x 128).
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void down0_kernel(Down0Args a) {
  __shared__ __attribute__((aligned(16))) float w[6 * 2 * 128];
  const int tid = threadIdx.x;
  for (int i = tid; i < 6 * 2 * 128; i += 256) w[i] = a.w0[i];
  __syncthreads();
  const int pos = blockIdx.x * 16 + (tid >> 4);   // (sample, pooled position)
  if (pos >= a.B * 24) return;
  const int b = pos / 24, lp = pos - b * 24;
  const int n0 = (tid & 15) * 8;
  const int l0 = 2 * lp;
  const float* xb = a.x + (size_t)b * 96;
  float xv[7][2];
#pragma unroll
  for (int q = 0; q < 7; ++q) {
    const int p = l0 - 2 + q;
    const bool ok = (p >= 0 && p < 48);
    xv[q][0] = ok ? xb[p * 2] : 0.f;
    xv[q][1] = ok ? xb[p * 2 + 1] : 0.f;
  }
  const int tac = a.tac ? a.tac[b] : 0;
  const int t = a.t_uniform >= 0 ? a.t_uniform : a.tvec[b];
  float v[2][8];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int l = l0 + e;
    const float* tm = a.tmap + ((size_t)t * 48 + l) * 128 + n0;
    const float* cm = a.cmap + ((size_t)tac * 48 + l) * 128 + n0;
    f32x4 m0 = *reinterpret_cast<const f32x4*>(tm) + *reinterpret_cast<const f32x4*>(cm);
    f32x4 m1 = *reinterpret_cast<const f32x4*>(tm + 4) + *reinterpret_cast<const f32x4*>(cm + 4);
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 6; ++j) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const f32x4 w0 = *reinterpret_cast<const f32x4*>(w + (j * 2 + c) * 128 + n0);
        const f32x4 w1 = *reinterpret_cast<const f32x4*>(w + (j * 2 + c) * 128 + n0 + 4);
        acc0 += w0 * xv[e + j][c];
        acc1 += w1 * xv[e + j][c];
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[e][q] = fmaxf(acc0[q] + m0[q], 0.f);
      v[e][4 + q] = fmaxf(acc1[q] + m1[q], 0.f);
    }
    Vec8<T>::store(reinterpret_cast<T*>(a.s0) + ((size_t)b * 48 + l) * 128 + n0, v[e]);
  }
  float pv[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) pv[q] = fmaxf(v[0][q], v[1][q]);
  Vec8<T>::store(reinterpret_cast<T*>(a.p0) + ((size_t)b * 24 + lp) * 128 + n0, pv);
}

// ---------------------------------------------------------------------------
// Setup kernels (run once per model / per condition, fp32)
// ---------------------------------------------------------------------------
// SinusoidalPosEmb(sin_dim) -> Dense(hid) -> GELU(erf) for every t in [0, T)
__global__ void time_emb_kernel(const float* w, const float* bvec, int sin_dim, int hid, float* out) {
  extern __shared__ float emb[];
  const int t = blockIdx.x;
  const int half = sin_dim / 2;
  for (int i = threadIdx.x; i < half; i += blockDim.x) {
    const float sc = logf(10000.f) / (float)(half - 1);
    const float fr = expf((float)i * -sc);
    const float ar = (float)t * fr;
    emb[i] = sinf(ar);
    emb[half + i] = cosf(ar);
  }
  __syncthreads();
  for (int o = threadIdx.x; o < hid; o += blockDim.x) {
    float acc = 0.f;
    for (int k = 0; k < sin_dim; ++k) acc = fmaf(emb[k], w[k * hid + o], acc);
    acc += bvec[o];
    out[(size_t)t * hid + o] = 0.5f * acc * (1.0f + erff(acc / 1.4142135623730951f));
  }
}

// rows x Din  @ (Din x Dout) + b, act: 0 none, 1 relu
__global__ void dense_kernel(const float* in, int rows, int din, const float* w, const float* bvec,
                             int dout, int act, float* out) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)rows * dout) return;
  const int r = (int)(idx / dout), o = (int)(idx - (size_t)r * dout);
  float acc = 0.f;
  for (int k = 0; k < din; ++k) acc = fmaf(in[(size_t)r * din + k], w[(size_t)k * dout + o], acc);
  acc += bvec[o];
  if (act == 1) acc = fmaxf(acc, 0.f);
  out[idx] = acc;
}

// Contribution of a constant channel group (label: 49 ch at offset 0, time: 1 ch
// at offset 49) of a Conv1D('same') input to its output, + biases.
// seq: [n][Lseq][Cs]; out: [n][Lout][cout].  ups: the conv input is the
// UpSampling1D(2) of seq (Lout = 2*Lseq, pad_before = 0).
__global__ void fold_map_kernel(const float* seq, int n, int Lseq, int Cs, const float* wk, int taps,
                                int padl, int ups, int cin_full, int ch0, const float* wr,
                                const float* b1, const float* b2, float* out, int Lout, int cout) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)n * Lout * cout) return;
  const int o = (int)(idx % cout);
  const int l = (int)((idx / cout) % Lout);
  const int k = (int)(idx / ((size_t)cout * Lout));
  const float* sq = seq + (size_t)k * Lseq * Cs;
  float acc = 0.f;
  for (int j = 0; j < taps; ++j) {
    int p = ups ? l + j : l + j - padl;
    if (p < 0 || p >= Lout) continue;
    const int sp = ups ? (p >> 1) : p;
    for (int c = 0; c < Cs; ++c) acc = fmaf(wk[((size_t)j * cin_full + ch0 + c) * cout + o], sq[sp * Cs + c], acc);
  }
  if (wr)
    for (int c = 0; c < Cs; ++c) acc = fmaf(wr[(size_t)(ch0 + c) * cout + o], sq[l * Cs + c], acc);
  if (b1) acc += b1[o];
  if (b2) acc += b2[o];
  out[idx] = acc;
}

// Per (TAC, column) count / mean / M2 in fp64 (main_script.py:433-436 summary).
__global__ void posterior_stats_kernel(const float* x0, const int* tac, int B, int ncol, double* stats) {
  __shared__ double red[256];
  __shared__ long long redc[256];
  const int tc = blockIdx.x / ncol, col = blockIdx.x - tc * ncol;
  double s = 0.0;
  long long cnt = 0;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    if ((tac ? tac[b] : 0) != tc) continue;
    s += (double)x0[(size_t)b * ncol + col];
    ++cnt;
  }
  red[threadIdx.x] = s;
  redc[threadIdx.x] = cnt;
  __syncthreads();
  for (int k = blockDim.x / 2; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) { red[threadIdx.x] += red[threadIdx.x + k]; redc[threadIdx.x] += redc[threadIdx.x + k]; }
    __syncthreads();
  }
  const long long n = redc[0];
  const double mean = n > 0 ? red[0] / (double)n : 0.0;
  __syncthreads();
  double m2 = 0.0;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    if ((tac ? tac[b] : 0) != tc) continue;
    const double d = (double)x0[(size_t)b * ncol + col] - mean;
    m2 += d * d;
  }
  red[threadIdx.x] = m2;
  __syncthreads();
  for (int k = blockDim.x / 2; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    stats[((size_t)tc * ncol + col) * 3 + 0] = (double)n;
    stats[((size_t)tc * ncol + col) * 3 + 1] = mean;
    stats[((size_t)tc * ncol + col) * 3 + 2] = red[0];
  }
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
template <typename T, int L, bool UPS, int TAPS, int PADL, int EPI>
static hipError_t launch_one(const ConvArgs<T>& a, hipStream_t s) {
  constexpr int ROWB = conv_rowb<T>(TAPS);
  using G = ConvGeom<T, L, UPS, TAPS, PADL, EPI, ROWB>;
  if (a.B <= 0) return hipSuccess;
  if (a.cout % kNT != 0 || a.c1 % G::KC != 0 || a.c2 % G::KC != 0) return hipErrorInvalidValue;
  if (EPI == EPI_FINAL && a.cout != kNT) return hipErrorInvalidValue;
  const int nM = (a.B + G::S - 1) / G::S;
  const int total = nM * (a.cout / kNT);
  hipLaunchKernelGGL((conv_kernel<T, L, UPS, TAPS, PADL, EPI, ROWB>), dim3(total), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_conv(int kind, const ConvArgs<T>& a, hipStream_t s) {
  switch (kind) {
    case LK_DOWN1: return launch_one<T, 24, false, 6, 2, EPI_POOL>(a, s);
    case LK_DOWN2: return launch_one<T, 12, false, 6, 2, EPI_POOL>(a, s);
    case LK_DOWN3: return launch_one<T, 6, false, 6, 2, EPI_RELU>(a, s);
    case LK_UP0_CONV2: return launch_one<T, 12, true, 2, 0, EPI_LIN>(a, s);
    case LK_UP0_BLOCK: return launch_one<T, 12, false, 6, 2, EPI_RELU>(a, s);
    case LK_UP1_CONV2: return launch_one<T, 24, true, 2, 0, EPI_LIN>(a, s);
    case LK_UP1_BLOCK: return launch_one<T, 24, false, 6, 2, EPI_RELU>(a, s);
    case LK_UP2_CONV2: return launch_one<T, 48, true, 2, 0, EPI_LIN>(a, s);
    case LK_UP2_BLOCK: return launch_one<T, 48, false, 6, 2, EPI_FINAL>(a, s);
  }
  return hipErrorInvalidValue;
}

template <typename T>
hipError_t launch_down0(const Down0Args& a, hipStream_t s) {
  if (a.B <= 0) return hipSuccess;
  hipLaunchKernelGGL(down0_kernel<T>, dim3((a.B * 24 + 15) / 16), dim3(256), 0, s, a);
  return hipGetLastError();
}

template hipError_t launch_conv<bf16>(int, const ConvArgs<bf16>&, hipStream_t);
template hipError_t launch_conv<float>(int, const ConvArgs<float>&, hipStream_t);
template hipError_t launch_down0<bf16>(const Down0Args&, hipStream_t);
template hipError_t launch_down0<float>(const Down0Args&, hipStream_t);

hipError_t launch_time_emb(const float* w, const float* b, int T, int sin_dim, int hid, float* out,
                           hipStream_t s) {
  hipLaunchKernelGGL(time_emb_kernel, dim3(T), dim3(64), sin_dim * sizeof(float), s, w, b, sin_dim, hid, out);
  return hipGetLastError();
}

hipError_t launch_dense(const float* in, int rows, int din, const float* w, const float* b, int dout,
                        int act, float* out, hipStream_t s) {
  const size_t n = (size_t)rows * dout;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(dense_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, rows, din, w, b, dout,
                     act, out);
  return hipGetLastError();
}

hipError_t launch_fold(const float* seq, int n, int Lseq, int Cs, const float* wk, int taps, int padl,
                       int ups, int cin_full, int ch0, const float* wr, const float* b1,
                       const float* b2, float* out, int Lout, int cout, hipStream_t s) {
  const size_t tot = (size_t)n * Lout * cout;
  if (tot == 0) return hipSuccess;
  hipLaunchKernelGGL(fold_map_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, seq, n, Lseq, Cs, wk,
                     taps, padl, ups, cin_full, ch0, wr, b1, b2, out, Lout, cout);
  return hipGetLastError();
}

hipError_t launch_posterior_stats(const float* x0, const int* tac, int B, int n_tac, int ncol, double* stats,
                                  hipStream_t s) {
  if (n_tac <= 0) return hipSuccess;
  hipLaunchKernelGGL(posterior_stats_kernel, dim3(n_tac * ncol), dim3(256), 0, s, x0, tac, B, ncol, stats);
  return hipGetLastError();
}

}  // namespace petdiff
