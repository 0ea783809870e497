// HIP kernels of the training step (include/pettrain.h).
//
// The GEMM-shaped work (conv forward / weight grad / data grad, dense layers)
// runs as rocBLAS fp32 GEMMs in train_api.cpp; these kernels are the memory-bound
// glue around them: im2col / col2im over the reference's concat layouts, bias +
// activation epilogues, pooling, the q-sample draw, the loss with its analytic
// gradient, and the clipped Adam update.  fp32 throughout.
#include "petdiff_internal.h"
#include "train_internal.h"

#include <cmath>

namespace pettrain_k {

using namespace petdiff;

namespace {

constexpr int kT = 256;

inline int blocks_for(size_t n, int per = kT) {
  size_t b = (n + per - 1) / per;
  return (int)(b > 65535u * 8u ? 65535u * 8u : b);
}

// ---------------------------------------------------------------------------
// im2col / col2im over [label | time | x1 | x2] (networks.py:1022, 1043, 1057)
//   A[((b*Lout + l)*taps + j)*Cf + c] = X(b, p = l + j - padl, c), 0 outside [0, Lout);
//   with UpSampling1D(2) the source position of p is p / 2.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float conv_src(const ConvIn& ci, int b, int sp, int c, const float* lab,
                                          const float* tim, const float* x1, const float* x2) {
  if (ci.has_cond) {
    if (c < 49) return lab[((size_t)b * ci.Lsrc + sp) * 49 + c];
    if (c == 49) return tim[(size_t)b * ci.Lsrc + sp];
    c -= 50;
  }
  if (c < ci.c1) return x1[((size_t)b * ci.Lsrc + sp) * ci.c1 + c];
  return x2[((size_t)b * ci.Lsrc + sp) * ci.c2 + (c - ci.c1)];
}

__global__ void im2col_kernel(ConvIn ci, int B, const float* lab, const float* tim, const float* x1,
                              const float* x2, float* A) {
  // rows of K + 1: the last column is 1, so the GEMMs against [W ; bias] add the bias in the
  // forward pass and produce the bias gradient as the last row of the weight gradient.
  // One block per output row m = (b, l); threads walk the row's taps x channels.
  const int Cf = ci.cfull(), Lout = ci.lout();
  const int Kd = ci.taps * Cf, ld = Kd + 1;
  const int m = blockIdx.x;
  const int l = m % Lout, b = m / Lout;
  float* row = A + (size_t)m * ld;
  for (int j = 0; j < ci.taps; ++j) {
    const int p = l + j - ci.padl;
    const bool in = p >= 0 && p < Lout;
    const int sp = ci.ups ? p >> 1 : p;
    for (int c = threadIdx.x; c < Cf; c += blockDim.x)
      row[j * Cf + c] = in ? conv_src(ci, b, sp, c, lab, tim, x1, x2) : 0.f;
  }
  if (threadIdx.x == 0) row[Kd] = 1.0f;
}

// dX(b, sp, c) = sum over the fine positions p of sp and the taps j of dA[(b, p - j + padl), j, c]
// one block per source row (b, sp); threads walk the channels
__global__ void col2im_kernel(ConvIn ci, int B, const float* dA, float* dlab, float* dtim, float* dx1,
                              float* dx2) {
  const int Cf = ci.cfull(), Lout = ci.lout();
  const int r = blockIdx.x;
  const int sp = r % ci.Lsrc, b = r / ci.Lsrc;
  const int np = ci.ups ? 2 : 1;
  for (int c = threadIdx.x; c < Cf; c += blockDim.x) {
    float acc = 0.f;
    for (int q = 0; q < np; ++q) {
      const int p = ci.ups ? 2 * sp + q : sp;
      for (int j = 0; j < ci.taps; ++j) {
        const int l = p - j + ci.padl;
        if (l >= 0 && l < Lout) acc += dA[(((size_t)b * Lout + l) * ci.taps + j) * Cf + c];
      }
    }
    int cc = c;
    if (ci.has_cond) {
      if (cc < 49) {
        if (dlab) dlab[((size_t)b * ci.Lsrc + sp) * 49 + cc] = acc;
        continue;
      }
      if (cc == 49) {
        if (dtim) dtim[(size_t)b * ci.Lsrc + sp] = acc;
        continue;
      }
      cc -= 50;
    }
    if (cc < ci.c1) {
      if (dx1) dx1[((size_t)b * ci.Lsrc + sp) * ci.c1 + cc] = acc;
    } else if (dx2) {
      dx2[((size_t)b * ci.Lsrc + sp) * ci.c2 + (cc - ci.c1)] = acc;
    }
  }
}

__global__ void bias_act_kernel(float* Y, int M, int N, int ld, const float* b1, int relu) {
  const size_t n = (size_t)M * N;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const size_t m = i / N;
    const int c = (int)(i - m * N);
    float& y = Y[m * ld + c];
    float v = y;
    if (b1) v += b1[c];
    y = relu ? fmaxf(v, 0.f) : v;
  }
}

__global__ void gelu_fwd_kernel(const float* a, float* h, int M, int N, int ldh) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < M * N; i += gridDim.x * blockDim.x) {
    const int m = i / N, c = i - m * N;
    const float x = a[i];
    h[(size_t)m * ldh + c] = 0.5f * x * (1.0f + erff(x / 1.4142135623730951f));    // networks.py:236-241, exact
  }
}

__global__ void gelu_bwd_kernel(const float* dh, const float* a, float* da, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float x = a[i];
    const float g = 0.5f * (1.0f + erff(x / 1.4142135623730951f)) + x * expf(-0.5f * x * x) * 0.3989422804014327f;
    da[i] = dh[i] * g;
  }
}

__global__ void relu_mask_kernel(float* d, const float* y, int M, int N, int ldy) {
  const size_t n = (size_t)M * N;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const size_t m = i / N;
    if (!(y[m * ldy + (i - m * N)] > 0.f)) d[i] = 0.f;
  }
}

__global__ void copy_rows_kernel(const float* src, int M, int N, float* dst, int ldd) {
  const size_t n = (size_t)M * N;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const size_t m = i / N;
    dst[m * ldd + (i - m * N)] = src[i];
  }
}

__global__ void fill_kernel(float* p, size_t n, size_t stride, float v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i * stride] = v;
}

__global__ void maxpool_fwd_kernel(const float* out, float* pool, int B, int L, int C) {
  const size_t n = (size_t)B * (L / 2) * C;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const size_t r = i / C;                       // b * L/2 + q
    const size_t e = (2 * r) * C + c;
    pool[i] = fmaxf(out[e], out[e + C]);
  }
}

// MaxPool gradient goes to the first maximum of each pair (TF MaxPoolGrad).
__global__ void pool_mask_bwd_kernel(const float* out, const float* dpool, const float* dskip, float* dpre,
                                     int B, int L, int C) {
  const size_t n = (size_t)B * L * C;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const size_t r = i / C;
    const int l = (int)(r % L);
    const size_t b = r / L;
    const float o = out[i];
    float g = dskip ? dskip[i] : 0.f;
    if (dpool) {
      const size_t e0 = (b * L + (l & ~1)) * C + c;
      const bool first = out[e0] >= out[e0 + C];
      if ((l & 1) == (first ? 0 : 1)) g += dpool[(b * (L / 2) + (l >> 1)) * C + c];
    }
    dpre[i] = o > 0.f ? g : 0.f;
  }
}

// Weff [(taps*C + 1) x N]: conv kernel with the residual 1x1 kernel added to the centre tap,
// and the bias row conv.bias + res.bias (inputs: the blob's kernel / bias / res kernel / res bias).
__global__ void fold_weff_kernel(const float* W, const float* bw, const float* R, const float* br, float* Weff,
                                 int taps, int padl, int C, int N) {
  const size_t CN = (size_t)C * N, n = (size_t)taps * CN + N;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    if (i >= (size_t)taps * CN) {
      const size_t c = i - (size_t)taps * CN;
      Weff[i] = bw[c] + br[c];
    } else {
      const int j = (int)(i / CN);
      Weff[i] = W[i] + (j == padl ? R[i - (size_t)padl * CN] : 0.f);
    }
  }
}

// SinusoidalPosEmb (networks.py:189-198), same fp32 formula as time_emb_kernel
__global__ void time_embed_kernel(const int* t, int B, int dim, float* emb, int ld) {
  const int half = dim / 2;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < B * half; i += gridDim.x * blockDim.x) {
    const int b = i / half, k = i - b * half;
    const float sc = logf(10000.f) / (float)(half - 1);
    const float fr = expf((float)k * -sc);
    const float ar = (float)t[b] * fr;
    emb[(size_t)b * ld + k] = sinf(ar);
    emb[(size_t)b * ld + half + k] = cosf(ar);
  }
}

// ---------------------------------------------------------------------------
// q-sample with counter-based draws (diffusion_model.py:542-551)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void philox10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}

constexpr uint32_t kTagT = 0x54000000u;      // counter word 0 of the timestep draw
constexpr uint64_t kKeyTrain = 0x7472616E5F6B6579ull;   // key tweak: training stream

__global__ void qsample_kernel(const float* x0, const int* t_in, const float* noise_in, uint64_t seed, uint64_t goff,
                               int64_t iter, int B, int T, const float* tab, int* t_out, float* noise_out,
                               float* xt) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;     // (b, roi)
  if (i >= B * 48) return;
  const int b = i / 48, roi = i - b * 48;
  const uint64_t key = seed ^ kKeyTrain;
  const uint64_t g = goff + (uint64_t)b;
  int t;
  if (t_in) {
    t = t_in[b];
  } else {
    uint32_t c[4] = {kTagT, (uint32_t)iter, (uint32_t)(g & 0xffffffffu), (uint32_t)(g >> 32)};
    philox10(c, (uint32_t)(key & 0xffffffffu), (uint32_t)(key >> 32));
    t = (int)(((uint64_t)c[0] * (uint64_t)T) >> 32);
  }
  if (roi == 0) t_out[b] = t;
  float z[2];
  const size_t e = (size_t)i * 2;
  if (noise_in) {
    z[0] = noise_in[e];
    z[1] = noise_in[e + 1];
  } else {
    uint32_t c[4] = {(uint32_t)roi, (uint32_t)iter, (uint32_t)(g & 0xffffffffu), (uint32_t)(g >> 32)};
    philox10(c, (uint32_t)(key & 0xffffffffu), (uint32_t)(key >> 32));
    const double u1 = ((double)c[0] + 1.0) * 2.3283064365386963e-10;
    const double u2 = ((double)c[1] + 0.5) * 2.3283064365386963e-10;
    const double r = sqrt(-2.0 * log(u1));
    double sn, cs;
    sincos(6.283185307179586 * u2, &sn, &cs);
    z[0] = (float)(r * cs);
    z[1] = (float)(r * sn);
  }
  const float sa = tab[TAB_SQRT_AB * T + t], sm = tab[TAB_SQRT_1M_AB * T + t];
  for (int q = 0; q < 2; ++q) {
    noise_out[e + q] = z[q];
    xt[e + q] = sa * x0[e + q] + sm * z[q];
  }
}

// ---------------------------------------------------------------------------
// loss + its gradient (diffusion_model.py:498-578, networks.py:29-80)
// one 128-thread block per sample, thread i < 96 -> (roi i/2, parameter i%2)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float approx_cdf(float x) {
  return 0.5f * (1.0f + tanhf(0.7978845608028654f * (x + 0.044715f * x * x * x)));
}
__device__ __forceinline__ float approx_cdf_grad(float x) {
  const float th = tanhf(0.7978845608028654f * (x + 0.044715f * x * x * x));
  return 0.5f * (1.0f - th * th) * 0.7978845608028654f * (1.0f + 3.0f * 0.044715f * x * x);
}

__device__ __forceinline__ float block_sum128(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  const float r = red[0] + red[1];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(128) void loss_kernel(LossArgs a) {
  __shared__ float red[2];
  const int b = blockIdx.x, i = threadIdx.x;
  const int T = a.T, n_out = a.n_out;
  const float* tab = a.tab;
  const int t = a.t[b];
  float se = 0.f, term = 0.f;
  if (i < 96) {
    const int roi = i >> 1, p = i & 1;
    const size_t e = (size_t)b * 96 + i;
    const size_t yo = ((size_t)b * 48 + roi) * n_out;
    const float pred = a.y[yo + p];
    const float x0 = a.x0[e], xt = a.xt[e], nz = a.noise[e];
    float target;
    if (a.param_mode == 3) target = tab[TAB_C1 * T + t] * x0 + tab[TAB_C2 * T + t] * xt;
    else if (a.param_mode == 1) target = x0;
    else if (a.param_mode == 2) target = tab[TAB_SQRT_AB * T + t] * nz - tab[TAB_SQRT_1M_AB * T + t] * x0;
    else target = nz;
    const float d = target - pred;
    se = d * d;
    // B * mse: d/dpred = B * 2 (pred - target) / (B * 96)
    a.dy[yo + p] = 2.0f * (pred - target) / 96.0f;
    if (a.learn_mode != 0) {
      const float vv = a.y[yo + 2 + p];
      const float plvc = tab[TAB_PLVC * T + t], lb = tab[TAB_LOG_BETA * T + t];
      float lv2, dlv_dv;
      if (a.learn_mode == 2) {
        const float frac = (vv + 1.0f) / 2.0f;
        lv2 = frac * lb + (1.0f - frac) * plvc;
        dlv_dv = 0.5f * (lb - plvc);
      } else {
        lv2 = vv;
        dlv_dv = 1.0f;
      }
      // model mean from the frozen prediction (p_mean_variance, :464-496)
      float m2;
      if (a.param_mode == 3) {
        m2 = pred;
      } else {
        float px0;
        if (a.param_mode == 0) px0 = tab[TAB_INV_SQRT_AB * T + t] * xt - tab[TAB_SQRT_RECIP_M1 * T + t] * pred;
        else if (a.param_mode == 2) px0 = tab[TAB_SQRT_AB * T + t] * xt - tab[TAB_SQRT_1M_AB * T + t] * pred;
        else px0 = pred;
        m2 = tab[TAB_C1 * T + t] * px0 + tab[TAB_C2 * T + t] * xt;
      }
      float dterm;
      if (t != 0) {
        // KL(q(x_{t-1} | x_t, x_0) || p)  (normal_kl, networks.py:29-36)
        const float m1 = tab[TAB_C1 * T + t] * x0 + tab[TAB_C2 * T + t] * xt;
        const float lv1 = plvc;
        const float dm = m1 - m2;
        const float e12 = expf(lv1 - lv2), en2 = expf(-lv2);
        term = 0.5f * (-1.0f + lv2 - lv1 + e12 + dm * dm * en2);
        dterm = 0.5f * (1.0f - e12 - dm * dm * en2);
      } else {
        // decoder NLL (discretized_gaussian_log_likelihood, networks.py:47-80), log_scales = lv2 / 2
        const float ls = 0.5f * lv2;
        const float cx = x0 - m2;
        const float inv = expf(-ls);
        const float pin = inv * (cx + a.bin_width), mn = inv * (cx - a.bin_width);
        const float cp = approx_cdf(pin), cm = approx_cdf(mn);
        const float dcp = -approx_cdf_grad(pin) * pin, dcm = -approx_cdf_grad(mn) * mn;   // d/d ls
        const float lo = 1e-12f;
        float lp, g;
        if (x0 < -0.999f) {
          lp = logf(fmaxf(cp, lo));
          g = cp > lo ? dcp / cp : 0.f;
        } else if (x0 > 0.999f) {
          const float om = 1.0f - cm;
          lp = logf(fmaxf(om, lo));
          g = om > lo ? -dcm / om : 0.f;
        } else {
          const float dl = cp - cm;
          lp = logf(fmaxf(dl, lo));
          g = dl > lo ? (dcp - dcm) / dl : 0.f;
        }
        term = -lp;
        dterm = -0.5f * g;
      }
      a.dy[yo + 2 + p] = a.lambda_vlb * dterm / 96.0f / 0.6931471805599453f * dlv_dv;
    }
  }
  const float sse = block_sum128(se, red);
  const float st = block_sum128(term, red);
  // per-sample column sums of dy (final.bias gradient, reduced over samples in loss_finish)
  for (int q = 0; q < n_out; ++q) {
    const float v = (i < 96 && (i & 1) == (q & 1) && (q < 2 || a.learn_mode != 0))
                        ? a.dy[((size_t)b * 48 + (i >> 1)) * n_out + q] : 0.f;
    const float cs = block_sum128(v, red);
    if (i == 0) a.dbias_part[(size_t)b * n_out + q] = cs;
  }
  if (i == 0) {
    a.sse[b] = sse;
    a.vlb[b] = a.learn_mode ? a.lambda_vlb * (st / 96.0f) / 0.6931471805599453f : 0.f;
  }
}

__global__ void loss_finish_kernel(const float* sse, const float* vlb, const float* dbias_part, int B, int n_out,
                                   int n_el, float* loss_out, double* stats, float* dbias) {
  // one block: deterministic fixed-order sums
  __shared__ double s_sse[256], s_vlb[256];
  double a = 0.0, c = 0.0;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    a += sse[b];
    c += vlb[b];
  }
  s_sse[threadIdx.x] = a;
  s_vlb[threadIdx.x] = c;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      s_sse[threadIdx.x] += s_sse[threadIdx.x + o];
      s_vlb[threadIdx.x] += s_vlb[threadIdx.x + o];
    }
    __syncthreads();
  }
  const double mse = s_sse[0] / (double)n_el;
  if (loss_out)
    for (int b = threadIdx.x; b < B; b += blockDim.x) loss_out[b] = (float)mse + vlb[b];
  for (int q = 0; q < n_out; ++q) {           // fixed-order tree over samples
    __syncthreads();
    double g = 0.0;
    for (int b = threadIdx.x; b < B; b += blockDim.x) g += dbias_part[(size_t)b * n_out + q];
    s_sse[threadIdx.x] = g;
    __syncthreads();
    for (int o = blockDim.x / 2; o > 0; o >>= 1) {
      if (threadIdx.x < o) s_sse[threadIdx.x] += s_sse[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0 && dbias) dbias[q] = (float)s_sse[0];   // null: loss-only pass
  }
  if (threadIdx.x == 0) {
    stats[0] = mse + s_vlb[0] / B;
    stats[1] = mse;
    stats[2] = s_vlb[0] / B;
  }
}

// ---------------------------------------------------------------------------
// clip_by_norm per variable + Keras Adam (keras/optimizers/adam.py update_step)
// ---------------------------------------------------------------------------
__global__ void sumsq_kernel(AdamArgs a) {
  __shared__ double red[kT / 64];
  const int c = blockIdx.x;
  const float* g = a.g + a.cstart[c];
  double s = 0.0;
  for (int i = threadIdx.x; i < a.clen[c]; i += blockDim.x) {
    const double v = g[i];
    s += v * v;
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double r = 0.0;
    for (int w = 0; w < kT / 64; ++w) r += red[w];
    a.partial[c] = r;
  }
}

__global__ void clip_scale_kernel(AdamArgs a) {
  __shared__ double red[kT / 64];
  const int k = blockIdx.x;
  double s = 0.0;
  for (int c = a.vfirst[k] + threadIdx.x; c < a.vfirst[k] + a.vcount[k]; c += blockDim.x) s += a.partial[c];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x != 0) return;
  s = 0.0;
  for (int w = 0; w < kT / 64; ++w) s += red[w];
  const double gs = a.grad_scale;
  double scale = gs;
  if (a.clipnorm > 0.f) {
    const double nrm = sqrt(s) * fabs(gs);                 // norm of the scaled gradient
    scale = gs * (double)a.clipnorm / fmax(nrm, (double)a.clipnorm);
  }
  a.vscale[k] = (float)scale;
}

__global__ void adam_kernel(AdamArgs a) {
#pragma clang fp contract(off)
  const int c = blockIdx.x;
  const long long o = a.cstart[c];
  const float sc = a.vscale[a.cvar[c]];
  const float b1c = 1.0f - a.beta_1, b2c = 1.0f - a.beta_2;
  for (int i = threadIdx.x; i < a.clen[c]; i += blockDim.x) {
    const long long e = o + i;
    const float g = a.g[e] * sc;
    float m = a.m[e], v = a.v[e];
    m = m + (g - m) * b1c;
    v = v + (g * g - v) * b2c;
    a.m[e] = m;
    a.v[e] = v;
    a.w[e] = a.w[e] - (m * a.alpha) / (sqrtf(v) + a.epsilon);
  }
}

}  // namespace

hipError_t im2col(const ConvIn& ci, int B, const float* lab, const float* tim, const float* x1, const float* x2,
                  float* A, hipStream_t s) {
  hipLaunchKernelGGL(im2col_kernel, dim3(B * ci.lout()), dim3(kT), 0, s, ci, B, lab, tim, x1, x2, A);
  return hipGetLastError();
}

hipError_t col2im(const ConvIn& ci, int B, const float* dA, float* dlab, float* dtim, float* dx1, float* dx2,
                  hipStream_t s) {
  hipLaunchKernelGGL(col2im_kernel, dim3(B * ci.Lsrc), dim3(kT), 0, s, ci, B, dA, dlab, dtim, dx1, dx2);
  return hipGetLastError();
}

hipError_t bias_act(float* Y, int M, int N, int ld, const float* b1, int relu, hipStream_t s) {
  hipLaunchKernelGGL(bias_act_kernel, dim3(blocks_for((size_t)M * N)), dim3(kT), 0, s, Y, M, N, ld, b1, relu);
  return hipGetLastError();
}

hipError_t gelu_fwd(const float* a, float* h, int M, int N, int ldh, hipStream_t s) {
  hipLaunchKernelGGL(gelu_fwd_kernel, dim3(blocks_for((size_t)M * N)), dim3(kT), 0, s, a, h, M, N, ldh);
  return hipGetLastError();
}

hipError_t gelu_bwd(const float* dh, const float* a, float* da, int n, hipStream_t s) {
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3(blocks_for(n)), dim3(kT), 0, s, dh, a, da, n);
  return hipGetLastError();
}

hipError_t relu_mask(float* d, const float* y, int M, int N, int ldy, hipStream_t s) {
  hipLaunchKernelGGL(relu_mask_kernel, dim3(blocks_for((size_t)M * N)), dim3(kT), 0, s, d, y, M, N, ldy);
  return hipGetLastError();
}

hipError_t copy_rows(const float* src, int M, int N, float* dst, int ldd, hipStream_t s) {
  hipLaunchKernelGGL(copy_rows_kernel, dim3(blocks_for((size_t)M * N)), dim3(kT), 0, s, src, M, N, dst, ldd);
  return hipGetLastError();
}

hipError_t fill_strided(float* p, size_t n, size_t stride, float v, hipStream_t s) {
  hipLaunchKernelGGL(fill_kernel, dim3(blocks_for(n)), dim3(kT), 0, s, p, n, stride, v);
  return hipGetLastError();
}

hipError_t maxpool_fwd(const float* out, float* pool, int B, int L, int C, hipStream_t s) {
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(blocks_for((size_t)B * (L / 2) * C)), dim3(kT), 0, s, out, pool, B,
                     L, C);
  return hipGetLastError();
}

hipError_t pool_mask_bwd(const float* out, const float* dpool, const float* dskip, float* dpre, int B, int L,
                         int C, hipStream_t s) {
  hipLaunchKernelGGL(pool_mask_bwd_kernel, dim3(blocks_for((size_t)B * L * C)), dim3(kT), 0, s, out, dpool, dskip,
                     dpre, B, L, C);
  return hipGetLastError();
}

hipError_t fold_weff(const float* W, const float* bw, const float* R, const float* br, float* Weff, int taps,
                     int padl, int C, int N, hipStream_t s) {
  hipLaunchKernelGGL(fold_weff_kernel, dim3(blocks_for((size_t)taps * C * N + N)), dim3(kT), 0, s, W, bw, R, br, Weff,
                     taps, padl, C, N);
  return hipGetLastError();
}

hipError_t time_embed(const int* t, int B, int dim, float* emb, int ld, hipStream_t s) {
  hipLaunchKernelGGL(time_embed_kernel, dim3(blocks_for((size_t)B * dim / 2)), dim3(kT), 0, s, t, B, dim, emb, ld);
  return hipGetLastError();
}

hipError_t qsample(const float* x0, const int* t_in, const float* noise_in, uint64_t seed, uint64_t goff,
                   int64_t iter, int B, int T, const float* tab, int* t_out, float* noise_out, float* xt,
                   hipStream_t s) {
  hipLaunchKernelGGL(qsample_kernel, dim3((B * 48 + kT - 1) / kT), dim3(kT), 0, s, x0, t_in, noise_in, seed, goff,
                     iter, B, T, tab, t_out, noise_out, xt);
  return hipGetLastError();
}

hipError_t loss(const LossArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(loss_kernel, dim3(a.B), dim3(128), 0, s, a);
  return hipGetLastError();
}

hipError_t loss_finish(const float* sse, const float* vlb, const float* dbias_part, int B, int n_out, int n_el,
                       float* loss_out, double* stats, float* dbias, hipStream_t s) {
  hipLaunchKernelGGL(loss_finish_kernel, dim3(1), dim3(256), 0, s, sse, vlb, dbias_part, B, n_out, n_el, loss_out,
                     stats, dbias);
  return hipGetLastError();
}

hipError_t adam(const AdamArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(sumsq_kernel, dim3(a.n_chunks), dim3(kT), 0, s, a);
  hipLaunchKernelGGL(clip_scale_kernel, dim3(a.n_vars), dim3(kT), 0, s, a);
  hipLaunchKernelGGL(adam_kernel, dim3(a.n_chunks), dim3(kT), 0, s, a);
  return hipGetLastError();
}

}  // namespace pettrain_k
