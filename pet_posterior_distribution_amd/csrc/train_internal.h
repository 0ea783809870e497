// Internal declarations of the training step (train_kernels.hip <-> train_api.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstddef>

namespace pettrain_k {

// im2col rows carry K + 1 columns (last = 1): GEMMs against [W ; bias] add the bias and
// return the bias gradient as the weight gradient's last row (kernel and bias are adjacent in
// the weight blob).
// Channels of a conv input, in the reference's concat order:
//   [label (49) | time (1) | x1 (c1) | x2 (c2)]   (networks.py:1022, 1043, 1057)
// over Lsrc source positions; ups = 1 inserts UpSampling1D(2) before the conv
// (Lout = 2 Lsrc), else Lout = Lsrc.  label is the label projection's raw
// (B, 49*Lsrc) output (Reshape((L, -1)) reinterprets it: position p, channel c
// at p*49 + c); time is (B, Lsrc).
struct ConvIn {
  int has_cond;     // label + time channels present
  int c1, c2;
  int Lsrc, ups;
  int taps, padl;
  __host__ __device__ int cfull() const { return (has_cond ? 50 : 0) + c1 + c2; }
  __host__ __device__ int lout() const { return ups ? 2 * Lsrc : Lsrc; }
};

hipError_t im2col(const ConvIn& ci, int B, const float* lab, const float* tim, const float* x1, const float* x2,
                  float* A, hipStream_t s);
hipError_t col2im(const ConvIn& ci, int B, const float* dA, float* dlab, float* dtim, float* dx1, float* dx2,
                  hipStream_t s);
hipError_t bias_act(float* Y, int M, int N, int ld, const float* b1, int relu, hipStream_t s);
hipError_t gelu_fwd(const float* a, float* h, int M, int N, int ldh, hipStream_t s);
hipError_t gelu_bwd(const float* dh, const float* a, float* da, int n, hipStream_t s);
hipError_t relu_mask(float* d, const float* y, int M, int N, int ldy, hipStream_t s);   // d[M][N] *= (y > 0)
hipError_t copy_rows(const float* src, int M, int N, float* dst, int ldd, hipStream_t s);
hipError_t fill_strided(float* p, size_t n, size_t stride, float v, hipStream_t s);
hipError_t maxpool_fwd(const float* out, float* pool, int B, int L, int C, hipStream_t s);
// dpre = (out > 0) * (maxpool routing of dpool (or 0) + dskip (or 0))
hipError_t pool_mask_bwd(const float* out, const float* dpool, const float* dskip, float* dpre, int B, int L,
                         int C, hipStream_t s);
hipError_t fold_weff(const float* W, const float* bw, const float* R, const float* br, float* Weff, int taps,
                     int padl, int C, int N, hipStream_t s);
hipError_t time_embed(const int* t, int B, int dim, float* emb, int ld, hipStream_t s);
hipError_t qsample(const float* x0, const int* t_in, const float* noise_in, uint64_t seed, uint64_t goff,
                   int64_t iter, int B, int T, const float* tab, int* t_out, float* noise_out, float* xt,
                   hipStream_t s);

struct LossArgs {
  const float* y;        // network output [B][48][n_out]
  const float* x0;       // [B][48][2]
  const float* noise;
  const float* xt;
  const int* t;
  const float* tab;      // [kNTab][T]
  int T, B, n_out;
  int learn_mode;        // 0 fixed, 1 learn, 2 learn_ranged
  int param_mode;        // 0 eps, 1 x0, 2 v, 3 x_prev
  float lambda_vlb;
  float bin_width;
  float* dy;             // [B][48][n_out]
  float* sse;            // [B]
  float* vlb;            // [B]
  float* dbias_part;     // [B][n_out] per-sample column sums of dy
};
hipError_t loss(const LossArgs& a, hipStream_t s);
// loss_out[b] = mse + vlb[b] (mse = sum(sse) / (B*96)); stats[3] = {mean loss, mse, mean vlb};
// dbias[q] = sum_b dbias_part[b][q] (the final layer's bias gradient)
hipError_t loss_finish(const float* sse, const float* vlb, const float* dbias_part, int B, int n_out, int n_el,
                       float* loss_out, double* stats, float* dbias, hipStream_t s);

// Optimizer over the whole blob, described as chunks of at most kChunk elements of
// one variable each (chunk c: variable var[c], elements [start[c], start[c]+len[c])).
constexpr int kChunk = 4096;
struct AdamArgs {
  float* w; const float* g; float* m; float* v;
  const int* cvar; const long long* cstart; const int* clen; int n_chunks;
  const int* vfirst; const int* vcount; int n_vars;   // chunks of variable k: vfirst[k] .. + vcount[k]
  double* partial;       // [n_chunks]
  float* vscale;         // [n_vars]: grad_scale * clip factor
  float grad_scale, clipnorm, alpha, beta_1, beta_2, epsilon;
};
hipError_t adam(const AdamArgs& a, hipStream_t s);

}  // namespace pettrain_k
