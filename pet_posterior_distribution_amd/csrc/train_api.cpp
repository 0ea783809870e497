// C-ABI implementation of the training step (include/pettrain.h), SURVEY.md 8(f) row 4.
//
// ImprovedDDPM.train_step (diffusion_model.py:533-598) on one GPU, fp32:
//   q-sample -> U-Net forward (im2col + rocBLAS GEMM per conv, activations kept)
//   -> loss + analytic output gradient -> backward through every layer
//   (weight grads A^T dY, data grads dY W^T + col2im) -> per-variable clip + Adam.
// The layer walk mirrors UnetConditional.call (networks.py:994-1093) at the
// shipped config; the CPU restatement of every gradient is oracle/train_ref.py.
#include "pettrain.h"
#include "petdiff_internal.h"
#include "petdiff_spec.h"
#include "train_internal.h"

#include <rocblas/rocblas.h>

#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

using namespace petdiff;
namespace K = pettrain_k;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPC(expr)                                                                        \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail(PETDIFF_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));    \
  } while (0)

#define RBC(expr)                                                                                   \
  do {                                                                                              \
    rocblas_status s_ = (expr);                                                                     \
    if (s_ != rocblas_status_success)                                                               \
      return fail(PETDIFF_ERR_HIP, std::string(#expr) + ": " + rocblas_status_to_string(s_));      \
  } while (0)

#define CHK(expr)                    \
  do {                               \
    int r_ = (expr);                 \
    if (r_ != PETDIFF_OK) return r_; \
  } while (0)

struct Buf {
  void* p = nullptr;
  size_t bytes = 0;
  ~Buf() { if (p) (void)hipFree(p); }
  hipError_t alloc(size_t b) {
    if (b <= bytes && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    hipError_t e = hipMalloc(&p, b ? b : 16);
    if (e == hipSuccess) bytes = b;
    return e;
  }
  float* f() const { return reinterpret_cast<float*>(p); }
  int* i() const { return reinterpret_cast<int*>(p); }
};

// Shipped-config geometry
constexpr int kDownL[4] = {48, 24, 12, 6};
constexpr int kDownCin[4] = {2, 128, 256, 512};
constexpr int kDownCout[4] = {128, 256, 512, 1024};
constexpr int kUpLc[3] = {6, 12, 24};          // coarse length (label/time length)
constexpr int kUpCin[3] = {1024, 512, 256};
constexpr int kUpCout[3] = {512, 256, 128};
constexpr int kLevelL[7] = {48, 24, 12, 6, 6, 12, 24};   // label/time length of cond level p

K::ConvIn down_in(int d) { return K::ConvIn{1, kDownCin[d], 0, kDownL[d], 0, 6, 2}; }
K::ConvIn upconv_in(int u) { return K::ConvIn{1, kUpCin[u], 0, kUpLc[u], 1, 2, 0}; }
K::ConvIn block_in(int u) { return K::ConvIn{0, kUpCout[u], kUpCout[u], 2 * kUpLc[u], 0, 6, 2}; }

}  // namespace

struct pettrain_ctx {
  petdiff_config cfg;
  pettrain_config opt;
  int device = 0, n_out = 4, T = 0, learn_mode = 2, param_mode = 0;
  std::vector<Spec> spec;
  std::map<std::string, size_t> off;
  size_t n_w = 0;
  Buf w, g, m, v, tab;
  Buf cvar, cstart, clen, vfirst, vcount, partial, vscale;
  int n_chunks = 0, n_vars = 0;
  Buf weff[7];                     // folded ConvBlock kernels: down0..3, up0..2 blocks
  rocblas_handle rb = nullptr;
  int B_cap = 0;
  // forward
  Buf t, noise, xt, emb, a_t, h_t, cond_aug, e1, e2, e3, z, lab[7], tim[7];
  Buf A_dn[4], out_dn[4], pool[3], A_uc[3], hu[3], A_bk[3], out_up[3], y4;
  // backward
  Buf dy4, dA, dpre, d_out_up[3], d_out_dn3, d_pool[3], dskip[3], dhu, dlab, dtim, dz, dh_t, da_t, de1, de2, de3,
      sse, vlb, dbias_part, stats;
  int64_t iter = 0;
  int last_B = 0;          // batch of the last backward pass (gradients valid)
  bool has_stats = false;  // a forward + loss ran (pettrain_last_stats valid)

  float* W(const std::string& n) const { return w.f() + off.at(n); }
  float* G(const std::string& n) const { return g.f() + off.at(n); }
};

namespace {

// Row-major C[M,N] = op(A)[M,K] op(B)[K,N] (+ beta C) on the handle's rocBLAS stream.
int gemm(pettrain_ctx* h, bool ta, bool tb, int M, int N, int Kd, const float* A, int lda, const float* B, int ldb,
         float* C, int ldc, float beta) {
  const float one = 1.0f;
  RBC(rocblas_sgemm(h->rb, tb ? rocblas_operation_transpose : rocblas_operation_none,
                    ta ? rocblas_operation_transpose : rocblas_operation_none, N, M, Kd, &one, B, ldb, A, lda, &beta,
                    C, ldc));
  return PETDIFF_OK;
}

// Augmented activations: every tensor that feeds a Dense layer or a conv GEMM carries a
// trailing column of ones (row stride K + 1), and the weight operand is the blob's
// [kernel ; bias] block (adjacent in the blob), so the GEMM adds the bias and the
// weight-gradient GEMM returns [d kernel ; d bias] in one pass.
int ensure(pettrain_ctx* h, int B) {
  if (B <= h->B_cap) return PETDIFF_OK;
  const size_t Bz = (size_t)B, F = 4, R = Bz * 49;
  HIPC(h->t.alloc(Bz * 4));
  HIPC(h->noise.alloc(Bz * 96 * F));
  HIPC(h->xt.alloc(Bz * 96 * F));
  HIPC(h->emb.alloc(Bz * 65 * F));
  HIPC(h->a_t.alloc(Bz * 48 * F));
  HIPC(h->h_t.alloc(Bz * 49 * F));
  HIPC(h->cond_aug.alloc(R * 55 * F));
  HIPC(h->e1.alloc(R * 257 * F));
  HIPC(h->e2.alloc(R * 129 * F));
  HIPC(h->e3.alloc(R * 65 * F));
  HIPC(h->z.alloc(R * 33 * F));
  for (int p = 0; p < 7; ++p) {
    HIPC(h->lab[p].alloc(R * kLevelL[p] * F));
    HIPC(h->tim[p].alloc(Bz * kLevelL[p] * F));
  }
  size_t maxA = 0;
  for (int d = 0; d < 4; ++d) {
    const K::ConvIn ci = down_in(d);
    const size_t k = (size_t)ci.taps * ci.cfull();
    maxA = std::max(maxA, Bz * ci.lout() * k);
    HIPC(h->A_dn[d].alloc(Bz * ci.lout() * (k + 1) * F));
    HIPC(h->out_dn[d].alloc(Bz * kDownL[d] * kDownCout[d] * F));
    if (d < 3) {
      HIPC(h->pool[d].alloc(Bz * (kDownL[d] / 2) * kDownCout[d] * F));
      HIPC(h->d_pool[d].alloc(Bz * (kDownL[d] / 2) * kDownCout[d] * F));
      HIPC(h->dskip[d].alloc(Bz * kDownL[d] * kDownCout[d] * F));
    }
  }
  for (int u = 0; u < 3; ++u) {
    const K::ConvIn uc = upconv_in(u), bk = block_in(u);
    const size_t k1 = (size_t)uc.taps * uc.cfull(), k2 = (size_t)bk.taps * bk.cfull();
    maxA = std::max(maxA, std::max(Bz * uc.lout() * k1, Bz * bk.lout() * k2));
    HIPC(h->A_uc[u].alloc(Bz * uc.lout() * (k1 + 1) * F));
    HIPC(h->A_bk[u].alloc(Bz * bk.lout() * (k2 + 1) * F));
    HIPC(h->hu[u].alloc(Bz * 2 * kUpLc[u] * kUpCout[u] * F));
    HIPC(h->out_up[u].alloc(Bz * 2 * kUpLc[u] * kUpCout[u] * F));
    HIPC(h->d_out_up[u].alloc(Bz * 2 * kUpLc[u] * kUpCout[u] * F));
  }
  HIPC(h->y4.alloc(Bz * 48 * h->n_out * F));
  HIPC(h->dy4.alloc(Bz * 48 * h->n_out * F));
  HIPC(h->dA.alloc(maxA * F));
  HIPC(h->dpre.alloc(Bz * 6144 * F));
  HIPC(h->d_out_dn3.alloc(Bz * 6 * 1024 * F));
  HIPC(h->dhu.alloc(Bz * 6144 * F));
  HIPC(h->dlab.alloc(R * 48 * F));
  HIPC(h->dtim.alloc(Bz * 48 * F));
  HIPC(h->dz.alloc(R * 32 * F));
  HIPC(h->dh_t.alloc(Bz * 48 * F));
  HIPC(h->da_t.alloc(Bz * 48 * F));
  HIPC(h->de1.alloc(R * 256 * F));
  HIPC(h->de2.alloc(R * 128 * F));
  HIPC(h->de3.alloc(R * 64 * F));
  HIPC(h->sse.alloc(Bz * F));
  HIPC(h->vlb.alloc(Bz * F));
  HIPC(h->dbias_part.alloc(Bz * h->n_out * F));
  HIPC(h->stats.alloc(3 * sizeof(double)));
  // the ones columns (never overwritten: GEMMs write N of the N + 1 columns)
  struct { Buf* b; size_t rows; int ld; } aug[] = {{&h->emb, Bz, 65}, {&h->h_t, Bz, 49}, {&h->cond_aug, R, 55},
                                                   {&h->e1, R, 257}, {&h->e2, R, 129}, {&h->e3, R, 65},
                                                   {&h->z, R, 33}};
  for (auto& a : aug) HIPC(K::fill_strided(a.b->f() + (a.ld - 1), a.rows, a.ld, 1.0f, 0));
  HIPC(hipDeviceSynchronize());
  h->B_cap = B;
  return PETDIFF_OK;
}

// dense forward: Y[M, N] (row stride ldy) = [X | 1] [kernel ; bias], X of row stride Kd + 1
int dense_fwd(pettrain_ctx* h, const float* X, int M, int Kd, const std::string& name, int N, float* Y, int ldy,
              int relu, hipStream_t s) {
  CHK(gemm(h, false, false, M, N, Kd + 1, X, Kd + 1, h->W(name + ".kernel"), N, Y, ldy, 0.f));
  if (relu) HIPC(K::bias_act(Y, M, N, ldy, nullptr, 1, s));
  return PETDIFF_OK;
}

// dense backward: G [kernel ; bias] = [X | 1]^T dY; dX (=|+=) dY kernel^T (dX may be null)
int dense_bwd(pettrain_ctx* h, const float* X, const float* dY, int M, int Kd, const std::string& name, int N,
              float* dX, float beta) {
  CHK(gemm(h, true, false, Kd + 1, N, M, X, Kd + 1, dY, N, h->G(name + ".kernel"), N, 0.f));
  if (dX) CHK(gemm(h, false, true, M, Kd, N, dY, N, h->W(name + ".kernel"), N, dX, Kd, beta));
  return PETDIFF_OK;
}

// conv forward: out[B*Lout, cout] = [im2col | 1] [W ; bias] (relu optional)
int conv_fwd(pettrain_ctx* h, const K::ConvIn& ci, int B, const float* lab, const float* tim, const float* x1,
             const float* x2, float* A, const float* Wk, int cout, int relu, float* out, hipStream_t s) {
  HIPC(K::im2col(ci, B, lab, tim, x1, x2, A, s));
  const int M = B * ci.lout(), Kd = ci.taps * ci.cfull();
  CHK(gemm(h, false, false, M, cout, Kd + 1, A, Kd + 1, Wk, cout, out, cout, 0.f));
  if (relu) HIPC(K::bias_act(out, M, cout, cout, nullptr, 1, s));
  return PETDIFF_OK;
}

// conv backward from dpre: G [kernel ; bias] = [A | 1]^T dpre, dA = dpre W^T, col2im
int conv_bwd(pettrain_ctx* h, const K::ConvIn& ci, int B, const float* A, const float* Wk, int cout,
             const float* dpre, float* Gk, float* dlab, float* dtim, float* dx1, float* dx2, hipStream_t s) {
  const int M = B * ci.lout(), Kd = ci.taps * ci.cfull();
  CHK(gemm(h, true, false, Kd + 1, cout, M, A, Kd + 1, dpre, cout, Gk, cout, 0.f));
  CHK(gemm(h, false, true, M, Kd, cout, dpre, cout, Wk, cout, h->dA.f(), Kd, 0.f));
  HIPC(K::col2im(ci, B, h->dA.f(), dlab, dtim, dx1, dx2, s));
  return PETDIFF_OK;
}

// the residual 1x1 kernel / bias share the gradient of the centre tap / conv bias
int copy_res_grads(pettrain_ctx* h, const std::string& p, int cin_full, int cout, hipStream_t s) {
  const size_t cn = (size_t)cin_full * cout;
  HIPC(hipMemcpyAsync(h->G(p + ".res.kernel"), h->G(p + ".conv.kernel") + 2 * cn, cn * 4, hipMemcpyDeviceToDevice,
                      s));
  HIPC(hipMemcpyAsync(h->G(p + ".res.bias"), h->G(p + ".conv.bias"), (size_t)cout * 4, hipMemcpyDeviceToDevice, s));
  return PETDIFF_OK;
}

std::string level_prefix(int p) { return p < 4 ? "down" + std::to_string(p) : "up" + std::to_string(p - 4); }

// label / time projection backward of cond level p (networks.py:915-921, 958-964)
int cond_bwd(pettrain_ctx* h, int p, int B, bool first) {
  const std::string pre = level_prefix(p);
  const int L = kLevelL[p], R = B * 49;
  CHK(dense_bwd(h, h->z.f(), h->dlab.f(), R, 32, pre + ".label_proj", L, h->dz.f(), first ? 0.f : 1.f));
  CHK(dense_bwd(h, h->h_t.f(), h->dtim.f(), B, 48, pre + ".time_proj", L, h->dh_t.f(), first ? 0.f : 1.f));
  return PETDIFF_OK;
}

int forward_backward(pettrain_ctx* h, const float* x0, const float* cond, int B, const int32_t* t_in,
                     const float* noise_in, uint64_t seed, uint64_t goff, float* loss_out, hipStream_t s,
                     bool backward = true) {
  CHK(ensure(h, B));
  RBC(rocblas_set_stream(h->rb, s));
  const int R = B * 49;
  // q-sample (diffusion_model.py:542-551)
  HIPC(K::qsample(x0, t_in, noise_in, seed, goff, h->iter, B, h->T, h->tab.f(), h->t.i(), h->noise.f(), h->xt.f(),
                  s));
  // time MLP and condition encoder (networks.py:182-198, 235-258, 574-586)
  HIPC(K::time_embed(h->t.i(), B, 64, h->emb.f(), 65, s));
  CHK(dense_fwd(h, h->emb.f(), B, 64, "time_mlp", 48, h->a_t.f(), 48, 0, s));
  HIPC(K::gelu_fwd(h->a_t.f(), h->h_t.f(), B, 48, 49, s));
  HIPC(K::copy_rows(cond, R, 54, h->cond_aug.f(), 55, s));
  CHK(dense_fwd(h, h->cond_aug.f(), R, 54, "cond_enc.hidden0", 256, h->e1.f(), 257, 1, s));
  CHK(dense_fwd(h, h->e1.f(), R, 256, "cond_enc.hidden1", 128, h->e2.f(), 129, 1, s));
  CHK(dense_fwd(h, h->e2.f(), R, 128, "cond_enc.hidden2", 64, h->e3.f(), 65, 1, s));
  CHK(dense_fwd(h, h->e3.f(), R, 64, "cond_enc.z", 32, h->z.f(), 33, 0, s));
  for (int p = 0; p < 7; ++p) {
    const std::string pre = level_prefix(p);
    CHK(dense_fwd(h, h->z.f(), R, 32, pre + ".label_proj", kLevelL[p], h->lab[p].f(), kLevelL[p], 0, s));
    CHK(dense_fwd(h, h->h_t.f(), B, 48, pre + ".time_proj", kLevelL[p], h->tim[p].f(), kLevelL[p], 0, s));
  }
  // down path (networks.py:1010-1031)
  for (int d = 0; d < 4; ++d) {
    const std::string p = "down" + std::to_string(d);
    const K::ConvIn ci = down_in(d);
    HIPC(K::fold_weff(h->W(p + ".conv.kernel"), h->W(p + ".conv.bias"), h->W(p + ".res.kernel"),
                      h->W(p + ".res.bias"), h->weff[d].f(), 6, 2, ci.cfull(), kDownCout[d], s));
    CHK(conv_fwd(h, ci, B, h->lab[d].f(), h->tim[d].f(), d == 0 ? h->xt.f() : h->pool[d - 1].f(), nullptr,
                 h->A_dn[d].f(), h->weff[d].f(), kDownCout[d], 1, h->out_dn[d].f(), s));
    if (d < 3) HIPC(K::maxpool_fwd(h->out_dn[d].f(), h->pool[d].f(), B, kDownL[d], kDownCout[d], s));
  }
  // up path (networks.py:1033-1072)
  for (int u = 0; u < 3; ++u) {
    const std::string p = "up" + std::to_string(u);
    const K::ConvIn uc = upconv_in(u), bk = block_in(u);
    const float* hin = u == 0 ? h->out_dn[3].f() : h->out_up[u - 1].f();
    CHK(conv_fwd(h, uc, B, h->lab[4 + u].f(), h->tim[4 + u].f(), hin, nullptr, h->A_uc[u].f(),
                 h->W(p + ".upconv.kernel"), kUpCout[u], 0, h->hu[u].f(), s));
    HIPC(K::fold_weff(h->W(p + ".conv.kernel"), h->W(p + ".conv.bias"), h->W(p + ".res.kernel"),
                      h->W(p + ".res.bias"), h->weff[4 + u].f(), 6, 2, bk.cfull(), kUpCout[u], s));
    CHK(conv_fwd(h, bk, B, nullptr, nullptr, h->out_dn[2 - u].f(), h->hu[u].f(), h->A_bk[u].f(), h->weff[4 + u].f(),
                 kUpCout[u], 1, h->out_up[u].f(), s));
  }
  // final Conv1D 1x1 (networks.py:1074)
  const int n_out = h->n_out;
  CHK(gemm(h, false, false, B * 48, n_out, 128, h->out_up[2].f(), 128, h->W("final.kernel"), n_out, h->y4.f(), n_out,
           0.f));
  HIPC(K::bias_act(h->y4.f(), B * 48, n_out, n_out, h->W("final.bias"), 0, s));
  // loss + d loss / d output (diffusion_model.py:498-578)
  K::LossArgs la{};
  la.y = h->y4.f();
  la.x0 = x0;
  la.noise = h->noise.f();
  la.xt = h->xt.f();
  la.t = h->t.i();
  la.tab = h->tab.f();
  la.T = h->T;
  la.B = B;
  la.n_out = n_out;
  la.learn_mode = h->learn_mode;
  la.param_mode = h->param_mode;
  la.lambda_vlb = h->opt.lambda_vlb;
  la.bin_width = (float)(2.0 * 1.34896 / std::cbrt((double)B * 48.0));    // freedman_diaconis_rule (:529-531)
  la.dy = h->dy4.f();
  la.sse = h->sse.f();
  la.vlb = h->vlb.f();
  la.dbias_part = h->dbias_part.f();
  HIPC(K::loss(la, s));
  HIPC(K::loss_finish(h->sse.f(), h->vlb.f(), h->dbias_part.f(), B, n_out, B * 96, loss_out,
                      reinterpret_cast<double*>(h->stats.p), backward ? h->G("final.bias") : nullptr, s));
  h->has_stats = true;
  if (!backward) return PETDIFF_OK;   // test_step: loss only, the gradient blob is untouched

  // ---------------- backward ----------------
  CHK(gemm(h, true, false, 128, n_out, B * 48, h->out_up[2].f(), 128, h->dy4.f(), n_out, h->G("final.kernel"), n_out,
           0.f));
  CHK(gemm(h, false, true, B * 48, 128, n_out, h->dy4.f(), n_out, h->W("final.kernel"), n_out, h->d_out_up[2].f(),
           128, 0.f));
  bool first = true;
  for (int u = 2; u >= 0; --u) {
    const std::string p = "up" + std::to_string(u);
    const K::ConvIn uc = upconv_in(u), bk = block_in(u);
    HIPC(K::pool_mask_bwd(h->out_up[u].f(), nullptr, h->d_out_up[u].f(), h->dpre.f(), B, bk.lout(), kUpCout[u], s));
    CHK(conv_bwd(h, bk, B, h->A_bk[u].f(), h->weff[4 + u].f(), kUpCout[u], h->dpre.f(), h->G(p + ".conv.kernel"),
                 nullptr, nullptr, h->dskip[2 - u].f(), h->dhu.f(), s));
    CHK(copy_res_grads(h, p, bk.cfull(), kUpCout[u], s));
    float* dhin = u == 0 ? h->d_out_dn3.f() : h->d_out_up[u - 1].f();
    CHK(conv_bwd(h, uc, B, h->A_uc[u].f(), h->W(p + ".upconv.kernel"), kUpCout[u], h->dhu.f(),
                 h->G(p + ".upconv.kernel"), h->dlab.f(), h->dtim.f(), dhin, nullptr, s));
    CHK(cond_bwd(h, 4 + u, B, first));
    first = false;
  }
  for (int d = 3; d >= 0; --d) {
    const std::string p = "down" + std::to_string(d);
    const K::ConvIn ci = down_in(d);
    if (d == 3)
      HIPC(K::pool_mask_bwd(h->out_dn[3].f(), nullptr, h->d_out_dn3.f(), h->dpre.f(), B, 6, 1024, s));
    else
      HIPC(K::pool_mask_bwd(h->out_dn[d].f(), h->d_pool[d].f(), h->dskip[d].f(), h->dpre.f(), B, kDownL[d],
                            kDownCout[d], s));
    CHK(conv_bwd(h, ci, B, h->A_dn[d].f(), h->weff[d].f(), kDownCout[d], h->dpre.f(), h->G(p + ".conv.kernel"),
                 h->dlab.f(), h->dtim.f(), d > 0 ? h->d_pool[d - 1].f() : nullptr, nullptr, s));
    CHK(copy_res_grads(h, p, ci.cfull(), kDownCout[d], s));
    CHK(cond_bwd(h, d, B, false));
  }
  // condition encoder backward (ReLU masks read the augmented activations)
  CHK(dense_bwd(h, h->e3.f(), h->dz.f(), R, 64, "cond_enc.z", 32, h->de3.f(), 0.f));
  HIPC(K::relu_mask(h->de3.f(), h->e3.f(), R, 64, 65, s));
  CHK(dense_bwd(h, h->e2.f(), h->de3.f(), R, 128, "cond_enc.hidden2", 64, h->de2.f(), 0.f));
  HIPC(K::relu_mask(h->de2.f(), h->e2.f(), R, 128, 129, s));
  CHK(dense_bwd(h, h->e1.f(), h->de2.f(), R, 256, "cond_enc.hidden1", 128, h->de1.f(), 0.f));
  HIPC(K::relu_mask(h->de1.f(), h->e1.f(), R, 256, 257, s));
  CHK(dense_bwd(h, h->cond_aug.f(), h->de1.f(), R, 54, "cond_enc.hidden0", 256, nullptr, 0.f));
  // time MLP backward (GELU exact)
  HIPC(K::gelu_bwd(h->dh_t.f(), h->a_t.f(), h->da_t.f(), B * 48, s));
  CHK(dense_bwd(h, h->emb.f(), h->da_t.f(), B, 64, "time_mlp", 48, nullptr, 0.f));
  h->last_B = B;
  return PETDIFF_OK;
}

}  // namespace

extern "C" {

const char* pettrain_last_error(void) { return g_err.c_str(); }

int pettrain_default_config(pettrain_config* o) {
  if (!o) return fail(PETDIFF_ERR_INVALID, "null argument");
  o->learning_rate = 2e-4f;
  o->decay_steps = 1.0f;
  o->decay_rate = 1.0f;
  o->beta_1 = 0.9f;
  o->beta_2 = 0.999f;
  o->epsilon = 1e-7f;
  o->clipnorm = 1.5f;
  o->lambda_vlb = 0.1f;
  return PETDIFF_OK;
}

int pettrain_create(const petdiff_config* cfg, const float* weights, size_t n_weights, const float* tab, int T,
                    const pettrain_config* opt, int device, pettrain_handle* out) {
  if (!cfg || !weights || !tab || !opt || !out || T <= 1) return fail(PETDIFF_ERR_INVALID, "bad arguments");
  if (!is_shipped_arch(*cfg))
    return fail(PETDIFF_ERR_UNSUPPORTED, "only the shipped UnetConditional architecture is compiled");
  if (cfg->learn_variance < 0 || cfg->learn_variance > 2 || cfg->parameterization < 0 || cfg->parameterization > 3)
    return fail(PETDIFF_ERR_INVALID, "bad learn_variance / parameterization");
  if (!(opt->decay_steps > 0.f) || !(opt->learning_rate >= 0.f))
    return fail(PETDIFF_ERR_INVALID, "bad optimizer config");
  std::unique_ptr<pettrain_ctx> h(new pettrain_ctx());
  h->cfg = *cfg;
  h->opt = *opt;
  h->device = device;
  h->T = T;
  h->learn_mode = cfg->learn_variance;
  h->param_mode = cfg->parameterization;
  h->n_out = cfg->learn_variance == PETDIFF_LEARN_FIXED ? cfg->n_par : 2 * cfg->n_par;
  h->spec = make_spec(*cfg, h->n_out);
  h->n_w = h->spec.back().off + h->spec.back().size;
  if (n_weights != h->n_w)
    return fail(PETDIFF_ERR_INVALID, "weight blob has " + std::to_string(n_weights) + " values, expected " +
                                         std::to_string(h->n_w));
  for (auto& s : h->spec) h->off[s.name] = s.off;
  HIPC(hipSetDevice(device));
  if (rocblas_create_handle(&h->rb) != rocblas_status_success) return fail(PETDIFF_ERR_HIP, "rocblas_create_handle");
  RBC(rocblas_set_atomics_mode(h->rb, rocblas_atomics_not_allowed));   // run-to-run deterministic GEMMs
  const size_t wb = h->n_w * 4;
  HIPC(h->w.alloc(wb));
  HIPC(h->g.alloc(wb));
  HIPC(h->m.alloc(wb));
  HIPC(h->v.alloc(wb));
  HIPC(hipMemcpy(h->w.p, weights, wb, hipMemcpyHostToDevice));
  HIPC(hipMemset(h->g.p, 0, wb));
  HIPC(hipMemset(h->m.p, 0, wb));
  HIPC(hipMemset(h->v.p, 0, wb));
  HIPC(h->tab.alloc((size_t)kNTab * T * 4));
  HIPC(hipMemcpy(h->tab.p, tab, (size_t)kNTab * T * 4, hipMemcpyHostToDevice));
  for (int d = 0; d < 4; ++d) HIPC(h->weff[d].alloc(((size_t)6 * down_in(d).cfull() + 1) * kDownCout[d] * 4));
  for (int u = 0; u < 3; ++u) HIPC(h->weff[4 + u].alloc(((size_t)6 * block_in(u).cfull() + 1) * kUpCout[u] * 4));
  // optimizer chunk tables
  std::vector<int> cvar, clen, vfirst, vcount;
  std::vector<long long> cstart;
  for (size_t k = 0; k < h->spec.size(); ++k) {
    vfirst.push_back((int)cvar.size());
    const Spec& s = h->spec[k];
    int n = 0;
    for (size_t o = 0; o < s.size; o += K::kChunk, ++n) {
      cvar.push_back((int)k);
      cstart.push_back((long long)(s.off + o));
      clen.push_back((int)std::min<size_t>(K::kChunk, s.size - o));
    }
    vcount.push_back(n);
  }
  h->n_chunks = (int)cvar.size();
  h->n_vars = (int)h->spec.size();
  HIPC(h->cvar.alloc(cvar.size() * 4));
  HIPC(h->clen.alloc(clen.size() * 4));
  HIPC(h->cstart.alloc(cstart.size() * 8));
  HIPC(h->vfirst.alloc(vfirst.size() * 4));
  HIPC(h->vcount.alloc(vcount.size() * 4));
  HIPC(h->partial.alloc(cvar.size() * 8));
  HIPC(h->vscale.alloc(vfirst.size() * 4));
  HIPC(hipMemcpy(h->cvar.p, cvar.data(), cvar.size() * 4, hipMemcpyHostToDevice));
  HIPC(hipMemcpy(h->clen.p, clen.data(), clen.size() * 4, hipMemcpyHostToDevice));
  HIPC(hipMemcpy(h->cstart.p, cstart.data(), cstart.size() * 8, hipMemcpyHostToDevice));
  HIPC(hipMemcpy(h->vfirst.p, vfirst.data(), vfirst.size() * 4, hipMemcpyHostToDevice));
  HIPC(hipMemcpy(h->vcount.p, vcount.data(), vcount.size() * 4, hipMemcpyHostToDevice));
  *out = h.release();
  return PETDIFF_OK;
}

void pettrain_destroy(pettrain_handle h) {
  if (!h) return;
  if (h->rb) (void)rocblas_destroy_handle(h->rb);
  delete h;
}

int pettrain_compute_gradients(pettrain_handle h, const float* x0_dev, const float* cond_dev, int B,
                               const int32_t* t_dev, const float* noise_dev, uint64_t seed, uint64_t sample_offset,
                               float* loss_dev, void* stream) {
  if (!h) return fail(PETDIFF_ERR_INVALID, "null handle");
  if (B <= 0 || !x0_dev || !cond_dev) return fail(PETDIFF_ERR_INVALID, "bad arguments");
  HIPC(hipSetDevice(h->device));
  return forward_backward(h, x0_dev, cond_dev, B, t_dev, noise_dev, seed, sample_offset, loss_dev,
                          (hipStream_t)stream);
}

int pettrain_compute_loss(pettrain_handle h, const float* x0_dev, const float* cond_dev, int B, const int32_t* t_dev,
                          const float* noise_dev, uint64_t seed, uint64_t sample_offset, float* loss_dev,
                          void* stream) {
  if (!h) return fail(PETDIFF_ERR_INVALID, "null handle");
  if (B <= 0 || !x0_dev || !cond_dev) return fail(PETDIFF_ERR_INVALID, "bad arguments");
  HIPC(hipSetDevice(h->device));
  return forward_backward(h, x0_dev, cond_dev, B, t_dev, noise_dev, seed, sample_offset, loss_dev,
                          (hipStream_t)stream, false);
}

int pettrain_apply_gradients(pettrain_handle h, float grad_scale, void* stream) {
  if (!h) return fail(PETDIFF_ERR_INVALID, "null handle");
  if (h->last_B <= 0) return fail(PETDIFF_ERR_INVALID, "no gradients computed yet");
  HIPC(hipSetDevice(h->device));
  // Keras: lr from the schedule at `iterations`, then alpha in the variable dtype (fp32)
  const pettrain_config& o = h->opt;
  const float lr = (float)((double)o.learning_rate * std::pow((double)o.decay_rate, (double)h->iter / o.decay_steps));
  const float step = (float)(h->iter + 1);
  const float b1p = std::pow(o.beta_1, step), b2p = std::pow(o.beta_2, step);
  K::AdamArgs a{};
  a.w = h->w.f();
  a.g = h->g.f();
  a.m = h->m.f();
  a.v = h->v.f();
  a.cvar = h->cvar.i();
  a.cstart = reinterpret_cast<const long long*>(h->cstart.p);
  a.clen = h->clen.i();
  a.n_chunks = h->n_chunks;
  a.vfirst = h->vfirst.i();
  a.vcount = h->vcount.i();
  a.n_vars = h->n_vars;
  a.partial = reinterpret_cast<double*>(h->partial.p);
  a.vscale = h->vscale.f();
  a.grad_scale = grad_scale;
  a.clipnorm = o.clipnorm;
  a.alpha = lr * std::sqrt(1.0f - b2p) / (1.0f - b1p);
  a.beta_1 = o.beta_1;
  a.beta_2 = o.beta_2;
  a.epsilon = o.epsilon;
  HIPC(K::adam(a, (hipStream_t)stream));
  h->iter += 1;
  return PETDIFF_OK;
}

int pettrain_step(pettrain_handle h, const float* x0_dev, const float* cond_dev, int B, const int32_t* t_dev,
                  const float* noise_dev, uint64_t seed, uint64_t sample_offset, float* loss_dev, void* stream) {
  CHK(pettrain_compute_gradients(h, x0_dev, cond_dev, B, t_dev, noise_dev, seed, sample_offset, loss_dev, stream));
  return pettrain_apply_gradients(h, 1.0f, stream);
}

float* pettrain_gradients(pettrain_handle h) { return h ? h->g.f() : nullptr; }

int pettrain_get_gradients(pettrain_handle h, float* dst_dev, void* stream) {
  if (!h || !dst_dev) return fail(PETDIFF_ERR_INVALID, "bad arguments");
  HIPC(hipMemcpyAsync(dst_dev, h->g.p, h->n_w * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return PETDIFF_OK;
}

int pettrain_set_gradients(pettrain_handle h, const float* src_dev, void* stream) {
  if (!h || !src_dev) return fail(PETDIFF_ERR_INVALID, "bad arguments");
  HIPC(hipMemcpyAsync(h->g.p, src_dev, h->n_w * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return PETDIFF_OK;
}

int pettrain_get_weights(pettrain_handle h, float* dst_dev, void* stream) {
  if (!h || !dst_dev) return fail(PETDIFF_ERR_INVALID, "bad arguments");
  HIPC(hipMemcpyAsync(dst_dev, h->w.p, h->n_w * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return PETDIFF_OK;
}

int pettrain_last_stats(pettrain_handle h, double* out3, void* stream) {
  if (!h || !out3) return fail(PETDIFF_ERR_INVALID, "bad arguments");
  if (!h->has_stats) return fail(PETDIFF_ERR_INVALID, "no step run yet");
  HIPC(hipMemcpyAsync(out3, h->stats.p, 3 * sizeof(double), hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPC(hipStreamSynchronize((hipStream_t)stream));
  return PETDIFF_OK;
}

int64_t pettrain_iterations(pettrain_handle h) { return h ? h->iter : -1; }

}  // extern "C"
