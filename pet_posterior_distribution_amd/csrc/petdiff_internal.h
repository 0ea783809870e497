// Internal declarations shared by the HIP kernels (unet_kernels.hip) and the
// C-ABI host implementation (petdiff_api.cpp).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstddef>

namespace petdiff {

typedef __bf16 bf16;
typedef _Float16 f16;

// Tile geometry of the implicit-GEMM Conv1D kernel (see DESIGN.md "conv kernel").
constexpr int kThreads = 256; // 4 waves; every wave owns a 96 x 64 output block (3 x 2 MFMA 32x32)

// Epilogue kinds
enum Epi : int {
  EPI_POOL = 0,   // relu, write skip + maxpool(2) output       (down blocks 1,2)
  EPI_RELU = 1,   // relu, write                                (down3, up blocks 0,1)
  EPI_LIN = 2,    // linear, write                              (up-sampling conv2)
  EPI_FINAL = 3,  // relu -> LDS -> final 1x1 conv -> p_sample  (up block 2)
};

// Per-timestep fp32 tables, row k of a [kNTab][T] array (computed on the host
// exactly like diffusion_model.py:98-105, 337-355; see petdiff.h).
enum Tab : int {
  TAB_BETA = 0, TAB_LOG_BETA, TAB_PLVC, TAB_POST_VAR, TAB_C1, TAB_C2, TAB_ALPHA_BAR,
  TAB_SQRT_AB, TAB_SQRT_1M_AB, TAB_INV_SQRT_AB, TAB_SQRT_RECIP_M1, TAB_RECIP_C1,
  TAB_C2_OVER_C1, kNTab
};

struct Down0Args {
  const float* x;            // [B][48][2]
  const float* w0;           // [6][2][128], residual folded into tap 2
  const float* cmap;         // [n_tac][48][128]
  const float* tmap;         // [T][48][128]
  const int* tac; const int* tvec; int t_uniform;
  void* s0; void* p0;        // T*
  int B;
};

struct FinalArgs {
  const float* wf;     // [128][n_out] final Conv1D 1x1 kernel
  const float* wf4;    // the same as [128][4], zero-padded when n_out == 2 (16-B rows for the fused final level)
  const float* bf;     // [n_out]
  int n_out;           // 4 (learned variance) or 2
  const float* x_t;    // [B][n_roi][2] current sample
  const float* z;      // injected noise [B][n_roi][2] or null -> Philox
  const unsigned long long* rng;  // device {seed, sample_offset}
  int rng_step;
  const float* tab;    // [kNTab][T]
  int T;
  int learn_mode;      // 0 fixed, 1 learn, 2 learn_ranged
  int param_mode;      // 0 eps, 1 x0, 2 v, 3 x_prev
  int flag_var_tilde;
  float* x_next;       // mean + noise (loop mode) or null
  float* x_all;        // keep_all_xt slot for this step or null
  float* mean_out;     // p_sample outputs or null
  float* var_out;
  float* var_tilde_out;
  float* net_out;      // raw network output [B][n_roi][n_out] or null (then no p_sample)
  // Fused first layer of the NEXT reverse step (loop mode): when next.t_uniform >= 0 the
  // epilogue also runs down0 on x_next for its own samples (writing next.s0 / next.p0),
  // which removes the down0 launch from every step but the first.
  Down0Args next;
};

template <typename T>
struct ConvArgs {
  const T* src1; int c1;     // first input (channels-last rows)
  const T* src2; int c2;     // second input (concat [src1 | src2]) or null
  const T* wpack;            // packed weights [Cout/NT][NC][taps][NT][ROWB] (fused: see pack_fused)
  const T* epack;            // fused up levels: left-edge correction weights [Cout/NT][NC2][2][NT][KC]
  T* out;                    // [B*L][cout]
  T* out_pool;               // [B*L/2][cout] (EPI_POOL)
  const float* cmap;         // [n_tac][L][cout] label contribution or null
  const float* tmap;         // [T][L][cout] time contribution + biases, or null
  const float* bias;         // [cout] when tmap is null
  const int* tac;            // [B] condition index per sample (null -> 0)
  const int* tvec;           // [B] timestep per sample (used when t_uniform < 0)
  int t_uniform;
  int B, cout;
  int n_t, n_tac;            // rows of tmap / cmap (buffer bounds of the epilogue map prefetch)
  FinalArgs fin;
};



// Launch helpers (unet_kernels.hip).  Return hipError_t.
// x3: the bf16x3 network (T = bf16 only; activations stored as [hi | lo] rows, see DmaPlan)
template <typename T>
hipError_t launch_conv(int layer_kind, const ConvArgs<T>& a, hipStream_t s, bool x3 = false);
template <typename T>
hipError_t launch_down0(const Down0Args& a, hipStream_t s, bool x3 = false);
hipError_t launch_split_to_f32(const bf16* src, size_t rows, int C, float* dst, hipStream_t s);

hipError_t launch_set_rng(unsigned long long* dst, unsigned long long seed, unsigned long long off, hipStream_t s);
template <typename T>
hipError_t launch_to_f32(const T* src, size_t n, float* dst, hipStream_t s);

hipError_t launch_time_emb(const float* w, const float* b, int T, int sin_dim, int hid, float* out,
                           hipStream_t s);
hipError_t launch_dense(const float* in, int rows, int din, const float* w, const float* b, int dout,
                        int act, float* out, hipStream_t s);
hipError_t launch_fold(const float* seq, int n, int Lseq, int Cs, const float* wk, int taps, int padl,
                       int ups, int cin_full, int ch0, const float* wr, const float* b1,
                       const float* b2, float* out, int Lout, int cout, hipStream_t s);
// fused up levels: composite taps [10][cbn][cout] and u-path maps through the block conv
hipError_t launch_compose(const float* wup, int cin_up, int xoff, int cbn, int cu, const float* kblk,
                          const float* kres, int cin_blk, int ch0, int cout, float* out, hipStream_t s);
hipError_t launch_map_through(const float* in, int n, int L, int cu, const float* kblk, const float* kres, int taps,
                              int padl, int cin_blk, int ch0, const float* b1, const float* b2, float* out, int cout,
                              hipStream_t s);
// out[i] = a[i] + b[i % per] (fp32), i < n: the combined time + label map table of a one-condition handle
hipError_t launch_add_rows(const float* a, const float* b, size_t per, size_t n, float* out, hipStream_t s);
hipError_t launch_philox_normal(unsigned long long seed, unsigned long long goff, int step, int B, float* out,
                                hipStream_t s);
hipError_t launch_posterior_stats(const float* x0, const int* tac, int B, int n_tac, int ncol,
                                  double* stats, hipStream_t s);

// Layer kinds of launch_conv (fixed shapes of the shipped config).
enum LayerKind : int {
  LK_DOWN1 = 0, LK_DOWN2, LK_DOWN3, LK_UP0_CONV2, LK_UP0_BLOCK, LK_UP1_CONV2, LK_UP1_BLOCK,
  LK_UP2_CONV2, LK_UP2_BLOCK, kNumConvLayers,
  // Fused up levels (16-bit path): UpSampling1D -> Conv1D(k2) -> concat -> ConvBlock as ONE
  // implicit GEMM.  The k2 conv is linear, so it composes with the block's k6 conv into a
  // 2-phase (even / odd output position) 4-tap conv on the coarse input; see DESIGN.md.
  LK_UP0_F = kNumConvLayers, LK_UP1_F, LK_UP2_F,
  // the final fused level of the bf16x3 network: paired [hi | lo] 64-B chunks on a 2-stage ring (the
  // 32-B rows of LK_UP2_F cannot hold a 16-channel pair; 3 stages of 64-B rows exceed the LDS)
  LK_UP2_FX3, kNumKinds
};
constexpr bool is_fused_kind(int kind) { return kind >= LK_UP0_F && kind < kNumKinds; }

// Per-layer tile configuration, shared by the kernels and the host weight packer.
//   wm x wn waves (wm*wn == 4): output tile (96*wm) rows x (64*wn) channels;
//   stages: LDS ring depth of the K loop; rowb: bytes of input channels per K chunk.
struct TileCfg {
  int wm, wn, stages, rowb;
};
// Co-residency experiment (scripts/micro/coresident.sh): down1 on a 2-stage ring of
// 32-B chunks, about 61 KB of LDS and 186 VGPRs, so two workgroups share a CU.  Product builds use 0.
#ifndef CONV_DOWN1_CORES
#define CONV_DOWN1_CORES 0
#endif
constexpr TileCfg layer_tile(int kind) {
  return CONV_DOWN1_CORES && kind == LK_DOWN1 ? TileCfg{4, 1, 2, 32}
         : kind == LK_UP2_BLOCK ? TileCfg{2, 2, 2, 64}                // final conv needs all 128 channels
         : kind == LK_UP2_F ? TileCfg{2, 2, 3, 32}                 // + 2-phase B tiles: 3 x 32-B chunks
         : kind == LK_UP2_FX3 ? TileCfg{2, 2, 2, 64}               // bf16x3: 2 x 64-B paired chunks
         : (kind == LK_UP0_CONV2 || kind == LK_UP1_CONV2 || kind == LK_UP2_CONV2) ? TileCfg{4, 1, 3, 128}
                                                                                  : TileCfg{4, 1, 3, 64};
}
constexpr int layer_ntile(int kind) { return 64 * layer_tile(kind).wn; }
// bf16x3 K chunks on the 64-B-row layers (down1, down2, down3, up0 / up1 fused, the unfused up blocks) are
// paired: a chunk holds 16 channels as [hi(16) | lo(16)] of both operands and runs the three products
// (a_hi, w_hi), (a_hi, w_lo), (a_lo, w_hi) on it, so each byte is staged once (2 x the bf16 chunks).  The
// 32-B-row final level walks three passes over the channels, (a_hi, w_hi) then (a_hi, w_lo) then
// (a_lo, w_hi), staging a_hi and w_hi twice (3 x the bf16 chunks).
// 16x16x32 MFMA K loops on the 16-bit down2, down3, up0.fused and up1.fused layers (unet_kernels.hip M16;
// 0: 32x32x16 everywhere).  Shared with the host: those layers' LDS rows and packed weight rows use the
// 16-row XOR key (piece_key).
#ifndef CONV_M16
#define CONV_M16 1
#endif
// bf16x3 on the 16x16x32 layers (down2, down3, up0.fused, up1.fused; unet_kernels.hip M16 / PX):
//   2: paired [hi | lo] chunks, two at a time -- units CX, HH, CY of full k = 32 MFMAs (conv_body PX), each
//      hi / lo byte staged once;
//   1: three passes (a_hi w_hi, a_hi w_lo, a_lo w_hi) of plain 64-B rows, a_hi and w_hi staged twice.
#ifndef CONV_M16_X3
#define CONV_M16_X3 2
#endif
static_assert(CONV_M16_X3 == 1 || CONV_M16_X3 == 2, "CONV_M16_X3: 1 three passes, 2 paired units");
constexpr bool m16_kind(int kind) { return kind == LK_DOWN2 || kind == LK_DOWN3 || kind == LK_UP0_F || kind == LK_UP1_F; }
constexpr bool x3_paired(int kind) { return layer_tile(kind).rowb == 64 && !(CONV_M16_X3 == 1 && m16_kind(kind)); }
// XOR key of 16-B piece index p within a row (an A row in LDS, a packed weight row n): conflict-free ds_read_b128
// for the lane groups of MI355X_MICROARCH.md's LDS table.  32x32x16 reads 16 rows of one piece per lane group:
// (row >> 2) & 3.  The 16x16x32 layers (m16: CONV_M16, 16-bit, m16_kind) read 16 rows x 4 pieces per
// instruction (lane l: row l & 15, piece l >> 4), whose lane groups {0-3, 12-15, 20-27} ... mix two pieces:
// 2 ((row >> 2) & 1) (the 32x32 key is 2-way there).
constexpr int piece_key(int row, int cpr, bool m16) {
  return (m16 && cpr == 4) ? 2 * ((row >> 2) & 1) : cpr == 4 ? ((row >> 2) & 3) : cpr == 2 ? ((row >> 3) & 1) : ((row >> 1) & 7);
}
template <typename T>
constexpr int layer_kc(int kind) { return layer_tile(kind).rowb / (int)sizeof(T); }

}  // namespace petdiff
