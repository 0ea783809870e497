// C-ABI implementation of libpetdiff.so (declared in include/petdiff.h).
//
// Host-side runtime of the sampler: weight packing into the MFMA layouts,
// per-level condition/time map folding, workspace management, the reverse
// loop (eager or captured once into a hipGraph and replayed), posterior
// statistics and per-layer event timing.
#include "petdiff.h"
#include "petdiff_internal.h"
#include "petdiff_spec.h"

#include <cmath>
#include <cstring>
#include <type_traits>
#include <cstdlib>
#include <map>
#include <memory>
#include <string>
#include <vector>

using namespace petdiff;

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

#define CHK(expr)                   \
  do {                              \
    int r_ = (expr);                \
    if (r_ != PETDIFF_OK) return r_; \
  } while (0)

uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

uint16_t f2h(float f) {   // IEEE binary16, round to nearest even (compiler conversion)
  const _Float16 h = (_Float16)f;
  uint16_t u;
  std::memcpy(&u, &h, 2);
  return u;
}


// geometry of the 7 condition-carrying levels (4 down blocks + 3 up-sampling convs)
struct CondLevel {
  const char* prefix;     // "down0" ...
  const char* conv;       // "conv" or "upconv"
  bool res;               // has a residual conv folded in
  int Lseq;               // length of the label/time sequence
  int Lout;               // output length of the conv
  int taps, padl, ups;
  int cin_full, cout;
};

const CondLevel kLevels[7] = {
    {"down0", "conv", true, 48, 48, 6, 2, 0, 52, 128},
    {"down1", "conv", true, 24, 24, 6, 2, 0, 178, 256},
    {"down2", "conv", true, 12, 12, 6, 2, 0, 306, 512},
    {"down3", "conv", true, 6, 6, 6, 2, 0, 562, 1024},
    {"up0", "upconv", false, 6, 12, 2, 0, 1, 1074, 512},
    {"up1", "upconv", false, 12, 24, 2, 0, 1, 562, 256},
    {"up2", "upconv", false, 24, 48, 2, 0, 1, 306, 128},
};

struct ConvLayer {
  int kind;
  const char* wname;       // weight prefix of the conv ("down1.conv", "up0.upconv", ...)
  const char* resname;     // residual kernel or nullptr
  int taps, padl;
  int cin_full, xoff, cin_x, cout;
  int cond_level;          // index into kLevels or -1 (bias only)
};

const ConvLayer kConv[kNumConvLayers] = {
    {LK_DOWN1, "down1.conv", "down1.res", 6, 2, 178, 50, 128, 256, 1},
    {LK_DOWN2, "down2.conv", "down2.res", 6, 2, 306, 50, 256, 512, 2},
    {LK_DOWN3, "down3.conv", "down3.res", 6, 2, 562, 50, 512, 1024, 3},
    {LK_UP0_CONV2, "up0.upconv", nullptr, 2, 0, 1074, 50, 1024, 512, 4},
    {LK_UP0_BLOCK, "up0.conv", "up0.res", 6, 2, 1024, 0, 1024, 512, -1},
    {LK_UP1_CONV2, "up1.upconv", nullptr, 2, 0, 562, 50, 512, 256, 5},
    {LK_UP1_BLOCK, "up1.conv", "up1.res", 6, 2, 512, 0, 512, 256, -1},
    {LK_UP2_CONV2, "up2.upconv", nullptr, 2, 0, 306, 50, 256, 128, 6},
    {LK_UP2_BLOCK, "up2.conv", "up2.res", 6, 2, 256, 0, 256, 128, -1},
};

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  ~DevBuf() { if (p) (void)hipFree(p); }
  hipError_t alloc(size_t b) {
    if (b <= bytes && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    hipError_t e = hipMalloc(&p, b ? b : 16);
    if (e == hipSuccess) bytes = b;
    return e;
  }
  template <typename T> T* as() const { return reinterpret_cast<T*>(p); }
};


struct GraphEntry {
  hipGraphExec_t exec = nullptr;
  hipGraph_t graph = nullptr;
};

}  // namespace

struct petdiff_ctx {
  petdiff_config cfg;
  int device = 0;
  int n_out = 4;
  std::vector<Spec> spec;
  std::map<std::string, size_t> off;
  DevBuf w32;                        // fp32 Keras blob on device
  DevBuf wpack[kNumConvLayers];      // packed conv weights (bf16 or f32)
  DevBuf w0;                         // down0 x weights [6][2][128] fp32 (res folded)
  DevBuf wf4;                        // final Conv1D kernel as [128][4] fp32, zero-padded (FinalArgs::wf4)
  DevBuf bias_only[kNumConvLayers];  // conv bias + res bias for up blocks
  DevBuf tmap[7], cmap[7];           // per cond level
  // fused up levels (16-bit path; PETDIFF_FUSE_UP=0 keeps the separate k2-conv launches)
  bool fuse_up = false;
  DevBuf wpack_f[3], epack_f[3];     // packed composite weights / left-edge correction weights
  DevBuf tmap_f[3], cmap_f[3];       // u-path maps through the block conv (+ block biases)
  // One condition (n_tac == 1): the time and label maps summed once per schedule / condition change,
  // cmb = tmap[t] + cmap[0] in fp32 (the sum every epilogue formed before adding the accumulators, so
  // the outputs are bitwise the same), passed as the non-final layers' tmap with cmap null: their
  // epilogues stage and read one map instead of two.  The fused final level reads it too (round 6: its
  // transposed epilogue stages the tile's rows in LDS, CONV_FIN_REGMAPS); down0 and the unfused final level
  // keep both tables.
  // PETDIFF_COMBINE_MAPS=0 keeps the two tables everywhere (A/B switch).
  bool combine_ok = true;
  bool use_cmb = false;
  DevBuf cmb[7], cmb_f[3];
  DevBuf tab;                        // [kNTab][T]
  DevBuf temb, tseq;                 // [T][48], scratch [T][L]
  int T = 0;
  bool sched_set = false;
  int n_tac = 0;
  DevBuf enc_a, enc_b;               // encoder scratch
  // workspace
  int B_cap = 0;
  int last_B = 0;                    // batch of the last forward / p_sample (petdiff_get_activation)
  DevBuf s0, p0, s1, p1, s2, p2, d3, u0, b0, u1, b1, u2;
  DevBuf s0b;                        // second s0 buffer (fused next-step down0 writes it)
  // run the next step's down0 inside the previous step's up2.block epilogue (generate);
  // PETDIFF_FUSE_DOWN0=0 restores the standalone down0 launch per step (A/B switch)
  bool fuse_down0 = true;
  DevBuf xa, xb, tacbuf, tbuf, rng;
  hipStream_t cap_stream = nullptr;
  int seg_steps = 0;                   // reverse steps per captured graph segment (0: the whole loop)
  std::map<std::vector<int>, GraphEntry> graphs;
  // timing
  bool timing = false;
  int timing_reps = 1;               // launches per timed layer call (back to back between the two events)
  std::vector<hipEvent_t> ev_pool;
  struct TimedCall { int layer, reps; hipEvent_t e0, e1; };
  std::vector<TimedCall> ev_used;
  size_t ev_next = 0;

  const float* W(const std::string& n) const { return w32.as<float>() + off.at(n); }
  // bf16x3 (PETDIFF_DTYPE_BF16X3): activations are [hi | lo] bf16 rows, 4 bytes per value
  bool x3 = false;
  size_t act_bytes() const { return (cfg.dtype == PETDIFF_DTYPE_F32 || x3) ? 4 : 2; }
};

namespace {


// K chunks of a packed weight tile in kernel order: (channel chunk, part) with part 0 = the value
// (bf16x3: its hi half) and 1 = its lo half.  bf16x3 walks every input segment of nc chunks three
// times -- (a_hi, w_hi), (a_hi, w_lo), (a_lo, w_hi) -- see DmaPlan in unet_kernels.hip.
// Paired bf16x3 (x3_paired(kind), petdiff_internal.h): part 2, the chunk index counts half chunks
// (KC / 2 channels) whose rows hold [hi | lo].
std::vector<std::pair<int, int>> chunk_order(int nc1, int nc2, bool x3, bool paired = false) {
  std::vector<std::pair<int, int>> o;
  for (int seg = 0; seg < 2; ++seg) {
    const int base = seg ? nc1 : 0, n = seg ? nc2 : nc1;
    if (x3 && paired) {
      for (int k = 0; k < 2 * n; ++k) o.push_back({2 * base + k, 2});
      continue;
    }
    for (int g = 0; g < (x3 ? 3 : 1); ++g)
      for (int k = 0; k < n; ++k) o.push_back({base + k, g == 1 ? 1 : 0});
  }
  return o;
}

// input channel and part (0 = the value / its hi half, 1 = its lo half) of element e of 16-B piece c
// (CPR pieces of EPC elements per row) of chunk ck
void chunk_elem(const std::pair<int, int>& ck, int KC, int CPR, int EPC, int c, int e, int& ch, int& part) {
  if (ck.second == 2) {
    const int hc = CPR / 2;
    ch = ck.first * (KC / 2) + (c % hc) * EPC + e;
    part = c >= hc;
  } else {
    ch = ck.first * KC + c * EPC + e;
    part = ck.second;
  }
}

float bf_hi(float v) { const uint32_t u = (uint32_t)f2bf(v) << 16; float f; std::memcpy(&f, &u, 4); return f; }
// part 1 of a bf16x3 weight: the bf16 of its residual after the hi half
float split_part(float v, int part) { return part ? v - bf_hi(v) : v; }

template <typename T, typename H>
int pack_conv(petdiff_ctx* h, const std::vector<float>& wk_host, int li) {
  const ConvLayer& cl = kConv[li];
  const int ROWB = layer_tile(cl.kind).rowb;
  const int KC = layer_kc<T>(cl.kind);
  const int NT = layer_ntile(cl.kind);
  const int CPR = ROWB / 16;
  const int EPC = 16 / (int)sizeof(T);
  const Spec* sk = nullptr;
  const Spec* sr = nullptr;
  for (auto& s : h->spec) {
    if (s.name == std::string(cl.wname) + ".kernel") sk = &s;
    if (cl.resname && s.name == std::string(cl.resname) + ".kernel") sr = &s;
  }
  if (!sk) return fail(PETDIFF_ERR_INVALID, "missing weight " + std::string(cl.wname));
  const float* wk = wk_host.data() + sk->off;
  const float* wr = sr ? wk_host.data() + sr->off : nullptr;
  if (cl.cin_x % KC != 0) return fail(PETDIFF_ERR_UNSUPPORTED, "channel count not a multiple of the K chunk");
  if (cl.cout % NT != 0) return fail(PETDIFF_ERR_UNSUPPORTED, "cout not a multiple of the N tile");
  const int NC = cl.cin_x / KC, nNT = cl.cout / NT;
  const bool m16 = CONV_M16 && sizeof(T) == 2 && m16_kind(cl.kind);   // = ConvGeom::M16G (piece_key)
  // the up blocks read [skip | u] from two inputs of cin_x / 2 channels each (run_network's lio)
  const bool two = cl.xoff == 0 && cl.cond_level < 0;
  const auto order = chunk_order(two ? NC / 2 : NC, two ? NC / 2 : 0, h->x3, x3_paired(cl.kind));
  // [n_tile][chunk][tap][n (NT)][CPR x 16-B pieces], piece index XOR-swizzled by n
  // exactly like ConvGeom::key (piece_key) so a linear LDS-DMA copy yields the swizzled image.
  std::vector<H> out((size_t)nNT * order.size() * cl.taps * NT * KC);
  size_t q = 0;
  for (int nt = 0; nt < nNT; ++nt)
    for (const auto& ck : order)
      for (int j = 0; j < cl.taps; ++j)
        for (int n = 0; n < NT; ++n)
          for (int p = 0; p < CPR; ++p) {
            const int c = p ^ piece_key(n, CPR, m16);
            for (int e = 0; e < EPC; ++e) {
              int ch, part;
              chunk_elem(ck, KC, CPR, EPC, c, e, ch, part);
              const int ci = cl.xoff + ch;
              const int co = nt * NT + n;
              float v = wk[((size_t)j * cl.cin_full + ci) * cl.cout + co];
              if (wr && j == cl.padl) v += wr[(size_t)ci * cl.cout + co];
              v = split_part(v, part);
              if constexpr (std::is_same<T, f16>::value) out[q++] = f2h(v);
              else if constexpr (sizeof(H) == 2) out[q++] = f2bf(v);
              else out[q++] = v;
            }
          }
  HIPC(h->wpack[li].alloc(out.size() * sizeof(H)));
  HIPC(hipMemcpy(h->wpack[li].p, out.data(), out.size() * sizeof(H), hipMemcpyHostToDevice));
  return PETDIFF_OK;
}

// Fused up level u (0..2): kinds, the k2 conv and the block it feeds (kConv indices).
struct FusedLevel {
  int kind, conv2_li, block_li, cond_level;
  int L, cs, cb, cout;   // output length, skip channels, coarse-input channels, output channels
};
const FusedLevel kFused[3] = {
    {LK_UP0_F, LK_UP0_CONV2, LK_UP0_BLOCK, 4, 12, 512, 1024, 512},
    {LK_UP1_F, LK_UP1_CONV2, LK_UP1_BLOCK, 5, 24, 256, 512, 256},
    {LK_UP2_F, LK_UP2_CONV2, LK_UP2_BLOCK, 6, 48, 128, 256, 128},
};

// kernel kind of fused level u (the bf16x3 network's final level runs its paired-chunk instance)
int fused_kind(const petdiff_ctx* h, int u) { return (u == 2 && h->x3) ? LK_UP2_FX3 : kFused[u].kind; }

// Weights of a fused up level: per N tile, the block's skip-half chunks [6 taps][NT][ROWB]
// (residual folded into tap 2) then the coarse-input chunks [phase][4 taps][NT][ROWB] of the
// composite taps (compose_kernel), both with the 16-B pieces XOR-swizzled by n; plus the
// left-edge correction weights [n_tile][chunk][phase][NT][KC] (plain).
template <typename T, typename H>
int pack_fused(petdiff_ctx* h, const std::vector<float>& host, int u) {
  FusedLevel fl = kFused[u];
  fl.kind = fused_kind(h, u);
  const ConvLayer& blk = kConv[fl.block_li];
  const ConvLayer& c2 = kConv[fl.conv2_li];
  const int ROWB = layer_tile(fl.kind).rowb, KC = layer_kc<T>(fl.kind), NT = layer_ntile(fl.kind);
  const int CPR = ROWB / 16, EPC = 16 / (int)sizeof(T);
  const int n1 = fl.cs / KC, n2 = fl.cb / KC, nNT = fl.cout / NT;
  const bool m16 = CONV_M16 && sizeof(T) == 2 && m16_kind(fl.kind);   // = ConvGeom::M16G (piece_key)
  if (fl.cs % KC || fl.cb % KC || fl.cout % NT || n1 < 3 || n2 < 2)
    return fail(PETDIFF_ERR_UNSUPPORTED, "fused up level geometry");
  // composite taps on the device (fp64 sums), then packed on the host
  DevBuf comp;
  HIPC(comp.alloc((size_t)10 * fl.cb * fl.cout * 4));
  HIPC(launch_compose(h->W(std::string(c2.wname) + ".kernel"), c2.cin_full, c2.xoff, fl.cb, c2.cout,
                      h->W(std::string(blk.wname) + ".kernel"), h->W(std::string(blk.resname) + ".kernel"),
                      blk.cin_full, fl.cs, fl.cout, comp.as<float>(), 0));
  std::vector<float> D((size_t)10 * fl.cb * fl.cout);
  HIPC(hipMemcpy(D.data(), comp.p, D.size() * 4, hipMemcpyDeviceToHost));
  const float* wk = host.data() + h->off.at(std::string(blk.wname) + ".kernel");
  const float* wr = host.data() + h->off.at(std::string(blk.resname) + ".kernel");
  auto cvt = [](float v) -> H {
    if constexpr (std::is_same<T, f16>::value) return f2h(v);
    else return f2bf(v);
  };
  const bool pr = x3_paired(fl.kind);
  const auto order1 = chunk_order(n1, 0, h->x3, pr), order2 = chunk_order(n2, 0, h->x3, pr);
  std::vector<H> out((size_t)nNT * (order1.size() * 6 + order2.size() * 8) * NT * KC);
  std::vector<H> eout((size_t)nNT * order2.size() * 2 * NT * KC);
  size_t q = 0, qe = 0;
  for (int nt = 0; nt < nNT; ++nt) {
    for (const auto& ck : order1)
      for (int j = 0; j < 6; ++j)
        for (int n = 0; n < NT; ++n)
          for (int p = 0; p < CPR; ++p) {
            const int c = p ^ piece_key(n, CPR, m16);
            for (int e = 0; e < EPC; ++e) {
              int ci, part;
              chunk_elem(ck, KC, CPR, EPC, c, e, ci, part);
              const int co = nt * NT + n;
              float v = wk[((size_t)j * blk.cin_full + ci) * blk.cout + co];
              if (j == blk.padl) v += wr[(size_t)ci * blk.cout + co];
              out[q++] = cvt(split_part(v, part));
            }
          }
    for (const auto& ck : order2) {
      for (int t = 0; t < 8; ++t)
        for (int n = 0; n < NT; ++n)
          for (int p = 0; p < CPR; ++p) {
            const int c = p ^ piece_key(n, CPR, m16);
            for (int e = 0; e < EPC; ++e) {
              int cb, part;
              chunk_elem(ck, KC, CPR, EPC, c, e, cb, part);
              const int co = nt * NT + n;
              out[q++] = cvt(split_part(D[((size_t)t * fl.cb + cb) * fl.cout + co], part));
            }
          }
      for (int ph = 0; ph < 2; ++ph)
        for (int n = 0; n < NT; ++n)
          for (int kk = 0; kk < KC; ++kk) {
            int cb, part;
            chunk_elem(ck, KC, CPR, EPC, kk / EPC, kk % EPC, cb, part);
            eout[qe++] = cvt(split_part(D[((size_t)(8 + ph) * fl.cb + cb) * fl.cout + nt * NT + n], part));
          }
    }
  }
  HIPC(h->wpack_f[u].alloc(out.size() * sizeof(H)));
  HIPC(hipMemcpy(h->wpack_f[u].p, out.data(), out.size() * sizeof(H), hipMemcpyHostToDevice));
  HIPC(h->epack_f[u].alloc(eout.size() * sizeof(H)));
  HIPC(hipMemcpy(h->epack_f[u].p, eout.data(), eout.size() * sizeof(H), hipMemcpyHostToDevice));
  return PETDIFF_OK;
}

// u-path maps of fused level u through its block conv: from the k2 conv's time (+ biases) or
// label map [n][L][cu] to [n][L][cout] (time: + the block's conv and residual biases)
int fused_maps(petdiff_ctx* h, int u, bool time, int n, hipStream_t s) {
  const FusedLevel& fl = kFused[u];
  const ConvLayer& blk = kConv[fl.block_li];
  DevBuf& dst = time ? h->tmap_f[u] : h->cmap_f[u];
  HIPC(dst.alloc((size_t)n * fl.L * fl.cout * 4));
  const DevBuf& src = time ? h->tmap[fl.cond_level] : h->cmap[fl.cond_level];
  HIPC(launch_map_through(src.as<float>(), n, fl.L, fl.cout, h->W(std::string(blk.wname) + ".kernel"),
                          h->W(std::string(blk.resname) + ".kernel"), blk.taps, blk.padl, blk.cin_full, fl.cs,
                          time ? h->W(std::string(blk.wname) + ".bias") : nullptr,
                          time ? h->W(std::string(blk.resname) + ".bias") : nullptr, dst.as<float>(), fl.cout, s));
  return PETDIFF_OK;
}

// destroy every captured graph (they hold the addresses of the tables and the workspace)
void clear_graphs(petdiff_ctx* h) {
  for (auto& kv : h->graphs) {
    if (kv.second.exec) (void)hipGraphExecDestroy(kv.second.exec);
    if (kv.second.graph) (void)hipGraphDestroy(kv.second.graph);
  }
  h->graphs.clear();
}

// the combined tables of a one-condition handle (see petdiff_ctx::cmb); called whenever the schedule or the
// conditions change.  A reallocated table invalidates the captured graphs (they hold its address).
int combine_maps(petdiff_ctx* h, hipStream_t s) {
  h->use_cmb = false;
  if (!h->combine_ok || !h->sched_set || h->n_tac != 1) return PETDIFF_OK;
  const int nlv = h->fuse_up ? 4 : 7;
  auto need = [&](int lv) { return (size_t)h->T * kLevels[lv].Lout * kLevels[lv].cout * 4; };
  auto need_f = [&](int u) { return (size_t)h->T * kFused[u].L * kFused[u].cout * 4; };
  // a table that has to grow is freed and reallocated, so the graphs that hold its address go first (also
  // when an allocation or launch below fails: no graph survives that could replay a freed table)
  bool grow = false;
  for (int lv = 1; lv < nlv; ++lv) grow = grow || h->cmb[lv].bytes < need(lv) || !h->cmb[lv].p;
  if (h->fuse_up)
    for (int u = 0; u < 3; ++u) grow = grow || h->cmb_f[u].bytes < need_f(u) || !h->cmb_f[u].p;
  if (grow) clear_graphs(h);
  auto one = [&](DevBuf& dst, const DevBuf& tm, const DevBuf& cm, size_t bytes) -> hipError_t {
    hipError_t e = dst.alloc(bytes);
    if (e != hipSuccess) return e;
    return launch_add_rows(tm.as<float>(), cm.as<float>(), bytes / 4 / h->T, bytes / 4, dst.as<float>(), s);
  };
  // the non-final layers' tables and the fused final level's (down0 and the unfused final level keep two)
  // (the fused path's up levels read cmb_f; their k2-conv levels 4-6 then run no layer)
  hipError_t e = hipSuccess;
  for (int lv = 1; lv < nlv && e == hipSuccess; ++lv) e = one(h->cmb[lv], h->tmap[lv], h->cmap[lv], need(lv));
  if (h->fuse_up)
    for (int u = 0; u < 3 && e == hipSuccess; ++u) e = one(h->cmb_f[u], h->tmap_f[u], h->cmap_f[u], need_f(u));
  if (e != hipSuccess) clear_graphs(h);   // the tables are partly rewritten: no captured graph may replay them
  HIPC(e);
  h->use_cmb = true;
  return PETDIFF_OK;
}

int ensure_workspace(petdiff_ctx* h, int B) {
  if (B > PETDIFF_MAX_BATCH) return fail(PETDIFF_ERR_INVALID, "batch exceeds PETDIFF_MAX_BATCH (65536); split it into chunks");
  if (B <= h->B_cap) return PETDIFF_OK;
  const size_t e = h->act_bytes();
  const size_t Bz = (size_t)B;
  HIPC(h->s0.alloc(Bz * 48 * 128 * e));
  HIPC(h->s0b.alloc(Bz * 48 * 128 * e));
  HIPC(h->p0.alloc(Bz * 24 * 128 * e));
  HIPC(h->s1.alloc(Bz * 24 * 256 * e));
  HIPC(h->p1.alloc(Bz * 12 * 256 * e));
  HIPC(h->s2.alloc(Bz * 12 * 512 * e));
  HIPC(h->p2.alloc(Bz * 6 * 512 * e));
  HIPC(h->d3.alloc(Bz * 6 * 1024 * e));
  HIPC(h->u0.alloc(Bz * 12 * 512 * e));
  HIPC(h->b0.alloc(Bz * 12 * 512 * e));
  HIPC(h->u1.alloc(Bz * 24 * 256 * e));
  HIPC(h->b1.alloc(Bz * 24 * 256 * e));
  HIPC(h->u2.alloc(Bz * 48 * 128 * e));
  HIPC(h->xa.alloc(Bz * 96 * 4));
  HIPC(h->xb.alloc(Bz * 96 * 4));
  HIPC(h->tacbuf.alloc(Bz * 4));
  HIPC(h->tbuf.alloc(Bz * 4));
  HIPC(h->rng.alloc(16));
  // workspace moved: cached graphs hold stale pointers
  clear_graphs(h);
  h->B_cap = B;
  h->last_B = 0;   // the level buffers are new: nothing to read back until a forward / p_sample runs
  return PETDIFF_OK;
}

hipEvent_t next_event(petdiff_ctx* h) {
  if (h->ev_next >= h->ev_pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    h->ev_pool.push_back(e);
  }
  return h->ev_pool[h->ev_next++];
}

struct StepIO {
  const float* x_in;
  int t_uniform;              // >= 0: all samples use this t
  const int* tvec;            // else per-sample t (device)
  const int* tac;             // device or null
  FinalArgs fin;
  int s0_sel;                 // skip buffer of this step: 0 -> s0, 1 -> s0b
  bool skip_down0;            // s0/p0 already written by the previous step's fused epilogue
  bool fuse_next;             // up2.block epilogue also runs down0 of the next step (t = next_t)
  int next_t;
};

template <typename T>
int run_network(petdiff_ctx* h, const StepIO& io, int B, hipStream_t s) {
  // layer 0: down0 on VALU
  auto timed = [&](int layer, auto&& fn) -> int {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (h->timing) {
      e0 = next_event(h);
      e1 = next_event(h);
      if (e0) (void)hipEventRecord(e0, s);
    }
    // timing_reps > 1: the launch is repeated back to back (every layer kernel is idempotent: it reads
    // its inputs and writes other buffers), so the event pair brackets reps launches and one queue gap
    const int reps = h->timing ? h->timing_reps : 1;
    for (int r = 0; r < reps; ++r) {
      hipError_t e = fn();
      if (e != hipSuccess) return fail(PETDIFF_ERR_HIP, std::string("kernel launch failed: ") + hipGetErrorString(e));
    }
    if (h->timing && e0 && e1) {
      (void)hipEventRecord(e1, s);
      h->ev_used.push_back({layer, reps, e0, e1});
    }
    return PETDIFF_OK;
  };
  void* s0 = io.s0_sel ? h->s0b.p : h->s0.p;
  void* s0_other = io.s0_sel ? h->s0.p : h->s0b.p;
  void* p0 = h->p0.p;
  void* s1 = h->s1.p;
  void* p1 = h->p1.p;
  void* s2 = h->s2.p;
  void* p2 = h->p2.p;
  void* d3 = h->d3.p;
  void* u0 = h->u0.p;
  void* b0 = h->b0.p;
  void* u1 = h->u1.p;
  void* b1 = h->b1.p;
  void* u2 = h->u2.p;
  Down0Args d0{};
  d0.x = io.x_in;
  d0.w0 = h->w0.as<float>();
  d0.cmap = h->cmap[0].as<float>();
  d0.tmap = h->tmap[0].as<float>();
  d0.tac = io.tac;
  d0.tvec = io.tvec;
  d0.t_uniform = io.t_uniform;
  d0.s0 = s0;
  d0.p0 = p0;
  d0.B = B;
  if (!io.skip_down0) CHK(timed(0, [&] { return launch_down0<T>(d0, s, h->x3); }));

  struct LIO { const void* s1; int c1; const void* s2; int c2; void* out; void* pool; };
  const LIO lio[kNumConvLayers] = {
      {p0, 128, nullptr, 0, s1, p1},
      {p1, 256, nullptr, 0, s2, p2},
      {p2, 512, nullptr, 0, d3, nullptr},
      {d3, 1024, nullptr, 0, u0, nullptr},
      {s2, 512, u0, 512, b0, nullptr},
      {b0, 512, nullptr, 0, u1, nullptr},
      {s1, 256, u1, 256, b1, nullptr},
      {b1, 256, nullptr, 0, u2, nullptr},
      {s0, 128, u2, 128, nullptr, nullptr},
  };
  // fused up levels replace (k2 conv, block) pairs: {kind, timing id, src1, c1, src2, c2, out}
  const bool fused = sizeof(T) == 2 && h->fuse_up;
  for (int li = 0; li < kNumConvLayers; ++li) {
    const ConvLayer& cl = kConv[li];
    if (fused && li >= LK_UP0_CONV2) {
      if (li == LK_UP0_CONV2 || li == LK_UP1_CONV2 || li == LK_UP2_CONV2) continue;
      const int u = (li - LK_UP0_BLOCK) / 2;
      const FusedLevel& fl = kFused[u];
      ConvArgs<T> a{};
      a.src1 = reinterpret_cast<const T*>(lio[li].s1);                 // the skip
      a.c1 = fl.cs;
      a.src2 = reinterpret_cast<const T*>(lio[fl.conv2_li].s1);        // the k2 conv's input
      a.c2 = fl.cb;
      a.wpack = h->wpack_f[u].as<T>();
      a.epack = h->epack_f[u].as<T>();
      a.out = reinterpret_cast<T*>(lio[li].out);
      // (the final level reads the combined table too: its transposed epilogue stages the tile's rows in LDS
      // during the K loop, CONV_FIN_REGMAPS; its fused next-step down0 keeps level 0's two tables)
      const bool cmb = h->use_cmb;
      a.tmap = (cmb ? h->cmb_f[u] : h->tmap_f[u]).as<float>();
      a.cmap = cmb ? nullptr : h->cmap_f[u].as<float>();
      a.tac = io.tac;
      a.tvec = io.tvec;
      a.t_uniform = io.t_uniform;
      a.n_t = h->T;
      a.n_tac = h->n_tac;
      a.B = B;
      a.cout = fl.cout;
      if (li == kNumConvLayers - 1) {
        a.fin = io.fin;
        a.fin.next = Down0Args{};
        a.fin.next.t_uniform = -1;
        if (io.fuse_next) {
          a.fin.next = d0;
          a.fin.next.x = nullptr;
          a.fin.next.tvec = nullptr;
          a.fin.next.t_uniform = io.next_t;
          a.fin.next.s0 = s0_other;
        }
      }
      CHK(timed(1 + li, [&] { return launch_conv<T>(fused_kind(h, u), a, s, h->x3); }));
      continue;
    }
    ConvArgs<T> a{};
    a.src1 = reinterpret_cast<const T*>(lio[li].s1);
    a.c1 = lio[li].c1;
    a.src2 = reinterpret_cast<const T*>(lio[li].s2);
    a.c2 = lio[li].c2;
    a.wpack = h->wpack[li].as<T>();
    a.out = reinterpret_cast<T*>(lio[li].out);
    a.out_pool = reinterpret_cast<T*>(lio[li].pool);
    if (cl.cond_level >= 0) {
      const bool cmb = h->use_cmb && li != kNumConvLayers - 1;
      a.cmap = cmb ? nullptr : h->cmap[cl.cond_level].as<float>();
      a.tmap = (cmb ? h->cmb[cl.cond_level] : h->tmap[cl.cond_level]).as<float>();
    } else {
      a.bias = h->bias_only[li].as<float>();
    }
    a.tac = io.tac;
    a.tvec = io.tvec;
    a.t_uniform = io.t_uniform;
    a.n_t = h->T;
    a.n_tac = h->n_tac;
    a.B = B;
    a.cout = cl.cout;
    if (li == kNumConvLayers - 1) {
      a.fin = io.fin;
      a.fin.next = Down0Args{};
      a.fin.next.t_uniform = -1;
      if (io.fuse_next) {
        // p0 is free again (down1 of this step has read it); s0 goes to the other buffer
        // because this very kernel still reads the current one.
        a.fin.next = d0;
        a.fin.next.x = nullptr;
        a.fin.next.tvec = nullptr;
        a.fin.next.t_uniform = io.next_t;
        a.fin.next.s0 = s0_other;
      }
    }
    CHK(timed(1 + li, [&] { return launch_conv<T>(cl.kind, a, s, h->x3); }));
  }
  return PETDIFF_OK;
}

int network(petdiff_ctx* h, const StepIO& io, int B, hipStream_t s) {
  if (!h->sched_set) return fail(PETDIFF_ERR_INVALID, "schedule not set (petdiff_set_schedule)");
  if (h->n_tac <= 0) return fail(PETDIFF_ERR_INVALID, "conditions not set (petdiff_set_conditions)");
  if (h->cfg.dtype == PETDIFF_DTYPE_BF16 || h->x3) return run_network<bf16>(h, io, B, s);
  if (h->cfg.dtype == PETDIFF_DTYPE_F16) return run_network<f16>(h, io, B, s);
  return run_network<float>(h, io, B, s);
}

FinalArgs base_final(petdiff_ctx* h) {
  FinalArgs f{};
  f.wf = h->W("final.kernel");
  f.wf4 = h->wf4.as<float>();
  f.bf = h->W("final.bias");
  f.n_out = h->n_out;
  f.tab = h->tab.as<float>();
  f.T = h->T;
  f.learn_mode = h->cfg.learn_variance;
  f.param_mode = h->cfg.parameterization;
  f.rng = h->rng.as<unsigned long long>();
  return f;
}

int valid_handle(petdiff_handle h) {
  if (!h) return fail(PETDIFF_ERR_INVALID, "null handle");
  HIPC(hipSetDevice(h->device));
  return PETDIFF_OK;
}

}  // namespace

extern "C" {

const char* petdiff_last_error(void) { return g_err.c_str(); }

int petdiff_default_config(petdiff_config* c) {
  if (!c) return fail(PETDIFF_ERR_INVALID, "null config");
  c->n_roi = 48;
  c->n_par = 2;
  c->n_frames = 54;
  c->n_cond_rows = 49;
  c->num_filt_start = 128;
  c->depth = 4;
  c->kernel_size = 6;
  c->pool_size = 2;
  c->sin_emb_dim = 64;
  c->enc_size[0] = 256;
  c->enc_size[1] = 128;
  c->enc_size[2] = 64;
  c->latent_dim = 32;
  c->timesteps = 1000;
  c->learn_variance = PETDIFF_LEARN_RANGED;
  c->parameterization = PETDIFF_PARAM_EPS;
  c->dtype = PETDIFF_DTYPE_BF16;
  return PETDIFF_OK;
}

size_t petdiff_param_count(const petdiff_config* c) {
  if (!c) return 0;
  const int n_out = c->learn_variance == PETDIFF_LEARN_FIXED ? c->n_par : 2 * c->n_par;
  const auto s = make_spec(*c, n_out);
  return s.back().off + s.back().size;
}

int petdiff_cosine_schedule(int T, double offset_s, double max_beta, float* beta_out) {
  if (T <= 0 || !beta_out) return fail(PETDIFF_ERR_INVALID, "bad arguments");
  const double pi = 3.141592653589793;
  for (int i = 0; i < T; ++i) {
    const double t1 = (double)i / T, t2 = (double)(i + 1) / T;
    const float a1 = cosf((float)((t1 + offset_s) / (1 + offset_s) * pi / 2));
    const float a2 = cosf((float)((t2 + offset_s) / (1 + offset_s) * pi / 2));
    const float ab1 = a1 * a1, ab2 = a2 * a2;
    const float b = 1.0f - ab2 / ab1;
    beta_out[i] = (double)b < max_beta ? b : (float)max_beta;
  }
  return PETDIFF_OK;
}

int petdiff_create(const petdiff_config* cfg, const float* weights, size_t n_weights, int device,
                   petdiff_handle* out) {
  if (!cfg || !weights || !out) return fail(PETDIFF_ERR_INVALID, "null argument");
  if (!is_shipped_arch(*cfg))
    return fail(PETDIFF_ERR_UNSUPPORTED,
                "only the shipped UnetConditional (f128/d4, k6, L48, enc 256-128-64-32) is compiled");
  if (cfg->dtype != PETDIFF_DTYPE_F32 && cfg->dtype != PETDIFF_DTYPE_BF16 && cfg->dtype != PETDIFF_DTYPE_F16 &&
      cfg->dtype != PETDIFF_DTYPE_BF16X3)
    return fail(PETDIFF_ERR_INVALID,
                "dtype must be PETDIFF_DTYPE_F32, PETDIFF_DTYPE_BF16, PETDIFF_DTYPE_F16 or PETDIFF_DTYPE_BF16X3");
  if (cfg->learn_variance < 0 || cfg->learn_variance > 2 || cfg->parameterization < 0 ||
      cfg->parameterization > 3)
    return fail(PETDIFF_ERR_INVALID, "bad learn_variance / parameterization");
  std::unique_ptr<petdiff_ctx> h(new petdiff_ctx());
  h->cfg = *cfg;
  h->device = device;
  h->n_out = cfg->learn_variance == PETDIFF_LEARN_FIXED ? cfg->n_par : 2 * cfg->n_par;
  h->x3 = cfg->dtype == PETDIFF_DTYPE_BF16X3;
  h->spec = make_spec(*cfg, h->n_out);
  if (const char* e = std::getenv("PETDIFF_FUSE_DOWN0")) h->fuse_down0 = std::atoi(e) != 0;
  h->fuse_up = cfg->dtype != PETDIFF_DTYPE_F32;
  if (const char* e = std::getenv("PETDIFF_FUSE_UP")) h->fuse_up = h->fuse_up && std::atoi(e) != 0;
  const size_t need = h->spec.back().off + h->spec.back().size;
  if (n_weights != need)
    return fail(PETDIFF_ERR_INVALID, "weight blob has " + std::to_string(n_weights) + " values, expected " +
                                         std::to_string(need));
  for (auto& s : h->spec) h->off[s.name] = s.off;
  HIPC(hipSetDevice(device));
  HIPC(hipStreamCreateWithFlags(&h->cap_stream, hipStreamNonBlocking));
  if (const char* e = std::getenv("PETDIFF_GRAPH_SEG")) h->seg_steps = std::max(0, std::atoi(e));
  if (const char* e = std::getenv("PETDIFF_COMBINE_MAPS")) h->combine_ok = std::atoi(e) != 0;
  HIPC(h->w32.alloc(need * 4));
  HIPC(hipMemcpy(h->w32.p, weights, need * 4, hipMemcpyHostToDevice));
  std::vector<float> host(weights, weights + need);
  for (int li = 0; li < kNumConvLayers; ++li) {
    if (cfg->dtype == PETDIFF_DTYPE_BF16 || h->x3) CHK((pack_conv<bf16, uint16_t>(h.get(), host, li)));
    else if (cfg->dtype == PETDIFF_DTYPE_F16) CHK((pack_conv<f16, uint16_t>(h.get(), host, li)));
    else CHK((pack_conv<float, float>(h.get(), host, li)));
    const ConvLayer& cl = kConv[li];
    if (cl.cond_level < 0) {
      std::vector<float> b(cl.cout);
      const float* bc = host.data() + h->off.at(std::string(cl.wname) + ".bias");
      const float* br = host.data() + h->off.at(std::string(cl.resname) + ".bias");
      for (int n = 0; n < cl.cout; ++n) b[n] = bc[n] + br[n];
      HIPC(h->bias_only[li].alloc(cl.cout * 4));
      HIPC(hipMemcpy(h->bias_only[li].p, b.data(), cl.cout * 4, hipMemcpyHostToDevice));
    }
  }
  if (h->fuse_up)
    for (int u = 0; u < 3; ++u) {
      if (cfg->dtype == PETDIFF_DTYPE_BF16 || h->x3) CHK((pack_fused<bf16, uint16_t>(h.get(), host, u)));
      else CHK((pack_fused<f16, uint16_t>(h.get(), host, u)));
    }
  // down0: x channels 50, 51 of down0.conv (6, 52, 128) with the res kernel folded into tap 2
  {
    std::vector<float> w0(6 * 2 * 128);
    const float* wk = host.data() + h->off.at("down0.conv.kernel");
    const float* wr = host.data() + h->off.at("down0.res.kernel");
    for (int j = 0; j < 6; ++j)
      for (int c = 0; c < 2; ++c)
        for (int n = 0; n < 128; ++n) {
          float v = wk[((size_t)j * 52 + 50 + c) * 128 + n];
          if (j == 2) v += wr[(size_t)(50 + c) * 128 + n];
          w0[(j * 2 + c) * 128 + n] = v;
        }
    HIPC(h->w0.alloc(w0.size() * 4));
    HIPC(hipMemcpy(h->w0.p, w0.data(), w0.size() * 4, hipMemcpyHostToDevice));
  }
  {
    std::vector<float> wf4(128 * 4, 0.f);
    const float* wf = host.data() + h->off.at("final.kernel");
    for (int n = 0; n < 128; ++n)
      for (int o = 0; o < h->n_out; ++o) wf4[n * 4 + o] = wf[n * h->n_out + o];
    HIPC(h->wf4.alloc(wf4.size() * 4));
    HIPC(hipMemcpy(h->wf4.p, wf4.data(), wf4.size() * 4, hipMemcpyHostToDevice));
  }
  *out = h.release();
  return PETDIFF_OK;
}

int petdiff_destroy(petdiff_handle h) {
  if (!h) return PETDIFF_OK;
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();
  for (auto& kv : h->graphs) {
    if (kv.second.exec) (void)hipGraphExecDestroy(kv.second.exec);
    if (kv.second.graph) (void)hipGraphDestroy(kv.second.graph);
  }
  for (auto e : h->ev_pool) (void)hipEventDestroy(e);
  if (h->cap_stream) (void)hipStreamDestroy(h->cap_stream);
  delete h;
  return PETDIFF_OK;
}

int petdiff_set_schedule(petdiff_handle h, const float* tables, int T) {
  CHK(valid_handle(h));
  if (!tables || T <= 0) return fail(PETDIFF_ERR_INVALID, "bad schedule tables");
  // tab, tmap and tmap_f may be reallocated and are rewritten: no captured graph may keep replaying them
  clear_graphs(h);
  h->use_cmb = false;
  HIPC(h->tab.alloc((size_t)kNTab * T * 4));
  HIPC(hipMemcpy(h->tab.p, tables, (size_t)kNTab * T * 4, hipMemcpyHostToDevice));
  h->T = T;
  // time path: SinusoidalPosEmb -> Dense(48) -> GELU for every t, then each
  // level's Dense(L) and its folded conv contribution (+ the conv biases).
  HIPC(h->temb.alloc((size_t)T * h->cfg.n_roi * 4));
  HIPC(h->tseq.alloc((size_t)T * 48 * 4));
  HIPC(launch_time_emb(h->W("time_mlp.kernel"), h->W("time_mlp.bias"), T, h->cfg.sin_emb_dim, h->cfg.n_roi,
                       h->temb.as<float>(), 0));
  for (int lv = 0; lv < 7; ++lv) {
    const CondLevel& c = kLevels[lv];
    const std::string p = c.prefix;
    HIPC(launch_dense(h->temb.as<float>(), T, h->cfg.n_roi, h->W(p + ".time_proj.kernel"),
                      h->W(p + ".time_proj.bias"), c.Lseq, 0, h->tseq.as<float>(), 0));
    HIPC(h->tmap[lv].alloc((size_t)T * c.Lout * c.cout * 4));
    const std::string cv = p + "." + c.conv;
    HIPC(launch_fold(h->tseq.as<float>(), T, c.Lseq, 1, h->W(cv + ".kernel"), c.taps, c.padl, c.ups, c.cin_full,
                     h->cfg.n_cond_rows, c.res ? h->W(p + ".res.kernel") : nullptr, h->W(cv + ".bias"),
                     c.res ? h->W(p + ".res.bias") : nullptr, h->tmap[lv].as<float>(), c.Lout, c.cout, 0));
  }
  if (h->fuse_up)
    for (int u = 0; u < 3; ++u) CHK(fused_maps(h, u, true, T, 0));
  HIPC(hipDeviceSynchronize());
  h->sched_set = true;
  CHK(combine_maps(h, 0));
  HIPC(hipDeviceSynchronize());
  return PETDIFF_OK;
}

int petdiff_set_conditions(petdiff_handle h, const float* cond, int n_tac, void* stream) {
  CHK(valid_handle(h));
  if (!cond || n_tac <= 0) return fail(PETDIFF_ERR_INVALID, "bad conditions");
  hipStream_t s = (hipStream_t)stream;
  const int rows = n_tac * h->cfg.n_cond_rows;
  // a new TAC count reallocates cmap / cmap_f (and changes which map tables the layers read): the
  // captured graphs go before any table moves
  if (n_tac != h->n_tac) {
    clear_graphs(h);
    h->use_cmb = false;
  }
  HIPC(h->enc_a.alloc((size_t)rows * 256 * 4));
  HIPC(h->enc_b.alloc((size_t)rows * 256 * 4));
  float* A = h->enc_a.as<float>();
  float* Bf = h->enc_b.as<float>();
  // Encoder_v3_noskip (networks.py:574-586): 54-256-128-64 relu, -> 32 linear
  HIPC(launch_dense(cond, rows, 54, h->W("cond_enc.hidden0.kernel"), h->W("cond_enc.hidden0.bias"), 256, 1, A, s));
  HIPC(launch_dense(A, rows, 256, h->W("cond_enc.hidden1.kernel"), h->W("cond_enc.hidden1.bias"), 128, 1, Bf, s));
  HIPC(launch_dense(Bf, rows, 128, h->W("cond_enc.hidden2.kernel"), h->W("cond_enc.hidden2.bias"), 64, 1, A, s));
  HIPC(launch_dense(A, rows, 64, h->W("cond_enc.z.kernel"), h->W("cond_enc.z.bias"), 32, 0, Bf, s));
  for (int lv = 0; lv < 7; ++lv) {
    const CondLevel& c = kLevels[lv];
    const std::string p = c.prefix;
    // label projection Dense(L) on (n_tac*49, 32) -> flat (n_tac, 49*L) == raw Reshape((L, 49))
    HIPC(launch_dense(Bf, rows, 32, h->W(p + ".label_proj.kernel"), h->W(p + ".label_proj.bias"), c.Lseq, 0, A, s));
    HIPC(h->cmap[lv].alloc((size_t)n_tac * c.Lout * c.cout * 4));
    const std::string cv = p + "." + c.conv;
    HIPC(launch_fold(A, n_tac, c.Lseq, h->cfg.n_cond_rows, h->W(cv + ".kernel"), c.taps, c.padl, c.ups,
                     c.cin_full, 0, c.res ? h->W(p + ".res.kernel") : nullptr, nullptr, nullptr,
                     h->cmap[lv].as<float>(), c.Lout, c.cout, s));
  }
  if (h->fuse_up)
    for (int u = 0; u < 3; ++u) CHK(fused_maps(h, u, false, n_tac, s));
  h->n_tac = n_tac;
  CHK(combine_maps(h, s));
  return PETDIFF_OK;
}

int petdiff_forward(petdiff_handle h, const float* x, const int32_t* t, const int32_t* tac, float* out, int B,
                    void* stream) {
  CHK(valid_handle(h));
  if (B < 0 || (B > 0 && (!x || !t || !out))) return fail(PETDIFF_ERR_INVALID, "bad arguments");
  if (B == 0) return PETDIFF_OK;
  CHK(ensure_workspace(h, B));
  StepIO io{};
  io.x_in = x;
  io.t_uniform = -1;
  io.tvec = t;
  io.tac = tac;
  io.fin = base_final(h);
  io.fin.x_t = x;
  io.fin.net_out = out;
  CHK(network(h, io, B, (hipStream_t)stream));
  h->last_B = B;
  return PETDIFF_OK;
}

int petdiff_p_sample(petdiff_handle h, const float* x, const int32_t* t, const int32_t* tac, const float* z,
                     uint64_t seed, uint64_t sample_offset, int rng_step, float* mean, float* var,
                     float* var_tilde, int B, void* stream) {
  CHK(valid_handle(h));
  if (B < 0 || (B > 0 && (!x || !t))) return fail(PETDIFF_ERR_INVALID, "bad arguments");
  if (B == 0) return PETDIFF_OK;
  CHK(ensure_workspace(h, B));
  hipStream_t s = (hipStream_t)stream;
  HIPC(launch_set_rng(h->rng.as<unsigned long long>(), seed, sample_offset, s));
  StepIO io{};
  io.x_in = x;
  io.t_uniform = -1;
  io.tvec = t;
  io.tac = tac;
  io.fin = base_final(h);
  io.fin.x_t = x;
  io.fin.z = z;
  io.fin.rng_step = rng_step;
  io.fin.mean_out = mean;
  io.fin.var_out = var;
  io.fin.var_tilde_out = var_tilde;
  CHK(network(h, io, B, s));
  h->last_B = B;
  return PETDIFF_OK;
}

int petdiff_generate(petdiff_handle h, const float* x_T, const int32_t* tac, const int32_t* t_seq, int n_steps,
                     int flag_var_tilde, const float* z_all, uint64_t seed, uint64_t sample_offset, float* x_out,
                     float* all_xt, int B, int use_graph, void* stream) {
  CHK(valid_handle(h));
  if (B < 0 || n_steps < 0 || (B > 0 && (!x_T || !x_out)) || (n_steps > 0 && !t_seq))
    return fail(PETDIFF_ERR_INVALID, "bad arguments");
  if (B == 0) return PETDIFF_OK;
  for (int i = 0; i < n_steps; ++i)
    if (t_seq[i] < 0 || t_seq[i] >= h->T) return fail(PETDIFF_ERR_INVALID, "timestep index out of range");
  CHK(ensure_workspace(h, B));
  // the loop overwrites the level buffers (with the fused down0, s0 / p0 end up holding the next step's
  // data): petdiff_get_activation fails until a forward / p_sample runs again
  h->last_B = 0;
  hipStream_t s = (hipStream_t)stream;
  const size_t xbytes = (size_t)B * h->cfg.n_roi * h->cfg.n_par * 4;
  const bool graph = use_graph && !z_all && !all_xt && !h->timing && n_steps > 0;
  HIPC(launch_set_rng(h->rng.as<unsigned long long>(), seed, sample_offset, s));
  HIPC(hipMemcpyAsync(h->xa.p, x_T, xbytes, hipMemcpyDeviceToDevice, s));
  const int* tacp = nullptr;
  if (tac) {
    HIPC(hipMemcpyAsync(h->tacbuf.p, tac, (size_t)B * 4, hipMemcpyDeviceToDevice, s));
    tacp = h->tacbuf.as<int>();
  }
  float* bufs[2] = {h->xa.as<float>(), h->xb.as<float>()};
  auto enqueue = [&](hipStream_t q, int i0, int i1) -> int {
    for (int i = i0; i < i1; ++i) {
      StepIO io{};
      io.x_in = bufs[i & 1];
      io.t_uniform = t_seq[i];
      io.tvec = nullptr;
      io.tac = tacp;
      io.fin = base_final(h);
      io.fin.x_t = io.x_in;
      io.fin.z = z_all ? z_all + (size_t)i * B * 96 : nullptr;
      io.fin.rng_step = i;
      io.fin.flag_var_tilde = flag_var_tilde;
      io.fin.x_next = bufs[(i + 1) & 1];
      io.fin.x_all = all_xt ? all_xt + (size_t)i * B * 96 : nullptr;
      if (h->fuse_down0) {
        io.s0_sel = i & 1;
        io.skip_down0 = i > 0;
        io.fuse_next = i + 1 < n_steps;
        io.next_t = io.fuse_next ? t_seq[i + 1] : -1;
      }
      CHK(network(h, io, B, q));
    }
    return PETDIFF_OK;
  };
  if (!graph) {
    CHK(enqueue(s, 0, n_steps));
  } else {
    // The loop is captured as graph segments of seg_steps reverse steps (default: the whole loop in one):
    // hipGraphLaunch enqueues a graph's kernel nodes on the host, so a 5000-node graph costs milliseconds
    // of host time before its first kernel runs; with segments only the first one's enqueue is exposed,
    // the others are enqueued while the GPU runs the earlier ones.
    const int seg = h->seg_steps > 0 ? std::min(h->seg_steps, n_steps) : n_steps;
    const int nseg = (n_steps + seg - 1) / seg;
    std::vector<hipGraphExec_t> ex((size_t)nseg);
    for (int sg = 0; sg < nseg; ++sg) {
      const int i0 = sg * seg, i1 = std::min(n_steps, i0 + seg);
      // (use_cmb and T: the captured layers read the combined or the two map tables of this schedule)
      std::vector<int> key{B, flag_var_tilde, tac ? 1 : 0, n_steps, i0, i1, h->use_cmb ? 1 : 0, h->T};
      key.insert(key.end(), t_seq, t_seq + n_steps);
      auto it = h->graphs.find(key);
      if (it == h->graphs.end()) {
        GraphEntry ge;
        HIPC(hipStreamBeginCapture(h->cap_stream, hipStreamCaptureModeThreadLocal));
        int rc = enqueue(h->cap_stream, i0, i1);
        hipGraph_t g = nullptr;
        hipError_t ee = hipStreamEndCapture(h->cap_stream, &g);
        if (rc != PETDIFF_OK) {
          if (g) (void)hipGraphDestroy(g);
          return rc;
        }
        HIPC(ee);
        ge.graph = g;
        HIPC(hipGraphInstantiate(&ge.exec, g, nullptr, nullptr, 0));
        it = h->graphs.emplace(key, ge).first;
      }
      ex[sg] = it->second.exec;
    }
    for (int sg = 0; sg < nseg; ++sg) HIPC(hipGraphLaunch(ex[sg], s));
  }
  HIPC(hipMemcpyAsync(x_out, bufs[n_steps & 1], xbytes, hipMemcpyDeviceToDevice, s));
  return PETDIFF_OK;
}

int petdiff_philox_normal(petdiff_handle h, uint64_t seed, uint64_t sample_offset, int rng_step, float* out, int B,
                          void* stream) {
  CHK(valid_handle(h));
  if (B < 0 || (B > 0 && !out)) return fail(PETDIFF_ERR_INVALID, "bad arguments");
  HIPC(launch_philox_normal(seed, sample_offset, rng_step, B, out, (hipStream_t)stream));
  return PETDIFF_OK;
}

int petdiff_posterior_stats(petdiff_handle h, const float* x0, const int32_t* tac, int B, int n_tac,
                            double* stats, void* stream) {
  CHK(valid_handle(h));
  if (!x0 || !stats || B < 0 || n_tac <= 0) return fail(PETDIFF_ERR_INVALID, "bad arguments");
  hipStream_t s = (hipStream_t)stream;
  const int ncol = h->cfg.n_roi * h->cfg.n_par;
  DevBuf d;
  HIPC(d.alloc((size_t)n_tac * ncol * 3 * 8));
  HIPC(launch_posterior_stats(x0, tac, B, n_tac, ncol, d.as<double>(), s));
  HIPC(hipMemcpyAsync(stats, d.p, (size_t)n_tac * ncol * 3 * 8, hipMemcpyDeviceToHost, s));
  HIPC(hipStreamSynchronize(s));
  return PETDIFF_OK;
}

int petdiff_get_activation(petdiff_handle h, int level, float* out, int B, void* stream) {
  CHK(valid_handle(h));
  if (level < 0 || level >= PETDIFF_NUM_LEVELS) return fail(PETDIFF_ERR_INVALID, "level out of range");
  if (B < 0 || (B > 0 && !out)) return fail(PETDIFF_ERR_INVALID, "bad arguments");
  if (B > h->last_B) return fail(PETDIFF_ERR_INVALID, "B exceeds the batch of the last forward / p_sample");
  const DevBuf* bufs[PETDIFF_NUM_LEVELS] = {&h->s0, &h->s1, &h->s2, &h->d3, &h->b0, &h->b1};
  const size_t per[PETDIFF_NUM_LEVELS] = {48 * 128, 24 * 256, 12 * 512, 6 * 1024, 12 * 512, 24 * 256};
  const size_t n = (size_t)B * per[level];
  hipStream_t s = (hipStream_t)stream;
  const void* src = bufs[level]->p;
  static const int chan[PETDIFF_NUM_LEVELS] = {128, 256, 512, 1024, 512, 256};
  if (h->x3) HIPC(launch_split_to_f32(static_cast<const bf16*>(src), n / chan[level], chan[level], out, s));
  else if (h->cfg.dtype == PETDIFF_DTYPE_BF16) HIPC(launch_to_f32<bf16>(static_cast<const bf16*>(src), n, out, s));
  else if (h->cfg.dtype == PETDIFF_DTYPE_F16) HIPC(launch_to_f32<f16>(static_cast<const f16*>(src), n, out, s));
  else HIPC(launch_to_f32<float>(static_cast<const float*>(src), n, out, s));
  return PETDIFF_OK;
}

int petdiff_piece_key(int row, int cpr, int m16) { return piece_key(row, cpr, m16 != 0); }

int petdiff_set_timing(petdiff_handle h, int enable) {
  CHK(valid_handle(h));
  h->timing = enable > 0;
  h->timing_reps = enable > 0 ? std::min(enable, 64) : 1;
  return PETDIFF_OK;
}

int petdiff_get_timing(petdiff_handle h, float* total_ms, int* count) {
  CHK(valid_handle(h));
  for (int i = 0; i < PETDIFF_NUM_LAYERS; ++i) {
    if (total_ms) total_ms[i] = 0.f;
    if (count) count[i] = 0;
  }
  for (auto& u : h->ev_used) {
    HIPC(hipEventSynchronize(u.e1));
    float ms = 0.f;
    HIPC(hipEventElapsedTime(&ms, u.e0, u.e1));
    if (total_ms) total_ms[u.layer] += ms;
    if (count) count[u.layer] += u.reps;
  }
  h->ev_used.clear();
  h->ev_next = 0;
  return PETDIFF_OK;
}

}  // extern "C"
