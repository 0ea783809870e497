// Launch-boundary micro-benchmark (diagnostic, not the product).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 seq_micro.hip -o seq_micro
// Run:   ./seq_micro [B] [x]     (x: the bf16x3 instances)
//
// The six conv launches of one reverse step (down1, down2, down3, up0.fused, up1.fused, up2.fused), each on
// its own buffers, timed four ways with events:
//   R  each layer repeated back to back (sum of the per-layer averages): what conv_micro and bench.py's
//      kernel-timing reps measure;
//   S  the step order, layer after layer, independent buffers;
//   D  the step order with every layer launched twice in a row (D - S: the warm second launches);
//   C  the step order on chained buffers (each layer reads the previous one's output, as the loop does).
// S - R is the cost of a boundary between two different kernels; C - S what the data dependency adds.
// Built with -DCONV_EXP_MODE=128 it also prints, for the last step of S and of C, each layer's workgroup
// start / end stamps (s_memrealtime, one 100 MHz clock for the whole chip; the end stamp after the
// workgroup's stores drained): the start ramp, the tail, and the idle gap at every boundary (the time a
// ticket queue across the boundary could reclaim).
#include <algorithm>
#include "../../pet_posterior_distribution_amd/csrc/unet_kernels.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <string>

using namespace petdiff;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void fill_bf16(bf16* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = (bf16)(((int)(h & 0xffff) - 32768) * (1.0f / 262144.f));
  }
}
__global__ void fill_f32(float* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = ((int)(h & 0xffff) - 32768) * (1.0f / 262144.f);
  }
}

// every activation buffer has this many bytes, more than any layer reads or writes at B <= 1024 (bf16x3:
// [hi | lo] rows, 2 x), so re-pointing a layer's input at another layer's output stays in bounds
constexpr size_t kAct = 64ull << 20;

struct Layer {
  const char* name;
  int kind;
  ConvArgs<bf16> a;
  bf16 *in1, *in2, *out, *pool;   // own buffers (kAct bytes each)
  unsigned long long* dbg;         // CONV_EXP_MODE & 128: the stamps (fin.x_all)
  int grid;
};

bf16* act(unsigned seed) {
  bf16* p;
  CK(hipMalloc(&p, kAct));
  fill_bf16<<<1024, 256>>>(p, kAct / 2, seed);
  return p;
}
float* f32(size_t n, unsigned seed) {
  float* p;
  CK(hipMalloc(&p, n * 4));
  fill_f32<<<256, 256>>>(p, n, seed);
  return p;
}

template <int KIND, int XS>
Layer make(const char* name, int B, int c1, int c2, int cout, unsigned seed) {
  using G = ConvGeom<bf16, KIND>;
  constexpr int XM = XS ? (x3_paired(KIND) ? 2 : 3) : 1;
  const int n1 = XM * (c1 / G::KC), n2 = XM * (c2 / G::KC), NC = n1 + n2;
  const size_t wbytes = G::FUSED ? (size_t)(cout / G::NT) * (n1 * G::B_BYTES + n2 * G::B2_BYTES)
                                 : (size_t)(cout / G::NT) * NC * G::B_BYTES;
  const size_t ebytes = (size_t)(cout / G::NT) * (n2 > 0 ? n2 : 1) * 2 * G::NT * G::ROWB;
  Layer l{name, KIND, {}, act(seed), c2 ? act(seed + 1) : nullptr, act(seed + 2), act(seed + 3), nullptr,
          ((B + G::S - 1) / G::S) * (cout / G::NT)};
  bf16 *w, *ep;
  CK(hipMalloc(&w, wbytes));
  CK(hipMalloc(&ep, ebytes));
  fill_bf16<<<1024, 256>>>(w, wbytes / 2, seed + 4);
  fill_bf16<<<1024, 256>>>(ep, ebytes / 2, seed + 5);
  ConvArgs<bf16>& a = l.a;
  a.src1 = l.in1; a.c1 = c1; a.src2 = l.in2; a.c2 = c2; a.wpack = w; a.epack = ep; a.out = l.out; a.out_pool = l.pool;
  a.cmap = f32((size_t)G::L * cout, seed + 6);
  a.tmap = f32((size_t)1000 * G::L * cout, seed + 7);
  a.bias = f32(cout, seed + 8);
  a.t_uniform = 500; a.B = B; a.cout = cout; a.n_t = 1000; a.n_tac = 1;
  if (G::EPI == EPI_FINAL) {
    a.fin.wf = f32(512, seed + 9); a.fin.wf4 = a.fin.wf; a.fin.bf = f32(4, seed + 10); a.fin.n_out = 4;
    a.fin.x_t = f32((size_t)B * 96, seed + 11); a.fin.z = nullptr;
    unsigned long long* rng;
    CK(hipMalloc(&rng, 16));
    CK(hipMemset(rng, 0, 16));
    a.fin.rng = rng; a.fin.rng_step = 3; a.fin.tab = f32((size_t)kNTab * 1000, seed + 12); a.fin.T = 1000;
    a.fin.learn_mode = 2; a.fin.param_mode = 0; a.fin.flag_var_tilde = 1;
    a.fin.x_next = f32((size_t)B * 96, seed + 13);
    a.fin.next.x = a.fin.x_next; a.fin.next.w0 = f32(6 * 2 * 128, seed + 14); a.fin.next.cmap = f32(48 * 128, seed + 15);
    a.fin.next.tmap = f32((size_t)1000 * 48 * 128, seed + 16); a.fin.next.t_uniform = 499;
    a.fin.next.s0 = act(seed + 17); a.fin.next.p0 = act(seed + 18); a.fin.next.B = B;
  }
#if CONV_EXP_MODE & 128
  // stamps [0, 8192 + 4 * grid) and [16384, 16384 + grid), plus the final level's keep_all_xt rows
  const size_t dbg_bytes = 6 * 4096 * 8 + (size_t)B * 96 * 4;
  CK(hipMalloc(&l.dbg, dbg_bytes));
  CK(hipMemset(l.dbg, 0, dbg_bytes));
  a.fin.x_all = reinterpret_cast<float*>(l.dbg);
#endif
  return l;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 1024;
  const bool x3 = argc > 2 && argv[2][0] == 'x';
  if (B > 1024) { printf("B <= 1024 (buffer sizes)\n"); return 1; }
  std::vector<Layer> L;
  if (x3) {
    L.push_back(make<LK_DOWN1, 1>("down1", B, 128, 0, 256, 100));
    L.push_back(make<LK_DOWN2, 1>("down2", B, 256, 0, 512, 200));
    L.push_back(make<LK_DOWN3, 1>("down3", B, 512, 0, 1024, 300));
    L.push_back(make<LK_UP0_F, 1>("up0.fused", B, 512, 1024, 512, 400));
    L.push_back(make<LK_UP1_F, 1>("up1.fused", B, 256, 512, 256, 500));
    L.push_back(make<LK_UP2_FX3, 1>("up2.fused", B, 128, 256, 128, 600));
  } else {
    L.push_back(make<LK_DOWN1, 0>("down1", B, 128, 0, 256, 100));
    L.push_back(make<LK_DOWN2, 0>("down2", B, 256, 0, 512, 200));
    L.push_back(make<LK_DOWN3, 0>("down3", B, 512, 0, 1024, 300));
    L.push_back(make<LK_UP0_F, 0>("up0.fused", B, 512, 1024, 512, 400));
    L.push_back(make<LK_UP1_F, 0>("up1.fused", B, 256, 512, 256, 500));
    L.push_back(make<LK_UP2_F, 0>("up2.fused", B, 128, 256, 128, 600));
  }
  CK(hipDeviceSynchronize());
  // chained copies: each layer's input is the previous layer's output, as in the reverse loop
  std::vector<Layer> Ch = L;
  Ch[0].a.src1 = static_cast<const bf16*>(L[5].a.fin.next.p0);                  // down1 <- the fused next-step down0's pooled rows
  Ch[1].a.src1 = L[0].pool;                           // down2 <- down1's pooled output
  Ch[2].a.src1 = L[1].pool;                           // down3 <- down2's pooled output
  Ch[3].a.src1 = L[1].out; Ch[3].a.src2 = L[2].out;   // up0 <- skip of down2, coarse from down3
  Ch[4].a.src1 = L[0].out; Ch[4].a.src2 = L[3].out;   // up1 <- skip of down1, coarse from up0
  Ch[5].a.src1 = static_cast<const bf16*>(L[5].a.fin.next.s0); Ch[5].a.src2 = L[4].out;   // up2 <- s0, coarse from up1
  auto launch = [&](const Layer& l) { CK(launch_conv<bf16>(l.kind, l.a, 0, x3)); };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timed = [&](int iters, auto&& body) {
    for (int i = 0; i < 5; ++i) body();
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) body();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / iters;
  };
  auto stamps = [&](const std::vector<Layer>& ls, const char* tag) {
#if CONV_EXP_MODE & 128
    // per layer: first / last workgroup start, median / last end (us from the first layer's first start)
    std::vector<double> s0(ls.size()), s1(ls.size()), em(ls.size()), e1(ls.size());
    unsigned long long t0 = 0;
    for (size_t k = 0; k < ls.size(); ++k) {
      std::vector<unsigned long long> t4(4 * ls[k].grid);
      CK(hipMemcpy(t4.data(), ls[k].dbg + 8192, t4.size() * 8, hipMemcpyDeviceToHost));
      std::vector<unsigned long long> st, en;
      for (int b = 0; b < ls[k].grid; ++b) { st.push_back(t4[4 * b]); en.push_back(t4[4 * b + 3]); }
      std::sort(st.begin(), st.end());
      std::sort(en.begin(), en.end());
      if (k == 0) t0 = st[0];
      s0[k] = (double)(st[0] - t0) * 0.01; s1[k] = (double)(st.back() - t0) * 0.01;
      em[k] = (double)(en[en.size() / 2] - t0) * 0.01; e1[k] = (double)(en.back() - t0) * 0.01;
    }
    printf("  %s stamps of the last step (us):\n", tag);
    double idle = 0.0;
    for (size_t k = 0; k < ls.size(); ++k) {
      const double gap = k + 1 < ls.size() ? s0[k + 1] - e1[k] : 0.0;
      idle += gap + (e1[k] - em[k]);
      printf("    %-10s start %7.2f ramp %5.2f | end median %7.2f last %7.2f tail %5.2f | gap to next %5.2f\n",
             ls[k].name, s0[k], s1[k] - s0[k], em[k], e1[k], e1[k] - em[k], gap);
    }
    printf("    first start -> last end %.2f us; tails + gaps %.2f us\n", e1.back() - s0[0], idle);
    // the layer with the longest tail: its last workgroups (XCC, CU, phases) and the per-XCC median end
    size_t kt = 0;
    for (size_t k = 1; k < ls.size(); ++k) if (e1[k] - em[k] > e1[kt] - em[kt]) kt = k;
    const int g = ls[kt].grid;
    std::vector<unsigned long long> t4(4 * g), loc(g);
    CK(hipMemcpy(t4.data(), ls[kt].dbg + 8192, t4.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(loc.data(), ls[kt].dbg + 16384, loc.size() * 8, hipMemcpyDeviceToHost));
    std::vector<int> ord(g);
    for (int b = 0; b < g; ++b) ord[b] = b;
    std::sort(ord.begin(), ord.end(), [&](int x, int y) { return t4[4 * x + 3] > t4[4 * y + 3]; });
    printf("    %s, last workgroups (bid xcc cu | start prologue loop epilogue us):\n", ls[kt].name);
    for (int q = 0; q < 6; ++q) {
      const int b = ord[q];
      printf("      %3d %2llu %3llu | %6.2f %5.2f %6.2f %5.2f\n", b, loc[b] >> 16, loc[b] & 0xff,
             (double)(t4[4 * b] - t0) * 0.01 - s0[kt], (t4[4 * b + 1] - t4[4 * b]) * 0.01,
             (t4[4 * b + 2] - t4[4 * b + 1]) * 0.01, (t4[4 * b + 3] - t4[4 * b + 2]) * 0.01);
    }
    printf("      per-XCC median loop us:");
    for (unsigned x = 0; x < 8; ++x) {
      std::vector<double> lp;
      for (int b = 0; b < g; ++b) if ((loc[b] >> 16) == x) lp.push_back((t4[4 * b + 2] - t4[4 * b + 1]) * 0.01);
      std::sort(lp.begin(), lp.end());
      if (!lp.empty()) printf(" %.2f", lp[lp.size() / 2]);
    }
    printf("\n      per-XCC max loop us:");
    for (unsigned x = 0; x < 8; ++x) {
      double mx = 0.0;
      for (int b = 0; b < g; ++b) if ((loc[b] >> 16) == x) mx = std::max(mx, (t4[4 * b + 2] - t4[4 * b + 1]) * 0.01);
      printf(" %.2f", mx);
    }
    printf("\n");
#else
    (void)ls; (void)tag;
#endif
  };
  const int it = 100;
  for (int rep = 0; rep < 2; ++rep) {
    double r = 0.0;
    printf("%s B = %d, round %d\n", x3 ? "bf16x3" : "bf16", B, rep);
    for (auto& l : L) {
      const double t = timed(it, [&] { launch(l); });
      printf("  R %-10s %8.2f us\n", l.name, t);
      r += t;
    }
    const double s = timed(it, [&] { for (auto& l : L) launch(l); });
    stamps(L, "S");
    const double d = timed(it, [&] { for (auto& l : L) { launch(l); launch(l); } });
    const double c = timed(it, [&] { for (auto& l : Ch) launch(l); });
    stamps(Ch, "C");
    printf("  R sum %.2f | S %.2f (S - R %+.2f) | D %.2f (D - S %.2f) | C %.2f (C - S %+.2f) us per step\n", r, s, s - r,
           d, d - s, c, c - s);
  }
  return 0;
}
