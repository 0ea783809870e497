// Micro-benchmark of the conv layers in isolation (diagnostic, not the product).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -DCONV_EXP_MODE=<m> conv_micro.hip
// Prints avg us per launch for each layer over random bf16 data.
#include "../../pet_posterior_distribution_amd/csrc/unet_kernels.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <string>
#include <cstring>

using namespace petdiff;

__global__ void fill_bf16(bf16* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = (bf16)(((int)(h & 0xffff) - 32768) * (1.0f / 65536.f));
  }
}
__global__ void fill_f32(float* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = ((int)(h & 0xffff) - 32768) * (1.0f / 65536.f);
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// XS = 1: the bf16x3 instance ([hi | lo] activation rows; paired chunks on the 64-B-row layers, 2 x the
// bf16 chunks, three passes on the 32-B final level, 3 x)
template <int KIND, int XS = 0>
void run(const char* name, int B, int c1, int c2, int cout, int iters) {
  using G = ConvGeom<bf16, KIND>;
  constexpr int RS = XS ? 2 : 1, XM = XS ? (x3_paired(KIND) ? 2 : 3) : 1;
  const size_t rows_in = (size_t)B * G::LIN, rows_out = (size_t)B * G::L;
  const int NC = XM * (c1 / G::KC + c2 / G::KC);
  bf16 *s1, *s2 = nullptr, *w, *out, *pool;
  float *cmap, *tmap, *bias;
  CK(hipMalloc(&s1, rows_in * c1 * 2 * RS));
  const size_t rows_in2 = G::FUSED ? (size_t)B * G::LH : rows_in;   // fused: src2 = the coarse input b
  if (c2) CK(hipMalloc(&s2, rows_in2 * c2 * 2 * RS));
  const int n1 = XM * (c1 / G::KC), n2 = XM * (c2 / G::KC);
  const size_t wbytes = G::FUSED ? (size_t)(cout / G::NT) * (n1 * G::B_BYTES + n2 * G::B2_BYTES)
                                 : (size_t)(cout / G::NT) * NC * G::B_BYTES;
  bf16* ep = nullptr;
  const size_t ebytes = (size_t)(cout / G::NT) * (n2 > 0 ? n2 : 1) * 2 * G::NT * G::ROWB;
  CK(hipMalloc(&ep, ebytes));
  fill_bf16<<<1024, 256>>>(ep, ebytes / 2, 11);
  CK(hipMalloc(&w, wbytes));
  CK(hipMalloc(&out, rows_out * cout * 2 * RS));
  CK(hipMalloc(&pool, rows_out * cout * RS));
  CK(hipMalloc(&cmap, (size_t)G::L * cout * 4));
  CK(hipMalloc(&tmap, (size_t)1000 * G::L * cout * 4));
  CK(hipMalloc(&bias, cout * 4));
  fill_bf16<<<1024, 256>>>(s1, rows_in * c1 * RS, 1);
  if (c2) fill_bf16<<<1024, 256>>>(s2, rows_in2 * c2 * RS, 2);
  fill_bf16<<<1024, 256>>>(w, wbytes / 2, 3);
  fill_f32<<<1024, 256>>>(cmap, (size_t)G::L * cout, 4);
  fill_f32<<<1024, 256>>>(tmap, (size_t)1000 * G::L * cout, 5);
  fill_f32<<<64, 256>>>(bias, cout, 6);
  // final-epilogue buffers
  float *wf, *bfv, *xt, *xn, *tab;
  unsigned long long* rng;
  CK(hipMalloc(&wf, 128 * 4 * 4));
  CK(hipMalloc(&bfv, 16));
  CK(hipMalloc(&xt, (size_t)B * 96 * 4));
  CK(hipMalloc(&xn, (size_t)B * 96 * 4));
  CK(hipMalloc(&tab, (size_t)kNTab * 1000 * 4));
  CK(hipMalloc(&rng, 16));
  fill_f32<<<64, 256>>>(wf, 512, 7);
  fill_f32<<<64, 256>>>(bfv, 4, 8);
  fill_f32<<<256, 256>>>(xt, (size_t)B * 96, 9);
  fill_f32<<<256, 256>>>(tab, (size_t)kNTab * 1000, 10);
  CK(hipMemset(rng, 0, 16));
  ConvArgs<bf16> a{};
  a.src1 = s1; a.c1 = c1; a.src2 = s2; a.c2 = c2; a.wpack = w; a.out = out; a.out_pool = pool;
  a.cmap = cmap; a.tmap = tmap; a.bias = bias; a.tac = nullptr; a.tvec = nullptr; a.t_uniform = 500;
  a.B = B; a.cout = cout; a.n_t = 1000; a.n_tac = 1;
  // the fused final level of a one-condition handle reads one combined map table (CONV_FIN_REGMAPS, as the
  // product: petdiff_api.cpp passes cmb_f[2] and no label map)
  if (G::FIN_MAPS && CONV_FIN_REGMAPS) a.cmap = nullptr;
  // wf: [128][4] (n_out = 4), which is also the packed wf4 layout the fused final level reads
  a.fin.wf = wf; a.fin.wf4 = wf; a.fin.bf = bfv; a.fin.n_out = 4; a.fin.x_t = xt; a.fin.z = nullptr; a.fin.rng = rng;
  a.fin.rng_step = 3; a.fin.tab = tab; a.fin.T = 1000; a.fin.learn_mode = 2; a.fin.param_mode = 0;
  a.fin.flag_var_tilde = 1; a.fin.x_next = xn;
  a.epack = ep;
  // fused next-step down0 (final level): weights, maps and the s0 / p0 outputs
  float *w0, *m0c, *m0t;
  bf16 *s0n, *p0n;
  CK(hipMalloc(&w0, 6 * 2 * 128 * 4));
  CK(hipMalloc(&m0c, 48 * 128 * 4));
  CK(hipMalloc(&m0t, (size_t)1000 * 48 * 128 * 4));
  CK(hipMalloc(&s0n, (size_t)B * 48 * 128 * 2 * RS));
  CK(hipMalloc(&p0n, (size_t)B * 24 * 128 * 2 * RS));
  fill_f32<<<64, 256>>>(w0, 6 * 2 * 128, 12);
  fill_f32<<<64, 256>>>(m0c, 48 * 128, 13);
  fill_f32<<<1024, 256>>>(m0t, (size_t)1000 * 48 * 128, 14);
  a.fin.next.x = xn; a.fin.next.w0 = w0; a.fin.next.cmap = m0c; a.fin.next.tmap = m0t;
  a.fin.next.tac = nullptr; a.fin.next.tvec = nullptr; a.fin.next.t_uniform = G::EPI == EPI_FINAL ? 499 : -1;
  a.fin.next.s0 = s0n; a.fin.next.p0 = p0n; a.fin.next.B = B;
  unsigned long long* dbg;
  // stamps [0, 8192 + 4 * grid) plus, on the final level, the keep_all_xt rows it writes through x_all
  const size_t dbg_bytes = 6 * 4096 * 8 + (size_t)B * 96 * 4;
  CK(hipMalloc(&dbg, dbg_bytes));
  CK(hipMemset(dbg, 0, dbg_bytes));
#if CONV_EXP_MODE & 128
  a.fin.x_all = reinterpret_cast<float*>(dbg);
#endif
  CK(hipDeviceSynchronize());
  if (G::EPI == EPI_FINAL) {   // launch_one's null-pointer guards (the r4f / r4g faults): refused, nothing launched
    ConvArgs<bf16> bad = a;
    bad.fin.x_t = nullptr;
    const hipError_t e = launch_conv<bf16>(KIND, bad, 0, XS != 0);
    (void)hipGetLastError();
    if (e != hipErrorInvalidValue) { printf("null-guard FAILED: %s\n", hipGetErrorString(e)); exit(1); }
    printf("   null-guard: a final level without x_t is refused (hipErrorInvalidValue)\n");
  }
  for (int i = 0; i < 20; ++i) CK(launch_conv<bf16>(KIND, a, 0, XS != 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) CK(launch_conv<bf16>(KIND, a, 0, XS != 0));
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / iters;
#if CONV_EXP_MODE & 128
  {
    const int nb = ((B + G::S - 1) / G::S) * (cout / G::NT);
    std::vector<unsigned long long> h(2 * nb);
    CK(hipMemcpy(h.data(), dbg, 2 * nb * 8, hipMemcpyDeviceToHost));
    std::vector<double> cyc, clk;
    for (int b = 0; b < nb; ++b) { cyc.push_back((double)h[2 * b]); clk.push_back(h[2 * b] / (h[2 * b + 1] * 1e-8) * 1e-9); }
    std::sort(cyc.begin(), cyc.end());
    std::sort(clk.begin(), clk.end());
    const double nmfma = (XS ? 3 : 1) * (G::FUSED ? ((double)c1 / G::KC * G::TAPS + (double)c2 / G::KC * G::TAPS2) * (G::ROWB / 32) * 6
                                  : (double)(c1 + c2) / G::KC * G::TAPS * (G::ROWB / 32) * 6);
    std::vector<unsigned long long> t4(4 * nb);
    CK(hipMemcpy(t4.data(), dbg + 8192, 4 * nb * 8, hipMemcpyDeviceToHost));
    unsigned long long tmin = ~0ull, tmax = 0;
    std::vector<double> pro, lp, epi, st;
    for (int b = 0; b < nb; ++b) tmin = std::min(tmin, t4[4 * b]);
    for (int b = 0; b < nb; ++b) {
      tmax = std::max(tmax, t4[4 * b + 3]);
      st.push_back((t4[4 * b] - tmin) * 0.01);
      pro.push_back((t4[4 * b + 1] - t4[4 * b]) * 0.01);
      lp.push_back((t4[4 * b + 2] - t4[4 * b + 1]) * 0.01);
      epi.push_back((t4[4 * b + 3] - t4[4 * b + 2]) * 0.01);
    }
    std::vector<unsigned long long> e2(2 * nb);
    CK(hipMemcpy(e2.data(), dbg + 4096, 2 * nb * 8, hipMemcpyDeviceToHost));
    std::vector<double> ea, eb, ec;
    for (int b = 0; b < nb; ++b) {
      ea.push_back((e2[2 * b] - t4[4 * b + 2]) * 0.01);
      eb.push_back((e2[2 * b + 1] - e2[2 * b]) * 0.01);
      ec.push_back((t4[4 * b + 3] - e2[2 * b + 1]) * 0.01);
    }
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    auto mx = [](std::vector<double> v) { return *std::max_element(v.begin(), v.end()); };
    printf("   us: start skew max %.2f | prologue med %.2f max %.2f | loop med %.2f max %.2f | epilogue med %.2f max %.2f | span %.2f\n",
           mx(st), med(pro), mx(pro), med(lp), mx(lp), med(epi), mx(epi), (tmax - tmin) * 0.01);
    printf("   epilogue us: acc->LDS+barrier %.2f | read/add/store issue %.2f | store drain %.2f\n", med(ea), med(eb),
           med(ec));
    {   // co-residency: workgroups whose [start, end] overlap on one CU (HW_ID cu/sh/se + XCC_ID)
      std::vector<unsigned long long> loc(nb);
      CK(hipMemcpy(loc.data(), dbg + 16384, nb * 8, hipMemcpyDeviceToHost));
      std::vector<std::pair<unsigned long long, int>> ev;
      std::vector<std::pair<unsigned long long, std::pair<unsigned long long, unsigned long long>>> iv;
      for (int b = 0; b < nb; ++b) iv.push_back({loc[b], {t4[4 * b], t4[4 * b + 3]}});
      std::sort(iv.begin(), iv.end());
      int maxc = 0, ncu = 0;
      double ovl = 0.0, busy = 0.0;
      for (size_t i = 0; i < iv.size();) {
        size_t j = i;
        while (j < iv.size() && iv[j].first == iv[i].first) ++j;
        ++ncu;
        std::vector<std::pair<unsigned long long, int>> e;
        for (size_t k = i; k < j; ++k) { e.push_back({iv[k].second.first, 1}); e.push_back({iv[k].second.second, -1}); }
        std::sort(e.begin(), e.end());
        int c = 0;
        for (size_t k = 0; k + 1 < e.size(); ++k) {
          c += e[k].second;
          maxc = std::max(maxc, c);
          const double d = (e[k + 1].first - e[k].first) * 0.01;
          if (c >= 1) busy += d;
          if (c >= 2) ovl += d;
        }
        i = j;
      }
      printf("   co-residency: %d CUs used, max %d workgroups at once on a CU, %.1f %% of CU-busy time with >= 2\n", ncu, maxc,
             busy > 0 ? 100.0 * ovl / busy : 0.0);
    }
    printf("   loop cycles median %.0f (%.1f per MFMA), clock median %.3f GHz [%.3f..%.3f]\n", cyc[nb / 2],
           cyc[nb / 2] / nmfma, clk[nb / 2], clk[0], clk[nb - 1]);
  }
#endif
  {   // output checksum (variants of one layer must agree to rounding)
    const size_t n = std::min<size_t>(rows_out * cout, 1 << 20);
    std::vector<unsigned short> hb(n);
    CK(hipMemcpy(hb.data(), out, n * 2, hipMemcpyDeviceToHost));
    double cs = 0.0;
    for (size_t i = 0; i < n; ++i) {
      unsigned u = (unsigned)hb[i] << 16;
      float f;
      memcpy(&f, &u, 4);
      cs += f;
    }
    printf("   checksum %.6e over %zu outputs, LDS %d B per workgroup, %d threads\n", cs, n, G::SMEM, G::NTH);
  }
  const double flop = G::FUSED ? 2.0 * rows_out * cout * ((double)c1 * G::TAPS + (double)c2 * G::TAPS2)
                               : 2.0 * rows_out * cout * (double)(c1 + c2) * G::TAPS;
  printf("%-12s mode %d  %8.2f us  %7.1f TF/s (executed)  grid %d\n", name, CONV_EXP_MODE, us, (XS ? 3 : 1) * flop / us * 1e-6,
         ((B + G::S - 1) / G::S) * (cout / G::NT));
  if (getenv("MICRO_2S")) {
    // Split-batch experiment: the same B samples as two halves on two streams (a graph of `iters` launch
    // pairs, fork / join by events), against one stream of whole-batch launches in a graph.  Do the halves'
    // phases (DMA prologue, MFMA loop, store epilogue) desynchronise and overlap across the chip?
    const int B1 = B / 2, B2 = B - B1;
    ConvArgs<bf16> a1 = a, a2 = a;
    a1.B = B1;
    a2.B = B2;
    a2.src1 = s1 + (size_t)B1 * G::LIN * c1 * RS;
    if (c2) a2.src2 = s2 + (size_t)B1 * (G::FUSED ? G::LH : G::LIN) * c2 * RS;
    a2.out = out + (size_t)B1 * G::L * cout * RS;
    a2.out_pool = pool + (size_t)B1 * (G::L / 2) * cout * RS;
    a2.fin.x_t = xt + (size_t)B1 * 96;
    a2.fin.x_next = xn + (size_t)B1 * 96;
    a1.fin.next.B = B1;
    a2.fin.next.B = B2;
    a2.fin.next.s0 = s0n + (size_t)B1 * 48 * 128 * RS;
    a2.fin.next.p0 = p0n + (size_t)B1 * 24 * 128 * RS;
    hipStream_t sa, sb;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    hipEvent_t fk, jn;
    CK(hipEventCreateWithFlags(&fk, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&jn, hipEventDisableTiming));
    auto capture = [&](bool split) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(sa, hipStreamCaptureModeThreadLocal));
      if (split) {
        CK(hipEventRecord(fk, sa));
        CK(hipStreamWaitEvent(sb, fk, 0));
      }
      for (int i = 0; i < iters; ++i) {
        if (split) {
          CK(launch_conv<bf16>(KIND, a1, sa, XS != 0));
          CK(launch_conv<bf16>(KIND, a2, sb, XS != 0));
        } else {
          CK(launch_conv<bf16>(KIND, a, sa, XS != 0));
        }
      }
      if (split) {
        CK(hipEventRecord(jn, sb));
        CK(hipStreamWaitEvent(sa, jn, 0));
      }
      CK(hipStreamEndCapture(sa, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphDestroy(g));
      return ge;
    };
    double t[2];
    for (int split = 0; split < 2; ++split) {
      hipGraphExec_t ge = capture(split != 0);
      CK(hipGraphLaunch(ge, sa));
      CK(hipStreamSynchronize(sa));
      CK(hipEventRecord(e0, sa));
      CK(hipGraphLaunch(ge, sa));
      CK(hipEventRecord(e1, sa));
      CK(hipEventSynchronize(e1));
      float gms;
      CK(hipEventElapsedTime(&gms, e0, e1));
      t[split] = gms * 1e3 / iters;
      CK(hipGraphExecDestroy(ge));
    }
    printf("   graph of %d launches: one stream %.2f us / batch | two streams x B/2 %.2f us / batch (%+.1f %%)\n", iters,
           t[0], t[1], 100.0 * (t[0] / t[1] - 1.0));
    CK(hipStreamDestroy(sa));
    CK(hipStreamDestroy(sb));
  }
  hipFree(s1); if (s2) hipFree(s2); hipFree(w); hipFree(out); hipFree(pool); hipFree(cmap); hipFree(tmap);
  hipFree(bias); hipFree(wf); hipFree(bfv); hipFree(xt); hipFree(xn); hipFree(tab); hipFree(rng); hipFree(dbg);
  hipFree(ep); hipFree(w0); hipFree(m0c); hipFree(m0t); hipFree(s0n); hipFree(p0n);
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 1024;
  const int it = 200;
  const char* only = argc > 2 ? argv[2] : "";
  if (std::string(only) == "u2") {   // the final level alone
    run<LK_UP2_F>("up2.fused", B, 128, 256, 128, it);
    return 0;
  }
  if (std::string(only) == "u2x") {   // the bf16x3 final level alone
    run<LK_UP2_FX3, 1>("up2.fused.x3", B, 128, 256, 128, it);
    return 0;
  }
  if (std::string(only) == "d1") {   // down1 alone (co-residency experiment: B = 1024 and 2048)
    run<LK_DOWN1>("down1", B, 128, 0, 256, it);
    return 0;
  }
  if (std::string(only) == "u0") {   // the dominant level alone
    run<LK_UP0_F>("up0.fused", B, 512, 1024, 512, it);
    return 0;
  }
  if (only[0] == 'x') {   // the bf16x3 step: down layers + fused up levels (the final level's paired instance)
    run<LK_DOWN1, 1>("down1.x3", B, 128, 0, 256, it);
    run<LK_DOWN2, 1>("down2.x3", B, 256, 0, 512, it);
    run<LK_DOWN3, 1>("down3.x3", B, 512, 0, 1024, it);
    run<LK_UP0_F, 1>("up0.fused.x3", B, 512, 1024, 512, it);
    run<LK_UP1_F, 1>("up1.fused.x3", B, 256, 512, 256, it);
    run<LK_UP2_FX3, 1>("up2.fused.x3", B, 128, 256, 128, it);
    return 0;
  }
  if (only[0] == 'f') {   // the product's 16-bit step: down layers + fused up levels
    run<LK_DOWN1>("down1", B, 128, 0, 256, it);
    run<LK_DOWN2>("down2", B, 256, 0, 512, it);
    run<LK_DOWN3>("down3", B, 512, 0, 1024, it);
    run<LK_UP0_F>("up0.fused", B, 512, 1024, 512, it);
    run<LK_UP1_F>("up1.fused", B, 256, 512, 256, it);
    run<LK_UP2_F>("up2.fused", B, 128, 256, 128, it);
    return 0;
  }
  run<LK_DOWN1>("down1", B, 128, 0, 256, it);
  run<LK_DOWN2>("down2", B, 256, 0, 512, it);
  run<LK_DOWN3>("down3", B, 512, 0, 1024, it);
  run<LK_UP0_CONV2>("up0.conv2", B, 1024, 0, 512, it);
  run<LK_UP0_BLOCK>("up0.block", B, 512, 512, 512, it);
  run<LK_UP1_CONV2>("up1.conv2", B, 512, 0, 256, it);
  run<LK_UP1_BLOCK>("up1.block", B, 256, 256, 256, it);
  run<LK_UP2_CONV2>("up2.conv2", B, 256, 0, 128, it);
  run<LK_UP2_BLOCK>("up2.block", B, 128, 128, 128, it);
  return 0;
}
