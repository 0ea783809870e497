// Timeline of the down2 -> down3 seam (diagnostic, not the product): down2 and down3 as two launches,
// then the same two layers as one seam23_kernel launch (PETDIFF_SEAM23), with in-kernel s_memrealtime
// stamps (10 ns ticks, one clock for the whole chip) per workgroup: start, first chunk landed (for a
// seam consumer: after its wait), K loop end, end; and the consumer's poll end.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -DCONV_EXP_MODE=128 seam_micro.hip -o seam_micro
#include "../../pet_posterior_distribution_amd/csrc/unet_kernels.hip"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

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

static const size_t kDbg = 6 * 4096;   // stamp words per buffer

template <int KIND>
ConvArgs<bf16> layer(int B, int c1, int cout, bf16* src, bf16** pool_out, unsigned seed) {
  using G = ConvGeom<bf16, KIND>;
  ConvArgs<bf16> a{};
  const size_t rows_out = (size_t)B * G::L;
  bf16 *w, *out, *pool;
  float *cmap, *tmap, *bias;
  const size_t wbytes = (size_t)(cout / G::NT) * (c1 / G::KC) * G::B_BYTES;
  CK(hipMalloc(&w, wbytes));
  CK(hipMalloc(&out, rows_out * cout * 2));
  CK(hipMalloc(&pool, rows_out * cout));
  CK(hipMalloc(&cmap, (size_t)G::L * cout * 4));
  CK(hipMalloc(&tmap, (size_t)1000 * G::L * cout * 4));
  CK(hipMalloc(&bias, cout * 4));
  fill_bf16<<<1024, 256>>>(w, wbytes / 2, seed);
  fill_f32<<<1024, 256>>>(cmap, (size_t)G::L * cout, seed + 1);
  fill_f32<<<1024, 256>>>(tmap, (size_t)1000 * G::L * cout, seed + 2);
  fill_f32<<<64, 256>>>(bias, cout, seed + 3);
  a.src1 = src; a.c1 = c1; a.src2 = nullptr; a.c2 = 0; a.wpack = w; a.out = out; a.out_pool = pool;
  a.cmap = cmap; a.tmap = tmap; a.bias = bias; a.tac = nullptr; a.tvec = nullptr; a.t_uniform = 500;
  a.B = B; a.cout = cout; a.n_t = 1000; a.n_tac = 1;
  *pool_out = pool;
  return a;
}

struct Tl { std::vector<double> st, pro, wait, lp, epi, en; };

static Tl read_tl(const unsigned long long* dbg_dev, int b0, int nb, unsigned long long t0, bool cons) {
  std::vector<unsigned long long> h(kDbg);
  CK(hipMemcpy(h.data(), dbg_dev, kDbg * 8, hipMemcpyDeviceToHost));
  Tl t;
  for (int b = b0; b < b0 + nb; ++b) {
    const unsigned long long* q = &h[8192 + 4 * b];
    t.st.push_back((q[0] - t0) * 0.01);
    t.pro.push_back((q[1] - q[0]) * 0.01);
    t.lp.push_back((q[2] - q[1]) * 0.01);
    t.epi.push_back((q[3] - q[2]) * 0.01);
    t.en.push_back((q[3] - t0) * 0.01);
    if (cons) t.wait.push_back((h[12288 + b] - q[0]) * 0.01);
  }
  return t;
}

static unsigned long long first_start(const unsigned long long* dbg_dev, int nb) {
  std::vector<unsigned long long> h(kDbg);
  CK(hipMemcpy(h.data(), dbg_dev, kDbg * 8, hipMemcpyDeviceToHost));
  unsigned long long m = ~0ull;
  for (int b = 0; b < nb; ++b) m = std::min(m, h[8192 + 4 * b]);
  return m;
}

static void show(const char* name, const Tl& t) {
  auto q = [](std::vector<double> v, double f) { std::sort(v.begin(), v.end()); return v[(size_t)(f * (v.size() - 1))]; };
  printf("  %-10s start [min %.2f med %.2f max %.2f] | prologue med %.2f max %.2f", name, q(t.st, 0), q(t.st, .5),
         q(t.st, 1), q(t.pro, .5), q(t.pro, 1));
  if (!t.wait.empty()) printf(" (poll end med %.2f max %.2f)", q(t.wait, .5), q(t.wait, 1));
  printf(" | K loop med %.2f max %.2f | epilogue med %.2f max %.2f | end [min %.2f med %.2f max %.2f]\n", q(t.lp, .5),
         q(t.lp, 1), q(t.epi, .5), q(t.epi, 1), q(t.en, 0), q(t.en, .5), q(t.en, 1));
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 1024;
  const int iters = 200;
  using G2 = ConvGeom<bf16, LK_DOWN2>;
  using G3 = ConvGeom<bf16, LK_DOWN3>;
  bf16* s1;
  const size_t rows_in = (size_t)B * G2::LIN;
  CK(hipMalloc(&s1, rows_in * 256 * 2));
  fill_bf16<<<1024, 256>>>(s1, rows_in * 256, 1);
  bf16 *p2, *p3;
  ConvArgs<bf16> a2 = layer<LK_DOWN2>(B, 256, 512, s1, &p2, 10);
  ConvArgs<bf16> a3 = layer<LK_DOWN3>(B, 512, 1024, p2, &p3, 20);
  unsigned long long *dbg2, *dbg3, *dbgs;
  CK(hipMalloc(&dbg2, kDbg * 8));
  CK(hipMalloc(&dbg3, kDbg * 8));
  CK(hipMalloc(&dbgs, kDbg * 8));
  CK(hipMemset(dbg2, 0, kDbg * 8));
  CK(hipMemset(dbg3, 0, kDbg * 8));
  CK(hipMemset(dbgs, 0, kDbg * 8));
  const int n2 = ((B + G2::S - 1) / G2::S) * (512 / G2::NT), n3 = ((B + G3::S - 1) / G3::S) * (1024 / G3::NT);
  int* seam;
  const int n_grp = (B + G3::S - 1) / G3::S;
  CK(hipMalloc(&seam, (n_grp + 2) * 4));
  CK(hipMemset(seam, 0, (n_grp + 2) * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms;

  // two launches
  a2.fin.x_all = reinterpret_cast<float*>(dbg2);
  a3.fin.x_all = reinterpret_cast<float*>(dbg3);
  for (int i = 0; i < 20; ++i) { CK(launch_conv<bf16>(LK_DOWN2, a2, 0)); CK(launch_conv<bf16>(LK_DOWN3, a3, 0)); }
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) { CK(launch_conv<bf16>(LK_DOWN2, a2, 0)); CK(launch_conv<bf16>(LK_DOWN3, a3, 0)); }
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("two launches: %.2f us per down2 + down3 pair (B = %d, grids %d + %d)\n", ms * 1e3 / iters, B, n2, n3);
  {
    const unsigned long long t0 = first_start(dbg2, n2);
    show("down2", read_tl(dbg2, 0, n2, t0, false));
    show("down3", read_tl(dbg3, 0, n3, t0, false));
  }

  // one seam launch
  a2.fin.x_all = reinterpret_cast<float*>(dbgs);
  a3.fin.x_all = reinterpret_cast<float*>(dbgs);
  for (int i = 0; i < 20; ++i) CK(launch_seam23<bf16>(a2, a3, seam, 0, false));
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) CK(launch_seam23<bf16>(a2, a3, seam, 0, false));
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<int> st(n_grp + 2);
  CK(hipMemcpy(st.data(), seam, (n_grp + 2) * 4, hipMemcpyDeviceToHost));
  printf("seam launch:  %.2f us per launch (grid %d + %d), spins given up: %d\n", ms * 1e3 / iters, n2, n3, st[n_grp + 1]);
  {
    const unsigned long long t0 = first_start(dbgs, n2);
    show("producer", read_tl(dbgs, 0, n2, t0, false));
    show("consumer", read_tl(dbgs, n2, n3, t0, true));
  }
  return 0;
}
