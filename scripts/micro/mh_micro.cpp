// MH kernel micro-benchmark (diagnostic, not the product): throughput at 10k chains and
// single-chain latency, through the C ABI.  Build: see scripts/micro/build_mh.sh.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "petmh.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "mh_problem.bin";
  std::vector<double> d(54 + 54 + 1 + 48 * 54 * 2 + 48 * 2 + 48 * 48 * 2);
  FILE* f = fopen(path, "rb");
  if (!f || fread(d.data(), 8, d.size(), f) != d.size()) { printf("bad problem file\n"); return 1; }
  fclose(f);
  size_t o = 0;
  auto take = [&](size_t n) { const double* p = d.data() + o; o += n; return p; };
  petmh_problem p{};
  p.n_roi = 48; p.n_frames = 54;
  p.time_vector = take(54); p.tac_ref = take(54); p.k2p = *take(1);
  p.y_obs = take(48 * 54); p.sigma_noise = take(48 * 54);
  p.mu_DVR = take(48); p.cov_DVR = take(48 * 48); p.mu_R1 = take(48); p.cov_R1 = take(48 * 48);
  petmh_handle h;
  if (petmh_create(&p, 0, &h)) { printf("create: %s\n", petmh_last_error()); return 1; }
  double *stats, *acc;
  const int nmax = 10000;
  CK(hipMalloc(&stats, (size_t)nmax * 96 * 3 * 8));
  CK(hipMalloc(&acc, (size_t)nmax * 96 * 8));
  auto run = [&](int n, int draws, int tune) {
    CK(hipDeviceSynchronize());
    auto t0 = std::chrono::steady_clock::now();
    if (petmh_run(h, nullptr, n, draws, tune, 7, stats, acc, nullptr, nullptr)) { printf("run: %s\n", petmh_last_error()); exit(1); }
    CK(hipDeviceSynchronize());
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  };
  run(256, 2, 0);
  const double t1 = run(10000, 150, 50);
  const double t2 = run(4, 200, 100);
  std::vector<double> a(96 * 10000);
  CK(hipMemcpy(a.data(), acc, a.size() * 8, hipMemcpyDeviceToHost));
  double ar = 0;
  for (double v : a) ar += v;
  printf("%s: 10k chains x 200 steps %.3f s = %.3e chain-steps/s | 4 chains x 300 steps %.3f s = %.2f us/update | accept %.4f\n",
         MH_VARIANT, t1, 10000.0 * 200 / t1, t2, t2 / (300.0 * 96) * 1e6, ar / (96.0 * 4 * 200));
  return 0;
}
