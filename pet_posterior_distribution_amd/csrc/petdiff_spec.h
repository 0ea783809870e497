// Ordered tensor list of the fp32 weight blob (include/petdiff.h), shared by the
// sampler (petdiff_api.cpp) and the training step (train_api.cpp).
#pragma once
#include "petdiff.h"

#include <string>
#include <vector>

namespace petdiff {

struct Spec {
  std::string name;
  std::vector<int> shape;
  size_t off;
  size_t size;
};

// Ordered tensor list of the weight blob (see petdiff.h); mirrors networks.py:781-992.
inline std::vector<Spec> make_spec(const petdiff_config& c, int n_out) {
  std::vector<Spec> s;
  size_t off = 0;
  auto add = [&](const std::string& n, std::vector<int> sh) {
    size_t sz = 1;
    for (int d : sh) sz *= (size_t)d;
    s.push_back({n, sh, off, sz});
    off += sz;
  };
  std::vector<int> dl{c.n_roi};
  for (int d = 1; d < c.depth; ++d) dl.push_back((dl.back() + 1) / c.pool_size);
  add("time_mlp.kernel", {c.sin_emb_dim, c.n_roi});
  add("time_mlp.bias", {c.n_roi});
  int prev = c.n_frames;
  for (int i = 0; i < 3; ++i) {
    add("cond_enc.hidden" + std::to_string(i) + ".kernel", {prev, c.enc_size[i]});
    add("cond_enc.hidden" + std::to_string(i) + ".bias", {c.enc_size[i]});
    prev = c.enc_size[i];
  }
  add("cond_enc.z.kernel", {prev, c.latent_dim});
  add("cond_enc.z.bias", {c.latent_dim});
  int cin = c.n_par;
  for (int d = 0; d < c.depth; ++d) {
    const int L = dl[d], cout = c.num_filt_start << d, ci = c.n_cond_rows + 1 + cin;
    const std::string p = "down" + std::to_string(d);
    add(p + ".time_proj.kernel", {c.n_roi, L});
    add(p + ".time_proj.bias", {L});
    add(p + ".label_proj.kernel", {c.latent_dim, L});
    add(p + ".label_proj.bias", {L});
    add(p + ".conv.kernel", {c.kernel_size, ci, cout});
    add(p + ".conv.bias", {cout});
    add(p + ".res.kernel", {1, ci, cout});
    add(p + ".res.bias", {cout});
    cin = cout;
  }
  for (int u = 0; u < c.depth - 1; ++u) {
    const int L = dl[c.depth - 1 - u], cout = c.num_filt_start << (c.depth - 2 - u);
    const int ci = c.n_cond_rows + 1 + cin;
    const std::string p = "up" + std::to_string(u);
    add(p + ".time_proj.kernel", {c.n_roi, L});
    add(p + ".time_proj.bias", {L});
    add(p + ".label_proj.kernel", {c.latent_dim, L});
    add(p + ".label_proj.bias", {L});
    add(p + ".upconv.kernel", {c.pool_size, ci, cout});
    add(p + ".upconv.bias", {cout});
    add(p + ".conv.kernel", {c.kernel_size, 2 * cout, cout});
    add(p + ".conv.bias", {cout});
    add(p + ".res.kernel", {1, 2 * cout, cout});
    add(p + ".res.bias", {cout});
    cin = cout;
  }
  add("final.kernel", {1, c.num_filt_start, n_out});
  add("final.bias", {n_out});
  return s;
}


inline bool is_shipped_arch(const petdiff_config& c) {
  return c.n_roi == 48 && c.n_par == 2 && c.n_frames == 54 && c.n_cond_rows == 49 && c.num_filt_start == 128 &&
         c.depth == 4 && c.kernel_size == 6 && c.pool_size == 2 && c.sin_emb_dim == 64 && c.enc_size[0] == 256 &&
         c.enc_size[1] == 128 && c.enc_size[2] == 64 && c.latent_dim == 32;
}

}  // namespace petdiff
