// CPU emulation of the colour-sharded chromatic sweep (graph_prep.h
// ShardPlan; capi.hip nngp_sweep_chains_group / the RCCL path) against the
// single-rank sweep on the same layout: G ranks, each with its own r and w
// replica, sweep their own chunks of every colour, publish {dw, w_new} into
// their segment of the colour's exchange region, "all-gather" it, then apply
// the ghost cells (r_k += B[k,j] dw_j) and the replica updates (w_j = w_new).
// Checks, bitwise: every rank's w replica and its r on the rows its columns
// touch equal the single-rank sweep after every colour; the ranks' segments
// partition every colour; every ghost cell's B value is the one of the
// single-rank sweep; normal pairs cover every owned location.
//   shard_check <n> <m> <G> <sweeps> <seed>   (prints "ok <stats>")
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "graph_prep.h"

using namespace nngp;

#define REQUIRE(c)                                                   \
  do {                                                               \
    if (!(c)) {                                                      \
      std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);        \
      return 1;                                                      \
    }                                                                \
  } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 5000;
  const int m = argc > 2 ? std::atoi(argv[2]) : 10;
  const int G = argc > 3 ? std::atoi(argv[3]) : 2;
  const int S = argc > 4 ? std::atoi(argv[4]) : 2;
  const int seed = argc > 5 ? std::atoi(argv[5]) : 1;
  const int d = 2, b = m + 1;
  std::mt19937_64 g(seed);
  std::uniform_real_distribution<double> U(0, 1);
  std::normal_distribution<double> N01(0, 1);
  std::vector<double> raw((size_t)n * d), locs((size_t)n * d);
  for (auto& v : raw) v = U(g);
  std::vector<int> ord;
  order_maxmin(raw.data(), n, d, ord);
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < d; ++k) locs[i + (size_t)k * n] = raw[ord[i] + (size_t)k * n];
  std::vector<int> nn, col;
  find_ordered_nn(locs.data(), n, d, m, nn);
  greedy_coloring(nn.data(), n, b, col);
  SweepLayout L;
  std::string err;
  REQUIRE(build_sweep_layout(nn.data(), n, b, col.data(), locs.data(), d, 64, L, err));
  const int K = L.K;
  // B in device order (row-major n x b by Morton row), random values
  std::vector<double> linv((size_t)n * b, 0.0);
  for (int k = 0; k < n; ++k)
    for (int t = 0; t < b; ++t)
      if (nn[(size_t)k * b + t] >= 0) linv[(size_t)L.rpos[k] * b + t] = t == 0 ? 1.0 + U(g) : 0.5 * N01(g);
  // columns: (device row, Linv index) of each nonzero of column i
  std::vector<std::vector<std::pair<int, int>>> colv(n);
  for (int k = 0; k < n; ++k)
    for (int t = 0; t < b; ++t) {
      const int j = nn[(size_t)k * b + t];
      if (j >= 0) colv[j].push_back({L.rpos[k], L.rpos[k] * b + t});
    }
  std::vector<double> D(n, 0.0), w0(n), Rs(n), z((size_t)S * n);
  for (int i = 0; i < n; ++i)
    for (auto& e : colv[i]) D[i] += linv[e.second] * linv[e.second];
  for (int i = 0; i < n; ++i) { w0[i] = N01(g); Rs[i] = N01(g); }
  for (auto& v : z) v = N01(g);
  const double inv_s2 = 0.7, inv_t2 = 1.3;
  auto draw = [&](int i, double acc, double w, int s) {
    const double P = D[i] * inv_s2 + inv_t2;
    const double cR = inv_t2 * Rs[i] + inv_s2 * (D[i] * w);
    return (cR - inv_s2 * acc) * (1.0 / P) + z[(size_t)s * n + i] / std::sqrt(P);
  };
  auto initial_r = [&](const std::vector<double>& w) {  // r = B w, device rows
    std::vector<double> r(n, 0.0);
    for (int k = 0; k < n; ++k)
      for (int t = 0; t < b; ++t) {
        const int j = nn[(size_t)k * b + t];
        if (j >= 0) r[L.rpos[k]] += linv[(size_t)L.rpos[k] * b + t] * w[j];
      }
    return r;
  };
  // plans of every rank
  std::vector<ShardPlan> P(G);
  for (int h = 0; h < G; ++h) REQUIRE(build_shard_plan(nn.data(), n, b, col.data(), L, G, h, P[h], err));
  long long owned = 0, ghosts = 0;
  for (int h = 0; h < G; ++h) {
    owned += P[h].owned;
    ghosts += (long long)P[h].grow.size();
    REQUIRE(P[h].cb == P[0].cb && P[h].seg0 == P[0].seg0 && P[h].cnt == P[0].cnt);
  }
  REQUIRE(owned == n);
  for (int c = 0; c < K; ++c) {
    const int* sg = &P[0].seg0[(size_t)c * (G + 1)];
    REQUIRE(sg[0] == L.color_loc_ptr[c] && sg[G] == L.color_loc_ptr[c + 1]);
    for (int h = 0; h < G; ++h) REQUIRE(sg[h] <= sg[h + 1] && sg[h + 1] - sg[h] <= P[0].cnt[c]);
  }
  // owner of each location; normal pairs cover every owned location
  std::vector<int> owner_loc(n);
  for (int c = 0; c < K; ++c)
    for (int h = 0; h < G; ++h)
      for (int x = P[0].seg0[(size_t)c * (G + 1) + h]; x < P[0].seg0[(size_t)c * (G + 1) + h + 1]; ++x)
        owner_loc[L.compact_loc[x]] = h;
  for (int h = 0; h < G; ++h) {
    std::vector<char> has(n, 0);
    for (int p : P[h].pairs) { has[2 * p] = 1; if (2 * p + 1 < n) has[2 * p + 1] = 1; }
    for (int i = 0; i < n; ++i) REQUIRE(owner_loc[i] != h || has[i]);
  }
  // single-rank sweep (reference) and the G-rank emulation, colour by colour
  std::vector<double> w = w0, r = initial_r(w0);
  std::vector<std::vector<double>> wg(G, w0), rg(G, r);
  std::vector<std::vector<char>> needed(G, std::vector<char>(n, 0));
  for (int h = 0; h < G; ++h)
    for (int c = 0; c < K; ++c)
      for (int x = P[0].seg0[(size_t)c * (G + 1) + h]; x < P[0].seg0[(size_t)c * (G + 1) + h + 1]; ++x)
        for (auto& e : colv[L.compact_loc[x]]) needed[h][e.first] = 1;
  for (int h = 0; h < G; ++h) {
    long long cntn = 0;
    for (int k = 0; k < n; ++k) cntn += needed[h][k];
    REQUIRE(cntn == P[h].needed_rows);
  }
  for (int s = 0; s < S; ++s) {
    for (int c = 0; c < K; ++c) {
      for (int x = L.color_loc_ptr[c]; x < L.color_loc_ptr[c + 1]; ++x) {
        const int i = L.compact_loc[x];
        double acc = 0.0;
        for (auto& e : colv[i]) acc += linv[e.second] * r[e.first];
        acc -= D[i] * w[i];
        const double wn = draw(i, acc, w[i], s), dw = wn - w[i];
        for (auto& e : colv[i]) r[e.first] = std::fma(linv[e.second], dw, r[e.first]);
        w[i] = wn;
      }
      // ranks: own slots -> exchange region
      std::vector<double> xdw((size_t)G * P[0].cnt[c], 0.0), xwn((size_t)G * P[0].cnt[c], 0.0);
      for (int h = 0; h < G; ++h) {
        const int x0 = P[0].seg0[(size_t)c * (G + 1) + h], x1 = P[0].seg0[(size_t)c * (G + 1) + h + 1];
        for (int x = x0; x < x1; ++x) {
          const int i = L.compact_loc[x];
          double acc = 0.0;
          for (auto& e : colv[i]) acc += linv[e.second] * rg[h][e.first];
          acc -= D[i] * wg[h][i];
          const double wn = draw(i, acc, wg[h][i], s), dw = wn - wg[h][i];
          for (auto& e : colv[i]) rg[h][e.first] = std::fma(linv[e.second], dw, rg[h][e.first]);
          wg[h][i] = wn;
          xdw[(size_t)h * P[0].cnt[c] + (x - x0)] = dw;
          xwn[(size_t)h * P[0].cnt[c] + (x - x0)] = wn;
        }
      }
      // ghost cells and replica updates
      for (int h = 0; h < G; ++h) {
        const ShardPlan& Q = P[h];
        for (int e = Q.gptr[c]; e < Q.gptr[c + 1]; ++e)
          rg[h][Q.grow[e]] = std::fma(linv[Q.gsrc[e]], xdw[Q.grecv[e]], rg[h][Q.grow[e]]);
        for (int o = 0; o < G; ++o) {
          if (o == h) continue;
          const int x0 = P[0].seg0[(size_t)c * (G + 1) + o], x1 = P[0].seg0[(size_t)c * (G + 1) + o + 1];
          for (int x = x0; x < x1; ++x) wg[h][L.compact_loc[x]] = xwn[(size_t)o * P[0].cnt[c] + (x - x0)];
        }
      }
      for (int h = 0; h < G; ++h) {
        for (int i = 0; i < n; ++i) REQUIRE(wg[h][i] == w[i]);
        for (int k = 0; k < n; ++k) REQUIRE(!needed[h][k] || rg[h][k] == r[k]);
      }
    }
  }
  std::printf("ok K=%d G=%d owned=%lld ghosts=%lld needed_rows_rank0=%lld exchange_slots=%lld\n", K, G, owned,
              ghosts, P[0].needed_rows, P[0].xoff[K]);
  return 0;
}
