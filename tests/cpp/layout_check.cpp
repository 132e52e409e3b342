// Invariants of the sweep layout planner (graph_prep.cpp), checked on CPU:
// every nonzero B[k,i] appears exactly once, in its slot's lane group, at the
// closed-form address the sweep kernel computes from the colour class table;
// padding is inert; chunk classes tile each colour.  Usage:
//   layout_check <n> <m> <lanes_per_chain> <seed>   (prints "ok <stats>")
#include <cstdio>
#include <cstdlib>
#include <random>
#include <set>
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
  const int LW = argc > 3 ? std::atoi(argv[3]) : 64;
  const int seed = argc > 4 ? std::atoi(argv[4]) : 1;
  const int d = 2, b = m + 1;
  std::mt19937_64 g(seed);
  std::uniform_real_distribution<double> U(0, 1);
  std::vector<double> raw((size_t)n * d), locs((size_t)n * d);
  for (auto& v : raw) v = U(g);
  std::vector<int> ord;
  order_maxmin(raw.data(), n, d, ord);
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < d; ++k) locs[i + (size_t)k * n] = raw[ord[i] + (size_t)k * n];
  std::vector<int> nn, col;
  find_ordered_nn(locs.data(), n, d, m, nn);
  const int K = greedy_coloring(nn.data(), n, b, col);
  SweepLayout L;
  std::string err;
  REQUIRE(build_sweep_layout(nn.data(), n, b, col.data(), locs.data(), d, LW, L, err));
  REQUIRE(L.K == K && L.LW == LW);
  // expected (row position, src) multiset per location
  std::vector<std::set<std::pair<int, int>>> want(n);
  long long nnz = 0;
  for (int k = 0; k < n; ++k)
    for (int t = 0; t < b; ++t) {
      const int a = nn[(size_t)k * b + t];
      if (a < 0) continue;
      want[a].insert({L.rpos[k], L.rpos[k] * b + t});
      ++nnz;
    }
  REQUIRE(nnz == L.nnz);
  std::vector<char> seen_slot(n, 0);
  std::vector<char> used((size_t)L.n_entries, 0);
  long long found = 0;
  for (int c = 0; c < K; ++c) {
    const int ch0 = L.color_chunk_ptr[c], nch = L.color_chunk_ptr[c + 1] - ch0;
    const int ncls = L.n_class[c];
    REQUIRE(ncls >= 1 && ncls <= kMaxClasses);
    REQUIRE(L.class_end[(size_t)c * kMaxClasses + ncls - 1] == nch);
    for (int lch = 0; lch < nch; ++lch) {
      // the kernel's closed form (chunk_class in kernels.hip)
      int q = 0;
      while (q + 1 < ncls && lch >= L.class_end[(size_t)c * kMaxClasses + q]) ++q;
      const int R = L.class_rows[(size_t)c * kMaxClasses + q];
      const int start = q ? L.class_end[(size_t)c * kMaxClasses + q - 1] : 0;
      const long long base = L.class_base[(size_t)c * kMaxClasses + q] + (long long)(lch - start) * LW * R;
      REQUIRE(R >= 1 && R <= kRowsMax);
      REQUIRE(base + (long long)LW * R <= L.n_entries);
      const int ch = ch0 + lch;
      for (int l = 0; l < LW; ++l) {
        const int v = L.lane_tab[(size_t)ch * LW + l];
        if (!v) continue;
        const int s = (v & 0x0FFFFFFF) - 1, lk = v >> 28, k = 1 << lk;
        REQUIRE(s >= L.color_slot_ptr[c] && s < L.color_slot_ptr[c + 1]);
        REQUIRE((l & (k - 1)) == (l % k));  // aligned group
        const int i = L.slot_loc[s];
        REQUIRE(col[i] == c + 1);
        const int len = L.collen[s];
        REQUIRE(len == (int)want[i].size());
        REQUIRE((len + k - 1) / k <= R);
        const int u = l & (k - 1);
        if (u == 0) { REQUIRE(!seen_slot[s]); seen_slot[s] = 1; }
        for (int j = 0; j < R; ++j) {
          const long long e = base + (long long)j * LW + l;
          REQUIRE(!used[e]);
          used[e] = 1;
          if (j * k + u < len) {
            REQUIRE(want[i].count({L.ent_rowpos[e], L.ent_src[e]}) == 1);
            ++found;
          } else {
            REQUIRE(L.ent_src[e] == -1);
          }
        }
      }
    }
  }
  REQUIRE(found == nnz);
  for (int s = 0; s < n; ++s) REQUIRE(seen_slot[s]);
  for (int i = 0; i < n; ++i) REQUIRE(L.slot_loc[L.loc_slot[i]] == i);
  std::printf("ok K=%d nnz=%lld entries=%lld chunks=%d max_collen=%d\n", K, nnz, L.n_entries, L.nchunks,
              L.max_collen);
  return 0;
}
