// Invariants of the sweep layout planner (graph_prep.cpp), checked on CPU:
// every nonzero B[k,i] appears exactly once, in its slot's stream range
// (through ent_pos), in a chunk whose cells are sorted by row; padding is
// inert and only at the stream tail.  Usage:
//   layout_check <n> <m> <lanes_per_chain> <seed>   (prints "ok <stats>")
#include <cstdio>
#include <cstdlib>
#include <random>
#include <set>
#include <string>
#include <vector>
#include <algorithm>

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
  const int cap = LW * kRowsMax, dummy = 2 * LW - 1;
  REQUIRE(L.n_entries == (long long)L.nchunks * cap);
  REQUIRE((int)L.chunk_first.size() == L.nchunks + 1 && L.chunk_first[L.nchunks] == n);
  REQUIRE(L.color_loc_ptr[K] == n);
  long long found = 0;
  int located = 0;
  std::vector<long long> at(cap);  // stream position -> entry
  for (int c = 0; c < K; ++c) {
    for (int ch = L.color_chunk_ptr[c]; ch < L.color_chunk_ptr[c + 1]; ++ch) {
      const long long base = (long long)ch * cap;  // the kernel's closed form
      std::fill(at.begin(), at.end(), -1);
      int prev_row = -1;
      for (int k = 0; k < cap; ++k) {
        const long long e = base + k;
        const int f = L.ent_pos[e];
        REQUIRE(f < cap && at[f] < 0);  // a permutation of the stream
        at[f] = e;
        const int row = L.ent_pk[e] & kPadRow;
        REQUIRE(row > prev_row || row == kPadRow);  // sorted by row, padding last
        if (row != kPadRow) prev_row = row;
      }
      REQUIRE(L.chunk_first[ch] >= L.color_loc_ptr[c] && L.chunk_first[ch + 1] <= L.color_loc_ptr[c + 1]);
      const int nsl = L.chunk_first[ch + 1] - L.chunk_first[ch];
      REQUIRE(nsl >= 1 && nsl <= 2 * LW - 1);
      int f = 0;
      for (int q = 0; q < nsl; ++q) {
        const int x = L.chunk_first[ch] + q;
        const int i = L.compact_loc[x];
        ++located;
        REQUIRE(col[i] == c + 1);
        REQUIRE(L.slot_f0[x] == f);
        const int len = L.collen[x];
        REQUIRE(len == (int)want[i].size());
        for (int t = 0; t < len; ++t, ++f) {
          const long long e = at[f];
          const int pk = L.ent_pk[e];
          REQUIRE((int)((unsigned)pk >> kRowBits) == q);
          REQUIRE(want[i].count({pk & kPadRow, L.ent_src[e]}) == 1);
          ++found;
        }
      }
      REQUIRE(f <= cap);
      // start mask: exactly the slot starts (and the padding tail start)
      for (int g = 0; g < cap; ++g) {
        bool start = (g == f && f < cap);
        for (int q2 = 0; q2 < nsl; ++q2) start = start || (L.slot_f0[L.chunk_first[ch] + q2] == g);
        const bool bit = (L.start_mask[(size_t)ch * LW + g / kRowsMax] >> (g % kRowsMax)) & 1;
        REQUIRE(bit == start);
      }
      for (int g = f; g < cap; ++g) {  // padding tail of the stream
        const long long e = at[g];
        REQUIRE((L.ent_pk[e] & kPadRow) == kPadRow && (int)((unsigned)L.ent_pk[e] >> kRowBits) == dummy);
        REQUIRE(L.ent_src[e] == -1);
      }
    }
  }
  REQUIRE(found == nnz);
  REQUIRE(located == n);
  std::printf("ok K=%d nnz=%lld entries=%lld chunks=%d max_collen=%d\n", K, nnz, L.n_entries, L.nchunks,
              L.max_collen);
  return 0;
}
