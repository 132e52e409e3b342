// Tile-layout statistics (diagnostic): per colour, the rows per thread R of
// each tile's own batch (mean, max over the tile's neighbourhood, max), ghost
// cells and foreign slots, at the bench workload.  Build (host only):
//   g++ -O3 -std=c++17 -I<pkg>/csrc scripts/layout_stats.cpp <pkg>/csrc/graph_prep.cpp -o /tmp/layout_stats
// usage: layout_stats [n] [m] [tiles] [cell threads] [RMAX]
#include "graph_prep.h"
#include <cstdio>
#include <random>
#include <algorithm>
#include <cmath>
using namespace nngp;
int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 1000000, m = argc > 2 ? atoi(argv[2]) : 15;
  int T = argc > 3 ? atoi(argv[3]) : 256, NT = argc > 4 ? atoi(argv[4]) : 448, RMAX = argc > 5 ? atoi(argv[5]) : 8;
  const int WAVES = argc > 6 ? atoi(argv[6]) : 0;  // wave-local batches (NT = 64)
  std::mt19937_64 g(1000); std::uniform_real_distribution<double> U(0, 1);
  std::vector<double> xy(2 * (size_t)n);
  for (auto& v : xy) v = U(g);
  std::vector<int> ord; order_maxmin(xy.data(), n, 2, ord);
  std::vector<double> lo(2 * (size_t)n);
  for (int i = 0; i < n; ++i) { lo[i] = xy[ord[i]]; lo[n + i] = xy[n + ord[i]]; }
  std::vector<int> nn; find_ordered_nn(lo.data(), n, 2, m, nn);
  std::vector<int> col; int K = greedy_coloring(nn.data(), n, m + 1, col);
  printf("K=%d\n", K);
  std::vector<int> csz(K); for (int c : col) csz[c - 1]++;
  for (int c = 0; c < K; ++c) printf("%d ", csz[c]); printf("\n");
  TileLayout L; std::string err;
  if (!build_tile_layout(nn.data(), n, m + 1, col.data(), lo.data(), 2, T, NT, RMAX, L, err, 1, false, WAVES)) { printf("err %s\n", err.c_str()); return 1; }
  {
    std::vector<int> lr(T);
    for (int t = 0; t < T; ++t) lr[t] = L.erow_ptr[t + 1] - L.erow_ptr[t];
    std::vector<int> srt = lr; std::sort(srt.begin(), srt.end());
    double mean = 0; for (int v : lr) mean += v; mean /= T;
    int own_max = 0; for (int t = 0; t < T; ++t) own_max = std::max(own_max, L.tile_row0[t + 1] - L.tile_row0[t]);
    printf("local rows per tile: mean %.0f p50 %d p90 %d max %d (own rows max %d)\n", mean, srt[T / 2], srt[T * 9 / 10],
           srt[T - 1], own_max);
  }
  printf("max_rows %d max_batches %d max_gslots %d cells %zu (nnz %lld, x%.3f) batches %zu\n", L.max_rows, L.max_batches,
         L.max_gslots, L.cell_pk.size(), L.nnz, (double)L.cell_pk.size() / L.nnz, L.batch.size());
  // per (tile, colour): cells, R, ghost cells, foreign slots
  long sumR = 0, sumRmaxNb = 0; 
  std::vector<int> Rtc((size_t)T * K, 0), ctc((size_t)T*K,0);
  for (int t = 0; t < T; ++t) for (int c = 0; c < K; ++c) {
    int R = 0, cells = 0;
    for (int q = L.batch_ptr[t*K+c]; q < L.batch_ptr[t*K+c+1]; ++q) { R += L.batch[q].R; cells += L.batch[q].nthr; }
    Rtc[t*K+c] = R;
    if (WAVES > 0) {  // wave-local: the critical R = sum over rounds of the round's max R
      const int b0 = L.batch_ptr[t*K+c], b1 = L.batch_ptr[t*K+c+1];
      int crit = 0;
      for (int r0 = b0; r0 < b1; r0 += WAVES) {
        int rm = 0;
        for (int q = r0; q < std::min(b1, r0 + WAVES); ++q) rm = std::max(rm, L.batch[q].R);
        crit += rm;
      }
      Rtc[t*K+c] = crit;
      ctc[t*K+c] = (b1 - b0 + WAVES - 1) / WAVES;  // rounds
    }
  }
  if (WAVES > 0)
    for (int c = 0; c < K; ++c) {
      int r1 = 0, r2 = 0, r3 = 0;
      for (int t = 0; t < T; ++t) { const int r = ctc[t*K+c]; r1 += r == 1; r2 += r == 2; r3 += r >= 3; }
      if (r2 + r3) printf("c%2d tiles with 1 / 2 / 3+ wave rounds: %d / %d / %d\n", c, r1, r2, r3);
    }
  // per colour: mean R, max R, mean over tiles of max R over neighbours
  double tot_mean = 0, tot_nbmax = 0, tot_max = 0, gh = 0, fs = 0;
  for (int c = 0; c < K; ++c) {
    double mean = 0; int mx = 0; double nbm = 0; double gm = 0, fm = 0; int gmx = 0;
    for (int t = 0; t < T; ++t) {
      int R = Rtc[t*K+c]; mean += R; mx = std::max(mx, R);
      int m2 = R;
      for (int e = L.nb_ptr[t*K+c]; e < L.nb_ptr[t*K+c+1]; ++e) m2 = std::max(m2, Rtc[L.nb[e]*K+c]);
      nbm += m2;
      int ng = L.gptr[t*K+c+1]-L.gptr[t*K+c]; gm += ng; gmx = std::max(gmx, ng);
      fm += L.gslot_ptr[t*K+c+1]-L.gslot_ptr[t*K+c];
    }
    printf("c%2d R mean %.2f nbmax %.2f max %d | ghost mean %.0f max %d | fslots mean %.0f\n", c, mean/T, nbm/T, mx, gm/T, gmx, fm/T);
    tot_mean += mean/T; tot_nbmax += nbm/T; tot_max += mx; gh += gm/T; fs += fm/T;
  }
  printf("sum over colours: R mean %.1f nbmax %.1f max %.1f ghost %.0f fslots %.0f\n", tot_mean, tot_nbmax, tot_max, gh, fs);
  long exported = 0; for (int x = 0; x < n; ++x) if (L.slot_f0[x] & kSlotExported) exported++;
  printf("exported slots %ld (%.1f%%)\n", exported, 100.0*exported/n);
  // HBM bytes per sweep by stream at C chains (what the kernel loads and
  // stores; DESIGN.md §3 "traffic budget"), against SURVEY §8d's algorithmic
  // C*(8*nnz + 40*n) + 4*nnz
  const int C = argc > 7 ? atoi(argv[7]) : 3;
  long long live = 0;  // cells the kernel loads: rows < R of threads < nthr
  for (const TileBatch& tb : L.batch) live += (long long)tb.R * tb.nthr;
  const double MB = 1e6;
  const double cells = live * (4.0 + 8.0 * C), ghosts = (double)L.gsrc.size() * (8.0 + 8.0 * C);
  const double recs = (double)n * (8 + 4 + C * (16 + 8 + 8));  // sinfo, loc, dr, w read, w write
  long long fsl = (long long)L.gslot.size();
  const double gran = (double)exported * C * 16 + (double)fsl * C * 16 + (double)fsl * 4;  // stores, polls, indices
  const double alg = C * (8.0 * L.nnz + 40.0 * n) + 4.0 * L.nnz;
  printf("per sweep at C=%d (MB): cells %.1f (padding %.1f) ghosts %.1f records %.1f granules %.1f | total %.1f "
         "algorithmic %.1f ratio %.3f\n", C, cells / MB, (live - L.nnz) * (4.0 + 8.0 * C) / MB, ghosts / MB, recs / MB,
         gran / MB, (cells + ghosts + recs + gran) / MB, alg / MB, (cells + ghosts + recs + gran) / alg);
}
