// CPU emulation of the tile-resident sweep (kernels.hip sweep_tiles_kernel)
// on the tile layout of graph_prep.cpp, against a plain serial local-form
// chromatic sweep (update_Gaussian.R:257-275 restated: acc_i = sum_k B[k,i]
// (B w)_k - D_i w_i, colours in order).  The emulation follows the kernel
// step by step -- per (sweep, colour): every tile's own batches (thread runs,
// tails, slot totals, draws, LDS scatter), then every tile's ghost cells from
// the published dw -- with each tile's r in its own local-row array, so it
// checks the layout (local rows, batches, stream positions, start/end flags,
// ghost cells, exported flags, neighbour lists) and the algorithm together.
// With G > 1 (a tile shard): the tiles of rank g = [g*T/G, (g+1)*T/G), one
// granule buffer per rank, poisoned (NaN) before each colour: a draw reaches
// a reader of another rank only through the remote puts of the plan (rmask),
// which must be exactly the set of reader ranks; rank slot ranges checked.
// With SPLIT = 1 (the 3+-chain kernel's schedule): per phase, every tile's
// interior batches of colour c, then the ghost cells of colour c-1 (their
// hand-off), then the boundary batches of c -- an interior slot must not read
// a row still missing its colour-(c-1) ghost update.
// With WAVES > 0 (NT = 64): wave-local batches (one wave's each, rounds of
// WAVES per colour, tiles.hip tile_phase_wl); the batches of a colour touch
// disjoint rows, so emulating them one after another is the kernel's result.
// Usage: tile_sweep_check <n> <m> <tiles> <chains> <seed> [NT RMAX G SPLIT SWEEPS WAVES]  (prints "ok <stats>")
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <set>
#include <string>
#include <vector>

#include "graph_prep.h"

using namespace nngp;

#define REQUIRE(c)                                            \
  do {                                                        \
    if (!(c)) {                                               \
      std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
      return 1;                                               \
    }                                                         \
  } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 4000;
  const int m = argc > 2 ? std::atoi(argv[2]) : 10;
  const int T = argc > 3 ? std::atoi(argv[3]) : 16;
  const int C = argc > 4 ? std::atoi(argv[4]) : 2;
  const int seed = argc > 5 ? std::atoi(argv[5]) : 1;
  const int NT = argc > 6 ? std::atoi(argv[6]) : 256;
  const int RMAX = argc > 7 ? std::atoi(argv[7]) : 16;
  const int G = argc > 8 ? std::atoi(argv[8]) : 1;
  const bool SPLIT = argc > 9 && std::atoi(argv[9]) != 0;
  const int sweeps = argc > 10 ? std::atoi(argv[10]) : 3;
  const int WAVES = argc > 11 ? std::atoi(argv[11]) : 0;  // wave-local batches (NT = 64) in rounds of WAVES
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
  const int K = greedy_coloring(nn.data(), n, b, col);
  TileLayout L;
  std::string err;
  if (!build_tile_layout(nn.data(), n, b, col.data(), locs.data(), d, T, NT, RMAX, L, err, G, SPLIT, WAVES)) {
    std::printf("FAIL build: %s\n", err.c_str());
    return 1;
  }
  REQUIRE(L.K == K && L.T == std::min(T, n));
  // per-chain B values (device layout: row rpos[k], position u), D, R, n_i, w, z
  std::vector<std::vector<double>> linv(C, std::vector<double>((size_t)n * b, 0.0));
  for (int ch = 0; ch < C; ++ch)
    for (int k = 0; k < n; ++k)
      for (int u = 0; u < b; ++u)
        if (nn[(size_t)k * b + u] >= 0) linv[ch][(size_t)L.rpos[k] * b + u] = u == 0 ? 1.0 + U(g) : 0.3 * N01(g);
  std::vector<int> nobs(n);
  for (auto& v : nobs) v = (int)(U(g) * 3);
  std::vector<std::vector<double>> Dg(C, std::vector<double>(n, 0.0)), Rs(C, std::vector<double>(n)),
      w0(C, std::vector<double>(n));
  for (int ch = 0; ch < C; ++ch) {
    for (int k = 0; k < n; ++k)
      for (int u = 0; u < b; ++u) {
        const int j = nn[(size_t)k * b + u];
        if (j >= 0) Dg[ch][j] += linv[ch][(size_t)L.rpos[k] * b + u] * linv[ch][(size_t)L.rpos[k] * b + u];
      }
    for (int i = 0; i < n; ++i) { Rs[ch][i] = N01(g); w0[ch][i] = N01(g); }
  }
  std::vector<double> z((size_t)sweeps * n * C);  // per sweep, loc x C
  for (auto& v : z) v = N01(g);
  const double inv_s2[4] = {0.7, 1.3, 0.9, 1.1}, inv_t2[4] = {2.0, 0.5, 1.0, 4.0};
  // ---- reference: serial local-form sweep in colour order
  std::vector<std::vector<std::pair<int, int>>> colB(n);  // column i -> (row k, position u)
  for (int k = 0; k < n; ++k)
    for (int u = 0; u < b; ++u)
      if (nn[(size_t)k * b + u] >= 0) colB[nn[(size_t)k * b + u]].push_back({k, u});
  std::vector<std::vector<double>> wr = w0;
  for (int ch = 0; ch < C; ++ch)
    for (int s = 0; s < sweeps; ++s) {
      std::vector<double> r(n, 0.0);  // r_k = (B w)_k
      for (int k = 0; k < n; ++k)
        for (int u = 0; u < b; ++u) {
          const int j = nn[(size_t)k * b + u];
          if (j >= 0) r[k] += linv[ch][(size_t)L.rpos[k] * b + u] * wr[ch][j];
        }
      for (int c = 1; c <= K; ++c) {
        std::vector<double> dw(n, 0.0);
        for (int i = 0; i < n; ++i) {
          if (col[i] != c) continue;
          double acc = 0.0;
          for (const auto& ku : colB[i]) acc += linv[ch][(size_t)L.rpos[ku.first] * b + ku.second] * r[ku.first];
          acc -= Dg[ch][i] * wr[ch][i];
          const double P = Dg[ch][i] * inv_s2[ch] + nobs[i] * inv_t2[ch];
          const double wn = (Rs[ch][i] * inv_t2[ch] - acc * inv_s2[ch]) / P + z[((size_t)s * n + i) * C + ch] / std::sqrt(P);
          dw[i] = wn - wr[ch][i];
          wr[ch][i] = wn;
        }
        for (int k = 0; k < n; ++k)
          for (int u = 0; u < b; ++u) {
            const int j = nn[(size_t)k * b + u];
            if (j >= 0 && col[j] == c) r[k] += linv[ch][(size_t)L.rpos[k] * b + u] * dw[j];
          }
      }
    }
  // ---- emulation of the kernel on the tile layout
  const size_t ncell = L.cell_pk.size(), ng = L.gsrc.size();
  std::vector<double> cval((size_t)C * ncell, 0.0), gval((size_t)C * ng);
  for (int ch = 0; ch < C; ++ch) {
    for (size_t e = 0; e < ncell; ++e) cval[ch * ncell + e] = L.cell_src[e] >= 0 ? linv[ch][L.cell_src[e]] : 0.0;
    for (size_t q = 0; q < ng; ++q) gval[ch * ng + q] = linv[ch][L.gsrc[q]];
  }
  // slot data
  std::vector<double> w((size_t)n * C), dwx((size_t)n * C, 0.0);
  for (int x = 0; x < n; ++x)
    for (int ch = 0; ch < C; ++ch) w[(size_t)x * C + ch] = w0[ch][L.compact_loc[x]];
  // each tile's local r
  std::vector<std::vector<double>> rt(L.T);
  auto init_r = [&]() {
    std::vector<double> rg((size_t)n * C, 0.0);  // by device row
    for (int ch = 0; ch < C; ++ch)
      for (int k = 0; k < n; ++k)
        for (int u = 0; u < b; ++u) {
          const int j = nn[(size_t)k * b + u];
          if (j < 0) continue;
          // w of loc j: find its slot
          rg[(size_t)L.rpos[k] * C + ch] += linv[ch][(size_t)L.rpos[k] * b + u] * 0.0;
        }
    return rg;
  };
  (void)init_r;
  std::vector<int> slot_of(n);
  for (int x = 0; x < n; ++x) slot_of[L.compact_loc[x]] = x;
  std::vector<int> perm(n);
  for (int i = 0; i < n; ++i) perm[L.rpos[i]] = i;
  // checks of the layout itself
  {
    long long own_cells = 0;
    for (size_t e = 0; e < ncell; ++e) own_cells += (L.cell_pk[e] & kTilePadRow) != kTilePadRow;
    REQUIRE(own_cells == L.nnz);
    for (int t = 0; t < L.T; ++t) {
      // every local row distinct, own rows first
      std::set<int> seen(L.erow.begin() + L.erow_ptr[t], L.erow.begin() + L.erow_ptr[t + 1]);
      REQUIRE((int)seen.size() == L.erow_ptr[t + 1] - L.erow_ptr[t]);
      for (int r = L.tile_row0[t]; r < L.tile_row0[t + 1]; ++r) REQUIRE(L.erow[L.erow_ptr[t] + r - L.tile_row0[t]] == r);
    }
    // tile shard: rank slot ranges = the slots of the rank's tiles; rmask = the
    // ranks (other than the owner's) of the tiles with a ghost cell of the slot
    REQUIRE(L.G == G && (int)L.rank_slot0.size() == G + 1 && L.rank_slot0[0] == 0 && L.rank_slot0[G] == n);
    const int Tl = L.T / G;
    for (int t = 0; t < L.T; ++t)
      for (int bi = L.batch_ptr[(size_t)t * K]; bi < L.batch_ptr[(size_t)t * K + K]; ++bi) {
        const TileBatch B = L.batch[bi];
        REQUIRE(B.slot0 >= L.rank_slot0[t / Tl] && B.slot0 + B.nslots <= L.rank_slot0[t / Tl + 1]);
      }
    // a tile's batches, in order, cover one contiguous slot range with no gap
    // (the kernel's beta_0-shift pass over [first batch's slot0, last batch's
    // end), tiles.hip prologue), and the tiles' ranges partition the slots
    {
      int next = 0;
      for (int t = 0; t < L.T; ++t) {
        const int b0 = L.batch_ptr[(size_t)t * K], b1 = L.batch_ptr[(size_t)t * K + K];
        if (b0 == b1) continue;
        REQUIRE(L.batch[b0].slot0 == next);
        for (int bi = b0; bi < b1; ++bi) {
          REQUIRE(L.batch[bi].slot0 == next);
          next += L.batch[bi].nslots;
        }
      }
      REQUIRE(next == n);
    }
    if (G > 1) {
      std::vector<uint32_t> want(n, 0u);
      for (int t = 0; t < L.T; ++t)
        for (int pc = t * K; pc < t * K + K; ++pc)
          for (int q = L.gslot_ptr[pc]; q < L.gslot_ptr[pc + 1]; ++q) {
            const int x = L.gslot[q];
            int ro = 0;
            while (L.rank_slot0[ro + 1] <= x) ++ro;
            if (ro != t / Tl) want[x] |= 1u << (t / Tl);
          }
      REQUIRE(L.rmask == want);
    }
  }
  const int Tl = L.T / G;
  std::vector<std::vector<double>> gbuf(G, std::vector<double>((size_t)n * C, 0.0));  // per-rank granule buffers
  long long remote_puts = 0;
  std::vector<double> f0s(NT);
  long long ghosts_applied = 0;
  for (int s = 0; s < sweeps; ++s) {
    // call start (kernel prologue): r of every local row from w (= B w);
    // later sweeps of the call continue from the maintained local r
    for (int t = 0; t < L.T && s == 0; ++t) {
      const int nr = L.erow_ptr[t + 1] - L.erow_ptr[t];
      rt[t].assign((size_t)nr * C, 0.0);
      for (int lr = 0; lr < nr; ++lr) {
        const int k = perm[L.erow[L.erow_ptr[t] + lr]];
        for (int ch = 0; ch < C; ++ch) {
          double acc = 0.0;
          for (int u = 0; u < b; ++u) {
            const int j = nn[(size_t)k * b + u];
            if (j >= 0) acc += linv[ch][(size_t)L.rpos[k] * b + u] * w[(size_t)slot_of[j] * C + ch];
          }
          rt[t][(size_t)lr * C + ch] = acc;
        }
      }
    }
    auto own = [&](int t, int c, int bi_lo, int bi_hi) -> int {
        std::vector<double>& r_s = rt[t];
        for (int bi = bi_lo; bi < bi_hi; ++bi) {
          const TileBatch B = L.batch[bi];
          REQUIRE(B.nslots <= NT && B.R <= RMAX);
          REQUIRE(WAVES == 0 || B.nslots <= kWaveSlotsMax);
          // threads past nthr hold padding only (the kernel skips their loads)
          REQUIRE(B.nthr >= 1 && B.nthr <= NT);
          for (int j = 0; j < B.R; ++j)
            for (int th = B.nthr; th < NT; ++th) REQUIRE(L.cell_pk[(size_t)B.off + (size_t)j * NT + th] == kTilePadRow);
          std::vector<double> pr((size_t)NT * RMAX * C), tails((size_t)NT * C), acc_s((size_t)NT * C, 0.0);
          std::vector<int> f0(NT, 0);
          for (int th = 0; th < B.nslots; ++th) f0[th] = L.slot_f0[B.slot0 + th] & 0xFFFFF;
          for (int th = 0; th < NT; ++th) {
            std::vector<double> run(C, 0.0);
            for (int j = 0; j < B.R; ++j) {
              const size_t e = (size_t)B.off + (size_t)j * NT + th;
              const uint32_t pk = L.cell_pk[e], lr = pk & kTilePadRow;
              for (int ch = 0; ch < C; ++ch) {
                const double p = lr != kTilePadRow ? cval[ch * ncell + e] * r_s[(size_t)lr * C + ch] : 0.0;
                run[ch] = (pk & kCellStart) ? p : run[ch] + p;
                pr[((size_t)th * RMAX + j) * C + ch] = run[ch];
              }
            }
            for (int ch = 0; ch < C; ++ch) tails[(size_t)th * C + ch] = run[ch];
          }
          std::vector<int> done(B.nslots, 0);
          for (int th = 0; th < NT; ++th)
            for (int j = 0; j < B.R; ++j) {
              const size_t e = (size_t)B.off + (size_t)j * NT + th;
              const uint32_t pk = L.cell_pk[e];
              if (!(pk & kCellEnd)) continue;
              const int q = (int)((pk >> kTileQShift) & kTileQMask);
              REQUIRE(q < B.nslots);
              done[q]++;
              const int t0 = f0[q] / B.R;
              REQUIRE(t0 <= th);
              for (int ch = 0; ch < C; ++ch) {
                double acc = 0.0;
                for (int tt = t0; tt < th; ++tt) acc += tails[(size_t)tt * C + ch];
                acc_s[(size_t)q * C + ch] = acc + pr[((size_t)th * RMAX + j) * C + ch];
              }
            }
          for (int q = 0; q < B.nslots; ++q) REQUIRE(done[q] == 1);
          for (int q = 0; q < B.nslots; ++q) {
            const int x = B.slot0 + q, i = L.compact_loc[x];
            REQUIRE(col[i] == c + 1);
            for (int ch = 0; ch < C; ++ch) {
              const double wv = w[(size_t)x * C + ch];
              const double P = Dg[ch][i] * inv_s2[ch] + nobs[i] * inv_t2[ch];
              const double cR = inv_t2[ch] * Rs[ch][i] + inv_s2[ch] * (Dg[ch][i] * wv);
              const double wn = (cR - inv_s2[ch] * acc_s[(size_t)q * C + ch]) / P +
                                z[((size_t)s * n + i) * C + ch] / std::sqrt(P);
              const double dw = wn - wv;
              w[(size_t)x * C + ch] = wn;
              acc_s[(size_t)q * C + ch] = dw;
              if (L.slot_f0[x] & kSlotExported) {
                dwx[(size_t)x * C + ch] = dw;
                gbuf[t / Tl][(size_t)x * C + ch] = dw;  // own rank's buffer
                for (int h = 0; h < G; ++h)
                  if (G > 1 && ((L.rmask[x] >> h) & 1u)) {
                    gbuf[h][(size_t)x * C + ch] = dw;  // remote put
                    ++remote_puts;
                  }
              }
            }
          }
          for (size_t e = B.off; e < (size_t)B.off + (size_t)B.R * NT; ++e) {
            const uint32_t pk = L.cell_pk[e], lr = pk & kTilePadRow;
            if (lr == kTilePadRow) continue;
            const int q = (int)((pk >> kTileQShift) & kTileQMask);
            for (int ch = 0; ch < C; ++ch) r_s[(size_t)lr * C + ch] += cval[ch * ncell + e] * acc_s[(size_t)q * C + ch];
          }
        }
        return 0;
    };
    auto ghosts = [&](int t, int c) -> int {
        const int pc = t * K + c;
        std::set<int> nbs(L.nb.begin() + L.nb_ptr[pc], L.nb.begin() + L.nb_ptr[pc + 1]);
        for (int gi = L.gptr[pc]; gi < L.gptr[pc + 1]; ++gi) {
          const int lr = L.gcell[2 * gi], gx = L.gcell[2 * gi + 1];
          REQUIRE(gx >= 0 && gx < L.gslot_ptr[pc + 1] - L.gslot_ptr[pc] && gx < L.max_gslots);
          const int x = L.gslot[L.gslot_ptr[pc] + gx];
          REQUIRE(L.slot_f0[x] & kSlotExported);
          REQUIRE(col[L.compact_loc[x]] == c + 1);
          // the owner of x is a listed neighbour
          const int row = L.rpos[L.compact_loc[x]];
          int owner = 0;
          while (L.tile_row0[owner + 1] <= row) ++owner;
          REQUIRE(owner != t && nbs.count(owner));
          for (int ch = 0; ch < C; ++ch) {
            const double dwv = gbuf[t / Tl][(size_t)x * C + ch];  // the reader polls its own rank's buffer
            REQUIRE(!std::isnan(dwv) && dwv == dwx[(size_t)x * C + ch]);
            rt[t][(size_t)lr * C + ch] += gval[ch * ng + gi] * dwv;
          }
          ++ghosts_applied;
        }
        return 0;
    };
    for (int c = 0; c < K; ++c) {
      // the granules of colour c are rewritten in this phase: poison them
      for (int x = 0; x < n; ++x)
        if (col[L.compact_loc[x]] == c + 1)
          for (auto& gb : gbuf)
            for (int ch = 0; ch < C; ++ch) gb[(size_t)x * C + ch] = std::nan("");
      if (!SPLIT) {
        for (int t = 0; t < L.T; ++t)
          if (own(t, c, L.batch_ptr[t * K + c], L.batch_ptr[t * K + c + 1])) return 1;
        for (int t = 0; t < L.T; ++t)
          if (ghosts(t, c)) return 1;
      } else {
        // interior batches, the hand-off of the previous colour, boundary batches
        REQUIRE(L.split && L.batch_split.size() == (size_t)L.T * K);
        for (int t = 0; t < L.T; ++t)
          if (own(t, c, L.batch_ptr[t * K + c], L.batch_split[t * K + c])) return 1;
        if (s > 0 || c > 0)
          for (int t = 0; t < L.T; ++t)
            if (ghosts(t, (c + K - 1) % K)) return 1;
        for (int t = 0; t < L.T; ++t)
          if (own(t, c, L.batch_split[t * K + c], L.batch_ptr[t * K + c + 1])) return 1;
      }
    }
  }
  double maxrel = 0.0;
  for (int ch = 0; ch < C; ++ch)
    for (int i = 0; i < n; ++i) {
      const double a = w[(size_t)slot_of[i] * C + ch], r = wr[ch][i];
      maxrel = std::max(maxrel, std::fabs(a - r) / std::max(1.0, std::fabs(r)));
    }
  if (!(maxrel < 1e-11)) { std::printf("FAIL maxrel %.3e\n", maxrel); return 1; }
  // FNV hash of every layout array (the layout must not depend on the host thread count)
  unsigned long long lh = 1469598103934665603ULL;
  auto mix = [&](const void* p, size_t bytes) {
    for (size_t i = 0; i < bytes; ++i) lh = (lh ^ ((const unsigned char*)p)[i]) * 1099511628211ULL;
  };
  auto mixv = [&](const auto& v) { mix(v.data(), v.size() * sizeof(v[0])); };
  mixv(L.rpos); mixv(L.compact_loc); mixv(L.slot_f0); mixv(L.erow_ptr); mixv(L.erow); mixv(L.batch_ptr);
  mixv(L.cell_pk); mixv(L.cell_src); mixv(L.gcell); mixv(L.gsrc); mixv(L.gptr); mixv(L.gslot); mixv(L.gslot_ptr);
  mixv(L.nb_ptr); mixv(L.nb); mixv(L.rmask); mixv(L.batch_split);
  for (const TileBatch& tb : L.batch) mix(&tb, sizeof tb);
  // dynamic LDS of one 512-thread workgroup (exchange-wave tiles) at 1..4
  // chains with r in LDS, and with r in global memory (RG tiles)
  int lds[5], lds_rg[5];
  for (int c = 1; c <= 4; ++c) {
    lds[c] = tile_lds_bytes(L.max_rows, c, 512, K, L.max_batches, L.max_gslots);
    lds_rg[c] = tile_lds_bytes(0, c, 512, K, L.max_batches, L.max_gslots);
  }
  std::printf("ok K=%d T=%d G=%d max_rows=%d batches=%zu cells=%zu ghosts=%zu nb=%zu remote_puts=%lld maxrel=%.2e "
              "layout=%016llx lds=%d,%d,%d,%d lds_rg=%d,%d,%d,%d cu_lds=%d\n", K, L.T, G, L.max_rows, L.batch.size(),
              ncell, ng, L.nb.size(), remote_puts, maxrel, lh, lds[1], lds[2], lds[3], lds[4], lds_rg[1], lds_rg[2],
              lds_rg[3], lds_rg[4], kTileCuLds);
  return 0;
}
