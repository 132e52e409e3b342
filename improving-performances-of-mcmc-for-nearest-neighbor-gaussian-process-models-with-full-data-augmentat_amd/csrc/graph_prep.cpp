// Host-side init-time graph preparation (C++).
//
// Replaces, with the same semantics and bit-exact outputs given the ordering:
//   GpGp::find_ordered_nn ........ Scripts/mcmc_nngp_initialize.R:93
//   moral graph + colouring ...... Scripts/mcmc_nngp_initialize.R:97-110,
//                                  Scripts/Coloring.R:2-20
//   GpGp::order_maxmin ........... Scripts/mcmc_nngp_initialize.R:29 (exact
//                                  max-min; GpGp's is approximate+jittered)
// and plans the HBM layout of the chromatic sweep (DESIGN.md "Layout").
//
// Squared distances are accumulated in coordinate order as
// t = x_query - x_other; s += t*t (compiled with -ffp-contract=off) so ties
// and orderings are reproducible bit-for-bit.
#include "graph_prep.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <numeric>
#include <thread>

namespace nngp {
namespace {

inline double sqdist(const double* locs, int n, int d, int a, int b) {
  double s = 0.0;
  for (int k = 0; k < d; ++k) {
    double t = locs[a + (size_t)k * n] - locs[b + (size_t)k * n];
    s += t * t;
  }
  return s;
}

// Uniform grid over the first dg = min(d,3) coordinates of points [0, P).
struct Grid {
  int dg = 1;
  double lo[3] = {0, 0, 0};
  double cs = 1.0;
  long long nc[3] = {1, 1, 1};
  std::vector<int> start;  // ncells + 1
  std::vector<int> pts;    // point ids grouped by cell, ascending inside a cell

  long long ncells() const { return nc[0] * nc[1] * nc[2]; }

  long long coord(double x, int k) const {
    long long c = (long long)std::floor((x - lo[k]) / cs);
    if (c < 0) c = 0;
    if (c >= nc[k]) c = nc[k] - 1;
    return c;
  }
  long long cell_of(const double* locs, int n, int i, long long* cc) const {
    long long id = 0;
    for (int k = 2; k >= 0; --k) {
      cc[k] = (k < dg) ? coord(locs[i + (size_t)k * n], k) : 0;
      id = id * nc[k] + cc[k];
    }
    return id;
  }
  long long id_of(const long long* cc) const { return (cc[2] * nc[1] + cc[1]) * nc[0] + cc[0]; }

  void build(const double* locs, int n, int d, int P, double pts_per_cell) {
    dg = std::min(d, 3);
    double hi[3];
    for (int k = 0; k < 3; ++k) { lo[k] = 0; hi[k] = 0; nc[k] = 1; }
    for (int k = 0; k < dg; ++k) {
      double a = std::numeric_limits<double>::infinity(), b = -a;
      for (int i = 0; i < n; ++i) {  // bounding box of ALL points: stable across prefixes
        double x = locs[i + (size_t)k * n];
        a = std::min(a, x); b = std::max(b, x);
      }
      lo[k] = a; hi[k] = b;
    }
    double target = std::max(1.0, P / pts_per_cell);
    double ext[3];
    double maxext = 0;
    for (int k = 0; k < dg; ++k) { ext[k] = hi[k] - lo[k]; maxext = std::max(maxext, ext[k]); }
    if (!(maxext > 0)) maxext = 1.0;
    // choose cs so that prod ceil(ext/cs) ~ target (bisection on cs)
    double a = maxext / target, b = maxext * 1.0000001;
    if (a <= 0) a = maxext * 1e-9;
    for (int it = 0; it < 60; ++it) {
      double mid = std::sqrt(a * b);
      double cells = 1;
      for (int k = 0; k < dg; ++k) cells *= std::max(1.0, std::ceil(ext[k] / mid));
      if (cells > target) a = mid; else b = mid;
    }
    cs = b;
    for (int k = 0; k < dg; ++k) nc[k] = std::max(1LL, (long long)std::ceil(ext[k] / cs));
    long long C = ncells();
    start.assign(C + 1, 0);
    pts.resize(P);
    std::vector<long long> cid(P);
    long long cc[3];
    for (int i = 0; i < P; ++i) { cid[i] = cell_of(locs, n, i, cc); start[cid[i] + 1]++; }
    for (long long c = 0; c < C; ++c) start[c + 1] += start[c];
    std::vector<int> fill(start.begin(), start.end() - 1);
    for (int i = 0; i < P; ++i) pts[fill[cid[i]]++] = i;
  }
};

struct Cand {
  double s;
  int j;
};
inline bool lex_less(double s1, int j1, double s2, int j2) { return s1 < s2 || (s1 == s2 && j1 < j2); }

struct TopM {
  int m, cnt = 0;
  Cand* c;
  void reset() { cnt = 0; }
  void offer(double s, int j) {
    if (cnt == m && !lex_less(s, j, c[cnt - 1].s, c[cnt - 1].j)) return;
    int p = cnt < m ? cnt++ : cnt - 1;
    while (p > 0 && lex_less(s, j, c[p - 1].s, c[p - 1].j)) { c[p] = c[p - 1]; --p; }
    c[p].s = s; c[p].j = j;
  }
  double worst() const { return c[cnt - 1].s; }
};

// host threads for the embarrassingly parallel init loops (NNGP_HOST_THREADS
// overrides; results never depend on the count)
int host_threads() {
  if (const char* e = std::getenv("NNGP_HOST_THREADS")) return std::max(1, std::atoi(e));
  unsigned h = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(h, 32u));
}

// f(t, lo, hi) over [0, n) split into contiguous chunks, one per thread
template <class F>
void parallel_chunks(long long n, F f) {
  const int T = (int)std::min<long long>(host_threads(), std::max(1LL, n / 4096));
  if (T <= 1) { f(0, 0LL, n); return; }
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    const long long lo = n * t / T, hi = n * (t + 1) / T;
    th.emplace_back([=, &f] { f(t, lo, hi); });
  }
  for (auto& x : th) x.join();
}

}  // namespace

void morton_keys(const double* locs, int n, int d, std::vector<uint64_t>& keys) {
  int dg = std::min(d, 3);
  double lo[3] = {0, 0, 0}, hi[3] = {1, 1, 1};
  for (int k = 0; k < dg; ++k) {
    double a = std::numeric_limits<double>::infinity(), b = -a;
    for (int i = 0; i < n; ++i) { double x = locs[i + (size_t)k * n]; a = std::min(a, x); b = std::max(b, x); }
    lo[k] = a; hi[k] = (b > a) ? b : a + 1.0;
  }
  const int bits = dg == 1 ? 63 : (dg == 2 ? 31 : 21);
  const double scale = (double)((1ULL << bits) - 1);
  keys.resize(n);
  for (int i = 0; i < n; ++i) {
    uint64_t q[3] = {0, 0, 0};
    for (int k = 0; k < dg; ++k) {
      double u = (locs[i + (size_t)k * n] - lo[k]) / (hi[k] - lo[k]);
      u = std::min(1.0, std::max(0.0, u));
      q[k] = (uint64_t)(u * scale);
    }
    uint64_t key = 0;
    for (int bit = bits - 1; bit >= 0; --bit)
      for (int k = dg - 1; k >= 0; --k) key = (key << 1) | ((q[k] >> bit) & 1ULL);
    keys[i] = key;
  }
}

// Hilbert-curve keys (d == 2; other d: Morton): contiguous key ranges are
// compact regions, so tiles cut from them have shorter boundaries (fewer
// foreign rows and ghost cells) than Morton ranges
void hilbert_keys(const double* locs, int n, int d, std::vector<uint64_t>& keys) {
  if (d != 2) { morton_keys(locs, n, d, keys); return; }
  double lo[2], hi[2];
  for (int k = 0; k < 2; ++k) {
    double a = std::numeric_limits<double>::infinity(), b = -a;
    for (int i = 0; i < n; ++i) { double x = locs[i + (size_t)k * n]; a = std::min(a, x); b = std::max(b, x); }
    lo[k] = a; hi[k] = (b > a) ? b : a + 1.0;
  }
  const int bits = 31;
  const double scale = (double)((1ULL << bits) - 1);
  keys.resize(n);
  for (int i = 0; i < n; ++i) {
    uint64_t q[2];
    for (int k = 0; k < 2; ++k) {
      double u = (locs[i + (size_t)k * n] - lo[k]) / (hi[k] - lo[k]);
      u = std::min(1.0, std::max(0.0, u));
      q[k] = (uint64_t)(u * scale);
    }
    uint64_t x = q[0], y = q[1], key = 0;
    for (uint64_t s = 1ULL << (bits - 1); s > 0; s >>= 1) {
      const uint64_t rx = (x & s) ? 1 : 0, ry = (y & s) ? 1 : 0;
      key += s * s * ((3 * rx) ^ ry);
      if (ry == 0) {  // rotate the quadrant
        if (rx == 1) { x = s - 1 - (x & (s - 1)) + (x & ~(s - 1)); y = s - 1 - (y & (s - 1)) + (y & ~(s - 1)); }
        std::swap(x, y);
      }
    }
    keys[i] = key;
  }
}

// ---------------------------------------------------------------- max-min
void order_maxmin(const double* locs, int n, int d, std::vector<int>& order) {
  order.clear();
  if (n <= 0) return;
  order.reserve(n);
  double cen[8] = {0};
  for (int k = 0; k < d && k < 8; ++k) {
    for (int i = 0; i < n; ++i) cen[k] += locs[i + (size_t)k * n];
    cen[k] /= n;
  }
  int first = 0;
  double best = std::numeric_limits<double>::infinity();
  for (int i = 0; i < n; ++i) {
    double s = 0;
    for (int k = 0; k < d; ++k) { double t = locs[i + (size_t)k * n] - cen[k]; s += t * t; }
    if (s < best) { best = s; first = i; }
  }
  Grid g;
  g.build(locs, n, d, n, 2.0);
  std::vector<double> dist(n, std::numeric_limits<double>::infinity());
  std::vector<char> used(n, 0);
  // indexed max-heap on (dist, -idx)
  std::vector<int> heap, pos(n, -1);
  auto better = [&](int a, int b) { return dist[a] > dist[b] || (dist[a] == dist[b] && a < b); };
  auto sift_down = [&](int p) {
    int sz = (int)heap.size();
    for (;;) {
      int l = 2 * p + 1, r = l + 1, t = p;
      if (l < sz && better(heap[l], heap[t])) t = l;
      if (r < sz && better(heap[r], heap[t])) t = r;
      if (t == p) return;
      std::swap(heap[p], heap[t]); pos[heap[p]] = p; pos[heap[t]] = t; p = t;
    }
  };
  // first selection: every point's distance to `first`
  order.push_back(first);
  used[first] = 1;
  for (int i = 0; i < n; ++i)
    if (!used[i]) dist[i] = sqdist(locs, n, d, i, first);
  heap.reserve(n);
  for (int i = 0; i < n; ++i) if (!used[i]) { pos[i] = (int)heap.size(); heap.push_back(i); }
  for (int p = (int)heap.size() / 2 - 1; p >= 0; --p) sift_down(p);
  long long cc[3], lo_c[3], hi_c[3];
  while (!heap.empty()) {
    int p = heap[0];
    int last = heap.back(); heap.pop_back();
    pos[p] = -1;
    if (!heap.empty()) { heap[0] = last; pos[last] = 0; sift_down(0); }
    order.push_back(p);
    used[p] = 1;
    double r2 = dist[p];
    double r = std::sqrt(r2);
    g.cell_of(locs, n, p, cc);
    for (int k = 0; k < 3; ++k) {
      if (k < g.dg) {
        double x = locs[p + (size_t)k * n];
        lo_c[k] = g.coord(x - r, k);
        hi_c[k] = g.coord(x + r, k);
      } else { lo_c[k] = hi_c[k] = 0; }
    }
    long long q[3];
    for (q[2] = lo_c[2]; q[2] <= hi_c[2]; ++q[2])
      for (q[1] = lo_c[1]; q[1] <= hi_c[1]; ++q[1])
        for (q[0] = lo_c[0]; q[0] <= hi_c[0]; ++q[0]) {
          long long id = g.id_of(q);
          for (int t = g.start[id]; t < g.start[id + 1]; ++t) {
            int j = g.pts[t];
            if (used[j]) continue;
            double s = sqdist(locs, n, d, j, p);
            if (s < dist[j]) { dist[j] = s; sift_down(pos[j]); }
          }
        }
  }
}

// ---------------------------------------------------------------- ordered NN
void find_ordered_nn(const double* locs, int n, int d, int m, std::vector<int>& nn) {
  const int b = m + 1;
  nn.assign((size_t)n * b, -1);
  auto write_row = [&](int i, const TopM& top) {
    nn[(size_t)i * b] = i;
    for (int t = 0; t < top.cnt; ++t) nn[(size_t)i * b + 1 + t] = top.c[t].j;
  };
  const int brute = std::min(n, std::max(64, 4 * b));
  {
    std::vector<Cand> buf(std::max(m, 1));
    TopM top{m, 0, buf.data()};
    for (int i = 0; i < brute; ++i) {
      top.reset();
      if (m > 0)
        for (int j = 0; j < i; ++j) top.offer(sqdist(locs, n, d, i, j), j);
      write_row(i, top);
    }
  }
  if (m == 0) { for (int i = brute; i < n; ++i) nn[(size_t)i * b] = i; return; }
  Grid g;
  for (int lo = brute; lo < n;) {
    int hi = (int)std::min<long long>((long long)n, 2LL * lo);
    g.build(locs, n, d, hi, std::max(2.0, m / 3.0));
    // the queries of a block are independent given the grid of [0, hi)
    parallel_chunks(hi - lo, [&](int, long long q0, long long q1) {
      std::vector<Cand> buf(std::max(m, 1));
      TopM top{m, 0, buf.data()};
      long long cc[3], q[3];
      for (int i = lo + (int)q0; i < lo + (int)q1; ++i) {
        top.reset();
        g.cell_of(locs, n, i, cc);
        long long maxR = std::max(g.nc[0], std::max(g.nc[1], g.nc[2]));
        for (long long R = 0;; ++R) {
          // visit cells at Chebyshev distance exactly R
          long long lo_c[3], hi_c[3];
          for (int k = 0; k < 3; ++k) {
            if (k < g.dg) { lo_c[k] = std::max(0LL, cc[k] - R); hi_c[k] = std::min(g.nc[k] - 1, cc[k] + R); }
            else { lo_c[k] = hi_c[k] = 0; }
          }
          auto scan_cell = [&](const long long* qq) {
            long long id = g.id_of(qq);
            for (int t = g.start[id]; t < g.start[id + 1]; ++t) {
              int j = g.pts[t];
              if (j >= i) break;  // pts ascending inside a cell
              top.offer(sqdist(locs, n, d, i, j), j);
            }
          };
          for (q[2] = lo_c[2]; q[2] <= hi_c[2]; ++q[2])
            for (q[1] = lo_c[1]; q[1] <= hi_c[1]; ++q[1]) {
              long long outer = 0;
              if (g.dg >= 2) outer = std::max(outer, std::llabs(q[1] - cc[1]));
              if (g.dg >= 3) outer = std::max(outer, std::llabs(q[2] - cc[2]));
              if (outer == R) {
                for (q[0] = lo_c[0]; q[0] <= hi_c[0]; ++q[0]) scan_cell(q);
              } else {
                // only the two cells at |dq0| == R are on the ring
                q[0] = cc[0] - R;
                if (q[0] >= 0) scan_cell(q);
                q[0] = cc[0] + R;
                if (R > 0 && q[0] < g.nc[0]) scan_cell(q);
              }
            }
          if (R >= maxR) break;
          // every unvisited point is >= R*cs away (tiny margin for cell rounding)
          if (top.cnt == std::min(m, i)) {
            double bound = ((double)R - 1e-6) * g.cs;
            if (bound > 0 && bound * bound > top.worst()) break;
          }
        }
        write_row(i, top);
      }
    });
    lo = hi;
  }
}

// ---------------------------------------------------------------- colouring
int greedy_coloring(const int* nn, int n, int b, std::vector<int>& colors) {
  // CSC of the pattern of B: column i -> rows k with i in row(k)
  std::vector<int> cptr(n + 1, 0);
  for (long long e = 0; e < (long long)n * b; ++e) if (nn[e] >= 0) cptr[nn[e] + 1]++;
  for (int i = 0; i < n; ++i) cptr[i + 1] += cptr[i];
  std::vector<int> crow(cptr[n]);
  std::vector<int> fill(cptr.begin(), cptr.end() - 1);
  for (int k = 0; k < n; ++k)
    for (int t = 0; t < b; ++t) {
      int a = nn[(size_t)k * b + t];
      if (a >= 0) crow[fill[a]++] = k;
    }
  colors.assign(n, 0);
  // Blocks of nodes: the moral predecessors j < i of every node of the block
  // (the members of the rows through i, Coloring.R:14-16) are gathered in
  // parallel, deduplicated per node; then the first-fit pass runs over the
  // block in index order (Coloring.R:14-18), so the colours are those of the
  // sequential algorithm.
  const int nthr = host_threads();
  const int blk = 1 << 18;
  std::vector<long long> pptr(blk + 1);
  std::vector<std::vector<int>> pred(nthr);
  std::vector<std::vector<int>> seen(nthr);
  std::vector<int> mark(64, 0);
  int K = 0;
  for (int i0 = 0; i0 < n; i0 += blk) {
    const int i1 = std::min(n, i0 + blk);
    const int nb = i1 - i0;
    std::vector<int> cnt(nb, 0);
    const int T = std::max(1, std::min(nthr, nb / 1024));
    std::vector<std::vector<int>> part(T);
    std::vector<int> tlo(T + 1);
    for (int t = 0; t <= T; ++t) tlo[t] = (int)((long long)nb * t / T);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
      th.emplace_back([&, t] {
        std::vector<int>& sn = seen[t];
        if ((int)sn.size() < n) sn.assign(n, -1);
        std::vector<int>& out = part[t];
        out.clear();
        for (int ii = tlo[t]; ii < tlo[t + 1]; ++ii) {
          const int i = i0 + ii;
          for (int p = cptr[i]; p < cptr[i + 1]; ++p) {
            const int k = crow[p];
            for (int u = 0; u < b; ++u) {
              const int j = nn[(size_t)k * b + u];
              if (j >= 0 && j < i && sn[j] != i) { sn[j] = i; out.push_back(j); ++cnt[ii]; }
            }
          }
        }
      });
    for (auto& x : th) x.join();
    for (int t = 0; t < T; ++t) {
      const int* pj = part[t].data();
      for (int ii = tlo[t]; ii < tlo[t + 1]; ++ii) {
        const int i = i0 + ii, stamp = i + 1;
        for (int q = 0; q < cnt[ii]; ++q) mark[colors[pj[q]]] = stamp;
        pj += cnt[ii];
        int c = 1;
        while (c < (int)mark.size() && mark[c] == stamp) ++c;
        if (c + 1 >= (int)mark.size()) mark.resize(2 * mark.size() + 2, 0);
        colors[i] = c;
        K = std::max(K, c);
      }
    }
  }
  return K;
}

// ---------------------------------------------------------------- layout
bool build_sweep_layout(const int* nn, int n, int b, const int* colors, const double* locs, int d,
                        int LW, SweepLayout& L, std::string& err) {
  L = SweepLayout();
  L.n = n; L.b = b; L.LW = LW;
  if (LW != 64 && LW != 32 && LW != 21 && LW != 16) { err = "lanes_per_chain must be 64, 32, 21 or 16"; return false; }
  if (n >= kPadRow) { err = "n too large for the packed sweep row index (< 2^25 - 1)"; return false; }
  int K = 0;
  for (int i = 0; i < n; ++i) {
    if (colors[i] < 1) { err = "coloring must be 1-based positive"; return false; }
    K = std::max(K, colors[i]);
  }
  L.K = K;
  std::vector<uint64_t> key;
  morton_keys(locs, n, d, key);
  // r positions: global Morton rank
  std::vector<int> perm(n);
  std::iota(perm.begin(), perm.end(), 0);
  std::sort(perm.begin(), perm.end(), [&](int a, int c) { return key[a] < key[c] || (key[a] == key[c] && a < c); });
  L.rpos.resize(n);
  for (int r = 0; r < n; ++r) L.rpos[perm[r]] = r;
  // CSC of B (rows ascending inside a column)
  std::vector<long long> cptr(n + 1, 0);
  for (long long e = 0; e < (long long)n * b; ++e) {
    int a = nn[e];
    if (a >= n) { err = "NNarray index out of range"; return false; }
    if (a >= 0) cptr[a + 1]++;
  }
  for (int i = 0; i < n; ++i) cptr[i + 1] += cptr[i];
  L.nnz = cptr[n];
  std::vector<int> crow(L.nnz), csrc(L.nnz);
  {
    std::vector<long long> f(cptr.begin(), cptr.end() - 1);
    for (int k = 0; k < n; ++k)
      for (int t = 0; t < b; ++t) {
        int a = nn[(size_t)k * b + t];
        if (a < 0) continue;
        long long p = f[a]++;
        crow[p] = k; csrc[p] = L.rpos[k] * b + t;  // device rows are Morton-ordered
      }
  }
  const int cap = LW * kRowsMax, max_slots = 2 * LW - 1;
  for (int i = 0; i < n; ++i) {
    const int len = (int)(cptr[i + 1] - cptr[i]);
    L.max_collen = std::max(L.max_collen, len);
    if (len > cap) {
      err = "a column of B has " + std::to_string(len) + " entries, more than a sweep chunk (" +
            std::to_string(cap) + "; use fewer chains per context)";
      return false;
    }
  }
  // locations of each colour in Morton order, packed greedily into chunks
  // (<= cap cells, <= max_slots locations)
  std::vector<int> cptr_col(K + 1, 0);
  for (int i = 0; i < n; ++i) cptr_col[colors[i]]++;
  for (int c = 0; c < K; ++c) cptr_col[c + 1] += cptr_col[c];
  for (int c = 0; c < K; ++c)
    if (cptr_col[c + 1] == cptr_col[c]) { err = "coloring has an empty colour class"; return false; }
  std::vector<int> by_col(n);
  {
    std::vector<int> f(cptr_col.begin(), cptr_col.end() - 1);
    for (int r = 0; r < n; ++r) { int i = perm[r]; by_col[f[colors[i] - 1]++] = i; }
  }
  std::vector<int> chunk_first;  // index into by_col of each chunk's first location
  L.color_chunk_ptr.assign(K + 1, 0);
  for (int c = 0; c < K; ++c) {
    int fill = 0, cnt = 0;
    for (int x = cptr_col[c]; x < cptr_col[c + 1]; ++x) {
      const int len = (int)(cptr[by_col[x] + 1] - cptr[by_col[x]]);
      if (cnt == 0 || fill + len > cap || cnt + 1 > max_slots) {
        chunk_first.push_back(x);
        fill = 0;
        cnt = 0;
      }
      fill += len;
      ++cnt;
    }
    L.color_chunk_ptr[c + 1] = (int)chunk_first.size();
  }
  L.nchunks = (int)chunk_first.size();
  chunk_first.push_back(n);
  L.compact_loc = by_col;
  L.color_loc_ptr = cptr_col;
  L.chunk_first = chunk_first;
  L.n_entries = (long long)L.nchunks * cap;
  L.collen.assign(n, 0);
  L.slot_f0.assign(n, 0);
  L.ent_pk.assign(L.n_entries, 0);
  L.ent_src.assign(L.n_entries, -1);
  L.ent_pos.assign(L.n_entries, 0);
  L.start_mask.assign((size_t)L.nchunks * LW, 0);
  struct Cell { int p, q, src, f; };
  std::vector<Cell> cells;
  for (int ch = 0; ch < L.nchunks; ++ch) {
    const long long base = (long long)ch * cap;
    cells.clear();
    int f = 0;
    for (int x = chunk_first[ch], q = 0; x < chunk_first[ch + 1]; ++x, ++q) {
      const int i = by_col[x];
      L.collen[x] = (int)(cptr[i + 1] - cptr[i]);
      L.slot_f0[x] = f;
      L.start_mask[(size_t)ch * LW + f / kRowsMax] |= (uint16_t)(1u << (f % kRowsMax));
      for (long long p = cptr[i]; p < cptr[i + 1]; ++p, ++f) cells.push_back({L.rpos[crow[p]], q, csrc[p], f});
    }
    // row order (rows are distinct inside a colour); padding cells last
    std::sort(cells.begin(), cells.end(), [](const Cell& a, const Cell& b2) { return a.p < b2.p; });
    for (int g = f; g < cap; ++g) cells.push_back({kPadRow, max_slots, -1, g});
    if (f < cap) L.start_mask[(size_t)ch * LW + f / kRowsMax] |= (uint16_t)(1u << (f % kRowsMax));
    for (int k = 0; k < cap; ++k) {
      const long long e = base + k;
      L.ent_pk[e] = (int)((unsigned)cells[k].p | ((unsigned)cells[k].q << kRowBits));
      L.ent_src[e] = cells[k].src;
      L.ent_pos[e] = (uint16_t)cells[k].f;
    }
  }
  return true;
}

// ---------------------------------------------------------------- tile layout
bool build_tile_layout(const int* nn, int n, int b, const int* colors, const double* locs, int d, int T,
                       int NT, int RMAX, TileLayout& L, std::string& err, int G, bool split, int waves) {
  L = TileLayout();
  L.n = n; L.b = b; L.NT = NT; L.RMAX = RMAX; L.W = waves;
  if (NT < 64 || NT > 1024 || RMAX < 1 || (long long)NT * RMAX > (1 << 20)) { err = "tile layout: bad NT/RMAX"; return false; }
  if (waves < 0 || (waves > 0 && (NT != 64 || waves * kWaveSlotsMax > kAccSlots))) {
    err = "tile layout: wave-local batches need NT = 64 and waves x kWaveSlotsMax <= kAccSlots";
    return false;
  }
  if (T < 1) T = 1;
  if (T > n) T = n;
  if (G < 1 || G > kMaxTileRanks || T % G != 0) { err = "tile layout: need 1 <= G <= 16 ranks dividing the tile count"; return false; }
  L.T = T;
  L.G = G;
  const int Tl = T / G;  // tiles per rank
  int K = 0;
  for (int i = 0; i < n; ++i) {
    if (colors[i] < 1) { err = "coloring must be 1-based positive"; return false; }
    K = std::max(K, colors[i]);
  }
  L.K = K;
  std::vector<uint64_t> key;
  // tiles along the Hilbert curve (NNGP_TILE_CURVE=morton: Morton): at n =
  // 1e6, m = 15, 256 tiles 7 % fewer ghost cells and 9 % fewer foreign slots,
  // 0.5-1 % faster sweeps
  const char* curve = std::getenv("NNGP_TILE_CURVE");
  if (curve && std::string(curve) == "morton") morton_keys(locs, n, d, key);
  else hilbert_keys(locs, n, d, key);
  std::vector<int> perm(n);  // curve rank -> loc
  std::iota(perm.begin(), perm.end(), 0);
  std::sort(perm.begin(), perm.end(), [&](int a, int c) { return key[a] < key[c] || (key[a] == key[c] && a < c); });
  L.rpos.resize(n);
  for (int r = 0; r < n; ++r) L.rpos[perm[r]] = r;
  // CSC of B: column i -> (row k, position u of i in row k)
  std::vector<long long> cptr(n + 1, 0);
  for (long long e = 0; e < (long long)n * b; ++e) {
    const int a = nn[e];
    if (a >= n) { err = "NNarray index out of range"; return false; }
    if (a >= 0) cptr[a + 1]++;
  }
  for (int i = 0; i < n; ++i) cptr[i + 1] += cptr[i];
  L.nnz = cptr[n];
  std::vector<int> crow(L.nnz), cu(L.nnz);
  {
    std::vector<long long> f(cptr.begin(), cptr.end() - 1);
    for (int k = 0; k < n; ++k)
      for (int u = 0; u < b; ++u) {
        const int a = nn[(size_t)k * b + u];
        if (a < 0) continue;
        const long long p = f[a]++;
        crow[p] = k; cu[p] = u;
      }
  }
  for (int i = 0; i < n; ++i) L.max_collen = std::max(L.max_collen, (int)(cptr[i + 1] - cptr[i]));
  if (L.max_collen > NT * RMAX) { err = "tile layout: a column of B is longer than a batch"; return false; }
  // tiles: contiguous Morton ranges with equal column work (collen + 1)
  L.tile_row0.assign(T + 1, n);
  {
    long long tot = 0;
    for (int i = 0; i < n; ++i) tot += (cptr[i + 1] - cptr[i]) + 1;
    long long acc = 0;
    int t = 0;
    L.tile_row0[0] = 0;
    for (int r = 0; r < n && t + 1 < T; ++r) {
      const int i = perm[r];
      acc += (cptr[i + 1] - cptr[i]) + 1;
      // tile t ends when its share is reached, leaving >= 1 row per later tile
      if (acc * T >= tot * (long long)(t + 1) || n - (r + 1) <= T - (t + 1)) L.tile_row0[++t] = r + 1;
    }
    while (t + 1 < T) { L.tile_row0[t + 1] = L.tile_row0[t] + 1; ++t; }
    L.tile_row0[T] = n;
  }
  std::vector<int> tile_of(n);  // loc -> tile
  for (int t = 0; t < T; ++t)
    for (int r = L.tile_row0[t]; r < L.tile_row0[t + 1]; ++r) tile_of[perm[r]] = t;
  // split layouts: a slot is "boundary" when a row of its column has a
  // member of the previous colour (cyclic) owned by another tile
  L.split = split;
  std::vector<char> bnd(split ? n : 0, 0);
  if (split) {
    parallel_chunks(n, [&](int, long long i0, long long i1) {
      for (long long i = i0; i < i1; ++i) {
        const int cp = (colors[i] - 1 + K - 1) % K + 1, t = tile_of[i];
        for (long long p = cptr[i]; p < cptr[i + 1] && !bnd[i]; ++p) {
          const int k = crow[p];
          for (int u = 0; u < b; ++u) {
            const int j = nn[(size_t)k * b + u];
            if (j >= 0 && colors[j] == cp && tile_of[j] != t) { bnd[i] = 1; break; }
          }
        }
      }
    });
  }
  // slot order: tile, colour, (split: interior before boundary), Morton
  L.compact_loc.resize(n);
  std::vector<int> slot_of(n);
  std::vector<int> tc_ptr((size_t)T * K + 1, 0);  // slots of (tile, colour)
  for (int i = 0; i < n; ++i) tc_ptr[(size_t)tile_of[i] * K + colors[i]]++;
  for (size_t p = 0; p < (size_t)T * K; ++p) tc_ptr[p + 1] += tc_ptr[p];
  std::vector<int> tc_split;  // split: first boundary slot of (tile, colour)
  {
    std::vector<int> f(tc_ptr.begin(), tc_ptr.end() - 1);
    for (int pass = 0; pass < (split ? 2 : 1); ++pass) {
      for (int r = 0; r < n; ++r) {
        const int i = perm[r];
        if (split && bnd[i] != pass) continue;
        const int x = f[(size_t)tile_of[i] * K + colors[i] - 1]++;
        L.compact_loc[x] = i;
        slot_of[i] = x;
      }
      if (split && pass == 0) tc_split = f;
    }
  }
  L.rank_slot0.assign(G + 1, 0);
  for (int g = 0; g <= G; ++g) L.rank_slot0[g] = tc_ptr[(size_t)g * Tl * K];
  if (G > 1) L.rmask.assign(n, 0u);
  L.slot_f0.assign(n, 0);
  L.batch_ptr.assign((size_t)T * K + 1, 0);
  L.gptr.assign((size_t)T * K + 1, 0);
  L.gslot_ptr.assign((size_t)T * K + 1, 0);
  L.nb_ptr.assign((size_t)T * K + 1, 0);
  L.erow_ptr.assign(T + 1, 0);
  if (split) L.batch_split.assign((size_t)T * K, 0);
  // Per tile independently (threads over tile ranges), then concatenated in
  // tile order: the layout is the same for any thread count.
  struct TileOut {
    std::vector<int> rows;                 // local rows (device rows)
    std::vector<TileBatch> batch;          // off relative to the tile's first cell
    std::vector<int> bptr, bsplit;         // K+1 / K, relative to the tile's first batch
    std::vector<uint32_t> cell_pk;
    std::vector<int> cell_src;
    std::vector<int> slot_f0;              // own slots [tc_ptr[t*K], tc_ptr[t*K+K]): f0 bits
    std::vector<int> gcell, gsrc, gslot, nb;
    std::vector<int> gptr, gsptr, nbptr;   // K+1, relative
    std::vector<int> exported;             // foreign slots this tile reads
    std::vector<std::pair<int, int>> rbits;  // (slot, reader rank) across ranks
    int max_gslots = 0;
    std::string err;
  };
  const int nth = std::max(1, std::min(std::min(host_threads(), 8), T));
  std::vector<TileOut> outs(T);
  auto build_range = [&](int t0, int t1) {
    std::vector<int> gidx(n, -1);   // slot -> index in the current (tile, colour)'s foreign slots
    std::vector<int> lr_of(n, -1);  // device row -> local row of the current tile
    std::vector<int> nbmark(T, -1);
    std::vector<std::vector<int>> gh(K);  // ghost cells of the current tile by colour: (lr, x, src)
    for (int t = t0; t < t1; ++t) {
      TileOut& o = outs[t];
      std::vector<int>& rows = o.rows;
      // local rows: own rows, then ghost rows in curve order
      for (int r = L.tile_row0[t]; r < L.tile_row0[t + 1]; ++r) rows.push_back(r);
      const size_t n_own = rows.size();
      for (int r = L.tile_row0[t]; r < L.tile_row0[t + 1]; ++r) {
        const int i = perm[r];
        for (long long p = cptr[i]; p < cptr[i + 1]; ++p) {
          const int k = crow[p];
          if (tile_of[k] != t) rows.push_back(L.rpos[k]);
        }
      }
      std::sort(rows.begin() + n_own, rows.end());
      rows.erase(std::unique(rows.begin() + n_own, rows.end()), rows.end());
      if (rows.size() > kTilePadRow) { o.err = "tile layout: too many local rows in a tile"; return; }
      for (size_t q = 0; q < rows.size(); ++q) lr_of[rows[q]] = (int)q;
      // own batches, colour by colour (split: the interior run, then the boundary run)
      const int xs0 = tc_ptr[(size_t)t * K];
      o.slot_f0.assign(tc_ptr[(size_t)t * K + K] - xs0, 0);
      o.bptr.assign(K + 1, 0);
      if (split) o.bsplit.assign(K, 0);
      for (int c = 0; c < K; ++c) {
        const size_t pc = (size_t)t * K + c;
        int x = tc_ptr[pc];
        const int xe_all = tc_ptr[pc + 1];
        if (split) o.bsplit[c] = (int)o.batch.size();
        for (int run = 0; run < (split ? 2 : 1); ++run) {
          const int xe = split && run == 0 ? tc_split[pc] : xe_all;
          if (split && run == 1) o.bsplit[c] = (int)o.batch.size();
          // wave-local: the run's batches in rounds of `waves`, cut where the
          // prefix of the run's cells crosses g/nb of its total (balanced
          // waves), capped at kWaveSlotsMax slots and NT*RMAX cells
          long long run_cells = 0;
          int nbw = 0, bw = 0;
          long long acc_cells = 0;
          if (waves > 0 && x < xe) {
            for (int y = x; y < xe; ++y) run_cells += cptr[L.compact_loc[y] + 1] - cptr[L.compact_loc[y]];
            const long long by_cells = (run_cells + (long long)NT * RMAX * 7 / 8 - 1) / ((long long)NT * RMAX * 7 / 8);
            const long long by_slots = (xe - x + kWaveSlotsMax - 1) / kWaveSlotsMax;
            nbw = (int)std::max<long long>(1, std::max(by_cells, by_slots));
            nbw = (nbw + waves - 1) / waves * waves;
            nbw = std::min(nbw, xe - x);
          }
          while (x < xe) {
            int cells = 0, ns = 0;
            const int smax = waves > 0 ? kWaveSlotsMax : std::min(NT, kTileSlotsMax);
            while (x + ns < xe && ns < smax) {
              const int len = (int)(cptr[L.compact_loc[x + ns] + 1] - cptr[L.compact_loc[x + ns]]);
              if (cells + len > NT * RMAX) break;
              // balanced cut: stop once this batch reaches its share of the run
              if (waves > 0 && ns > 0 && bw + 1 < nbw &&
                  2 * (acc_cells + cells) + len > 2 * run_cells * (bw + 1) / nbw)
                break;
              cells += len;
              ++ns;
            }
            acc_cells += cells;
            ++bw;
            const int R = std::max(1, (cells + NT - 1) / NT);
            TileBatch tb{(int)o.cell_pk.size(), R, ns, x, (cells + R - 1) / R};
            o.cell_pk.resize(o.cell_pk.size() + (size_t)R * NT, kTilePadRow);
            o.cell_src.resize(o.cell_pk.size(), -1);
            int f = 0;
            for (int q = 0; q < ns; ++q) {
              const int i = L.compact_loc[x + q];
              o.slot_f0[x + q - xs0] = f;
              const long long p0 = cptr[i], p1 = cptr[i + 1];
              for (long long p = p0; p < p1; ++p, ++f) {
                const int k = crow[p];
                uint32_t pk = (uint32_t)lr_of[L.rpos[k]] | ((uint32_t)q << kTileQShift);
                if (p == p0) pk |= kCellStart;
                if (p == p1 - 1) pk |= kCellEnd;
                const size_t e = (size_t)tb.off + (size_t)(f % R) * NT + f / R;
                o.cell_pk[e] = pk;
                o.cell_src[e] = L.rpos[k] * b + cu[p];
              }
            }
            o.batch.push_back(tb);
            x += ns;
          }
        }
        o.bptr[c + 1] = (int)o.batch.size();
      }
      // ghost cells: foreign members j of the tile's rows, by colour of j
      for (auto& g : gh) g.clear();
      for (size_t q = 0; q < rows.size(); ++q) {
        const int k = perm[rows[q]];
        for (int u = 0; u < b; ++u) {
          const int j = nn[(size_t)k * b + u];
          if (j < 0 || tile_of[j] == t) continue;
          auto& g = gh[colors[j] - 1];
          g.push_back((int)q);
          g.push_back(slot_of[j]);
          g.push_back(L.rpos[k] * b + u);
          o.exported.push_back(slot_of[j]);
        }
      }
      o.gptr.assign(K + 1, 0);
      o.gsptr.assign(K + 1, 0);
      o.nbptr.assign(K + 1, 0);
      for (int c = 0; c < K; ++c) {
        const size_t pc = (size_t)t * K + c;
        const int gs0 = (int)o.gslot.size();
        for (size_t g = 0; g < gh[c].size(); g += 3) {
          const int x = gh[c][g + 1];
          if (gidx[x] < 0) { gidx[x] = (int)o.gslot.size() - gs0; o.gslot.push_back(x); }
          o.gcell.push_back(gh[c][g]);
          o.gcell.push_back(gidx[x]);
          o.gsrc.push_back(gh[c][g + 2]);
          const int u = tile_of[L.compact_loc[x]];
          if (nbmark[u] != (int)pc) { nbmark[u] = (int)pc; o.nb.push_back(u); }
          if (G > 1 && u / Tl != t / Tl) o.rbits.emplace_back(x, t / Tl);
        }
        for (size_t q = gs0; q < o.gslot.size(); ++q) gidx[o.gslot[q]] = -1;
        o.gsptr[c + 1] = (int)o.gslot.size();
        o.max_gslots = std::max(o.max_gslots, (int)o.gslot.size() - gs0);
        o.gptr[c + 1] = (int)o.gsrc.size();
        o.nbptr[c + 1] = (int)o.nb.size();
      }
      for (int r : rows) lr_of[r] = -1;
    }
  };
  {
    std::vector<std::thread> th;
    for (int h = 0; h < nth; ++h) {
      const int t0 = (int)((long long)T * h / nth), t1 = (int)((long long)T * (h + 1) / nth);
      if (nth == 1) build_range(t0, t1);
      else th.emplace_back([=, &build_range] { build_range(t0, t1); });
    }
    for (auto& x : th) x.join();
  }
  // concatenate in tile order
  for (int t = 0; t < T; ++t) {
    TileOut& o = outs[t];
    if (!o.err.empty()) { err = o.err; return false; }
    L.max_rows = std::max(L.max_rows, (int)o.rows.size());
    L.erow.insert(L.erow.end(), o.rows.begin(), o.rows.end());
    L.erow_ptr[t + 1] = (int)L.erow.size();
    const long long cell0 = (long long)L.cell_pk.size();
    if (cell0 + (long long)o.cell_pk.size() > INT32_MAX) { err = "tile layout: too many cells"; return false; }
    const int b0 = (int)L.batch.size();
    for (TileBatch tb : o.batch) {
      tb.off += (int)cell0;
      L.batch.push_back(tb);
    }
    for (int c = 0; c < K; ++c) {
      L.batch_ptr[(size_t)t * K + c + 1] = b0 + o.bptr[c + 1];
      if (split) L.batch_split[(size_t)t * K + c] = b0 + o.bsplit[c];
    }
    L.max_batches = std::max(L.max_batches, (int)o.batch.size());
    L.cell_pk.insert(L.cell_pk.end(), o.cell_pk.begin(), o.cell_pk.end());
    L.cell_src.insert(L.cell_src.end(), o.cell_src.begin(), o.cell_src.end());
    const int xs0 = tc_ptr[(size_t)t * K];
    for (size_t q = 0; q < o.slot_f0.size(); ++q) L.slot_f0[xs0 + q] |= o.slot_f0[q];
    const int gc0 = (int)L.gsrc.size(), gs0 = (int)L.gslot.size(), nb0 = (int)L.nb.size();
    L.gcell.insert(L.gcell.end(), o.gcell.begin(), o.gcell.end());
    L.gsrc.insert(L.gsrc.end(), o.gsrc.begin(), o.gsrc.end());
    L.gslot.insert(L.gslot.end(), o.gslot.begin(), o.gslot.end());
    L.nb.insert(L.nb.end(), o.nb.begin(), o.nb.end());
    for (int c = 0; c < K; ++c) {
      L.gptr[(size_t)t * K + c + 1] = gc0 + o.gptr[c + 1];
      L.gslot_ptr[(size_t)t * K + c + 1] = gs0 + o.gsptr[c + 1];
      L.nb_ptr[(size_t)t * K + c + 1] = nb0 + o.nbptr[c + 1];
    }
    L.max_gslots = std::max(L.max_gslots, o.max_gslots);
    for (int x : o.exported) L.slot_f0[x] |= kSlotExported;
    for (const auto& xb : o.rbits) L.rmask[xb.first] |= 1u << xb.second;
    o = TileOut();  // free as we go
  }
  return true;
}

// ---------------------------------------------------------------- shard plan
bool build_shard_plan(const int* nn, int n, int b, const int* colors, const SweepLayout& L, int G, int rank,
                      ShardPlan& P, std::string& err) {
  P = ShardPlan();
  if (G < 1 || G > kMaxRanks || rank < 0 || rank >= G) { err = "shard plan: need 1 <= G <= 64, 0 <= rank < G"; return false; }
  if (L.nchunks == 0 || (int)L.compact_loc.size() != n) { err = "shard plan: needs the colour-launch layout"; return false; }
  const int K = L.K;
  P.G = G; P.rank = rank; P.K = K;
  // chunk -> rank by the Morton rank of its first slot (monotone inside a colour)
  P.cb.assign((size_t)K * (G + 1), 0);
  P.seg0.assign((size_t)K * (G + 1), 0);
  P.cnt.assign(K, 0);
  P.xoff.assign(K + 1, 0);
  std::vector<int> owner(n, 0);  // compact slot -> rank
  for (int c = 0; c < K; ++c) {
    const int ch0 = L.color_chunk_ptr[c], ch1 = L.color_chunk_ptr[c + 1];
    int* cb = &P.cb[(size_t)c * (G + 1)];
    int* sg = &P.seg0[(size_t)c * (G + 1)];
    int ch = ch0;
    for (int g = 0; g < G; ++g) {
      cb[g] = ch;
      const long long hi = (long long)(g + 1) * n / G;  // Morton ranks of rank g: [g*n/G, hi)
      while (ch < ch1 && (g == G - 1 || L.rpos[L.compact_loc[L.chunk_first[ch]]] < hi)) ++ch;
    }
    cb[G] = ch1;
    for (int g = 0; g <= G; ++g) sg[g] = L.chunk_first[cb[g]];
    for (int g = 0; g < G; ++g) {
      P.cnt[c] = std::max(P.cnt[c], sg[g + 1] - sg[g]);
      for (int x = sg[g]; x < sg[g + 1]; ++x) owner[x] = g;
    }
    P.cnt[c] = std::max(P.cnt[c], 1);
    P.xoff[c + 1] = P.xoff[c] + (long long)G * P.cnt[c];
    P.owned += sg[rank + 1] - sg[rank];
  }
  std::vector<int> loc_rank(n), col_of(n);
  for (int x = 0; x < n; ++x) loc_rank[L.compact_loc[x]] = x;
  for (int c = 0; c < K; ++c)
    for (int x = L.color_loc_ptr[c]; x < L.color_loc_ptr[c + 1]; ++x) col_of[x] = c;
  // ghost cells: rows (Morton order) with an owned member; their foreign members
  std::vector<int> perm(n);
  for (int i = 0; i < n; ++i) perm[L.rpos[i]] = i;
  std::vector<std::vector<int>> gh(K);  // per colour: triples (row, src, recv)
  for (int r = 0; r < n; ++r) {
    const int k = perm[r];
    bool need = false;
    for (int t = 0; t < b && !need; ++t) {
      const int j = nn[(size_t)k * b + t];
      need = j >= 0 && owner[loc_rank[j]] == rank;
    }
    if (!need) continue;
    ++P.needed_rows;
    for (int t = 0; t < b; ++t) {
      const int j = nn[(size_t)k * b + t];
      if (j < 0) continue;
      const int x = loc_rank[j], h = owner[x];
      if (h == rank) continue;
      const int c = col_of[x];
      if (colors[j] - 1 != c) { err = "shard plan: colouring and layout disagree"; return false; }
      gh[c].insert(gh[c].end(), {r, r * b + t, h * P.cnt[c] + (x - P.seg0[(size_t)c * (G + 1) + h])});
    }
  }
  P.gptr.assign(K + 1, 0);
  for (int c = 0; c < K; ++c) {
    for (size_t g = 0; g < gh[c].size(); g += 3) {
      P.grow.push_back(gh[c][g]);
      P.gsrc.push_back(gh[c][g + 1]);
      P.grecv.push_back(gh[c][g + 2]);
    }
    P.gptr[c + 1] = (int)P.grow.size();
  }
  // normal pairs with an owned member, in the order of the full layout
  P.pair_ptr.assign(K + 1, 0);
  for (int c = 0; c < K; ++c) {
    for (int x = L.color_loc_ptr[c]; x < L.color_loc_ptr[c + 1]; ++x) {
      const int i = L.compact_loc[x];
      if (i & 1) continue;
      const bool mine = owner[x] == rank || (i + 1 < n && owner[loc_rank[i + 1]] == rank);
      if (mine) P.pairs.push_back(i >> 1);
    }
    P.pair_ptr[c + 1] = (int)P.pairs.size();
  }
  return true;
}

void dag_levels(const int* nn, int n, int b, std::vector<int>& level_ptr, std::vector<int>& level_rows) {
  std::vector<int> lev(n, 0);
  int maxl = 0;
  for (int i = 0; i < n; ++i) {
    int l = 0;
    for (int t = 1; t < b; ++t) {
      int j = nn[(size_t)i * b + t];
      if (j >= 0) l = std::max(l, lev[j] + 1);
    }
    lev[i] = l;
    maxl = std::max(maxl, l);
  }
  level_ptr.assign(maxl + 2, 0);
  for (int i = 0; i < n; ++i) level_ptr[lev[i] + 1]++;
  for (int l = 0; l <= maxl; ++l) level_ptr[l + 1] += level_ptr[l];
  level_rows.resize(n);
  std::vector<int> f(level_ptr.begin(), level_ptr.end() - 1);
  for (int i = 0; i < n; ++i) level_rows[f[lev[i]]++] = i;
}

int tile_lds_bytes(int max_rows, int C, int NT, int K, int max_batches, int max_gslots) {
  const int rbytes = ((max_rows * C * 8 + 15) / 16) * 16;
  return rbytes + kAccSlots * C * 8 + (NT / 64) * C * 8 + 5 * C * 8 + ((max_gslots * C + 1) / 2) * 16 +
         max_batches * 16 + 4 * (K + 1) * 4 + (NT / 64) * 4 + 64;
}

}  // namespace nngp
