// Host-side (C++) init-time graph preparation for the NNGP chromatic sweep.
// Internal header: nothing here crosses the C ABI (see include/nngp.h).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace nngp {

// Exact max-min ordering (first point closest to the centroid, then the point
// farthest from the selected set; ties -> smaller index).  order: 0-based.
void order_maxmin(const double* locs_colmajor, int n, int d, std::vector<int>& order);

// Exact ordered nearest neighbours (GpGp::find_ordered_nn semantics without
// GpGp's RNG jitter): nn[i*b + 0] = i, nn[i*b + 1..] = the m nearest j < i by
// ascending squared Euclidean distance (ties -> smaller j), -1 padded.
void find_ordered_nn(const double* locs_colmajor, int n, int d, int m, std::vector<int>& nn_rowmajor);

// Greedy first-fit colouring of the moral graph pattern(B^T B) in index order
// (Coloring.R:2-20).  nn: row-major 0-based, -1 = NA.  Returns K; colors 1-based.
int greedy_coloring(const int* nn_rowmajor, int n, int b, std::vector<int>& colors);

// Morton (Z-order) key of each location on a 21-bit-per-axis grid over the
// bounding box of the first min(d,3) coordinates.
void morton_keys(const double* locs_colmajor, int n, int d, std::vector<uint64_t>& keys);

// Device layout of the chromatic sweep ("sliced ELL with row-count classes").
//  - slots: locations re-indexed colour-major; inside a colour by row-count
//    class R (descending), Morton order inside a class;
//  - r / field / Linv rows: Morton rank of the location (rpos);
//  - slot i (column i of B, len_i entries) gets k_i = 2^lk_i lanes and
//    R_i = ceil(len_i / k_i) rows, k_i the smallest power of two with
//    R_i <= kRowsMax (so len <= 16 => k = 1, R = len: no padding);
//  - chunk: one wavefront's share of ONE chain: LW lanes (LW = 64 / chains
//    per wave) over a Morton-contiguous run of slots of one (colour, class);
//    all chunks of a class have R rows, so chunk q of the class starts at
//    entry base_class + q * LW * R: a closed form of per-colour kernel
//    arguments (no metadata load in front of the entry loads);
//  - lane_tab[ch*LW + l] = (slot + 1) | lk << 28 (0: idle lane); lane groups
//    sorted by descending k inside a chunk => aligned power-of-two groups;
//  - entry q of slot i lives at chunk_base + (q >> lk) * LW + o_i + (q & (k-1))
//    (o_i = first lane of the slot's group).
constexpr int kRowsMax = 16;  // rows per lane of a sweep chunk (== kSweepRows)
constexpr int kMaxClasses = kRowsMax;

struct SweepLayout {
  int n = 0, b = 0, K = 0, nchunks = 0, LW = 64;
  long long nnz = 0, n_entries = 0;
  int max_collen = 0;
  std::vector<int> color_slot_ptr;   // K+1
  std::vector<int> color_chunk_ptr;  // K+1
  std::vector<int> slot_loc;         // n
  std::vector<int> loc_slot;         // n
  std::vector<int> rpos;             // n: loc -> device row (Morton rank): r, field, Linv rows
  std::vector<int> collen;           // n (slot order)
  std::vector<int> lane_tab;         // nchunks x LW
  // per colour: n_class[c] classes; class q of colour c (index c*kMaxClasses+q):
  // rows, exclusive chunk end relative to the colour's first chunk, first entry
  std::vector<int> n_class;          // K
  std::vector<int> class_rows;       // K * kMaxClasses
  std::vector<int> class_end;        // K * kMaxClasses
  std::vector<long long> class_base; // K * kMaxClasses
  std::vector<int> ent_rowpos;       // n_entries (padding: 0)
  std::vector<int> ent_src;          // n_entries (device Linv index rpos[k]*b+j; padding: -1)
};

// lanes_per_chain: 64, 32 or 16 (1, 2 or 3-4 chains per wavefront).  Fails if
// a column of B is longer than lanes_per_chain * kRowsMax.
bool build_sweep_layout(const int* nn_rowmajor, int n, int b, const int* colors,
                        const double* locs_colmajor, int d, int lanes_per_chain, SweepLayout& L,
                        std::string& err);

// Level sets of the Vecchia DAG for the sparse triangular solve:
// level(i) = 1 + max level(NN(i)), level 0 rows have no neighbours.
void dag_levels(const int* nn_rowmajor, int n, int b, std::vector<int>& level_ptr,
                std::vector<int>& level_rows);

}  // namespace nngp
