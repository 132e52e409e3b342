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

// Device layout of the chromatic sweep ("sliced-ELL by colour").
//  - slots: locations re-indexed colour-major (colour 1 first), spatially
//    (Morton) sorted inside a colour;
//  - r positions: Morton rank of each Vecchia row;
//  - chunks: one wavefront over 64/k consecutive slots of one colour, k =
//    lanes per slot (power of two) chosen so that no chunk has more than
//    kRowsMax rows (long columns of coarse max-min points are split over lanes);
//  - entries: entry j of the t-th slot of a chunk stored at
//    chunk_off[ch] + (j / k) * 64 + t * k + (j % k).
constexpr int kRowsMax = 16;
constexpr int kSlotGroup = 512;  // spatial group of same-colour slots (see build_sweep_layout)
struct SweepLayout {
  int n = 0, b = 0, K = 0, nchunks = 0;
  long long nnz = 0, n_entries = 0;
  int max_collen = 0;
  std::vector<int> color_slot_ptr;   // K+1
  std::vector<int> color_chunk_ptr;  // K+1
  std::vector<int> slot_loc;         // n
  std::vector<int> loc_slot;         // n
  std::vector<int> rpos;             // n: loc -> device row (Morton rank): r, field, Linv rows
  std::vector<int> collen;           // n (slot order)
  std::vector<int> chunk_slot0;      // nchunks
  std::vector<int> chunk_len;        // nchunks: rows of the chunk
  std::vector<int> chunk_nslot;      // nchunks: slots in the chunk (<= 64/k)
  std::vector<int> chunk_lk;         // nchunks: log2(k)
  std::vector<long long> chunk_off;  // nchunks
  std::vector<int> ent_rowpos;       // n_entries (padding: 0)
  std::vector<int> ent_src;          // n_entries (device Linv index rpos[k]*b+j; padding: -1)
};

bool build_sweep_layout(const int* nn_rowmajor, int n, int b, const int* colors,
                        const double* locs_colmajor, int d, SweepLayout& L, std::string& err);

// Level sets of the Vecchia DAG for the sparse triangular solve:
// level(i) = 1 + max level(NN(i)), level 0 rows have no neighbours.
void dag_levels(const int* nn_rowmajor, int n, int b, std::vector<int>& level_ptr,
                std::vector<int>& level_rows);

}  // namespace nngp
