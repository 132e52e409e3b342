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

// Device layout of the chromatic sweep ("sliced ELL with per-slot lane groups").
//  - slots: locations re-indexed colour-major; inside a colour grouped by
//    spatial tile (a Morton range) and boundary/interior class, Morton order
//    inside a group;
//  - r / field / Linv rows: Morton rank of the location (rpos);
//  - chunks: one wavefront over a Morton-contiguous run of slots of one
//    group; slot i gets k_i = 2^lk_i lanes (aligned sub-group, k_i lanes
//    cover ceil(len_i / kRowsMax) <= k_i), so no lane holds more than
//    kRowsMax entries and the chunk stays spatially compact (its r gathers and
//    scatters hit a few Morton-contiguous lines);
//  - lane_tab[ch*64 + lane] = (slot + 1) | lk << 28 (0: idle lane);
//  - entry j of slot i lives at ch * kRowsMax * 64 + (j / k_i) * 64 + o_i + j % k_i
//    (o_i = first lane of the slot's group; fixed chunk stride).
constexpr int kRowsMax = 16;  // entries per lane of a sweep chunk (== kSweepRows)

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
  std::vector<int> chunk_nslot;      // nchunks: slots in the chunk
  std::vector<int> chunk_lk;         // nchunks: log2(max k over the chunk's slots)
  std::vector<int> lane_tab;         // nchunks x 64
  std::vector<long long> chunk_off;  // nchunks
  // spatial tiles for the persistent sweep: tile(loc) = rpos[loc]*T/n
  int n_tiles = 1;
  std::vector<int> tile_chunks;      // (K*T) x 3: chunk range [a, m) boundary, [m, e) interior of (colour, tile)
  std::vector<int> nbr_ptr;          // T+1: CSR of neighbour tiles (moral-graph edges across tiles)
  std::vector<int> nbr_idx;
  long long n_boundary = 0;          // slots with a moral neighbour in another tile
  std::vector<int> ent_rowpos;       // n_entries (padding: 0)
  std::vector<int> ent_src;          // n_entries (device Linv index rpos[k]*b+j; padding: -1)
};

// n_tiles: spatial tiles (Morton ranges) for the persistent sweep (>= 1).
bool build_sweep_layout(const int* nn_rowmajor, int n, int b, const int* colors,
                        const double* locs_colmajor, int d, int n_tiles, SweepLayout& L,
                        std::string& err);

// Level sets of the Vecchia DAG for the sparse triangular solve:
// level(i) = 1 + max level(NN(i)), level 0 rows have no neighbours.
void dag_levels(const int* nn_rowmajor, int n, int b, std::vector<int>& level_ptr,
                std::vector<int>& level_rows);

}  // namespace nngp
