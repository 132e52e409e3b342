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

// Device layout of the chromatic sweep ("merge-path slot streams").
//  - r / field / Linv rows: Morton rank of the location (rpos);
//  - chunk: one chain group of a wavefront (LW lanes = floor(64 / chains per
//    wave)) x kRowsMax rows = LW*16 entry cells.  A chunk holds a contiguous
//    run of whole locations ("slots") of one colour, Morton order, at most
//    2*LW - 1 of them: their columns of B concatenated in the lane-major
//    stream f = lane*16 + row, so a column may continue from one lane into
//    the next; the unused tail of the stream is padding.  Every chunk has the
//    same size, so cell k of chunk ch is entry ch*LW*16 + k, loaded by lane
//    k % LW in row k / LW (coalesced loads, no metadata in front of them).
//    Inside a chunk the cells are sorted by their row of B (rowpos), so the
//    64 lanes of one load/gather/scatter instruction touch a few consecutive
//    lines of r; ent_pos[e] (uint16) is the cell's stream position f, through
//    which the kernel regroups the products by slot in LDS;
//  - ent_pk[e] = rowpos | q << 25 (padding: rowpos = kPadRow, q = 2*LW - 1);
//  - compact order: the locations colour-major, Morton order inside a colour
//    (= chunk order); chunk ch holds compact indices [chunk_first[ch],
//    chunk_first[ch+1]), slot q of the chunk is compact index chunk_first[ch]+q.
//    Per-slot data (column length, first stream cell f0, per-chain state and
//    normals) is stored in compact order.
constexpr int kRowsMax = 16;          // rows per lane (== kSweepRows)
constexpr int kRowBits = 25;          // rowpos bits of ent_pk (n < 2^25)
constexpr int kPadRow = (1 << kRowBits) - 1;

struct SweepLayout {
  int n = 0, b = 0, K = 0, nchunks = 0, LW = 64;
  long long nnz = 0, n_entries = 0;
  int max_collen = 0;
  std::vector<int> color_chunk_ptr;  // K+1
  std::vector<int> rpos;             // n: loc -> device row (Morton rank): r, field, Linv rows
  std::vector<int> collen;           // n, compact order
  std::vector<int> slot_f0;          // n, compact order
  std::vector<int> ent_pk;           // n_entries
  std::vector<int> ent_src;          // n_entries (device Linv index rpos[k]*b+j; padding: -1)
  std::vector<uint16_t> ent_pos;     // n_entries: stream position of the cell
  std::vector<uint16_t> start_mask;  // nchunks x LW: bit j = stream cell lane*16+j starts a slot (or the padding tail)
  std::vector<int> compact_loc;      // n: location at each compact index
  std::vector<int> color_loc_ptr;    // K+1: compact range of each colour
  std::vector<int> chunk_first;      // nchunks+1: first compact index of each chunk
};

// lanes_per_chain: 64, 32, 21 or 16 (1, 2, 3 or 4 chains per wavefront).  Fails if
// a column of B is longer than a chunk (lanes_per_chain * 16 entries) or n
// does not fit the packed row index.
bool build_sweep_layout(const int* nn_rowmajor, int n, int b, const int* colors,
                        const double* locs_colmajor, int d, int lanes_per_chain, SweepLayout& L,
                        std::string& err);

// Level sets of the Vecchia DAG for the sparse triangular solve:
// level(i) = 1 + max level(NN(i)), level 0 rows have no neighbours.
void dag_levels(const int* nn_rowmajor, int n, int b, std::vector<int>& level_ptr,
                std::vector<int>& level_rows);

}  // namespace nngp
