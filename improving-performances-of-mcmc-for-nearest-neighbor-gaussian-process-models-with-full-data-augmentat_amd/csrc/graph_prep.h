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
void hilbert_keys(const double* locs_colmajor, int n, int d, std::vector<uint64_t>& keys);

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


// Device layout of the tile-resident chromatic sweep (one persistent launch
// per call; DESIGN.md "Tile-resident sweep").
//  - tiles: T contiguous ranges of the Morton order (device rows), balanced
//    by column work; tile t owns the locations / rows of its range;
//  - local rows of tile t (E_t): every row of B with a member in t -- its own
//    rows first (local row = Morton rank - tile start), then the foreign
//    ("ghost") rows in Morton order; r of these rows lives in the tile's LDS
//    for the whole call;
//  - compact (slot) order: tile-major, then colour, then Morton;
//  - own batches of (tile, colour): runs of <= 256 whole slots and <= NT*RMAX
//    cells (the slots' columns of B, concatenated in stream order f); cell f of
//    a batch with R = ceil(cells/NT) rows sits at entry off + (f % R)*NT + f / R
//    (thread f / R, register f % R: coalesced loads, contiguous runs per
//    thread).  cell_pk = local row | q << 17 | start << 30 | end << 31
//    (q = slot inside the batch; start/end: first/last cell of a slot);
//    padding cells carry local row kTilePadRow and no flags;
//  - foreign slots of (tile, colour): the distinct foreign members j of colour
//    c of the tile's local rows (the tile reads each one's published dw_j once);
//  - ghost cells of (tile, colour): (local row k, index of j in the foreign
//    slots of (tile, colour)): r_k += B[k,j] dw_j once j's owner has published dw_j;
//  - neighbours of (tile, colour): the owner tiles of those ghost slots.
constexpr int kTileRowBits = 17;
constexpr uint32_t kTilePadRow = (1u << kTileRowBits) - 1;
constexpr int kTileQShift = 17;
constexpr uint32_t kTileQMask = 0x7FF;  // q < 2048
constexpr uint32_t kCellStart = 1u << 30;
constexpr uint32_t kCellEnd = 1u << 31;
constexpr int kSlotExported = 1 << 30;  // slot_f0 flag: dw of the slot is read by other tiles
constexpr int kTileSlotsMax = 256;      // slots per own batch

// dynamic LDS of one sweep_tiles_kernel workgroup (tiles.hip sweep_tiles_body
// lays it out in this order): r of max_rows local rows x C (0: r in global
// memory), slot totals kTileSlotsMax x C, NT/64 wave totals x C, C x 4 scalars,
// the dw of max_gslots foreign slots x C, max_batches batch records, 4 x (K+1)
// colour pointers, NT/64 wave flags, 64 B of probe words.  Host code (the
// engine choice at context creation, the layout checks of tests/cpp) and the
// launch use this one definition.
int tile_lds_bytes(int max_rows, int C, int NT, int K, int max_batches, int max_gslots);
constexpr int kTileCuLds = 160 * 1024;  // LDS per CU (MI355X)

// nthr = ceil(cells / R): threads holding cells (the others hold padding only)
struct TileBatch { int off, R, nslots, slot0, nthr; };

struct TileLayout {
  int n = 0, b = 0, K = 0, T = 0, NT = 0, RMAX = 0;  // NT: cell threads of a batch (the stream width)
  int NTK = 0;                       // threads of the sweep workgroup (NT, or NT + 64: exchange wave)
  long long nnz = 0;
  int max_rows = 0;                  // max |E_t|
  int max_batches = 0;               // max own batches of a tile
  int max_collen = 0;
  std::vector<int> rpos;             // n: loc -> device row (Morton rank)
  std::vector<int> compact_loc;      // n: slot -> loc
  std::vector<int> slot_f0;          // n: first stream cell inside its batch | kSlotExported
  std::vector<int> tile_row0;        // T+1: device rows owned by each tile
  std::vector<int> erow_ptr, erow;   // local rows of each tile -> device row
  std::vector<TileBatch> batch;      // own batches, grouped by (tile, colour)
  std::vector<int> batch_ptr;        // T*K + 1
  // split layouts (interior first): the slots of (tile, colour c) whose rows
  // have no foreign member of colour c-1 (cyclic) come first, in batches of
  // their own; batch_split[t*K + c] = the first batch of the others
  // ("boundary" slots: they wait for the hand-off of colour c-1)
  bool split = false;
  std::vector<int> batch_split;      // T*K (split layouts)
  std::vector<uint32_t> cell_pk;     // own cells (padded batches)
  std::vector<int> cell_src;         // device Linv index rpos[k]*b + j, or -1 (padding)
  std::vector<int> gcell;            // 2 per ghost cell: local row, index of its foreign slot
  std::vector<int> gsrc;             // device Linv index of each ghost cell
  std::vector<int> gptr;             // T*K + 1
  std::vector<int> gslot;            // foreign slots (slot index) of each (tile, colour)
  std::vector<int> gslot_ptr;        // T*K + 1
  int max_gslots = 0;                // max foreign slots of a (tile, colour)
  std::vector<int> nb_ptr, nb;       // T*K + 1, neighbour tiles of each (tile, colour)
  // tile-sharded sweep over G ranks (G > 1): rank g runs tiles [g*T/G, (g+1)*T/G)
  // and owns their slots [rank_slot0[g], rank_slot0[g+1]) (slot order is tile-major)
  int G = 1;
  std::vector<int> rank_slot0;       // G + 1
  std::vector<uint32_t> rmask;       // n (G > 1): bit h = a tile of rank h != the owner's reads the slot's dw
  // wave-local layouts (W = waves > 0; NT = 64): every batch is one wave's
  // (<= kWaveSlotsMax slots, 64 lanes x R cells), and the batches of a (tile,
  // colour) come in rounds of W balanced by cells -- wave w of the tile runs
  // batches first + w, first + w + W, ... with no workgroup barrier inside a
  // colour (the batches of one colour touch disjoint rows of B)
  int W = 0;
};
constexpr int kWaveSlotsMax = 42;  // slots of a wave-local batch (7 x 42 = 294 >= the 257 slots of the
                                   // largest colour of a headline tile: one round)
// slot totals a tile workgroup keeps in LDS (acc_s): a workgroup batch's
// kTileSlotsMax, or the 7 cell waves' wave-local batches of a 512-thread tile
constexpr int kAccSlots = 7 * kWaveSlotsMax > kTileSlotsMax ? 7 * kWaveSlotsMax : kTileSlotsMax;

// Fails (returns false, err set) when the layout does not fit the packed
// formats; the caller checks the LDS budget (max_rows).
// G > 1: the tiles of a G-rank tile shard (T a multiple of G, G <= kMaxTileRanks):
// also the ranks' slot ranges and the remote-reader mask of every slot.
constexpr int kMaxTileRanks = 16;
bool build_tile_layout(const int* nn_rowmajor, int n, int b, const int* colors, const double* locs_colmajor,
                       int d, int T, int NT, int RMAX, TileLayout& L, std::string& err, int G = 1,
                       bool split = false, int waves = 0);

// Colour-sharded sweep over G ranks on top of a
// SweepLayout (every rank builds the same layout from the same inputs):
//  - rank g owns, in every colour c, the chunks whose first slot has a Morton
//    rank in [g*n/G, (g+1)*n/G): a contiguous chunk range, hence a contiguous
//    compact range [seg0[c][g], seg0[c][g+1]) of the colour's slots -- the
//    same spatial block of the domain in every colour;
//  - exchange region of colour c: G x cnt[c] slots (cnt = the largest rank
//    segment of the colour), slot units; rank g's segment starts at g*cnt[c];
//    after colour c every rank holds {dw, w_new} of every slot of the colour
//    (one all-gather);
//  - ghost cells of colour c: (device row k, Linv index of B[k,j], exchange
//    index of j) for every row k the rank's own columns touch (any colour) and
//    every foreign member j of colour c of that row: r_k += B[k,j] dw_j.  A
//    row has at most one member per colour, so own and ghost updates of a
//    colour never touch the same row;
//  - pairs of colour c: normal pairs (2p, 2p+1) generated by the colour of 2p
//    with at least one member owned by the rank.
constexpr int kMaxRanks = 64;

struct ShardPlan {
  int G = 1, rank = 0, K = 0;
  std::vector<int> cb;          // K x (G+1): chunk boundaries of the ranks inside each colour
  std::vector<int> seg0;        // K x (G+1): compact boundaries of the ranks inside each colour
  std::vector<int> cnt;         // K: all-gather count of each colour (slots per rank, padded)
  std::vector<long long> xoff;  // K+1: exchange region of each colour (slot units)
  std::vector<int> gptr;        // K+1: ghost cells of each colour
  std::vector<int> grow;        // device row of each ghost cell
  std::vector<int> gsrc;        // device Linv index (row-major n x b) of B[k, j]
  std::vector<int> grecv;       // exchange index of j (slot units, relative to xoff[c])
  std::vector<int> pair_ptr;    // K+1
  std::vector<int> pairs;       // normal pairs of the rank, grouped by the colour of 2p
  long long owned = 0;          // slots owned by the rank
  long long needed_rows = 0;    // rows of B the rank's columns touch
};

bool build_shard_plan(const int* nn_rowmajor, int n, int b, const int* colors, const SweepLayout& L, int G,
                      int rank, ShardPlan& P, std::string& err);

// Level sets of the Vecchia DAG for the sparse triangular solve:
// level(i) = 1 + max level(NN(i)), level 0 rows have no neighbours.
void dag_levels(const int* nn_rowmajor, int n, int b, std::vector<int>& level_ptr,
                std::vector<int>& level_rows);

}  // namespace nngp
