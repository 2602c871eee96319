// grid.h — multi-frame neighbour grid shared by outlier.hip (single clouds) and filter_batch.hip (frame batches).
//
// A cloud of n points grouped in F frames (frame f = point indices [foff[f], foff[f+1])) is binned into cubic cells
// of size h anchored at a per-frame origin.  Keys pack (frame, x, y, z) with z in the low bits, so a frame's points
// stay one contiguous range of the sorted order and cells (x', y', z-R .. z+R) of one frame are ONE contiguous range
// whichever of them are occupied.  The hash is over COLUMNS (frame, x, y) -> the column's run of occupied cells in
// the sorted cell list, so any z-range of a column costs one probe plus a short scan of the column's cells.  Per
// occupied cell the 3x3 (and optionally 5x5) column ranges of its block are precomputed.  The grid only decides
// which candidates a query scans, never a result.
#pragma once

#include "common.h"

namespace ot {

constexpr int NBR3 = 9;   // 3x3 columns, z-1 .. z+1
constexpr int NBR5 = 25;  // 5x5 columns, z-2 .. z+2

// SOR (outlier.hip): radius (in cells) of the block a query scans first, and the matching cell occupancy target
// (points per occupied cell of a surface-like cloud); both only change speed, never a result.  Measured and settled
// (DESIGN.md §4): R = 2 with finer cells, occupancies 0.6-1.3 k, precomputed 5x5 ranges for stage 2 -- all slower.
constexpr int SOR_BLOCK_R = 1;
inline double sor_cell_target(int nb_neighbors) {
    const double t = 0.9 * (double)nb_neighbors;
    return t > 2.0 ? t : 2.0;
}

// neighbour structures a grid build can precompute (bit mask)
enum { GRID_NBR3 = 1, GRID_NBR5 = 2 };
constexpr int SOR_GRID_NBR = GRID_NBR3;

struct GridDev {
    const double* sxyz;        // [n][3] points in sorted (frame, cell) order
    const unsigned* sidx;      // sorted position -> point index (nullptr: the identity, a presorted cloud)
    const unsigned long long* pkey;  // sorted position -> its cell key (the cell a query's guards are measured from)
    const int* pcell;          // sorted position -> cell (position in the sorted cell list)
    const int2* nbr3;          // per cell: NBR3 column ranges
    const int2* nbr5;          // per cell: NBR5 column ranges (nullptr unless built)
    unsigned long long* hkeys; // column hash: keys (cell key >> sy; KEY_EMPTY = free)
    int2* hval;                // column hash: {first cell, number of cells} (cells sorted by z inside a column)
    int hash_mask;
    int2* crange;              // per cell: [start, end) in the sorted order
    int* cz;                   // per cell: z
    int dim[3];                // cells per axis (every frame's cells lie in [0, dim))
    int sy, sx, sf;            // key = f << sf | x << sx | y << sy | z
    const double* origin;      // [F][3] per-frame grid origins (device)
    const int* foff;           // [F + 1] frame offsets (device; the same in input and sorted order)
    int nframes;
    double h;
};

struct GridBuild {
    GridDev g;
    int64_t ncells = 0;
};

// Build the grid of n points (xyz device [n][3]) grouped in nframes frames.  d_foff / d_origin: device arrays
// ([F+1] ints, [F][3] doubles) that must outlive the grid; dims: cells per axis covering every frame; nbr: the
// GRID_* structures to precompute; h_foff (optional host copy of the frame offsets, <= 64 frames): the cell sort
// runs per frame (segmented, cell bits only) instead of over frame-prefixed keys.  Scratch
// slots slot0 .. slot0 + 2.  Synchronises (cell count).
ot_status build_grid_frames(const double* xyz, int64_t n, int nframes, const int* d_foff, const double* d_origin,
                            double h, const int dims[3], int nbr, hipStream_t stream, GridBuild& out, int slot0,
                            const int* h_foff = nullptr);

// The grid of a cloud already in cell order (filter_batch.hip: voxels sorted by cell-major keys): ckeys[i] = point i's
// cell key (frame << (bits[0] + bits[1] + bits[2]) | x << (bits[1] + bits[2]) | y << bits[2] | z, non-decreasing),
// cells of edge h at the per-frame origins; no sort, no copy (the grid reads xyz in place).  Scratch slots slot0 ..
// slot0 + 2.  Synchronises (cell count).
ot_status build_grid_sorted(const double* xyz, const unsigned long long* ckeys, int64_t n, int nframes,
                            const int* d_foff, const double* d_origin, double h, const int bits[3], int nbr,
                            hipStream_t stream, GridBuild& out, int slot0);

// Statistical outlier removal over a built grid (Open3D RemoveStatisticalOutliers per frame):
// avg[i] = mean kNN distance of point i (-1 when none); per frame the cloud mean and squared-deviation sum are
// Open3D's sequential float64 accumulations (exact chains), stats[f] = {mean, std, valid, threshold}.
// h_foff: host copy of the frame offsets.  Scratch slots slot0 .. slot0 + 1.  Synchronises once (job table).
ot_status sor_frames(const GridBuild& gb, int64_t n, const int* h_foff, int nb_neighbors, double std_ratio,
                     double* avg, double* stats, hipStream_t stream, int slot0);

// The statistics half of sor_frames: from the mean kNN distances avg[0 .. n) (frame-major, d_foff / h_foff: device /
// host frame offsets) to stats[f] = {mean, std, valid, threshold}.  Scratch slot `slot`.  Synchronises once.
ot_status sor_stats_frames(const double* avg, const int* d_foff, const int* h_foff, int F, double std_ratio,
                           double* stats, hipStream_t stream, int slot);

// keep predicate of frame f's points: avg > 0 && avg < stats[f].threshold
struct SorKeep {
    const double* avg;
    const double* stats;  // [F][4]
    const int* foff;
    int nframes;
    __device__ inline bool operator()(int64_t i) const {
        int lo = 0, hi = nframes;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (foff[mid] <= i) lo = mid;
            else hi = mid;
        }
        const double a = avg[i];
        return a > 0 && a < stats[lo * 4 + 3];
    }
};

}  // namespace ot
