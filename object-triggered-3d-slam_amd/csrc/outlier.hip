// outlier.hip — PointCloud::RemoveStatisticalOutliers / RemoveRadiusOutliers on MI355X.
//
// Neighbour search uses a uniform cell grid instead of Open3D's KD-tree (the results are defined by the
// distances, not by the search structure):
//   grid build : cell key per point -> stable radix sort (cell, index) -> cell heads -> open-addressing hash
//                (cell key -> [start, end) in the sorted order); points are re-laid out in sorted order so a
//                cell's points are contiguous in HBM.
//   ROR        : cell = radius; count |{j : d2(i, j) < r^2}| over the 27 neighbour cells (exact integers).
//   SOR        : exact k nearest neighbours by shell expansion: cells at Chebyshev ring 0, 1, 2, ... are
//                scanned into a register-resident sorted top-k list until the k-th distance is provably
//                inside the scanned cube.  Distances d2 = ((dx*dx + dy*dy) + dz*dz) (nanoflann L2 order),
//                sqrt'ed and summed in ascending order, divided by the count (std::accumulate in Open3D).
//                Cloud mean / std use a fixed-order two-level reduction in float64.
// Queries run in sorted (cell) order, so a wave's neighbourhoods overlap and stay in L2.
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "compact.h"
#include "sort.h"

namespace ot {

struct GridDev {
    const double* sxyz;           // points in sorted (cell) order [n][3]
    const unsigned* sidx;         // sorted position -> original index
    const int* pcell;             // sorted position -> cell index (position in the sorted cell list)
    const int2* nbr3;             // per cell: 9 merged z-column ranges covering its 3x3x3 cell block
    const int2* nbr5;             // per cell: 25 merged z-column ranges covering its 5x5x5 block (SOR only)
    unsigned long long* hkeys;    // cell hash keys (compact keys, KEY_EMPTY = free)
    int2* hval;                   // cell hash values: [start, end) in the sorted order
    int hash_mask;
    int dim[3];                   // cells per axis (cell coordinates are >= 0: origin = the cloud's minimum)
    int sy, sx;                   // key = x << sx | y << sy | z  (z in the low bits)
    double origin[3];
    double h;
};

// A block of cells around a cell as z-columns: cells (x', y', z-R .. z+R) have consecutive keys, so their points
// are ONE contiguous range of the sorted order whichever of those cells are occupied.  The 3x3x3 block is 9
// ranges, the 5x5x5 block 25; a 5-column minus its 3-column is the two ranges on either side.
constexpr int NBR3 = 9;
constexpr int NBR5 = 25;

__device__ inline int cell_coord(double v, double origin, double h) { return (int)floor((v - origin) / h); }

__device__ inline bool cell_valid(const GridDev& g, int x, int y, int z) {
    return x >= 0 && x < g.dim[0] && y >= 0 && y < g.dim[1] && z >= 0 && z < g.dim[2];
}
__device__ inline unsigned long long cell_key(const GridDev& g, int x, int y, int z) {
    return ((unsigned long long)x << g.sx) | ((unsigned long long)y << g.sy) | (unsigned long long)z;
}

__device__ inline int2 grid_probe(const GridDev& g, unsigned long long key, unsigned slot) {
    for (int probe = 0; probe <= g.hash_mask; ++probe) {
        const unsigned long long k = g.hkeys[slot];
        if (k == key) return g.hval[slot];
        if (k == KEY_EMPTY) return make_int2(0, 0);
        slot = (slot + 1) & (unsigned)g.hash_mask;
    }
    return make_int2(0, 0);
}

__device__ inline int2 grid_find(const GridDev& g, int x, int y, int z) {
    if (!cell_valid(g, x, y, z)) return make_int2(0, 0);
    const unsigned long long key = cell_key(g, x, y, z);
    return grid_probe(g, key, (unsigned)mix64(key) & (unsigned)g.hash_mask);
}

__global__ __launch_bounds__(256) void k_cell_keys(const double* __restrict__ xyz, int64_t n, GridDev g,
                                                   unsigned long long* keys, unsigned* idx, int* err) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int x = cell_coord(xyz[i * 3 + 0], g.origin[0], g.h);
    const int y = cell_coord(xyz[i * 3 + 1], g.origin[1], g.h);
    const int z = cell_coord(xyz[i * 3 + 2], g.origin[2], g.h);
    if (!cell_valid(g, x, y, z)) *err = 1;
    keys[i] = cell_valid(g, x, y, z) ? cell_key(g, x, y, z) : 0ull;
    idx[i] = (unsigned)i;
}

// per occupied cell: hash insert of [start, end)
__global__ __launch_bounds__(256) void k_grid_insert(const unsigned long long* __restrict__ skeys,
                                                     const int* __restrict__ heads, int64_t ncells, int64_t n,
                                                     GridDev g) {
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= ncells) return;
    const int beg = heads[c];
    const int end = (c + 1 < ncells) ? heads[c + 1] : (int)n;
    const unsigned long long key = skeys[beg];
    unsigned slot = (unsigned)mix64(key) & (unsigned)g.hash_mask;
    while (true) {  // capacity >= 2 * ncells: always terminates
        const unsigned long long old = atomicCAS(&g.hkeys[slot], KEY_EMPTY, key);
        if (old == KEY_EMPTY) {
            g.hval[slot] = make_int2(beg, end);
            return;
        }
        slot = (slot + 1) & (unsigned)g.hash_mask;
    }
}

// One lane per (cell, z-column of its (2R+1)^2 neighbourhood): 2R+1 hash lookups whose first probes are issued
// together, merged into the column's range over z-R..z+R (and, R = 2, over z-1..z+1 for the inner 3x3 columns).
template <int R>
__global__ __launch_bounds__(256) void k_cell_nbr(const unsigned long long* __restrict__ skeys,
                                                  const int* __restrict__ heads, int64_t ncells, GridDev g,
                                                  int2* __restrict__ nbr3, int2* __restrict__ nbr5) {
    constexpr int W = 2 * R + 1, COLS = W * W;
    const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (gid >= ncells * COLS) return;
    const int64_t c = gid / COLS;
    const int t = (int)(gid - c * COLS);
    const int dx = t / W - R, dy = t % W - R;
    const unsigned long long key = skeys[heads[c]];
    const int z = (int)(key & ((1ull << g.sy) - 1));
    const int y = (int)((key >> g.sy) & ((1ull << (g.sx - g.sy)) - 1)) + dy;
    const int x = (int)(key >> g.sx) + dx;
    unsigned long long kq[W];
    unsigned slot[W];
    unsigned long long k0[W];
    bool valid[W];
#pragma unroll
    for (int i = 0; i < W; ++i) {
        valid[i] = cell_valid(g, x, y, z + i - R);
        kq[i] = valid[i] ? cell_key(g, x, y, z + i - R) : 0ull;
        slot[i] = (unsigned)mix64(kq[i]) & (unsigned)g.hash_mask;
    }
#pragma unroll
    for (int i = 0; i < W; ++i) k0[i] = valid[i] ? g.hkeys[slot[i]] : KEY_EMPTY;
    int2 se[W];
#pragma unroll
    for (int i = 0; i < W; ++i) {
        se[i] = make_int2(0, 0);
        if (valid[i] && k0[i] != KEY_EMPTY)
            se[i] = (k0[i] == kq[i]) ? g.hval[slot[i]] : grid_probe(g, kq[i], (slot[i] + 1) & (unsigned)g.hash_mask);
    }
    int b5 = 0x7FFFFFFF, e5 = 0, b3 = 0x7FFFFFFF, e3 = 0;
#pragma unroll
    for (int i = 0; i < W; ++i)
        if (se[i].y > se[i].x) {
            b5 = min(b5, se[i].x);
            e5 = max(e5, se[i].y);
            if (i >= R - 1 && i <= R + 1) {
                b3 = min(b3, se[i].x);
                e3 = max(e3, se[i].y);
            }
        }
    const int2 r5 = e5 > 0 ? make_int2(b5, e5) : make_int2(0, 0);
    const int2 r3 = e3 > 0 ? make_int2(b3, e3) : make_int2(0, 0);
    if (R == 2) nbr5[c * NBR5 + t] = r5;
    if (dx >= -1 && dx <= 1 && dy >= -1 && dy <= 1) nbr3[c * NBR3 + (dx + 1) * 3 + (dy + 1)] = r3;
}

__global__ __launch_bounds__(256) void k_gather_sorted(const double* __restrict__ xyz, const unsigned* __restrict__ sidx,
                                                       int64_t n, double* __restrict__ sxyz) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n * 3) return;
    const int64_t j = t / 3, a = t % 3;
    sxyz[t] = xyz[(int64_t)sidx[j] * 3 + a];
}

__device__ inline double d2_l2(const double* q, const double* p) {
    const double d0 = q[0] - p[0], d1 = q[1] - p[1], d2 = q[2] - p[2];
    return ((d0 * d0) + d1 * d1) + d2 * d2;
}

// ------------------------------------------------------------------------------------------------ ROR
// cell = radius: every neighbour within the radius lies in the 3x3x3 block, i.e. in the 9 merged ranges.
__global__ __launch_bounds__(256) void k_ror(GridDev g, int64_t n, double r2, int nb, unsigned char* keep) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    const double q[3] = {g.sxyz[j * 3], g.sxyz[j * 3 + 1], g.sxyz[j * 3 + 2]};
    const int2* rg = g.nbr3 + (int64_t)g.pcell[j] * NBR3;
    long long cnt = 0;
    for (int t = 0; t < NBR3; ++t) {
        const int2 se = rg[t];
        for (int k = se.x; k < se.y; ++k) cnt += d2_l2(q, g.sxyz + (int64_t)k * 3) < r2 ? 1 : 0;
    }
    keep[g.sidx[j]] = cnt > nb ? 1 : 0;
}

// ------------------------------------------------------------------------------------------------ SOR
// Register top-k list, RIGHT-aligned ascending: best[KMAX-kk .. KMAX-1] hold the kk smallest squared distances
// and best[0 .. KMAX-kk-1] = -inf.  Insertion is a branch-free min/max exchange chain, skipped for a whole wave
// when no lane's candidate beats its current k-th distance best[KMAX-1]; lanes whose candidate does not enter
// leave the list unchanged (their d is >= every entry).  NaN never enters (d < kth is false).
template <int KMAX>
__device__ inline void topk_insert(double (&best)[KMAX], double d) {
#pragma unroll
    for (int i = 0; i < KMAX; ++i) {
        const double lo = fmin(best[i], d);
        d = fmax(best[i], d);
        best[i] = lo;
    }
}

template <int KMAX>
__device__ inline void scan_range(const GridDev& g, const double q[3], int beg, int end, double (&best)[KMAX]) {
    for (int m = beg; m < end; ++m) {
        const double d = d2_l2(q, g.sxyz + (int64_t)m * 3);
        if (d < best[KMAX - 1]) topk_insert<KMAX>(best, d);
    }
}

template <int KMAX>
__device__ inline void topk_reset(double (&best)[KMAX], int kk) {
#pragma unroll
    for (int i = 0; i < KMAX; ++i) best[i] = (i < KMAX - kk) ? -INFINITY : INFINITY;
}

constexpr int SOR_RMAX = 8;  // beyond this ring a query falls back to an exact scan of every point

// Exact kNN for a query the 5x5x5 block does not settle (isolated points): Chebyshev shell expansion through the
// hash until the k-th distance lies inside the scanned cube, else a scan of the whole cloud.
template <int KMAX>
__device__ inline void sor_fallback(const GridDev& g, const double q[3], int64_t n, int kk,
                                                       double (&best)[KMAX]) {
    const int cx = cell_coord(q[0], g.origin[0], g.h), cy = cell_coord(q[1], g.origin[1], g.h),
              cz = cell_coord(q[2], g.origin[2], g.h);
    topk_reset<KMAX>(best, kk);
    long long have = 0;
    for (int r = 0; r <= SOR_RMAX; ++r) {
        for (int dx = -r; dx <= r; ++dx)
            for (int dy = -r; dy <= r; ++dy) {
                const bool face = (dx == -r || dx == r || dy == -r || dy == r);
                for (int dz = -r; dz <= r; dz += (face || r == 0) ? 1 : 2 * r) {
                    const int2 se = grid_find(g, cx + dx, cy + dy, cz + dz);
                    scan_range<KMAX>(g, q, se.x, se.y, best);
                    have += se.y - se.x;
                }
            }
        if (have >= kk) {
            const double kth = best[KMAX - 1];
            // every point within distance (r - margin) * h of q lies in rings 0..r
            const double guard = (r > 0 ? (double)r - 0.01 : 0.0) * g.h;
            if (kth <= guard * guard || have >= n) return;
        }
    }
    topk_reset<KMAX>(best, kk);
    scan_range<KMAX>(g, q, 0, (int)n, best);
}

// distance from q to the faces of its (2R+1)^3 cell block, minus a rounding margin
__device__ inline double block_guard(const GridDev& g, const double q[3], double R) {
    double guard = (R + 1.0) * g.h;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double u = (q[a] - g.origin[a]) / g.h;
        const double f = u - floor(u);
        guard = fmin(guard, fmin(R + f, R + 1.0 - f) * g.h);
    }
    return guard - 1e-6 * g.h;
}

#ifndef OT_SOR_SKIP
#define OT_SOR_SKIP 1
#endif

// One lane per query (sorted order: a wave's queries share cells and candidate ranges).  Stage 1 scans the 9
// ranges of the query's 3x3x3 block; the k-th distance is final when it does not exceed the distance from q to
// the block's faces (>= h).  Stage 2 adds the rest of the 5x5x5 block (guard >= 2h).  Isolated points fall back.
template <int KMAX>
__global__ __launch_bounds__(256) void k_sor_knn(GridDev g, int64_t n, int k, double* avg) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    const double q[3] = {g.sxyz[j * 3], g.sxyz[j * 3 + 1], g.sxyz[j * 3 + 2]};
    const int kk = (int)((int64_t)k < n ? k : n);
    double best[KMAX];
    topk_reset<KMAX>(best, kk);
    const int c = g.pcell[j];
    const int2* r3 = g.nbr3 + (int64_t)c * NBR3;
    long long have = 0;
#if OT_SOR_SKIP
    // distances from q to its cell's faces in x and y (conservatively shrunk): a neighbouring column (dx, dy) lies
    // at least sqrt(ex^2 + ey^2) away, so once that reaches the current k-th distance none of its points can enter
    double lo[2], hi[2];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        const double uu = (q[a] - g.origin[a]) / g.h;
        const double fr = uu - floor(uu);
        lo[a] = fmax(fr * g.h * (1.0 - 1e-9) - 1e-12 * g.h, 0.0);
        hi[a] = fmax((1.0 - fr) * g.h * (1.0 - 1e-9) - 1e-12 * g.h, 0.0);
    }
#endif
    for (int u = 0; u < NBR3; ++u) {
        // own column, then the 4 face-adjacent columns, then the 4 diagonal ones: the k-th distance tightens
        // before the farthest candidates, so fewer of them pass the early-reject test into the insertion chain
        const int t = (int)((0x862075314ull >> (4 * u)) & 0xF);
        const int2 se = r3[t];
#if OT_SOR_SKIP
        const int dx = t / 3 - 1, dy = t % 3 - 1;
        const double ex = dx < 0 ? lo[0] : (dx > 0 ? hi[0] : 0.0);
        const double ey = dy < 0 ? lo[1] : (dy > 0 ? hi[1] : 0.0);
        if (!(ex * ex + ey * ey >= best[KMAX - 1]))
#endif
            scan_range<KMAX>(g, q, se.x, se.y, best);
        have += se.y - se.x;
    }
    double guard = block_guard(g, q, 1.0);
    bool settled = have >= n || (have >= kk && best[KMAX - 1] <= guard * guard);
    int stage = 1;
    if (!settled) {
        stage = 2;
        const int2* r5 = g.nbr5 + (int64_t)c * NBR5;
        for (int t = 0; t < NBR5; ++t) {
            const int dx = t / 5 - 2, dy = t % 5 - 2;
            const int2 o = r5[t];
            if (dx >= -1 && dx <= 1 && dy >= -1 && dy <= 1) {
                const int2 i3 = r3[(dx + 1) * 3 + (dy + 1)];
                if (i3.y > i3.x) {  // the column's cells at z-2 and z+2 only
                    scan_range<KMAX>(g, q, o.x, i3.x, best);
                    scan_range<KMAX>(g, q, i3.y, o.y, best);
                    have += (o.y - o.x) - (i3.y - i3.x);
                    continue;
                }
            }
            scan_range<KMAX>(g, q, o.x, o.y, best);
            have += o.y - o.x;
        }
        guard = block_guard(g, q, 2.0);
        settled = have >= n || (have >= kk && best[KMAX - 1] <= guard * guard);
        if (!settled) {
            stage = 3;
#ifndef OT_SOR_NOFB  // timing-only ablation build: isolated queries skip the exact fallback (results wrong)
            sor_fallback<KMAX>(g, q, n, kk, best);
#endif
        }
    }
    double s = 0.0;
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < KMAX; ++i)
        if (i >= KMAX - kk && best[i] < INFINITY) {
            s += sqrt(best[i]);
            ++cnt;
        }
#ifdef OT_SOR_DIAG  // diagnostic build (tools/sor_work.py): (sorted position, stage, candidates scanned)
    avg[g.sidx[j]] = (double)((j << 26) | ((long long)stage << 24) | (have < (1 << 24) ? have : (1 << 24) - 1));
#else
    (void)stage;
    avg[g.sidx[j]] = cnt > 0 ? s / (double)cnt : -1.0;
#endif
}

// ------------------------------------------------------------------------------------ cross-cloud 1-NN distance
// PointCloud::ComputePointCloudDistance (eval_cone.py:99,103): per source point the distance to its nearest target
// point, sqrt of the exact float64 squared distance.  The grid is built over the target.  A query inside the
// target's bounding box whose cell is occupied runs the SOR stages (3x3x3 then 5x5x5 block of its cell); any other
// query expands Chebyshev rings around the cell of q' = clamp(q, box).  For every target point p (inside the box)
// |q - p|^2 >= |q - q'|^2 + |q' - p|^2, so the ring guard of q' plus |q - q'|^2 bounds every unscanned point.
constexpr int NN_RMAX = 6;

__device__ inline int2 grid_cell_range(const GridDev& g, int x, int y, int z, int& cell) {
    const int2 se = grid_find(g, x, y, z);
    cell = se.y > se.x ? g.pcell[se.x] : -1;
    return se;
}

__device__ inline void nn_range(const GridDev& g, const double q[3], int beg, int end, double& best) {
    for (int m = beg; m < end; ++m) best = fmin(best, d2_l2(q, g.sxyz + (int64_t)m * 3));
}

__global__ __launch_bounds__(256) void k_nn_dist(GridDev g, const double* __restrict__ src, int64_t n, int64_t m,
                                                 double mnx, double mny, double mnz, double mxx, double mxy,
                                                 double mxz, double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const double q[3] = {src[i * 3], src[i * 3 + 1], src[i * 3 + 2]};
    const double lo[3] = {mnx, mny, mnz}, hi[3] = {mxx, mxy, mxz};
    double qc[3], off2 = 0.0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        qc[a] = fmin(fmax(q[a], lo[a]), hi[a]);
        const double dd = q[a] - qc[a];
        off2 += dd * dd;
    }
    // lower bound used only for the stopping test: shave a relative margin off the exact-arithmetic bound
    off2 *= (1.0 - 1e-9);
    double best = INFINITY;
    bool settled = false;
    const int cx = cell_coord(qc[0], g.origin[0], g.h), cy = cell_coord(qc[1], g.origin[1], g.h),
              cz = cell_coord(qc[2], g.origin[2], g.h);
    if (off2 == 0.0) {
        int c;
        grid_cell_range(g, cx, cy, cz, c);
        if (c >= 0) {
            const int2* r3 = g.nbr3 + (int64_t)c * NBR3;
            for (int u = 0; u < NBR3; ++u) {
                const int2 se = r3[(u + 4) % NBR3];
                nn_range(g, q, se.x, se.y, best);
            }
            double guard = block_guard(g, q, 1.0);
            settled = best <= guard * guard;
            if (!settled) {
                const int2* r5 = g.nbr5 + (int64_t)c * NBR5;
                for (int t = 0; t < NBR5; ++t) {
                    const int dx = t / 5 - 2, dy = t % 5 - 2;
                    const int2 o = r5[t];
                    if (dx >= -1 && dx <= 1 && dy >= -1 && dy <= 1) {
                        const int2 i3 = r3[(dx + 1) * 3 + (dy + 1)];
                        if (i3.y > i3.x) {
                            nn_range(g, q, o.x, i3.x, best);
                            nn_range(g, q, i3.y, o.y, best);
                            continue;
                        }
                    }
                    nn_range(g, q, o.x, o.y, best);
                }
                guard = block_guard(g, q, 2.0);
                settled = best <= guard * guard;
            }
        }
    }
    if (!settled) {
        best = INFINITY;
        long long have = 0;
        for (int r = 0; r <= NN_RMAX && !settled; ++r) {
            for (int dx = -r; dx <= r; ++dx)
                for (int dy = -r; dy <= r; ++dy) {
                    const bool face = (dx == -r || dx == r || dy == -r || dy == r);
                    for (int dz = -r; dz <= r; dz += (face || r == 0) ? 1 : 2 * r) {
                        const int2 se = grid_find(g, cx + dx, cy + dy, cz + dz);
                        nn_range(g, q, se.x, se.y, best);
                        have += se.y - se.x;
                    }
                }
            const double guard = (r > 0 ? (double)r - 0.01 : 0.0) * g.h;
            if (have >= m || (have > 0 && best <= off2 + guard * guard)) settled = true;
        }
        if (!settled) {
            best = INFINITY;
            nn_range(g, q, 0, (int)m, best);
        }
    }
    out[i] = sqrt(best);
}

// fixed-order two-level reduction: blocks reduce contiguous chunks in a fixed tree, then one block reduces
// the block partials in the same fixed order.  mode 0: sum of avg > 0 and count; mode 1: sum of (avg-mean)^2
__global__ __launch_bounds__(256) void k_sor_partial(const double* __restrict__ avg, int64_t n, int mode,
                                                     const double* __restrict__ stats, double* partial,
                                                     long long* pcount) {
    __shared__ double sd[256];
    __shared__ long long sc[256];
    const int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
    const int64_t beg = (int64_t)blockIdx.x * chunk, end = beg + chunk < n ? beg + chunk : n;
    double acc = 0.0;
    long long c = 0;
    const double mean = mode == 1 ? stats[0] : 0.0;
    for (int64_t i = beg + threadIdx.x; i < end; i += 256) {
        const double a = avg[i];
        if (a > 0) {
            acc += mode == 0 ? a : (a - mean) * (a - mean);
            ++c;
        }
    }
    sd[threadIdx.x] = acc;
    sc[threadIdx.x] = c;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            sd[threadIdx.x] += sd[threadIdx.x + s];
            sc[threadIdx.x] += sc[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        partial[blockIdx.x] = sd[0];
        pcount[blockIdx.x] = sc[0];
    }
}

__global__ __launch_bounds__(256) void k_sor_final(const double* partial, const long long* pcount, int nb, int mode,
                                                   double std_ratio, double* stats) {
    __shared__ double sd[256];
    __shared__ long long sc[256];
    double acc = 0.0;
    long long c = 0;
    for (int i = threadIdx.x; i < nb; i += 256) {
        acc += partial[i];
        c += pcount[i];
    }
    sd[threadIdx.x] = acc;
    sc[threadIdx.x] = c;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            sd[threadIdx.x] += sd[threadIdx.x + s];
            sc[threadIdx.x] += sc[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (mode == 0) {
            stats[2] = (double)sc[0];                  // valid
            stats[0] = sc[0] > 0 ? sd[0] / (double)sc[0] : 0.0;  // cloud mean
        } else {
            const double valid = stats[2];
            const double sdv = sqrt(sd[0] / (valid - 1.0));
            stats[1] = sdv;
            stats[3] = stats[0] + std_ratio * sdv;  // threshold
        }
    }
}

struct SorPred {
    const double* avg;
    const double* stats;
    __device__ bool operator()(int64_t i) const {
        const double a = avg[i];
        return a > 0 && a < stats[3];
    }
};
struct RorPred {
    const unsigned char* keep;
    __device__ bool operator()(int64_t i) const { return keep[i] != 0; }
};
struct IndexEmit {
    int64_t* out;
    __device__ void operator()(int64_t i, int64_t pos) const { out[pos] = i; }
};

// ------------------------------------------------------------------------------------ grid builder (host)
struct GridBuild {
    GridDev g;
    int64_t ncells = 0;
};

static int bits_for_host(int64_t v) {  // bits to represent 0..v
    int b = 1;
    while (b < 62 && (v >> b) != 0) ++b;
    return b;
}

// Cell grid of size h anchored at the cloud's minimum corner (mn, mx: exact bounds on the host).  Keys are
// compact (only the bits the extent needs), so the stable radix sort runs ceil(bits / 8) passes.  with5: also
// build the 5x5x5 ranges (SOR).
static ot_status build_grid(const double* xyz, int64_t n, double h, const double mn[3], const double mx[3], bool with5,
                            hipStream_t stream, GridBuild& out) {
    GridDev& g = out.g;
    g.h = h;
    int bits[3];
    for (int a = 0; a < 3; ++a) {
        g.origin[a] = mn[a];
        const double span = std::floor((mx[a] - mn[a]) / h);
        if (!(span < 1.0e6)) return fail(OT_ERR_INVALID_ARGUMENT, "neighbour grid out of range (radius too small for the extent)");
        g.dim[a] = (int)span + 1;
        bits[a] = bits_for_host(g.dim[a] - 1);
    }
    g.sy = bits[2];
    g.sx = bits[1] + bits[2];
    const int end_bit = bits[0] + bits[1] + bits[2];
    char* ws = (char*)scratch(256 + (size_t)n * (8 + 8 + 4 + 4 + 4 + 4 + 24), 8);
    if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
    int* err = (int*)ws;
    unsigned long long* kin = (unsigned long long*)(ws + 256);
    unsigned long long* kout = kin + n;
    unsigned* vin = (unsigned*)(kout + n);
    unsigned* vout = vin + n;
    int* heads = (int*)(vout + n);
    int* pcell = heads + n;
    double* sxyz = (double*)(((uintptr_t)(pcell + n) + 15) & ~(uintptr_t)15);
    OT_HIP_TRY(hipMemsetAsync(err, 0, sizeof(int), stream));
    hipLaunchKernelGGL(k_cell_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, xyz, n, g, kin, vin, err);
    OT_LAUNCH_CHECK();
    ot_status st = sort_pairs_u64_u32(kin, kout, vin, vout, (size_t)n, end_bit, stream, 3);
    if (st != OT_OK) return st;
    int64_t ncells = 0;
    st = compact_segments(n, kout, heads, pcell, stream, &ncells, 9);  // synchronises
    if (st != OT_OK) return st;
    int e = 0;
    OT_HIP_TRY(hipMemcpyAsync(&e, err, sizeof(int), hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipStreamSynchronize(stream));
    if (e) return fail(OT_ERR_INVALID_ARGUMENT, "neighbour grid out of range (non-finite point coordinates)");
    int64_t cap = 1;
    while (cap < 2 * ncells + 2) cap <<= 1;
    char* hs = (char*)scratch((size_t)cap * (8 + 8) + (size_t)ncells * (NBR3 + (with5 ? NBR5 : 0)) * 8 + 64, 10);
    if (!hs) return fail(OT_ERR_HIP, "scratch allocation failed");
    g.hkeys = (unsigned long long*)hs;
    g.hval = (int2*)(g.hkeys + cap);
    int2* nbr3 = g.hval + cap;
    int2* nbr5 = with5 ? nbr3 + ncells * NBR3 : nullptr;
    g.hash_mask = (int)(cap - 1);
    OT_HIP_TRY(hipMemsetAsync(g.hkeys, 0xFF, sizeof(unsigned long long) * cap, stream));
    hipLaunchKernelGGL(k_grid_insert, dim3((unsigned)((ncells + 255) / 256)), dim3(256), 0, stream, kout, heads,
                       ncells, n, g);
    if (with5)
        hipLaunchKernelGGL(k_cell_nbr<2>, dim3((unsigned)((ncells * NBR5 + 255) / 256)), dim3(256), 0, stream, kout,
                           heads, ncells, g, nbr3, nbr5);
    else
        hipLaunchKernelGGL(k_cell_nbr<1>, dim3((unsigned)((ncells * NBR3 + 255) / 256)), dim3(256), 0, stream, kout,
                           heads, ncells, g, nbr3, nbr5);
    hipLaunchKernelGGL(k_gather_sorted, dim3((unsigned)((n * 3 + 255) / 256)), dim3(256), 0, stream, xyz, vout, n, sxyz);
    OT_LAUNCH_CHECK();
    g.sxyz = sxyz;
    g.sidx = vout;
    g.pcell = pcell;
    g.nbr3 = nbr3;
    g.nbr5 = nbr5;
    out.ncells = ncells;
    return OT_OK;
}

}  // namespace ot

using namespace ot;

static ot_status bounds_host(const double* xyz, int64_t n, hipStream_t stream, double mn[3], double mx[3]) {
    Bounds* b = (Bounds*)scratch(sizeof(Bounds) + 64, 11);
    if (!b) return fail(OT_ERR_HIP, "scratch allocation failed");
    unsigned long long* part = (unsigned long long*)scratch(sizeof(unsigned long long) * BOUNDS_BLOCKS * 6, 19);
    if (!part) return fail(OT_ERR_HIP, "scratch allocation failed");
    launch_bounds(xyz, n, b, part, stream);
    OT_LAUNCH_CHECK();
    Bounds hb;
    OT_HIP_TRY(hipMemcpyAsync(&hb, b, sizeof(Bounds), hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipStreamSynchronize(stream));
    for (int a = 0; a < 3; ++a) {
        mn[a] = ordered_to_dbl(hb.mn[a]);
        mx[a] = ordered_to_dbl(hb.mx[a]);
    }
    return OT_OK;
}

extern "C" {

ot_status ot_remove_radius_outlier(const double* xyz, int64_t n, int32_t nb_points, double radius,
                                   int64_t* out_indices, int64_t* n_kept_host, void* stream_) {
    hipStream_t stream = S(stream_);
    if (nb_points < 1 || !(radius > 0))
        return fail(OT_ERR_INVALID_ARGUMENT, "[RemoveRadiusOutliers] Illegal input parameters, number of points "
                                             "and radius must be positive");
    if (!n_kept_host) return fail(OT_ERR_INVALID_ARGUMENT, "[RemoveRadiusOutliers] n_kept is NULL");
    *n_kept_host = 0;
    if (n <= 0) return OT_OK;
    if (!xyz || !out_indices || n > 0x7FFFFFFF) return fail(OT_ERR_INVALID_ARGUMENT, "[RemoveRadiusOutliers] invalid buffers");
    double mn[3], mx[3];
    ot_status st = bounds_host(xyz, n, stream, mn, mx);
    if (st != OT_OK) return st;
    GridBuild gb;
    st = build_grid(xyz, n, radius, mn, mx, false, stream, gb);
    if (st != OT_OK) return st;
    unsigned char* keep = (unsigned char*)scratch((size_t)n + 64, 12);
    if (!keep) return fail(OT_ERR_HIP, "scratch allocation failed");
    hipLaunchKernelGGL(k_ror, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, gb.g, n, radius * radius,
                       (int)nb_points, keep);
    OT_LAUNCH_CHECK();
    return compact(n, RorPred{keep}, IndexEmit{out_indices}, stream, n_kept_host, 13);
}

ot_status ot_remove_statistical_outlier(const double* xyz, int64_t n, int32_t nb_neighbors, double std_ratio,
                                        int64_t* out_indices, double* out_avg_dist, int64_t* n_kept_host,
                                        void* stream_) {
    hipStream_t stream = S(stream_);
    if (nb_neighbors < 1 || !(std_ratio > 0))
        return fail(OT_ERR_INVALID_ARGUMENT, "[RemoveStatisticalOutliers] Illegal input parameters, the number of "
                                             "neighbors and standard deviation ratio must be positive.");
    if (nb_neighbors > 64)
        return fail(OT_ERR_INVALID_ARGUMENT, "[RemoveStatisticalOutliers] nb_neighbors > 64 is not supported");
    if (!n_kept_host) return fail(OT_ERR_INVALID_ARGUMENT, "[RemoveStatisticalOutliers] n_kept is NULL");
    *n_kept_host = 0;
    if (n <= 0) return OT_OK;
    if (!xyz || !out_indices || n > 0x7FFFFFFF)
        return fail(OT_ERR_INVALID_ARGUMENT, "[RemoveStatisticalOutliers] invalid buffers");
    double mn[3], mx[3];
    ot_status st = bounds_host(xyz, n, stream, mn, mx);
    if (st != OT_OK) return st;
    // Cell size: the grid only changes speed, never the result.  Aim for ~occ_target points per occupied cell
    // of a surface-like cloud (0.7 k: the k-th neighbour then lies ~0.7 h away, inside the 3x3x3 block that settles
    // most queries).  First guess: the points cover half of the bounding box's largest face; refined once from the
    // measured occupancy (2-D scaling) when it is off by more than 2.5x.
    const double k = (double)nb_neighbors;
    static const double occ_env = [] {
        const char* e = std::getenv("OT_SOR_OCC");
        return e ? std::atof(e) : 0.0;
    }();
    const double target = occ_env > 0.0 ? occ_env : std::max(0.7 * k, 2.0);
    double ext[3];
    for (int a = 0; a < 3; ++a) ext[a] = std::max(mx[a] - mn[a], 1e-9);
    std::sort(ext, ext + 3);
    const double hmin = ext[2] / 5.0e5;
    double h = std::max(std::sqrt(0.5 * ext[2] * ext[1] * target / (double)n), hmin);
    GridBuild gb;
    st = build_grid(xyz, n, h, mn, mx, true, stream, gb);
    if (st != OT_OK) return st;
    const double occ = (double)n / (double)std::max<int64_t>(gb.ncells, 1);
    if (occ > 2.5 * target || occ < 0.4 * target) {
        h = std::max(h * std::sqrt(target / occ), hmin);
        st = build_grid(xyz, n, h, mn, mx, true, stream, gb);
        if (st != OT_OK) return st;
    }
    char* ws = (char*)scratch((size_t)n * 8 + 1024 * 16 + 256, 12);
    if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
    double* stats = (double*)ws;                  // [0] mean [1] std [2] valid [3] threshold
    double* partial = (double*)(ws + 64);         // 1024
    long long* pcount = (long long*)(ws + 64 + 1024 * 8);
    double* avg = out_avg_dist ? out_avg_dist : (double*)(ws + 256 + 1024 * 16);
    const unsigned grid = (unsigned)((n + 255) / 256);
    const int kk = (int)std::min<int64_t>(nb_neighbors, n);  // list length actually needed
#define OT_SOR_LAUNCH(KM) \
    hipLaunchKernelGGL(k_sor_knn<KM>, dim3(grid), dim3(256), 0, stream, gb.g, n, (int)nb_neighbors, avg)
    if (kk <= 4) OT_SOR_LAUNCH(4);
    else if (kk <= 8) OT_SOR_LAUNCH(8);
    else if (kk <= 12) OT_SOR_LAUNCH(12);
    else if (kk <= 16) OT_SOR_LAUNCH(16);
    else if (kk <= 20) OT_SOR_LAUNCH(20);
    else if (kk <= 24) OT_SOR_LAUNCH(24);
    else if (kk <= 32) OT_SOR_LAUNCH(32);
    else if (kk <= 48) OT_SOR_LAUNCH(48);
    else OT_SOR_LAUNCH(64);
#undef OT_SOR_LAUNCH
    const int nb = (int)std::min<int64_t>(1024, (n + 255) / 256);
    hipLaunchKernelGGL(k_sor_partial, dim3(nb), dim3(256), 0, stream, avg, n, 0, stats, partial, pcount);
    hipLaunchKernelGGL(k_sor_final, dim3(1), dim3(256), 0, stream, partial, pcount, nb, 0, std_ratio, stats);
    hipLaunchKernelGGL(k_sor_partial, dim3(nb), dim3(256), 0, stream, avg, n, 1, stats, partial, pcount);
    hipLaunchKernelGGL(k_sor_final, dim3(1), dim3(256), 0, stream, partial, pcount, nb, 1, std_ratio, stats);
    OT_LAUNCH_CHECK();
    return compact(n, SorPred{avg, stats}, IndexEmit{out_indices}, stream, n_kept_host, 13);
}


ot_status ot_compute_point_cloud_distance(const double* src, int64_t n, const double* tgt, int64_t m, double* out,
                                          void* stream_) {
    hipStream_t stream = S(stream_);
    if (n < 0 || m < 0) return fail(OT_ERR_INVALID_ARGUMENT, "[ComputePointCloudDistance] negative size");
    if (n == 0) return OT_OK;
    if (!src || !out || (m > 0 && !tgt) || n > 0x7FFFFFFF || m > 0x7FFFFFFF)
        return fail(OT_ERR_INVALID_ARGUMENT, "[ComputePointCloudDistance] invalid buffers");
    if (m == 0) {  // Open3D: no neighbour found -> 0.0
        OT_HIP_TRY(hipMemsetAsync(out, 0, sizeof(double) * (size_t)n, stream));
        OT_HIP_TRY(hipStreamSynchronize(stream));
        return OT_OK;
    }
    double mn[3], mx[3];
    ot_status st = bounds_host(tgt, m, stream, mn, mx);
    if (st != OT_OK) return st;
    // ~4 target points per occupied cell of a surface-like cloud (the grid only changes speed)
    double ext[3];
    for (int a = 0; a < 3; ++a) ext[a] = std::max(mx[a] - mn[a], 1e-9);
    std::sort(ext, ext + 3);
    const double target = 4.0;
    const double hmin = ext[2] / 5.0e5;
    double h = std::max(std::sqrt(0.5 * ext[2] * ext[1] * target / (double)m), hmin);
    GridBuild gb;
    st = build_grid(tgt, m, h, mn, mx, true, stream, gb);
    if (st != OT_OK) return st;
    const double occ = (double)m / (double)std::max<int64_t>(gb.ncells, 1);
    if (occ > 2.5 * target || occ < 0.4 * target) {
        h = std::max(h * std::sqrt(target / occ), hmin);
        st = build_grid(tgt, m, h, mn, mx, true, stream, gb);
        if (st != OT_OK) return st;
    }
    hipLaunchKernelGGL(k_nn_dist, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, gb.g, src, n, m, mn[0],
                       mn[1], mn[2], mx[0], mx[1], mx[2], out);
    OT_LAUNCH_CHECK();
    OT_HIP_TRY(hipStreamSynchronize(stream));
    return OT_OK;
}

}  // extern "C"
