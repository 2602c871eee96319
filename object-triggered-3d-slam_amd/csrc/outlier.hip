// outlier.hip — PointCloud::RemoveStatisticalOutliers / RemoveRadiusOutliers / ComputePointCloudDistance on
// MI355X (eval_cone.py:99-110).
//
// Neighbour search uses a uniform cell grid (grid.h) instead of Open3D's KD-tree (the results are defined by the
// distances, not by the search structure):
//   grid build : (frame, cell) key per point -> stable radix sort -> cell heads -> open-addressing hash (cell key ->
//                [start, end) in the sorted order) -> per cell the z-column ranges of its 3x3 / 5x5 block; points
//                are re-laid out in sorted order so a cell's points are contiguous in HBM.
//   ROR        : cell = radius; count |{j : d2(i, j) < r^2}| over the 27 neighbour cells (exact integers).
//   SOR        : exact k nearest neighbours: the columns of the query's block are scanned nearest-first into a
//                register-resident sorted top-k list (columns that cannot hold a closer point are skipped) until the
//                k-th distance is provably inside the scanned block, else Chebyshev rings continue it.  Distances
//                d2 = ((dx*dx + dy*dy) + dz*dz) (nanoflann L2 order), sqrt'ed and summed in ascending order, divided
//                by the count (std::accumulate).  The cloud mean and squared-deviation sum are Open3D's sequential
//                float64 accumulations, computed exactly by the chain kernels (chain.h); `valid` counts every point
//                with a non-empty neighbour list (Open3D: valid_distances), the sums take only avg > 0.
// Queries run in sorted (cell) order, so a wave's neighbourhoods overlap and stay in L1/L2.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "chain.h"
#include "compact.h"
#include "grid.h"
#include "sort.h"

namespace ot {

__device__ inline int cell_coord(double v, double origin, double h) { return (int)floor((v - origin) / h); }

__device__ inline bool cell_valid(const GridDev& g, int x, int y, int z) {
    return x >= 0 && x < g.dim[0] && y >= 0 && y < g.dim[1] && z >= 0 && z < g.dim[2];
}
__device__ inline unsigned long long cell_key(const GridDev& g, int f, int x, int y, int z) {
    return ((unsigned long long)f << g.sf) | ((unsigned long long)x << g.sx) | ((unsigned long long)y << g.sy) |
           (unsigned long long)z;
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

// the occupied cells of column (f, x, y): {first cell, count}
__device__ inline int2 grid_column(const GridDev& g, int f, int x, int y) {
    if (x < 0 || x >= g.dim[0] || y < 0 || y >= g.dim[1]) return make_int2(0, 0);
    const unsigned long long key = cell_key(g, f, x, y, 0) >> g.sy;
    return grid_probe(g, key, (unsigned)mix64(key) & (unsigned)g.hash_mask);
}

// points of the column's cells with zlo <= z <= zhi: one contiguous range of the sorted order (or empty)
__device__ inline int2 column_range(const GridDev& g, int2 col, int zlo, int zhi) {
    int b = 0, e = 0;
    bool any = false;
    int i0 = 0;
    if (col.y > 8) {  // tall column (a wall seen edge-on): bisect for the first cell with z >= zlo
        int lo = -1, hi = col.y;  // cz[lo] < zlo <= cz[hi]
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (g.cz[col.x + mid] < zlo) lo = mid;
            else hi = mid;
        }
        i0 = hi;
    }
    for (int i = i0; i < col.y; ++i) {
        const int z = g.cz[col.x + i];
        if (z > zhi) break;
        if (z >= zlo) {
            const int2 r = g.crange[col.x + i];
            if (!any) b = r.x;
            e = r.y;
            any = true;
        }
    }
    return any ? make_int2(b, e) : make_int2(0, 0);
}

__device__ inline int2 grid_find(const GridDev& g, int f, int x, int y, int z) {
    return column_range(g, grid_column(g, f, x, y), z, z);
}

// the cell the grid assigned to sorted point j (its key): SOR measures every guard from this cell's faces, so a
// point the rounding of its coordinates puts a hair outside its cell still gets correct (conservative) bounds
__device__ inline void query_cell(const GridDev& g, int64_t j, int& cx, int& cy, int& cz) {
    const unsigned long long key = g.pkey[j];
    cz = (int)(key & ((1ull << g.sy) - 1));
    cy = (int)((key >> g.sy) & ((1ull << (g.sx - g.sy)) - 1));
    cx = (int)((key >> g.sx) & ((1ull << (g.sf - g.sx)) - 1));
}
__device__ inline int64_t sor_out(const GridDev& g, int64_t j) { return g.sidx ? (int64_t)g.sidx[j] : j; }
// the frame of sorted point j: its cell key's frame field (one load, which query_cell makes anyway, instead of a
// dependent binary search over the frame offsets at the head of every query's chain)
__device__ inline int sorted_frame(const GridDev& g, int64_t j) {
    return g.nframes > 1 ? (int)(g.pkey[j] >> g.sf) : 0;
}

template <typename KeyT>
__global__ __launch_bounds__(256) void k_cell_keys(const double* __restrict__ xyz, int64_t n, GridDev g, KeyT* keys,
                                                   unsigned* idx, int* err) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int f = g.nframes > 1 ? frame_of(g.foff, g.nframes, i) : 0;
    const double* o = g.origin + 3 * f;
    const int x = cell_coord(xyz[i * 3 + 0], o[0], g.h);
    const int y = cell_coord(xyz[i * 3 + 1], o[1], g.h);
    const int z = cell_coord(xyz[i * 3 + 2], o[2], g.h);
    const bool ok = cell_valid(g, x, y, z);
    if (!ok) *err = 1;
    keys[i] = ok ? (KeyT)cell_key(g, f, x, y, z) : (KeyT)0;
    idx[i] = (unsigned)i;
}

__global__ __launch_bounds__(256) void k_widen_keys(const unsigned* __restrict__ in, int64_t n,
                                                    unsigned long long* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = in[i];
}

// per occupied cell: its range and z; a column's first cell also inserts the column (its run of cells) into the hash
__global__ __launch_bounds__(256) void k_grid_insert(const unsigned long long* __restrict__ skeys,
                                                     const int* __restrict__ heads, int64_t ncells, int64_t n,
                                                     GridDev g) {
    const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= ncells) return;
    const int beg = heads[c];
    const int end = (c + 1 < ncells) ? heads[c + 1] : (int)n;
    const unsigned long long key = skeys[beg];
    g.crange[c] = make_int2(beg, end);
    g.cz[c] = (int)(key & ((1ull << g.sy) - 1));
    const unsigned long long col = key >> g.sy;
    if (c > 0 && (skeys[heads[c - 1]] >> g.sy) == col) return;
    // the column's cells are contiguous (cell-major keys): its end by galloping, then bisection -- a wall's column
    // holds dozens of cells, and a probe is two dependent loads
    int64_t lo = c, hi = ncells, step = 1;
    while (true) {
        const int64_t p = c + step;
        if (p >= ncells) break;
        if ((skeys[heads[p]] >> g.sy) != col) {
            hi = p;
            break;
        }
        lo = p;
        step <<= 1;
    }
    while (hi - lo > 1) {  // colkey(lo) == col; hi == ncells or colkey(hi) != col
        const int64_t mid = (lo + hi) >> 1;
        if ((skeys[heads[mid]] >> g.sy) == col) lo = mid;
        else hi = mid;
    }
    const int cnt = (int)(hi - c);
    unsigned slot = (unsigned)mix64(col) & (unsigned)g.hash_mask;
    while (true) {  // capacity >= 2 * ncells >= 2 * columns: always terminates
        const unsigned long long old = atomicCAS(&g.hkeys[slot], KEY_EMPTY, col);
        if (old == KEY_EMPTY) {
            g.hval[slot] = make_int2((int)c, cnt);
            return;
        }
        slot = (slot + 1) & (unsigned)g.hash_mask;
    }
}

// One lane per (cell, column of its (2R+1)^2 neighbourhood): one column probe, then the column's cells in
// z-R..z+R (and, R = 2, z-1..z+1 for the inner 3x3 columns) as contiguous point ranges.
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
    const int f = (int)(key >> g.sf);
    const int z = (int)(key & ((1ull << g.sy) - 1));
    const int y = (int)((key >> g.sy) & ((1ull << (g.sx - g.sy)) - 1)) + dy;
    const int x = (int)((key >> g.sx) & ((1ull << (g.sf - g.sx)) - 1)) + dx;
    const int2 col = grid_column(g, f, x, y);
    if (R == 2) nbr5[c * NBR5 + t] = column_range(g, col, z - 2, z + 2);
    if (nbr3 && dx >= -1 && dx <= 1 && dy >= -1 && dy <= 1)
        nbr3[c * NBR3 + (dx + 1) * 3 + (dy + 1)] = column_range(g, col, z - 1, z + 1);
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
// and best[0 .. KMAX-kk-1] = -inf.  Inserting d (< best[KMAX-1]) keeps the kk smallest of the list and d: entry i
// becomes max(best[i-1], min(best[i], d)) -- i < p keeps best[i], i == p takes d, i > p takes best[i-1] for the
// insertion position p -- so every entry is two independent min/max (no serial dependency through the list).
// Skipped for a whole wave when no lane's candidate beats its k-th distance; NaN never enters (d < kth is false).
// fmin / fmax in IEEE mode cost a v_max_f64 canonicalisation of each operand the compiler cannot prove canonical (the
// loop-carried list): one extra instruction per min/max.  Every operand here is a product of arithmetic or of these
// selections (canonical, never NaN), so the bare instructions give the same values.
__device__ inline double dmin(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ inline double dmax(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// Issue order: the min of entry i - 1 goes between the min and the max of entry i, so no max reads the result of the
// instruction right before it (a dependent float64 pair needs a wait state: one s_nop per entry otherwise); entry i - 1
// is still the old value when entry i's max reads it.
template <int KMAX>
__device__ inline void topk_insert(double (&best)[KMAX], double d) {
    double m = dmin(best[KMAX - 1], d);
#pragma unroll
    for (int i = KMAX - 1; i > 0; --i) {
        const double mi = m;
        m = dmin(best[i - 1], d);
        best[i] = dmax(best[i - 1], mi);
    }
    best[0] = m;
}

// candidates [beg, end) of the sorted points, two per step with both rows loaded before either is tested
template <int KMAX>
__device__ inline void scan_range(const double* __restrict__ P, const double q[3], int beg, int end,
                                  double (&best)[KMAX]) {
    int m = beg;
    for (; m + 2 <= end; m += 2) {
        const double* p = P + (int64_t)m * 3;
        const double a[3] = {p[0], p[1], p[2]}, b[3] = {p[3], p[4], p[5]};
        const double da = d2_l2(q, a), db = d2_l2(q, b);
        if (da < best[KMAX - 1]) topk_insert<KMAX>(best, da);
        if (db < best[KMAX - 1]) topk_insert<KMAX>(best, db);
    }
    if (m < end) {
        const double d = d2_l2(q, P + (int64_t)m * 3);
        if (d < best[KMAX - 1]) topk_insert<KMAX>(best, d);
    }
}

// Sorting network for the first KMAX candidates of a query (its own column's first ones): Batcher's odd-even merge
// sort for 32 inputs restricted to the comparators among the first KMAX positions -- valid because inputs past KMAX
// would be +inf, which every comparator keeps at the higher index (checked exhaustively for 20 inputs with the 0-1
// principle when generated).  103 compare-exchanges instead of KMAX sequential insertions of ~2 KMAX min / max each.
constexpr unsigned char k_net20[103][2] = {  // compile-time indices: the list stays in registers
    {0, 1}, {2, 3}, {4, 5}, {6, 7}, {8, 9}, {10, 11}, {12, 13}, {14, 15}, {16, 17}, {18, 19}, {0, 2}, {1, 3}, {4, 6},
    {5, 7}, {8, 10}, {9, 11}, {12, 14}, {13, 15}, {16, 18}, {17, 19}, {1, 2}, {5, 6}, {9, 10}, {13, 14}, {17, 18},
    {0, 4}, {1, 5}, {2, 6}, {3, 7}, {8, 12}, {9, 13}, {10, 14}, {11, 15}, {2, 4}, {3, 5}, {10, 12}, {11, 13}, {1, 2},
    {3, 4}, {5, 6}, {9, 10}, {11, 12}, {13, 14}, {17, 18}, {0, 8}, {1, 9}, {2, 10}, {3, 11}, {4, 12}, {5, 13},
    {6, 14}, {7, 15}, {4, 8}, {5, 9}, {6, 10}, {7, 11}, {2, 4}, {3, 5}, {6, 8}, {7, 9}, {10, 12}, {11, 13}, {1, 2},
    {3, 4}, {5, 6}, {7, 8}, {9, 10}, {11, 12}, {13, 14}, {17, 18}, {0, 16}, {1, 17}, {2, 18}, {3, 19}, {8, 16},
    {9, 17}, {10, 18}, {11, 19}, {4, 8}, {5, 9}, {6, 10}, {7, 11}, {12, 16}, {13, 17}, {14, 18}, {15, 19}, {2, 4},
    {3, 5}, {6, 8}, {7, 9}, {10, 12}, {11, 13}, {14, 16}, {15, 17}, {1, 2}, {3, 4}, {5, 6}, {7, 8}, {9, 10},
    {11, 12}, {13, 14}, {15, 16}, {17, 18}};
template <int KMAX>
__device__ inline void sort_net(double (&v)[KMAX]) {
    static_assert(KMAX == 20, "network for 20 inputs");
#pragma unroll
    for (int c = 0; c < 103; ++c) {
        const int a = k_net20[c][0], b = k_net20[c][1];
        const double lo = dmin(v[a], v[b]), hi = dmax(v[a], v[b]);
        v[a] = lo;
        v[b] = hi;
    }
}

template <int KMAX>
__device__ inline void topk_reset(double (&best)[KMAX], int kk) {
#pragma unroll
    for (int i = 0; i < KMAX; ++i) best[i] = (i < KMAX - kk) ? -INFINITY : INFINITY;
}

// distance from q to the faces of the (2R+1)^3 cell block around cell c, minus a rounding margin (f = q's position
// inside c: in [0, 1) up to rounding; outside it the formula is still q's distance to the block's faces)
__device__ inline double block_guard(const GridDev& g, const double q[3], const double* o, const int c[3], double R) {
    double guard = (R + 1.0) * g.h;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double u = (q[a] - o[a]) / g.h;
        const double f = u - (double)c[a];
        guard = fmin(guard, fmin(R + f, R + 1.0 - f) * g.h);
    }
    return guard - 1e-6 * g.h;
}

// column visiting order of a (2R+1)^2 block, nearest first (t = (dx + R) * (2R + 1) + dy + R)
__constant__ unsigned char c_cols3[NBR3] = {4, 1, 3, 5, 7, 0, 2, 6, 8};
__constant__ unsigned char c_cols5[NBR5] = {12, 7, 11, 13, 17, 6, 8, 16, 18, 2, 10, 14, 22,
                                            1, 3, 5, 9, 15, 19, 21, 23, 0, 4, 20, 24};

// Queries stage 1 could not settle, deferred to a second launch so that its waves are full of them (a wave runs a
// stage for all its lanes when one lane needs it): sorted position, candidates counted, the top-k list (SoA).  Stage 2
// writes an unsettled query's count and list back into its slot and lists the slot for stage 3 (pd3: count and slots
// only, capacity n, so no query ever falls back to a serial ring walk -- that path held stage 2 at 162 VGPRs).
struct SorPend {
    int* count;
    int* j;
    long long* have;
    double* best;  // best[i * cap + slot]
    int64_t cap;
};

template <int KMAX>
__device__ inline double sor_mean(const double (&best)[KMAX], int kk) {
    double s = 0.0;
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < KMAX; ++i)
        if (i >= KMAX - kk && best[i] < INFINITY) {
            s += sqrt(best[i]);
            ++cnt;
        }
    return cnt > 0 ? s / (double)cnt : -1.0;
}

// distance from q to the near face of the column / cell at signed offset d (0: q's own), conservatively shrunk
__device__ inline double face_gap(double lo, double hi, int d, double h) {
    return d < 0 ? lo + (double)(-d - 1) * h : (d > 0 ? hi + (double)(d - 1) * h : 0.0);
}
__device__ inline void cell_fracs(const GridDev& g, const double q[3], const double* o, const int c[3], double lo[3],
                                  double hi[3]) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double uu = (q[a] - o[a]) / g.h;
        const double fr = uu - (double)c[a];  // q's place in its cell c (distances below clamp at 0 outside it)
        lo[a] = fmax(fr * g.h * (1.0 - 1e-9) - 1e-12 * g.h, 0.0);
        hi[a] = fmax((1.0 - fr) * g.h * (1.0 - 1e-9) - 1e-12 * g.h, 0.0);
    }
}

// Stage 1, one lane per query (sorted order: a wave's queries share cells and candidate ranges): the columns of the
// query's (2R+1)^3 block nearest-first into the register top-k list, a column skipped once its distance from q
// reaches the current k-th distance; the k-th distance is final when it does not exceed the distance from q to the
// block's faces.  Unsettled queries go to the pending list.
// Workgroups are dispatched round-robin over the 8 XCDs (each with its own L2): XCD x runs the blocks b = x mod 8.
// Block b is remapped so that XCD x takes one contiguous range of the sorted queries instead, keeping a query's
// neighbourhood in the L2 that the neighbouring workgroups (the neighbouring cells) just filled (a bijection of
// [0, G); configs[2] SOR -2 %).
__device__ inline int64_t xcd_block() {
    const int64_t b = blockIdx.x, G = gridDim.x;
    const int64_t x = b & 7, per = G >> 3, rem = G & 7;
    return x * per + (x < rem ? x : rem) + (b >> 3);
}

template <int KMAX, int R, bool NETFILL = true>
__global__ __launch_bounds__(256) void k_sor_knn(GridDev g, int64_t n, int k, double* avg, SorPend pd) {
    constexpr int W = 2 * R + 1;
    const int64_t j = xcd_block() * 256 + threadIdx.x;
    if (j >= n) return;
    const int f = sorted_frame(g, j);
    const int64_t fbeg = g.foff[f], fend = g.foff[f + 1];
    const double* o = g.origin + 3 * f;
    const double q[3] = {g.sxyz[j * 3], g.sxyz[j * 3 + 1], g.sxyz[j * 3 + 2]};
    const int kk = (int)((int64_t)k < fend - fbeg ? k : fend - fbeg);
    double best[KMAX];
    topk_reset<KMAX>(best, kk);
    const int c = g.pcell[j];
    const int2* rr = (R == 1 ? g.nbr3 + (int64_t)c * NBR3 : g.nbr5 + (int64_t)c * NBR5);
    int cc[3];
    query_cell(g, j, cc[0], cc[1], cc[2]);
    double lo[3], hi[3];
    cell_fracs(g, q, o, cc, lo, hi);
    long long have = 0;
    // The own column's first KMAX candidates fill the empty list at once: their distances, +inf past the column's end,
    // sorted by a network -- the list 20 sequential insertions would leave (each of the first KMAX is accepted, the
    // list holding +inf), so every later decision and the final sum are the same bits.  Only for lists of KMAX (kk <
    // KMAX lists keep their -inf padding and the sequential fill)
    int m0 = 0;
    if constexpr (KMAX == 20 && NETFILL) {
        const int2 se = rr[R == 1 ? c_cols3[0] : c_cols5[0]];
        m0 = kk == KMAX ? min(KMAX, se.y - se.x) : 0;
#pragma unroll
        for (int i = 0; i < KMAX; ++i)
            if (i < m0) best[i] = d2_l2(q, g.sxyz + (int64_t)(se.x + i) * 3);
        sort_net<KMAX>(best);
    }
    for (int u = 0; u < W * W; ++u) {
        const int t = R == 1 ? c_cols3[u] : c_cols5[u];
        const int dx = t / W - R, dy = t % W - R;
        const int2 se = rr[t];
        const double ex = face_gap(lo[0], hi[0], dx, g.h), ey = face_gap(lo[1], hi[1], dy, g.h);
        if (!(ex * ex + ey * ey >= best[KMAX - 1])) scan_range<KMAX>(g.sxyz, q, se.x + (u == 0 ? m0 : 0), se.y, best);
        have += se.y - se.x;
    }
    const double guard = block_guard(g, q, o, cc, (double)R);
    if (have >= fend - fbeg || (have >= kk && best[KMAX - 1] <= guard * guard)) {
        avg[sor_out(g, j)] = sor_mean<KMAX>(best, kk);
        return;
    }
    const unsigned long long m = __ballot(1);  // the wave's unsettled lanes: one atomic per wave
    const int leader = __ffsll((long long)m) - 1;
    int base = 0;
    if ((int)lane_id() == leader) base = atomicAdd(pd.count, __popcll(m));
    base = __shfl(base, leader);
    const int slot = base + __popcll(m & ((1ull << lane_id()) - 1));
    pd.j[slot] = (int)j;
    pd.have[slot] = have;
#pragma unroll
    for (int i = 0; i < KMAX; ++i) pd.best[(int64_t)i * pd.cap + slot] = best[i];
}

// Stage 2 for the pending queries (grid-stride over the device count): R = 1 completes the 5x5x5 block (the inner
// columns' cells at z-2 / z+2 and the 16 outer columns, each skipped when provably too far); what is still unsettled
// goes to stage 3.
template <int KMAX, int R>
__global__ __launch_bounds__(256) void k_sor_knn_rest(GridDev g, int k, double* avg, SorPend pd, SorPend pd3) {
    static_assert(R == 1 || R == 2, "stage 3 starts at ring 3");
    const int cnt = *pd.count;
    for (int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x; s < cnt; s += (int64_t)gridDim.x * 256) {
        const int64_t j = pd.j[s];
        const int f = sorted_frame(g, j);
        const int64_t fbeg = g.foff[f], fend = g.foff[f + 1];
        const double* o = g.origin + 3 * f;
        const double q[3] = {g.sxyz[j * 3], g.sxyz[j * 3 + 1], g.sxyz[j * 3 + 2]};
        const int kk = (int)((int64_t)k < fend - fbeg ? k : fend - fbeg);
        double best[KMAX];
#pragma unroll
        for (int i = 0; i < KMAX; ++i) best[i] = pd.best[(int64_t)i * pd.cap + s];
        long long have = pd.have[s];
        bool settled = false;
        int cc[3];
        query_cell(g, j, cc[0], cc[1], cc[2]);
        if (R == 1) {
            const int c = g.pcell[j];
            const int cx = cc[0], cy = cc[1], cz = cc[2];
            double lo[3], hi[3];
            cell_fracs(g, q, o, cc, lo, hi);
            const int2* r3 = g.nbr3 + (int64_t)c * NBR3;  // the inner columns' z-1 .. z+1 ranges (stage 1's)
            bool counted_all = true;  // have counts every point of the 5x5x5 block
#pragma nounroll
            for (int u = 0; u < NBR5; ++u) {
                const int t = c_cols5[u];
                const int dx = t / 5 - 2, dy = t % 5 - 2;
                const bool inner = dx >= -1 && dx <= 1 && dy >= -1 && dy <= 1;
                const double ex = face_gap(lo[0], hi[0], dx, g.h), ey = face_gap(lo[1], hi[1], dy, g.h);
                const double e2 = ex * ex + ey * ey;
                if (e2 >= best[KMAX - 1]) {  // the whole column is at least the k-th distance away: not even probed
                    counted_all = false;
                    continue;
                }
                const int2 full = column_range(g, grid_column(g, f, cx + dx, cy + dy), cz - 2, cz + 2);
                const int2 mid = inner ? r3[(dx + 1) * 3 + (dy + 1)] : make_int2(0, 0);
                if (inner && mid.y > mid.x) {  // the column's cells at z-2 and z+2 only
                    const double ez = face_gap(lo[2], hi[2], 2, g.h);  // both are >= one cell plus q's gap away
                    const double ezl = face_gap(lo[2], hi[2], -2, g.h);
                    if (!(e2 + ezl * ezl >= best[KMAX - 1])) scan_range<KMAX>(g.sxyz, q, full.x, mid.x, best);
                    if (!(e2 + ez * ez >= best[KMAX - 1])) scan_range<KMAX>(g.sxyz, q, mid.y, full.y, best);
                    have += (full.y - full.x) - (mid.y - mid.x);
                } else {
                    if (!(e2 >= best[KMAX - 1])) scan_range<KMAX>(g.sxyz, q, full.x, full.y, best);
                    have += full.y - full.x;
                }
            }
            const double guard = block_guard(g, q, o, cc, 2.0);
            // the list is full exactly when kk points were scanned (nothing is skipped while the k-th distance is
            // infinite); a skipped column lies beyond the k-th distance
            settled = (counted_all && have >= fend - fbeg) ||
                      (best[KMAX - 1] < INFINITY && best[KMAX - 1] <= guard * guard);
            if (!counted_all) have = -1;  // only a full count may end the rings through the whole-frame test
        }
        if (!settled) {  // stage 3 (one wave per query): the pending slot listed, its count and list back in place
            pd3.j[atomicAdd(pd3.count, 1)] = (int)s;  // capacity: every pending slot is listed at most once
            pd.have[s] = have;
            double* wp = pd.best + s;  // one running address (20 precomputed ones held stage 2 at 158 VGPRs)
#pragma unroll
            for (int i = 0; i < KMAX; ++i) {
                *wp = best[i];
                wp += pd.cap;
            }
            continue;
        }
        avg[sor_out(g, j)] = sor_mean<KMAX>(best, kk);
    }
}

// Stage 3: the few queries whose k-th distance lies beyond their 5x5x5 block (isolated points: 0.02-0.2 % of a
// configs[2] frame) — one WAVE per query.  Run by one lane each, their Chebyshev rings cost thousands of dependent
// hash probes in series and set the whole kernel's tail.  Here ring r's (2r+1)^2 columns are split over the lanes
// (outer columns: cells z-r..z+r, inner columns: z-r and z+r only, each skipped when provably beyond the current
// k-th distance); every lane keeps its own register list, and after each ring the wave merges the 64 lists into the
// shared list (LDS, kk extraction rounds of a wave-wide minimum).  Lane 0 starts a ring from the shared list and
// the other lanes from an empty list whose top is the shared k-th distance: a candidate enters only when it beats
// that, and a copy of the k-th value ties the real one, so the merged multiset of the kk smallest distances (all
// the mean needs) is exactly the serial walk's.  After SOR_RMAX3 rings the wave scans the whole frame.
constexpr int SOR_RMAX3 = 16;

__device__ inline double wave_min_d(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmin(v, __shfl_xor(v, off));
    return v;
}

// gl[0..KMAX) = the kk smallest of the 64 lanes' lists (ascending, right-aligned, -inf padding); lds: 64*KMAX
template <int KMAX>
__device__ inline void wave_merge(double* lds, double* gl, const double (&L)[KMAX], int kk) {
    const int l = (int)lane_id();
#pragma unroll
    for (int i = 0; i < KMAX; ++i) lds[i * 64 + l] = L[i];
    __syncthreads();
    int p = KMAX - kk;
    for (int i = 0; i < KMAX; ++i) {
        if (i < KMAX - kk) {
            if (l == 0) gl[i] = -INFINITY;
            continue;
        }
        const double v = p < KMAX ? lds[p * 64 + l] : INFINITY;
        const double m = wave_min_d(v);
        const unsigned long long b = __ballot(v == m);
        if (l == __ffsll((long long)b) - 1) ++p;
        if (l == 0) gl[i] = m;
    }
    __syncthreads();
}

template <int KMAX>
__global__ __launch_bounds__(64) void k_sor_knn_wave(GridDev g, int k, double* avg, SorPend pd, SorPend pd3) {
    __shared__ double lds[64 * KMAX];
    __shared__ double gl[KMAX];
    const int cnt = *pd3.count;
    const int l = (int)lane_id();
    for (int64_t s3 = blockIdx.x; s3 < cnt; s3 += gridDim.x) {
        const int64_t s = pd3.j[s3];  // the stage-2 pending slot
        const int64_t j = pd.j[s];
        const int f = sorted_frame(g, j);
        const int64_t fbeg = g.foff[f], fend = g.foff[f + 1];
        const double* o = g.origin + 3 * f;
        const double q[3] = {g.sxyz[j * 3], g.sxyz[j * 3 + 1], g.sxyz[j * 3 + 2]};
        const int kk = (int)((int64_t)k < fend - fbeg ? k : fend - fbeg);
        if (l < KMAX) gl[l] = pd.best[(int64_t)l * pd.cap + s];
        if (KMAX > 64 && l == 0)
            for (int i = 64; i < KMAX; ++i) gl[i] = pd.best[(int64_t)i * pd.cap + s];
        __syncthreads();
        long long have = pd.have[s];  // < 0: not every point of the scanned cube was counted
        int cc[3];
        query_cell(g, j, cc[0], cc[1], cc[2]);
        const int cx = cc[0], cy = cc[1], cz = cc[2];
        double lo[3], hi[3];
        cell_fracs(g, q, o, cc, lo, hi);
        double L[KMAX];
        bool settled = false;
        for (int r = 3; r <= SOR_RMAX3 && !settled; ++r) {
            const double gk = gl[KMAX - 1];
            if (l == 0) {
#pragma unroll
                for (int i = 0; i < KMAX; ++i) L[i] = gl[i];
            } else {
                topk_reset<KMAX>(L, kk);
                L[KMAX - 1] = gk;
            }
            long long hl = 0;
            bool cull = false;
            const int W = 2 * r + 1;
            for (int t = l; t < W * W; t += 64) {
                const int dx = t / W - r, dy = t % W - r;
                const double ex = face_gap(lo[0], hi[0], dx, g.h), ey = face_gap(lo[1], hi[1], dy, g.h);
                const double e2 = ex * ex + ey * ey;
                if (dx == -r || dx == r || dy == -r || dy == r) {
                    if (!(e2 < gk)) {
                        cull = true;
                        continue;
                    }
                    const int2 se = column_range(g, grid_column(g, f, cx + dx, cy + dy), cz - r, cz + r);
                    scan_range<KMAX>(g.sxyz, q, se.x, se.y, L);
                    hl += se.y - se.x;
                } else {
                    const double ezl = face_gap(lo[2], hi[2], -r, g.h), ezh = face_gap(lo[2], hi[2], r, g.h);
                    const bool a = e2 + ezl * ezl < gk, b = e2 + ezh * ezh < gk;
                    if (!a || !b) cull = true;
                    if (!a && !b) continue;
                    const int2 col = grid_column(g, f, cx + dx, cy + dy);
                    if (a) {
                        const int2 se = column_range(g, col, cz - r, cz - r);
                        scan_range<KMAX>(g.sxyz, q, se.x, se.y, L);
                        hl += se.y - se.x;
                    }
                    if (b) {
                        const int2 se = column_range(g, col, cz + r, cz + r);
                        scan_range<KMAX>(g.sxyz, q, se.x, se.y, L);
                        hl += se.y - se.x;
                    }
                }
            }
            wave_merge<KMAX>(lds, gl, L, kk);
            if (__any(cull)) have = -1;
            if (have >= 0) have += wave_sum(hl);
            const double guard = block_guard(g, q, o, cc, (double)r);
            const double kth = gl[KMAX - 1];
            settled = have >= fend - fbeg || (kth < INFINITY && kth <= guard * guard);
        }
        if (!settled) {  // the whole frame from scratch, the points split over the lanes
            topk_reset<KMAX>(L, kk);
            for (int64_t m = fbeg + l; m < fend; m += 64) {
                const double d = d2_l2(q, g.sxyz + m * 3);
                if (d < L[KMAX - 1]) topk_insert<KMAX>(L, d);
            }
            wave_merge<KMAX>(lds, gl, L, kk);
        }
        if (l == 0) {
            double best[KMAX];
#pragma unroll
            for (int i = 0; i < KMAX; ++i) best[i] = gl[i];
            avg[sor_out(g, j)] = sor_mean<KMAX>(best, kk);
        }
        __syncthreads();  // gl is reloaded for the next query
    }
}

// ------------------------------------------------------------------------------------ cross-cloud 1-NN distance
// PointCloud::ComputePointCloudDistance (eval_cone.py:99,103): per source point the distance to its nearest target
// point, sqrt of the exact float64 squared distance.  The grid is built over the target.  A query inside the
// target's bounding box whose cell is occupied runs the SOR stages (3x3x3 then 5x5x5 block of its cell); any other
// query expands Chebyshev rings around the cell of q' = clamp(q, box).  For every target point p (inside the box)
// |q - p|^2 >= |q - q'|^2 + |q' - p|^2, so the ring guard of q' plus |q - q'|^2 bounds every unscanned point.
constexpr int NN_RMAX = 6;

__device__ inline int2 grid_cell_range(const GridDev& g, int x, int y, int z, int& cell) {
    const int2 se = grid_find(g, 0, x, y, z);
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
    const int cq[3] = {cx, cy, cz};  // q's own cell (a query, not a grid point: its cell is computed, as the grid's)
    if (off2 == 0.0) {
        int c;
        grid_cell_range(g, cx, cy, cz, c);
        if (c >= 0) {
            const int2* r3 = g.nbr3 + (int64_t)c * NBR3;
            for (int u = 0; u < NBR3; ++u) {
                const int2 se = r3[(u + 4) % NBR3];
                nn_range(g, q, se.x, se.y, best);
            }
            double guard = block_guard(g, q, g.origin, cq, 1.0);
            settled = best <= guard * guard;
            if (!settled) {
                const int czc = g.cz[c];
                for (int t = 0; t < NBR5; ++t) {
                    const int dx = t / 5 - 2, dy = t % 5 - 2;
                    const int2 col = grid_column(g, 0, cx + dx, cy + dy);
                    if (col.y == 0) continue;
                    if (dx >= -1 && dx <= 1 && dy >= -1 && dy <= 1) {
                        const int2 a = column_range(g, col, czc - 2, czc - 2), b = column_range(g, col, czc + 2, czc + 2);
                        nn_range(g, q, a.x, a.y, best);
                        nn_range(g, q, b.x, b.y, best);
                    } else {
                        const int2 r = column_range(g, col, czc - 2, czc + 2);
                        nn_range(g, q, r.x, r.y, best);
                    }
                }
                guard = block_guard(g, q, g.origin, cq, 2.0);
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
                        const int2 se = grid_find(g, 0, cx + dx, cy + dy, cz + dz);
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

// ---- cloud statistics per frame (RemoveStatisticalOutliers after the kNN loop) -----------------------------------
// mode 0: x[i] = avg > 0 ? avg : 0 (the accumulate's lambda) and the block's count of points with neighbours
//         (avg >= 0: Open3D's valid_distances) -> vpart[f][block]
// mode 1: x[i] = avg > 0 ? (avg - mean)^2 : 0 with mean = sum1[f] / valid[f] (the inner_product's op2)
// grid (chunks, frames): a workgroup stays inside one frame
__global__ __launch_bounds__(256) void k_sor_values(const double* __restrict__ avg, const int* __restrict__ foff,
                                                    int mode, const double* __restrict__ stats, double* __restrict__ x,
                                                    int* __restrict__ vpart) {
    const int f = blockIdx.y;
    const int64_t beg = foff[f], end = foff[f + 1];
    const int64_t i = beg + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if ((int64_t)blockIdx.x * 256 >= end - beg) {
        if (mode == 0 && threadIdx.x == 0) vpart[(int64_t)f * gridDim.x + blockIdx.x] = 0;
        return;
    }
    double mean = 0.0;
    if (mode == 1) mean = stats[f * 4 + 0] / stats[f * 4 + 2];
    int c = 0;
    if (i < end) {
        const double a = avg[i];
        if (mode == 0) {
            x[i] = a > 0 ? a : 0.0;
            c = a >= 0 ? 1 : 0;
        } else {
            x[i] = a > 0 ? (a - mean) * (a - mean) : 0.0;
        }
    }
    if (mode == 0) {
        c = wave_sum(c);
        __shared__ int ws[4];
        if (lane_id() == 0) ws[threadIdx.x >> 6] = c;
        __syncthreads();
        if (threadIdx.x == 0) vpart[(int64_t)f * gridDim.x + blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
    }
}

// one workgroup per frame: valid = sum of the block counts; stats[f] = {sum (mean after mode 1), -, valid, -}
__global__ __launch_bounds__(256) void k_sor_valid(const int* __restrict__ vpart, int nblocks,
                                                   const double* __restrict__ sums, double* __restrict__ stats) {
    const int f = blockIdx.x;
    long long c = 0;
    for (int b = threadIdx.x; b < nblocks; b += 256) c += vpart[(int64_t)f * nblocks + b];
    c = wave_sum(c);
    __shared__ long long ws[4];
    if (lane_id() == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        stats[f * 4 + 0] = sums[f];  // the sum; mode 1 divides it by valid exactly as cloud_mean /= valid
        stats[f * 4 + 2] = (double)(ws[0] + ws[1] + ws[2] + ws[3]);
    }
}

// stats[f] = {cloud_mean, std, valid, threshold} (Bessel-corrected std)
__global__ void k_sor_stats(int nframes, const double* __restrict__ sums, double std_ratio, double* __restrict__ stats) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nframes) return;
    const double v = stats[f * 4 + 2];
    if (v == 0.0) {  // Open3D returns an empty cloud
        stats[f * 4 + 0] = 0.0;
        stats[f * 4 + 1] = 0.0;
        stats[f * 4 + 3] = -INFINITY;
        return;
    }
    const double mean = stats[f * 4 + 0] / v;
    const double sd = sqrt(sums[f] / (v - 1.0));  // valid - 1 exactly (valid < 2^53)
    stats[f * 4 + 0] = mean;
    stats[f * 4 + 1] = sd;
    stats[f * 4 + 3] = mean + std_ratio * sd;
}

struct RorPred {
    const unsigned char* keep;
    __device__ bool operator()(int64_t i) const { return keep[i] != 0; }
};
struct IndexEmit {
    int64_t* out;
    __device__ void operator()(int64_t i, int64_t pos) const { out[pos] = i; }
};

// ------------------------------------------------------------------------------------ grid builder (host)
static int bits_for_host(int64_t v) {  // bits to represent 0..v
    int b = 1;
    while (b < 62 && (v >> b) != 0) ++b;
    return b;
}

ot_status build_grid_frames(const double* xyz, int64_t n, int nframes, const int* d_foff, const double* d_origin,
                            double h, const int dims[3], int nbr, hipStream_t stream, GridBuild& out, int slot0,
                            const int* h_foff) {
    GridDev& g = out.g;
    g.h = h;
    g.origin = d_origin;
    g.foff = d_foff;
    g.nframes = nframes;
    int bits[3];
    for (int a = 0; a < 3; ++a) {
        if (dims[a] < 1 || dims[a] > 1000000)
            return fail(OT_ERR_INVALID_ARGUMENT, "neighbour grid out of range (radius too small for the extent)");
        g.dim[a] = dims[a];
        bits[a] = bits_for_host(g.dim[a] - 1);
    }
    g.sy = bits[2];
    g.sx = bits[1] + bits[2];
    g.sf = bits[0] + bits[1] + bits[2];
    const int end_bit = g.sf + (nframes > 1 ? bits_for_host(nframes - 1) : 0);
    if (end_bit > 64) return fail(OT_ERR_INVALID_ARGUMENT, "neighbour grid keys exceed 64 bits");
    char* ws = (char*)scratch(256 + (size_t)n * (8 + 8 + 4 + 4 + 4 + 4 + 24), slot0);
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
    ot_status st;
    if (end_bit <= 32 && n > (int64_t)(1 << 21)) {  // large sorts on 32-bit keys: 8 B per pair per pass, not 12
        unsigned* k32 = (unsigned*)kin;
        unsigned* k32o = k32 + n;
        hipLaunchKernelGGL(k_cell_keys<unsigned>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, xyz, n, g,
                           k32, vin, err);
        OT_LAUNCH_CHECK();
        if (h_foff && nframes > 1 && nframes <= 64) {  // frames are contiguous: sort each on its cell bits alone
            std::vector<int64_t> seg((size_t)nframes + 1);
            for (int f = 0; f <= nframes; ++f) seg[f] = h_foff[f];
            st = sort_segments_u32_u32(k32, k32o, vin, vout, seg.data(), nframes, std::max(g.sf, 1), stream, 3);
        } else {
            st = sort_pairs_u32_u32(k32, k32o, vin, vout, (size_t)n, std::max(end_bit, 1), stream, 3);
        }
        if (st != OT_OK) return st;
        hipLaunchKernelGGL(k_widen_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, (const unsigned*)k32o,
                           n, kout);
    } else {
        hipLaunchKernelGGL(k_cell_keys<unsigned long long>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                           xyz, n, g, kin, vin, err);
        OT_LAUNCH_CHECK();
        st = sort_pairs_u64_u32(kin, kout, vin, vout, (size_t)n, std::max(end_bit, 1), stream, 3);
        if (st != OT_OK) return st;
    }
    int64_t ncells = 0;
    st = compact_segments(n, kout, heads, pcell, stream, &ncells, slot0 + 1);  // synchronises
    if (st != OT_OK) return st;
    int e = 0;
    OT_HIP_TRY(hipMemcpyAsync(&e, err, sizeof(int), hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipStreamSynchronize(stream));
    if (e) return fail(OT_ERR_INVALID_ARGUMENT, "neighbour grid out of range (non-finite point coordinates)");
    int64_t cap = 1;
    while (cap < 2 * ncells + 2) cap <<= 1;
    const bool w3 = nbr & GRID_NBR3, w5 = nbr & GRID_NBR5;
    const size_t per_cell = (w3 ? NBR3 * 8 : 0) + (w5 ? NBR5 * 8 : 0) + 12;
    char* hs = (char*)scratch((size_t)cap * (8 + 8) + (size_t)ncells * per_cell + 128, slot0 + 2);
    if (!hs) return fail(OT_ERR_HIP, "scratch allocation failed");
    g.hkeys = (unsigned long long*)hs;
    g.hval = (int2*)(g.hkeys + cap);
    int2* cur = g.hval + cap;
    int2* nbr3 = w3 ? cur : nullptr;
    cur += w3 ? ncells * NBR3 : 0;
    int2* nbr5 = w5 ? cur : nullptr;
    cur += w5 ? ncells * NBR5 : 0;
    g.crange = cur;
    g.cz = (int*)(g.crange + ncells);
    g.hash_mask = (int)(cap - 1);
    OT_HIP_TRY(hipMemsetAsync(g.hkeys, 0xFF, sizeof(unsigned long long) * cap, stream));
    hipLaunchKernelGGL(k_grid_insert, dim3((unsigned)((ncells + 255) / 256)), dim3(256), 0, stream, kout, heads,
                       ncells, n, g);  // cell ranges / z and the column hash, read by k_cell_nbr
    if (w5)
        hipLaunchKernelGGL(k_cell_nbr<2>, dim3((unsigned)((ncells * NBR5 + 255) / 256)), dim3(256), 0, stream, kout,
                           heads, ncells, g, nbr3, nbr5);
    else if (w3)
        hipLaunchKernelGGL(k_cell_nbr<1>, dim3((unsigned)((ncells * NBR3 + 255) / 256)), dim3(256), 0, stream, kout,
                           heads, ncells, g, nbr3, nbr5);
    hipLaunchKernelGGL(k_gather_sorted, dim3((unsigned)((n * 3 + 255) / 256)), dim3(256), 0, stream, xyz, vout, n, sxyz);
    OT_LAUNCH_CHECK();
    g.sxyz = sxyz;
    g.sidx = vout;
    g.pkey = kout;
    g.pcell = pcell;
    g.nbr3 = nbr3;
    g.nbr5 = nbr5;
    out.ncells = ncells;
    return OT_OK;
}

ot_status build_grid_sorted(const double* xyz, const unsigned long long* ckeys, int64_t n, int nframes,
                            const int* d_foff, const double* d_origin, double h, const int bits[3], int nbr,
                            hipStream_t stream, GridBuild& out, int slot0) {
    GridDev& g = out.g;
    g.h = h;
    g.origin = d_origin;
    g.foff = d_foff;
    g.nframes = nframes;
    for (int a = 0; a < 3; ++a) {
        if (bits[a] < 0 || bits[a] > 20)
            return fail(OT_ERR_INVALID_ARGUMENT, "neighbour grid out of range (radius too small for the extent)");
        g.dim[a] = 1 << bits[a];
    }
    g.sy = bits[2];
    g.sx = bits[1] + bits[2];
    g.sf = bits[0] + bits[1] + bits[2];
    char* ws = (char*)scratch(256 + (size_t)n * 8, slot0);
    if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
    int* heads = (int*)ws;
    int* pcell = heads + n;
    int64_t ncells = 0;
    ot_status st = compact_segments(n, ckeys, heads, pcell, stream, &ncells, slot0 + 1);  // synchronises
    if (st != OT_OK) return st;
    int64_t cap = 1;
    while (cap < 2 * ncells + 2) cap <<= 1;
    const bool w3 = nbr & GRID_NBR3, w5 = nbr & GRID_NBR5;
    const size_t per_cell = (w3 ? NBR3 * 8 : 0) + (w5 ? NBR5 * 8 : 0) + 12;
    char* hs = (char*)scratch((size_t)cap * (8 + 8) + (size_t)ncells * per_cell + 128, slot0 + 2);
    if (!hs) return fail(OT_ERR_HIP, "scratch allocation failed");
    g.hkeys = (unsigned long long*)hs;
    g.hval = (int2*)(g.hkeys + cap);
    int2* cur = g.hval + cap;
    int2* nbr3 = w3 ? cur : nullptr;
    cur += w3 ? ncells * NBR3 : 0;
    int2* nbr5 = w5 ? cur : nullptr;
    cur += w5 ? ncells * NBR5 : 0;
    g.crange = cur;
    g.cz = (int*)(g.crange + ncells);
    g.hash_mask = (int)(cap - 1);
    OT_HIP_TRY(hipMemsetAsync(g.hkeys, 0xFF, sizeof(unsigned long long) * cap, stream));
    if (ncells > 0) {
        hipLaunchKernelGGL(k_grid_insert, dim3((unsigned)((ncells + 255) / 256)), dim3(256), 0, stream, ckeys, heads,
                           ncells, n, g);
        if (w5)
            hipLaunchKernelGGL(k_cell_nbr<2>, dim3((unsigned)((ncells * NBR5 + 255) / 256)), dim3(256), 0, stream,
                               ckeys, heads, ncells, g, nbr3, nbr5);
        else if (w3)
            hipLaunchKernelGGL(k_cell_nbr<1>, dim3((unsigned)((ncells * NBR3 + 255) / 256)), dim3(256), 0, stream,
                               ckeys, heads, ncells, g, nbr3, nbr5);
        OT_LAUNCH_CHECK();
    }
    g.sxyz = xyz;
    g.sidx = nullptr;
    g.pkey = ckeys;
    g.pcell = pcell;
    g.nbr3 = nbr3;
    g.nbr5 = nbr5;
    out.ncells = ncells;
    return OT_OK;
}

// test hook otx_sor_netfill: 0 = the sequential fill of the stage-1 list (A/B timing and parity of the network fill)
static bool g_sor_netfill = true;

ot_status sor_frames(const GridBuild& gb, int64_t n, const int* h_foff, int nb_neighbors, double std_ratio,
                     double* avg, double* stats, hipStream_t stream, int slot0) {
    const int F = gb.g.nframes;
    int64_t max_n = 0;
    for (int f = 0; f < F; ++f) max_n = std::max<int64_t>(max_n, h_foff[f + 1] - h_foff[f]);
    const unsigned grid = (unsigned)((n + 255) / 256);
    const int kk = (int)std::min<int64_t>(nb_neighbors, std::max<int64_t>(max_n, 1));  // list length actually needed
    // pending list of stage-1 misses (device count; capacity n)
    const int km = kk <= 4 ? 4 : kk <= 8 ? 8 : kk <= 12 ? 12 : kk <= 16 ? 16 : kk <= 20 ? 20 : kk <= 24 ? 24
                 : kk <= 32 ? 32 : kk <= 48 ? 48 : 64;
    // and of stage-2 misses (stage 3, one wave each): their pending slots (capacity n; count and list stay in place)
    const size_t per = 4 + 8 + 8 * (size_t)km;
    char* pw = (char*)scratch((size_t)n * (per + 4) + 1024, slot0 + 1);
    if (!pw) return fail(OT_ERR_HIP, "scratch allocation failed");
    SorPend pd, pd3;
    pd.count = (int*)pw;
    pd3.count = pd.count + 1;
    pd.j = (int*)(pw + 256);
    pd.have = (long long*)(((uintptr_t)(pd.j + n) + 15) & ~(uintptr_t)15);
    pd.best = (double*)(pd.have + n);
    pd.cap = n;
    pd3.j = (int*)(((uintptr_t)(pd.best + (size_t)km * n) + 255) & ~(uintptr_t)255);
    pd3.have = nullptr;  // in the stage-2 slot (pd)
    pd3.best = nullptr;
    pd3.cap = n;
    OT_HIP_TRY(hipMemsetAsync(pd.count, 0, 2 * sizeof(int), stream));
    const unsigned rgrid = (unsigned)std::min<int64_t>(std::max<int64_t>(grid / 4, 1), 2048);
#define OT_SOR_LAUNCH(KM)                                                                                           \
    do {                                                                                                            \
        if (g_sor_netfill)                                                                                          \
            hipLaunchKernelGGL((k_sor_knn<KM, SOR_BLOCK_R, true>), dim3(grid), dim3(256), 0, stream, gb.g, n,       \
                               (int)nb_neighbors, avg, pd);                                                         \
        else                                                                                                        \
            hipLaunchKernelGGL((k_sor_knn<KM, SOR_BLOCK_R, false>), dim3(grid), dim3(256), 0, stream, gb.g, n,      \
                               (int)nb_neighbors, avg, pd);                                                         \
        hipLaunchKernelGGL((k_sor_knn_rest<KM, SOR_BLOCK_R>), dim3(rgrid), dim3(256), 0, stream, gb.g,              \
                           (int)nb_neighbors, avg, pd, pd3);                                                        \
        hipLaunchKernelGGL((k_sor_knn_wave<KM>), dim3(4096), dim3(64), 0, stream, gb.g, (int)nb_neighbors, avg, pd,   \
                           pd3);                                                                                    \
    } while (0)
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
    OT_LAUNCH_CHECK();
    return sor_stats_frames(avg, gb.g.foff, h_foff, F, std_ratio, stats, stream, slot0);
}

ot_status sor_stats_frames(const double* avg, const int* d_foff, const int* h_foff, int F, double std_ratio,
                           double* stats, hipStream_t stream, int slot) {
    int64_t max_n = 0;
    for (int f = 0; f < F; ++f) max_n = std::max<int64_t>(max_n, h_foff[f + 1] - h_foff[f]);
    const int64_t n = h_foff[F];
    const int slot0 = slot;
    // the two sequential float64 sums per frame (exact chains): x values, chain jobs, valid counts, sums
    const int nvb = (int)std::max<int64_t>((max_n + 255) / 256, 1);
    size_t aux = 0;
    for (int f = 0; f < F; ++f) aux += chain_aux_bytes(h_foff[f + 1] - h_foff[f]);
    const size_t bytes = (size_t)n * 8 + 256 + aux + (sizeof(ChainJob) + 32) * (size_t)F + (size_t)F * nvb * 4 + 512;
    char* ws = (char*)scratch(bytes, slot0);
    if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
    double* x = (double*)ws;
    double* sums = (double*)(((uintptr_t)(x + n) + 63) & ~(uintptr_t)63);
    int* vpart = (int*)(sums + F);
    char* cur = (char*)(((uintptr_t)(vpart + (size_t)F * nvb) + 63) & ~(uintptr_t)63);
    std::vector<ChainJob> jobs((size_t)F);
    for (int f = 0; f < F; ++f) {
        ChainJob& jb = jobs[f];
        jb.x = x + h_foff[f];
        jb.n = h_foff[f + 1] - h_foff[f];
        jb.out = sums + f;
        cur = chain_aux(cur, jb.n, jb);
    }
    ChainJob* djobs = (ChainJob*)cur;
    OT_HIP_TRY(hipMemcpyAsync(djobs, jobs.data(), sizeof(ChainJob) * F, hipMemcpyHostToDevice, stream));
    const dim3 vgrid((unsigned)nvb, (unsigned)F);
    hipLaunchKernelGGL(k_sor_values, vgrid, dim3(256), 0, stream, (const double*)avg, d_foff, 0,
                       (const double*)stats, x, vpart);
    launch_sum_chains(djobs, F, max_n, stream);
    hipLaunchKernelGGL(k_sor_valid, dim3(F), dim3(256), 0, stream, (const int*)vpart, nvb, (const double*)sums, stats);
    hipLaunchKernelGGL(k_sor_values, vgrid, dim3(256), 0, stream, (const double*)avg, d_foff, 1,
                       (const double*)stats, x, vpart);
    launch_sum_chains(djobs, F, max_n, stream);
    hipLaunchKernelGGL(k_sor_stats, dim3((unsigned)((F + 63) / 64)), dim3(64), 0, stream, F, (const double*)sums,
                       std_ratio, stats);
    OT_LAUNCH_CHECK();
    // the host job table is consumed by the copy above before the caller's next synchronisation point returns
    OT_HIP_TRY(hipStreamSynchronize(stream));
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

// one frame: origin = the cloud's minimum corner, cells per axis from the extent.  frame_dev receives the device
// origin [3] and offsets {0, n} (scratch slot 20).
static ot_status single_frame_grid(const double* xyz, int64_t n, double h, const double mn[3], const double mx[3],
                                   int nbr, hipStream_t stream, GridBuild& gb) {
    int dims[3];
    for (int a = 0; a < 3; ++a) {
        const double span = std::floor((mx[a] - mn[a]) / h);
        if (!(span < 1.0e6)) return fail(OT_ERR_INVALID_ARGUMENT, "neighbour grid out of range (radius too small for the extent)");
        dims[a] = (int)span + 1;
    }
    char* fr = (char*)scratch(64, 20);
    if (!fr) return fail(OT_ERR_HIP, "scratch allocation failed");
    const double org[4] = {mn[0], mn[1], mn[2], 0.0};
    const int off[2] = {0, (int)n};
    OT_HIP_TRY(hipMemcpyAsync(fr, org, sizeof(org), hipMemcpyHostToDevice, stream));
    OT_HIP_TRY(hipMemcpyAsync(fr + 32, off, sizeof(off), hipMemcpyHostToDevice, stream));
    // build_grid_frames synchronises the stream before returning, so org / off outlive their copies
    return build_grid_frames(xyz, n, 1, (const int*)(fr + 32), (const double*)fr, h, dims, nbr, stream, gb, 22);
}

extern "C" {
// test / diagnostic hook (not part of the drop-in boundary): 1 (default) = stage 1 fills its list with the own
// column's first 20 candidates through a sorting network, 0 = by sequential insertion (same bits)
ot_status otx_sor_netfill(int32_t on) {
    ot::g_sor_netfill = on != 0;
    return OT_OK;
}
}  // extern "C"

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
    st = single_frame_grid(xyz, n, radius, mn, mx, GRID_NBR3, stream, gb);
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
    // Cell size: the grid only changes speed, never the result.  Aim for ~target points per occupied cell of a
    // surface-like cloud.  First guess: the points cover half of the bounding box's largest face; refined once from
    // the measured occupancy (2-D scaling) when it is off by more than 2.5x.
    const double target = sor_cell_target(nb_neighbors);
    double ext[3];
    for (int a = 0; a < 3; ++a) ext[a] = std::max(mx[a] - mn[a], 1e-9);
    std::sort(ext, ext + 3);
    const double hmin = ext[2] / 5.0e5;
    double h = std::max(std::sqrt(0.5 * ext[2] * ext[1] * target / (double)n), hmin);
    GridBuild gb;
    st = single_frame_grid(xyz, n, h, mn, mx, SOR_GRID_NBR, stream, gb);
    if (st != OT_OK) return st;
    const double occ = (double)n / (double)std::max<int64_t>(gb.ncells, 1);
    if (occ > 2.5 * target || occ < 0.4 * target) {
        h = std::max(h * std::sqrt(target / occ), hmin);
        st = single_frame_grid(xyz, n, h, mn, mx, SOR_GRID_NBR, stream, gb);
        if (st != OT_OK) return st;
    }
    char* ws = (char*)scratch((size_t)n * 8 + 256, 12);
    if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
    double* stats = (double*)ws;  // [mean, std, valid, threshold]
    double* avg = out_avg_dist ? out_avg_dist : (double*)(ws + 256);
    const int foff[2] = {0, (int)n};
    st = sor_frames(gb, n, foff, nb_neighbors, std_ratio, avg, stats, stream, 41);
    if (st != OT_OK) return st;
    return compact(n, SorKeep{avg, stats, gb.g.foff, 1}, IndexEmit{out_indices}, stream, n_kept_host, 13);
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
    st = single_frame_grid(tgt, m, h, mn, mx, GRID_NBR3, stream, gb);
    if (st != OT_OK) return st;
    const double occ = (double)m / (double)std::max<int64_t>(gb.ncells, 1);
    if (occ > 2.5 * target || occ < 0.4 * target) {
        h = std::max(h * std::sqrt(target / occ), hmin);
        st = single_frame_grid(tgt, m, h, mn, mx, GRID_NBR3, stream, gb);
        if (st != OT_OK) return st;
    }
    hipLaunchKernelGGL(k_nn_dist, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, gb.g, src, n, m, mn[0],
                       mn[1], mn[2], mx[0], mx[1], mx[2], out);
    OT_LAUNCH_CHECK();
    OT_HIP_TRY(hipStreamSynchronize(stream));
    return OT_OK;
}

}  // extern "C"
