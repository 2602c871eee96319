// filter_batch.hip — the configs[2] filter chain for a batch of RGB-D frames in one device-resident pass.
//
// Per frame f (check_one_frame.py:22-28 with a pose, then the north_star's statistical filter):
//   create_from_color_and_depth(depth_scale, depth_trunc) -> PointCloud.create_from_rgbd_image(intr, extrinsic_f)
//   -> voxel_down_sample(voxel_size) -> remove_statistical_outlier(nb_neighbors, std_ratio) -> select_by_index
// Results are bit-identical to that sequence of single calls (ot_depth_to_float, ot_unproject, ot_voxel_down_sample,
// ot_remove_statistical_outlier, ot_gather_rows3) frame by frame; the frames never leave HBM and the whole batch
// takes a fixed ~30 launches and 6 host synchronisations (sizes), instead of ~30 launches and 8 syncs per frame.
//
//   k_fb_pixels   tile of 2048 pixels of one frame: depth -> float (Open3D ConvertDepthToFloatImage), unprojection
//                 of the valid pixels in float64 (camera_pose = inverse(extrinsic)), per-tile bounds + valid count
//   k_fb_setup    per frame: bounds -> voxel origin (min - vs/2), key widths; one block scans the tile counts
//   k_fb_keys     the same pixels again: CELL-MAJOR voxel key (the SOR cell (kx, ky, kz) >> m, then the voxel inside
//                 the cell; one sort segment per frame), written by stable
//                 compaction in pixel (= point index) order, value = point index, and the point's 8-B record (pixel,
//                 raw depth, RGB8) at that index (the u64-key fallback for huge grids / batches: frame in the key,
//                 value = global pixel index)
//   radix sort    stable => every voxel's points stay in point-index order
//   heads         voxel segment starts (stable compaction)
//   k_fb_reduce   one lane per voxel: its points re-unprojected from their records (no xyz/rgb intermediates in HBM,
//                 one 8-B gather per point), summed in index order, divided by the count (Open3D AccumulatedPoint);
//                 also the voxel's SOR cell key
//   SOR           grid.h over all frames' voxel clouds at once (frame in the key's top bits) + sor_frames.  The SOR
//                 cells are blocks of 2^m x 2^m x 2^m voxels on the voxel lattice (m from nb_neighbors: ~0.9 k points
//                 per occupied cell of a surface), so the voxel order IS the grid's cell order: the grid is built
//                 from the voxel list directly (cell heads, column hash, neighbour ranges) -- no cell keys from the
//                 coordinates, no second sort, no re-laid-out copy of the cloud.  A frame's voxel cloud therefore
//                 comes out in cell-major key order (Open3D's is hash order: any fixed order is as valid); the SOR
//                 statistics sum in that order
//   keep          stable compaction of avg > 0 && avg < threshold_f; rows gathered per frame
#include <algorithm>
#include <cmath>
#include <vector>

#include "compact.h"
#include "grid.h"
#include "sort.h"

namespace ot {

constexpr int FB_THREADS = 256;
constexpr int FB_PIX = 8;                        // consecutive pixels per lane (one 16-B depth load)
constexpr int FB_TILE = FB_THREADS * FB_PIX;     // pixels per workgroup tile

struct FbFrame {  // per-frame constants (device table)
    double pose[16];    // inverse(extrinsic), row-major
    double vmin[3];     // voxel grid origin: min_bound - vs / 2
    int err;
    int tag;            // u32-key chain: parity of the frame's rank among the batch's non-empty frames
};

struct FbParams {
    const uint16_t* depth;  // [F][h][w]
    const uint8_t* color;   // [F][h][w][3]
    int w, h, tpf;          // tiles per frame
    float scale_f, rscale_f;  // rscale_f = fl(1 / scale_f) (div_rn)
    double trunc, fx, fy, cx, cy, vs, inv_vs;
    double rfx, rfy;  // fl(1 / fx), fl(1 / fy)
    FbFrame* frames;
    int F;
};

// one pixel: Open3D's float depth, then (valid) the float64 point camera_pose * ((c-cx) z / fx, (r-cy) z / fy, z, 1)
__device__ inline bool fb_point(const FbParams& p, const double* m, float d, int pix, double xyz[3]) {
    if (!(d > 0.0f)) return false;
    const unsigned pu = (unsigned)pix, rq = pu / (unsigned)p.w;
    const int r = (int)rq, c = (int)(pu - rq * (unsigned)p.w);
    const double z = (double)d;
    const double x = div_rn(((double)c - p.cx) * z, p.fx, p.rfx);
    const double y = div_rn(((double)r - p.cy) * z, p.fy, p.rfy);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double a = m[k * 4 + 0] * x;
        const double b = m[k * 4 + 1] * y;
        const double cc = m[k * 4 + 2] * z;
        xyz[k] = ((a + b) + cc) + m[k * 4 + 3];
    }
    return true;
}

// floor(fl(a / b)) (Open3D's voxel index) without the division when it cannot matter: q = fl(a * fl(1/b)) and
// fl(a / b) both lie within 2^-52 (a/b) of a / b (a >= 0 here), so |q - fl(a/b)| < 2.3e-16 q; when q's distance to
// the nearest integer exceeds 1e-15 q both floor the same, otherwise the exact quotient decides
__device__ inline double floor_div(double a, double b, double inv_b) {
    const double q = a * inv_b;
    const double fq = floor(q);
    const double fr = q - fq;  // exact (Sterbenz)
    const double eps = 1e-15 * q;
    if (fr > eps && fr < 1.0 - eps) return fq;
    return floor(a / b);
}

// the lane's 8 depth values as Open3D's float image: f = (float)u16 / (float)scale; 0 when f >= trunc (raw: the
// u16 values themselves)
__device__ inline void fb_depth8(const FbParams& p, const uint16_t* __restrict__ dep, int pix0, int npx, float f[8],
                                 unsigned raw[8]) {
    if (pix0 + FB_PIX <= npx && ((reinterpret_cast<uintptr_t>(dep + pix0) & 15) == 0)) {
        const uint4 r4 = *reinterpret_cast<const uint4*>(dep + pix0);
        const uint32_t wd[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            raw[2 * k] = wd[k] & 0xFFFFu;
            raw[2 * k + 1] = wd[k] >> 16;
        }
    } else {
#pragma unroll
        for (int k = 0; k < FB_PIX; ++k) raw[k] = pix0 + k < npx ? (unsigned)dep[pix0 + k] : 0u;
    }
#pragma unroll
    for (int k = 0; k < FB_PIX; ++k) {
        f[k] = div_rn((float)raw[k], p.scale_f, p.rscale_f);
        if ((double)f[k] >= p.trunc) f[k] = 0.0f;
    }
}
__device__ inline void fb_depth8(const FbParams& p, const uint16_t* __restrict__ dep, int pix0, int npx, float f[8]) {
    unsigned raw[8];
    fb_depth8(p, dep, pix0, npx, f, raw);
}

// the lane's 8 RGB8 pixels as 24-bit words (r | g << 8 | b << 16): three 8-B loads when the 24 bytes are aligned
__device__ inline void fb_color8(const uint8_t* __restrict__ col, int pix0, int npx, unsigned rgb[8]) {
    const uint8_t* c = col + (int64_t)pix0 * 3;
    if (pix0 + FB_PIX <= npx && ((reinterpret_cast<uintptr_t>(c) & 7) == 0)) {
        const uint2* c8 = reinterpret_cast<const uint2*>(c);
        const uint2 a = c8[0], b = c8[1], d = c8[2];
        const unsigned long long w0 = ((unsigned long long)a.y << 32) | a.x, w1 = ((unsigned long long)b.y << 32) | b.x,
                                 w2 = ((unsigned long long)d.y << 32) | d.x;
        rgb[0] = (unsigned)(w0 & 0xFFFFFF);
        rgb[1] = (unsigned)((w0 >> 24) & 0xFFFFFF);
        rgb[2] = (unsigned)(((w0 >> 48) | (w1 << 16)) & 0xFFFFFF);
        rgb[3] = (unsigned)((w1 >> 8) & 0xFFFFFF);
        rgb[4] = (unsigned)((w1 >> 32) & 0xFFFFFF);
        rgb[5] = (unsigned)(((w1 >> 56) | (w2 << 8)) & 0xFFFFFF);
        rgb[6] = (unsigned)((w2 >> 16) & 0xFFFFFF);
        rgb[7] = (unsigned)(w2 >> 40);
    } else {
#pragma unroll
        for (int k = 0; k < FB_PIX; ++k)
            rgb[k] = pix0 + k < npx ? (unsigned)c[3 * k] | ((unsigned)c[3 * k + 1] << 8) | ((unsigned)c[3 * k + 2] << 16)
                                    : 0u;
    }
}

// a valid point of the u32-key chain as one 8-B record, written in point order by k_fb_runs so the voxel reduce
// gathers one word per point instead of a depth and three colour bytes: pixel within its frame
// (23), run head (1: the first point of a run, below), raw depth (16), RGB8 (24)
constexpr int FB_PACK_PIX_BITS = 23;
constexpr unsigned long long FB_PACK_HEAD = 1ull << FB_PACK_PIX_BITS;
constexpr int FB_PACK_DEPTH_SHIFT = FB_PACK_PIX_BITS + 1;
__device__ inline unsigned long long fb_pack(unsigned pix, unsigned raw_depth, unsigned rgb, bool head) {
    return (unsigned long long)pix | (head ? FB_PACK_HEAD : 0ull) | ((unsigned long long)raw_depth << FB_PACK_DEPTH_SHIFT) |
           ((unsigned long long)rgb << (FB_PACK_DEPTH_SHIFT + 16));
}

// per tile: valid count and bounds (order-preserving u64 encodings) of the valid pixels' points
__global__ __launch_bounds__(FB_THREADS) void k_fb_pixels(FbParams p, int* __restrict__ tcount,
                                                          unsigned long long* __restrict__ tbounds,
                                                          unsigned long long* __restrict__ run_status) {
    const int f = blockIdx.y, tile = blockIdx.x;
    if (threadIdx.x == 0) run_status[(int64_t)f * p.tpf + tile] = 0ull;  // k_fb_runs' look-back word of this tile
    const int npx = p.w * p.h;
    const int pix0 = tile * FB_TILE + threadIdx.x * FB_PIX;
    const uint16_t* dep = p.depth + (int64_t)f * npx;
    double m[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) m[k] = p.frames[f].pose[k];
    float d[FB_PIX];
    fb_depth8(p, dep, pix0, npx, d);
    unsigned long long mn[3] = {~0ull, ~0ull, ~0ull}, mx[3] = {0, 0, 0};
    int c = 0;
#pragma unroll
    for (int k = 0; k < FB_PIX; ++k) {
        double xyz[3];
        if (pix0 + k < npx && fb_point(p, m, d[k], pix0 + k, xyz)) {
            ++c;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const unsigned long long o = dbl_to_ordered(xyz[a]);
                mn[a] = o < mn[a] ? o : mn[a];
                mx[a] = o > mx[a] ? o : mx[a];
            }
        }
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            unsigned long long t = __shfl_xor(mn[a], off, 64);
            mn[a] = t < mn[a] ? t : mn[a];
            t = __shfl_xor(mx[a], off, 64);
            mx[a] = t > mx[a] ? t : mx[a];
        }
    }
    c = wave_sum(c);
    __shared__ unsigned long long s[4][6];
    __shared__ int sc[4];
    const int w = threadIdx.x >> 6;
    if (lane_id() == 0) {
        for (int a = 0; a < 3; ++a) {
            s[w][a] = mn[a];
            s[w][3 + a] = mx[a];
        }
        sc[w] = c;
    }
    __syncthreads();
    const int64_t t = (int64_t)f * p.tpf + tile;
    if (threadIdx.x < 6) {
        const int q = threadIdx.x;
        unsigned long long v = s[0][q];
        for (int k = 1; k < 4; ++k) v = q < 3 ? (s[k][q] < v ? s[k][q] : v) : (s[k][q] > v ? s[k][q] : v);
        tbounds[t * 6 + q] = v;
    }
    if (threadIdx.x == 0) tcount[t] = sc[0] + sc[1] + sc[2] + sc[3];
}

// blocks 0..F-1: frame bounds -> voxel origin, per-axis largest voxel index (atomicMax into kbits), Open3D's size
// check;
// block F: exclusive scan of the F * tpf tile counts in place (-> output offsets), totals[0] = P
__global__ __launch_bounds__(256) void k_fb_setup(FbParams p, int* __restrict__ tcount,
                                                  const unsigned long long* __restrict__ tbounds,
                                                  unsigned long long* __restrict__ fbounds, int* __restrict__ kbits,
                                                  long long* __restrict__ totals, int* __restrict__ poff,
                                                  int* __restrict__ run_ticket) {
    const int f = blockIdx.x;
    if (f < p.F && threadIdx.x == 0) run_ticket[f] = 0;  // k_fb_runs' tile tickets of frame f
    if (f == p.F) {  // scan
        __shared__ int wsum[4];
        __shared__ long long carry_s;
        const int n = p.F * p.tpf;
        const int lane = (int)lane_id(), wid = threadIdx.x >> 6;
        if (threadIdx.x == 0) carry_s = 0;
        __syncthreads();
        for (int base = 0; base < n; base += 256) {
            const int i = base + threadIdx.x;
            const int x = i < n ? tcount[i] : 0;
            int inc = x;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int tt = __shfl_up(inc, o, 64);
                if (lane >= o) inc += tt;
            }
            if (lane == 63) wsum[wid] = inc;
            __syncthreads();
            int off = 0, tot = 0;
            for (int w = 0; w < 4; ++w) {
                off += w < wid ? wsum[w] : 0;
                tot += wsum[w];
            }
            const long long carry = carry_s;
            if (i < n) tcount[i] = (int)(carry + off + inc - x);
            __syncthreads();
            if (threadIdx.x == 0) carry_s = carry + tot;
            __syncthreads();
        }
        if (threadIdx.x == 0) totals[0] = carry_s;
        __syncthreads();
        for (int g = threadIdx.x; g < p.F; g += 256) poff[g] = tcount[g * p.tpf];  // frame g's first tile offset
        return;
    }
    __shared__ unsigned long long s[256][6];
    unsigned long long v[6] = {~0ull, ~0ull, ~0ull, 0, 0, 0};
    for (int t = threadIdx.x; t < p.tpf; t += 256)
        for (int q = 0; q < 6; ++q) {
            const unsigned long long x = tbounds[((int64_t)f * p.tpf + t) * 6 + q];
            v[q] = q < 3 ? (x < v[q] ? x : v[q]) : (x > v[q] ? x : v[q]);
        }
    for (int q = 0; q < 6; ++q) s[threadIdx.x][q] = v[q];
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < 256; ++i)
            for (int q = 0; q < 6; ++q) v[q] = q < 3 ? (s[i][q] < v[q] ? s[i][q] : v[q]) : (s[i][q] > v[q] ? s[i][q] : v[q]);
        for (int q = 0; q < 6; ++q) fbounds[f * 6 + q] = v[q];
        FbFrame& fr = p.frames[f];
        fr.err = 0;
        if (v[0] == ~0ull) {  // no valid pixel: an empty frame
            for (int a = 0; a < 3; ++a) fr.vmin[a] = 0.0;
            return;
        }
        double ext = 0.0;
        for (int a = 0; a < 3; ++a) {
            const double mnv = ordered_to_dbl(v[a]), mxv = ordered_to_dbl(v[3 + a]);
            fr.vmin[a] = mnv - p.vs * 0.5;
            const double vmax = mxv + p.vs * 0.5;
            ext = fmax(ext, vmax - fr.vmin[a]);
            const long long kmax = (long long)floor((vmax - fr.vmin[a]) / p.vs);
            atomicMax(&kbits[a], (int)(kmax < 0x3FFFFFFF ? kmax : 0x3FFFFFFF));  // voxels per axis - 1
        }
        if (p.vs * 2147483647.0 < ext) fr.err = 1;  // Open3D: "voxel_size is too small."
    }
}

// voxel key = frame << vbits | cell << 3m | local: cell = ((kx >> m) << (by + bz)) | ((ky >> m) << bz) | (kz >> m) on
// the batch's largest per-axis cell ranges (bx, by, bz bits), local = (kx & M) << 2m | (ky & M) << m | (kz & M) --
// lexicographic (cell x, y, z, then voxel x, y, z inside the cell).  key >> 3m is the SOR grid's cell key (grid.h:
// z in the low bits), so the sorted voxels are already grouped by cell, cells of one (frame, x, y) column in z order
struct FbKeys {
    int m;       // log2 of the SOR cell edge in voxels
    int by, bz;  // bits of the cell y / z fields
    int vbits;   // key bits: bx + by + bz + 3m
    int tag;     // u32 keys: the frame tag in bit 31 (vbits <= 31), so that adjacent frames' keys always differ
};
__device__ inline unsigned long long fb_voxel_key(const FbKeys& kb, unsigned long long kx, unsigned long long ky,
                                                  unsigned long long kz) {
    const int m = kb.m;
    const unsigned long long M = (1ull << m) - 1ull;
    const unsigned long long cell = ((kx >> m) << (kb.by + kb.bz)) | ((ky >> m) << kb.bz) | (kz >> m);
    return (cell << (3 * m)) | ((kx & M) << (2 * m)) | ((ky & M) << m) | (kz & M);
}

// the tile again: voxel keys of the valid pixels, emitted in pixel order at the tile's scanned offset, value = global
// pixel index (the unpacked paths: frames above 2^23 pixels, or keys wider than 32 bits).  KeyT = u64: the frame in
// the key's top bits (one sort over the batch); u32: the voxel key only (segmented sort by frame) with the frame's tag
// bit (FbKeys::tag) on top.  The workgroup's outputs are one contiguous range: staged in LDS and stored with
// consecutive lanes on consecutive entries
template <typename KeyT>
__global__ __launch_bounds__(FB_THREADS) void k_fb_keys(FbParams p, FbKeys kb, const int* __restrict__ toff,
                                                        KeyT* __restrict__ keys, unsigned* __restrict__ vals) {
    const int f = blockIdx.y, tile = blockIdx.x;
    const int npx = p.w * p.h;
    const int pix0 = tile * FB_TILE + threadIdx.x * FB_PIX;
    const uint16_t* dep = p.depth + (int64_t)f * npx;
    double m[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) m[k] = p.frames[f].pose[k];
    const double vmin[3] = {p.frames[f].vmin[0], p.frames[f].vmin[1], p.frames[f].vmin[2]};
    float d[FB_PIX];
    unsigned raw[FB_PIX];
    fb_depth8(p, dep, pix0, npx, d, raw);
    int c = 0;
#pragma unroll
    for (int k = 0; k < FB_PIX; ++k) c += (pix0 + k < npx && d[k] > 0.0f) ? 1 : 0;
    // exclusive prefix of the lanes' counts over the workgroup (lane-major = pixel order)
    const int lane = (int)lane_id(), wid = threadIdx.x >> 6;
    int inc = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
    }
    __shared__ int wsum[4];
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    const int base = toff[(int64_t)f * p.tpf + tile];
    int loc = inc - c;
    for (int w = 0; w < wid; ++w) loc += wsum[w];
    const unsigned long long fkey = sizeof(KeyT) == 8 ? (unsigned long long)f << kb.vbits
                                                      : (unsigned long long)(kb.tag ? p.frames[f].tag : 0) << 31;
    __shared__ KeyT s_key[FB_TILE];
    __shared__ unsigned s_val[FB_TILE];
#pragma unroll
    for (int k = 0; k < FB_PIX; ++k) {
        double xyz[3];
        if (pix0 + k < npx && fb_point(p, m, d[k], pix0 + k, xyz)) {
            long long kk[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) kk[a] = (long long)(int)floor_div(xyz[a] - vmin[a], p.vs, p.inv_vs);
            s_key[loc] = (KeyT)(fkey | fb_voxel_key(kb, (unsigned long long)kk[0], (unsigned long long)kk[1],
                                                    (unsigned long long)kk[2]));
            s_val[loc] = (unsigned)((int64_t)f * npx + pix0 + k);
            ++loc;
        }
    }
    __syncthreads();
    const int n = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    for (int i = threadIdx.x; i < n; i += FB_THREADS) {
        keys[base + i] = s_key[i];
        vals[base + i] = s_val[i];
    }
}

// the voxel's SOR grid cell key (grid.h layout: frame << sf | cell): sorted keys k32 (u32 chain, frame tag in bit 31
// when vbits <= 31) or k64 (frame << vbits | voxel key)
struct FbCellKeys {
    const unsigned* k32;
    const unsigned long long* k64;
    int shift;  // 3m
    int vbits;
    int sf;     // grid frame shift (u32 chain: the cell bits)
    unsigned long long* out;
};

// ---- runs (the u32 chain with packed point records) ---------------------------------------------------------
// A run = consecutive pixels of one image row whose points fall in the same voxel (at 5 mm and 1280x720 a voxel spans
// ~1.7 pixels of a row: 813k points -> ~480k runs per configs[2] frame).  The sort groups RUNS instead of points:
// runs of one voxel keep their emission order, which is row-major pixel order, and a run's points are consecutive
// in point order -- so a voxel's points are still summed in point-index order (Open3D's AddPoint order), while the
// sort moves ~0.6x the pairs.  A run's sort value is the point index of its first point; its other points follow in
// the packed records until the next record flagged as a run head (FB_PACK_HEAD) or the frame's end.
// Each tile of a frame emits its runs at the frame's point offset poff[f] + (runs of the frame's earlier tiles),
// found by a decoupled look-back inside the frame (tiles take tickets in start order, so a tile only waits on running
// ones); rlen[f] = the frame's run count (its segment of the sort holds that many, the rest is capacity).

__global__ __launch_bounds__(FB_THREADS) void k_fb_runs(FbParams p, FbKeys kb, const int* __restrict__ toff,
                                                        const int* __restrict__ poff, unsigned* __restrict__ rkeys,
                                                        unsigned* __restrict__ rvals,
                                                        unsigned long long* __restrict__ packed,
                                                        unsigned long long* status, int* ticket, int* __restrict__ rlen) {
    const int f = blockIdx.y;
    __shared__ int s_tile;
    __shared__ int wsum[4];
    __shared__ unsigned s_lastkey[4];
    __shared__ int s_lastval[4];
    __shared__ int s_excl;
    __shared__ unsigned long long s_rec[FB_TILE];
    __shared__ unsigned s_rkey[FB_TILE];
    __shared__ unsigned s_rval[FB_TILE];
    if (threadIdx.x == 0) s_tile = atomicAdd(&ticket[f], 1);
    __syncthreads();
    const int tile = s_tile;  // tiles start in ticket order: the look-back below only waits on running tiles
    const int npx = p.w * p.h;
    const int pix0 = tile * FB_TILE + threadIdx.x * FB_PIX;
    const uint16_t* dep = p.depth + (int64_t)f * npx;
    double m[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) m[k] = p.frames[f].pose[k];
    const double vmin[3] = {p.frames[f].vmin[0], p.frames[f].vmin[1], p.frames[f].vmin[2]};
    float d[FB_PIX];
    unsigned raw[FB_PIX], rgb[FB_PIX], key[FB_PIX];
    bool val[FB_PIX];
    fb_depth8(p, dep, pix0, npx, d, raw);
    fb_color8(p.color + (int64_t)f * npx * 3, pix0, npx, rgb);
#pragma unroll
    for (int k = 0; k < FB_PIX; ++k) {
        double xyz[3];
        val[k] = pix0 + k < npx && fb_point(p, m, d[k], pix0 + k, xyz);
        key[k] = 0u;
        if (val[k]) {
            long long kk[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) kk[a] = (long long)(int)floor_div(xyz[a] - vmin[a], p.vs, p.inv_vs);
            key[k] = (unsigned)fb_voxel_key(kb, (unsigned long long)kk[0], (unsigned long long)kk[1],
                                            (unsigned long long)kk[2]);
        }
    }
    // the previous pixel of the lane's first: the previous lane's last (a shuffle) or the previous wave's last (LDS)
    const int lane = (int)lane_id(), wid = threadIdx.x >> 6;
    unsigned pk = __shfl_up(key[FB_PIX - 1], 1, 64);
    int pv = __shfl_up(val[FB_PIX - 1] ? 1 : 0, 1, 64);
    if (lane == 63) {
        s_lastkey[wid] = key[FB_PIX - 1];
        s_lastval[wid] = val[FB_PIX - 1] ? 1 : 0;
    }
    __syncthreads();
    if (lane == 0) {
        // a tile's first pixel always starts a run (splitting a run at a tile border changes no sum: the pieces
        // stay consecutive in the stable sort), so no tile recomputes its predecessor's last key
        pk = wid == 0 ? 0u : s_lastkey[wid - 1];
        pv = wid == 0 ? 0 : s_lastval[wid - 1];
    }
    int c = 0, nr = 0;
    bool head[FB_PIX];
    int col = pix0 % p.w;  // column of the lane's first pixel; a row starts where it wraps to 0
#pragma unroll
    for (int k = 0; k < FB_PIX; ++k) {
        const bool pvk = k == 0 ? pv != 0 : val[k - 1];
        const unsigned pkk = k == 0 ? pk : key[k - 1];
        head[k] = val[k] && !(pvk && col != 0 && pkk == key[k]);
        c += val[k] ? 1 : 0;
        nr += head[k] ? 1 : 0;
        if (++col >= p.w) col = 0;
    }
    // exclusive prefixes of the lanes' point and run counts over the workgroup (packed: both <= 2048)
    const int both = (nr << 16) | c;
    int inc = both;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
    }
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    int loc = inc - both;
    for (int w = 0; w < wid; ++w) loc += wsum[w];
    const int tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    const int n_pts = tot & 0xFFFF, n_runs = tot >> 16;
    int ploc = loc & 0xFFFF, rloc = loc >> 16;
    const int base = toff[(int64_t)f * p.tpf + tile];  // this tile's first point
    // the frame's runs before this tile: decoupled look-back by wave 0
    if (threadIdx.x < 64) {
        const long long excl = lookback_wave(status + (int64_t)f * p.tpf, tile, (unsigned long long)n_runs);
        if (threadIdx.x == 0) {
            s_excl = (int)excl;
            if (tile == p.tpf - 1) rlen[f] = (int)excl + n_runs;
        }
    }
#pragma unroll
    for (int k = 0; k < FB_PIX; ++k) {
        if (!val[k]) continue;
        s_rec[ploc] = fb_pack((unsigned)(pix0 + k), raw[k], rgb[k], head[k]);
        if (head[k]) {
            s_rkey[rloc] = key[k];
            s_rval[rloc] = (unsigned)(base + ploc);
            ++rloc;
        }
        ++ploc;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n_pts; i += FB_THREADS) packed[base + i] = s_rec[i];
    const int rbase = poff[f] + s_excl;
    for (int i = threadIdx.x; i < n_runs; i += FB_THREADS) {
        rkeys[rbase + i] = s_rkey[i];
        rvals[rbase + i] = s_rval[i];
    }
}

// Voxel heads over the sorted runs, frame by frame (segment f = [poff[f], poff[f] + rlen[f]); the rest of the frame's
// range is capacity the sort left untouched): a frame's first run or a new key.  Grid (chunks, F): the block knows its
// frame; per block the head count, then (after the scan) the heads in order.
constexpr int FB_HEAD_CHUNK = 2048;  // runs per block (256 threads x 8)
__device__ inline bool fb_run_head(const unsigned* __restrict__ keys, int i, int beg) {
    return i == beg || keys[i] != keys[i - 1];
}
__global__ __launch_bounds__(256) void k_fb_heads_count(const unsigned* __restrict__ keys, const int* __restrict__ poff,
                                                        const int* __restrict__ rlen, int chunks, int* __restrict__ counts) {
    const int f = blockIdx.y, b = blockIdx.x;
    const int beg = poff[f], n = rlen[f];
    int c = 0;
    for (int k = 0; k < FB_HEAD_CHUNK / 256; ++k) {
        const int j = b * FB_HEAD_CHUNK + k * 256 + threadIdx.x;
        c += (j < n && fb_run_head(keys, beg + j, beg)) ? 1 : 0;
    }
    c = wave_sum(c);
    __shared__ int ws[4];
    if (lane_id() == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) counts[f * chunks + b] = ws[0] + ws[1] + ws[2] + ws[3];
}
__global__ __launch_bounds__(256) void k_fb_heads_emit(const unsigned* __restrict__ keys, const int* __restrict__ poff,
                                                       const int* __restrict__ rlen, int chunks,
                                                       const int* __restrict__ offs, int* __restrict__ heads) {
    const int f = blockIdx.y, b = blockIdx.x;
    const int beg = poff[f], n = rlen[f];
    int out = offs[f * chunks + b];
    const int lane = (int)lane_id(), wid = threadIdx.x >> 6;
    __shared__ int ws[4];
    for (int k = 0; k < FB_HEAD_CHUNK / 256; ++k) {  // 256 consecutive runs per round, emitted in order
        const int j = b * FB_HEAD_CHUNK + k * 256 + threadIdx.x;
        const bool h = j < n && fb_run_head(keys, beg + j, beg);
        int tot = 0;
        const int ex = wave_excl_count(h, tot);
        if (lane == 0) ws[wid] = tot;
        __syncthreads();
        int before = 0, all = 0;
        for (int w = 0; w < 4; ++w) {
            before += w < wid ? ws[w] : 0;
            all += ws[w];
        }
        if (h) heads[out + before + ex] = beg + j;
        out += all;
        __syncthreads();
    }
}

// one lane per voxel: its runs (sorted values = the runs' first point indices, in emission order) and each run's points
// (consecutive packed records up to the next run head) re-unprojected and summed in point order.  Grid (chunks, F): the
// block knows its frame (voxels voff[f] .. voff[f+1]); the next run's first index is loaded before the current run's
// walk, and each record's successor before its sums.
__global__ __launch_bounds__(256) void k_fb_reduce_runs(FbParams p, const unsigned* __restrict__ sval,
                                                        const unsigned long long* __restrict__ packed,
                                                        const int* __restrict__ poff, const int* __restrict__ rlen,
                                                        const int* __restrict__ heads, const int* __restrict__ voff,
                                                        int64_t P, double* __restrict__ vx, double* __restrict__ vc,
                                                        FbCellKeys ck) {
    const int f = blockIdx.y;
    const int v1 = voff[f + 1];
    const int s = voff[f] + blockIdx.x * 256 + threadIdx.x;
    if (s >= v1) return;
    const int fend = poff[f] + rlen[f];                   // the frame's runs end
    const int pend = f + 1 < p.F ? poff[f + 1] : (int)P;  // the frame's points end
    const int beg = heads[s];
    const int end = s + 1 < v1 ? heads[s + 1] : fend;
    {
        const unsigned vk = ck.vbits < 32 ? (ck.k32[beg] & ((1u << ck.vbits) - 1u)) : ck.k32[beg];
        ck.out[s] = ((unsigned long long)f << ck.sf) | (unsigned long long)(vk >> ck.shift);
    }
    double m[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) m[k] = p.frames[f].pose[k];
    double sp[3] = {0, 0, 0}, sc[3] = {0, 0, 0};
    int cnt = 0;
    int q = (int)sval[beg];
    for (int r = beg; r < end; ++r) {
        const int qn = r + 1 < end ? (int)sval[r + 1] : 0;  // the next run's first point
        unsigned long long rec = packed[q];
        while (true) {
            const unsigned long long nxt = q + 1 < pend ? packed[q + 1] : FB_PACK_HEAD;  // issued before the sums
            const int pix = (int)(rec & ((1u << FB_PACK_PIX_BITS) - 1));
            const float dd = (float)(unsigned)((rec >> FB_PACK_DEPTH_SHIFT) & 0xFFFFu);
            const unsigned rgb = (unsigned)(rec >> (FB_PACK_DEPTH_SHIFT + 16));
            double xyz[3];
            fb_point(p, m, div_rn(dd, p.scale_f, p.rscale_f), pix, xyz);  // valid by construction
#pragma unroll
            for (int a = 0; a < 3; ++a) sp[a] += xyz[a];
            sc[0] += div_rn((double)(rgb & 0xFF), 255.0, 1.0 / 255.0);
            sc[1] += div_rn((double)((rgb >> 8) & 0xFF), 255.0, 1.0 / 255.0);
            sc[2] += div_rn((double)(rgb >> 16), 255.0, 1.0 / 255.0);
            ++cnt;
            if (nxt & FB_PACK_HEAD) break;  // the next record starts another run (or the frame ended)
            rec = nxt;
            ++q;
        }
        q = qn;
    }
    const double cntd = (double)cnt, rc = 1.0 / cntd;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        vx[(int64_t)s * 3 + a] = div_rn(sp[a], cntd, rc);
        vc[(int64_t)s * 3 + a] = div_rn(sc[a], cntd, rc);
    }
}

// one lane per voxel: its points (sorted values = global pixel indices, in index order) re-unprojected from the
// depth / colour images and summed
__global__ __launch_bounds__(256) void k_fb_reduce(FbParams p, const unsigned* __restrict__ sval,
                                                   const int* __restrict__ heads, int64_t K, int64_t P,
                                                   double* __restrict__ vx, double* __restrict__ vc, FbCellKeys ck) {
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= K) return;
    const int64_t beg = heads[s], end = (s + 1 < K) ? heads[s + 1] : P;
    const int npx = p.w * p.h;
    const int f = (int)(sval[beg] / (unsigned)npx);
    if (ck.k32) {
        const unsigned vk = ck.vbits < 32 ? (ck.k32[beg] & ((1u << ck.vbits) - 1u)) : ck.k32[beg];
        ck.out[s] = ((unsigned long long)f << ck.sf) | (unsigned long long)(vk >> ck.shift);
    } else {
        ck.out[s] = ck.k64[beg] >> ck.shift;
    }
    double m[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) m[k] = p.frames[f].pose[k];
    const uint16_t* dep = p.depth + (int64_t)f * npx;
    const uint8_t* col = p.color + (int64_t)f * npx * 3;
    double sp[3] = {0, 0, 0}, sc[3] = {0, 0, 0};
    // points in batches of 4: the batch's index, depth and colour loads are all issued before its in-order sums
    constexpr int VB = 4;
    for (int64_t j0 = beg; j0 < end; j0 += VB) {
        int pix[VB];
        float dd[VB];
        unsigned cc[VB][3];
#pragma unroll
        for (int k = 0; k < VB; ++k) pix[k] = (int)(sval[j0 + k < end ? j0 + k : j0] - (unsigned)f * (unsigned)npx);
#pragma unroll
        for (int k = 0; k < VB; ++k) {
            dd[k] = (float)dep[pix[k]];
            const uint8_t* cp = col + (int64_t)pix[k] * 3;
            cc[k][0] = cp[0], cc[k][1] = cp[1], cc[k][2] = cp[2];
        }
#pragma unroll
        for (int k = 0; k < VB; ++k) {
            if (j0 + k >= end) break;
            double xyz[3];
            // valid by construction (d > 0, below trunc)
            fb_point(p, m, div_rn(dd[k], p.scale_f, p.rscale_f), pix[k], xyz);
#pragma unroll
            for (int a = 0; a < 3; ++a) sp[a] += xyz[a];
            sc[0] += div_rn((double)cc[k][0], 255.0, 1.0 / 255.0);
            sc[1] += div_rn((double)cc[k][1], 255.0, 1.0 / 255.0);
            sc[2] += div_rn((double)cc[k][2], 255.0, 1.0 / 255.0);
        }
    }
    const double cnt = (double)(end - beg), rc = 1.0 / cnt;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        vx[s * 3 + a] = div_rn(sp[a], cnt, rc);
        vc[s * 3 + a] = div_rn(sc[a], cnt, rc);
    }
}

// offs[f] = first voxel whose frame is >= f (f = 0..F); a voxel's frame = its first point's global pixel / npx
__global__ void k_fb_frame_offsets(const unsigned* __restrict__ sval, const int* __restrict__ heads, int64_t K,
                                   int npx, int F, int* __restrict__ offs) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f > F) return;
    int64_t lo = 0, hi = K;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int)(sval[heads[mid]] / (unsigned)npx) < f) lo = mid + 1;
        else hi = mid;
    }
    offs[f] = (int)lo;
}

// the same from the point offsets (segmented sort: frame f's points stay in [poff[f], poff[f + 1]), and each frame's
// first point is a voxel head): offs[f] = first voxel whose head is >= poff[f]
__global__ void k_fb_voxel_offsets(const int* __restrict__ hc, int chunks, int F, const int64_t* __restrict__ total,
                                   int* __restrict__ offs) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;  // the scanned head counts: frame f's first chunk's offset
    if (f < F) offs[f] = hc[f * chunks];
    else if (f == F) offs[F] = (int)*total;
}

// kept_off[f] = first kept entry whose voxel index is >= voff[f]
__global__ void k_fb_kept_offsets(const int64_t* __restrict__ kept, int64_t nk, const int* __restrict__ voff, int F,
                                  int64_t* __restrict__ koff) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f > F) return;
    int64_t lo = 0, hi = nk;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (kept[mid] < voff[f]) lo = mid + 1;
        else hi = mid;
    }
    koff[f] = lo;
}

// kept rows: xyz / rgb of the kept voxels and their index inside their frame's voxel cloud
__global__ __launch_bounds__(256) void k_fb_gather(const int64_t* __restrict__ kept, int64_t nk,
                                                   const int* __restrict__ voff, int F, const double* __restrict__ vx,
                                                   const double* __restrict__ vc, double* __restrict__ ox,
                                                   double* __restrict__ oc, int64_t* __restrict__ oidx) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= nk) return;
    const int64_t i = kept[t];
    int lo = 0, hi = F;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (voff[mid] <= i) lo = mid;
        else hi = mid;
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        ox[t * 3 + a] = vx[i * 3 + a];
        oc[t * 3 + a] = vc[i * 3 + a];
    }
    oidx[t] = i - voff[lo];
}

// voxel heads of the segmented (u32-key, unpacked) sort: a new key, or the first point of a frame.  With the frame tags
// in the keys (FbKeys::tag) adjacent frames' keys always differ; otherwise the frame starts are found from the values'
// global pixel indices
struct SegHeadPredTag {
    const unsigned* keys;
    __device__ bool operator()(int64_t i) const { return i == 0 || keys[i] != keys[i - 1]; }
};
struct SegHeadPredPix {
    const unsigned* keys;
    const unsigned* vals;
    unsigned npx;
    __device__ bool operator()(int64_t i) const {
        return i == 0 || keys[i] != keys[i - 1] || vals[i] / npx != vals[i - 1] / npx;
    }
};

struct KeptEmit {
    int64_t* out;
    __device__ void operator()(int64_t i, int64_t pos) const { out[pos] = i; }
};

}  // namespace ot

using namespace ot;

// grow-only device buffers owned by a filter handle
struct FbBuf {
    void* p = nullptr;
    size_t n = 0;
    void* get(size_t bytes) {
        if (bytes <= n) return p;
        if (p) {
            (void)hipDeviceSynchronize();
            (void)hipFree(p);
            p = nullptr;
            n = 0;
        }
        const size_t nb = bytes + bytes / 8 + 256;
        if (hipMalloc(&p, nb) != hipSuccess) return nullptr;
        n = nb;
        note_alloc();
        return p;
    }
    ~FbBuf() {
        if (p) (void)hipFree(p);
    }
};

struct ot_rgbd_filter {
    ot_intrinsics intr;
    int max_frames;
    double depth_scale, depth_trunc, voxel_size, std_ratio;
    int nb_neighbors;
    // per-run state
    int F = 0;
    int64_t P = 0, K = 0, kept = 0;
    std::vector<int64_t> poff, voff, koff;  // host offsets [F + 1]
    FbBuf b_frames, b_tiles, b_keys, b_vals, b_heads, b_vox, b_avg, b_out, b_misc, b_packed;
    double* vx = nullptr;
    double* vc = nullptr;
    double* kx = nullptr;
    double* kc = nullptr;
    int64_t* kidx = nullptr;
    double* avg = nullptr;
    FbFrame* h_frames = nullptr;  // pinned
};

extern "C" {

ot_status ot_rgbd_filter_create(const ot_intrinsics* intrinsic, int32_t max_frames, double depth_scale,
                                double depth_trunc, double voxel_size, int32_t nb_neighbors, double std_ratio,
                                ot_rgbd_filter** out) {
    if (!out || !intrinsic || intrinsic->width <= 0 || intrinsic->height <= 0 || max_frames < 1 || max_frames > 1024)
        return fail(OT_ERR_INVALID_ARGUMENT, "[rgbd_filter] invalid arguments");
    if (!(voxel_size > 0.0)) return fail(OT_ERR_INVALID_ARGUMENT, "[VoxelDownSample] voxel_size <= 0.");
    if (nb_neighbors < 1 || !(std_ratio > 0))
        return fail(OT_ERR_INVALID_ARGUMENT, "[RemoveStatisticalOutliers] Illegal input parameters, the number of "
                                             "neighbors and standard deviation ratio must be positive.");
    if (nb_neighbors > 64)
        return fail(OT_ERR_INVALID_ARGUMENT, "[RemoveStatisticalOutliers] nb_neighbors > 64 is not supported");
    const int64_t npx = (int64_t)intrinsic->width * intrinsic->height;
    if (npx * max_frames > 0x7FFFFFFF) return fail(OT_ERR_INVALID_ARGUMENT, "[rgbd_filter] batch too large");
    auto* f = new ot_rgbd_filter();
    f->intr = *intrinsic;
    f->max_frames = max_frames;
    f->depth_scale = depth_scale;
    f->depth_trunc = depth_trunc;
    f->voxel_size = voxel_size;
    f->nb_neighbors = nb_neighbors;
    f->std_ratio = std_ratio;
    if (hipHostMalloc((void**)&f->h_frames, sizeof(FbFrame) * max_frames, hipHostMallocDefault) != hipSuccess) {
        delete f;
        return fail(OT_ERR_HIP, "[rgbd_filter] pinned allocation failed");
    }
    *out = f;
    return OT_OK;
}

ot_status ot_rgbd_filter_destroy(ot_rgbd_filter* f) {
    if (!f) return OT_OK;
    (void)hipDeviceSynchronize();
    if (f->h_frames) (void)hipHostFree(f->h_frames);
    delete f;
    return OT_OK;
}

ot_status ot_rgbd_filter_run(ot_rgbd_filter* fl, int32_t n_frames, const uint16_t* depth, const uint8_t* color,
                             const double* extrinsics_host, void* stream_) {
    hipStream_t stream = S(stream_);
    if (!fl || n_frames < 0 || n_frames > fl->max_frames || (n_frames > 0 && (!depth || !color || !extrinsics_host)))
        return fail(OT_ERR_INVALID_ARGUMENT, "[rgbd_filter] invalid arguments");
    const int F = n_frames;
    fl->F = F;
    fl->P = fl->K = fl->kept = 0;
    fl->poff.assign(F + 1, 0);
    fl->voff.assign(F + 1, 0);
    fl->koff.assign(F + 1, 0);
    if (F == 0) return OT_OK;
    const int W = fl->intr.width, H = fl->intr.height, npx = W * H;
    const int tpf = (npx + FB_TILE - 1) / FB_TILE;
    const double vs = fl->voxel_size;
    // ---- frame table: camera poses (Eigen 4x4 inverse of each extrinsic, as Open3D) ------------------------
    // the pinned table is rewritten only after the previous run's copy has completed (every run synchronises)
    for (int f = 0; f < F; ++f) inverse4(extrinsics_host + 16 * f, fl->h_frames[f].pose);
    FbFrame* d_frames = (FbFrame*)fl->b_frames.get(sizeof(FbFrame) * F);
    // layout: tile counts i32 [F*tpf] | align 64 | tile bounds u64 [F*tpf][6] | frame bounds u64 [F][6] | kbits i32 [4]
    // | totals i64 [2] | voff i32 [F+1] | poff i32 [F] | run tickets i32 [F] | run counts i32 [F] | align 8 |
    // run look-back status u64 [F*tpf]
    const size_t tiles_bytes = (size_t)F * tpf * 4 + 63 + (size_t)F * tpf * 48 + (size_t)F * 48 + 16 + 16 +
                               (size_t)(F + 1) * 4 + (size_t)F * 12 + 8 + (size_t)F * tpf * 8;
    int* d_tc = (int*)fl->b_tiles.get(tiles_bytes);
    if (!d_frames || !d_tc) return fail(OT_ERR_HIP, "[rgbd_filter] allocation failed");
    unsigned long long* d_tb = (unsigned long long*)(((uintptr_t)(d_tc + (size_t)F * tpf) + 63) & ~(uintptr_t)63);
    unsigned long long* d_fb = d_tb + (size_t)F * tpf * 6;
    int* d_kbits = (int*)(d_fb + (size_t)F * 6);
    long long* d_tot = (long long*)(d_kbits + 4);
    int* d_voff = (int*)(d_tot + 2);
    int* d_poff = d_voff + (F + 1);
    int* d_ticket = d_poff + F;
    int* d_rlen = d_ticket + F;
    unsigned long long* d_status = (unsigned long long*)(((uintptr_t)(d_rlen + F) + 7) & ~(uintptr_t)7);
    OT_HIP_TRY(hipMemcpyAsync(d_frames, fl->h_frames, sizeof(FbFrame) * F, hipMemcpyHostToDevice, stream));
    OT_HIP_TRY(hipMemsetAsync(d_kbits, 0, sizeof(int) * 4, stream));
    FbParams p;
    p.depth = depth;
    p.color = color;
    p.w = W;
    p.h = H;
    p.tpf = tpf;
    p.scale_f = (float)fl->depth_scale;
    p.rscale_f = 1.0f / p.scale_f;
    p.trunc = fl->depth_trunc;
    p.fx = fl->intr.fx;
    p.fy = fl->intr.fy;
    p.rfx = 1.0 / p.fx;
    p.rfy = 1.0 / p.fy;
    p.cx = fl->intr.cx;
    p.cy = fl->intr.cy;
    p.vs = vs;
    p.inv_vs = 1.0 / vs;
    p.frames = d_frames;
    p.F = F;
    hipLaunchKernelGGL(k_fb_pixels, dim3(tpf, F), dim3(FB_THREADS), 0, stream, p, d_tc, d_tb, d_status);
    hipLaunchKernelGGL(k_fb_setup, dim3(F + 1), dim3(256), 0, stream, p, d_tc, (const unsigned long long*)d_tb, d_fb,
                       d_kbits, d_tot, d_poff, d_ticket);
    OT_LAUNCH_CHECK();
    // ---- sync 1: point count, key widths, frame bounds / origins -------------------------------------------
    struct {
        int kbits[4];
        long long tot[2];
    } hs;
    std::vector<unsigned long long> hfb((size_t)F * 6);
    std::vector<int> hpoff(F);
    OT_HIP_TRY(hipMemcpyAsync(&hs, d_kbits, sizeof(hs), hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipMemcpyAsync(hfb.data(), d_fb, sizeof(unsigned long long) * F * 6, hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipMemcpyAsync(fl->h_frames, d_frames, sizeof(FbFrame) * F, hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipMemcpyAsync(hpoff.data(), d_poff, sizeof(int) * F, hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipStreamSynchronize(stream));
    for (int f = 0; f < F; ++f) fl->poff[f] = hpoff[f];
    for (int f = 0; f < F; ++f)
        if (fl->h_frames[f].err) return fail(OT_ERR_INVALID_ARGUMENT, "[VoxelDownSample] voxel_size is too small.");
    const int64_t P = hs.tot[0];
    fl->P = P;
    fl->poff[F] = P;
    if (P == 0) return OT_OK;
    // SOR cells of 2^m voxels per axis: ~0.9 k points per occupied cell of a surface sampled once per voxel
    // (cell edge vs * sqrt(target) rounded to a power of two in ratio, ties up: the largest m <= 4 with
    // 4^m <= 2 target; m = 2 for nb_neighbors 20; oracle.batch_cell_shift)
    const double ctarget = sor_cell_target(fl->nb_neighbors);
    int m = 0;
    while (m < 4 && std::ldexp(1.0, 2 * (m + 1)) <= 2.0 * ctarget) ++m;
    int cbits[3];
    for (int a = 0; a < 3; ++a) {
        cbits[a] = 0;
        while (cbits[a] < 31 && ((hs.kbits[a] >> m) >> cbits[a]) != 0) ++cbits[a];  // bits of the largest cell index
    }
    int fbits = 0;
    while ((1 << fbits) < F) ++fbits;
    const int vbits = std::max(1, cbits[0] + cbits[1] + cbits[2] + 3 * m);
    const int end_bit = vbits + fbits;
    if (end_bit > 63) return fail(OT_ERR_INVALID_ARGUMENT, "[VoxelDownSample] voxel grid exceeds 64-bit key packing");
    const FbKeys kb{m, cbits[1], cbits[2], vbits, 0};
    // ---- voxel keys in point order, stable sort ------------------------------------------------------------
    unsigned long long* kin = (unsigned long long*)fl->b_keys.get((size_t)P * 16 + 256);
    unsigned* vin = (unsigned*)fl->b_vals.get((size_t)P * 8 + 256);
    int* heads = (int*)fl->b_heads.get((size_t)P * 4 + 256);
    if (!kin || !vin || !heads) return fail(OT_ERR_HIP, "[rgbd_filter] allocation failed");
    unsigned long long* kout = kin + P;
    unsigned* vout = vin + P;
    ot_status st;
    int64_t K = 0;
    const bool seg32 = vbits <= 32 && F <= 64;
    // the bench / production path: u32 keys, frames up to 2^24 pixels -> runs of pixels sorted (packed point records)
    const bool pack = seg32 && npx <= (1 << FB_PACK_PIX_BITS);
    unsigned long long* packed = nullptr;
    std::vector<int> hvoff(F + 1);
    if (pack) {  // runs: one sort segment per frame, [poff[f], poff[f] + rlen[f]) of each frame's point range
        unsigned* k32 = (unsigned*)kin;
        unsigned* k32o = k32 + P;
        packed = (unsigned long long*)fl->b_packed.get((size_t)P * 8 + 256);
        if (!packed) return fail(OT_ERR_HIP, "[rgbd_filter] allocation failed");
        hipLaunchKernelGGL(k_fb_runs, dim3(tpf, F), dim3(FB_THREADS), 0, stream, p, kb, (const int*)d_tc,
                           (const int*)d_poff, k32, vin, packed, d_status, d_ticket, d_rlen);
        OT_LAUNCH_CHECK();
        st = sort_segments_u32_u32(k32, k32o, vin, vout, fl->poff.data(), F, vbits, stream, 3, d_rlen);
        if (st != OT_OK) return st;
        // voxel heads frame by frame: count per (chunk, frame), one scan, emit; sync 2 reads the total
        int maxpts = 0;
        for (int f = 0; f < F; ++f) maxpts = std::max(maxpts, (int)(fl->poff[f + 1] - fl->poff[f]));
        const int chunks = std::max(1, (maxpts + FB_HEAD_CHUNK - 1) / FB_HEAD_CHUNK);
        char* ws = (char*)scratch(sizeof(int) * (size_t)chunks * F + 64, 7);
        if (!ws) return fail(OT_ERR_HIP, "[rgbd_filter] allocation failed");
        int64_t* d_total = (int64_t*)ws;
        int* d_hc = (int*)(ws + 64);
        hipLaunchKernelGGL(k_fb_heads_count, dim3(chunks, F), dim3(256), 0, stream, (const unsigned*)k32o,
                           (const int*)d_poff, (const int*)d_rlen, chunks, d_hc);
        hipLaunchKernelGGL(k_scan_inplace, dim3(1), dim3(1024), 0, stream, d_hc, chunks * F, d_total);
        hipLaunchKernelGGL(k_fb_heads_emit, dim3(chunks, F), dim3(256), 0, stream, (const unsigned*)k32o,
                           (const int*)d_poff, (const int*)d_rlen, chunks, (const int*)d_hc, heads);
        hipLaunchKernelGGL(k_fb_voxel_offsets, dim3((F + 64) / 64), dim3(64), 0, stream, (const int*)d_hc, chunks, F,
                           (const int64_t*)d_total, d_voff);
        OT_LAUNCH_CHECK();
        OT_HIP_TRY(hipMemcpyAsync(&K, d_total, sizeof(int64_t), hipMemcpyDeviceToHost, stream));
        OT_HIP_TRY(hipMemcpyAsync(hvoff.data(), d_voff, sizeof(int) * (F + 1), hipMemcpyDeviceToHost, stream));
        OT_HIP_TRY(hipStreamSynchronize(stream));
    } else if (seg32) {  // 32-bit voxel keys of single points, one sort segment per frame: 8 B per pair per pass
        unsigned* k32 = (unsigned*)kin;
        unsigned* k32o = k32 + P;
        FbKeys kt = kb;
        kt.tag = vbits <= 31;
        if (kt.tag) {  // frame tags: parity of each frame's rank among the non-empty frames (frame table re-sent)
            int r = 0;
            for (int f = 0; f < F; ++f) {
                fl->h_frames[f].tag = r & 1;
                r += fl->poff[f + 1] > fl->poff[f] ? 1 : 0;
            }
            OT_HIP_TRY(hipMemcpyAsync(d_frames, fl->h_frames, sizeof(FbFrame) * F, hipMemcpyHostToDevice, stream));
        }
        hipLaunchKernelGGL((k_fb_keys<unsigned>), dim3(tpf, F), dim3(FB_THREADS), 0, stream, p, kt, (const int*)d_tc,
                           k32, vin);
        OT_LAUNCH_CHECK();
        st = sort_segments_u32_u32(k32, k32o, vin, vout, fl->poff.data(), F, vbits, stream, 3);
        if (st != OT_OK) return st;
        if (kt.tag) st = compact(P, SegHeadPredTag{k32o}, SegHeadEmit{heads}, stream, &K, 7);  // sync 2
        else st = compact(P, SegHeadPredPix{k32o, vout, (unsigned)npx}, SegHeadEmit{heads}, stream, &K, 7);
        if (st != OT_OK) return st;
    } else {
        hipLaunchKernelGGL((k_fb_keys<unsigned long long>), dim3(tpf, F), dim3(FB_THREADS), 0, stream, p, kb,
                           (const int*)d_tc, kin, vin);
        OT_LAUNCH_CHECK();
        st = sort_pairs_u64_u32(kin, kout, vin, vout, (size_t)P, end_bit, stream, 3);
        if (st != OT_OK) return st;
        st = compact(P, SegHeadPred{kout}, SegHeadEmit{heads}, stream, &K, 7);  // synchronises (sync 2)
        if (st != OT_OK) return st;
    }
    if (!pack)
        hipLaunchKernelGGL(k_fb_frame_offsets, dim3((F + 64) / 64), dim3(64), 0, stream, (const unsigned*)vout,
                           (const int*)heads, K, npx, F, d_voff);
    fl->K = K;
    // ---- voxel averages (frame-major, cell-major key order inside a frame) and their SOR cell keys ------------
    double* vox = (double*)fl->b_vox.get((size_t)K * 56 + 256);
    if (!vox) return fail(OT_ERR_HIP, "[rgbd_filter] allocation failed");
    fl->vx = vox;
    fl->vc = vox + K * 3;
    unsigned long long* ckeys = (unsigned long long*)(vox + K * 6);
    const int gsf = cbits[0] + cbits[1] + cbits[2];  // grid key: frame << gsf | cell (z in the low cbits[2] bits)
    // sorted keys: the u32 chain's are at (unsigned*)kin + P (k32o), the u64 path's at kout
    const FbCellKeys ck{seg32 ? (const unsigned*)kin + P : nullptr, seg32 ? nullptr : (const unsigned long long*)kout,
                        3 * m, vbits, gsf, ckeys};
    if (pack) {
        int maxv = 1;
        for (int f = 0; f < F; ++f) maxv = std::max(maxv, hvoff[f + 1] - hvoff[f]);
        hipLaunchKernelGGL(k_fb_reduce_runs, dim3((unsigned)((maxv + 255) / 256), F), dim3(256), 0, stream, p,
                           (const unsigned*)vout, (const unsigned long long*)packed, (const int*)d_poff,
                           (const int*)d_rlen, (const int*)heads, (const int*)d_voff, P, fl->vx, fl->vc, ck);
    } else
        hipLaunchKernelGGL(k_fb_reduce, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, stream, p,
                           (const unsigned*)vout, (const int*)heads, K, P, fl->vx, fl->vc, ck);
    OT_LAUNCH_CHECK();
    if (!pack) OT_HIP_TRY(hipMemcpyAsync(hvoff.data(), d_voff, sizeof(int) * (F + 1), hipMemcpyDeviceToHost, stream));
    // ---- statistical outlier removal over all frames' voxel clouds at once ----------------------------------
    // grid origin per frame = its voxel origin, cell edge 2^m voxels: the cells are the keys' cell fields
    double* d_org = (double*)fl->b_misc.get(sizeof(double) * 3 * F + 64);
    if (!d_org) return fail(OT_ERR_HIP, "[rgbd_filter] allocation failed");
    const double hcell = vs * (double)(1 << m);  // exact (power-of-two scaling)
    std::vector<double> horg((size_t)F * 3);
    for (int f = 0; f < F; ++f)
        for (int a = 0; a < 3; ++a) horg[f * 3 + a] = fl->h_frames[f].vmin[a];
    OT_HIP_TRY(hipMemcpyAsync(d_org, horg.data(), sizeof(double) * 3 * F, hipMemcpyHostToDevice, stream));
    GridBuild gb;
    OT_HIP_TRY(hipStreamSynchronize(stream));  // hvoff (copied above) is needed on the host from here
    st = build_grid_sorted(fl->vx, ckeys, K, F, d_voff, d_org, hcell, cbits, SOR_GRID_NBR, stream, gb,
                           25);  // synchronises
    if (st != OT_OK) return st;
    for (int f = 0; f <= F; ++f) fl->voff[f] = hvoff[f];
    double* avg = (double*)fl->b_avg.get((size_t)K * 8 + (size_t)F * 32 + 256);
    if (!avg) return fail(OT_ERR_HIP, "[rgbd_filter] allocation failed");
    fl->avg = avg;
    double* stats = avg + K;
    st = sor_frames(gb, K, hvoff.data(), fl->nb_neighbors, fl->std_ratio, avg, stats, stream, 28);
    if (st != OT_OK) return st;
    // ---- kept voxels: indices, per-frame offsets, rows ------------------------------------------------------
    int64_t* kept = (int64_t*)fl->b_out.get((size_t)K * (8 + 8 + 48) + (size_t)(F + 1) * 8 + 512);
    if (!kept) return fail(OT_ERR_HIP, "[rgbd_filter] allocation failed");
    int64_t nk = 0;
    st = compact(K, SorKeep{avg, stats, d_voff, F}, KeptEmit{kept}, stream, &nk, 13);  // synchronises
    if (st != OT_OK) return st;
    fl->kept = nk;
    int64_t* d_koff = kept + K;
    fl->kidx = d_koff + (F + 1);
    fl->kx = (double*)(fl->kidx + K);
    fl->kc = fl->kx + K * 3;
    hipLaunchKernelGGL(k_fb_kept_offsets, dim3((F + 64) / 64), dim3(64), 0, stream, (const int64_t*)kept, nk,
                       (const int*)d_voff, F, d_koff);
    if (nk > 0)
        hipLaunchKernelGGL(k_fb_gather, dim3((unsigned)((nk + 255) / 256)), dim3(256), 0, stream, (const int64_t*)kept,
                           nk, (const int*)d_voff, F, (const double*)fl->vx, (const double*)fl->vc, fl->kx, fl->kc,
                           fl->kidx);
    OT_LAUNCH_CHECK();
    OT_HIP_TRY(hipMemcpyAsync(fl->koff.data(), d_koff, sizeof(int64_t) * (F + 1), hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipStreamSynchronize(stream));
    return OT_OK;
}

ot_status ot_rgbd_filter_sizes(const ot_rgbd_filter* fl, int64_t* points_host, int64_t* voxels_host,
                               int64_t* kept_host, int64_t* point_offsets_host, int64_t* voxel_offsets_host,
                               int64_t* kept_offsets_host) {
    if (!fl) return fail(OT_ERR_INVALID_ARGUMENT, "[rgbd_filter] invalid handle");
    if (points_host) *points_host = fl->P;
    if (voxels_host) *voxels_host = fl->K;
    if (kept_host) *kept_host = fl->kept;
    for (int f = 0; f <= fl->F; ++f) {
        if (point_offsets_host) point_offsets_host[f] = fl->poff[f];
        if (voxel_offsets_host) voxel_offsets_host[f] = fl->voff[f];
        if (kept_offsets_host) kept_offsets_host[f] = fl->koff[f];
    }
    return OT_OK;
}

ot_status ot_rgbd_filter_outputs(const ot_rgbd_filter* fl, const double** kept_xyz, const double** kept_rgb,
                                 const int64_t** kept_index, const double** voxel_xyz, const double** voxel_rgb,
                                 const double** voxel_avg_dist) {
    if (!fl) return fail(OT_ERR_INVALID_ARGUMENT, "[rgbd_filter] invalid handle");
    if (kept_xyz) *kept_xyz = fl->kx;
    if (kept_rgb) *kept_rgb = fl->kc;
    if (kept_index) *kept_index = fl->kidx;
    if (voxel_xyz) *voxel_xyz = fl->vx;
    if (voxel_rgb) *voxel_rgb = fl->vc;
    if (voxel_avg_dist) *voxel_avg_dist = fl->avg;
    return OT_OK;
}

ot_status ot_rgbd_filter_copy(const ot_rgbd_filter* fl, int32_t frame, double* kept_xyz, double* kept_rgb,
                              int64_t* kept_index, double* voxel_xyz, double* voxel_rgb, double* voxel_avg_dist,
                              void* stream_) {
    hipStream_t stream = S(stream_);
    if (!fl || frame < -1 || frame >= fl->F) return fail(OT_ERR_INVALID_ARGUMENT, "[rgbd_filter] invalid frame");
    if (fl->F == 0) return OT_OK;
    const int f0 = frame < 0 ? 0 : frame, f1 = frame < 0 ? fl->F : frame + 1;
    const int64_t kb = fl->koff[f0], kn = fl->koff[f1] - kb, vb = fl->voff[f0], vn = fl->voff[f1] - vb;
    if (kn > 0) {
        if (kept_xyz) OT_HIP_TRY(hipMemcpyAsync(kept_xyz, fl->kx + kb * 3, kn * 24, hipMemcpyDeviceToDevice, stream));
        if (kept_rgb) OT_HIP_TRY(hipMemcpyAsync(kept_rgb, fl->kc + kb * 3, kn * 24, hipMemcpyDeviceToDevice, stream));
        if (kept_index) OT_HIP_TRY(hipMemcpyAsync(kept_index, fl->kidx + kb, kn * 8, hipMemcpyDeviceToDevice, stream));
    }
    if (vn > 0) {
        if (voxel_xyz) OT_HIP_TRY(hipMemcpyAsync(voxel_xyz, fl->vx + vb * 3, vn * 24, hipMemcpyDeviceToDevice, stream));
        if (voxel_rgb) OT_HIP_TRY(hipMemcpyAsync(voxel_rgb, fl->vc + vb * 3, vn * 24, hipMemcpyDeviceToDevice, stream));
        if (voxel_avg_dist)
            OT_HIP_TRY(hipMemcpyAsync(voxel_avg_dist, fl->avg + vb, vn * 8, hipMemcpyDeviceToDevice, stream));
    }
    return OT_OK;
}

}  // extern "C"
