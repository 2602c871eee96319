// change.hip — change detection against a saved map (config 5 "diff vs saved map").
//
//   ot_grid_smart_paste : 2d_selective_merge.py:58-69 smart_paste — inside a rectangle, every cell of the new
//                         occupancy grid that carries data (value outside unknown ± threshold) overwrites the
//                         base grid; one lane per cell of the rectangle, plus the count of cells it changed.
//   ot_voxel_key_diff   : voxel-key set difference of two clouds on a common lattice (added = keys of the new
//                         cloud absent from the saved one, removed = the converse), sorted key lists.
//   ot_scan_diff        : diff_node.cpp:103-160 — per beam of a batch of LaserScan pairs (real vs virtual):
//                         "new" when no virtual return within ±window beams lies closer than dist_thresh,
//                         "gone" for the converse; flagged beams are transformed to the map frame and binned
//                         into grid_res cells (C++ truncation).  One lane per (scan, beam).
//   ot_change_grid_*    : diff_node.cpp:163-185 — the time-decayed evidence grid (host state machine: per scan,
//                         hit cells += dt capped at 1.5 time_thresh, others -= decay dt, erased at <= 0), and
//                         publishCloud's cell centres for cells above time_thresh.
#include <algorithm>
#include <cmath>
#include <unordered_map>
#include <vector>

#include "compact.h"
#include "sort.h"

namespace ot {

// ------------------------------------------------------------------------------------------- smart paste
__global__ __launch_bounds__(256) void k_smart_paste(uint8_t* __restrict__ base, const uint8_t* __restrict__ over,
                                                     int w_img, int x, int y, int w, int h, int lo, int hi,
                                                     unsigned long long* changed) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    bool ch = false;
    if (t < (int64_t)w * h) {
        const int r = y + (int)(t / w), c = x + (int)(t % w);
        const int64_t o = (int64_t)r * w_img + c;
        const int v = over[o];
        if (v < lo || v > hi) {
            ch = base[o] != (uint8_t)v;
            base[o] = (uint8_t)v;
        }
    }
    const unsigned long long m = __ballot(ch);
    if (lane_id() == 0 && m) atomicAdd(changed, (unsigned long long)__popcll(m));
}

// ------------------------------------------------------------------------------------------ voxel-key diff
__global__ __launch_bounds__(256) void k_lattice_keys(const double* __restrict__ xyz, int64_t n, double vs, double ox,
                                                      double oy, double oz, unsigned long long* keys, unsigned* idx,
                                                      int* err) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const double fx = floor((xyz[i * 3 + 0] - ox) / vs), fy = floor((xyz[i * 3 + 1] - oy) / vs),
                 fz = floor((xyz[i * 3 + 2] - oz) / vs);
    const bool ok = fabs(fx) < (double)KEY_BIAS && fabs(fy) < (double)KEY_BIAS && fabs(fz) < (double)KEY_BIAS;
    if (!ok) *err = 1;
    keys[i] = ok ? pack_key((int)fx, (int)fy, (int)fz) : 0ull;
    idx[i] = (unsigned)i;
}

struct UniqPred {
    const unsigned long long* k;
    __device__ bool operator()(int64_t i) const { return i == 0 || k[i] != k[i - 1]; }
};
struct UniqEmit {
    const unsigned long long* k;
    unsigned long long* out;
    __device__ void operator()(int64_t i, int64_t pos) const { out[pos] = k[i]; }
};

// keys of `a` absent from the sorted unique list `b`
struct AbsentPred {
    const unsigned long long* a;
    const unsigned long long* b;
    int64_t nb;
    __device__ bool operator()(int64_t i) const {
        const unsigned long long key = a[i];
        int64_t lo = 0, hi = nb;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (b[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        return !(lo < nb && b[lo] == key);
    }
};
struct KeyEmit {
    const unsigned long long* a;
    int32_t* out;
    __device__ void operator()(int64_t i, int64_t pos) const {
        int x, y, z;
        unpack_key(a[i], x, y, z);
        out[pos * 3 + 0] = x;
        out[pos * 3 + 1] = y;
        out[pos * 3 + 2] = z;
    }
};

// sorted unique lattice keys of a cloud -> uniq (device), count on the host
static ot_status unique_keys(const double* xyz, int64_t n, double vs, const double o[3], unsigned long long* uniq,
                             int64_t* nu, int slot, hipStream_t stream) {
    *nu = 0;
    if (n == 0) return OT_OK;
    char* ws = (char*)scratch(256 + (size_t)n * (8 + 8 + 4 + 4), slot);
    if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
    int* err = (int*)ws;
    unsigned long long* kin = (unsigned long long*)(ws + 256);
    unsigned long long* kout = kin + n;
    unsigned* vin = (unsigned*)(kout + n);
    unsigned* vout = vin + n;
    OT_HIP_TRY(hipMemsetAsync(err, 0, sizeof(int), stream));
    hipLaunchKernelGGL(k_lattice_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, xyz, n, vs, o[0], o[1],
                       o[2], kin, vin, err);
    OT_LAUNCH_CHECK();
    ot_status st = sort_pairs_u64_u32(kin, kout, vin, vout, (size_t)n, 63, stream, 3);
    if (st != OT_OK) return st;
    st = compact(n, UniqPred{kout}, UniqEmit{kout, uniq}, stream, nu, slot + 1);  // synchronises
    if (st != OT_OK) return st;
    int e = 0;
    OT_HIP_TRY(hipMemcpyAsync(&e, err, sizeof(int), hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipStreamSynchronize(stream));
    if (e) return fail(OT_ERR_INVALID_ARGUMENT, "[voxel_key_diff] lattice key out of range (voxel_size too small)");
    return OT_OK;
}

// Multi-object form: key = object id | x | y | z lattice offsets, each field with only the bits its range
// needs (one layout for the new and the old clouds, from their joint bounds), so ONE sort / unique / set
// difference serves every object of a hybrid map in as few radix passes as the data allows; equal keys imply
// the same object.
struct ObjLayout {
    int mn[3];       // lattice minimum per axis
    int sx, sy, so;  // key = obj << so | (x - mn0) << sx | (y - mn1) << sy | (z - mn2)
};

constexpr double LATTICE_MAX = 1073741824.0;  // |lattice coordinate| < 2^30

// grid-stride over the points (a fixed grid of at most LB_BLOCKS blocks): per-thread bounds, wave reductions, a
// block reduction in LDS, then one atomic per block and field (a few thousand atomics on 6 words, not one per wave)
constexpr int LB_BLOCKS = 512;
__global__ __launch_bounds__(256) void k_lattice_bounds(const double* __restrict__ xyz, int64_t n, double vs,
                                                        double ox, double oy, double oz, int* b6, int* err) {
    __shared__ int red[6][4];
    const double o[3] = {ox, oy, oz};
    int lo[3] = {0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF}, hi[3] = {-0x7FFFFFFF, -0x7FFFFFFF, -0x7FFFFFFF};
    bool bad = false;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const double f = floor((xyz[i * 3 + a] - o[a]) / vs);
            if (fabs(f) < LATTICE_MAX) {
                lo[a] = min(lo[a], (int)f);
                hi[a] = max(hi[a], (int)f);
            } else {
                bad = true;
            }
        }
    }
    if (bad) *err = 1;
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int a = 0; a < 3; ++a) {  // every lane reaches the whole-wave reductions
        const int l = __ockl_wfred_min_i32(lo[a]), h = __ockl_wfred_max_i32(hi[a]);
        if ((threadIdx.x & 63) == 0) {
            red[a][w] = l;
            red[3 + a][w] = h;
        }
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        const int a = threadIdx.x;
        atomicMin(&b6[a], min(min(red[a][0], red[a][1]), min(red[a][2], red[a][3])));
        atomicMax(&b6[3 + a], max(max(red[3 + a][0], red[3 + a][1]), max(red[3 + a][2], red[3 + a][3])));
    }
}

__global__ __launch_bounds__(256) void k_lattice_keys_obj(const double* __restrict__ xyz, int64_t n, int obj,
                                                          double vs, double ox, double oy, double oz, ObjLayout lay,
                                                          unsigned long long* keys) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const double o[3] = {ox, oy, oz};
    unsigned long long f[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) f[a] = (unsigned long long)((int)floor((xyz[i * 3 + a] - o[a]) / vs) - lay.mn[a]);
    keys[i] = ((unsigned long long)obj << lay.so) | (f[0] << lay.sx) | (f[1] << lay.sy) | f[2];
}

struct ObjKeyEmit {
    const unsigned long long* a;
    int32_t* out;  // [k][4]: object, x, y, z
    ObjLayout lay;
    __device__ void operator()(int64_t i, int64_t pos) const {
        const unsigned long long k = a[i];
        out[pos * 4 + 0] = (int)(k >> lay.so);
        out[pos * 4 + 1] = (int)((k >> lay.sx) & ((1ull << (lay.so - lay.sx)) - 1ull)) + lay.mn[0];
        out[pos * 4 + 2] = (int)((k >> lay.sy) & ((1ull << (lay.sx - lay.sy)) - 1ull)) + lay.mn[1];
        out[pos * 4 + 3] = (int)(k & ((1ull << lay.sy) - 1ull)) + lay.mn[2];
    }
};

// sorted unique object-lattice keys of the concatenated clouds of n_obj objects (offsets: host, n_obj + 1)
static ot_status unique_obj_keys(const double* xyz, const int64_t* off, int n_obj, double vs, const double o[3],
                                 const ObjLayout& lay, int end_bit, unsigned long long* uniq, int64_t* nu, int slot,
                                 hipStream_t stream) {
    *nu = 0;
    const int64_t n = off[n_obj];
    if (n == 0) return OT_OK;
    char* ws = (char*)scratch(256 + (size_t)n * (8 + 8 + 4 + 4), slot);
    if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
    unsigned long long* kin = (unsigned long long*)(ws + 256);
    unsigned long long* kout = kin + n;
    unsigned* vin = (unsigned*)(kout + n);
    unsigned* vout = vin + n;
    for (int j = 0; j < n_obj; ++j) {
        const int64_t m = off[j + 1] - off[j];
        if (m > 0)
            hipLaunchKernelGGL(k_lattice_keys_obj, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, stream,
                               xyz + off[j] * 3, m, j, vs, o[0], o[1], o[2], lay, kin + off[j]);
    }
    OT_LAUNCH_CHECK();
    ot_status st = sort_pairs_u64_u32(kin, kout, vin, vout, (size_t)n, end_bit, stream, 3);  // values unused
    if (st != OT_OK) return st;
    return compact(n, UniqPred{kout}, UniqEmit{kout, uniq}, stream, nu, slot + 1);  // synchronises
}

// ------------------------------------------------------------------------------------------- scan diff
struct ScanPose {
    double tx, ty, cyaw, syaw;  // translation and cos / sin of the map-frame yaw (host-computed)
};

// beam endpoint in the sensor frame, float as the reference: r * std::cos(angle), angle = angle_min + i * inc.
// The per-beam cos / sin tables are computed on the host with the same libm float functions the node calls
// (glibc cosf / sinf are not correctly rounded, so a device-side evaluation would differ in the last ulp).
__device__ inline void beam_xy(float r, const float2* __restrict__ cs, int i, float& x, float& y) {
    const float2 c = cs[i];
    x = r * c.x;
    y = r * c.y;
}

// hypotf(dx, dy) as glibc computes it: sqrt of the double sum of double squares, rounded to float
__device__ inline float hypot_f(float dx, float dy) {
    const double x = dx, y = dy;
    return (float)sqrt(x * x + y * y);
}

__global__ __launch_bounds__(256) void k_scan_diff(const float* __restrict__ real, const float* __restrict__ virt,
                                                   int n_scans, int n_beams, const float2* __restrict__ rcs,
                                                   float r_max, const float2* __restrict__ vcs, double thresh, int window,
                                                   const ScanPose* __restrict__ poses, double grid_res,
                                                   uint8_t* __restrict__ new_flag, uint8_t* __restrict__ gone_flag,
                                                   int32_t* __restrict__ new_key, int32_t* __restrict__ gone_key) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)n_scans * n_beams) return;
    const int b = (int)(t / n_beams), i = (int)(t % n_beams);
    const float* R = real + (int64_t)b * n_beams;
    const float* V = virt + (int64_t)b * n_beams;
    const ScanPose P = poses[b];
    const int j0 = max(0, i - window), j1 = min(n_beams, i + window);
    // --- 1. new: a real return with no virtual return nearby
    uint8_t fn = 0;
    int kx = 0, ky = 0;
    const float rr = R[i];
    if (!(isnan(rr) || isinf(rr) || rr > r_max)) {
        float rx, ry;
        beam_xy(rr, rcs, i, rx, ry);
        bool near = false;
        for (int j = j0; j < j1 && !near; ++j) {
            const float rv = V[j];
            if (isinf(rv)) continue;
            float vx, vy;
            beam_xy(rv, vcs, j, vx, vy);
            near = (double)hypot_f(rx - vx, ry - vy) < thresh;
        }
        if (!near) {
            fn = 1;
            const double px = P.tx + ((double)rx * P.cyaw - (double)ry * P.syaw);
            const double py = P.ty + ((double)rx * P.syaw + (double)ry * P.cyaw);
            kx = (int)(px / grid_res);
            ky = (int)(py / grid_res);
        }
    }
    new_flag[t] = fn;
    new_key[t * 2 + 0] = kx;
    new_key[t * 2 + 1] = ky;
    // --- 2. gone: a virtual return with no real return nearby
    uint8_t fg = 0;
    kx = ky = 0;
    const float rv = V[i];
    if (!(isinf(rv) || isnan(rv))) {
        float vx, vy;
        beam_xy(rv, vcs, i, vx, vy);
        bool still = false;
        for (int j = j0; j < j1 && !still; ++j) {
            const float r2 = R[j];
            if (isinf(r2) || r2 > r_max) continue;
            float rx, ry;
            beam_xy(r2, rcs, j, rx, ry);
            still = (double)hypot_f(vx - rx, vy - ry) < thresh;
        }
        if (!still) {
            fg = 1;
            const double px = P.tx + ((double)vx * P.cyaw - (double)vy * P.syaw);
            const double py = P.ty + ((double)vx * P.syaw + (double)vy * P.cyaw);
            kx = (int)(px / grid_res);
            ky = (int)(py / grid_res);
        }
    }
    gone_flag[t] = fg;
    gone_key[t * 2 + 0] = kx;
    gone_key[t * 2 + 1] = ky;
}

// ------------------------------------------------------------------------------------------- virtual scan
// virtual_scan_node.cpp:258-290: per beam, march the ray from the robot in steps of one map resolution:
// dist += res; p = robot + dist * (cos, sin)(global angle); cell = (int)((p - origin) / res); stop off-map; a cell
// equal to 100 (occupied) returns dist as the range.  All double, as the node; cos / sin of the global angle come
// from a host table (libm double cos / sin, as the node links).
__global__ __launch_bounds__(256) void k_virtual_scan(const int8_t* __restrict__ grid, int height, int width,
                                                      double res, double ox, double oy, int n_scans, int n_beams,
                                                      double range_max, const double* __restrict__ robot,
                                                      const double2* __restrict__ cs, float* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)n_scans * n_beams) return;
    const int b = (int)(t / n_beams);
    const double rx = robot[b * 2 + 0], ry = robot[b * 2 + 1];
    const double2 c = cs[t];
    float r = INFINITY;
    double dist = 0.0;
    while (dist < range_max) {
        dist += res;
        const double px = rx + dist * c.x;
        const double py = ry + dist * c.y;
        const int gx = (int)((px - ox) / res);
        const int gy = (int)((py - oy) / res);
        if (gx < 0 || gx >= width || gy < 0 || gy >= height) break;
        if (grid[(int64_t)gy * width + gx] == 100) {
            r = (float)dist;
            break;
        }
    }
    out[t] = r;
}

}  // namespace ot

// time-decayed evidence grid of diff_node.cpp (host state; the per-scan update is O(cells))
struct ot_change_grid {
    double time_thresh = 2.0, decay_rate = 0.5, grid_res = 0.1;
    std::unordered_map<unsigned long long, float> cells;
};

using namespace ot;

static inline unsigned long long key2(int x, int y) {
    return ((unsigned long long)(unsigned)x << 32) | (unsigned long long)(unsigned)y;
}

extern "C" {

ot_status ot_grid_smart_paste(uint8_t* base, const uint8_t* overlay, int32_t height, int32_t width, int32_t x,
                              int32_t y, int32_t w, int32_t h, int32_t unknown, int32_t threshold,
                              int64_t* n_changed_host, void* stream_) {
    hipStream_t stream = S(stream_);
    if (n_changed_host) *n_changed_host = 0;
    if (!base || !overlay || height < 0 || width < 0)
        return fail(OT_ERR_INVALID_ARGUMENT, "[smart_paste] invalid arguments");
    // 2d_selective_merge.py:59-60: a rectangle reaching outside the image leaves the base unchanged
    if (x < 0 || y < 0 || (int64_t)x + w > width || (int64_t)y + h > height || w <= 0 || h <= 0) return OT_OK;
    unsigned long long* d = (unsigned long long*)scratch(64, 30);
    if (!d) return fail(OT_ERR_HIP, "scratch allocation failed");
    OT_HIP_TRY(hipMemsetAsync(d, 0, sizeof(unsigned long long), stream));
    const int64_t nt = (int64_t)w * h;
    hipLaunchKernelGGL(k_smart_paste, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, stream, base, overlay, width,
                       x, y, w, h, unknown - threshold, unknown + threshold, d);
    OT_LAUNCH_CHECK();
    if (n_changed_host) {
        unsigned long long c = 0;
        OT_HIP_TRY(hipMemcpyAsync(&c, d, sizeof(c), hipMemcpyDeviceToHost, stream));
        OT_HIP_TRY(hipStreamSynchronize(stream));
        *n_changed_host = (int64_t)c;
    }
    return OT_OK;
}

ot_status ot_voxel_key_diff(const double* new_xyz, int64_t n, const double* old_xyz, int64_t m, double voxel_size,
                            const double origin[3], int32_t* out_added, int64_t* n_added_host, int32_t* out_removed,
                            int64_t* n_removed_host, void* stream_) {
    hipStream_t stream = S(stream_);
    if (!n_added_host || !n_removed_host || !origin)
        return fail(OT_ERR_INVALID_ARGUMENT, "[voxel_key_diff] invalid arguments");
    *n_added_host = *n_removed_host = 0;
    if (!(voxel_size > 0.0)) return fail(OT_ERR_INVALID_ARGUMENT, "[voxel_key_diff] voxel_size <= 0.");
    if (n < 0 || m < 0 || (n > 0 && !new_xyz) || (m > 0 && !old_xyz) || n > 0x7FFFFFFF || m > 0x7FFFFFFF)
        return fail(OT_ERR_INVALID_ARGUMENT, "[voxel_key_diff] invalid buffers");
    unsigned long long* ua = (unsigned long long*)scratch((size_t)std::max<int64_t>(n, 1) * 8 + 64, 31);
    unsigned long long* ub = (unsigned long long*)scratch((size_t)std::max<int64_t>(m, 1) * 8 + 64, 32);
    if (!ua || !ub) return fail(OT_ERR_HIP, "scratch allocation failed");
    int64_t na = 0, nb = 0;
    ot_status st = unique_keys(new_xyz, n, voxel_size, origin, ua, &na, 33, stream);
    if (st != OT_OK) return st;
    st = unique_keys(old_xyz, m, voxel_size, origin, ub, &nb, 33, stream);
    if (st != OT_OK) return st;
    if (na > 0) {
        if (!out_added) return fail(OT_ERR_INVALID_ARGUMENT, "[voxel_key_diff] out_added is NULL");
        st = compact(na, AbsentPred{ua, ub, nb}, KeyEmit{ua, out_added}, stream, n_added_host, 35);
        if (st != OT_OK) return st;
    }
    if (nb > 0) {
        if (!out_removed) return fail(OT_ERR_INVALID_ARGUMENT, "[voxel_key_diff] out_removed is NULL");
        st = compact(nb, AbsentPred{ub, ua, na}, KeyEmit{ub, out_removed}, stream, n_removed_host, 36);
        if (st != OT_OK) return st;
    }
    return OT_OK;
}

ot_status ot_voxel_key_diff_multi(const double* new_xyz, const int64_t* new_offsets, const double* old_xyz,
                                  const int64_t* old_offsets, int32_t n_objects, double voxel_size,
                                  const double origin[3], int32_t* out_added, int64_t* n_added_host,
                                  int32_t* out_removed, int64_t* n_removed_host, void* stream_) {
    hipStream_t stream = S(stream_);
    if (!n_added_host || !n_removed_host || !origin || !new_offsets || !old_offsets || n_objects < 0 ||
        n_objects > (1 << 11))
        return fail(OT_ERR_INVALID_ARGUMENT, "[voxel_key_diff] invalid arguments");
    *n_added_host = *n_removed_host = 0;
    if (!(voxel_size > 0.0)) return fail(OT_ERR_INVALID_ARGUMENT, "[voxel_key_diff] voxel_size <= 0.");
    if (n_objects == 0) return OT_OK;
    const int64_t n = new_offsets[n_objects], m = old_offsets[n_objects];
    if (n < 0 || m < 0 || (n > 0 && !new_xyz) || (m > 0 && !old_xyz) || n > 0x7FFFFFFF || m > 0x7FFFFFFF)
        return fail(OT_ERR_INVALID_ARGUMENT, "[voxel_key_diff] invalid buffers");
    unsigned long long* ua = (unsigned long long*)scratch((size_t)std::max<int64_t>(n, 1) * 8 + 64, 31);
    unsigned long long* ub = (unsigned long long*)scratch((size_t)std::max<int64_t>(m, 1) * 8 + 64, 32);
    if (!ua || !ub) return fail(OT_ERR_HIP, "scratch allocation failed");
    if (n + m == 0) return OT_OK;
    // joint lattice bounds of both cloud sets -> the key layout
    int* b6 = (int*)scratch(64, 37);
    if (!b6) return fail(OT_ERR_HIP, "scratch allocation failed");
    OT_HIP_TRY(hipMemsetAsync(b6, 0x7F, sizeof(int) * 3, stream));      // +large: minima
    OT_HIP_TRY(hipMemsetAsync(b6 + 3, 0x80, sizeof(int) * 3, stream));  // -large: maxima
    OT_HIP_TRY(hipMemsetAsync(b6 + 6, 0, sizeof(int), stream));         // error flag
    if (n > 0)
        hipLaunchKernelGGL(k_lattice_bounds, dim3((unsigned)std::min<int64_t>((n + 255) / 256, LB_BLOCKS)), dim3(256), 0,
                           stream, new_xyz, n, voxel_size, origin[0], origin[1], origin[2], b6, b6 + 6);
    if (m > 0)
        hipLaunchKernelGGL(k_lattice_bounds, dim3((unsigned)std::min<int64_t>((m + 255) / 256, LB_BLOCKS)), dim3(256), 0,
                           stream, old_xyz, m, voxel_size, origin[0], origin[1], origin[2], b6, b6 + 6);
    OT_LAUNCH_CHECK();
    int hb[7];
    OT_HIP_TRY(hipMemcpyAsync(hb, b6, sizeof(hb), hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipStreamSynchronize(stream));
    if (hb[6]) return fail(OT_ERR_INVALID_ARGUMENT, "[voxel_key_diff] lattice key out of range (voxel_size too small)");
    auto bits_for = [](long long v) {  // bits to represent 0..v
        int b = 1;
        while (b < 62 && (v >> b) != 0) ++b;
        return b;
    };
    ObjLayout lay;
    int bx[3];
    for (int a = 0; a < 3; ++a) {
        lay.mn[a] = hb[a];
        bx[a] = bits_for((long long)hb[3 + a] - hb[a]);
    }
    lay.sy = bx[2];
    lay.sx = bx[1] + bx[2];
    lay.so = bx[0] + bx[1] + bx[2];
    const int end_bit = lay.so + (n_objects > 1 ? bits_for(n_objects - 1) : 0);
    if (end_bit > 64) return fail(OT_ERR_INVALID_ARGUMENT, "[voxel_key_diff] lattice extent too large for 64-bit keys");
    int64_t na = 0, nb = 0;
    ot_status st = unique_obj_keys(new_xyz, new_offsets, n_objects, voxel_size, origin, lay, end_bit, ua, &na, 33,
                                   stream);
    if (st != OT_OK) return st;
    st = unique_obj_keys(old_xyz, old_offsets, n_objects, voxel_size, origin, lay, end_bit, ub, &nb, 33, stream);
    if (st != OT_OK) return st;
    if (na > 0) {
        if (!out_added) return fail(OT_ERR_INVALID_ARGUMENT, "[voxel_key_diff] out_added is NULL");
        st = compact(na, AbsentPred{ua, ub, nb}, ObjKeyEmit{ua, out_added, lay}, stream, n_added_host, 35);
        if (st != OT_OK) return st;
    }
    if (nb > 0) {
        if (!out_removed) return fail(OT_ERR_INVALID_ARGUMENT, "[voxel_key_diff] out_removed is NULL");
        st = compact(nb, AbsentPred{ub, ua, na}, ObjKeyEmit{ub, out_removed, lay}, stream, n_removed_host, 36);
        if (st != OT_OK) return st;
    }
    return OT_OK;
}

ot_status ot_scan_diff(const float* real_ranges, const float* virtual_ranges, int32_t n_scans, int32_t n_beams,
                       float real_angle_min, float real_angle_increment, float real_range_max,
                       float virtual_angle_min, float virtual_angle_increment, double distance_threshold,
                       int32_t search_window, const double* poses_host, double grid_resolution, uint8_t* new_flags,
                       uint8_t* gone_flags, int32_t* new_keys, int32_t* gone_keys, void* stream_) {
    hipStream_t stream = S(stream_);
    if (n_scans < 0 || n_beams < 0 || search_window < 0 || !(grid_resolution > 0.0))
        return fail(OT_ERR_INVALID_ARGUMENT, "[ChangeDetector] invalid arguments");
    const int64_t nt = (int64_t)n_scans * n_beams;
    if (nt == 0) return OT_OK;
    if (!real_ranges || !virtual_ranges || !poses_host || !new_flags || !gone_flags || !new_keys || !gone_keys)
        return fail(OT_ERR_INVALID_ARGUMENT, "[ChangeDetector] invalid buffers");
    // map-frame yaw of each scan from its quaternion, as transformPoint (diff_node.cpp:231-236), on the host
    std::vector<ScanPose> hp(n_scans);
    for (int b = 0; b < n_scans; ++b) {
        const double* p = poses_host + (size_t)b * 7;  // tx ty tz qx qy qz qw
        const double qx = p[3], qy = p[4], qz = p[5], qw = p[6];
        const double yaw = std::atan2(2.0 * (qw * qz + qx * qy), 1.0 - 2.0 * (qy * qy + qz * qz));
        hp[b] = ScanPose{p[0], p[1], std::cos(yaw), std::sin(yaw)};
    }
    // beam directions: angle = angle_min + i * increment in float, then std::cos / std::sin of that float
    std::vector<float2> cs((size_t)n_beams * 2);
    for (int i = 0; i < n_beams; ++i) {
        const float ar = real_angle_min + i * real_angle_increment;
        const float av = virtual_angle_min + i * virtual_angle_increment;
        cs[i] = make_float2(std::cos(ar), std::sin(ar));
        cs[(size_t)n_beams + i] = make_float2(std::cos(av), std::sin(av));
    }
    ScanPose* dp = (ScanPose*)scratch(sizeof(ScanPose) * (size_t)n_scans + 64, 37);
    float2* dcs = (float2*)scratch(sizeof(float2) * cs.size() + 64, 38);
    if (!dp || !dcs) return fail(OT_ERR_HIP, "scratch allocation failed");
    OT_HIP_TRY(hipMemcpyAsync(dp, hp.data(), sizeof(ScanPose) * (size_t)n_scans, hipMemcpyHostToDevice, stream));
    OT_HIP_TRY(hipMemcpyAsync(dcs, cs.data(), sizeof(float2) * cs.size(), hipMemcpyHostToDevice, stream));
    hipLaunchKernelGGL(k_scan_diff, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, stream, real_ranges,
                       virtual_ranges, n_scans, n_beams, (const float2*)dcs, real_range_max,
                       (const float2*)(dcs + n_beams), distance_threshold, search_window, (const ScanPose*)dp,
                       grid_resolution, new_flags, gone_flags, new_keys, gone_keys);
    OT_LAUNCH_CHECK();
    OT_HIP_TRY(hipStreamSynchronize(stream));  // hp / cs are released on return
    return OT_OK;
}

ot_status ot_virtual_scan(const int8_t* grid, int32_t height, int32_t width, float resolution, float origin_x,
                          float origin_y, int32_t n_scans, int32_t n_beams, float angle_min, float angle_increment,
                          float range_max, const double* poses_host, float* out_ranges, void* stream_) {
    hipStream_t stream = S(stream_);
    if (!grid || !poses_host || !out_ranges || height <= 0 || width <= 0 || n_scans < 0 || n_beams < 0 ||
        !(resolution > 0.0f) || (int64_t)height * width > 0x7FFFFFFF)
        return fail(OT_ERR_INVALID_ARGUMENT, "[VirtualScan] invalid arguments");
    const int64_t nt = (int64_t)n_scans * n_beams;
    if (nt == 0) return OT_OK;
    // global beam angles as the node forms them: angle = angle_min + i * angle_increment (float), promoted to
    // double and added to the robot yaw; their cos / sin from the host libm
    std::vector<double2> cs((size_t)nt);
    std::vector<double> robot((size_t)n_scans * 2);
    for (int b = 0; b < n_scans; ++b) {
        const double x = poses_host[b * 3 + 0], y = poses_host[b * 3 + 1], yaw = poses_host[b * 3 + 2];
        robot[(size_t)b * 2] = x;
        robot[(size_t)b * 2 + 1] = y;
        for (int i = 0; i < n_beams; ++i) {
            const double angle = angle_min + i * angle_increment;
            const double g = yaw + angle;
            cs[(size_t)b * n_beams + i] = make_double2(std::cos(g), std::sin(g));
        }
    }
    double2* dcs = (double2*)scratch(sizeof(double2) * (size_t)nt + 64, 39);
    double* drob = (double*)scratch(sizeof(double) * robot.size() + 64, 40);
    if (!dcs || !drob) return fail(OT_ERR_HIP, "scratch allocation failed");
    OT_HIP_TRY(hipMemcpyAsync(dcs, cs.data(), sizeof(double2) * cs.size(), hipMemcpyHostToDevice, stream));
    OT_HIP_TRY(hipMemcpyAsync(drob, robot.data(), sizeof(double) * robot.size(), hipMemcpyHostToDevice, stream));
    hipLaunchKernelGGL(k_virtual_scan, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, stream, grid, height, width,
                       (double)resolution, (double)origin_x, (double)origin_y, n_scans, n_beams, (double)range_max,
                       (const double*)drob, (const double2*)dcs, out_ranges);
    OT_LAUNCH_CHECK();
    OT_HIP_TRY(hipStreamSynchronize(stream));  // host tables are released on return
    return OT_OK;
}

ot_status ot_change_grid_create(double time_threshold, double decay_rate, double grid_resolution,
                                ot_change_grid** out) {
    if (!out || !(grid_resolution > 0.0)) return fail(OT_ERR_INVALID_ARGUMENT, "[ChangeDetector] invalid grid");
    ot_change_grid* g = new ot_change_grid();
    g->time_thresh = time_threshold;
    g->decay_rate = decay_rate;
    g->grid_res = grid_resolution;
    *out = g;
    return OT_OK;
}

ot_status ot_change_grid_destroy(ot_change_grid* g) {
    delete g;
    return OT_OK;
}

ot_status ot_change_grid_update(ot_change_grid* g, const int32_t* keys_host, const uint8_t* flags_host, int64_t n,
                                double dt) {
    if (!g || (n > 0 && (!keys_host || !flags_host)))
        return fail(OT_ERR_INVALID_ARGUMENT, "[ChangeDetector] invalid arguments");
    std::unordered_map<unsigned long long, bool> hits;
    for (int64_t i = 0; i < n; ++i)
        if (flags_host[i]) hits[key2(keys_host[i * 2], keys_host[i * 2 + 1])] = true;
    const double cap = g->time_thresh * 1.5;
    for (const auto& h : hits) {
        float& v = g->cells[h.first];
        v += dt;
        if (v > cap) v = (float)cap;
    }
    for (auto it = g->cells.begin(); it != g->cells.end();) {
        if (hits.find(it->first) == hits.end()) it->second -= (g->decay_rate * dt);
        if (it->second <= 0.0) it = g->cells.erase(it);
        else ++it;
    }
    return OT_OK;
}

ot_status ot_change_grid_publish(const ot_change_grid* g, float* out_xyz_host, int64_t capacity, int64_t* n_host) {
    if (!g || !n_host) return fail(OT_ERR_INVALID_ARGUMENT, "[ChangeDetector] invalid arguments");
    std::vector<unsigned long long> keys;
    for (const auto& c : g->cells)
        if (c.second > g->time_thresh) keys.push_back(c.first);
    // canonical order (the node emits unordered_map order): by (x, y) as signed integers
    std::sort(keys.begin(), keys.end(), [](unsigned long long a, unsigned long long b) {
        const int ax = (int)(unsigned)(a >> 32), bx = (int)(unsigned)(b >> 32);
        if (ax != bx) return ax < bx;
        return (int)(unsigned)a < (int)(unsigned)b;
    });
    *n_host = (int64_t)keys.size();
    if (!out_xyz_host) return OT_OK;
    if (capacity < (int64_t)keys.size()) return fail(OT_ERR_CAPACITY, "[ChangeDetector] output capacity too small");
    for (size_t i = 0; i < keys.size(); ++i) {
        const int x = (int)(unsigned)(keys[i] >> 32), y = (int)(unsigned)keys[i];
        out_xyz_host[i * 3 + 0] = (float)((x * g->grid_res) + (g->grid_res / 2.0));
        out_xyz_host[i * 3 + 1] = (float)((y * g->grid_res) + (g->grid_res / 2.0));
        out_xyz_host[i * 3 + 2] = 0.0f;
    }
    return OT_OK;
}

}  // extern "C"
