// voxel.hip — PointCloud::VoxelDownSample on MI355X (check_one_frame.py:28).
//
//   1. bounds      : per-axis min/max with order-preserving u64 atomics (exact, order independent)
//   2. keys        : key = floor((p - (min - vs/2)) / vs) per axis in float64, packed x-major into u64 with
//                    per-axis bit widths from the extent (device-side, no host round trip)
//   3. sort        : stable LSD radix sort of (key, point index)  => equal keys keep input-index order
//   4. heads       : stable compaction of segment starts
//   5. reduce      : one lane per voxel sums its points in index order and divides by the count — the same
//                    float64 operation sequence as Open3D's AccumulatedPoint, so averages are bit-exact.
// Output voxels are in key order (Open3D: unordered_map order; parity compares sorted sets).
#include <cmath>

#include "compact.h"
#include "sort.h"

namespace ot {

__device__ inline int bits_for(long long v) {  // bits to represent 0..v
    int b = 1;
    while (b < 62 && (v >> b) != 0) ++b;
    return b;
}

__global__ __launch_bounds__(256) void k_voxel_keys(const double* __restrict__ xyz, int64_t n, double vs,
                                                    Bounds* b, unsigned long long* keys, unsigned* idx) {
    double vmin[3];
    int bits[3];
    long long kmax[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        vmin[a] = ordered_to_dbl(b->mn[a]) - vs * 0.5;
        const double vmax = ordered_to_dbl(b->mx[a]) + vs * 0.5;
        kmax[a] = (long long)floor((vmax - vmin[a]) / vs);
        bits[a] = bits_for(kmax[a]);
    }
    const double ext = fmax(fmax(ordered_to_dbl(b->mx[0]) + vs * 0.5 - vmin[0], ordered_to_dbl(b->mx[1]) + vs * 0.5 - vmin[1]),
                            ordered_to_dbl(b->mx[2]) + vs * 0.5 - vmin[2]);
    const bool too_small = vs * 2147483647.0 < ext;
    const bool too_wide = bits[0] + bits[1] + bits[2] > 64;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i == 0 && (too_small || too_wide)) b->err = too_small ? 1 : 2;
    if (i >= n) return;
    long long k[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) k[a] = (long long)(int)floor((xyz[i * 3 + a] - vmin[a]) / vs);
    keys[i] = ((unsigned long long)k[0] << (bits[1] + bits[2])) | ((unsigned long long)k[1] << bits[2]) |
              (unsigned long long)k[2];
    idx[i] = (unsigned)i;
}

__global__ __launch_bounds__(256) void k_voxel_reduce(const double* __restrict__ xyz, const double* __restrict__ rgb,
                                                      const double* __restrict__ nrm, const unsigned* __restrict__ sidx,
                                                      const unsigned long long* __restrict__ skeys,
                                                      const int* __restrict__ heads, int64_t K, int64_t n,
                                                      const Bounds* b, double vs, double* oxyz, double* orgb,
                                                      double* onrm, int32_t* okeys) {
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= K) return;
    const int64_t beg = heads[s];
    const int64_t end = (s + 1 < K) ? heads[s + 1] : n;
    double p[3] = {0, 0, 0}, c[3] = {0, 0, 0}, q[3] = {0, 0, 0};
    // points in batches of 4: the batch's index and row loads are all issued before its (in-order) sums
    constexpr int VB = 4;
    for (int64_t j0 = beg; j0 < end; j0 += VB) {
        int64_t ii[VB];
#pragma unroll
        for (int k = 0; k < VB; ++k) ii[k] = sidx[j0 + k < end ? j0 + k : j0];
        double xp[VB][3], xc[VB][3], xq[VB][3];
#pragma unroll
        for (int k = 0; k < VB; ++k)
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                xp[k][a] = xyz[ii[k] * 3 + a];
                xc[k][a] = rgb ? rgb[ii[k] * 3 + a] : 0.0;
                xq[k][a] = nrm ? nrm[ii[k] * 3 + a] : 0.0;
            }
#pragma unroll
        for (int k = 0; k < VB; ++k) {
            if (j0 + k >= end) break;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                p[a] += xp[k][a];
                if (rgb) c[a] += xc[k][a];
                if (nrm) q[a] += xq[k][a];
            }
        }
    }
    const double cnt = (double)(end - beg);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        oxyz[s * 3 + a] = p[a] / cnt;
        if (rgb) orgb[s * 3 + a] = c[a] / cnt;
        if (nrm) onrm[s * 3 + a] = q[a] / cnt;
    }
    if (okeys) {
        // recover the integer key of this voxel from its first point (same formula as k_voxel_keys)
        const int64_t i = sidx[beg];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const double vmin = ordered_to_dbl(b->mn[a]) - vs * 0.5;
            okeys[s * 3 + a] = (int)floor((xyz[i * 3 + a] - vmin) / vs);
        }
    }
}

}  // namespace ot

using namespace ot;

extern "C" ot_status ot_voxel_down_sample(const double* xyz, const double* rgb, const double* normals, int64_t n,
                                          double voxel_size, double* out_xyz, double* out_rgb, double* out_normals,
                                          int32_t* out_keys, int64_t* n_out_host, void* stream_) {
    hipStream_t stream = S(stream_);
    if (!n_out_host) return fail(OT_ERR_INVALID_ARGUMENT, "[VoxelDownSample] n_out is NULL");
    if (!(voxel_size > 0.0)) return fail(OT_ERR_INVALID_ARGUMENT, "[VoxelDownSample] voxel_size <= 0.");
    *n_out_host = 0;
    if (n <= 0) return OT_OK;
    if (!xyz || !out_xyz || (rgb && !out_rgb) || (normals && !out_normals))
        return fail(OT_ERR_INVALID_ARGUMENT, "[VoxelDownSample] invalid buffers");
    if (n > 0x7FFFFFFF) return fail(OT_ERR_INVALID_ARGUMENT, "[VoxelDownSample] too many points");
    char* ws = (char*)scratch(256 + (size_t)n * (8 + 8 + 4 + 4 + 4), 6);
    if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
    Bounds* b = (Bounds*)ws;
    unsigned long long* kin = (unsigned long long*)(ws + 256);
    unsigned long long* kout = kin + n;
    unsigned* vin = (unsigned*)(kout + n);
    unsigned* vout = vin + n;
    int* heads = (int*)(vout + n);
    unsigned long long* part = (unsigned long long*)scratch(sizeof(unsigned long long) * BOUNDS_BLOCKS * 6, 18);
    if (!part) return fail(OT_ERR_HIP, "scratch allocation failed");
    launch_bounds(xyz, n, b, part, stream);
    // key width on the host (same float64 formula as k_voxel_keys) so the radix sort runs only the passes the
    // packed key needs
    Bounds hb;
    OT_HIP_TRY(hipMemcpyAsync(&hb, b, sizeof(Bounds), hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipStreamSynchronize(stream));
    int end_bit = 0;
    for (int a = 0; a < 3; ++a) {
        const double vmin = ordered_to_dbl(hb.mn[a]) - voxel_size * 0.5;
        const double vmax = ordered_to_dbl(hb.mx[a]) + voxel_size * 0.5;
        const double span = std::floor((vmax - vmin) / voxel_size);
        int bits = 1;
        while (bits < 62 && span >= std::ldexp(1.0, bits)) ++bits;
        end_bit += bits;
    }
    end_bit = std::min(end_bit, 64);
    hipLaunchKernelGGL(k_voxel_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, xyz, n, voxel_size, b,
                       kin, vin);
    OT_LAUNCH_CHECK();
    ot_status st = sort_pairs_u64_u32(kin, kout, vin, vout, (size_t)n, end_bit, stream, 3);
    if (st != OT_OK) return st;
    int64_t K = 0;
    st = compact(n, SegHeadPred{kout}, SegHeadEmit{heads}, stream, &K, 7);  // synchronises
    if (st != OT_OK) return st;
    int err = 0;
    OT_HIP_TRY(hipMemcpyAsync(&err, &b->err, sizeof(int), hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipStreamSynchronize(stream));
    if (err == 1) return fail(OT_ERR_INVALID_ARGUMENT, "[VoxelDownSample] voxel_size is too small.");
    if (err == 2) return fail(OT_ERR_INVALID_ARGUMENT, "[VoxelDownSample] voxel grid exceeds 64-bit key packing");
    hipLaunchKernelGGL(k_voxel_reduce, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, stream, xyz, rgb, normals,
                       vout, kout, heads, K, n, b, voxel_size, out_xyz, out_rgb, out_normals, out_keys);
    OT_LAUNCH_CHECK();
    OT_HIP_TRY(hipStreamSynchronize(stream));
    *n_out_host = K;
    return OT_OK;
}
