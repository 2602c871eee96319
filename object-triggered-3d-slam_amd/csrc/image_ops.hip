// image_ops.hip — depth conversion, ray-length multiplier, unprojection with stable compaction,
// Z-mask compaction, row gather and occupancy-grid → point conversion.
//
// All parity-critical arithmetic is compiled with -ffp-contract=off (no FMA contraction) and uses IEEE
// division / sqrt (HIP's default correctly-rounded f32 div/sqrt), so results are bit-identical to the CPU
// restatement in oracle/otslam_oracle.cpp.
#include "compact.h"

namespace ot {

// ---------------------------------------------------------------------------------------------------
// Image::ConvertDepthToFloatImage: f = (float)u16; f /= (float)scale; if (f >= trunc) f = 0.
// 8 pixels per lane (16-B load, 2 x 16-B stores).
__global__ __launch_bounds__(256) void k_depth_to_float(const uint16_t* __restrict__ in, float* __restrict__ out,
                                                        int64_t n, float scale, double trunc) {
    const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
    if (i0 + 8 <= n && ((reinterpret_cast<uintptr_t>(in) & 15) == 0) && ((reinterpret_cast<uintptr_t>(out) & 15) == 0)) {
        uint4 raw = *reinterpret_cast<const uint4*>(in + i0);
        const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
        float f[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            f[2 * k] = (float)(w[k] & 0xFFFFu);
            f[2 * k + 1] = (float)(w[k] >> 16);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            f[k] = f[k] / scale;
            if ((double)f[k] >= trunc) f[k] = 0.0f;
        }
        *reinterpret_cast<float4*>(out + i0) = make_float4(f[0], f[1], f[2], f[3]);
        *reinterpret_cast<float4*>(out + i0 + 4) = make_float4(f[4], f[5], f[6], f[7]);
    } else {
        for (int64_t i = i0; i < n && i < i0 + 8; ++i) {
            float f = (float)in[i];
            f = f / scale;
            if ((double)f >= trunc) f = 0.0f;
            out[i] = f;
        }
    }
}

// Image::CreateDepthToCameraDistanceMultiplierFloatImage
__global__ __launch_bounds__(256) void k_depth_multiplier(int w, int h, float inv_fx, float inv_fy, float cx,
                                                          float cy, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)w * h) return;
    const int row = (int)(i / w), col = (int)(i % w);
    const float xx = ((float)col - cx) * inv_fx;
    const float yy = ((float)row - cy) * inv_fy;
    const float a = xx * xx;
    const float b = yy * yy;
    out[i] = sqrtf((a + b) + 1.0f);
}

// ------------------------------------------------------------------------------------ unprojection
struct UnprojPred {
    const float* depth;
    int w, ws, stride;
    __device__ bool operator()(int64_t s) const {
        const unsigned su = (unsigned)s, q = su / (unsigned)ws;  // sample index < 2^31
        const int r = (int)q * stride, c = (int)(su - q * (unsigned)ws) * stride;
        return depth[(int64_t)r * w + c] > 0.0f;
    }
};
struct UnprojEmit {
    const float* depth;
    const uint8_t* color;
    int w, ws, stride;
    double fx, fy, cx, cy;
    Mat4d pose;
    double* xyz;
    double* rgb;
    __device__ void operator()(int64_t s, int64_t pos) const {
        const unsigned su = (unsigned)s, q = su / (unsigned)ws;
        const int r = (int)q * stride, c = (int)(su - q * (unsigned)ws) * stride;
        const int64_t pix = (int64_t)r * w + c;
        const double z = (double)depth[pix];
        unsigned c0 = 0, c1 = 0, c2 = 0;  // colour loaded before the stores (byte data may alias them)
        if (color) {
            const uint8_t* p = color + pix * 3;
            c0 = p[0], c1 = p[1], c2 = p[2];
        }
        const double x = ((double)c - cx) * z / fx;
        const double y = ((double)r - cy) * z / fy;
        const double* m = pose.m;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double a = m[k * 4 + 0] * x;
            const double b = m[k * 4 + 1] * y;
            const double cc = m[k * 4 + 2] * z;
            xyz[pos * 3 + k] = ((a + b) + cc) + m[k * 4 + 3];
        }
        if (color) {
            rgb[pos * 3 + 0] = (double)c0 / 255.0;
            rgb[pos * 3 + 1] = (double)c1 / 255.0;
            rgb[pos * 3 + 2] = (double)c2 / 255.0;
        }
    }
};

struct MinZPred {
    const double* xyz;
    double zmin;
    __device__ bool operator()(int64_t i) const { return xyz[i * 3 + 2] >= zmin; }
};
struct CopyRowsEmit {
    const double* xyz;
    const double* rgb;
    double* oxyz;
    double* orgb;
    __device__ void operator()(int64_t i, int64_t pos) const {
#pragma unroll
        for (int d = 0; d < 3; ++d) oxyz[pos * 3 + d] = xyz[i * 3 + d];
        if (rgb) {
#pragma unroll
            for (int d = 0; d < 3; ++d) orgb[pos * 3 + d] = rgb[i * 3 + d];
        }
    }
};

struct OccPred {
    const uint8_t* img;
    int thr;
    __device__ bool operator()(int64_t i) const { return (int)img[i] < thr; }
};
struct OccEmit {
    int w, h;
    double res, ox, oy;
    double* out;
    __device__ void operator()(int64_t i, int64_t pos) const {
        const unsigned iu = (unsigned)i, q = iu / (unsigned)w;  // h * w < 2^31 (checked on the host)
        const int r = (int)q, c = (int)(iu - q * (unsigned)w);
        out[pos * 3 + 0] = ox + ((double)c * res);
        out[pos * 3 + 1] = oy + ((double)(h - 1 - r) * res);
        out[pos * 3 + 2] = 0.0;
    }
};

__global__ __launch_bounds__(256) void k_gather_rows3(const double* __restrict__ in, const int64_t* __restrict__ idx,
                                                      int64_t m, double* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= m * 3) return;
    const int64_t k = t / 3, d = t % 3;
    out[t] = in[idx[k] * 3 + d];
}

}  // namespace ot

using namespace ot;

extern "C" {

ot_status ot_depth_to_float(const uint16_t* depth_u16, float* depth_f32, int64_t n_pixels, double depth_scale,
                            double depth_trunc, void* stream) {
    if (n_pixels < 0 || (n_pixels > 0 && (!depth_u16 || !depth_f32)))
        return fail(OT_ERR_INVALID_ARGUMENT, "[ConvertDepthToFloatImage] invalid buffers");
    if (n_pixels == 0) return OT_OK;
    const int64_t threads = (n_pixels + 7) / 8;
    hipLaunchKernelGGL(k_depth_to_float, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, S(stream), depth_u16,
                       depth_f32, n_pixels, (float)depth_scale, depth_trunc);
    OT_LAUNCH_CHECK();
    return OT_OK;
}

ot_status ot_depth_multiplier(const ot_intrinsics* in, float* out, void* stream) {
    if (!in || !out || in->width <= 0 || in->height <= 0)
        return fail(OT_ERR_INVALID_ARGUMENT, "[CreateDepthToCameraDistanceMultiplierFloatImage] invalid intrinsic");
    const int64_t n = (int64_t)in->width * in->height;
    const float inv_fx = 1.0f / (float)in->fx, inv_fy = 1.0f / (float)in->fy;
    hipLaunchKernelGGL(k_depth_multiplier, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, S(stream), in->width,
                       in->height, inv_fx, inv_fy, (float)in->cx, (float)in->cy, out);
    OT_LAUNCH_CHECK();
    return OT_OK;
}

ot_status ot_unproject(const float* depth, const uint8_t* color, const ot_intrinsics* in, const double extrinsic[16],
                       int32_t stride, double* out_xyz, double* out_rgb, int64_t capacity, int64_t* n_points_host,
                       void* stream) {
    if (!depth || !in || !extrinsic || !out_xyz || !n_points_host || stride < 1 || in->width <= 0 || in->height <= 0)
        return fail(OT_ERR_INVALID_ARGUMENT, "[CreatePointCloudFromRGBDImage] invalid arguments");
    if (color && !out_rgb) return fail(OT_ERR_INVALID_ARGUMENT, "[CreatePointCloudFromRGBDImage] out_rgb is NULL");
    const int ws = (in->width + stride - 1) / stride, hs = (in->height + stride - 1) / stride;
    const int64_t n = (int64_t)ws * hs;
    if (capacity < n) return fail(OT_ERR_CAPACITY, "[CreatePointCloudFromRGBDImage] output capacity too small");
    if (n > 0x7FFFFFFF) return fail(OT_ERR_INVALID_ARGUMENT, "[CreatePointCloudFromRGBDImage] image too large");
    UnprojPred pred{depth, in->width, ws, stride};
    UnprojEmit emit;
    emit.depth = depth;
    emit.color = color;
    emit.w = in->width;
    emit.ws = ws;
    emit.stride = stride;
    emit.fx = in->fx;
    emit.fy = in->fy;
    emit.cx = in->cx;
    emit.cy = in->cy;
    inverse4(extrinsic, emit.pose.m);
    emit.xyz = out_xyz;
    emit.rgb = out_rgb;
    return compact(n, pred, emit, S(stream), n_points_host, 0);
}

ot_status ot_filter_min_z(const double* xyz, const double* rgb, int64_t n, double z_min, double* out_xyz,
                          double* out_rgb, int64_t* n_out_host, void* stream) {
    if (n < 0 || !n_out_host || (n > 0 && (!xyz || !out_xyz)) || (rgb && !out_rgb))
        return fail(OT_ERR_INVALID_ARGUMENT, "[filter_min_z] invalid arguments");
    MinZPred pred{xyz, z_min};
    CopyRowsEmit emit{xyz, rgb, out_xyz, out_rgb};
    return compact(n, pred, emit, S(stream), n_out_host, 1);
}

ot_status ot_gather_rows3(const double* in, const int64_t* idx, int64_t m, double* out, void* stream) {
    if (m < 0 || (m > 0 && (!in || !idx || !out))) return fail(OT_ERR_INVALID_ARGUMENT, "[SelectByIndex] invalid");
    if (m == 0) return OT_OK;
    hipLaunchKernelGGL(k_gather_rows3, dim3((unsigned)((m * 3 + 255) / 256)), dim3(256), 0, S(stream), in, idx, m, out);
    OT_LAUNCH_CHECK();
    return OT_OK;
}

ot_status ot_occupancy_to_points(const uint8_t* img, int32_t height, int32_t width, int32_t threshold,
                                 double resolution, double origin_x, double origin_y, double* out_xyz,
                                 int64_t* n_out_host, void* stream) {
    if (!img || !out_xyz || !n_out_host || height <= 0 || width <= 0 || (int64_t)height * width > 0x7FFFFFFF)
        return fail(OT_ERR_INVALID_ARGUMENT, "[create_map_cloud] invalid arguments");
    OccPred pred{img, threshold};
    OccEmit emit{width, height, resolution, origin_x, origin_y, out_xyz};
    return compact((int64_t)width * height, pred, emit, S(stream), n_out_host, 2);
}

}  // extern "C"
