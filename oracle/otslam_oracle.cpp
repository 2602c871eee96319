/*
 * otslam_oracle.cpp — CPU ORACLE (test infrastructure only; never linked or called by the product path).
 *
 * A strict-IEEE C++ restatement of the Open3D algorithms that the reference scripts call on the hot path
 * (SURVEY.md §8(a), Appendix A).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / the timed CPU baseline.
 *
 * PARITY STATUS: "parity unpinned" against Open3D.  The arithmetic of the reference path lives in Open3D,
 * which is not vendored in /root/reference, not version-pinned (no requirements/setup/pyproject) and not
 * installed in this image (import open3d -> ModuleNotFoundError; no network).  The reference has no tests or
 * fixtures.  This file therefore follows the Open3D upstream C++ semantics as restated in
 * SURVEY.md Appendix A (Open3D ~0.13-0.19, structurally stable), with operation order written out and no
 * contraction (built with -ffp-contract=off, no -ffast-math).  What pins it: analytic known-answer tests,
 * the caller-sequence fixture captured by importing the reference scripts (tests/golden/), and MC-table
 * watertightness tests.
 *
 * Build: oracle/Makefile -> oracle/libotslam_oracle.so (g++ -O2 -ffp-contract=off -fopenmp).
 * OpenMP is placed where Open3D places it (TSDF: parallel over x inside each unit, units serial;
 * SOR/ROR: over points; unproject and voxel downsample serial), so the CPU baseline times the same shape of
 * parallelism as the reference path.
 */
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <map>
#include <numeric>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../include/otslam_mc_tables.h"

namespace {

struct Key3 {
    int x, y, z;
    bool operator==(const Key3& o) const { return x == o.x && y == o.y && z == o.z; }
    bool operator<(const Key3& o) const {
        if (x != o.x) return x < o.x;
        if (y != o.y) return y < o.y;
        return z < o.z;
    }
};
struct Key3Hash {
    size_t operator()(const Key3& k) const {
        // utility::hash_eigen-like combine (order of iteration is irrelevant: outputs are sorted)
        size_t h = 0;
        h ^= std::hash<int>()(k.x) + 0x9e3779b9 + (h << 6) + (h >> 2);
        h ^= std::hash<int>()(k.y) + 0x9e3779b9 + (h << 6) + (h >> 2);
        h ^= std::hash<int>()(k.z) + 0x9e3779b9 + (h << 6) + (h >> 2);
        return h;
    }
};

/* Eigen generic 4x4 inverse (Eigen/src/LU/InverseImpl.h, compute_inverse_size4 + cofactor_4x4). */
inline double det3_helper(const double* m, int i1, int i2, int i3, int j1, int j2, int j3) {
    return m[i1 * 4 + j1] * (m[i2 * 4 + j2] * m[i3 * 4 + j3] - m[i2 * 4 + j3] * m[i3 * 4 + j2]);
}
inline double cofactor4(const double* m, int i, int j) {
    int i1 = (i + 1) % 4, i2 = (i + 2) % 4, i3 = (i + 3) % 4;
    int j1 = (j + 1) % 4, j2 = (j + 2) % 4, j3 = (j + 3) % 4;
    return (det3_helper(m, i1, i2, i3, j1, j2, j3) + det3_helper(m, i2, i3, i1, j1, j2, j3)) +
           det3_helper(m, i3, i1, i2, j1, j2, j3);
}
void inverse4(const double* m, double* r) {
    for (int row = 0; row < 4; ++row)
        for (int col = 0; col < 4; ++col) {
            double c = cofactor4(m, col, row);
            r[row * 4 + col] = ((row + col) & 1) ? -c : c;
        }
    // det = sum_k m(k,0) * r(0,k), unrolled pairwise ((a0+a1)+(a2+a3))
    double p0 = m[0 * 4 + 0] * r[0 * 4 + 0], p1 = m[1 * 4 + 0] * r[0 * 4 + 1];
    double p2 = m[2 * 4 + 0] * r[0 * 4 + 2], p3 = m[3 * 4 + 0] * r[0 * 4 + 3];
    double det = (p0 + p1) + (p2 + p3);
    for (int k = 0; k < 16; ++k) r[k] = r[k] / det;
}

/* camera_pose * (x, y, z, 1): ((m0*x + m1*y) + m2*z) + m3, per row (Appendix A.2). */
inline void transform_point(const double* T, double x, double y, double z, double* out) {
    for (int r = 0; r < 3; ++r) {
        double a = T[r * 4 + 0] * x;
        double b = T[r * 4 + 1] * y;
        double c = T[r * 4 + 2] * z;
        out[r] = ((a + b) + c) + T[r * 4 + 3];
    }
}

struct Intr {
    int w, h;
    double fx, fy, cx, cy;
};

/* Sensitivity probe (tools/parity_sensitivity.py): Eigen may compute camera_pose = extrinsic.inverse()
 * with its vectorised 4x4 path, whose last bits can differ from the scalar cofactor restatement above.  Mode 1 / 2
 * moves every entry of rows 0..2 of the pose by one ulp (direction by a fixed pattern / its opposite) to measure how
 * many unit-touch decisions such a difference moves.  Mode 0 (the default) leaves the pose as computed. */
static int g_pose_ulp_mode = 0;
void perturb_pose(double* pose) {
    if (!g_pose_ulp_mode) return;
    for (int k = 0; k < 12; ++k) {
        const bool up = (((k * 7 + 3) >> 1) & 1) ^ (g_pose_ulp_mode == 2);
        pose[k] = std::nextafter(pose[k], up ? INFINITY : -INFINITY);
    }
}

/* CreatePointCloudFromFloatDepthImage (Appendix A.2 / A.3(ii)). */
int64_t unproject_impl(const float* depth, const uint8_t* color, const Intr& in, const double* extrinsic,
                       int stride, double* xyz, double* rgb) {
    double pose[16];
    inverse4(extrinsic, pose);
    perturb_pose(pose);
    int64_t cnt = 0;
    for (int i = 0; i < in.h; i += stride) {
        for (int j = 0; j < in.w; j += stride) {
            float d = depth[(int64_t)i * in.w + j];
            if (d > 0) {
                double z = (double)d;
                double x = ((double)j - in.cx) * z / in.fx;
                double y = ((double)i - in.cy) * z / in.fy;
                double p[3];
                transform_point(pose, x, y, z, p);
                xyz[cnt * 3 + 0] = p[0];
                xyz[cnt * 3 + 1] = p[1];
                xyz[cnt * 3 + 2] = p[2];
                if (color && rgb) {
                    const uint8_t* c = color + ((int64_t)i * in.w + j) * 3;
                    rgb[cnt * 3 + 0] = c[0] / 255.0;
                    rgb[cnt * 3 + 1] = c[1] / 255.0;
                    rgb[cnt * 3 + 2] = c[2] / 255.0;
                }
                ++cnt;
            }
        }
    }
    return cnt;
}

/* ------------------------------------------------------------------------------------------------ TSDF */
constexpr int RES = 16;
constexpr int NVOX = RES * RES * RES;

struct Unit {
    std::vector<float> tsdf, weight;
    std::vector<double> color;  // Open3D TSDFVoxel::color_ is Eigen::Vector3d
    Unit() : tsdf(NVOX, 0.f), weight(NVOX, 0.f), color(NVOX * 3, 0.0) {}
};

struct Tsdf {
    double voxel_length, sdf_trunc, unit_length;
    int color_type, stride;
    std::unordered_map<Key3, Unit, Key3Hash> units;
    int64_t last_updates = 0, total_updates = 0, unit_integrations = 0;
    // extracted mesh
    std::vector<double> V, VC;
    std::vector<int32_t> T;
};

/* UniformTSDFVolume::IntegrateWithDepthToCameraDistanceMultiplier (Appendix A.3(iv)). */
int64_t integrate_unit(Tsdf& vol, const Key3& key, Unit& u, const float* depth, const uint8_t* color,
                       const Intr& in, const double* extrinsic, const float* mult) {
    const float fx = (float)in.fx, fy = (float)in.fy, cx = (float)in.cx, cy = (float)in.cy;
    float E[16];
    for (int k = 0; k < 16; ++k) E[k] = (float)extrinsic[k];
    const double unit_voxel_length = vol.unit_length / (double)RES;  // UniformTSDFVolume: length / resolution
    const float vl = (float)unit_voxel_length;
    const float half = vl * 0.5f;
    const float trunc = (float)vol.sdf_trunc;
    const float trunc_inv = 1.0f / trunc;
    float Es[16];
    for (int k = 0; k < 16; ++k) Es[k] = E[k] * vl;
    const float safe_w = (float)in.w - 0.0001f;
    const float safe_h = (float)in.h - 0.0001f;
    const float ox = (float)((double)key.x * vol.unit_length);
    const float oy = (float)((double)key.y * vol.unit_length);
    const float oz = (float)((double)key.z * vol.unit_length);
    int64_t updates = 0;
#pragma omp parallel for schedule(static) reduction(+ : updates)
    for (int x = 0; x < RES; ++x) {
        for (int y = 0; y < RES; ++y) {
            const float px = (half + vl * (float)x) + ox;
            const float py = (half + vl * (float)y) + oy;
            const float pz = half + oz;
            float pc[3];
            for (int r = 0; r < 3; ++r) {
                float a = E[r * 4 + 0] * px;
                float b = E[r * 4 + 1] * py;
                float c = E[r * 4 + 2] * pz;
                pc[r] = ((a + b) + c) + E[r * 4 + 3];
            }
            for (int z = 0; z < RES; ++z) {
                if (pc[2] > 0) {
                    float u_f = ((pc[0] * fx) / pc[2] + cx) + 0.5f;
                    float v_f = ((pc[1] * fy) / pc[2] + cy) + 0.5f;
                    if (u_f >= 0.0001f && u_f < safe_w && v_f >= 0.0001f && v_f < safe_h) {
                        int uu = (int)u_f, vv = (int)v_f;
                        float d = depth[(int64_t)vv * in.w + uu];
                        if (d > 0.0f) {
                            float sdf = (d - pc[2]) * mult[(int64_t)vv * in.w + uu];
                            if (sdf > -trunc) {
                                float s = sdf * trunc_inv;
                                float t = (s < 1.0f) ? s : 1.0f;  // std::min(1.0f, s)
                                int idx = x * RES * RES + y * RES + z;
                                float w = u.weight[idx];
                                u.tsdf[idx] = (u.tsdf[idx] * w + t) / (w + 1.0f);
                                if (vol.color_type == 1 && color) {
                                    const uint8_t* c = color + ((int64_t)vv * in.w + uu) * 3;
                                    double wd = (double)w, w1 = (double)(w + 1.0f);
                                    for (int ch = 0; ch < 3; ++ch)
                                        u.color[idx * 3 + ch] = (u.color[idx * 3 + ch] * wd + (double)c[ch]) / w1;
                                }
                                u.weight[idx] = w + 1.0f;
                                ++updates;
                            }
                        }
                    }
                }
                pc[0] += Es[0 * 4 + 2];
                pc[1] += Es[1 * 4 + 2];
                pc[2] += Es[2 * 4 + 2];
            }
        }
    }
    return updates;
}

inline int locate(double v, double unit_length) { return (int)std::floor(v / unit_length); }

}  // namespace

extern "C" {

const char* oro_name(void) { return "otslam CPU oracle (restatement of Open3D semantics; parity unpinned)"; }

void oro_inverse4(const double* m, double* out) { inverse4(m, out); }
void oro_set_pose_ulp_mode(int mode) { g_pose_ulp_mode = mode; }

/* Image::ConvertDepthToFloatImage (Appendix A.1). */
void oro_depth_to_float(const uint16_t* in, float* out, int64_t n, double depth_scale, double depth_trunc) {
    const float scale = (float)depth_scale;
    for (int64_t i = 0; i < n; ++i) {
        float f = (float)in[i];
        f = f / scale;
        if (f >= depth_trunc) f = 0.0f;  // float promoted to double for the compare, as in Open3D
        out[i] = f;
    }
}

/* Image::CreateDepthToCameraDistanceMultiplierFloatImage (Appendix A.3(i)). */
void oro_depth_multiplier(int w, int h, double fx, double fy, double cx, double cy, float* out) {
    const float inv_fx = 1.0f / (float)fx, inv_fy = 1.0f / (float)fy;
    const float fcx = (float)cx, fcy = (float)cy;
    std::vector<float> xx(w), yy(h);
    for (int j = 0; j < w; ++j) xx[j] = ((float)j - fcx) * inv_fx;
    for (int i = 0; i < h; ++i) yy[i] = ((float)i - fcy) * inv_fy;
    for (int i = 0; i < h; ++i)
        for (int j = 0; j < w; ++j) {
            float a = xx[j] * xx[j];
            float b = yy[i] * yy[i];
            out[(int64_t)i * w + j] = std::sqrt((a + b) + 1.0f);
        }
}

int64_t oro_unproject(const float* depth, const uint8_t* color, int w, int h, double fx, double fy, double cx,
                      double cy, const double* extrinsic, int stride, double* xyz, double* rgb) {
    Intr in{w, h, fx, fy, cx, cy};
    return unproject_impl(depth, color, in, extrinsic, stride, xyz, rgb);
}

/* PointCloud::VoxelDownSample (Appendix A.6).  Output sorted by key; returns K, or -1 on error. */
int64_t oro_voxel_down_sample(const double* xyz, const double* rgb, const double* nrm, int64_t n, double vs,
                              double* out_xyz, double* out_rgb, double* out_nrm, int32_t* out_keys) {
    if (vs <= 0.0) return -1;
    if (n == 0) return 0;
    double mn[3] = {xyz[0], xyz[1], xyz[2]}, mx[3] = {xyz[0], xyz[1], xyz[2]};
    for (int64_t i = 1; i < n; ++i)
        for (int a = 0; a < 3; ++a) {
            mn[a] = std::min(mn[a], xyz[i * 3 + a]);
            mx[a] = std::max(mx[a], xyz[i * 3 + a]);
        }
    double vmin[3], vmax[3];
    for (int a = 0; a < 3; ++a) {
        vmin[a] = mn[a] - vs * 0.5;
        vmax[a] = mx[a] + vs * 0.5;
    }
    double ext = std::max(std::max(vmax[0] - vmin[0], vmax[1] - vmin[1]), vmax[2] - vmin[2]);
    if (vs * (double)INT32_MAX < ext) return -2;
    struct Acc {
        double p[3] = {0, 0, 0}, c[3] = {0, 0, 0}, nn[3] = {0, 0, 0};
        int64_t cnt = 0;
    };
    std::map<Key3, Acc> acc;  // ordered -> emits sorted by key
    for (int64_t i = 0; i < n; ++i) {
        Key3 k;
        k.x = (int)std::floor((xyz[i * 3 + 0] - vmin[0]) / vs);
        k.y = (int)std::floor((xyz[i * 3 + 1] - vmin[1]) / vs);
        k.z = (int)std::floor((xyz[i * 3 + 2] - vmin[2]) / vs);
        Acc& a = acc[k];
        for (int d = 0; d < 3; ++d) {
            a.p[d] += xyz[i * 3 + d];
            if (rgb) a.c[d] += rgb[i * 3 + d];
            if (nrm) a.nn[d] += nrm[i * 3 + d];
        }
        a.cnt++;
    }
    int64_t k = 0;
    for (auto& kv : acc) {
        double c = (double)kv.second.cnt;
        for (int d = 0; d < 3; ++d) {
            out_xyz[k * 3 + d] = kv.second.p[d] / c;
            if (rgb && out_rgb) out_rgb[k * 3 + d] = kv.second.c[d] / c;
            if (nrm && out_nrm) out_nrm[k * 3 + d] = kv.second.nn[d] / c;
        }
        if (out_keys) {
            out_keys[k * 3 + 0] = kv.first.x;
            out_keys[k * 3 + 1] = kv.first.y;
            out_keys[k * 3 + 2] = kv.first.z;
        }
        ++k;
    }
    return k;
}

/* ---------------------------------------------------------------- ScalableTSDFVolume (Appendix A.3-A.4) */
void* oro_tsdf_create(double voxel_length, double sdf_trunc, int color_type, int stride) {
    Tsdf* t = new Tsdf();
    t->voxel_length = voxel_length;
    t->sdf_trunc = sdf_trunc;
    t->unit_length = voxel_length * RES;
    t->color_type = color_type;
    t->stride = stride;
    return t;
}
void oro_tsdf_destroy(void* h) { delete (Tsdf*)h; }

/* ScalableTSDFVolume::Integrate: returns the voxel updates of this frame. */
int64_t oro_tsdf_integrate(void* h, const float* depth, const uint8_t* color, int w, int hgt, double fx,
                           double fy, double cx, double cy, const double* extrinsic) {
    Tsdf& vol = *(Tsdf*)h;
    Intr in{w, hgt, fx, fy, cx, cy};
    std::vector<float> mult((size_t)w * hgt);
    oro_depth_multiplier(w, hgt, fx, fy, cx, cy, mult.data());
    const int64_t cap = (int64_t)((hgt + vol.stride - 1) / vol.stride) * ((w + vol.stride - 1) / vol.stride);
    std::vector<double> pts((size_t)cap * 3);
    int64_t np = unproject_impl(depth, nullptr, in, extrinsic, vol.stride, pts.data(), nullptr);
    std::unordered_set<Key3, Key3Hash> touched;
    int64_t updates = 0;
    const double tr = vol.sdf_trunc;
    for (int64_t p = 0; p < np; ++p) {
        const double* q = &pts[p * 3];
        int lo[3], hi[3];
        for (int a = 0; a < 3; ++a) {
            lo[a] = locate(q[a] - tr, vol.unit_length);
            hi[a] = locate(q[a] + tr, vol.unit_length);
        }
        for (int x = lo[0]; x <= hi[0]; ++x)
            for (int y = lo[1]; y <= hi[1]; ++y)
                for (int z = lo[2]; z <= hi[2]; ++z) {
                    Key3 k{x, y, z};
                    if (touched.find(k) == touched.end()) {
                        touched.insert(k);
                        Unit& u = vol.units[k];
                        updates += integrate_unit(vol, k, u, depth, color, in, extrinsic, mult.data());
                        vol.unit_integrations++;
                    }
                }
    }
    vol.last_updates = updates;
    vol.total_updates += updates;
    return updates;
}

int64_t oro_tsdf_num_units(void* h) { return (int64_t)((Tsdf*)h)->units.size(); }
int64_t oro_tsdf_total_updates(void* h) { return ((Tsdf*)h)->total_updates; }
int64_t oro_tsdf_unit_integrations(void* h) { return ((Tsdf*)h)->unit_integrations; }

/* Units sorted by key; voxels in IndexOf order; color as double (0..255). */
void oro_tsdf_export(void* h, int32_t* keys, float* tsdf, float* weight, double* color) {
    Tsdf& vol = *(Tsdf*)h;
    std::vector<Key3> ks;
    ks.reserve(vol.units.size());
    for (auto& kv : vol.units) ks.push_back(kv.first);
    std::sort(ks.begin(), ks.end());
    for (size_t i = 0; i < ks.size(); ++i) {
        const Unit& u = vol.units.at(ks[i]);
        if (keys) {
            keys[i * 3 + 0] = ks[i].x;
            keys[i * 3 + 1] = ks[i].y;
            keys[i * 3 + 2] = ks[i].z;
        }
        if (tsdf) std::memcpy(tsdf + i * NVOX, u.tsdf.data(), sizeof(float) * NVOX);
        if (weight) std::memcpy(weight + i * NVOX, u.weight.data(), sizeof(float) * NVOX);
        if (color) std::memcpy(color + i * NVOX * 3, u.color.data(), sizeof(double) * NVOX * 3);
    }
}

/* ScalableTSDFVolume::ExtractTriangleMesh (Appendix A.4), units visited in sorted key order.  Vertices are
 * then renumbered canonically: sorted by (owner unit key, local voxel IndexOf, axis) of their edge key. */
void oro_tsdf_extract_mesh(void* h, int64_t* nv, int64_t* nt) {
    Tsdf& vol = *(Tsdf*)h;
    const double vl = vol.voxel_length;
    const double half = vl * 0.5;
    std::vector<Key3> ks;
    for (auto& kv : vol.units) ks.push_back(kv.first);
    std::sort(ks.begin(), ks.end());
    struct EKey {
        int x, y, z, a;
        bool operator==(const EKey& o) const { return x == o.x && y == o.y && z == o.z && a == o.a; }
    };
    struct EKeyHash {
        size_t operator()(const EKey& k) const {
            return Key3Hash()(Key3{k.x, k.y, k.z}) * 31 + (size_t)k.a;
        }
    };
    std::unordered_map<EKey, int, EKeyHash> e2v;
    std::vector<EKey> vkeys;
    std::vector<double> V, VC;
    std::vector<int32_t> T;
    for (const Key3& k0 : ks) {
        const Unit& u0 = vol.units.at(k0);
        for (int x = 0; x < RES; ++x)
            for (int y = 0; y < RES; ++y)
                for (int z = 0; z < RES; ++z) {
                    int cube = 0;
                    float w[8], f[8];
                    double c[8][3];
                    for (int i = 0; i < 8; ++i) {
                        int ix = x + OT_MC_SHIFT[i][0], iy = y + OT_MC_SHIFT[i][1], iz = z + OT_MC_SHIFT[i][2];
                        Key3 k1 = k0;
                        const Unit* u1 = &u0;
                        if (ix >= RES || iy >= RES || iz >= RES) {
                            if (ix >= RES) { ix -= RES; k1.x += 1; }
                            if (iy >= RES) { iy -= RES; k1.y += 1; }
                            if (iz >= RES) { iz -= RES; k1.z += 1; }
                            auto it = vol.units.find(k1);
                            u1 = (it == vol.units.end()) ? nullptr : &it->second;
                        }
                        if (u1) {
                            int idx = ix * RES * RES + iy * RES + iz;
                            w[i] = u1->weight[idx];
                            f[i] = u1->tsdf[idx];
                            for (int ch = 0; ch < 3; ++ch) c[i][ch] = u1->color[idx * 3 + ch] / 255.0;
                        } else {
                            w[i] = 0.0f;
                            f[i] = 0.0f;
                        }
                        if (w[i] == 0.0f) {
                            cube = 0;
                            break;
                        } else if (f[i] < 0.0f) {
                            cube |= (1 << i);
                        }
                    }
                    if (cube == 0 || cube == 255) continue;
                    int eidx[12];
                    const signed char* tri = OT_MC_TRI_TABLE[cube];
                    for (int e = 0; e < 12; ++e) {
                        int v0 = OT_MC_EDGE_TO_VERT[e][0], v1 = OT_MC_EDGE_TO_VERT[e][1];
                        bool cut = (((cube >> v0) & 1) != ((cube >> v1) & 1));
                        if (!cut) continue;
                        EKey ek{k0.x * RES + x + OT_MC_EDGE_SHIFT[e][0], k0.y * RES + y + OT_MC_EDGE_SHIFT[e][1],
                                k0.z * RES + z + OT_MC_EDGE_SHIFT[e][2], OT_MC_EDGE_SHIFT[e][3]};
                        auto it = e2v.find(ek);
                        if (it == e2v.end()) {
                            int id = (int)vkeys.size();
                            e2v[ek] = id;
                            vkeys.push_back(ek);
                            double pt[3] = {half + vl * (double)ek.x, half + vl * (double)ek.y,
                                            half + vl * (double)ek.z};
                            double f0 = std::fabs((double)f[v0]);
                            double f1 = std::fabs((double)f[v1]);
                            pt[ek.a] += f0 * vl / (f0 + f1);
                            for (int d = 0; d < 3; ++d) V.push_back(pt[d]);
                            for (int ch = 0; ch < 3; ++ch) VC.push_back((f1 * c[v0][ch] + f0 * c[v1][ch]) / (f0 + f1));
                            eidx[e] = id;
                        } else {
                            eidx[e] = it->second;
                        }
                    }
                    for (int t = 0; tri[t] != -1; t += 3) {
                        T.push_back(eidx[tri[t]]);
                        T.push_back(eidx[tri[t + 2]]);
                        T.push_back(eidx[tri[t + 1]]);
                    }
                }
    }
    // canonical renumbering of vertices
    auto floordiv = [](int a) { return (a >= 0) ? a / RES : -((-a + RES - 1) / RES); };
    auto canon_less = [&](const EKey& a, const EKey& b) {
        Key3 ua{floordiv(a.x), floordiv(a.y), floordiv(a.z)}, ub{floordiv(b.x), floordiv(b.y), floordiv(b.z)};
        if (!(ua == ub)) return ua < ub;
        int la = ((a.x - ua.x * RES) * RES + (a.y - ua.y * RES)) * RES + (a.z - ua.z * RES);
        int lb = ((b.x - ub.x * RES) * RES + (b.y - ub.y * RES)) * RES + (b.z - ub.z * RES);
        if (la != lb) return la < lb;
        return a.a < b.a;
    };
    std::vector<int> order(vkeys.size());
    std::iota(order.begin(), order.end(), 0);
    std::sort(order.begin(), order.end(), [&](int i, int j) { return canon_less(vkeys[i], vkeys[j]); });
    std::vector<int> newid(vkeys.size());
    for (size_t r = 0; r < order.size(); ++r) newid[order[r]] = (int)r;
    vol.V.assign(V.size(), 0.0);
    vol.VC.assign(VC.size(), 0.0);
    for (size_t i = 0; i < vkeys.size(); ++i)
        for (int d = 0; d < 3; ++d) {
            vol.V[newid[i] * 3 + d] = V[i * 3 + d];
            vol.VC[newid[i] * 3 + d] = VC[i * 3 + d];
        }
    vol.T.resize(T.size());
    for (size_t i = 0; i < T.size(); ++i) vol.T[i] = newid[T[i]];
    *nv = (int64_t)vkeys.size();
    *nt = (int64_t)(T.size() / 3);
}

void oro_tsdf_fetch_mesh(void* h, double* V, double* VC, int32_t* T) {
    Tsdf& vol = *(Tsdf*)h;
    if (V) std::memcpy(V, vol.V.data(), sizeof(double) * vol.V.size());
    if (VC) std::memcpy(VC, vol.VC.data(), sizeof(double) * vol.VC.size());
    if (T) std::memcpy(T, vol.T.data(), sizeof(int32_t) * vol.T.size());
}

/* TriangleMesh::ComputeVertexNormals (Appendix A.5). */
void oro_mesh_vertex_normals(const double* V, int64_t nv, const int32_t* T, int64_t nt, double* N) {
    std::fill(N, N + nv * 3, 0.0);
    for (int64_t t = 0; t < nt; ++t) {
        const int32_t a = T[t * 3], b = T[t * 3 + 1], c = T[t * 3 + 2];
        double e1[3], e2[3], n[3];
        for (int d = 0; d < 3; ++d) {
            e1[d] = V[b * 3 + d] - V[a * 3 + d];
            e2[d] = V[c * 3 + d] - V[a * 3 + d];
        }
        n[0] = e1[1] * e2[2] - e1[2] * e2[1];
        n[1] = e1[2] * e2[0] - e1[0] * e2[2];
        n[2] = e1[0] * e2[1] - e1[1] * e2[0];
        for (int d = 0; d < 3; ++d) {
            N[a * 3 + d] += n[d];
            N[b * 3 + d] += n[d];
            N[c * 3 + d] += n[d];
        }
    }
    for (int64_t i = 0; i < nv; ++i) {
        double* n = N + i * 3;
        double sq = (n[0] * n[0] + n[1] * n[1]) + n[2] * n[2];
        if (sq > 0.0) {
            double s = std::sqrt(sq);
            n[0] /= s;
            n[1] /= s;
            n[2] /= s;
        }
        if (std::isnan(n[0])) {
            n[0] = 0.0;
            n[1] = 0.0;
            n[2] = 1.0;
        }
    }
}

/* Counter-based RNG shared (as a definition) with the HIP sampler: splitmix64 of seed + (ctr+1)*golden. */
static inline double u01(uint64_t seed, uint64_t ctr) {
    uint64_t z = seed + (ctr + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

/* TriangleMesh::GetSurfaceArea (Open3D TriangleMesh.cpp; called by SamplePointsUniformly, Appendix A.8): the
 * triangle areas 0.5 |(p0 - p1) x (p0 - p2)| summed in index order. */
double oro_mesh_surface_area(const double* V, const int32_t* T, int64_t nt) {
    double surface = 0.0;
    for (int64_t t = 0; t < nt; ++t) {
        const double *p0 = V + T[t * 3] * 3, *p1 = V + T[t * 3 + 1] * 3, *p2 = V + T[t * 3 + 2] * 3;
        double x[3], y[3], c[3];
        for (int d = 0; d < 3; ++d) {
            x[d] = p0[d] - p1[d];
            y[d] = p0[d] - p2[d];
        }
        c[0] = x[1] * y[2] - x[2] * y[1];
        c[1] = x[2] * y[0] - x[0] * y[2];
        c[2] = x[0] * y[1] - x[1] * y[0];
        surface += 0.5 * std::sqrt((c[0] * c[0] + c[1] * c[1]) + c[2] * c[2]);
    }
    return surface;
}

/* TriangleMesh::SamplePointsUniformly (Appendix A.8) with the seeded RNG. */
int oro_mesh_sample_uniform(const double* V, const double* VN, const double* VC, int64_t nv, const int32_t* T,
                            int64_t nt, int64_t n_points, uint64_t seed, double* P, double* PN, double* PC) {
    (void)nv;
    if (n_points <= 0 || nt == 0) return -1;
    std::vector<double> area(nt);
    double surface = 0.0;
    for (int64_t t = 0; t < nt; ++t) {
        const double *p0 = V + T[t * 3] * 3, *p1 = V + T[t * 3 + 1] * 3, *p2 = V + T[t * 3 + 2] * 3;
        double x[3], y[3], c[3];
        for (int d = 0; d < 3; ++d) {
            x[d] = p0[d] - p1[d];
            y[d] = p0[d] - p2[d];
        }
        c[0] = x[1] * y[2] - x[2] * y[1];
        c[1] = x[2] * y[0] - x[0] * y[2];
        c[2] = x[0] * y[1] - x[1] * y[0];
        area[t] = 0.5 * std::sqrt((c[0] * c[0] + c[1] * c[1]) + c[2] * c[2]);
        surface += area[t];
    }
    area[0] /= surface;
    for (int64_t t = 1; t < nt; ++t) area[t] = area[t] / surface + area[t - 1];
    int64_t k = 0;
    for (int64_t t = 0; t < nt; ++t) {
        int64_t n = (int64_t)std::llround(area[t] * (double)n_points);
        while (k < n && k < n_points) {
            double r1 = u01(seed, (uint64_t)(2 * k)), r2 = u01(seed, (uint64_t)(2 * k + 1));
            double s1 = std::sqrt(r1);
            double a = 1.0 - s1, b = s1 * (1.0 - r2), c = s1 * r2;
            const int32_t i0 = T[t * 3], i1 = T[t * 3 + 1], i2 = T[t * 3 + 2];
            for (int d = 0; d < 3; ++d) {
                P[k * 3 + d] = (a * V[i0 * 3 + d] + b * V[i1 * 3 + d]) + c * V[i2 * 3 + d];
                if (VN && PN) PN[k * 3 + d] = (a * VN[i0 * 3 + d] + b * VN[i1 * 3 + d]) + c * VN[i2 * 3 + d];
                if (VC && PC) PC[k * 3 + d] = (a * VC[i0 * 3 + d] + b * VC[i1 * 3 + d]) + c * VC[i2 * 3 + d];
            }
            ++k;
        }
    }
    for (; k < n_points; ++k)  // rounding shortfall (Open3D leaves these zero-initialised)
        for (int d = 0; d < 3; ++d) {
            P[k * 3 + d] = 0.0;
            if (VN && PN) PN[k * 3 + d] = 0.0;
            if (VC && PC) PC[k * 3 + d] = 0.0;
        }
    return 0;
}

/* Z-mask stable compaction (reconstruct_rgbd_filter.py:126-132). */
int64_t oro_filter_min_z(const double* xyz, const double* rgb, int64_t n, double zmin, double* oxyz, double* orgb) {
    int64_t k = 0;
    for (int64_t i = 0; i < n; ++i)
        if (xyz[i * 3 + 2] >= zmin) {
            for (int d = 0; d < 3; ++d) {
                oxyz[k * 3 + d] = xyz[i * 3 + d];
                if (rgb && orgb) orgb[k * 3 + d] = rgb[i * 3 + d];
            }
            ++k;
        }
    return k;
}

/* ------------------------------------------------------------------ outlier removal (Appendix A.7) */
namespace {
struct Grid {
    double cell;
    double mn[3];
    std::unordered_map<Key3, std::vector<int64_t>, Key3Hash> cells;
    Key3 key_of(const double* p) const {
        return Key3{(int)std::floor((p[0] - mn[0]) / cell), (int)std::floor((p[1] - mn[1]) / cell),
                    (int)std::floor((p[2] - mn[2]) / cell)};
    }
};
inline double dist2(const double* a, const double* b) {
    double d0 = a[0] - b[0], d1 = a[1] - b[1], d2 = a[2] - b[2];
    return ((d0 * d0) + d1 * d1) + d2 * d2;  // nanoflann L2_Adaptor accumulation order
}
void build_grid(Grid& g, const double* xyz, int64_t n, double cell) {
    g.cell = cell;
    g.mn[0] = g.mn[1] = g.mn[2] = INFINITY;
    for (int64_t i = 0; i < n; ++i)
        for (int a = 0; a < 3; ++a) g.mn[a] = std::min(g.mn[a], xyz[i * 3 + a]);
    for (int64_t i = 0; i < n; ++i) g.cells[g.key_of(xyz + i * 3)].push_back(i);
}
}  // namespace

/* RemoveStatisticalOutliers; returns the kept count (indices ascending in out_idx), -1 on bad args. */
int64_t oro_remove_statistical_outlier(const double* xyz, int64_t n, int k, double std_ratio, int64_t* out_idx,
                                       double* out_avg) {
    if (k < 1 || std_ratio <= 0) return -1;
    if (n == 0) return 0;
    // exact kNN on a uniform grid with shell expansion; cell ~ mean spacing estimate
    double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = 0; i < n; ++i)
        for (int a = 0; a < 3; ++a) {
            mn[a] = std::min(mn[a], xyz[i * 3 + a]);
            mx[a] = std::max(mx[a], xyz[i * 3 + a]);
        }
    double vol = std::max((mx[0] - mn[0]) * (mx[1] - mn[1]) * (mx[2] - mn[2]), 1e-12);
    double cell = std::cbrt(vol * (double)k / (double)n);
    if (!(cell > 0) || !std::isfinite(cell)) cell = 1.0;
    Grid g;
    build_grid(g, xyz, n, cell);
    const int64_t kk = std::min<int64_t>(k, n);
    std::vector<double> avg(n);
    int64_t valid = 0;
#pragma omp parallel for schedule(static) reduction(+ : valid)
    for (int64_t i = 0; i < n; ++i) {
        const double* q = xyz + i * 3;
        Key3 c = g.key_of(q);
        std::vector<double> best;  // k smallest squared distances
        for (int r = 0;; ++r) {
            // visit shell r
            for (int dx = -r; dx <= r; ++dx)
                for (int dy = -r; dy <= r; ++dy)
                    for (int dz = -r; dz <= r; ++dz) {
                        if (std::max(std::max(std::abs(dx), std::abs(dy)), std::abs(dz)) != r) continue;
                        auto it = g.cells.find(Key3{c.x + dx, c.y + dy, c.z + dz});
                        if (it == g.cells.end()) continue;
                        for (int64_t j : it->second) best.push_back(dist2(q, xyz + j * 3));
                    }
            if ((int64_t)best.size() >= kk) {
                std::nth_element(best.begin(), best.begin() + (kk - 1), best.end());
                double kth = best[kk - 1];
                // every point within distance r*cell of q lies inside shells 0..r (margin for key rounding)
                double guard = std::max(0.0, (double)r - 0.01) * cell;
                if (kth <= guard * guard || (int64_t)best.size() == n) {
                    best.resize(kk);
                    break;
                }
                // keep all candidates; continue expanding
            }
            if (r > 1000000) break;
        }
        std::sort(best.begin(), best.end());
        double m = -1.0;
        if (!best.empty()) {
            double s = 0.0;
            for (double d : best) s += std::sqrt(d);
            m = s / (double)best.size();
            valid++;
        }
        avg[i] = m;
    }
    if (out_avg) std::memcpy(out_avg, avg.data(), sizeof(double) * n);
    if (valid == 0) return 0;
    double cloud_mean = 0.0;
    for (int64_t i = 0; i < n; ++i)
        if (avg[i] > 0) cloud_mean = cloud_mean + avg[i];
    cloud_mean /= (double)valid;
    double sq_sum = 0.0;
    for (int64_t i = 0; i < n; ++i) sq_sum = sq_sum + (avg[i] > 0 ? (avg[i] - cloud_mean) * (avg[i] - cloud_mean) : 0.0);
    double std_dev = std::sqrt(sq_sum / (double)(valid - 1));
    double thr = cloud_mean + std_ratio * std_dev;
    int64_t kept = 0;
    for (int64_t i = 0; i < n; ++i)
        if (avg[i] > 0 && avg[i] < thr) out_idx[kept++] = i;
    return kept;
}

/* RemoveRadiusOutliers; returns the kept count, -1 on bad args. */
int64_t oro_remove_radius_outlier(const double* xyz, int64_t n, int nb_points, double radius, int64_t* out_idx) {
    if (nb_points < 1 || radius <= 0) return -1;
    if (n == 0) return 0;
    Grid g;
    build_grid(g, xyz, n, radius);
    const double r2 = radius * radius;
    std::vector<char> mask(n, 0);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        const double* q = xyz + i * 3;
        Key3 c = g.key_of(q);
        int64_t cnt = 0;
        for (int dx = -1; dx <= 1; ++dx)
            for (int dy = -1; dy <= 1; ++dy)
                for (int dz = -1; dz <= 1; ++dz) {
                    auto it = g.cells.find(Key3{c.x + dx, c.y + dy, c.z + dz});
                    if (it == g.cells.end()) continue;
                    for (int64_t j : it->second)
                        if (dist2(q, xyz + j * 3) < r2) ++cnt;
                }
        mask[i] = cnt > nb_points;
    }
    int64_t kept = 0;
    for (int64_t i = 0; i < n; ++i)
        if (mask[i]) out_idx[kept++] = i;
    return kept;
}

/* PointCloud::ComputePointCloudDistance (eval_cone.py:99,103): per source point sqrt of the minimum squared
 * distance to the target (KDTreeFlann SearchKNN(1); nanoflann L2 order), 0.0 when the target is empty.
 * Exhaustive minimum (the search structure does not change the minimum); OpenMP over points as Open3D. */
void oro_point_cloud_distance(const double* src, int64_t n, const double* tgt, int64_t m, double* out) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        if (m == 0) {
            out[i] = 0.0;
            continue;
        }
        double best = INFINITY;
        for (int64_t j = 0; j < m; ++j) best = std::min(best, dist2(src + i * 3, tgt + j * 3));
        out[i] = std::sqrt(best);
    }
}

/* ChangeDetectorNode::scanCallback (diff_node.cpp:103-160) for a batch of scan pairs, written as the node does it
 * (float beam geometry with std::cos / std::sin / std::hypot on floats, double map transform from the
 * quaternion, C++ truncation to grid cells).  poses [n_scans][7] = tx ty tz qx qy qz qw. */
void oro_scan_diff(const float* real, const float* virt, int n_scans, int n_beams, float r_amin, float r_inc,
                   float r_max, float v_amin, float v_inc, double thresh, int window, const double* poses,
                   double grid_res, uint8_t* new_flag, uint8_t* gone_flag, int32_t* new_key, int32_t* gone_key) {
    for (int b = 0; b < n_scans; ++b) {
        const float* R = real + (int64_t)b * n_beams;
        const float* V = virt + (int64_t)b * n_beams;
        const double* P = poses + (int64_t)b * 7;
        const double qx = P[3], qy = P[4], qz = P[5], qw = P[6];
        const double yaw = std::atan2(2.0 * (qw * qz + qx * qy), 1.0 - 2.0 * (qy * qy + qz * qz));
        auto to_key = [&](float r, float angle, int32_t* k) {
            const float lx = r * std::cos(angle);
            const float ly = r * std::sin(angle);
            const double px = P[0] + (lx * std::cos(yaw) - ly * std::sin(yaw));
            const double py = P[1] + (lx * std::sin(yaw) + ly * std::cos(yaw));
            k[0] = (int)(px / grid_res);
            k[1] = (int)(py / grid_res);
        };
        for (int i = 0; i < n_beams; ++i) {
            const int64_t t = (int64_t)b * n_beams + i;
            new_flag[t] = gone_flag[t] = 0;
            new_key[t * 2] = new_key[t * 2 + 1] = gone_key[t * 2] = gone_key[t * 2 + 1] = 0;
        }
        for (int i = 0; i < n_beams; ++i) {  // 1. new
            const float r_real = R[i];
            if (std::isnan(r_real) || std::isinf(r_real) || r_real > r_max) continue;
            const float angle = r_amin + i * r_inc;
            const float rx = r_real * std::cos(angle), ry = r_real * std::sin(angle);
            bool near_wall = false;
            for (int j = std::max(0, i - window); j < std::min(n_beams, i + window); ++j) {
                const float r_virt = V[j];
                if (std::isinf(r_virt)) continue;
                const float v_angle = v_amin + j * v_inc;
                const float vx = r_virt * std::cos(v_angle), vy = r_virt * std::sin(v_angle);
                if (std::hypot(rx - vx, ry - vy) < thresh) {
                    near_wall = true;
                    break;
                }
            }
            if (!near_wall) {
                const int64_t t = (int64_t)b * n_beams + i;
                new_flag[t] = 1;
                to_key(r_real, angle, new_key + t * 2);
            }
        }
        for (int i = 0; i < n_beams; ++i) {  // 2. removed
            const float r_virt = V[i];
            if (std::isinf(r_virt) || std::isnan(r_virt)) continue;
            const float angle = v_amin + i * v_inc;
            const float vx = r_virt * std::cos(angle), vy = r_virt * std::sin(angle);
            bool still = false;
            for (int j = std::max(0, i - window); j < std::min(n_beams, i + window); ++j) {
                const float r_real = R[j];
                if (std::isinf(r_real) || r_real > r_max) continue;
                const float r_angle = r_amin + j * r_inc;
                const float rx = r_real * std::cos(r_angle), ry = r_real * std::sin(r_angle);
                if (std::hypot(vx - rx, vy - ry) < thresh) {
                    still = true;
                    break;
                }
            }
            if (!still) {
                const int64_t t = (int64_t)b * n_beams + i;
                gone_flag[t] = 1;
                to_key(r_virt, angle, gone_key + t * 2);
            }
        }
    }
}

/* updateGrid + publishCloud (diff_node.cpp:163-222) over a sequence of scans: float cell values, per scan
 * hit cells += dt (cap 1.5 time_thresh), others -= decay * dt, erase at <= 0.  Returns the published cell count;
 * out_xyz (float32 [k][3]) sorted by (x, y). */
int64_t oro_change_grid_run(const int32_t* keys, const uint8_t* flags, int n_scans, int n_beams, const double* dts,
                            double time_thresh, double decay_rate, double grid_res, float* out_xyz) {
    std::map<std::pair<int, int>, float> grid;
    for (int b = 0; b < n_scans; ++b) {
        std::map<std::pair<int, int>, bool> hits;
        for (int i = 0; i < n_beams; ++i) {
            const int64_t t = (int64_t)b * n_beams + i;
            if (flags[t]) hits[{keys[t * 2], keys[t * 2 + 1]}] = true;
        }
        const double dt = dts[b];
        for (const auto& h : hits) {
            grid[h.first] += dt;
            if (grid[h.first] > (time_thresh * 1.5)) grid[h.first] = time_thresh * 1.5;
        }
        for (auto it = grid.begin(); it != grid.end();) {
            if (hits.find(it->first) == hits.end()) it->second -= (decay_rate * dt);
            if (it->second <= 0.0) it = grid.erase(it);
            else ++it;
        }
    }
    int64_t k = 0;
    for (const auto& c : grid)
        if (c.second > time_thresh) {
            if (out_xyz) {
                out_xyz[k * 3 + 0] = (float)((c.first.first * grid_res) + (grid_res / 2.0));
                out_xyz[k * 3 + 1] = (float)((c.first.second * grid_res) + (grid_res / 2.0));
                out_xyz[k * 3 + 2] = 0.0f;
            }
            ++k;
        }
    return k;
}

/* VirtualScanNode::publish_virtual_scan (virtual_scan_node.cpp:245-292) for a batch of robot poses
 * (poses [n][3] = x, y, yaw), written as the node does it. */
void oro_virtual_scan(const int8_t* data, int height, int width, float resolution, float origin_x, float origin_y,
                      int n_scans, int n_beams, float angle_min, float angle_increment, float range_max,
                      const double* poses, float* out) {
    for (int b = 0; b < n_scans; ++b) {
        const double robot_x = poses[b * 3], robot_y = poses[b * 3 + 1], robot_yaw = poses[b * 3 + 2];
        for (int i = 0; i < n_beams; ++i) {
            float r = std::numeric_limits<float>::infinity();
            const double angle = angle_min + i * angle_increment;
            const double global_angle = robot_yaw + angle;
            double dist = 0.0;
            const double step = resolution;
            while (dist < range_max) {
                dist += step;
                const double ray_x = robot_x + dist * cos(global_angle);
                const double ray_y = robot_y + dist * sin(global_angle);
                const int grid_x = (int)((ray_x - origin_x) / resolution);
                const int grid_y = (int)((ray_y - origin_y) / resolution);
                if (grid_x < 0 || grid_x >= width || grid_y < 0 || grid_y >= height) break;
                if (data[grid_y * width + grid_x] == 100) {
                    r = dist;
                    break;
                }
            }
            out[(int64_t)b * n_beams + i] = r;
        }
    }
}

/* hybrid_map.create_map_cloud (hybrid_map.py:25-60). */
int64_t oro_occupancy_to_points(const uint8_t* img, int h, int w, int threshold, double res, double ox, double oy,
                                double* out) {
    int64_t k = 0;
    for (int r = 0; r < h; ++r)
        for (int c = 0; c < w; ++c)
            if (img[(int64_t)r * w + c] < threshold) {
                out[k * 3 + 0] = ox + ((double)c * res);
                out[k * 3 + 1] = oy + ((double)(h - 1 - r) * res);
                out[k * 3 + 2] = 0.0;
                ++k;
            }
    return k;
}

}  // extern "C"
