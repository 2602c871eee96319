// TEST INFRASTRUCTURE ONLY: drives every entry point of the CPU oracle (otslam_oracle.cpp) on a small synthetic
// scene so that `make -C oracle sanitize` can run it under AddressSanitizer + UndefinedBehaviorSanitizer
// (sanitizers on the CPU build).  The checks here are sanity bounds only; parity is the business of
// tests/.  Exit status 0 = no sanitizer report and every bound held.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

extern "C" {
const char* oro_name(void);
void oro_inverse4(const double* m, double* out);
void oro_depth_to_float(const uint16_t* in, float* out, int64_t n, double depth_scale, double depth_trunc);
void oro_depth_multiplier(int w, int h, double fx, double fy, double cx, double cy, float* out);
int64_t oro_unproject(const float* depth, const uint8_t* color, int w, int h, double fx, double fy, double cx,
                      double cy, const double* extrinsic, int stride, double* xyz, double* rgb);
int64_t oro_voxel_down_sample(const double* xyz, const double* rgb, const double* nrm, int64_t n, double vs,
                              double* out_xyz, double* out_rgb, double* out_nrm, int32_t* out_keys);
void* oro_tsdf_create(double voxel_length, double sdf_trunc, int color_type, int stride);
void oro_tsdf_destroy(void* h);
int64_t oro_tsdf_integrate(void* h, const float* depth, const uint8_t* color, int w, int hgt, double fx, double fy,
                           double cx, double cy, const double* extrinsic);
int64_t oro_tsdf_num_units(void* h);
int64_t oro_tsdf_total_updates(void* h);
int64_t oro_tsdf_unit_integrations(void* h);
void oro_tsdf_export(void* h, int32_t* keys, float* tsdf, float* weight, double* color);
void oro_tsdf_extract_mesh(void* h, int64_t* nv, int64_t* nt);
void oro_tsdf_fetch_mesh(void* h, double* V, double* VC, int32_t* T);
void oro_mesh_vertex_normals(const double* V, int64_t nv, const int32_t* T, int64_t nt, double* N);
double oro_mesh_surface_area(const double* V, const int32_t* T, int64_t nt);
int oro_mesh_sample_uniform(const double* V, const double* VN, const double* VC, int64_t nv, const int32_t* T,
                            int64_t nt, int64_t n_points, uint64_t seed, double* P, double* PN, double* PC);
int64_t oro_filter_min_z(const double* xyz, const double* rgb, int64_t n, double zmin, double* oxyz, double* orgb);
int64_t oro_remove_statistical_outlier(const double* xyz, int64_t n, int k, double std_ratio, int64_t* out_idx,
                                       double* out_avg);
int64_t oro_remove_radius_outlier(const double* xyz, int64_t n, int nb_points, double radius, int64_t* out_idx);
void oro_point_cloud_distance(const double* src, int64_t n, const double* tgt, int64_t m, double* out);
void oro_scan_diff(const float* real, const float* virt, int n_scans, int n_beams, float r_amin, float r_inc,
                   float r_max, float v_amin, float v_inc, double thresh, int window, const double* poses,
                   double grid_res, uint8_t* new_flag, uint8_t* gone_flag, int32_t* new_key, int32_t* gone_key);
int64_t oro_change_grid_run(const int32_t* keys, const uint8_t* flags, int n_scans, int n_beams, const double* dts,
                            double time_thresh, double decay_rate, double grid_res, float* out_xyz);
void oro_virtual_scan(const int8_t* data, int height, int width, float resolution, float origin_x, float origin_y,
                      int n_scans, int n_beams, float angle_min, float angle_increment, float range_max,
                      const double* poses, float* out);
int64_t oro_occupancy_to_points(const uint8_t* img, int h, int w, int threshold, double res, double ox, double oy,
                                double* out);
}

static int g_fail = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            std::fprintf(stderr, "check failed: %s (line %d)\n", #c, __LINE__); \
            g_fail = 1;                                                 \
        }                                                               \
    } while (0)

int main() {
    std::printf("%s\n", oro_name());
    const int W = 80, H = 60;
    const double fx = 70.0, fy = 70.0, cx = 39.5, cy = 29.5;
    // a floor at 1.2 m with a box (0.9 m) in the middle, plus some invalid and far pixels
    std::vector<uint16_t> draw(W * H);
    std::vector<uint8_t> color(W * H * 3);
    for (int r = 0; r < H; ++r)
        for (int c = 0; c < W; ++c) {
            uint16_t d = 1200 + (uint16_t)(r / 4);
            if (c > 25 && c < 55 && r > 15 && r < 45) d = 900;
            if ((r * 7 + c * 3) % 97 == 0) d = 0;
            if ((r + c) % 113 == 0) d = 65535;
            draw[r * W + c] = d;
            color[(r * W + c) * 3 + 0] = (uint8_t)(c * 3);
            color[(r * W + c) * 3 + 1] = (uint8_t)(r * 4);
            color[(r * W + c) * 3 + 2] = (uint8_t)((r * c) & 255);
        }
    std::vector<float> depth(W * H), mult(W * H);
    oro_depth_to_float(draw.data(), depth.data(), W * H, 1000.0, 3.0);
    oro_depth_multiplier(W, H, fx, fy, cx, cy, mult.data());
    CHECK(mult[0] >= 1.0f);

    double ext[16] = {1, 0, 0, 0.01, 0, 1, 0, -0.02, 0, 0, 1, 0.03, 0, 0, 0, 1}, inv[16];
    oro_inverse4(ext, inv);
    CHECK(std::fabs(inv[3] + 0.01) < 1e-12);

    std::vector<double> xyz(W * H * 3), rgb(W * H * 3);
    const int64_t n = oro_unproject(depth.data(), color.data(), W, H, fx, fy, cx, cy, ext, 1, xyz.data(), rgb.data());
    CHECK(n > 0 && n <= W * H);

    std::vector<double> vx(n * 3), vc(n * 3), vn(n * 3), nrm(n * 3, 0.0);
    std::vector<int32_t> vk(n * 3);
    const int64_t nv = oro_voxel_down_sample(xyz.data(), rgb.data(), nrm.data(), n, 0.01, vx.data(), vc.data(),
                                             vn.data(), vk.data());
    CHECK(nv > 0 && nv <= n);

    std::vector<int64_t> idx(nv);
    std::vector<double> avg(nv);
    const int64_t ns = oro_remove_statistical_outlier(vx.data(), nv, 20, 2.0, idx.data(), avg.data());
    CHECK(ns > 0 && ns <= nv);
    const int64_t nr = oro_remove_radius_outlier(vx.data(), nv, 4, 0.03, idx.data());
    CHECK(nr >= 0 && nr <= nv);
    std::vector<double> dist(nv);
    oro_point_cloud_distance(vx.data(), nv, xyz.data(), n, dist.data());
    CHECK(dist[0] >= 0.0);

    std::vector<double> zx(nv * 3), zc(nv * 3);
    const int64_t nz = oro_filter_min_z(vx.data(), vc.data(), nv, 0.0, zx.data(), zc.data());
    CHECK(nz >= 0 && nz <= nv);

    // TSDF: three poses, export, mesh, normals, area, sampling
    void* vol = oro_tsdf_create(0.01, 0.04, 1, 1);
    for (int f = 0; f < 3; ++f) {
        double e[16] = {1, 0, 0, 0.01 * f, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
        oro_tsdf_integrate(vol, depth.data(), color.data(), W, H, fx, fy, cx, cy, e);
    }
    const int64_t units = oro_tsdf_num_units(vol);
    CHECK(units > 0);
    CHECK(oro_tsdf_total_updates(vol) > 0 && oro_tsdf_unit_integrations(vol) >= units);
    {
        std::vector<int32_t> k(units * 3);
        std::vector<float> t(units * 4096), w(units * 4096);
        std::vector<double> c(units * 4096 * 3);
        oro_tsdf_export(vol, k.data(), t.data(), w.data(), c.data());
    }
    int64_t mv = 0, mt = 0;
    oro_tsdf_extract_mesh(vol, &mv, &mt);
    CHECK(mv > 0 && mt > 0);
    std::vector<double> V(mv * 3), VC(mv * 3), VN(mv * 3);
    std::vector<int32_t> T(mt * 3);
    oro_tsdf_fetch_mesh(vol, V.data(), VC.data(), T.data());
    oro_tsdf_destroy(vol);
    oro_mesh_vertex_normals(V.data(), mv, T.data(), mt, VN.data());
    CHECK(oro_mesh_surface_area(V.data(), T.data(), mt) > 0.0);
    const int64_t np = 500;
    std::vector<double> P(np * 3), PN(np * 3), PC(np * 3);
    oro_mesh_sample_uniform(V.data(), VN.data(), VC.data(), mv, T.data(), mt, np, 42, P.data(), PN.data(), PC.data());

    // change detection: scan diff over 4 scans, the evidence grid, the virtual scan, the map cloud
    const int S = 4, B = 90;
    std::vector<float> real(S * B), virt(S * B);
    for (int i = 0; i < S * B; ++i) {
        real[i] = 2.0f + 0.3f * std::sin(0.1f * (float)i);
        virt[i] = (i % 17 == 0) ? INFINITY : 2.0f + ((i % 11 == 0) ? 0.5f : 0.0f);
    }
    std::vector<double> poses(S * 7, 0.0);
    for (int s = 0; s < S; ++s) {
        poses[s * 7 + 0] = 0.1 * s;
        poses[s * 7 + 6] = 1.0;
    }
    std::vector<uint8_t> nf(S * B), gf(S * B);
    std::vector<int32_t> nk(S * B * 2), gk(S * B * 2);
    oro_scan_diff(real.data(), virt.data(), S, B, -1.5f, 0.0333f, 10.0f, -1.5f, 0.0333f, 0.1, 5, poses.data(), 0.05,
                  nf.data(), gf.data(), nk.data(), gk.data());
    std::vector<double> dts(S, 0.5);
    const int64_t cells = oro_change_grid_run(nk.data(), nf.data(), S, B, dts.data(), 0.6, 0.5, 0.05, nullptr);
    std::vector<float> cxyz(cells * 3 + 3);
    CHECK(oro_change_grid_run(nk.data(), nf.data(), S, B, dts.data(), 0.6, 0.5, 0.05, cxyz.data()) == cells);

    const int MH = 64, MW = 64;
    std::vector<int8_t> grid(MH * MW, 0);
    for (int i = 0; i < MW; ++i) grid[10 * MW + i] = grid[50 * MW + i] = 100;
    std::vector<double> rp = {1.6, 1.6, 0.0, 1.2, 1.7, 0.5};
    std::vector<float> scan(2 * B);
    oro_virtual_scan(grid.data(), MH, MW, 0.05f, 0.0f, 0.0f, 2, B, -1.5f, 0.0333f, 5.0f, rp.data(), scan.data());
    std::vector<uint8_t> img(MH * MW);
    for (int i = 0; i < MH * MW; ++i) img[i] = (uint8_t)(i * 37);
    std::vector<double> pts(MH * MW * 3);
    CHECK(oro_occupancy_to_points(img.data(), MH, MW, 100, 0.05, -1.0, -2.0, pts.data()) > 0);

    std::printf("points %lld voxels %lld sor %lld ror %lld units %lld mesh %lld/%lld grid cells %lld\n",
                (long long)n, (long long)nv, (long long)ns, (long long)nr, (long long)units, (long long)mv,
                (long long)mt, (long long)cells);
    std::printf(g_fail ? "FAIL\n" : "OK\n");
    return g_fail;
}
