/*
 * otslam.h — C ABI of the MI355X-native RGB-D reconstruction / voxel-filter path.
 *
 * This is the drop-in boundary.  The reference (TakiRyo/object-triggered-3D-SLAM) has no FFI of its own:
 * its scripts call the Open3D Python API directly.  Every entry point below replaces one
 * Open3D call made on the hot path; the reference call site it stands behind is cited per function.
 * The Python facade (object-triggered-3d-slam_amd/) binds these with ctypes and keeps Open3D's names,
 * keyword arguments, defaults and RuntimeError behaviour.
 *
 * Conventions
 *   - All bulk arrays are DEVICE pointers (HBM of the device current for the calling thread) unless the
 *     parameter name ends in `_host`.  Small parameter blocks (intrinsics, 4x4 matrices) are host memory.
 *   - `stream` is a hipStream_t passed as void*; NULL = the null stream.  Functions that must return a
 *     size to the host (n_points, n_kept, ...) synchronise that stream before returning.
 *   - Matrices are row-major double[16] (numpy's default layout for a 4x4 float64 array).
 *   - Return value: OT_OK (0) or an error code; ot_last_error() returns a thread-local message in the
 *     Open3D style ("[ScalableTSDFVolume::Integrate] Unsupported image format.").
 *   - Point clouds are SoA-free AoS float64 [n][3] exactly like Open3D's std::vector<Eigen::Vector3d>.
 */
#ifndef OTSLAM_H
#define OTSLAM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int ot_status;
#define OT_OK 0
#define OT_ERR_INVALID_ARGUMENT 1
#define OT_ERR_UNSUPPORTED_FORMAT 2
#define OT_ERR_CAPACITY 3
#define OT_ERR_HIP 4

/* TSDFVolumeColorType (open3d.pipelines.integration.TSDFVolumeColorType) */
#define OT_COLOR_NONE 0
#define OT_COLOR_RGB8 1

/* camera.PinholeCameraIntrinsic(width, height, fx, fy, cx, cy) — reconstruct_rgbd_filter.py:26-29 */
typedef struct ot_intrinsics {
    int32_t width;
    int32_t height;
    double fx, fy, cx, cy;
} ot_intrinsics;

const char* ot_last_error(void);
const char* ot_version(void);
int32_t ot_abi_version(void);

/* ---------------------------------------------------------------------------------------------------
 * Images
 * ------------------------------------------------------------------------------------------------- */

/* geometry.RGBDImage.create_from_color_and_depth(color, depth, depth_scale, depth_trunc,
 *     convert_rgb_to_intensity=False) — depth part (Open3D Image::ConvertDepthToFloatImage).
 * Replaces reconstruct_rgbd_filter.py:98-103 and check_one_frame.py:22-25.
 * out[i] = (float)in[i] / (float)depth_scale; out[i] = 0 if out[i] >= depth_trunc. */
ot_status ot_depth_to_float(const uint16_t* depth_u16, float* depth_f32, int64_t n_pixels,
                            double depth_scale, double depth_trunc, void* stream);

/* Open3D Image::CreateDepthToCameraDistanceMultiplierFloatImage (called inside
 * ScalableTSDFVolume::Integrate, reconstruct_rgbd_filter.py:105).  out: float [height][width]. */
ot_status ot_depth_multiplier(const ot_intrinsics* intrinsic, float* out, void* stream);

/* ---------------------------------------------------------------------------------------------------
 * Point clouds
 * ------------------------------------------------------------------------------------------------- */

/* geometry.PointCloud.create_from_rgbd_image(rgbd, intrinsic, extrinsic)   (color != NULL, RGB8)
 * geometry.PointCloud.create_from_depth_image(depth, intrinsic, extrinsic, stride) (color == NULL)
 * Replaces check_one_frame.py:27.  Valid pixels (d > 0) in row-major order; xyz = inverse(extrinsic) *
 * ((j-cx)*z/fx, (i-cy)*z/fy, z, 1) in float64; rgb = color/255.  out_xyz/out_rgb: [capacity][3].
 * capacity must be >= ceil(h/stride)*ceil(w/stride).  *n_points_host receives P. */
ot_status ot_unproject(const float* depth, const uint8_t* color, const ot_intrinsics* intrinsic,
                       const double extrinsic[16], int32_t stride, double* out_xyz, double* out_rgb,
                       int64_t capacity, int64_t* n_points_host, void* stream);

/* geometry.PointCloud.voxel_down_sample(voxel_size) — check_one_frame.py:28.
 * Voxels are emitted sorted by (kx, ky, kz) lexicographically (Open3D emits hash order; parity compares
 * the sorted set).  Averages are sum/count in float64 with the sum taken in input-index order.
 * rgb / normals may be NULL (then their outputs are ignored).  out_keys (nullable): int32 [K][3].
 * Output buffers must hold n rows. */
ot_status ot_voxel_down_sample(const double* xyz, const double* rgb, const double* normals, int64_t n,
                               double voxel_size, double* out_xyz, double* out_rgb, double* out_normals,
                               int32_t* out_keys, int64_t* n_out_host, void* stream);

/* geometry.PointCloud.remove_statistical_outlier(nb_neighbors, std_ratio) — north_star (not called by
 * the reference scripts; Open3D API contract).  Writes the kept indices
 * (ascending, int64) and, if out_avg_dist != NULL, the per-point mean kNN distance (-1 when none). */
ot_status ot_remove_statistical_outlier(const double* xyz, int64_t n, int32_t nb_neighbors,
                                        double std_ratio, int64_t* out_indices, double* out_avg_dist,
                                        int64_t* n_kept_host, void* stream);

/* geometry.PointCloud.remove_radius_outlier(nb_points, radius) — Appendix A.7.  Keeps i when
 * |{j : |pj - pi|^2 < radius^2}| > nb_points (self included).  Writes kept indices ascending. */
ot_status ot_remove_radius_outlier(const double* xyz, int64_t n, int32_t nb_points, double radius,
                                   int64_t* out_indices, int64_t* n_kept_host, void* stream);

/* Stable compaction `mask = points[:, 2] >= z_min` — reconstruct_rgbd_filter.py:126-132.
 * rgb may be NULL.  Output buffers hold n rows. */
ot_status ot_filter_min_z(const double* xyz, const double* rgb, int64_t n, double z_min,
                          double* out_xyz, double* out_rgb, int64_t* n_out_host, void* stream);

/* Gather rows: out[k] = in[idx[k]] for k < m (PointCloud.select_by_index / SelectByIndex). */
ot_status ot_gather_rows3(const double* in, const int64_t* idx, int64_t m, double* out, void* stream);

/* ---------------------------------------------------------------------------------------------------
 * Scalable TSDF volume — pipelines.integration.ScalableTSDFVolume (reconstruct_rgbd_filter.py:81-85)
 * ------------------------------------------------------------------------------------------------- */
typedef struct ot_tsdf ot_tsdf;

/* ScalableTSDFVolume(voxel_length, sdf_trunc, color_type, volume_unit_resolution=16,
 * depth_sampling_stride=4).  max_units bounds the block pool in HBM (0 = default 65536 units). */
ot_status ot_tsdf_create(double voxel_length, double sdf_trunc, int32_t color_type,
                         int32_t volume_unit_resolution, int32_t depth_sampling_stride, int64_t max_units,
                         ot_tsdf** out);
ot_status ot_tsdf_destroy(ot_tsdf* vol);
ot_status ot_tsdf_reset(ot_tsdf* vol);  /* ScalableTSDFVolume.reset() */

/* volume.integrate(rgbd, intrinsic, extrinsic) — reconstruct_rgbd_filter.py:105.
 * depth: float32 [h][w] (already scaled/truncated); color: uint8 [h][w][3] (RGB8) or NULL (NoColor). */
ot_status ot_tsdf_integrate(ot_tsdf* vol, const float* depth, const uint8_t* color,
                            const ot_intrinsics* intrinsic, const double extrinsic[16], void* stream);

/* Fused RGBDImage.create_from_color_and_depth + integrate on raw uint16 depth (bit-identical to the
 * two-step path).  Frames are queued and integrated in batches (temporal blocking: each block is read
 * and written once per batch, voxels see frames in call order).  The queue is flushed by
 * ot_tsdf_flush, by any read of the volume and when it is full.  Input buffers must stay valid and
 * unmodified until the next flush returns (the Python facade keeps them alive). */
ot_status ot_tsdf_integrate_u16(ot_tsdf* vol, const uint16_t* depth, const uint8_t* color,
                                const ot_intrinsics* intrinsic, const double extrinsic[16],
                                double depth_scale, double depth_trunc, void* stream);
ot_status ot_tsdf_flush(ot_tsdf* vol, void* stream);
/* Batch size used by ot_tsdf_integrate_u16 (1 = integrate immediately, default 32). */
ot_status ot_tsdf_set_batch(ot_tsdf* vol, int32_t max_frames);

/* Number of allocated volume units (synchronises). */
ot_status ot_tsdf_num_units(ot_tsdf* vol, int64_t* n_units_host);
/* Cumulative voxel updates and volume-unit integrations since create/reset (synchronises). */
ot_status ot_tsdf_counters(ot_tsdf* vol, int64_t* voxel_updates_host, int64_t* unit_integrations_host);

/* Kernel timing for roofline reporting: when enabled, HIP events bracket every launch of the dominant
 * integration kernel on the caller's stream; ot_tsdf_kernel_time returns the summed device time (ms) and the
 * number of timed launches since profiling was enabled (synchronises). */
ot_status ot_tsdf_set_profiling(ot_tsdf* vol, int32_t enable);
ot_status ot_tsdf_kernel_time(ot_tsdf* vol, double* total_ms_host, int64_t* launches_host);

/* Dump every unit sorted by key (kx, ky, kz): keys int32 [U][3]; per unit 4096 voxels in Open3D
 * IndexOf order (x*256 + y*16 + z): tsdf f32, weight f32, color f32 [3] (0..255).  Any pointer may be
 * NULL.  Device pointers. */
ot_status ot_tsdf_export_units(ot_tsdf* vol, int32_t* keys, float* tsdf, float* weight, float* color,
                               void* stream);

/* volume.extract_triangle_mesh() — reconstruct_rgbd_filter.py:112 (marching cubes, Appendix A.4).
 * Runs the extraction and stores the mesh inside the handle; returns its sizes.  Vertices are ordered by
 * (unit key, local voxel, edge) — a canonical order; Open3D's is hash order. */
ot_status ot_tsdf_extract_triangle_mesh(ot_tsdf* vol, int64_t* n_vertices_host, int64_t* n_triangles_host,
                                        void* stream);
/* Copy the extracted mesh out: vertices f64 [V][3], colors f64 [V][3] (0..1, NULL to skip),
 * triangles int32 [T][3].  Device pointers. */
ot_status ot_tsdf_fetch_triangle_mesh(ot_tsdf* vol, double* vertices, double* vertex_colors,
                                      int32_t* triangles, void* stream);

/* ---------------------------------------------------------------------------------------------------
 * Triangle meshes
 * ------------------------------------------------------------------------------------------------- */

/* mesh.compute_vertex_normals() — reconstruct_rgbd_filter.py:113 (Appendix A.5). */
ot_status ot_mesh_compute_vertex_normals(const double* vertices, int64_t n_vertices,
                                         const int32_t* triangles, int64_t n_triangles, double* out_normals,
                                         void* stream);

/* mesh.sample_points_uniformly(number_of_points) — reconstruct_rgbd_filter.py:123 (Appendix A.8), with a
 * seeded counter-based RNG (Open3D's is unseeded).  normals / colors may be NULL. */
ot_status ot_mesh_sample_points_uniformly(const double* vertices, const double* vertex_normals,
                                          const double* vertex_colors, int64_t n_vertices,
                                          const int32_t* triangles, int64_t n_triangles, int64_t n_points,
                                          uint64_t seed, double* out_xyz, double* out_normals,
                                          double* out_colors, void* stream);

/* ---------------------------------------------------------------------------------------------------
 * Hybrid map — fusion/hybrid_map.py
 * ------------------------------------------------------------------------------------------------- */

/* create_map_cloud (hybrid_map.py:25-60): occupied pixels (img < threshold) in row-major order →
 * (ox + c*res, oy + (h-1-r)*res, 0).  img: uint8 [h][w].  out_xyz holds h*w rows. */
ot_status ot_occupancy_to_points(const uint8_t* img, int32_t height, int32_t width, int32_t threshold,
                                 double resolution, double origin_x, double origin_y, double* out_xyz,
                                 int64_t* n_out_host, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* OTSLAM_H */
