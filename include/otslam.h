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

/* geometry.PointCloud.compute_point_cloud_distance(target) — eval_cone.py:99,103 (accuracy / completeness).
 * out[i] = sqrt(min_j |src_i - tgt_j|^2) in float64 (exact minimum, nanoflann L2 accumulation order);
 * 0.0 for every point when the target is empty (Open3D: no neighbour found). */
ot_status ot_compute_point_cloud_distance(const double* src, int64_t n, const double* tgt, int64_t m,
                                          double* out, void* stream);

/* The configs[2] filter chain for a batch of frames, device-resident end to end (not an Open3D API: the batch form
 * of the per-frame calls below, results bit-identical to them).  Per frame f of a run:
 *   create_from_color_and_depth(depth_scale, depth_trunc) -> PointCloud.create_from_rgbd_image(intrinsic,
 *   extrinsic_f) -> voxel_down_sample(voxel_size) -> remove_statistical_outlier(nb_neighbors, std_ratio)
 *   -> select_by_index(kept)
 * i.e. check_one_frame.py:22-28 (with a pose) followed by the north_star's statistical filter.  A handle keeps its
 * device buffers between runs (grow-only).  Not thread-safe per handle. */
typedef struct ot_rgbd_filter ot_rgbd_filter;
ot_status ot_rgbd_filter_create(const ot_intrinsics* intrinsic, int32_t max_frames, double depth_scale,
                                double depth_trunc, double voxel_size, int32_t nb_neighbors, double std_ratio,
                                ot_rgbd_filter** out);
ot_status ot_rgbd_filter_destroy(ot_rgbd_filter* filter);
/* depth: uint16 [n_frames][h][w], color: uint8 [n_frames][h][w][3] (device, contiguous); extrinsics_host:
 * double [n_frames][16] row-major.  Synchronises `stream` (the result sizes come back to the host). */
ot_status ot_rgbd_filter_run(ot_rgbd_filter* filter, int32_t n_frames, const uint16_t* depth, const uint8_t* color,
                             const double* extrinsics_host, void* stream);
/* Sizes of the last run: valid points, voxels and kept voxels in total, and (nullable) per-frame offsets
 * [n_frames + 1] into the point / voxel / kept arrays. */
ot_status ot_rgbd_filter_sizes(const ot_rgbd_filter* filter, int64_t* points_host, int64_t* voxels_host,
                               int64_t* kept_host, int64_t* point_offsets_host, int64_t* voxel_offsets_host,
                               int64_t* kept_offsets_host);
/* Device arrays of the last run (valid until the next run / destroy; any out-pointer may be NULL): the kept
 * points xyz / rgb f64 [kept][3] and their index inside their frame's voxel cloud (int64, ascending per frame: the
 * indices remove_statistical_outlier returns), the voxel clouds xyz / rgb f64 [voxels][3] (per frame in key order,
 * as ot_voxel_down_sample) and every voxel's mean kNN distance f64 [voxels]. */
ot_status ot_rgbd_filter_outputs(const ot_rgbd_filter* filter, const double** kept_xyz, const double** kept_rgb,
                                 const int64_t** kept_index, const double** voxel_xyz, const double** voxel_rgb,
                                 const double** voxel_avg_dist);
/* Copy frame `frame`'s results (or every frame's, frame = -1) of the last run into caller device buffers, ordered on
 * `stream`; any pointer may be NULL.  Sizes: ot_rgbd_filter_sizes' offsets. */
ot_status ot_rgbd_filter_copy(const ot_rgbd_filter* filter, int32_t frame, double* kept_xyz, double* kept_rgb,
                              int64_t* kept_index, double* voxel_xyz, double* voxel_rgb, double* voxel_avg_dist,
                              void* stream);

/* ---------------------------------------------------------------------------------------------------
 * Scalable TSDF volume — pipelines.integration.ScalableTSDFVolume (reconstruct_rgbd_filter.py:81-85)
 * ------------------------------------------------------------------------------------------------- */
typedef struct ot_tsdf ot_tsdf;

/* ScalableTSDFVolume(voxel_length, sdf_trunc, color_type, volume_unit_resolution=16,
 * depth_sampling_stride=4).  max_units is the INITIAL block-pool capacity in HBM (0 = default 32768 units): like
 * Open3D's volume the pool is unbounded -- a batch that needs more units grows the pool and the hash (records copied,
 * keys rehashed) and its dropped units are integrated again from the staged frames, bit-identical to a large pool;
 * only a failed device allocation is an error (OT_ERR_HIP, from the integrate / flush call whose batch needed it). */
ot_status ot_tsdf_create(double voxel_length, double sdf_trunc, int32_t color_type,
                         int32_t volume_unit_resolution, int32_t depth_sampling_stride, int64_t max_units,
                         ot_tsdf** out);
ot_status ot_tsdf_destroy(ot_tsdf* vol);
ot_status ot_tsdf_reset(ot_tsdf* vol);  /* ScalableTSDFVolume.reset() */
/* The same reset ordered on `stream` (no device-wide synchronisation): several volumes driven from several
 * host threads / streams do not stall each other.  Frames still queued for a batch are integrated first. */
ot_status ot_tsdf_reset_async(ot_tsdf* vol, void* stream);

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
/* n frames of a scan already resident in device memory in one call: frame k's u16 depth at depth + k*W*H, its RGB8 at
 * color + 3*k*W*H (color may be NULL), its extrinsic at extrinsics + 16*k (host).  The same queueing, batching and
 * bits as n calls of ot_tsdf_integrate_u16, without n host round trips (the front of one object's latency). */
ot_status ot_tsdf_integrate_u16_frames(ot_tsdf* vol, int32_t n, const uint16_t* depth, const uint8_t* color,
                                       const ot_intrinsics* in, const double* extrinsics, double depth_scale,
                                       double depth_trunc, void* stream);
ot_status ot_tsdf_flush(ot_tsdf* vol, void* stream);
/* Frames queued on the host for the next batch (their input buffers are still referenced; every frame queued before
 * them has been enqueued on its stream).  Host-only, no synchronisation. */
ot_status ot_tsdf_pending_frames(const ot_tsdf* vol, int32_t* n_host);
/* Batch size used by ot_tsdf_integrate_u16 (1 = integrate immediately, default and maximum 64). */
ot_status ot_tsdf_set_batch(ot_tsdf* vol, int32_t max_frames);
/* Double-buffered batch front end (spatial sharding of one object: reconstruct_rgbd_filter.py:88-109):
 * with mode 1 batch k+1's staging, touch and unit headers run on the caller's stream while batch k's integrate runs on
 * a second stream of the volume (two staging sets); readers (num_units, export, extraction, flush, reset) order the
 * caller's stream after the last integrate.  -1 (default): on for spatially sharded volumes (their split front end
 * stages only their units' tiles; measured faster at 2, 4 and 8 ranks), off otherwise; 0 off; 1 on.
 * Results are identical in every mode.  Fails with OT_ERR_INVALID_ARGUMENT while frames are queued (flush on their stream first). */
ot_status ot_tsdf_set_frontend_overlap(ot_tsdf* vol, int32_t mode);

/* Batch statistics since the last reset (measurement; not an Open3D API): integrate batches run, the units they touched
 * summed over batches, and how many of those were new in their batch (allocated by it: their state starts at zero and
 * is not read).  Frames still queued are not counted (flush first).  The bench's compulsory-bytes figure of the integrate kernel:
 * (2 x unit_batches - new_units) unit records + the staged pixels. */
ot_status ot_tsdf_batch_stats(ot_tsdf* vol, int64_t* batches, int64_t* unit_batches, int64_t* new_units);

/* Number of allocated volume units.  Queued frames are integrated first, on `stream`; synchronises `stream`. */
ot_status ot_tsdf_num_units(ot_tsdf* vol, int64_t* n_units_host, void* stream);
/* Cumulative voxel updates and volume-unit integrations since create/reset (flushes on `stream`, synchronises it). */
ot_status ot_tsdf_counters(ot_tsdf* vol, int64_t* voxel_updates_host, int64_t* unit_integrations_host,
                           void* stream);
/* Colour state precision: 64 (the default, as in the Python facade) keeps each voxel's running colour mean in float64
 * with exact IEEE division, as Open3D's TSDFVoxel::color_ (Eigen::Vector3d; reconstruct_rgbd_filter.py:81-85 ->
 * SURVEY A.3(iv)) -- bit-exact colours, 128-KiB unit records; 32 keeps float32 with one hardware reciprocal per update
 * (|rel| <= 1e-4, 80-KiB records, faster).  NoColor volumes keep no colour state whatever the setting (get reports
 * 32).  Call before the first integrate (the unit pool is reallocated when the record size changes). */
ot_status ot_tsdf_set_color_precision(ot_tsdf* vol, int32_t bits);
ot_status ot_tsdf_get_color_precision(const ot_tsdf* vol, int32_t* bits_host);

/* Kernel timing for roofline reporting: when enabled, HIP events bracket every launch of the dominant
 * integration kernel on the caller's stream; ot_tsdf_kernel_time returns the summed device time (ms) and the
 * number of timed launches since profiling was enabled (synchronises). */
ot_status ot_tsdf_set_profiling(ot_tsdf* vol, int32_t enable);
ot_status ot_tsdf_kernel_time(ot_tsdf* vol, double* total_ms_host, int64_t* launches_host);
/* The same for each batch's front end (frame staging + unit touch + unit headers): the work every rank of a
 * spatially sharded volume repeats for all pixels (bench.py's Amdahl bound of single-object sharding). */
ot_status ot_tsdf_frontend_time(ot_tsdf* vol, double* total_ms_host, int64_t* batches_host);

/* Dump every unit sorted by key (kx, ky, kz): keys int32 [U][3]; per unit 4096 voxels in Open3D
 * IndexOf order (x*256 + y*16 + z): tsdf f32, weight f32, color f32 [3] (0..255).  Any pointer may be
 * NULL.  Device pointers; every output holds `capacity` units. */
ot_status ot_tsdf_export_units(ot_tsdf* vol, int64_t capacity, int32_t* keys, float* tsdf, float* weight,
                               float* color, void* stream);
/* The colours as float64, [U][4096][3] in export_units' order: exact for a colour-precision-64 volume, the float32
 * state widened otherwise.  Both exports fail with OT_ERR_CAPACITY when the volume holds more than `capacity` units
 * (outputs sized from an older unit count).  A spatially sharded volume exports (and ot_tsdf_num_units counts) only
 * its own units, not the halo units ot_tsdf_import_border added. */
ot_status ot_tsdf_export_color64(ot_tsdf* vol, int64_t capacity, double* color, void* stream);

/* The inverse of ot_tsdf_export_units (same layouts): insert n units, overwriting any unit with the same key;
 * keys must be unique within one call.  color may be NULL (zeros).  Used to assemble a spatially sharded volume
 * on one GPU before extract_triangle_mesh.  Device pointers. */
ot_status ot_tsdf_import_units(ot_tsdf* vol, int64_t n, const int32_t* keys, const float* tsdf, const float* weight,
                               const float* color, void* stream);
/* The same for a colour-precision-64 volume (float64 colours, export_color64's layout). */
ot_status ot_tsdf_import_units_color64(ot_tsdf* vol, int64_t n, const int32_t* keys, const float* tsdf,
                                       const float* weight, const double* color, void* stream);

/* Spatial sharding of ONE object's volume over `world` GPUs (not an Open3D API): this volume
 * allocates and integrates only the units whose owner hash(key) mod world == rank.  Every rank integrates every
 * frame; each voxel still sees the frames in call order, so the union of the ranks' exported units is bit-identical
 * to one unsharded volume.  Call before the first integrate.  The hash is of the unit's ownership block (below). */
ot_status ot_tsdf_set_shard(ot_tsdf* vol, int32_t rank, int32_t world);
/* Ownership granularity of a sharded volume: blocks of 2^log2_units units per axis share one owner (the hash is taken
 * of the block key).  Set by ot_tsdf_set_shard to 2 (4^3 units) up to 4 ranks and 1 beyond; call after it, before the
 * first integrate. */
ot_status ot_tsdf_set_shard_block(ot_tsdf* vol, int32_t log2_units);
/* Sector ownership (round 6): the unit is owned by the azimuth sector (world equal sectors of the pseudo-angle; the true
 * 90 / 45 degree sectors at 4 / 8 ranks) of its centre around the scan centre (cx, cy) in metres -- for a ring scan the
 * look-at point, e.g. the ScanObject goal's x, y (otslam_interfaces/action/ScanObject.action) or the mean camera
 * position.  Each frame then sees a contiguous arc of a rank's units, so a sharded rank stages only the image tiles its
 * units project to (the split front end: tools/shard_sector_model.py).  Integer arithmetic on the unit
 * key only: results are exact for any centre.  Call instead of ot_tsdf_set_shard, before the first integrate. */
ot_status ot_tsdf_set_shard_sector(ot_tsdf* vol, int32_t rank, int32_t world, double cx, double cy);
/* Border-halo routing: per border row key int32 [n][3] (export_border's), the bitmask (bit r = rank r,
 * world <= 64) of the other ranks that own one of the unit's 7 -x/-y/-z neighbours -- the only ranks whose marching
 * cubes can read the row.  Device pointers; ordered on `stream`. */
ot_status ot_tsdf_border_destinations(const ot_tsdf* vol, int64_t n, const int32_t* keys, int64_t* dest_mask,
                                      void* stream);

/* Border halo of a spatially sharded volume (SURVEY §8(e) "all-gather of border faces"; not an Open3D API).
 * export_border: per OWN unit (sorted key order; halo units are not exported) its 721 low-face voxels (x == 0 ||
 * y == 0 || z == 0, increasing x*256 + y*16 + z): keys int32 [n][3], tsdf / weight f32 [n][721], colour
 * [n][721][3] in the volume's colour precision (f32, or f64 after ot_tsdf_set_color_precision(64); NULL to skip);
 * the row count to *n_exported_host (capacity: rows the buffers hold, ot_tsdf_num_units is enough).
 * import_border: rows of other shards; a row becomes a halo unit when its key is not owned by this shard and one of
 * its -x/-y/-z neighbours is (marching cubes of the own units reads exactly these voxels); other rows are skipped.
 * Marching cubes of a sharded volume then emits only the own units' cubes; ot_tsdf_fetch_mesh_keys gives the keys
 * that merge the shards' meshes into the unsharded mesh (distributed.extract_sharded_mesh). */
ot_status ot_tsdf_export_border(ot_tsdf* vol, int64_t capacity, int32_t* keys, float* tsdf, float* weight, void* color,
                                int64_t* n_exported_host, void* stream);
ot_status ot_tsdf_import_border(ot_tsdf* vol, int64_t n, const int32_t* keys, const float* tsdf, const float* weight,
                                const void* color, void* stream);

/* volume.extract_triangle_mesh() — reconstruct_rgbd_filter.py:112 (marching cubes, Appendix A.4).
 * Runs the extraction and stores the mesh inside the handle; returns its sizes.  Vertices are ordered by
 * (unit key, local voxel, edge) — a canonical order; Open3D's is hash order. */
ot_status ot_tsdf_extract_triangle_mesh(ot_tsdf* vol, int64_t* n_vertices_host, int64_t* n_triangles_host,
                                        void* stream);
/* Copy the extracted mesh out: vertices f64 [V][3], colors f64 [V][3] (0..1, NULL to skip),
 * triangles int32 [T][3].  Device pointers; ordered on `stream` (no synchronisation: the extraction and these copies
 * complete in stream order, before any later work on that stream). */
ot_status ot_tsdf_fetch_triangle_mesh(ot_tsdf* vol, double* vertices, double* vertex_colors,
                                      int32_t* triangles, void* stream);
/* The extraction in two phases, writing the mesh straight into the caller's arrays (no copy out of the volume's own
 * buffers): _count classifies, counts and returns the vertex / triangle totals (one read-back); _emit then writes
 * vertices [nv][3], vertex colours [nv][3] (may be NULL; zeros for NoColor) and triangles [nt][3] into device arrays
 * sized from those totals, in stream order.  _emit fails once the volume has changed since _count.  After a _count,
 * ot_tsdf_fetch_triangle_mesh emits again into its arguments (same bits) while the volume is unchanged;
 * ot_tsdf_fetch_mesh_keys needs one emission first. */
ot_status ot_tsdf_extract_triangle_mesh_count(ot_tsdf* vol, int64_t* n_vertices, int64_t* n_triangles, void* stream);
ot_status ot_tsdf_emit_triangle_mesh(ot_tsdf* vol, double* vertices, double* vertex_colors, int32_t* triangles,
                                     void* stream);
/* Count and emit in one call, for callers that can guess the size (e.g. the last extraction of this volume): the
 * emission into the given arrays (capacity_vertices / capacity_triangles rows) is queued before the totals are read
 * back, so the GPU does not wait for the host.  Returns OT_OK with the totals when they fit; otherwise
 * OT_ERR_CAPACITY with the totals set (rows past the capacities were not written): emit with
 * ot_tsdf_emit_triangle_mesh into arrays of that size. */
ot_status ot_tsdf_extract_triangle_mesh_into(ot_tsdf* vol, double* vertices, double* vertex_colors,
                                             int32_t* triangles, int64_t capacity_vertices, int64_t capacity_triangles,
                                             int64_t* n_vertices, int64_t* n_triangles, void* stream);
/* Serial of the last extraction (ot_tsdf_extract_triangle_mesh), or -1 once the volume has changed since (frames
 * integrated, reset, units imported). */
ot_status ot_tsdf_mesh_serial(const ot_tsdf* vol, int64_t* serial_host);
/* mesh.compute_vertex_normals() (reconstruct_rgbd_filter.py:113) of the mesh of extraction `serial`, whose
 * arrays (device pointers, unmodified) are passed: the same bits as ot_mesh_compute_vertex_normals, from the
 * marching-cubes structure kept with the volume (each vertex is a cut edge; its triangles are those of the <= 4 cubes
 * sharing it, walked in triangle order) instead of a sort of the 3T corners.  OT_ERR_INVALID_ARGUMENT when the volume
 * changed since that extraction or the sizes differ (take ot_mesh_compute_vertex_normals then).  Ordered on `stream`,
 * no synchronisation. */
ot_status ot_tsdf_mesh_vertex_normals(ot_tsdf* vol, int64_t serial, const double* vertices, int64_t n_vertices,
                                      const int32_t* triangles, int64_t n_triangles, double* out, void* stream);
/* Merge keys of the extracted mesh (device pointers, NULL to skip): per vertex int32 [V][4] = owner unit key
 * (x, y, z) and edge bit (local voxel x*256+y*16+z times 3 plus axis) -- the canonical vertex order; per triangle
 * int32 [T][3] = the unit key of its cube. */
ot_status ot_tsdf_fetch_mesh_keys(ot_tsdf* vol, int32_t* vertex_keys, int32_t* triangle_units, void* stream);

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

/* mesh.get_surface_area() — Open3D TriangleMesh::GetSurfaceArea, the first of SamplePointsUniformly's two serial
 * float64 chains (reconstruct_rgbd_filter.py:123): ((0 + a_0) + a_1) + ... over the triangle areas in index order,
 * bit-exact.  area_host: host double. */
ot_status ot_mesh_get_surface_area(const double* vertices, int64_t n_vertices, const int32_t* triangles,
                                   int64_t n_triangles, double* area_host, void* stream);

/* The same sampling for several meshes in one call (e.g. the objects of a multi-object run on one GPU): results
 * are identical to one ot_mesh_sample_points_uniformly call per mesh; the meshes' area sums and CDFs are computed
 * side by side.  jobs_host: host array; every pointer inside is a device pointer. */
typedef struct ot_mesh_sample_job {
    const double* vertices;
    const double* vertex_normals;  /* may be NULL */
    const double* vertex_colors;   /* may be NULL */
    int64_t n_vertices;
    const int32_t* triangles;
    int64_t n_triangles;
    double* out_xyz;               /* [n_points][3] */
    double* out_normals;           /* may be NULL */
    double* out_colors;            /* may be NULL */
} ot_mesh_sample_job;
ot_status ot_mesh_sample_points_uniformly_batch(const ot_mesh_sample_job* jobs_host, int32_t n_jobs,
                                                int64_t n_points, uint64_t seed, void* stream);
/* The same, with a hipEvent_t (nullable) that the point emission waits for: the area sums and CDFs read only the
 * vertices and triangles and start at once, while the vertex normals (or colours) the emission interpolates may
 * still be computed on another stream (the facade's compute_vertex_normals of a fresh mesh,
 * reconstruct_rgbd_filter.py:113 -> :123). */
ot_status ot_mesh_sample_points_uniformly_after(const ot_mesh_sample_job* jobs_host, int32_t n_jobs,
                                                int64_t n_points, uint64_t seed, void* inputs_ready_event,
                                                void* stream);
/* reconstruct_rgbd_filter.py:123-132 in one pass per mesh: sample_points_uniformly(n_points) (the same points as
 * ot_mesh_sample_points_uniformly with this seed), then the Z mask points[:, 2] >= z_min (NaN fails) applied in
 * the sampling order.  The reference rebuilds its cloud from the points and colours alone, so the kept rows are written
 * to out_xyz / out_colors (each with room for n_points rows; out_colors may be NULL) and normals are not interpolated
 * (out_normals and vertex_normals are ignored: the vertex normals need not be ready).  n_kept_host: host int64_t
 * [n_jobs], the kept row count of each job.  Synchronises the stream. */
ot_status ot_mesh_sample_points_min_z(const ot_mesh_sample_job* jobs_host, int32_t n_jobs, int64_t n_points,
                                      uint64_t seed, double z_min, int64_t* n_kept_host, void* stream);
/* reconstruct_rgbd_filter.py:112-132 of one volume in ONE host call (replaces the facade's extract_triangle_mesh ->
 * compute_vertex_normals -> sample_points_uniformly + Z-mask sequence at :112-132; no host work between the
 * marching-cubes totals and the sampler's first launch): the mesh into vertices / vertex_colors / triangles with the
 * given capacities exactly as ot_tsdf_extract_triangle_mesh_into, then ot_mesh_sample_points_min_z of it (n_points,
 * seed, z_min; kept rows into out_xyz / out_rgb, each with room for n_points rows; out_rgb may be NULL), and its vertex
 * normals (ot_tsdf_mesh_vertex_normals, bit-identical to ot_mesh_compute_vertex_normals) into vertex_normals (NULL:
 * none) on normals_stream beside the sampling -- a reader of the normals orders itself after normals_stream.
 * OT_ERR_CAPACITY: the mesh did not fit; *n_vertices / *n_triangles are its size, nothing was sampled (emit it with
 * ot_tsdf_emit_triangle_mesh and sample it separately).  An empty mesh samples nothing (*n_kept_host = 0).
 * Synchronises `stream`. */
ot_status ot_tsdf_extract_sample_min_z(ot_tsdf* vol, double* vertices, double* vertex_colors, int32_t* triangles,
                                       int64_t capacity_vertices, int64_t capacity_triangles, double* vertex_normals,
                                       void* normals_stream, int64_t n_points, uint64_t seed, double z_min,
                                       double* out_xyz, double* out_rgb, int64_t* n_vertices_host,
                                       int64_t* n_triangles_host, int64_t* n_kept_host, void* stream);
/* The same in two calls: _async queues the sampling and returns without synchronising (the output arrays must stay
 * allocated), _wait synchronises it and fills n_kept_host.  Between them the calling thread may queue other work (the
 * facade queues a fresh mesh's deferred vertex normals there, beside the sampling's walks) but no other sampling. */
ot_status ot_mesh_sample_points_min_z_async(const ot_mesh_sample_job* jobs_host, int32_t n_jobs, int64_t n_points,
                                            uint64_t seed, double z_min, void* stream);
ot_status ot_mesh_sample_points_min_z_wait(int32_t n_jobs, int64_t* n_kept_host);

/* ---------------------------------------------------------------------------------------------------
 * Hybrid map — fusion/hybrid_map.py
 * ------------------------------------------------------------------------------------------------- */

/* create_map_cloud (hybrid_map.py:25-60): occupied pixels (img < threshold) in row-major order →
 * (ox + c*res, oy + (h-1-r)*res, 0).  img: uint8 [h][w].  out_xyz holds h*w rows. */
ot_status ot_occupancy_to_points(const uint8_t* img, int32_t height, int32_t width, int32_t threshold,
                                 double resolution, double origin_x, double origin_y, double* out_xyz,
                                 int64_t* n_out_host, void* stream);

/* ---------------------------------------------------------------------------------------------------
 * Change detection against a saved map (BASELINE configs[4])
 * ------------------------------------------------------------------------------------------------- */

/* 2d_selective_merge.py:58-69 smart_paste(base_img, overlay_img, x, y, w, h), in place on device uint8
 * [height][width] grids: inside the rectangle, cells of `overlay` outside [unknown - threshold,
 * unknown + threshold] (205 ± 5 in the reference) overwrite `base`.  A rectangle reaching outside the image
 * leaves `base` unchanged (:59-60).  n_changed_host (optional) = cells whose value changed. */
ot_status ot_grid_smart_paste(uint8_t* base, const uint8_t* overlay, int32_t height, int32_t width, int32_t x,
                              int32_t y, int32_t w, int32_t h, int32_t unknown, int32_t threshold,
                              int64_t* n_changed_host, void* stream);

/* Voxel-key set difference of a new cloud against a saved cloud on the lattice floor((p - origin) / voxel_size)
 * (origin: host double[3]).  out_added = keys of `new` absent from `old`, out_removed = keys of `old` absent
 * from `new`, each int32 [k][3] sorted lexicographically (capacity: the cloud's point count). */
ot_status ot_voxel_key_diff(const double* new_xyz, int64_t n, const double* old_xyz, int64_t m, double voxel_size,
                            const double origin[3], int32_t* out_added, int64_t* n_added_host,
                            int32_t* out_removed, int64_t* n_removed_host, void* stream);

/* The same for n_objects objects at once (a hybrid map's object clouds vs their saved versions): clouds are
 * concatenated, object j = rows [offsets[j], offsets[j+1]) (host offsets, n_objects + 1 each); outputs are
 * int32 [k][4] = (object, x, y, z), sorted by object then key.  Lattice coordinates must lie in (-2^30, 2^30)
 * and the joint extent plus the object id must pack into 64 bits; at most 2048 objects.  Equals n_objects calls
 * of ot_voxel_key_diff. */
ot_status ot_voxel_key_diff_multi(const double* new_xyz, const int64_t* new_offsets, const double* old_xyz,
                                  const int64_t* old_offsets, int32_t n_objects, double voxel_size,
                                  const double origin[3], int32_t* out_added, int64_t* n_added_host,
                                  int32_t* out_removed, int64_t* n_removed_host, void* stream);

/* diff_node.cpp:103-160 ChangeDetectorNode::scanCallback, batched: n_scans pairs of float ranges
 * [n_scans][n_beams] (real scan, virtual scan of the saved map).  Per beam: new_flags = a real return with no
 * virtual return within +-search_window beams closer than distance_threshold; gone_flags = the converse.
 * Flagged beams are moved to the map frame with poses_host[n_scans][7] = (tx, ty, tz, qx, qy, qz, qw) and
 * binned to (int)(p / grid_resolution) cells (int32 [n_scans][n_beams][2]; 0 where not flagged). */
ot_status ot_scan_diff(const float* real_ranges, const float* virtual_ranges, int32_t n_scans, int32_t n_beams,
                       float real_angle_min, float real_angle_increment, float real_range_max,
                       float virtual_angle_min, float virtual_angle_increment, double distance_threshold,
                       int32_t search_window, const double* poses_host, double grid_resolution, uint8_t* new_flags,
                       uint8_t* gone_flags, int32_t* new_keys, int32_t* gone_keys, void* stream);

/* virtual_scan_node.cpp:245-292 publish_virtual_scan, batched: the saved map (OccupancyGrid int8 [height][width],
 * 100 = occupied; resolution / origin as the message's float fields) ray-marched per beam in steps of one
 * resolution from each robot pose (poses_host [n_scans][3] = x, y, yaw — yaw as tf2::getYaw); out_ranges float32
 * [n_scans][n_beams], +inf where no occupied cell is met before range_max or the map edge. */
ot_status ot_virtual_scan(const int8_t* grid, int32_t height, int32_t width, float resolution, float origin_x,
                          float origin_y, int32_t n_scans, int32_t n_beams, float angle_min, float angle_increment,
                          float range_max, const double* poses_host, float* out_ranges, void* stream);

/* diff_node.cpp:163-185 updateGrid / :188-222 publishCloud: time-decayed evidence grid (host state). */
typedef struct ot_change_grid ot_change_grid;
ot_status ot_change_grid_create(double time_threshold, double decay_rate, double grid_resolution,
                                ot_change_grid** out);
ot_status ot_change_grid_destroy(ot_change_grid* grid);
/* one scan: cells of the flagged beams (host keys [n][2], flags [n]) += dt (capped at 1.5 time_threshold);
 * all other cells -= decay_rate * dt; cells at <= 0 are erased. */
ot_status ot_change_grid_update(ot_change_grid* grid, const int32_t* keys_host, const uint8_t* flags_host,
                                int64_t n, double dt);
/* cells above time_threshold as float32 (x*res + res/2, y*res + res/2, 0), sorted by (x, y); out may be NULL
 * to query the count. */
ot_status ot_change_grid_publish(const ot_change_grid* grid, float* out_xyz_host, int64_t capacity,
                                 int64_t* n_host);

#ifdef __cplusplus
}
#endif

#endif /* OTSLAM_H */
