// tsdf.h — device layout of the scalable TSDF volume (pipelines.integration.ScalableTSDFVolume).
//
// HBM layout (one allocation per field group, sized at create time):
//   hash table  : open addressing, linear probing, capacity = pow2 >= 4 * max_units
//                 hkeys u64 (packed int3 unit key, KEY_EMPTY = ~0), hvals i32 (unit id, -1 = not allocated),
//                 fmask u64 (frames of the current batch touching the unit)
//   unit pool   : max_units blocks of 16^3 voxels, field-planar inside a block:
//                 vox[id][field][z][x*16 + y], field = {tsdf, weight, r, g, b} (f32).  One 256-lane
//                 workgroup owns a block; lane (x, y) walks z, so every z step is one coalesced 1-KiB row
//                 per field (the per-column z walk is what reproduces Open3D's incremental float math).
//   unit_keys   : int32 [max_units][3]
// max_units and the hash capacity grow on demand (tsdf.hip grow_pool): Open3D's volume is unbounded.
#pragma once

#include <vector>

#include "common.h"

namespace ot {

constexpr int UNIT_RES = 16;
constexpr int UNIT_VOX = UNIT_RES * UNIT_RES * UNIT_RES;  // 4096
constexpr int UNIT_FIELDS = 5;
constexpr int UNIT_FLOATS = UNIT_FIELDS * UNIT_VOX;  // float32 colour record: 20480 floats = 80 KiB
constexpr int UNIT_FLOATS_C64 = 8 * UNIT_VOX;        // float64 colour record: tsdf, weight (f32) + r, g, b (f64) = 128 KiB

// counters[] slots
constexpr int C_UNUSED0 = 0;  // (was the per-frame path's touched count)
constexpr int C_UNITS = 1;     // units allocated
constexpr int C_OVERFLOW = 2;  // pool exhausted (units dropped)
constexpr int C_HASHERR = 3;   // hash full or key out of range
constexpr int C_BATCH_PAIRS = 4;  // (frame, unit) pairs of a batch: counters[4 + parity] (batches alternate, see k_batch_units)
constexpr int C_ORDER_HEAVY = 6;  // k_batch_units: work-list entries placed from the front (units seen by >= half the
constexpr int C_ORDER_LIGHT = 7;  // batch's frames) / from the back (the rest); the last workgroup zeroes both
constexpr int C_KMAX = 8;   // [8, 11): max over allocated units of key_a + KEY_BIAS + 1 (0: no unit yet)
constexpr int C_KNEG = 11;  // [11, 14): max over allocated units of KEY_BIAS - key_a + 1 (so min key_a = KEY_BIAS + 1 - it)
constexpr int C_UNITS_DONE = 14;  // k_batch_units: workgroups finished (the last one mails the counters, then zeroes it)
constexpr int N_COUNTERS = 16;

// stats[] slots (u64)
constexpr int S_UPDATES = 0;
constexpr int S_UNIT_INTEGRATIONS = 1;

struct TsdfDev {
    unsigned long long* hkeys;
    int* hvals;
    int* counters;
    unsigned long long* stats;
    int* unit_keys;
    float* vox;                 // unit pool: max_units records of unit_floats floats
    int unit_floats;            // record stride: UNIT_FLOATS (float32 colour / NoColor) or UNIT_FLOATS_C64
    int color64;                // 1: the record's colour planes are float64 (colour precision 64, RGB8 volumes)
    unsigned long long* fmask;  // per hash slot: frames of the current batch that touch the unit (bit f)
    int* bslots;                // hash slots touched by the current batch (first-touch order)
    void* work;                 // per touched slot of the batch: unit header (UnitWork, 32 B) for the integrate
    int hash_mask;
    int max_units;
    int shard_rank;   // spatial sharding of one volume over `shard_world` GPUs: this volume keeps only the units
    int shard_world;  // with owner(key) == shard_rank (<= 1: no sharding)
    int shard_shift;  // ownership granularity: blocks of 2^shift units per axis share an owner
    int shard_mode;   // SHARD_BLOCKS: hashed blocks of 2^shift units; SHARD_SECTORS: azimuth sectors around a centre
    int shard_cx2, shard_cy2;  // sector centre in half units (round(2 * centre / unit_length)) per axis
};
constexpr int SHARD_BLOCKS = 0;
constexpr int SHARD_SECTORS = 1;

// owner rank of a unit, a function of its key alone (exact on host and device: integers only).
// SHARD_BLOCKS: a hash of its block key (unit key >> shard_shift per axis), independent of the table's slot hash
// mix64(key), so a shard's keys still spread over all slots.  Blocks of units keep most marching-cubes neighbours on one
// rank (the border halo only crosses block faces) while still balancing the ranks' units.
// SHARD_SECTORS (round 6): the azimuth sector of the unit's centre around the scan centre (x, y).  A ring scan's frames
// each see a contiguous arc of the object, so a rank's units project into a fraction of every frame and its front end
// stages only those tiles (tools/shard_sector_model.py: 0.23 of the pixels at 8 ranks against 0.54 for blocks).  The
// sector is floor(N * pa / 4) of the pseudo-angle pa = quadrant + a / (a + b) in [0, 4), exact in int64 (the octants at
// N = 8 and the quadrants at N = 4 are the true 45 / 90 degree sectors); the centre point itself goes to sector 0.
__host__ __device__ inline int unit_sector(long long X, long long Y, int n) {
    if (X == 0 && Y == 0) return 0;
    long long a, b, q;
    if (X > 0 && Y >= 0) { q = 0; a = Y; b = X; }
    else if (X <= 0 && Y > 0) { q = 1; a = -X; b = Y; }
    else if (X < 0 && Y <= 0) { q = 2; a = -Y; b = -X; }
    else { q = 3; a = X; b = -Y; }
    return (int)(((q * (a + b) + a) * (long long)n) / (4 * (a + b)));
}
__host__ __device__ inline int unit_owner(const TsdfDev& d, int x, int y, int z) {
    if (d.shard_mode == SHARD_SECTORS)
        return unit_sector(2ll * x + 1 - d.shard_cx2, 2ll * y + 1 - d.shard_cy2, d.shard_world);
    const unsigned long long bk = pack_key(x >> d.shard_shift, y >> d.shard_shift, z >> d.shard_shift);
    return (int)((unsigned)(mix64(bk + 0x9E3779B97F4A7C15ull) >> 32) % (unsigned)d.shard_world);
}
__host__ __device__ inline bool unit_owned(const TsdfDev& d, unsigned long long key) {
    if (d.shard_world <= 1) return true;
    int x, y, z;
    unpack_key(key, x, y, z);
    if (d.shard_mode == SHARD_SECTORS) {  // unit_sector(...) == rank without the division: 4 r s <= N v < 4 (r + 1) s
        const long long X = 2ll * x + 1 - d.shard_cx2, Y = 2ll * y + 1 - d.shard_cy2;
        if (X == 0 && Y == 0) return d.shard_rank == 0;
        long long a, b, q;
        if (X > 0 && Y >= 0) { q = 0; a = Y; b = X; }
        else if (X <= 0 && Y > 0) { q = 1; a = -X; b = Y; }
        else if (X < 0 && Y <= 0) { q = 2; a = -Y; b = -X; }
        else { q = 3; a = X; b = -Y; }
        const long long s = a + b, v = (q * s + a) * (long long)d.shard_world;
        return v >= 4ll * d.shard_rank * s && v < 4ll * (d.shard_rank + 1) * s;
    }
    return unit_owner(d, x, y, z) == d.shard_rank;
}

// a newly allocated unit widens the volume's key bounds (read back with the counters: the sorted-unit order packs keys
// on their actual ranges without a bounds pass)
__device__ inline void note_unit_key(const TsdfDev& d, int x, int y, int z) {
    const int k[3] = {x, y, z};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        atomicMax(&d.counters[C_KMAX + a], k[a] + KEY_BIAS + 1);
        atomicMax(&d.counters[C_KNEG + a], KEY_BIAS - k[a] + 1);
    }
}

// a unit's record: tsdf plane, weight plane, then the colour planes r, g, b (4096 each, voxel vi = z*256 + x*16 + y)
// in float32 or, when the volume keeps colour at Open3D's precision, float64 (the record is then 128 KiB)
__host__ __device__ inline float* unit_base(const TsdfDev& d, int id) { return d.vox + (size_t)id * d.unit_floats; }
template <typename CT>
__device__ inline CT* color_base(const TsdfDev& d, int id) {
    return reinterpret_cast<CT*>(unit_base(d, id) + 2 * UNIT_VOX);
}

// Border voxels of a unit: every voxel with x == 0, y == 0 or z == 0 (3 * 256 - 3 * 16 + 1 = 721), the only
// voxels of a unit that marching cubes reads from its -x/-y/-z neighbours (the 17^3 tile of a unit is the unit plus
// the low faces of its +1 neighbours).  Order: increasing Open3D index x*256 + y*16 + z.
constexpr int BORDER_VOX = 721;
__host__ __device__ inline void border_voxel(int b, int& x, int& y, int& z) {
    if (b < 256) {
        x = 0, y = b >> 4, z = b & 15;
        return;
    }
    const int c = b - 256, r = c % 31;
    x = 1 + c / 31;
    if (r < 16) y = 0, z = r;
    else y = r - 15, z = 0;
}

constexpr int MAX_BATCH = 64;      // frames per fused launch (one bit each in fmask)
constexpr int OT_MAIL_WORDS = 64;  // capacity of the pinned host mailbox (4-B words per read-back, mail_words)
// sequence words of the kernels that mail on their own (mail_wait): the marching-cubes scans (words 62, 63: one per
// scan block) and the units kernel's counters (the last word of the second half)
constexpr int MAIL_SEQ_MC = OT_MAIL_WORDS - 2;
constexpr int MAIL_SEQ_UNITS = 2 * OT_MAIL_WORDS - 1;

// per-frame parameters of a batch (device resident)
struct BatchFrame {
    const uint16_t* depth16;  // raw depth (u16 path) or nullptr
    const float* depthf;      // caller's float depth (float path) or nullptr
    const uint8_t* color;     // caller's RGB8 or nullptr
    float2* dm;               // packed per-pixel (depth, ray multiplier) staged by k_batch_touch
    uint32_t* rgba;           // packed per-pixel colour r | g << 8 | b << 16 staged by k_batch_touch
    double pose[12];          // rows 0..2 of inverse(extrinsic) (stride unprojection, float64)
    float E[12];              // rows 0..2 of (float)extrinsic
    float es[3];              // column 2 of (float)extrinsic * voxel_length
    float scale;              // (float)depth_scale
    double trunc;             // depth_trunc
};

struct PendingFrame {
    const uint16_t* depth;  // u16 path (nullptr for the float path)
    const float* depthf;    // float path
    const uint8_t* color;
    ot_intrinsics intr;
    double extrinsic[16];
    double depth_scale, depth_trunc;
};

struct MeshBuffers {
    // the marching-cubes structure of the last extraction (per-unit cube bytes, triangle offsets, ...; mc.hip
    // mc_layout), kept with the volume so ComputeVertexNormals can walk each vertex's cubes instead of sorting corners
    void* ws = nullptr;
    size_t ws_bytes = 0;
    int64_t ws_units = 0;
    int64_t serial = 0;   // extraction count; the structure is valid for `serial` while `valid`
    bool valid = false;   // cleared by anything that changes the volume (integrate, reset, import)
    bool internal = false;  // the last extraction's mesh sits in v / c / t (else it was emitted to the caller)
    bool emitted = false;   // the merge keys vk / tk of the last extraction are written (by an emission)
    double* v = nullptr;
    double* c = nullptr;
    int32_t* t = nullptr;
    int4* vk = nullptr;     // per vertex: owner unit key (x, y, z) and edge bit (local voxel * 3 + axis)
    int* vown = nullptr;    // per vertex: owner unit id (the vertex-normal walk starts from it: no hash probe)
    int32_t* tk = nullptr;  // per triangle: its cube's unit key (x, y, z)
    int64_t nv = 0, nt = 0;
    int64_t cap_v = 0, cap_t = 0, cap_vk = 0, cap_tk = 0, cap_vown = 0;
};

}  // namespace ot

struct ot_tsdf {
    int device = 0;
    double voxel_length = 0.0, sdf_trunc = 0.0, unit_length = 0.0;
    int color_type = 1, stride = 4;
    bool color64 = false;  // colour state in float64 (Open3D's Vector3d) instead of float32
    int64_t max_units = 0;  // current pool capacity (grows: grow_pool)
    int64_t hash_cap = 0;
    ot::TsdfDev dev{};
    int frame_id = 0;
    bool imported = false;  // units imported since reset (arbitrary state: no reciprocal-table integrate)
    // multiplier image cache
    float* mult = nullptr;
    ot_intrinsics mult_intr{};
    bool mult_valid = false;
    // batching of integrate_u16: frames per fused launch (ot_tsdf_set_batch; 64 = MAX_BATCH, measured best, §4)
    int batch_max = ot::MAX_BATCH;
    std::vector<ot::PendingFrame> pending;
    ot::BatchFrame* hbframes = nullptr;    // pinned host staging [2][MAX_BATCH]
    unsigned* hmail = nullptr;             // pinned coherent host mailbox [OT_MAIL_WORDS]: small read-backs stored
                                           // by a one-wave kernel (mail_words) instead of staged D2H copies
    // staging half of the next batch; a batch's parameter copy has run once its units kernel has mailed (settle_batch
    // waits for that before integrate_batch returns), so the halves need no event
    int hb_next = 0;
    // the counters as the last batch's units kernel left them (the integrate does not change them), mailed by its last
    // workgroup to hmail + OT_MAIL_WORDS, then sequence number `units_seq` to word MAIL_SEQ_UNITS: the host spins on
    // that word (mail_wait) instead of an event behind the units kernel -- an event recorded between two kernels of a
    // stream idles the GPU ~4 us (tools/event_gap.hip, r05j) -- and an extraction reads the unit count without waiting
    // for the integrate (valid while early_frame == frame_id, no reset or import since)
    unsigned units_seq = 0;
    int early_frame = -1;
    unsigned mc_seq = 0;  // the marching-cubes totals' sequence number (words MAIL_SEQ_MC, MAIL_SEQ_MC + 1)
    int batch_pc = ot::C_BATCH_PAIRS;      // pair counter of the next batch (alternates 4, 5)
    // A batch's staging: per-frame parameters, packed (depth, multiplier) and colour per pixel, and the unit work list.
    // Two sets: with the front end double-buffered (overlap, ot_tsdf_set_frontend_overlap: off by default, measured slower
    // sharded volume, whose integrate is 1/N of the work) batch k+1's staging / touch / units run on the caller's stream
    // while batch k's integrate runs on `istream`; otherwise set 0 only, everything on the caller's stream.
    struct BatchSet {
        ot::BatchFrame* bframes = nullptr;  // device [MAX_BATCH]
        float2* bdm = nullptr;              // device [batch][h][w] packed (depth, multiplier)
        uint32_t* brgba = nullptr;          // device [batch][h][w] packed colour
        int64_t cap = 0;                    // pixels (frames * h * w) the two buffers hold
        void* work = nullptr;               // UnitWork [hash_cap]; set 0 uses dev.work
        hipEvent_t ev_units = nullptr;      // the set's units kernel (its integrate waits for it)
        hipEvent_t ev_done = nullptr;       // the set's integrate (the set's next front end waits for it)
    } bset[2];
    int overlap_mode = -1;        // -1 (default) and 0 off, 1 on
    // Split front end of a sharded volume (round 6): the touch stages nothing (only each stride sample's own pixel, for a
    // replay), k_stage_mask marks the image tiles the batch's owned units can project to, k_stage_tiles stages those.
    unsigned* tmask = nullptr;    // device [MAX_BATCH][tile rows][words per row]
    int64_t tmask_words = 0;
    int tmask_w = 0, tmask_h = 0;  // the image size the masks are laid out for
    int split_mode = -1;          // -1 (default): split for sharded volumes; 0 off; 1 on (test hook)
    // Deferred integrate of a sharded volume's last batch (round 6): its front end ran, its integrate waits to be launched
    // together with the next batch's touch (k_integrate_touch) or alone by the next flush.  dfr_ctx holds the batch's
    // context (tsdf.hip BatchCtx), dfr_stream the stream its front end ran on.
    bool dfr_on = false;
    hipStream_t dfr_stream = nullptr;
    hipEvent_t ev_dfr = nullptr;  // dfr_stream -> a flush on another stream
    alignas(16) unsigned char dfr_ctx[1024];
    // batch statistics since reset (ot_tsdf_batch_stats; the bench's compulsory-bytes figure): batches, units touched
    // summed over batches, units new in their batch; units the last batch left (-1: unknown after an import)
    int64_t stat_batches = 0, stat_unit_batches = 0, stat_fresh = 0, stat_prev_units = 0;
    int64_t last_batch_slots = -1;  // units the last batch touched (mailed): the next batch's integrate granularity
    int bset_next = 0;            // set of the next batch (alternates in overlap mode)
    int last_set = -1;            // set of the last batch whose integrate ran on istream (joined by readers)
    hipStream_t istream = nullptr;
    int* wcount = nullptr;        // device [2]: the sets' work-list lengths (k_batch_units -> k_batch_integrate)
    // sorted-unit cache (rank -> id), valid for `sorted_units` units
    unsigned* sorted_ids = nullptr;
    int64_t sorted_units = -1;
    int sorted_frame = -1;
    // extracted mesh
    ot::MeshBuffers mesh;
    // a second stream for independent extraction stages (vertex positions beside triangle indices), fork / join
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    // deferred vertex normals (ot_tsdf_mesh_vertex_normals on the caller's side stream) read the marching-cubes
    // structure (mesh.ws, vk, vown): work that rewrites it or the units waits for this event first (wait_normals)
    hipEvent_t ev_normals = nullptr;
    bool normals_pending = false;
    hipEvent_t ev_made = nullptr;  // ot_tsdf_extract_sample_min_z: the mesh arrays are complete (the normals wait on it)
    // kernel timing (events around the dominant integration kernel)
    bool profiling = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_events;
    double prof_ms = 0.0;
    int64_t prof_launches = 0;
    // and around each batch's front end (staging + touch + units), the part a sharded volume does not divide
    std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_fe_events;
    double prof_fe_ms = 0.0;
    int64_t prof_fe_batches = 0;
};

namespace ot {
// shared between tsdf.hip and mc.hip
ot_status tsdf_sorted_units(ot_tsdf* vol, hipStream_t stream, int64_t* n_units);
// small read-back: the 4-byte words at p[0 .. n) copied to vol->hmail by one kernel, then the stream synchronised
struct MailSrc {
    const unsigned* p[ot::OT_MAIL_WORDS];
    int n;
};
ot_status mail_words(ot_tsdf* vol, const MailSrc& s, hipStream_t stream);
// spin until a kernel on `stream` stores `seq` to the mailbox word (system-scope release after its mailed values); the
// stream is polled now and then, so a fault or a drained stream without the mail ends the wait with an error
ot_status mail_wait(const unsigned* word, unsigned seq, hipStream_t stream);
// integrate the queued frames; readers (join = true) also order `stream` after the last batch's integrate when it ran on
// the volume's integrate stream (double-buffered front end)
ot_status tsdf_flush(ot_tsdf* vol, hipStream_t stream, bool join = true);
// order `stream` after the volume's deferred vertex normals, if any are still in flight
ot_status wait_normals(ot_tsdf* vol, hipStream_t stream);
// the fused sampler's two phases (mesh_ops.hip): queue the chains + emission on `stream`, then wait for the kept counts.
// mark (nullable) is recorded on `stream` just before the area-sum walk (mark_at 1) or the CDF walk (mark_at 2)
ot_status sample_min_z_enqueue(const ot_mesh_sample_job* jobs, int32_t n_jobs, int64_t n_points, uint64_t seed,
                               double z_min, hipStream_t stream, hipStream_t* hs, hipEvent_t mark = nullptr,
                               int mark_at = 0);
ot_status sample_min_z_wait(hipStream_t hs, int32_t n_jobs, int64_t* n_kept_host);
}  // namespace ot
