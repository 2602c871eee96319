// tsdf.hip — ScalableTSDFVolume on MI355X: GPU block hash + block pool in HBM, batched touched-unit detection and
// temporally blocked integration.
//
// Reference semantics (Open3D ScalableTSDFVolume::Integrate and
// UniformTSDFVolume::IntegrateWithDepthToCameraDistanceMultiplier), called from
// reconstruct_rgbd_filter.py:105, reconstruct_rgbd.py:107, multi_reconstruct_rgbd_filter.py:98,
// reconstruct_rgbd_gt.py:82:
//   (i)   multiplier image m(i,j) = sqrtf(xx^2 + yy^2 + 1)                      (cached per intrinsic)
//   (ii)  stride-4 unprojection with camera_pose = inverse(extrinsic) in float64
//   (iii) touched units = union over samples of [floor((p - trunc)/L), floor((p + trunc)/L)]^3
//   (iv)  per touched unit, per voxel: project, sample depth, sdf update — all f32, z walked incrementally.
// Every flush is a batch of 1..64 frames (a single frame is a batch of one): k_batch_touch -> k_batch_units ->
// k_batch_integrate, below.  The unit pool is unbounded like Open3D's: when a batch needs more units than the pool
// holds, the pool and the hash grow (records copied, keys rehashed) and the batch's dropped units are integrated
// again from its staged frames (settle_batch), so the result is the one an unbounded pool gives.
#include <algorithm>
#include <cmath>
#include <sched.h>
#include <chrono>
#include <thread>
#include <cstring>
#include <type_traits>
#include <utility>

#include "compact.h"
#include "sort.h"
#include "tsdf.h"

namespace ot {

struct IntegrateParams {
    const float* depth;
    const uint8_t* color;
    const float* mult;
    int W, H;
    float fx, fy, cx, cy;
    float E[12];
    float es0, es1, es2;
    float vl, half, trunc, trunc_inv, safe_w, safe_h;
    float inv_fx, inv_fy;  // (float)(1 / (float)fx) as CreateDepthToCameraDistanceMultiplierFloatImage
    float proj_eps;  // certified fast projection: |u - rint(u)| > proj_eps decides floor and bounds exactly
    double unit_len;
};

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

// Raw buffer resource over [base, base + bytes): gfx9 dword3 (0x00020000, 32-bit raw data); loads past the end
// return 0 instead of faulting.
__device__ inline __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}

// element i of a float64 array behind a buffer resource (32-bit offsets: no per-lane 64-bit address registers)
__device__ inline double ld_f64(__amdgpu_buffer_rsrc_t r, int i) {
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, i * 8, 0, 0);
    return __hiloint2double((int)v.y, (int)v.x);
}
__device__ inline void st_f64(__amdgpu_buffer_rsrc_t r, int i, double x) {
    u32x2 v;
    v.x = (unsigned)__double2loint(x);
    v.y = (unsigned)__double2hiint(x);
    __builtin_amdgcn_raw_buffer_store_b64(v, r, i * 8, 0, 0);
}

__device__ inline int hash_insert(const TsdfDev& d, unsigned long long key) {
    unsigned slot = (unsigned)mix64(key) & (unsigned)d.hash_mask;
    for (int probe = 0; probe <= d.hash_mask; ++probe) {
        const unsigned long long k = d.hkeys[slot];
        if (k == key) return (int)slot;
        if (k == KEY_EMPTY) {
            const unsigned long long old = atomicCAS(&d.hkeys[slot], KEY_EMPTY, key);
            if (old == KEY_EMPTY || old == key) return (int)slot;
        }
        slot = (slot + 1) & (unsigned)d.hash_mask;
    }
    return -1;
}

__device__ inline int hash_find(const TsdfDev& d, unsigned long long key) {
    unsigned slot = (unsigned)mix64(key) & (unsigned)d.hash_mask;
    for (int probe = 0; probe <= d.hash_mask; ++probe) {
        const unsigned long long k = d.hkeys[slot];
        if (k == key) return (int)slot;
        if (k == KEY_EMPTY) return -1;
        slot = (slot + 1) & (unsigned)d.hash_mask;
    }
    return -1;
}

// ============================================================================ batched (temporal blocking)
// One launch per batch of F <= 64 frames:
//   staging           : per-pixel (depth, multiplier) float2 + packed colour for every frame, done by k_batch_touch's
//                       workgroups (each stages a contiguous pixel chunk of its frames)
//   k_batch_touch     : stride samples of every frame; a unit touched by frame f gets bit f in its slot's
//                       fmask (64-bit atomicOr); the first bit set in a batch appends the slot to bslots
//   k_batch_units     : per touched slot: allocate the unit if new, move its frame mask into a 32-B header
//   k_batch_integrate : persistent independent waves over (unit, slice) items: a slice's 64 x BZ voxels are
//                       loaded into registers (5 x BZ VGPRs/lane), the batch's frames are applied in call order
//                       (ascending bits of the mask) and the state is written back once.  Per-voxel arithmetic is
//                       the per-frame path's, so results are bit-identical to integrating frame by frame.
// Per-pixel staging of a batch: (depth, multiplier) as float2 and the colour as one u32, so the integrate
// kernel fetches a voxel's inputs with two aligned loads it can issue ahead of use.
// depth: u16 path converted exactly as Image::ConvertDepthToFloatImage; float path copied.
__device__ inline float prep_depth(const BatchFrame& fr, uint32_t raw16) {
    float dv = (float)raw16;
    dv = dv / fr.scale;
    if ((double)dv >= fr.trunc) dv = 0.0f;
    return dv;
}

// 4 pixels per lane: 8-B depth load, 12-B colour load (3 aligned dwords), 16-B multiplier load,
// 2 x 16-B (depth, multiplier) stores and one 16-B colour store.
__device__ inline void prep_quad(const BatchFrame& fr, const float* __restrict__ mult, int64_t i0, int64_t npx) {
    const bool aligned = ((reinterpret_cast<uintptr_t>(fr.depth16) & 7) == 0) &&
                         ((reinterpret_cast<uintptr_t>(fr.depthf) & 15) == 0) &&
                         ((reinterpret_cast<uintptr_t>(fr.color) & 3) == 0);
    if (aligned && i0 + 4 <= npx && (npx & 3) == 0) {
        float d[4];
        if (fr.depth16) {
            const uint2 raw = *reinterpret_cast<const uint2*>(fr.depth16 + i0);
            d[0] = prep_depth(fr, raw.x & 0xFFFFu);
            d[1] = prep_depth(fr, raw.x >> 16);
            d[2] = prep_depth(fr, raw.y & 0xFFFFu);
            d[3] = prep_depth(fr, raw.y >> 16);
        } else {
            const float4 v = *reinterpret_cast<const float4*>(fr.depthf + i0);
            d[0] = v.x, d[1] = v.y, d[2] = v.z, d[3] = v.w;
        }
        const float4 m = *reinterpret_cast<const float4*>(mult + i0);
        uint32_t w0 = 0u, w1 = 0u, w2 = 0u;  // colour loaded before the stores (char data may alias them)
        if (fr.color) {
            const uint32_t* c = reinterpret_cast<const uint32_t*>(fr.color + i0 * 3);  // 12 B, 4-B aligned
            w0 = c[0], w1 = c[1], w2 = c[2];
        }
        float4* dm = reinterpret_cast<float4*>(fr.dm + i0);
        dm[0] = make_float4(d[0], m.x, d[1], m.y);
        dm[1] = make_float4(d[2], m.z, d[3], m.w);
        if (fr.color) {
            // bytes: r0 g0 b0 r1 | g1 b1 r2 g2 | b2 r3 g3 b3
            const uint32_t p0 = w0 & 0xFFFFFFu;
            const uint32_t p1 = (w0 >> 24) | ((w1 & 0xFFFFu) << 8);
            const uint32_t p2 = (w1 >> 16) | ((w2 & 0xFFu) << 16);
            const uint32_t p3 = w2 >> 8;
            *reinterpret_cast<uint4*>(fr.rgba + i0) = make_uint4(p0, p1, p2, p3);
        }
    } else {
        for (int64_t i = i0; i < npx && i < i0 + 4; ++i) {
            const float dv = fr.depth16 ? prep_depth(fr, fr.depth16[i]) : fr.depthf[i];
            fr.dm[i] = make_float2(dv, mult[i]);
            if (fr.color) {
                const uint8_t* c = fr.color + i * 3;
                fr.rgba[i] = (uint32_t)c[0] | ((uint32_t)c[1] << 8) | ((uint32_t)c[2] << 16);
            }
        }
    }
}

// Quads [q, q1) with stride 256 (one lane's share of a chunk): on the common path (u16 depth, RGB8, aligned, W*H
// a multiple of 4) PREP_K quads per step with all of their loads issued before any store.
constexpr int PREP_K = 2;  // 3 or 4 (more VGPRs, fewer resident touch waves): step +2-3 %
__device__ inline void prep_range(const BatchFrame& fr, const float* __restrict__ mult, int64_t q, int64_t q1,
                                  int64_t npx) {
    const bool fast = fr.depth16 && fr.color && (npx & 3) == 0 &&
                      ((reinterpret_cast<uintptr_t>(fr.depth16) & 7) == 0) &&
                      ((reinterpret_cast<uintptr_t>(fr.color) & 3) == 0);
    if (fast) {
        for (; q + 256 * (PREP_K - 1) < q1; q += 256 * PREP_K) {
            uint2 raw[PREP_K];
            float4 m[PREP_K];
            uint32_t w[PREP_K][3];
#pragma unroll
            for (int k = 0; k < PREP_K; ++k) {
                const int64_t i0 = (q + 256 * k) * 4;
                raw[k] = *reinterpret_cast<const uint2*>(fr.depth16 + i0);
                m[k] = *reinterpret_cast<const float4*>(mult + i0);
                const uint32_t* c = reinterpret_cast<const uint32_t*>(fr.color + i0 * 3);
                w[k][0] = c[0], w[k][1] = c[1], w[k][2] = c[2];
            }
#pragma unroll
            for (int k = 0; k < PREP_K; ++k) {
                const int64_t i0 = (q + 256 * k) * 4;
                const float d0 = prep_depth(fr, raw[k].x & 0xFFFFu), d1 = prep_depth(fr, raw[k].x >> 16);
                const float d2 = prep_depth(fr, raw[k].y & 0xFFFFu), d3 = prep_depth(fr, raw[k].y >> 16);
                float4* dm = reinterpret_cast<float4*>(fr.dm + i0);
                dm[0] = make_float4(d0, m[k].x, d1, m[k].y);
                dm[1] = make_float4(d2, m[k].z, d3, m[k].w);
                const uint32_t p0 = w[k][0] & 0xFFFFFFu;
                const uint32_t p1 = (w[k][0] >> 24) | ((w[k][1] & 0xFFFFu) << 8);
                const uint32_t p2 = (w[k][1] >> 16) | ((w[k][2] & 0xFFu) << 16);
                const uint32_t p3 = w[k][2] >> 8;
                *reinterpret_cast<uint4*>(fr.rgba + i0) = make_uint4(p0, p1, p2, p3);
            }
        }
    }
    for (; q < q1; q += 256) prep_quad(fr, mult, q * 4, npx);
}

// The batch's per-frame parameters from the pinned host staging into device memory: one small kernel reading host
// memory instead of a copy command (the runtime's blit copy cost ~5 us of host API time and left the stream idle ~4 us
// behind it, on every batch's critical path: one object's timeline, r05m).  One 16-B word per lane, so every PCIe read
// is in flight at once (a 256-lane loop took 8.4 us: four round trips, r05n)
static_assert(sizeof(BatchFrame) % 16 == 0, "BatchFrame is copied in 16-B words");
constexpr int COPY_FRAMES_LANES = 1024;
static_assert(sizeof(BatchFrame) / 16 * MAX_BATCH <= COPY_FRAMES_LANES, "one word per lane");
__global__ __launch_bounds__(COPY_FRAMES_LANES) void k_copy_frames(const uint4* __restrict__ src,
                                                                   uint4* __restrict__ dst, int n16) {
    const int i = threadIdx.x;
    if (i < n16) dst[i] = src[i];
}

struct BatchTouchParams {
    int W, stride, ws, hs;
    double fx, fy, cx, cy;
    double trunc, unit_len;
    double inv_unit;    // RN(1 / unit_len): floor_div's certified product
    int slot_cap;
    const float* mult;  // fused staging (k_batch_touch stages the batch's pixels too): ray multipliers
    int64_t npx;        // pixels per frame
    int pc;             // this batch's pair counter index
    int tiles;          // touch workgroups per frame group (blockIdx.x below it)
    int stage_blocks;   // staging-only workgroups per frame group after them (0: each touch workgroup stages a share)
    int tf;             // frames per group (TF)
    int sample_stage;   // split front end (stage_blocks < 0): each stride sample stores its own pixel's staged pair
                        // (a replay touch reads it; k_stage_tiles stages only the owned units' footprints)
};

// floor(RN(a / b)) -- Open3D's LocateVolumeUnit on a float64 quotient -- with one multiply in the common case: v =
// RN(a * RN(1/b)) is within 2^-52 |a/b| of a/b (and RN(a/b) within 2^-53), so when v lies farther than 1e-14 |v| (+ an
// absolute floor far below any unit index) from every integer, floor(v) is floor(RN(a/b)); otherwise the IEEE division.
__device__ inline int floor_div(double a, double b, double inv_b) {
    const double v = a * inv_b;
    const double fv = floor(v);
    const double eps = 1e-14 * fabs(v) + 1e-300;
    if (v - fv > eps && (fv + 1.0) - v > eps) return (int)fv;
    return (int)floor(a / b);
}

__device__ inline void touch_unit_batch(const TsdfDev& d, int f, int slot_cap, int pc, int x, int y, int z) {
    if (!key_in_range(x, y, z)) {
        atomicOr(&d.counters[C_HASHERR], 2);
        return;
    }
    const unsigned long long key = pack_key(x, y, z);
    if (!unit_owned(d, key)) return;
    const int slot = hash_insert(d, key);
    if (slot < 0) {
        atomicOr(&d.counters[C_HASHERR], 1);
        return;
    }
    const unsigned long long bit = 1ull << f;
    if (d.fmask[slot] & bit) return;  // fast path; a stale read only costs the atomic below
    const unsigned long long old = atomicOr(&d.fmask[slot], bit);
    if (old == 0ull) {
        const int pos = atomicAdd(&d.counters[pc], 1);
        if (pos < slot_cap) d.bslots[pos] = slot;
        else atomicOr(&d.counters[C_HASHERR], 1);
    }
}

// Touch pass with LDS de-duplication.  A workgroup owns a 16x16 tile of stride samples and a group of TF frames;
// each (unit key, frame) hit is first merged into an LDS table (key -> frame bitmask, 64-bit LDS atomics), then
// every distinct unit of the tile does ONE global hash insert + ONE atomicOr of its merged mask.  A key that does
// not fit the LDS table falls back to the direct global path.
constexpr int TT = 16;          // tile edge in samples
// frames per workgroup: 2 since the staging-only workgroups (r05au / r05av, tools/touch_stage_ab.py: unsharded step
// within 0.2 % of 4, a rank of 8 shards 3 % faster -- front end 99 vs 105 us per batch; 8: +10 %); with every touch
// workgroup staging a share first, 4 was 1 % faster than 2 (round 3)
constexpr int TF = 2;
static int g_touch_tf = TF;  // test hook otx_touch_frames: frames per touch workgroup (A/B timing)
constexpr int LTAB = 1024;   // LDS table entries (16 B each + a 4-B slot in the list of used entries)

__device__ inline bool lds_merge(unsigned long long* keys, unsigned long long* masks, unsigned short* used, int* nused,
                                 unsigned long long key, unsigned long long bit) {
    unsigned h = (unsigned)mix64(key) & (LTAB - 1);
    for (int probe = 0; probe < 64; ++probe) {
        unsigned long long k = keys[h];
        if (k == KEY_EMPTY) {
            const unsigned long long old = atomicCAS(&keys[h], KEY_EMPTY, key);
            if (old == KEY_EMPTY) used[atomicAdd(nused, 1)] = (unsigned short)h;  // the inserting lane lists the entry
            k = (old == KEY_EMPTY) ? key : old;
        }
        if (k == key) {
            atomicOr(&masks[h], bit);
            return true;
        }
        h = (h + 1) & (LTAB - 1);
    }
    return false;
}

// staging share `part` of `parts` of the pixels of frame group `grp`
__device__ inline void stage_share(const BatchFrame* __restrict__ frames, const BatchTouchParams& p, int nframes,
                                   int grp, int part, int parts) {
    const int64_t quads = (p.npx + 3) >> 2;
    const int64_t per = (quads + parts - 1) / parts;
    const int64_t q0 = (int64_t)part * per, q1 = q0 + per < quads ? q0 + per : quads;
    for (int f = grp * p.tf; f < grp * p.tf + p.tf && f < nframes; ++f)
        prep_range(frames[f], p.mult, q0 + threadIdx.x, q1, p.npx);
}

// Staging (every pixel of the batch: HBM streaming) and the touch (stride samples: LDS merges and global hash atomics)
// as separate workgroups: stage_blocks > 0 staging-only workgroups follow each frame group's touch tiles in the grid
// (blockIdx.x >= tiles), so the touches' global atomics are spread over the time the staging streams.  Measured
// (tools/touch_stage_ab.py, front end per 64-frame batch): every touch workgroup staging a share first (stage_blocks 0,
// the round-4 form) 115 us, 1 / 2 / 4 / 8 staging workgroups per tile 120 / 111 / 112 / 122 us (r05aq, r05ar: step
// -1.2 % at 2); all touch workgroups dispatched first and the staging after them 123-128 us (r05as: the touches'
// atomics then contend at once).  The touch reads raw depth itself, so nothing in it waits on the staging stores.
// Every rank of a spatially sharded volume stages every pixel: integrating from the raw frames instead (a u16 depth +
// a multiplier-table gather per voxel visit) made the integrate 1.9x slower per unit (round 4,
// tools/shard_frontend.py), more than the staging it saves.
// REPLAY (settle_batch, after the pool grew): the batch's touch again from its STAGED depths (the caller's frames may be
// gone by then; the staged depth is exactly the value the first pass computed from them), no staging.
// LDS of one touch workgroup (k_batch_touch, and the touch half of k_integrate_touch)
struct TouchLds {
    unsigned long long keys[LTAB];
    unsigned long long masks[LTAB];
    unsigned short used[LTAB];  // 16-bit entry indices: 18 KiB in all, so 8 workgroups fit a CU's 160 KiB
    int nused;
};
// STAGE: the staging code paths (stage_blocks >= 0) are compiled in; the split front end's touch has none (the touch half
// of k_integrate_touch: without them it fits 64 VGPRs instead of 96)
template <bool REPLAY, bool STAGE = !REPLAY>
__device__ __forceinline__ void touch_body(const BatchFrame* __restrict__ frames, const BatchTouchParams& p,
                                           const TsdfDev& d, int nframes, TouchLds& L, int tile, int grp) {
    unsigned long long* s_keys = L.keys;
    unsigned long long* s_masks = L.masks;
    unsigned short* s_used = L.used;
    int& s_nused = L.nused;
    const int tid = threadIdx.x;
    if constexpr (STAGE) {
        if (p.stage_blocks > 0 && tile >= p.tiles) {  // block-uniform
            stage_share(frames, p, nframes, grp, tile - p.tiles, p.stage_blocks);
            return;
        }
    }
    for (int e = tid; e < LTAB; e += 256) {
        s_keys[e] = KEY_EMPTY;
        s_masks[e] = 0ull;
    }
    if (tid == 0) s_nused = 0;
    // (stage_blocks 0) this touch workgroup also stages a contiguous 1/tiles of its frames' pixels
    if constexpr (STAGE) {
        if (p.stage_blocks == 0) stage_share(frames, p, nframes, grp, tile, p.tiles);
    }
    __syncthreads();
    const int tiles_x = (p.ws + TT - 1) / TT;
    const int sx = (tile % tiles_x) * TT + (tid & (TT - 1));
    const int sy = (tile / tiles_x) * TT + (tid / TT);
    const int f0 = grp * p.tf;
    if (sx < p.ws && sy < p.hs) {
        const int r = sy * p.stride, c = sx * p.stride;
        for (int f = f0; f < f0 + p.tf && f < nframes; ++f) {
            const BatchFrame& fr = frames[f];
            const int64_t pix = (int64_t)r * p.W + c;  // the staged depth, computed as the staging does
            const float df = REPLAY ? fr.dm[pix].x : fr.depth16 ? prep_depth(fr, fr.depth16[pix]) : fr.depthf[pix];
            if constexpr (!REPLAY) {
                if (p.sample_stage) fr.dm[pix] = make_float2(df, p.mult[pix]);  // what the staging writes there
            }
            if (!(df > 0.0f)) continue;
            const double z = (double)df;
            const double x = ((double)c - p.cx) * z / p.fx;
            const double y = ((double)r - p.cy) * z / p.fy;
            double q[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const double a = fr.pose[k * 4 + 0] * x;
                const double b = fr.pose[k * 4 + 1] * y;
                const double cc = fr.pose[k * 4 + 2] * z;
                q[k] = ((a + b) + cc) + fr.pose[k * 4 + 3];
            }
            int lo[3], hi[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                lo[k] = floor_div(q[k] - p.trunc, p.unit_len, p.inv_unit);
                hi[k] = floor_div(q[k] + p.trunc, p.unit_len, p.inv_unit);
            }
            const unsigned long long bit = 1ull << f;
            for (int ux = lo[0]; ux <= hi[0]; ++ux)
                for (int uy = lo[1]; uy <= hi[1]; ++uy)
                    for (int uz = lo[2]; uz <= hi[2]; ++uz) {
                        if (!key_in_range(ux, uy, uz)) {
                            atomicOr(&d.counters[C_HASHERR], 2);
                            continue;
                        }
                        const unsigned long long key = pack_key(ux, uy, uz);
                        if (!unit_owned(d, key)) continue;
                        if (!lds_merge(s_keys, s_masks, s_used, &s_nused, key, bit)) touch_unit_batch(d, f, p.slot_cap, p.pc, ux, uy, uz);
                    }
        }
    }
    __syncthreads();
    // only the entries this tile filled (listed by their inserting lanes), not the whole table
    // The slots this batch touches first get a place in its list through ONE counter atomic per wave (ballot, the
    // first such lane adds the wave's count, each lane takes its rank): a batch's thousands of first touches on one
    // counter word no longer serialise in L2 one lane at a time
    const int nused = s_nused;
    for (int t0 = 0; t0 < nused; t0 += 256) {  // block-uniform trip count: every lane reaches the ballot
        const int t = t0 + tid;
        bool fresh = false;
        int slot = -1;
        if (t < nused) {
            const int e = s_used[t];
            slot = hash_insert(d, s_keys[e]);
            if (slot < 0) {
                atomicOr(&d.counters[C_HASHERR], 1);
            } else {
                // no read of the mask first: another frame group's workgroup set the unit's other bits, so the
                // bits are almost never all present, and the read was one more dependent global round trip on
                // every tile's chain (front end 112 -> 104 us per 64-frame batch, r05ax)
                fresh = atomicOr(&d.fmask[slot], s_masks[e]) == 0ull;
            }
        }
        int cnt;
        const int rank = wave_excl_count(fresh, cnt);
        if (cnt) {  // wave-uniform
            const int leader = __ffsll((long long)__ballot(fresh)) - 1;
            int base = 0;
            if ((int)lane_id() == leader) base = atomicAdd(&d.counters[p.pc], cnt);
            base = __builtin_amdgcn_readlane(base, leader);
            if (fresh) {
                const int pos = base + rank;
                if (pos < p.slot_cap) d.bslots[pos] = slot;
                else atomicOr(&d.counters[C_HASHERR], 1);
            }
        }
    }
}

template <bool REPLAY>
__global__ __launch_bounds__(256) void k_batch_touch(const BatchFrame* __restrict__ frames, BatchTouchParams p,
                                                     TsdfDev d, int nframes) {
    __shared__ TouchLds lds;
    touch_body<REPLAY>(frames, p, d, nframes, lds, (int)blockIdx.x, (int)blockIdx.y);
}
// the split front end's touch (no staging paths compiled in: 69 instead of 96 VGPRs)
__global__ __launch_bounds__(256) void k_batch_touch_split(const BatchFrame* __restrict__ frames, BatchTouchParams p,
                                                           TsdfDev d, int nframes) {
    __shared__ TouchLds lds;
    touch_body<false, false>(frames, p, d, nframes, lds, (int)blockIdx.x, (int)blockIdx.y);
}

// ------------------------------------------------------------------------------------------------ integrate
// Work item = (unit, slice): a slice is one wave of 64 (x, y) columns times BZ consecutive z, so a unit is
// SLICES = 4 * (16 / BZ) independent waves.  Lane (x, y) of slice (g, h) owns z in [BZ*h, BZ*h + BZ); its
// camera-space position still advances by exactly z sequential additions of Es.col(2) from the column origin,
// as in Open3D, so every slice reproduces the single-lane z walk bit for bit.  Waves never synchronise: the
// unit header (id, key, frame mask) is resolved once by k_batch_units and read with scalar loads.
constexpr int BZ = 4;                         // voxels per lane along z (2: slower, profiles/r03w_*)
constexpr int SLICES = 4 * (UNIT_RES / BZ);   // waves per unit
// waves per integrate workgroup: a quarter unit (measured per 32-frame launch, float64 colour: 16 waves 0.511 ms,
// 8 waves 0.452 ms, 4 waves 0.426 ms; float32 colour 0.402 / 0.383 / 0.378)
constexpr int INT_WG = 4;
constexpr int INT_PARTS = SLICES / INT_WG;  // workgroups per unit

struct UnitWork {
    int id;                   // pool id, | 0x80000000 when fresh (state starts at zero), -1 when dropped
    int kx, ky, kz;           // unit key
    unsigned long long mask;  // frames of the batch that touch the unit (bit f = frame f)
    unsigned long long pad;
};

// Unit headers of the batch: allocate new units, move and clear the frame masks (ready for the next batch).  A unit the
// pool cannot hold is dropped (id -1, C_OVERFLOW; not counted) and integrated by the replay once the pool has grown.
// REPLAY: units that already have an id were integrated by the batch's first pass: skipped (id -1, not counted).
constexpr int WORK_HEAVY_FRAMES = 32;
// a work-list position for each live lane: one atomic per wave and class (every lane of the wave calls it)
__device__ inline int work_slot(TsdfDev& d, int n, bool live, bool heavy) {
    int nh, nl;
    const int rh = wave_excl_count(live && heavy, nh), rl = wave_excl_count(live && !heavy, nl);
    int bh = 0, bl = 0;
    if (lane_id() == 0) {
        if (nh) bh = atomicAdd(&d.counters[C_ORDER_HEAVY], nh);
        if (nl) bl = atomicAdd(&d.counters[C_ORDER_LIGHT], nl);
    }
    bh = __builtin_amdgcn_readlane(bh, 0);
    bl = __builtin_amdgcn_readlane(bl, 0);
    return heavy ? bh + rh : n - 1 - (bl + rl);
}

template <bool REPLAY>
// wcount: where the integrate reads the batch's work-list length (the pair counter itself, or -- with the front end
// double-buffered -- a per-set copy, since the next batch's units kernel zeroes the other pair counter while this
// batch's integrate may still run)
// early_mail: hmail + OT_MAIL_WORDS; its last word (MAIL_SEQ_UNITS) receives `seq` once the counters are stored
__global__ __launch_bounds__(256) void k_batch_units(TsdfDev d, UnitWork* __restrict__ work, int pc,
                                                     unsigned* __restrict__ early_mail, int* __restrict__ wcount,
                                                     unsigned seq) {
    __shared__ unsigned long long red[4];
    const int n = d.counters[pc];
    // the other counter belongs to the next batch; the previous batch's integrate (its last reader) has finished
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        d.counters[pc ^ 1] = 0;
        if (wcount) *wcount = n;
    }
    // only the workgroups that have slots take part (a batch's few thousand units need a tenth of the grid): the rest
    // leave before the done ticket below, which the last of the active ones draws
    const int active = min((int)gridDim.x, max(1, (n + 255) / 256));
    if ((int)blockIdx.x >= active) return;  // block-uniform
    unsigned long long pairs = 0;
    // the new units' key bounds (note_unit_key's counters), reduced over the wave before its atomics: a fresh volume
    // allocates thousands of units in one batch, and one atomic per unit on six shared words serialised in L2
    int kmax[3] = {0, 0, 0}, kneg[3] = {0, 0, 0};  // 0: none (the counters hold k + KEY_BIAS + 1 >= 1)
    // block-uniform trip count, so every lane reaches the wave's one allocation atomic (ballot + rank, as the touch)
    for (int t0 = blockIdx.x * 256; t0 < n; t0 += gridDim.x * 256) {
        const int t = t0 + (int)threadIdx.x;
        const bool live = t < n;
        const int slot = live ? d.bslots[t] : 0;
        int id = live ? d.hvals[slot] : 0;
        // requested with the id, ahead of the allocation atomic (the compiler keeps loads behind an atomic)
        const unsigned long long mask = live ? d.fmask[slot] : 0ull;
        const unsigned long long hkey = live ? d.hkeys[slot] : 0ull;
        int cnt;
        const int rank = wave_excl_count(live && id < 0, cnt);
        if (cnt) {  // wave-uniform
            const int leader = __ffsll((long long)__ballot(live && id < 0)) - 1;
            int base = 0;
            if ((int)lane_id() == leader) base = atomicAdd(&d.counters[C_UNITS], cnt);
            base = __builtin_amdgcn_readlane(base, leader);
            if (live && id < 0) id = -2 - (base + rank);  // the new id, encoded below -1 until it is checked
        }
        // the entry's place in the work list.  A spatial shard's batch is ~1.5 rounds of resident workgroups, so its
        // heavy units (seen by >= WORK_HEAVY_FRAMES of the batch's frames) go to the front and the rest to the back:
        // the integrate's workgroups (dispatched in item order) start the long items first and the short ones fill
        // the tail (8 sector ranks: 174 -> 165 us per batch).  A whole volume keeps the touch's order, whose
        // neighbouring units share staged pixels in L2 (heavy-first there: 715 -> 734 us per batch)
        const int wpos = d.shard_world > 1 ? work_slot(d, n, live, __popcll(mask) >= WORK_HEAVY_FRAMES) : t;
        if (!live) continue;
        d.fmask[slot] = 0ull;
        int kx, ky, kz;
        unpack_key(hkey, kx, ky, kz);
        if (id <= -2) {
            id = -2 - id;
            if (id >= d.max_units) {
                atomicOr(&d.counters[C_OVERFLOW], 1);
                id = -1;
            } else {
                d.hvals[slot] = id;
                d.unit_keys[id * 3 + 0] = kx;
                d.unit_keys[id * 3 + 1] = ky;
                d.unit_keys[id * 3 + 2] = kz;
                const int k3[3] = {kx, ky, kz};
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    kmax[a] = max(kmax[a], k3[a] + KEY_BIAS + 1);
                    kneg[a] = max(kneg[a], KEY_BIAS - k3[a] + 1);
                }
                id |= (int)0x80000000u;
            }
        } else if (REPLAY) {
            id = -1;
        }
        UnitWork w;
        w.id = id;
        w.kx = kx;
        w.ky = ky;
        w.kz = kz;
        w.mask = mask;
        w.pad = 0ull;
        work[wpos] = w;
        if (id != -1) pairs += (unsigned long long)__popcll(mask);
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        kmax[a] = wave_max(kmax[a]);
        kneg[a] = wave_max(kneg[a]);
    }
    if (lane_id() == 0) {  // before this workgroup's done ticket below: the last workgroup mails the final bounds
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            if (kmax[a]) atomicMax(&d.counters[C_KMAX + a], kmax[a]);
            if (kneg[a]) atomicMax(&d.counters[C_KNEG + a], kneg[a]);
        }
    }
    pairs = wave_sum(pairs);
    if (lane_id() == 0) red[threadIdx.x >> 6] = pairs;
    __syncthreads();
    __shared__ int s_last;
    if (threadIdx.x == 0) {
        const unsigned long long tot = red[0] + red[1] + red[2] + red[3];
        if (tot) atomicAdd(&d.stats[S_UNIT_INTEGRATIONS], tot);
        __threadfence();
        s_last = atomicAdd(&d.counters[C_UNITS_DONE], 1) == active - 1;
    }
    __syncthreads();
    if (s_last && threadIdx.x < 64) {  // every workgroup's counter atomics are done: wave 0 mails the final values
        if (threadIdx.x < N_COUNTERS) {
            const int v = __hip_atomic_load(&d.counters[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            early_mail[threadIdx.x] = threadIdx.x == C_UNITS_DONE ? 0u : (unsigned)v;
            // the heavy units' count (the list's front; the light ones fill the back in reverse touch order, which
            // integrate_body reads forward again) next to the length the integrate reads
            if (threadIdx.x == C_ORDER_HEAVY && wcount) wcount[2] = d.shard_world > 1 ? v : n;
            if (threadIdx.x == C_UNITS_DONE || threadIdx.x == C_ORDER_HEAVY || threadIdx.x == C_ORDER_LIGHT)
                d.counters[threadIdx.x] = 0;
        }
        __threadfence_system();  // the values reach the host before the sequence word
        if (threadIdx.x == 0)
            __hip_atomic_store(early_mail + (MAIL_SEQ_UNITS - OT_MAIL_WORDS), seq, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ------------------------------------------------------------------------------------ split front end (sharded)
// A rank of a spatially sharded volume integrates only its own units, so it reads only the pixels those units project
// to.  With sector ownership (tsdf.h unit_owner) that is a fraction of every frame (tools/shard_sector_model.py, the
// configs[1] ring scan: 0.23 of the 32x16 tiles at 8 ranks; 0.54 with hashed blocks), so the front end splits:
// touch (no staging) -> units -> k_stage_mask (the tiles each (owned unit, frame) pair can project to) -> k_stage_tiles
// (only those tiles).  The staged values are a pure function of the pixel, so staging a superset changes no bit.
constexpr int STX = 32, STY = 16;  // staging tile: 32 pixels (one 8-lane group of quads per row) x 16 rows
struct StageMaskParams {
    int W, H, tiles_x, tiles_y, wpr;  // wpr: 32-bit mask words per tile row
    float fx, fy, cx, cy, vl, half;
    double unit_len;
    int nframes;
};
// Footprint of a unit in a frame: the voxel centres span the box [p(0), p(15)] per axis (the integrate's own float
// expressions for x, y = 0 and 15; z from the unit origin by 15 voxel lengths), so in exact arithmetic their projections
// lie in the projected corners' bounding box (the box is in front of the camera).  The integrate's float projection of a
// voxel differs from the exact one by < 0.02 px here (|pc| error ~6e-6 m at z >= 0.05 m); the box is widened by 2 px
// and any corner nearer than 5 cm marks the whole frame.
// One workgroup per FRAME: its threads walk the batch's work list, each unit whose frame mask has this frame's bit ORs
// its footprint's tiles into the frame's map in LDS, and the map is stored whole -- no global atomics (one per (unit,
// frame, tile row) had contended on the frames' few words: 8-18 us per batch, r06e), nothing to clear between batches.
// SM_PARTS workgroups per frame, each over every SM_PARTS-th 256-unit chunk of the list into its own map (64 workgroups
// for a 64-frame batch had left the mask kernel latency-bound: 5-8 us per batch, r06st); the staging kernel ORs them.
constexpr int SM_WORDS = 2048;  // LDS map words: tile rows * words per row (8 KiB; 16K x 16K-pixel frames)
constexpr int SM_PARTS = 4;
__global__ __launch_bounds__(256) void k_stage_mask(const BatchFrame* __restrict__ frames, StageMaskParams q,
                                                    const UnitWork* __restrict__ work, const int* __restrict__ wcount,
                                                    unsigned* __restrict__ mask) {
    __shared__ unsigned s_map[SM_WORDS];
    const int f = blockIdx.x, part = blockIdx.y;
    const int words = q.tiles_y * q.wpr;
    for (int i = threadIdx.x; i < words; i += 256) s_map[i] = 0u;
    __syncthreads();
    const int n = *wcount;
    const BatchFrame& fr = frames[f];
    for (int u = part * 256 + threadIdx.x; u < n; u += 256 * SM_PARTS) {
        const UnitWork& w = work[u];
        if (!((w.mask >> f) & 1ull)) continue;
        const float ox = (float)((double)w.kx * q.unit_len);
        const float oy = (float)((double)w.ky * q.unit_len);
        const float oz = (float)((double)w.kz * q.unit_len);
        const double xs[2] = {(double)((q.half + q.vl * 0.0f) + ox), (double)((q.half + q.vl * 15.0f) + ox)};
        const double ys[2] = {(double)((q.half + q.vl * 0.0f) + oy), (double)((q.half + q.vl * 15.0f) + oy)};
        const double zs[2] = {(double)(q.half + oz), (double)(q.half + oz) + 15.0 * (double)q.vl};
        bool full = false;
        double umin = 1e300, umax = -1e300, vmin = 1e300, vmax = -1e300;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const double px = xs[c & 1], py = ys[(c >> 1) & 1], pz = zs[c >> 2];
            double pc[3];
#pragma unroll
            for (int r = 0; r < 3; ++r)
                pc[r] = (double)fr.E[r * 4 + 0] * px + (double)fr.E[r * 4 + 1] * py + (double)fr.E[r * 4 + 2] * pz +
                        (double)fr.E[r * 4 + 3];
            if (!(pc[2] >= 0.05)) {
                full = true;
            } else {
                const double rz = 1.0 / pc[2];
                const double uf = (double)q.fx * pc[0] * rz + (double)q.cx + 0.5;
                const double vf = (double)q.fy * pc[1] * rz + (double)q.cy + 0.5;
                umin = fmin(umin, uf), umax = fmax(umax, uf), vmin = fmin(vmin, vf), vmax = fmax(vmax, vf);
            }
        }
        int u0 = 0, u1 = q.W - 1, v0 = 0, v1 = q.H - 1;
        if (!full) {
            if (umax < -2.0 || vmax < -2.0 || umin > (double)q.W + 2.0 || vmin > (double)q.H + 2.0) continue;
            u0 = max(0, (int)floor(umin) - 2), u1 = min(q.W - 1, (int)floor(umax) + 2);
            v0 = max(0, (int)floor(vmin) - 2), v1 = min(q.H - 1, (int)floor(vmax) + 2);
            if (u0 > u1 || v0 > v1) continue;
        }
        const int tx0 = u0 / STX, tx1 = u1 / STX, ty0 = v0 / STY, ty1 = v1 / STY;
        for (int ty = ty0; ty <= ty1; ++ty)
            for (int k = tx0 >> 5; k <= (tx1 >> 5); ++k) {
                const int a = max(tx0, k * 32) - k * 32, b = min(tx1, k * 32 + 31) - k * 32;  // bits [a, b]
                const unsigned bits = (b == 31 ? ~0u : ((1u << (b + 1)) - 1u)) & ~((1u << a) - 1u);
                atomicOr(&s_map[ty * q.wpr + k], bits);
            }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < words; i += 256) mask[((size_t)f * SM_PARTS + part) * words + i] = s_map[i];
}

// Stage the marked tiles: one workgroup per (tile row, frame); its lanes take the marked tiles' quads in turn (a row of
// a 32-pixel tile is 8 quads, 9 slots when W % 4 != 0 lets a quad straddle the tile edge), so the work of a sparse row is
// spread over all 256 lanes (one wave per tile left 77 % of the waves idle: 23 us per batch, r06e).  A quad staged
// twice writes the same bytes.
constexpr int ST_MAX_TILES_X = 256;
constexpr int ST_K = 4;  // quads per lane per step on the common path
__global__ __launch_bounds__(256) void k_stage_tiles(const BatchFrame* __restrict__ frames, const float* __restrict__ mult,
                                                     const unsigned* __restrict__ mask, int W, int H, int tiles_x,
                                                     int tiles_y, int wpr, int64_t npx) {
    __shared__ int s_tx[ST_MAX_TILES_X];
    __shared__ int s_m;
    const int ty = blockIdx.x, f = blockIdx.y;
    if (threadIdx.x == 0) s_m = 0;
    __syncthreads();
    const size_t words = (size_t)tiles_y * wpr;
    const unsigned* row = mask + (size_t)f * SM_PARTS * words + (size_t)ty * wpr;
    for (int tx = threadIdx.x; tx < tiles_x; tx += 256) {
        unsigned w = 0u;
#pragma unroll
        for (int part = 0; part < SM_PARTS; ++part) w |= row[part * words + (tx >> 5)];
        if ((w >> (tx & 31)) & 1u) s_tx[atomicAdd(&s_m, 1)] = tx;
    }
    __syncthreads();
    const int m = s_m;
    if (m == 0) return;
    const int y0 = ty * STY, rows = min(H, y0 + STY) - y0;
    const int slots = (W & 3) ? STX / 4 + 1 : STX / 4;
    const int per_tile = rows * slots;
    const BatchFrame& fr = frames[f];
    const bool fast = fr.depth16 && fr.color && (npx & 3) == 0 && (W & 3) == 0 &&
                      ((reinterpret_cast<uintptr_t>(fr.depth16) & 7) == 0) &&
                      ((reinterpret_cast<uintptr_t>(fr.color) & 3) == 0);
    if (fast) {  // (u16 depth, RGB8, W % 4 == 0: every slot is a whole quad) a lane's ST_K quads' loads before any store
        const int total = m * per_tile;
        for (int i0 = threadIdx.x; i0 < total; i0 += 256 * ST_K) {
            int64_t px[ST_K];
            uint2 raw[ST_K];
            float4 mv[ST_K];
            uint32_t w[ST_K][3];
#pragma unroll
            for (int k = 0; k < ST_K; ++k) {
                const int i = i0 + 256 * k;
                px[k] = -1;
                const int t = i / per_tile, rem = i - t * per_tile;
                const int r = y0 + rem / slots, x = s_tx[min(t, m - 1)] * STX + (rem - (rem / slots) * slots) * 4;
                if (i < total && x < W) {  // (the frame's last tile column may be narrower than STX)
                    px[k] = (int64_t)r * W + x;
                    raw[k] = *reinterpret_cast<const uint2*>(fr.depth16 + px[k]);
                    mv[k] = *reinterpret_cast<const float4*>(mult + px[k]);
                    const uint32_t* c = reinterpret_cast<const uint32_t*>(fr.color + px[k] * 3);
                    w[k][0] = c[0], w[k][1] = c[1], w[k][2] = c[2];
                }
            }
#pragma unroll
            for (int k = 0; k < ST_K; ++k) {
                if (px[k] < 0) continue;
                const float d0 = prep_depth(fr, raw[k].x & 0xFFFFu), d1 = prep_depth(fr, raw[k].x >> 16);
                const float d2 = prep_depth(fr, raw[k].y & 0xFFFFu), d3 = prep_depth(fr, raw[k].y >> 16);
                float4* dm = reinterpret_cast<float4*>(fr.dm + px[k]);
                dm[0] = make_float4(d0, mv[k].x, d1, mv[k].y);
                dm[1] = make_float4(d2, mv[k].z, d3, mv[k].w);
                const uint32_t p0 = w[k][0] & 0xFFFFFFu;
                const uint32_t p1 = (w[k][0] >> 24) | ((w[k][1] & 0xFFFFu) << 8);
                const uint32_t p2 = (w[k][1] >> 16) | ((w[k][2] & 0xFFu) << 16);
                const uint32_t p3 = w[k][2] >> 8;
                *reinterpret_cast<uint4*>(fr.rgba + px[k]) = make_uint4(p0, p1, p2, p3);
            }
        }
        return;
    }
    for (int i = threadIdx.x; i < m * per_tile; i += 256) {
        const int t = i / per_tile, rem = i - t * per_tile;
        const int r = y0 + rem / slots, kq = rem - (rem / slots) * slots;
        const int x0 = s_tx[t] * STX, x1 = min(W, x0 + STX);
        const int64_t qa = ((int64_t)r * W + x0) >> 2, qb = ((int64_t)r * W + x1 - 1) >> 2;
        if (qa + kq <= qb) prep_quad(fr, mult, (qa + kq) * 4, npx);
    }
}

// compile-time loops over slot indices (std::integral_constant arguments): f(0), ..., f(N - 1); static_all stops at the
// first false
template <int N, class F>
__device__ __forceinline__ void static_for(F& f) {
    if constexpr (N > 0) {
        static_for<N - 1>(f);
        f(std::integral_constant<int, N - 1>{});
    }
}
template <int N, class F>
__device__ __forceinline__ bool static_all(F& f) {
    if constexpr (N == 0) {
        return true;
    } else {
        if (!static_all<N - 1>(f)) return false;
        return f(std::integral_constant<int, N - 1>{});
    }
}

// Phases A and B of one frame for a lane's ZB voxels: the certified projections and the depth gathers (no voxel state
// read) -- the fine slices' frame skew issues them for frame f+1 before frame f's updates (k_batch_integrate).  The same
// arithmetic as the phases inside the coarse loop.
template <int ZB>
__device__ __forceinline__ void frame_tap(const BatchFrame& fr, const IntegrateParams& p, int npx, float px, float py,
                                          float pz, int z0, int (&pixv)[ZB], float (&pcz)[ZB], float (&dv)[ZB],
                                          float (&mv)[ZB]) {
    const __amdgpu_buffer_rsrc_t dm_rsrc = make_rsrc(fr.dm, npx * 8);
    float pc[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const float a = fr.E[r * 4 + 0] * px;
        const float b = fr.E[r * 4 + 1] * py;
        const float c = fr.E[r * 4 + 2] * pz;
        pc[r] = ((a + b) + c) + fr.E[r * 4 + 3];
    }
    const float es0 = fr.es[0], es1 = fr.es[1], es2 = fr.es[2];
    for (int k = 0; k < z0; ++k) {  // wave-uniform: advance to this slice's first voxel
        pc[0] += es0;
        pc[1] += es1;
        pc[2] += es2;
    }
#pragma unroll
    for (int k = 0; k < ZB; ++k) {
        const float nu = pc[0] * p.fx, nv = pc[1] * p.fy;
        const float rz = __builtin_amdgcn_rcpf(pc[2]);
        float u_f = (nu * rz + p.cx) + 0.5f;
        float v_f = (nv * rz + p.cy) + 0.5f;
        const bool sure = !(pc[2] > 0.0f) || ((int)(fabsf(u_f - __builtin_rintf(u_f)) > p.proj_eps) &
                                              (int)(fabsf(v_f - __builtin_rintf(v_f)) > p.proj_eps));
        if (!sure) {
            u_f = ((nu / pc[2]) + p.cx) + 0.5f;
            v_f = ((nv / pc[2]) + p.cy) + 0.5f;
        }
        const bool ok = (pc[2] > 0.0f) & (u_f >= 0.0001f) & (u_f < p.safe_w) & (v_f >= 0.0001f) & (v_f < p.safe_h);
        pixv[k] = ok ? (int)__umul24((unsigned)(int)v_f, (unsigned)p.W) + (int)u_f : -1;
        pcz[k] = pc[2];
        pc[0] += es0;
        pc[1] += es1;
        pc[2] += es2;
    }
#pragma unroll
    for (int k = 0; k < ZB; ++k) {
        dv[k] = mv[k] = 0.0f;
        if (pixv[k] >= 0) {
            const u32x2 raw = __builtin_amdgcn_raw_buffer_load_b64(dm_rsrc, pixv[k] * 8, 0, 0);
            dv[k] = __uint_as_float(raw.x);
            mv[k] = __uint_as_float(raw.y);
        }
    }
}

// Occupancy: the integrate lives on it: 64 VGPRs, 8 waves per SIMD for both colour precisions with
// quarter-unit workgroups (float64 colour at 5 / 6 / 8 waves: 0.426 / 0.428 / 0.414 ms per 32-frame launch; the IEEE-
// division float64 kernel needs more registers and runs at 5).  Measured and settled: lanes whose voxel
// projects outside the image issue no depth gather (0.415-0.421 -> 0.409-0.412 ms); slices with no update in the
// batch are not written back (-1.5 %).
constexpr int INT_WAVES_PER_EU = 8;
// Reciprocal table: y[n] = RN(1/n) for n in [1, RCP_N].  For b = w + 1 an integer in that range, q0 = RN(a*y),
// r = fma(-b, q0, a) (exact), q = RN(q0 + r*y) is RN(a/b) -- Markstein's theorem (y correctly rounded, q0 within one
// ulp, no underflow in r; binary32 and binary64 alike): the IEEE quotient bit for bit with 3 operations and an LDS
// load instead of the ~10-instruction division sequence.  The host takes this kernel (FAST) only while every weight
// is an integer count of updates below RCP_N (frames since reset + the batch < RCP_N) and the state comes from
// integration alone (no imported units): then |a| is 0 or far above the underflow range (tsdf: a sum of a running
// mean and a term quantised by the depth / camera-distance floats; colour: c*w + rgb >= 0 with c a mean of bytes).
// Otherwise the IEEE divisions (FAST = false: tests/test_gpu_tsdf.py::test_long_scan_crosses_reciprocal_table and
// ::test_ieee_division_kernel_after_import run both across the switch).
constexpr int RCP_N = 2048;  // 16 KiB (float64) / 8 KiB (float32) of LDS per workgroup: 8 quarter-unit workgroups per CU

// One workgroup of INT_WG waves per unit part (a quarter unit by default: small workgroups let the CU keep 6-8 of them
// resident instead of one 16-wave unit -- a unit-sized workgroup left the float64-colour kernel at 4 waves per SIMD
// whatever its registers); the parts of a unit run on one XCD.  Work items are assigned by a static grid stride that
// every wave derives on its own: no atomics, one barrier (the reciprocal table).
// C64: colour state in float64 (Open3D's TSDFVoxel::color_ is Eigen::Vector3d), in the record's float64 planes.
// one table per kernel: float64 reciprocals for the float64-colour kernel (its float32 ones are their roundings:
// (float)RN64(1/n) == RN32(1/n) for every n <= 2^20, no double-rounding case -- tools/markstein_check.cpp), float32
// ones otherwise
template <bool C64, bool FAST>
struct RcpLds {
    float r32[(FAST && !C64) ? RCP_N + 1 : 1];
    double r64[(FAST && C64) ? RCP_N + 1 : 1];
};
// the integrate of a batch as workgroup `bid` of `nblk` (k_batch_integrate; the integrate half of k_integrate_touch)
template <bool C64, bool FAST, int ZB, int KT>
__device__ __forceinline__ void integrate_body(const BatchFrame* __restrict__ frames, const IntegrateParams& p,
                                               const TsdfDev& d, const UnitWork* __restrict__ work,
                                               const int* __restrict__ wcount, RcpLds<C64, FAST>& R, int bid, int nblk) {
    using CT = typename std::conditional<C64, double, float>::type;
    constexpr int PARTS = 4 * (UNIT_RES / ZB) / INT_WG;  // workgroups per unit (INT_PARTS at the default ZB)
    float* s_r32 = R.r32;
    double* s_r64 = R.r64;
    // work item = (unit, part): the PARTS parts of a unit are items 8 apart, so they run on one XCD (blocks are dealt
    // round-robin over the 8 XCDs) at about the same time and share its L2's copy of the footprint.
    // The grid is sized for large batches (8x the resident workgroups): a workgroup without an item leaves before
    // building the reciprocal table -- for a batch of few units (a spatial shard) the idle workgroups' tables had cost
    // more than the integrate itself (r05e: a 1/8 shard's 64-frame batch 165-200 us whatever its slicing)
    {
        const int n0 = __builtin_amdgcn_readfirstlane(__hip_atomic_load(wcount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (bid >= (PARTS == 1 ? n0 : ((n0 + 7) / 8) * 8 * PARTS)) return;
    }
    if constexpr (FAST) {
        for (int r = threadIdx.x; r <= RCP_N; r += 64 * INT_WG) {
            if constexpr (C64) s_r64[r] = 1.0 / (double)r;  // IEEE (correctly rounded) quotients
            else s_r32[r] = 1.0f / (float)r;
        }
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int n = *wcount;
    const int nh = wcount[2];  // heavy units first; the rest are stored back to front (k_batch_units)
    const int npx = p.W * p.H;
    unsigned upd = 0;  // per lane: <= ZB voxels x 64 frames x units per workgroup, far below 2^32
    {
        const int b = bid;
        const int items = PARTS == 1 ? n : ((n + 7) / 8) * 8 * PARTS;
        for (int it = b; it < items; it += nblk) {
            const int u = PARTS == 1 ? it : (it / (8 * PARTS)) * 8 + (it & 7);
            if (PARTS > 1 && u >= n) continue;
            const int part = PARTS == 1 ? 0 : (it >> 3) % PARTS;
            const int s = __builtin_amdgcn_readfirstlane(part * INT_WG + (int)(threadIdx.x >> 6));  // slice of this wave
            const UnitWork& w = work[u < nh ? u : n - 1 - (u - nh)];
            const int ent = w.id;
            const unsigned long long mask = w.mask;
            if (ent != -1) {
                const int id = ent & 0x7FFFFFFF;
                const bool fresh = ent < 0;
                // wave = 8 x 8 columns: a square patch of the unit's xy plane projects to fewer pixel rows
                const int x = (s & 2) * 4 + (lane >> 3), y = (s & 1) * 8 + (lane & 7);
                const int col = x * 16 + y;
                const int z0 = (s >> 2) * ZB;
                float* base = d.vox + (size_t)id * (C64 ? UNIT_FLOATS_C64 : UNIT_FLOATS);
                // colour plane c of voxel vi: float32 planes addressed from base (one address register for the
                // whole record: a separate colour pointer costs ~34 VGPRs in this kernel), float64 through a buffer
                // resource over the record's float64 planes
                const __amdgpu_buffer_rsrc_t col64 = make_rsrc(base + 2 * UNIT_VOX, 3 * UNIT_VOX * 8);
                float ts[ZB], wt[ZB];
                CT cr[ZB], cg[ZB], cb[ZB];
#pragma unroll
                for (int k = 0; k < ZB; ++k) {
                    const int vi = (z0 + k) * 256 + col;
                    if (fresh) {
                        ts[k] = wt[k] = 0.0f;
                        cr[k] = cg[k] = cb[k] = (CT)0;
                    } else {
                        ts[k] = base[vi];
                        wt[k] = base[UNIT_VOX + vi];
                        if constexpr (C64) {
                            cr[k] = ld_f64(col64, vi);
                            cg[k] = ld_f64(col64, UNIT_VOX + vi);
                            cb[k] = ld_f64(col64, 2 * UNIT_VOX + vi);
                        } else {
                            cr[k] = base[2 * UNIT_VOX + vi];
                            cg[k] = base[3 * UNIT_VOX + vi];
                            cb[k] = base[4 * UNIT_VOX + vi];
                        }
                    }
                }
                const float ox = (float)((double)w.kx * p.unit_len);
                const float oy = (float)((double)w.ky * p.unit_len);
                const float oz = (float)((double)w.kz * p.unit_len);
                const float px = (p.half + p.vl * (float)x) + ox;
                const float py = (p.half + p.vl * (float)y) + oy;
                const float pz = p.half + oz;
                const unsigned upd0 = upd;
                if constexpr (ZB == 2) {
                    // Frame pipeline (the fine slices serve batches with few units, whose waves cannot hide a frame's
                    // dependent gathers behind other waves: the wave's chain of frames IS the batch's time).  Every
                    // load of a frame is state-independent -- the projections and depth gathers (tap), the depth test,
                    // clamped tsdf term and colour gather (stage C) -- only the running means (stage D) read the
                    // voxel state.  So frame f+KT's tap and frame f+KC's stage C are issued before frame f's update,
                    // from KT + 1 register slots (the loop is unrolled over the slots so every slot is a fixed
                    // register set: a rotating copy would wait for the loads in flight).  The updates still run in
                    // frame order with the same arithmetic: the bits are the unpipelined loop's.  KT = 1, KC = 0 is the
                    // round-5 one-frame skew.
                    constexpr int KC = KT - 1, RS = KT + 1;
                    unsigned long long mt = mask;  // frames not yet tapped
                    int fs[RS];                     // frame of each slot (wave-uniform), -1: past the last frame
                    int pixv[RS][ZB];
                    float pcz[RS][ZB], dv[RS][ZB], mv[RS][ZB], tnv[RS][ZB];
                    uint32_t cv[RS][ZB];
                    bool dov[RS][ZB];
                    auto tap = [&](auto J) __attribute__((always_inline)) {
                        constexpr int j = decltype(J)::value;
                        if (mt) {
                            const int f = __ffsll((long long)mt) - 1;
                            mt &= mt - 1;
                            fs[j] = f;
                            frame_tap<ZB>(frames[f], p, npx, px, py, pz, z0, pixv[j], pcz[j], dv[j], mv[j]);
                        } else {
                            fs[j] = -1;
                        }
                    };
                    auto stage_c = [&](auto J) __attribute__((always_inline)) {
                        constexpr int j = decltype(J)::value;
                        if (fs[j] < 0) return;
                        const BatchFrame& fr = frames[fs[j]];
                        const __amdgpu_buffer_rsrc_t rgba_rsrc = make_rsrc(fr.rgba, npx * 4);
                        const bool use_color = fr.color != nullptr;
#pragma unroll
                        for (int k = 0; k < ZB; ++k) {
                            const float sdf = (dv[j][k] - pcz[j][k]) * mv[j][k];
                            dov[j][k] = (pixv[j][k] >= 0) & (dv[j][k] > 0.0f) & (sdf > -p.trunc);
                            const float sv = sdf * p.trunc_inv;
                            tnv[j][k] = (sv < 1.0f) ? sv : 1.0f;
                            cv[j][k] = 0u;
                            if (use_color && dov[j][k])
                                cv[j][k] = __builtin_amdgcn_raw_buffer_load_b32(rgba_rsrc, pixv[j][k] * 4, 0, 0);
                        }
                    };
                    auto stage_d = [&](auto J) __attribute__((always_inline)) -> bool {
                        constexpr int j = decltype(J)::value;
                        if (fs[j] < 0) return false;
                        const bool use_color = frames[fs[j]].color != nullptr;
#pragma unroll
                        for (int k = 0; k < ZB; ++k) {
                            const bool doit = dov[j][k];
                            const float tn = tnv[j][k];
                            const float wv = wt[k];
                            const float w1 = wv + 1.0f;
                            const float ta = ts[k] * wv + tn;
                            float tsn;
                            const double y64 = (FAST && C64) ? s_r64[(int)w1] : 0.0;
                            if constexpr (FAST) {
                                const float y = C64 ? (float)y64 : s_r32[(int)w1];
                                const float q0 = ta * y;
                                tsn = __builtin_fmaf(__builtin_fmaf(-w1, q0, ta), y, q0);
                            } else {
                                tsn = ta / w1;
                            }
                            ts[k] = doit ? tsn : ts[k];
                            if (use_color) {
                                const uint32_t c = cv[j][k];
                                if constexpr (C64) {
                                    const double wd = (double)wv, w1d = (double)w1;
                                    const double ar = cr[k] * wd + (double)(c & 0xFFu);
                                    const double ag = cg[k] * wd + (double)((c >> 8) & 0xFFu);
                                    const double ab = cb[k] * wd + (double)((c >> 16) & 0xFFu);
                                    double nr, ng, nb;
                                    if constexpr (FAST) {
                                        const double y = y64;
                                        const double q0r = ar * y, q0g = ag * y, q0b = ab * y;
                                        nr = __builtin_fma(__builtin_fma(-w1d, q0r, ar), y, q0r);
                                        ng = __builtin_fma(__builtin_fma(-w1d, q0g, ag), y, q0g);
                                        nb = __builtin_fma(__builtin_fma(-w1d, q0b, ab), y, q0b);
                                    } else {
                                        nr = ar / w1d;
                                        ng = ag / w1d;
                                        nb = ab / w1d;
                                    }
                                    cr[k] = doit ? nr : cr[k];
                                    cg[k] = doit ? ng : cg[k];
                                    cb[k] = doit ? nb : cb[k];
                                } else {
                                    const float rw = __builtin_amdgcn_rcpf(w1);
                                    const float nr = ((float)cr[k] * wv + (float)(c & 0xFFu)) * rw;
                                    const float ng = ((float)cg[k] * wv + (float)((c >> 8) & 0xFFu)) * rw;
                                    const float nb = ((float)cb[k] * wv + (float)((c >> 16) & 0xFFu)) * rw;
                                    cr[k] = doit ? nr : cr[k];
                                    cg[k] = doit ? ng : cg[k];
                                    cb[k] = doit ? nb : cb[k];
                                }
                            }
                            wt[k] = doit ? w1 : wv;
                            upd += doit ? 1u : 0u;
                        }
                        return true;
                    };
                    // one iteration = frame f in slot J: stage C of f + KC, the tap of f + KT (into the slot frame f - 1
                    // left), the update of f
                    auto iter = [&](auto J) __attribute__((always_inline)) -> bool {
                        constexpr int j = decltype(J)::value;
                        stage_c(std::integral_constant<int, (j + KC) % RS>{});
                        tap(std::integral_constant<int, (j + KT) % RS>{});
                        return stage_d(J);
                    };
                    // prologue: taps of the first KT frames, stage C of the first KC
                    static_for<KT>(tap);
                    static_for<KC>(stage_c);
                    while (static_all<RS>(iter)) {
                    }
                } else {
                    for (unsigned long long m = mask; m; m &= m - 1) {
                        const int f = __ffsll((long long)m) - 1;
                        const BatchFrame& fr = frames[f];
                        const __amdgpu_buffer_rsrc_t dm_rsrc = make_rsrc(fr.dm, npx * 8);
                        const __amdgpu_buffer_rsrc_t rgba_rsrc = make_rsrc(fr.rgba, npx * 4);
                        const bool use_color = fr.color != nullptr;
                        float pc[3];
#pragma unroll
                        for (int r = 0; r < 3; ++r) {
                            const float a = fr.E[r * 4 + 0] * px;
                            const float b = fr.E[r * 4 + 1] * py;
                            const float c = fr.E[r * 4 + 2] * pz;
                            pc[r] = ((a + b) + c) + fr.E[r * 4 + 3];
                        }
                        const float es0 = fr.es[0], es1 = fr.es[1], es2 = fr.es[2];
                        for (int k = 0; k < z0; ++k) {  // wave-uniform: advance to this slice's first voxel
                            pc[0] += es0;
                            pc[1] += es1;
                            pc[2] += es2;
                        }
                        // phase A: projections of the ZB voxels
                        int pixv[ZB];
                        float pcz[ZB];
#pragma unroll
                        for (int k = 0; k < ZB; ++k) {
                            const float nu = pc[0] * p.fx, nv = pc[1] * p.fy;
                            // Certified fast projection.  Only floor(u), floor(v) and the bound tests are used, so
                            // u = nu * rcp(z) decides them exactly unless u lies within proj_eps of an integer (the
                            // bound tests 0.0001 and W - 0.0001 sit 1e-4 from integers); those rare waves redo the
                            // IEEE quotients.
                            const float rz = __builtin_amdgcn_rcpf(pc[2]);
                            float u_f = (nu * rz + p.cx) + 0.5f;
                            float v_f = (nv * rz + p.cy) + 0.5f;
                            const bool sure = !(pc[2] > 0.0f) ||
                                              ((int)(fabsf(u_f - __builtin_rintf(u_f)) > p.proj_eps) &
                                               (int)(fabsf(v_f - __builtin_rintf(v_f)) > p.proj_eps));
                            if (!sure) {
                                u_f = ((nu / pc[2]) + p.cx) + 0.5f;
                                v_f = ((nv / pc[2]) + p.cy) + 0.5f;
                            }
                            // non-short-circuit test keeps all ZB projections in one basic block
                            const bool ok = (pc[2] > 0.0f) & (u_f >= 0.0001f) & (u_f < p.safe_w) & (v_f >= 0.0001f) &
                                            (v_f < p.safe_h);
                            pixv[k] = ok ? (int)__umul24((unsigned)(int)v_f, (unsigned)p.W) + (int)u_f : -1;
                            pcz[k] = pc[2];
                            pc[0] += es0;
                            pc[1] += es1;
                            pc[2] += es2;
                        }
                        // phase B: every depth gather issued before any use (buffer loads: wave-uniform resource +
                        // 32-bit byte offset, no per-lane 64-bit address math)
                        float dv[ZB], mv[ZB];
#pragma unroll
                        for (int k = 0; k < ZB; ++k) {
                            dv[k] = mv[k] = 0.0f;
                            if (pixv[k] >= 0) {  // lanes projecting outside the image issue no gather
                                const u32x2 raw = __builtin_amdgcn_raw_buffer_load_b64(dm_rsrc, pixv[k] * 8, 0, 0);
                                dv[k] = __uint_as_float(raw.x);
                                mv[k] = __uint_as_float(raw.y);
                            }
                        }
                        // phase C: the depth test; colour gathered only by the lanes whose voxel updates
                        bool doitv[ZB];
                        float sdfv[ZB];
                        uint32_t cv[ZB];
#pragma unroll
                        for (int k = 0; k < ZB; ++k) {
                            sdfv[k] = (dv[k] - pcz[k]) * mv[k];
                            doitv[k] = (pixv[k] >= 0) & (dv[k] > 0.0f) & (sdfv[k] > -p.trunc);
                            cv[k] = 0u;
                            if (use_color && doitv[k]) cv[k] = __builtin_amdgcn_raw_buffer_load_b32(rgba_rsrc, pixv[k] * 4, 0, 0);
                        }
                        // phase D: updates in frame order (select form: identical values, no exec-mask branches)
#pragma unroll
                        for (int k = 0; k < ZB; ++k) {
                            const bool doit = doitv[k];
                            const float sv = sdfv[k] * p.trunc_inv;
                            const float tn = (sv < 1.0f) ? sv : 1.0f;
                            const float wv = wt[k];
                            const float w1 = wv + 1.0f;
                            const float ta = ts[k] * wv + tn;
                            float tsn;  // (tsdf * w + t) / (w + 1): the IEEE quotient, tsdf bit-exact
                            // one table read per voxel for the tsdf and the colour quotients (round 3: +0.8 %)
                            const double y64 = (FAST && C64) ? s_r64[(int)w1] : 0.0;
                            if constexpr (FAST) {
                                const float y = C64 ? (float)y64 : s_r32[(int)w1];
                                const float q0 = ta * y;
                                tsn = __builtin_fmaf(__builtin_fmaf(-w1, q0, ta), y, q0);
                            } else {
                                tsn = ta / w1;
                            }
                            ts[k] = doit ? tsn : ts[k];
                            if (use_color) {
                                if constexpr (C64) {  // Open3D: color = (color * weight + rgb) / (weight + 1.0f) in float64
                                    {  // every lane, in select form (skipping voxels without an updating lane: slower)
                                        const double wd = (double)wv, w1d = (double)w1;
                                        const double ar = cr[k] * wd + (double)(cv[k] & 0xFFu);
                                        const double ag = cg[k] * wd + (double)((cv[k] >> 8) & 0xFFu);
                                        const double ab = cb[k] * wd + (double)((cv[k] >> 16) & 0xFFu);
                                        double nr, ng, nb;
                                        if constexpr (FAST) {
                                            const double y = y64;
                                            const double q0r = ar * y, q0g = ag * y, q0b = ab * y;
                                            nr = __builtin_fma(__builtin_fma(-w1d, q0r, ar), y, q0r);
                                            ng = __builtin_fma(__builtin_fma(-w1d, q0g, ag), y, q0g);
                                            nb = __builtin_fma(__builtin_fma(-w1d, q0b, ab), y, q0b);
                                        } else {
                                            nr = ar / w1d;
                                            ng = ag / w1d;
                                            nb = ab / w1d;
                                        }
                                        cr[k] = doit ? nr : cr[k];
                                        cg[k] = doit ? ng : cg[k];
                                        cb[k] = doit ? nb : cb[k];
                                    }
                                } else {  // float32 state, one reciprocal for the three channels (|rel| <= 1e-4)
                                    const float rw = __builtin_amdgcn_rcpf(w1);
                                    const float nr = ((float)cr[k] * wv + (float)(cv[k] & 0xFFu)) * rw;
                                    const float ng = ((float)cg[k] * wv + (float)((cv[k] >> 8) & 0xFFu)) * rw;
                                    const float nb = ((float)cb[k] * wv + (float)((cv[k] >> 16) & 0xFFu)) * rw;
                                    cr[k] = doit ? nr : cr[k];
                                    cg[k] = doit ? ng : cg[k];
                                    cb[k] = doit ? nb : cb[k];
                                }
                            }
                            wt[k] = doit ? w1 : wv;
                            upd += doit ? 1u : 0u;
                        }
                    }
                }
                // a slice none of whose voxels updated in this batch still holds its HBM values (fresh ones: zeros)
                if (!fresh && !__any(upd != upd0)) continue;
#pragma unroll
                for (int k = 0; k < ZB; ++k) {
                    const int vi = (z0 + k) * 256 + col;
                    base[vi] = ts[k];
                    base[UNIT_VOX + vi] = wt[k];
                    if constexpr (C64) {
                        st_f64(col64, vi, cr[k]);
                        st_f64(col64, UNIT_VOX + vi, cg[k]);
                        st_f64(col64, 2 * UNIT_VOX + vi, cb[k]);
                    } else {
                        base[2 * UNIT_VOX + vi] = cr[k];
                        base[3 * UNIT_VOX + vi] = cg[k];
                        base[4 * UNIT_VOX + vi] = cb[k];
                    }
                }
            }
        }
    }
    const unsigned long long tot = wave_sum((unsigned long long)upd);
    if (lane == 0 && tot) atomicAdd(&d.stats[S_UPDATES], tot);
}

// The product kernel keeps its own text (the same per-voxel code as integrate_body): compiled from the shared inlined
// body, its frame loop gained five uniform branches and lost 1.3 % (0.726 vs 0.717 ms per launch, r06n vs r06j)
template <bool C64, bool FAST, int ZB = BZ, int KT = 1>
__global__ __launch_bounds__(64 * INT_WG, (C64 && !FAST) ? 5 : (ZB == 2 ? 4 : INT_WAVES_PER_EU)) void k_batch_integrate(
    const BatchFrame* __restrict__ frames, IntegrateParams p, TsdfDev d, const UnitWork* __restrict__ work,
    const int* __restrict__ wcount) {
    using CT = typename std::conditional<C64, double, float>::type;
    constexpr int PARTS = 4 * (UNIT_RES / ZB) / INT_WG;  // workgroups per unit (INT_PARTS at the default ZB)
    // one table per kernel: float64 reciprocals for the float64-colour kernel (its float32 ones are their roundings:
    // (float)RN64(1/n) == RN32(1/n) for every n <= 2^20, no double-rounding case -- tools/markstein_check.cpp),
    // float32 ones otherwise
    __shared__ float s_r32[(FAST && !C64) ? RCP_N + 1 : 1];
    __shared__ double s_r64[(FAST && C64) ? RCP_N + 1 : 1];
    // work item = (unit, part): the PARTS parts of a unit are items 8 apart, so they run on one XCD (blocks are dealt
    // round-robin over the 8 XCDs) at about the same time and share its L2's copy of the footprint.
    // The grid is sized for large batches (8x the resident workgroups): a workgroup without an item leaves before
    // building the reciprocal table -- for a batch of few units (a spatial shard) the idle workgroups' tables had cost
    // more than the integrate itself (r05e: a 1/8 shard's 64-frame batch 165-200 us whatever its slicing)
    {
        const int n0 = __builtin_amdgcn_readfirstlane(__hip_atomic_load(wcount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if ((int)blockIdx.x >= (PARTS == 1 ? n0 : ((n0 + 7) / 8) * 8 * PARTS)) return;
    }
    if constexpr (FAST) {
        for (int r = threadIdx.x; r <= RCP_N; r += 64 * INT_WG) {
            if constexpr (C64) s_r64[r] = 1.0 / (double)r;  // IEEE (correctly rounded) quotients
            else s_r32[r] = 1.0f / (float)r;
        }
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int n = *wcount;
    const int npx = p.W * p.H;
    unsigned upd = 0;  // per lane: <= ZB voxels x 64 frames x units per workgroup, far below 2^32
    {
        const int b = blockIdx.x;
        const int items = PARTS == 1 ? n : ((n + 7) / 8) * 8 * PARTS;
        for (int it = b; it < items; it += gridDim.x) {
            const int u = PARTS == 1 ? it : (it / (8 * PARTS)) * 8 + (it & 7);
            if (PARTS > 1 && u >= n) continue;
            const int part = PARTS == 1 ? 0 : (it >> 3) % PARTS;
            const int s = __builtin_amdgcn_readfirstlane(part * INT_WG + (int)(threadIdx.x >> 6));  // slice of this wave
            const UnitWork& w = work[u];
            const int ent = w.id;
            const unsigned long long mask = w.mask;
            if (ent != -1) {
                const int id = ent & 0x7FFFFFFF;
                const bool fresh = ent < 0;
                // wave = 8 x 8 columns: a square patch of the unit's xy plane projects to fewer pixel rows
                const int x = (s & 2) * 4 + (lane >> 3), y = (s & 1) * 8 + (lane & 7);
                const int col = x * 16 + y;
                const int z0 = (s >> 2) * ZB;
                float* base = d.vox + (size_t)id * (C64 ? UNIT_FLOATS_C64 : UNIT_FLOATS);
                // colour plane c of voxel vi: float32 planes addressed from base (one address register for the
                // whole record: a separate colour pointer costs ~34 VGPRs in this kernel), float64 through a buffer
                // resource over the record's float64 planes
                const __amdgpu_buffer_rsrc_t col64 = make_rsrc(base + 2 * UNIT_VOX, 3 * UNIT_VOX * 8);
                float ts[ZB], wt[ZB];
                CT cr[ZB], cg[ZB], cb[ZB];
#pragma unroll
                for (int k = 0; k < ZB; ++k) {
                    const int vi = (z0 + k) * 256 + col;
                    if (fresh) {
                        ts[k] = wt[k] = 0.0f;
                        cr[k] = cg[k] = cb[k] = (CT)0;
                    } else {
                        ts[k] = base[vi];
                        wt[k] = base[UNIT_VOX + vi];
                        if constexpr (C64) {
                            cr[k] = ld_f64(col64, vi);
                            cg[k] = ld_f64(col64, UNIT_VOX + vi);
                            cb[k] = ld_f64(col64, 2 * UNIT_VOX + vi);
                        } else {
                            cr[k] = base[2 * UNIT_VOX + vi];
                            cg[k] = base[3 * UNIT_VOX + vi];
                            cb[k] = base[4 * UNIT_VOX + vi];
                        }
                    }
                }
                const float ox = (float)((double)w.kx * p.unit_len);
                const float oy = (float)((double)w.ky * p.unit_len);
                const float oz = (float)((double)w.kz * p.unit_len);
                const float px = (p.half + p.vl * (float)x) + ox;
                const float py = (p.half + p.vl * (float)y) + oy;
                const float pz = p.half + oz;
                const unsigned upd0 = upd;
                if constexpr (ZB == 2) {
                    // Frame pipeline (the fine slices serve batches with few units, whose waves cannot hide a frame's
                    // dependent gathers behind other waves: the wave's chain of frames IS the batch's time).  Every
                    // load of a frame is state-independent -- the projections and depth gathers (tap), the depth test,
                    // clamped tsdf term and colour gather (stage C) -- only the running means (stage D) read the
                    // voxel state.  So frame f+KT's tap and frame f+KC's stage C are issued before frame f's update,
                    // from KT + 1 register slots (the loop is unrolled over the slots so every slot is a fixed
                    // register set: a rotating copy would wait for the loads in flight).  The updates still run in
                    // frame order with the same arithmetic: the bits are the unpipelined loop's.  KT = 1, KC = 0 is the
                    // round-5 one-frame skew.
                    constexpr int KC = KT - 1, RS = KT + 1;
                    unsigned long long mt = mask;  // frames not yet tapped
                    int fs[RS];                     // frame of each slot (wave-uniform), -1: past the last frame
                    int pixv[RS][ZB];
                    float pcz[RS][ZB], dv[RS][ZB], mv[RS][ZB], tnv[RS][ZB];
                    uint32_t cv[RS][ZB];
                    bool dov[RS][ZB];
                    auto tap = [&](auto J) __attribute__((always_inline)) {
                        constexpr int j = decltype(J)::value;
                        if (mt) {
                            const int f = __ffsll((long long)mt) - 1;
                            mt &= mt - 1;
                            fs[j] = f;
                            frame_tap<ZB>(frames[f], p, npx, px, py, pz, z0, pixv[j], pcz[j], dv[j], mv[j]);
                        } else {
                            fs[j] = -1;
                        }
                    };
                    auto stage_c = [&](auto J) __attribute__((always_inline)) {
                        constexpr int j = decltype(J)::value;
                        if (fs[j] < 0) return;
                        const BatchFrame& fr = frames[fs[j]];
                        const __amdgpu_buffer_rsrc_t rgba_rsrc = make_rsrc(fr.rgba, npx * 4);
                        const bool use_color = fr.color != nullptr;
#pragma unroll
                        for (int k = 0; k < ZB; ++k) {
                            const float sdf = (dv[j][k] - pcz[j][k]) * mv[j][k];
                            dov[j][k] = (pixv[j][k] >= 0) & (dv[j][k] > 0.0f) & (sdf > -p.trunc);
                            const float sv = sdf * p.trunc_inv;
                            tnv[j][k] = (sv < 1.0f) ? sv : 1.0f;
                            cv[j][k] = 0u;
                            if (use_color && dov[j][k])
                                cv[j][k] = __builtin_amdgcn_raw_buffer_load_b32(rgba_rsrc, pixv[j][k] * 4, 0, 0);
                        }
                    };
                    auto stage_d = [&](auto J) __attribute__((always_inline)) -> bool {
                        constexpr int j = decltype(J)::value;
                        if (fs[j] < 0) return false;
                        const bool use_color = frames[fs[j]].color != nullptr;
#pragma unroll
                        for (int k = 0; k < ZB; ++k) {
                            const bool doit = dov[j][k];
                            const float tn = tnv[j][k];
                            const float wv = wt[k];
                            const float w1 = wv + 1.0f;
                            const float ta = ts[k] * wv + tn;
                            float tsn;
                            const double y64 = (FAST && C64) ? s_r64[(int)w1] : 0.0;
                            if constexpr (FAST) {
                                const float y = C64 ? (float)y64 : s_r32[(int)w1];
                                const float q0 = ta * y;
                                tsn = __builtin_fmaf(__builtin_fmaf(-w1, q0, ta), y, q0);
                            } else {
                                tsn = ta / w1;
                            }
                            ts[k] = doit ? tsn : ts[k];
                            if (use_color) {
                                const uint32_t c = cv[j][k];
                                if constexpr (C64) {
                                    const double wd = (double)wv, w1d = (double)w1;
                                    const double ar = cr[k] * wd + (double)(c & 0xFFu);
                                    const double ag = cg[k] * wd + (double)((c >> 8) & 0xFFu);
                                    const double ab = cb[k] * wd + (double)((c >> 16) & 0xFFu);
                                    double nr, ng, nb;
                                    if constexpr (FAST) {
                                        const double y = y64;
                                        const double q0r = ar * y, q0g = ag * y, q0b = ab * y;
                                        nr = __builtin_fma(__builtin_fma(-w1d, q0r, ar), y, q0r);
                                        ng = __builtin_fma(__builtin_fma(-w1d, q0g, ag), y, q0g);
                                        nb = __builtin_fma(__builtin_fma(-w1d, q0b, ab), y, q0b);
                                    } else {
                                        nr = ar / w1d;
                                        ng = ag / w1d;
                                        nb = ab / w1d;
                                    }
                                    cr[k] = doit ? nr : cr[k];
                                    cg[k] = doit ? ng : cg[k];
                                    cb[k] = doit ? nb : cb[k];
                                } else {
                                    const float rw = __builtin_amdgcn_rcpf(w1);
                                    const float nr = ((float)cr[k] * wv + (float)(c & 0xFFu)) * rw;
                                    const float ng = ((float)cg[k] * wv + (float)((c >> 8) & 0xFFu)) * rw;
                                    const float nb = ((float)cb[k] * wv + (float)((c >> 16) & 0xFFu)) * rw;
                                    cr[k] = doit ? nr : cr[k];
                                    cg[k] = doit ? ng : cg[k];
                                    cb[k] = doit ? nb : cb[k];
                                }
                            }
                            wt[k] = doit ? w1 : wv;
                            upd += doit ? 1u : 0u;
                        }
                        return true;
                    };
                    // one iteration = frame f in slot J: stage C of f + KC, the tap of f + KT (into the slot frame f - 1
                    // left), the update of f
                    auto iter = [&](auto J) __attribute__((always_inline)) -> bool {
                        constexpr int j = decltype(J)::value;
                        stage_c(std::integral_constant<int, (j + KC) % RS>{});
                        tap(std::integral_constant<int, (j + KT) % RS>{});
                        return stage_d(J);
                    };
                    // prologue: taps of the first KT frames, stage C of the first KC
                    static_for<KT>(tap);
                    static_for<KC>(stage_c);
                    while (static_all<RS>(iter)) {
                    }
                } else {
                    for (unsigned long long m = mask; m; m &= m - 1) {
                        const int f = __ffsll((long long)m) - 1;
                        const BatchFrame& fr = frames[f];
                        const __amdgpu_buffer_rsrc_t dm_rsrc = make_rsrc(fr.dm, npx * 8);
                        const __amdgpu_buffer_rsrc_t rgba_rsrc = make_rsrc(fr.rgba, npx * 4);
                        const bool use_color = fr.color != nullptr;
                        float pc[3];
#pragma unroll
                        for (int r = 0; r < 3; ++r) {
                            const float a = fr.E[r * 4 + 0] * px;
                            const float b = fr.E[r * 4 + 1] * py;
                            const float c = fr.E[r * 4 + 2] * pz;
                            pc[r] = ((a + b) + c) + fr.E[r * 4 + 3];
                        }
                        const float es0 = fr.es[0], es1 = fr.es[1], es2 = fr.es[2];
                        for (int k = 0; k < z0; ++k) {  // wave-uniform: advance to this slice's first voxel
                            pc[0] += es0;
                            pc[1] += es1;
                            pc[2] += es2;
                        }
                        // phase A: projections of the ZB voxels
                        int pixv[ZB];
                        float pcz[ZB];
#pragma unroll
                        for (int k = 0; k < ZB; ++k) {
                            const float nu = pc[0] * p.fx, nv = pc[1] * p.fy;
                            // Certified fast projection.  Only floor(u), floor(v) and the bound tests are used, so
                            // u = nu * rcp(z) decides them exactly unless u lies within proj_eps of an integer (the
                            // bound tests 0.0001 and W - 0.0001 sit 1e-4 from integers); those rare waves redo the
                            // IEEE quotients.
                            const float rz = __builtin_amdgcn_rcpf(pc[2]);
                            float u_f = (nu * rz + p.cx) + 0.5f;
                            float v_f = (nv * rz + p.cy) + 0.5f;
                            const bool sure = !(pc[2] > 0.0f) ||
                                              ((int)(fabsf(u_f - __builtin_rintf(u_f)) > p.proj_eps) &
                                               (int)(fabsf(v_f - __builtin_rintf(v_f)) > p.proj_eps));
                            if (!sure) {
                                u_f = ((nu / pc[2]) + p.cx) + 0.5f;
                                v_f = ((nv / pc[2]) + p.cy) + 0.5f;
                            }
                            // non-short-circuit test keeps all ZB projections in one basic block
                            const bool ok = (pc[2] > 0.0f) & (u_f >= 0.0001f) & (u_f < p.safe_w) & (v_f >= 0.0001f) &
                                            (v_f < p.safe_h);
                            pixv[k] = ok ? (int)__umul24((unsigned)(int)v_f, (unsigned)p.W) + (int)u_f : -1;
                            pcz[k] = pc[2];
                            pc[0] += es0;
                            pc[1] += es1;
                            pc[2] += es2;
                        }
                        // phase B: every depth gather issued before any use (buffer loads: wave-uniform resource +
                        // 32-bit byte offset, no per-lane 64-bit address math)
                        float dv[ZB], mv[ZB];
#pragma unroll
                        for (int k = 0; k < ZB; ++k) {
                            dv[k] = mv[k] = 0.0f;
                            if (pixv[k] >= 0) {  // lanes projecting outside the image issue no gather
                                const u32x2 raw = __builtin_amdgcn_raw_buffer_load_b64(dm_rsrc, pixv[k] * 8, 0, 0);
                                dv[k] = __uint_as_float(raw.x);
                                mv[k] = __uint_as_float(raw.y);
                            }
                        }
                        // phase C: the depth test; colour gathered only by the lanes whose voxel updates
                        bool doitv[ZB];
                        float sdfv[ZB];
                        uint32_t cv[ZB];
#pragma unroll
                        for (int k = 0; k < ZB; ++k) {
                            sdfv[k] = (dv[k] - pcz[k]) * mv[k];
                            doitv[k] = (pixv[k] >= 0) & (dv[k] > 0.0f) & (sdfv[k] > -p.trunc);
                            cv[k] = 0u;
                            if (use_color && doitv[k]) cv[k] = __builtin_amdgcn_raw_buffer_load_b32(rgba_rsrc, pixv[k] * 4, 0, 0);
                        }
                        // phase D: updates in frame order (select form: identical values, no exec-mask branches)
#pragma unroll
                        for (int k = 0; k < ZB; ++k) {
                            const bool doit = doitv[k];
                            const float sv = sdfv[k] * p.trunc_inv;
                            const float tn = (sv < 1.0f) ? sv : 1.0f;
                            const float wv = wt[k];
                            const float w1 = wv + 1.0f;
                            const float ta = ts[k] * wv + tn;
                            float tsn;  // (tsdf * w + t) / (w + 1): the IEEE quotient, tsdf bit-exact
                            // one table read per voxel for the tsdf and the colour quotients (round 3: +0.8 %)
                            const double y64 = (FAST && C64) ? s_r64[(int)w1] : 0.0;
                            if constexpr (FAST) {
                                const float y = C64 ? (float)y64 : s_r32[(int)w1];
                                const float q0 = ta * y;
                                tsn = __builtin_fmaf(__builtin_fmaf(-w1, q0, ta), y, q0);
                            } else {
                                tsn = ta / w1;
                            }
                            ts[k] = doit ? tsn : ts[k];
                            if (use_color) {
                                if constexpr (C64) {  // Open3D: color = (color * weight + rgb) / (weight + 1.0f) in float64
                                    {  // every lane, in select form (skipping voxels without an updating lane: slower)
                                        const double wd = (double)wv, w1d = (double)w1;
                                        const double ar = cr[k] * wd + (double)(cv[k] & 0xFFu);
                                        const double ag = cg[k] * wd + (double)((cv[k] >> 8) & 0xFFu);
                                        const double ab = cb[k] * wd + (double)((cv[k] >> 16) & 0xFFu);
                                        double nr, ng, nb;
                                        if constexpr (FAST) {
                                            const double y = y64;
                                            const double q0r = ar * y, q0g = ag * y, q0b = ab * y;
                                            nr = __builtin_fma(__builtin_fma(-w1d, q0r, ar), y, q0r);
                                            ng = __builtin_fma(__builtin_fma(-w1d, q0g, ag), y, q0g);
                                            nb = __builtin_fma(__builtin_fma(-w1d, q0b, ab), y, q0b);
                                        } else {
                                            nr = ar / w1d;
                                            ng = ag / w1d;
                                            nb = ab / w1d;
                                        }
                                        cr[k] = doit ? nr : cr[k];
                                        cg[k] = doit ? ng : cg[k];
                                        cb[k] = doit ? nb : cb[k];
                                    }
                                } else {  // float32 state, one reciprocal for the three channels (|rel| <= 1e-4)
                                    const float rw = __builtin_amdgcn_rcpf(w1);
                                    const float nr = ((float)cr[k] * wv + (float)(cv[k] & 0xFFu)) * rw;
                                    const float ng = ((float)cg[k] * wv + (float)((cv[k] >> 8) & 0xFFu)) * rw;
                                    const float nb = ((float)cb[k] * wv + (float)((cv[k] >> 16) & 0xFFu)) * rw;
                                    cr[k] = doit ? nr : cr[k];
                                    cg[k] = doit ? ng : cg[k];
                                    cb[k] = doit ? nb : cb[k];
                                }
                            }
                            wt[k] = doit ? w1 : wv;
                            upd += doit ? 1u : 0u;
                        }
                    }
                }
                // a slice none of whose voxels updated in this batch still holds its HBM values (fresh ones: zeros)
                if (!fresh && !__any(upd != upd0)) continue;
#pragma unroll
                for (int k = 0; k < ZB; ++k) {
                    const int vi = (z0 + k) * 256 + col;
                    base[vi] = ts[k];
                    base[UNIT_VOX + vi] = wt[k];
                    if constexpr (C64) {
                        st_f64(col64, vi, cr[k]);
                        st_f64(col64, UNIT_VOX + vi, cg[k]);
                        st_f64(col64, 2 * UNIT_VOX + vi, cb[k]);
                    } else {
                        base[2 * UNIT_VOX + vi] = cr[k];
                        base[3 * UNIT_VOX + vi] = cg[k];
                        base[4 * UNIT_VOX + vi] = cb[k];
                    }
                }
            }
        }
    }
    const unsigned long long tot = wave_sum((unsigned long long)upd);
    if (lane == 0 && tot) atomicAdd(&d.stats[S_UPDATES], tot);
}

// The deferred integrate of a sharded volume's batch k and the touch of batch k + 1 in ONE launch (round 6): workgroups
// [0, nint) integrate batch k (its set's staging and work list), the rest are batch k + 1's touch tiles (frame groups
// along the grid).  A rank's integrate fills few of the CUs (a shard's batch is a few hundred units), so its latency-bound
// touch runs in the gaps, with no second stream and no event between them (two streams' fork + join cost ~25 us of idle
// GPU per batch: the double-buffered front end).  The touch writes only batch k + 1's state: its frame
// masks / slot list / pair counter, hash inserts of its units, and the staged pixels of its samples in its own set --
// nothing the integrate of batch k reads.  LDS: the touch's tables and the reciprocal table share one block.
template <bool C64, bool FAST>
__global__ __launch_bounds__(64 * INT_WG, INT_WAVES_PER_EU) void k_integrate_touch(
    const BatchFrame* __restrict__ frames, IntegrateParams p, TsdfDev d, const UnitWork* __restrict__ work,
    const int* __restrict__ wcount, int nint, const BatchFrame* __restrict__ tframes, BatchTouchParams tp, int tn) {
    union Lds {
        TouchLds t;
        RcpLds<C64, FAST> r;
    };
    __shared__ Lds lds;
    const int b = (int)blockIdx.x;
    if (b < nint) {
        integrate_body<C64, FAST, BZ, 1>(frames, p, d, work, wcount, lds.r, b, nint);
    } else {
        const int t = b - nint;
        touch_body<false, false>(tframes, tp, d, tn, lds.t, t % tp.tiles, t / tp.tiles);
    }
}
// The same launch with the integrate in fine slices (2 voxels per lane along z, k_batch_integrate<.., 2, 1>'s per-voxel
// code and occupancy): the deferred batch's unit count is known on the host by then (its units kernel mailed it), so a
// batch of few units takes the fine slices without the guess the direct path makes from the previous batch
template <bool C64, bool FAST>
__global__ __launch_bounds__(64 * INT_WG, (C64 && !FAST) ? 5 : 4) void k_integrate_touch_fine(
    const BatchFrame* __restrict__ frames, IntegrateParams p, TsdfDev d, const UnitWork* __restrict__ work,
    const int* __restrict__ wcount, int nint, const BatchFrame* __restrict__ tframes, BatchTouchParams tp, int tn) {
    union Lds {
        TouchLds t;
        RcpLds<C64, FAST> r;
    };
    __shared__ Lds lds;
    const int b = (int)blockIdx.x;
    if (b < nint) {
        integrate_body<C64, FAST, 2, 1>(frames, p, d, work, wcount, lds.r, b, nint);
    } else {
        const int t = b - nint;
        touch_body<false, false>(tframes, tp, d, tn, lds.t, t % tp.tiles, t / tp.tiles);
    }
}

// export: units in sorted order, voxels transposed to Open3D IndexOf order (x*256 + y*16 + z); colour as CT
// (float export of a float64 volume rounds to nearest)
template <typename CT, typename OT>
__global__ __launch_bounds__(256) void k_export(TsdfDev d, const unsigned* sorted_ids, int32_t* keys, float* tsdf,
                                                float* weight, OT* color) {
    const int r = blockIdx.x;
    const int id = (int)sorted_ids[r];
    const int tid = threadIdx.x;
    const float* base = unit_base(d, id);
    const CT* cbase = color_base<CT>(d, id);
    if (keys && tid < 3) keys[(int64_t)r * 3 + tid] = d.unit_keys[id * 3 + tid];
    for (int z = 0; z < UNIT_RES; ++z) {
        const int vi = z * 256 + tid;
        const int64_t o = (int64_t)r * UNIT_VOX + tid * 16 + z;
        if (tsdf) tsdf[o] = base[vi];
        if (weight) weight[o] = base[UNIT_VOX + vi];
        if (color) {
            color[o * 3 + 0] = (OT)cbase[vi];
            color[o * 3 + 1] = (OT)cbase[UNIT_VOX + vi];
            color[o * 3 + 2] = (OT)cbase[2 * UNIT_VOX + vi];
        }
    }
}

// border export: the BORDER_VOX low-face voxels of every unit, units in sorted order; colour as the volume keeps it
template <typename CT>
__global__ __launch_bounds__(256) void k_export_border(TsdfDev d, const unsigned* sorted_ids, int32_t* keys,
                                                       float* tsdf, float* weight, CT* color) {
    const int r = blockIdx.x;
    const int id = (int)sorted_ids[r];
    const float* base = unit_base(d, id);
    const CT* cbase = color_base<CT>(d, id);
    if (threadIdx.x < 3) keys[(int64_t)r * 3 + threadIdx.x] = d.unit_keys[id * 3 + threadIdx.x];
    for (int b = threadIdx.x; b < BORDER_VOX; b += 256) {
        int x, y, z;
        border_voxel(b, x, y, z);
        const int vi = z * 256 + x * 16 + y;
        const int64_t o = (int64_t)r * BORDER_VOX + b;
        tsdf[o] = base[vi];
        weight[o] = base[UNIT_VOX + vi];
        if (color) {
            color[o * 3 + 0] = cbase[vi];
            color[o * 3 + 1] = cbase[UNIT_VOX + vi];
            color[o * 3 + 2] = cbase[2 * UNIT_VOX + vi];
        }
    }
}

__device__ inline int find_unit_id(const TsdfDev& d, int x, int y, int z) {
    if (!key_in_range(x, y, z)) return -1;
    const unsigned long long key = pack_key(x, y, z);
    unsigned slot = (unsigned)mix64(key) & (unsigned)d.hash_mask;
    for (int probe = 0; probe <= d.hash_mask; ++probe) {
        const unsigned long long k = d.hkeys[slot];
        if (k == key) {
            const int id = d.hvals[slot];
            return id < d.max_units ? id : -1;
        }
        if (k == KEY_EMPTY) return -1;
        slot = (slot + 1) & (unsigned)d.hash_mask;
    }
    return -1;
}

// border import (halo): a row becomes a halo unit of this volume when its key is not owned here and one of its
// -x/-y/-z neighbours (the units whose marching cubes read it) is; a new halo unit is zeroed (weight 0 = unobserved)
// and receives the border voxels.  Rows of owned or unneeded units are skipped.
template <typename CT>
__global__ __launch_bounds__(256) void k_import_border(TsdfDev d, const int32_t* __restrict__ keys,
                                                       const float* __restrict__ tsdf, const float* __restrict__ weight,
                                                       const CT* __restrict__ color) {
    __shared__ int s_id, s_fresh;
    const int r = blockIdx.x;
    if (threadIdx.x == 0) {
        const int x = keys[(int64_t)r * 3], y = keys[(int64_t)r * 3 + 1], z = keys[(int64_t)r * 3 + 2];
        int id = -1, fresh = 0;
        bool needed = false;
        if (key_in_range(x, y, z) && !unit_owned(d, pack_key(x, y, z))) {
            for (int t = 1; t < 8 && !needed; ++t) {
                const int nx = x - ((t >> 2) & 1), ny = y - ((t >> 1) & 1), nz = z - (t & 1);
                needed = key_in_range(nx, ny, nz) && unit_owned(d, pack_key(nx, ny, nz)) &&
                         find_unit_id(d, nx, ny, nz) >= 0;
            }
        }
        if (needed) {
            const int slot = hash_insert(d, pack_key(x, y, z));
            if (slot < 0) {
                atomicOr(&d.counters[C_HASHERR], 1);
            } else {
                id = d.hvals[slot];
                if (id < 0) {
                    id = atomicAdd(&d.counters[C_UNITS], 1);
                    if (id >= d.max_units) {
                        atomicOr(&d.counters[C_OVERFLOW], 1);
                        id = -1;
                    } else {
                        d.hvals[slot] = id;
                        d.unit_keys[id * 3 + 0] = x;
                        d.unit_keys[id * 3 + 1] = y;
                        d.unit_keys[id * 3 + 2] = z;
                        fresh = 1;
                        note_unit_key(d, x, y, z);
                    }
                }
            }
        }
        s_id = id;
        s_fresh = fresh;
    }
    __syncthreads();
    const int id = s_id;
    if (id < 0) return;
    float* base = unit_base(d, id);
    CT* cbase = color_base<CT>(d, id);
    if (s_fresh) {
        for (int vi = threadIdx.x; vi < UNIT_VOX; vi += 256) {
            base[vi] = 0.0f;
            base[UNIT_VOX + vi] = 0.0f;
            cbase[vi] = cbase[UNIT_VOX + vi] = cbase[2 * UNIT_VOX + vi] = (CT)0;
        }
        __syncthreads();
    }
    for (int b = threadIdx.x; b < BORDER_VOX; b += 256) {
        int x, y, z;
        border_voxel(b, x, y, z);
        const int vi = z * 256 + x * 16 + y;
        const int64_t o = (int64_t)r * BORDER_VOX + b;
        base[vi] = tsdf[o];
        base[UNIT_VOX + vi] = weight[o];
        cbase[vi] = color ? color[o * 3 + 0] : (CT)0;
        cbase[UNIT_VOX + vi] = color ? color[o * 3 + 1] : (CT)0;
        cbase[2 * UNIT_VOX + vi] = color ? color[o * 3 + 2] : (CT)0;
    }
}

// destinations of a border row (SURVEY §8(e) halo): the ranks owning the unit's 7 -x/-y/-z neighbours (the units whose
// marching cubes read its low faces), this rank excluded -- a superset of the rows k_import_border keeps there
__global__ __launch_bounds__(256) void k_border_dest(TsdfDev d, int64_t n, const int32_t* __restrict__ keys,
                                                     unsigned long long* __restrict__ mask) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n) return;
    const int x = keys[r * 3], y = keys[r * 3 + 1], z = keys[r * 3 + 2];
    unsigned long long m = 0ull;
    if (d.shard_world > 1)
        for (int t = 1; t < 8; ++t) {
            const int nx = x - ((t >> 2) & 1), ny = y - ((t >> 1) & 1), nz = z - (t & 1);
            if (key_in_range(nx, ny, nz)) m |= 1ull << unit_owner(d, nx, ny, nz);
        }
    mask[r] = m & ~(1ull << d.shard_rank);
}

// owned units of the sorted order (a sharded volume's own units; every unit when unsharded)
struct OwnedPred {
    TsdfDev d;
    const unsigned* sorted_ids;
    __device__ bool operator()(int64_t r) const {
        const int id = (int)sorted_ids[r];
        return d.shard_world <= 1 ||
               unit_owned(d, pack_key(d.unit_keys[id * 3], d.unit_keys[id * 3 + 1], d.unit_keys[id * 3 + 2]));
    }
};
struct OwnedEmit {
    const unsigned* sorted_ids;
    unsigned* out;
    __device__ void operator()(int64_t r, int64_t pos) const { out[pos] = sorted_ids[r]; }
};

// Units an export lists: every unit in sorted key order or, for a spatially sharded volume, only its own units -- the
// halo units imported for marching cubes (k_import_border) are copies of other shards' border rows, and exporting
// them would hand their keys to an assembly twice (the second time with zeros inside the unit).
static ot_status export_list(ot_tsdf* vol, hipStream_t stream, const unsigned** ids, int64_t* n) {
    int64_t nu = 0;
    ot_status st = tsdf_sorted_units(vol, stream, &nu);
    if (st != OT_OK) return st;
    *ids = vol->sorted_ids;
    *n = nu;
    if (vol->dev.shard_world <= 1 || nu == 0) return OT_OK;
    unsigned* own = (unsigned*)scratch(sizeof(unsigned) * (size_t)nu + 256, 16);
    if (!own) return fail(OT_ERR_HIP, "scratch allocation failed");
    int64_t no = 0;
    st = compact(nu, OwnedPred{vol->dev, vol->sorted_ids}, OwnedEmit{vol->sorted_ids, own}, stream, &no, 13);
    if (st != OT_OK) return st;
    *ids = own;
    *n = no;
    return OT_OK;
}

// import: the inverse of k_export (keys unique within one call; an existing unit is overwritten); colour as the
// volume keeps it (CT)
template <typename CT>
__global__ __launch_bounds__(256) void k_import(TsdfDev d, const int32_t* __restrict__ keys,
                                                const float* __restrict__ tsdf, const float* __restrict__ weight,
                                                const CT* __restrict__ color) {
    __shared__ int s_id;
    const int r = blockIdx.x;
    const int tid = threadIdx.x;
    if (tid == 0) {
        const int x = keys[(int64_t)r * 3], y = keys[(int64_t)r * 3 + 1], z = keys[(int64_t)r * 3 + 2];
        int id = -1;
        if (!key_in_range(x, y, z)) {
            atomicOr(&d.counters[C_HASHERR], 2);
        } else {
            const int slot = hash_insert(d, pack_key(x, y, z));
            if (slot < 0) {
                atomicOr(&d.counters[C_HASHERR], 1);
            } else {
                id = d.hvals[slot];
                if (id < 0) {
                    id = atomicAdd(&d.counters[C_UNITS], 1);
                    if (id >= d.max_units) {
                        atomicOr(&d.counters[C_OVERFLOW], 1);
                        id = -1;
                    } else {
                        d.hvals[slot] = id;
                        d.unit_keys[id * 3 + 0] = x;
                        d.unit_keys[id * 3 + 1] = y;
                        d.unit_keys[id * 3 + 2] = z;
                        note_unit_key(d, x, y, z);
                    }
                }
            }
        }
        s_id = id;
    }
    __syncthreads();
    const int id = s_id;
    if (id < 0) return;
    float* base = unit_base(d, id);
    CT* cbase = color_base<CT>(d, id);
    for (int z = 0; z < UNIT_RES; ++z) {
        const int vi = z * 256 + tid;
        const int64_t o = (int64_t)r * UNIT_VOX + tid * 16 + z;
        base[vi] = tsdf[o];
        base[UNIT_VOX + vi] = weight[o];
        cbase[vi] = color ? color[o * 3 + 0] : (CT)0;
        cbase[UNIT_VOX + vi] = color ? color[o * 3 + 1] : (CT)0;
        cbase[2 * UNIT_VOX + vi] = color ? color[o * 3 + 2] : (CT)0;
    }
}

// order-preserving compact keys: (x - x0) << (by + bz) | (y - y0) << bz | (z - z0), only the bits the ranges need
struct UnitKeyPack {
    int x0, y0, z0, sy, sx;
};

__global__ void k_pack_unit_keys(TsdfDev d, int n, UnitKeyPack pk, unsigned long long* keys, unsigned* ids) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    keys[i] = ((unsigned long long)(d.unit_keys[i * 3 + 0] - pk.x0) << pk.sx) |
              ((unsigned long long)(d.unit_keys[i * 3 + 1] - pk.y0) << pk.sy) |
              (unsigned long long)(d.unit_keys[i * 3 + 2] - pk.z0);
    ids[i] = (unsigned)i;
}

// Unit order in ONE launch when the packed keys need <= USORT_BITS bits (a volume a few metres across): unit keys are
// distinct (one id per hash slot), so a unit's place in key order is the number of smaller keys -- a presence bitmap
// of the key space in LDS, a block scan of its popcounts per 8-word group, then per unit the group prefix plus the
// popcounts before its bit.  The same ids as the radix sort (k_pack_unit_keys + 4 launches of sort_pairs_u64_u32),
// whose launches dominated the unit sort of a single object (38 us for 5.6k units, profiles/r04z_obj_timeline.txt).
constexpr int USORT_BITS = 20;                   // 2^20-bit bitmap: 128 KiB of LDS
constexpr int USORT_WORDS = 1 << (USORT_BITS - 5);
constexpr int USORT_GROUPS = USORT_WORDS / 8;    // 4096 group prefixes: 16 KiB
__device__ inline unsigned unit_key_bits(const TsdfDev& d, const UnitKeyPack& pk, int i) {
    return ((unsigned)(d.unit_keys[i * 3 + 0] - pk.x0) << pk.sx) | ((unsigned)(d.unit_keys[i * 3 + 1] - pk.y0) << pk.sy) |
           (unsigned)(d.unit_keys[i * 3 + 2] - pk.z0);
}
__global__ __launch_bounds__(1024) void k_unit_rank_sort(TsdfDev d, int n, UnitKeyPack pk, int kb,
                                                         unsigned* __restrict__ sorted_ids) {
    __shared__ unsigned s_bits[USORT_WORDS];
    __shared__ unsigned s_gp[USORT_GROUPS];
    __shared__ unsigned s_w[16];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int words = kb > 5 ? 1 << (kb - 5) : 1, groups = (words + 7) >> 3;
    for (int q = t; q < words; q += 1024) s_bits[q] = 0u;
    __syncthreads();
    for (int i = t; i < n; i += 1024) {
        const unsigned k = unit_key_bits(d, pk, i);
        atomicOr(&s_bits[k >> 5], 1u << (k & 31));
    }
    __syncthreads();
    // thread t: groups [g0, g1), a contiguous stretch (4 groups = 32 words at 20 bits)
    const int per = (groups + 1023) >> 10, g0 = t * per, g1 = g0 + per < groups ? g0 + per : groups;
    unsigned loc = 0u;
    for (int g = g0; g < g1; ++g)
        for (int q = g * 8; q < g * 8 + 8 && q < words; ++q) loc += __popc(s_bits[q]);
    unsigned inc = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned v = __shfl_up(inc, o);
        if (lane >= o) inc += v;
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    unsigned run = inc - loc;
    for (int q = 0; q < w; ++q) run += s_w[q];
    for (int g = g0; g < g1; ++g) {
        s_gp[g] = run;
        for (int q = g * 8; q < g * 8 + 8 && q < words; ++q) run += __popc(s_bits[q]);
    }
    __syncthreads();
    for (int i = t; i < n; i += 1024) {
        const unsigned k = unit_key_bits(d, pk, i);
        const int q = (int)(k >> 5);
        unsigned r = s_gp[q >> 3] + __popc(s_bits[q] & ((1u << (k & 31)) - 1u));
        for (int p = q & ~7; p < q; ++p) r += __popc(s_bits[p]);
        sorted_ids[r] = (unsigned)i;
    }
}
static bool g_unit_sort_radix = false;  // test hook otx_unit_sort_radix: force the radix path (parity of the two)

// ------------------------------------------------------------------------------------ host helpers
static IntegrateParams make_integrate_params(const ot_tsdf* vol, const float* depth, const uint8_t* color,
                                             const float* mult, const ot_intrinsics* in, const double* ext) {
    IntegrateParams p;
    p.depth = depth;
    p.color = (vol->color_type == OT_COLOR_RGB8) ? color : nullptr;
    p.mult = mult;
    p.W = in->width;
    p.H = in->height;
    p.fx = (float)in->fx;
    p.fy = (float)in->fy;
    p.cx = (float)in->cx;
    p.cy = (float)in->cy;
    p.inv_fx = 1.0f / (float)in->fx;
    p.inv_fy = 1.0f / (float)in->fy;
    float E[16];
    for (int k = 0; k < 16; ++k) E[k] = (float)ext[k];
    for (int k = 0; k < 12; ++k) p.E[k] = E[k];
    const double unit_voxel_length = vol->unit_length / (double)UNIT_RES;
    p.vl = (float)unit_voxel_length;
    p.half = p.vl * 0.5f;
    p.es0 = E[0 * 4 + 2] * p.vl;
    p.es1 = E[1 * 4 + 2] * p.vl;
    p.es2 = E[2 * 4 + 2] * p.vl;
    p.trunc = (float)vol->sdf_trunc;
    p.trunc_inv = 1.0f / p.trunc;
    p.safe_w = (float)in->width - 0.0001f;
    p.safe_h = (float)in->height - 0.0001f;
    // |fast u - IEEE u| <= 2^-21 (max(W, H) + 2) on [-1, W + 1] (rcp 1 ulp, four roundings); the bound tests sit
    // 1e-4 from integers, so any margin above both keeps every decision identical (see k_batch_integrate)
    p.proj_eps = (float)(std::ldexp((double)std::max(in->width, in->height) + 2.0, -21) + 1.2e-4);
    p.unit_len = vol->unit_length;
    return p;
}

static ot_status ensure_mult(ot_tsdf* vol, const ot_intrinsics* in, hipStream_t stream) {
    if (vol->mult_valid && std::memcmp(&vol->mult_intr, in, sizeof(ot_intrinsics)) == 0) return OT_OK;
    if (vol->mult) {
        OT_HIP_TRY(hipStreamSynchronize(stream));
        OT_HIP_TRY(hipFree(vol->mult));
        vol->mult = nullptr;
    }
    OT_HIP_TRY(hipMalloc(&vol->mult, sizeof(float) * (size_t)in->width * in->height));
    ot_status st = ot_depth_multiplier(in, vol->mult, stream);
    if (st != OT_OK) return st;
    vol->mult_intr = *in;
    vol->mult_valid = true;
    return OT_OK;
}

static ot_status check_frame(const ot_tsdf* vol, const void* depth, const uint8_t* color, const ot_intrinsics* in,
                             const double* ext) {
    if (!vol) return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume::Integrate] volume is NULL");
    if (!depth || !in || !ext || in->width <= 0 || in->height <= 0 ||
        (vol->color_type == OT_COLOR_RGB8 && !color))
        return fail(OT_ERR_UNSUPPORTED_FORMAT, "[ScalableTSDFVolume::Integrate] Unsupported image format.");
    return OT_OK;
}

// Grid of k_batch_integrate: INT_GRID_MULT x the co-resident workgroups (cached per device and kernel; a benign race at
// worst computes the same value twice).  A 64-frame batch of the configs[1] scan has ~12k (unit, quarter) items: at 8x
// (16k workgroups) nearly every workgroup takes one item and the dispatcher balances them; at 4x some take two in a
// static stride (0.77 vs 0.72 ms per launch; 6x / 12x / 16x / 32x: within 2 %, slower).
constexpr int INT_GRID_MULT = 8;

// the integrate instantiation of a batch: colour precision 64 (bit 1), reciprocal table (bit 0), fine slices (bit 2:
// 2 voxels per lane along z, 32 waves per unit instead of 16 -- for batches with few units, below)
static int g_int_fine = -1;  // test hook otx_integrate_fine: -1 by the batch's size (default), 0 coarse, 1 fine
constexpr int DEFER_FINE_NUM = 21, DEFER_FINE_DEN = 8;  // units * 16 < 21/8 of the resident workgroups: 336 units
static int g_fine_units = -1;  // its threshold form (deferred integrate: fine below this many units; -1 the default)
static int g_stage_blocks = -1;  // test hook otx_touch_stage_blocks: staging-only touch workgroups (-1: 2 per tile)
// bits 3-4 of a fine variant: the frame pipeline's depth KT - 1 (k_batch_integrate's ZB == 2 loop)
static int g_int_depth = -1;  // test hook otx_integrate_depth: -1 the default (INT_FINE_KT), else KT in 1..3
constexpr int INT_FINE_KT = 1;
static const void* integrate_kernel(int variant) {
    static const void* const k[20] = {
        (const void*)k_batch_integrate<false, false>, (const void*)k_batch_integrate<false, true>,
        (const void*)k_batch_integrate<true, false>, (const void*)k_batch_integrate<true, true>,
        (const void*)k_batch_integrate<false, false, 2, 1>, (const void*)k_batch_integrate<false, true, 2, 1>,
        (const void*)k_batch_integrate<true, false, 2, 1>, (const void*)k_batch_integrate<true, true, 2, 1>,
        nullptr, nullptr, nullptr, nullptr,
        (const void*)k_batch_integrate<false, false, 2, 2>, (const void*)k_batch_integrate<false, true, 2, 2>,
        (const void*)k_batch_integrate<true, false, 2, 2>, (const void*)k_batch_integrate<true, true, 2, 2>,
        nullptr, nullptr, nullptr, nullptr};
    static const void* const k3[4] = {
        (const void*)k_batch_integrate<false, false, 2, 3>, (const void*)k_batch_integrate<false, true, 2, 3>,
        (const void*)k_batch_integrate<true, false, 2, 3>, (const void*)k_batch_integrate<true, true, 2, 3>};
    if ((variant & 4) && ((variant >> 3) & 3) == 2) return k3[variant & 3];
    return k[(variant & 4) ? (variant & 7) + 8 * ((variant >> 3) & 1) : (variant & 3)];
}

static int integrate_grid(int variant) {
    static int cache[32][64] = {{0}};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 4096;
    int* cache_c = cache[variant & 31];
    if (!cache_c[dev]) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, integrate_kernel(variant), 64 * INT_WG, 0) !=
                hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per_cu <= 0 ||
            cus <= 0)
            return 4096;
        cache_c[dev] = per_cu * cus * INT_GRID_MULT;
    }
    return cache_c[dev];
}

// the context a batch's settle (and a replay) needs
struct BatchCtx {
    BatchTouchParams tp;
    IntegrateParams ip0;
    unsigned tiles;
    int n, pc, variant, set;
    bool defer = false;         // deferred integrate (k_integrate_touch / the next flush launches it)
    bool split = false;         // split front end: a replay stages its units' tiles too (units the full hash dropped
    StageMaskParams sq{};       // were in no work list of the first pass, so their footprints were never staged)
    unsigned* smask = nullptr;  // the batch's tile masks (its parity)
};
static ot_status settle_batch(ot_tsdf* vol, const BatchCtx& bc, hipStream_t stream);

// auto (-1): on for sharded volumes (round 6, with their split front end: rank steps at 2 / 4 / 8 sector ranks 2.025 /
// 1.383 / 1.024 ms with it against 2.117 / 1.416 / 1.050 without, r06h; 0.953 vs 0.985 at 8 with coarse slices, r06i),
// off for whole volumes.  Round 5 had found it slower at every shard count when every rank still staged whole frames
// (its cross-stream events cost more than the co-running front end saved: DESIGN_HISTORY.md D).
static bool overlap_on(const ot_tsdf* vol) {
    return vol->overlap_mode > 0 || (vol->overlap_mode < 0 && vol->dev.shard_world > 1);
}
static bool split_on(const ot_tsdf* vol);
static bool tmask_fits(int w, int h);
static bool defer_on(const ot_tsdf* vol, bool split);
// the split front end: sharded volumes.  Its tile masks are written and read on the caller's stream only (mask kernel,
// then staging), so one buffer serves the double-buffered front end too: the integrate on istream never reads them.
static int g_split = -1;  // test hook otx_split_frontend: -1 by the volume (default), 0 never, 1 always (unsharded too)
static bool split_on(const ot_tsdf* vol) {
    const int mode = g_split >= 0 ? g_split : vol->split_mode;
    return mode > 0 || (mode < 0 && vol->dev.shard_world > 1);
}
// tile masks for w x h frames (each split batch's mask kernel writes its frames' maps whole)
static bool tmask_fits(int w, int h) {
    const int tx = (w + STX - 1) / STX;
    return tx <= ST_MAX_TILES_X && (int64_t)((h + STY - 1) / STY) * ((tx + 31) / 32) <= SM_WORDS;
}
static ot_status ensure_tmask(ot_tsdf* vol, int w, int h, hipStream_t stream) {
    if (vol->tmask && vol->tmask_w == w && vol->tmask_h == h) return OT_OK;
    const int64_t words = (int64_t)MAX_BATCH * SM_PARTS * ((h + STY - 1) / STY) * (((w + STX - 1) / STX + 31) / 32);
    if (vol->tmask) {
        OT_HIP_TRY(hipStreamSynchronize(stream));
        OT_HIP_TRY(hipFree(vol->tmask));
        vol->tmask = nullptr;
    }
    OT_HIP_TRY(hipMalloc(&vol->tmask, sizeof(unsigned) * words));
    vol->tmask_words = words;
    vol->tmask_w = w, vol->tmask_h = h;
    note_alloc();
    return OT_OK;
}
// mark the tiles the units of the work list (`wcount` entries) project to, then stage those tiles
static void launch_stage(const BatchFrame* bf, const StageMaskParams& q, const UnitWork* work, const int* wcount,
                         unsigned* smask, const float* mult, hipStream_t stream) {
    hipLaunchKernelGGL(k_stage_mask, dim3((unsigned)q.nframes, SM_PARTS), dim3(256), 0, stream, bf, q, work, wcount,
                       smask);
    hipLaunchKernelGGL(k_stage_tiles, dim3((unsigned)q.tiles_y, (unsigned)q.nframes), dim3(256), 0, stream, bf, mult,
                       (const unsigned*)smask, q.W, q.H, q.tiles_x, q.tiles_y, q.wpr, (int64_t)q.W * q.H);
}
static void* set_work(ot_tsdf* vol, int s) { return s == 0 ? vol->dev.work : vol->bset[1].work; }
// Deferred integrate (round 6): a sharded volume with the split front end launches batch k's integrate together with
// batch k + 1's touch (k_integrate_touch, one stream, no events) -- the default from 4 ranks on (r06k, sector rank steps:
// 0.919 vs 1.003 ms at 8, 1.301 vs 1.336 at 4, but 2.165 vs 2.075 at 2, where the rank's integrate fills the GPU and the
// double-buffered front end stays the default) unless the double-buffered front end is asked for (overlap mode 1)
static int g_defer = -1;  // test hook otx_defer_integrate: -1 by the volume (default), 0 never, 1 with any split batch
static bool defer_on(const ot_tsdf* vol, bool split) {
    if (!split || g_defer == 0 || vol->overlap_mode > 0) return false;
    return g_defer > 0 || vol->dev.shard_world >= 4;
}

// order `stream` after the last batch's integrate when it ran on the volume's integrate stream
static ot_status join_integrate(ot_tsdf* vol, hipStream_t stream) {
    if (vol->last_set >= 0) {
        OT_HIP_TRY(hipStreamWaitEvent(stream, vol->bset[vol->last_set].ev_done, 0));
        vol->last_set = -1;
    }
    return OT_OK;
}

// the second batch set, the integrate stream and the sets' events (once per volume)
static ot_status ensure_overlap(ot_tsdf* vol) {
    if (vol->istream) return OT_OK;
    OT_HIP_TRY(hipStreamCreateWithFlags(&vol->istream, hipStreamNonBlocking));
    if (!vol->wcount) OT_HIP_TRY(hipMalloc(&vol->wcount, sizeof(int) * 4));  // [set]: length, [2 + set]: heavy units
    if (!vol->bset[1].bframes) OT_HIP_TRY(hipMalloc(&vol->bset[1].bframes, sizeof(BatchFrame) * MAX_BATCH));
    if (!vol->bset[1].work) OT_HIP_TRY(hipMalloc(&vol->bset[1].work, sizeof(UnitWork) * vol->hash_cap));
    for (auto& b : vol->bset) {
        if (!b.ev_units) OT_HIP_TRY(hipEventCreateWithFlags(&b.ev_units, hipEventDisableTiming));
        if (!b.ev_done) OT_HIP_TRY(hipEventCreateWithFlags(&b.ev_done, hipEventDisableTiming));
    }
    note_alloc();
    return OT_OK;
}

// Launch the deferred batch's integrate on `stream`: with the touch of batch `next` in one launch (k_integrate_touch), or
// alone (next == nullptr: a flush).  Coarse slices, the variant's colour precision and division form.
static ot_status launch_deferred(ot_tsdf* vol, hipStream_t stream, const BatchCtx* next) {
    if (!vol->dfr_on) return OT_OK;
    BatchCtx D;
    std::memcpy(&D, vol->dfr_ctx, sizeof(BatchCtx));
    vol->dfr_on = false;
    if (stream != vol->dfr_stream) {  // the batch's front end ran on another stream
        if (!vol->ev_dfr) OT_HIP_TRY(hipEventCreateWithFlags(&vol->ev_dfr, hipEventDisableTiming));
        OT_HIP_TRY(hipEventRecord(vol->ev_dfr, vol->dfr_stream));
        OT_HIP_TRY(hipStreamWaitEvent(stream, vol->ev_dfr, 0));
    }
    const BatchFrame* bf = vol->bset[D.set].bframes;
    const UnitWork* uw = (const UnitWork*)set_work(vol, D.set);
    const int* wc = vol->wcount + D.set;
    // coarse, or fine slices for a batch of few units: its count is known here (settle_batch read the mail of its
    // units kernel; the direct path guesses it from the previous batch), the rule of integrate_batch
    int variant = D.variant & 3;
    {
        const int64_t units = vol->last_batch_slots;
        const int resident = integrate_grid(variant) / INT_GRID_MULT;
        // below DEFER_FINE_UNITS: 8 sector ranks' batches of 135 / 161 / 317 units ran fine in 112 / 126 / 131 us
        // against 146 / 146 / 142 coarse, one of 367 units 167 against 148 (r06fn); a fraction of the resident
        // workgroups, as the direct path's rule
        const bool small = g_fine_units >= 2 ? units >= 0 && units < g_fine_units
                                             : units >= 0 && units * INT_PARTS * 4 * DEFER_FINE_DEN <
                                                                 (int64_t)resident * DEFER_FINE_NUM;
        if (g_int_fine > 0 || ((g_int_fine < 0 || g_fine_units >= 2) && small))
            variant |= 4 | ((INT_FINE_KT - 1) << 3);
    }
    const bool fine = (variant & 4) != 0;
    const int nint = integrate_grid(variant);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (vol->profiling) {
        OT_HIP_TRY(hipEventCreate(&e0));
        OT_HIP_TRY(hipEventCreate(&e1));
        OT_HIP_TRY(hipEventRecord(e0, stream));
    }
    if (next) {
        const BatchFrame* tf = vol->bset[next->set].bframes;
        BatchTouchParams tp = next->tp;
        int tn = next->n;
        int ni = nint;
        void* args[] = {(void*)&bf, (void*)&D.ip0, (void*)&vol->dev, (void*)&uw, (void*)&wc, (void*)&ni,
                        (void*)&tf, (void*)&tp, (void*)&tn};
        static const void* const kt[8] = {
            (const void*)k_integrate_touch<false, false>,      (const void*)k_integrate_touch<false, true>,
            (const void*)k_integrate_touch<true, false>,       (const void*)k_integrate_touch<true, true>,
            (const void*)k_integrate_touch_fine<false, false>, (const void*)k_integrate_touch_fine<false, true>,
            (const void*)k_integrate_touch_fine<true, false>,  (const void*)k_integrate_touch_fine<true, true>};
        const unsigned grid = (unsigned)nint + next->tiles * (unsigned)((tn + tp.tf - 1) / tp.tf);
        OT_HIP_TRY(hipLaunchKernel(kt[(variant & 3) + (fine ? 4 : 0)], dim3(grid), dim3(64 * INT_WG), args, 0, stream));
    } else {
        void* args[] = {(void*)&bf, (void*)&D.ip0, (void*)&vol->dev, (void*)&uw, (void*)&wc};
        OT_HIP_TRY(hipLaunchKernel(integrate_kernel(variant), dim3(nint), dim3(64 * INT_WG), args, 0, stream));
    }
    OT_LAUNCH_CHECK();
    if (vol->profiling) {
        OT_HIP_TRY(hipEventRecord(e1, stream));
        vol->prof_events.emplace_back(e0, e1);
    }
    return OT_OK;
}

static ot_status integrate_batch(ot_tsdf* vol, const PendingFrame* frames, int n, hipStream_t stream) {
    const ot_intrinsics& in = frames[0].intr;
    ot_status st = wait_normals(vol, stream);  // deferred vertex normals of the last mesh still read the volume
    if (st != OT_OK) return st;
    st = ensure_mult(vol, &in, stream);
    if (st != OT_OK) return st;
    const bool split = split_on(vol) && tmask_fits(in.width, in.height);
    const bool defer = defer_on(vol, split);
    const bool ovl = !defer && overlap_on(vol);
    if ((ovl || defer) && (st = ensure_overlap(vol)) != OT_OK) return st;
    const int set = (ovl || defer) ? vol->bset_next : 0;
    if (ovl || defer) vol->bset_next ^= 1;
    auto& bs = vol->bset[set];
    // (deferred: the set's last batch was integrated inside the launch with the previous batch's touch, queued on
    // this stream before that batch's units kernel -- done before anything below restages the set)
    // the set's previous batch (two batches ago) must have finished its integrate before its buffers are restaged
    // (an event never recorded counts as complete)
    if (ovl) OT_HIP_TRY(hipStreamWaitEvent(stream, bs.ev_done, 0));
    const int64_t npx = (int64_t)in.width * in.height;
    if (bs.cap < npx * n) {
        if (bs.bdm) {
            OT_HIP_TRY(hipStreamSynchronize(stream));
            if (vol->istream) OT_HIP_TRY(hipStreamSynchronize(vol->istream));
            OT_HIP_TRY(hipFree(bs.bdm));
            OT_HIP_TRY(hipFree(bs.brgba));
            bs.bdm = nullptr;
            bs.brgba = nullptr;
        }
        const int64_t cap = npx * std::max(n, std::min(vol->batch_max, MAX_BATCH));
        OT_HIP_TRY(hipMalloc(&bs.bdm, sizeof(float2) * cap));
        OT_HIP_TRY(hipMalloc(&bs.brgba, sizeof(uint32_t) * cap));
        bs.cap = cap;
    }
    // per-frame parameters: pinned host staging (double-buffered, event-guarded) -> device
    const int hb = vol->hb_next;  // (the last batch from this half was copied: settle_batch saw its units kernel mail)
    vol->hb_next ^= 1;
    BatchFrame* host = vol->hbframes + hb * MAX_BATCH;
    BatchCtx bc;
    bc.ip0 = make_integrate_params(vol, nullptr, nullptr, vol->mult, &in, frames[0].extrinsic);
    for (int k = 0; k < n; ++k) {
        const PendingFrame& f = frames[k];
        BatchFrame& b = host[k];
        b.depth16 = f.depth;
        b.depthf = f.depth ? nullptr : f.depthf;
        b.color = (vol->color_type == OT_COLOR_RGB8) ? f.color : nullptr;
        b.dm = bs.bdm + npx * k;
        b.rgba = bs.brgba + npx * k;
        double pose[16];
        inverse4(f.extrinsic, pose);
        for (int i = 0; i < 12; ++i) b.pose[i] = pose[i];
        float E[16];
        for (int i = 0; i < 16; ++i) E[i] = (float)f.extrinsic[i];
        for (int i = 0; i < 12; ++i) b.E[i] = E[i];
        b.es[0] = E[0 * 4 + 2] * bc.ip0.vl;
        b.es[1] = E[1 * 4 + 2] * bc.ip0.vl;
        b.es[2] = E[2 * 4 + 2] * bc.ip0.vl;
        b.scale = (float)f.depth_scale;
        b.trunc = f.depth_trunc;
    }
    hipLaunchKernelGGL(k_copy_frames, dim3(1), dim3(COPY_FRAMES_LANES), 0, stream, (const uint4*)host,
                       (uint4*)bs.bframes, (int)(sizeof(BatchFrame) / 16) * n);
    // this batch's pair counter: zeroed by reset, or by the previous batch's k_batch_units (no memset here)
    const int pc = vol->batch_pc;
    BatchTouchParams& tp = bc.tp;
    tp.mult = vol->mult;
    tp.npx = npx;
    tp.pc = pc;
    tp.W = in.width;
    tp.stride = vol->stride;
    tp.ws = (in.width + vol->stride - 1) / vol->stride;
    tp.hs = (in.height + vol->stride - 1) / vol->stride;
    tp.fx = in.fx;
    tp.fy = in.fy;
    tp.cx = in.cx;
    tp.cy = in.cy;
    tp.trunc = vol->sdf_trunc;
    tp.unit_len = vol->unit_length;
    tp.inv_unit = 1.0 / vol->unit_length;
    tp.slot_cap = (int)vol->hash_cap;
    bc.tiles = (unsigned)(((tp.ws + TT - 1) / TT) * ((tp.hs + TT - 1) / TT));
    tp.tiles = (int)bc.tiles;
    tp.stage_blocks = g_stage_blocks < 0 ? 2 * (int)bc.tiles : g_stage_blocks;
    tp.tf = g_touch_tf;
    // sharded volume: split front end (touch without staging -> units -> tile mask -> staging of the marked tiles)
    tp.sample_stage = split ? 1 : 0;
    if (split) {
        tp.stage_blocks = -1;
        if ((st = ensure_tmask(vol, in.width, in.height, stream)) != OT_OK) return st;
    }
    bc.n = n;
    bc.pc = pc;
    bc.set = set;
    bc.defer = defer;
    hipEvent_t f0 = nullptr, f1 = nullptr;  // front end (staging + touch + units): the part a sharded volume repeats
    if (vol->profiling) {
        OT_HIP_TRY(hipEventCreate(&f0));
        OT_HIP_TRY(hipEventCreate(&f1));
        OT_HIP_TRY(hipEventRecord(f0, stream));
    }
    UnitWork* work = (UnitWork*)set_work(vol, set);
    int* wcount = (ovl || defer) ? vol->wcount + set : vol->dev.counters + pc;
    if (defer && vol->dfr_on) {  // the last batch's integrate and this batch's touch in one launch
        if ((st = launch_deferred(vol, stream, &bc)) != OT_OK) return st;
    } else if (split) {
        hipLaunchKernelGGL(k_batch_touch_split, dim3(bc.tiles, (unsigned)((n + tp.tf - 1) / tp.tf)), dim3(256), 0,
                           stream, (const BatchFrame*)bs.bframes, tp, vol->dev, n);
    } else {
        hipLaunchKernelGGL(k_batch_touch<false>,
                           dim3(bc.tiles + (unsigned)std::max(0, tp.stage_blocks), (unsigned)((n + tp.tf - 1) / tp.tf)),
                           dim3(256), 0, stream, (const BatchFrame*)bs.bframes, tp, vol->dev, n);
    }
    hipLaunchKernelGGL(k_batch_units<false>, dim3(256), dim3(256), 0, stream, vol->dev, work, pc,
                       vol->hmail + OT_MAIL_WORDS, (ovl || defer) ? wcount : (int*)nullptr, ++vol->units_seq);
    if (split) {
        StageMaskParams q;
        q.W = in.width;
        q.H = in.height;
        q.tiles_x = (in.width + STX - 1) / STX;
        q.tiles_y = (in.height + STY - 1) / STY;
        q.wpr = (q.tiles_x + 31) / 32;
        q.fx = bc.ip0.fx, q.fy = bc.ip0.fy, q.cx = bc.ip0.cx, q.cy = bc.ip0.cy;
        q.vl = bc.ip0.vl, q.half = bc.ip0.half;
        q.unit_len = vol->unit_length;
        q.nframes = n;
        bc.split = true;
        bc.sq = q;
        bc.smask = vol->tmask;
        launch_stage((const BatchFrame*)bs.bframes, q, (const UnitWork*)work, (const int*)wcount, vol->tmask,
                     (const float*)vol->mult, stream);
    }
    // reciprocal-table kernel while every weight + 1 is an integer <= RCP_N: weights count updates, at most one
    // per frame since reset, unless units were imported (k_batch_integrate: Markstein's exact correction)
    const bool fast = !vol->imported && (int64_t)vol->frame_id + n < RCP_N;
    bc.variant = (vol->color64 ? 2 : 0) + (fast ? 1 : 0);
    // Few units (a spatial shard, a small object): a (unit, quarter) item is a chain of the batch's frames, each frame
    // two dependent gather round trips plus ~270 dependent VALU instructions, so a batch too small to fill the GPU is
    // bound by that chain -- ~130 us per 64 frames whatever the unit count (tools/shard_scaling.py, r05g: rank 0 of
    // 16 / 32 / 64 shards 142 / 134 / 132 us).  Such batches take the fine slices (2 voxels per lane along z, twice
    // the items, the next frame's gathers issued beside this frame's colour gathers: 107 / 90 / 85 us; the same
    // per-voxel arithmetic, the same bits).  With a quarter of the GPU's resident workgroups in items or more the
    // coarse slices are as fast or faster (1/8 shard 167 / 167 us, 1/4 242 / 280 us).  The unit count of a batch is
    // known on the device only: the previous batch's (mailed) stands in for it, and a sharded volume's first batch
    // counts as small from 16 ranks on.
    {
        const int resident = integrate_grid(bc.variant) / INT_GRID_MULT;
        // 2..15 ranks: coarse always.  A sector rank's batches swing between a few units and a full arc (r06e, rank 0
        // of 8: 135 / 677 / 662 / 317 units), so the previous batch mispredicts: the 677-unit batch took 214 us fine
        // against ~145 us coarse, and coarse-only steps were the faster (0.985 vs 1.053 ms, r06i)
        const int64_t est = vol->dev.shard_world > 1 && vol->dev.shard_world < 16 ? (int64_t)1 << 30
                            : vol->last_batch_slots >= 0 ? vol->last_batch_slots
                                                         : (vol->dev.shard_world >= 16 ? 0 : (int64_t)1 << 30);
        const bool fine = !defer && (g_int_fine > 0 || (g_int_fine < 0 && est * INT_PARTS * 4 < (int64_t)resident * 3));
        if (fine) bc.variant |= 4 | (((g_int_depth > 0 ? g_int_depth : INT_FINE_KT) - 1) << 3);
    }
    if (defer) {  // the integrate waits for the next batch's touch (or the next flush)
        if (vol->profiling) {
            OT_HIP_TRY(hipEventRecord(f1, stream));
            vol->prof_fe_events.emplace_back(f0, f1);
        }
        static_assert(sizeof(BatchCtx) <= sizeof(vol->dfr_ctx), "deferred batch context");
        std::memcpy(vol->dfr_ctx, &bc, sizeof(BatchCtx));
        vol->dfr_on = true;
        vol->dfr_stream = stream;
        vol->batch_pc ^= 1;
        vol->frame_id += n;
        vol->sorted_frame = -1;
        vol->early_frame = vol->frame_id;
        return settle_batch(vol, bc, stream);
    }
    const int grid = integrate_grid(bc.variant);
    // overlap: the integrate on istream behind this set's units kernel (and the previous batch's integrate: same
    // stream), so the caller's stream is free for the next batch's front end
    hipStream_t is = stream;
    if (ovl) {
        OT_HIP_TRY(hipEventRecord(bs.ev_units, stream));
        OT_HIP_TRY(hipStreamWaitEvent(vol->istream, bs.ev_units, 0));
        is = vol->istream;
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (vol->profiling) {
        OT_HIP_TRY(hipEventRecord(f1, stream));
        vol->prof_fe_events.emplace_back(f0, f1);
        OT_HIP_TRY(hipEventCreate(&e0));
        OT_HIP_TRY(hipEventCreate(&e1));
        OT_HIP_TRY(hipEventRecord(e0, is));
    }
    const BatchFrame* bf = bs.bframes;
    const UnitWork* uw = work;
    const int* wc = wcount;
    void* args[] = {(void*)&bf, (void*)&bc.ip0, (void*)&vol->dev, (void*)&uw, (void*)&wc};
    OT_HIP_TRY(hipLaunchKernel(integrate_kernel(bc.variant), dim3(grid), dim3(64 * INT_WG), args, 0, is));
    vol->batch_pc ^= 1;  // only once this batch's kernels are queued (its units kernel zeroes the other counter)
    OT_LAUNCH_CHECK();
    if (vol->profiling) {
        OT_HIP_TRY(hipEventRecord(e1, is));
        vol->prof_events.emplace_back(e0, e1);
    }
    if (ovl) {
        OT_HIP_TRY(hipEventRecord(bs.ev_done, is));
        vol->last_set = set;
    }
    vol->frame_id += n;
    vol->sorted_frame = -1;
    vol->early_frame = vol->frame_id;  // the mailed counters are final for this frame count (see units_seq)
    return settle_batch(vol, bc, stream);
}

// ------------------------------------------------------------------------------------------ unbounded unit pool
// Open3D's ScalableTSDFVolume allocates blocks without bound (a fixed pool dropped units and failed at the
// next read, outside the reference caller's per-frame try/except).  Here the pool grows: records, keys and the sorted
// order are copied into pools twice as large (or more), and the hash is rebuilt from the unit keys at >= 4x the pool.

__global__ __launch_bounds__(256) void k_rehash(TsdfDev d, int n) {
    const int id = blockIdx.x * 256 + threadIdx.x;
    if (id >= n) return;
    const int slot = hash_insert(d, pack_key(d.unit_keys[id * 3], d.unit_keys[id * 3 + 1], d.unit_keys[id * 3 + 2]));
    if (slot < 0) atomicOr(&d.counters[C_HASHERR], 1);  // cannot happen: capacity >= 4x the units
    else d.hvals[slot] = id;
}

// Grow to hold at least `need` units (stream-ordered copies; the stream is synchronised first: the kernels queued on
// the volume may still read the old buffers).  Every allocation is made before any old buffer is freed, so a failed
// allocation leaves the volume as it was and is reported as the error of the call that needed the room.
static ot_status grow_pool(ot_tsdf* vol, int64_t need, int n_used, hipStream_t stream) {
    constexpr int64_t MAX_UNITS = 1 << 24;
    if (need > MAX_UNITS) return fail(OT_ERR_CAPACITY, "[ScalableTSDFVolume] more than 2^24 units");
    int64_t nmax = std::max<int64_t>(2 * vol->max_units, need + need / 2);
    nmax = std::min<int64_t>(nmax, MAX_UNITS);
    int64_t cap = 1;
    while (cap < 4 * nmax) cap <<= 1;
    ot_status st = wait_normals(vol, stream);
    if (st != OT_OK) return st;
    OT_HIP_TRY(hipStreamSynchronize(stream));
    if (vol->istream) OT_HIP_TRY(hipStreamSynchronize(vol->istream));
    TsdfDev& d = vol->dev;
    TsdfDev nd = d;
    unsigned* nsorted = nullptr;
    void* work1 = nullptr;
    void* fresh[9] = {nullptr};
    auto alloc = [&](void** p, size_t bytes, int k) {
        const hipError_t e = hipMalloc(p, bytes);
        fresh[k] = *p;
        return e;
    };
    hipError_t e = hipSuccess;
    if ((e = alloc((void**)&nd.vox, sizeof(float) * (size_t)d.unit_floats * nmax, 0)) == hipSuccess &&
        (e = alloc((void**)&nd.unit_keys, sizeof(int) * 3 * nmax, 1)) == hipSuccess &&
        (e = alloc((void**)&nsorted, sizeof(unsigned) * nmax, 2)) == hipSuccess &&
        (e = alloc((void**)&nd.hkeys, sizeof(unsigned long long) * cap, 3)) == hipSuccess &&
        (e = alloc((void**)&nd.hvals, sizeof(int) * cap, 4)) == hipSuccess &&
        (e = alloc((void**)&nd.fmask, sizeof(unsigned long long) * cap, 5)) == hipSuccess &&
        (e = alloc((void**)&nd.bslots, sizeof(int) * cap, 6)) == hipSuccess &&
        (e = alloc((void**)&nd.work, sizeof(UnitWork) * cap, 7)) == hipSuccess &&
        (!vol->bset[1].work || (e = alloc(&work1, sizeof(UnitWork) * cap, 8)) == hipSuccess)) {
    }
    if (e != hipSuccess) {
        for (void* p : fresh)
            if (p) (void)hipFree(p);
        (void)hipGetLastError();
        return fail(OT_ERR_HIP, std::string("[ScalableTSDFVolume] allocation failed while growing the unit pool to ") +
                                    std::to_string(nmax) + " units: " + hipGetErrorString(e));
    }
    note_alloc();
    const size_t rec = sizeof(float) * (size_t)d.unit_floats;
    if (n_used > 0) {
        OT_HIP_TRY(hipMemcpyAsync(nd.vox, d.vox, rec * n_used, hipMemcpyDeviceToDevice, stream));
        OT_HIP_TRY(hipMemcpyAsync(nd.unit_keys, d.unit_keys, sizeof(int) * 3 * n_used, hipMemcpyDeviceToDevice, stream));
        OT_HIP_TRY(hipMemcpyAsync(nsorted, vol->sorted_ids, sizeof(unsigned) * n_used, hipMemcpyDeviceToDevice, stream));
    }
    OT_HIP_TRY(hipMemsetAsync(nd.hkeys, 0xFF, sizeof(unsigned long long) * cap, stream));
    OT_HIP_TRY(hipMemsetAsync(nd.hvals, 0xFF, sizeof(int) * cap, stream));
    OT_HIP_TRY(hipMemsetAsync(nd.fmask, 0, sizeof(unsigned long long) * cap, stream));
    nd.hash_mask = (int)(cap - 1);
    nd.max_units = (int)nmax;
    if (n_used > 0) hipLaunchKernelGGL(k_rehash, dim3((unsigned)((n_used + 255) / 256)), dim3(256), 0, stream, nd, n_used);
    OT_LAUNCH_CHECK();
    OT_HIP_TRY(hipStreamSynchronize(stream));
    for (void* p : {(void*)d.vox, (void*)d.unit_keys, (void*)vol->sorted_ids, (void*)d.hkeys, (void*)d.hvals,
                    (void*)d.fmask, (void*)d.bslots, d.work, vol->bset[1].work})
        if (p) (void)hipFree(p);
    d = nd;
    vol->bset[1].work = work1;
    vol->sorted_ids = nsorted;
    vol->max_units = nmax;
    vol->hash_cap = cap;
    return OT_OK;
}

// After each batch: the counters its units kernel mailed (mail_wait on units_seq: the host waits for the units kernel,
// not for the integrate queued behind it, so the GPU keeps its queue).  Units the pool could not hold (C_OVERFLOW), or keys the
// hash could not hold (C_HASHERR bit 0), were skipped by the batch's integrate: grow, then replay the batch for exactly
// those units -- touch again from the staged depths (still resident: the next batch has not been staged yet), allocate
// the missing units (units that have an id were integrated and are skipped), integrate them with the batch's frames.
// Units are independent and each sees the batch's frames in call order, so the volume equals an unbounded pool's.
// A pool more than 3/4 full also grows here, ahead of need.
static ot_status settle_batch(ot_tsdf* vol, const BatchCtx& bc, hipStream_t stream) {
    for (int round = 0;; ++round) {
        ot_status ws = mail_wait(vol->hmail + MAIL_SEQ_UNITS, vol->units_seq, stream);
        if (ws != OT_OK) return ws;
        int c[N_COUNTERS];
        std::memcpy(c, vol->hmail + OT_MAIL_WORDS, sizeof(c));
        vol->last_batch_slots = c[bc.pc];  // units the batch touched: the next batch's item estimate
        if (round == 0) {
            ++vol->stat_batches;
            vol->stat_unit_batches += c[bc.pc];
        }
        const bool short_of_room = c[C_OVERFLOW] != 0 || (c[C_HASHERR] & 1) != 0;
        if (!short_of_room) {
            if (vol->stat_prev_units >= 0) vol->stat_fresh += c[C_UNITS] - vol->stat_prev_units;
            vol->stat_prev_units = c[C_UNITS];
            if ((int64_t)c[C_UNITS] * 4 > vol->max_units * 3)
                return grow_pool(vol, (int64_t)c[C_UNITS] * 2, c[C_UNITS], stream);
            return OT_OK;
        }
        if (round >= 8) return fail(OT_ERR_CAPACITY, "[ScalableTSDFVolume] unit pool: growth did not converge");
        // ids below the old capacity were all handed out; the allocations past it were dropped (C_UNITS overshoots)
        const int used = (int)std::min<int64_t>(c[C_UNITS], vol->max_units);
        const int64_t need = std::max<int64_t>((int64_t)c[C_UNITS], vol->max_units) + 1;
        ot_status st = grow_pool(vol, need, used, stream);  // synchronises both of the volume's streams
        if (st != OT_OK) return st;
        int h[N_COUNTERS];
        OT_HIP_TRY(hipMemcpy(h, vol->dev.counters, sizeof(h), hipMemcpyDeviceToHost));
        h[C_UNITS] = used;
        h[C_OVERFLOW] = 0;
        h[C_HASHERR] &= ~1;
        h[bc.pc] = 0;  // the replay's touched-slot count (the batch's own pair counter; the next batch's stays zero)
        OT_HIP_TRY(hipMemcpy(vol->dev.counters, h, sizeof(h), hipMemcpyHostToDevice));
        // the replay, all on the caller's stream, from the batch's set (its staging is intact: nothing restaged it)
        BatchTouchParams tp = bc.tp;
        tp.slot_cap = (int)vol->hash_cap;
        const BatchFrame* bf = vol->bset[bc.set].bframes;
        UnitWork* work = (UnitWork*)set_work(vol, bc.set);
        hipLaunchKernelGGL(k_batch_touch<true>, dim3(bc.tiles, (unsigned)((bc.n + tp.tf - 1) / tp.tf)), dim3(256), 0, stream,
                           bf, tp, vol->dev, bc.n);
        if (bc.defer) {  // nothing of the batch is integrated yet: rebuild its whole work list, restage, stay deferred
            hipLaunchKernelGGL(k_batch_units<false>, dim3(256), dim3(256), 0, stream, vol->dev, work, bc.pc,
                               vol->hmail + OT_MAIL_WORDS, vol->wcount + bc.set, ++vol->units_seq);
            launch_stage(bf, bc.sq, (const UnitWork*)work, (const int*)(vol->wcount + bc.set), bc.smask,
                         (const float*)vol->mult, stream);
            OT_LAUNCH_CHECK();
            continue;
        }
        hipLaunchKernelGGL(k_batch_units<true>, dim3(256), dim3(256), 0, stream, vol->dev, work, bc.pc,
                           vol->hmail + OT_MAIL_WORDS, (int*)nullptr, ++vol->units_seq);
        if (bc.split) {  // the replayed units' tiles, from the caller's frames (valid until this flush returns)
            launch_stage(bf, bc.sq, (const UnitWork*)work, (const int*)(vol->dev.counters + bc.pc), bc.smask,
                         (const float*)vol->mult, stream);
        }
        const UnitWork* uw = work;
        const int* wc = vol->dev.counters + bc.pc;
        void* args[] = {(void*)&bf, (void*)&bc.ip0, (void*)&vol->dev, (void*)&uw, (void*)&wc};
        OT_HIP_TRY(hipLaunchKernel(integrate_kernel(bc.variant), dim3(integrate_grid(bc.variant)), dim3(64 * INT_WG),
                                   args, 0, stream));
        OT_LAUNCH_CHECK();
        vol->last_set = -1;  // the replay ran on the caller's stream, after both streams drained
        vol->sorted_frame = -1;
    }
}

// room for `extra` more units before a kernel that allocates up to that many (imports): grow now if needed
static ot_status reserve_units(ot_tsdf* vol, int64_t extra, hipStream_t stream) {
    int nu = 0;
    OT_HIP_TRY(hipMemcpyAsync(&nu, vol->dev.counters + C_UNITS, sizeof(int), hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipStreamSynchronize(stream));
    const int used = (int)std::min<int64_t>(nu, vol->max_units);
    if (used + extra <= vol->max_units) return OT_OK;
    return grow_pool(vol, used + extra, used, stream);
}

ot_status wait_normals(ot_tsdf* vol, hipStream_t stream) {
    if (!vol->normals_pending) return OT_OK;
    const hipError_t q = hipEventQuery(vol->ev_normals);
    if (q == hipSuccess) {
        vol->normals_pending = false;
        return OT_OK;
    }
    if (q != hipErrorNotReady) OT_HIP_TRY(q);
    OT_HIP_TRY(hipStreamWaitEvent(stream, vol->ev_normals, 0));
    return OT_OK;
}

ot_status tsdf_flush(ot_tsdf* vol, hipStream_t stream, bool join) {
    size_t i = 0;
    std::vector<PendingFrame> frames;
    frames.swap(vol->pending);
    if (!frames.empty()) vol->mesh.valid = false;  // the volume changes: the last extraction's structure is stale
    while (i < frames.size()) {
        // a batch: consecutive frames with identical intrinsics, at most batch_max (<= 64)
        size_t n = 1;
        const int cap = std::min(vol->batch_max, MAX_BATCH);
        while (i + n < frames.size() && (int)n < cap &&
               std::memcmp(&frames[i + n].intr, &frames[i].intr, sizeof(ot_intrinsics)) == 0)
            ++n;
        ot_status st = integrate_batch(vol, frames.data() + i, (int)n, stream);
        if (st != OT_OK) return st;
        i += n;
    }
    if (!join) return OT_OK;
    ot_status st = launch_deferred(vol, stream, nullptr);  // a reader needs the last batch integrated
    if (st != OT_OK) return st;
    return join_integrate(vol, stream);
}

static ot_status counter_errors(const int* c) {
    if (c[C_OVERFLOW]) return fail(OT_ERR_CAPACITY, "[ScalableTSDFVolume] volume unit pool exhausted (max_units)");
    if (c[C_HASHERR] & 1) return fail(OT_ERR_CAPACITY, "[ScalableTSDFVolume] unit hash table full");
    if (c[C_HASHERR] & 2) return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] unit index out of range");
    return OT_OK;
}

// one wave copies n <= OT_MAIL_WORDS 4-byte words into the volume's pinned coherent mailbox (plain vector stores over
// PCIe); the caller synchronises the stream and reads vol->hmail.  One launch replaces a staged D2H copy per value
__global__ void k_mail_words(MailSrc s, unsigned* __restrict__ out) {
    const int i = threadIdx.x;
    if (i < s.n) out[i] = *s.p[i];
}

ot_status mail_words(ot_tsdf* vol, const MailSrc& s, hipStream_t stream) {
    if (s.n > MAIL_SEQ_MC) return fail(OT_ERR_INVALID_ARGUMENT, "mailbox overflow");
    hipLaunchKernelGGL(k_mail_words, dim3(1), dim3(64), 0, stream, s, vol->hmail);
    OT_LAUNCH_CHECK();
    OT_HIP_TRY(hipStreamSynchronize(stream));
    return OT_OK;
}

// The stream is polled only once the wait has lasted 20 ms (then every ~1 ms): a stream query puts commands on the
// stream's queue, and while the host spins the queue already holds the work launched after the mailing kernel -- polling
// every ~20 us had left ~6 us of idle GPU behind that work at each wait (host launch trace against the kernel trace,
// tools/launch_lag.py, r05ah: the gaps before the unit sort and before the sampler).
// Host CPU bound: the loop spins with `pause` only for the first ~50 us -- the mails the headline
// waits for arrive within that (the units kernel ~10 us after the touch, the marching-cubes totals) -- then yields the
// core on every check (sched_yield: a rank's other threads and RCCL's proxy threads get it), and past 2 ms sleeps
// 20 us per check, so 8 ranks x 2 object streams waiting on a long kernel do not hold 16 cores at 100 %.
ot_status mail_wait(const unsigned* word, unsigned seq, hipStream_t stream) {
    using clk = std::chrono::steady_clock;
    const clk::time_point t0 = clk::now();
    const clk::time_point t_yield = t0 + std::chrono::microseconds(50);
    const clk::time_point t_sleep = t0 + std::chrono::milliseconds(2);
    clk::time_point next = t0 + std::chrono::milliseconds(20);
    for (unsigned it = 1;; ++it) {
        if (__atomic_load_n(word, __ATOMIC_ACQUIRE) == seq) return OT_OK;
        const bool spin = (it & 63u) != 0;
        if (spin && it < (1u << 20)) {  // the clock is read every 64 polls while spinning
            __builtin_ia32_pause();
            continue;
        }
        const clk::time_point now = clk::now();
        if (now < t_yield) {
            __builtin_ia32_pause();
            continue;
        }
        it = 1u << 20;  // from here every poll reads the clock
        if (now >= next) {  // has the stream faulted, or drained without the mail?
            next = now + std::chrono::milliseconds(1);
            const hipError_t q = hipStreamQuery(stream);
            if (q == hipSuccess) {
                if (__atomic_load_n(word, __ATOMIC_ACQUIRE) == seq) return OT_OK;
                return fail(OT_ERR_HIP, "mailbox: the stream drained without the kernel's mail");
            }
            if (q != hipErrorNotReady) OT_HIP_TRY(q);
        }
        if (now < t_sleep) sched_yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

static ot_status check_errors(ot_tsdf* vol, hipStream_t stream) {
    int c[N_COUNTERS];
    OT_HIP_TRY(hipMemcpyAsync(c, vol->dev.counters, sizeof(c), hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipStreamSynchronize(stream));
    if (c[C_OVERFLOW]) return fail(OT_ERR_CAPACITY, "[ScalableTSDFVolume] volume unit pool exhausted (max_units)");
    if (c[C_HASHERR] & 1) return fail(OT_ERR_CAPACITY, "[ScalableTSDFVolume] unit hash table full");
    if (c[C_HASHERR] & 2) return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] unit index out of range");
    return OT_OK;
}

ot_status tsdf_sorted_units(ot_tsdf* vol, hipStream_t stream, int64_t* n_units) {
    ot_status st = tsdf_flush(vol, stream);
    if (st != OT_OK) return st;
    int c[N_COUNTERS];  // error flags and the unit count in one read-back (the pinned mailbox)
    if (vol->early_frame == vol->frame_id && !vol->imported && vol->units_seq != 0) {
        // mailed by the last batch's units kernel (settle_batch saw it): not waiting for the integrate behind it
        st = mail_wait(vol->hmail + MAIL_SEQ_UNITS, vol->units_seq, stream);
        if (st != OT_OK) return st;
        std::memcpy(c, vol->hmail + OT_MAIL_WORDS, sizeof(c));
    } else {
        MailSrc ms;
        ms.n = N_COUNTERS;
        for (int i = 0; i < N_COUNTERS; ++i) ms.p[i] = (const unsigned*)vol->dev.counters + i;
        st = mail_words(vol, ms, stream);
        if (st != OT_OK) return st;
        std::memcpy(c, vol->hmail, sizeof(c));
    }
    st = counter_errors(c);
    if (st != OT_OK) return st;
    int nu = (int)std::min<int64_t>(c[C_UNITS], vol->max_units);
    *n_units = nu;
    if (vol->sorted_frame == vol->frame_id && vol->sorted_units == nu) return OT_OK;
    if (nu > 0) {
        int hb[6];  // per-axis key bounds, kept by the allocating kernels (note_unit_key)
        for (int a = 0; a < 3; ++a) {
            hb[a] = KEY_BIAS + 1 - c[C_KNEG + a];
            hb[3 + a] = c[C_KMAX + a] - KEY_BIAS - 1;
        }
        int bits[3];
        for (int a = 0; a < 3; ++a) {
            const long long span = (long long)hb[3 + a] - hb[a];
            bits[a] = 1;
            while (bits[a] < 31 && (span >> bits[a]) != 0) ++bits[a];
        }
        const UnitKeyPack pk{hb[0], hb[1], hb[2], bits[2], bits[1] + bits[2]};
        const int kb = bits[0] + bits[1] + bits[2];
        if (kb <= USORT_BITS && !g_unit_sort_radix) {
            hipLaunchKernelGGL(k_unit_rank_sort, dim3(1), dim3(1024), 0, stream, vol->dev, nu, pk, kb, vol->sorted_ids);
            OT_LAUNCH_CHECK();
            vol->sorted_units = nu;
            vol->sorted_frame = vol->frame_id;
            return OT_OK;
        }
        char* ws = (char*)scratch((size_t)nu * 24 + 256, 5);
        if (!ws) return fail(OT_ERR_HIP, "scratch allocation failed");
        unsigned long long* kin = (unsigned long long*)(ws + 256);
        unsigned long long* kout = kin + nu;
        unsigned* vin = (unsigned*)(kout + nu);
        hipLaunchKernelGGL(k_pack_unit_keys, dim3((nu + 255) / 256), dim3(256), 0, stream, vol->dev, nu, pk, kin, vin);
        OT_LAUNCH_CHECK();
        st = sort_pairs_u64_u32(kin, kout, vin, vol->sorted_ids, (size_t)nu, std::min(63, bits[0] + bits[1] + bits[2]),
                                stream, 3);
        if (st != OT_OK) return st;
    }
    vol->sorted_units = nu;
    vol->sorted_frame = vol->frame_id;
    return OT_OK;
}

}  // namespace ot

using namespace ot;

namespace ot {
__global__ __launch_bounds__(256) void k_tsdf_clear(TsdfDev d, int64_t cap) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < cap; i += (int64_t)gridDim.x * 256) {
        d.hkeys[i] = ~0ull;
        d.hvals[i] = -1;
        d.fmask[i] = 0ull;
    }
    if (blockIdx.x == 0) {
        if (threadIdx.x < N_COUNTERS) d.counters[threadIdx.x] = 0;
        if (threadIdx.x < 4) d.stats[threadIdx.x] = 0ull;
    }
}
}  // namespace ot

extern "C" {

ot_status ot_tsdf_create(double voxel_length, double sdf_trunc, int32_t color_type, int32_t unit_res, int32_t stride,
                         int64_t max_units, ot_tsdf** out) {
    if (!out) return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] out is NULL");
    *out = nullptr;
    if (!(voxel_length > 0.0) || !(sdf_trunc > 0.0))
        return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] voxel_length and sdf_trunc must be positive");
    if (unit_res != UNIT_RES)
        return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] only volume_unit_resolution=16 is supported");
    if (stride < 1) return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] depth_sampling_stride must be >= 1");
    if (color_type != OT_COLOR_NONE && color_type != OT_COLOR_RGB8)
        return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] unsupported color_type (NoColor or RGB8)");
    if (max_units <= 0) max_units = 32768;
    if (max_units > (1 << 24)) return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] max_units too large");
    ot_tsdf* v = new ot_tsdf();
    (void)hipGetDevice(&v->device);
    v->voxel_length = voxel_length;
    v->sdf_trunc = sdf_trunc;
    v->unit_length = voxel_length * (double)UNIT_RES;
    v->color_type = color_type;
    v->stride = stride;
    v->max_units = max_units;
    int64_t cap = 1;
    while (cap < 4 * max_units) cap <<= 1;
    v->hash_cap = cap;
    TsdfDev& d = v->dev;
    d.hash_mask = (int)(cap - 1);
    d.max_units = (int)max_units;
    auto cleanup = [&](hipError_t e) {
        set_error(std::string("[ScalableTSDFVolume] allocation failed: ") + hipGetErrorString(e));
        ot_tsdf_destroy(v);
        return OT_ERR_HIP;
    };
    hipError_t e;
    if ((e = hipMalloc(&d.hkeys, sizeof(unsigned long long) * cap)) != hipSuccess) return cleanup(e);
    if ((e = hipMalloc(&d.hvals, sizeof(int) * cap)) != hipSuccess) return cleanup(e);
    if ((e = hipMalloc(&d.counters, sizeof(int) * N_COUNTERS)) != hipSuccess) return cleanup(e);
    if ((e = hipMalloc(&d.stats, sizeof(unsigned long long) * 4)) != hipSuccess) return cleanup(e);
    if ((e = hipMalloc(&d.unit_keys, sizeof(int) * 3 * max_units)) != hipSuccess) return cleanup(e);
    // RGB8 volumes keep colour at Open3D's precision (float64, 128-KiB records) unless set_color_precision(32)
    v->color64 = color_type == OT_COLOR_RGB8;
    d.color64 = v->color64 ? 1 : 0;
    d.unit_floats = v->color64 ? UNIT_FLOATS_C64 : UNIT_FLOATS;
    if ((e = hipMalloc(&d.vox, sizeof(float) * (size_t)d.unit_floats * max_units)) != hipSuccess) return cleanup(e);
    if ((e = hipMalloc(&v->sorted_ids, sizeof(unsigned) * max_units)) != hipSuccess) return cleanup(e);
    if ((e = hipMalloc(&d.fmask, sizeof(unsigned long long) * cap)) != hipSuccess) return cleanup(e);
    if ((e = hipMalloc(&d.bslots, sizeof(int) * cap)) != hipSuccess) return cleanup(e);
    if ((e = hipMalloc(&d.work, sizeof(UnitWork) * cap)) != hipSuccess) return cleanup(e);
    if ((e = hipMalloc(&v->bset[0].bframes, sizeof(BatchFrame) * MAX_BATCH)) != hipSuccess) return cleanup(e);
    // coherent: k_copy_frames reads the staging straight from host memory, and non-coherent host memory may be cached
    // by the GPU (the halves are rewritten every other batch)
    if ((e = hipHostMalloc(&v->hbframes, sizeof(BatchFrame) * MAX_BATCH * 2, hipHostMallocCoherent)) != hipSuccess)
        return cleanup(e);
    if ((e = hipHostMalloc(&v->hmail, sizeof(unsigned) * 2 * OT_MAIL_WORDS, hipHostMallocCoherent)) != hipSuccess)
        return cleanup(e);
    std::memset(v->hmail, 0, sizeof(unsigned) * 2 * OT_MAIL_WORDS);  // sequence words start below every seq sent (>= 1)
    ot_status st = ot_tsdf_reset(v);
    if (st != OT_OK) {
        ot_tsdf_destroy(v);
        return st;
    }
    *out = v;
    return OT_OK;
}

ot_status ot_tsdf_destroy(ot_tsdf* v) {
    if (!v) return OT_OK;
    (void)hipDeviceSynchronize();
    TsdfDev& d = v->dev;
    ot_tsdf_set_profiling(v, 0);
    void* ptrs[] = {d.hkeys, d.hvals, d.counters, d.stats, d.unit_keys, d.vox, v->mult, v->sorted_ids, v->mesh.ws,
                    v->mesh.v, v->mesh.c, v->mesh.t, v->mesh.vk, v->mesh.tk, v->mesh.vown, d.fmask, d.bslots, d.work,
                    v->wcount, v->bset[0].bframes, v->bset[0].bdm, v->bset[0].brgba, v->bset[1].bframes,
                    v->bset[1].bdm, v->bset[1].brgba, v->bset[1].work, v->tmask};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (v->hbframes) (void)hipHostFree(v->hbframes);
    if (v->hmail) (void)hipHostFree(v->hmail);
    if (v->ev_fork) (void)hipEventDestroy(v->ev_fork);
    if (v->ev_join) (void)hipEventDestroy(v->ev_join);
    if (v->ev_normals) (void)hipEventDestroy(v->ev_normals);
    if (v->ev_made) (void)hipEventDestroy(v->ev_made);
    if (v->ev_dfr) (void)hipEventDestroy(v->ev_dfr);
    if (v->side) (void)hipStreamDestroy(v->side);
    if (v->istream) (void)hipStreamDestroy(v->istream);
    for (auto& b : v->bset) {
        if (b.ev_units) (void)hipEventDestroy(b.ev_units);
        if (b.ev_done) (void)hipEventDestroy(b.ev_done);
    }
    delete v;
    return OT_OK;
}

ot_status ot_tsdf_reset(ot_tsdf* v) {
    if (!v) return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume::Reset] volume is NULL");
    TsdfDev& d = v->dev;
    OT_HIP_TRY(hipDeviceSynchronize());  // queued work on the volume (deferred normals included) first
    v->normals_pending = false;
    v->last_set = -1;
    OT_HIP_TRY(hipMemset(d.hkeys, 0xFF, sizeof(unsigned long long) * v->hash_cap));
    OT_HIP_TRY(hipMemset(d.hvals, 0xFF, sizeof(int) * v->hash_cap));
    OT_HIP_TRY(hipMemset(d.fmask, 0, sizeof(unsigned long long) * v->hash_cap));
    OT_HIP_TRY(hipMemset(d.counters, 0, sizeof(int) * N_COUNTERS));
    OT_HIP_TRY(hipMemset(d.stats, 0, sizeof(unsigned long long) * 4));
    OT_HIP_TRY(hipDeviceSynchronize());
    v->batch_pc = C_BATCH_PAIRS;
    v->frame_id = 0;
    v->imported = false;
    v->early_frame = -1;
    v->pending.clear();
    v->dfr_on = false;  // a deferred batch's integrate belongs to the old contents (its work list is stale now)
    v->stat_batches = v->stat_unit_batches = v->stat_fresh = v->stat_prev_units = 0;
    v->sorted_frame = -1;
    v->sorted_units = -1;
    v->mesh.nv = v->mesh.nt = 0;
    v->mesh.valid = false;
    return OT_OK;
}

ot_status ot_tsdf_reset_async(ot_tsdf* v, void* stream_) {
    if (!v) return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume::Reset] volume is NULL");
    hipStream_t stream = S(stream_);
    ot_status st = tsdf_flush(v, stream);  // queued frames belong to the old contents: apply, then clear
    if (st != OT_OK) return st;
    st = wait_normals(v, stream);  // the last mesh's deferred normals may still read the volume
    if (st != OT_OK) return st;
    // the hash table, frame masks, counters and statistics in one launch (six fill commands cost ~5 us of host time
    // each, on one object's critical path)
    const unsigned blocks = (unsigned)std::min<int64_t>((v->hash_cap + 255) / 256, 2048);
    hipLaunchKernelGGL(k_tsdf_clear, dim3(blocks), dim3(256), 0, stream, v->dev, (int64_t)v->hash_cap);
    OT_LAUNCH_CHECK();
    v->batch_pc = C_BATCH_PAIRS;
    v->frame_id = 0;
    v->imported = false;
    v->early_frame = -1;
    v->last_batch_slots = -1;
    v->stat_batches = v->stat_unit_batches = v->stat_fresh = v->stat_prev_units = 0;
    v->sorted_frame = -1;
    v->sorted_units = -1;
    v->mesh.nv = v->mesh.nt = 0;
    v->mesh.valid = false;
    return OT_OK;
}

ot_status ot_tsdf_integrate(ot_tsdf* vol, const float* depth, const uint8_t* color, const ot_intrinsics* in,
                            const double extrinsic[16], void* stream) {
    ot_status st = check_frame(vol, depth, color, in, extrinsic);
    if (st != OT_OK) return st;
    PendingFrame f;
    f.depth = nullptr;
    f.depthf = depth;
    f.color = color;
    f.intr = *in;
    std::memcpy(f.extrinsic, extrinsic, sizeof(double) * 16);
    f.depth_scale = 1.0;
    f.depth_trunc = 0.0;
    vol->pending.push_back(f);
    // a full queue is integrated; the integrate may keep running on the volume's integrate stream (overlap mode)
    if ((int)vol->pending.size() >= std::min(vol->batch_max, MAX_BATCH)) return tsdf_flush(vol, S(stream), false);
    return OT_OK;
}

ot_status ot_tsdf_integrate_u16(ot_tsdf* vol, const uint16_t* depth, const uint8_t* color, const ot_intrinsics* in,
                                const double extrinsic[16], double depth_scale, double depth_trunc, void* stream) {
    ot_status st = check_frame(vol, depth, color, in, extrinsic);
    if (st != OT_OK) return st;
    PendingFrame f;
    f.depth = depth;
    f.depthf = nullptr;
    f.color = color;
    f.intr = *in;
    std::memcpy(f.extrinsic, extrinsic, sizeof(double) * 16);
    f.depth_scale = depth_scale;
    f.depth_trunc = depth_trunc;
    vol->pending.push_back(f);
    if ((int)vol->pending.size() >= std::min(vol->batch_max, MAX_BATCH)) return tsdf_flush(vol, S(stream), false);
    return OT_OK;
}

ot_status ot_tsdf_integrate_u16_frames(ot_tsdf* vol, int32_t n, const uint16_t* depth, const uint8_t* color,
                                       const ot_intrinsics* in, const double* extrinsics, double depth_scale,
                                       double depth_trunc, void* stream) {
    if (!vol || n < 0 || !in || (n > 0 && (!depth || !extrinsics)))
        return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume::Integrate] invalid arguments");
    const int64_t npx = (int64_t)in->width * in->height;
    for (int32_t k = 0; k < n; ++k) {  // exactly n calls of ot_tsdf_integrate_u16, without n host round trips
        ot_status st = ot_tsdf_integrate_u16(vol, depth + (size_t)k * npx, color ? color + (size_t)k * npx * 3 : nullptr,
                                             in, extrinsics + 16 * (size_t)k, depth_scale, depth_trunc, stream);
        if (st != OT_OK) return st;
    }
    return OT_OK;
}

ot_status ot_tsdf_flush(ot_tsdf* vol, void* stream) {
    if (!vol) return fail(OT_ERR_INVALID_ARGUMENT, "volume is NULL");
    return tsdf_flush(vol, S(stream));
}

ot_status ot_tsdf_pending_frames(const ot_tsdf* vol, int32_t* n_host) {
    if (!vol || !n_host) return fail(OT_ERR_INVALID_ARGUMENT, "invalid arguments");
    *n_host = (int32_t)vol->pending.size();
    return OT_OK;
}

ot_status ot_tsdf_set_batch(ot_tsdf* vol, int32_t max_frames) {
    if (!vol || max_frames < 1) return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] batch must be >= 1");
    vol->batch_max = max_frames;
    return OT_OK;
}

ot_status ot_tsdf_set_frontend_overlap(ot_tsdf* vol, int32_t mode) {
    if (!vol || mode < -1 || mode > 1)
        return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] front-end overlap mode must be -1, 0 or 1");
    // the mode changes only on a drained volume: queued frames would be staged on whichever stream this call named,
    // not the one their producers ran on -- flush or read the volume on the frames' stream first
    if (!vol->pending.empty())
        return fail(OT_ERR_INVALID_ARGUMENT,
                    "[ScalableTSDFVolume] front-end overlap can change only with no queued frames (flush first)");
    if (vol->istream) OT_HIP_TRY(hipStreamSynchronize(vol->istream));  // a running integrate of the old mode
    vol->last_set = -1;
    vol->overlap_mode = mode;
    return OT_OK;
}

ot_status ot_tsdf_num_units(ot_tsdf* vol, int64_t* n, void* stream_) {
    if (!vol || !n) return fail(OT_ERR_INVALID_ARGUMENT, "invalid arguments");
    hipStream_t stream = S(stream_);
    ot_status st = tsdf_flush(vol, stream);  // queued frames, on the caller's stream
    if (st != OT_OK) return st;
    if (vol->dev.shard_world > 1) {  // a shard counts its own units (halo units are not exported)
        const unsigned* ids = nullptr;
        return export_list(vol, stream, &ids, n);
    }
    int nu = 0;
    OT_HIP_TRY(hipMemcpyAsync(&nu, vol->dev.counters + C_UNITS, sizeof(int), hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipStreamSynchronize(stream));
    *n = std::min<int64_t>(nu, vol->max_units);
    return OT_OK;
}

ot_status ot_tsdf_batch_stats(ot_tsdf* vol, int64_t* batches, int64_t* unit_batches, int64_t* new_units) {
    if (!vol) return fail(OT_ERR_INVALID_ARGUMENT, "invalid arguments");
    if (batches) *batches = vol->stat_batches;  // batches run (frames still queued are not counted: flush first)
    if (unit_batches) *unit_batches = vol->stat_unit_batches;
    if (new_units) *new_units = vol->stat_fresh;
    return OT_OK;
}

ot_status ot_tsdf_counters(ot_tsdf* vol, int64_t* updates, int64_t* unit_integrations, void* stream_) {
    if (!vol) return fail(OT_ERR_INVALID_ARGUMENT, "invalid arguments");
    hipStream_t stream = S(stream_);
    ot_status st = tsdf_flush(vol, stream);
    if (st != OT_OK) return st;
    unsigned long long s[4];
    OT_HIP_TRY(hipMemcpyAsync(s, vol->dev.stats, sizeof(s), hipMemcpyDeviceToHost, stream));
    OT_HIP_TRY(hipStreamSynchronize(stream));
    if (updates) *updates = (int64_t)s[S_UPDATES];
    if (unit_integrations) *unit_integrations = (int64_t)s[S_UNIT_INTEGRATIONS];
    return OT_OK;
}

ot_status ot_tsdf_set_color_precision(ot_tsdf* vol, int32_t bits) {
    if (!vol || (bits != 32 && bits != 64))
        return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] colour precision must be 32 or 64 bits");
    int nu = 0;
    OT_HIP_TRY(hipMemcpy(&nu, vol->dev.counters + C_UNITS, sizeof(int), hipMemcpyDeviceToHost));
    if (nu != 0 || !vol->pending.empty())
        return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] set the colour precision before the first integrate");
    // NoColor volumes keep no colour state: the float32 record (zero colour planes) whatever the precision
    const bool c64 = bits == 64 && vol->color_type == OT_COLOR_RGB8;
    if (c64 != vol->color64) {  // the record stride changes: reallocate the (still empty) pool
        const int uf = c64 ? UNIT_FLOATS_C64 : UNIT_FLOATS;
        OT_HIP_TRY(hipDeviceSynchronize());
        // the new pool first: if the allocation fails the volume keeps its old, consistent layout
        float* pool = nullptr;
        OT_HIP_TRY(hipMalloc(&pool, sizeof(float) * (size_t)uf * vol->max_units));
        (void)hipFree(vol->dev.vox);
        vol->dev.vox = pool;
        vol->dev.unit_floats = uf;
        vol->dev.color64 = c64 ? 1 : 0;
        vol->color64 = c64;
    }
    return OT_OK;
}

ot_status ot_tsdf_get_color_precision(const ot_tsdf* vol, int32_t* bits) {
    if (!vol || !bits) return fail(OT_ERR_INVALID_ARGUMENT, "invalid arguments");
    *bits = vol->color64 ? 64 : 32;
    return OT_OK;
}

ot_status ot_tsdf_set_profiling(ot_tsdf* vol, int32_t enable) {
    if (!vol) return fail(OT_ERR_INVALID_ARGUMENT, "invalid arguments");
    vol->profiling = enable != 0;
    vol->prof_ms = vol->prof_fe_ms = 0.0;
    vol->prof_launches = vol->prof_fe_batches = 0;
    for (auto* lst : {&vol->prof_events, &vol->prof_fe_events}) {
        for (auto& e : *lst) {
            (void)hipEventDestroy(e.first);
            (void)hipEventDestroy(e.second);
        }
        lst->clear();
    }
    return OT_OK;
}

// accumulate (and release) an event-pair list into (ms, count)
static ot_status drain_events(std::vector<std::pair<hipEvent_t, hipEvent_t>>& lst, double& ms_acc, int64_t& n_acc) {
    for (auto& e : lst) {
        OT_HIP_TRY(hipEventSynchronize(e.second));
        float ms = 0.0f;
        OT_HIP_TRY(hipEventElapsedTime(&ms, e.first, e.second));
        ms_acc += ms;
        n_acc += 1;
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    lst.clear();
    return OT_OK;
}

ot_status ot_tsdf_kernel_time(ot_tsdf* vol, double* total_ms, int64_t* launches) {
    if (!vol) return fail(OT_ERR_INVALID_ARGUMENT, "invalid arguments");
    ot_status st = tsdf_flush(vol, nullptr);
    if (st != OT_OK) return st;
    if ((st = drain_events(vol->prof_events, vol->prof_ms, vol->prof_launches)) != OT_OK) return st;
    if (total_ms) *total_ms = vol->prof_ms;
    if (launches) *launches = vol->prof_launches;
    return OT_OK;
}

ot_status ot_tsdf_frontend_time(ot_tsdf* vol, double* total_ms, int64_t* batches) {
    if (!vol) return fail(OT_ERR_INVALID_ARGUMENT, "invalid arguments");
    ot_status st = tsdf_flush(vol, nullptr);
    if (st != OT_OK) return st;
    if ((st = drain_events(vol->prof_fe_events, vol->prof_fe_ms, vol->prof_fe_batches)) != OT_OK) return st;
    if (total_ms) *total_ms = vol->prof_fe_ms;
    if (batches) *batches = vol->prof_fe_batches;
    return OT_OK;
}

ot_status ot_tsdf_export_units(ot_tsdf* vol, int64_t capacity, int32_t* keys, float* tsdf, float* weight, float* color,
                               void* stream) {
    if (!vol) return fail(OT_ERR_INVALID_ARGUMENT, "invalid arguments");
    int64_t nu = 0;
    const unsigned* ids = nullptr;
    ot_status st = export_list(vol, S(stream), &ids, &nu);
    if (st != OT_OK) return st;
    if (nu > capacity) return fail(OT_ERR_CAPACITY, "[ScalableTSDFVolume] export: more units than the output capacity");
    if (nu == 0) return OT_OK;
    if (vol->color64)
        hipLaunchKernelGGL((k_export<double, float>), dim3((unsigned)nu), dim3(256), 0, S(stream), vol->dev, ids, keys,
                           tsdf, weight, color);
    else
        hipLaunchKernelGGL((k_export<float, float>), dim3((unsigned)nu), dim3(256), 0, S(stream), vol->dev, ids, keys,
                           tsdf, weight, color);
    OT_LAUNCH_CHECK();
    OT_HIP_TRY(hipStreamSynchronize(S(stream)));
    return OT_OK;
}

ot_status ot_tsdf_export_color64(ot_tsdf* vol, int64_t capacity, double* color, void* stream) {
    if (!vol || !color) return fail(OT_ERR_INVALID_ARGUMENT, "invalid arguments");
    int64_t nu = 0;
    const unsigned* ids = nullptr;
    ot_status st = export_list(vol, S(stream), &ids, &nu);
    if (st != OT_OK) return st;
    if (nu > capacity) return fail(OT_ERR_CAPACITY, "[ScalableTSDFVolume] export: more units than the output capacity");
    if (nu == 0) return OT_OK;
    if (vol->color64)
        hipLaunchKernelGGL((k_export<double, double>), dim3((unsigned)nu), dim3(256), 0, S(stream), vol->dev, ids,
                           nullptr, nullptr, nullptr, color);
    else  // float32 colour state (or NoColor's zero planes) widens exactly
        hipLaunchKernelGGL((k_export<float, double>), dim3((unsigned)nu), dim3(256), 0, S(stream), vol->dev, ids,
                           nullptr, nullptr, nullptr, color);
    OT_LAUNCH_CHECK();
    OT_HIP_TRY(hipStreamSynchronize(S(stream)));
    return OT_OK;
}

// test / diagnostic hook (not part of the drop-in boundary): the volume's raw u64 stats[4] (0 voxel updates,
// 1 unit integrations; 2, 3 unused)
ot_status otx_tsdf_stats(ot_tsdf* vol, uint64_t* out4) {
    if (!vol || !out4) return fail(OT_ERR_INVALID_ARGUMENT, "invalid arguments");
    ot_status st = tsdf_flush(vol, nullptr);
    if (st != OT_OK) return st;
    OT_HIP_TRY(hipMemcpy(out4, vol->dev.stats, sizeof(uint64_t) * 4, hipMemcpyDeviceToHost));
    return OT_OK;
}

// test hook: the integrate's slice granularity (-1 = by the batch's estimated unit count, 0 = 4 voxels per lane along z
// always, 1 = 2 always; >= 2: the deferred integrate takes the fine slices below that many units, a threshold sweep):
// A/B timing and the parity of both instantiations
ot_status otx_integrate_fine(int32_t mode) {
    g_int_fine = mode < 0 ? -1 : (mode == 1 ? 1 : 0);
    g_fine_units = mode >= 2 ? mode : -1;
    return OT_OK;
}

// test hook: the batch touch's staging-only workgroups per frame group (-1 = two per touch tile, the default;
// 0 = every touch workgroup stages a share first): A/B timing and the parity of both forms
ot_status otx_touch_stage_blocks(int32_t blocks) {
    if (blocks > 4096) return fail(OT_ERR_INVALID_ARGUMENT, "otx_touch_stage_blocks: at most 4096");
    g_stage_blocks = blocks < 0 ? -1 : blocks;
    return OT_OK;
}

// test hook: frames per touch workgroup (1..64, default TF): A/B timing and the parity of other groupings
ot_status otx_touch_frames(int32_t tf) {
    if (tf < 1 || tf > MAX_BATCH) return fail(OT_ERR_INVALID_ARGUMENT, "otx_touch_frames: 1..64");
    g_touch_tf = tf;
    return OT_OK;
}

// test hook: 1 = sort units with the radix sort at every key width (the rank sort's parity test), 0 = default
ot_status otx_unit_sort_radix(int32_t on) {
    g_unit_sort_radix = on != 0;
    return OT_OK;
}

ot_status ot_tsdf_set_shard(ot_tsdf* vol, int32_t rank, int32_t world) {
    if (!vol || world < 1 || rank < 0 || rank >= world)
        return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] shard needs 0 <= rank < world");
    int nu = 0;
    OT_HIP_TRY(hipMemcpy(&nu, vol->dev.counters + C_UNITS, sizeof(int), hipMemcpyDeviceToHost));
    if (nu != 0 || !vol->pending.empty())
        return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] set the shard before the first integrate");
    vol->dev.shard_rank = rank;
    vol->dev.shard_world = world;
    vol->dev.shard_mode = SHARD_BLOCKS;
    // ownership blocks: 4^3 units up to 4 ranks, 2^3 beyond (configs[1] scan, 5 mm: largest shard / mean 1.09 / 1.13 /
    // 1.09 at 2 / 4 / 8 ranks; border rows sent 0.42 / 0.25 / 0.24 of an all-gather's)
    vol->dev.shard_shift = world <= 4 ? 2 : 1;
    return OT_OK;
}

ot_status ot_tsdf_set_shard_sector(ot_tsdf* vol, int32_t rank, int32_t world, double cx, double cy) {
    if (!vol || world < 1 || rank < 0 || rank >= world || !std::isfinite(cx) || !std::isfinite(cy))
        return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] shard needs 0 <= rank < world and a finite centre");
    const double hx = std::nearbyint(2.0 * cx / vol->unit_length), hy = std::nearbyint(2.0 * cy / vol->unit_length);
    if (std::fabs(hx) > (double)(1 << 22) || std::fabs(hy) > (double)(1 << 22))
        return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] sector centre out of the unit key range");
    ot_status st = ot_tsdf_set_shard(vol, rank, world);
    if (st != OT_OK) return st;
    vol->dev.shard_mode = SHARD_SECTORS;
    vol->dev.shard_cx2 = (int)hx;
    vol->dev.shard_cy2 = (int)hy;
    return OT_OK;
}

ot_status otx_integrate_depth(int32_t kt) {
    if (kt != -1 && (kt < 1 || kt > 3)) return fail(OT_ERR_INVALID_ARGUMENT, "integrate pipeline depth must be -1 or 1..3");
    g_int_depth = kt;
    return OT_OK;
}

ot_status otx_defer_integrate(int32_t mode) {
    if (mode < -1 || mode > 1) return fail(OT_ERR_INVALID_ARGUMENT, "deferred integrate mode must be -1, 0 or 1");
    g_defer = mode;
    return OT_OK;
}

ot_status otx_split_frontend(int32_t mode) {
    if (mode < -1 || mode > 1) return fail(OT_ERR_INVALID_ARGUMENT, "split front end mode must be -1, 0 or 1");
    g_split = mode;
    return OT_OK;
}

ot_status ot_tsdf_set_shard_block(ot_tsdf* vol, int32_t log2_units) {
    if (!vol || log2_units < 0 || log2_units > 8)
        return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] shard block must be 2^0 .. 2^8 units per axis");
    int nu = 0;
    OT_HIP_TRY(hipMemcpy(&nu, vol->dev.counters + C_UNITS, sizeof(int), hipMemcpyDeviceToHost));
    if (nu != 0 || !vol->pending.empty())
        return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] set the shard before the first integrate");
    vol->dev.shard_shift = log2_units;
    return OT_OK;
}

ot_status ot_tsdf_border_destinations(const ot_tsdf* vol, int64_t n, const int32_t* keys, int64_t* dest_mask,
                                      void* stream) {
    if (!vol || n < 0 || (n > 0 && (!keys || !dest_mask)) || vol->dev.shard_world > 64)
        return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] border_destinations: invalid arguments");
    if (n == 0) return OT_OK;
    hipLaunchKernelGGL(k_border_dest, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, S(stream), vol->dev, n, keys,
                       (unsigned long long*)dest_mask);
    OT_LAUNCH_CHECK();
    return OT_OK;
}

}  // extern "C"

template <typename CT>
static ot_status import_units(ot_tsdf* vol, int64_t n, const int32_t* keys, const float* tsdf, const float* weight,
                              const CT* color, hipStream_t stream) {
    if (!vol || n < 0 || (n > 0 && (!keys || !tsdf || !weight)))
        return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] import: invalid arguments");
    const bool rgb8 = vol->color_type == OT_COLOR_RGB8;
    if (rgb8 && vol->color64 != (sizeof(CT) == 8))
        return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] import: colour dtype does not match the volume's "
                                             "colour precision");
    ot_status st = tsdf_flush(vol, stream);
    if (st != OT_OK) return st;
    if (n == 0) return OT_OK;
    st = reserve_units(vol, n, stream);  // the pool grows instead of dropping imported units
    if (st != OT_OK) return st;
    if (rgb8)
        hipLaunchKernelGGL(k_import<CT>, dim3((unsigned)n), dim3(256), 0, stream, vol->dev, keys, tsdf, weight, color);
    else  // NoColor: float32 record, zero colour planes
        hipLaunchKernelGGL(k_import<float>, dim3((unsigned)n), dim3(256), 0, stream, vol->dev, keys, tsdf, weight,
                           (const float*)nullptr);
    OT_LAUNCH_CHECK();
    vol->sorted_units = -1;  // the sorted-unit cache no longer matches
    vol->imported = true;    // arbitrary state: the IEEE-division integrate from now on
    vol->stat_prev_units = -1;
    vol->mesh.valid = false;
    st = check_errors(vol, stream);
    if (st != OT_OK) return st;
    OT_HIP_TRY(hipStreamSynchronize(stream));
    return OT_OK;
}

extern "C" {

ot_status ot_tsdf_import_units(ot_tsdf* vol, int64_t n, const int32_t* keys, const float* tsdf, const float* weight,
                               const float* color, void* stream) {
    return import_units<float>(vol, n, keys, tsdf, weight, color, S(stream));
}

ot_status ot_tsdf_import_units_color64(ot_tsdf* vol, int64_t n, const int32_t* keys, const float* tsdf,
                                       const float* weight, const double* color, void* stream) {
    return import_units<double>(vol, n, keys, tsdf, weight, color, S(stream));
}

ot_status ot_tsdf_export_border(ot_tsdf* vol, int64_t capacity, int32_t* keys, float* tsdf, float* weight, void* color,
                                int64_t* n_exported_host, void* stream) {
    if (!vol || !keys || !tsdf || !weight || !n_exported_host) return fail(OT_ERR_INVALID_ARGUMENT, "invalid arguments");
    *n_exported_host = 0;
    int64_t no = 0;  // the own units (halo units imported earlier are not this shard's border)
    const unsigned* own = nullptr;
    ot_status st = export_list(vol, S(stream), &own, &no);
    if (st != OT_OK) return st;
    if (no == 0) return OT_OK;
    if (no > capacity) return fail(OT_ERR_CAPACITY, "[ScalableTSDFVolume] export: more units than the output capacity");
    if (no > 0) {
        if (vol->color_type != OT_COLOR_RGB8)  // NoColor: no colour rows (the caller's buffer is left as it is)
            hipLaunchKernelGGL(k_export_border<float>, dim3((unsigned)no), dim3(256), 0, S(stream), vol->dev, own,
                               keys, tsdf, weight, (float*)nullptr);
        else if (vol->color64)
            hipLaunchKernelGGL(k_export_border<double>, dim3((unsigned)no), dim3(256), 0, S(stream), vol->dev, own,
                               keys, tsdf, weight, (double*)color);
        else
            hipLaunchKernelGGL(k_export_border<float>, dim3((unsigned)no), dim3(256), 0, S(stream), vol->dev, own,
                               keys, tsdf, weight, (float*)color);
        OT_LAUNCH_CHECK();
    }
    OT_HIP_TRY(hipStreamSynchronize(S(stream)));
    *n_exported_host = no;
    return OT_OK;
}

ot_status ot_tsdf_import_border(ot_tsdf* vol, int64_t n, const int32_t* keys, const float* tsdf, const float* weight,
                                const void* color, void* stream_) {
    hipStream_t stream = S(stream_);
    if (!vol || n < 0 || (n > 0 && (!keys || !tsdf || !weight)))
        return fail(OT_ERR_INVALID_ARGUMENT, "[ScalableTSDFVolume] import_border: invalid arguments");
    ot_status st = tsdf_flush(vol, stream);
    if (st != OT_OK) return st;
    if (n == 0) return OT_OK;
    st = reserve_units(vol, n, stream);  // halo units: room for every row (a superset of those kept)
    if (st != OT_OK) return st;
    const void* c = vol->color_type == OT_COLOR_RGB8 ? color : nullptr;
    if (vol->color64)  // (only RGB8 volumes store float64 colour)
        hipLaunchKernelGGL(k_import_border<double>, dim3((unsigned)n), dim3(256), 0, stream, vol->dev, keys, tsdf,
                           weight, (const double*)c);
    else
        hipLaunchKernelGGL(k_import_border<float>, dim3((unsigned)n), dim3(256), 0, stream, vol->dev, keys, tsdf,
                           weight, (const float*)c);
    OT_LAUNCH_CHECK();
    vol->sorted_units = -1;
    vol->imported = true;  // halo units hold other shards' state (read by marching cubes; kept exact anyway)
    vol->stat_prev_units = -1;
    vol->mesh.valid = false;
    st = check_errors(vol, stream);
    if (st != OT_OK) return st;
    OT_HIP_TRY(hipStreamSynchronize(stream));
    return OT_OK;
}

}  // extern "C"
