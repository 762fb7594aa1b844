// spt_internal.h — device-side data layout and kernel launchers (not part of
// the public C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spt_math.h"

namespace spt {

constexpr uint32_t kMaxDepthCasts = 64;     // spt_render_params.max_depth limit
constexpr uint32_t kNode8Quads = 8;         // BVH8 node stride in 16-B units (80 B used, padded to one 128-B line)
// Triangle record: 16 floats, one 64-B half-line per BVH slot.  Each vertex is
// stored as x y z x y (five floats), the original triangle id in float 15.  A
// lane loads vertex i as the three floats at 5 i + r: r = 0 gives (x, y, z),
// 1 gives (y, z, x), 2 gives (z, x, y) — the vertex already permuted into the
// Woop test's (kx, ky, kz) order for a ray whose dominant axis is kz = (r + 2)
// mod 3, so the test needs no per-lane component selects (spt_math.h
// woop_shear_rot).
constexpr uint32_t kTriQuads = 4;           // triangle record stride in 16-B units
constexpr uint32_t kTriFloats = 16;
constexpr uint32_t kTriIdFloat = 15;
SPT_HD void tri_record_fill(float* rec, const float* v9, uint32_t id) {
    for (int k = 0; k < 3; k++) {
        rec[5 * k] = v9[3 * k];
        rec[5 * k + 1] = v9[3 * k + 1];
        rec[5 * k + 2] = v9[3 * k + 2];
        rec[5 * k + 3] = v9[3 * k];
        rec[5 * k + 4] = v9[3 * k + 1];
    }
    rec[kTriIdFloat] = u2f(id);
}
constexpr uint32_t kNode6Quads = 4;         // 64-B node (at most six children, bvh_build.h): one 64-B half-line
constexpr uint32_t kIsectBlock = 128;       // isect: 2 waves, LDS stack [depth][128]
#ifndef SPT_SHADE_BLOCK
#define SPT_SHADE_BLOCK 512
#endif
constexpr uint32_t kShadeBlock = SPT_SHADE_BLOCK;  // shade: 8 waves, one queue atomic per block (A/B: 256 / 512 / 1024)
constexpr uint32_t kMetaDepthBits = 8;      // meta = sample << 8 | depth
constexpr uint32_t kIsectChunk = 128;       // dynamic-share queue indices a wave takes per atomic
constexpr uint32_t kRefillIdle = 16;        // refill a wave once this many lanes are idle
// SPT_WORK_AUTO: pixel-major for scenes beyond the Infinity Cache, and in the
// fused kernel for tiles of at least 16M paths (capi.cpp spt_render)
constexpr uint64_t kPixelMajorMinSceneBytes = 256ull << 20;
constexpr uint64_t kPixelMajorMinFusedPaths = 16ull << 20;
// ... and in the wavefront for scenes beyond one XCD's L2 on tiles of <= 4M
// pixels, with 24M paths in flight when the in-flight count is left at its
// default (32M)
constexpr uint64_t kPixelMajorMinWaveSceneBytes = 4ull << 20;
constexpr uint64_t kPixelMajorMaxWaveTilePx = 4ull << 20;
constexpr uint32_t kDefaultWavefrontPaths = 1u << 25;
constexpr uint64_t kPixelMajorWavefrontPaths = 24ull << 20;
// spt_config.drain_q8 default: a sub-wavefront's queue shorter than this many
// 1/256ths of its persistent isect lanes goes to the drain launch
constexpr uint32_t kDefaultDrainQ8 = 1024;
// spt_config.fused_max_paths default: AUTO runs the fused kernel only for jobs
// of at most 1M paths, fewer than two chip fills of lanes (config 0's 262k:
// the wavefront's launches and streams outweigh the work, 372 vs 823 Mpaths/s)
constexpr uint64_t kDefaultFusedMaxPaths = 1ull << 20;
// spt_config.fit_paths default: jobs (or sample chunks, fit_chunks) of at most
// 2^28 paths start every path at once: 21 GB of queues per working set in unit
// mode, 34 GB with emitters (HBM is 288 GB); config 3 +3.7 % over 2^27, config
// 2 -0.7 % (profiles/r05_exp/fit_paths_rgb_waves/)
constexpr uint64_t kDefaultFitPaths = 1ull << 28;
// spt_config.drain_casts default: the drain runs this many casts after a
// sub-wavefront's last work item started, whatever its queue holds
constexpr uint32_t kDefaultDrainCasts = 1;
// spt_config.drain_refill_idle AUTO (0): free lanes a drain wave waits for
// before it refills and shades — scenes with analytic spheres (tested in the
// shade, with smallpt's mirror / glass: the pass costs several trace steps),
// scenes whose queue is streamed (beyond the Infinity Cache), the rest
constexpr uint32_t kDrainIdleSpheres = 56;
constexpr uint32_t kDrainIdleStream = 40;
constexpr uint32_t kDrainIdleCached = 24;

// Path modes: what a path carries besides its ray.  The scene decides
// (spt_render): unit = every albedo 1 and no emitters, the reference's own
// case (main.cpp:234,244) — the throughput is always 1, roulette
// never fires, and a path's film contribution is "escaped or not".
enum PathMode : int {
    kModeUnit = 0,    // q1, q2                  (32 B / path); film: one byte per (sample, pixel)
    kModeAlbedo = 1,  // + q0 throughput          (48 B / path); film: RGB floats per (sample, pixel)
    kModeEmit = 2     // + rad gathered radiance  (56 B / path); film: RGB floats
};
SPT_HD uint32_t mode_planes(int mode) { return mode == kModeUnit ? 2u : mode == kModeAlbedo ? 3u : 4u; }
SPT_HD uint32_t mode_film_bytes(int mode) { return mode == kModeUnit ? 1u : 12u; }
// Film slots are filled with 0xff bytes before a chunk renders (spt_render):
// no path writes these values (a flag is 0 or 1; 0xffffffff is a NaN no
// arithmetic produces), so the resolve can count slots nothing wrote.
constexpr uint32_t kFlagSentinel = 0xffu;
constexpr uint32_t kFilmSentinel = 0xffffffffu;

// Path queue: planes of 16-B quads grouped by who reads them, so a kernel
// moves a path in a few dwordx4 accesses (one coalesced 1-KB wave instruction
// each) instead of one 4-B plane per field:
//   q1 = (o.x, o.y, o.z, meta)    origin, sample << 8 | cast    [isect, shade]
//   q2 = (d.x, d.y, d.z, pix)     direction, tile-local pixel   [isect, shade]
//   q0 = (tr, tg, tb, lr)         throughput (+ red radiance)   [shade; albedo / emit modes]
//   rad = (lg, lb)                radiance gathered so far      [shade; emit mode; 8-B plane]
// The PCG32 state is not stored: (pixel, sample, cast) fix how many draws the
// path has consumed, s * (4 + 2D) + 4 + 2 * cast (main.cpp:395,396,413), so
// shade re-derives it with two jump-ahead applications.
struct PathQueue {
    float4 *q1, *q2, *q0;
    float2* rad;
};

// Geometry on device, leaf ("slot") order.
struct DeviceScene {
    const float4* nodes;   // BVH2: 4 per node (bvh_build.h)
    const uint4* nodes8;   // compressed BVH8: 5 per node (bvh_build.h); non-null selects it
    uint32_t node6;        // nodes8 holds 64-B nodes (at most six children, bvh_build.h)
    uint32_t group_shift;  // child s of a node at (group word << group_shift) + s (gpu_bvh8_holes)
    const float4* tris;    // kTriQuads per slot: the rotated-vertex record (tri_record_fill)
    const float4* snrm;    // 3 per slot: n0 (w = material id bits), n1, n2
    const float* tc;       // 6 per slot (u0 v0 u1 v1 u2 v2) or null
    const int32_t* orig2slot;
    const float* albedo;   // 3 per material
    uint32_t nmat;
    const float* emission; // 3 per material or null (no emitters)
    uint32_t nemit;
    uint32_t stack_depth;  // LDS stack entries per lane (one word each)
    uint32_t empty;        // no triangles
    const uint4* tex_info; // per material: first texel, width, height, 1 if it has an image (null: none)
    uint32_t ntex;         // entries of tex_info
    const float4* texels;  // RGB(-) texels of every image
    const float4* spheres; // analytic spheres (cx, cy, cz, r), tested after the BVH (null: none)
    const int32_t* sph_mat;
    uint32_t nsph;
    const uint32_t* mat_kind;  // per material SPT_MAT_* (null: every material diffuse)
    uint32_t nkind;
};

constexpr uint32_t kMatDiffuse = 0, kMatMirror = 1, kMatGlass = 2;  // SPT_MAT_*
SPT_HD uint32_t material_kind(const DeviceScene& sc, uint32_t mat) {
    return (sc.mat_kind && mat < sc.nkind) ? sc.mat_kind[mat] : kMatDiffuse;
}

// smallpt Sphere::intersect in the ray's own t units (d need not be unit):
// the nearer root in [tmin, tmax], else +inf.  f32 with the sphere-relative
// origin; the oracle restates the same operation order.
SPT_HD float sphere_t(V3 o, V3 d, float4 s, float tmin, float tmax) {
    const V3 op = v3(s.x - o.x, s.y - o.y, s.z - o.z);
    const float a = dot(d, d);
    const float b = dot(op, d);
    const float c = dot(op, op) - s.w * s.w;
    const float det = b * b - a * c;
    if (!(det >= 0.0f)) return INFINITY;
    const float sq = sqrtf(det);
    const float t0 = (b - sq) / a, t1 = (b + sq) / a;
    if (t0 >= tmin && t0 <= tmax) return t0;
    if (t1 >= tmin && t1 <= tmax) return t1;
    return INFINITY;
}

// The new direction of a bounce and its weight.  Triangles with a diffuse
// material: the reference's Lambert bounce (main.cpp:413-424; Frame3 of the
// un-normalised shading normal, coordframe.h:17-30, cosine hemisphere,
// mapping.h:5-11).  Spheres and the mirror / glass kinds follow smallpt's
// radiance(): the unit normal (a sphere's (x - c) / r direction, a triangle's
// normalised shading normal) flipped toward the ray for diffuse (nl); SPEC
// reflects; REFR refracts with index 1.5 and Schlick's Fresnel term, choosing
// reflection with probability P = 1/4 + Re/2 by xi_x (weight Re/P, else
// (1 - Re)/(1 - P)); total internal reflection reflects with weight 1.
SPT_HD V3 scatter(const DeviceScene& sc, uint32_t kind, int32_t slot, V3 d, V3 p, V3 sn, float xi_x, float xi_y,
                  float& weight) {
    weight = 1.0f;
    V3 n;
    if (slot >= 0) {
        if (kind == kMatDiffuse) return to_world(frame_from_normal(sn), cosine_hemisphere(xi_x, xi_y));
        n = normalize(sn);
    } else {
        const float4 s = sc.spheres[-2 - slot];
        n = normalize(v3(p.x - s.x, p.y - s.y, p.z - s.z));
        if (kind == kMatDiffuse) {
            const V3 nl = dot(n, d) < 0.0f ? n : v3(-n.x, -n.y, -n.z);
            return to_world(frame_from_normal(nl), cosine_hemisphere(xi_x, xi_y));
        }
    }
    const V3 dn = normalize(d);
    const float ndd = dot(n, dn);
    const float k2 = 2.0f * ndd;
    const V3 refl = v3(dn.x - n.x * k2, dn.y - n.y * k2, dn.z - n.z * k2);  // r.d - n * 2 * n.dot(r.d)
    if (kind != kMatGlass) return refl;
    const bool into = ndd < 0.0f;                       // n.dot(nl) > 0
    const V3 nl = into ? n : v3(-n.x, -n.y, -n.z);
    const float nc = 1.0f, nt = 1.5f;
    const float nnt = into ? nc / nt : nt / nc;
    const float ddn = dot(dn, nl);
    const float cos2t = 1.0f - (nnt * nnt) * (1.0f - ddn * ddn);
    if (cos2t < 0.0f) return refl;                      // total internal reflection
    const float ks = (into ? 1.0f : -1.0f) * (ddn * nnt + sqrtf(cos2t));
    const V3 tdir = normalize(v3(dn.x * nnt - n.x * ks, dn.y * nnt - n.y * ks, dn.z * nnt - n.z * ks));
    const float ea = nt - nc, eb = nt + nc;
    const float R0 = (ea * ea) / (eb * eb);
    const float c = 1.0f - (into ? -ddn : dot(tdir, n));
    const float Re = R0 + (1.0f - R0) * ((((c * c) * c) * c) * c);
    const float Tr = 1.0f - Re, P = 0.25f + 0.5f * Re;
    if (xi_x < P) { weight = Re / P; return refl; }
    weight = Tr / (1.0f - P);
    return tdir;
}

// ImageTexture::texel_fetch_wrap / texel_fetch (main.cpp:47-60): clamp, then
// the reference's index y * size.y + x (main.cpp:52), kept inside the image.
SPT_HD float4 texel_fetch(const float4* img, uint32_t w, uint32_t h, int32_t x, int32_t y) {
    x = x < 0 ? 0 : (x > (int32_t)w - 1 ? (int32_t)w - 1 : x);
    y = y < 0 ? 0 : (y > (int32_t)h - 1 ? (int32_t)h - 1 : y);
    uint64_t idx = (uint64_t)y * h + (uint64_t)x;
    const uint64_t last = (uint64_t)w * h - 1;
    return img[idx > last ? last : idx];
}
// ImageTexture::eval (main.cpp:62-76): bilinear with clamp in the reference's
// operation order; the scaled coordinate is clamped to +-2^30 before
// floor2int (NaN -> -2^30), the oracle does the same.
SPT_HD V3 texture_eval(const float4* img, uint32_t w, uint32_t h, float u, float v) {
    float sx = u * (float)w - 0.5f, sy = v * (float)h - 0.5f;
    sx = fminf(fmaxf(sx, -1073741824.0f), 1073741824.0f);
    sy = fminf(fmaxf(sy, -1073741824.0f), 1073741824.0f);
    const int32_t x = (int32_t)floorf(sx), y = (int32_t)floorf(sy);
    const float dx1 = sx - (float)x, dy1 = sy - (float)y;
    const float dx2 = 1.0f - dx1, dy2 = 1.0f - dy1;
    const float4 f00 = texel_fetch(img, w, h, x, y), f01 = texel_fetch(img, w, h, x, y + 1);
    const float4 f10 = texel_fetch(img, w, h, x + 1, y), f11 = texel_fetch(img, w, h, x + 1, y + 1);
    return v3((((f00.x * dx2) * dy2 + (f01.x * dx2) * dy1) + (f10.x * dx1) * dy2) + (f11.x * dx1) * dy1,
              (((f00.y * dx2) * dy2 + (f01.y * dx2) * dy1) + (f10.y * dx1) * dy2) + (f11.y * dx1) * dy1,
              (((f00.z * dx2) * dy2 + (f01.z * dx2) * dy1) + (f10.z * dx1) * dy2) + (f11.z * dx1) * dy1);
}

// LambertBsdf::sample's contribution (main.cpp:109-117, 422): the material's
// image at the hit's texcoord, else its albedo constant (material ids outside
// the table use material 0).
SPT_HD V3 reflectance(const DeviceScene& sc, uint32_t mat, uint32_t slot, float u, float v) {
    if (mat < sc.ntex && sc.tex_info[mat].w) {
        const uint4 ti = sc.tex_info[mat];
        float tu = 0.0f, tv = 0.0f;
        if (sc.tc && (int32_t)slot >= 0) {  // barycentric_interpolate (add_math.h:4-7, optix_backend.h:395-401); spheres: (0, 0)
            const float* c = sc.tc + (size_t)slot * 6;
            const float w = (1.0f - u) - v;
            tu = (w * c[0] + u * c[2]) + v * c[4];
            tv = (w * c[1] + u * c[3]) + v * c[5];
        }
        return texture_eval(sc.texels + ti.x, ti.y, ti.z, tu, tv);
    }
    if (mat >= sc.nmat) mat = 0;
    return v3(sc.albedo[mat * 3], sc.albedo[mat * 3 + 1], sc.albedo[mat * 3 + 2]);
}

// A queue filled by a sharded producer (camera_cast_kernel): survivors of
// block b go to shard b mod kShards — the XCD the block runs on — through
// that shard's own counter, into segment [shard_base(j), shard_base(j) +
// count_j) of the queue.  One queue counter takes at most ~88 atomics per us
// (MI355X_MICROARCH.md, dequeue), so a first cast of 67M paths in 262144
// blocks on one counter waited ~3 ms for its compaction atomics; eight
// counters (and the drain's per-XCD pools over the same segments) take
// eight times that.  Segment j holds as many slots as shard j has threads.
constexpr uint32_t kShards = 8;
constexpr uint32_t kShardStride = 32;  // words between shard counters (one 128-B line each)
SPT_HD uint32_t shard_base(uint32_t j, uint32_t items, uint32_t block) {
    const uint32_t nb = (items + block - 1) / block;
    uint32_t base = 0;
    for (uint32_t i = 0; i < j; i++) {
        if (i >= nb) break;
        base += ((nb - 1 - i) / kShards + 1) * block;  // blocks i, i + 8, ... of `block` threads
        if ((nb - 1) % kShards == i) base -= nb * block - items;  // the last block is short
    }
    return base;
}

struct RefillArgs {
    PathQueue q;
    Camera cam;
    const uint32_t* surv;       // survivors already in the queue
    const uint64_t* cursor_in;  // null: start at cursor_init (the first refill of a chunk)
    uint64_t cursor_init;
    uint64_t* cursor_out;       // written by thread 0 only
    uint32_t* qn_out;           // queue count for the next isect, thread 0 only
    uint32_t* isect_next;       // zeroed by thread 0 for the next isect launch
    uint32_t* surv_clear;       // zeroed by thread 0: the next shade's survivor counter (may be null)
    uint32_t* xcd_next;         // zeroed by thread 0 (8 counters, 32 words apart): the drain's (may be null)
    const uint32_t* casts_in;   // the preceding shade's queue count (null for a chunk's first refill):
                                // thread 0 adds it and *surv to stats[0] / stats[1]
    const PcgJump* sample_jump; // [spp]: seeded, then s * (4 + 2D) draws on (pcg_seeded_jump)
    unsigned long long* stats;  // casts, continuations, regenerations
    uint32_t* exhausted;        // thread 0 writes iter_tag here when this refill starts the last work item
    uint32_t iter_tag;          // the host's iteration number + 2 (the chunk's first refill: 1)
    uint64_t work_end;          // W_total (work items of this chunk end here)
    uint32_t capacity, P, W, rng_order;
    uint32_t tile_index, tile_count, rows_per_group;
    uint32_t pixel_block;       // camera-path order: B x B pixel blocks (<= 1: scanline)
    uint32_t work_order;        // 0: sample-major work items, 1: pixel-major inside the chunk
    uint32_t chunk_s0, chunk_ns;  // the chunk's first sample and sample count
    uint64_t initstate;
    int mode;                   // PathMode: which planes a new path fills
    uint32_t nt;                     // 1: non-temporal queue / hit accesses (spt_config.queue_cache)
    uint32_t book_only;         // 1: thread 0's bookkeeping only, no queue writes (camera_cast_kernel
                                // makes, traces and shades the paths this refill starts)
    const uint32_t* surv_shards;  // non-null: the survivors are the sum of these kShards counters
                                  // (kShardStride apart; a sharded shade: ShadeArgs::shard_items)
};

struct IsectQueueArgs {
    DeviceScene sc;
    PathQueue q;
    const uint32_t* count;
    float4* hits;                    // AoS per queue slot: (slot bits, t, u, v)
    uint32_t max_depth;
    uint32_t* next;                  // launch-wide ray counter (zeroed before the launch)
    uint32_t refill_idle;            // refill a wave once this many lanes are idle (1..64)
    uint32_t static_share_q8;        // static share of the queue per wave, in 1/256ths
    uint32_t chunk;                  // dynamic chunk (rays per atomic)
    uint32_t grid_q8;                // persistent grid scale in 1/256ths of full occupancy (0 = full)
    uint32_t xcd_remap;              // 1: blocks sharing an XCD take adjacent static shares
    uint32_t drain_below;            // skip the launch when *count < drain_below (launch_drain takes the queue)
    unsigned long long* trav_stats;  // non-null: nodes, tris, lane steps, wave steps
    // Camera paths started inside the launch (SPT_ISECT_CAMERA): the queue
    // holds cam.surv survivors in slots [0, surv); the launch starts
    // min(capacity - surv, work left) new camera paths in the slots after them
    // (writing their rays for the shade) and does refill_kernel's bookkeeping
    // in block 0's first thread (cam.isect_next: the NEXT launch's counter).
    RefillArgs cam;
    uint32_t nt;                     // 1: non-temporal queue / hit accesses (spt_config.queue_cache)
};

struct IsectPublicArgs {
    DeviceScene sc;
    const float *ox, *oy, *oz, *dx, *dy, *dz, *tmin, *tmax;
    const uint8_t* mask;
    uint32_t mask_size;
    int32_t* tri_id;
    float *t, *u, *v;
    uint32_t n;
    int32_t closest;
    uint32_t refill_idle;  // persistent BVH8 kernel: refill a wave once this many lanes are idle
    uint32_t persistent;   // 1: the persistent lane-refill kernel (spt_config.public_persistent)
};

// Blocks are dealt round-robin over the 8 XCDs (block b and b + 8 share one
// L2; MI355X_MICROARCH.md, workgroup dispatch).  This maps the launch's blocks
// so that those sharing an XCD take adjacent logical indices: each XCD then
// works on a contiguous eighth of the queue (speed only, never correctness).
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb) {
    const uint32_t full = nb & ~7u;
    if (b >= full) return b;
    return (b & 7u) * (full >> 3) + (b >> 3);
}

struct ShadeArgs {
    DeviceScene sc;
    PathQueue in, out;
    const float4* hits;
    const uint32_t* count_in;
    uint32_t* count_out;        // survivors appended here (zeroed before the launch)
    float* sfilm;               // [spp_chunk][3][P]: one contribution per (sample, pixel) (albedo / emit)
    uint8_t* sflag;             // [spp_chunk][P]: escaped or not per (sample, pixel) (unit mode)
    const PcgJump* sample_jump; // [spp]: seeded, then s * (4 + 2D) draws on (pcg_seeded_jump)
    const PcgJump* cast_jump;   // [max_depth]: jump by 4 + 2 * cast draws
    uint64_t initstate;
    uint32_t P, W, sample0, max_depth, rr_start, rng_order;
    uint32_t tile_index, tile_count, rows_per_group;
    uint32_t work_order, chunk_ns;  // film layout follows the work order (film_slot)
    float env_r, env_g, env_b;
    uint32_t xcd_remap;         // 1: blocks sharing an XCD take adjacent slot ranges
    uint32_t nt;                     // 1: non-temporal queue / hit accesses (spt_config.queue_cache)
    uint32_t drain_below;       // skip the launch when *count_in < drain_below (launch_drain takes the queue)
    uint32_t shard_items;       // != 0: survivors compacted into kShards segments of the out queue
                                // (shard_base over this many items), counters count_out[j * kShardStride]
};

// camera_cast_kernel: work items [r.cursor_init, r.cursor_init + n) of the
// sub-wavefront started (r: the refill's camera / work-item fields), traced
// and shaded (s: the shade's; survivors appended to s.out at *s.count_out).
struct CameraCastArgs {
    RefillArgs r;
    ShadeArgs s;
    uint32_t n;
};

// Starts new paths in queue slots [*surv, capacity): work item w (sample-major:
// sample = w / P, tile pixel = w % P) for w in [*cursor_in, W_total).

// Fused persistent render (one launch per sample chunk): every lane owns a
// path from camera ray to termination — trace, shade, bounce in registers.
// Work items [0, count) of the chunk map to w = work0 + i (sample-major).
struct FusedArgs {
    DeviceScene sc;
    Camera cam;
    const PcgJump* sample_jump;
    float* sfilm;               // [spp_chunk][3][P] (albedo / emit)
    uint8_t* sflag;             // [spp_chunk][P] (unit mode)
    unsigned long long* stats;  // casts, continuations, regenerations
    uint32_t* next;             // dynamic work counter (zeroed before the launch)
    uint64_t work0, initstate;
    uint32_t count, P, W, sample0, max_depth, rr_start, rng_order;
    uint32_t tile_index, tile_count, rows_per_group;
    uint32_t pm_ns;             // pixel-major work items: the chunk's sample count (0: sample-major);
                                // one argument for both, the kernel is short of SGPRs
    uint32_t refill_idle, static_share_q8, chunk, grid_q8;
    float env_r, env_g, env_b;
    // Drain mode (launch_drain): the same lane loop over the paths of a
    // wavefront queue instead of new camera paths.  The launch runs only when
    // *qcount < drain_below (else the isect and shade launches of the same
    // iteration do); it takes queue slots [0, *qcount), continues every path
    // in its lane to termination and adds to the stats only the casts after
    // each path's first (the refill that follows counts the queue itself).
    PathQueue q;
    const uint32_t* qcount;
    const PcgJump* cast_jump;       // [max_depth]: jump by 4 + 2 * cast draws (both modes: the shade re-derives the state)
    uint32_t drain_below;
    uint32_t nt;                    // 1: non-temporal queue loads (spt_config.queue_cache)
    unsigned long long* drained;    // paths the drain launches took over
    unsigned long long* drained_casts;  // ray casts the drain launches traced
    const uint32_t* perm;           // null, or the order the drain takes queue slots in (launch_drain_sort)
    uint32_t* xcd_next;             // null, or 8 per-XCD dynamic work counters, 32 words apart (zeroed
                                    // before the launch): XCD-aware work distribution (spt_config.xcd_remap bit 2)
    // A sharded queue (kShards segments, shard_base over seg_items in blocks of
    // seg_block): the drain's per-XCD pools (xcd_next) take segment j's
    // seg_count[j * kShardStride] paths first, then steal; no static share.
    const uint32_t* seg_count;
    uint32_t seg_items, seg_block;
    uint32_t count_queue;           // 1: add the queue's paths (their casts here) to stats[0] (a forced
                                    // drain, which no bookkeeping refill follows)
};

struct HitInfoArgs {
    DeviceScene sc;
    const float *ox, *oy, *oz, *dx, *dy, *dz;
    const int32_t* tri_id;
    const float *t, *u, *v;
    const uint8_t* mask;
    uint32_t mask_size, n;
    float *px, *py, *pz, *gnx, *gny, *gnz, *snx, *sny, *snz, *tcu, *tcv;
    int32_t* mat_id;
    uint64_t ntri;  // triangle ids >= ntri are skipped
};

// Tile-local row -> global row for interleaved row groups.
SPT_HD uint32_t tile_global_row(uint32_t local_row, uint32_t tile_index, uint32_t tile_count,
                                uint32_t rows_per_group) {
    if (tile_count == 1u) return local_row;  // one tile: the identity below, without its divisions
    uint32_t g = local_row / rows_per_group;
    return (g * tile_count + tile_index) * rows_per_group + local_row % rows_per_group;
}
// Tile pixel -> global pixel (main.cpp:379-382's index); a whole image (one
// tile) is its own tile, so the two divisions are skipped (a wave-uniform test)
SPT_HD uint32_t tile_global_pixel(uint32_t pix, uint32_t W, uint32_t tile_index, uint32_t tile_count,
                                  uint32_t rows_per_group) {
    if (tile_count == 1u) return pix;
    return tile_global_row(pix / W, tile_index, tile_count, rows_per_group) * W + pix % W;
}

// Tile pixel of the q-th camera path of a sample (q in [0, P), P = W * H):
// row bands of B rows, each cut into B-wide blocks taken in order, q running
// row-major inside a block (the last band / block may be shorter).  A wave's
// 64 consecutive camera paths then cover an 8 x 8 footprint instead of 64
// pixels of one row (B = 8), and bounce rays inherit that locality through
// the order-preserving compaction.  Any B covers every pixel once, so the
// image does not depend on it.  B <= 1: scanline order.
// Work item `local` (counted from the chunk's start) of the chunk of samples
// [s0, s0 + ns) -> (sample, pixel-order index q).  Sample-major (pm false):
// local = (s - s0) * P + q, so the paths in flight cover a few samples of the
// whole tile.  Pixel-major: a pixel's ns samples are consecutive work items,
// so a wave starts 64 samples of one pixel and a contiguous share of the queue
// covers a band of the tile.  One 32-bit division by d = pm ? ns : P serves
// both.  Both cover every (sample, pixel) of the chunk once.
SPT_HD void work_item(uint32_t local, uint32_t s0, uint32_t ns, uint32_t P, bool pm, uint32_t& s, uint32_t& q) {
    const uint32_t d = pm ? ns : P;
    const uint32_t a = udiv(local, d), b = local - a * d;
    s = s0 + (pm ? b : a);
    q = pm ? a : b;
}

// Per-(sample, pixel) film slot of a chunk of ns samples: [sample][pixel] for
// sample-major work, [pixel][sample] for pixel-major work, so the paths a wave
// ends together write neighbouring slots either way.  The RGB film (albedo /
// emit modes) keeps three floats per slot: channel stride P or 1 (film_rgb).
SPT_HD size_t film_slot(uint32_t sl, uint32_t pix, uint32_t P, uint32_t ns, uint32_t order) {
    return order ? (size_t)pix * ns + sl : (size_t)sl * P + pix;
}
SPT_HD float* film_rgb(float* sfilm, uint32_t sl, uint32_t pix, uint32_t P, uint32_t ns, uint32_t order,
                       size_t& stride) {
    stride = order ? 1 : P;
    return order ? sfilm + ((size_t)pix * ns + sl) * 3 : sfilm + (size_t)sl * 3 * P + pix;
}

SPT_HD void work_pixel(uint32_t q, uint32_t W, uint32_t P, uint32_t B, uint32_t& lx, uint32_t& ly) {
    if (B <= 1) { ly = udiv(q, W); lx = q - ly * W; return; }
    const uint32_t H = P / W;
    const uint32_t band = q / (B * W);
    const uint32_t off = q - band * B * W;
    const uint32_t rb = H - band * B < B ? H - band * B : B;
    const uint32_t cb = off / (B * rb);
    const uint32_t inner = off - cb * B * rb;
    const uint32_t cw = W - cb * B < B ? W - cb * B : B;
    const uint32_t r = inner / cw;
    lx = cb * B + (inner - r * cw);
    ly = band * B + r;
}

hipError_t launch_isect_queue(const IsectQueueArgs& a, uint32_t grid_items, hipStream_t s);
// one lane per queued ray, no lane refill: a fitting job's first cast (coherent camera rays)
hipError_t launch_isect_lockstep(const IsectQueueArgs& a, uint32_t grid_items, hipStream_t s);
hipError_t launch_isect_queue_stats(const IsectQueueArgs& a, uint32_t grid_items, hipStream_t s);
hipError_t launch_isect_queue_cam(const IsectQueueArgs& a, uint32_t grid_items, hipStream_t s);
hipError_t launch_isect_public(const IsectPublicArgs& a, hipStream_t s);
hipError_t launch_fused(const FusedArgs& a, int mode, hipStream_t s, uint32_t* lanes_out);
// The wavefront's drain: render_fused_kernel's lane loop over the paths of a
// queue (FusedArgs drain fields); runs only when the queue holds fewer than
// drain_below paths.  grid_q8 scales the chip-wide persistent grid.
hipError_t launch_drain(const FusedArgs& a, int mode, hipStream_t s);
// spt_config.drain_sort: the drain's order — a queue's `cap` slots sorted by
// (direction octant, Morton code of the origin in the scene box) into perm
// (slots past *count sort last).  tmp / tmp_bytes: hipcub scratch; with a
// null tmp only *tmp_bytes is set (the size to allocate).
hipError_t launch_drain_sort(const DeviceScene& sc, const PathQueue& q, const uint32_t* count, uint32_t cap,
                             uint32_t* keys, uint32_t* vals, uint32_t* keys_out, uint32_t* perm, void* tmp,
                             size_t* tmp_bytes, hipStream_t s);
// Lanes of the persistent isect grid a launch with these arguments gets (the
// drain threshold is counted in them).
uint32_t isect_queue_lanes(const IsectQueueArgs& a);
hipError_t launch_shade(const ShadeArgs& a, int mode, uint32_t grid_items, hipStream_t s);
// A fitting job's first cast — camera rays made, traced and shaded in one
// launch (camera_cast_kernel); wide-BVH scenes.
hipError_t launch_camera_cast(const CameraCastArgs& a, int mode, hipStream_t s);
hipError_t launch_refill(const RefillArgs& a, uint32_t grid_items, hipStream_t s);
// Both count the film slots still holding the pre-render sentinel (never
// written: a lost path) into *unwritten.
hipError_t launch_resolve(const float* sfilm, float* acc, float* out, uint32_t P, uint32_t nsamples,
                          uint32_t first_chunk, uint32_t last_chunk, uint32_t spp, uint32_t order,
                          unsigned long long* unwritten, hipStream_t s);
// unit mode: film = env added once per escaped sample, in sample order
hipError_t launch_resolve_flags(const uint8_t* sflag, float* acc, float* out, uint32_t P, uint32_t nsamples,
                                uint32_t first_chunk, uint32_t last_chunk, uint32_t spp, float env_r, float env_g,
                                float env_b, uint32_t order, unsigned long long* unwritten, hipStream_t s);
hipError_t launch_hit_info(const HitInfoArgs& a, hipStream_t s);

}  // namespace spt
