// kernels.hip — the hot path on gfx950: BVH traversal (isect), Lambertian
// shade + sample + Russian roulette with wave-ballot compaction and path
// regeneration (shade), camera generation and film resolve.
//
// Replaces wavefront_isect.cu:36-112 (OptiX raygen / closest-hit / miss) and
// the Enoki-JIT bounce loop body main.cpp:385-426.
#include <hipcub/hipcub.hpp>
#include <type_traits>

#include "spt_internal.h"

namespace spt {

// A wave-uniform value (every lane active and holding the same value) as a
// scalar: the compiler cannot tell that threadIdx.x >> 6 or a value shuffled
// from lane 0 is uniform, and would otherwise keep the work-pool state in
// VGPRs and branch on it per lane.
#ifndef SPT_UNIFORM
#define SPT_UNIFORM 1
#endif
__device__ __forceinline__ uint32_t wave_uniform(uint32_t v) {
#if SPT_UNIFORM
    return __builtin_amdgcn_readfirstlane(v);
#else
    return v;
#endif
}

// Path-queue and hit-record accesses: each element is written once and read
// once per cast.  kNt (spt_config.queue_cache): non-temporal, so they leave
// L2 / Infinity Cache to the BVH nodes and triangles — a gain where the scene
// itself overflows the Infinity Cache (config 4 +1.7 %), a loss where the
// queue's lines would still be cached when the next kernel reads them
// (config 2 -3.7 %, EXPERIMENTS.md round 4).
typedef float spt_f4v __attribute__((ext_vector_type(4)));
typedef float spt_f2v __attribute__((ext_vector_type(2)));
template <bool kNt = false>
__device__ __forceinline__ float4 ldq(const float4* p) {
    if constexpr (kNt) {
        const spt_f4v v = __builtin_nontemporal_load((const spt_f4v*)p);
        return make_float4(v.x, v.y, v.z, v.w);
    } else {
        return *p;
    }
}
template <bool kNt = false>
__device__ __forceinline__ void stq(float4* p, float4 x) {
    if constexpr (kNt) {
        spt_f4v v = {x.x, x.y, x.z, x.w};
        __builtin_nontemporal_store(v, (spt_f4v*)p);
    } else {
        *p = x;
    }
}
template <bool kNt = false>
__device__ __forceinline__ float2 ldq2(const float2* p) {
    if constexpr (kNt) {
        const spt_f2v v = __builtin_nontemporal_load((const spt_f2v*)p);
        return make_float2(v.x, v.y);
    } else {
        return *p;
    }
}
template <bool kNt = false>
__device__ __forceinline__ void stq2(float2* p, float2 x) {
    if constexpr (kNt) {
        spt_f2v v = {x.x, x.y};
        __builtin_nontemporal_store(v, (spt_f2v*)p);
    } else {
        *p = x;
    }
}

// minimum waves per SIMD the isect kernels are compiled for (register budget)
#ifndef SPT_ISECT_WAVES
#define SPT_ISECT_WAVES 1
#endif
#ifndef SPT_ISECT_WAVES6
#define SPT_ISECT_WAVES6 8
#endif
#ifndef SPT_FUSED_WAVES
#define SPT_FUSED_WAVES 5  // the fused kernel: 6 (80 VGPRs, no spills in unit mode) ran 2 % slower
#endif
// The drain: the unit-mode instance for scenes the caches hold (queue accesses
// cached) at 7 waves (72 VGPRs, 8 B of scratch): config 1 +4 % (5404 vs 5216);
// the streamed-queue instance (scenes beyond the Infinity Cache) at the
// compiler's 6: config 4 at 7 waves -2 % (profiles/r05_exp/ab_diet_waves_sort.log);
// albedo / emitter modes keep the fused kernel's budget (they would spill).
#ifndef SPT_DRAIN_WAVES
#define SPT_DRAIN_WAVES 7
#endif
// the albedo / emitter drains at 6 (80 VGPRs, 32 B of scratch with the path's
// throughput and radiance parked in LDS, SPT_PARK_PATH) instead of the fused
// kernel's 5: config 2 +1.7 % (profiles/r05_exp/fit_paths_rgb_waves/), parking
// +2.5 % more (profiles/r05_exp/park_path/); 7 waves (64 B of scratch) no better
// albedo / emitter lane loops keep a path's throughput and radiance in LDS
// while its ray traces (render_fused_kernel)
#ifndef SPT_PARK_PATH
#define SPT_PARK_PATH 1
#endif
#ifndef SPT_DRAIN_WAVES_RGB
#define SPT_DRAIN_WAVES_RGB 6
#endif
#ifndef SPT_DRAIN_WAVES_NT
#define SPT_DRAIN_WAVES_NT 6
#endif
// lane loops (render_fused_kernel): continued and refilled lanes set up their
// new rays in one tr.init after the refill instead of one each
#ifndef SPT_MERGED_INIT
#define SPT_MERGED_INIT 1
#endif

// Diagnostic build only (make BUILD=build_wlog EXTRA=-DSPT_WAVE_LOG=1,
// tools/wave_log.py): every wave of a lane-loop launch (fused kernel, drain)
// records its start and end on the 100-MHz wall clock, the HW_ID / XCC_ID
// registers (CU, SIMD, SE, hardware queue, XCD), the launch's queue-count
// address (which sub-wavefront) and the paths it shaded.  Read back with
// spt_debug_wave_log (below).  Not in the product build.
#ifndef SPT_WAVE_LOG
#define SPT_WAVE_LOG 0
#endif
#if SPT_WAVE_LOG
struct WaveRec {
    unsigned long long t0, t1;
    uint32_t hw, xcc, tag, casts, block, drain;
};
constexpr uint32_t kWaveLogMax = 1u << 18;
__device__ uint32_t g_wlog_n;
__device__ WaveRec g_wlog[kWaveLogMax];
// ... and, summed over every wave of the lane-loop launches, where a wave's
// time goes (shader clock, s_memtime): [0] cycles in trace steps, [1] cycles
// in shade + refill passes, [2] trace steps, [3] passes, [4] busy lanes summed
// over trace steps, [5] lanes shaded, [6] lanes refilled, [7] cycles in the
// refill part of the passes
constexpr uint32_t kPhaseWords = 8;
__device__ unsigned long long g_phase[kPhaseWords];
#endif

// ------------------------------------------------------------- traversal
// Triangle records (spt_internal.h): vertex i of slot s rotated by r starts at
// float 5 i + r, the original id is float 15.
__device__ __forceinline__ const float* tri_rec(const DeviceScene& sc, uint32_t s) {
    return (const float*)sc.tris + (size_t)s * kTriFloats;
}
__device__ __forceinline__ uint32_t tri_id(const DeviceScene& sc, uint32_t s) { return f2u(tri_rec(sc, s)[kTriIdFloat]); }
__device__ __forceinline__ void tri_vertices(const float* f, V3& a, V3& b, V3& c) {
    a = v3(f[0], f[1], f[2]);
    b = v3(f[5], f[6], f[7]);
    c = v3(f[10], f[11], f[12]);
}

// woop_test's double-precision fallback re-reads the triangle (rare path) so
// the single-precision path need not keep the sheared vertices live; f points
// at the record plus the lane's rotation.
struct TriReload {
    const float* f;
    __device__ __forceinline__ void operator()(V3& a, V3& b, V3& c) const {
        const auto ld = [this](int i) { return __builtin_nontemporal_load(f + i); };
        a = v3(ld(0), ld(1), ld(2)); b = v3(ld(5), ld(6), ld(7)); c = v3(ld(10), ld(11), ld(12));
    }
};

// The block's dynamic LDS: the traversal stacks, [stack_depth][kIsectBlock]
// words (lane-interleaved: conflict-free), then per-lane 16-B records.  Only
// wave-uniform values are kept (SGPRs); a lane derives its slot from its lane
// id, so no per-lane LDS address has to stay live in a VGPR.
struct Lds {
    uint32_t* base;
    uint32_t wbase;  // this wave's first thread index in the block
};
__device__ __forceinline__ uint32_t lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ Lds block_lds(uint32_t* base) {
    return Lds{base, (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u};
}

struct TraceHit {
    int32_t slot;
    uint32_t id;
    float t, u, v;
};

// Analytic spheres after the BVH (smallpt's primitives, spt_scene_set_spheres):
// a sphere nearer than the current hit wins (ties keep it); slot = -2 - k.
// Any-hit queries stop at the first hit.
__device__ __forceinline__ void trace_spheres(const DeviceScene& sc, V3 o, V3 d, float tmin, bool anyhit,
                                              TraceHit& h) {
    if (anyhit && h.slot != -1) return;
    for (uint32_t k = 0; k < sc.nsph; k++) {
        const float t = sphere_t(o, d, sc.spheres[k], tmin, h.t);
        if (t < h.t) {
            h.t = t;
            h.slot = -2 - (int32_t)k;
            h.id = 0xffffffffu;
            h.u = 0.0f;
            h.v = 0.0f;
            if (anyhit) return;
        }
    }
}

struct NoStats {
    __device__ void empty_visit() {}
    __device__ void node() {}
    __device__ void tri() {}
    __device__ void step() {}
    __device__ void push(uint32_t) {}
    __device__ void wave_blocks(bool, bool) {}
};
struct TravStats {
    uint32_t nodes = 0, tris = 0, steps = 0, max_sp = 0, empties = 0;
    uint32_t tri_waves = 0, node_waves = 0;  // wave steps that ran the triangle / the visit block
    __device__ void empty_visit() { empties++; }
    __device__ void node() { nodes++; }
    __device__ void tri() { tris++; }
    __device__ void step() { steps++; }
    __device__ void push(uint32_t sp) { max_sp = max(max_sp, sp); }
    // called by every stepping lane: whether any stepping lane of the wave
    // tests a triangle / visits a node in this step (the SIMD pays the
    // block); the lowest stepping lane counts it, so lane sums are exact
    __device__ void wave_blocks(bool tri_lane, bool node_lane) {
        const uint64_t act = __ballot(true), bt = __ballot(tri_lane), bn = __ballot(node_lane);
        if (lane_id() == (uint32_t)__ffsll((unsigned long long)act) - 1u) {
            tri_waves += bt != 0 ? 1u : 0u;
            node_waves += bn != 0 ? 1u : 0u;
        }
    }
};

// Stack-based BVH2 traversal, near child first, stack in LDS at
// stk[i * kIsectBlock] (lane-interleaved: conflict-free, one bank per lane).
// Closest hit: smallest t, ties broken toward the smaller original triangle
// id so the answer does not depend on the tree.  anyhit: stop at the first
// accepted triangle (OPTIX_RAY_FLAG_TERMINATE_ON_FIRST_HIT).
//
// Resumable: step() advances one node or one leaf and returns true when the
// ray is finished, so a persistent wave can swap finished lanes for new rays.
// One slab of the BVH2 box test: the plane distances (p0 - o) / d, (p1 - o) / d
// as t0, t1 (in either order).  A direction component with an infinite
// reciprocal (d = +-0 or denormal) leaves the ray parallel to the slab: inside
// it for every t (t0, t1 = -inf, +inf) or never (+inf, +inf) — the product
// would be NaN for an origin on a plane.
__device__ __forceinline__ void slab(float p0, float p1, float o, float inv, float& t0, float& t1) {
    if (isinf(inv)) {
        const bool in = o >= p0 && o <= p1;
        t0 = in ? -INFINITY : INFINITY;
        t1 = INFINITY;
        return;
    }
    t0 = (p0 - o) * inv;
    t1 = (p1 - o) * inv;
}

// Box culling lower bound (tbox): boxes the ray leaves before cull_tmin(tmin),
// 4e-6 below tmin, are culled.  With the box-exit rule of the triangle test
// (spt_math.h left_box_before_tmin) every triangle under such a box that the
// Woop test would accept past tmin is dropped by the rule too, so the closest
// hit does not depend on the tree's box sizes.
__device__ __forceinline__ float box_tmin(float tmin) { return cull_tmin(tmin); }

struct Tracer {
    static constexpr int kMinWaves = 1;
    WoopRay wr;
    V3 o;
    float ix, iy, iz, tmin, tbox;
    int32_t node;
    uint32_t sp;
    bool anyhit;
    TraceHit h;

    static constexpr uint32_t kExtraLds = 0;  // LDS bytes per block besides the stack
    __device__ __forceinline__ TraceHit hit(const DeviceScene&, const Lds&) const { return h; }
    __device__ __forceinline__ void init(const DeviceScene& sc, V3 o_, V3 d, float tmin_, float tmax_, bool anyhit_,
                                         const Lds&) {
        o = o_;
        wr = woop_setup(o_, d);
        ix = 1.0f / d.x; iy = 1.0f / d.y; iz = 1.0f / d.z;
        tmin = tmin_;
        tbox = box_tmin(tmin_);
        anyhit = anyhit_;
        node = sc.empty ? kDone : 0;
        sp = 0;
        h.slot = -1; h.id = 0xffffffffu; h.t = tmax_; h.u = 0.0f; h.v = 0.0f;
    }
    static constexpr int32_t kDone = (int32_t)0x7fffffff;
    static constexpr uint32_t kStackWords = 1;
    __device__ __forceinline__ bool finished() const { return node == kDone; }

    __device__ __forceinline__ bool pop(const uint32_t* __restrict__ stk) {
        if (sp == 0) { node = kDone; return true; }
        sp--;
        node = (int32_t)stk[sp * kIsectBlock];
        return false;
    }

    template <typename Stats>
    __device__ __forceinline__ bool step(const DeviceScene& sc, const Lds& L, Stats& stats) {
        stats.step();
        uint32_t* stk = L.base + L.wbase + lane_id();
        if (node >= 0) {
            stats.node();
            const float4* np = sc.nodes + (size_t)node * 4;
            const float4 n0 = np[0], n1 = np[1], n2 = np[2], n3 = np[3];
            float a0, a1, b0, b1, c0, c1;
            slab(n0.x, n0.y, o.x, ix, a0, a1);
            slab(n0.z, n0.w, o.y, iy, b0, b1);
            slab(n2.x, n2.y, o.z, iz, c0, c1);
            const float tn0 = fmaxf(fmaxf(fminf(a0, a1), fminf(b0, b1)), fmaxf(fminf(c0, c1), tbox));
            // exits padded toward +inf (pad_up: a negative per-ray tmin allows negative exits)
            const float tf0 = pad_up(fminf(fminf(fmaxf(a0, a1), fmaxf(b0, b1)), fmaxf(c0, c1)));
            float d0, d1, e0, e1, f0, f1;
            slab(n1.x, n1.y, o.x, ix, d0, d1);
            slab(n1.z, n1.w, o.y, iy, e0, e1);
            slab(n2.z, n2.w, o.z, iz, f0, f1);
            const float tn1 = fmaxf(fmaxf(fminf(d0, d1), fminf(e0, e1)), fmaxf(fminf(f0, f1), tbox));
            const float tf1 = pad_up(fminf(fminf(fmaxf(d0, d1), fmaxf(e0, e1)), fmaxf(f0, f1)));
            // the current hit padded like the exit planes: a box entered at the
            // hit's t (a tie at a shared edge or vertex) is still visited, so
            // the smaller triangle id wins whatever the traversal order
            const float th = pad_up(h.t);
            const bool h0 = tn0 <= fminf(tf0, th);
            const bool h1 = tn1 <= fminf(tf1, th);
            const int32_t ch0 = (int32_t)f2u(n3.x), ch1 = (int32_t)f2u(n3.y);
            if (h0 && h1) {
                const bool swp = tn1 < tn0;
                stk[sp * kIsectBlock] = (uint32_t)(swp ? ch0 : ch1);
                sp++;
                stats.push(sp);
                node = swp ? ch1 : ch0;
                return false;
            }
            if (h0) { node = ch0; return false; }
            if (h1) { node = ch1; return false; }
            return pop(stk);
        }
        const uint32_t code = ~(uint32_t)node;
        const uint32_t first = code >> 3, cnt = (code & 7u) + 1u;
        for (uint32_t i = 0; i < cnt; i++) {
            stats.tri();
            const uint32_t s = first + i;
            const float* f = tri_rec(sc, s);
            V3 p0, p1, p2;
            tri_vertices(f, p0, p1, p2);  // world order (rotation 0)
            float t, u, v;
            if (woop_test(wr, p0, p1, p2, TriReload{f}, tmin, h.t, t, u, v)) {
                const uint32_t id = f2u(f[kTriIdFloat]);
                if (t < h.t || id < h.id) {
                    h.t = t;
                    h.id = id;
                    h.slot = (int32_t)s;
                    h.u = u;
                    h.v = v;
                }
            }
        }
        if (anyhit && h.slot >= 0) { node = kDone; return true; }
        return pop(stk);
    }
};

// Compressed 8-wide BVH traversal (layout: bvh_build.h; after Ylitie et al.
// 2017).  A "node group" (nhits) holds the unvisited inner children of one
// node: hit bits 24..31 at position 24 + (slot ^ oct_inv), so the highest bit
// is the child nearest for this ray's octant, and the node's child-group word
// in bits 0..23 (child s at (word << sc.group_shift) + s, gpu_bvh8_holes).  A "triangle
// group" (tbase, thits) holds the triangles of the hit leaves.
// Child slabs are evaluated as t = q * (2^e / d) + (p - o) / d with one fma;
// each axis is widened by a margin that bounds the fp32 error of that form
// relative to the exact quantised planes (which already enclose the child),
// so culling stays conservative and the closest hit is the exact Woop one.
// (the margin is formed as one mul and one fma: it bounds the rounding of the
// slab form with several ulps to spare, so its own rounding does not matter)
constexpr float kMarginRel = 1e-6f;
// Step modes (template argument of Tracer8T): 0 = one triangle test OR one
// node visit per step; 1 = the last triangle of a group rides along with the
// next node visit; 2 = as 1 with a second triangle-group slot, so a node visit
// rides along with any triangle test while that slot is free.
#ifndef SPT_MERGED_STEP
#define SPT_MERGED_STEP 2
#endif
#ifndef SPT_FUSED_STEP
#define SPT_FUSED_STEP 2
#endif
#ifndef SPT_EARLY_DONE
#define SPT_EARLY_DONE 1
#endif
constexpr float kMinDir = 1e-20f;

// kLds: the per-ray Woop constants (Sx, Sy, Sz, axis indices) and the hit
// record (slot, id, u, v) live in LDS, one 16-B record each per lane after the
// stack (ds_read_b128 / ds_write_b128, conflict-free), not in VGPRs; only the
// hit distance stays in a register (every box test reads it).
//
// kW = 6: the 64-B node of bvh_build.h (at most six children; one 64-B
// half-line per visit, four loads instead of five; same hit-bit scheme).
//
// kDefer (with kLds): the hit record keeps the un-divided barycentrics and
// the divides run once per ray (the fused kernel: +2.6 %; the isect kernel,
// which finishes a ray about as often as it accepts a hit: -0.7 %).
template <int kStep, bool kLds, int kW = 8, bool kDefer = false>
struct Tracer8T {
    static constexpr uint32_t kQuads = kW == 6 ? kNode6Quads : kNode8Quads;
    // the 64-B node's visit fits 64 VGPRs: 8 waves per SIMD where the LDS
    // stack allows it (the 80-B node's spills there)
    static constexpr int kMinWaves = kW == 6 ? SPT_ISECT_WAVES6 : SPT_ISECT_WAVES;
    WoopRay wr;
    V3 o;
    float ix, iy, iz, tmin, tbox;
    // the ray's inverted octant (0..7) replicated in every byte; bits 3-4 of the
    // low byte hold the triangle-record rotation (0..2) of the ray's dominant
    // axis (the octant users mask each byte to its low 3 bits)
    uint32_t oct_rep;
    // node group: unvisited hit children in bits 24..31 (bit 24 + (slot ^
    // octant)), the child-group word in bits 0..23 (child s of a node sits at
    // (word << group_shift) + s, gpu_bvh8_holes) — one word, also one LDS stack entry
    uint32_t nhits;
    uint32_t tbase, thits;
    uint32_t tbase2, thits2;  // kStep 2: a second triangle group, queued behind (tbase, thits)
    uint32_t spa;  // byte offset of this lane's stack top in the block's LDS: tid * 4 + depth * 512
    bool anyhit, done;
    TraceHit h;
    static constexpr uint32_t kStackWords = 1;
    static constexpr uint32_t kExtraLds = kLds ? 2 * kIsectBlock * 16 : 0;
    static constexpr uint32_t kRow = kIsectBlock * 4;  // bytes per stack level
    __device__ __forceinline__ bool finished() const { return done; }

    __device__ __forceinline__ uint32_t* stack_top(const Lds& L) const { return (uint32_t*)((char*)L.base + spa); }
    // this lane's records (tid * 16 = (spa % kRow) * 4)
    __device__ __forceinline__ uint4* wrec(const DeviceScene& sc, const Lds& L) const {
        return (uint4*)((char*)L.base + sc.stack_depth * kRow + (spa & (kRow - 1u)) * 4u);
    }
    __device__ __forceinline__ uint4* hrec(const DeviceScene& sc, const Lds& L) const {
        return wrec(sc, L) + kIsectBlock;
    }
    // The LDS hit record: (slot, -, u, v); with kDefer (slot, V, W, det),
    // u = V / det and v = W / det divided once for the hit the ray keeps.  The
    // original id is read back from the triangle record (the isect queue
    // kernel writes the slot and never asks for it).
    __device__ __forceinline__ TraceHit hit(const DeviceScene& sc, const Lds& L) const {
        if constexpr (!kLds) return h;
        const uint4 r = *hrec(sc, L);
        TraceHit x;
        x.slot = (int32_t)r.x;
        x.t = h.t;
        if (r.x == 0xffffffffu) {
            x.id = 0xffffffffu; x.u = 0.0f; x.v = 0.0f;
        } else if constexpr (!kDefer) {
            x.id = tri_id(sc, r.x); x.u = u2f(r.z); x.v = u2f(r.w);
        } else {
            x.id = tri_id(sc, r.x);
            x.u = u2f(r.y) / u2f(r.w) + 0.0f;  // as woop_test: a zero is +0
            x.v = u2f(r.z) / u2f(r.w) + 0.0f;
        }
        return x;
    }
    __device__ __forceinline__ uint32_t rot() const { return (oct_rep >> 3) & 3u; }
    // the origin in the rotated records' (kx, ky, kz) order
    __device__ __forceinline__ V3 rot_origin() const {
        const uint32_t r = rot();
        return r == 0 ? o : (r == 1 ? v3(o.y, o.z, o.x) : v3(o.z, o.x, o.y));
    }

    __device__ __forceinline__ void init(const DeviceScene& sc, V3 o_, V3 d, float tmin_, float tmax_, bool anyhit_,
                                         const Lds& L) {
        o = o_;
        wr = woop_setup(o_, d);
        spa = (L.wbase + lane_id()) * 4u;
        if constexpr (kLds) {
            *wrec(sc, L) = make_uint4(f2u(wr.Sx), f2u(wr.Sy), f2u(wr.Sz), wr.k);
            // "no hit": slot -1, id ~0 (materialised here: a constant vector
            // hoisted out of the ray loop would occupy four VGPRs throughout)
            uint32_t none, zero;
            asm volatile("v_mov_b32 %0, -1" : "=v"(none));
            asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
            *hrec(sc, L) = make_uint4(none, none, zero, zero);
        }
        const float dx = fabsf(d.x) < kMinDir ? copysignf(kMinDir, d.x) : d.x;
        const float dy = fabsf(d.y) < kMinDir ? copysignf(kMinDir, d.y) : d.y;
        const float dz = fabsf(d.z) < kMinDir ? copysignf(kMinDir, d.z) : d.z;
        // hardware reciprocal (<= 1 ulp): the slab margins (kMarginRel) absorb
        // it, and the triangle test keeps its own correctly rounded divides
        ix = __builtin_amdgcn_rcpf(dx); iy = __builtin_amdgcn_rcpf(dy); iz = __builtin_amdgcn_rcpf(dz);
        const uint32_t oct = (ix < 0.0f ? 1u : 0u) | (iy < 0.0f ? 2u : 0u) | (iz < 0.0f ? 4u : 0u);
        const uint32_t oct_inv = oct ^ 7u;
        const uint32_t kz = wr.k >> 4;  // rotation r = (kz + 1) mod 3 puts kz last
        oct_rep = oct_inv * 0x01010101u | ((kz == 2u ? 0u : kz + 1u) << 3);
        tmin = tmin_;
        tbox = box_tmin(tmin_);
        anyhit = anyhit_;
        nhits = 1u << (24u + oct_inv);  // the root: slot 0 of a virtual group at node 0
        tbase = 0;
        thits = 0;
        tbase2 = 0;
        thits2 = 0;
        done = sc.empty != 0;
        h.slot = -1; h.id = 0xffffffffu; h.t = tmax_; h.u = 0.0f; h.v = 0.0f;
    }

    __device__ __forceinline__ void visit(const DeviceScene& sc, uint32_t node) {
        const uint4* np = sc.nodes8 + (size_t)node * kQuads;
        if constexpr (kW == 6) visit_words6(np[0], np[1], np[2], np[3]);
        else visit_words(np[0], np[1], np[2], np[3], np[4]);
    }

    // inner children's meta bytes 0b001_11sss (24 + slot) take the ray's
    // octant in their low 3 bits (byte-wise, once per meta word), so every
    // child contributes (m >> 5) << (m & 31) with no branch.  A byte is an
    // inner child iff its bits 3 and 4 are set (leaf offsets are < 24).
    __device__ __forceinline__ uint32_t octx(uint32_t mw) const {
        const uint32_t t8 = mw & (mw >> 1) & 0x08080808u;  // 0x08 in inner bytes
        return mw ^ ((t8 - (t8 >> 3)) & oct_rep);          // 0x07 & octant
    }

    __device__ __forceinline__ void take_hits(uint32_t hm, uint32_t group, uint32_t tri_base) {
        nhits = (hm & 0xff000000u) | group;
        if constexpr (kStep >= 2) {
            if (thits) {  // the current group still has triangles: queue the new one
                tbase2 = tri_base;
                thits2 = hm & 0x00ffffffu;
                return;
            }
        }
        tbase = tri_base;
        thits = hm & 0x00ffffffu;
    }

    // The 64-B node: q0 = (origin, tri_base), q1 = (meta 0-3, meta 4-5 | ex |
    // ey, group | ez, lo.x 0-3), q2 = (hi.x, lo.y, hi.y, lo.z 0-3), q3 =
    // (hi.z 0-3, then per axis lo4 lo5 hi4 hi5).
    __device__ __forceinline__ void visit_words6(const uint4 q0, const uint4 q1, const uint4 q2, const uint4 q3) {
        const float ax = u2f(((q1.y >> 16) & 0xffu) << 23) * ix;
        const float ay = u2f((q1.y >> 24) << 23) * iy;
        const float az = u2f((q1.z >> 24) << 23) * iz;
        const float bx = (u2f(q0.x) - o.x) * ix;
        const float by = (u2f(q0.y) - o.y) * iy;
        const float bz = (u2f(q0.z) - o.z) * iz;
        const float mx = fmaf(fabsf(ax), 255.0f * kMarginRel, fabsf(bx) * kMarginRel);
        const float my = fmaf(fabsf(ay), 255.0f * kMarginRel, fabsf(by) * kMarginRel);
        const float mz = fmaf(fabsf(az), 255.0f * kMarginRel, fabsf(bz) * kMarginRel);
        const float bxe = bx - mx, bxx = bx + mx, bye = by - my, byx = by + my, bze = bz - mz, bzx = bz + mz;
        const bool px = ix >= 0.0f, py = iy >= 0.0f, pz = iz >= 0.0f;
        const uint32_t exl = px ? q1.w : q2.x, xxl = px ? q2.x : q1.w;
        const uint32_t eyl = py ? q2.y : q2.z, xyl = py ? q2.z : q2.y;
        const uint32_t ezl = pz ? q2.w : q3.x, xzl = pz ? q3.x : q2.w;
        // children 4 and 5: entry planes into bytes 0-1, exit planes into 2-3
        const uint32_t e45x = px ? q3.y : __builtin_amdgcn_alignbit(q3.y, q3.y, 16u);
        const uint32_t e45y = py ? q3.z : __builtin_amdgcn_alignbit(q3.z, q3.z, 16u);
        const uint32_t e45z = pz ? q3.w : __builtin_amdgcn_alignbit(q3.w, q3.w, 16u);
        uint32_t hm = 0;
        const uint32_t mlo = octx(q1.x), mhi = octx(q1.y);
#pragma unroll
        for (uint32_t c = 0; c < 6; c++) {
            const uint32_t sh = (c & 3u) * 8u;
            const bool lo = c < 4;
            const float tex = fmaf((float)(((lo ? exl : e45x) >> sh) & 0xffu), ax, bxe);
            const float txx = fmaf((float)(((lo ? xxl : e45x) >> (lo ? sh : sh + 16u)) & 0xffu), ax, bxx);
            const float tey = fmaf((float)(((lo ? eyl : e45y) >> sh) & 0xffu), ay, bye);
            const float txy = fmaf((float)(((lo ? xyl : e45y) >> (lo ? sh : sh + 16u)) & 0xffu), ay, byx);
            const float tez = fmaf((float)(((lo ? ezl : e45z) >> sh) & 0xffu), az, bze);
            const float txz = fmaf((float)(((lo ? xzl : e45z) >> (lo ? sh : sh + 16u)) & 0xffu), az, bzx);
            const float tn = fmaxf(fmaxf(tex, tey), fmaxf(tez, tbox));
            const float tf = fminf(fminf(txx, txy), fminf(txz, h.t));
            const uint32_t mw = lo ? mlo : mhi;
            const uint32_t bits = __builtin_amdgcn_ubfe(mw, sh + 5u, 3u) << __builtin_amdgcn_ubfe(mw, sh, 5u);
            hm = (tn <= tf) ? (hm | bits) : hm;
        }
        take_hits(hm, q1.z & 0x00ffffffu, q0.w);
    }

    __device__ __forceinline__ void visit_words(const uint4 w0, const uint4 w1, const uint4 w2, const uint4 w3,
                                                const uint4 w4) {
        const uint32_t ew = w0.w;
        const float ax = u2f((ew & 0xffu) << 23) * ix;
        const float ay = u2f(((ew >> 8) & 0xffu) << 23) * iy;
        const float az = u2f(((ew >> 16) & 0xffu) << 23) * iz;
        const float bx = (u2f(w0.x) - o.x) * ix;
        const float by = (u2f(w0.y) - o.y) * iy;
        const float bz = (u2f(w0.z) - o.z) * iz;
        const float mx = fmaf(fabsf(ax), 255.0f * kMarginRel, fabsf(bx) * kMarginRel);
        const float my = fmaf(fabsf(ay), 255.0f * kMarginRel, fabsf(by) * kMarginRel);
        const float mz = fmaf(fabsf(az), 255.0f * kMarginRel, fabsf(bz) * kMarginRel);
        const float bxe = bx - mx, bxx = bx + mx, bye = by - my, byx = by + my, bze = bz - mz, bzx = bz + mz;
        // entry planes are the lo planes for a positive direction, hi otherwise
        const bool px = ix >= 0.0f, py = iy >= 0.0f, pz = iz >= 0.0f;
        const uint32_t exl = px ? w2.x : w3.z, exh = px ? w2.y : w3.w, xxl = px ? w3.z : w2.x, xxh = px ? w3.w : w2.y;
        const uint32_t eyl = py ? w2.z : w4.x, eyh = py ? w2.w : w4.y, xyl = py ? w4.x : w2.z, xyh = py ? w4.y : w2.w;
        const uint32_t ezl = pz ? w3.x : w4.z, ezh = pz ? w3.y : w4.w, xzl = pz ? w4.z : w3.x, xzh = pz ? w4.w : w3.y;
        uint32_t hm = 0;
        const uint32_t mlo = octx(w1.z), mhi = octx(w1.w);
#pragma unroll
        for (uint32_t c = 0; c < 8; c++) {
            const uint32_t sh = (c & 3u) * 8u;
            const bool lo = c < 4;
            const float tex = fmaf((float)(((lo ? exl : exh) >> sh) & 0xffu), ax, bxe);
            const float txx = fmaf((float)(((lo ? xxl : xxh) >> sh) & 0xffu), ax, bxx);
            const float tey = fmaf((float)(((lo ? eyl : eyh) >> sh) & 0xffu), ay, bye);
            const float txy = fmaf((float)(((lo ? xyl : xyh) >> sh) & 0xffu), ay, byx);
            const float tez = fmaf((float)(((lo ? ezl : ezh) >> sh) & 0xffu), az, bze);
            const float txz = fmaf((float)(((lo ? xzl : xzh) >> sh) & 0xffu), az, bzx);
            const float tn = fmaxf(fmaxf(tex, tey), fmaxf(tez, tbox));
            const float tf = fminf(fminf(txx, txy), fminf(txz, h.t));
            const uint32_t mw = lo ? mlo : mhi;
            const uint32_t bits = __builtin_amdgcn_ubfe(mw, sh + 5u, 3u) << __builtin_amdgcn_ubfe(mw, sh, 5u);
            hm = (tn <= tf) ? (hm | bits) : hm;
        }
        take_hits(hm, w1.x, w1.y);
    }

    // P0..P2: the slot's vertices loaded rotated by rot() (f: the record + rot)
    __device__ __forceinline__ bool tri_test(const DeviceScene& sc, V3 P0, V3 P1, V3 P2, const float* f, uint32_t s,
                                             const Lds& L, const uint4 wk) {
        float t, u, v;
        WoopRay wl;
        wl.o = o;
        if constexpr (kLds) { wl.Sx = u2f(wk.x); wl.Sy = u2f(wk.y); wl.Sz = u2f(wk.z); wl.k = wk.w; }
        else wl = wr;
        const V3 O = rot_origin();
        if constexpr (kLds) {
            uint4* hr = hrec(sc, L);
            if constexpr (!kDefer) {
                if (woop_test_rot(wl, O, P0, P1, P2, TriReload{f}, tmin, h.t, t, u, v)) {
                    // accepted means t <= h.t; a tie goes to the smaller original
                    // id (both read from the triangle records: rare)
                    bool take = t < h.t;
                    if (!take) {
                        const uint32_t cs = hr->x;
                        take = cs == 0xffffffffu || tri_id(sc, s) < tri_id(sc, cs);
                    }
                    if (take) {
                        h.t = t;
                        *hr = make_uint4((uint32_t)s, 0u, f2u(u), f2u(v));
                    }
                    return true;
                }
                return false;
            }
            float V, W, det;
            if (woop_test_raw_rot(wl, O, P0, P1, P2, TriReload{f}, tmin, h.t, t, V, W, det)) {
                bool take = t < h.t;
                if (!take) {
                    const uint32_t cs = hr->x;
                    take = cs == 0xffffffffu || tri_id(sc, s) < tri_id(sc, cs);
                }
                if (take) {
                    h.t = t;
                    *hr = make_uint4((uint32_t)s, f2u(V), f2u(W), f2u(det));
                }
                return true;
            }
            return false;
        }
        if (woop_test_rot(wl, O, P0, P1, P2, TriReload{f}, tmin, h.t, t, u, v)) {
            const uint32_t id = tri_id(sc, s);
            if (t < h.t || id < h.id) {
                h.t = t;
                h.id = id;
                h.slot = (int32_t)s;
                h.u = u;
                h.v = v;
            }
            return true;
        }
        return false;
    }

    template <typename Stats>
    __device__ __forceinline__ bool step(const DeviceScene& sc, const Lds& L, Stats& stats) {
        if constexpr (kStep == 0) return step_single(sc, L, stats);
        else return step_merged(sc, L, stats);
    }

    // One step = at most one triangle test and one node visit, their loads in
    // flight together: a lane whose triangle group is down to its last
    // triangle also visits its next node (the visit may start a new group),
    // so most triangle tests cost no dependent memory round trip of their own.
    // The visit culls against the hit the triangle test just made.
    template <typename Stats>
    __device__ __forceinline__ bool step_merged(const DeviceScene& sc, const Lds& L, Stats& stats) {
        stats.step();
        if constexpr (kStep >= 2) {
            if (!thits) {
                tbase = tbase2;
                thits = thits2;
                thits2 = 0u;
            }
        }
        const bool has_tri = thits != 0u;
        const bool has_node = (nhits & 0xff000000u) != 0u || spa >= kRow;
        if (!has_tri && !has_node) { done = true; return true; }
        const bool do_node = kStep >= 2 ? has_node && thits2 == 0u     // a free slot for the visit's triangles
                                        : has_node && (thits & (thits - 1u)) == 0u;
        // loads are unconditional (idle sides read slot / node 0, always
        // cached) so both sets are in flight before either is waited on
        const uint32_t s = has_tri ? tbase + (uint32_t)__builtin_ctz(thits) : 0u;
        if (has_tri) stats.tri();
        thits &= thits - 1u;
        const float* f = tri_rec(sc, s) + rot();
        V3 P0, P1, P2;
        tri_vertices(f, P0, P1, P2);
        uint4 wk = make_uint4(0u, 0u, 0u, 0u);
        if constexpr (kLds) wk = *wrec(sc, L);
        if (do_node && !(nhits & 0xff000000u)) {
            spa -= kRow;
            nhits = *stack_top(L);
        }
        const uint32_t bit = 31u - (uint32_t)__builtin_clz(nhits | 1u);
        const uint32_t child = ((nhits & 0x00ffffffu) << sc.group_shift) + (((bit - 24u) ^ oct_rep) & 7u);
        const uint32_t node = do_node ? child : 0u;
        stats.wave_blocks(has_tri, do_node);
        if (do_node) {
            stats.node();
            nhits &= ~(1u << bit);
            if (nhits & 0xff000000u) {
                *stack_top(L) = nhits;
                spa += kRow;
                stats.push(spa / kRow);
            }
        }
        const uint4* np = sc.nodes8 + (size_t)node * kQuads;
        const uint4 w0 = np[0], w1 = np[1], w2 = np[2], w3 = np[3];
        uint4 w4 = w3;
        if constexpr (kW != 6) w4 = np[4];
        if (has_tri && tri_test(sc, P0, P1, P2, f, s, L, wk) && anyhit) { done = true; return true; }
        if (do_node) {
            const uint32_t tb = thits | thits2;
            if constexpr (kW == 6) visit_words6(w0, w1, w2, w3);
            else visit_words(w0, w1, w2, w3, w4);
            if (!(nhits & 0xff000000u) && (thits | thits2) == tb) stats.empty_visit();  // no child box hit
        }
#if SPT_EARLY_DONE
        // nothing left (no triangles, no hit children, empty stack): finish
        // now rather than in a step of its own, so the lane is idle (and can
        // be refilled) one step sooner
        if (!(thits | thits2 | (nhits & 0xff000000u)) && spa < kRow) { done = true; return true; }
#endif
        return false;
    }

    template <typename Stats>
    __device__ __forceinline__ bool step_single(const DeviceScene& sc, const Lds& L, Stats& stats) {
        stats.step();
        if (thits) {
            stats.tri();
            const uint32_t s = tbase + (uint32_t)__builtin_ctz(thits);
            thits &= thits - 1u;
            const float* f = tri_rec(sc, s) + rot();
            V3 P0, P1, P2;
            tri_vertices(f, P0, P1, P2);
            uint4 wk = make_uint4(0u, 0u, 0u, 0u);
            if constexpr (kLds) wk = *wrec(sc, L);
            if (tri_test(sc, P0, P1, P2, f, s, L, wk) && anyhit) { done = true; return true; }
            return false;
        }
        if (!(nhits & 0xff000000u)) {
            // current group exhausted: pop the next one (stacked groups always
            // hold inner children) and visit its nearest child in this step
            if (spa < kRow) { done = true; return true; }
            spa -= kRow;
            nhits = *stack_top(L);
        }
        stats.node();
        const uint32_t bit = 31u - (uint32_t)__builtin_clz(nhits);
        const uint32_t child = ((nhits & 0x00ffffffu) << sc.group_shift) + (((bit - 24u) ^ oct_rep) & 7u);
        nhits &= ~(1u << bit);
        if (nhits & 0xff000000u) {
            *stack_top(L) = nhits;
            spa += kRow;
            stats.push(spa / kRow);
        }
        visit(sc, child);
        return false;
    }
};
#ifndef SPT_LDS_RAY
#define SPT_LDS_RAY 1
#endif
using Tracer8 = Tracer8T<SPT_MERGED_STEP, SPT_LDS_RAY>;  // isect kernels
using Tracer6 = Tracer8T<SPT_MERGED_STEP, SPT_LDS_RAY, 6>;  // isect kernels, 64-B nodes
#ifndef SPT_FUSED_LDS
#define SPT_FUSED_LDS 1
#endif
using Tracer8F = Tracer8T<SPT_FUSED_STEP, SPT_FUSED_LDS, 8, true>;  // fused trace+shade kernel
using Tracer6F = Tracer8T<SPT_FUSED_STEP, SPT_FUSED_LDS, 6, true>;

template <typename Tr, typename Stats = NoStats>
__device__ __forceinline__ TraceHit trace(const DeviceScene& sc, V3 o, V3 d, float tmin, float tmax,
                                          bool anyhit, const Lds& L, Stats& stats) {
    Tr tr;
    tr.init(sc, o, d, tmin, tmax, anyhit, L);
    if (!tr.finished())
        while (!tr.step(sc, L, stats)) {
        }
    return tr.hit(sc, L);
}

// Persistent wavefront isect over the path queue.  The grid holds only as
// many workgroups as fit on the chip; each wave keeps 64 rays in flight and,
// whenever kRefillIdle lanes have finished (or all have), refills them from
// its work pool.  Each wave first owns a static contiguous share of 3/4 of the
// queue (no atomics), then takes kIsectChunk-ray chunks of the remaining
// quarter from the launch-wide counter *a.next, which evens out the tail.
// The last cast of a path only needs a yes/no answer (a miss is the only thing
// that contributes, main.cpp:407), so it runs as an any-hit query.
__device__ __forceinline__ void camera_ray(const Camera& cam, Pcg32& rng, uint32_t order, uint32_t x, uint32_t y,
                                           V3& o, V3& d);

// A new camera path for work item w (refill_kernel's arithmetic): its ray,
// tile pixel p and meta (sample << 8, cast 0).
__device__ __forceinline__ void start_path(const RefillArgs& r, uint64_t w, V3& o, V3& d, uint32_t& p, uint32_t& meta) {
    uint32_t s, q, lx, ly;
    work_item((uint32_t)(w - (uint64_t)r.chunk_s0 * r.P), r.chunk_s0, r.chunk_ns, r.P, r.work_order != 0, s, q);
    work_pixel(q, r.W, r.P, r.pixel_block, lx, ly);
    p = ly * r.W + lx;
    const uint32_t gy = tile_global_row(ly, r.tile_index, r.tile_count, r.rows_per_group);
    const uint32_t gpix = gy * r.W + lx;                    // main.cpp:379-382
    Pcg32 rng = pcg_start(r.sample_jump[s], (uint64_t)gpix);  // main.cpp:376, then the sample's draws
    camera_ray(r.cam, rng, r.rng_order, lx, gy, o, d);
    meta = s << kMetaDepthBits;
}

#ifndef SPT_ISECT_CAM_WAVES
#define SPT_ISECT_CAM_WAVES 8
#endif
template <typename Tr, bool kStats, bool kCam = false, bool kNt = false>
__global__ __launch_bounds__(kIsectBlock)
__attribute__((amdgpu_waves_per_eu(kStats ? 1 : (kCam ? SPT_ISECT_CAM_WAVES : Tr::kMinWaves), 8)))
void isect_queue_kernel(IsectQueueArgs a) {
    extern __shared__ uint32_t lds_stack[];
    const Lds L = block_lds(lds_stack);
    uint32_t n, nq = 0;
    uint64_t cur = 0;
    if constexpr (kCam) {
        // survivors in [0, nq), new camera paths in [nq, n) (refill_kernel's rule)
        nq = wave_uniform(*a.cam.surv);
        cur = a.cam.cursor_in ? *a.cam.cursor_in : a.cam.cursor_init;
        const uint64_t avail = a.cam.work_end > cur ? a.cam.work_end - cur : 0;
        const uint32_t room = a.cam.capacity - nq;
        const uint32_t total = (uint32_t)(avail < room ? avail : room);
        n = nq + total;
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            *a.cam.cursor_out = cur + total;
            *a.cam.qn_out = n;
            *a.cam.isect_next = 0;  // the next launch's work counter
            *a.cam.surv_clear = 0;  // the shade after this launch appends survivors there
            if (cur < a.cam.work_end && cur + total >= a.cam.work_end) *a.cam.exhausted = a.cam.iter_tag;
            if (n) atomicAdd(&a.cam.stats[0], (unsigned long long)n);       // casts
            if (nq) atomicAdd(&a.cam.stats[1], (unsigned long long)nq);     // continuations
            if (total) atomicAdd(&a.cam.stats[2], (unsigned long long)total);  // camera paths started
        }
    } else {
        n = *a.count;
        if (n < a.drain_below) return;  // the drain launch after the shade takes this queue
    }
    typename std::conditional<kStats, TravStats, NoStats>::type st;
    Tr tr;
    uint32_t ray = 0;
    bool busy = false;
    // wave-uniform pool state
    const uint32_t nwaves = gridDim.x * (kIsectBlock / 64);
    const uint32_t blk = a.xcd_remap ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint32_t wave_id = wave_uniform(blk * (kIsectBlock / 64) + (threadIdx.x >> 6));
    const uint32_t share = (uint32_t)(((uint64_t)n * a.static_share_q8 / 256) / nwaves);
    const uint32_t dyn_base = share * nwaves;
    uint32_t pool = wave_id * share, pool_end = pool + share;
    bool drained = false;
    uint32_t wave_steps = 0;
    while (true) {
        uint64_t idle = __ballot(!busy);
        const uint32_t nidle = (uint32_t)__popcll(idle);
        if (nidle >= a.refill_idle) {
            while (idle && !(drained && pool == pool_end)) {
                if (pool == pool_end) {
                    uint32_t base = 0;
                    if ((threadIdx.x & 63u) == 0) base = atomicAdd(a.next, a.chunk);
                    base = dyn_base + wave_uniform((uint32_t)__shfl((int)base, 0));
                    if (base >= n) { drained = true; break; }
                    pool = base;
                    pool_end = min(base + a.chunk, n);
                }
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                const uint32_t take = min((uint32_t)__popcll(idle), pool_end - pool);
                if (!busy && rank < take) {
                    ray = pool + rank;
                    V3 o, d;
                    uint32_t depth;
                    if (!kCam || ray < nq) {
                        const float4 q1 = ldq<kNt>(a.q.q1 + ray), q2 = ldq<kNt>(a.q.q2 + ray);
                        o = v3(q1.x, q1.y, q1.z);
                        d = v3(q2.x, q2.y, q2.z);
                        depth = f2u(q1.w) & ((1u << kMetaDepthBits) - 1u);
                    } else {
                        // a new camera path: its ray is made here and stored for the shade
                        uint32_t p, meta;
                        start_path(a.cam, cur + (ray - nq), o, d, p, meta);
                        stq<kNt>(a.q.q1 + ray, make_float4(o.x, o.y, o.z, u2f(meta)));
                        stq<kNt>(a.q.q2 + ray, make_float4(d.x, d.y, d.z, u2f(p)));
                        if (a.cam.mode >= kModeAlbedo) stq<kNt>(a.q.q0 + ray, make_float4(1.0f, 1.0f, 1.0f, 0.0f));
                        if (a.cam.mode == kModeEmit) stq2<kNt>(a.q.rad + ray, make_float2(0.0f, 0.0f));
                        depth = 0;
                    }
                    // any-hit for the last cast unless emitters need the surface
                    tr.init(a.sc, o, d, kRayTmin, kRayTmax, depth + 1 >= a.max_depth && !a.sc.emission, L);
                    busy = !tr.finished();
                    if (!busy) {  // empty scene: the miss record init made
                        const TraceHit hh = tr.hit(a.sc, L);
                        stq<kNt>(a.hits + ray, make_float4(u2f((uint32_t)hh.slot), hh.t, hh.u, hh.v));
                    }
                }
                pool += take;
                idle = __ballot(!busy);
            }
        }
        if (!__ballot(busy)) break;
        wave_steps++;
        if (busy && tr.step(a.sc, L, st)) {
            const TraceHit hh = tr.hit(a.sc, L);
            stq<kNt>(a.hits + ray, make_float4(u2f((uint32_t)hh.slot), hh.t, hh.u, hh.v));
            busy = false;
        }
    }
    if constexpr (kStats) {
        atomicAdd(&a.trav_stats[0], (unsigned long long)st.nodes);
        atomicAdd(&a.trav_stats[1], (unsigned long long)st.tris);
        atomicAdd(&a.trav_stats[2], (unsigned long long)st.steps);
        if ((threadIdx.x & 63u) == 0) atomicAdd(&a.trav_stats[3], (unsigned long long)wave_steps);
        atomicAdd(&a.trav_stats[5], (unsigned long long)st.tri_waves);
        atomicAdd(&a.trav_stats[6], (unsigned long long)st.node_waves);
#if SPT_EMPTY_VISIT_STAT
        atomicAdd(&a.trav_stats[4], (unsigned long long)st.empties);  // experiment: visits with no child hit
#else
        atomicMax(&a.trav_stats[4], (unsigned long long)st.max_sp);
#endif
    }
}

// The first cast of a job that fits in flight (spt_config.lockstep_first):
// one lane per queued ray, no lane refill.  Those are the camera rays, and
// coherent ones (a wave holds one pixel's 64 samples in pixel-major order:
// 94 % SIMD efficiency on config 1, tools/trav_stats.py), so a wave's lanes
// finish together and the persistent kernel's machinery — pool atomics,
// idle-lane ballots, a refill branch whose temporaries sit beside the
// traversal state — only costs: config 1's camera casts trace at 17.5 Grays/s
// here against 10.4 in isect_queue_kernel (profiles/r05_exp/lockstep_first/).
// Later casts are incoherent, where the persistent kernel wins.  The same
// tracer and hit record as isect_queue_kernel, so the same bits.
template <typename Tr, bool kNt>
__global__ __launch_bounds__(kIsectBlock) __attribute__((amdgpu_waves_per_eu(Tr::kMinWaves, 8)))
void isect_lockstep_kernel(IsectQueueArgs a) {
    extern __shared__ uint32_t lds_stack[];
    const Lds L = block_lds(lds_stack);
    const uint32_t n = *a.count;
    if (n < a.drain_below) return;  // the drain launch after the shade takes this queue
    const uint32_t i = blockIdx.x * kIsectBlock + threadIdx.x;
    if (i >= n) return;
    const float4 q1 = ldq<kNt>(a.q.q1 + i), q2 = ldq<kNt>(a.q.q2 + i);
    const uint32_t depth = f2u(q1.w) & ((1u << kMetaDepthBits) - 1u);
    NoStats st;
    Tr tr;
    // any-hit for the last cast unless emitters need the surface (isect_queue_kernel)
    tr.init(a.sc, v3(q1.x, q1.y, q1.z), v3(q2.x, q2.y, q2.z), kRayTmin, kRayTmax,
            depth + 1 >= a.max_depth && !a.sc.emission, L);
    if (!tr.finished())
        while (!tr.step(a.sc, L, st)) {
        }
    const TraceHit hh = tr.hit(a.sc, L);
    stq<kNt>(a.hits + i, make_float4(u2f((uint32_t)hh.slot), hh.t, hh.u, hh.v));
}

// __raygen__rg (wavefront_isect.cu:80-112) semantics for the public C ABI.
// One instance per node format, so each keeps only its own tracer's registers.
template <typename Tr>
__global__ __launch_bounds__(kIsectBlock) void isect_public_kernel(IsectPublicArgs a) {
    extern __shared__ uint32_t lds_stack[];
    const uint32_t i = blockIdx.x * kIsectBlock + threadIdx.x;
    if (i >= a.n) return;
    const bool m = !a.mask || ((a.mask_size == 1) ? (a.mask[0] != 0) : (a.mask[i] != 0));
    if (!m) return;
    const V3 o = v3(a.ox[i], a.oy[i], a.oz[i]);
    const V3 d = v3(a.dx[i], a.dy[i], a.dz[i]);
    const float tmin = a.tmin ? a.tmin[i] : kRayTmin, tmax = a.tmax ? a.tmax[i] : kRayTmax;
    NoStats st;
    TraceHit h = trace<Tr>(a.sc, o, d, tmin, tmax, a.closest == 0, block_lds(lds_stack), st);
    if (a.sc.nsph) trace_spheres(a.sc, o, d, tmin, a.closest == 0, h);
    if (h.slot == -1) {
        a.tri_id[i] = -1;
        return;
    }
    a.tri_id[i] = h.slot >= 0 ? (int32_t)h.id : h.slot;  // spheres: -2 - k
    a.t[i] = h.t;
    a.u[i] = h.u;
    a.v[i] = h.v;
}

// The same semantics over the compressed BVH8 as a persistent kernel: a grid
// of at most the chip's occupancy, each wave owning a contiguous share of the
// rays (no atomics, so concurrent calls on different streams need no shared
// counter) and refilling its finished lanes from that share, so lanes do not
// idle behind a wave's slowest ray.  Masked-off rays take a slot and write
// nothing (wavefront_isect.cu:86).
template <typename Tr>
__global__ __launch_bounds__(kIsectBlock) __attribute__((amdgpu_waves_per_eu(Tr::kMinWaves, 8)))
void isect_public_persistent_kernel(IsectPublicArgs a) {
    extern __shared__ uint32_t lds_stack[];
    const Lds L = block_lds(lds_stack);
    NoStats st;
    Tr tr;
    uint32_t ray = 0;
    bool busy = false;
    const uint32_t nwaves = gridDim.x * (kIsectBlock / 64);
    const uint32_t wave_id = wave_uniform(blockIdx.x * (kIsectBlock / 64) + (threadIdx.x >> 6));
    const uint32_t share = (uint32_t)(((uint64_t)a.n + nwaves - 1) / nwaves);
    uint32_t pool = min(a.n, wave_id * share);
    const uint32_t pool_end = min(a.n, pool + share);
    while (true) {
        uint64_t idle = __ballot(!busy);
        if ((uint32_t)__popcll(idle) >= a.refill_idle) {
            while (idle && pool < pool_end) {
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                const uint32_t take = min((uint32_t)__popcll(idle), pool_end - pool);
                if (!busy && rank < take) {
                    ray = pool + rank;
                    const bool m = !a.mask || ((a.mask_size == 1) ? (a.mask[0] != 0) : (a.mask[ray] != 0));
                    if (m) {
                        const V3 o = v3(a.ox[ray], a.oy[ray], a.oz[ray]);
                        const V3 d = v3(a.dx[ray], a.dy[ray], a.dz[ray]);
                        const float tmin = a.tmin ? a.tmin[ray] : kRayTmin, tmax = a.tmax ? a.tmax[ray] : kRayTmax;
                        tr.init(a.sc, o, d, tmin, tmax, a.closest == 0, L);
                        busy = !tr.finished();
                        if (!busy) {  // empty triangle set: the spheres alone
                            TraceHit h = tr.hit(a.sc, L);
                            if (a.sc.nsph) trace_spheres(a.sc, o, d, tmin, a.closest == 0, h);
                            if (h.slot == -1) {
                                a.tri_id[ray] = -1;
                            } else {
                                a.tri_id[ray] = h.slot;
                                a.t[ray] = h.t;
                                a.u[ray] = h.u;
                                a.v[ray] = h.v;
                            }
                        }
                    }
                }
                pool += take;
                idle = __ballot(!busy);
            }
        }
        if (!__ballot(busy)) break;
        if (busy && tr.step(a.sc, L, st)) {
            TraceHit h = tr.hit(a.sc, L);
            if (a.sc.nsph) {
                const float tmin = a.tmin ? a.tmin[ray] : kRayTmin;
                trace_spheres(a.sc, v3(a.ox[ray], a.oy[ray], a.oz[ray]), v3(a.dx[ray], a.dy[ray], a.dz[ray]), tmin,
                              a.closest == 0, h);
            }
            if (h.slot == -1) {
                a.tri_id[ray] = -1;
            } else {
                a.tri_id[ray] = h.slot >= 0 ? (int32_t)h.id : h.slot;
                a.t[ray] = h.t;
                a.u[ray] = h.u;
                a.v[ray] = h.v;
            }
            busy = false;
        }
    }
}

// ------------------------------------------------------------ camera gen
__device__ __forceinline__ void camera_ray(const Camera& cam, Pcg32& rng, uint32_t order, uint32_t x, uint32_t y,
                                           V3& o, V3& d) {
    float xi_x, xi_y;
    draw2(rng, order, xi_x, xi_y);              // main.cpp:395
    o = camera_sample_pos(cam, xi_x, xi_y);
    draw2(rng, order, xi_x, xi_y);              // main.cpp:396
    d = camera_sample_dir(cam, x, y, o, xi_x, xi_y);
}

// A path's planes (PathQueue): the ray always, throughput / radiance as the mode needs.
template <int kMode, bool kNt = false>
__device__ __forceinline__ void store_path(const PathQueue& q, uint32_t j, V3 o, V3 d, uint32_t pix, uint32_t meta,
                                           float tr, float tg, float tb, float lr, float lg, float lb) {
    stq<kNt>(q.q1 + j, make_float4(o.x, o.y, o.z, u2f(meta)));
    stq<kNt>(q.q2 + j, make_float4(d.x, d.y, d.z, u2f(pix)));
    if (kMode >= kModeAlbedo) stq<kNt>(q.q0 + j, make_float4(tr, tg, tb, kMode == kModeEmit ? lr : 0.0f));
    if (kMode == kModeEmit) stq2<kNt>(q.rad + j, make_float2(lg, lb));
}

// PCG32 of global pixel gpix (main.cpp:376) advanced past the draws a path
// has consumed: the sample's jump (s * (4 + 2D)) then the cast's (4 camera
// draws + 2 per earlier cast, main.cpp:395,396,413).
// (js: the seeded sample map of pcg_seeded_jump, capi.cpp ensure_jumps)
__device__ __forceinline__ Pcg32 path_rng(uint32_t gpix, const PcgJump& js, const PcgJump& jc) {
    Pcg32 r = pcg_start(js, (uint64_t)gpix);
    r.state = pcg_apply(jc, r.state, r.inc);
    return r;
}

// Refill: start work items [cursor, cursor + total) in queue slots
// [surv, surv + total).  Work item w is sample w / P of tile pixel w % P, so a
// refill hands consecutive lanes consecutive pixels of one sample (coherent
// camera rays).  RNG: the pixel's PCG32 stream (main.cpp:376) advanced to the
// sample's first draw, s * (4 + 2D) draws (main.cpp:395,396,413 per sample).
// Refill grid: at most kRefillMaxBlocks blocks striding over the new paths
// instead of one thread per queue slot the host may have to fill (the host
// sizes it before it knows how many paths ended): config 1 +0.9 %, config 2
// +1.8 % (profiles/r03_tune/knob_sweep.log).
#ifndef SPT_REFILL_STRIDE
#define SPT_REFILL_STRIDE 1
#endif
#ifndef SPT_REFILL_MAX_BLOCKS
#define SPT_REFILL_MAX_BLOCKS 4096
#endif
constexpr uint32_t kRefillMaxBlocks = SPT_REFILL_MAX_BLOCKS;
template <int kMode, bool kNt = false>
__global__ __launch_bounds__(256) void refill_kernel(RefillArgs a) {
    uint32_t surv = 0;
    if (a.surv_shards)
        for (uint32_t j = 0; j < kShards; j++) surv += a.surv_shards[j * kShardStride];
    else
        surv = *a.surv;
    const uint64_t cur = a.cursor_in ? *a.cursor_in : a.cursor_init;
    const uint64_t avail = a.work_end > cur ? a.work_end - cur : 0;
    const uint32_t room = a.capacity - surv;
    const uint32_t total = (uint32_t)(avail < room ? avail : room);
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i == 0) {
        *a.cursor_out = cur + total;
        *a.qn_out = surv + total;
        *a.isect_next = 0;
        if (a.surv_clear) *a.surv_clear = 0;
        if (a.xcd_next)
            for (uint32_t x = 0; x < 8u; x++) a.xcd_next[x * 32u] = 0;
        if (cur < a.work_end && cur + total >= a.work_end) *a.exhausted = a.iter_tag;
        if (a.casts_in) {  // the shade before: its queue count and its survivors
            const uint32_t casts = *a.casts_in;
            if (casts) atomicAdd(&a.stats[0], (unsigned long long)casts);
            if (surv) atomicAdd(&a.stats[1], (unsigned long long)surv);
        }
        if (total) atomicAdd(&a.stats[2], (unsigned long long)total);
    }
    if (a.book_only) return;
#if SPT_REFILL_STRIDE
    for (uint32_t j = i; j < total; j += gridDim.x * 256u) {
#else
    if (i >= total) return;
    {
        const uint32_t j = i;
#endif
        uint32_t s, q, lx, ly;
        work_item((uint32_t)(cur + j - (uint64_t)a.chunk_s0 * a.P), a.chunk_s0, a.chunk_ns, a.P, a.work_order != 0, s,
                  q);
        work_pixel(q, a.W, a.P, a.pixel_block, lx, ly);
        const uint32_t p = ly * a.W + lx;
        const uint32_t gy = tile_global_row(ly, a.tile_index, a.tile_count, a.rows_per_group);
        const uint32_t gpix = gy * a.W + lx;                    // main.cpp:379-382
        Pcg32 rng = pcg_start(a.sample_jump[s], (uint64_t)gpix);  // main.cpp:376, then the sample's draws
        V3 o, d;
        camera_ray(a.cam, rng, a.rng_order, lx, gy, o, d);
        store_path<kMode, kNt>(a.q, surv + j, o, d, p, s << kMetaDepthBits, 1.0f, 1.0f, 1.0f, 0.0f, 0.0f, 0.0f);  // main.cpp:391
    }
}

// ----------------------------------------------------------------- shade
#ifndef SPT_OCT_GROUP
#define SPT_OCT_GROUP 0
#endif
// main.cpp:404-425 for one cast of every queued path.  A path that ends
// writes its contribution once per (sample, pixel): unit mode one byte
// (escaped or not: the sky term is added in sample order by the resolve),
// otherwise its gathered radiance (throughput x sky radiance on escape, plus
// emitted radiance with emitters) to its film slot (film_slot / film_rgb).  Survivors are
// compacted into the out queue with a wave ballot + mbcnt rank and one
// atomicAdd per block.  Phase 1 decides which paths survive (miss, last cast,
// albedo, roulette) from the hit and the material word alone, so the block's
// queue atomic is issued before phase 2 (new ray: RNG derivation and draw,
// interpolated normal, Frame3, cosine sample) and its latency hides behind
// that work.
// kSpt: the scene has smallpt spheres or mirror / glass materials (a separate
// instance, so plain scenes keep the leaner register budget).
//
// shade_block is the whole of it for one block of kBlock threads, each holding
// one path or none (valid): the path's queue entry, hit record and (albedo /
// emitter modes) throughput and radiance come from Src — the queue and the
// hit records in shade_kernel, registers in camera_cast_kernel (the first
// cast, traced in the same launch) — so both run the same arithmetic and
// compaction.  Every thread of the block must call it (barriers, ballots).
template <bool kNt>
struct QueueSrc {  // shade_kernel: queue slot i of a.in and its hit record
    const ShadeArgs& a;
    uint32_t i;
    __device__ __forceinline__ float4 q1() const { return ldq<kNt>(a.in.q1 + i); }
    __device__ __forceinline__ float4 q2() const { return ldq<kNt>(a.in.q2 + i); }
    __device__ __forceinline__ float4 hit() const { return ldq<kNt>(a.hits + i); }
    __device__ __forceinline__ float4 q0() const { return ldq<kNt>(a.in.q0 + i); }
    __device__ __forceinline__ float2 rad() const { return ldq2<kNt>(a.in.rad + i); }
};
template <int kMode, bool kSpt, bool kNt, uint32_t kBlock, typename Src>
__device__ __forceinline__ void shade_block(const ShadeArgs& a, bool valid, const Src& src) {
    __shared__ uint32_t s_wave_cnt[kBlock / 64];
    __shared__ uint32_t s_wave_off[kBlock / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;

    // ---- phase 1: survive or terminate (the bounce inputs load alongside)
    bool emit = false;
    uint32_t pix = 0, meta = 0, kind = kMatDiffuse;
    int32_t slot = -1;
    // The bounce inputs (hit, m0-m2, o, d, gpix) are read only where they were
    // set (phase 2 runs for survivors, emit); left uninitialised the compiler
    // materialises no zeros for them at every join (~45 VALU moves per
    // thread, issue slots the co-running isect grids want).  With spheres a
    // sphere hit keeps m0-m2 at zero on purpose (scatter ignores them).
    uint32_t gpix;
    float4 hit, m0, m1, m2;
    V3 o, d;
    if constexpr (kSpt) {
        gpix = 0;
        hit = m0 = m1 = m2 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        o = d = v3(0, 0, 0);
    }
    float tr = 1.0f, tg = 1.0f, tb = 1.0f, lr = 0.0f, lg = 0.0f, lb = 0.0f;
    if (valid) {
        const float4 q1 = src.q1(), q2 = src.q2();
        meta = f2u(q1.w);
        pix = f2u(q2.w);
        const uint32_t depth = meta & ((1u << kMetaDepthBits) - 1u);
        const uint32_t sample = meta >> kMetaDepthBits;
        hit = src.hit();
        slot = (int32_t)f2u(hit.x);
        if (kSpt && a.sc.nsph) {
            // smallpt's analytic spheres after the triangle BVH (the isect kernel
            // traces triangles only); a miss record carries t = tmax
            TraceHit h;
            h.slot = slot; h.id = 0u; h.t = hit.y; h.u = hit.z; h.v = hit.w;
            trace_spheres(a.sc, v3(q1.x, q1.y, q1.z), v3(q2.x, q2.y, q2.z), kRayTmin,
                          depth + 1 >= a.max_depth && !a.sc.emission, h);
            slot = h.slot;
            hit = make_float4(u2f((uint32_t)slot), h.t, h.u, h.v);
        }
        if (kMode >= kModeAlbedo) {
            const float4 q0 = src.q0();
            tr = q0.x; tg = q0.y; tb = q0.z;
            if (kMode == kModeEmit) lr = q0.w;
        }
        if (kMode == kModeEmit) { const float2 l = src.rad(); lg = l.x; lb = l.y; }
        bool term = true, escaped = false;
        if (slot == -1) {
            // miss: film += select(!hit && active, contrib, 0)  (main.cpp:407)
            escaped = true;
            if (kMode != kModeUnit) {
                lr = lr + tr * a.env_r;
                lg = lg + tg * a.env_g;
                lb = lb + tb * a.env_b;
            }
        } else {
            const bool bounce = depth + 1 < a.max_depth;
            const bool sph = kSpt && slot < -1;
            if (!sph && (kMode == kModeEmit || bounce)) m0 = a.sc.snrm[(size_t)slot * 3];  // n0 + material id
            if (bounce) {
                if (!sph) {
                    m1 = a.sc.snrm[(size_t)slot * 3 + 1];
                    m2 = a.sc.snrm[(size_t)slot * 3 + 2];
                }
                o = v3(q1.x, q1.y, q1.z);
                d = v3(q2.x, q2.y, q2.z);
                gpix = tile_global_pixel(pix, a.W, a.tile_index, a.tile_count, a.rows_per_group);
            }
            if (kMode == kModeUnit) {
                term = !bounce;  // albedo 1: the throughput stays 1, roulette never fires
            } else {
                uint32_t mat = 0;  // (m0 was loaded iff emitters or a bounce need it)
                if (sph) mat = a.sc.sph_mat ? (uint32_t)a.sc.sph_mat[-2 - slot] : 0u;
                else if (kMode == kModeEmit || bounce) mat = f2u(m0.w);
                if (kSpt) kind = material_kind(a.sc, mat);
                if (kMode == kModeEmit && mat < a.sc.nemit) {
                    // emitted radiance at the hit (smallpt obj.e; not in the reference)
                    lr = lr + tr * a.sc.emission[mat * 3];
                    lg = lg + tg * a.sc.emission[mat * 3 + 1];
                    lb = lb + tb * a.sc.emission[mat * 3 + 2];
                }
                if (bounce) {
                    const V3 rf = reflectance(a.sc, mat, (uint32_t)slot, hit.z, hit.w);  // main.cpp:418
                    tr = tr * rf.x;                                  // main.cpp:422
                    tg = tg * rf.y;
                    tb = tb * rf.z;
                    term = false;
                    if (depth + 1 >= a.rr_start) {
                        const float q = fmaxf(tr, fmaxf(tg, tb));
                        if (q < 1.0f) {
                            if (rr_uniform(gpix, sample, depth) >= q) {
                                term = true;
                            } else {
                                tr = tr / q; tg = tg / q; tb = tb / q;
                            }
                        }
                    }
                }
            }
            // else: hit on the last cast — the path ends (no sky contribution).
        }
        emit = !term;
        if (term) {
            if (kMode == kModeUnit) {
                a.sflag[film_slot(sample - a.sample0, pix, a.P, a.chunk_ns, a.work_order)] = escaped ? 1 : 0;
            } else {
                size_t cs;
                float* f = film_rgb(a.sfilm, sample - a.sample0, pix, a.P, a.chunk_ns, a.work_order, cs);
                f[0] = lr;
                f[cs] = lg;
                f[2 * cs] = lb;
            }
        }
    }

    // ---- compaction: wave ballot + mbcnt rank, one queue atomic per block.
    // (Casts and continuations are the queue counts: the refill that follows
    // adds them to the stats, so no per-block stats atomics contend here.)
    const uint64_t ball = __ballot(emit);
    const uint32_t rank =
        __builtin_amdgcn_mbcnt_hi((uint32_t)(ball >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ball, 0u));
    if (lane == 0) s_wave_cnt[wave] = (uint32_t)__popcll(ball);
    __syncthreads();
    uint32_t base = 0, total = 0;
    if (tid == 0) {
        for (uint32_t w = 0; w < kBlock / 64; w++) total += s_wave_cnt[w];
        // returns during phase 2.  The address goes through an opaque VGPR
        // zero: for a uniform address the compiler's atomic optimizer wraps
        // the add in a wave scan whose readfirstlane waits for the return
        // right here, serialising the atomic's latency with phase 2.
        uint32_t zero;
        asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
        if (a.shard_items) {  // the block's shard: its XCD's counter and segment (shard_base)
            const uint32_t j = blockIdx.x % kShards;
            if (total) base = atomicAdd(a.count_out + j * kShardStride + zero, total);
            base += shard_base(j, a.shard_items, kBlock);
        } else if (total) {
            base = atomicAdd(a.count_out + zero, total);
        }
    }

    // ---- phase 2: the bounce ray of every survivor
    V3 no, nd;
    if (emit) {
        const uint32_t depth = meta & ((1u << kMetaDepthBits) - 1u);
        const uint32_t sample = meta >> kMetaDepthBits;
        Pcg32 rng = path_rng(gpix, a.sample_jump[sample], a.cast_jump[depth]);
        const float t = hit.y, u = hit.z, v = hit.w;
        float xi_x, xi_y;
        draw2(rng, a.rng_order, xi_x, xi_y);                   // main.cpp:413
        const float w = (1.0f - u) - v;                          // add_math.h:6
        const V3 sn = v3((w * m0.x + u * m1.x) + v * m2.x,      // optix_backend.h:483-484
                         (w * m0.y + u * m1.y) + v * m2.y,
                         (w * m0.z + u * m1.z) + v * m2.z);
        no = v3(o.x + t * d.x, o.y + t * d.y, o.z + t * d.z);   // optix_backend.h:469, main.cpp:423
        if (!kSpt) {
            const Frame fr = frame_from_normal(sn);              // main.cpp:414
            nd = to_world(fr, cosine_hemisphere(xi_x, xi_y));    // main.cpp:418-419, 424
        } else {
            // Lambert on triangles as above; spheres / mirror / glass as smallpt
            float wgt;
            nd = scatter(a.sc, kind, slot, d, no, sn, xi_x, xi_y, wgt);
            tr = tr * wgt; tg = tg * wgt; tb = tb * wgt;
        }
    }
    if (tid == 0) {
        uint32_t off = base;
        for (uint32_t w = 0; w < kBlock / 64; w++) {
            s_wave_off[w] = off;
            off += s_wave_cnt[w];
        }
    }
    __syncthreads();
    uint32_t slot_in_wave = rank;
#if SPT_OCT_GROUP
    // a wave's survivors in the order of their bounce direction's octant (then
    // lane order): the drain's lanes take consecutive queue entries, so rays
    // refilled together start out heading the same way (order only: the same
    // paths, the same bits)
    {
        const uint32_t oct = emit ? (nd.x < 0.0f ? 1u : 0u) | (nd.y < 0.0f ? 2u : 0u) | (nd.z < 0.0f ? 4u : 0u) : 8u;
        uint32_t before = 0, mine = 0;
#pragma unroll
        for (uint32_t o = 0; o < 8u; o++) {
            const uint64_t b = __ballot(oct == o);
            const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
            if (oct == o) mine = before + r;
            before += (uint32_t)__popcll(b);
        }
        slot_in_wave = mine;
    }
#endif
    if (emit)
        store_path<kMode, kNt>(a.out, s_wave_off[wave] + slot_in_wave, no, nd, pix, meta + 1u, tr, tg, tb, lr, lg, lb);
}

template <int kMode, bool kSpt, bool kNt = false>
__global__ __launch_bounds__(kShadeBlock) void shade_kernel(ShadeArgs a) {
    const uint32_t n = *a.count_in;
    if (n < a.drain_below) return;  // the drain launch takes this queue (launch_drain)
    // the grid may be sized from a stale (larger) count: remap only the
    // blocks that hold queued paths, so every XCD gets its eighth of them
    const uint32_t nreal = min(gridDim.x, (n + kShadeBlock - 1) / kShadeBlock);
    const uint32_t i =
        (a.xcd_remap && blockIdx.x < nreal ? xcd_block(blockIdx.x, nreal) : blockIdx.x) * kShadeBlock + threadIdx.x;
    shade_block<kMode, kSpt, kNt, kShadeBlock>(a, i < n, QueueSrc<kNt>{a, i});
}

// ----------------------------------------------------------- camera cast
#ifndef SPT_CAM_RECOMPUTE
#define SPT_CAM_RECOMPUTE 0
#endif
#ifndef SPT_CAM_WAVES
#define SPT_CAM_WAVES 0  // 0: the tracer's (8 for the 64-B node)
#endif
// A fitting job's first cast in one launch (spt_config.camera_cast): one lane
// per work item of the sub-wavefront — its camera ray (refill_kernel's
// arithmetic, start_path), its trace in lockstep with the wave's other lanes
// (isect_lockstep_kernel: a wave holds one pixel's 64 samples in pixel-major
// order, coherent rays), then its shade (shade_block: film write, or the
// bounce ray compacted into the drain's queue).  The camera rays and their
// hit records never touch memory: the refill's 32-B queue write, the isect's
// 32-B read and 16-B hit write and the shade's 48-B read per path are gone,
// and so are two launches per render.  Same arithmetic, same bits.
struct CamSrc {  // the path in registers: its first cast, just traced
    V3 o, d;
    uint32_t pix, meta;
    TraceHit h;
    __device__ __forceinline__ float4 q1() const { return make_float4(o.x, o.y, o.z, u2f(meta)); }
    __device__ __forceinline__ float4 q2() const { return make_float4(d.x, d.y, d.z, u2f(pix)); }
    __device__ __forceinline__ float4 hit() const { return make_float4(u2f((uint32_t)h.slot), h.t, h.u, h.v); }
    __device__ __forceinline__ float4 q0() const { return make_float4(1.0f, 1.0f, 1.0f, 0.0f); }  // main.cpp:391
    __device__ __forceinline__ float2 rad() const { return make_float2(0.0f, 0.0f); }
};
template <typename Tr, int kMode, bool kSpt, bool kNt>
__global__ __launch_bounds__(kIsectBlock)
__attribute__((amdgpu_waves_per_eu(SPT_CAM_WAVES ? SPT_CAM_WAVES : Tr::kMinWaves, 8)))
void camera_cast_kernel(CameraCastArgs a) {
    extern __shared__ uint32_t lds_stack[];
    const Lds L = block_lds(lds_stack);
    const uint32_t i = blockIdx.x * kIsectBlock + threadIdx.x;
    const bool valid = i < a.n;
    CamSrc c;
    c.o = c.d = v3(0.0f, 0.0f, 0.0f);
    c.pix = c.meta = 0;
    c.h.slot = -1;
    c.h.id = 0xffffffffu;
    c.h.t = kRayTmax;
    c.h.u = c.h.v = 0.0f;
    if (valid) {
        start_path(a.r, a.r.cursor_init + i, c.o, c.d, c.pix, c.meta);
        NoStats st;
        Tr tr;
        // any-hit for the last cast unless emitters need the surface (isect_queue_kernel)
        tr.init(a.s.sc, c.o, c.d, kRayTmin, kRayTmax, a.s.max_depth <= 1 && !a.s.sc.emission, L);
        if (!tr.finished())
            while (!tr.step(a.s.sc, L, st)) {
            }
        c.h = tr.hit(a.s.sc, L);
#if SPT_CAM_RECOMPUTE
        // the ray again (the same arithmetic, the same bits) rather than keeping
        // its direction, pixel and sample live across the traversal: the
        // traversal keeps its 64 VGPRs (8 waves) with no spill.  The opaque
        // copy of the work item stops the compiler from reusing the first one.
        uint32_t w = i;
        asm volatile("" : "+v"(w));
        start_path(a.r, a.r.cursor_init + w, c.o, c.d, c.pix, c.meta);
#endif
    }
    shade_block<kMode, kSpt, kNt, kIsectBlock>(a.s, valid, c);
}

// ------------------------------------------------------------ fused render
// The whole of main.cpp:385-426 in one persistent launch per sample chunk:
// each lane owns one path from its camera ray to termination.  Lanes whose
// ray has finished wait (as "pending") until at least refill_idle lanes of
// the wave are not tracing; then the wave shades all pending lanes at once
// (same arithmetic as shade_kernel) and starts new paths (same as
// refill_kernel) in the lanes that became free.  Path state never leaves the
// registers, so there are no queues, compaction or per-bounce launches.  The
// per-(sample, pixel) film writes are the same, so the image is bit-identical.
//
// kDrain: the wavefront's drain (launch_drain).  The same lane loop, but a
// free lane takes the next path of a wavefront queue — its ray, pixel,
// sample and cast as the shade would read them, its PCG32 state re-derived at
// its cast's bounce draw (path_rng) — instead of a new camera path, and
// continues it to termination in registers.  Once a sub-wavefront's queue
// falls below drain_below the per-cast launches (each ending in the latency
// tail of its slowest ray) stop and one launch finishes every path.  Same
// arithmetic, same film writes, so the same bits as the queue kernels.
template <typename Tr, int kMode, bool kDrain = false, bool kNt = false>
__global__ __launch_bounds__(kIsectBlock)
__attribute__((amdgpu_waves_per_eu(kDrain && kMode == kModeUnit ? (kNt ? SPT_DRAIN_WAVES_NT : SPT_DRAIN_WAVES)
                                   : kDrain ? SPT_DRAIN_WAVES_RGB : SPT_FUSED_WAVES, 8)))
void render_fused_kernel(FusedArgs a) {
    constexpr bool kEmit = kMode == kModeEmit;
    constexpr bool kMergedInit = SPT_MERGED_INIT != 0;
#if SPT_WAVE_LOG
    const unsigned long long wl_t0 = (unsigned long long)wall_clock64();
#endif
    extern __shared__ uint32_t lds_stack[];
    const Lds L = block_lds(lds_stack);
    uint32_t n = a.count;
    if constexpr (kDrain) {
        if (a.seg_count) {  // a sharded queue: the sum of its segments
            n = 0;
            for (uint32_t j = 0; j < kShards; j++) n += a.seg_count[j * kShardStride];
            n = wave_uniform(n);
        } else {
            n = wave_uniform(*a.qcount);
        }
        if (n >= a.drain_below) return;  // the isect and shade launches take this queue
        if (blockIdx.x == 0 && threadIdx.x == 0 && n) {
            atomicAdd(a.drained, (unsigned long long)n);
            // a forced drain ends its sub-wavefront: the queued paths' first casts
            // here go to the stats directly (no bookkeeping refill follows)
            if (a.count_queue) atomicAdd(&a.stats[0], (unsigned long long)n);
        }
    }
    NoStats st;
    Tr tr;
    V3 dir = v3(0, 0, 0);
    // A lane carries no PCG32 state: the shade re-derives it at the cast's
    // bounce draw from (pixel, sample, cast) as shade_kernel does (path_rng),
    // and the work counters are wave-uniform (ballot counts), so the path
    // state the traversal loop keeps live is the ray, pixel, sample, cast and
    // throughput only (VGPRs: occupancy).
    uint32_t pix = 0, meta = 0;  // tile pixel; sample << 8 | cast (as a queue path's q1.w)
    float thr = 1.0f, thg = 1.0f, thb = 1.0f, lr = 0.0f, lg = 0.0f, lb = 0.0f;
    // albedo / emitter modes: a lane's throughput and gathered radiance wait in
    // LDS while its ray traces (two float4 per lane after the tracer's records),
    // so the traversal loop does not hold them in VGPRs
    constexpr bool kPark = kMode != kModeUnit && SPT_PARK_PATH;
    float4* const park = kPark ? (float4*)((char*)L.base + a.sc.stack_depth * kIsectBlock * 4u + Tr::kExtraLds) +
                                     2u * threadIdx.x
                               : nullptr;
    bool busy = false, pending = false;
    uint32_t casts = 0, conts = 0, starts = 0;  // wave-uniform
    // wave-uniform work pool: static share, then dynamic chunks.  XCD-aware
    // (a.xcd_next): blocks are dealt round-robin over the 8 XCDs (block b on
    // XCD b mod 8, MI355X_MICROARCH.md), so the waves of one XCD take adjacent
    // static shares, and dynamic chunks first from their XCD's eighth of the
    // rest (its own counter), then from the other XCDs' (stealing): each
    // XCD's L2 then serves a contiguous range of the work — a band of the
    // tile in pixel-major order — instead of chunks from all over it.
    const uint32_t nwaves = gridDim.x * (kIsectBlock / 64);
    const uint32_t blk = a.xcd_next ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint32_t wave_id = wave_uniform(blk * (kIsectBlock / 64) + (threadIdx.x >> 6));
    // (a sharded queue's segments are taken only through the per-XCD pools)
    const uint32_t share =
        kDrain && a.seg_count ? 0u : (uint32_t)(((uint64_t)n * a.static_share_q8 / 256) / nwaves);
    const uint32_t dyn_base = share * nwaves;
    uint32_t pool = wave_id * share, pool_end = pool + share;
    bool drained = false;
    uint32_t xcd = wave_uniform(blockIdx.x & 7u), xcd_tries = 0;
#if SPT_WAVE_LOG
    unsigned long long ph[kPhaseWords] = {};
#endif
    while (true) {
        if ((uint32_t)__popcll(__ballot(!busy)) >= a.refill_idle) {
#if SPT_WAVE_LOG
            const unsigned long long ph_t0 = __builtin_readcyclecounter();
            ph[3]++;
            ph[5] += (uint32_t)__popcll(__ballot(pending));
#endif
            // ---- shade every pending lane (shade_kernel, main.cpp:404-425)
            casts += (uint32_t)__popcll(__ballot(pending));
            bool cont = false;
            bool need_init = false;  // kMergedInit: a new ray in tr.o / dir to set up after the refill
            if (pending) {
                pending = false;
                bool term = true;
                if constexpr (kPark) {
                    const float4 p0 = park[0], p1 = park[1];
                    thr = p0.x; thg = p0.y; thb = p0.z; lr = p0.w; lg = p1.x; lb = p1.y;
                }
                const uint32_t depth = meta & ((1u << kMetaDepthBits) - 1u), sample = meta >> kMetaDepthBits;
                TraceHit hh = tr.hit(a.sc, L);
                if (kMode != kModeUnit && a.sc.nsph)  // smallpt's spheres after the BVH
                    trace_spheres(a.sc, tr.o, dir, kRayTmin, depth + 1 >= a.max_depth && !kEmit, hh);
                const int32_t slot = hh.slot;
                const bool sph = kMode != kModeUnit && slot < -1;
                if (slot == -1) {
                    if (kMode != kModeUnit) {
                        lr = lr + thr * a.env_r;                   // main.cpp:407
                        lg = lg + thg * a.env_g;
                        lb = lb + thb * a.env_b;
                    }
                } else {
                    const float4 m0 = sph ? make_float4(0.0f, 0.0f, 0.0f, 0.0f) : a.sc.snrm[(size_t)slot * 3];
                    uint32_t mat = sph ? (a.sc.sph_mat ? (uint32_t)a.sc.sph_mat[-2 - slot] : 0u) : f2u(m0.w);
                    if (kEmit && mat < a.sc.nemit) {
                        lr = lr + thr * a.sc.emission[mat * 3];
                        lg = lg + thg * a.sc.emission[mat * 3 + 1];
                        lb = lb + thb * a.sc.emission[mat * 3 + 2];
                    }
                    if (depth + 1 < a.max_depth) {
                        // the global pixel (main.cpp:379-382), for the roulette draw and the PCG32 stream
                        const uint32_t gpix =
                            tile_global_pixel(pix, a.W, a.tile_index, a.tile_count, a.rows_per_group);
                        if (kMode != kModeUnit) {
                            const V3 rf = reflectance(a.sc, mat, (uint32_t)slot, hh.u, hh.v);  // main.cpp:418
                            thr = thr * rf.x;                        // main.cpp:422
                            thg = thg * rf.y;
                            thb = thb * rf.z;
                        }
                        term = false;
                        if (kMode != kModeUnit && depth + 1 >= a.rr_start) {
                            const float q = fmaxf(thr, fmaxf(thg, thb));
                            if (q < 1.0f) {
                                if (rr_uniform(gpix, sample, depth) >= q) {
                                    term = true;
                                } else {
                                    thr = thr / q; thg = thg / q; thb = thb / q;
                                }
                            }
                        }
                        if (!term) {
                            const float4 zero = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                            const float4 m1 = sph ? zero : a.sc.snrm[(size_t)slot * 3 + 1];
                            const float4 m2 = sph ? zero : a.sc.snrm[(size_t)slot * 3 + 2];
                            // at this cast's bounce draw, 4 + 2 depth past the sample's first
                            Pcg32 rng = path_rng(gpix, a.sample_jump[sample], a.cast_jump[depth]);
                            float xi_x, xi_y;
                            draw2(rng, a.rng_order, xi_x, xi_y);   // main.cpp:413
                            const float t = hh.t, u = hh.u, v = hh.v;
                            const float w = (1.0f - u) - v;          // add_math.h:6
                            const V3 sn = v3((w * m0.x + u * m1.x) + v * m2.x,  // optix_backend.h:483-484
                                             (w * m0.y + u * m1.y) + v * m2.y,
                                             (w * m0.z + u * m1.z) + v * m2.z);
                            const V3 o = tr.o;
                            const V3 hp = v3(o.x + t * dir.x, o.y + t * dir.y, o.z + t * dir.z);  // :469
                            if (kMode == kModeUnit) {
                                const Frame fr = frame_from_normal(sn);  // main.cpp:414
                                dir = to_world(fr, cosine_hemisphere(xi_x, xi_y));  // main.cpp:418-419, 424
                            } else {  // Lambert on triangles as above; spheres / mirror / glass as smallpt
                                float wgt;
                                dir = scatter(a.sc, material_kind(a.sc, mat), slot, dir, hp, sn, xi_x, xi_y, wgt);
                                thr = thr * wgt; thg = thg * wgt; thb = thb * wgt;
                            }
                            meta++;  // the next cast
                            if constexpr (kPark) {
                                park[0] = make_float4(thr, thg, thb, lr);
                                park[1] = make_float4(lg, lb, 0.0f, 0.0f);
                            }
                            if constexpr (kMergedInit) {
                                tr.o = hp;  // traced from here: set up below with the refilled lanes
                                need_init = true;
                            } else {
                                tr.init(a.sc, hp, dir, kRayTmin, kRayTmax, depth + 2 >= a.max_depth && !kEmit, L);
                            }
                            busy = true;
                            cont = true;
                        }
                    }
                }
                if (term) {
                    if (kMode == kModeUnit) {
                        a.sflag[film_slot(sample - a.sample0, pix, a.P, a.pm_ns, a.pm_ns != 0)] = slot == -1 ? 1 : 0;
                    } else {
                        size_t cs;
                        float* f = film_rgb(a.sfilm, sample - a.sample0, pix, a.P, a.pm_ns, a.pm_ns != 0, cs);
                        f[0] = lr;
                        f[cs] = lg;
                        f[2 * cs] = lb;
                    }
                }
            }
            conts += (uint32_t)__popcll(__ballot(cont));
#if SPT_WAVE_LOG
            const unsigned long long ph_t2 = __builtin_readcyclecounter();
#endif
            // ---- new camera paths in free lanes (refill_kernel)
            uint64_t idle = __ballot(!busy && !pending);
            while (idle && !(drained && pool == pool_end)) {
                if (pool == pool_end && a.xcd_next) {
                    // this XCD's eighth of [dyn_base, n), then the next XCD's
                    while (xcd_tries < 8u) {
                        uint32_t lo, hi;
                        if (kDrain && a.seg_count) {  // this XCD's segment of a sharded queue
                            lo = shard_base(xcd, a.seg_items, a.seg_block);
                            hi = lo + wave_uniform(a.seg_count[xcd * kShardStride]);
                        } else {
                            lo = dyn_base + (uint32_t)((uint64_t)(n - dyn_base) * xcd / 8u);
                            hi = dyn_base + (uint32_t)((uint64_t)(n - dyn_base) * (xcd + 1u) / 8u);
                        }
                        uint32_t got = 0;
                        if ((threadIdx.x & 63u) == 0) got = atomicAdd(a.xcd_next + xcd * 32u, a.chunk);
                        got = wave_uniform((uint32_t)__shfl((int)got, 0));
                        if (got < hi - lo) {
                            pool = lo + got;
                            pool_end = min(pool + a.chunk, hi);
                            break;
                        }
                        xcd = (xcd + 1u) & 7u;
                        xcd_tries++;
                    }
                    if (xcd_tries >= 8u) { drained = true; break; }
                } else if (pool == pool_end) {
                    uint32_t base = 0;
                    if ((threadIdx.x & 63u) == 0) base = atomicAdd(a.next, a.chunk);
                    base = dyn_base + wave_uniform((uint32_t)__shfl((int)base, 0));
                    if (base >= n) { drained = true; break; }
                    pool = base;
                    pool_end = min(base + a.chunk, n);
                }
                const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                const uint32_t take = min((uint32_t)__popcll(idle), pool_end - pool);
                if (kDrain && !busy && !pending && rank < take) {
                    // the next queued path (shade_kernel's reads), continued here
                    const uint32_t j = a.perm ? a.perm[pool + rank] : pool + rank;
                    const float4 q1 = ldq<kNt>(a.q.q1 + j), q2 = ldq<kNt>(a.q.q2 + j);
                    meta = f2u(q1.w);
                    const uint32_t depth = meta & ((1u << kMetaDepthBits) - 1u);
                    pix = f2u(q2.w);
                    dir = v3(q2.x, q2.y, q2.z);
                    thr = thg = thb = 1.0f;
                    lr = lg = lb = 0.0f;
                    if (kMode >= kModeAlbedo) {
                        const float4 q0 = ldq<kNt>(a.q.q0 + j);
                        thr = q0.x; thg = q0.y; thb = q0.z;
                        if (kEmit) lr = q0.w;
                    }
                    if (kEmit) {
                        const float2 l = ldq2<kNt>(a.q.rad + j);
                        lg = l.x; lb = l.y;
                    }
                    if constexpr (kPark) {
                        park[0] = make_float4(thr, thg, thb, lr);
                        park[1] = make_float4(lg, lb, 0.0f, 0.0f);
                    }
                    busy = true;
                    if constexpr (kMergedInit) {
                        tr.o = v3(q1.x, q1.y, q1.z);
                        need_init = true;
                    } else {
                        tr.init(a.sc, v3(q1.x, q1.y, q1.z), dir, kRayTmin, kRayTmax, depth + 1 >= a.max_depth && !kEmit,
                                L);
                        if (tr.finished()) {  // empty scene: a miss
                            busy = false;
                            pending = true;
                        }
                    }
                } else if (!kDrain && !busy && !pending && rank < take) {
                    uint32_t sample;
                    work_item(pool + rank, a.sample0, a.pm_ns, a.P, a.pm_ns != 0, sample, pix);  // work0 = sample0 * P
                    const uint32_t lx = pix % a.W, ly = pix / a.W;  // scanline (pixel blocks: refill_kernel only)
                    const uint32_t gy = tile_global_row(ly, a.tile_index, a.tile_count, a.rows_per_group);
                    const uint32_t gpix = gy * a.W + lx;           // main.cpp:379-382
                    Pcg32 rng = pcg_start(a.sample_jump[sample], (uint64_t)gpix);  // main.cpp:376 + the sample's draws
                    V3 o;
                    camera_ray(a.cam, rng, a.rng_order, lx, gy, o, dir);
                    meta = sample << kMetaDepthBits;  // cast 0
                    thr = thg = thb = 1.0f;                        // main.cpp:391
                    lr = lg = lb = 0.0f;
                    if constexpr (kPark) {
                        park[0] = make_float4(thr, thg, thb, lr);
                        park[1] = make_float4(lg, lb, 0.0f, 0.0f);
                    }
                    busy = true;
                    if constexpr (kMergedInit) {
                        tr.o = o;
                        need_init = true;
                    } else {
                        tr.init(a.sc, o, dir, kRayTmin, kRayTmax, a.max_depth <= 1 && !kEmit, L);
                        if (tr.finished()) {  // empty scene: a miss
                            busy = false;
                            pending = true;
                        }
                    }
                }
                if (!kDrain) starts += take;
                pool += take;
#if SPT_WAVE_LOG
                ph[6] += take;
#endif
                idle = __ballot(!busy && !pending);
            }
            if (kMergedInit && need_init) {
                // one ray set-up for the continued and the refilled lanes (one
                // copy of the code instead of two); the last cast of a path is
                // an any-hit query (unit mode)
                tr.init(a.sc, tr.o, dir, kRayTmin, kRayTmax,
                        (meta & ((1u << kMetaDepthBits) - 1u)) + 1u >= a.max_depth && !kEmit, L);
                if (tr.finished()) {  // empty scene: a miss
                    busy = false;
                    pending = true;
                }
            }
#if SPT_WAVE_LOG
            const unsigned long long ph_t3 = __builtin_readcyclecounter();
            ph[1] += ph_t3 - ph_t0;
            ph[7] += ph_t3 - ph_t2;
#endif
        }
        if (!__ballot(busy || pending)) break;
#if SPT_WAVE_LOG
        const unsigned long long ph_t1 = __builtin_readcyclecounter();
        ph[2]++;
        ph[4] += (uint32_t)__popcll(__ballot(busy));
#endif
        if (busy && tr.step(a.sc, L, st)) {
            busy = false;
            pending = true;
        }
#if SPT_WAVE_LOG
        ph[0] += __builtin_readcyclecounter() - ph_t1;
#endif
    }
#if SPT_WAVE_LOG
    if ((threadIdx.x & 63u) == 0) {
        const uint32_t i = atomicAdd(&g_wlog_n, 1u);
        if (i < kWaveLogMax) {
            WaveRec r;
            r.t0 = wl_t0;
            r.t1 = (unsigned long long)wall_clock64();
            r.hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
            r.xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);
            r.tag = kDrain ? (uint32_t)(uintptr_t)a.qcount : 0u;
            r.casts = casts;
            r.block = blockIdx.x;
            r.drain = kDrain ? 1u : 0u;
            g_wlog[i] = r;
        }
        for (uint32_t k = 0; k < kPhaseWords; k++)
            if (ph[k]) atomicAdd(&g_phase[k], ph[k]);
    }
#endif
    // the drain: a queued path's first cast here was counted with the queue
    // (by the refill that follows), so only the casts after it are added;
    // every cast it traced goes to drained_casts
    if constexpr (kDrain) {
        if ((threadIdx.x & 63u) == 0 && casts) atomicAdd(a.drained_casts, (unsigned long long)casts);
        casts = conts;
        starts = 0;
    }
    // the wave's counts (uniform), one atomic per counter per wave
    if ((threadIdx.x & 63u) == 0) {
        if (casts) atomicAdd(&a.stats[0], (unsigned long long)casts);
        if (conts) atomicAdd(&a.stats[1], (unsigned long long)conts);
        if (starts) atomicAdd(&a.stats[2], (unsigned long long)starts);
    }
}

// Per-pixel sum of the per-sample contributions in sample order
// (film += ... once per sample, main.cpp:407), then film /= spp (main.cpp:429).
// Chunks of samples carry the running sum in acc.
// Every slot of the chunk was set to kFilmSentinel before the render: a slot
// still holding it was never written (a lost path), counted in *unwritten
// (no atomic at all when every path wrote its slot).
__global__ __launch_bounds__(256) void resolve_kernel(const float* __restrict__ sfilm, float* __restrict__ acc,
                                                      float* __restrict__ out, uint32_t P, uint32_t nsamples,
                                                      uint32_t first_chunk, uint32_t last_chunk, uint32_t spp,
                                                      uint32_t order, unsigned long long* __restrict__ unwritten) {
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    if (p >= P) return;
    uint32_t lost = 0;
    for (uint32_t c = 0; c < 3; c++) {
        float sum = first_chunk ? 0.0f : acc[(size_t)c * P + p];
        for (uint32_t s = 0; s < nsamples; s++) {
            size_t cs;
            const float x = film_rgb(const_cast<float*>(sfilm), s, p, P, nsamples, order, cs)[c * cs];
            if (c == 0 && f2u(x) == kFilmSentinel) lost++;
            sum = sum + x;
        }
        if (last_chunk)
            out[(size_t)c * P + p] = sum / (float)spp;
        else
            acc[(size_t)c * P + p] = sum;
    }
    if (lost) atomicAdd(unwritten, (unsigned long long)lost);
}

// Unit mode: every escaped sample adds the sky radiance once, in sample order
// (film += select(!hit && active, 1 x env, 0), main.cpp:407): the same
// sequence of fp32 additions as the reference (adding the 0 of a sample that
// did not escape leaves the sum as it is), then film /= spp (main.cpp:429).
__global__ __launch_bounds__(256) void resolve_flags_kernel(const uint8_t* __restrict__ sflag,
                                                            float* __restrict__ acc, float* __restrict__ out,
                                                            uint32_t P, uint32_t nsamples, uint32_t first_chunk,
                                                            uint32_t last_chunk, uint32_t spp, float env_r,
                                                            float env_g, float env_b, uint32_t order,
                                                            unsigned long long* __restrict__ unwritten) {
    const uint32_t p = blockIdx.x * 256 + threadIdx.x;
    if (p >= P) return;
    uint32_t k = 0, lost = 0;
    if (order && nsamples % 16u == 0u) {
        // pixel-major: this pixel's flags are nsamples contiguous bytes (16-B
        // aligned), read 16 at a time; a flag byte is 0, 1 or the sentinel
        // 0xff, so bit 7 counts the sentinels and bit 0 the escapes plus them
        const uint4* f4 = reinterpret_cast<const uint4*>(sflag + (size_t)p * nsamples);
        for (uint32_t c = 0; c < nsamples / 16u; c++) {
            const uint4 w = f4[c];
            const uint32_t hi = __popc(w.x & 0x80808080u) + __popc(w.y & 0x80808080u) + __popc(w.z & 0x80808080u) +
                                __popc(w.w & 0x80808080u);
            const uint32_t lo = __popc(w.x & 0x01010101u) + __popc(w.y & 0x01010101u) + __popc(w.z & 0x01010101u) +
                                __popc(w.w & 0x01010101u);
            lost += hi;
            k += lo - hi;
        }
    } else {
        for (uint32_t s = 0; s < nsamples; s++) {
            const uint32_t f = sflag[film_slot(s, p, P, nsamples, order)];
            lost += f == kFlagSentinel ? 1u : 0u;
            k += f == 1u ? 1u : 0u;
        }
    }
    if (lost) atomicAdd(unwritten, (unsigned long long)lost);
    const float env[3] = {env_r, env_g, env_b};
    for (uint32_t c = 0; c < 3; c++) {
        float sum = first_chunk ? 0.0f : acc[(size_t)c * P + p];
        for (uint32_t j = 0; j < k; j++) sum = sum + env[c];
        if (last_chunk)
            out[(size_t)c * P + p] = sum / (float)spp;
        else
            acc[(size_t)c * P + p] = sum;
    }
}

// optix_backend.h:462-486 + main.cpp:325 for the public ABI.
__global__ __launch_bounds__(256) void hit_info_kernel(HitInfoArgs a) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n) return;
    const bool m = !a.mask || ((a.mask_size == 1) ? (a.mask[0] != 0) : (a.mask[i] != 0));
    const int32_t id = a.tri_id[i];
    if (!m || id == -1) return;                                  // active = neq(tri_id,-1) && mask
    const float t = a.t[i], u = a.u[i], v = a.v[i];
    if (id < -1) {  // an analytic sphere (spt_scene_set_spheres): -2 - k
        const uint32_t k = (uint32_t)(-2 - id);
        if (k >= a.sc.nsph) return;
        // the hit point (and from it the normal) only when an output needs it:
        // texcoord / material outputs never read the ray planes, which may be
        // NULL then (spt_hit_info_compute checks the rest)
        const bool want_n = a.gnx || a.gny || a.gnz || a.snx || a.sny || a.snz;
        if (want_n || a.px || a.py || a.pz) {
            const float4 sp = a.sc.spheres[k];
            const V3 p = v3(a.ox[i] + t * a.dx[i], a.oy[i] + t * a.dy[i], a.oz[i] + t * a.dz[i]);
            if (a.px) a.px[i] = p.x;
            if (a.py) a.py[i] = p.y;
            if (a.pz) a.pz[i] = p.z;
            if (want_n) {
                const V3 n = normalize(v3(p.x - sp.x, p.y - sp.y, p.z - sp.z));
                if (a.gnx) a.gnx[i] = n.x;
                if (a.gny) a.gny[i] = n.y;
                if (a.gnz) a.gnz[i] = n.z;
                if (a.snx) a.snx[i] = n.x;
                if (a.sny) a.sny[i] = n.y;
                if (a.snz) a.snz[i] = n.z;
            }
        }
        if (a.tcu) a.tcu[i] = 0.0f;
        if (a.tcv) a.tcv[i] = 0.0f;
        if (a.mat_id) a.mat_id[i] = a.sc.sph_mat ? a.sc.sph_mat[k] : 0;
        return;
    }
    if (id < 0 || (uint64_t)id >= a.ntri) return;
    const int32_t slot = a.sc.orig2slot[id];
    // every output plane may be NULL on its own (spt.h spt_hit_info)
    if (a.px) a.px[i] = a.ox[i] + t * a.dx[i];
    if (a.py) a.py[i] = a.oy[i] + t * a.dy[i];
    if (a.pz) a.pz[i] = a.oz[i] + t * a.dz[i];
    if (a.gnx || a.gny || a.gnz) {
        V3 q0, q1, q2;
        tri_vertices(tri_rec(a.sc, (uint32_t)slot), q0, q1, q2);
        const float4 p0 = make_float4(q0.x, q0.y, q0.z, 0.0f), p1 = make_float4(q1.x, q1.y, q1.z, 0.0f),
                     p2 = make_float4(q2.x, q2.y, q2.z, 0.0f);
        const V3 g = normalize(cross(v3(p1.x - p0.x, p1.y - p0.y, p1.z - p0.z),  // add_math.h:9-16
                                     v3(p2.x - p0.x, p2.y - p0.y, p2.z - p0.z)));
        if (a.gnx) a.gnx[i] = g.x;
        if (a.gny) a.gny[i] = g.y;
        if (a.gnz) a.gnz[i] = g.z;
    }
    const float w = (1.0f - u) - v;
    const float4 m0 = a.sc.snrm[(size_t)slot * 3];
    if (a.snx || a.sny || a.snz) {
        const float4 m1 = a.sc.snrm[(size_t)slot * 3 + 1], m2 = a.sc.snrm[(size_t)slot * 3 + 2];
        if (a.snx) a.snx[i] = (w * m0.x + u * m1.x) + v * m2.x;
        if (a.sny) a.sny[i] = (w * m0.y + u * m1.y) + v * m2.y;
        if (a.snz) a.snz[i] = (w * m0.z + u * m1.z) + v * m2.z;
    }
    if (a.tcu || a.tcv) {
        float cu = 0.0f, cv = 0.0f;
        if (a.sc.tc) {
            const float* c = a.sc.tc + (size_t)slot * 6;
            cu = (w * c[0] + u * c[2]) + v * c[4];
            cv = (w * c[1] + u * c[3]) + v * c[5];
        }
        if (a.tcu) a.tcu[i] = cu;
        if (a.tcv) a.tcv[i] = cv;
    }
    if (a.mat_id) a.mat_id[i] = (int32_t)f2u(m0.w);
}

// ------------------------------------------------------------- launchers
static inline uint32_t blocks_for(uint32_t items, uint32_t block) { return (items + block - 1) / block; }

// Workgroups resident on the whole chip for this LDS stack size (cached).
template <typename Tr, bool kStats, bool kCam, bool kNt>
static uint32_t persistent_blocks(size_t lds) {
    static thread_local size_t cached_lds = 0;
    static thread_local uint32_t cached = 0;
    static thread_local int cached_dev = -1;
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (cached && cached_lds == lds && cached_dev == dev) return cached;
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, isect_queue_kernel<Tr, kStats, kCam, kNt>, kIsectBlock, lds) !=
            hipSuccess || per_cu <= 0)
        per_cu = 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    cached = (uint32_t)(per_cu * cus);
    cached_lds = lds;
    cached_dev = dev;
    return cached;
}

template <typename Tr, bool kStats, bool kCam = false, bool kNt = false>
static hipError_t launch_isect_queue_t(const IsectQueueArgs& a, uint32_t grid_items, hipStream_t s) {
    if (grid_items == 0) return hipSuccess;
    const size_t lds = (size_t)a.sc.stack_depth * Tr::kStackWords * kIsectBlock * sizeof(uint32_t) + Tr::kExtraLds;
    const uint32_t full = persistent_blocks<Tr, kStats, kCam, kNt>(lds);
    const uint32_t scaled = a.grid_q8 ? max(1u, (uint32_t)(((uint64_t)full * a.grid_q8) >> 8)) : full;
    const uint32_t blocks = min(scaled, blocks_for(grid_items, kIsectBlock));
    hipLaunchKernelGGL((isect_queue_kernel<Tr, kStats, kCam, kNt>), dim3(blocks), dim3(kIsectBlock), lds, s, a);
    return hipGetLastError();
}

template <typename Tr, bool kNt>
static uint32_t isect_queue_lanes_t(const IsectQueueArgs& a) {
    const size_t lds = (size_t)a.sc.stack_depth * Tr::kStackWords * kIsectBlock * sizeof(uint32_t) + Tr::kExtraLds;
    const uint32_t full = persistent_blocks<Tr, false, false, kNt>(lds);
    const uint32_t scaled = a.grid_q8 ? max(1u, (uint32_t)(((uint64_t)full * a.grid_q8) >> 8)) : full;
    return scaled * kIsectBlock;
}

uint32_t isect_queue_lanes(const IsectQueueArgs& a) {
    if (!a.sc.nodes8) return isect_queue_lanes_t<Tracer, false>(a);
    if (a.nt) return a.sc.node6 ? isect_queue_lanes_t<Tracer6, true>(a) : isect_queue_lanes_t<Tracer8, true>(a);
    return a.sc.node6 ? isect_queue_lanes_t<Tracer6, false>(a) : isect_queue_lanes_t<Tracer8, false>(a);
}

hipError_t launch_isect_queue(const IsectQueueArgs& a, uint32_t grid_items, hipStream_t s) {
    if (!a.sc.nodes8)
        return a.nt ? launch_isect_queue_t<Tracer, false, false, true>(a, grid_items, s)
                    : launch_isect_queue_t<Tracer, false>(a, grid_items, s);
    if (a.nt)
        return a.sc.node6 ? launch_isect_queue_t<Tracer6, false, false, true>(a, grid_items, s)
                          : launch_isect_queue_t<Tracer8, false, false, true>(a, grid_items, s);
    return a.sc.node6 ? launch_isect_queue_t<Tracer6, false>(a, grid_items, s)
                      : launch_isect_queue_t<Tracer8, false>(a, grid_items, s);
}

// the isect launch that also starts the camera paths (IsectQueueArgs::cam)
hipError_t launch_isect_queue_cam(const IsectQueueArgs& a, uint32_t grid_items, hipStream_t s) {
    if (!a.sc.nodes8) return launch_isect_queue_t<Tracer, false, true>(a, grid_items, s);
    return a.sc.node6 ? launch_isect_queue_t<Tracer6, false, true>(a, grid_items, s)
                      : launch_isect_queue_t<Tracer8, false, true>(a, grid_items, s);
}

template <typename Tr, bool kNt>
static hipError_t launch_isect_lockstep_t(const IsectQueueArgs& a, uint32_t grid_items, hipStream_t s) {
    if (grid_items == 0) return hipSuccess;
    const size_t lds = (size_t)a.sc.stack_depth * Tr::kStackWords * kIsectBlock * sizeof(uint32_t) + Tr::kExtraLds;
    hipLaunchKernelGGL((isect_lockstep_kernel<Tr, kNt>), dim3(blocks_for(grid_items, kIsectBlock)), dim3(kIsectBlock),
                       lds, s, a);
    return hipGetLastError();
}

// grid_items: the queue count, known exactly (a fitting job's first cast)
hipError_t launch_isect_lockstep(const IsectQueueArgs& a, uint32_t grid_items, hipStream_t s) {
    if (!a.sc.nodes8)
        return a.nt ? launch_isect_lockstep_t<Tracer, true>(a, grid_items, s)
                    : launch_isect_lockstep_t<Tracer, false>(a, grid_items, s);
    if (a.nt)
        return a.sc.node6 ? launch_isect_lockstep_t<Tracer6, true>(a, grid_items, s)
                          : launch_isect_lockstep_t<Tracer8, true>(a, grid_items, s);
    return a.sc.node6 ? launch_isect_lockstep_t<Tracer6, false>(a, grid_items, s)
                      : launch_isect_lockstep_t<Tracer8, false>(a, grid_items, s);
}

template <typename Tr, int kMode, bool kSpt, bool kNt>
static hipError_t launch_camera_cast_t(const CameraCastArgs& a, hipStream_t s) {
    const size_t lds = (size_t)a.s.sc.stack_depth * Tr::kStackWords * kIsectBlock * sizeof(uint32_t) + Tr::kExtraLds;
    hipLaunchKernelGGL((camera_cast_kernel<Tr, kMode, kSpt, kNt>), dim3(blocks_for(a.n, kIsectBlock)),
                       dim3(kIsectBlock), lds, s, a);
    return hipGetLastError();
}

template <typename Tr, bool kNt>
static hipError_t launch_camera_cast_m(const CameraCastArgs& a, int mode, hipStream_t s) {
    const bool spt = a.s.sc.nsph || a.s.sc.nkind;  // never in unit mode (launch_shade)
    if (mode == kModeEmit && spt) return launch_camera_cast_t<Tr, kModeEmit, true, kNt>(a, s);
    if (mode == kModeEmit) return launch_camera_cast_t<Tr, kModeEmit, false, kNt>(a, s);
    if (mode == kModeAlbedo && spt) return launch_camera_cast_t<Tr, kModeAlbedo, true, kNt>(a, s);
    if (mode == kModeAlbedo) return launch_camera_cast_t<Tr, kModeAlbedo, false, kNt>(a, s);
    return launch_camera_cast_t<Tr, kModeUnit, false, kNt>(a, s);
}

// wide-BVH scenes only (camera_cast_supported); a.n: the work items, known exactly
hipError_t launch_camera_cast(const CameraCastArgs& a, int mode, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    if (!a.s.sc.nodes8) return hipErrorInvalidValue;
    if (a.s.nt)
        return a.s.sc.node6 ? launch_camera_cast_m<Tracer6, true>(a, mode, s)
                            : launch_camera_cast_m<Tracer8, true>(a, mode, s);
    return a.s.sc.node6 ? launch_camera_cast_m<Tracer6, false>(a, mode, s)
                        : launch_camera_cast_m<Tracer8, false>(a, mode, s);
}

hipError_t launch_isect_queue_stats(const IsectQueueArgs& a, uint32_t grid_items, hipStream_t s) {
    if (!a.sc.nodes8) return launch_isect_queue_t<Tracer, true>(a, grid_items, s);
    return a.sc.node6 ? launch_isect_queue_t<Tracer6, true>(a, grid_items, s)
                      : launch_isect_queue_t<Tracer8, true>(a, grid_items, s);
}

template <typename Tr>
static uint32_t public_persistent_blocks(size_t lds) {
    static thread_local size_t cached_lds = 0;
    static thread_local uint32_t cached = 0;
    static thread_local int cached_dev = -1;
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (!cached || cached_lds != lds || cached_dev != dev) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, isect_public_persistent_kernel<Tr>, kIsectBlock,
                                                         lds) != hipSuccess || per_cu <= 0)
            per_cu = 1;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        cached = (uint32_t)(per_cu * cus);
        cached_lds = lds;
        cached_dev = dev;
    }
    return cached;
}

hipError_t launch_isect_public(const IsectPublicArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    // one word per stack entry (both layouts), plus the BVH8 tracer's records
    const size_t lds = (size_t)a.sc.stack_depth * kIsectBlock * sizeof(uint32_t) + Tracer8::kExtraLds;
    // one lane per ray by default: the reference's first bounce (camera rays)
    // traces 25-30 % faster in lockstep waves; the persistent kernel wins on
    // incoherent rays (+25-36 %) — tools/isect_api_bench.py, DESIGN.md §4
    if (a.sc.nodes8 && a.persistent) {
        const uint32_t cached = a.sc.node6 ? public_persistent_blocks<Tracer6>(lds) : public_persistent_blocks<Tracer8>(lds);
        // at least 64 rays per wave (a wave's share), at most the chip's occupancy
        const uint32_t blocks = max(1u, min(cached, blocks_for(a.n, kIsectBlock / 64 * 64 * 2)));
        if (a.sc.node6)
            hipLaunchKernelGGL(isect_public_persistent_kernel<Tracer6>, dim3(blocks), dim3(kIsectBlock), lds, s, a);
        else
            hipLaunchKernelGGL(isect_public_persistent_kernel<Tracer8>, dim3(blocks), dim3(kIsectBlock), lds, s, a);
        return hipGetLastError();
    }
    const dim3 g(blocks_for(a.n, kIsectBlock)), b(kIsectBlock);
    if (!a.sc.nodes8) hipLaunchKernelGGL(isect_public_kernel<Tracer>, g, b, lds, s, a);
    else if (a.sc.node6) hipLaunchKernelGGL(isect_public_kernel<Tracer6>, g, b, lds, s, a);
    else hipLaunchKernelGGL(isect_public_kernel<Tracer8>, g, b, lds, s, a);
    return hipGetLastError();
}

hipError_t launch_shade(const ShadeArgs& a, int mode, uint32_t grid_items, hipStream_t s) {
    if (grid_items == 0) return hipSuccess;
    const dim3 g(blocks_for(grid_items, kShadeBlock)), b(kShadeBlock);
    const bool spt = a.sc.nsph || a.sc.nkind;  // never in unit mode (spt_render)
    if (a.nt) {  // non-temporal queue accesses (spt_config.queue_cache), every instance
        if (mode == kModeEmit && spt) hipLaunchKernelGGL((shade_kernel<kModeEmit, true, true>), g, b, 0, s, a);
        else if (mode == kModeEmit) hipLaunchKernelGGL((shade_kernel<kModeEmit, false, true>), g, b, 0, s, a);
        else if (mode == kModeAlbedo && spt) hipLaunchKernelGGL((shade_kernel<kModeAlbedo, true, true>), g, b, 0, s, a);
        else if (mode == kModeAlbedo) hipLaunchKernelGGL((shade_kernel<kModeAlbedo, false, true>), g, b, 0, s, a);
        else hipLaunchKernelGGL((shade_kernel<kModeUnit, false, true>), g, b, 0, s, a);
        return hipGetLastError();
    }
    if (mode == kModeEmit && spt) hipLaunchKernelGGL((shade_kernel<kModeEmit, true>), g, b, 0, s, a);
    else if (mode == kModeEmit) hipLaunchKernelGGL((shade_kernel<kModeEmit, false>), g, b, 0, s, a);
    else if (mode == kModeAlbedo && spt) hipLaunchKernelGGL((shade_kernel<kModeAlbedo, true>), g, b, 0, s, a);
    else if (mode == kModeAlbedo) hipLaunchKernelGGL((shade_kernel<kModeAlbedo, false>), g, b, 0, s, a);
    else hipLaunchKernelGGL((shade_kernel<kModeUnit, false>), g, b, 0, s, a);
    return hipGetLastError();
}

template <typename Tr, int kMode, bool kDrain = false, bool kNt = false>
static hipError_t launch_fused_t(const FusedArgs& a, hipStream_t s, uint32_t* lanes_out) {
    static thread_local size_t cached_lds = 0;
    static thread_local uint32_t cached = 0;
    static thread_local int cached_dev = -1;
    // + the parked throughput / radiance of albedo / emitter lanes (render_fused_kernel)
    const size_t park = kMode != kModeUnit && SPT_PARK_PATH ? (size_t)kIsectBlock * 32 : 0;
    const size_t lds = (size_t)a.sc.stack_depth * Tr::kStackWords * kIsectBlock * sizeof(uint32_t) + Tr::kExtraLds + park;
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (!cached || cached_lds != lds || cached_dev != dev) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, render_fused_kernel<Tr, kMode, kDrain, kNt>,
                                                         kIsectBlock, lds) != hipSuccess || per_cu <= 0)
            per_cu = 1;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        cached = (uint32_t)(per_cu * cus);
        cached_lds = lds;
        cached_dev = dev;
    }
    const uint32_t scaled = a.grid_q8 ? max(1u, (uint32_t)(((uint64_t)cached * a.grid_q8) >> 8)) : cached;
    // (the drain's grid cannot follow its count, which is on the device)
    const uint32_t blocks = kDrain ? scaled : min(scaled, blocks_for(a.count > 0 ? a.count : 1, kIsectBlock));
    if (lanes_out) *lanes_out = blocks * kIsectBlock;
    hipLaunchKernelGGL((render_fused_kernel<Tr, kMode, kDrain, kNt>), dim3(blocks), dim3(kIsectBlock), lds, s, a);
    return hipGetLastError();
}

template <int kMode, bool kNt>
static hipError_t launch_drain_m(const FusedArgs& a, hipStream_t s) {
    if (a.sc.nodes8 && a.sc.node6) return launch_fused_t<Tracer6F, kMode, true, kNt>(a, s, nullptr);
    if (a.sc.nodes8) return launch_fused_t<Tracer8F, kMode, true, kNt>(a, s, nullptr);
    return launch_fused_t<Tracer, kMode, true, kNt>(a, s, nullptr);
}

// Sort key of a queued path (launch_drain_sort): its direction's octant, then
// the Morton code of its origin on a 512^3 grid over the root node's box, so
// that a wave's lanes take bounce rays that start near each other and head
// the same way (the drain continues each path in its lane, so the order
// decides which rays a wave traces together).  Slots past the count: last.
__global__ __launch_bounds__(256) void drain_keys_kernel(DeviceScene sc, PathQueue q, const uint32_t* count,
                                                         uint32_t cap, uint32_t* keys, uint32_t* vals) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= cap) return;
    uint32_t key = 0xffffffffu;
    if (i < *count) {
        const uint4 w0 = sc.nodes8[0], w1 = sc.nodes8[1];  // the root: origin, exponents
        uint32_t ex, ey, ez;
        if (sc.node6) {
            ex = (w1.y >> 16) & 0xffu; ey = w1.y >> 24; ez = w1.z >> 24;
        } else {
            ex = w0.w & 0xffu; ey = (w0.w >> 8) & 0xffu; ez = (w0.w >> 16) & 0xffu;
        }
        const float4 q1 = q.q1[i], q2 = q.q2[i];
        const auto cell = [](float o, uint32_t p, uint32_t e) {
            const float ext = 255.0f * u2f(e << 23);  // the root box: p + [0, 255 * 2^(e - 127)]
            const float f = (o - u2f(p)) / ext * 512.0f;
            return (uint32_t)fminf(fmaxf(f, 0.0f), 511.0f);
        };
        const auto spread = [](uint32_t v) {  // 9 bits -> every third bit
            v = (v | (v << 16)) & 0x030000ffu;
            v = (v | (v << 8)) & 0x0300f00fu;
            v = (v | (v << 4)) & 0x030c30c3u;
            v = (v | (v << 2)) & 0x09249249u;
            return v;
        };
        const uint32_t m = spread(cell(q1.x, w0.x, ex)) | spread(cell(q1.y, w0.y, ey)) << 1 |
                           spread(cell(q1.z, w0.z, ez)) << 2;
        const uint32_t oct = (q2.x < 0.0f ? 1u : 0u) | (q2.y < 0.0f ? 2u : 0u) | (q2.z < 0.0f ? 4u : 0u);
        key = oct << 27 | m;
    }
    keys[i] = key;
    vals[i] = i;
}

hipError_t launch_drain_sort(const DeviceScene& sc, const PathQueue& q, const uint32_t* count, uint32_t cap,
                             uint32_t* keys, uint32_t* vals, uint32_t* keys_out, uint32_t* perm, void* tmp,
                             size_t* tmp_bytes, hipStream_t s) {
    if (!tmp)
        return hipcub::DeviceRadixSort::SortPairs(nullptr, *tmp_bytes, keys, keys_out, vals, perm, (int)cap, 0, 30, s);
    if (!sc.nodes8 || cap == 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(drain_keys_kernel, dim3(blocks_for(cap, 256)), dim3(256), 0, s, sc, q, count, cap, keys, vals);
    hipError_t e = hipGetLastError();
    if (e) return e;
    // 30 key bits: the octant above the 27-bit Morton code (an empty slot's
    // all-ones key sorts after every real one in its low 30 bits too)
    return hipcub::DeviceRadixSort::SortPairs(tmp, *tmp_bytes, keys, keys_out, vals, perm, (int)cap, 0, 30, s);
}

hipError_t launch_drain(const FusedArgs& a, int mode, hipStream_t s) {
    if (a.nt) {
        if (mode == kModeEmit) return launch_drain_m<kModeEmit, true>(a, s);
        if (mode == kModeAlbedo) return launch_drain_m<kModeAlbedo, true>(a, s);
        return launch_drain_m<kModeUnit, true>(a, s);
    }
    if (mode == kModeEmit) return launch_drain_m<kModeEmit, false>(a, s);
    if (mode == kModeAlbedo) return launch_drain_m<kModeAlbedo, false>(a, s);
    return launch_drain_m<kModeUnit, false>(a, s);
}

hipError_t launch_fused(const FusedArgs& a, int mode, hipStream_t s, uint32_t* lanes_out) {
    if (a.sc.nodes8 && a.sc.node6) {
        if (mode == kModeEmit) return launch_fused_t<Tracer6F, kModeEmit>(a, s, lanes_out);
        if (mode == kModeAlbedo) return launch_fused_t<Tracer6F, kModeAlbedo>(a, s, lanes_out);
        return launch_fused_t<Tracer6F, kModeUnit>(a, s, lanes_out);
    }
    if (a.sc.nodes8) {
        if (mode == kModeEmit) return launch_fused_t<Tracer8F, kModeEmit>(a, s, lanes_out);
        if (mode == kModeAlbedo) return launch_fused_t<Tracer8F, kModeAlbedo>(a, s, lanes_out);
        return launch_fused_t<Tracer8F, kModeUnit>(a, s, lanes_out);
    }
    if (mode == kModeEmit) return launch_fused_t<Tracer, kModeEmit>(a, s, lanes_out);
    if (mode == kModeAlbedo) return launch_fused_t<Tracer, kModeAlbedo>(a, s, lanes_out);
    return launch_fused_t<Tracer, kModeUnit>(a, s, lanes_out);
}

hipError_t launch_refill(const RefillArgs& a, uint32_t grid_items, hipStream_t s) {
#if SPT_REFILL_STRIDE
    const dim3 g(std::min<uint32_t>(blocks_for(grid_items > 0 ? grid_items : 1, 256), kRefillMaxBlocks)), b(256);
#else
    const dim3 g(blocks_for(grid_items > 0 ? grid_items : 1, 256)), b(256);
#endif
    if (a.nt) {
        if (a.mode == kModeEmit) hipLaunchKernelGGL((refill_kernel<kModeEmit, true>), g, b, 0, s, a);
        else if (a.mode == kModeAlbedo) hipLaunchKernelGGL((refill_kernel<kModeAlbedo, true>), g, b, 0, s, a);
        else hipLaunchKernelGGL((refill_kernel<kModeUnit, true>), g, b, 0, s, a);
    } else if (a.mode == kModeEmit) hipLaunchKernelGGL(refill_kernel<kModeEmit>, g, b, 0, s, a);
    else if (a.mode == kModeAlbedo) hipLaunchKernelGGL(refill_kernel<kModeAlbedo>, g, b, 0, s, a);
    else hipLaunchKernelGGL(refill_kernel<kModeUnit>, g, b, 0, s, a);
    return hipGetLastError();
}

hipError_t launch_resolve(const float* sfilm, float* acc, float* out, uint32_t P, uint32_t nsamples,
                          uint32_t first_chunk, uint32_t last_chunk, uint32_t spp, uint32_t order,
                          unsigned long long* unwritten, hipStream_t s) {
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(resolve_kernel, dim3(blocks_for(P, 256)), dim3(256), 0, s, sfilm, acc, out, P, nsamples,
                       first_chunk, last_chunk, spp, order, unwritten);
    return hipGetLastError();
}

hipError_t launch_resolve_flags(const uint8_t* sflag, float* acc, float* out, uint32_t P, uint32_t nsamples,
                                uint32_t first_chunk, uint32_t last_chunk, uint32_t spp, float env_r, float env_g,
                                float env_b, uint32_t order, unsigned long long* unwritten, hipStream_t s) {
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(resolve_flags_kernel, dim3(blocks_for(P, 256)), dim3(256), 0, s, sflag, acc, out, P, nsamples,
                       first_chunk, last_chunk, spp, env_r, env_g, env_b, order, unwritten);
    return hipGetLastError();
}

hipError_t launch_hit_info(const HitInfoArgs& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    hipLaunchKernelGGL(hit_info_kernel, dim3(blocks_for(a.n, 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace spt

#if SPT_WAVE_LOG
// Diagnostic build only: copy up to `max` wave records (8 x 8-byte words each:
// t0, t1, hw | xcc << 32, tag | casts << 32, block | drain << 32) to `out`,
// return how many waves logged since the last reset (device synchronised first).
extern "C" long long spt_debug_wave_log(void* out, unsigned long long max, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    uint32_t n = 0;
    if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(spt::g_wlog_n), sizeof(n)) != hipSuccess) return -1;
    const unsigned long long take = std::min<unsigned long long>(std::min<unsigned long long>(n, spt::kWaveLogMax), max);
    if (out && take &&
        hipMemcpyFromSymbol(out, HIP_SYMBOL(spt::g_wlog), take * sizeof(spt::WaveRec)) != hipSuccess)
        return -1;
    if (reset) {
        const uint32_t z = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(spt::g_wlog_n), &z, sizeof(z)) != hipSuccess) return -1;
    }
    return (long long)n;
}

// Diagnostic build only: the kPhaseWords phase counters (g_phase above) into
// `out` (8 unsigned 64-bit words), zeroed after when `reset`.
extern "C" int spt_debug_phase_log(unsigned long long* out, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(spt::g_phase), sizeof(spt::g_phase)) != hipSuccess) return -1;
    if (reset) {
        const unsigned long long z[spt::kPhaseWords] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(spt::g_phase), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
