// gpu_build.hip — the acceleration structure built on the GPU (gfx950):
// PLOC BVH2 (Meister & Bittner, "Parallel Locally-Ordered Clustering for
// Bounding Volume Hierarchy Construction", TVCG 2018) over 63-bit Morton
// order, then a level-by-level collapse into the compressed 8-wide layout of
// bvh_build.h (the same greedy collapse, octant slot order and conservative
// 8-bit quantisation as bvh8_build.cpp, one thread per BVH8 node).
//
// Replaces the reference's on-device GAS build (optixAccelBuild +
// optixAccelCompact, optix_backend.h:336-358); the host binned-SAH build
// (bvh_build.cpp) stays as the default for small scenes.  Every step is
// deterministic: node and triangle offsets come from prefix sums, never from
// atomics, so a scene always gets the same tree.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#include "bvh_build.h"
#include "gpu_build.h"
#include "spt_internal.h"

namespace spt {
namespace {

constexpr uint32_t kBlock = 256;
constexpr uint32_t kLeafMaxTris = 3;  // a BVH8 leaf holds up to 3 triangles


inline uint32_t blocks(uint64_t n, uint32_t b = kBlock) { return (uint32_t)((n + b - 1) / b); }

// order-preserving float <-> uint map, for atomicMin/Max on floats
__device__ __forceinline__ uint32_t f2ord(float f) {
    const uint32_t u = __builtin_bit_cast(uint32_t, f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t u) {
    return __builtin_bit_cast(float, (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__device__ __forceinline__ float half_area(float4 lo, float4 hi) {
    const float dx = hi.x - lo.x, dy = hi.y - lo.y, dz = hi.z - lo.z;
    return dx * dy + dy * dz + dz * dx;
}

__device__ __forceinline__ uint64_t spread21(uint64_t x) {
    x &= 0x1fffff;
    x = (x | x << 32) & 0x1f00000000ffffull;
    x = (x | x << 16) & 0x1f0000ff0000ffull;
    x = (x | x << 8) & 0x100f00f00f00f00full;
    x = (x | x << 4) & 0x10c30c30c30c30c3ull;
    x = (x | x << 2) & 0x1249249249249249ull;
    return x;
}

// Per-triangle box, and the centroid bounds (ordered-uint atomics, 6 words).
__global__ __launch_bounds__(kBlock) void tri_box_kernel(const float* __restrict__ tv, uint32_t n,
                                                         float4* __restrict__ lo, float4* __restrict__ hi,
                                                         uint32_t* __restrict__ cb) {
    __shared__ uint32_t s[6];
    if (threadIdx.x < 6) s[threadIdx.x] = threadIdx.x < 3 ? 0xffffffffu : 0u;
    __syncthreads();
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) {
        const float* v = tv + (size_t)i * 9;
        float l[3], h[3];
        for (int a = 0; a < 3; a++) {
            l[a] = fminf(fminf(v[a], v[3 + a]), v[6 + a]);
            h[a] = fmaxf(fmaxf(v[a], v[3 + a]), v[6 + a]);
        }
        lo[i] = make_float4(l[0], l[1], l[2], 0.0f);
        hi[i] = make_float4(h[0], h[1], h[2], 0.0f);
        for (int a = 0; a < 3; a++) {
            const float c = 0.5f * (l[a] + h[a]);
            atomicMin(&s[a], f2ord(c));
            atomicMax(&s[3 + a], f2ord(c));
        }
    }
    __syncthreads();
    if (threadIdx.x < 3) atomicMin(&cb[threadIdx.x], s[threadIdx.x]);
    else if (threadIdx.x < 6) atomicMax(&cb[threadIdx.x], s[threadIdx.x]);
}

// Morton codes of the triangle centroids on a cubic grid over the centroid
// bounds (the longest axis's extent for all three: cells are cubes, so the
// code's locality is the same along every axis).  Per-axis normalisation
// gave the city's 20 x 5 x 16 extent 4x finer cells in y: its PLOC tree had a
// 2.5 % higher SAH cost (96.6 vs 94.3) and rendered 1.4 % slower; a 4D code
// with the box diagonal as the fourth coordinate (Vinkler et al. 2017) had
// the same SAH and rendered 3.6 % slower (EXPERIMENTS.md round 4).
#ifndef SPT_MORTON
#define SPT_MORTON 1  // 0: per-axis normalised 63-bit, 1: cube-normalised 63-bit, 2: 4D (x, y, z, size) 60-bit
#endif
__device__ __forceinline__ uint64_t spread15_4(uint64_t x) {  // bit k of x to bit 4k
    x &= 0x7fff;
    uint64_t r = 0;
    for (int k = 0; k < 15; k++) r |= ((x >> k) & 1ull) << (4 * k);
    return r;
}
__global__ __launch_bounds__(kBlock) void morton_kernel(const float4* __restrict__ lo, const float4* __restrict__ hi,
                                                        uint32_t n, const uint32_t* __restrict__ cb,
                                                        uint64_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float4 l = lo[i], h = hi[i];
    const float c[3] = {0.5f * (l.x + h.x), 0.5f * (l.y + h.y), 0.5f * (l.z + h.z)};
    uint64_t key = 0;
    float cube = 0.0f;
    for (int a = 0; a < 3; a++) cube = fmaxf(cube, ord2f(cb[3 + a]) - ord2f(cb[a]));
    for (int a = 0; a < 3; a++) {
        const float b0 = ord2f(cb[a]), b1 = ord2f(cb[3 + a]);
        const float ext = SPT_MORTON ? cube : b1 - b0;
        float t = ext > 0.0f ? (c[a] - b0) / ext : 0.5f;
        t = fminf(fmaxf(t, 0.0f), 1.0f);
        if (SPT_MORTON == 2) key |= spread15_4((uint64_t)(t * 32767.0f)) << (3 - a);
        else key |= spread21((uint64_t)(t * 2097151.0f)) << (2 - a);
    }
    if (SPT_MORTON == 2) {
        // the box diagonal as a fourth coordinate (Vinkler et al. 2017's
        // extended Morton codes): large and small triangles part early
        const float dx = h.x - l.x, dy = h.y - l.y, dz = h.z - l.z;
        float sz = cube > 0.0f ? sqrtf(dx * dx + dy * dy + dz * dz) / (1.7320508f * cube) : 0.0f;
        sz = fminf(fmaxf(sz, 0.0f), 1.0f);
        key |= spread15_4((uint64_t)(sz * 32767.0f));
    }
    keys[i] = key;
    vals[i] = i;
}

// Clusters start as the Morton-sorted triangles (BVH2 leaf node id = triangle id).
__global__ __launch_bounds__(kBlock) void init_clusters_kernel(const uint32_t* __restrict__ order, uint32_t n,
                                                               const float4* __restrict__ lo,
                                                               const float4* __restrict__ hi,
                                                               uint32_t* __restrict__ cnode, float4* __restrict__ clo,
                                                               float4* __restrict__ chi) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t t = order[i];
    cnode[i] = t;
    clo[i] = lo[t];
    chi[i] = hi[t];
}

__global__ __launch_bounds__(kBlock) void leaf_ones_kernel(uint32_t* __restrict__ ntris, uint32_t n) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) ntris[i] = 1u;
}

// Nearest neighbour within +-r in the cluster array: the one whose merged box
// has the smallest area; ties go to the smaller index, so the candidate pair
// with the smallest (area, lower index, higher index) is always mutual and
// every iteration merges at least one pair.
template <int kPlocRadius>  // neighbours searched on each side (PLOC's r)
__global__ __launch_bounds__(kBlock) void nn_kernel(const float4* __restrict__ clo, const float4* __restrict__ chi,
                                                    uint32_t n, uint32_t* __restrict__ nn) {
    __shared__ float4 slo[kBlock + 2 * kPlocRadius], shi[kBlock + 2 * kPlocRadius];
    const int64_t b0 = (int64_t)blockIdx.x * kBlock - kPlocRadius;
    for (uint32_t k = threadIdx.x; k < kBlock + 2 * kPlocRadius; k += kBlock) {
        const int64_t j = b0 + k;
        if (j >= 0 && j < (int64_t)n) {
            slo[k] = clo[j];
            shi[k] = chi[j];
        }
    }
    __syncthreads();
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t li = threadIdx.x + kPlocRadius;
    const float4 l = slo[li], h = shi[li];
    float best = INFINITY;
    uint32_t bj = i;
    const int64_t jlo = std::max<int64_t>(0, (int64_t)i - kPlocRadius);
    const int64_t jhi = std::min<int64_t>((int64_t)n - 1, (int64_t)i + kPlocRadius);
    for (int64_t j = jlo; j <= jhi; j++) {
        if (j == (int64_t)i) continue;
        const uint32_t lj = (uint32_t)(j - b0);
        const float4 ol = slo[lj], oh = shi[lj];
        const float a = half_area(make_float4(fminf(l.x, ol.x), fminf(l.y, ol.y), fminf(l.z, ol.z), 0.0f),
                                  make_float4(fmaxf(h.x, oh.x), fmaxf(h.y, oh.y), fmaxf(h.z, oh.z), 0.0f));
        if (a < best) {
            best = a;
            bj = (uint32_t)j;
        }
    }
    nn[i] = bj;
}

// flags[i] = merge << 32 | keep: cluster i opens a merge with its mutual
// nearest neighbour (the lower of the pair), or survives (all but the higher).
__global__ __launch_bounds__(kBlock) void merge_flags_kernel(const uint32_t* __restrict__ nn, uint32_t n,
                                                             uint64_t* __restrict__ flags) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t j = nn[i];
    const bool mutual = j != i && nn[j] == i;
    const uint64_t merge = mutual && i < j, keep = !(mutual && i > j);
    flags[i] = (merge << 32) | keep;
}

// Merge and compact in one pass.  New inner node ids: leaves occupy [0, ntri),
// inner nodes are numbered in creation order from ntri.
__global__ __launch_bounds__(kBlock) void merge_compact_kernel(
    const uint32_t* __restrict__ nn, const uint64_t* __restrict__ flags, const uint64_t* __restrict__ scan,
    uint32_t n, uint32_t node_base, const uint32_t* __restrict__ cnode, const float4* __restrict__ clo,
    const float4* __restrict__ chi, uint32_t* __restrict__ onode, float4* __restrict__ olo,
    float4* __restrict__ ohi, float4* __restrict__ nlo, float4* __restrict__ nhi, int2* __restrict__ nkids,
    uint32_t* __restrict__ ntris) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint64_t f = flags[i];
    if (!(f & 1u)) return;
    const uint32_t dst = (uint32_t)(scan[i] & 0xffffffffu);
    if (f >> 32) {
        const uint32_t j = nn[i];
        const uint32_t id = node_base + (uint32_t)(scan[i] >> 32);
        const float4 a = clo[i], b = clo[j], c = chi[i], d = chi[j];
        const float4 l = make_float4(fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z), 0.0f);
        const float4 h = make_float4(fmaxf(c.x, d.x), fmaxf(c.y, d.y), fmaxf(c.z, d.z), 0.0f);
        const uint32_t ci = cnode[i], cj = cnode[j];
        nlo[id] = l;
        nhi[id] = h;
        nkids[id] = make_int2((int)ci, (int)cj);
        ntris[id] = ntris[ci] + ntris[cj];
        onode[dst] = id;
        olo[dst] = l;
        ohi[dst] = h;
    } else {
        onode[dst] = cnode[i];
        olo[dst] = clo[i];
        ohi[dst] = chi[i];
    }
}

// totals of an exclusive scan: out = scan[n-1] + flags[n-1]
__global__ void scan_total_kernel(const uint64_t* __restrict__ flags, const uint64_t* __restrict__ scan, uint32_t n,
                                  uint64_t* __restrict__ out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *out = n ? scan[n - 1] + flags[n - 1] : 0ull;
}

// SAH cost of the BVH2 (bvh_build.cpp's accounting: inner nodes 1, triangles
// 1, both weighted by area / root area).
__global__ __launch_bounds__(kBlock) void sah_kernel(const float4* __restrict__ lo, const float4* __restrict__ hi,
                                                     uint32_t nnodes, uint32_t ntri, uint32_t root,
                                                     double* __restrict__ out) {
    __shared__ double s[kBlock];
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const double ra = (double)half_area(lo[root], hi[root]);
    s[threadIdx.x] = (i < nnodes && ra > 0.0) ? (double)half_area(lo[i], hi[i]) / ra : 0.0;
    __syncthreads();
    for (uint32_t k = kBlock / 2; k > 0; k >>= 1) {
        if (threadIdx.x < k) s[threadIdx.x] += s[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicAdd(out, s[0]);
    (void)ntri;
}

// ---------------------------------------------------------------- collapse
// SAH-optimal collapse (Ylitie et al. 2017 §3.1, as bvh8_build.cpp mode 3),
// bottom-up over the PLOC nodes one merge iteration at a time (a node's
// children were made in earlier iterations).  Per inner node: cost[i-1] =
// least cost of the subtree as at most i BVH8 children (i = 1..8); take bit
// i: that is cost[i-2] (i >= 2), bit 1: as a leaf (else a BVH8 node); split
// 3 bits per i = 2..8: the left child's share of i slots.
struct DpNode {
    float cost[8];
    uint32_t split;
    uint32_t take;
};
constexpr float kCNode = 1.0f, kCPrim = (float)SPT_C_PRIM;

__device__ __forceinline__ float dp_kid_cost(const DpNode* __restrict__ dp, const float4* __restrict__ lo,
                                             const float4* __restrict__ hi, uint32_t ntri, uint32_t k, int i) {
    return k < ntri ? 2.0f * half_area(lo[k], hi[k]) * kCPrim : dp[k - ntri].cost[i - 1];
}

__global__ __launch_bounds__(kBlock) void dp_kernel(const float4* __restrict__ lo, const float4* __restrict__ hi,
                                                    const int2* __restrict__ kids2, const uint32_t* __restrict__ ntris,
                                                    uint32_t ntri, uint32_t first, uint32_t count,
                                                    DpNode* __restrict__ dp, int width) {
    const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    if (j >= count) return;
    const uint32_t n = first + j;
    const int2 c = kids2[n];
    const uint32_t l = (uint32_t)c.x, r = (uint32_t)c.y;
    float cl[9], cr[9];
    for (int i = 1; i <= 8; i++) {
        cl[i] = i <= width ? dp_kid_cost(dp, lo, hi, ntri, l, i) : INFINITY;
        cr[i] = i <= width ? dp_kid_cost(dp, lo, hi, ntri, r, i) : INFINITY;
    }
    float D[9];
    uint32_t split = 0;
    for (int i = 2; i <= 8; i++) {
        D[i] = INFINITY;
        uint32_t bs = 1;
        for (int k = 1; k < i; k++) {
            const float v = cl[k] + cr[i - k];
            if (v < D[i]) { D[i] = v; bs = (uint32_t)k; }
        }
        split |= bs << (3 * (i - 2));
    }
    const float area = 2.0f * half_area(lo[n], hi[n]);
    const float lc = ntris[n] <= kLeafMaxTris ? area * kCPrim * (float)ntris[n] : INFINITY;
    const float ic = area * kCNode + D[width];
    DpNode out;
    out.cost[0] = fminf(lc, ic);
    // a leaf only when it may be one (with overflowing areas both costs are inf)
    uint32_t take = (ntris[n] <= kLeafMaxTris && lc <= ic) ? 2u : 0u;
    for (int i = 2; i <= 8; i++) {
        if (out.cost[i - 2] <= D[i]) take |= 1u << i;
        out.cost[i - 1] = fminf(out.cost[i - 2], D[i]);
    }
    out.split = split;
    out.take = take;
    dp[n - ntri] = out;
}

struct CollapseArgs {
    const float4* lo;
    const float4* hi;
    const int2* kids2;       // BVH2 inner children (node id >= ntri)
    const uint32_t* ntris;   // triangles under each BVH2 node
    uint32_t ntri;
    const uint32_t* queue;   // BVH2 node of each BVH8 node of this level (root-leaf: a leaf id)
    uint32_t count;
    uint32_t* kids8;         // [count][8] chosen BVH2 children | kLeafKid, 0xffffffff = empty
    uint64_t* counts;        // inner << 32 | leaf triangles
    const DpNode* dp;        // SAH-optimal decisions (null: greedy collapse)
    uint32_t width;          // children per node: 8, or 6 (the 64-B device node)
};

constexpr uint32_t kLeafKid = 0x80000000u;  // kids8 flag: the child becomes a BVH8 leaf

__device__ __forceinline__ bool leafable(const CollapseArgs& a, uint32_t node) {
    return node < a.ntri || a.ntris[node] <= kLeafMaxTris;
}

// Pass A: one thread per BVH8 node of the level: the DP's distribution of the
// 8 slots (or the greedy collapse: open the largest-area child that cannot be
// a leaf while fewer than 8 children).
__global__ __launch_bounds__(kBlock) void collapse_pick_kernel(CollapseArgs a) {
    const uint32_t e = blockIdx.x * kBlock + threadIdx.x;
    if (e >= a.count) return;
    const uint32_t root = a.queue[e];
    uint32_t k[8];
    uint32_t nk = 0;
    if (root < a.ntri) {  // single-triangle scene: the root is a leaf
        k[nk++] = root | kLeafKid;
    } else if (a.dp) {
        // collect(element, slots), left child first, with an explicit stack
        uint32_t sn[8], si[8], sp = 0;
        const int2 c = a.kids2[root];
        const uint32_t s8 = (a.dp[root - a.ntri].split >> (3u * (a.width - 2u))) & 7u;
        sn[sp] = (uint32_t)c.y; si[sp++] = a.width - s8;
        sn[sp] = (uint32_t)c.x; si[sp++] = s8;
        while (sp) {
            const uint32_t x = sn[--sp];
            uint32_t i = si[sp];
            if (x < a.ntri) { k[nk++] = x | kLeafKid; continue; }
            const DpNode& d = a.dp[x - a.ntri];
            while (i > 1 && ((d.take >> i) & 1u)) i--;
            if (i == 1) { k[nk++] = x | (((d.take >> 1) & 1u) ? kLeafKid : 0u); continue; }
            const uint32_t s = (d.split >> (3 * (i - 2))) & 7u;
            const int2 cc = a.kids2[x];
            sn[sp] = (uint32_t)cc.y; si[sp++] = i - s;
            sn[sp] = (uint32_t)cc.x; si[sp++] = s;
        }
    } else {
        const int2 c = a.kids2[root];
        k[nk++] = (uint32_t)c.x;
        k[nk++] = (uint32_t)c.y;
    }
    while (!a.dp && nk < a.width && root >= a.ntri) {
        int best = -1;
        float ba = -1.0f;
        for (uint32_t i = 0; i < nk; i++)
            if (!leafable(a, k[i])) {
                const float ar = half_area(a.lo[k[i]], a.hi[k[i]]);
                if (ar > ba) { ba = ar; best = (int)i; }
            }
        if (best < 0) break;
        const int2 c = a.kids2[k[best]];
        k[best] = (uint32_t)c.x;
        k[nk++] = (uint32_t)c.y;
    }
    if (!a.dp)
        for (uint32_t i = 0; i < nk; i++)
            if (!(k[i] & kLeafKid) && leafable(a, k[i])) k[i] |= kLeafKid;
    uint32_t ninner = 0, nleaf = 0;
    for (uint32_t i = 0; i < 8; i++) {
        const uint32_t v = i < nk ? k[i] : 0xffffffffu;
        a.kids8[(size_t)e * 8 + i] = v;
        if (i < nk) {
            if (v & kLeafKid) nleaf += a.ntris[v & ~kLeafKid];
            else ninner++;
        }
    }
    a.counts[e] = ((uint64_t)ninner << 32) | nleaf;
}

struct EmitArgs {
    CollapseArgs c;
    const uint64_t* scan;     // exclusive scan of counts
    uint32_t next_first;      // BVH8 index of the next level's first node
    uint32_t tri_first;       // first triangle slot of this level
    uint32_t level_first;     // BVH8 index of this level's first node
    uint32_t* nodes8;         // kNode8Quads * 4 words per node
    uint32_t* slot2tri;
    uint32_t* next_queue;
    unsigned long long* leaves;  // leaf slots (statistics)
};

// Pass B: octant slot order, quantisation frame, node words, leaf triangles
// and the next level's queue (same arithmetic as bvh8_build.cpp emit()).
__global__ __launch_bounds__(kBlock) void collapse_emit_kernel(EmitArgs a) {
    const uint32_t e = blockIdx.x * kBlock + threadIdx.x;
    if (e >= a.c.count) return;
    uint32_t k[8];
    uint32_t nk = 0, leafbits = 0;
    for (uint32_t i = 0; i < 8; i++) {
        const uint32_t v = a.c.kids8[(size_t)e * 8 + i];
        if (v == 0xffffffffu) continue;
        if (v & kLeafKid) leafbits |= 1u << nk;
        k[nk++] = v & ~kLeafKid;
    }
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = 0; i < nk; i++) {
        const float4 l = a.c.lo[k[i]], h = a.c.hi[k[i]];
        lo[0] = fminf(lo[0], l.x); lo[1] = fminf(lo[1], l.y); lo[2] = fminf(lo[2], l.z);
        hi[0] = fmaxf(hi[0], h.x); hi[1] = fmaxf(hi[1], h.y); hi[2] = fmaxf(hi[2], h.z);
    }
    double ctr[3];
    for (int ax = 0; ax < 3; ax++) ctr[ax] = 0.5 * ((double)lo[ax] + (double)hi[ax]);
    // greedy octant assignment: repeatedly the cheapest free (kid, slot) pair
    int kid_in[8];
    for (int s = 0; s < 8; s++) kid_in[s] = -1;
    uint32_t kdone = 0;
    for (uint32_t m = 0; m < nk; m++) {
        double bc = INFINITY;
        int bk = -1, bs = -1;
        for (uint32_t i = 0; i < nk; i++) {
            if ((kdone >> i) & 1u) continue;
            const float4 l = a.c.lo[k[i]], h = a.c.hi[k[i]];
            const double d0 = 0.5 * ((double)l.x + (double)h.x) - ctr[0];
            const double d1 = 0.5 * ((double)l.y + (double)h.y) - ctr[1];
            const double d2 = 0.5 * ((double)l.z + (double)h.z) - ctr[2];
            for (int s = 0; s < 8; s++) {
                if (kid_in[s] >= 0) continue;
                const double c = ((s & 1) ? -d0 : d0) + ((s & 2) ? -d1 : d1) + ((s & 4) ? -d2 : d2);
                if (c < bc) { bc = c; bk = (int)i; bs = s; }
            }
        }
        if (bk < 0) {  // NaN costs: first free kid into the first free slot
            for (uint32_t i = 0; i < nk; i++)
                if (!((kdone >> i) & 1u)) { bk = (int)i; break; }
            for (int s = 0; s < 8; s++)
                if (kid_in[s] < 0) { bs = s; break; }
        }
        kdone |= 1u << bk;
        kid_in[bs] = bk;
    }
    const uint32_t idx = a.level_first + e;
    uint32_t* w = a.nodes8 + (size_t)idx * kNode8Quads * 4;
    int ebias[3];
    for (int ax = 0; ax < 3; ax++) {
        const double ext = (double)hi[ax] - (double)lo[ax];
        int ex = -100;
        if (!(ext <= 1e300)) {
            ex = 127;  // infinite (or NaN) extent: the widest step; such triangles are never hit
        } else if (ext > 0.0) {
            ex = (int)ceil(log2(ext / 255.0));
            while (ldexp(255.0, ex) < ext) ex++;
            ex = min(max(ex, -100), 127);
        }
        ebias[ax] = ex + 127;
        w[ax] = __builtin_bit_cast(uint32_t, lo[ax]);
    }
    const uint64_t sc = a.scan[e];
    const uint32_t child_base = a.next_first + (uint32_t)(sc >> 32);
    const uint32_t tri_base = a.tri_first + (uint32_t)(sc & 0xffffffffu);
    uint32_t imask = 0, toff = 0, r = 0, nleaves = 0;
    uint8_t meta[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint8_t q[6][8];
    for (int s = 0; s < 8; s++)
        for (int ax = 0; ax < 3; ax++) { q[ax][s] = 255; q[3 + ax][s] = 0; }  // empty: inverted
    for (int s = 0; s < 8; s++) {
        const int kk = kid_in[s];
        if (kk < 0) continue;
        const uint32_t node = k[kk];
        const float4 l = a.c.lo[node], h = a.c.hi[node];
        const float kl[3] = {l.x, l.y, l.z}, kh[3] = {h.x, h.y, h.z};
        for (int ax = 0; ax < 3; ax++) {
            const double step = ldexp(1.0, ebias[ax] - 127);
            double ql = floor(((double)kl[ax] - (double)lo[ax]) / step);
            double qh = ceil(((double)kh[ax] - (double)lo[ax]) / step);
            if (!(ql >= 0.0)) ql = 0.0;
            if (!(qh <= 255.0)) qh = 255.0;
            if (ql > 255.0) ql = 255.0;
            if (qh < 0.0) qh = 0.0;
            q[ax][s] = (uint8_t)ql;
            q[3 + ax][s] = (uint8_t)qh;
        }
        if (!((leafbits >> kk) & 1u)) {
            imask |= 1u << s;
            meta[s] = (uint8_t)(0x20u | (24u + (uint32_t)s));
            a.next_queue[child_base - a.next_first + r] = node;
            r++;
        } else {
            // the <= 3 triangles of the subtree, left to right
            uint32_t stack[4], sp = 0, cnt = 0;
            stack[sp++] = node;
            while (sp) {
                const uint32_t x = stack[--sp];
                if (x < a.c.ntri) {
                    a.slot2tri[tri_base + toff + cnt] = x;
                    cnt++;
                } else {
                    const int2 c = a.c.kids2[x];
                    stack[sp++] = (uint32_t)c.y;
                    stack[sp++] = (uint32_t)c.x;
                }
            }
            meta[s] = (uint8_t)((((1u << cnt) - 1u) << 5) | toff);
            toff += cnt;
            nleaves++;
        }
    }
    w[3] = (uint32_t)ebias[0] | ((uint32_t)ebias[1] << 8) | ((uint32_t)ebias[2] << 16) | (imask << 24);
    w[4] = imask ? child_base : 0u;
    w[5] = tri_base;
    w[6] = (uint32_t)meta[0] | ((uint32_t)meta[1] << 8) | ((uint32_t)meta[2] << 16) | ((uint32_t)meta[3] << 24);
    w[7] = (uint32_t)meta[4] | ((uint32_t)meta[5] << 8) | ((uint32_t)meta[6] << 16) | ((uint32_t)meta[7] << 24);
    for (int p = 0; p < 6; p++) {
        w[8 + 2 * p] = (uint32_t)q[p][0] | ((uint32_t)q[p][1] << 8) | ((uint32_t)q[p][2] << 16) |
                       ((uint32_t)q[p][3] << 24);
        w[9 + 2 * p] = (uint32_t)q[p][4] | ((uint32_t)q[p][5] << 8) | ((uint32_t)q[p][6] << 16) |
                       ((uint32_t)q[p][7] << 24);
    }
    for (uint32_t z = 20; z < kNode8Quads * 4; z++) w[z] = 0u;
    atomicAdd(a.leaves, (unsigned long long)nleaves);
}

template <typename T>
hipError_t dmalloc(T** p, size_t count) {
    return hipMalloc((void**)p, sizeof(T) * std::max<size_t>(count, 1));
}

struct Temp {
    std::vector<void*> ptrs;
    ~Temp() {
        for (void* p : ptrs) (void)hipFree(p);
    }
    template <typename T>
    hipError_t get(T** p, size_t count) {
        hipError_t e = dmalloc(p, count);
        if (e == hipSuccess) ptrs.push_back((void*)*p);
        return e;
    }
};

#define GB_TRY(call)                          \
    do {                                      \
        hipError_t e_ = (call);               \
        if (e_ != hipSuccess) return e_;      \
    } while (0)

// Holes layout (gpu_bvh8_holes): flag nodes with inner children; their
// exclusive scan numbers the child groups g; group g's child in octant slot s
// goes to slot (gword[g] << shift) + s — packed (shift 0: gword a slot
// index chosen on the host so that groups fill each other's holes) or
// aligned (shift 3: gword = g + 1, eight slots per group).
__global__ __launch_bounds__(kBlock) void holes_flag_kernel(const uint32_t* __restrict__ nodes, uint32_t n,
                                                            uint32_t* __restrict__ flags) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i < n) flags[i] = (nodes[(size_t)i * kNode8Quads * 4 + 3] >> 24) ? 1u : 0u;
}

__global__ __launch_bounds__(kBlock) void holes_mask_kernel(const uint32_t* __restrict__ nodes, uint32_t n,
                                                            const uint32_t* __restrict__ group,
                                                            uint8_t* __restrict__ gmask) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t imask = nodes[(size_t)i * kNode8Quads * 4 + 3] >> 24;
    if (imask) gmask[group[i]] = (uint8_t)imask;
}

__global__ __launch_bounds__(kBlock) void holes_index_kernel(const uint32_t* __restrict__ nodes, uint32_t n,
                                                             const uint32_t* __restrict__ group,
                                                             const uint32_t* __restrict__ gword, uint32_t shift,
                                                             uint32_t* __restrict__ newidx) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    if (i == 0) newidx[0] = 0u;  // the root keeps slot 0
    const uint32_t* w = nodes + (size_t)i * kNode8Quads * 4;
    const uint32_t imask = w[3] >> 24;
    if (!imask) return;
    const uint32_t base = gword[group[i]] << shift, first = w[4];
    uint32_t r = 0;
    for (uint32_t s = 0; s < 8; s++)
        if ((imask >> s) & 1u) newidx[first + r++] = base + s;  // r-th inner child sits in slot s
}

__global__ __launch_bounds__(kBlock) void holes_copy_kernel(const uint32_t* __restrict__ nodes, uint32_t n,
                                                            const uint32_t* __restrict__ group,
                                                            const uint32_t* __restrict__ gword,
                                                            const uint32_t* __restrict__ newidx,
                                                            uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint4* src = (const uint4*)(nodes + (size_t)i * kNode8Quads * 4);
    uint4* dst = (uint4*)(out + (size_t)newidx[i] * kNode8Quads * 4);
    for (uint32_t q = 0; q < kNode8Quads; q++) dst[q] = src[q];
    uint4 w1 = src[1];
    w1.x = (src[0].w >> 24) ? gword[group[i]] : 0u;  // w4: the child group's word
    dst[1] = w1;
}

// width 6: the same re-lay, each node re-encoded as the 64-B node of
// bvh_build.h — its (at most six) non-empty slots become children 0..5 in
// slot order, with their meta bytes and planes; unused children get meta 0.
// A node with more than six children sets *bad (the build used width 8).
__global__ __launch_bounds__(kBlock) void holes_copy6_kernel(const uint32_t* __restrict__ nodes, uint32_t n,
                                                             const uint32_t* __restrict__ group,
                                                             const uint32_t* __restrict__ gword,
                                                             const uint32_t* __restrict__ newidx,
                                                             uint32_t* __restrict__ out, uint32_t* __restrict__ bad) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t* w = nodes + (size_t)i * kNode8Quads * 4;
    uint32_t meta[6] = {0, 0, 0, 0, 0, 0};
    uint32_t q[6][6];  // [plane lo.x hi.x lo.y hi.y lo.z hi.z][child]
    for (int p = 0; p < 6; p++)
        for (int c = 0; c < 6; c++) q[p][c] = (p & 1) ? 0u : 255u;  // empty: inverted
    uint32_t c = 0;
    for (uint32_t s = 0; s < 8; s++) {
        const uint32_t m = (w[6 + (s >> 2)] >> ((s & 3u) * 8u)) & 0xffu;
        if (!m) continue;
        if (c == 6) { *bad = 1u; return; }
        meta[c] = m;
        for (uint32_t ax = 0; ax < 3; ax++) {
            q[2 * ax][c] = (w[8 + 2 * ax + (s >> 2)] >> ((s & 3u) * 8u)) & 0xffu;
            q[2 * ax + 1][c] = (w[14 + 2 * ax + (s >> 2)] >> ((s & 3u) * 8u)) & 0xffu;
        }
        c++;
    }
    const uint32_t ew = w[3];
    const uint32_t grp = (ew >> 24) ? gword[group[i]] : 0u;  // the child group's word
    uint32_t o[16];
    o[0] = w[0]; o[1] = w[1]; o[2] = w[2];
    o[3] = w[5];
    o[4] = meta[0] | meta[1] << 8 | meta[2] << 16 | meta[3] << 24;
    o[5] = meta[4] | meta[5] << 8 | (ew & 0xffu) << 16 | ((ew >> 8) & 0xffu) << 24;
    o[6] = grp | ((ew >> 16) & 0xffu) << 24;
    for (uint32_t p = 0; p < 6; p++) o[7 + p] = q[p][0] | q[p][1] << 8 | q[p][2] << 16 | q[p][3] << 24;
    for (uint32_t ax = 0; ax < 3; ax++)
        o[13 + ax] = q[2 * ax][4] | q[2 * ax][5] << 8 | q[2 * ax + 1][4] << 16 | q[2 * ax + 1][5] << 24;
    uint4* dst = (uint4*)(out + (size_t)newidx[i] * kNode6Quads * 4);
    for (uint32_t k = 0; k < 4; k++) dst[k] = make_uint4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
}

}  // namespace

// Packed group bases (host, first fit over a slot bitmap): each group, in
// order, takes the lowest base at which its occupied octant slots are all
// free, so the slots left empty by one group's leaf children hold other
// groups' nodes.  The search starts no further back than kPackWindow slots
// behind the packed end (holes older than that are given up), so it is
// linear in the group count.  Returns the slot count, 0 if it would not fit
// 24 bits.
constexpr size_t kPackWindow = 64;
static size_t pack_groups(const std::vector<uint8_t>& gmask, std::vector<uint32_t>& gword) {
    std::vector<uint64_t> used(2, 0u);
    used[0] = 1u;  // slot 0: the root
    const auto window = [&](size_t x) -> uint32_t {  // used bits of slots x .. x + 7
        const size_t w = x / 64, o = x % 64;
        uint64_t v = used[w] >> o;
        if (o) v |= used[w + 1] << (64 - o);
        return (uint32_t)(v & 0xffu);
    };
    size_t lo = 1, end = 1;
    gword.resize(gmask.size());
    for (size_t g = 0; g < gmask.size(); g++) {
        const uint32_t m = gmask[g];
        if (end > lo + kPackWindow) lo = end - kPackWindow;  // give up the old holes
        while (window(lo) & 1u) lo++;
        const size_t c = (size_t)__builtin_ctz(m | 0x100u);
        size_t b = lo > c ? lo - c : 1;
        while (window(b) & m) b++;
        if (b + 8 >= (1u << 24)) return 0;
        gword[g] = (uint32_t)b;
        if ((b + 8) / 64 + 2 > used.size()) used.resize((b + 8) / 64 + 2, 0u);
        const size_t w = b / 64, o = b % 64;
        used[w] |= (uint64_t)m << o;
        if (o > 56) used[w + 1] |= (uint64_t)m >> (64 - o);
        end = std::max(end, b + 8 - (size_t)__builtin_clz(m) + 24);  // one past the highest occupied slot
    }
    return end;
}

// Group ids in depth-first order from the root: group g holds the inner
// children of the g-th node (in node order) that has any; a node's inner
// children are nodes w4 .. w4 + popcount(imask) - 1 (compact layout).
static std::vector<uint32_t> depth_first_groups(const std::vector<uint32_t>& w34, uint32_t n, uint32_t groups) {
    std::vector<uint32_t> gid(n, UINT32_MAX);
    for (uint32_t i = 0, g = 0; i < n; i++)
        if (w34[2 * i] >> 24) gid[i] = g++;
    std::vector<uint32_t> order;
    order.reserve(groups);
    std::vector<uint32_t> stack{0u};
    while (!stack.empty()) {
        const uint32_t i = stack.back();
        stack.pop_back();
        const uint32_t imask = w34[2 * i] >> 24;
        if (!imask || i >= n) continue;
        order.push_back(gid[i]);
        const uint32_t first = w34[2 * i + 1], cnt = (uint32_t)__builtin_popcount(imask);
        for (uint32_t c = cnt; c-- > 0;)  // first child on top: visited first
            if (first + c < n) stack.push_back(first + c);
    }
    // groups the walk did not reach (none in a well-formed tree) keep build order
    if (order.size() != groups) {
        std::vector<uint8_t> seen(groups, 0);
        for (uint32_t g : order) seen[g] = 1;
        for (uint32_t g = 0; g < groups; g++)
            if (!seen[g]) order.push_back(g);
    }
    return order;
}

hipError_t gpu_bvh8_holes(const uint32_t* d_nodes, uint32_t n, hipStream_t s, uint32_t** out, uint32_t* nslots,
                          int width, uint32_t* group_shift, bool depth_first) {
    *out = nullptr;
    *nslots = 0;
    if (group_shift) *group_shift = 3;
    Temp tmp;
    uint32_t *flags, *group, *newidx, *bad;
    const uint32_t quads = width == 6 ? kNode6Quads : kNode8Quads;
    GB_TRY(tmp.get(&bad, 1));
    GB_TRY(hipMemsetAsync(bad, 0, sizeof(uint32_t), s));
    GB_TRY(tmp.get(&flags, n));
    GB_TRY(tmp.get(&group, n));
    GB_TRY(tmp.get(&newidx, n));
    uint32_t groups = 0;
    if (n) {
        hipLaunchKernelGGL(holes_flag_kernel, dim3(blocks(n)), dim3(kBlock), 0, s, d_nodes, n, flags);
        GB_TRY(hipGetLastError());
        size_t bytes = 0;
        GB_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, flags, group, (int)n, s));
        char* ws = nullptr;
        GB_TRY(tmp.get(&ws, bytes));
        GB_TRY(hipcub::DeviceScan::ExclusiveSum((void*)ws, bytes, flags, group, (int)n, s));
        uint32_t last[2] = {0u, 0u};
        GB_TRY(hipMemcpyAsync(&last[0], group + n - 1, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        GB_TRY(hipMemcpyAsync(&last[1], flags + n - 1, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        GB_TRY(hipStreamSynchronize(s));
        groups = last[0] + last[1];
    }
    // group words: packed bases when a caller takes the shift, else aligned groups
    std::vector<uint32_t> gw(groups);
    size_t slots = 0;
    uint32_t shift = 3;
    if (group_shift && groups) {
        uint8_t* gmask = nullptr;
        GB_TRY(tmp.get(&gmask, groups));
        hipLaunchKernelGGL(holes_mask_kernel, dim3(blocks(n)), dim3(kBlock), 0, s, d_nodes, n, group, gmask);
        GB_TRY(hipGetLastError());
        std::vector<uint8_t> hm(groups);
        GB_TRY(hipMemcpyAsync(hm.data(), gmask, groups, hipMemcpyDeviceToHost, s));
        GB_TRY(hipStreamSynchronize(s));
        if (depth_first) {
            // words 3 (inner mask) and 4 (first inner child) of every node
            std::vector<uint32_t> w34(2 * (size_t)n);
            GB_TRY(hipMemcpy2DAsync(w34.data(), 8, d_nodes + 3, kNode8Quads * 16, 8, n, hipMemcpyDeviceToHost, s));
            GB_TRY(hipStreamSynchronize(s));
            const std::vector<uint32_t> order = depth_first_groups(w34, n, groups);
            std::vector<uint8_t> pm(groups);
            for (uint32_t k = 0; k < groups; k++) pm[k] = hm[order[k]];
            std::vector<uint32_t> pw;
            slots = pack_groups(pm, pw);
            for (uint32_t k = 0; k < groups && slots; k++) gw[order[k]] = pw[k];
        } else {
            slots = pack_groups(hm, gw);
        }
        if (slots) shift = 0;
    }
    if (shift) {
        if (groups >= (1u << 24)) return hipErrorInvalidValue;  // the group word must fit the 24-bit stack field
        for (uint32_t g = 0; g < groups; g++) gw[g] = g + 1u;
        slots = 8 * ((size_t)groups + 1);
    }
    if (slots == 0) slots = 1;
    uint32_t* gword = nullptr;
    GB_TRY(tmp.get(&gword, groups));
    if (groups) GB_TRY(hipMemcpyAsync(gword, gw.data(), sizeof(uint32_t) * groups, hipMemcpyHostToDevice, s));
    uint32_t* o = nullptr;
    GB_TRY(dmalloc(&o, slots * quads * 4));
    hipError_t e = hipMemsetAsync(o, 0, slots * quads * 16, s);
    if (!e && n) {
        hipLaunchKernelGGL(holes_index_kernel, dim3(blocks(n)), dim3(kBlock), 0, s, d_nodes, n, group, gword, shift,
                           newidx);
        if (width == 6)
            hipLaunchKernelGGL(holes_copy6_kernel, dim3(blocks(n)), dim3(kBlock), 0, s, d_nodes, n, group, gword,
                               newidx, o, bad);
        else
            hipLaunchKernelGGL(holes_copy_kernel, dim3(blocks(n)), dim3(kBlock), 0, s, d_nodes, n, group, gword,
                               newidx, o);
        e = hipGetLastError();
    }
    if (!e) e = hipStreamSynchronize(s);
    if (!e && width == 6) {
        uint32_t hb = 0;
        e = hipMemcpy(&hb, bad, sizeof(hb), hipMemcpyDeviceToHost);
        if (!e && hb) e = hipErrorInvalidValue;  // a node with more than six children
    }
    if (e) {
        (void)hipFree(o);
        return e;
    }
    *out = o;
    *nslots = (uint32_t)slots;
    if (group_shift) *group_shift = shift;
    return hipSuccess;
}

hipError_t gpu_build_bvh8(const float* d_tv, uint32_t ntri, hipStream_t s, GpuBvh8* out, int radius, bool greedy,
                          int width) {
    width = width == 6 ? 6 : 8;
    *out = GpuBvh8();
    if (ntri == 0) return hipSuccess;
    const auto t0 = std::chrono::steady_clock::now();
    Temp tmp;
    const uint32_t nnodes = 2 * ntri - 1;
    float4 *lo, *hi, *clo[2], *chi[2];
    int2* kids2;
    uint32_t *ntris, *cnode[2], *nn, *cb, *vals[2];
    uint64_t *keys[2], *flags, *scan, *total;
    unsigned long long* leaves;
    double* sah;
    GB_TRY(tmp.get(&lo, nnodes));
    GB_TRY(tmp.get(&hi, nnodes));
    GB_TRY(tmp.get(&kids2, nnodes));
    GB_TRY(tmp.get(&ntris, nnodes));
    for (int b = 0; b < 2; b++) {
        GB_TRY(tmp.get(&clo[b], ntri));
        GB_TRY(tmp.get(&chi[b], ntri));
        GB_TRY(tmp.get(&cnode[b], ntri));
        GB_TRY(tmp.get(&keys[b], ntri));
        GB_TRY(tmp.get(&vals[b], ntri));
    }
    GB_TRY(tmp.get(&nn, ntri));
    GB_TRY(tmp.get(&flags, ntri));
    GB_TRY(tmp.get(&scan, ntri));
    GB_TRY(tmp.get(&total, 2));
    GB_TRY(tmp.get(&cb, 6));
    GB_TRY(tmp.get(&sah, 1));
    GB_TRY(tmp.get(&leaves, 1));
    GB_TRY(hipMemsetAsync(leaves, 0, sizeof(unsigned long long), s));

    // leaves, Morton order
    const uint32_t cb_init[6] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u};
    GB_TRY(hipMemcpyAsync(cb, cb_init, sizeof(cb_init), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(tri_box_kernel, dim3(blocks(ntri)), dim3(kBlock), 0, s, d_tv, ntri, lo, hi, cb);
    hipLaunchKernelGGL(morton_kernel, dim3(blocks(ntri)), dim3(kBlock), 0, s, lo, hi, ntri, cb, keys[0], vals[0]);
    GB_TRY(hipGetLastError());
    {
        hipcub::DoubleBuffer<uint64_t> dk(keys[0], keys[1]);
        hipcub::DoubleBuffer<uint32_t> dv(vals[0], vals[1]);
        size_t bytes = 0;
        GB_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, dk, dv, (int)ntri, 0, 63, s));
        void* ws = nullptr;
        GB_TRY(tmp.get((char**)&ws, bytes));
        GB_TRY(hipcub::DeviceRadixSort::SortPairs(ws, bytes, dk, dv, (int)ntri, 0, 63, s));
        hipLaunchKernelGGL(init_clusters_kernel, dim3(blocks(ntri)), dim3(kBlock), 0, s, dv.Current(), ntri, lo, hi,
                           cnode[0], clo[0], chi[0]);
    }
    hipLaunchKernelGGL(leaf_ones_kernel, dim3(blocks(ntri)), dim3(kBlock), 0, s, ntris, ntri);  // 1 tri per leaf
    GB_TRY(hipGetLastError());

    // PLOC iterations (search radius 8, 16, 32 or 64: spt_config.ploc_radius)
    size_t scan_bytes = 0;
    GB_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, flags, scan, (int)ntri, s));
    void* scan_ws = nullptr;
    GB_TRY(tmp.get((char**)&scan_ws, scan_bytes));
    uint32_t n = ntri, cur = 0, node_base = ntri, iters = 0;
    uint64_t tot = 0;
    std::vector<std::pair<uint32_t, uint32_t>> made;  // inner nodes made per iteration (first, count)
    while (n > 1) {
        switch (radius) {
            case 8: hipLaunchKernelGGL(nn_kernel<8>, dim3(blocks(n)), dim3(kBlock), 0, s, clo[cur], chi[cur], n, nn); break;
            case 32: hipLaunchKernelGGL(nn_kernel<32>, dim3(blocks(n)), dim3(kBlock), 0, s, clo[cur], chi[cur], n, nn); break;
            case 64: hipLaunchKernelGGL(nn_kernel<64>, dim3(blocks(n)), dim3(kBlock), 0, s, clo[cur], chi[cur], n, nn); break;
            default: hipLaunchKernelGGL(nn_kernel<16>, dim3(blocks(n)), dim3(kBlock), 0, s, clo[cur], chi[cur], n, nn);
        }
        hipLaunchKernelGGL(merge_flags_kernel, dim3(blocks(n)), dim3(kBlock), 0, s, nn, n, flags);
        GB_TRY(hipGetLastError());
        GB_TRY(hipcub::DeviceScan::ExclusiveSum(scan_ws, scan_bytes, flags, scan, (int)n, s));
        hipLaunchKernelGGL(merge_compact_kernel, dim3(blocks(n)), dim3(kBlock), 0, s, nn, flags, scan, n, node_base,
                           cnode[cur], clo[cur], chi[cur], cnode[1 - cur], clo[1 - cur], chi[1 - cur], lo, hi, kids2,
                           ntris);
        hipLaunchKernelGGL(scan_total_kernel, dim3(1), dim3(1), 0, s, flags, scan, n, total);
        GB_TRY(hipGetLastError());
        GB_TRY(hipMemcpyAsync(&tot, total, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        GB_TRY(hipStreamSynchronize(s));
        const uint32_t merged = (uint32_t)(tot >> 32), kept = (uint32_t)(tot & 0xffffffffu);
        if (merged == 0) return hipErrorUnknown;  // cannot happen (see nn_kernel)
        made.push_back({node_base, merged});
        node_base += merged;
        n = kept;
        cur = 1 - cur;
        iters++;
    }
    uint32_t root = 0;
    GB_TRY(hipMemcpyAsync(&root, cnode[cur], sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    GB_TRY(hipMemsetAsync(sah, 0, sizeof(double), s));
    hipLaunchKernelGGL(sah_kernel, dim3(blocks(nnodes)), dim3(kBlock), 0, s, lo, hi, nnodes, ntri, root, sah);
    GB_TRY(hipGetLastError());
    GB_TRY(hipMemcpyAsync(&out->sah_cost, sah, sizeof(double), hipMemcpyDeviceToHost, s));
    GB_TRY(hipStreamSynchronize(s));
    out->bvh2_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    out->ploc_iterations = iters;

    // SAH-optimal collapse decisions, bottom-up by merge iteration
    // (spt_config.collapse = 1 keeps the greedy collapse)
    DpNode* dp = nullptr;
    if (!greedy && ntri > 1) {
        GB_TRY(tmp.get(&dp, ntri - 1));
        for (const auto& m : made)
            hipLaunchKernelGGL(dp_kernel, dim3(blocks(m.second)), dim3(kBlock), 0, s, lo, hi, kids2, ntris, ntri,
                               m.first, m.second, dp, width);
        GB_TRY(hipGetLastError());
    }

    // Collapse, level by level.  At most ntri BVH8 nodes (every node holds
    // at least two children or is the single root).
    uint32_t *queue[2], *kids8, *nodes8, *slot2tri;
    uint64_t* counts;
    const size_t max8 = std::max<size_t>(1, ntri);
    GB_TRY(tmp.get(&queue[0], max8));
    GB_TRY(tmp.get(&queue[1], max8));
    GB_TRY(tmp.get(&kids8, max8 * 8));
    GB_TRY(tmp.get(&counts, max8));
    GB_TRY(dmalloc(&nodes8, max8 * kNode8Quads * 4));
    GB_TRY(dmalloc(&slot2tri, ntri));
    GB_TRY(hipMemcpyAsync(queue[0], &root, sizeof(uint32_t), hipMemcpyHostToDevice, s));
    uint32_t count = 1, level_first = 0, next_first = 1, tri_first = 0, depth = 0, q = 0;
    size_t scan8_bytes = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan8_bytes, counts, scan, (int)max8, s);
    void* scan8_ws = nullptr;
    hipError_t err = tmp.get((char**)&scan8_ws, scan8_bytes);
    while (err == hipSuccess && count > 0) {
        CollapseArgs c{lo, hi, kids2, ntris, ntri, queue[q], count, kids8, counts, dp, (uint32_t)width};
        hipLaunchKernelGGL(collapse_pick_kernel, dim3(blocks(count)), dim3(kBlock), 0, s, c);
        if ((err = hipGetLastError())) break;
        if ((err = hipcub::DeviceScan::ExclusiveSum(scan8_ws, scan8_bytes, counts, scan, (int)count, s))) break;
        EmitArgs ea{c, scan, next_first, tri_first, level_first, nodes8, slot2tri, queue[1 - q], leaves};
        hipLaunchKernelGGL(collapse_emit_kernel, dim3(blocks(count)), dim3(kBlock), 0, s, ea);
        hipLaunchKernelGGL(scan_total_kernel, dim3(1), dim3(1), 0, s, counts, scan, count, total);
        if ((err = hipGetLastError())) break;
        if ((err = hipMemcpyAsync(&tot, total, sizeof(uint64_t), hipMemcpyDeviceToHost, s))) break;
        if ((err = hipStreamSynchronize(s))) break;
        depth++;
        level_first = next_first;
        count = (uint32_t)(tot >> 32);
        next_first += count;
        tri_first += (uint32_t)(tot & 0xffffffffu);
        q = 1 - q;
    }
    if (err == hipSuccess && tri_first != ntri) err = hipErrorUnknown;  // every triangle in exactly one leaf
    if (err != hipSuccess) {
        (void)hipFree(nodes8);
        (void)hipFree(slot2tri);
        return err;
    }
    unsigned long long nleaves = 0;
    (void)hipMemcpy(&nleaves, leaves, sizeof(nleaves), hipMemcpyDeviceToHost);
    out->leaves = nleaves;
    out->nodes8 = nodes8;
    out->slot2tri = slot2tri;
    out->nnodes = level_first;  // == next_first after the last (empty) level
    out->depth = depth;
    out->build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return hipSuccess;
}

}  // namespace spt

namespace spt {
namespace {

__global__ __launch_bounds__(kBlock) void mesh_soup_kernel(DeviceMeshIn m, float* __restrict__ tv) {
    const uint32_t t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= m.ntri) return;
    for (int k = 0; k < 3; k++) {
        const int64_t pi = m.pos_tri[(size_t)t * 3 + k];
        for (int c = 0; c < 3; c++) tv[(size_t)t * 9 + k * 3 + c] = m.pos[pi * 3 + c];
    }
}

__global__ __launch_bounds__(kBlock) void scene_slots_kernel(DeviceMeshIn m, const float* __restrict__ tv,
                                                             const uint32_t* __restrict__ slot2tri,
                                                             float4* __restrict__ tris, float4* __restrict__ snrm,
                                                             float* __restrict__ tc, int32_t* __restrict__ o2s) {
    const uint32_t sl = blockIdx.x * kBlock + threadIdx.x;
    if (sl >= m.ntri) return;
    const uint32_t t = slot2tri[sl];
    o2s[t] = (int32_t)sl;
    const float* v = tv + (size_t)t * 9;
    float rec[kTriFloats];
    tri_record_fill(rec, v, t);
    for (int k = 0; k < 4; k++)
        tris[(size_t)sl * kTriQuads + k] = make_float4(rec[4 * k], rec[4 * k + 1], rec[4 * k + 2], rec[4 * k + 3]);
    // geometric normal fallback for a missing vertex normal (as spt_scene_create's host loop)
    const V3 g = normalize(cross(v3(v[3] - v[0], v[4] - v[1], v[5] - v[2]), v3(v[6] - v[0], v[7] - v[1], v[8] - v[2])));
    const int32_t mat = m.mat_id ? m.mat_id[t] : 0;
    for (int k = 0; k < 3; k++) {
        const int64_t ni = m.nrm_tri ? m.nrm_tri[(size_t)t * 3 + k] : -1;
        const V3 nv = ni >= 0 ? v3(m.nrm[ni * 3], m.nrm[ni * 3 + 1], m.nrm[ni * 3 + 2]) : g;
        snrm[(size_t)sl * 3 + k] = make_float4(nv.x, nv.y, nv.z, k == 0 ? __builtin_bit_cast(float, mat) : 0.0f);
    }
    if (tc)
        for (int k = 0; k < 3; k++) {
            const int64_t ti = m.tc_tri[(size_t)t * 3 + k];
            tc[(size_t)sl * 6 + k * 2] = ti >= 0 ? m.tc[ti * 2] : 0.0f;
            tc[(size_t)sl * 6 + k * 2 + 1] = ti >= 0 ? m.tc[ti * 2 + 1] : 0.0f;
        }
}

}  // namespace

hipError_t gpu_mesh_soup(const DeviceMeshIn& m, float* tv, hipStream_t s) {
    if (m.ntri == 0) return hipSuccess;
    hipLaunchKernelGGL(mesh_soup_kernel, dim3(blocks(m.ntri)), dim3(kBlock), 0, s, m, tv);
    return hipGetLastError();
}

hipError_t gpu_scene_slots(const DeviceMeshIn& m, const float* tv, const uint32_t* slot2tri, float4* tris,
                           float4* snrm, float* tc, int32_t* orig2slot, hipStream_t s) {
    if (m.ntri == 0) return hipSuccess;
    hipLaunchKernelGGL(scene_slots_kernel, dim3(blocks(m.ntri)), dim3(kBlock), 0, s, m, tv, slot2tri, tris, snrm,
                       tc, orig2slot);
    return hipGetLastError();
}

}  // namespace spt
