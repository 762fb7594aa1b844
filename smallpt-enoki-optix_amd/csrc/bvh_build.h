// bvh_build.h — host binned-SAH BVH2 builder.
//
// Replaces the OptiX GAS build (optixAccelBuild + optixAccelCompact,
// optix_backend.h:283-364).  Output layout (64 B per node, 4 x float4) keeps
// both children's boxes in the parent so one node fetch tests two boxes:
//   [0] c0.lo.x c0.hi.x c0.lo.y c0.hi.y
//   [1] c1.lo.x c1.hi.x c1.lo.y c1.hi.y
//   [2] c0.lo.z c0.hi.z c1.lo.z c1.hi.z
//   [3] c0 code, c1 code (int32 bits), 0, 0
// child code >= 0: inner node index; < 0: leaf ~(first_slot << 3 | (count-1)).
#pragma once
#include <cstdint>
#include <vector>

namespace spt {

constexpr uint32_t kMaxLeafSize = 8;    // 3 count bits in the leaf code
// SAH cost of one triangle test relative to one wide-node visit in the
// collapse's dynamic program.  Ylitie et al. 2017 use 0.3; here a triangle
// test is ~120 VALU against ~185 for a six-child visit, and 1.0 (smaller
// leaves: 2.20 instead of 2.47 tests and 7.60 instead of 7.70 visits per ray)
// measured +1.8 % on config 1 and neutral on configs 2 and 4 (0.15 / 0.6 /
// 1.5 / 2.5: profiles/r02_v6/cprim_ab.log).
#ifndef SPT_C_PRIM
#define SPT_C_PRIM 1.0
#endif
constexpr uint32_t kMaxTriangles = 1u << 28;

struct BvhBuildResult {
    std::vector<float> nodes;        // 16 floats per node
    std::vector<uint32_t> slot2tri;  // leaf order slot -> original triangle id
    uint32_t max_depth = 0;          // deepest leaf (root = 0)
    uint64_t leaves = 0;
    uint32_t max_leaf = 0;
    double sah_cost = 0.0;
};

// tri_verts: ntri x 9 floats (v0 v1 v2).  ntri == 0 gives an empty result.
// Leaves hold at most max_leaf (<= kMaxLeafSize) triangles.
BvhBuildResult build_bvh(const float* tri_verts, uint64_t ntri, uint32_t max_leaf = kMaxLeafSize);

// Compressed 8-wide BVH (80 B per node = 20 words, see kernels.hip Tracer8):
//   w0-2  p.xyz        quantisation origin (f32)
//   w3    ex | ey<<8 | ez<<16 | imask<<24   (biased exponents; imask: inner slots)
//   w4    child_base   first inner child (inner children are contiguous, slot order);
//                      on the device (gpu_bvh8_holes) w4 is the child-group word and
//                      child s sits at (w4 << group_shift) + s
//   w5    tri_base     first triangle slot of this node's leaves (contiguous)
//   w6-7  meta[8]      0 empty; inner 0b001_(24+s); leaf unary(count)<<5 | offset
//   w8-9  qlo.x[8]  w10-11 qlo.y[8]  w12-13 qlo.z[8]
//   w14-15 qhi.x[8] w16-17 qhi.y[8]  w18-19 qhi.z[8]
// Child slots are ordered by ray octant (slot s is nearest for octant s).
struct Bvh8BuildResult {
    std::vector<uint32_t> nodes;     // 20 words per node
    std::vector<uint32_t> slot2tri;  // triangle slot -> original triangle id
    uint32_t depth = 0;              // deepest node level (root = 1)
    uint64_t leaves = 0;
    double sah_cost = 0.0;           // of the underlying BVH2
};
// greedy: the greedy collapse instead of the SAH-optimal dynamic program.
// width: at most 8 children per node, or 6 (the 64-B device node below).
Bvh8BuildResult build_bvh8(const float* tri_verts, uint64_t ntri, bool greedy = false, int width = 8);

// 64-B device node (gpu_bvh8_holes with width 6; kernels.hip Tracer8T<..., 6>):
// at most six children, physical index p in slot order; one 64-B half-line
// per visit instead of the 80-B node's two.  16 words:
//   w0-2  p.xyz        quantisation origin (f32)
//   w3    tri_base
//   w4    meta[0..3]   (as above: inner 0b001_(24+s) with s its octant slot)
//   w5    meta[4] | meta[5]<<8 | ex<<16 | ey<<24
//   w6    group | ez<<24    group word (child s at (group << group_shift) + s)
//   w7-12 qlo.x qhi.x qlo.y qhi.y qlo.z qhi.z of children 0..3 (one byte each)
//   w13-15 per axis x, y, z: lo4 | lo5<<8 | hi4<<16 | hi5<<24

}  // namespace spt
