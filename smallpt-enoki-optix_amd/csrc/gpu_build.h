// gpu_build.h — acceleration structure built on the GPU (gpu_build.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace spt {

struct GpuBvh8 {
    uint32_t* nodes8 = nullptr;    // device, kNode8Quads * 4 words per node (bvh_build.h layout)
    uint32_t* slot2tri = nullptr;  // device, triangle slot -> original triangle id
    uint32_t nnodes = 0;
    uint32_t depth = 0;            // deepest node level (root = 1)
    uint64_t leaves = 0;
    uint32_t ploc_iterations = 0;
    double sah_cost = 0.0;         // of the BVH2 (bvh_build.cpp accounting)
    double bvh2_ms = 0.0;          // PLOC part
    double build_ms = 0.0;         // whole build (host wall time, synchronised)
};

// d_tv: device, ntri x 9 floats (v0 v1 v2).  On success the caller owns
// out->nodes8 and out->slot2tri (hipFree).  Synchronises stream s.
// radius: PLOC search radius (8, 16, 32 or 64); greedy: greedy collapse
// instead of the SAH-optimal one; width: at most 8 or 6 children per node.
hipError_t gpu_build_bvh8(const float* d_tv, uint32_t ntri, hipStream_t s, GpuBvh8* out, int radius = 16,
                          bool greedy = false, int width = 8);

// Re-lays a compact BVH8 (both builders' output: nnodes nodes of kNode8Quads
// quads, the inner children of a node contiguous from w4 in slot order) so
// that every child sits at a fixed offset from its group: child s of a node
// at (group word << shift) + s, the slots of leaf and empty children left to
// other groups or unused ("holes").  The traversal then finds a child without
// a popcount and keeps one word per stack entry (hit bits + group word).
// Root stays at slot 0.  On
// success the caller owns *out (device, *nslots nodes).  Synchronises s.
// width 6: every node has at most six children and is re-encoded as the
// 64-B node of bvh_build.h (kNode6Quads quads per slot); else copied as is
// (kNode8Quads quads per slot).  group_shift non-null: the groups are packed
// into each other's holes (a node's group word is its first child slot,
// *group_shift = 0) when that fits 24 bits, else aligned (group word = slot /
// 8, *group_shift = 3); null: aligned.  Child s of a node sits at
// (group word << shift) + s.  depth_first: the groups are packed in the
// order a depth-first walk from the root meets them (children in slot order)
// instead of build order, so a subtree's groups lie near each other.
hipError_t gpu_bvh8_holes(const uint32_t* d_nodes, uint32_t nnodes, hipStream_t s, uint32_t** out,
                          uint32_t* nslots, int width = 8, uint32_t* group_shift = nullptr,
                          bool depth_first = false);

}  // namespace spt

namespace spt {

// Raw indexed mesh on the device (spt_scene_create's arrays, uploaded as is).
struct DeviceMeshIn {
    const int32_t* pos_tri;  // 3 per triangle
    const float* pos;        // 3 per vertex
    const int32_t* nrm_tri;  // 3 per triangle or null (-1 = missing: geometric normal)
    const float* nrm;
    const int32_t* tc_tri;   // 3 per triangle or null
    const float* tc;
    const int32_t* mat_id;   // per triangle or null (material 0)
    uint32_t ntri;
};

// Triangle soup (ntri x 9 floats) from the indexed mesh.
hipError_t gpu_mesh_soup(const DeviceMeshIn& m, float* tv, hipStream_t s);

// Slot-ordered scene arrays from the build's slot2tri (the device side of
// spt_scene_create's host loop): tris 3 x float4 per slot (v + original id
// bits), snrm 3 x float4 (normals + material id bits), tc 6 floats per slot
// (may be null), orig2slot.
hipError_t gpu_scene_slots(const DeviceMeshIn& m, const float* tv, const uint32_t* slot2tri, float4* tris,
                           float4* snrm, float* tc, int32_t* orig2slot, hipStream_t s);

}  // namespace spt
