// bvh_build.cpp — host binned-SAH BVH2 builder (see bvh_build.h).
#include "bvh_build.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <future>
#include <limits>

namespace spt {
namespace {

// 64 / 256 bins lower config 1's BVH2 SAH by up to 2 % yet render 0.5-1.2 % slower
// (profiles/r02_v6/sah_bins_ab.log); an exact sweep below 256 triangles changes nothing
#ifndef SPT_SAH_BINS
#define SPT_SAH_BINS 32
#endif
constexpr int kBins = SPT_SAH_BINS;
constexpr uint32_t kSahDepthLimit = 48;  // below this depth: object-median splits
constexpr float kNodeCost = 1.0f;
constexpr float kTriCost = 1.0f;
constexpr uint64_t kParallelGrain = 1u << 15;  // subtrees this large build on their own thread

struct Box {
    float lo[3], hi[3];
    void reset() {
        for (int k = 0; k < 3; k++) { lo[k] = std::numeric_limits<float>::infinity(); hi[k] = -lo[k]; }
    }
    void grow(const float* l, const float* h) {
        for (int k = 0; k < 3; k++) { lo[k] = std::fmin(lo[k], l[k]); hi[k] = std::fmax(hi[k], h[k]); }
    }
    void grow(const Box& b) { grow(b.lo, b.hi); }
    void grow_pt(const float* p) { grow(p, p); }
    bool empty() const { return !(lo[0] <= hi[0]); }
    float area() const {
        if (empty()) return 0.0f;
        float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return 2.0f * (dx * dy + dy * dz + dz * dx);
    }
};

struct PrimRef {
    float lo[3], hi[3], c[3];
    uint32_t id;
};

// A subtree built into its own node list; node indices are local and get
// rebased when the subtree is spliced into its parent's list.
struct SubTree {
    std::vector<float> nodes;  // 16 floats per node
    uint32_t max_depth = 0;
    uint64_t leaves = 0;
    uint32_t max_leaf = 0;
    double sah = 0.0;
};

int32_t leaf_code(uint64_t first, uint64_t count) {
    return (int32_t)~(uint32_t)((first << 3) | (count - 1));
}

struct Builder {
    PrimRef* refs;
    double root_area_inv;
    uint32_t max_leaf;

    // Returns the child code of range [b, e) and its box; inner nodes are
    // appended to st.nodes in depth-first order (parent before children).
    int32_t build(SubTree& st, uint64_t b, uint64_t e, uint32_t depth, Box& out_box, bool allow_async) {
        Box box, cbox;
        box.reset();
        cbox.reset();
        for (uint64_t i = b; i < e; i++) {
            box.grow(refs[i].lo, refs[i].hi);
            cbox.grow_pt(refs[i].c);
        }
        out_box = box;
        uint64_t n = e - b;
        double area_ratio = (double)box.area() * root_area_inv;
        auto make_leaf = [&]() {
            st.leaves++;
            st.max_depth = std::max(st.max_depth, depth);
            st.max_leaf = std::max(st.max_leaf, (uint32_t)n);
            st.sah += area_ratio * kTriCost * (double)n;
            return leaf_code(b, n);
        };
        if (n <= 1) return make_leaf();

        uint64_t mid = b + n / 2;
        bool split_found = false;
        float best_cost = std::numeric_limits<float>::infinity();
        int best_axis = -1, best_bin = -1;
        float ext[3];
        for (int k = 0; k < 3; k++) ext[k] = cbox.hi[k] - cbox.lo[k];

        if (depth < kSahDepthLimit) {
            for (int axis = 0; axis < 3; axis++) {
                if (!(ext[axis] > 0.0f)) continue;
                float scale = (float)kBins * (1.0f - 1e-6f) / ext[axis];
                uint32_t cnt[kBins] = {0};
                Box bb[kBins];
                for (int i = 0; i < kBins; i++) bb[i].reset();
                for (uint64_t i = b; i < e; i++) {
                    float f = (refs[i].c[axis] - cbox.lo[axis]) * scale;
                    int bin = (f >= 0.0f) ? std::min((int)f, kBins - 1) : 0;
                    cnt[bin]++;
                    bb[bin].grow(refs[i].lo, refs[i].hi);
                }
                float right_area[kBins];
                uint32_t right_cnt[kBins];
                Box acc;
                acc.reset();
                uint32_t c = 0;
                for (int i = kBins - 1; i > 0; i--) {
                    acc.grow(bb[i]);
                    c += cnt[i];
                    right_area[i] = acc.area();
                    right_cnt[i] = c;
                }
                acc.reset();
                c = 0;
                for (int i = 0; i < kBins - 1; i++) {
                    acc.grow(bb[i]);
                    c += cnt[i];
                    if (c == 0 || right_cnt[i + 1] == 0) continue;
                    float cost = acc.area() * (float)c + right_area[i + 1] * (float)right_cnt[i + 1];
                    if (cost < best_cost) { best_cost = cost; best_axis = axis; best_bin = i; }
                }
            }
            if (best_axis >= 0) {
                float parent_area = box.area();
                float split_cost = kNodeCost + (parent_area > 0.0f ? best_cost / parent_area : 0.0f) * kTriCost;
                float leaf_cost = (float)n * kTriCost;
                if (n <= max_leaf && leaf_cost <= split_cost) return make_leaf();
                int axis = best_axis;
                float scale = (float)kBins * (1.0f - 1e-6f) / ext[axis];
                float lo = cbox.lo[axis];
                PrimRef* m = std::partition(refs + b, refs + e, [&](const PrimRef& r) {
                    float f = (r.c[axis] - lo) * scale;
                    int bin = (f >= 0.0f) ? std::min((int)f, kBins - 1) : 0;
                    return bin <= best_bin;
                });
                mid = (uint64_t)(m - refs);
                split_found = mid > b && mid < e;
            }
        }
        if (!split_found) {
            if (n <= max_leaf && depth >= kSahDepthLimit) return make_leaf();
            if (n <= max_leaf && best_axis < 0) return make_leaf();
            // object median on the widest centroid axis (bounded depth)
            int axis = 0;
            if (ext[1] > ext[axis]) axis = 1;
            if (ext[2] > ext[axis]) axis = 2;
            mid = b + n / 2;
            std::nth_element(refs + b, refs + mid, refs + e, [&](const PrimRef& x, const PrimRef& y) {
                if (x.c[axis] != y.c[axis]) return x.c[axis] < y.c[axis];
                return x.id < y.id;
            });
        }

        uint32_t self = (uint32_t)(st.nodes.size() / 16);
        st.nodes.resize(st.nodes.size() + 16, 0.0f);
        st.sah += area_ratio * kNodeCost;
        Box lb, rb;
        int32_t lc, rc;
        if (allow_async && n >= 2 * kParallelGrain) {
            // Right subtree on another thread into its own list, then splice.
            SubTree rst;
            auto fut = std::async(std::launch::async, [&]() {
                return build(rst, mid, e, depth + 1, rb, true);
            });
            lc = build(st, b, mid, depth + 1, lb, true);
            rc = fut.get();
            if (rc >= 0) {
                uint32_t base = (uint32_t)(st.nodes.size() / 16);
                size_t off = st.nodes.size();
                st.nodes.insert(st.nodes.end(), rst.nodes.begin(), rst.nodes.end());
                for (size_t k = off; k < st.nodes.size(); k += 16) {
                    for (int c = 0; c < 2; c++) {
                        int32_t code;
                        std::memcpy(&code, &st.nodes[k + 12 + c], 4);
                        if (code >= 0) code += (int32_t)base;
                        std::memcpy(&st.nodes[k + 12 + c], &code, 4);
                    }
                }
                rc += (int32_t)base;
            }
            st.max_depth = std::max(st.max_depth, rst.max_depth);
            st.leaves += rst.leaves;
            st.max_leaf = std::max(st.max_leaf, rst.max_leaf);
            st.sah += rst.sah;
        } else {
            lc = build(st, b, mid, depth + 1, lb, allow_async);
            rc = build(st, mid, e, depth + 1, rb, allow_async);
        }
        float* nd = &st.nodes[(size_t)self * 16];
        nd[0] = lb.lo[0]; nd[1] = lb.hi[0]; nd[2] = lb.lo[1]; nd[3] = lb.hi[1];
        nd[4] = rb.lo[0]; nd[5] = rb.hi[0]; nd[6] = rb.lo[1]; nd[7] = rb.hi[1];
        nd[8] = lb.lo[2]; nd[9] = lb.hi[2]; nd[10] = rb.lo[2]; nd[11] = rb.hi[2];
        std::memcpy(&nd[12], &lc, 4);
        std::memcpy(&nd[13], &rc, 4);
        return (int32_t)self;
    }
};

}  // namespace

BvhBuildResult build_bvh(const float* tv, uint64_t ntri, uint32_t max_leaf) {
    BvhBuildResult res;
    if (ntri == 0) return res;
    std::vector<PrimRef> refs(ntri);
    Box root;
    root.reset();
    for (uint64_t t = 0; t < ntri; t++) {
        PrimRef& r = refs[t];
        const float* v = tv + t * 9;
        for (int k = 0; k < 3; k++) {
            r.lo[k] = std::fmin(std::fmin(v[k], v[3 + k]), v[6 + k]);
            r.hi[k] = std::fmax(std::fmax(v[k], v[3 + k]), v[6 + k]);
            // NaN-only coordinates: park the primitive at the origin (its
            // triangle test rejects every ray anyway).
            if (!(r.lo[k] <= r.hi[k])) { r.lo[k] = 0.0f; r.hi[k] = 0.0f; }
            r.c[k] = 0.5f * r.lo[k] + 0.5f * r.hi[k];
        }
        r.id = (uint32_t)t;
        root.grow(r.lo, r.hi);
    }
    Builder bld;
    bld.refs = refs.data();
    bld.max_leaf = std::max<uint32_t>(1, std::min<uint32_t>(max_leaf, kMaxLeafSize));
    double ra = root.area();
    bld.root_area_inv = ra > 0.0 ? 1.0 / ra : 0.0;
    SubTree st;
    st.nodes.reserve((size_t)ntri * 16);
    Box box;
    int32_t code = bld.build(st, 0, ntri, 0, box, true);
    if (code < 0) {
        // The whole scene is one leaf: give it an inner root whose second
        // child is the same leaf behind a far-away point box (never entered
        // by a finite ray; entering it would only re-test real triangles).
        st.nodes.assign(16, 0.0f);
        float* nd = st.nodes.data();
        const float far_pt = 3.0e38f;
        nd[0] = box.lo[0]; nd[1] = box.hi[0]; nd[2] = box.lo[1]; nd[3] = box.hi[1];
        nd[4] = far_pt; nd[5] = far_pt; nd[6] = far_pt; nd[7] = far_pt;
        nd[8] = box.lo[2]; nd[9] = box.hi[2]; nd[10] = far_pt; nd[11] = far_pt;
        std::memcpy(&nd[12], &code, 4);
        std::memcpy(&nd[13], &code, 4);
        st.max_depth = 1;
    }
    res.nodes = std::move(st.nodes);
    res.max_depth = st.max_depth;
    res.leaves = st.leaves;
    res.max_leaf = st.max_leaf;
    res.sah_cost = st.sah;
    res.slot2tri.resize(ntri);
    for (uint64_t i = 0; i < ntri; i++) res.slot2tri[i] = refs[i].id;
    return res;
}

}  // namespace spt
