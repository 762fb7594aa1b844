// bvh8_build.cpp — collapse the binned-SAH BVH2 (leaf size 1) into
// the compressed 8-wide layout of bvh_build.h (after Ylitie, Karras, Laine,
// "Efficient Incoherent Ray Traversal on GPUs Through Compressed Wide BVHs",
// HPG 2017): the SAH-optimal collapse of their §3.1 by dynamic programming
// (default; the greedy "open the largest-area inner child until 8 children"
// is mode 1), octant-ordered child slots, 8-bit conservative quantisation.
// width 6 caps a node at six children (still in eight octant slots) for the
// 64-B device node (gpu_bvh8_holes).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "bvh_build.h"

namespace spt {
namespace {


struct Kid {
    float lo[3], hi[3];
    int32_t code;  // BVH2 child code: >= 0 inner node, < 0 leaf ~(first << 3 | count - 1)
    uint32_t ntri = 0;  // triangles in the subtree
    bool leaf = false;  // becomes a BVH8 leaf (all its <= 3 triangles) rather than a BVH8 node
    double area() const {  // double: boxes near FLT_MAX would overflow a float area
        const double dx = (double)hi[0] - lo[0], dy = (double)hi[1] - lo[1], dz = (double)hi[2] - lo[2];
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
};

struct Collapser {
    const std::vector<float>& n2;          // BVH2 nodes, 16 floats each
    const std::vector<uint32_t>& slot2tri;  // BVH2 leaf order -> triangle id
    std::vector<uint32_t> nodes;           // BVH8 nodes, 20 words each
    std::vector<uint32_t> tri_order;       // BVH8 triangle slot -> triangle id
    uint32_t depth = 0;
    uint64_t leaves = 0;
    std::vector<uint32_t> ntri2;           // triangles under each BVH2 inner node
    int mode = 1;                          // 0: BVH2 leaves as is; 1: leaf-size-1 BVH2, greedy;
                                           // 2: greedy, fill to 8; 3: SAH-optimal collapse (DP)
    // mode 3 (Ylitie et al. 2017 §3.1): cost[n*9+i] = least SAH cost of BVH2
    // subtree n as at most i BVH8 children; take[n*9+i] = 1 if that is
    // cost[n, i-1] (i >= 2), for i = 1: 1 = leaf, 0 = BVH8 node; split[n*9+i]
    // = the left child's share of i slots in the best distribution.
    std::vector<double> cost, dist;
    std::vector<uint8_t> take, split;
    double c_node = 1.0, c_prim = SPT_C_PRIM;
    int width = 8;                         // children per node: 8, or 6 for the 64-B device node

    uint32_t count_tris(int32_t code) {
        if (code < 0) return ((~(uint32_t)code) & 7u) + 1u;
        const float* nd = &n2[(size_t)code * 16];
        int32_t c0, c1;
        std::memcpy(&c0, &nd[12], 4);
        std::memcpy(&c1, &nd[13], 4);
        return ntri2[code] = count_tris(c0) + count_tris(c1);
    }
    // Leaf candidate: a subtree small enough to become one BVH8 leaf (<= 3 triangles).
    bool leafable(const Kid& k) const { return k.code < 0 || (mode >= 1 && k.ntri <= 3); }
    // Triangles (BVH2 leaf-order slots) of a subtree, in order.
    void gather(int32_t code, std::vector<uint32_t>& out) const {
        if (code < 0) {
            const uint32_t c = ~(uint32_t)code;
            for (uint32_t i = 0; i < (c & 7u) + 1u; i++) out.push_back((c >> 3) + i);
            return;
        }
        const float* nd = &n2[(size_t)code * 16];
        int32_t c0, c1;
        std::memcpy(&c0, &nd[12], 4);
        std::memcpy(&c1, &nd[13], 4);
        gather(c0, out);
        gather(c1, out);
    }

    Kid child(int32_t node, int c) const {
        const float* nd = &n2[(size_t)node * 16];
        Kid k;
        if (c == 0) {
            k.lo[0] = nd[0]; k.hi[0] = nd[1]; k.lo[1] = nd[2]; k.hi[1] = nd[3]; k.lo[2] = nd[8]; k.hi[2] = nd[9];
        } else {
            k.lo[0] = nd[4]; k.hi[0] = nd[5]; k.lo[1] = nd[6]; k.hi[1] = nd[7]; k.lo[2] = nd[10]; k.hi[2] = nd[11];
        }
        std::memcpy(&k.code, &nd[12 + c], 4);
        k.ntri = k.code < 0 ? ((~(uint32_t)k.code) & 7u) + 1u : ntri2[k.code];
        return k;
    }

    static uint32_t alloc(std::vector<uint32_t>& v, uint32_t count) {
        uint32_t first = (uint32_t)(v.size() / 20);
        v.resize(v.size() + (size_t)20 * count, 0u);
        return first;
    }

    // ---- mode 3: SAH-optimal collapse by dynamic programming over the BVH2
    double leaf_cost(const Kid& k) const {
        return k.ntri <= 3 ? (double)k.area() * c_prim * (double)k.ntri : INFINITY;
    }
    double kid_cost(const Kid& k, int i) const {  // cost of a BVH2 child with i slots
        return k.code < 0 ? leaf_cost(k) : cost[(size_t)k.code * 9 + i];
    }
    void dp(int32_t root, const Kid& root_kid) {
        const size_t nn = n2.size() / 16;
        cost.assign(nn * 9, INFINITY);
        dist.assign(nn * 9, INFINITY);
        take.assign(nn * 9, 0);
        split.assign(nn * 9, 0);
        std::vector<double> area(nn, 0.0);
        area[root] = root_kid.area();
        // post-order over inner nodes (parents before children in a pre-order list)
        std::vector<int32_t> order, stack{root};
        while (!stack.empty()) {
            int32_t n = stack.back();
            stack.pop_back();
            order.push_back(n);
            for (int c = 0; c < 2; c++) {
                Kid k = child(n, c);
                if (k.code >= 0) {
                    area[k.code] = k.area();
                    stack.push_back(k.code);
                }
            }
        }
        for (size_t oi = order.size(); oi-- > 0;) {
            const int32_t n = order[oi];
            const Kid l = child(n, 0), r = child(n, 1);
            double* C = &cost[(size_t)n * 9];
            double* D = &dist[(size_t)n * 9];
            for (int i = 2; i <= width; i++) {
                split[(size_t)n * 9 + i] = 1;  // a valid share even when every cost is inf / NaN
                for (int k = 1; k < i; k++) {
                    const double v = kid_cost(l, k) + kid_cost(r, i - k);
                    if (v < D[i]) { D[i] = v; split[(size_t)n * 9 + i] = (uint8_t)k; }
                }
            }
            Kid self;
            self.code = n;
            self.ntri = ntri2[n];
            const double lc = self.ntri <= 3 ? (double)area[n] * c_prim * (double)self.ntri : INFINITY;
            const double ic = (double)area[n] * c_node + D[width];
            C[1] = std::min(lc, ic);
            take[(size_t)n * 9 + 1] = (self.ntri <= 3 && lc <= ic) ? 1 : 0;
            for (int i = 2; i <= width; i++) {
                take[(size_t)n * 9 + i] = C[i - 1] <= D[i] ? 1 : 0;
                C[i] = std::min(C[i - 1], D[i]);
            }
        }
    }
    // The BVH8 children of BVH2 element k given i slots.
    void collect(const Kid& k, int i, std::vector<Kid>& out) const {
        if (k.code < 0) {
            Kid x = k;
            x.leaf = true;
            out.push_back(x);
            return;
        }
        const size_t b = (size_t)k.code * 9;
        while (i > 1 && take[b + i]) i--;
        if (i == 1) {
            Kid x = k;
            x.leaf = take[b + 1] != 0;
            out.push_back(x);
            return;
        }
        const int s = split[b + i];
        collect(child(k.code, 0), s, out);
        collect(child(k.code, 1), i - s, out);
    }
    std::vector<Kid> dp_kids(int32_t node) const {
        std::vector<Kid> kids;
        const int s = split[(size_t)node * 9 + width];
        collect(child(node, 0), s, kids);
        collect(child(node, 1), width - s, kids);
        return kids;
    }

    // Fill node `idx` from the kids list (the BVH2 children of one BVH2 node;
    // mode 3: the final children).
    void emit(uint32_t idx, std::vector<Kid> kids, uint32_t level) {
        depth = std::max(depth, level);
        // Greedy collapse: open the largest-area kid that cannot be a leaf while
        // room remains; in mode 2 then keep splitting multi-triangle leaf
        // candidates (largest first) to fill the 8 slots.
        while (mode < 3 && kids.size() < (size_t)width) {
            int best = -1;
            double best_area = -1.0;
            for (size_t i = 0; i < kids.size(); i++)
                if (kids[i].code >= 0 && !leafable(kids[i]) && kids[i].area() > best_area) {
                    best_area = kids[i].area();
                    best = (int)i;
                }
            if (best < 0 && mode >= 2)
                for (size_t i = 0; i < kids.size(); i++)
                    if (kids[i].code >= 0 && kids[i].area() > best_area) {
                        best_area = kids[i].area();
                        best = (int)i;
                    }
            if (best < 0) break;
            int32_t c = kids[best].code;
            kids[best] = child(c, 0);
            kids.push_back(child(c, 1));
        }
        if (mode < 3)
            for (Kid& k : kids) k.leaf = leafable(k);
        // Node box and octant-ordered slots: slot s gets the kid that rays of
        // octant s (bit i set <=> direction component i negative) reach first.
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (const Kid& k : kids)
            for (int a = 0; a < 3; a++) {
                lo[a] = std::fmin(lo[a], k.lo[a]);
                hi[a] = std::fmax(hi[a], k.hi[a]);
            }
        double ctr[3];
        for (int a = 0; a < 3; a++) ctr[a] = 0.5 * ((double)lo[a] + (double)hi[a]);
        int slot_of[8];
        int kid_in[8];
        for (int s = 0; s < 8; s++) kid_in[s] = -1;
        {
            double cost[8][8];
            for (size_t k = 0; k < kids.size(); k++)
                for (int s = 0; s < 8; s++) {
                    double c = 0.0;
                    for (int a = 0; a < 3; a++) {
                        double d = 0.5 * ((double)kids[k].lo[a] + (double)kids[k].hi[a]) - ctr[a];
                        c += ((s >> a) & 1) ? -d : d;
                    }
                    cost[k][s] = c;
                }
            bool kdone[8] = {false};
            for (size_t n = 0; n < kids.size(); n++) {
                double bc = INFINITY;
                int bk = -1, bs = -1;
                for (size_t k = 0; k < kids.size(); k++) {
                    if (kdone[k]) continue;
                    for (int s = 0; s < 8; s++)
                        if (kid_in[s] < 0 && cost[k][s] < bc) { bc = cost[k][s]; bk = (int)k; bs = s; }
                }
                if (bk < 0) {  // NaN costs: first free slot
                    for (size_t k = 0; k < kids.size(); k++)
                        if (!kdone[k]) { bk = (int)k; break; }
                    for (int s = 0; s < 8; s++)
                        if (kid_in[s] < 0) { bs = s; break; }
                }
                kdone[bk] = true;
                kid_in[bs] = bk;
                slot_of[bk] = bs;
            }
        }
        (void)slot_of;
        // Quantisation frame: p = node lo, per-axis power-of-two step with
        // 255 steps covering the node; child boxes rounded outward.
        uint32_t* w = &nodes[(size_t)idx * 20];
        int ebias[3];
        for (int a = 0; a < 3; a++) {
            double ext = (double)hi[a] - (double)lo[a];
            int e = -100;
            if (!(ext <= 1e300)) {
                e = 127;  // infinite (or NaN) extent: the widest step; such triangles are never hit
            } else if (ext > 0.0) {
                e = (int)std::ceil(std::log2(ext / 255.0));
                while (std::ldexp(255.0, e) < ext) e++;
                e = std::min(std::max(e, -100), 127);
            }
            ebias[a] = e + 127;
            std::memcpy(&w[a], &lo[a], 4);
        }
        uint32_t imask = 0;
        uint8_t meta[8] = {0};
        uint8_t qlo[3][8], qhi[3][8];
        for (int s = 0; s < 8; s++)
            for (int a = 0; a < 3; a++) { qlo[a][s] = 255; qhi[a][s] = 0; }  // empty: inverted
        // triangles of the leaf kids, contiguous in slot order
        const uint32_t tri_base = (uint32_t)tri_order.size();
        uint32_t toff = 0;
        uint32_t ninner = 0;
        for (int s = 0; s < 8; s++) {
            int k = kid_in[s];
            if (k < 0) continue;
            const Kid& kd = kids[k];
            for (int a = 0; a < 3; a++) {
                double step = std::ldexp(1.0, ebias[a] - 127);
                double ql = std::floor(((double)kd.lo[a] - (double)lo[a]) / step);
                double qh = std::ceil(((double)kd.hi[a] - (double)lo[a]) / step);
                if (!(ql >= 0.0)) ql = 0.0;  // NaN-safe
                if (!(qh <= 255.0)) qh = 255.0;
                if (ql > 255.0) ql = 255.0;
                if (qh < 0.0) qh = 0.0;
                qlo[a][s] = (uint8_t)ql;
                qhi[a][s] = (uint8_t)qh;
            }
            if (!kd.leaf) {
                imask |= 1u << s;
                meta[s] = (uint8_t)(0x20u | (24u + (uint32_t)s));
                ninner++;
            } else {
                std::vector<uint32_t> ts;
                gather(kd.code, ts);  // <= 3 triangles
                const uint32_t cnt = (uint32_t)ts.size();
                meta[s] = (uint8_t)((((1u << cnt) - 1u) << 5) | toff);
                for (uint32_t t : ts) tri_order.push_back(slot2tri[t]);
                toff += cnt;
                leaves++;
            }
        }
        const uint32_t child_base = ninner ? alloc(nodes, ninner) : 0u;
        w = &nodes[(size_t)idx * 20];  // (alloc may have moved the vector)
        w[3] = (uint32_t)ebias[0] | ((uint32_t)ebias[1] << 8) | ((uint32_t)ebias[2] << 16) | (imask << 24);
        w[4] = child_base;
        w[5] = tri_base;
        std::memcpy(&w[6], meta, 8);
        for (int a = 0; a < 3; a++) {
            std::memcpy(&w[8 + 2 * a], qlo[a], 8);
            std::memcpy(&w[14 + 2 * a], qhi[a], 8);
        }
        // recurse into the inner kids, in slot order, at their reserved indices
        uint32_t r = 0;
        for (int s = 0; s < 8; s++) {
            int k = kid_in[s];
            if (k < 0 || kids[k].leaf) continue;
            const int32_t c = kids[k].code;
            if (mode >= 3) emit(child_base + r, dp_kids(c), level + 1);
            else emit(child_base + r, {child(c, 0), child(c, 1)}, level + 1);
            r++;
        }
    }
};

}  // namespace

Bvh8BuildResult build_bvh8(const float* tv, uint64_t ntri, bool greedy, int width) {
    Bvh8BuildResult res;
    if (ntri == 0) return res;
    // 3: SAH-optimal collapse (+6 % on config 1 over the greedy mode 1)
    const int mode = greedy ? 1 : 3;
    BvhBuildResult b2 = build_bvh(tv, ntri, mode >= 1 ? 1 : 3);
    Collapser col{b2.nodes, b2.slot2tri, {}, {}, 0, 0};
    col.mode = mode;
    col.width = width == 6 ? 6 : 8;
    col.ntri2.assign(b2.nodes.size() / 16, 0);
    {
        int32_t r0, r1;
        std::memcpy(&r0, &b2.nodes[12], 4);
        std::memcpy(&r1, &b2.nodes[13], 4);
        if (r1 != r0) col.count_tris(0);  // (a duplicated root leaf needs no counts)
    }
    col.nodes.reserve(b2.nodes.size() / 16 * 20 / 4 + 20);
    col.tri_order.reserve(ntri);
    Collapser::alloc(col.nodes, 1);
    // build_bvh duplicates a root leaf into both children: keep one copy.
    int32_t c0, c1;
    std::memcpy(&c0, &b2.nodes[12], 4);
    std::memcpy(&c1, &b2.nodes[13], 4);
    if (b2.nodes.size() == 16 && c0 < 0 && c0 == c1) {
        Kid k = col.child(0, 0);
        k.leaf = true;
        col.emit(0, {k}, 1);
    } else if (mode >= 3) {
        Kid root = col.child(0, 0), r1 = col.child(0, 1);
        for (int a = 0; a < 3; a++) {
            root.lo[a] = std::fmin(root.lo[a], r1.lo[a]);
            root.hi[a] = std::fmax(root.hi[a], r1.hi[a]);
        }
        root.code = 0;
        root.ntri = col.ntri2[0];
        col.dp(0, root);
        col.emit(0, col.dp_kids(0), 1);
    } else {
        col.emit(0, {col.child(0, 0), col.child(0, 1)}, 1);
    }
    res.nodes = std::move(col.nodes);
    res.slot2tri = std::move(col.tri_order);
    res.depth = col.depth;
    res.leaves = col.leaves;
    res.sah_cost = b2.sah_cost;
    return res;
}

}  // namespace spt
