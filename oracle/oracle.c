/*
 * oracle.c — CPU restatement of jamornsriwasansak/smallpt-enoki-optix's
 * wavefront path tracer (the BASELINE.json north_star path).
 *
 * TEST INFRASTRUCTURE ONLY: the checker and the CPU baseline.  The product
 * (smallpt-enoki-optix_amd/, libspt.so) never includes, links or calls it.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * the reference root).  Third-party arithmetic restated from published
 * algorithms:
 *   - PCG32 (Enoki include/enoki/random.h; canonical pcg32 by M. O'Neill) —
 *     pinned by the canonical (42, 54) known-answer vector.
 *   - sincos (Enoki array_math.h: Cephes single-precision sin/cos) — parity
 *     unpinned (Enoki absent); our op order is fixed below and shared by
 *     specification (not by code) with the HIP kernels.
 *   - OptiX 7 closest-hit triangle test: restated as the Woop/Benthin/Wald
 *     2013 watertight test with PBRT's double-precision edge fallback; the
 *     barycentric convention is OptiX's p = (1-u-v) v0 + u v1 + v v2
 *     (add_math.h:3-7).  Parity vs OptiX unpinned (OptiX absent).
 * Floating-point: compiled with -ffp-contract=off; every fused multiply-add
 * is an explicit fmaf().
 *
 * Arithmetic variants (compile-time, oracle/Makefile builds each as its own
 * liboracle_alt_*.so): the choices the reference leaves to code we cannot
 * run, each swapped for a plausible alternative so the tests can bound how
 * much the image depends on it (tests/test_parity_tolerance.py):
 *   ORACLE_ALT_SINCOS     libm sinf/cosf instead of Cephes (Enoki sincos, mapping.h:9,25)
 *   ORACLE_ALT_RSQRT      normalize with a 1-ulp-high reciprocal square root
 *                         (Enoki normalize = v * rsqrt(|v|^2), CUDA rsqrt.approx)
 *   (fp-contract)         -ffp-contract=fast -mfma: products fused into FMAs
 *                         wherever the compiler likes (nvcc's default contraction)
 *   ORACLE_ALT_TRI        Moller-Trumbore (not watertight) instead of the Woop
 *                         test standing in for OptiX's triangle test (optix_backend.h:314)
 *   (all)                 the four together
 *   ORACLE_ALT_ENOKI      (separately) Enoki's own op forms on the CUDA backend, as
 *                         its published headers define them: dot = an fmadd chain
 *                         (x*x, then fma y, then fma z), Matrix x Array = an fmadd
 *                         chain over the columns (coordframe.h:42,47 to_local /
 *                         to_world: bx*l.x, fma by*l.y, fma bz*l.z), normalize =
 *                         v * rsqrt(|v|^2) with the reciprocal square root
 *                         correctly rounded (rsqrt.approx's own bits are NVIDIA's),
 *                         and .ftz arithmetic (denormal inputs / results flushed
 *                         to zero: MXCSR FTZ+DAZ in the worker threads)
 *   ORACLE_ALT_TEX1X1     (separately) every material's constant colour through
 *                         ImageTexture::eval as the reference's 1x1 image
 *                         (main.cpp:40-44, 62-76): bilinear weights that sum to
 *                         1 only up to rounding, instead of the exact constant
 */
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#ifdef ORACLE_ALT_ENOKI
#include <xmmintrin.h>
#endif
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

#define PCG32_MULT 0x5851f42d4c957f2dULL
#define PI_F 3.14159265358979323846f

/* ------------------------------------------------------------------ PCG32 */
/* Enoki random.h (external): seed / next_uint32 / next_float32.  Seeding call
 * site main.cpp:376 (initstate = PCG32_DEFAULT_STATE, initseq = pixel index). */
typedef struct { uint64_t state, inc; } pcg32_t;

static inline uint32_t pcg32_next(pcg32_t* r) {
    uint64_t old = r->state;
    r->state = old * PCG32_MULT + r->inc;
    uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((32u - rot) & 31u));
}
static inline void pcg32_seed(pcg32_t* r, uint64_t initstate, uint64_t initseq) {
    r->state = 0;
    r->inc = (initseq << 1u) | 1u;
    pcg32_next(r);
    r->state += initstate;
    pcg32_next(r);
}
static inline float u32_as_float(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t float_as_u32(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float pcg32_float(pcg32_t* r) {
    return u32_as_float((pcg32_next(r) >> 9) | 0x3f800000u) - 1.0f;
}

void oracle_pcg32_seq(uint64_t initstate, uint64_t initseq, uint32_t* out, int32_t n) {
    pcg32_t r; pcg32_seed(&r, initstate, initseq);
    for (int32_t i = 0; i < n; i++) out[i] = pcg32_next(&r);
}
void oracle_pcg32_floats(uint64_t initstate, uint64_t initseq, float* out, int32_t n) {
    pcg32_t r; pcg32_seed(&r, initstate, initseq);
    for (int32_t i = 0; i < n; i++) out[i] = pcg32_float(&r);
}

/* ---------------------------------------------------------------- sincos */
/* Cephes single-precision joint sin/cos as used by Enoki's sincos (called at
 * mapping.h:9 and mapping.h:25). */
void oracle_sincos(float x, float* s_out, float* c_out) {
#ifdef ORACLE_ALT_SINCOS
    *s_out = sinf(x);
    *c_out = cosf(x);
    return;
#endif
    float xa = fabsf(x);
    int32_t j = (int32_t)(xa * 1.2732395447351626862f);
    j = (j + 1) & ~1;
    float y = (float)j;
    uint32_t sign_sin = (((uint32_t)j << 29) & 0x80000000u) ^ (float_as_u32(x) & 0x80000000u);
    uint32_t sign_cos = ((uint32_t)(~(j - 2)) << 29) & 0x80000000u;
    y = ((xa - y * 0.78515625f) - y * 2.4187564849853515625e-4f) - y * 3.77489497744594108e-8f;
    float z = y * y;
    float s = fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f) * z;
    float c = fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f) * z;
    s = fmaf(s, y, y);
    c = fmaf(c, z, fmaf(z, -0.5f, 1.0f));
    int poly = (j & 2) == 0;
    float rs = poly ? s : c;
    float rc = poly ? c : s;
    *s_out = u32_as_float(float_as_u32(rs) ^ sign_sin);
    *c_out = u32_as_float(float_as_u32(rc) ^ sign_cos);
}

/* ------------------------------------------------------------ vector math */
typedef struct { float x, y, z; } v3;
static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
#ifdef ORACLE_ALT_ENOKI
/* Enoki dot: coeff(0) * coeff(0), then fmadd of each further coefficient */
static inline float dot3(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
#else
static inline float dot3(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
#endif
static inline v3 cross3(v3 a, v3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* Enoki normalize: v * rsqrt(squared_norm(v)); restated as v * (1/sqrt). */
static inline v3 normalize3(v3 v) {
#ifdef ORACLE_ALT_ENOKI
    float inv = (float)(1.0 / sqrt((double)dot3(v, v)));  /* one rounding: rsqrt, not 1 / sqrt */
#else
    float inv = 1.0f / sqrtf(dot3(v, v));
#endif
#ifdef ORACLE_ALT_RSQRT
    inv = nextafterf(inv, INFINITY);
#endif
    return mk(v.x * inv, v.y * inv, v.z * inv);
}
static inline float get(v3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }

/* Frame3 (coordframe.h:5-51): columns bx, by, bz; to_world = M * l. */
typedef struct { v3 bx, by, bz; } frame3;
static inline v3 to_world(const frame3* f, v3 l) {
#ifdef ORACLE_ALT_ENOKI
    /* Matrix x Array over the columns bx, by, bz (coordframe.h:47) */
    return mk(fmaf(f->bz.x, l.z, fmaf(f->by.x, l.y, f->bx.x * l.x)),
              fmaf(f->bz.y, l.z, fmaf(f->by.y, l.y, f->bx.y * l.x)),
              fmaf(f->bz.z, l.z, fmaf(f->by.z, l.y, f->bx.z * l.x)));
#else
    return mk((f->bx.x * l.x + f->by.x * l.y) + f->bz.x * l.z,
              (f->bx.y * l.x + f->by.y * l.y) + f->bz.y * l.z,
              (f->bx.z * l.x + f->by.z * l.y) + f->bz.z * l.z);
#endif
}
static inline v3 to_local(const frame3* f, v3 w) {
    return mk(dot3(f->bx, w), dot3(f->by, w), dot3(f->bz, w));
}
/* coordframe.h:17-30 — branchless ONB with the normal as local +y.  The
 * normal is NOT renormalised (reference feeds an un-normalised interpolated
 * shading normal, optix_backend.h:412-420). */
static inline frame3 frame_from_normal(v3 n) {
    float sign = copysignf(1.0f, n.y);
    float a = -1.0f / (sign + n.y);
    float b = (n.z * n.x) * a;
    frame3 f;
    f.bx = mk(sign + (n.x * n.x) * a, -n.x, b);
    f.by = n;
    f.bz = mk(sign * b, (-sign) * n.z, 1.0f + ((sign * n.z) * n.z) * a);
    return f;
}
void oracle_frame_to_world(const float* n3, const float* l3, float* out3) {
    frame3 f = frame_from_normal(mk(n3[0], n3[1], n3[2]));
    v3 w = to_world(&f, mk(l3[0], l3[1], l3[2]));
    out3[0] = w.x; out3[1] = w.y; out3[2] = w.z;
}

/* mapping.h:5-11 */
static inline v3 cosine_hemisphere(float xi_x, float xi_y) {
    float sin_phi = sqrtf(1.0f - xi_x);
    float theta = (PI_F * 2.0f) * xi_y;
    float s, c;
    oracle_sincos(theta, &s, &c);
    return mk(c * sin_phi, sqrtf(xi_x), s * sin_phi);
}
void oracle_cosine_hemisphere(float xi_x, float xi_y, float* out3) {
    v3 r = cosine_hemisphere(xi_x, xi_y);
    out3[0] = r.x; out3[1] = r.y; out3[2] = r.z;
}
/* mapping.h:15-27 (Shirley-Chiu concentric map via Dave Cline). */
static inline void disk_from_square(float xi_x, float xi_y, float* ox, float* oy) {
    float ax = xi_x * 2.0f - 1.0f, ay = xi_y * 2.0f - 1.0f;
    float ax2 = ax * ax, ay2 = ay * ay;
    int cond = ax2 > ay2;
    float r = cond ? ax : ay;
    float phi = cond ? (PI_F / 4.0f) * (ay / ax) : (PI_F / 2.0f) - (PI_F / 4.0f) * (ax / ay);
    float s, c;
    oracle_sincos(phi, &s, &c);
    *ox = r * c;
    *oy = r * s;
}
void oracle_disk_from_square(float xi_x, float xi_y, float* out2) {
    disk_from_square(xi_x, xi_y, &out2[0], &out2[1]);
}

/* ----------------------------------------------------------------- camera */
/* ThinlensCamera (pinhole.h:7-72). */
typedef struct {
    v3 origin;
    frame3 frame;
    float lens_radius, focal_dist, dist_lens_to_film, ratio, film_y;
    int32_t W, H;
} camera_t;

static void camera_setup(camera_t* c, const oracle_params* p) {
    v3 from = mk(p->look_from[0], p->look_from[1], p->look_from[2]);
    v3 at = mk(p->look_at[0], p->look_at[1], p->look_at[2]);
    v3 up = mk(p->up[0], p->up[1], p->up[2]);
    c->origin = from;
    v3 z = normalize3(sub(at, from));          /* pinhole.h:20 */
    v3 x = normalize3(cross3(up, z));          /* pinhole.h:21 */
    v3 y = normalize3(cross3(z, x));           /* pinhole.h:22 */
    c->frame.bx = x; c->frame.by = y; c->frame.bz = z;
    c->lens_radius = p->lens_radius;
    c->focal_dist = p->focal_dist;
    c->film_y = p->film_size_y;
    c->dist_lens_to_film = (p->film_size_y * 0.5f) / tanf(p->fov_y * 0.5f); /* pinhole.h:40 */
    c->ratio = (float)p->width / (float)p->height;                         /* pinhole.h:41 */
    c->W = p->width; c->H = p->height;
}
/* pinhole.h:27-32 */
static v3 camera_sample_pos(const camera_t* c, float xi_x, float xi_y) {
    float lx, ly;
    disk_from_square(xi_x, xi_y, &lx, &ly);
    lx = lx * c->lens_radius; ly = ly * c->lens_radius;
    v3 w = to_world(&c->frame, mk(lx, 0.0f, ly));
    return mk(w.x + c->origin.x, w.y + c->origin.y, w.z + c->origin.z);
}
/* pinhole.h:34-56 */
static v3 camera_sample_dir(const camera_t* c, int32_t px, int32_t py, v3 pos, float xi_x, float xi_y) {
    v3 lens = to_local(&c->frame, sub(pos, c->origin));
    float ndc_x = ((float)px + xi_x) / (float)c->W;
    float ndc_y = ((float)py + xi_y) / (float)c->H;
    float fx = (0.5f - ndc_x) * (c->ratio * c->film_y);
    float fy = (0.5f - ndc_y) * c->film_y;
    float fz = c->dist_lens_to_film;
    v3 focal = mk((c->focal_dist * fx) / fz, (c->focal_dist * fy) / fz, (c->focal_dist * fz) / fz);
    v3 d = normalize3(sub(focal, lens));
    return to_world(&c->frame, d);
}
void oracle_camera_ray(const oracle_params* p, int32_t px, int32_t py, const float* xi4,
                       float* org3, float* dir3, float* basis9) {
    camera_t c;
    camera_setup(&c, p);
    v3 o = camera_sample_pos(&c, xi4[0], xi4[1]);
    v3 d = camera_sample_dir(&c, px, py, o, xi4[2], xi4[3]);
    org3[0] = o.x; org3[1] = o.y; org3[2] = o.z;
    dir3[0] = d.x; dir3[1] = d.y; dir3[2] = d.z;
    if (basis9) {
        basis9[0] = c.frame.bx.x; basis9[1] = c.frame.bx.y; basis9[2] = c.frame.bx.z;
        basis9[3] = c.frame.by.x; basis9[4] = c.frame.by.y; basis9[5] = c.frame.by.z;
        basis9[6] = c.frame.bz.x; basis9[7] = c.frame.bz.y; basis9[8] = c.frame.bz.z;
    }
}

/* ------------------------------------------------------------------ scene */
typedef struct {
    float bmin[3], bmax[3];
    int32_t left;   /* inner: index of left child (right = left + 1); leaf: first prim */
    int32_t count;  /* 0 = inner */
} onode;

typedef struct {
    int64_t ntri;
    float* v;       /* ntri * 9: v0 v1 v2 */
    float* n;       /* ntri * 9: shading normals n0 n1 n2 */
    int32_t* mat;   /* ntri */
    float* albedo;  /* nmat * 3 */
    int32_t nmat;
    float* emission; /* nemit * 3 or NULL */
    int32_t nemit;
    float* tc;       /* ntri * 6: texcoords t0 t1 t2 (0 where missing) or NULL */
    /* per-material reflectance images (LambertBsdf::m_reflectance, main.cpp:102-120):
     * tex_w[m] = 0 -> the albedo table's constant */
    int32_t ntex;
    int32_t* tex_w; int32_t* tex_h;
    float** tex_rgb; /* interleaved RGB, w * h texels */
    /* smallpt's analytic spheres (cx, cy, cz, r) + material, after the BVH */
    float* sph; int32_t* sph_mat; int32_t nsph;
    uint32_t* kind; int32_t nkind;  /* SPT_MAT_*: 0 diffuse, 1 mirror, 2 glass */
    int32_t use_bvh;
    onode* nodes;
    int64_t nnodes;
    int32_t* prims; /* leaf order -> triangle id */
} oscene;

typedef struct { float* cen; int32_t axis; } sortctx;
static __thread sortctx g_sort;
static int cmp_prim(const void* a, const void* b) {
    float ca = g_sort.cen[*(const int32_t*)a * 3 + g_sort.axis];
    float cb = g_sort.cen[*(const int32_t*)b * 3 + g_sort.axis];
    if (ca < cb) return -1;
    if (ca > cb) return 1;
    return (*(const int32_t*)a < *(const int32_t*)b) ? -1 : 1;
}

/* Binned-SAH BVH2 (16 bins per axis over the centroid bounds; leaves of at
 * most 4 triangles unless splitting does not pay; a degenerate centroid
 * spread, or depth 48, falls back to a median split, so the tree is at most
 * 48 + log2(n) deep).  Independent of the product's
 * builders (bvh_build.cpp, gpu_build.hip); the closest hit does not depend on
 * the tree (ties go to the smaller id), which tests/test_oracle.py checks
 * against brute force. */
#define SAH_BINS 16
static float half_area(const float* lo, const float* hi) {
    float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    if (!(dx >= 0.0f)) return 0.0f;
    return dx * dy + dy * dz + dz * dx;
}
static void build_node(oscene* s, float* cen, int64_t ni, int64_t first, int64_t count, int depth) {
    onode* nd = &s->nodes[ni];
    for (int k = 0; k < 3; k++) { nd->bmin[k] = INFINITY; nd->bmax[k] = -INFINITY; }
    float cmin[3] = {INFINITY, INFINITY, INFINITY}, cmax[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t i = first; i < first + count; i++) {
        int32_t p = s->prims[i];
        for (int vtx = 0; vtx < 3; vtx++)
            for (int k = 0; k < 3; k++) {
                float x = s->v[p * 9 + vtx * 3 + k];
                if (x < nd->bmin[k]) nd->bmin[k] = x;
                if (x > nd->bmax[k]) nd->bmax[k] = x;
            }
        for (int k = 0; k < 3; k++) {
            float c = cen[p * 3 + k];
            if (c < cmin[k]) cmin[k] = c;
            if (c > cmax[k]) cmax[k] = c;
        }
    }
    if (count <= 2) { nd->left = (int32_t)first; nd->count = (int32_t)count; return; }
    /* SAH over binned centroids: cost = A_l * n_l + A_r * n_r (traversal cost 1 per node area) */
    int best_axis = -1, best_split = 0;
    float best_cost = INFINITY;
    for (int axis = 0; axis < 3; axis++) {
        float ext = cmax[axis] - cmin[axis];
        if (!(ext > 0.0f)) continue;
        float lo[SAH_BINS][3], hi[SAH_BINS][3];
        int64_t cnt[SAH_BINS];
        for (int b = 0; b < SAH_BINS; b++) {
            cnt[b] = 0;
            for (int k = 0; k < 3; k++) { lo[b][k] = INFINITY; hi[b][k] = -INFINITY; }
        }
        float scale = (float)SAH_BINS / ext;
        for (int64_t i = first; i < first + count; i++) {
            int32_t p = s->prims[i];
            int b = (int)((cen[p * 3 + axis] - cmin[axis]) * scale);
            if (b >= SAH_BINS) b = SAH_BINS - 1;
            if (b < 0) b = 0;
            cnt[b]++;
            for (int vtx = 0; vtx < 3; vtx++)
                for (int k = 0; k < 3; k++) {
                    float x = s->v[p * 9 + vtx * 3 + k];
                    if (x < lo[b][k]) lo[b][k] = x;
                    if (x > hi[b][k]) hi[b][k] = x;
                }
        }
        float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        float rarea[SAH_BINS];
        int64_t rcnt[SAH_BINS], acc = 0;
        for (int b = SAH_BINS - 1; b > 0; b--) {
            for (int k = 0; k < 3; k++) {
                if (lo[b][k] < rlo[k]) rlo[k] = lo[b][k];
                if (hi[b][k] > rhi[k]) rhi[k] = hi[b][k];
            }
            acc += cnt[b];
            rcnt[b] = acc;
            rarea[b] = half_area(rlo, rhi);
        }
        float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        int64_t lcnt = 0;
        for (int b = 0; b < SAH_BINS - 1; b++) {
            for (int k = 0; k < 3; k++) {
                if (lo[b][k] < llo[k]) llo[k] = lo[b][k];
                if (hi[b][k] > lhi[k]) lhi[k] = hi[b][k];
            }
            lcnt += cnt[b];
            if (lcnt == 0 || rcnt[b + 1] == 0) continue;
            float cost = half_area(llo, lhi) * (float)lcnt + rarea[b + 1] * (float)rcnt[b + 1];
            if (cost < best_cost) { best_cost = cost; best_axis = axis; best_split = b + 1; }
        }
    }
    float leaf_cost = half_area(nd->bmin, nd->bmax) * (float)count;
    if (count <= 4 && !(best_cost < leaf_cost)) { nd->left = (int32_t)first; nd->count = (int32_t)count; return; }
    int64_t half;
    if (depth >= 48) best_axis = -1;  /* bound the depth (stack, recursion): median splits below 48 levels */
    if (best_axis >= 0) {
        /* partition in place by bin (stable enough: ties only decide the tree shape) */
        float scale = (float)SAH_BINS / (cmax[best_axis] - cmin[best_axis]);
        int64_t i = first, j = first + count - 1;
        while (i <= j) {
            int32_t p = s->prims[i];
            int b = (int)((cen[p * 3 + best_axis] - cmin[best_axis]) * scale);
            if (b >= SAH_BINS) b = SAH_BINS - 1;
            if (b < best_split) i++;
            else { s->prims[i] = s->prims[j]; s->prims[j] = p; j--; }
        }
        half = i - first;
    } else {
        /* every centroid coincides (or too deep): a median split on the widest axis */
        int ax = 0;
        if (cmax[1] - cmin[1] > cmax[ax] - cmin[ax]) ax = 1;
        if (cmax[2] - cmin[2] > cmax[ax] - cmin[ax]) ax = 2;
        g_sort.cen = cen; g_sort.axis = ax;
        qsort(&s->prims[first], (size_t)count, sizeof(int32_t), cmp_prim);
        half = count / 2;
    }
    if (half <= 0 || half >= count) half = count / 2;
    int64_t l = s->nnodes;
    s->nnodes += 2;
    nd->left = (int32_t)l;
    nd->count = 0;
    build_node(s, cen, l, first, half, depth + 1);
    build_node(s, cen, l + 1, first + half, count - half, depth + 1);
}

void* oracle_scene_create(const int32_t* pos_tri, const float* pos, int64_t nvert, int64_t ntri,
                          const int32_t* nrm_tri, const float* nrm, int64_t nnrm,
                          const int32_t* mat_id, const float* albedo, int32_t nmat,
                          int32_t use_bvh) {
    oscene* s = (oscene*)calloc(1, sizeof(oscene));
    s->ntri = ntri;
    s->use_bvh = use_bvh;
    s->v = (float*)malloc(sizeof(float) * 9 * (size_t)(ntri > 0 ? ntri : 1));
    s->n = (float*)malloc(sizeof(float) * 9 * (size_t)(ntri > 0 ? ntri : 1));
    s->mat = (int32_t*)malloc(sizeof(int32_t) * (size_t)(ntri > 0 ? ntri : 1));
    for (int64_t t = 0; t < ntri; t++) {
        for (int vtx = 0; vtx < 3; vtx++) {
            int32_t pi = pos_tri[t * 3 + vtx];
            for (int k = 0; k < 3; k++)
                s->v[t * 9 + vtx * 3 + k] = (pi >= 0 && pi < nvert) ? pos[pi * 3 + k] : NAN;
        }
        /* A vertex without a normal (index -1) takes the geometric normal
         * normalize(cross(v1 - v0, v2 - v0)) (add_math.h:9-16); the reference
         * would gather out of bounds there. */
        const float* tv = &s->v[t * 9];
        v3 g = normalize3(cross3(mk(tv[3] - tv[0], tv[4] - tv[1], tv[5] - tv[2]),
                                 mk(tv[6] - tv[0], tv[7] - tv[1], tv[8] - tv[2])));
        for (int vtx = 0; vtx < 3; vtx++) {
            int32_t qi = nrm_tri ? nrm_tri[t * 3 + vtx] : -1;
            int ok = qi >= 0 && qi < nnrm;
            s->n[t * 9 + vtx * 3 + 0] = ok ? nrm[qi * 3 + 0] : g.x;
            s->n[t * 9 + vtx * 3 + 1] = ok ? nrm[qi * 3 + 1] : g.y;
            s->n[t * 9 + vtx * 3 + 2] = ok ? nrm[qi * 3 + 2] : g.z;
        }
        s->mat[t] = mat_id ? mat_id[t] : 0;
    }
    s->nmat = nmat > 0 ? nmat : 1;
    s->albedo = (float*)malloc(sizeof(float) * 3 * (size_t)s->nmat);
    for (int32_t m = 0; m < s->nmat; m++)
        for (int k = 0; k < 3; k++) s->albedo[m * 3 + k] = (albedo && nmat > 0) ? albedo[m * 3 + k] : 1.0f;
    if (use_bvh && ntri > 0) {
        float* cen = (float*)malloc(sizeof(float) * 3 * (size_t)ntri);
        for (int64_t t = 0; t < ntri; t++)
            for (int k = 0; k < 3; k++)
                cen[t * 3 + k] = (s->v[t * 9 + k] + s->v[t * 9 + 3 + k] + s->v[t * 9 + 6 + k]) * (1.0f / 3.0f);
        s->prims = (int32_t*)malloc(sizeof(int32_t) * (size_t)ntri);
        for (int64_t t = 0; t < ntri; t++) s->prims[t] = (int32_t)t;
        s->nodes = (onode*)malloc(sizeof(onode) * (size_t)(2 * ntri + 1));
        s->nnodes = 1;
        build_node(s, cen, 0, 0, ntri, 0);
        free(cen);
    }
    return s;
}

void oracle_scene_set_emission(void* scene, const float* emission, int32_t nmat) {
    oscene* s = (oscene*)scene;
    free(s->emission);
    s->emission = NULL;
    s->nemit = 0;
    if (!emission || nmat <= 0) return;
    s->emission = (float*)malloc(sizeof(float) * 3 * (size_t)nmat);
    memcpy(s->emission, emission, sizeof(float) * 3 * (size_t)nmat);
    s->nemit = nmat;
}

void oracle_scene_set_texcoords(void* scene, const int32_t* tc_tri, const float* tc, int64_t ntc) {
    oscene* s = (oscene*)scene;
    free(s->tc);
    s->tc = NULL;
    if (!tc_tri || !tc) return;
    s->tc = (float*)malloc(sizeof(float) * 6 * (size_t)(s->ntri > 0 ? s->ntri : 1));
    for (int64_t t = 0; t < s->ntri; t++)
        for (int k = 0; k < 3; k++) {
            int32_t i = tc_tri[t * 3 + k];
            int ok = i >= 0 && i < ntc;
            s->tc[t * 6 + k * 2] = ok ? tc[(int64_t)i * 2] : 0.0f;
            s->tc[t * 6 + k * 2 + 1] = ok ? tc[(int64_t)i * 2 + 1] : 0.0f;
        }
}

void oracle_scene_set_texture(void* scene, int32_t mat, const float* rgb, int32_t w, int32_t h) {
    oscene* s = (oscene*)scene;
    if (mat < 0) return;
    if (mat >= s->ntex) {
        int32_t n = mat + 1;
        s->tex_w = (int32_t*)realloc(s->tex_w, sizeof(int32_t) * (size_t)n);
        s->tex_h = (int32_t*)realloc(s->tex_h, sizeof(int32_t) * (size_t)n);
        s->tex_rgb = (float**)realloc(s->tex_rgb, sizeof(float*) * (size_t)n);
        for (int32_t i = s->ntex; i < n; i++) { s->tex_w[i] = 0; s->tex_h[i] = 0; s->tex_rgb[i] = NULL; }
        s->ntex = n;
    }
    free(s->tex_rgb[mat]);
    s->tex_rgb[mat] = NULL;
    s->tex_w[mat] = 0;
    s->tex_h[mat] = 0;
    if (!rgb || w <= 0 || h <= 0) return;
    s->tex_rgb[mat] = (float*)malloc(sizeof(float) * 3 * (size_t)w * (size_t)h);
    memcpy(s->tex_rgb[mat], rgb, sizeof(float) * 3 * (size_t)w * (size_t)h);
    s->tex_w[mat] = w;
    s->tex_h[mat] = h;
}

void oracle_scene_set_spheres(void* scene, const float* cr, const int32_t* mat, int32_t n) {
    oscene* s = (oscene*)scene;
    free(s->sph); free(s->sph_mat);
    s->sph = NULL; s->sph_mat = NULL; s->nsph = 0;
    if (!cr || n <= 0) return;
    s->sph = (float*)malloc(sizeof(float) * 4 * (size_t)n);
    s->sph_mat = (int32_t*)malloc(sizeof(int32_t) * (size_t)n);
    memcpy(s->sph, cr, sizeof(float) * 4 * (size_t)n);
    for (int32_t k = 0; k < n; k++) s->sph_mat[k] = mat ? mat[k] : 0;
    s->nsph = n;
}

void oracle_scene_set_material_kinds(void* scene, const uint32_t* kinds, int32_t n) {
    oscene* s = (oscene*)scene;
    free(s->kind);
    s->kind = NULL; s->nkind = 0;
    if (!kinds || n <= 0) return;
    s->kind = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n);
    memcpy(s->kind, kinds, sizeof(uint32_t) * (size_t)n);
    s->nkind = n;
}

void oracle_scene_destroy(void* scene) {
    oscene* s = (oscene*)scene;
    if (!s) return;
    free(s->v); free(s->n); free(s->mat); free(s->albedo); free(s->emission); free(s->nodes); free(s->prims);
    free(s->tc); free(s->sph); free(s->sph_mat); free(s->kind);
    for (int32_t i = 0; i < s->ntex; i++) free(s->tex_rgb[i]);
    free(s->tex_w); free(s->tex_h); free(s->tex_rgb);
    free(s);
}

/* ImageTexture::texel_fetch_wrap / texel_fetch (main.cpp:47-60): clamp to the
 * image, then the reference's index y * size.y + x (main.cpp:52; the row
 * stride is the height, harmless for square images), kept inside the image
 * (the reference would gather out of bounds when height > width). */
static inline const float* texel(const float* img, int32_t w, int32_t h, int32_t x, int32_t y) {
    x = x < 0 ? 0 : (x > w - 1 ? w - 1 : x);
    y = y < 0 ? 0 : (y > h - 1 ? h - 1 : y);
    int64_t idx = (int64_t)y * h + x;
    if (idx > (int64_t)w * h - 1) idx = (int64_t)w * h - 1;
    return img + idx * 3;
}
/* ImageTexture::eval (main.cpp:62-76): bilinear with clamp, in the
 * reference's operation order; uv scaled by the size, minus half a texel;
 * floor2int of a coordinate clamped to +-2^30 (NaN -> -2^30). */
static inline void texture_eval(const float* img, int32_t w, int32_t h, float u, float v, float out[3]) {
    float sx = u * (float)w - 0.5f, sy = v * (float)h - 0.5f;
    sx = fminf(fmaxf(sx, -1073741824.0f), 1073741824.0f);
    sy = fminf(fmaxf(sy, -1073741824.0f), 1073741824.0f);
    int32_t x = (int32_t)floorf(sx), y = (int32_t)floorf(sy);
    float dx1 = sx - (float)x, dy1 = sy - (float)y;
    float dx2 = 1.0f - dx1, dy2 = 1.0f - dy1;
    const float* f00 = texel(img, w, h, x, y);
    const float* f01 = texel(img, w, h, x, y + 1);
    const float* f10 = texel(img, w, h, x + 1, y);
    const float* f11 = texel(img, w, h, x + 1, y + 1);
    for (int c = 0; c < 3; c++)
        out[c] = (((f00[c] * dx2) * dy2 + (f01[c] * dx2) * dy1) + (f10[c] * dx1) * dy2) + (f11[c] * dx1) * dy1;
}
void oracle_texture_eval(const float* rgb, int32_t w, int32_t h, float u, float v, float* out3) {
    texture_eval(rgb, w, h, u, v, out3);
}

/* ------------------------------------------------------ triangle (Woop) */
typedef struct {
    float o[3], d[3];
    int kx, ky, kz;
    float Sx, Sy, Sz;
    float inv[3];
} wray;

static inline void wray_setup(wray* r) {
    float ax = fabsf(r->d[0]), ay = fabsf(r->d[1]), az = fabsf(r->d[2]);
    int kz = (ax > ay) ? ((ax > az) ? 0 : 2) : ((ay > az) ? 1 : 2);
    int kx = kz + 1; if (kx == 3) kx = 0;
    int ky = kx + 1; if (ky == 3) ky = 0;
    if (r->d[kz] < 0.0f) { int tmp = kx; kx = ky; ky = tmp; }
    r->kx = kx; r->ky = ky; r->kz = kz;
    /* one divide, two products (spt_math.h woop_setup) */
    r->Sz = 1.0f / r->d[kz];
    r->Sx = r->d[kx] * r->Sz;
    r->Sy = r->d[ky] * r->Sz;
    for (int k = 0; k < 3; k++) r->inv[k] = 1.0f / r->d[k];
}

#define BOX_PAD 1.000001f
/* node culling runs 4e-6 below tmin (spt_math.h cull_tmin): a box culled there
 * holds only triangles the box-exit rule drops anyway */
#define BOX_PAD_LO 0.999999f
static inline float pad_up(float x) { return x * (x >= 0.0f ? BOX_PAD : BOX_PAD_LO); }
#define CULL_TMIN_REL 4e-6f
static inline float cull_tmin(float tmin) { return tmin - fabsf(tmin) * CULL_TMIN_REL; }
static inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
/* max over the vertices of sign(d_k) * (v_k - o_k), sign(d_k) = sign(S) * sign(Sz) */
static inline float exit_offset(float a, float b, float c, float S, float Sz) {
    const int neg = ((fbits(S) ^ fbits(Sz)) >> 31) != 0u;
    return neg ? -fminf(fminf(a, b), c) : fmaxf(fmaxf(a, b), c);
}

/* Returns 1 and t/u/v when the triangle is hit with t in [tmin, tmax].
 * rule: 1 applies the box-exit rule (every tracer); 2 (oracle_box_rule_audit)
 * returns 2 for a hit the rule drops, with t/u/v set. */
static inline int woop_test_r(const wray* r, const float* tv, float tmin, float tmax,
                              float* t_out, float* u_out, float* v_out, int rule) {
#ifdef ORACLE_ALT_TRI
    /* Moller-Trumbore, barycentrics in the same p = (1-u-v) v0 + u v1 + v v2 convention */
    {
        const float e1[3] = {tv[3] - tv[0], tv[4] - tv[1], tv[5] - tv[2]};
        const float e2[3] = {tv[6] - tv[0], tv[7] - tv[1], tv[8] - tv[2]};
        const float pv[3] = {r->d[1] * e2[2] - r->d[2] * e2[1], r->d[2] * e2[0] - r->d[0] * e2[2],
                             r->d[0] * e2[1] - r->d[1] * e2[0]};
        const float det = (e1[0] * pv[0] + e1[1] * pv[1]) + e1[2] * pv[2];
        if (det == 0.0f) return 0;
        const float inv = 1.0f / det;
        const float tvec[3] = {r->o[0] - tv[0], r->o[1] - tv[1], r->o[2] - tv[2]};
        const float u = ((tvec[0] * pv[0] + tvec[1] * pv[1]) + tvec[2] * pv[2]) * inv;
        if (u < 0.0f || u > 1.0f) return 0;
        const float q[3] = {tvec[1] * e1[2] - tvec[2] * e1[1], tvec[2] * e1[0] - tvec[0] * e1[2],
                            tvec[0] * e1[1] - tvec[1] * e1[0]};
        const float v = ((r->d[0] * q[0] + r->d[1] * q[1]) + r->d[2] * q[2]) * inv;
        if (v < 0.0f || u + v > 1.0f) return 0;
        const float t = ((e2[0] * q[0] + e2[1] * q[1]) + e2[2] * q[2]) * inv;
        if (!(t >= tmin && t <= tmax)) return 0;
        *t_out = t; *u_out = u; *v_out = v;
        return 1;
    }
#endif
    float A[3], B[3], C[3];
    for (int k = 0; k < 3; k++) {
        A[k] = tv[k] - r->o[k];
        B[k] = tv[3 + k] - r->o[k];
        C[k] = tv[6 + k] - r->o[k];
    }
    /* the box-exit rule's farthest vertex offsets along the ray's motion in kx,
     * ky (sign(d_k) = sign(S) * sign(Sz)); spt_math.h exit_offset */
    const float ex = exit_offset(A[r->kx], B[r->kx], C[r->kx], r->Sx, r->Sz);
    const float ey = exit_offset(A[r->ky], B[r->ky], C[r->ky], r->Sy, r->Sz);
    float Ax = A[r->kx] - r->Sx * A[r->kz], Ay = A[r->ky] - r->Sy * A[r->kz];
    float Bx = B[r->kx] - r->Sx * B[r->kz], By = B[r->ky] - r->Sy * B[r->kz];
    float Cx = C[r->kx] - r->Sx * C[r->kz], Cy = C[r->ky] - r->Sy * C[r->kz];
    float U = Cx * By - Cy * Bx;
    float V = Ax * Cy - Ay * Cx;
    float W = Bx * Ay - By * Ax;
    if (U == 0.0f || V == 0.0f || W == 0.0f) {
        U = (float)((double)Cx * (double)By - (double)Cy * (double)Bx);
        V = (float)((double)Ax * (double)Cy - (double)Ay * (double)Cx);
        W = (float)((double)Bx * (double)Ay - (double)By * (double)Ax);
    }
    if ((U < 0.0f || V < 0.0f || W < 0.0f) && (U > 0.0f || V > 0.0f || W > 0.0f)) return 0;
    float det = (U + V) + W;
    if (det == 0.0f) return 0;
    float Az = r->Sz * A[r->kz], Bz = r->Sz * B[r->kz], Cz = r->Sz * C[r->kz];
    float T = (U * Az + V * Bz) + W * Cz;
    float t = T / det;
    if (!(t >= tmin && t <= tmax)) return 0;
    /* Box-exit rule (spt_math.h left_box_before_tmin): the hit counts only if
     * the ray has not left the triangle's own box before tmin, so the closest
     * hit does not depend on the tree (wavefront_isect.cu:103).
     * Per axis the exit t padded toward +inf (x BOX_PAD, or x BOX_PAD_LO when
     * negative: a negative tmin allows that) against tmin, without a divide. */
    const int drop = rule && (pad_up(fmaxf(fmaxf(Az, Bz), Cz)) < tmin ||
                              pad_up(ex * fabsf(r->Sz)) < tmin * fabsf(r->Sx) ||
                              pad_up(ey * fabsf(r->Sz)) < tmin * fabsf(r->Sy));
    if (drop && rule != 2) return 0;
    /* + 0.0f: a zero t, u or v is +0 (spt_math.h woop_core: its sign would
     * follow det's, which the kx / ky order flips) */
    *t_out = t + 0.0f;
    *u_out = V / det + 0.0f;
    *v_out = W / det + 0.0f;
    return drop ? 2 : 1;
}
static inline int woop_test(const wray* r, const float* tv, float tmin, float tmax,
                            float* t_out, float* u_out, float* v_out) {
    return woop_test_r(r, tv, tmin, tmax, t_out, u_out, v_out, 1);
}

/* Slab test over the closed box.  A direction component whose reciprocal is
 * infinite (d = +-0 or denormal) makes the ray parallel to that slab pair: it
 * is inside the slab for every t or never ((b - o) * inf would give NaN when
 * the origin lies on a plane). */
static inline int box_test(const wray* r, const onode* nd, float tmin, float tmax) {
    float tn = tmin, tf = tmax;
    for (int k = 0; k < 3; k++) {
        if (isinf(r->inv[k])) {
            if (r->o[k] < nd->bmin[k] || r->o[k] > nd->bmax[k]) return 0;
            continue;
        }
        float t0 = (nd->bmin[k] - r->o[k]) * r->inv[k];
        float t1 = (nd->bmax[k] - r->o[k]) * r->inv[k];
        float lo = fminf(t0, t1), hi = pad_up(fmaxf(t0, t1));  /* toward +inf, either sign */
        tn = fmaxf(tn, lo);
        tf = fminf(tf, hi);
    }
    return tn <= tf;
}

typedef struct { int32_t id; float t, u, v; } ohit;

/* Closest hit over [tmin, tmax]; equal t broken toward the smaller triangle id
 * so the result is independent of traversal order (OptiX returns one of the
 * tied hits; we fix the choice). */
static inline void consider(const oscene* s, const wray* r, int32_t p, float tmin, ohit* h) {
    float t, u, v;
    if (woop_test(r, &s->v[(int64_t)p * 9], tmin, h->t, &t, &u, &v)) {
        if (t < h->t || h->id < 0 || p < h->id) { h->id = p; h->t = t; h->u = u; h->v = v; }
    }
}

static void trace(const oscene* s, const wray* r, float tmin, float tmax, int closest, ohit* h) {
    h->id = -1; h->t = tmax; h->u = 0; h->v = 0;
    if (s->ntri <= 0) return;
    if (!s->use_bvh) {
        for (int64_t p = 0; p < s->ntri; p++) {
            consider(s, r, (int32_t)p, tmin, h);
            if (!closest && h->id >= 0) return;
        }
        return;
    }
    int32_t stack[256];
    int sp = 0;
    stack[sp++] = 0;
    while (sp) {
        const onode* nd = &s->nodes[stack[--sp]];
        /* the current hit padded like the exit planes: boxes entered at the
         * hit's t (ties at shared edges / vertices) are still visited; boxes
         * the ray leaves before cull_tmin(tmin) are culled, as on the GPU */
        if (!box_test(r, nd, cull_tmin(tmin), pad_up(h->t))) continue;
        if (nd->count) {
            for (int32_t i = 0; i < nd->count; i++) {
                consider(s, r, s->prims[nd->left + i], tmin, h);
                if (!closest && h->id >= 0) return;
            }
        } else {
            stack[sp++] = nd->left + 1;
            stack[sp++] = nd->left;
        }
    }
}

/* ------------------------------------------------------ thread helpers */
typedef struct {
    void (*fn)(void* ctx, int64_t i);
    void* ctx;
    int64_t n;
    atomic_llong next;
    int64_t chunk;
} pfor_t;
static void* pfor_worker(void* arg) {
    pfor_t* p = (pfor_t*)arg;
#ifdef ORACLE_ALT_ENOKI
    const unsigned int csr = _mm_getcsr();
    _mm_setcsr(csr | 0x8040u);  /* FTZ + DAZ: PTX .ftz */
#endif
    for (;;) {
        int64_t b = atomic_fetch_add(&p->next, p->chunk);
        if (b >= p->n) break;
        int64_t e = b + p->chunk < p->n ? b + p->chunk : p->n;
        for (int64_t i = b; i < e; i++) p->fn(p->ctx, i);
    }
#ifdef ORACLE_ALT_ENOKI
    _mm_setcsr(csr);  /* the caller's thread (nthreads <= 1) gets its mode back */
#endif
    return NULL;
}
static void parallel_for(int64_t n, int64_t chunk, int nthreads, void (*fn)(void*, int64_t), void* ctx) {
    pfor_t p;
    p.fn = fn; p.ctx = ctx; p.n = n; p.chunk = chunk < 1 ? 1 : chunk;
    atomic_init(&p.next, 0);
    if (nthreads <= 1) { pfor_worker(&p); return; }
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, pfor_worker, &p);
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
    free(th);
}

/* ------------------------------------------------------------ intersect */
typedef struct {
    const oscene* s;
    const float *ox, *oy, *oz, *dx, *dy, *dz, *tmin, *tmax;
    const uint8_t* mask; uint32_t mask_size;
    int32_t* id; float *t, *u, *v;
    int closest;
} isect_ctx;
/* ------------------------------------------------- smallpt spheres, kinds */
/* smallpt's Sphere::intersect in the ray's own t units: the nearer root in
 * [tmin, tmax], else +inf (op relative to the centre; same order as the GPU). */
static inline float sphere_t(v3 o, v3 d, const float* sp, float tmin, float tmax) {
    v3 op = mk(sp[0] - o.x, sp[1] - o.y, sp[2] - o.z);
    float a = dot3(d, d);
    float b = dot3(op, d);
    float c = dot3(op, op) - sp[3] * sp[3];
    float det = b * b - a * c;
    if (!(det >= 0.0f)) return INFINITY;
    float sq = sqrtf(det);
    float t0 = (b - sq) / a, t1 = (b + sq) / a;
    if (t0 >= tmin && t0 <= tmax) return t0;
    if (t1 >= tmin && t1 <= tmax) return t1;
    return INFINITY;
}
/* The spheres after the BVH: a sphere nearer than the current hit wins (ties
 * keep the triangle); id = -2 - k.  Any-hit: the first sphere hit, only when
 * no triangle was hit. */
static inline void trace_spheres(const oscene* s, v3 o, v3 d, float tmin, int anyhit, ohit* h) {
    if (anyhit && h->id != -1) return;
    for (int32_t k = 0; k < s->nsph; k++) {
        float t = sphere_t(o, d, &s->sph[k * 4], tmin, h->t);
        if (t < h->t) {
            h->t = t; h->id = -2 - k; h->u = 0.0f; h->v = 0.0f;
            if (anyhit) return;
        }
    }
}

static void isect_one(void* c_, int64_t i) {
    isect_ctx* c = (isect_ctx*)c_;
    uint8_t m = (c->mask_size == 1) ? c->mask[0] : c->mask[i];  /* wavefront_isect.cu:86 */
    if (!m) return;                                              /* masked lanes untouched */
    wray r;
    r.o[0] = c->ox[i]; r.o[1] = c->oy[i]; r.o[2] = c->oz[i];
    r.d[0] = c->dx[i]; r.d[1] = c->dy[i]; r.d[2] = c->dz[i];
    wray_setup(&r);
    ohit h;
    trace(c->s, &r, c->tmin[i], c->tmax[i], c->closest, &h);
    if (c->s->nsph) trace_spheres(c->s, mk(r.o[0], r.o[1], r.o[2]), mk(r.d[0], r.d[1], r.d[2]), c->tmin[i],
                                  !c->closest, &h);
    c->id[i] = h.id;                                             /* -1 on miss (wavefront_isect.cu:70) */
    if (h.id != -1) { c->t[i] = h.t; c->u[i] = h.u; c->v[i] = h.v; }
}
void oracle_intersect(void* scene, const float* ox, const float* oy, const float* oz,
                      const float* dx, const float* dy, const float* dz,
                      const float* tmin, const float* tmax, const uint8_t* mask,
                      uint32_t mask_size, int32_t* tri_id, float* t, float* u, float* v,
                      int64_t n, int32_t do_closest, int32_t nthreads) {
    isect_ctx c = {(const oscene*)scene, ox, oy, oz, dx, dy, dz, tmin, tmax, mask, mask_size,
                   tri_id, t, u, v, do_closest};
    parallel_for(n, 256, nthreads, isect_one, &c);
}

/* ------------------------------------------------ box-exit rule audit */
/* Every (ray, triangle) pair whose Woop test accepts a t in [tmin, tmax] that
 * the box-exit rule then drops (test infrastructure: tests/test_oracle.py and
 * tests/test_gpu_configs.py check each against a float64 box exit).  The
 * triangles are enumerated along the whole ray line — boxes grown by 1e-4 of
 * their extent and position, nothing culled on the near side — so no culling
 * decides which pairs are seen. */
typedef struct {
    const oscene* s;
    const float *ox, *oy, *oz, *dx, *dy, *dz, *tmin, *tmax;
    int64_t* ray; int32_t* tri; float* t;
    int64_t cap;
    atomic_llong found, accepted;
} audit_ctx;
static inline int line_box(const wray* r, const onode* nd, float tmax) {
    float tn = -INFINITY, tf = tmax;
    for (int k = 0; k < 3; k++) {
        const float g = 1e-4f * ((nd->bmax[k] - nd->bmin[k]) + fmaxf(fabsf(nd->bmin[k]), fabsf(nd->bmax[k]))) + 1e-30f;
        const float lo = nd->bmin[k] - g, hi = nd->bmax[k] + g;
        if (isinf(r->inv[k])) {
            if (r->o[k] < lo || r->o[k] > hi) return 0;
            continue;
        }
        const float t0 = (lo - r->o[k]) * r->inv[k], t1 = (hi - r->o[k]) * r->inv[k];
        tn = fmaxf(tn, fminf(t0, t1));
        tf = fminf(tf, fmaxf(t0, t1) * 1.0001f + 1e-30f);
    }
    return tn <= tf;
}
static void audit_pair(audit_ctx* c, const wray* r, int64_t i, int32_t p) {
    float t, u, v;
    const int res = woop_test_r(r, &c->s->v[(int64_t)p * 9], c->tmin[i], c->tmax[i], &t, &u, &v, 2);
    if (!res) return;
    atomic_fetch_add(&c->accepted, 1);
    if (res != 2) return;
    const int64_t k = atomic_fetch_add(&c->found, 1);
    if (k < c->cap) { c->ray[k] = i; c->tri[k] = p; c->t[k] = t; }
}
static void audit_one(void* c_, int64_t i) {
    audit_ctx* c = (audit_ctx*)c_;
    const oscene* s = c->s;
    if (s->ntri <= 0) return;
    wray r;
    r.o[0] = c->ox[i]; r.o[1] = c->oy[i]; r.o[2] = c->oz[i];
    r.d[0] = c->dx[i]; r.d[1] = c->dy[i]; r.d[2] = c->dz[i];
    wray_setup(&r);
    if (!s->use_bvh) {
        for (int64_t p = 0; p < s->ntri; p++) audit_pair(c, &r, i, (int32_t)p);
        return;
    }
    int32_t stack[256];
    int sp = 0;
    stack[sp++] = 0;
    while (sp) {
        const onode* nd = &s->nodes[stack[--sp]];
        if (!line_box(&r, nd, c->tmax[i])) continue;
        if (nd->count) {
            for (int32_t j = 0; j < nd->count; j++) audit_pair(c, &r, i, s->prims[nd->left + j]);
        } else {
            stack[sp++] = nd->left + 1;
            stack[sp++] = nd->left;
        }
    }
}
int64_t oracle_box_rule_audit(void* scene, const float* ox, const float* oy, const float* oz, const float* dx,
                              const float* dy, const float* dz, const float* tmin, const float* tmax, int64_t n,
                              int64_t* out_ray, int32_t* out_tri, float* out_t, int64_t cap, int64_t* accepted,
                              int32_t nthreads) {
    audit_ctx c;
    c.s = (const oscene*)scene;
    c.ox = ox; c.oy = oy; c.oz = oz; c.dx = dx; c.dy = dy; c.dz = dz; c.tmin = tmin; c.tmax = tmax;
    c.ray = out_ray; c.tri = out_tri; c.t = out_t; c.cap = cap;
    atomic_init(&c.found, 0);
    atomic_init(&c.accepted, 0);
    parallel_for(n, 64, nthreads, audit_one, &c);
    if (accepted) *accepted = (int64_t)atomic_load(&c.accepted);
    return (int64_t)atomic_load(&c.found);
}

static inline uint32_t material_kind(const oscene* s, int32_t mat) {
    return (s->kind && mat >= 0 && mat < s->nkind) ? s->kind[mat] : 0u;
}
/* Bounce direction and weight: triangles + diffuse = the reference's Lambert
 * bounce (Frame3 of the un-normalised shading normal); spheres and the mirror /
 * glass kinds = smallpt's radiance(): unit normal, flipped toward the ray for
 * diffuse; SPEC reflects; REFR: index 1.5, Schlick, reflect with probability
 * P = 1/4 + Re/2 by xi_x (weight Re/P, else Tr/(1-P)); TIR reflects. */
static v3 scatter(const oscene* s, uint32_t kind, int32_t id, v3 d, v3 p, v3 sn, float xi_x, float xi_y,
                  float* weight) {
    *weight = 1.0f;
    v3 n;
    if (id >= 0) {
        if (kind == 0) { frame3 f = frame_from_normal(sn); return to_world(&f, cosine_hemisphere(xi_x, xi_y)); }
        n = normalize3(sn);
    } else {
        const float* sp = &s->sph[(-2 - id) * 4];
        n = normalize3(mk(p.x - sp[0], p.y - sp[1], p.z - sp[2]));
        if (kind == 0) {
            v3 nl = dot3(n, d) < 0.0f ? n : mk(-n.x, -n.y, -n.z);
            frame3 f = frame_from_normal(nl);
            return to_world(&f, cosine_hemisphere(xi_x, xi_y));
        }
    }
    v3 dn = normalize3(d);
    float ndd = dot3(n, dn);
    float k2 = 2.0f * ndd;
    v3 refl = mk(dn.x - n.x * k2, dn.y - n.y * k2, dn.z - n.z * k2);
    if (kind != 2) return refl;
    int into = ndd < 0.0f;
    v3 nl = into ? n : mk(-n.x, -n.y, -n.z);
    float nc = 1.0f, nt = 1.5f;
    float nnt = into ? nc / nt : nt / nc;
    float ddn = dot3(dn, nl);
    float cos2t = 1.0f - (nnt * nnt) * (1.0f - ddn * ddn);
    if (cos2t < 0.0f) return refl;
    float ks = (into ? 1.0f : -1.0f) * (ddn * nnt + sqrtf(cos2t));
    v3 tdir = normalize3(mk(dn.x * nnt - n.x * ks, dn.y * nnt - n.y * ks, dn.z * nnt - n.z * ks));
    float ea = nt - nc, eb = nt + nc;
    float R0 = (ea * ea) / (eb * eb);
    float c = 1.0f - (into ? -ddn : dot3(tdir, n));
    float Re = R0 + (1.0f - R0) * ((((c * c) * c) * c) * c);
    float Tr = 1.0f - Re, P = 0.25f + 0.5f * Re;
    if (xi_x < P) { *weight = Re / P; return refl; }
    *weight = Tr / (1.0f - P);
    return tdir;
}

/* --------------------------------------------------------------- render */
/* Russian-roulette side stream (build addition, absent in the reference —
 * SURVEY F7/A14): a counter-based hash so the 4+2D PCG32 layout is untouched. */
static inline float rr_uniform(uint32_t pixel, uint32_t sample, uint32_t depth) {
    uint32_t h = pixel * 0x9E3779B1u ^ (sample + 0x7F4A7C15u) * 0x85EBCA77u ^ (depth + 1u) * 0xC2B2AE3Du;
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
    return (float)(h >> 8) * (1.0f / 16777216.0f);
}

typedef struct {
    const oscene* s;
    const oracle_params* p;
    camera_t cam;
    const int32_t* rows;
    float* film;
    int64_t nrow_pixels;
    atomic_llong casts;
} render_ctx;

static inline void draw2(pcg32_t* rng, int order, float* x, float* y) {
    float a = pcg32_float(rng);
    float b = pcg32_float(rng);
    if (order == 0) { *y = a; *x = b; } else { *x = a; *y = b; }
}

/* One sample of one pixel (main.cpp:391-426): its radiance in L; rng is the
 * pixel's stream at this sample's first draw.  rec (may be NULL) records each
 * cast's ray and hit, for tests/diag that follow one path (oracle_trace_sample). */
typedef struct {
    float* rays;     /* [max_depth][6]: origin, direction */
    int32_t* ids;    /* [max_depth] hit id (-1 miss) */
    float* tuv;      /* [max_depth][3] */
    int32_t n;
} cast_rec;

static void sample_path(const oscene* s, const oracle_params* p, const camera_t* cam, pcg32_t* rng, uint32_t pixel,
                        int32_t px, int32_t py, int32_t smp, float L[3], long long* casts, cast_rec* rec) {
    float contrib[3] = {1.0f, 1.0f, 1.0f};                        /* main.cpp:391 */
    L[0] = L[1] = L[2] = 0.0f;  /* this sample's radiance, added to film once */
    int active = 1;                                               /* main.cpp:392 */
    float xi_x, xi_y;
    draw2(rng, p->rng_order, &xi_x, &xi_y);                       /* main.cpp:395 */
    v3 o = camera_sample_pos(cam, xi_x, xi_y);
    draw2(rng, p->rng_order, &xi_x, &xi_y);                       /* main.cpp:396 */
    v3 d = camera_sample_dir(cam, px, py, o, xi_x, xi_y);
    for (int32_t j = 0; j < p->max_depth; j++) {                  /* main.cpp:399 */
        ohit h; h.id = -1;
        if (active) {                                              /* main.cpp:402-404 */
            wray r;
            r.o[0] = o.x; r.o[1] = o.y; r.o[2] = o.z;
            r.d[0] = d.x; r.d[1] = d.y; r.d[2] = d.z;
            wray_setup(&r);
            trace(s, &r, 0.001f, 1e20f, 1, &h);                   /* ray.h:15-17 */
            if (s->nsph) trace_spheres(s, o, d, 0.001f, 0, &h);   /* smallpt's spheres */
            (*casts)++;
            if (rec) {
                float* q = rec->rays + rec->n * 6;
                q[0] = o.x; q[1] = o.y; q[2] = o.z; q[3] = d.x; q[4] = d.y; q[5] = d.z;
                rec->ids[rec->n] = h.id;
                rec->tuv[rec->n * 3] = h.id == -1 ? 0.0f : h.t;
                rec->tuv[rec->n * 3 + 1] = h.id == -1 ? 0.0f : h.u;
                rec->tuv[rec->n * 3 + 2] = h.id == -1 ? 0.0f : h.v;
                rec->n++;
            }
            if (h.id == -1) {                                     /* main.cpp:407 */
                for (int k = 0; k < 3; k++) L[k] = L[k] + contrib[k] * p->env[k];
            } else if (s->emission) {
                /* emitted radiance at every hit (smallpt's obj.e; the
                 * reference has no emitters — SURVEY §8f row 3) */
                int32_t me = h.id >= 0 ? s->mat[h.id] : s->sph_mat[-2 - h.id];
                if (me >= 0 && me < s->nemit)
                    for (int k = 0; k < 3; k++) L[k] = L[k] + contrib[k] * s->emission[me * 3 + k];
            }
        }
        active = active && (h.id != -1);                          /* main.cpp:410 */
        draw2(rng, p->rng_order, &xi_x, &xi_y);                   /* main.cpp:413 (always drawn) */
        if (!active) continue;
        /* optix_backend.h:469 (position), :483-484 (interpolated shading normal) */
        const int sph = h.id < -1;
        float w = (1.0f - h.u) - h.v;
        v3 n = mk(0.0f, 0.0f, 0.0f);
        if (!sph) {
            const float* nv = &s->n[(int64_t)h.id * 9];
            n = mk((w * nv[0] + h.u * nv[3]) + h.v * nv[6],
                   (w * nv[1] + h.u * nv[4]) + h.v * nv[7],
                   (w * nv[2] + h.u * nv[5]) + h.v * nv[8]);
        }
        v3 hp = mk(o.x + h.t * d.x, o.y + h.t * d.y, o.z + h.t * d.z);
        int32_t m = sph ? s->sph_mat[-2 - h.id] : s->mat[h.id];
        float sw = 1.0f;   /* the scatter weight (glass), applied after roulette */
        v3 out;
        if (!s->nsph && !s->nkind) {
            frame3 f = frame_from_normal(n);                      /* main.cpp:414 */
            v3 lo = cosine_hemisphere(xi_x, xi_y);                /* main.cpp:418, :109-117 */
            out = to_world(&f, lo);                               /* main.cpp:419 */
        } else {
            out = scatter(s, material_kind(s, m), h.id, d, hp, n, xi_x, xi_y, &sw);
        }
        int32_t mt = m;
        if (m < 0 || m >= s->nmat) m = 0;
        float refl[3] = {s->albedo[m * 3], s->albedo[m * 3 + 1], s->albedo[m * 3 + 2]};
#ifdef ORACLE_ALT_TEX1X1
        int tex = 1;  /* every material is an ImageTexture: a 1x1 image of its colour (main.cpp:40-44) */
        const float* timg = (mt >= 0 && mt < s->ntex && s->tex_w[mt] > 0) ? s->tex_rgb[mt] : &s->albedo[m * 3];
        int32_t tw = (mt >= 0 && mt < s->ntex && s->tex_w[mt] > 0) ? s->tex_w[mt] : 1;
        int32_t th = (mt >= 0 && mt < s->ntex && s->tex_w[mt] > 0) ? s->tex_h[mt] : 1;
#else
        int tex = mt >= 0 && mt < s->ntex && s->tex_w[mt] > 0;
        const float* timg = tex ? s->tex_rgb[mt] : NULL;
        int32_t tw = tex ? s->tex_w[mt] : 0, th = tex ? s->tex_h[mt] : 0;
#endif
        if (tex) {
            /* LambertBsdf::sample -> m_reflectance->eval(texcoord) (main.cpp:109-117):
             * texcoord = barycentric_interpolate (optix_backend.h:395-401, add_math.h:4-7) */
            float tu = 0.0f, tv = 0.0f;
            if (s->tc && !sph) {
                const float* c = &s->tc[(int64_t)h.id * 6];
                tu = (w * c[0] + h.u * c[2]) + h.v * c[4];
                tv = (w * c[1] + h.u * c[3]) + h.v * c[5];
            }
            texture_eval(timg, tw, th, tu, tv, refl);
        }
        for (int k = 0; k < 3; k++) contrib[k] = contrib[k] * refl[k];   /* :422 */
        o = hp;                                                   /* main.cpp:423 */
        d = out;                                                  /* main.cpp:424 */
        if (j + 1 >= p->rr_start_depth && j + 1 < p->max_depth) {
            float q = fmaxf(contrib[0], fmaxf(contrib[1], contrib[2]));
            if (q < 1.0f) {
                if (rr_uniform(pixel, (uint32_t)smp, (uint32_t)j) >= q) { active = 0; continue; }
                for (int k = 0; k < 3; k++) contrib[k] = contrib[k] / q;
            }
        }
        for (int k = 0; k < 3; k++) contrib[k] = contrib[k] * sw;  /* smallpt's glass weight */
    }
}

static void render_pixel(void* c_, int64_t li) {
    render_ctx* c = (render_ctx*)c_;
    const oracle_params* p = c->p;
    const oscene* s = c->s;
    int32_t W = p->width;
    int64_t lrow = li / W;
    int32_t px = (int32_t)(li % W);
    int32_t py = c->rows[lrow];
    uint32_t pixel = (uint32_t)py * (uint32_t)W + (uint32_t)px;   /* main.cpp:379-382 */
    pcg32_t rng;
    pcg32_seed(&rng, p->rng_initstate, (uint64_t)pixel);          /* main.cpp:376 */
    float film[3] = {0.0f, 0.0f, 0.0f};
    long long casts = 0;
    for (int32_t smp = 0; smp < p->spp; smp++) {                  /* main.cpp:385 */
        float L[3];
        sample_path(s, p, &c->cam, &rng, pixel, px, py, smp, L, &casts, NULL);
        /* Without emitters L is 0 or contrib * env: the same film sum as the
         * reference's per-miss film += contrib (main.cpp:407). */
        for (int k = 0; k < 3; k++) film[k] = film[k] + L[k];
    }
    int64_t npx = c->nrow_pixels;
    for (int k = 0; k < 3; k++) c->film[k * npx + li] = film[k] / (float)p->spp; /* main.cpp:429 */
    atomic_fetch_add(&c->casts, casts);
}

/* Diagnostics (tools/diag_parity.py): the casts of sample `smp` of pixel (px,
 * py) — each cast's ray and closest hit — and the sample's radiance.  Returns
 * the number of casts (at most max_depth). */
int32_t oracle_trace_sample(void* scene, const oracle_params* p, int32_t px, int32_t py, int32_t smp, float* rays,
                            int32_t* ids, float* tuv, float* L3) {
    const oscene* s = (const oscene*)scene;
    camera_t cam;
    camera_setup(&cam, p);
    uint32_t pixel = (uint32_t)py * (uint32_t)p->width + (uint32_t)px;
    pcg32_t rng;
    pcg32_seed(&rng, p->rng_initstate, (uint64_t)pixel);
    long long casts = 0;
    float L[3];
    for (int32_t k = 0; k < smp; k++) sample_path(s, p, &cam, &rng, pixel, px, py, k, L, &casts, NULL);
    cast_rec rec = {rays, ids, tuv, 0};
    sample_path(s, p, &cam, &rng, pixel, px, py, smp, L3, &casts, &rec);
    return rec.n;
}

int oracle_render(void* scene, const oracle_params* p, const int32_t* rows, int32_t nrows,
                  float* film, int32_t nthreads, uint64_t* ray_casts_out) {
    if (!scene || !p || p->width <= 0 || p->height <= 0 || p->spp <= 0 || p->max_depth <= 0) return -1;
    for (int32_t i = 0; i < nrows; i++)
        if (rows[i] < 0 || rows[i] >= p->height) return -2;
    render_ctx c;
    c.s = (const oscene*)scene;
    c.p = p;
    camera_setup(&c.cam, p);
    c.rows = rows;
    c.film = film;
    c.nrow_pixels = (int64_t)nrows * p->width;
    atomic_init(&c.casts, 0);
    parallel_for(c.nrow_pixels, 64, nthreads, render_pixel, &c);
    if (ray_casts_out) *ray_casts_out = (uint64_t)atomic_load(&c.casts);
    return 0;
}
