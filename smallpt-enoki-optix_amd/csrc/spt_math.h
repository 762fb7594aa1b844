// spt_math.h — __host__ __device__ math of the hot path (camera, PCG32,
// sampling, shading frame, watertight triangle test).  Compiled by hipcc for
// gfx950 (kernels) and for the host (camera constants, jump tables).
//
// Floating point: every translation unit is built with -ffp-contract=off and
// correctly rounded f32 division/sqrt; every FMA below is an explicit fmaf().
// The op order of each function is the specification the CPU oracle
// (oracle/oracle.c) restates independently; parity tests compare bitwise.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SPT_HD __host__ __device__ __forceinline__

namespace spt {

constexpr float kPi = 3.14159265358979323846f;
constexpr uint64_t kPcgMult = 0x5851f42d4c957f2dULL;
constexpr uint64_t kPcgDefaultState = 0x853c49e6748fea9bULL;  // main.cpp:376
constexpr float kRayTmin = 0.001f;                             // ray.h:16
constexpr float kRayTmax = 1e20f;                              // ray.h:16
constexpr float kBoxPad = 1.000001f;  // conservative slab exit (Ize 2013 + margin)

SPT_HD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
SPT_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
// n / d for a wave-uniform d: a shift when d is a power of two (image sizes,
// sample counts), the divide otherwise
SPT_HD uint32_t udiv(uint32_t n, uint32_t d) {
    if ((d & (d - 1u)) == 0u) return n >> (uint32_t)__builtin_ctz(d);
    return n / d;
}

// ------------------------------------------------------------------ PCG32
// Enoki random.h (external): next_uint32 / next_float32; seeded at
// main.cpp:376 with initseq = pixel index.
struct Pcg32 {
    uint64_t state, inc;
    SPT_HD uint32_t next() {
        uint64_t old = state;
        state = old * kPcgMult + inc;
        uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (xs >> rot) | (xs << ((32u - rot) & 31u));
    }
    SPT_HD float next_float() { return u2f((next() >> 9) | 0x3f800000u) - 1.0f; }
    SPT_HD void seed(uint64_t initstate, uint64_t initseq) {
        state = 0;
        inc = (initseq << 1u) | 1u;
        next();
        state += initstate;
        next();
    }
};

// Jump-ahead: after n steps, state' = mul * state + add * inc (mod 2^64).
struct PcgJump { uint64_t mul, add; };
SPT_HD PcgJump pcg_jump_coeffs(uint64_t n) {
    uint64_t acc_mul = 1, acc_add = 0, cur_mul = kPcgMult, cur_add = 1;
    while (n > 0) {
        if (n & 1) { acc_mul *= cur_mul; acc_add = acc_add * cur_mul + cur_add; }
        cur_add = (cur_mul + 1) * cur_add;
        cur_mul *= cur_mul;
        n >>= 1;
    }
    return {acc_mul, acc_add};
}
SPT_HD uint64_t pcg_apply(PcgJump j, uint64_t state, uint64_t inc) { return j.mul * state + j.add * inc; }
// seed(initstate S0, initseq) followed by jump j, as one affine map of the
// stream constant inc = 2 initseq + 1: seed leaves state (inc + S0) M + inc,
// the jump maps it to mul ((inc + S0) M + inc) + add inc = A inc + B with
// A = mul (M + 1) + add and B = mul S0 M (mod 2^64) — one 64-bit multiply-add
// per path start instead of three multiplies.  Stored as PcgJump {A, B}.
SPT_HD PcgJump pcg_seeded_jump(uint64_t S0, PcgJump j) {
    return {j.mul * (kPcgMult + 1u) + j.add, j.mul * S0 * kPcgMult};
}
SPT_HD Pcg32 pcg_start(PcgJump seeded, uint64_t initseq) {
    Pcg32 r;
    r.inc = (initseq << 1u) | 1u;
    r.state = seeded.mul * r.inc + seeded.add;
    return r;
}

// Real2C(next(), next()) — argument evaluation order is unspecified in the
// reference (main.cpp:395,396,413); y-first = first draw to .y.
SPT_HD void draw2(Pcg32& r, uint32_t order, float& x, float& y) {
    float a = r.next_float();
    float b = r.next_float();
    if (order == 0) { y = a; x = b; } else { x = a; y = b; }
}

// ------------------------------------------------------------------ sincos
// Cephes single-precision joint sin/cos (Enoki's sincos; used at mapping.h:9,25).
SPT_HD void sincos_cephes(float x, float& s_out, float& c_out) {
    float xa = fabsf(x);
    int32_t j = (int32_t)(xa * 1.2732395447351626862f);
    j = (j + 1) & ~1;
    float y = (float)j;
    uint32_t sign_sin = (((uint32_t)j << 29) & 0x80000000u) ^ (f2u(x) & 0x80000000u);
    uint32_t sign_cos = ((uint32_t)(~(j - 2)) << 29) & 0x80000000u;
    y = ((xa - y * 0.78515625f) - y * 2.4187564849853515625e-4f) - y * 3.77489497744594108e-8f;
    float z = y * y;
    float s = fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f) * z;
    float c = fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f) * z;
    s = fmaf(s, y, y);
    c = fmaf(c, z, fmaf(z, -0.5f, 1.0f));
    bool poly = (j & 2) == 0;
    float rs = poly ? s : c;
    float rc = poly ? c : s;
    s_out = u2f(f2u(rs) ^ sign_sin);
    c_out = u2f(f2u(rc) ^ sign_cos);
}

// ------------------------------------------------------------------ vectors
struct V3 { float x, y, z; };
SPT_HD V3 v3(float x, float y, float z) { return {x, y, z}; }
SPT_HD V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
SPT_HD float dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
SPT_HD V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
// Enoki normalize = v * rsqrt(|v|^2), restated as v * (1 / sqrt(|v|^2)).
SPT_HD V3 normalize(V3 v) {
    float inv = 1.0f / sqrtf(dot(v, v));
    return {v.x * inv, v.y * inv, v.z * inv};
}
SPT_HD float comp(V3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }

// Frame3 (coordframe.h:5-51): columns bx, by, bz; to_world = M * l.
struct Frame { V3 bx, by, bz; };
SPT_HD V3 to_world(const Frame& f, V3 l) {
    return {(f.bx.x * l.x + f.by.x * l.y) + f.bz.x * l.z,
            (f.bx.y * l.x + f.by.y * l.y) + f.bz.y * l.z,
            (f.bx.z * l.x + f.by.z * l.y) + f.bz.z * l.z};
}
SPT_HD V3 to_local(const Frame& f, V3 w) { return {dot(f.bx, w), dot(f.by, w), dot(f.bz, w)}; }
// coordframe.h:17-30; the normal is used as given (not renormalised).
SPT_HD Frame frame_from_normal(V3 n) {
    float sign = copysignf(1.0f, n.y);
    float a = -1.0f / (sign + n.y);
    float b = (n.z * n.x) * a;
    Frame f;
    f.bx = {sign + (n.x * n.x) * a, -n.x, b};
    f.by = n;
    f.bz = {sign * b, (-sign) * n.z, 1.0f + ((sign * n.z) * n.z) * a};
    return f;
}

// mapping.h:5-11 (local +y is the normal).
SPT_HD V3 cosine_hemisphere(float xi_x, float xi_y) {
    float sin_phi = sqrtf(1.0f - xi_x);
    float theta = (kPi * 2.0f) * xi_y;
    float s, c;
    sincos_cephes(theta, s, c);
    return {c * sin_phi, sqrtf(xi_x), s * sin_phi};
}
// mapping.h:15-27.
SPT_HD void disk_from_square(float xi_x, float xi_y, float& ox, float& oy) {
    float ax = xi_x * 2.0f - 1.0f, ay = xi_y * 2.0f - 1.0f;
    float ax2 = ax * ax, ay2 = ay * ay;
    bool cond = ax2 > ay2;
    float r = cond ? ax : ay;
    // one divide for either branch (the lanes of a wave take both)
    const float q = (cond ? ay : ax) / (cond ? ax : ay);
    float phi = cond ? (kPi / 4.0f) * q : (kPi / 2.0f) - (kPi / 4.0f) * q;
    float s, c;
    sincos_cephes(phi, s, c);
    ox = r * c;
    oy = r * s;
}

// ------------------------------------------------------------------ camera
// ThinlensCamera (pinhole.h:7-72); the constants are computed once on the host.
struct Camera {
    V3 origin;
    Frame frame;
    float lens_radius, focal_dist, dist_lens_to_film, ratio, film_y;
    float fw, fh;  // image resolution as float
    // 1 / fw and 1 / fh when fw, fh are powers of two, else 0: then x / fw and
    // x * (1 / fw) are the same correctly rounded value, bit for bit
    float inv_fw, inv_fh;
    float focal_z;  // (focal_dist * fz) / fz of sample_dir (pinhole.h:47), a per-camera constant
};

// pinhole.h:27-32
SPT_HD V3 camera_sample_pos(const Camera& c, float xi_x, float xi_y) {
    float lx, ly;
    disk_from_square(xi_x, xi_y, lx, ly);
    lx = lx * c.lens_radius;
    ly = ly * c.lens_radius;
    V3 w = to_world(c.frame, v3(lx, 0.0f, ly));
    return {w.x + c.origin.x, w.y + c.origin.y, w.z + c.origin.z};
}
// pinhole.h:34-56
SPT_HD V3 camera_sample_dir(const Camera& c, uint32_t px, uint32_t py, V3 pos, float xi_x, float xi_y) {
    V3 lens = to_local(c.frame, pos - c.origin);
    float ndc_x, ndc_y;
    if (c.inv_fw != 0.0f) ndc_x = ((float)px + xi_x) * c.inv_fw;
    else ndc_x = ((float)px + xi_x) / c.fw;
    if (c.inv_fh != 0.0f) ndc_y = ((float)py + xi_y) * c.inv_fh;
    else ndc_y = ((float)py + xi_y) / c.fh;
    float fx = (0.5f - ndc_x) * (c.ratio * c.film_y);
    float fy = (0.5f - ndc_y) * c.film_y;
    float fz = c.dist_lens_to_film;
    V3 focal = {(c.focal_dist * fx) / fz, (c.focal_dist * fy) / fz, c.focal_z};
    return to_world(c.frame, normalize(focal - lens));
}

// --------------------------------------------------------------- triangles
// Watertight ray/triangle test (Woop, Benthin, Wald 2013) standing in for
// OptiX's built-in triangle intersector (optix_backend.h:314-324), with the
// double-precision edge fallback.  Barycentrics follow OptiX / add_math.h:6:
// p = (1-u-v) v0 + u v1 + v v2.
struct WoopRay {
    V3 o;
    uint32_t k;  // kx | ky << 2 | kz << 4 (one register on the device)
    float Sx, Sy, Sz;
    SPT_HD int kx() const { return (int)(k & 3u); }
    SPT_HD int ky() const { return (int)((k >> 2) & 3u); }
    SPT_HD int kz() const { return (int)(k >> 4); }
};
SPT_HD WoopRay woop_setup(V3 o, V3 d) {
    float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    int kz = (ax > ay) ? ((ax > az) ? 0 : 2) : ((ay > az) ? 1 : 2);
    int kx = kz + 1; if (kx == 3) kx = 0;
    int ky = kx + 1; if (ky == 3) ky = 0;
    float dkz = comp(d, kz);
    // Woop et al. swap kx and ky when d_kz < 0 to keep the winding; this test
    // accepts both windings, and with kx and ky swapped every nonzero edge
    // function, det and T change sign exactly (IEEE round-to-nearest is
    // symmetric), so every accept decision and, with zeros made +0 (woop_core),
    // every bit of t, u, v are the same: the device keeps the cyclic order
    // (kx, ky, kz), which the rotated triangle records hold (spt_internal.h);
    // the oracle keeps the swap (oracle.c wray_setup), an independent check of
    // that identity (tests/test_woop_rotated.py).
    WoopRay r;
    r.o = o; r.k = (uint32_t)kx | (uint32_t)ky << 2 | (uint32_t)kz << 4;
    // one correctly rounded divide, then two products (Woop et al. divide
    // three times): config 1 +1.1 % from the ray set-up alone; the oracle
    // computes the same (oracle.c wray_setup)
    r.Sz = 1.0f / dkz;
    r.Sx = comp(d, kx) * r.Sz;
    r.Sy = comp(d, ky) * r.Sz;
    return r;
}

// The sheared, permuted vertices (Woop et al. 2013 §3), and for the box-exit
// rule below the triangle's farthest vertex offset along the ray's motion in
// kx and in ky (ex, ey: max of sign(d_k) * (v_k - o_k) over the vertices).
struct WoopShear {
    float Akz, Bkz, Ckz, Ax, Ay, Bx, By, Cx, Cy;
    float ex, ey;
};
// sign(d_kx) = sign(Sx) * sign(Sz), so the direction itself need not be kept
SPT_HD float exit_offset(float a, float b, float c, float S, float Sz) {
    // (a branch-free select of both maxima, or an xor of the sign bits, made
    // the isect kernel spill at its 64-VGPR budget; this form does not)
    const bool neg = ((f2u(S) ^ f2u(Sz)) >> 31) != 0u;
    return neg ? -fminf(fminf(a, b), c) : fmaxf(fmaxf(a, b), c);
}
SPT_HD WoopShear woop_shear(const WoopRay& r, V3 p0, V3 p1, V3 p2) {
    V3 A = p0 - r.o, B = p1 - r.o, C = p2 - r.o;
    const int kx = r.kx(), ky = r.ky(), kz = r.kz();
    WoopShear w;
    w.Akz = comp(A, kz); w.Bkz = comp(B, kz); w.Ckz = comp(C, kz);
    const float Akx = comp(A, kx), Bkx = comp(B, kx), Ckx = comp(C, kx);
    const float Aky = comp(A, ky), Bky = comp(B, ky), Cky = comp(C, ky);
    w.ex = exit_offset(Akx, Bkx, Ckx, r.Sx, r.Sz);
    w.ey = exit_offset(Aky, Bky, Cky, r.Sy, r.Sz);
    w.Ax = Akx - r.Sx * w.Akz; w.Ay = Aky - r.Sy * w.Akz;
    w.Bx = Bkx - r.Sx * w.Bkz; w.By = Bky - r.Sy * w.Bkz;
    w.Cx = Ckx - r.Sx * w.Ckz; w.Cy = Cky - r.Sy * w.Ckz;
    return w;
}

// Box-exit rule: a hit is kept only if the ray has not left the triangle's
// own bounding box before tmin.  Exactly, a point of the triangle lies in its
// box, so a ray that left the box before tmin cannot meet the triangle at
// t >= tmin; a Woop t just past tmin there is rounding (the origin on or next
// to the triangle's plane).  Without the rule such a hit is kept or not
// depending on whether the tree's boxes around it are culled at tmin (a tight
// box drops it, a loose one keeps it: DESIGN.md §2), so the closest hit would
// depend on the acceleration structure, which wavefront_isect.cu:103 does not
// allow.  Per axis k the exit is E_k = (farthest vertex offset) / |d_k|:
//   kz: E = max(Az, Bz, Cz)  (Az = Sz (v_kz - o_kz) is already in t units),
//   kx: E = ex |Sz| / |Sx|   (|d_kx| = |Sx| / |Sz|), ky likewise,
// tested as pad_up(E) < tmin without a divide.  Each side has <= 4 ulps of
// rounding, under the pad's 8.4 (toward +inf: x kBoxPad when E >= 0, x
// kBoxPadLo when E < 0, which a negative per-ray tmin allows), so a hit whose
// exact box exit is >= tmin is never dropped; and node culling runs at
// cull_tmin() (4e-6 below tmin) so a box the tree culls holds only triangles
// this rule drops anyway.  For tmin > 0 the negative branch never decides
// (E < 0 is below tmin either way), so the render's bits do not depend on it.
#ifndef SPT_TRI_BOX_RULE
#define SPT_TRI_BOX_RULE 1
#endif
constexpr float kCullTminRel = 4e-6f;
SPT_HD float cull_tmin(float tmin) { return tmin - fabsf(tmin) * kCullTminRel; }
constexpr float kBoxPadLo = 0.999999f;  // the pad for a negative exit (toward +inf)
SPT_HD float pad_up(float x) { return x * (x >= 0.0f ? kBoxPad : kBoxPadLo); }
SPT_HD bool left_box_before_tmin(const WoopRay& r, const WoopShear& w, float Az, float Bz, float Cz, float tmin) {
    if (pad_up(fmaxf(fmaxf(Az, Bz), Cz)) < tmin) return true;
    const float asz = fabsf(r.Sz);
    if (pad_up(w.ex * asz) < tmin * fabsf(r.Sx)) return true;
    return pad_up(w.ey * asz) < tmin * fabsf(r.Sy);
}

// The same shear from vertices and origin already in (kx, ky, kz) order
// (rotated triangle records): A = P0 - O component by component, which is
// comp(p0 - o, k) bit for bit.
SPT_HD WoopShear woop_shear_rot(const WoopRay& r, V3 O, V3 P0, V3 P1, V3 P2) {
    const V3 A = P0 - O, B = P1 - O, C = P2 - O;
    WoopShear w;
    w.Akz = A.z; w.Bkz = B.z; w.Ckz = C.z;
    w.ex = exit_offset(A.x, B.x, C.x, r.Sx, r.Sz);
    w.ey = exit_offset(A.y, B.y, C.y, r.Sy, r.Sz);
    w.Ax = A.x - r.Sx * w.Akz; w.Ay = A.y - r.Sy * w.Akz;
    w.Bx = B.x - r.Sx * w.Bkz; w.By = B.y - r.Sy * w.Bkz;
    w.Cx = C.x - r.Sx * w.Ckz; w.Cy = C.y - r.Sy * w.Ckz;
    return w;
}

struct NoReload {  // the vertices stay in registers (host)
    V3 p0, p1, p2;
    SPT_HD void operator()(V3& q0, V3& q1, V3& q2) const { q0 = p0; q1 = p1; q2 = p2; }
};

// Returns true with t/u/v when hit at t in [tmin, tmax] (NaN-safe).  The
// double-precision edge fallback (an edge function exactly 0) re-derives the
// sheared vertices from reload() — on the device a re-read of the triangle,
// so the single-precision path does not keep them live.
//
// woop_test_raw stops before the barycentric divides: it returns t and the
// edge functions V, W with det, so a caller that keeps only the closest hit
// divides once, u = V / det and v = W / det, for the hit it keeps (the same
// correctly rounded quotients).
template <typename Reshear>
SPT_HD bool woop_core(const WoopRay& r, const WoopShear& w, Reshear reshear, float tmin, float tmax,
                      float& t_out, float& V_out, float& W_out, float& det_out) {
    const float Akz = w.Akz, Bkz = w.Bkz, Ckz = w.Ckz;
    float U = w.Cx * w.By - w.Cy * w.Bx;
    float V = w.Ax * w.Cy - w.Ay * w.Cx;
    float W = w.Bx * w.Ay - w.By * w.Ax;
    if (U == 0.0f || V == 0.0f || W == 0.0f) {
        const WoopShear x = reshear();
        // px qy - py qx for (p, q) = (C, B), (A, C), (B, A): one per iteration
        // of a rolled loop (the rotation keeps few doubles live at a time)
        float px = x.Cx, py = x.Cy, qx = x.Bx, qy = x.By, rx = x.Ax, ry = x.Ay;
        float e0 = 0.0f, e1 = 0.0f, e2 = 0.0f;
#pragma unroll 1
        for (int i = 0; i < 3; i++) {
            const float e = (float)((double)px * (double)qy - (double)py * (double)qx);
            e0 = e1; e1 = e2; e2 = e;
            const float tx = rx, ty = ry;
            rx = qx; ry = qy; qx = px; qy = py; px = tx; py = ty;
        }
        U = e0; V = e1; W = e2;
    }
    if ((U < 0.0f || V < 0.0f || W < 0.0f) && (U > 0.0f || V > 0.0f || W > 0.0f)) return false;
    float det = (U + V) + W;
    if (det == 0.0f) return false;
    float Az = r.Sz * Akz, Bz = r.Sz * Bkz, Cz = r.Sz * Ckz;
    float T = (U * Az + V * Bz) + W * Cz;
    float t = T / det;
    if (!(t >= tmin && t <= tmax)) return false;
#if SPT_TRI_BOX_RULE
    if (left_box_before_tmin(r, w, Az, Bz, Cz, tmin)) return false;
#endif
    // + 0.0f: a zero t, u or v is +0.  Its sign would otherwise follow det's,
    // which the kx / ky order flips (the oracle keeps Woop's swap, the device
    // does not): with it every output bit is independent of that order.
    t_out = t + 0.0f;
    V_out = V;
    W_out = W;
    det_out = det;
    return true;
}

// The vertices in world order (the BVH2 tracer, the host).
template <typename Reload>
SPT_HD bool woop_test_raw(const WoopRay& r, V3 p0, V3 p1, V3 p2, Reload reload, float tmin, float tmax,
                          float& t_out, float& V_out, float& W_out, float& det_out) {
    const auto reshear = [&]() {
        V3 q0, q1, q2;
        reload(q0, q1, q2);
        return woop_shear(r, q0, q1, q2);
    };
    return woop_core(r, woop_shear(r, p0, p1, p2), reshear, tmin, tmax, t_out, V_out, W_out, det_out);
}

// The vertices and origin already in (kx, ky, kz) order (rotated records):
// reload() re-reads the rotated vertices.
template <typename Reload>
SPT_HD bool woop_test_raw_rot(const WoopRay& r, V3 O, V3 P0, V3 P1, V3 P2, Reload reload, float tmin, float tmax,
                              float& t_out, float& V_out, float& W_out, float& det_out) {
    const auto reshear = [&]() {
        V3 q0, q1, q2;
        reload(q0, q1, q2);
        return woop_shear_rot(r, O, q0, q1, q2);
    };
    return woop_core(r, woop_shear_rot(r, O, P0, P1, P2), reshear, tmin, tmax, t_out, V_out, W_out, det_out);
}

template <typename Reload>
SPT_HD bool woop_test(const WoopRay& r, V3 p0, V3 p1, V3 p2, Reload reload, float tmin, float tmax,
                      float& t_out, float& u_out, float& v_out) {
    float V, W, det;
    if (!woop_test_raw(r, p0, p1, p2, reload, tmin, tmax, t_out, V, W, det)) return false;
    u_out = V / det + 0.0f;
    v_out = W / det + 0.0f;
    return true;
}

template <typename Reload>
SPT_HD bool woop_test_rot(const WoopRay& r, V3 O, V3 P0, V3 P1, V3 P2, Reload reload, float tmin, float tmax,
                          float& t_out, float& u_out, float& v_out) {
    float V, W, det;
    if (!woop_test_raw_rot(r, O, P0, P1, P2, reload, tmin, tmax, t_out, V, W, det)) return false;
    u_out = V / det + 0.0f;
    v_out = W / det + 0.0f;
    return true;
}

// ------------------------------------------------------------ roulette
// Russian-roulette side stream (a build addition: the reference has none,
// SURVEY F7/A14).  Counter-based so the 4+2D PCG32 draw layout is untouched.
SPT_HD float rr_uniform(uint32_t pixel, uint32_t sample, uint32_t depth) {
    uint32_t h = pixel * 0x9E3779B1u ^ (sample + 0x7F4A7C15u) * 0x85EBCA77u ^ (depth + 1u) * 0xC2B2AE3Du;
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
    return (float)(h >> 8) * (1.0f / 16777216.0f);
}

}  // namespace spt
