/*
 * oracle.h — CPU restatement of the reference path tracer.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libspt.so, the HIP kernels,
 * the host driver) links, includes or calls this code.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it, as the
 * checker / CPU baseline.
 *
 * Parity status: PCG32 is pinned by the canonical pcg32 known-answer vector
 * (tests/test_oracle.py).  The reference itself cannot be built in this
 * container (no CUDA, OptiX, Enoki or tinyobjloader; DiffuseBsdf undefined at
 * main.cpp:234) and ships no tests or golden vectors, so the geometry /
 * shading arithmetic is "parity unpinned" beyond the analytic and
 * formula-derived known answers in tests/test_oracle.py.
 */
#ifndef SPT_ORACLE_H
#define SPT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_params {
    int32_t width, height, spp, max_depth;   /* main.cpp:357-361 (max_depth = ray casts) */
    float look_from[3], look_at[3], up[3];   /* main.cpp:383 */
    float lens_radius, focal_dist, fov_y, film_size_y; /* pinhole.h:9-16 */
    int32_t rng_order;       /* 0 = y-first (MSVC/GCC arg order), 1 = x-first */
    int32_t rr_start_depth;  /* RR from this cast index on; >= max_depth disables */
    float env[3];            /* sky radiance on miss (main.cpp:407 = 1) */
    uint64_t rng_initstate;  /* PCG32_DEFAULT_STATE (main.cpp:376) */
} oracle_params;

void* oracle_scene_create(const int32_t* pos_tri, const float* pos, int64_t nvert, int64_t ntri,
                          const int32_t* nrm_tri, const float* nrm, int64_t nnrm,
                          const int32_t* mat_id, const float* albedo, int32_t nmat,
                          int32_t use_bvh);
void oracle_scene_destroy(void* scene);
/* Per-material emission (nmat x 3), NULL/0 = none (see oracle_render). */
void oracle_scene_set_emission(void* scene, const float* emission, int32_t nmat);
/* Texcoord triplets + texcoords (main.cpp:141-251 layout); missing (-1) -> (0, 0). */
void oracle_scene_set_texcoords(void* scene, const int32_t* tc_tri, const float* tc, int64_t ntc);
/* Material mat's reflectance image (ImageTexture, main.cpp:34-80): interleaved RGB,
 * w x h texels; rgb NULL removes it (the albedo constant applies). */
void oracle_scene_set_texture(void* scene, int32_t mat, const float* rgb, int32_t w, int32_t h);
/* smallpt's analytic spheres: n x (cx, cy, cz, r) and a material per sphere,
 * tested after the triangles (id -2 - k); kinds: SPT_MAT_* per material
 * (0 diffuse, 1 mirror, 2 glass). */
void oracle_scene_set_spheres(void* scene, const float* center_radius, const int32_t* mat, int32_t n);
void oracle_scene_set_material_kinds(void* scene, const uint32_t* kinds, int32_t n);
void oracle_texture_eval(const float* rgb, int32_t w, int32_t h, float u, float v, float* out3);

/* wavefront_isect.cu:80-112 semantics: masked lanes untouched; miss -> id -1. */
void oracle_intersect(void* scene, const float* ox, const float* oy, const float* oz,
                      const float* dx, const float* dy, const float* dz,
                      const float* tmin, const float* tmax, const uint8_t* mask,
                      uint32_t mask_size, int32_t* tri_id, float* t, float* u, float* v,
                      int64_t n, int32_t do_closest, int32_t nthreads);

/* main.cpp:354-446.  Renders rows[0..nrows) (global row indices) into
 * film[3][nrows][width] (planar RGB, already divided by spp). */
int oracle_render(void* scene, const oracle_params* p, const int32_t* rows, int32_t nrows,
                  float* film, int32_t nthreads, uint64_t* ray_casts_out);

/* Known-answer helpers. */
void oracle_pcg32_seq(uint64_t initstate, uint64_t initseq, uint32_t* out, int32_t n);
void oracle_pcg32_floats(uint64_t initstate, uint64_t initseq, float* out, int32_t n);
/* tools/diag_parity.py: the casts (ray, closest hit) of one sample of one pixel */
int32_t oracle_trace_sample(void* scene, const oracle_params* p, int32_t px, int32_t py, int32_t smp, float* rays,
                            int32_t* ids, float* tuv, float* L3);
void oracle_camera_ray(const oracle_params* p, int32_t px, int32_t py, const float* xi4,
                       float* org3, float* dir3, float* basis9);
void oracle_sincos(float x, float* s, float* c);
void oracle_cosine_hemisphere(float xi_x, float xi_y, float* out3);
void oracle_disk_from_square(float xi_x, float xi_y, float* out2);
void oracle_frame_to_world(const float* n3, const float* local3, float* out3);

#ifdef __cplusplus
}
#endif
#endif
