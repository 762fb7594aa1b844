/*
 * spt.h — C ABI of the MI355X-native wavefront path tracer (the drop-in
 * boundary for the reference's OptiX backend + Enoki bounce loop).
 *
 * Plain C: pointers, sizes, status codes.  Device buffers are HIP device
 * pointers (hipMalloc / torch CUDA tensors); `stream` is a hipStream_t passed
 * as void* (NULL = default stream).  Citations are reference paths:lines
 * (jamornsriwasansak/smallpt-enoki-optix).
 *
 * Error behaviour: every call returns SPT_OK (0) or an error code and stores a
 * message for spt_last_error() (the reference throws std::runtime_error from
 * OPTIX_CHECK / CUDA_CHECK, optix_backend.h:25-66; the C++ host wrapper in
 * smallpt-enoki-optix_amd/csrc/spt.hpp rethrows with that convention).
 */
#ifndef SPT_H
#define SPT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t spt_status;
enum {
    SPT_OK = 0,
    SPT_ERR_INVALID = 1,   /* bad argument / shape */
    SPT_ERR_HIP = 2,       /* HIP runtime failure */
    SPT_ERR_NO_DEVICE = 3, /* no GPU visible */
    SPT_ERR_OOM = 4,       /* device allocation failed */
    SPT_ERR_IO = 5,        /* file could not be read / written */
    SPT_ERR_LIMIT = 6      /* size beyond a documented limit */
};

typedef struct spt_scene_t* spt_scene;

/* SoA ray planes — optixdata.h:13-20 (Params::m_ray_*), ray.h:28-31. */
typedef struct spt_rays {
    const float* ox; const float* oy; const float* oz;
    const float* dx; const float* dy; const float* dz;
    const float* tmin; const float* tmax;
} spt_rays;

/* SoA hit planes — optixdata.h:23-26 (m_result_tri_id / _t / _barycentric_u / _v). */
typedef struct spt_hits {
    int32_t* tri_id; float* t; float* u; float* v;
} spt_hits;

/* Reconstructed surface — optix_backend.h:99-134 (TriangleHitInfo) plus the
 * material id gathered by Scene::intersect (main.cpp:325).  Each plane pointer
 * may be NULL on its own to skip that output (e.g. px alone).  Planar SoA, n
 * elements per plane. */
typedef struct spt_hit_info {
    float* px; float* py; float* pz;          /* position o + t d          (:469)     */
    float* gnx; float* gny; float* gnz;       /* geometric normal          (:472-476) */
    float* snx; float* sny; float* snz;       /* shading normal, un-normalised (:483-484) */
    float* tcu; float* tcv;                   /* texcoord                  (:479-480) */
    int32_t* mat_id;                          /* material id (obj id + 1)  (main.cpp:325) */
} spt_hit_info;

/* ThinlensCamera — pinhole.h:9-16, constructed at main.cpp:383. */
typedef struct spt_camera {
    float look_from[3];
    float look_at[3];
    float up[3];
    float lens_radius;
    float focal_dist;
    float fov_y;        /* radians */
    float film_size_y;  /* 0.035 default (pinhole.h:11) */
} spt_camera;

enum {
    SPT_RNG_Y_FIRST = 0,  /* Real2C(a, b) with b drawn first (MSVC/GCC order) */
    SPT_RNG_X_FIRST = 1
};

enum {
    SPT_FLAG_TIMING = 1u,          /* record HIP events around every isect launch (isect_ms) */
    SPT_FLAG_TRAVERSAL_STATS = 2u, /* count node visits / triangle tests (slower variant; wavefront) */
    SPT_FLAG_FUSED = 4u,           /* one persistent trace+shade kernel per sample chunk */
    SPT_FLAG_WAVEFRONT = 8u,       /* isect / shade / refill kernels over path queues, with the
                                      drain (neither flag: spt_config.pipeline; AUTO = fused iff
                                      the tile has at most fused_max_paths paths, 2^20 by default,
                                      or at most wavefront_paths when that is set) */
    SPT_FLAG_TIMING_ALL = 16u      /* with SPT_FLAG_TIMING: also shade / refill / resolve launches */
};

/* The render loop of main.cpp:354-429 plus the tile/wavefront knobs. */
typedef struct spt_render_params {
    uint32_t width, height;     /* main.cpp:357-358 */
    uint32_t spp;               /* main.cpp:360 */
    uint32_t max_depth;         /* ray casts per path, main.cpp:361 (num_bounces) */
    spt_camera camera;
    /* Interleaved row-group tiling: global row r belongs to tile
     * (r / rows_per_group) % tile_count.  tile_count = 1 renders the image. */
    uint32_t tile_index, tile_count, rows_per_group;
    uint32_t wavefront_paths;   /* paths in flight per launch (0 = the scene's config: 32M) */
    uint32_t rr_start_depth;    /* Russian roulette from this cast on (>= max_depth: off) */
    uint32_t rng_order;         /* SPT_RNG_* */
    uint64_t rng_initstate;     /* PCG32_DEFAULT_STATE 0x853c49e6748fea9b (main.cpp:376) */
    float env[3];               /* sky radiance on miss, 1 in the reference (main.cpp:407) */
    uint32_t flags;             /* SPT_FLAG_* */
} spt_render_params;

typedef struct spt_render_stats {
    uint64_t paths;             /* paths rendered by this call, counted on the device (= paths_terminated);
                                   a complete render has paths == tile pixels x spp */
    uint64_t ray_casts;         /* closest/any-hit queries traced */
    uint64_t continuations;     /* paths that bounced into a next cast */
    uint64_t regenerations;     /* camera rays started by refills after the first launch */
    uint64_t iterations;        /* isect+shade+refill rounds (each over every sub-wavefront) */
    uint32_t paths_in_flight;   /* wavefront capacity (queue slots) */
    uint32_t tile_rows;
    double isect_ms, shade_ms, camera_ms, resolve_ms; /* isect: SPT_FLAG_TIMING; others: + SPT_FLAG_TIMING_ALL (camera = refills) */
    double total_ms;            /* host wall time of the call (includes final sync) */
    uint64_t isect_nodes;       /* SPT_FLAG_TRAVERSAL_STATS: inner nodes visited (all lanes) */
    uint64_t isect_tris;        /*   triangle tests */
    uint64_t isect_lane_steps;  /*   traversal loop iterations summed over lanes */
    uint64_t isect_wave_steps;  /*   traversal loop iterations summed over waves */
    uint64_t isect_launches;    /* SPT_FLAG_TIMING: isect launches timed (all streams) */
    uint32_t streams;           /* sub-wavefronts (HIP streams) used (spt_config.streams) */
    uint32_t fused;             /* 1: the fused pipeline ran, 0: the wavefront */
    double isect_busy_ms;       /* SPT_FLAG_TIMING: union of the isect launch intervals
                                   (launches on the K streams overlap; isect_ms sums them) */
    uint64_t isect_max_stack;   /* SPT_FLAG_TRAVERSAL_STATS: deepest LDS stack entry used */
    /* Work accounting, counted on the device (not derived from the params):
     * every (sample, pixel) of the tile is one path; a complete render has
     * paths_started == paths_terminated == tile pixels x spp and
     * film_slots_unwritten == 0, which together mean every path's film slot
     * was written exactly once (main.cpp:385-429 renders every pixel x sample). */
    uint64_t paths_started;     /* camera rays generated (refill launches / fused kernel) */
    uint64_t paths_terminated;  /* paths that ended: casts - continuations, from the queue counts */
    uint64_t film_slots_unwritten; /* per-(sample, pixel) film slots still holding the pre-render
                                      sentinel when the resolve read them */
    uint32_t work_order;        /* the order that ran: SPT_WORK_SAMPLE_MAJOR or SPT_WORK_PIXEL_MAJOR */
    uint32_t queue_cache;       /* the queue caching that ran: SPT_QUEUE_CACHE_CACHED or _STREAM (0: fused) */
    uint64_t isect_tri_wave_steps;  /* SPT_FLAG_TRAVERSAL_STATS: wave steps in which some lane tested a triangle */
    uint64_t isect_node_wave_steps; /*   ... in which some lane visited a node */
    double isect_begin_ms, isect_end_ms; /* SPT_FLAG_TIMING: start of the first / end of the last isect launch
                                            (the fused kernel's launches in the fused pipeline), in ms from one
                                            clock per scene (the first timed render): renders queued back to
                                            back may overlap, and their union is the kernel's busy time */
    uint64_t drained_paths;     /* wavefront: paths the drain launches finished (spt_config.drain_q8) */
    uint64_t drain_launches;    /* wavefront: drain launches queued (each runs only if its queue is short) */
    uint64_t drained_casts;     /* wavefront: ray casts the drain launches traced (the rest: isect launches) */
    double drain_ms, drain_busy_ms; /* SPT_FLAG_TIMING: drain launch time summed / the union of its intervals */
    uint64_t lockstep_casts;    /* wavefront: ray casts traced by the one-lane-per-ray isect launches
                                   (spt_config.lockstep_first), part of the isect launches' casts */
    uint64_t fit_paths;         /* the fit size in effect: spt_config.fit_paths, or fewer when the
                                   queues would not fit in device memory (spt_config.fit_bytes) */
    uint64_t fit_retries;       /* working-set allocations that failed and were retried with half
                                   the paths in flight (device memory taken by someone else) */
    uint32_t drain_refill_idle; /* wavefront: the drain's refill threshold that ran
                                   (spt_config.drain_refill_idle or its AUTO choice; 0: no drain) */
} spt_render_stats;

typedef struct spt_scene_stats {
    uint64_t ntri, nodes, leaves;
    uint32_t max_depth;         /* BVH depth (sets the LDS stack depth) */
    uint32_t max_leaf;
    uint32_t bvh_width;         /* 8 / 6: compressed 8-wide / 64-B 6-wide BVH, 2: BVH2 (spt_config.bvh_width) */
    uint32_t builder;           /* SPT_BUILD_HOST_SAH or SPT_BUILD_GPU_PLOC: the build that ran */
    uint64_t device_bytes;
    double build_ms;            /* BVH build (host SAH, or GPU PLOC + collapse, synchronised) */
    double sah_cost;
} spt_scene_stats;

/* Host-side mesh (main.cpp:133-251 load_meshes; flat arrays like
 * set_triangles_soup's inputs).  Owned by the library; free with spt_mesh_free. */
typedef struct spt_mesh {
    int32_t* pos_tri; float* pos; uint64_t nvert, ntri;
    int32_t* nrm_tri; float* nrm; uint64_t nnrm;
    int32_t* tc_tri; float* tc; uint64_t ntc;
    int32_t* mat_id;            /* per triangle: obj material id + 1 (main.cpp:185) */
    float* kd;                  /* (nmat) x 3 diffuse colours, [0] = default (main.cpp:229-245) */
    uint32_t nmat;
    float* ke;                  /* (nmat) x 3 emitted radiance (.mtl Ke), [0] = 0; not read by the reference */
} spt_mesh;

/* ---------------------------------------------------------------- device */
/* OptixBackend::init (optix_backend.h:178-186): select + initialise the GPU. */
spt_status spt_init(int32_t device);

/* OptixBackend::set_triangles_soup (optix_backend.h:283-364) + Scene::commit
 * (main.cpp:312-318).  Host arrays; the library builds a binned-SAH BVH on
 * the host and uploads it (the reference builds the GAS on device).
 * pos_tri/nrm_tri/tc_tri: 3 x int32 per triangle; pos/nrm: 3 floats per
 * entry; tc: 2 floats.  nrm_tri/tc_tri/mat_id may be NULL.  A normal index
 * of -1 falls back to the geometric normal (the reference would gather out
 * of bounds). */
spt_status spt_scene_create(const int32_t* pos_tri, const float* pos, uint64_t nvert, uint64_t ntri,
                            const int32_t* nrm_tri, const float* nrm, uint64_t nnrm,
                            const int32_t* tc_tri, const float* tc, uint64_t ntc,
                            const int32_t* mat_id, spt_scene* out);

/* Acceleration-structure builders (the reference builds its GAS on the device,
 * optix_backend.h:336-358).  Both give the compressed 8-wide BVH; closest
 * hits do not depend on the tree (ties go to the smaller triangle id). */
typedef enum spt_build {
    SPT_BUILD_AUTO = 0,         /* GPU from spt_config.gpu_build_min_tris (2M) triangles up */
    SPT_BUILD_HOST_SAH = 1,     /* binned-SAH BVH2 on the host threads, collapsed on the host */
    SPT_BUILD_GPU_PLOC = 2      /* PLOC BVH2 + collapse on the GPU (gpu_build.hip) */
} spt_build;

/* spt_scene_create with an explicit builder (spt_build). */
spt_status spt_scene_create_ex(const int32_t* pos_tri, const float* pos, uint64_t nvert, uint64_t ntri,
                               const int32_t* nrm_tri, const float* nrm, uint64_t nnrm,
                               const int32_t* tc_tri, const float* tc, uint64_t ntc,
                               const int32_t* mat_id, uint32_t build, spt_scene* out);

/* Tuning and build knobs of one scene.  The library reads no environment
 * variables: every knob is here (the Python host maps its SPT_* variables onto
 * these fields as overrides).  spt_default_config fills the measured defaults
 * (DESIGN.md §4); spt_scene_set_config validates ranges and returns
 * SPT_ERR_INVALID for a value outside them.  Build fields are read only by
 * spt_scene_create_cfg; render / intersect fields by every later call. */
enum {
    SPT_PIPELINE_AUTO = 0,      /* fused iff W*H*spp of the tile <= fused_max_paths (2^20) */
    SPT_PIPELINE_WAVEFRONT = 1, /* isect / shade / refill over path queues */
    SPT_PIPELINE_FUSED = 2      /* one persistent trace+shade kernel per sample chunk */
};
enum {
    SPT_WORK_AUTO = 0,
    SPT_WORK_SAMPLE_MAJOR = 1,
    SPT_WORK_PIXEL_MAJOR = 2
};
enum {
    SPT_QUEUE_CACHE_AUTO = 0,
    SPT_QUEUE_CACHE_CACHED = 1,   /* path-queue / hit accesses through the caches as usual */
    SPT_QUEUE_CACHE_STREAM = 2    /* non-temporal: the caches stay with the BVH and triangles */
};
typedef struct spt_config {
    /* --- scene build (spt_scene_create_cfg) */
    uint32_t build;                 /* spt_build (AUTO: GPU from gpu_build_min_tris up)      [0..2] */
    uint32_t bvh_width;             /* 8: compressed BVH8 (80-B nodes), 6: at most six
                                       children in one 64-B node, 2: BVH2 (host build) {2, 6, 8} */
    uint64_t gpu_build_min_tris;    /* SPT_BUILD_AUTO threshold, 2,000,000                          */
    uint32_t collapse;              /* BVH8 collapse: 0 SAH-optimal DP (default), 1 greedy    [0..1] */
    uint32_t ploc_radius;           /* GPU PLOC search radius                        {8, 16, 32, 64} */
    uint32_t stack_slack;           /* extra LDS stack entries per lane (0)                  [0..64] */
    /* --- spt_render */
    uint32_t pipeline;              /* SPT_PIPELINE_* (the params' FUSED / WAVEFRONT flags win) [0..2] */
    uint64_t fused_max_paths;       /* AUTO rule: fused for jobs of <= this many paths, 2^20 (fewer
                                       than two chip fills of lanes; from config 1's 1/8 tile up
                                       the wavefront with its drain matches or beats the fused
                                       kernel: DESIGN.md §6)                                   */
    uint32_t wavefront_paths;       /* paths in flight when params.wavefront_paths == 0, 2^25 [1..2^31) */
    uint32_t streams;               /* sub-wavefronts (HIP streams) of the wavefront, 4      [1..4] */
    uint32_t isect_refill_idle;     /* refill a wave once this many lanes are idle, 24       [1..64] */
    uint32_t isect_static_share_q8; /* static share of the queue per wave, 128/256          [0..255] */
    uint32_t isect_chunk;           /* queue indices per dynamic grab, 128                 [1..4096] */
    uint32_t isect_grid_q8;         /* persistent grid per stream in 1/256 chip, 0 = 256/streams [0..4096] */
    uint32_t xcd_remap;             /* bit 0: isect, bit 1: shade XCD-aware block numbering, 3 [0..3] */
    uint32_t fused_refill_idle;     /* fused kernel: shade/refill once this many lanes idle, 32 [1..64] */
    uint32_t fused_static_share_q8; /* fused kernel static share, 32/256                    [0..255] */
    uint32_t fused_grid_q8;         /* fused grid in 1/256 of the chip, 256                [0..4096] */
    uint32_t plane_pad;             /* path-queue plane padding (elements), 0            [0..2^20] */
    uint64_t film_budget_bytes;     /* per-sample film chunk budget (4 GiB): smaller values
                                       split the samples into more chunks            [>= 12 x tile px] */
    /* --- spt_intersect */
    uint32_t public_persistent;     /* 1: lane-refill persistent kernel, 0: one lane per ray  [0..1] */
    uint32_t public_refill_idle;    /* its refill threshold, 16                              [1..64] */
    /* --- scene build, continued */
    uint32_t pack_groups;           /* 1: wide-BVH child groups packed into each other's empty
                                       slots (denser node lines) in build order (level by level
                                       for the GPU builder), 2: packed in depth-first order (a
                                       subtree's groups near each other), 0: eight aligned slots
                                       each [0..2] */
    /* --- spt_render, continued */
    uint32_t pixel_block;           /* camera paths start in B x B pixel blocks, 0 (0 or 1:
                                       scanline, measured fastest: DESIGN.md §4); the image
                                       does not depend on it                             [0..64] */
    uint32_t work_order;            /* SPT_WORK_*: the order paths start in — sample-major (every
                                       pixel of a sample, then the next sample) or pixel-major (a
                                       pixel's samples together); AUTO: pixel-major for scenes of
                                       >= 256 MiB on the device, for fused tiles of >= 16M
                                       paths, and for wavefront tiles of <= 4M pixels over
                                       scenes of >= 4 MiB (then 24M paths in flight if
                                       wavefront_paths is left at 32M); the
                                       image does not depend on it                       [0..2] */
    uint32_t queue_cache;           /* SPT_QUEUE_CACHE_*: how the wavefront's path-queue and hit
                                       records (written once, read once per cast) use the
                                       caches; AUTO: STREAM for scenes of >= 256 MiB on the
                                       device (they overflow the Infinity Cache anyway: config 4
                                       +1.7 %), CACHED otherwise (config 2 -3.7 % streamed:
                                       DESIGN.md §4); the image does not depend on it     [0..2] */
    /* --- spt_render, the wavefront's drain */
    uint32_t drain_q8;              /* once every work item of a sub-wavefront has started, a queue
                                       holding fewer paths than drain_q8/256 of that stream's
                                       persistent isect lanes is finished by one drain launch (each
                                       lane continues its paths to termination) instead of one
                                       isect + shade launch per cast; 0: off.  The image does not
                                       depend on it                   [0..65535] */
    uint32_t drain_grid_q8;         /* the drain's persistent grid in 1/256 of the chip,
                                       0 = 256/streams                                  [0..4096] */
    uint32_t drain_casts;           /* with drain_q8: the drain also runs, whatever the queue's
                                       length, this many casts after the stream's last work
                                       item started, and ends the stream's launches; 0: only
                                       on a short queue                                  [0..64] */
    uint32_t fit_streams;           /* sub-wavefronts of a job that fits in flight (below), 1: one
                                       camera cast and one drain over the whole job (two concurrent
                                       persistent drains split the chip unevenly: the older launch's
                                       waves win issue); always 1 on a caller's null
                                       stream (shared hardware queues)                        [1..4] */
    uint64_t fit_paths;             /* a job of at most this many paths (tile px x spp) starts every
                                       path in the first refill (paths in flight = the job, unless
                                       params.wavefront_paths or config.wavefront_paths is set) on fit_streams
                                       sub-wavefronts: its last work item starts at once, so the
                                       drain takes over drain_casts casts later; 2^28 (21 GB of
                                       queues per working set in unit mode, 34 GB with emitters),
                                       0: off                                   */
    uint32_t sub_queues;            /* 1: a render runs on its working set's own streams, created
                                       with a full CU mask, which gives each a hardware queue of
                                       its own whatever GPU_MAX_HW_QUEUES allows; they are blocking
                                       streams, so a set bound to the legacy null stream uses plain
                                       non-blocking streams instead.  0: plain streams always
                                       (they share the process's queues)       [0..1] */
    uint32_t drain_sort;            /* 1: a forced drain takes its queue sorted by the direction's
                                       octant and the origin's Morton code (coherent bounce rays
                                       per wave; wide-BVH scenes); 0: queue order.  The image does
                                       not depend on it                                       [0..1] */
    uint32_t lockstep_first;        /* the first cast of a job that fits in flight (fit_paths): 1: a
                                       one-lane-per-ray isect kernel without lane refill (coherent
                                       camera rays finish together), then the shade kernel; 2: one
                                       camera-cast kernel that makes the camera rays, traces them in
                                       lockstep and shades the hits (no queue round trip); 3: the
                                       same with its survivors compacted per XCD shard and the
                                       drain's per-XCD pools over those segments (one queue counter
                                       takes ~88 atomics per us; config 1 +11 % over 1, a single
                                       render +18 %); 0: the persistent isect kernel
                                       for every cast.  Wide-BVH scenes (2 and 3; BVH2 scenes run
                                       1).  The image does not depend on it                 [0..3] */
    uint32_t fit_chunks;            /* 1: a job of more than fit_paths paths whose tile has at most
                                       fit_paths pixels runs as sample chunks of at most fit_paths
                                       paths, each started at once like a fitting job (config 3
                                       +8 %); 0: such jobs keep the per-cast
                                       wavefront with wavefront_paths in flight.  The image does not
                                       depend on it                                           [0..1] */
    uint64_t fit_bytes;             /* device memory a fitting job's path queues, hit records and
                                       film chunk may take per working set (2 x 16 B x planes +
                                       16 B + the film slot per path); fit_paths shrinks to what
                                       fits (more sample chunks; below one chunk of the tile's
                                       pixels the per-cast wavefront).  0: the free device memory
                                       plus what the caller's set holds, less 1/16 (processes or
                                       scenes sharing the GPU); an allocation that fails anyway
                                       halves the fit and retries.  The image does not depend on
                                       it                                                      */
    uint32_t drain_refill_idle;     /* the drain's lane loop refills (and shades) once this many of a
                                       wave's lanes are idle.  0 = AUTO: 56 for scenes with analytic
                                       spheres (tested in the shade: a pass costs several
                                       trace steps; config 2 +20 % over 24), 40 when the queue
                                       is streamed (queue_cache; config 4 +3 %), else 24
                                       (config 1 +1.8 % over 32).  The fused kernel keeps fused_refill_idle.
                                       The image does not depend on it   [0..64] */
} spt_config;

void spt_default_config(spt_config* cfg);

/* spt_scene_create with a configuration (NULL = spt_default_config). */
spt_status spt_scene_create_cfg(const int32_t* pos_tri, const float* pos, uint64_t nvert, uint64_t ntri,
                                const int32_t* nrm_tri, const float* nrm, uint64_t nnrm,
                                const int32_t* tc_tri, const float* tc, uint64_t ntc,
                                const int32_t* mat_id, const spt_config* cfg, spt_scene* out);

/* Replace / read the scene's configuration (the build fields are kept as built). */
spt_status spt_scene_set_config(spt_scene scene, const spt_config* cfg);
spt_status spt_scene_get_config(spt_scene scene, spt_config* out);

/* Per-material albedo (RGB, nmat x 3).  Default: 1 for every material, as in
 * the reference (main.cpp:234,244 — Kd is read and discarded). */
spt_status spt_scene_set_albedo(spt_scene scene, const float* albedo_rgb, uint32_t nmat);

/* Per-material emitted radiance (RGB, nmat x 3), added as throughput x Le at
 * every surface hit (smallpt's obj.e; the reference has no emitters, SURVEY
 * F6 / §8f row 3).  Default: none.  With emitters the last cast is a closest
 * hit (it must know which surface it reached). */
spt_status spt_scene_set_emission(spt_scene scene, const float* emission_rgb, uint32_t nmat);

/* smallpt's scene primitives and materials (the reference renders triangle
 * meshes with Lambert BSDFs only; BASELINE config 2 is smallpt's Cornell box).
 *
 * spt_scene_set_spheres: n analytic spheres, center_radius = n x (cx, cy, cz,
 * r) floats, mat_id = n material ids (NULL: material 0), tested against every
 * ray after the triangle BVH (a list: smallpt-sized sets, n <= 256).  A sphere
 * hit reports tri_id = -2 - k in spt_intersect (k = the sphere's index).
 * NULL / n = 0 removes them.
 *
 * spt_scene_set_material_kinds: per material SPT_MAT_DIFFUSE (Lambert with
 * the reference's un-normalised, unflipped shading normal on triangles, the
 * outward normal flipped toward the ray on spheres — smallpt's nl),
 * SPT_MAT_MIRROR (smallpt SPEC: ideal reflection) or SPT_MAT_GLASS (smallpt
 * REFR: index 1.5, Schlick Fresnel, reflect with probability P = 1/4 + Re/2
 * chosen by the bounce draw's first number, weight Re/P or (1-Re)/(1-P)).
 * Albedo (and textures) multiply every kind.  Default: all diffuse. */
enum { SPT_MAT_DIFFUSE = 0, SPT_MAT_MIRROR = 1, SPT_MAT_GLASS = 2 };
spt_status spt_scene_set_spheres(spt_scene scene, const float* center_radius, const int32_t* mat_id, uint32_t n);
spt_status spt_scene_set_material_kinds(spt_scene scene, const uint32_t* kinds, uint32_t nmat);

/* LambertBsdf's reflectance image for one material (ImageTexture,
 * main.cpp:34-80; the reference only ever builds 1 x 1 images, main.cpp:40-44,
 * and its loader is empty, :37-39): rgb = width x height interleaved RGB
 * floats.  A bounce off the material multiplies the throughput by the
 * bilinear, clamped lookup at the hit's interpolated texcoord (main.cpp:62-76,
 * 109-117), including the reference's texel index y * height + x (main.cpp:52;
 * it equals y * width + x for square images), kept inside the image.  Without
 * texcoords the lookup is at (0, 0).  rgb NULL removes the image (the albedo
 * table's constant applies again).  At most 2^26 texels per image. */
spt_status spt_scene_set_texture(spt_scene scene, uint32_t material, const float* rgb, uint32_t width,
                                 uint32_t height);

spt_status spt_scene_get_stats(spt_scene scene, spt_scene_stats* out);

/* The host builders alone, without a device (diagnostics; the host sanitizer
 * run drives the builders through it): triangle soup tri_verts (ntri x 9
 * floats: v0 v1 v2), cfg->bvh_width 2, 6 or 8 and cfg->collapse (NULL =
 * defaults).  Fills ntri, nodes, leaves, max_depth, max_leaf, bvh_width,
 * builder (SPT_BUILD_HOST_SAH), build_ms and sah_cost; device_bytes = 0. */
spt_status spt_bvh_build_stats(const float* tri_verts, uint64_t ntri, const spt_config* cfg,
                               spt_scene_stats* out);
spt_status spt_scene_destroy(spt_scene scene);

/* Binary scene cache ("a binary scene cache format").  The
 * reference re-parses its OBJ and rebuilds the OptiX GAS on every run
 * (main.cpp:288-318 → optix_backend.h:283-364); its pbrt-parser dependency
 * caches only the parse.  spt_scene_save writes a committed scene to one
 * file: the BVH in its device layout (node slots, packed child groups), the
 * slot-ordered triangle / normal / texcoord / orig2slot arrays, albedo,
 * emission, spheres, material kinds, textures, the scene's spt_config and
 * spt_scene_stats, and `extra` (extra_bytes opaque application bytes, e.g. the
 * pbrt camera; may be NULL / 0).  spt_scene_load uploads it onto the current
 * device with no parse, build or re-layout (stats.build_ms = the load time,
 * builder as saved); the result renders bit-identically to the saved scene.
 *
 * Format (little endian): a fixed header {magic "SPTSCENE", version, the
 * writer's layout constants (triangle and node quads, node6, group_shift,
 * sizeof spt_config / spt_scene_stats), counts, section sizes, one 64-bit
 * checksum per section, spt_config, spt_scene_stats} then the sections in
 * that order.  Load refuses (SPT_ERR_INVALID) another magic / version /
 * layout, a size mismatch or a truncated file before touching the device, and
 * a bad checksum before the scene is returned (its uploads are freed).
 * spt_scene_cache_info runs all the checks without a device and
 * reports the saved stats / config / extra size (each out pointer may be
 * NULL).  spt_scene_load copies at most extra_cap bytes of extra into `extra`
 * and the full size into *extra_bytes (both may be NULL / 0). */
spt_status spt_scene_save(spt_scene scene, const char* path, const void* extra, uint64_t extra_bytes);
spt_status spt_scene_load(const char* path, spt_scene* out, void* extra, uint64_t extra_cap, uint64_t* extra_bytes);
spt_status spt_scene_cache_info(const char* path, spt_scene_stats* stats, spt_config* cfg, uint64_t* extra_bytes);

/* OptixBackend::intersect (optix_backend.h:422-460) → __raygen__rg
 * (wavefront_isect.cu:80-112): one lane per ray; mask_size == 1 broadcasts
 * mask[0]; masked lanes write nothing; a miss writes tri_id = -1 (t/u/v
 * untouched).  do_closest = 0 is the reference's any-hit query
 * (OPTIX_RAY_FLAG_TERMINATE_ON_FIRST_HIT): traversal stops at the first
 * triangle (or sphere) accepted in [tmin, tmax].  Deviation, documented: the
 * reference launches that query with the closest-hit program disabled
 * (OPTIX_RAY_FLAG_DISABLE_CLOSESTHIT, wavefront_isect.cu:104-105), so on a hit
 * its tri_id / t / u / v come from payload registers nothing wrote
 * (uninitialised); only "tri_id != -1" is meaningful there.  This library
 * writes the first accepted hit's real record (tri_id, t, u, v of that
 * triangle, not necessarily the nearest), which satisfies every use the
 * reference makes of the result.  All pointers are device pointers; n rays. */
spt_status spt_intersect(spt_scene scene, const spt_rays* rays, const uint8_t* mask,
                         uint32_t mask_size, const spt_hits* hits, uint32_t n,
                         int32_t do_closest, void* stream);

/* Hit reconstruction (optix_backend.h:462-486 + main.cpp:325): for lanes with
 * tri_id != -1 && mask, fills the requested spt_hit_info planes. */
spt_status spt_hit_info_compute(spt_scene scene, const spt_rays* rays, const spt_hits* hits,
                                const uint8_t* mask, uint32_t mask_size, uint32_t n,
                                const spt_hit_info* out, void* stream);

/* main.cpp:354-429: the whole wavefront render of one tile.  film_dev is a
 * device buffer of 3 x tile_rows x width floats (planar R, G, B as the
 * reference's SpectrumC film, main.cpp:369), already divided by spp.  The
 * call returns after the stream has drained.  stats may be NULL.
 * Threading: every call on a scene holds a per-scene mutex while it enqueues
 * (a second thread waits); render concurrently from one scene per thread /
 * device.  spt_intersect and spt_hit_info_compute launch while holding it and
 * record an event on their stream.  The scene setters (albedo, emission,
 * textures, spheres, material kinds) and spt_scene_destroy block the host
 * until every queued render of the scene and the last public call on every
 * stream have finished before they free or replace a device array, so a
 * launch already queued always reads the state it was queued with; no caller
 * synchronisation is needed (spt_scene_set_config changes only knobs the
 * next call reads).  A render does not run on `stream` itself: it runs on its
 * working set's own streams (below), after `stream`'s prior work (an event),
 * and `stream`'s next work waits for the render's end (an event). */
spt_status spt_render(spt_scene scene, const spt_render_params* params, float* film_dev,
                      spt_render_stats* stats, void* stream);

/* spt_render in two halves, so that renders can be queued back to back: the
 * GPU then runs one frame into the next with no gap for the host's return,
 * the caller's own work between frames, and the next call's set-up
 * (the reference's host loop likewise only queues work, main.cpp:385-429).
 * spt_render_async queues the whole render of `params` on `stream` and returns
 * a ticket; its host loop still follows the wavefront's queue counters while
 * the render runs, so the call returns near the end of the render's GPU work,
 * not at its start.  The film is complete once the stream reaches the point
 * where the call returned.  spt_render_wait(ticket) waits for that render and
 * fills its statistics (stats may be NULL); every ticket must be collected
 * once, and at most 64 renders of a scene may be queued without being
 * collected (SPT_ERR_LIMIT).  spt_render(...) = spt_render_async +
 * spt_render_wait.  A scene keeps two working sets (queues, film chunk,
 * sub-wavefront streams), each bound to the caller stream it was first used
 * with: renders queued alternately on two streams overlap (one drains while
 * the next starts); a third stream takes over the least recently used set.
 * A set's streams are created with a full CU mask (spt_config.sub_queues),
 * which gives each a hardware queue of its own; such streams are blocking
 * streams, so legacy null-stream work serialises with them.  A set bound to
 * the legacy null stream (or the per-thread default stream) therefore uses
 * plain non-blocking streams and runs a fitting job on one sub-wavefront.
 * For overlapping renders, queue them on two streams of your own that have
 * hardware queues of their own. */
spt_status spt_render_async(spt_scene scene, const spt_render_params* params, float* film_dev, void* stream,
                            uint64_t* ticket);
spt_status spt_render_wait(spt_scene scene, uint64_t ticket, spt_render_stats* stats);

/* The isect kernel's busy time across queued renders (a build addition, for the
 * roofline: renders queued back to back overlap, so per-render busy times do
 * not add up).  After _begin, every SPT_FLAG_TIMING render collected by
 * spt_render_wait / spt_render contributes its isect launch intervals (the
 * fused kernel's in the fused pipeline) on the scene's clock; _end returns the
 * union of all of them in ms and the number of launches, and stops collecting. */
spt_status spt_scene_isect_busy_begin(spt_scene scene);
spt_status spt_scene_isect_busy_end(spt_scene scene, double* busy_ms, uint64_t* launches);
/* Between busy_begin and busy_end: the union of the launch intervals of the
 * renders collected so far, for a mask of kernels (SPT_KERNEL_ISECT: the isect
 * launches — the fused kernel's in the fused pipeline —, SPT_KERNEL_DRAIN: the
 * wavefront's drain launches; both: the time either traced rays), and the
 * number of launches.  Does not stop the collection. */
enum { SPT_KERNEL_ISECT = 1u, SPT_KERNEL_DRAIN = 2u };
spt_status spt_scene_kernel_busy(spt_scene scene, uint32_t kernels, double* busy_ms, uint64_t* launches);

/* Rows of tile `tile_index` (in increasing order).  Returns the row count;
 * writes at most `cap` row indices into rows (may be NULL). */
uint32_t spt_tile_rows(uint32_t height, uint32_t tile_index, uint32_t tile_count,
                       uint32_t rows_per_group, uint32_t* rows, uint32_t cap);

/* Default parameters of the reference's main() (main.cpp:357-383). */
void spt_default_params(spt_render_params* p);

const char* spt_last_error(void);
const char* spt_version(void);
/* A hash of the sources and compiler flags this library was built from: profile
 * data (profiles/isect_pmc.json) names the build it measured by this id. */
const char* spt_build_id(void);
/* Test hook (not for production use): the working-set allocation numbered
 * `nth` (0-based, counted over the device allocations spt_render makes for its
 * path queues, hit records, counters, film chunk and running sum, from this
 * call on, in any scene) fails with an out-of-memory error once, as when another
 * process took the memory between the fit rule's check and the allocation;
 * nth < 0 disarms it.  Lets a test drive the render's halve-and-retry path
 * (spt_render_stats.fit_retries) deterministically, without exhausting the
 * device. */
void spt_debug_fail_workspace_alloc(int32_t nth);

/* ------------------------------------------------------------------ host */
/* load_meshes (main.cpp:141-251): triangulating OBJ reader with tinyobj's
 * index semantics (position / normal / texcoord triplets, material id + 1). */
spt_status spt_obj_load(const char* path, spt_mesh* out);
void spt_mesh_free(spt_mesh* mesh);

/* pbrt-v3 scene reader (the reference's pbrt-parser dependency, .gitmodules:7-9,
 * CMakeLists.txt:57-61): triangle meshes ("trianglemesh",
 * "plymesh"), transforms, attribute scopes, object instances (flattened),
 * materials' diffuse Kd, diffuse area lights (emission), the perspective
 * camera, film size and a constant infinite light.  Same spt_mesh as
 * spt_obj_load (material 0 = default, shapes get their material + 1). */
typedef struct spt_pbrt_info {
    uint32_t has_camera;        /* a Camera directive was seen */
    spt_camera camera;          /* look_from/at/up from the CTM at Camera; fov_y (radians) from "fov"
                                   (pbrt's fov spans the shorter image axis) */
    float fov_deg;              /* "float fov" as written (default 90) */
    uint32_t xres, yres;        /* Film "xresolution" / "yresolution" (default 640 x 480) */
    uint32_t has_env;           /* LightSource "infinite" seen */
    float env[3];               /*   its radiance ("rgb L" x "scale") */
    uint64_t shapes;            /* triangle shapes loaded (instanced ones once per definition) */
    uint64_t shapes_skipped;    /* other shape types (sphere, curve, ...) */
    uint64_t instances;         /* ObjectInstance directives flattened */
} spt_pbrt_info;

spt_status spt_pbrt_load(const char* path, spt_mesh* out, spt_pbrt_info* info);

/* Fimage::save_pfm (fimage.h:33-58): planar R, G, B → interleaved,
 * rows bottom-up, scale -1 (little endian). */
spt_status spt_pfm_write(const char* path, const float* r, const float* g, const float* b,
                         uint32_t width, uint32_t height);

#ifdef __cplusplus
}
#endif
#endif /* SPT_H */
