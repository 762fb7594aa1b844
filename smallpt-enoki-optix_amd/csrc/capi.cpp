// capi.cpp — the C ABI (include/spt.h): scene upload, public intersect,
// hit reconstruction and the wavefront render loop (main.cpp:354-429).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/spt.h"
#include "bvh_build.h"
#include "gpu_build.h"
#include "host_error.h"
#include "spt_internal.h"

// Diagnostic build only (make BUILD=build_dbg EXTRA="-g -DSPT_SEGV_TRACE=1"):
// a host segmentation fault prints the native backtrace (library offsets for
// addr2line) before the default action.  Not in the product build.
#ifndef SPT_SEGV_TRACE
#define SPT_SEGV_TRACE 0
#endif
#if SPT_SEGV_TRACE
#include <execinfo.h>
#include <signal.h>
namespace {
void segv_trace(int sig) {
    void* bt[64];
    const int n = backtrace(bt, 64);
    backtrace_symbols_fd(bt, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}
struct SegvTraceInstall {
    SegvTraceInstall() { signal(SIGSEGV, segv_trace); }
} segv_trace_install;
}  // namespace
#endif

using namespace spt;

namespace {

thread_local std::string g_last_error;

spt_status fail(spt_status code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_TRY(call)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (call);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return fail(e_ == hipErrorOutOfMemory ? SPT_ERR_OOM : SPT_ERR_HIP, "HIP call '%s' failed: %s (%s:%d)", \
                        #call, hipGetErrorString(e_), __FILE__, __LINE__);                         \
    } while (0)

template <typename T>
void hfree(T*& p) {
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Path queue planes (spt_internal.h PathQueue): 2 (unit), 3 (albedo) or 4
// (emitters) 16-B quads per path.
constexpr size_t kHitBytes = 16;
// an out-of-memory render retries with half its paths in flight down to this many
constexpr uint64_t kMinRetryPaths = 1u << 16;

// Planes are `stride` elements apart (stride = cap + pad, see queue_stride).
PathQueue carve_queue(char* base, size_t stride, uint32_t planes) {
    PathQueue q;
    float4* f4 = (float4*)base;
    q.q1 = f4;
    q.q2 = f4 + stride;
    q.q0 = planes > 2 ? f4 + 2 * stride : nullptr;
    q.rad = planes > 3 ? (float2*)(f4 + 3 * stride) : nullptr;  // 8 B per path (16 allocated)
    return q;
}

// Plane stride: cap plus a pad (spt_config.plane_pad) so the SoA planes (and
// the two queues) need not sit a power of two apart.
size_t queue_stride(size_t cap, uint32_t pad) { return cap + pad; }

// Device counters of one sub-wavefront (zeroed per chunk; see spt_render).
// The atomically updated counters sit in 128-B lines of their own: a line that
// takes atomics (shade blocks' survivor counts, isect waves' work grabs) slows
// every plain load of the same line from the other waves (config 1 +1.2 %;
// EXPERIMENTS.md, r3_counter_lines).
struct Counters {
    uint32_t qn[2];      // queue counts (isect/shade input)
    alignas(128) uint32_t surv[2];    // survivors appended by shade
    uint64_t cursor[2];  // next work item (double-buffered across refills)
    alignas(128) uint32_t isect_next; // persistent isect work counter (zeroed by each refill)
    uint32_t exhausted;  // RefillArgs::iter_tag of the refill that started the last work item (0: not yet)
    uint32_t pad[2];
    alignas(128) uint32_t isect_next_b;  // SPT_ISECT_CAMERA: the counter of the launches on queue 1
    alignas(128) uint32_t xcd_next[8][32];  // the drain / fused kernel's per-XCD work counters (one line each)
    alignas(128) uint32_t surv_shard[kShards][kShardStride];  // a sharded camera cast's survivors per shard
};
uint32_t* isect_next_of(Counters* c, int queue) { return queue ? &c->isect_next_b : &c->isect_next; }

// Camera paths started inside the isect launches (no refill launch per
// iteration): an experiment, VERDICT r3 item 3 (EXPERIMENTS.md round 4).
#ifndef SPT_ISECT_CAMERA
#define SPT_ISECT_CAMERA 0
#endif
constexpr bool kIsectCam = SPT_ISECT_CAMERA != 0;

// Render-wide device statistics.
struct Stats {
    unsigned long long stats[3];  // casts, continuations, camera rays started
    unsigned long long trav[7];   // SPT_FLAG_TRAVERSAL_STATS: nodes, tris, lane steps, wave steps, max stack,
                                  // wave steps running the triangle block, the visit block
    unsigned long long unwritten; // film slots still holding the sentinel at resolve time
    unsigned long long drained;   // paths finished by drain launches
    unsigned long long drained_casts;  // ray casts traced by drain launches
};

constexpr int kMaxStreams = 4;
// the drain phase starts when the host's (lagging) view of a stream's unstarted
// work falls below this many queue capacities (spt_render_async)
constexpr uint64_t kDrainLookahead = 6;

// One render's own state, so that renders can be queued back to back
// (spt_render_async) while earlier ones are still on the GPU: its device
// counters and their pinned readback, its timing events, and the host-side
// statistics known at enqueue time.  The workspace keeps a ring of them.
constexpr int kRenderSlots = 64;
struct RenderSlot {
    Stats* dev = nullptr;                       // device counters of this render
    Stats* host = nullptr;                      // pinned readback, complete once `done` has fired
    std::vector<hipEvent_t> events;             // [0] = time origin, then start/end pairs of timed launches
    std::vector<std::pair<size_t, int>> timed;  // (start event index, 0 refill 1 isect 2 shade 3 resolve)
    hipEvent_t done = nullptr;                  // recorded after the readback
    spt_render_stats rs{};                      // fields known when the render was queued
    uint64_t regen_base = 0;                    // camera rays of the first launch (for rs.regenerations)
    bool timing = false;
    double wall0 = 0.0;
    uint64_t ticket = 0;
    bool pending = false;                       // queued, not yet collected by spt_render_wait
};

// One sub-wavefront: its own double-buffered path queue, hit records and
// counters, driven on its own stream so its launch tails overlap the others'.
struct Sub {
    size_t cap = 0;
    uint32_t pad = 0;                   // plane pad the queues were carved with
    uint32_t planes = 0;                // 16-B planes per path allocated
    char* qa = nullptr;
    char* qb = nullptr;
    char* hits = nullptr;
    Counters* cnt = nullptr;
    hipStream_t stream = nullptr;       // the library's own stream (spt_config.sub_queues)
    // spt_config.drain_sort: sort keys / values (in, out) over cap slots and hipcub scratch
    uint32_t* sort_buf = nullptr;
    size_t sort_cap = 0;
    void* sort_tmp = nullptr;
    size_t sort_tmp_bytes = 0;
    bool own_queue = false;             // created with a full CU mask (spt_config.sub_queues)
    Counters* host_cnt = nullptr;       // pinned, 2 slots (counter snapshots read one batch behind)
    hipEvent_t count_ev[2] = {nullptr, nullptr};
    hipEvent_t join_ev = nullptr;
};

// One render's working memory: path queues, counters and sub-wavefront
// streams, the per-sample film chunk and the running sum.  A scene keeps two
// (kWorkSets), one per caller stream (pick_set), so a render queued on another
// stream can start while the previous one drains; a render waits for the last
// render that used its set (free_ev), so any stream use stays race-free.
constexpr int kWorkSets = 2;
struct WorkSet {
    Sub sub[kMaxStreams];
    hipStream_t home = nullptr;         // the caller stream the set was first used with (bound)
    bool bound = false;
    uint64_t last_ticket = 0;           // the last render that used the set
    size_t film_cap = 0, acc_cap = 0;
    char* film = nullptr;               // per-sample contributions of a chunk (bytes or RGB floats)
    float* acc = nullptr;               // [3][P] running sum across chunks
    hipEvent_t fork_ev = nullptr;
    hipEvent_t free_ev = nullptr;       // recorded on the set's stream 0 after the last render that used it
    hipEvent_t call_ev = nullptr;       // the caller stream's work before a render (the render waits for it)
    bool used = false;                  // free_ev has been recorded

    void release() {
        for (Sub& b : sub) {
            hfree(b.qa); hfree(b.qb); hfree(b.hits); hfree(b.cnt); hfree(b.sort_buf);
            if (b.sort_tmp) (void)hipFree(b.sort_tmp);
            if (b.host_cnt) (void)hipHostFree(b.host_cnt);
            for (auto& e : b.count_ev) if (e) (void)hipEventDestroy(e);
            if (b.join_ev) (void)hipEventDestroy(b.join_ev);
            if (b.stream) (void)hipStreamDestroy(b.stream);
        }
        hfree(film); hfree(acc);
        if (fork_ev) (void)hipEventDestroy(fork_ev);
        if (free_ev) (void)hipEventDestroy(free_ev);
        if (call_ev) (void)hipEventDestroy(call_ev);
        *this = WorkSet();
    }
};

// Before a scene mutator frees or replaces a device array that queued work may
// still read (materials, textures, spheres, kinds): wait for every render of
// both working sets (free_ev) and for the last public call on every stream
// that made one (spt_intersect / spt_hit_info_compute, record_public_use).  The
// caller holds the scene mutex, so nothing new is queued meanwhile.
struct PublicUse {
    hipStream_t stream;
    hipEvent_t ev;
};

// The PCG32 jump table of one (spp, depth, seed) key: [spp] seeded sample maps,
// then [depth] cast jumps (read-only while renders run).  A workspace keeps a
// few, so a caller that changes the seed per render (progressive accumulation)
// reuses them; a table is rewritten (on the render's stream, from its own
// pinned staging copy) only after every render that read it has finished —
// ev[s] is recorded after each render of working set s that used the table,
// and a set's renders run in order — and a render on another stream waits
// for the write (write_ev).  No device-wide synchronisation.
constexpr int kJumpTables = 4;
struct JumpTable {
    PcgJump* dev = nullptr;
    PcgJump* host = nullptr;            // pinned staging of the last write
    size_t cap = 0;
    uint32_t spp = 0, depth = 0;
    uint64_t state = 0;
    bool valid = false;
    uint64_t lru = 0;
    hipEvent_t write_ev = nullptr;
    hipEvent_t ev[kWorkSets] = {};
    bool ev_used[kWorkSets] = {};
    void release() {
        hfree(dev);
        if (host) (void)hipHostFree(host);
        if (write_ev) (void)hipEventDestroy(write_ev);
        for (auto& e : ev) if (e) (void)hipEventDestroy(e);
        *this = JumpTable();
    }
};

struct Workspace {
    WorkSet sets[kWorkSets];
    // The working set of a render on caller stream `s`: the set bound to that
    // stream, else one never used, else the least recently used (rebound).
    // HIP maps streams onto GPU_MAX_HW_QUEUES (4) hardware queues as they are
    // first used, and a set's sub-wavefront streams were mapped beside the
    // caller stream they first ran with (sub 0 is the caller's own): the same
    // set on another caller stream can put two of the four sub-wavefronts on
    // one queue, which serialises them (config 3 / 4: -17 % / -16 %,
    // profiles/r03_queues/).
    // the set bound to caller stream s, if any (pick_set without binding one)
    const WorkSet* bound_set(hipStream_t s) const {
        for (const WorkSet& w : sets)
            if (w.bound && w.home == s) return &w;
        return nullptr;
    }
    WorkSet& pick_set(hipStream_t s) {
        WorkSet* lru = &sets[0];
        for (WorkSet& w : sets)
            if (w.bound && w.home == s) return w;
        for (WorkSet& w : sets)
            if (!w.bound) {
                w.bound = true;
                w.home = s;
                return w;
            }
        for (WorkSet& w : sets)
            if (w.last_ticket < lru->last_ticket) lru = &w;
        lru->home = s;
        return *lru;
    }
    JumpTable jt[kJumpTables];          // PCG32 jump tables for recent (spp, depth, seed) keys
    uint64_t jt_clock = 0;
    RenderSlot slots[kRenderSlots];     // renders queued by spt_render_async (ticket % kRenderSlots)
    uint64_t next_ticket = 1;
    hipEvent_t epoch = nullptr;         // the first timed render's time origin: isect_begin/end_ms count from it
    // spt_scene_isect_busy_begin/end: every isect [0] and drain [1] launch
    // interval (scene clock) of the renders collected in between, so the union
    // across overlapping queued renders is exact (not one render's span less
    // its overlap)
    bool collect_iv = false;
    std::vector<std::pair<double, double>> iv_all[2];

    void release() {
        for (WorkSet& w : sets) w.release();
        if (epoch) (void)hipEventDestroy(epoch);
        for (JumpTable& t : jt) t.release();
        for (RenderSlot& r : slots) {
            hfree(r.dev);
            if (r.host) (void)hipHostFree(r.host);
            for (auto e : r.events) (void)hipEventDestroy(e);
            if (r.done) (void)hipEventDestroy(r.done);
        }
        for (auto& v : iv_all) v.clear();
        collect_iv = false;
        const uint64_t t = next_ticket;  // tickets stay unique over the scene's life
        *this = Workspace();
        next_ticket = t;
    }
};

}  // namespace

struct spt_scene_t {
    int device = 0;
    spt_config cfg{};
    std::mutex mu;  // one workspace per scene: spt_render / spt_scene_set_config serialise here
    uint64_t ntri = 0;
    float4* nodes = nullptr;
    uint4* nodes8 = nullptr;
    uint32_t node6 = 0;  // nodes8 holds the 64-B six-wide nodes (spt_config.bvh_width 6)
    uint32_t group_shift = 3;  // 0: packed child groups, 3: aligned groups of eight slots
    float4* tris = nullptr;
    float4* snrm = nullptr;
    float* tc = nullptr;
    int32_t* orig2slot = nullptr;
    float* albedo = nullptr;
    uint32_t nmat = 1;
    float* emission = nullptr;
    uint32_t nemit = 0;
    bool albedo_unit = true;  // every albedo entry is exactly 1 (the reference's case)
    // per-material reflectance images (spt_scene_set_texture): host copies and
    // the device arrays rebuilt from them
    std::vector<std::vector<float4>> tex_img;
    std::vector<uint32_t> tex_w, tex_h;
    uint4* tex_info = nullptr;
    float4* texels = nullptr;
    uint32_t ntex = 0;      // entries of tex_info (0: no images)
    float4* spheres = nullptr;   // smallpt's analytic spheres (spt_scene_set_spheres)
    int32_t* sph_mat = nullptr;
    uint32_t nsph = 0;
    uint32_t* mat_kind = nullptr;  // SPT_MAT_* per material (spt_scene_set_material_kinds)
    uint32_t nkind = 0;
    uint64_t node_bytes = 0;  // bytes behind nodes / nodes8 (spt_scene_save)
    uint32_t stack_depth = 1;
    spt_scene_stats stats{};
    Workspace ws;
    std::vector<PublicUse> pub;  // streams of public calls, with an event after the last one (quiesce)

    DeviceScene dev() const {
        DeviceScene d;
        d.nodes = nodes; d.nodes8 = nodes8; d.node6 = node6; d.group_shift = group_shift; d.tris = tris; d.snrm = snrm; d.tc = tc; d.orig2slot = orig2slot;
        d.albedo = albedo; d.nmat = nmat; d.emission = emission; d.nemit = nemit; d.stack_depth = stack_depth; d.empty = ntri == 0;
        d.tex_info = tex_info; d.ntex = ntex; d.texels = texels;
        d.spheres = spheres; d.sph_mat = sph_mat; d.nsph = nsph;
        d.mat_kind = mat_kind; d.nkind = nkind;
        return d;
    }
    void release() {
        for (auto& u : pub) (void)hipEventDestroy(u.ev);
        pub.clear();
        ws.release();
        hfree(nodes); hfree(nodes8); hfree(emission); hfree(tris); hfree(snrm); hfree(tc); hfree(orig2slot); hfree(albedo);
        hfree(tex_info); hfree(texels); hfree(spheres); hfree(sph_mat); hfree(mat_kind);
    }
};

namespace {

// Makes the scene's device current for one API call and restores the
// caller's afterwards: a scene's arrays, streams and events live on the device
// it was committed on, whatever device the calling thread has current (the C++
// host destroys every rank's scene from one thread).
struct DeviceGuard {
    int prev = -1;
    bool switched = false;
    explicit DeviceGuard(int device) {
        if (hipGetDevice(&prev) == hipSuccess && prev != device) switched = hipSetDevice(device) == hipSuccess;
    }
    ~DeviceGuard() {
        if (switched) (void)hipSetDevice(prev);
    }
};

// (see PublicUse) caller holds sc->mu
spt_status quiesce_scene(spt_scene_t* sc) {
    for (WorkSet& w : sc->ws.sets)
        if (w.used && w.free_ev) HIP_TRY(hipEventSynchronize(w.free_ev));
    for (auto& u : sc->pub) HIP_TRY(hipEventSynchronize(u.ev));
    return SPT_OK;
}

// After a public call's launch on `s` (caller holds sc->mu).  At most 64
// streams are tracked: beyond that the list is drained and restarted.
spt_status record_public_use(spt_scene_t* sc, hipStream_t s) {
    for (auto& u : sc->pub)
        if (u.stream == s) {
            HIP_TRY(hipEventRecord(u.ev, s));
            return SPT_OK;
        }
    if (sc->pub.size() >= 64) {
        for (auto& u : sc->pub) {
            HIP_TRY(hipEventSynchronize(u.ev));
            (void)hipEventDestroy(u.ev);
        }
        sc->pub.clear();
    }
    hipEvent_t e = nullptr;
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    sc->pub.push_back({s, e});
    HIP_TRY(hipEventRecord(e, s));
    return SPT_OK;
}

spt_status ensure_device() {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) return fail(SPT_ERR_NO_DEVICE, "no HIP device visible (%s)", hipGetErrorString(e));
    return SPT_OK;
}

spt_status upload_textures(spt_scene_t* sc);

template <typename T>
spt_status upload(T** dst, const void* src, size_t bytes) {
    *dst = nullptr;
    if (bytes == 0) return SPT_OK;
    HIP_TRY(hipMalloc((void**)dst, bytes));
    HIP_TRY(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
    return SPT_OK;
}

// ThinlensCamera constructor (pinhole.h:9-25) + the per-call constants of
// sample_dir (pinhole.h:40-41), evaluated once on the host.
Camera make_camera(const spt_render_params& p) {
    const spt_camera& c = p.camera;
    Camera cam;
    V3 from = v3(c.look_from[0], c.look_from[1], c.look_from[2]);
    V3 at = v3(c.look_at[0], c.look_at[1], c.look_at[2]);
    V3 up = v3(c.up[0], c.up[1], c.up[2]);
    cam.origin = from;
    V3 z = normalize(at - from);
    V3 x = normalize(cross(up, z));
    V3 y = normalize(cross(z, x));
    cam.frame.bx = x; cam.frame.by = y; cam.frame.bz = z;
    cam.lens_radius = c.lens_radius;
    cam.focal_dist = c.focal_dist;
    cam.film_y = c.film_size_y;
    cam.dist_lens_to_film = (c.film_size_y * 0.5f) / std::tan(c.fov_y * 0.5f);
    cam.ratio = (float)p.width / (float)p.height;
    cam.fw = (float)p.width;
    cam.fh = (float)p.height;
    // exact reciprocals of power-of-two sizes (camera_sample_dir), else 0
    cam.inv_fw = p.width && (p.width & (p.width - 1u)) == 0u ? 1.0f / cam.fw : 0.0f;
    cam.inv_fh = p.height && (p.height & (p.height - 1u)) == 0u ? 1.0f / cam.fh : 0.0f;
    {
        volatile float fz = cam.dist_lens_to_film;  // the device's operation order, no folding
        volatile float num = cam.focal_dist * fz;
        cam.focal_z = num / fz;
    }
    return cam;
}

// A set's buffers for this render; a buffer that must grow is freed only after
// the last render that used the set has finished with it.
// A sub-wavefront stream of the library's own.  With own_queue, a full CU
// mask: HIP gives a CU-masked stream a hardware queue of its own instead of
// one of the GPU_MAX_HW_QUEUES the process's streams share, so the two working
// sets' sub-wavefronts never serialise behind each other or behind the
// caller's streams on a shared queue.  Falls back to a plain
// non-blocking stream if the runtime refuses the mask.
hipError_t create_sub_stream(hipStream_t* s, bool own_queue) {
    if (own_queue) {
        int dev = 0, cus = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0) {
            std::vector<uint32_t> mask(((uint32_t)cus + 31u) / 32u, 0xffffffffu);
            if (cus % 32) mask.back() = (1u << (cus % 32)) - 1u;
            if (hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data()) == hipSuccess) return hipSuccess;
            (void)hipGetLastError();
        }
    }
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

// spt_debug_fail_workspace_alloc: the allocation that fails once (-1: none)
std::atomic<int32_t> g_fail_ws_alloc{-1};
hipError_t ws_malloc(void** p, size_t bytes) {
    int32_t n = g_fail_ws_alloc.load();
    while (n >= 0 && !g_fail_ws_alloc.compare_exchange_weak(n, n - 1)) {
    }
    if (n == 0) {
        *p = nullptr;
        return hipErrorOutOfMemory;
    }
    return hipMalloc(p, bytes);
}

spt_status ensure_workspace(WorkSet& ws, int nsub, size_t cap, uint32_t pad, uint32_t planes, size_t film_bytes,
                            size_t acc_floats, bool own_queues, bool drain_sort) {
    bool quiet = !ws.used;
    const auto quiesce = [&]() -> spt_status {
        if (!quiet) HIP_TRY(hipEventSynchronize(ws.free_ev));
        quiet = true;
        return SPT_OK;
    };
    spt_status st;
    for (int k = 0; k < nsub; k++) {
        Sub& b = ws.sub[k];
        if (cap > b.cap || pad != b.pad || planes > b.planes) {
            if ((st = quiesce())) return st;
            hfree(b.qa); hfree(b.qb); hfree(b.hits);
            b.cap = 0;
            HIP_TRY(ws_malloc((void**)&b.qa, (size_t)16 * planes * queue_stride(cap, pad)));
            HIP_TRY(ws_malloc((void**)&b.qb, (size_t)16 * planes * queue_stride(cap, pad)));
            HIP_TRY(ws_malloc((void**)&b.hits, kHitBytes * cap));
            b.cap = cap;
            b.pad = pad;
            b.planes = planes;
        }
        // spt_config.drain_sort: the forced drain's sort keys / values and hipcub
        // scratch over cap slots, allocated here, where the set is quiesced
        // (not in the middle of an enqueue, behind a host sync)
        if (drain_sort && b.sort_cap < b.cap) {
            if ((st = quiesce())) return st;
            hfree(b.sort_buf);
            if (b.sort_tmp) (void)hipFree(b.sort_tmp);
            b.sort_tmp = nullptr;
            b.sort_cap = 0;
            HIP_TRY(ws_malloc((void**)&b.sort_buf, sizeof(uint32_t) * 4 * b.cap));
            HIP_TRY(launch_drain_sort(DeviceScene{}, PathQueue{}, nullptr, (uint32_t)b.cap, nullptr, nullptr, nullptr,
                                      nullptr, nullptr, &b.sort_tmp_bytes, nullptr));
            HIP_TRY(ws_malloc(&b.sort_tmp, std::max<size_t>(b.sort_tmp_bytes, 16)));
            b.sort_cap = b.cap;
        }
        if (!b.cnt) HIP_TRY(ws_malloc((void**)&b.cnt, sizeof(Counters)));
        if (!b.host_cnt) HIP_TRY(hipHostMalloc((void**)&b.host_cnt, 2 * sizeof(Counters), hipHostMallocDefault));
        for (auto& e : b.count_ev)
            if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        if (!b.join_ev) HIP_TRY(hipEventCreateWithFlags(&b.join_ev, hipEventDisableTiming));
        if (b.stream && b.own_queue != own_queues) {  // the stream kind changed (spt_config.sub_queues)
            if ((st = quiesce())) return st;
            HIP_TRY(hipStreamDestroy(b.stream));
            b.stream = nullptr;
        }
        if (!b.stream) {
            HIP_TRY(create_sub_stream(&b.stream, own_queues));
            b.own_queue = own_queues;
        }
    }
    if (film_bytes > ws.film_cap) {
        if ((st = quiesce())) return st;
        hfree(ws.film);
        ws.film_cap = 0;
        HIP_TRY(ws_malloc((void**)&ws.film, film_bytes));
        ws.film_cap = film_bytes;
    }
    if (acc_floats > ws.acc_cap) {
        if ((st = quiesce())) return st;
        hfree(ws.acc);
        ws.acc_cap = 0;
        HIP_TRY(ws_malloc((void**)&ws.acc, sizeof(float) * acc_floats));
        ws.acc_cap = acc_floats;
    }
    if (!ws.fork_ev) HIP_TRY(hipEventCreateWithFlags(&ws.fork_ev, hipEventDisableTiming));
    if (!ws.free_ev) HIP_TRY(hipEventCreateWithFlags(&ws.free_ev, hipEventDisableTiming));
    if (!ws.call_ev) HIP_TRY(hipEventCreateWithFlags(&ws.call_ev, hipEventDisableTiming));
    return SPT_OK;
}

// After an allocation that failed: the set's path queues, hit records and film
// chunk are freed (once its last render has finished with them), so a retry
// with fewer paths in flight allocates from scratch.  Streams, counters and
// events stay.
spt_status release_queues(WorkSet& ws) {
    if (ws.used) HIP_TRY(hipEventSynchronize(ws.free_ev));
    for (Sub& b : ws.sub) {
        hfree(b.qa); hfree(b.qb); hfree(b.hits); hfree(b.sort_buf);
        if (b.sort_tmp) (void)hipFree(b.sort_tmp);
        b.sort_tmp = nullptr;
        b.cap = 0;
        b.planes = 0;
        b.sort_cap = 0;
    }
    hfree(ws.film);
    ws.film_cap = 0;
    return SPT_OK;
}

// The PCG32 jump table of a render (JumpTable): to each sample's first draw,
// s * (4 + 2D), and from there to the bounce draw of each cast, 4 + 2 * cast
// (main.cpp:395,396,413).  [spp] per sample: seed(initstate, .) then the jump
// past s * (4 + 2D) draws, as one affine map of the stream constant
// (spt_math.h pcg_seeded_jump); then [depth] per cast: the jump past 4 + 2 cast
// draws.  A hit costs nothing; a miss rewrites the least recently used table
// on `stream` once the renders that read it are done.
spt_status ensure_jumps(Workspace& w, hipStream_t stream, uint32_t spp, uint32_t depth, uint64_t initstate,
                        JumpTable** out) {
    JumpTable* t = nullptr;
    for (JumpTable& x : w.jt)
        if (x.valid && x.spp == spp && x.depth == depth && x.state == initstate) t = &x;
    if (t) {
        t->lru = ++w.jt_clock;
        HIP_TRY(hipStreamWaitEvent(stream, t->write_ev, 0));  // written on another stream, perhaps
        *out = t;
        return SPT_OK;
    }
    t = &w.jt[0];
    for (JumpTable& x : w.jt)
        if (!x.valid ? t->valid : x.lru < t->lru) t = &x;
    for (int k = 0; k < kWorkSets; k++)
        if (t->ev_used[k]) HIP_TRY(hipEventSynchronize(t->ev[k]));  // the renders that read it
    if (t->write_ev) HIP_TRY(hipEventSynchronize(t->write_ev));     // and its last write (staging reuse)
    t->valid = false;
    const size_t n = (size_t)spp + kMaxDepthCasts;
    if (n > t->cap) {
        hfree(t->dev);
        if (t->host) (void)hipHostFree(t->host);
        t->host = nullptr;
        t->cap = 0;
        HIP_TRY(hipMalloc((void**)&t->dev, sizeof(PcgJump) * n));
        HIP_TRY(hipHostMalloc((void**)&t->host, sizeof(PcgJump) * n, hipHostMallocDefault));
        t->cap = n;
    }
    if (!t->write_ev) HIP_TRY(hipEventCreateWithFlags(&t->write_ev, hipEventDisableTiming));
    for (auto& e : t->ev)
        if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    const uint64_t per_sample = 4ull + 2ull * depth;
    for (uint32_t s = 0; s < spp; s++) t->host[s] = pcg_seeded_jump(initstate, pcg_jump_coeffs((uint64_t)s * per_sample));
    for (uint32_t j = 0; j < depth; j++) t->host[(size_t)spp + j] = pcg_jump_coeffs(4ull + 2ull * j);
    HIP_TRY(hipMemcpyAsync(t->dev, t->host, sizeof(PcgJump) * ((size_t)spp + depth), hipMemcpyHostToDevice, stream));
    HIP_TRY(hipEventRecord(t->write_ev, stream));
    for (bool& u : t->ev_used) u = false;
    t->spp = spp;
    t->depth = depth;
    t->state = initstate;
    t->valid = true;
    t->lru = ++w.jt_clock;
    *out = t;
    return SPT_OK;
}

spt_status get_event(RenderSlot& r, size_t idx, hipEvent_t* out) {
    while (r.events.size() <= idx) {
        hipEvent_t e;
        HIP_TRY(hipEventCreate(&e));
        r.events.push_back(e);
    }
    *out = r.events[idx];
    return SPT_OK;
}

// The slot of the next render; SPT_ERR_LIMIT when the render kRenderSlots
// tickets earlier was never collected.
spt_status render_slot(Workspace& ws, RenderSlot** out) {
    RenderSlot& r = ws.slots[ws.next_ticket % kRenderSlots];
    if (r.pending)
        return fail(SPT_ERR_LIMIT, "spt_render_async: %d renders queued without spt_render_wait", kRenderSlots);
    if (!r.dev) HIP_TRY(hipMalloc((void**)&r.dev, sizeof(Stats)));
    if (!r.host) HIP_TRY(hipHostMalloc((void**)&r.host, sizeof(Stats), hipHostMallocDefault));
    if (!r.done) HIP_TRY(hipEventCreateWithFlags(&r.done, hipEventDisableTiming));
    r.timed.clear();
    r.rs = spt_render_stats{};
    r.timing = false;
    *out = &r;
    return SPT_OK;
}

// Total length of a set of intervals (their union), sorted by start.
template <typename T>
double interval_union(const std::vector<std::pair<T, T>>& iv) {
    double busy = 0.0, lo = 0.0, hi = -1.0;
    for (auto& x : iv) {
        if (x.first > hi) {
            if (hi > lo) busy += hi - lo;
            lo = x.first;
            hi = x.second;
        } else {
            hi = std::max<double>(hi, x.second);
        }
    }
    if (hi > lo) busy += hi - lo;
    return busy;
}

// Waits for a queued render and fills its statistics (device counters, the
// union of its isect launch intervals, host wall time since it was queued).
spt_status render_collect(RenderSlot& r, Workspace& ws, spt_render_stats* out) {
    const hipEvent_t epoch = ws.epoch;
    spt_render_stats rs = r.rs;
    r.pending = false;
    if (rs.tile_rows) {  // an empty tile queued nothing
        HIP_TRY(hipEventSynchronize(r.done));
        const unsigned long long* hstats = reinterpret_cast<const unsigned long long*>(r.host);
        static_assert(sizeof(Stats) == 13 * sizeof(unsigned long long), "Stats is the 13 counters read back here");
        rs.ray_casts = hstats[0];
        rs.continuations = hstats[1];
        rs.regenerations = hstats[2] > r.regen_base ? hstats[2] - r.regen_base : 0;
        rs.isect_nodes = hstats[3];
        rs.isect_tris = hstats[4];
        rs.isect_lane_steps = hstats[5];
        rs.isect_wave_steps = hstats[6];
        rs.isect_max_stack = hstats[7];
        rs.paths_started = hstats[2];
        rs.paths_terminated = hstats[0] - hstats[1];  // every cast either continues or ends its path
        rs.paths = rs.paths_terminated;
        rs.film_slots_unwritten = hstats[10];
        rs.isect_tri_wave_steps = hstats[8];
        rs.isect_node_wave_steps = hstats[9];
        rs.drained_paths = hstats[11];
        rs.drained_casts = hstats[12];
        if (r.timing) {
            uint64_t nis = 0;
            // launch intervals from the origin: [0] isect (the fused kernel in
            // the fused pipeline), [1] the wavefront's drain
            std::vector<std::pair<float, float>> iv[2];
            for (auto& tk : r.timed) {
                float ms = 0.0f;
                HIP_TRY(hipEventElapsedTime(&ms, r.events[tk.first], r.events[tk.first + 1]));
                if (tk.second == 0) rs.camera_ms += ms;
                else if (tk.second == 1 || tk.second == 4) {
                    float t0 = 0.0f;
                    HIP_TRY(hipEventElapsedTime(&t0, r.events[0], r.events[tk.first]));
                    if (tk.second == 1) {
                        rs.isect_ms += ms;
                        nis++;
                    } else {
                        rs.drain_ms += ms;
                    }
                    iv[tk.second == 4].push_back({t0, t0 + ms});
                } else if (tk.second == 2) rs.shade_ms += ms;
                else rs.resolve_ms += ms;
            }
            rs.isect_launches = nis;
            // launches on the K streams overlap: busy time = union of their intervals
            for (auto& v : iv) std::sort(v.begin(), v.end());
            if (!iv[0].empty() && epoch) {  // the span on the scene's clock, for unions across queued renders
                float t_origin = 0.0f;
                HIP_TRY(hipEventElapsedTime(&t_origin, epoch, r.events[0]));
                float last = iv[0][0].second;
                for (auto& x : iv[0]) last = std::max(last, x.second);
                rs.isect_begin_ms = (double)t_origin + iv[0][0].first;
                rs.isect_end_ms = (double)t_origin + last;
                if (ws.collect_iv)
                    for (int k = 0; k < 2; k++)
                        for (auto& x : iv[k])
                            ws.iv_all[k].push_back({(double)t_origin + x.first, (double)t_origin + x.second});
            }
            rs.isect_busy_ms = interval_union(iv[0]);
            rs.drain_busy_ms = interval_union(iv[1]);
        }
    }
    rs.total_ms = now_ms() - r.wall0;
    if (out) *out = rs;
    return SPT_OK;
}

// LDS stack entries per lane for a BVH8 of `depth` node levels (root = 1).
// Tracer8 pushes the group of node X (level L) only when descending into one
// of X's inner children (level L + 1 <= depth), and the stack then holds one
// group per node on the path root..X: at most depth - 1 entries.  A tight
// stack is LDS, and LDS sets the occupancy (spt_config.stack_slack adds entries).
#ifndef SPT_STACK_CAP
#define SPT_STACK_CAP 0  // experiment only (no overflow handling): cap the LDS stack entries
#endif
uint32_t bvh8_stack_entries(uint32_t depth, uint32_t slack) {
    const uint32_t n = std::max<uint32_t>(1, depth > 1 ? depth - 1 + slack : 1 + slack);
    return SPT_STACK_CAP ? std::min<uint32_t>(n, SPT_STACK_CAP) : n;
}

// Range checks of spt_scene_set_config / spt_scene_create_cfg.
spt_status check_config(const spt_config& c) {
#define CFG_RANGE(f, lo, hi)                                                                         \
    if ((uint64_t)c.f < (uint64_t)(lo) || (uint64_t)c.f > (uint64_t)(hi))                           \
        return fail(SPT_ERR_INVALID, "spt_config.%s = %llu outside [%llu, %llu]", #f, (unsigned long long)c.f, \
                    (unsigned long long)(lo), (unsigned long long)(hi));
    CFG_RANGE(build, 0, SPT_BUILD_GPU_PLOC)
    if (c.bvh_width != 2 && c.bvh_width != 6 && c.bvh_width != 8)
        return fail(SPT_ERR_INVALID, "spt_config.bvh_width must be 2, 6 or 8");
    CFG_RANGE(collapse, 0, 1)
    if (c.ploc_radius != 8 && c.ploc_radius != 16 && c.ploc_radius != 32 && c.ploc_radius != 64)
        return fail(SPT_ERR_INVALID, "spt_config.ploc_radius must be 8, 16, 32 or 64");
    CFG_RANGE(stack_slack, 0, 64)
    CFG_RANGE(pipeline, 0, SPT_PIPELINE_FUSED)
    CFG_RANGE(wavefront_paths, 1, 0x7fffffffu)
    CFG_RANGE(streams, 1, kMaxStreams)
    CFG_RANGE(isect_refill_idle, 1, 64)
    CFG_RANGE(isect_static_share_q8, 0, 255)
    CFG_RANGE(isect_chunk, 1, 4096)
    CFG_RANGE(isect_grid_q8, 0, 4096)
    CFG_RANGE(xcd_remap, 0, 7)
    CFG_RANGE(fused_refill_idle, 1, 64)
    CFG_RANGE(fused_static_share_q8, 0, 255)
    CFG_RANGE(fused_grid_q8, 0, 4096)
    CFG_RANGE(plane_pad, 0, 1u << 20)
    CFG_RANGE(film_budget_bytes, 12, UINT64_MAX)
    CFG_RANGE(public_persistent, 0, 1)
    CFG_RANGE(public_refill_idle, 1, 64)
    CFG_RANGE(pack_groups, 0, 2)
    CFG_RANGE(pixel_block, 0, 64)
    CFG_RANGE(work_order, 0, SPT_WORK_PIXEL_MAJOR)
    CFG_RANGE(queue_cache, 0, SPT_QUEUE_CACHE_STREAM)
    CFG_RANGE(drain_q8, 0, 65535)
    CFG_RANGE(drain_grid_q8, 0, 4096)
    CFG_RANGE(drain_casts, 0, 64)
    CFG_RANGE(fit_streams, 1, kMaxStreams)
    CFG_RANGE(fit_paths, 0, 1ull << 31)
    CFG_RANGE(sub_queues, 0, 1)
    CFG_RANGE(drain_sort, 0, 1)
    CFG_RANGE(lockstep_first, 0, 3)
    CFG_RANGE(fit_chunks, 0, 1)
    CFG_RANGE(drain_refill_idle, 0, 64)
#undef CFG_RANGE
    return SPT_OK;
}

// spt_scene_create on the GPU: upload the indexed mesh as is, assemble the
// triangle soup, PLOC + collapse (gpu_build.hip), slot-ordered arrays.
spt_status create_scene_gpu(const int32_t* pos_tri, const float* pos, uint64_t nvert, uint64_t ntri,
                            const int32_t* nrm_tri, const float* nrm, uint64_t nnrm, const int32_t* tc_tri,
                            const float* tc, uint64_t ntc, const int32_t* mat_id, const spt_config& cfg, double t0,
                            spt_scene* out) {
    struct Raw {
        int32_t *pt = nullptr, *nt = nullptr, *tt = nullptr, *mat = nullptr;
        float *p = nullptr, *n = nullptr, *t = nullptr, *tv = nullptr;
        ~Raw() { hfree(pt); hfree(nt); hfree(tt); hfree(mat); hfree(p); hfree(n); hfree(t); hfree(tv); }
    } raw;
    spt_status us = SPT_OK;
    if (!us) us = upload(&raw.pt, pos_tri, ntri * 3 * sizeof(int32_t));
    if (!us) us = upload(&raw.p, pos, nvert * 3 * sizeof(float));
    if (!us && nrm_tri) us = upload(&raw.nt, nrm_tri, ntri * 3 * sizeof(int32_t));
    if (!us && nrm_tri) us = upload(&raw.n, nrm, nnrm * 3 * sizeof(float));
    const bool with_tc = tc_tri && tc;
    if (!us && with_tc) us = upload(&raw.tt, tc_tri, ntri * 3 * sizeof(int32_t));
    if (!us && with_tc) us = upload(&raw.t, tc, ntc * 2 * sizeof(float));
    if (!us && mat_id) us = upload(&raw.mat, mat_id, ntri * sizeof(int32_t));
    if (us) return us;
    HIP_TRY(hipMalloc((void**)&raw.tv, sizeof(float) * 9 * std::max<uint64_t>(ntri, 1)));
    DeviceMeshIn m{raw.pt, raw.p, raw.nt, raw.n, raw.tt, raw.t, raw.mat, (uint32_t)ntri};
    hipStream_t s = nullptr;  // the null stream: scene creation is synchronous
    HIP_TRY(gpu_mesh_soup(m, raw.tv, s));
    GpuBvh8 g;
    const int width = (int)cfg.bvh_width;
    HIP_TRY(gpu_build_bvh8(raw.tv, (uint32_t)ntri, s, &g, (int)cfg.ploc_radius, cfg.collapse == 1, width));
    spt_scene_t* sc = new spt_scene_t();
    sc->cfg = cfg;
    (void)hipGetDevice(&sc->device);
    sc->ntri = ntri;
    sc->stack_depth = bvh8_stack_entries(g.depth, cfg.stack_slack);
    uint32_t nslots = 0;
    {
        uint32_t* holes = nullptr;
        const hipError_t he = gpu_bvh8_holes(g.nodes8, g.nnodes, s, &holes, &nslots, width,
                                             cfg.pack_groups ? &sc->group_shift : nullptr, cfg.pack_groups == 2);
        (void)hipFree(g.nodes8);
        if (he) {
            (void)hipFree(g.slot2tri);
            delete sc;
            return fail(he == hipErrorOutOfMemory ? SPT_ERR_OOM : SPT_ERR_HIP, "spt_scene_create (BVH8 layout): %s",
                        hipGetErrorString(he));
        }
        sc->nodes8 = (uint4*)holes;
        sc->node6 = width == 6;
        sc->node_bytes = holes ? (uint64_t)nslots * (width == 6 ? kNode6Quads : kNode8Quads) * 16 : 0;
    }
    auto bail = [&](hipError_t e) {
        (void)hipFree(g.slot2tri);
        sc->release();
        delete sc;
        return fail(e == hipErrorOutOfMemory ? SPT_ERR_OOM : SPT_ERR_HIP, "spt_scene_create (GPU build): %s",
                    hipGetErrorString(e));
    };
    hipError_t e = hipSuccess;
    if (!e) e = hipMalloc((void**)&sc->tris, sizeof(float4) * kTriQuads * std::max<uint64_t>(ntri, 1));
    if (!e) e = hipMalloc((void**)&sc->snrm, sizeof(float4) * 3 * std::max<uint64_t>(ntri, 1));
    if (!e && with_tc) e = hipMalloc((void**)&sc->tc, sizeof(float) * 6 * ntri);
    if (!e) e = hipMalloc((void**)&sc->orig2slot, sizeof(int32_t) * std::max<uint64_t>(ntri, 1));
    if (!e) e = gpu_scene_slots(m, raw.tv, g.slot2tri, sc->tris, sc->snrm, with_tc ? sc->tc : nullptr,
                                sc->orig2slot, s);
    if (!e) e = hipStreamSynchronize(s);
    if (e) return bail(e);
    (void)hipFree(g.slot2tri);
    const float one[3] = {1.0f, 1.0f, 1.0f};
    if ((us = upload(&sc->albedo, one, sizeof(one)))) {
        sc->release();
        delete sc;
        return us;
    }
    sc->nmat = 1;
    spt_scene_stats& ss = sc->stats;
    ss.ntri = ntri;
    ss.nodes = g.nnodes;
    ss.leaves = g.leaves;
    ss.max_depth = g.depth;
    ss.max_leaf = 3;
    ss.bvh_width = (uint32_t)width;
    ss.builder = SPT_BUILD_GPU_PLOC;
    ss.device_bytes = (uint64_t)nslots * (width == 6 ? kNode6Quads : kNode8Quads) * 16 + ntri * (kTriQuads + 3) * 16 +
                      (with_tc ? ntri * 24 : 0) + ntri * 4;
    ss.build_ms = now_ms() - t0;
    ss.sah_cost = g.sah_cost;
    *out = sc;
    return SPT_OK;
}

}  // namespace

spt_status spt_set_error(spt_status code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

extern "C" {

const char* spt_last_error(void) { return g_last_error.c_str(); }
const char* spt_version(void) { return "spt-mi355x 0.1 (gfx950 wavefront path tracer)"; }

#ifndef SPT_BUILD_ID
#define SPT_BUILD_ID "unknown"
#endif
const char* spt_build_id(void) { return SPT_BUILD_ID; }

void spt_debug_fail_workspace_alloc(int32_t nth) { g_fail_ws_alloc.store(nth < 0 ? -1 : nth); }

spt_status spt_init(int32_t device) {
    spt_status st = ensure_device();
    if (st) return st;
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipFree(nullptr));  // create the context now, not in the first timed call
    return SPT_OK;
}

void spt_default_params(spt_render_params* p) {
    std::memset(p, 0, sizeof(*p));
    p->width = 512; p->height = 512; p->spp = 100; p->max_depth = 2;  // main.cpp:357-361
    const float from[3] = {0.0f, 3.03f, 5.0f}, at[3] = {0.0f, 0.03f, 0.0f}, up[3] = {0.0f, 1.0f, 0.0f};
    std::memcpy(p->camera.look_from, from, sizeof(from));               // main.cpp:383
    std::memcpy(p->camera.look_at, at, sizeof(at));
    std::memcpy(p->camera.up, up, sizeof(up));
    p->camera.lens_radius = 0.0f;
    p->camera.focal_dist = 1.0f;
    p->camera.fov_y = 40.0f / 180.0f * (float)M_PI;
    p->camera.film_size_y = 0.035f;                                    // pinhole.h:11
    p->tile_index = 0; p->tile_count = 1; p->rows_per_group = 1;
    p->wavefront_paths = 0;
    p->rr_start_depth = 1;
    p->rng_order = SPT_RNG_Y_FIRST;
    p->rng_initstate = kPcgDefaultState;
    p->env[0] = p->env[1] = p->env[2] = 1.0f;
    p->flags = 0;
}

uint32_t spt_tile_rows(uint32_t height, uint32_t tile_index, uint32_t tile_count, uint32_t rows_per_group,
                       uint32_t* rows, uint32_t cap) {
    if (tile_count == 0 || rows_per_group == 0 || tile_index >= tile_count) return 0;
    uint32_t n = 0;
    for (uint32_t r = 0; r < height; r++) {
        if ((r / rows_per_group) % tile_count != tile_index) continue;
        if (rows && n < cap) rows[n] = r;
        n++;
    }
    return n;
}

spt_status spt_scene_create(const int32_t* pos_tri, const float* pos, uint64_t nvert, uint64_t ntri,
                            const int32_t* nrm_tri, const float* nrm, uint64_t nnrm, const int32_t* tc_tri,
                            const float* tc, uint64_t ntc, const int32_t* mat_id, spt_scene* out) {
    return spt_scene_create_ex(pos_tri, pos, nvert, ntri, nrm_tri, nrm, nnrm, tc_tri, tc, ntc, mat_id, SPT_BUILD_AUTO,
                               out);
}

spt_status spt_scene_create_ex(const int32_t* pos_tri, const float* pos, uint64_t nvert, uint64_t ntri,
                               const int32_t* nrm_tri, const float* nrm, uint64_t nnrm, const int32_t* tc_tri,
                               const float* tc, uint64_t ntc, const int32_t* mat_id, uint32_t build,
                               spt_scene* out) {
    if (build > SPT_BUILD_GPU_PLOC) return fail(SPT_ERR_INVALID, "spt_scene_create: unknown builder %u", build);
    spt_config cfg;
    spt_default_config(&cfg);
    cfg.build = build;
    return spt_scene_create_cfg(pos_tri, pos, nvert, ntri, nrm_tri, nrm, nnrm, tc_tri, tc, ntc, mat_id, &cfg, out);
}

spt_status spt_scene_create_cfg(const int32_t* pos_tri, const float* pos, uint64_t nvert, uint64_t ntri,
                                const int32_t* nrm_tri, const float* nrm, uint64_t nnrm, const int32_t* tc_tri,
                                const float* tc, uint64_t ntc, const int32_t* mat_id, const spt_config* cfg_in,
                                spt_scene* out) {
    if (!out) return fail(SPT_ERR_INVALID, "spt_scene_create: out is NULL");
    *out = nullptr;
    spt_config cfg;
    if (cfg_in) cfg = *cfg_in;
    else spt_default_config(&cfg);
    spt_status st = check_config(cfg);
    if (st) return st;
    if (ntri > 0 && (!pos_tri || !pos)) return fail(SPT_ERR_INVALID, "spt_scene_create: NULL positions");
    if (ntri >= kMaxTriangles) return fail(SPT_ERR_LIMIT, "spt_scene_create: %llu triangles exceeds 2^28", (unsigned long long)ntri);
    if (nrm_tri && !nrm && nnrm) return fail(SPT_ERR_INVALID, "spt_scene_create: normal indices without normals");
    st = ensure_device();
    if (st) return st;
    uint32_t build = cfg.build;
    if (build == SPT_BUILD_AUTO) build = ntri >= cfg.gpu_build_min_tris ? SPT_BUILD_GPU_PLOC : SPT_BUILD_HOST_SAH;
    const bool use8 = cfg.bvh_width != 2;  // compressed wide BVH (8 or 6 children per node)
    const int width = (int)cfg.bvh_width;
    if (build == SPT_BUILD_GPU_PLOC && !use8) build = SPT_BUILD_HOST_SAH;  // the GPU builder makes BVH8 only
    const double t0 = now_ms();
    const bool host = build == SPT_BUILD_HOST_SAH;
    std::vector<float> tv(host ? (size_t)ntri * 9 : 0);
    for (uint64_t t = 0; t < ntri; t++) {
        for (int k = 0; k < 3; k++) {
            int64_t pi = pos_tri[t * 3 + k];
            if (pi < 0 || (uint64_t)pi >= nvert)
                return fail(SPT_ERR_INVALID, "spt_scene_create: triangle %llu position index %lld out of range [0,%llu)",
                            (unsigned long long)t, (long long)pi, (unsigned long long)nvert);
            if (host)
                for (int c = 0; c < 3; c++) tv[t * 9 + k * 3 + c] = pos[pi * 3 + c];
        }
        if (nrm_tri)
            for (int k = 0; k < 3; k++) {
                int64_t ni = nrm_tri[t * 3 + k];
                if (ni < -1 || (ni >= 0 && (uint64_t)ni >= nnrm))
                    return fail(SPT_ERR_INVALID, "spt_scene_create: triangle %llu normal index %lld out of range",
                                (unsigned long long)t, (long long)ni);
            }
        if (tc_tri && tc)
            for (int k = 0; k < 3; k++) {
                int64_t ti = tc_tri[t * 3 + k];
                if (ti < -1 || (ti >= 0 && (uint64_t)ti >= ntc))
                    return fail(SPT_ERR_INVALID, "spt_scene_create: triangle %llu texcoord index %lld out of range",
                                (unsigned long long)t, (long long)ti);
            }
    }
    if (!host)
        return create_scene_gpu(pos_tri, pos, nvert, ntri, nrm_tri, nrm, nnrm, tc_tri, tc, ntc, mat_id, cfg, t0, out);
    // Acceleration structure: the compressed 8-wide BVH by default;
    // spt_config.bvh_width = 2 selects the plain BVH2 (the simple reference layout).
    BvhBuildResult bvh;
    Bvh8BuildResult bvh8;
    if (use8)
        bvh8 = build_bvh8(tv.data(), ntri, cfg.collapse == 1, width);
    else
        bvh = build_bvh(tv.data(), ntri);
    const std::vector<uint32_t>& slot2tri = use8 ? bvh8.slot2tri : bvh.slot2tri;
    const double t1 = now_ms();

    // Slot-ordered device arrays.
    std::vector<float4> h_tris((size_t)ntri * kTriQuads), h_snrm((size_t)ntri * 3);
    std::vector<float> h_tc(tc_tri && tc ? (size_t)ntri * 6 : 0);
    std::vector<int32_t> h_o2s((size_t)ntri);
    for (uint64_t s = 0; s < ntri; s++) {
        const uint32_t t = slot2tri[s];
        h_o2s[t] = (int32_t)s;
        const float* v = &tv[(size_t)t * 9];
        tri_record_fill((float*)&h_tris[s * kTriQuads], v, t);
        // Geometric normal fallback for a missing vertex normal (index -1).
        V3 g = normalize(cross(v3(v[3] - v[0], v[4] - v[1], v[5] - v[2]), v3(v[6] - v[0], v[7] - v[1], v[8] - v[2])));
        int32_t mat = mat_id ? mat_id[t] : 0;
        for (int k = 0; k < 3; k++) {
            int64_t ni = nrm_tri ? nrm_tri[t * 3 + k] : -1;
            V3 n = ni >= 0 ? v3(nrm[ni * 3], nrm[ni * 3 + 1], nrm[ni * 3 + 2]) : g;
            float w = 0.0f;
            if (k == 0) std::memcpy(&w, &mat, 4);
            h_snrm[s * 3 + k] = make_float4(n.x, n.y, n.z, w);
        }
        if (!h_tc.empty())
            for (int k = 0; k < 3; k++) {
                int64_t ti = tc_tri[t * 3 + k];
                h_tc[s * 6 + k * 2] = ti >= 0 ? tc[ti * 2] : 0.0f;
                h_tc[s * 6 + k * 2 + 1] = ti >= 0 ? tc[ti * 2 + 1] : 0.0f;
            }
    }

    spt_scene_t* sc = new spt_scene_t();
    sc->cfg = cfg;
    (void)hipGetDevice(&sc->device);
    sc->ntri = ntri;
    sc->stack_depth = use8 ? bvh8_stack_entries(bvh8.depth, cfg.stack_slack) : std::max<uint32_t>(1, bvh.max_depth + 1);
    const float one[3] = {1.0f, 1.0f, 1.0f};
    spt_status us = SPT_OK;
    uint32_t nslots = 0;
    if (use8) {
        // pad each 80-B node to its own 128-B cache line (kNode8Quads x 16 B),
        // then re-lay it on the device with the children at w4 + slot
        const size_t nn = bvh8.nodes.size() / 20;
        std::vector<uint32_t> padded(nn * kNode8Quads * 4, 0u);
        for (size_t i = 0; i < nn; i++)
            std::memcpy(&padded[i * kNode8Quads * 4], &bvh8.nodes[i * 20], 80);
        uint32_t* compact = nullptr;
        if (!us) us = upload(&compact, padded.data(), padded.size() * sizeof(uint32_t));
        if (!us) {
            uint32_t* holes = nullptr;
            const hipError_t he = gpu_bvh8_holes(compact, (uint32_t)nn, nullptr, &holes, &nslots, width,
                                                 cfg.pack_groups ? &sc->group_shift : nullptr, cfg.pack_groups == 2);
            if (he) us = fail(he == hipErrorOutOfMemory ? SPT_ERR_OOM : SPT_ERR_HIP,
                              "spt_scene_create (BVH8 layout): %s", hipGetErrorString(he));
            else {
                sc->nodes8 = (uint4*)holes;
                sc->node6 = width == 6;
                sc->node_bytes = holes ? (uint64_t)nslots * (width == 6 ? kNode6Quads : kNode8Quads) * 16 : 0;
            }
        }
        hfree(compact);
    } else {
        if (!us) us = upload(&sc->nodes, bvh.nodes.data(), bvh.nodes.size() * sizeof(float));
        if (!us && sc->nodes) sc->node_bytes = bvh.nodes.size() * sizeof(float);
    }
    if (!us) us = upload(&sc->tris, h_tris.data(), h_tris.size() * sizeof(float4));
    if (!us) us = upload(&sc->snrm, h_snrm.data(), h_snrm.size() * sizeof(float4));
    if (!us) us = upload(&sc->tc, h_tc.data(), h_tc.size() * sizeof(float));
    if (!us) us = upload(&sc->orig2slot, h_o2s.data(), h_o2s.size() * sizeof(int32_t));
    if (!us) us = upload(&sc->albedo, one, sizeof(one));
    if (us) {
        sc->release();
        delete sc;
        return us;
    }
    sc->nmat = 1;
    spt_scene_stats& ss = sc->stats;
    ss.ntri = ntri;
    ss.nodes = use8 ? bvh8.nodes.size() / 20 : bvh.nodes.size() / 16;
    ss.leaves = use8 ? bvh8.leaves : bvh.leaves;
    ss.max_depth = use8 ? bvh8.depth : bvh.max_depth;
    ss.max_leaf = use8 ? 3 : bvh.max_leaf;
    ss.bvh_width = (uint32_t)width;
    ss.device_bytes = (use8 ? (uint64_t)nslots * (width == 6 ? kNode6Quads : kNode8Quads) * 16 : bvh.nodes.size() * 4) +
                      (h_tris.size() + h_snrm.size()) * 16 +
                      h_tc.size() * 4 + h_o2s.size() * 4;
    ss.build_ms = t1 - t0;
    ss.sah_cost = use8 ? bvh8.sah_cost : bvh.sah_cost;
    ss.builder = SPT_BUILD_HOST_SAH;
    *out = sc;
    return SPT_OK;
}

spt_status spt_scene_set_albedo(spt_scene sc, const float* albedo_rgb, uint32_t nmat) {
    if (!sc || !albedo_rgb || nmat == 0) return fail(SPT_ERR_INVALID, "spt_scene_set_albedo: bad arguments");
    DeviceGuard dg(sc->device);
    float* d = nullptr;
    HIP_TRY(hipMalloc((void**)&d, sizeof(float) * 3 * nmat));
    HIP_TRY(hipMemcpy(d, albedo_rgb, sizeof(float) * 3 * nmat, hipMemcpyHostToDevice));
    std::lock_guard<std::mutex> lk(sc->mu);
    spt_status qs = quiesce_scene(sc);  // queued renders / calls may still read the old table
    if (qs) {
        hfree(d);
        return qs;
    }
    hfree(sc->albedo);
    sc->albedo = d;
    sc->nmat = nmat;
    bool unit = true;
    for (uint32_t i = 0; i < 3 * nmat; i++) unit = unit && albedo_rgb[i] == 1.0f;
    sc->albedo_unit = unit;
    return SPT_OK;
}

spt_status spt_scene_set_emission(spt_scene sc, const float* emission_rgb, uint32_t nmat) {
    if (!sc) return fail(SPT_ERR_INVALID, "spt_scene_set_emission: NULL scene");
    DeviceGuard dg(sc->device);
    std::lock_guard<std::mutex> lk(sc->mu);
    spt_status qs = quiesce_scene(sc);  // queued renders may still read the old table
    if (qs) return qs;
    hfree(sc->emission);
    sc->nemit = 0;
    if (!emission_rgb || nmat == 0) return SPT_OK;  // no emitters
    bool any = false;
    for (uint32_t i = 0; i < 3 * nmat; i++) any |= emission_rgb[i] != 0.0f;
    if (!any) return SPT_OK;
    float* d = nullptr;
    HIP_TRY(hipMalloc((void**)&d, sizeof(float) * 3 * nmat));
    HIP_TRY(hipMemcpy(d, emission_rgb, sizeof(float) * 3 * nmat, hipMemcpyHostToDevice));
    sc->emission = d;
    sc->nemit = nmat;
    return SPT_OK;
}

void spt_default_config(spt_config* c) {
    if (!c) return;
    std::memset(c, 0, sizeof(*c));
    c->build = SPT_BUILD_AUTO;
    c->bvh_width = 6;
    c->gpu_build_min_tris = 2000000;
    c->collapse = 0;
    c->ploc_radius = 16;
    c->stack_slack = 0;
    c->pipeline = SPT_PIPELINE_AUTO;
    c->fused_max_paths = kDefaultFusedMaxPaths;
    c->wavefront_paths = kDefaultWavefrontPaths;
    c->streams = 4;
    c->isect_refill_idle = 24;
    c->isect_static_share_q8 = 128;
    c->isect_chunk = kIsectChunk;
    c->isect_grid_q8 = 0;
    c->xcd_remap = 3;
    c->fused_refill_idle = 32;
    c->fused_static_share_q8 = 32;
    c->fused_grid_q8 = 256;
    c->plane_pad = 0;
    c->film_budget_bytes = 4ull << 30;
    c->public_persistent = 0;
    c->public_refill_idle = kRefillIdle;
    c->pack_groups = 1;
    c->pixel_block = 0;
    c->work_order = SPT_WORK_AUTO;
    c->queue_cache = SPT_QUEUE_CACHE_AUTO;
    c->drain_q8 = kDefaultDrainQ8;
    c->drain_grid_q8 = 0;
    c->drain_casts = kDefaultDrainCasts;
    c->fit_streams = 1;
    c->drain_refill_idle = 0;
    c->fit_paths = kDefaultFitPaths;
    c->sub_queues = 1;
    c->drain_sort = 0;
    c->lockstep_first = 3;
    c->fit_chunks = 1;
}

spt_status spt_scene_set_config(spt_scene sc, const spt_config* cfg) {
    if (!sc || !cfg) return fail(SPT_ERR_INVALID, "spt_scene_set_config: NULL argument");
    spt_status st = check_config(*cfg);
    if (st) return st;
    std::lock_guard<std::mutex> lk(sc->mu);
    const spt_config old = sc->cfg;
    sc->cfg = *cfg;
    // the scene keeps the build it has
    sc->cfg.build = old.build; sc->cfg.bvh_width = old.bvh_width; sc->cfg.gpu_build_min_tris = old.gpu_build_min_tris;
    sc->cfg.collapse = old.collapse; sc->cfg.ploc_radius = old.ploc_radius; sc->cfg.stack_slack = old.stack_slack;
    sc->cfg.pack_groups = old.pack_groups;
    return SPT_OK;
}

spt_status spt_scene_get_config(spt_scene sc, spt_config* out) {
    if (!sc || !out) return fail(SPT_ERR_INVALID, "spt_scene_get_config: NULL argument");
    std::lock_guard<std::mutex> lk(sc->mu);
    *out = sc->cfg;
    return SPT_OK;
}

spt_status spt_scene_set_texture(spt_scene sc, uint32_t material, const float* rgb, uint32_t width, uint32_t height) {
    if (!sc) return fail(SPT_ERR_INVALID, "spt_scene_set_texture: NULL scene");
    DeviceGuard dg(sc->device);
    if (rgb && (width == 0 || height == 0)) return fail(SPT_ERR_INVALID, "spt_scene_set_texture: empty image");
    if (rgb && (uint64_t)width * height > (1ull << 26))
        return fail(SPT_ERR_LIMIT, "spt_scene_set_texture: %u x %u texels exceeds 2^26", width, height);
    if (material >= (1u << 20)) return fail(SPT_ERR_LIMIT, "spt_scene_set_texture: material %u >= 2^20", material);
    std::lock_guard<std::mutex> lk(sc->mu);
    spt_status qs = quiesce_scene(sc);  // queued renders may still read the old images (upload_textures frees them)
    if (qs) return qs;
    if (material >= sc->tex_img.size()) {
        sc->tex_img.resize(material + 1);
        sc->tex_w.resize(material + 1, 0);
        sc->tex_h.resize(material + 1, 0);
    }
    std::vector<float4>& img = sc->tex_img[material];
    img.clear();
    sc->tex_w[material] = sc->tex_h[material] = 0;
    if (rgb) {
        img.resize((size_t)width * height);
        for (size_t i = 0; i < img.size(); i++) img[i] = make_float4(rgb[i * 3], rgb[i * 3 + 1], rgb[i * 3 + 2], 0.0f);
        sc->tex_w[material] = width;
        sc->tex_h[material] = height;
    }
    return upload_textures(sc);
}

namespace {

// Rebuild the texture device arrays from the host copies (caller holds sc->mu):
// one texel array, one (first, w, h, has) entry per material.
spt_status upload_textures(spt_scene_t* sc) {
    std::vector<uint4> info(sc->tex_img.size());
    std::vector<float4> all;
    uint32_t used = 0;
    for (size_t m = 0; m < sc->tex_img.size(); m++) {
        const bool has = !sc->tex_img[m].empty();
        info[m] = make_uint4((uint32_t)all.size(), sc->tex_w[m], sc->tex_h[m], has ? 1u : 0u);
        all.insert(all.end(), sc->tex_img[m].begin(), sc->tex_img[m].end());
        if (has) used = (uint32_t)m + 1;
    }
    hfree(sc->tex_info);
    hfree(sc->texels);
    sc->ntex = 0;
    if (used) {
        spt_status us = upload(&sc->tex_info, info.data(), sizeof(uint4) * used);
        if (!us) us = upload(&sc->texels, all.data(), sizeof(float4) * all.size());
        if (us) return us;
        sc->ntex = used;
    }
    return SPT_OK;
}

}  // namespace

spt_status spt_scene_set_spheres(spt_scene sc, const float* center_radius, const int32_t* mat_id, uint32_t n) {
    if (!sc) return fail(SPT_ERR_INVALID, "spt_scene_set_spheres: NULL scene");
    DeviceGuard dg(sc->device);
    if (n > 256) return fail(SPT_ERR_LIMIT, "spt_scene_set_spheres: %u spheres (at most 256)", n);
    if (n && !center_radius) return fail(SPT_ERR_INVALID, "spt_scene_set_spheres: NULL spheres");
    for (uint32_t k = 0; k < n; k++) {
        const float* c = center_radius + (size_t)k * 4;
        if (!std::isfinite(c[0]) || !std::isfinite(c[1]) || !std::isfinite(c[2]))
            return fail(SPT_ERR_INVALID, "spt_scene_set_spheres: sphere %u centre must be finite", k);
        if (!(c[3] > 0.0f) || !std::isfinite(c[3]))
            return fail(SPT_ERR_INVALID, "spt_scene_set_spheres: sphere %u radius must be finite and > 0", k);
    }
    std::lock_guard<std::mutex> lk(sc->mu);
    spt_status qs = quiesce_scene(sc);  // queued renders / calls may still read the old spheres
    if (qs) return qs;
    hfree(sc->spheres);
    hfree(sc->sph_mat);
    sc->nsph = 0;
    if (!n) return SPT_OK;
    std::vector<int32_t> mats(n, 0);
    if (mat_id) std::memcpy(mats.data(), mat_id, sizeof(int32_t) * n);
    spt_status us = upload(&sc->spheres, center_radius, sizeof(float4) * n);
    if (!us) us = upload(&sc->sph_mat, mats.data(), sizeof(int32_t) * n);
    if (us) return us;
    sc->nsph = n;
    return SPT_OK;
}

spt_status spt_scene_set_material_kinds(spt_scene sc, const uint32_t* kinds, uint32_t nmat) {
    if (!sc) return fail(SPT_ERR_INVALID, "spt_scene_set_material_kinds: NULL scene");
    DeviceGuard dg(sc->device);
    for (uint32_t i = 0; kinds && i < nmat; i++)
        if (kinds[i] > SPT_MAT_GLASS) return fail(SPT_ERR_INVALID, "spt_scene_set_material_kinds: kind %u of material %u", kinds[i], i);
    std::lock_guard<std::mutex> lk(sc->mu);
    spt_status qs = quiesce_scene(sc);  // queued renders may still read the old kinds
    if (qs) return qs;
    hfree(sc->mat_kind);
    sc->nkind = 0;
    bool any = false;
    for (uint32_t i = 0; kinds && i < nmat; i++) any = any || kinds[i] != SPT_MAT_DIFFUSE;
    if (!any) return SPT_OK;  // all diffuse: the default
    spt_status us = upload(&sc->mat_kind, kinds, sizeof(uint32_t) * nmat);
    if (us) return us;
    sc->nkind = nmat;
    return SPT_OK;
}

spt_status spt_scene_get_stats(spt_scene sc, spt_scene_stats* out) {
    if (!sc || !out) return fail(SPT_ERR_INVALID, "spt_scene_get_stats: NULL argument");
    *out = sc->stats;
    return SPT_OK;
}

spt_status spt_bvh_build_stats(const float* tv, uint64_t ntri, const spt_config* cfg_in, spt_scene_stats* out) {
    if (!out || (ntri > 0 && !tv)) return fail(SPT_ERR_INVALID, "spt_bvh_build_stats: NULL argument");
    if (ntri >= kMaxTriangles) return fail(SPT_ERR_LIMIT, "spt_bvh_build_stats: %llu triangles exceeds 2^28",
                                           (unsigned long long)ntri);
    spt_config cfg;
    if (cfg_in) cfg = *cfg_in;
    else spt_default_config(&cfg);
    spt_status st = check_config(cfg);
    if (st) return st;
    spt_scene_stats ss{};
    const double t0 = now_ms();
    if (cfg.bvh_width != 2) {
        const Bvh8BuildResult b = build_bvh8(tv, ntri, cfg.collapse == 1, (int)cfg.bvh_width);
        ss.nodes = b.nodes.size() / 20; ss.leaves = b.leaves; ss.max_depth = b.depth; ss.max_leaf = 3;
        ss.sah_cost = b.sah_cost;
        if (b.slot2tri.size() != ntri) return fail(SPT_ERR_HIP, "spt_bvh_build_stats: BVH8 lost triangles");
    } else {
        const BvhBuildResult b = build_bvh(tv, ntri);
        ss.nodes = b.nodes.size() / 16; ss.leaves = b.leaves; ss.max_depth = b.max_depth; ss.max_leaf = b.max_leaf;
        ss.sah_cost = b.sah_cost;
        if (b.slot2tri.size() != ntri) return fail(SPT_ERR_HIP, "spt_bvh_build_stats: BVH2 lost triangles");
    }
    ss.ntri = ntri;
    ss.bvh_width = cfg.bvh_width;
    ss.builder = SPT_BUILD_HOST_SAH;
    ss.build_ms = now_ms() - t0;
    *out = ss;
    return SPT_OK;
}

spt_status spt_scene_destroy(spt_scene sc) {
    if (!sc) return SPT_OK;
    DeviceGuard dg(sc->device);
    {
        std::lock_guard<std::mutex> lk(sc->mu);
        (void)quiesce_scene(sc);  // nothing queued may still read what is freed
    }
    sc->release();
    delete sc;
    return SPT_OK;
}

// ---------------------------------------------------------------- scene cache
// spt_scene_save / spt_scene_load / spt_scene_cache_info (include/spt.h).
namespace {

constexpr char kCacheMagic[8] = {'S', 'P', 'T', 'S', 'C', 'E', 'N', 'E'};
constexpr uint32_t kCacheVersion = 2;  // 2: 64-B rotated triangle records (spt_internal.h)
constexpr size_t kCacheChunk = size_t(64) << 20;  // host staging per read / write / download

// Sections, in file order.
enum : uint32_t {
    kSecNodes, kSecTris, kSecSnrm, kSecTc, kSecOrig2Slot, kSecAlbedo, kSecEmission, kSecSpheres, kSecSphMat,
    kSecKinds, kSecTexDims, kSecTexels, kSecExtra, kNumSecs
};
const char* const kSecName[kNumSecs] = {"nodes", "triangles", "normals", "texcoords", "orig2slot", "albedo",
                                        "emission", "spheres", "sphere materials", "material kinds",
                                        "texture sizes", "texels", "extra"};

struct CacheHeader {
    char magic[8];
    uint32_t version, header_bytes;
    uint32_t tri_quads, node_quads;      // the writer's layout: 16-B quads per triangle slot / node slot
    uint32_t node6, group_shift;
    uint32_t config_bytes, stats_bytes;  // sizeof(spt_config), sizeof(spt_scene_stats)
    uint32_t stack_depth, nmat, nemit, nsph, nkind, ntexmat;
    uint64_t ntri;
    uint64_t bytes[kNumSecs];
    uint64_t sum[kNumSecs];
    spt_config cfg;
    spt_scene_stats stats;
};

// 16-B quads per node slot of a scene of this build with the given width.
uint32_t node_quads_of(uint32_t width, uint32_t node6) {
    return width == 2 ? 4u : (node6 ? (uint32_t)kNode6Quads : (uint32_t)kNode8Quads);
}

// Section checksum: four 64-bit multiply-xorshift lanes over 32-B blocks
// (streamed in any split), folded with the length.
class CacheHash {
    static constexpr uint64_t kMul = 0x9fb21c651e98df25ull;
    uint64_t h_[4] = {0x243f6a8885a308d3ull, 0x13198a2e03707344ull, 0xa4093822299f31d0ull, 0x082efa98ec4e6c89ull};
    uint8_t tail_[32];
    size_t nt_ = 0;
    uint64_t len_ = 0;
    void block(const uint8_t* p) {
        for (int k = 0; k < 4; k++) {
            uint64_t w;
            std::memcpy(&w, p + 8 * k, 8);
            h_[k] = (h_[k] ^ w) * kMul;
            h_[k] ^= h_[k] >> 31;
        }
    }

  public:
    void update(const void* data, size_t n) {
        const uint8_t* p = (const uint8_t*)data;
        len_ += n;
        if (nt_) {
            const size_t take = std::min(32 - nt_, n);
            std::memcpy(tail_ + nt_, p, take);
            nt_ += take; p += take; n -= take;
            if (nt_ < 32) return;
            block(tail_);
            nt_ = 0;
        }
        for (; n >= 32; p += 32, n -= 32) block(p);
        std::memcpy(tail_, p, n);
        nt_ = n;
    }
    uint64_t digest() {
        std::memset(tail_ + nt_, 0, 32 - nt_);
        block(tail_);
        uint64_t r = len_;
        for (int k = 0; k < 4; k++) {
            r = (r ^ h_[k]) * kMul;
            r ^= r >> 29;
        }
        return r;
    }
};

// Closes f when still set; a file being written (unlink_path) is then also
// removed, so a failed spt_scene_save leaves no partial cache behind.
struct FileCloser {
    FILE* f;
    const char* unlink_path = nullptr;
    ~FileCloser() {
        if (!f) return;
        std::fclose(f);
        if (unlink_path) std::remove(unlink_path);
    }
};

// The header checks of spt_scene_load / spt_scene_cache_info (no device).
spt_status cache_read_header(FILE* f, const char* path, const char* what, CacheHeader& h) {
    if (std::fseek(f, 0, SEEK_END) != 0) return fail(SPT_ERR_IO, "%s: cannot seek %s", what, path);
    const long long fsize = (long long)std::ftell(f);
    std::rewind(f);
    std::memset(&h, 0, sizeof(h));
    if (fsize < (long long)sizeof(h) || std::fread(&h, sizeof(h), 1, f) != 1)
        return fail(SPT_ERR_INVALID, "%s: %s is not a scene cache (shorter than its header)", what, path);
    if (std::memcmp(h.magic, kCacheMagic, 8) != 0)
        return fail(SPT_ERR_INVALID, "%s: %s is not a scene cache (bad magic)", what, path);
    if (h.version != kCacheVersion || h.header_bytes != sizeof(CacheHeader) || h.config_bytes != sizeof(spt_config) ||
        h.stats_bytes != sizeof(spt_scene_stats))
        return fail(SPT_ERR_INVALID, "%s: %s has version %u / header %u B (this library reads version %u / %zu B)",
                    what, path, h.version, h.header_bytes, kCacheVersion, sizeof(CacheHeader));
    const uint32_t width = h.stats.bvh_width;
    if ((width != 2 && width != 6 && width != 8) || h.node6 != (width == 6 ? 1u : 0u))
        return fail(SPT_ERR_INVALID, "%s: %s: BVH width %u / node6 %u", what, path, width, h.node6);
    if (h.tri_quads != (uint32_t)kTriQuads || h.node_quads != node_quads_of(width, h.node6) ||
        (h.group_shift != 0 && h.group_shift != 3))
        return fail(SPT_ERR_INVALID, "%s: %s was written with another layout (triangle %u / node %u quads, group "
                    "shift %u; this library: %u / %u)", what, path, h.tri_quads, h.node_quads, h.group_shift,
                    (uint32_t)kTriQuads, node_quads_of(width, h.node6));
    if (h.ntri >= kMaxTriangles || h.ntri != h.stats.ntri || h.nmat == 0 || h.nsph > 256 || h.stack_depth == 0)
        return fail(SPT_ERR_INVALID, "%s: %s: bad counts (ntri %llu, nmat %u, spheres %u, stack %u)", what, path,
                    (unsigned long long)h.ntri, h.nmat, h.nsph, h.stack_depth);
    const uint64_t n = h.ntri;
    const uint64_t want[kNumSecs] = {
        h.bytes[kSecNodes], n * kTriQuads * 16, n * 48, h.bytes[kSecTc] ? n * 24 : 0, n * 4, (uint64_t)h.nmat * 12,
        (uint64_t)h.nemit * 12, (uint64_t)h.nsph * 16, (uint64_t)h.nsph * 4, (uint64_t)h.nkind * 4,
        (uint64_t)h.ntexmat * 8, h.bytes[kSecTexels], h.bytes[kSecExtra]};
    for (uint32_t s = 0; s < kNumSecs; s++)
        if (h.bytes[s] != want[s])
            return fail(SPT_ERR_INVALID, "%s: %s: section %s holds %llu bytes, expected %llu", what, path, kSecName[s],
                        (unsigned long long)h.bytes[s], (unsigned long long)want[s]);
    if (h.bytes[kSecNodes] % ((uint64_t)h.node_quads * 16) != 0 || (n > 0 && h.bytes[kSecNodes] == 0) ||
        h.bytes[kSecTexels] % 16 != 0)
        return fail(SPT_ERR_INVALID, "%s: %s: node / texel sections are not whole records", what, path);
    long long total = (long long)sizeof(CacheHeader);
    for (uint32_t s = 0; s < kNumSecs; s++) total += (long long)h.bytes[s];
    if (total != fsize)
        return fail(SPT_ERR_INVALID, "%s: %s holds %lld bytes, its header describes %lld (truncated?)", what, path,
                    fsize, total);
    return SPT_OK;
}

// Read section s (h.bytes[s] bytes at the file position) into dst, checking its sum.
spt_status cache_read_section(FILE* f, const char* path, const char* what, const CacheHeader& h, uint32_t s,
                              std::vector<uint8_t>& dst) {
    dst.resize(h.bytes[s]);
    CacheHash hash;
    for (size_t off = 0; off < dst.size(); off += kCacheChunk) {
        const size_t len = std::min(kCacheChunk, dst.size() - off);
        if (std::fread(dst.data() + off, 1, len, f) != len)
            return fail(SPT_ERR_IO, "%s: short read of section %s of %s", what, kSecName[s], path);
        hash.update(dst.data() + off, len);
    }
    if (hash.digest() != h.sum[s])
        return fail(SPT_ERR_INVALID, "%s: %s: checksum mismatch in section %s", what, path, kSecName[s]);
    return SPT_OK;
}

// Texture section checks: one (w, h) pair per material, texels = their sum.
spt_status cache_check_textures(const char* path, const char* what, const CacheHeader& h, const uint32_t* dims) {
    uint64_t texels = 0;
    for (uint32_t m = 0; m < h.ntexmat; m++) {
        const uint64_t wh = (uint64_t)dims[2 * m] * dims[2 * m + 1];
        if (wh > (1ull << 26)) return fail(SPT_ERR_INVALID, "%s: %s: texture %u is %llu texels", what, path, m,
                                           (unsigned long long)wh);
        texels += wh;
    }
    if (texels * 16 != h.bytes[kSecTexels])
        return fail(SPT_ERR_INVALID, "%s: %s: texture sizes describe %llu texels, the section holds %llu", what, path,
                    (unsigned long long)texels, (unsigned long long)(h.bytes[kSecTexels] / 16));
    return SPT_OK;
}

// Content checks of a loaded BVH before it reaches the device (the checksums
// only catch accidents): from the root, every reachable node index lies in the
// node section and is reached once (a tree: traversal ends), the tree fits
// the LDS stack the header declares, and every leaf's triangle slots lie in
// [0, ntri).  Unreachable slots (holes between packed child groups) are not read.
spt_status cache_check_nodes(const char* path, const char* what, const CacheHeader& h, const std::vector<uint8_t>& buf) {
    const uint64_t nt = h.ntri;
    if (nt == 0) return SPT_OK;
    const uint64_t nslots = buf.size() / ((uint64_t)h.node_quads * 16);
    const uint32_t* w = (const uint32_t*)buf.data();
    const uint64_t stride = (uint64_t)h.node_quads * 4;  // words per node slot
    std::vector<uint8_t> seen(nslots, 0);
    std::vector<std::pair<uint64_t, uint32_t>> todo{{0, 1}};  // (node, level; root = 1)
    seen[0] = 1;
    uint32_t depth = 0;
    const auto bad = [&](const char* why, uint64_t node) {
        return fail(SPT_ERR_INVALID, "%s: %s: BVH node %llu: %s", what, path, (unsigned long long)node, why);
    };
    while (!todo.empty()) {
        const uint64_t node = todo.back().first;
        const uint32_t level = todo.back().second;
        todo.pop_back();
        depth = std::max(depth, level);
        const uint32_t* n = w + node * stride;
        auto child = [&](uint64_t c) -> bool {
            if (c >= nslots || seen[c]) return false;
            seen[c] = 1;
            todo.push_back({c, level + 1});
            return true;
        };
        if (h.stats.bvh_width == 2) {  // bvh_build.h: codes in word 12, 13
            for (int k = 0; k < 2; k++) {
                const int32_t code = (int32_t)n[12 + k];
                if (code >= 0) {
                    if (!child((uint64_t)code)) return bad("inner child out of range or reached twice", node);
                } else {
                    const uint32_t leaf = ~(uint32_t)code;
                    if ((uint64_t)(leaf >> 3) + (leaf & 7u) + 1u > nt) return bad("leaf beyond the triangles", node);
                }
            }
            continue;
        }
        // wide nodes: meta bytes, child-group word, triangle base (bvh_build.h)
        uint8_t meta[8];
        uint32_t nmeta, group, tri_base;
        if (h.node6) {
            std::memcpy(meta, &n[4], 4);
            meta[4] = (uint8_t)n[5];
            meta[5] = (uint8_t)(n[5] >> 8);
            nmeta = 6;
            group = n[6] & 0x00ffffffu;
            tri_base = n[3];
        } else {
            std::memcpy(meta, &n[6], 8);
            nmeta = 8;
            group = n[4];
            tri_base = n[5];
        }
        for (uint32_t c = 0; c < nmeta; c++) {
            const uint32_t m = meta[c];
            if (!m) continue;
            if ((m & 0x18u) == 0x18u) {  // inner: 0b001_(24 + s)
                const uint64_t cn = ((uint64_t)group << h.group_shift) + ((m & 31u) - 24u);
                if (!child(cn)) return bad("inner child out of range or reached twice", node);
            } else {  // leaf: unary(count) << 5 | offset
                const uint32_t cnt = (uint32_t)__builtin_popcount(m >> 5);
                if ((uint64_t)tri_base + (m & 31u) + cnt > nt) return bad("leaf beyond the triangles", node);
            }
        }
    }
    // the traversal stacks: BVH2 one entry per level below the root, a wide
    // BVH depth - 1 entries (bvh8_stack_entries)
    const uint32_t need = h.stats.bvh_width == 2 ? depth : (depth > 1 ? depth - 1 : 1);
    if (need > h.stack_depth)
        return fail(SPT_ERR_INVALID, "%s: %s: the BVH is %u levels deep, its stack holds %u entries", what, path, depth,
                    h.stack_depth);
    return SPT_OK;
}

// Index arrays of a loaded scene: orig2slot maps into the slots, every slot's
// original id (float 15 of its record) lies in [0, ntri), material kinds are SPT_MAT_*.
spt_status cache_check_indices(const char* path, const char* what, const CacheHeader& h, uint32_t s,
                               const std::vector<uint8_t>& buf) {
    const uint64_t nt = h.ntri;
    if (s == kSecOrig2Slot) {
        const int32_t* o = (const int32_t*)buf.data();
        for (uint64_t i = 0; i < nt; i++)
            if (o[i] < 0 || (uint64_t)o[i] >= nt)
                return fail(SPT_ERR_INVALID, "%s: %s: orig2slot[%llu] = %d outside [0, %llu)", what, path,
                            (unsigned long long)i, o[i], (unsigned long long)nt);
    } else if (s == kSecTris) {
        const uint32_t* t = (const uint32_t*)buf.data();
        for (uint64_t i = 0; i < nt; i++)
            if (t[i * kTriFloats + kTriIdFloat] >= nt)
                return fail(SPT_ERR_INVALID, "%s: %s: triangle slot %llu has id %u", what, path, (unsigned long long)i,
                            t[i * kTriFloats + kTriIdFloat]);
    } else if (s == kSecKinds) {
        const uint32_t* k = (const uint32_t*)buf.data();
        for (uint32_t i = 0; i < h.nkind; i++)
            if (k[i] > SPT_MAT_GLASS)
                return fail(SPT_ERR_INVALID, "%s: %s: material %u has kind %u", what, path, i, k[i]);
    }
    return SPT_OK;
}

}  // namespace

spt_status spt_scene_save(spt_scene sc, const char* path, const void* extra, uint64_t extra_bytes) {
    static const char* what = "spt_scene_save";
    if (!sc || !path) return fail(SPT_ERR_INVALID, "%s: NULL argument", what);
    DeviceGuard dg(sc->device);
    if (extra_bytes && !extra) return fail(SPT_ERR_INVALID, "%s: extra is NULL with %llu bytes", what,
                                           (unsigned long long)extra_bytes);
    std::lock_guard<std::mutex> lk(sc->mu);
    CacheHeader h;
    std::memset(&h, 0, sizeof(h));
    std::memcpy(h.magic, kCacheMagic, 8);
    h.version = kCacheVersion;
    h.header_bytes = sizeof(CacheHeader);
    h.tri_quads = kTriQuads;
    h.node_quads = node_quads_of(sc->stats.bvh_width, sc->node6);
    h.node6 = sc->node6;
    h.group_shift = sc->group_shift;
    h.config_bytes = sizeof(spt_config);
    h.stats_bytes = sizeof(spt_scene_stats);
    h.stack_depth = sc->stack_depth;
    h.nmat = sc->nmat;
    h.nemit = sc->nemit;
    h.nsph = sc->nsph;
    h.nkind = sc->nkind;
    h.ntexmat = sc->ntex;
    h.ntri = sc->ntri;
    h.cfg = sc->cfg;
    h.stats = sc->stats;
    // textures: their host copies
    std::vector<uint32_t> dims(2 * (size_t)sc->ntex);
    std::vector<float4> texels;
    for (uint32_t m = 0; m < sc->ntex; m++) {
        dims[2 * m] = sc->tex_w[m];
        dims[2 * m + 1] = sc->tex_h[m];
        texels.insert(texels.end(), sc->tex_img[m].begin(), sc->tex_img[m].end());
    }
    struct Src { const void* dev; const void* host; uint64_t bytes; };
    const uint64_t n = sc->ntri;
    const Src src[kNumSecs] = {
        {sc->nodes8 ? (const void*)sc->nodes8 : (const void*)sc->nodes, nullptr, sc->node_bytes},
        {sc->tris, nullptr, n * kTriQuads * 16},
        {sc->snrm, nullptr, n * 48},
        {sc->tc, nullptr, sc->tc ? n * 24 : 0},
        {sc->orig2slot, nullptr, n * 4},
        {sc->albedo, nullptr, (uint64_t)sc->nmat * 12},
        {sc->emission, nullptr, (uint64_t)sc->nemit * 12},
        {sc->spheres, nullptr, (uint64_t)sc->nsph * 16},
        {sc->sph_mat, nullptr, (uint64_t)sc->nsph * 4},
        {sc->mat_kind, nullptr, (uint64_t)sc->nkind * 4},
        {nullptr, dims.data(), dims.size() * 4},
        {nullptr, texels.data(), texels.size() * 16},
        {nullptr, extra, extra_bytes}};
    for (uint32_t s = 0; s < kNumSecs; s++)
        if (src[s].bytes && !src[s].dev && !src[s].host)
            return fail(SPT_ERR_INVALID, "%s: the scene has no %s array", what, kSecName[s]);
    FILE* f = std::fopen(path, "wb");
    if (!f) return fail(SPT_ERR_IO, "%s: cannot open %s: %s", what, path, std::strerror(errno));
    FileCloser closer{f, path};
    if (std::fwrite(&h, sizeof(h), 1, f) != 1) return fail(SPT_ERR_IO, "%s: short write to %s", what, path);
    std::vector<uint8_t> stage;
    for (uint32_t s = 0; s < kNumSecs; s++) {
        CacheHash hash;
        for (uint64_t off = 0; off < src[s].bytes; off += kCacheChunk) {
            const size_t len = (size_t)std::min<uint64_t>(kCacheChunk, src[s].bytes - off);
            const uint8_t* p;
            if (src[s].dev) {
                stage.resize(len);
                HIP_TRY(hipMemcpy(stage.data(), (const uint8_t*)src[s].dev + off, len, hipMemcpyDeviceToHost));
                p = stage.data();
            } else {
                p = (const uint8_t*)src[s].host + off;
            }
            hash.update(p, len);
            if (std::fwrite(p, 1, len, f) != len) return fail(SPT_ERR_IO, "%s: short write to %s", what, path);
        }
        h.bytes[s] = src[s].bytes;
        h.sum[s] = hash.digest();
    }
    std::rewind(f);
    if (std::fwrite(&h, sizeof(h), 1, f) != 1) return fail(SPT_ERR_IO, "%s: short write to %s", what, path);
    closer.f = nullptr;
    if (std::fclose(f) == 0) return SPT_OK;
    std::remove(path);
    return fail(SPT_ERR_IO, "%s: closing %s failed", what, path);
}

spt_status spt_scene_cache_info(const char* path, spt_scene_stats* stats, spt_config* cfg, uint64_t* extra_bytes) {
    static const char* what = "spt_scene_cache_info";
    if (!path) return fail(SPT_ERR_INVALID, "%s: NULL path", what);
    FILE* f = std::fopen(path, "rb");
    if (!f) return fail(SPT_ERR_IO, "%s: cannot open %s: %s", what, path, std::strerror(errno));
    FileCloser closer{f};
    CacheHeader h;
    spt_status st = cache_read_header(f, path, what, h);
    if (st) return st;
    std::vector<uint8_t> buf;
    for (uint32_t s = 0; s < kNumSecs; s++) {
        if (s == kSecTexDims) {  // small (8 B per material): read whole and check against the texel section
            if ((st = cache_read_section(f, path, what, h, s, buf))) return st;
            if ((st = cache_check_textures(path, what, h, (const uint32_t*)buf.data()))) return st;
            continue;
        }
        // sums only: stream through one chunk at a time
        CacheHash hash;
        for (uint64_t off = 0; off < h.bytes[s]; off += kCacheChunk) {
            const size_t len = (size_t)std::min<uint64_t>(kCacheChunk, h.bytes[s] - off);
            buf.resize(len);
            if (std::fread(buf.data(), 1, len, f) != len)
                return fail(SPT_ERR_IO, "%s: short read of section %s of %s", what, kSecName[s], path);
            hash.update(buf.data(), len);
        }
        if (hash.digest() != h.sum[s])
            return fail(SPT_ERR_INVALID, "%s: %s: checksum mismatch in section %s", what, path, kSecName[s]);
    }
    if (stats) *stats = h.stats;
    if (cfg) *cfg = h.cfg;
    if (extra_bytes) *extra_bytes = h.bytes[kSecExtra];
    return SPT_OK;
}

spt_status spt_scene_load(const char* path, spt_scene* out, void* extra, uint64_t extra_cap, uint64_t* extra_bytes) {
    static const char* what = "spt_scene_load";
    if (!path || !out) return fail(SPT_ERR_INVALID, "%s: NULL argument", what);
    *out = nullptr;
    if (extra_cap && !extra) return fail(SPT_ERR_INVALID, "%s: extra is NULL with capacity %llu", what,
                                         (unsigned long long)extra_cap);
    const double t0 = now_ms();
    FILE* f = std::fopen(path, "rb");
    if (!f) return fail(SPT_ERR_IO, "%s: cannot open %s: %s", what, path, std::strerror(errno));
    FileCloser closer{f};
    CacheHeader h;
    spt_status st = cache_read_header(f, path, what, h);
    if (!st) st = check_config(h.cfg);
    if (st) return st;
    if ((st = ensure_device())) return st;
    spt_scene_t* sc = new spt_scene_t();
    auto bail = [&](spt_status e) {
        sc->release();
        delete sc;
        return e;
    };
    sc->cfg = h.cfg;
    (void)hipGetDevice(&sc->device);
    sc->ntri = h.ntri;
    sc->node6 = h.node6;
    sc->group_shift = h.group_shift;
    sc->stack_depth = h.stack_depth;
    std::vector<uint8_t> buf;
    for (uint32_t s = 0; s < kNumSecs; s++) {
        if ((st = cache_read_section(f, path, what, h, s, buf))) return bail(st);
        if ((st = s == kSecNodes ? cache_check_nodes(path, what, h, buf) : cache_check_indices(path, what, h, s, buf)))
            return bail(st);
        switch (s) {
            case kSecNodes:
                st = h.stats.bvh_width == 2 ? upload(&sc->nodes, buf.data(), buf.size())
                                            : upload(&sc->nodes8, buf.data(), buf.size());
                sc->node_bytes = buf.size();
                break;
            case kSecTris: st = upload(&sc->tris, buf.data(), buf.size()); break;
            case kSecSnrm: st = upload(&sc->snrm, buf.data(), buf.size()); break;
            case kSecTc: st = upload(&sc->tc, buf.data(), buf.size()); break;
            case kSecOrig2Slot: st = upload(&sc->orig2slot, buf.data(), buf.size()); break;
            case kSecAlbedo: {
                st = upload(&sc->albedo, buf.data(), buf.size());
                const float* a = (const float*)buf.data();
                bool unit = true;
                for (size_t i = 0; i < buf.size() / 4; i++) unit = unit && a[i] == 1.0f;
                sc->albedo_unit = unit;
                sc->nmat = h.nmat;
                break;
            }
            case kSecEmission: st = upload(&sc->emission, buf.data(), buf.size()); sc->nemit = h.nemit; break;
            case kSecSpheres: st = upload(&sc->spheres, buf.data(), buf.size()); break;
            case kSecSphMat: st = upload(&sc->sph_mat, buf.data(), buf.size()); sc->nsph = h.nsph; break;
            case kSecKinds: st = upload(&sc->mat_kind, buf.data(), buf.size()); sc->nkind = h.nkind; break;
            case kSecTexDims: {
                const uint32_t* dims = (const uint32_t*)buf.data();
                if ((st = cache_check_textures(path, what, h, dims))) break;
                sc->tex_img.resize(h.ntexmat);
                sc->tex_w.resize(h.ntexmat);
                sc->tex_h.resize(h.ntexmat);
                for (uint32_t m = 0; m < h.ntexmat; m++) {
                    sc->tex_w[m] = dims[2 * m];
                    sc->tex_h[m] = dims[2 * m + 1];
                }
                break;
            }
            case kSecTexels: {
                const float4* t = (const float4*)buf.data();
                for (uint32_t m = 0; m < h.ntexmat; m++) {
                    const size_t wh = (size_t)sc->tex_w[m] * sc->tex_h[m];
                    sc->tex_img[m].assign(t, t + wh);
                    t += wh;
                }
                st = upload_textures(sc);
                break;
            }
            case kSecExtra:
                if (extra && extra_cap) std::memcpy(extra, buf.data(), (size_t)std::min<uint64_t>(extra_cap, buf.size()));
                if (extra_bytes) *extra_bytes = buf.size();
                break;
        }
        if (st) return bail(st);
    }
    sc->stats = h.stats;
    sc->stats.build_ms = now_ms() - t0;
    *out = sc;
    return SPT_OK;
}

spt_status spt_intersect(spt_scene sc, const spt_rays* rays, const uint8_t* mask, uint32_t mask_size,
                         const spt_hits* hits, uint32_t n, int32_t do_closest, void* stream) {
    if (!sc || !rays || !hits) return fail(SPT_ERR_INVALID, "spt_intersect: NULL argument");
    if (n == 0) return SPT_OK;
    if (!rays->ox || !rays->oy || !rays->oz || !rays->dx || !rays->dy || !rays->dz)
        return fail(SPT_ERR_INVALID, "spt_intersect: NULL ray plane");
    if (!hits->tri_id || !hits->t || !hits->u || !hits->v) return fail(SPT_ERR_INVALID, "spt_intersect: NULL hit plane");
    if (mask && mask_size != 1 && mask_size != n)
        return fail(SPT_ERR_INVALID, "spt_intersect: mask_size %u must be 1 or n=%u", mask_size, n);
    IsectPublicArgs a;
    a.ox = rays->ox; a.oy = rays->oy; a.oz = rays->oz;
    a.dx = rays->dx; a.dy = rays->dy; a.dz = rays->dz;
    a.tmin = rays->tmin; a.tmax = rays->tmax;
    a.mask = mask; a.mask_size = mask_size;
    a.tri_id = hits->tri_id; a.t = hits->t; a.u = hits->u; a.v = hits->v;
    a.n = n;
    a.closest = do_closest;
    // a consistent snapshot of the device arrays and knobs, launched and
    // recorded under the mutex: a scene mutator waits for this launch before it
    // frees an array the snapshot holds (quiesce_scene)
    DeviceGuard dg(sc->device);
    std::lock_guard<std::mutex> lock(sc->mu);
    a.sc = sc->dev();
    a.refill_idle = sc->cfg.public_refill_idle;
    a.persistent = sc->cfg.public_persistent;
    HIP_TRY(launch_isect_public(a, (hipStream_t)stream));
    return record_public_use(sc, (hipStream_t)stream);
}

spt_status spt_hit_info_compute(spt_scene sc, const spt_rays* rays, const spt_hits* hits, const uint8_t* mask,
                                uint32_t mask_size, uint32_t n, const spt_hit_info* out, void* stream) {
    if (!sc || !rays || !hits || !out) return fail(SPT_ERR_INVALID, "spt_hit_info_compute: NULL argument");
    if (n == 0) return SPT_OK;
    if (!hits->tri_id || !hits->t || !hits->u || !hits->v)
        return fail(SPT_ERR_INVALID, "spt_hit_info_compute: NULL hit plane");
    // the rays are read for the position (o + t d), and on a scene with
    // spheres for their normals too (the normal of a sphere hit is (p - c) / r)
    const bool no_rays = !rays->ox || !rays->oy || !rays->oz || !rays->dx || !rays->dy || !rays->dz;
    if ((out->px || out->py || out->pz) && no_rays)
        return fail(SPT_ERR_INVALID, "spt_hit_info_compute: NULL ray plane (needed for the position)");
    if (no_rays && sc->nsph > 0 && (out->gnx || out->gny || out->gnz || out->snx || out->sny || out->snz))
        return fail(SPT_ERR_INVALID, "spt_hit_info_compute: NULL ray plane (a sphere hit's normal needs the hit point)");
    if (mask && mask_size != 1 && mask_size != n)
        return fail(SPT_ERR_INVALID, "spt_hit_info_compute: mask_size %u must be 1 or n=%u", mask_size, n);
    if (sc->ntri == 0 && sc->nsph == 0) return SPT_OK;
    HitInfoArgs a;
    DeviceGuard dg(sc->device);
    std::lock_guard<std::mutex> lock(sc->mu);  // as spt_intersect: launched and recorded under the mutex
    a.sc = sc->dev();
    a.ox = rays->ox; a.oy = rays->oy; a.oz = rays->oz;
    a.dx = rays->dx; a.dy = rays->dy; a.dz = rays->dz;
    a.tri_id = hits->tri_id; a.t = hits->t; a.u = hits->u; a.v = hits->v;
    a.mask = mask; a.mask_size = mask_size; a.n = n;
    a.px = out->px; a.py = out->py; a.pz = out->pz;
    a.gnx = out->gnx; a.gny = out->gny; a.gnz = out->gnz;
    a.snx = out->snx; a.sny = out->sny; a.snz = out->snz;
    a.tcu = out->tcu; a.tcv = out->tcv;
    a.mat_id = out->mat_id;
    a.ntri = sc->ntri;
    HIP_TRY(launch_hit_info(a, (hipStream_t)stream));
    return record_public_use(sc, (hipStream_t)stream);
}

spt_status spt_render_async(spt_scene sc, const spt_render_params* pp, float* film_dev, void* caller_,
                            uint64_t* ticket_out) {
    const double wall0 = now_ms();
    if (!sc || !pp || !ticket_out) return fail(SPT_ERR_INVALID, "spt_render: NULL argument");
    const spt_render_params& p = *pp;
    if (p.width == 0 || p.height == 0 || p.spp == 0 || p.max_depth == 0)
        return fail(SPT_ERR_INVALID, "spt_render: width/height/spp/max_depth must be > 0");
    if (p.max_depth > kMaxDepthCasts) return fail(SPT_ERR_LIMIT, "spt_render: max_depth %u > %u", p.max_depth, kMaxDepthCasts);
    if (p.spp >= (1u << 24)) return fail(SPT_ERR_LIMIT, "spt_render: spp must be < 2^24");
    if ((uint64_t)p.width * p.height >= (1ull << 31)) return fail(SPT_ERR_LIMIT, "spt_render: image too large");
    if (p.tile_count == 0 || p.rows_per_group == 0 || p.tile_index >= p.tile_count)
        return fail(SPT_ERR_INVALID, "spt_render: bad tile (%u of %u, %u rows/group)", p.tile_index, p.tile_count,
                    p.rows_per_group);
    if (p.rng_order > 1) return fail(SPT_ERR_INVALID, "spt_render: rng_order must be 0 or 1");
    // The caller's stream orders the render with the caller's work (it starts
    // after what was queued there, and what is queued there next waits for
    // it); the render itself runs on its working set's own streams.
    const hipStream_t caller = (hipStream_t)caller_;
    const uint32_t rows = spt_tile_rows(p.height, p.tile_index, p.tile_count, p.rows_per_group, nullptr, 0);
    const uint64_t P = (uint64_t)rows * p.width;
    if (P != 0 && !film_dev) return fail(SPT_ERR_INVALID, "spt_render: NULL film");
    DeviceGuard dg(sc->device);
    std::lock_guard<std::mutex> lock(sc->mu);  // the scene's one workspace
    RenderSlot* slot = nullptr;
    spt_status st = render_slot(sc->ws, &slot);
    if (st) return st;
    spt_render_stats& rs = slot->rs;
    rs.tile_rows = rows;
    slot->wall0 = wall0;
    if (P == 0) {  // an empty tile: nothing to render, film untouched
        slot->ticket = sc->ws.next_ticket++;
        slot->pending = true;
        *ticket_out = slot->ticket;
        return SPT_OK;
    }
    const spt_config& cfg = sc->cfg;

    // Wavefront capacity.  Each isect launch ends in a tail where its last rays
    // finish while most lanes idle, and every iteration pays launch gaps and a
    // shade + refill during which its stream's share of the chip is not
    // tracing; 32M paths in flight (~5 GB of queues: HBM is 288 GB) amortise
    // both.  Config 1, Mpaths/s: 8M 3235, 12M 3470, 16M 3463, 24M 3755,
    // 32M 3715, 48M 3722; configs 2 / 3 / 4: 8M 1712 / 3824 / 851 against
    // 32M 1790 / 4080 / 860.  Default: spt_config.wavefront_paths = 32M.
    // (a render whose working set could not be allocated comes back here with
    // half its paths in flight as the limit: fit_limit)
    uint64_t fit_limit = UINT64_MAX;
retry_fit:
    uint64_t C = p.wavefront_paths ? p.wavefront_paths : cfg.wavefront_paths;

    // Pipeline: the wavefront (isect / shade / refill over path queues, the
    // north-star design) or the fused persistent kernel (bit-identical).  The
    // flags choose; else spt_config.pipeline; else (AUTO) by job size: a job of at most
    // two wavefronts is mostly per-cast launch tails on the wavefront (queues
    // shrink cast by cast with no work left to refill them), where the fused
    // kernel's single tail wins — e.g. one rank's 1/8 of the headline image:
    // fused 2308 vs wavefront 1982 Mpaths/s; whole image: 2353 vs 2825.
    // Traversal counters exist in the wavefront isect kernel only.
    const bool trav_stats = (p.flags & SPT_FLAG_TRAVERSAL_STATS) != 0;
    // the job-size rule: the fused kernel up to fused_max_paths = 2^20 paths
    // (fewer than two chip fills of lanes, config 0), the wavefront above: with
    // the drain and the fit rule it carries every tile of config 1 at 1.00-1.05x
    // the fused kernel; an explicit wavefront size moves the rule
    // with it
    const uint64_t fused_max = p.wavefront_paths ? p.wavefront_paths : cfg.fused_max_paths;
    bool fused = cfg.pipeline == SPT_PIPELINE_AUTO ? P * p.spp <= fused_max : cfg.pipeline == SPT_PIPELINE_FUSED;
    if (p.flags & SPT_FLAG_FUSED) fused = true;
    if ((p.flags & SPT_FLAG_WAVEFRONT) || trav_stats) fused = false;
    // Work order (spt_config.work_order).  AUTO, measured (DESIGN.md §4,
    // profiles/r02_workorder): pixel-major for a scene larger than the
    // Infinity Cache (config 4: +3.8 %; the paths in flight then cover a band
    // of the tile, whose scene working set is smaller); in the fused kernel
    // for tiles of >= 16M paths (config 1 tiles of N = 1 / 2 / 4: +6 / +3 /
    // +2.8 %, N = 8: -1.5 %); in the wavefront for a scene that outgrows an
    // XCD's L2 on a tile of <= 4M pixels, with 24M paths in flight unless
    // set (config 1 +5.5 %); sample-major otherwise (config 3's 16.7M-pixel
    // tile -2.1 %, smallpt's cache-resident scene -4.6 %).
    // A job that fits in flight (spt_config.fit_paths): every path starts in
    // the first refill on fit_streams sub-wavefronts, so its last work item
    // starts at once and the drain finishes it drain_casts casts later.  The
    // per-cast launches then run only while the whole job is in flight, and
    // a render is a handful of launches, which two renders queued on two
    // streams overlap without sub-wavefront streams of their own (DESIGN.md §6:
    // stable at the box's four hardware queues, where four sub-wavefront
    // streams per working set could share a queue with the other set's).
    // A larger job runs as sample chunks that each fit (spt_config.fit_chunks:
    // config 3 +8 %, config 2 +0.9 %, profiles/r05_exp/fit_chunks/).
    // (an explicit paths-in-flight count, in the params or the config, wins)
    // What a path carries (spt_internal.h PathMode): the reference's case
    // (every albedo 1, no emitters) needs only the ray and an escaped flag.
    const bool unit = sc->albedo_unit && sc->ntex == 0 && sc->nsph == 0 && sc->nkind == 0;
    const int mode = sc->emission ? kModeEmit : (unit ? kModeUnit : kModeAlbedo);
    const uint64_t film_unit = mode_film_bytes(mode);
    // A fitting job's queues, hit records and film chunk must fit in device
    // memory (spt_config.fit_bytes; 0: the free memory plus what this caller's
    // set holds, less 1/16 — processes or scenes sharing the GPU): fit_paths
    // shrinks to what fits, into more sample chunks, and below one chunk of
    // the tile's pixels the job keeps the per-cast wavefront.  Asked only when
    // the set must grow; an allocation that fails all the same (another
    // process took the memory in between) halves the fit and tries again.
    // (the set's streams, below: a caller's null stream gets plain streams and
    // a fitting job one sub-wavefront on them)
    const bool null_caller = caller == nullptr || caller == hipStreamLegacy || caller == hipStreamPerThread;
    const bool own_queues = cfg.sub_queues != 0 && !null_caller;
    uint64_t fit_paths = std::min<uint64_t>(cfg.fit_paths, fit_limit);
    uint64_t mem_paths = fit_limit;  // paths in flight the memory allows (queues + film chunk)
    if (fit_paths && !fused) {
        const uint64_t per_path = 2ull * 16 * mode_planes(mode) + kHitBytes + film_unit;
        const uint64_t want = std::min<uint64_t>(fit_paths, P * p.spp) * per_path;
        // what this render may reuse of the set it will get: the queues and hit
        // records of the sub-wavefronts a fitting job runs on (as allocated,
        // plane padding included) and the film chunk; a sub-wavefront beyond
        // those keeps its buffers and is not counted
        uint64_t held = 0;
        if (const WorkSet* hs = sc->ws.bound_set(caller)) {
            const int kf = own_queues ? (int)cfg.fit_streams : 1;
            for (int k = 0; k < kf && k < kMaxStreams; k++) {
                const Sub& b = hs->sub[k];
                held += 2ull * 16 * b.planes * queue_stride(b.cap, b.pad) + (uint64_t)kHitBytes * b.cap;
            }
            held += hs->film_cap;
        }
        uint64_t room = cfg.fit_bytes;
        if (!room && want > held) {
            size_t fr = 0, tot = 0;
            if (hipMemGetInfo(&fr, &tot) == hipSuccess)
                room = held + fr - fr / 16;
            else
                (void)hipGetLastError();
        }
        if (room && want > room) mem_paths = fit_paths = std::max<uint64_t>(1, room / per_path);
    }
    rs.fit_paths = fit_paths;
    const bool fit_ok = !fused && !p.wavefront_paths && cfg.wavefront_paths == kDefaultWavefrontPaths && fit_paths &&
                        cfg.drain_q8;
    uint32_t fit_chunk = 0;  // samples per chunk of a job run as fitting chunks
    if (fit_ok && P * p.spp > fit_paths && cfg.fit_chunks && P <= fit_paths)
        fit_chunk = (uint32_t)std::min<uint64_t>(p.spp, fit_paths / P);
    const bool fit = fit_ok && (P * p.spp <= fit_paths || fit_chunk != 0);
    const uint64_t scene_bytes = sc->stats.device_bytes;
    // (a fitting job of any tile size: pixel-major over scenes beyond an
    // XCD's L2 — config 3's 16.7M-pixel chunks +8 % with it, its per-cast
    // wavefront -2.1 %; smallpt's cache-resident scene -4 % either way)
    const bool wave_pm = !fused && scene_bytes >= kPixelMajorMinWaveSceneBytes && (P <= kPixelMajorMaxWaveTilePx || fit);
    const uint32_t pixel_major =
        cfg.work_order == SPT_WORK_PIXEL_MAJOR ||
        (cfg.work_order == SPT_WORK_AUTO && (scene_bytes >= kPixelMajorMinSceneBytes ||
                                             (fused && P * p.spp >= kPixelMajorMinFusedPaths) || wave_pm));
    // Queue caching (spt_config.queue_cache).  AUTO: non-temporal path-queue
    // and hit accesses for a scene beyond the Infinity Cache, so the caches
    // keep BVH nodes and triangles (config 4 +1.7 %); cached otherwise, where
    // the next kernel still finds the queue's lines (config 2 -3.7 %, config 3
    // -0.7 % streamed; config 1 within noise: profiles/r04_exp2/).
    const uint32_t queue_nt =
        cfg.queue_cache == SPT_QUEUE_CACHE_STREAM ||
        (cfg.queue_cache == SPT_QUEUE_CACHE_AUTO && scene_bytes >= kPixelMajorMinSceneBytes);
    // The drain's refill threshold (spt_config.drain_refill_idle).  AUTO: a
    // wave refills and shades once per batch of free lanes, at a cost that
    // does not depend on how many lanes take part, while a trace step costs
    // in proportion to how long its busiest lane traverses.  With analytic
    // spheres the shade tests them and runs smallpt's mirror / glass, so a
    // pass costs several trace steps and batching more lanes pays (config 2:
    // 56 +20 % over 24); a scene beyond the Infinity Cache (config 4) +3 % at
    // 40; triangle scenes 24 (configs 1, 3, and the mitsuba mesh from 200 to
    // 231k triangles: 56 costs 13-17 %), though closed ones (the tessellated
    // Cornell spheres) gain 1-3 % at 40 (profiles/r06_exp/refill_idle/).
    const uint32_t drain_idle = cfg.drain_refill_idle ? cfg.drain_refill_idle
                                : sc->nsph > 0 ? kDrainIdleSpheres
                                : queue_nt ? kDrainIdleStream : kDrainIdleCached;
    if (cfg.work_order == SPT_WORK_AUTO && wave_pm && !p.wavefront_paths && cfg.wavefront_paths == kDefaultWavefrontPaths)
        C = kPixelMajorWavefrontPaths;
    if (fit) C = fit_chunk ? (uint64_t)fit_chunk * P : P * p.spp;
    C = std::max<uint64_t>(1, std::min<uint64_t>(std::min<uint64_t>(C, mem_paths), P * p.spp));
    if (C >= (1ull << 31)) return fail(SPT_ERR_LIMIT, "spt_render: wavefront of %llu paths exceeds 2^31",
                                       (unsigned long long)C);
    // The wavefront is split into K sub-wavefronts on their own streams, so one
    // sub-wavefront's launch tail overlaps the others' work.
    // Measured on the headline config: 1 stream 1982, 2: 2649, 3: 2769, 4: 2791 Mpaths/s
    // (4 = the box's hardware queues per process, GPU_MAX_HW_QUEUES).
    // The set's streams get hardware queues of their own (CU-masked streams,
    // spt_config.sub_queues) unless the caller renders on the legacy null
    // stream: CU-masked streams are blocking, and every null-stream operation
    // (the event this render waits for, the one the caller waits on) would
    // wait for them — the other working set's render included — so renders
    // queued there would not overlap.  Such a set uses plain non-blocking
    // streams, which share the process's GPU_MAX_HW_QUEUES, and a fitting job
    // then runs on one sub-wavefront: more would share queues with the other
    // set's and serialise behind them.
    int K = fused ? 1 : fit ? (own_queues ? (int)cfg.fit_streams : 1) : (int)cfg.streams;
    if (fused) C = 64;  // no queues
    if ((uint64_t)K > C) K = (int)C;
    const uint64_t Ck = (C + K - 1) / K;
    // Per-sample contribution film [chunk][P] bytes (unit) or [chunk][3][P]
    // floats, at most film_budget_bytes (4 GiB) per chunk; chunks carry the
    // running sum in acc.  (A chunk's work items are counted in 32 bits: at
    // most 2^31 per chunk.)
    const uint64_t budget = cfg.film_budget_bytes;
    uint32_t chunk = (uint32_t)std::max<uint64_t>(
        1, std::min<uint64_t>(std::min<uint64_t>(p.spp, budget / (film_unit * P)), 0x7fffffffull / P));
    if (fit_chunk) chunk = std::min(chunk, fit_chunk);  // each chunk fits in flight
    if (mem_paths != UINT64_MAX) chunk = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(chunk, mem_paths / P));
    rs.paths_in_flight = (uint32_t)C;
    WorkSet& ws = sc->ws.pick_set(caller);
    ws.last_ticket = sc->ws.next_ticket;
    st = ensure_workspace(ws, K, Ck, cfg.plane_pad, mode_planes(mode), (size_t)chunk * film_unit * P, 3 * P,
                          own_queues, !fused && cfg.drain_q8 != 0 && cfg.drain_sort != 0 && sc->nodes8 != nullptr);
    if (st == SPT_ERR_OOM && !fused && C > kMinRetryPaths) {
        // the fit, or below it the per-cast wavefront and its film chunk, halved;
        // first the queues, hit records and film chunk this attempt allocated
        // (ensure_workspace only grows them) are freed, so the halved attempt
        // holds half, not more
        (void)hipGetLastError();
        if ((st = release_queues(ws))) return st;
        rs.fit_retries++;
        fit_limit = C / 2;
        goto retry_fit;
    }
    if (st) return st;
    // the set's stream 0 (its own): the render's first and last launches, the
    // fork and join of the other sub-wavefronts
    const hipStream_t stream = ws.sub[0].stream;
    HIP_TRY(hipEventRecord(ws.call_ev, caller));
    HIP_TRY(hipStreamWaitEvent(stream, ws.call_ev, 0));
    JumpTable* jtab = nullptr;
    if ((st = ensure_jumps(sc->ws, stream, p.spp, p.max_depth, p.rng_initstate, &jtab))) return st;
    const PcgJump* jumps = jtab->dev;
    const int set_idx = (int)(&ws - sc->ws.sets);
    // HIP events around the isect launches (the roofline kernel); every other
    // launch only with SPT_FLAG_TIMING_ALL (each event pair costs host time).
    const bool timing = (p.flags & SPT_FLAG_TIMING) != 0;
    const bool timing_all = timing && (p.flags & SPT_FLAG_TIMING_ALL) != 0;


    const Camera cam = make_camera(p);
    float* sfilm = (float*)ws.film;
    uint8_t* sflag = (uint8_t*)ws.film;
    float* acc = ws.acc;
    // film slots follow the work order (film_slot)
    const uint32_t film_order = pixel_major;
    const auto resolve = [&](uint32_t s0, uint32_t ns) {
        return mode == kModeUnit
                   ? launch_resolve_flags(sflag, acc, film_dev, (uint32_t)P, ns, s0 == 0, s0 + ns >= p.spp, p.spp,
                                          p.env[0], p.env[1], p.env[2], film_order, &slot->dev->unwritten, stream)
                   : launch_resolve(sfilm, acc, film_dev, (uint32_t)P, ns, s0 == 0, s0 + ns >= p.spp, p.spp,
                                    film_order, &slot->dev->unwritten, stream);
    };
    // every slot of a chunk starts as the sentinel (kFlagSentinel / kFilmSentinel
    // bytes), so the resolve counts slots no path wrote (spt_render_stats)
    const auto clear_film = [&](uint32_t ns) {
        return hipMemsetAsync(ws.film, 0xff, (size_t)ns * film_unit * P, stream);
    };
    hipStream_t strm[kMaxStreams];
    for (int k = 0; k < K; k++) strm[k] = ws.sub[k].stream;
    // the set's previous render (another stream, perhaps) must be done with it
    if (ws.used) HIP_TRY(hipStreamWaitEvent(stream, ws.free_ev, 0));
    // From here on work is queued on the set's streams.  Any early return
    // (a failed launch, a queue that did not drain) still joins the
    // sub-wavefront streams into `stream` and records free_ev, so the next
    // render that picks this set waits for whatever this one left running.
    struct EnqueueGuard {
        WorkSet& ws;
        hipStream_t stream, caller;
        JumpTable& jt;
        int set = 0;
        int K = 1;
        bool armed = true;
        ~EnqueueGuard() {
            if (!armed) return;
            for (int k = 1; k < K; k++) {
                (void)hipEventRecord(ws.sub[k].join_ev, ws.sub[k].stream);
                (void)hipStreamWaitEvent(stream, ws.sub[k].join_ev, 0);
            }
            (void)hipEventRecord(ws.free_ev, stream);
            (void)hipEventRecord(jt.ev[set], stream);
            (void)hipStreamWaitEvent(caller, ws.free_ev, 0);
            jt.ev_used[set] = true;
            ws.used = true;
        }
    } guard{ws, stream, caller, *jtab, set_idx, K};
    HIP_TRY(hipMemsetAsync(slot->dev, 0, sizeof(Stats), stream));
    // time origin for the isect launch intervals (their union = isect busy time)
    slot->timing = timing;
    if (timing) {
        hipEvent_t origin_ev = nullptr;
        if ((st = get_event(*slot, 0, &origin_ev))) return st;
        if (!sc->ws.epoch) {
            HIP_TRY(hipEventCreate(&sc->ws.epoch));
            HIP_TRY(hipEventRecord(sc->ws.epoch, stream));
        }
        HIP_TRY(hipEventRecord(origin_ev, stream));
    }

    std::vector<std::pair<size_t, int>>& timed = slot->timed;
    size_t ev = 1;  // events[0] is the origin
    auto mark = [&](int kind, hipStream_t sk, auto&& launch) -> spt_status {
        hipEvent_t e0 = nullptr, e1 = nullptr;
        spt_status s2;
        const bool tm = (kind == 1 || kind == 4) ? timing : timing_all;  // isect and drain: the tracing kernels
        if (tm) {
            if ((s2 = get_event(*slot, ev, &e0)) || (s2 = get_event(*slot, ev + 1, &e1))) return s2;
            HIP_TRY(hipEventRecord(e0, sk));
        }
        HIP_TRY(launch());
        if (tm) {
            HIP_TRY(hipEventRecord(e1, sk));
            timed.push_back({ev, kind});
            ev += 2;
        }
        return SPT_OK;
    };

    // Per sub-wavefront kernel arguments (queues and counters differ).
    IsectQueueArgs ia[kMaxStreams];
    ShadeArgs sa[kMaxStreams];
    RefillArgs ra[kMaxStreams];
    FusedArgs da[kMaxStreams];   // the drain launches (launch_drain)
    uint32_t drain_T[kMaxStreams] = {};
    // the drain: not with traversal counters (isect kernel only) or camera
    // paths started inside the isect launches (an experiment)
    const bool drain_on = cfg.drain_q8 != 0 && !trav_stats && !kIsectCam;
    // spt_config.xcd_remap bit 2: XCD-aware work distribution in the lane loops (drain, fused)
    const bool lane_xcd = (cfg.xcd_remap & 4u) != 0;
    // spt_config.drain_sort: a forced drain takes its queue sorted (wide-BVH scenes)
    const bool drain_sort = drain_on && cfg.drain_sort != 0 && sc->nodes8 != nullptr;
    // spt_config.lockstep_first = 2: the lockstep first cast also makes its
    // camera rays and shades its hits in the same launch (camera_cast_kernel;
    // wide-BVH scenes): no queue round trip for the first cast
    const bool cam_cast = cfg.lockstep_first >= 2 && sc->nodes8 != nullptr;
    // = 3: its survivors compacted per XCD shard, the drain's pools per shard
    const bool cam_shards = cam_cast && cfg.lockstep_first >= 3;
    uint64_t drain_launches = 0;
    PathQueue q[kMaxStreams][2];
    for (int k = 0; k < K; k++) {
        Sub& b = ws.sub[k];
        q[k][0] = carve_queue(b.qa, queue_stride(b.cap, b.pad), mode_planes(mode));
        q[k][1] = carve_queue(b.qb, queue_stride(b.cap, b.pad), mode_planes(mode));
        IsectQueueArgs& I = ia[k];
        I.sc = sc->dev();
        I.hits = (float4*)b.hits;
        I.nt = queue_nt && !trav_stats;
        I.max_depth = p.max_depth;
        I.trav_stats = trav_stats ? slot->dev->trav : nullptr;
        I.next = &b.cnt->isect_next;
        // 24 idle lanes / a 1/2 static share: +1.5 % over 16 / 5/8 at the
        // 32M wavefront (tools/envsweep.sh, tools/envsweep_r01_v11.txt)
        I.refill_idle = cfg.isect_refill_idle;
        I.static_share_q8 = cfg.isect_static_share_q8;
        I.xcd_remap = cfg.xcd_remap & 1u;
        I.chunk = cfg.isect_chunk;
        // each stream's persistent grid covers 1/K of the chip (measured best)
        I.grid_q8 = cfg.isect_grid_q8 ? cfg.isect_grid_q8 : 256u / (uint32_t)K;
        ShadeArgs& S = sa[k];
        S.sc = sc->dev();
        S.hits = (const float4*)b.hits;
        S.sfilm = sfilm;
        S.sflag = sflag;
        S.sample_jump = jumps;
        S.cast_jump = jumps + p.spp;
        S.initstate = p.rng_initstate;
        S.P = (uint32_t)P; S.W = p.width; S.max_depth = p.max_depth;
        S.xcd_remap = (cfg.xcd_remap >> 1) & 1u;
        S.rr_start = p.rr_start_depth; S.rng_order = p.rng_order;
        S.tile_index = p.tile_index; S.tile_count = p.tile_count; S.rows_per_group = p.rows_per_group;
        S.work_order = pixel_major;
        S.nt = queue_nt;
        S.env_r = p.env[0]; S.env_g = p.env[1]; S.env_b = p.env[2];
        RefillArgs& R = ra[k];
        R.cam = cam;
        R.sample_jump = jumps;
        R.stats = slot->dev->stats;
        R.capacity = (uint32_t)b.cap; R.P = (uint32_t)P; R.W = p.width; R.rng_order = p.rng_order;
        R.tile_index = p.tile_index; R.tile_count = p.tile_count; R.rows_per_group = p.rows_per_group;
        R.pixel_block = cfg.pixel_block;
        R.work_order = pixel_major;
        R.nt = queue_nt;
        R.initstate = p.rng_initstate;
        R.mode = mode;
        R.isect_next = &b.cnt->isect_next;
        R.exhausted = &b.cnt->exhausted;
        R.xcd_next = lane_xcd ? &b.cnt->xcd_next[0][0] : nullptr;
        R.book_only = 0;
        R.surv_shards = nullptr;
        I.drain_below = 0;
        S.drain_below = 0;
        if (drain_on) {
            // a queue shorter than drain_q8/256 of this stream's isect lanes
            drain_T[k] = (uint32_t)std::min<uint64_t>(
                0xffffffffull, (uint64_t)isect_queue_lanes(I) * cfg.drain_q8 / 256u);
            FusedArgs& D = da[k];
            D = FusedArgs{};
            D.sc = sc->dev();
            D.cam = cam;
            D.sample_jump = jumps;
            D.cast_jump = jumps + p.spp;
            D.sfilm = sfilm;
            D.sflag = sflag;
            D.stats = slot->dev->stats;
            D.drained = &slot->dev->drained;
            D.drained_casts = &slot->dev->drained_casts;
            D.next = &b.cnt->isect_next;  // zeroed by the refill before; an isect that skips leaves it
            D.xcd_next = lane_xcd ? &b.cnt->xcd_next[0][0] : nullptr;  // zeroed by the refill before
            D.initstate = p.rng_initstate;
            D.P = (uint32_t)P; D.W = p.width; D.max_depth = p.max_depth;
            D.rr_start = p.rr_start_depth; D.rng_order = p.rng_order;
            D.tile_index = p.tile_index; D.tile_count = p.tile_count; D.rows_per_group = p.rows_per_group;
            D.refill_idle = drain_idle;
            D.static_share_q8 = cfg.fused_static_share_q8;
            D.chunk = cfg.isect_chunk;
            D.grid_q8 = cfg.drain_grid_q8 ? cfg.drain_grid_q8 : 256u / (uint32_t)K;
            D.env_r = p.env[0]; D.env_g = p.env[1]; D.env_b = p.env[2];
            D.nt = queue_nt;
            D.seg_count = nullptr;
        }
        S.shard_items = 0;
    }

    uint64_t iters = 0;
    if (fused) {
        FusedArgs F{};
        F.sc = sc->dev();
        F.cam = cam;
        F.sample_jump = jumps;
        F.cast_jump = jumps + p.spp;
        F.sfilm = sfilm;
        F.sflag = sflag;
        F.stats = slot->dev->stats;
        F.next = &ws.sub[0].cnt->isect_next;
        F.xcd_next = lane_xcd ? &ws.sub[0].cnt->xcd_next[0][0] : nullptr;
        F.initstate = p.rng_initstate;
        F.P = (uint32_t)P; F.W = p.width; F.max_depth = p.max_depth;
        F.rr_start = p.rr_start_depth; F.rng_order = p.rng_order;
        F.tile_index = p.tile_index; F.tile_count = p.tile_count; F.rows_per_group = p.rows_per_group;
        F.refill_idle = cfg.fused_refill_idle;
        // a small static share: the fused lanes' path lengths vary far more
        // than one cast's, so most work is taken dynamically (1/8 tile of
        // config 1: 32/256 3006, 0: 2938, 64: 2912, 160: 2558 Mpaths/s)
        F.static_share_q8 = cfg.fused_static_share_q8;
        F.chunk = cfg.isect_chunk;
        F.grid_q8 = cfg.fused_grid_q8;
        F.env_r = p.env[0]; F.env_g = p.env[1]; F.env_b = p.env[2];
        uint32_t lanes = 0;
        for (uint32_t s0 = 0; s0 < p.spp; s0 += chunk) {
            const uint32_t ns = std::min(chunk, p.spp - s0);
            F.work0 = (uint64_t)s0 * P;
            F.count = (uint32_t)((uint64_t)ns * P);  // <= 4 GiB / 12 B per chunk
            F.sample0 = s0;
            F.pm_ns = pixel_major ? ns : 0;
            HIP_TRY(clear_film(ns));
            HIP_TRY(hipMemsetAsync(F.next, 0, sizeof(uint32_t), stream));
            if (F.xcd_next) HIP_TRY(hipMemsetAsync(F.xcd_next, 0, sizeof(uint32_t) * 8 * 32, stream));
            if ((st = mark(1, stream, [&] { return launch_fused(F, mode, stream, &lanes); }))) return st;
            if ((st = mark(3, stream, [&] { return resolve(s0, ns); }))) return st;
            iters++;
        }
        C = lanes;
        rs.paths_in_flight = lanes;
    }
    for (uint32_t s0 = 0; s0 < p.spp && !fused; s0 += chunk) {
        const uint32_t ns = std::min(chunk, p.spp - s0);
        const uint64_t w0 = (uint64_t)s0 * P, L = (uint64_t)ns * P;
        HIP_TRY(clear_film(ns));
        // fork: the sub-wavefront streams start after everything queued so far
        HIP_TRY(hipEventRecord(ws.fork_ev, stream));
        for (int k = 1; k < K; k++) HIP_TRY(hipStreamWaitEvent(strm[k], ws.fork_ev, 0));
        // spt_config.lockstep_first: the first cast of a fitting job — every
        // path started by the first refill, the count known exactly and long
        // enough that the isect and shade run (not the drain) — in the
        // one-lane-per-ray kernel (launch_isect_lockstep)
        bool lock0[kMaxStreams] = {};
        uint64_t started[kMaxStreams], sub_begin[kMaxStreams], sub_end[kMaxStreams];  // work items known
                                                                                      // started; the share
        for (int k = 0; k < K; k++) {
            Sub& b = ws.sub[k];
            // contiguous share of the chunk's work items (sample-major); pixel-major
            // work splits the chunk's samples instead, so that every stream
            // covers the whole tile (a band of rows per stream would leave the
            // streams unevenly loaded) and starts its samples of a pixel together
            uint64_t wb = w0 + L * k / K, we = w0 + L * (k + 1) / K;
            ra[k].chunk_s0 = s0; ra[k].chunk_ns = ns;
            if (ra[k].work_order && ns >= (uint32_t)K) {
                const uint32_t sk0 = s0 + ns * k / K, sk1 = s0 + ns * (k + 1) / K;
                wb = (uint64_t)sk0 * P; we = (uint64_t)sk1 * P;
                ra[k].chunk_s0 = sk0; ra[k].chunk_ns = sk1 - sk0;
            }
            HIP_TRY(hipMemsetAsync(b.cnt, 0, sizeof(Counters), strm[k]));
            ra[k].work_end = we;
            sa[k].sample0 = s0; sa[k].chunk_ns = ns;
            da[k].sample0 = s0; da[k].pm_ns = pixel_major ? ns : 0;  // the shade's film layout
            da[k].seg_count = nullptr;  // (set by a sharded camera cast of this chunk)
            da[k].xcd_next = lane_xcd ? &b.cnt->xcd_next[0][0] : nullptr;
            // the first refill starts at the sub-wavefront's first work item
            ra[k].q = q[k][0]; ra[k].surv = &b.cnt->surv[0]; ra[k].cursor_in = nullptr; ra[k].cursor_init = wb;
            ra[k].cursor_out = &b.cnt->cursor[0]; ra[k].qn_out = &b.cnt->qn[0];
            ra[k].surv_clear = nullptr;
            ra[k].casts_in = nullptr;
            ra[k].iter_tag = 1;
            const uint32_t first = (uint32_t)std::min<uint64_t>(b.cap, we - wb);
            sub_begin[k] = wb;
            sub_end[k] = we;
            started[k] = wb + first;
            lock0[k] = cfg.lockstep_first && fit && drain_on && !trav_stats && first >= drain_T[k];
            // (SPT_ISECT_CAMERA: the first isect launch starts these paths; the
            // camera cast makes them itself: the refill only keeps the books)
            ra[k].book_only = lock0[k] && cam_cast ? 1u : 0u;
            if (!kIsectCam &&
                (st = mark(0, strm[k], [&] { return launch_refill(ra[k], ra[k].book_only ? 1u : first, strm[k]); })))
                return st;
            ra[k].book_only = 0;
        }
        // isect -> shade -> refill per sub-wavefront until every queue drains.
        // A path cast in iteration i was started by the refill after iteration
        // <= i - 1 and makes at most max_depth casts, so once every work item
        // has been started (the cursor, read back one batch behind the
        // launches, reached the end) the queue is empty max_depth iterations
        // later: the loop stops there without a further readback.  Live counts
        // never grow after that, so a stale count is a safe grid size, and a
        // refill's grid is bounded by the work not yet known to be started.
        const uint64_t max_iters = (L * p.max_depth + Ck - 1) / Ck + p.max_depth + 64;
        uint32_t known[kMaxStreams];
        int cur[kMaxStreams], pending[kMaxStreams], pend_cur[kMaxStreams];
        uint64_t pend_it[kMaxStreams], limit[kMaxStreams];
        bool live[kMaxStreams];
        for (int k = 0; k < K; k++) {
            known[k] = (uint32_t)std::min<uint64_t>(ws.sub[k].cap, started[k] - sub_begin[k]);
            cur[k] = 0;
            pending[k] = -1;
            pend_cur[k] = 0;
            pend_it[k] = 0;
            // everything fit in the first refill: exactly max_depth iterations
            limit[k] = started[k] >= sub_end[k] ? p.max_depth : UINT64_MAX;
            live[k] = known[k] > 0;
        }
        uint64_t it = 0;
        const uint32_t batch = 4;
        uint32_t nbatch = 0;
        int nlive = 0;
        for (int k = 0; k < K; k++) nlive += live[k] ? 1 : 0;
        while (nlive > 0) {
            for (uint32_t bi = 0; bi < batch && nlive > 0; bi++) {
                for (int k = 0; k < K; k++) {
                    if (!live[k]) continue;
                    if (it >= limit[k]) {  // drained by construction
                        live[k] = false;
                        nlive--;
                        continue;
                    }
                    Sub& b = ws.sub[k];
                    const int c = cur[k], nx = 1 - c;
                    ia[k].q = q[k][c];
                    ia[k].count = &b.cnt->qn[c];
                    const bool cam = kIsectCam && !trav_stats;
                    if (cam) {
                        // survivors in q[c] (surv[c]) plus new camera paths after
                        // them; the previous launch (queue nx) left its cursor in
                        // cursor[nx]; this one's shade appends to surv[nx]
                        RefillArgs& R = ia[k].cam;
                        R = ra[k];
                        R.q = q[k][c];
                        R.surv = &b.cnt->surv[c];
                        R.cursor_in = it == 0 ? nullptr : &b.cnt->cursor[nx];
                        R.cursor_out = &b.cnt->cursor[c];
                        R.qn_out = &b.cnt->qn[c];
                        R.isect_next = isect_next_of(b.cnt, nx);
                        R.surv_clear = &b.cnt->surv[nx];
                        R.casts_in = nullptr;
                        R.iter_tag = (uint32_t)it + 1;
                        ia[k].next = isect_next_of(b.cnt, c);
                    }
                    // The drain phase: once the stream's last work items are (about
                    // to be) started — the host's view lags one or two batches, in
                    // which the cursor moves < kDrainLookahead capacities — a drain
                    // launch follows the shade.  Whichever sees the queue short
                    // (< drain_T) runs: the isect and shade skip and the drain
                    // finishes every queued path, or the drain skips.  Later
                    // iterations find the queue empty (no-op launches).
                    const bool dph = drain_on && (limit[k] != UINT64_MAX ||
                                                  sub_end[k] - started[k] < kDrainLookahead * (uint64_t)b.cap);
                    // drain_casts after the exhausting refill (limit - max_depth) the
                    // drain runs whatever the queue holds, and the stream ends: no
                    // work is left to start, so nothing can enter its queue again
                    const bool force = dph && cfg.drain_casts && limit[k] != UINT64_MAX &&
                                       it + p.max_depth >= limit[k] + cfg.drain_casts;
                    ia[k].drain_below = force ? 0xffffffffu : dph ? drain_T[k] : 0u;
                    sa[k].drain_below = ia[k].drain_below;
                    if (force) {
                        da[k].q = q[k][c];
                        da[k].qcount = &b.cnt->qn[c];
                        da[k].drain_below = 0xffffffffu;
                        da[k].perm = nullptr;
                        if (drain_sort) {  // the drain's order: by direction octant, then origin (kernels.hip)
                            const size_t cap = b.cap;  // (buffers: ensure_workspace)
                            uint32_t* kb = b.sort_buf;
                            HIP_TRY(launch_drain_sort(sc->dev(), q[k][c], &b.cnt->qn[c], (uint32_t)b.cap, kb, kb + cap,
                                                      kb + 2 * cap, kb + 3 * cap, b.sort_tmp, &b.sort_tmp_bytes,
                                                      strm[k]));
                            da[k].perm = kb + 3 * cap;
                        }
                        // (the drain counts the queued paths' first casts itself: the stream
                        // ends here, and a bookkeeping refill behind it would wait for CU
                        // slots behind the other working set's persistent drain, 0.4 ms on
                        // the 1/8 tile, profiles/r06_exp/tile8_trace/)
                        da[k].count_queue = 1;
                        if ((st = mark(4, strm[k], [&] { return launch_drain(da[k], mode, strm[k]); }))) return st;
                        da[k].count_queue = 0;
                        drain_launches++;
                        cur[k] = nx;
                        live[k] = false;
                        nlive--;
                        continue;
                    }
                    const bool lockstep = it == 0 && lock0[k];
                    if (lockstep) rs.lockstep_casts += known[k];
                    // sharded survivors (spt_internal.h kShards): when the camera cast
                    // holds the sub-wavefront's every path and the drain takes the
                    // queue next, its per-XCD pools over the same segments
                    bool sharded = false;
                    if (lockstep && cam_cast) {
                        // the first cast, camera ray to shade, in one launch; survivors
                        // into queue nx (surv[nx] zeroed with the counters), the
                        // refill below keeps the books as after a shade
                        sharded = cam_shards && started[k] >= sub_end[k] && cfg.drain_casts == 1 && !drain_sort;
                        CameraCastArgs ca;
                        ca.r = ra[k];  // the first refill's work items (cursor_init: the share's start)
                        ca.s = sa[k];
                        ca.s.in = q[k][c];
                        ca.s.out = q[k][nx];
                        ca.s.hits = nullptr;
                        ca.s.count_in = &b.cnt->qn[c];
                        ca.s.count_out = sharded ? &b.cnt->surv_shard[0][0] : &b.cnt->surv[nx];
                        ca.s.shard_items = sharded ? known[k] : 0u;
                        ca.n = known[k];
                        if ((st = mark(1, strm[k], [&] { return launch_camera_cast(ca, mode, strm[k]); }))) return st;
                        if (sharded) {
                            da[k].seg_count = &b.cnt->surv_shard[0][0];
                            da[k].seg_items = known[k];
                            da[k].seg_block = kIsectBlock;
                            da[k].xcd_next = &b.cnt->xcd_next[0][0];
                        }
                    } else if ((st = mark(1, strm[k], [&] {
                             if (lockstep) return launch_isect_lockstep(ia[k], known[k], strm[k]);
                             return trav_stats ? launch_isect_queue_stats(ia[k], known[k], strm[k])
                                               : cam ? launch_isect_queue_cam(ia[k], known[k], strm[k])
                                                     : launch_isect_queue(ia[k], known[k], strm[k]);
                         })))
                        return st;
                    // surv[nx] was zeroed by the previous refill (surv_clear)
                    sa[k].in = q[k][c]; sa[k].out = q[k][nx];
                    sa[k].count_in = &b.cnt->qn[c];
                    sa[k].count_out = &b.cnt->surv[nx];
                    if (!(lockstep && cam_cast) &&
                        (st = mark(2, strm[k], [&] { return launch_shade(sa[k], mode, known[k], strm[k]); })))
                        return st;
                    // (at a chunk's first iteration the count is known exactly: no
                    // conditional drain when it cannot be short)
                    if (dph && !(it == 0 && known[k] >= drain_T[k])) {
                        da[k].q = q[k][c];
                        da[k].qcount = &b.cnt->qn[c];
                        da[k].drain_below = drain_T[k];
                        da[k].perm = nullptr;
                        if ((st = mark(4, strm[k], [&] { return launch_drain(da[k], mode, strm[k]); }))) return st;
                        drain_launches++;
                    }
                    if (cam) {  // no refill launch: the next isect starts the new paths
                        cur[k] = nx;
                        continue;
                    }
                    ra[k].q = q[k][nx]; ra[k].surv = &b.cnt->surv[nx]; ra[k].cursor_in = &b.cnt->cursor[c];
                    ra[k].cursor_out = &b.cnt->cursor[nx]; ra[k].qn_out = &b.cnt->qn[nx];
                    ra[k].surv_clear = &b.cnt->surv[c];
                    ra[k].casts_in = &b.cnt->qn[c];
                    ra[k].iter_tag = (uint32_t)it + 2;
                    // (after a sharded camera cast: its survivors are the shards' sum, and
                    // the drain's per-XCD pool counters start at zero)
                    uint32_t* const xcd_keep = ra[k].xcd_next;
                    if (sharded) {
                        ra[k].surv_shards = &b.cnt->surv_shard[0][0];
                        ra[k].xcd_next = &b.cnt->xcd_next[0][0];
                    }
                    // new paths: at most the work not yet known to be started (one
                    // block still runs to carry the counters over)
                    const uint32_t fill = (uint32_t)std::min<uint64_t>(b.cap, sub_end[k] - started[k]);
                    if ((st = mark(0, strm[k], [&] { return launch_refill(ra[k], fill, strm[k]); })))
                        return st;
                    ra[k].surv_shards = nullptr;
                    ra[k].xcd_next = xcd_keep;
                    cur[k] = nx;
                }
                it++;
            }
            if (nlive == 0) break;
            const int slot = (int)(nbatch++ & 1u);
            for (int k = 0; k < K; k++) {
                if (!live[k] || limit[k] != UINT64_MAX) continue;  // bounded streams need no readback
                Sub& b = ws.sub[k];
                HIP_TRY(hipMemcpyAsync(b.host_cnt + slot, b.cnt, sizeof(Counters), hipMemcpyDeviceToHost, strm[k]));
                HIP_TRY(hipEventRecord(b.count_ev[slot], strm[k]));
            }
            for (int k = 0; k < K; k++) {
                if (!live[k] || limit[k] != UINT64_MAX) continue;
                Sub& b = ws.sub[k];
                if (pending[k] >= 0) {
                    HIP_TRY(hipEventSynchronize(b.count_ev[pending[k]]));
                    const Counters& hc = b.host_cnt[pending[k]];
                    if (kIsectCam && !trav_stats) {
                        // after an isect on queue 1 - pend_cur and its shade into
                        // pend_cur: the next launch holds those survivors plus as
                        // many new paths as fit
                        const uint32_t sv = hc.surv[pend_cur[k]];
                        const uint64_t cu = hc.cursor[1 - pend_cur[k]];
                        started[k] = std::max<uint64_t>(started[k], cu);
                        const uint64_t left = sub_end[k] > started[k] ? sub_end[k] - started[k] : 0;
                        known[k] = (uint32_t)std::min<uint64_t>(ws.sub[k].cap, sv + left);
                    } else {
                        known[k] = hc.qn[pend_cur[k]];
                        started[k] = std::max<uint64_t>(started[k], hc.cursor[pend_cur[k]]);
                    }
                    if (known[k] == 0) {
                        live[k] = false;
                        nlive--;
                        continue;
                    }
                    // the refill after iteration T - 2 (tag T) started the last
                    // work item: its paths cast in iterations T - 1 .. T + max_depth - 2
                    if (hc.exhausted) limit[k] = hc.exhausted - 1 + p.max_depth;
                    else if (started[k] >= sub_end[k]) limit[k] = pend_it[k] + p.max_depth;
                }
                pending[k] = slot;
                pend_cur[k] = cur[k];
                pend_it[k] = it;
            }
            if (it > max_iters)
                return fail(SPT_ERR_HIP, "spt_render: queue did not drain after %llu iterations",
                            (unsigned long long)it);
            // the batch stays short: the first readback that shows the last work
            // item started bounds the loop, and a long batch would overshoot it
            // (the GPU still has one batch queued while the host waits)
        }
        iters += it;
        // join the sub-wavefront streams back into the caller's stream
        for (int k = 1; k < K; k++) {
            HIP_TRY(hipEventRecord(ws.sub[k].join_ev, strm[k]));
            HIP_TRY(hipStreamWaitEvent(stream, ws.sub[k].join_ev, 0));
        }
        if ((st = mark(3, stream, [&] { return resolve(s0, ns); }))) return st;
    }
    // pinned destination: a pageable one makes the copy a staged, slower transfer
    HIP_TRY(hipMemcpyAsync(slot->host, slot->dev, sizeof(Stats), hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipEventRecord(slot->done, stream));
    HIP_TRY(hipEventRecord(ws.free_ev, stream));  // every sub-stream joined `stream` before the resolve
    HIP_TRY(hipEventRecord(jtab->ev[set_idx], stream));  // this render is done with the jump table
    jtab->ev_used[set_idx] = true;
    HIP_TRY(hipStreamWaitEvent(caller, ws.free_ev, 0));  // the caller's next work sees the film
    ws.used = true;
    guard.armed = false;
    rs.iterations = iters;
    rs.drain_launches = drain_launches;
    rs.work_order = pixel_major ? SPT_WORK_PIXEL_MAJOR : SPT_WORK_SAMPLE_MAJOR;
    // the policy that ran: every queue kernel has a non-temporal instance,
    // except the traversal-statistics isect variant (diagnostics)
    rs.queue_cache = fused ? 0u : (queue_nt && !trav_stats ? SPT_QUEUE_CACHE_STREAM : SPT_QUEUE_CACHE_CACHED);
    rs.streams = (uint32_t)K;
    rs.fused = fused ? 1u : 0u;
    rs.drain_refill_idle = !fused && drain_on ? drain_idle : 0u;
    slot->regen_base = std::min<uint64_t>(C, P * p.spp);
    slot->ticket = sc->ws.next_ticket++;
    slot->pending = true;
    *ticket_out = slot->ticket;
    return SPT_OK;
}

spt_status spt_render_wait(spt_scene sc, uint64_t ticket, spt_render_stats* stats_out) {
    if (!sc) return fail(SPT_ERR_INVALID, "spt_render_wait: NULL scene");
    DeviceGuard dg(sc->device);
    std::lock_guard<std::mutex> lock(sc->mu);
    RenderSlot& r = sc->ws.slots[ticket % kRenderSlots];
    if (!r.pending || r.ticket != ticket)
        return fail(SPT_ERR_INVALID, "spt_render_wait: ticket %llu is not a queued render (already collected, "
                    "or %d renders were queued after it)", (unsigned long long)ticket, kRenderSlots);
    return render_collect(r, sc->ws, stats_out);
}

spt_status spt_render(spt_scene sc, const spt_render_params* pp, float* film_dev, spt_render_stats* stats_out,
                      void* stream) {
    uint64_t ticket = 0;
    spt_status st = spt_render_async(sc, pp, film_dev, stream, &ticket);
    if (st) return st;
    return spt_render_wait(sc, ticket, stats_out);
}

spt_status spt_scene_isect_busy_begin(spt_scene sc) {
    if (!sc) return fail(SPT_ERR_INVALID, "spt_scene_isect_busy_begin: NULL scene");
    std::lock_guard<std::mutex> lock(sc->mu);
    for (auto& v : sc->ws.iv_all) v.clear();
    sc->ws.collect_iv = true;
    return SPT_OK;
}

spt_status spt_scene_kernel_busy(spt_scene sc, uint32_t kernels, double* busy_ms, uint64_t* launches) {
    if (!sc || !busy_ms) return fail(SPT_ERR_INVALID, "spt_scene_kernel_busy: NULL argument");
    if (kernels == 0 || kernels > (SPT_KERNEL_ISECT | SPT_KERNEL_DRAIN))
        return fail(SPT_ERR_INVALID, "spt_scene_kernel_busy: kernels must be a non-empty mask of SPT_KERNEL_*");
    std::lock_guard<std::mutex> lock(sc->mu);
    std::vector<std::pair<double, double>> iv;
    if (kernels & SPT_KERNEL_ISECT) iv.insert(iv.end(), sc->ws.iv_all[0].begin(), sc->ws.iv_all[0].end());
    if (kernels & SPT_KERNEL_DRAIN) iv.insert(iv.end(), sc->ws.iv_all[1].begin(), sc->ws.iv_all[1].end());
    std::sort(iv.begin(), iv.end());
    *busy_ms = interval_union(iv);
    if (launches) *launches = iv.size();
    return SPT_OK;
}

spt_status spt_scene_isect_busy_end(spt_scene sc, double* busy_ms, uint64_t* launches) {
    if (!sc || !busy_ms) return fail(SPT_ERR_INVALID, "spt_scene_isect_busy_end: NULL argument");
    std::lock_guard<std::mutex> lock(sc->mu);
    std::vector<std::pair<double, double>> iv;
    iv.swap(sc->ws.iv_all[0]);
    sc->ws.iv_all[1].clear();
    sc->ws.collect_iv = false;
    std::sort(iv.begin(), iv.end());
    *busy_ms = interval_union(iv);
    if (launches) *launches = iv.size();
    return SPT_OK;
}

}  // extern "C"
