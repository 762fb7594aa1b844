// main.cpp — C++ host driver mirroring the reference's main() (main.cpp:354-446):
// load an OBJ (or a pbrt-v3 scene), commit the scene, render, normalise, read
// back, write a PFM, print the wall time.  Every constant defaults to the
// reference's; a .pbrt file's camera, film size and infinite light replace
// them, and flags override both.  A .sptc file is a binary scene cache
// (spt_scene_load: no parse, no BVH build); --save-cache writes one after commit.
//
// --gpus N renders the image on N devices of this node (the
// reference is single-GPU): one host thread per device commits its own copy
// of the scene (replicated BVH) and renders its interleaved row-group tile
// (spt_render_params.tile_*), then ONE RCCL collective, ncclGather over xGMI
// from a communicator per device (ncclCommInitAll, driven from one thread in
// an ncclGroupStart/End), queued on each rank's stream behind its render
// (spt_render_async, no host synchronisation between them), brings the fp32
// tiles to device 0, whose rows are put back in place.  Pixel RNG streams are keyed by the global pixel, so
// the image is bit-identical for any N.  --rehearse-shared-gpu places every
// tile on device 0 and gathers with device copies instead (a one-GPU box
// cannot host two RCCL ranks), so the tiling and assembly run anywhere.
//
//   spt_render_cli [scene.obj|scene.pbrt|scene.sptc] [-w W] [-h H] [-s spp] [-d casts] [-o out.pfm]
//                  [--wavefront paths] [--rr depth] [--rng-x-first] [--device N] [--save-cache f.sptc]
//                  [--gpus N] [--rows-per-group R] [--rehearse-shared-gpu]
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <iostream>
#include <memory>
#include <thread>
#include <vector>

#include "spt.hpp"

namespace {

using clock_t_ = std::chrono::steady_clock;
double ms_since(clock_t_::time_point t0) {
    return std::chrono::duration<double, std::milli>(clock_t_::now() - t0).count();
}

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
void nccl_check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}

// One device's share of a multi-GPU render.
struct Rank {
    int index = 0;                // tile index (the rank)
    int device = 0;
    spt::Scene scene;
    std::vector<uint32_t> rows;   // this tile's image rows (spt_tile_rows)
    float* tile = nullptr;        // (3, max_rows, W) fp32, padded to the largest tile
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;    // recorded on `stream` behind the queued render
    uint64_t ticket = 0;          // spt_render_async's, collected after the gather
    spt_render_stats st{};
    std::exception_ptr err;
};

// Renders p over ranks.size() tiles and assembles the (3, H, W) image on the
// host.  The scene is committed on each device (or loaded from the cache).
void render_multi(const std::string& path, const spt::Mesh* mesh, spt_render_params p, int ngpu, bool shared,
                  uint32_t rows_per_group, std::vector<float>& image, spt_render_stats& total, double& ms) {
    int ndev = 0;
    hip_check(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
    if (!shared && ngpu > ndev)
        throw std::runtime_error("--gpus " + std::to_string(ngpu) + " but " + std::to_string(ndev) + " devices visible");
    const uint32_t W = p.width, H = p.height;
    std::vector<std::unique_ptr<Rank>> ranks;
    uint32_t max_rows = 1;
    for (int r = 0; r < ngpu; r++) {
        ranks.emplace_back(new Rank);
        Rank& k = *ranks.back();
        k.index = r;
        k.device = shared ? 0 : r;
        const uint32_t n = spt_tile_rows(H, (uint32_t)r, (uint32_t)ngpu, rows_per_group, nullptr, 0);
        k.rows.resize(n);
        spt_tile_rows(H, (uint32_t)r, (uint32_t)ngpu, rows_per_group, k.rows.data(), n);
        max_rows = std::max(max_rows, n);
    }
    const size_t count = (size_t)3 * max_rows * W;  // floats per rank in the gather
    // set-up, one thread per device: scene commit (replicated BVH), film tile, stream
    auto each = [&](auto&& fn) {
        std::vector<std::thread> th;
        for (auto& k : ranks)
            th.emplace_back([&fn, &k] {
                try {
                    hip_check(hipSetDevice(k->device), "hipSetDevice");
                    fn(*k);
                } catch (...) {
                    k->err = std::current_exception();
                }
            });
        for (auto& t : th) t.join();
        for (auto& k : ranks)
            if (k->err) std::rethrow_exception(k->err);
    };
    each([&](Rank& k) {
        if (mesh) k.scene.commit_from(*mesh, k.device);
        else k.scene.load(path, k.device);
        hip_check(hipStreamCreateWithFlags(&k.stream, hipStreamNonBlocking), "hipStreamCreate");
        hip_check(hipEventCreateWithFlags(&k.done, hipEventDisableTiming), "hipEventCreate");
        hip_check(hipMalloc((void**)&k.tile, sizeof(float) * count), "hipMalloc tile");
        hip_check(hipMemsetAsync(k.tile, 0, sizeof(float) * count, k.stream), "hipMemset tile");
        hip_check(hipStreamSynchronize(k.stream), "hipStreamSynchronize");
    });
    std::vector<ncclComm_t> comms;
    if (!shared) {
        std::vector<int> devs;
        for (auto& k : ranks) devs.push_back(k->device);
        comms.resize(ngpu);
        nccl_check(ncclCommInitAll(comms.data(), ngpu, devs.data()), "ncclCommInitAll");
    }
    float* recv = nullptr;  // device 0: ngpu x count floats
    hip_check(hipSetDevice(ranks[0]->device), "hipSetDevice");
    hip_check(hipMalloc((void**)&recv, sizeof(float) * count * ngpu), "hipMalloc gather");

    const auto t0 = clock_t_::now();
    // every rank queues its tile's render (main.cpp:385-429 on its rows) on its
    // stream and returns: the gather below is queued on the same streams behind
    // the renders (spt_render_async: the caller stream's next work waits for
    // the render), so no host synchronisation sits between render and gather
    each([&](Rank& k) {
        spt_render_params q = p;
        q.tile_index = (uint32_t)k.index;
        q.tile_count = (uint32_t)ngpu;
        q.rows_per_group = rows_per_group;
        if (!k.rows.empty()) k.ticket = k.scene.render_async(q, k.tile, k.stream);
        hip_check(hipEventRecord(k.done, k.stream), "hipEventRecord");
    });
    // the one exchange step: the fp32 tiles to device 0
    if (!shared) {
        nccl_check(ncclGroupStart(), "ncclGroupStart");
        for (int r = 0; r < ngpu; r++) {
            hip_check(hipSetDevice(ranks[r]->device), "hipSetDevice");
            nccl_check(ncclGather(ranks[r]->tile, r == 0 ? recv : nullptr, count, ncclFloat, 0, comms[r],
                                  ranks[r]->stream),
                       "ncclGather");
        }
        nccl_check(ncclGroupEnd(), "ncclGroupEnd");
        for (auto& k : ranks) {
            hip_check(hipSetDevice(k->device), "hipSetDevice");
            hip_check(hipStreamSynchronize(k->stream), "hipStreamSynchronize");
        }
    } else {
        hip_check(hipSetDevice(ranks[0]->device), "hipSetDevice");
        for (int r = 0; r < ngpu; r++) {
            // (device copies on rank 0's stream, each behind that rank's render)
            hip_check(hipStreamWaitEvent(ranks[0]->stream, ranks[r]->done, 0), "hipStreamWaitEvent");
            hip_check(hipMemcpyAsync(recv + (size_t)r * count, ranks[r]->tile, sizeof(float) * count,
                                     hipMemcpyDeviceToDevice, ranks[0]->stream),
                      "hipMemcpy gather");
        }
        hip_check(hipStreamSynchronize(ranks[0]->stream), "hipStreamSynchronize");
    }
    ms = ms_since(t0);
    each([&](Rank& k) {  // the renders' statistics (their work is done: the gather waited for it)
        if (!k.rows.empty()) k.scene.render_wait(k.ticket, &k.st);
    });

    // rank 0 puts every tile's rows back in place
    std::vector<float> gathered(count * ngpu);
    hip_check(hipSetDevice(ranks[0]->device), "hipSetDevice");
    hip_check(hipMemcpy(gathered.data(), recv, sizeof(float) * gathered.size(), hipMemcpyDeviceToHost), "hipMemcpy");
    image.assign((size_t)3 * H * W, 0.0f);
    total = spt_render_stats{};
    for (int r = 0; r < ngpu; r++) {
        const Rank& k = *ranks[r];
        const size_t n = k.rows.size();
        const float* t = gathered.data() + (size_t)r * count;
        for (int c = 0; c < 3; c++)
            for (size_t i = 0; i < n; i++)
                std::memcpy(&image[((size_t)c * H + k.rows[i]) * W], t + ((size_t)c * n + i) * W, sizeof(float) * W);
        total.paths += k.st.paths;
        total.ray_casts += k.st.ray_casts;
    }
    for (auto& c : comms) ncclCommDestroy(c);
    (void)hipFree(recv);
    for (auto& k : ranks) {
        hip_check(hipSetDevice(k->device), "hipSetDevice");
        (void)hipFree(k->tile);
        (void)hipEventDestroy(k->done);
        (void)hipStreamDestroy(k->stream);
    }
}

}  // namespace

int main(int argc, char** argv) {
    std::string obj = "mitsuba.obj";  // main.cpp:365
    std::string out = "wurst.pfm";    // main.cpp:442
    std::string cache_out;
    int device = 0, ngpu = 0;
    uint32_t rows_per_group = 8;
    bool shared = false;
    spt_render_params p;
    spt_default_params(&p);            // 512 x 512, 100 spp, 2 casts (main.cpp:357-361)
    bool set_w = false, set_h = false;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) { std::cerr << "missing value for " << a << "\n"; std::exit(2); }
            return argv[++i];
        };
        if (a == "-w") { p.width = (uint32_t)std::atoi(next()); set_w = true; }
        else if (a == "-h") { p.height = (uint32_t)std::atoi(next()); set_h = true; }
        else if (a == "-s") p.spp = (uint32_t)std::atoi(next());
        else if (a == "-d") p.max_depth = (uint32_t)std::atoi(next());
        else if (a == "-o") out = next();
        else if (a == "--wavefront") p.wavefront_paths = (uint32_t)std::atoi(next());
        else if (a == "--rr") p.rr_start_depth = (uint32_t)std::atoi(next());
        else if (a == "--rng-x-first") p.rng_order = SPT_RNG_X_FIRST;
        else if (a == "--device") device = std::atoi(next());
        else if (a == "--save-cache") cache_out = next();
        else if (a == "--gpus") ngpu = std::atoi(next());
        else if (a == "--rows-per-group") rows_per_group = (uint32_t)std::atoi(next());
        else if (a == "--rehearse-shared-gpu") shared = true;
        else if (!a.empty() && a[0] != '-') obj = a;
        else { std::cerr << "unknown flag " << a << "\n"; return 2; }
    }
    if (ngpu < 0 || rows_per_group == 0) { std::cerr << "--gpus must be >= 1, --rows-per-group >= 1\n"; return 2; }
    try {
        const bool cache = spt::ends_with(obj, ".sptc");
        std::unique_ptr<spt::Mesh> mesh;
        spt_pbrt_info pi{};
        spt::Scene scene;  // the single-device path
        auto tl = clock_t_::now();
        if (ngpu >= 1) {  // multi-GPU: the host mesh once, a scene per device in render_multi
            if (cache) {
                spt::Scene probe;  // the cache's pbrt camera / film / sky
                probe.load(obj, device);
                pi = probe.pbrt_info();
            } else {
                mesh.reset(new spt::Mesh(obj));
                pi = mesh->pbrt;
            }
        } else if (cache) {
            scene.load(obj, device);
            pi = scene.pbrt_info();
        } else {
            scene.add_triangle_mesh(obj);  // main.cpp:365
            scene.commit(device);          // main.cpp:366
            pi = scene.pbrt_info();
        }
        std::cerr << "scene ready in " << ms_since(tl) << " ms" << std::endl;
        if (!cache_out.empty()) {
            if (ngpu >= 1) throw std::runtime_error("--save-cache: use it without --gpus");
            scene.save(cache_out);
        }
        if (pi.has_camera) {
            p.camera = pi.camera;
            if (!set_w) p.width = pi.xres;
            if (!set_h) p.height = pi.yres;
        }
        if (pi.has_env)
            for (int c = 0; c < 3; c++) p.env[c] = pi.env[c];
        const size_t npx = (size_t)p.width * p.height;
        std::vector<float> host(3 * npx);
        spt_render_stats st{};
        double ms = 0.0;
        if (ngpu >= 1) {
            render_multi(obj, mesh.get(), p, ngpu, shared, rows_per_group, host, st, ms);
            std::cout << ms << std::endl;  // main.cpp:431 (render + gather)
        } else {
            float* film = nullptr;
            hip_check(hipMalloc((void**)&film, sizeof(float) * 3 * npx), "hipMalloc film");
            auto t0 = clock_t_::now();
            scene.render(p, film, &st);    // main.cpp:385-429
            ms = ms_since(t0);
            std::cout << ms << std::endl;  // main.cpp:431
            hip_check(hipMemcpy(host.data(), film, sizeof(float) * 3 * npx, hipMemcpyDeviceToHost), "hipMemcpy film");
            (void)hipFree(film);
        }
        std::cout << "writing image" << std::endl;  // main.cpp:441
        spt::check(spt_pfm_write(out.c_str(), host.data(), host.data() + npx, host.data() + 2 * npx, p.width, p.height),
                   "spt_pfm_write");
        std::cout << "paths " << st.paths << " casts " << st.ray_casts << " Mpaths/s " << st.paths / (ms * 1e3)
                  << std::endl;
        std::cout << "done" << std::endl;  // main.cpp:444
    } catch (const std::exception& e) {
        std::cerr << e.what() << std::endl;
        return 1;
    }
    return 0;
}
