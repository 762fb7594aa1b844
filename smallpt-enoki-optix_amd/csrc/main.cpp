// main.cpp — C++ host driver mirroring the reference's main() (main.cpp:354-446):
// load an OBJ (or a pbrt-v3 scene), commit the scene, render, normalise, read
// back, write a PFM, print the wall time.  Every constant defaults to the
// reference's; a .pbrt file's camera, film size and infinite light replace
// them, and flags override both.  A .sptc file is a binary scene cache
// (spt_scene_load: no parse, no BVH build); --save-cache writes one after commit.
//
//   spt_render_cli [scene.obj|scene.pbrt|scene.sptc] [-w W] [-h H] [-s spp] [-d casts] [-o out.pfm]
//                  [--wavefront paths] [--rr depth] [--rng-x-first] [--device N] [--save-cache f.sptc]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <vector>

#include "spt.hpp"

int main(int argc, char** argv) {
    std::string obj = "mitsuba.obj";  // main.cpp:365
    std::string out = "wurst.pfm";    // main.cpp:442
    std::string cache_out;
    int device = 0;
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
        else if (!a.empty() && a[0] != '-') obj = a;
        else { std::cerr << "unknown flag " << a << "\n"; return 2; }
    }
    try {
        spt::Scene scene;
        auto tl = std::chrono::steady_clock::now();
        if (spt::ends_with(obj, ".sptc")) {
            scene.load(obj, device);
        } else {
            scene.add_triangle_mesh(obj);  // main.cpp:365
            scene.commit(device);          // main.cpp:366
        }
        std::cerr << "scene ready in "
                  << std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tl).count() << " ms"
                  << std::endl;
        if (!cache_out.empty()) scene.save(cache_out);
        const spt_pbrt_info& pi = scene.pbrt_info();
        if (pi.has_camera) {
            p.camera = pi.camera;
            if (!set_w) p.width = pi.xres;
            if (!set_h) p.height = pi.yres;
        }
        if (pi.has_env)
            for (int c = 0; c < 3; c++) p.env[c] = pi.env[c];
        const size_t npx = (size_t)p.width * p.height;
        float* film = nullptr;
        if (hipMalloc((void**)&film, sizeof(float) * 3 * npx) != hipSuccess) throw std::runtime_error("hipMalloc film");
        spt_render_stats st;
        auto t0 = std::chrono::steady_clock::now();
        scene.render(p, film, &st);    // main.cpp:385-429
        double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        std::cout << ms << std::endl;  // main.cpp:431
        std::vector<float> host(3 * npx);
        if (hipMemcpy(host.data(), film, sizeof(float) * 3 * npx, hipMemcpyDeviceToHost) != hipSuccess)
            throw std::runtime_error("hipMemcpy film");
        (void)hipFree(film);
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
