// spt.hpp — C++ host wrapper over include/spt.h keeping the reference's
// exception convention (OPTIX_CHECK / CUDA_CHECK throw std::runtime_error,
// optix_backend.h:25-66) and its Scene / backend call shape
// (Scene::add_triangle_mesh / commit / intersect, main.cpp:286-352).
#pragma once
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/spt.h"

namespace spt {

inline void check(spt_status s, const char* what) {
    if (s != SPT_OK) throw std::runtime_error(std::string(what) + " failed (" + std::to_string(s) + "): " + spt_last_error());
}

inline bool ends_with(const std::string& s, const char* suffix) {
    const size_t n = std::char_traits<char>::length(suffix);
    return s.size() >= n && s.compare(s.size() - n, n, suffix) == 0;
}

// An OBJ (main.cpp:141-251) or a pbrt-v3 scene (the pbrt-parser path), by extension.
struct Mesh {
    spt_mesh m{};
    spt_pbrt_info pbrt{};
    explicit Mesh(const std::string& path) {
        if (ends_with(path, ".pbrt")) check(spt_pbrt_load(path.c_str(), &m, &pbrt), "spt_pbrt_load");
        else check(spt_obj_load(path.c_str(), &m), "spt_obj_load");
    }
    ~Mesh() { spt_mesh_free(&m); }
    Mesh(const Mesh&) = delete;
    Mesh& operator=(const Mesh&) = delete;
};

// main.cpp:286-352 Scene, minus the Enoki arrays: geometry lives on the GPU
// behind spt_scene.
class Scene {
  public:
    Scene() = default;
    ~Scene() { if (scene_) spt_scene_destroy(scene_); }
    Scene(const Scene&) = delete;
    Scene& operator=(const Scene&) = delete;

    void add_triangle_mesh(const std::string& path) {  // main.cpp:288
        mesh_.reset(new Mesh(path));
        pbrt_ = mesh_->pbrt;
    }
    void commit(int device = 0) {                      // main.cpp:312
        if (!mesh_) throw std::runtime_error("Scene::commit: no mesh added");
        check(spt_init(device), "spt_init");
        const spt_mesh& m = mesh_->m;
        check(spt_scene_create(m.pos_tri, m.pos, m.nvert, m.ntri, m.nrm_tri, m.nrm, m.nnrm, m.tc_tri, m.tc, m.ntc,
                               m.mat_id, &scene_),
              "spt_scene_create");
    }
    // Binary scene cache (spt_scene_save / spt_scene_load): the committed
    // scene, with the pbrt camera / film / sky as its extra bytes.
    void save(const std::string& path) const {
        const bool has = pbrt_.has_camera || pbrt_.has_env;
        check(spt_scene_save(scene_, path.c_str(), has ? &pbrt_ : nullptr, has ? sizeof(pbrt_) : 0), "spt_scene_save");
    }
    void load(const std::string& path, int device = 0) {
        check(spt_init(device), "spt_init");
        if (scene_) spt_scene_destroy(scene_);
        scene_ = nullptr;
        mesh_.reset();
        pbrt_ = spt_pbrt_info{};
        uint64_t n = 0;
        check(spt_scene_load(path.c_str(), &scene_, &pbrt_, sizeof(pbrt_), &n), "spt_scene_load");
        if (n != 0 && n != sizeof(pbrt_)) throw std::runtime_error(path + ": extra bytes are not an spt_pbrt_info");
        if (n == 0) pbrt_ = spt_pbrt_info{};
    }
    // spt_render_async / spt_render_wait: queue the render on `stream` (the
    // stream's next work waits for it) and collect its statistics later
    uint64_t render_async(const spt_render_params& p, float* film_dev, void* stream) {
        uint64_t ticket = 0;
        check(spt_render_async(scene_, &p, film_dev, stream, &ticket), "spt_render_async");
        return ticket;
    }
    void render_wait(uint64_t ticket, spt_render_stats* stats) {
        check(spt_render_wait(scene_, ticket, stats), "spt_render_wait");
    }
    void render(const spt_render_params& p, float* film_dev, spt_render_stats* stats, void* stream = nullptr) {
        check(spt_render(scene_, &p, film_dev, stats, stream), "spt_render");
    }
    // Commit a mesh loaded elsewhere (read only: several devices' scenes may
    // be built from one host mesh, one thread per device).
    void commit_from(const Mesh& mesh, int device) {
        check(spt_init(device), "spt_init");
        const spt_mesh& m = mesh.m;
        check(spt_scene_create(m.pos_tri, m.pos, m.nvert, m.ntri, m.nrm_tri, m.nrm, m.nnrm, m.tc_tri, m.tc, m.ntc,
                               m.mat_id, &scene_),
              "spt_scene_create");
        pbrt_ = mesh.pbrt;
    }
    spt_scene handle() const { return scene_; }
    const spt_mesh& mesh() const { return mesh_->m; }  // not after load()
    const spt_pbrt_info& pbrt_info() const { return pbrt_; }

  private:
    std::unique_ptr<Mesh> mesh_;
    spt_pbrt_info pbrt_{};
    spt_scene scene_ = nullptr;
};

}  // namespace spt
