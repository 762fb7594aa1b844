// host_io.cpp — host side of the reference that stays on the CPU:
//   spt_obj_load  : load_meshes (main.cpp:133-251).  tinyobjloader is an
//                   absent submodule, so this is our own reader with its
//                   index semantics: `f` polygons triangulated as a fan,
//                   1-based / negative relative indices, missing vn/vt -> -1,
//                   per-face material id = (usemtl index in the .mtl) + 1
//                   with 0 the default material (main.cpp:185,229-245).
//   spt_pfm_write : Fimage::save_pfm (fimage.h:33-58).
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/spt.h"
#include "host_error.h"

namespace {

struct Idx { int v, t, n; };

bool parse_index(const char*& p, int nv, int nt, int nn, Idx& out) {
    // 1-based, or relative to the elements read so far; 0 and anything
    // beyond int range are invalid (-2; the caller range-checks the rest)
    auto fix = [](long i, int n) -> int {
        if (i > 0) return i <= 0x7fffffffL ? (int)(i - 1) : -2;
        if (i < 0) return i >= -(long)n ? (int)(n + i) : -2;
        return -2;
    };
    char* end;
    long v = std::strtol(p, &end, 10);
    if (end == p) return false;
    p = end;
    out.v = fix(v, nv);
    out.t = -1;
    out.n = -1;
    if (*p == '/') {
        p++;
        if (*p != '/') {
            long t = std::strtol(p, &end, 10);
            if (end != p) { out.t = fix(t, nt); p = end; }
        }
        if (*p == '/') {
            p++;
            long n = std::strtol(p, &end, 10);
            if (end != p) { out.n = fix(n, nn); p = end; }
        }
    }
    return out.v >= 0;
}

void load_mtl(const std::string& path, std::map<std::string, int>& names, std::vector<float>& kd,
              std::vector<float>& ke) {
    FILE* f = std::fopen(path.c_str(), "r");
    if (!f) return;
    char line[4096];
    int cur = -1;
    while (std::fgets(line, sizeof(line), f)) {
        const char* p = line;
        while (*p == ' ' || *p == '\t') p++;
        if (!std::strncmp(p, "newmtl", 6) && (p[6] == ' ' || p[6] == '\t')) {
            p += 6;
            while (*p == ' ' || *p == '\t') p++;
            std::string name(p);
            while (!name.empty() && (name.back() == '\n' || name.back() == '\r' || name.back() == ' ')) name.pop_back();
            cur = (int)(kd.size() / 3);
            names[name] = cur;
            kd.push_back(0.0f); kd.push_back(0.0f); kd.push_back(0.0f);
            ke.push_back(0.0f); ke.push_back(0.0f); ke.push_back(0.0f);
        } else if (cur >= 0 && p[0] == 'K' && (p[1] == 'd' || p[1] == 'e') && (p[2] == ' ' || p[2] == '\t')) {
            float r = 0, g = 0, b = 0;
            std::sscanf(p + 2, "%f %f %f", &r, &g, &b);
            std::vector<float>& dst = p[1] == 'd' ? kd : ke;
            dst[cur * 3] = r; dst[cur * 3 + 1] = g; dst[cur * 3 + 2] = b;
        }
    }
    std::fclose(f);
}

template <typename T>
T* dup(const std::vector<T>& v) {
    if (v.empty()) return nullptr;
    T* p = (T*)std::malloc(sizeof(T) * v.size());
    std::memcpy(p, v.data(), sizeof(T) * v.size());
    return p;
}

}  // namespace

extern "C" {

spt_status spt_obj_load(const char* path, spt_mesh* out) {
    if (!path || !out) return spt_set_error(SPT_ERR_INVALID, "spt_obj_load: NULL argument");
    std::memset(out, 0, sizeof(*out));
    FILE* f = std::fopen(path, "r");
    if (!f) return spt_set_error(SPT_ERR_IO, "spt_obj_load: cannot open %s: %s", path, std::strerror(errno));
    std::string dir(path);
    size_t slash = dir.find_last_of('/');
    dir = slash == std::string::npos ? std::string() : dir.substr(0, slash + 1);

    std::vector<float> pos, nrm, tc, kd, ke;
    std::vector<int32_t> pt, nt, tt, mat;
    std::map<std::string, int> names;
    int cur_mat = -1;
    std::vector<Idx> poly;
    char* line = nullptr;
    size_t cap = 0;
    ssize_t len;
    bool bad = false;
    long lineno = 0;
    while ((len = getline(&line, &cap, f)) >= 0) {
        lineno++;
        const char* p = line;
        while (*p == ' ' || *p == '\t') p++;
        if (p[0] == 'v' && (p[1] == ' ' || p[1] == '\t')) {
            float x = 0, y = 0, z = 0;
            std::sscanf(p + 1, "%f %f %f", &x, &y, &z);
            pos.push_back(x); pos.push_back(y); pos.push_back(z);
        } else if (p[0] == 'v' && p[1] == 'n' && (p[2] == ' ' || p[2] == '\t')) {
            float x = 0, y = 0, z = 0;
            std::sscanf(p + 2, "%f %f %f", &x, &y, &z);
            nrm.push_back(x); nrm.push_back(y); nrm.push_back(z);
        } else if (p[0] == 'v' && p[1] == 't' && (p[2] == ' ' || p[2] == '\t')) {
            float u = 0, v = 0;
            std::sscanf(p + 2, "%f %f", &u, &v);
            tc.push_back(u); tc.push_back(v);
        } else if (p[0] == 'f' && (p[1] == ' ' || p[1] == '\t')) {
            p++;
            poly.clear();
            int nv = (int)(pos.size() / 3), ntc = (int)(tc.size() / 2), nn = (int)(nrm.size() / 3);
            while (true) {
                while (*p == ' ' || *p == '\t') p++;
                if (*p == '\0' || *p == '\n' || *p == '\r' || *p == '#') break;
                Idx ix;
                if (!parse_index(p, nv, ntc, nn, ix) || ix.t == -2 || ix.n == -2) { bad = true; break; }
                poly.push_back(ix);
                while (*p && *p != ' ' && *p != '\t' && *p != '\n' && *p != '\r') p++;
            }
            if (bad) break;
            for (size_t k = 1; k + 1 < poly.size(); k++) {  // fan triangulation
                const Idx* tri[3] = {&poly[0], &poly[k], &poly[k + 1]};
                for (int c = 0; c < 3; c++) {
                    pt.push_back(tri[c]->v);
                    nt.push_back(tri[c]->n);
                    tt.push_back(tri[c]->t);
                }
                mat.push_back(cur_mat + 1);  // main.cpp:185
            }
        } else if (!std::strncmp(p, "usemtl", 6) && (p[6] == ' ' || p[6] == '\t')) {
            p += 6;
            while (*p == ' ' || *p == '\t') p++;
            std::string name(p);
            while (!name.empty() && (name.back() == '\n' || name.back() == '\r' || name.back() == ' ')) name.pop_back();
            auto it = names.find(name);
            cur_mat = it == names.end() ? -1 : it->second;
        } else if (!std::strncmp(p, "mtllib", 6) && (p[6] == ' ' || p[6] == '\t')) {
            p += 6;
            while (*p == ' ' || *p == '\t') p++;
            std::string name(p);
            while (!name.empty() && (name.back() == '\n' || name.back() == '\r' || name.back() == ' ')) name.pop_back();
            load_mtl(dir + name, names, kd, ke);
        }
    }
    std::free(line);
    std::fclose(f);
    if (bad) return spt_set_error(SPT_ERR_INVALID, "spt_obj_load: %s:%ld: bad face index", path, lineno);
    // Index range check (tinyobj would hand out-of-range indices through).
    const long nv = (long)(pos.size() / 3), nvt = (long)(tc.size() / 2), nvn = (long)(nrm.size() / 3);
    for (int32_t i : pt)
        if (i < 0 || i >= nv) return spt_set_error(SPT_ERR_INVALID, "spt_obj_load: %s: vertex index %d of %ld", path, i + 1, nv);
    for (int32_t i : tt)
        if (i < -1 || i >= nvt) return spt_set_error(SPT_ERR_INVALID, "spt_obj_load: %s: texcoord index %d of %ld", path, i + 1, nvt);
    for (int32_t i : nt)
        if (i < -1 || i >= nvn) return spt_set_error(SPT_ERR_INVALID, "spt_obj_load: %s: normal index %d of %ld", path, i + 1, nvn);

    // Material table: [0] = default, then one entry per .mtl material (its Kd).
    std::vector<float> kd_all(3, 1.0f);
    kd_all.insert(kd_all.end(), kd.begin(), kd.end());
    std::vector<float> ke_all(3, 0.0f);  // Ke (emission, not read by the reference)
    ke_all.insert(ke_all.end(), ke.begin(), ke.end());

    out->ntri = mat.size();
    out->nvert = pos.size() / 3;
    out->nnrm = nrm.size() / 3;
    out->ntc = tc.size() / 2;
    out->pos_tri = dup(pt);
    out->pos = dup(pos);
    out->nrm_tri = dup(nt);
    out->nrm = dup(nrm);
    out->tc_tri = dup(tt);
    out->tc = dup(tc);
    out->mat_id = dup(mat);
    out->kd = dup(kd_all);
    out->ke = dup(ke_all);
    out->nmat = (uint32_t)(kd_all.size() / 3);
    return SPT_OK;
}

void spt_mesh_free(spt_mesh* m) {
    if (!m) return;
    std::free(m->pos_tri); std::free(m->pos); std::free(m->nrm_tri); std::free(m->nrm);
    std::free(m->tc_tri); std::free(m->tc); std::free(m->mat_id); std::free(m->kd);
    std::free(m->ke);
    std::memset(m, 0, sizeof(*m));
}

spt_status spt_pfm_write(const char* path, const float* r, const float* g, const float* b, uint32_t w, uint32_t h) {
    if (!path || !r || !g || !b) return spt_set_error(SPT_ERR_INVALID, "spt_pfm_write: NULL argument");
    FILE* f = std::fopen(path, "wb");
    if (!f) return spt_set_error(SPT_ERR_IO, "spt_pfm_write: cannot open %s: %s", path, std::strerror(errno));
    std::fprintf(f, "PF\n%u %u\n-1\n", w, h);
    std::vector<float> row((size_t)w * 3);
    for (uint32_t y = 0; y < h; y++) {
        const size_t src = (size_t)(h - y - 1) * w;  // rows bottom-up (fimage.h:46-55)
        for (uint32_t x = 0; x < w; x++) {
            row[x * 3] = r[src + x];
            row[x * 3 + 1] = g[src + x];
            row[x * 3 + 2] = b[src + x];
        }
        if (std::fwrite(row.data(), sizeof(float), row.size(), f) != row.size()) {
            std::fclose(f);
            return spt_set_error(SPT_ERR_IO, "spt_pfm_write: short write to %s", path);
        }
    }
    return std::fclose(f) == 0 ? SPT_OK : spt_set_error(SPT_ERR_IO, "spt_pfm_write: closing %s failed", path);
}

}  // extern "C"
