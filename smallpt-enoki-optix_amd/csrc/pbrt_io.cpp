// pbrt_io.cpp — a pbrt-v3 scene reader for the triangle path tracer.
//
// The reference lists ingowald/pbrt-parser as a submodule for San Miguel
// (.gitmodules:7-9; commented out at CMakeLists.txt:57-61,95) but the
// submodule is empty and no source calls it.  This is our own
// reader for the subset a triangle scene needs:
//
//   geometry   Shape "trianglemesh" (indices, P, N, uv/st), Shape "plymesh"
//              (ascii / binary little / big endian PLY; polygons fanned);
//              other shapes are counted as skipped
//   transforms Identity Translate Scale Rotate LookAt Transform
//              ConcatTransform CoordinateSystem CoordSysTransform;
//              AttributeBegin/End, TransformBegin/End; WorldBegin resets
//   instances  ObjectBegin/End + ObjectInstance (flattened)
//   materials  Material / MakeNamedMaterial / NamedMaterial: the diffuse
//              colour "Kd" (rgb, or a constant "rgb value" Texture), else
//              pbrt's matte default 0.5; AreaLightSource "diffuse" "rgb L"
//              ("float scale") becomes the emission of the shapes under it
//   camera     Camera "perspective" "float fov" with the CTM at that point,
//              Film "xresolution"/"yresolution"
//   sky        LightSource "infinite" "rgb L" (constant radiance)
//   Include    relative to the including file
//
// The output is the same spt_mesh the OBJ reader returns (material 0 is the
// default, shapes get their material index + 1, as main.cpp:185), plus an
// spt_pbrt_info with the camera, film size and sky.  Normals are transformed
// by the inverse transpose and not renormalised (pbrt-v3 stores them so).
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/spt.h"
#include "host_error.h"

namespace {

// ------------------------------------------------------------------ math
struct Mat4 {
    double m[4][4];
    static Mat4 identity() {
        Mat4 r;
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) r.m[i][j] = i == j ? 1.0 : 0.0;
        return r;
    }
    Mat4 operator*(const Mat4& b) const {
        Mat4 r;
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) {
                double s = 0.0;
                for (int k = 0; k < 4; k++) s += m[i][k] * b.m[k][j];
                r.m[i][j] = s;
            }
        return r;
    }
    bool is_identity() const {
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++)
                if (m[i][j] != (i == j ? 1.0 : 0.0)) return false;
        return true;
    }
    // Gauss-Jordan with partial pivoting; false if singular.
    bool inverse(Mat4& out) const {
        double a[4][8];
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 8; j++) a[i][j] = j < 4 ? m[i][j] : (j - 4 == i ? 1.0 : 0.0);
        for (int c = 0; c < 4; c++) {
            int p = c;
            for (int r = c + 1; r < 4; r++)
                if (std::fabs(a[r][c]) > std::fabs(a[p][c])) p = r;
            if (std::fabs(a[p][c]) < 1e-300) return false;
            for (int j = 0; j < 8; j++) std::swap(a[c][j], a[p][j]);
            const double inv = 1.0 / a[c][c];
            for (int j = 0; j < 8; j++) a[c][j] *= inv;
            for (int r = 0; r < 4; r++)
                if (r != c) {
                    const double f = a[r][c];
                    for (int j = 0; j < 8; j++) a[r][j] -= f * a[c][j];
                }
        }
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) out.m[i][j] = a[i][j + 4];
        return true;
    }
    void point(const double in[3], double out[3]) const {
        double w = m[3][0] * in[0] + m[3][1] * in[1] + m[3][2] * in[2] + m[3][3];
        for (int i = 0; i < 3; i++) out[i] = (m[i][0] * in[0] + m[i][1] * in[1] + m[i][2] * in[2] + m[i][3]) / w;
    }
    void vector(const double in[3], double out[3]) const {
        for (int i = 0; i < 3; i++) out[i] = m[i][0] * in[0] + m[i][1] * in[1] + m[i][2] * in[2];
    }
};

Mat4 translate(double x, double y, double z) {
    Mat4 r = Mat4::identity();
    r.m[0][3] = x; r.m[1][3] = y; r.m[2][3] = z;
    return r;
}
Mat4 scale(double x, double y, double z) {
    Mat4 r = Mat4::identity();
    r.m[0][0] = x; r.m[1][1] = y; r.m[2][2] = z;
    return r;
}
// pbrt-v3 Rotate(theta, axis) (transform.cpp): Rodrigues about the normalised axis.
Mat4 rotate(double deg, double x, double y, double z) {
    const double len = std::sqrt(x * x + y * y + z * z);
    Mat4 r = Mat4::identity();
    if (len == 0.0) return r;
    x /= len; y /= len; z /= len;
    const double th = deg * M_PI / 180.0, s = std::sin(th), c = std::cos(th);
    r.m[0][0] = x * x + (1 - x * x) * c; r.m[0][1] = x * y * (1 - c) - z * s; r.m[0][2] = x * z * (1 - c) + y * s;
    r.m[1][0] = x * y * (1 - c) + z * s; r.m[1][1] = y * y + (1 - y * y) * c; r.m[1][2] = y * z * (1 - c) - x * s;
    r.m[2][0] = x * z * (1 - c) - y * s; r.m[2][1] = y * z * (1 - c) + x * s; r.m[2][2] = z * z + (1 - z * z) * c;
    return r;
}
// pbrt-v3 LookAt: the world-to-camera matrix (camera looks down +z, +y up).
bool look_at(const double e[3], const double l[3], const double u[3], Mat4& out) {
    double dir[3] = {l[0] - e[0], l[1] - e[1], l[2] - e[2]};
    double dl = std::sqrt(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
    double ul = std::sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
    if (dl == 0.0 || ul == 0.0) return false;
    for (double& d : dir) d /= dl;
    const double un[3] = {u[0] / ul, u[1] / ul, u[2] / ul};
    double right[3] = {un[1] * dir[2] - un[2] * dir[1], un[2] * dir[0] - un[0] * dir[2], un[0] * dir[1] - un[1] * dir[0]};
    double rl = std::sqrt(right[0] * right[0] + right[1] * right[1] + right[2] * right[2]);
    if (rl == 0.0) return false;
    for (double& d : right) d /= rl;
    const double nu[3] = {dir[1] * right[2] - dir[2] * right[1], dir[2] * right[0] - dir[0] * right[2],
                          dir[0] * right[1] - dir[1] * right[0]};
    Mat4 c2w = Mat4::identity();
    for (int i = 0; i < 3; i++) {
        c2w.m[i][0] = right[i];
        c2w.m[i][1] = nu[i];
        c2w.m[i][2] = dir[i];
        c2w.m[i][3] = e[i];
    }
    return c2w.inverse(out);
}

// ----------------------------------------------------------------- lexer
struct Token {
    enum Kind { END, STRING, NUMBER, LBRACK, RBRACK, IDENT } kind = END;
    std::string s;
    double num = 0.0;
    int line = 0;
};

struct Source {
    std::string path, text;
    size_t pos = 0;
    int line = 1;
};

struct Lexer {
    std::vector<std::unique_ptr<Source>> stack;
    bool have_peek = false;
    Token peeked;

    bool open(const std::string& path) {
        FILE* f = std::fopen(path.c_str(), "rb");
        if (!f) return false;
        auto src = std::make_unique<Source>();
        src->path = path;
        char buf[1 << 16];
        size_t n;
        while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) src->text.append(buf, n);
        std::fclose(f);
        stack.push_back(std::move(src));
        return true;
    }
    std::string where() const {
        if (stack.empty()) return "end of input";
        return stack.back()->path + ":" + std::to_string(stack.back()->line);
    }
    std::string dir() const {
        if (stack.empty()) return "";
        const std::string& p = stack.back()->path;
        size_t s = p.find_last_of('/');
        return s == std::string::npos ? std::string() : p.substr(0, s + 1);
    }
    Token raw() {
        while (!stack.empty()) {
            Source& s = *stack.back();
            const std::string& t = s.text;
            while (s.pos < t.size()) {
                const char c = t[s.pos];
                if (c == '\n') { s.line++; s.pos++; continue; }
                if (c == ' ' || c == '\t' || c == '\r') { s.pos++; continue; }
                if (c == '#') {
                    while (s.pos < t.size() && t[s.pos] != '\n') s.pos++;
                    continue;
                }
                Token tok;
                tok.line = s.line;
                if (c == '[') { s.pos++; tok.kind = Token::LBRACK; return tok; }
                if (c == ']') { s.pos++; tok.kind = Token::RBRACK; return tok; }
                if (c == '"') {
                    size_t e = t.find('"', s.pos + 1);
                    if (e == std::string::npos) {
                        tok.kind = Token::END;
                        tok.s = "unterminated string";
                        s.pos = t.size();
                        return tok;
                    }
                    tok.kind = Token::STRING;
                    tok.s = t.substr(s.pos + 1, e - s.pos - 1);
                    for (char ch : tok.s) s.line += ch == '\n';
                    s.pos = e + 1;
                    return tok;
                }
                size_t e = s.pos;
                while (e < t.size() && !std::strchr(" \t\r\n[]\"#", t[e])) e++;
                tok.s = t.substr(s.pos, e - s.pos);
                s.pos = e;
                char* end = nullptr;
                tok.num = std::strtod(tok.s.c_str(), &end);
                tok.kind = (end && *end == '\0' && !tok.s.empty()) ? Token::NUMBER : Token::IDENT;
                return tok;
            }
            stack.pop_back();
        }
        return Token();
    }
    Token next() {
        if (have_peek) { have_peek = false; return peeked; }
        return raw();
    }
    const Token& peek() {
        if (!have_peek) { peeked = raw(); have_peek = true; }
        return peeked;
    }
};

// ------------------------------------------------------------ parameters
struct Param {
    std::string type, name;
    std::vector<double> nums;
    std::vector<std::string> strs;
};

struct ParamList {
    std::vector<Param> ps;
    const Param* find(const char* name) const {
        for (const Param& p : ps)
            if (p.name == name) return &p;
        return nullptr;
    }
    const Param* find_typed(const char* name, const char* type) const {
        for (const Param& p : ps)
            if (p.name == name && p.type == type) return &p;
        return nullptr;
    }
    double num(const char* name, double dflt) const {
        const Param* p = find(name);
        return p && !p->nums.empty() ? p->nums[0] : dflt;
    }
    std::string str(const char* name, const std::string& dflt) const {
        const Param* p = find(name);
        return p && !p->strs.empty() ? p->strs[0] : dflt;
    }
};

struct Material {
    float kd[3] = {0.5f, 0.5f, 0.5f};
};

struct Chunk {  // triangles of one shape, world space (or object space inside ObjectBegin)
    std::vector<double> p, n, uv;  // per vertex
    std::vector<int32_t> idx;      // 3 per triangle
    int32_t mat = 0;               // output material index (0 = default)
};

struct GState {
    Mat4 ctm = Mat4::identity();
    int material = -1;   // index into mats, -1 = default
    bool has_le = false;
    float le[3] = {0, 0, 0};
};

class Parser {
  public:
    Lexer lex;
    std::string err;
    GState gs;
    std::vector<GState> attr_stack;
    std::vector<Mat4> xform_stack;
    std::map<std::string, Mat4> coord_sys;
    std::vector<Material> mats;                 // parsed materials
    std::map<std::string, int> named_mats;
    std::map<std::string, float> tex_gray;      // constant float textures
    std::map<std::string, std::vector<float>> tex_rgb;  // constant rgb textures
    // output material table: [0] default (albedo 1, no emission, as main.cpp:234)
    std::vector<float> out_kd{1.0f, 1.0f, 1.0f}, out_ke{0.0f, 0.0f, 0.0f};
    std::map<std::string, int32_t> out_key;      // (material, Le) -> output index
    std::vector<float> pos, nrm, tc;
    std::vector<int32_t> pt, nt, tt, mat;
    std::map<std::string, std::vector<Chunk>> objects;
    std::vector<Chunk>* cur_object = nullptr;
    spt_pbrt_info info{};

    bool fail(const char* fmt, ...) {
        char buf[768];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        err = lex.where() + ": " + buf;
        return false;
    }

    bool numbers(int count, double* out) {
        for (int i = 0; i < count; i++) {
            Token t = lex.next();
            if (t.kind != Token::NUMBER) return fail("expected a number, got '%s'", t.s.c_str());
            out[i] = t.num;
        }
        return true;
    }

    bool params(ParamList& pl) {
        while (lex.peek().kind == Token::STRING) {
            Token decl = lex.next();
            Param p;
            const std::string& d = decl.s;
            size_t sp = d.find_first_of(" \t");
            if (sp == std::string::npos) return fail("parameter '%s' has no type", d.c_str());
            p.type = d.substr(0, sp);
            size_t ns = d.find_first_not_of(" \t", sp);
            p.name = ns == std::string::npos ? std::string() : d.substr(ns);
            while (!p.name.empty() && (p.name.back() == ' ' || p.name.back() == '\t')) p.name.pop_back();
            auto value = [&](const Token& t) -> bool {
                if (t.kind == Token::NUMBER) p.nums.push_back(t.num);
                else if (t.kind == Token::STRING) p.strs.push_back(t.s);
                else if (t.kind == Token::IDENT && (t.s == "true" || t.s == "false")) p.strs.push_back(t.s);
                else return fail("bad value for parameter '%s'", d.c_str());
                return true;
            };
            Token v = lex.next();
            if (v.kind == Token::LBRACK) {
                while (true) {
                    Token x = lex.next();
                    if (x.kind == Token::RBRACK) break;
                    if (x.kind == Token::END) return fail("unterminated '[' in parameter '%s'", d.c_str());
                    if (!value(x)) return false;
                }
            } else if (!value(v)) {
                return false;
            }
            pl.ps.push_back(std::move(p));
        }
        return true;
    }

    // Kd of a material's parameters: rgb, a constant texture, else 0.5.
    void material_kd(const ParamList& pl, Material& m) {
        const Param* kd = pl.find("Kd");
        if (!kd) return;
        if ((kd->type == "rgb" || kd->type == "color") && kd->nums.size() >= 3) {
            for (int c = 0; c < 3; c++) m.kd[c] = (float)kd->nums[c];
        } else if (kd->type == "float" && !kd->nums.empty()) {
            for (int c = 0; c < 3; c++) m.kd[c] = (float)kd->nums[0];
        } else if (kd->type == "texture" && !kd->strs.empty()) {
            auto it = tex_rgb.find(kd->strs[0]);
            if (it != tex_rgb.end())
                for (int c = 0; c < 3; c++) m.kd[c] = it->second[c];
            auto ig = tex_gray.find(kd->strs[0]);
            if (ig != tex_gray.end())
                for (int c = 0; c < 3; c++) m.kd[c] = ig->second;
        }
    }

    int32_t output_material() {
        if (gs.material < 0 && !gs.has_le) return 0;
        char key[128];
        std::snprintf(key, sizeof(key), "%d|%d|%.9g|%.9g|%.9g", gs.material, (int)gs.has_le, gs.le[0], gs.le[1],
                      gs.le[2]);
        auto it = out_key.find(key);
        if (it != out_key.end()) return it->second;
        const int32_t id = (int32_t)(out_kd.size() / 3);
        const Material m = gs.material >= 0 ? mats[gs.material] : Material();
        for (int c = 0; c < 3; c++) {
            out_kd.push_back(gs.material >= 0 ? m.kd[c] : 1.0f);
            out_ke.push_back(gs.has_le ? gs.le[c] : 0.0f);
        }
        out_key[key] = id;
        return id;
    }

    // Append a chunk transformed by M (normals by the inverse transpose).
    bool emit(const Chunk& c, const Mat4& M) {
        Mat4 inv;
        const bool ident = M.is_identity();
        if (!ident && !M.inverse(inv)) return fail("singular transform");
        const size_t nv = c.p.size() / 3;
        const int32_t vbase = (int32_t)(pos.size() / 3), nbase = (int32_t)(nrm.size() / 3),
                      tbase = (int32_t)(tc.size() / 2);
        if ((uint64_t)vbase + nv >= (1ull << 31)) return fail("more than 2^31 vertices");
        for (size_t i = 0; i < nv; i++) {
            double q[3];
            if (ident) { q[0] = c.p[i * 3]; q[1] = c.p[i * 3 + 1]; q[2] = c.p[i * 3 + 2]; }
            else M.point(&c.p[i * 3], q);
            for (int k = 0; k < 3; k++) pos.push_back((float)q[k]);
        }
        const bool hn = c.n.size() == c.p.size(), ht = c.uv.size() == nv * 2;
        if (hn)
            for (size_t i = 0; i < nv; i++) {
                double q[3];
                if (ident) { q[0] = c.n[i * 3]; q[1] = c.n[i * 3 + 1]; q[2] = c.n[i * 3 + 2]; }
                else
                    for (int r = 0; r < 3; r++)  // (M^-1)^T n
                        q[r] = inv.m[0][r] * c.n[i * 3] + inv.m[1][r] * c.n[i * 3 + 1] + inv.m[2][r] * c.n[i * 3 + 2];
                for (int k = 0; k < 3; k++) nrm.push_back((float)q[k]);
            }
        if (ht)
            for (size_t i = 0; i < nv * 2; i++) tc.push_back((float)c.uv[i]);
        for (size_t t = 0; t + 2 < c.idx.size(); t += 3) {
            for (int k = 0; k < 3; k++) {
                const int32_t v = c.idx[t + k];
                pt.push_back(vbase + v);
                nt.push_back(hn ? nbase + v : -1);
                tt.push_back(ht ? tbase + v : -1);
            }
            mat.push_back(c.mat);
        }
        return true;
    }

    bool add_shape(Chunk&& c) {
        const size_t nv = c.p.size() / 3;
        if (c.idx.size() % 3) return fail("triangle index count %zu is not a multiple of 3", c.idx.size());
        for (int32_t v : c.idx)
            if (v < 0 || (size_t)v >= nv) return fail("vertex index %d out of range [0,%zu)", v, nv);
        c.mat = output_material();
        info.shapes++;
        if (cur_object) {
            // object space = the CTM at definition (flattened at instancing)
            Chunk w = c;
            const Mat4& M = gs.ctm;
            if (!M.is_identity()) {
                Mat4 inv;
                if (!M.inverse(inv)) return fail("singular transform");
                for (size_t i = 0; i < nv; i++) M.point(&c.p[i * 3], &w.p[i * 3]);
                if (c.n.size() == c.p.size())
                    for (size_t i = 0; i < nv; i++)
                        for (int r = 0; r < 3; r++)
                            w.n[i * 3 + r] = inv.m[0][r] * c.n[i * 3] + inv.m[1][r] * c.n[i * 3 + 1] +
                                             inv.m[2][r] * c.n[i * 3 + 2];
            }
            cur_object->push_back(std::move(w));
            return true;
        }
        return emit(c, gs.ctm);
    }

    bool read_ply(const std::string& path, Chunk& c);

    bool shape() {
        Token t = lex.next();
        if (t.kind != Token::STRING) return fail("Shape needs a type string");
        ParamList pl;
        if (!params(pl)) return false;
        Chunk c;
        if (t.s == "trianglemesh") {
            const Param* P = pl.find("P");
            const Param* I = pl.find("indices");
            if (!P || P->nums.size() % 3) return fail("trianglemesh needs \"point P\"");
            c.p = P->nums;
            if (I) {
                for (double v : I->nums) {
                    // -1 is out of range for every mesh; UB-free for any double
                    c.idx.push_back(v >= -2147483648.0 && v < 2147483648.0 ? (int32_t)v : -1);
                }
            } else if (c.p.size() == 9) {
                c.idx = {0, 1, 2};
            } else {
                return fail("trianglemesh needs \"integer indices\"");
            }
            if (const Param* N = pl.find("N")) c.n = N->nums;
            const Param* uv = pl.find("uv");
            if (!uv) uv = pl.find("st");
            if (uv) c.uv = uv->nums;
        } else if (t.s == "plymesh") {
            const std::string f = pl.str("filename", "");
            if (f.empty()) return fail("plymesh needs \"string filename\"");
            const std::string full = (!f.empty() && f[0] == '/') ? f : lex.dir() + f;
            if (!read_ply(full, c)) return false;
        } else {
            info.shapes_skipped++;
            return true;
        }
        return add_shape(std::move(c));
    }

    bool run(const std::string& path) {
        if (!lex.open(path)) return fail("cannot open %s", path.c_str());
        info.fov_deg = 90.0f;  // pbrt-v3 perspective default
        info.xres = 640;
        info.yres = 480;
        while (true) {
            Token t = lex.next();
            if (t.kind == Token::END) {
                if (!t.s.empty()) return fail("%s", t.s.c_str());
                break;
            }
            if (t.kind != Token::IDENT) return fail("expected a directive, got '%s'", t.s.c_str());
            const std::string& d = t.s;
            double v[16];
            if (d == "AttributeBegin") {
                attr_stack.push_back(gs);
            } else if (d == "AttributeEnd") {
                if (attr_stack.empty()) return fail("unmatched AttributeEnd");
                gs = attr_stack.back();
                attr_stack.pop_back();
            } else if (d == "TransformBegin") {
                xform_stack.push_back(gs.ctm);
            } else if (d == "TransformEnd") {
                if (xform_stack.empty()) return fail("unmatched TransformEnd");
                gs.ctm = xform_stack.back();
                xform_stack.pop_back();
            } else if (d == "Identity") {
                gs.ctm = Mat4::identity();
            } else if (d == "Translate") {
                if (!numbers(3, v)) return false;
                gs.ctm = gs.ctm * translate(v[0], v[1], v[2]);
            } else if (d == "Scale") {
                if (!numbers(3, v)) return false;
                gs.ctm = gs.ctm * scale(v[0], v[1], v[2]);
            } else if (d == "Rotate") {
                if (!numbers(4, v)) return false;
                gs.ctm = gs.ctm * rotate(v[0], v[1], v[2], v[3]);
            } else if (d == "LookAt") {
                if (!numbers(9, v)) return false;
                Mat4 la;
                if (!look_at(v, v + 3, v + 6, la)) return fail("degenerate LookAt");
                gs.ctm = gs.ctm * la;
            } else if (d == "Transform" || d == "ConcatTransform") {
                const bool br = lex.peek().kind == Token::LBRACK;
                if (br) lex.next();
                if (!numbers(16, v)) return false;
                if (br && lex.next().kind != Token::RBRACK) return fail("expected ']' after 16 numbers");
                Mat4 m;  // given column-major (pbrt-v3 transposes)
                for (int i = 0; i < 4; i++)
                    for (int j = 0; j < 4; j++) m.m[i][j] = v[j * 4 + i];
                gs.ctm = d == "Transform" ? m : gs.ctm * m;
            } else if (d == "CoordinateSystem" || d == "CoordSysTransform") {
                Token n = lex.next();
                if (n.kind != Token::STRING) return fail("%s needs a name", d.c_str());
                if (d == "CoordinateSystem") coord_sys[n.s] = gs.ctm;
                else if (coord_sys.count(n.s)) gs.ctm = coord_sys[n.s];
            } else if (d == "Camera") {
                Token n = lex.next();
                ParamList pl;
                if (n.kind != Token::STRING || !params(pl)) return err.empty() ? fail("Camera needs a type") : false;
                Mat4 c2w;
                if (!gs.ctm.inverse(c2w)) return fail("singular camera transform");
                const double o[3] = {0, 0, 0}, z[3] = {0, 0, 1}, y[3] = {0, 1, 0};
                double from[3], fwd[3], up[3];
                c2w.point(o, from);
                c2w.vector(z, fwd);
                c2w.vector(y, up);
                for (int k = 0; k < 3; k++) {
                    info.camera.look_from[k] = (float)from[k];
                    info.camera.look_at[k] = (float)(from[k] + fwd[k]);
                    info.camera.up[k] = (float)up[k];
                }
                info.fov_deg = (float)pl.num("fov", 90.0);
                info.camera.lens_radius = (float)pl.num("lensradius", 0.0);
                info.camera.focal_dist = (float)pl.num("focaldistance", 1.0);
                info.camera.film_size_y = 0.035f;
                info.has_camera = 1;
                coord_sys["camera"] = c2w;
            } else if (d == "Film") {
                Token n = lex.next();
                ParamList pl;
                if (n.kind != Token::STRING || !params(pl)) return err.empty() ? fail("Film needs a type") : false;
                const double xr = pl.num("xresolution", 640), yr = pl.num("yresolution", 480);
                if (!(xr >= 1.0 && xr <= 1048576.0 && yr >= 1.0 && yr <= 1048576.0))
                    return fail("Film resolution %g x %g outside [1, 2^20]", xr, yr);
                info.xres = (uint32_t)xr;
                info.yres = (uint32_t)yr;
            } else if (d == "WorldBegin") {
                gs.ctm = Mat4::identity();
                coord_sys["world"] = gs.ctm;
            } else if (d == "WorldEnd") {
            } else if (d == "Material" || d == "MakeNamedMaterial") {
                std::string name;
                if (d == "MakeNamedMaterial") {
                    Token n = lex.next();
                    if (n.kind != Token::STRING) return fail("MakeNamedMaterial needs a name");
                    name = n.s;
                } else {
                    Token n = lex.next();
                    if (n.kind != Token::STRING) return fail("Material needs a type");
                }
                ParamList pl;
                if (!params(pl)) return false;
                Material m;
                material_kd(pl, m);
                mats.push_back(m);
                if (d == "MakeNamedMaterial") named_mats[name] = (int)mats.size() - 1;
                else gs.material = (int)mats.size() - 1;
            } else if (d == "NamedMaterial") {
                Token n = lex.next();
                if (n.kind != Token::STRING) return fail("NamedMaterial needs a name");
                auto it = named_mats.find(n.s);
                if (it == named_mats.end()) return fail("unknown named material '%s'", n.s.c_str());
                gs.material = it->second;
            } else if (d == "Texture") {
                Token n = lex.next(), ty = lex.next(), cls = lex.next();
                ParamList pl;
                if (n.kind != Token::STRING || ty.kind != Token::STRING || cls.kind != Token::STRING || !params(pl))
                    return err.empty() ? fail("Texture needs name, type and class") : false;
                if (cls.s == "constant") {
                    const Param* val = pl.find("value");
                    if (val && val->nums.size() >= 3)
                        tex_rgb[n.s] = {(float)val->nums[0], (float)val->nums[1], (float)val->nums[2]};
                    else if (val && !val->nums.empty())
                        tex_gray[n.s] = (float)val->nums[0];
                }
            } else if (d == "AreaLightSource") {
                Token n = lex.next();
                ParamList pl;
                if (n.kind != Token::STRING || !params(pl)) return err.empty() ? fail("AreaLightSource needs a type") : false;
                const Param* L = pl.find("L");
                const double sc = pl.num("scale", 1.0);
                gs.has_le = true;
                for (int c = 0; c < 3; c++)
                    gs.le[c] = (float)(sc * (L && L->nums.size() >= 3 ? L->nums[c] : (L && !L->nums.empty() ? L->nums[0] : 1.0)));
            } else if (d == "LightSource") {
                Token n = lex.next();
                ParamList pl;
                if (n.kind != Token::STRING || !params(pl)) return err.empty() ? fail("LightSource needs a type") : false;
                if (n.s == "infinite") {
                    const Param* L = pl.find("L");
                    const double sc = pl.num("scale", 1.0);
                    info.has_env = 1;
                    for (int c = 0; c < 3; c++)
                        info.env[c] = (float)(sc * (L && L->nums.size() >= 3 ? L->nums[c] : 1.0));
                }
            } else if (d == "Shape") {
                if (!shape()) return false;
            } else if (d == "ObjectBegin") {
                Token n = lex.next();
                if (n.kind != Token::STRING) return fail("ObjectBegin needs a name");
                attr_stack.push_back(gs);
                cur_object = &objects[n.s];
            } else if (d == "ObjectEnd") {
                if (!cur_object) return fail("ObjectEnd without ObjectBegin");
                cur_object = nullptr;
                if (!attr_stack.empty()) {
                    gs = attr_stack.back();
                    attr_stack.pop_back();
                }
            } else if (d == "ObjectInstance") {
                Token n = lex.next();
                if (n.kind != Token::STRING) return fail("ObjectInstance needs a name");
                auto it = objects.find(n.s);
                if (it == objects.end()) return fail("unknown object '%s'", n.s.c_str());
                info.instances++;
                for (const Chunk& c : it->second)
                    if (!emit(c, gs.ctm)) return false;
            } else if (d == "Include" || d == "Import") {
                Token n = lex.next();
                if (n.kind != Token::STRING) return fail("Include needs a file name");
                const std::string full = (!n.s.empty() && n.s[0] == '/') ? n.s : lex.dir() + n.s;
                if (!lex.open(full)) return fail("cannot open included file %s", full.c_str());
            } else if (d == "ReverseOrientation" || d == "ActiveTransform" || d == "TransformTimes") {
                // no effect on a two-sided Lambertian scene; consume arguments
                if (d == "ActiveTransform") lex.next();
                if (d == "TransformTimes" && !numbers(2, v)) return false;
            } else if (d == "Sampler" || d == "Integrator" || d == "PixelFilter" || d == "Accelerator" ||
                       d == "SurfaceIntegrator" || d == "VolumeIntegrator" || d == "Renderer" ||
                       d == "MakeNamedMedium" || d == "ColorSpace" || d == "Option") {
                Token n = lex.next();
                ParamList pl;
                if (n.kind != Token::STRING || !params(pl)) return err.empty() ? fail("%s needs a type", d.c_str()) : false;
            } else if (d == "MediumInterface") {
                lex.next();
                if (lex.peek().kind == Token::STRING) lex.next();
            } else {
                return fail("unsupported directive '%s'", d.c_str());
            }
        }
        if (!attr_stack.empty()) return fail("%zu AttributeBegin without AttributeEnd", attr_stack.size());
        // pbrt's fov spans the shorter image axis; spt_camera.fov_y is vertical
        double fy = info.fov_deg * M_PI / 180.0;
        if (info.xres < info.yres && info.yres > 0)
            fy = 2.0 * std::atan(std::tan(0.5 * fy) * (double)info.yres / (double)info.xres);
        info.camera.fov_y = (float)fy;
        return true;
    }
};

// ------------------------------------------------------------------- PLY
template <typename T>
T swap_bytes(T v) {
    unsigned char b[sizeof(T)];
    std::memcpy(b, &v, sizeof(T));
    for (size_t i = 0; i < sizeof(T) / 2; i++) std::swap(b[i], b[sizeof(T) - 1 - i]);
    std::memcpy(&v, b, sizeof(T));
    return v;
}

enum PlyType { P_NONE, P_I8, P_U8, P_I16, P_U16, P_I32, P_U32, P_F32, P_F64 };
PlyType ply_type(const std::string& s) {
    if (s == "char" || s == "int8") return P_I8;
    if (s == "uchar" || s == "uint8") return P_U8;
    if (s == "short" || s == "int16") return P_I16;
    if (s == "ushort" || s == "uint16") return P_U16;
    if (s == "int" || s == "int32") return P_I32;
    if (s == "uint" || s == "uint32") return P_U32;
    if (s == "float" || s == "float32") return P_F32;
    if (s == "double" || s == "float64") return P_F64;
    return P_NONE;
}

struct PlyProp {
    std::string name;
    PlyType type = P_NONE, count_type = P_NONE;  // count_type != NONE: list
};
struct PlyElem {
    std::string name;
    uint64_t count = 0;
    std::vector<PlyProp> props;
};

struct PlyReader {
    const unsigned char* p;
    const unsigned char* end;
    int fmt;  // 0 ascii, 1 little, 2 big
    bool ok = true;

    double ascii_num() {
        while (p < end && (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n')) p++;
        if (p >= end) { ok = false; return 0.0; }
        char buf[64];
        size_t n = 0;
        while (p < end && n < sizeof(buf) - 1 && !(*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n')) buf[n++] = (char)*p++;
        buf[n] = 0;
        char* e = nullptr;
        double v = std::strtod(buf, &e);
        if (e == buf) ok = false;
        return v;
    }
    template <typename T>
    double bin() {
        if (p + sizeof(T) > end) { ok = false; p = end; return 0.0; }
        T v;
        std::memcpy(&v, p, sizeof(T));
        p += sizeof(T);
        if (fmt == 2) v = swap_bytes(v);
        return (double)v;
    }
    double read(PlyType t) {
        if (fmt == 0) return ascii_num();
        switch (t) {
            case P_I8: return bin<int8_t>();
            case P_U8: return bin<uint8_t>();
            case P_I16: return bin<int16_t>();
            case P_U16: return bin<uint16_t>();
            case P_I32: return bin<int32_t>();
            case P_U32: return bin<uint32_t>();
            case P_F32: return bin<float>();
            case P_F64: return bin<double>();
            default: ok = false; return 0.0;
        }
    }
};

bool Parser::read_ply(const std::string& path, Chunk& c) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return fail("cannot open PLY %s", path.c_str());
    std::string data;
    {
        char buf[1 << 16];
        size_t n;
        while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) data.append(buf, n);
        std::fclose(f);
    }
    size_t hdr_end = data.find("end_header");
    if (data.compare(0, 3, "ply") != 0 || hdr_end == std::string::npos) return fail("%s: not a PLY file", path.c_str());
    size_t body = data.find('\n', hdr_end);
    if (body == std::string::npos) return fail("%s: truncated header", path.c_str());
    body++;
    // header
    std::vector<PlyElem> elems;
    int fmt = -1;
    size_t lp = 0;
    while (lp < hdr_end) {
        size_t le = data.find('\n', lp);
        std::string line = data.substr(lp, le - lp);
        lp = le + 1;
        while (!line.empty() && (line.back() == '\r' || line.back() == ' ')) line.pop_back();
        std::vector<std::string> w;
        size_t i = 0;
        while (i < line.size()) {
            while (i < line.size() && line[i] == ' ') i++;
            size_t j = i;
            while (j < line.size() && line[j] != ' ') j++;
            if (j > i) w.push_back(line.substr(i, j - i));
            i = j;
        }
        if (w.empty()) continue;
        if (w[0] == "format" && w.size() >= 2) {
            fmt = w[1] == "ascii" ? 0 : w[1] == "binary_little_endian" ? 1 : w[1] == "binary_big_endian" ? 2 : -1;
        } else if (w[0] == "element" && w.size() >= 3) {
            PlyElem e;
            e.name = w[1];
            e.count = std::strtoull(w[2].c_str(), nullptr, 10);
            elems.push_back(e);
        } else if (w[0] == "property" && !elems.empty()) {
            PlyProp pr;
            if (w.size() >= 5 && w[1] == "list") {
                pr.count_type = ply_type(w[2]);
                pr.type = ply_type(w[3]);
                pr.name = w[4];
                if (pr.count_type == P_NONE || pr.type == P_NONE) return fail("%s: bad list property", path.c_str());
            } else if (w.size() >= 3) {
                pr.type = ply_type(w[1]);
                pr.name = w[2];
                if (pr.type == P_NONE) return fail("%s: bad property type '%s'", path.c_str(), w[1].c_str());
            }
            elems.back().props.push_back(pr);
        }
    }
    if (fmt < 0) return fail("%s: unknown PLY format", path.c_str());
    PlyReader r{(const unsigned char*)data.data() + body, (const unsigned char*)data.data() + data.size(), fmt};
    for (const PlyElem& e : elems) {
        const bool vert = e.name == "vertex", face = e.name == "face";
        int ix[3] = {-1, -1, -1}, in[3] = {-1, -1, -1}, iu[2] = {-1, -1}, ilist = -1;
        for (size_t k = 0; k < e.props.size(); k++) {
            const std::string& n = e.props[k].name;
            if (n == "x") ix[0] = (int)k; else if (n == "y") ix[1] = (int)k; else if (n == "z") ix[2] = (int)k;
            else if (n == "nx") in[0] = (int)k; else if (n == "ny") in[1] = (int)k; else if (n == "nz") in[2] = (int)k;
            else if (n == "u" || n == "s" || n == "texture_u" || n == "texture_s") iu[0] = (int)k;
            else if (n == "v" || n == "t" || n == "texture_v" || n == "texture_t") iu[1] = (int)k;
            else if ((n == "vertex_indices" || n == "vertex_index") && e.props[k].count_type != P_NONE) ilist = (int)k;
        }
        if (vert && (ix[0] < 0 || ix[1] < 0 || ix[2] < 0)) return fail("%s: vertex element without x y z", path.c_str());
        const bool hn = vert && in[0] >= 0 && in[1] >= 0 && in[2] >= 0, hu = vert && iu[0] >= 0 && iu[1] >= 0;
        std::vector<double> vals(e.props.size());
        std::vector<int32_t> poly;
        for (uint64_t i = 0; i < e.count && r.ok; i++) {
            for (size_t k = 0; k < e.props.size() && r.ok; k++) {
                const PlyProp& pr = e.props[k];
                if (pr.count_type == P_NONE) {
                    vals[k] = r.read(pr.type);
                    continue;
                }
                const double cnt = r.read(pr.count_type);
                if (cnt < 0 || cnt > 1e6) { r.ok = false; break; }
                if ((int)k == ilist) poly.clear();
                for (int64_t j = 0; j < (int64_t)cnt && r.ok; j++) {
                    const double x = r.read(pr.type);
                    if ((int)k == ilist) {
                        if (!(x >= -2147483648.0 && x < 2147483648.0)) { r.ok = false; break; }
                        poly.push_back((int32_t)x);
                    }
                }
            }
            if (!r.ok) break;
            if (vert) {
                for (int a = 0; a < 3; a++) c.p.push_back(vals[ix[a]]);
                if (hn)
                    for (int a = 0; a < 3; a++) c.n.push_back(vals[in[a]]);
                if (hu) { c.uv.push_back(vals[iu[0]]); c.uv.push_back(vals[iu[1]]); }
            } else if (face && ilist >= 0) {
                for (size_t k = 1; k + 1 < poly.size(); k++) {  // fan, as the OBJ reader
                    c.idx.push_back(poly[0]);
                    c.idx.push_back(poly[k]);
                    c.idx.push_back(poly[k + 1]);
                }
            }
        }
        if (!r.ok) return fail("%s: truncated or malformed %s data", path.c_str(), e.name.c_str());
    }
    return true;
}

template <typename T>
T* dup(const std::vector<T>& v) {
    if (v.empty()) return nullptr;
    T* p = (T*)std::malloc(sizeof(T) * v.size());
    if (p) std::memcpy(p, v.data(), sizeof(T) * v.size());
    return p;
}

}  // namespace

extern "C" spt_status spt_pbrt_load(const char* path, spt_mesh* out, spt_pbrt_info* info) {
    if (!path || !out) return spt_set_error(SPT_ERR_INVALID, "spt_pbrt_load: NULL argument");
    std::memset(out, 0, sizeof(*out));
    if (info) std::memset(info, 0, sizeof(*info));
    Parser ps;
    if (!ps.run(path)) {
        const bool io = ps.err.find("cannot open") != std::string::npos;
        return spt_set_error(io ? SPT_ERR_IO : SPT_ERR_INVALID, "spt_pbrt_load: %s", ps.err.c_str());
    }
    out->ntri = ps.mat.size();
    out->nvert = ps.pos.size() / 3;
    out->nnrm = ps.nrm.size() / 3;
    out->ntc = ps.tc.size() / 2;
    out->pos_tri = dup(ps.pt);
    out->pos = dup(ps.pos);
    out->nrm_tri = dup(ps.nt);
    out->nrm = dup(ps.nrm);
    out->tc_tri = dup(ps.tt);
    out->tc = dup(ps.tc);
    out->mat_id = dup(ps.mat);
    out->kd = dup(ps.out_kd);
    out->ke = dup(ps.out_ke);
    out->nmat = (uint32_t)(ps.out_kd.size() / 3);
    if (info) *info = ps.info;
    return SPT_OK;
}
