// scene.cpp — C++ restatement of the reference's scene loader (host side of libmirt).
//
//   shared/state/environment.go:162-234 EnvironmentFromFile: objects get id i+1 and
//       share one mesh per distinct model path; lights Col = NewRGB(u8)/255; camera via
//       NewCamera.  Mesh path tried relative to the scene file, then as given.
//   shared/state/mesh.go:109-213 MeshFromFile: float32 coordinates widened to fp64,
//       vertices deduplicated by exact value, vertex normals deduplicated by their
//       un-normalised value and stored normalised, one material per `usemtl` group
//       (MTL Ka/Kd/Ks float32 clamped to [0,1], Ns = float64(f32)), default material
//       Ka=16/255, Kd=1, Ks=0, Ns=0 when the group's material is unknown.
//   shared/state/util.go:11-13 relativePath.
// gwob semantics assumed (github.com/mwindels/gwob is unpinned and not vendored):
// polygons are fan-triangulated (v0, vi, vi+1); numbers parse as float32 (ParseFloat(s, 32)).
// Go's encoding/json matches keys to struct fields case-insensitively.
#include <ctype.h>
#include <strings.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/mirt_scene.h"
#include "gob.hpp"

namespace {

thread_local std::string g_scene_err;

// ------------------------------------------------------------------ tiny JSON
struct JVal {
    enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
    double num = 0;
    bool b = false;
    std::string str;
    std::vector<JVal> arr;
    std::vector<std::pair<std::string, JVal>> obj;

    const JVal* get(const char* key) const {  // case-insensitive, first match (Go json)
        if (kind != Obj) return nullptr;
        for (auto& kv : obj)
            if (strcasecmp(kv.first.c_str(), key) == 0) return &kv.second;
        return nullptr;
    }
};

struct JParser {
    const char* p;
    const char* end;
    std::string err;

    void ws() {
        while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
    }
    bool parse(JVal& v) {
        ws();
        if (p >= end) return fail("unexpected end");
        char c = *p;
        if (c == '{') return object(v);
        if (c == '[') return array(v);
        if (c == '"') {
            v.kind = JVal::Str;
            return string(v.str);
        }
        if (!strncmp(p, "true", std::min<size_t>(4, end - p)) && end - p >= 4) {
            v.kind = JVal::Bool;
            v.b = true;
            p += 4;
            return true;
        }
        if (!strncmp(p, "false", std::min<size_t>(5, end - p)) && end - p >= 5) {
            v.kind = JVal::Bool;
            p += 5;
            return true;
        }
        if (!strncmp(p, "null", std::min<size_t>(4, end - p)) && end - p >= 4) {
            v.kind = JVal::Null;
            p += 4;
            return true;
        }
        return number(v);
    }
    bool fail(const char* m) {
        err = m;
        return false;
    }
    bool number(JVal& v) {
        std::string s;
        while (p < end && (isdigit((unsigned char)*p) || *p == '-' || *p == '+' || *p == '.' || *p == 'e' || *p == 'E'))
            s += *p++;
        if (s.empty()) return fail("bad value");
        char* e = nullptr;
        v.num = strtod(s.c_str(), &e);  // correctly rounded, as Go's strconv.ParseFloat
        if (!e || *e) return fail("bad number");
        v.kind = JVal::Num;
        return true;
    }
    bool string(std::string& out) {
        ++p;
        while (p < end && *p != '"') {
            if (*p == '\\') {
                ++p;
                if (p >= end) return fail("bad escape");
                char e = *p++;
                switch (e) {
                    case 'n': out += '\n'; break;
                    case 't': out += '\t'; break;
                    case 'r': out += '\r'; break;
                    case 'b': out += '\b'; break;
                    case 'f': out += '\f'; break;
                    case 'u': {
                        if (end - p < 4) return fail("bad \\u");
                        unsigned cp = (unsigned)strtoul(std::string(p, 4).c_str(), nullptr, 16);
                        p += 4;
                        if (cp < 0x80) out += (char)cp;
                        else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
                        else { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
                        break;
                    }
                    default: out += e;
                }
            } else {
                out += *p++;
            }
        }
        if (p >= end) return fail("unterminated string");
        ++p;
        return true;
    }
    bool array(JVal& v) {
        v.kind = JVal::Arr;
        ++p;
        ws();
        if (p < end && *p == ']') { ++p; return true; }
        for (;;) {
            JVal e;
            if (!parse(e)) return false;
            v.arr.push_back(std::move(e));
            ws();
            if (p < end && *p == ',') { ++p; continue; }
            if (p < end && *p == ']') { ++p; return true; }
            return fail("expected , or ]");
        }
    }
    bool object(JVal& v) {
        v.kind = JVal::Obj;
        ++p;
        ws();
        if (p < end && *p == '}') { ++p; return true; }
        for (;;) {
            ws();
            if (p >= end || *p != '"') return fail("expected key");
            std::string k;
            if (!string(k)) return false;
            ws();
            if (p >= end || *p != ':') return fail("expected :");
            ++p;
            JVal e;
            if (!parse(e)) return false;
            v.obj.emplace_back(std::move(k), std::move(e));
            ws();
            if (p < end && *p == ',') { ++p; continue; }
            if (p < end && *p == '}') { ++p; return true; }
            return fail("expected , or }");
        }
    }
};

double jnum(const JVal* v) { return (v && v->kind == JVal::Num) ? v->num : 0.0; }
void jvec(const JVal* v, double out[3]) {
    out[0] = jnum(v ? v->get("x") : nullptr);
    out[1] = jnum(v ? v->get("y") : nullptr);
    out[2] = jnum(v ? v->get("z") : nullptr);
}

bool read_file(const std::string& path, std::string& out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::stringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

// util.go:11-13
std::string relative_path(const std::string& original, const std::string& other) {
    size_t i = original.size();
    while (i > 0 && original[i - 1] != '/' && original[i - 1] != '\\') --i;
    size_t j = 0;
    while (j < other.size() && (other[j] == '/' || other[j] == '\\')) ++j;
    return original.substr(0, i) + other.substr(j);
}

// gwob: strconv.ParseFloat(s, 32), the decimal rounded once, correctly, to float32 (glibc's
// strtof rounds correctly; (float)strtod would round twice and differ near float32
// halfway points), widened to fp64.
double f32(const std::string& s, bool& ok) {
    char* e = nullptr;
    const float f = strtof(s.c_str(), &e);
    ok = e && !*e && !s.empty();
    return (double)f;
}
double clamp01(double v) {  // colour.go:33-35 Max(0, Min(v, 1)) (NaN propagates)
    if (v != v) return v;
    return v < 0 ? 0.0 : (v > 1 ? 1.0 : v);
}

struct Mtl {
    double ka[3] = {0, 0, 0}, kd[3] = {0, 0, 0}, ks[3] = {0, 0, 0};
    double ns = 0;
};

bool parse_mtl(const std::string& path, std::map<std::string, Mtl>& lib) {
    std::string text;
    if (!read_file(path, text)) return false;
    std::istringstream in(text);
    std::string line;
    Mtl* cur = nullptr;
    while (std::getline(in, line)) {
        std::istringstream ls(line);
        std::string tag;
        if (!(ls >> tag) || tag[0] == '#') continue;
        if (tag == "newmtl") {
            std::string name, w;
            while (ls >> w) name += (name.empty() ? "" : " ") + w;
            cur = &lib[name];
            *cur = Mtl();
        } else if (cur && (tag == "Ka" || tag == "Kd" || tag == "Ks")) {
            double* dst = tag == "Ka" ? cur->ka : (tag == "Kd" ? cur->kd : cur->ks);
            for (int k = 0; k < 3; ++k) {
                std::string w;
                bool ok = false;
                if (ls >> w) dst[k] = f32(w, ok);
            }
        } else if (cur && tag == "Ns") {
            std::string w;
            bool ok = false;
            if (ls >> w) cur->ns = f32(w, ok);
        }
    }
    return true;
}

struct MeshData {
    std::vector<double> v, vn;
    std::vector<uint32_t> fv, fn, fmat;
    std::vector<mirt_material> mats;
};

struct VKey {
    double x, y, z;
    bool operator<(const VKey& o) const {
        // map key with Go's == semantics for finite values (-0 == +0)
        double a[3] = {x == 0 ? 0.0 : x, y == 0 ? 0.0 : y, z == 0 ? 0.0 : z};
        double b[3] = {o.x == 0 ? 0.0 : o.x, o.y == 0 ? 0.0 : o.y, o.z == 0 ? 0.0 : o.z};
        return std::tie(a[0], a[1], a[2]) < std::tie(b[0], b[1], b[2]);
    }
};

int resolve(long i, size_t count) { return i > 0 ? (int)(i - 1) : (int)((long)count + i); }

bool load_mesh(const std::string& path, MeshData& m, std::string& err) {
    std::string text;
    if (!read_file(path, text)) {
        err = "cannot read OBJ " + path;
        return false;
    }
    std::vector<std::array<double, 3>> pos, nrm;
    std::string mtllib, cur_mtl;
    struct Tri { int v[3], n[3]; std::string mtl; };
    std::vector<Tri> tris;
    std::istringstream in(text);
    std::string line;
    size_t lineno = 0;
    while (std::getline(in, line)) {
        ++lineno;
        std::istringstream ls(line);
        std::string tag;
        if (!(ls >> tag) || tag[0] == '#') continue;
        if (tag == "v" || tag == "vn") {
            std::array<double, 3> a{0, 0, 0};
            for (int k = 0; k < 3; ++k) {
                std::string w;
                bool ok = false;
                if (!(ls >> w) || (a[k] = f32(w, ok), !ok)) {
                    err = path + ":" + std::to_string(lineno) + ": bad coordinate";
                    return false;
                }
            }
            (tag == "v" ? pos : nrm).push_back(a);
        } else if (tag == "mtllib") {
            std::string w;
            mtllib.clear();
            while (ls >> w) mtllib += (mtllib.empty() ? "" : " ") + w;
        } else if (tag == "usemtl") {
            std::string w;
            cur_mtl.clear();
            while (ls >> w) cur_mtl += (cur_mtl.empty() ? "" : " ") + w;
        } else if (tag == "f") {
            std::vector<std::pair<int, int>> cs;
            std::string w;
            while (ls >> w) {
                int vi = -1, ni = -1;
                size_t s1 = w.find('/');
                vi = resolve(strtol(w.substr(0, s1).c_str(), nullptr, 10), pos.size());
                if (s1 != std::string::npos) {
                    size_t s2 = w.find('/', s1 + 1);
                    if (s2 != std::string::npos && s2 + 1 < w.size())
                        ni = resolve(strtol(w.substr(s2 + 1).c_str(), nullptr, 10), nrm.size());
                }
                if (vi < 0 || (size_t)vi >= pos.size()) {
                    err = path + ":" + std::to_string(lineno) + ": vertex index out of range";
                    return false;
                }
                if (ni >= 0 && (size_t)ni >= nrm.size()) {
                    err = path + ":" + std::to_string(lineno) + ": normal index out of range";
                    return false;
                }
                cs.emplace_back(vi, ni);
            }
            for (size_t k = 1; k + 1 < cs.size(); ++k) {  // fan triangulation (gwob)
                Tri t;
                t.v[0] = cs[0].first; t.n[0] = cs[0].second;
                t.v[1] = cs[k].first; t.n[1] = cs[k].second;
                t.v[2] = cs[k + 1].first; t.n[2] = cs[k + 1].second;
                t.mtl = cur_mtl;
                tris.push_back(t);
            }
        }
    }
    std::map<std::string, Mtl> lib;
    if (!mtllib.empty()) {
        if (!parse_mtl(relative_path(path, mtllib), lib) && !parse_mtl(mtllib, lib)) {
            err = "cannot read MTL " + mtllib;
            return false;
        }
    }
    const bool has_n = !nrm.empty();
    std::map<VKey, uint32_t> vmap, nmap;
    std::vector<std::pair<std::array<double, 10>, uint32_t>> mmap;
    for (const Tri& t : tris) {
        std::array<double, 10> mk;
        auto it = lib.find(t.mtl);
        if (it != lib.end()) {
            for (int k = 0; k < 3; ++k) {
                mk[k] = clamp01(it->second.ka[k]);
                mk[3 + k] = clamp01(it->second.kd[k]);
                mk[6 + k] = clamp01(it->second.ks[k]);
            }
            mk[9] = it->second.ns;
        } else {  // mesh.go:151 default material
            mk = {16 / 255.0, 16 / 255.0, 16 / 255.0, 1.0, 1.0, 1.0, 0.0, 0.0, 0.0, 0.0};
        }
        uint32_t mi = (uint32_t)mmap.size();
        for (auto& e : mmap)
            if (e.first == mk) { mi = e.second; break; }
        if (mi == mmap.size()) {
            mmap.emplace_back(mk, mi);
            mirt_material mm;
            for (int k = 0; k < 3; ++k) { mm.ka[k] = mk[k]; mm.kd[k] = mk[3 + k]; mm.ks[k] = mk[6 + k]; }
            mm.ns = mk[9];
            m.mats.push_back(mm);
        }
        for (int c = 0; c < 3; ++c) {
            const auto& p = pos[t.v[c]];
            VKey key{p[0], p[1], p[2]};
            auto vi = vmap.find(key);
            uint32_t idx;
            if (vi == vmap.end()) {
                idx = (uint32_t)(m.v.size() / 3);
                vmap.emplace(key, idx);
                m.v.insert(m.v.end(), {p[0], p[1], p[2]});
            } else {
                idx = vi->second;
            }
            m.fv.push_back(idx);
            if (has_n) {
                std::array<double, 3> n = t.n[c] >= 0 ? nrm[t.n[c]] : std::array<double, 3>{0, 0, 0};
                VKey nk{n[0], n[1], n[2]};
                auto ni = nmap.find(nk);
                if (ni == nmap.end()) {
                    idx = (uint32_t)(m.vn.size() / 3);
                    nmap.emplace(nk, idx);
                    // mesh.go:203 vertexNormals append vVertexNormal.Norm()
                    double mag = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
                    m.vn.insert(m.vn.end(), {n[0] / mag, n[1] / mag, n[2] / mag});
                } else {
                    idx = ni->second;
                }
                m.fn.push_back(idx);
            } else {
                m.fn.push_back(0);
            }
        }
        m.fmat.push_back(mi);
    }
    return true;
}

}  // namespace

struct mirt_scene {
    // shared: a scene linked from a gob diff (mirt_scene_link_gob) uses its environment's meshes
    std::vector<std::shared_ptr<MeshData>> meshes;
    std::vector<mirt_object> objects;
    std::vector<mirt_light> lights;
    mirt_camera cam;
    bool has_cam = false;
    // object id -> mesh index (envImmutables.paths through .meshes; gob environments only)
    std::map<uint64_t, uint32_t> id_mesh;
};

extern "C" {

int mirt_camera_init(const double pos[3], const double dir[3], double fov, mirt_camera* out);

int mirt_scene_load(const char* path, mirt_scene** out) {
    if (!path || !out) return MIRT_E_INVALID;
    *out = nullptr;
    std::string text;
    if (!read_file(path, text)) {
        g_scene_err = std::string("cannot read scene ") + path;
        return MIRT_E_IO;
    }
    JVal doc;
    JParser jp{text.data(), text.data() + text.size(), {}};
    if (!jp.parse(doc) || doc.kind != JVal::Obj) {
        g_scene_err = "scene JSON: " + jp.err;
        return MIRT_E_IO;
    }
    std::unique_ptr<mirt_scene> s(new mirt_scene());
    std::map<std::string, uint32_t> by_model;
    const JVal* objs = doc.get("objs");
    if (objs && objs->kind == JVal::Arr) {
        for (const JVal& o : objs->arr) {
            const JVal* model = o.get("model");
            std::string mp = model && model->kind == JVal::Str ? model->str : "";
            auto it = by_model.find(mp);
            uint32_t mi;
            if (it == by_model.end()) {
                std::shared_ptr<MeshData> md(new MeshData());
                std::string err;
                if (!load_mesh(relative_path(path, mp), *md, err)) {
                    md.reset(new MeshData());
                    std::string err2;
                    if (!load_mesh(mp, *md, err2)) {
                        g_scene_err = err;
                        return MIRT_E_IO;
                    }
                }
                mi = (uint32_t)s->meshes.size();
                s->meshes.push_back(std::move(md));
                by_model.emplace(mp, mi);
            } else {
                mi = it->second;
            }
            mirt_object ob{};
            ob.mesh_id = mi;
            jvec(o.get("pos"), ob.pos);
            s->objects.push_back(ob);
        }
    }
    const JVal* lights = doc.get("lights");
    if (lights && lights->kind == JVal::Arr) {
        for (const JVal& l : lights->arr) {
            mirt_light lt{};
            jvec(l.get("pos"), lt.pos);
            const JVal* col = l.get("col");
            const char* ch[3] = {"r", "g", "b"};
            for (int k = 0; k < 3; ++k) {
                double c = jnum(col ? col->get(ch[k]) : nullptr);
                if (c < 0 || c > 255 || c != std::floor(c)) {
                    g_scene_err = "light colour channel is not a uint8";
                    return MIRT_E_IO;
                }
                lt.col[k] = (double)(uint8_t)c / 255.0;  // colour.go:28-30 NewRGB
            }
            s->lights.push_back(lt);
        }
    }
    const JVal* cam = doc.get("cam");
    double cp[3], cd[3];
    jvec(cam ? cam->get("pos") : nullptr, cp);
    jvec(cam ? cam->get("dir") : nullptr, cd);
    double fov = jnum(cam ? cam->get("fov") : nullptr);
    if (mirt_camera_init(cp, cd, fov, &s->cam) != MIRT_OK) {
        g_scene_err = "Camera dir is parallel to global up";
        return MIRT_E_CAMERA;
    }
    s->has_cam = true;
    *out = s.release();
    return MIRT_OK;
}

// worker/distributed/main.go:118-126 register: MasterState.state -> the immutable scene.
// Meshes in model-path order (the wire carries a Go map, whose order is random).
int mirt_scene_from_gob(const uint8_t* state, size_t n, mirt_scene** out) {
    if (!state || !out) return MIRT_E_INVALID;
    *out = nullptr;
    mirt::gob::Immutables im;
    std::string err;
    if (!mirt::gob::decode_environment(state, n, im, err)) {
        g_scene_err = err;
        return MIRT_E_IO;
    }
    std::sort(im.meshes.begin(), im.meshes.end(),
              [](const auto& a, const auto& b) { return a.first < b.first; });
    std::unique_ptr<mirt_scene> s(new mirt_scene());
    std::map<std::string, uint32_t> by_path;
    for (auto& pm : im.meshes) {
        if (by_path.count(pm.first)) {
            g_scene_err = "gob Environment: model path twice in the mesh map";
            return MIRT_E_IO;
        }
        const mirt::gob::Mesh& g = pm.second;
        std::shared_ptr<MeshData> md(new MeshData());
        if (g.v.size() / 3 > 0xffffffffull || g.fmat.size() > 0xffffffffull) {
            g_scene_err = "gob Environment: mesh too large";
            return MIRT_E_IO;
        }
        md->v = g.v;
        md->vn = g.vn;
        // a mesh without normals carries zero normal indices (mesh.go:167-169); keep them so
        md->fv.assign(g.fv.begin(), g.fv.end());
        md->fn.assign(g.fn.begin(), g.fn.end());
        md->fmat.assign(g.fmat.begin(), g.fmat.end());
        md->mats = g.mats;
        by_path.emplace(pm.first, (uint32_t)s->meshes.size());
        s->meshes.push_back(std::move(md));
    }
    for (auto& ip : im.paths) {  // LinkTo (environment.go:80-88): id -> path -> mesh
        auto it = by_path.find(ip.second);
        if (it != by_path.end()) s->id_mesh[ip.first] = it->second;
    }
    *out = s.release();
    return MIRT_OK;
}

// worker/distributed/main.go:56-64 BulkTrace: WorkOrder.diff decoded and linked to env.
int mirt_scene_link_gob(const mirt_scene* env, const uint8_t* diff, size_t n, mirt_scene** out) {
    if (!env || !diff || !out) return MIRT_E_INVALID;
    *out = nullptr;
    mirt::gob::Mutables mu;
    std::string err;
    if (!mirt::gob::decode_mutables(diff, n, mu, err)) {
        g_scene_err = err;
        return MIRT_E_IO;
    }
    std::unique_ptr<mirt_scene> s(new mirt_scene());
    s->meshes = env->meshes;
    s->id_mesh = env->id_mesh;
    for (const auto& o : mu.objects) {
        mirt_object ob{};
        auto it = env->id_mesh.find(o.id);
        ob.mesh_id = it == env->id_mesh.end() ? MIRT_NO_MESH : it->second;  // environment.go:80-88
        ob.pos[0] = o.pos[0];
        ob.pos[1] = o.pos[1];
        ob.pos[2] = o.pos[2];
        s->objects.push_back(ob);
    }
    s->lights = mu.lights;
    // camera.go:196-200: NewCamera(pos, forward, fov), an error if forward is parallel to up
    if (mirt_camera_init(mu.cam_pos, mu.cam_forward, mu.fov, &s->cam) != MIRT_OK) {
        g_scene_err = "gob EnvMutables: Camera dir is parallel to global up";
        return MIRT_E_CAMERA;
    }
    s->has_cam = true;
    *out = s.release();
    return MIRT_OK;
}

int mirt_gob_json(const uint8_t* data, size_t n, char* out, size_t cap, size_t* len) {
    if (!data || !len) return MIRT_E_INVALID;
    std::string js, err;
    if (!mirt::gob::to_json(data, n, js, err)) {
        g_scene_err = err;
        return MIRT_E_IO;
    }
    *len = js.size();
    if (out && cap) {
        const size_t k = std::min(cap - 1, js.size());
        memcpy(out, js.data(), k);
        out[k] = 0;
    }
    return MIRT_OK;
}

const char* mirt_scene_last_error(void) { return g_scene_err.c_str(); }

void mirt_scene_free(mirt_scene* s) { delete s; }
uint32_t mirt_scene_mesh_count(const mirt_scene* s) { return s ? (uint32_t)s->meshes.size() : 0; }
int mirt_scene_mesh(const mirt_scene* s, uint32_t i, mirt_mesh_view* out) {
    if (!s || !out || i >= s->meshes.size()) return MIRT_E_INVALID;
    const MeshData& m = *s->meshes[i];
    out->vertices = m.v.data();
    out->n_vertices = (uint32_t)(m.v.size() / 3);
    out->normals = m.vn.empty() ? nullptr : m.vn.data();
    out->n_normals = (uint32_t)(m.vn.size() / 3);
    out->face_v = m.fv.data();
    out->face_n = m.fn.data();
    out->face_mat = m.fmat.data();
    out->n_faces = (uint32_t)m.fmat.size();
    out->materials = m.mats.data();
    out->n_materials = (uint32_t)m.mats.size();
    return MIRT_OK;
}
uint32_t mirt_scene_object_count(const mirt_scene* s) { return s ? (uint32_t)s->objects.size() : 0; }
int mirt_scene_object(const mirt_scene* s, uint32_t i, mirt_object* out) {
    if (!s || !out || i >= s->objects.size()) return MIRT_E_INVALID;
    *out = s->objects[i];
    return MIRT_OK;
}
uint32_t mirt_scene_light_count(const mirt_scene* s) { return s ? (uint32_t)s->lights.size() : 0; }
int mirt_scene_light(const mirt_scene* s, uint32_t i, mirt_light* out) {
    if (!s || !out || i >= s->lights.size()) return MIRT_E_INVALID;
    *out = s->lights[i];
    return MIRT_OK;
}
int mirt_scene_camera(const mirt_scene* s, mirt_camera* out) {
    if (!s || !out || !s->has_cam) return MIRT_E_INVALID;
    *out = s->cam;
    return MIRT_OK;
}

}  // extern "C"
