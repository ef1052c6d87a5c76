// rs_obj_loader.cpp -- OBJ/MTL scene loader (host), standing in for the reference's assimp-based
// ModelLoader (pg/ModelLoader.cpp:41-216; assimp is not available here).  Conventions kept:
//   * MTL "Pc" (read by assimp as AI_MATKEY_CLEARCOAT_FACTOR) selects the material class
//     (pg/ModelLoader.cpp:52-72): 0 NORMAL, 1 LAMBERT, 2 PHONG, 3 MIRROR, 4 DIELECTRIC,
//     5 DIELECTRIC_TRANSPARENT, anything else UNSUPPORTED
//   * Kd / Ks are sRGB-expanded at load (Raytracer::gammaCorrect = true, :86-97 -> Utils::expand,
//     pg/utils.cpp:209-218); Ke and Ns are taken as is (:103-109)
//   * polygons are fan-triangulated (aiProcess_Triangulate), triangles de-indexed
//   * vertex normals from "vn"; faces without normals get the geometric face normal
//   * texture coordinates from "vt" (attribute slot 1, :199-202,284-285), textures map_Kd / map_Ks /
//     map_Ns / norm (map_Kn) relative to the MTL's directory (:121-148), one texture per file
//     (TextureProxy's cache, :18-36); diffuse/specular maps are sRGB-expanded (Texture::expand, :127,135)
//   * tangents (slot 3) per triangle with the face formula of assimp's aiProcess_CalcTangentSpace,
//     projected onto each vertex normal (assimp additionally averages over vertices within its
//     smoothing angle -- parity unpinned; only normal-mapped materials read tangents)
// Triangles keep file order.
#include "../../include/restir_c.h"
#include "rs_image.h"
#include "rs_libm.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

namespace rs {

// Utils::expand (pg/utils.cpp:209-218)
static float srgb_expand(float u) {
    if (u <= 0.0f) return 0.0f;
    if (u >= 1.0f) return 1.0f;
    if (u <= 0.04045f) return u / 12.92f;
    return rs_powf((u + 0.055f) / 1.055f, 2.4f);
}

struct MtlTex { std::string dir; std::map<std::string, int> ids; std::vector<std::string> files; };

// last token of a map_* line is the file name (options such as -bm come first)
static int tex_ref(std::istringstream& ss, MtlTex& T) {
    std::string tok, name;
    while (ss >> tok) name = tok;
    if (name.empty()) return 0;
    const std::string full = T.dir + name;
    auto it = T.ids.find(full);
    if (it != T.ids.end()) return it->second;
    T.files.push_back(full);
    return T.ids[full] = (int)T.files.size();         // 1-based
}

static bool load_mtl(const std::string& path, std::vector<rs_material_desc>& mats, std::map<std::string, int>& ids,
                     MtlTex& T, std::string& err) {
    std::ifstream f(path);
    if (!f) { err = "cannot open MTL file " + path; return false; }
    size_t slash = path.find_last_of('/');
    T.dir = slash == std::string::npos ? std::string() : path.substr(0, slash + 1);
    std::string line;
    rs_material_desc* cur = nullptr;
    while (std::getline(f, line)) {
        std::istringstream ss(line);
        std::string tag;
        if (!(ss >> tag) || tag[0] == '#') continue;
        if (tag == "newmtl") {
            std::string name;
            ss >> name;
            rs_material_desc m;
            std::memset(&m, 0, sizeof m);
            m.shininess = 0.0f;
            m.type = 0;                           // no Pc => MaterialNormal (clearcoat 0)
            ids[name] = (int)mats.size();
            mats.push_back(m);
            cur = &mats.back();
            continue;
        }
        if (!cur) continue;
        auto rd3 = [&](float* v) { ss >> v[0] >> v[1] >> v[2]; };
        if (tag == "Kd") { rd3(cur->diffuse); for (int i = 0; i < 3; ++i) cur->diffuse[i] = srgb_expand(cur->diffuse[i]); }
        else if (tag == "Ks") { rd3(cur->specular); for (int i = 0; i < 3; ++i) cur->specular[i] = srgb_expand(cur->specular[i]); }
        else if (tag == "Ke") rd3(cur->emission);
        else if (tag == "Ns") ss >> cur->shininess;
        else if (tag == "Pc") {
            float pc = 0; ss >> pc;
            int t = (int)pc;
            cur->type = (pc == (float)t && t >= 0 && t <= 5) ? t : 6;
        }
        else if (tag == "map_Kd") cur->diffuse_map = tex_ref(ss, T);
        else if (tag == "map_Ks") cur->specular_map = tex_ref(ss, T);
        else if (tag == "map_Ns") cur->shininess_map = tex_ref(ss, T);
        else if (tag == "norm" || tag == "map_Kn") cur->normal_map = tex_ref(ss, T);
    }
    return true;
}

static int parse_index(const std::string& tok, int n) {
    int v = std::atoi(tok.c_str());
    if (v < 0) return n + v;
    return v - 1;
}

// aiProcess_CalcTangentSpace, per face (assimp CalcTangentsProcess::ProcessMesh): tangent from the uv
// derivatives, then per vertex projected onto the vertex normal and normalised
static void face_tangents(const float* P, const float* Nn, const float* UV, float* Tout) {
    const float v[3] = {P[3] - P[0], P[4] - P[1], P[5] - P[2]}, w[3] = {P[6] - P[0], P[7] - P[1], P[8] - P[2]};
    float sx = UV[2] - UV[0], sy = UV[3] - UV[1], tx = UV[4] - UV[0], ty = UV[5] - UV[1];
    const float dir = (tx * sy - ty * sx) < 0.0f ? -1.0f : 1.0f;
    if (sx * ty == sy * tx) { sx = 0.0f; sy = 1.0f; tx = 1.0f; ty = 0.0f; }
    float t[3];
    for (int a = 0; a < 3; ++a) t[a] = (w[a] * sy - v[a] * ty) * dir;
    for (int j = 0; j < 3; ++j) {
        const float* n = Nn + 3 * j;
        const float d = t[0] * n[0] + t[1] * n[1] + t[2] * n[2];
        float l[3] = {t[0] - n[0] * d, t[1] - n[1] * d, t[2] - n[2] * d};
        const float len = std::sqrt(l[0] * l[0] + l[1] * l[1] + l[2] * l[2]);
        for (int a = 0; a < 3; ++a) Tout[3 * j + a] = len > 0 ? l[a] / len : 0.0f;
    }
}

int load_obj_file(const char* path, ObjScene& out, std::string& err) {
    std::ifstream f(path);
    if (!f) { err = std::string("cannot open OBJ file ") + path; return -1; }
    std::string dir(path);
    size_t slash = dir.find_last_of('/');
    dir = slash == std::string::npos ? std::string() : dir.substr(0, slash + 1);
    std::vector<float> V, N, VT;
    std::map<std::string, int> ids;
    MtlTex T;
    std::vector<rs_material_desc>& mats = out.mats;
    int cur_mat = -1;
    std::string line;
    size_t lineno = 0;
    while (std::getline(f, line)) {
        ++lineno;
        std::istringstream ss(line);
        std::string tag;
        if (!(ss >> tag) || tag[0] == '#') continue;
        if (tag == "v") { float x, y, z; ss >> x >> y >> z; V.insert(V.end(), {x, y, z}); }
        else if (tag == "vn") { float x, y, z; ss >> x >> y >> z; N.insert(N.end(), {x, y, z}); }
        else if (tag == "vt") { float u = 0, v = 0; ss >> u >> v; VT.insert(VT.end(), {u, v}); }
        else if (tag == "mtllib") {
            std::string name; ss >> name;
            if (!load_mtl(dir + name, mats, ids, T, err)) return -1;
        } else if (tag == "usemtl") {
            std::string name; ss >> name;
            auto it = ids.find(name);
            if (it == ids.end()) { err = "unknown material " + name; return -1; }
            cur_mat = it->second;
        } else if (tag == "f") {
            std::vector<int> vi, ti, ni;
            std::string tok;
            while (ss >> tok) {
                std::string a = tok, b, c;
                size_t s1 = tok.find('/');
                if (s1 != std::string::npos) {
                    a = tok.substr(0, s1);
                    size_t s2 = tok.find('/', s1 + 1);
                    b = tok.substr(s1 + 1, s2 == std::string::npos ? std::string::npos : s2 - s1 - 1);
                    if (s2 != std::string::npos) c = tok.substr(s2 + 1);
                }
                vi.push_back(parse_index(a, (int)V.size() / 3));
                ti.push_back(b.empty() ? -1 : parse_index(b, (int)VT.size() / 2));
                ni.push_back(c.empty() ? -1 : parse_index(c, (int)N.size() / 3));
            }
            if (vi.size() < 3) continue;
            if (cur_mat < 0) {
                if (mats.empty() || ids.find("__default__") == ids.end()) {
                    rs_material_desc m; std::memset(&m, 0, sizeof m); m.type = 0;
                    ids["__default__"] = (int)mats.size(); mats.push_back(m);
                }
                cur_mat = ids["__default__"];
            }
            for (size_t k = 1; k + 1 < vi.size(); ++k) {
                int tv[3] = {vi[0], vi[k], vi[k + 1]}, tt[3] = {ti[0], ti[k], ti[k + 1]}, tn[3] = {ni[0], ni[k], ni[k + 1]};
                float P[9], Nn[9], UV[6], Tg[9];
                for (int j = 0; j < 3; ++j) {
                    if (tv[j] < 0 || 3 * (size_t)tv[j] + 2 >= V.size()) {
                        err = "vertex index out of range at line " + std::to_string(lineno);
                        return -1;
                    }
                    for (int a = 0; a < 3; ++a) P[3 * j + a] = V[3 * tv[j] + a];
                    const bool okt = tt[j] >= 0 && 2 * (size_t)tt[j] + 1 < VT.size();
                    UV[2 * j] = okt ? VT[2 * tt[j]] : 0.0f;
                    UV[2 * j + 1] = okt ? VT[2 * tt[j] + 1] : 0.0f;
                }
                float e1[3] = {P[3] - P[0], P[4] - P[1], P[5] - P[2]}, e2[3] = {P[6] - P[0], P[7] - P[1], P[8] - P[2]};
                float fn[3] = {e1[1] * e2[2] - e2[1] * e1[2], e1[2] * e2[0] - e2[2] * e1[0], e1[0] * e2[1] - e2[0] * e1[1]};
                float l = std::sqrt(fn[0] * fn[0] + fn[1] * fn[1] + fn[2] * fn[2]);
                if (l > 0) for (float& q : fn) q /= l;
                for (int j = 0; j < 3; ++j) {
                    bool ok = tn[j] >= 0 && 3 * (size_t)tn[j] + 2 < N.size();
                    for (int a = 0; a < 3; ++a) Nn[3 * j + a] = ok ? N[3 * tn[j] + a] : fn[a];
                }
                face_tangents(P, Nn, UV, Tg);
                out.pos.insert(out.pos.end(), P, P + 9);
                out.nrm.insert(out.nrm.end(), Nn, Nn + 9);
                out.uv.insert(out.uv.end(), UV, UV + 6);
                out.tan.insert(out.tan.end(), Tg, Tg + 9);
                out.tri_mat.push_back((uint32_t)cur_mat);
            }
        }
    }
    if (out.tri_mat.empty()) { err = std::string("no triangles in ") + path; return -1; }
    // textures, in first-reference order (1-based ids in the material map slots)
    out.images.resize(T.files.size());
    out.srgb.assign(T.files.size(), 0);
    for (size_t i = 0; i < T.files.size(); ++i) {
        int rc = load_image(T.files[i], out.images[i], err);
        if (rc) return rc == -3 ? -3 : -1;
    }
    for (const rs_material_desc& m : mats) {              // Raytracer::gammaCorrect: colour maps expanded
        if (m.diffuse_map > 0) out.srgb[m.diffuse_map - 1] = 1;
        if (m.specular_map > 0) out.srgb[m.specular_map - 1] = 1;
    }
    return 0;
}

}  // namespace rs
