// scene_file.hpp — plain-text scene files for the host CLI (SURVEY §8f:
// scene authoring instead of the reference's compiled-in allocateScene(),
// Main.cu:38-109).  One primitive per line, '#' starts a comment:
//
//   camera   px py pz  angle0 angle1  fov
//   sphere   cx cy cz  radius                       ar ag ab [emit [rough [ior]]]
//   plane    ox oy oz  d0x d0y d0z  d1x d1y d1z     ar ag ab [emit [rough [ior]]]
//   triangle v0x v0y v0z  v1x v1y v1z  v2x v2y v2z  ar ag ab [emit [rough [ior]]]
//   quad     v0 v1 v2 v3 (12 numbers)               ar ag ab [emit [rough [ior]]]
//
// Omitted material fields take the reference defaults (WorldTypes.cuh:15-20:
// emittance 0, roughness 1, refractiveIndex 1.05).  save_scene writes every
// float with %.9g, which reads back bit-exactly.  bwrt/scenefile.py is the
// Python twin (tests check both against each other).
#pragma once

#include <cstdio>
#include <cstdlib>
#include <sstream>
#include <string>
#include <vector>

#include "scenes.hpp"

namespace bwrt {

inline bool parse_floats(std::istringstream& in, std::vector<float>& out) {
    std::string tok;
    while (in >> tok) {
        if (tok[0] == '#') break;
        char* end = nullptr;
        const float v = std::strtof(tok.c_str(), &end);
        if (end == tok.c_str() || *end) return false;
        out.push_back(v);
    }
    return true;
}

inline bool material_from(const std::vector<float>& f, size_t at, rt_material& m) {
    const size_t n = f.size() - at;
    if (n < 3 || n > 6) return false;
    m = mat(rt_vec3{f[at], f[at + 1], f[at + 2]});
    if (n > 3) m.emittance = f[at + 3];
    if (n > 4) m.roughness = f[at + 4];
    if (n > 5) m.refractive_index = f[at + 5];
    return true;
}

// Returns "" on success, else an error message naming the line.
inline std::string load_scene(const std::string& path, SceneData& sd) {
    FILE* fp = std::fopen(path.c_str(), "r");
    if (!fp) return "cannot open " + path;
    sd = SceneData{};
    sd.camera = rt_camera{rt_vec3{0, 1, 0}, {0, 0}, 1.57079637f};  // Main.cu:39
    char buf[4096];
    int line = 0;
    std::string err;
    while (err.empty() && std::fgets(buf, sizeof buf, fp)) {
        line++;
        std::istringstream in(buf);
        std::string kind;
        if (!(in >> kind) || kind[0] == '#') continue;
        std::vector<float> f;
        if (!parse_floats(in, f)) {
            err = "line " + std::to_string(line) + ": bad number";
            break;
        }
        auto vec = [&](size_t i) { return rt_vec3{f[i], f[i + 1], f[i + 2]}; };
        rt_material m;
        if (kind == "camera" && f.size() == 6) {
            sd.camera = rt_camera{vec(0), {f[3], f[4]}, f[5]};
        } else if (kind == "sphere" && f.size() >= 7 && material_from(f, 4, m)) {
            sd.spheres.push_back(rt_sphere{vec(0), f[3], m});
        } else if (kind == "plane" && f.size() >= 12 && material_from(f, 9, m)) {
            sd.planes.push_back(rt_plane{vec(0), {vec(3), vec(6)}, m});
        } else if (kind == "triangle" && f.size() >= 12 && material_from(f, 9, m)) {
            sd.triangles.push_back(rt_triangle{{vec(0), vec(3), vec(6)}, m});
        } else if (kind == "quad" && f.size() >= 15 && material_from(f, 12, m)) {
            sd.quads.push_back(rt_quad{{vec(0), vec(3), vec(6), vec(9)}, m});
        } else {
            err = "line " + std::to_string(line) + ": cannot parse '" + kind + "' with " +
                  std::to_string(f.size()) + " numbers";
        }
    }
    std::fclose(fp);
    return err;
}

inline bool save_scene(const std::string& path, const SceneData& sd) {
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) return false;
    auto v = [&](const rt_vec3& a) { std::fprintf(f, " %.9g %.9g %.9g", a.x, a.y, a.z); };
    auto m = [&](const rt_material& a) {
        std::fprintf(f, " ");
        v(a.albedo);
        std::fprintf(f, " %.9g %.9g %.9g\n", a.emittance, a.roughness, a.refractive_index);
    };
    std::fprintf(f, "# bwrt scene: camera / sphere / plane / triangle / quad (host/scene_file.hpp)\n");
    std::fprintf(f, "camera");
    v(sd.camera.position);
    std::fprintf(f, " %.9g %.9g %.9g\n", sd.camera.angle[0], sd.camera.angle[1], sd.camera.fov);
    for (const rt_sphere& s : sd.spheres) {
        std::fprintf(f, "sphere");
        v(s.position);
        std::fprintf(f, " %.9g", s.radius);
        m(s.mat);
    }
    for (const rt_plane& p : sd.planes) {
        std::fprintf(f, "plane");
        v(p.origin);
        v(p.directions[0]);
        v(p.directions[1]);
        m(p.mat);
    }
    for (const rt_triangle& t : sd.triangles) {
        std::fprintf(f, "triangle");
        for (int k = 0; k < 3; k++) v(t.vertices[k]);
        m(t.mat);
    }
    for (const rt_quad& q : sd.quads) {
        std::fprintf(f, "quad");
        for (int k = 0; k < 4; k++) v(q.vertices[k]);
        m(q.mat);
    }
    return std::fclose(f) == 0;
}

}  // namespace bwrt
