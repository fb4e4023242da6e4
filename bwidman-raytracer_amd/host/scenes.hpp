// scenes.hpp — C++ host-side scene definitions over the C ABI structs.
//
// scene07() is allocateScene() of /root/reference/bwidman-raytracer/src/
// Main.cu:38-109 (same aggregate values, double literals narrowed to float);
// the others mirror bwrt/scenes.py (tests pin both to the same bytes).
#pragma once

#include <vector>

#include "rt_abi.h"

namespace bwrt {

inline rt_vec3 v(float x, float y, float z) { return rt_vec3{x, y, z}; }

inline rt_material mat(rt_vec3 albedo, float emittance = 0.0f, float roughness = 1.0f,
                       float ior = (float)1.05) {
    return rt_material{albedo, emittance, roughness, ior};  // WorldTypes.cuh:15-20 defaults
}

struct SceneData {
    rt_camera camera{};
    std::vector<rt_sphere> spheres;
    std::vector<rt_plane> planes;
    std::vector<rt_triangle> triangles;
    std::vector<rt_quad> quads;

    rt_scene view() const {
        rt_scene s;
        s.camera = camera;
        s.spheres = spheres.data();
        s.sphere_count = (int)spheres.size();
        s.planes = planes.data();
        s.plane_count = (int)planes.size();
        s.triangles = triangles.data();
        s.triangle_count = (int)triangles.size();
        s.quads = quads.data();
        s.quad_count = (int)quads.size();
        return s;
    }
};

constexpr float kPi = 3.1415926535f;  // Math.cuh:5

inline SceneData scene07() {
    SceneData s;
    s.camera = rt_camera{v(0, 1, 0), {0, 0}, kPi / 2};
    s.spheres = {
        {v(-6, 3, -4), 1, mat(v(1, (float)0.6, (float)0.2), 20)},
        {v(6, 3, -4), 1, mat(v(1, (float)0.2, (float)0.6), 20)},
        {v((float)-0.5, (float)0.2, -3), (float)0.2, mat(v((float)0.2, (float)0.8, (float)0.2), 5)},
        {v(0, (float)0.75, -4), (float)0.75, mat(v(1, 1, 1), 0, 0.001f, 10)},
        {v(-4, 1, -6), 1, mat(v((float)0.2, 0, (float)0.8), 0, 1)},
        {v(4, 2, -8), 2, mat(v(1, (float)0.1, 0), 0, 1)},
    };
    s.planes = {{v(0, 0, 0), {v(0, 0, 1), v(1, 0, 0)}, mat(v((float)0.5, (float)0.5, (float)0.5))}};
    const rt_material py = mat(v((float)0.95, (float)0.9, (float)0.2));
    const float h = (float)1.5, a = (float)3.5;
    s.triangles = {
        {{v(-2, 0, -3), v(-1, 0, -3), v(-h, 1, -a)}, py},
        {{v(-1, 0, -4), v(-2, 0, -4), v(-h, 1, -a)}, py},
        {{v(-2, 0, -4), v(-2, 0, -3), v(-h, 1, -a)}, py},
        {{v(-1, 0, -3), v(-1, 0, -4), v(-h, 1, -a)}, py},
    };
    return s;
}

inline SceneData scene01() {
    SceneData s;
    s.camera = rt_camera{v(0, 0, 0), {0, 0}, kPi / 2};
    s.spheres = {{v(0, 0, -3), 1, mat(v(1, 0, 0), 1)}};
    return s;
}

inline SceneData scene04() {
    SceneData a = scene07(), s;
    s.camera = a.camera;
    s.spheres = {a.spheres[0], a.spheres[1], a.spheres[4], a.spheres[5]};
    s.planes = a.planes;
    return s;
}

inline SceneData scene04box() {  // + mirror quads of Main.cu:80-84
    SceneData s = scene04();
    const float w = 10;
    const rt_material m = mat(v(1, (float)0.8, (float)0.2), 0, (float)0.005, 10);
    s.quads = {
        {{v(w, 0, -w), v(w, w, -w), v(-w, w, -w), v(-w, 0, -w)}, m},
        {{v(-w, 0, -w - 1), v(-w, w, -w - 1), v(w, w, -w - 1), v(w, 0, -w - 1)}, m},
        {{v(-w, 0, -w), v(-w, w, -w), v(-w, w, -w - 1), v(-w, 0, -w - 1)}, m},
        {{v(w, 0, -w - 1), v(w, w, -w - 1), v(w, w, -w), v(w, 0, -w)}, m},
        {{v(w, w, -w), v(w, w, -w - 1), v(-w, w, -w - 1), v(-w, w, -w)}, m},
    };
    return s;
}

}  // namespace bwrt
