// bwrt_render — C++ host driver over the C ABI (the reference's main loop,
// /root/reference/bwidman-raytracer/src/Main.cu:401-517, without the GLFW
// window: frames are rendered progressively, FPS / sample count are printed
// once per second like Main.cu:486-495, and the final image is written as a
// binary PPM (top row first, i.e. the RGBA8 buffer flipped: row 0 = bottom).
//
//   bwrt_render [--scene 07|01|04|04_box] [--width 1920] [--height 1080]
//               [--frames 8] [--frames-per-call 1] [--max-bounces 5]
//               [--device 0] [--out image.ppm] [--dump-scene file.bin]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rt_abi.h"
#include "scenes.hpp"

static int die(rt_context* ctx, int rc, const char* what) {
    std::fprintf(stderr, "%s failed: %s (%s)\n", what, rt_error_string(rc), ctx ? rt_last_error(ctx) : "");
    return 1;
}

int main(int argc, char** argv) {
    std::string scene_name = "07", out, dump;
    int width = 1920, height = 1080, frames = 8, per_call = 1, max_bounces = RT_DEFAULT_MAX_BOUNCES, device = 0;
    for (int i = 1; i < argc; i++) {
        auto next = [&](void) -> const char* { return i + 1 < argc ? argv[++i] : ""; };
        if (!std::strcmp(argv[i], "--scene")) scene_name = next();
        else if (!std::strcmp(argv[i], "--width")) width = std::atoi(next());
        else if (!std::strcmp(argv[i], "--height")) height = std::atoi(next());
        else if (!std::strcmp(argv[i], "--frames")) frames = std::atoi(next());
        else if (!std::strcmp(argv[i], "--frames-per-call")) per_call = std::atoi(next());
        else if (!std::strcmp(argv[i], "--max-bounces")) max_bounces = std::atoi(next());
        else if (!std::strcmp(argv[i], "--device")) device = std::atoi(next());
        else if (!std::strcmp(argv[i], "--out")) out = next();
        else if (!std::strcmp(argv[i], "--dump-scene")) dump = next();
        else {
            std::fprintf(stderr, "unknown option %s\n", argv[i]);
            return 2;
        }
    }
    bwrt::SceneData sd = scene_name == "01" ? bwrt::scene01()
                         : scene_name == "04" ? bwrt::scene04()
                         : scene_name == "04_box" ? bwrt::scene04box()
                                                  : bwrt::scene07();
    if (!dump.empty()) {  // camera + primitive bytes (compared with bwrt.scenes by the tests)
        FILE* f = std::fopen(dump.c_str(), "wb");
        if (!f) return 1;
        std::fwrite(&sd.camera, sizeof sd.camera, 1, f);
        std::fwrite(sd.spheres.data(), sizeof(rt_sphere), sd.spheres.size(), f);
        std::fwrite(sd.planes.data(), sizeof(rt_plane), sd.planes.size(), f);
        std::fwrite(sd.triangles.data(), sizeof(rt_triangle), sd.triangles.size(), f);
        std::fwrite(sd.quads.data(), sizeof(rt_quad), sd.quads.size(), f);
        std::fclose(f);
        return 0;
    }
    rt_context* ctx = nullptr;
    int rc = rt_create(device, &ctx);
    if (rc) return die(ctx, rc, "rt_create");
    rt_scene view = sd.view();
    if ((rc = rt_set_scene(ctx, &view))) return die(ctx, rc, "rt_set_scene");
    if ((rc = rt_set_max_bounces(ctx, max_bounces))) return die(ctx, rc, "rt_set_max_bounces");
    std::vector<uint8_t> rgba((size_t)width * height * 4);
    using clk = std::chrono::steady_clock;
    double delta = 0.0;
    int frame_count = 0;
    for (int done = 0; done < frames;) {
        const int n = std::min(per_call, frames - done);
        auto t0 = clk::now();
        if ((rc = rt_render(ctx, width, height, n, rgba.data()))) return die(ctx, rc, "rt_render");
        done += n;
        delta += std::chrono::duration<double>(clk::now() - t0).count();
        frame_count += n;
        if (delta > 1.0 || done == frames) {  // Main.cu:486-495
            std::printf("FPS: %d | Samples: %u | kernel %.3f ms\n", (int)(frame_count / delta),
                        rt_frame_counter(ctx) - 1, rt_last_kernel_ms(ctx));
            delta = 0.0;
            frame_count = 0;
        }
    }
    if (!out.empty()) {
        FILE* f = std::fopen(out.c_str(), "wb");
        if (!f) return 1;
        std::fprintf(f, "P6\n%d %d\n255\n", width, height);
        for (int y = height - 1; y >= 0; y--)
            for (int x = 0; x < width; x++) std::fwrite(&rgba[((size_t)y * width + x) * 4], 1, 3, f);
        std::fclose(f);
    }
    rt_destroy(ctx);
    return 0;
}
