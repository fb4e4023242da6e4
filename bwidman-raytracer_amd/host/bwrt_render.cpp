// bwrt_render — C++ host driver over the C ABI: the reference's main loop
// (/root/reference/bwidman-raytracer/src/Main.cu:401-517) without the GLFW
// window.  Frames are rendered progressively; after each frame controls()
// (Controls.cuh:5-75) is applied with the keys a scripted timeline holds
// (--keys) and the frame's duration (or a fixed --dt); FPS / sample count
// are printed once per second like Main.cu:486-495; the final image is
// written as PNG or PPM (top row first: the buffer's row 0 is the bottom).
//
//   bwrt_render [--scene 07|01|04|04_box | --scene-file FILE] [--save-scene FILE]
//               [--width 1920] [--height 1080] [--frames 8] [--frames-per-call 1]
//               [--max-bounces 5] [--background r,g,b] [--spp 1] [--device 0] [--gpus 1]
//               [--cpu [THREADS]] [--keys "W*10,W+LEFT*5,*3"] [--dt SECONDS]
//               [--out image.png|image.ppm] [--dump-scene file.bin]
//
// --keys: comma-separated steps KEY[+KEY...]*FRAMES (keys W A S D SPACE
// LEFT_SHIFT LEFT RIGHT UP DOWN ESCAPE; an empty key list holds nothing);
// the timeline repeats its last step.  ESCAPE ends the loop like
// glfwSetWindowShouldClose.  --gpus N renders every frame across N contexts
// (devices device..device+N-1, modulo the visible count) with rt_render_multi.
// --cpu renders on the library's scalar C++ CPU fallback instead (THREADS
// host threads, 0 or omitted = all; BASELINE config 1's "scalar C++ CPU
// path").  --spp sets samplesPerPixel (Main.cu:27; the in-frame loop keeps
// the last of n paths, Main.cu:296-299), and "Samples:" prints
// accumulatedFrames * samplesPerPixel like Main.cu:491.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "image_io.hpp"
#include "rt_abi.h"
#include "scene_file.hpp"
#include "scenes.hpp"

static int die(rt_context* ctx, int rc, const char* what) {
    std::fprintf(stderr, "%s failed: %s (%s)\n", what, rt_error_string(rc), ctx ? rt_last_error(ctx) : "");
    return 1;
}

static const char* kUsage =
    "usage: bwrt_render [--scene 07|01|04|04_box | --scene-file FILE] [--save-scene FILE]\n"
    "                   [--width 1920] [--height 1080] [--frames 8] [--frames-per-call 1]\n"
    "                   [--max-bounces 5] [--background r,g,b] [--spp 1] [--device 0] [--gpus 1]\n"
    "                   [--cpu [THREADS]] [--keys \"W*10,W+LEFT*5,*3\"] [--dt SECONDS]\n"
    "                   [--out image.png|image.ppm] [--dump-scene file.bin]\n";

struct KeyStep {
    unsigned keys;
    int frames;
};

static bool parse_keys(const std::string& spec, std::vector<KeyStep>& steps) {
    static const struct {
        const char* name;
        unsigned bit;
    } names[] = {{"W", RT_KEY_W},         {"A", RT_KEY_A},       {"S", RT_KEY_S},
                 {"D", RT_KEY_D},         {"SPACE", RT_KEY_SPACE}, {"LEFT_SHIFT", RT_KEY_LEFT_SHIFT},
                 {"LEFT", RT_KEY_LEFT},   {"RIGHT", RT_KEY_RIGHT}, {"UP", RT_KEY_UP},
                 {"DOWN", RT_KEY_DOWN},   {"ESCAPE", RT_KEY_ESCAPE}};
    size_t pos = 0;
    while (pos <= spec.size()) {
        size_t end = spec.find(',', pos);
        if (end == std::string::npos) end = spec.size();
        std::string step = spec.substr(pos, end - pos);
        pos = end + 1;
        if (step.empty()) {
            if (end == spec.size()) break;
            continue;
        }
        int frames = 1;
        const size_t star = step.find('*');
        if (star != std::string::npos) {
            frames = std::atoi(step.c_str() + star + 1);
            step = step.substr(0, star);
            if (frames < 1) return false;
        }
        unsigned keys = 0;
        size_t k = 0;
        while (k < step.size()) {
            size_t plus = step.find('+', k);
            if (plus == std::string::npos) plus = step.size();
            const std::string name = step.substr(k, plus - k);
            bool found = false;
            for (const auto& n : names)
                if (name == n.name) {
                    keys |= n.bit;
                    found = true;
                }
            if (!found) return false;
            k = plus + 1;
        }
        steps.push_back({keys, frames});
    }
    return true;
}

int main(int argc, char** argv) {
    std::string scene_name = "07", scene_file, save, out, dump, keys_spec;
    int width = 1920, height = 1080, frames = 8, per_call = 1, max_bounces = RT_DEFAULT_MAX_BOUNCES, device = 0;
    int gpus = 1, spp = 1, cpu_threads = -1;  // -1: GPU
    float bg[3] = {0.0f, 0.0f, 0.0f};
    double fixed_dt = -1.0;
    for (int i = 1; i < argc; i++) {
        auto next = [&](void) -> const char* { return i + 1 < argc ? argv[++i] : ""; };
        if (!std::strcmp(argv[i], "--help") || !std::strcmp(argv[i], "-h")) {
            std::fputs(kUsage, stdout);
            return 0;
        } else if (!std::strcmp(argv[i], "--scene")) scene_name = next();
        else if (!std::strcmp(argv[i], "--scene-file")) scene_file = next();
        else if (!std::strcmp(argv[i], "--save-scene")) save = next();
        else if (!std::strcmp(argv[i], "--width")) width = std::atoi(next());
        else if (!std::strcmp(argv[i], "--height")) height = std::atoi(next());
        else if (!std::strcmp(argv[i], "--frames")) frames = std::atoi(next());
        else if (!std::strcmp(argv[i], "--frames-per-call")) per_call = std::atoi(next());
        else if (!std::strcmp(argv[i], "--max-bounces")) max_bounces = std::atoi(next());
        else if (!std::strcmp(argv[i], "--background")) {
            if (std::sscanf(next(), "%f,%f,%f", &bg[0], &bg[1], &bg[2]) != 3) {
                std::fprintf(stderr, "--background expects r,g,b\n");
                return 2;
            }
        } else if (!std::strcmp(argv[i], "--device")) device = std::atoi(next());
        else if (!std::strcmp(argv[i], "--gpus")) gpus = std::atoi(next());
        else if (!std::strcmp(argv[i], "--spp")) spp = std::atoi(next());
        else if (!std::strcmp(argv[i], "--cpu")) {
            cpu_threads = 0;
            if (i + 1 < argc && argv[i + 1][0] >= '0' && argv[i + 1][0] <= '9') cpu_threads = std::atoi(argv[++i]);
        }
        else if (!std::strcmp(argv[i], "--keys")) keys_spec = next();
        else if (!std::strcmp(argv[i], "--dt")) fixed_dt = std::atof(next());
        else if (!std::strcmp(argv[i], "--out")) out = next();
        else if (!std::strcmp(argv[i], "--dump-scene")) dump = next();
        else {
            std::fprintf(stderr, "unknown option %s\n%s", argv[i], kUsage);
            return 2;
        }
    }
    std::vector<KeyStep> steps;
    if (!keys_spec.empty()) {
        if (!parse_keys(keys_spec, steps)) {
            std::fprintf(stderr, "bad --keys '%s'\n", keys_spec.c_str());
            return 2;
        }
        per_call = 1;  // controls() runs between frames
    }
    bwrt::SceneData sd;
    if (!scene_file.empty()) {
        const std::string err = bwrt::load_scene(scene_file, sd);
        if (!err.empty()) {
            std::fprintf(stderr, "%s: %s\n", scene_file.c_str(), err.c_str());
            return 2;
        }
    } else {
        sd = scene_name == "01"       ? bwrt::scene01()
             : scene_name == "04"     ? bwrt::scene04()
             : scene_name == "04_box" ? bwrt::scene04box()
                                      : bwrt::scene07();
    }
    if (!save.empty() && !bwrt::save_scene(save, sd)) {
        std::fprintf(stderr, "cannot write %s\n", save.c_str());
        return 1;
    }
    if (!dump.empty()) {  // camera + primitive bytes (compared with bwrt.scenes by the tests)
        FILE* f = std::fopen(dump.c_str(), "wb");
        if (!f) return 1;
        std::fwrite(&sd.camera, sizeof sd.camera, 1, f);
        std::fwrite(sd.spheres.data(), sizeof(rt_sphere), sd.spheres.size(), f);
        std::fwrite(sd.planes.data(), sizeof(rt_plane), sd.planes.size(), f);
        std::fwrite(sd.triangles.data(), sizeof(rt_triangle), sd.triangles.size(), f);
        std::fwrite(sd.quads.data(), sizeof(rt_quad), sd.quads.size(), f);
        std::fclose(f);
    }
    if (!dump.empty() || (!save.empty() && frames <= 0)) return 0;

    if (gpus < 1 || cpu_threads >= 0) gpus = 1;
    const int ndev = cpu_threads >= 0 ? 1 : rt_device_count() > 0 ? rt_device_count() : 1;
    std::vector<rt_context*> ctxs(gpus, nullptr);
    int rc = 0;
    rt_scene view = sd.view();
    for (int g = 0; g < gpus; g++) {
        if (cpu_threads >= 0) {
            if ((rc = rt_create_cpu(cpu_threads, &ctxs[g]))) return die(ctxs[g], rc, "rt_create_cpu");
            std::printf("CPU fallback: %d threads\n", rt_context_threads(ctxs[g]));
        } else if ((rc = rt_create((device + g) % ndev, &ctxs[g]))) {
            return die(ctxs[g], rc, "rt_create");
        }
        if ((rc = rt_set_samples_per_pixel(ctxs[g], spp))) return die(ctxs[g], rc, "rt_set_samples_per_pixel");
        if ((rc = rt_set_scene(ctxs[g], &view))) return die(ctxs[g], rc, "rt_set_scene");
        if ((rc = rt_set_max_bounces(ctxs[g], max_bounces))) return die(ctxs[g], rc, "rt_set_max_bounces");
        if ((rc = rt_set_background(ctxs[g], bg[0], bg[1], bg[2]))) return die(ctxs[g], rc, "rt_set_background");
    }
    rt_context* ctx = ctxs[0];
    std::vector<uint8_t> rgba((size_t)width * height * 4);
    using clk = std::chrono::steady_clock;
    double delta = 0.0;
    int frame_count = 0;
    size_t step = 0;
    int step_left = steps.empty() ? 0 : steps[0].frames;
    for (int done = 0; done < frames;) {  // Main.cu:471-496
        const int n = std::min(per_call, frames - done);
        auto t0 = clk::now();
        rc = gpus == 1 ? rt_render(ctx, width, height, n, rgba.data())
                       : rt_render_multi(ctxs.data(), gpus, width, height, n, rgba.data());
        if (rc) return die(ctx, rc, "rt_render");
        done += n;
        const double frame_s = std::chrono::duration<double>(clk::now() - t0).count();
        bool quit = false;
        if (!steps.empty()) {  // controls(window, camera, deltaTime, accumulatedFrames)
            const unsigned keys = steps[step].keys;
            if (--step_left == 0 && step + 1 < steps.size()) step_left = steps[++step].frames;
            int flags = 0;
            for (int g = 0; g < gpus; g++) {  // every context keeps the same camera / frame counter
                flags = rt_controls(ctxs[g], keys, (float)(fixed_dt >= 0 ? fixed_dt : frame_s));
                if (flags < 0) return die(ctxs[g], flags, "rt_controls");
            }
            quit = flags & RT_CONTROLS_QUIT;
        }
        delta += frame_s;
        frame_count += n;
        if (delta > 1.0 || done == frames || quit) {  // Main.cu:486-495
            // Main.cu:491 prints accumulatedFrames * samplesPerPixel after
            // accumulatedFrames++ and controls(): the next frame's index
            // (rendered frames since the last reset + 1), which is
            // rt_frame_counter() after rt_controls()
            std::printf("FPS: %d | Samples: %u | kernel %.3f ms\n", (int)(frame_count / delta),
                        rt_frame_counter(ctx) * (unsigned)spp, rt_last_kernel_ms(ctx));
            delta = 0.0;
            frame_count = 0;
        }
        if (quit) break;
    }
    if (!out.empty()) {
        const bool png = out.size() > 4 && out.compare(out.size() - 4, 4, ".png") == 0;
        const bool ok = png ? bwrt::write_png(out, width, height, rgba.data())
                            : bwrt::write_ppm(out, width, height, rgba.data());
        if (!ok) {
            std::fprintf(stderr, "cannot write %s\n", out.c_str());
            return 1;
        }
    }
    rt_camera cam;
    if (!steps.empty() && rt_get_camera(ctx, &cam) == RT_OK)
        std::printf("camera %.9g %.9g %.9g %.9g %.9g\n", cam.position.x, cam.position.y, cam.position.z,
                    cam.angle[0], cam.angle[1]);
    for (rt_context* c : ctxs) rt_destroy(c);
    return 0;
}
