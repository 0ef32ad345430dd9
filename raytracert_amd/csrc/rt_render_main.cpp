// rt_render — command-line replacement for the reference's interactive 'r' key
// (CG_Project/main.cpp:340-411): load an OBJ (init, raytracing.cpp:42-73), render the default
// view through librtamd.so on one GPU and write result.ppm (Image::writeImage, main.cpp:102-128).
//
//   rt_render [--obj cube.obj] [--w 500] [--h 500] [--pf 3] [--depth 10] [--light x,y,z]...
//             [--flags 63] [--device 0] [--out result.ppm]
// Defaults are the reference's: 500x500 window (main.cpp:137-138), pixelfactor 3
// (raytracing.cpp:23), max_lvl 10 (:29), every feature on (:15-20), one light at the camera
// position (0,0,4) (:72).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "raytracert.h"

int main(int argc, char **argv) {
    std::string obj = "cube.obj", out = "result.ppm";
    int w = 500, h = 500, pf = 3, depth = 10, device = 0;
    unsigned flags = RT_ALL_FEATURES;
    std::vector<std::vector<float>> lights;
    for (int i = 1; i < argc; ++i) {
        auto next = [&](const char *name) -> const char * {
            if (i + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", name); std::exit(2); }
            return argv[++i];
        };
        if (!std::strcmp(argv[i], "--obj")) obj = next("--obj");
        else if (!std::strcmp(argv[i], "--out")) out = next("--out");
        else if (!std::strcmp(argv[i], "--w")) w = std::atoi(next("--w"));
        else if (!std::strcmp(argv[i], "--h")) h = std::atoi(next("--h"));
        else if (!std::strcmp(argv[i], "--pf")) pf = std::atoi(next("--pf"));
        else if (!std::strcmp(argv[i], "--depth")) depth = std::atoi(next("--depth"));
        else if (!std::strcmp(argv[i], "--device")) device = std::atoi(next("--device"));
        else if (!std::strcmp(argv[i], "--flags")) flags = static_cast<unsigned>(std::strtoul(next("--flags"), nullptr, 0));
        else if (!std::strcmp(argv[i], "--light")) {
            float x, y, z;
            if (std::sscanf(next("--light"), "%f,%f,%f", &x, &y, &z) != 3) { std::fprintf(stderr, "bad --light\n"); return 2; }
            lights.push_back({x, y, z});
        } else {
            std::fprintf(stderr, "unknown argument %s\n", argv[i]);
            return 2;
        }
    }
    if (lights.empty()) lights.push_back({0.0f, 0.0f, 4.0f});
    rt_params p{};
    p.width = w; p.height = h; p.pfx = pf; p.pfy = pf; p.max_lvl = depth; p.flags = flags;
    p.n_lights = static_cast<int>(lights.size());
    std::vector<float> list;   // any number of lights (more than RT_MAX_LIGHTS go through light_list)
    for (int l = 0; l < p.n_lights; ++l)
        for (int k = 0; k < 3; ++k) list.push_back(lights[l][k]);
    p.light_list = list.data();
    p.camera_pos[0] = 0; p.camera_pos[1] = 0; p.camera_pos[2] = 4;
    if (rt_default_corners(w, h, p.corners) != RT_OK) { std::fprintf(stderr, "%s\n", rt_last_error_string()); return 1; }
    rt_scene *scene = nullptr;
    if (rt_scene_load_obj(obj.c_str(), device, &scene) != RT_OK) {
        std::fprintf(stderr, "load failed: %s\n", rt_last_error_string());
        return 1;
    }
    std::vector<uint8_t> img(static_cast<size_t>(w) * h * 3);
    uint64_t counts[3] = {0, 0, 0};
    const auto t0 = std::chrono::steady_clock::now();
    if (rt_render_tile(scene, &p, 0, 0, w, h, img.data(), nullptr, counts) != RT_OK) {
        std::fprintf(stderr, "render failed: %s\n", rt_last_error_string());
        rt_scene_destroy(scene);
        return 1;
    }
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const double rays = static_cast<double>(counts[0] + counts[1] + counts[2]);
    std::printf("rendered %dx%d pf %d depth %d: %.0f rays (%llu primary, %llu secondary, %llu shadow) in %.3f s = %.2f Mrays/s\n",
                w, h, pf, depth, rays, (unsigned long long)counts[0], (unsigned long long)counts[1],
                (unsigned long long)counts[2], s, rays / s * 1e-6);
    int rc = rt_write_ppm(out.c_str(), w, h, img.data());
    rt_scene_destroy(scene);
    if (rc != RT_OK) { std::fprintf(stderr, "%s\n", rt_last_error_string()); return 1; }
    return 0;
}
