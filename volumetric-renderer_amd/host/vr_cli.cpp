// vr_cli — headless host for the MI355X ray-march, in C++ above the C ABI.
//
// Plays the role of the reference application's render loop (src/application.cpp:59-95)
// without SDL/ImGui/Vulkan: import a dataset (NrrdFileParser / CsvFileParser restatements),
// set up the orbit camera and the gradient transfer function as the UI would, render frames
// through Vol::Rendering::Hip::OffscreenPass (include/vr/offscreen_pass_hip.hpp) and write the
// RGBA8 image as a binary PPM (the presentation shim of SURVEY.md §8f-3, headless form).
//
//   vr_cli <file.nhdr|file.nrrd|synthetic:N> <out.ppm> [--size WxH] [--radius R]
//          [--rotate DX,DY] [--tf default|demo] [--shading] [--exact-gradient] [--ert EPS]
//          [--skip-empty] [--frames K] [--device-mask M]   (M: render every frame across these GPUs)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/vr/offscreen_pass_hip.hpp"
#include "../../include/vr/vr_host.h"

int main(int argc, char **argv)
{
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s <file.nhdr|synthetic:N> <out.ppm> [--size WxH] [--radius R] "
                             "[--rotate DX,DY] [--tf default|demo] [--shading] [--exact-gradient] [--ert EPS] [--skip-empty] "
                             "[--frames K] [--device-mask M]\n",
                     argv[0]);
        return 2;
    }
    std::string src = argv[1], out = argv[2];
    uint32_t W = 800, H = 600;
    float radius = 3.0f, rx = 0.0f, ry = 0.0f, ert = 0.0f;
    int shading = 0, skip_empty = 0, frames = 1, exact_gradient = 0;
    uint32_t mask = 0;
    std::string tfname = "default";
    for (int i = 3; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "--size" && i + 1 < argc) std::sscanf(argv[++i], "%ux%u", &W, &H);
        else if (a == "--radius" && i + 1 < argc) radius = std::strtof(argv[++i], nullptr);
        else if (a == "--rotate" && i + 1 < argc) std::sscanf(argv[++i], "%f,%f", &rx, &ry);
        else if (a == "--tf" && i + 1 < argc) tfname = argv[++i];
        else if (a == "--shading") shading = 1;
        else if (a == "--exact-gradient") exact_gradient = 1;
        else if (a == "--skip-empty") skip_empty = 1;
        else if (a == "--ert" && i + 1 < argc) ert = std::strtof(argv[++i], nullptr);
        else if (a == "--frames" && i + 1 < argc) frames = std::atoi(argv[++i]);
        else if (a == "--device-mask" && i + 1 < argc) mask = (uint32_t)std::strtoul(argv[++i], nullptr, 0);
        else {
            std::fprintf(stderr, "unknown argument %s\n", a.c_str());
            return 2;
        }
    }
    try {
        Vol::Rendering::Hip::OffscreenPass pass = mask ? Vol::Rendering::Hip::OffscreenPass(
                                                             nullptr, W, H, Vol::Rendering::Hip::DeviceMask{mask})
                                                       : Vol::Rendering::Hip::OffscreenPass(W, H);
        if (src.rfind("synthetic:", 0) == 0) {
            const uint32_t n = (uint32_t)std::atoi(src.c_str() + 10);
            float lo, hi;
            if (vr_generate_volume(pass.handle(), 0, VR_DTYPE_F32, n, n, n, 2024, &lo, &hi) != VR_OK)
                throw std::runtime_error(vr_last_error(pass.handle()));
        } else {
            vr_dataset ds{};
            if (vr_nrrd_load(src.c_str(), &ds) != 0) throw std::runtime_error(vr_host_last_error());
            const int rc = vr_set_volume(pass.handle(), ds.data, ds.dtype, ds.dims[0], ds.dims[1],
                                         ds.dims[2], ds.vmin, ds.vmax);
            vr_dataset_free(&ds);
            if (rc != VR_OK) throw std::runtime_error(vr_last_error(pass.handle()));
        }
        // transfer function as the UI produces it (main_window.cpp:248-257)
        vr_gradient *g = vr_gradient_create();
        if (tfname == "demo") {  // alpha markers (0,0) (0.14,0) (1,1)
            vr_gradient_set_alpha_marker(g, 0, 0.0f, 0.0f);
            float s[4];
            vr_gradient_sample(g, 0.14f, s);
            int idx = vr_gradient_add_alpha_marker(g, 0.14f, s[3]);
            vr_gradient_set_alpha_marker(g, (size_t)idx, 0.14f, 0.0f);
        }
        std::vector<uint32_t> tf(256);
        vr_gradient_discretize(g, tf.size(), tf.data());
        vr_gradient_destroy(g);
        pass.transfer_function_changed(tf);

        vr_orbit_camera oc;
        vr_cam_init(&oc);
        vr_cam_rotate(&oc, rx, ry);
        oc.radius = radius;
        Vol::Rendering::Hip::Camera cam{};
        vr_cam_view(&oc, cam.view);
        vr_cam_position(&oc, cam.position);
        pass.params().shading = shading;
        pass.params().exact_gradient = exact_gradient;
        pass.params().skip_empty = skip_empty;
        pass.params().ert_eps = ert;

        auto t0 = std::chrono::steady_clock::now();
        for (int f = 0; f < frames; ++f) pass.render(cam);
        auto t1 = std::chrono::steady_clock::now();
        const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count() / frames;
        const std::vector<uint32_t> &img = pass.image();
        FILE *fp = std::fopen(out.c_str(), "wb");
        if (!fp) throw std::runtime_error("cannot write " + out);
        std::fprintf(fp, "P6\n%u %u\n255\n", W, H);
        for (uint32_t px : img) {
            const unsigned char rgb[3] = {(unsigned char)(px & 0xFF), (unsigned char)((px >> 8) & 0xFF),
                                          (unsigned char)((px >> 16) & 0xFF)};
            std::fwrite(rgb, 1, 3, fp);
        }
        std::fclose(fp);
        std::printf("rendered %ux%u in %.3f ms/frame (incl. device->host copy) -> %s\n", W, H, ms,
                    out.c_str());
    } catch (std::exception &e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}
