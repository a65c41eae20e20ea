// offscreen_pass_hip.hpp — header-only C++ drop-in for Vol::Rendering::OffscreenPass
// (reference: src/rendering/offscreen_pass.h:27-148) over the C ABI in vr.h.
//
// Same public method names, argument meaning and error behaviour as the reference: every
// failure throws std::runtime_error (the reference throws on every failed vk* call), zero
// framebuffer sizes are ignored, the constructor installs the 1x1x1 {0} volume and the
// 1-texel 0xFFFFFFFF transfer function.  What changes at the boundary:
//   * record(VkCommandBuffer, frame) becomes record(const Camera&) — the reference pulls the
//     camera from Application::main() inside update_uniform_buffer (offscreen_pass.cpp:1155);
//     here the caller passes Camera::get_view()/get_position() explicitly;
//   * get_sampler()/get_image_view() become image(): the RGBA8 frame in host memory (or
//     record_device() into a caller-owned device buffer) for the presentation layer.
// No glm dependency: the caller converts glm types with glm::value_ptr.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "vr.h"

namespace Vol::Rendering::Hip {

// Vol::Data::Dataset (src/data/dataset.h:9-13), float voxels as the reference loader produces.
struct Dataset {
    uint32_t dimensions[3];
    float min, max;
    std::vector<float> data;
};

struct Camera {
    float view[16];     // glm::mat4 column-major (Camera::get_view, camera.cpp:42-48)
    float position[3];  // Camera::get_position (camera.cpp:36-40)
};

class OffscreenPass {
  public:
    OffscreenPass(uint32_t width, uint32_t height, int device = 0)
        : ctx_(vr_create(device, width, height)), width_(width), height_(height)
    {
        if (!ctx_) throw std::runtime_error(std::string("vr_create: ") + vr_last_error(nullptr));
        vr_params_default(&params_);
    }
    ~OffscreenPass() { vr_destroy(ctx_); }
    OffscreenPass(const OffscreenPass &) = delete;
    OffscreenPass &operator=(const OffscreenPass &) = delete;

    // offscreen_pass.cpp:163-230 + 1152-1171: one frame with the current state.
    const std::vector<uint32_t> &record(const Camera &camera)
    {
        vr_camera cam{};
        for (int i = 0; i < 16; ++i) cam.view[i] = camera.view[i];
        for (int i = 0; i < 3; ++i) cam.position[i] = camera.position[i];
        image_.resize((size_t)width_ * height_);
        check(vr_render(ctx_, &cam, &params_, image_.data(), VR_OUT_RGBA8));
        return image_;
    }
    // Same into device memory on a HIP stream (no host round trip), e.g. for Vulkan interop.
    void record_device(const Camera &camera, void *out_dev, void *hip_stream)
    {
        vr_camera cam{};
        for (int i = 0; i < 16; ++i) cam.view[i] = camera.view[i];
        for (int i = 0; i < 3; ++i) cam.position[i] = camera.position[i];
        check(vr_render_device(ctx_, &cam, &params_, out_dev, VR_OUT_RGBA8, 16, 0, 1, hip_stream));
    }

    void framebuffer_size_changed(uint32_t width, uint32_t height)  // :232-255
    {
        if (width == 0 || height == 0) return;
        check(vr_resize(ctx_, width, height));
        width_ = width;
        height_ = height;
    }
    void volume_dataset_changed(Dataset &dataset)  // :257-269
    {
        check(vr_set_volume(ctx_, dataset.data.data(), VR_DTYPE_F32, dataset.dimensions[0],
                            dataset.dimensions[1], dataset.dimensions[2], dataset.min, dataset.max));
    }
    void slicing_changed(const float min[3], const float max[3])  // :271-277
    {
        check(vr_set_slicing(ctx_, min, max));
    }
    void transfer_function_changed(const std::vector<uint32_t> &data)  // :279-288
    {
        check(vr_set_transfer_function(ctx_, data.data(), (uint32_t)data.size()));
    }

    const std::vector<uint32_t> &image() const { return image_; }
    vr_params &params() { return params_; }  // step, ERT, shading (reference defaults)
    vr_ctx *handle() { return ctx_; }

  private:
    void check(int rc)
    {
        if (rc != VR_OK) throw std::runtime_error(vr_last_error(ctx_));
    }
    vr_ctx *ctx_;
    uint32_t width_, height_;
    vr_params params_{};
    std::vector<uint32_t> image_;
};

}  // namespace Vol::Rendering::Hip
