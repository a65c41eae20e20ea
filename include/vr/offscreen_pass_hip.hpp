// offscreen_pass_hip.hpp — header-only C++ drop-in for Vol::Rendering::OffscreenPass
// (reference: src/rendering/offscreen_pass.h:27-148) over the C ABI in vr.h.
//
// The public surface is the reference's, with the same call shapes (offscreen_pass.h:40-54):
//
//   OffscreenPass(VulkanContext *context, uint32_t width, uint32_t height);
//   void record(VkCommandBuffer command_buffer, uint32_t frame_index);
//   void framebuffer_size_changed(uint32_t width, uint32_t height);
//   void volume_dataset_changed(Vol::Data::Dataset &dataset);
//   void slicing_changed(const glm::vec3 &min, const glm::vec3 &max);
//   void transfer_function_changed(const std::vector<glm::uint32_t> &data);
//   VkSampler get_sampler() const;   VkImageView get_image_view() const;
//
// so the reference's callers (vulkan_context.cpp:51, main_pass.cpp:91, imgui_context.cpp:67-74
// and :130-135, importer.cpp:43-46, main_window.cpp:233-238 and :250-257) compile unchanged
// against it (tests/shim/reference_call_shapes.cpp holds those lines verbatim).  The header
// carries no Vulkan, glm or SDL dependency: the host's types come in through a Traits class,
//
//   struct Traits {
//     using Context = VulkanContext;            // constructor's first argument
//     using CommandBuffer = VkCommandBuffer;    // record()'s first argument
//     using Sampler = VkSampler;  using ImageView = VkImageView;
//     static Camera camera();                   // pulled once per record(), as
//                                               // update_uniform_buffer pulls
//                                               // Application::main().get_scene().get_camera()
//                                               // (offscreen_pass.cpp:1155)
//     struct Presenter {                        // the host's colour attachment + sampler
//       Presenter(Context *, uint32_t w, uint32_t h);   // create_color_attachment & co.
//       void resize(uint32_t w, uint32_t h);             // framebuffer_size_changed
//       void present(CommandBuffer, uint32_t frame_index, const FrameImage &);
//                                               // staging buffer + copy_buffer_to_image
//                                               // (offscreen_pass.cpp:1379-1406)
//       Sampler get_sampler() const;  ImageView get_image_view() const;
//     };
//     static uint32_t device_mask();            // OPTIONAL: the GPUs every frame is split
//                                               // over (bit d = device d; vr_create_mask);
//                                               // absent or 0: device 0 alone
//   };
//
// and `using OffscreenPass = Vol::Rendering::Hip::BasicOffscreenPass<Traits>;`.  The HIP
// ray-march renders each frame (the reference's cube draw + volume.frag) into R8G8B8A8_UNORM
// pixels, get_image() is the handle to them, and the Presenter puts them where ImGui samples
// them.  Error behaviour as the reference: every failure throws std::runtime_error, zero
// framebuffer sizes are ignored (offscreen_pass.cpp:237-239), and construction installs the
// 1x1x1 {0} volume and the 1-texel 0xFFFFFFFF transfer function (:118-119).
//
// `HeadlessTraits` (no Vulkan: frames stay in host memory, camera from a callback) serves the
// CLI and tests; `OffscreenPass` below is BasicOffscreenPass<HeadlessTraits>.
#pragma once

#include <cstdint>
#include <functional>
#include <type_traits>
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

// The frame record() produced: W*H R8G8B8A8_UNORM pixels (R in the low byte), row 0 at the
// top, in host memory owned by the pass (valid until the next record() or resize).
struct FrameImage {
    const uint32_t *rgba8 = nullptr;
    uint32_t width = 0, height = 0;
    uint32_t frame_index = 0;  // the frame_index record() was called with
    uint64_t frame = 0;        // frames recorded so far
};

// No Vulkan: frames stay in host memory; the camera comes from a settable callback.
struct HeadlessTraits {
    using Context = void;
    using CommandBuffer = void *;
    using Sampler = const FrameImage *;
    using ImageView = const FrameImage *;
    static std::function<Camera()> &camera_source()
    {
        static std::function<Camera()> f;
        return f;
    }
    static Camera camera()
    {
        if (!camera_source()) throw std::runtime_error("HeadlessTraits: no camera source set");
        return camera_source()();
    }
    struct Presenter {
        FrameImage last;
        Presenter(Context *, uint32_t, uint32_t) {}
        void resize(uint32_t, uint32_t) { last = FrameImage{}; }
        void present(CommandBuffer, uint32_t, const FrameImage &img) { last = img; }
        Sampler get_sampler() const { return &last; }
        ImageView get_image_view() const { return &last; }
    };
};

// The GPUs a pass renders on: an explicit DeviceMask argument, else Traits::device_mask() when
// the host's Traits declares it, else device 0.  The reference's construction call
// (vulkan_context.cpp:51, `new OffscreenPass(this, 100, 100)`) thus stays unchanged while a
// Traits with device_mask() = 0xFF renders every frame across a node's 8 GPUs.
struct DeviceMask {
    uint32_t bits;
};

namespace detail {
template <class T, class = void>
struct has_device_mask : std::false_type {};
template <class T>
struct has_device_mask<T, std::void_t<decltype(T::device_mask())>> : std::true_type {};
template <class T>
uint32_t traits_device_mask()
{
    if constexpr (has_device_mask<T>::value)
        return (uint32_t)T::device_mask();
    else
        return 0u;
}
inline vr_ctx *create_ctx(uint32_t mask, int device, uint32_t w, uint32_t h)
{
    return mask ? vr_create_mask(mask, w, h) : vr_create(device, w, h);
}
}  // namespace detail

template <class Traits>
class BasicOffscreenPass {
  public:
    using Context = typename Traits::Context;
    using CommandBuffer = typename Traits::CommandBuffer;
    using Sampler = typename Traits::Sampler;
    using ImageView = typename Traits::ImageView;

    // The host's glm clip form (vr_params.depth_zero_to_one, ABI 8).  glm fixes it when it is
    // first included (setup.hpp: GLM_CONFIG_CLIP_CONTROL from GLM_FORCE_DEPTH_ZERO_TO_ONE), so
    // read glm's own configuration when glm came before this header; without glm the default
    // [-1, 1] form -- the reference's build, whose define at offscreen_pass.cpp:3 comes after
    // glm's first include through offscreen_pass.h:3.
    static constexpr int32_t host_depth_zero_to_one()
    {
#if defined(GLM_CONFIG_CLIP_CONTROL) && defined(GLM_CLIP_CONTROL_ZO_BIT)
        return (GLM_CONFIG_CLIP_CONTROL & GLM_CLIP_CONTROL_ZO_BIT) ? 1 : 0;
#else
        return 0;
#endif
    }

    // offscreen_pass.cpp:112-134 (the GPUs: Traits::device_mask() if declared, else `device`)
    explicit BasicOffscreenPass(Context *context, uint32_t width, uint32_t height, int device = 0)
        : ctx_(detail::create_ctx(detail::traits_device_mask<Traits>(), device, width, height)),
          presenter_(context, width, height), width_(width), height_(height)
    {
        if (!ctx_) throw std::runtime_error(std::string("vr_create: ") + vr_last_error(nullptr));
        vr_params_default(&params_);
        params_.depth_zero_to_one = host_depth_zero_to_one();
    }
    // every frame split over the devices of `mask` (vr_create_mask)
    BasicOffscreenPass(Context *context, uint32_t width, uint32_t height, DeviceMask mask)
        : ctx_(vr_create_mask(mask.bits, width, height)), presenter_(context, width, height),
          width_(width), height_(height)
    {
        if (!ctx_) throw std::runtime_error(std::string("vr_create_mask: ") + vr_last_error(nullptr));
        vr_params_default(&params_);
        params_.depth_zero_to_one = host_depth_zero_to_one();
    }
    uint32_t device_mask() const
    {
        uint32_t m = 0;
        vr_get_device_mask(ctx_, &m);
        return m;
    }
    ~BasicOffscreenPass() { vr_destroy(ctx_); }
    BasicOffscreenPass(const BasicOffscreenPass &) = delete;
    BasicOffscreenPass &operator=(const BasicOffscreenPass &) = delete;

    // offscreen_pass.cpp:163-230 + update_uniform_buffer :1152-1171: pull the camera, render
    // the frame (HIP), hand it to the presenter for this command buffer.
    void record(CommandBuffer command_buffer, uint32_t frame_index)
    {
        const Camera camera = Traits::camera();
        render(camera);
        FrameImage img = get_image();
        img.frame_index = frame_index;
        presenter_.present(command_buffer, frame_index, img);
    }

    void framebuffer_size_changed(uint32_t width, uint32_t height)  // :232-255
    {
        if (width == 0 || height == 0) return;
        check(vr_resize(ctx_, width, height));
        width_ = width;
        height_ = height;
        image_.clear();
        presenter_.resize(width, height);
    }
    // :257-269; DatasetT: Vol::Data::Dataset ({glm::u32vec3 dimensions; float min, max;
    // std::vector<float> data}) or Hip::Dataset
    template <class DatasetT>
    void volume_dataset_changed(DatasetT &dataset)
    {
        check(vr_set_volume(ctx_, dataset.data.data(), VR_DTYPE_F32, dataset.dimensions[0],
                            dataset.dimensions[1], dataset.dimensions[2], dataset.min, dataset.max));
    }
    // :271-277; Vec3: glm::vec3 or anything indexable by [0..2]
    template <class Vec3>
    void slicing_changed(const Vec3 &min, const Vec3 &max)
    {
        const float a[3] = {(float)min[0], (float)min[1], (float)min[2]};
        const float b[3] = {(float)max[0], (float)max[1], (float)max[2]};
        check(vr_set_slicing(ctx_, a, b));
    }
    void transfer_function_changed(const std::vector<uint32_t> &data)  // :279-288
    {
        check(vr_set_transfer_function(ctx_, data.data(), (uint32_t)data.size()));
    }

    // offscreen_pass.h:53-54: the presenter's sampler / view of the frame's image
    Sampler get_sampler() const { return presenter_.get_sampler(); }
    ImageView get_image_view() const { return presenter_.get_image_view(); }
    // the image handle: the last frame's pixels (empty before the first record())
    FrameImage get_image() const
    {
        FrameImage f;
        f.rgba8 = image_.empty() ? nullptr : image_.data();
        f.width = width_;
        f.height = height_;
        f.frame = frames_;
        return f;
    }

    // One frame for an explicit camera into the pass's host image (no presenter).
    const std::vector<uint32_t> &render(const Camera &camera)
    {
        vr_camera cam{};
        for (int i = 0; i < 16; ++i) cam.view[i] = camera.view[i];
        for (int i = 0; i < 3; ++i) cam.position[i] = camera.position[i];
        image_.resize((size_t)width_ * height_);
        check(vr_render(ctx_, &cam, &params_, image_.data(), VR_OUT_RGBA8));
        ++frames_;
        return image_;
    }
    // Same into device memory on a HIP stream (no host round trip), e.g. for Vulkan interop.
    void render_device(const Camera &camera, void *out_dev, void *hip_stream)
    {
        vr_camera cam{};
        for (int i = 0; i < 16; ++i) cam.view[i] = camera.view[i];
        for (int i = 0; i < 3; ++i) cam.position[i] = camera.position[i];
        check(vr_render_device(ctx_, &cam, &params_, out_dev, VR_OUT_RGBA8, 16, 0, 1, hip_stream));
    }

    const std::vector<uint32_t> &image() const { return image_; }
    vr_params &params() { return params_; }  // step, ERT, shading (reference defaults)
    vr_ctx *handle() { return ctx_; }
    typename Traits::Presenter &presenter() { return presenter_; }

  private:
    void check(int rc)
    {
        if (rc != VR_OK) throw std::runtime_error(vr_last_error(ctx_));
    }
    vr_ctx *ctx_;
    typename Traits::Presenter presenter_;
    uint32_t width_, height_;
    uint64_t frames_ = 0;
    vr_params params_{};
    std::vector<uint32_t> image_;
};

// Headless form: OffscreenPass(nullptr, w, h) or OffscreenPass(w, h).
class OffscreenPass : public BasicOffscreenPass<HeadlessTraits> {
  public:
    using BasicOffscreenPass<HeadlessTraits>::BasicOffscreenPass;
    OffscreenPass(uint32_t width, uint32_t height, int device = 0)
        : BasicOffscreenPass<HeadlessTraits>(nullptr, width, height, device)
    {
    }
};

}  // namespace Vol::Rendering::Hip
