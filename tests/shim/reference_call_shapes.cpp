// reference_call_shapes.cpp — the reference's OffscreenPass call sites, compiled against the
// HIP drop-in (include/vr/offscreen_pass_hip.hpp).
//
// The Vulkan, glm, ImGui and Application types below are minimal stand-ins with the
// reference's names and signatures (the real ones live in the reference's SDK/submodules,
// absent here).  Each CALL line inside the marked blocks keeps the reference's own call shape,
// cited file:line.  The integration Traits (what a maintainer adds to the reference) pull the
// camera from Application::main() as update_uniform_buffer does (offscreen_pass.cpp:1155) and
// present each frame through a staging buffer + copy_buffer_to_image (offscreen_pass.cpp:
// 1379-1406), here into a host-side "image".
//
// Built by tests/test_shim.py (CPU: compile + link against lib/libvr_amd.so) and run by the
// GPU test there, which checks the presented pixels against vr_render for the same camera.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <vector>

#include "vr/offscreen_pass_hip.hpp"
#include "vr/vr_host.h"

// ---- stand-ins: Vulkan handles (vulkan_core.h declares them as opaque pointers) -------------
typedef struct VkCommandBuffer_T *VkCommandBuffer;
typedef struct VkSampler_T *VkSampler;
typedef struct VkImageView_T *VkImageView;
typedef struct VkImage_T *VkImage;
enum VkImageLayout { VK_IMAGE_LAYOUT_SHADER_READ_ONLY_OPTIMAL = 5 };
typedef void *VkDescriptorSet;

// ---- stand-ins: glm ---------------------------------------------------------------------------
namespace glm {
using uint32_t = std::uint32_t;
struct vec3 {
    float x = 0, y = 0, z = 0;
    vec3() = default;
    vec3(float a, float b, float c) : x(a), y(b), z(c) {}
    float &operator[](int i) { return (&x)[i]; }
    const float &operator[](int i) const { return (&x)[i]; }
};
struct u32vec3 {
    uint32_t x = 0, y = 0, z = 0;
    uint32_t &operator[](int i) { return (&x)[i]; }
    const uint32_t &operator[](int i) const { return (&x)[i]; }
};
struct mat4 {
    float m[16];
};
inline const float *value_ptr(const mat4 &a) { return a.m; }
inline const float *value_ptr(const vec3 &a) { return &a.x; }
}  // namespace glm

// ---- stand-ins: the reference's data / scene types ------------------------------------------
namespace Vol::Data {
struct Dataset {  // src/data/dataset.h:9-13
    glm::u32vec3 dimensions;
    float min, max;
    std::vector<float> data;
};
}  // namespace Vol::Data

namespace Vol::Scene {
class Camera {  // src/scene/camera.{h,cpp}: orbit camera (here: vr_cam_* from vr_host.h)
  public:
    Camera() { vr_cam_init(&oc_); }
    void rotate(float dx, float dy) { vr_cam_rotate(&oc_, dx, dy); }
    glm::mat4 get_view() const
    {
        glm::mat4 v;
        vr_cam_view(&oc_, v.m);
        return v;
    }
    glm::vec3 get_position() const
    {
        float p[3];
        vr_cam_position(&oc_, p);
        return glm::vec3(p[0], p[1], p[2]);
    }
    vr_orbit_camera oc_;
};
struct Scene {
    Camera camera;
    Camera &get_camera() { return camera; }
};
}  // namespace Vol::Scene

namespace Vol::Rendering {
class VulkanContext;
class MainPass {
  public:
    explicit MainPass(VulkanContext *c) : context(c) {}
    uint32_t get_frame_index() const { return frame_index; }
    void render();
    VulkanContext *context;
    uint32_t frame_index = 0;
};
}  // namespace Vol::Rendering

// ---- the integration a maintainer adds: Traits for the drop-in -------------------------------
struct ImageStandIn {  // the colour attachment's pixels as the ImGui pass would sample them
    std::vector<uint32_t> pixels;
    uint32_t width = 0, height = 0;
};

struct VkTraits {
    using Context = Vol::Rendering::VulkanContext;
    using CommandBuffer = VkCommandBuffer;
    using Sampler = VkSampler;
    using ImageView = VkImageView;
    static Vol::Rendering::Hip::Camera camera();  // below: Application::main()...get_camera()
    // the GPUs every frame is split over (offscreen_pass_hip.hpp): set from argv here, as a
    // host would from its configuration; 0 = device 0 alone
    static uint32_t &mask()
    {
        static uint32_t m = 0;
        return m;
    }
    static uint32_t device_mask() { return mask(); }
    struct Presenter {
        ImageStandIn color;  // create_color_attachment (offscreen_pass.cpp:290-382)
        std::vector<uint32_t> staging;
        uint32_t presents = 0;
        Presenter(Context *, uint32_t w, uint32_t h) { resize(w, h); }
        void resize(uint32_t w, uint32_t h)  // framebuffer_size_changed re-creates it
        {
            color.width = w;
            color.height = h;
            color.pixels.assign((size_t)w * h, 0u);
        }
        void present(CommandBuffer, uint32_t, const Vol::Rendering::Hip::FrameImage &img)
        {
            // create_buffer + memcpy into the mapped staging buffer, transition_image_layout
            // (UNDEFINED -> TRANSFER_DST), copy_buffer_to_image(staging, color.image, extent)
            // (offscreen_pass.cpp:1379-1406), transition to SHADER_READ_ONLY_OPTIMAL
            staging.assign(img.rgba8, img.rgba8 + (size_t)img.width * img.height);
            color.pixels = staging;
            ++presents;
        }
        VkSampler get_sampler() const { return reinterpret_cast<VkSampler>(0x5A); }
        VkImageView get_image_view() const
        {
            return reinterpret_cast<VkImageView>(const_cast<ImageStandIn *>(&color));
        }
    };
};

namespace Vol::Rendering {
using OffscreenPass = Hip::BasicOffscreenPass<VkTraits>;

class VulkanContext {
  public:
    VulkanContext();
    ~VulkanContext()
    {
        delete offscreen_pass;
        delete main_pass;
    }
    OffscreenPass *get_offscreen_pass() { return offscreen_pass; }
    MainPass *get_main_pass() { return main_pass; }
    MainPass *main_pass = nullptr;
    OffscreenPass *offscreen_pass = nullptr;
};
}  // namespace Vol::Rendering

class Application {  // src/application.h: the singleton the reference pulls state from
  public:
    static Application &main()
    {
        static Application app;
        return app;
    }
    Vol::Scene::Scene &get_scene() { return scene; }
    Vol::Rendering::VulkanContext &get_vulkan_context() { return *vulkan_context; }
    Vol::Scene::Scene scene;
    std::unique_ptr<Vol::Rendering::VulkanContext> vulkan_context;
};

Vol::Rendering::Hip::Camera VkTraits::camera()
{
    // update_uniform_buffer (offscreen_pass.cpp:1155-1165)
    Vol::Scene::Camera &camera = Application::main().get_scene().get_camera();
    Vol::Rendering::Hip::Camera c;
    std::memcpy(c.view, glm::value_ptr(camera.get_view()), sizeof c.view);
    std::memcpy(c.position, glm::value_ptr(camera.get_position()), sizeof c.position);
    return c;
}

static VkDescriptorSet ImGui_ImplVulkan_AddTexture(VkSampler s, VkImageView v, VkImageLayout)
{
    return (s && v) ? reinterpret_cast<VkDescriptorSet>(v) : nullptr;
}

// ==== the reference's call sites (call shapes unchanged) ======================================
Vol::Rendering::VulkanContext::VulkanContext()
{
    main_pass = new MainPass(this);
    offscreen_pass = new OffscreenPass(this, 100, 100);  // vulkan_context.cpp:51
}

void Vol::Rendering::MainPass::render()
{
    VkCommandBuffer command_buffer = nullptr;
    // Record offscreen pass                                main_pass.cpp:90-91
    context->get_offscreen_pass()->record(command_buffer, frame_index);
    frame_index = (frame_index + 1) % 2;  // MAX_FRAMES_IN_FLIGHT (vulkan_context.h:17)
}

static VkDescriptorSet descriptor = nullptr;
static void recreate_viewport_texture(uint32_t width, uint32_t height)  // imgui_context.cpp:55-75
{
    if (width == 0 || height == 0) {
        return;
    }
    Vol::Rendering::OffscreenPass *const offscreen_pass =
        Application::main().get_vulkan_context().get_offscreen_pass();

    offscreen_pass->framebuffer_size_changed(width, height);

    descriptor = ImGui_ImplVulkan_AddTexture(
        offscreen_pass->get_sampler(), offscreen_pass->get_image_view(),
        VK_IMAGE_LAYOUT_SHADER_READ_ONLY_OPTIMAL);
}

static void import_dataset(Vol::Data::Dataset (*parse)())  // importer.cpp:41-46
{
    Vol::Data::Dataset dataset = parse();
    Application::main()
        .get_vulkan_context()
        .get_offscreen_pass()
        ->volume_dataset_changed(dataset);
}

static void update_controls(glm::vec3 min_slice, glm::vec3 max_slice,
                            std::vector<uint32_t> gradient_data)
{
    Application::main()  // main_window.cpp:233-238
        .get_vulkan_context()
        .get_offscreen_pass()
        ->slicing_changed(min_slice, max_slice);
    Application::main()  // main_window.cpp:253-257
        .get_vulkan_context()
        .get_offscreen_pass()
        ->transfer_function_changed(gradient_data);
}
// ==============================================================================================

static Vol::Data::Dataset parse_blob()
{
    Vol::Data::Dataset d;
    d.dimensions.x = 24;
    d.dimensions.y = 20;
    d.dimensions.z = 16;
    d.data.resize(24 * 20 * 16);
    for (uint32_t z = 0; z < 16; ++z)
        for (uint32_t y = 0; y < 20; ++y)
            for (uint32_t x = 0; x < 24; ++x) {
                const float dx = x - 11.5f, dy = y - 9.5f, dz = z - 7.5f;
                d.data[x + 24 * (y + 20 * z)] = std::exp(-(dx * dx + dy * dy + dz * dz) / 40.0f);
            }
    d.min = d.data[0];
    d.max = d.data[0];
    for (float v : d.data) {
        d.min = v < d.min ? v : d.min;
        d.max = v > d.max ? v : d.max;
    }
    return d;
}

// An 8-bit scan as the reference's loader hands it over: NrrdFileParser::convert makes every
// voxel a float (nrrd_file_parser.cpp:49-77), here integers 0..255.
static std::vector<uint8_t> g_u8;
static Vol::Data::Dataset parse_u8_as_float()
{
    Vol::Data::Dataset d;
    d.dimensions.x = 40;
    d.dimensions.y = 36;
    d.dimensions.z = 30;
    g_u8.resize(40 * 36 * 30);
    for (uint32_t z = 0; z < 30; ++z)
        for (uint32_t y = 0; y < 36; ++y)
            for (uint32_t x = 0; x < 40; ++x) {
                const float dx = x - 19.5f, dy = y - 17.5f, dz = z - 14.5f;
                const float v = 255.0f * std::exp(-(dx * dx + dy * dy + dz * dz) / 120.0f);
                g_u8[x + 40 * (y + 36 * z)] = (uint8_t)(v + 0.5f);
            }
    d.data.assign(g_u8.begin(), g_u8.end());
    d.min = 255.0f;
    d.max = 0.0f;
    for (float v : d.data) {
        d.min = v < d.min ? v : d.min;
        d.max = v > d.max ? v : d.max;
    }
    return d;
}

// --u8-dataset: the float Dataset of an 8-bit scan through the unchanged import call
// (importer.cpp:41-46) is stored as 8-bit voxels (an unsigned char march kernel), and its frame
// equals the frame of the same voxels uploaded natively as u8, byte for byte.
static int u8_dataset_check()
{
    Application &app = Application::main();
    app.vulkan_context.reset(new Vol::Rendering::VulkanContext());
    recreate_viewport_texture(96, 80);
    import_dataset(parse_u8_as_float);
    vr_gradient *g = vr_gradient_create();
    vr_gradient_set_alpha_marker(g, 0, 0.0f, 0.0f);
    std::vector<uint32_t> tf(256);
    vr_gradient_discretize(g, tf.size(), tf.data());
    vr_gradient_destroy(g);
    update_controls(glm::vec3(0.0f, 0.0f, 0.0f), glm::vec3(1.0f, 1.0f, 1.0f), tf);
    app.get_scene().get_camera().rotate(100.0f, 60.0f);
    auto *pass = app.get_vulkan_context().get_offscreen_pass();
    app.get_vulkan_context().get_main_pass()->render();
    const std::vector<uint32_t> shown = pass->presenter().color.pixels;
    vr_params p;
    vr_params_default(&p);
    const std::string kname = vr_kernel_name(pass->handle(), &p);
    // the same voxels as native u8 in a context of their own
    Vol::Rendering::Hip::OffscreenPass native(96, 80);
    if (vr_set_volume(native.handle(), g_u8.data(), VR_DTYPE_U8, 40, 36, 30, 0.0f, 255.0f) != VR_OK)
        throw std::runtime_error(vr_last_error(native.handle()));
    float mm[2];
    int st_grp = -1, st_nat = -1;
    vr_debug_volume_info(pass->handle(), nullptr, mm, &st_grp);
    vr_debug_volume_info(native.handle(), nullptr, nullptr, &st_nat);
    if (vr_set_volume(native.handle(), g_u8.data(), VR_DTYPE_U8, 40, 36, 30, mm[0], mm[1]) != VR_OK)
        throw std::runtime_error(vr_last_error(native.handle()));
    native.transfer_function_changed(tf);
    const std::vector<uint32_t> &ref = native.render(VkTraits::camera());
    const bool u8kernel = kname.find("unsigned char") != std::string::npos;
    const bool same = shown == ref;
    std::printf("kernel=%s storage=%d native_storage=%d narrow=%d match=%d\n", kname.c_str(), st_grp,
                st_nat, (int)u8kernel, (int)same);
    return same && u8kernel && st_grp == st_nat ? 0 : 1;
}

int main(int argc, char **argv)
{
    if (argc > 2 && std::string(argv[1]) == "--device-mask")
        VkTraits::mask() = (uint32_t)std::stoul(argv[2], nullptr, 0);
    if (argc > 1 && std::string(argv[1]) == "--u8-dataset") {
        try {
            return u8_dataset_check();
        } catch (std::exception &e) {
            std::fprintf(stderr, "error: %s\n", e.what());
            return 2;
        }
    }
    try {
        Application &app = Application::main();
        app.vulkan_context.reset(new Vol::Rendering::VulkanContext());
        recreate_viewport_texture(0, 10);  // ignored, as the reference
        recreate_viewport_texture(64, 48);
        if (!descriptor) throw std::runtime_error("no descriptor");
        import_dataset(parse_blob);
        vr_gradient *g = vr_gradient_create();  // Gradient::discretize(256) (gradient.cpp:90-108)
        vr_gradient_set_alpha_marker(g, 0, 0.0f, 0.0f);
        std::vector<uint32_t> tf(256);
        vr_gradient_discretize(g, tf.size(), tf.data());
        vr_gradient_destroy(g);
        update_controls(glm::vec3(0.0f, 0.1f, 0.0f), glm::vec3(1.0f, 0.9f, 1.0f), tf);
        app.get_scene().get_camera().rotate(100.0f, 60.0f);
        auto *pass = app.get_vulkan_context().get_offscreen_pass();
        app.get_vulkan_context().get_main_pass()->render();
        app.get_vulkan_context().get_main_pass()->render();
        // the presented image equals an explicit render of the same state and camera
        const auto &shown = pass->presenter().color;
        std::vector<uint32_t> expect = pass->render(VkTraits::camera());
        const bool same = shown.width == 64 && shown.height == 48 && shown.pixels == expect &&
                          pass->presenter().presents == 2 && pass->get_image().frame == 3;
        uint32_t covered = 0;
        for (uint32_t px : shown.pixels) covered += (px & 0xFFFFFFu) != 0x1C1C1Cu;
        std::printf("presented %ux%u frames=%u covered=%u device_mask=0x%x match=%d\n", shown.width,
                    shown.height, pass->presenter().presents, covered, pass->device_mask(), (int)same);
        return same && covered > 0 ? 0 : 1;
    } catch (std::exception &e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 2;
    }
}
