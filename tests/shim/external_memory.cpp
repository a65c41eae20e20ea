// external_memory.cpp — zero-copy presentation through vr_import_memory_fd.
//
// The exporter here stands in for the reference's Vulkan side: a device allocation created
// shareable as a POSIX file descriptor (what vkGetMemoryFdKHR hands over for a VkDeviceMemory
// allocated with VkExportMemoryAllocateInfo), made with HIP's virtual-memory API because no
// Vulkan loader is in the image.  The program
//   1. creates the exporter's allocation (hipMemCreate, POSIX fd handle type) and maps it,
//   2. exports the fd and imports it into the renderer (vr_import_memory_fd),
//   3. renders a frame into the imported pointer (vr_render_device, RGBA8),
//   4. reads the frame back through the EXPORTER's own mapping and compares it byte for byte
//      with vr_render of the same camera (host output),
//   5. releases the import before the exporter unmaps and frees.
// Built by tests/test_shim.py (CPU: compile + link); run by its GPU test.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <unistd.h>
#include <vector>

#include "vr/vr.h"
#include "vr/vr_host.h"

#define HIP_OK(x)                                                                  \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            return 3;                                                              \
        }                                                                          \
    } while (0)
#define VR_CALL(ctx, x)                                                            \
    do {                                                                           \
        if ((x) != VR_OK) {                                                        \
            std::fprintf(stderr, "%s: %s\n", #x, vr_last_error(ctx));              \
            return 2;                                                              \
        }                                                                          \
    } while (0)

int main(int argc, char **argv)
{
    const uint32_t W = 160, H = 120;
    const size_t frame_bytes = (size_t)W * H * 4;
    // --device-mask M: a multi-device context (vr_create_mask); frames land on its lowest device
    const bool group = argc > 2 && std::strcmp(argv[1], "--device-mask") == 0;
    vr_ctx *ctx = group ? vr_create_mask((uint32_t)std::strtoul(argv[2], nullptr, 0), W, H)
                        : vr_create(0, W, H);
    if (!ctx) return 2;
    float mm[2];
    VR_CALL(ctx, vr_generate_volume(ctx, 0, VR_DTYPE_F32, 96, 80, 64, 7, &mm[0], &mm[1]));
    vr_gradient *g = vr_gradient_create();
    vr_gradient_set_alpha_marker(g, 0, 0.0f, 0.0f);
    std::vector<uint32_t> tf(256);
    vr_gradient_discretize(g, tf.size(), tf.data());
    vr_gradient_destroy(g);
    VR_CALL(ctx, vr_set_transfer_function(ctx, tf.data(), (uint32_t)tf.size()));
    vr_orbit_camera oc;
    vr_cam_init(&oc);
    vr_cam_rotate(&oc, 100.0f, 60.0f);
    vr_camera cam;
    vr_cam_to_camera(&oc, &cam);
    vr_params p;
    vr_params_default(&p);
    p.shading = 1;

    // ---- the exporter: a shareable device allocation, mapped in its own address range ----
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gran = 0;
    HIP_OK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
    const size_t offset = gran;  // the frame starts one granule in, as inside a larger heap
    const size_t size = ((offset + frame_bytes + gran - 1) / gran) * gran;
    hipMemGenericAllocationHandle_t handle;
    HIP_OK(hipMemCreate(&handle, size, &prop, 0));
    void *exp_ptr = nullptr;
    HIP_OK(hipMemAddressReserve(&exp_ptr, size, 0, nullptr, 0));
    HIP_OK(hipMemMap(exp_ptr, size, 0, handle, 0));
    hipMemAccessDesc acc{};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    HIP_OK(hipMemSetAccess(exp_ptr, size, &acc, 1));
    HIP_OK(hipMemset(exp_ptr, 0xAB, size));
    HIP_OK(hipDeviceSynchronize());
    int fd = -1;
    HIP_OK(hipMemExportToShareableHandle(&fd, handle, hipMemHandleTypePosixFileDescriptor, 0));

    // ---- the renderer: import, render into it, release ----
    vr_external_memory *mem = nullptr;
    void *frame = nullptr;
    VR_CALL(ctx, vr_import_memory_fd(ctx, fd, frame_bytes, offset, &mem, &frame));
    VR_CALL(ctx, vr_render_device(ctx, &cam, &p, frame, VR_OUT_RGBA8, 8, 0, 1, nullptr));
    HIP_OK(hipDeviceSynchronize());
    // a second frame after a camera move, into the same imported memory
    vr_cam_rotate(&oc, -30.0f, 10.0f);
    vr_cam_to_camera(&oc, &cam);
    VR_CALL(ctx, vr_render_device(ctx, &cam, &p, frame, VR_OUT_RGBA8, 8, 0, 1, nullptr));
    HIP_OK(hipDeviceSynchronize());
    VR_CALL(ctx, vr_release_external_memory(ctx, mem));
    // the caller keeps the fd (vr.h): still open after the release
    const int fd_open = fcntl(fd, F_GETFD) != -1;

    // ---- the exporter reads what it was handed (its own mapping) ----
    std::vector<uint8_t> shown(size);
    HIP_OK(hipMemcpy(shown.data(), exp_ptr, size, hipMemcpyDeviceToHost));
    std::vector<uint8_t> expect(frame_bytes);
    VR_CALL(ctx, vr_render(ctx, &cam, &p, expect.data(), VR_OUT_RGBA8));
    const bool same = std::memcmp(shown.data() + offset, expect.data(), frame_bytes) == 0;
    bool guard = true;  // bytes outside [offset, offset + frame_bytes) untouched
    for (size_t i = 0; i < size; ++i)
        if ((i < offset || i >= offset + frame_bytes) && shown[i] != 0xAB) guard = false;
    uint32_t covered = 0;
    for (size_t i = 0; i < frame_bytes; i += 4) {
        uint32_t px;
        std::memcpy(&px, expect.data() + i, 4);
        covered += (px & 0xFFFFFFu) != 0x1C1C1Cu;
    }

    HIP_OK(hipMemUnmap(exp_ptr, size));
    HIP_OK(hipMemAddressFree(exp_ptr, size));
    HIP_OK(hipMemRelease(handle));
    vr_destroy(ctx);
    std::printf("external frame %ux%u group=%d offset=%zu covered=%u guard=%d match=%d "
                "fd_open_after_release=%d\n", W, H, (int)group, offset, covered, (int)guard,
                (int)same, fd_open);
    if (fd_open) close(fd);
    return same && guard && fd_open && covered > 0 ? 0 : 1;
}
