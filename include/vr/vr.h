/*
 * vr.h — C ABI of the MI355X-native volume ray-marcher.
 *
 * This is the drop-in boundary for the reference renderer's raycast pass,
 * `Vol::Rendering::OffscreenPass` (reference: src/rendering/offscreen_pass.h:27-148)
 * together with the fragment shader it drives (res/shaders/volume.frag:21-52) and the
 * Vulkan fixed-function state around it (sampler, cull, depth, blend, UNORM store).
 *
 * Every entry point is `extern "C"`, takes plain pointers and sizes, never throws, and
 * returns 0 on success or a negative errno-style code (VR_E*) on failure; the message of
 * the last failure is available from vr_last_error().  A context is not thread-safe (one
 * host thread calls it, as the reference's single render thread).  vr_create binds one HIP
 * device; vr_create_mask (SURVEY.md §8b `vr_create(int device_mask, ...)`) binds every device
 * of a mask and renders each frame across them inside the context: the volume, TF and slicing
 * are replicated on every device, each device ray-marches its 8-row blocks of the frame
 * (block b -> device b mod N), one RCCL ncclGather per frame collects them on the mask's
 * lowest device over xGMI, and the frame is assembled there.  The unchanged single-threaded
 * host thus drives a node of GPUs through the same calls.  (One process per GPU is the other
 * multi-GPU form: vr_render_device() row-block sharding + vr_dist.h.)  Volume and TF changes
 * wait for the device(s) first (the reference's vkDeviceWaitIdle before a resource swap), so
 * frames still in flight on any stream finish on the old data.
 *
 * Mapping to the reference (each function lists the interface it replaces):
 *   vr_create / vr_create_mask
 *                             OffscreenPass::OffscreenPass(VulkanContext*, w, h)   offscreen_pass.cpp:112-134
 *   vr_destroy                OffscreenPass::~OffscreenPass()                      offscreen_pass.cpp:136-161
 *   vr_resize                 OffscreenPass::framebuffer_size_changed(w, h)        offscreen_pass.cpp:232-255
 *   vr_set_volume             OffscreenPass::volume_dataset_changed(Dataset&)      offscreen_pass.cpp:257-269
 *   vr_set_transfer_function  OffscreenPass::transfer_function_changed(vector<u32>) offscreen_pass.cpp:279-288
 *   vr_set_slicing            OffscreenPass::slicing_changed(vec3 min, vec3 max)   offscreen_pass.cpp:271-277
 *   vr_render / vr_render_device
 *                             OffscreenPass::record(cmd, frame) + update_uniform_buffer
 *                             offscreen_pass.cpp:163-230, 1152-1171; volume.vert:19-24;
 *                             volume.frag:21-52
 *   vr_last_error             (the reference throws std::runtime_error instead)
 */
#ifndef VR_VR_H
#define VR_VR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VR_ABI_VERSION 9

/* ---- status codes (negative errno style) ---- */
#define VR_OK 0
#define VR_EINVAL (-22)  /* bad argument */
#define VR_ENOMEM (-12)  /* device or host allocation failed */
#define VR_ENODEV (-19)  /* no such HIP device / HIP runtime failure */
#define VR_ENODATA (-61) /* render called before a volume/TF is present (never: defaults exist) */
#define VR_EIO (-5)      /* HIP runtime error during a launch or copy */

/* ---- voxel element types accepted by vr_set_volume (NRRD element types the reference's
 *      NrrdFileParser::convert accepts, nrrd_file_parser.cpp:49-66) ---- */
enum vr_dtype {
    VR_DTYPE_I8 = 1,  /* nrrdTypeChar   */
    VR_DTYPE_U8 = 2,  /* nrrdTypeUChar  */
    VR_DTYPE_I16 = 3, /* nrrdTypeShort  */
    VR_DTYPE_U16 = 4, /* nrrdTypeUShort */
    VR_DTYPE_I32 = 5, /* nrrdTypeInt    */
    VR_DTYPE_U32 = 6, /* nrrdTypeUInt   */
    VR_DTYPE_I64 = 7, /* nrrdTypeLLong  */
    VR_DTYPE_U64 = 8, /* nrrdTypeULLong */
    VR_DTYPE_F32 = 9, /* nrrdTypeFloat  */
    VR_DTYPE_F64 = 10 /* nrrdTypeDouble */
};

/* ---- output pixel formats ---- */
enum vr_out_format {
    VR_OUT_RGBA8 = 0,  /* R8G8B8A8_UNORM, the reference colour attachment (offscreen_pass.cpp:293) */
    VR_OUT_RGBA32F = 1 /* float RGBA after blend, before UNORM quantisation (parity format) */
};

/* Camera as the reference's Scene::Camera supplies it to the UBO
 * (offscreen_pass.cpp:1155-1169; camera.cpp:36-48).
 * view: column-major 4x4 (glm layout: element [col*4+row]).
 * fovy_deg/znear/zfar: the projection constants of update_uniform_buffer
 * (perspectiveRH(radians(40), W/H, 0.1, 10)); 0 selects those defaults. */
typedef struct vr_camera {
    float view[16];
    float position[3];
    float fovy_deg;
    float znear;
    float zfar;
} vr_camera;

/* Per-frame render parameters.  Defaults (vr_params_default) equal the reference
 * constants: step 0.005, ray_dist 1.8 (volume.frag:29-30), clear (0.11,0.11,0.11,1)
 * (offscreen_pass.cpp:170-173), no early-ray termination, no shading.
 * Early-ray termination with ert_eps > 0 stops a ray once its transmittance T < ert_eps
 * (bounded colour error <= ert_eps per channel).  T == 0 always terminates: bit-identical.
 * shading = 1 enables the build's central-difference gradient Phong extension
 * (the reference has none; see DESIGN.md "Shading extension"). */
typedef struct vr_params {
    float step;
    float ray_dist;
    float ert_eps;
    int32_t shading;
    float clear_color[4];
    float ambient;
    float diffuse;
    float specular;
    int32_t spec_power; /* integer exponent in [0, 256], binary exponentiation */
    /* Work order of the 16x16-pixel tiles over the chip (speed only, never results):
     * 0 auto (= 4), 1 raster (consecutive tiles round-robin over the 8 XCDs), 2 XCD bands
     * (each XCD a contiguous band of rows), 3 XCD-interleaved 64x64-pixel super-tiles,
     * 4 adaptive: as 3, each XCD's tiles dispatched longest first by the durations the
     * previous launch of the same tile geometry recorded (the first launch runs as 3).
     * 5 (ABI 7, the wavefront work queue) runs as 4 since ABI 8 (measured 2-4x slower). */
    int32_t tile_order;
    /* 1: skip the trilinear fetch of samples proven fully transparent: the sample's cell lies
     * in an 8^3 brick whose stored value range (widened by a rounding margin) maps only to TF
     * texels with alpha 0.  Such a sample composites to exactly nothing (C += rgb*0*T,
     * T *= 1 - 0), so the frame is bit-identical to skip_empty = 0 (DESIGN.md "Empty-space
     * skipping").  The brick classification is rebuilt lazily after a volume or TF change. */
    int32_t skip_empty;
    /* Pixel footprint of one 64-lane wavefront inside the 16x16 workgroup tile (speed only,
     * never results): 0 auto (16x4), 1 8x8, 2 16x4, 3 4x16. */
    int32_t wave_shape;
    /* Frames the caller keeps in flight on different streams (speed only, never results).
     * 0 or 1: frames are rendered one after another, so a small launch (one rank's share of
     * a multi-GPU frame) is bound by its longest rays and runs the lane-group kernel that
     * shortens them.  >= 2: consecutive frames overlap on the device (the reference keeps
     * MAX_FRAMES_IN_FLIGHT = 2, vulkan_context.h:17), the next frame fills the chip while
     * this one drains, and every launch runs the single-lane kernels, which do the least
     * work per sample.  Must be in [0, 16]. */
    int32_t frames_in_flight;
    /* Shading of f32 volumes only: how a frame that reads the precomputed difference field
     * (the shaded dense-row views) holds the central differences.
     * 0 (default): as binary16 scaled by 2^k, k from the volume's min/max so that every
     * difference lies in f16's range (|D| 2^k <= 65504).  The shading normalises the gradient,
     * so the scale cancels exactly; the f16 rounding perturbs the normal by <= 2^-11 relative
     * per difference (C3: RMSE 1.8e-6, max 3.3e-4 against the f32 frame; the oracle restates
     * the rounding bit for bit).  3 instead of 6 loads per shaded sample.
     * 1: exact f32 differences: every frame bit-identical to the f32 oracle.
     * Frames that form the gradient from the density stencil are exact either way. */
    int32_t exact_gradient;
    /* (ABI 8) glm's clip-space depth form of the projection (offscreen_pass.cpp:1166
     * glm::perspectiveRH).  0 (default): the [-1, 1] form (perspectiveRH_NO) -- the reference
     * defines GLM_FORCE_DEPTH_ZERO_TO_ONE at offscreen_pass.cpp:3, after glm was first included
     * through offscreen_pass.h, so the define has no effect there and Vulkan's 0 <= z_ndc <= 1
     * clip puts the effective near plane at 0.198 (not 0.1).  1: the [0, 1] form
     * (perspectiveRH_ZO), for a host built so that the define does take effect: the near
     * plane is the camera's znear.  Only views whose front face lies nearer than 0.198 differ
     * (the camera's radius clamp [0.1, 10], camera.cpp:33, allows them). */
    int32_t depth_zero_to_one;
} vr_params;

/* Work counters of one frame (filled by vr_count_work). */
typedef struct vr_stats {
    uint64_t rays;            /* covered pixels (rays that enter the box)            */
    uint64_t samples;         /* executed density samples (trilinear fetches in slab) */
    uint64_t shaded_samples;  /* samples that also took the 6-tap gradient            */
    uint64_t steps;           /* loop iterations taken (incl. out-of-slab steps)      */
    uint64_t skipped_samples; /* in-slab samples not fetched (skip_empty): samples +
                                 skipped_samples = the reference's sample count          */
} vr_stats;

/* ---- lifecycle ---- */
int vr_abi_version(void);
void vr_params_default(vr_params *p);

/* Create a context on HIP device `device` with a w x h framebuffer.  Like the reference
 * constructor it installs a 1x1x1 volume {0} with min 0 / max 1 and a 1-texel TF
 * 0xFFFFFFFF (offscreen_pass.cpp:118-119).  Returns NULL on failure (see
 * vr_last_error(NULL)). */
typedef struct vr_ctx vr_ctx;
vr_ctx *vr_create(int device, uint32_t width, uint32_t height);
/* A context over every HIP device of device_mask (bit d = device d), e.g. 0xFF for the 8 GPUs
 * of a node: same entry points, same results (every frame byte-identical to a one-device
 * context's), each frame's rows split over the devices (8-row blocks, block-cyclic) and
 * gathered with RCCL on the lowest device of the mask, which holds vr_render_device's output.
 * Every device's memory holds a replica of the volume.  NULL with VR_ENODEV (message naming the
 * missing device) when a device of the mask is not present. */
vr_ctx *vr_create_mask(uint32_t device_mask, uint32_t width, uint32_t height);
void vr_destroy(vr_ctx *ctx);
const char *vr_last_error(const vr_ctx *ctx);

/* framebuffer_size_changed: 0 sizes are ignored (offscreen_pass.cpp:237-239). */
int vr_resize(vr_ctx *ctx, uint32_t width, uint32_t height);
int vr_get_size(const vr_ctx *ctx, uint32_t *width, uint32_t *height);
/* The HIP device index the context renders on (vr_create's `device`; for vr_create_mask the
 * lowest device of the mask, where frames are assembled). */
int vr_get_device(const vr_ctx *ctx, int *device);
/* The devices the context renders on (bit d = device d; one bit for vr_create). */
int vr_get_device_mask(const vr_ctx *ctx, uint32_t *device_mask);

/* ---- inputs (the callee copies; the caller keeps ownership) ---- */

/* volume_dataset_changed: `data` is nx*ny*nz elements of `dtype`, x fastest (NRRD axis 0),
 * host memory.  vmin/vmax are Dataset.min/max (nrrd_file_parser.cpp:39-40).  8- and
 * 16-bit integer and f32 voxels stay native on the device (float(v) is exact); 32/64-bit
 * integers and f64 are converted to f32 exactly as NrrdFileParser::convert does. */
int vr_set_volume(vr_ctx *ctx, const void *data, int dtype, uint32_t nx, uint32_t ny,
                  uint32_t nz, float vmin, float vmax);
/* Same, with `data` already in device memory of this context's device (linear layout).
 * `stream` is a hipStream_t (NULL = default stream); the call is stream-ordered and
 * returns after the bricking kernel was enqueued and completed. */
int vr_set_volume_device(vr_ctx *ctx, const void *data_dev, int dtype, uint32_t nx,
                         uint32_t ny, uint32_t nz, float vmin, float vmax, void *stream);
/* Generate a synthetic volume directly into the bricked device layout (no host copy):
 * kind 0 = sum of Gaussians (f32 or u8), parameters in DESIGN.md.  Used for the
 * multi-GiB benchmark configurations. */
int vr_generate_volume(vr_ctx *ctx, int kind, int dtype, uint32_t nx, uint32_t ny,
                       uint32_t nz, uint32_t seed, float *vmin_out, float *vmax_out);
/* Bytes the bricked volume occupies on the device. */
uint64_t vr_volume_bytes(const vr_ctx *ctx);
/* Debug/test helpers: read the resident volume back as dense float (x fastest, nx*ny*nz
 * floats); query dims, min/max and the storage type (0 u8, 1 i8, 2 u16, 3 i16, 4 f32). */
int vr_debug_read_volume(vr_ctx *ctx, float *out_host);
/* The same voxels in the storage type (u8/i8 -> 1 B, u16/i16 -> 2 B, everything else the f32
 * conversion NrrdFileParser::convert makes), x fastest: 1/4 of the host memory for 8-bit
 * volumes (C5 2048^3: 8 GiB). */
int vr_debug_read_volume_native(vr_ctx *ctx, void *out_host);
int vr_debug_volume_info(const vr_ctx *ctx, uint32_t dims[3], float minmax[2], int *storage);

/* transfer_function_changed: n texels, RGBA8 sRGB, R in the low byte (ImGui packing,
 * gradient.cpp:102-103). */
int vr_set_transfer_function(vr_ctx *ctx, const uint32_t *rgba8_srgb, uint32_t n);

/* slicing_changed: samples are taken only strictly inside (min, max) (volume.frag:39-40). */
int vr_set_slicing(vr_ctx *ctx, const float min_slice[3], const float max_slice[3]);

/* ---- render ---- */

/* Render one full frame synchronously into host memory `out` (W*H*4 bytes for RGBA8,
 * W*H*16 for RGBA32F), row 0 = top (Vulkan framebuffer order).  Replaces
 * OffscreenPass::record + update_uniform_buffer (offscreen_pass.cpp:163-230, 1152-1171) plus
 * the readback a host-side presenter needs.  Frames of >= 256 rows render as 4 row bands
 * whose device->host copies overlap the later bands; returns once `out` holds the frame. */
int vr_render(vr_ctx *ctx, const vr_camera *cam, const vr_params *p, void *out,
              int out_format);

/* Render into DEVICE memory `out_dev` on `stream` (hipStream_t, NULL = default),
 * asynchronously.  Image-space sharding for multi-GPU: the frame's rows are cut into
 * blocks of `row_block` rows and block b is rendered by rank (b % nranks); this rank's
 * blocks are written densely, in order, to `out_dev`: vr_shard_rows_ctx(ctx, H, row_block,
 * nranks) rows x W pixels, sized with the row share in force at this call (vr_set_row_share;
 * with the default 1:1 share that is vr_shard_rows()).  A buffer sized before the share was
 * changed may be too small: size it again (vr_dist_render refuses a changed share).
 * nranks = 1, rank = 0 renders the whole frame.  A vr_create_mask context renders whole frames
 * only (rank 0 of 1; row_block is ignored), into memory of its lowest device, complete once
 * `stream` (a stream of that device) passes this point; p->frames_in_flight (1..8) frames may
 * be in flight across its devices. */
int vr_render_device(vr_ctx *ctx, const vr_camera *cam, const vr_params *p, void *out_dev,
                     int out_format, uint32_t row_block, uint32_t rank, uint32_t nranks,
                     void *stream);
/* Rows each rank writes for (H, row_block, nranks): ceil(ceil(H/row_block)/nranks)*row_block. */
uint32_t vr_shard_rows(uint32_t height, uint32_t row_block, uint32_t nranks);
/* Weighted row shares (ABI 7): block b of a frame split over nranks goes, per period of
 * first_weight + (nranks - 1) * other_weight blocks, to rank 0 for the period's first
 * first_weight blocks and to rank r > 0 for the other_weight blocks after first_weight +
 * (r - 1) * other_weight.  (1, 1), the default, is block b -> rank b % nranks.  A lighter rank 0
 * (e.g. 7, 8) leaves it time for receiving the other shards and assembling the frame.  Applies
 * to vr_render_device with nranks > 1, vr_assemble_rows, vr_count_work and every frame of a
 * vr_create_mask context (whose pipelines are rebuilt); every rank of one frame must use the
 * same weights.  Frames are byte-identical for every choice.  Weights in [1, 64]. */
int vr_set_row_share(vr_ctx *ctx, uint32_t first_weight, uint32_t other_weight);
int vr_get_row_share(const vr_ctx *ctx, uint32_t *first_weight, uint32_t *other_weight);
/* vr_shard_rows under the context's row share: the rows every rank's shard buffer holds (the
 * largest share; ranks with fewer blocks leave their last rows unwritten). */
uint32_t vr_shard_rows_ctx(const vr_ctx *ctx, uint32_t height, uint32_t row_block, uint32_t nranks);
/* Rank-0 assembly after the gather: `gathered_dev` holds nranks shards back to back
 * (rank-major, vr_shard_rows() rows each); writes the H x W frame to `out_dev`. */
int vr_assemble_rows(vr_ctx *ctx, const void *gathered_dev, void *out_dev, int out_format,
                     uint32_t row_block, uint32_t nranks, void *stream);

/* ---- zero-copy presentation ----
 * Import device memory that another API exported as a POSIX file descriptor -- Vulkan:
 * VK_KHR_external_memory_fd (vkGetMemoryFdKHR on the VkDeviceMemory of a device-local buffer
 * or linear image; the reference's copy_buffer_to_image, offscreen_pass.cpp:1379-1406, then
 * copies it into the colour image on the GPU, no host round trip) -- and map `size` bytes at
 * `offset` of it on the context's device (the lowest device of a vr_create_mask context).
 * *dev_ptr can be passed to vr_render_device.  The caller keeps `fd`: neither call closes it
 * (measured on ROCm 7.2: the descriptor is still open after the release), so close it after
 * vr_release_external_memory.  Release the mapping before the exporter frees the memory.
 * The import describes the whole exported allocation as `offset + size` bytes (the HIP import
 * descriptor's size): pass offset + size == the exporter's allocation size (Vulkan
 * VkMemoryAllocateInfo::allocationSize), i.e. map the window that runs to the allocation's
 * end; a smaller window of a larger allocation may fail to import on some drivers. */
typedef struct vr_external_memory vr_external_memory;
int vr_import_memory_fd(vr_ctx *ctx, int fd, uint64_t size, uint64_t offset,
                        vr_external_memory **mem, void **dev_ptr);
int vr_release_external_memory(vr_ctx *ctx, vr_external_memory *mem);

/* ---- derived structures and their memory (ABI 7) ----
 * Beside the bricked volume the library may build, per device, structures that speed particular
 * views up without changing a pixel: the difference field of shaded f32 dense-row views (3x the
 * bricks; binary16 unless vr_params.exact_gradient), a 7x15x8-brick copy for oblique f32 views,
 * a plain copy for unshaded sparse ones and a stencil copy for shaded sparse ones (sparse views
 * whose image rows follow the bricks' rows; DESIGN.md section 4.1 has the policy), and the
 * skip-empty classification.  Each is built on the first frame that wants it (0.6-1.8 ms for 512^3,
 * inside that frame) unless vr_prepare built it first.
 * vr_set_memory_budget caps their total bytes on each device (the bricks never count): a
 * structure that would not fit is not built, and its frames read the bricks instead (the same
 * pixels; with the binary16 field absent a shaded frame forms exact f32 differences, i.e. the
 * exact_gradient = 1 pixels).  An alternative copy may evict the others to fit.  0 keeps only
 * the bricks.  VR_MEMORY_BUDGET_DEFAULT (the default) is 5x the bricked volume's bytes (ABI 9;
 * 4x in ABI 8) (+ the skip-empty classification): the difference field (3x) and the oblique and
 * stencil copies a shaded camera orbit visits, e.g. C3 512^3 f32: 1.6 GB of bricks, at most
 * 8.0 GB derived (the three: 7.1 GB).  VR_MEMORY_BUDGET_UNLIMITED builds whatever fits beside a 2 GiB
 * free-memory reserve (ABI 7's default).  A multi-device context applies the budget on every
 * device (each holds its replica's structures).
 * (ABI 9) A structure that does not fit evicts the least recently read others, one at a time,
 * never one the frame reads; an evicted (or rewritten) structure is released stream-ordered on
 * the evicting frame's stream after every frame in flight on the context's other streams (frame
 * fences), so no frame synchronises the device.  Every frame whose view wanted a structure the
 * budget or free memory refused -- a slower kernel; the same pixels, except that a refused
 * binary16 difference field gives the exact_gradient = 1 pixels -- is counted in
 * vr_memory_info.downgrades, with the refused structure in last_downgrade.
 * Lowering the budget waits for the device and frees the structures.
 * vr_memory_report: the bytes each structure takes now on the (first) device.
 * vr_prepare: builds everything a frame with this camera and params would read, synchronously,
 * so that the next such frame builds nothing (e.g. before a camera move crosses view classes). */
typedef struct vr_memory_info {
    uint64_t volume_bytes;        /* the bricked volume (vr_volume_bytes)              */
    uint64_t field_bytes;         /* difference field                                  */
    uint64_t oblique_copy_bytes;  /* 7x15x8-cell z-pair copy (oblique views)           */
    uint64_t plain_copy_bytes;    /* plain 15^3-cell copy (unshaded sparse views)      */
    uint64_t stencil_copy_bytes;  /* 29^3-cell stencil copy (shaded sparse views)      */
    uint64_t skip_bytes;          /* skip-empty brick ranges + distance field          */
    uint64_t derived_bytes;       /* the sum of the five above: what the budget caps   */
    uint64_t budget_bytes;        /* the budget in force, in bytes (the default's value
                                     for this volume; VR_MEMORY_BUDGET_UNLIMITED)       */
    /* (ABI 9) history since the context was created */
    uint64_t builds;              /* structures built (every (re)build counts)          */
    uint64_t evictions;           /* structures evicted to fit another in the budget    */
    uint64_t downgrades;          /* frames that read the bricks because the budget or
                                     free memory refused the structure their view wanted */
    uint64_t last_downgrade;      /* VR_DERIVED_* refused at the latest downgrade (0: none) */
} vr_memory_info;
enum vr_derived {
    VR_DERIVED_FIELD = 1,          /* difference field            */
    VR_DERIVED_OBLIQUE_COPY = 2,   /* 7x15x8-cell z-pair copy     */
    VR_DERIVED_PLAIN_COPY = 3,     /* plain 15^3-cell copy        */
    VR_DERIVED_STENCIL_COPY = 4,   /* stencil copy                */
    VR_DERIVED_SKIP = 5            /* skip-empty classification   */
};
#define VR_MEMORY_BUDGET_UNLIMITED (~(uint64_t)0)
#define VR_MEMORY_BUDGET_DEFAULT (~(uint64_t)0 - 1)
int vr_set_memory_budget(vr_ctx *ctx, uint64_t bytes);
int vr_memory_report(const vr_ctx *ctx, vr_memory_info *out);
int vr_prepare(vr_ctx *ctx, const vr_camera *cam, const vr_params *p);

/* Count the work of one frame (same camera/params/shard) exactly; synchronous. */
int vr_count_work(vr_ctx *ctx, const vr_camera *cam, const vr_params *p, uint32_t row_block,
                  uint32_t rank, uint32_t nranks, vr_stats *out);

/* Kernel timing: when enabled, every vr_render_device brackets the ray-march kernel with
 * HIP events on the launch stream.  vr_timing_read synchronises and returns the summed
 * kernel milliseconds and launch count since the last reset. */
int vr_timing_enable(vr_ctx *ctx, int enable);
int vr_timing_read(vr_ctx *ctx, double *total_ms, uint64_t *launches);
int vr_timing_reset(vr_ctx *ctx);

/* Name of the ray-march kernel variant vr_render_device launches for the current volume
 * and params (for matching rocprof rows), full frame, single-lane: a serial launch that runs
 * lane groups (march_pair_kernel: small row shares, serial frames of sparse oblique views)
 * is named by the march_kernel variant it stands in for; returns a static string. */
const char *vr_kernel_name(const vr_ctx *ctx, const vr_params *p);

#ifdef __cplusplus
}
#endif

#endif /* VR_VR_H */
