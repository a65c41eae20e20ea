// vr_api.hip — the C ABI (include/vr/vr.h) over the gfx950 kernels.
//
// Restates the resource side of Vol::Rendering::OffscreenPass
// (src/rendering/offscreen_pass.cpp): volume upload (:940-989, here: native dtype, bricked
// on the device), TF upload (:1049-1099, here: sRGB decoded once on the host, staged in LDS by
// the kernel), slicing (:271-277), and update_uniform_buffer (:1152-1171, here: the per-frame
// unprojection matrix the kernel's ray setup uses).  No exceptions cross the ABI; HIP errors
// become negative status codes with a message in vr_last_error().
#include "../../include/vr/vr.h"
#include "../../include/vr/vr_debug.h"
#include "vr_internal.h"
#include "vr_group.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#pragma clang fp contract(off)

using namespace vr;

// vr_render (host output): row bands per frame, each copied to the host while later bands
// render (kHostBandMinRows rows at least, vr_internal.h).  C3 into pageable host memory, ms
// per frame, three rounds (profiles/r03/host_bands/): 4 bands 0.589-0.603 shaded, 0.470-0.488
// unshaded; 8 bands 0.730-0.753 / 0.557-0.560; 16 bands 1.13-1.63 / 0.86-0.90.  A page-locked
// destination changes nothing (4 bands 0.582 against 0.583; 2 bands 0.635-0.655, both
// kinds; profiles/r03/host_pinned/): the bands' own launches, not the copies, set the time.
#ifndef VR_HOST_BANDS
#define VR_HOST_BANDS 4
#endif
constexpr int kRenderBands = VR_HOST_BANDS;

struct vr_ctx {
    int device = 0;
    uint32_t width = 0, height = 0;
    // volume (bricked, native storage type)
    void *bricks = nullptr;
    size_t brick_bytes = 0;
    int storage = ST_F32;
    int layout = ST_F32;  // brick layout code (storage | kQuadFlag for 8-bit yz-quads)
    // the last frame's view (view_dense_rows): image x along the bricks' rows, dense sampling
    bool dense_rows = false;
    double pixel_span = 0.0;  // voxels per pixel step at the volume centre (view_dense_rows)
    double axis_align = 1.0;  // largest |component| of the centre ray's unit direction
    int ray_axis = 2;         // the volume axis of that component (0 x, 1 y, 2 z)
    double row_align = 1.0;   // |x component| of the unit pixel step along the image x axis
    // f32 volumes: further resident copies in the alternative geometries (kAltFlag for
    // oblique views, the plain and stencil copies for sparse ones), each built lazily on the
    // first frame that wants it after a volume change
    struct AltCopy {
        void *bricks = nullptr;  // stream-ordered allocation (hipMallocAsync)
        size_t bytes = 0;
        bool valid = false, failed = false;
        uint64_t used = 0;  // frame_no of the latest frame that read it (eviction order)
    } alt[3];
    uint32_t nx = 1, ny = 1, nz = 1;
    float vmin = 0.0f, vmax = 1.0f;
    // transfer function (decoded, linear float RGBA)
    float4 *tf = nullptr;
    uint32_t tf_n = 0;
    uint32_t *tf_nz = nullptr;  // prefix count of nonzero-alpha texels (tf_n + 1)
    float smin[3] = {0.0f, 0.0f, 0.0f};
    float smax[3] = {1.0f, 1.0f, 1.0f};
    // empty-space classification (skip_empty), built lazily: per-brick value range after a
    // volume change, the brick distance field after a volume or TF change
    float2 *brick_range = nullptr;
    uint8_t *skip_dist = nullptr;  // 2 x nbricks: distance field + pass scratch
    size_t nbricks_alloc = 0;
    bool range_valid = false, dist_valid = false;
    // f32 shading: precomputed central differences (3 x the bricked density), built lazily
    // on the first shaded frame after a volume change; absent when memory is short
    float *grad = nullptr;  // stream-ordered allocation (hipMallocAsync)
    size_t grad_bytes = 0;
    bool grad_valid = false;
    uint64_t grad_used = 0;  // frame_no of the latest frame that read it
    bool grad_half = false;      // the field's precision (vr_params.exact_gradient == 0: binary16)
    int grad_scale_log2 = 0;     // and its scale (field_scale_log2 of the data's own range)
    // f32 storage: the stored voxels' min and max, zero border included (measured on the bricks
    // at upload): the binary16 field's scale comes from these, never from the caller's
    // vmin/vmax, which may be a display window narrower than the data
    float data_lo = 0.0f, data_hi = 1.0f;
    // adaptive tile order (tile_order 4): per launch geometry, the last launch's per-tile
    // durations and the workgroup -> tile permutation built from them
    // Keyed by the launch stream too: frames in flight on different streams each own their
    // duration/permutation buffers, so one stream's order kernel never rewrites a permutation
    // another stream's march kernel is reading.
    // Keyed by the row shard as well: one stream may render several shares of a frame (the
    // row bands of vr_render), each with its own tile durations.
    struct TileSched {
        uint32_t tiles_x = 0, tiles_y = 0, supers_x = 0, per_xcd = 0;
        uint32_t row_block = 0, rank = 0, nranks = 0, share_w0 = 1, share_w = 1;
        int pair = 0;
        uint32_t kernel = 0;  // march variant (tile_kernel_key): its tiles' durations differ
        void *stream = nullptr;
        uint32_t *cost = nullptr, *perm = nullptr, *lists = nullptr;
        bool have_perm = false;
        uint32_t launches = 0;
    };
    std::vector<TileSched> sched;
    // lazily built derived fields (gradient, skip-empty) are produced on the stream of the
    // frame that first needs them; frames on other streams wait for this event
    hipEvent_t built_ev = nullptr;
    bool built_recorded = false;
    // Frame fences (round 6): for each stream that launched frames of this context, an event
    // recorded after its latest frame.  A derived structure that frames in flight may still read
    // is freed (or rewritten) stream-ordered on the evicting frame's stream after that stream
    // waited on every other stream's fence -- no device synchronisation on the frame path.
    struct Fence {
        hipStream_t stream;
        hipEvent_t ev;
        uint64_t used;
        bool external;        // recorded by the caller (vr_dist slot streams, vr_group.h)
        uint64_t build_seen;  // build_gen this stream last waited for (ensure_derived)
    };
    std::vector<Fence> fences;
    uint64_t build_gen = 0;  // records of built_ev so far
    uint64_t frame_no = 0;  // launches so far (the derived structures' recency)
    // derived-structure history (vr_memory_report, ABI 9)
    uint64_t n_builds = 0, n_evictions = 0, n_downgrades = 0;
    uint32_t last_downgrade = 0;
    // scratch
    unsigned long long *counters = nullptr;
    void *frame_dev = nullptr;
    size_t frame_bytes = 0;
    // vr_render (host output): row bands rendered on two streams while finished bands copy
    // to the host on a third, so the PCIe copy hides behind the rest of the frame
    hipStream_t band_stream[2] = {nullptr, nullptr};
    hipStream_t copy_stream = nullptr;
    hipEvent_t band_ev[kRenderBands] = {};
    // timing
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending;
    double timed_ms = 0.0;
    uint64_t timed_launches = 0;
    // launch-policy overrides for tests and A/B experiments (include/vr/vr_debug.h); the
    // product path never reads the process environment
    struct Knobs {
        int pipeline = -1, pair = -1, pair_lanes = 0, grad_field = -1, u8_layout = -1,
            tile_order = 0, narrow = 1, alt = -1;
    } knobs;
    // multi-device context (vr_create_mask): one member context per device of the mask, the
    // volume/TF/slicing replicated on each, frames rendered across them by `group`
    std::vector<vr_ctx *> members;
    vr::Group *group = nullptr;
    uint32_t device_mask = 0;
    hipStream_t group_stream = nullptr;  // vr_render's frame stream (device 0)
    // row blocks over ranks for vr_render_device (nranks > 1), vr_assemble_rows and every frame
    // of a multi-device context (vr_set_row_share; vr_internal.h RowShare)
    RowShare share{1, 1};
    // device bytes the derived structures (difference field, alternative copies, skip-empty
    // classification) may take together (vr_set_memory_budget): VR_MEMORY_BUDGET_DEFAULT
    // (kDerivedBudgetBricks x the bricks), VR_MEMORY_BUDGET_UNLIMITED, or a byte count
    uint64_t budget = VR_MEMORY_BUDGET_DEFAULT;
    std::string err;
};

namespace {

thread_local std::string g_err;

int fail(vr_ctx *c, int code, const std::string &msg)
{
    if (c)
        c->err = msg;
    else
        g_err = msg;
    return code;
}

int hip_fail(vr_ctx *c, hipError_t e, const char *what)
{
    std::string m = std::string(what) + ": " + hipGetErrorString(e);
    // reported here: clear the thread's last error, which the launch helpers read after each
    // launch (a stale one would fail the next, unrelated launch)
    (void)hipGetLastError();
    return fail(c, e == hipErrorOutOfMemory ? VR_ENOMEM : VR_EIO, m);
}

#define HIP_TRY(c, expr, what)                        \
    do {                                              \
        hipError_t _e = (expr);                       \
        if (_e != hipSuccess) return hip_fail(c, _e, what); \
    } while (0)

// Resource swaps wait for the device first, as the reference does (vkDeviceWaitIdle,
// offscreen_pass.cpp:242,260,282): a frame still in flight on any stream may read the volume,
// TF or derived fields that are about to be rewritten or freed.
int wait_idle(vr_ctx *c)
{
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    HIP_TRY(c, hipDeviceSynchronize(), "hipDeviceSynchronize (resource swap)");
    return VR_OK;
}

int storage_for(int dtype)
{
    switch (dtype) {
        case VR_DTYPE_U8: return ST_U8;
        case VR_DTYPE_I8: return ST_I8;
        case VR_DTYPE_U16: return ST_U16;
        case VR_DTYPE_I16: return ST_I16;
        case VR_DTYPE_I32:
        case VR_DTYPE_U32:
        case VR_DTYPE_I64:
        case VR_DTYPE_U64:
        case VR_DTYPE_F32:
        case VR_DTYPE_F64: return ST_F32;  // static_cast<float>, nrrd_file_parser.cpp:67-77
        default: return -1;
    }
}

size_t dtype_size(int dtype)
{
    switch (dtype) {
        case VR_DTYPE_U8:
        case VR_DTYPE_I8: return 1;
        case VR_DTYPE_U16:
        case VR_DTYPE_I16: return 2;
        case VR_DTYPE_I32:
        case VR_DTYPE_U32:
        case VR_DTYPE_F32: return 4;
        default: return 8;
    }
}

// ---- glm restatements (float), offscreen_pass.cpp:1158-1167 ----
void glm_mul(const float *a, const float *b, float *r)
{
    float t[16];
    for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 4; ++i) {
            float acc = a[0 * 4 + i] * b[j * 4 + 0];
            acc = acc + a[1 * 4 + i] * b[j * 4 + 1];
            acc = acc + a[2 * 4 + i] * b[j * 4 + 2];
            acc = acc + a[3 * 4 + i] * b[j * 4 + 3];
            t[j * 4 + i] = acc;
        }
    std::memcpy(r, t, sizeof(t));
}

void perspective_rh_no(float fovy, float aspect, float zn, float zf, float *m)
{
    std::memset(m, 0, 16 * sizeof(float));
    const float th = std::tan(fovy / 2.0f);
    m[0] = 1.0f / (aspect * th);
    m[5] = 1.0f / th;
    m[10] = -(zf + zn) / (zf - zn);
    m[11] = -1.0f;
    m[14] = -(2.0f * zf * zn) / (zf - zn);
}

// glm::perspectiveRH_ZO (GLM_FORCE_DEPTH_ZERO_TO_ONE in effect; vr_params.depth_zero_to_one)
void perspective_rh_zo(float fovy, float aspect, float zn, float zf, float *m)
{
    std::memset(m, 0, 16 * sizeof(float));
    const float th = std::tan(fovy / 2.0f);
    m[0] = 1.0f / (aspect * th);
    m[5] = 1.0f / th;
    m[10] = zf / (zn - zf);
    m[11] = -1.0f;
    m[14] = -(zf * zn) / (zf - zn);
}

void coordinate_conversion(float *m)
{
    const float angle = 90.0f * 0.01745329251994329576923690768489f;
    const float c = std::cos(angle), s = std::sin(angle);
    const float ax = 1.0f, ay = 0.0f, az = 0.0f;
    const float tx = (1.0f - c) * ax, ty = (1.0f - c) * ay, tz = (1.0f - c) * az;
    float rot[16] = {0};
    rot[0] = c + tx * ax;
    rot[1] = tx * ay + s * az;
    rot[2] = tx * az - s * ay;
    rot[4] = ty * ax - s * az;
    rot[5] = c + ty * ay;
    rot[6] = ty * az + s * ax;
    rot[8] = tz * ax + s * ay;
    rot[9] = tz * ay - s * ax;
    rot[10] = c + tz * az;
    rot[15] = 1.0f;
    float sc[16] = {0};
    sc[0] = -1.0f;
    sc[5] = 1.0f;
    sc[10] = 1.0f;
    sc[15] = 1.0f;
    glm_mul(rot, sc, m);
}

bool inverse4d(const double *m, double *inv)
{
    double a[16];
    a[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] +
           m[9] * m[7] * m[14] + m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
    a[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] -
           m[8] * m[7] * m[14] - m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
    a[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] +
           m[8] * m[7] * m[13] + m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
    a[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] -
            m[8] * m[6] * m[13] - m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
    a[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] -
           m[9] * m[3] * m[14] - m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
    a[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] +
           m[8] * m[3] * m[14] + m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
    a[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] -
           m[8] * m[3] * m[13] - m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
    a[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] +
            m[8] * m[2] * m[13] + m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
    a[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] +
           m[5] * m[3] * m[14] + m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
    a[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] -
           m[4] * m[3] * m[14] - m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
    a[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] +
            m[4] * m[3] * m[13] + m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
    a[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] -
            m[4] * m[2] * m[13] - m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
    a[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] -
           m[5] * m[3] * m[10] - m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
    a[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] +
           m[4] * m[3] * m[10] + m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
    a[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] -
            m[4] * m[3] * m[9] - m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
    a[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] +
            m[4] * m[2] * m[9] + m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
    const double det = m[0] * a[0] + m[1] * a[4] + m[2] * a[8] + m[3] * a[12];
    if (det == 0.0) return false;
    const double id = 1.0 / det;
    for (int i = 0; i < 16; ++i) inv[i] = a[i] * id;
    return true;
}

// update_uniform_buffer (offscreen_pass.cpp:1152-1169): proj = perspectiveRH(fovy, W/H, n, f)
// * coordinate_conversion; the kernel needs inverse(proj * view) (volume.vert:23 order).
// zo: glm's [0, 1] clip form (perspectiveRH_ZO) instead of its default [-1, 1] (_NO); the
// kernel clips at 0 <= z_ndc <= 1 (Vulkan) either way, so only the near plane moves.
bool unprojection(const vr_camera *cam, uint32_t W, uint32_t H, bool zo, double *inv)
{
    const float fovy = (cam->fovy_deg > 0.0f ? cam->fovy_deg : 40.0f) *
                       0.01745329251994329576923690768489f;
    const float zn = cam->znear > 0.0f ? cam->znear : 0.1f;
    const float zf = cam->zfar > 0.0f ? cam->zfar : 10.0f;
    const float aspect = (float)W / (float)H;
    float persp[16], conv[16], proj[16], pv[16];
    if (zo)
        perspective_rh_zo(fovy, aspect, zn, zf, persp);
    else
        perspective_rh_no(fovy, aspect, zn, zf, persp);
    coordinate_conversion(conv);
    glm_mul(persp, conv, proj);
    glm_mul(proj, cam->view, pv);
    double pvd[16];
    for (int i = 0; i < 16; ++i) pvd[i] = (double)pv[i];
    return inverse4d(pvd, inv);
}

// R8G8B8A8_SRGB decode (offscreen_pass.cpp:1076): RGB sRGB->linear before filtering.
float srgb_to_linear(uint32_t c8)
{
    const double c = (double)c8 / 255.0;
    const double l = c <= 0.04045 ? c / 12.92 : std::pow((c + 0.055) / 1.055, 2.4);
    return (float)l;
}

// splitmix64 -> uniform [0,1) floats (synthetic volume parameters; restated in
// tests/vrtools.py for the generator test)
struct SplitMix {
    uint64_t s;
    uint64_t next()
    {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    float uniform() { return (float)(next() >> 40) * (1.0f / 16777216.0f); }
};

// Brick layout of an nx x ny x nz volume of storage type st (vr_internal.h kQuadFlag): 8-bit
// volumes of at most kQuadMaxVoxels voxels in yz-quads, larger ones in plain bricks.
// VR_U8_LAYOUT=quad|plain overrides (A/B, tests).
int brick_layout(const vr_ctx *c, int st, uint32_t nx, uint32_t ny, uint32_t nz)
{
    if (!VR_U8_PLAIN || (st != ST_U8 && st != ST_I8)) return st;
    bool quad = (size_t)nx * ny * nz <= kQuadMaxVoxels;
    if (c->knobs.u8_layout >= 0) quad = c->knobs.u8_layout == 1;
    return quad ? (st | kQuadFlag) : st;
}

// The reference converts every NRRD element type to float (nrrd_file_parser.cpp:49-77) and hands
// volume_dataset_changed a float Dataset, so an 8/16-bit scan arrives as floats.  When every
// voxel of a 32/64-bit (non-f64) upload is an integer (not -0.0) that fits an 8- or 16-bit
// type, it is stored in the narrowest such type: float(v) of the stored value is exactly the
// uploaded float, so every frame is the same, bit for bit (knob VR_KNOB_NARROW = 0 keeps f32;
// tests compare both), while the brick layout is the 8/16-bit one (C2/C4/C5: 1.45 B per voxel
// instead of 11 B for f32 z-pairs + difference field).  One read pass over the upload.
int narrow_storage(vr_ctx *c, const void *data_dev, int dtype, size_t count, hipStream_t s,
                   int *st)
{
    int *r = reinterpret_cast<int *>(c->counters);  // scratch: 3 ints
    const int init[3] = {0x7FFFFFFF, (int)0x80000000, 0};
    HIP_TRY(c, hipMemcpyAsync(r, init, sizeof init, hipMemcpyHostToDevice, s), "hipMemcpy(range)");
    HIP_TRY(c, launch_int_range(dtype, data_dev, count, r, s), "integer range kernel");
    int h[3];
    HIP_TRY(c, hipMemcpyAsync(h, r, sizeof h, hipMemcpyDeviceToHost, s), "hipMemcpy(range)");
    HIP_TRY(c, hipStreamSynchronize(s), "integer range sync");
    if (h[2]) return VR_OK;  // fractions, specials or a wide range: stays f32
    if (h[0] >= 0 && h[1] <= 255)
        *st = ST_U8;
    else if (h[0] >= -128 && h[1] <= 127)
        *st = ST_I8;
    else if (h[0] >= 0 && h[1] <= 65535)
        *st = ST_U16;
    else if (h[0] >= -32768 && h[1] <= 32767)
        *st = ST_I16;
    return VR_OK;
}

void free_derived(vr_ctx *c);

// (Re)allocate the bricked volume for layout code `storage`.
int set_bricks(vr_ctx *c, int storage, uint32_t nx, uint32_t ny, uint32_t nz, void **out)
{
    c->range_valid = c->dist_valid = false;  // the bricks are about to be rewritten
    c->grad_valid = false;
    for (auto &a : c->alt) a.valid = a.failed = false;
    const size_t bytes = (size_t)bricks_for(nx, 0, storage) * bricks_for(ny, 1, storage) *
                         bricks_for(nz, 2, storage) * brick_elems(storage) * element_size(storage);
    if (c->bricks && c->brick_bytes == bytes) {
        *out = c->bricks;
        return VR_OK;
    }
    // another volume size: the derived structures' allocations (sized for the old volume) would
    // hold budget and memory they can no longer use (the caller drained the device)
    free_derived(c);
    if (c->bricks) {
        hipFree(c->bricks);
        c->bricks = nullptr;
        c->brick_bytes = 0;
    }
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, bytes + kBrickSlackBytes);  // wide loads past the last brick
    if (e != hipSuccess) return hip_fail(c, e, "hipMalloc(volume bricks)");
    c->bricks = p;
    c->brick_bytes = bytes;
    *out = p;
    return VR_OK;
}

// f32 storage: min and max over every stored element of the bricks (z-pairs duplicate voxels,
// the apron and the border hold zeros), i.e. [min(data, 0), max(data, 0)] -- exactly the
// bound field_scale_log2 needs for the central differences, zero border included.
// Synchronous on `s` (uploads are).
int data_range(vr_ctx *c, hipStream_t s)
{
    c->data_lo = 0.0f;
    c->data_hi = 0.0f;
    if (c->storage != ST_F32) return VR_OK;
    uint32_t *mm = reinterpret_cast<uint32_t *>(c->counters);  // scratch: 2 words
    const uint32_t init[2] = {0xFFFFFFFFu, 0u};
    HIP_TRY(c, hipMemcpyAsync(mm, init, sizeof init, hipMemcpyHostToDevice, s), "hipMemcpy(range)");
    HIP_TRY(c, launch_minmax(ST_F32, c->bricks, c->brick_bytes / sizeof(float),
                             reinterpret_cast<float *>(mm), s),
            "data range kernel");
    uint32_t h[2];
    HIP_TRY(c, hipMemcpyAsync(h, mm, sizeof h, hipMemcpyDeviceToHost, s), "hipMemcpy(range)");
    HIP_TRY(c, hipStreamSynchronize(s), "data range sync");
    auto unorder = [](uint32_t o) {
        const uint32_t u = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
        float f;
        std::memcpy(&f, &u, 4);
        return f;
    };
    c->data_lo = unorder(h[0]);
    c->data_hi = unorder(h[1]);
    return VR_OK;
}

int upload_tf(vr_ctx *c, const uint32_t *tf, uint32_t n)
{
    // entry i + 1 = texel i as {c_i, c_(i+1) - c_i} (0 for the last), entries 0 and n + 1 the
    // clamp-to-edge sentinels {c_0, 0} and {c_(n-1), 0}: tf_lookup's one-fma linear filter
    std::vector<float4> col(n);
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t t = tf[i];
        col[i] = make_float4(srgb_to_linear(t & 0xFFu), srgb_to_linear((t >> 8) & 0xFFu),
                             srgb_to_linear((t >> 16) & 0xFFu), (float)((t >> 24) & 0xFFu) / 255.0f);
    }
    std::vector<float4> lut(2 * ((size_t)n + 2), make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    for (uint32_t i = 0; i < n; ++i) {
        const float4 a = col[i], b = i + 1 < n ? col[i + 1] : a;
        lut[2 * (i + 1)] = a;
        lut[2 * (i + 1) + 1] = make_float4(b.x - a.x, b.y - a.y, b.z - a.z, b.w - a.w);
    }
    lut[0] = col[0];
    lut[2 * ((size_t)n + 1)] = col[n - 1];
    if (c->tf && c->tf_n != n) {
        hipFree(c->tf);
        hipFree(c->tf_nz);
        c->tf = nullptr;
        c->tf_nz = nullptr;
    }
    std::vector<uint32_t> nz(n + 1);
    nz[0] = 0;
    for (uint32_t i = 0; i < n; ++i) nz[i + 1] = nz[i] + ((tf[i] >> 24) != 0u ? 1u : 0u);
    if (!c->tf) {
        HIP_TRY(c, hipMalloc(&c->tf, 2 * ((size_t)n + 2) * sizeof(float4)), "hipMalloc(TF)");
        HIP_TRY(c, hipMalloc(&c->tf_nz, (n + 1) * sizeof(uint32_t)), "hipMalloc(TF alpha prefix)");
    }
    HIP_TRY(c, hipMemcpy(c->tf, lut.data(), lut.size() * sizeof(float4), hipMemcpyHostToDevice),
            "hipMemcpy(TF)");
    HIP_TRY(c, hipMemcpy(c->tf_nz, nz.data(), (n + 1) * sizeof(uint32_t), hipMemcpyHostToDevice),
            "hipMemcpy(TF alpha prefix)");
    c->tf_n = n;
    c->dist_valid = false;
    return VR_OK;
}

int check_params(vr_ctx *c, const vr_params *p)
{
    if (!p) return fail(c, VR_EINVAL, "params is NULL");
    if (!(p->step > 0.0f) || !std::isfinite(p->step))
        return fail(c, VR_EINVAL, "params.step must be a positive finite float");
    if (!(p->ray_dist >= 0.0f) || !std::isfinite(p->ray_dist))
        return fail(c, VR_EINVAL, "params.ray_dist must be finite and >= 0");
    if (p->spec_power < 0 || p->spec_power > 256)
        return fail(c, VR_EINVAL, "params.spec_power must be in [0, 256]");
    if (p->frames_in_flight < 0 || p->frames_in_flight > 16)
        return fail(c, VR_EINVAL, "params.frames_in_flight must be in [0, 16]");
    if (p->exact_gradient != 0 && p->exact_gradient != 1)
        return fail(c, VR_EINVAL, "params.exact_gradient must be 0 or 1");
    if (p->depth_zero_to_one != 0 && p->depth_zero_to_one != 1)
        return fail(c, VR_EINVAL, "params.depth_zero_to_one must be 0 or 1");
    const float n = p->ray_dist / p->step;
    if (n > 1.0e8f) return fail(c, VR_EINVAL, "params.ray_dist / step too large");
    return VR_OK;
}

// View shape for the launch policy, from inverse(proj * view): at the depth where the centre
// pixel's ray passes closest to the volume centre, the world step of one pixel along the image
// x axis.  True when that step runs along the volume's x (|x component| >= 0.9 of it: a
// wavefront's 16-pixel rows follow the bricks' contiguous rows) and spans at most 0.8 voxels
// (neighbouring lanes share cache lines).  *span = that step's length in voxels, *row_align =
// its unit |x component|; *align = the centre ray's largest unit |component|, *axis = its axis.
bool view_dense_rows(const double *inv, uint32_t W, uint32_t nx, uint32_t ny, uint32_t nz,
                     double *span, double *align, int *axis, double *row_align)
{
    *span = 0.0;
    *align = 1.0;
    *axis = 2;
    *row_align = 1.0;
    auto unproject = [&](double x, double z, double out[3]) {
        double h[4];
        for (int r = 0; r < 4; ++r) h[r] = inv[0 * 4 + r] * x + inv[2 * 4 + r] * z + inv[3 * 4 + r];
        for (int a = 0; a < 3; ++a) out[a] = h[a] / h[3];
    };
    double o[3], f[3], o2[3], f2[3], d[3], s[3];
    unproject(0.0, 0.0, o);
    unproject(0.0, 1.0, f);
    const double dx = 2.0 / (double)W;
    unproject(dx, 0.0, o2);
    unproject(dx, 1.0, f2);
    double od = 0.0, dd = 0.0;
    for (int a = 0; a < 3; ++a) {
        d[a] = f[a] - o[a];
        od += o[a] * d[a];
        dd += d[a] * d[a];
    }
    if (!(dd > 0.0)) return false;
    *align = std::fmax(std::fabs(d[0]), std::fmax(std::fabs(d[1]), std::fabs(d[2]))) / std::sqrt(dd);
    *axis = std::fabs(d[0]) >= std::fabs(d[1]) ? (std::fabs(d[0]) >= std::fabs(d[2]) ? 0 : 2)
                                               : (std::fabs(d[1]) >= std::fabs(d[2]) ? 1 : 2);
    const double t = -od / dd;
    double n2 = 0.0, v2 = 0.0;
    const double nv[3] = {(double)nx, (double)ny, (double)nz};
    for (int a = 0; a < 3; ++a) {
        s[a] = (o2[a] + t * (f2[a] - o2[a])) - (o[a] + t * d[a]);
        n2 += s[a] * s[a];
        v2 += (s[a] * nv[a]) * (s[a] * nv[a]);
    }
    if (!(n2 > 0.0)) return false;
    *span = std::sqrt(v2);
    *row_align = std::fabs(s[0]) / std::sqrt(n2);
    return *row_align >= 0.9 && *span <= 0.8;
}

// Shaded f32 frames read the difference field only on dense-row views (view_dense_rows:
// image x along the bricks' rows, <= 0.8 voxels per pixel), where a wavefront's rays share
// the field's cache lines.  Every other view forms the gradient from the density stencil,
// pipelined (use_pipeline): the field is 3x the density's bytes, and off the bricks' rows its
// 6 loads per shaded sample miss more than the stencil's extra loads of the density lines the
// ray already holds.  C3, 3 frames in flight, ms per frame (field -> stencil + pipelined;
// profiles/r02/sparse_view_grad/): default camera r = 3 0.363 -> 0.302, diagonal 0.812 ->
// 0.770, side 0.600 -> 0.587; the fill view keeps the field (stencil: 0.500 -> 0.565).
// With the binary16 field (half: vr_params.exact_gradient == 0, 3 loads per shaded sample)
// the axis-aligned views that are neither oblique nor sparse (want_alt keeps them on the 8^3
// bricks: the side views) read the field too; the diagonal and the default camera keep the
// stencil and their alternative copies.  C3, 3 frames in flight, ms per frame, two rounds
// (profiles/r03/field_views/): side 0.566 / 0.563 -> 0.541 / 0.542; diagonal 0.651 -> 0.80 and
// default camera 0.244 -> 0.307 with the field, so those stay.
// Round 6, measured over a grid of views and along the orbit (yaw x pitch x radius, every
// variant forced; profiles/r06/policy/): rays along the volume's x lose with the field (1.23-
// 1.38x the oblique copy's time at 0.7-0.8 voxels per pixel, even at 0.55), so axis-aligned
// views read it only when the ray runs along y or z; and rays along z keep it on sparse views
// whose image rows follow the bricks' rows (row_align >= kRowsAlign: the stencil copy there
// takes 1.11-1.40x the field's time, while rays along y keep the stencil copy, want_alt).
// Knob VR_KNOB_GRAD_FIELD 0 / 1: the stencil / the field for every view (A/B, tests).
constexpr double kAltAlign = 0.9, kAltSpan = 0.8, kRowsAlign = 0.97;
bool use_grad_field(const vr_ctx *c, bool half)
{
    if (c->storage != ST_F32) return false;
    if (c->knobs.grad_field >= 0) return c->knobs.grad_field == 1;
    if (c->dense_rows) return true;
    if (!half || c->axis_align < kAltAlign || c->ray_axis == 0) return false;
    return c->pixel_span <= kAltSpan || (c->ray_axis == 2 && c->row_align >= kRowsAlign);
}

// Pipelined march (two samples of a ray in flight, vr_kernels.hip PIPE): for launches of
// fewer than kPipelineMaxWaves
// wavefronts -- one rank's share of a multi-GPU frame -- where per-ray latency, not the
// chip's throughput, bounds the kernel (N = 8 rank share: 0.153 -> 0.094 ms); for large
// volumes, whose gathers miss the caches more: >= kPipelineMinBytes bricked bytes, or
// >= kPipelineMinVoxels voxels (C4 1024^3 u8 in plain bricks, 1.6 GB: 421 -> 451 Gsamples/s,
// every view 7-10% faster serially; C2 256^3 u8 loses 4%); and for frames whose view is
// view_dense_rows (3 frames in flight, C3 volume, ms per frame: unshaded fill -11%, oblique
// -12%, top -18%; shaded fill -7%, oblique -7%, top -11%; the side, diagonal and r = 3 views,
// which lose 2-12% unshaded and 2-7% shaded pipelined, are not dense-row views;
// profiles/r02/kernel_choice/inflight3_pipeline_views*.txt); and for every shaded f32 frame:
// off the dense-row views they form the gradient from the stencil (use_grad_field), and
// pipelined that runs 5-8% faster (3 frames in flight: r = 3 0.329 -> 0.306, diagonal
// 0.812 -> 0.770 ms; profiles/r02/sparse_view_grad/).  Knob VR_KNOB_PIPELINE 0/1 overrides.
bool use_pipeline(bool shading, uint32_t tiles, const vr_ctx *c)
{
    if (c->knobs.pipeline >= 0) return c->knobs.pipeline == 1;
    const size_t voxels = (size_t)c->nx * c->ny * c->nz;
    return tiles * (kThreadsPerTile / 64) < kPipelineMaxWaves ||
           c->brick_bytes >= kPipelineMinBytes || voxels >= kPipelineMinVoxels || c->dense_rows ||
           (shading && c->storage == ST_F32);
}

// Lane-pair march (two lanes per ray, each lane pipelined) for SHADED launches of fewer than
// kPairMaxWaves single-lane wavefronts -- a rank's share of a multi-GPU frame, small frames:
// twice the wavefronts, half of each ray's serial chain per lane.  Measured on the C3 rank
// share: N = 8 0.190 -> 0.153 ms, N = 4 0.270 -> 0.227 ms; the full frame and unshaded shares
// stay faster single-lane (tools/shard_sweep.py, profiles/r01/multi_gpu/).  Serial frames
// only (vr_params.frames_in_flight <= 1).  Not for
// skip-empty frames or TFs beyond the LDS copy.  Knob VR_KNOB_PAIR 0/1 overrides (A/B).
int want_alt(const vr_ctx *c, const vr_params *p, const MarchParams &P);
bool use_pair(const vr_ctx *c, const MarchParams &P, const vr_params *p)
{
    if (p->skip_empty || P.tf_n > 256) return false;
    if (c->knobs.pair >= 0) return c->knobs.pair == 1;
    // frames overlapping on the device: the next frame hides this one's tail, so throughput
    // per sample decides and the single-lane kernel wins (N = 8 C3 share with 3 frames in
    // flight: 0.070 against 0.107 ms per frame, tools/inflight_sweep.py)
    if (p->frames_in_flight >= 2) return false;
    if (!p->shading) return false;
    if (P.tiles_x * P.tiles_y * (kThreadsPerTile / 64) < kPairMaxWaves) return true;
    // Full serial frames of sparse views that would read the oblique copy: their rays are few
    // and slow (10-23 ps per sample against 3 on the frame-filling view), so halving each
    // ray's serial chain pays more than the copy's geometry -- 0.64-0.96x the time on such
    // views of the orbit and the round-6 grid, 6% of the orbit's serial time, its slowest
    // frames most; not on rays along z, whose sparse views lost (1.10-1.32x), nor on the field
    // and stencil-copy views (1.06-1.28x) (profiles/r06/policy/pair/).
    if (c->knobs.alt >= 0 || c->layout != ST_F32 || c->dense_rows || c->pixel_span <= kAltSpan ||
        (c->ray_axis == 2 && c->axis_align >= kAltAlign))
        return false;
    return want_alt(c, p, P) == (ST_F32 | kAltFlag);
}

int build_params(vr_ctx *c, const vr_camera *cam, const vr_params *p, void *out,
                 int out_format, uint32_t row_block, uint32_t rank, uint32_t nranks,
                 RowShare share, MarchParams &P)
{
    if (!cam) return fail(c, VR_EINVAL, "camera is NULL");
    int rc = check_params(c, p);
    if (rc) return rc;
    if (out_format != VR_OUT_RGBA8 && out_format != VR_OUT_RGBA32F)
        return fail(c, VR_EINVAL, "unknown out_format");
    if (nranks == 0 || rank >= nranks || row_block == 0)
        return fail(c, VR_EINVAL, "bad shard (row_block, rank, nranks)");
    std::memset(&P, 0, sizeof(P));
    if (!unprojection(cam, c->width, c->height, p->depth_zero_to_one != 0, P.inv))
        return fail(c, VR_EINVAL, "proj * view is singular");
    P.vol = c->bricks;
    P.vol_bytes = c->brick_bytes;
    P.tf = c->tf;
    P.out = out;
    P.counters = c->counters;
    P.fw = (double)c->width;
    P.fh = (double)c->height;
    P.nx = c->nx;
    P.ny = c->ny;
    P.nz = c->nz;
    P.nbx = bricks_for(c->nx, 0, c->layout);
    P.nby = bricks_for(c->ny, 1, c->layout);
    P.fnx = (float)c->nx;
    P.fny = (float)c->ny;
    P.fnz = (float)c->nz;
    P.vmin = c->vmin;
    P.range = c->vmax - c->vmin;
    // reciprocal division domain (div_by_range in vr_kernels.hip)
    P.div_fast = P.range >= 0x1p-40f && P.range < 0x1p100f && std::fabs(c->vmin) < 0x1p100f &&
                 std::fabs(c->vmax) < 0x1p100f;
    P.inv_range = P.div_fast ? 1.0f / P.range : 0.0f;
    P.tf_n = (int32_t)c->tf_n;
    P.tf_nf = (float)c->tf_n;
    for (int a = 0; a < 3; ++a) {
        P.smin[a] = c->smin[a];
        P.smax[a] = c->smax[a];
        P.cam[a] = cam->position[a];
    }
    P.step = p->step;
    P.nsteps = (int32_t)(p->ray_dist / p->step);  // volume.frag:31
    P.ert_eps = p->ert_eps;
    for (int k = 0; k < 4; ++k) P.clear[k] = p->clear_color[k];
    P.ka = p->ambient;
    P.kd = p->diffuse;
    P.ks = p->specular;
    P.spec_power = p->spec_power;
    P.W = c->width;
    P.H = c->height;
    P.row_block = row_block;
    P.rank = rank;
    P.nranks = nranks;
    P.local_rows = share_shard_rows(c->height, row_block, nranks, share);
    P.out_bytes = (unsigned long long)P.local_rows * c->width * (out_format == VR_OUT_RGBA32F ? 16 : 4);
    P.share_w0 = share.w0;
    P.share_w = share.w;
    P.tiles_x = (c->width + 15) / 16;
    P.tiles_y = (P.local_rows + kMarchRows - 1) / kMarchRows;
    // 5 (ABI 7's wavefront queue, measured 2-4x slower and removed in round 5) runs as 4
    P.tile_order = p->tile_order >= 1 && p->tile_order <= 4 ? (uint32_t)p->tile_order : 4u;
    if (p->tile_order == 0 && c->knobs.tile_order >= 1)  // experiment knob: the default order
        P.tile_order = (uint32_t)c->knobs.tile_order;
    // wavefront footprint: 1 8x8, 2 16x4, 3 4x16; auto = 16x4 (x-contiguous brick rows:
    // fewer cache lines per wave-level load; measured -11% on the r=3 view, even on others)
    P.wave_w_shift = p->wave_shape == 1 ? 3u : (p->wave_shape == 3 ? 2u : 4u);
    // a wavefront is at most kMarchRows tall (experiment builds with shorter tiles)
    while ((64u >> P.wave_w_shift) > kMarchRows) ++P.wave_w_shift;
    P.supers_x = (P.tiles_x + kSuper - 1) / kSuper;
    P.supers_total = P.supers_x * ((P.tiles_y + kSuper - 1) / kSuper);
    P.out_format = out_format;
    P.slab_default = c->smin[0] == 0.0f && c->smin[1] == 0.0f && c->smin[2] == 0.0f &&
                     c->smax[0] == 1.0f && c->smax[1] == 1.0f && c->smax[2] == 1.0f;
    c->dense_rows = view_dense_rows(P.inv, c->width, c->nx, c->ny, c->nz, &c->pixel_span,
                                    &c->axis_align, &c->ray_axis, &c->row_align);
    P.pipelined = use_pipeline(p->shading != 0, P.tiles_x * P.tiles_y, c);
    return VR_OK;
}

// After a build on `s`: frames on other streams wait for it (ensure_derived).
// The frame fence of stream s (nullptr: none yet).
vr_ctx::Fence *fence_of(vr_ctx *c, hipStream_t s)
{
    for (auto &x : c->fences)
        if (x.stream == s) return &x;
    return nullptr;
}
int record_build(vr_ctx *c, hipStream_t s)
{
    if (!c->built_ev)
        HIP_TRY(c, hipEventCreateWithFlags(&c->built_ev, hipEventDisableTiming), "hipEventCreate");
    HIP_TRY(c, hipEventRecord(c->built_ev, s), "hipEventRecord(build)");
    c->built_recorded = true;
    ++c->build_gen;
    if (vr_ctx::Fence *f = fence_of(c, s)) f->build_seen = c->build_gen;  // stream order
    return VR_OK;
}

// ---- memory budget of the derived structures (vr_set_memory_budget) ----
constexpr size_t kSkipBytesPerBrick = sizeof(float2) + 2;  // range + distance field + scratch
size_t derived_bytes(const vr_ctx *c)
{
    size_t b = c->grad ? c->grad_bytes : 0;
    for (const auto &a : c->alt)
        if (a.bricks) b += a.bytes + kBrickSlackBytes;
    return b + c->nbricks_alloc * kSkipBytesPerBrick;
}
// The default budget (ABI 9): the difference field (3x the bricks) plus the copies a shaded camera
// orbit visits (the oblique copy, about 1x, and the stencil copy, about 0.5x), plus the skip-empty
// classification -- at C3 the field, the oblique and the stencil copy (7.1 GB beside 1.6 GB of
// bricks) fit, so the reference's drag orbit builds each once and evicts nothing (4x thrashed:
// 4 builds and 4 evictions per lap, profiles/r06/orbit/).  A fourth structure evicts the least
// recently read.
constexpr uint64_t kDerivedBudgetBricks = 5;
uint64_t effective_budget(const vr_ctx *c)
{
    if (c->budget != VR_MEMORY_BUDGET_DEFAULT) return c->budget;
    // + brick_bytes / 32: the skip-empty classification, 10 B per brick of >= 648 B
    return kDerivedBudgetBricks * (uint64_t)c->brick_bytes + (uint64_t)c->brick_bytes / 32 +
           64ull * kBrickSlackBytes;
}
// Would adding `extra` bytes (replacing `replaced` bytes of the same structure) stay within the
// budget?  VR_MEMORY_BUDGET_UNLIMITED always allows; the 2 GiB free-memory reserve applies apart.
bool budget_allows(const vr_ctx *c, size_t extra, size_t replaced)
{
    if (c->budget == VR_MEMORY_BUDGET_UNLIMITED) return true;
    const size_t now = derived_bytes(c) - replaced;
    return now + extra <= effective_budget(c);
}
// ---- frame fences and stream-ordered release of derived structures ----
constexpr size_t kMaxFences = 32;
#ifndef VR_FENCE_SYSTEM_SCOPE  // experiment builds: 1 = default (system-scope) fence events
#define VR_FENCE_SYSTEM_SCOPE 0
#endif
constexpr unsigned kFenceEventFlags =
    hipEventDisableTiming | (VR_FENCE_SYSTEM_SCOPE ? 0u : (unsigned)hipEventDisableSystemFence);
// After this frame's launches on `s`: re-record the stream's fence.  A stream seen for the first
// time gets a fence; past kMaxFences streams the least recently used one's is recycled once its
// last frame has finished (a host wait, only with more than 32 frame streams in use).
int fence_record(vr_ctx *c, hipStream_t s)
{
    vr_ctx::Fence *f = fence_of(c, s);
    if (f && f->external) {  // the caller records it right after this render (vr_dist)
        f->used = c->frame_no;
        return VR_OK;
    }
    if (!f) {
        if (c->fences.size() < kMaxFences) {
            // ordering between this device's streams only: no system-scope release (a default
            // event writes back and invalidates the caches at every record, i.e. every frame;
            // the timing events avoid it for the same reason)
            hipEvent_t e = nullptr;
            HIP_TRY(c, hipEventCreateWithFlags(&e, kFenceEventFlags), "hipEventCreate(fence)");
            c->fences.push_back(vr_ctx::Fence{s, e, 0, false, 0});
            f = &c->fences.back();
        } else {
            vr_ctx::Fence *old = nullptr;
            for (auto &x : c->fences)
                if (!x.external && (!old || x.used < old->used)) old = &x;
            if (!old) return VR_OK;  // every fence external: nothing of ours to record
            HIP_TRY(c, hipEventSynchronize(old->ev), "hipEventSynchronize(fence)");
            old->stream = s;
            old->build_seen = 0;
            f = old;
        }
    }
    f->used = c->frame_no;
    HIP_TRY(c, hipEventRecord(f->ev, s), "hipEventRecord(fence)");
    return VR_OK;
}
// Order `s` after every frame issued so far on every other stream (a structure's readers).  A
// caller may have destroyed a stream it rendered on (ROCm then refuses waits on events recorded
// there, reading the dead stream's capture state): the device is drained instead, once, and the
// context's own fences are dropped (all complete).
int fence_others(vr_ctx *c, hipStream_t s)
{
    for (const auto &x : c->fences)
        if (x.stream != s && hipStreamWaitEvent(s, x.ev, 0) != hipSuccess) {
            (void)hipGetLastError();
            HIP_TRY(c, hipDeviceSynchronize(), "hipDeviceSynchronize (fence fallback)");
            for (size_t i = c->fences.size(); i-- > 0;)
                if (!c->fences[i].external) {
                    hipEventDestroy(c->fences[i].ev);
                    c->fences.erase(c->fences.begin() + (long)i);
                }
            return VR_OK;
        }
    return VR_OK;
}
// Free a derived structure that frames in flight may still read: stream-ordered on `s`, after
// every other stream's latest frame (and, on `s`, after everything enqueued there).
int release_async(vr_ctx *c, void *p, hipStream_t s)
{
    if (!p) return VR_OK;
    if (int rc = fence_others(c, s)) return rc;
    HIP_TRY(c, hipFreeAsync(p, s), "hipFreeAsync(derived structure)");
    return VR_OK;
}
// Evict derived structures, least recently read first, until `extra` more bytes (replacing
// `replaced` bytes of the same structure) fit the budget; never the copy `keep_alt` (alt index,
// or -1) the frame reads, nor the field when `keep_field`.  Returns VR_OK with *fits.
int make_room(vr_ctx *c, size_t extra, size_t replaced, int keep_alt, bool keep_field, hipStream_t s,
              bool *fits)
{
    *fits = budget_allows(c, extra, replaced);
    while (!*fits) {
        int pick = -2;  // -1 the field, 0..2 an alternative copy
        uint64_t oldest = ~0ull;
        if (c->grad && !keep_field && c->grad_used < oldest) {
            pick = -1;
            oldest = c->grad_used;
        }
        for (int i = 0; i < (int)(sizeof c->alt / sizeof c->alt[0]); ++i)
            if (i != keep_alt && c->alt[i].bricks && c->alt[i].used < oldest) {
                pick = i;
                oldest = c->alt[i].used;
            }
        if (pick == -2) return VR_OK;  // nothing left to evict: does not fit
        if (pick == -1) {
            if (int rc = release_async(c, c->grad, s)) return rc;
            c->grad = nullptr;
            c->grad_bytes = 0;
            c->grad_valid = false;
        } else {
            if (int rc = release_async(c, c->alt[pick].bricks, s)) return rc;
            c->alt[pick] = vr_ctx::AltCopy();
        }
        ++c->n_evictions;
        *fits = budget_allows(c, extra, replaced);
    }
    return VR_OK;
}
// Free every derived structure (after the device drained); rebuilt lazily within the budget.
void free_derived(vr_ctx *c)
{
    if (c->grad) (void)hipFreeAsync(c->grad, nullptr);
    c->grad = nullptr;
    c->grad_bytes = 0;
    c->grad_valid = false;
    for (auto &a : c->alt) {
        if (a.bricks) (void)hipFreeAsync(a.bricks, nullptr);
        a = vr_ctx::AltCopy();
    }
    if (c->brick_range) hipFree(c->brick_range);
    if (c->skip_dist) hipFree(c->skip_dist);
    c->brick_range = nullptr;
    c->skip_dist = nullptr;
    c->nbricks_alloc = 0;
    c->range_valid = c->dist_valid = false;
    (void)hipStreamSynchronize(nullptr);
}

// skip_empty: (re)build the per-brick ranges and the distance field when stale, on `s` ahead of
// the march that reads them.
int ensure_skip(vr_ctx *c, MarchParams &P, hipStream_t s)
{
    const size_t nb = (size_t)bricks_for(c->nx, 0, c->layout) * bricks_for(c->ny, 1, c->layout) * bricks_for(c->nz, 2, c->layout);
    if (nb > 0xFFFFFFFFull) return fail(c, VR_EINVAL, "skip_empty: too many bricks");
    if (c->nbricks_alloc != nb && !budget_allows(c, nb * kSkipBytesPerBrick, c->nbricks_alloc * kSkipBytesPerBrick))
        return VR_OK;  // over the memory budget: the frame samples every step (same pixels)
    if (c->nbricks_alloc != nb) {
        if (c->brick_range) hipFree(c->brick_range);
        if (c->skip_dist) hipFree(c->skip_dist);
        c->brick_range = nullptr;
        c->skip_dist = nullptr;
        c->nbricks_alloc = 0;
        c->range_valid = c->dist_valid = false;
        HIP_TRY(c, hipMalloc(&c->brick_range, nb * sizeof(float2)), "hipMalloc(brick ranges)");
        HIP_TRY(c, hipMalloc(&c->skip_dist, 2 * nb), "hipMalloc(skip distance field)");
        c->nbricks_alloc = nb;
    }
    if (!c->range_valid || !c->dist_valid) ++c->n_builds;
    if (!c->range_valid) {
        HIP_TRY(c, launch_brick_range(c->layout, c->bricks, bricks_for(c->nx, 0, c->layout), bricks_for(c->ny, 1, c->layout),
                                      bricks_for(c->nz, 2, c->layout), c->brick_range, s),
                "brick range kernel");
        c->range_valid = true;
        c->dist_valid = false;
    }
    if (!c->dist_valid) {
        HIP_TRY(c, launch_skip_dist(c->brick_range, bricks_for(c->nx, 0, c->layout), bricks_for(c->ny, 1, c->layout),
                                    bricks_for(c->nz, 2, c->layout), c->tf_nz, (int)c->tf_n, c->vmin,
                                    c->vmax - c->vmin, c->skip_dist, c->skip_dist + nb, s),
                "skip distance kernels");
        c->dist_valid = true;
    }
    P.skip_dist = c->skip_dist;
    P.skip_empty = 1;
    return VR_OK;
}

// Shaded f32 frames: (re)build the gradient field when stale.  It needs 3 x the bricked
// density; when that does not fit beside a 2 GiB reserve the kernel forms the differences
// from the 4-wide stencil instead (exact f32 differences).  half: the binary16 field
// (vr_params.exact_gradient == 0), the same 24-B elements.  Switching precision rebuilds the
// field in place after the device has drained (frames in flight may still read it).  Returns
// true when it launched a (re)build on `s`: frames on other streams must then wait for it
// (ensure_derived records the build event).
bool ensure_grad(vr_ctx *c, MarchParams &P, hipStream_t s, bool half, bool *refused)
{
    bool built = false;
    *refused = false;
    if (!use_grad_field(c, half)) return built;
    *refused = true;  // until the field is in place
    const int k = half ? field_scale_log2(c->data_lo, c->data_hi) : 0;
    if (c->grad_valid && (c->grad_half != half || c->grad_scale_log2 != k)) {
        // rewritten in place: after every frame in flight that may still read it
        if (fence_others(c, s) != VR_OK) {
            (void)hipGetLastError();
            return built;
        }
        c->grad_valid = false;
    }
    const size_t bytes = c->brick_bytes / element_size(ST_F32) * kGradElemBytes;
    if (!c->grad || c->grad_bytes != bytes) {
        if (c->grad && release_async(c, c->grad, s) != VR_OK) return built;
        c->grad = nullptr;
        c->grad_bytes = 0;
        c->grad_valid = false;
        // over the budget: the least recently read alternative copies make room (the field
        // serves the dense-row view drawn now; a frame that reads it reads no copy)
        bool fits = false;
        if (make_room(c, bytes, 0, -1, false, s, &fits) != VR_OK || !fits) return built;
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess || free_b < bytes + (2ull << 30))
            return built;
        void *g = nullptr;
        if (hipMallocAsync(&g, bytes, s) != hipSuccess) {
            (void)hipGetLastError();
            return built;
        }
        c->grad = static_cast<float *>(g);
        c->grad_bytes = bytes;
    }
    if (!c->grad_valid) {
        if (launch_grad_field(static_cast<const float *>(c->bricks), c->grad, c->nx, c->ny, c->nz,
                              half, k, s) != hipSuccess)
            return built;
        built = true;
        ++c->n_builds;
        c->grad_valid = true;
        c->grad_half = half;
        c->grad_scale_log2 = k;
    }
    *refused = false;
    P.grad = c->grad;
    P.grad_half = half ? 1 : 0;
    c->grad_used = c->frame_no;
    return built;
}

// The derived fields a frame reads (skip-empty classification, gradient field, alternative
// brick copies), built on `s` when stale.  A frame on another stream may follow before a build
// has run, so builds are chained through one event: every frame first waits on the event
// recorded after the last build (a no-op once it has completed), and a frame that builds
// records it again after its own builds.  Since that frame's stream already waited on the
// previous record, the new record also covers every earlier build, on whichever stream it ran
// (a frame that reads a field built on one stream and builds another on its own, e.g. a
// shaded skip-empty frame, or a later frame reading both).
int ensure_derived(vr_ctx *c, const vr_params *p, MarchParams &P, hipStream_t s, uint32_t *refused)
{
    if (c->built_recorded) {  // once per stream and build record (a wait costs ~3.7 us of host time)
        vr_ctx::Fence *f = fence_of(c, s);
        if (!f || f->build_seen != c->build_gen) {
            HIP_TRY(c, hipStreamWaitEvent(s, c->built_ev, 0), "hipStreamWaitEvent(build)");
            if (f) f->build_seen = c->build_gen;
        }
    }
    const bool r0 = c->range_valid, d0 = c->dist_valid;
    if (p->skip_empty) {
        int rc = ensure_skip(c, P, s);
        if (rc) return rc;
        if (!P.skip_empty) *refused = VR_DERIVED_SKIP;
    }
    // (a precision switch rebuilds a field that was valid on entry: ask ensure_grad, not the flag)
    bool g_refused = false;
    const bool g_built = p->shading && ensure_grad(c, P, s, p->exact_gradient == 0, &g_refused);
    if (g_refused) *refused = VR_DERIVED_FIELD;
    const bool built = (!r0 && c->range_valid) || (!d0 && c->dist_valid) || g_built;
    if (built) return record_build(c, s);
    return VR_OK;
}

// f32 frames of oblique views (the centre ray's direction less than kAltAlign along every axis)
// read the kAltFlag copy (7x15x8-cell bricks), sparse axis-aligned views (more than kAltSpan
// voxels per pixel step) the kWideFlag copy (15x15x8): their rows never straddle a 128-B line,
// and these views' wavefronts put their lanes on different brick rows.  C3, 4 frames in flight,
// ms per frame (profiles/r03/alt_geometry/): diagonal 0.81 (8^3) -> 0.72 (7x7x8) -> 0.68
// (7x15x8), shaded default camera r = 3 0.34 (8^3) -> 0.31 (7x7x8) -> 0.28 (15x15x8); the
// frame-filling, side and top views are 2-4% faster in 8^3 and stay there.  Not for
// skip-empty, difference-field, lane-group or LDS-staged launches (the 8^3 copy keeps those
// structures).  Returns the layout code to launch: c->layout, or ST_F32 | kAltFlag / kWideFlag
// / kPlainF32Flag / kStencilF32Flag.  Knob VR_KNOB_ALT_GEOMETRY: 0 never, 1 the oblique copy, 2
// the z-pair sparse copy, 3 the plain f32 copy, 4 the stencil copy.
// Sparse views read the whole copy from HBM every frame, so unshaded they take the plain f32
// copy (kPlainF32Flag, 15^3-cell bricks, 1.2x the voxels: 0.65 GB for 512^3 against 1.37 GB of
// z-pairs); shaded, the stencil gradient's extra loads cost more there than the bytes save.
// C3 volume, default camera r = 3, 3 frames in flight, ms per frame, two rounds
// (profiles/r03/plain_copy/): unshaded 0.205 / 0.208 (15x15x8 z-pairs) -> 0.191 / 0.191
// (plain); shaded 0.256 / 0.260 -> 0.260 / 0.262.  Plain bricks of 15x15x7 or 31x15x7 cells
// measured 1-2% slower than 15^3.  Shaded, they take the stencil copy (kStencilF32Flag: plain
// voxels with the gradient's apron, vr_internal.h): 0.260 / 0.261 -> 0.232 / 0.230
// (profiles/r03/stencil2/ .. stencil4/); on the diagonal it loses to the oblique copy.
// Round 6 (profiles/r06/policy/: a grid of views and the orbit, every variant forced): the plain
// and stencil copies pay only when the image rows follow the bricks' rows (row_align >=
// kRowsAlign), whatever the ray's tilt -- elsewhere they took 1.5-2.1x the oblique copy's time
// (the orbit's slowest frames, side views at r 2.3-2.5) -- and the oblique copy beats the 8^3
// bricks on every view whose ray runs along x.  So, off the dense-row views: sparse views along
// the rows take the plain / stencil copy; axis-aligned views with the ray along y or z and at
// most kAltSpan voxels per pixel keep the 8^3 bricks; every other view reads the oblique copy.
int want_alt(const vr_ctx *c, const vr_params *p, const MarchParams &P)
{
    if (c->layout != ST_F32 || p->skip_empty || P.pair || P.grad) return c->layout;
    int which = 0;
    if (c->knobs.alt >= 0)
        which = c->knobs.alt;
    else if (!c->dense_rows) {
        if (c->pixel_span > kAltSpan && c->row_align >= kRowsAlign)
            which = p->shading ? 4 : 3;
        else if (c->axis_align >= kAltAlign && c->ray_axis != 0 && c->pixel_span <= kAltSpan)
            which = 0;
        else
            which = 1;
    }
    switch (which) {
        case 1: return ST_F32 | kAltFlag;
        case 3: return ST_F32 | kPlainF32Flag;
        case 4: return ST_F32 | kStencilF32Flag;
        default: return c->layout;
    }
}

int alt_index(int layout)
{
    if (layout & kAltFlag) return 0;
    return (layout & kPlainF32Flag) ? 1 : 2;
}

// Bytes of the copy of the current volume in layout `lay`.
size_t alt_bytes_for(const vr_ctx *c, int lay)
{
    return (size_t)bricks_for(c->nx, 0, lay) * bricks_for(c->ny, 1, lay) * bricks_for(c->nz, 2, lay) *
           brick_elems(lay) * element_size(lay);
}

// The copy in layout `lay` (kAltFlag, kPlainF32Flag or kStencilF32Flag), (re)built on `s` from
// the 8^3 bricks when stale (one pass, launch_rebrick_f32; stream-ordered allocation).  *ready =
// false when it cannot exist (memory short beside a 2 GiB reserve): the launch then stays on
// the 8^3 copy (same frames).
int ensure_alt(vr_ctx *c, int lay, hipStream_t s, bool *ready)
{
    *ready = false;
    vr_ctx::AltCopy &a = c->alt[alt_index(lay)];
    const size_t bytes = alt_bytes_for(c, lay);
    if (a.valid && a.bricks && a.bytes == bytes) {
        *ready = true;
        a.used = c->frame_no;
        return VR_OK;
    }
    if (a.failed) return VR_OK;
    if (!a.bricks || a.bytes != bytes) {
        const size_t had = a.bricks ? a.bytes + kBrickSlackBytes : 0;
        // over the budget: the least recently read other copies, then the field (read only by
        // dense-row views, never by a frame that reads a copy), make room; else this frame reads
        // the 8^3 bricks (same pixels)
        bool fits = false;
        if (int rc = make_room(c, bytes + kBrickSlackBytes, had, alt_index(lay), false, s, &fits))
            return rc;
        if (!fits) return VR_OK;
        if (int rc = release_async(c, a.bricks, s)) return rc;
        a.bricks = nullptr;
        a.bytes = 0;
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess ||
            free_b < bytes + kBrickSlackBytes + (2ull << 30) ||
            hipMallocAsync(&a.bricks, bytes + kBrickSlackBytes, s) != hipSuccess) {
            (void)hipGetLastError();
            a.bricks = nullptr;
            a.failed = true;
            return VR_OK;
        }
        a.bytes = bytes;
    }
    const hipError_t e = launch_rebrick_f32(static_cast<const float *>(c->bricks), a.bricks, c->nx,
                                            c->ny, c->nz, lay, s);
    if (e != hipSuccess) return hip_fail(c, e, "alt geometry copy");
    a.valid = true;
    a.used = c->frame_no;
    ++c->n_builds;
    *ready = true;
    // frames on other streams that read the copy wait for this build (ensure_derived; `s`
    // already waited on the previous build record there)
    return record_build(c, s);
}

// The march variant a launch runs, as part of the schedule key: a shaded, unshaded or
// skip-empty frame of the same geometry on the same stream has other tile durations, so one
// variant's order is not learned from another's (speed only; no measured change on the bench,
// whose runs use fresh streams).
uint32_t tile_kernel_key(const MarchParams &P, bool shading, int layout)
{
    return (shading ? 1u : 0u) | (P.skip_empty ? 2u : 0u) | (P.grad ? 4u : 0u) |
           (P.pipelined ? 8u : 0u) | (P.grad && P.grad_half ? 16u : 0u) | ((uint32_t)layout << 8);
}

// Adaptive tile order (tile_order 4): the schedule entry of this launch geometry (created on
// first use, at most kMaxTileScheds kept, one per geometry, stream and march variant); sets
// P.tile_cost, and P.tile_perm once a permutation exists.
vr_ctx::TileSched *tile_sched(vr_ctx *c, MarchParams &P, void *stream, uint32_t kernel)
{
    if (P.tile_order != 4) return nullptr;
    auto use = [&P](vr_ctx::TileSched &t) {
        P.tile_cost = t.cost;
        if (t.have_perm) {
            P.tile_perm = t.perm;
            P.nperm = 8 * t.per_xcd;
        }
    };
    for (auto &t : c->sched)
        if (t.tiles_x == P.tiles_x && t.tiles_y == P.tiles_y && t.pair == P.pair &&
            t.kernel == kernel &&
            t.stream == stream && t.row_block == P.row_block && t.rank == P.rank &&
            t.nranks == P.nranks && t.share_w0 == P.share_w0 && t.share_w == P.share_w) {
            use(t);
            return &t;
        }
    if (c->sched.size() >= kMaxTileScheds) {
        hipFree(c->sched.front().cost);
        hipFree(c->sched.front().perm);
        hipFree(c->sched.front().lists);
        c->sched.erase(c->sched.begin());
    }
    vr_ctx::TileSched t;
    t.tiles_x = P.tiles_x;
    t.tiles_y = P.tiles_y;
    t.supers_x = P.supers_x;
    t.pair = P.pair;
    t.kernel = kernel;
    t.stream = stream;
    t.row_block = P.row_block;
    t.rank = P.rank;
    t.nranks = P.nranks;
    t.share_w0 = P.share_w0;
    t.share_w = P.share_w;
    // per-XCD tile lists (tile_order 3's super-tile assignment), padded with ~0
    std::vector<std::vector<uint32_t>> xl(8);
    if (VR_LIST_ORDER == 1) {  // super-tile major
        const uint32_t sy_n = (P.tiles_y + kSuper - 1) / kSuper;
        for (uint32_t sy = 0; sy < sy_n; ++sy)
            for (uint32_t sx = 0; sx < P.supers_x; ++sx)
                for (uint32_t w = 0; w < kSuper * kSuper; ++w) {
                    const uint32_t tx = sx * kSuper + w % kSuper, ty = sy * kSuper + w / kSuper;
                    if (tx < P.tiles_x && ty < P.tiles_y)
                        xl[(sy * P.supers_x + sx) & 7u].push_back(ty * P.tiles_x + tx);
                }
    } else {  // frame raster
        for (uint32_t ty = 0; ty < P.tiles_y; ++ty)
            for (uint32_t tx = 0; tx < P.tiles_x; ++tx)
                xl[((ty >> kSuperShift) * P.supers_x + (tx >> kSuperShift)) & 7u].push_back(
                    ty * P.tiles_x + tx);
    }
    for (int x = 0; x < 8; ++x) t.per_xcd = xl[x].size() > t.per_xcd ? (uint32_t)xl[x].size() : t.per_xcd;
    std::vector<uint32_t> lists(8 * (size_t)t.per_xcd, 0xFFFFFFFFu);
    for (int x = 0; x < 8; ++x)
        std::copy(xl[x].begin(), xl[x].end(), lists.begin() + (size_t)x * t.per_xcd);
    const size_t nt = (size_t)P.tiles_x * P.tiles_y;
    // upload on the frame's stream: a plain hipMemcpy from pageable memory may return before its
    // DMA lands, and the order kernel, on a non-blocking stream, would then read recycled memory.
    // Pageable sources are staged before hipMemcpyAsync returns, so the vector may go out of
    // scope.
    hipStream_t hs = static_cast<hipStream_t>(stream);
    if (hipMalloc(&t.cost, nt * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&t.perm, lists.size() * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&t.lists, lists.size() * sizeof(uint32_t)) != hipSuccess ||
        hipMemcpyAsync(t.lists, lists.data(), lists.size() * sizeof(uint32_t),
                       hipMemcpyHostToDevice, hs) != hipSuccess) {
        (void)hipGetLastError();
        hipFree(t.cost);
        hipFree(t.perm);
        hipFree(t.lists);
        return nullptr;  // no adaptive order (tile_order 3 mapping)
    }
    c->sched.push_back(t);
    use(c->sched.back());
    return &c->sched.back();
}

// ---- multi-device contexts (vr_create_mask) ----
bool is_group(const vr_ctx *c) { return c && c->group; }

// Resource swaps on a multi-device context: every issued frame done on every device first.
int group_idle(vr_ctx *c)
{
    std::string m;
    if (vr::group_synchronize(c->group, &m) != VR_OK) return fail(c, VR_EIO, m);
    return VR_OK;
}

// Member 0 holds the new volume: copy its bricks to every other member over xGMI (device to
// device, one stream per destination, all in flight together), so each device renders from
// its own replica (the volume replicated per GPU).
int replicate_volume(vr_ctx *c)
{
    vr_ctx *src = c->members[0];
    const size_t n = c->members.size();
    std::vector<hipStream_t> st(n, nullptr);
    int rc = VR_OK;
    for (size_t k = 1; k < n && rc == VR_OK; ++k) {
        vr_ctx *d = c->members[k];
        if ((rc = wait_idle(d)) != VR_OK) break;
        void *dst = nullptr;
        if ((rc = set_bricks(d, src->layout, src->nx, src->ny, src->nz, &dst)) != VR_OK) break;
        hipError_t e = hipStreamCreateWithFlags(&st[k], hipStreamNonBlocking);
        if (e == hipSuccess)
            e = hipMemcpyPeerAsync(dst, d->device, src->bricks, src->device, src->brick_bytes, st[k]);
        if (e != hipSuccess) rc = hip_fail(c, e, "replicate volume (peer copy)");
        if (rc == VR_OK) {
            d->storage = src->storage;
            d->layout = src->layout;
            d->nx = src->nx;
            d->ny = src->ny;
            d->nz = src->nz;
            d->vmin = src->vmin;
            d->vmax = src->vmax;
            d->data_lo = src->data_lo;
            d->data_hi = src->data_hi;
            d->range_valid = d->dist_valid = d->grad_valid = false;
        }
    }
    for (size_t k = 1; k < n; ++k)
        if (st[k]) {
            hipSetDevice(c->members[k]->device);
            const hipError_t e = hipStreamSynchronize(st[k]);
            if (e != hipSuccess && rc == VR_OK) rc = hip_fail(c, e, "replicate volume (sync)");
            hipStreamDestroy(st[k]);
        }
    hipSetDevice(c->device);
    return rc;
}

// A member's failure reported on the multi-device context.
int member_rc(vr_ctx *c, vr_ctx *m, int rc)
{
    if (rc != VR_OK) c->err = m->err;
    return rc;
}

// include/vr/vr_debug.h knobs
int *knob_slot(vr_ctx *c, int knob)
{
    switch (knob) {
        case VR_KNOB_PIPELINE: return &c->knobs.pipeline;
        case VR_KNOB_PAIR: return &c->knobs.pair;
        case VR_KNOB_PAIR_LANES: return &c->knobs.pair_lanes;
        case VR_KNOB_GRAD_FIELD: return &c->knobs.grad_field;
        case VR_KNOB_U8_LAYOUT: return &c->knobs.u8_layout;
        case VR_KNOB_TILE_ORDER: return &c->knobs.tile_order;
        case VR_KNOB_NARROW: return &c->knobs.narrow;
        case VR_KNOB_ALT_GEOMETRY: return &c->knobs.alt;
        default: return nullptr;
    }
}

bool knob_value_ok(int knob, int v)
{
    switch (knob) {
        case VR_KNOB_PAIR_LANES: return v == 0 || v == 2 || v == 4;
        case VR_KNOB_NARROW: return v == 0 || v == 1;
        case VR_KNOB_ALT_GEOMETRY: return v >= -1 && v <= 4 && v != 2;
        case VR_KNOB_TILE_ORDER: return v >= 0 && v <= 4;
        default: return v >= -1 && v <= 1;
    }
}

#ifdef VR_EXPERIMENTS
// Experiment builds only: seed the knobs from the A/B scripts' environment variables.
void knobs_from_env(vr_ctx *c)
{
    auto flag = [](const char *name, int &dst) {
        if (const char *e = std::getenv(name)) dst = e[0] == '1' ? 1 : 0;
    };
    flag("VR_PIPELINE", c->knobs.pipeline);
    flag("VR_PAIR", c->knobs.pair);
    if (const char *e = std::getenv("VR_PAIR_LANES")) c->knobs.pair_lanes = e[0] == '4' ? 4 : 2;
    if (std::getenv("VR_NO_GRAD_FIELD")) c->knobs.grad_field = 0;
    if (std::getenv("VR_GRAD_FIELD_ALWAYS")) c->knobs.grad_field = 1;
    if (const char *e = std::getenv("VR_U8_LAYOUT")) c->knobs.u8_layout = e[0] == 'q' ? 1 : 0;
    if (const char *e = std::getenv("VR_TILE_ORDER_DEFAULT"))
        if (e[0] >= '1' && e[0] <= '4') c->knobs.tile_order = e[0] - '0';
}
#endif

hipEvent_t pooled_event(vr_ctx *c)
{
    if (!c->ev_pool.empty()) {
        hipEvent_t e = c->ev_pool.back();
        c->ev_pool.pop_back();
        return e;
    }
    // timing-only events: no system-scope fence when recorded.  The default event's fence
    // writes back and invalidates the caches between this frame's kernel and the next one on
    // the stream (C3 with 3 frames in flight: 5-10% per frame with timing on)
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
    return e;
}

// A multi-device context over `devices` (member m on devices[m]; member 0 assembles).
vr_ctx *create_members(const std::vector<int> &devices, uint32_t width, uint32_t height,
                       int exchange)
{
    if (width == 0 || height == 0) {
        fail(nullptr, VR_EINVAL, "framebuffer size must be non-zero");
        return nullptr;
    }
    vr_ctx *c = new (std::nothrow) vr_ctx();
    if (!c) {
        fail(nullptr, VR_ENOMEM, "out of host memory");
        return nullptr;
    }
    c->device = devices[0];
    for (int d : devices)
        if (d < 32) c->device_mask |= 1u << d;  // vr_get_device_mask reports devices 0..31
    c->width = width;
    c->height = height;
#ifdef VR_EXPERIMENTS
    knobs_from_env(c);
#endif
    for (int d : devices) {
        vr_ctx *m = vr_create(d, width, height);  // the reference constructor's placeholders
        if (!m) {
            const std::string e = g_err;
            vr_destroy(c);
            fail(nullptr, VR_ENODEV, "device " + std::to_string(d) + ": " + e);
            return nullptr;
        }
        m->knobs = c->knobs;
        c->members.push_back(m);
    }
    std::string err;
    c->group = vr::group_create(c->members, exchange, &err);
    if (!c->group) {
        vr_destroy(c);
        fail(nullptr, VR_ENODEV, "multi-device context: " + err);
        return nullptr;
    }
    hipSetDevice(c->device);
    return c;
}

}  // namespace

bool vr::is_multi_device(const vr_ctx *c) { return is_group(c); }

int vr::register_stream_fence(vr_ctx *c, hipStream_t stream, hipEvent_t ev)
{
    if (vr_ctx::Fence *f = fence_of(c, stream)) {
        // the context's own fence of this stream: wait for its last record (the caller's event
        // covers only the caller's frames; setup time, rare)
        if (!f->external) {
            HIP_TRY(c, hipEventSynchronize(f->ev), "hipEventSynchronize(fence)");
            hipEventDestroy(f->ev);
        }
        *f = vr_ctx::Fence{stream, ev, c->frame_no, true, 0};
        return VR_OK;
    }
    c->fences.push_back(vr_ctx::Fence{stream, ev, c->frame_no, true, 0});
    return VR_OK;
}

// Fold the kernel-timing event pairs into the totals (vr_timing_read), e.g. before the streams
// they were recorded on are destroyed: ROCm refuses to synchronise an event whose recording
// stream is gone.  The caller has drained those streams.
void vr::settle_timing(vr_ctx *c)
{
    for (auto &pr : c->ev_pending) {
        float ms = 0.0f;
        if (hipEventSynchronize(pr.second) == hipSuccess &&
            hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) {
            c->timed_ms += ms;
            c->timed_launches++;
        } else {
            (void)hipGetLastError();
        }
        c->ev_pool.push_back(pr.first);
        c->ev_pool.push_back(pr.second);
    }
    c->ev_pending.clear();
}

void vr::unregister_stream_fence(vr_ctx *c, hipStream_t stream)
{
    for (size_t i = 0; i < c->fences.size(); ++i)
        if (c->fences[i].stream == stream && c->fences[i].external) {
            c->fences.erase(c->fences.begin() + (long)i);
            return;
        }
}

namespace {
int render_device_impl(vr_ctx *c, const vr_camera *cam, const vr_params *p, void *out_dev,
                       int out_format, uint32_t row_block, uint32_t rank, uint32_t nranks,
                       RowShare share, void *stream, bool launch = true);
}

extern "C" {

int vr_abi_version(void) { return VR_ABI_VERSION; }

void vr_params_default(vr_params *p)
{
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->step = 0.005f;      // volume.frag:30
    p->ray_dist = 1.8f;    // volume.frag:29
    p->ert_eps = 0.0f;     // reference: no early-ray termination
    p->shading = 0;        // reference: no shading
    p->clear_color[0] = 0.11f;  // offscreen_pass.cpp:171
    p->clear_color[1] = 0.11f;
    p->clear_color[2] = 0.11f;
    p->clear_color[3] = 1.0f;
    p->ambient = 0.3f;
    p->diffuse = 0.7f;
    p->specular = 0.25f;
    p->spec_power = 16;
}

const char *vr_last_error(const vr_ctx *ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

vr_ctx *vr_create(int device, uint32_t width, uint32_t height)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        fail(nullptr, VR_ENODEV, "no HIP device available");
        return nullptr;
    }
    if (device < 0 || device >= ndev) {
        fail(nullptr, VR_ENODEV, "device index out of range");
        return nullptr;
    }
    if (width == 0 || height == 0) {
        fail(nullptr, VR_EINVAL, "framebuffer size must be non-zero");
        return nullptr;
    }
    if (hipSetDevice(device) != hipSuccess) {
        fail(nullptr, VR_ENODEV, "hipSetDevice failed");
        return nullptr;
    }
    vr_ctx *c = new (std::nothrow) vr_ctx();
    if (!c) {
        fail(nullptr, VR_ENOMEM, "out of host memory");
        return nullptr;
    }
    c->device = device;
    c->width = width;
    c->height = height;
#ifdef VR_EXPERIMENTS
    knobs_from_env(c);
#endif
    if (hipMalloc(&c->counters, 8 * sizeof(unsigned long long)) != hipSuccess) {
        fail(nullptr, VR_ENOMEM, "hipMalloc(counters)");
        delete c;
        return nullptr;
    }
    // reference constructor placeholders (offscreen_pass.cpp:118-119)
    const float zero = 0.0f;
    const uint32_t white = 0xFFFFFFFFu;
    if (vr_set_volume(c, &zero, VR_DTYPE_F32, 1, 1, 1, 0.0f, 1.0f) != VR_OK ||
        vr_set_transfer_function(c, &white, 1) != VR_OK) {
        g_err = c->err;
        vr_destroy(c);
        return nullptr;
    }
    return c;
}

vr_ctx *vr_create_mask(uint32_t device_mask, uint32_t width, uint32_t height)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        fail(nullptr, VR_ENODEV, "no HIP device available");
        return nullptr;
    }
    if (device_mask == 0) {
        fail(nullptr, VR_EINVAL, "device_mask is empty");
        return nullptr;
    }
    std::vector<int> devices;
    for (int d = 0; d < 32; ++d) {
        if (!((device_mask >> d) & 1u)) continue;
        if (d >= ndev) {
            fail(nullptr, VR_ENODEV, "device " + std::to_string(d) + " of device_mask 0x" +
                                         [&] { char b[16]; std::snprintf(b, sizeof b, "%x", device_mask); return std::string(b); }() +
                                         " is not present (" + std::to_string(ndev) +
                                         " HIP device(s) visible)");
            return nullptr;
        }
        devices.push_back(d);
    }
    return create_members(devices, width, height, VR_EXCHANGE_RCCL);
}

vr_ctx *vr_debug_create_members(const int *devices, int n, uint32_t width, uint32_t height,
                                int exchange)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        fail(nullptr, VR_ENODEV, "no HIP device available");
        return nullptr;
    }
    if (!devices || n < 1 || n > 64) {
        fail(nullptr, VR_EINVAL, "devices must list 1..64 members");
        return nullptr;
    }
    if (exchange != VR_EXCHANGE_RCCL && exchange != VR_EXCHANGE_COPY) {
        fail(nullptr, VR_EINVAL, "exchange must be VR_EXCHANGE_RCCL or VR_EXCHANGE_COPY");
        return nullptr;
    }
    std::vector<int> devs(devices, devices + n);
    for (int d : devs)
        if (d < 0 || d >= ndev) {
            fail(nullptr, VR_ENODEV, "device " + std::to_string(d) + " is not present (" +
                                         std::to_string(ndev) + " HIP device(s) visible)");
            return nullptr;
        }
    return create_members(devs, width, height, exchange);
}

void vr_destroy(vr_ctx *c)
{
    if (!c) return;
    if (c->group) vr::group_destroy(c->group);
    for (vr_ctx *m : c->members) vr_destroy(m);
    c->members.clear();
    c->group = nullptr;
    if (c->group_stream) {
        hipSetDevice(c->device);
        hipStreamDestroy(c->group_stream);
    }
    hipSetDevice(c->device);
    hipDeviceSynchronize();
    for (auto &pr : c->ev_pending) {
        hipEventDestroy(pr.first);
        hipEventDestroy(pr.second);
    }
    for (auto e : c->ev_pool) hipEventDestroy(e);
    if (c->built_ev) hipEventDestroy(c->built_ev);
    if (c->bricks) hipFree(c->bricks);
    if (c->tf) hipFree(c->tf);
    if (c->tf_nz) hipFree(c->tf_nz);
    free_derived(c);  // field, copies, skip-empty classification
    for (auto &f : c->fences)
        if (!f.external) hipEventDestroy(f.ev);
    for (auto &t : c->sched) {
        hipFree(t.cost);
        hipFree(t.perm);
        hipFree(t.lists);
    }
    if (c->counters) hipFree(c->counters);
    if (c->frame_dev) hipFree(c->frame_dev);
    for (auto e : c->band_ev)
        if (e) hipEventDestroy(e);
    for (auto st : c->band_stream)
        if (st) hipStreamDestroy(st);
    if (c->copy_stream) hipStreamDestroy(c->copy_stream);
    delete c;
}

int vr_resize(vr_ctx *c, uint32_t width, uint32_t height)
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    if (width == 0 || height == 0) return VR_OK;  // offscreen_pass.cpp:237-239
    if (is_group(c)) {
        if (int rc = group_idle(c)) return rc;
        for (vr_ctx *m : c->members)
            if (int rc = vr_resize(m, width, height)) return member_rc(c, m, rc);
    }
    c->width = width;
    c->height = height;
    return VR_OK;
}

int vr_get_size(const vr_ctx *c, uint32_t *w, uint32_t *h)
{
    if (!c || !w || !h) return fail(nullptr, VR_EINVAL, "NULL argument");
    *w = c->width;
    *h = c->height;
    return VR_OK;
}

int vr_get_device(const vr_ctx *c, int *device)
{
    if (!c || !device) return fail(nullptr, VR_EINVAL, "NULL argument");
    *device = c->device;
    return VR_OK;
}

int vr_get_device_mask(const vr_ctx *c, uint32_t *device_mask)
{
    if (!c || !device_mask) return fail(nullptr, VR_EINVAL, "NULL argument");
    *device_mask = is_group(c) ? c->device_mask : (1u << c->device);
    return VR_OK;
}

int vr_set_volume_device(vr_ctx *c, const void *data_dev, int dtype, uint32_t nx, uint32_t ny,
                         uint32_t nz, float vmin, float vmax, void *stream)
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    if (!data_dev) return fail(c, VR_EINVAL, "volume data is NULL");
    int st = storage_for(dtype);
    if (st < 0) return fail(c, VR_EINVAL, "unsupported volume dtype");
    if (nx == 0 || ny == 0 || nz == 0) return fail(c, VR_EINVAL, "volume dims must be non-zero");
    if (nx > 65536 || ny > 65536 || nz > 65536) return fail(c, VR_EINVAL, "volume dim > 65536");
    if (is_group(c)) {  // upload and brick on member 0 (the data's device), then replicate
        if (int rc = group_idle(c)) return rc;
        vr_ctx *m0 = c->members[0];
        if (int rc = vr_set_volume_device(m0, data_dev, dtype, nx, ny, nz, vmin, vmax, stream))
            return member_rc(c, m0, rc);
        return replicate_volume(c);
    }
    int rc = wait_idle(c);
    if (rc) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (st == ST_F32 && c->knobs.narrow && dtype != VR_DTYPE_F64) {
        rc = narrow_storage(c, data_dev, dtype, (size_t)nx * ny * nz, s, &st);
        if (rc) return rc;
    }
    void *dst = nullptr;
    const int lay = brick_layout(c, st, nx, ny, nz);
    rc = set_bricks(c, lay, nx, ny, nz, &dst);
    if (rc) return rc;
    HIP_TRY(c, launch_brick_from_linear(dtype, data_dev, dst, nx, ny, nz, lay, s), "brick kernel");
    HIP_TRY(c, hipStreamSynchronize(s), "brick kernel sync");
    c->storage = st;
    c->layout = lay;
    c->nx = nx;
    c->ny = ny;
    c->nz = nz;
    c->vmin = vmin;  // offscreen_pass.cpp:265-266
    c->vmax = vmax;
    c->range_valid = c->dist_valid = false;
    return data_range(c, s);
}

int vr_set_volume(vr_ctx *c, const void *data, int dtype, uint32_t nx, uint32_t ny, uint32_t nz,
                  float vmin, float vmax)
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    if (!data) return fail(c, VR_EINVAL, "volume data is NULL");
    if (storage_for(dtype) < 0) return fail(c, VR_EINVAL, "unsupported volume dtype");
    if (nx == 0 || ny == 0 || nz == 0) return fail(c, VR_EINVAL, "volume dims must be non-zero");
    if (nx > 65536 || ny > 65536 || nz > 65536) return fail(c, VR_EINVAL, "volume dim > 65536");
    if (is_group(c)) {
        if (int rc = group_idle(c)) return rc;
        vr_ctx *m0 = c->members[0];
        if (int rc = vr_set_volume(m0, data, dtype, nx, ny, nz, vmin, vmax)) return member_rc(c, m0, rc);
        return replicate_volume(c);
    }
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    const size_t bytes = (size_t)nx * ny * nz * dtype_size(dtype);
    void *tmp = nullptr;
    HIP_TRY(c, hipMalloc(&tmp, bytes), "hipMalloc(volume staging)");
    // ROCm's pageable copy already stages through pinned buffers: 39-50 GB/s for C3/C4, where
    // a hand-rolled two-chunk pinned pipeline measured 27-29 GB/s (tools/ingest_bench.py)
    hipError_t e = hipMemcpy(tmp, data, bytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        hipFree(tmp);
        return hip_fail(c, e, "hipMemcpy(volume)");
    }
    int rc = vr_set_volume_device(c, tmp, dtype, nx, ny, nz, vmin, vmax, nullptr);
    hipFree(tmp);
    return rc;
}

int vr_generate_volume(vr_ctx *c, int kind, int dtype, uint32_t nx, uint32_t ny, uint32_t nz,
                       uint32_t seed, float *vmin_out, float *vmax_out)
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    if (is_group(c)) {
        if (int rc = group_idle(c)) return rc;
        vr_ctx *m0 = c->members[0];
        if (int rc = vr_generate_volume(m0, kind, dtype, nx, ny, nz, seed, vmin_out, vmax_out))
            return member_rc(c, m0, rc);
        return replicate_volume(c);
    }
    if (kind != 0) return fail(c, VR_EINVAL, "unknown synthetic volume kind");
    int st;
    float scale;
    switch (dtype) {
        case VR_DTYPE_U8: st = ST_U8; scale = 160.0f; break;
        case VR_DTYPE_U16: st = ST_U16; scale = 40000.0f; break;
        case VR_DTYPE_F32: st = ST_F32; scale = 1.0f; break;
        default: return fail(c, VR_EINVAL, "generator supports u8, u16, f32");
    }
    if (nx == 0 || ny == 0 || nz == 0) return fail(c, VR_EINVAL, "volume dims must be non-zero");
    if (nx > 65536 || ny > 65536 || nz > 65536) return fail(c, VR_EINVAL, "volume dim > 65536");
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    const int ng = 32;
    std::vector<float> prm(3 + 5 * ng);
    prm[0] = (float)ng;
    prm[1] = 0.05f;
    prm[2] = scale;
    SplitMix rng{(uint64_t)seed};
    const float dims[3] = {(float)nx, (float)ny, (float)nz};
    const float nmin = std::fmin(dims[0], std::fmin(dims[1], dims[2]));
    for (int g = 0; g < ng; ++g) {
        float *q = &prm[3 + 5 * g];
        for (int a = 0; a < 3; ++a) q[a] = dims[a] * (0.15f + 0.7f * rng.uniform());
        const float sigma = nmin * (0.04f + 0.10f * rng.uniform());
        q[3] = 1.0f / (2.0f * sigma * sigma);
        q[4] = 0.3f + 0.7f * rng.uniform();
    }
    // generate into a linear staging buffer of the storage type, then brick it like an
    // uploaded volume (vr_set_volume_device path)
    const size_t count = (size_t)nx * ny * nz;
    if (int rc0 = wait_idle(c)) return rc0;
    float *prm_dev = nullptr;
    void *lin = nullptr;
    HIP_TRY(c, hipMalloc(&prm_dev, prm.size() * sizeof(float) + 2 * sizeof(uint32_t)),
            "hipMalloc(generator params)");
    hipError_t e = hipMalloc(&lin, count * storage_size(st));
    if (e != hipSuccess) {
        hipFree(prm_dev);
        return hip_fail(c, e, "hipMalloc(generator staging)");
    }
    uint32_t *mm = reinterpret_cast<uint32_t *>(prm_dev + prm.size());
    const uint32_t mm_init[2] = {0xFFFFFFFFu, 0u};
    e = hipMemcpy(prm_dev, prm.data(), prm.size() * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(mm, mm_init, sizeof(mm_init), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = launch_generate(kind, st, lin, nx, ny, nz, prm_dev, (int)prm.size(), nullptr);
    if (e == hipSuccess) e = launch_minmax(st, lin, count, reinterpret_cast<float *>(mm), nullptr);
    uint32_t mm_host[2] = {0, 0};
    if (e == hipSuccess) e = hipMemcpy(mm_host, mm, sizeof(mm_host), hipMemcpyDeviceToHost);
    hipFree(prm_dev);
    if (e != hipSuccess) {
        hipFree(lin);
        return hip_fail(c, e, "generate volume");
    }
    const int src_dtype = st == ST_U8 ? VR_DTYPE_U8 : (st == ST_U16 ? VR_DTYPE_U16 : VR_DTYPE_F32);
    void *dst = nullptr;
    const int lay = brick_layout(c, st, nx, ny, nz);
    int rc = set_bricks(c, lay, nx, ny, nz, &dst);
    if (rc == VR_OK) {
        e = launch_brick_from_linear(src_dtype, lin, dst, nx, ny, nz, lay, nullptr);
        if (e != hipSuccess) rc = hip_fail(c, e, "brick generated volume");
        if (rc == VR_OK && (e = hipDeviceSynchronize()) != hipSuccess)
            rc = hip_fail(c, e, "brick generated volume");
    }
    hipFree(lin);
    if (rc) return rc;
    auto unorder = [](uint32_t o) {
        const uint32_t u = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
        float f;
        std::memcpy(&f, &u, 4);
        return f;
    };
    c->storage = st;
    c->layout = lay;
    c->nx = nx;
    c->ny = ny;
    c->nz = nz;
    c->vmin = unorder(mm_host[0]);
    c->vmax = unorder(mm_host[1]);
    c->range_valid = c->dist_valid = false;
    if (vmin_out) *vmin_out = c->vmin;
    if (vmax_out) *vmax_out = c->vmax;
    return data_range(c, nullptr);
}

uint64_t vr_volume_bytes(const vr_ctx *c)
{
    if (is_group(c)) return vr_volume_bytes(c->members[0]);  // per device (replicated)
    return c ? (uint64_t)c->brick_bytes : 0;
}

int vr_debug_read_volume_native(vr_ctx *c, void *out)
{
    if (!c || !out) return fail(c, VR_EINVAL, "NULL argument");
    if (is_group(c)) return member_rc(c, c->members[0], vr_debug_read_volume_native(c->members[0], out));
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    // unbricked on the device in slabs of z-slices (<= 256 MiB of scratch), then copied out
    const size_t vb = storage_size(c->storage), slice = (size_t)c->nx * c->ny * vb;
    const uint32_t cz = (uint32_t)std::max<size_t>(1, std::min<size_t>(c->nz, (256u << 20) / slice));
    void *tmp = nullptr;
    HIP_TRY(c, hipMalloc(&tmp, slice * cz), "hipMalloc(readback)");
    int rc = VR_OK;
    for (uint32_t z0 = 0; z0 < c->nz && rc == VR_OK; z0 += cz) {
        const uint32_t n = std::min(cz, c->nz - z0);
        hipError_t e = launch_unbrick(c->layout, c->bricks, tmp, c->nx, c->ny, z0, n, nullptr);
        if (e == hipSuccess)
            e = hipMemcpy(static_cast<char *>(out) + slice * z0, tmp, slice * n, hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = hip_fail(c, e, "read volume");
    }
    hipFree(tmp);
    return rc;
}

int vr_debug_read_volume(vr_ctx *c, float *out)
{
    if (!c || !out) return fail(c, VR_EINVAL, "NULL argument");
    if (is_group(c)) return member_rc(c, c->members[0], vr_debug_read_volume(c->members[0], out));
    const size_t n = (size_t)c->nx * c->ny * c->nz;
    if (c->storage == ST_F32) return vr_debug_read_volume_native(c, out);
    std::vector<unsigned char> host(n * storage_size(c->storage));
    const int rc = vr_debug_read_volume_native(c, host.data());
    if (rc) return rc;
    for (size_t i = 0; i < n; ++i) {  // float(v) is exact for 8/16-bit voxels
        switch (c->storage) {
            case ST_U8: out[i] = (float)host[i]; break;
            case ST_I8: out[i] = (float)(int8_t)host[i]; break;
            case ST_U16: { uint16_t t; std::memcpy(&t, &host[2 * i], 2); out[i] = (float)t; } break;
            default: { int16_t t; std::memcpy(&t, &host[2 * i], 2); out[i] = (float)t; } break;
        }
    }
    return VR_OK;
}

int vr_debug_volume_info(const vr_ctx *c, uint32_t dims[3], float minmax[2], int *storage)
{
    if (!c) return VR_EINVAL;
    if (is_group(c)) return vr_debug_volume_info(c->members[0], dims, minmax, storage);
    if (dims) {
        dims[0] = c->nx;
        dims[1] = c->ny;
        dims[2] = c->nz;
    }
    if (minmax) {
        minmax[0] = c->vmin;
        minmax[1] = c->vmax;
    }
    if (storage) *storage = c->storage;
    return VR_OK;
}

int vr_set_transfer_function(vr_ctx *c, const uint32_t *rgba8_srgb, uint32_t n)
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    if (!rgba8_srgb || n == 0) return fail(c, VR_EINVAL, "transfer function is empty");
    if (n > (1u << 20)) return fail(c, VR_EINVAL, "transfer function too large");
    if (is_group(c)) {
        if (int rc = group_idle(c)) return rc;
        for (vr_ctx *m : c->members)
            if (int rc = vr_set_transfer_function(m, rgba8_srgb, n)) return member_rc(c, m, rc);
        return VR_OK;
    }
    if (int rc = wait_idle(c)) return rc;
    return upload_tf(c, rgba8_srgb, n);
}

int vr_set_slicing(vr_ctx *c, const float min_slice[3], const float max_slice[3])
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    if (!min_slice || !max_slice) return fail(c, VR_EINVAL, "slice bounds are NULL");
    if (is_group(c)) {  // frames already issued keep the old box (as the reference's UBO ring)
        if (int rc = group_idle(c)) return rc;
        for (vr_ctx *m : c->members)
            if (int rc = vr_set_slicing(m, min_slice, max_slice)) return member_rc(c, m, rc);
    }
    for (int a = 0; a < 3; ++a) {
        c->smin[a] = min_slice[a];
        c->smax[a] = max_slice[a];
    }
    return VR_OK;
}

uint32_t vr_shard_rows(uint32_t height, uint32_t row_block, uint32_t nranks)
{
    if (row_block == 0 || nranks == 0) return 0;
    const uint32_t blocks = (height + row_block - 1) / row_block;
    return ((blocks + nranks - 1) / nranks) * row_block;
}

uint32_t vr_shard_rows_ctx(const vr_ctx *c, uint32_t height, uint32_t row_block, uint32_t nranks)
{
    return c ? share_shard_rows(height, row_block, nranks, c->share) : 0;
}

int vr_set_row_share(vr_ctx *c, uint32_t first_weight, uint32_t other_weight)
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    if (first_weight < 1 || other_weight < 1 || first_weight > 64 || other_weight > 64)
        return fail(c, VR_EINVAL, "row share weights must be in [1, 64]");
    if (is_group(c)) {  // frames in flight keep their split; the pipelines are rebuilt
        if (int rc = group_idle(c)) return rc;
        for (vr_ctx *m : c->members)
            if (int rc = vr_set_row_share(m, first_weight, other_weight)) return member_rc(c, m, rc);
    }
    c->share = RowShare{first_weight, other_weight};
    return VR_OK;
}

int vr_get_row_share(const vr_ctx *c, uint32_t *first_weight, uint32_t *other_weight)
{
    if (!c || !first_weight || !other_weight) return fail(nullptr, VR_EINVAL, "NULL argument");
    *first_weight = c->share.w0;
    *other_weight = c->share.w;
    return VR_OK;
}

int vr_set_memory_budget(vr_ctx *c, uint64_t bytes)
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    if (is_group(c)) {  // per device: every member holds its own replica's structures
        if (int rc = group_idle(c)) return rc;
        for (vr_ctx *m : c->members)
            if (int rc = vr_set_memory_budget(m, bytes)) return member_rc(c, m, rc);
        c->budget = bytes;
        return VR_OK;
    }
    if (int rc = wait_idle(c)) return rc;  // frames in flight may read what is freed
    c->budget = bytes;
    if (bytes != VR_MEMORY_BUDGET_UNLIMITED && derived_bytes(c) > effective_budget(c)) free_derived(c);
    return VR_OK;
}

int vr_memory_report(const vr_ctx *c, vr_memory_info *out)
{
    if (!c || !out) return fail(nullptr, VR_EINVAL, "NULL argument");
    if (is_group(c)) return vr_memory_report(c->members[0], out);  // per device (replicated)
    std::memset(out, 0, sizeof *out);
    out->volume_bytes = c->brick_bytes;
    out->field_bytes = c->grad ? c->grad_bytes : 0;
    uint64_t *copies[3] = {&out->oblique_copy_bytes, &out->plain_copy_bytes, &out->stencil_copy_bytes};
    for (int i = 0; i < 3; ++i)
        *copies[i] = c->alt[i].bricks ? c->alt[i].bytes + kBrickSlackBytes : 0;
    out->skip_bytes = c->nbricks_alloc * kSkipBytesPerBrick;
    out->derived_bytes = derived_bytes(c);
    out->budget_bytes = c->budget == VR_MEMORY_BUDGET_UNLIMITED ? c->budget : effective_budget(c);
    out->builds = c->n_builds;
    out->evictions = c->n_evictions;
    out->downgrades = c->n_downgrades;
    out->last_downgrade = c->last_downgrade;
    return VR_OK;
}

int vr_prepare(vr_ctx *c, const vr_camera *cam, const vr_params *p)
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    if (is_group(c)) {
        if (int rc = group_idle(c)) return rc;
        for (vr_ctx *m : c->members)
            if (int rc = vr_prepare(m, cam, p)) return member_rc(c, m, rc);
        hipSetDevice(c->device);
        return VR_OK;
    }
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    // the whole frame as vr_render_device launches it (one rank), up to the launch
    if (int rc = render_device_impl(c, cam, p, c->counters, VR_OUT_RGBA8, 16, 0, 1, c->share,
                                    nullptr, false))
        return rc;
    HIP_TRY(c, hipStreamSynchronize(nullptr), "hipStreamSynchronize (prepare)");
    return VR_OK;
}

int vr_render_device(vr_ctx *c, const vr_camera *cam, const vr_params *p, void *out_dev,
                     int out_format, uint32_t row_block, uint32_t rank, uint32_t nranks,
                     void *stream)
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    return render_device_impl(c, cam, p, out_dev, out_format, row_block, rank, nranks, c->share,
                              stream);
}

}  // extern "C"
namespace {
// launch = false (vr_prepare): everything up to the launch -- the derived structures this frame
// reads are built on `stream` -- and no launch.
int render_device_impl(vr_ctx *c, const vr_camera *cam, const vr_params *p, void *out_dev,
                       int out_format, uint32_t row_block, uint32_t rank, uint32_t nranks,
                       RowShare share, void *stream, bool launch)
{
    if (!out_dev) return fail(c, VR_EINVAL, "output buffer is NULL");
    if (is_group(c)) {
        // the whole frame, split over the devices internally (8-row blocks, block-cyclic)
        if (rank != 0 || nranks != 1)
            return fail(c, VR_EINVAL, "a multi-device context renders whole frames (rank 0 of 1)");
        if (!cam) return fail(c, VR_EINVAL, "camera is NULL");
        if (int rc = check_params(c, p)) return rc;
        if (out_format != VR_OUT_RGBA8 && out_format != VR_OUT_RGBA32F)
            return fail(c, VR_EINVAL, "unknown out_format");
        std::string m;
        if (int rc = vr::group_render(c->group, cam, p, out_dev, out_format,
                                      static_cast<hipStream_t>(stream), &m))
            return fail(c, rc, m);
        return VR_OK;
    }
    MarchParams P;
    int rc = build_params(c, cam, p, out_dev, out_format, row_block, rank, nranks, share, P);
    if (rc) return rc;
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    hipStream_t s = static_cast<hipStream_t>(stream);
    ++c->frame_no;
    uint32_t refused = 0;  // VR_DERIVED_* the budget or free memory refused this frame
    rc = ensure_derived(c, p, P, s, &refused);
    if (rc) return rc;
    if (use_pair(c, P, p)) {  // L lanes per ray on 16 x (16 / L) tiles (march_pair_kernel)
        // 4 lanes below kPairQuadMaxWaves (N = 8 C3 share: 0.151 -> 0.144 ms), else 2
        P.pair = P.tiles_x * P.tiles_y * (kThreadsPerTile / 64) < kPairQuadMaxWaves ? 4 : 2;
        if (c->knobs.pair_lanes == 2 || c->knobs.pair_lanes == 4) P.pair = c->knobs.pair_lanes;
        const uint32_t th = 16 / P.pair;
        P.tiles_y = (P.local_rows + th - 1) / th;
        P.supers_total = P.supers_x * ((P.tiles_y + kSuper - 1) / kSuper);
    }
    // oblique and sparse f32 views: an alternative-geometry copy (want_alt)
    int layout = c->layout;
    if (const int lay = want_alt(c, p, P); lay != c->layout) {
        bool ready = false;
        rc = ensure_alt(c, lay, s, &ready);
        if (rc) return rc;
        if (ready) {
            layout = lay;
            P.vol = c->alt[alt_index(lay)].bricks;
            P.vol_bytes = c->alt[alt_index(lay)].bytes;
            P.nbx = bricks_for(c->nx, 0, layout);
            P.nby = bricks_for(c->ny, 1, layout);
        } else {
            refused = (uint32_t)(VR_DERIVED_OBLIQUE_COPY + alt_index(lay));
        }
    }
    if (!launch) return VR_OK;
    if (refused) {  // a budget-forced downgrade: recorded (vr_memory_report), never silent
        ++c->n_downgrades;
        c->last_downgrade = refused;
    }
    vr_ctx::TileSched *ts =
        tile_sched(c, P, stream, tile_kernel_key(P, p->shading != 0, layout));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const bool timing = c->timing;  // read once: the pair is recorded and queued together
    if (timing) {
        e0 = pooled_event(c);
        e1 = pooled_event(c);
        if (!e0 || !e1) return fail(c, VR_EIO, "hipEventCreate failed");
        HIP_TRY(c, hipEventRecord(e0, s), "hipEventRecord");
    }
    HIP_TRY(c, launch_march(layout, p->shading != 0, false, P, s), "march kernel launch");
    if (timing) {
        HIP_TRY(c, hipEventRecord(e1, s), "hipEventRecord");
        c->ev_pending.emplace_back(e0, e1);
    }
    // next launches of this geometry: longest tiles first, re-ordered every kReorderEvery
    // launches (the order kernel runs after the timed march kernel, inside the frame)
    if (ts && ts->launches++ % kReorderEvery == 0) {
        HIP_TRY(c, launch_order_tiles(ts->cost, ts->lists, ts->perm, ts->per_xcd, s),
                "tile order kernel");
        ts->have_perm = true;
    }
    return fence_record(c, s);
}
}  // namespace
extern "C" {

int vr_render(vr_ctx *c, const vr_camera *cam, const vr_params *p, void *out, int out_format)
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    if (!out) return fail(c, VR_EINVAL, "output buffer is NULL");
    if (!p) return fail(c, VR_EINVAL, "params is NULL");
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    const size_t bpp = out_format == VR_OUT_RGBA32F ? 16 : 4;
    const uint32_t W = c->width, H = c->height;
    if (is_group(c)) {  // the frame across the devices into device 0, then one copy out
        const size_t fb = (size_t)W * H * bpp;
        if (c->frame_bytes < fb) {
            if (c->frame_dev) hipFree(c->frame_dev);
            c->frame_dev = nullptr;
            c->frame_bytes = 0;
            HIP_TRY(c, hipMalloc(&c->frame_dev, fb), "hipMalloc(frame)");
            c->frame_bytes = fb;
        }
        if (!c->group_stream)
            HIP_TRY(c, hipStreamCreateWithFlags(&c->group_stream, hipStreamNonBlocking),
                    "hipStreamCreate");
        int rc = vr_render_device(c, cam, p, c->frame_dev, out_format, vr::kGroupRowBlock, 0, 1,
                                  c->group_stream);
        if (rc) return rc;
        HIP_TRY(c, hipMemcpyAsync(out, c->frame_dev, fb, hipMemcpyDeviceToHost, c->group_stream),
                "hipMemcpyAsync(frame)");
        HIP_TRY(c, hipStreamSynchronize(c->group_stream), "hipStreamSynchronize(frame)");
        return VR_OK;
    }
    // kRenderBands row bands of R rows (a multiple of the 16-row tile): band b is the row shard
    // (row_block R, rank b, nranks kRenderBands), rendered densely at rows [b R, b R + R)
    const int nb = H >= kHostBandMinRows ? kRenderBands : 1;
    const uint32_t R = nb == 1 ? 16 : ((H + nb - 1) / nb + 15) / 16 * 16;
    const size_t bytes = (size_t)W * (nb == 1 ? H : (size_t)R * nb) * bpp;
    if (c->frame_bytes < bytes) {
        if (c->frame_dev) hipFree(c->frame_dev);
        c->frame_dev = nullptr;
        c->frame_bytes = 0;
        HIP_TRY(c, hipMalloc(&c->frame_dev, bytes), "hipMalloc(frame)");
        c->frame_bytes = bytes;
    }
    if (nb == 1) {
        int rc = render_device_impl(c, cam, p, c->frame_dev, out_format, 16, 0, 1, RowShare{1, 1},
                                    nullptr);
        if (rc) return rc;
        HIP_TRY(c, hipMemcpy(out, c->frame_dev, (size_t)W * H * bpp, hipMemcpyDeviceToHost),
                "hipMemcpy(frame)");
        return VR_OK;
    }
    if (!c->copy_stream) {
        for (auto &s : c->band_stream)
            HIP_TRY(c, hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate(band)");
        HIP_TRY(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking),
                "hipStreamCreate(copy)");
        for (auto &e : c->band_ev)
            HIP_TRY(c, hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate(band)");
    }
    // the bands overlap on two streams: the throughput kernels, not the latency-oriented lane
    // groups (use_pair), as for frames in flight
    vr_params pb = *p;
    if (pb.frames_in_flight < 2) pb.frames_in_flight = 2;
    for (int b = 0; b < nb; ++b) {
        hipStream_t s = c->band_stream[b & 1];
        int rc = render_device_impl(c, cam, &pb,
                                    static_cast<char *>(c->frame_dev) + (size_t)b * R * W * bpp,
                                    out_format, R, (uint32_t)b, (uint32_t)nb, RowShare{1, 1}, s);
        if (rc) return rc;
        HIP_TRY(c, hipEventRecord(c->band_ev[b], s), "hipEventRecord(band)");
    }
    // band b's copy starts as soon as it is rendered; a pageable destination makes each copy
    // return once its bytes are in `out`, while the device renders the later bands
    for (int b = 0; b < nb; ++b) {
        const size_t row0 = (size_t)b * R;
        if (row0 >= H) break;
        const size_t rows = std::min<size_t>(R, H - row0);
        HIP_TRY(c, hipStreamWaitEvent(c->copy_stream, c->band_ev[b], 0), "hipStreamWaitEvent(band)");
        HIP_TRY(c, hipMemcpyAsync(static_cast<char *>(out) + row0 * W * bpp,
                                  static_cast<char *>(c->frame_dev) + row0 * W * bpp,
                                  rows * W * bpp, hipMemcpyDeviceToHost, c->copy_stream),
                "hipMemcpyAsync(band)");
    }
    HIP_TRY(c, hipStreamSynchronize(c->copy_stream), "hipStreamSynchronize(copy)");
    return VR_OK;
}

int vr_assemble_rows(vr_ctx *c, const void *gathered_dev, void *out_dev, int out_format,
                     uint32_t row_block, uint32_t nranks, void *stream)
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    if (!gathered_dev || !out_dev) return fail(c, VR_EINVAL, "NULL buffer");
    if (row_block == 0 || nranks == 0) return fail(c, VR_EINVAL, "bad shard");
    if (out_format != VR_OUT_RGBA8 && out_format != VR_OUT_RGBA32F)
        return fail(c, VR_EINVAL, "unknown out_format");
    if (is_group(c))
        return member_rc(c, c->members[0], vr_assemble_rows(c->members[0], gathered_dev, out_dev,
                                                            out_format, row_block, nranks, stream));
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    HIP_TRY(c, launch_assemble(gathered_dev, out_dev, out_format, c->width, c->height, row_block,
                               nranks, share_shard_rows(c->height, row_block, nranks, c->share),
                               c->share,
                               static_cast<hipStream_t>(stream)),
            "assemble kernel");
    return VR_OK;
}

// Zero-copy presentation: memory another API exported as a POSIX fd (Vulkan
// VK_KHR_external_memory_fd), imported on the device vr_render_device writes to.
struct vr_external_memory {
    hipExternalMemory_t ext;
    void *ptr;
    int device;
};

int vr_import_memory_fd(vr_ctx *c, int fd, uint64_t size, uint64_t offset,
                        vr_external_memory **mem, void **dev_ptr)
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    if (!mem || !dev_ptr) return fail(c, VR_EINVAL, "NULL output");
    *mem = nullptr;
    *dev_ptr = nullptr;
    if (fd < 0 || size == 0 || offset > UINT64_MAX - size)
        return fail(c, VR_EINVAL, "bad fd, size or offset");
    const int device = is_group(c) ? c->members[0]->device : c->device;
    HIP_TRY(c, hipSetDevice(device), "hipSetDevice");
    hipExternalMemoryHandleDesc hd;
    std::memset(&hd, 0, sizeof hd);
    hd.type = hipExternalMemoryHandleTypeOpaqueFd;
    hd.handle.fd = fd;
    hd.size = offset + size;
    hipExternalMemory_t ext = nullptr;
    HIP_TRY(c, hipImportExternalMemory(&ext, &hd), "hipImportExternalMemory");
    hipExternalMemoryBufferDesc bd;
    std::memset(&bd, 0, sizeof bd);
    bd.offset = offset;
    bd.size = size;
    void *ptr = nullptr;
    const hipError_t e = hipExternalMemoryGetMappedBuffer(&ptr, ext, &bd);
    if (e != hipSuccess) {
        (void)hipDestroyExternalMemory(ext);
        return hip_fail(c, e, "hipExternalMemoryGetMappedBuffer");
    }
    *mem = new vr_external_memory{ext, ptr, device};
    *dev_ptr = ptr;
    return VR_OK;
}

int vr_release_external_memory(vr_ctx *c, vr_external_memory *m)
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    if (!m) return fail(c, VR_EINVAL, "mem is NULL");
    HIP_TRY(c, hipSetDevice(m->device), "hipSetDevice");
    // frames still rendering into the mapping finish first
    HIP_TRY(c, hipDeviceSynchronize(), "hipDeviceSynchronize");
    const hipError_t e1 = hipFree(m->ptr);
    const hipError_t e2 = hipDestroyExternalMemory(m->ext);
    delete m;
    if (e1 != hipSuccess) return hip_fail(c, e1, "hipFree(external mapping)");
    if (e2 != hipSuccess) return hip_fail(c, e2, "hipDestroyExternalMemory");
    return VR_OK;
}

int vr_count_work(vr_ctx *c, const vr_camera *cam, const vr_params *p, uint32_t row_block,
                  uint32_t rank, uint32_t nranks, vr_stats *out)
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    if (!out) return fail(c, VR_EINVAL, "stats is NULL");
    if (is_group(c)) {  // every device holds the same scene: count on member 0
        if (int rc = group_idle(c)) return rc;
        return member_rc(c, c->members[0],
                         vr_count_work(c->members[0], cam, p, row_block, rank, nranks, out));
    }
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    const size_t bytes = (size_t)c->width *
                         share_shard_rows(c->height, row_block ? row_block : 1, nranks ? nranks : 1,
                                          c->share) * 4;
    if (c->frame_bytes < bytes) {
        if (c->frame_dev) hipFree(c->frame_dev);
        c->frame_dev = nullptr;
        c->frame_bytes = 0;
        HIP_TRY(c, hipMalloc(&c->frame_dev, bytes), "hipMalloc(frame)");
        c->frame_bytes = bytes;
    }
    MarchParams P;
    int rc = build_params(c, cam, p, c->frame_dev, VR_OUT_RGBA8, row_block, rank, nranks,
                          c->share, P);
    if (rc) return rc;
    uint32_t refused = 0;  // a count is not a frame: not a downgrade
    rc = ensure_derived(c, p, P, nullptr, &refused);
    if (rc) return rc;
    HIP_TRY(c, hipMemset(c->counters, 0, 8 * sizeof(unsigned long long)), "hipMemset(counters)");
    HIP_TRY(c, launch_march(c->layout, p->shading != 0, true, P, nullptr), "march (count) launch");
    unsigned long long h[5];
    HIP_TRY(c, hipMemcpy(h, c->counters, sizeof(h), hipMemcpyDeviceToHost), "hipMemcpy(counters)");
    out->rays = h[0];
    out->samples = h[1];
    out->shaded_samples = h[2];
    out->steps = h[3];
    out->skipped_samples = h[4];
    return VR_OK;
}

int vr_timing_enable(vr_ctx *c, int enable)
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    // the members' frame workers may be inside vr_render_device: drain them first
    if (is_group(c)) {
        if (int rc = group_idle(c)) return rc;
        vr::group_timing_enable(c->group, enable != 0);
    }
    for (vr_ctx *m : c->members) vr_timing_enable(m, enable);
    c->timing = enable != 0;
    return VR_OK;
}

int vr_debug_timing_member(vr_ctx *c, int member, vr_member_timing *out)
{
    if (!c || !out) return fail(c, VR_EINVAL, "NULL argument");
    std::memset(out, 0, sizeof *out);
    if (!is_group(c)) {  // one device: its kernel time only
        if (member != 0) return fail(c, VR_EINVAL, "no such member");
        out->device = c->device;
        return vr_timing_read(c, &out->kernel_ms, &out->frames);
    }
    double ms[3] = {0.0, 0.0, 0.0};
    uint64_t frames = 0;
    std::string m;
    if (int rc = vr::group_timing_member(c->group, member, ms, &frames, &m)) return fail(c, rc, m);
    vr_ctx *mc = c->members[(size_t)member];
    uint64_t launches = 0;
    if (int rc = vr_timing_read(mc, &out->kernel_ms, &launches)) return member_rc(c, mc, rc);
    hipSetDevice(c->device);
    out->device = mc->device;
    out->frames = frames;
    out->render_ms = ms[0];
    out->gather_ms = ms[1];
    out->assemble_ms = ms[2];
    return VR_OK;
}

int vr_debug_host_profile_enable(vr_ctx *c, int enable)
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    if (!is_group(c)) return fail(c, VR_EINVAL, "not a multi-device context");
    vr::group_host_profile_enable(c->group, enable != 0);
    return VR_OK;
}

int vr_debug_host_profile_member(vr_ctx *c, int member, vr_dist_host_profile *out)
{
    if (!c || !out) return fail(c, VR_EINVAL, "NULL argument");
    if (!is_group(c)) return fail(c, VR_EINVAL, "not a multi-device context");
    std::string m;
    if (int rc = vr::group_host_profile_member(c->group, member, out, &m)) return fail(c, rc, m);
    return VR_OK;
}

int vr_debug_fail_member(vr_ctx *c, int member, uint64_t frame)
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    if (!is_group(c)) return fail(c, VR_EINVAL, "not a multi-device context");
    std::string m;
    if (int rc = vr::group_fail_member(c->group, member, frame, &m)) return fail(c, rc, m);
    return VR_OK;
}

int vr_timing_read(vr_ctx *c, double *total_ms, uint64_t *launches)
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    if (is_group(c)) {  // summed over the devices' launches
        if (int rc = group_idle(c)) return rc;
        double ms = 0.0;
        uint64_t n = 0;
        for (vr_ctx *m : c->members) {
            double a = 0.0;
            uint64_t b = 0;
            if (int rc = vr_timing_read(m, &a, &b)) return member_rc(c, m, rc);
            ms += a;
            n += b;
        }
        hipSetDevice(c->device);
        if (total_ms) *total_ms = ms;
        if (launches) *launches = n;
        return VR_OK;
    }
    HIP_TRY(c, hipSetDevice(c->device), "hipSetDevice");
    for (auto &pr : c->ev_pending) {
        if (hipEventSynchronize(pr.second) != hipSuccess) {
            // recorded on a stream the caller destroyed since (fence_others): drain the device
            (void)hipGetLastError();
            HIP_TRY(c, hipDeviceSynchronize(), "hipDeviceSynchronize (timing)");
        }
        float ms = 0.0f;
        HIP_TRY(c, hipEventElapsedTime(&ms, pr.first, pr.second), "hipEventElapsedTime");
        c->timed_ms += ms;
        c->timed_launches++;
        c->ev_pool.push_back(pr.first);
        c->ev_pool.push_back(pr.second);
    }
    c->ev_pending.clear();
    if (total_ms) *total_ms = c->timed_ms;
    if (launches) *launches = c->timed_launches;
    return VR_OK;
}

int vr_timing_reset(vr_ctx *c)
{
    if (is_group(c)) {
        if (int rc = group_idle(c)) return rc;
        std::string m;
        if (int rc = vr::group_timing_reset(c->group, &m)) return fail(c, rc, m);
        for (vr_ctx *m : c->members)
            if (int rc = vr_timing_reset(m)) return member_rc(c, m, rc);
        return VR_OK;
    }
    double ms;
    uint64_t n;
    int rc = vr_timing_read(c, &ms, &n);
    if (rc) return rc;
    c->timed_ms = 0.0;
    c->timed_launches = 0;
    return VR_OK;
}

const char *vr_kernel_name(const vr_ctx *c, const vr_params *p)
{
    if (!c) return "";
    if (is_group(c)) return vr_kernel_name(c->members[0], p);
    // the variant the next vr_render_device launches (after a shaded frame built the field)
    const bool gf = p && p->shading && use_grad_field(c, p->exact_gradient == 0) && c->grad &&
                    c->grad_valid;
    // the full frame (row_block 16, one rank), as vr_render launches it
    const uint32_t tiles = ((c->width + 15) / 16) * ((c->height + kMarchRows - 1) / kMarchRows);
    const bool pipe = use_pipeline(p && p->shading, tiles, c) &&
                      !(p && p->skip_empty) && c->tf_n <= 256;
    int layout = c->layout;
    if (p && !gf) {  // want_alt for the full frame of the last view, once its copy exists
        MarchParams P;
        std::memset(&P, 0, sizeof P);
        const int lay = want_alt(c, p, P);
        if (lay != c->layout && c->alt[alt_index(lay)].valid) layout = lay;
    }
    if (gf && p->exact_gradient == 0 && c->storage == ST_F32) layout |= kHalfFieldFlag;
    return march_kernel_name(layout, p && p->shading != 0, false, p && p->skip_empty != 0, gf,
                             pipe);
}

int vr_debug_set_knob(vr_ctx *c, int knob, int value)
{
    if (!c) return fail(nullptr, VR_EINVAL, "ctx is NULL");
    int *k = knob_slot(c, knob);
    if (!k) return fail(c, VR_EINVAL, "unknown knob");
    if (!knob_value_ok(knob, value)) return fail(c, VR_EINVAL, "knob value out of range");
    if (is_group(c))  // no member may be inside a frame while its knobs change
        if (int rc = group_idle(c)) return rc;
    *k = value;
    for (vr_ctx *m : c->members) vr_debug_set_knob(m, knob, value);
    return VR_OK;
}

int vr_debug_get_knob(const vr_ctx *c, int knob, int *value)
{
    if (!c || !value) return fail(nullptr, VR_EINVAL, "NULL argument");
    int *k = knob_slot(const_cast<vr_ctx *>(c), knob);
    if (!k) return fail(nullptr, VR_EINVAL, "unknown knob");
    *value = *k;
    return VR_OK;
}

#ifdef VR_WG_TIMES
// Experiment builds only: per-workgroup (start, end) wall-clock pairs of the march launches
// since the last reset (tools/wg_timeline.py).
int vr_debug_wg_times(unsigned long long *out, unsigned int max, unsigned int *count, int reset)
{
    if (reset) return debug_wg_times_reset() == hipSuccess ? VR_OK : VR_EIO;
    return debug_wg_times_read(out, max, count) == hipSuccess ? VR_OK : VR_EIO;
}
#endif

}  // extern "C"
