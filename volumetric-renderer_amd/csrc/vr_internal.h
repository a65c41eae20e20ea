// vr_internal.h — shared definitions between the C-ABI layer (vr_api.hip) and the
// gfx950 kernels (vr_kernels.hip).  Not installed; the public boundary is include/vr/vr.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <cmath>
#include <type_traits>

namespace vr {

// ---- Bricked volume layout in HBM ----------------------------------------------------------
// The logical volume (nx, ny, nz) is shifted by kPad = 2 zero voxels on the low side of each
// axis ("padded index" p = logical + 2) and cut into bricks of BX x BY x BZ cells (BrickGeom
// below).  A brick stores ELEMENTS for padded indices [B b, B b + B] on each axis (B + 1: a
// 1-element apron), bricks in brick_slot order, elements x-fastest in a brick, so every
// trilinear footprint lies in one brick.  Per storage type:
//   f32 (and 32/64-bit inputs, converted): "z-pair" element = {v(x,y,z), v(x,y,z+1)}, 8 B, in
//         8^3-cell bricks; a sample = 2 x 16-B loads (elements x, x+1 of rows y and y+1).
//         2 x (9/8)^3 = 2.85x the f32 voxels.
//   16-bit: "yz-quad" element = {v(y,z), v(y,z+1), v(y+1,z), v(y+1,z+1)} at x, 8 B, in 8^3
//         bricks; a sample = 1 x 16-B load of elements x, x+1.  4 x (9/8)^3 = 5.7x.
//   8-bit: plain voxels in 7 x 8 x 8-cell bricks (8-B rows, 648-B bricks); a sample = 2 x
//         16-B loads (rows y, y+1 of slices z and z+1, from the 4-aligned address at or below
//         the cell).  8 x 9 x 9 / (7 x 8 x 8) = 1.45x the voxels (VR_U8_PLAIN=0: yz-quads).
// Voxels outside [0, N) are stored as 0: CLAMP_TO_BORDER/TRANSPARENT_BLACK without a bounds
// test.
// Brick geometry (compile-time): BX x BY x BZ cells per brick, each axis storing cells + 1
// elements (the apron); element (x, y, z) of a brick at x + EX (y + EY z), the brick padded to
// Elems.  f32 and 16-bit volumes use GeomWide (default 8^3 cells, 9^3 = 729 elements), 8-bit
// volumes GeomByte.  Experiment builds may set VR_BRICK_CELLS="bx,by,bz" (e.g. 15,7,8: 16-element
// rows = one 128-B line of f32 z-pairs) and VR_BRICK_ALIGN (elements a brick is rounded up to).
#ifndef VR_BRICK_CELLS
#define VR_BRICK_CELLS 8, 8, 8
#endif
#ifndef VR_BRICK_ALIGN
#define VR_BRICK_ALIGN 1
#endif
// LO = 1 (the stencil copy below): every axis also stores one element below the brick's first
// cell and one more above, so a cell's gradient taps (x - 1 .. x + 2, per axis) never leave it.
template <int X, int Y, int Z, int LO = 0>
struct BrickGeom {
    static constexpr int BX = X, BY = Y, BZ = Z;
    static constexpr int Lo = LO;  // apron elements below the first cell
    static constexpr int EX = X + 1 + 2 * LO, EY = Y + 1 + 2 * LO, EZ = Z + 1 + 2 * LO;  // elements per axis
    static constexpr int Row = EX, Slice = EX * EY;           // element strides of y, z
    static constexpr int Elems = (EX * EY * EZ + VR_BRICK_ALIGN - 1) / VR_BRICK_ALIGN * VR_BRICK_ALIGN;
    __host__ __device__ static constexpr int cells(int a) { return a == 0 ? X : (a == 1 ? Y : Z); }
};
using GeomWide = BrickGeom<VR_BRICK_CELLS>;
// 8-bit volumes (VR_U8_PLAIN = 1): one voxel per element, bricks of 7 x 8 x 8 cells, so a brick
// row is 8 bytes and a 648-B brick keeps every row 4-aligned: one dwordx4 from the 4-aligned
// address at or below the cell's element holds elements x, x + 1 of rows y and y + 1 (byte
// offsets s, s+1, s+8, s+9 with s = x mod 4 <= 3), a second one the same at z + 1.
// VR_U8_BRICK_CELLS="3,8,8" (experiment builds): 4-byte rows, one dwordx2 per slice (half the
// bytes per sample), 1.69x the voxels: C4 +1.5%, C5 +-0, views -2..+4%
// (profiles/r02/u8_geometry/).
// VR_U8_PLAIN = 0: yz-quad elements in GeomWide bricks (one 8-B load, 5.7x the voxels).
#ifndef VR_U8_PLAIN
#define VR_U8_PLAIN 1
#endif
#ifndef VR_U8_BRICK_CELLS
#define VR_U8_BRICK_CELLS 7, 8, 8
#endif
using GeomByte = std::conditional_t<VR_U8_PLAIN != 0, BrickGeom<VR_U8_BRICK_CELLS>, GeomWide>;
// wide loads of the last brick read up to this many bytes past its end
constexpr size_t kBrickSlackBytes = 64;
// VR_F32_PLAIN=1 (experiment builds): f32 elements hold one voxel (no z-pair duplication);
// a sample is then 4 x 8-B loads (elements x, x+1 of the rows (y|y+1, z|z+1)).
#ifndef VR_F32_PLAIN
#define VR_F32_PLAIN 0
#endif
constexpr size_t kF32VoxelsPerElement = VR_F32_PLAIN ? 1 : 2;
constexpr int kPad = 2;

// Brick memory order (north_star: "Z-ordered bricks").  kGroupShift = 0: bricks x-fastest over
// the brick grid.  kGroupShift = g > 0: the grid is cut into groups of 2^g bricks per axis,
// groups x-fastest, and the 2^3g bricks of a group in Morton (Z) order, so bricks near in 3-D
// are near in memory (fewer distinct pages per wave-level load on oblique views).
#ifndef VR_BRICK_GROUP_SHIFT
#define VR_BRICK_GROUP_SHIFT 0
#endif
constexpr int kGroupShift = VR_BRICK_GROUP_SHIFT;
constexpr uint32_t kGroupMask = (1u << kGroupShift) - 1;

// Bits 0..g-1 of v moved to bits 0, 3, 6, ... (one axis of a Morton code).
__host__ __device__ __forceinline__ uint32_t morton_spread(uint32_t v)
{
    uint32_t r = 0;
#pragma unroll
    for (int t = 0; t < kGroupShift; ++t) r |= ((v >> t) & 1u) << (3 * t);
    return r;
}

// Memory slot of brick (bx, by, bz) of an nbx x nby x * grid (whole groups per axis).
__host__ __device__ __forceinline__ uint32_t brick_slot(uint32_t bx, uint32_t by, uint32_t bz,
                                                        uint32_t nbx, uint32_t nby)
{
    if constexpr (kGroupShift == 0) {
        return (bz * nby + by) * nbx + bx;
    } else {
        constexpr uint32_t G = kGroupShift;
        const uint32_t grp = ((bz >> G) * (nby >> G) + (by >> G)) * (nbx >> G) + (bx >> G);
        return (grp << (3 * G)) | morton_spread(bx & kGroupMask) |
               (morton_spread(by & kGroupMask) << 1) | (morton_spread(bz & kGroupMask) << 2);
    }
}

// Inverse of brick_slot.
__host__ __device__ __forceinline__ void brick_coords(uint32_t slot, uint32_t nbx, uint32_t nby,
                                                      uint32_t &bx, uint32_t &by, uint32_t &bz)
{
    if constexpr (kGroupShift == 0) {
        bx = slot % nbx;
        by = (slot / nbx) % nby;
        bz = slot / (nbx * nby);
    } else {
        constexpr uint32_t G = kGroupShift;
        const uint32_t grp = slot >> (3 * G), m = slot & ((1u << (3 * G)) - 1);
        const uint32_t gx = nbx >> G, gy = nby >> G;
        uint32_t lx = 0, ly = 0, lz = 0;
#pragma unroll
        for (int t = 0; t < (int)G; ++t) {
            lx |= ((m >> (3 * t)) & 1u) << t;
            ly |= ((m >> (3 * t + 1)) & 1u) << t;
            lz |= ((m >> (3 * t + 2)) & 1u) << t;
        }
        bx = ((grp % gx) << G) | lx;
        by = (((grp / gx) % gy) << G) | ly;
        bz = ((grp / (gx * gy)) << G) | lz;
    }
}

enum StorageType { ST_U8 = 0, ST_I8 = 1, ST_U16 = 2, ST_I16 = 3, ST_F32 = 4 };
// Brick layout code = storage type | kQuadFlag: 8-bit voxels kept in yz-quad elements (GeomWide
// bricks, one 8-B load per sample) instead of plain 7x8x8-cell bricks.  Volumes of at most
// kQuadMaxVoxels voxels use it (the quads, 5.7x the voxels, stay cache-resident: C2 256^3
// 459 against 420 Gsamples/s plain); larger ones the plain bricks (C4 HBM 5.70 -> 1.89 GB per
// frame).  The layout code is what the brick helpers below and the march launchers take.
constexpr int kQuadFlag = 0x10;
constexpr size_t kQuadMaxVoxels = 1ull << 25;
// kernel-side tag type of 8-bit voxels T in yz-quad elements
template <typename T>
struct Quad8 {
    T v;
};
// Alternative f32 geometry: a further resident copy of an f32 volume in bricks whose z-pair
// rows never straddle a 128-B line, for the views where a wavefront's lanes sit on different
// brick rows and every straddled line is another L1 miss:
//   kAltFlag  (F32Alt):  7 x 15 x 8 cells (8-element, 64-B rows; 8704-B bricks, 68 lines), for
//                        oblique views (diagonal: 0.81 -> 0.68 ms per C3 frame).
// The frame-filling, side and top views stay in 8^3 bricks (2-4% faster there).  (A 15 x 15 x 8
// z-pair copy for sparse views, superseded by the plain and stencil copies below, is kept as a
// patch: tools/experiments/r04_pruned/.)
constexpr int kAltFlag = 0x20;
#ifndef VR_ALT_BRICK_CELLS
#define VR_ALT_BRICK_CELLS 7, 15, 8
#endif
using GeomAlt = BrickGeom<VR_ALT_BRICK_CELLS>;
// kernel-side tag type of f32 voxels in the kAltFlag layout
struct F32Alt {
    float v;
};
// A plain f32 copy (kPlainF32Flag, kernel tag F32P): one voxel per 4-B element, no z-pair
// duplication (1.2x the voxels against 2.6x), in GeomPlainRows bricks; a sample is 4 x 8-B
// loads (elements x, x + 1 of the rows (y | y+1, z | z+1)).  For sparse views, which read their
// whole copy from HBM every frame.
constexpr int kPlainF32Flag = 0x100;
#ifndef VR_PLAIN_BRICK_CELLS
#define VR_PLAIN_BRICK_CELLS 15, 15, 15
#endif
using GeomPlainRows = BrickGeom<VR_PLAIN_BRICK_CELLS>;
struct F32P {
    float v;
};
// The stencil copy (kStencilF32Flag, kernel tag F32S): plain f32 voxels in GeomStencil bricks,
// which store one element below and two above every cell on each axis (32^3 elements for 29^3
// cells: 128-B rows, 1.34x the voxels, 0.76 GB for 512^3), so a shaded
// sample's central-difference taps are constant element offsets inside the brick: its density
// loads are rows x - 1 .. x + 2 (16 B each) and carry the x differences, y / z taps are 8-B
// loads, no neighbour-brick selection.  For shaded sparse views: the
// reference's default camera 0.260 (15x15x8 z-pairs) -> 0.231 ms (profiles/r03/stencil2/ ..
// stencil4/: 13^3 cells 0.240, 29x13x13 0.236, 29x13x29 / 29x13x61 / 29^3 0.231).
constexpr int kStencilF32Flag = 0x200;
#ifndef VR_STENCIL_BRICK_CELLS
#define VR_STENCIL_BRICK_CELLS 29, 29, 29
#endif
using GeomStencil = BrickGeom<VR_STENCIL_BRICK_CELLS, 1>;
struct F32S {
    float v;
};
// kernel-side tag type of the f32 8^3-brick volume read with the difference field in binary16
// (MarchParams::grad_half); kHalfFieldFlag marks that variant in kernel names and schedule keys
// only (the bricks are the ST_F32 ones)
struct F32H {
    float v;
};
constexpr int kHalfFieldFlag = 0x80;

// Bytes of one voxel of storage type (or layout code) st.
inline size_t storage_size(int st)
{
    switch (st & 0xF) {
        case ST_U8:
        case ST_I8: return 1;
        case ST_U16:
        case ST_I16: return 2;
        default: return 4;
    }
}
// layout code st holds plain 8-bit voxels (one per element, GeomByte bricks)
inline bool byte_storage(int st)
{
    return VR_U8_PLAIN && !(st & kQuadFlag) && (st == ST_U8 || st == ST_I8);
}
inline size_t voxels_per_element(int st)
{
    if (st & (kPlainF32Flag | kStencilF32Flag)) return 1;
    return (st & 0xF) == ST_F32 ? kF32VoxelsPerElement : (byte_storage(st) ? 1 : 4);
}
inline size_t element_size(int st) { return storage_size(st) * voxels_per_element(st); }
// Brick geometry of layout code st: cells along axis a (0 x, 1 y, 2 z), elements per brick.
inline int brick_cells(int st, int a)
{
    if (st & kAltFlag) return GeomAlt::cells(a);
    if (st & kPlainF32Flag) return GeomPlainRows::cells(a);
    if (st & kStencilF32Flag) return GeomStencil::cells(a);
    return byte_storage(st) ? GeomByte::cells(a) : GeomWide::cells(a);
}
inline size_t brick_elems(int st)
{
    if (st & kAltFlag) return GeomAlt::Elems;
    if (st & kPlainF32Flag) return GeomPlainRows::Elems;
    if (st & kStencilF32Flag) return GeomStencil::Elems;
    return byte_storage(st) ? GeomByte::Elems : GeomWide::Elems;
}

// Bricks along axis a of an n-voxel axis: fetch base indices lie in [1, N + 1] (march) and
// gradient taps reach one element below and (in z-pair x/y) two above, i.e. padded [0, N + 3];
// rounded up to whole brick groups.
inline uint32_t bricks_for(uint32_t n, int a, int st)
{
    return ((n + 3) / (uint32_t)brick_cells(st, a) + 1 + kGroupMask) & ~kGroupMask;
}

// ---- Frame rows over ranks (sort-first tiling) ------------------------------
// The frame's rows are cut into blocks of row_block rows and dealt in periods of
// w0 + (n - 1) w blocks: rank 0 takes the first w0 blocks of each period, rank r > 0 the w
// blocks after w0 + (r - 1) w.  w0 = w = 1 (the default) is block b -> rank b mod n.  A smaller
// w0 / w lightens rank 0, which also receives the other shards and assembles the frame
// (vr_set_row_share).  Every rank sends the same number of rows (ncclGather
// counts are equal): the largest share, padded.
struct RowShare {
    uint32_t w0, w;
};
__host__ __device__ inline uint32_t share_period(uint32_t n, RowShare s) { return s.w0 + (n - 1) * s.w; }
__host__ __device__ inline uint32_t share_offset(uint32_t r, RowShare s)
{
    return r == 0 ? 0u : s.w0 + (r - 1) * s.w;
}
// global block of rank r's local block lb
__host__ __device__ inline uint32_t share_global_block(uint32_t lb, uint32_t r, uint32_t n, RowShare s)
{
    const uint32_t w = r == 0 ? s.w0 : s.w;
    return (lb / w) * share_period(n, s) + share_offset(r, s) + lb % w;
}
// owner rank and local block of global block gb
__host__ __device__ inline void share_owner(uint32_t gb, uint32_t n, RowShare s, uint32_t &r,
                                            uint32_t &lb)
{
    const uint32_t P = share_period(n, s), q = gb / P, o = gb - q * P;
    if (o < s.w0) {
        r = 0;
        lb = q * s.w0 + o;
    } else {
        const uint32_t t = o - s.w0;
        r = 1 + t / s.w;
        lb = q * s.w + t % s.w;
    }
}
// blocks rank r owns among the nb blocks of a frame
inline uint32_t share_blocks(uint32_t nb, uint32_t r, uint32_t n, RowShare s)
{
    const uint32_t P = share_period(n, s), q = nb / P, o = nb - q * P;
    const uint32_t w = r == 0 ? s.w0 : s.w, off = share_offset(r, s);
    const uint32_t tail = o > off ? (o - off < w ? o - off : w) : 0u;
    return q * w + tail;
}
// rows of every rank's shard buffer: the largest share
inline uint32_t share_shard_rows(uint32_t height, uint32_t row_block, uint32_t n, RowShare s)
{
    if (row_block == 0 || n == 0 || s.w0 == 0 || s.w == 0) return 0;
    const uint32_t nb = (height + row_block - 1) / row_block;
    uint32_t m = share_blocks(nb, 0, n, s);
    if (n > 1) {
        const uint32_t b1 = share_blocks(nb, 1, n, s);  // rank 1 owns the most of ranks >= 1
        m = b1 > m ? b1 : m;
    }
    return m * row_block;
}

// ---- Kernel parameters (one frame) -------------------------------------------------------
struct MarchParams {
    const void *vol;        // bricked voxels, storage type per kernel instantiation
    const float4 *tf;       // decoded TF texels (linear RGB, linear A), device
    void *out;              // shard buffer (local_rows x W pixels)
    unsigned long long *counters;  // COUNT variant: rays, samples, shaded, steps

    double inv[16];         // inverse of float (proj * view), column-major
    double fw, fh;          // framebuffer W, H as double

    uint32_t nx, ny, nz;
    uint32_t nbx, nby;      // bricks per axis (x, y)
    float fnx, fny, fnz;    // float(nx) ...
    float vmin, range;      // Dataset.min, max - min
    int32_t tf_n;
    float tf_nf;

    float smin[3], smax[3];
    float cam[3];
    float step;
    int32_t nsteps;
    float ert_eps;
    float clear[4];
    float ka, kd, ks;
    int32_t spec_power;

    uint32_t W, H;
    uint32_t row_block, rank, nranks, local_rows;
    uint32_t tiles_x, tiles_y;
    uint32_t tile_order;    // 1 raster, 2 XCD bands, 3 XCD-interleaved super-tiles
    uint32_t supers_x, supers_total;  // super-tile grid (tile_order 3)
    uint32_t wave_w_shift;  // wavefront pixel footprint: 2^shift x (64 >> shift) (8x8: 3)
    int32_t out_format;
    int32_t slab_default;   // slicing is the whole volume (0,0,0)-(1,1,1)
    int32_t pipelined;      // two samples in flight per ray (few waves per CU: see PIPE)
    int32_t pair;           // lane-pair march (march_pair_kernel), 16x8-pixel tiles
    // adaptive tile order (tile_order 4): workgroup b renders tile tile_perm[b] (tile id =
    // ty * tiles_x + tx, ~0 = none; nperm workgroups) and records its duration in
    // tile_cost[tile id]; null: order by tile_order
    const uint32_t *tile_perm;
    uint32_t *tile_cost;
    uint32_t nperm;
    // skip_empty: per brick (index as in cell_offset) the Chebyshev distance in bricks to the
    // nearest brick that can produce a visible sample, capped at kSkipCap; 0 = not empty
    const uint8_t *skip_dist;
    int32_t skip_empty;
    int32_t div_fast;       // density normalisation by reciprocal + fma correction
    // f32 shading: precomputed central differences, element e = {Dx, Dy, Dz} x {z, z + 1}
    // (24 B, same element index as the density); null -> formed from the stencil
    const float *grad;
    // the field holds {Dx, Dy, Dz} x {(y,z), (y,z+1), (y+1,z), (y+1,z+1)} as binary16, scaled by
    // 2^k (field_scale_log2; the shading normalises the gradient, so the scale cancels)
    int32_t grad_half;
    float inv_range;        // RN(1 / range) (div_fast)
    uint32_t share_w0, share_w;  // RowShare of the row blocks over nranks
    // bytes of the volume copy P.vol points at and of the output buffer (bounds-checking
    // debug builds, -DVR_BOUNDS_CHECK: an out-of-range access is printed and skipped)
    unsigned long long vol_bytes, out_bytes;
};

// Launchers (vr_kernels.hip).  All asynchronous on `stream`.
hipError_t launch_march(int storage, bool shade, bool count, const MarchParams &p,
                        hipStream_t stream);
const char *march_kernel_name(int storage, bool shade, bool count, bool skip, bool gf, bool pipe);
// Wavefront count below which a launch uses the pipelined kernel (see build_params).
constexpr uint32_t kPipelineMaxWaves = 24576;  // between N = 2 (16 K) and N = 1 (33 K) at 1080p
constexpr size_t kPipelineMinBytes = 4ull << 30;  // large volumes: always pipelined
constexpr size_t kPipelineMinVoxels = 1ull << 29;
// march_kernel tiles: 16 pixels wide, kMarchRows tall, one lane per pixel (experiment
// builds may set VR_MARCH_ROWS=32: 512-thread workgroups whose 8 wavefronts share one CU's L1)
#ifndef VR_MARCH_ROWS
#define VR_MARCH_ROWS 16
#endif
constexpr uint32_t kMarchRows = VR_MARCH_ROWS;
// super-tiles (tile orders 3 and 4): 2^kSuperShift tiles per side, dealt round-robin over the
// 8 XCDs; experiment builds may change the size (VR_SUPER_SHIFT) and the order an XCD's tile
// list is kept in for the adaptive sort (VR_LIST_ORDER 0: frame raster, 1: super-tile major)
#ifndef VR_SUPER_SHIFT
#define VR_SUPER_SHIFT 2
#endif
#ifndef VR_LIST_ORDER
#define VR_LIST_ORDER 0
#endif
constexpr uint32_t kSuperShift = VR_SUPER_SHIFT;
constexpr uint32_t kSuper = 1u << kSuperShift;
constexpr uint32_t kThreadsPerTile = 16 * kMarchRows;
// vr_render (host output): row bands per frame, each copied to the host while later bands render
constexpr int kHostBands = 4;
constexpr uint32_t kHostBandMinRows = 256;  // shorter frames: one band
// Adaptive tile order: from the per-tile durations of the last launch with the same tile
// geometry, the next launch's workgroup -> tile permutation, longest first within each XCD's
// super-tiles (as tile_order 3 assigns them).
hipError_t launch_order_tiles(const uint32_t *cost, const uint32_t *lists, uint32_t *perm,
                              uint32_t per_xcd, hipStream_t stream);
// launches of one geometry per re-ordering (the order kernel runs on every 4th)
#ifndef VR_REORDER_EVERY
#define VR_REORDER_EVERY 4
#endif
constexpr uint32_t kReorderEvery = VR_REORDER_EVERY;
// schedules kept (one per geometry, stream and march variant; oldest dropped first)
constexpr size_t kMaxTileScheds = 64;
// Wavefront count (single-lane tiling) below which a launch uses the lane-pair kernel.
constexpr uint32_t kPairMaxWaves = 24576;
constexpr uint32_t kPairQuadMaxWaves = 6144;  // below: 4 lanes per ray
hipError_t launch_brick_from_linear(int src_dtype, const void *src, void *dst, uint32_t nx,
                                    uint32_t ny, uint32_t nz, int storage, hipStream_t stream);
// Bricked volume -> linear x-fastest voxels of the storage type, slices [z0, z0 + cz).
hipError_t launch_unbrick(int storage, const void *bricks, void *dst, uint32_t nx, uint32_t ny,
                          uint32_t z0, uint32_t cz, hipStream_t stream);
// Synthetic volume into a LINEAR buffer of the storage type (then bricked).
hipError_t launch_generate(int kind, int storage, void *dst_linear, uint32_t nx, uint32_t ny,
                           uint32_t nz, const float *params_dev, int nparams,
                           hipStream_t stream);
hipError_t launch_assemble(const void *gathered, void *out, int out_format, uint32_t W,
                           uint32_t H, uint32_t row_block, uint32_t nranks,
                           uint32_t shard_rows, RowShare share, hipStream_t stream);
// Integer range of a LINEAR buffer of 32-bit or 64-bit voxels (vr_dtype 5..9): out3_dev = {min,
// max, not-all-integers flag}, pre-set by the caller to {INT_MAX, INT_MIN, 0}.  Integers are
// counted only in [-32768, 65535]; -0.0, NaN, infinities and fractions set the flag.
hipError_t launch_int_range(int src_dtype, const void *src, size_t count, int *out3_dev,
                            hipStream_t stream);
// min/max over a LINEAR buffer of the storage type (ordered-uint encoding in minmax_dev).
hipError_t launch_minmax(int storage, const void *linear, size_t count, float *minmax_dev,
                         hipStream_t stream);

// Empty-space skipping (skip_empty): per-brick value range of the stored elements, then per
// (volume, TF) the capped Chebyshev distance field over the brick grid (1 byte per brick;
// scratch_dev: the same size, for the separable passes).
constexpr int kSkipCap = 16;
// f32 gradient field (see MarchParams::grad) from the bricked density: same brick grid.
constexpr size_t kGradElemBytes = 24;
// half: the binary16 field of MarchParams::grad_half, each difference times 2^scale_log2 and
// clamped to +-65504 (NaN kept) before rounding to nearest even
hipError_t launch_grad_field(const float *bricks, float *grad, uint32_t nx, uint32_t ny,
                             uint32_t nz, bool half, int scale_log2, hipStream_t stream);
// The f32 copy in layout `storage` (kAltFlag / kPlainF32Flag / kStencilF32Flag) straight from the
// 8^3 z-pair bricks: the same bytes as launch_unbrick + launch_brick_from_linear.
hipError_t launch_rebrick_f32(const float *src_bricks, void *dst, uint32_t nx, uint32_t ny,
                              uint32_t nz, int storage, hipStream_t stream);
// The binary16 field's scale: the largest k in [-120, 120] with B 2^k <= 65504, where
// B = max(vmax, 0) - min(vmin, 0) bounds every central difference of voxels in [vmin, vmax]
// (and of the zero border); 0 when B is 0 or not finite.  oracle/oracle.c restates it.
inline int field_scale_log2(float vmin, float vmax)
{
    const double B = (double)(vmax > 0.0f ? vmax : 0.0f) - (double)(vmin < 0.0f ? vmin : 0.0f);
    if (!(B > 0.0) || B > 1e300) return 0;
    int k = 0;
    while (k > -120 && B * std::ldexp(1.0, k) > 65504.0) --k;
    while (k < 120 && B * std::ldexp(1.0, k + 1) <= 65504.0) ++k;
    return k;
}
hipError_t launch_brick_range(int storage, const void *bricks, uint32_t nbx, uint32_t nby,
                              uint32_t nbz, float2 *range_dev, hipStream_t stream);
hipError_t launch_skip_dist(const float2 *range_dev, uint32_t nbx, uint32_t nby, uint32_t nbz,
                            const uint32_t *tf_nz_dev, int tf_n, float vmin, float vrange,
                            uint8_t *dist_dev, uint8_t *scratch_dev, hipStream_t stream);

#ifdef VR_WG_TIMES
hipError_t debug_wg_times_reset();
hipError_t debug_wg_times_read(unsigned long long *out, unsigned int max, unsigned int *count);
#endif

}  // namespace vr
