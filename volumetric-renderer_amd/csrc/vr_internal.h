// vr_internal.h — shared definitions between the C-ABI layer (vr_api.hip) and the
// gfx950 kernels (vr_kernels.hip).  Not installed; the public boundary is include/vr/vr.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace vr {

// ---- Bricked volume layout in HBM -------------------------------------------------------
// The logical volume (nx, ny, nz) is shifted by kPad = 2 zero voxels on the low side of each
// axis ("padded index" p = logical + 2) and cut into bricks of kBrick^3 base cells.  Brick b
// stores padded indices [16 b, 16 b + 16] on each axis (kStore = 17 = 16 + 1-voxel apron), so
// the 2x2x2 footprint of every trilinear fetch lies in ONE brick: one base address plus the 7
// immediate offsets {1, 17, 18, 289, 290, 306, 307}.  Voxels outside [0, N) are stored as 0,
// which realises CLAMP_TO_BORDER/TRANSPARENT_BLACK without a bounds test.  Bricks are ordered
// x-fastest in the brick grid; the odd 17-voxel strides keep neighbouring rows/slices of a
// brick out of the same L1/L2 sets (a 512^3 dense f32 volume has 2 KiB / 1 MiB strides).
constexpr int kBrick = 16;
constexpr int kStore = 17;
constexpr int kBrickVoxels = kStore * kStore * kStore;  // 4913
constexpr int kPad = 2;

// Bricks per axis: base padded indices of every fetch lie in [0, N + 2] (march fetches in
// [1, N + 1]; gradient taps one further either side).
inline uint32_t bricks_for(uint32_t n) { return (n + 3 + kBrick - 1) / kBrick; }

enum StorageType { ST_U8 = 0, ST_I8 = 1, ST_U16 = 2, ST_I16 = 3, ST_F32 = 4 };

inline size_t storage_size(int st)
{
    switch (st) {
        case ST_U8:
        case ST_I8: return 1;
        case ST_U16:
        case ST_I16: return 2;
        default: return 4;
    }
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
    int32_t out_format;
};

// Launchers (vr_kernels.hip).  All asynchronous on `stream`.
hipError_t launch_march(int storage, bool shade, bool count, const MarchParams &p,
                        hipStream_t stream);
const char *march_kernel_name(int storage, bool shade, bool count);
hipError_t launch_brick_from_linear(int src_dtype, const void *src, void *dst, uint32_t nx,
                                    uint32_t ny, uint32_t nz, int storage, hipStream_t stream);
hipError_t launch_generate(int kind, int storage, void *dst, uint32_t nx, uint32_t ny,
                           uint32_t nz, const float *params_dev, int nparams,
                           hipStream_t stream);
hipError_t launch_assemble(const void *gathered, void *out, int out_format, uint32_t W,
                           uint32_t H, uint32_t row_block, uint32_t nranks,
                           uint32_t shard_rows, hipStream_t stream);
hipError_t launch_minmax(int storage, const void *bricks, uint32_t nx, uint32_t ny,
                         uint32_t nz, float *minmax_dev, hipStream_t stream);

}  // namespace vr
