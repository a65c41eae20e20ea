// vr_kernels.hip — gfx950 (CDNA4) kernels of the volume ray-marcher.
//
// The hot path is march_kernel: one lane per pixel, a 64-lane wavefront marches a 16x4
// pixel strip by default (vr_params.wave_shape), a 256-thread workgroup a 16x16 tile.  It
// restates the
// reference fragment shader res/shaders/volume.frag:21-52 plus the Vulkan fixed-function
// state it runs under (src/rendering/offscreen_pass.cpp: cube ray entry :55-90 + cull
// :680-681 + depth clip :701-712, border trilinear sampler :1014-1039, sRGB TF sampler
// :1076/:1125-1150, blend :715-725 over the clear colour :170-173, UNORM8 store :293).
//
// Design points (DESIGN.md has the roofline discussion):
//  * memory-bound gather, no MFMA: each density sample is a 2x2x2 trilinear footprint;
//  * bricked native-dtype volume with paired elements (vr_internal.h): f32 z-pairs (a sample
//    is 2 x 16-B loads), 8/16-bit yz-quads (one load); zero apron = CLAMP_TO_BORDER without
//    bounds tests; shaded f32 frames read a precomputed central-difference field;
//  * TF decoded to linear float4 (with forward differences) once per upload on the host and
//    staged in LDS;
//  * XCD-aware tile order (block_tile / order_tiles_kernel): tiles grouped in 64x64-pixel
//    super-tiles dealt over the 8 XCDs (balance); each XCD dispatches its tiles longest first
//    by the last launches' durations, stable within a duration octave (co-running tiles stay
//    neighbours in its L2);
//  * pipelined variant (two samples of a ray in flight) for shaded frames, small launches and
//    volumes >= 4 GiB; lane-group variant for small shaded launches with serial frames;
//  * fp contraction is OFF (pragma below + -ffp-contract=off): every fused multiply-add is
//    an explicit fmaf(), matching the CPU oracle's operation order bit for bit.
#include "vr_exact_math.h"
#include "vr_internal.h"

#include <cstdlib>
#include <string>
#include <type_traits>
#include <vector>

#pragma clang fp contract(off)

namespace vr {
namespace {

constexpr int kTile = 16;       // pixels per workgroup side
constexpr int kThreads = 256;   // lane-pair kernel workgroup: 4 waves
constexpr int kTfLds = 256;     // TF texels staged in LDS
constexpr int kTfLut = 2 * (kTfLds + 2);  // float4s of the staged LUT (tf_lookup: + 2 sentinels)

__device__ __forceinline__ float lerpf(float a, float b, float w) { return fmaf(w, b - a, a); }

// Bounds-checking debug builds (-DVR_BOUNDS_CHECK): an out-of-range index is printed (the first
// 32 per process) and the access redirected to element 0.  Product builds compile it away.
#ifdef VR_BOUNDS_CHECK
__device__ unsigned int g_oob_reports;
__device__ __noinline__ void oob_report(int what, unsigned long long a, unsigned long long b)
{
    if (atomicAdd(&g_oob_reports, 1u) < 32u)
        printf("VR_OOB what=%d index=%llu limit=%llu block=%u thread=%u\n", what, a, b,
               (unsigned)blockIdx.x, (unsigned)threadIdx.x);
}
#define VR_OOB(what, a, b) ((unsigned long long)(a) >= (unsigned long long)(b) ? (oob_report((what), (a), (b)), true) : false)
#else
#define VR_OOB(what, a, b) false
#endif

// Two independent lerps in one packed-FP32 pair (v_pk_add_f32 + v_pk_fma_f32): the same IEEE
// operations per element as lerpf, so bit-identical to two scalar lerps.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v lerp2(f2v a, f2v b, float w)
{
    const f2v ww = {w, w};
    return __builtin_elementwise_fma(ww, b - a, a);
}

// Unaligned-capable vector types: element pairs are 4- or 8-byte aligned, and gfx950 global
// loads only need dword alignment, so these compile to single global_load_dwordx2/x4.
typedef float f2a __attribute__((ext_vector_type(2))) __attribute__((aligned(4)));
typedef float f4a __attribute__((ext_vector_type(4))) __attribute__((aligned(4)));
typedef uint32_t u2a __attribute__((ext_vector_type(2))) __attribute__((aligned(4)));
typedef uint32_t u4a __attribute__((ext_vector_type(4))) __attribute__((aligned(4)));

template <typename VT>
struct is_quad8 : std::false_type {};
template <typename T>
struct is_quad8<Quad8<T>> : std::true_type {};
// bytes per element; 32-bit words per element (quad layouts)
// VT is the voxel type, or Quad8<T> for 8-bit voxels in yz-quads (vr_internal.h kQuadFlag);
// Vox<VT> the voxel type either way
template <typename VT>
struct VoxOf {
    using type = VT;
};
template <typename T>
struct VoxOf<Quad8<T>> {
    using type = T;
};
template <>
struct VoxOf<F32Alt> {
    using type = float;
};
template <>
struct VoxOf<F32H> {
    using type = float;
};
template <>
struct VoxOf<F32P> {
    using type = float;
};
template <>
struct VoxOf<F32S> {
    using type = float;
};
template <typename VT>
using Vox = typename VoxOf<VT>::type;
template <typename VT>
constexpr bool kIsQuad8 = is_quad8<VT>::value;
// the f32 volume read with the binary16 difference field (MarchParams::grad_half)
template <typename VT>
constexpr bool kHalfField = std::is_same<VT, F32H>::value;
// f32 z-pair elements (8^3 bricks, or GeomAlt bricks for F32Alt)
template <typename VT>
constexpr bool kZPair = std::is_same<Vox<VT>, float>::value;
// f32 voxels one per element (the F32P copy, or every f32 volume in VR_F32_PLAIN builds)
template <typename VT>
constexpr bool kPlainF32 = std::is_same<VT, F32P>::value || std::is_same<VT, F32S>::value ||
                          (kZPair<VT> && VR_F32_PLAIN);
// the stencil copy (GeomStencil: gradient taps inside the brick)
template <typename VT>
constexpr bool kStencil = std::is_same<VT, F32S>::value;
// VR_STENCIL_WIDE = 1 (default): the stencil copy's density loads are 16 B from x - 1 (x - 1 ..
// x + 2 of each row), so a shaded sample's x differences need no further load.  0: 8-B density
// loads and one 16-B load per row at shade time (shaded default camera 0.240 -> 0.260 ms,
// profiles/r03/stencil_copy/)
#ifndef VR_STENCIL_WIDE
#define VR_STENCIL_WIDE 1
#endif
template <typename VT>
constexpr bool kStencilWide = kStencil<VT> && VR_STENCIL_WIDE;
// 8-bit volumes stored one voxel per element (VR_U8_PLAIN, vr_internal.h)
template <typename VT>
constexpr bool kPlainByte = sizeof(VT) == 1 && VR_U8_PLAIN && !kIsQuad8<VT>;
template <typename VT>
constexpr int kElemBytes = kZPair<VT> ? (kPlainF32<VT> ? 4 : 8)
                                      : (kPlainByte<VT> ? 1 : 4 * (int)sizeof(VT));
template <typename VT>
using GeomOf = std::conditional_t<kPlainByte<VT>, GeomByte,
                                  std::conditional_t<std::is_same<VT, F32Alt>::value, GeomAlt,
                                  std::conditional_t<std::is_same<VT, F32P>::value, GeomPlainRows,
                                  std::conditional_t<kStencil<VT>, GeomStencil, GeomWide>>>>;
template <typename VT>
constexpr int kQuadWords = sizeof(VT) == 1 ? 1 : 2;

// Element index of padded cell (pi, pj, pk) in the bricked layout (vr_internal.h).  64-bit:
// a 2048^3 volume has 257^3 x 729 elements.  (A 32-bit index with SGPR-base loads for
// volumes < 4 GiB measured slower on the shaded kernel and on the diagonal view.)
template <typename VT>
__device__ __forceinline__ size_t cell_offset(int pi, int pj, int pk, uint32_t nbx, uint32_t nby)
{
    using G = GeomOf<VT>;
    const uint32_t ux = (uint32_t)pi, uy = (uint32_t)pj, uz = (uint32_t)pk;
    const uint32_t bx = ux / G::BX, by = uy / G::BY, bz = uz / G::BZ;
    const uint32_t l = ((uz - bz * G::BZ + G::Lo) * G::EY + (uy - by * G::BY + G::Lo)) * G::EX +
                       (ux - bx * G::BX + G::Lo);
    return (size_t)brick_slot(bx, by, bz, nbx, nby) * (size_t)G::Elems + l;
}

// Trilinear filter of a 2x2x2 cell given its voxels v[dz][dy][dx]: lerp x, then y, then z
// (the oracle's tri_cell operation order).  tri8x2: two independent cells at once (packed).
__device__ __forceinline__ float tri8(float v000, float v100, float v010, float v110, float v001,
                                      float v101, float v011, float v111, float ax, float ay,
                                      float az)
{
    // scalar: packing the z = 0 / z = 1 halves into v_pk_fma_f32 pairs (8 instructions for 14)
    // measured 2-7% slower (u8 C4 view sweep, profiles/r02/valu/packed_tri_ab.txt)
    const float c00 = lerpf(v000, v100, ax);
    const float c10 = lerpf(v010, v110, ax);
    const float c01 = lerpf(v001, v101, ax);
    const float c11 = lerpf(v011, v111, ax);
    const float c0 = lerpf(c00, c10, ay);
    const float c1 = lerpf(c01, c11, ay);
    return lerpf(c0, c1, az);
}
// element-wise: .x = tri8 of the .x voxels, .y = tri8 of the .y voxels
__device__ __forceinline__ f2v tri8x2(f2v v000, f2v v100, f2v v010, f2v v110, f2v v001,
                                      f2v v101, f2v v011, f2v v111, float ax, float ay, float az)
{
    const f2v c00 = lerp2(v000, v100, ax);
    const f2v c10 = lerp2(v010, v110, ax);
    const f2v c01 = lerp2(v001, v101, ax);
    const f2v c11 = lerp2(v011, v111, ax);
    const f2v c0 = lerp2(c00, c10, ay);
    const f2v c1 = lerp2(c01, c11, ay);
    return lerp2(c0, c1, az);
}

// Byte b of w as the voxel value (float of an 8-bit integer is exact).
template <typename VT>
__device__ __forceinline__ float byte_value(uint32_t w, int b)
{
    const uint32_t u = (w >> (8 * b)) & 0xFFu;
    if constexpr (std::is_signed<Vox<VT>>::value) return (float)(int)(int8_t)u;
    return (float)u;
}

// Component c of a yz-quad element held in 32-bit words w (c: 0 (y,z), 1 (y,z+1), 2 (y+1,z),
// 3 (y+1,z+1)); float(v) is exact for 8/16-bit voxels.
template <typename VT>
__device__ __forceinline__ float qc(const uint32_t *w, int c)
{
    if constexpr (sizeof(VT) == 1) {
        const uint32_t b = (w[0] >> (8 * c)) & 0xFFu;
        if constexpr (std::is_signed<Vox<VT>>::value) return (float)(int)(int8_t)b;
        return (float)b;
    } else {
        const uint32_t h = (w[c >> 1] >> (16 * (c & 1))) & 0xFFFFu;
        if constexpr (std::is_signed<Vox<VT>>::value) return (float)(int)(int16_t)h;
        return (float)h;
    }
}

// Load the elements at e and e + 1 (one 8-B or 16-B load) / the element at e alone.
template <typename VT>
__device__ __forceinline__ void quad_load2(const char *__restrict__ base, size_t e, uint32_t *w)
{
    const char *p = base + e * kElemBytes<VT>;
    if constexpr (sizeof(VT) == 1) {
        const u2a r = *reinterpret_cast<const u2a *>(p);
        w[0] = r.x;
        w[1] = r.y;
    } else {
        const u4a r = *reinterpret_cast<const u4a *>(p);
        w[0] = r.x;
        w[1] = r.y;
        w[2] = r.z;
        w[3] = r.w;
    }
}
template <typename VT>
__device__ __forceinline__ void quad_load1(const char *__restrict__ base, size_t e, uint32_t *w)
{
    const char *p = base + e * kElemBytes<VT>;
    if constexpr (sizeof(VT) == 1) {
        w[0] = *reinterpret_cast<const uint32_t *>(p);
    } else {
        const u2a r = *reinterpret_cast<const u2a *>(p);
        w[0] = r.x;
        w[1] = r.y;
    }
}
__device__ __forceinline__ f4a zpair_load2(const char *__restrict__ base, size_t e)
{
    return *reinterpret_cast<const f4a *>(base + e * 8);
}
__device__ __forceinline__ f2a zpair_load1(const char *__restrict__ base, size_t e)
{
    return *reinterpret_cast<const f2a *>(base + e * 8);
}

// The 8 voxels of the cell whose low corner element is e:
//   f32 z-pair: rows y and y+1, elements x and x+1 -> 2 x 16-B loads;
//   8/16-bit yz-quad: elements x and x+1 -> 1 x 8-B (u8) / 16-B (u16) load.
// The raw loaded words of one cell, decoded later.  The pipelined march keeps the words of the
// sample in flight in the Stage and decodes (byte extraction, int -> float) only when the
// sample is consumed, after the next sample's loads are issued: decoding at load time put the
// decode, and with it a wait for the loads, before the loop back-edge (vmcnt(0) right after
// issue), so only one sample per ray was really in flight.
template <typename VT, typename = void>
struct CellRaw {  // generic: the decoded cell itself (loaded and decoded together)
    float v[8];
};
template <typename VT>
struct CellRaw<VT, std::enable_if_t<kZPair<VT> && !kPlainF32<VT>>> {
    f4a r0, r1;  // rows y and y + 1: elements x, x + 1 as z-pairs
};
template <typename VT>
struct CellRaw<VT, std::enable_if_t<kStencilWide<VT>>> {
    f4a q[4];  // rows (y|y+1, z|z+1): elements x - 1 .. x + 2
};
template <typename VT>
struct CellRaw<VT, std::enable_if_t<kPlainByte<VT> && GeomByte::EX == 8>> {
    u4a q0, q1;    // slices z and z + 1: the 16 bytes from the 4-aligned address at or below e
    uint32_t sh;   // e mod 4
};

// (Cross-lane sharing of a cell's loads, VR_U8_SHARE for 8-bit and VR_F32_SHARE for f32 cells,
// measured 1.5-1.8x and 1.6x slower in round 5: tools/experiments/r05_pruned/.)

// the stencil copy with 16-B density loads keeps each row's x - 1 / x + 2 voxels for the
// gradient (row r = dy + 2 dz)
template <typename VT, typename = void>
struct CellTaps {};
template <typename VT>
struct CellTaps<VT, std::enable_if_t<kStencilWide<VT>>> {
    float xm[4], xp[4];
};
template <typename VT>
struct Cell8 : CellTaps<VT> {
    float v[8];  // index dx + 2 dy + 4 dz
    // issue the loads of the cell whose low corner element is e (decode() converts them)
    static __device__ __forceinline__ void issue(CellRaw<VT> &w, const char *__restrict__ base,
                                                 size_t e)
    {
        if constexpr (kZPair<VT> && !kPlainF32<VT>) {
            w.r0 = zpair_load2(base, e);
            w.r1 = zpair_load2(base, e + GeomOf<VT>::Row);
        } else if constexpr (kStencilWide<VT>) {
            using G = GeomOf<VT>;
#pragma unroll
            for (int r = 0; r < 4; ++r)
                w.q[r] = *reinterpret_cast<const f4a *>(
                    base + (e - 1 + (size_t)((r & 1) * G::Row + (r >> 1) * G::Slice)) * 4);
        } else if constexpr (kPlainByte<VT> && GeomByte::EX == 8) {
            const size_t a = e & ~(size_t)3;
            w.sh = (uint32_t)e & 3u;
            w.q0 = *reinterpret_cast<const u4a *>(base + a);
            w.q1 = *reinterpret_cast<const u4a *>(base + a + GeomByte::Slice);
        } else {
            Cell8 c;
            c.load(base, e);
#pragma unroll
            for (int i = 0; i < 8; ++i) w.v[i] = c.v[i];
        }
    }
    __device__ __forceinline__ void decode(const CellRaw<VT> &w)
    {
        if constexpr (kZPair<VT> && !kPlainF32<VT>) {
            v[0] = w.r0.x;
            v[4] = w.r0.y;
            v[1] = w.r0.z;
            v[5] = w.r0.w;
            v[2] = w.r1.x;
            v[6] = w.r1.y;
            v[3] = w.r1.z;
            v[7] = w.r1.w;
        } else if constexpr (kStencilWide<VT>) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                this->xm[r] = w.q[r].x;
                v[2 * r] = w.q[r].y;
                v[2 * r + 1] = w.q[r].z;
                this->xp[r] = w.q[r].w;
            }
        } else if constexpr (kPlainByte<VT> && GeomByte::EX == 8) {
            const uint32_t q[4] = {__builtin_amdgcn_alignbyte(w.q0.y, w.q0.x, w.sh),
                                   __builtin_amdgcn_alignbyte(w.q0.w, w.q0.z, w.sh),
                                   __builtin_amdgcn_alignbyte(w.q1.y, w.q1.x, w.sh),
                                   __builtin_amdgcn_alignbyte(w.q1.w, w.q1.z, w.sh)};
#pragma unroll
            for (int r = 0; r < 4; ++r) {  // r = dy + 2 dz
                v[2 * r] = byte_value<VT>(q[r], 0);
                v[2 * r + 1] = byte_value<VT>(q[r], 1);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = w.v[i];
        }
    }
    __device__ __forceinline__ void load(const char *__restrict__ base, size_t e)
    {
        if constexpr (kStencilWide<VT>) {
            CellRaw<VT> w;
            issue(w, base, e);
            decode(w);
        } else if constexpr (kPlainF32<VT>) {  // rows (y, z), (y+1, z), (y, z+1), (y+1, z+1)
            using G = GeomOf<VT>;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const f2a q = *reinterpret_cast<const f2a *>(
                    base + (e + (size_t)((r & 1) * G::Row + (r >> 1) * G::Slice)) * 4);
                v[2 * r] = q.x;
                v[2 * r + 1] = q.y;
            }
        } else if constexpr (kZPair<VT>) {
            const f4a r0 = zpair_load2(base, e);
            const f4a r1 = zpair_load2(base, e + GeomOf<VT>::Row);
            v[0] = r0.x;
            v[4] = r0.y;
            v[1] = r0.z;
            v[5] = r0.w;
            v[2] = r1.x;
            v[6] = r1.y;
            v[3] = r1.z;
            v[7] = r1.w;
        } else if constexpr (kPlainByte<VT> && GeomByte::EX == 4) {
            // 4-byte rows (3-cell-wide bricks): the row of the cell starts at the 4-aligned
            // address at or below e; one dwordx2 per slice holds rows y and y+1, the cell's
            // voxels at bytes s, s+1 of each dword (s = x <= 2)
            const size_t a = e & ~(size_t)3;
            const uint32_t sh = 8u * ((uint32_t)e & 3u);
            const u2a q0 = *reinterpret_cast<const u2a *>(base + a);
            const u2a q1 = *reinterpret_cast<const u2a *>(base + a + GeomByte::Slice);
            const uint32_t w[4] = {q0.x >> sh, q0.y >> sh, q1.x >> sh, q1.y >> sh};
#pragma unroll
            for (int r = 0; r < 4; ++r) {  // r = dy + 2 dz
                v[2 * r] = byte_value<VT>(w[r], 0);
                v[2 * r + 1] = byte_value<VT>(w[r], 1);
            }
        } else if constexpr (kPlainByte<VT>) {
            // one dwordx4 per slice from the 4-aligned address at or below e (bricks and rows
            // are 4-aligned: s = e mod 4 = x mod 4): bytes s, s+1 = row y, s+8, s+9 = row y+1
            static_assert(GeomByte::EX == 8, "plain 8-bit rows are 4 or 8 bytes");
            const size_t a = e & ~(size_t)3;
            const uint32_t sh = (uint32_t)e & 3u;
            const u4a q0 = *reinterpret_cast<const u4a *>(base + a);
            const u4a q1 = *reinterpret_cast<const u4a *>(base + a + GeomByte::Slice);
            const uint32_t w[4] = {__builtin_amdgcn_alignbyte(q0.y, q0.x, sh),
                                   __builtin_amdgcn_alignbyte(q0.w, q0.z, sh),
                                   __builtin_amdgcn_alignbyte(q1.y, q1.x, sh),
                                   __builtin_amdgcn_alignbyte(q1.w, q1.z, sh)};
#pragma unroll
            for (int r = 0; r < 4; ++r) {  // r = dy + 2 dz
                v[2 * r] = byte_value<VT>(w[r], 0);
                v[2 * r + 1] = byte_value<VT>(w[r], 1);
            }
        } else {
            constexpr int QW = kQuadWords<VT>;
            uint32_t w[2 * QW];
            quad_load2<VT>(base, e, w);
            v[0] = qc<VT>(w, 0);
            v[4] = qc<VT>(w, 1);
            v[2] = qc<VT>(w, 2);
            v[6] = qc<VT>(w, 3);
            v[1] = qc<VT>(w + QW, 0);
            v[5] = qc<VT>(w + QW, 1);
            v[3] = qc<VT>(w + QW, 2);
            v[7] = qc<VT>(w + QW, 3);
        }
    }
    __device__ __forceinline__ float tri(float ax, float ay, float az) const
    {
        return tri8(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], ax, ay, az);
    }
};

// Central-difference gradient (extension): per axis e, the trilinear filter (the centre
// cell's weights, tri8's lerp order) of the per-voxel difference D_e(c) = v(c+e) - v(c-e)
// over the cell's 8 corners -- the oracle's grad_cell.  The differences need the 4-wide
// stencil's 24 outer voxels (10 loads for z-pair f32, 6 for yz-quads).  Taps one element
// below, or two above in z-pair x/y, may sit in the neighbouring brick (the apron covers
// +1): the per-axis deltas pick that brick.  Corner index: dx + 2 dy + 4 dz.
// PACKED: D_x / D_y and their filters as packed-FP32 pairs (fewer VALU, more VGPRs; the
// scalar form serves the register-tight skip-empty kernel).
template <bool PACKED>
__device__ __forceinline__ void grad_filter(const float *dx, const float *dy, const float *dz,
                                            float ax, float ay, float az, float &gx, float &gy,
                                            float &gz)
{
    if constexpr (PACKED) {
        const f2v g = tri8x2(f2v{dx[0], dy[0]}, f2v{dx[1], dy[1]}, f2v{dx[2], dy[2]},
                             f2v{dx[3], dy[3]}, f2v{dx[4], dy[4]}, f2v{dx[5], dy[5]},
                             f2v{dx[6], dy[6]}, f2v{dx[7], dy[7]}, ax, ay, az);
        gx = g.x;
        gy = g.y;
    } else {
        gx = tri8(dx[0], dx[1], dx[2], dx[3], dx[4], dx[5], dx[6], dx[7], ax, ay, az);
        gy = tri8(dy[0], dy[1], dy[2], dy[3], dy[4], dy[5], dy[6], dy[7], ax, ay, az);
    }
    gz = tri8(dz[0], dz[1], dz[2], dz[3], dz[4], dz[5], dz[6], dz[7], ax, ay, az);
}

template <typename VT, bool PACKED>
__device__ __forceinline__ void gradient(const char *__restrict__ base, size_t e,
                                         const Cell8<VT> &c, int pi, int pj, int pk,
                                         uint32_t nbx, uint32_t nby, long by_stride,
                                         long bz_stride, float ax, float ay, float az, float &gx,
                                         float &gy, float &gz)
{
    using G = GeomOf<VT>;
    constexpr long S = G::Row, S2 = G::Slice, B = G::Elems;
    constexpr long Lx = G::BX - 1, Ly = G::BY - 1, Lz = G::BZ - 1;
    const int lx = pi % G::BX, ly = pj % G::BY, lz = pk % G::BZ;
    // element-index deltas of the taps one element below / two above the cell's low corner;
    // a tap outside the brick reads the neighbouring brick (constant strides in x-fastest
    // brick order, the neighbour's slot otherwise)
    long dxm, dxp, dym, dyp, dzm, dzp;
    if constexpr (G::Lo == 1) {  // the stencil copy: every tap inside the brick
        dxm = -1;
        dxp = 2;
        dym = -S;
        dyp = 2 * S;
        dzm = -S2;
        dzp = 2 * S2;
    } else if constexpr (kGroupShift == 0) {
        dxm = lx > 0 ? -1 : (Lx - B);
        dxp = lx < Lx ? 2 : (B - (Lx - 1));
        dym = ly > 0 ? -S : (Ly * S - by_stride);
        dyp = ly < Ly ? 2 * S : (by_stride - (Ly - 1) * S);
        dzm = lz > 0 ? -S2 : (Lz * S2 - bz_stride);
        dzp = lz < Lz ? 2 * S2 : (bz_stride - (Lz - 1) * S2);
    } else {
        auto cross = [&](int ox, int oy, int oz) {
            return (long)cell_offset<VT>(pi + ox, pj + oy, pk + oz, nbx, nby) - (long)e;
        };
        dxm = lx > 0 ? -1 : cross(-1, 0, 0);
        dxp = lx < Lx ? 2 : cross(2, 0, 0);
        dym = ly > 0 ? -S : cross(0, -1, 0);
        dyp = ly < Ly ? 2 * S : cross(0, 2, 0);
        dzm = lz > 0 ? -S2 : cross(0, 0, -1);
        dzp = lz < Lz ? 2 * S2 : cross(0, 0, 2);
    }
    (void)dyp;
    (void)dzp;
    const float *v = c.v;
    float Dx[8], Dy[8], Dz[8];
    if constexpr (kPlainF32<VT>) {
        auto ld1 = [&](long o) { return *reinterpret_cast<const float *>(base + (e + o) * 4); };
        auto ld2 = [&](long o) { return *reinterpret_cast<const f2a *>(base + (e + o) * 4); };
#pragma unroll
        for (int dz_ = 0; dz_ < 2; ++dz_)
#pragma unroll
            for (int dy_ = 0; dy_ < 2; ++dy_) {
                const int o = 2 * dy_ + 4 * dz_;
                const long r = dy_ * S + dz_ * S2;
                if constexpr (kStencilWide<VT>) {  // taps kept by the density loads
                    Dx[o] = v[o + 1] - c.xm[dy_ + 2 * dz_];
                    Dx[o + 1] = c.xp[dy_ + 2 * dz_] - v[o];
                } else if constexpr (kStencil<VT>) {  // x - 1 .. x + 2 in one load
                    const f4a q = *reinterpret_cast<const f4a *>(base + (e - 1 + r) * 4);
                    Dx[o] = v[o + 1] - q.x;
                    Dx[o + 1] = q.w - v[o];
                } else {
                    Dx[o] = v[o + 1] - ld1(dxm + r);
                    Dx[o + 1] = ld1(dxp + r) - v[o];
                }
            }
#pragma unroll
        for (int dz_ = 0; dz_ < 2; ++dz_) {
            const f2a m = ld2(dym + dz_ * S2), q = ld2(dyp + dz_ * S2);
            const int o = 4 * dz_;
            Dy[o] = v[o + 2] - m.x;
            Dy[o + 1] = v[o + 3] - m.y;
            Dy[o + 2] = q.x - v[o];
            Dy[o + 3] = q.y - v[o + 1];
        }
#pragma unroll
        for (int dy_ = 0; dy_ < 2; ++dy_) {
            const f2a m = ld2(dzm + dy_ * S), q = ld2(dzp + dy_ * S);
            const int o = 2 * dy_;
            Dz[o] = v[o + 4] - m.x;
            Dz[o + 1] = v[o + 5] - m.y;
            Dz[o + 4] = q.x - v[o];
            Dz[o + 5] = q.y - v[o + 1];
        }
    } else if constexpr (kZPair<VT>) {
        // z-pairs (.x = z, .y = z + 1) of the x - 1 and x + 2 columns, rows y and y + 1
        const f2a xm0 = zpair_load1(base, e + dxm), xm1 = zpair_load1(base, e + dxm + S);
        const f2a xp0 = zpair_load1(base, e + dxp), xp1 = zpair_load1(base, e + dxp + S);
        // elements x, x + 1 of rows y - 1 and y + 2: (.x, .y) column x, (.z, .w) column x + 1
        const f4a ym = zpair_load2(base, e + dym), yp = zpair_load2(base, e + dyp);
        // elements x, x + 1 at z - 1 (pairs z - 1, z) and z + 1 (pairs z + 1, z + 2)
        const f4a zm0 = zpair_load2(base, e + dzm), zm1 = zpair_load2(base, e + dzm + S);
        const f4a zp0 = zpair_load2(base, e + S2), zp1 = zpair_load2(base, e + S2 + S);
        Dx[0] = v[1] - xm0.x; Dx[1] = xp0.x - v[0]; Dx[2] = v[3] - xm1.x; Dx[3] = xp1.x - v[2];
        Dx[4] = v[5] - xm0.y; Dx[5] = xp0.y - v[4]; Dx[6] = v[7] - xm1.y; Dx[7] = xp1.y - v[6];
        Dy[0] = v[2] - ym.x;  Dy[1] = v[3] - ym.z;  Dy[2] = yp.x - v[0];  Dy[3] = yp.z - v[1];
        Dy[4] = v[6] - ym.y;  Dy[5] = v[7] - ym.w;  Dy[6] = yp.y - v[4];  Dy[7] = yp.w - v[5];
        Dz[0] = v[4] - zm0.x; Dz[1] = v[5] - zm0.z; Dz[2] = v[6] - zm1.x; Dz[3] = v[7] - zm1.z;
        Dz[4] = zp0.y - v[0]; Dz[5] = zp0.w - v[1]; Dz[6] = zp1.y - v[2]; Dz[7] = zp1.w - v[3];
    } else if constexpr (kPlainByte<VT>) {
        // the 24 outer voxels one byte load each (8-bit shading is off the benchmarked path)
        auto ld = [&](long o) {
            return byte_value<VT>((uint32_t)*reinterpret_cast<const uint8_t *>(base + e + o), 0);
        };
#pragma unroll
        for (int dz_ = 0; dz_ < 2; ++dz_)
#pragma unroll
            for (int dy_ = 0; dy_ < 2; ++dy_) {
                const int o = 2 * dy_ + 4 * dz_;
                const long r = dy_ * S + dz_ * S2;
                Dx[o] = v[o + 1] - ld(dxm + r);
                Dx[o + 1] = ld(dxp + r) - v[o];
            }
#pragma unroll
        for (int dz_ = 0; dz_ < 2; ++dz_)
#pragma unroll
            for (int dx_ = 0; dx_ < 2; ++dx_) {
                const int o = dx_ + 4 * dz_;
                const long r = dx_ + dz_ * S2;
                Dy[o] = v[o + 2] - ld(dym + r);
                Dy[o + 2] = ld(dyp + r) - v[o];
            }
#pragma unroll
        for (int dy_ = 0; dy_ < 2; ++dy_)
#pragma unroll
            for (int dx_ = 0; dx_ < 2; ++dx_) {
                const int o = dx_ + 2 * dy_;
                const long r = dx_ + dy_ * S;
                Dz[o] = v[o + 4] - ld(dzm + r);
                Dz[o + 4] = ld(dzp + r) - v[o];
            }
    } else {
        constexpr int QW = kQuadWords<VT>;
        uint32_t xm[QW], xp[QW], ym[2 * QW], yp[2 * QW], zm[2 * QW], zp[2 * QW];
        quad_load1<VT>(base, e + dxm, xm);  // (x-1): comps (y,z) (y,z+1) (y+1,z) (y+1,z+1)
        quad_load1<VT>(base, e + dxp, xp);  // (x+2)
        quad_load2<VT>(base, e + dym, ym);  // (x, y-1), (x+1, y-1): comps 0,1 = y-1
        quad_load2<VT>(base, e + S, yp);    // (x, y+1), (x+1, y+1): comps 2,3 = y+2
        quad_load2<VT>(base, e + dzm, zm);  // (x, y, z-1), (x+1, y, z-1): comps 0,2 = z-1
        quad_load2<VT>(base, e + S2, zp);   // (x, y, z+1), (x+1, y, z+1): comps 1,3 = z+2
#pragma unroll
        for (int dz_ = 0; dz_ < 2; ++dz_)
#pragma unroll
            for (int dy_ = 0; dy_ < 2; ++dy_) {
                const int q = dz_ + 2 * dy_, o = 2 * dy_ + 4 * dz_;
                Dx[o] = v[o + 1] - qc<VT>(xm, q);
                Dx[o + 1] = qc<VT>(xp, q) - v[o];
            }
#pragma unroll
        for (int dz_ = 0; dz_ < 2; ++dz_)
#pragma unroll
            for (int dx_ = 0; dx_ < 2; ++dx_) {
                const int o = dx_ + 4 * dz_;
                Dy[o] = v[o + 2] - qc<VT>(ym + dx_ * QW, dz_);
                Dy[o + 2] = qc<VT>(yp + dx_ * QW, 2 + dz_) - v[o];
            }
#pragma unroll
        for (int dy_ = 0; dy_ < 2; ++dy_)
#pragma unroll
            for (int dx_ = 0; dx_ < 2; ++dx_) {
                const int o = dx_ + 2 * dy_;
                Dz[o] = v[o + 4] - qc<VT>(zm + dx_ * QW, 2 * dy_);
                Dz[o + 4] = qc<VT>(zp + dx_ * QW, 2 * dy_ + 1) - v[o];
            }
    }
    grad_filter<PACKED>(Dx, Dy, Dz, ax, ay, az, gx, gy, gz);
}

#ifndef VR_GRAD_ZPACK
#define VR_GRAD_ZPACK 1  // A/B: 0 = (Dx, Dy)-packed tri8x2 + scalar Dz
#endif
// The difference field's words one shaded sample reads.  f32 (H = false): rows y and y + 1 of
// the cell, elements x and x + 1, 3 x 16 B each.  binary16 (H = true): element e holds per
// axis {D(y,z), D(y,z+1), D(y+1,z), D(y+1,z+1)}, so elements x and x + 1 are 48 contiguous
// bytes: 3 x 16 B.
template <bool H>
struct FieldRowsT {
    f4a a0, a1, a2, b0, b1, b2;
};
template <>
struct FieldRowsT<true> {
    u4a a0, a1, a2;
};
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v h2f(uint32_t w)  // two binary16 -> two f32 (exact)
{
    return __builtin_convertvector(__builtin_bit_cast(h2v, w), f2v);
}
__device__ __forceinline__ void field_rows_load(const char *__restrict__ gbase, size_t e,
                                                FieldRowsT<true> &r)
{
    const char *p = gbase + e * kGradElemBytes;
    r.a0 = *reinterpret_cast<const u4a *>(p);
    r.a1 = *reinterpret_cast<const u4a *>(p + 16);
    r.a2 = *reinterpret_cast<const u4a *>(p + 32);
}
// The f32 path's filter (below) on the converted pairs: per axis a, words 2a / 2a + 1 of
// element x are the y / y + 1 pairs {D(z), D(z+1)}, words 6 + 2a / 7 + 2a those of x + 1.
// VR_FIELD_MIX = 1 (default): the x lerps of the binary16 pairs as v_fma_mix_f32 (binary16
// operands read in place: b * 1 - a, then w * d + a, each rounded once as lerpf's subtraction
// and fma), instead of converting every half first: 12 fewer VALU per shaded sample, C3 +2-3%
// (profiles/r03/field_mix/; bit-identical frames)
#ifndef VR_FIELD_MIX
#define VR_FIELD_MIX 1
#endif
template <bool HI>
__device__ __forceinline__ float mix_lerp(uint32_t a, uint32_t b, float w)
{
    float d, r;
    if constexpr (HI) {
        asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[1,0,1] op_sel_hi:[1,0,1]" : "=v"(d) : "v"(b), "v"(a));
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "=v"(r) : "v"(w), "v"(d), "v"(a));
    } else {
        asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[1,0,1]" : "=v"(d) : "v"(b), "v"(a));
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,0,1]" : "=v"(r) : "v"(w), "v"(d), "v"(a));
    }
    return r;
}
__device__ __forceinline__ void field_rows_filter(const FieldRowsT<true> &r, float ax, float ay,
                                                  float az, float &gx, float &gy, float &gz)
{
    const uint32_t w[12] = {r.a0.x, r.a0.y, r.a0.z, r.a0.w, r.a1.x, r.a1.y,
                            r.a1.z, r.a1.w, r.a2.x, r.a2.y, r.a2.z, r.a2.w};
    auto axis = [&](int a) {
#if VR_FIELD_MIX
        const f2v c0 = {mix_lerp<false>(w[2 * a], w[6 + 2 * a], ax),
                        mix_lerp<true>(w[2 * a], w[6 + 2 * a], ax)};
        const f2v c1 = {mix_lerp<false>(w[2 * a + 1], w[7 + 2 * a], ax),
                        mix_lerp<true>(w[2 * a + 1], w[7 + 2 * a], ax)};
        const f2v q = lerp2(c0, c1, ay);
#else
        const f2v q = lerp2(lerp2(h2f(w[2 * a]), h2f(w[6 + 2 * a]), ax),
                            lerp2(h2f(w[2 * a + 1]), h2f(w[7 + 2 * a]), ax), ay);
#endif
        return lerpf(q.x, q.y, az);
    };
    gx = axis(0);
    gy = axis(1);
    gz = axis(2);
}
__device__ __forceinline__ void field_rows_load(const char *__restrict__ gbase, size_t e,
                                                FieldRowsT<false> &r)
{
    const char *row0 = gbase + e * kGradElemBytes;
    const char *row1 = row0 + (size_t)GeomWide::Row * kGradElemBytes;
    r.a0 = *reinterpret_cast<const f4a *>(row0);       // Dx(x) z,z+1  Dy(x) z,z+1
    r.a1 = *reinterpret_cast<const f4a *>(row0 + 16);  // Dz(x) z,z+1  Dx(x+1) z,z+1
    r.a2 = *reinterpret_cast<const f4a *>(row0 + 32);  // Dy(x+1) ...  Dz(x+1) ...
    r.b0 = *reinterpret_cast<const f4a *>(row1);
    r.b1 = *reinterpret_cast<const f4a *>(row1 + 16);
    r.b2 = *reinterpret_cast<const f4a *>(row1 + 32);
}
// Each axis filtered with its z = 0 / z = 1 halves as packed pairs, which the field's element
// layout already holds adjacent ({D(z), D(z+1)}): lerp2 over x of rows y and y + 1 gives
// {c00, c01} and {c10, c11}, lerp2 over y {c0, c1}, then the z lerp -- tri8's IEEE operations
// per element, without repacking (Dx, Dy) pairs.
__device__ __forceinline__ void field_rows_filter(const FieldRowsT<false> &r, float ax, float ay,
                                                  float az, float &gx, float &gy, float &gz)
{
    auto axis = [&](f2v y0x0, f2v y0x1, f2v y1x0, f2v y1x1) {
        const f2v q = lerp2(lerp2(y0x0, y0x1, ax), lerp2(y1x0, y1x1, ax), ay);
        return lerpf(q.x, q.y, az);
    };
    gx = axis(f2v{r.a0.x, r.a0.y}, f2v{r.a1.z, r.a1.w}, f2v{r.b0.x, r.b0.y}, f2v{r.b1.z, r.b1.w});
    gy = axis(f2v{r.a0.z, r.a0.w}, f2v{r.a2.x, r.a2.y}, f2v{r.b0.z, r.b0.w}, f2v{r.b2.x, r.b2.y});
    gz = axis(f2v{r.a1.x, r.a1.y}, f2v{r.a2.z, r.a2.w}, f2v{r.b1.x, r.b1.y}, f2v{r.b2.z, r.b2.w});
}
// Gradient from the precomputed f32 field: the cell's 8 corners of {Dx, Dy, Dz}, rows y and
// y + 1 of elements x, x + 1 (48 B each: 3 x 16-B loads), filtered as grad_filter.
template <bool PACKED, bool H = false>
__device__ __forceinline__ void grad_field(const char *__restrict__ gbase, size_t e, float ax,
                                           float ay, float az, float &gx, float &gy, float &gz)
{
    if constexpr (H) {
        FieldRowsT<true> r;
        field_rows_load(gbase, e, r);
        field_rows_filter(r, ax, ay, az, gx, gy, gz);
        return;
    }
#if VR_GRAD_ZPACK
    if constexpr (PACKED) {
        FieldRowsT<false> r;
        field_rows_load(gbase, e, r);
        field_rows_filter(r, ax, ay, az, gx, gy, gz);
        return;
    }
#endif
    float Dx[8], Dy[8], Dz[8];
#pragma unroll
    for (int dy_ = 0; dy_ < 2; ++dy_) {
        const char *row = gbase + (e + (size_t)dy_ * GeomWide::Row) * kGradElemBytes;
        const f4a r0 = *reinterpret_cast<const f4a *>(row);       // Dx(x) z,z+1  Dy(x) z,z+1
        const f4a r1 = *reinterpret_cast<const f4a *>(row + 16);  // Dz(x) z,z+1  Dx(x+1) z,z+1
        const f4a r2 = *reinterpret_cast<const f4a *>(row + 32);  // Dy(x+1) ...  Dz(x+1) ...
        const int o = 2 * dy_;  // corner dx + 2 dy + 4 dz
        Dx[o] = r0.x; Dx[o + 4] = r0.y; Dy[o] = r0.z; Dy[o + 4] = r0.w;
        Dz[o] = r1.x; Dz[o + 4] = r1.y; Dx[o + 1] = r1.z; Dx[o + 5] = r1.w;
        Dy[o + 1] = r2.x; Dy[o + 5] = r2.y; Dz[o + 1] = r2.z; Dz[o + 5] = r2.w;
    }
    grad_filter<PACKED>(Dx, Dy, Dz, ax, ay, az, gx, gy, gz);
}

// Steps k in [1, K] of a ray whose positions provably stay strictly inside (0, 1)^3, where the
// reference's bounds test (volume.frag:34-37) never breaks and, with the default slicing, the
// strict slab test (:39-40) always passes: the loop skips both there.  p_k is p_0 plus k float
// additions of s = fl(d * step); while |p| < 1 each addition rounds by at most 2^-25, so with
// delta = 2^-24 per step, p_k lies within p_0 + k s +- k delta.  Each bound is linear in k:
// f(k) = A + B k > 0 holds on [1, K] iff it holds at both ends.
__device__ __forceinline__ int interior_steps(const float *p, const float *d, float step,
                                              int nsteps)
{
    constexpr double delta = 0x1p-24;
    double K = (double)(nsteps - 1);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double s = (double)(d[a] * step), q = (double)p[a];
        const double A[2] = {q, 1.0 - q}, B[2] = {s - delta, -(s + delta)};
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if (!(A[c] + B[c] > 0.0)) return 0;
            if (B[c] < 0.0) K = fmin(K, floor(A[c] / -B[c]) - 1.0);
        }
    }
    return K > 0.0 ? (int)K : 0;
}

__device__ __forceinline__ void texel_coord(float p, float n, int &i, float &a)
{
    const float u = p * n - 0.5f;
    const float f = floorf(u);
    a = u - f;
    i = (int)f;
}

// Pixel-centre ray -> cube entry (front face inside the clip volume), as the oracle's
// pixel_ray: unproject ndc z = 0 and z = 1 through inverse(proj*view) in double.
__device__ __forceinline__ bool pixel_ray(const MarchParams &P, uint32_t px, uint32_t py,
                                          float tex[3], float dir[3])
{
    const double *m = P.inv;
    const double x = ((double)px + 0.5) / P.fw * 2.0 - 1.0;
    const double y = ((double)py + 0.5) / P.fh * 2.0 - 1.0;
    double h0[4], h1[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        h0[r] = m[0 * 4 + r] * x + m[1 * 4 + r] * y + m[3 * 4 + r];
        h1[r] = h0[r] + m[2 * 4 + r];
    }
    double p0[3], d[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        p0[r] = h0[r] / h0[3];
        d[r] = h1[r] / h1[3] - p0[r];
    }
    double te = -__builtin_inf(), tx = __builtin_inf();
    int axis = 0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        double lo, hi;
        if (d[a] == 0.0) {
            if (p0[a] < -0.5 || p0[a] > 0.5) return false;
            lo = -__builtin_inf();
            hi = __builtin_inf();
        } else {
            const double t1 = (-0.5 - p0[a]) / d[a];
            const double t2 = (0.5 - p0[a]) / d[a];
            lo = t1 < t2 ? t1 : t2;
            hi = t1 < t2 ? t2 : t1;
        }
        if (lo > te) {
            te = lo;
            axis = a;
        }
        if (hi < tx) tx = hi;
    }
    if (!(te < tx) || te < 0.0 || te > 1.0) return false;
    float frag[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double e = p0[a] + te * d[a];
        frag[a] = (float)e;
        tex[a] = (float)(e + 0.5);
    }
    // the entry face's coordinate is constant over the face (volume.vert:20, cube :55-90)
    frag[axis] = d[axis] > 0.0 ? -0.5f : 0.5f;
    tex[axis] = d[axis] > 0.0 ? 0.0f : 1.0f;
    // volume.frag:23
    const float vx = frag[0] - P.cam[0];
    const float vy = frag[1] - P.cam[1];
    const float vz = frag[2] - P.cam[2];
    const float len = sqrtf(vx * vx + vy * vy + vz * vz);
    dir[0] = vx / len;
    dir[1] = vy / len;
    dir[2] = vz / len;
    return true;
}

// (x / range) correctly rounded.  P.div_fast (host: 2^-40 <= range < 2^100, |min|, |max| <
// 2^100): q = x * RN(1/range), then one fma residual correction.  Markstein's theorem gives
// the IEEE quotient when the residual is exact (|x| >= 2^-100 here); checked against x86
// IEEE division on 3.8e9 (x, range) pairs of that domain, 0 mismatches.  Smaller |x| give
// |t| < 2^-60, where t * n - 0.5 rounds to -0.5 whatever t's last bit: the frame is the
// same.  Otherwise the full IEEE division sequence.
__device__ __forceinline__ float div_by_range(float x, const MarchParams &P)
{
    if (P.div_fast) {
        const float q = x * P.inv_range;
        const float e = fmaf(-q, P.range, x);
        return fmaf(e, P.inv_range, q);
    }
    return x / P.range;
}

// 1D TF, linear filter, clamp-to-edge (offscreen_pass.cpp:1125-1150).  lut holds n + 2
// entries {c, d} (float4 pairs): entry i + 1 is texel i as {c_i, c_(i+1) - c_i} (difference 0
// for the last texel, computed on the host with the same IEEE subtraction), entry 0 = {c_0, 0}
// and entry n + 1 = {c_(n-1), 0} are the clamp-to-edge sentinels.  With u clamped to [-1, n],
// floor(u) = i0 lies in [-1, n] and lerp(c_i0, c_i1, w) = fma(w, d, c) is one fma per channel
// with no index clamp: below the first texel centre (i0 = -1) and at u = n the sentinel's
// difference 0 returns the edge texel for any w.  NaN t clamps to u = -1 (texel 0).
// The LUT is read through an LDS-typed pointer (LdsF4) when staged, a global one otherwise:
// never through a generic pointer chosen between the two.  (With one generic pointer the
// compiler merged both lookups into FLAT loads and folded the +1 texel offset into the
// instruction offset; for u < 0 (texel -1, the low sentinel) the base then sat 32 B below the
// LDS aperture, the access was routed as a global one to the aperture's base address, and the
// launch faulted with MEMORY_APERTURE_VIOLATION.)
typedef float F4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const F4v LdsF4;
template <typename Lut>
__device__ __forceinline__ float4 tf_lookup(Lut *lut, int n, float nf, float t)
{
    (void)n;
    float u = t * nf - 0.5f;
    u = fminf(fmaxf(u, -1.0f), nf);
    const float f = floorf(u);
    const float w = u - f;
    int e = (int)f + 1;
    if (VR_OOB(1, (unsigned long long)(long long)e, (unsigned long long)(n + 2))) e = 0;
    const auto a = lut[2 * e], d = lut[2 * e + 1];
    return make_float4(fmaf(w, d.x, a.x), fmaf(w, d.y, a.y), fmaf(w, d.z, a.z),
                       fmaf(w, d.w, a.w));
}

__device__ __forceinline__ uint32_t unorm8(float x)
{
    const float v = fminf(fmaxf(x, 0.0f), 1.0f);
    return (uint32_t)(v * 255.0f + 0.5f);
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// skip_empty: longest leap in steps (bounds the float drift the leap margin must cover)
constexpr int kMaxLeap = 256;

// Minimum of k in [0, kMaxLeap] over the ACTIVE lanes (binary search on ballots: a ballot
// sees only active lanes, where a DPP reduction would read stale values of inactive ones).
__device__ __forceinline__ int wave_min_leap(int k)
{
    int lo = 0, hi = kMaxLeap;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (__ballot(k <= mid) != 0ull)
            hi = mid;
        else
            lo = mid + 1;
    }
    return lo;
}

#ifdef VR_WG_TIMES
// Experiment builds: per workgroup of the march launches since the last reset, 4 words: start
// and end wall clock (100 MHz), the tile id, and (XCC_ID << 32 | HW_ID) from the hardware
// registers (which XCD / SE / CU ran it); read by vr_debug_wg_times (tools/wg_timeline.py).
constexpr uint32_t kWgTimesMax = 1u << 17;
__device__ unsigned long long g_wg_times[4 * kWgTimesMax];
__device__ unsigned int g_wg_count;
__device__ __forceinline__ void wg_times_record(unsigned long long t0, uint32_t tile)
{
    const unsigned int slot = atomicAdd(&g_wg_count, 1u);
    if (slot < kWgTimesMax) {
        const unsigned long long hw = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
        const unsigned long long xcc = (unsigned)__builtin_amdgcn_s_getreg((3 << 11) | 20);
        g_wg_times[4 * slot] = t0;
        g_wg_times[4 * slot + 1] = (unsigned long long)wall_clock64();
        g_wg_times[4 * slot + 2] = ((unsigned long long)blockIdx.x << 32) | tile;
        g_wg_times[4 * slot + 3] = (xcc << 32) | hw;
    }
}
#endif

// Occupancy floor (waves per SIMD): the shaded f32 kernel holds 2 x 16-B centre loads plus
// 10 gradient loads in flight and would take 102 VGPRs (4 waves) unconstrained; 6 waves
// measured best (A/B: 0.79 vs 0.91 ms for C3).  The skip-empty kernel (scalar gradient) is
// left unconstrained (96 VGPRs, 5 waves: a floor of 5 yields the same occupancy but measured
// 12% slower), the counting kernels (not timed) get 4: no spills.
#ifndef VR_MARCH_MIN_WAVES
#define VR_MARCH_MIN_WAVES 6
#endif
#ifndef VR_SKIP_MIN_WAVES
#define VR_SKIP_MIN_WAVES 1
#endif
#ifndef VR_DEFER_SHADE
#define VR_DEFER_SHADE 1  // pipelined + difference field: shade a sample one sample later
#endif
#ifndef VR_PIPE_MIN_WAVES
#define VR_PIPE_MIN_WAVES 1
#endif
// The pipelined shaded kernel with the difference field (the C3 headline kernel).  Round 2,
// without deferred shading: 6 waves (78 VGPRs, no spills) against 5 unconstrained (84): C3
// +1.1% (profiles/r02/pipeline/min_waves6_*).  Deferred shading holds 24 more VGPRs of field
// rows: 94 VGPRs at 5 waves (at 6 it spills); C3 +1.2% against the round-2 kernel, shaded
// fill/oblique/top views 1-2% faster (profiles/r03/deferred_shading/).
#ifndef VR_PIPE_GF_MIN_WAVES
#define VR_PIPE_GF_MIN_WAVES (VR_DEFER_SHADE ? 5 : 6)
#endif
template <bool COUNT, bool SKIP, bool GF, bool PIPE>
constexpr int kMarchMinWaves =
    PIPE ? (GF ? VR_PIPE_GF_MIN_WAVES : VR_PIPE_MIN_WAVES)
         : (GF ? 1 : (COUNT ? 4 : (SKIP ? VR_SKIP_MIN_WAVES : VR_MARCH_MIN_WAVES)));

#ifndef VR_SKIP_PACKED_GRADIENT
#define VR_SKIP_PACKED_GRADIENT 0
#endif
template <bool SKIP>
constexpr bool kPackedGradient = !SKIP || VR_SKIP_PACKED_GRADIENT;

// GF: shaded f32 with the precomputed difference field (P.grad); without it the kernel forms
// the differences from the stencil (60 vs 80 VGPRs: 8 vs 6 waves per SIMD).
// Block -> tile.  Workgroups b and b+8 run on the same XCD (round-robin dispatch; speed
// only, never correctness).  Orders: 1 raster; 2 each XCD a contiguous band of tiles
// (bijective remap); 3 each XCD every 8th 4x4-tile super-tile in raster order, its tiles
// consecutive on that XCD: L2 locality inside a super-tile, every XCD sampling the whole
// frame (load balance when the volume covers part of it).  false: no tile (grid padding).
__device__ __forceinline__ bool block_tile(const MarchParams &P, uint32_t &tile_x,
                                           uint32_t &tile_y)
{
    const uint32_t nwg = gridDim.x, b = blockIdx.x;
    if (P.tile_perm) {  // adaptive order (launch_order_tiles)
        if (VR_OOB(5, b, P.nperm)) return false;
        const uint32_t t = P.tile_perm[b];
        if (t != 0xFFFFFFFFu && VR_OOB(6, t, P.tiles_x * P.tiles_y)) return false;
        tile_x = t % P.tiles_x;
        tile_y = t / P.tiles_x;
        return t != 0xFFFFFFFFu;
    }
    if (P.tile_order >= 3) {  // 3, and 4 before its first permutation
        const uint32_t k = b >> 3, w = k & (kSuper * kSuper - 1);
        const uint32_t s = (b & 7u) + 8u * (k >> (2 * kSuperShift));
        tile_x = (s % P.supers_x) * kSuper + (w & (kSuper - 1));
        tile_y = (s / P.supers_x) * kSuper + (w >> kSuperShift);
        return s < P.supers_total && tile_x < P.tiles_x && tile_y < P.tiles_y;
    }
    if (P.tile_order == 2) {
        const uint32_t xcd = b & 7u, q = nwg >> 3, r = nwg & 7u;
        const uint32_t t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
        tile_x = t % P.tiles_x;
        tile_y = t / P.tiles_x;
        return true;
    }
    tile_x = b % P.tiles_x;
    tile_y = b / P.tiles_x;
    return true;
}

// Headlight Phong of one sample from its filtered central differences (gx, gy, gz): gradient
// scaled to normalised coordinates, ndl = |n . dir|, rgb' = rgb (ka + kd ndl) + ks ndl^p; a
// zero gradient leaves the colour unshaded.  The oracle's march_pixel, same operation order.
__device__ __forceinline__ void phong(const MarchParams &P, float gx, float gy_, float gz,
                                      float d0, float d1, float d2, float4 &s)
{
    const float wx = gx * P.fnx, wy = gy_ * P.fny, wz = gz * P.fnz;
    const float g2 = wx * wx + wy * wy + wz * wz;
    if (g2 > 0.0f) {
        const float inv = inv_sqrt_ieee(g2);  // 1.0f / sqrtf(g2), vr_exact_math.h
        const float ndl = fabsf((wx * d0 + wy * d1 + wz * d2) * inv);
        const float kdiff = P.ka + P.kd * ndl;
        // ndl^p by binary exponentiation (the oracle's powi): p uniform.  The default p = 16
        // unrolled: powi squares four times and multiplies 1 by the result (exact), so
        // ((ndl^2)^2)^2)^2 is its value bit for bit, without the loop's scalar branches.
        float sp = 1.0f, b = ndl;
        if (P.spec_power == 16) {
            b = b * b;
            b = b * b;
            b = b * b;
            sp = b * b;
        } else {
            for (int e = P.spec_power; e;) {
                if (e & 1) sp = sp * b;
                e >>= 1;
                if (e) b = b * b;
            }
        }
        const float spec = P.ks * sp;
        s.x = s.x * kdiff + spec;
        s.y = s.y * kdiff + spec;
        s.z = s.z * kdiff + spec;
    }
}

// Gradient Phong extension for one sample with alpha > 0 (s: TF colour in/out): gradient from
// the difference field (GF) or the stencil, scaled to normalised coordinates, headlight
// ndl = |n . dir|, rgb' = rgb (ka + kd ndl) + ks ndl^p.  The oracle's march_pixel, same order.
template <typename VT, bool GF, bool PACKED>
__device__ __forceinline__ void shade_sample(const MarchParams &P, const char *__restrict__ vol,
                                             size_t ce, const Cell8<VT> &c, int pi, int pj,
                                             int pk, long by_stride, long bz_stride, float ax,
                                             float ay, float az, float d0, float d1, float d2,
                                             float4 &s)
{
    float gx, gy_, gz;
    if constexpr (GF) {  // f32: precomputed difference field
        grad_field<PACKED, kHalfField<VT>>(reinterpret_cast<const char *>(P.grad), ce, ax, ay, az,
                                           gx, gy_, gz);
    } else {
        gradient<VT, PACKED>(vol, ce, c, pi, pj, pk, P.nbx, P.nby, by_stride, bz_stride, ax, ay,
                             az, gx, gy_, gz);
    }
    phong(P, gx, gy_, gz, d0, d1, d2, s);
}

// PIPE: the loads of sample k + 1 are issued before sample k is filtered, shaded and
// composited (two samples of the ray in flight).  For launches with few waves per CU (one
// rank's share of a multi-GPU frame), where every wave's serial chain of memory round trips,
// not the chip's throughput, sets the time.  Reference-semantics results are identical.
// One wavefront's strip of a tile (wave index `wave` of the 16 x kMarchRows tile (tile_x,
// tile_y)): every ray of it marched and its pixels written.  s_tf: the TF staged in LDS (when
// tf_in_lds).  march_kernel runs one tile per workgroup.
template <typename VT, bool SHADE, bool COUNT, bool SKIP, bool GF, bool PIPE>
__device__ __forceinline__ void march_strip(const MarchParams &P, LdsF4 *s_tf,
                                            bool tf_in_lds, uint32_t tile_x, uint32_t tile_y,
                                            uint32_t wave, uint32_t lane)
{
    using G = GeomOf<VT>;
    const long by_stride = (long)P.nbx * G::Elems;  // elements between brick rows/slabs
    const long bz_stride = (long)P.nbx * P.nby * G::Elems;

    // wavefront -> (ww x wh) pixels, ww = 2^wave_w_shift, together tiling the 16 x kMarchRows tile
    const uint32_t ws = P.wave_w_shift, ww = 1u << ws, wh = 64u >> ws;
    const uint32_t wpr = kTile >> ws;  // wavefronts per tile row
    const uint32_t lx_ = lane & (ww - 1), ly_ = lane >> ws;
    const uint32_t px = tile_x * kTile + (wave % wpr) * ww + lx_;
    const uint32_t ly = tile_y * kMarchRows + (wave / wpr) * wh + ly_;
    bool active = px < P.W && ly < P.local_rows;
    const uint32_t blk = ly / P.row_block;
    const uint32_t gy = share_global_block(blk, P.rank, P.nranks, RowShare{P.share_w0, P.share_w}) *
                            P.row_block + (ly - blk * P.row_block);
    active = active && gy < P.H;

    float tex[3] = {0.f, 0.f, 0.f}, dir[3] = {0.f, 0.f, 0.f};
    const bool covered = active && pixel_ray(P, px, gy, tex, dir);

    float T = 1.0f, cr = 0.0f, cg = 0.0f, cb = 0.0f;
    unsigned long long n_samples = 0, n_shaded = 0, n_steps = 0, n_skipped = 0;
    uint32_t cur_brick = 0xFFFFFFFFu, cur_dist = 0;
    const char *__restrict__ vol = static_cast<const char *>(P.vol);
    const int nsteps = covered ? P.nsteps : 0;
    float p0 = tex[0], p1 = tex[1], p2 = tex[2];
    const float d0 = dir[0], d1 = dir[1], d2 = dir[2];
    // steps 1..kin need neither the bounds nor (default slicing) the slab test
    const int kin = (covered && P.slab_default) ? interior_steps(tex, dir, P.step, nsteps) : 0;
    // skip_empty leap constants: steps per cell along each axis, and a margin (cells) covering
    // the leap's float-accumulation drift (<= kMaxLeap half-ulps of p < 2, times N) + rounding
    float inv_du[3] = {0.f, 0.f, 0.f}, leap_margin[3] = {0.f, 0.f, 0.f};
    if (!COUNT && SKIP) {
        const float dd[3] = {d0, d1, d2}, fn[3] = {P.fnx, P.fny, P.fnz};
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            inv_du[a] = 1.0f / (fabsf(dd[a]) * P.step * fn[a]);
            leap_margin[a] = 0.5f + (float)kMaxLeap * 1.2e-7f * fn[a];
        }
    }
    if constexpr (PIPE) {
        // Positions, predicates and operations exactly as the loop below.  Loads are
        // unconditional (a cell of the first brick off-slab) and alpha is 0 off-slab, which
        // composites +0 and leaves T: no load sits under a data-dependent branch, so the
        // compiler waits with counted vmcnt(N) and the next sample's loads stay in flight.
        // The TF is LDS-resident (host guarantees tf_n <= kTfLds for PIPE).
        struct Stage {
            CellRaw<VT> w;  // loaded words, decoded at consume
            size_t ce;
            float ax, ay, az;
            int pi, pj, pk;
            bool ok, slab;
        };
        // live = false: a lane whose ray has ended; its stage is not ok and loads the first
        // brick's first cell (one cached line per wave), so the wave's loads stay unconditional
        auto prep = [&](Stage &S, int k, bool live = true) {
            const bool interior = (unsigned)(k - 1) < (unsigned)kin;
            S.ok = live && k < nsteps &&
                   (interior || !(p0 > 1.0f || p1 > 1.0f || p2 > 1.0f || p0 < 0.0f ||
                                  p1 < 0.0f || p2 < 0.0f));
            S.slab = S.ok && (interior || (p0 < P.smax[0] && p1 < P.smax[1] && p2 < P.smax[2] &&
                                           p0 > P.smin[0] && p1 > P.smin[1] && p2 > P.smin[2]));
            int i, j, kk;
            texel_coord(p0, P.fnx, i, S.ax);
            texel_coord(p1, P.fny, j, S.ay);
            texel_coord(p2, P.fnz, kk, S.az);
            if (!S.slab) i = j = kk = 0;
            S.pi = i + kPad;
            S.pj = j + kPad;
            S.pk = kk + kPad;
            S.ce = cell_offset<VT>(S.pi, S.pj, S.pk, P.nbx, P.nby);
            if (VR_OOB(3, S.ce * kElemBytes<VT>, P.vol_bytes)) S.ce = 0;
            Cell8<VT>::issue(S.w, vol, S.ce);
        };
        auto composite = [&](const float4 &sm) -> bool {  // volume.frag:44-45
            cr = cr + (sm.x * sm.w) * T;
            cg = cg + (sm.y * sm.w) * T;
            cb = cb + (sm.z * sm.w) * T;
            T = T * (1.0f - sm.w);
            return T == 0.0f || T < P.ert_eps;
        };
        // Deferred shading (shaded frames with the difference field): a sample with alpha > 0
        // issues its 6 field loads and is shaded and composited one sample later, when the next
        // sample is consumed (its loads landed under the same wait as that sample's density
        // loads, with the sample after it in flight).  Composites keep the sample order, an
        // alpha-0 sample composites exactly nothing (C += (rgb 0) T = +0, T *= 1) and is not
        // held back, and the ray still ends at the first T == 0 / T < eps: the same bits.
        constexpr bool kDefer = VR_DEFER_SHADE && SHADE && GF;
        struct Pend {
            FieldRowsT<kHalfField<VT>> g;
            float4 sm;
            float ax, ay, az;
            bool on;
        } X;
        X.on = false;
        auto finish = [&]() -> bool {  // shade + composite the held sample; true: the ray ends
            if (!kDefer || !X.on) return false;
            X.on = false;
            float gx, gy_, gz;
            field_rows_filter(X.g, X.ax, X.ay, X.az, gx, gy_, gz);
            phong(P, gx, gy_, gz, d0, d1, d2, X.sm);
            return composite(X.sm);
        };
        auto consume_cell = [&](const Stage &S, const Cell8<VT> &c) -> bool {  // true: the ray ends
            if (kDefer && finish()) return true;
            const float d = c.tri(S.ax, S.ay, S.az);
            const float tt = div_by_range(d - P.vmin, P);
            float4 sm = tf_lookup(s_tf, P.tf_n, P.tf_nf, tt);
            if (!S.slab) sm.w = 0.0f;
            if constexpr (kDefer) {
                if (sm.w > 0.0f) {
                    field_rows_load(reinterpret_cast<const char *>(P.grad), S.ce, X.g);
                    X.sm = sm;
                    X.ax = S.ax;
                    X.ay = S.ay;
                    X.az = S.az;
                    X.on = true;
                }
                return false;
            }
            if (SHADE && sm.w > 0.0f)
                shade_sample<VT, GF, true>(P, vol, S.ce, c, S.pi, S.pj, S.pk, by_stride,
                                           bz_stride, S.ax, S.ay, S.az, d0, d1, d2, sm);
            return composite(sm);
        };
        auto consume = [&](const Stage &S) -> bool {
            Cell8<VT> c;
            c.decode(S.w);
            return consume_cell(S, c);
        };
        auto advance = [&]() {
            p0 = p0 + d0 * P.step;
            p1 = p1 + d1 * P.step;
            p2 = p2 + d2 * P.step;
        };
        Stage A, B;
        int k = 0;
        {
            prep(A, k);
            while (A.ok) {  // ping-pong: no register copies between the two stages
                advance();
                prep(B, ++k);
                if (consume(A) || !B.ok) break;
                advance();
                prep(A, ++k);
                if (consume(B)) break;
            }
        }
        finish();  // deferred shading: the sample still held when the ray left the volume
    } else
    for (int it = 0; it < nsteps; ++it) {
        const bool interior = (unsigned)(it - 1) < (unsigned)kin;  // it in [1, kin]
        // volume.frag:34-37
        if (!interior &&
            (p0 > 1.0f || p1 > 1.0f || p2 > 1.0f || p0 < 0.0f || p1 < 0.0f || p2 < 0.0f))
            break;
        if (COUNT) ++n_steps;
        // volume.frag:39-40 (strict)
        if (interior || (p0 < P.smax[0] && p1 < P.smax[1] && p2 < P.smax[2] && p0 > P.smin[0] &&
                         p1 > P.smin[1] && p2 > P.smin[2])) {
            int i, j, k;
            float ax, ay, az;
            texel_coord(p0, P.fnx, i, ax);
            texel_coord(p1, P.fny, j, ay);
            texel_coord(p2, P.fnz, k, az);
            const int pi = i + kPad, pj = j + kPad, pk = k + kPad;
            uint32_t dist = 0;
            if (SKIP) {
                // skip_empty: distance (in bricks) from the cell's brick to the nearest brick
                // that can produce a visible sample (classify_kernel); cached per brick
                const uint32_t bb = ((uint32_t)pk / G::BZ * P.nby + (uint32_t)pj / G::BY) * P.nbx +
                                    (uint32_t)pi / G::BX;
                if (bb != cur_brick) {
                    cur_brick = bb;
                    cur_dist = P.skip_dist[bb];
                }
                dist = cur_dist;
            }
            // the wavefront leaps only when every lane sampling here is in empty space, and
            // by the smallest safe leap of its lanes: lanes stay in lock-step (a lane-private
            // leap desynchronises the wave and multiplies its fetch instructions)
            const bool wave_empty = SKIP && !COUNT && __all(dist != 0);
            if (dist != 0) {
                if (COUNT) {
                    ++n_skipped;  // the counting kernel walks every step (exact counters)
                } else if (wave_empty) {
                    // Leap: every brick within Chebyshev radius dist - 1 of this one is empty.
                    // Take the steps whose cells provably stay inside that box (cell
                    // coordinate u = p N - 0.5, brick of u: (floor(u) + 2) >> 3), advancing p
                    // with the same float additions as the reference loop, so the first
                    // non-empty sample is reached at the bit-identical position.
                    float kf = (float)min(nsteps - 1 - it, kMaxLeap);
                    const int bi[3] = {pi / G::BX, pj / G::BY, pk / G::BZ};
                    const float pp[3] = {p0, p1, p2}, dd[3] = {d0, d1, d2};
                    const float fn[3] = {P.fnx, P.fny, P.fnz};
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
                        const float u = pp[a] * fn[a] - 0.5f;
                        const int bc = G::cells(a);
                        const float reach = (float)((int)(dist - 1) * bc);
                        const float room = dd[a] > 0.0f
                                               ? (float)((bi[a] + 1) * bc - kPad) + reach - u
                                               : u - (float)(bi[a] * bc - kPad) + reach;
                        // NaN (axis not moving) is ignored by fminf
                        kf = fminf(kf, (room - leap_margin[a]) * inv_du[a]);
                    }
                    const int k = wave_min_leap(kf >= 1.0f ? (int)kf : 0);
                    for (int j = 0; j < k; ++j) {
                        p0 = p0 + d0 * P.step;
                        p1 = p1 + d1 * P.step;
                        p2 = p2 + d2 * P.step;
                    }
                    it += k;
                }
            } else {
                size_t ce = cell_offset<VT>(pi, pj, pk, P.nbx, P.nby);
                if (VR_OOB(2, ce * kElemBytes<VT>, P.vol_bytes)) ce = 0;
                Cell8<VT> c;
                c.load(vol, ce);
                const float d = c.tri(ax, ay, az);
                // volume.frag:42 (d - min) / (max - min), correctly rounded; for a normal
                // range the reciprocal + one fma correction gives the IEEE quotient (see
                // div_by_range)
                const float tt = div_by_range(d - P.vmin, P);
                float4 s = tf_in_lds ? tf_lookup(s_tf, P.tf_n, P.tf_nf, tt)
                                     : tf_lookup(P.tf, P.tf_n, P.tf_nf, tt);
                if (COUNT) ++n_samples;
                if (SHADE && s.w > 0.0f) {
                    shade_sample<VT, GF, kPackedGradient<SKIP>>(P, vol, ce, c, pi, pj, pk, by_stride,
                                                                bz_stride, ax, ay, az, d0, d1, d2, s);
                    if (COUNT) ++n_shaded;
                }
                // volume.frag:44-45
                cr = cr + (s.x * s.w) * T;
                cg = cg + (s.y * s.w) * T;
                cb = cb + (s.z * s.w) * T;
                T = T * (1.0f - s.w);
                if (T == 0.0f) break;
                if (T < P.ert_eps) break;
            }
        }
        // volume.frag:47
        p0 = p0 + d0 * P.step;
        p1 = p1 + d1 * P.step;
        p2 = p2 + d2 * P.step;
    }

    if (COUNT) {
        const unsigned long long rays = wave_sum(covered ? 1ull : 0ull);
        const unsigned long long sm = wave_sum(n_samples);
        const unsigned long long sh = wave_sum(n_shaded);
        const unsigned long long st = wave_sum(n_steps);
        const unsigned long long sk = wave_sum(n_skipped);
        if (lane == 0) {
            atomicAdd(&P.counters[0], rays);
            atomicAdd(&P.counters[1], sm);
            atomicAdd(&P.counters[2], sh);
            atomicAdd(&P.counters[3], st);
            atomicAdd(&P.counters[4], sk);
        }
    }
    if (!active) return;

    // volume.frag:50 + blend (offscreen_pass.cpp:715-725); uncovered: T = 1, C = 0 -> clear
    const float A = 1.0f - T;
    const float omA = 1.0f - A;
    const float o0 = cr * A + P.clear[0] * omA;
    const float o1 = cg * A + P.clear[1] * omA;
    const float o2 = cb * A + P.clear[2] * omA;
    const float o3 = A * A + P.clear[3] * omA;
    const size_t idx = (size_t)ly * P.W + px;
    if (VR_OOB(4, idx * (P.out_format == 0 ? 4 : 16), P.out_bytes)) return;
    if (P.out_format == 0) {
        static_cast<uint32_t *>(P.out)[idx] =
            unorm8(o0) | (unorm8(o1) << 8) | (unorm8(o2) << 16) | (unorm8(o3) << 24);
    } else {
        static_cast<float4 *>(P.out)[idx] = make_float4(o0, o1, o2, o3);
    }
}

template <typename VT, bool SHADE, bool COUNT, bool SKIP, bool GF, bool PIPE>
__global__ __launch_bounds__(kThreadsPerTile, (kMarchMinWaves<COUNT, SKIP, GF, PIPE>)) void march_kernel(const MarchParams P)
{
    __shared__ float4 s_tf[kTfLut];  // {texel, difference to the next} pairs + sentinels
    const int tid = threadIdx.x;

    uint32_t tile_x, tile_y;
    if (!block_tile(P, tile_x, tile_y)) return;
    const long long wg_start = wall_clock64();

    const bool tf_in_lds = P.tf_n <= kTfLds;
    if (tf_in_lds)
        for (int i = tid; i < 2 * (P.tf_n + 2); i += (int)kThreadsPerTile) s_tf[i] = P.tf[i];
    __syncthreads();
    march_strip<VT, SHADE, COUNT, SKIP, GF, PIPE>(P, (LdsF4 *)s_tf, tf_in_lds, tile_x, tile_y,
                                                  (uint32_t)tid >> 6, (uint32_t)tid & 63u);
    if (P.tile_cost) {  // adaptive order: this tile's duration for the next launch
        __syncthreads();
        if (tid == 0)
            P.tile_cost[tile_y * P.tiles_x + tile_x] =
                (uint32_t)min(wall_clock64() - wg_start, 0x7FFFFFFFLL);
    }
#ifdef VR_WG_TIMES
    __syncthreads();
    if (tid == 0) wg_times_record((unsigned long long)wg_start, tile_y * P.tiles_x + tile_x);
#endif
}

// ---- lane-pair march (small launches) ----------------------------------------------------------
// Two lanes per ray: lane 0 of the pair fetches, filters and shades the even samples, lane 1 the
// odd ones; both keep the ray position with the same float additions (p_(k+1) = p_k + d step,
// every step), exchange their sample through a lane shuffle, and composite the pair in sample
// order with identical operations, so C and T are the single-lane march's bit for bit (an
// off-slab sample composites alpha 0: +0, T unchanged).  Halves each ray's serial chain and
// doubles the wavefronts of a launch: for a rank's share of a multi-GPU frame.  A workgroup is
// a 16x8-pixel tile (wavefront: 16x2 pixels); the TF is LDS-resident (host: tf_n <= kTfLds).
template <typename VT, bool SHADE, bool GF, int L>
__global__ __launch_bounds__(kThreads) void march_pair_kernel(const MarchParams P)
{
    __shared__ float4 s_tf[kTfLut];
    const int tid = threadIdx.x;
    uint32_t tile_x, tile_y;
    if (!block_tile(P, tile_x, tile_y)) return;
    for (int i = tid; i < 2 * (P.tf_n + 2); i += kThreads) s_tf[i] = P.tf[i];
    __syncthreads();
    const long long wg_start = wall_clock64();
#ifdef VR_WG_TIMES
    const unsigned long long wg_t0 = wg_start;
#endif
    using G = GeomOf<VT>;
    const long by_stride = (long)P.nbx * G::Elems;
    const long bz_stride = (long)P.nbx * P.nby * G::Elems;

    // L lanes per ray; wavefront = 16 x (4 / L) pixels; workgroup tile 16 x (16 / L)
    const uint32_t wave = tid >> 6, lane = tid & 63, q = lane / L, half = lane % L;
    const uint32_t px = tile_x * kTile + (q & 15);
    const uint32_t ly = tile_y * (kTile / L) + wave * (4 / L) + (q >> 4);
    bool active = px < P.W && ly < P.local_rows;
    const uint32_t blk = ly / P.row_block;
    const uint32_t gy = share_global_block(blk, P.rank, P.nranks, RowShare{P.share_w0, P.share_w}) *
                            P.row_block + (ly - blk * P.row_block);
    active = active && gy < P.H;

    float tex[3] = {0.f, 0.f, 0.f}, dir[3] = {0.f, 0.f, 0.f};
    const bool covered = active && pixel_ray(P, px, gy, tex, dir);
    const char *__restrict__ vol = static_cast<const char *>(P.vol);
    const int nsteps = covered ? P.nsteps : 0;
    float p0 = tex[0], p1 = tex[1], p2 = tex[2];
    const float d0 = dir[0], d1 = dir[1], d2 = dir[2];
    const int kin = (covered && P.slab_default) ? interior_steps(tex, dir, P.step, nsteps) : 0;
    auto advance = [&]() {
        p0 = p0 + d0 * P.step;
        p1 = p1 + d1 * P.step;
        p2 = p2 + d2 * P.step;
    };
    float T = 1.0f, cr = 0.0f, cg = 0.0f, cb = 0.0f;
    // Each lane also runs its own samples software-pipelined (its next sample's loads in
    // flight while the current one is filtered): unconditional loads (a first-brick cell
    // off-slab, alpha 0 there), ping-pong stages, as march_kernel's PIPE path.
    struct Stage {
        Cell8<VT> c;
        size_t ce;
        float ax, ay, az;
        int pi, pj, pk;
        bool ok, slab;
    };
    auto prep = [&](Stage &S, int k) {
        const bool interior = (unsigned)(k - 1) < (unsigned)kin;
        S.ok = k < nsteps && (interior || !(p0 > 1.0f || p1 > 1.0f || p2 > 1.0f || p0 < 0.0f ||
                                            p1 < 0.0f || p2 < 0.0f));
        S.slab = S.ok && (interior || (p0 < P.smax[0] && p1 < P.smax[1] && p2 < P.smax[2] &&
                                       p0 > P.smin[0] && p1 > P.smin[1] && p2 > P.smin[2]));
        int i, j, kk;
        texel_coord(p0, P.fnx, i, S.ax);
        texel_coord(p1, P.fny, j, S.ay);
        texel_coord(p2, P.fnz, kk, S.az);
        if (!S.slab) i = j = kk = 0;
        S.pi = i + kPad;
        S.pj = j + kPad;
        S.pk = kk + kPad;
        S.ce = cell_offset<VT>(S.pi, S.pj, S.pk, P.nbx, P.nby);
        S.c.load(vol, S.ce);
    };
    // this lane's sample -> exchange -> the pair's two samples composited in order; true: the
    // ray ends (bounds, nsteps, T == 0 or ERT), identically in both lanes
    auto consume = [&](const Stage &S) -> bool {
        float4 sm = tf_lookup((LdsF4 *)s_tf, P.tf_n, P.tf_nf,
                              div_by_range(S.c.tri(S.ax, S.ay, S.az) - P.vmin, P));
        if (!S.slab) sm.w = 0.0f;
        if (SHADE && sm.w > 0.0f)
            shade_sample<VT, GF, true>(P, vol, S.ce, S.c, S.pi, S.pj, S.pk, by_stride, bz_stride,
                                       S.ax, S.ay, S.az, d0, d1, d2, sm);
        // the group's L samples, in sample order (lane j of the group holds sample k0 + j)
        const int base = (int)(lane - half);
#pragma unroll
        for (int j = 0; j < L; ++j) {
            const float sx = __shfl(sm.x, base + j, 64), sy = __shfl(sm.y, base + j, 64);
            const float sz = __shfl(sm.z, base + j, 64), sw = __shfl(sm.w, base + j, 64);
            const int sok = __shfl((int)S.ok, base + j, 64);
            if (!sok) return true;
            cr = cr + (sx * sw) * T;  // volume.frag:44-45
            cg = cg + (sy * sw) * T;
            cb = cb + (sz * sw) * T;
            T = T * (1.0f - sw);
            if (T == 0.0f || T < P.ert_eps) return true;
        }
        return false;
    };
    for (uint32_t j = 0; j < half; ++j) advance();  // lane j of the group starts at sample j
    Stage S0, S1;
    int k = (int)half;
    prep(S0, k);
    for (;;) {  // the lanes of a group leave together (same ok flags and T)
#pragma unroll
        for (int j = 0; j < L; ++j) advance();
        k += L;
        prep(S1, k);
        if (consume(S0)) break;
#pragma unroll
        for (int j = 0; j < L; ++j) advance();
        k += L;
        prep(S0, k);
        if (consume(S1)) break;
    }
    if (P.tile_cost) {  // adaptive order: this tile's duration for the next launch
        __syncthreads();
        if (tid == 0)
            P.tile_cost[tile_y * P.tiles_x + tile_x] =
                (uint32_t)min(wall_clock64() - wg_start, 0x7FFFFFFFLL);
    }
#ifdef VR_WG_TIMES
    __syncthreads();
    if (tid == 0) wg_times_record((unsigned long long)wg_t0, tile_y * P.tiles_x + tile_x);
#endif
    if (!active || half) return;
    const float A = 1.0f - T;  // volume.frag:50 + blend (offscreen_pass.cpp:715-725)
    const float omA = 1.0f - A;
    const float o0 = cr * A + P.clear[0] * omA;
    const float o1 = cg * A + P.clear[1] * omA;
    const float o2 = cb * A + P.clear[2] * omA;
    const float o3 = A * A + P.clear[3] * omA;
    const size_t idx = (size_t)ly * P.W + px;
    if (P.out_format == 0) {
        static_cast<uint32_t *>(P.out)[idx] =
            unorm8(o0) | (unorm8(o1) << 8) | (unorm8(o2) << 16) | (unorm8(o3) << 24);
    } else {
        static_cast<float4 *>(P.out)[idx] = make_float4(o0, o1, o2, o3);
    }
}

// ---- adaptive tile order --------------------------------------------------------------------

// One workgroup per XCD x over its tile list (the tiles of the super-tiles s = x (mod 8), as
// tile_order 3 assigns them; built on the host once per geometry: lists[x * per_xcd + j],
// ~0 = none): counting-sorted by their last duration into 64 log-scale buckets, longest
// first, written to perm[x + 8 j] (j = rank), the XCD's remaining slots ~0.  Workgroups are
// dispatched in index order round-robin over the XCDs, so each XCD starts its longest tiles
// first and the frame no longer ends on a few long rays.
// Each XCD's tiles, longest first by the last launch's durations: a stable counting sort
// over one bucket per octave of duration (bucket 31 = longest).  Thread t owns list entries
// [t chunk, (t + 1) chunk); counts per (bucket, thread), offsets bucket-major (longest
// first) and thread-minor, so the tiles of one bucket keep their list order (the XCD's
// super-tiles in raster order) and tiles running together on an XCD stay neighbours.
// Against 4 buckets per octave in arbitrary order: C3 +1.8%, shaded views 1-4% faster
// (profiles/r01/tile_order/stable_octave_ab.txt).
#ifndef VR_ORDER_OCTAVES
#define VR_ORDER_OCTAVES 1
#endif
__global__ __launch_bounds__(256) void order_tiles_kernel(const uint32_t *__restrict__ cost,
                                                          const uint32_t *__restrict__ lists,
                                                          uint32_t *__restrict__ perm,
                                                          uint32_t per_xcd)
{
    constexpr int NB = 32;
    __shared__ uint32_t cnt[NB][257];  // [b][t]: offset within bucket b; [b][256]: bucket base
    __shared__ uint32_t n_tiles;
    const uint32_t x = blockIdx.x, tid = threadIdx.x;
    const uint32_t *list = lists + (size_t)x * per_xcd;
    // experiment builds: VR_ORDER_OCTAVES octaves per bucket
    auto bucket = [](uint32_t c) -> uint32_t { return c < 2 ? 0u : (31u - __clz(c)) / VR_ORDER_OCTAVES; };
    const uint32_t chunk = (per_xcd + 255) / 256;
    const uint32_t j0 = min(per_xcd, tid * chunk), j1 = min(per_xcd, j0 + chunk);
    for (int b = 0; b < NB; ++b) cnt[b][tid] = 0;
    __syncthreads();
    for (uint32_t j = j0; j < j1; ++j) {
        const uint32_t t = list[j];
        if (t != 0xFFFFFFFFu) ++cnt[bucket(cost[t])][tid];
    }
    __syncthreads();
    if (tid < NB) {  // exclusive prefix over the threads of bucket tid; its total in [256]
        uint32_t acc = 0;
        for (int k = 0; k < 256; ++k) {
            const uint32_t v = cnt[tid][k];
            cnt[tid][k] = acc;
            acc += v;
        }
        cnt[tid][256] = acc;
    }
    __syncthreads();
    if (tid == 0) {  // bucket bases, longest first
        uint32_t acc = 0;
        for (int b = NB - 1; b >= 0; --b) {
            const uint32_t v = cnt[b][256];
            cnt[b][256] = acc;
            acc += v;
        }
        n_tiles = acc;
    }
    __syncthreads();
    for (uint32_t j = j0; j < j1; ++j) {
        const uint32_t t = list[j];
        if (t != 0xFFFFFFFFu) {
            const uint32_t b = bucket(cost[t]);
            perm[x + 8 * (cnt[b][256] + cnt[b][tid]++)] = t;
        }
    }
    for (uint32_t j = n_tiles + tid; j < per_xcd; j += blockDim.x) perm[x + 8 * j] = 0xFFFFFFFFu;
}

// ---- volume ingest: linear (any NRRD element type) -> bricked paired elements -------------

// One thread per stored element: padded element coordinates -> the voxels it holds (2 z-pair,
// 4 yz-quad), 0 outside the logical volume (border).
template <typename SrcT, typename DstT>
__global__ __launch_bounds__(256) void brick_kernel(const SrcT *__restrict__ src,
                                                    Vox<DstT> *__restrict__ dst, uint32_t nx,
                                                    uint32_t ny, uint32_t nz, uint32_t nbx,
                                                    uint32_t nby, size_t nbricks)
{
    constexpr bool zpair = kZPair<DstT>;
    using G = GeomOf<DstT>;
    using V = Vox<DstT>;
    // a workgroup per brick (grid-stride over bricks), its threads over the brick's elements:
    // brick coordinates once per brick, element coordinates by constant divisors, and each
    // brick's elements written contiguously
    for (size_t bidx = blockIdx.x; bidx < nbricks; bidx += gridDim.x)
    for (uint32_t l = threadIdx.x; l < (uint32_t)G::Elems; l += blockDim.x) {
        const size_t g = bidx * G::Elems + l;
        const uint32_t lx = l % G::EX, lyz = l / G::EX, lyy = lyz % G::EY, lz = lyz / G::EY;
        uint32_t bx, by, bz;
        brick_coords((uint32_t)bidx, nbx, nby, bx, by, bz);
        const long x = (long)bx * G::BX + lx - G::Lo - kPad;
        const long y = (long)by * G::BY + lyy - G::Lo - kPad;
        const long z = (long)bz * G::BZ + lz - G::Lo - kPad;
        auto at = [&](long xx, long yy, long zz) -> V {
            if (xx < 0 || yy < 0 || zz < 0 || xx >= (long)nx || yy >= (long)ny || zz >= (long)nz)
                return (V)0;
            return (V)src[(size_t)xx + (size_t)nx * ((size_t)yy + (size_t)ny * (size_t)zz)];
        };
        // one store per element (a u8 quad is one dword, not four byte stores)
        if constexpr (kPlainF32<DstT> || kPlainByte<DstT>) {
            dst[g] = at(x, y, z);
        } else if constexpr (zpair) {
            reinterpret_cast<float2 *>(dst)[g] = make_float2(at(x, y, z), at(x, y, z + 1));
        } else {
            struct alignas(4 * sizeof(V)) Quad {
                V v[4];
            };
            Quad q;
            q.v[0] = at(x, y, z);
            q.v[1] = at(x, y, z + 1);
            q.v[2] = at(x, y + 1, z);
            q.v[3] = at(x, y + 1, z + 1);
            reinterpret_cast<Quad *>(dst)[g] = q;
        }
    }
}

// ---- synthetic volumes (multi-GiB configs): generated linear, then bricked --------------------

__device__ __forceinline__ float hash01(uint32_t x, uint32_t y, uint32_t z)
{
    uint32_t h = (x * 73856093u) ^ (y * 19349663u) ^ (z * 83492791u);
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    return (float)(h & 0xFFFFFFu) * (1.0f / 16777216.0f);
}

template <typename DstT>
__device__ __forceinline__ DstT to_storage(float v)
{
    if constexpr (sizeof(DstT) == 4) {
        return v;
    } else {
        constexpr float lo = (DstT)(-1) < (DstT)0 ? (sizeof(DstT) == 1 ? -128.f : -32768.f) : 0.f;
        constexpr float hi = (DstT)(-1) < (DstT)0 ? (sizeof(DstT) == 1 ? 127.f : 32767.f)
                                                  : (sizeof(DstT) == 1 ? 255.f : 65535.f);
        return (DstT)fminf(fmaxf(rintf(v), lo), hi);
    }
}

// params: [ng, noise_amp, out_scale, ng * (cx, cy, cz, k, amp)] in voxel units;
// value = out_scale * (sum_g amp exp(-k |x - c|^2) + noise_amp * hash01(x,y,z)).
template <typename DstT>
__global__ __launch_bounds__(256) void generate_kernel(DstT *__restrict__ dst, uint32_t nx,
                                                       uint32_t ny, size_t total,
                                                       const float *__restrict__ prm)
{
    const int ng = (int)prm[0];
    const float noise = prm[1], scale = prm[2];
    for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (size_t)gridDim.x * blockDim.x) {
        const uint32_t x = (uint32_t)(g % nx);
        const size_t yz = g / nx;
        const uint32_t y = (uint32_t)(yz % ny), z = (uint32_t)(yz / ny);
        const float fx = (float)x, fy = (float)y, fz = (float)z;
        float acc = 0.0f;
        for (int q = 0; q < ng; ++q) {
            const float *c = prm + 3 + 5 * q;
            const float dx = fx - c[0], dy = fy - c[1], dz = fz - c[2];
            acc += c[4] * __expf(-c[3] * (dx * dx + dy * dy + dz * dz));
        }
        acc += noise * hash01(x, y, z);
        dst[g] = to_storage<DstT>(acc * scale);
    }
}

// ---- min/max over a linear buffer -------------------------------------------------------------

__device__ __forceinline__ uint32_t ordered(float f)
{
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

template <typename VT>
__global__ __launch_bounds__(256) void minmax_kernel(const VT *__restrict__ vol, size_t total,
                                                     uint32_t *out)
{
    uint32_t lo = 0xFFFFFFFFu, hi = 0u;
    for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (size_t)gridDim.x * blockDim.x) {
        const uint32_t o = ordered((float)vol[g]);
        lo = o < lo ? o : lo;
        hi = o > hi ? o : hi;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t l2 = __shfl_xor(lo, off, 64), h2 = __shfl_xor(hi, off, 64);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
    }
    // one atomic pair per workgroup: the waves' results meet in LDS first (a pair per wave on
    // one address serialised the kernel: 1.55 ms for 512^3 f32)
    __shared__ uint32_t s_lo[4], s_hi[4];
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_lo[w] = lo;
        s_hi[w] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint32_t i = 1; i < (blockDim.x >> 6); ++i) {
            lo = s_lo[i] < lo ? s_lo[i] : lo;
            hi = s_hi[i] > hi ? s_hi[i] : hi;
        }
        atomicMin(&out[0], lo);
        atomicMax(&out[1], hi);
    }
}

// ---- narrowest exact storage of 32/64-bit input ---------------------------------------------
// The reference converts every NRRD element type to float (nrrd_file_parser.cpp:49-77), so an
// 8-bit CT volume reaches volume_dataset_changed as floats.  out[0] / out[1]: the minimum and
// maximum voxel (as int) when every voxel is an integer in [kIntRangeLo, kIntRangeHi]; out[2]
// != 0 otherwise (a fraction, NaN, infinity, -0.0, or a value outside that range).  A float
// voxel counts as an integer only if v == rint(v) and it is not -0.0, so storing it in an
// 8/16-bit type and converting back (float(int) is exact) gives the same bits.
constexpr int kIntRangeLo = -32768, kIntRangeHi = 65535;
template <typename SrcT>
__global__ __launch_bounds__(256) void int_range_kernel(const SrcT *__restrict__ src, size_t total,
                                                        int *out)
{
    int lo = kIntRangeHi, hi = kIntRangeLo, bad = 0;
    for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (size_t)gridDim.x * blockDim.x) {
        const SrcT v = src[g];
        int iv;
        if constexpr (std::is_floating_point<SrcT>::value) {
            const float f = (float)v;
            const bool ok = f >= (float)kIntRangeLo && f <= (float)kIntRangeHi && f == rintf(f) &&
                            !(f == 0.0f && signbit(f));
            bad |= ok ? 0 : 1;
            iv = ok ? (int)f : 0;
        } else {
            const bool ok = (long long)v >= kIntRangeLo && (long long)v <= kIntRangeHi &&
                            !(std::is_unsigned<SrcT>::value && (unsigned long long)v > (unsigned long long)kIntRangeHi);
            bad |= ok ? 0 : 1;
            iv = ok ? (int)v : 0;
        }
        lo = iv < lo ? iv : lo;
        hi = iv > hi ? iv : hi;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const int l2 = __shfl_xor(lo, off, 64), h2 = __shfl_xor(hi, off, 64), b2 = __shfl_xor(bad, off, 64);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
        bad |= b2;
    }
    __shared__ int s_lo[4], s_hi[4], s_bad[4];  // one atomic set per workgroup (minmax_kernel)
    const uint32_t w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_lo[w] = lo;
        s_hi[w] = hi;
        s_bad[w] = bad;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint32_t i = 1; i < (blockDim.x >> 6); ++i) {
            lo = s_lo[i] < lo ? s_lo[i] : lo;
            hi = s_hi[i] > hi ? s_hi[i] : hi;
            bad |= s_bad[i];
        }
        atomicMin(&out[0], lo);
        atomicMax(&out[1], hi);
        if (bad) atomicOr(&out[2], 1);
    }
}

// ---- f32 gradient field (shading) ------------------------------------------------------------

// Voxel at padded coordinates (p = logical + kPad) from the bricked z-pair density: component
// 0 of the element at p (cell_offset); 0 outside the logical volume.
__device__ __forceinline__ float padded_voxel(const float *__restrict__ bricks, int px, int py,
                                              int pz, uint32_t nx, uint32_t ny, uint32_t nz,
                                              uint32_t nbx, uint32_t nby)
{
    if (px < kPad || py < kPad || pz < kPad || px >= (int)nx + kPad || py >= (int)ny + kPad ||
        pz >= (int)nz + kPad)
        return 0.0f;
    return bricks[kF32VoxelsPerElement * cell_offset<float>(px, py, pz, nbx, nby)];
}

// The f32 alternative-geometry copies straight from the 8^3 z-pair bricks (round 6; before: an
// unbrick to a linear f32 temporary, then brick_kernel from it): one thread per stored element
// of the copy, its voxels read as padded_voxel (0 outside the volume) -- the same values
// brick_kernel stores, so the same bytes, without the volume-sized temporary and one pass less.
template <typename DstT>
__global__ __launch_bounds__(256) void rebrick_f32_kernel(const float *__restrict__ src,
                                                          float *__restrict__ dst, uint32_t nx,
                                                          uint32_t ny, uint32_t nz, uint32_t snbx,
                                                          uint32_t snby, uint32_t snbz, uint32_t nbx,
                                                          uint32_t nby, size_t nbricks)
{
    using G = GeomOf<DstT>;
    for (size_t bidx = blockIdx.x; bidx < nbricks; bidx += gridDim.x) {
        uint32_t bx, by, bz;
        brick_coords((uint32_t)bidx, nbx, nby, bx, by, bz);
        for (uint32_t l = threadIdx.x; l < (uint32_t)G::Elems; l += blockDim.x) {
            const size_t g = bidx * G::Elems + l;
            const uint32_t lx = l % G::EX, lyz = l / G::EX, lyy = lyz % G::EY, lz = lyz / G::EY;
            // padded coordinates of the element (brick_kernel's logical ones + kPad)
            const int x = (int)(bx * G::BX + lx) - G::Lo, y = (int)(by * G::BY + lyy) - G::Lo,
                      z = (int)(bz * G::BZ + lz) - G::Lo;
            if constexpr (kPlainF32<DstT>) {
                dst[g] = padded_voxel(src, x, y, z, nx, ny, nz, snbx, snby);
            } else if (kF32VoxelsPerElement == 2 && x >= 0 && y >= 0 && z >= 0 &&
                       x < (int)(snbx * GeomWide::BX) && y < (int)(snby * GeomWide::BY) &&
                       z < (int)(snbz * GeomWide::BZ)) {
                // a source z-pair element holds {v(z), v(z + 1)} with the border stored as 0
                reinterpret_cast<float2 *>(dst)[g] =
                    reinterpret_cast<const float2 *>(src)[cell_offset<float>(x, y, z, snbx, snby)];
            } else {
                reinterpret_cast<float2 *>(dst)[g] =
                    make_float2(padded_voxel(src, x, y, z, nx, ny, nz, snbx, snby),
                                padded_voxel(src, x, y, z + 1, nx, ny, nz, snbx, snby));
            }
        }
    }
}

// binary16 of d * 2^k (scale = 2^k): clamped to +-65504 first (NaN passes), rounded to nearest
// even (v_cvt_f16_f32; f16 denormals kept).  The oracle's round_f16 restates it.
__device__ __forceinline__ _Float16 field_half(float d, float scale)
{
    float x = d * scale;
    x = x > 65504.0f ? 65504.0f : (x < -65504.0f ? -65504.0f : x);
    return (_Float16)x;
}

// One thread per stored element: D_e(p) = v(p + e) - v(p - e) (the oracle's dvox).  f32 (H =
// false): the element's two voxels p = (x, y, z) and (x, y, z + 1), written as {Dx, Dx', Dy,
// Dy', Dz, Dz'}.  binary16 (H = true): the four voxels (x, y + dy, z + dz), per axis
// {D(y,z), D(y,z+1), D(y+1,z), D(y+1,z+1)}, each field_half(D, scale).
// A workgroup per brick (grid-stride over bricks): the brick's voxel neighbourhood -- padded
// coordinates [B b - 1, B b + E] in x, [B b - 1, B b + E + H] in y, [B b - 1, B b + E + 1] in z
// (E = elements per axis) -- is staged in LDS once, with one gather per voxel, and every
// element's differences read from there (the same subtractions, so the same bits): one global
// load per staged voxel instead of 12 (f32) or 24 (binary16) per element.  Each brick's
// elements are written contiguously.
template <bool H>
__global__ __launch_bounds__(256) void grad_field_kernel(const float *__restrict__ bricks,
                                                         float *__restrict__ grad, uint32_t nx,
                                                         uint32_t ny, uint32_t nz, uint32_t nbx,
                                                         uint32_t nby, size_t nbricks, float scale)
{
    using G = GeomWide;
    constexpr int LX = G::EX + 2, LY = G::EY + 2 + (H ? 1 : 0), LZ = G::EZ + 3;
    __shared__ float box[LX * LY * LZ];
    // the brick's 24-B elements, assembled here and stored as consecutive 8-B words per lane
    __shared__ uint2 ostage[3 * G::Elems];
    uint2 *__restrict__ out = reinterpret_cast<uint2 *>(grad);
    const uint32_t nbz = (uint32_t)(nbricks / ((size_t)nbx * nby));
    for (size_t bidx = blockIdx.x; bidx < nbricks; bidx += gridDim.x) {
        uint32_t bx, by, bz;
        brick_coords((uint32_t)bidx, nbx, nby, bx, by, bz);
        const int x0 = (int)(bx * G::BX) - 1, y0 = (int)(by * G::BY) - 1, z0 = (int)(bz * G::BZ) - 1;
        __syncthreads();  // the previous brick's elements have read the box and left ostage
        // two z-slices per load: the z-pair element at (x, y, z) holds {v(z), v(z + 1)}, the
        // border stored as 0 (padded_voxel where the element is outside the stored grid)
        static_assert(LZ % 2 == 0, "the box is loaded in z-pairs");
        for (int i = (int)threadIdx.x; i < LX * LY * (LZ / 2); i += (int)blockDim.x) {
            const int ix = i % LX, iyz = i / LX, iy = iyz % LY, iz = 2 * (iyz / LY);
            const int px = x0 + ix, py = y0 + iy, pz = z0 + iz;
            float2 v;
            if (kF32VoxelsPerElement == 2 && px >= 0 && py >= 0 && pz >= 0 &&
                px < (int)(nbx * G::BX) && py < (int)(nby * G::BY) && pz < (int)(nbz * G::BZ))
                v = reinterpret_cast<const float2 *>(bricks)[cell_offset<float>(px, py, pz, nbx, nby)];
            else
                v = make_float2(padded_voxel(bricks, px, py, pz, nx, ny, nz, nbx, nby),
                                padded_voxel(bricks, px, py, pz + 1, nx, ny, nz, nbx, nby));
            box[(iz * LY + iy) * LX + ix] = v.x;
            box[((iz + 1) * LY + iy) * LX + ix] = v.y;
        }
        __syncthreads();
        for (uint32_t l = threadIdx.x; l < (uint32_t)G::Elems; l += blockDim.x) {
            const uint32_t lx = l % G::EX, lyz = l / G::EX, lyy = lyz % G::EY, lz = lyz / G::EY;
            uint2 *o = ostage + 3 * l;
            if (lz >= (uint32_t)G::EZ) {  // alignment padding of the brick: never read
                o[0] = o[1] = o[2] = make_uint2(0u, 0u);
                continue;
            }
            // box index of padded voxel (x0 + 1 + lx + dx, y0 + 1 + lyy + dy, z0 + 1 + lz + dz)
            const int c = ((int)lz + 1) * (LX * LY) + ((int)lyy + 1) * LX + ((int)lx + 1);
            if constexpr (H) {
                _Float16 hv[12];
#pragma unroll
                for (int q = 0; q < 4; ++q) {  // q = dz + 2 dy
                    const int cq = c + (q >> 1) * LX + (q & 1) * (LX * LY);
                    auto V = [&](int dx, int dy, int dz) { return box[cq + dx + dy * LX + dz * (LX * LY)]; };
                    hv[0 + q] = field_half(V(1, 0, 0) - V(-1, 0, 0), scale);
                    hv[4 + q] = field_half(V(0, 1, 0) - V(0, -1, 0), scale);
                    hv[8 + q] = field_half(V(0, 0, 1) - V(0, 0, -1), scale);
                }
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    const h2v lo = {hv[4 * i], hv[4 * i + 1]}, hi = {hv[4 * i + 2], hv[4 * i + 3]};
                    o[i] = make_uint2(__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi));
                }
            } else {
                float d[6];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int ch = c + h * (LX * LY);
                    auto V = [&](int dx, int dy, int dz) { return box[ch + dx + dy * LX + dz * (LX * LY)]; };
                    d[0 + h] = V(1, 0, 0) - V(-1, 0, 0);
                    d[2 + h] = V(0, 1, 0) - V(0, -1, 0);
                    d[4 + h] = V(0, 0, 1) - V(0, 0, -1);
                }
#pragma unroll
                for (int i = 0; i < 3; ++i)
                    o[i] = make_uint2(__float_as_uint(d[2 * i]), __float_as_uint(d[2 * i + 1]));
            }
        }
        __syncthreads();
        uint2 *__restrict__ ob = out + bidx * (3 * (size_t)G::Elems);
        for (uint32_t j = threadIdx.x; j < 3u * (uint32_t)G::Elems; j += blockDim.x) ob[j] = ostage[j];
    }
}

// ---- empty-space classification (skip_empty) --------------------------------------------------

// One wavefront per brick: min/max over every voxel its stored elements hold (apron and zero
// border included: exactly the values a sample whose cell lies in the brick can read).  A
// brick holding a NaN gets (NaN, NaN), which the classifier never calls empty.
template <typename VT>
__global__ __launch_bounds__(256) void brick_range_kernel(const VT *__restrict__ bricks,
                                                          uint32_t nbricks, uint32_t per_brick,
                                                          uint32_t nbx, uint32_t nby,
                                                          float2 *__restrict__ range)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= nbricks) return;  // wave-uniform
    const VT *src = bricks + (size_t)b * per_brick;
    float lo = INFINITY, hi = -INFINITY;
    bool nan = false;
    for (uint32_t e = lane; e < per_brick; e += 64) {
        const float v = (float)src[e];
        nan = nan || v != v;
        lo = fminf(lo, v);
        hi = fmaxf(hi, v);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        lo = fminf(lo, __shfl_xor(lo, off, 64));
        hi = fmaxf(hi, __shfl_xor(hi, off, 64));
    }
    const bool any_nan = __ballot(nan) != 0;
    // range is indexed by the brick grid (x-fastest), whatever the memory order
    uint32_t bx, by, bz;
    brick_coords(b, nbx, nby, bx, by, bz);
    if (lane == 0) range[(bz * nby + by) * nbx + bx] = any_nan ? make_float2(NAN, NAN) : make_float2(lo, hi);
}

// One thread per brick: 0 if the brick can produce a visible sample, kSkipCap if EMPTY.
// Brick b is empty when every density d the trilinear filter can produce from its values maps
// to TF texels of alpha 0.  d lies in [lo, hi] up to the filter's rounding (3 levels of fmaf
// lerps: well under 1e-6 |d|), so the bounds are widened by kRangeMargin; t = (d - vmin) /
// range, u = t * n - 0.5 and floor are monotone, so the texels tf_lookup can touch are
// [floor(u(lo)), floor(u(hi)) + 1] clamped to [0, n - 1].  tf_nz is the prefix count of
// nonzero-alpha texels (n + 1 entries).  A sample whose alpha is lerp(0, 0, w) = 0 adds
// (rgb * 0) * T = +0 to C and leaves T unchanged: skipping it is exact.
__global__ __launch_bounds__(256) void classify_kernel(const float2 *__restrict__ range,
                                                       uint32_t nbricks,
                                                       const uint32_t *__restrict__ tf_nz,
                                                       int tf_n, float tf_nf, float vmin,
                                                       float vrange, uint8_t *__restrict__ dist)
{
    constexpr float kRangeMargin = 4.0e-6f;
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nbricks) return;
    bool empty = false;
    if (vrange > 0.0f) {
        const float2 r = range[b];
        if (r.x == r.x && r.y == r.y) {  // no NaN in the brick
            const float m = (fabsf(r.x) + fabsf(r.y)) * kRangeMargin;
            const float t0 = ((r.x - m) - vmin) / vrange;
            const float t1 = ((r.y + m) - vmin) / vrange;
            float u0 = t0 * tf_nf - 0.5f, u1 = t1 * tf_nf - 0.5f;
            u0 = fminf(fmaxf(u0, -1.0f), tf_nf);
            u1 = fminf(fmaxf(u1, -1.0f), tf_nf);
            int i0 = (int)floorf(u0), i1 = (int)floorf(u1) + 1;
            i0 = i0 < 0 ? 0 : (i0 > tf_n - 1 ? tf_n - 1 : i0);
            i1 = i1 < 0 ? 0 : (i1 > tf_n - 1 ? tf_n - 1 : i1);
            empty = tf_nz[i1 + 1] == tf_nz[i0];
        }
    }
    dist[b] = empty ? (uint8_t)kSkipCap : (uint8_t)0;
}

// One separable pass of the Chebyshev (L-inf) distance transform of the non-empty bricks,
// along axis `axis`: out(b) = min over |o| <= kSkipCap of max(|o|, in(b + o e_axis)), capped.
// Three passes (x, y, z) from the classification give min(kSkipCap, distance in bricks to
// the nearest non-empty brick); bricks past the grid count as empty (a ray there has left
// the volume, and the march's bounds test ends it).
__global__ __launch_bounds__(256) void dist_pass_kernel(const uint8_t *__restrict__ in,
                                                        uint8_t *__restrict__ out, uint32_t nbx,
                                                        uint32_t nby, uint32_t nbz, int axis)
{
    const uint32_t nb = nbx * nby * nbz;
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const uint32_t bx = b % nbx, by = (b / nbx) % nby, bz = b / (nbx * nby);
    const int pos = axis == 0 ? (int)bx : (axis == 1 ? (int)by : (int)bz);
    const int len = axis == 0 ? (int)nbx : (axis == 1 ? (int)nby : (int)nbz);
    const long stride = axis == 0 ? 1 : (axis == 1 ? (long)nbx : (long)nbx * nby);
    int best = in[b];
    for (int o = 1; o < kSkipCap && o < best; ++o) {
        if (pos - o >= 0) {
            const int v = in[b - o * stride];
            best = min(best, max(o, v));
        }
        if (pos + o < len) {
            const int v = in[b + o * stride];
            best = min(best, max(o, v));
        }
    }
    out[b] = (uint8_t)best;
}

// ---- rank-0 framebuffer assembly after the RCCL gather ---------------------------------------

template <typename PixT>
__global__ __launch_bounds__(256) void assemble_kernel(const PixT *__restrict__ gathered,
                                                       PixT *__restrict__ out, uint32_t W,
                                                       uint32_t H, uint32_t rb, uint32_t nranks,
                                                       uint32_t shard_rows, RowShare share)
{
    const size_t total = (size_t)W * H;
    for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (size_t)gridDim.x * blockDim.x) {
        const uint32_t y = (uint32_t)(g / W), x = (uint32_t)(g - (size_t)y * W);
        const uint32_t blk = y / rb;
        uint32_t rank, lb;
        share_owner(blk, nranks, share, rank, lb);
        const uint32_t ly = lb * rb + (y - blk * rb);
        out[g] = gathered[((size_t)rank * shard_rows + ly) * W + x];
    }
}

#ifdef VR_EXPERIMENTS
// Experiment builds only: dynamic LDS reserved per march workgroup (VR_MARCH_LDS_PAD bytes),
// which caps the workgroups resident on a CU -- fewer waves sharing its L1.
static uint32_t march_lds_pad()
{
    static const uint32_t v = [] {
        const char *e = std::getenv("VR_MARCH_LDS_PAD");
        return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 0u;
    }();
    return v;
}
#else
constexpr uint32_t march_lds_pad() { return 0; }
#endif

template <typename VT, bool SHADE, bool COUNT, bool SKIP, bool GF = false, bool PIPE = false>
hipError_t launch_march_t(const MarchParams &p, hipStream_t stream)
{
    const uint32_t nblocks = p.tile_perm ? p.nperm
                             : p.tile_order >= 3 ? ((p.supers_total + 7) / 8) * 8 * kSuper * kSuper
                                                 : p.tiles_x * p.tiles_y;
    if (p.tiles_x * p.tiles_y == 0) return hipSuccess;
    hipLaunchKernelGGL((march_kernel<VT, SHADE, COUNT, SKIP, GF, PIPE>), dim3(nblocks), dim3(kThreadsPerTile),
                       march_lds_pad(), stream, p);
    return hipGetLastError();
}

template <typename VT, bool SHADE, bool GF>
hipError_t launch_pair_t(const MarchParams &p, hipStream_t stream)
{
    const uint32_t nblocks = p.tile_perm ? p.nperm
                             : p.tile_order >= 3 ? ((p.supers_total + 7) / 8) * 8 * kSuper * kSuper
                                                 : p.tiles_x * p.tiles_y;
    if (p.tiles_x * p.tiles_y == 0) return hipSuccess;
    if (p.pair == 4)
        hipLaunchKernelGGL((march_pair_kernel<VT, SHADE, GF, 4>), dim3(nblocks), dim3(kThreads),
                           0, stream, p);
    else
        hipLaunchKernelGGL((march_pair_kernel<VT, SHADE, GF, 2>), dim3(nblocks), dim3(kThreads),
                           0, stream, p);
    return hipGetLastError();
}

template <typename VT>
hipError_t launch_march_vt(bool shade, bool count, const MarchParams &p, hipStream_t s)
{
    if (p.pair) {  // host: not counting, no skip-empty, tf_n <= kTfLds, 16x8 tiles
        if (!shade) return launch_pair_t<VT, false, false>(p, s);
        if constexpr (kZPair<VT>)
            if (p.grad) return launch_pair_t<VT, true, true>(p, s);
        return launch_pair_t<VT, true, false>(p, s);
    }
    if (p.pipelined && !count && !p.skip_empty && p.tf_n <= kTfLds) {
        if (!shade) return launch_march_t<VT, false, false, false, false, true>(p, s);
        if constexpr (kZPair<VT>)
            if (p.grad) return launch_march_t<VT, true, false, false, true, true>(p, s);
        return launch_march_t<VT, true, false, false, false, true>(p, s);
    }
    if constexpr (kZPair<VT>) {
        if (shade && p.grad) {
            if (p.skip_empty)
                return count ? launch_march_t<VT, true, true, true, true>(p, s)
                             : launch_march_t<VT, true, false, true, true>(p, s);
            return count ? launch_march_t<VT, true, true, false, true>(p, s)
                         : launch_march_t<VT, true, false, false, true>(p, s);
        }
    }
    if (p.skip_empty) {
        if (shade)
            return count ? launch_march_t<VT, true, true, true>(p, s)
                         : launch_march_t<VT, true, false, true>(p, s);
        return count ? launch_march_t<VT, false, true, true>(p, s)
                     : launch_march_t<VT, false, false, true>(p, s);
    }
    if (shade)
        return count ? launch_march_t<VT, true, true, false>(p, s)
                     : launch_march_t<VT, true, false, false>(p, s);
    return count ? launch_march_t<VT, false, true, false>(p, s)
                 : launch_march_t<VT, false, false, false>(p, s);
}

// The f32 volume with the binary16 difference field (MarchParams::grad_half; shaded launches
// that read the field, not LDS-staged): the field variants of launch_march_vt.
template <typename VT>
hipError_t launch_march_half_field(bool count, const MarchParams &p, hipStream_t s)
{
    if (p.pair) return launch_pair_t<VT, true, true>(p, s);
    if (p.pipelined && !count && !p.skip_empty && p.tf_n <= kTfLds)
        return launch_march_t<VT, true, false, false, true, true>(p, s);
    if (p.skip_empty)
        return count ? launch_march_t<VT, true, true, true, true>(p, s)
                     : launch_march_t<VT, true, false, true, true>(p, s);
    return count ? launch_march_t<VT, true, true, false, true>(p, s)
                 : launch_march_t<VT, true, false, false, true>(p, s);
}

// The f32 volume's GeomAlt copy (kAltFlag) serves full-frame launches without skip-empty, the
// difference field, lane groups or LDS staging (the host picks it for oblique and sparse views
// only): single-stage or pipelined, shaded (stencil gradient) or not.
template <typename VT>
hipError_t launch_march_alt(bool shade, const MarchParams &p, hipStream_t s)
{
    if (p.pipelined && p.tf_n <= kTfLds)
        return shade ? launch_march_t<VT, true, false, false, false, true>(p, s)
                     : launch_march_t<VT, false, false, false, false, true>(p, s);
    return shade ? launch_march_t<VT, true, false, false>(p, s)
                 : launch_march_t<VT, false, false, false>(p, s);
}

// workgroups for the per-brick kernels (brick_kernel, grad_field_kernel): one per brick
inline unsigned grid_bricks(size_t nb)
{
    return (unsigned)(nb > 65536 ? 65536 : (nb == 0 ? 1 : nb));
}

inline unsigned grid_for(size_t total)
{
    size_t g = (total + 255) / 256;
    return (unsigned)(g > 2048 * 8 ? 2048 * 8 : (g == 0 ? 1 : g));
}

// Readback (vr_debug_read_volume*): voxel v(x, y, z) is component 0 of element (x, y, z) of the
// bricked layout; slices [z0, z0 + cz) into a linear x-fastest buffer of the storage type.
template <typename T>
__global__ __launch_bounds__(256) void unbrick_kernel(const Vox<T> *__restrict__ bricks,
                                                     Vox<T> *__restrict__ dst, uint32_t nx,
                                                     uint32_t ny, uint32_t nbx, uint32_t nby,
                                                     uint32_t z0, size_t count)
{
    constexpr size_t vpe = std::is_same<T, float>::value ? kF32VoxelsPerElement
                                                         : (kPlainByte<T> ? 1 : 4);
    for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < count;
         g += (size_t)gridDim.x * blockDim.x) {
        const uint32_t x = (uint32_t)(g % nx);
        const size_t yz = g / nx;
        const uint32_t y = (uint32_t)(yz % ny), z = z0 + (uint32_t)(yz / ny);
        const uint32_t pi = x + kPad, pj = y + kPad, pk = z + kPad;
        dst[g] = bricks[cell_offset<T>((int)pi, (int)pj, (int)pk, nbx, nby) * vpe];
    }
}

template <typename SrcT>
hipError_t brick_from(const void *src, void *dst, uint32_t nx, uint32_t ny, uint32_t nz,
                      int storage, hipStream_t s)
{
    const uint32_t nbx = bricks_for(nx, 0, storage), nby = bricks_for(ny, 1, storage),
                   nbz = bricks_for(nz, 2, storage);
    const size_t total = (size_t)nbx * nby * nbz;  // bricks
    const SrcT *sp = static_cast<const SrcT *>(src);
    switch (storage) {
        case ST_U8: hipLaunchKernelGGL((brick_kernel<SrcT, uint8_t>), dim3(grid_bricks(total)), dim3(256), 0, s, sp, (uint8_t *)dst, nx, ny, nz, nbx, nby, total); break;
        case ST_I8: hipLaunchKernelGGL((brick_kernel<SrcT, int8_t>), dim3(grid_bricks(total)), dim3(256), 0, s, sp, (int8_t *)dst, nx, ny, nz, nbx, nby, total); break;
        case ST_U8 | kQuadFlag: hipLaunchKernelGGL((brick_kernel<SrcT, Quad8<uint8_t>>), dim3(grid_bricks(total)), dim3(256), 0, s, sp, (uint8_t *)dst, nx, ny, nz, nbx, nby, total); break;
        case ST_I8 | kQuadFlag: hipLaunchKernelGGL((brick_kernel<SrcT, Quad8<int8_t>>), dim3(grid_bricks(total)), dim3(256), 0, s, sp, (int8_t *)dst, nx, ny, nz, nbx, nby, total); break;
        case ST_U16: hipLaunchKernelGGL((brick_kernel<SrcT, uint16_t>), dim3(grid_bricks(total)), dim3(256), 0, s, sp, (uint16_t *)dst, nx, ny, nz, nbx, nby, total); break;
        case ST_I16: hipLaunchKernelGGL((brick_kernel<SrcT, int16_t>), dim3(grid_bricks(total)), dim3(256), 0, s, sp, (int16_t *)dst, nx, ny, nz, nbx, nby, total); break;
        case ST_F32 | kAltFlag: hipLaunchKernelGGL((brick_kernel<SrcT, F32Alt>), dim3(grid_bricks(total)), dim3(256), 0, s, sp, (float *)dst, nx, ny, nz, nbx, nby, total); break;
        case ST_F32 | kPlainF32Flag: hipLaunchKernelGGL((brick_kernel<SrcT, F32P>), dim3(grid_bricks(total)), dim3(256), 0, s, sp, (float *)dst, nx, ny, nz, nbx, nby, total); break;
        case ST_F32 | kStencilF32Flag: hipLaunchKernelGGL((brick_kernel<SrcT, F32S>), dim3(grid_bricks(total)), dim3(256), 0, s, sp, (float *)dst, nx, ny, nz, nbx, nby, total); break;
        default: hipLaunchKernelGGL((brick_kernel<SrcT, float>), dim3(grid_bricks(total)), dim3(256), 0, s, sp, (float *)dst, nx, ny, nz, nbx, nby, total); break;
    }
    return hipGetLastError();
}

}  // namespace

hipError_t launch_march(int storage, bool shade, bool count, const MarchParams &p,
                        hipStream_t stream)
{
    switch (storage) {
        case ST_U8: return launch_march_vt<uint8_t>(shade, count, p, stream);
        case ST_I8: return launch_march_vt<int8_t>(shade, count, p, stream);
        case ST_U8 | kQuadFlag: return launch_march_vt<Quad8<uint8_t>>(shade, count, p, stream);
        case ST_I8 | kQuadFlag: return launch_march_vt<Quad8<int8_t>>(shade, count, p, stream);
        case ST_U16: return launch_march_vt<uint16_t>(shade, count, p, stream);
        case ST_I16: return launch_march_vt<int16_t>(shade, count, p, stream);
        case ST_F32:
            if (shade && p.grad && p.grad_half)
                return launch_march_half_field<F32H>(count, p, stream);
            return launch_march_vt<float>(shade, count, p, stream);
        case ST_F32 | kAltFlag:
        case ST_F32 | kPlainF32Flag:
        case ST_F32 | kStencilF32Flag:
            if (count || p.pair || p.skip_empty || p.grad) return hipErrorInvalidValue;
            if (storage & kPlainF32Flag) return launch_march_alt<F32P>(shade, p, stream);
            if (storage & kStencilF32Flag) return launch_march_alt<F32S>(shade, p, stream);
            return launch_march_alt<F32Alt>(shade, p, stream);
        default: return hipErrorInvalidValue;
    }
}

const char *march_kernel_name(int storage, bool shade, bool count, bool skip, bool gf, bool pipe)
{
    // demangled names as rocprofv3 reports them (kernel-trace "Kernel_Name"); storage is the
    // layout code (8-bit yz-quads: the Quad8 instantiations)
    static const std::vector<std::string> names = [] {
        const char *types[11] = {"unsigned char", "signed char", "unsigned short", "short", "float",
                                 "vr::Quad8<unsigned char>", "vr::Quad8<signed char>", "vr::F32Alt",
                                 "vr::F32H", "vr::F32P", "vr::F32S"};
        std::vector<std::string> v;
        for (int t = 0; t < 11; ++t)
            for (int k = 0; k < 32; ++k) {
                std::string n = std::string("void vr::(anonymous namespace)::march_kernel<") + types[t];
                for (int bit = 4; bit >= 0; --bit) n += (k >> bit) & 1 ? ", true" : ", false";
                v.push_back(n + ">(vr::MarchParams)");
            }
        return v;
    }();
    if (storage & kQuadFlag) storage = 5 + (storage & 0xF);
    if (storage & kAltFlag) storage = 7;
    if (storage & kHalfFieldFlag) storage = 8;
    if (storage & kPlainF32Flag) storage = 9;
    if (storage & kStencilF32Flag) storage = 10;
    if (storage < 0 || storage > 10) return "march_kernel<?>";
    const int k = (shade ? 16 : 0) + (count ? 8 : 0) + (skip ? 4 : 0) + (gf ? 2 : 0) + (pipe ? 1 : 0);
    return names[storage * 32 + k].c_str();
}

hipError_t launch_unbrick(int storage, const void *bricks, void *dst, uint32_t nx, uint32_t ny,
                          uint32_t z0, uint32_t cz, hipStream_t s)
{
    const size_t n = (size_t)nx * ny * cz;
    const unsigned g = grid_for(n);
    const uint32_t bx = bricks_for(nx, 0, storage), by = bricks_for(ny, 1, storage);
    switch (storage) {
        case ST_U8: case ST_I8: hipLaunchKernelGGL((unbrick_kernel<uint8_t>), dim3(g), dim3(256), 0, s, (const uint8_t *)bricks, (uint8_t *)dst, nx, ny, bx, by, z0, n); break;
        case ST_U8 | kQuadFlag: case ST_I8 | kQuadFlag: hipLaunchKernelGGL((unbrick_kernel<Quad8<uint8_t>>), dim3(g), dim3(256), 0, s, (const uint8_t *)bricks, (uint8_t *)dst, nx, ny, bx, by, z0, n); break;
        case ST_U16: case ST_I16: hipLaunchKernelGGL((unbrick_kernel<uint16_t>), dim3(g), dim3(256), 0, s, (const uint16_t *)bricks, (uint16_t *)dst, nx, ny, bx, by, z0, n); break;
        default: hipLaunchKernelGGL((unbrick_kernel<float>), dim3(g), dim3(256), 0, s, (const float *)bricks, (float *)dst, nx, ny, bx, by, z0, n); break;
    }
    return hipGetLastError();
}

hipError_t launch_brick_from_linear(int src_dtype, const void *src, void *dst, uint32_t nx,
                                    uint32_t ny, uint32_t nz, int storage, hipStream_t s)
{
    switch (src_dtype) {  // enum vr_dtype
        case 1: return brick_from<int8_t>(src, dst, nx, ny, nz, storage, s);
        case 2: return brick_from<uint8_t>(src, dst, nx, ny, nz, storage, s);
        case 3: return brick_from<int16_t>(src, dst, nx, ny, nz, storage, s);
        case 4: return brick_from<uint16_t>(src, dst, nx, ny, nz, storage, s);
        case 5: return brick_from<int32_t>(src, dst, nx, ny, nz, storage, s);
        case 6: return brick_from<uint32_t>(src, dst, nx, ny, nz, storage, s);
        case 7: return brick_from<int64_t>(src, dst, nx, ny, nz, storage, s);
        case 8: return brick_from<uint64_t>(src, dst, nx, ny, nz, storage, s);
        case 9: return brick_from<float>(src, dst, nx, ny, nz, storage, s);
        case 10: return brick_from<double>(src, dst, nx, ny, nz, storage, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_generate(int kind, int storage, void *dst, uint32_t nx, uint32_t ny,
                           uint32_t nz, const float *params_dev, int nparams, hipStream_t s)
{
    (void)nparams;
    if (kind != 0) return hipErrorInvalidValue;
    const size_t total = (size_t)nx * ny * nz;
    switch (storage) {
        case ST_U8: hipLaunchKernelGGL((generate_kernel<uint8_t>), dim3(grid_for(total)), dim3(256), 0, s, (uint8_t *)dst, nx, ny, total, params_dev); break;
        case ST_U16: hipLaunchKernelGGL((generate_kernel<uint16_t>), dim3(grid_for(total)), dim3(256), 0, s, (uint16_t *)dst, nx, ny, total, params_dev); break;
        case ST_F32: hipLaunchKernelGGL((generate_kernel<float>), dim3(grid_for(total)), dim3(256), 0, s, (float *)dst, nx, ny, total, params_dev); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_minmax(int storage, const void *linear, size_t count, float *minmax_dev,
                         hipStream_t s)
{
    uint32_t *o = reinterpret_cast<uint32_t *>(minmax_dev);
    const unsigned g = std::min(grid_for(count), 2048u);  // 8 workgroups per CU, grid-stride
    switch (storage) {
        case ST_U8: hipLaunchKernelGGL((minmax_kernel<uint8_t>), dim3(g), dim3(256), 0, s, (const uint8_t *)linear, count, o); break;
        case ST_I8: hipLaunchKernelGGL((minmax_kernel<int8_t>), dim3(g), dim3(256), 0, s, (const int8_t *)linear, count, o); break;
        case ST_U16: hipLaunchKernelGGL((minmax_kernel<uint16_t>), dim3(g), dim3(256), 0, s, (const uint16_t *)linear, count, o); break;
        case ST_I16: hipLaunchKernelGGL((minmax_kernel<int16_t>), dim3(g), dim3(256), 0, s, (const int16_t *)linear, count, o); break;
        default: hipLaunchKernelGGL((minmax_kernel<float>), dim3(g), dim3(256), 0, s, (const float *)linear, count, o); break;
    }
    return hipGetLastError();
}

hipError_t launch_int_range(int src_dtype, const void *src, size_t count, int *out3_dev,
                            hipStream_t s)
{
    const unsigned g = std::min(grid_for(count), 2048u);  // 8 workgroups per CU, grid-stride
    switch (src_dtype) {  // enum vr_dtype: the 32/64-bit types NrrdFileParser makes float
        case 5: hipLaunchKernelGGL((int_range_kernel<int32_t>), dim3(g), dim3(256), 0, s, (const int32_t *)src, count, out3_dev); break;
        case 6: hipLaunchKernelGGL((int_range_kernel<uint32_t>), dim3(g), dim3(256), 0, s, (const uint32_t *)src, count, out3_dev); break;
        case 7: hipLaunchKernelGGL((int_range_kernel<int64_t>), dim3(g), dim3(256), 0, s, (const int64_t *)src, count, out3_dev); break;
        case 8: hipLaunchKernelGGL((int_range_kernel<uint64_t>), dim3(g), dim3(256), 0, s, (const uint64_t *)src, count, out3_dev); break;
        case 9: hipLaunchKernelGGL((int_range_kernel<float>), dim3(g), dim3(256), 0, s, (const float *)src, count, out3_dev); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_assemble(const void *gathered, void *out, int out_format, uint32_t W,
                           uint32_t H, uint32_t row_block, uint32_t nranks,
                           uint32_t shard_rows, RowShare share, hipStream_t s)
{
    const unsigned g = grid_for((size_t)W * H);
    if (out_format == 0)
        hipLaunchKernelGGL((assemble_kernel<uint32_t>), dim3(g), dim3(256), 0, s,
                           (const uint32_t *)gathered, (uint32_t *)out, W, H, row_block, nranks,
                           shard_rows, share);
    else
        hipLaunchKernelGGL((assemble_kernel<float4>), dim3(g), dim3(256), 0, s,
                           (const float4 *)gathered, (float4 *)out, W, H, row_block, nranks,
                           shard_rows, share);
    return hipGetLastError();
}

hipError_t launch_brick_range(int storage, const void *bricks, uint32_t nbx, uint32_t nby,
                              uint32_t nbz, float2 *range_dev, hipStream_t s)
{
    const uint32_t nbricks = nbx * nby * nbz;
    const unsigned g = (nbricks + 3) / 4;
    const uint32_t per = (uint32_t)(brick_elems(storage) * voxels_per_element(storage));
    switch (storage & 0xF) {  // the voxels of every element, whatever the layout
        case ST_U8: hipLaunchKernelGGL((brick_range_kernel<uint8_t>), dim3(g), dim3(256), 0, s, (const uint8_t *)bricks, nbricks, per, nbx, nby, range_dev); break;
        case ST_I8: hipLaunchKernelGGL((brick_range_kernel<int8_t>), dim3(g), dim3(256), 0, s, (const int8_t *)bricks, nbricks, per, nbx, nby, range_dev); break;
        case ST_U16: hipLaunchKernelGGL((brick_range_kernel<uint16_t>), dim3(g), dim3(256), 0, s, (const uint16_t *)bricks, nbricks, per, nbx, nby, range_dev); break;
        case ST_I16: hipLaunchKernelGGL((brick_range_kernel<int16_t>), dim3(g), dim3(256), 0, s, (const int16_t *)bricks, nbricks, per, nbx, nby, range_dev); break;
        default: hipLaunchKernelGGL((brick_range_kernel<float>), dim3(g), dim3(256), 0, s, (const float *)bricks, nbricks, per, nbx, nby, range_dev); break;
    }
    return hipGetLastError();
}

hipError_t launch_grad_field(const float *bricks, float *grad, uint32_t nx, uint32_t ny,
                             uint32_t nz, bool half, int scale_log2, hipStream_t s)
{
    const uint32_t nbx = bricks_for(nx, 0, ST_F32), nby = bricks_for(ny, 1, ST_F32),
                   nbz = bricks_for(nz, 2, ST_F32);
    const size_t total = (size_t)nbx * nby * nbz;  // bricks
    const float scale = std::ldexp(1.0f, scale_log2);
    if (half)
        hipLaunchKernelGGL(grad_field_kernel<true>, dim3(grid_bricks(total)), dim3(256), 0, s,
                           bricks, grad, nx, ny, nz, nbx, nby, total, scale);
    else
        hipLaunchKernelGGL(grad_field_kernel<false>, dim3(grid_bricks(total)), dim3(256), 0, s,
                           bricks, grad, nx, ny, nz, nbx, nby, total, scale);
    return hipGetLastError();
}

hipError_t launch_rebrick_f32(const float *src_bricks, void *dst, uint32_t nx, uint32_t ny,
                              uint32_t nz, int storage, hipStream_t s)
{
    const uint32_t snbx = bricks_for(nx, 0, ST_F32), snby = bricks_for(ny, 1, ST_F32),
                   snbz = bricks_for(nz, 2, ST_F32);
    const uint32_t nbx = bricks_for(nx, 0, storage), nby = bricks_for(ny, 1, storage),
                   nbz = bricks_for(nz, 2, storage);
    const size_t total = (size_t)nbx * nby * nbz;
    float *d = static_cast<float *>(dst);
    switch (storage) {
        case ST_F32 | kAltFlag: hipLaunchKernelGGL((rebrick_f32_kernel<F32Alt>), dim3(grid_bricks(total)), dim3(256), 0, s, src_bricks, d, nx, ny, nz, snbx, snby, snbz, nbx, nby, total); break;
        case ST_F32 | kPlainF32Flag: hipLaunchKernelGGL((rebrick_f32_kernel<F32P>), dim3(grid_bricks(total)), dim3(256), 0, s, src_bricks, d, nx, ny, nz, snbx, snby, snbz, nbx, nby, total); break;
        case ST_F32 | kStencilF32Flag: hipLaunchKernelGGL((rebrick_f32_kernel<F32S>), dim3(grid_bricks(total)), dim3(256), 0, s, src_bricks, d, nx, ny, nz, snbx, snby, snbz, nbx, nby, total); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_skip_dist(const float2 *range_dev, uint32_t nbx, uint32_t nby, uint32_t nbz,
                            const uint32_t *tf_nz_dev, int tf_n, float vmin, float vrange,
                            uint8_t *dist_dev, uint8_t *scratch_dev, hipStream_t s)
{
    const uint32_t nb = nbx * nby * nbz;
    const unsigned g = (nb + 255) / 256;
    hipLaunchKernelGGL(classify_kernel, dim3(g), dim3(256), 0, s, range_dev, nb, tf_nz_dev, tf_n,
                       (float)tf_n, vmin, vrange, dist_dev);
    hipLaunchKernelGGL(dist_pass_kernel, dim3(g), dim3(256), 0, s, (const uint8_t *)dist_dev,
                       scratch_dev, nbx, nby, nbz, 0);
    hipLaunchKernelGGL(dist_pass_kernel, dim3(g), dim3(256), 0, s, (const uint8_t *)scratch_dev,
                       dist_dev, nbx, nby, nbz, 1);
    hipLaunchKernelGGL(dist_pass_kernel, dim3(g), dim3(256), 0, s, (const uint8_t *)dist_dev,
                       scratch_dev, nbx, nby, nbz, 2);
    return hipMemcpyAsync(dist_dev, scratch_dev, nb, hipMemcpyDeviceToDevice, s);
}

#ifdef VR_WG_TIMES
hipError_t debug_wg_times_reset()
{
    const unsigned int z = 0;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_wg_count), &z, sizeof(z));
}
hipError_t debug_wg_times_read(unsigned long long *out, unsigned int max, unsigned int *count)
{
    unsigned int n = 0;
    hipError_t e = hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_wg_count), sizeof(n));
    if (e != hipSuccess) return e;
    n = n < kWgTimesMax ? n : kWgTimesMax;
    n = n < max ? n : max;
    *count = n;
    return n ? hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wg_times), 4 * n * sizeof(unsigned long long))
             : hipSuccess;
}
#endif

hipError_t launch_order_tiles(const uint32_t *cost, const uint32_t *lists, uint32_t *perm,
                              uint32_t per_xcd, hipStream_t s)
{
    hipLaunchKernelGGL(order_tiles_kernel, dim3(8), dim3(256), 0, s, cost, lists, perm, per_xcd);
    return hipGetLastError();
}

}  // namespace vr
