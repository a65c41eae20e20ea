/*
 * oracle.h — CPU restatement of the reference ray-march (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity checker for the MI355X HIP path.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product library never links it.
 *
 * It restates, in plain C (OpenMP over pixel rows):
 *   res/shaders/volume.frag:21-52      the ray-march loop, predicates, composite, op order
 *   res/shaders/volume.vert:19-24      tex_coords / frag_position attributes (ray entry)
 *   src/rendering/offscreen_pass.cpp   :55-90 cube geometry (tex = pos + 0.5), :170-173 clear,
 *                                      :293 RGBA8 target, :680-681 cull back, :701-712 depth,
 *                                      :715-725 blend, :968 + :1014-1039 R32F volume + border
 *                                      sampler, :1076 + :1125-1150 sRGB TF + clamp sampler,
 *                                      :1152-1171 projection * coordinate_conversion
 *   src/data/nrrd_file_parser.cpp:39-40 min/max density normalisation inputs
 * plus the build's own extension (central-difference gradient Phong shading; the reference
 * has no shading).
 *
 * Fixed-function semantics the shader runs under, and the Vulkan 1.3 specification text each
 * rule restates (chapter "Image Operations" unless noted; section titles, not numbers, since
 * numbering moves between spec revisions):
 *   texel centres, u = s*N - 0.5       "Texel Coordinate Systems" + "Texel Filtering":
 *                                      VK_FILTER_LINEAR takes i0 = floor(u - 0.5), i1 = i0 + 1,
 *                                      weight alpha = frac(u - 0.5)   (texel_coord, tf_lookup)
 *   trilinear order: x, then y, z      "Texel Filtering", the LINEAR formula for 3D images as a
 *                                      weighted sum; the lerp nesting is this restatement's
 *                                      choice (hardware precision is implementation-defined)
 *   border = transparent black         "Wrapping Operations" (CLAMP_TO_BORDER keeps texels
 *                                      outside the image as border texels) + "Texel
 *                                      Replacement" (VK_BORDER_COLOR_FLOAT_TRANSPARENT_BLACK
 *                                      = (0,0,0,0); R32_SFLOAT reads R = 0)      (voxel)
 *   TF clamp-to-edge                   "Wrapping Operations": CLAMP_TO_EDGE i = clamp(i, 0, N-1)
 *   sRGB decode BEFORE filtering       "Format Conversion" (each texel of an _SRGB format is
 *                                      UNORM-converted, then R,G,B go through the sRGB EOTF of
 *                                      the Khronos Data Format Specification; A unchanged),
 *                                      which the sampling pipeline applies per texel ahead of
 *                                      "Texel Filtering"                   (srgb_to_linear)
 *   UNORM8 decode c / 255              "Fixed-Point Data Conversions": normalized fixed-point
 *                                      to float, f = c / (2^b - 1)
 *   RGBA8 UNORM store                  same section, float to normalized fixed-point:
 *                                      convertFloatToUint(f * 255, 8) returns one of the two
 *                                      nearest integers ("should" round to nearest) -- hence
 *                                      the 1-LSB tolerance of the RGBA8 parity tests
 *   blend                              chapter "The Framebuffer", "Blend Operations":
 *                                      VK_BLEND_OP_ADD, RGB = src*Sf + dst*Df with the factors
 *                                      of offscreen_pass.cpp:715-725
 *   back-face cull, depth              chapter "Rasterization", "Basic Polygon Rasterization"
 *                                      (facing from the signed area) / offscreen_pass.cpp:680-712
 *
 * These are cited to the published spec; no Vulkan implementation ran here to confirm them.
 *
 * Parity status: the reference's hot path is a Vulkan fragment shader that cannot run in
 * this container (no Vulkan/ICD/glslc) and the reference ships no tests or
 * golden images, so pixel parity against the REAL reference is unpinned.  This restatement
 * is pinned by (1) closed-form known-answer tests (constant TF,
 * transparent TF, startup TF, sampler unit KATs) and (2) an independent float64 numpy
 * restatement (oracle/ref_numpy.py); both are committed under tests/golden/.
 */
#ifndef VR_ORACLE_H
#define VR_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_scene {
    /* Dataset (src/data/dataset.h:9-13): dense float voxels, x fastest. */
    const float *vol;
    int32_t nx, ny, nz;
    float vmin, vmax;
    /* transfer function texels, RGBA8 sRGB, R in the low byte */
    const uint32_t *tf;
    int32_t tf_n;
    /* slicing box */
    float smin[3], smax[3];
    /* camera (view column-major, as Camera::get_view) */
    float view[16];
    float cam_pos[3];
    float fovy_deg, znear, zfar;
    int32_t width, height;
    /* params */
    float step, ray_dist, ert_eps;
    int32_t shading;
    float clear[4];
    float ka, kd, ks;
    int32_t spec_power;
    /* u8 voxels instead of vol (same layout; float(v) exact), for multi-GiB u8 volumes */
    const uint8_t *vol_u8;
    /* shading: 1 = the device's binary16 difference field (vr_params.exact_gradient == 0 on a
     * frame that reads the field): every central difference D becomes round_f16(D * 2^k),
     * k = or_field_scale_log2(vmin, vmax); 0 = exact f32 differences */
    int32_t grad_f16;
    /* Conformance study (tools/conformance_gap.py).  Each field restates one
     * implementation-defined freedom a conformant Vulkan run of the reference may take; all
     * are 0 (off) by default, and the product kernel's parity target is that default.
     * conf_weight_bits: 0 = exact float filter weights; b > 0 = the texel coordinate
     *   u = s*N - 0.5 of the 3D and 1D LINEAR filters rounded to a multiple of 2^-b
     *   (subTexelPrecisionBits; spec minimum 4), round to nearest, before floor/frac. */
    int32_t conf_weight_bits;
    int32_t conf_flags; /* OR_CONF_* below */
    /* grad_f16: the range the device takes the field's scale from -- the stored data's own
     * min/max (vr_api.hip data_range), not vmin/vmax, which may be a narrower display window.
     * grad_range_set == 0: use vmin/vmax (equal to the data range for every Dataset). */
    int32_t grad_range_set;
    float grad_range[2];
} or_scene;

/* FMA contraction the SPIR-V permits (volume_frag.spv carries no NoContraction decoration,
 * tests/test_spirv_facts.py): ray_pos = fma(ray_dir, step, ray_pos) (volume.frag:47) and
 * C.rgb = fma(rgb*a, T, C.rgb) (volume.frag:44). */
#define OR_CONF_FMA 1
/* glm's [0, 1] clip form: perspectiveRH_ZO instead of _NO (offscreen_pass.cpp:3,1166), i.e.
 * GLM_FORCE_DEPTH_ZERO_TO_ONE in effect; moves the effective near plane 0.198 -> 0.1.  Also the
 * product switch vr_params.depth_zero_to_one (vr.h ABI 8): alone it keeps the oracle's march
 * (only the ray frame changes), so parity in both forms is bit-exact. */
#define OR_CONF_CLIP_ZO 2
/* Entry attributes (in_tex_coords, in_frag_position) from a rasteriser model instead of the
 * exact double ray/box intersection: float clip positions ((proj*view)*v, volume.vert:23),
 * window coordinates snapped to 2^-8 pixel (subPixelPrecisionBits = 8), exact integer edge
 * functions, float perspective-correct barycentrics ("Basic Polygon Rasterization").  Needs
 * every front-facing vertex inside 0 <= z <= w (no near clipping); returns -95 otherwise. */
#define OR_CONF_RASTER 4
/* GPU shader arithmetic at its permitted precision: the density quotient as d * rcp(range)
 * and normalize() as v * rsqrt(dot(v, v)) with correctly rounded rcp/rsqrt (GLSL's OpFDiv
 * allows 2.5 ulp, inversesqrt 2 ulp; this is the common 1-instruction code generation). */
#define OR_CONF_GPU_MATH 8

typedef struct or_stats {
    uint64_t rays, samples, shaded_samples, steps;
} or_stats;

/* Render rows [row0, row1) of the frame into out (float RGBA, row-major, full-frame
 * indexing: out[(y*W + x)*4 + c]).  nthreads <= 0 uses the OpenMP default. */
int or_render_rows(const or_scene *s, float *out, int row0, int row1, int nthreads,
                   or_stats *stats);

/* Render the listed rows (any order) — the bounded CPU-baseline sample. */
int or_render_row_list(const or_scene *s, float *out, const int32_t *rows, int nrows,
                       int nthreads, or_stats *stats);

/* Sampler unit functions (KATs). */
float or_trilinear(const float *vol, int nx, int ny, int nz, float px, float py, float pz);
void or_tf_decode(const uint32_t *tf, int n, float *lut /* n*4 */);
void or_tf_sample(const uint32_t *tf, int n, float t, float out[4]);

/* Ray setup of one pixel: returns 1 if the pixel is covered by the cube's front face.
 * tex_out = in_tex_coords, frag_out = in_frag_position, dir_out = normalize(frag - cam). */
int or_pixel_ray(const or_scene *s, int px, int py, float tex_out[3], float frag_out[3],
                 float dir_out[3]);

/* The binary16 field's scale exponent (vr_internal.h field_scale_log2, restated): the largest
 * k in [-120, 120] with (max(vmax, 0) - min(vmin, 0)) 2^k <= 65504; 0 if that bound is 0 or
 * not finite. */
int or_field_scale_log2(float vmin, float vmax);
/* x rounded to binary16, round to nearest even, returned as float; |x| <= 65504 or NaN. */
float or_round_f16(float x);

/* Number of OpenMP threads this build would use by default. */
int or_max_threads(void);

#ifdef __cplusplus
}
#endif

#endif /* VR_ORACLE_H */
