/*
 * oracle.c — CPU restatement of the reference ray-march.  TEST INFRASTRUCTURE ONLY:
 * loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline; never by the
 * product library.  See oracle.h for what it restates and its parity status.
 *
 * Build: oracle/Makefile (gcc -O2 -fopenmp -ffp-contract=off -mfma).  Contraction is OFF:
 * every fused multiply-add below is an explicit fmaf(), so the HIP kernel (built with the
 * same rule) performs the same IEEE operations in the same order.
 */
#include "oracle.h"

#include <math.h>
#include <stddef.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------------ */
/* glm restatements (float), as used by offscreen_pass.cpp:1158-1167.                    */
/* Matrices are column-major: m[col*4 + row].                                            */
/* ------------------------------------------------------------------------------------ */

/* glm operator*(mat4, mat4): Result[j] = A0*B[j][0] + A1*B[j][1] + A2*B[j][2] + A3*B[j][3] */
static void glm_mul(const float *a, const float *b, float *r)
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
    memcpy(r, t, sizeof(t));
}

/* glm::perspectiveRH_NO (offscreen_pass.cpp:1166; GLM_FORCE_DEPTH_ZERO_TO_ONE is defined
 * after glm was first included via offscreen_pass.h:3, so the [-1,1] form is in effect). */
static void glm_perspective_rh_no(float fovy, float aspect, float zn, float zf, float *m)
{
    memset(m, 0, 16 * sizeof(float));
    float th = tanf(fovy / 2.0f);
    m[0 * 4 + 0] = 1.0f / (aspect * th);
    m[1 * 4 + 1] = 1.0f / th;
    m[2 * 4 + 2] = -(zf + zn) / (zf - zn);
    m[2 * 4 + 3] = -1.0f;
    m[3 * 4 + 2] = -(2.0f * zf * zn) / (zf - zn);
}

/* glm::perspectiveRH_ZO: the form GLM_FORCE_DEPTH_ZERO_TO_ONE selects (OR_CONF_CLIP_ZO: the
 * define at offscreen_pass.cpp:3 taking effect after all; the product's
 * vr_params.depth_zero_to_one = 1). */
static void glm_perspective_rh_zo(float fovy, float aspect, float zn, float zf, float *m)
{
    memset(m, 0, 16 * sizeof(float));
    float th = tanf(fovy / 2.0f);
    m[0 * 4 + 0] = 1.0f / (aspect * th);
    m[1 * 4 + 1] = 1.0f / th;
    m[2 * 4 + 2] = zf / (zn - zf);
    m[2 * 4 + 3] = -1.0f;
    m[3 * 4 + 2] = -(zf * zn) / (zf - zn);
}

/* coordinate_conversion = rotate(I, radians(90), x) * scale(I, (-1,1,1)), glm float math
 * (offscreen_pass.cpp:1159-1162). */
static void coordinate_conversion(float *m)
{
    const float angle = 90.0f * 0.01745329251994329576923690768489f; /* glm::radians */
    const float c = cosf(angle), s = sinf(angle);
    const float ax = 1.0f, ay = 0.0f, az = 0.0f; /* normalize((1,0,0)) */
    const float tx = (1.0f - c) * ax, ty = (1.0f - c) * ay, tz = (1.0f - c) * az;
    float rot[16] = {0};
    rot[0 * 4 + 0] = c + tx * ax;
    rot[0 * 4 + 1] = tx * ay + s * az;
    rot[0 * 4 + 2] = tx * az - s * ay;
    rot[1 * 4 + 0] = ty * ax - s * az;
    rot[1 * 4 + 1] = c + ty * ay;
    rot[1 * 4 + 2] = ty * az + s * ax;
    rot[2 * 4 + 0] = tz * ax + s * ay;
    rot[2 * 4 + 1] = tz * ay - s * ax;
    rot[2 * 4 + 2] = c + tz * az;
    rot[3 * 4 + 3] = 1.0f;
    float sc[16] = {0};
    sc[0] = -1.0f;
    sc[5] = 1.0f;
    sc[10] = 1.0f;
    sc[15] = 1.0f;
    glm_mul(rot, sc, m);
}

/* Inverse of a 4x4 column-major matrix in double (cofactor expansion, fixed order). */
static int inverse4d(const double *m, double *inv)
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
    double det = m[0] * a[0] + m[1] * a[4] + m[2] * a[8] + m[3] * a[12];
    if (det == 0.0) return 0;
    double id = 1.0 / det;
    for (int i = 0; i < 16; ++i) inv[i] = a[i] * id;
    return 1;
}

/* Per-frame unprojection: inverse of the float matrix (proj * view) that volume.vert:23
 * applies ((proj*view)*v), in double. */
typedef struct ray_frame {
    double inv[16];
    int ok;
    /* OR_CONF_RASTER: window coordinates of the cube's 24 vertices in 2^-8 pixel units, their
     * clip w, which of the 12 triangles face the camera, twice their signed window area */
    int raster, raster_bad;
    int64_t sx[24], sy[24];
    float w[24];
    int front[12];
    int64_t area[12];
} ray_frame;

/* The cube of offscreen_pass.cpp:55-90 as faces: 4 vertices each in the table's order (tex =
 * position + 0.5), indexed {0,1,2, 0,2,3} per face (:87-89).  Face f: axis, side of the
 * constant coordinate, and the (u, v) axes walked by its 4 vertices. */
static const int CUBE_FACE[6][2] = {{2, +1}, {1, -1}, {0, +1}, {1, +1}, {0, -1}, {2, -1}};
static const float CUBE_VERT[24][3] = {
    {-0.5f, -0.5f, 0.5f}, {0.5f, -0.5f, 0.5f}, {0.5f, 0.5f, 0.5f}, {-0.5f, 0.5f, 0.5f},
    {-0.5f, -0.5f, -0.5f}, {0.5f, -0.5f, -0.5f}, {0.5f, -0.5f, 0.5f}, {-0.5f, -0.5f, 0.5f},
    {0.5f, -0.5f, -0.5f}, {0.5f, 0.5f, -0.5f}, {0.5f, 0.5f, 0.5f}, {0.5f, -0.5f, 0.5f},
    {0.5f, 0.5f, -0.5f}, {-0.5f, 0.5f, -0.5f}, {-0.5f, 0.5f, 0.5f}, {0.5f, 0.5f, 0.5f},
    {-0.5f, 0.5f, -0.5f}, {-0.5f, -0.5f, -0.5f}, {-0.5f, -0.5f, 0.5f}, {-0.5f, 0.5f, 0.5f},
    {-0.5f, 0.5f, -0.5f}, {0.5f, 0.5f, -0.5f}, {0.5f, -0.5f, -0.5f}, {-0.5f, -0.5f, -0.5f},
};
static inline int cube_index(int t, int k)
{
    static const int q[6] = {0, 1, 2, 0, 2, 3};
    return (t / 2) * 4 + q[(t % 2) * 3 + k];
}

static void make_raster(const or_scene *s, const float *pv, ray_frame *f)
{
    f->raster = 1;
    f->raster_bad = 0;
    const float W = (float)s->width, H = (float)s->height;
    float cz[24];
    for (int v = 0; v < 24; ++v) {
        /* volume.vert:23 gl_Position = (proj * view) * vec4(in_position, 1): glm mat * vec */
        float c[4];
        for (int r = 0; r < 4; ++r) {
            float acc = pv[0 * 4 + r] * CUBE_VERT[v][0];
            acc = acc + pv[1 * 4 + r] * CUBE_VERT[v][1];
            acc = acc + pv[2 * 4 + r] * CUBE_VERT[v][2];
            acc = acc + pv[3 * 4 + r];
            c[r] = acc;
        }
        f->w[v] = c[3];
        cz[v] = c[2];
        /* viewport (0, 0, W, H): xf = W/2 * xd + W/2 (Vulkan "Controlling the Viewport"),
         * snapped to the 2^-8 sub-pixel grid */
        const float xf = (W * 0.5f) * (c[0] / c[3]) + W * 0.5f;
        const float yf = (H * 0.5f) * (c[1] / c[3]) + H * 0.5f;
        f->sx[v] = llrintf(xf * 256.0f);
        f->sy[v] = llrintf(yf * 256.0f);
    }
    for (int t = 0; t < 12; ++t) {
        const int face = t / 2, ax = CUBE_FACE[face][0], side = CUBE_FACE[face][1];
        /* back-face cull (offscreen_pass.cpp:680-681); the object-space facing test equals the
         * window-area sign for every non-degenerate triangle */
        f->front[t] = (float)side * s->cam_pos[ax] > 0.5f;
        const int a = cube_index(t, 0), b = cube_index(t, 1), c = cube_index(t, 2);
        f->area[t] = (f->sx[b] - f->sx[a]) * (f->sy[c] - f->sy[a]) -
                     (f->sy[b] - f->sy[a]) * (f->sx[c] - f->sx[a]);
        if (f->front[t])
            for (int k = 0; k < 3; ++k) {
                const int v = cube_index(t, k);
                if (!(f->w[v] > 0.0f) || cz[v] < 0.0f || cz[v] > f->w[v]) f->raster_bad = 1;
            }
    }
}

static void make_ray_frame(const or_scene *s, ray_frame *f)
{
    float fovy = (s->fovy_deg > 0.0f ? s->fovy_deg : 40.0f) * 0.01745329251994329576923690768489f;
    float zn = s->znear > 0.0f ? s->znear : 0.1f;
    float zf = s->zfar > 0.0f ? s->zfar : 10.0f;
    float aspect = (float)s->width / (float)s->height;
    float persp[16], conv[16], proj[16], pv[16];
    if (s->conf_flags & OR_CONF_CLIP_ZO)
        glm_perspective_rh_zo(fovy, aspect, zn, zf, persp);
    else
        glm_perspective_rh_no(fovy, aspect, zn, zf, persp);
    coordinate_conversion(conv);
    glm_mul(persp, conv, proj);
    glm_mul(proj, s->view, pv);
    double pvd[16];
    for (int i = 0; i < 16; ++i) pvd[i] = (double)pv[i];
    f->ok = inverse4d(pvd, f->inv);
    f->raster = 0;
    f->raster_bad = 0;
    if (s->conf_flags & OR_CONF_RASTER) make_raster(s, pv, f);
}

/* volume.frag:23 ray_dir = normalize(in_frag_position - camera_position) */
static void ray_direction(const or_scene *s, const float frag[3], float dir[3])
{
    float vx = frag[0] - s->cam_pos[0];
    float vy = frag[1] - s->cam_pos[1];
    float vz = frag[2] - s->cam_pos[2];
    float len2 = vx * vx + vy * vy + vz * vz;
    if (s->conf_flags & OR_CONF_GPU_MATH) {
        const float rs = (float)(1.0 / sqrt((double)len2)); /* correctly rounded rsqrt */
        dir[0] = vx * rs;
        dir[1] = vy * rs;
        dir[2] = vz * rs;
        return;
    }
    float len = sqrtf(len2);
    dir[0] = vx / len;
    dir[1] = vy / len;
    dir[2] = vz / len;
}

/* OR_CONF_RASTER: the front triangle covering the pixel centre (exact integer edge functions
 * on the snapped grid; a sample exactly on an edge belongs to the triangle for which that edge
 * is a "top-left" one, so a shared edge is covered once) and its perspective-correct
 * attributes, f = sum(l_k f_k / w_k) / sum(l_k / w_k) in float. */
static int pixel_ray_raster(const or_scene *s, const ray_frame *f, int px, int py, float tex[3],
                            float frag[3], float dir[3])
{
    const int64_t X = (int64_t)px * 256 + 128, Y = (int64_t)py * 256 + 128;
    for (int t = 0; t < 12; ++t) {
        if (!f->front[t] || f->area[t] == 0) continue;
        int v[3] = {cube_index(t, 0), cube_index(t, 1), cube_index(t, 2)};
        int64_t area = f->area[t];
        if (area < 0) {
            const int tmp = v[1];
            v[1] = v[2];
            v[2] = tmp;
            area = -area;
        }
        int64_t e[3];
        int inside = 1;
        for (int k = 0; k < 3 && inside; ++k) {
            const int a = v[(k + 1) % 3], b = v[(k + 2) % 3]; /* the edge opposite vertex k */
            const int64_t dx = f->sx[b] - f->sx[a], dy = f->sy[b] - f->sy[a];
            e[k] = dx * (Y - f->sy[a]) - dy * (X - f->sx[a]);
            if (e[k] < 0 || (e[k] == 0 && !(dy < 0 || (dy == 0 && dx > 0)))) inside = 0;
        }
        if (!inside) continue;
        float a[3], sum = 0.0f;
        for (int k = 0; k < 3; ++k) {
            a[k] = ((float)e[k] / (float)area) / f->w[v[k]];
            sum = sum + a[k];
        }
        for (int c = 0; c < 3; ++c) {
            float fp = a[0] * CUBE_VERT[v[0]][c];
            fp = fp + a[1] * CUBE_VERT[v[1]][c];
            fp = fp + a[2] * CUBE_VERT[v[2]][c];
            float tc = a[0] * (CUBE_VERT[v[0]][c] + 0.5f);
            tc = tc + a[1] * (CUBE_VERT[v[1]][c] + 0.5f);
            tc = tc + a[2] * (CUBE_VERT[v[2]][c] + 0.5f);
            frag[c] = fp / sum;
            tex[c] = tc / sum;
        }
        ray_direction(s, frag, dir);
        return 1;
    }
    return 0;
}

/* Ray entry of one pixel: the cube's camera-facing face hit by the pixel-centre ray,
 * inside the Vulkan clip volume 0 <= z_ndc <= 1 (back faces culled, :680-681; clipped
 * front faces leave the clear colour).  Returns 1 if covered. */
static int pixel_ray(const or_scene *s, const ray_frame *f, int px, int py, float tex[3],
                     float frag[3], float dir[3])
{
    if (f->raster) return pixel_ray_raster(s, f, px, py, tex, frag, dir);
    if (!f->ok) return 0;
    const double *m = f->inv;
    double x = ((double)px + 0.5) / (double)s->width * 2.0 - 1.0;
    double y = ((double)py + 0.5) / (double)s->height * 2.0 - 1.0;
    double h0[4], h1[4];
    for (int r = 0; r < 4; ++r) {
        h0[r] = m[0 * 4 + r] * x + m[1 * 4 + r] * y + m[3 * 4 + r];
        h1[r] = h0[r] + m[2 * 4 + r];
    }
    double p0[3], d[3];
    for (int r = 0; r < 3; ++r) {
        p0[r] = h0[r] / h0[3];
        d[r] = h1[r] / h1[3] - p0[r];
    }
    double te = -INFINITY, tx = INFINITY;
    int axis = 0;
    for (int a = 0; a < 3; ++a) {
        double lo, hi;
        if (d[a] == 0.0) {
            if (p0[a] < -0.5 || p0[a] > 0.5) return 0;
            lo = -INFINITY;
            hi = INFINITY;
        } else {
            double t1 = (-0.5 - p0[a]) / d[a];
            double t2 = (0.5 - p0[a]) / d[a];
            lo = t1 < t2 ? t1 : t2;
            hi = t1 < t2 ? t2 : t1;
        }
        if (lo > te) {
            te = lo;
            axis = a;
        }
        if (hi < tx) tx = hi;
    }
    if (!(te < tx) || te < 0.0 || te > 1.0) return 0;
    for (int a = 0; a < 3; ++a) {
        double e = p0[a] + te * d[a];
        frag[a] = (float)e;
        tex[a] = (float)(e + 0.5);
    }
    frag[axis] = d[axis] > 0.0 ? -0.5f : 0.5f;
    tex[axis] = d[axis] > 0.0 ? 0.0f : 1.0f;
    ray_direction(s, frag, dir);
    return 1;
}

int or_pixel_ray(const or_scene *s, int px, int py, float tex_out[3], float frag_out[3],
                 float dir_out[3])
{
    ray_frame f;
    make_ray_frame(s, &f);
    return pixel_ray(s, &f, px, py, tex_out, frag_out, dir_out);
}

/* ------------------------------------------------------------------------------------ */
/* Samplers                                                                              */
/* ------------------------------------------------------------------------------------ */

static inline float lerpf(float a, float b, float w) { return fmaf(w, b - a, a); }

/* R32_SFLOAT 3D image, CLAMP_TO_BORDER with TRANSPARENT_BLACK (offscreen_pass.cpp:968,
 * 1016-1031): texels outside [0,N) read 0. */
/* The Dataset's voxels: dense float (the reference's vector<float>), or u8 for the multi-GiB
 * u8 configurations (C5: 8 GiB instead of a 32 GiB float copy; float(u8) is exact, so the
 * samples are the same). */
typedef struct vsrc {
    const float *f;
    const uint8_t *u8;
} vsrc;

static inline float voxel(const vsrc *v, int nx, int ny, int nz, int x, int y, int z)
{
    if (x < 0 || y < 0 || z < 0 || x >= nx || y >= ny || z >= nz) return 0.0f;
    const size_t i = (size_t)x + (size_t)nx * ((size_t)y + (size_t)ny * (size_t)z);
    return v->u8 ? (float)v->u8[i] : v->f[i];
}

/* Trilinear filter of the 2x2x2 cell whose low corner is (i,j,k), weights (ax,ay,az):
 * lerp along x, then y, then z. */
static inline float tri_cell(const vsrc *v, int nx, int ny, int nz, int i, int j, int k,
                             float ax, float ay, float az)
{
    float c00 = lerpf(voxel(v, nx, ny, nz, i, j, k), voxel(v, nx, ny, nz, i + 1, j, k), ax);
    float c10 = lerpf(voxel(v, nx, ny, nz, i, j + 1, k), voxel(v, nx, ny, nz, i + 1, j + 1, k), ax);
    float c01 = lerpf(voxel(v, nx, ny, nz, i, j, k + 1), voxel(v, nx, ny, nz, i + 1, j, k + 1), ax);
    float c11 = lerpf(voxel(v, nx, ny, nz, i, j + 1, k + 1),
                      voxel(v, nx, ny, nz, i + 1, j + 1, k + 1), ax);
    float c0 = lerpf(c00, c10, ay);
    float c1 = lerpf(c01, c11, ay);
    return lerpf(c0, c1, az);
}

/* Gradient extension: trilinear filter (same cell, weights and lerp order as tri_cell) of
 * the per-voxel central difference D_e(c) = v(c + e) - v(c - e) along axis e, i.e.
 * tri(v(. + e)) - tri(v(. - e)) with the subtraction done per voxel: one rounding per
 * difference, then the filter.  (The device reads D from precomputed arrays for f32 volumes
 * and forms it from the 4-wide stencil otherwise; same operations either way.) */
static inline float dvox(const vsrc *v, int nx, int ny, int nz, int x, int y, int z, int axis)
{
    const int ex = axis == 0, ey = axis == 1, ez = axis == 2;
    return voxel(v, nx, ny, nz, x + ex, y + ey, z + ez) - voxel(v, nx, ny, nz, x - ex, y - ey, z - ez);
}
static inline float grad_cell(const vsrc *v, int nx, int ny, int nz, int i, int j, int k,
                              float ax, float ay, float az, int axis)
{
    float c00 = lerpf(dvox(v, nx, ny, nz, i, j, k, axis), dvox(v, nx, ny, nz, i + 1, j, k, axis), ax);
    float c10 = lerpf(dvox(v, nx, ny, nz, i, j + 1, k, axis),
                      dvox(v, nx, ny, nz, i + 1, j + 1, k, axis), ax);
    float c01 = lerpf(dvox(v, nx, ny, nz, i, j, k + 1, axis),
                      dvox(v, nx, ny, nz, i + 1, j, k + 1, axis), ax);
    float c11 = lerpf(dvox(v, nx, ny, nz, i, j + 1, k + 1, axis),
                      dvox(v, nx, ny, nz, i + 1, j + 1, k + 1, axis), ax);
    float c0 = lerpf(c00, c10, ay);
    float c1 = lerpf(c01, c11, ay);
    return lerpf(c0, c1, az);
}

/* The device's binary16 difference field (extension, vr_params.exact_gradient == 0; the
 * kernel's field_half): D * 2^k clamped to +-65504 (NaN passes), rounded to the nearest
 * binary16, ties to even, subnormals kept. */
int or_field_scale_log2(float vmin, float vmax)
{
    const double B = (double)(vmax > 0.0f ? vmax : 0.0f) - (double)(vmin < 0.0f ? vmin : 0.0f);
    if (!(B > 0.0) || B > 1e300) return 0;
    int k = 0;
    while (k > -120 && B * ldexp(1.0, k) > 65504.0) --k;
    while (k < 120 && B * ldexp(1.0, k + 1) <= 65504.0) ++k;
    return k;
}

float or_round_f16(float x)
{
    if (x != x) return x;
    const float a = fabsf(x);
    float r;
    if (a < 6.103515625e-05f) {            /* below 2^-14: binary16 subnormals, step 2^-24 */
        r = rintf(a * 16777216.0f) * 5.9604644775390625e-08f;
    } else {                               /* normal: keep 10 of the 23 mantissa bits */
        uint32_t u;
        memcpy(&u, &a, sizeof u);
        u += 0x0FFFu + ((u >> 13) & 1u);   /* round to nearest, ties to even */
        u &= ~0x1FFFu;
        memcpy(&r, &u, sizeof r);
    }
    return copysignf(r, x);
}

static inline float dvox_f16(const vsrc *v, int nx, int ny, int nz, int x, int y, int z, int axis,
                             float scale)
{
    float d = dvox(v, nx, ny, nz, x, y, z, axis) * scale;
    d = d > 65504.0f ? 65504.0f : (d < -65504.0f ? -65504.0f : d);
    return or_round_f16(d);
}
static inline float grad_cell_f16(const vsrc *v, int nx, int ny, int nz, int i, int j, int k,
                                  float ax, float ay, float az, int axis, float scale)
{
#define DV(x, y, z) dvox_f16(v, nx, ny, nz, x, y, z, axis, scale)
    float c00 = lerpf(DV(i, j, k), DV(i + 1, j, k), ax);
    float c10 = lerpf(DV(i, j + 1, k), DV(i + 1, j + 1, k), ax);
    float c01 = lerpf(DV(i, j, k + 1), DV(i + 1, j, k + 1), ax);
    float c11 = lerpf(DV(i, j + 1, k + 1), DV(i + 1, j + 1, k + 1), ax);
#undef DV
    float c0 = lerpf(c00, c10, ay);
    float c1 = lerpf(c01, c11, ay);
    return lerpf(c0, c1, az);
}

/* Normalised coordinate -> texel space: u = s*N - 0.5 (texel i's centre at (i+0.5)/N). */
/* Conformance variant conf_weight_bits = b > 0: u on the 2^-b grid (subTexelPrecisionBits),
 * round to nearest even, so floor(u) and frac(u) come from the quantised coordinate. */
static inline float quantise_u(float u, int bits)
{
    return bits > 0 ? ldexpf(rintf(ldexpf(u, bits)), -bits) : u;
}

static inline void texel_coord_q(float p, int n, int bits, int *i, float *a)
{
    float u = quantise_u(p * (float)n - 0.5f, bits);
    float f = floorf(u);
    *a = u - f;
    *i = (int)f;
}

static inline void texel_coord(float p, int n, int *i, float *a)
{
    float u = p * (float)n - 0.5f;
    float f = floorf(u);
    *a = u - f;
    *i = (int)f;
}

float or_trilinear(const float *vol, int nx, int ny, int nz, float px, float py, float pz)
{
    /* keep the integer conversion defined far outside the box (KAT helper only) */
    px = fminf(fmaxf(px, -1.0f), 2.0f);
    py = fminf(fmaxf(py, -1.0f), 2.0f);
    pz = fminf(fmaxf(pz, -1.0f), 2.0f);
    int i, j, k;
    float ax, ay, az;
    texel_coord(px, nx, &i, &ax);
    texel_coord(py, ny, &j, &ay);
    texel_coord(pz, nz, &k, &az);
    const vsrc src = {vol, NULL};
    return tri_cell(&src, nx, ny, nz, i, j, k, ax, ay, az);
}

/* R8G8B8A8_SRGB texels (offscreen_pass.cpp:1076): RGB UNORM-decoded then sRGB->linear
 * BEFORE filtering; A linear c/255. */
static float srgb_to_linear(uint32_t c8)
{
    double c = (double)c8 / 255.0;
    double l = c <= 0.04045 ? c / 12.92 : pow((c + 0.055) / 1.055, 2.4);
    return (float)l;
}

void or_tf_decode(const uint32_t *tf, int n, float *lut)
{
    for (int i = 0; i < n; ++i) {
        uint32_t t = tf[i];
        lut[i * 4 + 0] = srgb_to_linear(t & 0xFFu);
        lut[i * 4 + 1] = srgb_to_linear((t >> 8) & 0xFFu);
        lut[i * 4 + 2] = srgb_to_linear((t >> 16) & 0xFFu);
        lut[i * 4 + 3] = (float)((t >> 24) & 0xFFu) / 255.0f;
    }
}

/* 1D LINEAR filter, CLAMP_TO_EDGE (offscreen_pass.cpp:1125-1150).  The clamp of u to
 * [-1, n] keeps the float->int conversion defined for t = +-inf/NaN (min == max). */
static inline void tf_lookup_q(const float *lut, int n, float t, int bits, float out[4])
{
    float u = t * (float)n - 0.5f;
    u = fminf(fmaxf(u, -1.0f), (float)n);
    u = quantise_u(u, bits);
    float f = floorf(u);
    float w = u - f;
    int i0 = (int)f, i1 = i0 + 1;
    i0 = i0 < 0 ? 0 : (i0 > n - 1 ? n - 1 : i0);
    i1 = i1 < 0 ? 0 : (i1 > n - 1 ? n - 1 : i1);
    for (int c = 0; c < 4; ++c) out[c] = lerpf(lut[i0 * 4 + c], lut[i1 * 4 + c], w);
}

static inline void tf_lookup(const float *lut, int n, float t, float out[4])
{
    float u = t * (float)n - 0.5f;
    u = fminf(fmaxf(u, -1.0f), (float)n);
    float f = floorf(u);
    float w = u - f;
    int i0 = (int)f, i1 = i0 + 1;
    i0 = i0 < 0 ? 0 : (i0 > n - 1 ? n - 1 : i0);
    i1 = i1 < 0 ? 0 : (i1 > n - 1 ? n - 1 : i1);
    for (int c = 0; c < 4; ++c) out[c] = lerpf(lut[i0 * 4 + c], lut[i1 * 4 + c], w);
}

void or_tf_sample(const uint32_t *tf, int n, float t, float out[4])
{
    float *lut = (float *)malloc((size_t)n * 4 * sizeof(float));
    or_tf_decode(tf, n, lut);
    tf_lookup(lut, n, t, out);
    free(lut);
}

/* ------------------------------------------------------------------------------------ */
/* The ray-march (volume.frag:21-52) + blend (offscreen_pass.cpp:715-725)                */
/* ------------------------------------------------------------------------------------ */

/* Specular power (extension): binary exponentiation, the kernel's operation sequence --
 * square the base once per remaining exponent bit, multiply it in for each set bit. */
static float powi(float x, int p)
{
    float r = 1.0f;
    while (p) {
        if (p & 1) r = r * x;
        p >>= 1;
        if (p) x = x * x;
    }
    return r;
}

/* conf = 0: the oracle (conformance fields ignored, the baseline's hot path unchanged);
 * conf = 1: the conformance variants of s->conf_weight_bits / s->conf_flags. */
static inline __attribute__((always_inline)) void
march_pixel_impl(const or_scene *s, const ray_frame *f, const float *lut, int px, int py,
                 float *out, or_stats *st, const int conf)
{
    float tex[3], frag[3], dir[3];
    if (!pixel_ray(s, f, px, py, tex, frag, dir)) {
        for (int c = 0; c < 4; ++c) out[c] = s->clear[c];
        return;
    }
    st->rays++;
    const int nx = s->nx, ny = s->ny, nz = s->nz;
    const vsrc src = {s->vol, s->vol_u8};
    const float step = s->step;
    const int nsteps = (int)(s->ray_dist / step); /* volume.frag:31 int(ray_dist/step_size) */
    const float range = s->vmax - s->vmin;
    float T = 1.0f, cr = 0.0f, cg = 0.0f, cb = 0.0f;
    float p0 = tex[0], p1 = tex[1], p2 = tex[2];
    for (int it = 0; it < nsteps; ++it) {
        /* volume.frag:34-37: break if any component > 1 or < 0 */
        if (p0 > 1.0f || p1 > 1.0f || p2 > 1.0f || p0 < 0.0f || p1 < 0.0f || p2 < 0.0f) break;
        st->steps++;
        /* volume.frag:39-40: strict slab test */
        if (p0 < s->smax[0] && p1 < s->smax[1] && p2 < s->smax[2] && p0 > s->smin[0] &&
            p1 > s->smin[1] && p2 > s->smin[2]) {
            int i, j, k;
            float ax, ay, az;
            const int qb = conf ? s->conf_weight_bits : 0;
            texel_coord_q(p0, nx, qb, &i, &ax);
            texel_coord_q(p1, ny, qb, &j, &ay);
            texel_coord_q(p2, nz, qb, &k, &az);
            const float d = tri_cell(&src, nx, ny, nz, i, j, k, ax, ay, az); /* :41 */
            const float t = (conf && (s->conf_flags & OR_CONF_GPU_MATH))
                                ? (d - s->vmin) * (float)(1.0 / (double)range)
                                : (d - s->vmin) / range; /* :42 */
            float sc[4];
            tf_lookup_q(lut, s->tf_n, t, qb, sc); /* :43 */
            st->samples++;
            if (s->shading && sc[3] > 0.0f) {
                /* extension: central differences one texel apart, same weights (grad_cell) */
                float gx, gy, gz;
                if (s->grad_f16) {
                    const float sc = ldexpf(1.0f, s->grad_range_set
                                                      ? or_field_scale_log2(s->grad_range[0], s->grad_range[1])
                                                      : or_field_scale_log2(s->vmin, s->vmax));
                    gx = grad_cell_f16(&src, nx, ny, nz, i, j, k, ax, ay, az, 0, sc);
                    gy = grad_cell_f16(&src, nx, ny, nz, i, j, k, ax, ay, az, 1, sc);
                    gz = grad_cell_f16(&src, nx, ny, nz, i, j, k, ax, ay, az, 2, sc);
                } else {
                    gx = grad_cell(&src, nx, ny, nz, i, j, k, ax, ay, az, 0);
                    gy = grad_cell(&src, nx, ny, nz, i, j, k, ax, ay, az, 1);
                    gz = grad_cell(&src, nx, ny, nz, i, j, k, ax, ay, az, 2);
                }
                st->shaded_samples++;
                const float wx = gx * (float)nx, wy = gy * (float)ny, wz = gz * (float)nz;
                const float g2 = wx * wx + wy * wy + wz * wz;
                if (g2 > 0.0f) {
                    const float inv = 1.0f / sqrtf(g2);
                    const float ndl = fabsf((wx * dir[0] + wy * dir[1] + wz * dir[2]) * inv);
                    const float kdiff = s->ka + s->kd * ndl;
                    const float spec = s->ks * powi(ndl, s->spec_power);
                    sc[0] = sc[0] * kdiff + spec;
                    sc[1] = sc[1] * kdiff + spec;
                    sc[2] = sc[2] * kdiff + spec;
                }
            }
            /* volume.frag:44-45  C.rgb += T * (s.a * s.rgb);  T *= 1 - s.a */
            if (conf && (s->conf_flags & OR_CONF_FMA)) {
                cr = fmaf(sc[0] * sc[3], T, cr);
                cg = fmaf(sc[1] * sc[3], T, cg);
                cb = fmaf(sc[2] * sc[3], T, cb);
            } else {
                cr = cr + (sc[0] * sc[3]) * T;
                cg = cg + (sc[1] * sc[3]) * T;
                cb = cb + (sc[2] * sc[3]) * T;
            }
            T = T * (1.0f - sc[3]);
            if (T == 0.0f) break; /* exact: later samples add (rgb*a)*0 */
            if (T < s->ert_eps) break;
        }
        /* volume.frag:47  ray_pos += ray_dir * step_size */
        if (conf && (s->conf_flags & OR_CONF_FMA)) {
            p0 = fmaf(dir[0], step, p0);
            p1 = fmaf(dir[1], step, p1);
            p2 = fmaf(dir[2], step, p2);
        } else {
            p0 = p0 + dir[0] * step;
            p1 = p1 + dir[1] * step;
            p2 = p2 + dir[2] * step;
        }
    }
    /* volume.frag:50 alpha = 1 - T; blend SRC_ALPHA / ONE_MINUS_SRC_ALPHA over clear */
    const float A = 1.0f - T;
    const float omA = 1.0f - A;
    out[0] = cr * A + s->clear[0] * omA;
    out[1] = cg * A + s->clear[1] * omA;
    out[2] = cb * A + s->clear[2] * omA;
    out[3] = A * A + s->clear[3] * omA;
}

static void march_pixel(const or_scene *s, const ray_frame *f, const float *lut, int px,
                        int py, float *out, or_stats *st)
{
    /* OR_CONF_CLIP_ZO only changes the ray frame (make_ray_frame): it is also the product's
     * vr_params.depth_zero_to_one (ABI 8), so it keeps the oracle's own march */
    if ((s->conf_flags & ~OR_CONF_CLIP_ZO) == 0 && s->conf_weight_bits == 0)
        march_pixel_impl(s, f, lut, px, py, out, st, 0);
    else
        march_pixel_impl(s, f, lut, px, py, out, st, 1);
}

int or_render_rows(const or_scene *s, float *out, int row0, int row1, int nthreads,
                   or_stats *stats)
{
    if (!s || !out || !(s->vol || s->vol_u8) || !s->tf || s->tf_n <= 0 || s->width <= 0 || s->height <= 0)
        return -22;
    if (row0 < 0) row0 = 0;
    if (row1 > s->height) row1 = s->height;
    ray_frame f;
    make_ray_frame(s, &f);
    if (f.raster_bad) return -95; /* OR_CONF_RASTER needs no near/far clipping */
    float *lut = (float *)malloc((size_t)s->tf_n * 4 * sizeof(float));
    if (!lut) return -12;
    or_tf_decode(s->tf, s->tf_n, lut);
    uint64_t rays = 0, samples = 0, shaded = 0, steps = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) \
    reduction(+ : rays, samples, shaded, steps)
#endif
    for (int y = row0; y < row1; ++y) {
        or_stats st = {0, 0, 0, 0};
        for (int x = 0; x < s->width; ++x)
            march_pixel(s, &f, lut, x, y, out + ((size_t)y * s->width + x) * 4, &st);
        rays += st.rays;
        samples += st.samples;
        shaded += st.shaded_samples;
        steps += st.steps;
    }
    free(lut);
    if (stats) {
        stats->rays = rays;
        stats->samples = samples;
        stats->shaded_samples = shaded;
        stats->steps = steps;
    }
    return 0;
}

int or_render_row_list(const or_scene *s, float *out, const int32_t *rows, int nrows,
                       int nthreads, or_stats *stats)
{
    if (!s || !out || !rows || !(s->vol || s->vol_u8) || !s->tf || s->tf_n <= 0 || s->width <= 0 || s->height <= 0)
        return -22;
    ray_frame f;
    make_ray_frame(s, &f);
    if (f.raster_bad) return -95; /* OR_CONF_RASTER needs no near/far clipping */
    float *lut = (float *)malloc((size_t)s->tf_n * 4 * sizeof(float));
    if (!lut) return -12;
    or_tf_decode(s->tf, s->tf_n, lut);
    uint64_t rays = 0, samples = 0, shaded = 0, steps = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) \
    reduction(+ : rays, samples, shaded, steps)
#endif
    for (int r = 0; r < nrows; ++r) {
        const int y = rows[r];
        if (y < 0 || y >= s->height) continue;
        or_stats st = {0, 0, 0, 0};
        for (int x = 0; x < s->width; ++x)
            march_pixel(s, &f, lut, x, y, out + ((size_t)y * s->width + x) * 4, &st);
        rays += st.rays;
        samples += st.samples;
        shaded += st.shaded_samples;
        steps += st.steps;
    }
    free(lut);
    if (stats) {
        stats->rays = rays;
        stats->samples = samples;
        stats->shaded_samples = shaded;
        stats->steps = steps;
    }
    return 0;
}

int or_max_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
