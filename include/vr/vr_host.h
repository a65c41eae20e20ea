/*
 * vr_host.h — host-side inputs of the ray-march path (C ABI, CPU only, no HIP calls).
 *
 * These restate the reference components that FEED the replaced raycast pass, so a host
 * without the reference's SDL/ImGui/glm stack (tests, the benchmark, the CLI) produces the
 * same camera, transfer function and dataset the reference would hand to OffscreenPass:
 *   vr_cam_*       Vol::Scene::Camera           src/scene/camera.cpp:7-48 (glm quaternion math)
 *   vr_gradient_*  Vol::UI::Components::Gradient src/ui/components/gradient.cpp:64-108,471-515
 *                  + ImGui::ColorConvertFloat4ToU32 packing (R in the low byte)
 *   vr_nrrd_*      Vol::Data::NrrdFileParser     src/data/nrrd_file_parser.cpp:21-77 (own reader,
 *                  raw/ascii/hex encodings, detached .nhdr data files; gzip/bzip2 rejected as in
 *                  the reference's NrrdIO build without zlib)
 *   vr_csv_*       Vol::Data::CsvFileParser      src/data/csv_file_parser.cpp:14-50
 */
#ifndef VR_VR_HOST_H
#define VR_VR_HOST_H

#include <stddef.h>
#include <stdint.h>

#include "vr.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- orbit camera (camera.cpp) ---- */
typedef struct vr_orbit_camera {
    float center[3];
    float orientation[4]; /* quaternion (w, x, y, z) */
    float radius;
} vr_orbit_camera;

void vr_cam_init(vr_orbit_camera *c);                          /* Camera::Camera, :7-13 */
void vr_cam_rotate(vr_orbit_camera *c, float dx, float dy);    /* Camera::rotate, :15-29 */
void vr_cam_zoom(vr_orbit_camera *c, float delta);             /* Camera::zoom, :31-34 */
void vr_cam_position(const vr_orbit_camera *c, float out[3]);  /* get_position, :36-40 */
void vr_cam_view(const vr_orbit_camera *c, float out[16]);     /* get_view, :42-48 */
/* Fill a vr_camera (view + position, default projection constants) from the orbit camera. */
void vr_cam_to_camera(const vr_orbit_camera *c, vr_camera *out);

/* ---- transfer-function gradient editor model (gradient.cpp) ---- */
typedef struct vr_gradient vr_gradient;
vr_gradient *vr_gradient_create(void); /* black->white, alpha 1 -> 1 (:64-70) */
void vr_gradient_destroy(vr_gradient *g);
/* add_marker (:487-504): returns the insertion index, or -1 */
int vr_gradient_add_color_marker(vr_gradient *g, float location, float r, float gr, float b);
int vr_gradient_add_alpha_marker(vr_gradient *g, float location, float a);
/* remove_marker (:506-515): first/last cannot be removed; returns 1 if removed */
int vr_gradient_remove_color_marker(vr_gradient *g, size_t index);
int vr_gradient_remove_alpha_marker(vr_gradient *g, size_t index);
/* Edit marker `index` in place as the marker editor does (opacity/colour field, location
 * drag; gradient.cpp:337-432, 637-658): the first and last markers keep their location
 * (locked, :386-400); the edited marker is then shuffled to keep the list sorted
 * (:577-593).  Returns the marker's new index, or -1 for a bad index. */
int vr_gradient_set_alpha_marker(vr_gradient *g, size_t index, float location, float a);
int vr_gradient_set_color_marker(vr_gradient *g, size_t index, float location, float r,
                                 float gr, float b);
size_t vr_gradient_marker_count(const vr_gradient *g, int alpha);
/* sample (:81-87) -> RGBA float */
void vr_gradient_sample(const vr_gradient *g, float location, float out[4]);
/* discretize (:90-108): count texels, RGBA8 packed, R low byte */
int vr_gradient_discretize(const vr_gradient *g, size_t count, uint32_t *out);

/* ---- dataset loaders ---- */
typedef struct vr_dataset {
    uint32_t dims[3];   /* axis 0 fastest */
    int dtype;          /* enum vr_dtype of the file's elements */
    void *data;         /* native elements, host byte order, dims[0]*dims[1]*dims[2] */
    float vmin, vmax;   /* over static_cast<float>(element), as Dataset.min/max */
} vr_dataset;

/* Returns 0, or -1 "Failed to read file", -2 "Invalid file properties" (dim != 3),
 * -3 unsupported element type / encoding; message via vr_host_last_error(). */
int vr_nrrd_load(const char *path, vr_dataset *out);
/* Write a raw-encoded detached NRRD pair (path.nhdr + path.raw) from native data. */
int vr_nrrd_write_raw(const char *nhdr_path, const void *data, int dtype, const uint32_t dims[3]);
/* CSV slices, one file per z (csv_file_parser.cpp): float data, min/max seeded at 0. */
int vr_csv_load(const char *const *paths, size_t npaths, vr_dataset *out);
void vr_dataset_free(vr_dataset *d);
const char *vr_host_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* VR_VR_HOST_H */
