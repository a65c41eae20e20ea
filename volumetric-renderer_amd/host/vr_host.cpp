// vr_host.cpp — host-side inputs of the ray-march path (include/vr/vr_host.h).
//
// CPU-only restatements of the reference components that feed OffscreenPass: the orbit
// camera (src/scene/camera.cpp, glm quaternion math in float), the TF gradient model
// (src/ui/components/gradient.cpp + ImGui packing) and the dataset loaders
// (src/data/nrrd_file_parser.cpp via the build's own NRRD reader; src/data/csv_file_parser.cpp).
#include "../../include/vr/vr_host.h"

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <unistd.h>

namespace {

thread_local std::string g_host_err;

int herr(int code, const std::string &m)
{
    g_host_err = m;
    return code;
}

// ---------------------------------------------------------------------------------------
// glm restatements (float): quat (w, x, y, z), vec3, column-major mat4
// ---------------------------------------------------------------------------------------
struct Q {
    float w, x, y, z;
};
struct V3 {
    float x, y, z;
};

constexpr float kDegToRad = 0.01745329251994329576923690768489f;  // glm::radians

Q angle_axis(float angle, V3 v)  // glm::angleAxis: no normalisation of v
{
    const float s = std::sin(angle * 0.5f);
    return Q{std::cos(angle * 0.5f), v.x * s, v.y * s, v.z * s};
}

Q qmul(const Q &p, const Q &q)  // glm qua operator*
{
    Q r;
    r.w = p.w * q.w - p.x * q.x - p.y * q.y - p.z * q.z;
    r.x = p.w * q.x + p.x * q.w + p.y * q.z - p.z * q.y;
    r.y = p.w * q.y + p.y * q.w + p.z * q.x - p.x * q.z;
    r.z = p.w * q.z + p.z * q.w + p.x * q.y - p.y * q.x;
    return r;
}

V3 cross(V3 a, V3 b)
{
    return V3{a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}

V3 qrot(const Q &q, V3 v)  // glm qua * vec3
{
    const V3 qv{q.x, q.y, q.z};
    const V3 uv = cross(qv, v);
    const V3 uuv = cross(qv, uv);
    return V3{v.x + ((uv.x * q.w) + uuv.x) * 2.0f, v.y + ((uv.y * q.w) + uuv.y) * 2.0f,
              v.z + ((uv.z * q.w) + uuv.z) * 2.0f};
}

void mat4_cast(const Q &q, float *m)  // glm::mat4_cast
{
    const float qxx = q.x * q.x, qyy = q.y * q.y, qzz = q.z * q.z;
    const float qxz = q.x * q.z, qxy = q.x * q.y, qyz = q.y * q.z;
    const float qwx = q.w * q.x, qwy = q.w * q.y, qwz = q.w * q.z;
    std::memset(m, 0, 16 * sizeof(float));
    m[0] = 1.0f - 2.0f * (qyy + qzz);
    m[1] = 2.0f * (qxy + qwz);
    m[2] = 2.0f * (qxz - qwy);
    m[4] = 2.0f * (qxy - qwz);
    m[5] = 1.0f - 2.0f * (qxx + qzz);
    m[6] = 2.0f * (qyz + qwx);
    m[8] = 2.0f * (qxz + qwy);
    m[9] = 2.0f * (qyz - qwx);
    m[10] = 1.0f - 2.0f * (qxx + qyy);
    m[15] = 1.0f;
}

void mat_mul(const float *a, const float *b, float *r)  // glm mat4 operator*
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

Q load_q(const vr_orbit_camera *c)
{
    return Q{c->orientation[0], c->orientation[1], c->orientation[2], c->orientation[3]};
}
void store_q(vr_orbit_camera *c, const Q &q)
{
    c->orientation[0] = q.w;
    c->orientation[1] = q.x;
    c->orientation[2] = q.y;
    c->orientation[3] = q.z;
}

// ---------------------------------------------------------------------------------------
// Gradient (gradient.cpp)
// ---------------------------------------------------------------------------------------
template <typename T>
struct Marker {
    float location;
    T value;
};
struct RGB {
    float r, g, b;
};

RGB lerp(const RGB &a, const RGB &b, float t)  // a * (1 - t) + b * t (gradient.cpp:14-17)
{
    return RGB{a.r * (1.0f - t) + b.r * t, a.g * (1.0f - t) + b.g * t,
               a.b * (1.0f - t) + b.b * t};
}
float lerp(float a, float b, float t) { return a * (1.0f - t) + b * t; }

template <typename T>
typename std::vector<Marker<T>>::const_iterator lower(const std::vector<Marker<T>> &m, float loc)
{
    return std::lower_bound(m.begin(), m.end(), loc,
                            [](const Marker<T> &a, float l) { return a.location < l; });
}

template <typename T>
T sample_markers(const std::vector<Marker<T>> &markers, float location)  // :471-485
{
    location = std::clamp(location, 0.0f, 1.0f);
    auto it = lower(markers, location);
    if (it == markers.begin()) return it->value;
    if (it == markers.end()) return markers.back().value;
    const float curr = it->location, prev = (it - 1)->location;
    const float t = (location - prev) / (curr - prev);
    return lerp((it - 1)->value, it->value, t);
}

template <typename T>
int add_marker(std::vector<Marker<T>> &markers, float location, const T &value)  // :487-504
{
    location = std::clamp(location, 0.0f, 1.0f);
    auto it = std::lower_bound(markers.begin(), markers.end(), location,
                               [](const Marker<T> &a, float l) { return a.location < l; });
    if (it == markers.begin()) it++;
    if (it == markers.end()) it = markers.end() - 1;
    const size_t index = (size_t)std::distance(markers.begin(), it);
    markers.insert(it, Marker<T>{location, value});
    return (int)index;
}

template <typename T>
int remove_marker(std::vector<T> &markers, size_t index)  // :506-515
{
    if (index >= markers.size()) return 0;
    auto it = markers.begin() + (long)index;
    if (it == markers.begin() || it == markers.end() - 1) return 0;
    markers.erase(it);
    return 1;
}

// update_markers' re-sort (gradient.cpp:577-593): shuffle the selected marker down/up, never
// past the first or last marker.
template <typename T>
size_t keep_sorted(std::vector<Marker<T>> &markers, size_t sel)
{
    const Marker<T> marker = markers[sel];
    while (sel > 1 && marker.location < markers[sel - 1].location) {
        markers[sel] = markers[sel - 1];
        sel--;
    }
    while (markers.size() >= 2 && sel < markers.size() - 2 &&
           marker.location > markers[sel + 1].location) {
        markers[sel] = markers[sel + 1];
        sel++;
    }
    markers[sel] = marker;
    return sel;
}

template <typename T>
int set_marker(std::vector<Marker<T>> &markers, size_t index, float location, const T &value)
{
    if (index >= markers.size()) return -1;
    markers[index].value = value;
    const bool locked = index == 0 || index == markers.size() - 1;
    if (!locked) markers[index].location = std::clamp(location, 0.0f, 1.0f);
    return (int)keep_sorted(markers, index);
}

inline float saturate(float f) { return (f < 0.0f) ? 0.0f : (f > 1.0f) ? 1.0f : f; }
inline uint32_t f32_to_int8_sat(float v) { return (uint32_t)(int)(saturate(v) * 255.0f + 0.5f); }

}  // namespace

struct vr_gradient {
    std::vector<Marker<RGB>> color{{0.0f, RGB{0.0f, 0.0f, 0.0f}}, {1.0f, RGB{1.0f, 1.0f, 1.0f}}};
    std::vector<Marker<float>> alpha{{0.0f, 1.0f}, {1.0f, 1.0f}};
};

extern "C" {

const char *vr_host_last_error(void) { return g_host_err.c_str(); }

// ---- camera.cpp ----
void vr_cam_init(vr_orbit_camera *c)
{
    c->center[0] = c->center[1] = c->center[2] = 0.0f;
    store_q(c, angle_axis(180.0f * kDegToRad, V3{0.0f, 0.0f, 1.0f}));
    c->radius = 3.0f;
}

void vr_cam_rotate(vr_orbit_camera *c, float dx, float dy)
{
    const float ax = dx * 0.25f, ay = dy * 0.25f;
    Q o = load_q(c);
    const Q yaw = angle_axis((-ax) * kDegToRad, V3{0.0f, 0.0f, 1.0f});
    o = qmul(yaw, o);
    const V3 right = qrot(o, V3{1.0f, 0.0f, 0.0f});
    const Q pitch = angle_axis(ay * kDegToRad, right);
    o = qmul(pitch, o);
    store_q(c, o);
}

void vr_cam_zoom(vr_orbit_camera *c, float delta)
{
    c->radius = std::clamp(c->radius - delta, 0.1f, 10.0f);
}

void vr_cam_position(const vr_orbit_camera *c, float out[3])
{
    const V3 fwd = qrot(load_q(c), V3{0.0f, -1.0f, 0.0f});
    out[0] = c->center[0] + c->radius * -fwd.x;
    out[1] = c->center[1] + c->radius * -fwd.y;
    out[2] = c->center[2] + c->radius * -fwd.z;
}

void vr_cam_view(const vr_orbit_camera *c, float out[16])
{
    float pos[3];
    vr_cam_position(c, pos);
    float tr[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    // glm::translate(I, v): Result[3] = m[0]*v0 + m[1]*v1 + m[2]*v2 + m[3]
    const float v[3] = {-pos[0], -pos[1], -pos[2]};
    for (int i = 0; i < 4; ++i) {
        const float id0 = (i == 0) ? 1.0f : 0.0f, id1 = (i == 1) ? 1.0f : 0.0f;
        const float id2 = (i == 2) ? 1.0f : 0.0f, id3 = (i == 3) ? 1.0f : 0.0f;
        tr[12 + i] = id0 * v[0] + id1 * v[1] + id2 * v[2] + id3;
    }
    float rot[16], rt[16];
    mat4_cast(load_q(c), rot);
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) rt[j * 4 + i] = rot[i * 4 + j];  // transpose
    mat_mul(rt, tr, out);
}

void vr_cam_to_camera(const vr_orbit_camera *c, vr_camera *out)
{
    vr_cam_view(c, out->view);
    vr_cam_position(c, out->position);
    out->fovy_deg = 40.0f;
    out->znear = 0.1f;
    out->zfar = 10.0f;
}

// ---- gradient.cpp ----
vr_gradient *vr_gradient_create(void) { return new vr_gradient(); }
void vr_gradient_destroy(vr_gradient *g) { delete g; }

int vr_gradient_add_color_marker(vr_gradient *g, float location, float r, float gr, float b)
{
    if (!g) return -1;
    return add_marker(g->color, location, RGB{r, gr, b});
}
int vr_gradient_add_alpha_marker(vr_gradient *g, float location, float a)
{
    if (!g) return -1;
    return add_marker(g->alpha, location, a);
}
int vr_gradient_remove_color_marker(vr_gradient *g, size_t index)
{
    return g ? remove_marker(g->color, index) : 0;
}
int vr_gradient_remove_alpha_marker(vr_gradient *g, size_t index)
{
    return g ? remove_marker(g->alpha, index) : 0;
}

int vr_gradient_set_alpha_marker(vr_gradient *g, size_t index, float location, float a)
{
    return g ? set_marker(g->alpha, index, location, std::clamp(a, 0.0f, 1.0f)) : -1;
}
int vr_gradient_set_color_marker(vr_gradient *g, size_t index, float location, float r, float gr,
                                 float b)
{
    return g ? set_marker(g->color, index, location, RGB{r, gr, b}) : -1;
}
size_t vr_gradient_marker_count(const vr_gradient *g, int alpha)
{
    return g ? (alpha ? g->alpha.size() : g->color.size()) : 0;
}

void vr_gradient_sample(const vr_gradient *g, float location, float out[4])
{
    const RGB c = sample_markers(g->color, location);
    out[0] = c.r;
    out[1] = c.g;
    out[2] = c.b;
    out[3] = sample_markers(g->alpha, location);
}

int vr_gradient_discretize(const vr_gradient *g, size_t count, uint32_t *out)
{
    if (!g || !out || count == 0) return -22;
    const float stride = 1.0f / (float)count;
    const float offset = stride / 2.0f;
    float location = offset;
    for (size_t i = 0; i < count; ++i) {
        float s[4];
        vr_gradient_sample(g, location, s);
        // ImGui::ColorConvertFloat4ToU32: IM_F32_TO_INT8_SAT, R << 0, G << 8, B << 16, A << 24
        out[i] = f32_to_int8_sat(s[0]) | (f32_to_int8_sat(s[1]) << 8) |
                 (f32_to_int8_sat(s[2]) << 16) | (f32_to_int8_sat(s[3]) << 24);
        location += stride;
    }
    return 0;
}

void vr_dataset_free(vr_dataset *d)
{
    if (d && d->data) {
        std::free(d->data);
        d->data = nullptr;
    }
}

}  // extern "C"

// ---------------------------------------------------------------------------------------
// NRRD reader (the reference reads through NrrdIO, nrrd_file_parser.cpp:21-47)
// ---------------------------------------------------------------------------------------
namespace {

std::string trim(const std::string &s)
{
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a])) ++a;
    while (b > a && std::isspace((unsigned char)s[b - 1])) --b;
    return s.substr(a, b - a);
}

int parse_type(std::string t)
{
    static const struct {
        const char *name;
        int dtype;
    } table[] = {
        {"signed char", VR_DTYPE_I8}, {"int8", VR_DTYPE_I8}, {"int8_t", VR_DTYPE_I8},
        {"uchar", VR_DTYPE_U8}, {"unsigned char", VR_DTYPE_U8}, {"uint8", VR_DTYPE_U8},
        {"uint8_t", VR_DTYPE_U8}, {"short", VR_DTYPE_I16}, {"short int", VR_DTYPE_I16},
        {"signed short", VR_DTYPE_I16}, {"signed short int", VR_DTYPE_I16},
        {"int16", VR_DTYPE_I16}, {"int16_t", VR_DTYPE_I16}, {"ushort", VR_DTYPE_U16},
        {"unsigned short", VR_DTYPE_U16}, {"unsigned short int", VR_DTYPE_U16},
        {"uint16", VR_DTYPE_U16}, {"uint16_t", VR_DTYPE_U16}, {"int", VR_DTYPE_I32},
        {"signed int", VR_DTYPE_I32}, {"int32", VR_DTYPE_I32}, {"int32_t", VR_DTYPE_I32},
        {"uint", VR_DTYPE_U32}, {"unsigned int", VR_DTYPE_U32}, {"uint32", VR_DTYPE_U32},
        {"uint32_t", VR_DTYPE_U32}, {"longlong", VR_DTYPE_I64}, {"long long", VR_DTYPE_I64},
        {"long long int", VR_DTYPE_I64}, {"signed long long", VR_DTYPE_I64},
        {"signed long long int", VR_DTYPE_I64}, {"int64", VR_DTYPE_I64},
        {"int64_t", VR_DTYPE_I64}, {"ulonglong", VR_DTYPE_U64},
        {"unsigned long long", VR_DTYPE_U64}, {"unsigned long long int", VR_DTYPE_U64},
        {"uint64", VR_DTYPE_U64}, {"uint64_t", VR_DTYPE_U64}, {"float", VR_DTYPE_F32},
        {"double", VR_DTYPE_F64},
    };
    for (auto &e : table)
        if (t == e.name) return e.dtype;
    return -1;
}

size_t elem_size(int dtype)
{
    switch (dtype) {
        case VR_DTYPE_I8:
        case VR_DTYPE_U8: return 1;
        case VR_DTYPE_I16:
        case VR_DTYPE_U16: return 2;
        case VR_DTYPE_I32:
        case VR_DTYPE_U32:
        case VR_DTYPE_F32: return 4;
        default: return 8;
    }
}

// Large raw payloads are read and reduced by up to kIoThreads threads, each on its own
// contiguous chunk (the page faults of the fresh buffer and the page-cache copy are the cost).
constexpr size_t kParallelMinBytes = 64ull << 20;
constexpr unsigned kIoThreads = 16;

unsigned io_threads(size_t bytes)
{
    if (bytes < kParallelMinBytes) return 1;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    return (unsigned)std::min<size_t>({(size_t)kIoThreads, (size_t)hw, bytes / (16ull << 20)});
}

template <typename F>
void parallel_chunks(size_t count, unsigned nt, F &&fn)  // fn(chunk, begin, end)
{
    if (nt <= 1) {
        fn(0u, (size_t)0, count);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (count + nt - 1) / nt;
    for (unsigned t = 0; t < nt; ++t) {
        const size_t b = std::min(count, (size_t)t * per), e = std::min(count, b + per);
        th.emplace_back(fn, t, b, e);
    }
    for (auto &x : th) x.join();
}

// std::min_element / std::max_element over static_cast<float> (nrrd_file_parser.cpp:39-40):
// the first element, replaced by every later one that compares smaller (larger).  Integer
// -> float conversion is monotone, so integers reduce in their own type (vectorised) and
// convert once.  Floats: each chunk reduces from +inf / -inf (a NaN never replaces), and the
// chunk results fold into element 0 in chunk order with the same strict compare -- the
// sequential result exactly: a NaN first element stays the result, later NaNs never enter,
// and among equal values (0.0 / -0.0) the first occurrence wins.
template <typename T>
void minmax_t(const void *data, size_t count, float &lo, float &hi)
{
    const T *p = static_cast<const T *>(data);
    const unsigned nt = io_threads(count * sizeof(T));
    if constexpr (std::is_integral_v<T>) {
        std::vector<T> a(nt, p[0]), b(nt, p[0]);
        parallel_chunks(count, nt, [&](unsigned t, size_t s, size_t e) {
            T x = p[0], y = p[0];
            for (size_t i = s; i < e; ++i) {
                x = p[i] < x ? p[i] : x;
                y = y < p[i] ? p[i] : y;
            }
            a[t] = x;
            b[t] = y;
        });
        lo = static_cast<float>(*std::min_element(a.begin(), a.end()));
        hi = static_cast<float>(*std::max_element(b.begin(), b.end()));
    } else {
        std::vector<float> a(nt, INFINITY), b(nt, -INFINITY);
        parallel_chunks(count, nt, [&](unsigned t, size_t s, size_t e) {
            float x = INFINITY, y = -INFINITY;
            for (size_t i = s; i < e; ++i) {
                const float v = static_cast<float>(p[i]);
                if (v < x) x = v;
                if (y < v) y = v;
            }
            a[t] = x;
            b[t] = y;
        });
        float x = static_cast<float>(p[0]), y = x;
        for (unsigned t = 0; t < nt; ++t) {
            if (a[t] < x) x = a[t];
            if (y < b[t]) y = b[t];
        }
        lo = x;
        hi = y;
    }
}

// Raw payload of `bytes` at byte offset `off` of `path` into dst: pread by chunks in parallel.
bool read_raw_parallel(const std::string &path, std::streamoff off, char *dst, size_t bytes)
{
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) return false;
    const unsigned nt = io_threads(bytes);
    std::vector<char> ok(nt, 0);
    parallel_chunks(bytes, nt, [&](unsigned t, size_t s, size_t e) {
        size_t done = s;
        while (done < e) {
            const ssize_t r = ::pread(fd, dst + done, std::min<size_t>(e - done, 1ull << 30),
                                      (off_t)(off + (std::streamoff)done));
            if (r <= 0) return;
            done += (size_t)r;
        }
        ok[t] = 1;
    });
    ::close(fd);
    return std::all_of(ok.begin(), ok.end(), [](char c) { return c != 0; });
}

void minmax(vr_dataset *d, size_t count)
{
    float lo = 0.0f, hi = 0.0f;
    switch (d->dtype) {
        case VR_DTYPE_I8: minmax_t<int8_t>(d->data, count, lo, hi); break;
        case VR_DTYPE_U8: minmax_t<uint8_t>(d->data, count, lo, hi); break;
        case VR_DTYPE_I16: minmax_t<int16_t>(d->data, count, lo, hi); break;
        case VR_DTYPE_U16: minmax_t<uint16_t>(d->data, count, lo, hi); break;
        case VR_DTYPE_I32: minmax_t<int32_t>(d->data, count, lo, hi); break;
        case VR_DTYPE_U32: minmax_t<uint32_t>(d->data, count, lo, hi); break;
        case VR_DTYPE_I64: minmax_t<int64_t>(d->data, count, lo, hi); break;
        case VR_DTYPE_U64: minmax_t<uint64_t>(d->data, count, lo, hi); break;
        case VR_DTYPE_F32: minmax_t<float>(d->data, count, lo, hi); break;
        default: minmax_t<double>(d->data, count, lo, hi); break;
    }
    d->vmin = lo;
    d->vmax = hi;
}

bool host_little_endian()
{
    const uint16_t one = 1;
    uint8_t b;
    std::memcpy(&b, &one, 1);
    return b == 1;
}

template <typename T>
bool store_ascii(void *dst, size_t i, const std::string &tok)
{
    char *end = nullptr;
    errno = 0;
    T v;
    if constexpr (std::is_floating_point_v<T>) {
        v = (T)std::strtod(tok.c_str(), &end);
    } else if constexpr (std::is_signed_v<T>) {
        v = (T)std::strtoll(tok.c_str(), &end, 10);
    } else {
        v = (T)std::strtoull(tok.c_str(), &end, 10);
    }
    if (end == tok.c_str()) return false;
    std::memcpy(static_cast<char *>(dst) + i * sizeof(T), &v, sizeof(T));
    return true;
}

bool ascii_elem(void *dst, int dtype, size_t i, const std::string &tok)
{
    switch (dtype) {
        case VR_DTYPE_I8: return store_ascii<int8_t>(dst, i, tok);
        case VR_DTYPE_U8: return store_ascii<uint8_t>(dst, i, tok);
        case VR_DTYPE_I16: return store_ascii<int16_t>(dst, i, tok);
        case VR_DTYPE_U16: return store_ascii<uint16_t>(dst, i, tok);
        case VR_DTYPE_I32: return store_ascii<int32_t>(dst, i, tok);
        case VR_DTYPE_U32: return store_ascii<uint32_t>(dst, i, tok);
        case VR_DTYPE_I64: return store_ascii<int64_t>(dst, i, tok);
        case VR_DTYPE_U64: return store_ascii<uint64_t>(dst, i, tok);
        case VR_DTYPE_F32: return store_ascii<float>(dst, i, tok);
        default: return store_ascii<double>(dst, i, tok);
    }
}

std::string dir_of(const std::string &p)
{
    const size_t s = p.find_last_of('/');
    return s == std::string::npos ? std::string(".") : p.substr(0, s);
}

}  // namespace

extern "C" int vr_nrrd_load(const char *path, vr_dataset *out)
{
    if (!path || !out) return herr(-22, "NULL argument");
    std::memset(out, 0, sizeof(*out));
    std::ifstream f(path, std::ios::binary);
    if (!f) return herr(-1, "Failed to read file");
    std::string line;
    if (!std::getline(f, line) || line.rfind("NRRD000", 0) != 0)
        return herr(-1, "Failed to read file");
    int dtype = -1, dim = -1;
    std::vector<uint64_t> sizes;
    std::string encoding = "raw", endian, datafile;
    long long byteskip = 0, lineskip = 0;
    bool header_done = false;
    while (std::getline(f, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        if (line.empty()) {
            header_done = true;
            break;
        }
        if (line[0] == '#') continue;
        if (line.find(":=") != std::string::npos) continue;  // key/value pairs
        const size_t colon = line.find(": ");
        if (colon == std::string::npos) return herr(-1, "Failed to read file");
        const std::string key = line.substr(0, colon);
        const std::string val = trim(line.substr(colon + 2));
        if (key == "type") {
            if (val == "block") return herr(-3, "unsupported element type 'block'");
            dtype = parse_type(val);
            if (dtype < 0) return herr(-1, "Failed to read file");
        } else if (key == "dimension") {
            dim = std::atoi(val.c_str());
        } else if (key == "sizes") {
            std::istringstream ss(val);
            uint64_t v;
            while (ss >> v) sizes.push_back(v);
        } else if (key == "encoding") {
            encoding = val;
        } else if (key == "endian") {
            endian = val;
        } else if (key == "data file" || key == "datafile") {
            datafile = val;
        } else if (key == "byte skip" || key == "byteskip") {
            byteskip = std::atoll(val.c_str());
        } else if (key == "line skip" || key == "lineskip") {
            lineskip = std::atoll(val.c_str());
        }
        // every other field (spacings, space directions, kinds, content, ...) is ignored by
        // the reference parser, which reads sizes only (nrrd_file_parser.cpp:32-33)
    }
    if (dtype < 0 || dim <= 0 || (int)sizes.size() != dim) return herr(-1, "Failed to read file");
    if (dim != 3) return herr(-2, "Invalid file properties");
    for (uint64_t s : sizes)
        if (s == 0) return herr(-1, "Failed to read file");
    const size_t count = (size_t)(sizes[0] * sizes[1] * sizes[2]);
    const size_t es = elem_size(dtype);
    if (encoding == "gz" || encoding == "gzip" || encoding == "bz2" || encoding == "bzip2")
        return herr(-1, "Failed to read file");  // NrrdIO built without zlib/bzip2
    const bool raw = encoding == "raw";
    const bool ascii = encoding == "txt" || encoding == "text" || encoding == "ascii";
    const bool hex = encoding == "hex";
    if (!raw && !ascii && !hex) return herr(-1, "Failed to read file");
    if (es > 1 && (raw || hex) && endian.empty()) return herr(-1, "Failed to read file");

    std::ifstream detached;
    std::string data_path;
    std::istream *in = &f;
    if (!datafile.empty()) {
        if (datafile.find(' ') != std::string::npos || datafile == "LIST")
            return herr(-3, "multi-file NRRD data is not supported");
        data_path = datafile[0] == '/' ? datafile : dir_of(path) + "/" + datafile;
        detached.open(data_path, std::ios::binary);
        if (!detached) return herr(-1, "Failed to read file");
        in = &detached;
    } else if (!header_done) {
        return herr(-1, "Failed to read file");
    }
    for (long long k = 0; k < lineskip; ++k)
        if (!std::getline(*in, line)) return herr(-1, "Failed to read file");

    void *data = std::malloc(count * es + 1);
    if (!data) return herr(-12, "out of memory");
    bool ok = true;
    if (raw) {
        if (byteskip == -1) {
            in->seekg(0, std::ios::end);
            const std::streamoff end = in->tellg();
            in->seekg(end - (std::streamoff)(count * es), std::ios::beg);
        } else if (byteskip > 0) {
            in->seekg(byteskip, std::ios::cur);
        }
        const size_t bytes = count * es;
        const std::streamoff pos = in->tellg();
        const std::string &src = datafile.empty() ? std::string(path) : data_path;
        if (io_threads(bytes) > 1 && pos >= 0) {
            // the payload must be all there, as a sequential read of `bytes` would find it
            in->seekg(0, std::ios::end);
            const std::streamoff end = in->tellg();
            ok = end - pos >= (std::streamoff)bytes &&
                 read_raw_parallel(src, pos, static_cast<char *>(data), bytes);
        } else {
            in->read(static_cast<char *>(data), (std::streamsize)bytes);
            ok = (size_t)in->gcount() == bytes;
        }
    } else if (hex) {
        unsigned char *d = static_cast<unsigned char *>(data);
        size_t n = 0;
        int nib = -1;
        char ch;
        while (n < count * es && in->get(ch)) {
            int v;
            if (ch >= '0' && ch <= '9') v = ch - '0';
            else if (ch >= 'a' && ch <= 'f') v = ch - 'a' + 10;
            else if (ch >= 'A' && ch <= 'F') v = ch - 'A' + 10;
            else continue;
            if (nib < 0) {
                nib = v;
            } else {
                d[n++] = (unsigned char)(nib * 16 + v);
                nib = -1;
            }
        }
        ok = n == count * es;
    } else {
        size_t n = 0;
        std::string tok;
        char ch;
        auto flush = [&]() {
            if (tok.empty()) return true;
            if (n >= count) return true;
            bool r = ascii_elem(data, dtype, n++, tok);
            tok.clear();
            return r;
        };
        while (ok && n < count && in->get(ch)) {
            if (std::isspace((unsigned char)ch) || ch == ',')
                ok = flush();
            else
                tok.push_back(ch);
        }
        if (ok) ok = flush();
        ok = ok && n == count;
    }
    if (!ok) {
        std::free(data);
        return herr(-1, "Failed to read file");
    }
    const bool file_little = endian != "big";
    if ((raw || hex) && es > 1 && file_little != host_little_endian()) {
        unsigned char *d = static_cast<unsigned char *>(data);
        for (size_t i = 0; i < count; ++i) std::reverse(d + i * es, d + (i + 1) * es);
    }
    out->dims[0] = (uint32_t)sizes[0];
    out->dims[1] = (uint32_t)sizes[1];
    out->dims[2] = (uint32_t)sizes[2];
    out->dtype = dtype;
    out->data = data;
    minmax(out, count);
    return 0;
}

extern "C" int vr_nrrd_write_raw(const char *nhdr_path, const void *data, int dtype,
                                 const uint32_t dims[3])
{
    static const char *names[] = {"", "int8", "uint8", "int16", "uint16", "int32",
                                  "uint32", "int64", "uint64", "float", "double"};
    if (!nhdr_path || !data || dtype < 1 || dtype > 10) return herr(-22, "bad argument");
    std::string hp(nhdr_path);
    std::string base = hp.size() > 5 && hp.substr(hp.size() - 5) == ".nhdr" ? hp.substr(0, hp.size() - 5) : hp;
    std::string rawp = base + ".raw";
    std::string rawname = rawp.substr(rawp.find_last_of('/') == std::string::npos ? 0 : rawp.find_last_of('/') + 1);
    FILE *h = std::fopen(hp.c_str(), "w");
    if (!h) return herr(-1, "cannot write header");
    std::fprintf(h, "NRRD0004\n# written by vr_nrrd_write_raw\ntype: %s\ndimension: 3\n", names[dtype]);
    std::fprintf(h, "sizes: %u %u %u\nencoding: raw\n", dims[0], dims[1], dims[2]);
    if (elem_size(dtype) > 1) std::fprintf(h, "endian: %s\n", host_little_endian() ? "little" : "big");
    std::fprintf(h, "data file: %s\n", rawname.c_str());
    std::fclose(h);
    FILE *r = std::fopen(rawp.c_str(), "wb");
    if (!r) return herr(-1, "cannot write data");
    const size_t bytes = (size_t)dims[0] * dims[1] * dims[2] * elem_size(dtype);
    const size_t w = std::fwrite(data, 1, bytes, r);
    std::fclose(r);
    return w == bytes ? 0 : herr(-1, "short write");
}

namespace {

// One z-slice of a CSV volume (CsvFileParser::parse, csv_file_parser.cpp:14-50): each line is a
// row, fields split on ',' the way std::getline splits them (a trailing ',' adds no field, an
// empty field is a std::stof error), each field read by std::stof.  The row width is fixed by
// the first row of the first slice; any other width is "Inconsistant dimensions" (the
// reference's message), checked as each row completes.  Returns the slice's row count.
uint32_t append_csv_slice(const char *path, std::vector<float> &data, float &vmin, float &vmax,
                          bool first_slice, uint32_t &width)
{
    std::ifstream in(path);
    std::string line;
    uint32_t rows = 0;
    while (std::getline(in, line)) {
        uint32_t fields = 0;
        for (size_t pos = 0; pos < line.size();) {
            size_t end = line.find(',', pos);
            if (end == std::string::npos) end = line.size();
            const float v = std::stof(line.substr(pos, end - pos));
            // Dataset{} seeds min = max = 0 (csv_file_parser.cpp:16); NaN never replaces them
            vmin = std::min(vmin, v);
            vmax = std::max(vmax, v);
            data.push_back(v);
            ++fields;
            pos = end + 1;
        }
        if (first_slice && rows == 0)
            width = fields;
        else if (fields != width)
            throw std::runtime_error("Inconsistant dimensions");
        ++rows;
    }
    return rows;
}

}  // namespace

extern "C" int vr_csv_load(const char *const *paths, size_t npaths, vr_dataset *out)
{
    if (!out || (!paths && npaths)) return herr(-22, "NULL argument");
    std::memset(out, 0, sizeof(*out));
    std::vector<float> data;
    float vmin = 0.0f, vmax = 0.0f;
    uint32_t dx = 0, dy = 0, z = 0;
    try {
        for (; z < npaths; ++z) {
            const uint32_t rows = append_csv_slice(paths[z], data, vmin, vmax, z == 0, dx);
            if (z == 0)
                dy = rows;
            else if (rows != dy)  // every slice has the first slice's row count
                throw std::runtime_error("Inconsistant dimensions");
        }
    } catch (std::exception &e) {
        return herr(-1, e.what());
    }
    if (data.empty() || (size_t)dx * dy * z != data.size())
        return herr(-2, "Invalid file properties");
    void *buf = std::malloc(data.size() * sizeof(float));
    if (!buf) return herr(-12, "out of memory");
    std::memcpy(buf, data.data(), data.size() * sizeof(float));
    out->dims[0] = dx;
    out->dims[1] = dy;
    out->dims[2] = z;
    out->dtype = VR_DTYPE_F32;
    out->data = buf;
    out->vmin = vmin;
    out->vmax = vmax;
    return 0;
}
