/*
 * nrrd_ref.c — loader oracle (TEST INFRASTRUCTURE ONLY).
 *
 * Linked against the reference's own vendored NrrdIO, compiled from its sources where they
 * lie (/root/reference/extern/NrrdIO, recipe in oracle/Makefile, output in oracle/_ref/).
 * Restates Vol::Data::NrrdFileParser::parse + convert (src/data/nrrd_file_parser.cpp:21-77):
 * nrrdLoad, dim == 3 check, dims = axis[0..2].size (axis 0 fastest), every element type
 * static_cast<float>, min/max over all voxels, nrrdNuke.  Used to pin the product's own
 * NRRD reader and the synthetic fixture files.
 */
#include <NrrdIO.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* Returns 0 on success; -1 load failure ("Failed to read file"), -2 dim != 3 ("Invalid file
 * properties"), -3 unsupported element type (the reference returns an empty vector). */
int nref_load(const char *path, uint32_t dims[3], int *nrrd_type, float **data_out,
              float *vmin, float *vmax)
{
    *data_out = NULL;
    Nrrd *n = nrrdNew();
    if (nrrdLoad(n, path, NULL)) {
        char *err = biffGetDone(NRRD);
        free(err);
        nrrdNuke(n);
        return -1;
    }
    if (n->dim != 3) {
        nrrdNuke(n);
        return -2;
    }
    dims[0] = (uint32_t)n->axis[0].size;
    dims[1] = (uint32_t)n->axis[1].size;
    dims[2] = (uint32_t)n->axis[2].size;
    *nrrd_type = n->type;
    size_t count = (size_t)dims[0] * dims[1] * dims[2];
    float *out = (float *)malloc(count * sizeof(float) + 1);
    if (!out) {
        nrrdNuke(n);
        return -4;
    }
#define CONV(T)                                                        \
    do {                                                               \
        const T *src = (const T *)n->data;                             \
        for (size_t i = 0; i < count; ++i) out[i] = (float)src[i];     \
    } while (0)
    switch (n->type) {
        case nrrdTypeChar: CONV(int8_t); break;
        case nrrdTypeUChar: CONV(uint8_t); break;
        case nrrdTypeShort: CONV(int16_t); break;
        case nrrdTypeUShort: CONV(uint16_t); break;
        case nrrdTypeInt: CONV(int32_t); break;
        case nrrdTypeUInt: CONV(uint32_t); break;
        case nrrdTypeLLong: CONV(int64_t); break;
        case nrrdTypeULLong: CONV(uint64_t); break;
        case nrrdTypeFloat: CONV(float); break;
        case nrrdTypeDouble: CONV(double); break;
        default:
            free(out);
            nrrdNuke(n);
            return -3;
    }
#undef CONV
    float lo = out[0], hi = out[0];
    for (size_t i = 1; i < count; ++i) {
        /* std::min_element / max_element semantics: first strict improvement */
        if (out[i] < lo) lo = out[i];
        if (hi < out[i]) hi = out[i];
    }
    *vmin = lo;
    *vmax = hi;
    *data_out = out;
    nrrdNuke(n);
    return 0;
}

void nref_free(float *p) { free(p); }
