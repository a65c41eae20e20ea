// Host-side sanitizer harness (tests/test_host_sanitize.py): the NRRD reader, gradient and
// dataset entry points of host/vr_host.cpp built with -fsanitize=address,undefined or thread,
// run over every fixture in the given directories/files.  No GPU code is involved.
#include "vr/vr_host.h"
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <dirent.h>
#include <string>
int main(int argc, char **argv) {
    int n = 0, ok = 0;
    for (int a = 1; a < argc; ++a) {
        DIR *d = opendir(argv[a]);
        if (!d) { // a file
            vr_dataset ds; if (vr_nrrd_load(argv[a], &ds) == 0) { ++ok; vr_dataset_free(&ds); } ++n; continue;
        }
        while (dirent *e = readdir(d)) {
            std::string p = std::string(argv[a]) + "/" + e->d_name;
            if (p.find(".nrrd") == std::string::npos && p.find(".nhdr") == std::string::npos) continue;
            vr_dataset ds; ++n;
            if (vr_nrrd_load(p.c_str(), &ds) == 0) { ++ok; vr_dataset_free(&ds); }
        }
        closedir(d);
    }
    // gradient + csv paths
    vr_gradient *g = vr_gradient_create();
    vr_gradient_add_alpha_marker(g, 0.14f, 0.0f);
    std::vector<uint32_t> tf(256); vr_gradient_discretize(g, 256, tf.data());
    vr_gradient_destroy(g);
    std::printf("loaded %d of %d\n", ok, n);
    return 0;
}
