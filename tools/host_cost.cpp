// host_cost.cpp — host time of every call one multi-GPU frame makes (measurement tool, not
// product).  Each call is timed alone with steady_clock, and the device is synchronised (untimed)
// every kBatch calls so that no queue fills and the host never waits on the device inside a
// timed call: the medians are enqueue costs, not device time.
//
//   tools/bin/host_cost [frames] > out.json
//
// Rows: the HIP primitives the frame schedule uses (hipSetDevice, hipEventRecord,
// hipStreamWaitEvent), one kernel launch through the library (vr_assemble_rows), a bare
// vr_render_device, ncclGather on a one-rank communicator, and the whole vr_dist_render at 1 and
// 3 frames in flight (one rank), and vr_render_device on a multi-device context of 2, 3 and 8
// members on device 0 (copy exchange; the per-member profile is what each frame-worker thread
// spent enqueueing its part).  The frame is 128x72 over a 256^3 f32 volume with the
// reference's startup TF (one opaque texel: every ray ends at its first sample), so the kernels
// take microseconds.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "vr/vr.h"
#include "vr/vr_debug.h"
#include "vr/vr_dist.h"
#include "vr/vr_host.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

namespace {

constexpr int kBatch = 16;

struct Row {
    std::string name;
    double median = 0, mean = 0, p90 = 0;
    double wall_per_call = 0;  // the same calls back to back, no syncs, to the end of the device work
};

double now_us()
{
    return std::chrono::duration<double, std::micro>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

void die(const char *what, int rc)
{
    std::fprintf(stderr, "host_cost: %s failed (%d)\n", what, rc);
    std::exit(1);
}

Row measure(const char *name, int n, const std::function<void(int)> &call,
            const std::function<void()> &sync)
{
    for (int i = 0; i < 200; ++i) call(i);  // warm
    sync();
    std::vector<double> t;
    t.reserve(n);
    for (int i = 0; i < n; ++i) {
        const double t0 = now_us();
        call(i);
        t.push_back(now_us() - t0);
        if (i % kBatch == kBatch - 1) sync();
    }
    sync();
    Row r;
    r.name = name;
    double s = 0;
    for (double v : t) s += v;
    r.mean = s / n;
    std::sort(t.begin(), t.end());
    r.median = t[n / 2];
    r.p90 = t[n * 9 / 10];
    const double w0 = now_us();
    for (int i = 0; i < n; ++i) call(i);
    sync();
    r.wall_per_call = (now_us() - w0) / n;
    return r;
}

}  // namespace

int main(int argc, char **argv)
{
    const int n = argc > 1 ? std::atoi(argv[1]) : 3000;
    const uint32_t W = 128, H = 72;
    if (hipSetDevice(0) != hipSuccess) die("hipSetDevice", -1);
    vr_ctx *ctx = vr_create(0, W, H);
    if (!ctx) die("vr_create", -1);
    float lo, hi;
    if (int rc = vr_generate_volume(ctx, 0, VR_DTYPE_F32, 256, 256, 256, 2024, &lo, &hi))
        die("vr_generate_volume", rc);
    const uint32_t tf = 0xFFFFFFFFu;
    if (int rc = vr_set_transfer_function(ctx, &tf, 1)) die("vr_set_transfer_function", rc);
    vr_orbit_camera oc;
    vr_cam_init(&oc);
    oc.radius = 1.6f;
    vr_camera cam;
    vr_cam_to_camera(&oc, &cam);

    std::vector<Row> rows;
    std::vector<std::string> breakdown;  // vr_dist_host_profile per frame, per frames in flight
    hipStream_t s[3], caller;
    for (auto &x : s) hipStreamCreateWithFlags(&x, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&caller, hipStreamNonBlocking);
    hipEvent_t ev;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    auto sync = [] { (void)hipDeviceSynchronize(); };

    rows.push_back(measure("hipSetDevice", n, [](int) { hipSetDevice(0); }, sync));
    rows.push_back(measure("hipEventRecord", n, [&](int i) { hipEventRecord(ev, s[i % 3]); }, sync));
    rows.push_back(measure("hipStreamWaitEvent", n, [&](int i) {
        hipStreamWaitEvent(s[(i + 1) % 3], ev, 0);
    }, sync));

    const uint32_t sr = vr_shard_rows(H, 8, 1);
    void *shard[3], *gbuf, *frame;
    for (auto &b : shard) hipMalloc(&b, (size_t)sr * W * 4);
    hipMalloc(&gbuf, (size_t)sr * W * 4);
    hipMalloc(&frame, (size_t)W * H * 4);
    rows.push_back(measure("vr_assemble_rows (one kernel launch)", n, [&](int i) {
        if (int rc = vr_assemble_rows(ctx, gbuf, frame, VR_OUT_RGBA8, 8, 1, s[i % 3]))
            die("vr_assemble_rows", rc);
    }, sync));
    for (int fif : {1, 3}) {
        vr_params p;
        vr_params_default(&p);
        p.shading = 1;
        p.ert_eps = 1e-5f;
        p.frames_in_flight = fif;
        const std::string nm = "vr_render_device (frames_in_flight " + std::to_string(fif) + ")";
        rows.push_back(measure(nm.c_str(), n, [&](int i) {
            if (int rc = vr_render_device(ctx, &cam, &p, shard[i % fif], VR_OUT_RGBA8, 8, 0, 1,
                                          s[i % fif]))
                die("vr_render_device", rc);
        }, sync));
    }

    // ncclGather on a one-rank communicator (the library's own gather call)
    ncclComm_t comm;
    int dev0 = 0;
    if (ncclCommInitAll(&comm, 1, &dev0) != ncclSuccess) die("ncclCommInitAll", -1);
    rows.push_back(measure("ncclGather (1 rank)", n, [&](int) {
        if (ncclGather(shard[0], gbuf, (size_t)sr * W, ncclUint32, 0, comm, caller) != ncclSuccess)
            die("ncclGather", -1);
    }, sync));
    // rank r > 0's frame (vr_frame_schedule.h) restated on the raw calls, 3 slots: render on the
    // slot stream, wait for the previous frame's gather, ncclGather on the slot stream, record --
    // what a multi-GPU rank other than 0 (and a mask context's member worker) issues per frame.
    // ncclGather on a one-rank communicator stands in for the 8-rank one.
    {
        hipEvent_t g[3];
        for (auto &e : g) hipEventCreateWithFlags(&e, hipEventDisableTiming);
        vr_params p;
        vr_params_default(&p);
        p.shading = 1;
        p.ert_eps = 1e-5f;
        p.frames_in_flight = 3;
        uint64_t f = 0;
        rows.push_back(measure("rank r > 0 frame restated (render, wait, ncclGather, record; 3 slots)", n,
                               [&](int) {
            const int k = (int)(f % 3);
            if (int rc = vr_render_device(ctx, &cam, &p, shard[k], VR_OUT_RGBA8, 8, 0, 1, s[k]))
                die("vr_render_device", rc);
            if (f) hipStreamWaitEvent(s[k], g[(k + 2) % 3], 0);
            if (ncclGather(shard[k], gbuf, (size_t)sr * W, ncclUint32, 0, comm, s[k]) != ncclSuccess)
                die("ncclGather", -1);
            hipEventRecord(g[k], s[k]);
            ++f;
        }, sync));
        for (auto &e : g) hipEventDestroy(e);
    }
    ncclCommDestroy(comm);

    for (int fif : {1, 3}) {
        unsigned char id[VR_DIST_ID_BYTES];
        if (int rc = vr_dist_unique_id(id)) die("vr_dist_unique_id", rc);
        vr_dist *d = vr_dist_create(ctx, id, 1, 0, 8, fif);
        if (!d) die("vr_dist_create", -1);
        vr_params p;
        vr_params_default(&p);
        p.shading = 1;
        p.ert_eps = 1e-5f;
        p.frames_in_flight = fif;
        const std::string nm = "vr_dist_render (1 rank, frames_in_flight " + std::to_string(fif) + ")";
        vr_dist_host_profile_enable(d, 1);
        rows.push_back(measure(nm.c_str(), n, [&](int) {
            if (int rc = vr_dist_render(d, &cam, &p, frame, caller)) die("vr_dist_render", rc);
        }, [&] {
            vr_dist_synchronize(d);
            (void)hipDeviceSynchronize();
        }));
        vr_dist_host_profile hp;
        vr_dist_host_profile_read(d, &hp);
        const double f = hp.frames ? (double)hp.frames : 1.0;
        char buf[512];
        std::snprintf(buf, sizeof buf,
                      "{\"frames_in_flight\": %d, \"frames\": %llu, \"render_us\": %.2f, "
                      "\"gather_us\": %.2f, \"assemble_us\": %.2f, \"record_us\": %.2f, "
                      "\"wait_us\": %.2f, \"total_us\": %.2f}",
                      fif, (unsigned long long)hp.frames, hp.render_us / f, hp.gather_us / f,
                      hp.assemble_us / f, hp.record_us / f, hp.wait_us / f, hp.total_us / f);
        breakdown.push_back(buf);
        vr_dist_destroy(d);
    }

    // multi-device contexts on device 0 (vr_debug_create_members, copy exchange): the caller's
    // vr_render_device (member 0 on its thread: its render, the wait for every member's shard,
    // the copies, the assembly) and each member's host profile (the worker's enqueue)
    std::vector<std::string> members;
    for (int nm : {2, 3, 8}) {
        std::vector<int> devs(nm, 0);
        vr_ctx *g = vr_debug_create_members(devs.data(), nm, W, H, VR_EXCHANGE_COPY);
        if (!g) die("vr_debug_create_members", -1);
        if (int rc = vr_generate_volume(g, 0, VR_DTYPE_F32, 256, 256, 256, 2024, &lo, &hi))
            die("vr_generate_volume (members)", rc);
        if (int rc = vr_set_transfer_function(g, &tf, 1)) die("vr_set_transfer_function", rc);
        vr_params p;
        vr_params_default(&p);
        p.shading = 1;
        p.ert_eps = 1e-5f;
        p.frames_in_flight = 3;
        vr_debug_host_profile_enable(g, 1);
        const std::string nm_s = "vr_render_device (" + std::to_string(nm) +
                                 " members on device 0, copy exchange, frames_in_flight 3)";
        rows.push_back(measure(nm_s.c_str(), n, [&](int) {
            if (int rc = vr_render_device(g, &cam, &p, frame, VR_OUT_RGBA8, 8, 0, 1, caller))
                die("vr_render_device (members)", rc);
        }, [&] {
            double ms;
            uint64_t launches;
            (void)vr_timing_read(g, &ms, &launches);  // drains the workers and the devices
        }));
        std::string row = "{\"members\": " + std::to_string(nm) + ", \"per_member\": [";
        for (int m = 0; m < nm; ++m) {
            vr_dist_host_profile hp;
            if (int rc = vr_debug_host_profile_member(g, m, &hp)) die("vr_debug_host_profile_member", rc);
            const double f = hp.frames ? (double)hp.frames : 1.0;
            char buf[400];
            std::snprintf(buf, sizeof buf,
                          "%s{\"member\": %d, \"frames\": %llu, \"render_us\": %.2f, "
                          "\"gather_us\": %.2f, \"assemble_us\": %.2f, \"record_us\": %.2f, "
                          "\"wait_us\": %.2f, \"total_us\": %.2f}",
                          m ? ", " : "", m, (unsigned long long)hp.frames, hp.render_us / f,
                          hp.gather_us / f, hp.assemble_us / f, hp.record_us / f, hp.wait_us / f,
                          hp.total_us / f);
            row += buf;
        }
        members.push_back(row + "]}");
        vr_destroy(g);
    }

    std::printf("{\"viewport\": \"%ux%u\", \"volume\": \"256^3 f32\", \"calls\": %d, "
                "\"sync_every\": %d, \"rows\": [\n", W, H, n, kBatch);
    for (size_t i = 0; i < rows.size(); ++i)
        std::printf("  {\"call\": \"%s\", \"median_us\": %.2f, \"mean_us\": %.2f, \"p90_us\": %.2f, "
                    "\"back_to_back_wall_us\": %.2f}%s\n",
                    rows[i].name.c_str(), rows[i].median, rows[i].mean, rows[i].p90,
                    rows[i].wall_per_call, i + 1 < rows.size() ? "," : "");
    std::printf("], \"dist_render_breakdown_per_frame\": [\n");
    for (size_t i = 0; i < breakdown.size(); ++i)
        std::printf("  %s%s\n", breakdown[i].c_str(), i + 1 < breakdown.size() ? "," : "");
    std::printf("], \"members_host_profile_per_frame\": [\n");
    for (size_t i = 0; i < members.size(); ++i)
        std::printf("  %s%s\n", members[i].c_str(), i + 1 < members.size() ? "," : "");
    std::printf("]}\n");
    vr_destroy(ctx);
    return 0;
}
