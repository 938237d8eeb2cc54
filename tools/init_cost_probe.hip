// init_cost_probe.hip -- diagnostic only: whether HIP stream creation and
// pinned host allocation (the fixed costs of a short-lived make-chunks
// process, profiles/startup_r01.json) overlap when issued from several
// threads.  Mode "seq" or "par" (argv[1]); prints one JSON line.
//   hipcc --offload-arch=gfx950 -O2 tools/init_cost_probe.hip -o tools/init_cost_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main(int argc, char** argv) {
    const bool par = argc > 1 && !strcmp(argv[1], "par");
    int n = 0;
    auto t0 = std::chrono::steady_clock::now();
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return 1;
    (void)hipSetDevice(0);
    const double t_init = ms_since(t0);
    hipStream_t s[4];
    t0 = std::chrono::steady_clock::now();
    if (par) {
        std::vector<std::thread> th;
        for (int i = 0; i < 4; ++i)
            th.emplace_back([&, i] {
                (void)hipSetDevice(0);
                (void)hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking);
            });
        for (auto& t : th) t.join();
    } else {
        for (int i = 0; i < 4; ++i) (void)hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking);
    }
    const double t_streams = ms_since(t0);
    void* p[3];
    const size_t bytes = size_t(512) << 20;
    t0 = std::chrono::steady_clock::now();
    if (par) {
        std::vector<std::thread> th;
        for (int i = 0; i < 3; ++i)
            th.emplace_back([&, i] {
                (void)hipSetDevice(0);
                (void)hipHostMalloc(&p[i], bytes, 0);
            });
        for (auto& t : th) t.join();
    } else {
        for (int i = 0; i < 3; ++i) (void)hipHostMalloc(&p[i], bytes, 0);
    }
    const double t_pin = ms_since(t0);
    printf("{\"mode\": \"%s\", \"init_ms\": %.1f, \"4_streams_ms\": %.1f, \"3x512MiB_pinned_ms\": %.1f}\n",
           par ? "par" : "seq", t_init, t_streams, t_pin);
    fflush(stdout);
    for (int i = 0; i < 3; ++i) (void)hipHostFree(p[i]);
    for (int i = 0; i < 4; ++i) (void)hipStreamDestroy(s[i]);
    return 0;
}
