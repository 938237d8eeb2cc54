// init_cost_probe.hip -- diagnostic only: whether HIP stream creation and
// pinned host allocation (the fixed costs of a short-lived make-chunks
// process, profiles/startup_r01.json) overlap when issued from several
// threads.  Mode "seq" or "par" (argv[1]); prints one JSON line, exits 1 if
// any HIP call fails.  The first process on a fresh box pays a cold-start
// cost (stream creation ~196 ms vs ~50 ms in later processes), so run one
// throwaway process first, or alternate par/seq and compare like with like:
//   for m in warm par seq par seq; do tools/init_cost_probe $m; done
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

#define OK(x) ((x) == hipSuccess)

int main(int argc, char** argv) {
    const bool par = argc > 1 && !strcmp(argv[1], "par");
    const char* mode = argc > 1 ? argv[1] : "seq";
    int n = 0;
    auto t0 = std::chrono::steady_clock::now();
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return 1;
    if (!OK(hipSetDevice(0))) return 1;
    const double t_init = ms_since(t0);
    hipStream_t s[4] = {nullptr, nullptr, nullptr, nullptr};
    bool ok[7] = {false, false, false, false, false, false, false};  // 4 streams, 3 buffers
    t0 = std::chrono::steady_clock::now();
    if (par) {
        std::vector<std::thread> th;
        for (int i = 0; i < 4; ++i)
            th.emplace_back([&, i] {
                ok[i] = OK(hipSetDevice(0)) && OK(hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking));
            });
        for (auto& t : th) t.join();
    } else {
        for (int i = 0; i < 4; ++i) ok[i] = OK(hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking));
    }
    const double t_streams = ms_since(t0);
    void* p[3] = {nullptr, nullptr, nullptr};
    const size_t bytes = size_t(512) << 20;
    t0 = std::chrono::steady_clock::now();
    if (par) {
        std::vector<std::thread> th;
        for (int i = 0; i < 3; ++i)
            th.emplace_back([&, i] { ok[4 + i] = OK(hipSetDevice(0)) && OK(hipHostMalloc(&p[i], bytes, 0)); });
        for (auto& t : th) t.join();
    } else {
        for (int i = 0; i < 3; ++i) ok[4 + i] = OK(hipHostMalloc(&p[i], bytes, 0));
    }
    const double t_pin = ms_since(t0);
    bool all = true;
    for (bool b : ok) all = all && b;
    printf("{\"mode\": \"%s\", \"ok\": %s, \"init_ms\": %.1f, \"4_streams_ms\": %.1f, "
           "\"3x512MiB_pinned_ms\": %.1f}\n",
           mode, all ? "true" : "false", t_init, t_streams, t_pin);
    fflush(stdout);
    for (int i = 0; i < 3; ++i)
        if (ok[4 + i]) (void)hipHostFree(p[i]);
    for (int i = 0; i < 4; ++i)
        if (ok[i]) (void)hipStreamDestroy(s[i]);
    return all ? 0 : 1;
}
