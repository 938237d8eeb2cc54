// part_pool.hpp -- host-side helper threads of the SHA-1 chunk runtime
// (sha1_runtime.hip): the verify queue's chunk copies, the pageable-batch
// packing and the file pipeline's parallel preads run their pieces on a
// PartPool.  Plain C++ (no HIP), so tests/test_sanitizers.py can also run it
// under ThreadSanitizer on the CPU.
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <pthread.h>
#include <sched.h>
#include <string>
#include <thread>
#include <vector>

namespace s1host {

inline void cpu_relax() { __builtin_ia32_pause(); }

// Persistent helper threads that run the parts of one job (a host copy
// split in pieces, a file read split over pread calls) together with the
// calling thread.  run() returns when every part is done.  Between jobs the
// helpers poll for the next one for a while (a caller streaming chunks or
// file pieces comes back within microseconds) before sleeping, so a job does
// not pay a thread start or a futex wake-up.
class PartPool {
public:
    // cpus (optional): the helpers run on these host CPUs only -- the ones
    // near the GPU whose pinned buffers they fill (sha1_runtime.hip
    // near_cpus); the calling thread's own placement is the caller's
    explicit PartPool(int helpers, const cpu_set_t* cpus = nullptr) {
        if (cpus) {
            cpus_ = *cpus;
            pin_ = true;
        }
        for (int i = 0; i < helpers; ++i) th_.emplace_back([this] { loop(); });
    }
    ~PartPool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_.store(true);
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    size_t width() const { return th_.size() + 1; }
    // fn(i) for i in [0, parts), on the caller and the helpers
    void run(size_t parts, const std::function<void(size_t)>& fn) {
        if (parts <= 1 || th_.empty() || parts > 0xffffffffu) {
            for (size_t i = 0; i < parts; ++i) fn(i);
            return;
        }
        {
            std::lock_guard<std::mutex> g(mu_);
            fn_ = &fn;
            parts_ = parts;
            left_.store(parts);
            job_ = gen_.load() + 1;
            next_.store((job_ & 0xffffffffu) << 32);
            gen_.store(job_);
        }
        // helpers still polling see gen_ at once; only sleeping ones need the
        // (syscall) wake-up
        if (sleepers_.load() > 0) cv_.notify_all();
        work(job_, parts, &fn);
        // the caller's own parts are done; wait for the helpers' parts
        for (int spin = 0; left_.load() != 0 && spin < 200000; ++spin) cpu_relax();
        if (left_.load() != 0) {
            std::unique_lock<std::mutex> g(mu_);
            done_.wait(g, [this] { return left_.load() == 0; });
        }
    }

private:
    static constexpr int kSpin = 20000;  // pause loops (tens of microseconds)
    // Claims part indices of job `job` only: the counter carries the job
    // number in its high half, so a helper that finished (or never started)
    // an older job cannot claim an index of the next one, and every part of a
    // job runs exactly once.
    void work(uint64_t job, size_t parts, const std::function<void(size_t)>* fn) {
        uint64_t cur = next_.load();
        for (;;) {
            if ((cur >> 32) != (job & 0xffffffffu) || (cur & 0xffffffffu) >= parts) return;
            if (!next_.compare_exchange_weak(cur, cur + 1)) continue;
            (*fn)(size_t(cur & 0xffffffffu));
            if (left_.fetch_sub(1) == 1) {
                std::lock_guard<std::mutex> g(mu_);
                done_.notify_all();
            }
            cur = next_.load();
        }
    }
    void loop() {
        if (pin_) (void)pthread_setaffinity_np(pthread_self(), sizeof cpus_, &cpus_);
        uint64_t seen = 0;
        for (;;) {
            int spin = 0;
            while (gen_.load() == seen && !stop_.load() && spin++ < kSpin) cpu_relax();
            if (gen_.load() == seen && !stop_.load()) {
                std::unique_lock<std::mutex> g(mu_);
                sleepers_.fetch_add(1);
                cv_.wait(g, [&] { return stop_.load() || gen_.load() != seen; });
                sleepers_.fetch_sub(1);
            }
            if (stop_.load()) return;
            uint64_t job;
            size_t parts;
            const std::function<void(size_t)>* fn;
            {
                // a job's fields are published under mu_
                std::lock_guard<std::mutex> g(mu_);
                seen = job = gen_.load();
                parts = parts_;
                fn = fn_;
            }
            work(job, parts, fn);
        }
    }
    std::vector<std::thread> th_;
    cpu_set_t cpus_{};
    bool pin_ = false;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    std::atomic<uint64_t> gen_{0};
    std::atomic<int> sleepers_{0};
    std::atomic<bool> stop_{false};
    const std::function<void(size_t)>* fn_ = nullptr;
    size_t parts_ = 0;      // guarded by mu_
    uint64_t job_ = 0;      // caller side only
    std::atomic<uint64_t> next_{0};  // job << 32 | next part index
    std::atomic<size_t> left_{0};
};

// The CPUs of a sysfs cpulist ("0-63,128-191\n") that are also in `allowed`,
// into *out; returns their count (malformed pieces are skipped).  The
// runtime's NUMA placement (sha1_runtime.hip near_cpus) reads the GPU's
// node's list with it.
inline int cpus_from_list(const char* list, const cpu_set_t& allowed, cpu_set_t* out) {
    CPU_ZERO(out);
    for (const char* p = list; p && *p;) {
        char* end = nullptr;
        const long a = strtol(p, &end, 10);
        if (end == p) {  // not a number: skip to the next piece
            p = strchr(p, ',');
            if (p) ++p;
            continue;
        }
        long b = a;
        p = end;
        if (*p == '-') {
            b = strtol(p + 1, &end, 10);
            if (end == p + 1) b = a;  // "5-": just 5
            p = end;
        }
        for (long c = a; c <= b && c >= 0 && c < CPU_SETSIZE; ++c)
            if (CPU_ISSET(static_cast<int>(c), &allowed)) CPU_SET(static_cast<int>(c), out);
        p = strchr(p, ',');
        if (p) ++p;
    }
    return CPU_COUNT(out);
}

// The L3 domains (CPUs that share a last-level cache: a CCD on the EPYC
// hosts of the MI355X boxes) of the CPUs in `within`, in CPU order, into
// *out; list_of(cpu) gives a CPU's sysfs shared_cpu_list ("0-7,128-135\n"),
// empty if unknown.  A CPU whose list is unknown or leaves it out is a
// domain of its own; a CPU lands in the first domain that names it.  The
// runtime hands one domain per receive thread (sha1chunk_receive_cpus).
template <class ListOf>
inline int l3_domains(const cpu_set_t& within, std::vector<cpu_set_t>* out, ListOf list_of) {
    out->clear();
    cpu_set_t seen;
    CPU_ZERO(&seen);
    for (int c = 0; c < CPU_SETSIZE; ++c) {
        if (!CPU_ISSET(c, &within) || CPU_ISSET(c, &seen)) continue;
        cpu_set_t d;
        const std::string list = list_of(c);
        if (cpus_from_list(list.c_str(), within, &d) == 0 || !CPU_ISSET(c, &d)) {
            CPU_ZERO(&d);
            CPU_SET(c, &d);
        }
        for (int x = 0; x < CPU_SETSIZE; ++x)
            if (CPU_ISSET(x, &d) && CPU_ISSET(x, &seen)) CPU_CLR(x, &d);
        CPU_OR(&seen, &seen, &d);
        out->push_back(d);
    }
    return static_cast<int>(out->size());
}

// memcpy split over a pool (pieces of >= 64 KiB)
inline void pool_copy(PartPool& pool, uint8_t* dst, const uint8_t* src, size_t n) {
    const size_t parts = std::min<size_t>(pool.width(), n / (size_t(64) << 10));
    if (parts <= 1) {
        memcpy(dst, src, n);
        return;
    }
    pool.run(parts, [&](size_t i) {
        const size_t a = n * i / parts, b = n * (i + 1) / parts;
        memcpy(dst + a, src + a, b - a);
    });
}

}  // namespace s1host
