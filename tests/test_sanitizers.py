"""Host C code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md
5: the reference builds with -g -Wall only, so the build checks its CPU
code with sanitizers instead).  CPU only:

* the oracle restatement (oracle/sha1_oracle.c) hashing every length 0..300
  and a few long ones, one-shot and streamed at odd split points, checked
  against hashlib;
* the chunk-file readers of the library (csrc/chunk_file.c, compiled on
  their own) on CRLF / LF / comment / master-header files, including a digit
  line without a hash and a hash that is absent;
* the runtime's host thread pool (csrc/part_pool.hpp: verify-queue copies,
  pageable packing, parallel file reads) under ThreadSanitizer, hammered
  with back-to-back jobs of every width while helpers spin or sleep; its
  cpulist parser and helpers pinned to a CPU set (the NUMA placement).
Any sanitizer report fails the run (halt_on_error, exit code != 0)."""
import hashlib
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")

_ORACLE_DRV = r'''
#include <stdio.h>
#include <stdlib.h>
#include "sha1_oracle.h"
/* argv[1]: data file; then lengths.  For each length L: one-shot digest of
 * the first L bytes, and the same L bytes streamed in pieces of 1, 7, 63,
 * 64, 65, ... bytes; prints "L oneshot streamed". */
int main(int argc, char **argv) {
    FILE *f = fopen(argv[1], "rb");
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char *buf = malloc(n ? n : 1);
    if (fread(buf, 1, n, f) != (size_t)n) return 2;
    fclose(f);
    static const unsigned steps[] = {1, 7, 63, 64, 65, 1000, 4096};
    for (int a = 2; a < argc; ++a) {
        int L = atoi(argv[a]);
        uint8_t d1[20], d2[20];
        oracle_shahash(buf, L, d1);
        oracle_sha1_ctx c;
        oracle_sha1_init(&c);
        for (int p = 0, k = 0; p < L; ++k) {
            int s = (int)steps[k % 7];
            if (s > L - p) s = L - p;
            oracle_sha1_update(&c, buf + p, (uint32_t)s);
            p += s;
        }
        oracle_sha1_final(&c, d2);
        printf("%d ", L);
        for (int i = 0; i < 20; ++i) printf("%02x", d1[i]);
        printf(" ");
        for (int i = 0; i < 20; ++i) printf("%02x", d2[i]);
        printf("\n");
    }
    free(buf);
    return 0;
}
'''

_CHUNKFILE_DRV = r'''
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "chunk_hash.h"
typedef struct vector { int ele_size; int len; int size; void *val; } vector;
void vec_add(vector *v, void *ele) {
    if (v->size == v->len) { v->val = realloc(v->val, (size_t)v->ele_size * v->size * 2); v->size *= 2; }
    memcpy((char *)v->val + (size_t)v->len * v->ele_size, ele, v->ele_size);
    v->len++;
}
int main(int argc, char **argv) {
    vector v = {45, 0, 2, malloc(90)};
    read_chunk(argv[1], &v);
    printf("N %d\n", v.len);
    for (int q = 2; q < argc; ++q) printf("I %zd\n", (ssize_t)find_chunk_idx_from_hash(argv[q], argv[1]));
    FILE *f = fopen(argv[1], "r");
    seek_to_chunk_pos(f, 9000);
    seek_to_packet_pos(f, 3, 7);
    printf("S %lld\n", (long long)ftello(f));
    fclose(f);
    free(v.val);
    return 0;
}
'''


def _gcc(tmp_path, name, src, extra):
    (tmp_path / f"{name}.c").write_text(src)
    exe = tmp_path / name
    r = subprocess.run(["gcc", *SAN, "-I", os.path.join(ROOT, "include"), *extra,
                        str(tmp_path / f"{name}.c"), "-o", str(exe)], capture_output=True, text=True)
    if r.returncode != 0 and "sanitizer" in r.stderr.lower():
        pytest.skip("sanitizer runtime not available: " + r.stderr[-200:])
    assert r.returncode == 0, r.stderr
    return exe


def test_oracle_under_asan_ubsan(tmp_path):
    exe = _gcc(tmp_path, "odrv", _ORACLE_DRV,
               ["-I", os.path.join(ROOT, "oracle"), os.path.join(ROOT, "oracle", "sha1_oracle.c"), "-lpthread"])
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, 200000, dtype=np.uint8).tobytes()
    (tmp_path / "data.bin").write_bytes(data)
    lens = list(range(0, 301)) + [4095, 4096, 4097, 65535, 131072, 199999]
    r = subprocess.run([str(exe), str(tmp_path / "data.bin"), *map(str, lens)], capture_output=True,
                       text=True, env=ENV)
    assert r.returncode == 0, r.stderr[-2000:]
    rows = r.stdout.split("\n")[:-1]
    assert len(rows) == len(lens)
    for row, L in zip(rows, lens):
        l, one, streamed = row.split()
        want = hashlib.sha1(data[:L]).hexdigest()
        assert int(l) == L and one == want and streamed == want, L


def test_chunk_file_readers_under_asan_ubsan(tmp_path):
    exe = _gcc(tmp_path, "cdrv", _CHUNKFILE_DRV,
               [os.path.join(ROOT, "congestion-control-with-bittorren_amd", "csrc", "chunk_file.c")])
    hashes = [hashlib.sha1(bytes([i])).hexdigest() for i in range(5)]
    files = {
        "crlf": "".join(f"{i} {h}\r\n" for i, h in enumerate(hashes)),
        "lf": "".join(f"{i} {h}\n" for i, h in enumerate(hashes)),
        "comments": "# c\n0 " + hashes[0] + "\nnot a chunk\n7\n\n1 " + hashes[1] + "\n",
        "master": f"File: /tmp/C.tar Chunks:0 {hashes[0]}\r\n" +
                  "".join(f"{i} {h}\r\n" for i, h in enumerate(hashes) if i),
        "empty": "",
        "no_newline": f"0 {hashes[0]}",
    }
    for name, text in files.items():
        p = tmp_path / f"{name}.chunks"
        p.write_bytes(text.encode())
        r = subprocess.run([str(exe), str(p), *hashes, "0" * 40], capture_output=True, text=True, env=ENV)
        assert r.returncode == 0, (name, r.stderr[-2000:])
        assert f"S {3 * 524288 + (1500 - 16) * 7}" in r.stdout


_POOL_DRV = r'''
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include <pthread.h>
#include <sched.h>
#include "part_pool.hpp"
using s1host::PartPool;
int main() {
    int bad = 0;
    for (int helpers : {0, 1, 3, 7}) {
        PartPool pool(helpers);
        std::vector<uint8_t> src(3 << 20), dst(3 << 20);
        for (size_t i = 0; i < src.size(); ++i) src[i] = (uint8_t)(i * 2654435761u >> 13);
        for (int job = 0; job < 160; ++job) {
            const size_t n = (size_t)(job * 7919) % src.size();
            std::fill(dst.begin(), dst.begin() + n, 0);
            s1host::pool_copy(pool, dst.data(), src.data(), n);
            for (size_t i = 0; i < n; i += 4093) bad += dst[i] != src[i];
            bad += n && dst[n - 1] != src[n - 1];
            // a job of many small parts touching a shared counter per part
            std::vector<int> hit(1 + job % 40, 0);
            pool.run(hit.size(), [&](size_t i) { hit[i] += 1; });
            for (int h : hit) bad += h != 1;
            if (job % 50 == 0) {  // let the helpers fall asleep between jobs
                struct timespec ts = {0, 2000000};
                nanosleep(&ts, nullptr);
            }
        }
    }
    // cpulist parsing (the runtime's NUMA placement reads the GPU node's list)
    {
        cpu_set_t all, some, out;
        CPU_ZERO(&all);
        for (int c = 0; c < 64; ++c) CPU_SET(c, &all);
        CPU_ZERO(&some);
        for (int c : {2, 3, 8, 40}) CPU_SET(c, &some);
        bad += s1host::cpus_from_list("0-3,8,10-11\n", all, &out) != 7;
        for (int c : {0, 1, 2, 3, 8, 10, 11}) bad += !CPU_ISSET(c, &out);
        bad += s1host::cpus_from_list("0-63,128-191\n", some, &out) != 4;
        bad += s1host::cpus_from_list("x,5,,7-,9-8,12-13", all, &out) != 4;  // 5, 7, 12, 13
        for (int c : {5, 7, 12, 13}) bad += !CPU_ISSET(c, &out);
        bad += s1host::cpus_from_list("", all, &out) != 0;
    }
    // L3 domains (sha1chunk_receive_cpus): four 4-core CCDs with SMT
    // siblings at +16, CPU 4's list unreadable, CPU 8's naming a domain that
    // leaves CPU 8 out, CPUs 20-31 not allowed
    {
        cpu_set_t within;
        CPU_ZERO(&within);
        for (int c = 0; c < 20; ++c) CPU_SET(c, &within);
        auto list_of = [](int c) -> std::string {
            if (c == 4) return "";
            if (c == 8) return "10-11";
            const int ccd = (c % 16) / 4;
            char b[64];
            std::snprintf(b, sizeof b, "%d-%d,%d-%d\n", 4 * ccd, 4 * ccd + 3, 16 + 4 * ccd, 19 + 4 * ccd);
            return b;
        };
        std::vector<cpu_set_t> dom;
        const int n = s1host::l3_domains(within, &dom, list_of);
        // {0-3,16-19} {4} {5,6,7} {8} {9,10,11} {12-15}
        bad += n != 6;
        if (n == 6) {
            bad += CPU_COUNT(&dom[0]) != 8 || !CPU_ISSET(16, &dom[0]) || !CPU_ISSET(19, &dom[0]);
            bad += CPU_COUNT(&dom[1]) != 1 || !CPU_ISSET(4, &dom[1]);
            bad += CPU_COUNT(&dom[2]) != 3 || CPU_ISSET(4, &dom[2]);
            bad += CPU_COUNT(&dom[3]) != 1 || !CPU_ISSET(8, &dom[3]);
            bad += CPU_COUNT(&dom[4]) != 3 || CPU_ISSET(8, &dom[4]) || !CPU_ISSET(9, &dom[4]);
            bad += CPU_COUNT(&dom[5]) != 4 || !CPU_ISSET(12, &dom[5]);
        }
        cpu_set_t u;
        CPU_ZERO(&u);
        int total = 0;
        for (auto& d : dom) {
            CPU_OR(&u, &u, &d);
            total += CPU_COUNT(&d);
        }
        bad += !CPU_EQUAL(&u, &within) || total != 20;  // a partition of `within`
        cpu_set_t none;
        CPU_ZERO(&none);
        bad += s1host::l3_domains(none, &dom, list_of) != 0;
    }
    // helpers pinned to a CPU set run their parts there (the caller's own
    // parts run wherever the caller runs)
    {
        cpu_set_t aff, pin;
        sched_getaffinity(0, sizeof aff, &aff);
        CPU_ZERO(&pin);
        int first = -1;
        for (int c = 0; c < CPU_SETSIZE && first < 0; ++c)
            if (CPU_ISSET(c, &aff)) first = c;
        CPU_SET(first, &pin);
        PartPool pool(3, &pin);
        const pthread_t me = pthread_self();
        std::vector<int> where(4096, -2);
        std::vector<char> by_helper(4096, 0);
        for (int job = 0; job < 20; ++job)
            pool.run(where.size(), [&](size_t i) {
                where[i] = sched_getcpu();
                by_helper[i] = !pthread_equal(pthread_self(), me);
            });
        for (size_t i = 0; i < where.size(); ++i) bad += by_helper[i] && where[i] != first;
    }
    std::printf("pool %s\n", bad ? "BAD" : "ok");
    return bad ? 1 : 0;
}
'''


def test_part_pool_under_tsan(tmp_path):
    src = tmp_path / "pool.cpp"
    src.write_text(_POOL_DRV)
    exe = tmp_path / "pool"
    r = subprocess.run(["g++", "-std=c++17", "-fsanitize=thread", "-g", "-O1", "-I",
                        os.path.join(ROOT, "congestion-control-with-bittorren_amd", "csrc"), str(src), "-o",
                        str(exe), "-lpthread"], capture_output=True, text=True)
    if r.returncode != 0 and "tsan" in r.stderr.lower():
        pytest.skip("ThreadSanitizer runtime not available: " + r.stderr[-200:])
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0 and "pool ok" in r.stdout, (r.stdout, r.stderr[-3000:])
