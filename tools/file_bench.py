#!/usr/bin/env python3
"""End-to-end make-chunks on a real file: file -> fread
into pinned slots -> H2D -> kernel -> D2H -> "%d %s\\n" lines, timed for the
repo's make-chunks CLI and the Python make_chunks (sha1chunk_hash_fd), next
to the two rates that bound it: reading the file from the page cache and a
pinned H2D copy.  Spot-checks digests with hashlib (stdlib).  The file is
written under $TMPDIR (default /tmp) and removed afterwards."""
from __future__ import annotations

import argparse
import hashlib
import importlib
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
L = 524288


def write_file(path: str, size: int) -> None:
    rng = np.random.default_rng(11)
    block = 64 << 20
    with open(path, "wb") as f:
        left = size
        while left:
            n = min(block, left)
            f.write(rng.integers(0, 2**63, n // 8 + 1, dtype=np.int64).tobytes()[:n])
            left -= n


def read_rate(path: str) -> float:
    buf = bytearray(64 << 20)
    mv = memoryview(buf)
    t0 = time.perf_counter()
    total = 0
    with open(path, "rb", buffering=0) as f:
        while True:
            n = f.readinto(mv)
            if not n:
                break
            total += n
    return total / (time.perf_counter() - t0) / 2**30


def h2d_rate(size: int) -> float:
    import torch
    n = min(size, 4 << 30)
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    return 3 * n / (time.perf_counter() - t0) / 2**30


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=8.0)
    ap.add_argument("--tail", type=int, default=123457, help="extra bytes: a short last chunk")
    ap.add_argument("--out", default="")
    ap.add_argument("--reps", type=int, default=3, help="timed runs (median reported)")
    ap.add_argument("--cli-slot-ab", default="",
                    help="e.g. 128,512: only time the make-chunks CLI with each "
                         "SHA1CHUNK_STREAM_SLOT_MIB, interleaved, and check every digest")
    a = ap.parse_args()
    if a.cli_slot_ab:
        return cli_slot_ab(a)
    pkg = importlib.import_module("congestion-control-with-bittorren_amd")
    size = int(a.gib * 2**30) + a.tail
    fd, path = tempfile.mkstemp(prefix="sha1bench_", suffix=".dat")
    os.close(fd)
    try:
        write_file(path, size)
        nchunks = (size + L - 1) // L
        read_gibs = max(read_rate(path), read_rate(path))
        h2d = h2d_rate(size)
        pkg.make_chunks(path)  # warm-up: device init, pinned slots
        py_t = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            digs = pkg.make_chunks(path)
            py_t.append(time.perf_counter() - t0)
        py_s = float(np.median(py_t))
        exe = os.path.join(ROOT, "congestion-control-with-bittorren_amd", "make-chunks")
        cli_t = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            out = subprocess.run([exe, path], capture_output=True, text=True, check=True).stdout
            cli_t.append(time.perf_counter() - t0)
        cli_s = float(np.median(cli_t))
        # the CLI's fixed cost (process start, HIP init, first slot): a 1-chunk file
        small = path + ".small"
        with open(path, "rb") as f, open(small, "wb") as g:
            g.write(f.read(L))
        small_t = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            subprocess.run([exe, small], capture_output=True, text=True, check=True)
            small_t.append(time.perf_counter() - t0)
        os.unlink(small)
        lines = out.splitlines()
        ok = len(digs) == nchunks and len(lines) == nchunks
        with open(path, "rb") as f:
            for i in sorted({0, 1, nchunks // 2, nchunks - 2, nchunks - 1}):
                f.seek(i * L)
                want = hashlib.sha1(f.read(L)).hexdigest()
                ok &= digs[i].hex() == want and lines[i] == f"{i} {want}"
        row = {"file_bytes": size, "chunks": nchunks,
               "make_chunks_py_GiBps": round(size / py_s / 2**30, 3),
               "make_chunks_cli_GiBps": round(size / cli_s / 2**30, 3),
               "cli_seconds": round(cli_s, 3), "cli_one_chunk_seconds": round(float(np.median(small_t)), 3),
               "py_runs_s": [round(t, 4) for t in py_t],
               "stream_slots": os.environ.get("SHA1CHUNK_STREAM_SLOTS", "default"),
               "stream_slot_mib": os.environ.get("SHA1CHUNK_STREAM_SLOT_MIB", "default"),
               "read_threads": os.environ.get("SHA1CHUNK_READ_THREADS", "default"),
               "stream_piece_mib": os.environ.get("SHA1CHUNK_STREAM_PIECE_MIB", "default"),
               "page_cache_read_GiBps": round(read_gibs, 3),
               "pinned_h2d_GiBps": round(h2d, 3), "digests_spot_checked_ok": bool(ok)}
        print(json.dumps(row), flush=True)
        if a.out:
            json.dump(row, open(a.out, "w"), indent=1)
        if not ok:
            sys.exit(1)
    finally:
        os.unlink(path)


def cli_slot_ab(a) -> None:
    """The make-chunks CLI's slot-size choice (make_chunks_main.c: 128 MiB
    below 16 GiB, 512 MiB above) measured around the cutoff: each slot size
    in turn, interleaved over the reps, on the same page-cached file; every
    digest line checked against hashlib (16 threads)."""
    from concurrent.futures import ThreadPoolExecutor
    size = int(a.gib * 2**30) + a.tail
    nchunks = (size + L - 1) // L
    fd, path = tempfile.mkstemp(prefix="sha1bench_", suffix=".dat")
    os.close(fd)
    exe = os.path.join(ROOT, "congestion-control-with-bittorren_amd", "make-chunks")
    slots = [int(x) for x in a.cli_slot_ab.split(",")]
    try:
        write_file(path, size)
        read_rate(path)  # page cache warm

        def sha(i):
            with open(path, "rb") as f:
                f.seek(i * L)
                return hashlib.sha1(f.read(L)).hexdigest()

        with ThreadPoolExecutor(16) as ex:
            want = "".join(f"{i} {h}\n" for i, h in enumerate(ex.map(sha, range(nchunks))))
        times = {m: [] for m in slots}
        ok = True
        for _ in range(a.reps):
            for m in slots:
                env = dict(os.environ, SHA1CHUNK_STREAM_SLOT_MIB=str(m))
                t0 = time.perf_counter()
                out = subprocess.run([exe, path], capture_output=True, text=True, check=True,
                                     env=env).stdout
                times[m].append(time.perf_counter() - t0)
                ok &= out == want
                print(f"slot {m} MiB: {times[m][-1]:.3f} s", flush=True)
        row = {"file_bytes": size, "chunks": nchunks, "reps": a.reps,
               "cli_seconds": {str(m): [round(t, 3) for t in v] for m, v in times.items()},
               "cli_median_GiBps": {str(m): round(size / float(np.median(v)) / 2**30, 3)
                                    for m, v in times.items()},
               "all_digests_match_hashlib": bool(ok)}
        print(json.dumps(row), flush=True)
        if a.out:
            json.dump(row, open(a.out, "w"), indent=1)
        if not ok:
            sys.exit(1)
    finally:
        os.unlink(path)


if __name__ == "__main__":
    main()
