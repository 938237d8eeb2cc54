#!/usr/bin/env python3
"""Throughput of the receive-path verify queue (sha1chunk_vq_*, SURVEY 8f
rank 2): a peer that reassembled N 512 KiB chunks in host memory submits
each with its expected digest and drains 0/1 results, as packet_handler.c:472
-> job.c:217 would.  Expected digests come from hashlib (stdlib) so this tool
needs nothing from oracle/.  Reports chunks/s and GiB/s end-to-end (host
bytes -> pinned staging -> H2D -> kernel -> compare -> D2H -> results)."""
from __future__ import annotations

import argparse
import hashlib
import importlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=4096)
    ap.add_argument("--distinct", type=int, default=256, help="distinct host buffers reused round-robin")
    ap.add_argument("--chunk-len", type=int, default=0, help="bytes per chunk (default CHUNK_LEN, 512 KiB)")
    ap.add_argument("--batches", default="64,256,1024")
    ap.add_argument("--reps", type=int, default=1, help="timed passes per batch size (best and median reported)")
    ap.add_argument("--modes", default="batch,persistent",
                    help="queue implementations (SHA1CHUNK_VQ_MODE): batch launches, persistent drain; "
                         "host1 = a batch-1 queue on the host path (SHA1CHUNK_HOST_SMALL)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    pkg = importlib.import_module("congestion-control-with-bittorren_amd")
    L = a.chunk_len or pkg.sha1chunk.CHUNK_LEN
    if "host1" in a.modes.split(","):  # read once per process, before the first call
        os.environ.setdefault("SHA1CHUNK_HOST_SMALL", str(L))
    rng = np.random.default_rng(5)
    bufs = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for _ in range(a.distinct)]
    digs = [hashlib.sha1(b).digest() for b in bufs]
    bad = set(range(3, a.chunks, 97))
    rows = []
    for mode in a.modes.split(","):
        os.environ["SHA1CHUNK_VQ_MODE"] = "persistent" if mode == "host1" else mode
        qbatch = 1 if mode == "host1" else 256
        # one chunk at a time (the peer's synchronous pattern): submit, then
        # non-blocking polls until its result is back (batch mode needs the
        # flush of poll(wait=1): a lone chunk never fills a batch)
        with pkg.VerifyQueue(batch=qbatch, max_chunk_len=L) as q:
            lat = []
            for i in range(12):
                t0 = time.perf_counter()
                q.submit(bufs[i % a.distinct], digs[i % a.distinct], i)
                got = []
                while not got:
                    got = q.poll(wait=(mode == "batch"))
                lat.append(time.perf_counter() - t0)
            lat = sorted(lat[2:])
            row = {"mode": mode, "lone_chunk_ms_median": round(lat[len(lat) // 2] * 1e3, 3),
                   "lone_chunk_ms_min": round(lat[0] * 1e3, 3)}
            print(json.dumps(row), flush=True)
            rows.append(row)
        for batch in ([1] if mode == "host1" else [int(x) for x in a.batches.split(",")]):
            with pkg.VerifyQueue(batch=batch, max_chunk_len=L) as q:
                # warm-up batch
                for i in range(batch):
                    q.submit(bufs[i % a.distinct], digs[i % a.distinct], i)
                q.poll(wait=True)
                times, subs, ok = [], [], True
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    got = {}
                    for i in range(a.chunks):
                        d = digs[i % a.distinct]
                        if i in bad:
                            d = bytes([d[0] ^ 1]) + d[1:]
                        q.submit(bufs[i % a.distinct], d, i)
                        if (i & 63) == 63:
                            got.update(q.poll())
                    subs.append(time.perf_counter() - t0)  # the submit loop (copies included)
                    got.update(q.poll(wait=True))
                    times.append(time.perf_counter() - t0)
                    ok &= len(got) == a.chunks and all(got[i] == (1 if i in bad else 0) for i in range(a.chunks))
            dt = min(times)
            med = sorted(times)[len(times) // 2]
            row = {"mode": mode, "batch": batch, "chunks": a.chunks, "seconds": round(dt, 4),
                   "chunks_per_s": round(a.chunks / dt, 1), "GiBps": round(a.chunks * L / dt / 2**30, 3),
                   "GiBps_median": round(a.chunks * L / med / 2**30, 3), "reps": a.reps,
                   "submit_loop_s": round(min(subs), 4),
                   "copy_threads": os.environ.get("SHA1CHUNK_VQ_THREADS", "default"),
                   "results_correct": ok}
            print(json.dumps(row), flush=True)
            rows.append(row)
            if not ok:
                sys.exit(1)
    if a.out:
        json.dump(rows, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
