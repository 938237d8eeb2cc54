"""The tree that travels to the GPU box must hold every built file the GPU
tests, smoke() and bench.py load.  gpurun (and the driver's round-end run)
drops what .gpurunignore lists (tar --exclude semantics: './x' anchored at
the top, other patterns match any path component or basename), and the box
never builds.  A round-3 edit once listed build-asan/ there for an A/B run,
and test_host_paths_under_asan then failed on the box for want of its driver.
CPU test: no GPU, no compute calls."""
from __future__ import annotations

import fnmatch
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "congestion-control-with-bittorren_amd"

# built files a GPU run loads (tests/test_gpu_*.py, __graft_entry__.smoke, bench.py)
NEEDED = [
    f"{PKG}/libsha1chunk.so",
    f"{PKG}/libsha1chunk_hip.so",
    f"{PKG}/make-chunks",
    f"{PKG}/build-asan/asan_driver",
    f"{PKG}/build-asan/libsha1chunk.so",
    f"{PKG}/build-asan/libsha1chunk_hip.so",
    "oracle/liboracle.so",
    "oracle/_ref/libsharef.so",
    "oracle/_ref/dropin/make-chunks",
    "oracle/_ref/dropin/verify_driver",
    "tests/golden/golden.json",
    "tests/golden/synth_4096x512k.bin",
    "tests/golden/C.tar.gz",
    "bench.py",
    "__graft_entry__.py",
]


def _patterns():
    with open(os.path.join(ROOT, ".gpurunignore")) as f:
        return [ln.strip() for ln in f if ln.strip() and not ln.startswith("#")]


def _excluded(rel: str, pat: str) -> bool:
    parts = rel.split("/")
    if pat.startswith("./"):
        p = pat[2:]
        # anchored: the path itself or any of its leading directories
        return any(fnmatch.fnmatchcase("/".join(parts[:i]), p) for i in range(1, len(parts) + 1))
    return any(fnmatch.fnmatchcase(c, pat) for c in parts) or fnmatch.fnmatchcase(rel, pat)


def test_gpu_payload_not_ignored():
    bad = [(rel, pat) for rel in NEEDED for pat in _patterns() if _excluded(rel, pat)]
    assert not bad, f".gpurunignore drops files the GPU run loads: {bad}"


def test_matcher_semantics():
    assert _excluded(f"{PKG}/build-asan/asan_driver", f"./{PKG}/build-asan")
    assert _excluded("tools/x/y.o", "*.o")
    assert not _excluded(f"{PKG}/build-asan/asan_driver", f"./{PKG}/build")
    assert not _excluded("oracle/_ref/libsharef.so", "./ab")
