"""TEST INFRASTRUCTURE ONLY -- ctypes view of the CPU oracle.

`liboracle.so` is the clean-room restatement of the reference SHA-1 path
(oracle/sha1_oracle.c, citing /root/reference/sha.c and chunk.c line by line).
`_ref/libsharef.so` is the UNMODIFIED reference sha.c compiled by
oracle/Makefile (`make ref`) with a timing driver of ours.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module: it is the parity checker, never part of the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SEED = 0x5EED0001
CHUNK_LEN = 524288  # constants.h:14 CHUNK_LEN, chunk.h:17 BT_CHUNK_SIZE

_u8p = C.POINTER(C.c_uint8)
_u64p = C.POINTER(C.c_uint64)
_u32p = C.POINTER(C.c_uint32)


def build(ref: bool | None = None) -> None:
    """Compile liboracle.so (and oracle/_ref when /root/reference exists)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    if ref is None:
        ref = os.path.isdir("/root/reference")
    if ref:
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True,
                       stderr=subprocess.DEVNULL)


def _declare(lib: C.CDLL, prefix: str) -> C.CDLL:
    getattr(lib, prefix + "shahash").argtypes = [_u8p, C.c_int, _u8p]
    getattr(lib, prefix + "hash_batch").argtypes = [_u8p, _u64p, _u32p, C.c_size_t, _u8p, C.c_int]
    getattr(lib, prefix + "time_synth").argtypes = [C.c_uint64, C.c_uint64, C.c_uint32,
                                                    C.c_uint64, C.c_int, _u8p]
    getattr(lib, prefix + "time_synth").restype = C.c_double
    tb = getattr(lib, prefix + "time_batch")
    tb.argtypes = [_u8p, _u64p, _u32p, C.c_size_t, _u8p, C.c_int]
    tb.restype = C.c_double
    return lib


_lib = None
_ref = {}


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build(ref=False)
        _lib = _declare(C.CDLL(path), "oracle_")
        _lib.oracle_synth_fill.argtypes = [_u8p, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint64]
        _lib.oracle_synth_chunk.argtypes = [_u8p, C.c_uint64, C.c_uint32, C.c_uint64]
        _lib.oracle_mixed_len.argtypes = [C.c_uint64, C.c_uint64]
        _lib.oracle_mixed_len.restype = C.c_uint32
        _lib.oracle_splitmix64.argtypes = [C.c_uint64]
        _lib.oracle_splitmix64.restype = C.c_uint64
    return _lib


_port_o0 = None


def port_lib(opt: str = "O2") -> C.CDLL | None:
    """The restatement built -O2 (liboracle.so) or with the reference
    Makefile's flags (liboracle_O0.so; None when not built)."""
    global _port_o0
    if opt == "O2":
        return lib()
    if _port_o0 is None:
        path = os.path.join(HERE, "liboracle_O0.so")
        if not os.path.exists(path):
            return None
        _port_o0 = _declare(C.CDLL(path), "oracle_")
    return _port_o0


def ref_lib(opt: str = "O2") -> C.CDLL | None:
    """The compiled reference sha.c (None when oracle/_ref was never built)."""
    if opt not in _ref:
        name = "libsharef.so" if opt == "O2" else "libsharef_O0.so"
        path = os.path.join(HERE, "_ref", name)
        _ref[opt] = _declare(C.CDLL(path), "ref_") if os.path.exists(path) else None
    return _ref[opt]


def _p(a: np.ndarray, t):
    return a.ctypes.data_as(t)


def shahash(data: bytes) -> bytes:
    buf = np.frombuffer(bytes(data) + b"\0", dtype=np.uint8)
    out = np.zeros(20, np.uint8)
    lib().oracle_shahash(_p(buf, _u8p), len(data), _p(out, _u8p))
    return out.tobytes()


def hash_batch(base: np.ndarray, offsets: np.ndarray, lengths: np.ndarray,
               threads: int = 8, use_ref: bool = False) -> np.ndarray:
    base = np.ascontiguousarray(base, dtype=np.uint8)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    out = np.zeros((len(off), 20), np.uint8)
    if use_ref:
        r = ref_lib()
        assert r is not None, "oracle/_ref not built"
        r.ref_hash_batch(_p(base, _u8p), _p(off, _u64p), _p(ln, _u32p), len(off),
                         _p(out, _u8p), threads)
    else:
        lib().oracle_hash_batch(_p(base, _u8p), _p(off, _u64p), _p(ln, _u32p), len(off),
                                _p(out, _u8p), threads)
    return out


def synth_chunks(first: int, count: int, chunk_len: int = CHUNK_LEN, seed: int = SEED) -> np.ndarray:
    out = np.empty(count * chunk_len, np.uint8)
    lib().oracle_synth_fill(_p(out, _u8p), first, count, chunk_len, seed)
    return out


def synth_chunk(chunk: int, length: int, seed: int = SEED) -> np.ndarray:
    out = np.empty(max(length, 1), np.uint8)
    lib().oracle_synth_chunk(_p(out, _u8p), chunk, length, seed)
    return out[:length]


def mixed_lengths(n: int, seed: int = SEED) -> np.ndarray:
    f = lib().oracle_mixed_len
    return np.array([f(i, seed) for i in range(n)], dtype=np.uint32)


def splitmix64(x: int) -> int:
    return int(lib().oracle_splitmix64(x))


def digest_of_digests(digests: np.ndarray) -> bytes:
    return shahash(np.ascontiguousarray(digests, dtype=np.uint8).tobytes())


def time_batch(base: np.ndarray, offsets: np.ndarray, lengths: np.ndarray, threads: int = 1,
               opt: str = "O2", kind: str = "reference") -> tuple[float, np.ndarray]:
    """Seconds to hash a batch already in memory, and its digests: the
    reference sha.c (kind "reference", oracle/_ref) or the restatement
    (kind "port"), built -O2 or with the reference Makefile's flags ("O0")."""
    r = ref_lib(opt) if kind == "reference" else port_lib(opt)
    if r is None:
        raise FileNotFoundError(f"{kind} build {opt} missing")
    fn = r.ref_time_batch if kind == "reference" else r.oracle_time_batch
    base = np.ascontiguousarray(base, dtype=np.uint8)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    out = np.zeros((len(off), 20), np.uint8)
    secs = fn(_p(base, _u8p), _p(off, _u64p), _p(ln, _u32p), len(off), _p(out, _u8p), threads)
    return float(secs), out


def time_synth(count: int, chunk_len: int = CHUNK_LEN, threads: int = 1, first: int = 0,
               seed: int = SEED, kind: str = "reference") -> tuple[float, bytes]:
    """CPU throughput leg: seconds to hash `count` synthetic chunks + the
    digest-of-digests.  kind="reference" uses oracle/_ref (the real sha.c),
    kind="port" the restatement."""
    agg = np.zeros(20, np.uint8)
    if kind == "reference":
        r = ref_lib()
        if r is None:
            raise FileNotFoundError("oracle/_ref/libsharef.so not built")
        secs = r.ref_time_synth(first, count, chunk_len, seed, threads, _p(agg, _u8p))
    else:
        secs = lib().oracle_time_synth(first, count, chunk_len, seed, threads, _p(agg, _u8p))
    return float(secs), agg.tobytes()
