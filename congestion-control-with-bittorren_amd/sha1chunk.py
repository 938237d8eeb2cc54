"""Python view of libsha1chunk.so -- the MI355X SHA-1 chunk engine.

Mirrors the reference's C hashing interface (same names, argument meaning and
error behaviour; file:line into /root/reference):

    shahash(data)                   chunk.c:35-51    one-shot SHA-1 -> 20 bytes
    binary2hex / hex2binary         chunk.c:57-85    lowercase hex codec
    make_chunks(path | file)        chunk.c:15-27    512 KiB chunk digests of a file
    get_chunk_hash(chunk)           chunk.c:168-185  hex digest (prints 2 lines)
    verify_hash(hex, data)          job.c:217-228    0 = match, 1 = mismatch
    verify_chunk_hash(path, hex, i) chunk.c:204-217  exit(-1) on mismatch
    SHA1()  .init/.update/.final    sha.h:58-60      streaming context

plus the batch / device entry points of include/sha1chunk.h that replace a
loop of shahash() calls.  The batch, device and verify-queue calls run on
the gfx950 HIP kernels; the reference's single-message calls (shahash,
get_chunk_hash, verify_hash, the SHA1 trio, make_chunks on a file of at most
4 MiB) hash on the host by default, as SURVEY.md 7.1 step 2 asks, and on the
kernels under SHA1CHUNK_HOST_SMALL=0 (include/sha1chunk.h, "Routing").  A
gfx950 device is required either way: there is no CPU fallback.  The library must have been built (`make -C
congestion-control-with-bittorren_amd` or __graft_entry__.build()); a missing
library or device raises, it never falls back.

PyTorch is only used for device memory and streams in the *_device helpers.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Iterable, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# SHA1CHUNK_LIB selects another build of the library (the A/B build,
# `make ab` -> build-ab/libsha1chunk.so, for tools/sweep.py-style studies)
LIB_PATH = os.environ.get("SHA1CHUNK_LIB") or os.path.join(HERE, "libsha1chunk.so")
CHUNK_LEN = 524288  # constants.h:14
DIGEST_LEN = 20
SEED = 0x5EED0001

OK, EINVAL, ENODEV, ENOMEM, EHIP, EALIGN, EIO = 0, -1, -2, -3, -4, -5, -6
HOST, DEVICE, ALL_DEVICES = 0, 1, 2
KERNEL_AUTO, KERNEL_LANE, KERNEL_FUSED, KERNEL_SPLIT = 0, 1, 2, 3
KERNELS = {"auto": KERNEL_AUTO, "lane": KERNEL_LANE, "fused": KERNEL_FUSED, "split": KERNEL_SPLIT}


class Sha1ChunkError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where} failed ({code}): {msg}")
        self.code = code


class SHA1Context(C.Structure):
    """Same 96-byte layout as the reference SHA1Context (sha.h:39-52)."""
    _fields_ = [
        ("totalLength", C.c_uint64),
        ("hash", C.c_uint32 * 5),
        ("bufferLength", C.c_uint32),
        ("buffer", C.c_uint8 * 64),
    ]


_u8p = C.POINTER(C.c_uint8)
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)
_vp = C.c_void_p
READER_FN = C.CFUNCTYPE(C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t)
SINK_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_size_t, _u8p, C.c_size_t)

# (name, restype, argtypes) of every symbol the C ABI exports.
_SIGNATURES = [
    ("SHA1Init", None, [C.POINTER(SHA1Context)]),
    ("SHA1Update", None, [C.POINTER(SHA1Context), _vp, C.c_uint32]),
    ("SHA1Final", None, [C.POINTER(SHA1Context), _u8p]),
    ("shahash", None, [_u8p, C.c_int, _u8p]),
    ("binary2hex", None, [_u8p, C.c_int, C.c_char_p]),
    ("hex2binary", None, [C.c_char_p, C.c_int, _u8p]),
    ("make_chunks", C.c_int, [_vp, C.POINTER(_u8p)]),
    ("get_chunk_hash", C.c_void_p, [C.c_char_p, C.c_size_t]),
    ("verify_chunk_hash", None, [_vp, C.c_char_p, C.c_size_t]),
    ("verify_hash", C.c_int, [C.c_char_p, C.c_char_p]),
    # non-hash rest of chunk.h (csrc/chunk_file.c); read_chunk appends to the
    # peer's vector through the peer's vec_add, so it is called from C only
    ("read_chunk", None, [C.c_char_p, _vp]),
    ("find_chunk_idx_from_hash", C.c_size_t, [C.c_char_p, C.c_char_p]),
    ("seek_to_chunk_pos", None, [_vp, C.c_size_t]),
    ("seek_to_packet_pos", None, [_vp, C.c_size_t, C.c_size_t]),
    ("sha1chunk_hash_batch", C.c_int, [_vp, _u64p, _u32p, C.c_size_t, _u8p, C.c_uint]),
    ("sha1chunk_digest", C.c_int, [_vp, C.c_uint64, _u8p]),
    ("sha1chunk_verify_batch", C.c_int, [_vp, _u64p, _u32p, C.c_size_t, _u8p, _u8p, C.c_uint]),
    ("sha1chunk_hash_device_async", C.c_int, [_vp, _vp, _vp, C.c_size_t, _vp, _vp, C.c_int]),
    ("sha1chunk_hash_uniform_async", C.c_int, [_vp, C.c_uint32, C.c_size_t, _vp, _vp, C.c_int]),
    ("sha1chunk_compare_device_async", C.c_int, [_vp, _vp, C.c_size_t, _vp, _vp]),
    ("sha1chunk_hash_stream", C.c_long, [READER_FN, _vp, SINK_FN, _vp]),
    ("sha1chunk_hash_stream_sized", C.c_long, [READER_FN, _vp, SINK_FN, _vp, C.c_uint64]),
    ("sha1chunk_hash_fd", C.c_long, [C.c_int, _u8p, C.c_size_t, C.POINTER(C.c_size_t)]),
    ("sha1chunk_compress_blocks", C.c_int, [_u32p, _vp, C.c_size_t]),
    ("sha1chunk_finish", C.c_int, [_u32p, C.c_uint64, _vp, C.c_uint32, _u8p]),
    ("sha1chunk_synth_fill_async", C.c_int, [_vp, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint64, _vp]),
    ("sha1chunk_synth_fill_ragged_async", C.c_int, [_vp, _vp, _vp, C.c_uint64, C.c_uint64, C.c_uint64, _vp]),
    ("sha1chunk_vq_create", C.c_void_p, [C.c_size_t, C.c_uint32]),
    ("sha1chunk_vq_submit", C.c_int, [_vp, _vp, C.c_uint32, _u8p, C.c_uint64]),
    ("sha1chunk_vq_reserve", C.c_void_p, [_vp, C.c_uint32]),
    ("sha1chunk_vq_commit", C.c_int, [_vp, _vp, C.c_uint32, _u8p, C.c_uint64]),
    ("sha1chunk_vq_release", C.c_int, [_vp, _vp]),
    ("sha1chunk_vq_flush", C.c_int, [_vp]),
    ("sha1chunk_vq_poll", C.c_long, [_vp, _u64p, _u8p, C.c_size_t, C.c_int]),
    ("sha1chunk_vq_pending", C.c_size_t, [_vp]),
    ("sha1chunk_vq_destroy", None, [_vp]),
    ("sha1chunk_device_count", C.c_int, []),
    ("sha1chunk_set_device", C.c_int, [C.c_int]),
    ("sha1chunk_get_device", C.c_int, []),
    ("sha1chunk_device_pci_bus_id", C.c_int, [C.c_int, C.c_char_p, C.c_size_t]),
    ("sha1chunk_receive_cpus", C.c_int, [C.c_int, C.c_uint, _vp, C.c_size_t, C.POINTER(C.c_uint)]),
    ("sha1chunk_last_error", C.c_char_p, []),
    ("sha1chunk_version", C.c_char_p, []),
]

_lib: C.CDLL | None = None


def _one_hip_runtime() -> None:
    """One HIP runtime per process.  The library's backend binds to the HIP
    runtime already loaded in the process (same soname); loaded before
    PyTorch's, it brings /opt/rocm's own and the process then holds two, and
    torch sees no device (tools/order_probe.py, profiles/order_probe_r06.log).
    So where PyTorch is installed it is imported first, which maps its
    runtime without starting it (the host-routed calls still never open
    /dev/kfd: tests/test_host_small.py)."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def lib() -> C.CDLL:
    """Load libsha1chunk.so (raises if it was never built)."""
    global _lib
    if _lib is None:
        _one_hip_runtime()
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(
                f"{LIB_PATH} is missing: build it with __graft_entry__.build() or "
                "`make -C congestion-control-with-bittorren_amd`")
        L = C.CDLL(LIB_PATH)
        for name, res, args in _SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        L.free = C.CDLL(None).free
        L.free.argtypes = [C.c_void_p]
        _lib = L
    return _lib


def exported_symbols() -> list[str]:
    return [s[0] for s in _SIGNATURES]


def _check(rc: int, where: str) -> int:
    if rc < 0:
        raise Sha1ChunkError(rc, where, lib().sha1chunk_last_error().decode(errors="replace"))
    return rc


def _np_ptr(a: np.ndarray, t=_u8p):
    return a.ctypes.data_as(t)


# ------------------------------------------------------------ device mgmt --
def device_count() -> int:
    n = lib().sha1chunk_device_count()
    return max(n, 0)


def set_device(dev: int) -> None:
    _check(lib().sha1chunk_set_device(dev), "sha1chunk_set_device")


def device_pci_bus_id(dev: int) -> str:
    """PCI address of logical device `dev`'s physical GPU."""
    buf = C.create_string_buffer(64)
    _check(lib().sha1chunk_device_pci_bus_id(dev, buf, len(buf)), "sha1chunk_device_pci_bus_id")
    return buf.value.decode()


def receive_cpus(dev: int, slot: int) -> tuple[list[int], int]:
    """The CPUs for receive thread `slot` of a verify queue on `dev` (one L3
    domain of the device's NUMA node) and the number of such domains."""
    mask = (C.c_uint8 * 128)()  # a glibc cpu_set_t: 1024 CPUs
    doms = C.c_uint(0)
    _check(lib().sha1chunk_receive_cpus(dev, slot, mask, len(mask), C.byref(doms)), "sha1chunk_receive_cpus")
    return [8 * i + b for i in range(len(mask)) for b in range(8) if mask[i] >> b & 1], doms.value


def version() -> str:
    return lib().sha1chunk_version().decode()


# ------------------------------------------------- reference-named API ----
def binary2hex(buf: bytes) -> str:
    """chunk.c:57-63 -- lowercase hex of buf."""
    b = np.frombuffer(bytes(buf) + b"\0", np.uint8)
    out = C.create_string_buffer(2 * len(buf) + 1)
    lib().binary2hex(_np_ptr(b), len(buf), out)
    return out.value.decode()


def hex2binary(hexstr: str) -> bytes:
    """chunk.c:78-85 -- hex (either case) to bytes."""
    raw = hexstr.encode()
    out = np.zeros(max(len(raw) // 2, 1), np.uint8)
    lib().hex2binary(raw, len(raw), _np_ptr(out))
    return out[: len(raw) // 2].tobytes()


def shahash(data: bytes | np.ndarray) -> bytes:
    """chunk.c:35-51 -- SHA-1 of one message (sha1chunk_digest: on the host
    by default, on the kernels under SHA1CHUNK_HOST_SMALL=0; a device is
    required either way).  Raises instead of exit(-1)."""
    buf = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else \
        np.ascontiguousarray(data, np.uint8).reshape(-1)
    n = buf.size
    if n == 0:
        buf = np.zeros(1, np.uint8)
    out = np.zeros(DIGEST_LEN, np.uint8)
    _check(lib().sha1chunk_digest(buf.ctypes.data, n, _np_ptr(out)), "shahash")
    return out.tobytes()


def get_chunk_hash(chunk: bytes) -> str:
    """chunk.c:168-185 -- hex digest; the C side prints the reference's two lines."""
    p = lib().get_chunk_hash(bytes(chunk), len(chunk))
    try:
        return C.string_at(p).decode()
    finally:
        lib().free(p)


def verify_hash(chunk_hash: str, data: bytes) -> int:
    """job.c:217-228 -- hashes CHUNK_LEN bytes of data; 0 = match, 1 = mismatch."""
    buf = bytes(data)
    if len(buf) < CHUNK_LEN:
        raise ValueError("verify_hash reads CHUNK_LEN (524288) bytes of data")
    return lib().verify_hash(chunk_hash.encode(), buf)


def make_chunks(src) -> list[bytes]:
    """chunk.c:15-27 -- digests of every 512 KiB chunk of a file (path or
    binary file object opened on a real fd)."""
    if isinstance(src, (str, os.PathLike)):
        with open(src, "rb") as f:
            return make_chunks(f)
    fd = src.fileno()
    pos = src.tell()
    os.lseek(fd, pos, os.SEEK_SET)
    size = os.fstat(fd).st_size - pos
    cap = max((size + CHUNK_LEN - 1) // CHUNK_LEN, 1)
    out = np.zeros((cap, DIGEST_LEN), np.uint8)
    total = C.c_size_t(0)
    n = _check(lib().sha1chunk_hash_fd(fd, _np_ptr(out), cap, C.byref(total)), "make_chunks")
    if total.value > cap:
        raise Sha1ChunkError(EIO, "make_chunks", "file grew while hashing")
    return [out[i].tobytes() for i in range(n)]


class SHA1:
    """sha.h:58-60 streaming context (SHA1Init / SHA1Update / SHA1Final)."""

    def __init__(self):
        self.ctx = SHA1Context()
        lib().SHA1Init(C.byref(self.ctx))

    def update(self, data: bytes) -> "SHA1":
        b = bytes(data)
        lib().SHA1Update(C.byref(self.ctx), b, len(b))
        return self

    def final(self) -> bytes:
        out = np.zeros(DIGEST_LEN, np.uint8)
        lib().SHA1Final(C.byref(self.ctx), _np_ptr(out))
        return out.tobytes()


# ------------------------------------------------------------- batch API --
def hash_batch(base: np.ndarray | bytes, offsets: Sequence[int], lengths: Sequence[int],
               all_devices: bool = False) -> np.ndarray:
    """digests[i] = SHA-1(base[offsets[i]:offsets[i]+lengths[i]]) -> (n, 20) uint8."""
    b = np.frombuffer(base, np.uint8) if isinstance(base, (bytes, bytearray)) else \
        np.ascontiguousarray(base).view(np.uint8).reshape(-1)
    if b.size == 0:
        b = np.zeros(1, np.uint8)
    off = np.ascontiguousarray(offsets, np.uint64)
    ln = np.ascontiguousarray(lengths, np.uint32)
    if off.shape != ln.shape:
        raise ValueError("offsets and lengths differ in length")
    if off.size and int((off + ln).max()) > (b.size if len(base) else 0):
        raise ValueError("chunk range outside the buffer")
    out = np.zeros((off.size, DIGEST_LEN), np.uint8)
    flags = ALL_DEVICES if all_devices else HOST
    _check(lib().sha1chunk_hash_batch(b.ctypes.data, _np_ptr(off, _u64p), _np_ptr(ln, _u32p),
                                      off.size, _np_ptr(out), flags), "sha1chunk_hash_batch")
    return out


def verify_batch(base, offsets, lengths, expected: np.ndarray) -> np.ndarray:
    """verify_hash() semantics per chunk: 0 = match, 1 = mismatch."""
    b = np.ascontiguousarray(np.frombuffer(base, np.uint8) if isinstance(base, (bytes, bytearray))
                             else base).view(np.uint8).reshape(-1)
    off = np.ascontiguousarray(offsets, np.uint64)
    ln = np.ascontiguousarray(lengths, np.uint32)
    exp = np.ascontiguousarray(expected, np.uint8).reshape(-1, DIGEST_LEN)
    mism = np.zeros(off.size, np.uint8)
    _check(lib().sha1chunk_verify_batch(b.ctypes.data, _np_ptr(off, _u64p), _np_ptr(ln, _u32p),
                                        off.size, _np_ptr(exp), _np_ptr(mism), HOST),
           "sha1chunk_verify_batch")
    return mism


class Reservation:
    """A buffer handed out by VerifyQueue.reserve(): `view` is a writable
    uint8 array over it (valid until the queue releases it)."""

    def __init__(self, ptr: int, length: int):
        self.ptr = ptr
        self.length = length
        self.view = np.ctypeslib.as_array(C.cast(ptr, _u8p), shape=(max(length, 1),))[:length]


class VerifyQueue:
    """Asynchronous batched verify for the peer's receive path: the batched
    counterpart of verify_hash() (job.c:217-228).  submit() stages a chunk
    with its expected digest and a tag; poll() yields (tag, mismatch) with
    mismatch 0 = match, 1 = mismatch (re-GET), as verify_hash returns."""

    def __init__(self, batch: int = 256, max_chunk_len: int = CHUNK_LEN):
        self._q = lib().sha1chunk_vq_create(batch, max_chunk_len)
        if not self._q:
            raise Sha1ChunkError(ENODEV if device_count() == 0 else EINVAL, "sha1chunk_vq_create",
                                 lib().sha1chunk_last_error().decode(errors="replace"))

    def submit(self, chunk: bytes, expected: bytes | str, tag: int) -> None:
        exp = bytes.fromhex(expected) if isinstance(expected, str) else bytes(expected)
        if len(exp) != DIGEST_LEN:
            raise ValueError("expected digest must be 20 bytes / 40 hex chars")
        e = np.frombuffer(exp, np.uint8)
        b = bytes(chunk)
        _check(lib().sha1chunk_vq_submit(self._q, b, len(b), _np_ptr(e), tag), "sha1chunk_vq_submit")

    def reserve(self, length: int) -> "Reservation":
        """A buffer of `length` bytes inside the queue (the peer's session
        buffer, reliable_udp.c:121): fill `.view` in place, then commit()."""
        p = lib().sha1chunk_vq_reserve(self._q, length)
        if not p:
            raise Sha1ChunkError(ENOMEM, "sha1chunk_vq_reserve",
                                 lib().sha1chunk_last_error().decode(errors="replace"))
        return Reservation(p, length)

    def commit(self, r: "Reservation", expected: bytes | str, tag: int, length: int | None = None) -> None:
        """Verify a filled reservation where it lies (packet_handler.c:472)."""
        exp = bytes.fromhex(expected) if isinstance(expected, str) else bytes(expected)
        if len(exp) != DIGEST_LEN:
            raise ValueError("expected digest must be 20 bytes / 40 hex chars")
        e = np.frombuffer(exp, np.uint8)
        n = r.length if length is None else length
        _check(lib().sha1chunk_vq_commit(self._q, r.ptr, n, _np_ptr(e), tag), "sha1chunk_vq_commit")

    def release(self, r: "Reservation") -> None:
        """Give a reservation back (after its result, or instead of a commit)."""
        _check(lib().sha1chunk_vq_release(self._q, r.ptr), "sha1chunk_vq_release")

    def flush(self) -> None:
        _check(lib().sha1chunk_vq_flush(self._q), "sha1chunk_vq_flush")

    def poll(self, wait: bool = False, max_results: int = 1 << 16) -> list[tuple[int, int]]:
        tags = np.zeros(max_results, np.uint64)
        mism = np.zeros(max_results, np.uint8)
        n = _check(lib().sha1chunk_vq_poll(self._q, _np_ptr(tags, _u64p), _np_ptr(mism), max_results,
                                           1 if wait else 0), "sha1chunk_vq_poll")
        return [(int(tags[i]), int(mism[i])) for i in range(n)]

    @property
    def pending(self) -> int:
        return int(lib().sha1chunk_vq_pending(self._q))

    def close(self) -> None:
        if self._q:
            lib().sha1chunk_vq_destroy(self._q)
            self._q = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------ device (torch) ----
def _stream_ptr(stream) -> int | None:
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)


def hash_device(base, offsets, lengths, digests, stream=None, kernel: int | str = KERNEL_AUTO) -> None:
    """Enqueue the hash of a device-resident batch (torch CUDA tensors:
    base uint8, offsets int64, lengths int32, digests uint8 (n, 20))."""
    k = KERNELS[kernel] if isinstance(kernel, str) else kernel
    n = offsets.numel()
    _check(lib().sha1chunk_hash_device_async(base.data_ptr(), offsets.data_ptr(), lengths.data_ptr(),
                                             n, digests.data_ptr(), _stream_ptr(stream), k),
           "sha1chunk_hash_device_async")


def hash_uniform_device(base, chunk_len: int, n: int, digests, stream=None,
                        kernel: int | str = KERNEL_AUTO) -> None:
    k = KERNELS[kernel] if isinstance(kernel, str) else kernel
    _check(lib().sha1chunk_hash_uniform_async(base.data_ptr(), chunk_len, n, digests.data_ptr(),
                                              _stream_ptr(stream), k),
           "sha1chunk_hash_uniform_async")


def compare_device(digests, expected, mismatch, stream=None) -> None:
    _check(lib().sha1chunk_compare_device_async(digests.data_ptr(), expected.data_ptr(),
                                                mismatch.numel(), mismatch.data_ptr(),
                                                _stream_ptr(stream)),
           "sha1chunk_compare_device_async")


def synth_fill_device(dst, first: int, count: int, chunk_len: int = CHUNK_LEN, seed: int = SEED,
                      stream=None) -> None:
    _check(lib().sha1chunk_synth_fill_async(dst.data_ptr(), first, count, chunk_len, seed,
                                            _stream_ptr(stream)), "sha1chunk_synth_fill_async")


def synth_fill_ragged_device(base, offsets, lengths, first: int, seed: int = SEED,
                             stream=None) -> None:
    _check(lib().sha1chunk_synth_fill_ragged_async(base.data_ptr(), offsets.data_ptr(),
                                                   lengths.data_ptr(), first, offsets.numel(),
                                                   seed, _stream_ptr(stream)),
           "sha1chunk_synth_fill_ragged_async")


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def mixed_lengths(n: int, seed: int = SEED) -> np.ndarray:
    """Chunk lengths of the synthetic mixed batch (BASELINE config 5, the
    received-chunk verify shape): chunk i draws an
    octave o in 0..7 and a mantissa m in 0..4095 from splitmix64 and is
    (4096 + m) << o bytes (4 KiB .. just under 1 MiB); every 7th chunk gets
    1..63 more bytes so its tail is not 64-byte aligned.  The golden digests
    of tests/golden/ were generated over these lengths by the reference."""
    i = np.arange(n, dtype=np.uint64)
    r = _splitmix64(np.uint64(seed + 1) ^ i)
    octave = (r & np.uint64(7)).astype(np.uint32)
    mant = ((r >> np.uint64(8)) & np.uint64(4095)).astype(np.uint32)
    ln = (np.uint32(4096) + mant) << octave
    tail = (_splitmix64(np.uint64(seed + 2) ^ i) % np.uint64(63)).astype(np.uint32) + 1
    return np.where(i % 7 == 6, ln + tail, ln).astype(np.uint32)


def ragged_layout(lengths: Iterable[int], align: int = 128) -> tuple[np.ndarray, int]:
    """Offsets packing chunks back to back at `align`-byte boundaries."""
    ln = np.asarray(list(lengths) if not isinstance(lengths, np.ndarray) else lengths, np.uint64)
    padded = (ln + (align - 1)) // align * align
    off = np.zeros(ln.size, np.uint64)
    if ln.size > 1:
        off[1:] = np.cumsum(padded)[:-1]
    total = int(padded.sum()) if ln.size else 0
    return off, total
