"""CPU: pin the oracle (oracle/sha1_oracle.c) against the reference's own
known answers and fixtures, and against the compiled reference sha.c."""
import ctypes
import hashlib
import os

import numpy as np
import pytest


def test_kats(oracle, golden):
    for name, kat in golden["kats"].items():
        if "input_hex" in kat:
            data = bytes.fromhex(kat["input_hex"])
        else:
            data = bytes.fromhex(kat["input_repeat"][0]) * kat["input_repeat"][1]
        assert oracle.shahash(data).hex() == kat["digest"], name


def test_nist_vectors_quoted_in_reference(oracle):
    # sha.c:35-37 comment block
    assert oracle.shahash(b"abc").hex() == "a9993e364706816aba3e25717850c26c9cd0d89d"
    assert oracle.shahash(b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq").hex() == \
        "84983e441c3bd26ebaae4aa1f95129e5e54670f1"
    # chunk.c:235-255 self test input
    assert oracle.shahash(b"dash").hex() == "f3319963720d2293ed504bb1f5c1c4a879147a34"


def test_edge_lengths(oracle, golden):
    cid = golden["edge_lengths"]["chunk_id"]
    for L, want in golden["edge_lengths"]["digests"].items():
        data = oracle.synth_chunk(cid, int(L))
        assert oracle.shahash(data.tobytes()).hex() == want, L


def test_fixture_files(oracle, golden, fixture_files):
    mk = golden["fixtures"]["make_chunks"]
    assert mk["tmp/C.tar"] == golden["fixtures"]["C.chunks_file"]
    for name, want in mk.items():
        data = np.frombuffer(fixture_files[name], np.uint8)
        n = (data.size + oracle.CHUNK_LEN - 1) // oracle.CHUNK_LEN
        off = np.arange(n, dtype=np.uint64) * oracle.CHUNK_LEN
        ln = np.minimum(data.size - off, oracle.CHUNK_LEN).astype(np.uint32)
        got = [d.tobytes().hex() for d in oracle.hash_batch(data, off, ln)]
        assert got == want, name


def test_config2_prefix(oracle):
    want = np.fromfile(os.path.join(os.path.dirname(__file__), "golden/synth_4096x512k.bin"),
                       np.uint8).reshape(-1, 20)
    n = 32
    data = oracle.synth_chunks(4096 - n, n)
    off = np.arange(n, dtype=np.uint64) * oracle.CHUNK_LEN
    got = oracle.hash_batch(data, off, np.full(n, oracle.CHUNK_LEN, np.uint32))
    assert np.array_equal(got, want[-n:])


def test_mixed_prefix(oracle, golden):
    want = np.fromfile(os.path.join(os.path.dirname(__file__), "golden/mixed_16384.bin"),
                       np.uint8).reshape(-1, 20)
    ln = oracle.mixed_lengths(golden["config5"]["chunks"])
    assert hashlib.sha1(ln.tobytes()).hexdigest() == golden["config5"]["lengths_sha1"]
    fixture = np.fromfile(os.path.join(os.path.dirname(__file__), "golden/mixed_16384_len.bin"), "<u4")
    assert np.array_equal(fixture, ln)
    for i in list(range(48)) + [16383]:
        d = oracle.shahash(oracle.synth_chunk(i, int(ln[i])).tobytes())
        assert d == want[i].tobytes(), i


def test_streaming_split_points(oracle):
    """Update() staging across non-64-aligned boundaries (sha.c:501-522)."""
    import ctypes as C
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, 5000, dtype=np.uint8).tobytes()
    L = oracle.lib()
    L.oracle_sha1_update.argtypes = [C.c_void_p, C.c_char_p, C.c_uint32]
    L.oracle_sha1_init.argtypes = [C.c_void_p]
    L.oracle_sha1_final.argtypes = [C.c_void_p, C.c_char_p]
    for cuts in ([1, 63, 64, 65, 1000], [7] * 50, [4999]):
        ctx = C.create_string_buffer(96)
        L.oracle_sha1_init(ctx)
        pos = 0
        for c in cuts:
            L.oracle_sha1_update(ctx, data[pos:pos + c], c)
            pos += c
        L.oracle_sha1_update(ctx, data[pos:], len(data) - pos)
        out = C.create_string_buffer(20)
        L.oracle_sha1_final(ctx, out)
        assert out.raw == hashlib.sha1(data).digest()


def test_random_lengths_vs_stdlib(oracle):
    rng = np.random.default_rng(11)
    for _ in range(200):
        n = int(rng.integers(0, 3000))
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert oracle.shahash(b) == hashlib.sha1(b).digest()


def test_synth_formula(oracle):
    """Synthetic corpus = splitmix64(seed ^ (c << 24) ^ w), little-endian."""
    c, L = 3, 40
    data = oracle.synth_chunk(c, L)
    for w in range(L // 8):
        v = oracle.splitmix64(oracle.SEED ^ (c << 24) ^ w)
        assert data[8 * w:8 * w + 8].tobytes() == v.to_bytes(8, "little")


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(__file__), "..", "oracle", "_ref",
                                                    "libsharef.so")),
                    reason="oracle/_ref (compiled reference) not built")
def test_restatement_matches_reference_build(oracle):
    rng = np.random.default_rng(3)
    lens = rng.integers(0, 200000, 64).astype(np.uint32)
    off = np.zeros(64, np.uint64)
    off[1:] = np.cumsum(lens.astype(np.uint64) + 13)[:-1]  # ragged, unaligned
    buf = rng.integers(0, 256, int(off[-1] + lens[-1] + 1), dtype=np.uint8)
    a = oracle.hash_batch(buf, off, lens, threads=4)
    b = oracle.hash_batch(buf, off, lens, threads=4, use_ref=True)
    assert np.array_equal(a, b)


class _Ctx(ctypes.Structure):
    """SHA1Context (sha.h:39-52), 96 bytes."""
    _fields_ = [("totalLength", ctypes.c_uint64), ("hash", ctypes.c_uint32 * 5),
                ("bufferLength", ctypes.c_uint32), ("buffer", ctypes.c_uint8 * 64)]


def long_message_contexts(seed=3):
    """Consistent mid-stream contexts whose message is >= 2^32 bytes long, so
    the 64-bit big-endian bit count SHA1Final appends (sha.c:540-543) has a
    non-zero high word: K whole blocks already compressed, r bytes staged."""
    rng = np.random.default_rng(seed)
    out = []
    for K in (1 << 26, 5 * (1 << 26) + 3, (1 << 40) + 12345, (1 << 55) - 1):
        for r in (0, 1, 55, 56, 63):
            c = _Ctx()
            c.totalLength = 8 * (64 * K + r)
            for i, w in enumerate(rng.integers(0, 1 << 32, 5, dtype=np.uint64)):
                c.hash[i] = int(w)
            c.bufferLength = r
            for i, b in enumerate(rng.integers(0, 256, 64, dtype=np.uint8)):
                c.buffer[i] = int(b)
            out.append(c)
    return out


def _final(fn, ctx):
    """Call a SHA1Final-shaped C function on a copy of ctx (a private
    prototype, so the library's own ctypes bindings are left alone)."""
    c = _Ctx.from_buffer_copy(bytes(ctx))
    d = (ctypes.c_uint8 * 20)()
    f = ctypes.cast(fn, ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p))
    f(ctypes.addressof(c), ctypes.addressof(d))
    return bytes(d), (c.totalLength, tuple(c.hash), c.bufferLength)


def test_final_64bit_bit_count_vs_reference(oracle):
    """The restatement's SHA1Final against the reference sha.c's on contexts
    of >= 4 GiB messages (bit count >= 2^35): same digest, same context left
    behind (chaining value, padded length, nothing staged)."""
    ref = oracle.ref_lib()
    if ref is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    for ctx in long_message_contexts():
        assert _final(oracle.lib().oracle_sha1_final, ctx) == _final(ref.SHA1Final, ctx), ctx.totalLength


def test_package_mixed_length_law(pkg, golden, oracle):
    """bench.py's config-5 legs draw lengths from the package's numpy restatement
    of the length law; it must reproduce the lengths the reference hashed for
    the golden files (16384 and the 4x batch of 65536), and the oracle's."""
    import hashlib
    for key in ("config5", "config5x4"):
        n = golden[key]["chunks"]
        ln = pkg.sha1chunk.mixed_lengths(n)
        assert hashlib.sha1(ln.tobytes()).hexdigest() == golden[key]["lengths_sha1"], key
        assert int(ln.astype(np.uint64).sum()) == golden[key]["total_bytes"]
    assert np.array_equal(pkg.sha1chunk.mixed_lengths(2000), oracle.mixed_lengths(2000))


def test_cpu_baseline_builds_time_the_same_digests(oracle):
    """bench.py's CPU baseline rows: the reference sha.c and
    the restatement, each -O2 and with the reference Makefile's flags, time a
    batch in memory on 1 and 2 threads and return the reference golden
    digests of config 2's corpus."""
    n, L = 4, oracle.CHUNK_LEN
    data = oracle.synth_chunks(0, n, L)
    off = np.arange(n, dtype=np.uint64) * L
    ln = np.full(n, L, np.uint32)
    want = np.fromfile(os.path.join(os.path.dirname(__file__), "golden", "synth_4096x512k.bin"),
                       np.uint8).reshape(-1, 20)[:n]
    kinds = ["port"] + (["reference"] if oracle.ref_lib("O2") is not None else [])
    for kind in kinds:
        for opt in ("O2", "O0"):
            for threads in (1, 2):
                secs, dig = oracle.time_batch(data, off, ln, threads, opt, kind)
                assert secs > 0 and np.array_equal(dig, want), (kind, opt, threads)
