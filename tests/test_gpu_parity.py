"""GPU parity: the HIP engine, called through the C ABI, against the oracle
and the reference's golden vectors.  Bit-exact everywhere (integer work)."""
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest

from conftest import default_env

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
PKG_DIR = os.path.join(ROOT, "congestion-control-with-bittorren_amd")
L512 = 524288

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(pkg):
    import torch
    assert torch.cuda.is_available(), "GPU tests need a device"
    assert pkg.device_count() >= 1, pkg.lib().sha1chunk_last_error()
    torch.cuda.set_device(0)
    pkg.set_device(0)
    return torch


def _agg(oracle, digests: np.ndarray) -> str:
    return oracle.digest_of_digests(digests).hex()


# ---------------------------------------------------------------- KATs ----
def test_kats_shahash(pkg, dev, golden):
    for name, kat in golden["kats"].items():
        data = bytes.fromhex(kat["input_hex"]) if "input_hex" in kat else \
            bytes.fromhex(kat["input_repeat"][0]) * kat["input_repeat"][1]
        assert pkg.shahash(data).hex() == kat["digest"], name


def test_kats_streaming_trio(pkg, dev, golden):
    # sha.c:560-614 self test: "abc", the 56-byte message, 1000 x 1000 'a'
    s = pkg.SHA1()
    s.update(b"abc")
    assert s.final().hex() == golden["kats"]["abc"]["digest"]
    s = pkg.SHA1()
    s.update(bytes.fromhex(golden["kats"]["nist56"]["input_hex"]))
    assert s.final().hex() == golden["kats"]["nist56"]["digest"]
    s = pkg.SHA1()
    for _ in range(1000):
        s.update(b"a" * 1000)
    assert s.final().hex() == golden["kats"]["million_a"]["digest"]


def test_final_64bit_bit_count(pkg, dev, oracle):
    """SHA1Final on contexts of >= 4 GiB messages (the 64-bit bit count's
    high word non-zero, sha.c:540-543; up to 2^61 bytes) through the device
    finish kernel: digest and the context left behind equal the reference
    sha.c's (oracle/_ref; the restatement where it was not built)."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_oracle import _final, long_message_contexts
    ref = oracle.ref_lib()
    want_fn = ref.SHA1Final if ref is not None else oracle.lib().oracle_sha1_final
    for ctx in long_message_contexts():
        assert _final(pkg.lib().SHA1Final, ctx) == _final(want_fn, ctx), ctx.totalLength


@pytest.mark.parametrize("kernel", ["auto", "lane", "fused", "split"])
def test_streaming_odd_splits(pkg, dev, oracle, kernel, monkeypatch):
    """SHA1Update/SHA1Final (sha.c:453-558) with the device compressing the
    whole blocks of each update on every kernel (update mode: IV or chained
    state in, raw state out, no padding)."""
    if kernel != "auto":
        monkeypatch.setenv("SHA1CHUNK_FORCE_KERNEL", kernel)
    rng = np.random.default_rng(9)
    data = rng.integers(0, 256, 20000, dtype=np.uint8).tobytes()
    for cuts in ([1, 63, 64, 65, 1000, 130], [7] * 40, [0, 19999]):
        s = pkg.SHA1()
        pos = 0
        for c in cuts:
            s.update(data[pos:pos + c])
            pos += c
        s.update(data[pos:])
        assert s.final() == oracle.shahash(data)
    # one large update (bulk stages) after an unaligned prefix
    big = rng.integers(0, 256, 3 * 524288 + 77, dtype=np.uint8).tobytes()
    s = pkg.SHA1()
    s.update(big[:5])
    s.update(big[5:])
    assert s.final() == oracle.shahash(big)


def test_edge_lengths_all_kernels(pkg, dev, oracle, golden):
    torch = dev
    cid = golden["edge_lengths"]["chunk_id"]
    want = golden["edge_lengths"]["digests"]
    lens = [int(k) for k in want]
    # host path (packs + AUTO kernel)
    buf = np.concatenate([oracle.synth_chunk(cid, L) for L in lens] + [np.zeros(1, np.uint8)])
    off = np.zeros(len(lens), np.uint64)
    off[1:] = np.cumsum(lens)[:-1]
    got = pkg.hash_batch(buf, off, lens)
    assert [d.tobytes().hex() for d in got] == [want[str(L)] for L in lens]
    # device path, each kernel, 128-aligned layout
    doff, total = pkg.sha1chunk.ragged_layout(lens)
    host = np.zeros(total + 128, np.uint8)
    for i, L in enumerate(lens):
        host[int(doff[i]):int(doff[i]) + L] = oracle.synth_chunk(cid, L)
    d_base = torch.from_numpy(host).cuda()
    d_off = torch.from_numpy(doff.astype(np.int64)).cuda()
    d_len = torch.tensor(lens, dtype=torch.int32).cuda()
    for k in ("lane", "fused", "split"):
        d_dig = torch.zeros((len(lens), 20), dtype=torch.uint8, device="cuda")
        pkg.hash_device(d_base, d_off, d_len, d_dig, kernel=k)
        torch.cuda.synchronize()
        got = [d.tobytes().hex() for d in d_dig.cpu().numpy()]
        assert got == [want[str(L)] for L in lens], k


# ------------------------------------------------------ reference files ----
def test_make_chunks_fixture_files(pkg, dev, golden, fixture_files, tmp_path):
    for name, want in golden["fixtures"]["make_chunks"].items():
        p = tmp_path / os.path.basename(name)
        p.write_bytes(fixture_files[name])
        got = [d.hex() for d in pkg.make_chunks(str(p))]
        assert got == want, name


def test_make_chunks_cli_reproduces_C_chunks(pkg, dev, golden, fixture_files, tmp_path):
    p = tmp_path / "C.tar"
    p.write_bytes(fixture_files["tmp/C.tar"])
    out = subprocess.run([os.path.join(PKG_DIR, "make-chunks"), str(p)], capture_output=True,
                         text=True, check=True).stdout
    want = "".join(f"{i} {h}\n" for i, h in enumerate(golden["fixtures"]["C.chunks_file"]))
    assert out == want  # tmp/C.chunks with CRLF stripped


@pytest.mark.parametrize("size", [0, 1, L512 - 1, L512, L512 + 1, 2 * L512, 2 * L512 + 55])
def test_make_chunks_file_sizes(pkg, dev, tmp_path, size):
    """make_chunks (chunk.c:15-27) and the CLI (make_chunks.c) on files at
    the chunk boundaries: an empty file has no chunks, a partial last chunk
    is hashed at its true length.  Checked against hashlib."""
    import hashlib
    rng = np.random.default_rng(size)
    data = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
    p = tmp_path / "f.bin"
    p.write_bytes(data)
    want = [hashlib.sha1(data[i:i + L512]).hexdigest() for i in range(0, size, L512)]
    assert [d.hex() for d in pkg.make_chunks(str(p))] == want
    out = subprocess.run([os.path.join(PKG_DIR, "make-chunks"), str(p)], capture_output=True,
                         text=True, check=True).stdout
    assert out == "".join(f"{i} {h}\n" for i, h in enumerate(want))


def test_make_chunks_slot_ring_wraps(pkg, dev, tmp_path):
    """The stream pipeline's ring of 3 pinned slots going round several
    times: SHA1CHUNK_STREAM_SLOT_MIB=16 (32 chunks per slot) on a ~100 MiB
    file with a ragged tail = 201 chunks in 7 slot fills, through
    make_chunks in a fresh process (the slot size is read once per process)
    and through the make-chunks CLI (whose own 128 MiB choice below 16 GiB
    the explicit variable overrides, make_chunks_main.c).  Every digest is
    compared with hashlib."""
    import hashlib
    size = 100 * 2**20 + 12345
    data = np.random.default_rng(16).integers(0, 256, size, dtype=np.uint8).tobytes()
    p = tmp_path / "ring.bin"
    p.write_bytes(data)
    want = [hashlib.sha1(data[i:i + L512]).hexdigest() for i in range(0, size, L512)]
    assert len(want) == 201
    env = dict(os.environ, SHA1CHUNK_STREAM_SLOT_MIB="16", SHA1CHUNK_STREAM_PIECE_MIB="4")
    code = ("import importlib, sys; m = importlib.import_module('congestion-control-with-bittorren_amd'); "
            "m.set_device(0); print('\\n'.join(d.hex() for d in m.make_chunks(sys.argv[1])))")
    r = subprocess.run([sys.executable, "-c", code, str(p)], capture_output=True, text=True,
                       env=env, cwd=ROOT, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == want
    r = subprocess.run([os.path.join(PKG_DIR, "make-chunks"), str(p)], capture_output=True,
                       text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout == "".join(f"{i} {h}\n" for i, h in enumerate(want))


@pytest.mark.parametrize("size,skip", [(100 * 2**20 + 12345, 0), (2 * L512 - 3, 0), (7 * L512 + 9, L512 + 5)])
def test_make_chunks_file_over_devices(pkg, dev, tmp_path, size, skip):
    """make_chunks on a regular file split over devices
    (SHA1CHUNK_FILE_DEVICES=all; SHA1CHUNK_VIRTUAL_DEVICES=3 gives three
    logical devices, each with its own pread pool, thread and pipeline, over
    the one GPU of the test box): contiguous chunk-aligned byte ranges, the
    digests in one array in file order.  A 201-chunk file with 16 MiB slots
    (every device's ring wraps), a 2-chunk file (fewer chunks than devices),
    and a stream opened part-way in (chunks start at the stream position,
    chunk.c:15-27 reads from where the FILE* is).  Through make_chunks in a
    fresh process and through the make-chunks CLI; every digest against
    hashlib."""
    import hashlib
    data = np.random.default_rng(size).integers(0, 256, size, dtype=np.uint8).tobytes()
    p = tmp_path / "multi.bin"
    p.write_bytes(data)
    want = [hashlib.sha1(data[i:i + L512]).hexdigest() for i in range(skip, size, L512)]
    env = dict(os.environ, SHA1CHUNK_VIRTUAL_DEVICES="3", SHA1CHUNK_FILE_DEVICES="all",
               SHA1CHUNK_STREAM_SLOT_MIB="16", SHA1CHUNK_STREAM_PIECE_MIB="4")
    code = ("import importlib, sys; m = importlib.import_module('congestion-control-with-bittorren_amd'); "
            "m.set_device(0); f = open(sys.argv[1], 'rb'); f.seek(int(sys.argv[2])); "
            "import os; d = m.make_chunks(f); print(os.lseek(f.fileno(), 0, os.SEEK_CUR)); "
            "print('\\n'.join(x.hex() for x in d))")
    r = subprocess.run([sys.executable, "-c", code, str(p), str(skip)], capture_output=True, text=True,
                       env=env, cwd=ROOT, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.split()
    assert int(lines[0]) == size  # the stream is left at the end, as a read() loop leaves it
    assert lines[1:] == want
    if skip == 0:
        r = subprocess.run([os.path.join(PKG_DIR, "make-chunks"), str(p)], capture_output=True,
                           text=True, env=env, timeout=120)
        assert r.returncode == 0, r.stderr
        assert r.stdout == "".join(f"{i} {h}\n" for i, h in enumerate(want))


@pytest.mark.parametrize("hint_chunks", [0, 1, 2, 4, 64])
def test_stream_pipeline_size_hints(pkg, dev, hint_chunks):
    """sha1chunk_hash_stream_sized with a size hint that is absent (0), too
    small (the reader delivers more: the one-slot path must hand over to the
    copy stream and the other slots mid-call), exact (4 chunks: one fill on
    slot 0's own stream, no other stream) or too large.  The reader returns
    short reads of odd sizes; every digest is checked with hashlib and the
    sink must see ascending, contiguous chunk indices (chunk.c:15-27 order)."""
    import ctypes as C
    import hashlib
    size = 3 * L512 + 777
    data = np.random.default_rng(hint_chunks + 7).integers(0, 256, size, dtype=np.uint8).tobytes()
    want = [hashlib.sha1(data[i:i + L512]).digest() for i in range(0, size, L512)]
    pos = [0]

    def reader(ctx, dst, n):
        k = min(n, size - pos[0], 100_003)
        C.memmove(dst, data[pos[0]:pos[0] + k], k)
        pos[0] += k
        return k

    got, firsts = [], []

    def sink(ctx, first, dig, count):  # (an assert here would not propagate through ctypes)
        firsts.append((first, len(got)))
        got.extend(bytes(dig[20 * j:20 * (j + 1)]) for j in range(count))

    rf, sf = pkg.sha1chunk.READER_FN(reader), pkg.sha1chunk.SINK_FN(sink)
    n = pkg.lib().sha1chunk_hash_stream_sized(rf, None, sf, None, hint_chunks * L512)
    assert n == len(want), pkg.lib().sha1chunk_last_error()
    assert all(f == k for f, k in firsts), firsts
    assert got == want


def test_reference_make_chunks_main_dropin(pkg, dev, golden, fixture_files, tmp_path):
    """The reference's own make_chunks.c main, unmodified, linked without
    chunk.o/sha.o against libsha1chunk.so (oracle/Makefile `dropin`, built in
    the container from /root/reference): its output on the reference's
    fixture files equals the reference's make-chunks output."""
    exe = os.path.join(ROOT, "oracle", "_ref", "dropin", "make-chunks")
    if not os.path.exists(exe):
        pytest.skip("drop-in make-chunks was not built (needs /root/reference at build time)")
    fixtures = {"tmp/C.tar": golden["fixtures"]["C.chunks_file"]}
    fixtures.update(golden["fixtures"]["make_chunks"])
    for name, want in fixtures.items():
        p = tmp_path / os.path.basename(name)
        p.write_bytes(fixture_files[name])
        r = subprocess.run([exe, str(p)], capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr
        assert r.stdout == "".join(f"{i} {h}\n" for i, h in enumerate(want)), name


def test_config1_make_chunks_cli(pkg, dev, golden, fixture_files, tmp_path):
    """BASELINE config 1 (make-chunks on tmp/C.tar, 4 chunks), every way the
    CLI can run here, each against tmp/C.chunks: the reference's own
    make-chunks built from its sources (oracle/_ref, CPU sha.c), the repo's
    CLI (the default routing, which hashes this 2 MiB file on the host; the
    kernels, SHA1CHUNK_HOST_SMALL=0; the explicit 4 MiB knob), and the
    reference main linked against the library (default and kernels).
    Prints the median wall time of 5 runs of each (process start included)."""
    p = tmp_path / "C.tar"
    p.write_bytes(fixture_files["tmp/C.tar"])
    want = "".join(f"{i} {h}\n" for i, h in enumerate(golden["fixtures"]["C.chunks_file"]))
    cli = os.path.join(PKG_DIR, "make-chunks")
    runs = {"repo_cli_default": (cli, None),  # the library's default routing: host for a <= 4 MiB file
            "repo_cli_device": (cli, {"SHA1CHUNK_HOST_SMALL": "0"}),
            "repo_cli_host_small": (cli, {"SHA1CHUNK_HOST_SMALL": "4194304"})}
    ref_exe = os.path.join(ROOT, "oracle", "_ref", "make-chunks")
    dropin = os.path.join(ROOT, "oracle", "_ref", "dropin", "make-chunks")
    if os.path.exists(ref_exe):
        runs["reference_sha_c"] = (ref_exe, {})
    if os.path.exists(dropin):
        runs["reference_main_dropin_default"] = (dropin, None)
        runs["reference_main_dropin_device"] = (dropin, {"SHA1CHUNK_HOST_SMALL": "0"})
    times = {}
    for name, (exe, extra) in runs.items():
        env = default_env() if extra is None else dict(os.environ, **extra)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            r = subprocess.run([exe, str(p)], capture_output=True, text=True, env=env, timeout=60)
            ts.append(time.perf_counter() - t0)
            assert r.returncode == 0, (name, r.stderr)
            # the reference prints CRLF-free "%d %s\n" lines (make_chunks.c:53)
            assert r.stdout.replace("\r\n", "\n") == want, (name, r.stdout)
        times[name] = round(sorted(ts)[2] * 1e3, 2)
    print("config1_cli_ms " + json.dumps(times))


def test_reference_receive_path_dropin(pkg, dev, golden, fixture_files, tmp_path):
    """The reference's own job.c (job_init's read_chunk + vec_common,
    populate_chunks_to_download, verify_hash) and utility.c vectors,
    unmodified, linked without chunk.o/sha.o against libsha1chunk.so
    (oracle/dropin_driver.c): every reassembled chunk of C.tar verifies (0),
    every corrupted copy is rejected (1), chunk ids come from the master
    chunk file, ownership from the has-chunk file.  Fixture files in the
    reference's CRLF format, master header sharing a line with chunk 0."""
    exe = os.path.join(ROOT, "oracle", "_ref", "dropin", "verify_driver")
    if not os.path.exists(exe):
        pytest.skip("drop-in driver was not built (needs /root/reference at build time)")
    hashes = golden["fixtures"]["C.chunks_file"]
    crlf = lambda lines: "".join(l + "\r\n" for l in lines).encode()
    data = tmp_path / "C.tar"
    data.write_bytes(fixture_files["tmp/C.tar"])
    get = tmp_path / "C.chunks"  # tmp/C.chunks
    get.write_bytes(crlf(f"{i} {h}" for i, h in enumerate(hashes)))
    master = tmp_path / "C.masterchunks"  # tmp/C.masterchunks layout
    master.write_bytes(crlf([f"File: {data} Chunks:0 {hashes[0]}"] +
                            [f"{i} {h}" for i, h in enumerate(hashes) if i]))
    has = tmp_path / "A.haschunks"  # tmp/A.haschunks: chunks 0, 1 of C
    has.write_bytes(crlf(f"{i} {h}" for i, h in enumerate(hashes[:2])))
    r = subprocess.run([exe, str(data), str(get), str(master), str(has)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert "COMMON 2" in lines
    assert [l for l in lines if l.startswith("TODO")] == \
        [f"TODO {h} {i} {int(i < 2)}" for i, h in enumerate(hashes)]
    assert [l for l in lines if l.startswith("VERIFY")] == [f"VERIFY {i} 0 1" for i in range(4)]
    # job.c:219-220 prints the computed and the expected hash for each check
    for h in hashes:
        assert f"calculated hash is {h}" in r.stdout


def test_verify_hash_semantics(pkg, dev, golden, fixture_files, capfd):
    data = fixture_files["tmp/C.tar"][:L512]
    good = golden["fixtures"]["C.chunks_file"][0]
    assert pkg.verify_hash(good, data) == 0
    bad = good[:-1] + ("0" if good[-1] != "0" else "1")
    assert pkg.verify_hash(bad, data) == 1
    out = capfd.readouterr().out
    # job.c:219-220 and chunk.c:179,182 stdout side effects
    assert f"calculated hash is {good}" in out
    assert "calculating chunk hash for a chunk of size 524288" in out
    assert f"the ascii of calculated hash is {good}" in out


def test_get_chunk_hash(pkg, dev, golden, fixture_files):
    data = fixture_files["tmp/C.tar"][L512:2 * L512]
    assert pkg.get_chunk_hash(data) == golden["fixtures"]["C.chunks_file"][1]


# -------------------------------------------------- BASELINE config 2 ----
@pytest.mark.parametrize("kernel", ["lane", "fused", "split", "auto"])
def test_config2_full_vs_reference(pkg, dev, oracle, golden, kernel):
    """4096 x 512 KiB device-resident, every digest vs the reference's."""
    torch = dev
    n = 4096
    buf = torch.empty(n * L512, dtype=torch.uint8, device="cuda")
    pkg.synth_fill_device(buf, 0, n, L512)
    dig = torch.zeros((n, 20), dtype=torch.uint8, device="cuda")
    pkg.hash_uniform_device(buf, L512, n, dig, kernel=kernel)
    torch.cuda.synchronize()
    want = np.fromfile(os.path.join(GOLDEN, "synth_4096x512k.bin"), np.uint8).reshape(-1, 20)
    got = dig.cpu().numpy()
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} mismatching chunks, first {bad[:8]}"
    assert _agg(oracle, got) == golden["config2"]["agg"]
    # the synthetic bytes themselves match the oracle's generator
    host = oracle.synth_chunks(4000, 3)
    assert np.array_equal(buf[4000 * L512:4003 * L512].cpu().numpy(), host)


def test_verify_device_flags_corruption(pkg, dev):
    torch = dev
    n = 256
    buf = torch.empty(n * L512, dtype=torch.uint8, device="cuda")
    pkg.synth_fill_device(buf, 0, n, L512)
    want = np.fromfile(os.path.join(GOLDEN, "synth_4096x512k.bin"), np.uint8).reshape(-1, 20)[:n]
    buf[5 * L512 + 12345] ^= 1  # flip one bit in chunk 5
    buf[200 * L512 + L512 - 1] ^= 0x80  # last byte of chunk 200
    dig = torch.zeros((n, 20), dtype=torch.uint8, device="cuda")
    pkg.hash_uniform_device(buf, L512, n, dig)
    mism = torch.zeros(n, dtype=torch.uint8, device="cuda")
    pkg.compare_device(dig, torch.from_numpy(want).cuda(), mism)
    torch.cuda.synchronize()
    assert sorted(np.nonzero(mism.cpu().numpy())[0].tolist()) == [5, 200]


# -------------------------------------------------- BASELINE config 5 ----
@pytest.mark.parametrize("kernel", ["lane", "fused", "split", "auto"])
def test_config5_mixed_lengths(pkg, dev, oracle, golden, kernel):
    torch = dev
    n = golden["config5"]["chunks"]
    lens = oracle.mixed_lengths(n)
    off, total = pkg.sha1chunk.ragged_layout(lens)
    d_base = torch.zeros(total + 128, dtype=torch.uint8, device="cuda")
    d_off = torch.from_numpy(off.astype(np.int64)).cuda()
    d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
    pkg.synth_fill_ragged_device(d_base, d_off, d_len, 0)
    # sorted (heaviest first) like the persistent dispatch wants, and unsorted
    dig = torch.zeros((n, 20), dtype=torch.uint8, device="cuda")
    pkg.hash_device(d_base, d_off, d_len, dig, kernel=kernel)
    torch.cuda.synchronize()
    want = np.fromfile(os.path.join(GOLDEN, "mixed_16384.bin"), np.uint8).reshape(-1, 20)
    got = dig.cpu().numpy()
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} mismatching chunks, first {bad[:8]} lens {lens[bad[:8]]}"
    assert _agg(oracle, got) == golden["config5"]["agg"]


def test_host_batch_mixed_subset(pkg, dev, oracle, golden):
    n = 700
    lens = oracle.mixed_lengths(n)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens.astype(np.uint64) + 3)[:-1]  # unaligned host offsets
    buf = np.zeros(int(off[-1]) + int(lens[-1]) + 3, np.uint8)
    for i in range(n):
        buf[int(off[i]):int(off[i]) + int(lens[i])] = oracle.synth_chunk(i, int(lens[i]))
    got = pkg.hash_batch(buf, off, lens)
    want = np.fromfile(os.path.join(GOLDEN, "mixed_16384.bin"), np.uint8).reshape(-1, 20)[:n]
    assert np.array_equal(got, want)
    mism = pkg.verify_batch(buf, off, lens, want)
    assert not mism.any()


# ---------------------------------------------------- unaligned / ragged ----
@pytest.mark.parametrize("kernel", ["lane", "fused", "split"])
def test_unaligned_device_offsets(pkg, dev, oracle, kernel):
    """Chunk starts at every byte alignment: fused/split waves that see a
    misaligned lane fall back to per-lane loads; digests must not change."""
    torch = dev
    rng = np.random.default_rng(21)
    n = 300
    lens = rng.integers(0, 300000, n).astype(np.uint32)
    lens[:64] = 262144 + rng.integers(0, 200, 64)  # one wave of long chunks
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(lens.astype(np.uint64) + rng.integers(0, 17, n).astype(np.uint64)
                        + 1)[: n - 1]
    off += 5
    host = rng.integers(0, 256, int(off[-1] + lens[-1]) + 64, dtype=np.uint8)
    want = oracle.hash_batch(host, off, lens)
    d_dig = torch.zeros((n, 20), dtype=torch.uint8, device="cuda")
    pkg.hash_device(torch.from_numpy(host).cuda(), torch.from_numpy(off.astype(np.int64)).cuda(),
                    torch.from_numpy(lens.astype(np.int32)).cuda(), d_dig, kernel=kernel)
    torch.cuda.synchronize()
    assert np.array_equal(d_dig.cpu().numpy(), want)


@pytest.mark.parametrize("kernel", ["lane", "fused", "split"])
def test_partial_wave_and_empty(pkg, dev, oracle, kernel):
    torch = dev
    for n in (1, 63, 65, 130):
        buf = torch.empty(n * 4096, dtype=torch.uint8, device="cuda")
        pkg.synth_fill_device(buf, 17, n, 4096)
        dig = torch.zeros((n, 20), dtype=torch.uint8, device="cuda")
        pkg.hash_uniform_device(buf, 4096, n, dig, kernel=kernel)
        torch.cuda.synchronize()
        host = oracle.synth_chunks(17, n, 4096)
        want = oracle.hash_batch(host, np.arange(n, dtype=np.uint64) * 4096, np.full(n, 4096, np.uint32))
        assert np.array_equal(dig.cpu().numpy(), want), n
    # zero chunks: nothing launched, nothing written
    empty = torch.zeros((1, 20), dtype=torch.uint8, device="cuda")
    pkg.hash_uniform_device(torch.zeros(1, dtype=torch.uint8, device="cuda"), 4096, 0, empty,
                            kernel=kernel)
    torch.cuda.synchronize()
    assert not empty.cpu().numpy().any()


@pytest.mark.parametrize("chunk_len", [65, 1001, 4097])
def test_uniform_odd_lengths_every_regime(pkg, dev, oracle, chunk_len):
    """The make_chunks layout (chunk i at i * chunk_len, chunk.c:15-27) with a
    length that is not a multiple of 16, so almost every chunk starts
    misaligned: AUTO at one group per CU (4-wave split), two per CU (the
    8-wave uniform shape, lane-per-chunk loads) and beyond (fused), plus each
    forced kernel at the middle size."""
    torch = dev
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    rng = np.random.default_rng(chunk_len)
    for n, kernels in ((64 * cus - 3, ("auto",)), (128 * cus - 5, ("auto", "lane", "fused", "split")),
                       (192 * cus + 17, ("auto",))):
        host = rng.integers(0, 256, n * chunk_len, dtype=np.uint8)
        want = oracle.hash_batch(host, np.arange(n, dtype=np.uint64) * chunk_len,
                                 np.full(n, chunk_len, np.uint32))
        buf = torch.from_numpy(host).cuda()
        for k in kernels:
            dig = torch.zeros((n, 20), dtype=torch.uint8, device="cuda")
            pkg.hash_uniform_device(buf, chunk_len, n, dig, kernel=k)
            torch.cuda.synchronize()
            assert np.array_equal(dig.cpu().numpy(), want), (n, k)


def test_chunk_past_4gib_bit_count(pkg, dev, oracle):
    """One chunk of 2^29 + 55 bytes: its bit count (sha.c:529-558, the 64-bit
    totalLength) needs 33 bits, so the high length word of the final block is
    1.  Device (AUTO) and host batch paths; the chunk exceeds a host slot and
    goes alone in a grown one."""
    torch = dev
    L = (1 << 29) + 55
    host = np.random.default_rng(29).integers(0, 256, L, dtype=np.uint8)
    want = oracle.hash_batch(host, np.zeros(1, np.uint64), np.array([L], np.uint32))[0].tobytes()
    dig = torch.zeros((1, 20), dtype=torch.uint8, device="cuda")
    pkg.hash_uniform_device(torch.from_numpy(host).cuda(), L, 1, dig)
    torch.cuda.synchronize()
    assert dig.cpu().numpy()[0].tobytes() == want
    got = pkg.hash_batch(host, np.zeros(1, np.uint64), np.array([L], np.uint32))
    assert got[0].tobytes() == want


def test_zero_length_chunks_device(pkg, dev, golden):
    torch = dev
    n = 70
    d_base = torch.zeros(256, dtype=torch.uint8, device="cuda")
    d_off = torch.zeros(n, dtype=torch.int64, device="cuda")
    d_len = torch.zeros(n, dtype=torch.int32, device="cuda")
    for k in ("lane", "fused", "split"):
        dig = torch.zeros((n, 20), dtype=torch.uint8, device="cuda")
        pkg.hash_device(d_base, d_off, d_len, dig, kernel=k)
        torch.cuda.synchronize()
        assert all(d.tobytes().hex() == golden["kats"]["empty"]["digest"] for d in dig.cpu().numpy())


# -------------------------------------------- larger configs (properties) ----
def test_config4_shard_on_one_gpu(pkg, dev, oracle, golden):
    """BASELINE config 4 shard: rank r of 8 hashes chunks [32768 r, 32768 (r+1))."""
    torch = dev
    per = 262144 // 8
    r = 1
    buf = torch.empty(per * L512, dtype=torch.uint8, device="cuda")
    pkg.synth_fill_device(buf, r * per, per, L512)
    dig = torch.zeros((per, 20), dtype=torch.uint8, device="cuda")
    pkg.hash_uniform_device(buf, L512, per, dig)
    torch.cuda.synchronize()
    assert _agg(oracle, dig.cpu().numpy()) == golden["config4"]["shard_aggs"]["8"][r]
    del buf


def test_config3_device_resident_aggregate(pkg, dev, oracle, golden):
    """All 65536 x 512 KiB chunks resident in HBM (32 GiB): digest-of-digests
    and the sampled digests equal the reference's."""
    torch = dev
    n = 65536
    buf = torch.empty(n * L512, dtype=torch.uint8, device="cuda")
    pkg.synth_fill_device(buf, 0, n, L512)
    dig = torch.zeros((n, 20), dtype=torch.uint8, device="cuda")
    pkg.hash_uniform_device(buf, L512, n, dig)
    torch.cuda.synchronize()
    got = dig.cpu().numpy()
    for i, h in golden["config3"]["sample"].items():
        assert got[int(i)].tobytes().hex() == h, i
    assert _agg(oracle, got) == golden["config3"]["agg"]
    del buf


def test_config4_whole_on_one_gpu(pkg, dev, oracle, golden):
    """The largest BASELINE corpus, all 262144 x 512 KiB chunks (128 GiB)
    resident on one GPU, hashed in one launch (fused kernel regime): the
    digest-of-digests and every per-rank shard aggregate of the 1/2/4/8-way
    splits equal the reference's."""
    torch = dev
    n = 262144
    buf = torch.empty(n * L512, dtype=torch.uint8, device="cuda")
    pkg.synth_fill_device(buf, 0, n, L512)
    dig = torch.zeros((n, 20), dtype=torch.uint8, device="cuda")
    pkg.hash_uniform_device(buf, L512, n, dig)
    torch.cuda.synchronize()
    del buf
    torch.cuda.empty_cache()
    got = dig.cpu().numpy()
    assert _agg(oracle, got) == golden["config4"]["agg"]
    for N, aggs in golden["config4"]["shard_aggs"].items():
        per = n // int(N)
        assert [_agg(oracle, got[r * per:(r + 1) * per]) for r in range(int(N))] == aggs, N
    # and bench.py's weak-scaling ranks (4096 chunks each)
    assert [_agg(oracle, got[r * 4096:(r + 1) * 4096]) for r in range(8)] == golden["weak4096"]


def test_host_batch_all_devices(pkg, dev, oracle, golden):
    n = 512
    host = oracle.synth_chunks(0, n)
    off = np.arange(n, dtype=np.uint64) * L512
    got = pkg.hash_batch(host, off, np.full(n, L512, np.uint32), all_devices=True)
    want = np.fromfile(os.path.join(GOLDEN, "synth_4096x512k.bin"), np.uint8).reshape(-1, 20)[:n]
    assert np.array_equal(got, want)


# ------------------------------------------------------- verify queue ----
def test_host_paths_under_asan(pkg, dev):
    """Every host path of the library (batch pipelines, pinned staging, part
    pools, verify queue with growth, streaming trio, make_chunks(FILE*) on one
    and on two (virtual) devices,
    get_chunk_hash/verify_hash, the device ragged path's sort and mixed-kernel
    planning with forced and malformed plans) under host AddressSanitizer + UBSan
    (`make asan`: csrc/asan_driver.c against build-asan/libsha1chunk.so,
    built on the CPU beforehand like every other binary).  Device code is
    not instrumented; any host report makes the driver exit non-zero."""
    exe = os.path.join(PKG_DIR, "build-asan", "asan_driver")
    assert os.path.exists(exe), "run `make -C congestion-control-with-bittorren_amd asan` first"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               SHA1CHUNK_VIRTUAL_DEVICES="2")  # make_chunks split over two devices too
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0 and "asan-driver ok" in r.stdout, (r.stdout[-1500:], r.stderr[-3000:])
    # again with the opt-in host small-call path (csrc/sha1_host.c under
    # ASan/UBSan too): calls of <= 512 KiB hash on the host, so the driver's
    # shahash-vs-make_chunks checks now compare host digests with device ones
    env["SHA1CHUNK_HOST_SMALL"] = "524288"
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0 and "asan-driver ok" in r.stdout, (r.stdout[-1500:], r.stderr[-3000:])


_ALL_DEVICES_SCRIPT = r"""
import hashlib, importlib, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
pkg = importlib.import_module("congestion-control-with-bittorren_amd")
assert pkg.device_count() == int(sys.argv[2]), pkg.device_count()
rng = np.random.default_rng(31)
n = 700
lens = rng.integers(0, 300000, n).astype(np.uint32)
lens[:64] = 524288
lens[100:110] = 0
off = np.zeros(n, np.uint64)
off[1:] = np.cumsum(lens.astype(np.uint64) + rng.integers(0, 9, n).astype(np.uint64))[: n - 1]
buf = rng.integers(0, 256, int(off[-1] + lens[-1]) + 16, dtype=np.uint8)
want = np.array([np.frombuffer(hashlib.sha1(buf[int(o):int(o) + int(l)].tobytes()).digest(), np.uint8)
                 for o, l in zip(off, lens)])
got = pkg.hash_batch(buf, off, lens, all_devices=True)
assert np.array_equal(got, want), np.nonzero((got != want).any(axis=1))[0][:8]
assert np.array_equal(pkg.hash_batch(buf, off, lens), want)
print("all-devices ok")
"""


def test_host_batch_all_devices_virtual(pkg, dev, tmp_path):
    """SHA1CHUNK_ALL_DEVICES with several devices (byte-balanced
    slices, one host thread and pipeline per device, no collective), run on
    a one-GPU box through SHA1CHUNK_VIRTUAL_DEVICES=3 (three logical devices,
    each with its own streams and slots, over the physical one), in a child
    process because the device probe happens once per process.  Digests are
    checked against hashlib."""
    script = tmp_path / "alldev.py"
    script.write_text(_ALL_DEVICES_SCRIPT)
    env = dict(os.environ, SHA1CHUNK_VIRTUAL_DEVICES="3")
    r = subprocess.run([sys.executable, str(script), ROOT, "3"], capture_output=True, text=True, env=env,
                       timeout=120)
    assert r.returncode == 0 and "all-devices ok" in r.stdout, r.stdout + r.stderr


@pytest.fixture(params=["batch", "persistent"])
def vq_mode(request, monkeypatch):
    """The verify queue's two implementations: batch launches, and the
    persistent drain kernel reading a pinned host ring (SHA1CHUNK_VQ_MODE)."""
    monkeypatch.setenv("SHA1CHUNK_VQ_MODE", request.param)
    return request.param


def test_verify_queue_receive_path(pkg, dev, oracle, golden, fixture_files, vq_mode):
    """Batched async verify (packet_handler.c:469-472 -> job.c:217): every
    result comes back exactly once with verify_hash's 0/1 convention."""
    rng = np.random.default_rng(77)
    chunks, expected, want = [], [], {}
    ctar = fixture_files["tmp/C.tar"]
    for i in range(4):  # the reference's own fixture chunks
        chunks.append(ctar[i * L512:(i + 1) * L512])
        expected.append(golden["fixtures"]["C.chunks_file"][i])
    lens = oracle.mixed_lengths(150)
    for i in range(150):  # ragged, smaller-than-chunk payloads too
        d = oracle.synth_chunk(i, int(min(lens[i], L512))).tobytes()
        chunks.append(d)
        expected.append(oracle.shahash(d).hex())
    for t, (c, e) in enumerate(zip(chunks, expected)):
        bad = rng.random() < 0.2
        if bad:
            e = ("0" if e[0] != "0" else "1") + e[1:]
        want[1000 + t] = 1 if bad else 0
    got = {}
    with pkg.VerifyQueue(batch=32, max_chunk_len=L512) as q:
        for t, (c, e) in enumerate(zip(chunks, expected)):
            e2 = e if want[1000 + t] == 0 else ("0" if e[0] != "0" else "1") + e[1:]
            q.submit(c, e2, 1000 + t)
            for tag, m in q.poll():
                assert tag not in got
                got[tag] = m
        for tag, m in q.poll(wait=True):
            assert tag not in got
            got[tag] = m
        assert q.pending == 0
    assert got == want


@pytest.mark.parametrize("grow", ["1", "0"])
def test_verify_queue_full_batches_drain_by_polling(pkg, dev, monkeypatch, grow, vq_mode):
    """Submissions in whole batches come back through non-blocking poll()
    alone (no flush, no wait): a batch held back to grow while two earlier
    ones are on the device is launched by a later poll once one finishes."""
    import hashlib
    import time
    monkeypatch.setenv("SHA1CHUNK_VQ_GROW", grow)
    rng = np.random.default_rng(5)
    bufs = [rng.integers(0, 256, 4096 + 64 * k, dtype=np.uint8).tobytes() for k in range(16)]
    batch, n = 8, 8 * 7
    want, got = {}, {}
    with pkg.VerifyQueue(batch=batch, max_chunk_len=L512) as q:
        for t in range(n):
            b = bufs[t % len(bufs)]
            d = hashlib.sha1(b).digest()
            if t % 5 == 3:
                d = bytes([d[0] ^ 0x80]) + d[1:]
            want[t] = 1 if t % 5 == 3 else 0
            q.submit(b, d, t)
        t0 = time.time()
        while len(got) < n and time.time() - t0 < 30:
            for tag, m in q.poll():
                assert tag not in got
                got[tag] = m
            time.sleep(0.001)
        assert q.pending == 0
    assert got == want


# ------------------------------------- sender verify + master index ----
_VERIFY_DRIVER = r'''
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <fcntl.h>
#include <unistd.h>
#include "chunk_hash.h"
/* argv: file idx hex [idx hex ...] -> verify_chunk_hash each pair in order;
 * the pair "W src" instead rewrites the file in place with src's bytes (same
 * size) and puts its old atime/mtime back, as a copy tool preserving times
 * would */
static void rewrite_keep_mtime(const char *dst, const char *src) {
    struct stat st;
    static char buf[1 << 20];
    int in = open(src, O_RDONLY), out = open(dst, O_WRONLY);
    if (in < 0 || out < 0 || fstat(out, &st)) exit(3);
    ssize_t n;
    while ((n = read(in, buf, sizeof buf)) > 0)
        if (write(out, buf, (size_t)n) != n) exit(3);
    struct timespec t[2] = {st.st_atim, st.st_mtim};
    if (futimens(out, t)) exit(3);
    close(in);
    close(out);
}
int main(int argc, char **argv) {
    FILE *f = fopen(argv[1], "r");
    if (!f) return 2;
    for (int i = 2; i + 1 < argc; i += 2) {
        if (!strcmp(argv[i], "W")) {
            rewrite_keep_mtime(argv[1], argv[i + 1]);
            printf("rewrote\n");
            continue;
        }
        verify_chunk_hash(f, argv[i + 1], (size_t)atoll(argv[i]));
        printf("ok %s pos %ld\n", argv[i], ftell(f));
    }
    fclose(f);
    return 0;
}
'''


@pytest.fixture(scope="module")
def verify_driver(tmp_path_factory):
    d = tmp_path_factory.mktemp("vdrv")
    src = d / "vdrv.c"
    src.write_text(_VERIFY_DRIVER)
    exe = d / "vdrv"
    subprocess.run(["gcc", "-O1", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe),
                    "-L", PKG_DIR, "-lsha1chunk", f"-Wl,-rpath,{PKG_DIR}"], check=True)
    return str(exe)


def _run_verify(exe, path, pairs, index=True, settle_ms="0"):
    # settle 0: the index serves files changed just now too (the tests write
    # their master files a moment before the driver starts)
    env = dict(os.environ, SHA1CHUNK_MASTER_INDEX="1" if index else "0",
               SHA1CHUNK_MASTER_SETTLE_MS=settle_ms)
    args = [exe, path] + [x for i, h in pairs for x in (str(i), h)]
    return subprocess.run(args, capture_output=True, text=True, env=env)


def test_verify_chunk_hash_master_index(pkg, dev, golden, fixture_files, verify_driver, tmp_path):
    """chunk.c:204-217 as the sender calls it per GET (packet_handler.c:434):
    the C.tar fixture chunks, repeated so the master-file index serves the
    later calls; stdout and the stream position match the per-call path."""
    import hashlib
    p = tmp_path / "C.tar"
    p.write_bytes(fixture_files["tmp/C.tar"])
    want = golden["fixtures"]["C.chunks_file"]
    pairs = [(i, want[i]) for i in (0, 3, 1, 2, 2, 0, 3)]
    # a request past EOF hashes a zero chunk (calloc'd buffer, nothing read)
    pairs.append((5, hashlib.sha1(bytes(L512)).hexdigest()))
    a = _run_verify(verify_driver, str(p), pairs, index=True)
    b = _run_verify(verify_driver, str(p), pairs, index=False)
    assert a.returncode == 0, a.stderr
    assert b.returncode == 0, b.stderr
    assert a.stdout == b.stdout
    assert a.stdout.count("the ascii of calculated hash is") == len(pairs)


def test_verify_chunk_hash_ragged_master_and_mismatch(pkg, dev, oracle, verify_driver, tmp_path):
    """A master file whose last chunk is short: the verify hashes it zero-
    padded to CHUNK_LEN (both paths); a wrong hash served from the index
    still exits(-1) with the reference's message."""
    import hashlib
    size = 3 * L512 + 123457
    data = oracle.synth_chunks(900, 4, L512).tobytes()[:size]
    p = tmp_path / "master.dat"
    p.write_bytes(data)
    padded = data + bytes(4 * L512 - size)
    hexes = [hashlib.sha1(padded[i * L512:(i + 1) * L512]).hexdigest() for i in range(4)]
    pairs = [(3, hexes[3]), (0, hexes[0]), (3, hexes[3]), (2, hexes[2]), (1, hexes[1])]
    a = _run_verify(verify_driver, str(p), pairs, index=True)
    b = _run_verify(verify_driver, str(p), pairs, index=False)
    assert a.returncode == 0 and b.returncode == 0, (a.stderr, b.stderr)
    assert a.stdout == b.stdout
    bad = hexes[1][:-1] + ("0" if hexes[1][-1] != "0" else "1")
    c = _run_verify(verify_driver, str(p), [(0, hexes[0]), (2, hexes[2]), (1, bad)], index=True)
    assert c.returncode == 255
    assert "Unmatched chunk hashes" in c.stderr and hexes[1] in c.stderr
    assert c.stdout.count("ok ") == 2
    # the file changes under the peer: the index is rebuilt, not reused
    data2 = bytearray(data)
    data2[L512 + 5] ^= 0xFF
    p.write_bytes(bytes(data2))
    os.utime(p, ns=(1, 1))
    new1 = hashlib.sha1(bytes(data2[L512:2 * L512])).hexdigest()
    d = _run_verify(verify_driver, str(p), [(1, new1), (1, new1), (0, hexes[0])], index=True)
    assert d.returncode == 0, d.stderr


def test_verify_chunk_hash_index_default_routing(pkg, dev, oracle, verify_driver, tmp_path):
    """Round 6: the master index is built through sha1chunk_hash_fd (the
    parallel pread pipeline) and a short last chunk re-hashed zero-padded.
    A 9-chunk master with a ragged tail (above the 4 MiB host cut, so the
    default routing builds the table on the kernels and pads the tail on the
    host), every chunk requested in a scattered order: the same stdout and
    stream positions as the per-call path, every digest the zero-padded
    hashlib one, and a wrong digest served from the table still exits(-1)."""
    import hashlib
    size = 9 * L512 + 77777
    data = oracle.synth_chunks(1200, 10, L512).tobytes()[:size]
    p = tmp_path / "master9.dat"
    p.write_bytes(data)
    padded = data + bytes(10 * L512 - size)
    hexes = [hashlib.sha1(padded[i * L512:(i + 1) * L512]).hexdigest() for i in range(10)]
    order = [9, 0, 9, 4, 8, 1, 7, 2, 6, 3, 5, 9]
    pairs = [(i, hexes[i]) for i in order]

    def run(index, extra=()):
        env = default_env(SHA1CHUNK_MASTER_INDEX="1" if index else "0", SHA1CHUNK_MASTER_SETTLE_MS="0")
        args = [verify_driver, str(p)] + [x for i, h in list(pairs) + list(extra) for x in (str(i), h)]
        return subprocess.run(args, capture_output=True, text=True, env=env, timeout=120)

    a, b = run(True), run(False)
    assert a.returncode == 0 and b.returncode == 0, (a.stderr, b.stderr)
    assert a.stdout == b.stdout and a.stdout.count("ok ") == len(pairs)
    bad = hexes[4][:-1] + ("0" if hexes[4][-1] != "0" else "1")
    c = run(True, [(4, bad)])
    assert c.returncode == 255 and "Unmatched chunk hashes" in c.stderr
    assert c.stdout.count("ok ") == len(pairs)


@pytest.mark.parametrize("settle_ms", ["0", "2000"])
def test_verify_chunk_hash_index_not_stale(pkg, dev, oracle, verify_driver, tmp_path, settle_ms):
    """The sender re-verifies every GET against the master file (chunk.c:
    204-217).  After the index is built (2nd verify), the file is rewritten in
    place, same size, with its old mtime put back: the stale hash of the
    changed chunk must now fail with exit(-1) (the index is keyed on ctime
    too, and a file changed less than the settle time ago is re-hashed per
    call), and the new hash must pass."""
    import hashlib
    data = oracle.synth_chunks(700, 3, L512).tobytes()
    p = tmp_path / "master.dat"
    p.write_bytes(data)
    os.utime(p, ns=(10**18, 10**18))
    data2 = bytearray(data)
    data2[L512 + 77] ^= 0x01
    q = tmp_path / "new.dat"
    q.write_bytes(bytes(data2))
    old = [hashlib.sha1(data[i * L512:(i + 1) * L512]).hexdigest() for i in range(3)]
    new1 = hashlib.sha1(bytes(data2[L512:2 * L512])).hexdigest()
    seq = [(0, old[0]), (1, old[1]), (2, old[2]), (1, old[1]), ("W", str(q))]
    r = _run_verify(verify_driver, str(p), seq + [(1, old[1])], settle_ms=settle_ms)
    assert r.returncode == 255, (r.stdout, r.stderr)
    assert "Unmatched chunk hashes" in r.stderr and new1 in r.stderr
    assert r.stdout.count("ok ") == 4 and "rewrote" in r.stdout
    assert os.stat(p).st_mtime_ns == 10**18
    p.write_bytes(data)
    os.utime(p, ns=(10**18, 10**18))
    r = _run_verify(verify_driver, str(p), seq + [(1, new1), (0, old[0]), (1, new1)], settle_ms=settle_ms)
    assert r.returncode == 0, r.stderr
    assert r.stdout.count("ok ") == 7


_MAKE_CHUNKS_DRIVER = r'''
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include "chunk_hash.h"
/* argv: file skip_bytes -> make_chunks from the FILE* after fread(skip) */
int main(int argc, char **argv) {
    FILE *f = fopen(argv[1], "r");
    size_t skip = (size_t)atoll(argv[2]);
    char *tmp = malloc(skip + 1);
    if (!f || fread(tmp, 1, skip, f) != skip) return 2;
    uint8_t *store = malloc(20 * 64), *h[64];
    for (int i = 0; i < 64; ++i) h[i] = store + 20 * i;
    int n = make_chunks(f, h);
    char hex[41];
    for (int i = 0; i < n; ++i) { binary2hex(h[i], 20, hex); printf("%d %s\n", i, hex); }
    printf("eof %d\n", fgetc(f) == EOF);
    return 0;
}
'''


def test_make_chunks_from_stream_position(pkg, dev, golden, fixture_files, tmp_path):
    """chunk.c:15-27 hashes from the FILE*'s current position to EOF, even
    after stdio has buffered ahead of it."""
    src = tmp_path / "mc.c"
    src.write_text(_MAKE_CHUNKS_DRIVER)
    exe = tmp_path / "mc"
    subprocess.run(["gcc", "-O1", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe),
                    "-L", PKG_DIR, "-lsha1chunk", f"-Wl,-rpath,{PKG_DIR}"], check=True)
    p = tmp_path / "C.tar"
    p.write_bytes(fixture_files["tmp/C.tar"])
    want = golden["fixtures"]["C.chunks_file"]
    out = subprocess.run([str(exe), str(p), str(L512)], capture_output=True, text=True, check=True).stdout
    assert out == "".join(f"{i} {h}\n" for i, h in enumerate(want[1:])) + "eof 1\n"
    # an unaligned start: chunks are cut from the position, not the file start
    import hashlib
    data = fixture_files["tmp/C.tar"][1000:]
    exp = [hashlib.sha1(data[i:i + L512]).hexdigest() for i in range(0, len(data), L512)]
    out = subprocess.run([str(exe), str(p), "1000"], capture_output=True, text=True, check=True).stdout
    assert out == "".join(f"{i} {h}\n" for i, h in enumerate(exp)) + "eof 1\n"


@pytest.mark.parametrize("unit", [1, 4, 11])
def test_every_split_shape_ragged(pkg, dev, oracle, unit, monkeypatch):
    """Every split-kernel shape the product library builds (SHA1CHUNK_SPLIT_UNIT
    forces it: 1-block units, 4-block units with two producers, the 8-wave
    two-pair layout) on ragged lengths with byte-misaligned starts, a partial
    last workgroup and a lane-count that is not a multiple of 64: bit-exact
    vs the oracle.  (The round-1 study's other shapes live in the A/B build
    only, `make ab`.)"""
    torch = dev
    monkeypatch.setenv("SHA1CHUNK_SPLIT_UNIT", str(unit))
    rng = np.random.default_rng(1000 + unit)
    # 333 chunks: 6 groups of 64, the last one partial; 300: 5 groups, so a
    # two-group workgroup's second group has no valid lane at all
    for n, aligned in ((333, True), (333, False), (300, True)):
        lens = rng.integers(0, 40000, n).astype(np.uint32)
        lens[:140] = 65536 + rng.integers(0, 130, 140)   # two waves of long chunks
        lens[5] = 0
        lens[6], lens[7], lens[8] = 55, 56, 64
        # aligned: every start on a 64-byte boundary (the bulk 16-byte load path)
        step = ((lens.astype(np.uint64) + 63) // 64 * 64 + 64 if aligned
                else lens.astype(np.uint64) + rng.integers(1, 40, n).astype(np.uint64))
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(step)[: n - 1]
        host = rng.integers(0, 256, int(off[-1] + lens[-1]) + 64, dtype=np.uint8)
        want = oracle.hash_batch(host, off, lens)
        d_dig = torch.zeros((n, 20), dtype=torch.uint8, device="cuda")
        pkg.hash_device(torch.from_numpy(host).cuda(), torch.from_numpy(off.astype(np.int64)).cuda(),
                        torch.from_numpy(lens.astype(np.int32)).cuda(), d_dig, kernel="split")
        torch.cuda.synchronize()
        got = d_dig.cpu().numpy()
        bad = np.nonzero((got != want).any(axis=1))[0]
        assert bad.size == 0, f"unit {unit} n={n} aligned={aligned}: {bad.size} bad, first {bad[:8]}"


def test_unbuilt_split_shape_fails_loudly(pkg, dev, monkeypatch):
    """Forcing a split shape that only the A/B build holds (here the round-1
    study's 3-block units) is an error, not a silent run of another kernel."""
    torch = dev
    monkeypatch.setenv("SHA1CHUNK_SPLIT_UNIT", "3")
    buf = torch.zeros(64 * 4096, dtype=torch.uint8, device="cuda")
    dig = torch.zeros((64, 20), dtype=torch.uint8, device="cuda")
    with pytest.raises(pkg.Sha1ChunkError, match="not in this library"):
        pkg.hash_uniform_device(buf, 4096, 64, dig, kernel="split")
