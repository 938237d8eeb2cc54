"""CPU: chunk-file parse/emit on files of the reference's
formats, built from the reference's own chunk digests (golden.json
fixtures.C.chunks_file = tmp/C.chunks): CRLF ``idx hex`` lines as in
tmp/*.chunks and tmp/*.haschunks, and the master-chunk layout of
tmp/C.masterchunks whose header shares a line with chunk 0."""
import importlib

import pytest


@pytest.fixture(scope="module")
def cf():
    return importlib.import_module("congestion-control-with-bittorren_amd.chunkfile")


@pytest.fixture(scope="module")
def hashes(golden):
    return golden["fixtures"]["C.chunks_file"]


def _crlf(lines):
    return "".join(l + "\r\n" for l in lines)


def test_write_chunks_matches_make_chunks_output(cf, hashes, tmp_path):
    p = tmp_path / "C.chunks"
    n = cf.write_chunks(p, [bytes.fromhex(h) for h in hashes])
    assert n == 4
    # make_chunks.c:50 format; the shipped tmp/C.chunks is this with CRLF
    assert p.read_bytes() == "".join(f"{i} {h}\n" for i, h in enumerate(hashes)).encode()


def test_read_chunk_crlf_keeps_cr_like_reference(cf, hashes, tmp_path, capsys):
    p = tmp_path / "A.chunks"
    p.write_bytes(_crlf(f"{i} {h}" for i, h in enumerate(hashes[:2])).encode())
    got = cf.read_chunk(p)
    assert got == [h + "\r" for h in hashes[:2]]
    assert [g[:40] for g in got] == hashes[:2]
    q = tmp_path / "lf.chunks"
    cf.write_chunks(q, [bytes.fromhex(h) for h in hashes])
    assert cf.read_chunk(q) == hashes
    assert capsys.readouterr().out == ""


def test_read_chunk_comment_lines(cf, hashes, tmp_path, capsys):
    p = tmp_path / "m.chunks"
    p.write_text("# my chunks\n0 " + hashes[0] + "\nnot a chunk line\n1 " + hashes[1] + "\n")
    assert cf.read_chunk(p) == hashes[:2]
    assert capsys.readouterr().out.count("Comment line in chunk file\n") == 2


def test_find_idx_in_haschunks_and_master(cf, hashes, tmp_path):
    has = tmp_path / "B.haschunks"  # tmp/B.haschunks: chunks 2, 3 of C
    has.write_bytes(_crlf([f"2 {hashes[2]}", f"3 {hashes[3]}"]).encode())
    assert cf.find_chunk_idx_from_hash(hashes[3], has) == 3
    assert cf.find_chunk_idx_from_hash(hashes[2], has) == 2
    master = tmp_path / "C.masterchunks"  # header and chunk 0 on one line
    master.write_bytes(_crlf([f"File: /tmp/C.tar Chunks:0 {hashes[0]}"] +
                             [f"{i} {h}" for i, h in enumerate(hashes) if i]).encode())
    for i, h in enumerate(hashes):
        assert cf.find_chunk_idx_from_hash(h, master) == i
    with pytest.raises(KeyError):
        cf.find_chunk_idx_from_hash("0" * 40, master)


# ---- the C versions the peer links (csrc/chunk_file.c in libsha1chunk.so) ----
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "congestion-control-with-bittorren_amd")

# A peer-side caller: its own vector + vec_add with utility.c:14-34's
# semantics (copy ele_size bytes, double on growth), CHUNK_HASH_SIZE = 45
# (constants.h:13).  Prints every element as hex over all ele_size bytes,
# then the index of each query hash, then seek offsets.
_DRIVER = r'''
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
    for (int i = 0; i < v.len; ++i) {
        printf("E ");
        for (int b = 0; b < v.ele_size; ++b) printf("%02x", ((unsigned char *)v.val)[i * v.ele_size + b]);
        printf("\n");
    }
    for (int q = 3; q < argc; ++q) printf("I %zd\n", (ssize_t)find_chunk_idx_from_hash(argv[q], argv[2]));
    FILE *f = fopen(argv[1], "r");
    seek_to_chunk_pos(f, 9000);  /* 9000 x 512 KiB > 4 GiB: no uint32 wrap */
    printf("S %lld\n", (long long)ftello(f));
    seek_to_packet_pos(f, 3, 7);
    printf("S %lld\n", (long long)ftello(f));
    fclose(f);
    return 0;
}
'''


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    subprocess.run(["make", "-s", "-C", PKG_DIR], check=True)
    d = tmp_path_factory.mktemp("chunkfile_c")
    (d / "drv.c").write_text(_DRIVER)
    exe = d / "drv"
    subprocess.run(["gcc", "-Wall", "-I", os.path.join(ROOT, "include"), str(d / "drv.c"), "-o",
                    str(exe), "-L", PKG_DIR, "-lsha1chunk", f"-Wl,-rpath,{PKG_DIR}"], check=True)
    return exe


def _run(driver, chunks, master, *queries):
    r = subprocess.run([str(driver), str(chunks), str(master), *queries], capture_output=True,
                       text=True, check=True)
    lines = r.stdout.splitlines()
    elems = [bytes.fromhex(l[2:]) for l in lines if l.startswith("E ")]
    idx = [int(l[2:]) for l in lines if l.startswith("I ")]
    seeks = [int(l[2:]) for l in lines if l.startswith("S ")]
    return elems, idx, seeks, r.stdout.count("Comment line in chunk file\n")


def test_c_read_chunk_and_find_idx_match_python(cf, hashes, tmp_path, driver, capsys):
    files = {
        "crlf": _crlf(f"{i} {h}" for i, h in enumerate(hashes)),
        "lf": "".join(f"{i} {h}\n" for i, h in enumerate(hashes)),
        "comments": "# my chunks\n0 " + hashes[0] + "\nnot a chunk\n7\n\n1 " + hashes[1] + "\n",
        "master": _crlf([f"File: /tmp/C.tar Chunks:0 {hashes[0]}"] +
                        [f"{i} {h}" for i, h in enumerate(hashes) if i]),
    }
    queries = hashes + ["0" * 40]
    for name, text in files.items():
        p = tmp_path / f"{name}.chunks"
        p.write_bytes(text.encode())
        elems, idx, seeks, comments = _run(driver, p, p, *queries)
        want = cf.read_chunk(p)
        assert comments == capsys.readouterr().out.count("Comment line in chunk file\n")
        # same tokens, zero-filled to ele_size past the NUL (memcmp-safe)
        assert [e.rstrip(b"\0").decode() for e in elems] == want
        assert all(len(e) == 45 and e[len(w):] == b"\0" * (45 - len(w)) for e, w in zip(elems, want))
        for q, got in zip(queries, idx):
            try:
                exp = cf.find_chunk_idx_from_hash(q, p)
            except KeyError:
                exp = -1
            assert got == exp, (name, q)
        assert seeks == [9000 * 524288, 3 * 524288 + (1500 - 16) * 7]


def test_c_find_idx_on_master_header_line(hashes, tmp_path, driver):
    m = tmp_path / "C.masterchunks"
    m.write_bytes(_crlf([f"File: /tmp/C.tar Chunks:0 {hashes[0]}"] +
                        [f"{i} {h}" for i, h in enumerate(hashes) if i]).encode())
    # chunk 0 shares the header line: its index is the number after Chunks:
    _, idx, _, _ = _run(driver, m, m, *hashes)
    assert idx == [0, 1, 2, 3]


def test_c_read_chunk_missing_file_exits_like_fopen(driver, tmp_path):
    r = subprocess.run([str(driver), str(tmp_path / "nope"), str(tmp_path / "nope")],
                       capture_output=True, text=True)
    assert r.returncode == 255  # exit(-1), utility.c:263-266
    assert f"Failed to open file {tmp_path / 'nope'} \n" in r.stderr


def test_reference_peer_links_without_chunk_o_and_sha_o():
    """the reference's own peer sources, unmodified,
    linked without chunk.o and sha.o (oracle/Makefile `dropin`).  Every
    chunk.h / sha.h symbol the peer uses resolves to libsha1chunk.so."""
    exe = os.path.join(ROOT, "oracle", "_ref", "dropin", "peer")
    if os.path.isdir("/root/reference"):
        subprocess.run(["make", "-s", "-C", PKG_DIR], check=True)
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "dropin"], check=True,
                       stderr=subprocess.DEVNULL)
    if not os.path.exists(exe):
        pytest.skip("reference sources absent and no prebuilt drop-in peer")
    syms = subprocess.run(["nm", "-D", exe], capture_output=True, text=True, check=True).stdout
    undef = {l.split()[-1] for l in syms.splitlines() if l.split()[-2:-1] == ["U"]}
    assert {"read_chunk", "find_chunk_idx_from_hash", "seek_to_chunk_pos", "seek_to_packet_pos",
            "verify_chunk_hash", "get_chunk_hash"} <= undef
    local = subprocess.run(["nm", exe], capture_output=True, text=True, check=True).stdout
    for name in ("SHA1Guts", "SHA1Update", "shahash", "make_chunks", "read_chunk"):
        assert f" T {name}\n" not in local, name
    ldd = subprocess.run(["ldd", exe], capture_output=True, text=True).stdout
    assert "libsha1chunk.so" in ldd
