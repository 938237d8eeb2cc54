"""CPU: the drop-in boundary -- the C-ABI library builds, loads, and exports
every symbol include/*.h declares; the SHA1Context layout matches the
reference's; host-only logic (hex codec) behaves like chunk.c; without a
device the engine fails loudly instead of falling back to the CPU."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "congestion-control-with-bittorren_amd")


def _declared_functions():
    names = set()
    for h in ("sha.h", "chunk_hash.h", "sha1chunk.h"):
        text = open(os.path.join(ROOT, "include", h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        text = re.sub(r"typedef[^;]*;", "", text)
        text = re.sub(r"#define[^\n]*", "", text)
        for m in re.finditer(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{]*\)\s*;", text):
            names.add(m.group(1))
    return names


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-s", "-C", PKG_DIR], check=True)
    return os.path.join(PKG_DIR, "libsha1chunk.so")


def test_every_declared_symbol_is_exported(built, pkg):
    declared = _declared_functions()
    assert {"SHA1Init", "SHA1Update", "SHA1Final", "shahash", "make_chunks", "get_chunk_hash",
            "verify_chunk_hash", "binary2hex", "hex2binary", "verify_hash",
            "sha1chunk_hash_batch"} <= declared
    lib = C.CDLL(built)
    missing = [n for n in sorted(declared) if not hasattr(lib, n)]
    assert not missing, missing
    # the Python mirror binds exactly the declared C ABI
    assert set(pkg.sha1chunk.exported_symbols()) == declared


def test_sha1context_layout_matches_reference(pkg):
    # /root/reference/sha.h:39-52 (no RUNTIME_ENDIAN): 96 bytes
    ctx = pkg.SHA1Context
    assert C.sizeof(ctx) == 96
    assert ctx.totalLength.offset == 0
    assert ctx.hash.offset == 8
    assert ctx.bufferLength.offset == 28
    assert ctx.buffer.offset == 32


def test_sha_h_layout_compiles_to_96_bytes(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text('#include "sha.h"\n#include <stddef.h>\n'
                   '_Static_assert(sizeof(SHA1Context) == 96, "size");\n'
                   '_Static_assert(offsetof(SHA1Context, hash) == 8, "hash");\n'
                   '_Static_assert(offsetof(SHA1Context, bufferLength) == 28, "len");\n'
                   '_Static_assert(offsetof(SHA1Context, buffer) == 32, "buf");\n'
                   'int main(void) { return 0; }\n')
    subprocess.run(["gcc", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src),
                    "-o", str(tmp_path / "a.out")], check=True)


def test_hex_codec_matches_chunk_c(pkg):
    raw = bytes(range(0, 250, 13))
    h = pkg.binary2hex(raw)
    assert h == raw.hex()  # "%.2x" lowercase, chunk.c:60
    assert pkg.hex2binary(h) == raw
    assert pkg.hex2binary(h.upper()) == raw  # toupper in _hex2binary, chunk.c:68-72


def test_reference_style_caller_compiles_against_headers(tmp_path, built):
    """A caller written against the reference's API links as a drop-in."""
    src = tmp_path / "caller.c"
    src.write_text(r'''
#include <stdio.h>
#include "sha.h"
#include "chunk_hash.h"
int main(void) {
    uint8_t h[SHA1_HASH_SIZE]; char a[41];
    SHA1Context c; SHA1Init(&c); SHA1Update(&c, "abc", 3); SHA1Final(&c, h);
    hex2ascii(h, SHA1_HASH_SIZE, a); puts(a);
    shahash((uint8_t *)"dash", 4, h); binary2hex(h, 20, a); puts(a);
    return 0;
}''')
    exe = tmp_path / "caller"
    subprocess.run(["gcc", "-Wall", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe),
                    "-L", PKG_DIR, "-lsha1chunk", f"-Wl,-rpath,{PKG_DIR}"], check=True)
    assert exe.exists()


def _has_device(pkg):
    try:
        return pkg.device_count() > 0
    except Exception:
        return False


def test_no_device_fails_loudly(pkg, built):
    if _has_device(pkg):
        pytest.skip("a device is present")
    with pytest.raises(pkg.Sha1ChunkError) as ei:
        pkg.shahash(b"abc")
    assert ei.value.code == pkg.sha1chunk.ENODEV
    # the reference-signature C entry points exit(-1) with a message
    r = subprocess.run([os.path.join(PKG_DIR, "make-chunks"), os.path.join(ROOT, "tests/golden/C.tar.gz")],
                       capture_output=True, text=True)
    assert r.returncode == 255
    assert "no HIP device" in r.stderr
    assert r.stdout == ""


def test_verify_queue_without_device_fails_loudly(pkg):
    if _has_device(pkg):
        pytest.skip("a device is present")
    with pytest.raises(pkg.Sha1ChunkError):
        pkg.VerifyQueue(batch=16)


def test_python_mirror_names(pkg):
    for name in ("shahash", "binary2hex", "hex2binary", "make_chunks", "get_chunk_hash",
                 "verify_hash", "SHA1"):
        assert hasattr(pkg, name)


def test_product_does_not_link_the_oracle(built):
    out = subprocess.run(["ldd", built], capture_output=True, text=True).stdout
    assert "oracle" not in out and "sharef" not in out
    syms = subprocess.run(["nm", "-D", built], capture_output=True, text=True).stdout
    assert "oracle_" not in syms and "ref_" not in syms
