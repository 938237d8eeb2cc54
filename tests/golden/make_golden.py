"""Generate the golden vectors in tests/golden/ from the REFERENCE itself.

Run in the survey/build container (where /root/reference exists):

    python tests/golden/make_golden.py

Every digest written here is computed by the unmodified reference sha.c
(compiled by oracle/Makefile into oracle/_ref/libsharef.so) or, for the
file fixtures, copied from the reference's own tmp/*.chunks and re-derived
with the reference's make-chunks binary built from source.  The restatement
in oracle/ is cross-checked against the same vectors by tests/test_oracle.py.

Outputs (small; committed):
  golden.json             KATs, edge lengths, fixture digests, config aggregates
  C.tar.gz                the reference's tmp/C.tar fixture (= A.tar || B.tar)
  synth_4096x512k.bin     all 4096 digests of BASELINE config 2
  mixed_16384.bin         all digests of BASELINE config 5 (mixed lengths)
  mixed_16384_len.bin     its 16384 chunk lengths (uint32 LE)

`python tests/golden/make_golden.py --add config5x4` (or config5x8) adds only the 4x (8x) config-5
aggregate (65536 chunks of the same length law, bench.py's config5 leg) to an
existing golden.json.
"""
from __future__ import annotations

import concurrent.futures as cf
import gzip
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
THREADS = os.cpu_count() or 8

EDGE_LENGTHS = [0, 1, 3, 4, 5, 15, 16, 17, 55, 56, 57, 63, 64, 65, 119, 120, 121, 127, 128, 129,
                191, 192, 1000, 4095, 4096, 4097, 65535, 65536, 65537, 524287, 524288, 524289,
                1048576]
EDGE_CHUNK_ID = 7


def ref_digests(buf: np.ndarray, off: np.ndarray, ln: np.ndarray) -> np.ndarray:
    return O.hash_batch(buf, off, ln, threads=THREADS, use_ref=True)


def synth_digests(first: int, count: int, chunk_len: int, slice_chunks: int = 1024) -> np.ndarray:
    """Digests of synthetic chunks [first, first+count) via the reference,
    generated and hashed in slices so memory stays bounded."""
    out = np.zeros((count, 20), np.uint8)
    gen_threads = 4

    def gen(i0):
        m = min(slice_chunks, count - i0)
        return i0, O.synth_chunks(first + i0, m, chunk_len)

    starts = list(range(0, count, slice_chunks))
    # bounded look-ahead: at most gen_threads slices generated but not hashed
    with cf.ThreadPoolExecutor(gen_threads) as ex:
        pending = [ex.submit(gen, i0) for i0 in starts[:gen_threads]]
        nxt = gen_threads
        while pending:
            i0, data = pending.pop(0).result()
            if nxt < len(starts):
                pending.append(ex.submit(gen, starts[nxt]))
                nxt += 1
            m = data.size // chunk_len
            off = np.arange(m, dtype=np.uint64) * chunk_len
            ln = np.full(m, chunk_len, np.uint32)
            out[i0:i0 + m] = ref_digests(data, off, ln)
            del data
    return out


def mixed_golden(n: int) -> dict:
    """Digests of n chunks of the config-5 length law (chunk i: length
    mixed_len(i), content synth_chunk(i, len)), hashed by the reference in
    slices so host memory stays bounded: aggregate, lengths hash and a sample."""
    ln = O.mixed_lengths(n)
    dig = np.zeros((n, 20), np.uint8)
    step = 4096
    for i0 in range(0, n, step):
        part = ln[i0:i0 + step]
        off = np.zeros(part.size, np.uint64)
        pad = (part.astype(np.uint64) + 127) // 128 * 128
        off[1:] = np.cumsum(pad)[:-1]
        buf = np.zeros(int(pad.sum()), np.uint8)
        for j in range(part.size):
            L = int(part[j])
            buf[int(off[j]):int(off[j]) + L] = O.synth_chunk(i0 + j, L)
        dig[i0:i0 + part.size] = ref_digests(buf, off, part)
    longest = int(np.argmax(ln))
    sample = sorted(set(list(range(0, n, 997)) + [n - 1, longest]))
    return {"chunks": n, "total_bytes": int(ln.astype(np.uint64).sum()),
            "agg": O.digest_of_digests(dig).hex(),
            "lengths_sha1": hashlib.sha1(ln.tobytes()).hexdigest(),
            "sample": {str(i): dig[i].tobytes().hex() for i in sample}}


def add_config5x(k: int) -> None:
    """golden["config5x<k>"]: the config-5 law at k x 16384 chunks."""
    O.build(ref=True)
    assert O.ref_lib() is not None, "reference build failed"
    path = os.path.join(OUT, "golden.json")
    g = json.load(open(path))
    t0 = time.time()
    name = f"config5x{k}"
    g[name] = mixed_golden(k * 16384)
    # its first 16384 chunks are config 5 itself, its first 65536 config5x4
    d5 = np.fromfile(os.path.join(OUT, "mixed_16384.bin"), np.uint8).reshape(-1, 20)
    for i, v in g[name]["sample"].items():
        if int(i) < 16384:
            assert d5[int(i)].tobytes().hex() == v, i
        if k != 4 and "config5x4" in g and i in g["config5x4"]["sample"]:
            assert g["config5x4"]["sample"][i] == v, i
    print(f"{name} {time.time() - t0:.1f}s", flush=True)
    with open(path, "w") as f:
        json.dump(g, f, indent=1, sort_keys=True)
    print("wrote", path)


def main() -> None:
    if len(sys.argv) == 3 and sys.argv[1] == "--add" and sys.argv[2].startswith("config5x"):
        return add_config5x(int(sys.argv[2][len("config5x"):]))
    O.build(ref=True)
    assert O.ref_lib() is not None, "reference build failed"
    g: dict = {"seed": O.SEED, "chunk_len": O.CHUNK_LEN,
               "generator": "oracle/_ref/libsharef.so (unmodified /root/reference/sha.c, -O2)"}

    # --- known-answer tests (sha.c:32-38, chunk.c:235-255) --------------------
    def ref1(b: bytes) -> str:
        a = np.frombuffer(b + b"\0", np.uint8)
        return ref_digests(a, np.zeros(1, np.uint64), np.array([len(b)], np.uint32))[0].tobytes().hex()

    nist56 = b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq"
    kats = {
        "abc": {"input_hex": b"abc".hex(), "digest": ref1(b"abc")},
        "nist56": {"input_hex": nist56.hex(), "digest": ref1(nist56)},
        "empty": {"input_hex": "", "digest": ref1(b"")},
        "dash": {"input_hex": b"dash".hex(), "digest": ref1(b"dash")},
        "million_a": {"input_repeat": ["61", 1000000], "digest": ref1(b"a" * 1000000)},
    }
    # The reference's own self-test binary must print the same three NIST lines.
    st = subprocess.run([os.path.join(ROOT, "oracle/_ref/sha1_test")], capture_output=True,
                        text=True, check=True).stdout.split("\n")
    for line, key in zip(st, ["abc", "nist56", "million_a"]):
        assert line.replace(" ", "") == kats[key]["digest"], (line, key)
    for k, v in kats.items():  # stdlib as an independent second opinion
        data = bytes.fromhex(v["input_hex"]) if "input_hex" in v else b"a" * 1000000
        assert hashlib.sha1(data).hexdigest() == v["digest"], k
    g["kats"] = kats

    # --- edge lengths of one synthetic chunk -----------------------------------
    edges = {}
    for L in EDGE_LENGTHS:
        data = O.synth_chunk(EDGE_CHUNK_ID, L)
        edges[str(L)] = ref1(data.tobytes())
    g["edge_lengths"] = {"chunk_id": EDGE_CHUNK_ID, "digests": edges}

    # --- reference file fixtures ------------------------------------------------
    ctar = open(os.path.join(REF, "tmp/C.tar"), "rb").read()
    with gzip.open(os.path.join(OUT, "C.tar.gz"), "wb", compresslevel=9) as f:
        f.write(ctar)

    def parse_chunks(path):
        rows = []
        for line in open(path, "rb").read().decode().replace("\r", "").split("\n"):
            parts = line.split()
            if len(parts) == 2 and parts[0].isdigit():
                rows.append(parts[1])
        return rows

    mk = os.path.join(ROOT, "oracle/_ref/make-chunks")
    fixtures = {}
    for name in ["tmp/C.tar", "tmp/A.tar", "tmp/B.tar", "example/A.gif", "example/B.gif"]:
        out = subprocess.run([mk, os.path.join(REF, name)], capture_output=True, text=True,
                             check=True).stdout
        fixtures[name] = [l.split()[1] for l in out.strip().split("\n")]
    assert fixtures["tmp/C.tar"] == parse_chunks(os.path.join(REF, "tmp/C.chunks"))
    assert fixtures["tmp/A.tar"] == parse_chunks(os.path.join(REF, "tmp/A.chunks"))
    assert fixtures["tmp/B.tar"] == parse_chunks(os.path.join(REF, "tmp/B.chunks"))
    g["fixtures"] = {
        "make_chunks": fixtures,
        "C.chunks_file": parse_chunks(os.path.join(REF, "tmp/C.chunks")),
        "sizes": {k: os.path.getsize(os.path.join(REF, k)) for k in fixtures},
    }

    # --- BASELINE configs --------------------------------------------------------
    t0 = time.time()
    d2 = synth_digests(0, 4096, O.CHUNK_LEN)
    d2.tofile(os.path.join(OUT, "synth_4096x512k.bin"))
    g["config2"] = {"chunks": 4096, "first": 0, "agg": O.digest_of_digests(d2).hex()}
    print(f"config2 {time.time() - t0:.1f}s", flush=True)

    t0 = time.time()
    d3 = synth_digests(0, 65536, O.CHUNK_LEN)
    sample = list(range(0, 65536, 1021)) + list(range(65472, 65536))
    g["config3"] = {"chunks": 65536, "first": 0, "agg": O.digest_of_digests(d3).hex(),
                    "sample": {str(i): d3[i].tobytes().hex() for i in sample}}
    assert (d3[:4096] == d2).all()
    print(f"config3 {time.time() - t0:.1f}s", flush=True)

    t0 = time.time()
    d4 = np.concatenate([d3, synth_digests(65536, 262144 - 65536, O.CHUNK_LEN)])
    shards = {}
    for ws in (1, 2, 4, 8):
        per = 262144 // ws
        shards[str(ws)] = [O.digest_of_digests(d4[r * per:(r + 1) * per]).hex() for r in range(ws)]
    g["config4"] = {"chunks": 262144, "first": 0, "agg": O.digest_of_digests(d4).hex(),
                    "shard_aggs": shards}
    # weak-scaling bench shards: rank r hashes chunks [4096 r, 4096 (r+1))
    g["weak4096"] = [O.digest_of_digests(d4[r * 4096:(r + 1) * 4096]).hex() for r in range(8)]
    print(f"config4 {time.time() - t0:.1f}s", flush=True)

    # mixed lengths (config 5): chunk i has length mixed_len(i), content synth_chunk(i, len)
    t0 = time.time()
    n5 = 16384
    ln5 = O.mixed_lengths(n5)
    off5 = np.zeros(n5, np.uint64)
    pad = (ln5.astype(np.uint64) + 127) // 128 * 128
    off5[1:] = np.cumsum(pad)[:-1]
    buf = np.zeros(int(pad.sum()), np.uint8)
    for i in range(n5):
        L = int(ln5[i])
        buf[int(off5[i]):int(off5[i]) + L] = O.synth_chunk(i, L)
    d5 = ref_digests(buf, off5, ln5)
    d5.tofile(os.path.join(OUT, "mixed_16384.bin"))
    ln5.astype("<u4").tofile(os.path.join(OUT, "mixed_16384_len.bin"))
    g["config5"] = {"chunks": n5, "total_bytes": int(ln5.astype(np.uint64).sum()),
                    "agg": O.digest_of_digests(d5).hex(),
                    "lengths_sha1": hashlib.sha1(ln5.tobytes()).hexdigest()}
    print(f"config5 {time.time() - t0:.1f}s", flush=True)

    with open(os.path.join(OUT, "golden.json"), "w") as f:
        json.dump(g, f, indent=1, sort_keys=True)
    print("wrote", os.path.join(OUT, "golden.json"))


if __name__ == "__main__":
    main()
