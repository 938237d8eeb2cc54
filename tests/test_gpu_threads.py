"""Concurrent callers.  The reference's peer is single-threaded (peer.c
select loop), but the library is a shared object that any caller may use
from several threads: lazy device init, per-device state behind a mutex,
per-thread error strings, one verify queue per thread (include/sha1chunk.h).

Eight Python threads (ctypes drops the GIL for the duration of each call)
hammer every entry point at once -- shahash, get_chunk_hash / verify_hash,
the SHA1Init/Update/Final trio at random split points, ragged host batches,
verify_batch, make_chunks on a file, and a verify queue of their own -- and
every digest is checked against hashlib.  The same run again in a child
process with SHA1CHUNK_HOST_SMALL=524288 mixes the host small-call path with
the device paths under the same concurrency, and with the threads bound to
three logical devices."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

_WORKER = r"""
import hashlib, importlib, os, sys, tempfile
from concurrent.futures import ThreadPoolExecutor
import numpy as np
sys.path.insert(0, sys.argv[1])
pkg = importlib.import_module("congestion-control-with-bittorren_amd")
assert pkg.device_count() >= 1
L = 524288
ITERS = int(os.environ.get("SHA1CHUNK_THREAD_ITERS", "12"))  # per thread; widened for evidence runs
tmp = tempfile.mkdtemp()


def work(tid):
    rng = np.random.default_rng(1000 + tid)
    if os.environ.get("SHA1CHUNK_VIRTUAL_DEVICES"):  # threads spread over the logical devices
        pkg.set_device(tid % pkg.device_count())
    ops = 0
    with pkg.VerifyQueue(batch=8, max_chunk_len=L) as q:
        want_q = {}
        for it in range(ITERS):
            kind = it % 6
            if kind == 0:  # shahash on a random length up to 1 MiB + a tail
                n = int(rng.integers(0, 2 * L + 100))
                data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
                assert pkg.shahash(data) == hashlib.sha1(data).digest(), (tid, n)
            elif kind == 1:  # get_chunk_hash / verify_hash (job.c:217-228) on a 512 KiB chunk
                data = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
                h = hashlib.sha1(data).hexdigest()
                assert pkg.get_chunk_hash(data) == h
                assert pkg.verify_hash(h, data) == 0
                bad = bytearray(data); bad[int(rng.integers(0, L))] ^= 0x40
                assert pkg.verify_hash(h, bytes(bad)) == 1
            elif kind == 2:  # the streaming trio at random cuts
                data = rng.integers(0, 256, int(rng.integers(1, 3 * L)), dtype=np.uint8).tobytes()
                s, pos = pkg.SHA1(), 0
                while pos < len(data):
                    c = int(rng.integers(1, 200000))
                    s.update(data[pos:pos + c]); pos += c
                assert s.final() == hashlib.sha1(data).digest(), tid
            elif kind == 3:  # ragged host batch + verify_batch
                k = int(rng.integers(1, 40))
                lens = rng.integers(0, L + 1, k).astype(np.uint32)
                off = np.zeros(k, np.uint64)
                off[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
                buf = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
                want = np.array([np.frombuffer(hashlib.sha1(buf[int(o):int(o) + int(l)].tobytes()).digest(),
                                               np.uint8) for o, l in zip(off, lens)])
                assert np.array_equal(pkg.hash_batch(buf, off, lens), want), tid
                exp = want.copy(); exp[k // 2, 3] ^= 1
                mism = pkg.verify_batch(buf, off, lens, exp)
                assert list(mism) == [int(i == k // 2) for i in range(k)], tid
            elif kind == 4:  # make_chunks (chunk.c:15-27) on a file of its own
                n = int(rng.integers(1, 6 * L))
                data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
                p = os.path.join(tmp, f"t{tid}_{it}.bin")
                open(p, "wb").write(data)
                want = [hashlib.sha1(data[i:i + L]).digest() for i in range(0, n, L)]
                assert pkg.make_chunks(p) == want, (tid, n)
                os.remove(p)
            else:  # this thread's verify queue
                for j in range(10):
                    data = rng.integers(0, 256, int(rng.integers(0, L + 1)), dtype=np.uint8).tobytes()
                    d = hashlib.sha1(data).digest()
                    tag = it * 100 + j
                    corrupt = j % 4 == 3
                    q.submit(data, bytes([d[0] ^ 1]) + d[1:] if corrupt else d, tag)
                    want_q[tag] = int(corrupt)
                for tag, m in q.poll():
                    assert want_q.pop(tag) == m, (tid, tag)
            ops += 1
        for tag, m in q.poll(wait=True):
            assert want_q.pop(tag) == m, (tid, tag)
        assert not want_q, (tid, want_q)
    return ops


with ThreadPoolExecutor(8) as ex:
    done = list(ex.map(work, range(8)))
assert done == [ITERS] * 8, done
print("threads ok", sum(done))
"""


def _run(env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, "-c", _WORKER, ROOT], capture_output=True, text=True,
                       env=env, cwd=ROOT, timeout=600)
    assert r.returncode == 0 and "threads ok" in r.stdout, (r.stdout[-1500:], r.stderr[-3000:])


@pytest.mark.parametrize("mode", ["persistent", "batch"])
def test_concurrent_callers(pkg, mode):
    _run({"SHA1CHUNK_VQ_MODE": mode})


def test_concurrent_callers_host_small(pkg):
    _run({"SHA1CHUNK_HOST_SMALL": "524288"})


def test_concurrent_callers_over_devices(pkg):
    """Threads bound to different devices (three logical devices over the
    box's GPU, SHA1CHUNK_VIRTUAL_DEVICES=3, each with its own streams, slots
    and queues)."""
    _run({"SHA1CHUNK_VIRTUAL_DEVICES": "3"})
