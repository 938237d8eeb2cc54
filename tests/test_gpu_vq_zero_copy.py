"""Zero-copy receive on the verify queue and the queue's
resource rules.

The reference's receiver reassembles a 512 KiB chunk from DATA packets into
a per-session buffer (reliable_udp.c:121 `recv_session->data = Malloc(CHUNK_LEN)`,
filled at offset 1484*(seq-1), reliable_udp.c:339), verifies it in place
(packet_handler.c:472 -> job.c:217-228 verify_hash: 0 = match, 1 =
mismatch) and on a match copies it into the job buffer
(reliable_udp.c:696-709).  sha1chunk_vq_reserve hands out that session
buffer inside the queue's pinned ring, sha1chunk_vq_commit verifies it
where it lies, sha1chunk_vq_release gives it back after the job-buffer copy.

Checked against the reference's golden digests (config 2's corpus), with 20 %
of the chunks corrupted in place, in every queue implementation."""
import hashlib
import os
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L512 = 524288
PIECE = 1484  # DATA payload bytes per packet (constants.h:11,16: 1500 - 16)
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(pkg):
    import torch
    assert torch.cuda.is_available(), "GPU tests need a device"
    assert pkg.device_count() >= 1, pkg.lib().sha1chunk_last_error()
    torch.cuda.set_device(0)
    pkg.set_device(0)
    return torch


@pytest.fixture(scope="module")
def corpus(dev, pkg):
    """64 chunks of config 2's synthetic corpus (generated on the device) and
    their reference golden digests."""
    n = 64
    buf = dev.empty(n * L512, dtype=dev.uint8, device="cuda")
    pkg.synth_fill_device(buf, 0, n, L512)
    dev.cuda.synchronize()
    host = buf.cpu().numpy().reshape(n, L512)
    want = np.fromfile(os.path.join(ROOT, "tests/golden/synth_4096x512k.bin"), np.uint8).reshape(-1, 20)[:n]
    return host, want


def _fill_in_place(view: np.ndarray, chunk: np.ndarray) -> None:
    """The reassembly of reliable_udp.c:339: payload pieces at 1484*(seq-1)."""
    for o in range(0, chunk.size, PIECE):
        view[o:o + PIECE] = chunk[o:o + PIECE]


@pytest.mark.parametrize("mode", ["persistent", "persistent-pcie", "batch"])
def test_reserve_fill_commit_release(pkg, dev, corpus, monkeypatch, mode):
    """256 chunks through reserve -> in-place fill -> commit, up to 16
    sessions outstanding, every 5th chunk corrupted in its buffer before the
    commit; each result matches the golden digest's verdict, and each
    verified buffer still holds the chunk when its result comes back (the
    job-buffer copy reads it) until it is released.  persistent: the drain
    reads groups the copy engine staged in HBM (default); persistent-pcie:
    the drain reads the pinned ring over PCIe (SHA1CHUNK_VQ_DMA=0)."""
    monkeypatch.setenv("SHA1CHUNK_VQ_MODE", mode.split("-")[0])
    monkeypatch.setenv("SHA1CHUNK_VQ_DMA", "0" if mode.endswith("pcie") else "1")
    host, want = corpus
    n = 256
    held, results = {}, {}
    with pkg.VerifyQueue(batch=16, max_chunk_len=L512) as q:
        for i in range(n):
            r = q.reserve(L512)
            src = host[i % host.shape[0]]
            _fill_in_place(r.view, src)
            if i % 5 == 2:
                r.view[(i * 7919) % L512] ^= 0x40  # corrupted in flight
            held[i] = (r, src, i % 5 == 2)
            q.commit(r, want[i % host.shape[0]].tobytes(), i)
            while len(held) >= 16 or (i == n - 1 and held):
                for tag, m in q.poll(wait=len(held) >= 16 or i == n - 1):
                    r, src, bad = held.pop(tag)
                    results[tag] = m
                    assert m == (1 if bad else 0), (tag, m)
                    if not bad:  # the job-buffer copy of reliable_udp.c:696-709
                        assert np.array_equal(r.view, src), tag
                    q.release(r)
        assert sorted(results) == list(range(n)) and q.pending == 0
        assert sum(results.values()) == len(range(2, n, 5))


def test_reserve_on_the_host_batch1_path(pkg):
    """The batch-1 host queue (SHA1CHUNK_HOST_SMALL) takes reservations too:
    commit hashes the buffer in place on the host (child process: the knob
    is read once per process)."""
    code = r"""
import importlib, os, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
pkg = importlib.import_module("congestion-control-with-bittorren_amd")
want = np.fromfile(os.path.join(sys.argv[1], "tests/golden/synth_4096x512k.bin"), np.uint8).reshape(-1, 20)
import torch
buf = torch.empty(4 * 524288, dtype=torch.uint8, device="cuda")
pkg.synth_fill_device(buf, 0, 4, 524288)
torch.cuda.synchronize()
host = buf.cpu().numpy().reshape(4, 524288)
with pkg.VerifyQueue(batch=1, max_chunk_len=524288) as q:
    rs = []
    for i in range(4):
        r = q.reserve(524288)
        r.view[:] = host[i]
        if i == 3:
            r.view[0] ^= 1
        q.commit(r, want[i].tobytes(), 10 + i)
        rs.append(r)
    assert q.poll() == [(10, 0), (11, 0), (12, 0), (13, 1)]
    for r in rs:
        q.release(r)
    try:
        q.release(rs[0])
        raise AssertionError("double release accepted")
    except pkg.Sha1ChunkError:
        pass
print("host1 reserve ok")
"""
    env = dict(os.environ, SHA1CHUNK_HOST_SMALL=str(L512))
    r = subprocess.run([sys.executable, "-c", code, ROOT], capture_output=True, text=True, env=env,
                       cwd=ROOT, timeout=120)
    assert r.returncode == 0 and "host1 reserve ok" in r.stdout, (r.stdout[-1000:], r.stderr[-2000:])


def test_full_ring_of_unreleased_buffers_fails_fast(pkg, dev, monkeypatch):
    """Reservations the caller never releases fill the ring; the next
    reserve fails with ENOMEM at once (no 120 s wait for the drain), and
    releasing one makes room again."""
    monkeypatch.setenv("SHA1CHUNK_VQ_MODE", "persistent")
    monkeypatch.setenv("SHA1CHUNK_VQ_RING_MIB", "8")  # floor: 2 groups of 64 max-length chunks
    with pkg.VerifyQueue(batch=64, max_chunk_len=65536) as q:
        held = []
        t0 = time.time()
        with pytest.raises(pkg.Sha1ChunkError) as ei:
            for _ in range(1 << 12):
                held.append(q.reserve(65536))
        assert time.time() - t0 < 5.0
        assert ei.value.code == pkg.sha1chunk.ENOMEM and "not released" in str(ei.value)
        assert len(held) == (8 << 20) // 65536
        q.release(held.pop(0))
        r = q.reserve(65536)
        r.view[:] = 7
        q.commit(r, hashlib.sha1(bytes([7]) * 65536).digest(), 1)
        assert q.poll(wait=True) == [(1, 0)]
        for h in held + [r]:
            q.release(h)


def test_another_threads_reservation_makes_submit_wait(pkg, dev, monkeypatch):
    """on a queue shared by receive threads, another
    session's reservation at the ring's head is a buffer still filling, not a
    dead end: this thread's submits and reserves wait for it (bounded) instead
    of failing with ENOMEM.  A session thread reserves the ring's first
    buffer, fills it 0.3 s later, commits and releases it; meanwhile the main
    thread submits three rings' worth of chunks.  Every submit succeeds, none
    before the session's commit could free the head, every result is right."""
    import threading
    monkeypatch.setenv("SHA1CHUNK_VQ_MODE", "persistent")
    monkeypatch.setenv("SHA1CHUNK_VQ_RING_MIB", "8")  # 128 chunks of 64 KiB
    chunk = bytes(range(256)) * 256
    dig = hashlib.sha1(chunk).digest()
    with pkg.VerifyQueue(batch=64, max_chunk_len=65536) as q:
        reserved, committed = threading.Event(), threading.Event()
        errors = []

        def session():  # the session's own thread reserves, fills, commits, releases
            try:
                r0 = q.reserve(65536)
                reserved.set()
                time.sleep(0.3)
                r0.view[:] = np.frombuffer(chunk, np.uint8)
                committed.set()
                q.commit(r0, dig, 10**6)
                q.release(r0)
            except Exception as e:
                errors.append(repr(e))
                reserved.set()

        t = threading.Thread(target=session)
        t.start()
        try:
            assert reserved.wait(timeout=30) and not errors, errors
            t0 = time.time()
            got = {}
            for i in range(3 * 128):
                q.submit(chunk, dig if i % 7 else bytes(20), i)
                if i == 127:  # the ring's 128th buffer: room only once the session's head buffer is freed
                    assert committed.is_set() and time.time() - t0 >= 0.25
                for tag, m in q.poll():
                    got[tag] = m
        finally:
            t.join(timeout=60)  # destroy must not overlap the session's calls
        assert not errors and committed.is_set(), errors
        for tag, m in q.poll(wait=True, max_results=1 << 16):
            got[tag] = m
        want = {i: (0 if i % 7 else 1) for i in range(3 * 128)}
        want[10**6] = 0
        assert got == want


def test_other_threads_finished_unreleased_head_fails_fast(pkg, dev, monkeypatch):
    """Round 6: four receive threads all waiting in reserve() while the
    ring's head held another session's verified but unpolled buffer stalled
    for the whole 120 s bound -- nobody polled.  A session thread reserves,
    fills and commits a ring's worth of buffers and polls nothing; once their
    results are in, the main thread's reserve fails with ENOMEM within
    seconds (the grace is 2 ms) and names the fix; after a poll and the
    releases it succeeds."""
    monkeypatch.setenv("SHA1CHUNK_VQ_MODE", "persistent")
    monkeypatch.setenv("SHA1CHUNK_VQ_RING_MIB", "8")  # 128 chunks of 64 KiB
    chunk = np.frombuffer(bytes(range(256)) * 256, np.uint8)
    dig = hashlib.sha1(chunk.tobytes()).digest()
    with pkg.VerifyQueue(batch=64, max_chunk_len=65536) as q:
        held, errors = [], []

        def session():
            try:
                for i in range(128):
                    r = q.reserve(65536)
                    r.view[:] = chunk
                    q.commit(r, dig, i)
                    held.append(r)
            except Exception as e:
                errors.append(repr(e))

        t = threading.Thread(target=session)
        t.start()
        t.join(timeout=60)
        assert not errors and len(held) == 128, errors
        time.sleep(0.5)  # the drain finishes the 128 chunks (two groups)
        t0 = time.time()
        with pytest.raises(pkg.Sha1ChunkError) as ei:
            q.reserve(65536)
        assert time.time() - t0 < 5.0
        assert ei.value.code == pkg.sha1chunk.ENOMEM and "not yet polled and released" in str(ei.value)
        got = dict(q.poll(wait=True, max_results=256))
        assert got == {i: 0 for i in range(128)}
        for r in held:
            q.release(r)
        r = q.reserve(65536)
        r.view[:] = chunk
        q.commit(r, dig, 500)
        assert q.poll(wait=True) == [(500, 0)]
        q.release(r)


def test_queue_create_destroy_beside_a_busy_queue(pkg, dev, corpus, monkeypatch):
    """creating and destroying a queue must not wait for the
    whole device.  One thread keeps a persistent queue continuously busy for
    ~4 s; meanwhile another thread creates, uses and destroys queues, each
    cycle bounded (it used to wait in hipDeviceSynchronize for the busy
    drain, which only ends when its feed stops)."""
    monkeypatch.setenv("SHA1CHUNK_VQ_MODE", "persistent")
    monkeypatch.setenv("SHA1CHUNK_VQ_RING_MIB", "256")
    host, want = corpus
    stop = threading.Event()
    errors = []

    def feeder():
        try:
            with pkg.VerifyQueue(batch=64, max_chunk_len=L512) as q:
                i = 0
                while not stop.is_set():
                    q.submit(host[i % 64].tobytes(), want[i % 64].tobytes(), i)
                    i += 1
                    if i % 64 == 0:
                        assert all(m == 0 for _, m in q.poll())
                q.poll(wait=True)
        except Exception as e:  # surfaced below
            errors.append(e)

    t = threading.Thread(target=feeder)
    t.start()
    try:
        time.sleep(0.5)
        cycles = []
        t_end = time.time() + 3.0
        while time.time() < t_end:
            t0 = time.perf_counter()
            with pkg.VerifyQueue(batch=16, max_chunk_len=65536) as q2:
                q2.submit(bytes(100), hashlib.sha1(bytes(100)).digest(), 5)
                assert q2.poll(wait=True) == [(5, 0)]
            cycles.append(time.perf_counter() - t0)
        print(f"{len(cycles)} create/use/destroy cycles beside a busy queue: "
              f"max {max(cycles) * 1e3:.1f} ms, median {sorted(cycles)[len(cycles) // 2] * 1e3:.1f} ms")
        assert len(cycles) >= 3 and max(cycles) < 1.5, cycles
    finally:
        stop.set()
        t.join(timeout=60)
    assert not errors, errors


def test_five_busy_queues_and_a_device_batch(pkg, dev, corpus, monkeypatch):
    """the drains of all queues on a device stay within the CU
    budget (half the device by default; queues beyond it use batch
    launches), so five continuously fed queues leave room for a device
    batch, which completes with the golden digests while they run."""
    monkeypatch.setenv("SHA1CHUNK_VQ_MODE", "persistent")
    monkeypatch.setenv("SHA1CHUNK_VQ_RING_MIB", "256")
    host, want = corpus
    stop = threading.Event()
    errors, counts = [], [0] * 5

    def feeder(k):
        try:
            with pkg.VerifyQueue(batch=64, max_chunk_len=L512) as q:
                i = 0
                while not stop.is_set():
                    q.submit(host[i % 64].tobytes(), want[i % 64].tobytes(), i)
                    i += 1
                    if i % 32 == 0:
                        res = q.poll()
                        assert all(m == 0 for _, m in res)
                        counts[k] += len(res)
                res = q.poll(wait=True)
                assert all(m == 0 for _, m in res)
                counts[k] += len(res)
        except Exception as e:
            errors.append(e)

    ts = [threading.Thread(target=feeder, args=(k,)) for k in range(5)]
    for t in ts:
        t.start()
    try:
        time.sleep(1.0)
        n = 4096
        buf = dev.empty(n * L512, dtype=dev.uint8, device="cuda")
        dig = dev.zeros((n, 20), dtype=dev.uint8, device="cuda")
        st = dev.cuda.Stream()
        st.wait_stream(dev.cuda.current_stream())  # dig's zero fill runs on torch's stream
        pkg.synth_fill_device(buf, 0, n, L512, stream=st)
        t0 = time.perf_counter()
        pkg.hash_uniform_device(buf, L512, n, dig, stream=st)
        st.synchronize()
        secs = time.perf_counter() - t0
        got = dig.cpu().numpy()
        gold = np.fromfile(os.path.join(ROOT, "tests/golden/synth_4096x512k.bin"), np.uint8).reshape(-1, 20)
        assert np.array_equal(got, gold)
        print(f"config-2 batch beside 5 busy queues: {secs * 1e3:.1f} ms")
        assert secs < 30.0
    finally:
        stop.set()
        for t in ts:
            t.join(timeout=120)
    assert not errors, errors
    assert all(c > 0 for c in counts), counts


def _config2_on_fresh_stream(pkg, dev):
    """One config-2 batch (4096 x 512 KiB, device-resident) hashed on a new
    stream: wall seconds from the launch to the stream's completion, and
    whether its digests equal the reference's golden ones."""
    n = 4096
    buf = dev.empty(n * L512, dtype=dev.uint8, device="cuda")
    dig = dev.zeros((n, 20), dtype=dev.uint8, device="cuda")
    st = dev.cuda.Stream()
    st.wait_stream(dev.cuda.current_stream())
    pkg.synth_fill_device(buf, 0, n, L512, stream=st)
    st.synchronize()
    t0 = time.perf_counter()
    pkg.hash_uniform_device(buf, L512, n, dig, stream=st)
    st.synchronize()
    secs = time.perf_counter() - t0
    gold = np.fromfile(os.path.join(ROOT, "tests/golden/synth_4096x512k.bin"), np.uint8).reshape(-1, 20)
    ok = np.array_equal(dig.cpu().numpy(), gold)
    del buf, dig
    return secs, ok


def test_wait_behind_busy_drains_is_bounded(pkg, dev, corpus, monkeypatch):
    """a config-2 batch launched on a fresh stream while
    four verify queues are continuously fed is not held behind their drains.
    The regression this guards (the queues' streams at the default priority)
    took 12-26 ms against 6 ms solo; the pass/fail check compares medians
    with a relative margin (1.5x) so host or GIL jitter alone cannot fail it
    (ADVICE r5); the absolute "solo + 10 ms" of include/sha1chunk.h is
    printed, measured in the bench tooling, not asserted here."""
    import threading
    monkeypatch.setenv("SHA1CHUNK_VQ_MODE", "persistent")
    monkeypatch.setenv("SHA1CHUNK_VQ_RING_MIB", "256")
    import sys
    host, want = corpus
    # the feeders' bytes made once: their loop then holds the GIL for a few
    # microseconds per submit (the C call releases it), so the timed thread's
    # wall clock measures the device, not the interpreter
    chunks = [host[i].tobytes() for i in range(64)]
    digs = [want[i].tobytes() for i in range(64)]
    old_switch = sys.getswitchinterval()
    sys.setswitchinterval(1e-4)
    solo = float(np.median([_config2_on_fresh_stream(pkg, dev)[0] for _ in range(3)]))
    stop, started = threading.Event(), threading.Barrier(5)
    errors, counts = [], [0] * 4

    def feeder(k):
        try:
            with pkg.VerifyQueue(batch=64, max_chunk_len=L512) as q:
                started.wait(timeout=60)
                i = 0
                while not stop.is_set():
                    q.submit(chunks[i % 64], digs[i % 64], i)
                    i += 1
                    if i % 32 == 0:
                        res = q.poll()
                        assert all(m == 0 for _, m in res)
                        counts[k] += len(res)
                res = q.poll(wait=True)
                assert all(m == 0 for _, m in res)
                counts[k] += len(res)
        except Exception as e:
            errors.append(e)

    ts = [threading.Thread(target=feeder, args=(k,)) for k in range(4)]
    for t in ts:
        t.start()
    busy = []
    try:
        started.wait(timeout=60)
        time.sleep(0.5)
        for _ in range(5):
            secs, ok = _config2_on_fresh_stream(pkg, dev)
            assert ok
            busy.append(secs)
    finally:
        stop.set()
        for t in ts:
            t.join(timeout=120)
        sys.setswitchinterval(old_switch)
    assert not errors, errors
    assert all(c > 0 for c in counts), counts
    print(f"config-2 batch on a fresh stream: solo {solo * 1e3:.2f} ms, beside 4 fed queues "
          f"{', '.join(f'{b * 1e3:.2f}' for b in busy)} ms")
    print(f"within solo + 10 ms: {max(busy) <= solo + 0.010}")
    assert float(np.median(busy)) <= 1.5 * solo, (solo, busy)
