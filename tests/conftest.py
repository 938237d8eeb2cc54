import importlib
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")

# Pin every call of this test process (and of the child processes it starts,
# unless a test sets its own value) to the gfx950 kernels.  By default the
# library hashes the reference's single-message calls (shahash, verify_hash,
# the SHA1Update trio, make_chunks on a file <= 4 MiB) on the host
# (csrc/frontend.c routing); the kernel-parity tests must reach the kernels
# with those calls too.  The default routing has its own tests
# (test_host_small.py::test_default_routing_gpu, test_config1_make_chunks_cli),
# which start their children without this variable (default_env()).
os.environ["SHA1CHUNK_HOST_SMALL"] = "0"


def default_env(**extra) -> dict:
    """This process's environment without the test pin: the library's
    default routing, plus `extra`."""
    env = {k: v for k, v in os.environ.items() if k != "SHA1CHUNK_HOST_SMALL"}
    env.update(extra)
    return env


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN_DIR, "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build(ref=os.path.isdir("/root/reference") and not os.path.exists(
        os.path.join(ROOT, "oracle", "_ref", "libsharef.so")))
    return O


@pytest.fixture(scope="session")
def pkg():
    return importlib.import_module("congestion-control-with-bittorren_amd")


@pytest.fixture(scope="session")
def fixture_files():
    """The reference's file fixtures, from the committed tests/golden/C.tar.gz:
    C.tar = A.tar || B.tar, A.tar holds A.gif, B.tar holds B.gif."""
    import gzip
    import io
    import tarfile
    ctar = gzip.open(os.path.join(GOLDEN_DIR, "C.tar.gz")).read()
    files = {"tmp/C.tar": ctar, "tmp/A.tar": ctar[:1048576], "tmp/B.tar": ctar[1048576:]}
    for name, gif in (("tmp/A.tar", "A.gif"), ("tmp/B.tar", "B.gif")):
        with tarfile.open(fileobj=io.BytesIO(files[name])) as t:
            files["example/" + gif] = t.extractfile(gif).read()
    return files


# ---- bounds-checked backend runs ----------------------
# SHA1CHUNK_CHECKED=1 with SHA1CHUNK_LIB=<dir>/libsha1chunk.so of `make
# checked` (or `checked-unclamped`, the negative control): every GPU test
# fails if the device counted an out-of-batch entry index or A.order value
# during it (csrc/sha1_split.hpp checked_index; this process's calls only,
# not those of child processes the test starts).
def _checked_backend():
    import ctypes
    lib = os.environ.get("SHA1CHUNK_LIB")
    path = os.environ.get("SHA1CHUNK_BACKEND") or (
        os.path.join(os.path.dirname(os.path.abspath(lib)), "libsha1chunk_hip.so") if lib else None)
    if not path:
        raise RuntimeError("SHA1CHUNK_CHECKED=1 needs SHA1CHUNK_LIB (or SHA1CHUNK_BACKEND) of a checked build")
    be = ctypes.CDLL(path)
    if not hasattr(be, "s1be_checked_violations"):
        raise RuntimeError(f"{path} is not a checked build (no s1be_checked_violations)")
    be.s1be_checked_violations.restype = ctypes.c_longlong
    be.s1be_checked_violations.argtypes = [ctypes.c_int]
    return be


@pytest.fixture(autouse=True)
def _checked_bounds(request):
    if os.environ.get("SHA1CHUNK_CHECKED") != "1" or request.node.get_closest_marker("gpu") is None:
        yield
        return
    be = _checked_backend()
    assert be.s1be_checked_violations(1) >= 0
    yield
    v = be.s1be_checked_violations(1)
    assert v == 0, f"checked build: {v} out-of-batch entry index / A.order reads (device printf above)"
