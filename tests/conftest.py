import importlib
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


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
