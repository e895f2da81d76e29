"""Shared fixtures. `-m gpu` tests need a HIP device and call the product
library through its C-ABI; everything else runs on CPU (oracle, host logic,
ABI loading, gloo multi-process)."""
import importlib.util
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# TSA_PKG_DIR: run the tests against a variant build (scripts/build_variant.sh)
PKG_DIR = os.environ.get("TSA_PKG_DIR", os.path.join(ROOT, "hw-accelerator-three-sequence-alignment_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs the HIP kernels")


def _srchash():
    spec = importlib.util.spec_from_file_location("tsa_srchash", os.path.join(PKG_DIR, "srchash.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _ensure_built():
    """Build when the library is missing or was built from other sources
    than this tree's (the hash tsa_version() carries, srchash.py)."""
    lib = os.path.join(PKG_DIR, "lib", "libtrialign.so")
    orc = os.path.join(ROOT, "oracle", "_build", "libtsa_oracle.so")
    if not (os.path.exists(lib) and os.path.exists(orc) and _srchash().is_current(lib)):
        subprocess.run(["make", "-s", "-j8"], cwd=ROOT, check=True)


def pytest_report_header(config):
    h = _srchash()
    lib = os.path.join(PKG_DIR, "lib", "libtrialign.so")
    return [f"trialign sources src={h.source_hash()}; libtrialign.so built from src={h.built_hash(lib)}"]


def load_pkg():
    _ensure_built()
    if "tsa_amd" in sys.modules:
        return sys.modules["tsa_amd"]
    spec = importlib.util.spec_from_file_location(
        "tsa_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["tsa_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def tsa():
    return load_pkg()


@pytest.fixture(scope="session")
def orc():
    _ensure_built()
    import oracle
    return oracle


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return json.load(f)["cases"]


@pytest.fixture(scope="session")
def synth(tsa):
    import importlib
    return importlib.import_module("tsa_amd.synth")


@pytest.fixture(scope="session")
def gpu(tsa):
    if tsa.device_count() < 1:
        pytest.fail("no HIP device visible: -m gpu tests must run on the MI355X box")
    return tsa
