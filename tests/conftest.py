"""Shared test plumbing.

Markers: `gpu` = needs an MI355X (run with -m gpu on the GPU box).
Everything else runs on a CPU-only host.
"""
import ctypes
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "h264-scroll-encoder_amd")
GOLD = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, PKG)
sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X)")


def _make(target_dir, *extra):
    subprocess.run(["make", "-s", "-C", target_dir, *extra], check=True,
                   stdout=subprocess.DEVNULL)


@pytest.fixture(scope="session")
def oracle():
    """The CPU checker (oracle/scroll_oracle.c), compiled on demand."""
    _make(os.path.join(REPO, "oracle"))
    lib = ctypes.CDLL(os.path.join(REPO, "oracle", "_build", "liboracle.so"))
    lib.or_bench_compose.restype = ctypes.c_double
    return lib


@pytest.fixture(scope="session")
def scroll():
    """The product library (fails loudly if it cannot be built/loaded)."""
    if not os.path.exists(os.path.join(PKG, "lib", "libh264scroll.so")):
        _make(PKG)
    import h264scroll
    return h264scroll


@pytest.fixture(scope="session")
def hostsim():
    """TEST-ONLY CPU build of the device header's logic (tests/hostsim)."""
    d = os.path.join(REPO, "tests", "hostsim")
    so = os.path.join(d, "libhostsim.so")
    src = [os.path.join(d, "sim.cpp"),
           os.path.join(PKG, "csrc", "scroll_device.h"),
           os.path.join(PKG, "csrc", "dyn_device.h")]
    if not os.path.exists(so) or any(os.path.getmtime(s) > os.path.getmtime(so) for s in src):
        tmp = f"{so}.{os.getpid()}"           # build aside, then rename: safe under pytest -n
        subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-I", d,
                        "-I", os.path.join(PKG, "csrc"), src[0], "-o", tmp], check=True)
        os.replace(tmp, so)
    return ctypes.CDLL(so)


@pytest.fixture(scope="session")
def golden_frames():
    with open(os.path.join(GOLD, "frames.jsonl")) as f:
        return [json.loads(line) for line in f]


@pytest.fixture(scope="session")
def golden_streams():
    with open(os.path.join(GOLD, "streams.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_md5():
    with open(os.path.join(GOLD, "md5.json")) as f:
        return json.load(f)


def golden_file(name):
    with open(os.path.join(GOLD, "files", name), "rb") as f:
        return f.read()


def synthetic_offsets(nstreams, nframes, h, first_stream=0):
    """stream s speed 1+(s%8), phase (97 s) mod 2H, triangle 0..H."""
    import numpy as np
    s = np.arange(first_stream, first_stream + nstreams, dtype=np.int64)[:, None]
    i = np.arange(nframes, dtype=np.int64)[None, :]
    x = i * (1 + s % 8) + (97 * s) % (2 * h)
    p = x % (2 * h)
    return np.where(p < h, p, 2 * h - p).astype(np.int32)
