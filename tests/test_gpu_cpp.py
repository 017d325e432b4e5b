"""The C++ host API (include/spec_amd.hpp) and its tests (tests/cpp/test_batch.cpp): built here
with g++ (CPU), run on the GPU."""
from __future__ import annotations

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build(out):
    cmd = ["g++", "-O2", "-std=c++17", "-Wall", os.path.join(ROOT, "tests", "cpp", "test_batch.cpp"), "-o", out,
           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "oracle"),
           "-L" + os.path.join(ROOT, "spec_amd"), "-lspec_amd", "-L" + os.path.join(ROOT, "oracle", "build"),
           "-lspec_oracle", "-Wl,-rpath," + os.path.join(ROOT, "spec_amd"),
           "-Wl,-rpath," + os.path.join(ROOT, "oracle", "build")]
    subprocess.run(cmd, check=True)


def test_cpp_api_builds(tmp_path):
    build(str(tmp_path / "test_batch"))


@pytest.mark.gpu
def test_cpp_api_on_gpu(tmp_path, dev):
    exe = str(tmp_path / "test_batch")
    build(exe)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout
