"""The C ABI from plain C (no torch): build tests/c/capi_roundtrip.c with gcc against
include/spec_amd.h + libspec_amd.so (and the oracle as the checker) and run it on the GPU."""
from __future__ import annotations

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build(out):
    cmd = ["gcc", "-O2", "-std=c11", os.path.join(ROOT, "tests", "c", "capi_roundtrip.c"), "-o", out,
           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "oracle"),
           "-L" + os.path.join(ROOT, "spec_amd"), "-lspec_amd", "-L" + os.path.join(ROOT, "oracle", "build"),
           "-lspec_oracle", "-Wl,-rpath," + os.path.join(ROOT, "spec_amd"),
           "-Wl,-rpath," + os.path.join(ROOT, "oracle", "build")]
    subprocess.run(cmd, check=True)


def test_capi_program_builds(tmp_path):
    build(str(tmp_path / "capi_roundtrip"))


@pytest.mark.gpu
def test_capi_roundtrip_on_gpu(tmp_path, dev):
    exe = str(tmp_path / "capi_roundtrip")
    build(exe)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    assert "capi roundtrip ok" in r.stdout
