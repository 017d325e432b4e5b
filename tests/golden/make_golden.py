"""Regenerate the committed golden fixtures (tests/golden/*.npz) from the CPU oracle.

The reference (basecomplextech/spec) ships no byte-level vectors and its Go toolchain and
varint module are absent here, so these fixtures are ORACLE-GENERATED:
they freeze the oracle's output so that (1) any change to the oracle is caught by the CPU
suite (tests/test_golden.py) and (2) the GPU suite can check the HIP path against fixed
bytes without the oracle in the loop (tests/test_gpu_golden.py).  The hand-derivable
known-answer vectors are asserted directly in
tests/test_oracle_decode.py.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from spec_amd import workload  # noqa: E402
from spec_amd.schema import FLAT16  # noqa: E402


def flat16(n=96, seed=0x5EC0DE):
    cols, heaps = workload.flat16(n, seed)
    stream, ends = O.encode_flat_batch(FLAT16.tags, FLAT16.kinds, cols, [heaps.get(f) for f in range(16)], n)
    dec, status = O.decode_flat_batch(FLAT16.tags, FLAT16.kinds, stream, ends, FLAT16.widths)
    out = {"stream": stream, "ends": ends, "status": status}
    for f in range(16):
        out[f"col{f}"] = cols[f]
        out[f"dec{f}"] = dec[f]
    for f, h in heaps.items():
        out[f"heap{f}"] = h
    np.savez_compressed(os.path.join(HERE, "flat16_small.npz"), **out)


def nested(n=64, seed=0x5EC0DE):
    w = workload.nested(n, seed)
    stream, ends = O.encode_nested_batch(w)
    d = O.decode_nested_batch(stream, ends)
    out = {"stream": stream, "ends": ends}
    for k, v in w.items():
        out[f"in_{k}"] = v
    for k, v in d.items():
        out[f"out_{k}"] = v
    np.savez_compressed(os.path.join(HERE, "nested_small.npz"), **out)


if __name__ == "__main__":
    flat16()
    nested()
    print("wrote", sorted(f for f in os.listdir(HERE) if f.endswith(".npz")))
