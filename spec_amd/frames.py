"""mpx frames: the hot path's real input (mpx/conn_reader.go:179-194, mpx/conn_writer.go:84-97).

An mpx connection carries `[u32 big-endian size][message]` frames back to back.  A batching
receiver indexes the frame heads on the host while the bytes arrive (`frames_index`, a C
loop in libspec_amd.so) and decodes the frames where they lie (`decode_frames`: each record
starts 4 bytes after the previous frame's end) — no compaction pass over the received bytes.
`make_frames` builds such a buffer from records (test / benchmark input).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from .batch import Columns, _check_dev, _ptr, _stream_handle, alloc_columns
from .schema import Schema


def frames_index(buf: np.ndarray, cap: int | None = None):
    """-> (ends uint64[count], consumed): ends[k] = offset just past frame k's message."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    cap = cap if cap is not None else max(1, buf.size // 4)
    ends = np.zeros(cap, dtype=np.uint64)
    cnt, used = C.c_uint64(0), C.c_uint64(0)
    rc = _lib.lib().spec_frames_index(C.c_void_p(buf.ctypes.data), buf.size, C.c_void_p(ends.ctypes.data), cap,
                                      C.byref(cnt), C.byref(used))
    if rc not in (0, -4):
        _lib.check(rc, "spec_frames_index")
    return ends[: cnt.value], used.value


def frames_index_device(buf: torch.Tensor, cap: int | None = None, cuda_stream=None):
    """spec_frames_index_device over a device buffer (4-byte aligned): -> (ends int64 device
    tensor [count], consumed, status) — the host walk's results, computed on the GPU (reads the
    three scalars back, so this wrapper synchronises; the C call itself does not)."""
    _check_dev(buf, "buf", torch.uint8)
    n = buf.numel()
    cap = cap if cap is not None else max(1, n // 4)
    dev = buf.device
    ends = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
    out = torch.zeros(3, dtype=torch.int64, device=dev)  # count, consumed, status (int32 in slot 2)
    L = _lib.lib()
    ws_bytes = L.spec_frames_index_device_workspace_size(n)
    ws = torch.empty((ws_bytes + 7) // 8, dtype=torch.int64, device=dev)
    rc = L.spec_frames_index_device(_ptr(buf), n, _ptr(ends), cap, C.c_void_p(out.data_ptr()),
                                    C.c_void_p(out.data_ptr() + 8), C.c_void_p(out.data_ptr() + 16), _ptr(ws),
                                    ws_bytes, _stream_handle(cuda_stream))
    _lib.check(rc, "spec_frames_index_device")
    cnt, used, st = out.cpu().tolist()
    st = st - (1 << 32) if st >= (1 << 31) else st  # int32 in the low half of the zeroed slot
    return ends[:cnt], used, st


def make_frames_device(stream: torch.Tensor, ends: torch.Tensor) -> torch.Tensor:
    """make_frames on the device (benchmark input): a 4-byte BE head before every record."""
    n = ends.numel()
    out = torch.empty(stream.numel() + 4 * n, dtype=torch.uint8, device=stream.device)
    if n == 0:
        return out
    starts = torch.cat([ends.new_zeros(1), ends[:-1]])
    sizes = ends - starts
    rec = torch.searchsorted(ends, torch.arange(stream.numel(), device=stream.device), right=True)
    out[torch.arange(stream.numel(), device=stream.device) + 4 * (rec + 1)] = stream
    hpos = starts + 4 * torch.arange(n, device=stream.device)
    for b in range(4):
        out[hpos + b] = ((sizes >> (8 * (3 - b))) & 0xff).to(torch.uint8)
    return out


def make_frames(stream: np.ndarray, ends: np.ndarray) -> np.ndarray:
    """Records (stream + ends) -> mpx frames [u32 BE size][record]..."""
    ends = np.asarray(ends, dtype=np.int64)
    starts = np.concatenate([[0], ends[:-1]]) if len(ends) else ends
    sizes = (ends - starts).astype(np.uint32)
    out = np.empty(int(stream.size) + 4 * len(ends), dtype=np.uint8)
    pos = 0
    for s, z in zip(starts, sizes):
        out[pos:pos + 4] = np.frombuffer(int(z).to_bytes(4, "big"), dtype=np.uint8)
        out[pos + 4:pos + 4 + z] = stream[s:s + z]
        pos += 4 + int(z)
    return out


def decode_frames(schema: Schema, frames: torch.Tensor, ends: torch.Tensor, r0: int = 0, r1: int | None = None,
                  *, cols=None, status=None, cuda_stream=None) -> Columns:
    """spec_decode_frames: decode records [r0, r1) of a framed device buffer in place."""
    _check_dev(frames, "frames", torch.uint8)
    _check_dev(ends, "ends", torch.int64)
    n = ends.numel()
    r1 = n if r1 is None else r1
    if cols is None:
        cols = alloc_columns(schema, n, frames.device)
    if status is None:
        status = torch.empty(n, dtype=torch.uint8, device=frames.device)
    ptrs = (C.c_void_p * max(1, len(cols)))(*[c.data_ptr() for c in cols])
    rc = _lib.lib().spec_decode_frames(C.byref(schema.c), _ptr(frames), frames.numel(), _ptr(ends), r0, r1, 0,
                                       ptrs, _ptr(status), _stream_handle(cuda_stream))
    _lib.check(rc, "spec_decode_frames")
    return Columns(schema, cols, status)
