"""LZ4 — mpx connection compression (mpx/conn_writer.go:42-56, mpx/conn_reader.go:53-62: one
LZ4 frame of independent 256 KiB blocks per connection, pierrec/lz4/v4).

`frame_blocks` walks the frame headers and block size words on the host (spec_lz4_frame_blocks:
one u32 per block, header/block checksums verified); `decompress` runs every block on the GPU
(spec_lz4_decompress: one wave per block) and packs the blocks back to back
(spec_lz4_pack) — the decompressed mpx frames then go to frames_index_device + decode_frames.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from .batch import _check_dev, _ptr, _stream_handle

BLOCK_DTYPE = np.dtype([("src_off", "<u8"), ("src_len", "<u4"), ("stored", "<u4")])


class Lz4Block(C.Structure):
    """spec_lz4_block (the records BLOCK_DTYPE arrays hold)."""
    _fields_ = [("src_off", C.c_uint64), ("src_len", C.c_uint32), ("stored", C.c_uint32)]


class Lz4State(C.Structure):
    """An open frame carried across calls (zero for a new connection).  After a call, flags bit 2
    says a frame with a content checksum ended in it; content_checksum is that checksum."""
    _fields_ = [("in_frame", C.c_uint32), ("block_max", C.c_uint32), ("flags", C.c_uint32),
                ("content_checksum", C.c_uint32)]


class Lz4Content(C.Structure):
    """spec_lz4_content (lives in device memory; zero = a fresh frame)."""
    _fields_ = [("v", C.c_uint32 * 4), ("total", C.c_uint64), ("buf", C.c_uint8 * 16), ("buffered", C.c_uint32),
                ("started", C.c_uint32)]


class ContentChecksum:
    """The frame's content checksum on the device (spec_lz4_content_update / _digest): xxHash32 of
    every decompressed byte appended, over any number of calls — what lz4.Reader verifies at the
    frame's end (compare with Lz4State.content_checksum once flags bit 2 is set)."""

    def __init__(self, device="cuda"):
        self.state = torch.zeros(C.sizeof(Lz4Content), dtype=torch.uint8, device=device)
        self.out = torch.zeros(1, dtype=torch.int32, device=device)

    def update(self, data: torch.Tensor, cuda_stream=None):
        _check_dev(data, "data", torch.uint8)
        _lib.check(_lib.lib().spec_lz4_content_update(_ptr(self.state), _ptr(data) if data.numel() else None,
                                                      data.numel(), _stream_handle(cuda_stream)),
                   "spec_lz4_content_update")

    def digest(self, cuda_stream=None) -> int:
        _lib.check(_lib.lib().spec_lz4_content_digest(_ptr(self.state), _ptr(self.out), _stream_handle(cuda_stream)),
                   "spec_lz4_content_digest")
        return int(self.out.item()) & 0xFFFFFFFF


def frame_blocks(buf: np.ndarray, state: Lz4State | None = None, cap: int | None = None):
    """-> (blocks: structured array [src_off, src_len, stored], consumed, block_max, rc).
    rc is 0, or SPEC_E_CORRUPT (-6) / SPEC_E_CAPACITY (-4) with the blocks listed before it."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    state = state if state is not None else Lz4State()
    cap = cap if cap is not None else buf.size // 4 + 1
    blocks = np.zeros(max(cap, 1), dtype=BLOCK_DTYPE)
    nb, used, bmax = C.c_uint64(0), C.c_uint64(0), C.c_uint32(0)
    rc = _lib.lib().spec_lz4_frame_blocks(C.c_void_p(buf.ctypes.data if buf.size else 0), buf.size, C.byref(state),
                                          C.c_void_p(blocks.ctypes.data), cap, C.byref(nb), C.byref(used),
                                          C.byref(bmax))
    if rc not in (0, -4, -6):
        _lib.check(rc, "spec_lz4_frame_blocks")
    return blocks[: nb.value], used.value, bmax.value, rc


def decompress(src: torch.Tensor, blocks: np.ndarray, block_max: int, cuda_stream=None):
    """Every block of `src` (device copy of the compressed bytes) decompressed and packed:
    -> (stream uint8 device tensor, sizes uint32 [nblocks], status uint8 [nblocks]).  Raises if
    any block is corrupt (status says which)."""
    _check_dev(src, "src", torch.uint8)
    dev = src.device
    nb = len(blocks)
    L = _lib.lib()
    d_blocks = torch.from_numpy(np.ascontiguousarray(blocks).view(np.uint8).copy()).to(dev)
    slot = max(int(block_max), 4)
    slots = torch.empty(max(nb, 1) * slot, dtype=torch.uint8, device=dev)
    sizes = torch.empty(max(nb, 1), dtype=torch.int32, device=dev)
    status = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
    s = _stream_handle(cuda_stream)
    rc = L.spec_lz4_decompress(_ptr(src), src.numel(), _ptr(d_blocks), nb, _ptr(slots), slot, _ptr(sizes),
                               _ptr(status), s)
    _lib.check(rc, "spec_lz4_decompress")
    out = torch.empty(max(nb, 1) * slot, dtype=torch.uint8, device=dev)
    wsb = L.spec_lz4_pack_workspace_size(nb)
    ws = torch.empty((wsb + 7) // 8, dtype=torch.int64, device=dev)
    total = torch.zeros(1, dtype=torch.int64, device=dev)
    rc = L.spec_lz4_pack(_ptr(slots), slot, _ptr(sizes), nb, _ptr(out), out.numel(), _ptr(total), _ptr(ws), wsb, s)
    _lib.check(rc, "spec_lz4_pack")
    t = int(total.item())
    if t < 0:
        raise _lib.SpecError(-6, "spec_lz4_decompress: corrupt block")
    return out[:t], sizes[:nb].view(torch.int32), status[:nb]
