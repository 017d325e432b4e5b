"""spec_amd — MI355X-native bulk encode/decode engine for the spec binary format.

Drop-in for the hot path of basecomplextech/spec (encode.go, decode.go, writer*.go over
internal/{encode,decode,format,writer,types}): batches of records resident in HBM are
decoded into SoA columns / encoded from them by hand-written gfx950 kernels
(spec_amd/csrc, C ABI in include/spec_amd.h).  See DESIGN.md.
"""
from ._lib import LIB_PATH, SpecError, header_symbols, lib, set_jit
from .batch import (PARSE_LIST, PARSE_MESSAGE, PARSE_VALUE, Columns, Decoder, Encoder, alloc_columns, decode_flat,
                    decode_flat_errors, encode_flat, parse_messages)
from . import lz4
from .frames import decode_frames, frames_index, frames_index_device, make_frames, make_frames_device
from .pipeline import HostDecoder
from .nested import NestedColumns, NestedDecoder, NestedEncoder, decode_nested, encode_nested
from .schema import FLAT16, NESTED, Field, Kind, NestedSchema, Schema
from .tree import (ListOf, Message, Struct, Tree, TreeColumns, TreeDecoder, TreeEncoder, decode_tree, decode_values,
                   encode_tree, pkg1_message, pkg1_tree, tree_rows)

__all__ = [
    "HostDecoder", "decode_frames", "frames_index", "frames_index_device", "make_frames", "make_frames_device", "LIB_PATH", "SpecError", "header_symbols", "lib", "set_jit", "Columns", "Decoder", "Encoder", "alloc_columns",
    "decode_flat", "decode_flat_errors", "encode_flat", "parse_messages", "PARSE_MESSAGE", "PARSE_LIST", "PARSE_VALUE",
    "FLAT16", "Field", "Kind", "Schema",
    "NESTED", "NestedSchema", "NestedColumns", "NestedDecoder", "NestedEncoder", "decode_nested",
    "encode_nested", "ListOf", "Message", "Struct", "Tree", "TreeColumns", "TreeDecoder", "TreeEncoder", "decode_tree",
    "decode_values", "encode_tree", "pkg1_message", "pkg1_tree", "tree_rows",
]
