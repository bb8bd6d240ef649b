"""covtiles_amd -- MI355X-native COVT Id/Geometry stream decoder (host side).

Python mirror of the reference's decoder API (springmeyer/cov-tiles, evaluation/java,
package ``com.covt.decoder``) over the C-ABI of ``libcovt.so`` (``include/covt.h``):

* ``DecodingUtils`` -- one static method per ``DecodingUtils.java`` method, same names, argument
  order and ``IntWrapper`` cursor semantics; errors raise the Python analogue of the Java exception.
* ``CovtParser.decode_covt`` -- the Id + Geometry part of ``CovtParser.decodeCovt`` for one tile.
* ``Plan`` / ``DeviceBatch`` -- the batch path: host metadata walk -> descriptor table -> one
  GPU launch over every stream of every tile, with device-resident inputs/outputs (torch tensors
  are used as device memory and for the HIP stream; they are plumbing, not the decoder).

The directory name contains a dash, so import it through ``load()`` below or
``importlib`` (``tests/conftest.py`` and ``bench.py`` do).  There is no CPU fallback: if
``libcovt.so`` is missing or no GPU is visible, the decode entry points raise.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, os.environ.get("COVT_LIB_VARIANT", "libcovt.so"))  # tools: libcovt_timing.so

OK = 0
ERR_UNSUPPORTED_ENCODING = -1
ERR_TRUNCATED = -2
ERR_COUNT_MISMATCH = -3
ERR_BAD_HEADER = -4
ERR_DEVICE = -5
ERR_INVALID_ARG = -6
INPUT_PADDING = 4096
FORMAT_GENC, FORMAT_GEND = 0, 1
FAMILY_RLE, FAMILY_VARINT, FAMILY_FASTPFOR, FAMILY_LANE, FAMILY_SPLIT, FAMILY_SPLIT_FPF, FAMILY_SPLIT_RLE = range(7)
NUM_FAMILIES = 7
DESC_LANE, DESC_SPLIT, DESC_SPLIT_PAD, DESC_SPLIT_FPF = 0x1, 0x2, 0x4, 0x8
DESC_SPLIT_RLE = 0x10
SPLIT_SLOTS = 8
ID_FORMAT, ID_JAVA = 0, 1
LAUNCH_AUTO, LAUNCH_FUSED, LAUNCH_FORKED = 0, 1, 2
LAUNCH_FPF_STREAM, LAUNCH_FPF_CLASSIC = 0x4, 0x8  # or-ed in: the FastPFOR family kernel variant (include/covt.h)

(OP_NONE, OP_BYTE_RLE_U8, OP_RLE_U64, OP_RLE_I32, OP_RLE_S64, OP_VARINT_I32, OP_VARINT_ZZ_I32,
 OP_VARINT_ZZ_DELTA_I32, OP_VARINT_ZZ_DELTA_XY, OP_VARINT_DELTA_MORTON, OP_FPF_ZZ_DELTA_I32, OP_FPF_ZZ_DELTA_XY,
 OP_FPF_DELTA_MORTON, OP_VARINT_U64, OP_VARINT_I32_AS_I64, OP_VARINT_ZZ_DELTA_I64, OP_BYTE_RLE_RAW,
 OP_VARINT_ZZ_I32_AS_I64, OP_VARINT_ZZ_S64, OP_VARINT_ZZ_DELTA_S64) = range(20)

# property columns (include/covt.h "Property columns")
PLAN_PROPERTIES = 0x1
RELEASE_PINNED = 0x2  # covt_release_scratch flag: also free blocks pinned by a graph capture
PROP_BOOLEAN, PROP_INT64, PROP_FLOAT, PROP_STRING = 0, 1, 2, 3
PROP_DICT_OWNER, PROP_DENSE_BOOL, PROP_UNSUPPORTED, PROP_DATA_SHORT, PROP_UNSUPPORTED_LATE = 0x1, 0x2, 0x4, 0x8, 0x10

# StreamType ordinals (converter/StreamType.java)
GEOMETRY_TYPES, GEOMETRY_OFFSETS, PART_OFFSETS, RING_OFFSETS, VERTEX_OFFSETS, VERTEX_BUFFER = range(4, 10)


# ---------------------------------------------------------------------------
# Java exception analogues (status -> exception), CovtParser.java:426 etc.
# ---------------------------------------------------------------------------
class CovtError(Exception):
    status = 0


class IllegalArgumentException(CovtError, ValueError):
    pass


class ArrayIndexOutOfBoundsException(CovtError, IndexError):
    pass


class DeviceError(CovtError, RuntimeError):
    pass


def _raise(status: int, what: str):
    if status == OK:
        return
    cls = {ERR_UNSUPPORTED_ENCODING: IllegalArgumentException, ERR_BAD_HEADER: IllegalArgumentException,
           ERR_INVALID_ARG: IllegalArgumentException, ERR_TRUNCATED: ArrayIndexOutOfBoundsException,
           ERR_COUNT_MISMATCH: ArrayIndexOutOfBoundsException}.get(status, DeviceError)
    e = cls("%s failed with status %d" % (what, status))
    e.status = status
    raise e


# ---------------------------------------------------------------------------
# C-ABI binding
# ---------------------------------------------------------------------------
class StreamDesc(C.Structure):
    _fields_ = [("in_off", C.c_uint64), ("out_off", C.c_uint64), ("avail", C.c_int32), ("num_values", C.c_int32),
                ("op", C.c_uint8), ("num_bits", C.c_uint8), ("flags", C.c_uint16), ("byte_length", C.c_int32)]


class StreamResult(C.Structure):
    _fields_ = [("status", C.c_int32), ("consumed", C.c_int32)]


class StreamInfo(C.Structure):
    _fields_ = [("tile", C.c_int32), ("layer", C.c_int32), ("column_kind", C.c_int32), ("stream_type", C.c_int32),
                ("encoding", C.c_int32), ("column_type", C.c_int32), ("num_values", C.c_int32),
                ("byte_length", C.c_int32), ("num_bits", C.c_int32), ("op", C.c_int32), ("elem_bytes", C.c_int32),
                ("desc_index", C.c_int32), ("in_off", C.c_int64), ("out_off", C.c_int64),
                ("out_elems", C.c_int64)]


class GeomDesc(C.Structure):
    _fields_ = [("in_off", C.c_int64 * 6), ("in_len", C.c_int32 * 6), ("in_res", C.c_int32 * 6),
                ("out_off", C.c_int64 * 6), ("part_cap", C.c_int32), ("ring_cap", C.c_int32),
                ("coord_cap", C.c_int32), ("flags", C.c_int32)]


class GeomResult(C.Structure):
    _fields_ = [("status", C.c_int32), ("num_parts", C.c_int32), ("num_rings", C.c_int32),
                ("num_coords", C.c_int32)]


GEOM_INFO_DTYPE = np.dtype([("tile", np.int32), ("layer", np.int32), ("column_type", np.int32),
                            ("n_features", np.int32), ("stream", np.int32, (6,)), ("part_cap", np.int32),
                            ("ring_cap", np.int32), ("coord_cap", np.int32), ("flags", np.uint32),
                            ("desc_index", np.int32), ("reserved", np.int32), ("out_off", np.int64, (6,))])
GEOM_RESULT_DTYPE = np.dtype([("status", np.int32), ("num_parts", np.int32), ("num_rings", np.int32),
                              ("num_coords", np.int32)])
PROP_INFO_DTYPE = np.dtype([("tile", np.int32), ("layer", np.int32), ("column", np.int32), ("type", np.int32),
                            ("column_type", np.int32), ("n_features", np.int32), ("n_data", np.int32),
                            ("n_dict", np.int32), ("lang", np.int32), ("name_len", np.int32), ("lang_len", np.int32),
                            ("dict_bytes", np.int32), ("stream", np.int32, (3,)), ("desc_index", np.int32),
                            ("name_off", np.int64), ("lang_off", np.int64), ("out_off", np.int64, (4,))])
PROP_DESC_DTYPE = np.dtype([("present_off", np.int64), ("data_off", np.int64), ("length_off", np.int64),
                            ("dict_in_off", np.int64), ("out_off", np.int64, (4,)), ("res", np.int32, (3,)),
                            ("n_features", np.int32), ("n_data", np.int32), ("n_dict", np.int32),
                            ("dict_bytes", np.int32), ("type", np.int16), ("flags", np.int16)])
PROP_RESULT_DTYPE = np.dtype([("status", np.int32), ("n_valid", np.int32)])
assert PROP_INFO_DTYPE.itemsize == 112 and PROP_DESC_DTYPE.itemsize == 96
GEOM_CLOSED_IN_STREAM = 0x1
GEOM_TOO_LARGE = 0x80000000
GEOM_MAX_CAP = 1 << 25
assert C.sizeof(GeomDesc) == 160 and GEOM_INFO_DTYPE.itemsize == 112

class PlanOptions(C.Structure):
    """covt_plan_options (include/covt.h): the plan-layout options.  ``PlanOptions()`` holds the
    library defaults (covt_plan_options_init); keyword arguments override fields, e.g.
    ``PlanOptions(split_min=-1)`` plans no split streams."""
    _fields_ = [("size", C.c_uint32), ("flags", C.c_uint32), ("split_min", C.c_int64), ("split_ratio", C.c_int64),
                ("split_chunk", C.c_int64), ("split_values", C.c_int64), ("fpf_split_weight", C.c_int32),
                ("lane_max_bytes", C.c_int32), ("lane_min_streams", C.c_int64), ("plan_threads", C.c_int32),
                ("host_prefault", C.c_int32), ("prefault_threads", C.c_int32), ("device_walk", C.c_int32),
                ("lane_max_values", C.c_int32), ("split_max_streams", C.c_int64),
                ("split_grow", C.c_int32)]

    def __init__(self, **kw):
        super().__init__()
        lib().covt_plan_options_init(C.byref(self))
        for k, v in kw.items():
            if k not in {f[0] for f in self._fields_} or k == "size":
                raise TypeError("unknown plan option %r" % k)
            setattr(self, k, v)

    def __repr__(self):
        return "PlanOptions(%s)" % ", ".join("%s=%r" % (f, getattr(self, f)) for f, _ in self._fields_[1:])


STREAM_INFO_DTYPE = np.dtype([(n, np.int32 if t is C.c_int32 else np.int64) for n, t in StreamInfo._fields_])
assert STREAM_INFO_DTYPE.itemsize == C.sizeof(StreamInfo)
assert C.sizeof(StreamDesc) == 32

EXPORTED_SYMBOLS = (
    "covt_decode_varint", "covt_decode_zigzag_varint", "covt_decode_zigzag_delta_varint",
    "covt_decode_zigzag_delta_varint_coordinates", "covt_decode_rle", "covt_decode_byte_rle",
    "covt_decode_fastpfor_zigzag_delta", "covt_decode_fastpfor_delta_coordinates",
    "covt_decode_delta_varint_morton_codes", "covt_decode_fastpfor_delta_morton_codes",
    "covt_plan_create", "covt_plan_destroy", "covt_plan_num_streams", "covt_plan_output_bytes",
    "covt_plan_totals", "covt_plan_streams", "covt_plan_descs", "covt_plan_tile_status",
    "covt_decode_streams_device", "covt_plan_decode_host", "covt_plan_decode_host_multi", "covt_version",
    "covt_device_count", "covt_plan_family_counts", "covt_decode_streams_device_grouped",
    "covt_decode_streams_device_grouped_mode",
    "covt_plan_num_geometry_columns", "covt_plan_assembly_bytes", "covt_plan_geometry_columns",
    "covt_plan_geometry_descs", "covt_assemble_geometry_device", "covt_plan_assemble_host",
    "covt_plan_create_ex", "covt_plan_num_property_columns", "covt_plan_property_bytes",
    "covt_plan_property_columns", "covt_plan_property_descs", "covt_materialize_properties_device",
    "covt_plan_properties_host", "covt_decode_byte_rle_reencode", "covt_decode_floats_le", "covt_decode_string",
    "covt_plan_decode_host_shards", "covt_plan_release_device", "covt_plan_num_descs", "covt_plan_desc_streams",
    "covt_device_plan_create", "covt_device_plan_destroy", "covt_device_plan_num_streams",
    "covt_device_plan_output_bytes", "covt_device_plan_totals", "covt_device_plan_family_counts",
    "covt_device_plan_descs_device", "covt_device_plan_streams_device", "covt_device_plan_tile_status_device",
    "covt_device_plan_order_device", "covt_device_plan_copy", "covt_device_plan_decode",
    "covt_plan_options_init", "covt_plan_create_opts", "covt_device_plan_create_opts",
    "covt_device_plan_num_descs", "covt_device_plan_geometry", "covt_device_plan_num_geometry_columns",
    "covt_device_plan_assembly_bytes", "covt_device_plan_geometry_descs_device", "covt_device_plan_geometry_copy",
    "covt_device_plan_assemble", "covt_device_plan_num_property_columns", "covt_device_plan_property_bytes",
    "covt_device_plan_property_descs_device", "covt_device_plan_property_copy", "covt_device_plan_materialize",
    "covt_release_scratch", "covt_scratch_blocks", "covt_device_plan_pool_trim",
)


def release_scratch(stream=None, all: bool = False, pinned: bool = False) -> int:
    """covt_release_scratch: free the small-batch assembly / property scratch of (current device, `stream`),
    or every block with all=True; blocks pinned by a graph capture only with pinned=True (no graph captured
    on them may replay afterwards); returns the number of blocks freed."""
    import torch

    s = stream if stream is not None else (torch.cuda.current_stream() if not all else None)
    flags = (1 if all else 0) | (RELEASE_PINNED if pinned else 0)
    return lib().covt_release_scratch(C.c_void_p(s.cuda_stream if s is not None else 0), flags)


def scratch_blocks() -> int:
    """Scratch blocks held by the small-batch paths (covt_scratch_blocks)."""
    return int(lib().covt_scratch_blocks())


def build(force: bool = False) -> str:
    """Compile libcovt.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    args = ["make", "-s", "-C", _HERE, "libcovt.so"]
    if force:
        subprocess.check_call(["make", "-s", "-C", _HERE, "clean"])
    subprocess.check_call(args)
    return _LIB


_lib = None


def lib() -> C.CDLL:
    """Load libcovt.so.  torch is imported first so libcovt binds to the same HIP runtime."""
    global _lib
    if _lib is not None:
        return _lib
    try:
        import torch  # noqa: F401  -- shares its libamdhip64 with libcovt (same SONAME)
    except ImportError:
        pass
    if not os.path.exists(_LIB):
        raise ImportError("libcovt.so is not built (run __graft_entry__.build() or make -C cov-tiles_amd)")
    L = C.CDLL(_LIB)
    u8p, i32p, i64p, vp = C.POINTER(C.c_uint8), C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.c_void_p
    sz = C.c_size_t
    for name in ("covt_decode_varint", "covt_decode_zigzag_varint", "covt_decode_zigzag_delta_varint",
                 "covt_decode_zigzag_delta_varint_coordinates"):
        getattr(L, name).argtypes = [u8p, sz, i32p, C.c_int32, i32p]
    L.covt_decode_rle.argtypes = [u8p, sz, C.c_int32, i32p, C.c_int32, i64p]
    L.covt_decode_byte_rle.argtypes = [u8p, sz, C.c_int32, i32p, C.c_int32, u8p]
    L.covt_decode_fastpfor_zigzag_delta.argtypes = [u8p, sz, C.c_int32, C.c_int32, i32p, i32p]
    L.covt_decode_fastpfor_delta_coordinates.argtypes = [u8p, sz, C.c_int32, C.c_int32, i32p, i32p]
    L.covt_decode_delta_varint_morton_codes.argtypes = [u8p, sz, i32p, C.c_int32, C.c_int32, i32p]
    L.covt_decode_fastpfor_delta_morton_codes.argtypes = [u8p, sz, C.c_int32, C.c_int32, i32p, C.c_int32, i32p]
    L.covt_plan_create.argtypes = [u8p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_int32, C.c_int32,
                                   C.c_int32, C.POINTER(vp)]
    L.covt_plan_destroy.argtypes = [vp]
    L.covt_plan_destroy.restype = None
    L.covt_plan_num_streams.argtypes = [vp]
    L.covt_plan_num_streams.restype = C.c_int64
    L.covt_plan_output_bytes.argtypes = [vp]
    L.covt_plan_output_bytes.restype = C.c_int64
    L.covt_plan_totals.argtypes = [vp, i64p, i64p, i64p]
    L.covt_plan_streams.argtypes = [vp, vp]
    L.covt_plan_descs.argtypes = [vp, vp]
    L.covt_plan_num_descs.argtypes = [vp]
    L.covt_plan_num_descs.restype = C.c_int64
    L.covt_plan_desc_streams.argtypes = [vp, i64p]
    L.covt_plan_tile_status.argtypes = [vp, i32p]
    L.covt_decode_streams_device.argtypes = [vp, vp, C.c_int64, vp, vp, vp]
    L.covt_decode_streams_device_grouped.argtypes = [vp, vp, i64p, vp, vp, vp]
    L.covt_decode_streams_device_grouped_mode.argtypes = [vp, vp, i64p, vp, vp, vp, C.c_int32]
    L.covt_plan_family_counts.argtypes = [vp, i64p]
    L.covt_plan_decode_host.argtypes = [vp, u8p, C.c_uint64, vp, vp]
    L.covt_plan_decode_host_multi.argtypes = [vp, u8p, C.c_uint64, C.c_int32, vp, vp]
    L.covt_plan_decode_host_shards.argtypes = [vp, u8p, C.c_uint64, C.c_int32, i32p, vp, vp]
    L.covt_plan_release_device.argtypes = [vp]
    L.covt_decode_byte_rle_reencode.argtypes = [u8p, sz, C.c_int32, i32p, u8p]
    L.covt_decode_floats_le.argtypes = [u8p, sz, i32p, C.c_int32, C.POINTER(C.c_float)]
    L.covt_decode_string.argtypes = [u8p, sz, i32p, i32p, i32p]
    L.covt_plan_num_geometry_columns.argtypes = [vp]
    L.covt_plan_num_geometry_columns.restype = C.c_int64
    L.covt_plan_assembly_bytes.argtypes = [vp]
    L.covt_plan_assembly_bytes.restype = C.c_int64
    L.covt_plan_geometry_columns.argtypes = [vp, vp]
    L.covt_plan_geometry_descs.argtypes = [vp, vp]
    L.covt_assemble_geometry_device.argtypes = [vp, vp, vp, C.c_int64, vp, vp, vp]
    L.covt_release_scratch.argtypes = [vp, C.c_int]
    L.covt_scratch_blocks.restype = C.c_int64
    L.covt_device_plan_pool_trim.argtypes = [C.c_int, C.c_uint64]
    L.covt_plan_assemble_host.argtypes = [vp, u8p, C.c_uint64, vp, vp]
    L.covt_plan_create_ex.argtypes = [u8p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_int32, C.c_int32,
                                      C.c_int32, C.c_uint32, C.POINTER(vp)]
    L.covt_plan_options_init.argtypes = [vp]
    L.covt_plan_options_init.restype = None
    L.covt_plan_create_opts.argtypes = [u8p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_int32, C.c_int32,
                                        C.c_int32, vp, C.POINTER(vp)]
    L.covt_device_plan_create_opts.argtypes = [vp, C.c_uint64, vp, vp, C.c_int32, C.c_int32, C.c_int32, vp, vp,
                                               C.POINTER(vp)]
    L.covt_plan_num_property_columns.argtypes = [vp]
    L.covt_plan_num_property_columns.restype = C.c_int64
    L.covt_plan_property_bytes.argtypes = [vp]
    L.covt_plan_property_bytes.restype = C.c_int64
    L.covt_plan_property_columns.argtypes = [vp, vp]
    L.covt_plan_property_descs.argtypes = [vp, vp]
    L.covt_materialize_properties_device.argtypes = [vp, vp, vp, vp, C.c_int64, vp, vp, vp]
    L.covt_plan_properties_host.argtypes = [vp, u8p, C.c_uint64, vp, vp]
    L.covt_device_plan_create.argtypes = [vp, C.c_uint64, vp, vp, C.c_int32, C.c_int32, C.c_int32, vp,
                                          C.POINTER(vp)]
    L.covt_device_plan_destroy.argtypes = [vp]
    L.covt_device_plan_destroy.restype = None
    for name in ("covt_device_plan_num_streams", "covt_device_plan_num_descs", "covt_device_plan_output_bytes"):
        getattr(L, name).argtypes = [vp]
        getattr(L, name).restype = C.c_int64
    L.covt_device_plan_totals.argtypes = [vp, i64p, i64p, i64p]
    L.covt_device_plan_family_counts.argtypes = [vp, i64p]
    for name in ("covt_device_plan_descs_device", "covt_device_plan_streams_device",
                 "covt_device_plan_tile_status_device", "covt_device_plan_order_device"):
        getattr(L, name).argtypes = [vp]
        getattr(L, name).restype = vp
    L.covt_device_plan_copy.argtypes = [vp, vp, vp, i32p]
    L.covt_device_plan_decode.argtypes = [vp, vp, vp, vp, vp]
    L.covt_device_plan_geometry.argtypes = [vp, vp]
    L.covt_device_plan_num_geometry_columns.argtypes = [vp]
    L.covt_device_plan_num_geometry_columns.restype = C.c_int64
    L.covt_device_plan_assembly_bytes.argtypes = [vp]
    L.covt_device_plan_assembly_bytes.restype = C.c_int64
    L.covt_device_plan_geometry_descs_device.argtypes = [vp]
    L.covt_device_plan_geometry_descs_device.restype = vp
    L.covt_device_plan_geometry_copy.argtypes = [vp, vp, vp]
    L.covt_device_plan_assemble.argtypes = [vp, vp, vp, vp, vp, vp]
    L.covt_device_plan_num_property_columns.argtypes = [vp]
    L.covt_device_plan_num_property_columns.restype = C.c_int64
    L.covt_device_plan_property_bytes.argtypes = [vp]
    L.covt_device_plan_property_bytes.restype = C.c_int64
    L.covt_device_plan_property_descs_device.argtypes = [vp]
    L.covt_device_plan_property_descs_device.restype = vp
    L.covt_device_plan_property_copy.argtypes = [vp, vp, vp]
    L.covt_device_plan_materialize.argtypes = [vp, vp, vp, vp, vp, vp, vp]
    L.covt_version.restype = C.c_char_p
    L.covt_device_count.argtypes = [i32p]
    _lib = L
    return L


def device_count() -> int:
    n = C.c_int32(0)
    lib().covt_device_count(C.byref(n))
    return n.value


def _u8(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        return np.ascontiguousarray(buf, dtype=np.uint8)
    return np.frombuffer(bytes(buf), dtype=np.uint8)


def _ptr(a: np.ndarray, t):
    return a.ctypes.data_as(C.POINTER(t))


# ---------------------------------------------------------------------------
# DecodingUtils mirror (DecodingUtils.java)
# ---------------------------------------------------------------------------
class IntWrapper:
    """me.lemire.integercompression.IntWrapper: the mutable cursor of the Java API."""

    def __init__(self, v: int = 0):
        self.value = int(v)

    def get(self) -> int:
        return self.value

    def set(self, v: int) -> None:
        self.value = int(v)

    def increment(self) -> None:
        self.value += 1

    def add(self, v: int) -> None:
        self.value += int(v)

    def __repr__(self):
        return "IntWrapper(%d)" % self.value


def _cursor(pos):
    return pos if isinstance(pos, IntWrapper) else IntWrapper(pos)


class DecodingUtils:
    """Static methods mirroring com.covt.decoder.DecodingUtils (names, argument order, semantics).
    Every call decodes on the GPU through libcovt."""

    @staticmethod
    def _varint_like(fn, src, pos, n, out_n, what):
        pos = _cursor(pos)
        a = _u8(src)
        out = np.zeros(max(out_n, 1), dtype=np.int32)
        p = C.c_int32(pos.get())
        _raise(getattr(lib(), fn)(_ptr(a, C.c_uint8), a.size, C.byref(p), int(n), _ptr(out, C.c_int32)), what)
        pos.set(p.value)
        return out[:out_n]

    @staticmethod
    def decodeVarint(src, pos: IntWrapper, numValues: int) -> np.ndarray:  # DecodingUtils.java:35
        return DecodingUtils._varint_like("covt_decode_varint", src, pos, numValues, numValues, "decodeVarint")

    @staticmethod
    def decodeZigZagVarint(src, pos: IntWrapper, numValues: int) -> np.ndarray:  # :46
        return DecodingUtils._varint_like("covt_decode_zigzag_varint", src, pos, numValues, numValues,
                                          "decodeZigZagVarint")

    @staticmethod
    def decodeZigZagDeltaVarint(src, pos: IntWrapper, numValues: int) -> np.ndarray:  # :55
        return DecodingUtils._varint_like("covt_decode_zigzag_delta_varint", src, pos, numValues, numValues,
                                          "decodeZigZagDeltaVarint")

    @staticmethod
    def decodeZigZagDeltaVarintCoordinates(src, pos: IntWrapper, numValues: int) -> np.ndarray:  # :95
        return DecodingUtils._varint_like("covt_decode_zigzag_delta_varint_coordinates", src, pos, numValues,
                                          numValues, "decodeZigZagDeltaVarintCoordinates")

    @staticmethod
    def decodeDeltaVarintMortonCodes(src, pos: IntWrapper, numVertices: int, numBits: int) -> np.ndarray:  # :394
        pos = _cursor(pos)
        a = _u8(src)
        out = np.zeros(max(2 * numVertices, 1), dtype=np.int32)
        p = C.c_int32(pos.get())
        _raise(lib().covt_decode_delta_varint_morton_codes(_ptr(a, C.c_uint8), a.size, C.byref(p), numVertices,
                                                           numBits, _ptr(out, C.c_int32)),
               "decodeDeltaVarintMortonCodes")
        pos.set(p.value)
        return out[:2 * numVertices]

    @staticmethod
    def decodeRle(buffer, numValues: int, pos: IntWrapper, signed: bool) -> np.ndarray:  # :257
        pos = _cursor(pos)
        a = _u8(buffer)
        out = np.zeros(max(numValues, 1), dtype=np.int64)
        p = C.c_int32(pos.get())
        _raise(lib().covt_decode_rle(_ptr(a, C.c_uint8), a.size, numValues, C.byref(p), int(bool(signed)),
                                     _ptr(out, C.c_int64)), "decodeRle")
        pos.set(p.value)
        return out[:numValues]

    @staticmethod
    def decodeByteRle(buffer, numValues: int, pos: IntWrapper, byteLength: Optional[int] = None) -> np.ndarray:
        """:275 (with byteLength: advance by it) and the :290 overload (without: advance by the length
        of the values' ORC re-encoding, as CovtParser.java:295 relies on for Gen D present streams)."""
        pos = _cursor(pos)
        a = _u8(buffer)
        out = np.zeros(max(numValues, 1), dtype=np.uint8)
        p = C.c_int32(pos.get())
        if byteLength is None:
            st = lib().covt_decode_byte_rle_reencode(_ptr(a, C.c_uint8), a.size, numValues, C.byref(p),
                                                     _ptr(out, C.c_uint8))
        else:
            st = lib().covt_decode_byte_rle(_ptr(a, C.c_uint8), a.size, numValues, C.byref(p), byteLength,
                                            _ptr(out, C.c_uint8))
        _raise(st, "decodeByteRle")
        pos.set(p.value)
        return out[:numValues]

    @staticmethod
    def decodeFloatsLE(encodedValues, pos: IntWrapper, numValues: int) -> np.ndarray:  # :446
        pos = _cursor(pos)
        a = _u8(encodedValues)
        out = np.zeros(max(numValues, 1), dtype=np.float32)
        p = C.c_int32(pos.get())
        _raise(lib().covt_decode_floats_le(_ptr(a, C.c_uint8), a.size, C.byref(p), numValues,
                                           out.ctypes.data_as(C.POINTER(C.c_float))), "decodeFloatsLE")
        pos.set(p.value)
        return out[:numValues]

    @staticmethod
    def decodeString(content, pos: IntWrapper, numChars: Optional[int] = None) -> str:  # :21 / :28
        pos = _cursor(pos)
        a = _u8(content)
        if numChars is not None:  # :28 -- the caller knows the length
            if pos.get() < 0 or pos.get() + numChars > a.size or numChars < 0:
                _raise(ERR_TRUNCATED, "decodeString")
            s = bytes(a[pos.get():pos.get() + numChars]).decode("utf-8", errors="replace")
            pos.set(pos.get() + numChars)
            return s
        p, off, ln = C.c_int32(pos.get()), C.c_int32(), C.c_int32()
        _raise(lib().covt_decode_string(_ptr(a, C.c_uint8), a.size, C.byref(p), C.byref(off), C.byref(ln)),
               "decodeString")
        pos.set(p.value)
        return bytes(a[off.value:off.value + ln.value]).decode("utf-8", errors="replace")

    @staticmethod
    def _fpf(fn, buf, n, byte_length, pos, out_n, extra, what):
        pos = _cursor(pos)
        a = _u8(buf)
        out = np.zeros(max(out_n, 1), dtype=np.int32)
        p = C.c_int32(pos.get())
        args = [_ptr(a, C.c_uint8), a.size, n, byte_length, C.byref(p)] + extra + [_ptr(out, C.c_int32)]
        _raise(getattr(lib(), fn)(*args), what)
        pos.set(p.value)
        return out[:out_n]

    @staticmethod
    def decodeFastPfor128ZigZagDelta(encodedValues, numValues: int, byteLength: int, pos: IntWrapper):  # :316
        return DecodingUtils._fpf("covt_decode_fastpfor_zigzag_delta", encodedValues, numValues, byteLength, pos,
                                  numValues, [], "decodeFastPfor128ZigZagDelta")

    @staticmethod
    def decodeFastPfor128DeltaCoordinates(encodedValues, numValues: int, byteLength: int, pos: IntWrapper):  # :349
        return DecodingUtils._fpf("covt_decode_fastpfor_delta_coordinates", encodedValues, numValues, byteLength,
                                  pos, numValues, [], "decodeFastPfor128DeltaCoordinates")

    @staticmethod
    def decodeFastPfor128DeltaMortonCodes(encodedValues, numVertices: int, byteLength: int, pos: IntWrapper,
                                          numBits: int):  # :411
        return DecodingUtils._fpf("covt_decode_fastpfor_delta_morton_codes", encodedValues, numVertices,
                                  byteLength, pos, 2 * numVertices, [numBits], "decodeFastPfor128DeltaMortonCodes")


# ---------------------------------------------------------------------------
# Batch path
# ---------------------------------------------------------------------------
def pack_tiles(tiles: List[bytes], align: int = 16):
    """Concatenate tiles (16-byte aligned starts) -> (uint8 blob incl. INPUT_PADDING, offsets, sizes)."""
    sizes = np.array([len(t) for t in tiles], dtype=np.uint64)
    offs = np.zeros(len(tiles), dtype=np.uint64)
    pos = 0
    for i, t in enumerate(tiles):
        offs[i] = pos
        pos += (len(t) + align - 1) // align * align
    blob = np.zeros(pos + INPUT_PADDING, dtype=np.uint8)
    for i, t in enumerate(tiles):
        blob[int(offs[i]):int(offs[i]) + len(t)] = np.frombuffer(t, dtype=np.uint8)
    return blob, offs, sizes


class Plan:
    """Host-side container walk of a tile batch -> per-stream descriptors (covt_plan_create)."""

    def __init__(self, blob: np.ndarray, offsets, sizes, fmt: int = FORMAT_GENC, id_mode: int = ID_FORMAT,
                 flags: int = 0, options: Optional[PlanOptions] = None):
        L = lib()
        self.blob = np.ascontiguousarray(blob, dtype=np.uint8)
        self.offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        self.sizes = np.ascontiguousarray(sizes, dtype=np.uint64)
        self.n_tiles = int(self.offsets.size)
        opts = PlanOptions() if options is None else PlanOptions(**{f: getattr(options, f) for f, _ in
                                                                   PlanOptions._fields_[1:]})
        opts.flags |= flags
        self.options = opts
        h = C.c_void_p()
        _raise(L.covt_plan_create_opts(_ptr(self.blob, C.c_uint8), _ptr(self.offsets, C.c_uint64),
                                       _ptr(self.sizes, C.c_uint64), self.n_tiles, fmt, id_mode, C.byref(opts),
                                       C.byref(h)), "covt_plan_create")
        self._h = h
        self.num_streams = int(L.covt_plan_num_streams(h))
        self.output_bytes = int(L.covt_plan_output_bytes(h))
        ib, ob, vx = C.c_int64(), C.c_int64(), C.c_int64()
        L.covt_plan_totals(h, C.byref(ib), C.byref(ob), C.byref(vx))
        self.in_bytes, self.out_bytes, self.vertices = ib.value, ob.value, vx.value
        self.streams = np.zeros(self.num_streams, dtype=STREAM_INFO_DTYPE)
        if self.num_streams:
            L.covt_plan_streams(h, self.streams.ctypes.data)
        self.num_descs = int(L.covt_plan_num_descs(h))  # >= num_streams: split chunks and their pads
        self.descs = np.zeros(self.num_descs * 32, dtype=np.uint8)
        self.desc_streams = np.zeros(self.num_descs, dtype=np.int64)
        if self.num_descs:
            L.covt_plan_descs(h, self.descs.ctypes.data)
            L.covt_plan_desc_streams(h, _ptr(self.desc_streams, C.c_int64))
        self.family_counts = np.zeros(NUM_FAMILIES, dtype=np.int64)
        L.covt_plan_family_counts(h, _ptr(self.family_counts, C.c_int64))
        self.tile_status = np.zeros(max(self.n_tiles, 1), dtype=np.int32)[:self.n_tiles]
        if self.n_tiles:
            L.covt_plan_tile_status(h, _ptr(self.tile_status, C.c_int32))
        # geometry assembly (include/covt.h "Geometry assembly")
        self.num_geometry_columns = int(L.covt_plan_num_geometry_columns(h))
        self.assembly_bytes = int(L.covt_plan_assembly_bytes(h))
        self.geom = np.zeros(self.num_geometry_columns, dtype=GEOM_INFO_DTYPE)
        self.gdescs = np.zeros(self.num_geometry_columns * C.sizeof(GeomDesc), dtype=np.uint8)
        if self.num_geometry_columns:
            L.covt_plan_geometry_columns(h, self.geom.ctypes.data)
            L.covt_plan_geometry_descs(h, self.gdescs.ctypes.data)
        # property columns (include/covt.h "Property columns"; plans made with PLAN_PROPERTIES)
        self.num_property_columns = int(L.covt_plan_num_property_columns(h))
        self.property_bytes = int(L.covt_plan_property_bytes(h))
        self.props = np.zeros(self.num_property_columns, dtype=PROP_INFO_DTYPE)
        self.pdescs = np.zeros(self.num_property_columns, dtype=PROP_DESC_DTYPE)
        if self.num_property_columns:
            L.covt_plan_property_columns(h, self.props.ctypes.data)
            L.covt_plan_property_descs(h, self.pdescs.ctypes.data)

    @classmethod
    def from_tiles(cls, tiles: List[bytes], fmt: int = FORMAT_GENC, id_mode: int = ID_FORMAT, flags: int = 0,
                   options: Optional[PlanOptions] = None):
        blob, offs, sizes = pack_tiles(tiles)
        return cls(blob, offs, sizes, fmt, id_mode, flags, options)

    def close(self):
        if getattr(self, "_h", None):
            lib().covt_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def release_device(self):
        """Free the device buffers decode_host cached on this plan (covt_plan_release_device)."""
        _raise(lib().covt_plan_release_device(self._h), "covt_plan_release_device")

    def decode_host(self, n_gpus: int = 1, out=None, res=None, shard_devices=None):
        """H2D + decode + D2H of the whole plan (covt_plan_decode_host[_multi]).
        Returns (uint8 output buffer, results[num_streams, 2] = (status, consumed)) in plan order.
        `out` / `res` may be caller-owned buffers reused across calls (C-contiguous uint8 of at least
        output_bytes, int32 of shape (>= num_streams, 2)); fresh zeroed ones are allocated otherwise."""
        if out is None:
            out = np.zeros(max(self.output_bytes, 1), dtype=np.uint8)
        if res is None:
            res = np.zeros((max(self.num_streams, 1), 2), dtype=np.int32)
        if (out.dtype != np.uint8 or not out.flags.c_contiguous or out.size < self.output_bytes
                or res.dtype != np.int32 or not res.flags.c_contiguous or res.ndim != 2 or res.shape[1] != 2
                or res.shape[0] < self.num_streams):
            raise ValueError("decode_host: out/res buffers have the wrong dtype, layout or size")
        if shard_devices is not None:
            devs = np.ascontiguousarray(shard_devices, dtype=np.int32)
            st = lib().covt_plan_decode_host_shards(self._h, _ptr(self.blob, C.c_uint8), self.blob.size, devs.size,
                                                    _ptr(devs, C.c_int32), out.ctypes.data, res.ctypes.data)
        elif n_gpus > 1:
            st = lib().covt_plan_decode_host_multi(self._h, _ptr(self.blob, C.c_uint8), self.blob.size, n_gpus,
                                                   out.ctypes.data, res.ctypes.data)
        else:
            st = lib().covt_plan_decode_host(self._h, _ptr(self.blob, C.c_uint8), self.blob.size, out.ctypes.data,
                                             res.ctypes.data)
        _raise(st, "covt_plan_decode_host")
        return out[:self.output_bytes], res[:self.num_streams]

    def assemble_host(self):
        """H2D + decode + geometry assembly + D2H (covt_plan_assemble_host).
        Returns (uint8 assembly buffer, results[num_geometry_columns] in tile order)."""
        asm = np.zeros(max(self.assembly_bytes, 1), dtype=np.uint8)
        gres = np.zeros(max(self.num_geometry_columns, 1), dtype=GEOM_RESULT_DTYPE)
        _raise(lib().covt_plan_assemble_host(self._h, _ptr(self.blob, C.c_uint8), self.blob.size, asm.ctypes.data,
                                             gres.ctypes.data), "covt_plan_assemble_host")
        return asm[:self.assembly_bytes], gres[:self.num_geometry_columns]

    def properties_host(self):
        """H2D + decode + property materialization + D2H (covt_plan_properties_host).
        Returns (uint8 property buffer, results[num_property_columns] in tile order)."""
        buf = np.zeros(max(self.property_bytes, 1), dtype=np.uint8)
        pres = np.zeros(max(self.num_property_columns, 1), dtype=PROP_RESULT_DTYPE)
        _raise(lib().covt_plan_properties_host(self._h, _ptr(self.blob, C.c_uint8), self.blob.size,
                                               buf.ctypes.data, pres.ctypes.data), "covt_plan_properties_host")
        return buf[:self.property_bytes], pres[:self.num_property_columns]

    def property_name(self, c: int) -> str:
        """Column name of property (sub)column c, plus ':<lang>' for a localized language stream."""
        p = self.props[c]
        name = bytes(self.blob[int(p["name_off"]):int(p["name_off"]) + int(p["name_len"])]).decode("utf-8") \
            if p["name_off"] >= 0 else ""
        if p["lang"] >= 0:
            name += ":" + bytes(self.blob[int(p["lang_off"]):int(p["lang_off"]) + int(p["lang_len"])]).decode("utf-8")
        return name

    def property_column(self, buf: np.ndarray, pres: np.ndarray, c: int) -> "PropertyColumn":
        """Property (sub)column c (tile order) of a property buffer (raises on its status)."""
        p, r = self.props[c], pres[c]
        _raise(int(r["status"]), "property column %d (tile %d, layer %d)" % (c, p["tile"], p["layer"]))
        n = int(p["n_features"])
        nb = (n + 7) // 8
        t = int(p["type"])

        def seg(k, nbytes):
            o = int(p["out_off"][k])
            return buf[o:o + nbytes]

        vals = {PROP_BOOLEAN: lambda: seg(1, nb), PROP_INT64: lambda: seg(1, 8 * n).view(np.int64),
                PROP_FLOAT: lambda: seg(1, 4 * n).view(np.float32), PROP_STRING: lambda: seg(1, 4 * n).view(np.int32)}[t]()
        doff = dby = None
        if t == PROP_STRING and p["out_off"][2] >= 0:
            doff = seg(2, 4 * (int(p["n_dict"]) + 1)).view(np.int32)
            dby = seg(3, int(p["dict_bytes"]))
        return PropertyColumn(self.property_name(c), t, n, seg(0, nb), vals, doff, dby, int(r["n_valid"]))

    def geometry_arrays(self, asm: np.ndarray, gres: np.ndarray, c: int):
        """Column c (tile order) of an assembly buffer -> GeoArrowGeometry (raises on its status)."""
        g, r = self.geom[c], gres[c]
        _raise(int(r["status"]), "geometry column %d (tile %d, layer %d)" % (c, g["tile"], g["layer"]))

        def seg(k, n, dt=np.int32, w=4):
            o = int(g["out_off"][k])
            return asm[o:o + n * w].view(dt)

        return GeoArrowGeometry(seg(0, int(g["n_features"]) + 1), seg(1, int(r["num_parts"]) + 1),
                                seg(2, int(r["num_rings"]) + 1), seg(3, 2 * int(r["num_coords"])).reshape(-1, 2))

    def subset_descs(self, mask):
        """Descriptor table of the streams selected by `mask` (bool per stream, plan order), in launch
        order (still grouped by family, largest first inside a family) -> (uint8 descs, family counts,
        plan-order stream index of each selected descriptor that holds a stream's result, else -1).
        Outputs keep their slices in the full output
        buffer; results land at the subset position."""
        mask = np.asarray(mask, dtype=bool)
        if mask.shape != (self.num_streams,):
            raise ValueError("subset mask must have one entry per stream")
        keep = mask[self.desc_streams]  # every descriptor of a selected stream (split chunks + pads)
        fam = np.repeat(np.arange(NUM_FAMILIES), self.family_counts)
        primary = np.full(self.num_descs, -1, dtype=np.int64)  # the descriptor holding the stream's result
        primary[self.streams["desc_index"]] = np.arange(self.num_streams)
        descs = np.ascontiguousarray(self.descs.reshape(-1, 32)[keep]).reshape(-1)
        counts = np.bincount(fam[keep], minlength=NUM_FAMILIES).astype(np.int64)
        return descs, counts, primary[keep]

    def stream_array(self, out: np.ndarray, i: int) -> np.ndarray:
        s = self.streams[i]
        dt = {1: np.uint8, 4: np.int32, 8: np.int64}[int(s["elem_bytes"])]
        off, n = int(s["out_off"]), int(s["out_elems"])
        return out[off:off + n * int(s["elem_bytes"])].view(dt)


class DeviceBatch:
    """A plan whose tile bytes, descriptors and outputs live in HBM (torch uint8 tensors on `device`).
    ``decode()`` enqueues the single decode launch on the current torch HIP stream."""

    def __init__(self, plan: Plan, device="cuda"):
        import torch

        self.plan = plan
        self.device = torch.device(device)
        self.d_in = torch.from_numpy(plan.blob).to(self.device)
        if self.d_in.data_ptr() % 16:
            raise DeviceError("device input buffer is not 16-byte aligned")
        n = max(plan.num_descs, 1)  # one result entry per descriptor (split pads hold look-back records)
        self.d_desc = torch.from_numpy(plan.descs).to(self.device) if plan.num_descs else \
            torch.zeros(32, dtype=torch.uint8, device=self.device)
        self.d_out = torch.zeros(max(plan.output_bytes, 16), dtype=torch.uint8, device=self.device)
        self.d_res = torch.zeros(n * 2, dtype=torch.int32, device=self.device)

    def decode_graph(self):
        """The same launch replayed from a captured HIP graph on the current torch stream: the fork,
        the four family kernels on their forked streams and the join become one graph launch, so
        back-to-back decodes pay one submission instead of eleven stream operations."""
        import torch

        g = getattr(self, "_graph", None)
        if g is None:
            side = torch.cuda.Stream(self.device)
            side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(side):  # the fork streams and events exist before the capture
                self.decode(side)
            torch.cuda.current_stream(self.device).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self.decode(torch.cuda.current_stream(self.device))
            self._graph = g
        g.replay()

    def decode(self, stream=None, launch: int = 0):
        """launch: LAUNCH_AUTO (0), LAUNCH_FUSED or LAUNCH_FORKED, optionally | LAUNCH_FPF_STREAM or LAUNCH_FPF_CLASSIC
        (covt_decode_streams_device_grouped_mode)."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        st = lib().covt_decode_streams_device_grouped_mode(self.d_in.data_ptr(), self.d_desc.data_ptr(),
                                                           _ptr(self.plan.family_counts, C.c_int64),
                                                           self.d_out.data_ptr(), self.d_res.data_ptr(), s.cuda_stream,
                                                           launch)
        _raise(st, "covt_decode_streams_device_grouped_mode")

    def subset(self, mask) -> "DeviceSubset":
        """A launch over only the streams selected by `mask` (Plan.subset_descs), sharing this batch's
        device input and output buffers."""
        return DeviceSubset(self, mask)


    def _asm_buffers(self):
        import torch

        if getattr(self, "d_asm", None) is None:
            p = self.plan
            self.d_gdesc = torch.from_numpy(p.gdescs).to(self.device) if p.num_geometry_columns else \
                torch.zeros(C.sizeof(GeomDesc), dtype=torch.uint8, device=self.device)
            self.d_asm = torch.empty(max(p.assembly_bytes, 16), dtype=torch.uint8, device=self.device)
            self.d_gres = torch.zeros(max(p.num_geometry_columns, 1) * 4, dtype=torch.int32, device=self.device)

    def assemble(self, stream=None):
        """Enqueue the geometry assembly (after decode() on the same stream)."""
        import torch

        self._asm_buffers()
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _raise(lib().covt_assemble_geometry_device(self.d_out.data_ptr(), self.d_res.data_ptr(),
                                                   self.d_gdesc.data_ptr(), self.plan.num_geometry_columns,
                                                   self.d_asm.data_ptr(), self.d_gres.data_ptr(), s.cuda_stream),
               "covt_assemble_geometry_device")

    def _prop_buffers(self):
        import torch

        if getattr(self, "d_props", None) is None:
            p = self.plan
            self.d_pdesc = torch.from_numpy(p.pdescs.view(np.uint8).reshape(-1)).to(self.device) \
                if p.num_property_columns else torch.zeros(PROP_DESC_DTYPE.itemsize, dtype=torch.uint8, device=self.device)
            self.d_props = torch.zeros(max(p.property_bytes, 16), dtype=torch.uint8, device=self.device)
            self.d_pres = torch.zeros(max(p.num_property_columns, 1) * 2, dtype=torch.int32, device=self.device)

    def materialize_properties(self, stream=None):
        """Enqueue the property-column materialization (after decode() on the same stream)."""
        import torch

        self._prop_buffers()
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _raise(lib().covt_materialize_properties_device(self.d_in.data_ptr(), self.d_out.data_ptr(),
                                                        self.d_res.data_ptr(), self.d_pdesc.data_ptr(),
                                                        self.plan.num_property_columns, self.d_props.data_ptr(),
                                                        self.d_pres.data_ptr(), s.cuda_stream),
               "covt_materialize_properties_device")

    def property_results(self):
        """(property bytes, results in tile order) copied to the host."""
        self._prop_buffers()
        buf = self.d_props.cpu().numpy()[:self.plan.property_bytes]
        r = self.d_pres.cpu().numpy().view(PROP_RESULT_DTYPE)[:self.plan.num_property_columns]
        return buf, r[self.plan.props["desc_index"]] if self.plan.num_property_columns else r

    def assembly_results(self):
        """(assembly bytes, geometry results in tile order) copied to the host."""
        self._asm_buffers()
        asm = self.d_asm.cpu().numpy()[:self.plan.assembly_bytes]
        g = self.d_gres.cpu().numpy().view(GEOM_RESULT_DTYPE)[:self.plan.num_geometry_columns]
        return asm, g[self.plan.geom["desc_index"]] if self.plan.num_geometry_columns else g

    def results(self):
        """(output bytes, results in plan order) copied to the host."""
        out = self.d_out.cpu().numpy()[:self.plan.output_bytes]
        res_launch = self.d_res.cpu().numpy().reshape(-1, 2)[:self.plan.num_descs]
        res = res_launch[self.plan.streams["desc_index"]] if self.plan.num_streams else res_launch
        return out, res


class DevicePlan:
    """covt_device_plan_create: the Id / Geometry plan built on the GPU from tiles already in HBM.

    `d_blob` is a uint8 torch tensor on the device holding the tiles, `offsets` / `sizes` the tiles'
    byte ranges in it (host arrays or device tensors).  The walk, prefix sums, launch-order sort and
    descriptor fill run on the current torch stream; the result has the host plan's layout exactly
    (Plan.streams / Plan.descs / Plan.family_counts with the same options, split chunks included)."""

    def __init__(self, d_blob, offsets, sizes, fmt: int = FORMAT_GENC, id_mode: int = ID_FORMAT, stream=None,
                 options: Optional[PlanOptions] = None):
        import torch

        self.device = d_blob.device
        if d_blob.dtype != torch.uint8 or not d_blob.is_contiguous() or d_blob.device.type != "cuda":
            raise IllegalArgumentException("d_blob must be a contiguous uint8 device tensor")
        self.d_in = d_blob
        as_dev = lambda a: torch.as_tensor(np.asarray(a, dtype=np.int64) if not torch.is_tensor(a) else a,
                                           dtype=torch.int64).to(self.device).contiguous()
        self.d_off, self.d_size = as_dev(offsets), as_dev(sizes)
        if self.d_off.numel() != self.d_size.numel():
            raise IllegalArgumentException("offsets and sizes differ in length")
        self.n_tiles = int(self.d_off.numel())
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            _raise(lib().covt_device_plan_create_opts(d_blob.data_ptr(), d_blob.numel(), self.d_off.data_ptr(),
                                                      self.d_size.data_ptr(), self.n_tiles, fmt, id_mode,
                                                      C.byref(options) if options is not None else None,
                                                      s.cuda_stream, C.byref(h)), "covt_device_plan_create")
        self._h = h
        L = lib()
        self.num_streams = L.covt_device_plan_num_streams(h)
        self.num_descs = L.covt_device_plan_num_descs(h)
        self.output_bytes = L.covt_device_plan_output_bytes(h)
        self.family_counts = np.zeros(NUM_FAMILIES, dtype=np.int64)
        L.covt_device_plan_family_counts(h, _ptr(self.family_counts, C.c_int64))
        a, b, c = C.c_int64(), C.c_int64(), C.c_int64()
        L.covt_device_plan_totals(h, C.byref(a), C.byref(b), C.byref(c))
        self.in_bytes, self.out_payload, self.vertices = a.value, b.value, c.value
        self.num_property_columns = L.covt_device_plan_num_property_columns(h)
        self.property_bytes = L.covt_device_plan_property_bytes(h)

    def close(self):
        if getattr(self, "_h", None):
            lib().covt_device_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def host_copy(self):
        """(stream records in tile order, descriptors in launch order, tile statuses) as host arrays."""
        info = np.zeros(self.num_streams, dtype=STREAM_INFO_DTYPE)
        descs = np.zeros(self.num_descs * 32, dtype=np.uint8)
        st = np.zeros(max(self.n_tiles, 1), dtype=np.int32)
        _raise(lib().covt_device_plan_copy(self._h, info.ctypes.data, descs.ctypes.data, _ptr(st, C.c_int32)),
               "covt_device_plan_copy")
        return info, descs, st[:self.n_tiles]

    def property_copy(self):
        """(property records in tile order, property descriptors in materialization order) as host arrays
        (plans made with PLAN_PROPERTIES in the options' flags; Plan.props / Plan.pdescs of the host plan)."""
        n = self.num_property_columns
        pinfo = np.zeros(n, dtype=PROP_INFO_DTYPE)
        pdesc = np.zeros(n, dtype=PROP_DESC_DTYPE)
        _raise(lib().covt_device_plan_property_copy(self._h, pinfo.ctypes.data, pdesc.ctypes.data),
               "covt_device_plan_property_copy")
        return pinfo, pdesc

    def alloc_properties(self):
        """(property buffer, property results) on the device, sized for this plan's property columns."""
        import torch

        return (torch.zeros(max(self.property_bytes, 16), dtype=torch.uint8, device=self.device),
                torch.zeros(max(self.num_property_columns, 1) * 2, dtype=torch.int32, device=self.device))

    def materialize(self, d_out, d_res, d_props, d_pres, stream=None):
        """Enqueue the property materialization over this plan's property descriptors (after decode())."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _raise(lib().covt_device_plan_materialize(self._h, self.d_in.data_ptr(), d_out.data_ptr(), d_res.data_ptr(),
                                                  d_props.data_ptr(), d_pres.data_ptr(), s.cuda_stream),
               "covt_device_plan_materialize")

    def alloc(self):
        """(output buffer, result buffer) on the device, sized for this plan."""
        import torch

        return (torch.zeros(max(self.output_bytes, 16), dtype=torch.uint8, device=self.device),
                torch.zeros(max(self.num_descs, 1) * 2, dtype=torch.int32, device=self.device))

    def decode(self, d_out, d_res, stream=None):
        """Enqueue the grouped decode launch over this plan's descriptors."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _raise(lib().covt_device_plan_decode(self._h, self.d_in.data_ptr(), d_out.data_ptr(), d_res.data_ptr(),
                                             s.cuda_stream), "covt_device_plan_decode")

    def geometry(self, stream=None):
        """Build the geometry-column records and descriptors on the device (once; synchronises the
        stream): Plan.geom / Plan.gdescs / Plan.assembly_bytes without the host plan."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        with torch.cuda.device(self.device):
            _raise(lib().covt_device_plan_geometry(self._h, s.cuda_stream), "covt_device_plan_geometry")
        self.num_geometry_columns = lib().covt_device_plan_num_geometry_columns(self._h)
        self.assembly_bytes = lib().covt_device_plan_assembly_bytes(self._h)
        return self.num_geometry_columns

    def geometry_copy(self):
        """(geometry records in tile order, geometry descriptors in launch order) as host arrays."""
        self.geometry()
        g = np.zeros(self.num_geometry_columns, dtype=GEOM_INFO_DTYPE)
        d = np.zeros(self.num_geometry_columns * C.sizeof(GeomDesc), dtype=np.uint8)
        _raise(lib().covt_device_plan_geometry_copy(self._h, g.ctypes.data, d.ctypes.data),
               "covt_device_plan_geometry_copy")
        return g, d

    def alloc_assembly(self):
        """(assembly buffer, geometry results) on the device, sized for this plan's geometry columns."""
        import torch

        self.geometry()
        return (torch.empty(max(self.assembly_bytes, 16), dtype=torch.uint8, device=self.device),
                torch.zeros(max(self.num_geometry_columns, 1) * 4, dtype=torch.int32, device=self.device))

    def assemble(self, d_out, d_res, d_asm, d_gres, stream=None):
        """Enqueue the geometry assembly over this plan's geometry descriptors (after decode())."""
        import torch

        self.geometry(stream)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _raise(lib().covt_device_plan_assemble(self._h, d_out.data_ptr(), d_res.data_ptr(), d_asm.data_ptr(),
                                               d_gres.data_ptr(), s.cuda_stream), "covt_device_plan_assemble")


class DeviceSubset:
    """One decode launch over a subset of a DeviceBatch's streams (e.g. BASELINE configs 2-4, which are
    stream selections of fixture tiles); its own descriptor table and result array on the device."""

    def __init__(self, batch: DeviceBatch, mask):
        import torch

        self.batch = batch
        descs, self.family_counts, self.stream_index = batch.plan.subset_descs(mask)
        self.num_descs = int(self.stream_index.size)
        self.num_streams = int((self.stream_index >= 0).sum())
        self.d_desc = torch.from_numpy(descs).to(batch.device) if self.num_descs else \
            torch.zeros(32, dtype=torch.uint8, device=batch.device)
        self.d_res = torch.zeros(max(self.num_descs, 1) * 2, dtype=torch.int32, device=batch.device)

    def decode(self, stream=None):
        import torch

        b = self.batch
        s = stream if stream is not None else torch.cuda.current_stream(b.device)
        _raise(lib().covt_decode_streams_device_grouped(b.d_in.data_ptr(), self.d_desc.data_ptr(),
                                                        _ptr(self.family_counts, C.c_int64), b.d_out.data_ptr(),
                                                        self.d_res.data_ptr(), s.cuda_stream),
               "covt_decode_streams_device_grouped")

    def decode_graph(self):
        """This subset's launch replayed from a captured HIP graph on the current torch stream (as
        DeviceBatch.decode_graph): the split-record memset, the fork, every family and chunk kernel on
        its queue and the join become one graph launch."""
        import torch

        g = getattr(self, "_graph", None)
        if g is None:
            dev = self.batch.device
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):  # the fork streams and events exist before the capture
                self.decode(side)
            torch.cuda.current_stream(dev).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self.decode(torch.cuda.current_stream(dev))
            self._graph = g
        g.replay()

    def results(self):
        """(full output bytes, results[k, 2] of the subset's k streams, their plan-order indices)."""
        out = self.batch.d_out.cpu().numpy()[:self.batch.plan.output_bytes]
        res = self.d_res.cpu().numpy().reshape(-1, 2)[:self.num_descs]
        prim = self.stream_index >= 0
        return out, res[prim], self.stream_index[prim]


# ---------------------------------------------------------------------------
# CovtParser mirror (Id + Geometry columns)
# ---------------------------------------------------------------------------
@dataclass
class GeometryColumn:
    """record GeometryColumn, CovtParser.java:29-36 (absent streams are None)."""
    geometryTypes: Optional[np.ndarray] = None
    geometryOffsets: Optional[np.ndarray] = None
    partOffsets: Optional[np.ndarray] = None
    ringOffsets: Optional[np.ndarray] = None
    vertexOffsets: Optional[np.ndarray] = None
    vertexBuffer: Optional[np.ndarray] = None


@dataclass
class GeoArrowGeometry:
    """One assembled geometry column (include/covt.h "Geometry assembly"): nested offsets
    feature -> parts -> rings -> coordinates, coords int32 [k, 2]; polygon rings closed."""
    geometry_offsets: np.ndarray
    part_offsets: np.ndarray
    ring_offsets: np.ndarray
    coords: np.ndarray

    def feature(self, i: int):
        """Parts of feature i as lists of rings, each an int32 [m, 2] array."""
        g, p, r = self.geometry_offsets, self.part_offsets, self.ring_offsets
        return [[self.coords[r[k]:r[k + 1]] for k in range(p[j], p[j + 1])] for j in range(g[i], g[i + 1])]


@dataclass
class PropertyColumn:
    """One materialized property (sub)column (include/covt.h "Property columns"): Arrow-style validity
    bitmap (LSB first) + values at feature positions (BOOLEAN: bitmap; INT64: int64; FLOAT: float32;
    STRING: int32 dictionary index) + dictionary offsets / UTF-8 bytes."""
    name: str
    type: int
    n_features: int
    validity: np.ndarray
    values: np.ndarray
    dict_offsets: Optional[np.ndarray]
    dict_bytes: Optional[np.ndarray]
    n_valid: int

    def valid(self, i: int) -> bool:
        return bool((int(self.validity[i >> 3]) >> (i & 7)) & 1)

    def value(self, i: int):
        """CovtParser's Optional for feature i: None (empty) or the value."""
        if not self.valid(i):
            return None
        if self.type == PROP_BOOLEAN:
            return bool((int(self.values[i >> 3]) >> (i & 7)) & 1)
        if self.type == PROP_INT64:
            return int(self.values[i])
        if self.type == PROP_FLOAT:
            return float(self.values[i])
        k = int(self.values[i])
        return bytes(self.dict_bytes[self.dict_offsets[k]:self.dict_offsets[k + 1]]).decode("utf-8")

    def to_list(self):
        """The List<Optional> of decodePropertyColumn (CovtParser.java:276-354)."""
        return [self.value(i) for i in range(self.n_features)]


@dataclass
class LayerColumns:
    layer: int
    ids: Optional[np.ndarray]
    geometry: GeometryColumn
    num_bits: int = 0
    column_type: int = 0
    properties: Optional[dict] = None


_GEOM_FIELD = {GEOMETRY_TYPES: "geometryTypes", GEOMETRY_OFFSETS: "geometryOffsets", PART_OFFSETS: "partOffsets",
               RING_OFFSETS: "ringOffsets", VERTEX_OFFSETS: "vertexOffsets", VERTEX_BUFFER: "vertexBuffer"}


def split_layers(plan: Plan, out: np.ndarray, res: np.ndarray, tile: int = 0) -> List[LayerColumns]:
    layers = {}
    for i in np.nonzero(plan.streams["tile"] == tile)[0]:
        s = plan.streams[i]
        _raise(int(res[i][0]), "stream %d (layer %d, type %d)" % (i, s["layer"], s["stream_type"]))
        if int(s["column_kind"]) == 2:  # property streams: see Plan.property_column
            continue
        lc = layers.setdefault(int(s["layer"]), LayerColumns(int(s["layer"]), None, GeometryColumn()))
        arr = plan.stream_array(out, int(i))
        if int(s["column_kind"]) == 0:
            lc.ids = arr
        else:
            setattr(lc.geometry, _GEOM_FIELD[int(s["stream_type"])], arr)
            lc.num_bits = int(s["num_bits"])
            lc.column_type = int(s["column_type"])
    return [layers[k] for k in sorted(layers)]


class CovtParser:
    @staticmethod
    def decode_covt(covt_buffer: bytes, fmt: int = FORMAT_GENC, id_mode: int = ID_FORMAT,
                    properties: bool = False) -> List[LayerColumns]:
        """CovtParser.decodeCovt (CovtParser.java:53-133) decoded on the GPU: Id + Geometry columns, and with
        ``properties`` every property column as a PropertyColumn (LayerColumns.properties, by name)."""
        plan = Plan.from_tiles([covt_buffer], fmt, id_mode, PLAN_PROPERTIES if properties else 0)
        _raise(int(plan.tile_status[0]), "decodeLayerMetadata")
        out, res = plan.decode_host()
        layers = split_layers(plan, out, res, 0)
        if properties and plan.num_property_columns:
            buf, pres = plan.properties_host()
            by_layer = {lc.layer: lc for lc in layers}
            for c in range(plan.num_property_columns):
                L = int(plan.props["layer"][c])
                lc = by_layer.setdefault(L, LayerColumns(L, None, GeometryColumn()))
                if lc.properties is None:
                    lc.properties = {}
                col = plan.property_column(buf, pres, c)
                lc.properties[col.name] = col
            layers = [by_layer[k] for k in sorted(by_layer)]
        return layers


def version() -> str:
    return lib().covt_version().decode()


# the files whose sha256 (in this order) the Makefile compiles into covt_version() as "src:<16 hex>"
_BUILD_SOURCES = ("csrc/covt_decode.hip", "csrc/covt_assemble.hip", "csrc/covt_props.hip", "csrc/covt_plan_device.hip",
                  "csrc/covt_host.cpp", "../include/covt.h", "csrc/covt_internal.h", "csrc/covt_wave.h",
                  "csrc/covt_walk.h", "csrc/covt_props_plan.h", "csrc/covt_scratch.h")


def source_build_id() -> str:
    """sha256 prefix of the library sources as they are in this tree (the Makefile's BUILD_ID)."""
    import hashlib

    h = hashlib.sha256()
    for f in _BUILD_SOURCES:
        with open(os.path.join(_HERE, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def library_build_id() -> str:
    """The build id compiled into the loaded libcovt.so (covt_version)."""
    v = version()
    return v.rsplit("src:", 1)[1] if "src:" in v else "unknown"
