"""Host-side mirror of TileDB's filter / filter-pipeline interface.

Names, option meanings and the serialized byte layout follow the reference:
  Filter::serialize                tiledb/sm/filter/filter.cc:96-112
  FilterPipeline::serialize        tiledb/sm/filter/filter_pipeline.cc:524-542
  FilterPipeline::deserialize      tiledb/sm/filter/filter_pipeline.cc:544-557
  FilterCreate::deserialize        tiledb/sm/filter/filter_create.cc:100-201
  CompressionFilter::output_datatype compression_filter.cc:729-738
  enums                            tiledb/api/c_api/filter/filter_api_enum.h,
                                   tiledb/sm/enums/compressor.h,
                                   tiledb/api/c_api/datatype/datatype_api_enum.h
The reverse direction (run_reverse) executes on the MI355X through the C-ABI
(include/tiledb_amd.h); this module only builds descriptors and moves
pointers.  There is no CPU execution path here.
"""
from __future__ import annotations

import struct
from enum import IntEnum
from typing import Iterable, List, Optional, Sequence

FORMAT_VERSION = 23  # tiledb/sm/misc/constants.cc:693
MAX_TILE_CHUNK_SIZE = 64 * 1024  # constants::max_tile_chunk_size (constants.cc:730)


class FilterType(IntEnum):
    FILTER_NONE = 0
    FILTER_GZIP = 1
    FILTER_ZSTD = 2
    FILTER_LZ4 = 3
    FILTER_RLE = 4
    FILTER_BZIP2 = 5
    FILTER_DOUBLE_DELTA = 6
    FILTER_BIT_WIDTH_REDUCTION = 7
    FILTER_BITSHUFFLE = 8
    FILTER_BYTESHUFFLE = 9
    FILTER_POSITIVE_DELTA = 10
    INTERNAL_FILTER_AES_256_GCM = 11
    FILTER_CHECKSUM_MD5 = 12
    FILTER_CHECKSUM_SHA256 = 13
    FILTER_DICTIONARY = 14
    FILTER_SCALE_FLOAT = 15
    FILTER_XOR = 16
    FILTER_DEPRECATED = 17
    FILTER_WEBP = 18
    FILTER_DELTA = 19


class Compressor(IntEnum):
    NO_COMPRESSION = 0
    GZIP = 1
    ZSTD = 2
    LZ4 = 3
    RLE = 4
    BZIP2 = 5
    DOUBLE_DELTA = 6
    DICTIONARY_ENCODING = 7
    DELTA = 8


class FilterOption(IntEnum):
    COMPRESSION_LEVEL = 0
    BIT_WIDTH_MAX_WINDOW = 1
    POSITIVE_DELTA_MAX_WINDOW = 2
    SCALE_FLOAT_BYTEWIDTH = 3
    SCALE_FLOAT_FACTOR = 4
    SCALE_FLOAT_OFFSET = 5
    WEBP_QUALITY = 6
    WEBP_INPUT_FORMAT = 7
    WEBP_LOSSLESS = 8
    COMPRESSION_REINTERPRET_DATATYPE = 9


class Datatype(IntEnum):
    INT32 = 0
    INT64 = 1
    FLOAT32 = 2
    FLOAT64 = 3
    CHAR = 4
    INT8 = 5
    UINT8 = 6
    INT16 = 7
    UINT16 = 8
    UINT32 = 9
    UINT64 = 10
    STRING_ASCII = 11
    STRING_UTF8 = 12
    STRING_UTF16 = 13
    STRING_UTF32 = 14
    STRING_UCS2 = 15
    STRING_UCS4 = 16
    ANY = 17
    DATETIME_YEAR = 18
    DATETIME_MONTH = 19
    DATETIME_WEEK = 20
    DATETIME_DAY = 21
    DATETIME_HR = 22
    DATETIME_MIN = 23
    DATETIME_SEC = 24
    DATETIME_MS = 25
    DATETIME_US = 26
    DATETIME_NS = 27
    DATETIME_PS = 28
    DATETIME_FS = 29
    DATETIME_AS = 30
    TIME_HR = 31
    TIME_MIN = 32
    TIME_SEC = 33
    TIME_MS = 34
    TIME_US = 35
    TIME_NS = 36
    TIME_PS = 37
    TIME_FS = 38
    TIME_AS = 39
    BLOB = 40
    BOOL = 41
    GEOM_WKB = 42
    GEOM_WKT = 43


def datatype_size(dt: int) -> int:
    """datatype_size (tiledb/sm/enums/datatype.h:67-140)."""
    dt = Datatype(dt)
    if dt in (Datatype.INT32, Datatype.FLOAT32, Datatype.UINT32, Datatype.STRING_UTF32,
              Datatype.STRING_UCS4):
        return 4
    if dt in (Datatype.INT64, Datatype.FLOAT64, Datatype.UINT64):
        return 8
    if dt in (Datatype.INT16, Datatype.UINT16, Datatype.STRING_UTF16, Datatype.STRING_UCS2):
        return 2
    if Datatype.DATETIME_YEAR <= dt <= Datatype.TIME_AS:
        return 8
    return 1


def datatype_is_real(dt: int) -> bool:
    return dt in (Datatype.FLOAT32, Datatype.FLOAT64)


def datatype_is_integer(dt: int) -> bool:
    return dt in (Datatype.BOOL, Datatype.INT8, Datatype.UINT8, Datatype.INT16, Datatype.UINT16,
                  Datatype.INT32, Datatype.UINT32, Datatype.INT64, Datatype.UINT64)


def datatype_is_datetime_or_time(dt: int) -> bool:
    return Datatype.DATETIME_YEAR <= dt <= Datatype.TIME_AS


def datatype_is_byte(dt: int) -> bool:
    return dt in (Datatype.BLOB, Datatype.GEOM_WKB, Datatype.GEOM_WKT)


class FilterStatusException(Exception):
    """Mirror of FilterStatusException (tiledb/sm/filter/filter.h:71-76)."""


_COMPRESSOR_TO_FILTER = {
    Compressor.NO_COMPRESSION: FilterType.FILTER_NONE,
    Compressor.GZIP: FilterType.FILTER_GZIP,
    Compressor.ZSTD: FilterType.FILTER_ZSTD,
    Compressor.LZ4: FilterType.FILTER_LZ4,
    Compressor.RLE: FilterType.FILTER_RLE,
    Compressor.BZIP2: FilterType.FILTER_BZIP2,
    Compressor.DOUBLE_DELTA: FilterType.FILTER_DOUBLE_DELTA,
    Compressor.DICTIONARY_ENCODING: FilterType.FILTER_DICTIONARY,
    Compressor.DELTA: FilterType.FILTER_DELTA,
}
_FILTER_TO_COMPRESSOR = {v: k for k, v in _COMPRESSOR_TO_FILTER.items()}


class Filter:
    """Base filter: type code + filter datatype (filter.h:85-267)."""

    type: FilterType = FilterType.FILTER_NONE

    def __init__(self, filter_data_type: int = Datatype.ANY):
        self.filter_data_type = Datatype(filter_data_type)

    def serialize_impl(self) -> bytes:
        return b""

    def serialize(self) -> bytes:
        impl = self.serialize_impl()
        return struct.pack("<BI", int(self.type), len(impl)) + impl

    def output_datatype(self, input_type: int) -> Datatype:
        return Datatype(input_type)

    def accepts_input_datatype(self, datatype: int) -> bool:
        return True

    def clone(self, data_type: Optional[int] = None) -> "Filter":
        import copy
        c = copy.copy(self)
        if data_type is not None:
            c.filter_data_type = Datatype(data_type)
        return c

    def __repr__(self) -> str:
        return f"{type(self).__name__}()"


class NoopFilter(Filter):
    type = FilterType.FILTER_NONE


class ByteshuffleFilter(Filter):
    type = FilterType.FILTER_BYTESHUFFLE


class BitshuffleFilter(Filter):
    type = FilterType.FILTER_BITSHUFFLE


class BitWidthReductionFilter(Filter):
    """bit_width_reduction_filter.cc; default window 256 B (:85-88)."""

    type = FilterType.FILTER_BIT_WIDTH_REDUCTION

    def __init__(self, max_window_size: int = 256, filter_data_type: int = Datatype.ANY):
        super().__init__(filter_data_type)
        self.max_window_size = int(max_window_size)

    def serialize_impl(self) -> bytes:
        return struct.pack("<I", self.max_window_size)

    def accepts_input_datatype(self, datatype: int) -> bool:  # :102-108
        return (datatype_is_integer(datatype) or datatype_is_datetime_or_time(datatype)
                or datatype_is_byte(datatype))

    def __repr__(self) -> str:
        return f"BitWidthReduction: BIT_WIDTH_MAX_WINDOW={self.max_window_size}"


class PositiveDeltaFilter(Filter):
    """positive_delta_filter.cc; default window 1024 B (:46-49)."""

    type = FilterType.FILTER_POSITIVE_DELTA

    def __init__(self, max_window_size: int = 1024, filter_data_type: int = Datatype.ANY):
        super().__init__(filter_data_type)
        self.max_window_size = int(max_window_size)

    def serialize_impl(self) -> bytes:
        return struct.pack("<I", self.max_window_size)

    def accepts_input_datatype(self, datatype: int) -> bool:
        return (datatype_is_integer(datatype) or datatype_is_datetime_or_time(datatype)
                or datatype_is_byte(datatype))

    def __repr__(self) -> str:
        return f"PositiveDelta: POSITIVE_DELTA_MAX_WINDOW={self.max_window_size}"


class XORFilter(Filter):
    """xor_filter.cc: prefix XOR of the input's integer width, any 1/2/4/8-byte
    type (:51-61); output type = the signed integer of that width (:63-78)."""

    type = FilterType.FILTER_XOR

    def accepts_input_datatype(self, datatype: int) -> bool:
        return datatype_size(datatype) in (1, 2, 4, 8)

    def output_datatype(self, input_type: int) -> Datatype:
        w = datatype_size(input_type)
        m = {1: Datatype.INT8, 2: Datatype.INT16, 4: Datatype.INT32, 8: Datatype.INT64}
        if w not in m:
            raise FilterStatusException(
                "XORFilter::output_datatype: datatype size cannot be converted to integer type.")
        return m[w]


class FloatScalingFilter(Filter):
    """float_scaling_filter.cc: FilterConfig {double scale, double offset,
    u64 byte_width} (.h:61-65); accepts 4/8-byte inputs (:306-310); output =
    the signed integer of byte_width (:313-327)."""

    type = FilterType.FILTER_SCALE_FLOAT

    def __init__(self, scale: float = 1.0, offset: float = 0.0, byte_width: int = 8,
                 filter_data_type: int = Datatype.ANY):
        super().__init__(filter_data_type)
        self.scale, self.offset, self.byte_width = float(scale), float(offset), int(byte_width)

    def serialize_impl(self) -> bytes:
        return struct.pack("<ddQ", self.scale, self.offset, self.byte_width)

    def accepts_input_datatype(self, datatype: int) -> bool:
        return datatype_size(datatype) in (4, 8)

    def output_datatype(self, input_type: int) -> Datatype:
        m = {1: Datatype.INT8, 2: Datatype.INT16, 4: Datatype.INT32, 8: Datatype.INT64}
        if self.byte_width not in m:
            raise FilterStatusException(
                "FloatScalingFilter::output_datatype: byte_width_ does not reflect the size of "
                "an integer type.")
        return m[self.byte_width]

    def __repr__(self) -> str:
        return (f"ScaleFloat: SCALE_FLOAT_BYTEWIDTH={self.byte_width}, "
                f"SCALE_FLOAT_FACTOR={self.scale}, SCALE_FLOAT_OFFSET={self.offset}")


class CompressionFilter(Filter):
    """compression_filter.cc.  The filter type follows the compressor."""

    def __init__(self, compressor: int, level: int = -1,
                 filter_data_type: int = Datatype.ANY,
                 reinterpret_datatype: int = Datatype.ANY,
                 version: int = FORMAT_VERSION):
        super().__init__(filter_data_type)
        if isinstance(compressor, FilterType):  # tiledb_filter_alloc(FILTER_*) style
            compressor = _FILTER_TO_COMPRESSOR[compressor]
        self.compressor = Compressor(int(compressor))
        self.level = int(level)
        self.reinterpret_datatype = Datatype(reinterpret_datatype)
        self.version = version
        self.type = _COMPRESSOR_TO_FILTER[self.compressor]

    def serialize_impl(self) -> bytes:
        if self.compressor == Compressor.NO_COMPRESSION:
            return b""
        b = struct.pack("<Bi", int(self.compressor), self.level)
        if self.compressor in (Compressor.DELTA, Compressor.DOUBLE_DELTA):
            b += struct.pack("<B", int(self.reinterpret_datatype))
        return b

    def output_datatype(self, input_type: int) -> Datatype:  # :729-738
        if self.compressor in (Compressor.DOUBLE_DELTA, Compressor.DELTA):
            return Datatype(input_type) if self.reinterpret_datatype == Datatype.ANY else \
                self.reinterpret_datatype
        return Datatype(input_type)

    def accepts_input_datatype(self, input_type: int) -> bool:  # :98-115
        if self.compressor in (Compressor.DOUBLE_DELTA, Compressor.DELTA):
            t = self.reinterpret_datatype if self.reinterpret_datatype != Datatype.ANY else input_type
            if datatype_is_real(t):
                return False
            if (self.reinterpret_datatype != Datatype.ANY and
                    datatype_size(input_type) % datatype_size(self.reinterpret_datatype) != 0):
                return False
        return True

    def __repr__(self) -> str:
        return f"{self.compressor.name}: COMPRESSION_LEVEL={self.level}"


class FilterPipeline:
    """Ordered filters + max chunk size (filter_pipeline.h)."""

    def __init__(self, max_chunk_size: int = MAX_TILE_CHUNK_SIZE,
                 filters: Iterable[Filter] = ()):
        self.max_chunk_size = int(max_chunk_size)
        self.filters: List[Filter] = [f.clone() for f in filters]

    def add_filter(self, f: Filter) -> None:
        self.filters.append(f.clone())

    def size(self) -> int:
        return len(self.filters)

    def empty(self) -> bool:
        return not self.filters

    def get_filter(self, i: int) -> Optional[Filter]:
        return self.filters[i] if 0 <= i < len(self.filters) else None

    def has_filter(self, t: int) -> bool:
        return any(f.type == t for f in self.filters)

    def with_datatype(self, on_disk_type: int) -> "FilterPipeline":
        """FilterPipeline(other, on_disk_type): chain filter datatypes (:80-88)."""
        out = FilterPipeline(self.max_chunk_size)
        cur = Datatype(on_disk_type)
        for f in self.filters:
            out.filters.append(f.clone(cur))
            cur = out.filters[-1].output_datatype(cur)
        return out

    def check_filter_types(self, first_input_type: int) -> None:
        """FilterPipeline::check_filter_types (:116-149), modern checks only."""
        if not self.filters:
            return
        t = Datatype(first_input_type)
        for f in self.filters:
            if f.type != FilterType.FILTER_NONE and not f.accepts_input_datatype(t):
                raise FilterStatusException(
                    f"Filter {f.type.name} does not accept input type {t.name}")
            t = f.output_datatype(t)

    def serialize(self) -> bytes:
        b = struct.pack("<II", self.max_chunk_size, len(self.filters))
        for f in self.filters:
            if isinstance(f, CompressionFilter) and f.type == FilterType.FILTER_NONE:
                b += NoopFilter().serialize()
            else:
                b += f.serialize()
        return b

    @classmethod
    def deserialize(cls, data: bytes, version: int = FORMAT_VERSION,
                    datatype: int = Datatype.ANY) -> "FilterPipeline":
        if len(data) < 8:
            raise FilterStatusException("Deserialization error; buffer too small")
        max_chunk, nf = struct.unpack_from("<II", data, 0)
        o = 8
        p = cls(max_chunk)
        dt = Datatype(datatype)
        for _ in range(nf):
            if o + 5 > len(data):
                raise FilterStatusException("Deserialization error; truncated filter")
            ftype, mdlen = struct.unpack_from("<BI", data, o)
            o += 5
            if len(data) - o < mdlen:
                raise FilterStatusException(
                    "Deserialization error; not enough data in buffer for metadata")
            ftype = FilterType(ftype)
            if ftype == FilterType.FILTER_NONE:
                f: Filter = NoopFilter(dt)
            elif ftype in (FilterType.FILTER_GZIP, FilterType.FILTER_ZSTD, FilterType.FILTER_LZ4,
                           FilterType.FILTER_RLE, FilterType.FILTER_BZIP2, FilterType.FILTER_DELTA,
                           FilterType.FILTER_DOUBLE_DELTA, FilterType.FILTER_DICTIONARY):
                comp, level = struct.unpack_from("<Bi", data, o)
                o += 5
                reinterp = Datatype.ANY
                if ((version >= 20 and ftype == FilterType.FILTER_DOUBLE_DELTA) or
                        (version >= 19 and ftype == FilterType.FILTER_DELTA)):
                    reinterp = Datatype(data[o])
                    o += 1
                f = CompressionFilter(Compressor(comp), level, dt, reinterp, version)
            elif ftype == FilterType.FILTER_BIT_WIDTH_REDUCTION:
                (w,) = struct.unpack_from("<I", data, o)
                o += 4
                f = BitWidthReductionFilter(w, dt)
            elif ftype == FilterType.FILTER_POSITIVE_DELTA:
                (w,) = struct.unpack_from("<I", data, o)
                o += 4
                f = PositiveDeltaFilter(w, dt)
            elif ftype == FilterType.FILTER_BITSHUFFLE:
                f = BitshuffleFilter(dt)
            elif ftype == FilterType.FILTER_BYTESHUFFLE:
                f = ByteshuffleFilter(dt)
            elif ftype == FilterType.FILTER_XOR:
                f = XORFilter(dt)
            elif ftype == FilterType.FILTER_SCALE_FLOAT:
                sc, of, bw = struct.unpack_from("<ddQ", data, o)
                o += 24
                f = FloatScalingFilter(sc, of, bw, dt)
            else:
                o += mdlen
                f = Filter(dt)
                f.type = ftype
            p.filters.append(f)
            dt = f.output_datatype(dt)
        return p

    def __repr__(self) -> str:
        return "FilterPipeline(" + ", ".join(repr(f) for f in self.filters) + ")"

    # ---- reverse (unfilter) on the MI355X --------------------------------
    def device_pipeline(self, on_disk_type: int, cell_size: int,
                        version: int = FORMAT_VERSION):
        """The engine-side pipeline for this descriptor (see engine.DevicePipeline)."""
        from .engine import DevicePipeline
        return DevicePipeline(self.serialize(), version, on_disk_type, cell_size)

    def run_reverse(self, tiles, out_sizes: Sequence[int], on_disk_type: int, cell_size: int,
                    version: int = FORMAT_VERSION, offsets_tiles: bool = False, device: int = 0):
        """Unfilter a batch of whole filtered tiles on the GPU.

        The batch analogue of FilterPipeline::run_reverse over every chunk of
        every tile (filter_pipeline.cc:439-517, reader_base.cc:966-989).
        `tiles` is a sequence of byte buffers (host) or a engine.TileBatch
        (device-resident).  Raises FilterStatusException on the first failing
        tile, as parallel_for_2d reports the first error.
        """
        from .engine import Context, TileBatch
        dp = self.device_pipeline(on_disk_type, cell_size, version)
        ctx = Context(device)
        batch = tiles if isinstance(tiles, TileBatch) else TileBatch.from_host(tiles, out_sizes,
                                                                              device=device)
        status = ctx.unfilter(dp, batch, offsets_tiles=offsets_tiles)
        bad = [i for i, s in enumerate(status) if s]
        if bad:
            from ._native import status_str
            raise FilterStatusException(f"tile {bad[0]}: {status_str(int(status[bad[0]]))}")
        return batch
