"""MI355X-native TileDB tile unfilter engine.

Drop-in for TileDB's read-path filter pipeline (FilterPipeline::run_reverse):
byteshuffle, bitshuffle, bit-width reduction, positive delta, double delta and
fixed-size RLE decoded by hand-written gfx950 HIP kernels behind the C-ABI in
include/tiledb_amd.h.  `tiledb_amd.filter_pipeline` mirrors the reference's
filter / pipeline interface; `tiledb_amd.engine` holds the device handles.
"""
from .filter_pipeline import (  # noqa: F401
    FORMAT_VERSION, MAX_TILE_CHUNK_SIZE, BitshuffleFilter, BitWidthReductionFilter,
    ByteshuffleFilter, CompressionFilter, Compressor, Datatype, Filter, FilterOption,
    FilterPipeline, FilterStatusException, FilterType, NoopFilter, PositiveDeltaFilter,
    datatype_size)

