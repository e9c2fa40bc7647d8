/*
 * tdb_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of TileDB's tile filter pipeline (reference at
 * TileDB-Inc/TileDB, tiledb/sm/filter + tiledb/sm/compressors), used as the
 * parity checker for the HIP engine and as the timed `cpu_baseline` leg of
 * bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * may load this library.  The product path (libtiledb_amd.so) never links it.
 *
 * Parity pinning: the reference cannot be built in this image without
 * stand-in headers (tiledb/common/logger.h needs spdlog, which is absent), so
 * this restatement is pinned by the reference's own golden vectors and
 * known-answer tests (descriptor bytes, RLE sizes, BWR header fields), by the
 * format_spec layouts, and for bitshuffle by fixtures produced with the
 * kiyo-masui bitshuffle 0.3.5 that ships in this image's imagecodecs.
 * See tests/golden/README.md and DESIGN.md section "Oracle".
 */
#ifndef TDB_ORACLE_H
#define TDB_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/tiledb_amd.h" /* shared enums and error codes */

#ifdef __cplusplus
extern "C" {
#endif

#define ORACLE_MAX_FILTERS 32

typedef struct oracle_filter {
  uint8_t type;        /* tdbg_filter_type (on-disk code)                   */
  uint8_t compressor;  /* tdbg_compressor, compression filters only         */
  int32_t level;       /* compression level (ignored by DD/RLE)             */
  uint8_t reinterpret; /* DD/DELTA reinterpret datatype, ANY if absent      */
  uint32_t window;     /* BWR / PD max window                               */
  uint8_t datatype;    /* filter_data_type_ from the datatype chain         */
  double scale, offset; /* FLOAT_SCALE FilterConfig (float_scaling_filter.h:61-65) */
  uint64_t byte_width;
} oracle_filter;

typedef struct oracle_pipeline {
  uint32_t max_chunk_size;
  uint32_t nfilters;
  uint32_t version;
  uint8_t on_disk_type;
  uint64_t cell_size;
  oracle_filter f[ORACLE_MAX_FILTERS];
} oracle_pipeline;

/* FilterPipeline::deserialize (filter_pipeline.cc:544-557) + datatype chain
 * (filter_pipeline.cc:80-88, FilterCreate::deserialize filter_create.cc:100). */
int oracle_pipeline_parse(const uint8_t* bytes, size_t len, uint32_t version,
                          uint8_t datatype, uint64_t cell_size,
                          oracle_pipeline* out, size_t* consumed);
/* FilterPipeline::serialize (filter_pipeline.cc:524-542). */
int oracle_pipeline_serialize(const oracle_pipeline* p, uint8_t* out,
                              size_t cap, size_t* len);

/* WriterTile::compute_chunk_size (tile.cc:87-100).  max_chunk==0 -> 64 KiB. */
uint32_t oracle_compute_chunk_size(uint64_t tile_size, uint64_t cell_size,
                                   uint64_t max_chunk);

/* FilterPipeline::run_forward (filter_pipeline.cc:382-426) for one tile.
 * offsets/noffsets: optional var-size offsets (get_var_chunk_sizes).
 * max_chunk: WriterTile::max_tile_chunk_size_ (0 = 64 KiB default).
 * Writes the filtered tile ([u64 nchunks][chunks...]) into out. */
int oracle_filter_tile(const oracle_pipeline* p, const uint8_t* tile,
                       uint64_t size, const uint64_t* offsets,
                       uint64_t noffsets, uint64_t max_chunk, uint8_t* out,
                       uint64_t cap, uint64_t* out_len);

/* Upper bound for oracle_filter_tile's output. */
uint64_t oracle_filtered_bound(const oracle_pipeline* p, uint64_t size,
                               uint64_t max_chunk);

/* Tile::load_chunk_data + FilterPipeline::run_reverse over all chunks
 * (tile.cc:280-313, filter_pipeline.cc:439-517).  is_offsets: the tile is an
 * offsets tile (expected size out_size - 8, tile.cc:241-248). */
int oracle_unfilter_tile(const oracle_pipeline* p, const uint8_t* filtered,
                         uint64_t fsize, uint8_t* out, uint64_t out_size,
                         int is_offsets);

/* Batched reverse over many tiles on nthreads host threads, the same
 * tile-level split as ReaderBase::unfilter_tiles (reader_base.cc:929-989).
 * status[i] receives each tile's error code.  Returns the first nonzero. */
int oracle_unfilter_tiles_mt(const oracle_pipeline* p, uint64_t ntiles,
                             const uint8_t* in_base, const uint64_t* in_off,
                             const uint64_t* in_size, uint8_t* out_base,
                             const uint64_t* out_off, const uint64_t* out_size,
                             int nthreads, int32_t* status);

/* Single-filter codec entry points (unit tests of the codecs themselves). */
int oracle_rle_compress(uint64_t value_size, const uint8_t* in, uint64_t n,
                        uint8_t* out, uint64_t cap, uint64_t* out_len);
int oracle_rle_decompress(uint64_t value_size, const uint8_t* in, uint64_t n,
                          uint8_t* out, uint64_t out_size);
int oracle_dd_compress(uint8_t dtype, const uint8_t* in, uint64_t n,
                       uint8_t* out, uint64_t cap, uint64_t* out_len);
int oracle_dd_decompress(uint8_t dtype, const uint8_t* in, uint64_t n,
                         uint8_t* out, uint64_t out_size);
int oracle_bitshuffle_block(int inverse, uint32_t ts, const uint8_t* in,
                            uint64_t n, uint8_t* out);
int oracle_byteshuffle(int inverse, uint32_t ts, const uint8_t* in, uint64_t n,
                       uint8_t* out);

uint64_t oracle_datatype_size(uint8_t dt);

#ifdef __cplusplus
}
#endif
#endif
