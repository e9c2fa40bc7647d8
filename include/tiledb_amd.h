/*
 * tiledb_amd.h -- C-ABI of the MI355X-native TileDB tile unfilter engine.
 *
 * Drop-in boundary for TileDB's read path:
 *   ReaderBase::unfilter_tile -> FilterPipeline::run_reverse
 *   (reference: tiledb/sm/query/readers/reader_base.cc:1075,1094,1118 and
 *    tiledb/sm/filter/filter_pipeline.h:250-258 / filter_pipeline.cc:439-517)
 * The contract that survives the swap is the on-disk byte layout
 * (format_spec/tile.md, format_spec/filter_pipeline.md): the engine consumes
 * the serialized pipeline descriptor exactly as FilterPipeline::serialize
 * writes it, and whole filtered tiles exactly as they sit on disk.
 *
 * Every function returns a tdbg_status (0 = OK) and never throws.  The last
 * error message of the calling thread is available through
 * tdbg_last_error().  Plain pointers and sizes only; no torch types.
 */
#ifndef TILEDB_AMD_H
#define TILEDB_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- on-disk codes (tiledb/api/c_api/filter/filter_api_enum.h:27-69) ---- */
enum tdbg_filter_type {
  TDBG_FILTER_NONE = 0,
  TDBG_FILTER_GZIP = 1,
  TDBG_FILTER_ZSTD = 2,
  TDBG_FILTER_LZ4 = 3,
  TDBG_FILTER_RLE = 4,
  TDBG_FILTER_BZIP2 = 5,
  TDBG_FILTER_DOUBLE_DELTA = 6,
  TDBG_FILTER_BIT_WIDTH_REDUCTION = 7,
  TDBG_FILTER_BITSHUFFLE = 8,
  TDBG_FILTER_BYTESHUFFLE = 9,
  TDBG_FILTER_POSITIVE_DELTA = 10,
  TDBG_FILTER_AES_256_GCM = 11, /* internal (filter_type.h:17) */
  TDBG_FILTER_CHECKSUM_MD5 = 12,
  TDBG_FILTER_CHECKSUM_SHA256 = 13,
  TDBG_FILTER_DICTIONARY = 14,
  TDBG_FILTER_SCALE_FLOAT = 15,
  TDBG_FILTER_XOR = 16,
  TDBG_FILTER_DEPRECATED = 17,
  TDBG_FILTER_WEBP = 18,
  TDBG_FILTER_DELTA = 19
};

/* tiledb/sm/enums/compressor.h:51-67 */
enum tdbg_compressor {
  TDBG_COMPRESSOR_NONE = 0,
  TDBG_COMPRESSOR_GZIP = 1,
  TDBG_COMPRESSOR_ZSTD = 2,
  TDBG_COMPRESSOR_LZ4 = 3,
  TDBG_COMPRESSOR_RLE = 4,
  TDBG_COMPRESSOR_BZIP2 = 5,
  TDBG_COMPRESSOR_DOUBLE_DELTA = 6,
  TDBG_COMPRESSOR_DICTIONARY = 7,
  TDBG_COMPRESSOR_DELTA = 8
};

/* tiledb/api/c_api/datatype/datatype_api_enum.h:34-120 (subset named) */
enum tdbg_datatype {
  TDBG_INT32 = 0,
  TDBG_INT64 = 1,
  TDBG_FLOAT32 = 2,
  TDBG_FLOAT64 = 3,
  TDBG_CHAR = 4,
  TDBG_INT8 = 5,
  TDBG_UINT8 = 6,
  TDBG_INT16 = 7,
  TDBG_UINT16 = 8,
  TDBG_UINT32 = 9,
  TDBG_UINT64 = 10,
  TDBG_STRING_ASCII = 11,
  TDBG_STRING_UTF8 = 12,
  TDBG_STRING_UTF16 = 13,
  TDBG_STRING_UTF32 = 14,
  TDBG_STRING_UCS2 = 15,
  TDBG_STRING_UCS4 = 16,
  TDBG_ANY = 17,
  TDBG_DATETIME_YEAR = 18, /* ... DATETIME_AS = 30 */
  TDBG_DATETIME_AS = 30,
  TDBG_TIME_HR = 31, /* ... TIME_AS = 39 */
  TDBG_TIME_AS = 39,
  TDBG_BLOB = 40,
  TDBG_BOOL = 41,
  TDBG_GEOM_WKB = 42,
  TDBG_GEOM_WKT = 43
};

/* ---- status codes: one per distinct reference failure class ---- */
enum tdbg_status {
  TDBG_OK = 0,
  TDBG_E_ARG = 1,           /* invalid argument / null pointer                */
  TDBG_E_TILE_FORMAT = 2,   /* chunk directory runs past the tile (Deserializer) */
  TDBG_E_TILE_SIZE = 3,     /* "Incorrect unfiltered tile size allocated." tile.cc:308 */
  TDBG_E_MD_READ = 4,       /* FilterBuffer::read past end of chunk metadata   */
  TDBG_E_DATA_READ = 5,     /* filter input read past end (get_const_buffer/read) */
  TDBG_E_OUT_FULL = 6,      /* output full / fixed allocation too small        */
  TDBG_E_RLE_FORMAT = 7,    /* RLE "invalid input buffer format" rle_compressor.cc:120 */
  TDBG_E_DD_TYPE = 8,       /* DoubleDelta float / unsupported type dd_compressor.cc:195 */
  TDBG_E_BWR_BITS = 9,      /* BWR compressed-bits field not 8/16/32/64        */
  TDBG_E_UNSUPPORTED = 10,  /* filter/pipeline not handled by this engine       */
  TDBG_E_SCRATCH = 11,      /* internal: stage larger than scratch (retried)   */
  TDBG_E_PD_DECREASING = 12,/* forward only: "delta is not positive"           */
  TDBG_E_DD_OVERFLOW = 13,  /* forward only: delta exceeds int64               */
  TDBG_E_DEVICE = 14,       /* HIP runtime error                               */
  TDBG_E_DESCRIPTOR = 15,   /* malformed serialized pipeline                    */
  TDBG_E_DELTA_TYPE = 16,   /* Delta float: "Decompression is not yet supported for
                               float datatypes." delta_compressor.cc:210-213   */
  TDBG_E_INTERNAL = 17,     /* internal engine error (a device work queue overflowed):
                               the tile was not unfiltered; never expected   */
  TDBG_E_IO = 18,           /* tdbg_read_unfilter_tiles: a block read failed
                               (VFS::read_exactly: short read or I/O error)  */
  TDBG_E_NOT_RUN = 19       /* the call stopped (a device or argument error)
                               before this tile was read or unfiltered       */
};

/* unfilter flags */
#define TDBG_TILE_OFFSETS 0x1u /* offsets tile: expected size = out_size - 8 (tile.cc:241-248) */
/* Chunk-parallel launch: a device pass first builds the chunk directory of
 * every tile (Tile::load_chunk_data, tile.cc:280-313) and the fused kernel
 * then takes chunks, not tiles, as work items -- the tile x chunk-range split
 * of reader_base.cc:970-989 on the device, for batches of few, multi-chunk
 * tiles.  Results and statuses are those of a tile launch.  Applied
 * automatically when a launch has fewer tiles than the device has CUs. */
#define TDBG_CHUNK_PARALLEL 0x8u
/* Some tile of the launch holds several chunks (an unfiltered size over the
 * pipeline's 64 KiB chunks, tile.cc:87-100).  Tile-mode launches of the
 * headline pipeline [BYTESHUFFLE, DOUBLE_DELTA, BIT_WIDTH_REDUCTION] on 4-byte
 * integers then run the C5 tile kernel's multi-chunk variant, in which a
 * workgroup decodes its tile's chunks one after the other
 * (FilterPipeline::run_reverse's loop, filter_pipeline.cc:439-517); without it
 * such tiles go to the fused kernel.  Results and statuses are the same
 * either way.  The host-resident entries set it themselves from the tile
 * sizes they are given. */
#define TDBG_MULTI_CHUNK 0x10u
/* tdbg_unfilter_tiles_host only: every input tile of the call lies in ONE host
 * allocation (e.g. a FilteredData block, filtered_data.h:152-644), so tiles
 * separated by at most 64 B of padding may move in one H2D copy (padding
 * included).  Without it every tile is its own copy. */
#define TDBG_HOST_CONTIGUOUS_INPUT 0x2u
/* tdbg_unfilter_tiles_host only: every output buffer lies in one host
 * allocation; exactly adjacent outputs may share one D2H copy. */
#define TDBG_HOST_CONTIGUOUS_OUTPUT 0x4u

typedef struct tdbg_pipeline tdbg_pipeline; /* immutable, shareable */
typedef struct tdbg_context tdbg_context;   /* per (device, host thread) */
typedef void* tdbg_stream;                  /* hipStream_t */

/* Message of the calling thread's last failure; returns bytes written. */
size_t tdbg_last_error(char* buf, size_t cap);
const char* tdbg_status_str(int status);

/* Parse the serialized pipeline exactly as FilterPipeline::deserialize
 * (filter_pipeline.cc:544-557, filter_create.cc:100-201) and assign each
 * filter its datatype along the chain starting at on_disk_datatype
 * (filter_pipeline.cc:80-88).  cell_size = Tile::cell_size() (RLE value width,
 * compression_filter.cc:357,418). */
int tdbg_pipeline_create(const uint8_t* serialized, size_t len,
                         uint32_t format_version, uint8_t on_disk_datatype,
                         uint64_t cell_size, tdbg_pipeline** out);
void tdbg_pipeline_destroy(tdbg_pipeline* p);
/* 1 if every filter runs on the engine, 0 if the caller must keep its own
 * path.  Supported: NONE/NOOP, BYTESHUFFLE, BITSHUFFLE, BIT_WIDTH_REDUCTION,
 * POSITIVE_DELTA, XOR (1/2/4/8-byte types), SCALE_FLOAT (float32/64 input,
 * byte width 1/2/4/8), and the compression filters NONE, RLE (fixed-size
 * cells), DOUBLE_DELTA and DELTA.  Unsupported (returns 0): checksums
 * (MD5/SHA256), AES-256-GCM, GZIP/ZSTD/LZ4/BZIP2, DICTIONARY, WEBP, RLE with
 * cell size 0, XOR / SCALE_FLOAT on widths the reference rejects. */
int tdbg_pipeline_supported(const tdbg_pipeline* p);
uint32_t tdbg_pipeline_num_filters(const tdbg_pipeline* p);
/* Filter i: type code and the datatype assigned by the chain. */
int tdbg_pipeline_filter(const tdbg_pipeline* p, uint32_t i, uint8_t* type,
                         uint8_t* datatype);

/* Per-device execution context (scratch, status arrays, streams).
 * Threading: the reference is re-entrant (reader_base.cc:929-934); here
 * each host thread uses its own context (contexts share nothing but the
 * immutable pipeline).  One context's launches are serialized: a launch on a
 * different stream than the context's previous launch first waits (on the
 * host) for that stream. */
int tdbg_context_create(int device, tdbg_context** out);
void tdbg_context_destroy(tdbg_context* ctx);

/* Device-resident batch unfilter: the replacement for the
 * parallel_for_2d(tile, range) -> FilterPipeline::run_reverse loop of
 * ReaderBase::unfilter_tiles (reader_base.cc:966-989).
 *   d_filtered[i] / d_filtered_size[i]: filtered tile i in device memory
 *   d_out[i] / d_out_size[i]: caller-allocated unfiltered buffer (device)
 *   d_status[i]: per-tile tdbg_status written by the device (may be NULL)
 * All four arrays live in device memory on ctx's device.  Enqueues on stream
 * and returns without synchronizing; per-tile failures are reported through
 * d_status (TDBG_E_SCRATCH means "re-run with tdbg_unfilter_tiles_sync"). */
int tdbg_unfilter_tiles_async(tdbg_context* ctx, const tdbg_pipeline* p,
                              uint64_t ntiles,
                              const uint8_t* const* d_filtered,
                              const uint64_t* d_filtered_size,
                              uint8_t* const* d_out,
                              const uint64_t* d_out_size, uint32_t flags,
                              int32_t* d_status, tdbg_stream stream);

/* Same, synchronous: resolves TDBG_E_SCRATCH tiles with the global-memory
 * path, copies the statuses to host_status (may be NULL) and returns the
 * first failing tile's status, like parallel_for_2d keeps the first error
 * (parallel_functions.h:340-345). */
int tdbg_unfilter_tiles_sync(tdbg_context* ctx, const tdbg_pipeline* p,
                             uint64_t ntiles, const uint8_t* const* d_filtered,
                             const uint64_t* d_filtered_size,
                             uint8_t* const* d_out, const uint64_t* d_out_size,
                             uint32_t flags, int32_t* host_status,
                             tdbg_stream stream);

/* Host-resident end-to-end: tiles start in host memory (as FilteredData
 * leaves them, filtered_data.h:397-398) and end in host result buffers.
 * Pinned staging + hipMemcpyAsync H2D / unfilter / D2H on ctx's device,
 * double-buffered over batches of batch_bytes. */
int tdbg_unfilter_tiles_host(tdbg_context* ctx, const tdbg_pipeline* p,
                             uint64_t ntiles, const uint8_t* const* filtered,
                             const uint64_t* filtered_size, uint8_t* const* out,
                             const uint64_t* out_size, uint32_t flags,
                             int32_t* host_status, uint64_t batch_bytes);

/* Tile::add_extra_offset (tile.h:144-146, called after an offsets tile is
 * unfiltered at reader_base.cc:893): for every tile whose d_status entry is
 * TDBG_OK (every tile when d_status is NULL), the last 8 bytes of d_out[i]
 * (the extra slot a TDBG_TILE_OFFSETS unfilter leaves) become d_var_size[i],
 * the size of the tile's var-data tile.  Device arrays; enqueued on stream. */
int tdbg_add_extra_offsets_async(tdbg_context* ctx, uint64_t ntiles, uint8_t* const* d_out,
                                 const uint64_t* d_out_size, const uint64_t* d_var_size,
                                 const int32_t* d_status, tdbg_stream stream);

/* tdbg_unfilter_tiles_host for offsets tiles with the extra offset fused
 * before the D2H: flags must include TDBG_TILE_OFFSETS; var_size (host array,
 * one per tile) is copied with the batch's pointer arrays and written into
 * each tile's last 8 bytes on the device, so the result buffers receive
 * complete offsets tiles in the same copy (reader_base.cc:885-893). */
int tdbg_unfilter_offsets_host(tdbg_context* ctx, const tdbg_pipeline* p, uint64_t ntiles,
                               const uint8_t* const* filtered, const uint64_t* filtered_size,
                               uint8_t* const* out, const uint64_t* out_size,
                               const uint64_t* var_size, uint32_t flags, int32_t* host_status,
                               uint64_t batch_bytes);

/* Contiguous tile shards balanced by filtered + unfiltered bytes: shard k is
 * tiles [cuts[k], cuts[k+1]), cuts has nshards + 1 entries.  Host-only; the
 * multi-GPU entry point and one-process-per-GPU callers (each rank takes its
 * shard, no collective on the data path) use the same cut. */
int tdbg_shard_tiles(uint64_t ntiles, const uint64_t* in_size, const uint64_t* out_size,
                     uint32_t nshards, uint64_t* cuts);

/* Multi-GPU host-resident end-to-end: tiles are sharded over devices by
 * contiguous ranges balanced by bytes, one host thread + context per device,
 * no inter-GPU communication.  The per-device contexts (staging, status and
 * scratch buffers) are kept in a process-wide pool and reused by later calls
 * (a reader calls this once per batch); tdbg_release_cached_contexts frees
 * the pooled ones. */
int tdbg_unfilter_tiles_multi_gpu(const tdbg_pipeline* p, uint64_t ntiles,
                                  const uint8_t* const* filtered,
                                  const uint64_t* filtered_size,
                                  uint8_t* const* out,
                                  const uint64_t* out_size, uint32_t flags,
                                  int32_t* host_status, const int* devices,
                                  int ndevices, uint64_t batch_bytes);
/* Destroys the contexts the multi-GPU entry keeps for reuse (none is in use
 * by a running call afterwards only if no call is running). */
int tdbg_release_cached_contexts(void);
/* Number of idle pooled contexts (diagnostics / tests). */
int tdbg_cached_context_count(void);

/* CPU entry: the same batch unfilter on host threads, for
 * host-resident tiles and the CPU baseline.  The work split is the
 * reference's: parallel_for_2d over (tile, range thread) with
 * num_range_threads = ceil(nthreads / ntiles) when ntiles < nthreads, each
 * range thread taking the chunk range compute_chunk_min_max gives it
 * (reader_base.cc:929-989, reader_base.h:185-210).  nthreads = 0: hardware
 * concurrency (sm.compute_concurrency_level's default, config.cc:128-131).
 * Per-tile statuses as the device path; returns the first failing tile's. */
int tdbg_unfilter_tiles_cpu(const tdbg_pipeline* p, uint64_t ntiles,
                            const uint8_t* const* filtered,
                            const uint64_t* filtered_size, uint8_t* const* out,
                            const uint64_t* out_size, uint32_t flags,
                            int32_t* host_status, uint32_t nthreads);

/* ---- forward (filter) direction: the write path ---------------------------
 * Replaces WriterBase::filter_tile -> FilterPipeline::run_forward
 * (writer_base.cc:870-915, filter_pipeline.cc:382-426; chunks
 * filter_pipeline.cc:208-369, WriterTile::compute_chunk_size tile.cc:87-100)
 * for fixed-size tiles: each unfiltered tile d_in[i] (d_in_size[i] bytes) is
 * chunked (max_chunk = 0: 64 KiB, constants.cc:730), run through every
 * filter's run_forward and written in the on-disk layout
 * [u64 nchunks]([u32 orig][u32 filtered][u32 md][md][data])* to d_out[i]
 * (capacity d_out_cap[i], tdbg_filtered_bound() always suffices); its length
 * goes to d_out_len[i].  Device arrays, like tdbg_unfilter_tiles_async.
 * Statuses: TDBG_E_PD_DECREASING, TDBG_E_DD_OVERFLOW, TDBG_E_RLE_FORMAT,
 * TDBG_E_DD_TYPE / TDBG_E_DELTA_TYPE, TDBG_E_OUT_FULL (capacity), TDBG_E_ARG
 * (a BWR / PD window smaller than one value: a division by zero in the
 * reference).  The BWR offset of a window whose range overflows T is
 * uninitialized in the reference (bit_width_reduction_filter.cc:421-430)
 * and written as 0 here. */
uint64_t tdbg_filtered_bound(const tdbg_pipeline* p, uint64_t tile_size, uint32_t max_chunk);
int tdbg_filter_tiles_async(tdbg_context* ctx, const tdbg_pipeline* p, uint64_t ntiles,
                            const uint8_t* const* d_in, const uint64_t* d_in_size,
                            uint8_t* const* d_out, const uint64_t* d_out_cap,
                            uint64_t* d_out_len, uint32_t max_chunk, int32_t* d_status,
                            tdbg_stream stream);
/* Same, synchronous; statuses to host_status (may be NULL); returns the first
 * failing tile's status. */
int tdbg_filter_tiles_sync(tdbg_context* ctx, const tdbg_pipeline* p, uint64_t ntiles,
                           const uint8_t* const* d_in, const uint64_t* d_in_size,
                           uint8_t* const* d_out, const uint64_t* d_out_cap,
                           uint64_t* d_out_len, uint32_t max_chunk, int32_t* host_status,
                           tdbg_stream stream);

/* Stats mirrored from the reference (filter_pipeline.cc:490-491,
 * reader_base.cc:1074): cumulative since context creation.  tiles_unfiltered
 * counts tiles submitted; read_unfiltered_byte_num counts the unfiltered bytes
 * of tiles that unfiltered successfully (device counters; synchronizes the
 * device). */
int tdbg_context_stats(const tdbg_context* ctx, uint64_t* tiles_unfiltered,
                       uint64_t* read_unfiltered_byte_num);

/* Which device path handled the tiles (cumulative, synchronizes the device):
 * fused_tiles = unfiltered by the fused LDS kernel, fallback_tiles = declined
 * by it and re-run by the general interpreter, general_tiles = unfiltered by
 * the general interpreter (fallbacks, pipelines without a fused spec and
 * scratch retries). */
int tdbg_context_path_stats(const tdbg_context* ctx, uint64_t* fused_tiles,
                            uint64_t* fallback_tiles, uint64_t* general_tiles);

/* Of the fused tiles: how many the streaming kernels for the headline
 * pipeline [BYTESHUFFLE, DOUBLE_DELTA, BIT_WIDTH_REDUCTION] on 4-byte integers
 * took (one 64 KiB chunk; DD bit-packed: tdbg_stream.hip, DD raw:
 * tdbg_stream_raw.hip).  The tiles they leave go to the fused kernel in the
 * same launch.  Cumulative; waits for the context's last launch. */
int tdbg_context_stream_stats(const tdbg_context* ctx, uint64_t* stream_tiles);
/* Of those, the tiles the raw-DoubleDelta streaming kernel took (C5 tiles
 * whose DD stage stored the values raw, tdbg_stream_raw.hip). */
int tdbg_context_stream_raw_stats(const tdbg_context* c, uint64_t* raw_tiles);
/* Chunk-parallel launches (TDBG_CHUNK_PARALLEL, or fewer tiles than CUs) of
 * the headline pipeline: the chunks the streaming kernels took from the
 * device chunk directory (each a 64 KiB chunk of a multi-chunk tile, decoded
 * as the one-chunk tiles are).  Cumulative; waits for the context's last
 * launch. */
int tdbg_context_stream_chunk_stats(const tdbg_context* c, uint64_t* chunks);
/* Chunks of multi-chunk tiles the C5 tile kernel decoded in tile mode
 * (TDBG_MULTI_CHUNK launches), cumulative per context. */
int tdbg_context_tile_chunk_stats(const tdbg_context* c, uint64_t* chunks);
/* Forward direction: tiles the LDS-resident forward kernels filtered --
 * [BYTESHUFFLE, DOUBLE_DELTA, BWR(256)] on INT32 / UINT32
 * (tdbg_forward_stream.hip) and, on 8-byte values, [DOUBLE_DELTA], [RLE] and
 * [POSITIVE_DELTA(1024), BWR(256)] (tdbg_forward_small.hip), 64 KiB tiles;
 * the others run on the general forward kernel.  Cumulative; waits for the
 * context's last launch. */
int tdbg_context_forward_stream_stats(const tdbg_context* c, uint64_t* tiles);

/* Device-side time (ms) of the last *armed* tdbg_unfilter_tiles_* launch on
 * ctx (fused/general kernel + fixup), from the hipEvents that
 * tdbg_context_time_launches arms.  Un-armed launches record no events: an
 * event record costs ~3 % of a C5 launch on the stream's timeline. */
int tdbg_context_last_kernel_ms(tdbg_context* ctx, float* ms);

/* Per-launch device timing for benchmarks: arm event recording for the next
 * n tdbg_unfilter_tiles_* launches on ctx, then read them back (waits for the
 * last armed launch).  A launch is up to three kernels on one stream: for the
 * headline pipeline [BYTESHUFFLE, DOUBLE_DELTA, BWR] on 4-byte integers the
 * streaming kernel and the fused kernel on the tiles it left, otherwise the
 * fused LDS kernel (or the general kernel); then the fallback fixup.
 * kernel_ms[i] = the unfilter kernel(s) of launch i before the fixup,
 * total_ms[i] = all of the launch.  Outputs may be NULL; reading disarms. */
int tdbg_context_time_launches(tdbg_context* ctx, uint32_t n);
int tdbg_context_launch_times(tdbg_context* ctx, float* kernel_ms, float* total_ms,
                              uint32_t cap, uint32_t* count);

/* Diagnostics (no reference counterpart): with TDBG_PROF=1 in the
 * environment, the fused kernel accumulates shader-clock cycles per phase
 * (0 tile wait, 1 headers, 2-4 intermediate stages, 5 final stage, 6 loop
 * tail); this sums them over the workgroups of the last launch. */
int tdbg_debug_phase_clocks(tdbg_context* ctx, uint64_t* out, uint32_t nphases);

/* Device memory helpers for FFI callers without their own allocator. */
int tdbg_device_alloc(int device, uint64_t bytes, void** out);
int tdbg_device_free(void* p);
int tdbg_memcpy_h2d(void* dst, const void* src, uint64_t bytes);
int tdbg_memcpy_d2h(void* dst, const void* src, uint64_t bytes);
int tdbg_device_count(int* n);

/* ======================================================================
 * The steps either side of the path
 * ====================================================================== */

/* Device index of a context. */
int tdbg_context_device(const tdbg_context* ctx);

/* Pinned host memory on the device's NUMA node (the calling thread is bound
 * to the device's local CPUs while the pages are allocated and first
 * touched), for staging and result buffers the H2D / D2H DMA reads/writes. */
int tdbg_host_alloc_local(int device, uint64_t bytes, void** out);
int tdbg_host_free(void* p);

/* FilteredData block rule (filtered_data.h:531-575): tiles in result-tile
 * order, tile i at file_offset[i] (size[i]) of file file_idx[i]; a tile
 * extends the current block when it is in the same file, the block stays <=
 * max_batch_size, and the block is <= min_batch_size or the gap to the tile
 * is <= min_batch_gap.  block_first_tile (ntiles + 1 entries) receives the
 * first tile of each block and, after the last block, ntiles. */
int tdbg_filtered_data_blocks(uint64_t ntiles, const uint32_t* file_idx, const uint64_t* file_offset,
                              const uint64_t* size, uint64_t min_batch_size, uint64_t max_batch_size,
                              uint64_t min_batch_gap, uint64_t* block_first_tile, uint64_t* nblocks);

typedef struct tdbg_read_config {
  uint64_t min_batch_size;  /* 0: vfs.min_batch_size default, 20 MiB (config.cc:165) */
  uint64_t max_batch_size;  /* 0: vfs.max_batch_size default, 100 MiB (config.cc:163) */
  uint64_t min_batch_gap;   /* 0: vfs.min_batch_gap default, 500 KB (config.cc:164),
                               unless TDBG_READ_ZERO_GAP */
  uint32_t io_threads;      /* 0: 4 (the reference's IO thread pool role) */
  uint32_t slots;           /* pinned block slots, >= 2 (0: 3) */
  uint32_t flags;
} tdbg_read_config;
#define TDBG_READ_ZERO_GAP 0x1u /* min_batch_gap = 0 is meant literally */

/* Read + unfilter: ReaderBase::read_tiles (reader_base.cc:689-789) ->
 * FilteredData blocks read with pread (VFS::read_exactly,
 * filtered_data.h:397-398) by IO threads into NUMA-local pinned slots, each
 * landed block unfiltered by tdbg_unfilter_tiles_host (H2D -> kernels ->
 * D2H into out[i]) while later blocks are read.  fds[f] is an open file
 * descriptor of fragment file f.  Tiles of a failed block read get
 * TDBG_E_IO.  For full speed the out buffers should be pinned
 * (tdbg_host_alloc_local). */
int tdbg_read_unfilter_tiles(tdbg_context* ctx, const tdbg_pipeline* p, uint64_t ntiles, const int* fds,
                             uint32_t nfiles, const uint32_t* file_idx, const uint64_t* file_offset,
                             const uint64_t* persisted_size, uint8_t* const* out, const uint64_t* out_size,
                             uint32_t flags, const tdbg_read_config* cfg, int32_t* host_status);

/* Dense cell-slab copy (DenseReader::copy_fixed_tiles,
 * dense_reader.cc:1555-1750) for one fragment covering the subarray: the
 * cells of subarray [sub_lo, sub_hi] (one inclusive range per dimension) are
 * copied from the unfiltered tiles -- tile t covers [tile_start[t*dim_num + d],
 * + tile_extent[d]) in cell order cell_order -- into a result buffer in the
 * query layout (row-major: last dimension fastest).  Same order: slab
 * memcpy; different: cell by cell, as the reference. */
#define TDBG_DENSE_MAX_DIMS 4
typedef struct tdbg_dense_copy_config {
  uint32_t dim_num;     /* 1..TDBG_DENSE_MAX_DIMS */
  uint32_t cell_size;   /* bytes per cell (fixed-size attribute) */
  uint32_t cell_order;  /* tile cell order: 0 row-major, 1 col-major */
  uint32_t layout;      /* result layout: 0 row-major, 1 col-major */
  int64_t tile_extent[TDBG_DENSE_MAX_DIMS];
  int64_t sub_lo[TDBG_DENSE_MAX_DIMS];
  int64_t sub_hi[TDBG_DENSE_MAX_DIMS];
} tdbg_dense_copy_config;

/* Bytes of the result buffer of a dense copy: prod(sub_hi - sub_lo + 1) * cell_size
 * (0 for an invalid config). */
uint64_t tdbg_dense_result_bytes(const tdbg_dense_copy_config* cfg);

/* Device-resident: unfiltered device tiles d_tiles[t] (tile starts in
 * d_tile_start, device) -> device result buffer; tiles whose d_status is not
 * TDBG_OK (if given) are skipped. */
int tdbg_dense_copy_async(tdbg_context* ctx, const tdbg_dense_copy_config* cfg, uint64_t ntiles,
                          const int64_t* d_tile_start, const uint8_t* const* d_tiles, const int32_t* d_status,
                          uint8_t* d_result, tdbg_stream stream);

/* The dense read of a field with copy_attribute fused into the transfer:
 * filtered host tiles -> H2D -> unfilter -> cell-slab copy into a device
 * result buffer -> one D2H of the result (result_size >=
 * tdbg_dense_result_bytes), so PCIe carries the filtered tiles in and only
 * the subarray's cells out.  tile_start: host, ntiles * dim_num. */
int tdbg_dense_read_host(tdbg_context* ctx, const tdbg_pipeline* p, uint64_t ntiles, const uint8_t* const* in,
                         const uint64_t* in_size, const int64_t* tile_start, const tdbg_dense_copy_config* cfg,
                         uint8_t* result, uint64_t result_size, uint32_t flags, int32_t* host_status,
                         uint64_t batch_bytes);

/* ---- dense reads with several fragments, fill values, var-sized cells -----
 * DenseReader::copy_fixed_tiles / copy_offset_tiles / fix_offsets_buffer /
 * copy_var_tiles (dense_reader.cc:1199-1236, 1521-2000).  Space tile t has
 * one unfiltered tile per fragment fd (pointer arrays of ntiles * nfrag
 * entries, [t * nfrag + fd]; NULL: the fragment has no tile there); fragment
 * fd covers the inclusive domain d_frag_dom[(fd * dim_num + d) * 2 + {0, 1}].
 * Where domains overlap, the fragment with the LOWER index wins (the
 * reference walks them from the last to the first, each overwriting); cells
 * no fragment covers get the fill value (Attribute::fill_value) and
 * fill_validity, and so do cells of the subarray in no given space tile (the
 * async entries write the fill value into every result cell first).  A
 * present fragment without a validity tile (d_validity NULL, or its entry
 * NULL) counts as valid.  Result buffers are in the query layout
 * (base.layout). */
typedef struct tdbg_dense_frag_config {
  tdbg_dense_copy_config base; /* dims, subarray, tile extents, cell/result order;
                                  base.cell_size: bytes per cell (fixed), 8 (var) */
  uint32_t nfrag;              /* fragments (0: every cell gets the fill value) */
  uint32_t nullable;           /* copy validity tiles (1 byte per cell) too */
  uint32_t fill_size;          /* bytes of the fill value (fixed: == cell_size) */
  uint32_t fill_validity;      /* Attribute::fill_value_validity (0 or 1) */
  uint32_t elements_mode;      /* var: offsets count elements of data_type_size (elements_mode_) */
  uint32_t data_type_size;     /* var: datatype_size of the attribute */
} tdbg_dense_frag_config;

/* Fixed-size cells: device tiles / validity tiles / fill value -> device
 * result (+ validity). */
int tdbg_dense_copy_fragments_async(tdbg_context* ctx, const tdbg_dense_frag_config* cfg, uint64_t ntiles,
                                    const int64_t* d_tile_start, const int64_t* d_frag_dom,
                                    const uint8_t* const* d_tiles, const uint8_t* const* d_validity,
                                    const uint8_t* d_fill_value, uint8_t* d_result, uint8_t* d_result_validity,
                                    tdbg_stream stream);

/* Var-sized cells, step 1 (copy_offset_tiles + fix_offsets_buffer): from the
 * unfiltered offsets tiles (uint64, tile cells + 1 entries: the extra offset
 * of tile.h:144-146 included) and var tiles, the result offsets (uint64, one
 * per result cell, in elements in elements mode) and their total
 * (*d_var_total, device); the cells' source addresses stay in ctx for step 2.
 * A cell whose offsets o[i] <= o[i + 1] <= o[tile cells] do not hold is
 * read as empty (nothing is read outside a var tile) and flags the context;
 * the flag is cleared on `stream` at the start of every call, and
 * tdbg_dense_var_status reports it (tdbg_dense_read_var_host returns
 * TDBG_E_DATA_READ for it). */
int tdbg_dense_var_offsets_async(tdbg_context* ctx, const tdbg_dense_frag_config* cfg, uint64_t ntiles,
                                 const int64_t* d_tile_start, const int64_t* d_frag_dom,
                                 const uint8_t* const* d_offset_tiles, const uint8_t* const* d_var_tiles,
                                 const uint8_t* const* d_validity, const uint8_t* d_fill_value,
                                 uint64_t* d_result_offsets, uint8_t* d_result_validity, uint64_t* d_var_total,
                                 tdbg_stream stream);
/* Step 2 (copy_var_tiles): every cell's bytes to d_result_var + offset (x the
 * type size in elements mode); d_result_var holds *d_var_total units. */
int tdbg_dense_var_copy_async(tdbg_context* ctx, const tdbg_dense_frag_config* cfg,
                              const uint64_t* d_result_offsets, const uint64_t* d_var_total, uint8_t* d_result_var,
                              tdbg_stream stream);
/* The data check of the last tdbg_dense_var_offsets_async on ctx: waits for
 * `stream` (the one that call ran on), then *status = TDBG_OK, or
 * TDBG_E_DATA_READ when a cell's offsets lay outside its var tile (those
 * cells were read as empty, as the reference's Status_ReaderError for a
 * corrupt offsets tile fails the read). */
int tdbg_dense_var_status(tdbg_context* ctx, tdbg_stream stream, int32_t* status);

/* Host-resident var-sized dense read fused with the transfers: the filtered
 * offsets and var tiles of every (space tile, fragment) -> H2D -> unfilter
 * (offsets tiles as TDBG_TILE_OFFSETS with the extra offset = the var tile's
 * unfiltered size, reader_base.cc:885-893) -> steps 1 and 2 -> D2H of the
 * result offsets (ncells uint64) and var bytes.  var_unfiltered_size[i]: the
 * var tile's unfiltered bytes; NULL filtered pointers: fragment absent.
 * *var_total receives the var bytes; TDBG_E_OUT_FULL if var_cap is smaller
 * (nothing copied to result_var).  Statuses per (tile, fragment) pair: the
 * offsets tile's, or the var tile's if that one failed.  cfg->nullable must
 * be 0 here (validity tiles: tdbg_dense_var_offsets_async).  The space tiles
 * must cover the subarray exactly once on one tile grid (TDBG_E_ARG
 * otherwise), as the reference iterates every space tile of the subarray;
 * tiles whose stages outgrow the default scratch are redone through the
 * sync entry's retry, as in tdbg_unfilter_tiles_sync. */
int tdbg_dense_read_var_host(tdbg_context* ctx, const tdbg_pipeline* p_offsets, const tdbg_pipeline* p_var,
                             const tdbg_dense_frag_config* cfg, uint64_t ntiles, const int64_t* tile_start,
                             const int64_t* frag_dom, const uint8_t* const* off_filtered,
                             const uint64_t* off_filtered_size, const uint8_t* const* var_filtered,
                             const uint64_t* var_filtered_size, const uint64_t* var_unfiltered_size,
                             const uint8_t* fill_value, uint64_t* result_offsets, uint8_t* result_var,
                             uint64_t var_cap, uint64_t* var_total, int32_t* host_status);

#ifdef __cplusplus
}
#endif
#endif /* TILEDB_AMD_H */
