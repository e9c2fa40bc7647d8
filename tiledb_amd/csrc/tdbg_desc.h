// tdbg_desc.h -- pipeline plan shared by the host orchestration
// (tdbg_host.cpp) and the gfx950 kernels (tdbg_kernels.hip).
//
// The host resolves every filter of a deserialized FilterPipeline into a
// "stage kind" plus the integer widths the reference picks at run time
// (bit_width_reduction_filter.cc:288-350, positive_delta_filter.cc:262-322,
// dd_compressor.cc:131-200, compression_filter.cc:357,418), so the device
// never switches on datatypes.
#pragma once
#include <stdint.h>

#define TDBG_MAX_FILTERS 16

enum tdbg_stage_kind : uint8_t {
  TDBG_K_PASS = 0,        // append_view pass-through (NOOP, NONE, BWR/PD on non-int)
  TDBG_K_BYTESHUFFLE = 1, // ByteshuffleFilter::run_reverse
  TDBG_K_BITSHUFFLE = 2,  // BitshuffleFilter::run_reverse
  TDBG_K_BWR = 3,         // BitWidthReductionFilter::run_reverse<T>
  TDBG_K_PD = 4,          // PositiveDeltaFilter::run_reverse<T>
  TDBG_K_DD = 5,          // CompressionFilter + DoubleDelta::decompress<T>
  TDBG_K_RLE = 6,         // CompressionFilter + RLE::decompress
  TDBG_K_XOR = 7,         // XORFilter::run_reverse<T> (prefix XOR; general interpreter only)
  TDBG_K_DELTA = 8,       // CompressionFilter + Delta::decompress<T> (general interpreter only)
  TDBG_K_FSCALE = 9,      // FloatScalingFilter::run_reverse<T, W> (general interpreter only)
  TDBG_K_UNSUPPORTED = 10
};

struct tdbg_stage {
  uint8_t kind;
  uint8_t w;    // element width: BWR/PD T, DD T (0 = DD type error), shuffle ts
  uint8_t sgn;  // T signed (BWR sign extension)
  uint8_t dts;  // datatype_size(filter datatype): md offset / output value width
  uint32_t window;
  uint64_t cs;  // RLE value size (Tile::cell_size)
};

struct tdbg_plan {
  uint32_t nstages;
  uint32_t fast;  // fused fast-path selector (tdbg_fast_kind), 0 = none
  tdbg_stage s[TDBG_MAX_FILTERS];
  double fs_scale[TDBG_MAX_FILTERS];   // FLOAT_SCALE stages: FilterConfig scale / offset
  double fs_offset[TDBG_MAX_FILTERS];
};

#define TDBG_E_FALLBACK 100  // internal status: the fast path declined the tile
#define TDBG_PROF_PHASES 16 // fused-kernel phase clocks per workgroup

enum tdbg_fast_kind : uint32_t {
  TDBG_FAST_NONE = 0,
};

// device path counters (KParams::stats), cumulative per context
enum tdbg_stat_slot : uint32_t {
  TDBG_STAT_FUSED_TILES = 0,    // tiles the fused LDS kernel unfiltered (status OK)
  TDBG_STAT_FUSED_BYTES = 1,    // their unfiltered bytes
  TDBG_STAT_FALLBACK = 2,       // tiles the fused kernel declined (re-run by the fixup)
  TDBG_STAT_GENERAL_TILES = 3,  // tiles the general interpreter unfiltered (status OK)
  TDBG_STAT_GENERAL_BYTES = 4,
  TDBG_STAT_STREAM_TILES = 5,   // of the fused tiles: those the streaming C5 kernels took (tdbg_stream*.hip)
  TDBG_STAT_STREAM_RAW_TILES = 6,  // of those: the raw-DoubleDelta kernel's (tdbg_stream_raw.hip)
  TDBG_STAT_FWD_STREAM_TILES = 7,  // forward: tiles the LDS-resident C5 kernel filtered (tdbg_forward_stream.hip)
  TDBG_STAT_STREAM_CHUNKS = 8,  // chunk-parallel launches: chunks the streaming kernels took
  TDBG_STAT_TILE_CHUNKS = 9,    // tile mode: chunks of multi-chunk tiles the C5 tile kernel took
  TDBG_STAT_N = 10
};
// The counters live in slots of TDBG_STAT_STRIDE u64 (one 128-B line each):
// slot 0 takes the persistent kernels' one add per workgroup, slots 1..64 the
// one-workgroup-per-tile kernels' (workgroup b adds to slot 1 + (b & 63), so
// a 100,000-workgroup launch spreads its atomics over 64 lines); the host
// sums the slots (tdbg_host.cpp read_stats).
#define TDBG_STAT_STRIDE 16
#define TDBG_STAT_SLOTS 65
static_assert(TDBG_STAT_N <= TDBG_STAT_STRIDE, "stat slot");

// host-side internals shared by tdbg_host.cpp and tdbg_cpu.cpp
struct tdbg_pipeline;
const tdbg_plan* tdbg_internal_plan(const tdbg_pipeline* p);  // null if unsupported
void tdbg_internal_set_error(const char* msg);                // tdbg_last_error text

namespace tdbg {
// One chunk of the device chunk directory (Tile::load_chunk_data,
// tile.cc:280-313, built on the device for every tile of a launch)
struct ChunkRec {
  uint32_t tile;      // index into the launch's tile arrays
  uint32_t ml, fl;    // chunk metadata / filtered data bytes
  uint32_t orig;      // unfiltered bytes
  uint64_t in_off;    // byte offset of the chunk's metadata in the filtered tile
  uint64_t out_off;   // byte offset of the chunk's output in the tile
};

// kernel parameters (passed by value)
struct KParams {
  const uint8_t* const* in;
  const uint64_t* in_size;
  uint8_t* const* out;
  const uint64_t* out_size;
  int32_t* status;
  uint64_t* need;            // per-tile scratch requirement on TDBG_E_SCRATCH
  const uint32_t* tile_list; // optional indirection (retry pass)
  uint64_t ntiles;
  uint32_t flags;
  uint8_t* scratch;
  uint64_t slot_bytes;
  uint32_t slot_cap, md_cap, tab_cap;
  uint32_t dbg_stop;  // timing-only ablation: stop after N fast stages (0 = off)
  uint32_t fixup;     // general kernel: only the tiles queued in fbq (TDBG_E_FALLBACK)
  // Fallback queue of this launch: fbq[0] = count, fbq[1 + k] = tile index,
  // k < fbq_cap (= ntiles: a tile is queued at most once per launch).  The
  // host zeroes the count on the launch stream right before the fused
  // kernel, so a queue never carries entries across launches; the fused
  // kernel appends the tiles it declines, the fixup launch walks the queue.
  uint32_t* fbq;
  uint32_t fbq_cap;
  // Device path counters (cumulative per context, TDBG_STAT_*): one atomic
  // add per workgroup at exit.
  uint64_t* stats;
  uint64_t* prof;     // diagnostics: per-workgroup phase clocks (TDBG_PROF_PHASES), or null
  // forward (filter) launches: per-tile filtered length out, Tile::cell_size
  // and WriterTile's max chunk size (0 = 64 KiB) for compute_chunk_size
  uint64_t* out_len;
  uint64_t cell_size;
  uint32_t max_chunk;
  // chunk-parallel launches: the device chunk directory (chunks[k], k <
  // *nchunks) replaces the tile loop of the fused kernel
  const ChunkRec* chunks;
  const uint32_t* nchunks;
  // Streaming C5 kernel (tdbg_stream.hip): the tiles it does not take go to
  // sq (sq[0] = count, sq[1 + k] = tile index, k < sq_cap); the fused kernel
  // then runs on that list with its length read on the device (ntiles_dev,
  // capped by ntiles).
  uint32_t* sq;
  uint32_t sq_cap;
  const uint32_t* ntiles_dev;
  tdbg_plan plan;
};


}  // namespace tdbg
