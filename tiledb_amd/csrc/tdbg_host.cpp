// tdbg_host.cpp -- host orchestration + C-ABI of the MI355X unfilter engine.
//
// Replaces, on the read path, ReaderBase::unfilter_tiles' CPU loop
// (tiledb/sm/query/readers/reader_base.cc:905-989) over
// FilterPipeline::run_reverse (filter_pipeline.cc:439-517).  The pipeline
// descriptor is parsed exactly as FilterPipeline::deserialize
// (filter_pipeline.cc:544-557) / FilterCreate::deserialize
// (filter_create.cc:100-201), datatypes are chained as in
// FilterPipeline(other, on_disk_type) (filter_pipeline.cc:80-88), and each
// filter is resolved to a device stage kind with the widths the reference
// picks at run time.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tiledb_amd.h"
#include "tdbg_desc.h"
#include "tdbg_launch.h"
#include "tdbg_hooks.h"

namespace tdbg {
thread_local EvArm ev_arm{nullptr, nullptr};  // tdbg_launch.h
}

extern "C" hipError_t tdbg_launch_general(const tdbg::KParams* kp, uint32_t grid,
                                          hipStream_t stream);
extern "C" hipError_t tdbg_launch_fixup(const tdbg::KParams* kp, uint32_t grid,
                                        hipStream_t stream);
extern "C" hipError_t tdbg_launch_filter(const tdbg::KParams* kp, uint32_t grid, hipStream_t stream);
extern "C" hipError_t tdbg_launch_filter_c5(const tdbg::KParams* kp, uint32_t grid, int sgn, int tile,
                                           hipStream_t s);
extern "C" hipError_t tdbg_launch_filter_small(const tdbg::KParams* kp, uint32_t grid, int mode, int sgn,
                                               hipStream_t s);
extern "C" hipError_t tdbg_launch_filter_shuffle4(const tdbg::KParams* kp, uint32_t grid, int mode, int sgn,
                                                  hipStream_t s);
extern "C" hipError_t tdbg_launch_chunk_dir(const tdbg::KParams* kp, uint32_t* cnt, uint32_t* base,
                                            tdbg::ChunkRec* recs, uint32_t cap, uint32_t* total,
                                            uint64_t* need, uint32_t* cq, hipStream_t stream);
extern "C" hipError_t tdbg_launch_extra_offset(uint64_t ntiles, uint8_t* const* out, const uint64_t* out_size,
                                               const uint64_t* var_size, const int32_t* status,
                                               hipStream_t stream);
#define TDBG_NPART_HOST 6  // = TDBG_NPART of the build (tiledb_amd/build.py)
#define TDBG_DECL_PART(k) \
  extern "C" hipError_t tdbg_launch_fast_part##k(const tdbg::KParams* kp, uint32_t grid, hipStream_t stream);
TDBG_DECL_PART(0)
TDBG_DECL_PART(1)
TDBG_DECL_PART(2)
TDBG_DECL_PART(3)
TDBG_DECL_PART(4)
TDBG_DECL_PART(5)
static hipError_t tdbg_launch_fast(const tdbg::KParams* kp, uint32_t grid, hipStream_t stream) {
  static hipError_t (*const parts[TDBG_NPART_HOST])(const tdbg::KParams*, uint32_t, hipStream_t) = {
      tdbg_launch_fast_part0, tdbg_launch_fast_part1, tdbg_launch_fast_part2,
      tdbg_launch_fast_part3, tdbg_launch_fast_part4, tdbg_launch_fast_part5};
  return parts[kp->plan.fast % TDBG_NPART_HOST](kp, grid, stream);
}
extern "C" uint32_t tdbg_fast_select(const tdbg_plan* plan);
#ifdef TDBG_EXPERIMENTS
// the retired round-4 C5 streaming kernels (experiments library only: A/B
// through TDBG_C5_OLD_RAW)
extern "C" hipError_t tdbg_launch_stream(const tdbg::KParams* kp, uint32_t grid, int sgn, hipStream_t s);
extern "C" uint32_t tdbg_stream_grid(int cus);
extern "C" hipError_t tdbg_launch_stream_raw(const tdbg::KParams* kp, uint32_t grid, int sgn, hipStream_t s);
extern "C" uint32_t tdbg_stream_raw_grid(int cus);
#endif
extern "C" hipError_t tdbg_launch_c5tile(const tdbg::KParams* kp, int sgn, int mc, hipStream_t s);
extern "C" hipError_t tdbg_launch_c2tile(const tdbg::KParams* kp, int mode, int sgn, hipStream_t s);
extern "C" hipError_t tdbg_launch_stream_small(const tdbg::KParams* kp, uint32_t grid, int mode, int sgn,
                                               hipStream_t s);
extern "C" hipError_t tdbg_launch_stream_small_512(const tdbg::KParams* kp, uint32_t grid, int mode, int sgn,
                                                  hipStream_t s);
extern "C" hipError_t tdbg_launch_stream_small_256np(const tdbg::KParams* kp, uint32_t grid, int mode, int sgn,
                                                    hipStream_t s);
extern "C" uint32_t tdbg_stream_small_grid(int cus, int mode);
extern "C" hipError_t tdbg_launch_stream_shuffle4(const tdbg::KParams* kp, hipStream_t s);
extern "C" hipError_t tdbg_launch_dense_frag_copy(const tdbg_dense_frag_config* fc, uint64_t ntiles,
                                                  const int64_t* tile_start, const int64_t* frag_dom,
                                                  const uint8_t* const* tiles, const uint8_t* const* validity,
                                                  const uint8_t* fill, uint8_t* result, uint8_t* result_validity,
                                                  uint64_t ncells, uint32_t grid, hipStream_t s);
extern "C" hipError_t tdbg_launch_dense_var_offsets(const tdbg_dense_frag_config* fc, uint64_t ntiles,
                                                    const int64_t* tile_start, const int64_t* frag_dom,
                                                    const uint8_t* const* off_tiles, const uint8_t* const* var_tiles,
                                                    const uint8_t* const* validity, const uint8_t* fill,
                                                    uint64_t* offsets, uint64_t ncells, uint64_t* src,
                                                    uint8_t* result_validity, uint64_t* bsum, uint64_t* total,
                                                    uint32_t* err, uint32_t grid, hipStream_t s);
extern "C" hipError_t tdbg_launch_dense_var_copy(const uint64_t* offsets, const uint64_t* src, uint64_t ncells,
                                                 const uint64_t* total, uint64_t mult, uint8_t* var_out,
                                                 uint32_t grid, hipStream_t s);
extern "C" hipError_t tdbg_launch_dense_copy(const tdbg_dense_copy_config* cfg, uint64_t ntiles,
                                             const int64_t* tile_start, const uint8_t* const* tiles,
                                             const int32_t* status, uint8_t* result, uint32_t grid,
                                             hipStream_t s);
extern "C" uint32_t tdbg_fast_grid(uint32_t fast, int cus);

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_OK(expr)                                                        \
  do {                                                                      \
    hipError_t e_ = (expr);                                                 \
    if (e_ != hipSuccess)                                                   \
      return fail(TDBG_E_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

// ---- datatypes (tiledb/sm/enums/datatype.h:67-140) -------------------------
uint32_t dt_size(uint8_t dt) {
  switch (dt) {
    case TDBG_INT32: case TDBG_FLOAT32: case TDBG_UINT32:
    case TDBG_STRING_UTF32: case TDBG_STRING_UCS4:
      return 4;
    case TDBG_INT64: case TDBG_FLOAT64: case TDBG_UINT64:
      return 8;
    case TDBG_INT16: case TDBG_UINT16: case TDBG_STRING_UTF16: case TDBG_STRING_UCS2:
      return 2;
    default:
      return (dt >= 18 && dt <= 39) ? 8 : 1;
  }
}
bool is_dt_time(uint8_t dt) { return dt >= 18 && dt <= 39; }

struct Filter {
  uint8_t type = 0;
  uint8_t compressor = 0;
  int32_t level = 0;
  uint8_t reinterpret = TDBG_ANY;
  uint32_t window = 0;
  uint8_t datatype = 0;
  double scale = 1.0, offset = 0.0;  // FLOAT_SCALE FilterConfig (float_scaling_filter.h:61-65)
  uint64_t byte_width = 8;
};

uint8_t compressor_filter(uint8_t c) {
  static const uint8_t m[] = {TDBG_FILTER_NONE, TDBG_FILTER_GZIP, TDBG_FILTER_ZSTD,
                              TDBG_FILTER_LZ4, TDBG_FILTER_RLE, TDBG_FILTER_BZIP2,
                              TDBG_FILTER_DOUBLE_DELTA, TDBG_FILTER_DICTIONARY,
                              TDBG_FILTER_DELTA};
  return c < sizeof(m) ? m[c] : 0xff;
}

}  // namespace

struct tdbg_pipeline {
  uint32_t max_chunk_size = 0;
  uint32_t version = 0;
  uint8_t on_disk_type = 0;
  uint64_t cell_size = 0;
  std::vector<Filter> filters;
  tdbg_plan plan{};
  bool supported = true;
};

// for the CPU entry (tdbg_cpu.cpp): the resolved plan of a supported pipeline
const tdbg_plan* tdbg_internal_plan(const tdbg_pipeline* p) {
  return p && p->supported ? &p->plan : nullptr;
}
void tdbg_internal_set_error(const char* msg) { g_err = msg; }

struct tdbg_context {
  int device = 0;
  int cus = 256;
  // general-path scratch (fixed slot sizes; the sync entry's TDBG_E_SCRATCH
  // retries use their own buffer, rscratch, so one oversized chunk never
  // inflates the slots of every later launch)
  uint8_t* scratch = nullptr;
  uint64_t scratch_bytes = 0;
  uint32_t slot_cap = 80 * 1024, md_cap = 16 * 1024, tab_cap = 32 * 1024;
  uint8_t* rscratch = nullptr;
  uint64_t rscratch_bytes = 0;
  // forward (filter) scratch slots
  uint8_t* fscratch = nullptr;
  uint64_t fscratch_bytes = 0;
  // device chunk directory (chunk-parallel launches): per-tile counts and
  // record bases, the records, the placed-record count
  uint32_t* dir_cnt = nullptr;
  uint32_t* dir_base = nullptr;
  tdbg::ChunkRec* dir_recs = nullptr;
  uint32_t* dir_total = nullptr;
  uint64_t dir_tiles = 0, dir_cap = 0;
  // records the largest launch so far asked for (host-mapped, written by the
  // directory pass): later launches size the directory from it
  volatile uint64_t* dir_need = nullptr;
  uint64_t* dir_need_dev = nullptr;
  // dense var reads: each result cell's source address (step 1 -> step 2)
  // and the scan's block sums
  uint64_t* dense_src = nullptr;
  uint64_t dense_src_cap = 0, dense_ncells = 0;
  uint64_t* dense_bsum = nullptr;
  uint32_t* dense_err = nullptr;  // set by the var sizes kernel: offsets outside their var tile
  uint8_t* dv_arena = nullptr;    // tdbg_dense_read_var_host's device buffers (grow-only)
  uint64_t dv_cap = 0;
  uint8_t* dv_extra = nullptr;    // its var result when overlapping offsets outgrow the carve (grow-only)
  uint64_t dv_extra_cap = 0;
  uint32_t fwd_retry_caps[3] = {0, 0, 0};  // diagnostics: largest retry slot
  // per-tile status / need
  int32_t* d_status = nullptr;
  uint64_t* d_need = nullptr;
  uint64_t status_cap = 0;
  uint32_t* d_list = nullptr;
  uint64_t list_cap = 0;
  // fused-kernel fallback queue (KParams::fbq): count + status_cap entries,
  // count zeroed on the launch stream before every fused launch
  uint32_t* d_fbq = nullptr;
  // streaming C5 kernel's queue (KParams::sq): the tiles it leaves to the
  // fused kernel, count + status_cap entries
  uint32_t* d_sq = nullptr;
  // chunk-mode streaming launches: the chunks the streaming kernels leave to
  // the fused kernel (count + cq_cap entries), cleared before every launch
  uint32_t* d_cq = nullptr;
  uint64_t cq_cap = 0;
  // d_sq[0] is 0 (the last streamed launch's fixup kernel reset it), so the
  // next streamed launch needs no memset for it
  bool sq_clean = true;
  // device path counters (KParams::stats, TDBG_STAT_*)
  uint64_t* d_stats = nullptr;
  // Launch ordering: scratch slots, the fallback queue and the status /
  // need arrays are per context, so a context's launches must not overlap.
  // Launches on one stream are ordered by the stream; when a launch comes on
  // a different stream than the previous one, the host first waits for the
  // previous stream (tdbg_order_stream).
  hipStream_t last_stream = nullptr;
  bool last_stream_set = false;
  int64_t last_te = -1;  // tev index of the last armed launch's events
  // armed per-launch timing (tdbg_context_time_launches): event triples
  // {before the fused/general kernel, after it, after the fixup launch}
  std::vector<hipEvent_t> tev;
  uint32_t tcap = 0, tcount = 0;
  uint64_t tiles_unfiltered = 0;  // tiles submitted (stats "tiles_unfiltered", reader_base.cc:1074)
  // host E2E staging
  struct Stage {
    uint8_t* d_in = nullptr;
    uint8_t* d_out = nullptr;
    uint64_t in_cap = 0, out_cap = 0;
    const uint8_t** h_ptrs = nullptr;  // pinned: in ptrs, sizes, out ptrs, sizes
    uint64_t ptr_cap = 0;
    void* d_ptrs = nullptr;
    int32_t* h_status = nullptr;
    int32_t* d_stat = nullptr;
    hipStream_t stream = nullptr;  // this slot's stream (one-tile scratch retries)
    hipEvent_t h2d = nullptr, kdone = nullptr, done = nullptr;
  } st[3];  // triple-buffered: H2D(b+1) and D2H(b-1) overlap kernel(b)
  hipStream_t cstream = nullptr;   // compute stream: kernels serialized (shared scratch)
  hipStream_t hstream = nullptr;   // every H2D of the host E2E path, in batch order
  hipStream_t dstream = nullptr;   // every D2H, in batch order (full-duplex PCIe with hstream)
  // diagnostics (TDBG_PROF=1): fused-kernel phase clocks of the last launch
  uint64_t* d_prof = nullptr;
  uint32_t prof_grid = 0;
};

namespace {

uint64_t slot_bytes(const tdbg_context* c) {
  return 2ull * c->slot_cap + 2ull * c->md_cap + c->tab_cap;
}

int ensure_scratch(tdbg_context* c, uint32_t grid) {
  const uint64_t need = slot_bytes(c) * grid;
  if (need <= c->scratch_bytes) return TDBG_OK;
  if (c->scratch) HIP_OK(hipFree(c->scratch));
  c->scratch = nullptr;
  c->scratch_bytes = 0;
  HIP_OK(hipMalloc(&c->scratch, need));
  c->scratch_bytes = need;
  return TDBG_OK;
}

// Serialize a context's launches across streams (see tdbg_context::last_stream).
int order_stream(tdbg_context* c, hipStream_t s) {
  if (c->last_stream_set && c->last_stream != s) HIP_OK(hipStreamSynchronize(c->last_stream));
  c->last_stream = s;
  c->last_stream_set = true;
  return TDBG_OK;
}

int ensure_status(tdbg_context* c, uint64_t n) {
  if (n <= c->status_cap) return TDBG_OK;
  if (c->d_status) HIP_OK(hipFree(c->d_status));
  if (c->d_need) HIP_OK(hipFree(c->d_need));
  if (c->d_fbq) HIP_OK(hipFree(c->d_fbq));
  if (c->d_sq) HIP_OK(hipFree(c->d_sq));
  c->d_status = nullptr;
  c->d_need = nullptr;
  c->d_fbq = nullptr;
  c->d_sq = nullptr;
  c->status_cap = 0;
  HIP_OK(hipMalloc(&c->d_status, n * sizeof(int32_t)));
  HIP_OK(hipMalloc(&c->d_need, n * sizeof(uint64_t)));
  HIP_OK(hipMalloc(&c->d_fbq, (n + 1) * sizeof(uint32_t)));
  HIP_OK(hipMemset(c->d_fbq, 0, sizeof(uint32_t)));
  HIP_OK(hipMalloc(&c->d_sq, (n + 1) * sizeof(uint32_t)));
  HIP_OK(hipMemset(c->d_sq, 0, sizeof(uint32_t)));
  c->sq_clean = true;
  c->status_cap = n;
  return TDBG_OK;
}

// Resolve filters to device stages (the run-time datatype switches of the
// reference): bit_width_reduction_filter.cc:288-350,
// positive_delta_filter.cc:262-322, dd_compressor.cc:131-200,
// compression_filter.cc:303-486.
void build_plan(tdbg_pipeline* p) {
  tdbg_plan& P = p->plan;
  memset(&P, 0, sizeof(P));
  P.nstages = (uint32_t)p->filters.size();
  p->supported = P.nstages <= TDBG_MAX_FILTERS;
  for (uint32_t i = 0; i < P.nstages && i < TDBG_MAX_FILTERS; i++) {
    const Filter& f = p->filters[i];
    tdbg_stage& s = P.s[i];
    const uint8_t dt = f.datatype;
    s.dts = (uint8_t)dt_size(dt);
    switch (f.type) {
      case TDBG_FILTER_NONE:
        s.kind = TDBG_K_PASS;
        break;
      case TDBG_FILTER_BYTESHUFFLE:
        s.kind = TDBG_K_BYTESHUFFLE;
        s.w = (uint8_t)dt_size(dt);
        break;
      case TDBG_FILTER_BITSHUFFLE:
        s.kind = TDBG_K_BITSHUFFLE;
        s.w = (uint8_t)dt_size(dt);
        break;
      case TDBG_FILTER_SCALE_FLOAT: {  // float_scaling_filter.cc:217-238: float/double in
        const uint64_t ts = dt_size(dt), bw = f.byte_width;
        if ((ts == 4 || ts == 8) && (bw == 1 || bw == 2 || bw == 4 || bw == 8)) {
          s.kind = TDBG_K_FSCALE;
          s.w = (uint8_t)bw;
          P.fs_scale[i] = f.scale;
          P.fs_offset[i] = f.offset;
        } else {
          s.kind = TDBG_K_UNSUPPORTED;
          p->supported = false;
        }
        break;
      }
      case TDBG_FILTER_XOR: {  // xor_filter.cc:179-218: integer of the type's width
        const uint64_t w = dt_size(dt);
        if (w == 1 || w == 2 || w == 4 || w == 8) {
          s.kind = TDBG_K_XOR;
          s.w = (uint8_t)w;
        } else {
          s.kind = TDBG_K_UNSUPPORTED;
          p->supported = false;
        }
        break;
      }
      case TDBG_FILTER_BIT_WIDTH_REDUCTION:
      case TDBG_FILTER_POSITIVE_DELTA: {
        const bool bwr = f.type == TDBG_FILTER_BIT_WIDTH_REDUCTION;
        int w = 0, sg = 0;
        switch (dt) {
          case TDBG_INT16: w = 2; sg = 1; break;
          case TDBG_UINT16: w = 2; break;
          case TDBG_INT32: w = 4; sg = 1; break;
          case TDBG_UINT32: w = 4; break;
          case TDBG_INT64: w = 8; sg = 1; break;
          case TDBG_UINT64: w = 8; break;
          case TDBG_INT8: if (!bwr) { w = 1; sg = 1; } break;
          case TDBG_UINT8: case TDBG_BLOB: case TDBG_GEOM_WKB: case TDBG_GEOM_WKT:
          case TDBG_BOOL: if (!bwr) w = 1; break;
          default:
            if (is_dt_time(dt) && p->version >= 20) { w = 8; sg = 1; }
        }
        if (w == 0) { s.kind = TDBG_K_PASS; break; }
        s.kind = bwr ? TDBG_K_BWR : TDBG_K_PD;
        s.w = (uint8_t)w;
        s.sgn = (uint8_t)sg;
        s.window = f.window;
        break;
      }
      case TDBG_FILTER_DOUBLE_DELTA: case TDBG_FILTER_RLE: case TDBG_FILTER_GZIP:
      case TDBG_FILTER_ZSTD: case TDBG_FILTER_LZ4: case TDBG_FILTER_BZIP2:
      case TDBG_FILTER_DICTIONARY: case TDBG_FILTER_DELTA:
        if (f.compressor == TDBG_COMPRESSOR_NONE) {
          s.kind = TDBG_K_PASS;
        } else if (f.compressor == TDBG_COMPRESSOR_RLE) {
          if ((dt == TDBG_STRING_ASCII || dt == TDBG_STRING_UTF8) && p->version >= 12) {
            // var-string RLE (compression_filter.cc:331-338) is only taken
            // with an offsets tile; fixed-size RLE otherwise.  Still fixed.
          }
          s.kind = TDBG_K_RLE;
          s.cs = p->cell_size;
          if (p->cell_size == 0) { s.kind = TDBG_K_UNSUPPORTED; p->supported = false; }
        } else if (f.compressor == TDBG_COMPRESSOR_DOUBLE_DELTA ||
                   f.compressor == TDBG_COMPRESSOR_DELTA) {
          // Delta::decompress (delta_compressor.cc:139-217) uses DoubleDelta's type table
          s.kind = f.compressor == TDBG_COMPRESSOR_DELTA ? TDBG_K_DELTA : TDBG_K_DD;
          const uint8_t t = f.reinterpret != TDBG_ANY ? f.reinterpret : dt;
          switch (t) {
            case TDBG_FLOAT32: case TDBG_FLOAT64: s.w = 0; break;  // DD_TYPE at run time
            default: s.w = (uint8_t)(t <= 43 ? dt_size(t) : 0);
          }
          if (t == TDBG_STRING_ASCII || t == TDBG_STRING_UTF8 || t == TDBG_STRING_UTF16 ||
              t == TDBG_STRING_UTF32 || t == TDBG_STRING_UCS2 || t == TDBG_STRING_UCS4 ||
              t == TDBG_ANY)
            s.w = 1;  // DoubleDelta::decompress<uint8_t> (dd_compressor.cc:187-194)
          // signedness of T (the forward pass's checked deltas, dd_compressor.cc:63-127)
          s.sgn = (t == TDBG_INT8 || t == TDBG_CHAR || t == TDBG_INT16 || t == TDBG_INT32 ||
                   t == TDBG_INT64 || is_dt_time(t)) ? 1 : 0;
        } else {
          s.kind = TDBG_K_UNSUPPORTED;
          p->supported = false;
        }
        break;
      default:
        s.kind = TDBG_K_UNSUPPORTED;
        p->supported = false;
    }
  }
  P.fast = p->supported ? tdbg_fast_select(&P) : 0;
}

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

size_t tdbg_last_error(char* buf, size_t cap) {
  if (!buf || cap == 0) return g_err.size();
  const size_t n = std::min(cap - 1, g_err.size());
  memcpy(buf, g_err.data(), n);
  buf[n] = 0;
  return n;
}

const char* tdbg_status_str(int s) {
  switch (s) {
    case TDBG_OK: return "ok";
    case TDBG_E_ARG: return "invalid argument";
    case TDBG_E_TILE_FORMAT: return "Tile chunk directory exceeds the filtered tile";
    case TDBG_E_TILE_SIZE: return "Incorrect unfiltered tile size allocated.";
    case TDBG_E_MD_READ: return "FilterBuffer error; could not read requested byte count.";
    case TDBG_E_DATA_READ: return "Filter input too short for its metadata";
    case TDBG_E_OUT_FULL: return "FilterBuffer error; could not write: buffer is full.";
    case TDBG_E_RLE_FORMAT: return "Failed decompressing with RLE; invalid input buffer format";
    case TDBG_E_DD_TYPE: return "DoubleDelta tile decompression is not yet supported for float types.";
    case TDBG_E_BWR_BITS: return "Bit width reduction: invalid compressed bit width";
    case TDBG_E_UNSUPPORTED: return "Filter not supported by the MI355X engine";
    case TDBG_E_SCRATCH: return "internal: scratch too small";
    case TDBG_E_PD_DECREASING: return "Positive delta filter error: delta is not positive.";
    case TDBG_E_DD_OVERFLOW: return "Cannot compress with DoubleDelta: delta exceeds range of int64_t";
    case TDBG_E_DEVICE: return "HIP runtime error";
    case TDBG_E_DESCRIPTOR: return "Deserialization error; malformed filter pipeline";
    case TDBG_E_DELTA_TYPE: return "Decompression is not yet supported for float datatypes.";
    case TDBG_E_INTERNAL: return "internal: device work queue overflow";
    case TDBG_E_IO: return "tile read failed (short read or I/O error)";
    case TDBG_E_NOT_RUN: return "tile not processed: the call stopped on an earlier error";
    default: return "unknown";
  }
}

int tdbg_pipeline_create(const uint8_t* b, size_t len, uint32_t version,
                         uint8_t datatype, uint64_t cell_size, tdbg_pipeline** out) {
  if (!b || !out) return fail(TDBG_E_ARG, "tdbg_pipeline_create: null argument");
  auto p = new tdbg_pipeline();
  size_t o = 0;
  auto need = [&](size_t k) { return o + k <= len; };
  auto rd32 = [&](size_t at) { uint32_t v; memcpy(&v, b + at, 4); return v; };
  if (!need(8)) { delete p; return fail(TDBG_E_DESCRIPTOR, "pipeline descriptor shorter than 8 bytes"); }
  p->max_chunk_size = rd32(0);
  const uint32_t nf = rd32(4);
  o = 8;
  p->version = version;
  p->on_disk_type = datatype;
  p->cell_size = cell_size;
  uint8_t cur = datatype;
  for (uint32_t i = 0; i < nf; i++) {
    if (!need(5)) { delete p; return fail(TDBG_E_DESCRIPTOR, "truncated filter header"); }
    Filter f;
    f.type = b[o];
    const uint32_t mdlen = rd32(o + 1);
    o += 5;
    if (len - o < mdlen) {
      delete p;
      return fail(TDBG_E_DESCRIPTOR, "Deserialization error; not enough data in buffer for metadata");
    }
    switch (f.type) {
      case TDBG_FILTER_NONE: break;
      case TDBG_FILTER_GZIP: case TDBG_FILTER_ZSTD: case TDBG_FILTER_LZ4: case TDBG_FILTER_RLE:
      case TDBG_FILTER_BZIP2: case TDBG_FILTER_DELTA: case TDBG_FILTER_DOUBLE_DELTA:
      case TDBG_FILTER_DICTIONARY: {
        if (!need(5)) { delete p; return fail(TDBG_E_DESCRIPTOR, "truncated compressor options"); }
        const uint8_t ftype = f.type;
        f.compressor = b[o];
        memcpy(&f.level, b + o + 1, 4);
        o += 5;
        if ((version >= 20 && ftype == TDBG_FILTER_DOUBLE_DELTA) ||
            (version >= 19 && ftype == TDBG_FILTER_DELTA)) {
          if (!need(1)) { delete p; return fail(TDBG_E_DESCRIPTOR, "truncated reinterpret type"); }
          f.reinterpret = b[o++];
        }
        f.type = compressor_filter(f.compressor);
        if (f.type == 0xff) { delete p; return fail(TDBG_E_DESCRIPTOR, "unknown compressor"); }
        break;
      }
      case TDBG_FILTER_BIT_WIDTH_REDUCTION: case TDBG_FILTER_POSITIVE_DELTA:
        if (!need(4)) { delete p; return fail(TDBG_E_DESCRIPTOR, "truncated window option"); }
        f.window = rd32(o);
        o += 4;
        break;
      case TDBG_FILTER_BITSHUFFLE: case TDBG_FILTER_BYTESHUFFLE: case TDBG_FILTER_AES_256_GCM:
      case TDBG_FILTER_CHECKSUM_MD5: case TDBG_FILTER_CHECKSUM_SHA256: case TDBG_FILTER_XOR:
        break;
      case TDBG_FILTER_SCALE_FLOAT:
        if (!need(24)) { delete p; return fail(TDBG_E_DESCRIPTOR, "truncated float scale config"); }
        memcpy(&f.scale, b + o, 8);
        memcpy(&f.offset, b + o + 8, 8);
        memcpy(&f.byte_width, b + o + 16, 8);
        o += 24;
        break;
      case TDBG_FILTER_WEBP:
        o += mdlen;
        break;
      default:
        delete p;
        return fail(TDBG_E_DESCRIPTOR, "Deserialization error; unknown type");
    }
    f.datatype = cur;
    if ((f.type == TDBG_FILTER_DOUBLE_DELTA || f.type == TDBG_FILTER_DELTA) &&
        f.reinterpret != TDBG_ANY)
      cur = f.reinterpret;  // CompressionFilter::output_datatype
    if (f.type == TDBG_FILTER_SCALE_FLOAT) {  // float_scaling_filter.cc:313-327
      switch (f.byte_width) {
        case 1: cur = TDBG_INT8; break;
        case 2: cur = TDBG_INT16; break;
        case 4: cur = TDBG_INT32; break;
        case 8: cur = TDBG_INT64; break;
        default: break;  // the reference throws; build_plan marks it unsupported
      }
    }
    if (f.type == TDBG_FILTER_XOR) {  // XORFilter::output_datatype xor_filter.cc:63-78
      switch (dt_size(cur)) {
        case 1: cur = TDBG_INT8; break;
        case 2: cur = TDBG_INT16; break;
        case 4: cur = TDBG_INT32; break;
        case 8: cur = TDBG_INT64; break;
        default: break;  // the reference throws; build_plan marks it unsupported
      }
    }
    p->filters.push_back(f);
  }
  build_plan(p);
  *out = p;
  return TDBG_OK;
}

void tdbg_pipeline_destroy(tdbg_pipeline* p) { delete p; }
int tdbg_pipeline_supported(const tdbg_pipeline* p) { return p && p->supported ? 1 : 0; }
uint32_t tdbg_pipeline_num_filters(const tdbg_pipeline* p) {
  return p ? (uint32_t)p->filters.size() : 0;
}
int tdbg_pipeline_filter(const tdbg_pipeline* p, uint32_t i, uint8_t* type, uint8_t* dt) {
  if (!p || i >= p->filters.size()) return fail(TDBG_E_ARG, "filter index out of range");
  if (type) *type = p->filters[i].type;
  if (dt) *dt = p->filters[i].datatype;
  return TDBG_OK;
}

int tdbg_context_create(int device, tdbg_context** out) {
  if (!out) return fail(TDBG_E_ARG, "null out");
  HIP_OK(hipSetDevice(device));
  auto c = new tdbg_context();
  c->device = device;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
    c->cus = cus;
  hipError_t e = hipMalloc(&c->d_stats, sizeof(uint64_t) * TDBG_STAT_STRIDE * TDBG_STAT_SLOTS);
  if (e == hipSuccess) e = hipMemset(c->d_stats, 0, sizeof(uint64_t) * TDBG_STAT_STRIDE * TDBG_STAT_SLOTS);
  if (e != hipSuccess) {
    if (c->d_stats) (void)hipFree(c->d_stats);
    delete c;
    return fail(TDBG_E_DEVICE, std::string("tdbg_context_create: ") + hipGetErrorString(e));
  }
  *out = c;
  return TDBG_OK;
}

void tdbg_context_destroy(tdbg_context* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();
  if (c->scratch) (void)hipFree(c->scratch);
  if (c->d_status) (void)hipFree(c->d_status);
  if (c->d_need) (void)hipFree(c->d_need);
  if (c->d_list) (void)hipFree(c->d_list);
  if (c->d_fbq) (void)hipFree(c->d_fbq);
  if (c->d_sq) (void)hipFree(c->d_sq);
  if (c->d_cq) (void)hipFree(c->d_cq);
  if (c->d_stats) (void)hipFree(c->d_stats);
  if (c->rscratch) (void)hipFree(c->rscratch);
  if (c->fscratch) (void)hipFree(c->fscratch);
  if (c->dir_cnt) (void)hipFree(c->dir_cnt);
  if (c->dir_base) (void)hipFree(c->dir_base);
  if (c->dir_recs) (void)hipFree(c->dir_recs);
  if (c->dir_total) (void)hipFree(c->dir_total);
  if (c->dir_need) (void)hipHostFree((void*)c->dir_need);
  if (c->dense_src) (void)hipFree(c->dense_src);
  if (c->dense_bsum) (void)hipFree(c->dense_bsum);
  if (c->dense_err) (void)hipFree(c->dense_err);
  if (c->dv_arena) (void)hipFree(c->dv_arena);
  if (c->dv_extra) (void)hipFree(c->dv_extra);
  for (auto& s : c->st) {
    if (s.d_in) (void)hipFree(s.d_in);
    if (s.d_out) (void)hipFree(s.d_out);
    if (s.d_ptrs) (void)hipFree(s.d_ptrs);
    if (s.h_ptrs) (void)hipHostFree(s.h_ptrs);
    if (s.h_status) (void)hipHostFree(s.h_status);
    if (s.d_stat) (void)hipFree(s.d_stat);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    if (s.h2d) (void)hipEventDestroy(s.h2d);
    if (s.kdone) (void)hipEventDestroy(s.kdone);
    if (s.done) (void)hipEventDestroy(s.done);
  }
  if (c->cstream) (void)hipStreamDestroy(c->cstream);
  if (c->hstream) (void)hipStreamDestroy(c->hstream);
  if (c->dstream) (void)hipStreamDestroy(c->dstream);
  if (c->d_prof) (void)hipFree(c->d_prof);
  for (auto e : c->tev) (void)hipEventDestroy(e);
  delete c;
}

static int launch(tdbg_context* c, const tdbg_pipeline* p, uint64_t ntiles,
                  const uint8_t* const* d_in, const uint64_t* d_in_size,
                  uint8_t* const* d_out, const uint64_t* d_out_size, uint32_t flags,
                  int32_t* d_status, uint64_t* d_need, const uint32_t* d_list,
                  hipStream_t stream, bool force_general) {
  if (ntiles == 0) return TDBG_OK;
  tdbg::KParams kp{};
  kp.in = d_in;
  kp.in_size = d_in_size;
  kp.out = d_out;
  kp.out_size = d_out_size;
  kp.status = d_status;
  kp.need = d_need;
  kp.tile_list = d_list;
  kp.ntiles = ntiles;
  kp.flags = flags;
  kp.plan = p->plan;
  {
    static const char* dbg = tdbg_hook("TDBG_DEBUG_STOP");  // timing-only ablation
    kp.dbg_stop = dbg ? (uint32_t)atoi(dbg) : 0;
  }
  const bool fast = !force_general && p->plan.fast != 0;
  uint32_t grid;
  if (fast) {
    grid = tdbg_fast_grid(p->plan.fast, c->cus);
    static const long fg = tdbg_hook_int("TDBG_FAST_GRID", 0);  // experiments: e.g. one tile per workgroup
    if (fg > 0) grid = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(ntiles, 1), (uint64_t)fg);
  } else {
    grid = (uint32_t)std::min<uint64_t>(ntiles, (uint64_t)c->cus * 8);
  }
  // Scratch slots serve the general interpreter (the general kernel, or the
  // fixup launch after the fused kernel); size them once, before enqueueing.
  const uint32_t ggrid = (uint32_t)std::min<uint64_t>(ntiles, (uint64_t)c->cus * 8);
  int rc = ensure_scratch(c, fast ? ggrid : grid);
  if (rc) return rc;
  kp.scratch = c->scratch;
  kp.slot_bytes = slot_bytes(c);
  kp.slot_cap = c->slot_cap;
  kp.md_cap = c->md_cap;
  kp.tab_cap = c->tab_cap;
  {
    static const bool prof = tdbg_hook("TDBG_PROF") != nullptr;
    if (prof && fast) {
      // (rows for every workgroup < 1024 of the tile kernels; the fused grid)
      const uint32_t pgrid = std::max<uint32_t>(grid, 1024u);
      if (c->prof_grid < pgrid) {
        if (c->d_prof) (void)hipFree(c->d_prof);
        c->d_prof = nullptr;
        c->prof_grid = 0;
        HIP_OK(hipMalloc(&c->d_prof, sizeof(uint64_t) * TDBG_PROF_PHASES * pgrid));
        c->prof_grid = pgrid;
      }
      HIP_OK(hipMemsetAsync(c->d_prof, 0, sizeof(uint64_t) * TDBG_PROF_PHASES * c->prof_grid, stream));
      kp.prof = c->d_prof;
    }
  }
  kp.stats = c->d_stats;
  const bool queued = fast && d_status && !kp.dbg_stop;
  if (queued) {
    if (ntiles > c->status_cap) return fail(TDBG_E_ARG, "internal: fallback queue smaller than the launch");
    kp.fbq = c->d_fbq;
    kp.fbq_cap = (uint32_t)ntiles;
  }
  // Chunk-parallel: asked for, or fewer tiles than CUs (tiles, not chunks,
  // would then bound the parallelism).  The directory pass runs first on
  // the same stream; its records feed the fused kernel.
  static const bool tile_mode = tdbg_hook("TDBG_DEBUG_TILE_MODE") != nullptr;  // ablation: no auto chunk mode
  // (TDBG_MULTI_CHUNK: the caller has tiles of several chunks; a launch of
  // fewer than two tiles per CU -- two workgroups of the C5 tile kernel fit
  // a CU -- then spreads their chunks through the directory, a bigger one
  // runs tile mode with the tile kernel's multi-chunk variant)
  const bool chunked = queued && !d_list &&
                       ((flags & TDBG_CHUNK_PARALLEL) ||
                        (!tile_mode && (ntiles < (uint64_t)c->cus ||
                                        ((flags & TDBG_MULTI_CHUNK) && ntiles < 2 * (uint64_t)c->cus))));
  // [BYTESHUFFLE] on 4-byte values (C1): the unit-parallel streaming kernel
  // (tdbg_stream_shuffle.hip) splits every one-chunk 64 KiB tile over 16
  // workgroups itself; batches of fewer tiles than CUs (e.g. a few
  // multi-chunk tiles, which that kernel declines) stay chunk-parallel
  const bool shuffle4 = !chunked && p->plan.fast == 1 && p->plan.nstages == 1 && p->plan.s[0].w == 4;
  // The headline pipeline [BYTESHUFFLE, DOUBLE_DELTA, BWR] on 4-byte
  // integers (fused specs 19/20) first goes through the streaming kernel
  // (tdbg_stream.hip); the fused kernel then runs on the tiles it left.
  static const bool no_stream = tdbg_hook("TDBG_NO_STREAM") != nullptr;  // ablation
#ifdef TDBG_EXPERIMENTS
  static const bool c5_old_raw = tdbg_hook("TDBG_C5_OLD_RAW") != nullptr;  // A/B: the persistent raw-DD kernel
#endif
  const bool c5_stream = (p->plan.fast == 19 || p->plan.fast == 20) && p->plan.nstages == 3 &&
                         p->plan.s[2].dts == 4 && p->plan.s[1].w == 4;
  // The scan pipelines of C3a / C3b / C4 on 8-byte values first go through
  // the small-image streaming kernel (tdbg_stream_small.hip): 0 [DD],
  // 1 [RLE] with 8-byte cells, 2 [PD, BWR]; -1 none.
  const tdbg_plan& P = p->plan;
  const int small_mode = (P.fast == 12 && P.nstages == 1 && P.s[0].w == 8)                     ? 0
                         : (P.fast == 14 && P.nstages == 1 && P.s[0].cs == 8)                  ? 1
                         : ((P.fast == 15 || P.fast == 16) && P.nstages == 2 && P.s[0].w == 8 &&
                            P.s[0].dts == 8 && P.s[1].w == 8 && P.s[1].dts == 8)               ? 2
                                                                                               : -1;
  // C2 [BITSHUFFLE] (+ a pass-through stage) and C2i [BITSHUFFLE, BWR] on
  // 4-byte values: the one-workgroup-per-tile kernel (tdbg_c2tile.hip),
  // 0 / 1; -1 none
  static const bool no_c2tile = tdbg_hook("TDBG_NO_C2TILE") != nullptr;  // A/B: the fused kernel alone
  const int c2_mode = (no_c2tile || chunked || P.fast == 0 || P.s[0].kind != TDBG_K_BITSHUFFLE || P.s[0].w != 4) ? -1
                      : (P.nstages == 1 || (P.nstages == 2 && P.s[1].kind == TDBG_K_PASS))            ? 0
                      : (P.nstages == 2 && P.s[1].kind == TDBG_K_BWR && P.s[1].w == 4 && P.s[1].dts == 4) ? 1
                                                                                                          : -1;
  const bool streamed =
      queued && !chunked && !d_list && !no_stream && (c5_stream || small_mode >= 0 || shuffle4 || c2_mode >= 0);
  // The fallback queue starts empty for this launch, whatever ran before on
  // any stream: a memset, or in a streamed launch the streaming kernel's first
  // thread (it runs before the fused kernel that appends).  The streaming
  // kernel's own queue count was reset by the last streamed launch's fixup
  // kernel (or is reset here): two memset launches fewer per C5 launch.
  // (chunked: the directory pass starts the queue counts)
  if (queued && !streamed && !chunked) HIP_OK(hipMemsetAsync(kp.fbq, 0, sizeof(uint32_t), stream));
  if (streamed && !c->sq_clean) HIP_OK(hipMemsetAsync(c->d_sq, 0, sizeof(uint32_t), stream));
  if (streamed) c->sq_clean = false;  // until this launch's fixup is enqueued
  if (chunked) {
    if (!c->dir_need) {
      void* h = nullptr;
      HIP_OK(hipHostMalloc(&h, sizeof(uint64_t), hipHostMallocMapped));
      c->dir_need = (volatile uint64_t*)h;
      *c->dir_need = 0;
      HIP_OK(hipHostGetDevicePointer((void**)&c->dir_need_dev, h, 0));
    }
    // 64 chunks per tile (4 MiB tiles of 64 KiB chunks), or what an earlier
    // launch asked for; a tile whose chunks still do not fit goes to the
    // general interpreter (correct, slower)
    const uint64_t asked = *c->dir_need;
    const uint64_t want = std::max<uint64_t>(std::max<uint64_t>(64 * ntiles, 4096), asked);
    if (ntiles > c->dir_tiles || want > c->dir_cap) {
      HIP_OK(hipStreamSynchronize(stream));  // earlier launches may still read the old directory
      if (ntiles > c->dir_tiles) {
        if (c->dir_cnt) HIP_OK(hipFree(c->dir_cnt));
        if (c->dir_base) HIP_OK(hipFree(c->dir_base));
        c->dir_cnt = nullptr;
        c->dir_base = nullptr;
        c->dir_tiles = 0;
        HIP_OK(hipMalloc(&c->dir_cnt, ntiles * 4));
        HIP_OK(hipMalloc(&c->dir_base, ntiles * 4));
        c->dir_tiles = ntiles;
      }
      if (want > c->dir_cap) {
        if (c->dir_recs) HIP_OK(hipFree(c->dir_recs));
        c->dir_recs = nullptr;
        c->dir_cap = 0;
        HIP_OK(hipMalloc(&c->dir_recs, want * sizeof(tdbg::ChunkRec)));
        c->dir_cap = want;
      }
    }
    if (!c->dir_total) HIP_OK(hipMalloc(&c->dir_total, 4));
    const bool cq_used = (c5_stream || small_mode >= 0) && !no_stream && !d_list;
    if (cq_used && c->cq_cap < c->dir_cap) {
      // the streaming kernels take the directory's chunk records; their
      // queue holds chunk indices
      HIP_OK(hipStreamSynchronize(stream));  // an earlier launch may still read the old queue
      if (c->d_cq) HIP_OK(hipFree(c->d_cq));
      c->d_cq = nullptr;
      c->cq_cap = 0;
      HIP_OK(hipMalloc(&c->d_cq, (c->dir_cap + 1) * sizeof(uint32_t)));
      c->cq_cap = c->dir_cap;
    }
    // (zeroes the fallback queue's and the chunk queue's counts first)
    hipError_t e = tdbg_launch_chunk_dir(&kp, c->dir_cnt, c->dir_base, c->dir_recs,
                                         (uint32_t)std::min<uint64_t>(c->dir_cap, 0xffffffffull), c->dir_total,
                                         c->dir_need_dev, cq_used ? c->d_cq : nullptr, stream);
    if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("chunk directory launch: ") + hipGetErrorString(e));
    kp.chunks = c->dir_recs;
    kp.nchunks = c->dir_total;
  }
  // the headline pipeline's streaming kernels on chunk records (chunk-parallel
  // launches of multi-chunk tiles, SURVEY 8(a) FilterPipeline::run_reverse's
  // loop over chunks, filter_pipeline.cc:439-517)
  const bool chunk_stream = chunked && (c5_stream || small_mode >= 0) && !no_stream && !d_list && c->d_cq != nullptr;
  hipEvent_t* te = c->tcount < c->tcap ? &c->tev[3 * c->tcount++] : nullptr;
  // Events only on armed launches (tdbg_context_time_launches), and bound to
  // the kernel dispatches themselves (tdbg_launch.h): te[0] = start of the
  // first kernel, te[1] = end of the fused/general kernel, te[2] = end of the
  // fixup.  Recorded as marker packets they cost ~4 us of stream time each.
  struct Disarm {  // no armed event outlives this launch (error returns included)
    ~Disarm() { tdbg::ev_arm = tdbg::EvArm{nullptr, nullptr}; }
  } disarm;
  // an armed event no dispatch took (ablations, no fixup): a marker packet
  auto settle = [&]() -> hipError_t {
    hipError_t r = hipSuccess;
    if (tdbg::ev_arm.start) r = hipEventRecord(tdbg::ev_arm.start, stream);
    if (r == hipSuccess && tdbg::ev_arm.stop) r = hipEventRecord(tdbg::ev_arm.stop, stream);
    tdbg::ev_arm = tdbg::EvArm{nullptr, nullptr};
    return r;
  };
  if (te) tdbg::ev_arm.start = te[0];
  hipError_t e = hipSuccess;
  static const bool skip_fused = tdbg_hook("TDBG_DEBUG_SKIP_FUSED") != nullptr;  // ablation
  static const bool skip_fixup = tdbg_hook("TDBG_DEBUG_SKIP_FIXUP") != nullptr;  // ablation
  if (chunk_stream) {
    const uint32_t cap = (uint32_t)std::min<uint64_t>(c->cq_cap, 0xffffffffull);
    tdbg::KParams ks = kp;
    ks.ntiles = cap;
    ks.ntiles_dev = c->dir_total;
    ks.sq = c->d_cq;
    ks.sq_cap = cap;
    ks.fbq = nullptr;  // (cleared before the directory pass, which may append)
    if (small_mode >= 0) {
      const int sgn = (small_mode == 2 && P.s[1].sgn) ? 1 : 0;
      if (!skip_fused)
        e = tdbg_launch_stream_small(&ks, tdbg_stream_small_grid(c->cus, small_mode), small_mode, sgn, stream);
      if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("small stream kernel launch: ") + hipGetErrorString(e));
    } else {
      const int sgn = p->plan.s[2].sgn ? 1 : 0;
#ifdef TDBG_EXPERIMENTS
      if (c5_old_raw) {
        if (!skip_fused) e = tdbg_launch_stream(&ks, tdbg_stream_grid(c->cus), sgn, stream);
        if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("stream kernel launch: ") + hipGetErrorString(e));
        if (!skip_fused) e = tdbg_launch_stream_raw(&ks, tdbg_stream_raw_grid(c->cus), sgn, stream);
      } else
#endif
      if (!skip_fused) {
        e = tdbg_launch_c5tile(&ks, sgn, 0, stream);
      }
      if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("raw stream kernel launch: ") + hipGetErrorString(e));
    }
    tdbg::KParams kf = kp;  // the fused kernel on the chunks they queued
    kf.ntiles = cap;
    kf.tile_list = c->d_cq + 1;
    kf.ntiles_dev = c->d_cq;
    if (te) tdbg::ev_arm.stop = te[1];
    if (!skip_fused) e = tdbg_launch_fast(&kf, grid, stream);
  } else if (streamed) {
    tdbg::KParams ks = kp;
    ks.sq = c->d_sq;
    ks.sq_cap = (uint32_t)ntiles;
    // the coded-DD kernel takes the tiles of at most its staging cap, the
    // raw-DD kernel the bigger ones; both queue what they decline
    if (shuffle4) {
      if (!skip_fused) e = tdbg_launch_stream_shuffle4(&ks, stream);
      if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("shuffle stream kernel launch: ") + hipGetErrorString(e));
    } else if (c2_mode >= 0) {
      if (!skip_fused) e = tdbg_launch_c2tile(&ks, c2_mode, c2_mode == 1 && P.s[1].sgn ? 1 : 0, stream);
      if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("bitshuffle tile kernel launch: ") + hipGetErrorString(e));
    } else if (small_mode >= 0) {
      const int sgn = (small_mode == 2 && P.s[1].sgn) ? 1 : 0;
      // One workgroup per tile: 256 threads for DD and PD + BWR (C3a 0.59 ->
      // 0.70-0.72, C4 0.69 -> 0.81), 512 for RLE (C3b 0.53 -> 0.68-0.70;
      // profiles/r05/small_np_ab.txt).  The persistent 256-thread kernel stays
      // for chunk-parallel launches (and A/B).
      static const bool small_p = tdbg_hook("TDBG_SMALL_P") != nullptr;                  // experiments
      static const long small_nt = tdbg_hook_int("TDBG_SMALL_NT", 0);                    // experiments: 256 / 512
      const bool w512 = small_nt ? small_nt == 512 : small_mode == 1;
      if (!skip_fused)
        e = small_p ? tdbg_launch_stream_small(&ks, tdbg_stream_small_grid(c->cus, small_mode), small_mode, sgn, stream)
            : w512  ? tdbg_launch_stream_small_512(&ks, 0, small_mode, sgn, stream)
                    : tdbg_launch_stream_small_256np(&ks, 0, small_mode, sgn, stream);
      if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("small stream kernel launch: ") + hipGetErrorString(e));
    } else {
      const int sgn = p->plan.s[2].sgn ? 1 : 0;
#ifdef TDBG_EXPERIMENTS
      if (c5_old_raw) {
        if (!skip_fused) e = tdbg_launch_stream(&ks, tdbg_stream_grid(c->cus), sgn, stream);
        if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("stream kernel launch: ") + hipGetErrorString(e));
        if (!skip_fused) e = tdbg_launch_stream_raw(&ks, tdbg_stream_raw_grid(c->cus), sgn, stream);
      } else
#endif
      if (!skip_fused) {
        e = tdbg_launch_c5tile(&ks, sgn, (flags & TDBG_MULTI_CHUNK) ? 1 : 0, stream);
      }
      if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("raw stream kernel launch: ") + hipGetErrorString(e));
    }
    tdbg::KParams kf = kp;  // the fused kernel on the streaming kernel's queue
    kf.tile_list = c->d_sq + 1;
    kf.ntiles_dev = c->d_sq;
    if (te) tdbg::ev_arm.stop = te[1];  // kernel time = the streaming kernels + the fused one
    static const int qgrid = tdbg_hook_int("TDBG_QGRID", 0);  // experiments: the fused grid on the queue
    if (!skip_fused) e = tdbg_launch_fast(&kf, qgrid > 0 ? std::min<uint32_t>(grid, (uint32_t)qgrid) : grid, stream);
  } else {
    if (te) tdbg::ev_arm.stop = te[1];
    if (!skip_fused) e = fast ? tdbg_launch_fast(&kp, grid, stream) : tdbg_launch_general(&kp, grid, stream);
  }
  if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("kernel launch: ") + hipGetErrorString(e));
  if (te) HIP_OK(settle());
  if (queued && !skip_fixup) {
    // tiles the fused kernel declined (queued in fbq, status TDBG_E_FALLBACK)
    // are redone by the general interpreter, same stream, no host round trip;
    // with an empty queue every workgroup exits after one load
    tdbg::KParams g = kp;
    g.fixup = 1;
    g.sq = streamed ? c->d_sq : nullptr;  // the fixup resets the streaming queue's count
    // After a streamed launch (tiles or chunk records) the queue holds only
    // tiles both fast kernels declined (malformed or unusual ones): a small
    // grid, whose dispatch is most of an empty fixup launch's cost
    static const int fxgrid = tdbg_hook_int("TDBG_FIXUP_GRID", 32);  // experiments
    const uint32_t fgrid = std::min<uint32_t>(ggrid, (streamed || chunk_stream) ? (uint32_t)fxgrid : (uint32_t)c->cus);
    if (te) tdbg::ev_arm.stop = te[2];
    e = tdbg_launch_fixup(&g, fgrid, stream);
    if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("fixup launch: ") + hipGetErrorString(e));
    if (streamed) c->sq_clean = true;
  }
  if (te) {
    if (!queued || skip_fixup) HIP_OK(hipEventRecord(te[2], stream));
    c->last_te = (int64_t)(te - c->tev.data());
  }
  return TDBG_OK;
}

int tdbg_unfilter_tiles_async(tdbg_context* c, const tdbg_pipeline* p, uint64_t ntiles,
                              const uint8_t* const* d_in, const uint64_t* d_in_size,
                              uint8_t* const* d_out, const uint64_t* d_out_size,
                              uint32_t flags, int32_t* d_status, tdbg_stream stream) {
  if (!c || !p) return fail(TDBG_E_ARG, "null context or pipeline");
  if (!p->supported) return fail(TDBG_E_UNSUPPORTED, "pipeline has a filter the engine does not run");
  if (ntiles && (!d_in || !d_in_size || !d_out || !d_out_size))
    return fail(TDBG_E_ARG, "null tile arrays");
  if (ntiles > 0xffffffffull) return fail(TDBG_E_ARG, "too many tiles in one call");
  HIP_OK(hipSetDevice(c->device));
  int rc = order_stream(c, (hipStream_t)stream);
  if (rc) return rc;
  rc = ensure_status(c, ntiles);
  if (rc) return rc;
  rc = launch(c, p, ntiles, d_in, d_in_size, d_out, d_out_size, flags,
              d_status ? d_status : c->d_status, c->d_need, nullptr, (hipStream_t)stream, false);
  if (rc) return rc;
  c->tiles_unfiltered += ntiles;
  return TDBG_OK;
}

int tdbg_unfilter_tiles_sync(tdbg_context* c, const tdbg_pipeline* p, uint64_t ntiles,
                             const uint8_t* const* d_in, const uint64_t* d_in_size,
                             uint8_t* const* d_out, const uint64_t* d_out_size,
                             uint32_t flags, int32_t* host_status, tdbg_stream stream) {
  if (!c || !p) return fail(TDBG_E_ARG, "null context or pipeline");
  if (!p->supported) return fail(TDBG_E_UNSUPPORTED, "pipeline has a filter the engine does not run");
  if (ntiles == 0) return TDBG_OK;
  if (!d_in || !d_in_size || !d_out || !d_out_size) return fail(TDBG_E_ARG, "null tile arrays");
  if (ntiles > 0xffffffffull) return fail(TDBG_E_ARG, "too many tiles in one call");
  HIP_OK(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  int rc = order_stream(c, s);
  if (rc) return rc;
  rc = ensure_status(c, ntiles);
  if (rc) return rc;
  rc = launch(c, p, ntiles, d_in, d_in_size, d_out, d_out_size, flags, c->d_status, c->d_need,
              nullptr, s, false);
  if (rc) return rc;
  std::vector<int32_t> st(ntiles);
  std::vector<uint64_t> need(ntiles);
  HIP_OK(hipMemcpyAsync(st.data(), c->d_status, ntiles * 4, hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(need.data(), c->d_need, ntiles * 8, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  // Resolve TDBG_E_SCRATCH tiles with the general interpreter and bigger
  // scratch slots; each pass discovers one more stage's size.
  for (int pass = 0; pass < 2 * TDBG_MAX_FILTERS + 2; pass++) {
    std::vector<uint32_t> list;
    uint64_t maxneed = 0;
    for (uint64_t i = 0; i < ntiles; i++)
      if (st[i] == TDBG_E_SCRATCH) { list.push_back((uint32_t)i); maxneed = std::max(maxneed, need[i]); }
    if (list.empty()) break;
    // retry-only slot sizes (the context's own slots keep their defaults):
    // the cap that was short is not known, so all three grow to the need
    const uint64_t grow = (std::max<uint64_t>(maxneed + maxneed / 4 + 256, 0) + 255) & ~255ull;
    if (grow > 0xffffffffull / 2) return fail(TDBG_E_SCRATCH, "chunk stage larger than 2 GiB");
    const uint32_t rslot = (uint32_t)std::max<uint64_t>(c->slot_cap, grow);
    const uint32_t rmd = (uint32_t)std::max<uint64_t>(c->md_cap, grow);
    const uint32_t rtab = (uint32_t)std::max<uint64_t>(c->tab_cap, grow);
    const uint64_t rslot_bytes = 2ull * rslot + 2ull * rmd + rtab;
    if (list.size() > c->list_cap) {
      if (c->d_list) HIP_OK(hipFree(c->d_list));
      c->d_list = nullptr;
      c->list_cap = 0;
      HIP_OK(hipMalloc(&c->d_list, list.size() * 4));
      c->list_cap = list.size();
    }
    HIP_OK(hipMemcpyAsync(c->d_list, list.data(), list.size() * 4, hipMemcpyHostToDevice, s));
    // few, big slots: at most 256 MiB of retry scratch (at least one slot)
    const uint64_t by_mem = std::max<uint64_t>(1, (256ull << 20) / rslot_bytes);
    const uint32_t grid = (uint32_t)std::min<uint64_t>(std::min<uint64_t>(list.size(), 64), by_mem);
    if (rslot_bytes * grid > c->rscratch_bytes) {
      HIP_OK(hipStreamSynchronize(s));
      if (c->rscratch) HIP_OK(hipFree(c->rscratch));
      c->rscratch = nullptr;
      c->rscratch_bytes = 0;
      HIP_OK(hipMalloc(&c->rscratch, rslot_bytes * grid));
      c->rscratch_bytes = rslot_bytes * grid;
    }
    tdbg::KParams kp{};
    kp.in = d_in; kp.in_size = d_in_size; kp.out = d_out; kp.out_size = d_out_size;
    kp.status = c->d_status; kp.need = c->d_need; kp.tile_list = c->d_list;
    kp.ntiles = list.size(); kp.flags = flags; kp.plan = p->plan;
    kp.scratch = c->rscratch; kp.slot_bytes = rslot_bytes;
    kp.slot_cap = rslot; kp.md_cap = rmd; kp.tab_cap = rtab;
    kp.stats = c->d_stats;
    hipError_t e = tdbg_launch_general(&kp, grid, s);
    if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("retry launch: ") + hipGetErrorString(e));
    HIP_OK(hipMemcpyAsync(st.data(), c->d_status, ntiles * 4, hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(need.data(), c->d_need, ntiles * 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
  }
  if (host_status) memcpy(host_status, st.data(), ntiles * 4);
  c->tiles_unfiltered += ntiles;
  for (uint64_t i = 0; i < ntiles; i++)
    if (st[i]) {
      char msg[160];
      snprintf(msg, sizeof(msg), "tile %llu: %s", (unsigned long long)i, tdbg_status_str(st[i]));
      return fail(st[i], msg);
    }
  return TDBG_OK;
}

// The counters as of this context's last launch: the copy is ordered on
// the stream of that launch (every launch of a context is ordered behind the
// previous one, order_stream), so other contexts and streams of the device
// keep running.
static int read_stats(const tdbg_context* c, uint64_t (&h)[TDBG_STAT_N]) {
  HIP_OK(hipSetDevice(c->device));
  const hipStream_t s = c->last_stream_set ? c->last_stream : nullptr;
  uint64_t all[TDBG_STAT_STRIDE * TDBG_STAT_SLOTS];
  HIP_OK(hipMemcpyAsync(all, c->d_stats, sizeof(all), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  for (int i = 0; i < TDBG_STAT_N; i++) {
    h[i] = 0;
    for (int k = 0; k < TDBG_STAT_SLOTS; k++) h[i] += all[TDBG_STAT_STRIDE * k + i];
  }
  return TDBG_OK;
}

// ---------------------------------------------------------------------------
// forward (filter) direction: FilterPipeline::run_forward
// ---------------------------------------------------------------------------
static uint64_t fwd_chunk_bound(uint64_t tile_size, uint64_t cell, uint32_t max_chunk) {
  const uint64_t mc = max_chunk ? max_chunk : 65536;
  uint64_t c = std::min<uint64_t>(mc, tile_size);
  c = c / (cell ? cell : 1) * (cell ? cell : 1);
  return std::max<uint64_t>(c, cell ? cell : 1);
}

// Worst-case filtered size, by walking the pipeline forward over one full
// chunk with every filter's largest growth: BWR / PD window metadata for
// one-element windows (bit_width_reduction_filter.cc:218-250: [u32 orig]
// [u32 nwin] + nwin x [T min][u8 bits][u32 bytes]; positive_delta_filter.cc:
// 183-205: [u32 nwin] + nwin x [T first][u32 bytes]) adding up over every
// such stage, shuffle / XOR / FLOAT_SCALE part tables, FLOAT_SCALE's width
// change, and the compression filters, which fold all earlier metadata into
// their data (compression_filter.cc:240-301) with DD / DELTA raw fallback
// headers (dd_compressor.cc:229-261) and RLE's (cell + 2) bytes per cell
// (rle_compressor.cc:51-101).  Parts per buffer are bounded by kParts.
uint64_t tdbg_filtered_bound(const tdbg_pipeline* p, uint64_t tile_size, uint32_t max_chunk) {
  if (!p) return 0;
  const uint64_t chunk = fwd_chunk_bound(tile_size, p->cell_size, max_chunk);
  const uint64_t nch = (tile_size + chunk - 1) / chunk + 1;
  constexpr uint64_t kParts = 4;
  uint64_t D = chunk, M = 0, MP = 0;  // data bytes, metadata bytes, metadata buffers
  for (const Filter& f : p->filters) {
    const uint64_t ts = dt_size(f.datatype);
    // (f.type of a compression filter is the one its compressor names,
    // resolved at parse time: a GZIP-typed filter carrying DOUBLE_DELTA is a
    // DOUBLE_DELTA stage here, one with compressor NONE a NONE stage)
    switch (f.type) {
      case TDBG_FILTER_BYTESHUFFLE: case TDBG_FILTER_BITSHUFFLE: case TDBG_FILTER_XOR:
        M += 4 + 8 * kParts;
        MP++;
        break;
      case TDBG_FILTER_SCALE_FLOAT:
        M += 4 + 8 * kParts;
        MP++;
        D = D / (ts ? ts : 1) * std::max<uint64_t>(f.byte_width, 1) + 8;
        break;
      case TDBG_FILTER_BIT_WIDTH_REDUCTION:
        M += 8 * kParts + (D / (ts ? ts : 1) + kParts) * (ts + 5);
        MP++;
        break;
      case TDBG_FILTER_POSITIVE_DELTA:
        M += 4 * kParts + (D / (ts ? ts : 1) + kParts) * (ts + 4);
        MP++;
        break;
      case TDBG_FILTER_DOUBLE_DELTA: case TDBG_FILTER_DELTA:
        D = M + D + 64 * (MP + kParts);
        M = 8 + 8 * (MP + kParts);
        MP = 1;
        break;
      case TDBG_FILTER_RLE: {
        const uint64_t cs = p->cell_size ? p->cell_size : 1;
        auto grow = [&](uint64_t x) { return x / cs * (cs + 2) + 2 * (cs + 2); };
        D = grow(M) + grow(D) + 64 * (MP + kParts);
        M = 8 + 8 * (MP + kParts);
        MP = 1;
        break;
      }
      default:
        break;  // NOOP / pass-through stages; unsupported pipelines never launch
    }
  }
  return 8 + nch * (12 + M + D) + 4096;
}

static int filter_launch(tdbg_context* c, const tdbg_pipeline* p, uint64_t n, const uint8_t* const* d_in,
                         const uint64_t* d_in_size, uint8_t* const* d_out, const uint64_t* d_out_cap,
                         uint64_t* d_out_len, uint32_t max_chunk, int32_t* d_status, uint64_t* d_need,
                         const uint32_t* d_list, uint8_t* scratch, uint64_t slot_bytes, uint32_t slot_cap,
                         uint32_t md_cap, uint32_t tab_cap, uint32_t grid, hipStream_t s) {
  tdbg::KParams kp{};
  kp.in = d_in;
  kp.in_size = d_in_size;
  kp.out = d_out;
  kp.out_size = d_out_cap;
  kp.out_len = d_out_len;
  kp.status = d_status;
  kp.need = d_need;
  kp.tile_list = d_list;
  kp.ntiles = n;
  kp.plan = p->plan;
  kp.cell_size = p->cell_size;
  kp.max_chunk = max_chunk;
  kp.scratch = scratch;
  kp.slot_bytes = slot_bytes;
  kp.slot_cap = slot_cap;
  kp.md_cap = md_cap;
  kp.tab_cap = tab_cap;
  // The headline pipeline [BYTESHUFFLE, DOUBLE_DELTA, BWR(256)] on INT32 /
  // UINT32 with one 64 KiB chunk per 64 KiB tile first goes through the
  // LDS-resident forward kernel (tdbg_forward_stream.hip); the tiles it does
  // not take (other sizes, alignments, capacities) are queued in the fused
  // fallback queue for the general forward kernel, which runs on the queue.
  static const bool no_fast = tdbg_hook("TDBG_NO_FWD_STREAM") != nullptr;  // ablation
  const tdbg_plan& P = p->plan;
  const bool c5 = !no_fast && !d_list && (P.fast == 19 || P.fast == 20) && P.nstages == 3 && P.s[0].w == 4 &&
                  P.s[1].w == 4 && P.s[2].w == 4 && P.s[2].dts == 4 && P.s[1].sgn == P.s[2].sgn &&
                  P.s[2].window == 256 && p->cell_size == 4 && (max_chunk == 0 || max_chunk >= 65536) &&
                  n <= c->status_cap;
  // The scan configs' pipelines on 8-byte values -- C3a [DOUBLE_DELTA]
  // (mode 0), C3b [RLE] with 8-byte cells (mode 1), C4 [POSITIVE_DELTA(1024),
  // BWR(256)] on uint64 (mode 2) -- with one
  // 64 KiB chunk per tile go through the LDS-resident small forward kernel
  // (tdbg_forward_small.hip) first, the same way
  const int fsmall = (no_fast || d_list || c5 || p->cell_size != 8 || (max_chunk != 0 && max_chunk < 65536) ||
                      n > c->status_cap)
                         ? -1
                     : (P.fast == 12 && P.nstages == 1 && P.s[0].w == 8)  ? 0
                     : (P.fast == 14 && P.nstages == 1 && P.s[0].cs == 8) ? 1
                     : ((P.fast == 15 || P.fast == 16) && P.nstages == 2 && P.s[0].kind == TDBG_K_PD &&
                        P.s[1].kind == TDBG_K_BWR && P.s[0].w == 8 && P.s[0].dts == 8 && P.s[1].w == 8 &&
                        P.s[1].dts == 8 && !P.s[0].sgn && !P.s[1].sgn && P.s[0].window == 1024 &&
                        P.s[1].window == 256)
                         ? 2
                         : -1;
  // C1 [BYTESHUFFLE] (mode 0), C2 [BITSHUFFLE] + pass-through BWR (mode 1)
  // and C2i [BITSHUFFLE, BWR(256)] (mode 2) on 4-byte values: the shuffle
  // forward kernel (tdbg_forward_shuffle.hip), the same way
  const bool sh_ok = !no_fast && !d_list && !c5 && p->cell_size == 4 && (max_chunk == 0 || max_chunk >= 65536) &&
                     n <= c->status_cap && P.s[0].w == 4;
  const int fshuf = !sh_ok ? -1
                    : (P.nstages == 1 && P.s[0].kind == TDBG_K_BYTESHUFFLE) ? 0
                    : (P.s[0].kind == TDBG_K_BITSHUFFLE &&
                       (P.nstages == 1 || (P.nstages == 2 && P.s[1].kind == TDBG_K_PASS)))
                        ? 1
                    : (P.nstages == 2 && P.s[0].kind == TDBG_K_BITSHUFFLE && P.s[1].kind == TDBG_K_BWR &&
                       P.s[1].w == 4 && P.s[1].dts == 4 && P.s[1].window == 256)
                        ? 2
                        : -1;
  // The shuffle and small forward kernels: one workgroup per tile (a grid of
  // the tiles rounded up to 8, XCD-contiguous) up to 2^22 tiles, else (and
  // for A/B) a persistent grid walking the tiles
  static const bool fwd_p = tdbg_hook("TDBG_FWD_P") != nullptr;  // experiments
  const bool fwd_np = !fwd_p && n <= (1ull << 22);
  const uint32_t np_grid = (uint32_t)(8 * ((std::max<uint64_t>(n, 1) + 7) / 8));
  hipError_t e = hipSuccess;
  if (fshuf >= 0) {
    HIP_OK(hipMemsetAsync(c->d_fbq, 0, sizeof(uint32_t), s));
    tdbg::KParams kf = kp;
    kf.fbq = c->d_fbq;
    kf.fbq_cap = (uint32_t)n;
    kf.stats = c->d_stats;
    // (C2i, BWR active: the persistent grid measured 1.5 % faster)
    const uint32_t fgrid = fwd_np && fshuf != 2 ? np_grid : (uint32_t)std::min<uint64_t>(n, (uint64_t)c->cus * 2);
    e = tdbg_launch_filter_shuffle4(&kf, fgrid, fshuf, fshuf == 2 && P.s[1].sgn ? 1 : 0, s);
    if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("forward shuffle launch: ") + hipGetErrorString(e));
    kp.tile_list = c->d_fbq + 1;  // the general kernel on the queue
    kp.ntiles_dev = c->d_fbq;
  }
  if (fsmall >= 0) {
    HIP_OK(hipMemsetAsync(c->d_fbq, 0, sizeof(uint32_t), s));
    tdbg::KParams kf = kp;
    kf.fbq = c->d_fbq;
    kf.fbq_cap = (uint32_t)n;
    kf.stats = c->d_stats;
    const uint32_t fgrid = fwd_np ? np_grid : (uint32_t)std::min<uint64_t>(n, (uint64_t)c->cus * (fsmall == 2 ? 3 : 4));
    e = tdbg_launch_filter_small(&kf, fgrid, fsmall, fsmall == 0 && P.s[0].sgn ? 1 : 0, s);
    if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("forward small launch: ") + hipGetErrorString(e));
    kp.tile_list = c->d_fbq + 1;  // the general kernel on the queue
    kp.ntiles_dev = c->d_fbq;
  }
  if (c5) {
    HIP_OK(hipMemsetAsync(c->d_fbq, 0, sizeof(uint32_t), s));
    tdbg::KParams kf = kp;
    kf.fbq = c->d_fbq;
    kf.fbq_cap = (uint32_t)n;
    kf.stats = c->d_stats;
    static const bool prof = tdbg_hook("TDBG_PROF") != nullptr;  // diagnostics: phase clocks
    // one 1024-thread workgroup per tile (tdbg_forward_stream.hip); the
    // persistent 512-thread grid stays as the A/B reference (experiments)
    static const bool persist = tdbg_hook("TDBG_FWD_PERSIST") != nullptr;
    const uint32_t fgrid = persist ? (uint32_t)std::min<uint64_t>(n, (uint64_t)c->cus * 2) : 512u;
    if (prof) {
      if (c->prof_grid < fgrid) {
        if (c->d_prof) (void)hipFree(c->d_prof);
        c->d_prof = nullptr;
        c->prof_grid = 0;
        HIP_OK(hipMalloc(&c->d_prof, sizeof(uint64_t) * TDBG_PROF_PHASES * fgrid));
        c->prof_grid = fgrid;
      }
      HIP_OK(hipMemsetAsync(c->d_prof, 0, sizeof(uint64_t) * TDBG_PROF_PHASES * c->prof_grid, s));
      kf.prof = c->d_prof;
    }
    e = tdbg_launch_filter_c5(&kf, fgrid, P.s[2].sgn ? 1 : 0, persist ? 0 : 1, s);
    if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("forward stream launch: ") + hipGetErrorString(e));
    kp.tile_list = c->d_fbq + 1;  // the general kernel on the queue
    kp.ntiles_dev = c->d_fbq;
  }
  // On a fast kernel's queue the general kernel sees only the tiles that
  // kernel declined (unusual shapes): a small grid, since dispatching the
  // full one costs ~28 us even when the queue is empty (C1 forward trace,
  // profiles/r04/c1_forward_trace_kernel_stats.csv)
  e = tdbg_launch_filter(&kp, kp.ntiles_dev ? std::min<uint32_t>(grid, 64) : grid, s);
  if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("filter launch: ") + hipGetErrorString(e));
  return TDBG_OK;
}

// forward scratch: per workgroup 2 data buffers (3 x chunk: RLE growth),
// 2 metadata buffers, a window / run table
static void fwd_caps(uint64_t chunk, uint32_t* slot, uint32_t* md, uint32_t* tab) {
  *slot = (uint32_t)(((3 * chunk + 4096) + 255) & ~255ull);
  *md = (uint32_t)(((chunk + 4096) + 255) & ~255ull);
  *tab = (uint32_t)(((8 * chunk + 256) + 255) & ~255ull);
}

int tdbg_filter_tiles_async(tdbg_context* c, const tdbg_pipeline* p, uint64_t ntiles,
                            const uint8_t* const* d_in, const uint64_t* d_in_size, uint8_t* const* d_out,
                            const uint64_t* d_out_cap, uint64_t* d_out_len, uint32_t max_chunk,
                            int32_t* d_status, tdbg_stream stream) {
  if (!c || !p) return fail(TDBG_E_ARG, "null context or pipeline");
  if (!p->supported) return fail(TDBG_E_UNSUPPORTED, "pipeline has a filter the engine does not run");
  if (ntiles == 0) return TDBG_OK;
  if (!d_in || !d_in_size || !d_out || !d_out_cap || !d_out_len)
    return fail(TDBG_E_ARG, "null tile arrays");
  if (ntiles > 0xffffffffull) return fail(TDBG_E_ARG, "too many tiles in one call");
  HIP_OK(hipSetDevice(c->device));
  int rc = order_stream(c, (hipStream_t)stream);
  if (rc) return rc;
  rc = ensure_status(c, ntiles);
  if (rc) return rc;
  const uint64_t chunk = fwd_chunk_bound(max_chunk ? max_chunk : 65536, p->cell_size, max_chunk);
  uint32_t sc, mc, tc;
  fwd_caps(chunk, &sc, &mc, &tc);
  const uint64_t sb = 2ull * sc + 2ull * mc + tc;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(ntiles, (uint64_t)c->cus * 8);
  if (sb * grid > c->fscratch_bytes) {
    HIP_OK(hipStreamSynchronize((hipStream_t)stream));
    if (c->fscratch) HIP_OK(hipFree(c->fscratch));
    c->fscratch = nullptr;
    c->fscratch_bytes = 0;
    HIP_OK(hipMalloc(&c->fscratch, sb * grid));
    c->fscratch_bytes = sb * grid;
  }
  rc = filter_launch(c, p, ntiles, d_in, d_in_size, d_out, d_out_cap, d_out_len, max_chunk,
                     d_status ? d_status : c->d_status, c->d_need, nullptr, c->fscratch, sb, sc, mc, tc, grid,
                     (hipStream_t)stream);
  return rc;
}

int tdbg_filter_tiles_sync(tdbg_context* c, const tdbg_pipeline* p, uint64_t ntiles,
                           const uint8_t* const* d_in, const uint64_t* d_in_size, uint8_t* const* d_out,
                           const uint64_t* d_out_cap, uint64_t* d_out_len, uint32_t max_chunk,
                           int32_t* host_status, tdbg_stream stream) {
  if (ntiles == 0) return TDBG_OK;
  if (!c) return fail(TDBG_E_ARG, "null context or pipeline");
  // the context's status buffer is (re)sized here, before its address is
  // taken: the async entry's own ensure_status would otherwise reallocate
  // it after the kernel was handed the old one, and the copy below would
  // read statuses no kernel wrote
  HIP_OK(hipSetDevice(c->device));
  int rc = ensure_status(c, ntiles);
  if (rc) return rc;
  rc = tdbg_filter_tiles_async(c, p, ntiles, d_in, d_in_size, d_out, d_out_cap, d_out_len, max_chunk,
                               c->d_status, stream);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  std::vector<int32_t> st(ntiles);
  std::vector<uint64_t> need(ntiles);
  HIP_OK(hipMemcpyAsync(st.data(), c->d_status, ntiles * 4, hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(need.data(), c->d_need, ntiles * 8, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  // TDBG_E_SCRATCH: a stage outgrew the default slots (tiny BWR/PD windows,
  // RLE of 1-byte cells ...); redo those tiles with retry-only slots
  for (int pass = 0; pass < 2 * TDBG_MAX_FILTERS + 2; pass++) {
    std::vector<uint32_t> list;
    uint64_t maxneed = 0;
    for (uint64_t i = 0; i < ntiles; i++)
      if (st[i] == TDBG_E_SCRATCH) { list.push_back((uint32_t)i); maxneed = std::max(maxneed, need[i]); }
    if (list.empty()) break;
    const uint64_t grow = ((maxneed + maxneed / 2 + 4096) + 255) & ~255ull;
    if (grow > 0xffffffffull / 4) return fail(TDBG_E_SCRATCH, "chunk stage larger than 1 GiB");
    const uint64_t chunk = fwd_chunk_bound(max_chunk ? max_chunk : 65536, p->cell_size, max_chunk);
    uint32_t sc, mc, tc;
    fwd_caps(chunk, &sc, &mc, &tc);
    sc = (uint32_t)std::max<uint64_t>(sc, grow);
    mc = (uint32_t)std::max<uint64_t>(mc, grow);
    tc = (uint32_t)std::max<uint64_t>(tc, grow);
    c->fwd_retry_caps[0] = std::max(c->fwd_retry_caps[0], sc);
    const uint64_t sb = 2ull * sc + 2ull * mc + tc;
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(list.size(), (256ull << 20) / sb));
    if (list.size() > c->list_cap) {
      if (c->d_list) HIP_OK(hipFree(c->d_list));
      c->d_list = nullptr;
      c->list_cap = 0;
      HIP_OK(hipMalloc(&c->d_list, list.size() * 4));
      c->list_cap = list.size();
    }
    HIP_OK(hipMemcpyAsync(c->d_list, list.data(), list.size() * 4, hipMemcpyHostToDevice, s));
    if (sb * grid > c->rscratch_bytes) {
      HIP_OK(hipStreamSynchronize(s));
      if (c->rscratch) HIP_OK(hipFree(c->rscratch));
      c->rscratch = nullptr;
      c->rscratch_bytes = 0;
      HIP_OK(hipMalloc(&c->rscratch, sb * grid));
      c->rscratch_bytes = sb * grid;
    }
    rc = filter_launch(c, p, list.size(), d_in, d_in_size, d_out, d_out_cap, d_out_len, max_chunk, c->d_status,
                       c->d_need, c->d_list, c->rscratch, sb, sc, mc, tc, grid, s);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(st.data(), c->d_status, ntiles * 4, hipMemcpyDeviceToHost, s));
    HIP_OK(hipMemcpyAsync(need.data(), c->d_need, ntiles * 8, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
  }
  if (host_status) memcpy(host_status, st.data(), ntiles * 4);
  for (uint64_t i = 0; i < ntiles; i++)
    if (st[i]) {
      char msg[160];
      snprintf(msg, sizeof(msg), "tile %llu: %s", (unsigned long long)i, tdbg_status_str(st[i]));
      return fail(st[i], msg);
    }
  return TDBG_OK;
}

int tdbg_context_stats(const tdbg_context* c, uint64_t* tiles, uint64_t* bytes) {
  if (!c) return fail(TDBG_E_ARG, "null context");
  uint64_t h[TDBG_STAT_N];
  int rc = read_stats(c, h);
  if (rc) return rc;
  if (tiles) *tiles = c->tiles_unfiltered;
  if (bytes) *bytes = h[TDBG_STAT_FUSED_BYTES] + h[TDBG_STAT_GENERAL_BYTES];
  return TDBG_OK;
}

int tdbg_context_path_stats(const tdbg_context* c, uint64_t* fused_tiles, uint64_t* fallback_tiles,
                            uint64_t* general_tiles) {
  if (!c) return fail(TDBG_E_ARG, "null context");
  uint64_t h[TDBG_STAT_N];
  int rc = read_stats(c, h);
  if (rc) return rc;
  if (fused_tiles) *fused_tiles = h[TDBG_STAT_FUSED_TILES];
  if (fallback_tiles) *fallback_tiles = h[TDBG_STAT_FALLBACK];
  if (general_tiles) *general_tiles = h[TDBG_STAT_GENERAL_TILES];
  return TDBG_OK;
}

int tdbg_context_stream_stats(const tdbg_context* c, uint64_t* stream_tiles) {
  if (!c) return fail(TDBG_E_ARG, "null context");
  uint64_t h[TDBG_STAT_N];
  int rc = read_stats(c, h);
  if (rc) return rc;
  if (stream_tiles) *stream_tiles = h[TDBG_STAT_STREAM_TILES];
  return TDBG_OK;
}

int tdbg_context_stream_chunk_stats(const tdbg_context* c, uint64_t* chunks) {
  if (!c) return fail(TDBG_E_ARG, "null context");
  uint64_t h[TDBG_STAT_N];
  int rc = read_stats(c, h);
  if (rc) return rc;
  if (chunks) *chunks = h[TDBG_STAT_STREAM_CHUNKS];
  return TDBG_OK;
}

int tdbg_context_tile_chunk_stats(const tdbg_context* c, uint64_t* chunks) {
  if (!c) return fail(TDBG_E_ARG, "null context");
  uint64_t h[TDBG_STAT_N];
  int rc = read_stats(c, h);
  if (rc) return rc;
  if (chunks) *chunks = h[TDBG_STAT_TILE_CHUNKS];
  return TDBG_OK;
}

int tdbg_context_forward_stream_stats(const tdbg_context* c, uint64_t* tiles) {
  if (!c) return fail(TDBG_E_ARG, "null context");
  uint64_t h[TDBG_STAT_N];
  int rc = read_stats(c, h);
  if (rc) return rc;
  if (tiles) *tiles = h[TDBG_STAT_FWD_STREAM_TILES];
  return TDBG_OK;
}

int tdbg_context_stream_raw_stats(const tdbg_context* c, uint64_t* raw_tiles) {
  if (!c) return fail(TDBG_E_ARG, "null context");
  uint64_t h[TDBG_STAT_N];
  int rc = read_stats(c, h);
  if (rc) return rc;
  if (raw_tiles) *raw_tiles = h[TDBG_STAT_STREAM_RAW_TILES];
  return TDBG_OK;
}

int tdbg_context_time_launches(tdbg_context* c, uint32_t n) {
  if (!c) return fail(TDBG_E_ARG, "null context");
  HIP_OK(hipSetDevice(c->device));
  while (c->tev.size() < 3ull * n) {
    hipEvent_t e;
    HIP_OK(hipEventCreate(&e));
    c->tev.push_back(e);
  }
  c->tcap = n;
  c->tcount = 0;
  return TDBG_OK;
}

int tdbg_context_launch_times(tdbg_context* c, float* kernel_ms, float* total_ms, uint32_t cap,
                              uint32_t* count) {
  if (!c || !count) return fail(TDBG_E_ARG, "null argument");
  const uint32_t n = std::min(c->tcount, cap);
  for (uint32_t i = 0; i < n; i++) {
    hipEvent_t* e = &c->tev[3 * i];
    HIP_OK(hipEventSynchronize(e[2]));
    if (kernel_ms) HIP_OK(hipEventElapsedTime(&kernel_ms[i], e[0], e[1]));
    if (total_ms) HIP_OK(hipEventElapsedTime(&total_ms[i], e[0], e[2]));
  }
  *count = n;
  c->tcap = 0;  // disarm
  c->tcount = 0;
  return TDBG_OK;
}

int tdbg_context_last_kernel_ms(tdbg_context* c, float* ms) {
  if (!c || !ms) return fail(TDBG_E_ARG, "null argument");
  if (c->last_te < 0)
    return fail(TDBG_E_ARG, "no timed launch yet (arm with tdbg_context_time_launches)");
  hipEvent_t* te = &c->tev[(size_t)c->last_te];
  HIP_OK(hipEventSynchronize(te[2]));
  HIP_OK(hipEventElapsedTime(ms, te[0], te[2]));
  return TDBG_OK;
}

int tdbg_debug_phase_clocks(tdbg_context* c, uint64_t* out, uint32_t nphases) {
  if (!c || !out) return fail(TDBG_E_ARG, "null argument");
  for (uint32_t k = 0; k < nphases; k++) out[k] = 0;
  if (!c->d_prof) return fail(TDBG_E_ARG, "no profiled launch (set TDBG_PROF=1)");
  HIP_OK(hipSetDevice(c->device));
  HIP_OK(hipDeviceSynchronize());
  std::vector<uint64_t> h((size_t)TDBG_PROF_PHASES * c->prof_grid);
  HIP_OK(hipMemcpy(h.data(), c->d_prof, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
  for (uint32_t g = 0; g < c->prof_grid; g++)
    for (uint32_t k = 0; k < nphases && k < TDBG_PROF_PHASES; k++) out[k] += h[(size_t)g * TDBG_PROF_PHASES + k];
  return TDBG_OK;
}

// ---------------------------------------------------------------------------
// host-resident end-to-end
// ---------------------------------------------------------------------------
static int stage_reserve(tdbg_context::Stage& s, uint64_t in_b, uint64_t out_b, uint64_t nt) {
  if (!s.stream) {
    HIP_OK(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    HIP_OK(hipEventCreateWithFlags(&s.h2d, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&s.kdone, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
  }
  if (in_b > s.in_cap) {
    if (s.d_in) HIP_OK(hipFree(s.d_in));
    HIP_OK(hipMalloc(&s.d_in, in_b));
    s.in_cap = in_b;
  }
  if (out_b > s.out_cap) {
    if (s.d_out) HIP_OK(hipFree(s.d_out));
    HIP_OK(hipMalloc(&s.d_out, out_b));
    s.out_cap = out_b;
  }
  if (nt > s.ptr_cap) {
    if (s.d_ptrs) HIP_OK(hipFree(s.d_ptrs));
    if (s.h_ptrs) HIP_OK(hipHostFree(s.h_ptrs));
    if (s.h_status) HIP_OK(hipHostFree(s.h_status));
    if (s.d_stat) HIP_OK(hipFree(s.d_stat));
    HIP_OK(hipMalloc(&s.d_stat, nt * 4));
    HIP_OK(hipMalloc(&s.d_ptrs, nt * 40));
    HIP_OK(hipHostMalloc((void**)&s.h_ptrs, nt * 40));
    HIP_OK(hipHostMalloc((void**)&s.h_status, nt * 4));
    s.ptr_cap = nt;
  }
  return TDBG_OK;
}

// Coalesced copies.  Input tiles join the previous tile's copy when they
// follow it in host memory with at most kInGap bytes of padding between them
// (e.g. the 16-B alignment a VFS batch read leaves): the padding is copied
// too, and device offsets keep the host spacing (in_dev_offsets).  Output
// tiles join only when exactly contiguous: padding must never be overwritten.
static constexpr uint64_t kInGap = 64;

// Only with TDBG_HOST_CONTIGUOUS_INPUT: without it, two tiles adjacent in
// the address space may sit in different allocations (e.g. two pinned
// blocks), and one copy must not span allocations.
static bool in_joins(const uint8_t* const* host, const uint64_t* size, uint64_t j, bool coalesce) {
  if (!coalesce) return false;
  const uint8_t* end = host[j - 1] + size[j - 1];
  return host[j] >= end && (uint64_t)(host[j] - end) <= kInGap;
}

// device offsets (relative to the stage's d_in) of tiles [lo, hi); returns the span
static uint64_t in_dev_offsets(const uint8_t* const* host, const uint64_t* size, uint64_t lo,
                               uint64_t hi, uint64_t* off, bool coalesce) {
  uint64_t o = 0;
  for (uint64_t i = lo; i < hi; i++) {
    if (i > lo && in_joins(host, size, i, coalesce)) o += (uint64_t)(host[i] - (host[i - 1] + size[i - 1]));
    if (off) off[i - lo] = o;
    o += size[i];
  }
  return o;
}

static int copy_ranges(hipStream_t st, uint64_t lo, uint64_t hi, const uint8_t* const* host,
                       const uint64_t* size, uint8_t* dev_base, bool h2d,
                       uint8_t* const* host_out, bool coalesce) {
  uint64_t i = lo;
  uint64_t doff = 0;
  while (i < hi) {
    uint64_t j = i + 1;
    uint64_t bytes = size[i];
    if (h2d) {
      while (j < hi && in_joins(host, size, j, coalesce)) { bytes = (uint64_t)(host[j] + size[j] - host[i]); j++; }
      if (bytes) HIP_OK(hipMemcpyAsync(dev_base + doff, host[i], bytes, hipMemcpyHostToDevice, st));
      doff += bytes;
      // the next span starts where in_dev_offsets puts it: right after this one
    } else {
      while (coalesce && j < hi && host_out[j] == host_out[j - 1] + size[j - 1]) { bytes += size[j]; j++; }
      if (bytes) HIP_OK(hipMemcpyAsync(host_out[i], dev_base + doff, bytes, hipMemcpyDeviceToHost, st));
      doff += bytes;
    }
    i = j;
  }
  return TDBG_OK;
}

// TDBG_MULTI_CHUNK when a tile of the call (host-known sizes) is larger than
// the pipeline's chunks (tile.cc:87-100)
static uint32_t multi_chunk_flag(const tdbg_pipeline* p, uint64_t ntiles, const uint64_t* out_size) {
  const uint64_t mc = p->max_chunk_size ? p->max_chunk_size : 65536;
  for (uint64_t i = 0; i < ntiles; i++)
    if (out_size[i] > mc) return TDBG_MULTI_CHUNK;
  return 0;
}

static int unfilter_host(tdbg_context* c, const tdbg_pipeline* p, uint64_t ntiles,
                         const uint8_t* const* in, const uint64_t* in_size,
                         uint8_t* const* out, const uint64_t* out_size, const uint64_t* var_size,
                         uint32_t flags, int32_t* host_status, uint64_t batch_bytes) {
  if (!c || !p) return fail(TDBG_E_ARG, "null context or pipeline");
  if (!p->supported) return fail(TDBG_E_UNSUPPORTED, "pipeline has a filter the engine does not run");
  if (ntiles == 0) return TDBG_OK;
  if (!in || !in_size || !out || !out_size) return fail(TDBG_E_ARG, "null tile arrays");
  HIP_OK(hipSetDevice(c->device));
  if (batch_bytes == 0) batch_bytes = 256ull << 20;
  const bool cin = (flags & TDBG_HOST_CONTIGUOUS_INPUT) != 0;
  const bool cout = (flags & TDBG_HOST_CONTIGUOUS_OUTPUT) != 0;
  flags &= ~(TDBG_HOST_CONTIGUOUS_INPUT | TDBG_HOST_CONTIGUOUS_OUTPUT);
  flags |= multi_chunk_flag(p, ntiles, out_size);
  if (!c->cstream) HIP_OK(hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
  if (!c->hstream) HIP_OK(hipStreamCreateWithFlags(&c->hstream, hipStreamNonBlocking));
  if (!c->dstream) HIP_OK(hipStreamCreateWithFlags(&c->dstream, hipStreamNonBlocking));
  {
    int rc = order_stream(c, c->cstream);
    if (rc) return rc;
  }
  // batches bounded by bytes on both sides
  std::vector<uint64_t> cuts{0};
  uint64_t bi = 0, bo = 0;
  for (uint64_t i = 0; i < ntiles; i++) {
    if (i > cuts.back() && (bi + in_size[i] > batch_bytes || bo + out_size[i] > batch_bytes)) {
      cuts.push_back(i);
      bi = bo = 0;
    }
    bi += in_size[i];
    bo += out_size[i];
  }
  cuts.push_back(ntiles);
  std::vector<int32_t> st(ntiles, 0);
  const size_t nb = cuts.size() - 1;
  constexpr int NS = (int)(sizeof(c->st) / sizeof(c->st[0]));
  std::vector<bool> pending(NS, false);
  std::vector<uint64_t> plo(NS), phi(NS);
  auto collect = [&](int k) -> int {
    auto& S = c->st[k];
    HIP_OK(hipEventSynchronize(S.done));
    memcpy(st.data() + plo[k], S.h_status, (phi[k] - plo[k]) * 4);
    pending[k] = false;
    return TDBG_OK;
  };
  for (size_t b = 0; b < nb; b++) {
    // slot k is reused once its previous batch's D2H is done (host wait);
    // the other slots' copies and kernels stay queued meanwhile
    const int k = (int)(b % NS);
    auto& S = c->st[k];
    if (pending[k]) { int rc = collect(k); if (rc) return rc; }
    const uint64_t lo = cuts[b], hi = cuts[b + 1], nt = hi - lo;
    uint64_t ob = 0;
    for (uint64_t i = lo; i < hi; i++) ob += out_size[i];
    const uint64_t ib = in_dev_offsets(in, in_size, lo, hi, nullptr, cin);
    int rc = stage_reserve(S, ib + 16, ob + 16, nt);
    if (rc) return rc;
    // pointer/size arrays (pinned) -> device
    const uint8_t** hp = S.h_ptrs;
    uint64_t* hs = (uint64_t*)(hp + nt);
    uint8_t** ho = (uint8_t**)(hs + nt);
    uint64_t* hos = (uint64_t*)(ho + nt);
    in_dev_offsets(in, in_size, lo, hi, (uint64_t*)hp, cin);  // offsets first, pointers below
    uint64_t oo = 0;
    for (uint64_t i = lo; i < hi; i++) {
      hp[i - lo] = S.d_in + (uint64_t)(uintptr_t)hp[i - lo];
      hs[i - lo] = in_size[i];
      ho[i - lo] = S.d_out + oo;
      hos[i - lo] = out_size[i];
      oo += out_size[i];
    }
    uint64_t* hv = (uint64_t*)(hos + nt);
    if (var_size) memcpy(hv, var_size + lo, nt * 8);
    HIP_OK(hipMemcpyAsync(S.d_ptrs, hp, nt * (var_size ? 40 : 32), hipMemcpyHostToDevice, c->hstream));
    rc = copy_ranges(c->hstream, lo, hi, in, in_size, S.d_in, true, nullptr, cin);
    if (rc) return rc;
    const uint8_t* const* dp = (const uint8_t* const*)S.d_ptrs;
    const uint64_t* ds = (const uint64_t*)(dp + nt);
    uint8_t* const* dop = (uint8_t* const*)(ds + nt);
    const uint64_t* dos = (const uint64_t*)(dop + nt);
    HIP_OK(hipEventRecord(S.h2d, c->hstream));
    // kernels serialize on the compute stream (they share the scratch slots)
    HIP_OK(hipStreamWaitEvent(c->cstream, S.h2d, 0));
    rc = ensure_status(c, nt);
    if (rc) return rc;
    rc = launch(c, p, nt, dp, ds, dop, dos, flags, S.d_stat, c->d_need, nullptr, c->cstream, false);
    if (rc) return rc;
    if (var_size) {  // Tile::add_extra_offset on the device, before the D2H
      hipError_t e = tdbg_launch_extra_offset(nt, dop, dos, dos + nt, S.d_stat, c->cstream);
      if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("extra offset launch: ") + hipGetErrorString(e));
    }
    HIP_OK(hipEventRecord(S.kdone, c->cstream));
    HIP_OK(hipStreamWaitEvent(c->dstream, S.kdone, 0));
    HIP_OK(hipMemcpyAsync(S.h_status, S.d_stat, nt * 4, hipMemcpyDeviceToHost, c->dstream));
    rc = copy_ranges(c->dstream, lo, hi, nullptr, out_size, S.d_out, false, out, cout);
    if (rc) return rc;
    HIP_OK(hipEventRecord(S.done, c->dstream));
    pending[k] = true;
    plo[k] = lo;
    phi[k] = hi;
  }
  for (int k = 0; k < NS; k++)
    if (pending[k]) { int rc = collect(k); if (rc) return rc; }
  c->tiles_unfiltered += ntiles;
  // tiles that needed bigger scratch: redo them one by one through the sync path
  for (uint64_t i = 0; i < ntiles; i++) {
    if (st[i] != TDBG_E_SCRATCH) continue;
    auto& S = c->st[0];
    int rc = stage_reserve(S, in_size[i] + 16, out_size[i] + 16, 1);
    if (rc) return rc;
    HIP_OK(hipMemcpy(S.d_in, in[i], in_size[i], hipMemcpyHostToDevice));
    const uint8_t* hp[4] = {S.d_in, (const uint8_t*)in_size[i], S.d_out, (const uint8_t*)out_size[i]};
    HIP_OK(hipMemcpy(S.d_ptrs, hp, 32, hipMemcpyHostToDevice));
    const uint8_t* const* dp = (const uint8_t* const*)S.d_ptrs;
    int32_t one = 0;
    rc = tdbg_unfilter_tiles_sync(c, p, 1, dp, (const uint64_t*)(dp + 1), (uint8_t* const*)(dp + 2),
                                  (const uint64_t*)(dp + 3), flags, &one, S.stream);
    st[i] = one;
    if (one == TDBG_OK) HIP_OK(hipMemcpy(out[i], S.d_out, out_size[i], hipMemcpyDeviceToHost));
    if (one == TDBG_OK && var_size && out_size[i] >= 8) memcpy(out[i] + out_size[i] - 8, &var_size[i], 8);
  }
  if (host_status) memcpy(host_status, st.data(), ntiles * 4);
  for (uint64_t i = 0; i < ntiles; i++)
    if (st[i]) {
      char msg[160];
      snprintf(msg, sizeof(msg), "tile %llu: %s", (unsigned long long)i, tdbg_status_str(st[i]));
      return fail(st[i], msg);
    }
  return TDBG_OK;
}

int tdbg_unfilter_tiles_host(tdbg_context* c, const tdbg_pipeline* p, uint64_t ntiles,
                             const uint8_t* const* in, const uint64_t* in_size,
                             uint8_t* const* out, const uint64_t* out_size, uint32_t flags,
                             int32_t* host_status, uint64_t batch_bytes) {
  return unfilter_host(c, p, ntiles, in, in_size, out, out_size, nullptr, flags, host_status, batch_bytes);
}

int tdbg_unfilter_offsets_host(tdbg_context* c, const tdbg_pipeline* p, uint64_t ntiles,
                               const uint8_t* const* in, const uint64_t* in_size,
                               uint8_t* const* out, const uint64_t* out_size, const uint64_t* var_size,
                               uint32_t flags, int32_t* host_status, uint64_t batch_bytes) {
  if (!(flags & TDBG_TILE_OFFSETS)) return fail(TDBG_E_ARG, "offsets entry without TDBG_TILE_OFFSETS");
  if (ntiles && !var_size) return fail(TDBG_E_ARG, "null var_size array");
  return unfilter_host(c, p, ntiles, in, in_size, out, out_size, var_size, flags, host_status, batch_bytes);
}

int tdbg_add_extra_offsets_async(tdbg_context* c, uint64_t ntiles, uint8_t* const* d_out,
                                 const uint64_t* d_out_size, const uint64_t* d_var_size,
                                 const int32_t* d_status, tdbg_stream stream) {
  if (!c) return fail(TDBG_E_ARG, "null context");
  if (ntiles == 0) return TDBG_OK;
  if (!d_out || !d_out_size || !d_var_size) return fail(TDBG_E_ARG, "null tile arrays");
  HIP_OK(hipSetDevice(c->device));
  int rc = order_stream(c, (hipStream_t)stream);
  if (rc) return rc;
  hipError_t e = tdbg_launch_extra_offset(ntiles, d_out, d_out_size, d_var_size, d_status, (hipStream_t)stream);
  if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("extra offset launch: ") + hipGetErrorString(e));
  return TDBG_OK;
}

int tdbg_shard_tiles(uint64_t ntiles, const uint64_t* in_size, const uint64_t* out_size,
                     uint32_t nshards, uint64_t* cuts) {
  if (!cuts || nshards == 0 || (ntiles && (!in_size || !out_size)))
    return fail(TDBG_E_ARG, "bad shard arguments");
  // contiguous shards balanced by filtered + unfiltered bytes: shard k ends
  // at the first tile where the running total reaches k/nshards of the whole
  uint64_t total = 0;
  for (uint64_t i = 0; i < ntiles; i++) total += in_size[i] + out_size[i];
  uint32_t k = 1;
  uint64_t acc = 0;
  cuts[0] = 0;
  for (uint64_t i = 0; i < ntiles && k < nshards; i++) {
    acc += in_size[i] + out_size[i];
    while (k < nshards && (unsigned __int128)acc * nshards >= (unsigned __int128)total * k) cuts[k++] = i + 1;
  }
  while (k <= nshards) cuts[k++] = ntiles;
  return TDBG_OK;
}

}  // extern "C"

// Contexts of the multi-GPU entry, kept across calls: a reader calls it once
// per batch of tiles, and a fresh context per call would hipMalloc its
// staging, status and scratch buffers every time.  A context serves one host
// thread at a time: taken out of the pool for the call, put back after.
namespace {
std::mutex g_pool_mu;
std::vector<tdbg_context*> g_pool;

int pool_acquire(int device, tdbg_context** out) {
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (size_t i = 0; i < g_pool.size(); i++)
      if (g_pool[i]->device == device) {
        *out = g_pool[i];
        g_pool.erase(g_pool.begin() + (std::ptrdiff_t)i);
        return TDBG_OK;
      }
  }
  return tdbg_context_create(device, out);
}

void pool_release(tdbg_context* c) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  g_pool.push_back(c);
}
}  // namespace

extern "C" {

int tdbg_release_cached_contexts(void) {
  std::vector<tdbg_context*> v;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    v.swap(g_pool);
  }
  for (auto c : v) tdbg_context_destroy(c);
  return TDBG_OK;
}

int tdbg_cached_context_count(void) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  return (int)g_pool.size();
}

int tdbg_unfilter_tiles_multi_gpu(const tdbg_pipeline* p, uint64_t ntiles,
                                  const uint8_t* const* in, const uint64_t* in_size,
                                  uint8_t* const* out, const uint64_t* out_size, uint32_t flags,
                                  int32_t* host_status, const int* devices, int ndev,
                                  uint64_t batch_bytes) {
  if (!p || !devices || ndev <= 0) return fail(TDBG_E_ARG, "bad device list");
  if (ntiles == 0) return TDBG_OK;
  std::vector<uint64_t> cut(ndev + 1);
  tdbg_shard_tiles(ntiles, in_size, out_size, (uint32_t)ndev, cut.data());
  std::vector<int> rcs(ndev, 0);
  std::vector<std::string> errs(ndev);
  std::vector<int32_t> st(ntiles, 0);
  std::vector<std::thread> th;
  for (int d = 0; d < ndev; d++) {
    th.emplace_back([&, d]() {
      const uint64_t lo = cut[d], hi = cut[d + 1];
      if (hi <= lo) return;
      tdbg_context* c = nullptr;
      int rc = pool_acquire(devices[d], &c);
      if (rc == TDBG_OK) {
        rc = tdbg_unfilter_tiles_host(c, p, hi - lo, in + lo, in_size + lo, out + lo, out_size + lo,
                                      flags, st.data() + lo, batch_bytes);
        pool_release(c);
      }
      rcs[d] = rc;
      if (rc) errs[d] = g_err;
    });
  }
  for (auto& t : th) t.join();
  if (host_status) memcpy(host_status, st.data(), ntiles * 4);
  for (int d = 0; d < ndev; d++)
    if (rcs[d] && rcs[d] != TDBG_OK) {
      // report the first failing tile in tile order when it is a tile status
      for (uint64_t i = 0; i < ntiles; i++)
        if (st[i]) {
          char msg[160];
          snprintf(msg, sizeof(msg), "tile %llu: %s", (unsigned long long)i, tdbg_status_str(st[i]));
          return fail(st[i], msg);
        }
      return fail(rcs[d], errs[d]);
    }
  return TDBG_OK;
}

int tdbg_context_device(const tdbg_context* c) { return c ? c->device : -1; }

// ---------------------------------------------------------------------------
// dense cell-slab copy (DenseReader::copy_fixed_tiles, dense_reader.cc:1555-1750)
// ---------------------------------------------------------------------------
static bool dense_cfg_ok(const tdbg_dense_copy_config* g) {
  if (!g || g->dim_num < 1 || g->dim_num > TDBG_DENSE_MAX_DIMS || g->cell_size == 0 || g->cell_order > 1 ||
      g->layout > 1)
    return false;
  for (uint32_t d = 0; d < g->dim_num; d++)
    if (g->tile_extent[d] <= 0 || g->sub_hi[d] < g->sub_lo[d]) return false;
  return true;
}

uint64_t tdbg_dense_result_bytes(const tdbg_dense_copy_config* g) {
  if (!dense_cfg_ok(g)) return 0;
  uint64_t n = g->cell_size;
  for (uint32_t d = 0; d < g->dim_num; d++) n *= (uint64_t)(g->sub_hi[d] - g->sub_lo[d] + 1);
  return n;
}

static uint64_t dense_tile_bytes(const tdbg_dense_copy_config* g) {
  uint64_t n = g->cell_size;
  for (uint32_t d = 0; d < g->dim_num; d++) n *= (uint64_t)g->tile_extent[d];
  return n;
}

int tdbg_dense_copy_async(tdbg_context* c, const tdbg_dense_copy_config* cfg, uint64_t ntiles,
                          const int64_t* d_tile_start, const uint8_t* const* d_tiles, const int32_t* d_status,
                          uint8_t* d_result, tdbg_stream stream) {
  if (!c) return fail(TDBG_E_ARG, "null context");
  if (!dense_cfg_ok(cfg)) return fail(TDBG_E_ARG, "invalid dense copy config");
  if (ntiles == 0) return TDBG_OK;
  if (!d_tile_start || !d_tiles || !d_result) return fail(TDBG_E_ARG, "null dense copy arrays");
  HIP_OK(hipSetDevice(c->device));
  int rc = order_stream(c, (hipStream_t)stream);
  if (rc) return rc;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(ntiles, (uint64_t)c->cus * 8);
  hipError_t e = tdbg_launch_dense_copy(cfg, ntiles, d_tile_start, d_tiles, d_status, d_result, grid,
                                        (hipStream_t)stream);
  if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("dense copy launch: ") + hipGetErrorString(e));
  return TDBG_OK;
}

// Host-side check of a dense read's space tiles (tile_start on the host): on
// one grid (tile 0's start as origin), distinct, and their intersections with
// the subarray add up to the whole subarray -- every result cell comes from
// exactly one given tile.  Returns nullptr when they do, else the reason.
static const char* dense_tiles_cover(const tdbg_dense_copy_config* cfg, uint64_t ntiles, const int64_t* tile_start) {
  const uint32_t nd = cfg->dim_num;
  uint64_t want = 1, got = 0;
  for (uint32_t d = 0; d < nd; d++) want *= (uint64_t)(cfg->sub_hi[d] - cfg->sub_lo[d] + 1);
  std::vector<std::vector<int64_t>> keys(ntiles);
  for (uint64_t t = 0; t < ntiles; t++) {
    uint64_t n = 1;
    for (uint32_t d = 0; d < nd; d++) {
      const int64_t s = tile_start[t * nd + d], e = cfg->tile_extent[d];
      if ((s - tile_start[d]) % e != 0) return "dense read: tile start off the tile grid";
      const int64_t lo = std::max(s, cfg->sub_lo[d]), hi = std::min(s + e - 1, cfg->sub_hi[d]);
      n = hi < lo ? 0 : n * (uint64_t)(hi - lo + 1);
    }
    got += n;
    keys[t].assign(tile_start + t * nd, tile_start + (t + 1) * nd);
  }
  std::sort(keys.begin(), keys.end());
  if (std::adjacent_find(keys.begin(), keys.end()) != keys.end()) return "dense read: a tile is given twice";
  if (got != want) return "dense read: the tiles do not cover the subarray";
  return nullptr;
}

int tdbg_dense_read_host(tdbg_context* c, const tdbg_pipeline* p, uint64_t ntiles, const uint8_t* const* in,
                         const uint64_t* in_size, const int64_t* tile_start, const tdbg_dense_copy_config* cfg,
                         uint8_t* result, uint64_t result_size, uint32_t flags, int32_t* host_status,
                         uint64_t batch_bytes) {
  if (!c || !p) return fail(TDBG_E_ARG, "null context or pipeline");
  if (!p->supported) return fail(TDBG_E_UNSUPPORTED, "pipeline has a filter the engine does not run");
  if (!dense_cfg_ok(cfg)) return fail(TDBG_E_ARG, "invalid dense copy config");
  const uint64_t rbytes = tdbg_dense_result_bytes(cfg);
  if (!result || result_size < rbytes) return fail(TDBG_E_ARG, "result buffer smaller than the subarray");
  if (ntiles == 0) return TDBG_OK;
  if (!in || !in_size || !tile_start) return fail(TDBG_E_ARG, "null tile arrays");
  // Every result cell must come from a tile (this entry has no fill value,
  // and the device result buffer is not initialised)
  if (const char* why = dense_tiles_cover(cfg, ntiles, tile_start)) return fail(TDBG_E_ARG, why);
  HIP_OK(hipSetDevice(c->device));
  if (batch_bytes == 0) batch_bytes = 256ull << 20;
  const bool cin = (flags & TDBG_HOST_CONTIGUOUS_INPUT) != 0;
  flags &= ~(TDBG_HOST_CONTIGUOUS_INPUT | TDBG_HOST_CONTIGUOUS_OUTPUT);
  if (!c->cstream) HIP_OK(hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
  if (!c->hstream) HIP_OK(hipStreamCreateWithFlags(&c->hstream, hipStreamNonBlocking));
  {
    int rc = order_stream(c, c->cstream);
    if (rc) return rc;
  }
  const uint32_t nd = cfg->dim_num;
  const uint64_t tb = dense_tile_bytes(cfg);
  // the device result buffer and the tile starts (kept until the D2H is done)
  uint8_t* d_result = nullptr;
  int64_t* d_start = nullptr;
  HIP_OK(hipMalloc(&d_result, rbytes));
  hipError_t e0 = hipMalloc(&d_start, ntiles * nd * sizeof(int64_t));
  if (e0 == hipSuccess) e0 = hipMemcpy(d_start, tile_start, ntiles * nd * sizeof(int64_t), hipMemcpyHostToDevice);
  if (e0 != hipSuccess) {
    (void)hipFree(d_result);
    if (d_start) (void)hipFree(d_start);
    return fail(TDBG_E_DEVICE, std::string("dense read setup: ") + hipGetErrorString(e0));
  }
  // batches bounded by bytes on both sides; two staging slots alternate
  std::vector<uint64_t> cuts{0};
  uint64_t bi = 0, bo = 0;
  for (uint64_t i = 0; i < ntiles; i++) {
    if (i > cuts.back() && (bi + in_size[i] > batch_bytes || bo + tb > batch_bytes)) {
      cuts.push_back(i);
      bi = bo = 0;
    }
    bi += in_size[i];
    bo += tb;
  }
  cuts.push_back(ntiles);
  std::vector<int32_t> st(ntiles, 0);
  int rc = TDBG_OK;
  bool used[2] = {false, false};
  for (size_t b = 0; b + 1 < cuts.size() && rc == TDBG_OK; b++) {
    auto& S = c->st[b % 2];
    const uint64_t lo = cuts[b], hi = cuts[b + 1], nt = hi - lo;
    if (used[b % 2]) {  // the slot's previous batch (kernels + status copy) is done
      if (hipEventSynchronize(S.done) != hipSuccess) { rc = fail(TDBG_E_DEVICE, "dense read: event wait"); break; }
    }
    const uint64_t ib = in_dev_offsets(in, in_size, lo, hi, nullptr, cin);
    rc = stage_reserve(S, ib + 16, nt * tb + 16, nt);
    if (rc) break;
    const uint8_t** hp = S.h_ptrs;
    uint64_t* hs = (uint64_t*)(hp + nt);
    uint8_t** ho = (uint8_t**)(hs + nt);
    uint64_t* hos = (uint64_t*)(ho + nt);
    in_dev_offsets(in, in_size, lo, hi, (uint64_t*)hp, cin);
    for (uint64_t i = lo; i < hi; i++) {
      hp[i - lo] = S.d_in + (uint64_t)(uintptr_t)hp[i - lo];
      hs[i - lo] = in_size[i];
      ho[i - lo] = S.d_out + (i - lo) * tb;
      hos[i - lo] = tb;
    }
    hipError_t e = hipMemcpyAsync(S.d_ptrs, hp, nt * 32, hipMemcpyHostToDevice, c->hstream);
    if (e != hipSuccess) { rc = fail(TDBG_E_DEVICE, "dense read: pointer copy"); break; }
    rc = copy_ranges(c->hstream, lo, hi, in, in_size, S.d_in, true, nullptr, cin);
    if (rc) break;
    if (hipEventRecord(S.h2d, c->hstream) != hipSuccess || hipStreamWaitEvent(c->cstream, S.h2d, 0) != hipSuccess) {
      rc = fail(TDBG_E_DEVICE, "dense read: stream ordering");
      break;
    }
    const uint8_t* const* dp = (const uint8_t* const*)S.d_ptrs;
    const uint64_t* ds = (const uint64_t*)(dp + nt);
    uint8_t* const* dop = (uint8_t* const*)(ds + nt);
    const uint64_t* dos = (const uint64_t*)(dop + nt);
    rc = ensure_status(c, nt);
    if (rc) break;
    rc = launch(c, p, nt, dp, ds, dop, dos, flags, S.d_stat, c->d_need, nullptr, c->cstream, false);
    if (rc) break;
    const uint32_t grid = (uint32_t)std::min<uint64_t>(nt, (uint64_t)c->cus * 8);
    e = tdbg_launch_dense_copy(cfg, nt, d_start + lo * nd, (const uint8_t* const*)dop, S.d_stat, d_result, grid,
                               c->cstream);
    if (e != hipSuccess) { rc = fail(TDBG_E_DEVICE, std::string("dense copy launch: ") + hipGetErrorString(e)); break; }
    e = hipMemcpyAsync(st.data() + lo, S.d_stat, nt * 4, hipMemcpyDeviceToHost, c->cstream);
    if (e == hipSuccess) e = hipEventRecord(S.done, c->cstream);
    if (e != hipSuccess) { rc = fail(TDBG_E_DEVICE, "dense read: status copy"); break; }
    used[b % 2] = true;
  }
  // the one D2H: the subarray's cells
  if (rc == TDBG_OK) {
    hipError_t e = hipMemcpyAsync(result, d_result, rbytes, hipMemcpyDeviceToHost, c->cstream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->cstream);
    if (e != hipSuccess) rc = fail(TDBG_E_DEVICE, std::string("dense read D2H: ") + hipGetErrorString(e));
  } else {
    (void)hipStreamSynchronize(c->cstream);
  }
  (void)hipFree(d_result);
  (void)hipFree(d_start);
  if (rc) return rc;
  c->tiles_unfiltered += ntiles;
  // tiles that needed bigger scratch: their cells are re-copied through the sync path
  for (uint64_t i = 0; i < ntiles; i++)
    if (st[i] == TDBG_E_SCRATCH) {
      std::vector<uint8_t> tile(tb);
      uint8_t* outp = tile.data();
      int32_t one = 0;
      int r2 = unfilter_host(c, p, 1, in + i, in_size + i, &outp, &tb, nullptr, flags, &one, 0);
      st[i] = one;
      if (r2 == TDBG_OK && one == TDBG_OK) {
        // host-side slab copy of this one tile (rare path)
        tdbg_dense_copy_config g = *cfg;
        std::vector<int64_t> cc(nd);
        const int64_t* s0 = tile_start + i * nd;
        int64_t lo2[TDBG_DENSE_MAX_DIMS], len[TDBG_DENSE_MAX_DIMS];
        bool empty = false;
        uint64_t ncell = 1;
        for (uint32_t d = 0; d < nd; d++) {
          lo2[d] = std::max(s0[d], g.sub_lo[d]);
          const int64_t hi2 = std::min(s0[d] + g.tile_extent[d] - 1, g.sub_hi[d]);
          if (hi2 < lo2[d]) empty = true;
          len[d] = hi2 - lo2[d] + 1;
          if (!empty) ncell *= (uint64_t)len[d];
        }
        if (empty) continue;
        for (uint64_t k = 0; k < ncell; k++) {
          uint64_t r = k;
          for (uint32_t d = 0; d < nd; d++) {
            cc[d] = (int64_t)(r % (uint64_t)len[d]);
            r /= (uint64_t)len[d];
          }
          uint64_t si = 0, di = 0;
          auto L = [&](const int64_t* ext, bool row, bool tilecoord) {
            uint64_t x = 0;
            if (row) {
              for (uint32_t d = 0; d < nd; d++)
                x = x * (uint64_t)ext[d] + (uint64_t)(lo2[d] + cc[d] - (tilecoord ? s0[d] : g.sub_lo[d]));
            } else {
              for (int d = (int)nd - 1; d >= 0; d--)
                x = x * (uint64_t)ext[d] + (uint64_t)(lo2[d] + cc[d] - (tilecoord ? s0[d] : g.sub_lo[d]));
            }
            return x;
          };
          int64_t sub_ext[TDBG_DENSE_MAX_DIMS];
          for (uint32_t d = 0; d < nd; d++) sub_ext[d] = g.sub_hi[d] - g.sub_lo[d] + 1;
          si = L(g.tile_extent, g.cell_order == 0, true);
          di = L(sub_ext, g.layout == 0, false);
          memcpy(result + di * g.cell_size, tile.data() + si * g.cell_size, g.cell_size);
        }
      }
    }
  if (host_status) memcpy(host_status, st.data(), ntiles * 4);
  for (uint64_t i = 0; i < ntiles; i++)
    if (st[i]) {
      char msg[160];
      snprintf(msg, sizeof(msg), "tile %llu: %s", (unsigned long long)i, tdbg_status_str(st[i]));
      return fail(st[i], msg);
    }
  return TDBG_OK;
}

int tdbg_device_alloc(int device, uint64_t bytes, void** out) {
  if (!out) return fail(TDBG_E_ARG, "null out");
  HIP_OK(hipSetDevice(device));
  HIP_OK(hipMalloc(out, bytes ? bytes : 1));
  return TDBG_OK;
}
int tdbg_device_free(void* p) {
  HIP_OK(hipFree(p));
  return TDBG_OK;
}
int tdbg_memcpy_h2d(void* dst, const void* src, uint64_t bytes) {
  HIP_OK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return TDBG_OK;
}
int tdbg_memcpy_d2h(void* dst, const void* src, uint64_t bytes) {
  HIP_OK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return TDBG_OK;
}
int tdbg_device_count(int* n) {
  if (!n) return fail(TDBG_E_ARG, "null out");
  HIP_OK(hipGetDeviceCount(n));
  return TDBG_OK;
}

// ---------------------------------------------------------------------------
// dense reads with several fragments / fill values / var-sized cells
// (dense_reader.cc:1199-1236, 1521-2000; tdbg_dense.hip)
// ---------------------------------------------------------------------------
static bool frag_cfg_ok(const tdbg_dense_frag_config* f, bool var) {
  if (!f || !dense_cfg_ok(&f->base)) return false;
  if (f->fill_validity > 1) return false;
  if (var) {
    if (f->elements_mode && (f->data_type_size == 0 || f->fill_size % f->data_type_size)) return false;
  } else if (f->fill_size != f->base.cell_size) {
    return false;
  }
  return true;
}

static uint64_t dense_cells(const tdbg_dense_copy_config* g) {
  uint64_t n = 1;
  for (uint32_t d = 0; d < g->dim_num; d++) n *= (uint64_t)(g->sub_hi[d] - g->sub_lo[d] + 1);
  return n;
}

int tdbg_dense_copy_fragments_async(tdbg_context* c, const tdbg_dense_frag_config* cfg, uint64_t ntiles,
                                    const int64_t* d_tile_start, const int64_t* d_frag_dom,
                                    const uint8_t* const* d_tiles, const uint8_t* const* d_validity,
                                    const uint8_t* d_fill_value, uint8_t* d_result, uint8_t* d_result_validity,
                                    tdbg_stream stream) {
  if (!c) return fail(TDBG_E_ARG, "null context");
  if (!frag_cfg_ok(cfg, false)) return fail(TDBG_E_ARG, "invalid dense fragment copy config");
  if (!d_result || !d_fill_value || (ntiles && !d_tile_start) || (ntiles && cfg->nfrag && (!d_tiles || !d_frag_dom)))
    return fail(TDBG_E_ARG, "null dense copy arrays");
  if (cfg->nullable && !d_result_validity) return fail(TDBG_E_ARG, "nullable copy without a result validity buffer");
  HIP_OK(hipSetDevice(c->device));
  int rc = order_stream(c, (hipStream_t)stream);
  if (rc) return rc;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(ntiles, (uint64_t)c->cus * 8);
  hipError_t e = tdbg_launch_dense_frag_copy(cfg, ntiles, d_tile_start, d_frag_dom, d_tiles, d_validity, d_fill_value,
                                             d_result, d_result_validity, dense_cells(&cfg->base), std::max(grid, 1u),
                                             (hipStream_t)stream);
  if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("dense copy launch: ") + hipGetErrorString(e));
  return TDBG_OK;
}

int tdbg_dense_var_offsets_async(tdbg_context* c, const tdbg_dense_frag_config* cfg, uint64_t ntiles,
                                 const int64_t* d_tile_start, const int64_t* d_frag_dom,
                                 const uint8_t* const* d_offset_tiles, const uint8_t* const* d_var_tiles,
                                 const uint8_t* const* d_validity, const uint8_t* d_fill_value,
                                 uint64_t* d_result_offsets, uint8_t* d_result_validity, uint64_t* d_var_total,
                                 tdbg_stream stream) {
  if (!c) return fail(TDBG_E_ARG, "null context");
  if (!frag_cfg_ok(cfg, true)) return fail(TDBG_E_ARG, "invalid dense var copy config");
  if (!d_result_offsets || !d_var_total || !d_fill_value || (ntiles && !d_tile_start) ||
      (ntiles && cfg->nfrag && (!d_offset_tiles || !d_var_tiles || !d_frag_dom)))
    return fail(TDBG_E_ARG, "null dense var arrays");
  if (cfg->nullable && !d_result_validity) return fail(TDBG_E_ARG, "nullable copy without a result validity buffer");
  HIP_OK(hipSetDevice(c->device));
  int rc = order_stream(c, (hipStream_t)stream);
  if (rc) return rc;
  if (!c->dense_err) HIP_OK(hipMalloc(&c->dense_err, 4));
  // (per call, ordered with this call's kernel on the caller's stream)
  HIP_OK(hipMemsetAsync(c->dense_err, 0, 4, (hipStream_t)stream));
  const uint64_t n = dense_cells(&cfg->base);
  const uint64_t nb = (n + 2047) / 2048;
  if (n > c->dense_src_cap) {
    HIP_OK(hipStreamSynchronize((hipStream_t)stream));  // an earlier step 2 may still read them
    if (c->dense_src) HIP_OK(hipFree(c->dense_src));
    if (c->dense_bsum) HIP_OK(hipFree(c->dense_bsum));
    c->dense_src = nullptr;
    c->dense_bsum = nullptr;
    c->dense_src_cap = 0;
    HIP_OK(hipMalloc(&c->dense_src, n * 8));
    HIP_OK(hipMalloc(&c->dense_bsum, std::max<uint64_t>(nb, 1) * 8));
    c->dense_src_cap = n;
  }
  c->dense_ncells = n;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(ntiles, 1), (uint64_t)c->cus * 8);
  hipError_t e = tdbg_launch_dense_var_offsets(cfg, ntiles, d_tile_start, d_frag_dom, d_offset_tiles, d_var_tiles,
                                               d_validity, d_fill_value, d_result_offsets, n, c->dense_src,
                                               d_result_validity, c->dense_bsum, d_var_total, c->dense_err, grid,
                                               (hipStream_t)stream);
  if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("dense var offsets launch: ") + hipGetErrorString(e));
  return TDBG_OK;
}

int tdbg_dense_var_copy_async(tdbg_context* c, const tdbg_dense_frag_config* cfg, const uint64_t* d_result_offsets,
                              const uint64_t* d_var_total, uint8_t* d_result_var, tdbg_stream stream) {
  if (!c) return fail(TDBG_E_ARG, "null context");
  if (!frag_cfg_ok(cfg, true)) return fail(TDBG_E_ARG, "invalid dense var copy config");
  if (!d_result_offsets || !d_var_total || !d_result_var) return fail(TDBG_E_ARG, "null dense var arrays");
  const uint64_t n = dense_cells(&cfg->base);
  if (n != c->dense_ncells || !c->dense_src)
    return fail(TDBG_E_ARG, "tdbg_dense_var_copy_async: run tdbg_dense_var_offsets_async on this context first");
  HIP_OK(hipSetDevice(c->device));
  int rc = order_stream(c, (hipStream_t)stream);
  if (rc) return rc;
  const uint32_t grid = (uint32_t)std::min<uint64_t>((n + 255) / 256, (uint64_t)c->cus * 8);
  hipError_t e = tdbg_launch_dense_var_copy(d_result_offsets, c->dense_src, n, d_var_total,
                                            cfg->elements_mode ? cfg->data_type_size : 1, d_result_var, grid,
                                            (hipStream_t)stream);
  if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("dense var copy launch: ") + hipGetErrorString(e));
  return TDBG_OK;
}

int tdbg_dense_var_status(tdbg_context* c, tdbg_stream stream, int32_t* status) {
  if (!c || !status) return fail(TDBG_E_ARG, "null context or status");
  if (!c->dense_err) return fail(TDBG_E_ARG, "tdbg_dense_var_status: no tdbg_dense_var_offsets_async on this context");
  HIP_OK(hipSetDevice(c->device));
  uint32_t herr = 0;
  HIP_OK(hipMemcpyAsync(&herr, c->dense_err, 4, hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIP_OK(hipStreamSynchronize((hipStream_t)stream));
  *status = herr ? TDBG_E_DATA_READ : TDBG_OK;
  return TDBG_OK;
}

int tdbg_dense_read_var_host(tdbg_context* c, const tdbg_pipeline* po, const tdbg_pipeline* pv,
                             const tdbg_dense_frag_config* cfg, uint64_t ntiles, const int64_t* tile_start,
                             const int64_t* frag_dom, const uint8_t* const* off_filtered,
                             const uint64_t* off_filtered_size, const uint8_t* const* var_filtered,
                             const uint64_t* var_filtered_size, const uint64_t* var_unfiltered_size,
                             const uint8_t* fill_value, uint64_t* result_offsets, uint8_t* result_var,
                             uint64_t var_cap, uint64_t* var_total, int32_t* host_status) {
  if (!c || !po || !pv) return fail(TDBG_E_ARG, "null context or pipeline");
  if (!po->supported || !pv->supported) return fail(TDBG_E_UNSUPPORTED, "pipeline has a filter the engine does not run");
  if (!frag_cfg_ok(cfg, true) || cfg->nullable) return fail(TDBG_E_ARG, "invalid dense var read config");
  if (!result_offsets || !var_total || (cfg->fill_size && !fill_value))
    return fail(TDBG_E_ARG, "null dense var read outputs");
  const uint32_t nd = cfg->base.dim_num, nf = cfg->nfrag;
  const uint64_t npair = ntiles * nf;
  if (npair && (!tile_start || !frag_dom || !off_filtered || !off_filtered_size || !var_filtered ||
                !var_filtered_size || !var_unfiltered_size))
    return fail(TDBG_E_ARG, "null dense var read inputs");
  if (ntiles && !tile_start) return fail(TDBG_E_ARG, "null dense var read inputs");
  // every result cell comes from exactly one given space tile (its value or
  // the fill value), as the reference iterates every space tile of the
  // subarray
  if (const char* why = dense_tiles_cover(&cfg->base, ntiles, tile_start)) return fail(TDBG_E_ARG, why);
  HIP_OK(hipSetDevice(c->device));
  if (!c->cstream) HIP_OK(hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
  hipStream_t s = c->cstream;
  int rc = order_stream(c, s);
  if (rc) return rc;
  uint64_t cells_per_tile = 1;
  for (uint32_t d = 0; d < nd; d++) cells_per_tile *= (uint64_t)cfg->base.tile_extent[d];
  // the present (tile, fragment) pairs: filtered bytes in, unfiltered out
  std::vector<uint64_t> idx;
  uint64_t fin = 0, unf_off = 0, unf_var = 0;
  for (uint64_t i = 0; i < npair; i++)
    if (off_filtered[i]) {
      if (!var_filtered[i]) return fail(TDBG_E_ARG, "offsets tile without its var tile");
      idx.push_back(i);
      fin += off_filtered_size[i] + var_filtered_size[i];
      unf_off += (cells_per_tile + 1) * 8;
      unf_var += var_unfiltered_size[i];
    }
  const uint64_t m = idx.size();
  const uint64_t n = dense_cells(&cfg->base);
  // every device buffer of the read carved from one grow-only context arena
  // (a hipMalloc / hipFree pair per buffer and call cost more than the read's
  // own kernels).  The var result holds at most every present tile's var
  // bytes plus the fill value once per cell (each result cell is one source
  // cell or the fill), and never more than the caller's var_cap.
  const uint64_t rvar_max = std::min<uint64_t>(var_cap, unf_var + n * (uint64_t)cfg->fill_size);
  const uint64_t sizes[11] = {fin, unf_off, unf_var, cfg->fill_size, ntiles * nd * 8, (uint64_t)nf * nd * 16,
                              (9 * m + 2 * npair) * 8, 2 * m * 4, n * 8, 8, rvar_max};
  uint64_t need = 0;
  for (uint64_t z : sizes) need += (std::max<uint64_t>(z, 16) + 255) & ~255ull;
  if (need > c->dv_cap) {
    HIP_OK(hipStreamSynchronize(s));
    if (c->dv_arena) (void)hipFree(c->dv_arena);
    c->dv_arena = nullptr;
    c->dv_cap = 0;
    if (hipMalloc(&c->dv_arena, need) != hipSuccess) return fail(TDBG_E_DEVICE, "dense var read: device allocation failed");
    c->dv_cap = need;
  }
  uint8_t* carve = c->dv_arena;
  auto take = [&](uint64_t z) -> uint8_t* {
    uint8_t* q = carve;
    carve += (std::max<uint64_t>(z, 16) + 255) & ~255ull;
    return q;
  };
  uint8_t* d_in = take(sizes[0]);
  uint8_t* d_off = take(sizes[1]);
  uint8_t* d_var = take(sizes[2]);
  uint8_t* d_fill = take(sizes[3]);
  int64_t* d_start = (int64_t*)take(sizes[4]);
  int64_t* d_dom = (int64_t*)take(sizes[5]);
  uint64_t* d_ptr = (uint64_t*)take(sizes[6]);  // unfilter tables for the 2m tiles, then per-pair tile tables
  int32_t* d_st = (int32_t*)take(sizes[7]);
  uint64_t* d_roff = (uint64_t*)take(sizes[8]);
  uint64_t* d_total = (uint64_t*)take(sizes[9]);
  uint8_t* const d_rvar_region = take(sizes[10]);
  // [2m in][2m in size][2m out][2m out size][m var size][npair offsets tile][npair var tile]
  std::vector<uint64_t> h(9 * m + 2 * npair, 0);
  uint64_t* hin = h.data();
  uint64_t* hisz = hin + 2 * m;
  uint64_t* hout = hisz + 2 * m;
  uint64_t* hosz = hout + 2 * m;
  uint64_t* hvsz = hosz + 2 * m;
  uint64_t* hoff_t = hvsz + m;
  uint64_t* hvar_t = hoff_t + npair;
  uint64_t io = 0, oo = 0, ov = 0;
  // host-to-device copies of adjacent host tiles coalesced (tiles read into
  // one FilteredData-style block, filtered_data.h:152-644, are back to back
  // in the order [offsets tile, var tile] per pair): one copy per run
  const uint8_t* run_src = nullptr;
  uint64_t run_dst = 0, run_len = 0;
  auto h2d = [&](const uint8_t* src, uint64_t len) -> hipError_t {
    hipError_t e = hipSuccess;
    if (run_len && src == run_src + run_len) {
      run_len += len;
    } else {
      if (run_len) e = hipMemcpyAsync(d_in + run_dst, run_src, run_len, hipMemcpyHostToDevice, s);
      run_src = src;
      run_dst = io;
      run_len = len;
    }
    io += len;
    return e;
  };
  for (uint64_t k = 0; k < m; k++) {
    const uint64_t i = idx[k];
    hin[k] = (uint64_t)(uintptr_t)(d_in + io);
    HIP_OK(h2d(off_filtered[i], off_filtered_size[i]));
    hisz[k] = off_filtered_size[i];
    hin[m + k] = (uint64_t)(uintptr_t)(d_in + io);
    HIP_OK(h2d(var_filtered[i], var_filtered_size[i]));
    hisz[m + k] = var_filtered_size[i];
    hout[k] = (uint64_t)(uintptr_t)(d_off + oo);
    hosz[k] = (cells_per_tile + 1) * 8;
    hoff_t[i] = hout[k];
    oo += hosz[k];
    hout[m + k] = (uint64_t)(uintptr_t)(d_var + ov);
    hosz[m + k] = var_unfiltered_size[i];
    hvar_t[i] = hout[m + k];
    ov += var_unfiltered_size[i];
    hvsz[k] = var_unfiltered_size[i];
  }
  if (run_len) HIP_OK(hipMemcpyAsync(d_in + run_dst, run_src, run_len, hipMemcpyHostToDevice, s));
  HIP_OK(hipMemcpyAsync(d_ptr, h.data(), h.size() * 8, hipMemcpyHostToDevice, s));
  if (cfg->fill_size) HIP_OK(hipMemcpyAsync(d_fill, fill_value, cfg->fill_size, hipMemcpyHostToDevice, s));
  if (ntiles) HIP_OK(hipMemcpyAsync(d_start, tile_start, ntiles * nd * 8, hipMemcpyHostToDevice, s));
  if (nf) HIP_OK(hipMemcpyAsync(d_dom, frag_dom, (uint64_t)nf * nd * 16, hipMemcpyHostToDevice, s));
  const uint64_t* dp = d_ptr;
  std::vector<int32_t> st(2 * m, 0);
  if (m) {
    rc = ensure_status(c, 2 * m);
    if (rc) return rc;
    // offsets tiles (the extra slot left for add_extra_offset), then
    // Tile::add_extra_offset with the var tile's size (reader_base.cc:885-893),
    // then the var tiles
    rc = launch(c, po, m, (const uint8_t* const*)dp, dp + 2 * m, (uint8_t* const*)(dp + 4 * m), dp + 6 * m,
                TDBG_TILE_OFFSETS, d_st, c->d_need, nullptr, s, false);
    if (rc) return rc;
    hipError_t e = tdbg_launch_extra_offset(m, (uint8_t* const*)(dp + 4 * m), dp + 6 * m, dp + 8 * m, d_st, s);
    if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("extra offset launch: ") + hipGetErrorString(e));
    rc = launch(c, pv, m, (const uint8_t* const*)(dp + m), dp + 3 * m, (uint8_t* const*)(dp + 5 * m), dp + 7 * m, 0,
                d_st + m, c->d_need, nullptr, s, false);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(st.data(), d_st, 2 * m * 4, hipMemcpyDeviceToHost, s));
  }
  HIP_OK(hipStreamSynchronize(s));
  // Tiles a stage outgrew the default scratch slots for (TDBG_E_SCRATCH: tiny
  // PD/BWR windows, RLE of 1-byte cells, ...): redone one by one through the
  // sync entry's bigger retry slots, in place (their table rows are one-tile
  // arrays); an offsets tile then takes its extra offset
  for (uint64_t k = 0; k < 2 * m; k++) {
    if (st[k] != TDBG_E_SCRATCH) continue;
    const bool offs = k < m;
    int32_t one = 0;
    rc = tdbg_unfilter_tiles_sync(c, offs ? po : pv, 1, (const uint8_t* const*)(dp + k), dp + 2 * m + k,
                                  (uint8_t* const*)(dp + 4 * m + k), dp + 6 * m + k, offs ? TDBG_TILE_OFFSETS : 0u,
                                  &one, (tdbg_stream)s);
    if (rc != TDBG_OK && one == TDBG_OK) return rc;  // (a launch failure, not a tile status)
    st[k] = one;
    if (offs && one == TDBG_OK) {
      HIP_OK(hipMemsetAsync(d_st + k, 0, 4, s));
      hipError_t e = tdbg_launch_extra_offset(1, (uint8_t* const*)(dp + 4 * m + k), dp + 6 * m + k, dp + 8 * m + k,
                                              d_st + k, s);
      if (e != hipSuccess) return fail(TDBG_E_DEVICE, std::string("extra offset launch: ") + hipGetErrorString(e));
    }
  }
  HIP_OK(hipStreamSynchronize(s));
  // per pair: the first failure of its two tiles; any failure stops the read
  // (an unfilter error fails the reference's query)
  std::vector<int32_t> pst(npair, 0);
  int first_err = TDBG_OK;
  for (uint64_t k = 0; k < m; k++) {
    const int32_t a = st[k] ? st[k] : st[m + k];
    pst[idx[k]] = a;
    if (a && first_err == TDBG_OK) first_err = a;
  }
  if (host_status && npair) memcpy(host_status, pst.data(), npair * 4);
  if (first_err != TDBG_OK) return fail(first_err, "dense var read: a tile failed to unfilter");
  tdbg_dense_frag_config g = *cfg;
  g.base.cell_size = 8;
  rc = tdbg_dense_var_offsets_async(c, &g, ntiles, d_start, d_dom, (const uint8_t* const*)(dp + 9 * m),
                                    (const uint8_t* const*)(dp + 9 * m + npair), nullptr, d_fill, d_roff, nullptr,
                                    d_total, s);
  if (rc) return rc;
  HIP_OK(hipMemcpyAsync(var_total, d_total, 8, hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(result_offsets, d_roff, n * 8, hipMemcpyDeviceToHost, s));
  uint32_t herr = 0;
  HIP_OK(hipMemcpyAsync(&herr, c->dense_err, 4, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  if (herr) return fail(TDBG_E_DATA_READ, "dense var read: a cell's offsets lie outside its var tile");
  const uint64_t mult = cfg->elements_mode ? cfg->data_type_size : 1;
  const uint64_t vbytes = *var_total * mult;
  if (vbytes > var_cap || (vbytes && !result_var))
    return fail(TDBG_E_OUT_FULL, "dense var read: var buffer too small");
  if (vbytes) {
    uint8_t* d_rvar = d_rvar_region;  // (rvar_max bytes, carved above)
    if (vbytes > rvar_max) {
      // overlapping (but in-bounds) cell offsets can read a var tile's bytes
      // more than once: the result outgrows the carve, never var_cap; a
      // grow-only buffer of its own (the arena's other carves are in use)
      if (vbytes > c->dv_extra_cap) {
        if (c->dv_extra) (void)hipFree(c->dv_extra);
        c->dv_extra = nullptr;
        c->dv_extra_cap = 0;
        if (hipMalloc(&c->dv_extra, vbytes) != hipSuccess)
          return fail(TDBG_E_DEVICE, "dense var read: device allocation failed");
        c->dv_extra_cap = vbytes;
      }
      d_rvar = c->dv_extra;
    }
    rc = tdbg_dense_var_copy_async(c, &g, d_roff, d_total, d_rvar, s);
    if (rc) return rc;
    HIP_OK(hipMemcpyAsync(result_var, d_rvar, vbytes, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
  }
  c->tiles_unfiltered += 2 * m;
  return TDBG_OK;
}

}  // extern "C"
