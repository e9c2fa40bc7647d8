// tdbg_dense.hip -- the step after the path: the dense
// reader's cell-slab copy from unfiltered tiles into the query's result
// buffer, on the device, so only result bytes cross PCIe.
//
// DenseReader::copy_attribute -> copy_fixed_tiles (dense_reader.cc:1241,
// 1555-1750) walks each tile's part of the subarray in cell slabs
// (TileCellSlabIter): runs of cells contiguous in the tile along its fastest
// dimension.  When the result layout equals the tile cell order (stride 1)
// a slab is one memcpy into the result at the cell's row/col-major offset in
// the subarray (dest_offset_row_col); otherwise it is copied cell by cell
// with the tile-side stride.  Here one workgroup takes a tile, computes the
// tile's intersection with the subarray, and copies it: slab-wise with
// 16/4/1-byte vectors (same order) or cell-wise (transposing order), into
// the device result buffer.  Scope of this first kernel: one fragment
// covering the subarray, one range per dimension, fixed-size cells; several
// fragments, fill values and var-sized cells follow below.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tiledb_amd.h"
#include "tdbg_device.h"

namespace tdbg {
namespace dense {

constexpr int NT = 256;

struct Box {
  int64_t lo[TDBG_DENSE_MAX_DIMS], len[TDBG_DENSE_MAX_DIMS];
};

// linear index of cell offsets c (relative) in a box of extents e, row-major
// (last dimension fastest) or col-major (first fastest)
__device__ __forceinline__ uint64_t lin(const int64_t* c, const int64_t* e, uint32_t nd, bool row) {
  uint64_t x = 0;
  if (row) {
    for (uint32_t d = 0; d < nd; d++) x = x * (uint64_t)e[d] + (uint64_t)c[d];
  } else {
    for (int d = (int)nd - 1; d >= 0; d--) x = x * (uint64_t)e[d] + (uint64_t)c[d];
  }
  return x;
}

__global__ void __launch_bounds__(NT) dense_copy_kernel(const tdbg_dense_copy_config cfg, uint64_t ntiles,
                                                        const int64_t* tile_start, const uint8_t* const* tiles,
                                                        const int32_t* status, uint8_t* result) {
  const uint32_t nd = cfg.dim_num;
  const bool trow = cfg.cell_order == 0, rrow = cfg.layout == 0;
  int64_t sub_ext[TDBG_DENSE_MAX_DIMS];
  for (uint32_t d = 0; d < nd; d++) sub_ext[d] = cfg.sub_hi[d] - cfg.sub_lo[d] + 1;
  const uint64_t cs = cfg.cell_size;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    if (status && status[t] != TDBG_OK) continue;
    const uint8_t* src = tiles[t];
    // the tile's box and its intersection with the subarray
    Box I;
    int64_t toff[TDBG_DENSE_MAX_DIMS];  // intersection start, relative to the tile
    bool empty = false;
    uint64_t ncell = 1;
    for (uint32_t d = 0; d < nd; d++) {
      const int64_t s = tile_start[t * nd + d];
      const int64_t a = s > cfg.sub_lo[d] ? s : cfg.sub_lo[d];
      const int64_t e = s + cfg.tile_extent[d] - 1;
      const int64_t b = e < cfg.sub_hi[d] ? e : cfg.sub_hi[d];
      if (b < a) empty = true;
      I.lo[d] = a;
      I.len[d] = b - a + 1;
      toff[d] = a - s;
      ncell *= empty ? 0 : (uint64_t)I.len[d];
    }
    if (empty || ncell == 0) continue;
    if (trow == rrow) {
      // slabs along the fastest dimension, contiguous on both sides
      const uint32_t f = trow ? nd - 1 : 0;
      const uint64_t slab = (uint64_t)I.len[f] * cs;
      const uint64_t nslab = ncell / (uint64_t)I.len[f];
      for (uint64_t k = 0; k < nslab; k++) {
        // slab k: the other dimensions' offsets, in the fastest-first order of the layout
        int64_t c[TDBG_DENSE_MAX_DIMS];
        uint64_t r = k;
        if (trow) {
          for (int d = (int)nd - 2; d >= 0; d--) {
            c[d] = (int64_t)(r % (uint64_t)I.len[d]);
            r /= (uint64_t)I.len[d];
          }
          c[nd - 1] = 0;
        } else {
          for (uint32_t d = 1; d < nd; d++) {
            c[d] = (int64_t)(r % (uint64_t)I.len[d]);
            r /= (uint64_t)I.len[d];
          }
          c[0] = 0;
        }
        int64_t ct[TDBG_DENSE_MAX_DIMS], cr[TDBG_DENSE_MAX_DIMS];
        for (uint32_t d = 0; d < nd; d++) {
          ct[d] = toff[d] + c[d];
          cr[d] = I.lo[d] - cfg.sub_lo[d] + c[d];
        }
        const uint8_t* s8 = src + lin(ct, cfg.tile_extent, nd, trow) * cs;
        uint8_t* d8 = result + lin(cr, sub_ext, nd, rrow) * cs;
        if (((((uintptr_t)s8) | ((uintptr_t)d8) | slab) & 15) == 0) {
          for (uint64_t i = threadIdx.x; i < slab / 16; i += NT) ((uint4*)d8)[i] = ((const uint4*)s8)[i];
        } else if (((((uintptr_t)s8) | ((uintptr_t)d8) | slab) & 3) == 0) {
          for (uint64_t i = threadIdx.x; i < slab / 4; i += NT) ((uint32_t*)d8)[i] = ((const uint32_t*)s8)[i];
        } else {
          for (uint64_t i = threadIdx.x; i < slab; i += NT) d8[i] = s8[i];
        }
      }
    } else {
      // different orders: cell by cell, consecutive threads on consecutive
      // result cells
      for (uint64_t k = threadIdx.x; k < ncell; k += NT) {
        int64_t c[TDBG_DENSE_MAX_DIMS];
        uint64_t r = k;
        if (rrow) {
          for (int d = (int)nd - 1; d >= 0; d--) {
            c[d] = (int64_t)(r % (uint64_t)I.len[d]);
            r /= (uint64_t)I.len[d];
          }
        } else {
          for (uint32_t d = 0; d < nd; d++) {
            c[d] = (int64_t)(r % (uint64_t)I.len[d]);
            r /= (uint64_t)I.len[d];
          }
        }
        int64_t ct[TDBG_DENSE_MAX_DIMS], cr[TDBG_DENSE_MAX_DIMS];
        for (uint32_t d = 0; d < nd; d++) {
          ct[d] = toff[d] + c[d];
          cr[d] = I.lo[d] - cfg.sub_lo[d] + c[d];
        }
        const uint8_t* s8 = src + lin(ct, cfg.tile_extent, nd, trow) * cs;
        uint8_t* d8 = result + lin(cr, sub_ext, nd, rrow) * cs;
        for (uint64_t i = 0; i < cs; i++) d8[i] = s8[i];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Several fragments and fill values (DenseReader::copy_fixed_tiles /
// copy_offset_tiles / fix_offsets_buffer / copy_var_tiles,
// dense_reader.cc:1199-1236, 1521-2000).  The reference walks a slab's
// fragment domains from the last to the first, each overwriting the cells it
// overlaps (cell_slab_overlaps_range :1521-1552: every coordinate inside the
// domain), and fills what the last one does not write: the surviving value of
// a cell is the first fragment (lowest fd) whose domain holds it and whose
// tile exists, else the fill value.  Here one workgroup takes a space tile
// and its threads take the result cells of the tile's part of the subarray
// in result order (consecutive threads, consecutive result cells), each
// finding its fragment and copying one cell.
// ---------------------------------------------------------------------------
struct Region {
  int64_t lo[TDBG_DENSE_MAX_DIMS], len[TDBG_DENSE_MAX_DIMS], toff[TDBG_DENSE_MAX_DIMS];
  uint64_t ncell;
};

__device__ __forceinline__ bool region_of(const tdbg_dense_copy_config& cfg, const int64_t* ts, Region& R) {
  const uint32_t nd = cfg.dim_num;
  R.ncell = 1;
  for (uint32_t d = 0; d < nd; d++) {
    const int64_t a = ts[d] > cfg.sub_lo[d] ? ts[d] : cfg.sub_lo[d];
    const int64_t e = ts[d] + cfg.tile_extent[d] - 1;
    const int64_t b = e < cfg.sub_hi[d] ? e : cfg.sub_hi[d];
    if (b < a) return false;
    R.lo[d] = a;
    R.len[d] = b - a + 1;
    R.toff[d] = a - ts[d];
    R.ncell *= (uint64_t)R.len[d];
  }
  return true;
}

// cell k of the region in result-layout order: its position in the tile
// (cell order) and in the result buffer (layout); the fragment that
// survives there (-1: the fill value)
__device__ __forceinline__ int cell_at(const tdbg_dense_copy_config& cfg, const Region& R, uint64_t k, uint32_t t,
                                       uint32_t nfrag, const int64_t* frag_dom, const uint8_t* const* present,
                                       uint64_t& pos, uint64_t& rc) {
  const uint32_t nd = cfg.dim_num;
  const bool trow = cfg.cell_order == 0, rrow = cfg.layout == 0;
  int64_t c[TDBG_DENSE_MAX_DIMS];
  uint64_t r = k;
  if (rrow) {
    for (int d = (int)nd - 1; d >= 0; d--) {
      c[d] = (int64_t)(r % (uint64_t)R.len[d]);
      r /= (uint64_t)R.len[d];
    }
  } else {
    for (uint32_t d = 0; d < nd; d++) {
      c[d] = (int64_t)(r % (uint64_t)R.len[d]);
      r /= (uint64_t)R.len[d];
    }
  }
  int64_t ct[TDBG_DENSE_MAX_DIMS], cr[TDBG_DENSE_MAX_DIMS], sub_ext[TDBG_DENSE_MAX_DIMS];
  for (uint32_t d = 0; d < nd; d++) {
    ct[d] = R.toff[d] + c[d];
    cr[d] = R.lo[d] - cfg.sub_lo[d] + c[d];
    sub_ext[d] = cfg.sub_hi[d] - cfg.sub_lo[d] + 1;
  }
  pos = lin(ct, cfg.tile_extent, nd, trow);
  rc = lin(cr, sub_ext, nd, rrow);
  for (uint32_t f = 0; f < nfrag; f++) {
    if (!present[(uint64_t)t * nfrag + f]) continue;
    const int64_t* dom = frag_dom + (uint64_t)f * nd * 2;
    bool in = true;
    for (uint32_t d = 0; d < nd; d++) {
      const int64_t x = R.lo[d] + c[d];
      in = in && x >= dom[2 * d] && x <= dom[2 * d + 1];
    }
    if (in) return (int)f;
  }
  return -1;
}

__device__ __forceinline__ void copy_bytes(uint8_t* d, const uint8_t* s, uint64_t n) {
  if (((((uintptr_t)d) | ((uintptr_t)s) | n) & 7) == 0) {
    for (uint64_t i = 0; i < n / 8; i++) ((uint64_t*)d)[i] = ((const uint64_t*)s)[i];
  } else if (((((uintptr_t)d) | ((uintptr_t)s) | n) & 3) == 0) {
    for (uint64_t i = 0; i < n / 4; i++) ((uint32_t*)d)[i] = ((const uint32_t*)s)[i];
  } else {
    for (uint64_t i = 0; i < n; i++) d[i] = s[i];
  }
}

// a present fragment's validity byte (a fragment given without a validity
// tile counts as valid)
__device__ __forceinline__ uint8_t valid_at(const uint8_t* const* validity, uint64_t i, uint64_t pos) {
  const uint8_t* v = validity ? validity[i] : nullptr;
  return v ? v[pos] : (uint8_t)1;
}

// The region R of a tile copied slab by slab (the tile's cell order equals
// the result layout): each run along the fastest dimension is contiguous on
// both sides, moved by the whole workgroup in 16/4/1-byte vectors
// (dense_reader.cc:1555-1748, a memcpy per cell slab).  cs = 1 with a NULL
// src writes `one` bytes (the validity of a fragment given without one).
__device__ void copy_region_slabs(const tdbg_dense_copy_config& cfg, const Region& R, const uint8_t* src,
                                  uint64_t cs, uint8_t* result, uint8_t one = 1) {
  const uint32_t nd = cfg.dim_num;
  const bool row = cfg.cell_order == 0;
  int64_t sub_ext[TDBG_DENSE_MAX_DIMS];
  for (uint32_t d = 0; d < nd; d++) sub_ext[d] = cfg.sub_hi[d] - cfg.sub_lo[d] + 1;
  const uint32_t f = row ? nd - 1 : 0;
  const uint64_t slab = (uint64_t)R.len[f] * cs;
  const uint64_t nslab = R.ncell / (uint64_t)R.len[f];
  for (uint64_t k = 0; k < nslab; k++) {
    int64_t c[TDBG_DENSE_MAX_DIMS];
    uint64_t r = k;
    if (row) {
      for (int d = (int)nd - 2; d >= 0; d--) {
        c[d] = (int64_t)(r % (uint64_t)R.len[d]);
        r /= (uint64_t)R.len[d];
      }
      c[nd - 1] = 0;
    } else {
      for (uint32_t d = 1; d < nd; d++) {
        c[d] = (int64_t)(r % (uint64_t)R.len[d]);
        r /= (uint64_t)R.len[d];
      }
      c[0] = 0;
    }
    int64_t ct[TDBG_DENSE_MAX_DIMS], cr[TDBG_DENSE_MAX_DIMS];
    for (uint32_t d = 0; d < nd; d++) {
      ct[d] = R.toff[d] + c[d];
      cr[d] = R.lo[d] - cfg.sub_lo[d] + c[d];
    }
    uint8_t* d8 = result + lin(cr, sub_ext, nd, row) * cs;
    if (!src) {
      for (uint64_t i = threadIdx.x; i < slab; i += NT) d8[i] = one;
      continue;
    }
    const uint8_t* s8 = src + lin(ct, cfg.tile_extent, nd, row) * cs;
    if (((((uintptr_t)s8) | ((uintptr_t)d8) | slab) & 15) == 0) {
      for (uint64_t i = threadIdx.x; i < slab / 16; i += NT) ((uint4*)d8)[i] = ((const uint4*)s8)[i];
    } else if (((((uintptr_t)s8) | ((uintptr_t)d8) | slab) & 3) == 0) {
      for (uint64_t i = threadIdx.x; i < slab / 4; i += NT) ((uint32_t*)d8)[i] = ((const uint32_t*)s8)[i];
    } else {
      for (uint64_t i = threadIdx.x; i < slab; i += NT) d8[i] = s8[i];
    }
  }
}

// the fragment's domain holds every cell of R
__device__ __forceinline__ bool dom_covers(const int64_t* dom, const Region& R, uint32_t nd) {
  bool in = true;
  for (uint32_t d = 0; d < nd; d++) in = in && dom[2 * d] <= R.lo[d] && dom[2 * d + 1] >= R.lo[d] + R.len[d] - 1;
  return in;
}

__global__ void __launch_bounds__(NT) dense_frag_copy_kernel(const tdbg_dense_frag_config fc, uint64_t ntiles,
                                                             const int64_t* tile_start, const int64_t* frag_dom,
                                                             const uint8_t* const* tiles,
                                                             const uint8_t* const* validity,
                                                             const uint8_t* fill, uint8_t* result,
                                                             uint8_t* result_validity) {
  const tdbg_dense_copy_config& cfg = fc.base;
  const uint64_t cs = cfg.cell_size;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    Region R;
    if (!region_of(cfg, tile_start + t * cfg.dim_num, R)) continue;
    // one fragment whose tile exists and whose domain holds the whole region,
    // in the result's order: slab copies (the common single-fragment read)
    if (fc.nfrag == 1 && tiles[t] && cfg.cell_order == cfg.layout && dom_covers(frag_dom, R, cfg.dim_num)) {
      copy_region_slabs(cfg, R, tiles[t], cs, result);
      if (fc.nullable && result_validity)
        copy_region_slabs(cfg, R, validity ? validity[t] : nullptr, 1, result_validity, 1);
      continue;
    }
    for (uint64_t k = threadIdx.x; k < R.ncell; k += NT) {
      uint64_t pos, rc;
      const int f = cell_at(cfg, R, k, (uint32_t)t, fc.nfrag, frag_dom, tiles, pos, rc);
      const uint8_t* src = f >= 0 ? tiles[t * fc.nfrag + f] + pos * cs : fill;
      copy_bytes(result + rc * cs, src, cs);
      if (fc.nullable && result_validity)
        result_validity[rc] = f < 0 ? (uint8_t)fc.fill_validity : valid_at(validity, t * fc.nfrag + f, pos);
    }
  }
}

// every result cell starts as the fill value (and the fill validity): cells
// that no given space tile covers keep it
__global__ void __launch_bounds__(NT) dense_fill_kernel(uint64_t n, uint64_t cs, const uint8_t* fill, uint8_t* result,
                                                        uint8_t* result_validity, uint8_t fill_validity) {
  for (uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (uint64_t)gridDim.x * NT) {
    copy_bytes(result + i * cs, fill, cs);
    if (result_validity) result_validity[i] = fill_validity;
  }
}

// var cells: every result cell starts as the fill value's size and bytes
__global__ void __launch_bounds__(NT) dense_var_fill_kernel(uint64_t n, uint64_t fill_units, const uint8_t* fill,
                                                            uint64_t* offsets, uint64_t* src,
                                                            uint8_t* result_validity, uint8_t fill_validity) {
  for (uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (uint64_t)gridDim.x * NT) {
    offsets[i] = fill_units;
    src[i] = (uint64_t)fill;
    if (result_validity) result_validity[i] = fill_validity;
  }
}

// copy_offset_tiles + the sentinel half of fix_offsets_buffer: each result
// cell's size (in elements in elements mode) into offsets[rc] and the address
// of its bytes into src[rc] (the fill value for cells no fragment writes)
__global__ void __launch_bounds__(NT) dense_var_sizes_kernel(const tdbg_dense_frag_config fc, uint64_t ntiles,
                                                             const int64_t* tile_start, const int64_t* frag_dom,
                                                             const uint8_t* const* off_tiles,
                                                             const uint8_t* const* var_tiles,
                                                             const uint8_t* const* validity, const uint8_t* fill,
                                                             uint64_t* offsets, uint64_t* src,
                                                             uint8_t* result_validity, uint32_t* err) {
  const tdbg_dense_copy_config& cfg = fc.base;
  const uint64_t div = fc.elements_mode ? fc.data_type_size : 1;
  const uint64_t fill_units = fc.fill_size / div;
  uint64_t tcells = 1;  // cells per tile: the offsets tile's last entry is the var tile's size
  for (uint32_t d = 0; d < cfg.dim_num; d++) tcells *= (uint64_t)cfg.tile_extent[d];
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    Region R;
    if (!region_of(cfg, tile_start + t * cfg.dim_num, R)) continue;
    for (uint64_t k = threadIdx.x; k < R.ncell; k += NT) {
      uint64_t pos, rc;
      const int f = cell_at(cfg, R, k, (uint32_t)t, fc.nfrag, frag_dom, off_tiles, pos, rc);
      if (f >= 0) {
        const uint64_t* o = (const uint64_t*)off_tiles[t * fc.nfrag + f];
        const uint64_t o0 = o[pos], o1 = o[pos + 1];
        if (o0 <= o1 && o1 <= o[tcells]) {
          offsets[rc] = (o1 - o0) / div;
          src[rc] = (uint64_t)(var_tiles[t * fc.nfrag + f] + o0);
        } else {
          // offsets outside the var tile: no read past it; the read fails
          // (TDBG_E_DATA_READ) when the caller checks err
          offsets[rc] = 0;
          src[rc] = (uint64_t)fill;
          if (err) *err = 1;
        }
      } else {
        offsets[rc] = fill_units;
        src[rc] = (uint64_t)fill;
      }
      if (fc.nullable && result_validity)
        result_validity[rc] = f < 0 ? (uint8_t)fc.fill_validity : valid_at(validity, t * fc.nfrag + f, pos);
    }
  }
}

// exclusive scan of n uint64 in place (fix_offsets_buffer's running
// var_buffer_size): SB = 2,048 values per block
constexpr uint32_t SB = NT * 8;

__device__ __forceinline__ uint64_t block_scan_ex(uint64_t v, uint64_t& total, uint64_t* red) {
  return block_exscan_u64<NT>(v, total, red);
}

__global__ void __launch_bounds__(NT) scan_sums_kernel(const uint64_t* x, uint64_t n, uint64_t* bsum) {
  __shared__ uint64_t red[NT / 64];
  const uint64_t b0 = (uint64_t)blockIdx.x * SB;
  uint64_t s = 0;
  for (uint32_t i = 0; i < 8; i++) {
    const uint64_t j = b0 + (uint64_t)threadIdx.x * 8 + i;
    s += j < n ? x[j] : 0;
  }
  uint64_t tot;
  (void)block_scan_ex(s, tot, red);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// one workgroup: exclusive prefix of the block sums (in place) and the total
__global__ void __launch_bounds__(NT) scan_prefix_kernel(uint64_t* bsum, uint64_t nb, uint64_t* total) {
  __shared__ uint64_t red[NT / 64];
  uint64_t carry = 0;
  for (uint64_t base = 0; base < nb; base += NT) {
    const uint64_t j = base + threadIdx.x;
    const uint64_t v = j < nb ? bsum[j] : 0;
    uint64_t tot;
    const uint64_t ex = block_scan_ex(v, tot, red);
    if (j < nb) bsum[j] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) *total = carry;
}

__global__ void __launch_bounds__(NT) scan_apply_kernel(uint64_t* x, uint64_t n, const uint64_t* bsum) {
  __shared__ uint64_t red[NT / 64];
  const uint64_t b0 = (uint64_t)blockIdx.x * SB;
  uint64_t v[8], s = 0;
  for (uint32_t i = 0; i < 8; i++) {
    const uint64_t j = b0 + (uint64_t)threadIdx.x * 8 + i;
    v[i] = j < n ? x[j] : 0;
    s += v[i];
  }
  uint64_t tot;
  uint64_t run = bsum[blockIdx.x] + block_scan_ex(s, tot, red);
  for (uint32_t i = 0; i < 8; i++) {
    const uint64_t j = b0 + (uint64_t)threadIdx.x * 8 + i;
    if (j < n) x[j] = run;
    run += v[i];
  }
}

// copy_var_tiles: every result cell's bytes to its offset (times the type
// size in elements mode); the last cell ends at the total
__global__ void __launch_bounds__(NT) dense_var_copy_kernel(const uint64_t* offsets, const uint64_t* src, uint64_t n,
                                                            const uint64_t* total, uint64_t mult, uint8_t* var_out) {
  const uint64_t tot = *total;
  for (uint64_t i = (uint64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (uint64_t)gridDim.x * NT) {
    const uint64_t o = offsets[i];
    const uint64_t e = i + 1 < n ? offsets[i + 1] : tot;
    copy_bytes(var_out + o * mult, (const uint8_t*)src[i], (e - o) * mult);
  }
}

}  // namespace dense
}  // namespace tdbg

extern "C" hipError_t tdbg_launch_dense_copy(const tdbg_dense_copy_config* cfg, uint64_t ntiles,
                                             const int64_t* tile_start, const uint8_t* const* tiles,
                                             const int32_t* status, uint8_t* result, uint32_t grid,
                                             hipStream_t s) {
  if (ntiles == 0) return hipSuccess;
  hipLaunchKernelGGL(tdbg::dense::dense_copy_kernel, dim3(grid), dim3(tdbg::dense::NT), 0, s, *cfg, ntiles,
                     tile_start, tiles, status, result);
  return hipGetLastError();
}

extern "C" hipError_t tdbg_launch_dense_frag_copy(const tdbg_dense_frag_config* fc, uint64_t ntiles,
                                                  const int64_t* tile_start, const int64_t* frag_dom,
                                                  const uint8_t* const* tiles, const uint8_t* const* validity,
                                                  const uint8_t* fill, uint8_t* result, uint8_t* result_validity,
                                                  uint64_t ncells, uint32_t grid, hipStream_t s) {
  using namespace tdbg::dense;
  if (ncells) {
    const uint32_t fg = (uint32_t)((ncells + NT - 1) / NT < 4096 ? (ncells + NT - 1) / NT : 4096);
    hipLaunchKernelGGL(dense_fill_kernel, dim3(fg), dim3(NT), 0, s, ncells, (uint64_t)fc->base.cell_size, fill,
                       result, fc->nullable ? result_validity : nullptr, (uint8_t)fc->fill_validity);
  }
  if (ntiles)
    hipLaunchKernelGGL(dense_frag_copy_kernel, dim3(grid), dim3(NT), 0, s, *fc, ntiles, tile_start, frag_dom, tiles,
                       validity, fill, result, result_validity);
  return hipGetLastError();
}

// sizes -> exclusive offsets in place (+ total); bsum: (n + 2047) / 2048 entries
extern "C" hipError_t tdbg_launch_dense_var_offsets(const tdbg_dense_frag_config* fc, uint64_t ntiles,
                                                    const int64_t* tile_start, const int64_t* frag_dom,
                                                    const uint8_t* const* off_tiles, const uint8_t* const* var_tiles,
                                                    const uint8_t* const* validity, const uint8_t* fill,
                                                    uint64_t* offsets, uint64_t ncells, uint64_t* src,
                                                    uint8_t* result_validity, uint64_t* bsum, uint64_t* total,
                                                    uint32_t* err, uint32_t grid, hipStream_t s) {
  using namespace tdbg::dense;
  if (ncells) {
    const uint32_t fg = (uint32_t)((ncells + NT - 1) / NT < 4096 ? (ncells + NT - 1) / NT : 4096);
    const uint64_t div = fc->elements_mode ? fc->data_type_size : 1;
    hipLaunchKernelGGL(dense_var_fill_kernel, dim3(fg), dim3(NT), 0, s, ncells, (uint64_t)fc->fill_size / div, fill,
                       offsets, src, fc->nullable ? result_validity : nullptr, (uint8_t)fc->fill_validity);
  }
  if (ntiles)
    hipLaunchKernelGGL(dense_var_sizes_kernel, dim3(grid), dim3(NT), 0, s, *fc, ntiles, tile_start, frag_dom,
                       off_tiles, var_tiles, validity, fill, offsets, src, result_validity, err);
  const uint64_t nb = (ncells + SB - 1) / SB;
  if (nb) hipLaunchKernelGGL(scan_sums_kernel, dim3((uint32_t)nb), dim3(NT), 0, s, offsets, ncells, bsum);
  hipLaunchKernelGGL(scan_prefix_kernel, dim3(1), dim3(NT), 0, s, bsum, nb, total);
  if (nb) hipLaunchKernelGGL(scan_apply_kernel, dim3((uint32_t)nb), dim3(NT), 0, s, offsets, ncells, bsum);
  return hipGetLastError();
}

extern "C" hipError_t tdbg_launch_dense_var_copy(const uint64_t* offsets, const uint64_t* src, uint64_t ncells,
                                                 const uint64_t* total, uint64_t mult, uint8_t* var_out,
                                                 uint32_t grid, hipStream_t s) {
  if (ncells == 0) return hipSuccess;
  hipLaunchKernelGGL(tdbg::dense::dense_var_copy_kernel, dim3(grid), dim3(tdbg::dense::NT), 0, s, offsets, src,
                     ncells, total, mult, var_out);
  return hipGetLastError();
}
