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
// the device result buffer.  Scope: one fragment covering the subarray, one
// range per dimension, fixed-size cells -- the single-fragment dense read;
// several overlapping fragments and fill values stay in the reader.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tiledb_amd.h"

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
