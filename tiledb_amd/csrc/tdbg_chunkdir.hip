// tdbg_chunkdir.hip -- the device chunk directory for chunk-parallel launches
// (TDBG_CHUNK_PARALLEL): Tile::load_chunk_data (tile.cc:280-313) for every
// tile of a launch, then a directory of chunk records that the fused kernel
// takes as work items -- the tile x chunk-range split of the reference's
// unfilter_tiles (reader_base.cc:970-989) mapped onto workgroups.
//
//   dir_count  one thread per tile: header walk, status, chunk count
//   dir_scan   one workgroup: exclusive scan of the counts -> record bases;
//              tiles whose records do not fit the directory are queued for
//              the general interpreter (status TDBG_E_FALLBACK)
//   dir_fill   one thread per tile: the tile's chunk records
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tiledb_amd.h"
#include "tdbg_desc.h"
#include "tdbg_device.h"

namespace tdbg {

// The tile-header checks of the fused kernel's tile path (tdbg_fast.hip) in
// the same order; on success *nch = the chunk count.
__device__ int tile_walk(const KParams& kp, uint64_t t, uint64_t* nch, uint64_t* expected_out) {
  const uint8_t* in = kp.in[t];
  const uint64_t fs = kp.in_size[t], os = kp.out_size[t];
  uint64_t expected = os;
  if (kp.flags & TDBG_TILE_OFFSETS) {
    if (os < 8) return TDBG_E_TILE_SIZE;
    expected = os - 8;
  }
  *expected_out = expected;
  if (fs < 8) return TDBG_E_TILE_FORMAT;
  const uint64_t n = ldn(in, 8);
  uint64_t o = 8, total = 0;
  for (uint64_t i = 0; i < n; i++) {
    if (o + 12 > fs) return TDBG_E_TILE_FORMAT;
    const uint64_t orig = ldn(in + o, 4), fl = ldn(in + o + 4, 4), ml = ldn(in + o + 8, 4);
    o += 12;
    if (ml > fs - o) return TDBG_E_TILE_FORMAT;
    o += ml;
    if (fl > fs - o) return TDBG_E_TILE_FORMAT;
    o += fl;
    total += orig;
  }
  if (total != expected) return TDBG_E_TILE_SIZE;
  *nch = n;
  return TDBG_OK;
}

__global__ void dir_count_kernel(const KParams kp, uint32_t* cnt) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= kp.ntiles) return;
  uint64_t nch = 0, expected = 0;
  const int rc = tile_walk(kp, t, &nch, &expected);
  kp.status[t] = rc;
  // (a chunk count past 2^32 - 1 cannot be placed: the tile goes to the
  // general interpreter through the directory overflow below)
  cnt[t] = rc == TDBG_OK ? (uint32_t)(nch < 0xffffffffull ? nch : 0xffffffffull) : 0u;
}

constexpr int DIR_NT = 1024;

__global__ void __launch_bounds__(DIR_NT) dir_scan_kernel(const KParams kp, uint32_t* cnt, uint32_t* base,
                                                          uint32_t cap, uint32_t* total, uint64_t* need) {
  __shared__ uint64_t red[DIR_NT / 64];
  __shared__ uint32_t placed;  // records written: the placed tiles are a prefix
  if (threadIdx.x == 0) placed = 0;
  __syncthreads();
  uint64_t carry = 0, ok_tiles = 0, ok_bytes = 0;
  for (uint64_t b0 = 0; b0 < kp.ntiles; b0 += DIR_NT) {
    const uint64_t t = b0 + threadIdx.x;
    const bool v = t < kp.ntiles;
    uint64_t c = v ? cnt[t] : 0;
    uint64_t tot;
    const uint64_t ex = carry + block_exscan_u64<DIR_NT>(c, tot, red);
    if (v) {
      if (ex + c > cap) {
        // no room in the directory: the general interpreter takes the tile
        cnt[t] = 0;
        if (kp.status[t] == TDBG_OK) {
          kp.status[t] = TDBG_E_FALLBACK;
          const uint32_t k = atomicAdd(kp.fbq, 1u);
          if (k < kp.fbq_cap) kp.fbq[1 + k] = (uint32_t)t;
        }
      } else {
        base[t] = (uint32_t)ex;
        if (c) atomicMax(&placed, (uint32_t)(ex + c));
      }
      if (kp.status[t] == TDBG_OK) {
        ok_tiles++;
        ok_bytes += kp.out_size[t];
      }
    }
    carry += tot;
    __syncthreads();
  }
  // once a tile overflows every later one does (the bases only grow), so
  // the records [0, placed) are exactly the placed tiles' chunks
  __syncthreads();
  if (threadIdx.x == 0) {
    *total = placed;
    // the records this launch asked for (host-mapped: the next launch on the
    // context sizes its directory from it, without a host wait here)
    if (need && carry > *need) *need = carry;
  }
  // fused-path counters: every tile the directory accepted; a chunk that
  // falls back later takes its tile out again (tdbg_fast.hip)
  if (kp.stats && (ok_tiles | ok_bytes)) {
    atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_FUSED_TILES], (unsigned long long)ok_tiles);
    atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_FUSED_BYTES], (unsigned long long)ok_bytes);
  }
}

__global__ void dir_fill_kernel(const KParams kp, const uint32_t* cnt, const uint32_t* base, ChunkRec* recs) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= kp.ntiles || cnt[t] == 0 || kp.status[t] != TDBG_OK) return;
  const uint8_t* in = kp.in[t];
  const uint32_t n = cnt[t], b = base[t];
  uint64_t o = 8, coff = 0;
  for (uint32_t i = 0; i < n; i++) {
    ChunkRec r;
    r.tile = (uint32_t)t;
    r.orig = (uint32_t)ldn(in + o, 4);
    r.fl = (uint32_t)ldn(in + o + 4, 4);
    r.ml = (uint32_t)ldn(in + o + 8, 4);
    o += 12;
    r.in_off = o;
    r.out_off = coff;
    recs[b + i] = r;
    o += (uint64_t)r.ml + r.fl;
    coff += r.orig;
  }
}

}  // namespace tdbg

extern "C" hipError_t tdbg_launch_chunk_dir(const tdbg::KParams* kp, uint32_t* cnt, uint32_t* base,
                                            tdbg::ChunkRec* recs, uint32_t cap, uint32_t* total,
                                            uint64_t* need, hipStream_t stream) {
  if (kp->ntiles == 0) return hipSuccess;
  const uint32_t grid = (uint32_t)((kp->ntiles + 255) / 256);
  hipLaunchKernelGGL(tdbg::dir_count_kernel, dim3(grid), dim3(256), 0, stream, *kp, cnt);
  hipLaunchKernelGGL(tdbg::dir_scan_kernel, dim3(1), dim3(tdbg::DIR_NT), 0, stream, *kp, cnt, base, cap, total,
                     need);
  hipLaunchKernelGGL(tdbg::dir_fill_kernel, dim3(grid), dim3(256), 0, stream, *kp, cnt, base, recs);
  return hipGetLastError();
}
