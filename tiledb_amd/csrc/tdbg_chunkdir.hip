// tdbg_chunkdir.hip -- the device chunk directory for chunk-parallel launches
// (TDBG_CHUNK_PARALLEL): Tile::load_chunk_data (tile.cc:280-313) for every
// tile of a launch, then a directory of chunk records that the fused kernel
// takes as work items -- the tile x chunk-range split of the reference's
// unfilter_tiles (reader_base.cc:970-989) mapped onto workgroups.
//
//   dir_count  one thread per tile: the tile header's chunk count (u64 at
//              byte 0), with the checks that need no walk (launches of up
//              to 4,096 tiles: done by dir_scan itself)
//   dir_scan   one workgroup: exclusive scan of the counts -> record bases;
//              tiles whose records do not fit the directory are queued for
//              the general interpreter (status TDBG_E_FALLBACK)
//   dir_fill   one thread per tile: the header walk (the chunk headers are a
//              chain: chunk i + 1 starts after chunk i's metadata and data,
//              one dependent load per chunk) that validates the tile and
//              writes its records on the way.  A tile the walk rejects gets
//              its status, and its records become empty ones no kernel takes.
//              One walk per tile, not two: a 4 MiB tile's 64-chunk chain is
//              ~40 us of load latency.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tiledb_amd.h"
#include "tdbg_desc.h"
#include "tdbg_device.h"

namespace tdbg {

// The checks of the fused kernel's tile path (tdbg_fast.hip), in the same
// order, that need no chunk walk.  A count past (fs - 8) / 12 cannot be
// walked (every chunk header is 12 bytes): the walk would stop with
// TDBG_E_TILE_FORMAT, so that is the status.
__device__ int tile_head(const KParams& kp, uint64_t t, uint64_t* nch) {
  const uint64_t fs = kp.in_size[t], os = kp.out_size[t];
  if ((kp.flags & TDBG_TILE_OFFSETS) && os < 8) return TDBG_E_TILE_SIZE;
  if (fs < 8) return TDBG_E_TILE_FORMAT;
  const uint64_t n = ldn(kp.in[t], 8);
  if (n > (fs - 8) / 12) return TDBG_E_TILE_FORMAT;
  *nch = n;
  return TDBG_OK;
}

__global__ void dir_count_kernel(const KParams kp, uint32_t* cnt) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= kp.ntiles) return;
  uint64_t nch = 0;
  const int rc = tile_head(kp, t, &nch);
  kp.status[t] = rc;
  // (a chunk count past 2^32 - 1 cannot be placed: the tile goes to the
  // general interpreter through the directory overflow below)
  cnt[t] = rc == TDBG_OK ? (uint32_t)(nch < 0xffffffffull ? nch : 0xffffffffull) : 0u;
}

constexpr int DIR_NT = 1024;

// heads: the launch has few tiles, so this kernel reads the tile headers
// itself (dir_count's work) instead of a launch of its own.  The launch's
// queue counts start here (fbq: this kernel is the first to append; cq: the
// streaming kernels' chunk queue), instead of two memset launches.
__global__ void __launch_bounds__(DIR_NT) dir_scan_kernel(const KParams kp, uint32_t* cnt, uint32_t* base,
                                                          uint32_t cap, uint32_t* total, uint64_t* need,
                                                          uint32_t* cq, int heads) {
  __shared__ uint64_t red[DIR_NT / 64];
  __shared__ uint32_t placed;  // records written: the placed tiles are a prefix
  if (threadIdx.x == 0) {
    placed = 0;
    if (kp.fbq) atomicExch(kp.fbq, 0u);
    if (cq) atomicExch(cq, 0u);
    __threadfence();  // (the other threads' appends below come after these)
  }
  __syncthreads();
  uint64_t carry = 0, ok_tiles = 0, ok_bytes = 0;
  for (uint64_t b0 = 0; b0 < kp.ntiles; b0 += DIR_NT) {
    const uint64_t t = b0 + threadIdx.x;
    const bool v = t < kp.ntiles;
    uint64_t c = 0;
    if (v && heads) {
      uint64_t nch = 0;
      const int rc = tile_head(kp, t, &nch);
      kp.status[t] = rc;
      c = rc == TDBG_OK ? (nch < 0xffffffffull ? nch : 0xffffffffull) : 0;
      cnt[t] = (uint32_t)c;
    } else if (v) {
      c = cnt[t];
    }
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

// The chunk walk of Tile::load_chunk_data (tile.cc:280-313) with the fused
// kernel's checks in its order (chunk header past the end, metadata or data
// past the end: TDBG_E_TILE_FORMAT; chunk sizes not summing to the tile:
// TDBG_E_TILE_SIZE), writing the records as it goes.
__global__ void dir_fill_kernel(const KParams kp, const uint32_t* cnt, const uint32_t* base, ChunkRec* recs) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= kp.ntiles || kp.status[t] != TDBG_OK) return;  // (rejected, or overflowed to the interpreter)
  const uint8_t* in = kp.in[t];
  const uint64_t fs = kp.in_size[t], os = kp.out_size[t];
  const uint64_t expected = (kp.flags & TDBG_TILE_OFFSETS) ? os - 8 : os;
  const uint32_t n = cnt[t], b = base[t];
  uint64_t o = 8, coff = 0;
  int rc = TDBG_OK;
  for (uint32_t i = 0; i < n; i++) {
    if (o + 12 > fs) {
      rc = TDBG_E_TILE_FORMAT;
      break;
    }
    // the 12-byte chunk header: four dword loads in flight at once (the
    // walk's one dependent latency per chunk)
    const uintptr_t a = (uintptr_t)(in + o);
    const uint32_t* q = (const uint32_t*)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t q0 = q[0], q1 = q[1], q2 = q[2], q3 = sh ? q[3] : 0u;
    ChunkRec r;
    r.tile = (uint32_t)t;
    r.orig = __builtin_amdgcn_alignbyte(q1, q0, sh);
    r.fl = __builtin_amdgcn_alignbyte(q2, q1, sh);
    r.ml = __builtin_amdgcn_alignbyte(q3, q2, sh);
    o += 12;
    if (r.ml > fs - o) {
      rc = TDBG_E_TILE_FORMAT;
      break;
    }
    r.in_off = o;
    o += r.ml;
    if (r.fl > fs - o) {
      rc = TDBG_E_TILE_FORMAT;
      break;
    }
    o += r.fl;
    r.out_off = coff;
    coff += r.orig;
    recs[b + i] = r;
  }
  if (rc == TDBG_OK && coff != expected) rc = TDBG_E_TILE_SIZE;
  if (rc == TDBG_OK) return;
  kp.status[t] = rc;
  // the tile's records: empty chunks of an impossible size (every streaming
  // kernel takes only 64 KiB outputs and queues the rest; the fused kernel
  // skips chunks of tiles whose status is not OK), so none touches its output
  ChunkRec z;
  z.tile = (uint32_t)t;
  z.orig = 0xffffffffu;
  z.fl = 0;
  z.ml = 0;
  z.in_off = 12;
  z.out_off = 0;
  for (uint32_t i = 0; i < n; i++) recs[b + i] = z;
  // the directory counted the tile as the fused path's
  if (kp.stats) {
    atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_FUSED_TILES], ~0ull);
    atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_FUSED_BYTES], (unsigned long long)(0 - os));
  }
}

}  // namespace tdbg

extern "C" hipError_t tdbg_launch_chunk_dir(const tdbg::KParams* kp, uint32_t* cnt, uint32_t* base,
                                            tdbg::ChunkRec* recs, uint32_t cap, uint32_t* total,
                                            uint64_t* need, uint32_t* cq, hipStream_t stream) {
  if (kp->ntiles == 0) {  // (the queue counts still start at zero)
    if (kp->fbq && hipMemsetAsync(kp->fbq, 0, 4, stream) != hipSuccess) return hipGetLastError();
    if (cq && hipMemsetAsync(cq, 0, 4, stream) != hipSuccess) return hipGetLastError();
    return hipSuccess;
  }
  // up to 4,096 tiles the scan workgroup reads the headers itself (four
  // rounds of one load each); more get the parallel count launch
  const int heads = kp->ntiles <= 4 * tdbg::DIR_NT;
  const uint32_t grid = (uint32_t)((kp->ntiles + 255) / 256);
  if (!heads) hipLaunchKernelGGL(tdbg::dir_count_kernel, dim3(grid), dim3(256), 0, stream, *kp, cnt);
  hipLaunchKernelGGL(tdbg::dir_scan_kernel, dim3(1), dim3(tdbg::DIR_NT), 0, stream, *kp, cnt, base, cap, total,
                     need, cq, heads);
  // the walk: one wave per 64 tiles, spread over CUs (a few hundred
  // multi-chunk tiles would otherwise share one CU's load path)
  const uint32_t wgrid = (uint32_t)((kp->ntiles + 63) / 64);
  hipLaunchKernelGGL(tdbg::dir_fill_kernel, dim3(wgrid), dim3(64), 0, stream, *kp, cnt, base, recs);
  return hipGetLastError();
}
