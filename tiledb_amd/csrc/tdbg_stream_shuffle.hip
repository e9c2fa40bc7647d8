// tdbg_stream_shuffle.hip -- streaming unfilter kernel for BASELINE C1
// [BYTESHUFFLE] on 4-byte values (one 64 KiB chunk per tile), gfx950.
//
// Byteshuffle⁻¹ (byteshuffle_filter.cc:111-166 -> blosc2 unshuffle) builds
// output unit j (16 bytes, elements 4j..4j+3) from dword j of each of the
// four byte planes.  Every unit is independent, so a tile is split over 16
// workgroups of 256 units each and nothing is staged: a thread loads its
// unit's four plane dwords (lane-consecutive, coalesced; realigned with
// v_alignbyte since tiles sit back to back at any byte offset), transposes
// them with v_perm and stores 16 bytes (lane-consecutive, nontemporal).  A
// C1 launch (256 tiles) is 4,096 workgroups instead of one tile-serial
// workgroup per tile, so it is no longer bound by one workgroup's latency
// chain.
//
// Any one-chunk tile of 4 n bytes (n <= 16,384 values: every tile of at
// most 64 KiB is one chunk, tile.cc:87-100) is taken: plane k starts at
// data byte k n (any alignment), the last unit is partial when n is not a
// multiple of 4, and outputs need only be 4-B aligned.  Each workgroup checks
// its tile's header (Tile::load_chunk_data, tile.cc:280-313; the byteshuffle
// metadata [u32 1][u32 4 n]); a tile of any other shape is queued by its
// first workgroup for the fused kernel, which runs on the queue right after,
// so statuses and bytes stay the reference's.  A workgroup writes only when
// the whole header validated.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tiledb_amd.h"
#include "tdbg_desc.h"
#include "tdbg_launch.h"

namespace tdbg {
namespace shf {

constexpr int NT = 256;
constexpr uint32_t OUTB = 65536;
constexpr uint32_t PARTS = OUTB / 16 / NT;  // workgroups per tile (16)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v4a __attribute__((ext_vector_type(4))) __attribute__((aligned(4)));
typedef __attribute__((address_space(1))) v4a g_a4;
typedef __attribute__((address_space(1))) const uint32_t g_cu32;

// bytes [p, p + 4) at any alignment, from the dwords that hold them (only
// the first when p is aligned: nothing past the tile is read)
__device__ __forceinline__ uint32_t ld32u(const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p;
  const g_cu32* q = (const g_cu32*)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  return sh ? __builtin_amdgcn_alignbyte(q[1], q[0], sh) : q[0];
}

__global__ void __launch_bounds__(NT) unfilter_shuffle4_kernel(const KParams kp) {
  // the fused kernel's fallback queue starts empty for this launch (it runs
  // next on the queue, in stream order, and is the only one to append)
  if (kp.fbq && blockIdx.x == 0 && threadIdx.x == 0) kp.fbq[0] = 0;
  const uint64_t t = blockIdx.x / PARTS;
  const uint32_t part = blockIdx.x % PARTS;
  if (t >= kp.ntiles) return;
  const uint8_t* in = kp.in[t];
  uint8_t* out = kp.out[t];
  const uint64_t fs = kp.in_size[t], os = kp.out_size[t];
  bool ok = !(kp.flags & TDBG_TILE_OFFSETS) && os >= 16 && os <= OUTB && (os & 3) == 0 &&
            (((uintptr_t)out) & 3) == 0 && fs >= 28 + os;
  if (ok) {
    // [u64 nchunks = 1][u32 orig][u32 filtered][u32 md][md = u32 1, u32 os]
    // (uniform loads; the image holds at least 28 + os bytes)
    const uint32_t nlo = ld32u(in), nhi = ld32u(in + 4), orig = ld32u(in + 8), fl = ld32u(in + 12),
                   ml = ld32u(in + 16), np = ld32u(in + 20), ps = ld32u(in + 24);
    ok = nlo == 1 && nhi == 0 && orig == os && fl == os && ml == 8 && np == 1 && ps == os &&
         (uint64_t)20 + ml + fl <= fs;
  }
  if (!ok) {
    if (part == 0 && threadIdx.x == 0) {
      const uint32_t k = atomicAdd(kp.sq, 1u);
      if (k < kp.sq_cap) kp.sq[1 + k] = (uint32_t)t;
      else if (kp.status) kp.status[t] = TDBG_E_INTERNAL;
    }
    return;
  }
  const uint32_t n = (uint32_t)os >> 2;       // values
  const uint32_t j = part * NT + threadIdx.x;  // output unit
  if (j >= (n + 3) >> 2) return;
  const uint8_t* d = in + 28 + 4 * j;
  uint32_t p0, p1, p2, p3;
  if (j < (n >> 2)) {
    p0 = ld32u(d), p1 = ld32u(d + n), p2 = ld32u(d + 2 * n), p3 = ld32u(d + 3 * n);
  } else {
    // the partial last unit: only the planes' n mod 4 remaining bytes (no
    // read past the tile image)
    const uint32_t r = n & 3;
    auto part_ld = [&](const uint8_t* q) -> uint32_t {
      uint32_t v = q[0];
      if (r > 1) v |= (uint32_t)q[1] << 8;
      if (r > 2) v |= (uint32_t)q[2] << 16;
      return v;
    };
    p0 = part_ld(d), p1 = part_ld(d + n), p2 = part_ld(d + 2 * n), p3 = part_ld(d + 3 * n);
  }
  // out dword b byte k = plane k byte b
  const uint32_t a = __builtin_amdgcn_perm(p1, p0, 0x05010400u);
  const uint32_t b = __builtin_amdgcn_perm(p3, p2, 0x05010400u);
  const uint32_t c = __builtin_amdgcn_perm(p1, p0, 0x07030602u);
  const uint32_t e = __builtin_amdgcn_perm(p3, p2, 0x07030602u);
  const v4u y{__builtin_amdgcn_perm(b, a, 0x05040100u), __builtin_amdgcn_perm(b, a, 0x07060302u),
              __builtin_amdgcn_perm(e, c, 0x05040100u), __builtin_amdgcn_perm(e, c, 0x07060302u)};
  if (j < (n >> 2)) {
    __builtin_nontemporal_store((v4a)y, (g_a4*)(out + 16 * j));
  } else {
    uint32_t* q = (uint32_t*)(out + 16 * j);
    q[0] = y.x;
    if ((n & 3) > 1) q[1] = y.y;
    if ((n & 3) > 2) q[2] = y.z;
  }
  if (part == 0 && threadIdx.x == 0) {
    if (kp.status) kp.status[t] = TDBG_OK;
    if (kp.stats) {
      atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_FUSED_TILES], 1ull);
      atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_FUSED_BYTES], (unsigned long long)os);
      atomicAdd((unsigned long long*)&kp.stats[TDBG_STAT_STREAM_TILES], 1ull);
    }
  }
}

}  // namespace shf
}  // namespace tdbg

extern "C" hipError_t tdbg_launch_stream_shuffle4(const tdbg::KParams* kp, hipStream_t s) {
  using namespace tdbg::shf;
  const uint64_t grid = kp->ntiles * PARTS;
  if (grid == 0 || grid > 0x7fffffffull) return hipErrorInvalidValue;
  TDBG_LAUNCH(unfilter_shuffle4_kernel, dim3((uint32_t)grid), dim3(NT), s, *kp);
  return hipGetLastError();
}
