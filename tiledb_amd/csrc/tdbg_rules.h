// tdbg_rules.h -- the reference's failure precedence as closed forms, shared
// by the device kernels (tdbg_device.h) and the CPU entry (tdbg_cpu.cpp), so
// both report the same status for the same malformed chunk.
#pragma once
#include <stdint.h>

#include "../../include/tiledb_amd.h"

#if defined(__HIPCC__) || defined(__HIP__)
#define TDBG_HD __host__ __device__
#else
#define TDBG_HD
#endif

namespace tdbg {

// ---- reference failure precedence (see tdb_oracle.c copy_in_out) ----------
// FilterBuffer::write(FilterBuffer*, n) (filter_buffer.cc:393-424).
TDBG_HD inline uint32_t copy_fail(uint64_t in_n, uint64_t ip,
                                              uint64_t cap, uint64_t op,
                                              uint64_t n) {
  const uint64_t avail = ip < in_n ? in_n - ip : 0;
  const uint64_t k = n < avail ? n : avail;
  const uint64_t room = op < cap ? cap - op : 0;
  if (k > 0 && room == 0) return TDBG_E_OUT_FULL;
  if (k > room) return TDBG_E_OUT_FULL;
  if (k < n) return TDBG_E_DATA_READ;
  return 0;
}

// ne elements, each read cb bytes at ip + j*cb then write wb bytes at
// op + j*wb; the read of element j precedes its write.
TDBG_HD inline uint32_t elem_fail(uint64_t in_n, uint64_t ip,
                                              uint32_t cb, uint64_t cap,
                                              uint64_t op, uint32_t wb,
                                              uint64_t ne) {
  uint64_t jr = ne, jw = ne;
  if (ip + ne * cb > in_n) jr = ip >= in_n ? 0 : (in_n - ip) / cb;
  if (op + ne * wb > cap) jw = op >= cap ? 0 : (cap - op) / wb;
  if (jr >= ne && jw >= ne) return 0;
  return jr <= jw ? TDBG_E_DATA_READ : TDBG_E_OUT_FULL;
}

// DoubleDelta::decompress read/write sequence (dd_compressor.cc:314-404):
// R v0, W v0, [num==1], R v1, W v1, [num==2], R word0, then per code i>=2
// the word reads it triggers and W x_i.  Returns the first failure.
TDBG_HD inline int dd_check(uint64_t cn, uint64_t un, uint32_t w,
                                        uint32_t b, uint64_t num) {
  const uint64_t NONE = ~0ull;
  uint64_t rord = NONE, word = NONE;
  const uint64_t nvals = num == 0 ? 2 : num;
  // reads
  if (cn < 9 + (uint64_t)w) rord = 0;
  else if (num != 1) {
    if (cn < 9 + 2ull * w) rord = 2;
    else if (num != 2) {
      const uint64_t base = 9 + 2ull * w;
      const uint64_t A = (cn - base) / 8, rem = (cn - base) % 8;
      if (A == 0) rord = 4;
      else {
        uint64_t ir = NONE;
        if (b == 0) {
          ir = 64 * A + 1;
          if (ir < 2) ir = 2;
        } else {
          ir = 2 + (64 * A) / (b + 1);
          if (rem > 0 && (64 * A) % (b + 1) == 0) {
            const uint64_t ib = 1 + (64 * A) / (b + 1);
            if (ib >= 2 && ib < ir) ir = ib;
          }
        }
        if (ir < num) rord = 5 + 2 * (ir - 2);
      }
    }
  }
  // writes
  const uint64_t iw = un / w;
  if (iw < nvals) {
    if (iw == 0) word = 1;
    else if (iw == 1) word = 3;
    else word = 6 + 2 * (iw - 2);
  }
  if (rord == NONE && word == NONE) return 0;
  return rord <= word ? TDBG_E_DATA_READ : TDBG_E_OUT_FULL;
}

}  // namespace tdbg
