// tdbg_io.cpp -- the step before the path: FilteredData-style
// batched tile reads feeding the device unfilter.
//
// On the read path the reference builds, per field, a list of data blocks
// over the fragment files (ReaderBase::read_tiles, reader_base.cc:689-789 ->
// FilteredData, filtered_data.h:152-300): tiles are taken in result-tile order
// and a tile extends the current block when it is in the same file, the
// block stays <= max_batch_size, and either the block is still <=
// min_batch_size or the gap to the tile is <= min_batch_gap
// (make_new_block_if_required, filtered_data.h:531-575; defaults
// vfs.min_batch_size 20 MiB, vfs.max_batch_size 100 MiB, vfs.min_batch_gap
// 500 KB, config.cc:163-165).  Every block is read with VFS::read_exactly on
// the IO thread pool (filtered_data.h:397-398) and tiles point into it
// (FilteredDataBlock::data_at, :100-101).
//
// Here the same rule forms the blocks; IO threads pread each block into a
// pinned host slot allocated on the GPU's NUMA node (so the H2D DMA does not
// cross sockets), and the host unfilter path (H2D -> unfilter kernels -> D2H
// into the caller's result buffers, tdbg_unfilter_tiles_host) takes each
// block as soon as it has landed, while the IO threads read the next ones
// into the other slots.
#include <hip/hip_runtime.h>
#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tiledb_amd.h"
#include "tdbg_desc.h"
#include "tdbg_hooks.h"

namespace {

int io_fail(int code, const std::string& msg) {
  tdbg_internal_set_error(msg.c_str());
  return code;
}

// CPUs local to the device (its PCI function's NUMA node), from sysfs
bool device_local_cpus(int device, cpu_set_t* set) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return false;
  for (char* p = bus; *p; p++) *p = (char)tolower(*p);
  const std::string path = std::string("/sys/bus/pci/devices/") + bus + "/local_cpulist";
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return false;
  char buf[4096] = {0};
  const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
  fclose(f);
  buf[n] = 0;
  CPU_ZERO(set);
  int count = 0;
  for (char* s = buf; *s;) {
    char* e = nullptr;
    const long a = strtol(s, &e, 10);
    if (e == s) break;
    long b = a;
    if (*e == '-') {
      s = e + 1;
      b = strtol(s, &e, 10);
    }
    for (long c = a; c <= b && c < CPU_SETSIZE; c++) {
      CPU_SET((int)c, set);
      count++;
    }
    s = e;
    while (*s == ',' || *s == '\n' || *s == ' ') s++;
  }
  return count > 0;
}

}  // namespace

extern "C" {

int tdbg_filtered_data_blocks(uint64_t ntiles, const uint32_t* file_idx, const uint64_t* file_offset,
                              const uint64_t* size, uint64_t min_batch_size, uint64_t max_batch_size,
                              uint64_t min_batch_gap, uint64_t* block_first_tile, uint64_t* nblocks) {
  if (!nblocks || (ntiles && (!file_idx || !file_offset || !size || !block_first_tile)))
    return io_fail(TDBG_E_ARG, "tdbg_filtered_data_blocks: null argument");
  uint64_t nb = 0;
  uint64_t boff = 0, bsize = 0;
  for (uint64_t i = 0; i < ntiles; i++) {
    const uint64_t off = file_offset[i], sz = size[i];
    if (i == 0) {
      block_first_tile[nb++] = 0;
      boff = off;
      bsize = sz;
      continue;
    }
    // filtered_data.h:521-530 (unsigned arithmetic, as there)
    const uint64_t new_size = (off + sz) - boff;
    const uint64_t gap = off - (boff + bsize);
    if (file_idx[i] == file_idx[i - 1] && new_size <= max_batch_size &&
        (new_size <= min_batch_size || gap <= min_batch_gap)) {
      bsize = new_size;
    } else {
      block_first_tile[nb++] = i;
      boff = off;
      bsize = sz;
    }
  }
  if (ntiles) block_first_tile[nb] = ntiles;
  *nblocks = nb;
  return TDBG_OK;
}

int tdbg_host_alloc_local(int device, uint64_t bytes, void** out) {
  if (!out) return io_fail(TDBG_E_ARG, "null out");
  *out = nullptr;
  cpu_set_t local, saved;
  const bool pin = device_local_cpus(device, &local) && sched_getaffinity(0, sizeof(saved), &saved) == 0;
  if (pin) (void)sched_setaffinity(0, sizeof(local), &local);
  if (hipSetDevice(device) != hipSuccess) {
    if (pin) (void)sched_setaffinity(0, sizeof(saved), &saved);
    return io_fail(TDBG_E_DEVICE, "hipSetDevice failed");
  }
  void* p = nullptr;
  hipError_t e = hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault);
  if (e == hipSuccess) memset(p, 0, bytes ? bytes : 1);  // first touch on the local node
  if (pin) (void)sched_setaffinity(0, sizeof(saved), &saved);
  if (e != hipSuccess) return io_fail(TDBG_E_DEVICE, std::string("hipHostMalloc: ") + hipGetErrorString(e));
  *out = p;
  return TDBG_OK;
}

int tdbg_host_free(void* p) {
  if (p && hipHostFree(p) != hipSuccess) return io_fail(TDBG_E_DEVICE, "hipHostFree failed");
  return TDBG_OK;
}

int tdbg_read_unfilter_tiles(tdbg_context* c, const tdbg_pipeline* p, uint64_t ntiles, const int* fds,
                             uint32_t nfiles, const uint32_t* file_idx, const uint64_t* file_offset,
                             const uint64_t* persisted_size, uint8_t* const* out, const uint64_t* out_size,
                             uint32_t flags, const tdbg_read_config* cfg, int32_t* host_status) {
  if (!c || !p) return io_fail(TDBG_E_ARG, "null context or pipeline");
  if (ntiles == 0) return TDBG_OK;
  if (!fds || !file_idx || !file_offset || !persisted_size || !out || !out_size)
    return io_fail(TDBG_E_ARG, "null tile arrays");
  for (uint64_t i = 0; i < ntiles; i++)
    if (file_idx[i] >= nfiles) return io_fail(TDBG_E_ARG, "tile file index out of range");
  tdbg_read_config rc{};
  if (cfg) rc = *cfg;
  if (!rc.min_batch_size) rc.min_batch_size = 20971520;  // vfs.min_batch_size (config.cc:165)
  if (!rc.max_batch_size) rc.max_batch_size = 104857600;  // vfs.max_batch_size (config.cc:163)
  if (!rc.min_batch_gap && !(rc.flags & TDBG_READ_ZERO_GAP)) rc.min_batch_gap = 512000;  // config.cc:164
  const uint32_t nio = rc.io_threads ? rc.io_threads : 4;
  const uint32_t nslots = std::max<uint32_t>(2, rc.slots ? rc.slots : 3);

  std::vector<uint64_t> first(ntiles + 1);
  uint64_t nb = 0;
  int r = tdbg_filtered_data_blocks(ntiles, file_idx, file_offset, persisted_size, rc.min_batch_size,
                                    rc.max_batch_size, rc.min_batch_gap, first.data(), &nb);
  if (r) return r;
  // block extents in the files
  std::vector<uint64_t> boff(nb), bsz(nb);
  uint64_t maxb = 0;
  for (uint64_t b = 0; b < nb; b++) {
    uint64_t lo = UINT64_MAX, hi = 0;
    for (uint64_t i = first[b]; i < first[b + 1]; i++) {
      lo = std::min(lo, file_offset[i]);
      hi = std::max(hi, file_offset[i] + persisted_size[i]);
    }
    boff[b] = lo;
    bsz[b] = hi - lo;
    maxb = std::max(maxb, bsz[b]);
  }
  // pinned slots on the GPU's NUMA node (allocated per call: nslots x the
  // largest block, first-touched on the device's node)
  std::vector<void*> slot(nslots, nullptr);
  for (uint32_t k = 0; k < nslots; k++) {
    r = tdbg_host_alloc_local(tdbg_context_device(c), maxb, &slot[k]);
    if (r) {
      for (auto q : slot) tdbg_host_free(q);
      return r;
    }
  }
  // IO threads: block b goes to slot b % nslots once block b - nslots is unfiltered
  std::mutex mu;
  std::condition_variable cv;
  std::vector<int> state(nb, 0);  // 0 pending, 1 landed, 2 read error, 3 consumed
  uint64_t consumed = 0;          // blocks [0, consumed) are done with their slots
  std::atomic<uint64_t> next{0};
  std::atomic<bool> stop{false};
  std::vector<std::thread> io;
  for (uint32_t t = 0; t < nio; t++) {
    io.emplace_back([&]() {
      for (;;) {
        const uint64_t b = next.fetch_add(1);
        if (b >= nb || stop.load()) return;
        {
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] { return stop.load() || consumed + nslots > b; });
          if (stop.load()) return;
        }
        uint8_t* dst = (uint8_t*)slot[b % nslots];
        const int fd = fds[file_idx[first[b]]];
        uint64_t done = 0;
        bool ok = true;
        while (done < bsz[b]) {  // VFS::read_exactly
          const ssize_t n = pread(fd, dst + done, bsz[b] - done, (off_t)(boff[b] + done));
          if (n <= 0) {
            ok = false;
            break;
          }
          done += (uint64_t)n;
        }
        {
          std::lock_guard<std::mutex> lk(mu);
          state[b] = ok ? 1 : 2;
        }
        cv.notify_all();
      }
    });
  }
  int result = TDBG_OK;
  std::string err;
  // test hook: block k's unfilter "fails" with a device error before any of
  // its statuses exist (the failure class of a HIP error in the host path)
  const long fail_block = tdbg_hook("TDBG_DEBUG_IO_FAIL_BLOCK") ? atol(tdbg_hook("TDBG_DEBUG_IO_FAIL_BLOCK")) : -1;
  // every tile is "not processed" until its block's unfilter reports it: a
  // block whose unfilter stops early (a device error before its statuses
  // are copied back), and every block after a device error, keep that
  std::vector<int32_t> st(ntiles, TDBG_E_NOT_RUN);
  std::vector<const uint8_t*> in(ntiles);
  for (uint64_t b = 0; b < nb; b++) {
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return state[b] != 0; });
    }
    const uint64_t lo = first[b], hi = first[b + 1];
    if (state[b] == 2) {
      for (uint64_t i = lo; i < hi; i++) st[i] = TDBG_E_IO;
      if (result == TDBG_OK) {
        result = TDBG_E_IO;
        err = "block read failed (short read or I/O error)";
      }
    } else {
      const uint8_t* base = (const uint8_t*)slot[b % nslots];
      for (uint64_t i = lo; i < hi; i++) in[i] = base + (file_offset[i] - boff[b]);
      const int rr =
          (long)b == fail_block
              ? (tdbg_internal_set_error("injected device failure (TDBG_DEBUG_IO_FAIL_BLOCK)"), TDBG_E_DEVICE)
              : tdbg_unfilter_tiles_host(c, p, hi - lo, in.data() + lo, persisted_size + lo, out + lo, out_size + lo,
                                         flags | TDBG_HOST_CONTIGUOUS_INPUT, st.data() + lo, 0);
      // the first failure wins, except that a call-level failure (device,
      // argument, internal) replaces a tile's: the statuses then do not
      // account for every tile (those not run say TDBG_E_NOT_RUN)
      const auto call_level = [](int s) { return s == TDBG_E_DEVICE || s == TDBG_E_ARG || s == TDBG_E_INTERNAL; };
      if (rr && (result == TDBG_OK || (call_level(rr) && !call_level(result)))) {
        result = rr;
        char buf[512];
        tdbg_last_error(buf, sizeof(buf));
        err = buf;
      }
      if (rr == TDBG_E_DEVICE) stop.store(true);
    }
    {
      std::lock_guard<std::mutex> lk(mu);
      state[b] = 3;
      consumed = b + 1;
    }
    cv.notify_all();
    if (stop.load()) break;
  }
  stop.store(true);
  cv.notify_all();
  for (auto& t : io) t.join();
  for (auto q : slot) tdbg_host_free(q);
  if (host_status) memcpy(host_status, st.data(), ntiles * 4);
  if (result != TDBG_OK) return io_fail(result, err);
  return TDBG_OK;
}

}  // extern "C"
