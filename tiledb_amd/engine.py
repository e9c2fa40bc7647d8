"""Python handles over the C-ABI: device pipelines, contexts, tile batches.

PyTorch is used only as plumbing: device allocations (torch.uint8 tensors on
cuda:N), the current HIP stream, and pinned host memory.  All unfilter work is
done by libtiledb_amd.so.
"""
from __future__ import annotations

import atexit
import ctypes
from typing import Optional, Sequence

import numpy as np

from . import _native
from ._native import lib

# At interpreter exit the HIP runtime may already be torn down: handles still
# alive then are left to the OS (no destroy calls, no errors during shutdown).
_SHUTDOWN: list = []
atexit.register(lambda: _SHUTDOWN.append(True))

TILE_OFFSETS = 0x1  # TDBG_TILE_OFFSETS
HOST_CONTIGUOUS_INPUT = 0x2   # TDBG_HOST_CONTIGUOUS_INPUT
HOST_CONTIGUOUS_OUTPUT = 0x4  # TDBG_HOST_CONTIGUOUS_OUTPUT
CHUNK_PARALLEL = 0x8  # TDBG_CHUNK_PARALLEL
MULTI_CHUNK = 0x10  # TDBG_MULTI_CHUNK
E_NOT_RUN = 19  # TDBG_E_NOT_RUN
# call-level failures (not a tile's status): raised even when tiles carry statuses
CALL_ERRORS = (1, 10, 14, 15, 17)  # TDBG_E_ARG, _UNSUPPORTED, _DEVICE, _DESCRIPTOR, _INTERNAL


class EngineError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def _check(rc: int, what: str) -> None:
    if rc:
        raise EngineError(rc, f"{what}: {_native.last_error() or _native.status_str(rc)}")


class DevicePipeline:
    """tdbg_pipeline: a parsed, immutable FilterPipeline descriptor."""

    def __init__(self, serialized: bytes, version: int, on_disk_type: int, cell_size: int):
        buf = (ctypes.c_uint8 * len(serialized)).from_buffer_copy(serialized)
        h = ctypes.c_void_p()
        _check(lib.tdbg_pipeline_create(buf, len(serialized), version, on_disk_type, cell_size,
                                        ctypes.byref(h)), "tdbg_pipeline_create")
        self.h = h
        self.serialized = bytes(serialized)
        self.version = version
        self.on_disk_type = on_disk_type
        self.cell_size = cell_size

    @property
    def supported(self) -> bool:
        return bool(lib.tdbg_pipeline_supported(self.h))

    @property
    def num_filters(self) -> int:
        return int(lib.tdbg_pipeline_num_filters(self.h))

    def filter_info(self, i: int):
        t = ctypes.c_uint8()
        d = ctypes.c_uint8()
        _check(lib.tdbg_pipeline_filter(self.h, i, ctypes.byref(t), ctypes.byref(d)),
               "tdbg_pipeline_filter")
        return int(t.value), int(d.value)

    def __del__(self, _destroy=lib.tdbg_pipeline_destroy, _down=_SHUTDOWN):
        h = getattr(self, "h", None)
        if h and not _down:
            _destroy(h)
            self.h = None


def pack_offsets(sizes: np.ndarray, align: int = 1) -> np.ndarray:
    """Start offsets of tiles packed in order, each start rounded up to `align`."""
    sizes = np.asarray(sizes, dtype=np.uint64)
    a = np.uint64(max(1, int(align)))
    al = (sizes + a - np.uint64(1)) // a * a
    offs = np.zeros_like(sizes)
    if sizes.size:
        offs[1:] = np.cumsum(al)[:-1]
    return offs


class TileBatch:
    """Device-resident batch of filtered tiles and their output buffers.

    Filtered tiles are packed back to back in `d_in` (uint8, device), outputs
    in `d_out`; the per-tile device pointer / size arrays the C-ABI takes are
    built once.
    """

    def __init__(self, d_in, in_off: np.ndarray, in_size: np.ndarray, d_out,
                 out_off: np.ndarray, out_size: np.ndarray):
        import torch
        self.d_in, self.d_out = d_in, d_out
        self.in_off = np.asarray(in_off, dtype=np.uint64)
        self.in_size = np.asarray(in_size, dtype=np.uint64)
        self.out_off = np.asarray(out_off, dtype=np.uint64)
        self.out_size = np.asarray(out_size, dtype=np.uint64)
        dev = d_in.device
        ib, ob = d_in.data_ptr(), d_out.data_ptr()
        meta = np.empty((4, self.ntiles), dtype=np.uint64)
        meta[0] = self.in_off + np.uint64(ib)
        meta[1] = self.in_size
        meta[2] = self.out_off + np.uint64(ob)
        meta[3] = self.out_size
        self.d_meta = torch.from_numpy(meta.view(np.int64)).to(dev)
        self.d_status = torch.zeros(max(self.ntiles, 1), dtype=torch.int32, device=dev)

    @property
    def ntiles(self) -> int:
        return int(self.in_off.size)

    def ptrs(self):
        base = self.d_meta.data_ptr()
        n = self.ntiles * 8
        return base, base + n, base + 2 * n, base + 3 * n

    @classmethod
    def from_packed(cls, packed: np.ndarray, in_off, in_size, out_sizes, device: int = 0,
                    fill: int = 0, arena=None, in_first: bool = False, gap: int = 0) -> "TileBatch":
        """arena: an optional device uint8 tensor of at least
        arena_bytes(packed.size, sum(out_sizes)) bytes; the outputs then sit at
        its start and the filtered tiles at the next 2 MiB boundary after them,
        so batches built in turn on one arena use the same device pages."""
        import torch
        dev = torch.device("cuda", device)
        packed = np.ascontiguousarray(packed, dtype=np.uint8)
        out_size = np.asarray(out_sizes, dtype=np.uint64)
        out_off = np.zeros_like(out_size)
        if out_size.size:
            out_off[1:] = np.cumsum(out_size)[:-1]
        total = int(out_size.sum()) if out_size.size else 0
        if arena is not None:
            need = cls.arena_bytes(packed.size, total)
            if arena.numel() < need:
                raise ValueError(f"arena of {arena.numel()} B < {need} B")
            ob = max(total, 16)
            if in_first:  # (layout experiments: tiles first, outputs after)
                d_in = arena[:max(packed.size, 16)]
                o0 = -(-max(packed.size, 16) // (2 << 20)) * (2 << 20) + gap
                d_out = arena[o0:o0 + ob]
            else:
                d_out = arena[:ob]
                ib = -(-ob // (2 << 20)) * (2 << 20) + gap
                d_in = arena[ib:ib + max(packed.size, 16)]
            d_out.fill_(fill)
            if packed.size:
                d_in[:packed.size].copy_(torch.from_numpy(packed))
            return cls(d_in, in_off, in_size, d_out, out_off, out_size)
        d_in = torch.from_numpy(packed).to(dev) if packed.size else torch.zeros(16, dtype=torch.uint8,
                                                                                device=dev)
        d_out = torch.full((max(total, 16),), fill, dtype=torch.uint8, device=dev)
        return cls(d_in, in_off, in_size, d_out, out_off, out_size)

    @staticmethod
    def arena_bytes(in_bytes: int, out_bytes: int) -> int:
        """Bytes from_packed(arena=...) needs for in_bytes of filtered tiles and
        out_bytes of outputs."""
        ob = max(out_bytes, 16)
        return -(-ob // (2 << 20)) * (2 << 20) + -(-max(in_bytes, 16) // (2 << 20)) * (2 << 20)

    @classmethod
    def from_host(cls, tiles: Sequence, out_sizes, device: int = 0, fill: int = 0,
                  align: int = 1) -> "TileBatch":
        """Packs the filtered tiles into one device buffer.  align=1 (default)
        packs them back to back, as a fragment file holds them and as
        FilteredData::data_at hands them over (filtered_data.h:100-101: tile
        starts at cumulative filtered sizes, i.e. arbitrary byte offsets)."""
        bufs = [np.frombuffer(bytes(t), dtype=np.uint8) if not isinstance(t, np.ndarray)
                else np.ascontiguousarray(t).view(np.uint8).reshape(-1) for t in tiles]
        sizes = np.array([b.size for b in bufs], dtype=np.uint64)
        offs = pack_offsets(sizes, align)
        packed = np.zeros(int(offs[-1] + sizes[-1]) if sizes.size else 0, dtype=np.uint8)
        for b, o in zip(bufs, offs):
            packed[int(o):int(o) + b.size] = b
        return cls.from_packed(packed, offs, sizes, out_sizes, device=device, fill=fill)

    def output(self, i: int) -> np.ndarray:
        o, n = int(self.out_off[i]), int(self.out_size[i])
        return self.d_out[o:o + n].cpu().numpy()

    def outputs_host(self) -> np.ndarray:
        return self.d_out.cpu().numpy()


class FilterBatch:
    """Device-resident forward batch: unfiltered tiles packed back to back in
    `d_in`, each filtered tile written at a 16-byte aligned slot of `d_out`
    sized by tdbg_filtered_bound; `d_meta` rows are the C-ABI's pointer /
    size / capacity / filtered-length arrays."""

    def __init__(self, dp: DevicePipeline, tiles: Sequence, device: int, max_chunk: int = 0):
        import torch
        bufs = [np.ascontiguousarray(t).view(np.uint8).reshape(-1) for t in tiles]
        n = len(bufs)
        self.max_chunk = int(max_chunk)
        self.in_size = np.array([b.size for b in bufs], dtype=np.uint64)
        offs = pack_offsets(self.in_size, 1)
        packed = np.zeros(int(offs[-1] + self.in_size[-1]) + 1 if n else 1, dtype=np.uint8)
        for b, o in zip(bufs, offs):
            packed[int(o):int(o) + b.size] = b
        dev = torch.device("cuda", device)
        self.d_in = torch.from_numpy(packed).to(dev)
        self.cap = np.array([lib.tdbg_filtered_bound(dp.h, int(sz), self.max_chunk) for sz in self.in_size],
                            dtype=np.uint64)
        self.out_off = pack_offsets(self.cap, 16)
        self.d_out = torch.zeros(int(self.out_off[-1] + self.cap[-1]) + 16 if n else 16, dtype=torch.uint8,
                                 device=dev)
        meta = np.zeros((5, max(n, 1)), dtype=np.uint64)
        meta[0, :n] = offs + np.uint64(self.d_in.data_ptr())
        meta[1, :n] = self.in_size
        meta[2, :n] = self.out_off + np.uint64(self.d_out.data_ptr())
        meta[3, :n] = self.cap
        self.d_meta = torch.from_numpy(meta.view(np.int64)).to(dev)
        self.d_status = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)

    @property
    def ntiles(self) -> int:
        return int(self.in_size.size)

    def ptrs(self):
        base, k = self.d_meta.data_ptr(), max(self.ntiles, 1) * 8
        return base, base + k, base + 2 * k, base + 3 * k, base + 4 * k

    def lengths(self) -> np.ndarray:
        return self.d_meta[4].cpu().numpy().view(np.uint64)[: self.ntiles].copy()

    def outputs(self):
        lens = self.lengths()
        out = self.d_out.cpu().numpy()
        return [out[int(o):int(o) + int(l)].copy() for o, l in zip(self.out_off, lens)]


class Context:
    """tdbg_context: per-device scratch, status arrays, timing."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        _check(lib.tdbg_context_create(device, ctypes.byref(h)), "tdbg_context_create")
        self.h = h
        self.device = device

    def __del__(self, _destroy=lib.tdbg_context_destroy, _down=_SHUTDOWN):
        h = getattr(self, "h", None)
        if h and not _down:
            _destroy(h)
            self.h = None

    @staticmethod
    def _stream(stream) -> int:
        if stream is not None:
            return int(stream)
        import torch
        return int(torch.cuda.current_stream().cuda_stream)

    @staticmethod
    def auto_chunk_parallel(dp: DevicePipeline, batch: TileBatch) -> bool:
        """Whether a tile holds more than one chunk (an unfiltered size above
        the pipeline's max chunk size, FilterPipeline::serialize's first u32;
        tile.cc:87-100): such launches carry TDBG_MULTI_CHUNK, and the engine
        then runs the C5 tile kernel's multi-chunk variant when the launch
        has tiles enough to fill the GPU, or the device chunk directory
        (chunk-parallel) when it has fewer."""
        if batch.ntiles == 0 or len(dp.serialized) < 4:
            return False
        mc = int(np.frombuffer(dp.serialized[:4], dtype="<u4")[0]) or 65536
        return bool(int(batch.out_size.max()) > mc)

    def _launch_flags(self, dp, batch, offsets_tiles, chunk_parallel) -> int:
        """chunk_parallel: None = TDBG_MULTI_CHUNK when auto_chunk_parallel
        (the engine picks tile or chunk mode); True = TDBG_CHUNK_PARALLEL;
        False = neither."""
        f = TILE_OFFSETS if offsets_tiles else 0
        if chunk_parallel is None:
            return f | (MULTI_CHUNK if self.auto_chunk_parallel(dp, batch) else 0)
        return f | (CHUNK_PARALLEL if chunk_parallel else 0)

    def unfilter(self, dp: DevicePipeline, batch: TileBatch, offsets_tiles: bool = False,
                 stream=None, chunk_parallel=None) -> np.ndarray:
        """Synchronous unfilter; returns the per-tile status array.
        chunk_parallel: see _launch_flags."""
        st = np.zeros(max(batch.ntiles, 1), dtype=np.int32)
        pin, psz, pout, posz = batch.ptrs()
        rc = lib.tdbg_unfilter_tiles_sync(
            self.h, dp.h, batch.ntiles, pin, psz, pout, posz,
            self._launch_flags(dp, batch, offsets_tiles, chunk_parallel),
            st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), self._stream(stream))
        if rc and not st[: batch.ntiles].any():
            _check(rc, "tdbg_unfilter_tiles_sync")
        return st[: batch.ntiles]

    def unfilter_async(self, dp: DevicePipeline, batch: TileBatch, offsets_tiles: bool = False,
                       stream=None, chunk_parallel=None) -> None:
        pin, psz, pout, posz = batch.ptrs()
        _check(lib.tdbg_unfilter_tiles_async(
            self.h, dp.h, batch.ntiles, pin, psz, pout, posz,
            self._launch_flags(dp, batch, offsets_tiles, chunk_parallel),
            batch.d_status.data_ptr(), self._stream(stream)), "tdbg_unfilter_tiles_async")

    def filter_batch(self, dp: DevicePipeline, tiles: Sequence, max_chunk: int = 0) -> "FilterBatch":
        """Device-resident forward batch: the unfiltered tiles packed back to
        back on this context's device, outputs sized by tdbg_filtered_bound."""
        return FilterBatch(dp, tiles, self.device, max_chunk)

    def filter_async(self, dp: DevicePipeline, fb: "FilterBatch", stream=None) -> None:
        """tdbg_filter_tiles_async over a FilterBatch (statuses and filtered
        lengths stay on the device)."""
        pin, psz, pout, pcap, plen = fb.ptrs()
        _check(lib.tdbg_filter_tiles_async(self.h, dp.h, fb.ntiles, pin, psz, pout, pcap, plen,
                                           fb.max_chunk, fb.d_status.data_ptr(), self._stream(stream)),
               "tdbg_filter_tiles_async")

    def filter(self, dp: DevicePipeline, tiles: Sequence, max_chunk: int = 0, stream=None):
        """Forward direction (FilterPipeline::run_forward): unfiltered tiles ->
        on-disk filtered tiles.  Returns (statuses, [filtered bytes as np.uint8])."""
        fb = self.filter_batch(dp, tiles, max_chunk)
        n = fb.ntiles
        st = np.zeros(max(n, 1), dtype=np.int32)
        pin, psz, pout, pcap, plen = fb.ptrs()
        rc = lib.tdbg_filter_tiles_sync(self.h, dp.h, n, pin, psz, pout, pcap, plen, max_chunk,
                                        st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                        self._stream(stream))
        if rc and not st[:n].any():
            _check(rc, "tdbg_filter_tiles_sync")
        return st[:n], fb.outputs()

    def path_stats(self):
        """(fused, fallback, general) tile counts, cumulative (synchronizes the device)."""
        f, b, g = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib.tdbg_context_path_stats(self.h, ctypes.byref(f), ctypes.byref(b), ctypes.byref(g)),
               "tdbg_context_path_stats")
        return int(f.value), int(b.value), int(g.value)

    def stream_tiles(self):
        """Fused tiles the streaming C5 kernel took, cumulative (synchronizes)."""
        n = ctypes.c_uint64()
        _check(lib.tdbg_context_stream_stats(self.h, ctypes.byref(n)), "tdbg_context_stream_stats")
        return int(n.value)

    def forward_stream_tiles(self):
        """Tiles the LDS-resident C5 forward kernel filtered, cumulative (synchronizes)."""
        n = ctypes.c_uint64()
        _check(lib.tdbg_context_forward_stream_stats(self.h, ctypes.byref(n)), "tdbg_context_forward_stream_stats")
        return int(n.value)

    def tile_chunks(self):
        """Chunks of multi-chunk tiles the C5 tile kernel took in tile mode
        (TDBG_MULTI_CHUNK launches), cumulative."""
        if "tdbg_context_tile_chunk_stats" in _native.MISSING:  # (an older TDBG_LIB build)
            return 0
        n = ctypes.c_uint64()
        _check(lib.tdbg_context_tile_chunk_stats(self.h, ctypes.byref(n)), "tdbg_context_tile_chunk_stats")
        return int(n.value)

    def stream_chunks(self):
        """Chunks of chunk-parallel launches the streaming kernels took, cumulative."""
        if "tdbg_context_stream_chunk_stats" in _native.MISSING:  # (an older TDBG_LIB build)
            return 0
        n = ctypes.c_uint64()
        _check(lib.tdbg_context_stream_chunk_stats(self.h, ctypes.byref(n)), "tdbg_context_stream_chunk_stats")
        return int(n.value)

    def stream_raw_tiles(self):
        """Of those, the tiles the raw-DoubleDelta streaming kernel took, cumulative."""
        n = ctypes.c_uint64()
        _check(lib.tdbg_context_stream_raw_stats(self.h, ctypes.byref(n)), "tdbg_context_stream_raw_stats")
        return int(n.value)

    def stats(self):
        """(tiles_unfiltered, read_unfiltered_byte_num)."""
        t, b = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib.tdbg_context_stats(self.h, ctypes.byref(t), ctypes.byref(b)), "tdbg_context_stats")
        return int(t.value), int(b.value)

    def last_kernel_ms(self) -> float:
        ms = ctypes.c_float()
        _check(lib.tdbg_context_last_kernel_ms(self.h, ctypes.byref(ms)), "last_kernel_ms")
        return float(ms.value)

    def time_launches(self, n: int) -> None:
        """Arm per-launch HIP-event timing for the next n launches on this context."""
        _check(lib.tdbg_context_time_launches(self.h, n), "tdbg_context_time_launches")

    def launch_times(self, cap: int = 4096):
        """(kernel_ms, total_ms) per armed launch: the fused/general kernel and
        the whole launch incl. the fallback fixup (waits for the last armed launch)."""
        k = np.zeros(cap, dtype=np.float32)
        t = np.zeros(cap, dtype=np.float32)
        n = ctypes.c_uint32()
        _check(lib.tdbg_context_launch_times(self.h, k.ctypes.data, t.ctypes.data,
                                             cap, ctypes.byref(n)), "tdbg_context_launch_times")
        m = n.value
        return k[:m].copy(), t[:m].copy()

    def phase_clocks(self, nphases: int = 8) -> np.ndarray:
        """Diagnostics: fused-kernel cycles per phase of the last launch (TDBG_PROF=1)."""
        out = np.zeros(nphases, dtype=np.uint64)
        _check(lib.tdbg_debug_phase_clocks(
            self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), nphases), "phase_clocks")
        return out

    def unfilter_host(self, dp: DevicePipeline, in_ptrs: np.ndarray, in_size: np.ndarray,
                      out_ptrs: np.ndarray, out_size: np.ndarray, offsets_tiles: bool = False,
                      batch_bytes: int = 0, contiguous_input: bool = False,
                      contiguous_output: bool = False, var_size=None) -> np.ndarray:
        """Host-resident end-to-end (pinned H2D, unfilter, D2H).  contiguous_*:
        the caller states that all input (output) buffers lie in one host
        allocation, which lets adjacent tiles share one copy.  var_size (offsets
        tiles only): Tile::add_extra_offset fused before the D2H."""
        n = int(in_size.size)
        st = np.zeros(max(n, 1), dtype=np.int32)
        ip = np.ascontiguousarray(in_ptrs, dtype=np.uint64)
        isz = np.ascontiguousarray(in_size, dtype=np.uint64)
        op = np.ascontiguousarray(out_ptrs, dtype=np.uint64)
        osz = np.ascontiguousarray(out_size, dtype=np.uint64)
        flags = _host_flags(offsets_tiles or var_size is not None, contiguous_input, contiguous_output)
        sp = st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        if var_size is not None:
            vs = np.ascontiguousarray(var_size, dtype=np.uint64)
            rc = lib.tdbg_unfilter_offsets_host(self.h, dp.h, n, ip.ctypes.data, isz.ctypes.data,
                                                op.ctypes.data, osz.ctypes.data, vs.ctypes.data, flags, sp,
                                                batch_bytes)
        else:
            rc = lib.tdbg_unfilter_tiles_host(self.h, dp.h, n, ip.ctypes.data, isz.ctypes.data,
                                              op.ctypes.data, osz.ctypes.data, flags, sp, batch_bytes)
        if rc and not st[:n].any():
            _check(rc, "tdbg_unfilter_offsets_host" if var_size is not None else "tdbg_unfilter_tiles_host")
        return st[:n]

    def add_extra_offsets(self, batch: "TileBatch", var_size, status: bool = True, stream=None) -> None:
        """Tile::add_extra_offset on a device batch of unfiltered offsets tiles
        (tdbg_add_extra_offsets_async; tiles with an error status untouched)."""
        import torch
        vs = torch.from_numpy(np.ascontiguousarray(var_size, dtype=np.uint64).view(np.int64)).to(batch.d_out.device)
        _, _, pout, posz = batch.ptrs()
        _check(lib.tdbg_add_extra_offsets_async(self.h, batch.ntiles, pout, posz, vs.data_ptr(),
                                                batch.d_status.data_ptr() if status else None,
                                                self._stream(stream)), "tdbg_add_extra_offsets_async")
        torch.cuda.synchronize(batch.d_out.device)

    def read_unfilter(self, dp: DevicePipeline, fds, file_idx, file_offset, size, out_ptrs, out_sizes,
                       flags: int = 0, cfg=None, status_out: Optional[np.ndarray] = None) -> np.ndarray:
        """tdbg_read_unfilter_tiles: FilteredData-style block reads from the open
        files `fds` -> H2D -> unfilter -> D2H into out_ptrs; per-tile statuses
        (also copied into status_out, if given, before a call-level error raises)."""
        n = int(np.asarray(size).size)
        st = np.zeros(max(n, 1), dtype=np.int32)
        fd = np.ascontiguousarray(fds, dtype=np.int32)
        fi = np.ascontiguousarray(file_idx, dtype=np.uint32)
        fo = np.ascontiguousarray(file_offset, dtype=np.uint64)
        sz = np.ascontiguousarray(size, dtype=np.uint64)
        op = np.ascontiguousarray(out_ptrs, dtype=np.uint64)
        osz = np.ascontiguousarray(out_sizes, dtype=np.uint64)
        rc = lib.tdbg_read_unfilter_tiles(self.h, dp.h, n, fd.ctypes.data, fd.size, fi.ctypes.data, fo.ctypes.data,
                                          sz.ctypes.data, op.ctypes.data, osz.ctypes.data, flags,
                                          ctypes.byref(cfg) if cfg is not None else None,
                                          st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        if status_out is not None:
            status_out[:n] = st[:n]
        # call-level failures raise even when some tiles carry statuses (those
        # after the failure say TDBG_E_NOT_RUN); tile-level ones are in st
        if rc and (rc in CALL_ERRORS or not st[:n].any()):
            _check(rc, "tdbg_read_unfilter_tiles")
        return st[:n]


    def dense_read(self, dp: DevicePipeline, tiles, tile_start, cfg, result: np.ndarray, flags: int = 0,
                    batch_bytes: int = 0) -> np.ndarray:
        """tdbg_dense_read_host: filtered host tiles -> unfilter -> cell-slab copy
        on the device -> one D2H of the subarray into `result` (uint8 array)."""
        bufs = [np.ascontiguousarray(t, dtype=np.uint8).reshape(-1) for t in tiles]
        n = len(bufs)
        st = np.zeros(max(n, 1), dtype=np.int32)
        ip = np.array([b.ctypes.data for b in bufs], dtype=np.uint64)
        isz = np.array([b.size for b in bufs], dtype=np.uint64)
        ts = np.ascontiguousarray(tile_start, dtype=np.int64)
        assert result.dtype == np.uint8 and result.flags.c_contiguous
        rc = lib.tdbg_dense_read_host(self.h, dp.h, n, ip.ctypes.data, isz.ctypes.data, ts.ctypes.data,
                                      ctypes.byref(cfg), result.ctypes.data, result.size, flags,
                                      st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), batch_bytes)
        if rc and (rc in CALL_ERRORS or not st[:n].any()):
            _check(rc, "tdbg_dense_read_host")
        return st[:n]


    def dense_copy_async(self, cfg, ntiles: int, d_tile_start, d_tiles, d_result, d_status=None, stream=None) -> None:
        """tdbg_dense_copy_async on device pointers (ints)."""
        _check(lib.tdbg_dense_copy_async(self.h, ctypes.byref(cfg), ntiles, d_tile_start, d_tiles,
                                         d_status if d_status else None, d_result, self._stream(stream)),
               "tdbg_dense_copy_async")


def _ptrs(xs):
    return np.array([0 if x is None else int(x) for x in xs], dtype=np.uint64)


def dense_copy_fragments_async(ctx, fcfg, ntiles: int, d_tile_start, d_frag_dom, d_tiles, d_fill, d_result,
                               d_validity=None, d_result_validity=None, stream=None) -> None:
    """tdbg_dense_copy_fragments_async on device pointers (ints)."""
    _check(lib.tdbg_dense_copy_fragments_async(ctx.h, ctypes.byref(fcfg), ntiles, d_tile_start, d_frag_dom, d_tiles,
                                               d_validity, d_fill, d_result, d_result_validity,
                                               ctx._stream(stream)), "tdbg_dense_copy_fragments_async")


def dense_var_offsets_async(ctx, fcfg, ntiles: int, d_tile_start, d_frag_dom, d_off_tiles, d_var_tiles, d_fill,
                            d_result_offsets, d_var_total, d_validity=None, d_result_validity=None,
                            stream=None) -> None:
    _check(lib.tdbg_dense_var_offsets_async(ctx.h, ctypes.byref(fcfg), ntiles, d_tile_start, d_frag_dom, d_off_tiles,
                                            d_var_tiles, d_validity, d_fill, d_result_offsets, d_result_validity,
                                            d_var_total, ctx._stream(stream)), "tdbg_dense_var_offsets_async")


def dense_var_copy_async(ctx, fcfg, d_result_offsets, d_var_total, d_result_var, stream=None) -> None:
    _check(lib.tdbg_dense_var_copy_async(ctx.h, ctypes.byref(fcfg), d_result_offsets, d_var_total, d_result_var,
                                         ctx._stream(stream)), "tdbg_dense_var_copy_async")


def dense_var_status(ctx, stream=None) -> int:
    """tdbg_dense_var_status: the data check of the context's last
    dense_var_offsets_async (TDBG_OK, or TDBG_E_DATA_READ when a cell's
    offsets lay outside its var tile); waits for `stream`."""
    st = ctypes.c_int32(0)
    _check(lib.tdbg_dense_var_status(ctx.h, ctx._stream(stream), ctypes.byref(st)), "tdbg_dense_var_status")
    return int(st.value)


def dense_read_var_host(ctx, dp_off: DevicePipeline, dp_var: DevicePipeline, fcfg, tile_start, frag_dom,
                        off_filtered, var_filtered, var_unfiltered_size, fill_value: bytes, var_cap: int,
                        out_offsets=None, out_var=None):
    """tdbg_dense_read_var_host: host filtered offsets / var tiles per (tile,
    fragment) (None: absent) -> (result offsets uint64, var bytes, statuses).
    out_offsets / out_var: optional caller result buffers (uint64 of the
    subarray's cells, uint8 of var_cap bytes), written in place; the var
    bytes are then returned as a view of out_var."""
    ntiles = len(tile_start)
    nf = fcfg.nfrag
    assert len(off_filtered) == ntiles * nf == len(var_filtered) == len(var_unfiltered_size)
    keep = [np.ascontiguousarray(b, dtype=np.uint8) if b is not None else None for b in off_filtered + var_filtered]
    op = _ptrs([None if b is None else b.ctypes.data for b in keep[:ntiles * nf]])
    vp = _ptrs([None if b is None else b.ctypes.data for b in keep[ntiles * nf:]])
    osz = np.array([0 if b is None else b.size for b in keep[:ntiles * nf]], dtype=np.uint64)
    vsz = np.array([0 if b is None else b.size for b in keep[ntiles * nf:]], dtype=np.uint64)
    vus = np.ascontiguousarray(var_unfiltered_size, dtype=np.uint64)
    ts = np.ascontiguousarray(tile_start, dtype=np.int64).reshape(-1)
    fd = np.ascontiguousarray(frag_dom, dtype=np.int64).reshape(-1)
    fill = np.frombuffer(bytes(fill_value) or b"\0", dtype=np.uint8)
    ncell = 1
    for d in range(fcfg.base.dim_num):
        ncell *= fcfg.base.sub_hi[d] - fcfg.base.sub_lo[d] + 1
    roff = out_offsets if out_offsets is not None else np.zeros(ncell, dtype=np.uint64)
    rvar = out_var if out_var is not None else np.zeros(max(var_cap, 1), dtype=np.uint8)
    assert roff.dtype == np.uint64 and roff.size >= ncell and rvar.dtype == np.uint8 and rvar.size >= max(var_cap, 1)
    total = ctypes.c_uint64()
    st = np.zeros(max(ntiles * nf, 1), dtype=np.int32)
    rc = lib.tdbg_dense_read_var_host(ctx.h, dp_off.h, dp_var.h, ctypes.byref(fcfg), ntiles, ts.ctypes.data,
                                      fd.ctypes.data, op.ctypes.data, osz.ctypes.data, vp.ctypes.data,
                                      vsz.ctypes.data, vus.ctypes.data, fill.ctypes.data, roff.ctypes.data,
                                      rvar.ctypes.data, var_cap, ctypes.byref(total),
                                      st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    if rc and (rc in CALL_ERRORS or not st[:ntiles * nf].any()):
        _check(rc, "tdbg_dense_read_var_host")
    data = rvar[:int(total.value) * (fcfg.data_type_size if fcfg.elements_mode else 1)]
    return rc, roff, (data if out_var is not None else bytes(data)), st[:ntiles * nf]


def unfilter_cpu(dp: DevicePipeline, in_ptrs, in_size, out_ptrs, out_size, nthreads: int = 0,
                 offsets_tiles: bool = False) -> np.ndarray:
    """tdbg_unfilter_tiles_cpu: host tiles -> host outputs on nthreads host
    threads (0 = hardware concurrency); returns per-tile statuses."""
    n = int(np.asarray(in_size).size)
    st = np.zeros(max(n, 1), dtype=np.int32)
    ip = np.ascontiguousarray(in_ptrs, dtype=np.uint64)
    isz = np.ascontiguousarray(in_size, dtype=np.uint64)
    op = np.ascontiguousarray(out_ptrs, dtype=np.uint64)
    osz = np.ascontiguousarray(out_size, dtype=np.uint64)
    rc = lib.tdbg_unfilter_tiles_cpu(dp.h, n, ip.ctypes.data, isz.ctypes.data, op.ctypes.data,
                                     osz.ctypes.data, TILE_OFFSETS if offsets_tiles else 0,
                                     st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), nthreads)
    if rc and not st[:n].any():
        _check(rc, "tdbg_unfilter_tiles_cpu")
    return st[:n]


def _host_flags(offsets_tiles: bool, contiguous_input: bool, contiguous_output: bool) -> int:
    return ((TILE_OFFSETS if offsets_tiles else 0) | (HOST_CONTIGUOUS_INPUT if contiguous_input else 0) |
            (HOST_CONTIGUOUS_OUTPUT if contiguous_output else 0))


def unfilter_multi_gpu(dp: DevicePipeline, in_ptrs, in_size, out_ptrs, out_size, devices,
                       offsets_tiles: bool = False, batch_bytes: int = 0,
                       contiguous_input: bool = False, contiguous_output: bool = False) -> np.ndarray:
    n = int(np.asarray(in_size).size)
    st = np.zeros(max(n, 1), dtype=np.int32)
    ip = np.ascontiguousarray(in_ptrs, dtype=np.uint64)
    isz = np.ascontiguousarray(in_size, dtype=np.uint64)
    op = np.ascontiguousarray(out_ptrs, dtype=np.uint64)
    osz = np.ascontiguousarray(out_size, dtype=np.uint64)
    devs = (ctypes.c_int * len(devices))(*devices)
    rc = lib.tdbg_unfilter_tiles_multi_gpu(
        dp.h, n, ip.ctypes.data, isz.ctypes.data, op.ctypes.data, osz.ctypes.data,
        _host_flags(offsets_tiles, contiguous_input, contiguous_output),
        st.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), devs, len(devices), batch_bytes)
    if rc and not st[:n].any():
        _check(rc, "tdbg_unfilter_tiles_multi_gpu")
    return st[:n]


def shard_tiles(in_size, out_size, nshards: int) -> np.ndarray:
    """Contiguous shard boundaries (nshards + 1 tile indices), byte-balanced.

    Rank r of a one-process-per-GPU job unfilters tiles [cuts[r], cuts[r+1]);
    the same cut drives tdbg_unfilter_tiles_multi_gpu."""
    isz = np.ascontiguousarray(in_size, dtype=np.uint64)
    osz = np.ascontiguousarray(out_size, dtype=np.uint64)
    if isz.size != osz.size:
        raise ValueError("in_size and out_size differ in length")
    cuts = np.zeros(nshards + 1, dtype=np.uint64)
    _check(lib.tdbg_shard_tiles(isz.size, isz.ctypes.data, osz.ctypes.data, nshards,
                                cuts.ctypes.data), "tdbg_shard_tiles")
    return cuts


def device_count() -> int:
    n = ctypes.c_int32()
    _check(lib.tdbg_device_count(ctypes.byref(n)), "tdbg_device_count")
    return int(n.value)


# ---------------------------------------------------------------------------
# the steps either side of the path
# ---------------------------------------------------------------------------
def filtered_data_blocks(file_idx, file_offset, size, min_batch_size: int = 20971520,
                         max_batch_size: int = 104857600, min_batch_gap: int = 512000) -> np.ndarray:
    """FilteredData blocks (filtered_data.h:531-575) of tiles in result-tile
    order: the first tile of every block, then ntiles."""
    fi = np.ascontiguousarray(file_idx, dtype=np.uint32)
    fo = np.ascontiguousarray(file_offset, dtype=np.uint64)
    sz = np.ascontiguousarray(size, dtype=np.uint64)
    first = np.zeros(fi.size + 1, dtype=np.uint64)
    nb = ctypes.c_uint64()
    _check(lib.tdbg_filtered_data_blocks(fi.size, fi.ctypes.data, fo.ctypes.data, sz.ctypes.data, min_batch_size,
                                         max_batch_size, min_batch_gap, first.ctypes.data, ctypes.byref(nb)),
           "tdbg_filtered_data_blocks")
    n = int(nb.value)
    return np.concatenate([first[:n], [fi.size]]).astype(np.uint64) if fi.size else np.zeros(1, np.uint64)


class HostBuffer:
    """Pinned host memory on a device's NUMA node (tdbg_host_alloc_local)."""

    def __init__(self, device: int, nbytes: int):
        p = ctypes.c_void_p()
        _check(lib.tdbg_host_alloc_local(device, nbytes, ctypes.byref(p)), "tdbg_host_alloc_local")
        self.ptr = int(p.value or 0)
        self.nbytes = nbytes
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * max(nbytes, 1)).from_address(self.ptr))[:nbytes]

    def __del__(self, _free=lib.tdbg_host_free, _down=_SHUTDOWN):
        if getattr(self, "ptr", 0) and not _down:
            _free(ctypes.c_void_p(self.ptr))
            self.ptr = 0


def dense_config(cell_size: int, tile_extent, sub_lo, sub_hi, cell_order: int = 0,
                 layout: int = 0) -> "_native.DenseCopyConfig":
    """tdbg_dense_copy_config: row-major = 0, col-major = 1."""
    g = _native.DenseCopyConfig()
    nd = len(tile_extent)
    g.dim_num, g.cell_size, g.cell_order, g.layout = nd, cell_size, cell_order, layout
    for d in range(nd):
        g.tile_extent[d], g.sub_lo[d], g.sub_hi[d] = int(tile_extent[d]), int(sub_lo[d]), int(sub_hi[d])
    return g


def dense_frag_config(cell_size: int, tile_extent, sub_lo, sub_hi, nfrag: int, fill_size: int, cell_order: int = 0,
                      layout: int = 0, nullable: bool = False, fill_validity: int = 0, elements_mode: bool = False,
                      data_type_size: int = 1) -> "_native.DenseFragConfig":
    """tdbg_dense_frag_config: several fragments (the lower index wins), fill values, var cells."""
    f = _native.DenseFragConfig()
    f.base = dense_config(cell_size, tile_extent, sub_lo, sub_hi, cell_order, layout)
    f.nfrag, f.nullable, f.fill_size, f.fill_validity = nfrag, int(nullable), fill_size, fill_validity
    f.elements_mode, f.data_type_size = int(elements_mode), data_type_size
    return f


def dense_result_bytes(cfg) -> int:
    return int(lib.tdbg_dense_result_bytes(ctypes.byref(cfg)))
