"""Tile-sharded frames across the GPUs of one node.

One process per GPU.  The 1080p (or 4K) frame is split into ``world`` row bands; every rank holds a
full scene replica (the GPU LBVH build is deterministic, so the trees are identical).  Per frame:

  rank r:  rs_tile_begin   G-buffer for band +- margin rows (recomputed, no exchange: one primary ray
                           per pixel), initial RIS (+ visibility) for the band
           rs_tile_temporal
           for each spatial pass p:
               halo exchange  reservoir rows [y0, y0+h) -> rank r-1, [y1-h, y1) -> rank r+1 and the
                              matching receives into [y0-h, y0) / [y1, y1+h): point-to-point
                              send/recv (RCCL over xGMI), 48 B/px, h = floor(sqrt(R)) rows
                              (the largest |offset| sampleDiskUniform can produce,
                              pg/Sampling.cpp:78-87 + truncation pg/ReSTIRIntegrator.cpp:338)
               rs_tile_spatial(p)
           rs_tile_finish  shade -> band framebuffer
  gather:  band framebuffers (12 B/px) -> rank 0 (each peer sends over its own xGMI link): one
           batched point-to-point group straight into rank 0's full-frame buffer (no staging copy);
           with async_gather the next frames render while it is in flight

Frames in flight: the library runs consecutive frames on rotating "lane" streams (run-ahead,
rs_context_set_run_ahead); each frame's halo exchange and gather are issued on its lane's stream
through that lane's own process group, so a frame's communication overlaps other frames' compute.

Load balance: bands start equal; ``rebalance`` moves the boundaries so every rank's measured cost
(per-row wave time recorded by the pass kernels, rs_context_track_row_costs) is equal -- the rows of a
Cornell box's ceiling (cheap emissive pixels) and floor (every light visible) differ ~2x in cost.
Band placement never changes the frame (tests), only which GPU computes which rows.

The per-pixel counter RNG is keyed by the full-frame pixel index, so the gathered frame is bit-identical
to a single-GPU frame (tests/test_distributed.py, tests/test_gpu_tiles.py).  Temporal reprojection
reads the previous (and, for its forward check, the current) G-buffer at reprojected pixels; a tile
holds its rows +- max(halo, ``temporal_margin``) and rebuilds the rare element beyond them from the
frame's camera (gBufferFillPass is a function of camera and pixel), so no margin beyond the spatial
halo is needed for bit-identical frames.
"""
from __future__ import annotations

import ctypes

import numpy as np


def band_rows(H: int, rank: int, world: int):
    return (rank * H) // world, ((rank + 1) * H) // world


def halo_rows(params) -> int:
    if not params.do_spatial or params.spatial_passes <= 0:
        return 0
    # float32 semantics, as the device forms the offset (trunc(sqrtf(U(0,R)) * cos)): for R just below a
    # perfect square (24.999998f) sqrtf rounds to 5.0 where a float64 sqrt would give a 4-row halo
    r = np.float32(max(0.0, float(params.spatial_radius)))
    return int(np.floor(np.sqrt(r, dtype=np.float32)))


class _CudaBuf:
    """Zero-copy view of a device pointer for torch.as_tensor (CUDA array interface)."""

    def __init__(self, ptr: int, nbytes: int, typestr="|u1", itemsize=1):
        self.__cuda_array_interface__ = {"shape": (nbytes // itemsize,), "typestr": typestr,
                                         "data": (int(ptr), False), "version": 2, "strides": None}


class GpuTileBackend:
    """Tile stages of librestir_amd.so on one HIP device (torch's current stream)."""

    def __init__(self, renderer):
        self.r = renderer
        self._views = {}
        self._streams = {}
        self._lane_stream = None

    def _sync_if_foreign_stream(self):
        """Tensor views are consumed on torch's current stream; unless that is the frame's own stream
        (TiledRenderer runs each frame's communication on it) or the context's, wait for the context."""
        import torch
        cur = torch.cuda.current_stream().cuda_stream
        if self.r.stream is None or cur not in (self.r.stream, self._lane_stream):
            self.r.synchronize()

    def frame_stream(self):
        """(torch stream of the frame in flight, its lane) -- the frame's run-ahead lane (rs_tile_stream)."""
        import torch
        ptr, lane = self.r.tile_stream()
        st = self._streams.get(ptr)
        if st is None:
            st = self._streams[ptr] = torch.cuda.ExternalStream(ptr)
        self._lane_stream = ptr
        return st, lane

    def _view(self, ptr, nbytes, typestr="|u1", itemsize=1):
        """Cached zero-copy tensor over device memory (the buffers live as long as the context)."""
        import torch
        key = (ptr, nbytes, typestr)
        t = self._views.get(key)
        if t is None:
            t = self._views[key] = torch.as_tensor(_CudaBuf(ptr, nbytes, typestr, itemsize), device="cuda")
        return t

    def load_scene(self, scene):
        return self.r.load_scene(scene)

    def run_ahead_lanes(self) -> int:
        return run_ahead_lanes()

    def set_frame_ring(self, n):
        self.r.set_frame_ring(n)

    def track_row_costs(self, enable=True):
        self.r.track_row_costs(enable)

    def row_costs(self, reset=True):
        return self.r.row_costs(reset)

    def begin(self, scene, camera, params, frame, y0, y1, margin, halo):
        self.y0, self.y1 = y0, y1
        self.r.tile_begin(scene, camera, params, frame, y0, y1, margin, halo)

    def halo_tensor(self, which: int, on_frame_stream: bool = False):
        if not on_frame_stream:
            self._sync_if_foreign_stream()
        ptr, n = self.r.tile_halo_ptr(which)
        if not ptr:
            return None
        return self._view(ptr, n)

    def temporal(self):
        self.r.tile_temporal()

    def spatial(self, p):
        self.r.tile_spatial(p)

    def finish(self, timed=False, on_frame_stream: bool = False):
        ptr = self.r.tile_finish(timed)
        if not on_frame_stream:
            self._sync_if_foreign_stream()
        n = (self.y1 - self.y0) * self.r.W * 3
        return self._view(ptr, n * 4, "<f4", 4)

    @property
    def last_times(self):
        return self.r.last_times

    def timing_totals(self, reset=False):
        return self.r.timing_totals(reset)

    def reset_history(self):
        self.r.reset_history()


def _torch_stream(st):
    import torch
    return torch.cuda.stream(st)


def balanced_bands(costs, world: int, min_rows: int = 1, grain: int = 1):
    """Contiguous row bands [(y0, y1)] * world with (as nearly as rows allow) equal summed cost.
    Deterministic (every rank computes the same split from the same all-reduced costs); every band
    keeps >= min_rows rows (the spatial halo must fit inside a neighbour's band).  grain > 1: boundaries on
    multiples of grain rows (csrc/rs_mgpu_core.h balanced_bounds_grain: whole 8-row wave tiles), falling back
    to single rows when H is not a multiple of grain or the bands of min_rows do not fit in whole units."""
    c = np.asarray(costs, np.float64)
    H = c.shape[0]
    if grain > 1:
        G, mg = -(-H // grain), -(-min_rows // grain)
        if H % grain == 0 and world * mg <= G:
            cc = np.where(np.isfinite(c) & (c > 0), c, 0.0)
            cg = np.zeros(G)
            np.add.at(cg, np.arange(H) // grain, cc)
            b = balanced_bands(cg, world, mg)
            ys = [0] + [min(e * grain, H) for _, e in b[:-1]] + [H]
            return [(ys[r], ys[r + 1]) for r in range(world)]
    if world * min_rows > H:
        raise ValueError(f"{world} bands of >= {min_rows} rows do not fit in {H} rows")
    c = np.where(np.isfinite(c) & (c > 0), c, 0.0)
    if c.sum() <= 0:
        return [band_rows(H, r, world) for r in range(world)]
    c = c + c.sum() * 1e-6 / H                      # no zero-cost plateaus: boundaries stay put
    cum = np.concatenate([[0.0], np.cumsum(c)])
    bounds = [0]
    for r in range(1, world):
        y = int(np.searchsorted(cum, cum[-1] * r / world))
        y = max(bounds[-1] + min_rows, min(y, H - (world - r) * min_rows))
        bounds.append(y)
    bounds.append(H)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


BAND_GRAIN = 8      # band boundaries on whole 8-row wave tiles (rs_mgpu.hip kBandGrain)
DEFAULT_LANES = 3   # lanes of a backend that does not say (the library's default run-ahead depth 2, + 1)


def run_ahead_lanes() -> int:
    """Run-ahead lanes of a context: rs_max_run_ahead() + 1 (the library's build constant)."""
    from .renderer import load_library
    return int(load_library().rs_max_run_ahead()) + 1


class TiledRenderer:
    def __init__(self, W: int, H: int, rank: int, world: int, device: int = 0, stream=None, backend=None,
                 temporal_margin: int = 0, group=None, async_gather: bool = False):
        self.W, self.H, self.rank, self.world = W, H, rank, world
        self.bands = [band_rows(H, r, world) for r in range(world)]
        self.temporal_margin = temporal_margin
        self.group = group
        if backend is None:
            from .renderer import Renderer
            backend = GpuTileBackend(Renderer(W, H, device=device, stream=stream))
        self.be = backend
        # one process group per run-ahead lane: frames in flight on different lanes exchange halos and
        # gather through independent communicators (one group's collectives run in issue order).  The lane
        # count is the backend's (a CPU backend never loads the HIP library for it -- ADVICE r4)
        lanes_of = getattr(backend, "run_ahead_lanes", None)
        lanes = int(lanes_of()) if callable(lanes_of) else DEFAULT_LANES
        self.lane_groups = [group] * lanes
        if world > 1:
            import torch.distributed as dist
            ranks = list(range(world)) if group is None else dist.get_process_group_ranks(group)
            self.lane_groups = [group] + [dist.new_group(ranks=ranks) for _ in range(lanes - 1)]
        self.frame = None
        self.async_gather = async_gather and world > 1
        if self.async_gather:
            self.be.set_frame_ring(2)
        self._inflight = [[] for _ in range(lanes)]   # gather works per lane (its framebuffer)
        self._out = [None] * lanes                    # rank 0's full-frame buffers, per lane
        self._recv_ops = {}

    @property
    def y0(self):
        return self.bands[self.rank][0]

    @property
    def y1(self):
        return self.bands[self.rank][1]

    def set_bands(self, bands):
        bands = [(int(a), int(b)) for a, b in bands]
        if len(bands) != self.world or bands[0][0] != 0 or bands[-1][1] != self.H or \
                any(a >= b for a, b in bands) or any(bands[i][1] != bands[i + 1][0] for i in range(self.world - 1)):
            raise ValueError(f"bands must tile [0, {self.H}) contiguously, one per rank: {bands}")
        self.wait()
        self.bands = bands

    def load_scene(self, scene):
        return self.be.load_scene(scene)

    @property
    def last_times(self):
        return self.be.last_times

    def timing_totals(self, reset=False):
        """This rank's (PassTimes totals, n_frames) -- see Renderer.timing_totals."""
        return self.be.timing_totals(reset)

    def reset_history(self):
        self.be.reset_history()

    def wait(self):
        """Order every in-flight gather before later work on the current stream."""
        for slot in self._inflight:
            for w in slot:
                w.wait()
            slot.clear()

    def rebalance(self, render_frame, n_frames: int = 2, min_rows: int | None = None):
        """Measure per-row cost over ``n_frames`` calls of ``render_frame(i)`` (this renderer's frames,
        any content), all-reduce the rows' costs, move the band boundaries to equalise them, reset the
        history (the previous G-buffer rows of a moved band belong to another rank).  Returns the bands."""
        import torch
        import torch.distributed as dist
        if self.world == 1:
            return self.bands
        self.be.track_row_costs(True)
        self.be.row_costs(reset=True)
        for i in range(n_frames):
            render_frame(i)
        self.wait()
        costs = self.be.row_costs(reset=True)
        self.be.track_row_costs(False)
        dev = "cpu" if dist.get_backend(self.group) == "gloo" else "cuda"
        t = torch.as_tensor(costs.astype(np.float64), device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        total = t.cpu().numpy()
        h = max(1, min_rows if min_rows is not None else 8)
        self.set_bands(balanced_bands(total, self.world, h, grain=BAND_GRAIN))
        self.reset_history()
        return self.bands

    def _staged(self, t) -> bool:
        """gloo cannot move device tensors: stage them through host memory (tests only -- RCCL refuses
        two ranks on one GPU, so multi-process GPU tests run the real backend over gloo)."""
        import torch.distributed as dist
        return t is not None and t.is_cuda and dist.get_backend(self.group) == "gloo"

    def _exchange_halo(self, group=None, on_frame_stream=False):
        import torch.distributed as dist
        group = self.group if group is None else group
        ops, copy_back = [], []
        up, down = self.rank - 1, self.rank + 1
        kw = {"on_frame_stream": True} if on_frame_stream else {}
        for peer, send_which, recv_which in ((up, 2, 0), (down, 3, 1)):
            if peer < 0 or peer >= self.world:
                continue
            s, r = self.be.halo_tensor(send_which, **kw), self.be.halo_tensor(recv_which, **kw)
            if s is None or r is None:
                continue
            if self._staged(s):
                rh = r.new_empty(r.shape, device="cpu")
                copy_back.append((r, rh))
                s, r = s.cpu(), rh
            ops += [dist.P2POp(dist.isend, s, peer, group), dist.P2POp(dist.irecv, r, peer, group)]
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        for dev, host in copy_back:
            dev.copy_(host)

    def render(self, scene, camera, params, frame_index: int, gather: bool = True, timed: bool = False):
        """One frame; returns the full (H, W, 3) frame on rank 0 when gather=True (else None / band).
        With async_gather the returned frame is complete once the stream (or ``wait()``) is synchronised."""
        halo = halo_rows(params) if self.world > 1 else 0
        if halo and min(b - a for a, b in self.bands) < halo:
            raise ValueError(f"a band is thinner than the spatial halo {halo}: too many ranks for H={self.H}")
        margin = max(halo, self.temporal_margin if params.do_temporal else 0) if self.world > 1 else 0
        be = self.be
        be.begin(scene, camera, params, frame_index, self.y0, self.y1, margin, halo)
        st, k = be.frame_stream() if hasattr(be, "frame_stream") else (None, 0)
        import contextlib
        with (contextlib.nullcontext() if st is None else _torch_stream(st)):
            for w in self._inflight[k]:        # the gather that last read this lane's framebuffer
                w.wait()
            self._inflight[k].clear()
            be.temporal()
            if params.do_spatial:
                for p in range(params.spatial_passes):
                    if self.world > 1:
                        self._exchange_halo(self.lane_groups[k], on_frame_stream=st is not None)
                    be.spatial(p)
            band = be.finish(timed, on_frame_stream=True) if st is not None else be.finish(timed)
            if not gather:
                return band
            return self._gather(band, k)

    def _gather(self, band, k=0):
        """Band framebuffers -> rank 0's full frame: rank r > 0 sends its band, rank 0 receives every
        band straight into its rows of the frame (one batched P2P group; sizes may differ per rank)."""
        import torch
        import torch.distributed as dist
        if self.world == 1:
            self.frame = band.reshape(self.H, self.W, 3)
            return self.frame
        staged = self._staged(band)
        src = band.cpu() if staged else band
        row = self.W * 3
        if self.rank == 0:
            out = self._out[k]
            if out is None or out.device != src.device:
                out = self._out[k] = torch.empty(self.H * row, dtype=torch.float32, device=src.device)
            key = (k, tuple(self.bands), out.data_ptr())
            ops = self._recv_ops.get(key)
            if ops is None:                    # the receive descriptors of a lane's frame buffer, reused
                grp = self.lane_groups[k]
                ops = self._recv_ops[key] = [dist.P2POp(dist.irecv, out[a * row:b * row], r, grp)
                                             for r, (a, b) in enumerate(self.bands) if r != 0]
            out[self.y0 * row:self.y1 * row].copy_(src)
            works = dist.batch_isend_irecv(ops) if ops else []
            self.frame = out.reshape(self.H, self.W, 3)
        else:
            works = dist.batch_isend_irecv([dist.P2POp(dist.isend, src, 0, self.lane_groups[k])])
            self.frame = None
        if self.async_gather and not staged:
            self._inflight[k].extend(works)
        else:
            for w in works:
                w.wait()
        return self.frame
