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
  gather:  band framebuffers (12 B/px) -> rank 0 (each peer sends over its own xGMI link)

The per-pixel counter RNG is keyed by the full-frame pixel index, so the gathered frame is bit-identical
to a single-GPU frame (tests/test_distributed.py, tests/test_gpu_tiles.py).  Temporal reprojection
reads the previous G-buffer at reprojected pixels; those must lie within ``temporal_margin`` rows of
the band (counted and treated as a failed reprojection otherwise -- SURVEY.md §8e deviation note).
"""
from __future__ import annotations

import ctypes
import math

import numpy as np


def band_rows(H: int, rank: int, world: int):
    return (rank * H) // world, ((rank + 1) * H) // world


def halo_rows(params) -> int:
    if not params.do_spatial or params.spatial_passes <= 0:
        return 0
    return int(math.floor(math.sqrt(max(0.0, float(params.spatial_radius)))))


class _CudaBuf:
    """Zero-copy view of a device pointer for torch.as_tensor (CUDA array interface)."""

    def __init__(self, ptr: int, nbytes: int, typestr="|u1", itemsize=1):
        self.__cuda_array_interface__ = {"shape": (nbytes // itemsize,), "typestr": typestr,
                                         "data": (int(ptr), False), "version": 2, "strides": None}


class GpuTileBackend:
    """Tile stages of librestir_amd.so on one HIP device (torch's current stream)."""

    def __init__(self, renderer):
        self.r = renderer

    def _sync_if_foreign_stream(self):
        """Tensor views are consumed on torch's current stream; if the context renders on a stream of
        its own, wait for it (the bench creates contexts on torch's stream, so this is a no-op there)."""
        import torch
        if self.r.stream is None or self.r.stream != torch.cuda.current_stream().cuda_stream:
            self.r.synchronize()

    def load_scene(self, scene):
        return self.r.load_scene(scene)

    def begin(self, scene, camera, params, frame, y0, y1, margin, halo):
        self.y0, self.y1 = y0, y1
        self.r.tile_begin(scene, camera, params, frame, y0, y1, margin, halo)

    def halo_tensor(self, which: int):
        import torch
        self._sync_if_foreign_stream()
        ptr, n = self.r.tile_halo_ptr(which)
        if not ptr:
            return None
        return torch.as_tensor(_CudaBuf(ptr, n), device="cuda")

    def temporal(self):
        self.r.tile_temporal()

    def spatial(self, p):
        self.r.tile_spatial(p)

    def finish(self, timed=False):
        import torch
        ptr = self.r.tile_finish(timed)
        self._sync_if_foreign_stream()
        n = (self.y1 - self.y0) * self.r.W * 3
        return torch.as_tensor(_CudaBuf(ptr, n * 4, "<f4", 4), device="cuda")

    @property
    def last_times(self):
        return self.r.last_times

    def timing_totals(self, reset=False):
        return self.r.timing_totals(reset)

    def reset_history(self):
        self.r.reset_history()


class TiledRenderer:
    def __init__(self, W: int, H: int, rank: int, world: int, device: int = 0, stream=None, backend=None,
                 temporal_margin: int = 64, group=None):
        self.W, self.H, self.rank, self.world = W, H, rank, world
        self.y0, self.y1 = band_rows(H, rank, world)
        self.temporal_margin = temporal_margin
        self.group = group
        if backend is None:
            from .renderer import Renderer
            backend = GpuTileBackend(Renderer(W, H, device=device, stream=stream))
        self.be = backend
        self.frame = None

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

    def _staged(self, t) -> bool:
        """gloo cannot move device tensors: stage them through host memory (tests only -- RCCL refuses
        two ranks on one GPU, so multi-process GPU tests run the real backend over gloo)."""
        import torch.distributed as dist
        return t is not None and t.is_cuda and dist.get_backend(self.group) == "gloo"

    def _exchange_halo(self):
        import torch.distributed as dist
        ops, copy_back = [], []
        up, down = self.rank - 1, self.rank + 1
        for peer, send_which, recv_which in ((up, 2, 0), (down, 3, 1)):
            if peer < 0 or peer >= self.world:
                continue
            s, r = self.be.halo_tensor(send_which), self.be.halo_tensor(recv_which)
            if s is None or r is None:
                continue
            if self._staged(s):
                rh = r.new_empty(r.shape, device="cpu")
                copy_back.append((r, rh))
                s, r = s.cpu(), rh
            ops += [dist.P2POp(dist.isend, s, peer, self.group), dist.P2POp(dist.irecv, r, peer, self.group)]
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        for dev, host in copy_back:
            dev.copy_(host)

    def render(self, scene, camera, params, frame_index: int, gather: bool = True, timed: bool = False):
        """One frame; returns the full (H, W, 3) frame on rank 0 when gather=True (else None / band)."""
        halo = halo_rows(params) if self.world > 1 else 0
        if halo and (self.H // self.world) < halo:
            raise ValueError(f"band height {self.H // self.world} < spatial halo {halo}: too many ranks for H={self.H}")
        margin = max(halo, self.temporal_margin if params.do_temporal else 0) if self.world > 1 else 0
        be = self.be
        be.begin(scene, camera, params, frame_index, self.y0, self.y1, margin, halo)
        be.temporal()
        if params.do_spatial:
            for p in range(params.spatial_passes):
                if self.world > 1:
                    self._exchange_halo()
                be.spatial(p)
        band = be.finish(timed)
        if not gather:
            return band
        return self._gather(band)

    def _gather(self, band):
        import torch
        import torch.distributed as dist
        if self.world == 1:
            self.frame = band.reshape(self.H, self.W, 3)
            return self.frame
        max_rows = max(band_rows(self.H, r, self.world)[1] - band_rows(self.H, r, self.world)[0]
                       for r in range(self.world))
        n = max_rows * self.W * 3
        dev = "cpu" if self._staged(band) else band.device
        buf = torch.zeros(n, dtype=torch.float32, device=dev)
        buf[: band.numel()].copy_(band)
        if self.rank == 0:
            parts = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(self.world)]
            dist.gather(buf, parts, dst=0, group=self.group)
            rows = []
            for r in range(self.world):
                a, b = band_rows(self.H, r, self.world)
                rows.append(parts[r][: (b - a) * self.W * 3].reshape(b - a, self.W, 3))
            self.frame = torch.cat(rows, 0)
            return self.frame
        dist.gather(buf, None, dst=0, group=self.group)
        return None
