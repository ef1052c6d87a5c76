"""Row-band sharded frames through the C ABI (rs_mgpu_*, include/restir_c.h).

The orchestration (stages, halo exchange, gather, band balancing) is native (csrc/rs_mgpu.hip over
rs_mgpu_core.h); this is a thin ctypes caller.  Two modes:

  * RCCL: one process per GPU, ``MultiGpuFrame(renderer, rank=r, world=n, unique_id=id)`` where rank 0
    made ``id = MultiGpuFrame.unique_id()`` and the caller distributed it (bench.py: torch.distributed
    gloo broadcast -- the control plane only; every frame transfer is RCCL point-to-point on the
    frame's stream inside the library);
  * local: ``MultiGpuFrame([r0, r1, ...])`` -- several contexts of one process (device copies).
"""
from __future__ import annotations

import ctypes

import numpy as np

from .renderer import CameraDesc, PassTimes, RestirError, camera_desc, load_library

ID_BYTES = 128
DEFAULT_REFINE = 2        # rs_mgpu_rebalance's time-based refinement rounds unless the caller says otherwise


class MgpuStats(ctypes.Structure):
    """rs_mgpu_stats (include/restir_c.h)"""
    _fields_ = [("frames", ctypes.c_uint64), ("halo_bytes_sent", ctypes.c_uint64), ("halo_bytes_recv", ctypes.c_uint64),
                ("gather_bytes", ctypes.c_uint64), ("halo_ms", ctypes.c_double), ("gather_ms", ctypes.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def _addr(h):
    return h.value if isinstance(h, ctypes.c_void_p) else int(h)


class MultiGpuFrame:
    def __init__(self, renderers, rank: int | None = None, world: int | None = None, unique_id: bytes | None = None):
        self.lib = load_library()
        self.h = ctypes.c_void_p()
        if isinstance(renderers, (list, tuple)):
            self.renderers = list(renderers)
            arr = (ctypes.c_void_p * len(self.renderers))(*[_addr(r.h) for r in self.renderers])
            self._check(self.lib.rs_mgpu_create_local(arr, len(self.renderers), ctypes.byref(self.h)))
            self.world, self.rank = len(self.renderers), 0
        else:
            self.renderers = [renderers]
            if rank is None or world is None or unique_id is None or len(unique_id) != ID_BYTES:
                raise ValueError("RCCL mode needs rank, world and the 128-byte unique id from rank 0")
            buf = (ctypes.c_uint8 * ID_BYTES).from_buffer_copy(bytes(unique_id))
            self._check(self.lib.rs_mgpu_create(renderers.h, int(rank), int(world), buf, ctypes.byref(self.h)))
            self.world, self.rank = int(world), int(rank)
        self.W, self.H = self.renderers[0].W, self.renderers[0].H
        self.last_times = PassTimes()

    @staticmethod
    def unique_id() -> bytes:
        lib = load_library()
        buf = (ctypes.c_uint8 * ID_BYTES)()
        rc = lib.rs_mgpu_unique_id(buf)
        if rc:
            raise RestirError(f"rs_mgpu_unique_id failed ({rc})")
        return bytes(buf)

    def _check(self, rc):
        if rc:
            msg = self.lib.rs_last_error(self.renderers[0].h if getattr(self, "renderers", None) else None)
            raise RestirError(f"rs_mgpu: {msg.decode() if msg else rc}")

    def _scenes(self, scenes):
        if not isinstance(scenes, (list, tuple)):
            scenes = [scenes]
        if len(scenes) != len(self.renderers):
            raise ValueError("one scene per local rank")
        return (ctypes.c_void_p * len(scenes))(*[_addr(s.h) for s in scenes])

    def bands(self):
        b = (ctypes.c_int32 * (self.world + 1))()
        self._check(self.lib.rs_mgpu_get_bands(self.h, b))
        return [(b[i], b[i + 1]) for i in range(self.world)]

    def set_bands(self, bands):
        b = [bands[0][0]] + [y1 for _, y1 in bands]
        arr = (ctypes.c_int32 * (self.world + 1))(*b)
        self._check(self.lib.rs_mgpu_set_bands(self.h, arr))

    def rebalance(self, scenes, camera, params, first_frame: int = 0, n_frames: int = 2, min_rows: int = 8,
                  refine: int | None = None):
        """Cost-balanced bands (rs_mgpu_rebalance): row costs, then `refine` rounds of time-based refinement
        (None: the library's default, DEFAULT_REFINE = 2, whatever an earlier call set; 0: row costs only).
        rebalance_times() has the measured rounds."""
        rounds = DEFAULT_REFINE if refine is None else int(refine)
        self._check(self.lib.rs_mgpu_set_rebalance_refine(self.h, rounds))
        cam = camera_desc(camera)
        self._check(self.lib.rs_mgpu_rebalance(self.h, self._scenes(scenes), ctypes.byref(cam), ctypes.byref(params),
                                               int(first_frame), int(n_frames), int(min_rows)))
        return self.bands()

    def rebalance_times(self):
        """Every rank's measured ms per frame for each measured refinement round of the last rebalance."""
        out = []
        buf = (ctypes.c_double * self.world)()
        while self.lib.rs_mgpu_rebalance_times(self.h, len(out), buf) == 0:
            out.append([float(v) for v in buf])
        return out

    def render(self, scenes, camera, params, frame_index: int, gather: bool = True, copy_out: bool = False,
               timed: bool = False):
        """One frame; with copy_out (rank 0) returns the gathered (H, W, 3) frame (synchronous)."""
        cam = camera_desc(camera)
        out = np.empty((self.H, self.W, 3), np.float32) if copy_out else None
        self._check(self.lib.rs_mgpu_render_frame(
            self.h, self._scenes(scenes), ctypes.byref(cam), ctypes.byref(params), int(frame_index), 1 if gather else 0,
            out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)) if out is not None else None,
            ctypes.byref(self.last_times) if timed else None))
        return out

    def frame_device_ptr(self) -> int:
        p = ctypes.c_void_p()
        self._check(self.lib.rs_mgpu_frame_device_ptr(self.h, ctypes.byref(p)))
        return int(p.value or 0)

    def reset_history(self):
        self._check(self.lib.rs_mgpu_reset_history(self.h))

    def allreduce(self, values, op: str = "sum") -> np.ndarray:
        v = np.ascontiguousarray(values, np.float64).copy()
        self._check(self.lib.rs_mgpu_allreduce(self.h, v.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), v.size,
                                               0 if op == "sum" else 1))
        return v

    def stats(self, reset: bool = False) -> dict:
        """Transfer statistics since creation / the last reset (synchronous): halo and gather bytes, and
        the HIP-event time of the exchanges on the first local rank's frame streams."""
        st = MgpuStats()
        self._check(self.lib.rs_mgpu_get_stats(self.h, ctypes.byref(st), 1 if reset else 0))
        return st.as_dict()

    def close(self):
        if self.h:
            self.lib.rs_mgpu_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


__all__ = ["MultiGpuFrame", "CameraDesc"]
