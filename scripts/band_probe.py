"""Diagnostic (GPU box, 1 GPU): what one rank of an N-GPU row-band frame costs, without the
communication -- the compute + host-overhead floor of bench.py --gpus N.  For N in (1, 2, 4, 8) it renders
the middle band of the frame (rank N//2, margin/halo as TiledRenderer sets them) K times through the
tile ABI and reports wall ms/frame, GPU ms/frame (event ring) and host ms per render() call.
--gather: rank 0 also receives the other ranks' band framebuffers -- N-1 device-to-device copies of their rows into
its frame on the frame's lane stream after its shade, as rs_mgpu issues the RCCL receives (the local stand-in for
the xGMI gather; on 8 GPUs each band arrives over its own link in parallel).
Usage: python scripts/band_probe.py [--scene C2|C3|C5] [--steps K] [--balanced] [--all-ranks N [--refine R]] [--gather]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "restir-embree_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="C2")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--split", default="auto", help="initial-pass candidate split: auto|on|off")
    ap.add_argument("--balanced", action="store_true", help="cost-balanced bands (row costs of a full frame)")
    ap.add_argument("--inflight", type=int, default=1, help="frames in flight (contexts on separate streams)")
    ap.add_argument("--ahead", type=int, default=-1, help="run-ahead depth (default: the library's)")
    ap.add_argument("--only-n", type=int, default=0, help="only this N (rank N//2)")
    ap.add_argument("--all-ranks", type=int, default=0, help="time every rank of this N instead")
    ap.add_argument("--refine", type=int, default=0,
                    help="with --all-ranks: rounds of time-based rebalancing (each band's row costs rescaled to its "
                         "measured time, bands balanced again; the rs_mgpu_rebalance refinement)")
    ap.add_argument("--gather", action="store_true", help="rank 0: + the N-1 band framebuffer copies into its frame")
    a = ap.parse_args()
    import torch
    from restir_amd import Renderer, scenes
    from restir_amd.params import metric_params, c3_params
    from restir_amd.distributed import band_rows, halo_rows, balanced_bands, BAND_GRAIN, _CudaBuf

    sc = scenes.sponza_like() if a.scene == "C3" else scenes.cornell_many_lights(1024)
    prm = metric_params() if a.scene == "C2" else c3_params()
    W, H = a.width, a.height
    streams = [torch.cuda.Stream() for _ in range(a.inflight)]
    rs = [Renderer(W, H, device=0, stream=st.cuda_stream) for st in streams]
    for x in rs:
        x.set_initial_split(a.split)
        if a.ahead >= 0:
            x.set_run_ahead(a.ahead)
    gss = [x.load_scene(sc) for x in rs]
    r, gs = rs[0], gss[0]
    costs = None
    if a.balanced:   # row costs from full frames of a separate context (the probed scene tunes on its band)
        rc = Renderer(W, H, device=0, stream=streams[0].cuda_stream)
        gc = rc.load_scene(sc)
        for f in range(6):          # traversal tuning first (bench.py order): costs of the settled kind only
            rc.produce_restir(gc, sc.camera, prm, f, copy_out=False, timed=False)
        rc.track_row_costs(True)
        for f in range(6, 10):
            rc.produce_restir(gc, sc.camera, prm, f, copy_out=False, timed=False)
        costs = rc.row_costs(reset=True)
        del rc, gc
    cases = [(N, N // 2) for N in (1, 2, 4, 8)]
    if a.only_n:
        cases = [(a.only_n, a.only_n // 2)]
    if a.all_ranks:
        cases = [(a.all_ranks, k) for k in range(a.all_ranks)]
    bands_of = {}
    for N in {n for n, _ in cases}:
        bands_of[N] = balanced_bands(costs, N, 8, grain=BAND_GRAIN) if costs is not None else [band_rows(H, k, N) for k in range(N)]

    gather_src = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda") if a.gather else None

    def probe(N, rank, y0, y1, tag="", bands=None):
        halo = halo_rows(prm) if N > 1 else 0
        gather = a.gather and rank == 0 and N > 1 and bands is not None
        margin = halo          # rs_mgpu_render_frame's G-buffer margin (a temporal reprojection beyond it rebuilds)

        def frame(f):
            r, gs = rs[f % len(rs)], gss[f % len(rs)]
            r.tile_begin(gs, sc.camera, prm, f, y0, y1, margin, halo)
            r.tile_temporal()
            for p in range(prm.spatial_passes if prm.do_spatial else 0):
                r.tile_halo_ptr(0)
                r.tile_spatial(p)
            sp = r.tile_stream()[0] if gather else None
            band = r.tile_finish(False)
            if gather:      # the other ranks' rows into this frame, on its lane stream (rs_mgpu's receive order)
                fb = torch.as_tensor(_CudaBuf(band - y0 * W * 12, W * H * 12, "<f4", 4), device="cuda")
                with torch.cuda.stream(torch.cuda.ExternalStream(sp)):
                    for k, (b0, b1) in enumerate(bands):
                        if k != rank:
                            fb[b0 * W * 3:b1 * W * 3].copy_(gather_src[b0 * W * 3:b1 * W * 3])

        for f in range(6):
            frame(f)
        for x in rs:
            x.reset_history()
        for f in range(3):
            frame(f)
        torch.cuda.synchronize()
        for x in rs:
            x.timing_totals(reset=True)
        host = 0.0
        t0 = time.perf_counter()
        for f in range(a.steps):
            h0 = time.perf_counter()
            frame(3 + f)
            host += time.perf_counter() - h0
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        tot, n = r.timing_totals()
        print(f"{tag}{a.scene} ahead={a.ahead} inflight={a.inflight} split={a.split}:{int(r.initial_split()[1])} N={N} rank={rank} rows={y1 - y0} margin={margin}{' +gather' if gather else ''}: wall {dt / a.steps * 1e3:.4f} ms/frame, "
              f"gpu {tot.total_ms / n:.4f} ms (initial {tot.gbuffer_initial_ms / n:.4f}, spatial {tot.spatial_ms / n:.4f}, "
              f"temporal {tot.temporal_ms / n:.4f}), host {host / a.steps * 1e3:.4f} ms/call; "
              f"ideal (N=1 / N) -> efficiency bound", flush=True)
        return dt / a.steps * 1e3

    if a.all_ranks and a.refine and costs is not None:
        N = a.all_ranks
        c = np.asarray(costs, np.float64).copy()
        bands = bands_of[N]
        for it in range(a.refine + 1):
            t = [probe(N, k, y0, y1, f"[round {it}] ", bands) for k, (y0, y1) in enumerate(bands)]
            print(f"[round {it}] bands {[y1 - y0 for y0, y1 in bands]}: max {max(t):.4f} mean {np.mean(t):.4f} ms",
                  flush=True)
            for (y0, y1), tk in zip(bands, t):          # each band's rows rescaled to its measured time
                ck = c[y0:y1].sum()
                if ck > 0:
                    c[y0:y1] *= tk / ck
            bands = balanced_bands(c, N, 8, grain=BAND_GRAIN)
        return
    for N, rank in cases:
        y0, y1 = bands_of[N][rank]
        probe(N, rank, y0, y1, bands=bands_of[N])


if __name__ == "__main__":
    main()
