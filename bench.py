#!/usr/bin/env python
"""bench.py -- BASELINE.json metric: Mrays/s + frames/s at 1080p, 32 candidates, 4 spatial neighbours.

Workload (configs[1], C2): Cornell box with 1024 emissive quads (2048 emissive triangles), 1920x1080,
A=32 area + B=1 BRDF candidates, spatial reuse k=4 P=1 R=30 CONSTANT MIS, temporal off, cap 20.
A "step" is one frame of the hot path (SimpleGuiDX11::produceRestir, pg/simpleguidx11.cpp:359-487):
G-buffer + initial RIS, spatial reuse, shade.  Scene + buffers are resident in HBM before timing.

N=1: one GPU renders the whole frame.  N>1 (torchrun): the frame is split into N row bands
(strong scaling, one process per GPU); reservoir halo rows are exchanged over RCCL before each
spatial pass and the band framebuffers are gathered to rank 0 (restir_amd/distributed.py).

Frames are pipelined by the library (run-ahead lanes, up to 3 frames in flight; RESTIR_RUNAHEAD=0
renders strictly one frame after the other); every frame is still rendered completely.

Output: one JSON line (rank 0) with value = whole-job frames/s, plus mrays_per_s, roofline of the
dominant kernel (k_gbuffer_initial, algorithmic bytes, HIP-event timed on its stream), the whole-frame
roofline at the job's frame rate, and cpu_baseline (the oracle restatement on this host's cores, N=1
only).
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "restir-embree_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
C5_FRAMES = 240
TUNE_FRAMES = 6                # RS_TRAVERSAL_AUTO tuning frames (2 kinds x kTuneRuns, restir_capi.hip)
VALU_PEAK_GIPS = 256 * 4 * 2.4 / 2   # wave64 VALU instr/ns: 1024 SIMD-32s, 2 cycles each, 2.4 GHz
WORKLOADS = {
    "C1": "Cornell box, 8 emissive quads, reference defaults (A=1 B=1, no reuse)",
    "C2": "Cornell box + 1024 emissive quads, A=32 B=1, spatial k=4 P=1 R=30 CONSTANT MIS, temporal off, cap 20",
    "C2V": "C2 with doVisibilityPass (initial candidates without shadow rays, one visibility ray per pixel)",
    "C3": "Sponza-like ~250k tris, 4096 emissive triangles (2048 lamp quads), A=32 B=1, temporal + spatial k=4 P=1 R=30, cap 20",
    "C5": "C2 scene, 240-frame camera orbit (r=0.3) + moving lights (light CDF recomputed + BVH refit on the GPU every frame), A=32 B=1, temporal + spatial k=4 P=1 R=30, cap 20",
}
# algorithmic bytes per pixel of the dominant kernel k_gbuffer_initial: G-buffer record write
# (5 x float4 = 80 B) + reservoir write (3 x float4 = 48 B); scene/BVH reads are cache-resident
# shared data, not per-pixel traffic.  DESIGN.md "Roofline".
DOMINANT_BYTES_PER_PX = 80 + 48


def frame_bytes_per_px(prm) -> int:
    """Compulsory HBM bytes per pixel of one whole frame in this build's layout (each per-pixel record
    read / written once per pass; neighbour and reprojected reads are the same records): initial
    G + R write 128; visibility pass 68; temporal G cur + G prev + R cur + R prev read, R write 304; each spatial pass G + R
    read, R write 176; framebuffer write 12 (fused into the last pass; a separate shade pass reads
    G + R: +128).  SURVEY.md §8(d) prices the reference's unfused passes (480 B at C2)."""
    b = 128
    if prm.do_visibility_pass:                 # G position + reservoir read, W write
        b += 16 + 48 + 4
    if prm.do_temporal:
        b += 304
    if prm.do_spatial and prm.spatial_passes > 0:
        b += 176 * prm.spatial_passes + 12
    else:
        b += 128 + 12
    return b


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--scene", default="C2", choices=["C1", "C2", "C2V", "C3", "C5"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    return ap.parse_args()


def cpu_baseline(sc, prm, W, H, threads):
    """The oracle (CPU restatement, OpenMP) timed on this host: one full frame of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib

    oracle_lib.build()
    L = oracle_lib.lib()
    n_threads = max(1, min(threads, os.cpu_count() or 1))
    L.or_set_num_threads(n_threads)
    osc = oracle_lib.OracleScene(sc)
    rr = oracle_lib.OracleRenderer(W, H)
    rr.render(osc, sc.camera, prm, 0)          # warm-up frame (page-in, caches)
    # median of up to 10 frames, bounded to ~10 s of CPU time (SURVEY.md §8d procedure, scaled down)
    times, rays = [], []
    t_start = time.perf_counter()
    for f in range(1, 11):
        t0 = time.perf_counter()
        rr.render(osc, sc.camera, prm, f)
        times.append(time.perf_counter() - t0)
        rays.append(rr.rays)
        if time.perf_counter() - t_start > 10.0:
            break
    dt = float(np.median(times))
    mr = float(np.median([r / t for r, t in zip(rays, times)])) / 1e6
    return {"value": round(1.0 / dt, 5), "unit": "frames/s", "cores": n_threads, "kind": "port",
            "sample": f"median of {len(times)} full {W}x{H} frames of the same workload after 1 warm-up frame "
                      f"(oracle/restir_oracle.c, OpenMP, {n_threads} threads); s/frame={dt:.3f}; "
                      f"Mrays/s={mr:.2f}"}


def main():
    args = parse()
    import torch
    from restir_amd import Renderer, scenes
    from restir_amd.params import metric_params, c3_params, default_params

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        if rank == 0:
            print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    # RESTIR_DIST_BACKEND=gloo rehearses the N>1 flow with more ranks than GPUs (ranks share devices,
    # halo/gather staged through host memory); the measured configuration is RCCL ("nccl"), one GPU per rank
    backend = os.environ.get("RESTIR_DIST_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist = None
    red_dev = "cpu" if backend == "gloo" else "cuda"
    if world > 1:
        import torch.distributed as dist
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    W, H = args.width, args.height
    camera = None                       # per-frame camera (C5 orbit); None = the scene's static camera
    light_pos = None                    # per-frame emissive positions (C5 moving lights)
    if args.scene == "C1":
        sc, prm = scenes.cornell_box(8), default_params()
    elif args.scene == "C2":
        sc, prm = scenes.cornell_many_lights(1024), metric_params()
    elif args.scene == "C2V":   # doVisibilityPass variant (1 shadow ray instead of A per pixel)
        sc, prm = scenes.cornell_many_lights(1024), metric_params(do_visibility_pass=1)
    elif args.scene == "C3":
        sc, prm = scenes.sponza_like(), c3_params()
    else:   # C5: C2's scene, 240-frame camera orbit + moving lights, temporal reuse with M-cap 20
        sc, prm = scenes.cornell_many_lights(1024), c3_params()
        camera = lambda f: scenes.orbit_camera(sc.camera, f % C5_FRAMES, C5_FRAMES, 0.3)
        light_pos = [scenes.moving_light_positions(sc, f, C5_FRAMES) for f in range(C5_FRAMES)]
    # render on a dedicated torch stream shared with the library, so RCCL ops and the kernels of
    # librestir_amd.so are ordered on one stream (torch's default stream has handle 0 = "none")
    torch.cuda.set_stream(torch.cuda.Stream(device=local))
    stream = torch.cuda.current_stream().cuda_stream

    if world == 1:
        r = Renderer(W, H, device=local, stream=stream)
        gs = r.load_scene(sc)
        render = lambda f: r.produce_restir(gs, camera(f) if camera else sc.camera, prm, f, copy_out=False,
                                            timed=False)
        eng = r
    else:
        from restir_amd.distributed import TiledRenderer
        # async gather: frame f's band framebuffers travel to rank 0 while frame f+1 renders
        tr = TiledRenderer(W, H, rank, world, device=local, stream=stream, async_gather=True)
        gs = tr.load_scene(sc)
        render = lambda f: tr.render(gs, camera(f) if camera else sc.camera, prm, f, gather=True, timed=False)
        eng = tr

    def step(f):
        if light_pos is not None:       # moving lights: new positions -> light CDF + BVH rebuilt (timed)
            gs.update_positions(light_pos[f % C5_FRAMES])
        return render(f)

    def barrier():
        if dist is not None:
            dist.barrier()

    # initialisation (like the scene load, outside warm-up and timing): RS_TRAVERSAL_AUTO times the two
    # BVH walk kinds over a scene's first 6 frames, then the history is reset
    for f in range(TUNE_FRAMES):
        step(f)
    if world > 1:   # cost-balanced bands from 2 frames' per-row wave times (all ranks agree; resets history)
        bands = tr.rebalance(step, n_frames=2)
        if rank == 0:
            print(f"bands: {bands}", file=sys.stderr)
    eng.reset_history()
    for f in range(args.warmup):
        step(f)
    barrier()
    torch.cuda.synchronize()
    eng.timing_totals(reset=True)            # folds the warm-up frames away; no per-frame sync below
    barrier()
    t0 = time.perf_counter()
    for f in range(args.steps):
        step(args.warmup + f)
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    tot, n_timed = eng.timing_totals()
    if n_timed != args.steps:
        print(f"warning: {n_timed} frames timed by events, expected {args.steps}", file=sys.stderr)
    keys = ("gbuffer_initial_ms", "spatial_ms", "temporal_ms", "shade_ms", "total_ms")
    acc = {k: float(getattr(tot, k)) for k in keys}
    rays = int(tot.rays)
    if dist is not None:
        tt = torch.tensor([dt, float(rays)], dtype=torch.float64, device=red_dev)
        dmax = tt.clone()
        dist.all_reduce(dmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(tt[1:], op=dist.ReduceOp.SUM)
        dt, rays = float(dmax[0]), int(tt[1])
        acc_t = torch.tensor([acc[k] for k in acc], dtype=torch.float64, device=tt.device)
        dist.all_reduce(acc_t, op=dist.ReduceOp.MAX)
        acc = {k: float(v) for k, v in zip(acc, acc_t.tolist())}
    ms_per_step = dt / args.steps * 1e3
    fps = args.steps / dt
    mrays = rays / dt / 1e6
    k_ms = acc["gbuffer_initial_ms"] / args.steps
    px_band = W * math.ceil(H / world)
    achieved = DOMINANT_BYTES_PER_PX * px_band / (k_ms * 1e-3) / 1e9 if k_ms > 0 else 0.0
    traffic = valu = frame_traffic = None
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tf) and world == 1:
        try:
            with open(tf) as f:
                pmc = json.load(f)
            if pmc.get("config") == f"{args.scene}_{W}x{H}":
                traffic = pmc.get("k_gbuffer_initial_bytes_per_launch")
                frame_traffic = pmc.get("frame_bytes")
                valu = pmc.get("k_gbuffer_initial_valu_per_launch")
        except Exception:
            traffic = valu = frame_traffic = None
    inflight = 1 + int(os.environ.get("RESTIR_RUNAHEAD", "2"))
    trav_name = None
    if world == 1:
        _, last_kind, _ = r.traversal(gs)
        trav_name = {0: "lockstep", 1: "lane"}.get(last_kind)
    else:
        _, last_kind, _ = tr.be.r.traversal(gs)
        trav_name = {0: "lockstep", 1: "lane"}.get(last_kind) + " (rank 0)"
    if rank == 0:
        out = {
            "metric": "Mrays/s + frames/s at 1080p, 32 candidates, 4 spatial neighbours",
            "value": round(fps, 4),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic (procedural scene, BASELINE.json configs[{ {'C1': 0, 'C2': 1, 'C2V': 1, 'C3': 2, 'C5': 4}[args.scene]}])",
            "config": {"workload": f"{args.scene}: {WORKLOADS[args.scene]}, {W}x{H}",
                       "width": W, "height": H, "parallelism": f"row-bands x{world}" if world > 1 else "1 GPU",
                       "traversal": trav_name, "frames_in_flight": inflight},
            "mrays_per_s": round(mrays, 2),
            "rays_per_frame": rays // max(1, args.steps),
            "pass_ms": {k: round(v / args.steps, 4) for k, v in acc.items()},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                         "kernel": "k_gbuffer_initial", "bytes_per_px": DOMINANT_BYTES_PER_PX,
                         "kernel_ms": round(k_ms, 4)},
            # the kernel's real limiter is instruction issue / latency, not HBM: VALU wave-instructions
            # per launch (PMC SQ_INSTS_VALU, profiles/pmc_traffic.json) over the live kernel time, against
            # 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU op (MI355X_MICROARCH.md)
            # the whole frame (all passes) at the job's frame rate -- with frames in flight on the
            # library's lanes the kernels overlap, so per-kernel launch durations (above) include the
            # time they share the GPU with other frames' kernels; this is the pipeline's figure
            "frame_roofline": {"bound": "hbm", "bytes_per_px": frame_bytes_per_px(prm), "unit": "GB/s",
                               "achieved": round(frame_bytes_per_px(prm) * W * H / (ms_per_step * 1e-3) / 1e9, 2),
                               "peak": HBM_PEAK_GBS, "traffic": frame_traffic,
                               "frac": round(frame_bytes_per_px(prm) * W * H / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 6)},
            "valu_issue": None if not valu or k_ms <= 0 else {
                "achieved": round(valu / (k_ms * 1e-3) / 1e9, 2), "peak": VALU_PEAK_GIPS, "unit": "G wave-instr/s",
                "frac": round(valu / (k_ms * 1e-3) / 1e9 / VALU_PEAK_GIPS, 4), "valu_per_launch": valu},
        }
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(sc, prm, W, H, args.cpu_threads)
            except Exception as e:  # the baseline is reported, never required for the GPU number
                out["cpu_baseline"] = {"value": None, "error": repr(e)}
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
