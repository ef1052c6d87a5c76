#!/usr/bin/env python
"""bench.py -- BASELINE.json metric: Mrays/s + frames/s at 1080p, 32 candidates, 4 spatial neighbours.

Headline workload (configs[1], C2): Cornell box with 1024 emissive 0.02 m quads (2048 emissive
triangles), 1920x1080, A=32 area + B=1 BRDF candidates, spatial reuse k=4 P=1 R=30 CONSTANT MIS,
temporal off, cap 20.  A "step" is one frame of the hot path (SimpleGuiDX11::produceRestir,
pg/simpleguidx11.cpp:359-487): G-buffer + initial RIS, spatial reuse, shade.  Scene + buffers are
resident in HBM before timing; the framebuffer stays in HBM (zero-copy, rs_get_frame_device_ptr).

N=1 also measures, under "configs" of the same JSON line, the other single-GPU configs (C3 Sponza-like
with temporal reuse, the full 240-frame C5 sequence, C2V = doVisibilityPass, C4_1gpu = C3 at 3840x2160 on
one GPU -- the denominator of the C4 speed-up), each with its own ms_per_step, Mrays/s, rooflines and a
bounded CPU baseline, the denoiser and the drop-in C++ host path (include/restir.hpp through
tools/restir_render, framebuffer copied to host memory every frame).  The printed line is compact (every
config's value, ms_per_step, rooflines and CPU baseline); the full record (per-pass times, host, limiter
details, per-layer denoiser times) goes to gpurun_out/bench_full.json.

N>1 (torchrun): the frame is split into N row bands (strong scaling, one process per GPU); reservoir
halo rows are exchanged over RCCL before each spatial pass and the band framebuffers are gathered to
rank 0 (csrc/rs_mgpu.hip).  The line carries the headline config (C2) and, under "configs", C4 (BASELINE
configs[3]: the C3 scene at 3840x2160 across the N GPUs), each with its per-rank band / halo / gather times.

Frames are pipelined by the library (run-ahead lanes, up to 3 frames in flight); every frame is still
rendered completely.  Rooflines (SURVEY.md §8(d) algorithmic bytes):
  roofline         the whole frame: B_px (480 B at C2) x pixels / ms_per_step
  kernel_roofline  the dominant kernel alone: its §8(d) bytes (186 B/px for G-buffer + initial) /
                   its launch time measured with HIP events in a second window with one frame in
                   flight (RESTIR_RUNAHEAD=0 semantics), flagged when that exceeds ms_per_step (the
                   pipelined frame hides the kernel's ramp-up and tail behind its neighbours)
  valu_issue       VALU wave-instructions per frame (rocprofv3 PMC, profiles/r04_pmc_<cfg>.json) /
                   ms_per_step against 1024 SIMDs x 2.4 GHz / 2 cycles
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "restir-embree_amd"))

import numpy as np  # noqa: E402

METRIC = "Mrays/s + frames/s at 1080p, 32 candidates, 4 spatial neighbours"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
VALU_PEAK_GIPS = 256 * 4 * 2.4 / 2   # wave64 VALU instr/ns: 1024 SIMDs, 2 cycles each, 2.4 GHz
MFMA_F16_PEAK_TFLOPS = 2500.0  # dense f16/bf16 MFMA peak (MI355X_MICROARCH.md; no sparsity)
C5_FRAMES = 240
TUNE_FRAMES = 6                # RS_TRAVERSAL_AUTO tuning frames (2 kinds x kTuneRuns, restir_capi.hip)
WORKLOADS = {
    "C1": "Cornell box, 8 emissive quads, reference defaults (A=1 B=1, no reuse)",
    "C2": "Cornell box + 1024 emissive 0.02 m quads, A=32 B=1, spatial k=4 P=1 R=30 CONSTANT MIS, temporal off, cap 20",
    "C2V": "C2 with doVisibilityPass (initial candidates without shadow rays, one visibility ray per pixel)",
    "C3": "Sponza-like ~250k tris, 4096 emissive triangles (2048 lamp quads), A=32 B=1, temporal + spatial k=4 P=1 R=30, cap 20",
    "C5": "C2 scene, 240-frame camera orbit (r=0.3) + moving lights (light CDF recomputed + BVH refit on the GPU every frame), A=32 B=1, temporal + spatial k=4 P=1 R=30, cap 20",
    "C4": "C3's Sponza-like scene and parameters at 3840x2160 (row bands across the GPUs)",
}
CONFIG_INDEX = {"C1": 0, "C2": 1, "C2V": 1, "C3": 2, "C4": 3, "C5": 4}
RES = {"C4": (3840, 2160)}      # configs quoted at another resolution than --width/--height


# SURVEY.md §8(d) algorithmic bytes per pixel-frame: G write 69, initial (G + R) 117, visibility 28,
# temporal 282, spatial pass 165, shade 129 (G = 69 B, R = 48 B, F = 12 B; history = pointer swap)
PASS_BYTES = {"gbuffer_initial_ms": 69 + 117, "visibility_ms": 28, "temporal_ms": 282, "spatial_ms": 165,
              "shade_ms": 129}
PASS_KERNEL = {"gbuffer_initial_ms": "k_gbuffer_initial", "visibility_ms": "k_visibility",
               "temporal_ms": "k_temporal", "spatial_ms": "k_spatial", "shade_ms": "k_shade"}


def survey_bytes_per_px(prm) -> int:
    V = 1 if prm.do_visibility_pass else 0
    T = 1 if prm.do_temporal else 0
    P = prm.spatial_passes if prm.do_spatial else 0
    return 69 + 117 + V * 28 + T * 282 + P * 165 + 129


def workload(name):
    from restir_amd import scenes
    from restir_amd.params import metric_params, c3_params, default_params
    camera = None                       # per-frame camera (C5 orbit); None = the scene's static camera
    light_pos = None                    # per-frame emissive positions (C5 moving lights)
    if name == "C1":
        sc, prm = scenes.cornell_box(8), default_params()
    elif name == "C2":
        sc, prm = scenes.cornell_many_lights(1024), metric_params()
    elif name == "C2V":   # doVisibilityPass variant (1 shadow ray instead of A per pixel)
        sc, prm = scenes.cornell_many_lights(1024), metric_params(do_visibility_pass=1)
    elif name in ("C3", "C4"):
        sc, prm = scenes.sponza_like(), c3_params()
        camera = lambda f: scenes.orbit_camera(sc.camera, f % C5_FRAMES, C5_FRAMES, 0.3)
    else:   # C5: C2's scene, 240-frame camera orbit + moving lights, temporal reuse with M-cap 20
        sc, prm = scenes.cornell_many_lights(1024), c3_params()
        camera = lambda f: scenes.orbit_camera(sc.camera, f % C5_FRAMES, C5_FRAMES, 0.3)
        light_pos = lambda f: scenes.moving_light_positions(sc, f % C5_FRAMES, C5_FRAMES)
    return sc, prm, camera, light_pos


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--scene", default="C2", choices=list(WORKLOADS))
    ap.add_argument("--multi-configs", default="C4",
                    help="N>1: further configs measured after --scene in the same run (comma list, '' for none)")
    ap.add_argument("--full-out", default=os.path.join(ROOT, "gpurun_out", "bench_full.json"),
                    help="the full record (the printed line is compact)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="N=1: skip the C3/C5/C2V and drop-in lines")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="oracle threads for the CPU baseline; 0 = every core available to this process")
    return ap.parse_args()


def host_cpu():
    """The host the CPU baseline runs on: CPU model (lscpu's 'Model name' = /proc/cpuinfo 'model name'),
    nproc, the cores this process may run on (sched_getaffinity), the cgroup CPU quota and OMP_NUM_THREADS
    (the pool's per-GPU CPU share)."""
    info = {"model": None, "nproc": os.cpu_count(), "affinity_cores": None, "cgroup_cpu_max": None,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.lower().startswith("model name"):
                    info["model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        info["affinity_cores"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            info["cgroup_cpu_max"] = f.read().strip()
    except OSError:
        pass
    return info


def baseline_threads(requested):
    """Every core available to the process, within the CPU share the pool grants (a cgroup quota or
    OMP_NUM_THREADS: the GPU box sets OMP_NUM_THREADS to the per-GPU share and asks worker pools to
    stay within it)."""
    if requested and requested > 0:
        return requested
    hc = host_cpu()
    n = hc["affinity_cores"] or hc["nproc"] or 1
    q = hc["cgroup_cpu_max"]
    if q and q.split()[0] != "max":
        try:
            quota, period = (int(v) for v in q.split()[:2])
            n = min(n, max(1, quota // period))
        except ValueError:
            pass
    omp = hc["omp_num_threads"]
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


# ---------------------------------------------------------------- CPU baseline (oracle = the checker)
def cpu_baseline(name, W, H, threads, budget_s=12.0):
    """The oracle (plain-C OpenMP restatement of the reference path, oracle/restir_oracle.c) timed on this
    host, on a bounded sample of the same workload: whole frames for C1/C2/C2V (median, after a warm-up
    frame); for C3/C5 (seconds per 1080p frame) a centred quarter-frame band of rows rendered through the
    oracle's tile stages (G-buffer + initial + temporal + spatial + shade of the band; the first frame
    only builds the temporal history), scaled to the full frame by rows.  Ray queries walk the oracle's
    8-wide tree with AVX2 box tests (or_scene_set_wide, SURVEY.md §8(d)'s SIMD-friendly traversal;
    the same hits as its binary walk, tests/test_oracle.py)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    oracle_lib.build()
    L = oracle_lib.lib()
    n_threads = baseline_threads(threads)
    L.or_set_num_threads(n_threads)
    sc, prm, camera, light_pos = workload(name)
    cam = camera or (lambda f: sc.camera)
    osc = oracle_lib.OracleScene(sc, wide=True)
    times, rays, band_t, refr = [], [], [], []
    t_start = time.perf_counter()
    if name in ("C3", "C5"):
        rows = max(8, H // 4)
        y0 = (H - rows) // 2
        be = oracle_lib.OracleTileBackend(W, H)
        halo = int(np.floor(np.sqrt(np.float32(prm.spatial_radius), dtype=np.float32)))
        for f in range(6):
            if light_pos is not None:
                osc = oracle_lib.OracleScene(type(sc)(light_pos(f), sc.normals, sc.tri_material, sc.materials, sc.camera),
                                             wide=True)
            t0 = time.perf_counter()
            be.begin(osc, cam(f), prm, f, y0, y0 + rows, halo, halo)
            be.temporal()
            for p in range(prm.spatial_passes):
                be.spatial(p)
            be.finish()
            dt = time.perf_counter() - t0
            if f > 0:
                times.append(dt * H / rows)
                rays.append(be.rays)
                band_t.append(dt)
                refr.append(be.reference_rays * H / rows)
            if time.perf_counter() - t_start > budget_s and len(times) >= 1:
                break
        sample = (f"{len(times)} frames of a centred {rows}-row band of {W}x{H} (oracle tile stages; after 1 "
                  f"history frame), scaled by {H}/{rows} rows")
        band = {"rows": rows, "y0": y0, "frames_timed": len(times),
                "full_frame_equivalents_timed": round(len(times) * rows / H, 4)}
        mr = float(np.median([r / t for r, t in zip(rays, band_t)])) / 1e6
    else:
        rr = oracle_lib.OracleRenderer(W, H)
        rr.render(osc, cam(0), prm, 0)          # warm-up frame (page-in, caches)
        for f in range(1, 11):
            t0 = time.perf_counter()
            rr.render(osc, cam(f), prm, f)
            times.append(time.perf_counter() - t0)
            rays.append(rr.rays)
            refr.append(rr.reference_rays)
            if time.perf_counter() - t_start > budget_s:
                break
        sample = f"median of {len(times)} full {W}x{H} frames after 1 warm-up frame"
        band = {"rows": H, "y0": 0, "frames_timed": len(times), "full_frame_equivalents_timed": len(times)}
        mr = float(np.median([r / t for r, t in zip(rays, times)])) / 1e6
    dt = float(np.median(times))
    out = {"value": round(1.0 / dt, 5), "unit": "frames/s", "cores": n_threads, "kind": "port",
           "sample": f"{sample}; oracle/restir_oracle.c (OpenMP, {n_threads} threads; ray queries walk an 8-wide "
                     f"tree with AVX2 box tests{'' if osc.wide else ' -- NOT available on this host: binary walk'}, "
                     f"shading scalar)",
           "traversal": "8-wide AVX2" if osc.wide else "binary scalar",
           "s_per_frame": round(dt, 4), "band": band, "host": host_cpu(),
           "timing_scope": "all passes of produceRestir (pg/simpleguidx11.cpp:361-486 totalFrameDuration), no post-frame"}
    if mr is not None:
        out["mrays_per_s"] = round(mr, 2)
    # rays the reference's code would trace for these frames (oracle-counted: every rtcIntersect1 and
    # testOcclusion it reaches, incl. zero-contribution shadow rays and re-evaluated final p-hats)
    out["reference_rays_per_frame"] = int(np.median(refr)) if refr else None
    return out


# ---------------------------------------------------------------- PMC figures committed under profiles/
def pmc_for(name, W, H):
    """The newest committed PMC summary of this config (profiles/r06_pmc_<cfg>.json, else rounds 5 / 4 / 3 / 2)."""
    for rnd in ("r06", "r05", "r04", "r03_v3", "r03", "r02"):
        path = os.path.join(ROOT, "profiles", f"{rnd}_pmc_{name}.json")
        if not os.path.exists(path):
            continue
        try:
            with open(path) as f:
                pmc = json.load(f)
        except (OSError, ValueError):
            continue
        if pmc.get("config") == f"{name}_{W}x{H}":
            pmc["_path"] = f"profiles/{rnd}_pmc_{name}.json"
            return pmc
    return None


def limiter_for(pmc, kernel):
    """What bounds `kernel` by its committed PMC passes (scripts/pmc_summary.py vmem_derived): the busiest
    of the texture-address (TA) and texture-data (TD) units and the VALU issue rate, each a fraction of
    the kernel's active cycles, with the HBM fraction beside them (these walks are far from HBM-bound)."""
    k = ((pmc or {}).get("kernels", {}) or {}).get(kernel) or {}
    v = k.get("vmem_derived")
    if not v:
        return None
    unit = {"ta_busy_frac": "TA (vector-memory address processing)",
            "td_busy_frac": "TD (vector-memory data return)",
            "valu_issue_frac": "VALU issue"}
    fr = {u: float(v[u]) for u in unit if v.get(u) is not None}
    top = max(fr, key=fr.get)
    return {"kernel": kernel, "bound_by": unit[top], **{u: round(x, 4) for u, x in fr.items()},
            "wait_any_over_wave_cycles": v.get("wait_any_over_wave_cycles"),
            "cache_lines_per_vmem_load": v.get("cache_accesses_per_vmem_rd"), "source": pmc.get("_path")}


# ---------------------------------------------------------------- one single-GPU config
def run_single(name, W, H, steps, warmup, device, stream, cpu_threads, with_cpu, kernel_frames=5):
    from restir_amd import Renderer
    sc, prm, camera, light_pos = workload(name)
    r = Renderer(W, H, device=device, stream=stream)
    gs = r.load_scene(sc)
    cam = camera or (lambda f: sc.camera)

    def step(f):
        if light_pos is not None:       # moving lights: new positions -> light CDF + BVH refit (timed)
            gs.update_positions(light_pos(f))
        r.produce_restir(gs, cam(f), prm, f, copy_out=False, timed=False)

    import torch
    # initialisation (like the scene load, outside warm-up and timing): RS_TRAVERSAL_AUTO times the two
    # BVH walk kinds over a scene's first 6 frames, then the history is reset
    for f in range(TUNE_FRAMES):
        step(f)
    r.reset_history()
    for f in range(warmup):
        step(f)
    torch.cuda.synchronize()
    r.timing_totals(reset=True)
    t0 = time.perf_counter()
    for f in range(steps):
        step(warmup + f)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    tot, n_timed = r.timing_totals(reset=True)
    ms_per_step = dt / steps * 1e3
    rays = int(tot.rays)
    # kernel window: one frame in flight (run-ahead 0), HIP events around every pass on the frame's stream
    r.set_run_ahead(0)
    for f in range(2):
        step(warmup + steps + f)
    r.timing_totals(reset=True)
    for f in range(kernel_frames):
        step(warmup + steps + 2 + f)
    ktot, kn = r.timing_totals(reset=True)
    r.set_run_ahead(2)
    iso = {k: float(getattr(ktot, k)) / max(1, kn) for k in PASS_BYTES}
    iso_total = float(ktot.total_ms) / max(1, kn)
    dom = max(iso, key=iso.get)
    px = W * H
    b_px = survey_bytes_per_px(prm)
    frame_gbs = b_px * px / (ms_per_step * 1e-3) / 1e9
    k_gbs = PASS_BYTES[dom] * px / (iso[dom] * 1e-3) / 1e9
    _, last_kind, _ = r.traversal(gs)
    pmc = pmc_for(name, W, H)
    out = {
        "value": round(steps / dt, 4), "unit": "frames/s", "ms_per_step": round(ms_per_step, 4), "steps": steps,
        "warmup": warmup, "frames_timed_by_events": n_timed,
        "config": {"workload": f"{name}: {WORKLOADS[name]}, {W}x{H}", "width": W, "height": H,
                   "traversal": {0: "lockstep", 1: "lane"}.get(last_kind, str(last_kind)), "frames_in_flight": 3,
                   "scene_build_ms": round(float(gs.build_ms), 2), "wide_tree": gs.wide_tree_nodes()},
        "mrays_per_s": round(rays / dt / 1e6, 2), "rays_per_frame": rays // max(1, steps),
        "pass_ms_one_frame_in_flight": {k: round(v, 4) for k, v in iso.items()},
        "frame_ms_one_frame_in_flight": round(iso_total, 4),
        "roofline": {"bound": "hbm", "scope": "frame (all passes, frames in flight)", "bytes_per_px": b_px,
                     "achieved": round(frame_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(frame_gbs / HBM_PEAK_GBS, 5),
                     "traffic": pmc.get("frame_bytes") if pmc else None},
        "kernel_roofline": {"bound": "hbm", "kernel": PASS_KERNEL[dom], "bytes_per_px": PASS_BYTES[dom],
                            "kernel_ms": round(iso[dom], 4), "achieved": round(k_gbs, 2), "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": round(k_gbs / HBM_PEAK_GBS, 5),
                            "kernel_ms_le_ms_per_step": bool(iso[dom] <= ms_per_step),
                            "traffic": (pmc.get("kernels", {}).get(PASS_KERNEL[dom], {}) or {}).get("hbm_bytes_corrected")
                            if pmc else None,
                            "timing": f"HIP events on the frame's stream, {kn} frames with one frame in flight"},
    }
    out["limiter"] = limiter_for(pmc, PASS_KERNEL[dom])
    if pmc and pmc.get("frame_valu"):
        v = float(pmc["frame_valu"])
        out["valu_issue"] = {"scope": "frame", "valu_per_frame": v, "achieved": round(v / (ms_per_step * 1e-3) / 1e9, 2),
                             "peak": VALU_PEAK_GIPS, "unit": "G wave-instr/s",
                             "frac": round(v / (ms_per_step * 1e-3) / 1e9 / VALU_PEAK_GIPS, 4),
                             "source": pmc.get("_path")}
    out["cpu_baseline"] = cpu_baseline(name, W, H, cpu_threads) if with_cpu else None
    rr = (out["cpu_baseline"] or {}).get("reference_rays_per_frame")
    if rr:
        # comparable with the reference's Mrays/s: the rays ITS code would trace for the same frames
        # (oracle-counted on the CPU-baseline sample; this build skips zero-contribution shadow rays and
        # re-evaluated final p-hats, so it traces fewer -- rays_per_frame above)
        out["reference_rays_per_frame"] = rr
        out["reference_equivalent_mrays_per_s"] = round(rr * steps / dt / 1e6, 2)
    if out["cpu_baseline"] and out["cpu_baseline"].get("value"):
        out["gpu_over_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
    gs.close()
    r.close()
    return out


# ---------------------------------------------------------------- denoiser
DN_LEVELS = [0, 0, 1, 2, 3, 4, 4, 3, 3, 2, 2, 1, 1, 0, 0, 0]     # pooling level of each convolution


def run_denoise(W, H, steps, warmup, device, stream, cpu_threads, with_cpu):
    """The reference's per-frame OIDN "RT" filter (pg/simpleguidx11.cpp:52-75, :255-256) on the C2 frame's
    accumulator with the frame's G-buffer albedo / normal (rs_denoise_frame): one step = one execute at
    W x H.  OIDN's trained weights are not shipped, so the weights are He-initialised ones of OIDN's UNet
    shape (the cost does not depend on their values)."""
    import torch
    from restir_amd import Renderer, tza
    from restir_amd.denoise import Denoiser, gflop_per_frame
    sc, prm, camera, _ = workload("C2")
    r = Renderer(W, H, device=device, stream=stream)
    gs = r.load_scene(sc)
    w = tza.random_unet_weights(seed=1)
    d = Denoiser(r, w)
    for f in range(2):
        r.produce_restir(gs, sc.camera, prm, f, copy_out=False, timed=False)
    r.post_frame(accumulate=False, stats=False)
    for _ in range(warmup):
        d.denoise_frame()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        d.denoise_frame()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    d.set_timing(True)
    lay, tot = [], []
    for _ in range(5):
        d.denoise_frame()
        lay.append(d.layer_ms())
        tot.append(d.last_ms())
    d.set_timing(False)
    lay = np.median(np.array(lay), axis=0)
    ms_ev = float(np.median(tot))
    info = d.info()
    gf = gflop_per_frame(info, W, H)
    hp, wp = -(-H // 16) * 16, -(-W // 16) * 16
    shapes = tza.unet_shapes(info.input_channels)
    names = list(shapes)
    lay_gf = [2.0 * shapes[n][0] * shapes[n][1] * 9 * (hp * wp) / 4 ** lv / 1e9 for n, lv in zip(names, DN_LEVELS)]
    dom = int(np.argmax(lay[1:]))
    dom_tf = lay_gf[dom] / float(lay[1 + dom])
    out = {
        "value": round(steps / dt, 3), "unit": "executes/s", "ms_per_step": round(dt / steps * 1e3, 4), "steps": steps,
        "warmup": warmup, "dtype": "f16 storage / f32 accumulation (MFMA 16x16x32 f16)",
        "data": "synthetic: the C2 frame's accumulator + G-buffer albedo / normal; He-initialised weights of OIDN's UNet shape",
        "config": {"workload": f"OIDN RT filter (hdr, auto-exposure) on a {W}x{H} frame", "width": W, "height": H,
                   "parameters": int(info.parameters), "gflop_per_execute": round(gf, 2)},
        "execute_ms_hip_events": round(ms_ev, 4),
        "layer_ms": {"input_transform": round(float(lay[0]), 4),
                     **{n: round(float(x), 4) for n, x in zip(names, lay[1:])}},
        "roofline": {"bound": "mfma", "scope": "one execute (auto-exposure, input transform, 16 convolutions)",
                     "achieved": round(gf / ms_ev, 1), "peak": MFMA_F16_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(gf / ms_ev / MFMA_F16_PEAK_TFLOPS, 4), "traffic": None},
        "kernel_roofline": {"bound": "mfma", "kernel": f"k_conv3 {names[dom]}", "kernel_ms": round(float(lay[1 + dom]), 4),
                            "gflop": round(lay_gf[dom], 2), "achieved": round(dom_tf, 1), "peak": MFMA_F16_PEAK_TFLOPS,
                            "unit": "TFLOP/s", "frac": round(dom_tf / MFMA_F16_PEAK_TFLOPS, 4),
                            "timing": "HIP events on the context's stream around each convolution, median of 5 executes"},
    }
    if with_cpu:
        frame = np.zeros((H, W, 3), np.float32)
        r.produce_restir(gs, sc.camera, prm, 3, copy_out=True, timed=False)
        frame[:] = r.frame_data
        g = r.gbuffer()
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import denoise_ref
        n_threads = baseline_threads(cpu_threads)
        denoise_ref.denoise(frame[:64, :64], g[:64, :64, 6:9], g[:64, :64, 3:6], w, threads=n_threads)   # warm-up
        ts = []
        t_start = time.perf_counter()
        for _ in range(3):
            t0 = time.perf_counter()
            denoise_ref.denoise(frame, g[..., 6:9], g[..., 3:6], w, threads=n_threads)
            ts.append(time.perf_counter() - t0)
            if time.perf_counter() - t_start > 20.0:
                break
        cs = float(np.median(ts))
        out["cpu_baseline"] = {"value": round(1.0 / cs, 4), "unit": "executes/s", "cores": n_threads, "kind": "port",
                               "sample": f"median of {len(ts)} full {W}x{H} executes of oracle/denoise_ref.py (PyTorch CPU "
                                         f"fp32 convolutions, {n_threads} threads; OIDN's own CPU path is not in the reference)",
                               "s_per_execute": round(cs, 3), "host": host_cpu()}
        out["gpu_over_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
    else:
        out["cpu_baseline"] = None
    d.close()
    gs.close()
    r.close()
    return out


def run_dropin(W, H, frames=120):
    """The drop-in path a reference user runs: C++ host code over include/restir.hpp (member names of
    SimpleGuiDX11) driving librestir_amd.so, the framebuffer landing in host memory every frame
    (tools/restir_render --bench: produceRestir + frame_data on the host)."""
    import tempfile
    from restir_amd import scenes
    exe = os.path.join(ROOT, "restir-embree_amd", "restir_render")
    if not os.path.exists(exe):
        return None
    sc = scenes.cornell_many_lights(1024)
    c = sc.camera
    with tempfile.TemporaryDirectory() as d:
        obj = os.path.join(d, "c2.obj")
        scenes.write_obj(sc, obj)          # Raytracer::LoadScene(file) path: OBJ/MTL through the C ABI loader
        cmd = [exe, "--bench", "--obj", obj, "--w", str(W), "--h", str(H), "--frames", str(frames),
               "--area", "32", "--brdf", "1", "--spatial", "4", "--eye", *map(str, c.eye), "--at", *map(str, c.at),
               "--fov", str(c.fov_y)]
        try:
            p = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        except (OSError, subprocess.TimeoutExpired) as e:
            return {"error": repr(e)}
    for line in p.stdout.splitlines()[::-1]:
        if line.startswith("{"):
            try:
                return json.loads(line)
            except ValueError:
                break
    return {"error": (p.stderr or p.stdout)[-400:], "rc": p.returncode}


def _compact_roofline(r, keep=("bound", "kernel", "kernel_ms", "bytes_per_px", "gflop", "achieved", "peak", "unit",
                                  "frac", "traffic")):
    return None if r is None else {k: r[k] for k in keep if k in r}


def compact(e):
    """The fields of a sub-config that the printed line keeps (workload text, samples, peaks and units of the
    rooflines -- the head line's -- and the rest go to the full record), so the driver's stored tail keeps every
    config's value."""
    out = {k: e[k] for k in ("value", "unit", "ms_per_step", "mrays_per_s", "gpu_over_cpu", "frac_of_zero_copy",
                              "error") if k in e}
    for k in ("roofline", "kernel_roofline"):
        if e.get(k):
            out[k] = _compact_roofline(e[k], ("bound", "kernel", "kernel_ms", "achieved", "frac", "traffic"))
    cb = e.get("cpu_baseline")
    if cb:
        out["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind") if k in cb}
    elif "cpu_baseline" in e:
        out["cpu_baseline"] = None
    if e.get("per_rank"):
        out["per_rank"] = [{k: v for k, v in q.items() if k in ("rank", "band_rows", "band_ms", "halo_ms", "gather_ms")}
                           for q in e["per_rank"]]
    return out


def write_full(path, rec):
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump(rec, f, indent=1)
    except OSError as ex:
        print(f"warning: cannot write {path}: {ex}", file=sys.stderr)


# ---------------------------------------------------------------- rank launcher (--gpus N without torchrun)
def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(base: dict, rank: int, world: int, port: int) -> dict:
    """The environment of rank `rank` of a `world`-rank job on this node (what torchrun would set)."""
    env = dict(base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                "MASTER_PORT": str(port)})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def check_world(gpus: int, env: dict):
    """None when this process should run as a rank (WORLD_SIZE set and equal to --gpus, or --gpus 1 alone);
    "launch" when it must start --gpus ranks itself; an error message on a --gpus / WORLD_SIZE mismatch."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return "launch" if gpus > 1 else None
    if int(ws) != gpus:
        return f"--gpus {gpus} but WORLD_SIZE={ws}: the launcher and the flag disagree"
    return None


def launch_ranks(argv, world: int, env=None, cmd=None, poll_s: float = 0.2) -> int:
    """Starts `world` child processes of this script (fresh interpreters: nothing here has touched the GPU),
    one per rank with torchrun's environment, and waits.  Rank 0's stdout (the JSON line) passes through;
    the first child to fail ends the others (their exact PIDs) and its exit code is returned."""
    base = dict(os.environ if env is None else env)
    port = free_port()
    cmd = cmd or [sys.executable, os.path.abspath(__file__)]
    procs = []
    for r in range(world):
        procs.append(subprocess.Popen(cmd + list(argv), env=rank_env(base, r, world, port),
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc, kill_at = 0, None
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the other ranks",
                          file=sys.stderr)
                    for q in live:
                        q.terminate()
                    kill_at = time.monotonic() + 30.0
            if live and kill_at is not None and time.monotonic() > kill_at:
                for q in live:
                    q.kill()
            if live:
                time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def main():
    args = parse()
    verdict = check_world(args.gpus, os.environ)
    if verdict == "launch":
        # --gpus N > 1 without a launcher: start N ranks here, before this process touches the GPU
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    if verdict is not None:
        print(f"bench.py: {verdict}", file=sys.stderr)
        sys.exit(2)
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    W, H = args.width, args.height
    # RESTIR_FORCE_MULTI=1 runs the N>1 code path with one rank (a rehearsal of the multi-GPU flow on a
    # one-GPU box: RCCL refuses two ranks on one device)
    if world == 1 and not os.environ.get("RESTIR_FORCE_MULTI"):
        torch.cuda.set_device(local)
        # render on a dedicated torch stream shared with the library (torch's default stream is handle 0)
        torch.cuda.set_stream(torch.cuda.Stream(device=local))
        stream = torch.cuda.current_stream().cuda_stream
        head = run_single(args.scene, W, H, args.steps, args.warmup, local, stream, args.cpu_threads,
                          not args.no_cpu_baseline)
        out = {"metric": METRIC, "value": head.pop("value"), "unit": "frames/s", "n_gpus": 1,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": head.pop("ms_per_step"),
               "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
               "data": f"synthetic (procedural scene, BASELINE.json configs[{CONFIG_INDEX[args.scene]}])"}
        head["config"]["parallelism"] = "1 GPU"
        out.update(head)
        full = dict(out)
        if not args.no_extras and args.scene == "C2" and (W, H) == (1920, 1080):
            extras = {}
            for name, steps, res in (("C3", 20, (W, H)), ("C5", C5_FRAMES, (W, H)), ("C2V", args.steps, (W, H)),
                                     ("C4_1gpu", 10, RES["C4"])):
                base = "C3" if name == "C4_1gpu" else name
                e = run_single(base, res[0], res[1], steps, args.warmup, local, stream, args.cpu_threads,
                               not args.no_cpu_baseline and name != "C4_1gpu")
                e["data"] = f"synthetic (procedural scene, BASELINE.json configs[{CONFIG_INDEX['C4' if name == 'C4_1gpu' else name]}])"
                if name == "C4_1gpu":
                    e["note"] = ("C4's scene and parameters on ONE GPU (the denominator of the N-GPU C4 speed-up); "
                                 "CPU baseline: C3's (same per-pixel work at 1080p)")
                extras[name] = e
            extras["denoise"] = run_denoise(W, H, args.steps, args.warmup, local, stream, args.cpu_threads,
                                            not args.no_cpu_baseline)
            torch.cuda.synchronize()
            d = run_dropin(W, H)
            if d is not None:
                if "value" in d:
                    d["frac_of_zero_copy"] = round(d["value"] / out["value"], 4)
                extras["dropin_host_framebuffer"] = d
            full["configs"] = extras
            out["configs"] = {k: compact(v) for k, v in extras.items()}
        full["host"] = host_cpu()
        write_full(args.full_out, full)
        for k in ("pass_ms_one_frame_in_flight", "frame_ms_one_frame_in_flight", "frames_timed_by_events",
                  "reference_rays_per_frame", "rays_per_frame"):
            out.pop(k, None)
        for k in ("roofline", "kernel_roofline"):
            out[k] = _compact_roofline(out.get(k))
        if out.get("cpu_baseline"):
            out["cpu_baseline"] = {k: out["cpu_baseline"][k] for k in ("value", "unit", "cores", "kind", "sample")}
        if out.get("limiter"):
            out["limiter"] = {k: out["limiter"][k] for k in ("kernel", "bound_by", "source") if k in out["limiter"]}
        if out.get("valu_issue"):
            out["valu_issue"] = {k: out["valu_issue"][k] for k in ("achieved", "peak", "unit", "frac") if k in out["valu_issue"]}
        out["full_record"] = os.path.relpath(args.full_out, ROOT)
        print(json.dumps(out), flush=True)
        return
    run_multi(args, world, rank, local, W, H)


def run_multi(args, world, rank, local, W, H):
    """N>1: the native multi-GPU path behind the C ABI (rs_mgpu_*: RCCL point-to-point halo exchange and
    gather on each frame's stream, csrc/rs_mgpu.hip) with torch.distributed over gloo as the control
    plane only (the RCCL id broadcast, barriers, max-over-ranks timing).  The headline config (--scene) and
    then every --multi-configs entry (C4 by default) are measured in turn, one renderer at a time.
    RESTIR_MGPU=python (or the RESTIR_DIST_BACKEND=gloo rehearsal with ranks sharing a GPU) runs the Python
    orchestration (restir_amd/distributed.py) instead."""
    if os.environ.get("RESTIR_MGPU", "cabi") == "python" or os.environ.get("RESTIR_DIST_BACKEND") == "gloo":
        return run_multi_python(args, world, rank, local, W, H)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo")
    torch.cuda.set_device(local)
    names = [args.scene] + [c for c in args.multi_configs.split(",") if c and c != args.scene]
    lines = {}
    for name in names:
        w, h = RES.get(name, (W, H))
        lines[name] = run_multi_config(args, name, world, rank, local, w, h)
    if rank == 0:
        head = lines[args.scene]
        full = dict(head)
        if len(names) > 1:
            full["configs"] = {n: lines[n] for n in names[1:]}
            head["configs"] = {n: compact(lines[n]) for n in names[1:]}
        full["host"] = host_cpu()
        write_full(args.full_out, full)
        head["per_rank"] = compact(head)["per_rank"]
        head["full_record"] = os.path.relpath(args.full_out, ROOT)
        print(json.dumps(head), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def run_multi_config(args, name, world, rank, local, W, H):
    import torch
    import torch.distributed as dist
    from restir_amd import Renderer
    from restir_amd.mgpu import MultiGpuFrame
    sc, prm, camera, light_pos = workload(name)
    cam = camera or (lambda f: sc.camera)
    r = Renderer(W, H, device=local)
    gs = r.load_scene(sc)
    uid = [MultiGpuFrame.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    m = MultiGpuFrame(r, rank=rank, world=world, unique_id=uid[0])

    def step(f):
        if light_pos is not None:
            gs.update_positions(light_pos(f))
        m.render([gs], cam(f), prm, f, gather=True)

    for f in range(TUNE_FRAMES):
        step(f)
    bands = m.rebalance([gs], cam(0), prm, 0, 2, 8)
    if rank == 0:
        print(f"{name} bands: {bands}", file=sys.stderr)
    for f in range(args.warmup):
        step(f)
    r.synchronize()
    torch.cuda.synchronize()
    dist.barrier()
    r.timing_totals(reset=True)
    m.stats(reset=True)
    t0 = time.perf_counter()
    for f in range(args.steps):
        step(args.warmup + f)
    r.synchronize()
    torch.cuda.synchronize()
    dist.barrier()
    dt = time.perf_counter() - t0
    tot, n_timed = r.timing_totals()
    xs = m.stats()
    red = torch.tensor([dt, float(tot.rays), float(tot.reproj_outside)], dtype=torch.float64)
    dmax = red[:1].clone()
    dist.all_reduce(dmax, op=dist.ReduceOp.MAX)
    sums = red[1:].clone()
    dist.all_reduce(sums, op=dist.ReduceOp.SUM)
    dt, rays, outside = float(dmax[0]), int(sums[0]), int(sums[1])
    # per rank: band kernel time per frame (pass events), halo bytes and exchange / gather time per frame
    nf = max(1, xs["frames"])
    mine = [float(tot.total_ms) / max(1, n_timed), xs["halo_bytes_sent"] / nf, xs["halo_bytes_recv"] / nf,
            xs["halo_ms"] / nf, xs["gather_ms"] / nf, xs["gather_bytes"] / nf]
    per_rank = [None] * world
    dist.all_gather_object(per_rank, mine)
    _, last_kind, _ = r.traversal(gs)
    line = None
    if rank == 0:
        line = multi_line(args, name, world, W, H, prm, dt, rays, outside, bands, last_kind,
                          "rs_mgpu (C ABI): RCCL point-to-point halo + gather")
        line["per_rank"] = [{"rank": q, "band_rows": bands[q][1] - bands[q][0], "band_ms": round(v[0], 4),
                             "halo_bytes_sent": int(v[1]), "halo_bytes_recv": int(v[2]), "halo_ms": round(v[3], 4),
                             "gather_ms": round(v[4], 4), "gather_bytes_recv": int(v[5])}
                            for q, v in enumerate(per_rank)]
        line["per_rank_note"] = ("per frame; band_ms = the rank's pass kernels (HIP events, frames overlap); halo_ms / "
                                 "gather_ms = HIP-event span of the RCCL group on the frame's stream incl. waiting for peers")
    dist.barrier()
    m.close()
    gs.close()
    r.close()
    return line


def multi_line(args, name, world, W, H, prm, dt, rays, outside, bands, last_kind, path):
    ms = dt / args.steps * 1e3
    b_px = survey_bytes_per_px(prm)
    gbs = b_px * W * H / (ms * 1e-3) / 1e9
    return {"metric": METRIC, "value": round(args.steps / dt, 4), "unit": "frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": f"synthetic (procedural scene, BASELINE.json configs[{CONFIG_INDEX[name]}])",
            "config": {"workload": f"{name}: {WORKLOADS[name]}, {W}x{H}", "width": W, "height": H,
                       "parallelism": f"row-bands x{world}", "bands": bands, "multi_gpu_path": path,
                       "traversal": {0: "lockstep", 1: "lane"}.get(last_kind, str(last_kind)) + " (rank 0)",
                       "frames_in_flight": 3},
            "mrays_per_s": round(rays / dt / 1e6, 2), "rays_per_frame": rays // max(1, args.steps),
            "reproj_rebuilt_per_frame": outside / max(1, args.steps),
            "roofline": {"bound": "hbm", "scope": "frame (all passes, all ranks)", "bytes_per_px": b_px,
                         "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
                         "frac": round(gbs / (HBM_PEAK_GBS * world), 5), "traffic": None},
            "cpu_baseline": None}


def run_multi_python(args, world, rank, local, W, H):
    import torch
    import torch.distributed as dist
    # RESTIR_DIST_BACKEND=gloo rehearses the N>1 flow with more ranks than GPUs (ranks share devices,
    # halo/gather staged through host memory); the measured configuration is RCCL ("nccl"), one GPU per rank
    backend = os.environ.get("RESTIR_DIST_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    red_dev = "cpu" if backend == "gloo" else "cuda"
    if backend == "gloo":
        dist.init_process_group("gloo")
    else:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    sc, prm, camera, light_pos = workload(args.scene)
    cam = camera or (lambda f: sc.camera)
    torch.cuda.set_stream(torch.cuda.Stream(device=local))
    stream = torch.cuda.current_stream().cuda_stream
    from restir_amd.distributed import TiledRenderer
    # async gather: frame f's band framebuffers travel to rank 0 while frame f+1 renders
    tr = TiledRenderer(W, H, rank, world, device=local, stream=stream, async_gather=True)
    gs = tr.load_scene(sc)

    def step(f):
        if light_pos is not None:
            gs.update_positions(light_pos(f))
        return tr.render(gs, cam(f), prm, f, gather=True, timed=False)

    for f in range(TUNE_FRAMES):
        step(f)
    bands = tr.rebalance(step, n_frames=2)
    if rank == 0:
        print(f"bands: {bands}", file=sys.stderr)
    tr.reset_history()
    for f in range(args.warmup):
        step(f)
    dist.barrier()
    torch.cuda.synchronize()
    tr.timing_totals(reset=True)
    dist.barrier()
    t0 = time.perf_counter()
    for f in range(args.steps):
        step(args.warmup + f)
    torch.cuda.synchronize()
    dist.barrier()
    dt = time.perf_counter() - t0
    tot, _ = tr.timing_totals()
    tt = torch.tensor([dt, float(tot.rays), float(tot.reproj_outside)], dtype=torch.float64, device=red_dev)
    dmax = tt[:1].clone()
    dist.all_reduce(dmax, op=dist.ReduceOp.MAX)
    sums = tt[1:].clone()
    dist.all_reduce(sums, op=dist.ReduceOp.SUM)
    dt, rays, outside = float(dmax[0]), int(sums[0]), int(sums[1])
    _, last_kind, _ = tr.be.r.traversal(gs)
    if rank == 0:
        print(json.dumps(multi_line(args, args.scene, world, W, H, prm, dt, rays, outside, bands, last_kind,
                                    "restir_amd.distributed (Python): torch.distributed halo + gather")), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
