"""Diagnostic (GPU box): host cost of each tile-ABI call of a frame, on a tiny image so the GPU never
back-pressures the host.  Prints the mean microseconds per call of rs_tile_begin / _temporal / _spatial
/ _finish and of the whole frame.  Usage: python scripts/host_overhead.py [--steps N] [--scene C2|C3]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "restir-embree_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--scene", default="C2")
    ap.add_argument("--width", type=int, default=128)
    ap.add_argument("--height", type=int, default=64)
    ap.add_argument("--light", action="store_true", help="1 area candidate: the GPU work per frame is tiny")
    ap.add_argument("--mgpu", type=int, default=0, help="time rs_mgpu_render_frame over this many local ranks instead")
    a = ap.parse_args()
    import torch
    from restir_amd import Renderer, scenes
    from restir_amd.params import metric_params, c3_params
    sc = scenes.sponza_like() if a.scene == "C3" else scenes.cornell_many_lights(1024)
    prm = metric_params() if a.scene == "C2" else c3_params()
    if a.light:
        prm = metric_params(m_area=1)
    st = torch.cuda.Stream()
    r = Renderer(a.width, a.height, device=0, stream=st.cuda_stream)
    gs = r.load_scene(sc)
    H = a.height
    if a.mgpu:
        from restir_amd.mgpu import MultiGpuFrame
        rs_ = [r] + [Renderer(a.width, a.height, device=0, stream=torch.cuda.Stream().cuda_stream) for _ in range(a.mgpu - 1)]
        gss = [gs] + [x.load_scene(sc) for x in rs_[1:]]
        m = MultiGpuFrame(rs_)
        for f in range(a.steps + 10):
            if f == 10:
                torch.cuda.synchronize()
                t_all = time.perf_counter()
            m.render(gss, sc.camera, prm, f, gather=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t_all
        print(f"{a.scene} {a.width}x{a.height} rs_mgpu_render_frame over {a.mgpu} local rank(s): "
              f"{dt / a.steps * 1e6:.1f} us per frame, {dt / a.steps / a.mgpu * 1e6:.1f} us per rank-frame", flush=True)
        m.close()
        return
    acc = {"begin": 0.0, "temporal": 0.0, "spatial": 0.0, "finish": 0.0}
    for f in range(a.steps + 10):
        if f == 10:
            torch.cuda.synchronize()
            acc = {k: 0.0 for k in acc}
            t_all = time.perf_counter()
        t0 = time.perf_counter()
        r.tile_begin(gs, sc.camera, prm, f, 0, H, 0, 0)
        t1 = time.perf_counter()
        r.tile_temporal()
        t2 = time.perf_counter()
        for p in range(prm.spatial_passes if prm.do_spatial else 0):
            r.tile_spatial(p)
        t3 = time.perf_counter()
        r.tile_finish(False)
        t4 = time.perf_counter()
        acc["begin"] += t1 - t0; acc["temporal"] += t2 - t1; acc["spatial"] += t3 - t2; acc["finish"] += t4 - t3
    torch.cuda.synchronize()
    dt = time.perf_counter() - t_all
    print(f"{a.scene} {a.width}x{a.height}: frame {dt / a.steps * 1e6:.1f} us wall; per call (us): " +
          " ".join(f"{k}={v / a.steps * 1e6:.1f}" for k, v in acc.items()), flush=True)


if __name__ == "__main__":
    main()
