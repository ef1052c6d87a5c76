"""GPU tests of the multi-GPU path behind the C ABI (rs_mgpu_*, csrc/rs_mgpu.hip): the C++ orchestration
renders row-band sharded frames that are bit-identical to a single context's frames.

On the one-GPU test box the ranks are contexts of one process (rs_mgpu_create_local: halo exchange and
gather as device copies -- RCCL refuses two ranks on one device); RCCL mode is exercised with world 1
(communicator setup, the frame path without peers).  The N-GPU RCCL runs are bench.py's."""
import numpy as np
import pytest

from restir_amd import params as P
from restir_amd import scenes
from restir_amd.mgpu import MultiGpuFrame
from restir_amd.renderer import Renderer

pytestmark = pytest.mark.gpu


def _full_frames(sc, W, H, prm, cams, light_pos=None):
    g = Renderer(W, H)
    gs = g.load_scene(sc)
    out = []
    for f, c in enumerate(cams):
        if light_pos is not None:
            gs.update_positions(light_pos(f))
        out.append(g.produce_restir(gs, c, prm, f).copy())
    return out


@pytest.mark.parametrize("world,which", [(2, "c2"), (4, "c3"), (3, "c5")])
def test_local_mgpu_bit_identical(world, which):
    W, H = 96, 64
    light_pos = None
    if which == "c2":
        sc, prm = scenes.cornell_many_lights(256), P.metric_params(m_area=8)
    elif which == "c3":
        sc, prm = scenes.sponza_like(target_tris=30_000, n_lamps=128), P.c3_params(m_area=6, spatial_passes=2)
    else:
        sc, prm = scenes.cornell_many_lights(256), P.c3_params(m_area=6)
        light_pos = lambda f: scenes.moving_light_positions(sc, f, 48)
    cams = [scenes.orbit_camera(sc.camera, f, 48, 0.3) for f in range(5)]
    ref = _full_frames(sc, W, H, prm, cams, light_pos)
    rs = [Renderer(W, H) for _ in range(world)]
    for r in rs:
        r.set_traversal("lockstep")               # frames on the run-ahead lanes (no AUTO tuning frames)
    ss = [r.load_scene(sc) for r in rs]
    m = MultiGpuFrame(rs)
    assert m.bands()[0][0] == 0 and m.bands()[-1][1] == H
    for f, c in enumerate(cams):
        if light_pos is not None:
            for s in ss:
                s.update_positions(light_pos(f))
        img = m.render(ss, c, prm, f, copy_out=True)
        assert np.array_equal(img, ref[f]), f"{which} world {world} frame {f}: {int(np.any(img != ref[f], -1).sum())} px"
    m.close()


def test_local_mgpu_rebalance_and_frames_in_flight():
    """rs_mgpu_rebalance (row costs all-reduced, balanced split, history reset) gives unequal bands; frames
    then rendered back to back without host sync (gather into rank 0's lane framebuffers, cloned on the
    stream) equal the single-context frames."""
    import torch
    from restir_amd.distributed import _CudaBuf
    W, H, world = 96, 96, 3
    sc, prm = scenes.cornell_many_lights(256), P.c3_params(m_area=6)
    # skewed row costs: the camera looks above the box, so the top ~40 % of the rows miss every triangle (no
    # candidates, no shadow rays) and the box fills the bottom rows
    base = scenes.Camera(eye=(0.0, -5.5, 1.0), at=(0.0, 0.0, 2.3), fov_y=40.0)
    cams = [scenes.orbit_camera(base, f, 48, 0.3) for f in range(6)]
    torch.cuda.set_stream(torch.cuda.Stream())
    st = torch.cuda.current_stream().cuda_stream
    rs = [Renderer(W, H, stream=st) for _ in range(world)]
    for r in rs:
        r.set_traversal("lockstep")
    ss = [r.load_scene(sc) for r in rs]
    m = MultiGpuFrame(rs)
    equal = m.bands()
    assert equal == [(0, 32), (32, 64), (64, 96)], equal
    bands0 = m.rebalance(ss, cams[0], prm, 0, 2, 6, refine=0)     # row costs only: nothing measured
    assert m.rebalance_times() == []
    # the cheap sky rows go to rank 0: the split moves off the equal one
    assert bands0 != equal and bands0[0][1] - bands0[0][0] > 32, bands0
    bands = m.rebalance(ss, cams[0], prm, 0, 2, 6)                 # refine=None: the default 2 rounds, not the 0 above
    assert bands[0][0] == 0 and bands[-1][1] == H and all(bands[i][1] == bands[i + 1][0] for i in range(world - 1)), bands
    assert all(b - a >= 6 for a, b in bands), bands
    assert bands != equal and bands[0][1] - bands[0][0] > 32, bands
    rounds = m.rebalance_times()                                   # every rank timed in every measured round
    assert 1 <= len(rounds) <= 3 and all(len(t) == world and min(t) > 0 for t in rounds), rounds
    clones = []
    for f, c in enumerate(cams):
        m.render(ss, c, prm, f)
        clones.append(torch.as_tensor(_CudaBuf(m.frame_device_ptr(), W * H * 12, "<f4", 4), device="cuda").clone())
    ref = _full_frames(sc, W, H, prm, cams)
    for f in range(len(cams)):
        assert np.array_equal(clones[f].cpu().numpy().reshape(H, W, 3), ref[f]), f
    m.close()


def test_rccl_world1_and_allreduce():
    """RCCL mode with one rank: unique id, communicators (one per lane), frames, all-reduce of host values."""
    W, H = 64, 48
    sc, prm = scenes.cornell_many_lights(128), P.metric_params(m_area=4)
    r = Renderer(W, H)
    s = r.load_scene(sc)
    m = MultiGpuFrame(r, rank=0, world=1, unique_id=MultiGpuFrame.unique_id())
    img = m.render([s], sc.camera, prm, 0, copy_out=True, timed=True)
    ref = _full_frames(sc, W, H, prm, [sc.camera])[0]
    assert np.array_equal(img, ref) and m.last_times.rays > 0
    assert np.allclose(m.allreduce([1.5, 2.0], "max"), [1.5, 2.0])
    m.close()


def test_local_mgpu_transfer_stats():
    """rs_mgpu_get_stats: the halo and gather bytes of the transfer plans (rs_mgpu_core.h) per frame, and
    event-timed exchange spans."""
    W, H, world, frames = 96, 64, 3, 4
    sc, prm = scenes.cornell_many_lights(128), P.metric_params(m_area=4)
    rs = [Renderer(W, H) for _ in range(world)]
    for r in rs:
        r.set_traversal("lockstep")
    ss = [r.load_scene(sc) for r in rs]
    m = MultiGpuFrame(rs)
    for f in range(frames):
        m.render(ss, sc.camera, prm, f)
    st = m.stats(reset=True)
    h = 5                                          # floor(sqrt(30))
    b = m.bands()
    assert st["frames"] == frames
    assert st["halo_bytes_sent"] == st["halo_bytes_recv"] == frames * 2 * (world - 1) * h * W * 48
    assert st["gather_bytes"] == frames * (H - b[0][1]) * W * 12
    assert st["halo_ms"] > 0 and st["gather_ms"] > 0
    assert m.stats()["frames"] == 0
    m.close()


@pytest.mark.parametrize("pipelined", [True, False])
def test_local_mgpu_moving_geometry_rebuilds_previous_geometry(pipelined):
    """Tiles whose temporal reprojection falls beyond their rows rebuild the previous frame's G element --
    against the PREVIOUS frame's geometry when the scene moved in between (rs_scene::dev_of: the a_* copy
    of the pipelined update, or the copy an in-place update makes first).  The whole scene moves every
    frame and the camera steps far with margin = halo, so rebuilds happen and every rebuilt element sees
    moved geometry; frames must equal the single context's bit for bit.  pipelined=False: run-ahead 0
    and updates with normals (the in-place path)."""
    W, H, world = 96, 64, 4
    sc = scenes.cornell_box(8)
    prm = P.c3_params(m_area=6)
    cams = [scenes.orbit_camera(sc.camera, 3 * f, 48, 0.6) for f in range(5)]
    base = np.asarray(sc.positions, np.float32)
    def pos(f):
        p = base.reshape(-1, 3, 3).copy()
        p[..., 2] += np.float32(0.02 * f)
        p[..., 0] += np.float32(0.01 * f)
        return p.reshape(-1, 9)
    nrm = None if pipelined else sc.normals

    def setup(r):
        if not pipelined:
            r.set_run_ahead(0)
        r.set_traversal("lockstep")
        return r
    g = setup(Renderer(W, H))
    gs = g.load_scene(sc)
    ref = []
    for f, c in enumerate(cams):
        gs.update_positions(pos(f), nrm)
        ref.append(g.produce_restir(gs, c, prm, f).copy())
    rs = [setup(Renderer(W, H)) for _ in range(world)]
    ss = [r.load_scene(sc) for r in rs]
    m = MultiGpuFrame(rs)
    for r in rs:
        r.timing_totals(reset=True)
    for f, c in enumerate(cams):
        for s in ss:
            s.update_positions(pos(f), nrm)
        img = m.render(ss, c, prm, f, copy_out=True)
        assert np.array_equal(img, ref[f]), f"frame {f}: {int(np.any(img != ref[f], -1).sum())} px differ"
    outside = sum(int(r.timing_totals()[0].reproj_outside) for r in rs)
    assert outside > 0
    m.close()


@pytest.mark.parametrize("traversal", ["lane", "lockstep"])
def test_local_mgpu_update_then_rebuild(traversal):
    """A tile frame after rs_scene_update_positions + rs_scene_rebuild: the rebuild brings the
    8-wide tree back while the previous frame's geometry generation is still the updated one, so a tile's
    temporal rebuild of a previous-frame G element traces a generation without (or with) its own wide tree;
    the launch must not fail and the bands must equal the single context's frames bit for bit, over a
    sequence of updates, rebuilds and plain frames."""
    W, H, world = 96, 64, 3
    sc = scenes.cornell_box(8)
    prm = P.c3_params(m_area=6)
    cams = [scenes.orbit_camera(sc.camera, 3 * f, 48, 0.6) for f in range(6)]
    base = np.asarray(sc.positions, np.float32)

    def pos(f):
        p = base.reshape(-1, 3, 3).copy()
        p[..., 2] += np.float32(0.02 * f)
        return p.reshape(-1, 9)
    ops = ["", "update+rebuild", "update", "rebuild", "update+rebuild", ""]

    def apply(s, f):
        if "update" in ops[f]:
            s.update_positions(pos(f))
        if "rebuild" in ops[f]:
            s.rebuild()
    g = Renderer(W, H)
    g.set_traversal(traversal)
    gs = g.load_scene(sc)
    ref = []
    for f, c in enumerate(cams):
        apply(gs, f)
        ref.append(g.produce_restir(gs, c, prm, f).copy())
    rs = [Renderer(W, H) for _ in range(world)]
    for r in rs:
        r.set_traversal(traversal)
    ss = [r.load_scene(sc) for r in rs]
    m = MultiGpuFrame(rs)
    for f, c in enumerate(cams):
        for s in ss:
            apply(s, f)
        img = m.render(ss, c, prm, f, copy_out=True)
        assert np.array_equal(img, ref[f]), f"frame {f} ({ops[f]}): {int(np.any(img != ref[f], -1).sum())} px differ"
    m.close()


@pytest.mark.parametrize("world,temporal", [(2, 0), (4, 1)])
def test_rccl_branch_threads_on_one_gpu(tmp_path, world, temporal):
    """the RCCL branch of rs_mgpu (rs_mgpu_create + ncclCommSplit per lane, NcclLink halo exchanges
    and gathers issued with frames in flight, rs_mgpu_rebalance's ncclAllReduce) with world 2 and 4 as threads of
    one process on this one GPU, linked against a stand-in librccl (tests/cpp/rccl_stub.cpp: sends and receives
    paired per communicator / sender / receiver in issue order and turned into device copies; every pair's byte
    counts equal, nothing left unpaired).  Every gathered frame (before and after a rebalance) is bit-identical
    to one context's frame."""
    import json
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "_build", "mgpu_rccl_driver")
    assert os.path.exists(exe), "build it first: make -C tests/cpp (run by __graft_entry__.build())"
    sc = scenes.cornell_many_lights(256)
    obj = tmp_path / "c2.obj"
    scenes.write_obj(sc, str(obj))
    c = sc.camera
    cmd = [exe, str(obj), "96", "64", str(world), "4", *map(str, c.eye), *map(str, c.at), str(c.fov_y), str(temporal)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and line, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    r = json.loads(line[-1])
    print(f"[rccl-stub] {r}")
    assert r["bad_frames"] == 0 and r["mismatches"] == 0 and r["unpaired"] == 0 and r["pairs"] > 0 and r["allreduces"] >= 1
    # the rebalance's time-based refinement ran through the RCCL branch: >= 1 measured round, each an all-reduce
    assert r["refine_rounds"] >= 1 and r["allreduces"] >= 1 + r["refine_rounds"], r
