"""bench.py's rank launcher (`--gpus N` without torchrun): the child environment, the
exit-code propagation and the --gpus / WORLD_SIZE mismatch error.  CPU only: the children here are a tiny
stand-in script, not bench.py, so nothing touches a GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

CHILD = r"""
import json, os, sys
keys = ["RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"]
rec = {k: os.environ.get(k) for k in keys}
rec["argv"] = sys.argv[1:]
with open(os.path.join(os.environ["OUT_DIR"], "rank%s.json" % os.environ["RANK"]), "w") as f:
    json.dump(rec, f)
if os.environ["RANK"] == "0":
    print(json.dumps({"metric": "x", "n_gpus": int(os.environ["WORLD_SIZE"])}), flush=True)
fail = os.environ.get("FAIL_RANK")
if fail is not None and fail == os.environ["RANK"]:
    sys.exit(7)
if fail is not None:               # the healthy ranks would wait for the failed one forever (a collective)
    import time
    time.sleep(120)
"""


def _run(tmp_path, world, fail_rank=None):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OUT_DIR"] = str(tmp_path)
    if fail_rank is not None:
        env["FAIL_RANK"] = str(fail_rank)
    return bench.launch_ranks(["--gpus", str(world), "--steps", "3"], world, env=env,
                              cmd=[sys.executable, str(script)], poll_s=0.05)


def test_children_get_torchrun_env(tmp_path):
    assert _run(tmp_path, 3) == 0
    recs = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(3)]
    ports = {r["MASTER_PORT"] for r in recs}
    assert len(ports) == 1 and int(ports.pop()) > 0
    for r, rec in enumerate(recs):
        assert rec["RANK"] == rec["LOCAL_RANK"] == str(r)
        assert rec["WORLD_SIZE"] == rec["LOCAL_WORLD_SIZE"] == "3"
        assert rec["MASTER_ADDR"] == "127.0.0.1"
        assert rec["argv"] == ["--gpus", "3", "--steps", "3"]


def test_failing_rank_propagates_and_stops_the_others(tmp_path):
    import time
    t0 = time.monotonic()
    rc = _run(tmp_path, 3, fail_rank=1)
    assert rc == 7
    assert time.monotonic() - t0 < 60          # the sleeping ranks were terminated, not waited for


def test_world_checks():
    assert bench.check_world(1, {}) is None
    assert bench.check_world(4, {}) == "launch"
    assert bench.check_world(4, {"WORLD_SIZE": "4"}) is None
    assert bench.check_world(1, {"WORLD_SIZE": "1"}) is None
    msg = bench.check_world(8, {"WORLD_SIZE": "4"})
    assert msg and "WORLD_SIZE=4" in msg


def test_mismatch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2, p.stderr
    assert "WORLD_SIZE=2" in p.stderr and p.stdout == ""


@pytest.mark.parametrize("gpus", [2])
def test_rank_env_keeps_ipc_mode(gpus):
    e = bench.rank_env({}, 1, gpus, 12345)
    assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["RANK"] == "1" and e["MASTER_PORT"] == "12345"
