"""GPU test of the C++ host mirror (include/restir.hpp) through its headless driver
(restir-embree_amd/tools/restir_render.cpp, the reference's tutorial_3 -> Producer loop without UI):
it renders frames with temporal + spatial reuse and writes the last frame as a PFM."""
import os
import subprocess

import numpy as np
import pytest

from restir_amd.renderer import decode_image

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "restir-embree_amd", "restir_render")


def test_cpp_driver_renders(tmp_path):
    assert os.path.exists(TOOL), "build restir-embree_amd (make) first"
    out = tmp_path / "frame.pfm"
    p = subprocess.run([TOOL, "--w", "64", "--h", "48", "--frames", "3", "--area", "4", "--spatial", "4",
                        "--temporal", "--out", str(out)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    img = decode_image(out)
    assert img.shape == (48, 64, 3) and np.isfinite(img).all()
    assert img.max() > 0.0                         # the light and lit walls
