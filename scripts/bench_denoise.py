"""bench.py's denoise sub-line alone (run_denoise at 1080p, CPU baseline included)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402

torch.cuda.set_device(0)
torch.cuda.set_stream(torch.cuda.Stream(device=0))
print(json.dumps(bench.run_denoise(1920, 1080, 20, 3, 0, torch.cuda.current_stream().cuda_stream, None,
                                   "--no-cpu" not in sys.argv)), flush=True)
