import os, sys, ctypes
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "restir-embree_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
from restir_amd import Renderer, params as P, scenes
from restir_amd.distributed import _CudaBuf
st = torch.cuda.current_stream().cuda_stream
r = Renderer(32, 32, stream=st)
s = r.load_scene(scenes.cornell_box(8))
prm = P.default_params(do_spatial=1)
r.tile_begin(s, s.__class__ and scenes.CORNELL_CAMERA, prm, 0, 8, 24, 5, 5)
ptr, n = r.tile_halo_ptr(2)
print("ptr", hex(ptr), "bytes", n)
t = torch.as_tensor(_CudaBuf(ptr, n), device="cuda")
print("tensor", t.device, t.dtype, t.shape, hex(t.data_ptr()), "same ptr:", t.data_ptr() == ptr)
torch.cuda.synchronize()
print("first bytes", t[:16].cpu().numpy())
t2 = torch.as_tensor(_CudaBuf(ptr, n, "<f4", 4), device="cuda")
print("as float", t2[:12].cpu().numpy())
print("hip last error after:", r.lib.rs_last_error(r.h))
