"""Writes tests/golden/jpeg_reference_hashes.json: for every JPEG under /root/reference/template (the
reference's textures, decoded there by FreeImage, pg/Texture.cpp:18-30), the shape and SHA-256 of the pixel
array PIL's libjpeg-turbo decodes (default settings: islow IDCT, fancy upsampling).  The reference files are
read as data, never executed; only the hashes are committed (tests/test_image_io.py compares rs_image_decode
with them when /root/reference is present).  Run: python tests/golden/gen_jpeg_hashes.py"""
import glob
import hashlib
import json
import os

import numpy as np
from PIL import Image

ROOT = "/root/reference/template"
out = {}
for path in sorted(glob.glob(os.path.join(ROOT, "**", "*.jp*g"), recursive=True)):
    with Image.open(path) as im:
        a = np.asarray(im)
        out[os.path.relpath(path, ROOT)] = {"shape": list(a.shape), "mode": im.mode,
                                            "progressive": bool(im.info.get("progressive", 0)),
                                            "sha256": hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()}
dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "jpeg_reference_hashes.json")
with open(dst, "w") as f:
    json.dump({"decoder": f"PIL {Image.__version__} (libjpeg-turbo, default decompression settings)", "files": out}, f,
              indent=1, sort_keys=True)
print(f"{len(out)} files -> {dst}")
