#!/bin/bash
# drop-in host-framebuffer throughput (tools/restir_render --bench, C2 1080p): DMA (default) vs copy-kernel readback
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
python3 -c "
import sys; sys.path.insert(0, '$R/restir-embree_amd')
from restir_amd import scenes; scenes.write_obj(scenes.cornell_many_lights(1024), '/tmp/c2.obj')" || exit 1
T=$R/restir-embree_amd/restir_render
A="--bench --obj /tmp/c2.obj --w 1920 --h 1080 --frames 120 --area 32 --brdf 1 --spatial 4 --eye 0 -3.9 1 --at 0 0 1 --fov 40"
timeout -k 10 120 $T $A && RESTIR_READBACK=kernel timeout -k 10 120 $T $A
