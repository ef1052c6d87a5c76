#!/bin/bash
# build_variant.sh NAME "EXTRA HIPCC FLAGS": librestir_amd built with the Makefile's flags plus extra -D flags
# into _variants/NAME.so (A/B runs load it through RESTIR_LIB)
set -e
cd "$(dirname "$0")/../restir-embree_amd"
mkdir -p _variants/$1
# the Makefile's HIPFLAGS (later -D flags override earlier ones)
BASE=$(sed -n '/^HIPFLAGS ?=/,/^[^ ]/p' Makefile | sed 's/^HIPFLAGS ?=//; s/\\$//' | tr '\n' ' ' | sed 's/CSRC.*//; s/$(ARCH)/gfx950/')
F="$BASE $2"
/opt/rocm/bin/hipcc $F -c csrc/restir_capi.hip -o _variants/$1/capi.o
/opt/rocm/bin/hipcc $F -c csrc/rs_bvh_build.hip -o _variants/$1/bvh.o
/opt/rocm/bin/hipcc $F -c csrc/rs_mgpu.hip -o _variants/$1/mgpu.o
/opt/rocm/bin/hipcc $F -c csrc/rs_denoise.hip -o _variants/$1/denoise.o
/opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -c csrc/rs_obj_loader.cpp -o _variants/$1/obj.o
/opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -ffp-contract=off -c csrc/rs_image.cpp -o _variants/$1/image.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o _variants/$1.so _variants/$1/*.o -lz -lrccl
