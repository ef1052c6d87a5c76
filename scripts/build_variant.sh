#!/bin/bash
# A/B builds of librestir_amd.so with changed compile-time switches (analysis tooling):
#   scripts/build_variant.sh NAME "-DRS_X=1 -DRS_Y=2"   -> restir-embree_amd/_ab/lib_NAME.so
# (REBUILD="rs_denoise ..." names the objects recompiled with the flags; default restir_capi rs_mgpu)
# A -DNAME=v given here replaces the Makefile's own -DNAME=...; run with RESTIR_LIB=restir-embree_amd/_ab/lib_NAME.so.
set -e
cd "$(dirname "$0")/../restir-embree_amd"
name=$1; shift
flags=$(python3 - "$*" <<'PY'
import re, sys
mk = open("Makefile").read()
f = re.search(r"HIPFLAGS \?=(.*?)\n(?!\s)", mk, re.S).group(1).replace("\\\n", " ").replace("$(ARCH)", "gfx950").split()
extra = sys.argv[1].split()
names = {e.split("=")[0] for e in extra}
print(" ".join([x for x in f if x.split("=")[0] not in names] + extra))
PY
)
mkdir -p _ab "_build_$name"
cp -p _build/*.o "_build_$name/"
for o in ${REBUILD:-restir_capi rs_mgpu}; do rm -f "_build_$name/$o.o"; done
make -s OBJ="_build_$name" LIB="_ab/lib_$name.so" HIPFLAGS="$flags" "_ab/lib_$name.so"
echo "built _ab/lib_$name.so: $flags"
