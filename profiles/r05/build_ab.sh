#!/bin/bash
# Build an A/B variant of libkmerhip.so with extra compile definitions, outside the tree's
# default library: build_ab/<name>/libkmerhip.so (travels to the GPU box; bench/tests load it
# with KMH_LIB_PATH).  usage: bash profiles/r05/build_ab.sh <name> "-DFOO=1 -DBAR=2"
name=$1; defs=$2
make -s lib OUTDIR=build_ab/$name OBJDIR=build_ab/$name/obj \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $defs" -j8
