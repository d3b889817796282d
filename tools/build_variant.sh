#!/bin/bash
# calibration build of libpcmkm.so with extra defines: tools/build_variant.sh NAME -DFLAG ...
# -> tools/ab/lib_NAME.so (tools/ab/ travels to the GPU box; load it with PCM_SO=tools/ab/lib_NAME.so)
set -e
name=$1; shift
cd "$(dirname "$0")/.."
mkdir -p tools/ab
P=3d-point-cloud-multiday-imagery_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -I include "$@" \
  -o tools/ab/lib_$name.so $P/csrc/pcm_engine.hip $P/csrc/pcm_dense.hip $P/csrc/pcm_stereo.hip $P/csrc/pcm_shard.hip \
  $P/csrc/pcm_xchg.hip
