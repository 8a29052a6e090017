#!/bin/bash
# Build an A/B variant of libffcv_hip.so with extra defines into build/ab/.
#   tools/build_variant.sh <name> -DJW=2 ...   (then bench.py --lib build/ab/<name>.so)
set -e
NAME=$1; shift
mkdir -p build/ab
cd ffcv_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=off -fno-fast-math \
  -Wno-unused-function "$@" -o ../../build/ab/$NAME.so ffcv_common.hip ffcv_rrc.hip ffcv_jpeg.hip ffcv_host.hip ffcv_cpu_jpeg.hip
