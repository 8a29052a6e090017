#!/bin/bash
# Build libffcv_hip.so of a git revision into build/ab/<name>.so (A/B baseline).
#   tools/build_rev.sh <name> <rev> [extra hipcc flags]
set -e
NAME=$1; REV=$2; shift 2
T=$(mktemp -d)
git archive $REV ffcv_amd/csrc include | tar -x -C $T
mkdir -p build/ab
OUT=$(pwd)/build/ab/$NAME.so
cd $T/ffcv_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=off -fno-fast-math \
  -Wno-unused-function "$@" -o $OUT ffcv_common.hip ffcv_rrc.hip ffcv_jpeg.hip ffcv_host.hip ffcv_cpu_jpeg.hip
rm -rf $T
