#!/bin/bash
# Build libffcv_hip.so from a git revision's sources into build/ab/<name>.so:
#   tools/build_rev.sh <name> <rev> [extra defines]
set -e
NAME=$1; REV=$2; shift 2
TMP=$(mktemp -d)
git archive $REV ffcv_amd/csrc include | tar -x -C $TMP
mkdir -p build/ab
(cd $TMP/ffcv_amd/csrc && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=off -fno-fast-math \
  -Wno-unused-function -I$TMP/include "$@" -o $OLDPWD/build/ab/$NAME.so ffcv_common.hip ffcv_rrc.hip ffcv_jpeg.hip ffcv_host.hip ffcv_cpu_jpeg.hip)
rm -rf $TMP
