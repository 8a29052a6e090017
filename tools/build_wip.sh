#!/bin/bash
# Build an A/B variant from a work-in-progress ffcv_jpeg.hip (the other
# sources from ffcv_amd/csrc) into build/ab/<name>.so:
#   tools/build_wip.sh <name> <path/to/ffcv_jpeg.hip> [-DX=...]
set -e
NAME=$1; SRC=$(readlink -f $2); shift 2
TMP=$(mktemp -d)
mkdir -p $TMP/include $TMP/a/b
cp include/ffcv_hip.h $TMP/include/
cp ffcv_amd/csrc/* $TMP/a/b/
cp $SRC $TMP/a/b/ffcv_jpeg.hip
mkdir -p build/ab
(cd $TMP/a/b && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=off -fno-fast-math \
  -Wno-unused-function -I$OLDPWD/include "$@" -o $OLDPWD/build/ab/$NAME.so ffcv_common.hip ffcv_rrc.hip ffcv_jpeg.hip ffcv_host.hip ffcv_cpu_jpeg.hip)
rm -rf $TMP
