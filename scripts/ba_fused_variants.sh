#!/bin/bash
# Builds fused LocalBA workgroup-size variants (threads per k_ba_iter workgroup) as
# lib/libvxslam_ft<T>.so for a bench sweep via VX_LIB (host-side build; run the bench on the box).
set -e
cd "$(dirname "$0")/../visionx-slam_amd"
ROCM=${ROCM:-/opt/rocm}
SRC="csrc/vx_ctx.cpp csrc/orb.hip csrc/match.hip csrc/ba.hip csrc/ba_window.hip csrc/sba.hip csrc/landmarks.hip csrc/ransac.hip csrc/essential.hip csrc/dmap.hip"
for T in "$@"; do
    D=build/var_ft$T; mkdir -p $D lib
    for f in $SRC; do
        $ROCM/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../include -Icsrc \
            -DVX_BA_FUSED_THREADS=$T -x hip -c $f -o $D/$(basename $f).o &
    done
    wait
    $ROCM/bin/hipcc --offload-arch=gfx950 $D/*.o -shared -L$ROCM/lib -lrccl -Wl,-rpath,$ROCM/lib -o lib/libvxslam_ft$T.so
done
