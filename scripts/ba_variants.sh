#!/bin/bash
# Builds LocalBA pose-stage variants (threads per k_pose_kf workgroup, max slices per keyframe) as
# lib/libvxslam_pb<B>_s<S>.so for a bench sweep via VX_LIB.  Host-side (no GPU): run here, then
# `VX_LIB=visionx-slam_amd/lib/libvxslam_pb256_s8.so python bench.py --no-cpu-baseline` on the box.
set -e
cd "$(dirname "$0")/../visionx-slam_amd"
ROCM=${ROCM:-/opt/rocm}
SRC="csrc/vx_ctx.cpp csrc/orb.hip csrc/match.hip csrc/ba.hip csrc/ba_window.hip csrc/sba.hip csrc/landmarks.hip csrc/ransac.hip csrc/essential.hip csrc/dmap.hip"
for v in "$@"; do
    B=${v%,*}; S=${v#*,}
    D=build/var_${B}_${S}; mkdir -p $D lib
    for f in $SRC; do
        $ROCM/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../include -Icsrc \
            -DVX_BA_POSE_BLOCK=$B -DVX_BA_MAX_SPLIT=$S -x hip -c $f -o $D/$(basename $f).o &
    done
    wait
    $ROCM/bin/hipcc --offload-arch=gfx950 $D/*.o -shared -L$ROCM/lib -lrccl -Wl,-rpath,$ROCM/lib -o lib/libvxslam_pb${B}_s${S}.so
done
