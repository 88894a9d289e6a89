#!/bin/bash
# Scoring: sub-tile loop unroll 1 / 2 / 4 (libraries in 3d-matching_amd/m3d/ab/), then a grid.y
# sweep (M3D_SCORE_GY) with the default build — score_ab at H = Nc = 1e5 (time + counts crc).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=3d-matching_amd/m3d
cp $L/libm3d.so $L/ab/libm3d_cur.so
for rep in 1 2; do
  for v in u2 u1 u4; do
    cp $L/ab/libm3d_$v.so $L/libm3d.so
    AB_TAG=$v NC=100000 H=100000 timeout -k 10 120 python tools/score_ab.py || exit 1
  done
done
cp $L/ab/libm3d_cur.so $L/libm3d.so
for rep in 1 2; do
  for gy in 0 7 9 11 12 14 16 20 26; do
    M3D_SCORE_GY=$gy AB_TAG=gy$gy NC=100000 H=100000 timeout -k 10 120 python tools/score_ab.py || exit 1
  done
done
