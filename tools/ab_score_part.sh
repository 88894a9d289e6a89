# brute NN: grid.y (target slices) sweep at cfg1, TH=4 (M3D_NN_GY) — default first
set -e
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for gy in 0 4 5 6 7 8 9 10 12 13; do
    echo "gy=$gy" >> gpurun_out/ab_gy.log
    M3D_NN_GY=$gy timeout -k 10 120 python tools/nn_timing.py 20 >> gpurun_out/ab_gy.log 2>&1
  done
done
echo done
