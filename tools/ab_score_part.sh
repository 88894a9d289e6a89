# NN kernel: GPU tests at the new default (TH=4), then A/B over M3D_NN_TH / M3D_NN_DEFER, bench
set -e
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/ab_tests.log 2>&1
for rep in 1 2; do
  for cfg in "4 1" "4 0" "2 1"; do
    set -- $cfg
    echo "th=$1 defer=$2" >> gpurun_out/ab_nn.log
    M3D_NN_TH=$1 M3D_NN_DEFER=$2 timeout -k 10 120 python tools/nn_timing.py 20 >> gpurun_out/ab_nn.log 2>&1
  done
done
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1
echo done
