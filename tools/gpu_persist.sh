set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_icp.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "persistent or empty or graph or grid_identical" > gpurun_out/persist_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/persist_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/persist_timing.py 50 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/persist_timing.log
M3D_PERSIST_PROF=1 timeout -k 10 120 python -u tools/persist_timing.py 50 2 > gpurun_out/persist_prof.log 2>&1 || exit $?
grep "m3d persist" gpurun_out/persist_prof.log | head -4
