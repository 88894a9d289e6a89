set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r4a_tests.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -u tools/persist_timing.py 50 20 2>&1 | grep -v amdgpu.ids | tee gpurun_out/persist_timing.log
M3D_PERSIST_PROF=1 timeout -k 10 120 python -u tools/persist_timing.py 50 2 > gpurun_out/persist_prof.log 2>&1 || exit $?
grep "m3d persist" gpurun_out/persist_prof.log | head -4
timeout -k 10 120 python -u tools/cold_timing.py --reps 7 2>&1 | grep -v amdgpu.ids
M3D_CREATE_PROF=1 timeout -k 10 120 python -u tools/cold_timing.py --reps 3 2>&1 | grep "m3d create" | tail -2
