set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for L in 1 2; do
M3D_PERSIST_PROF=1 M3D_PERSIST_LANES=$L timeout -k 10 120 python -u tools/persist_timing.py 50 3 > gpurun_out/persist_prof_L$L.log 2>&1 || exit $?
grep -v "m3d persist" gpurun_out/persist_prof_L$L.log; grep "m3d persist" gpurun_out/persist_prof_L$L.log | tail -2
done
M3D_CREATE_PROF=1 timeout -k 10 120 python -u tools/cold_timing.py --reps 5 > gpurun_out/cold_prof.log 2>&1 || exit $?
grep -v "m3d create" gpurun_out/cold_prof.log; grep "m3d create" gpurun_out/cold_prof.log | tail -4
