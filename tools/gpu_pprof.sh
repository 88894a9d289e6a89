set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for rb in 22 24 28 44; do
echo "RB=$rb"; M3D_PERSIST_RB=$rb timeout -k 10 120 python -u tools/persist_timing.py 50 10 2>&1 | grep persistent
done
M3D_PERSIST_RB=24 M3D_PERSIST_PROF=1 timeout -k 10 120 python -u tools/persist_timing.py 50 2 > gpurun_out/persist_prof_24.log 2>&1 || exit $?
grep "m3d persist" gpurun_out/persist_prof_24.log | head -4 | cut -c1-400
