# Round 6: the tightened fp32 error bound E (icp.hip refresh_rt32_from, M3D_TIGHT_E) against round
# 5's: ambiguous queries at cfg1's 20th evaluation (tail-clock builds) and grid_timing, alternated.
# Needs tools/ab/{tclk_new,tclk_old,e_old}.so (tools/ab_build.sh).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
for v in new old; do
  AB_LIB=tools/ab/tclk_$v.so timeout -k 10 120 python3 tools/tail_clock.py grid > gpurun_out/tclk_$v.log 2>&1 || exit $?
done
for rep in 1 2; do
  timeout -k 10 200 python3 tools/grid_timing.py 50 > gpurun_out/gt_new_$rep.log 2>&1 || exit $?
  AB_LIB=tools/ab/e_old.so timeout -k 10 200 python3 tools/grid_timing.py 50 > gpurun_out/gt_old_$rep.log 2>&1 || exit $?
done
grep -h -v amdgpu gpurun_out/tclk_*.log gpurun_out/gt_*.log
