#!/bin/bash
# dyn_tend C: vertices per vertex wave (MPAS_C_VE builds in abl/): parity of the default
# build, then step A/B at x1.2562 and x1.163842
set -e
OUT=${1:-gpurun_out/r03cv}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_decomp.py tests/test_gpu_mpas_dynamics.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
for r in 1 2; do
  for so in mpas-regent_amd/mpasdyn/libmpasdyn.so abl/libmpasdyn_cve1.so abl/libmpasdyn_cve2.so abl/libmpasdyn_cve8.so; do
    n=$(basename $so .so)
    timeout -k 10 120 env MPAS_LIB=$so python3 tools/abstep.py --ncells 2562 --rounds 4 --steps 20 --variants xcd=64 > "$OUT/s_${n}_$r.json"
    timeout -k 10 200 env MPAS_LIB=$so python3 tools/abstep.py --ncells 163842 --rounds 2 --steps 5 --variants xcd=64 > "$OUT/b_${n}_$r.json"
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$OUT/bench_prof.log 2>&1
