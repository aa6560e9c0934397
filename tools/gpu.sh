#!/bin/bash
# One parameterised GPU-box script for the round's runs (replaces the per-run
# tools/gpu_r0*.sh one-offs).  Run from the repo root on the GPU box, e.g.
#   gpurun -- 'bash tools/gpu.sh OUT suite bench trace'
# usage: bash tools/gpu.sh OUT RECIPE [RECIPE ...]
# Every GPU step has its own time limit and the steps are chained under set -e: the first
# failure (test failure, fault, abort, timeout) ends the script.  Environment knobs:
#   TESTS="tests/test_x.py ..."   the files / node ids of the "tests" recipe
#   BENCH_ARGS="--transport ..."  extra bench.py arguments (bench, trace, pmc)
#   AB="opt=1 opt=0"              the variants of the "abstep" / "kbench" recipes
#   RS_ARGS="--ncells 655362 ..." extra tools/rank_sim.py arguments
#   PMC_DIMS="163842 491520 327680 56"  also the per-task summary of the pmc passes (pmc_summary.py)
#   LIBS="abl/old.so ..."          the other library builds of the "libab" recipe (MPAS_LIB)
# Recipes:
#   tests   the listed GPU tests, verbose          suite   the whole GPU suite + smoke()
#   bench   one bench.py JSON line                 trace   rocprofv3 kernel trace + stats of bench.py
#   pmc     FETCH / WRITE / TCC hit-miss passes (one counter group per run) + per-kernel table
#   abstep  tools/abstep.py whole-step A/B (AB)    kbench  tools/kbench.py per-task A/B (AB)
#   ranksim tools/rank_sim.py, overlap 0/1 (RS_ARGS)
#   libab   whole-step kbench.py of the in-tree build and of each of LIBS, interleaved, twice
set -e
OUT=${1:?usage: gpu.sh OUT RECIPE...}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
PYT="python3 -u -m pytest -x --timeout 300 --timeout-method thread -m gpu"
BA=${BENCH_ARGS:-}
for R in "$@"; do
  echo "== $R $(date +%T)"
  case $R in
    tests)
      timeout -k 10 900 $PYT -v ${TESTS:?TESTS not set} > "$OUT/tests.log" 2>&1 ;;
    suite)
      timeout -k 10 1000 $PYT -q tests > "$OUT/gpu_tests.log" 2>&1
      timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    bench)
      timeout -k 10 500 python3 bench.py $BA > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    trace)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o kt --output-format csv -- \
        python3 bench.py $BA --no-cpu-baseline --traffic off > "$OUT/trace.log" 2>&1 ;;
    pmc)
      B="bench.py $BA --steps 1 --warmup 0 --no-cpu-baseline --traffic off"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/ptrace" -o kt --output-format csv -- python3 $B > "$OUT/ptrace.log" 2>&1
      for P in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
        n=$(echo $P | cut -d' ' -f1)
        timeout -s KILL 300 rocprofv3 --pmc $P -d "$OUT/pmc_$n" -o pmc --output-format csv -- python3 $B > "$OUT/pmc_$n.log" 2>&1
      done
      python3 tools/pmc_kernels.py "$OUT"/pmc_* --match "k_" > "$OUT/kernels.txt"
      if [ -n "${PMC_DIMS:-}" ]; then
        python3 tools/pmc_summary.py $([[ "$BA" == *--physics* || "$BA" == *--transport* ]] && echo --physics) \
          --trace "$OUT/ptrace" --fetch "$OUT/pmc_FETCH_SIZE" --write "$OUT/pmc_WRITE_SIZE" \
          --dims $PMC_DIMS --out "$OUT/pmc_summary.json" > "$OUT/pmc_summary.txt"
      fi ;;
    abstep)
      timeout -k 10 600 python3 tools/abstep.py ${ABSTEP_ARGS:-} --variants ${AB:?AB not set} > "$OUT/abstep.json" ;;
    kbench)
      timeout -k 10 600 python3 tools/kbench.py ${KBENCH_ARGS:-} --rounds 3 --variants ${AB:?AB not set} > "$OUT/kbench.json" ;;
    ranksim)
      for o in 0 1; do
        timeout -k 10 400 python3 tools/rank_sim.py ${RS_ARGS:-} --overlap $o > "$OUT/rank_sim_ov$o.json"
      done ;;
    libab)
      for r in 1 2; do
        timeout -k 10 300 python3 tools/kbench.py ${KBENCH_ARGS:-} --rounds 3 --variants xcd=64 > "$OUT/libab_new_$r.json"
        for so in ${LIBS:?LIBS not set}; do
          MPAS_LIB=$so timeout -k 10 300 python3 tools/kbench.py ${KBENCH_ARGS:-} --rounds 3 --variants xcd=64 \
            > "$OUT/libab_$(basename "$so" .so)_$r.json"
        done
      done ;;
    *)
      echo "unknown recipe $R" >&2; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
