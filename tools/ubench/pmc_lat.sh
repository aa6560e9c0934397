# latency / occupancy / unit-busy counters for every kernel of one benchmark step
# usage (GPU box, repo root): bash tools/ubench/pmc_lat.sh OUTDIR [bench.py args]
OUT=${1:-gpurun_out/pmc_lat}
shift || true
ARGS="$@"
mkdir -p $OUT && export TMPDIR=/tmp
i=0
for p in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LEVEL_WAVES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM" \
         "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" \
         "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum" \
         "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $p -d $OUT/p$i -o pmc --output-format csv -- python3 bench.py $ARGS --steps 1 --warmup 0 --no-cpu-baseline --traffic off > $OUT/p$i.log 2>&1 || exit 1
done
