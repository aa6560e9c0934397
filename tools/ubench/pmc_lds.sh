# LDS / VALU / occupancy counters for every kernel of one benchmark step (one counter group per pass)
# usage (GPU box, repo root): bash tools/ubench/pmc_lds.sh OUTDIR [bench.py args]
OUT=${1:-gpurun_out/pmc_lds}
shift || true
ARGS="$@"
mkdir -p $OUT && export TMPDIR=/tmp
i=0
for p in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_SALU SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_ANY" \
         "TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
         "FETCH_SIZE" "WRITE_SIZE" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $p -d $OUT/p$i -o pmc --output-format csv -- python3 bench.py $ARGS --steps 1 --warmup 0 --no-cpu-baseline --traffic off > $OUT/p$i.log 2>&1 || exit 1
done
