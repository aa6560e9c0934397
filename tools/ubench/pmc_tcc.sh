# L2 request mix of every kernel of one benchmark step (memory-side read request sizes)
# usage (GPU box, repo root): bash tools/ubench/pmc_tcc.sh OUTDIR
OUT=${1:-gpurun_out/pmc_tcc}
mkdir -p $OUT && export TMPDIR=/tmp
i=0
for p in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_REQ_sum TCC_READ_sum" \
         "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $p -d $OUT/p$i -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/p$i.log 2>&1 || exit 1
done
