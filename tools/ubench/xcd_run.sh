mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python tools/kbench.py --rounds 3 --variants xcd=0 xcd=1 xcd=8 xcd=24 xcd=30 xcd=32 xcd=48 xcd=100 xcd=250 > gpurun_out/kb_xcd3.log 2>&1 || exit 1
for x in 0 1 30; do
  timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T -d gpurun_out/pmc_hit_x$x -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --option xcd=$x > gpurun_out/pmc_hit_x$x.log 2>&1 || exit 1
done
