#!/bin/bash
source tools/gpu_run.sh
step bigpool 600 python -u -m pytest tests/test_gpu_bigpool.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
grep -q " passed" gpurun_out/bigpool.log && ! grep -q "failed" gpurun_out/bigpool.log || { echo "bigpool parity failed"; exit 1; }
for r in 1 2; do
  for v in head fbitop fbitop_u2 fu2 prio_audit; do
    step c3r_${v}_$r 180 python tools/prof_rollout.py --config c3r --envs 65536 --chunk 2000 --launches 5 --time --lib abx/lib_$v.so
  done
done
for P in 4096 16384; do
  step bench_c3_p$P 300 python bench.py --puzzles $P --steps 20 --warmup 3
done
