#!/bin/bash
source tools/gpu_run.sh
step c3quick 120 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 3 --time
step parity_valusel 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_iocodes.py tests/test_gpu_bigpool.py -k "not c4" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
grep -q " passed" gpurun_out/parity_valusel.log && ! grep -q "failed" gpurun_out/parity_valusel.log || { echo "parity failed"; exit 1; }
for r in 1 2 3; do
  for v in head valusel; do
    step c3_${v}_$r 120 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 20 --time --lib abx/lib_$v.so
  done
done
for r in 1 2; do
  for v in head valusel; do
    step c2_${v}_$r 120 python tools/prof_rollout.py --config c2 --envs 4096 --chunk 2000 --launches 20 --time --lib abx/lib_$v.so
  done
done
