#!/bin/bash
source tools/gpu_run.sh
step rules_rt15 600 python -u -m pytest tests/test_gpu_rules.py tests/test_gpu_rules_limits.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
grep -q " passed" gpurun_out/rules_rt15.log && ! grep -q "failed" gpurun_out/rules_rt15.log || { echo "rules parity failed"; exit 1; }
for r in 1 2 3; do
  for v in head rt15; do
    step c3r_${v}_$r 180 python tools/prof_rollout.py --config c3r --envs 65536 --chunk 2000 --launches 5 --time --lib abx/lib_$v.so
  done
done
