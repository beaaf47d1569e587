#!/bin/bash
source tools/gpu_run.sh
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
grep -q "smoke ok" gpurun_out/smoke.log || { echo "smoke failed"; exit 1; }
step c3quick 120 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 3 --time
step full 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_bigpool.py -k "c3 or c2 or slot or pool" -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
grep -q " passed" gpurun_out/full.log && ! grep -q "failed" gpurun_out/full.log || { echo "parity failed"; exit 1; }
for r in 1 2 3; do
  step c3_ps_$r 120 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 10 --time
  step c3_head_$r 120 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 10 --time --lib abx/lib_head_HEAD.so
done
for r in 1 2; do
  step c3p16k_ps_$r 180 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 10 --time --puzzles 16384
  step c3p16k_head_$r 180 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 10 --time --puzzles 16384 --lib abx/lib_head_HEAD.so
done
