#!/bin/bash
# A/B timing of library builds under ab/: parity tests of the in-tree build first, then
# tools/prof_rollout.py HIP-event means per variant (alternating, two rounds), logs in gpurun_out/.
# usage: tools/ab_run.sh "<pytest files>" <variant>... (config list in $AB_CONFIGS, default "c3 c2")
source tools/gpu_run.sh
tests=$1; shift
if [ -n "$tests" ]; then
  step parity 600 python -u -m pytest $tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
  grep -q " passed" gpurun_out/parity.log && ! grep -q "failed" gpurun_out/parity.log || { echo "parity failed"; exit 1; }
fi
for cfg in ${AB_CONFIGS:-c3 c2}; do
  envs=65536; [ "$cfg" = c2 ] && envs=4096
  chunk=2000; [ "$cfg" = c3r ] && chunk=50
  for r in 1 2; do
    for v in "$@"; do
      step ab_${cfg}_${v}_$r 120 python tools/prof_rollout.py --config $cfg --envs $envs --chunk $chunk --launches 20 --time --lib ab/lib_$v.so
    done
  done
done
