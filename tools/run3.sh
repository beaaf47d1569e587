source tools/gpu_run.sh
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
grep -q " passed" gpurun_out/gputests.log && ! grep -q "failed" gpurun_out/gputests.log || { echo "tests failed"; exit 1; }
for cfg in c2 c3; do
  envs=65536; [ "$cfg" = c2 ] && envs=4096
  for r in 1 2; do for v in base la64; do
    step ab_${cfg}_${v}_$r 120 python tools/prof_rollout.py --config $cfg --envs $envs --chunk 2000 --launches 20 --time --lib ab/lib_$v.so
  done; done
  step diag_$cfg 120 python tools/diag_split.py --config $cfg --envs $envs
done
