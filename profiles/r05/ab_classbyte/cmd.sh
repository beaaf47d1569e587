source tools/gpu_run.sh
for r in 1 2 3; do
  for v in head_HEAD new; do
    if [ $v = new ]; then L=""; else L="--lib ab/lib_$v.so"; fi
    step c3_${v}_$r 240 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 20 --time $L
    step c2_${v}_$r 240 python tools/prof_rollout.py --config c2 --envs 4096 --chunk 2000 --launches 20 --time $L
  done
done
step diag_c3 300 python tools/diag_split.py --config c3
step gputests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
