source tools/gpu_run.sh
export TMPDIR=/tmp
step gputests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
for r in 1 2; do
  for v in noalign new; do
    if [ $v = new ]; then L=""; else L="--lib ab/lib_$v.so"; fi
    step c3_${v}_$r 240 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 20 --time $L
    step c3p4096_${v}_$r 300 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 20 --time --puzzles 4096 $L
  done
done
step diag_c3 300 python tools/diag_split.py --config c3
