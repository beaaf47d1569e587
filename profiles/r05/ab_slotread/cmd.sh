source tools/gpu_run.sh
export TMPDIR=/tmp
step bigpool 600 python -u -m pytest tests/test_gpu_bigpool.py tests/test_gpu_fullsize.py -q --timeout 300 --timeout-method thread -p no:cacheprovider
for r in 1 2 3; do
  for v in head_HEAD new group8; do
    if [ $v = new ]; then L=""; else L="--lib ab/lib_$v.so"; fi
    step c3_${v}_$r 240 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 20 --time $L
    step c3p4096_${v}_$r 300 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 20 --time --puzzles 4096 $L
    step c3p16384_${v}_$r 300 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 20 --time --puzzles 16384 $L
  done
done
