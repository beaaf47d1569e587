source tools/gpu_run.sh
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in new group8 group16; do
    if [ $v = new ]; then L=""; else L="--lib ab/lib_$v.so"; fi
    step c3_${v}_$r 240 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 20 --time $L
    step c2_${v}_$r 240 python tools/prof_rollout.py --config c2 --envs 4096 --chunk 2000 --launches 20 --time $L
    step c3p4096_${v}_$r 300 python tools/prof_rollout.py --config c3 --chunk 2000 --launches 20 --time --puzzles 4096 $L
  done
done
