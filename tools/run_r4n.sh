source tools/gpu_run.sh
export TMPDIR=/tmp
for r in 1 2 3; do
  step ab_c4_head_$r 120 python tools/prof_rollout.py --config c4 --envs 262144 --chunk 50 --launches 10 --time --lib ab/lib_head.so
  step ab_c4_obsun2_$r 120 python tools/prof_rollout.py --config c4 --envs 262144 --chunk 50 --launches 10 --time --lib ab/lib_obsun2.so
done
