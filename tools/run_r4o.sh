source tools/gpu_run.sh
export TMPDIR=/tmp
for r in 1 2; do
  step ab_c3_head_$r 120 python tools/prof_rollout.py --config c3 --envs 65536 --chunk 2000 --launches 10 --time --lib ab/lib_head.so
  step ab_c3_noprio_$r 120 python tools/prof_rollout.py --config c3 --envs 65536 --chunk 2000 --launches 10 --time --lib ab/lib_noprio.so
  step ab_c2_head_$r 120 python tools/prof_rollout.py --config c2 --envs 4096 --chunk 2000 --launches 10 --time --lib ab/lib_head.so
  step ab_c2_noprio_$r 120 python tools/prof_rollout.py --config c2 --envs 4096 --chunk 2000 --launches 10 --time --lib ab/lib_noprio.so
done
