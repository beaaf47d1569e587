source tools/gpu_run.sh
export TMPDIR=/tmp
for r in 1 2; do
  step ab_c3_base_$r 120 python tools/prof_rollout.py --config c3 --envs 65536 --chunk 2000 --launches 10 --time --lib ab/lib_head_HEAD.so
  step ab_c3_pin_$r 120 python tools/prof_rollout.py --config c3 --envs 65536 --chunk 2000 --launches 10 --time
  step ab_c2_base_$r 120 python tools/prof_rollout.py --config c2 --envs 4096 --chunk 2000 --launches 10 --time --lib ab/lib_head_HEAD.so
  step ab_c2_pin_$r 120 python tools/prof_rollout.py --config c2 --envs 4096 --chunk 2000 --launches 10 --time
  step ab_c4_head_$r 120 python tools/prof_rollout.py --config c4 --envs 262144 --chunk 50 --launches 10 --time
  step ab_c4_obswb_$r 120 python tools/prof_rollout.py --config c4 --envs 262144 --chunk 50 --launches 10 --time --lib ab/lib_obswb.so
done
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
