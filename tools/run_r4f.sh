source tools/gpu_run.sh
export TMPDIR=/tmp
for r in 1 2; do
  step ab_c3r50_new_$r 120 python tools/prof_rollout.py --config c3r --envs 65536 --chunk 50 --launches 20 --time
  step ab_c3r50_base_$r 120 python tools/prof_rollout.py --config c3r --envs 65536 --chunk 50 --launches 20 --time --lib ab/lib_r1rbase.so
  step ab_c3r2k_new_$r 120 python tools/prof_rollout.py --config c3r --envs 65536 --chunk 2000 --launches 5 --time
  step ab_c3r2k_base_$r 120 python tools/prof_rollout.py --config c3r --envs 65536 --chunk 2000 --launches 5 --time --lib ab/lib_r1rbase.so
done
