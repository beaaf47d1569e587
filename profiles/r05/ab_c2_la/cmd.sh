source tools/gpu_run.sh
for r in 1 2 3; do
  step c2_new_$r 240 python tools/prof_rollout.py --config c2 --envs 4096 --chunk 2000 --launches 20 --time
  step c2_nola_$r 240 python tools/prof_rollout.py --config c2 --envs 4096 --chunk 2000 --launches 20 --time --lib ab/lib_nola.so
done
