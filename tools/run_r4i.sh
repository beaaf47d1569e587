source tools/gpu_run.sh
export TMPDIR=/tmp
step iotests 400 python -u -m pytest tests/test_gpu_iocodes.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider
for r in 1 2; do
  step ab_c3g7_base_$r 120 python tools/prof_rollout.py --config c3g7 --envs 65536 --chunk 2000 --launches 10 --time --lib ab/lib_head_HEAD.so
  step ab_c3g7_ior_$r 120 python tools/prof_rollout.py --config c3g7 --envs 65536 --chunk 2000 --launches 10 --time
  step ab_c4c_base_$r 120 python tools/prof_rollout.py --config c4c --envs 262144 --chunk 2000 --launches 5 --time --lib ab/lib_head_HEAD.so
  step ab_c4c_ior_$r 120 python tools/prof_rollout.py --config c4c --envs 262144 --chunk 2000 --launches 5 --time
  step ab_c3_ior_$r 120 python tools/prof_rollout.py --config c3 --envs 65536 --chunk 2000 --launches 10 --time
done
for r in 1 2; do
  step ab_c3r_head_$r 120 python tools/prof_rollout.py --config c3r --envs 65536 --chunk 2000 --launches 5 --time
  step ab_c3r_downfill_$r 120 python tools/prof_rollout.py --config c3r --envs 65536 --chunk 2000 --launches 5 --time --lib ab/lib_downfill.so
done
step diag_c3 120 python tools/diag_split.py --config c3
step diag_c2 120 python tools/diag_split.py --config c2 --envs 4096
