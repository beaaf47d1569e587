source tools/gpu_run.sh
export TMPDIR=/tmp
step iotests 300 python -u -m pytest tests/test_gpu_iocodes.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider
for r in 1 2; do
  step ab_c3_base_$r 120 python tools/prof_rollout.py --config c3 --envs 65536 --chunk 2000 --launches 10 --time --lib ab/lib_head_HEAD.so
  step ab_c3_ior_$r 120 python tools/prof_rollout.py --config c3 --envs 65536 --chunk 2000 --launches 10 --time
  step ab_c3_off_$r 120 env SPARC_IO_CODES=off python tools/prof_rollout.py --config c3 --envs 65536 --chunk 2000 --launches 10 --time
  step ab_c2_base_$r 120 python tools/prof_rollout.py --config c2 --envs 4096 --chunk 2000 --launches 10 --time --lib ab/lib_head_HEAD.so
  step ab_c2_ior_$r 120 python tools/prof_rollout.py --config c2 --envs 4096 --chunk 2000 --launches 10 --time
done
