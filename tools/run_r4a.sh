source tools/gpu_run.sh
export TMPDIR=/tmp
step gputests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
for sh in 0 1 2 3; do
  step c3r_shape$sh 120 env SPARC_R1R_SHAPE=$sh python tools/prof_rollout.py --config c3r --envs 65536 --chunk 50 --launches 20 --time
done
step c3r_gen 120 env SPARC_RULE_ROLLOUT=generic python tools/prof_rollout.py --config c3r --envs 65536 --chunk 50 --launches 20 --time
step calib_run 60 tools/pmc_calib/pmc_calib
mkdir -p gpurun_out/calib
for pass in "fetch:FETCH_SIZE" "write:WRITE_SIZE" "rdreq:TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"; do
  n=${pass%%:*}; c=${pass#*:}
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $c -d gpurun_out/calib/$n -o run --output-format csv -- tools/pmc_calib/pmc_calib > gpurun_out/calib/$n.log 2>&1 || { echo "calib pass $n failed"; exit 3; }
done
step prof_c3r 420 bash tools/collect_profiles.sh gpurun_out/prof_c3r c3r 65536 50 5
step bench_c3 300 python bench.py
step bench_c3r 300 python bench.py --config c3r
