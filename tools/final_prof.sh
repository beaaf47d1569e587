#!/bin/bash
# End-of-round measurement, part 1: the GPU suite, smoke, then per bench config the kernel
# stats + 4 PMC passes (tools/collect_profiles.sh) folded into profiles/pmc_traffic.json on the
# box (copied back to gpurun_out/pmc_traffic.json).  Part 2 (tools/final_bench.sh) runs the
# bench lines against that file.
source tools/gpu_run.sh
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
  grep -q " passed" gpurun_out/gputests.log && ! grep -q "failed" gpurun_out/gputests.log || { echo "tests failed"; exit 1; }
  step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
fi
for spec in ${PROF_SPECS:-"c3:65536:2000:k_rollout1s" "c2:4096:2000:k_rollout1s" "c3r:65536:2000:k_rollout1r" "c3g7:65536:2000:k_rolloutWs" "c4c:262144:2000:k_rolloutWs" "c4:262144:50:k_rollout"}; do
  IFS=: read cfg envs chunk kern <<< "$spec"
  step prof_$cfg 420 bash tools/collect_profiles.sh gpurun_out/prof_$cfg $cfg $envs $chunk 5
  d=gpurun_out/prof_$cfg
  step fold_$cfg 60 python tools/pmc_traffic.py ${cfg}_rollout_n${envs}_chunk${chunk} $kern $d/pmc_fetch.csv $d/pmc_write.csv $d/pmc_rdreq.csv $d/pmc_sq1.csv $d/pmc_sq2.csv
done
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
