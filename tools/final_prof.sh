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
# spec: config:envs:chunk:kernel[:puzzles] (a pool size other than 1,024 gets its own key, as bench.py)
for spec in ${PROF_SPECS:-"c3:65536:2000:k_rollout1s" "c2:4096:2000:k_rollout1s" "c3r:65536:2000:k_rollout1r" "c3g7:65536:2000:k_rolloutWs" "c4c:262144:2000:k_rolloutWs" "c4:262144:50:k_rollout_obsw" "c3:65536:2000:k_rollout1s:4096" "c3:65536:2000:k_rollout1s:16384"}; do
  IFS=: read cfg envs chunk kern pz <<< "$spec"
  pz=${pz:-1024}
  key=${cfg}_rollout_n${envs}_chunk${chunk}
  name=$cfg
  if [ "$pz" != 1024 ]; then key=${key}_p$pz; name=${cfg}_p$pz; fi
  # pools past 1,024 puzzles run the XCD-local first puzzles (bench.initial_puzzles, auto), as bench.py keys them
  if [ "$pz" -gt 1024 ] && [ $((pz % 8)) = 0 ]; then key=${key}_xcd; fi
  PUZZLES=$pz step prof_$name 420 bash tools/collect_profiles.sh gpurun_out/prof_$name $cfg $envs $chunk 5
  d=gpurun_out/prof_$name
  step fold_$name 60 python tools/pmc_traffic.py $key $kern $d/pmc_fetch.csv $d/pmc_write.csv $d/pmc_rdreq.csv $d/pmc_sq1.csv $d/pmc_sq2.csv
done
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
