#!/bin/bash
SKIP_TESTS=1 PROF_SPECS="c4c:262144:2000:k_rolloutWs c4:262144:50:k_rollout_obsw c3:65536:2000:k_rollout1s:4096 c3:65536:2000:k_rollout1s:16384" bash tools/final_prof.sh || exit $?
bash tools/final_bench.sh
