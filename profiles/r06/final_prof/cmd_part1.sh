#!/bin/bash
PROF_SPECS="c3:65536:2000:k_rollout1s c2:4096:2000:k_rollout1s c3r:65536:2000:k_rollout1r c3g7:65536:2000:k_rolloutWs" bash tools/final_prof.sh
