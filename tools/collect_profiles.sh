#!/bin/bash
# Kernel-trace stats and the four PMC passes of one rollout workload, for the bench's roofline
# (run on the GPU box from the repo root; fold the passes here afterwards with
#  tools/pmc_traffic.py <config>_rollout_n<envs>_chunk<chunk> <kernel> <dir>/pmc_{fetch,write,rdreq,sq1,sq2}.csv)
# usage: tools/collect_profiles.sh <out-dir> <config> <envs> <chunk> [launches]
set -u
out=$1; cfg=$2; envs=$3; chunk=$4; launches=${5:-5}
mkdir -p "$out"
export TMPDIR=/tmp
# PUZZLES: the pool size (default 1,024); the pool is built once before the profiler starts (the
# profiled runs load it from SPARC_POOL_CACHE and fork no workers)
export SPARC_POOL_CACHE=${SPARC_POOL_CACHE:-/tmp/sparc_pools} SPARC_POOL_WORKERS=1
P=(python3 tools/prof_rollout.py --config "$cfg" --envs "$envs" --chunk "$chunk" --launches "$launches" --time --puzzles "${PUZZLES:-1024}")
SPARC_POOL_WORKERS=8 timeout -k 10 300 python3 -c "import sys; sys.path[:0] = ['.', 'sparc-gym_amd']; import bench; bench.make_pool(${PUZZLES:-1024}, *bench.CONFIGS['$cfg'][:2])" \
    || { echo "pool build failed"; exit 3; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- "${P[@]}" \
    > "$out/trace.log" 2>&1 || { echo "trace pass failed"; exit 3; }
f=$(find "$out/trace" -name '*kernel_stats.csv' | head -n 1)
[ -n "$f" ] && cp "$f" "$out/kernel_stats.csv"
for pass in "fetch:FETCH_SIZE" "write:WRITE_SIZE" \
            "rdreq:TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
            "sq1:SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
            "sq2:SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
            ${EXTRA_PASSES:-}; do
    n=${pass%%:*}
    c=${pass#*:}
    c=${c//,/ }   # EXTRA_PASSES="name:CTR1,CTR2 ..." (comma-separated counters per pass)
    # shellcheck disable=SC2086
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d "$out/$n" -o run --output-format csv -- "${P[@]}" \
        > "$out/$n.log" 2>&1 || { echo "pmc pass $n failed"; exit 3; }
    f=$(find "$out/$n" -name '*counter_collection.csv' | head -n 1)
    [ -n "$f" ] && cp "$f" "$out/pmc_$n.csv"
done
rm -rf "$out/trace" "$out/fetch" "$out/write" "$out/rdreq" "$out/sq1" "$out/sq2" "$out/tcc"
ls -la "$out"
