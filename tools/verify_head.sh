source tools/gpu_run.sh
step gputests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c3 120 python bench.py
step bench_c3r 120 python bench.py --config c3r
step prof_c3r 600 bash tools/collect_profiles.sh gpurun_out/prof_c3r c3r 65536 50 5
