source tools/gpu_run.sh
step gputests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
bash tools/final_bench.sh
