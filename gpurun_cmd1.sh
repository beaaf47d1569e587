source tools/gpu_run.sh
step devinfo 300 python -c "import torch; print(torch.cuda.get_device_name(0), torch.cuda.device_count())"
step pytest_gpu 1200 python -m pytest tests -m gpu -x -q
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py --steps 1000 --warmup 100 --cpu-seconds 5
