#!/bin/bash
# One GPU iteration: kernel tests -> model tests -> kernel microbench -> bench.  Each step time-limited;
# stops at the first crash-like failure (rc > 1).
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out
python3 -c "import torch; p=torch.cuda.get_device_properties(0); print('CUs', p.multi_processor_count, p.name)" > gpurun_out/dev.log 2>&1
timeout -k 10 400 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu > gpurun_out/gpu_kernels.log 2>&1; rc=$?
echo "kernels rc=$rc" >> gpurun_out/gpu_kernels.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -m pytest tests/test_gpu_model.py -x -q -m gpu > gpurun_out/gpu_model.log 2>&1; rc=$?
echo "model rc=$rc" >> gpurun_out/gpu_model.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python tools/kbench.py > gpurun_out/kbench.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 4
echo iter done
