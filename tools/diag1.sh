R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/host_idle.py 1 2 > gpurun_out/host_idle.log 2>&1 || { echo host_idle failed; tail gpurun_out/host_idle.log; exit 1; }
cat gpurun_out/host_idle.log
bash tools/prof_step.sh m2 --micro 2 && bash tools/prof_step.sh m1 --micro 1 || exit 2
python3 tools/step_timeline.py gpurun_out/prof_m2/t_kernel_trace.csv 1 > gpurun_out/tl_m2.txt
python3 tools/step_timeline.py gpurun_out/prof_m1/t_kernel_trace.csv 1 > gpurun_out/tl_m1.txt
head -30 gpurun_out/tl_m2.txt gpurun_out/tl_m1.txt
