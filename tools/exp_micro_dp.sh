set -e
for args in "--micro 2" "--micro 1" "--micro 2 --force-dp" "--micro 1 --force-dp"; do
  echo "== $args" >> gpurun_out/exp1.log
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-inference --no-edsr --steps 20 --warmup 5 $args 2>>gpurun_out/exp1.err | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'])" >> gpurun_out/exp1.log
done
