set -o pipefail
mkdir -p gpurun_out/ramp
for i in 1 2 3 4 5 6; do
  timeout -k 10 150 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/ramp/b$i.json 2> gpurun_out/ramp/b$i.err || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/ramp/b$i.json').read().strip().splitlines()[-1]);print($i, round(d['value'],1), round(d['unramped']['TFLOP/s'],1), round(d['flash_causal']['TFLOP/s'],1), flush=True)"
done
