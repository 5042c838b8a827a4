# Round 4: the driver's invocation with and without the preheat (alternating,
# short legs), then the driver's full line and the default line.
set -e
mkdir -p gpurun_out/v
Q="--no-cpu-baseline --no-gather-stress --no-sweep --no-exchange-paths --no-messaging"
for i in 1 2; do
  for ph in 100 0; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --preheat-ms $ph $Q > gpurun_out/v/ab_${ph}_$i.json 2> gpurun_out/v/ab_${ph}_$i.err
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[1],d['value'],d['ms_per_step'],d['preheat'])" gpurun_out/v/ab_${ph}_$i.json
  done
done
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/v/bench_driver.json 2> gpurun_out/v/bench_driver.err
python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('driver',d['value'],d['ms_per_step'],d['step_ms_distribution'],d['roofline']['frac'])" gpurun_out/v/bench_driver.json
timeout -k 10 600 python bench.py > gpurun_out/v/bench.json 2> gpurun_out/v/bench.err
python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('default',d['value'],d['ms_per_step'],d['step_ms_distribution'],d['roofline']['frac'])" gpurun_out/v/bench.json
echo done
