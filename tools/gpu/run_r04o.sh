# no-grad-store: its test, then the main line with / without it (alternating);
# A/Bs of variant builds (conv1 tiles, zero-filled dconv1 image, fused conv1
# weight-gradient cost (timing only), small-map conv2 forward with 2 k groups).
set -e
mkdir -p gpurun_out/o
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "no_grad_store" --timeout 300 --timeout-method thread > gpurun_out/o/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/o/tests.log; exit 1; }
tail -1 gpurun_out/o/tests.log
for i in 1 2; do
  for m in store nostore; do
    F=""; [ $m = nostore ] && F="--no-grad-store"
    timeout -k 10 200 python bench.py --steps 400 --warmup 40 $F --no-cpu-baseline --no-gather-stress --no-sweep --no-exchange-paths --no-messaging --no-isolated > gpurun_out/o/$m$i.json 2> gpurun_out/o/$m$i.err || { echo BENCH_FAILED; tail -5 gpurun_out/o/$m$i.err; exit 1; }
    python3 tools/bench_summary.py gpurun_out/o/$m$i.json | sed "s/^/[$m$i] /" | head -3
  done
done
STEPS=400 bash tools/gpu/run_ab.sh c1t16 c1t20 c1t24 w1zf
NOPARITY=1 STEPS=400 bash tools/gpu/run_ab.sh now1
FRAME=16 STEPS=2000 bash tools/gpu/run_ab.sh c2fwk2
echo done
