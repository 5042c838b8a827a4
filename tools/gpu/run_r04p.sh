# Zero-filled dconv1 image + small-map conv2 k groups: parity / chain suites,
# then the main line and the 16x16 line.
set -e
mkdir -p gpurun_out/p
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_chain.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/p/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/p/tests.log | head -30; tail -5 gpurun_out/p/tests.log; exit 1; }
tail -1 gpurun_out/p/tests.log
for F in 64 16; do
  timeout -k 10 200 python bench.py --frame $F --steps 400 --warmup 40 --no-cpu-baseline --no-gather-stress --no-sweep --no-exchange-paths --no-messaging --no-isolated > gpurun_out/p/b$F.json 2> gpurun_out/p/b$F.err || { echo BENCH_FAILED; tail -5 gpurun_out/p/b$F.err; exit 1; }
  python3 tools/bench_summary.py gpurun_out/p/b$F.json | sed "s/^/[$F] /" | head -3
done
echo done
