# Round 4, final code, final measurements: the driver's invocation, the default
# line, the full C3 sweep, the step kernel trace (20 eager profile steps),
# the step-only PMC passes.
set -e
mkdir -p gpurun_out/q
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/q/bench_driver.json 2> gpurun_out/q/bench_driver.err || { echo BENCH_FAILED; tail -20 gpurun_out/q/bench_driver.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/q/bench_driver.json | head -3
timeout -k 10 600 python bench.py > gpurun_out/q/bench.json 2> gpurun_out/q/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/q/bench.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/q/bench.json
bash tools/gpu/run_r04_final.sh
