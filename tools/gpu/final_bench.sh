# Final round bench lines: the default command with --acting, then the
# driver's own short command.
set -e
mkdir -p gpurun_out
timeout -k 10 700 python bench.py --acting > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err
python tools/bench_summary.py gpurun_out/bench_final.json | head -12
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err
python tools/bench_summary.py gpurun_out/bench_driver.json | head -3
