# Round 4, measurement box: the driver's bench invocation, the default line
# (exchange paths, messaging, deepq16, gather stress, CPU baseline), a
# rocprofv3 kernel trace of the step chain alone, the step-only PMC passes,
# then an A/B of conv2's data gradient at 2 taps per ring step.
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gather-stress --no-sweep --no-exchange-paths --no-messaging > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench_driver.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_driver.json
timeout -k 10 600 python bench.py --no-sweep > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/bench.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_step -o run -- python3 $R/bench.py --steps 200 --warmup 20 --profile-steps 3 --chunks 0 --no-cpu-baseline --no-gather-stress --no-sweep --no-exchange-paths --no-messaging --no-isolated > $R/gpurun_out/prof_step.json 2> $R/gpurun_out/prof_step.err
cd $R
python3 tools/trace_summary.py gpurun_out/prof_step step
bash tools/gpu/run_pmc_step.sh
STEPS=400 bash tools/gpu/run_ab.sh c2dtps2
echo done
