# Round evidence (tools/gpu/run_final.sh), then only the summaries are kept
# under gpurun_out/keep (the raw rocprofv3 traces exceed gpurun's 64 MiB
# copy-back limit): GPU test log, bench lines, kernel stats, PMC summary.
set -e
bash tools/gpu/run_final.sh
du -sh gpurun_out/* 2>/dev/null | sort -h | tail -8
mkdir -p gpurun_out/keep
cp gpurun_out/gpu_tests.log gpurun_out/bench_full.json gpurun_out/bench_acting.json \
   gpurun_out/prof_bench.json gpurun_out/pmc_summary.txt gpurun_out/pmc.json \
   gpurun_out/trace_summary.txt gpurun_out/measure.log gpurun_out/keep/
cp gpurun_out/prof/run_kernel_stats.csv gpurun_out/keep/kernel_stats.csv
cp gpurun_out/prof_step/run_kernel_stats.csv gpurun_out/keep/kernel_stats_step.csv
find gpurun_out -mindepth 1 -maxdepth 1 ! -name keep -exec rm -rf {} +
ls -la gpurun_out/keep
