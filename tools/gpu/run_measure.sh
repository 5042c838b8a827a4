# rocprofv3 kernel-trace stats + PMC passes of the default bench (round profiles)
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 200 --warmup 20 --profile-steps 5 --no-cpu-baseline > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof.err
timeout -k 10 900 rocprofv3 -i $R/tools/pmc_passes.txt --output-format csv -d $R/gpurun_out/pmc -o pmc -- python3 $R/bench.py --steps 10 --warmup 2 --profile-steps 1 --no-cpu-baseline --eager > $R/gpurun_out/pmc_bench.json 2> $R/gpurun_out/pmc.err
cd $R
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt
python3 tools/pmc_json.py gpurun_out/pmc gpurun_out/pmc.json
t=$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)
python3 tools/timeline.py "$t" --nsteps 1 > gpurun_out/timeline.txt
cat gpurun_out/timeline.txt
