# Round profiles of the shipped step (profiles/r02_*): rocprofv3 kernel-trace
# stats of the graph bench, then one PMC pass per counter group (FETCH_SIZE and
# WRITE_SIZE in passes of their own, tools/pmc_passes.txt), then the summaries.
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 200 --warmup 20 --profile-steps 5 --no-cpu-baseline --no-gather-stress --no-sweep > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof.err
# the step alone (no exchange-path launches in the averages)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_step -o run -- python3 $R/bench.py --steps 200 --warmup 20 --profile-steps 5 --no-cpu-baseline --no-gather-stress --no-sweep --no-exchange-paths > $R/gpurun_out/prof_step_bench.json 2> $R/gpurun_out/prof_step.err
i=0
while read -r line; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc ${line#pmc: } --output-format csv -d $R/gpurun_out/pmc/p$i -o pmc -- python3 $R/bench.py --steps 10 --warmup 2 --profile-steps 1 --chunks 0 --no-cpu-baseline --no-gather-stress --no-sweep > $R/gpurun_out/pmc_bench$i.json 2> $R/gpurun_out/pmc$i.err
done < $R/tools/pmc_passes.txt
cd $R
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt
python3 tools/pmc_json.py gpurun_out/pmc gpurun_out/pmc.json
python3 tools/trace_summary.py gpurun_out/prof 0 > gpurun_out/trace_summary.txt
cat gpurun_out/trace_summary.txt
