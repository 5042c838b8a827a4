# kernel trace (durations) + PMC passes of the graph bench; summary per kernel
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/kt $R/gpurun_out/kp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt -o run -- python3 $R/bench.py --steps 200 --warmup 20 --profile-steps 1 --chunks 0 --no-cpu-baseline --no-gather-stress --no-sweep > $R/gpurun_out/kt.json 2> $R/gpurun_out/kt.err
timeout -k 10 600 rocprofv3 -i $R/tools/pmc_split.txt --output-format csv -d $R/gpurun_out/kp -o kp -- python3 $R/bench.py --steps 20 --warmup 2 --profile-steps 1 --chunks 0 --no-cpu-baseline --no-gather-stress --no-sweep > /dev/null 2> $R/gpurun_out/kp.err
cd $R
python3 tools/trace_summary.py gpurun_out/kt 0
python3 tools/pmc_kernels.py gpurun_out/kp "${PMC_FILTER:-wgrads}"
