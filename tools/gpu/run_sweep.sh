# kernel-trace stats of the default bench (roofline kernel timed back to back),
# then the C3 batch-256 frame sweep
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 200 --warmup 20 --profile-steps 5 --no-cpu-baseline > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof.err || { echo PROF_FAILED; tail -20 $R/gpurun_out/prof.err; exit 1; }
cd $R
python3 -c "
import json; d=json.load(open('gpurun_out/prof_bench.json')); print(d['value'], json.dumps(d['roofline']))"
grep -o '"[^"]*direct_conv_kernel<32, 64, 5[^"]*",[0-9]*,[0-9]*,[0-9.]*' gpurun_out/prof/run_kernel_stats.csv
timeout -k 10 600 python3 -c "
import json, bench; print(json.dumps(bench.frame_sweep()))" > gpurun_out/sweep.json 2> gpurun_out/sweep.err || { echo SWEEP_FAILED; tail -20 gpurun_out/sweep.err; exit 1; }
cat gpurun_out/sweep.json
