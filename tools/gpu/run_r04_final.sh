# Round 4, final measurement box: the full 16..128/8 C3 sweep, the rocprofv3
# kernel trace of the step chain (20 eager profile steps for the in-step
# segment), the step-only PMC passes.
set -e
mkdir -p gpurun_out/final
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py --steps 100 --warmup 20 --chunks 0 --no-cpu-baseline --no-gather-stress --no-exchange-paths --no-messaging --no-isolated --sweep > gpurun_out/final/sweep.json 2> gpurun_out/final/sweep.err || { echo SWEEP_FAILED; tail -20 gpurun_out/final/sweep.err; exit 1; }
python3 -c "import json;d=json.loads([l for l in open('gpurun_out/final/sweep.json') if l.startswith('{')][-1]);print([(f['frame'],f['updates_per_s']) for f in d['frame_sweep']['frames']])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/final/prof_step -o run -- python3 $R/bench.py --steps 200 --warmup 20 --profile-steps 20 --chunks 0 --no-cpu-baseline --no-gather-stress --no-sweep --no-exchange-paths --no-messaging --no-isolated > $R/gpurun_out/final/prof_step.json 2> $R/gpurun_out/final/prof_step.err
cd $R
python3 tools/trace_summary.py gpurun_out/final/prof_step step
bash tools/gpu/run_pmc_step.sh
echo done
