# kernel traces for a list of environment settings ($ENVS: space-separated, each "A=1,B=2")
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for e in $ENVS; do
  i=$((i+1))
  rm -rf $R/gpurun_out/tr_e$i
  env $(echo $e | tr ',' ' ') timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr_e$i -o run -- python3 $R/bench.py --steps 400 --warmup 20 --profile-steps 1 --chunks 0 --no-cpu-baseline --no-gather-stress > $R/gpurun_out/tr_e$i.json 2> $R/gpurun_out/tr_e$i.err || { echo BENCH_FAILED $e; tail -5 $R/gpurun_out/tr_e$i.err; exit 1; }
  python3 $R/tools/trace_summary.py $R/gpurun_out/tr_e$i "$e"
done
