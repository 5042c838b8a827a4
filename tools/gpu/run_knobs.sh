# Kernel traces of the graph bench for a list of tuning-knob settings (needs
# the experiment build: make -C distributed-deep-q_amd EXPERIMENTS=1).
# $ENVS: space-separated settings, each "A=1,B=2"; prints one summary line each.
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for e in $ENVS; do
  i=$((i + 1))
  rm -rf $R/gpurun_out/kn$i
  env $(echo $e | tr ',' ' ') timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/kn$i -o run -- python3 $R/bench.py --steps 120 --warmup 10 --profile-steps 1 --chunks 0 --no-cpu-baseline --no-gather-stress --no-sweep > $R/gpurun_out/kn$i.json 2> $R/gpurun_out/kn$i.err
  echo "== $e"
  (cd $R && python3 tools/trace_summary.py gpurun_out/kn$i 0)
done
