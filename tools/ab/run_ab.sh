# A/B timing of variant builds (distributed-deep-q_amd/ab/<name>/libddq_hip.so,
# built here with `make -C distributed-deep-q_amd variant NAME=... DEFS=...`):
# the bench main line + per-kernel eager times per variant, and a rocprofv3
# kernel-trace summary of each.  Usage: bash tools/ab/run_ab.sh name1 name2 ...
set -e
mkdir -p gpurun_out/ab
R=$GRAFT_REPO_ROOT
for v in "$@"; do
  if [ "$v" = product ]; then LIBP=""; else LIBP=$R/distributed-deep-q_amd/ab/$v/libddq_hip.so; fi
  DDQ_LIB_PATH=$LIBP timeout -k 10 200 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --no-gather-stress --no-sweep --no-exchange-paths > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || { echo "AB_FAILED $v"; tail -5 gpurun_out/ab/$v.err; exit 1; }
  python tools/bench_summary.py gpurun_out/ab/$v.json | sed "s/^/[$v] /" | head -3
  cd /tmp && export TMPDIR=/tmp
  DDQ_LIB_PATH=$LIBP timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab/prof_$v -o run -- python3 $R/bench.py --steps 200 --warmup 20 --profile-steps 2 --chunks 0 --no-cpu-baseline --no-gather-stress --no-sweep --no-exchange-paths > $R/gpurun_out/ab/prof_$v.json 2> $R/gpurun_out/ab/prof_$v.err || { echo "PROF_FAILED $v"; exit 1; }
  cd $R
  python3 tools/trace_summary.py gpurun_out/ab/prof_$v 0 | sed "s/^/[$v] /" | tail -2
done
