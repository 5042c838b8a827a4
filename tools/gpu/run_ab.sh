# A/B of variant libraries (distributed-deep-q_amd/ab/<name>/libddq_hip.so,
# make variant): a parity subset on each variant first, then the bench main
# line and a rocprofv3 kernel trace of the step for the product and each
# variant.  Usage: [FRAME=16] [STEPS=n] [NOPARITY=1] bash tools/gpu/run_ab.sh name1 [name2 ...]
set -e
mkdir -p gpurun_out/ab
R=$GRAFT_REPO_ROOT
for V in "$@"; do
  [ -n "$NOPARITY" ] && break   # (a variant already tested: e.g. the previous product)
  LIBV=$R/distributed-deep-q_amd/ab/$V/libddq_hip.so
  DDQ_LIB_PATH=$LIBV timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "full_pass_parity and (64-32 or 16-32 or 40-4 or 24-8 or 72-4 or 96-4 or 128-2)" > gpurun_out/ab/parity_$V.log 2>&1 || { echo VARIANT_PARITY_FAILED $V; tail -30 gpurun_out/ab/parity_$V.log; exit 1; }
  echo "[$V] $(tail -1 gpurun_out/ab/parity_$V.log)"
done
for lib in product "$@"; do
  if [ $lib = product ]; then LIBP=""; else LIBP=$R/distributed-deep-q_amd/ab/$lib/libddq_hip.so; fi
  DDQ_LIB_PATH=$LIBP timeout -k 10 200 python bench.py --frame ${FRAME:-64} --steps ${STEPS:-400} --warmup 40 --no-cpu-baseline --no-gather-stress --no-sweep --no-exchange-paths --no-messaging > gpurun_out/ab/$lib.json 2> gpurun_out/ab/$lib.err || { echo AB_FAILED $lib; tail -5 gpurun_out/ab/$lib.err; exit 1; }
  python tools/bench_summary.py gpurun_out/ab/$lib.json | sed "s/^/[$lib] /" | head -3
done
for lib in product "$@"; do
  if [ $lib = product ]; then LIBP=""; else LIBP=$R/distributed-deep-q_amd/ab/$lib/libddq_hip.so; fi
  cd /tmp && export TMPDIR=/tmp
  DDQ_LIB_PATH=$LIBP timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab/prof_$lib -o run -- python3 $R/bench.py --frame ${FRAME:-64} --steps 200 --warmup 20 --profile-steps 1 --chunks 0 --no-cpu-baseline --no-gather-stress --no-sweep --no-exchange-paths --no-messaging > $R/gpurun_out/ab/prof_$lib.json 2> $R/gpurun_out/ab/prof_$lib.err || { echo PROF_FAILED $lib; exit 1; }
  cd $R
  python3 tools/trace_summary.py gpurun_out/ab/prof_$lib $lib
done
