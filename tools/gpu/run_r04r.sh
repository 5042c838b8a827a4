# Batch gather (C5 stress): words per thread 16 (product) against 4 (base),
# 8 and 32; the gather parity tests on the product first.
set -e
mkdir -p gpurun_out/r
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_replay_batch.py tests/test_gpu_scale.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r/tests.log; exit 1; }
tail -1 gpurun_out/r/tests.log
for lib in product base gw8 gw32 product base; do
  if [ $lib = product ]; then LIBP=""; else LIBP=$R/distributed-deep-q_amd/ab/$lib/libddq_hip.so; fi
  DDQ_LIB_PATH=$LIBP timeout -k 10 300 python bench.py --steps 5 --warmup 2 --chunks 0 --profile-steps 1 --no-cpu-baseline --no-sweep --no-exchange-paths --no-messaging --no-isolated > gpurun_out/r/$lib.json 2> gpurun_out/r/$lib.err || { echo BENCH_FAILED $lib; tail -5 gpurun_out/r/$lib.err; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r/$lib.json') if l.startswith('{')][-1]);print('$lib', [(x['n'], x['gather_GBps'], x['frac']) for x in d['gather_stress']['launches']])"
done
# timing-only roles of the slab-reduce launch (wrong results): without the
# prefetch blocks, the fc4 apply tiles, the slab units -- at 16x16 and 64x64
NOPARITY=1 FRAME=16 STEPS=2000 bash tools/gpu/run_ab.sh nopf nofa noslab
NOPARITY=1 STEPS=400 bash tools/gpu/run_ab.sh nopf nofa noslab
echo done
