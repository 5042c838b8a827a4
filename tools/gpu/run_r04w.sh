# Round 4 exchange-path A/B: the exchange, async and chain suites on the
# product, then the world-1 exchange paths of the product and the variant
# build ab/$V (default nowt), alternating.  Usage: [V=name] bash tools/gpu/run_r04w.sh
set -e
mkdir -p gpurun_out/w
R=$GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests/test_gpu_exchange.py tests/test_gpu_async.py tests/test_gpu_chain.py -x -q --timeout 300 --timeout-method thread > gpurun_out/w/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/w/tests.log; exit 1; }
tail -1 gpurun_out/w/tests.log
Q="--steps 100 --warmup 20 --chunks 0 --no-cpu-baseline --no-gather-stress --no-sweep --no-messaging --no-isolated"
for i in 1 2; do
  for lib in product ${V:-nowt}; do
    if [ $lib = product ]; then LIBP=""; else LIBP=$R/distributed-deep-q_amd/ab/$lib/libddq_hip.so; fi
    DDQ_LIB_PATH=$LIBP timeout -k 10 300 python bench.py $Q > gpurun_out/w/${lib}_$i.json 2> gpurun_out/w/${lib}_$i.err || { echo BENCH_FAILED $lib; tail -5 gpurun_out/w/${lib}_$i.err; exit 1; }
    python3 - gpurun_out/w/${lib}_$i.json $lib <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["exchange_paths"]
print(sys.argv[2], "free", e["exchange_free"], {k: (v["updates_per_s"], v["vs_exchange_free"], {n: v.get("kernels_us", {}).get(n) for n in ("apply", "apply_shard", "refresh", "wgrad_reduce")}) for k, v in e["paths"].items()})
PY
  done
done
echo done
