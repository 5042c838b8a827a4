# PMC passes of the bench's step chain alone (no exchange paths, no isolated
# layer timing): one counter group per pass (tools/pmc_passes.txt), then the
# per-kernel JSON (FETCH x2 gfx950 correction) and the SQ summary.
set -e
mkdir -p gpurun_out/pmc_step
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
while read -r line; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc ${line#pmc: } --output-format csv -d $R/gpurun_out/pmc_step/p$i -o pmc -- python3 $R/bench.py --steps 40 --warmup 8 --profile-steps 1 --chunks 0 --no-cpu-baseline --no-gather-stress --no-sweep --no-exchange-paths --no-messaging --no-isolated > $R/gpurun_out/pmc_step_bench$i.json 2> $R/gpurun_out/pmc_step$i.err
done < $R/tools/pmc_passes.txt
cd $R
python3 tools/pmc_summary.py gpurun_out/pmc_step > gpurun_out/pmc_step_summary.txt
python3 tools/pmc_json.py gpurun_out/pmc_step gpurun_out/pmc_step.json
cat gpurun_out/pmc_step_summary.txt
