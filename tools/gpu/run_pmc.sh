set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 -i $R/tools/pmc_passes.txt --output-format csv -d $R/gpurun_out/pmc -o pmc -- python3 $R/bench.py --steps 10 --warmup 2 --profile-steps 1 --no-cpu-baseline --eager > $R/gpurun_out/pmc_bench.json 2> $R/gpurun_out/pmc.err
cd $R
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt
cat gpurun_out/pmc_summary.txt
