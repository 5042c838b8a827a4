set -e
mkdir -p gpurun_out
for v in ${VARIANTS:-0}; do
 for pl in "" "--no-pipeline"; do
  DDQ_VARIANT=$v timeout -k 10 300 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --profile-steps 2 $pl > gpurun_out/b4.json 2> gpurun_out/b4.err
  python -c "import json; d=json.load(open('gpurun_out/b4.json')); print('variant $v $pl', d['value'], d['ms_per_step'])"
 done
done
