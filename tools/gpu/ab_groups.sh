set -e
for cfg in "16 8" "8 4" "8 8" "16 4"; do
  set -- $cfg
  DDQ_G2=$1 DDQ_G3=$2 DDQ_LIB_PATH=distributed-deep-q_amd/ab/stamps/libddq_hip.so timeout -k 10 120 python tools/gpu/stamps.py 16 32 2 step > gpurun_out/st_$1_$2.txt 2>&1
  echo "== G2=$1 G3=$2"; grep "run 1" gpurun_out/st_$1_$2.txt | grep "slots 24\|slots 32" | sed 's/slot: median.*(us)://'
done
