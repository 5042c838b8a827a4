# Small-map slab groups with a row minimum (8 / 16 / 32 rows per group at
# S <= 32) at 16x16 and 32x32; conv2's data gradient with two k groups at 64x64.
set -e
mkdir -p gpurun_out/s
FRAME=16 STEPS=2000 bash tools/gpu/run_ab.sh rmin8 rmin16 rmin32
NOPARITY=1 FRAME=32 STEPS=1000 bash tools/gpu/run_ab.sh rmin16 rmin32
STEPS=400 bash tools/gpu/run_ab.sh c2dwk2
echo done
