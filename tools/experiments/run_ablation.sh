# time the Winograd conv (tools/bench_conv.py) for the in-tree build and every tools/exp_*.so variant
set -e
mkdir -p gpurun_out
echo "== in-tree" > gpurun_out/abl.log
ONLY=wino timeout -k 10 60 python tools/bench_conv.py >> gpurun_out/abl.log 2>&1
for f in tools/exp_*.so; do
  [ -e "$f" ] || continue
  echo "== $(basename $f .so)" >> gpurun_out/abl.log
  STIF_HIP_LIB=$PWD/$f ONLY=wino timeout -k 10 60 python tools/bench_conv.py >> gpurun_out/abl.log 2>&1
done
grep -v amdgpu.ids gpurun_out/abl.log
