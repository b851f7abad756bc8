# time the f16x3 Winograd conv (tools/bench_conv.py, ONLY=wino16) for the in-tree build and every tools/exp_*.so variant
mkdir -p gpurun_out
echo "== in-tree" > gpurun_out/abl_wino16.log
ONLY=wino16 timeout -k 10 90 python tools/bench_conv.py >> gpurun_out/abl_wino16.log 2>&1 || exit 1
for f in tools/exp_*.so; do
  [ -e "$f" ] || continue
  echo "== $(basename $f .so)" >> gpurun_out/abl_wino16.log
  ONLY=wino16 STIF_HIP_LIB=$PWD/$f timeout -k 10 90 python tools/bench_conv.py >> gpurun_out/abl_wino16.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/abl_wino16.log | grep -v "max |"
