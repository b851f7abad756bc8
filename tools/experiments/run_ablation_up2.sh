# time the x2 upsample (tools/bench_up2.py) for the in-tree build and every tools/exp_*.so variant
mkdir -p gpurun_out
echo "== in-tree" > gpurun_out/abl_up2.log
timeout -k 10 90 python tools/bench_up2.py >> gpurun_out/abl_up2.log 2>&1 || exit 1
for f in tools/exp_*.so; do
  [ -e "$f" ] || continue
  echo "== $(basename $f .so)" >> gpurun_out/abl_up2.log
  STIF_HIP_LIB=$PWD/$f timeout -k 10 90 python tools/bench_up2.py >> gpurun_out/abl_up2.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/abl_up2.log
