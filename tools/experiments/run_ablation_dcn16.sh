# time the fused DCN core (tools/bench_dcn16.py: f32 and f16x3) for the in-tree build and every tools/exp_*.so variant
set -e
mkdir -p gpurun_out
echo "== in-tree" > gpurun_out/abl_dcn16.log
timeout -k 10 90 python tools/bench_dcn16.py >> gpurun_out/abl_dcn16.log 2>&1
for f in tools/exp_*.so; do
  [ -e "$f" ] || continue
  echo "== $(basename $f .so)" >> gpurun_out/abl_dcn16.log
  STIF_HIP_LIB=$PWD/$f timeout -k 10 90 python tools/bench_dcn16.py >> gpurun_out/abl_dcn16.log 2>&1
done
grep -v amdgpu.ids gpurun_out/abl_dcn16.log
