# time the fused DCN kernel (tools/bench_dcn.py) for the in-tree build and every tools/exp_*.so variant
set -e
mkdir -p gpurun_out
echo "== in-tree" > gpurun_out/abl_dcn.log
timeout -k 10 60 python tools/bench_dcn.py >> gpurun_out/abl_dcn.log 2>&1
for f in tools/exp_*.so; do
  [ -e "$f" ] || continue
  echo "== $(basename $f .so)" >> gpurun_out/abl_dcn.log
  STIF_HIP_LIB=$PWD/$f timeout -k 10 60 python tools/bench_dcn.py >> gpurun_out/abl_dcn.log 2>&1
done
grep -v amdgpu.ids gpurun_out/abl_dcn.log
