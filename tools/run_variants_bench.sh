# full C1 bench (kernel report) for the in-tree build and every tools/exp_*.so variant
set -e
mkdir -p gpurun_out
echo "== in-tree" > gpurun_out/var_bench.log
timeout -k 10 300 python bench.py --kernel-report --no-cpu-baseline >> gpurun_out/var_bench.log 2>&1
for f in tools/exp_*.so; do
  [ -e "$f" ] || continue
  echo "== $(basename $f .so)" >> gpurun_out/var_bench.log
  STIF_HIP_LIB=$PWD/$f timeout -k 10 300 python bench.py --kernel-report --no-cpu-baseline >> gpurun_out/var_bench.log 2>&1
done
grep -v amdgpu.ids gpurun_out/var_bench.log | grep "==\|${GREP:-value}" | cut -c1-160
