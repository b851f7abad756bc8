# k_wino f16x3 trunk conv (C0 shape 16 x 128^2 x 64, RES / RELU epilogues): in-tree vs timing probes
# tools/exp_WINO_EXP_{1,2,3}.so (no staging DMA / no B refills / no output exchange)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r3
cd $R
for rep in 1 2; do
  echo "in-tree: $(N=16 HW=128 ONLY=wino16 timeout -k 10 120 python3 tools/bench_conv.py 2>&1 | grep -v amdgpu.ids | head -2 | tr '\n' ' ')"
  for lib in tools/exp_WINO_EXP_*.so; do
    echo "$lib: $(STIF_HIP_LIB=$R/$lib N=16 HW=128 ONLY=wino16 timeout -k 10 120 python3 tools/bench_conv.py 2>&1 | grep -v amdgpu.ids | head -2 | tr '\n' ' ')"
  done
done
