# trunk-conv microbenchmark (f16x3 Winograd, RES / RELU epilogues) at 128x128 maps over item counts: the
# per-launch fixed cost (ramp-up, final round, drain) is the intercept of time vs tiles
set -e
R=$GRAFT_REPO_ROOT
cd $R
for n in 9 18 27 36 72 144; do
  echo "N=$n: $(N=$n HW=128 ONLY=wino16 timeout -k 10 120 python3 tools/bench_conv.py 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')"
done
for n in 18 72; do
  echo "N=$n HW=256: $(N=$n HW=256 ONLY=wino16 timeout -k 10 120 python3 tools/bench_conv.py 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')"
done
