#!/bin/bash
# Round-4 A/B driver over explicit variant libraries (LIBS = space-separated tools/exp_*.so), every GPU step
# under its own timeout, the first failure ends the call:
#   1. TESTS (in-tree) and LIBTESTS (under each variant library) -- pytest files, "none" to skip, with
#      TESTK / LIBK as their -k expressions;
#   2. the C0 window's outputs of each variant compared bit for bit with the in-tree build (DUMP=0 skips);
#   3. REPS alternating reps of MICRO (a command line, run per library) and of the C0 bench kernel report
#      (GREP selects its kernel-kind lines).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4
mkdir -p $O
cd $R
REPS=${REPS:-2}
TESTS=${TESTS:-none}
LIBTESTS=${LIBTESTS:-none}
GREP=${GREP:-"'dcnsep'\\|'dec"}
if [ "$TESTS" != none ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -k "${TESTK:-}" -x -q --timeout 200 --timeout-method thread > $O/abx_tests.log 2>&1 \
    || { tail -40 $O/abx_tests.log; exit 1; }
  tail -2 $O/abx_tests.log
fi
for v in $LIBS; do
  if [ "$LIBTESTS" != none ]; then
    STIF_HIP_LIB=$R/$v timeout -k 10 600 python -u -m pytest $LIBTESTS -k "${LIBK:-}" -x -q --timeout 200 --timeout-method thread \
      > $O/abx_libtests.log 2>&1 || { echo "$v"; tail -40 $O/abx_libtests.log; exit 1; }
    echo "$v: $(tail -1 $O/abx_libtests.log)"
  fi
done
if [ "${DUMP:-1}" != 0 ]; then
  timeout -k 10 200 python -u tools/r4/dump_out.py 2>&1 | sed '/amdgpu.ids/d' || exit 1
  for v in $LIBS; do
    STIF_HIP_LIB=$R/$v TAG=$(basename $v .so) CMP=in-tree timeout -k 10 200 python -u tools/r4/dump_out.py 2>&1 \
      | sed '/amdgpu.ids/d' || exit 1
    rm -f $O/out_$(basename $v .so).npy
  done
  rm -f $O/out_in-tree.npy
fi
for rep in $(seq $REPS); do
  for v in in-tree $LIBS; do
    if [ "$v" != in-tree ]; then export STIF_HIP_LIB=$R/$v; else unset STIF_HIP_LIB; fi
    if [ -n "$MICRO" ]; then
      echo "$v: $(timeout -k 10 200 bash -c "$MICRO" 2>&1 | sed '/amdgpu.ids/d' | tr '\n' ' ')" || exit 1
    fi
    timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline --steps 20 --kernel-report > $O/ab.json 2> $O/ab.err \
      || { tail -30 $O/ab.err; exit 1; }
    python - $v <<'PY'
import json, sys
d = json.loads(open("gpurun_out/r4/ab.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:44s}", d["value"], "Mpix/s", d["ms_per_step"], "ms")
PY
    grep "$GREP" $O/ab.err
  done
done
exit 0
