for v in "" WINO_EXP_NOB WINO_EXP_NOXF WINO_EXP_NOSTAGE WINO_EXP_NOEPI; do
  echo "== $v"
  if [ -z "$v" ]; then lib=""; else lib=tools/exp_$v.so; fi
  STIF_HIP_LIB=$lib ONLY=wino16 timeout -k 10 60 python -u tools/bench_conv.py 2>&1 | grep wino16 || exit 1
  if [ -n "$v" ]; then tl=tools/exp_WINO_EXP_TRACE+$v.so; else tl=tools/exp_WINO_EXP_TRACE.so; fi
  F16=1 STIF_HIP_LIB=$tl timeout -k 10 60 python -u tools/trace_wino.py 2>&1 | grep "wave 0" || exit 1
done
