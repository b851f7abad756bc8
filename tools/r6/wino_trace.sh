#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
STIF_HIP_LIB=$R/tools/exp_WINO_TRACE_1.so timeout -k 10 300 python -u tools/r6/wino_trace.py
