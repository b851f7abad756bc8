# Round-end evidence on one MI355X: GPU suite, smoke, C1 (with CPU baseline) and C2 bench lines,
# rocprofv3 kernel stats and FETCH/WRITE PMC passes of the C1 bench.
set -e
R=$GRAFT_REPO_ROOT
bash $R/tools/round_check.sh
bash $R/tools/profile_round.sh
