# Round-2 final evidence on the committed build (tools/r2_round.sh: GPU suite, smoke, default bench with
# kernel report, kernel-trace stats, FETCH/WRITE/MFMA PMC passes), outputs tagged r2f.
TAG=r2f bash tools/r2_round.sh
