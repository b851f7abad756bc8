TAG=r2f bash tools/r2_round.sh && KINDS="'conv', 3, 2|'dcn'" REPS=2 bash tools/r2_kreport_ab.sh > gpurun_out/r2f_kreport_ab.log 2>&1; tail -30 gpurun_out/r2f_kreport_ab.log
