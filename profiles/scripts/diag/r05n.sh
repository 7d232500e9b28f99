ROOT=$(pwd)
bash profiles/scripts/ktrace_c.sh r05n_c1 1 && python3 profiles/ktrace_eval.py gpurun_out/r05n_c1_kt > gpurun_out/r05n_c1_eval.txt && bash profiles/scripts/ktrace_c4.sh r05n_c4 && cat gpurun_out/r05n_c1_probe.txt gpurun_out/r05n_c1_eval.txt gpurun_out/r05n_c4_probe.txt gpurun_out/r05n_c4_eval.txt
