for C in 1 16; do timeout -k 10 300 python -u profiles/scripts/diag/gram_parts_err.py 1e-2 $C || exit 1; done > gpurun_out/r05d_gram_parts.txt 2>&1; cat gpurun_out/r05d_gram_parts.txt
