timeout -k 10 300 python -u profiles/scripts/diag/gram_parts_err.py 1e-2 > gpurun_out/r05d_gram_parts.txt 2>&1; cat gpurun_out/r05d_gram_parts.txt
