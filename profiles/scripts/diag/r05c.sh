timeout -k 10 60 ./_ab/mfma_acc_bias > gpurun_out/r05c_mfma_bias.txt 2>&1 && cat gpurun_out/r05c_mfma_bias.txt && \
timeout -k 10 300 python -u profiles/scripts/diag/gram_fit_err.py 1e-2 3 > gpurun_out/r05c_gram_fit_err.txt 2>&1; cat gpurun_out/r05c_gram_fit_err.txt
