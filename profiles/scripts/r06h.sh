#!/bin/bash
# Round 6: PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes) and SQ counters of the gradient-only evaluation at 16
# chains with and without the two-chain T_t units (gram_pair2 = 1 / 0).
GRAD=1 OPT=gram_pair2=1 bash profiles/scripts/traffic_probe.sh r06h_p1 && \
GRAD=1 OPT=gram_pair2=0 bash profiles/scripts/traffic_probe.sh r06h_p0 && \
OPT=gram_pair2=1 bash profiles/scripts/pmc_sq_grad.sh r06h_p1 && \
OPT=gram_pair2=0 bash profiles/scripts/pmc_sq_grad.sh r06h_p0
