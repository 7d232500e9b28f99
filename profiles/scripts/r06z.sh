#!/bin/bash
# Round 6 final tree: PMC HBM traffic of the gradient-only evaluation at 16 chains (FETCH_SIZE / WRITE_SIZE passes),
# then the round check (GPU suite, smoke, bench line, rocprofv3 kernel stats).
GRAD=1 bash profiles/scripts/traffic_probe.sh r06z_grad && TAG=r06z AB=0 bash profiles/scripts/r06_round.sh
