# Probes of one GPU call: chain groups on separate streams (probe_groups.py), then a rocprofv3 kernel-stats pass over
# the bench (C = 16, short). TAG names the outputs.
TAG=${TAG:-r04p}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 300 python -u profiles/scripts/probes/probe_groups.py --groups 1 2 4 --steps 20 --reps 2 > gpurun_out/${TAG}_groups.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/${TAG}_ks -o s -- \
    python3 $ROOT/bench.py --steps 5 --warmup 2 --ess-steps 0 --cpu-seconds 0 --no-side-legs > $ROOT/gpurun_out/${TAG}_ks.log 2>&1
