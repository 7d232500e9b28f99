# One GPU check of the tree: the -m gpu suite, then (when no test crashed) the bench line. TAG names the outputs.
TAG=${TAG:-r04}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.txt
if [ $rc -le 1 ]; then timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err; echo "bench rc=$?"; fi
