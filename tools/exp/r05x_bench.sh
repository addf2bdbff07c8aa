set -e
mkdir -p gpurun_out/r05x
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05x/smoke.txt 2>&1
timeout -k 10 900 python3 -u bench.py > gpurun_out/r05x/bench.json 2> gpurun_out/r05x/bench.err
