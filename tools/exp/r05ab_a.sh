set -e
mkdir -p gpurun_out/r05ab
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r05ab/tests.txt 2>&1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05ab/smoke.txt 2>&1
timeout -k 10 600 python3 -u bench.py > gpurun_out/r05ab/bench.json 2> gpurun_out/r05ab/bench.err
