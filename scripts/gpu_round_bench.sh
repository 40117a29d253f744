#!/bin/bash
# Round-end measurement set: parity tests, smoke, and the bench lines
# committed under profiles/ (configs 2/3/4, host-array API, end-to-end).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/b_c2.json 2> gpurun_out/b_c2.err || exit $?
timeout -k 10 300 python bench.py --config 3 > gpurun_out/b_c3.json 2> gpurun_out/b_c3.err || exit $?
timeout -k 10 300 python bench.py --config 4 > gpurun_out/b_c4.json 2> gpurun_out/b_c4.err || exit $?
timeout -k 10 300 python bench.py --host-arrays --no-cpu-baseline > gpurun_out/b_c2_host.json 2> gpurun_out/b_c2_host.err || exit $?
timeout -k 10 300 python bench.py --e2e --no-cpu-baseline > gpurun_out/b_c2_e2e.json 2> gpurun_out/b_c2_e2e.err || exit $?
