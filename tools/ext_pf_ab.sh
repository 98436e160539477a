#!/bin/bash
# GPU box (round 5): k_extend cell loop reading two columns ahead -- extension / parity tests on the new library,
# then lone-launch C3 (2 rounds) and C4 (1) alternating with the previous build (tools/bin/libbsq_h.so).
tag=${1:-extpf}
mkdir -p gpurun_out/$tag
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_configs.py tests/test_gpu_long_reads.py tests/test_gpu_c4.py > gpurun_out/$tag/tests.log 2>&1
rc=$?; tail -3 gpurun_out/$tag/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs.sh $tag c3 1 2 tools/bin/libbsq_h.so && bash tools/ab_libs.sh $tag c4 1 1 tools/bin/libbsq_h.so
