#!/bin/bash
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03_bpd
PQGPU_LIB=$PWD/abx/libdiag.so timeout -k 10 300 python3 -u tools/diag_binplain.py str_plain > gpurun_out/r03_bpd/str_plain.txt 2>&1 || { tail -20 gpurun_out/r03_bpd/str_plain.txt; exit 1; }
cat gpurun_out/r03_bpd/str_plain.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_binary.py -m gpu \
  > gpurun_out/r03_bpd/pytest.log 2>&1 || { tail -40 gpurun_out/r03_bpd/pytest.log; exit 1; }
tail -2 gpurun_out/r03_bpd/pytest.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_bpd/prof -o run -- \
  python3 tools/bench_suite.py str_plain c3_mixed c4_lineitem str_dict --cpu-budget 0 \
  > gpurun_out/r03_bpd/suite.jsonl 2> gpurun_out/r03_bpd/suite.err || { tail -30 gpurun_out/r03_bpd/suite.err; exit 1; }
cut -c1-200 gpurun_out/r03_bpd/suite.jsonl
python3 tools/seg_kernels.py gpurun_out/r03_bpd/prof/run_kernel_trace.csv --names str_plain,c3,c4_8M,str_dict || true
