#!/bin/bash
# decode parity subset, then bench B and C (with the pipelined leg)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out/r04v; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_golden.py tests/test_gpu_decode.py tests/test_gpu_fullsize.py tests/test_gpu_host.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/b.log').read().strip().splitlines()[-1]); print('B', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_all'], d['pipelined']['value'])"
timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline --config C > $OUT/c.log 2>&1 || { tail -20 $OUT/c.log; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c.log').read().strip().splitlines()[-1]); print('C', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_all'], d['pipelined']['value'])"
