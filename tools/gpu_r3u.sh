#!/bin/bash
# quick: split tests, layer times, bench without the CPU baseline and extras
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r3u}
mkdir -p $OUT
export TMPDIR=/tmp
NO_BENCH=1 bash tools/gpu_r3j.sh ${1:-r3u} | tail -20 || exit $?
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-extra > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc"; grep "bench " $OUT/bench.err | head -8
python3 -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['hot_path']['op_ms'])"
exit $rc
