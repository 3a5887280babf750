#!/bin/bash
# final config 2 / 5 / 4 (N = 1) lines on the committed tree
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --model turbo --seconds 30 --max-windows 1 > gpurun_out/bench_cfg2_${tag}.json 2> gpurun_out/bench_cfg2_${tag}.err || exit 12
cat gpurun_out/bench_cfg2_${tag}.json
timeout -k 10 400 python3 bench.py --word-timestamps 1 --cpu-baseline 0 > gpurun_out/bench_cfg5_${tag}.json 2> gpurun_out/bench_cfg5_${tag}.err || exit 13
cat gpurun_out/bench_cfg5_${tag}.json
timeout -k 10 500 python3 bench.py --sharded-file 1 --seconds 3600 --verify 1 --cpu-baseline 0 --steps 1 > gpurun_out/bench_cfg4_${tag}.json 2> gpurun_out/bench_cfg4_${tag}.err || exit 14
cat gpurun_out/bench_cfg4_${tag}.json
