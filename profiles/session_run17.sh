#!/bin/bash
# GPU suite, single-window step profile, config 2 and config 3 bench lines
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_${tag}.log 2>&1 || { tail -30 gpurun_out/gpu_tests_${tag}.log; exit 1; }
tail -3 gpurun_out/gpu_tests_${tag}.log
bash profiles/profile_step.sh w1_${tag} --windows 1 --steps 32 || exit 2
head -3 gpurun_out/step_w1_${tag}_plain.txt
timeout -k 10 300 python3 bench.py --model turbo --seconds 30 --max-windows 1 > gpurun_out/bench_cfg2_${tag}.json 2> gpurun_out/bench_cfg2_${tag}.err || exit 3
cat gpurun_out/bench_cfg2_${tag}.json
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${tag}.json 2> gpurun_out/bench_${tag}.err || exit 4
cat gpurun_out/bench_${tag}.json
