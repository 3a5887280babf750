#!/bin/bash
# final round session: GPU suite, graph-mode step profiles, default bench line, and the
# rocprofv3 --kernel-trace --stats profile of the bench command in eager mode (the mode the
# bench's roofline events time k_proj in; tuning library for WHISPER_HIP_EAGER)
#   profiles/session_final.sh <tag>
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_${tag}.log 2>&1 || { tail -30 gpurun_out/gpu_tests_${tag}.log; exit 1; }
tail -3 gpurun_out/gpu_tests_${tag}.log
bash profiles/profile_step.sh w20_${tag} --windows 20 --steps 16 --encode 4 || exit 2
bash profiles/profile_step.sh w1_${tag} --windows 1 --steps 32 || exit 3
head -3 gpurun_out/step_w20_${tag}_plain.txt gpurun_out/step_w1_${tag}_plain.txt
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${tag}.json 2> gpurun_out/bench_${tag}.err || exit 4
cat gpurun_out/bench_${tag}.json
WHISPER_HIP_LIB=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so WHISPER_HIP_EAGER=1 timeout -k 10 400 \
  rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench_${tag}_eager -o run -- \
  python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/prof_bench_${tag}_eager.log 2>&1 || exit 5
db=$(ls gpurun_out/prof_bench_${tag}_eager/*/run_results.db gpurun_out/prof_bench_${tag}_eager/run_results.db 2>/dev/null | head -1)
python3 profiles/summarize_db.py $db 40 gpurun_out/bench_${tag}_eager_kernel_stats.csv > gpurun_out/bench_${tag}_eager_summary.txt
head -20 gpurun_out/bench_${tag}_eager_summary.txt
ls gpurun_out/prof_bench_${tag}_eager/ | head
