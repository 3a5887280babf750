#!/bin/bash
# encoder attention with 2 query row tiles per wave (tuning library, WHISPER_HIP_ENC_RT=2) A/B,
# then config 2 (turbo, one 30 s window) and config 5 (word timestamps) bench lines
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rt in 1 2 1 2; do
  WHISPER_HIP_LIB=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so WHISPER_HIP_ENC_RT=$rt \
    timeout -k 10 200 python3 profiles/enc_chunk_probe.py | sed "s/^/rt $rt: /" >> gpurun_out/enc_rt_${tag}.txt 2>&1 || exit 1
done
cat gpurun_out/enc_rt_${tag}.txt
timeout -k 10 300 python3 bench.py --model turbo --seconds 30 --max-windows 1 > gpurun_out/bench_cfg2_${tag}.json 2> gpurun_out/bench_cfg2_${tag}.err || exit 2
cat gpurun_out/bench_cfg2_${tag}.json
timeout -k 10 400 python3 bench.py --word-timestamps 1 --cpu-baseline 0 > gpurun_out/bench_cfg5_${tag}.json 2> gpurun_out/bench_cfg5_${tag}.err || exit 3
cat gpurun_out/bench_cfg5_${tag}.json
