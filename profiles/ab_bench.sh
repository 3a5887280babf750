#!/bin/bash
# A/B of two library builds on the same box: profiles/ab_bench.sh <libA> <libB> [bench args]
# alternates A B A B so box drift shows; one JSON line per run in gpurun_out/ab_*.json
set -o pipefail
a=$1; b=$2; shift 2
mkdir -p gpurun_out
for i in 1 2; do
  for tag in a b; do
    lib=$a; [ $tag = b ] && lib=$b
    WHISPER_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 "$@" \
      > gpurun_out/ab_${tag}${i}.json 2> gpurun_out/ab_${tag}${i}.err || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_${tag}${i}.json')); print('$tag$i', d['value'], d['p50_token_ms'], d['roofline']['ms_per_launch'], d['roofline_cross_attn']['ms_per_launch'], d['roofline_step']['ms_per_launch'], d['encoder_ms_per_window'])"
  done
done
