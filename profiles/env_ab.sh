#!/bin/bash
# A/B of environment settings on one library build: profiles/env_ab.sh "<envA>" "<envB>" [bench args]
# alternates A B A B; one JSON line per run in gpurun_out/envab_*.json
set -o pipefail
ea=$1; eb=$2; shift 2
mkdir -p gpurun_out
for i in 1 2; do
  for tag in a b; do
    envs=$ea; [ $tag = b ] && envs=$eb
    env $envs timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 "$@" \
      > gpurun_out/envab_${tag}${i}.json 2> gpurun_out/envab_${tag}${i}.err || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/envab_${tag}${i}.json')); print('$tag$i', d['value'], d['p50_token_ms'], d['p50_token_ms_batch'], d['roofline_cross_attn']['ms_per_launch'], d['roofline_step']['ms_per_launch'], d['encoder_ms_per_window'])"
  done
done
