#!/bin/bash
# in-situ k_proj tiling sweep (WHISPER_HIP_PROJ_FORCE="N:K:cfg"), one bench line per setting
set -o pipefail
mkdir -p gpurun_out
run() {
  tag=$1; force=$2
  WHISPER_HIP_PROJ_FORCE=$force timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 --latency 0 \
    > gpurun_out/sweep_$tag.json 2> gpurun_out/sweep_$tag.err || return 1
  python3 -c "import json; d=json.load(open('gpurun_out/sweep_$tag.json')); print('$tag', '$force', d['value'], d['p50_token_ms_batch'], d['roofline']['ms_per_launch'], d['roofline_step']['ms_per_launch'])"
}
for spec in "$@"; do
  tag=${spec%%=*}; force=${spec#*=}
  run "$tag" "$force" || exit 1
done
