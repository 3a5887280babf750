#!/bin/bash
# Library A/B on one box: profiles/lib_ab.sh <libA.so> <libB.so> — config 3 (no CPU
# baseline) and config 2 with each library (WHISPER_HIP_LIB), alternated A B A B; one
# line per run: xRT, p50 token ms, cross-attention us, step graph ms, encoder ms / window.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
la=$1; lb=$2
show() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['p50_token_ms'], round(d['roofline_cross_attn']['ms_per_launch']*1e3,2), d['roofline_step']['ms_per_launch'], d['encoder_ms_per_window'])" "$1" "$2"; }
for i in 1 2; do
  for tag in a b; do
    lib=$la; [ $tag = b ] && lib=$lb
    WHISPER_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --cpu-baseline 0 > gpurun_out/libab_c3_$tag$i.json 2> gpurun_out/libab_c3_$tag$i.err || exit 2
    show gpurun_out/libab_c3_$tag$i.json "cfg3 $tag$i" || exit 3
    WHISPER_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --model turbo --seconds 30 --max-windows 1 --cpu-baseline 0 \
      > gpurun_out/libab_c2_$tag$i.json 2> gpurun_out/libab_c2_$tag$i.err || exit 4
    show gpurun_out/libab_c2_$tag$i.json "cfg2 $tag$i" || exit 5
  done
done
