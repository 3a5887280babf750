# Round 6 (g): the W_q head slices prefetched into each XCD's L2 by the k_resid_ln ahead of
# the step cross-attention (WHISPER_HIP_XQ_PF=1) vs not (=0): chain traces (20 windows, early
# and after 150 tokens) and bench lines alternated on one box (tuning lib); then the parity
# tests the change touches (shipped lib).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for rep in 1 2; do
  for v in 0 1; do
    WHISPER_HIP_LIB=$N WHISPER_HIP_XQ_PF=$v timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctg_${v}_$rep.txt 2>&1 || exit 1
  done
done
for v in 0 1; do
  WHISPER_HIP_LIB=$N WHISPER_HIP_XQ_PF=$v timeout -k 10 120 python profiles/chain_trace.py 20 8 150 > gpurun_out/ctg_${v}_late.txt 2>&1 || exit 1
done
for rep in 1 2; do
  for v in 0 1; do
    WHISPER_HIP_LIB=$N WHISPER_HIP_XQ_PF=$v timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 --latency 0 > gpurun_out/bg_${v}_$rep.json 2> gpurun_out/bg_${v}_$rep.err || exit 3
    python3 -c "import json; d=json.load(open('gpurun_out/bg_${v}_$rep.json')); print('XQ_PF=$v rep $rep', d['value'], d['mean_token_ms_batch'], d['roofline_step']['ms_per_launch'])"
  done
done
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_batch.py tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_g.txt 2>&1 || exit 2
tail -3 gpurun_out/tests_g.txt
