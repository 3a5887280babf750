# Round 6 (d): the in-kernel query projection's load order (WHISPER_HIP_XQV 0 / 1 / 2,
# wh_kernels.hip xq_project) traced per phase at 20 / 15 / 2 windows; chain traces and
# bench lines with the split-K query slabs (WHISPER_HIP_XQP=0) against variant 2, same box,
# alternated; then the parity tests the change touches (shipped lib: variant 2).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for v in 0 1 2; do
  WHISPER_HIP_LIB=$N WHISPER_HIP_XQV=$v timeout -k 10 120 python profiles/xattn_trace.py 20,15,2 > gpurun_out/xtd_${v}.txt 2>&1 || exit 1
done
for rep in 1 2; do
  WHISPER_HIP_LIB=$N WHISPER_HIP_XQP=0 timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctd_p0_$rep.txt 2>&1 || exit 1
  WHISPER_HIP_LIB=$N WHISPER_HIP_XQV=2 timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctd_v2_$rep.txt 2>&1 || exit 1
done
WHISPER_HIP_LIB=$N WHISPER_HIP_XQP=0 timeout -k 10 120 python profiles/chain_trace.py 20 8 150 > gpurun_out/ctd_p0_late.txt 2>&1 || exit 1
WHISPER_HIP_LIB=$N WHISPER_HIP_XQV=2 timeout -k 10 120 python profiles/chain_trace.py 20 8 150 > gpurun_out/ctd_v2_late.txt 2>&1 || exit 1
for rep in 1 2; do
  for v in 0 1; do
    WHISPER_HIP_LIB=$N WHISPER_HIP_XQP=$v timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 --latency 0 > gpurun_out/bd_p${v}_$rep.json 2> gpurun_out/bd_p${v}_$rep.err || exit 3
    python3 -c "import json; d=json.load(open('gpurun_out/bd_p${v}_$rep.json')); print('XQP=$v rep $rep', d['value'], d['mean_token_ms_batch'], d['roofline_cross_attn']['ms_per_launch'], d['roofline_step']['ms_per_launch'])"
  done
done
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_batch.py tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_d.txt 2>&1 || exit 2
tail -3 gpurun_out/tests_d.txt
