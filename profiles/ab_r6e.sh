# Round 6 (e): the single-window step's cross-attention query projected in the kernel with
# the LayerNorm (WHISPER_HIP_XQP1=1, no cross-q k_proj1 launch) vs the k_proj1 launch (=0):
# chain traces (turbo and large-v3, one window), config-2 and large-v3 one-window bench lines
# alternated on one box (tuning lib); then the single-window parity tests (shipped lib).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for rep in 1 2; do
  for v in 0 1; do
    CT_MODEL=turbo WHISPER_HIP_LIB=$N WHISPER_HIP_XQP1=$v timeout -k 10 120 python profiles/chain_trace.py 1 10 0 > gpurun_out/cte_t_${v}_$rep.txt 2>&1 || exit 1
  done
done
for v in 0 1; do
  WHISPER_HIP_LIB=$N WHISPER_HIP_XQP1=$v timeout -k 10 120 python profiles/chain_trace.py 1 10 0 > gpurun_out/cte_l_${v}.txt 2>&1 || exit 1
done
for rep in 1 2; do
  for v in 0 1; do
    WHISPER_HIP_LIB=$N WHISPER_HIP_XQP1=$v timeout -k 10 300 python3 bench.py --model turbo --seconds 30 --max-windows 1 --steps 3 --cpu-baseline 0 > gpurun_out/be2_${v}_$rep.json 2> gpurun_out/be2_${v}_$rep.err || exit 3
    python3 -c "import json; d=json.load(open('gpurun_out/be2_${v}_$rep.json')); print('cfg2 XQP1=$v rep $rep', d['value'], d['p50_token_ms'], d['latency_1window']['step_graph_ms_1window'])"
  done
done
for v in 0 1; do
  WHISPER_HIP_LIB=$N WHISPER_HIP_XQP1=$v timeout -k 10 300 python3 bench.py --seconds 30 --max-windows 1 --steps 2 --cpu-baseline 0 > gpurun_out/bel_${v}.json 2> gpurun_out/bel_${v}.err || exit 3
  python3 -c "import json; d=json.load(open('gpurun_out/bel_${v}.json')); print('large-v3 1 window XQP1=$v', d['value'], d['p50_token_ms'], d['latency_1window']['step_graph_ms_1window'])"
done
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_tail.py tests/test_gpu_batch.py tests/test_gpu_models.py tests/test_gpu_beam_options.py tests/test_gpu_resume.py tests/test_gpu_repeat.py -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_e.txt 2>&1 || exit 2
tail -3 gpurun_out/tests_e.txt
