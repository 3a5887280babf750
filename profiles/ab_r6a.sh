# Round 6 A/B (a): the cross-attention query projected inside k_xattn_seg (WHISPER_HIP_XQP=1,
# no cross-q k_proj launch) vs the split-K projection + fp16 slabs (=0), tuning lib, 20 windows
# x beam 5, early and at 150 tokens; then the parity tests the change touches (shipped lib)
# and one config-3 bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for rep in 1 2; do
  for v in 0 1; do
    WHISPER_HIP_LIB=$N WHISPER_HIP_XQP=$v timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/cta_${v}_$rep.txt 2>&1 || exit 1
  done
done
for v in 0 1; do
  WHISPER_HIP_LIB=$N WHISPER_HIP_XQP=$v timeout -k 10 120 python profiles/chain_trace.py 20 8 150 > gpurun_out/cta_${v}_late.txt 2>&1 || exit 1
done
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_batch.py tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_a.txt 2>&1 || exit 2
tail -3 gpurun_out/tests_a.txt
timeout -k 10 300 python3 bench.py --cpu-baseline 0 > gpurun_out/cfg3_a.json 2> gpurun_out/cfg3_a.err || exit 3
cat gpurun_out/cfg3_a.json
