# Round 6 (i): W_q in the in-kernel query projection's fragment order (WHISPER_HIP_XQ_FRAG=1:
# every wave load 1 KB contiguous) vs the [n][n] rows (=0): phase marks, chain traces at 20
# windows, and the single-window form (WHISPER_HIP_XQP1=1) with it, one box (tuning lib); then
# the parity tests (shipped lib).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for v in 0 1; do
  WHISPER_HIP_LIB=$N WHISPER_HIP_XQ_FRAG=$v timeout -k 10 120 python profiles/xattn_trace.py 20,15,2 > gpurun_out/xti_${v}.txt 2>&1 || exit 1
done
for rep in 1 2; do
  for v in 0 1; do
    WHISPER_HIP_LIB=$N WHISPER_HIP_XQ_FRAG=$v timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/cti_${v}_$rep.txt 2>&1 || exit 1
  done
done
for v in 0 1; do
  CT_MODEL=turbo WHISPER_HIP_LIB=$N WHISPER_HIP_XQP1=$v timeout -k 10 120 python profiles/chain_trace.py 1 10 0 > gpurun_out/cti1_${v}.txt 2>&1 || exit 1
done
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_batch.py tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_i.txt 2>&1 || exit 2
tail -3 gpurun_out/tests_i.txt
