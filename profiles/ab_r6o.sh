# Round 6 (o): the single-window cross-attention query projected inside k_xattn_seg with the
# projection split over each pair's 8 workgroups (QV 6, tuning WHISPER_HIP_XQP1=2) against the
# shipped cross-q k_proj1 launch: parity suites of the one-window path on the tuning build with
# the split form, then turbo / large-v3 one-window chain traces and config-2 lines, alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
WHISPER_HIP_LIB=$N WHISPER_HIP_XQP1=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_tail.py > gpurun_out/o_tests_tail.txt 2>&1 || exit 1
WHISPER_HIP_LIB=$N WHISPER_HIP_XQP1=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_batch.py tests/test_gpu_models.py > gpurun_out/o_tests.txt 2>&1 || exit 2
for rep in 1 2; do
  for v in 0 2; do
    CT_MODEL=turbo WHISPER_HIP_LIB=$N WHISPER_HIP_XQP1=$v timeout -k 10 150 python profiles/chain_trace.py 1 10 0 > gpurun_out/cto_turbo_${v}_$rep.txt 2>&1 || exit 3
    WHISPER_HIP_LIB=$N WHISPER_HIP_XQP1=$v timeout -k 10 150 python profiles/chain_trace.py 1 10 0 > gpurun_out/cto_v3_${v}_$rep.txt 2>&1 || exit 4
  done
done
for v in 2 0; do
  WHISPER_HIP_LIB=$N WHISPER_HIP_XQP1=$v timeout -k 10 300 python bench.py --model turbo --seconds 30 --max-windows 1 --cpu-baseline 0 > gpurun_out/o_c2_$v.json 2>/dev/null || exit 5
done
