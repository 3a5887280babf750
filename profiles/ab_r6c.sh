# Round 6 (c): the selection's window-level arrival (k_logit_part<..., WIN>: one counter per
# window, the row combines and the merge in the last slice's workgroup, candidates in LDS;
# WHISPER_HIP_LP_WIN=1) vs the row-then-window arrivals (=0), tuning lib, chain traces at 20
# windows (large-v3) and one window (turbo, config 2); then the selection's parity tests
# (shipped lib) and the config-2 bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for rep in 1 2; do
  for v in 0 1; do
    WHISPER_HIP_LIB=$N WHISPER_HIP_LP_WIN=$v timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctc_${v}_$rep.txt 2>&1 || exit 1
    CT_MODEL=turbo WHISPER_HIP_LIB=$N WHISPER_HIP_LP_WIN=$v timeout -k 10 120 python profiles/chain_trace.py 1 10 0 > gpurun_out/ctc1_${v}_$rep.txt 2>&1 || exit 1
  done
done
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_tail.py tests/test_gpu_beam_options.py tests/test_gpu_sampling.py tests/test_gpu_repeat.py tests/test_gpu_resume.py "tests/test_gpu_batch.py::test_batch_invariance_fp16" -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_c.txt 2>&1 || exit 2
tail -3 gpurun_out/tests_c.txt
timeout -k 10 300 python3 bench.py --model turbo --seconds 30 --max-windows 1 --cpu-baseline 0 > gpurun_out/cfg2_c.json 2> gpurun_out/cfg2_c.err || exit 3
cat gpurun_out/cfg2_c.json
