# Round 6 (b + c) on one box: (b) phase marks of the step cross-attention with the in-kernel
# query projection (WHISPER_HIP_XQP=1) vs the split-K query slabs (=0); (c) the selection's
# window-level arrival (WHISPER_HIP_LP_WIN=1) vs row-then-window arrivals (=0), chain traces
# at 20 windows (large-v3) and one window (turbo); then the whole GPU suite (shipped lib:
# both changes on) and the config-3 / config-2 bench lines.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for v in 0 1; do
  WHISPER_HIP_LIB=$N WHISPER_HIP_XQP=$v timeout -k 10 120 python profiles/xattn_trace.py 20,15,2 > gpurun_out/xtb_${v}.txt 2>&1 || exit 1
done
for rep in 1 2; do
  for v in 0 1; do
    WHISPER_HIP_LIB=$N WHISPER_HIP_LP_WIN=$v timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctc_${v}_$rep.txt 2>&1 || exit 1
    CT_MODEL=turbo WHISPER_HIP_LIB=$N WHISPER_HIP_LP_WIN=$v timeout -k 10 120 python profiles/chain_trace.py 1 10 0 > gpurun_out/ctc1_${v}_$rep.txt 2>&1 || exit 1
  done
done
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_bc.txt 2>&1 || exit 2
tail -3 gpurun_out/tests_bc.txt
timeout -k 10 300 python3 bench.py --cpu-baseline 0 > gpurun_out/cfg3_bc.json 2> gpurun_out/cfg3_bc.err || exit 3
timeout -k 10 300 python3 bench.py --model turbo --seconds 30 --max-windows 1 --cpu-baseline 0 > gpurun_out/cfg2_bc.json 2> gpurun_out/cfg2_bc.err || exit 4
cat gpurun_out/cfg3_bc.json gpurun_out/cfg2_bc.json
