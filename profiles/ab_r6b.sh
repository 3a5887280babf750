# Round 6 (b): phase marks of the step cross-attention with the in-kernel query projection
# (WHISPER_HIP_XQP=1) against the split-K query slabs (=0), tuning lib, 20 and 15 windows;
# then the parity tests the change touches (shipped lib) and one config-3 bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for v in 0 1; do
  WHISPER_HIP_LIB=$N WHISPER_HIP_XQP=$v timeout -k 10 120 python profiles/xattn_trace.py 20,15,2 > gpurun_out/xtb_${v}.txt 2>&1 || exit 1
done
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_batch.py tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_b.txt 2>&1 || exit 2
tail -3 gpurun_out/tests_b.txt
timeout -k 10 300 python3 bench.py --cpu-baseline 0 > gpurun_out/cfg3_b.json 2> gpurun_out/cfg3_b.err || exit 3
cat gpurun_out/cfg3_b.json
