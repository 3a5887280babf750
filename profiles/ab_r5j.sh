# Round 5 A/B (j): fp16 split-K slabs (WHISPER_HIP_SLAB16=1, tuning build) re-measured after
# the round's issue-side fixes
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for rep in 1 2; do
  WHISPER_HIP_LIB=$N WHISPER_HIP_SLAB16=0 timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctj_0_$rep.txt 2>&1 || exit 1
  WHISPER_HIP_LIB=$N WHISPER_HIP_SLAB16=1 timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctj_1_$rep.txt 2>&1 || exit 1
done
WHISPER_HIP_LIB=$N WHISPER_HIP_SLAB16=0 timeout -k 10 120 python profiles/chain_trace.py 20 6 150 > gpurun_out/ctj_0_late.txt 2>&1 || exit 1
WHISPER_HIP_LIB=$N WHISPER_HIP_SLAB16=1 timeout -k 10 120 python profiles/chain_trace.py 20 6 150 > gpurun_out/ctj_1_late.txt 2>&1 || exit 1
WHISPER_HIP_LIB=$N WHISPER_HIP_SLAB16=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_j.txt 2>&1 || exit 2
