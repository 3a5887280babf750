# Round 5 A/B (k): the QKV projection's split-K slabs as fp16 too (WHISPER_HIP_SLAB16_QKV=1,
# tuning build; k_self_attn_qkv<fp16, pipe, half slabs>) vs fp32 (=0), 20 windows x beam 5
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for rep in 1 2; do
  WHISPER_HIP_LIB=$N WHISPER_HIP_SLAB16_QKV=0 timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctk_0_$rep.txt 2>&1 || exit 1
  WHISPER_HIP_LIB=$N WHISPER_HIP_SLAB16_QKV=1 timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctk_1_$rep.txt 2>&1 || exit 1
done
WHISPER_HIP_LIB=$N WHISPER_HIP_SLAB16_QKV=0 timeout -k 10 120 python profiles/chain_trace.py 20 6 150 > gpurun_out/ctk_0_late.txt 2>&1 || exit 1
WHISPER_HIP_LIB=$N WHISPER_HIP_SLAB16_QKV=1 timeout -k 10 120 python profiles/chain_trace.py 20 6 150 > gpurun_out/ctk_1_late.txt 2>&1 || exit 1
WHISPER_HIP_LIB=$N WHISPER_HIP_SLAB16_QKV=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_k.txt 2>&1 || exit 2
