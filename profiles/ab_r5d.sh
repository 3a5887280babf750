# Round 5 A/B (d): self-KV reads through 32-bit buffer offsets (slot pre-multiplied in LDS)
# in k_self_attn_qkv / k_self_attn; prev = b00f8a3-era tuning lib (64-bit kv_off chains)
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
P=$PWD/whisper.coreml_amd/lib/libwhisper_hip_prev_tune.so
timeout -k 10 300 python3 profiles/sa_share_probe.py > gpurun_out/sad_new.txt 2>&1 || exit 1
WHISPER_HIP_LIB=$P timeout -k 10 120 python profiles/chain_trace.py 1 8 0 > gpurun_out/ctsa_prev_w1.txt 2>&1 || exit 1
WHISPER_HIP_LIB=$N timeout -k 10 120 python profiles/chain_trace.py 1 8 0 > gpurun_out/ctsa_new_w1.txt 2>&1 || exit 1
WHISPER_HIP_LIB=$P timeout -k 10 120 python profiles/chain_trace.py 20 6 150 > gpurun_out/ctsa_prev_late.txt 2>&1 || exit 1
WHISPER_HIP_LIB=$N timeout -k 10 120 python profiles/chain_trace.py 20 6 150 > gpurun_out/ctsa_new_late.txt 2>&1 || exit 1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_batch.py tests/test_gpu_models.py tests/test_gpu_tail.py tests/test_gpu_micro.py tests/test_gpu_resume.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_d.txt 2>&1 || exit 2
timeout -k 10 300 python3 bench.py --cpu-baseline 0 > gpurun_out/cfg3_d.json 2> gpurun_out/cfg3_d.err || exit 3
timeout -k 10 300 python3 bench.py --model turbo --seconds 30 --max-windows 1 --cpu-baseline 0 > gpurun_out/cfg2_d.json 2> gpurun_out/cfg2_d.err || exit 4
