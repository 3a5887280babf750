T=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
X=$PWD/whisper.coreml_amd/lib/libwhisper_hip_xslow.so
for v in 0 2 3; do WHISPER_HIP_LIB=$T WHISPER_HIP_V2P8=$v timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ct_new_$v.txt 2>&1 || exit 1; done
WHISPER_HIP_LIB=$X timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ct_xslow.txt 2>&1 || exit 1
WHISPER_HIP_LIB=$T timeout -k 10 120 python profiles/chain_trace.py 1 8 0 > gpurun_out/ct_new_w1.txt 2>&1 || exit 1
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_batch.py tests/test_gpu_tail.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_xfast.txt 2>&1 || exit 2
timeout -k 10 300 python3 bench.py --cpu-baseline 0 > gpurun_out/cfg3_xfast.json 2> gpurun_out/cfg3_xfast.err || exit 3
