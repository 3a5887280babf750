N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
WHISPER_HIP_LIB=$N timeout -k 10 120 python profiles/chain_trace.py 1 8 0 > gpurun_out/ctd_w1.txt 2>&1 || exit 1
WHISPER_HIP_LIB=$N timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctd_w20.txt 2>&1 || exit 1
