# Round 5 probe (m): k_logit_part<16, 8, fused, merge> at 67 VGPRs runs 3 workgroups per CU
# (1600 workgroups at 100 rows: 3 rounds); capped at 64 (probe build -DWH_LP_OCC=2, 3 VGPRs
# spilled) it runs 4 (2 rounds)
T=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
L=$PWD/whisper.coreml_amd/lib/libwhisper_hip_lo.so
for rep in 1 2; do
  WHISPER_HIP_LIB=$T timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctm_t_$rep.txt 2>&1 || exit 1
  WHISPER_HIP_LIB=$L timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctm_l_$rep.txt 2>&1 || exit 1
done
WHISPER_HIP_LIB=$T timeout -k 10 120 python profiles/chain_trace.py 20 6 150 > gpurun_out/ctm_t_late.txt 2>&1 || exit 1
WHISPER_HIP_LIB=$L timeout -k 10 120 python profiles/chain_trace.py 20 6 150 > gpurun_out/ctm_l_late.txt 2>&1 || exit 1
