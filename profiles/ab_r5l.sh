# Round 5 probe (l): k_vocab_2p's pass order — the first pass over K takes ~22 us, the second
# ~9 (chain_trace marks).  Swapped order (second half of K first; probe build, not
# bit-compatible) tells a pass-order / start-up effect from a K-half one
T=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
V=$PWD/whisper.coreml_amd/lib/libwhisper_hip_vs.so
for rep in 1 2; do
  WHISPER_HIP_LIB=$T timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctl_t_$rep.txt 2>&1 || exit 1
  WHISPER_HIP_LIB=$V timeout -k 10 120 python profiles/chain_trace.py 20 8 0 > gpurun_out/ctl_v_$rep.txt 2>&1 || exit 1
done
