# Round 5 (h): wide logit stores as the default (k_vocab_2p, k_vocab1, k_vocab_small):
# GPU suite, smoke, config 3 with the CPU baseline, config 2
bash profiles/gpu_session.sh r5h tests smoke cfg3 cfg2
