"""Library GEMM (torch.matmul -> hipBLASLt, fp16, fp32 accumulate) at the encoder's GEMM
shapes, for comparison with k_gemm_256 (profiles/r02/gemm_bench.txt: same M, N, K).
Plain GEMM only: the library has no fused epilogue (bias / GELU / residual / head split),
so this is a lower bound on what the library path would cost."""
import torch

shapes = {"qkv": (30000, 1280, 3840), "out": (30000, 1280, 1280), "fc1": (30000, 1280, 5120),
          "fc2": (30000, 5120, 1280), "one-window": (1500, 1280, 5120), "1w-out": (1500, 1280, 1280),
          "1w-fc2": (1500, 5120, 1280)}
torch.manual_seed(0)
for name, (M, K, N) in shapes.items():
    a = (torch.rand(M, K, device="cuda", dtype=torch.float16) * 2 - 1)
    w = (torch.rand(N, K, device="cuda", dtype=torch.float16) * 2 - 1)
    for _ in range(5):
        torch.matmul(a, w.t())
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    st.record()
    for _ in range(reps):
        torch.matmul(a, w.t())
    en.record()
    torch.cuda.synchronize()
    ms = st.elapsed_time(en) / reps
    print(f"{name:10s} M {M} N {N} K {K}: {ms * 1e3:8.1f} us  {2 * M * N * K / ms / 1e9:7.1f} TFLOP/s", flush=True)
