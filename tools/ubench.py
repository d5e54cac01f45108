"""PPO-update GEMM micro-benchmark: weight-gradient GEMM variants at the PPO minibatch shape."""
import sys
import torch

def t(fn, it=30):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3

dev = "cuda"
M = 24576
for K, N in [(235, 512), (512, 256), (256, 128), (128, 12)]:
    x = torch.randn(M, K, device=dev); dy = torch.randn(M, N, device=dev)
    f = 2 * M * K * N
    base = t(lambda: dy.t() @ x)
    res = [f"dW[{N}x{K}] K={M}: default {base:.0f}us ({f/base/1e6:.0f} TF)"]
    for S in (4, 8, 16):
        fn = lambda: torch.bmm(dy.view(S, M // S, N).transpose(1, 2), x.view(S, M // S, K)).sum(0)
        us = t(fn); res.append(f"bmm-split{S} {us:.0f}us ({f/us/1e6:.0f} TF)")
    fw = t(lambda: x @ torch.randn(K, N, device=dev))
    res.append(f"fwd {fw:.0f}us ({f/fw/1e6:.0f} TF)")
    print("  ".join(res))
for lib in ("cublas", "cublaslt"):
    try:
        torch.backends.cuda.preferred_blas_library(lib)
        x = torch.randn(M, 235, device=dev); dy = torch.randn(M, 512, device=dev)
        us = t(lambda: dy.t() @ x)
        print(f"preferred_blas_library={lib}: dW[512x235] {us:.0f}us")
    except Exception as ex:
        print(lib, "failed", ex)
