"""Forward / input-gradient GEMM variants at the PPO minibatch shape (M = 24576 rows, 2 nets)."""
import torch


def t(fn, it=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


dev = "cuda"
M = 24576
for K in (235, 236, 240, 256):
    X = torch.randn(M, K, device=dev)
    W = torch.randn(1024, K, device=dev)
    out2 = torch.empty(2, M, 512, device=dev)
    out1 = torch.empty(M, 1024, device=dev)
    f = 2 * M * K * 1024

    def two():
        torch.mm(X, W[:512].t(), out=out2[0])
        torch.mm(X, W[512:].t(), out=out2[1])
    a = t(two)
    b = t(lambda: torch.mm(X, W.t(), out=out1))
    c = t(lambda: torch.bmm(X.unsqueeze(0).expand(2, M, K), W.view(2, 512, K).transpose(1, 2), out=out2))
    print(f"L1 K={K}: 2x mm {a:.0f}us ({f/a/1e6:.0f} TF)  1x mm N=1024 {b:.0f}us ({f/b/1e6:.0f} TF)  "
          f"bmm(expand) {c:.0f}us ({f/c/1e6:.0f} TF)")
Y = torch.randn(2, M, 512, device=dev)
W2 = torch.randn(2, 256, 512, device=dev)
o = torch.empty(2, M, 256, device=dev)
f = 2 * 2 * M * 512 * 256
a = t(lambda: torch.bmm(Y, W2.transpose(1, 2), out=o))
Yi = torch.randn(M, 1024, device=dev)
b = t(lambda: torch.bmm(Yi.view(M, 2, 512).permute(1, 0, 2), W2.transpose(1, 2), out=o))
print(f"L2 bmm net-major {a:.0f}us ({f/a/1e6:.0f} TF); interleaved input {b:.0f}us ({f/b/1e6:.0f} TF)")
