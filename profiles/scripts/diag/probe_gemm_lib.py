"""Probe: how fast do library bf16 GEMMs run at the Gram-form contraction shapes (the 6 bf16 products of a
bf16x6 dot product stacked along K)? Upper-bound reference for the hand-written kernel; not product code."""
import time
import torch

dev = torch.device("cuda", 0)
C, W, N, P = 16, 100, 1000, 10201


def bench(f, n=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


for (M, K, NN, tag) in [(P, N, C * W, "T_t = y^T Zb"), (N, P, C * W, "T_b = y Zt")]:
    for kk in (1, 6):
        a = torch.randn(M, K * kk, device=dev).to(torch.bfloat16)
        b = torch.randn(K * kk, NN, device=dev).to(torch.bfloat16)
        bt = b.t().contiguous()
        ms = bench(lambda: a @ b)
        ms2 = bench(lambda: a @ bt.t())
        fl = 2.0 * M * K * kk * NN
        print(f"{tag} K'={K*kk}: a@b {ms:.4f} ms ({fl/ms/1e9:.0f} TF/s bf16)  a@bt.t() {ms2:.4f} ms ({fl/ms2/1e9:.0f})",
              flush=True)
    a = torch.randn(M, K, device=dev)
    b = torch.randn(K, NN, device=dev)
    ms = bench(lambda: a @ b)
    print(f"{tag} fp32 sgemm: {ms:.4f} ms ({2.0*M*K*NN/ms/1e9:.0f} TF/s)", flush=True)
    torch.backends.cuda.matmul.allow_tf32 = False
