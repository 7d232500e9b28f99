"""Precision of fp32 dot products emulated on the bf16 MFMA (round-2 plan).

Each fp32 operand is split exactly into three bf16 planes x = x0 + x1 + x2 (round-to-nearest-even);
a.b keeps the six products of order <= 2 (a0b0, a0b1, a1b0, a0b2, a1b1, a2b0) accumulated in fp32.
Compared with the sequential fp32 dot product and with the 3-term variant, error relative to sum|a||b|,
K = 100 (the DeepONet latent width), 20,000 dot products.  Run: python profiles/bf16x6_precision.py
Recorded output (numpy 2.2):
    fp32 seq  mean 1.86e-08 max 1.84e-07
    bf16x6    mean 6.09e-09 max 8.69e-08
    bf16x3    mean 4.52e-07 max 2.34e-06
"""
import numpy as np


def bf16(x):
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)


def split3(x):
    x = x.astype(np.float32)
    a0 = bf16(x)
    r = (x - a0).astype(np.float32)
    a1 = bf16(r)
    a2 = bf16((r - a1).astype(np.float32))
    return a0, a1, a2


def main():
    rng = np.random.default_rng(0)
    K, n = 100, 20000
    A = (rng.standard_normal((n, K)) * 0.5).astype(np.float32)
    B = np.tanh(rng.standard_normal((n, K))).astype(np.float32)
    exact = (A.astype(np.float64) * B.astype(np.float64)).sum(1)
    scale = (np.abs(A.astype(np.float64)) * np.abs(B)).sum(1)
    f32 = np.zeros(n, np.float32)
    for k in range(K):
        f32 = (f32 + A[:, k] * B[:, k]).astype(np.float32)
    a, b = split3(A), split3(B)

    def emu(terms):
        acc = np.zeros(n, np.float32)
        for i, j in terms:
            p = a[i].astype(np.float64) * b[j].astype(np.float64)     # bf16 x bf16 is exact in fp32
            for k in range(K):
                acc = (acc + p[:, k].astype(np.float32)).astype(np.float32)
        return acc

    for name, v in [("fp32 seq", f32), ("bf16x6", emu([(2, 0), (1, 1), (0, 2), (1, 0), (0, 1), (0, 0)])),
                    ("bf16x3", emu([(1, 0), (0, 1), (0, 0)]))]:
        e = np.abs(v.astype(np.float64) - exact) / scale
        print(f"{name:9s} mean {e.mean():.2e} max {e.max():.2e}")


if __name__ == "__main__":
    main()
