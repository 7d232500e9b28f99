import torch, numpy as np
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
p = torch.randn(1 << 20, generator=g).to(dev); q = torch.randn(1 << 20, generator=g).to(dev)
h = 0.5 * 1.2345e-4
t = torch.add(p, q, alpha=h).cpu().numpy().astype(np.float64)
pn, qn = p.cpu().numpy(), q.cpu().numpy()
hf = np.float32(h)
two = (pn + (hf * qn).astype(np.float32)).astype(np.float32)
fma = (pn.astype(np.float64) + np.float64(hf) * qn.astype(np.float64)).astype(np.float32)
print("torch.add alpha: equal to two roundings", np.mean(t == two), " equal to fma", np.mean(t == fma))
t2 = (p + h * q).cpu().numpy()
print("p + h*q (two kernels): equal two roundings", np.mean(t2 == two))
