import os, sys
sys.argv = ['x']
sys.path[:0] = ['/root/repo', '/root/repo/vi-hmc_amd']
src = open('profiles/scripts/diag/tanh_emul_fit.py').read().split('noises = ')[0].replace('os.path.dirname(__file__)', '"/root/repo/profiles/scripts/diag"'); exec(src)
import torch.nn.functional as F

class LayerRef(TorchDeepONetRef):
    def __init__(self, *a, which=None, noise_ulp=0.0, **k):
        super().__init__(*a, **k)
        self.which = which; self.noise_ulp = noise_ulp; self.rng = np.random.default_rng(0)
    def functional_model(self, params):
        flat = self.mu.clone(); flat[self.idx] = params
        w = self._views(flat)
        nb = len(self.br)
        def act(z, i):
            if self.which is not None and i in self.which:
                return TanhAcc.apply(z)
            if self.noise_ulp:
                h = torch.tanh(z)
                hd = h.detach().numpy()
                u = np.spacing(np.abs(hd).astype(np.float32))
                n = torch.from_numpy((self.rng.standard_normal(hd.shape) * self.noise_ulp * u).astype(np.float32).round(0) if False else (np.round(self.rng.standard_normal(hd.shape) * self.noise_ulp) * u).astype(np.float32))
                return h + n
            return torch.tanh(z)
        xb = self.x1
        for i in range(nb):
            xb = F.linear(xb, *w[i])
            if i < nb - 1: xb = act(xb, i)
        X2 = self.x2
        x_bc = torch.stack([torch.sin(2*np.pi*X2[:,:,1]), torch.sin(4*np.pi*X2[:,:,1]), torch.cos(2*np.pi*X2[:,:,1]), torch.cos(4*np.pi*X2[:,:,1])], dim=2)
        xtr = torch.cat([X2[:,:,0].unsqueeze(dim=2), x_bc], dim=2)
        nt = len(self.tr)
        for i in range(nt):
            xtr = F.linear(xtr, *w[nb+i])
            if i < nt - 1: xtr = act(xtr, i)
        x = torch.einsum("...i,...i->...", xb, xtr)
        return torch.unsqueeze(x, 1) + flat[0]

lay = deeponet_layout(); SD = 1e3
p = deeponet_problem(seed=3, noise=1e-3, mu_noise=0.0)
t0 = p.teacher[p.grad_ind].astype(np.float32)
rng = np.random.default_rng(31)
ths = [t0] + [(t0 * (1 + 1e-6 * rng.standard_normal(t0.size))).astype(np.float32) for _ in range(2)]
g64s = [np_logp_grad(lay, p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, th, 0.0, SD, "NLL", 1.0)[1] for th in ths]
for name, kw in [("all", dict(which=set(range(8)))), ("last(7)", dict(which={7})), ("first7(0-6)", dict(which=set(range(7)))),
                 ("last2(6,7)", dict(which={6,7})), ("rand0.3ulp", dict(noise_ulp=0.3)), ("rand1ulp", dict(noise_ulp=1.0))]:
    m = LayerRef(lay, p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, 0.0, SD, "NLL", 1.0, **kw)
    e = [np.linalg.norm(m.logp_grad(th)[1] - g) / np.linalg.norm(g) for th, g in zip(ths, g64s)]
    print(f"{name:12s} median {np.median(e):.3e} {np.round(e,7).tolist()}", flush=True)

def tanh_cheap_np(x):
    x = x.astype(f32); ax = np.abs(x)
    a = (ax * f32(-2.885390043258667)).astype(f32)
    t = np.exp2(a.astype(np.float64)).astype(f32)
    r = (1.0 / (f32(1) + t).astype(np.float64)).astype(f32)
    y = ((f32(1) - t).astype(f32) * r).astype(f32)
    return np.copysign(y, x).astype(f32)

class TanhCheap(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z):
        h = torch.from_numpy(tanh_cheap_np(z.detach().numpy())); ctx.save_for_backward(h); return h
    @staticmethod
    def backward(ctx, g):
        h, = ctx.saved_tensors; return g * (1 - h * h)

class Mixed(LayerRef):
    def __init__(self, *a, cheap=set(), **k):
        super().__init__(*a, **k); self.cheap = cheap
    def functional_model(self, params):
        flat = self.mu.clone(); flat[self.idx] = params
        w = self._views(flat); nb = len(self.br)
        def act(z, i):
            return TanhCheap.apply(z) if i in self.cheap else torch.tanh(z)
        xb = self.x1
        for i in range(nb):
            xb = F.linear(xb, *w[i])
            if i < nb - 1: xb = act(xb, i)
        X2 = self.x2
        x_bc = torch.stack([torch.sin(2*np.pi*X2[:,:,1]), torch.sin(4*np.pi*X2[:,:,1]), torch.cos(2*np.pi*X2[:,:,1]), torch.cos(4*np.pi*X2[:,:,1])], dim=2)
        xtr = torch.cat([X2[:,:,0].unsqueeze(dim=2), x_bc], dim=2)
        for i in range(len(self.tr)):
            xtr = F.linear(xtr, *w[nb+i])
            if i < len(self.tr) - 1: xtr = act(xtr, i)
        return torch.unsqueeze(torch.einsum("...i,...i->...", xb, xtr), 1) + flat[0]

for name, ch in [("cheap0-6", set(range(7))), ("cheap all", set(range(8)))]:
    m = Mixed(lay, p.branch_in, p.trunk_in, p.y, p.mu, p.grad_ind, 0.0, SD, "NLL", 1.0, cheap=ch)
    e = [np.linalg.norm(m.logp_grad(th)[1] - g) / np.linalg.norm(g) for th, g in zip(ths, g64s)]
    print(f"{name:12s} median {np.median(e):.3e} {np.round(e,7).tolist()}", flush=True)
