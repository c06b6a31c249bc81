import sys, time
import numpy as np
import torch
sys.path.insert(0, '.')
from oracle import coracle as C
from plonky3_eon_amd import Context, Radix2Dit
ctx = Context(0)
d = Radix2Dit(ctx)
g5 = C.fr_from_u64(5)
dev = torch.device('cuda', 0)
def cmp(name, got, want):
    if isinstance(got, torch.Tensor):
        got = got.cpu().numpy().view(np.uint64)
    bad = np.nonzero(np.any(got != want, axis=(1, 2)))[0]
    print(name, 'rows bad', len(bad), bad[:8], flush=True)
for log_n, w in [(16, 8), (18, 8), (20, 8)]:
    x = C.random_fr(5 + log_n + w, (1 << log_n) * w).reshape(1 << log_n, w, 4)
    xt = torch.from_numpy(x.view(np.int64)).to(dev)
    want = C.coset_lde_batch(x, 1, g5)
    cmp(f'lde host {log_n}x{w}', d.coset_lde_batch(x, 1, g5), want)
    cmp(f'lde dev {log_n}x{w}', d.coset_lde_batch(xt, 1, g5), want)
    w2 = C.coset_idft_batch(want, g5)
    cmp(f'coset_idft host {log_n+1}x{w}', d.coset_idft_batch(want, g5), w2)
    cmp(f'coset_idft dev {log_n+1}x{w}', d.coset_idft_batch(torch.from_numpy(want.view(np.int64)).to(dev), g5), w2)
    cmp(f'idft dev {log_n}x{w}', d.idft_batch(xt), C.idft_batch(x))
