import os, sys, torch
sys.path.insert(0, '/root/repo')
from time_opt_ilqr_amd import _lib, engine, synth
_lib.check(_lib.load().hop_set_options(0, 41))  # developer build: the conditioned kernel alone
dev = torch.device('cuda', 0)
A, Bm, Q, Ri, z0, QT = synth.device_batch(4096, 13, 4, 100, seed=1234, device=dev)
r = engine.propagate(A, Bm, Q, Ri, z0, QT, t_min=40, t_max=100)
print('augmented: flagged', int((r.status & 16).ne(0).sum()))
