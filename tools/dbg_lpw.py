import numpy as np, sys
sys.path.insert(0, '.')
from ravest_amd.engine import RVEngine
from ravest_amd.synth import make_dataset, make_walkers
n = 16
ds = make_dataset(1, n, 1, seed=5)
th = make_walkers(ds, 4096, seed=1, frac_invalid=0.0)
eng = RVEngine(ds.time, ds.vel, ds.velerr, ds.inst_idx, 1, 1, ds.parameterisation, ds.t0)
same = np.repeat(th[:1], 4096, axis=0)
swap = th.copy(); swap[0::2] = th[1::2]; swap[1::2] = th[0::2]
for name, T in (("same", same), ("orig", th), ("swap", swap)):
    out = {}
    for l in (64, 32):
        eng.set_lanes_per_walker(l); out[l] = eng.loglike(T)
    print(name, out[64][:4], out[32][:4])
