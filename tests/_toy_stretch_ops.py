"""A host (torch CPU) stand-in for the device stretch-move operations of ShardedDeviceSampler
(ravest_amd.distributed.LibStretchOps): same interface and the same per-half-step contract --
draws keyed by (seed, global step), a slice of proposals evaluated per rank, the whole half's
accept / reject applied by every rank -- over a toy log-probability, so the multi-rank
orchestration (slices, the all-gather, NaN handling, chunking) runs under gloo on CPU."""
import numpy as np


class ToyStretchOps:
    def __init__(self, ndim: int, nan_at=None) -> None:
        self.n_free = ndim
        self.nan_at = nan_at            # (global step, half, proposal j): that proposal's log-prob is NaN
        self.table = None
        self.step0 = 0

    def reserve(self, n: int) -> None:
        pass

    @staticmethod
    def _lp(q):
        return -0.5 * np.sum(q * q, axis=-1) + 0.3 * q[..., 0]

    def logpost(self, x, out, stream) -> None:
        out.copy_(__import__("torch").from_numpy(self._lp(x.numpy())))

    def draws(self, W, n, a, seed, step0, flags, stream) -> None:
        H = W // 2
        tab = []
        for s in range(n):
            rng = np.random.default_rng([seed, step0 + s])
            if flags:
                sets = [np.arange(0, W, 2), np.arange(1, W, 2)]
            else:
                perm = rng.permutation(W)
                sets = [np.sort(perm[:H]), np.sort(perm[H:])]
            zu, au, rint = rng.random((2, H)), rng.random((2, H)), rng.integers(0, H, (2, H))
            z = ((a - 1.0) * zu + 1.0) ** 2 / a
            tab.append([(sets[h], sets[1 - h][rint[h]], z[h], (self.n_free - 1.0) * np.log(z[h]), np.log(au[h]))
                        for h in (0, 1)])
        self.table, self.step0 = tab, step0

    def _q(self, x, s, half, j):
        S, Cc, z, _, _ = self.table[s][half]
        xs, xc = x[S[j]], x[Cc[j]]
        return xc + (xs - xc) * z[j][:, None]

    def propose(self, x, W, s, half, j0, count, out, stream) -> None:
        import torch
        j = np.arange(j0, j0 + count)
        v = self._lp(self._q(x.numpy(), s, half, j))
        if self.nan_at is not None:
            st, h, jj = self.nan_at
            if st == self.step0 + s and h == half and j0 <= jj < j0 + count:
                v[jj - j0] = np.nan
        out[:count].copy_(torch.from_numpy(v))

    def update(self, x, lp, W, s, half, nlp, chain_step, lnp_step, nacc_in, nacc_out, status, stream) -> None:
        S, Cc, z, fac, lau = self.table[s][half]
        xn, lpn, nl = x.numpy(), lp.numpy(), nlp.numpy()
        q = self._q(xn, s, half, np.arange(len(S)))
        if np.any(np.isnan(nl)):
            status[0] = 1
        acc = fac + nl - lpn[S] > lau
        xn[S[acc]] = q[acc]
        lpn[S[acc]] = nl[acc]
        chain_step.numpy()[S] = xn[S]
        lnp_step.numpy()[S] = lpn[S]
        nacc_out.numpy()[S] = nacc_in.numpy()[S] + acc
