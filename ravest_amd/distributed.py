"""Walker-block sharding over GPUs (one process per GPU, torch.distributed).

The only exchange on the path: each rank evaluates a
contiguous block of the W proposals on its own MI355X, then the per-walker
log-probs are all-gathered (RCCL over xGMI with the "nccl" backend; gloo on
CPU for tests) so the rank that runs the stretch move sees all W values.
Every walker is computed wholly on one GPU with a fixed reduction order, so
results are bitwise identical for any number of ranks.

    lp = LogPosterior(..., device=local_rank)
    sharded = ShardedLogProbability(lp.log_probability_batch)
    sampler = EnsembleSampler(W, D, sharded)          # identical proposals on every rank
"""
from __future__ import annotations

import numpy as np


def shard_bounds(n: int, world: int, rank: int):
    """Contiguous [lo, hi) of n items for `rank`; the first n % world ranks get one extra."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


class ShardedLogProbability:
    def __init__(self, log_prob_batch, group=None, device=None, src: int = 0) -> None:
        import torch
        import torch.distributed as dist
        self.fn = log_prob_batch
        self.group = group
        self.dist = dist
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.src = src
        backend = dist.get_backend(group)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
        self.device = device

    def broadcast(self, theta: np.ndarray) -> np.ndarray:
        """Make rank `src`'s proposal block the block of every rank."""
        import torch
        shape = torch.tensor(list(np.shape(theta)) if self.rank == self.src else [0, 0], dtype=torch.int64,
                             device=self.device)
        self.dist.broadcast(shape, self.src, group=self.group)
        buf = (torch.as_tensor(np.ascontiguousarray(theta, np.float64), device=self.device) if self.rank == self.src
               else torch.empty(tuple(shape.tolist()), dtype=torch.float64, device=self.device))
        self.dist.broadcast(buf, self.src, group=self.group)
        return buf.cpu().numpy()

    def __call__(self, theta: np.ndarray) -> np.ndarray:
        import torch
        theta = np.atleast_2d(np.asarray(theta, np.float64))
        n = theta.shape[0]
        lo, hi = shard_bounds(n, self.world, self.rank)
        per = -(-n // self.world)                     # padded shard length for all_gather
        local = np.full(per, np.nan)
        if hi > lo:
            local[: hi - lo] = self.fn(theta[lo:hi])
        t = torch.as_tensor(local, device=self.device)
        out = torch.empty(per * self.world, dtype=torch.float64, device=self.device)
        self.dist.all_gather_into_tensor(out, t, group=self.group)
        full = out.cpu().numpy().reshape(self.world, per)
        return np.concatenate([full[r, : shard_bounds(n, self.world, r)[1] - shard_bounds(n, self.world, r)[0]]
                               for r in range(self.world)])


class ShardedDevicePosterior:
    """Device-resident walker sharding: the config-4 form of the drop-in.

    Every rank holds the same proposal block ``theta [W, D]`` in its own HBM (the stretch
    move is replicated, or the block was broadcast once); rank r evaluates its contiguous
    slice ``shard_bounds(W, world, r)`` with ``evaluate(theta_slice, out_slice, stream)`` --
    ``DevicePosterior.device`` (rvk_logpost_device) or ``RVEngine.loglike_device`` on a
    GPU, any tensor function on CPU -- and the per-walker log-probs are all-gathered
    (``all_gather_into_tensor``: RCCL over xGMI with the "nccl" backend, gloo on CPU) into
    ``out [W]`` on every rank.  No host staging: theta, the slices and the gathered block
    stay device tensors.  Each walker is computed wholly on one GPU by a kernel whose
    result does not depend on the batch it is in (tests/test_gpu_layout.py), so ``out``
    is bitwise the single-GPU evaluation of the whole block at any world size.
    Replaces ravest's ``pool.map`` of ``log_probability`` over walkers (fit.py:1068-1075)."""

    def __init__(self, evaluate, group=None) -> None:
        import torch.distributed as dist
        if hasattr(evaluate, "device") and callable(getattr(evaluate, "device")):
            evaluate = evaluate.device                    # a DevicePosterior
        self.evaluate = evaluate
        self.group = group
        self.dist = dist
        init = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if init else 1      # no process group: one GPU
        self.rank = dist.get_rank(group) if init else 0
        self._inplace = init and dist.get_backend(group) == "nccl"   # RCCL's in-place all-gather
        self._bufs = {}

    def bounds(self, n: int):
        return shard_bounds(n, self.world, self.rank)

    def _buf(self, key, n, like):
        import torch
        b = self._bufs.get(key)
        if b is None or b.numel() < n or b.device != like.device:
            b = torch.empty(n, dtype=torch.float64, device=like.device)
            self._bufs[key] = b
        return b[:n]

    def __call__(self, theta, out=None, stream=None):
        """theta: float64 tensor [W, >=D] (same on every rank); out: float64 [W] or None.
        Returns out, holding every walker's log-probability on every rank."""
        import torch
        W = theta.shape[0]
        if out is None:
            out = torch.empty(W, dtype=torch.float64, device=theta.device)
        lo, hi = self.bounds(W)
        per = -(-W // self.world)                         # all_gather needs equal shard sizes
        even = per * self.world == W
        gathered = out if even else self._buf("gather", per * self.world, theta)
        local = gathered[self.rank * per:self.rank * per + per] if even else self._buf("local", per, theta)
        if hi > lo:
            if stream is None:
                self.evaluate(theta[lo:hi], local[:hi - lo])
            else:
                self.evaluate(theta[lo:hi], local[:hi - lo], stream)
        if not even:
            local[hi - lo:] = float("nan")                # padding, dropped below
        if self.world > 1:
            src = local if (not even or self._inplace) else local.clone()
            self.dist.all_gather_into_tensor(gathered, src, group=self.group)
        if not even:
            for r in range(self.world):
                a, b = shard_bounds(W, self.world, r)
                out[a:b] = gathered[r * per:r * per + (b - a)]
        return out


class ShardedDeviceSampler:
    """The device stretch move over several GPUs (one process per GPU): config 4's 65536 walkers
    as a sampler, not only as a batch evaluator (SURVEY.md §8(e) + §8(f) row 3).

    Every rank holds the whole walker state x [W, D], lp [W] in its HBM.  Per half-step each rank
    makes, evaluates and accepts/rejects its contiguous slice of the active half's proposals
    (rvk_stretch_half: Philox draws keyed by the global proposal index and step, so the union
    over ranks is exactly the single-GPU half-step), then the updated rows of the half are
    all-gathered in place (RCCL over xGMI; x and lp of the half packed in one buffer, one
    collective per half-step) before the next half-step reads them as its complement.  The chain
    equals DeviceEnsembleSampler(rng="philox") with the same seed bit for bit at any world size.
    With the gloo backend (CPU tests, or a 1-GPU rehearsal with several ranks on one device) the
    gather is staged through host memory.  Replaces ravest's pool.map over walkers
    (fit.py:1068-1075) for a run that does not fit one GPU's time budget."""

    def __init__(self, log_posterior, nwalkers: int, a: float = 2.0, seed: int = 0, group=None) -> None:
        import torch
        import torch.distributed as dist
        from .posterior import DevicePosterior
        self.post = log_posterior if isinstance(log_posterior, DevicePosterior) else DevicePosterior(log_posterior)
        self.nwalkers, self.ndim, self.a, self.seed = nwalkers, self.post.n_free, float(a), int(seed)
        if nwalkers % 2 or nwalkers < 4 or nwalkers < 2 * self.ndim:
            raise ValueError("nwalkers must be even, >= 4 and >= 2 * ndim")
        self.group = group
        self.dist = dist
        init = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if init else 1
        self.rank = dist.get_rank(group) if init else 0
        self.rccl = init and dist.get_backend(group) == "nccl"
        H = nwalkers // 2
        if H % self.world:
            raise ValueError(f"walkers per half ({H}) must divide evenly over {self.world} ranks")
        self.chunk = H // self.world
        self.device = torch.device("cuda", torch.cuda.current_device())
        self.post.reserve(self.chunk)
        self.iteration = 0
        self._chain, self._lnp = [], []
        self.naccepted = np.zeros(nwalkers, dtype=np.int64)

    def _gather_half(self, state, half):
        """state [W, D + 1] (x | lp); all-gather the active half's rows, chunk per rank."""
        import torch
        H = self.nwalkers // 2
        rows = state[half * H:(half + 1) * H]
        mine = rows[self.rank * self.chunk:(self.rank + 1) * self.chunk]
        if self.world == 1:
            return
        if self.rccl:
            self.dist.all_gather_into_tensor(rows.reshape(-1), mine.reshape(-1).clone(), group=self.group)
        else:
            out = torch.empty(rows.numel(), dtype=torch.float64)
            self.dist.all_gather_into_tensor(out, mine.reshape(-1).cpu(), group=self.group)
            rows.copy_(out.view_as(rows))

    def run_mcmc(self, initial_state, nsteps: int):
        import torch
        from . import _lib
        W, D = self.nwalkers, self.ndim
        x0 = np.array(initial_state, dtype=np.float64, copy=True)
        if x0.shape != (W, D):
            raise ValueError(f"initial_state must have shape ({W}, {D})")
        dev = self.device
        x = torch.from_numpy(x0).to(dev)
        lp = torch.empty(W, dtype=torch.float64, device=dev)
        stream = torch.cuda.current_stream(dev)
        self.post.device(x, lp, stream)                    # every rank: the whole initial block
        lp0 = lp.cpu().numpy()
        if np.any(np.isnan(lp0)) or not np.all(np.isfinite(lp0)):
            raise ValueError("initial state has NaN or -inf log-probabilities")
        # packed state for the gathers: columns 0..D-1 = x, column D = lp (the kernel reads the views)
        state = torch.empty((W, D + 1), dtype=torch.float64, device=dev)
        nacc = torch.zeros(W, dtype=torch.int64, device=dev)
        status = torch.zeros(1, dtype=torch.int32, device=dev)
        L = _lib.load()
        H = W // 2
        j0 = self.rank * self.chunk
        xs = torch.empty((W, D), dtype=torch.float64, device=dev)
        lps = torch.empty(W, dtype=torch.float64, device=dev)
        xs.copy_(x)
        lps.copy_(lp)
        chain = torch.empty((nsteps, W, D), dtype=torch.float64, device=dev)
        lnpc = torch.empty((nsteps, W), dtype=torch.float64, device=dev)
        for t in range(nsteps):
            for half in (0, 1):
                _lib.check(L.rvk_stretch_half(self.post._p, xs.data_ptr(), lps.data_ptr(), W, half, j0, self.chunk,
                                              self.a, self.seed, self.iteration + t, nacc.data_ptr(),
                                              status.data_ptr(), stream.cuda_stream))
                if self.world > 1:
                    rows = slice(half * H, (half + 1) * H)
                    state[rows, :D] = xs[rows]
                    state[rows, D] = lps[rows]
                    self._gather_half(state, half)
                    xs[rows] = state[rows, :D]
                    lps[rows] = state[rows, D]
            chain[t] = xs
            lnpc[t] = lps
        if int(status.item()):
            raise ValueError("The log_prob was NaN")
        if self.world > 1:                                 # each rank counted its slices' acceptances
            if self.rccl:
                self.dist.all_reduce(nacc, group=self.group)
            else:
                c = nacc.cpu()
                self.dist.all_reduce(c, group=self.group)
                nacc.copy_(c)
        self._chain.append(chain.cpu().numpy())
        self._lnp.append(lnpc.cpu().numpy())
        self.naccepted += nacc.cpu().numpy()
        self.iteration += nsteps
        return xs.cpu().numpy(), lps.cpu().numpy()

    def get_chain(self) -> np.ndarray:
        return np.concatenate(self._chain) if self._chain else np.zeros((0, self.nwalkers, self.ndim))

    def get_log_prob(self) -> np.ndarray:
        return np.concatenate(self._lnp) if self._lnp else np.zeros((0, self.nwalkers))
