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
        self.grouped = init                       # a process group: the all-gather runs (even at world 1)
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
        if self.grouped:
            src = local if (not even or self._inplace) else local.clone()
            self.dist.all_gather_into_tensor(gathered, src, group=self.group)
        if not even:
            for r in range(self.world):
                a, b = shard_bounds(W, self.world, r)
                out[a:b] = gathered[r * per:r * per + (b - a)]
        return out


class LibStretchOps:
    """The device stretch move's operations for ShardedDeviceSampler, on librvk
    (include/rvk_post.h): draws, slice evaluation, whole-half update.  ``gp=True``: the GP
    log-posterior's (include/rvk_gp.h rvk_gp_stretch_*), GPFitter.run_mcmc's sampler."""

    def __init__(self, post, gp: bool = False) -> None:
        self.post = post
        self.n_free = post.n_free
        self._pre = "rvk_gp_stretch_" if gp else "rvk_stretch_"

    def reserve(self, n: int) -> None:
        self.post.reserve(n)

    def logpost(self, x, out, stream) -> None:
        self.post.device(x, out, stream)

    def draws(self, W, n, a, seed, step0, flags, stream) -> None:
        from . import _lib
        _lib.check(getattr(_lib.load(), self._pre + "draws")(self.post._p, W, n, a, seed, step0, flags,
                                                               stream.cuda_stream))

    def propose(self, x, W, s, half, j0, count, out, stream) -> None:
        from . import _lib
        _lib.check(getattr(_lib.load(), self._pre + "propose")(self.post._p, x.data_ptr(), W, s, half, j0, count,
                                                                 out.data_ptr(), stream.cuda_stream))

    def update(self, x, lp, W, s, half, nlp, chain_step, lnp_step, nacc_in, nacc_out, status, stream) -> None:
        from . import _lib
        _lib.check(getattr(_lib.load(), self._pre + "update")(self.post._p, x.data_ptr(), lp.data_ptr(), W, s, half,
                                                                nlp.data_ptr(), chain_step.data_ptr(),
                                                                lnp_step.data_ptr(), nacc_in.data_ptr(),
                                                                nacc_out.data_ptr(), status.data_ptr(),
                                                                stream.cuda_stream))


from .sampler import _Chunk, _DevicePipeline  # noqa: E402


class ShardedDeviceSampler(_DevicePipeline):
    """The device stretch move over several GPUs, one process per GPU: config 4's 65536 walkers as
    a sampler (SURVEY.md §8(e) + §8(f) row 3), with emcee 3.1's interface (``sample``,
    ``run_mcmc``, ``iteration``, ``get_chain``, ``get_autocorr_time``, ...).  Replaces ravest's
    ``pool.map`` over walkers (fit.py:1068-1075).

    Every rank holds the whole ensemble (x [W, D], lp [W]) and the same Philox draws (keyed by
    seed, global step and proposal).  Per half-step rank r evaluates only its contiguous slice of
    the H = W/2 proposals (rvk_stretch_propose), the H per-proposal log-posteriors are
    all-gathered -- the one exchange, H x 8 bytes in all (RCCL over xGMI with the "nccl"
    backend; staged through host memory with gloo) -- and every rank applies the accept / reject
    to the whole half itself (rvk_stretch_update), so the state stays replicated without moving
    any coordinates.  The chain equals DeviceEnsembleSampler(rng="philox") with the same seed
    and split bit for bit at any world size; a NaN log-probability is seen by every rank in the
    gathered block, so all ranks raise together.  (On one GPU DeviceEnsembleSampler is faster:
    one fused kernel per half-step instead of evaluate + update.)

    ``keep_chain``: "all", or the rank that stores the chain (in its HBM with the default
    ``chain_storage``, or its host memory with "host"; the others keep only the device chunk).
    Every rank counts the steps and acceptances alike (``iteration``, ``naccepted``), keeping a
    chain or not.  With one keeping rank ``get_autocorr_time`` is computed there and broadcast (a
    collective: call it on every rank, as ravest's convergence loop does); with "all" every rank
    holds the same chain and computes it locally (no collective; the chain storage is decided
    collectively at each ``sample`` call, so every rank's estimate takes the same code path and
    the ranks' convergence decisions agree).  A ``GPLogPosterior`` (GPFitter.run_mcmc,
    fit.py:4983-4990) shards the same way over rvk_gp_stretch_draws / _propose / _update; its
    chain equals DeviceEnsembleSampler(GPLogPosterior)'s bit for bit."""

    def __init__(self, log_posterior, nwalkers: int, a: float = 2.0, seed: int = 0, group=None,
                 randomize_split: bool = True, steps_per_call: int = 256, keep_chain="all",
                 ops=None, device=None, chain_storage: str = "auto") -> None:
        import torch
        import torch.distributed as dist
        if ops is None:
            from .gp import DeviceGPPosterior, GPLogPosterior
            from .posterior import DevicePosterior
            if isinstance(log_posterior, (GPLogPosterior, DeviceGPPosterior)):      # GPFitter.run_mcmc
                post = log_posterior if isinstance(log_posterior, DeviceGPPosterior) else DeviceGPPosterior(log_posterior)
                ops = LibStretchOps(post, gp=True)
            else:
                post = log_posterior if isinstance(log_posterior, DevicePosterior) else DevicePosterior(log_posterior)
                ops = LibStretchOps(post)
            device = torch.device("cuda", torch.cuda.current_device())
        self.ops = ops
        self.nwalkers, self.ndim, self.a, self.seed = nwalkers, ops.n_free, float(a), int(seed)
        if nwalkers % 2 or nwalkers < 4 or nwalkers < 2 * self.ndim:
            raise ValueError("nwalkers must be even, >= 4 and >= 2 * ndim")
        self.randomize_split = bool(randomize_split)
        self.steps_per_call = max(1, int(steps_per_call))
        self.group = group
        self.dist = dist
        init = dist.is_available() and dist.is_initialized()
        self.grouped = init                   # a process group: the collectives run (even at world 1)
        self.world = dist.get_world_size(group) if init else 1
        self.rank = dist.get_rank(group) if init else 0
        self.rccl = init and dist.get_backend(group) == "nccl"
        H = nwalkers // 2
        if H % self.world:
            raise ValueError(f"walkers per half ({H}) must divide evenly over {self.world} ranks")
        self.chunk = H // self.world
        if keep_chain != "all" and not (isinstance(keep_chain, int) and 0 <= keep_chain < self.world):
            raise ValueError("keep_chain must be 'all' or a rank")
        self.keep_chain = keep_chain
        ops.reserve(self.chunk)
        self._pipeline_init(device, keep_host=keep_chain == "all" or keep_chain == self.rank,
                            chain_storage=chain_storage)
        self._nlp_local = torch.empty(self.chunk, dtype=torch.float64, device=device)
        self._nlp_all = torch.empty(H, dtype=torch.float64, device=device)
        self._nacc_steps = [None, None]       # per slot: [steps_per_call, W] acceptance counts after each step
        self.exchange_bytes_per_half_step = 0

    def _flags(self) -> int:
        from . import _lib
        return 0 if self.randomize_split else _lib.STRETCH_FIXED_SPLIT

    def _initial_log_prob(self, x, lp) -> None:
        self.ops.logpost(x, lp, self._stream())

    def _gather(self, stream) -> None:
        import torch
        if not self.grouped:
            self._nlp_all.copy_(self._nlp_local)
        elif self.rccl:
            self.dist.all_gather_into_tensor(self._nlp_all, self._nlp_local, group=self.group)
        else:                                 # gloo: staged through host memory
            out = torch.empty(self._nlp_all.numel(), dtype=torch.float64)
            self.dist.all_gather_into_tensor(out, self._nlp_local.cpu(), group=self.group)
            self._nlp_all.copy_(out)
        self.exchange_bytes_per_half_step = self._nlp_all.numel() * self._nlp_all.element_size()

    def _begin_chunk(self, ch: _Chunk) -> None:
        import torch
        if self._nacc_steps[ch.slot] is None:
            self._nacc_steps[ch.slot] = torch.empty((self.steps_per_call, self.nwalkers), dtype=torch.int64,
                                                    device=self.device)
        ch.x0 = ch.lp0 = ch.nacc0 = ch.draws = ch.rstate0 = None

    def _run_chunk(self, ch: _Chunk, chain_d, lnp_d, stream) -> None:
        W, n = self.nwalkers, ch.n
        ns = self._nacc_steps[ch.slot]
        self.ops.draws(W, n, self.a, self.seed, ch.start, self._flags(), stream)
        j0 = self.rank * self.chunk
        prev = self._nacc
        for s in range(n):
            for half in (0, 1):
                self.ops.propose(self._x, W, s, half, j0, self.chunk, self._nlp_local, stream)
                self._gather(stream)
                self.ops.update(self._x, self._lp, W, s, half, self._nlp_all, chain_d[s], lnp_d[s], prev, ns[s],
                                self._status, stream)
            prev = ns[s]
        if ch.store:                          # emcee counts the acceptances of stored steps only
            self._nacc.copy_(ns[n - 1])

    def _state_at(self, target: int):
        """(x, lp, nacc) device views of the state after step `target` (a step of the last chunks,
        or the initial state): the chunk's own chain rows -- no replay, no collective."""
        if target == self._x_init[0]:
            return self._x_init[1], self._x_init[2], self._x_init[3]
        ch = next((c for c in self._chunks if c.start < target <= c.start + c.n), None)
        if ch is None:
            raise RuntimeError("internal: no chunk record covers the requested step")
        chain_d, lnp_d = ch.bufs
        k = target - 1 - ch.start
        return chain_d[k], lnp_d[k], (self._nacc_steps[ch.slot][k] if ch.store else self._nacc)

    def _settle(self) -> None:
        if self._x is None or self._dev_iter == self._pos:
            return
        x, lp, nacc = self._state_at(self._pos)
        self._x.copy_(x)
        self._lp.copy_(lp)
        self._nacc.copy_(nacc)
        self._dev_iter = self._pos
        self._chunks = []
        self._x_init = (self._dev_iter, self._x.clone(), self._lp.clone(), self._nacc.clone())
        self.backend.accepted = self._nacc.cpu().numpy()
        self._accepted_pos = self._pos

    @property
    def naccepted(self):
        if self._accepted_pos != self._pos:
            src = self._nacc if self._dev_iter == self._pos else self._state_at(self._pos)[2]
            self.backend.accepted = src.cpu().numpy()
            self._accepted_pos = self._pos
        return self.backend.accepted

    def get_chain(self, flat=False, thin=1, discard=0):
        if not self._keep_host:
            raise RuntimeError(f"rank {self.rank} keeps no chain (keep_chain={self.keep_chain})")
        return super().get_chain(flat=flat, thin=thin, discard=discard)

    def get_log_prob(self, flat=False, thin=1, discard=0):
        if not self._keep_host:
            raise RuntimeError(f"rank {self.rank} keeps no chain (keep_chain={self.keep_chain})")
        return super().get_log_prob(flat=flat, thin=thin, discard=discard)

    def _device_chain_fits(self, iterations: int) -> bool:
        """chain_storage="auto": the device chain grows only if it fits on EVERY rank (one MIN
        all-reduce; sample() is collective already), so all ranks keep their chains in the same
        storage and their autocorrelation estimates round alike."""
        fits = super()._device_chain_fits(iterations)
        if not self.grouped or self.chain_storage_requested != "auto" or self.keep_chain != "all":
            return fits
        import torch
        f = torch.tensor([1 if fits else 0], dtype=torch.int32, device=self.device if self.rccl else "cpu")
        self.dist.all_reduce(f, op=self.dist.ReduceOp.MIN, group=self.group)
        return bool(int(f[0]))

    def get_autocorr_time(self, discard=0, thin=1, **kwargs):
        """emcee's estimate.  keep_chain="all": computed locally on each rank (every rank holds the
        same chain bits in the same storage, so the estimates should be equal), then one small
        guard collective: a MAX all-reduce of [tau, -tau, failed] that raises on EVERY rank if
        the ranks' estimates differ in any bit (e.g. a different FFT plan on one GPU) or the
        estimate failed on any rank -- so a convergence test cannot break on one rank and not on
        another and leave the others waiting in the next all-gather.  One keeping rank: computed
        there and broadcast.  Both forms are collective: call it on every rank, as ravest's
        convergence loop does."""
        import torch
        if not self.grouped:
            return super().get_autocorr_time(discard=discard, thin=thin, **kwargs)
        if self.keep_chain == "all":
            from .sampler import AutocorrError
            dev = self.device if self.rccl else "cpu"
            g = torch.zeros(2 * self.ndim + 1, dtype=torch.float64, device=dev)
            tau, exc = None, None
            try:
                tau = np.asarray(super().get_autocorr_time(discard=discard, thin=thin, **kwargs), np.float64)
                t = torch.from_numpy(np.nan_to_num(tau, nan=np.inf)).to(dev)
                g[: self.ndim] = t
                g[self.ndim: 2 * self.ndim] = -t
            except AutocorrError as e:                # emcee's "chain too short": same on every rank
                g[-1] = 1.0
                exc = e
            except Exception as e:
                g[-1] = 2.0
                exc = e
            self.dist.all_reduce(g, op=self.dist.ReduceOp.MAX, group=self.group)
            flag = float(g[-1])
            if flag:
                if exc is not None:
                    raise exc
                raise AutocorrError(np.full(self.ndim, np.nan), "autocorrelation estimate failed on another rank")
            hi, lo = g[: self.ndim].cpu().numpy(), -g[self.ndim: 2 * self.ndim].cpu().numpy()
            if not np.array_equal(hi, lo):
                raise RuntimeError(f"ranks disagree on the autocorrelation time (max {hi}, min {lo}): "
                                   "their chains or FFTs differ")
            return tau
        src = self.keep_chain
        tau = torch.zeros(self.ndim, dtype=torch.float64, device=self.device if self.rccl else "cpu")
        err = torch.zeros(1, dtype=torch.float64, device=tau.device)
        if self.rank == src:
            try:
                tau.copy_(torch.from_numpy(super().get_autocorr_time(discard=discard, thin=thin, **kwargs)))
            except Exception:
                err.fill_(1.0)
        self.dist.broadcast(err, src, group=self.group)
        self.dist.broadcast(tau, src, group=self.group)
        if float(err[0]):
            from .sampler import AutocorrError
            raise AutocorrError(tau.cpu().numpy(), f"autocorrelation estimate failed on rank {src}")
        return tau.cpu().numpy()
