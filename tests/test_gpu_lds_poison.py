"""The LDS publish-order guard (RVK_OPT_LDS_POISON, include/rvk.h): with the option on, every
kernel that stages the sin/cos table in LDS writes each entry as NaN first and the real value
~10 us later, before the barrier that publishes it.  A table read that is not ordered after that
barrier (the race round 4 found in every table-filling kernel, which green parity tests had
missed) then reads NaN and turns the walker's result NaN -- so these tests fail if a read moves
ahead of its barrier again.  With the kernels race-free the poisoned run gives the same bits as
the normal one, which is what they check, on config 2 (the headline kernel), config 3 (the
segmented kernel), a shard of config 4 (2 planets), the device log-posterior and fused sampler
kernels, the posterior predictive and config 5's GP shape (fp64 and fp32 factorisations)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _engine(ds):
    from ravest_amd.engine import RVEngine
    return RVEngine(ds.time, ds.vel, ds.velerr, ds.inst_idx, len(ds.unique_instruments), len(ds.planet_letters),
                    ds.parameterisation, ds.t0, device=0)


def _both(eng, fn):
    eng.set_lds_poison(False)
    a = fn()
    eng.set_lds_poison(True)
    try:
        b = fn()
    finally:
        eng.set_lds_poison(False)
    return a, b


@pytest.mark.parametrize("cfg,W", [(2, None), (3, 16384), (4, 8192)])
def test_loglike_poisoned_table_same_bits(cfg, W):
    from ravest_amd.synth import make_config
    ds = make_config(cfg, n_walkers=W)
    eng = _engine(ds)
    a, b = _both(eng, lambda: eng.loglike(ds.theta))
    assert np.isfinite(a).sum() > 0.9 * len(a)
    assert np.array_equal(a, b, equal_nan=True), f"config {cfg}: {np.isnan(b).sum()} NaN walkers with the poisoned table"
    # the device-resident form too (the launch the bench times)
    th = torch.from_numpy(ds.theta).cuda()
    out = torch.empty(len(ds.theta), dtype=torch.float64, device="cuda")

    def dev():
        eng.loglike_device(th, out)
        torch.cuda.synchronize()
        return out.cpu().numpy()
    a2, b2 = _both(eng, dev)
    assert np.array_equal(a2, a, equal_nan=True) and np.array_equal(b2, a, equal_nan=True)


def test_posterior_sampler_predictive_poisoned_table_same_bits():
    from ravest_amd.sampler import DeviceEnsembleSampler
    from ravest_amd.synth import make_posterior
    lpost, x0 = make_posterior(2, n_walkers=1024, device=0)
    eng = lpost.log_likelihood.engine
    dp = lpost.device_posterior()
    a, b = _both(eng, lambda: dp(x0))
    assert np.array_equal(a, b, equal_nan=True), "device log-posterior (DIRECT kernel)"

    def run():
        s = DeviceEnsembleSampler(lpost, 1024, seed=3)
        s.run_mcmc(x0, 16)
        return np.concatenate([s.get_chain().ravel(), s.get_log_prob().ravel()])
    a, b = _both(eng, run)
    assert np.array_equal(a, b, equal_nan=True), "fused stretch-move half-step"
    from ravest_amd.synth import make_config
    ds = make_config(2, n_walkers=512)
    e2 = _engine(ds)
    tq = np.linspace(ds.time.min(), ds.time.max(), 300)
    a, b = _both(e2, lambda: e2.predict(ds.theta, tq))
    assert np.array_equal(a, b, equal_nan=True), "posterior predictive"


@pytest.mark.parametrize("precision", ["fp64", "fp32+fp64"])
def test_gp_poisoned_table_same_bits(precision):
    from ravest_amd.gp import GPKernel, GPLogLikelihood
    from ravest_amd.synth import make_gp_config
    ds, th, hy = make_gp_config(n_walkers=256)
    gp = GPLogLikelihood(ds.time, ds.vel, ds.velerr, ds.t0, ds.instrument, ds.unique_instruments, ds.planet_letters,
                         ds.parameterisation, GPKernel("Quasiperiodic"), precision=precision)
    a, b = _both(gp.engine, lambda: gp.batch(th, hy))
    assert np.isfinite(a).sum() > 0.9 * len(a)
    assert np.array_equal(a, b, equal_nan=True), f"GP {precision}: {np.isnan(b).sum()} NaN walkers when poisoned"


@pytest.mark.parametrize("cfg,W", [(2, None), (3, 16384)])
def test_poison_reaches_the_kernel(cfg, W):
    """Positive control: the poisoned fill really runs (each filling thread sleeps ~10 us between
    its NaN and its real store), so a poisoned launch is measurably slower -- the equality tests
    above would pass vacuously if the flag never reached the kernel."""
    from ravest_amd.synth import make_config
    ds = make_config(cfg, n_walkers=W)
    eng = _engine(ds)
    th = torch.from_numpy(ds.theta).cuda()
    out = torch.empty(len(ds.theta), dtype=torch.float64, device="cuda")

    def us_per_launch(n=20):
        eng.loglike_device(th, out)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(n):
            eng.loglike_device(th, out)
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3 / n
    plain, poisoned = _both(eng, us_per_launch)
    assert poisoned > plain + 5.0, (plain, poisoned)


def _nan_control(eng, fn):
    """Run fn with RVK_OPT_LDS_POISON = 2 (the real table values never stored)."""
    eng.set_lds_poison(2)
    try:
        return fn()
    finally:
        eng.set_lds_poison(False)


def test_poison_control_reaches_every_kernel_family():
    """Positive control for the equality tests above: with poison = 2 every table
    read is NaN, so each kernel family the option must reach -- the device log-posterior (DIRECT
    kernel), the fused sampler half-step, the posterior predictive, the fp64 and fp32 GP
    factorisations -- returns NaN where the plain run is finite.  If the flag did not reach one
    of them, its equality test above would pass without testing anything; this one fails."""
    from ravest_amd.gp import GPKernel, GPLogLikelihood
    from ravest_amd.sampler import DeviceEnsembleSampler
    from ravest_amd.synth import make_config, make_gp_config, make_posterior
    lpost, x0 = make_posterior(2, n_walkers=1024, device=0)
    eng = lpost.log_likelihood.engine
    dp = lpost.device_posterior()
    plain = dp(x0)
    ctl = _nan_control(eng, lambda: dp(x0))
    assert np.isnan(ctl[np.isfinite(plain)]).all(), "device log-posterior (DIRECT kernel)"

    def run():
        s = DeviceEnsembleSampler(lpost, 1024, seed=3)
        s.run_mcmc(x0, 4)
    with pytest.raises(ValueError, match="NaN"):
        _nan_control(eng, run)                     # the fused half-step's log-probs are NaN
    ds = make_config(2, n_walkers=512)
    e2 = _engine(ds)
    tq = np.linspace(ds.time.min(), ds.time.max(), 300)
    plain = e2.predict(ds.theta, tq)
    ctl = _nan_control(e2, lambda: e2.predict(ds.theta, tq))
    assert np.isfinite(plain).any() and np.isnan(ctl[np.isfinite(plain)]).all(), "posterior predictive"
    dsg, th, hy = make_gp_config(n_walkers=256)
    for precision in ("fp64", "fp32+fp64"):
        gp = GPLogLikelihood(dsg.time, dsg.vel, dsg.velerr, dsg.t0, dsg.instrument, dsg.unique_instruments,
                             dsg.planet_letters, dsg.parameterisation, GPKernel("Quasiperiodic"), precision=precision)
        plain = gp.batch(th, hy)
        ctl = _nan_control(gp.engine, lambda: gp.batch(th, hy))
        fin = np.isfinite(plain)
        assert fin.sum() > 0.9 * len(plain) and np.isnan(ctl[fin]).all(), f"GP {precision}"
