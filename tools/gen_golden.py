"""Generate the golden fixtures under tests/golden/ from the ravest reference.

Runs ONLY in the build container (it imports /root/reference, which never
travels to the GPU box); its outputs are small .npz / .json files that are
committed.  Recipe: ``ravest/__init__.py`` needs installed
metadata, so ``ravest`` is pre-registered as a namespace package; numba is
stubbed with an identity ``njit`` (the interpreted ``_solve_kepler`` is the
exact source numba compiles); astropy / jax / tinygp / emcee / corner are
stubbed with empty modules -- none of them is on the log-probability path.

Usage:  python tools/gen_golden.py   (≈1-2 min, single core)
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SRC = "/root/reference/src/ravest"
OUT = os.path.join(REPO, "tests", "golden")


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def import_reference():
    _stub("numba", njit=lambda *a, **k: (a[0] if a and callable(a[0]) else (lambda f: f)))
    _stub("astropy")
    _stub("astropy.constants")
    sys.modules["astropy"].constants = sys.modules["astropy.constants"]
    jnp = _stub("jax.numpy", **{k: getattr(np, k) for k in dir(np) if not k.startswith("__")})
    _stub("jax", config=types.SimpleNamespace(update=lambda *a, **k: None),
          jit=lambda f=None, **k: (f if f is not None else (lambda g: g)), numpy=jnp)

    class _Kernel:
        """tinygp 0.3 kernel algebra, restated for the GP goldens (the covariance the
        reference's GPKernel.build_kernel describes, gp.py:126-156; tinygp is absent, so
        this part is a restatement -- "parity unpinned" at the tinygp boundary)."""
        def __mul__(self, other):
            return _Product(self, other)

        def __rmul__(self, other):
            return _Product(other, self)

    class _Product(_Kernel):
        def __init__(self, a, b):
            self.a, self.b = a, b

        def evaluate(self, tau):
            ev = lambda k: k.evaluate(tau) if isinstance(k, _Kernel) else k   # noqa: E731
            return ev(self.a) * ev(self.b)

    class ExpSquared(_Kernel):
        def __init__(self, scale):
            self.scale = scale

        def evaluate(self, tau):
            return np.exp(-0.5 * (tau / self.scale) ** 2)

    class ExpSineSquared(_Kernel):
        def __init__(self, scale, gamma):
            self.scale, self.gamma = scale, gamma

        def evaluate(self, tau):
            return np.exp(-self.gamma * np.sin(np.pi * np.abs(tau) / self.scale) ** 2)
    kern = _stub("tinygp.kernels", Kernel=_Kernel, ExpSquared=ExpSquared, ExpSineSquared=ExpSineSquared)
    _stub("tinygp", GaussianProcess=None, kernels=kern)
    _stub("emcee")
    _stub("corner")
    pkg = types.ModuleType("ravest")
    pkg.__path__ = [REF_SRC]
    sys.modules["ravest"] = pkg
    import ravest.fit
    import ravest.model
    import ravest.param
    import ravest.prior
    return ravest


sys.path.insert(0, REPO)
from ravest_amd.synth import make_dataset, make_walkers  # noqa: E402


def prior_obj(ref, spec):
    cls, kw = spec
    return getattr(ref.prior, cls)(**kw)


# --------------------------------------------------------------------------
def gen_kepler(ref):
    es = [0.0, 1e-6, 0.1, 0.3, 0.5, 0.7, 0.8, 0.9, 0.95, 0.99, 0.999, 0.9999]
    rng = np.random.default_rng(11)
    Ms = np.concatenate([
        np.linspace(-np.pi, np.pi, 61),
        np.linspace(0, 2 * np.pi, 40),
        rng.uniform(-50, 50, 40),
        rng.uniform(-1e4, 1e4, 30),
        rng.uniform(-1e6, 1e6, 10),
        np.array([0.0, 1e-12, -1e-12, 1e-3, -1e-3, np.pi, -np.pi, 2 * np.pi, 1e5 + 0.5]),
    ])
    M = np.repeat(Ms[None, :], len(es), 0).ravel()
    e = np.repeat(np.array(es)[:, None], len(Ms), 1).ravel()
    cosE = np.empty_like(M)
    sinE = np.empty_like(M)
    for i in range(M.size):
        cosE[i], sinE[i] = ref.model._solve_kepler(float(M[i]), float(e[i]))
    np.savez(os.path.join(OUT, "kepler_grid.npz"), M=M, e=e, cosE=cosE, sinE=sinE)
    # _njit_kepler_rv / _compute_rv on a few (e, K, w)
    rows = []
    for (ee, K, w) in [(0.3, 25.0, 1.2), (0.8, 50.0, 2.5), (0.0, 10.0, np.pi / 4), (0.95, 7.0, -3.0)]:
        Mv = np.linspace(0, 2 * np.pi, 200)
        rows.append((ee, K, w, Mv, ref.model._compute_rv(Mv, ee, K, w)))
    np.savez(os.path.join(OUT, "compute_rv.npz"),
             params=np.array([[r[0], r[1], r[2]] for r in rows]),
             M=np.stack([r[3] for r in rows]), rv=np.stack([r[4] for r in rows]))


def gen_planets(ref):
    rng = np.random.default_rng(12)
    out = {}
    for pi, par in enumerate(["P K e w Tp", "P K e w Tc", "P K secosw sesinw Tp", "P K secosw sesinw Tc"]):
        P_ = ref.param.Parameterisation(par)
        prm, rvs = [], []
        t = np.concatenate([np.linspace(0, 100, 300), rng.uniform(2.45e6, 2.46e6, 50)])
        for k in range(12):
            e = [0.0, 0.05, 0.3, 0.6, 0.9, 0.97][k % 6]
            d = {"P": rng.uniform(0.5, 300), "K": rng.uniform(0.5, 200), "e": e,
                 "w": rng.uniform(-np.pi, np.pi), "Tp": rng.uniform(-100, 2.455e6 if k % 4 == 3 else 100)}
            conv = P_.convert_pars_from_default_parameterisation(d)
            prm.append([conv[x] for x in P_.pars])
            try:
                pl = ref.model.Planet("b", P_, {k2: float(v) for k2, v in conv.items()})
                rvs.append(pl.radial_velocity(t))
            except ValueError:   # e.g. e=0 in secosw form can land on w == pi exactly
                rvs.append(np.full(t.shape, np.nan))
        out[f"params_{pi}"] = np.array(prm)
        out[f"rv_{pi}"] = np.array(rvs)
        out[f"t_{pi}"] = t
    np.savez(os.path.join(OUT, "planet_rv.npz"), **out)


def gen_convert(ref):
    P_ = ref.param.Parameterisation("P K e w Tc")
    rng = np.random.default_rng(13)
    n = 400
    tc = rng.uniform(-1e3, 1e3, n); per = rng.uniform(0.3, 500, n)
    e = np.concatenate([rng.uniform(0, 0.99, n - 4), [0.0, 0.5, 0.999, 0.3]])
    w = np.concatenate([rng.uniform(-np.pi, np.pi, n - 4), [np.pi / 2, -np.pi, 3 * np.pi / 8, 0.0]])
    tp = np.array([P_.convert_tc_to_tp(float(a), float(b), float(c), float(d))
                   for a, b, c, d in zip(tc, per, e, w)])
    tc_back = np.array([P_.convert_tp_to_tc(float(a), float(b), float(c), float(d))
                        for a, b, c, d in zip(tp, per, e, w)])
    u = rng.uniform(-1, 1, n); v = rng.uniform(-1, 1, n)
    u[:3] = [-0.5, 0.0, 0.7]; v[:3] = [0.0, 0.0, -0.0]
    ee, ww = zip(*[P_.convert_secosw_sesinw_to_e_w(float(a), float(b)) for a, b in zip(u, v)])
    np.savez(os.path.join(OUT, "convert.npz"), tc=tc, per=per, e=e, w=w, tp=tp, tc_back=tc_back,
             u=u, v=v, e_uv=np.array(ee), w_uv=np.array(ww))


PRIOR_GRID = [
    ("Uniform", {"lower": -2.0, "upper": 3.0}),
    ("EccentricityUniform", {"upper": 0.8}),
    ("Normal", {"mean": 1.0, "std": 0.7}),
    ("TruncatedNormal", {"mean": 0.2, "std": 0.5, "lower": -0.5, "upper": 1.5}),
    ("HalfNormal", {"std": 0.3}),
    ("Rayleigh", {"scale": 0.25}),
    ("VanEylen19Mixture", {"sigma_normal": 0.049, "sigma_rayleigh": 0.26, "f": 0.08}),
    ("VanEylen19Mixture", {"sigma_normal": 0.1, "sigma_rayleigh": 0.3, "f": 0.0}),
    ("VanEylen19Mixture", {"sigma_normal": 0.1, "sigma_rayleigh": 0.3, "f": 1.0}),
    ("Beta", {"a": 0.867, "b": 3.03}),
    ("Beta", {"a": 1.0, "b": 1.0}),
    ("Beta", {"a": 2.5, "b": 0.5}),
]


def gen_priors(ref):
    x = np.concatenate([np.linspace(-3, 4, 281), [0.0, 1.0, 0.8, -0.5, 1.5, 3.0, -2.0, 1e-300]])
    vals = []
    for cls, kw in PRIOR_GRID:
        p = prior_obj(ref, (cls, kw))
        vals.append([float(p(float(xx))) for xx in x])
    np.savez(os.path.join(OUT, "priors.npz"), x=x, logp=np.array(vals))
    with open(os.path.join(OUT, "priors.json"), "w") as f:
        json.dump([[c, k] for c, k in PRIOR_GRID], f, indent=1)


# --------------------------------------------------------------------------
def posterior_case(ref, name, ds, theta_full, free_names, priors_spec, n_sub=None):
    """Evaluate the reference LogPosterior / LogLikelihood on every walker."""
    names = ds.names
    fixed = {n: float(ds.truth[n]) for n in names if n not in free_names}
    priors = {k: prior_obj(ref, v) for k, v in priors_spec.items()}
    Pz = ref.param.Parameterisation(ds.parameterisation.parameterisation)
    lpost = ref.fit.LogPosterior(ds.planet_letters, Pz, priors, fixed, list(free_names),
                                 ds.time, ds.vel, ds.velerr, ds.instrument,
                                 np.array(ds.unique_instruments), ds.t0)
    free_idx = [names.index(n) for n in free_names]
    theta_free = theta_full[:, free_idx]
    lp = np.empty(len(theta_full)); ll = np.empty(len(theta_full))
    for i in range(len(theta_full)):
        d = dict(zip(free_names, theta_full[i, free_idx]))
        lp[i] = lpost.log_probability(d)
        ll[i] = lpost.log_likelihood(fixed | d)
    meta = {"name": name, "names": names, "free_names": list(free_names), "fixed": fixed,
            "priors": priors_spec, "planet_letters": ds.planet_letters,
            "parameterisation": ds.parameterisation.parameterisation,
            "unique_instruments": list(ds.unique_instruments), "t0": ds.t0,
            "jacobian": lpost._logprob_jacobian_correction,
            "renorm": float(lpost._logprob_prior_renorm_correction)}
    np.savez(os.path.join(OUT, f"logpost_{name}.npz"), time=ds.time, vel=ds.vel, velerr=ds.velerr,
             inst_idx=ds.inst_idx, instrument=ds.instrument.astype("U16"), theta_full=theta_full,
             theta_free=theta_free, log_prob=lp, log_like=ll, meta=np.array(json.dumps(meta)))
    print(f"{name}: W={len(theta_full)} N={len(ds.time)} finite={np.isfinite(lp).sum()} "
          f"ll_finite={np.isfinite(ll).sum()}")


def uniform_around(ds, names, width=0.5):
    spec = {}
    for n in names:
        v = ds.truth[n]
        base = n.split("_")[0]
        if base in ("K",):
            spec[n] = ("Uniform", {"lower": 0.0, "upper": 2 * v + 10})
        elif base == "jit":
            spec[n] = ("Uniform", {"lower": 0.0, "upper": 10.0})
        elif base == "e":
            spec[n] = ("EccentricityUniform", {"upper": 1.0})
        elif base == "w":
            spec[n] = ("Uniform", {"lower": -np.pi, "upper": np.pi})
        elif base in ("secosw", "sesinw"):
            spec[n] = ("Uniform", {"lower": -1.0, "upper": 1.0})
        else:
            spec[n] = ("Uniform", {"lower": v - width * abs(v) - 5, "upper": v + width * abs(v) + 5})
    return spec


def gen_logpost(ref):
    # A: config-2 shape (1 planet, 256 epochs, P K e w Tp), bench walker ball subset
    ds = make_dataset(1, 256, 1, seed=2)
    th = make_walkers(ds, 4096, seed=2)[:256]
    free = [n for n in ds.names if n not in ("gd", "gdd")]
    posterior_case(ref, "cfg2", ds, th, free, uniform_around(ds, free))

    # B: config-3 shape (3 planets, 1024 epochs, 2 instruments), mixed prior classes
    ds = make_dataset(3, 1024, 2, seed=3)
    th = make_walkers(ds, 16384, seed=3)[:96]
    free = [n for n in ds.names if n not in ("gd", "gdd")]
    spec = uniform_around(ds, free)
    spec["P_b"] = ("Normal", {"mean": ds.truth["P_b"], "std": 0.1 * ds.truth["P_b"]})
    spec["K_c"] = ("TruncatedNormal", {"mean": ds.truth["K_c"], "std": 5.0, "lower": 0.0,
                                       "upper": 3 * ds.truth["K_c"]})
    spec["e_b"] = ("VanEylen19Mixture", {"sigma_normal": 0.049, "sigma_rayleigh": 0.26, "f": 0.08})
    spec["e_c"] = ("Beta", {"a": 0.867, "b": 3.03})
    spec["e_d"] = ("HalfNormal", {"std": 0.5})
    spec["jit_HARPS"] = ("HalfNormal", {"std": 3.0})
    spec["jit_HIRES"] = ("Rayleigh", {"scale": 2.0})
    posterior_case(ref, "cfg3", ds, th, free, spec)

    # C: config-4 shape (2 planets, 512 epochs) in secosw/sesinw/Tc, U(-1,1) priors (CASE_2)
    ds = make_dataset(2, 512, 1, seed=4, parameterisation="P K secosw sesinw Tc")
    th = make_walkers(ds, 512, seed=4)[:192]
    th[5, ds.names.index("sesinw_b")] = 0.0          # w = pi exactly -> -inf
    th[5, ds.names.index("secosw_b")] = -0.3
    th[6, ds.names.index("sesinw_b")] = -0.0         # w = -pi -> valid
    th[6, ds.names.index("secosw_b")] = -0.3
    th[7, ds.names.index("secosw_c")] = 0.8          # u^2+v^2 >= 1
    th[7, ds.names.index("sesinw_c")] = 0.7
    free = [n for n in ds.names if n not in ("gd", "gdd")]
    posterior_case(ref, "cfg4", ds, th, free, uniform_around(ds, free))

    # D: CASE_3 -- sample in secosw/sesinw/Tp, priors on (e, w); trend on; 2 instruments
    ds = make_dataset(2, 200, 2, seed=21, parameterisation="P K secosw sesinw Tp", trend=True)
    th = make_walkers(ds, 160, seed=21)
    th[3, ds.names.index("secosw_b")] = 0.9
    th[3, ds.names.index("sesinw_b")] = 0.6
    th[4, ds.names.index("sesinw_c")] = 0.0
    th[4, ds.names.index("secosw_c")] = -0.2
    free = list(ds.names)
    spec = {}
    for n in free:
        base = n.split("_")[0]
        if base == "secosw":
            spec["e_" + n.split("_")[1]] = ("Beta", {"a": 0.867, "b": 3.03})
        elif base == "sesinw":
            spec["w_" + n.split("_")[1]] = ("Uniform", {"lower": -np.pi, "upper": np.pi})
    for n, v in uniform_around(ds, [n for n in free if n.split("_")[0] not in ("secosw", "sesinw")]).items():
        spec[n] = v
    spec["gd"] = ("Normal", {"mean": 0.0, "std": 0.1})
    spec["gdd"] = ("Normal", {"mean": 0.0, "std": 1e-3})
    posterior_case(ref, "case3", ds, th, free, spec)

    # E: P K e w Tc with circular walkers (e == 0 -> NumPy branch, model.py:239-242)
    ds = make_dataset(1, 100, 1, seed=31, parameterisation="P K e w Tc")
    th = make_walkers(ds, 128, seed=31)
    th[::4, ds.names.index("e_b")] = 0.0
    th[1, ds.names.index("w_b")] = np.pi           # w == pi -> -inf
    th[2, ds.names.index("w_b")] = -np.pi          # valid
    free = [n for n in ds.names if n not in ("gd", "gdd")]
    posterior_case(ref, "pkewtc", ds, th, free, uniform_around(ds, free))

    # F: BJD-scale times (no range reduction in the reference), tiny epoch counts
    for nep, nm in [(1, "n1"), (7, "n7"), (129, "bjd")]:
        ds = make_dataset(2, nep, 1, seed=41 + nep, t_offset=2.457e6 if nm == "bjd" else 0.0)
        th = make_walkers(ds, 64, seed=41 + nep)
        free = [n for n in ds.names if n not in ("gd", "gdd")]
        posterior_case(ref, nm, ds, th, free, uniform_around(ds, free))

    # G: 51 Peg b (config 1): real ELODIE data, e/w/jit/trend fixed, Tc param
    gen_51peg(ref)


def gen_51peg(ref):
    import pandas as pd
    from ravest_amd.param import Parameterisation, full_param_names
    from ravest_amd.synth import Dataset
    data = pd.read_csv(os.path.join(OUT, "51Pegb.txt"), delimiter=r"\s+")
    t = data["time"].to_numpy() - 2457000
    vel = data["vel"].to_numpy(); err = data["verr"].to_numpy()
    inst = data["tel"].to_numpy().astype(str)
    par = Parameterisation("P K e w Tc")
    uniq = sorted(set(inst))
    truth = {"P_b": 4.2308, "K_b": 55.9, "e_b": 0.0, "w_b": np.pi / 2, "Tc_b": 2456325.94 - 2457000,
             "g_ELODIE": float(np.median(vel)), "jit_ELODIE": 0.0, "gd": 0.0, "gdd": 0.0}
    ds = Dataset(time=t, vel=vel, velerr=err, instrument=inst, unique_instruments=uniq,
                 inst_idx=np.zeros(len(t), np.int32), t0=float(np.mean(t)), planet_letters=["b"],
                 parameterisation=par, truth=truth, names=full_param_names(["b"], par, uniq))
    rng = np.random.default_rng(51)
    W = 64
    th = np.array([[truth[n] for n in ds.names]] * W)
    for n, s in [("P_b", 1e-4), ("K_b", 1.0), ("Tc_b", 0.01), ("g_ELODIE", 1.0)]:
        th[:, ds.names.index(n)] += s * rng.standard_normal(W)
    free = ["P_b", "K_b", "Tc_b", "g_ELODIE"]
    spec = {"P_b": ("Uniform", {"lower": 4.1, "upper": 4.3}),
            "K_b": ("Uniform", {"lower": 0.0, "upper": 100.0}),
            "Tc_b": ("Uniform", {"lower": truth["Tc_b"] - 2.0, "upper": truth["Tc_b"] + 2.0}),
            "g_ELODIE": ("Uniform", {"lower": truth["g_ELODIE"] - 60, "upper": truth["g_ELODIE"] + 60})}
    posterior_case(ref, "51peg", ds, th, free, spec)


# --------------------------------------------------------------------------
def _dense_gp_loglike(kernel, time_array, vel_array, verr_squared_array, mean_model):
    """Stand-in for GPLogLikelihood._compute_gp_log_likelihood (fit.py:8045-8060): tinygp 0.3's
    GaussianProcess(kernel, X, diag).log_probability(y) restated with a dense fp64 Cholesky
    (DirectSolver).  Everything around it -- the mean model, the jitter diagonal, the posterior's
    checks, priors, hyperpriors and corrections -- is the reference's own code."""
    from scipy.linalg import cholesky, solve_triangular
    t = np.asarray(time_array, np.float64)
    K = kernel.evaluate(np.subtract.outer(t, t))
    K[np.diag_indices(len(t))] += np.asarray(verr_squared_array)
    r = np.asarray(vel_array) - np.asarray(mean_model)
    try:
        L = cholesky(K, lower=True, check_finite=False)
    except np.linalg.LinAlgError:
        return np.nan
    alpha = solve_triangular(L, r, lower=True, check_finite=False)
    return -0.5 * alpha @ alpha - np.sum(np.log(np.diag(L))) - 0.5 * len(t) * np.log(2 * np.pi)


def gp_posterior_case(ref, name, ds, theta_full, hyper, free_names, free_hyper, priors_spec, hyper_spec,
                      fixed_hyper):
    """Evaluate the reference GPLogPosterior (fit.py:7596-7939) on every walker."""
    import ravest.gp
    names = ds.names
    fixed = {n: float(ds.truth[n]) for n in names if n not in free_names}
    priors = {k: prior_obj(ref, v) for k, v in priors_spec.items()}
    hyperpriors = {k: prior_obj(ref, v) for k, v in hyper_spec.items()}
    Pz = ref.param.Parameterisation(ds.parameterisation.parameterisation)
    kern = ravest.gp.GPKernel("Quasiperiodic")
    ref.fit.GPLogLikelihood._compute_gp_log_likelihood = staticmethod(_dense_gp_loglike)
    gpost = ref.fit.GPLogPosterior(ds.planet_letters, Pz, kern, priors, hyperpriors, fixed, fixed_hyper,
                                   list(free_names), list(free_hyper), ds.time, ds.vel, ds.velerr, ds.t0,
                                   ds.instrument, list(ds.unique_instruments))
    hnames = ["gp_amp", "gp_lambda_e", "gp_lambda_p", "gp_period"]
    free_idx = [names.index(n) for n in free_names]
    hidx = [hnames.index(n) for n in free_hyper]
    x = np.concatenate([theta_full[:, free_idx], hyper[:, hidx]], axis=1)
    lp = np.empty(len(x)); ll = np.empty(len(x))
    for i in range(len(x)):
        d = dict(zip(list(free_names) + list(free_hyper), x[i]))
        lp[i] = gpost.log_probability(d)
        allp = fixed | {n: d[n] for n in free_names}
        allh = dict(fixed_hyper) | {n: d[n] for n in free_hyper}
        try:
            ll[i] = gpost.gp_log_likelihood(allp, allh)
        except Exception:
            ll[i] = np.nan
    meta = {"name": name, "names": names, "free_names": list(free_names), "free_hyper": list(free_hyper),
            "fixed": fixed, "fixed_hyper": dict(fixed_hyper), "priors": priors_spec, "hyperpriors": hyper_spec,
            "planet_letters": ds.planet_letters, "parameterisation": ds.parameterisation.parameterisation,
            "unique_instruments": list(ds.unique_instruments), "t0": ds.t0,
            "jacobian": float(gpost._logprob_jacobian_correction),
            "renorm": float(gpost._logprob_prior_renorm_correction)}
    np.savez(os.path.join(OUT, f"gppost_{name}.npz"), time=ds.time, vel=ds.vel, velerr=ds.velerr,
             inst_idx=ds.inst_idx, instrument=ds.instrument.astype("U16"), theta_full=theta_full, hyper=hyper,
             x=x, log_prob=lp, log_like=ll, meta=np.array(json.dumps(meta)))
    print(f"gp {name}: W={len(x)} N={len(ds.time)} finite={np.isfinite(lp).sum()} ll_finite={np.isfinite(ll).sum()}")


def gen_gp_logpost(ref):
    def hyper_block(rng, W):
        return np.column_stack([rng.uniform(2, 6, W), rng.uniform(30, 120, W), rng.uniform(0.3, 1.0, W),
                                rng.uniform(10, 40, W)])
    hnames = ["gp_amp", "gp_lambda_e", "gp_lambda_p", "gp_period"]
    # A: 1 planet, P K e w Tp, every hyperparameter free; invalid jitter / hyper / eccentricity rows
    ds = make_dataset(1, 120, 1, seed=61)
    rng = np.random.default_rng(61)
    th = make_walkers(ds, 80, seed=61, scale=0.002)
    th[:, ds.names.index("jit_HARPS")] = np.abs(th[:, ds.names.index("jit_HARPS")])
    hy = hyper_block(rng, 80)
    th[1, ds.names.index("jit_HARPS")] = -0.5          # jitter < 0
    hy[2, 0] = -1.0                                     # gp_amp <= 0 (hyperparameter validity)
    hy[3, 2] = 0.0                                      # gp_lambda_p == 0
    hy[4, 1] = 500.0                                    # outside its hyperprior
    th[5, ds.names.index("e_b")] = 1.2                  # invalid planet
    free = [n for n in ds.names if n not in ("gd", "gdd")]
    hspec = {"gp_amp": ("Uniform", {"lower": 0.0, "upper": 10.0}),
             "gp_lambda_e": ("Uniform", {"lower": 1.0, "upper": 200.0}),
             "gp_lambda_p": ("TruncatedNormal", {"mean": 0.6, "std": 0.3, "lower": 0.05, "upper": 2.0}),
             "gp_period": ("Normal", {"mean": 25.0, "std": 10.0})}
    gp_posterior_case(ref, "a", ds, th, hy, free, hnames, uniform_around(ds, free), hspec, {})
    # B: 2 planets, 2 instruments, secosw/sesinw/Tc with U(-1, 1) priors (CASE_2), gp_period fixed
    ds = make_dataset(2, 160, 2, seed=62, parameterisation="P K secosw sesinw Tc")
    rng = np.random.default_rng(62)
    th = make_walkers(ds, 64, seed=62, scale=0.002)
    for inst in ds.unique_instruments:
        j = ds.names.index(f"jit_{inst}")
        th[:, j] = np.abs(th[:, j])
    hy = hyper_block(rng, 64)
    hy[:, 3] = 23.0
    free = [n for n in ds.names if n not in ("gd", "gdd")]
    fh = ["gp_amp", "gp_lambda_e", "gp_lambda_p"]
    hspec = {"gp_amp": ("HalfNormal", {"std": 5.0}), "gp_lambda_e": ("Rayleigh", {"scale": 80.0}),
             "gp_lambda_p": ("Uniform", {"lower": 0.1, "upper": 1.5})}
    gp_posterior_case(ref, "b", ds, th, hy, free, fh, uniform_around(ds, free), hspec, {"gp_period": 23.0})
    # C: CASE_3 -- secosw/sesinw/Tp sampled, priors on (e, w); trend free
    ds = make_dataset(1, 200, 1, seed=63, parameterisation="P K secosw sesinw Tp", trend=True)
    rng = np.random.default_rng(63)
    th = make_walkers(ds, 48, seed=63, scale=0.002)
    th[:, ds.names.index("jit_HARPS")] = np.abs(th[:, ds.names.index("jit_HARPS")])
    th[3, ds.names.index("secosw_b")] = 0.9            # conversion ValueError (e >= 1)
    th[3, ds.names.index("sesinw_b")] = 0.6
    hy = hyper_block(rng, 48)
    free = list(ds.names)
    spec = {"e_b": ("Beta", {"a": 0.867, "b": 3.03}), "w_b": ("Uniform", {"lower": -np.pi, "upper": np.pi})}
    for n, v in uniform_around(ds, [n for n in free if n.split("_")[0] not in ("secosw", "sesinw")]).items():
        spec[n] = v
    spec["gd"] = ("Normal", {"mean": 0.0, "std": 0.1})
    spec["gdd"] = ("Normal", {"mean": 0.0, "std": 1e-3})
    hspec = {k: ("Uniform", {"lower": 0.0, "upper": 500.0}) for k in hnames}
    gp_posterior_case(ref, "c", ds, th, hy, free, hnames, spec, hspec, {})


if __name__ == "__main__":
    ref = import_reference()
    os.makedirs(OUT, exist_ok=True)
    if sys.argv[1:] == ["gp"]:
        gen_gp_logpost(ref)
        sys.exit(0)
    gen_gp_logpost(ref)
    gen_kepler(ref)
    gen_planets(ref)
    gen_convert(ref)
    gen_priors(ref)
    gen_logpost(ref)
    print("golden fixtures written to", OUT)
