"""Priors: the host-side mirror of ``ravest.prior`` (src/ravest/prior.py:1-511).

Every class keeps the reference's constructor validation, scalar ``__call__``
(same formula, same scipy call, same -inf bounds) and ``__repr__``.  Each also
has ``logpdf(x)``, the same computation vectorised over a walker column, used
by the batched log-posterior (``posterior.LogPrior.batch``).  The vectorised
values are checked element-for-element against the reference's scalar calls
(tests/test_host.py, golden tests/golden/priors.npz and beta_reference.json).
"""
from __future__ import annotations

import numpy as np
from scipy.special import gammaln, logsumexp, xlog1py, xlogy
from scipy.stats import halfnorm, rayleigh, truncnorm

PRIOR_FUNCTIONS = ["Uniform", "EccentricityUniform", "Normal", "TruncatedNormal", "HalfNormal", "Rayleigh",
                   "VanEylen19Mixture", "Beta"]


def _arr(x):
    return np.asarray(x, dtype=np.float64)


class Uniform:
    """Closed interval [lower, upper] (prior.py:9-68)."""

    def __init__(self, lower: float, upper: float) -> None:
        if not np.isfinite(lower):
            raise ValueError(f"Lower bound must be finite, got {lower}")
        if not np.isfinite(upper):
            raise ValueError(f"Upper bound must be finite, got {upper}")
        if lower >= upper:
            raise ValueError(f"Lower bound ({lower}) must be less than upper bound ({upper})")
        self.lower = lower
        self.upper = upper

    def __call__(self, value: float) -> float:
        if value < self.lower or value > self.upper:
            return -np.inf
        return -np.log(self.upper - self.lower)

    def logpdf(self, x):
        x = _arr(x)
        return np.where((x < self.lower) | (x > self.upper), -np.inf, -np.log(self.upper - self.lower))

    def __repr__(self) -> str:
        return f"Uniform(lower={self.lower}, upper={self.upper})"


class EccentricityUniform:
    """Half-open [0, upper) (prior.py:71-125)."""

    def __init__(self, upper: float) -> None:
        if upper > 1:
            raise ValueError("Upper bound of eccentricity must be less than or equal to 1.")
        if upper <= 0:
            raise ValueError("Upper bound of eccentricity must be greater than 0.")
        self.upper = upper

    def __call__(self, value: float) -> float:
        if value < 0 or value >= self.upper:
            return -np.inf
        return -np.log(self.upper)

    def logpdf(self, x):
        x = _arr(x)
        return np.where((x < 0) | (x >= self.upper), -np.inf, -np.log(self.upper))

    def __repr__(self) -> str:
        return f"EccentricityUniform(upper={self.upper})"


class Normal:
    """prior.py:128-175."""

    def __init__(self, mean: float, std: float) -> None:
        if std <= 0:
            raise ValueError(f"Standard deviation must be positive, got {std}")
        self.mean = mean
        self.std = std
        self._log_norm_const = 0.5 * np.log((self.std ** 2) * 2. * np.pi)

    def __call__(self, value: float) -> float:
        return -0.5 * ((value - self.mean) / self.std) ** 2 - self._log_norm_const

    def logpdf(self, x):
        return -0.5 * ((_arr(x) - self.mean) / self.std) ** 2 - self._log_norm_const

    def __repr__(self) -> str:
        return f"Normal(mean={self.mean}, std={self.std})"


class TruncatedNormal:
    """prior.py:178-249 (scipy truncnorm.logpdf inside [lower, upper])."""

    def __init__(self, mean: float, std: float, lower: float, upper: float) -> None:
        if std <= 0:
            raise ValueError("Standard deviation must be positive")
        if lower >= upper:
            raise ValueError("Lower bound must be less than upper bound")
        self.mean = mean
        self.std = std
        self.lower = lower
        self.upper = upper
        self._a = (lower - mean) / std
        self._b = (upper - mean) / std

    def __call__(self, value: float) -> float:
        if value < self.lower or value > self.upper:
            return -np.inf
        return truncnorm.logpdf(value, self._a, self._b, loc=self.mean, scale=self.std)

    def logpdf(self, x):
        x = _arr(x)
        out = np.full(x.shape, -np.inf)
        m = ~((x < self.lower) | (x > self.upper))
        if m.any():
            out[m] = truncnorm.logpdf(x[m], self._a, self._b, loc=self.mean, scale=self.std)
        return out

    def __repr__(self) -> str:
        return f"TruncatedNormal(mean={self.mean}, std={self.std}, lower={self.lower}, upper={self.upper})"


class HalfNormal:
    """prior.py:252-306."""

    def __init__(self, std: float) -> None:
        if std <= 0:
            raise ValueError(f"Standard deviation must be positive, got {std}")
        self.std = float(std)

    def __call__(self, value: float) -> float:
        if value < 0.0:
            return -np.inf
        return halfnorm.logpdf(value, scale=self.std)

    def logpdf(self, x):
        x = _arr(x)
        out = np.full(x.shape, -np.inf)
        m = ~(x < 0.0)
        if m.any():
            out[m] = halfnorm.logpdf(x[m], scale=self.std)
        return out

    def __repr__(self) -> str:
        return f"HalfNormal(std={self.std})"


class Rayleigh:
    """prior.py:309-362."""

    def __init__(self, scale: float) -> None:
        if scale <= 0:
            raise ValueError(f"Scale parameter must be positive, got {scale}")
        self.scale = float(scale)

    def __call__(self, value: float) -> float:
        if value < 0.0:
            return -np.inf
        return rayleigh.logpdf(value, scale=self.scale)

    def logpdf(self, x):
        x = _arr(x)
        out = np.full(x.shape, -np.inf)
        m = ~(x < 0.0)
        if m.any():
            out[m] = rayleigh.logpdf(x[m], scale=self.scale)
        return out

    def __repr__(self) -> str:
        return f"Rayleigh(scale={self.scale})"


class VanEylen19Mixture:
    """(1-f) HalfNormal + f Rayleigh (prior.py:365-443)."""

    def __init__(self, sigma_normal: float, sigma_rayleigh: float, f: float) -> None:
        if sigma_normal <= 0:
            raise ValueError(f"sigma_normal must be positive, got {sigma_normal}")
        if sigma_rayleigh <= 0:
            raise ValueError(f"sigma_rayleigh must be positive, got {sigma_rayleigh}")
        if not (0 <= f <= 1):
            raise ValueError(f"Mixing fraction f must be between 0 and 1, got {f}")
        self.sigma_normal = float(sigma_normal)
        self.sigma_rayleigh = float(sigma_rayleigh)
        self.f = float(f)

    def __call__(self, value: float) -> float:
        if value < 0.0:
            return -np.inf
        log_halfnorm = halfnorm.logpdf(value, scale=self.sigma_normal)
        log_rayleigh = rayleigh.logpdf(value, scale=self.sigma_rayleigh)
        return logsumexp([log_halfnorm, log_rayleigh], b=[1 - self.f, self.f])

    def logpdf(self, x):
        x = _arr(x)
        out = np.full(x.shape, -np.inf)
        m = ~(x < 0.0)
        if m.any():
            a = np.stack([halfnorm.logpdf(x[m], scale=self.sigma_normal),
                          rayleigh.logpdf(x[m], scale=self.sigma_rayleigh)])
            b = np.array([1 - self.f, self.f])[:, None]
            out[m] = logsumexp(a, axis=0, b=b)
        return out

    def __repr__(self) -> str:
        return (f"VanEylen19Mixture(sigma_normal={self.sigma_normal}, sigma_rayleigh={self.sigma_rayleigh}, "
                f"f={self.f})")


class Beta:
    """prior.py:446-511."""

    def __init__(self, a: float, b: float) -> None:
        if not a > 0:
            raise ValueError(f"Value of a > 0 required, got {a}")
        if not b > 0:
            raise ValueError(f"Value of b > 0 required, got {b}")
        self.a = float(a)
        self.b = float(b)
        self._log_beta = gammaln(self.a) + gammaln(self.b) - gammaln(self.a + self.b)

    def __call__(self, value: float) -> float:
        if value < 0.0 or value > 1.0:
            return -np.inf
        return xlogy(self.a - 1, value) + xlog1py(self.b - 1, -value) - self._log_beta

    def logpdf(self, x):
        x = _arr(x)
        out = np.full(x.shape, -np.inf)
        m = ~((x < 0.0) | (x > 1.0))
        if m.any():
            out[m] = xlogy(self.a - 1, x[m]) + xlog1py(self.b - 1, -x[m]) - self._log_beta
        return out

    def __repr__(self) -> str:
        return f"Beta(a={self.a}, b={self.b})"


# Public constructor attributes of ravest's built-in priors (src/ravest/prior.py:39-488): a
# prior object of the reference's own classes is re-expressed from exactly these, so the
# derived constants (_log_norm_const, _a/_b, _log_beta) come from this module's
# constructors, i.e. the reference's expressions, never from another object's privates.
PUBLIC_ATTRS = {"Uniform": ("lower", "upper"), "EccentricityUniform": ("upper",), "Normal": ("mean", "std"),
                "TruncatedNormal": ("mean", "std", "lower", "upper"), "HalfNormal": ("std",),
                "Rayleigh": ("scale",), "VanEylen19Mixture": ("sigma_normal", "sigma_rayleigh", "f"),
                "Beta": ("a", "b")}


def as_prior(prior):
    """The drop-in boundary for priors: an instance of this module's classes is returned as is;
    an object whose class is named like one of ravest's built-in priors and carries that
    prior's public attributes (ravest.prior.Uniform(lower, upper), ...) becomes the
    equivalent built-in here (same validation, same formulas); anything else is a custom
    callable and stays one (host path, evaluated per walker like the reference)."""
    if is_builtin(prior):
        return prior
    if isinstance(prior, _BUILTIN):   # a user subclass of a built-in: its overrides are honoured
        return prior                  # (host path, per-walker __call__), never the parent's formula
    name = type(prior).__name__
    attrs = PUBLIC_ATTRS.get(name)
    if attrs is not None and all(hasattr(prior, a) for a in attrs):
        return globals()[name](*(getattr(prior, a) for a in attrs))
    return prior


def as_priors(priors: dict) -> dict:
    """``as_prior`` over a priors dict, keeping its key order (the reference sums in it)."""
    return {k: as_prior(v) for k, v in priors.items()}


def logpdf_vec(prior, x) -> np.ndarray:
    """Vectorised log-prior for any prior: built-ins use ``logpdf``; user callables are
    evaluated per element (the reference's per-walker semantics)."""
    if is_builtin(prior):
        return prior.logpdf(x)
    x = _arr(x)
    return np.array([float(prior(float(v))) for v in x.ravel()]).reshape(x.shape)


_BUILTIN = (Uniform, EccentricityUniform, Normal, TruncatedNormal, HalfNormal, Rayleigh, VanEylen19Mixture, Beta)


def is_builtin(prior) -> bool:
    """Exactly one of the built-in classes (a subclass may override __call__ / logpdf, so it is
    a custom callable: host path, its own formula)."""
    return type(prior) in _BUILTIN


# ---- device form (include/rvk_post.h RVK_PRIOR_*) --------------------------------------------
try:
    from scipy.stats._continuous_distns import _norm_pdf_logC as _LOG_SQRT_2PI
except ImportError:  # pragma: no cover - same expression as scipy's
    _LOG_SQRT_2PI = float(np.log(np.sqrt(2 * np.pi)))
_HALF_LOG_2_OVER_PI = float(0.5 * np.log(2.0 / np.pi))    # scipy halfnorm._logpdf constant


def device_params(prior):
    """(kind, p[8]) of a built-in prior for the device log-posterior: the constants the
    reference computes once (or scipy computes per call), evaluated here with the same
    expressions, so the device repeats the reference's arithmetic.  A prior that is not
    one of the built-in classes raises NotImplementedError: custom callables stay on the
    host path (posterior.LogPosterior.log_probability_batch)."""
    from . import _lib
    prior = as_prior(prior)
    p = np.zeros(_lib.PRIOR_NPAR)
    name = type(prior).__name__
    if not is_builtin(prior):
        raise NotImplementedError(f"prior {prior!r} ({name}) is not one of the built-in classes (a subclass "
                                  f"keeps its own formula on the host path); built-in priors: {PRIOR_FUNCTIONS}")
    if isinstance(prior, Uniform):
        p[:3] = prior.lower, prior.upper, -np.log(prior.upper - prior.lower)
    elif isinstance(prior, EccentricityUniform):
        p[:2] = prior.upper, -np.log(prior.upper)
    elif isinstance(prior, Normal):
        p[:3] = prior.mean, prior.std, prior._log_norm_const
    elif isinstance(prior, TruncatedNormal):
        from scipy.stats._continuous_distns import _log_gauss_mass
        p[:7] = (prior.mean, prior.std, prior.lower, prior.upper, _LOG_SQRT_2PI,
                 float(_log_gauss_mass(np.float64(prior._a), np.float64(prior._b))), np.log(prior.std))
    elif isinstance(prior, HalfNormal):
        p[:3] = prior.std, np.log(prior.std), _HALF_LOG_2_OVER_PI
    elif isinstance(prior, Rayleigh):
        p[:2] = prior.scale, np.log(prior.scale)
    elif isinstance(prior, VanEylen19Mixture):
        p[:7] = (prior.sigma_normal, np.log(prior.sigma_normal), prior.sigma_rayleigh, np.log(prior.sigma_rayleigh),
                 1 - prior.f, prior.f, _HALF_LOG_2_OVER_PI)
    elif isinstance(prior, Beta):
        p[:3] = prior.a, prior.b, prior._log_beta
    else:
        raise NotImplementedError(f"prior {prior!r} ({name}) has no device form; built-in priors: "
                                  f"{PRIOR_FUNCTIONS}")
    return _lib.PRIOR_KIND[name], p
