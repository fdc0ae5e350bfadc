"""The drop-in accepts ravest's OWN Parameterisation and prior objects (no GPU needed).

ravest's Fitter hands LogPosterior its own ``Parameterisation`` (only ``.parameterisation`` /
``.pars``, src/ravest/param.py:129-151) and its own prior instances (src/ravest/prior.py).
tests/_foreign.py holds stand-ins with exactly those public attributes; the classification
of the log-posterior corrections (fit.py:3306-3397), the vectorised log-prior and the
device prior slots must come out identical to the ones built from ravest_amd's classes.
When /root/reference is present (build container only), the same is checked with the
reference's real classes, imported in a subprocess by tools/gen_golden.py's recipe.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from ravest_amd import prior as P
from ravest_amd.param import Parameterisation, as_parameterisation
from ravest_amd.posterior import LogPosterior
from tests import _foreign as F
from tests._golden import load_case, logpost_cases

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ours(case):
    m = case["meta"]
    priors = {k: getattr(P, c)(**kw) for k, (c, kw) in m["priors"].items()}
    return LogPosterior(m["planet_letters"], Parameterisation(m["parameterisation"]), priors, m["fixed"],
                        m["free_names"], case["time"], case["vel"], case["velerr"], case["instrument"],
                        np.array(m["unique_instruments"]), m["t0"])


@pytest.mark.parametrize("name", logpost_cases())
def test_posterior_from_foreign_objects(name):
    case = load_case(name)
    m = case["meta"]
    lf = LogPosterior(*F.posterior_args(case))
    lo = _ours(case)
    # corrections: the reference's values recorded in the golden (CASE_2 for cfg4's Uniform(-1, 1) pairs)
    assert lf._logprob_jacobian_correction == m["jacobian"]
    assert lf._logprob_prior_renorm_correction == m["renorm"]
    assert lf._logprob_correction_breakdown == lo._logprob_correction_breakdown
    # vectorised log-prior + conversion mask: identical to the mirror-class build
    th = case["theta_free"]
    lp_f, ok_f = lf._log_prior_batch(th, lf._full(th))
    lp_o, ok_o = lo._log_prior_batch(th, lo._full(th))
    assert np.array_equal(ok_f, ok_o)
    assert np.array_equal(lp_f, lp_o)
    # and equal to the foreign objects' own scalar calls (LogPrior.__call__ path, fit.py:3672-3691)
    for i in range(0, len(th), max(1, len(th) // 16)):
        d = dict(zip(m["free_names"], th[i]))
        try:
            pd = lf._convert_params_for_prior_evaluation(d)
        except ValueError:
            assert not ok_f[i]
            continue
        ref = lf.log_prior(pd)
        assert (lp_f[i] == ref) or (np.isinf(ref) and lp_f[i] == ref) or abs(lp_f[i] - ref) <= 1e-12 * abs(ref)
    # the device prior slots are the same constants
    for k in lo._prior_order:
        kf, pf = P.device_params(lf.priors[k])
        ko, po = P.device_params(lo.priors[k])
        assert kf == ko and np.array_equal(pf, po), k


def test_case2_classified_from_foreign_uniform():
    """ravest's Uniform(-1, 1) on secosw/sesinw is CASE_2 (renorm log 4/pi), not NotImplementedError."""
    case = load_case("cfg4")
    args = list(F.posterior_args(case))
    lp = LogPosterior(*args)
    assert all(v["case"] == "CASE_2" for v in lp._logprob_correction_breakdown.values())
    # a non-Uniform(-1, 1) pair still raises the reference's NotImplementedError (fit.py:3352-3368)
    pri = dict(args[2])
    letter = args[0][0]
    pri[f"secosw_{letter}"] = F.Normal(0.0, 0.3)
    args[2] = pri
    with pytest.raises(NotImplementedError):
        LogPosterior(*args)


def test_adapters():
    p = as_parameterisation(F.Parameterisation("P K secosw sesinw Tc"))
    assert p.code == 3 and p.pars == ["P", "K", "secosw", "sesinw", "Tc"]
    with pytest.raises(ValueError):
        as_parameterisation(F.Parameterisation("P K ecosw esinw Tp"))
    with pytest.raises(TypeError):
        as_parameterisation(42)
    custom = lambda v: -0.5 * v * v          # noqa: E731  a custom callable prior stays a callable
    assert P.as_prior(custom) is custom
    u = P.Uniform(0, 1)
    assert P.as_prior(u) is u
    b = P.as_prior(F.Beta(0.867, 3.03))
    assert isinstance(b, P.Beta) and b._log_beta == F.Beta(0.867, 3.03)._log_beta
    with pytest.raises(NotImplementedError):
        P.device_params(custom)


_REF_SCRIPT = r"""
import json, sys
import numpy as np
sys.path.insert(0, {root!r})
from tools.gen_golden import import_reference
ref = import_reference()
from tests._golden import load_case, logpost_cases
from ravest_amd import prior as P
from ravest_amd.posterior import LogPosterior
out = {{}}
for name in logpost_cases():
    case = load_case(name)
    m = case["meta"]
    priors = {{k: getattr(ref.prior, c)(**kw) for k, (c, kw) in m["priors"].items()}}
    par = ref.param.Parameterisation(m["parameterisation"])
    lp = LogPosterior(m["planet_letters"], par, priors, m["fixed"], m["free_names"], case["time"], case["vel"],
                      case["velerr"], case["instrument"], np.array(m["unique_instruments"]), m["t0"])
    th = case["theta_free"]
    lpv, ok = lp._log_prior_batch(th, lp._full(th))
    # the reference's own LogPosterior, unmodified, for the prior half of log_prob
    rp = ref.fit.LogPosterior(m["planet_letters"], par, priors, m["fixed"], m["free_names"], case["time"],
                              case["vel"], case["velerr"], case["instrument"], np.array(m["unique_instruments"]),
                              m["t0"])
    bad = 0
    for i in range(len(th)):
        d = dict(zip(m["free_names"], th[i]))
        try:
            r = rp.log_prior(rp._convert_params_for_prior_evaluation(d))
        except ValueError:
            bad += int(ok[i])
            continue
        if not ((r == lpv[i]) or abs(r - lpv[i]) <= 1e-12 * abs(r)):
            bad += 1
    slots = [P.device_params(priors[k])[0] for k in lp._prior_order]
    out[name] = dict(bad=bad, jac=bool(lp._logprob_jacobian_correction == rp._logprob_jacobian_correction),
                     ren=bool(lp._logprob_prior_renorm_correction == rp._logprob_prior_renorm_correction), nslots=len(slots))
print(json.dumps(out))
"""


@pytest.mark.skipif(not os.path.isdir("/root/reference/src/ravest"), reason="reference not present (GPU box)")
def test_posterior_from_real_reference_objects():
    """ravest's real Parameterisation and prior instances (imported from /root/reference in a
    subprocess, numba stubbed) drive LogPosterior; the log-prior of every golden walker equals
    the reference LogPosterior's own log_prior, and the corrections are the reference's."""
    r = subprocess.run([sys.executable, "-c", _REF_SCRIPT.format(root=ROOT)], capture_output=True, text=True,
                       cwd=ROOT, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res and all(v["bad"] == 0 and v["jac"] and v["ren"] and v["nslots"] > 0 for v in res.values()), res
