"""Orbital parameterisations: the host-side mirror of ``ravest.param``.

Scalar behaviour follows the reference exactly (same names, same
``ValueError``s): ``src/ravest/param.py:5-435``.  On top of that every
conversion has a vectorised form over a walker block that returns a validity
mask instead of raising, which is what the batched log-posterior needs (the
reference maps every such ``ValueError`` to ``-inf``, ``fit.py:3478-3480`` and
``fit.py:3625-3627``).

The per-walker conversion on the hot path itself runs inside the HIP kernel
prologue (``ravest_amd/csrc/rvk_kernels.hip``); this module is used for the
prior-side conversion (Case 3 of ``fit.py:3399-3446``) and for setup.
"""
from __future__ import annotations

import numpy as np

# param.py:5-10 (ecosw/esinw are disabled in the reference, so not allowed here)
ALLOWED_PARAMETERISATIONS = ["P K e w Tp",
                             "P K e w Tc",
                             "P K secosw sesinw Tp",
                             "P K secosw sesinw Tc"]

# C-ABI codes (include/rvk.h RVK_PAR_*)
PARAMETERISATION_CODE = {p: i for i, p in enumerate(ALLOWED_PARAMETERISATIONS)}


class Parameterisation:
    """Handle conversions between orbital parameterisations (param.py:13-435)."""

    def __init__(self, parameterisation: str) -> None:
        if parameterisation not in ALLOWED_PARAMETERISATIONS:
            raise ValueError(f"parameterisation {parameterisation} not recognised. "
                             f"Must be one of {ALLOWED_PARAMETERISATIONS}")
        self.parameterisation = parameterisation
        self.pars = parameterisation.split()

    def __str__(self) -> str:
        return f"Parameterisation: {self.parameterisation}"

    def __repr__(self) -> str:
        return f"Parameterisation({self.parameterisation})"

    @property
    def code(self) -> int:
        return PARAMETERISATION_CODE[self.parameterisation]

    # ---- validators (param.py:16-105); NaN passes the '<=' tests as in the reference
    @staticmethod
    def _validate_period(per) -> None:
        if np.any(np.asarray(per) <= 0):
            raise ValueError(f"Invalid period: {per} <= 0")

    @staticmethod
    def _validate_semi_amplitude(k) -> None:
        if np.any(np.asarray(k) <= 0):
            raise ValueError(f"Invalid semi-amplitude: {k} <= 0")

    @staticmethod
    def _validate_eccentricity(e) -> None:
        e = np.asarray(e)
        if np.any(e < 0):
            raise ValueError(f"Invalid eccentricity: {e} < 0")
        if np.any(e >= 1.0):
            raise ValueError(f"Invalid eccentricity: {e} >= 1.0")

    @staticmethod
    def _validate_argument_periastron(w) -> None:
        w = np.asarray(w)
        if np.isscalar(w) or w.ndim == 0:
            if not -np.pi <= w < np.pi:
                raise ValueError(f"Invalid argument of periastron: {w} not in [-pi, +pi)")
        elif np.any(w < -np.pi) or np.any(w >= np.pi):
            raise ValueError("Invalid argument of periastron: some values not in [-pi, +pi)")

    def validate_default_parameterisation_params(self, params_dict) -> None:
        self._validate_period(params_dict["P"])
        self._validate_semi_amplitude(params_dict["K"])
        self._validate_eccentricity(params_dict["e"])
        self._validate_argument_periastron(params_dict["w"])

    def validate_planetary_params(self, params_dict) -> None:
        if self.parameterisation != "P K e w Tp":
            params_dict = self.convert_pars_to_default_parameterisation(params_dict)
        self.validate_default_parameterisation_params(params_dict)

    # ---- conversions (param.py:159-297)
    def _time_given_true_anomaly(self, true_anomaly, period, eccentricity, time_peri):
        E = 2 * np.arctan(np.sqrt((1 - eccentricity) / (1 + eccentricity)) * np.tan(true_anomaly / 2))
        M = E - (eccentricity * np.sin(E))
        return M * (period / (2 * np.pi)) + time_peri

    def convert_tp_to_tc(self, time_peri, period, eccentricity, arg_peri):
        theta_tc = (np.pi / 2) - arg_peri
        return self._time_given_true_anomaly(theta_tc, period, eccentricity, time_peri)

    def convert_tc_to_tp(self, time_conj, period, eccentricity, arg_peri):
        theta_tc = (np.pi / 2) - arg_peri
        self._validate_eccentricity(eccentricity)
        E = 2 * np.arctan(np.sqrt((1 - eccentricity) / (1 + eccentricity)) * np.tan(theta_tc / 2))
        M = E - (eccentricity * np.sin(E))
        return time_conj - (period / (2 * np.pi)) * M

    def convert_secosw_sesinw_to_e_w(self, secosw, sesinw):
        e = secosw ** 2 + sesinw ** 2
        w = np.arctan2(sesinw, secosw)
        return e, w

    def convert_e_w_to_secosw_sesinw(self, e, w):
        self._validate_eccentricity(e)
        sqrt_e = np.sqrt(e)
        return sqrt_e * np.cos(w), sqrt_e * np.sin(w)

    def convert_pars_to_default_parameterisation(self, inpars: dict) -> dict:
        p = self.parameterisation
        if p == "P K e w Tp":
            return {k: inpars[k] for k in ("P", "K", "e", "w", "Tp")}
        if p == "P K e w Tc":
            tp = self.convert_tc_to_tp(inpars["Tc"], inpars["P"], inpars["e"], inpars["w"])
            return {"P": inpars["P"], "K": inpars["K"], "e": inpars["e"], "w": inpars["w"], "Tp": tp}
        e, w = self.convert_secosw_sesinw_to_e_w(inpars["secosw"], inpars["sesinw"])
        if p == "P K secosw sesinw Tp":
            return {"P": inpars["P"], "K": inpars["K"], "e": e, "w": w, "Tp": inpars["Tp"]}
        tp = self.convert_tc_to_tp(inpars["Tc"], inpars["P"], e, w)
        return {"P": inpars["P"], "K": inpars["K"], "e": e, "w": w, "Tp": tp}

    def convert_pars_from_default_parameterisation(self, default_pars: dict) -> dict:
        p = self.parameterisation
        d = default_pars
        if p == "P K e w Tp":
            return {k: d[k] for k in self.pars}
        out = {"P": d["P"], "K": d["K"]}
        if "secosw" in p:
            out["secosw"], out["sesinw"] = self.convert_e_w_to_secosw_sesinw(d["e"], d["w"])
        else:
            out["e"], out["w"] = d["e"], d["w"]
        if p.endswith("Tc"):
            out["Tc"] = self.convert_tp_to_tc(d["Tp"], d["P"], d["e"], d["w"])
        else:
            out["Tp"] = d["Tp"]
        return out

    def log_jacobian_determinant(self) -> float:
        """param.py:428-435."""
        if "secosw" in self.parameterisation:
            return float(np.log(2))
        return 0.0

    # ---- vectorised forms (mask instead of raise)
    def to_default_vec(self, cols: dict):
        """Columns in this parameterisation -> (default columns, ok mask).

        ``ok`` is False exactly where :meth:`convert_pars_to_default_parameterisation`
        would raise (only the Tc conversion validates, param.py:208-209).
        """
        p = self.parameterisation
        P, K = np.asarray(cols["P"], float), np.asarray(cols["K"], float)
        ok = np.ones(P.shape, bool)
        if "secosw" in p:
            e, w = self.convert_secosw_sesinw_to_e_w(np.asarray(cols["secosw"], float),
                                                     np.asarray(cols["sesinw"], float))
        else:
            e, w = np.asarray(cols["e"], float), np.asarray(cols["w"], float)
        if p.endswith("Tc"):
            ok &= ~((e < 0) | (e >= 1.0))
            with np.errstate(invalid="ignore", divide="ignore"):
                theta_tc = (np.pi / 2) - w
                E = 2 * np.arctan(np.sqrt((1 - e) / (1 + e)) * np.tan(theta_tc / 2))
                M = E - (e * np.sin(E))
                Tp = np.asarray(cols["Tc"], float) - (P / (2 * np.pi)) * M
        else:
            Tp = np.asarray(cols["Tp"], float)
        return {"P": P, "K": K, "e": e, "w": w, "Tp": Tp}, ok

    @staticmethod
    def valid_default_vec(d: dict) -> np.ndarray:
        """Vector form of validate_default_parameterisation_params (param.py:88-105)."""
        P, K, e, w = d["P"], d["K"], d["e"], d["w"]
        return ~(P <= 0) & ~(K <= 0) & ~(e < 0) & ~(e >= 1.0) & ((-np.pi <= w) & (w < np.pi))


def as_parameterisation(obj) -> Parameterisation:
    """The drop-in boundary for parameterisations: a string, this module's class, or ravest's
    own ``Parameterisation`` -- or any object with its public ``.parameterisation`` string
    (src/ravest/param.py:129-151; ravest's class has no ``.code`` or vectorised forms, so
    it is re-expressed here from that string, with the reference's ValueError for an
    unknown one)."""
    if isinstance(obj, Parameterisation):
        return obj
    if isinstance(obj, str):
        return Parameterisation(obj)
    name = getattr(obj, "parameterisation", None)
    if isinstance(name, str):
        return Parameterisation(name)
    raise TypeError(f"{obj!r} is not a parameterisation: expected a string or an object with a "
                    "'.parameterisation' string (ravest.param.Parameterisation)")


def full_param_names(planet_letters, parameterisation: Parameterisation, unique_instruments) -> list:
    """Full parameter order of the C-ABI ``theta`` row (include/rvk.h)."""
    parameterisation = as_parameterisation(parameterisation)
    names = [f"{par}_{L}" for L in planet_letters for par in parameterisation.pars]
    names += [f"g_{s}" for s in unique_instruments]
    names += [f"jit_{s}" for s in unique_instruments]
    names += ["gd", "gdd"]
    return names


class Parameter:
    """Parameter value holder (param.py:597-625)."""

    def __init__(self, value: float, unit: str, fixed: bool = False) -> None:
        self.value = value
        self.unit = unit
        self.fixed = fixed

    def __repr__(self) -> str:
        return f"Parameter(value={self.value!r}, unit={self.unit!r}, fixed={self.fixed!r})"

    def __str__(self) -> str:
        return f"Parameter {self.value} {self.unit}"
