"""ravest_amd: MI355X-native RV log-likelihood engine for ravest.

The hot path (Kepler solve -> Keplerian RV sum -> trend/offsets ->
jittered Gaussian log-likelihood, per walker) runs as a HIP kernel for gfx950
behind the C-ABI declared in ``include/rvk.h`` (library ``lib/librvk.so``).
The host-side classes mirror ravest's ``LogPosterior`` / ``LogLikelihood`` /
``LogPrior`` / ``Parameterisation`` / priors.
"""
__version__ = "0.1.0"
