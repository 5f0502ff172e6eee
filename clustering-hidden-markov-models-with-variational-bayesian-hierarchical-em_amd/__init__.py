"""vbhem_amd -- MI355X-native VBHEM-H3M E-step (drop-in for the reference's
src/vbhem/vbhem_hmm_bwd_fwd_mex hot path) and the EM loop around it.

The directory name is not a Python identifier; import it through the repo-root
helper ``pkgload.load()`` (registers it as ``vbhem_amd``).
"""
from .h3m import (COV_DIAG, COV_FULL, CONFIGS, BaseSet, Posterior, baseem_draws,  # noqa: F401
                  baseem_init, clip_hyps, default_options, hmms_to_h3m_hem, synth_base_set,
                  synth_workload, weighted_kmeans, wtkmeans_init, wtkmeans_points,
                  gmm_mix_hier_em, gmmnew_init)
from . import host  # noqa: F401

__version__ = "0.1.0"


def engine(*args, **kw):
    """EStepEngine(...) -- imported lazily (loads the HIP library)."""
    from .estep import EStepEngine
    return EStepEngine(*args, **kw)
