"""impala_amd — MI355X-native IMPALA learner (HIP/CDNA4 kernels behind a C-ABI).

Drop-in for the learner path of d3sm0/impala: ``agents/core.py`` Learner/Builder plugin API,
``agents/impala/{builder,learning}.py`` ImpalaBuilder/ImpalaLearner, and
``models/distributed_models.py`` AtariPPOModel.  See DESIGN.md.
"""
from impala_amd.model import AtariPPOModel, param_count, param_specs  # noqa: F401

__all__ = ["AtariPPOModel", "param_count", "param_specs"]
