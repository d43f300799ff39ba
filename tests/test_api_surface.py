"""The reference e2e test's import closure resolves against this build (SURVEY.md §8(b)
table: module -> symbols), through the ``spectralmc`` alias package."""

from __future__ import annotations

import importlib

import pytest

CLOSURE = {
    "spectralmc.gbm": ["BlackScholes", "BlackScholesConfig", "SimulationParams", "ThreadsPerBlock",
                       "build_black_scholes_config", "build_simulation_params"],
    "spectralmc.gbm_trainer": ["ComplexValuedModel", "GbmCVNNPricer", "GbmCVNNPricerConfig", "TrainingConfig",
                               "build_training_config"],
    "spectralmc.cvnn_factory": ["ActivationCfg", "ActivationKind", "ExplicitWidth", "LayerCfg", "LinearCfg",
                                "build_cvnn_config", "build_model"],
    "spectralmc.effects": ["ForwardNormalization", "PathScheme"],
    "spectralmc.models.torch": ["AdamOptimizerState", "Device", "FullPrecisionDType", "default_dtype"],
    "spectralmc.models.numerical": ["Precision"],
    "spectralmc.sobol_sampler": ["BoundSpec", "DomainBounds", "build_bound_spec", "build_domain_bounds"],
    "spectralmc.validation": ["validate_model"],
    "spectralmc.result": ["Success", "Failure"],
    "spectralmc.storage": ["AsyncBlockchainModelStore", "commit_snapshot", "load_snapshot_from_checkpoint"],
}


@pytest.mark.parametrize("module", sorted(CLOSURE))
def test_reference_import_closure(module: str) -> None:
    mod = importlib.import_module(module)
    missing = [s for s in CLOSURE[module] if not hasattr(mod, s)]
    assert not missing, f"{module} lacks {missing}"
    assert mod.__name__.startswith(("spectralmc_amd", "spectralmc"))


def test_alias_serves_this_build() -> None:
    import spectralmc.gbm_trainer as a
    import spectralmc_amd.gbm_trainer as b

    assert a is b
