"""spectralmc_amd — MI355X-native (gfx950) GbmCVNNPricer training hot path.

A from-scratch re-design of Tuee22/SpectralMC's training loop (Sobol contracts -> GBM
Monte-Carlo -> characteristic-function targets -> complex-valued MLP + Adam) on hand-written
HIP kernels (libspectralmc_hip.so, C ABI in include/spectralmc_hip.h), PyTorch-ROCm for the
CVNN and RCCL for data-parallel training.  The reference's Python API is mirrored module by
module (gbm, gbm_trainer, sobol_sampler, cvnn, cvnn_factory, models, result, ...); the
``spectralmc`` package re-exports it under the reference's import paths.
"""

__version__ = "0.1.0"
