"""Batch-norm / residual CVNN architectures of the golden vectors (cvnn.py:213-480).

Each builder takes a module namespace with the reference's class names (the reference's
``spectralmc.cvnn`` in make_golden.py, ``spectralmc_amd.cvnn`` in the tests), so both sides are
constructed by the same code in the same parameter-creation order.
"""


def _bn_cov(m):
    """Linear -> covariance BN -> modReLU -> residual(Linear -> naive BN -> zReLU, post modReLU) -> Linear."""
    return m.ComplexSequential(
        m.ComplexLinear(6, 24), m.CovarianceComplexBatchNorm(24), m.modReLU(24),
        m.ComplexResidual(m.ComplexSequential(m.ComplexLinear(24, 24), m.NaiveComplexBatchNorm(24), m.zReLU()),
                          post_act=m.modReLU(24)),
        m.ComplexLinear(24, 40))


def _bn_proj(m):
    """Residual with a projection (24 -> 16) and no post-activation; BN without affine parameters."""
    return m.ComplexSequential(
        m.ComplexLinear(6, 24), m.NaiveComplexBatchNorm(24, affine=False), m.zReLU(),
        m.ComplexResidual(m.ComplexSequential(m.ComplexLinear(24, 16), m.CovarianceComplexBatchNorm(16, momentum=0.3)),
                          proj=m.ComplexLinear(24, 16)),
        m.ComplexLinear(16, 32))


# both module sets (the reference's cvnn and this build's) are built by the same functions
BN_ARCHS = {"cov": _bn_cov, "proj": _bn_proj}
