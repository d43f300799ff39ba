"""Complex-valued layers on (real, imag) tensor pairs (reference ``src/spectralmc/cvnn.py``).

Same modules, parameter names, initialisation order and arithmetic as the reference so
that ``cvnn_factory.build_model(seed)`` yields the reference's weights bit-for-bit and the
state_dict keys match (e.g. ``layers.0.layers.0.real_weight``).  On the GPU the matmuls run
on hipBLASLt/rocBLAS (f32 MFMA on gfx950); the whole training step is captured in a HIP
graph by the trainer, so the many small kernels are replayed without host launch cost.

Layer catalogue: ComplexLinear, zReLU, modReLU, NaiveComplexBatchNorm,
CovarianceComplexBatchNorm, ComplexSequential, ComplexResidual.
"""

from __future__ import annotations

import torch

nn = torch.nn
Tensor = torch.Tensor


class ComplexLinear(nn.Module):
    """Dense C^n -> C^m: (A x - B y) + i (B x + A y) + b for W = A + iB, z = x + iy."""

    real_weight: nn.Parameter
    imag_weight: nn.Parameter

    def __init__(self, in_features: int, out_features: int, bias: bool = True) -> None:
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.real_weight = nn.Parameter(torch.empty(out_features, in_features))
        self.imag_weight = nn.Parameter(torch.empty(out_features, in_features))
        if bias:
            self.real_bias = nn.Parameter(torch.empty(out_features))
            self.imag_bias = nn.Parameter(torch.empty(out_features))
        else:
            self.register_parameter("real_bias", None)
            self.register_parameter("imag_bias", None)
        self.reset_parameters()

    def reset_parameters(self) -> None:
        # RNG order matters for seeded builds: real weight, imag weight (biases draw nothing).
        nn.init.xavier_uniform_(self.real_weight)
        nn.init.xavier_uniform_(self.imag_weight)
        for b in (self.real_bias, self.imag_bias):
            if b is not None:
                nn.init.zeros_(b)

    def forward(self, real: Tensor, imag: Tensor) -> tuple[Tensor, Tensor]:
        a_t, b_t = self.real_weight.T, self.imag_weight.T
        out_re = real @ a_t - imag @ b_t
        out_im = real @ b_t + imag @ a_t
        if self.real_bias is not None:
            out_re = out_re + self.real_bias
        if self.imag_bias is not None:
            out_im = out_im + self.imag_bias
        return out_re, out_im


class zReLU(nn.Module):  # noqa: N801 - reference name
    """Keep z only where Re z >= 0 and Im z >= 0 (Guberman 2016)."""

    def forward(self, real: Tensor, imag: Tensor) -> tuple[Tensor, Tensor]:
        keep = (real >= 0) & (imag >= 0)
        return real * keep, imag * keep


class modReLU(nn.Module):  # noqa: N801 - reference name
    """relu(|z| + b) * z / |z| with a learned per-feature threshold b (Arjovsky 2016)."""

    bias: nn.Parameter

    def __init__(self, num_features: int) -> None:
        super().__init__()
        self.bias = nn.Parameter(torch.zeros(num_features))

    def forward(self, real: Tensor, imag: Tensor) -> tuple[Tensor, Tensor]:
        mag = torch.sqrt(real * real + imag * imag + 1e-9)
        gain = torch.relu(mag + self.bias.unsqueeze(0)) / mag
        return gain * real, gain * imag


class NaiveComplexBatchNorm(nn.Module):
    """BatchNorm1d applied to the real and imaginary parts independently."""

    def __init__(self, num_features: int, *, eps: float = 1e-5, momentum: float = 0.1, affine: bool = True,
                 track_running_stats: bool = True) -> None:
        super().__init__()
        kw = dict(eps=eps, momentum=momentum, affine=affine, track_running_stats=track_running_stats)
        self.bn_real = nn.BatchNorm1d(num_features, **kw)
        self.bn_imag = nn.BatchNorm1d(num_features, **kw)

    def forward(self, real: Tensor, imag: Tensor) -> tuple[Tensor, Tensor]:
        return self.bn_real(real), self.bn_imag(imag)


class CovarianceComplexBatchNorm(nn.Module):
    """Whitening batch norm with the per-feature 2x2 covariance of (Re, Im) (Trabelsi 2018)."""

    def __init__(self, num_features: int, *, eps: float = 1e-5, momentum: float = 0.1, affine: bool = True,
                 track_running_stats: bool = True) -> None:
        super().__init__()
        dt = torch.get_default_dtype()
        self.register_buffer("running_mean_real", torch.zeros(num_features, dtype=dt))
        self.register_buffer("running_mean_imag", torch.zeros(num_features, dtype=dt))
        self.register_buffer("running_C_rr", torch.full((num_features,), 0.5, dtype=dt))
        self.register_buffer("running_C_ri", torch.zeros(num_features, dtype=dt))
        self.register_buffer("running_C_ii", torch.full((num_features,), 0.5, dtype=dt))
        self.eps = eps
        self.momentum = momentum
        self.affine = affine
        self.track_running_stats = track_running_stats
        if affine:
            self.beta_real = nn.Parameter(torch.zeros(num_features, dtype=dt))
            self.beta_imag = nn.Parameter(torch.zeros(num_features, dtype=dt))
            self.gamma_rr = nn.Parameter(torch.ones(num_features, dtype=dt))
            self.gamma_ri = nn.Parameter(torch.zeros(num_features, dtype=dt))
            self.gamma_ii = nn.Parameter(torch.ones(num_features, dtype=dt))
        else:
            for name in ("beta_real", "beta_imag", "gamma_rr", "gamma_ri", "gamma_ii"):
                self.register_parameter(name, None)

    def _batch_stats(self, real: Tensor, imag: Tensor):
        mu_r, mu_i = real.mean(dim=0), imag.mean(dim=0)
        cr, ci = real - mu_r, imag - mu_i
        c_rr = (cr * cr).mean(dim=0)
        c_ii = (ci * ci).mean(dim=0)
        c_ri = (cr * ci).mean(dim=0)
        if self.track_running_stats:
            m = self.momentum
            with torch.no_grad():
                for buf, val in ((self.running_mean_real, mu_r), (self.running_mean_imag, mu_i),
                                 (self.running_C_rr, c_rr), (self.running_C_ri, c_ri), (self.running_C_ii, c_ii)):
                    buf.mul_(1 - m).add_(val * m)
        return cr, ci, c_rr, c_ri, c_ii

    def forward(self, real: Tensor, imag: Tensor) -> tuple[Tensor, Tensor]:
        if self.training or not self.track_running_stats:
            cr, ci, c_rr, c_ri, c_ii = self._batch_stats(real, imag)
        else:
            cr, ci = real - self.running_mean_real, imag - self.running_mean_imag
            c_rr, c_ri, c_ii = self.running_C_rr, self.running_C_ri, self.running_C_ii
        cov = torch.stack([torch.stack([c_rr + self.eps, c_ri], dim=1),
                           torch.stack([c_ri, c_ii + self.eps], dim=1)], dim=1)  # (C, 2, 2)
        evals, evecs = torch.linalg.eigh(cov)
        inv_sqrt = (1.0 / evals.clamp_min(self.eps).sqrt()).unsqueeze(1)
        whiten = (evecs * inv_sqrt) @ evecs.transpose(1, 2)
        pair = torch.stack([cr, ci], dim=2).unsqueeze(-1)  # (N, C, 2, 1)
        w = (whiten.unsqueeze(0) @ pair).squeeze(-1)
        wr, wi = w[..., 0], w[..., 1]
        if not self.affine:
            return wr, wi
        out_r = self.gamma_rr * wr + self.gamma_ri * wi + self.beta_real
        out_i = self.gamma_ri * wr + self.gamma_ii * wi + self.beta_imag
        return out_r, out_i


class ComplexSequential(nn.Module):
    """Sequential container threading (real, imag) through its children."""

    def __init__(self, *modules: nn.Module) -> None:
        super().__init__()
        self.layers = nn.ModuleList(modules)

    def forward(self, real: Tensor, imag: Tensor) -> tuple[Tensor, Tensor]:
        for layer in self.layers:
            real, imag = layer(real, imag)
        return real, imag


class ComplexResidual(nn.Module):
    """x + body(x), with an optional projection of x and an optional post-activation."""

    def __init__(self, body: nn.Module, proj: nn.Module | None = None, post_act: nn.Module | None = None) -> None:
        super().__init__()
        self.body = body
        self.proj = proj
        self.post_act = post_act

    def forward(self, real: Tensor, imag: Tensor) -> tuple[Tensor, Tensor]:
        br, bi = self.body(real, imag)
        sr, si = (real, imag) if self.proj is None else self.proj(real, imag)
        out_r, out_i = br + sr, bi + si
        if self.post_act is not None:
            out_r, out_i = self.post_act(out_r, out_i)
        return out_r, out_i


__all__ = ["ComplexLinear", "zReLU", "modReLU", "NaiveComplexBatchNorm", "CovarianceComplexBatchNorm",
           "ComplexSequential", "ComplexResidual"]
