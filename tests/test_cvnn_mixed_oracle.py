"""The oracle's explicit-precision restatement of the network step (oracle/cvnn_mixed.py), which
pins the MFMA kernels of csrc/cvnn_mfma.hip, checked on CPU:

* with f32 operands it equals torch autograd of ``_torch_step``'s loss (reference
  gbm_trainer.py:819-835) on the same model — the real-GEMM form of the complex layers
  ([[A, -B], [B, A]] blocks, dA / dB recombination, bias gradients) is the reference's math;
* the bf16 rounding is torch's ``float.bfloat16()`` (round to nearest even), and the bf16 step
  stays within bf16 precision of the f32 one.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle.cvnn_mixed import bf16_round, cvnn_step
from spectralmc_amd.cvnn import ComplexLinear, ComplexSequential, modReLU, zReLU
from spectralmc_amd.net import lower
from tests.helpers import make_test_cvnn


def layer_table(model) -> list[tuple[int, ...]]:
    params = list(model.parameters())
    return [(t.in_features, t.out_features, t.activation, t.w_re, t.w_im, t.b_re, t.b_im, t.act_bias)
            for t in lower(model, params)]


def flat_params(model) -> np.ndarray:
    return torch.cat([p.detach().reshape(-1) for p in model.parameters()]).numpy().astype(np.float32)


def torch_grads(model, x: torch.Tensor, targets: torch.Tensor) -> tuple[float, np.ndarray]:
    model.zero_grad(set_to_none=True)
    pr, pi = model(x, torch.zeros_like(x))
    loss = torch.nn.functional.mse_loss(pr, targets.real) + torch.nn.functional.mse_loss(pi, targets.imag)
    loss.backward()
    return float(loss), torch.cat([p.grad.reshape(-1) for p in model.parameters()]).double().numpy()


def zrelu_model(n_in: int, n_out: int) -> torch.nn.Module:
    torch.manual_seed(5)
    return ComplexSequential(ComplexLinear(n_in, 24), zReLU(), ComplexLinear(24, 40), modReLU(40),
                             ComplexLinear(40, n_out))


def inputs(B: int, n_in: int, n_out: int, seed: int = 3) -> tuple[torch.Tensor, torch.Tensor]:
    g = torch.Generator().manual_seed(seed)
    x = torch.rand((B, n_in), generator=g) * 2 - 1
    t = torch.complex(torch.randn((B, n_out), generator=g), torch.randn((B, n_out), generator=g))
    return x, t


@pytest.mark.parametrize("arch", ["c2", "c1", "zrelu"])
def test_f32_restatement_equals_torch_autograd(arch) -> None:
    if arch == "zrelu":
        model, n_in, n_out = zrelu_model(6, 64), 6, 64
    else:
        n_in, n_out = 6, 256
        model = make_test_cvnn(n_inputs=n_in, n_outputs=n_out, seed=123, dtype=torch.float32, device="cpu",
                               hidden_layers=2 if arch == "c2" else 1)
    # modest input scale so that every modReLU / zReLU region is populated
    x, t = inputs(96, n_in, n_out)
    loss_t, g_t = torch_grads(model, x, t)
    loss_o, g_o = cvnn_step(layer_table(model), flat_params(model), x.numpy(), None, t.numpy(), operand="f32")
    assert loss_o == pytest.approx(loss_t, rel=1e-6)
    assert np.linalg.norm(g_o - g_t) / np.linalg.norm(g_t) < 2e-6
    for name, (a, b) in {"max": (np.abs(g_o - g_t).max(), 1e-5 * np.abs(g_t).max())}.items():
        assert a <= b, name


def test_bf16_rounding_is_torch_round_to_nearest_even() -> None:
    g = torch.Generator().manual_seed(0)
    x = torch.cat([torch.randn(4096, generator=g) * 10.0 ** torch.randint(-30, 30, (4096,), generator=g),
                   torch.tensor([0.0, -0.0, 1.0, 1.00390625, 1.005859375, 3.0e38, -3.0e38, 1e-40])])
    want = x.bfloat16().float().numpy()
    np.testing.assert_array_equal(bf16_round(x.numpy()), want)


def test_bf16_step_within_bf16_precision_of_f32() -> None:
    model = make_test_cvnn(n_inputs=6, n_outputs=256, seed=123, dtype=torch.float32, device="cpu", hidden_layers=2)
    x, t = inputs(128, 6, 256)
    table, p = layer_table(model), flat_params(model)
    l32, g32 = cvnn_step(table, p, x.numpy(), None, t.numpy(), operand="f32")
    l16, g16 = cvnn_step(table, p, x.numpy(), None, t.numpy(), operand="bf16")
    assert l16 == pytest.approx(l32, rel=2e-2)
    assert np.linalg.norm(g16 - g32) / np.linalg.norm(g32) < 3e-2
    assert not np.array_equal(g16, g32)
