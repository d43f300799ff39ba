"""Which XCDs run the path kernel when the network has its own CUs (pricer.network_cus): a few C2-shaped
training steps on a trace build (SMC_EXPERIMENT_TRACE, SMC_LIB_PATH=tools/micro/libsmc_trace.so), then the
XCC ids the path kernel's workgroups recorded (gbm.hip g_trace slot 1).

    SMC_LIB_PATH=tools/micro/libsmc_trace.so python tools/xcc_probe.py [network_cus]
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from spectralmc_amd import _lib  # noqa: E402
from spectralmc_amd.gbm_trainer import GbmCVNNPricer  # noqa: E402
from spectralmc_amd.models.numerical import Precision  # noqa: E402
from tests.helpers import (expect_success, make_black_scholes_config, make_domain_bounds,  # noqa: E402
                           make_gbm_cvnn_config, make_simulation_params, make_test_cvnn, make_training_config)


def main() -> None:
    ncus = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    sp = make_simulation_params(timesteps=16, network_size=256, batches_per_mc_run=256, threads_per_block=256,
                                mc_seed=7, buffer_size=512, dtype=Precision.float32)
    model = make_test_cvnn(n_inputs=6, n_outputs=256, seed=123, dtype=torch.float32, device="cuda:0",
                           hidden_layers=2, hidden_width=32)
    cfg = make_gbm_cvnn_config(model, sim_params=sp, bs_config=make_black_scholes_config(sim_params=sp),
                               domain_bounds=make_domain_bounds())
    pricer = expect_success(GbmCVNNPricer.create(cfg))
    pricer.math_mode, pricer.network_cus = "hw", ncus
    session = expect_success(pricer.open_session(make_training_config(num_batches=4, batch_size=1024)))
    for _ in range(4):
        expect_success(session.step())
    session.close()
    torch.cuda.synchronize()
    fn = getattr(_lib.lib(), "smc_debug_trace")
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    buf = np.zeros((1024, 40), dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.size) == 0
    used = buf[:, 0] > 0
    xcc = buf[used, 1]
    print(f"network_cus={ncus}: {int(used.sum())} path workgroups traced; per XCC:",
          {int(k): int((xcc == k).sum()) for k in range(8)})


if __name__ == "__main__":
    main()
